"""Host-side plan of a window's reduced system (okvisgpu_plan_window; runtime.cpp analyse, chooseNd,
cholSchedule), checked on the CPU against invariants restated here independently:

  - the natural order is the identity; the nested-dissection order is a permutation of the same
    rows with gap rows (-1) after the left part, padded to a tile boundary;
  - the filled tile pattern is closed under elimination (k < j < i, L_ik, L_jk non-zero => L_ij);
  - the split parts share no non-zero tile (the premise of the two-workgroup schedules);
  - the tile-parallel schedule is a valid order of the right-looking factorisation: a step's
    updates run after the launch that factors its diagonal tile (the root launch 0 or the launch
    of that tile's last update), every tile's updates run in step order in distinct launches, and
    a panel tile is final before the step that uses it.
The GPU side of the same orders is tests/test_gpu_parity.py::test_cholesky_schedules_agree*."""
import numpy as np
import pytest

from _gps import gps_window


def _check_pattern(nz):
    T = nz.shape[0]
    assert (np.diag(nz) == 1).all() and not np.triu(nz, 1).any()
    for k in range(T):
        rows = [i for i in range(k + 1, T) if nz[i, k]]
        for a in rows:
            for b in rows:
                if b < a:
                    assert nz[a, b], (k, a, b)


def _check_schedule(nz, launch):
    """Replays the updates launch by launch; returns the number of launches (incl. launch 0)."""
    T = nz.shape[0]
    last = -np.ones((T, T), dtype=int)  # launch of each tile's last update so far
    writes = {}
    for k in range(T):
        targets = [(i, j) for i in range(k + 1, T) for j in range(k + 1, i + 1) if nz[i, k] and nz[j, k]]
        if not targets:
            assert launch[k] == 0
            continue
        assert launch[k] >= 1
        # the diagonal tile k is factored in launch 0 (root) or with its last update
        assert launch[k] > max(0, last[k, k]), (k, launch[k], last[k, k])
        for i in range(k + 1, T):
            if nz[i, k]:
                assert last[i, k] < launch[k], ("panel not final", i, k)
        for (i, j) in targets:
            assert last[i, j] < launch[k], ("updates out of order", i, j, k)
            key = (int(launch[k]), i, j)
            assert key not in writes, ("two writers in one launch", key)
            writes[key] = k
            last[i, j] = launch[k]
    return int(launch.max()) + 1


@pytest.mark.parametrize("shape", [(50, 2000, 16000), (10, 500, 4000), (20, 800, 6000)])
def test_natural_order(og, shape):
    w = og.SynthWindow(*shape, seed=20251015)
    r = og.plan_window(w.problem, 0)
    n = r["reduced_dim"]
    assert r["split_tL"] == r["split_tS"] == r["gap_rows"] == 0
    assert np.array_equal(r["natural"][:n], np.arange(n)) and (r["natural"][n:] == -1).all()
    _check_pattern(r["tile_nz"])
    assert _check_schedule(r["tile_nz"], r["step_launch"]) == r["launches"]
    assert r["nonzero_tiles"] == int(r["tile_nz"].sum())


def test_nested_dissection_s50(og):
    w = og.SynthWindow(50, 2000, 16000, seed=20251015)
    r0 = og.plan_window(w.problem, 0)
    r = og.plan_window(w.problem, 1)
    n, D, T = r["reduced_dim"], r["s_dim"], r["tiles"]
    assert n == r0["reduced_dim"] == 750 and T == r0["tiles"] == 12
    # a shorter launch chain for the same tile count (12 -> 8 on this window)
    assert r["launches"] <= r0["launches"] - 3 and r["nonzero_tiles"] <= r0["nonzero_tiles"] + 2
    nat = r["natural"]
    assert sorted(nat[nat >= 0].tolist()) == list(range(n)) and (nat < 0).sum() == D - n
    tL, tS = r["split_tL"], r["split_tS"]
    assert 0 < tL < tS <= T
    gap = np.flatnonzero(nat[:tL * 64] < 0)
    assert len(gap) == r["gap_rows"] and (gap == np.arange(tL * 64 - len(gap), tL * 64)).all()
    nz = r["tile_nz"]
    assert not nz[tL:tS, :tL].any()  # the parts are independent
    _check_pattern(nz)
    assert _check_schedule(nz, r["step_launch"]) == r["launches"]
    # both parts' chains run side by side: the right part's first step shares a launch with the left's
    assert r["step_launch"][tL] == r["step_launch"][0]


def test_nested_dissection_full_graph(og):
    """A 200-keyframe graph with GPS host factors (the full-graph shape): the chooser's strided
    search (more than 64 slots) and the same invariants."""
    p, _, _ = gps_window(seed=9, n_kf=200, n_lm=8000, n_obs=64000)
    r0 = og.plan_window(p.struct, 0)
    r = og.plan_window(p.struct, 1)
    assert r["reduced_dim"] == r0["reduced_dim"]
    for rr in (r0, r):
        _check_pattern(rr["tile_nz"])
        assert _check_schedule(rr["tile_nz"], rr["step_launch"]) == rr["launches"]
    assert r["launches"] <= r0["launches"]
    if r["split_tS"]:
        assert not r["tile_nz"][r["split_tL"]:r["split_tS"], :r["split_tL"]].any()
