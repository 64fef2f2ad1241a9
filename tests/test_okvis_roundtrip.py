"""okvis' own functor objects across the boundary and back.

okvis keeps each ImuError's preintegration state in protected members of the functor
(ImuError.hpp:266-305) and relies on it after a solve: a >= 50-sample factor keeps its
linearisation point (speedAndBiases_ref_) unless redoPropagationAlways (ImuError.cpp:834-858),
ImuError::append continues from it ("all left, not reset!", ImuError.cpp:93-94), and the
realtime -> full-graph copy duplicates it (ViSlamBackend.cpp:925-997). The facade's
okvis_access adapters (include/okvisgpu_problem.hpp) read those members into the C-ABI state and
write the solved state back; TwoPose / RelativePose / PoseError / SpeedAndBias terms are read the
same way (TwoPoseGraphError.hpp:178,283-284,364-372 etc.).

tests/cpp/okvis_roundtrip.cpp drives it against stand-ins that mirror the okvis members:
  cpu: accessor read / write of every adapted functor (CPU suite);
  gpu: three facade solves of a window whose IMU terms are live views of the okvis objects (solve 1
       on Problem P1; solve 2 on a NEW Problem P2 over the same objects; solve 3 on P2 again), its
       priors and pose-graph edges converted by fromOkvis*; after each the parameters and the objects'
       states (read back through the accessor) are dumped. Here the oracle replays the three solves
       on one problem whose state simply continues, then ImuError::append (the oracle's restatement)
       runs on the GPU-written-back states and on the oracle's own: equal."""
import os
import subprocess

import numpy as np
import pytest

from _paths import REPO

CPP = os.path.join(REPO, "tests", "cpp")
EXE = os.path.join(CPP, "okvis_roundtrip")
CHAIN = list(range(2, 66)) + list(range(292, 301))  # Delta_q .. dp_db_g, sb_ref, cross_
P_DELTA = slice(301, 526)
SQRT = slice(66, 291)
# the window: S10 shape with 0.5 s keyframe spacing (~100 samples per IMU factor, so
# ImuError.cpp:837 takes its >= 50-sample arm), pose-graph edges of all three kinds
KF, LM, OBS, KF_DT, SEED, N_REL = 10, 500, 4000, 0.5, 7101, 3
ITERS = (4, 3, 3)


@pytest.fixture(scope="module")
def exe():
    r = subprocess.run(["make", "-C", CPP], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    return EXE


def test_okvis_accessors_cpu(exe):
    r = subprocess.run([exe, "cpu"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "okvis_roundtrip cpu ok" in r.stdout


def _window(og):
    return og.SynthWindow(KF, LM, OBS, seed=SEED, kf_dt_s=KF_DT, n_relpose=N_REL, relpose_stride=2, relpose_kind=2)


def _info(state):
    U = state[SQRT].reshape(15, 15)
    return U.T @ U


def _zero_tol(og, iters):
    return og.default_options(max_num_iterations=iters, function_tolerance=0.0, gradient_tolerance=0.0,
                              parameter_tolerance=0.0)


def _read_dump(og, path, p, n_solves):
    per = 4 + 7 * p.n_poses + 9 * p.n_speed_biases + 4 * p.n_landmarks + 526 * p.n_imu
    d = np.fromfile(path, dtype=np.float64)
    assert d.size == per * n_solves, (d.size, per)
    out = []
    for k in range(n_solves):
        x = d[k * per:(k + 1) * per]
        o = 4
        rec = {"initial_cost": x[0], "final_cost": x[1], "num_iterations": int(x[2]),
               "termination": og.TERMINATION.get(int(x[3]), "?")}
        for name, n in (("poses", 7 * p.n_poses), ("sb", 9 * p.n_speed_biases), ("lm", 4 * p.n_landmarks),
                        ("states", 526 * p.n_imu)):
            rec[name] = x[o:o + n]
            o += n
        rec["poses"] = rec["poses"].reshape(-1, 7)
        rec["sb"] = rec["sb"].reshape(-1, 9)
        rec["states"] = rec["states"].reshape(-1, 526)
        out.append(rec)
    return out


def _states_match(g, ref, tol, what):
    for k in CHAIN:
        assert abs(g[k] - ref[k]) <= tol * max(1.0, abs(ref[k])), (what, k, g[k], ref[k])
    assert np.abs(g[P_DELTA] - ref[P_DELTA]).max() <= tol * np.abs(ref[P_DELTA]).max(), what
    Ig, Ir = _info(g), _info(ref)
    assert np.abs(Ig - Ir).max() <= 1e3 * tol * np.abs(Ir).max(), what
    assert g[0] == ref[0] and g[1] == ref[1], (what, g[:2], ref[:2])


@pytest.mark.gpu
def test_okvis_objects_roundtrip_gpu(exe, og, oracle, tmp_path, parity):
    dump_path = str(tmp_path / "roundtrip.bin")
    r = subprocess.run([exe, "gpu", dump_path, str(KF), str(LM), str(OBS), str(KF_DT), str(SEED), str(N_REL)],
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "okvis_roundtrip gpu ok" in r.stdout
    w = _window(og)
    p = w.problem
    gpu = _read_dump(og, dump_path, p, len(ITERS))
    sb_begin = np.ctypeslib.as_array(p.imu_sample_begin, shape=(p.n_imu + 1,))
    assert np.diff(sb_begin).min() >= 50  # every factor on the >= 50-sample arm
    imu_blocks = np.ctypeslib.as_array(p.imu_blocks, shape=(p.n_imu, 4))
    sb_initial = w.speed_biases().copy()
    # the oracle: the same three solves on ONE problem whose ImuError state simply continues
    worst = {"cost": 0.0, "pose": 0.0}
    for k, iters in enumerate(ITERS):
        so = oracle.solve(w.problem_ptr(), _zero_tol(og, iters))
        g = gpu[k]
        assert g["num_iterations"] == so["num_iterations"] and g["termination"] == so["termination"], (k, g, so)
        dc = abs(g["final_cost"] - so["final_cost"]) / so["final_cost"]
        dp = float(np.abs(g["poses"][:, :3] - w.poses()[:, :3]).max())
        worst["cost"], worst["pose"] = max(worst["cost"], dc), max(worst["pose"], dp)
        assert dc <= 1e-7 and dp <= 1e-6, (k, dc, dp)
        st = w.imu_state()
        for f in range(p.n_imu):
            _states_match(g["states"][f], st[f], 1e-9, (k, f))
    parity("okvis_roundtrip_cost_rel", worst["cost"], 1e-7)
    parity("okvis_roundtrip_pose_m", worst["pose"], 1e-6)
    # the reference point survived both later solves: integrated once (counter 1) at the initial
    # bias of the factor's first state, the redo flag set where the gyro bias moved > 3e-4
    # (ImuError.cpp:836) but no re-integration (>= 50 samples, no redoPropagationAlways)
    final = gpu[-1]["states"]
    assert (final[:, 0] == 1).all(), final[:, 0]
    assert np.array_equal(final[:, 57:66], sb_initial[imu_blocks[:, 1]])
    moved = np.linalg.norm(gpu[0]["sb"][imu_blocks[:, 1], 3:6] - sb_initial[imu_blocks[:, 1], 3:6], axis=1) > 3e-4
    assert moved.any() and (final[moved, 1] == 1).all()
    # control: a boundary that dropped the state after solve 1 (a fresh ImuError per Problem: counter
    # 0, so the first evaluation re-integrates at the current bias) gives a different solve 2, so the
    # comparisons above do see whether the state crossed
    w2 = _window(og)
    oracle.solve(w2.problem_ptr(), _zero_tol(og, ITERS[0]))
    w2.imu_state()[:] = 0.0
    s_fresh = oracle.solve(w2.problem_ptr(), _zero_tol(og, ITERS[1]))
    assert abs(s_fresh["final_cost"] - gpu[1]["final_cost"]) > 1e-6 * gpu[1]["final_cost"]  # 10x the bound above
    assert np.abs(w2.imu_state()[:, 57:66] - gpu[1]["states"][:, 57:66]).max() > 1e-4  # another reference point
    # ImuError::append (IMU-merge elimination, ViGraphEstimator.cpp:38-171) on the written-back states
    # vs on the oracle's: link f continued over link f+1's samples with state f+1's bias
    from test_imu_append import _merged_samples
    fs = list(range(0, p.n_imu - 1, 2))
    t1 = np.ctypeslib.as_array(p.imu_t1_ns, shape=(p.n_imu,))
    begin, ts, ga = [0], [], []
    for f in fs:
        _, _, (t_next, g_next) = _merged_samples(p, f)
        ts.append(t_next)
        ga.append(g_next)
        begin.append(begin[-1] + len(t_next))
    sbs = np.ascontiguousarray(w.speed_biases()[imu_blocks[fs, 3]])
    args = (t1[fs], t1[[f + 1 for f in fs]], sbs, begin, np.concatenate(ts), np.concatenate(ga))
    from_gpu = np.ascontiguousarray(final[fs])
    from_oracle = np.ascontiguousarray(w.imu_state()[fs])
    s1 = oracle.imu_append(p.imu_params, from_gpu, *args)
    s2 = oracle.imu_append(p.imu_params, from_oracle, *args)
    assert (s1 == s2).all() and (s1 > 0).all()
    for i, f in enumerate(fs):
        _states_match(from_gpu[i], from_oracle[i], 1e-9, ("append", f))
