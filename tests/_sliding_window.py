"""TEST INFRASTRUCTURE (the config-3 harness; not part of the product package). The okvis realtime sliding-window sequence driven through the okvisgpu C ABI (host logic only).

This is the CALLER of the accelerated path, restated so that a whole okvis VIO run (BASELINE config
3, "EuRoC MH_05 full sliding-window VIO": one realtime solve per frame, then marginalisation) can be
exercised against the C ABI. Per frame, as `ThreadedSlam::optimisePublishMarginalise`
(ThreadedSlam.cpp:945-977,1234-1237) does:

1. the new state joins the realtime graph with the IMU link from the previous state
   (`ViGraph::addStatesPropagate`, ViGraph.cpp:400-480) and its observations;
2. `ViSlamBackend::optimiseRealtimeGraph` (ViSlamBackend.cpp:811-1010): DENSE_SCHUR + DOGLEG,
   `realtime_max_iterations` (config/euroc/okvis2.yaml:91) -> `Backend.solve` (okvisgpu_solve);
3. `ViSlamBackend::applyStrategy` (ViSlamBackend.cpp:555-809):
   - `eliminateImuFrames` (:511-553): surplus IMU frames become keyframes, or are removed by
     `ViGraphEstimator::eliminateStateByImuMerge` (ViGraphEstimator.cpp:38-171) ->
     `Backend.imu_append` (okvisgpu_imu_append, ImuError::append);
   - keyframe conversion to the pose graph (:593-667) with `convertToPoseGraphMst`
     (ViGraphEstimator.cpp:334-610, Kruskal MST of the covisibility graph, MstGraph.hpp:132-169)
     -> `Backend.twopose` (okvisgpu_twopose_compute, TwoPoseStandardGraphError::compute);
   - freezing of old states (:669-712, `freezePosesUntil` / `freezeSpeedAndBiasesUntil`,
     ViGraphEstimator.cpp:216-298) -> constant parameter blocks of the next problem.

Everything structural (which frames are eliminated, converted, frozen) depends only on the graph
structure and time stamps, never on estimates, so two backends run the same sequence of problems.
Restatement limits (documented in DESIGN.md §7c): `overlapFraction` of the frontend's MultiFrames
(used by `mostOverlappedStateId`, ViSlamBackend.cpp:2780-2809) becomes the co-observed landmark
count; no loop-closure frames (VIO mode); `expandKeyframe` and re-converting an existing pose-graph
edge (`convertToReprojectionErrors`) are not restated and raise if the sequence would need them;
a new state starts at the world's perturbed estimate with the previous state's bias (instead of IMU
propagation); landmarks without observations stay out of the problem.

The backend is any object with `solve(problem_struct, options) -> summary dict` (results written
back into the problem's arrays), `imu_append(...)` (okvisgpu_imu_append semantics) and
`twopose(TwoPoseBatch) -> dict`; `GpuBackend` is the okvisgpu one. No solver logic lives here.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

import numpy as np

from okvisgpu import (IMU_STATE_DOUBLES, Camera, Context, ImuParams, Problem, SynthWindow, TwoPoseBatch,
               default_options, dptr)

_ip = C.POINTER(C.c_int32)
_lp = C.POINTER(C.c_int64)
_up = C.POINTER(C.c_uint8)


class GpuBackend:
    """okvisgpu on one device: one context (one HIP stream), re-used for every frame."""

    def __init__(self, device: int = 0):
        self.ctx = Context(device)

    def solve(self, problem: Problem, options):
        self.ctx.set_problems([problem])
        return self.ctx.solve(options)[0]

    def imu_append(self, *args):
        return self.ctx.imu_append(*args)

    def twopose(self, batch: TwoPoseBatch):
        return self.ctx.twopose_compute(batch)

    def close(self):
        self.ctx.close()


class World:
    """A synthetic VIO sequence: the frames of one long synthetic window (okvisgpu_synth_create,
    SURVEY.md §8d generator: EuRoC stereo rig, 200 Hz IMU, frames every kf_dt_s) fed one per step.
    Frame k's initial estimate is the generator's perturbed one; its observations, IMU samples to
    frame k+1 and the first-state priors come from the same window."""

    def __init__(self, n_frames=30, n_landmarks=900, n_observations=7200, seed=20251101, **cfg):
        w = SynthWindow(n_frames, n_landmarks, n_observations, seed=seed, **cfg)
        self.window = w
        p = w.problem
        self.n_frames = n_frames
        self.init_poses = w.poses().copy()
        self.init_sbs = w.speed_biases().copy()
        self.init_lms = w.landmarks().copy()
        self.gt_poses, self.gt_lms, self.gt_sbs = w.ground_truth()
        self.cameras = [Camera() for _ in range(p.n_cameras)]
        for i in range(p.n_cameras):
            C.pointer(self.cameras[i])[0] = p.cameras[i]
        self.extrinsics = w.extrinsics().copy()
        self.imu_params = ImuParams()
        C.pointer(self.imu_params)[0] = p.imu_params
        n = p.n_observations
        op = np.ctypeslib.as_array(p.obs_pose, shape=(n,)).copy()
        ol = np.ctypeslib.as_array(p.obs_landmark, shape=(n,)).copy()
        oc = np.ctypeslib.as_array(p.obs_camera, shape=(n,)).copy()
        kp = np.ctypeslib.as_array(p.obs_keypoint, shape=(n, 2)).copy()
        L = np.ctypeslib.as_array(p.obs_sqrt_info, shape=(n, 4)).copy()
        self.frame_obs = [[(int(oc[i]), int(ol[i]), kp[i], L[i]) for i in np.flatnonzero(op == k)]
                          for k in range(n_frames)]
        sb = np.ctypeslib.as_array(p.imu_sample_begin, shape=(p.n_imu + 1,))
        ts = np.ctypeslib.as_array(p.imu_sample_t_ns, shape=(sb[-1],))
        ga = np.ctypeslib.as_array(p.imu_sample_gyr_acc, shape=(sb[-1], 6))
        t0 = np.ctypeslib.as_array(p.imu_t0_ns, shape=(p.n_imu,))
        t1 = np.ctypeslib.as_array(p.imu_t1_ns, shape=(p.n_imu,))
        self.frame_t = np.r_[t0, t1[-1]].astype(np.int64)
        self.link_samples = [(ts[sb[k]:sb[k + 1]].copy(), ga[sb[k]:sb[k + 1]].copy()) for k in range(p.n_imu)]
        self.pose_prior = (np.ctypeslib.as_array(p.pose_prior_meas, shape=(7,)).copy(),
                           np.ctypeslib.as_array(p.pose_prior_sqrt_info, shape=(36,)).copy())
        self.sb_prior = (np.ctypeslib.as_array(p.sb_prior_meas, shape=(9,)).copy(),
                         np.ctypeslib.as_array(p.sb_prior_sqrt_info, shape=(81,)).copy())


@dataclass
class State:
    t_ns: int
    pose: np.ndarray
    sb: np.ndarray
    is_keyframe: bool
    pose_fixed: bool = False
    sb_fixed: bool = False
    pose_graph_frame: bool = False


@dataclass
class ImuLink:
    t0: int
    t1: int
    ts: np.ndarray
    ga: np.ndarray
    state: np.ndarray = field(default_factory=lambda: np.zeros(IMU_STATE_DOUBLES))


@dataclass
class Edge:
    delta_x: np.ndarray
    sqrt_info: np.ndarray
    lin_point: np.ndarray


class SlidingWindow:
    """One realtime graph (`ViSlamBackend::realtimeGraph_`) and its strategy state."""

    def __init__(self, world: World, backend, num_keyframes=5, num_imu_frames=3, num_realtime_pose_graph_frames=12,
                 min_delta_t=2.0, keyframe_every=2, max_iterations=10, num_threads=3, options=None):
        self.world = world
        self.backend = backend
        self.num_keyframes = num_keyframes            # config/euroc/okvis2.yaml:84
        self.num_imu_frames = num_imu_frames          # :86
        self.num_rt_pg_frames = num_realtime_pose_graph_frames  # ViSlamBackend.cpp:37
        self.min_delta_t = min_delta_t                # ViSlamBackend.cpp:36
        self.keyframe_every = keyframe_every
        self.options = options or default_options(max_num_iterations=max_iterations, num_threads=num_threads)
        self.states: dict[int, State] = {}
        self.links: dict[tuple, ImuLink] = {}
        self.landmarks: dict[int, np.ndarray] = {}
        self.obs: dict[tuple, tuple] = {}             # (frame, camera, landmark) -> (kp, sqrt_info)
        self.pending: dict[int, dict] = {}            # landmark -> observations not yet in the graph
        self.edges: dict[tuple, Edge] = {}            # (reference, other) -> pose-graph edge
        self.key_frames: set[int] = set()
        self.imu_frames: set[int] = set()
        self.last_freeze = None
        self.log = []                                 # structural events, backend independent

    # ------------------------------------------------------------------ graph bookkeeping
    def ids(self):
        return sorted(self.states)

    def add_frame(self, k: int):
        """ViGraph::addStatesPropagate + the frontend's observations of frame k."""
        w = self.world
        ids = self.ids()
        sb = w.init_sbs[k].copy()
        if ids:
            prev = ids[-1]
            sb[3:] = self.states[prev].sb[3:]  # biases carried over from the previous state
            ts, ga = w.link_samples[k - 1]
            assert prev == k - 1, "the newest state is always the previous frame"
            self.links[(prev, k)] = ImuLink(int(w.frame_t[prev]), int(w.frame_t[k]), ts.copy(), ga.copy())
        self.states[k] = State(int(w.frame_t[k]), w.init_poses[k].copy(), sb,
                               is_keyframe=(k % self.keyframe_every == 0))
        # The synthetic frontend: a landmark enters the graph once it has two observations (the
        # frontend triangulates before ViGraph::addLandmark / addObservation); later observations of
        # a landmark in the graph go straight in.
        in_graph = {lm for (_, _, lm) in self.obs}
        for cam, lm, kp, L in w.frame_obs[k]:
            if lm in in_graph:
                self.obs[(k, cam, lm)] = (kp, L)
                continue
            pend = self.pending.setdefault(lm, {})
            pend[(k, cam, lm)] = (kp, L)
            if len(pend) >= 2:
                if lm not in self.landmarks:
                    self.landmarks[lm] = w.init_lms[lm].copy()
                self.obs.update(self.pending.pop(lm))
                in_graph.add(lm)
        self.imu_frames.add(k)

    def remove_all_observations(self, sid):
        for key in [key for key in self.obs if key[0] == sid]:
            del self.obs[key]
        for lm in list(self.pending):
            self.pending[lm] = {k: v for k, v in self.pending[lm].items() if k[0] != sid}
            if not self.pending[lm]:
                del self.pending[lm]

    def clean_unobserved_landmarks(self):
        """ViGraph::cleanUnobservedLandmarks (ViGraph.cpp:1914-1940, called by the frontend every
        frame, Frontend.cpp:1140): a landmark left with one observation loses it."""
        count = {}
        for key in self.obs:
            count.setdefault(key[2], []).append(key)
        for lm, keys in count.items():
            if len(keys) == 1:
                del self.obs[keys[0]]

    def covisibilities(self):
        """ViGraph::computeCovisibilities (ViGraph.cpp:727-763): per landmark, every pair of distinct
        observing frames counts once. Returns {(larger id, smaller id): count}."""
        frames = {}
        for (f, _, lm) in self.obs:
            frames.setdefault(lm, set()).add(f)
        co = {}
        for fs in frames.values():
            fs = sorted(fs)
            for i in range(len(fs)):
                for j in range(i):
                    key = (fs[i], fs[j])
                    co[key] = co.get(key, 0) + 1
        return co

    @staticmethod
    def covis(co, a, b):
        """ViGraph::covisibilities (ViGraph.cpp:767-785)."""
        if a == b:
            return 0
        return co.get((max(a, b), min(a, b)), 0)

    def most_overlapped(self, frame, co):
        """ViSlamBackend::mostOverlappedStateId (ViSlamBackend.cpp:2780-2809) with the co-observed
        landmark count standing in for the frontend's image overlap fraction."""
        ret, overlap = None, 0
        for sid in sorted(self.key_frames | self.imu_frames):
            if sid == frame or not self.states[sid].is_keyframe:
                continue
            o = self.covis(co, sid, frame)
            if o >= overlap:
                ret, overlap = sid, o
        return ret

    # ------------------------------------------------------------------ the problem of one solve
    def build_problem(self):
        """The realtime graph as an okvisgpu_problem (what ViGraph hands to ::ceres::Solve)."""
        ids = self.ids()
        sidx = {s: i for i, s in enumerate(ids)}
        lm_ids = sorted({lm for (_, _, lm) in self.obs})
        lidx = {l: i for i, l in enumerate(lm_ids)}
        P = _OwnedProblem()
        P.poses = np.array([self.states[s].pose for s in ids])
        P.pose_constant = np.array([self.states[s].pose_fixed for s in ids], np.uint8)
        P.speed_biases = np.array([self.states[s].sb for s in ids])
        P.speed_bias_constant = np.array([self.states[s].sb_fixed for s in ids], np.uint8)
        P.landmarks = np.array([self.landmarks[l] for l in lm_ids]).reshape(-1, 4)
        P.cameras = self.world.cameras
        P.extrinsics = self.world.extrinsics.copy()
        keys = sorted(self.obs, key=lambda k: (k[2], k[0], k[1]))
        P.obs_pose = np.array([sidx[k[0]] for k in keys], np.int32)
        P.obs_landmark = np.array([lidx[k[2]] for k in keys], np.int32)
        P.obs_camera = np.array([k[1] for k in keys], np.int32)
        P.obs_keypoint = np.array([self.obs[k][0] for k in keys]).reshape(-1, 2)
        P.obs_sqrt_info = np.array([self.obs[k][1] for k in keys]).reshape(-1, 4)
        P.obs_cauchy = np.ones(len(keys), np.uint8)
        links = [(a, b) for a, b in zip(ids[:-1], ids[1:])]
        assert set(links) == set(self.links), "every consecutive pair of states holds an IMU link"
        P.imu_blocks = np.array([[sidx[a], sidx[a], sidx[b], sidx[b]] for a, b in links], np.int32).reshape(-1, 4)
        P.imu_t0_ns = np.array([self.links[l].t0 for l in links], np.int64)
        P.imu_t1_ns = np.array([self.links[l].t1 for l in links], np.int64)
        begin = np.cumsum([0] + [len(self.links[l].ts) for l in links]).astype(np.int32)
        P.imu_sample_begin = begin
        P.imu_sample_t_ns = np.concatenate([self.links[l].ts for l in links]) if links else np.zeros(0, np.int64)
        P.imu_sample_gyr_acc = np.concatenate([self.links[l].ga for l in links]) if links else np.zeros((0, 6))
        P.imu_params = self.world.imu_params
        P.imu_state = np.array([self.links[l].state for l in links]).reshape(-1, IMU_STATE_DOUBLES)
        if 0 in sidx:  # ViGraph::addStatesInitialise priors on the first state (ViGraph.cpp:347-370)
            P.pose_prior_block = np.array([sidx[0]], np.int32)
            P.pose_prior_meas = self.world.pose_prior[0][None]
            P.pose_prior_sqrt_info = self.world.pose_prior[1][None]
            P.sb_prior_block = np.array([sidx[0]], np.int32)
            P.sb_prior_meas = self.world.sb_prior[0][None]
            P.sb_prior_sqrt_info = self.world.sb_prior[1][None]
        ek = sorted(self.edges)
        P.relpose_blocks = np.array([[sidx[a], sidx[b]] for a, b in ek], np.int32).reshape(-1, 2)
        P.relpose_delta_x = np.array([self.edges[e].delta_x for e in ek]).reshape(-1, 6)
        P.relpose_sqrt_info = np.array([self.edges[e].sqrt_info.reshape(-1) for e in ek]).reshape(-1, 36)
        P.relpose_lin_point = np.array([self.edges[e].lin_point for e in ek]).reshape(-1, 7)
        P.relpose_kind = np.zeros(len(ek), np.uint8)
        P.bind()
        return P, ids, lm_ids, links

    def optimise(self):
        """ViSlamBackend::optimiseRealtimeGraph -> ViGraph::optimise (DENSE_SCHUR)."""
        P, ids, lm_ids, links = self.build_problem()
        return self.absorb(P, ids, lm_ids, links, self.backend.solve(P.struct, self.options))

    def absorb(self, P, ids, lm_ids, links, s):
        """Take a solved problem's estimates (and IMU states) back into the graph."""
        for i, sid in enumerate(ids):
            self.states[sid].pose[:] = P.poses[i]
            self.states[sid].sb[:] = P.speed_biases[i]
        for i, l in enumerate(lm_ids):
            self.landmarks[l][:] = P.landmarks[i]
        for i, l in enumerate(links):
            self.links[l].state[:] = P.imu_state[i]
        s["n_states"], s["n_landmarks"], s["n_observations"] = len(ids), len(lm_ids), len(P.obs_pose)
        s["n_relpose"], s["n_free_poses"] = len(self.edges), int(len(ids) - P.pose_constant.sum())
        return s

    # ------------------------------------------------------------------ marginalisation strategy
    def eliminate_imu_frames(self):
        """ViSlamBackend::eliminateImuFrames (ViSlamBackend.cpp:511-553)."""
        merges = []
        for sid in sorted(self.imu_frames):
            if len(self.imu_frames) <= self.num_imu_frames:
                break
            if self.states[sid].is_keyframe:
                self.imu_frames.discard(sid)
                self.key_frames.add(sid)
            else:
                self.remove_all_observations(sid)
                merges.append(sid)
                self.imu_frames.discard(sid)
        if merges:
            self.eliminate_by_imu_merge(merges)

    def eliminate_by_imu_merge(self, sids):
        """ViGraphEstimator::eliminateStateByImuMerge (ViGraphEstimator.cpp:38-171) for a batch of
        states (one okvisgpu_imu_append call): the link into the state is appended with the link out
        of it (ImuError::append at the state's speed/bias estimate), the state and its links go."""
        for sid in sids:
            assert not any(sid in e for e in self.edges), "no pose-graph edges at an IMU frame"
        ids = self.ids()
        plan = []
        for sid in sids:
            i = ids.index(sid)
            prev, nxt = ids[i - 1], ids[i + 1]
            plan.append((prev, sid, nxt))
            ids.pop(i)
        state = np.ascontiguousarray([self.links[(p, s)].state for p, s, _ in plan]).reshape(-1, IMU_STATE_DOUBLES)
        nxt_links = [self.links[(s, n)] for _, s, n in plan]
        begin = np.cumsum([0] + [len(l.ts) for l in nxt_links]).astype(np.int32)
        steps = self.backend.imu_append(self.world.imu_params, state, [self.links[(p, s)].t1 for p, s, _ in plan],
                                        [l.t1 for l in nxt_links], [self.states[s].sb for _, s, _ in plan], begin,
                                        np.concatenate([l.ts for l in nxt_links]),
                                        np.concatenate([l.ga for l in nxt_links]))
        for k, (p, s, n) in enumerate(plan):
            assert steps[k] > 0, f"IMU merge of state {s}: samples do not reach t1"
            a, b = self.links.pop((p, s)), self.links.pop((s, n))
            newer = b.ts > a.ts[-1]  # ImuError.cpp:74-81
            self.links[(p, n)] = ImuLink(a.t0, b.t1, np.r_[a.ts, b.ts[newer]], np.r_[a.ga, b.ga[newer]], state[k].copy())
            del self.states[s]
            self.log.append(("imu_merge", s, p, n, int(steps[k])))

    def build_mst(self, frames, co):
        """ViGraphEstimator::buildMst (ViGraphEstimator.cpp:935-990) + MstGraph::kruskalMst
        (MstGraph.hpp:132-169): edges (-covisibility, (idx of larger id, idx of smaller id)) sorted
        ascending, accepted when they join two components."""
        ids = sorted(frames)
        idx = {f: i for i, f in enumerate(ids)}
        edges = sorted((-c, (idx[a], idx[b])) for (a, b), c in co.items() if a in idx and b in idx)
        parent = list(range(len(ids) + 1))

        def find(u):
            while parent[u] != u:
                parent[u] = parent[parent[u]]
                u = parent[u]
            return u

        out = []
        for _, (u, v) in edges:
            su, sv = find(u), find(v)
            if su != sv:
                out.append((u, v))
                parent[su] = sv
        return ids, idx, out

    def convert_to_pose_graph_mst(self, states, to_consider):
        """ViGraphEstimator::convertToPoseGraphMst (ViGraphEstimator.cpp:334-610). The edges' compute
        inputs are collected in edge order (observation removal of earlier edges shapes later ones)
        and computed in one okvisgpu_twopose_compute batch (compute changes no estimate)."""
        co = self.covisibilities()
        ids, idx, mst = self.build_mst(to_consider, co)
        if not mst:
            return False
        num_edges = {}
        for u, v in mst:
            for f in (ids[u], ids[v]):
                num_edges[f] = num_edges.get(f, 0) + 1
        create = [(u, v) for u, v in mst if ids[u] in states or ids[v] in states]
        newest, oldest = ids[-1], ids[0]
        if oldest in states and self.covis(co, newest, oldest) >= 2 and newest != oldest:
            if not any({u, v} == {idx[oldest], idx[newest]} for u, v in create):
                create.append((idx[oldest], idx[newest]))
                num_edges[oldest] = num_edges.get(oldest, 0) + 1
                num_edges[newest] = num_edges.get(newest, 0) + 1
        pending = []
        for u, v in create:
            ref, other = min(ids[u], ids[v]), max(ids[u], ids[v])
            if (ref, other) in self.edges:
                raise NotImplementedError("re-converting an existing pose-graph edge (convertToReprojectionErrors)")
            keep_ref = num_edges[ref] > 1 or ref not in states
            keep_other = num_edges[other] > 1 or other not in states
            ref_obs = sorted(k for k in self.obs if k[0] == ref)
            other_obs = sorted(k for k in self.obs if k[0] == other)
            considered = {k[2] for k in ref_obs} & {k[2] for k in other_obs}
            per_lm = {}
            for side, keys, keep in ((False, ref_obs, keep_ref), (True, other_obs, keep_other)):
                for key in keys:
                    if key[2] in considered:
                        kp, L = self.obs[key]
                        per_lm.setdefault(key[2], []).append((side, key[1], kp.copy(), L.copy(), True))
                    if not keep:
                        del self.obs[key]
            if considered:
                lms = sorted(per_lm)
                pending.append(((ref, other), {
                    "ref_pose": self.states[ref].pose.copy(), "other_pose": self.states[other].pose.copy(),
                    "landmarks": np.array([self.landmarks[l] for l in lms]),
                    "observations": [per_lm[l] for l in lms]}))
            num_edges[ref] -= 1
            num_edges[other] -= 1
        if pending:
            batch = TwoPoseBatch([e for _, e in pending], self.world.cameras, self.world.extrinsics)
            out = self.backend.twopose(batch)
            for i, (key, e) in enumerate(pending):
                self.edges[key] = Edge(out["delta_x"][i].copy(), out["sqrt_info"][i].copy(), out["lin_point"][i].copy())
                self.log.append(("edge", key, len(e["landmarks"])))
        return True

    def freeze(self):
        """ViSlamBackend::applyStrategy "freeze old states" (ViSlamBackend.cpp:669-712)."""
        ids = self.ids()
        n = self.num_keyframes + self.num_imu_frames
        if len(ids) <= n:
            return
        pos = len(ids) - 1 - n
        ctr = 0
        while True:
            if ctr == self.num_rt_pg_frames:
                t_freeze = self.states[ids[-1]].t_ns
                while (t_freeze - self.states[ids[pos]].t_ns) * 1e-9 < self.min_delta_t:
                    if pos == 0:
                        break
                    pos -= 1
                if pos != 0:
                    fid = ids[pos] if self.last_freeze is None else max(self.last_freeze, ids[pos])
                    self.last_freeze = fid
                    if fid != ids[0]:
                        self._freeze_until(fid, "pose_fixed")
                    self._freeze_until(fid, "sb_fixed")
                    self.log.append(("freeze", fid))
                break
            if pos == 0:
                break
            ctr += 1
            pos -= 1

    def _freeze_until(self, fid, attr):
        """freezePosesUntil / freezeSpeedAndBiasesUntil (ViGraphEstimator.cpp:216-298),
        removeInCeres = false: constant blocks, kept in the problem."""
        for sid in reversed([s for s in self.ids() if s <= fid]):
            if getattr(self.states[sid], attr):
                break
            setattr(self.states[sid], attr, True)

    def apply_strategy(self):
        """ViSlamBackend::applyStrategy (ViSlamBackend.cpp:555-809), VIO mode (no loop closures)."""
        self.eliminate_imu_frames()
        co = self.covisibilities()
        cur = self.ids()[-1]
        if self.most_overlapped(cur, co) is None:
            return
        eliminated, ctr_pg = False, 0
        while len(self.key_frames) > self.num_keyframes:
            co = self.covisibilities()
            cur = self.ids()[-1]
            cur_kf = self.most_overlapped(cur, co)
            kfs = sorted(self.key_frames)
            min_id, min_obs = None, 100000
            for kf in kfs:
                c = max(self.covis(co, cur, kf), self.covis(co, cur_kf, kf))
                if kf == kfs[0] and c >= 2:
                    continue  # spare
                if c < min_obs:
                    min_obs, min_id = c, kf
            max_id, max_co, consider = None, 0, set()
            for f in kfs:
                c = self.covis(co, min_id, f)
                if c >= max_co:
                    max_id, max_co = f, c
                if any(f in e for e in self.edges):
                    consider.add(f)  # frontier node
            self.states[min_id].pose_graph_frame = True
            self.key_frames.discard(min_id)
            consider |= {min_id, max_id}
            eliminated = True
            self.log.append(("to_pose_graph", min_id, max_id, max_co))
            if max_co == 0:
                self.remove_all_observations(min_id)
                continue
            self.convert_to_pose_graph_mst({min_id}, consider)
            ctr_pg += 1
            assert not any(k[0] == min_id for k in self.obs), f"observations left at {min_id}"
            if ctr_pg >= 3:
                break
        if eliminated:
            self.freeze()
        # expandKeyframe (ViSlamBackend.cpp:790-806): the current keyframe as a frontier node
        co = self.covisibilities()
        cur_kf = self.most_overlapped(self.ids()[-1], co)
        if ctr_pg < 3 and cur_kf is not None and any(cur_kf in e for e in self.edges):
            raise NotImplementedError(f"expandKeyframe({cur_kf}) is not restated")

    def step(self, k):
        """One frame: add it, solve the realtime window, apply the marginalisation strategy."""
        self.add_frame(k)
        self.clean_unobserved_landmarks()
        s = self.optimise()
        self.apply_strategy()
        return s


class _OwnedProblem:
    """numpy-owned okvisgpu_problem (plain data)."""
    _F = {"poses": np.float64, "pose_constant": np.uint8, "speed_biases": np.float64,
          "speed_bias_constant": np.uint8, "landmarks": np.float64, "extrinsics": np.float64,
          "obs_pose": np.int32, "obs_landmark": np.int32, "obs_camera": np.int32, "obs_keypoint": np.float64,
          "obs_sqrt_info": np.float64, "obs_cauchy": np.uint8, "imu_blocks": np.int32, "imu_t0_ns": np.int64,
          "imu_t1_ns": np.int64, "imu_sample_begin": np.int32, "imu_sample_t_ns": np.int64,
          "imu_sample_gyr_acc": np.float64, "imu_state": np.float64, "pose_prior_block": np.int32,
          "pose_prior_meas": np.float64, "pose_prior_sqrt_info": np.float64, "sb_prior_block": np.int32,
          "sb_prior_meas": np.float64, "sb_prior_sqrt_info": np.float64, "relpose_blocks": np.int32,
          "relpose_delta_x": np.float64, "relpose_sqrt_info": np.float64, "relpose_lin_point": np.float64,
          "relpose_kind": np.uint8, "extrinsics_constant": np.uint8, "extrinsics_prior_camera": np.int32,
          "extrinsics_prior_meas": np.float64, "extrinsics_prior_sqrt_info": np.float64}
    _PTR = {np.float64: C.POINTER(C.c_double), np.int32: _ip, np.int64: _lp, np.uint8: _up}

    def __init__(self):
        for k, dt in self._F.items():
            setattr(self, k, np.zeros(0, dtype=dt))
        self.cameras = []
        self.imu_params = ImuParams()
        self.struct = Problem()

    def ptr(self):
        return C.pointer(self.struct)

    def snapshot(self):
        return {k: getattr(self, k).copy() for k in ("poses", "speed_biases", "landmarks", "imu_state")}

    def restore(self, snap):
        for k, v in snap.items():
            getattr(self, k)[...] = v

    def bind(self):
        s = self.struct
        for k, dt in self._F.items():
            a = np.ascontiguousarray(getattr(self, k), dtype=dt)
            setattr(self, k, a)
            setattr(s, k, a.ctypes.data_as(self._PTR[dt]) if a.size else None)
        s.n_poses = len(self.poses)
        s.n_speed_biases = len(self.speed_biases)
        s.n_landmarks = len(self.landmarks)
        s.n_cameras = len(self.cameras)
        s.n_observations = len(self.obs_pose)
        s.n_imu = len(self.imu_blocks)
        s.n_pose_priors = len(self.pose_prior_block)
        s.n_sb_priors = len(self.sb_prior_block)
        s.n_relpose = len(self.relpose_blocks)
        s.n_extrinsics_priors = len(self.extrinsics_prior_camera)
        self._cams = (Camera * max(1, len(self.cameras)))(*self.cameras)
        s.cameras = self._cams
        if s.n_imu == 0:
            s.imu_sample_begin = s.imu_sample_t_ns = s.imu_sample_gyr_acc = None
        s.imu_params = self.imu_params
        return self
