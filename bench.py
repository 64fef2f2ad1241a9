#!/usr/bin/env python3
"""bench.py — Gauss-Newton (dogleg trust-region) iterations/s of the MI355X okvis_ceres backend.

Metric (BASELINE.json): "Gauss-Newton iters/sec on 50-KF/2000-landmark window; ATE vs CPU ref".
A step = one trust-region iteration (Ceres semantics: linearise + Schur-reduce + LLT + dogleg +
candidate evaluation + accept/reject) of EVERY window in the job's batch of independent synthetic
S50 windows (50 keyframes, 2,000 landmarks, 16,000 reprojections, 49 IMU factors).
value = (windows x timed iterations) / wall time of the timed region, max over ranks
(window-iterations per second, whole job). Strong scaling (BASELINE.json north_star: ">=6x strong
scaling at 8 GPUs on batched independent windows"): the job is a fixed batch of --windows
independent windows (2,048 by default) split across the ranks, one process per GPU and no
data-path collective. --windows-per-gpu W instead gives every rank its own W
windows (weak scaling, distinct seeds across ranks). At the end of the
run the per-window summaries and final poses are all-gathered to rank 0 over RCCL (§8e), outside
the timed region, and rank 0 checks that every window of the job ran every iteration.

`--gpus N` without a launcher starts N ranks itself: a `torch.distributed.run` child process
(this process never touches the GPU), one rank per GPU, 127.0.0.1 rendezvous.

All tolerances are set to 0 so every timed iteration does real work (the K-iteration protocol of
BASELINE.md); inputs are resident in HBM before the timed region.

Also reported (rank 0): the single-window latency mode (the reference's own use: one window per
::ceres::Solve) — resident iters/s and the end-to-end set_problems + solve wall time; per-kernel
device time of one iteration (HIP events on the context's stream); the roofline of the dominant
kernel against both the builder's byte model and SURVEY.md §8(d)'s compulsory bytes, plus the
whole-iteration §8(d) HBM fraction; accuracy (ATE of window 0 vs ground truth for GPU and CPU
oracle, max pose deviation); the CPU baseline = the repo's CPU restatement (oracle/liboracle.so,
"port") at realtime_num_threads = 3 and at all host cores given to the job, median of 5.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "okvis2-x_amd"))

FP64_MFMA_PEAK_TFLOPS = 78.6   # MI355X FP64 matrix (spec; SURVEY.md §8d, not in the gfx950 guide)
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md chip table (spec)
SEED0 = 20251015
DEFAULT_WINDOWS = 2048         # the job's fixed batch of independent S50 windows (strong scaling)
METRIC = "Gauss-Newton iters/sec on 50-KF/2000-landmark window; ATE vs CPU ref"

CONFIGS = {
    "s50": dict(n_kf=50, n_lm=2000, n_obs=16000),
    "s10": dict(n_kf=10, n_lm=500, n_obs=4000),
}

# summary columns gathered to rank 0 (cost, iterations, status per window)
SUMMARY_COLS = ("window", "initial_cost", "final_cost", "num_iterations", "num_successful_steps",
                "termination_type")


def og_module():
    import okvisgpu
    return okvisgpu


def bench_options(max_iter):
    # all tolerances 0: every iteration is performed (BASELINE.md timing protocol)
    return og_module().default_options(max_num_iterations=max_iter, function_tolerance=0.0,
                                       gradient_tolerance=0.0, parameter_tolerance=0.0)


def make_windows(cfg, indices):
    """Synthetic windows, generated on host threads (the C generator runs outside the GIL)."""
    from concurrent.futures import ThreadPoolExecutor
    og = og_module()
    indices = list(indices)
    mk = lambda i: og.SynthWindow(cfg["n_kf"], cfg["n_lm"], cfg["n_obs"], seed=SEED0 + i)  # noqa: E731
    if len(indices) < 16:
        return [mk(i) for i in indices]
    with ThreadPoolExecutor(max_workers=min(16, host_threads())) as ex:
        return list(ex.map(mk, indices))


def host_threads():
    """Host cores given to this job: OMP_NUM_THREADS when the launcher sets it (16 per GPU on the
    MI355X box), else the CPU affinity mask."""
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def ate(P, gt):
    """SE(3)-aligned RMSE of keyframe positions (Horn/Umeyama without scale)."""
    a, b = P[:, :3], gt[:, :3]
    ma, mb = a.mean(0), b.mean(0)
    H = (a - ma).T @ (b - mb)
    U, _, Vt = np.linalg.svd(H)
    D = np.eye(3)
    D[2, 2] = np.sign(np.linalg.det(Vt.T @ U.T))
    R = Vt.T @ D @ U.T
    aligned = (R @ (a - ma).T).T + mb
    return float(np.sqrt(np.mean(np.sum((aligned - b) ** 2, axis=1))))


PMC_TRAFFIC = os.path.join(REPO, "profiles", "pmc_traffic.json")
# MFMA counters of the newest round that collected them (scripts/gpu_pmc_calib.sh)
PMC_CALIBS = [os.path.join(REPO, "profiles", f) for f in ("r06_pmc_calib.json", "r05_pmc_calib.json")]


def pmc_mfma():
    """MFMA counters of k_cholesky on this workload (scripts/gpu_pmc_calib.sh ->
    profiles/rNN_pmc_calib.json, the newest round's): the busy fraction of the matrix cores and the FLOPs the counted
    v_mfma_f64_16x16x4f64 instructions perform, or None."""
    for path in PMC_CALIBS:
        try:
            with open(path) as f:
                d = json.load(f)["k_cholesky_mfma"]
            return {"mfma_busy_frac": d["mfma_busy_frac"], "mfma_flops_per_dispatch": d["mfma_flops"],
                    "windows": 2048,
                    "source": f"profiles/{os.path.basename(path)} (SQ_VALU_MFMA_BUSY_CYCLES, SQ_INSTS_VALU_MFMA_F64, "
                              "GRBM_GUI_ACTIVE; 2,048 S50 windows)"}
        except (OSError, KeyError, ValueError, TypeError):
            continue
    return None


def issued_frac(d, windows, n_windows):
    """k_cholesky's FP64 matrix-core rate on the FLOPs its MFMA instructions perform (counted by
    SQ_INSTS_VALU_MFMA_F64 on 2,048 S50 windows, scaled per window) over the event-timed launch,
    beside the algorithmic `frac`; None without the counter file."""
    m = pmc_mfma()
    if not m or d["ms"] <= 0 or not n_windows:
        return None
    flops = m["mfma_flops_per_dispatch"] / m.get("windows", 2048) * windows
    return flops / (d["ms"] * 1e-3) / 1e12 / FP64_MFMA_PEAK_TFLOPS


def rank_windows(total, world, rank):
    """This rank's contiguous share of the job's windows."""
    per = [total // world + (1 if r < total % world else 0) for r in range(world)]
    start = sum(per[:rank])
    return list(range(start, start + per[rank]))


def job_windows(args, world):
    """Resolve the job's window count: --windows-per-gpu gives every rank its own batch (weak
    scaling), else the job is --windows windows split across the ranks (strong scaling, the
    default). Returns True for strong scaling."""
    if args.windows_per_gpu is not None:
        if args.windows is not None:
            raise SystemExit("bench.py: --windows and --windows-per-gpu are exclusive")
        args.windows = args.windows_per_gpu * world
        return False
    if args.windows is None:
        args.windows = DEFAULT_WINDOWS
    return True


def aggregate(dist, elapsed, early, device):
    """Max of the timed region over ranks, sum of early-terminated windows."""
    if dist is None:
        return elapsed, early
    import torch
    t = torch.tensor([elapsed, float(early)], dtype=torch.float64, device=device)
    tmax, tsum = t.clone(), t.clone()
    dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    dist.all_reduce(tsum, op=dist.ReduceOp.SUM)
    return float(tmax[0].item()), int(tsum[1].item())


def gather_rows(dist, rows, total, device):
    """SURVEY.md §8e end-of-run gather: every rank holds the rows of its windows (rank_windows
    order, float64 [n_mine, k]); returns the [total, k] array of the whole job on every rank (one
    all_gather over RCCL/xGMI on the GPU box, gloo in the CPU tests). Ranks may hold different
    counts (total % world != 0): rows are padded to the largest share and trimmed after."""
    rows = np.ascontiguousarray(rows, dtype=np.float64)
    if dist is None:
        return rows
    import torch
    world = dist.get_world_size()
    counts = [len(rank_windows(total, world, r)) for r in range(world)]
    per = max(counts)
    k = rows.shape[1]
    buf = torch.zeros((per, k), dtype=torch.float64, device=device)
    if len(rows):
        buf[: len(rows)] = torch.from_numpy(rows).to(device)
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf)
    return np.concatenate([p[:c].cpu().numpy() for p, c in zip(parts, counts)], axis=0)


def summary_rows(mine, sums):
    return np.array([[i, s["initial_cost"], s["final_cost"], s["num_iterations"], s["num_successful_steps"],
                      s["termination_type"]] for i, s in zip(mine, sums)], dtype=np.float64).reshape(-1, len(SUMMARY_COLS))


def roofline_table(ctx, reps):
    """Per-kernel device time (HIP events on the context's stream, `reps` back-to-back launches of
    one iteration's worth on the resident data) and achieved rate of its algorithmic work."""
    og = og_module()
    table = {}
    for name in og.kernel_names():  # every kernel okvisgpu_time_kernel exposes
        ms, work, bound = ctx.time_kernel(name, reps)
        rate = work / (ms * 1e-3) / (1e9 if bound == "hbm" else 1e12) if ms > 0 else 0.0
        peak = HBM_PEAK_GBS if bound == "hbm" else FP64_MFMA_PEAK_TFLOPS
        table[name] = {"ms": ms, "bound": bound, "work": work, "achieved": rate, "peak": peak, "frac": rate / peak}
    return table


def survey_bytes(st):
    """SURVEY.md §8(d) compulsory HBM bytes of one iteration of the whole batch, with S counted
    tile-sparse (the 64x64 tiles the LLT touches instead of d(d+1)/2), and its split onto the
    kernels that own each term (VERDICT r01 decomposition). Returns (whole_iteration, per_kernel)."""
    obs = 48.0 * st["n_observations"]                       # meas 16 + sqrtInfo 24 + idx 8
    lm_rw = 2 * 4 * 8.0 * st["n_landmarks_free"]            # landmark read + write
    params = 2 * 8.0 * (7 * st["n_poses"] + 9 * st["n_speed_biases"]) + lm_rw
    imu = 2336.0 * st["n_imu"]                              # ImuError state 292 doubles
    s_tiles = 64 * 64 * 8.0 * st["s_tiles_nonzero"]
    vinv = 2 * 9 * 8.0 * st["n_landmarks_free"]            # per-landmark V^-1 / rhs
    whole = obs + params + imu + 4 * s_tiles + vinv
    per = {
        "k_lm_visit": obs + lm_rw + vinv,                   # linearisation + landmark elimination
        "k_cholesky": 3 * s_tiles,                          # read S, write L, read L for the solves
        "k_assemble_pp": s_tiles,                           # write S (pose-pose and speed/bias blocks
        "k_eval_obs": obs + params,                         #  counted on the larger kernel)
        "k_eval_imu": imu,
    }
    return whole, per


def pmc_traffic(kernel, windows):
    """HBM bytes per iteration of `kernel` over `windows` windows from the committed rocprofv3 --pmc
    summary (scripts/pmc_traffic.py: FETCH_SIZE x 2 per the gfx950 calibration + WRITE_SIZE, measured
    per window-iteration on the default workload), or None."""
    try:
        with open(PMC_TRAFFIC) as f:
            d = json.load(f)
        return d["kernels"][kernel]["bytes_per_window_iteration"] * windows
    except (OSError, KeyError, ValueError, TypeError):
        return None


def run_cpu_baseline(cfg, iters, threads, n_windows, reps):
    """Oracle (CPU restatement, `port`) on the first `n_windows` windows of the workload, same
    options and iteration count; median over `reps` timed passes after one warm-up pass. Bounded
    sample of the same workload, reported in the metric's unit (window-iterations/s)."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import _oracle  # noqa: E402  (bench.py's cpu_baseline leg is an allowed oracle user)
    ws = make_windows(cfg, range(n_windows))
    opts = bench_options(iters)
    opts.num_threads = threads
    times, s0 = [], None
    for r in range(reps + 1):
        t0 = time.perf_counter()
        for i, w in enumerate(ws):
            w.reset()
            s = _oracle.solve(w.problem_ptr(), opts)
            if i == 0:
                s0 = s
        if r > 0:
            times.append(time.perf_counter() - t0)
    return ws[0], s0, float(np.median(times))


def run_cpu_baseline_batch(cfg, iters, host_threads, n_windows, reps):
    """Like-for-like CPU batch: `host_threads` workers each solve their own windows with one solver
    thread (num_threads = 1), all in flight together, like the GPU's batch of independent windows.
    The oracle's C solve runs without the GIL (ctypes), so the workers run in parallel. Returns the
    median wall time of `reps` passes over `n_windows` windows after one warm-up pass."""
    from concurrent.futures import ThreadPoolExecutor
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import _oracle  # noqa: E402  (bench.py's cpu_baseline leg is an allowed oracle user)
    ws = make_windows(cfg, range(n_windows))
    opts = bench_options(iters)
    opts.num_threads = 1

    def one(w):
        w.reset()
        return _oracle.solve(w.problem_ptr(), opts)["num_iterations"]

    times = []
    with ThreadPoolExecutor(max_workers=host_threads) as ex:
        for r in range(reps + 1):
            t0 = time.perf_counter()
            its = list(ex.map(one, ws))
            if r > 0:
                times.append(time.perf_counter() - t0)
            assert all(i == iters for i in its), its
    return float(np.median(times))


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(argv, n):
    """One process per GPU without an external launcher: run `torch.distributed.run` as a CHILD
    process (this parent never touches the GPU and does not exec) and return its exit code."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(cmd, env=env).returncode


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--windows", type=int, default=None,
                    help=f"job total split across ranks (strong scaling, default {DEFAULT_WINDOWS})")
    ap.add_argument("--windows-per-gpu", type=int, default=None, help="windows per rank instead (weak scaling)")
    ap.add_argument("--config", default="s50", choices=sorted(CONFIGS))
    ap.add_argument("--cpu-threads", type=int, default=3, help="realtime_num_threads (okvis2.yaml:93)")
    ap.add_argument("--cpu-iters", type=int, default=None, help="default: warmup + steps")
    ap.add_argument("--cpu-reps", type=int, default=5, help="median of this many timed passes after 1 warm-up")
    ap.add_argument("--cpu-windows", type=int, default=24, help="windows in the realtime (one at a time) CPU sample")
    ap.add_argument("--cpu-batch-windows", type=int, default=None,
                    help="windows in the batch CPU sample (default: 3 per host thread)")
    ap.add_argument("--kernel-reps", type=int, default=5, help="repetitions per kernel in the roofline table")
    ap.add_argument("--e2e-reps", type=int, default=5, help="single-window set_problems + solve repetitions")
    ap.add_argument("--cholesky-schedule", type=int, default=0, help="0 auto, 1 persistent per window, 2 tile-parallel, 3 persistent split over a nested-dissection window, 4 pipelined persistent (two teams per window), 5 split with each part pipelined")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-latency", action="store_true")
    ap.add_argument("--no-profile", action="store_true")
    return ap.parse_args(argv)


def single_window(og, cfg, opts, args, device):
    """The reference's own use: ONE window per ::ceres::Solve. Resident iters/s (K iterations timed
    between two synchronisations) and the end-to-end wall time a ViGraph caller sees for a fresh
    window: okvisgpu_set_problems (host structure analysis + upload) + okvisgpu_solve (K iterations +
    write-back), median over repetitions."""
    w1 = make_windows(cfg, [0])
    c1 = og.Context(device)
    c1.set_problems([w1[0].problem])
    c1.solve_begin(opts)
    c1.solve_iterate(args.warmup)
    c1.synchronize()
    a = time.perf_counter()
    c1.solve_iterate(args.steps)
    c1.synchronize()
    b = time.perf_counter()
    s1 = c1.solve_end()[0]
    st1 = c1.stats()
    out = {"iters_per_s": args.steps / (b - a), "ms_per_iter": (b - a) / args.steps * 1e3,
           "final_cost": s1["final_cost"], "cholesky_launches": st1["cholesky_launches"],
           "s_tiles_nonzero": st1["s_tiles_nonzero"]}
    gpu_pose = w1[0].poses().copy()
    gt_p, _, _ = w1[0].ground_truth()
    e2e = []
    total_iters = args.warmup + args.steps
    for _ in range(args.e2e_reps + 1):
        w1[0].reset()
        t0 = time.perf_counter()
        c1.set_problems([w1[0].problem])
        c1.solve(opts)
        e2e.append(time.perf_counter() - t0)
    e2e = float(np.median(e2e[1:]))
    out["e2e_set_problems_plus_solve_ms"] = e2e * 1e3
    out["e2e_iterations"] = total_iters
    out["e2e_iters_per_s"] = total_iters / e2e
    if not args.no_profile:
        # which iterations of window 0 re-integrate IMU factors (ImuError::redoPreintegration,
        # counted by redoCounter_ = imu_state[:, 0]): solves of 0..K iterations from the same start
        # (the same bits up to their last iteration), the counters written back after each; entry n
        # is the number of factors re-integrated during iteration n (entry 0: the initial evaluation)
        o2 = bench_options(total_iters)
        o2.cholesky_schedule = opts.cholesky_schedule
        counts = []
        for n in range(total_iters + 1):
            w1[0].reset()
            c1.update_params()
            o2.max_num_iterations = n
            c1.solve(o2)
            counts.append(float(w1[0].imu_state()[:, 0].sum()))
        per = [int(round(counts[0]))] + [int(round(counts[n] - counts[n - 1])) for n in range(1, len(counts))]
        out["imu_reintegrated_factors_per_iteration"] = per
        later = [n for n in range(1, len(per)) if per[n] > 0]
        last = later[-1] if later else 0
        out["imu_last_reintegrating_iteration"] = last
        out["imu_factors"] = int(w1[0].problem.n_imu)
        # per-phase device times of one real iteration (eager launches between HIP events): the
        # steady state = the first iteration after the last one that re-integrates (the biases have
        # settled, the candidate evaluations keep the IMU preintegration), and the first iteration of
        # the solve (the biases still move: ImuError re-integrates, ImuError.cpp:834-858); plus the
        # forced re-integration of every factor of the window (okvisgpu_time_kernel)
        steady = min(last, total_iters - 1)
        out["steady_state_iteration"] = steady + 1
        # (eager launches with an event at every phase boundary: their sum exceeds the captured
        # graph's iteration by the events' own cost, ~4.5 us per boundary on MI355X)
        for key, it in (("kernel_ms_per_iteration", steady), ("kernel_ms_first_iteration", 0)):
            w1[0].reset()
            c1.update_params()
            c1.solve_begin(opts)
            c1.solve_iterate(it)
            ph1 = c1.profile_iteration()
            c1.solve_end()
            out[key] = {k: round(v, 4) for k, v in ph1.items()}
            out[key + "_sum"] = round(sum(ph1.values()), 4)
        # the same iterations as the solve runs them (the captured graph, wall time like
        # iters_per_s): ms_per_iteration = the steady state (the iterations after the last
        # re-integrating one), ms_first_iteration = the leading re-integrating iterations
        def graph_ms(start, n):
            w1[0].reset()
            c1.update_params()
            c1.solve_begin(opts)
            c1.solve_iterate(start)
            c1.synchronize()
            a = time.perf_counter()
            c1.solve_iterate(n)
            c1.synchronize()
            ms = (time.perf_counter() - a) / n * 1e3
            c1.solve_end()
            return ms
        out["ms_per_iteration"] = round(graph_ms(steady, total_iters - steady), 4)
        first_n = max(1, next((n for n in range(1, len(per)) if per[n] == 0), len(per)) - 1)
        out["ms_first_iteration"] = round(graph_ms(0, first_n), 4)
        out["first_iterations_timed"] = first_n
        w1[0].reset()
        c1.update_params()
        out["eval_imu_forced_reintegration_ms"] = round(c1.time_kernel("k_eval_imu", 5)[0], 4)
    c1.close()
    return out, gpu_pose, gt_p


def dry_run(args, world, rank):
    """Launcher / gather plumbing without a GPU (tests/test_multirank.py): every rank takes its share,
    the window summaries go through the same gather over gloo, rank 0 prints what it received."""
    dist = None
    if world > 1:
        import torch.distributed as tdist
        tdist.init_process_group("gloo")
        dist = tdist
    job_windows(args, world)
    mine = rank_windows(args.windows, world, rank)
    rows = np.array([[i, 0.0, float(i), args.warmup + args.steps, 1, 0] for i in mine]).reshape(-1, len(SUMMARY_COLS))
    got = gather_rows(dist, rows, args.windows, "cpu")
    if rank == 0:
        print(json.dumps({"world": world, "gpus": args.gpus, "windows": int(len(got)),
                          "in_order": bool(np.array_equal(got[:, 0], np.arange(args.windows))),
                          "master_addr": os.environ.get("MASTER_ADDR")}), flush=True)
    if dist:
        dist.destroy_process_group()
    return 0


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse_args(argv)
    world_env = os.environ.get("WORLD_SIZE")
    if args.gpus > 1 and world_env is None:
        return launch_ranks(argv, args.gpus)
    world = int(world_env or "1")
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        return 2
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("OKVISGPU_BENCH_DRYRUN") == "1":
        return dry_run(args, world, rank)
    import torch
    og = og_module()
    dist = None
    device = f"cuda:{local_rank}"
    if world > 1:
        import torch.distributed as tdist
        torch.cuda.set_device(local_rank)
        tdist.init_process_group("nccl")
        dist = tdist
        assert dist.get_world_size() == args.gpus
    cfg = CONFIGS[args.config]

    # ---- this rank's windows: its own batch (weak scaling) or a share of a fixed total (strong)
    strong = job_windows(args, world)
    mine = rank_windows(args.windows, world, rank)
    windows = make_windows(cfg, mine)
    ctx = og.Context(local_rank)
    ctx.set_problems([w.problem for w in windows])
    stats = ctx.stats()
    total_iters = args.warmup + args.steps
    opts = bench_options(total_iters)
    opts.cholesky_schedule = args.cholesky_schedule

    ctx.solve_begin(opts)
    ctx.solve_iterate(args.warmup)
    ctx.synchronize()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    ctx.solve_iterate(args.steps)
    ctx.synchronize()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if dist:
        dist.barrier()
    sums = ctx.solve_end()
    elapsed = t1 - t0
    early = sum(1 for s in sums if s["num_iterations"] < total_iters)
    gn_frac = float(np.mean([(s["num_successful_steps"] - 1) / max(1, s["num_iterations"]) for s in sums]))
    elapsed, early = aggregate(dist, elapsed, early, device)

    # ---- §8e end-of-run gather (outside the timed region): summaries + final poses to every rank
    g0 = time.perf_counter()
    all_sums = gather_rows(dist, summary_rows(mine, sums), args.windows, device)
    all_poses = gather_rows(dist, np.stack([w.poses().reshape(-1) for w in windows]), args.windows, device)
    gather_s = time.perf_counter() - g0

    # per-solve rate including the PCIe upload of the parameters and the write-back (not `value`)
    for w in windows:
        w.reset()
    ctx.synchronize()
    a = time.perf_counter()
    ctx.solve(opts)  # okvisgpu_solve uploads the parameters itself
    pcie_s = time.perf_counter() - a

    value = args.windows * args.steps / elapsed
    result = {
        "metric": METRIC,
        "value": value,
        "unit": "window-iterations/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (EuRoC stereo rig, 200 Hz IMU, seeded windows; SURVEY.md §8d)",
        "config": {
            "workload": f"{args.windows} independent {args.config.upper()} windows "
                        f"({cfg['n_kf']} KF / {cfg['n_lm']} landmarks / {cfg['n_obs']} reprojections, "
                        f"{cfg['n_kf'] - 1} IMU factors), DENSE_SCHUR + DOGLEG, all tolerances 0",
            "windows_total": args.windows,
            "windows_per_gpu": len(mine),
            "parallelism": f"replicas x{world} (one window batch per GPU, no collective in the loop)",
        },
    }

    if args.cpu_iters is None:
        args.cpu_iters = total_iters
    if rank == 0:
        ran_k = bool(np.all(all_sums[:, 3] == total_iters)) and len(all_sums) == args.windows
        result["gather"] = {
            "windows": int(len(all_sums)), "all_windows_ran_k_iterations": ran_k,
            "windows_in_order": bool(np.array_equal(all_sums[:, 0], np.arange(args.windows))),
            "final_cost_sum": float(all_sums[:, 2].sum()), "pose_bytes": int(all_poses.nbytes),
            "ms": gather_s * 1e3,
            "collective": "all_gather (RCCL over xGMI)" if dist else "none (1 rank)",
        }
        result["early_terminated_windows"] = early
        result["per_solve_incl_pcie"] = {"wall_s": pcie_s, "iterations": total_iters,
                                         "window_iterations_per_s": len(windows) * total_iters / pcie_s}
        result["frac_iterations_with_gn_solve"] = gn_frac
        result["problem_stats_per_gpu"] = stats
        # ---- single-window latency mode (1 window, this GPU): the reference's own use
        if not args.no_latency:
            sw, gpu_pose_w0, gt_p = single_window(og, cfg, opts, args, local_rank)
            result["single_window"] = sw
            result["single_window_iters_per_s"] = sw["iters_per_s"]
        # ---- roofline: per-kernel device time on the resident batch, dominant kernel by time
        if not args.no_profile:
            table = roofline_table(ctx, args.kernel_reps)
            dominant = max(table, key=lambda k: table[k]["ms"])
            d = table[dominant]
            traffic = pmc_traffic(dominant, len(mine))
            whole, per = survey_bytes(stats)
            ms_it = elapsed / args.steps * 1e3
            survey = {k: {"bytes": v, "achieved_GBs": v / (table[k]["ms"] * 1e6),
                          "frac": v / (table[k]["ms"] * 1e6) / HBM_PEAK_GBS} for k, v in per.items() if k in table}
            result["roofline"] = {
                "kernel": dominant, "bound": d["bound"], "achieved": d["achieved"], "peak": d["peak"],
                "unit": "GB/s" if d["bound"] == "hbm" else "TFLOP/s", "frac": d["frac"],
                "traffic": traffic,
                "traffic_calibration": "FETCH_SIZE x2, WRITE_SIZE x1: measured for this code's 16-B, 8-B and "
                                       "tile-row access shapes (scripts/pmc_calib.hip, profiles/rNN_pmc_calib.json)",
                "counters": pmc_mfma() if dominant == "k_cholesky" else None,
                "frac_issued": issued_frac(d, len(mine), stats["n_windows"]) if dominant == "k_cholesky" else None,
                "work_per_iteration": d["work"], "ms_per_iteration": d["ms"],
                "frac_survey_8d": survey.get(dominant, {}).get("frac") if d["bound"] == "hbm" else None,
                "method": f"HIP events on the context stream, {args.kernel_reps} launches of one iteration's "
                          "worth on the resident batch; work = algorithmic bytes/FLOPs of the builder's model "
                          "(DESIGN.md §4; for k_cholesky the FP64 flops of the tile-sparse LLT: n^3/3 per "
                          "diagonal potrf, n^3 per panel TRSM, n^2(n+1) per diagonal SYRK, 2n^3 per GEMM "
                          "update, 2n^2 / 4n^2 per diagonal / panel tile for the two solves, n = 64); "
                          "frac_issued = the FLOPs of the v_mfma_f64 instructions the kernel issues "
                          "(SQ_INSTS_VALU_MFMA_F64, counters.source) / the same time; frac_survey_8d = "
                          "SURVEY.md §8(d) compulsory bytes (S tile-sparse) / the same time; traffic = "
                          "rocprofv3 --pmc HBM bytes per iteration from profiles/pmc_traffic.json",
            }
            result["survey_8d"] = {
                "whole_iteration_bytes": whole,
                "whole_iteration_GBs": whole / (ms_it * 1e6),
                "whole_iteration_frac_hbm": whole / (ms_it * 1e6) / HBM_PEAK_GBS,
                "kernels": survey,
                "note": "compulsory bytes of SURVEY.md §8(d) with S counted as its non-zero 64x64 tiles",
            }
            result["kernels"] = {k: {"ms": round(v["ms"], 4), "bound": v["bound"], "achieved": round(v["achieved"], 2),
                                     "frac": round(v["frac"], 4), "work": v["work"],
                                     "traffic": pmc_traffic(k, len(mine))} for k, v in table.items()}
        # ---- CPU baseline (oracle restatement timed on this host) + accuracy vs CPU
        if not args.no_cpu:
            allc = host_threads()
            variants = {}
            wc = sc = None
            for th in sorted({args.cpu_threads, allc}):
                wct, sct, dt = run_cpu_baseline(cfg, args.cpu_iters, th, args.cpu_windows, args.cpu_reps)
                variants[f"{th}_threads"] = {"value": args.cpu_windows * args.cpu_iters / dt, "wall_s": dt,
                                             "single_window_iters_per_s": args.cpu_iters * args.cpu_windows / dt}
                if th == args.cpu_threads:
                    wc, sc = wct, sct
            best = variants[f"{allc}_threads"]
            nb = args.cpu_batch_windows if args.cpu_batch_windows is not None else 3 * allc
            dtb = run_cpu_baseline_batch(cfg, args.cpu_iters, allc, nb, args.cpu_reps)
            variants[f"batch_{allc}x1_threads"] = {"value": nb * args.cpu_iters / dtb, "wall_s": dtb, "windows": nb}
            batch = variants[f"batch_{allc}x1_threads"]
            result["cpu_baseline"] = {
                "value": batch["value"],
                "unit": "window-iterations/s",
                "cores": allc,
                "kind": "port",
                "sample": f"batch: {nb} {args.config.upper()} windows x {args.cpu_iters} iterations each, "
                          f"{allc} host threads each solving its own windows with one solver thread (all in flight "
                          f"together, like the GPU batch), median of {args.cpu_reps} passes after 1 warm-up "
                          f"(oracle/liboracle.so, same options). Realtime variants: {args.cpu_windows} windows one at "
                          f"a time at {args.cpu_threads} = realtime_num_threads and at {allc} threads per solve",
                "host": {"cpu_model": cpu_model(), "host_threads": allc, "nproc": os.cpu_count()},
                "variants": variants,
            }
            if not args.no_latency and args.cpu_iters == total_iters:
                P0 = wc.poses()
                result["accuracy"] = {
                    "ate_gpu_m": ate(gpu_pose_w0, gt_p), "ate_cpu_m": ate(P0, gt_p),
                    "max_pose_dev_gpu_vs_cpu_m": float(np.abs(gpu_pose_w0[:, :3] - P0[:, :3]).max()),
                    "final_cost_gpu": result["single_window"]["final_cost"], "final_cost_cpu": sc["final_cost"],
                }
            if not args.no_latency:
                sw = result["single_window"]
                sw["speedup_vs_cpu_3_threads"] = sw["iters_per_s"] / variants[f"{args.cpu_threads}_threads"]["single_window_iters_per_s"]
                sw["speedup_vs_cpu_all_threads"] = sw["iters_per_s"] / best["single_window_iters_per_s"]
            result["speedup_vs_cpu_baseline"] = value / result["cpu_baseline"]["value"]
        print(json.dumps(result), flush=True)
    ctx.close()
    if dist:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
