#!/usr/bin/env python3
"""bench.py — Gauss-Newton (dogleg trust-region) iterations/s of the MI355X okvis_ceres backend.

Metric (BASELINE.json): "Gauss-Newton iters/sec on 50-KF/2000-landmark window; ATE vs CPU ref".
A step = one trust-region iteration (Ceres semantics: linearise + Schur-reduce + LLT + dogleg +
candidate evaluation + accept/reject) of EVERY window in the job's batch of independent synthetic
S50 windows (50 keyframes, 2,000 landmarks, 16,000 reprojections, 49 IMU factors).
value = (windows x timed iterations) / wall time of the timed region, max over ranks
(window-iterations per second, whole job). Strong scaling: the total window count is fixed and
split across ranks (one process per GPU, no data-path collective).

All tolerances are set to 0 so every timed iteration does real work (the K-iteration protocol of
BASELINE.md); inputs are resident in HBM before the timed region.

Also reported: the single-window latency mode (1 window on 1 GPU), per-kernel device time of one
iteration (HIP events on the context's stream), the roofline of the dominant kernel, accuracy (ATE
of window 0 vs ground truth for GPU and CPU oracle, max pose deviation GPU vs CPU), and the CPU
baseline = the repo's CPU restatement (oracle/liboracle.so, "port") timed on this host.
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "okvis2-x_amd"))
import okvisgpu as og  # noqa: E402

FP64_MFMA_PEAK_TFLOPS = 78.6   # MI355X FP64 matrix (spec; SURVEY.md §8d, not in the gfx950 guide)
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md chip table (spec)
SEED0 = 20251015

CONFIGS = {
    "s50": dict(n_kf=50, n_lm=2000, n_obs=16000),
    "s10": dict(n_kf=10, n_lm=500, n_obs=4000),
}


def bench_options(max_iter):
    # all tolerances 0: every iteration is performed (BASELINE.md timing protocol)
    return og.default_options(max_num_iterations=max_iter, function_tolerance=0.0, gradient_tolerance=0.0,
                              parameter_tolerance=0.0)


def make_windows(cfg, indices):
    """Synthetic windows, generated on host threads (the C generator runs outside the GIL)."""
    from concurrent.futures import ThreadPoolExecutor
    indices = list(indices)
    mk = lambda i: og.SynthWindow(cfg["n_kf"], cfg["n_lm"], cfg["n_obs"], seed=SEED0 + i)  # noqa: E731
    if len(indices) < 16:
        return [mk(i) for i in indices]
    with ThreadPoolExecutor(max_workers=min(16, os.cpu_count() or 4)) as ex:
        return list(ex.map(mk, indices))


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


def rank_windows(total, world, rank):
    """This rank's share of the fixed total window count (strong scaling)."""
    per = [total // world + (1 if r < total % world else 0) for r in range(world)]
    start = sum(per[:rank])
    return list(range(start, start + per[rank]))


def aggregate(dist, elapsed, early, device):
    """Max of the timed region over ranks, sum of early-terminated windows (the only exchange)."""
    if dist is None:
        return elapsed, early
    import torch
    t = torch.tensor([elapsed, float(early)], dtype=torch.float64, device=device)
    tmax, tsum = t.clone(), t.clone()
    dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    dist.all_reduce(tsum, op=dist.ReduceOp.SUM)
    return float(tmax[0].item()), int(tsum[1].item())


def roofline_table(ctx, reps):
    """Per-kernel device time (HIP events on the context's stream, `reps` back-to-back launches of
    one iteration's worth on the resident data) and achieved rate of its algorithmic work."""
    table = {}
    for name in og.kernel_names():  # every kernel okvisgpu_time_kernel exposes
        ms, work, bound = ctx.time_kernel(name, reps)
        rate = work / (ms * 1e-3) / (1e9 if bound == "hbm" else 1e12) if ms > 0 else 0.0
        peak = HBM_PEAK_GBS if bound == "hbm" else FP64_MFMA_PEAK_TFLOPS
        table[name] = {"ms": ms, "bound": bound, "work": work, "achieved": rate, "peak": peak, "frac": rate / peak}
    return table


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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--windows", type=int, default=2048, help="total windows in the job (strong scaling)")
    ap.add_argument("--config", default="s50", choices=sorted(CONFIGS))
    ap.add_argument("--cpu-threads", type=int, default=3, help="realtime_num_threads (okvis2.yaml:93)")
    ap.add_argument("--cpu-iters", type=int, default=None, help="default: warmup + steps")
    ap.add_argument("--cpu-reps", type=int, default=3, help="median of this many timed passes after 1 warm-up")
    ap.add_argument("--cpu-windows", type=int, default=24, help="windows in the CPU baseline sample")
    ap.add_argument("--kernel-reps", type=int, default=5, help="repetitions per kernel in the roofline table")
    ap.add_argument("--cholesky-schedule", type=int, default=0, help="0 auto, 1 persistent per window, 2 tile-parallel, 3 wave-specialised")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-latency", action="store_true")
    ap.add_argument("--no-profile", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    dist = None
    if world > 1:
        import torch.distributed as tdist
        torch.cuda.set_device(local_rank)
        tdist.init_process_group("nccl")
        dist = tdist
    cfg = CONFIGS[args.config]

    # ---- this rank's share of the fixed total (strong scaling)
    mine = rank_windows(args.windows, world, rank)
    windows = make_windows(cfg, mine)
    ctx = og.Context(local_rank)
    ctx.set_problems([w.problem for w in windows])
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
    sums = ctx.solve_end(len(windows))
    elapsed = t1 - t0
    early = sum(1 for s in sums if s["num_iterations"] < total_iters)
    gn_frac = float(np.mean([(s["num_successful_steps"] - 1) / max(1, s["num_iterations"]) for s in sums]))
    elapsed, early = aggregate(dist, elapsed, early, f"cuda:{local_rank}")

    # per-solve rate including the PCIe upload of the parameters and the write-back (not `value`)
    for w in windows:
        w.reset()
    ctx.synchronize()
    a = time.perf_counter()
    ctx.update_params()
    ctx.solve(opts, len(windows))
    pcie_s = time.perf_counter() - a

    value = args.windows * args.steps / elapsed
    result = {
        "metric": "Gauss-Newton iters/sec on 50-KF/2000-landmark window; ATE vs CPU ref",
        "value": value,
        "unit": "window-iterations/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
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
        result["early_terminated_windows"] = early
        result["per_solve_incl_pcie"] = {"wall_s": pcie_s, "iterations": total_iters,
                                         "window_iterations_per_s": len(windows) * total_iters / pcie_s}
        result["frac_iterations_with_gn_solve"] = gn_frac
        # ---- single-window latency mode (1 window, this GPU)
        if not args.no_latency:
            w1 = make_windows(cfg, [0])
            c1 = og.Context(local_rank)
            c1.set_problems([w1[0].problem])
            c1.solve_begin(opts)
            c1.solve_iterate(args.warmup)
            c1.synchronize()
            a = time.perf_counter()
            c1.solve_iterate(args.steps)
            c1.synchronize()
            b = time.perf_counter()
            s1 = c1.solve_end(1)[0]
            result["single_window"] = {"iters_per_s": args.steps / (b - a), "ms_per_iter": (b - a) / args.steps * 1e3,
                                       "final_cost": s1["final_cost"]}
            gpu_pose_w0 = w1[0].poses().copy()
            gt_p, _, _ = w1[0].ground_truth()
            if not args.no_profile:
                w1[0].reset()
                c1.update_params()
                c1.solve_begin(opts)
                c1.solve_iterate(args.warmup)
                ph1 = c1.profile_iteration()
                c1.solve_end(1)
                result["single_window"]["kernel_ms_per_iteration"] = {k: round(v, 4) for k, v in ph1.items()}
            c1.close()
        # ---- roofline: per-kernel device time on the resident batch, dominant kernel by time
        if not args.no_profile:
            table = roofline_table(ctx, args.kernel_reps)
            dominant = max(table, key=lambda k: table[k]["ms"])
            d = table[dominant]
            traffic = pmc_traffic(dominant, len(mine))
            result["roofline"] = {
                "kernel": dominant, "bound": d["bound"], "achieved": d["achieved"], "peak": d["peak"],
                "unit": "GB/s" if d["bound"] == "hbm" else "TFLOP/s", "frac": d["frac"],
                "traffic": traffic,
                "work_per_iteration": d["work"], "ms_per_iteration": d["ms"],
                "method": f"HIP events on the context stream, {args.kernel_reps} launches of one iteration's "
                          "worth on the resident batch; work = algorithmic bytes/FLOPs (DESIGN.md §4); traffic = "
                          "rocprofv3 --pmc HBM bytes per iteration from profiles/pmc_traffic.json",
            }
            result["kernels"] = {k: {"ms": round(v["ms"], 4), "bound": v["bound"], "achieved": round(v["achieved"], 2),
                                     "frac": round(v["frac"], 4), "work": v["work"],
                                     "traffic": pmc_traffic(k, len(mine))} for k, v in table.items()}
        # ---- CPU baseline (oracle restatement timed on this host) + accuracy vs CPU
        if not args.no_cpu:
            wc, sc, dt = run_cpu_baseline(cfg, args.cpu_iters, args.cpu_threads, args.cpu_windows, args.cpu_reps)
            result["cpu_baseline"] = {
                "value": args.cpu_windows * args.cpu_iters / dt,
                "unit": "window-iterations/s",
                "cores": args.cpu_threads,
                "kind": "port",
                "sample": f"{args.cpu_windows} {args.config.upper()} windows x {args.cpu_iters} iterations each, "
                          f"median of {args.cpu_reps} passes after 1 warm-up (oracle/liboracle.so, "
                          f"{args.cpu_threads} threads = realtime_num_threads, same options)",
                "wall_s": dt,
            }
            if not args.no_latency and args.cpu_iters == total_iters:
                P0 = wc.poses()
                result["accuracy"] = {
                    "ate_gpu_m": ate(gpu_pose_w0, gt_p), "ate_cpu_m": ate(P0, gt_p),
                    "max_pose_dev_gpu_vs_cpu_m": float(np.abs(gpu_pose_w0[:, :3] - P0[:, :3]).max()),
                    "final_cost_gpu": result["single_window"]["final_cost"], "final_cost_cpu": sc["final_cost"],
                }
            if not args.no_latency:
                cpu_single = args.cpu_iters * args.cpu_windows / dt
                result["single_window"]["speedup_vs_cpu"] = result["single_window"]["iters_per_s"] / cpu_single
            result["speedup_vs_cpu_baseline"] = value / result["cpu_baseline"]["value"]
        print(json.dumps(result), flush=True)
    ctx.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
