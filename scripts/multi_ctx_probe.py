"""Development: a batch split over C contexts (each its own stream and captured iteration graph)
whose iterations are enqueued back to back, so the GPU can run one context's MFMA-bound Cholesky
beside another's HBM-bound linearisation. Usage: python scripts/multi_ctx_probe.py TOTAL C [steps]"""
import sys
import time

sys.path.insert(0, ".")
import bench  # noqa: E402

total, nctx = int(sys.argv[1]), int(sys.argv[2])
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
warm = 3
og = bench.og_module()
cfg = bench.CONFIGS["s50"]
ws = bench.make_windows(cfg, range(total))
opts = bench.bench_options(warm + steps)
ctxs = []
for c in range(nctx):
    part = ws[c * total // nctx:(c + 1) * total // nctx]
    x = og.Context(0)
    x.set_problems([w.problem for w in part])
    ctxs.append(x)
for x in ctxs:
    x.solve_begin(opts)
for _ in range(warm):
    for x in ctxs:
        x.solve_iterate(1)
for x in ctxs:
    x.synchronize()
t0 = time.perf_counter()
for _ in range(steps):
    for x in ctxs:
        x.solve_iterate(1)
for x in ctxs:
    x.synchronize()
t1 = time.perf_counter()
sums = [s for x in ctxs for s in x.solve_end()]
print(f"{total} windows in {nctx} contexts: {total * steps / (t1 - t0):.0f} window-it/s, "
      f"{(t1 - t0) / steps * 1e3:.3f} ms/step, iterations {sorted(set(s['num_iterations'] for s in sums))}", flush=True)
