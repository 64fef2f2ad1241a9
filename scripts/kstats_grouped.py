"""rocprofv3 kernel_trace.csv -> per (kernel, grid size) launch count and mean duration, so the
batched launches can be compared with bench.py's event-timed roofline entry. last5_us = mean of the
group's last 5 dispatches: in a bench.py run those are the roofline table's okvisgpu_time_kernel
repetitions (every window armed), which is what the bench's roofline.ms_per_iteration times."""
import collections
import csv
import sys

g = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    name = r["Kernel_Name"].split("(")[0].replace("okg::", "").replace("void ", "")
    grid = int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0)
    g[(name, grid)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
rows = sorted(g.items(), key=lambda kv: -sum(kv[1]))
print(f"{'kernel':24s} {'grid':>9s} {'calls':>6s} {'avg_us':>10s} {'last5_us':>10s} {'total_ms':>9s}")
for (name, grid), d in rows[: int(sys.argv[2]) if len(sys.argv) > 2 else 40]:
    l5 = d[-5:]
    print(f"{name:24s} {grid:9d} {len(d):6d} {sum(d) / len(d):10.1f} {sum(l5) / len(l5):10.1f} {sum(d) / 1e3:9.2f}")
