"""One batched iteration of a rocprofv3 kernel trace (the bench's timed loop) as a timeline: start
offset, duration and end of every kernel relative to the iteration's k_zero_S. Usage:
batch_iter_timeline.py run_kernel_trace.csv [iteration index among the large k_zero_S launches]"""
import csv
import sys

rows = []
for r in csv.DictReader(open(sys.argv[1])):
    grid = int(r.get("Grid_Size_X") or r.get("Grid_Size") or 0)
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("okg::", "")
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, grid))
rows.sort()
zs = [i for i, r in enumerate(rows) if r[2] == "k_zero_S" and r[3] > 1000000]
it = int(sys.argv[2]) if len(sys.argv) > 2 else len(zs) // 2
a, b = zs[it], zs[it + 1]
t0 = rows[a][0]
for r in rows[a:b]:
    print(f"{(r[0] - t0) / 1e3:8.1f} {(r[1] - r[0]) / 1e3:8.1f} {(r[1] - t0) / 1e3:8.1f}  {r[2]}")
print(f"iteration span {(rows[b][0] - t0) / 1e3:.1f} us")
