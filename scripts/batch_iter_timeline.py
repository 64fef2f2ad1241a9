"""One batched iteration of a rocprofv3 kernel trace (the bench's timed loop) as a timeline: start
offset, duration and end of every kernel relative to the iteration's first kernel. Usage:
batch_iter_timeline.py run_kernel_trace.csv [iteration index among the large k_zero_S launches]"""
import csv
import sys

rows = []
for r in csv.DictReader(open(sys.argv[1])):
    grid = int(r.get("Grid_Size_X") or r.get("Grid_Size") or 0)
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("okg::", "")
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, grid))
rows.sort()
# iteration marker: the first kernel of the captured iteration (k_zero_S before round 3, then the
# assembly), the batch's launches (largest grid) only
names = {r[2] for r in rows}
if "k_lm_prep_windows<false>" in names:  # round 3: S cleared after the factorisation, prep first
    mark = "k_lm_prep_windows<false>"
elif sum(r[2] == "k_zero_S" for r in rows) > 4 and "k_lm_visit<2, false>" not in names:
    mark = "k_zero_S"
else:
    mark = "k_lm_visit<2, false>"
gmax = max(r[3] for r in rows if r[2] == mark)
zs = [i for i, r in enumerate(rows) if r[2] == mark and r[3] == gmax]
# the bench's batched solve: begin (iteration 0), warm-up + timed iterations, then the PCIe-inclusive
# solve; the timed iterations are the last K = 5 of the first run of consecutive iterations
it = int(sys.argv[2]) if len(sys.argv) > 2 else len(zs) // 2
a, b = zs[it], zs[it + 1]
t0 = rows[a][0]
for r in rows[a:b]:
    print(f"{(r[0] - t0) / 1e3:8.1f} {(r[1] - r[0]) / 1e3:8.1f} {(r[1] - t0) / 1e3:8.1f}  {r[2]}")
print(f"iteration span {(rows[b][0] - t0) / 1e3:.1f} us")
# mean over the iterations of the first solve after its warm-up (argv[3] = first timed iteration)
first = int(sys.argv[3]) if len(sys.argv) > 3 else None
if first is not None:
    k = int(sys.argv[4]) if len(sys.argv) > 4 else 5
    tot, spans = {}, []
    for j in range(first, first + k):
        a, b = zs[j], zs[j + 1]
        spans.append((rows[b][0] - rows[a][0]) / 1e3)
        for r in rows[a:b]:
            tot[r[2]] = tot.get(r[2], 0.0) + (r[1] - r[0]) / 1e3
    print(f"mean over iterations {first}..{first + k - 1}: span {sum(spans) / k:.1f} us")
    for n, v in sorted(tot.items(), key=lambda x: -x[1]):
        print(f"  {v / k:8.1f}  {n}")
