"""One iteration of a rocprofv3 kernel trace as a timeline: start offset, duration and end of each
kernel relative to the first kernel of the iteration (the n-th launch of ANCHOR, default k_zero_S)."""
import csv
import sys

rows = []
for r in csv.DictReader(open(sys.argv[1])):
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("okg::", "").replace("void ", "")))
rows.sort()
anchor = sys.argv[2] if len(sys.argv) > 2 else "k_zero_S"
idx = [i for i, r in enumerate(rows) if r[2] == anchor]
a, b = idx[-3], idx[-2]
t0 = rows[a][0]
for s, e, n in rows[a:b]:
    print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f} {(e - t0) / 1e3:8.1f}  {n}")
print(f"iteration span {(rows[b][0] - t0) / 1e3:.1f} us")
