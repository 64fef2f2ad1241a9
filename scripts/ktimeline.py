"""rocprofv3 kernel_trace.csv -> busy time (union of kernel intervals) vs wall span over the last
N launches, and the largest idle gaps between consecutive kernels (launch/dependency latency)."""
import csv
import sys

rows = []
for r in csv.DictReader(open(sys.argv[1])):
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("okg::", "")))
rows.sort()
n = int(sys.argv[2]) if len(sys.argv) > 2 else len(rows)
rows = rows[-n:]
span = rows[-1][1] - rows[0][0]
busy, cur_s, cur_e = 0, rows[0][0], rows[0][1]
gaps = []
prev = rows[0]
for s, e, name in rows[1:]:
    if s > cur_e:
        busy += cur_e - cur_s
        gaps.append((s - cur_e, prev[2], name))
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
    prev = (s, e, name)
busy += cur_e - cur_s
print(f"launches {len(rows)}  span {span/1e3:.1f} us  busy {busy/1e3:.1f} us  idle {(span-busy)/1e3:.1f} us  "
      f"mean gap {(span-busy)/1e3/max(1,len(gaps)):.2f} us over {len(gaps)} gaps")
agg = {}
for g, a, b in gaps:
    k = (a, b)
    agg.setdefault(k, [0, 0])
    agg[k][0] += g; agg[k][1] += 1
for (a, b), (g, c) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:15]:
    print(f"{a:22s} -> {b:22s} {c:5d} gaps {g/1e3/c:6.2f} us avg")
