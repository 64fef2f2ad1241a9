"""Summarise a rocprofv3 kernel_stats.csv: name, calls, average us, share."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in rows[:n]:
    print(f"{r['Name'][:58]:58s} {int(r['Calls']):7d} {float(r['AverageNs']) / 1e3:10.1f}us {float(r['Percentage']):6.2f}%")
print(f"total {tot / 1e6:.2f} ms")
