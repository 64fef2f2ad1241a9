"""Aggregate rocprofv3 --pmc counter_collection.csv files: per kernel, mean counter value per dispatch."""
import collections
import csv
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(list))
for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].split("(")[0].replace("okg::", "")
        agg[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
ctrs = sorted({c for k in agg.values() for c in k})
print(f"{'kernel':22s} " + " ".join(f"{c[:16]:>16s}" for c in ctrs))
for k, d in sorted(agg.items()):
    print(f"{k[:22]:22s} " + " ".join(f"{(sum(d[c]) / len(d[c]) if d.get(c) else float('nan')):16.4g}" for c in ctrs))
