#!/usr/bin/env python3
"""Per-kernel mean counter value per dispatch from rocprofv3 --pmc CSVs (one or more passes), as a
fixed-width table. Usage: python3 scripts/pmc_table.py pass3.csv pass4.csv > profiles/..._sq_tcc.txt"""
import csv
import re
import sys
from collections import defaultdict


def short(name):
    name = re.sub(r"^void ", "", name)
    name = re.sub(r"\(.*\)$", "", name)
    return name.replace("okg::", "")


def main(paths):
    acc = defaultdict(lambda: defaultdict(list))
    counters = set()
    for p in paths:
        with open(p) as f:
            for row in csv.DictReader(f):
                k, c = short(row["Kernel_Name"]), row["Counter_Name"]
                acc[k][c].append(float(row["Counter_Value"]))
                counters.add(c)
    cols = sorted(counters)
    print(f"{'kernel':22s} " + " ".join(f"{c[:16]:>16s}" for c in cols))
    for k in sorted(acc):
        vals = [sum(acc[k][c]) / len(acc[k][c]) if acc[k][c] else float("nan") for c in cols]
        print(f"{k[:22]:22s} " + " ".join(f"{v:16.4g}" for v in vals))


if __name__ == "__main__":
    main(sys.argv[1:])
