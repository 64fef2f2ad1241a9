"""Turn rocprofv3 --pmc passes (scripts/gpu_pmc.sh) into profiles/pmc_traffic.json: HBM bytes per
dispatch of each kernel. FETCH_SIZE / WRITE_SIZE are in KiB; FETCH_SIZE is doubled, WRITE_SIZE taken
as is: the calibration of scripts/pmc_calib.hip (profiles/rNN_pmc_calib.json, re-measured each round) measured exactly these
factors for every access shape these kernels use (16 B and 8 B per lane, the Cholesky's tile rows),
on a buffer four times the Infinity Cache.

Usage: pmc_traffic.py OUT.json WINDOWS pass1.csv pass2.csv ... (WINDOWS = windows in the profiled
batch; bench.py scales bytes_per_window_iteration by its own windows per GPU)."""
import collections
import csv
import json
import os
import sys

out = sys.argv[1]
windows = int(sys.argv[2])
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for path in sys.argv[3:]:
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].split("(")[0].replace("okg::", "").replace("void ", "")
        # template arguments: the extrinsics flag (<..., false|true>) and bool-only specialisations
        name = name.replace(", false>", ">").replace(", true>", ">").replace("<false>", "").replace("<true>", "")
        name = name.replace("<256>", "").replace("<1024>", "")  # per-window reduction workgroup sizes
        # the specialised k_lm_visit<mode> kernels under bench.py's table names
        name = {"k_lm_visit<1>": "k_lm_visit", "k_lm_visit<2>": "k_lm_visit_prep", "k_lm_visit<0>": "k_lm_visit_init",
                "k_lm_prep_windows": "k_lm_visit_prep", "k_cholesky<0>": "k_cholesky"}.get(name, name)
        vals[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
kern = {}
for k, d in vals.items():
    if "FETCH_SIZE" not in d or "WRITE_SIZE" not in d:
        continue
    f = sum(d["FETCH_SIZE"]) / len(d["FETCH_SIZE"]) * 1024 * 2
    w = sum(d["WRITE_SIZE"]) / len(d["WRITE_SIZE"]) * 1024
    kern[k] = {"fetch_bytes_per_dispatch": f, "write_bytes_per_dispatch": w, "bytes_per_dispatch": f + w}
    if k in ("k_assemble_pp", "k_assemble_sb", "k_eval_imu", "k_eval_obs", "k_fgrad", "k_cholesky", "k_lm_backsub", "k_lm_backsub_jv",
             "k_zero_S", "k_jv", "k_dogleg", "k_reduce", "k_gradnorm"):
        kern[k]["bytes_per_iteration"] = f + w  # one dispatch per iteration
    elif k in ("k_lm_visit", "k_lm_visit_prep"):
        # one dispatch each per iteration; the solve's dispatches only touch the windows that need
        # them (accepted steps / stale Z), the roofline table's dispatches every window: the
        # heaviest dispatch is the full-batch figure bench.py compares with
        kern[k]["bytes_per_iteration"] = max(a * 2 + b for a, b in zip(d["FETCH_SIZE"], d["WRITE_SIZE"])) * 1024
    if "bytes_per_iteration" in kern[k]:
        kern[k]["bytes_per_window_iteration"] = kern[k]["bytes_per_iteration"] / windows
json.dump({"source": sys.argv[3:], "windows": windows,
           "correction": "FETCH_SIZE x2, WRITE_SIZE x1 (calibrated: " + os.environ.get("PMC_CALIB_FILE", "profiles/r06_pmc_calib.json") + "), KiB -> bytes",
           "kernels": kern}, open(out, "w"), indent=1, sort_keys=True)
print(json.dumps({k: round(v["bytes_per_dispatch"] / 1e9, 3) for k, v in kern.items()}, indent=0))
