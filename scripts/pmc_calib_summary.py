"""profiles/<tag>_pmc_calib.json from scripts/gpu_pmc_calib.sh's output: the FETCH_SIZE / WRITE_SIZE
factor of each access shape of scripts/pmc_calib.hip (bytes touched / counter bytes) and the MFMA
counters of k_cholesky on the default bench workload (FP64 MFMA instructions, busy cycles, the busy
fraction of all SIMD-cycles of the dispatch, and the FLOPs they imply).
Usage: pmc_calib_summary.py gpurun_out/pmc_calib OUT.json [n_simd=1024]"""
import csv
import json
import os
import statistics
import sys

src, out = sys.argv[1], sys.argv[2]
n_simd = int(sys.argv[3]) if len(sys.argv) > 3 else 1024  # 256 CUs x 4 SIMDs
touched = {}
for line in open(os.path.join(src, "calib_bytes.txt")):
    k, v = line.split()
    touched[k] = int(v)
calib = {}
for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
    for r in csv.DictReader(open(os.path.join(src, f"calib_{ctr}", "run_counter_collection.csv"))):
        name = r["Kernel_Name"].split("(")[0]
        if name not in touched:
            continue
        kib = float(r["Counter_Value"])
        if (ctr == "FETCH_SIZE") == name.startswith("read"):
            calib.setdefault(name, {})["bytes"] = touched[name]
            calib[name][ctr] = kib * 1024
            calib[name]["factor"] = touched[name] / (kib * 1024)
per = {}
for d in ("mfma", "grbm"):
    for r in csv.DictReader(open(os.path.join(src, d, "run_counter_collection.csv"))):
        per.setdefault(r["Dispatch_Id"], {}).setdefault(r["Counter_Name"], 0.0)
        per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
rows = [v for v in per.values() if "SQ_VALU_MFMA_BUSY_CYCLES" in v] 
grbm = [v["GRBM_GUI_ACTIVE"] for v in per.values() if "GRBM_GUI_ACTIVE" in v]
busy = statistics.median(v["SQ_VALU_MFMA_BUSY_CYCLES"] for v in rows)
ninst = statistics.median(v["SQ_INSTS_VALU_MFMA_F64"] for v in rows)
mops = statistics.median(v["SQ_INSTS_VALU_MFMA_MOPS_F64"] for v in rows)
cycles_per_xcd = statistics.median(grbm) / 8  # GRBM_GUI_ACTIVE sums the 8 XCDs (MI355X_MICROARCH.md)
res = {
    "calibration": calib,
    "calibration_note": "scripts/pmc_calib.hip over a 1 GiB buffer (4x the Infinity Cache): factor = bytes "
                        "touched / counter bytes; FETCH_SIZE reports half the bytes for 16-B, 8-B and the "
                        "Cholesky's tile-row (loadC) read shapes alike, WRITE_SIZE the bytes exactly",
    "k_cholesky_mfma": {
        "dispatches": len(rows),
        "SQ_INSTS_VALU_MFMA_F64": ninst,
        "SQ_INSTS_VALU_MFMA_MOPS_F64": mops,
        "SQ_VALU_MFMA_BUSY_CYCLES": busy,
        "GRBM_GUI_ACTIVE_per_xcd": cycles_per_xcd,
        "mfma_busy_frac": busy / (n_simd * cycles_per_xcd),
        "mfma_flops": ninst * 16 * 16 * 4 * 2,  # v_mfma_f64_16x16x4f64
        "cycles_per_mfma": busy / ninst,
        "note": "busy fraction = SQ_VALU_MFMA_BUSY_CYCLES / (SIMDs x dispatch cycles per XCD); one "
                "v_mfma_f64_16x16x4f64 (2,048 FLOPs) holds a SIMD's matrix core 64 cycles, i.e. the "
                "78.6 TFLOP/s FP64 matrix peak at 2.4 GHz",
    },
}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res["k_cholesky_mfma"], indent=1))
print({k: round(v["factor"], 4) for k, v in calib.items()})
