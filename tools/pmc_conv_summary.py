"""MFMA utilisation of the U-Net conv kernels from one rocprofv3 --pmc pass (tools/gpu_conv_pmc.sh):
per dispatch of k_conv_cc, SQ_VALU_MFMA_BUSY_CYCLES (summed over the SIMDs) against the dispatch's
duration x clock x 1024 SIMDs, plus the wave-level busy / wait fractions.
python tools/pmc_conv_summary.py <pass dir> <label> [clock GHz]   (PMC_KERNEL: kernel name filter)"""
import collections
import csv
import glob
import json
import os
import sys

d, label = sys.argv[1], sys.argv[2]
ghz = float(sys.argv[3]) if len(sys.argv) > 3 else 2.4
per = collections.defaultdict(dict)
for f in glob.glob(d + "/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if os.environ.get("PMC_KERNEL", "k_conv_cc") not in r["Kernel_Name"]:
            continue
        k = r["Dispatch_Id"]
        per[k][r["Counter_Name"]] = float(r["Counter_Value"])
        per[k]["dur_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
rows = sorted(per.values(), key=lambda v: v.get("dur_ns", 0))
m = rows[len(rows) // 2] if rows else {}
out = {"label": label, "dispatches": len(rows), "median_dispatch": m}
if m and "SQ_VALU_MFMA_BUSY_CYCLES" in m:
    simd_cycles = m["dur_ns"] * ghz * 1024
    out["mfma_busy_frac_of_kernel"] = round(m["SQ_VALU_MFMA_BUSY_CYCLES"] / simd_cycles, 3)
    if m.get("SQ_WAVES"):
        out["mfma_busy_per_wave_cycles"] = round(m["SQ_VALU_MFMA_BUSY_CYCLES"] / m["SQ_WAVES"])
    if m.get("SQ_WAVE_CYCLES"):
        # SQ_WAVE_CYCLES counts in units of 4 cycles on gfx950 (matches the MFMA busy total)
        out["mfma_busy_frac_of_wave_lifetime"] = round(m["SQ_VALU_MFMA_BUSY_CYCLES"] / (4 * m["SQ_WAVE_CYCLES"]), 3)
        for c in ("SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_WAIT_ANY"):
            if c in m:
                out[c + "_frac"] = round(m[c] / m["SQ_WAVE_CYCLES"], 3)
print(json.dumps(out))
