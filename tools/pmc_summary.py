"""Summarise rocprofv3 PMC passes (gpurun_out/pmc/p*) per kernel: per-wave-step instruction mix,
wait fractions, L2 hit rate.  python tools/pmc_summary.py <pmc_dir> <kernel-substring> <steps> [waves]"""
import collections
import csv
import glob
import sys

d, kname, steps = sys.argv[1], sys.argv[2], int(sys.argv[3])
agg = collections.defaultdict(list)
for f in sorted(glob.glob(d + "/p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if kname in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
m = {k: sorted(v)[len(v) // 2] for k, v in agg.items()}
waves = float(sys.argv[4]) if len(sys.argv) > 4 else m.get("SQ_WAVES", 1)
out = {"kernel": kname, "waves": waves}
for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_SMEM"):
    if c in m:
        out[c + "_per_wave_step"] = round(m[c] / waves / steps, 1)
if "SQ_WAVE_CYCLES" in m:
    wc = m["SQ_WAVE_CYCLES"]
    for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
        if c in m:
            out[c + "_frac"] = round(m[c] / wc, 3)
if "TCC_HIT_sum" in m:
    out["L2_hit"] = round(m["TCC_HIT_sum"] / (m["TCC_HIT_sum"] + m["TCC_MISS_sum"]), 3)
if "GRBM_GUI_ACTIVE" in m:
    out["GRBM_GUI_ACTIVE"] = m["GRBM_GUI_ACTIVE"]
print(out)
print({k: v for k, v in sorted(m.items())})
