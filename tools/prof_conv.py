"""Summarise a rocprofv3 kernel trace of tools/unet_prof.py: per-kernel time per U-Net forward and,
for the convolution kernels, per-launch-shape averages.  python tools/prof_conv.py <dir> [reps]"""
import collections
import csv
import sys

d = sys.argv[1]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
rows = list(csv.DictReader(open(f"{d}/run_kernel_stats.csv")))
print("ms per forward", round(sum(float(r["TotalDurationNs"]) for r in rows) / reps / 1e6, 2))
for r in rows[:12]:
    print(f"{float(r['TotalDurationNs']) / reps / 1e6:8.2f} ms  {int(r['Calls']) // reps:4d}x  "
          f"{float(r['AverageNs']) / 1e3:8.1f} us  {r['Name'][:80]}")
g = collections.defaultdict(list)
for r in csv.DictReader(open(f"{d}/run_kernel_trace.csv")):
    n = r["Kernel_Name"]
    if "conv" in n:
        name = n.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
        g[(name, int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]), r["Grid_Size_Y"])].append(
            (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(g.items(), key=lambda kv: -sum(kv[1]))[:14]:
    print(f"{k[0]:28s} wg {k[1]:6d} x {k[2]:2s} {len(v) // reps:3d}x {sum(v) / len(v):8.1f} us")
