"""Kernel sequence of the LAST U-Net forward in a rocprofv3 kernel trace (csv or rocpd db): per launch
start offset, duration and grid, then per-kernel totals for that forward.
python tools/unet_timeline.py <kernel_trace.csv | results.db> [first-kernel-substring]"""
import collections
import csv
import sqlite3
import sys


def rows_of(path):
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        return [(r[0], int(r[1]), int(r[2]), (r[3], r[4], r[5])) for r in
                c.execute("select name, start, end, grid_x, grid_y, grid_z from kernels order by start")]
    out = []
    for r in csv.DictReader(open(path)):
        out.append((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                    (r.get("Grid_Size_X"), r.get("Grid_Size_Y"), r.get("Grid_Size_Z"))))
    return sorted(out, key=lambda r: r[1])


def short(n):
    return n.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]


if __name__ == "__main__":
    rows = rows_of(sys.argv[1])
    marks = [sys.argv[2]] if len(sys.argv) > 2 else ["k_unet_head", "k_conv_ig<7"]   # a forward's first kernel
    starts = []
    for first in marks:
        starts = [i for i, r in enumerate(rows) if first in r[0]]
        if starts:
            break
    fw = rows[starts[-1]:]
    t0 = fw[0][1]
    tot = collections.defaultdict(lambda: [0, 0.0])
    for name, s, e, g in fw:
        d = (e - s) / 1e3
        nm = short(name)
        tot[nm][0] += 1
        tot[nm][1] += d
        print(f"{(s - t0) / 1e3:8.1f} {d:7.2f}  {nm[:48]:48s} {g}")
    print(f"launches {len(fw)}  sum {sum(v[1] for v in tot.values()):.1f} us  span {(fw[-1][2] - t0) / 1e3:.1f} us")
    for nm, (n, d) in sorted(tot.items(), key=lambda kv: -kv[1][1]):
        print(f"{n:5d} {d:9.1f} us  {nm[:90]}")
