"""Per-kernel summary (calls, total / average ns) from a rocprofv3 rocpd database (ROCm 7 default
output), the same columns as --stats' kernel_stats.csv.  python tools/rocpd_stats.py DB [N] [--csv OUT]"""
import csv
import sqlite3
import sys


def stats(db):
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "name" if "name" in cols else "kernel_name"
    rows = c.execute(f"select {name}, count(*), sum(end - start), avg(end - start), min(end - start), "
                     f"max(end - start) from kernels group by {name} order by sum(end - start) desc").fetchall()
    tot = sum(r[2] for r in rows)
    return [(r[0], r[1], r[2], r[3], 100.0 * r[2] / tot, r[4], r[5]) for r in rows], c


if __name__ == "__main__":
    rows, c = stats(sys.argv[1])
    n = int(sys.argv[2]) if len(sys.argv) > 2 and sys.argv[2].isdigit() else 40
    if "--csv" in sys.argv:
        with open(sys.argv[sys.argv.index("--csv") + 1], "w", newline="") as f:
            w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
            w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
            w.writerows(rows)
    for r in rows[:n]:
        print(f"{r[1]:6d} {r[2] / 1e3:10.1f}us {r[3] / 1e3:8.2f}us {r[4]:5.1f}%  {r[0][:110]}")
