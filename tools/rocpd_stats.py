"""Per-kernel statistics (calls, total / average ns) from a rocprofv3 rocpd SQLite database
(rocprofv3 --kernel-trace without --output-format csv).
python tools/rocpd_stats.py <run_results.db> [--top N] [--csv out.csv]"""
import argparse
import csv
import sqlite3

ap = argparse.ArgumentParser()
ap.add_argument("db")
ap.add_argument("--top", type=int, default=30)
ap.add_argument("--csv", default=None)
a = ap.parse_args()
c = sqlite3.connect(a.db)
tabs = [r[0] for r in c.execute("select name from sqlite_master where type='table'")]
kd = next(t for t in tabs if t.startswith("rocpd_kernel_dispatch"))
ks = next(t for t in tabs if t.startswith("rocpd_info_kernel_symbol"))
cols = [r[1] for r in c.execute(f"pragma table_info({ks})")]
name_col = "display_name" if "display_name" in cols else "kernel_name"
rows = c.execute(f"select s.{name_col}, count(*), sum(d.end - d.start), avg(d.end - d.start) from {kd} d "
                 f"join {ks} s on d.kernel_id = s.id group by s.{name_col} order by 3 desc").fetchall()
tot = sum(r[2] for r in rows)
out = [{"Name": r[0], "Calls": r[1], "TotalDurationNs": r[2], "AverageNs": round(r[3], 1),
        "Percentage": round(100.0 * r[2] / tot, 2)} for r in rows]
for r in out[:a.top]:
    print(f"{r['TotalDurationNs'] / 1e6:9.3f} ms {r['Calls']:6d} {r['AverageNs'] / 1e3:9.1f} us {r['Percentage']:5.1f}%  {r['Name'][:100]}")
print(f"total {tot / 1e6:.3f} ms over {sum(r['Calls'] for r in out)} dispatches")
if a.csv:
    with open(a.csv, "w", newline="") as fh:
        w = csv.DictWriter(fh, fieldnames=list(out[0]))
        w.writeheader()
        w.writerows(out)
