"""Kernel timeline of one RED-DiffEq iteration (notebook configuration) from a rocprofv3 kernel trace:
the launches between two consecutive persistent forwards, with start offset, duration and queue.
python tools/loop_timeline.py <kernel_trace.csv>"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
fw = [i for i, r in enumerate(rows) if "k_fwd_pt" in r["Kernel_Name"]]
a, b = fw[-3], fw[-2]
t0 = int(rows[a]["Start_Timestamp"])
busy = {}
for r in rows[a:b + 1]:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    q = r.get("Queue_Id", r.get("Stream_Id", "?"))
    nm = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:48]
    print(f"{s / 1e3:9.1f} {(e - s) / 1e3:8.1f}  q{q:>3}  {nm}")
print("iteration span us", (int(rows[b]["Start_Timestamp"]) - t0) / 1e3)
