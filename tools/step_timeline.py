"""Kernel timeline of the configs[1] bench step (bench.py's step(): HIP forward + L1 + TV + adjoint
+ finalize + Adam) from a rocprofv3 rocpd database: per dispatch start offset, duration and the gap
before it, for the last traced step, and the step's kernel time vs its span.
Record:  rocprofv3 --kernel-trace -d OUT -o run -- python3 bench.py --steps 6 --warmup 3 --no-loop \
             --no-red --no-configs4 --no-cpu-baseline
Print:   python tools/step_timeline.py OUT/.../run_results.db"""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
tabs = [r[0] for r in c.execute("select name from sqlite_master where type='table'")]
kd = next(t for t in tabs if t.startswith("rocpd_kernel_dispatch"))
ks = next(t for t in tabs if t.startswith("rocpd_info_kernel_symbol"))
rows = c.execute(f"select s.display_name, d.start, d.end from {kd} d join {ks} s on d.kernel_id = s.id "
                 f"order by d.start").fetchall()
# one step = the dispatches after one Adam launch up to and including the next one, taken around the
# second-to-last persistent forward (the last one belongs to the phase timing that follows the loop)
fw = [i for i, r in enumerate(rows) if "k_fwd_pt" in r[0]]
ad = [i for i, r in enumerate(rows) if "adam" in r[0].lower()]
if len(fw) < 3 or not ad:
    sys.exit("not enough steps in the trace")
f = fw[-3]
prev = max(i for i in ad if i < f)
nxt = min(i for i in ad if i > f)
j0, i1 = prev + 1, nxt + 1
seg = rows[j0:i1]
t0 = seg[0][1]
busy, prev_end = 0, None
for name, s, e in seg:
    gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
    print(f"{(s - t0) / 1e3:9.1f} us  {(e - s) / 1e3:8.1f} us  gap {gap:6.1f}  {name[:90]}")
    busy += e - s
    prev_end = e
span = seg[-1][2] - t0
print(f"step span {span / 1e3:.1f} us, kernel time {busy / 1e3:.1f} us, {len(seg)} dispatches")
