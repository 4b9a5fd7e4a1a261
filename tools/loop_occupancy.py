"""GPU occupancy of a traced RED loop: reads a rocprofv3 --kernel-trace CSV and reports, over the
last N iterations (delimited by the persistent forward kernel's launches), the busy time of the
union of all kernels, the forward / adjoint spans and the idle gaps longer than 20 us.
python tools/loop_occupancy.py <kernel_trace.csv> [N]"""
import csv
import json
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
N = int(sys.argv[2]) if len(sys.argv) > 2 else 10
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
fwd = [k for k in ks if "k_fwd_pt" in k[2]]
starts = [k[0] for k in fwd][-(N + 1):]
out = []
for a, b in zip(starts, starts[1:]):
    sel = [k for k in ks if a <= k[0] < b]
    busy, cur_s, cur_e, gaps = 0, None, None, []
    for s, e, _ in sel:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
                if s - cur_e > 20000:
                    gaps.append(round((s - cur_e) / 1e3, 1))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    span = lambda p: [round((e - s) / 1e3, 1) for s, e, n in sel if p in n]   # noqa: E731
    out.append({"iter_us": round((b - a) / 1e3, 1), "busy_us": round(busy / 1e3, 1),
                "fwd_us": span("k_fwd_pt"), "adj_us": span("k_adj_p"), "n_kernels": len(sel), "gaps_us": gaps})
for o in out:
    print(json.dumps(o))
