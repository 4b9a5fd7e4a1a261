"""RED-DiffEq loop wallclock (bench.red_loop_wallclock) for the reference notebook configuration
(CurveFault, ns = 5) and configs[2] (CurveVel-A, ns = 32); env switches (RDQ_NO_OVERLAP,
RDQ_NO_XCD_LOCAL) select the variant.  python tools/red_loop_ab.py [steps]"""
import json
import os
import sys
import types

sys.path[:0] = [os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."),
                os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "red-diffeq_amd")]
import torch  # noqa: E402

import bench  # noqa: E402

if __name__ == "__main__":
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    a = types.SimpleNamespace(nt=1000, warmup=3, steps=steps)
    dev = torch.device("cuda:0")
    env = {k: v for k, v in os.environ.items() if k.startswith("RDQ_")}
    out = {"env": env,
           "notebook_ns5_ms": bench.red_loop_wallclock(dev, a, ns=5, family="curvefault"),
           "configs2_ns32_ms": bench.red_loop_wallclock(dev, a, ns=32, family="curvevel")}
    print(json.dumps(out), flush=True)
