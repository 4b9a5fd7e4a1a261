"""Host time of one U-Net hipGraph replay (B = 1, dim 64) against its device time: is the replay's node
submission the bound?"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "red-diffeq_amd"))
from red_diffeq.models.diffusion import Unet  # noqa: E402

torch.manual_seed(0)
net = Unet(dim=64, dim_mults=(1, 2, 4, 8), channels=1).cuda().eval()
with torch.no_grad():
    xs, ts = net.graph_io((1, 1, 72, 72), torch.device("cuda"))
    for _ in range(5):
        net.replay_static(xs, ts)
    torch.cuda.synchronize()
    n = 50
    h = 0.0
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        t0 = time.perf_counter()
        net.replay_static(xs, ts)
        h += time.perf_counter() - t0
    e1.record()
    t0 = time.perf_counter()
    torch.cuda.synchronize()
    tail = time.perf_counter() - t0
print(f"replay host {h / n * 1e3:.3f} ms per call; device {e0.elapsed_time(e1) / n:.3f} ms per forward; "
      f"host still waiting {tail * 1e3:.2f} ms at the end", flush=True)
