"""Profile target: the configs[2] loop's U-Net forward (dim 64, 72x72, B = 1, fp32), replayed
from its hipGraph `reps` times (run under rocprofv3 --kernel-trace --stats)."""
import sys
import os
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "red-diffeq_amd"))
from red_diffeq.models.diffusion import Unet  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
torch.manual_seed(0)
net = Unet(dim=64, dim_mults=(1, 2, 4, 8), channels=1).cuda().eval()
x = torch.randn(B, 1, 72, 72, device="cuda")
t = torch.randint(0, 1000, (B,), device="cuda")
def timed(f):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


with torch.no_grad():
    ms_call = timed(lambda: net(x, t))
    xs, ts = net.graph_io(x.shape, x.device)
    xs.copy_(x)
    ts.copy_(t)
    ms = timed(lambda: net.replay_static(xs, ts))
print(f"B={B}: {ms:.3f} ms per forward (static graph I/O, the RED loop's path); module call {ms_call:.3f} ms",
      flush=True)
