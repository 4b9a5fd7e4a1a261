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
with torch.no_grad():
    for _ in range(3):
        net(x, t)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        net(x, t)
    e1.record()
    torch.cuda.synchronize()
print(f"B={B}: {e0.elapsed_time(e1) / reps:.3f} ms per forward", flush=True)
