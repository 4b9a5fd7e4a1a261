"""One configs[4]-sized U-Net forward batch (344 tiles of 72x72, the 2-D tiled regulariser's batch for a
500 x 3000 model) in bf16 or fp32, repeated, for rocprofv3 --kernel-trace --stats.
python tools/unet_prof.py [--B 344] [--precision bf16] [--reps 5]"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "red-diffeq_amd"))
from red_diffeq.models.diffusion import Unet  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--B", type=int, default=344)
ap.add_argument("--precision", default="bf16")
ap.add_argument("--reps", type=int, default=5)
a = ap.parse_args()
dev = torch.device("cuda:0")
torch.manual_seed(0)
net = Unet(dim=64, dim_mults=(1, 2, 4, 8), channels=1).to(dev).eval()
net.set_precision(a.precision)
x = torch.randn(a.B, 1, 72, 72, device=dev).clamp(-1, 1)
t = torch.randint(0, 1000, (a.B,), device=dev)
with torch.no_grad():
    for _ in range(a.reps):
        net(x, t)
torch.cuda.synchronize()
print("done", flush=True)
