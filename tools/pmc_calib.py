"""FETCH_SIZE calibration for 4-B-per-lane coalesced loads (the access width of the FWI kernels):
runs rdq_l1_forward over two 256 MiB arrays (512 MiB read once, beyond the 256 MiB MALL)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "red-diffeq_amd"))
from red_diffeq.core.losses import l1_misfit  # noqa: E402

n = 64 * 1024 * 1024           # floats per array = 256 MiB
a = torch.randn(1, n, device="cuda")
b = torch.randn(1, n, device="cuda")
for _ in range(3):
    l1_misfit(a, b)
torch.cuda.synchronize()
print("read bytes per call", 2 * n * 4)
