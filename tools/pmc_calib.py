"""FETCH_SIZE / WRITE_SIZE calibration for 4-B-per-lane coalesced accesses (the access width of
the FWI kernels): rdq_l1_forward reads two 256 MiB arrays once (k_l1_partial: 512 MiB, beyond the
256 MiB MALL); rdq_l1_backward reads them again and writes one 256 MiB array (k_l1_backward)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "red-diffeq_amd"))
from red_diffeq.core.losses import l1_misfit  # noqa: E402

n = 64 * 1024 * 1024           # floats per array = 256 MiB
a = torch.randn(1, n, device="cuda", requires_grad=True)
b = torch.randn(1, n, device="cuda")
for _ in range(3):
    a.grad = None
    l1_misfit(a, b).sum().backward()
torch.cuda.synchronize()
print("k_l1_partial read bytes", 2 * n * 4, "k_l1_backward read bytes", 2 * n * 4, "write bytes", n * 4)
