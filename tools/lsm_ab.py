"""A/B of the first ResnetBlock's conv launch with every block's Linear(SiLU(t)) as a side job
(rdq_conv2d_gn_silu_lsm) against the separate launches: device time per call from a hipGraph of
back-to-back calls (the fused figure includes block2: subtract "block2 alone").  Round 2: at B = 1 the
side job saved 1.7 us of 23.4; at B = 8 it cost 2 us (side job first / after the conv tiles and 2-16
rows per wave all measured), so the U-Net uses it for B <= 2."""
import os
import sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "red-diffeq_amd"))
from red_diffeq.models.diffusion import Unet  # noqa: E402
from red_diffeq.models import unet_ops  # noqa: E402

torch.manual_seed(0)
net = Unet(dim=64, dim_mults=(1, 2, 4, 8), channels=1).cuda().eval()
blocks = net._resnet_blocks()
b0 = blocks[0]


def timed(f, inner=20, reps=10):
    for _ in range(2):
        f()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(inner):
            f()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (reps * inner)


with torch.no_grad():
    for B in (1, 8):
        x = torch.randn(B, 64, 72, 72, device="cuda")
        te = torch.randn(B, 256, device="cuda")
        sep = timed(lambda: (unet_ops.resnet_scale_shifts(te, blocks),
                             unet_ops.conv_group_norm_silu(x, b0.block1.proj, b0.block1.norm, te[:, :128])))
        print(f"B={B} separate (lsm + conv_gn): {sep:.2f} us", flush=True)
        us = timed(lambda: unet_ops.first_block_and_scale_shifts(x, b0, te, blocks))
        print(f"B={B} fused (conv + side job, gn pass, block2): {us:.2f} us", flush=True)
        blk2 = timed(lambda: b0.block2(x, post=x))
        print(f"B={B} block2 alone: {blk2:.2f} us", flush=True)
