"""Diagnostic: is a U-Net sample's output independent of the batch it is computed in?  For fp32 and
bf16, the dim-64 U-Net (synthetic weights) on N random 72x72 inputs: batched (B = N) vs each sample
alone (B = 1), and vs B = 8 chunks; prints max |diff| / max |out| per comparison."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "red-diffeq_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
from ckpt_weights import synth_param  # noqa: E402
from red_diffeq.models.diffusion import Unet  # noqa: E402

dev = torch.device("cuda:0")
net = Unet(dim=64, dim_mults=(1, 2, 4, 8), channels=1)
net.load_state_dict({k: torch.from_numpy(synth_param("model." + k, v.shape)) for k, v in net.state_dict().items()})
net = net.to(dev).eval()
N = int(sys.argv[1]) if len(sys.argv) > 1 else 40
g = torch.Generator(device=dev).manual_seed(1)
x = torch.randn(N, 1, 72, 72, device=dev, generator=g).clamp(-1, 1)
t = torch.randint(0, 1000, (N,), device=dev, generator=g)
for prec in ("fp32", "bf16"):
    net.set_precision(prec)
    with torch.no_grad():
        full = net(x, t)
        one = torch.cat([net(x[i:i + 1], t[i:i + 1]) for i in range(N)])
        eight = torch.cat([net(x[i:i + 8], t[i:i + 8]) for i in range(0, N, 8)])
    sc = float(full.abs().max())
    print(json.dumps({"precision": prec, "N": N, "full_vs_B1_max_rel": float((full - one).abs().max()) / sc,
                      "full_vs_B8_max_rel": float((full - eight).abs().max()) / sc,
                      "B8_vs_B1_max_rel": float((eight - one).abs().max()) / sc,
                      "per_sample_worst_B1": [round(float((full[i] - one[i]).abs().max()) / sc, 6) for i in range(min(N, 12))]}),
          flush=True)
