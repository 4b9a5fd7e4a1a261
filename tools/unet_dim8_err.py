"""Error of the HIP U-Net (dim 8, the reference's own fixture weights and inputs) against the
reference's outputs and against the torch fp32 restatement on the same device, per output."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "red-diffeq_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import load_golden  # noqa: E402
import unet_torch_ref as R  # noqa: E402
from red_diffeq.models.diffusion import Unet  # noqa: E402

z = load_golden("unet_dim8")
net = Unet(dim=8, dim_mults=(1, 2, 4, 8), channels=1)
net.load_state_dict({k[3:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("sd.")})
net = net.cuda().eval()
x = torch.from_numpy(z["x"]).cuda()
t = torch.from_numpy(z["t"]).cuda()
with torch.no_grad():
    out = net(x, t)
    ref_t = R.unet_forward(net, x, t)
ref = torch.from_numpy(z["out"]).cuda()
sc = ref.abs().max().item()
print(json.dumps({"max_abs_vs_reference": (out - ref).abs().max().item(), "scale": sc,
                  "rel_vs_reference": (out - ref).abs().max().item() / sc,
                  "rel_torch_vs_reference": (ref_t - ref).abs().max().item() / sc,
                  "rel_vs_torch_same_device": (out - ref_t).abs().max().item() / sc}))
