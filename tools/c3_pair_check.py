"""Bitwise fingerprint of the bf16 convolutions under the library RDQ_HIP_LIB selects (kernel A/B: a
restructured kernel must give the same bits as the product one).  Every tools/conv_micro.py shape at
B = 344 in bf16 (sha256 of the output) and the whole bf16 U-Net forward on 344 tiles (dim 64, seeded
weights and inputs).  python tools/c3_pair_check.py OUT.json; compare two outputs with --cmp A.json B.json"""
import hashlib
import json
import os
import sys

if sys.argv[1] == "--cmp":
    A, B = (json.load(open(f)) for f in sys.argv[2:4])
    bad = [k for k in A if A[k] != B.get(k)]
    print(json.dumps({"compared": len(A), "differ": bad}))
    sys.exit(1 if bad else 0)

import torch  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "red-diffeq_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from red_diffeq import ops  # noqa: E402,F401
from red_diffeq.models.diffusion import Unet  # noqa: E402
import conv_micro  # noqa: E402

out = {}
B = 344
for name, (cin1, cin2, cout, k, H, mode) in conv_micro.SHAPES.items():
    g = torch.Generator(device="cuda").manual_seed(1)
    hs = H // 2 if mode == 1 else H
    x = torch.randn(B, cin1, hs, hs, device="cuda", generator=g)
    x2 = torch.randn(B, cin2, H, H, device="cuda", generator=g) if cin2 else None
    w = torch.randn(cout, cin1 + cin2, k, k, device="cuda", generator=g) * 0.05
    b = torch.randn(cout, device="cuda", generator=g)
    y = torch.ops.red_diffeq.conv2d_mfma(x, x2, w, b, None, k // 2, mode, True)
    out[name] = hashlib.sha256(y.cpu().numpy().tobytes()).hexdigest()
    del x, x2, y
torch.manual_seed(0)
net = Unet(dim=64, dim_mults=(1, 2, 4, 8), channels=1).cuda().eval()
net.set_precision("bf16")
x = torch.randn(B, 1, 72, 72, device="cuda").clamp(-1, 1)
t = torch.randint(0, 1000, (B,), device="cuda")
with torch.no_grad():
    y = net(x, t)
out["unet_bf16_b344"] = hashlib.sha256(y.cpu().numpy().tobytes()).hexdigest()
out["unet_bf16_b344_finite"] = bool(torch.isfinite(y).all().item())
json.dump(out, open(sys.argv[1], "w"))
print(json.dumps(out))
