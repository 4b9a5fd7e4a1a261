"""SSIM of the reference's own final B = 25 models (tests/golden/loop_red_b25.npz) by K12 (fused metrics)
and by the torch port of the reference SSIM module on the GPU, against the reference's CPU value: how far
the metric itself reproduces across implementations on identical inputs."""
import sys, os, numpy as np, torch
sys.path.insert(0, "red-diffeq_amd"); sys.path.insert(0, "tests")
from red_diffeq.core.fused import metrics
from red_diffeq.utils.data_trans import v_normalize
from red_diffeq.utils.ssim import SSIM
z = np.load("tests/golden/loop_red_b25.npz")
mu = torch.from_numpy(z["mu"]).cuda().contiguous()
vt = v_normalize(torch.from_numpy(z["v_true"]).cuda()).contiguous()
m = metrics(mu, vt).cpu().numpy()
ref = z["ssim"][:, -1]
print("K12 ssim vs ref final ssim: max rel", np.max(np.abs(m[2] - ref) / np.abs(ref)))
s = SSIM(window_size=11)
ss = np.array([float(s((mu[i:i+1] + 1) / 2, (vt[i:i+1] + 1) / 2)) for i in range(25)])
print("torch SSIM port vs ref: max rel", np.max(np.abs(ss - ref) / np.abs(ref)))
print("K12 vs torch port: max rel", np.max(np.abs(ss - m[2]) / np.abs(ss)))
print("mae rel", np.max(np.abs(m[0]-z["mae"][:, -1])/z["mae"][:, -1]), "rmse rel", np.max(np.abs(m[1]-z["rmse"][:, -1])/z["rmse"][:, -1]))
