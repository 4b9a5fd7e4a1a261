"""Deterministic synthetic weights for the dim-64 checkpoint round-trip fixture (test infrastructure).

The reference's pretrained checkpoints (pretrained_models/model-3.pt / model-4.pt) are not shipped,
and a seeded dim-64 state_dict is 143 MB, too large to commit.  Instead both sides regenerate the
same weights from this function: tests/golden/make_golden.py loads them into the REFERENCE
GaussianDiffusion(Unet(dim=64, dim_mults=(1,2,4,8))) to record its eps-hat, and
tests/test_gpu_ckpt.py writes them (plus the fixture's schedule buffers) into a checkpoint file in
the reference's layout ({"model": state_dict, ...}, models/diffusion.py:617-625) and loads it
through the drop-in scripts/run_inversion.py reader.
"""
import zlib

import numpy as np


def synth_param(name, shape):
    """float32 array for state_dict entry `name`: fan-in-scaled normals for weights, gains near 1
    for norm scales, small normals for biases; a pure function of (name, shape)."""
    rng = np.random.default_rng(zlib.crc32(name.encode()))
    shape = tuple(int(s) for s in shape)
    z = rng.standard_normal(shape)
    if name.endswith(".g") or (".norm." in name and name.endswith(".weight")):
        return (1.0 + 0.1 * z).astype(np.float32)      # RMSNorm g (1,C,1,1) / GroupNorm weight
    if len(shape) >= 2:
        fan_in = int(np.prod(shape[1:]))
        return (z / np.sqrt(fan_in)).astype(np.float32)
    return (0.05 * z).astype(np.float32)
