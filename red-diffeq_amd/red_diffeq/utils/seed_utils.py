"""Seed control (reference red_diffeq/utils/seed_utils.py:12-170), same API.

The HIP kernels are deterministic by construction (no float atomics, fixed reduction order),
so the determinism switches below only concern PyTorch's own ops.
"""
import os
import random

import numpy as np
import torch


def set_seed(seed: int, verbose: bool = True, allow_tf32: bool = False):
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)
    torch.backends.cudnn.deterministic = True
    torch.backends.cudnn.benchmark = False
    try:
        torch.use_deterministic_algorithms(True, warn_only=True)
    except (AttributeError, TypeError):
        pass
    os.environ["CUBLAS_WORKSPACE_CONFIG"] = ":4096:8"
    if hasattr(torch.backends.cuda, "matmul"):
        torch.backends.cuda.matmul.allow_tf32 = allow_tf32
    if hasattr(torch.backends.cudnn, "allow_tf32"):
        torch.backends.cudnn.allow_tf32 = allow_tf32
    if verbose:
        print(f"   - Random seed set to: {seed} (python, numpy, torch CPU/GPU); deterministic algorithms on")


def worker_init_fn(worker_id: int, base_seed: int = 0):
    s = base_seed + worker_id
    random.seed(s)
    np.random.seed(s)
    torch.manual_seed(s)


def get_rng_state():
    state = {"python_random": random.getstate(), "numpy": np.random.get_state(),
             "torch": torch.get_rng_state()}
    if torch.cuda.is_available():
        state["cuda"] = torch.cuda.get_rng_state_all()
    return state


def set_rng_state(state: dict):
    random.setstate(state["python_random"])
    np.random.set_state(state["numpy"])
    torch.set_rng_state(state["torch"])
    if torch.cuda.is_available() and "cuda" in state:
        torch.cuda.set_rng_state_all(state["cuda"])


class SeedContext:
    """``with SeedContext(42): ...`` — temporary seed, previous RNG state restored on exit."""

    def __init__(self, seed: int):
        self.seed = seed
        self.saved_state = None

    def __enter__(self):
        self.saved_state = get_rng_state()
        set_seed(self.seed, verbose=False)
        return self

    def __exit__(self, exc_type, exc_val, exc_tb):
        set_rng_state(self.saved_state)
        return False
