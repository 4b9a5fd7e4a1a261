"""The oracle (CPU restatement, oracle/) pinned against fixtures produced by running the
reference itself (tests/golden/make_golden.py).  CPU only."""
import numpy as np
import pytest

from conftest import ctx_of, load_golden, vnorm
from oracle import oracle as O

FWD = [("fwd_small", {}), ("fwd_small_st3", dict(sample_temporal=3, sample_spatial=0.5)), ("fwd_wrap", {}),
       ("fwd_openfwi_ns1", {}), ("fwd_openfwi_ns5_nt400", {})]


@pytest.mark.parametrize("name,kw", FWD)
def test_oracle_forward_bitexact(name, kw):
    z = load_golden(name)
    f = O.OracleFWI(ctx_of(z), z["v"].shape[0], **kw)
    seis, _ = f.forward(vnorm(z["v"]))
    assert seis.shape == z["seis"].shape
    assert np.array_equal(seis.view(np.int32), z["seis"].view(np.int32)), "oracle must be bit-exact"


@pytest.mark.parametrize("name", ["grad_small", "grad_small_mask", "grad_openfwi_ns1"])
def test_oracle_gradient(name):
    z = load_golden(name)
    f = O.OracleFWI(ctx_of(z), z["v_init"].shape[0])
    seis, c = f.forward(vnorm(z["v_init"]), keep_history=True)
    mask = z["mask"] if "mask" in z.files else None
    loss, ds = O.l1_loss(seis, z["y"], mask)
    np.testing.assert_allclose(loss, z["loss"], rtol=2e-6)
    g = f.finalize(c, *f.adjoint(c, ds))
    rel = np.linalg.norm(g - z["grad"]) / np.linalg.norm(z["grad"])
    assert rel < 5e-5, rel
    np.testing.assert_allclose(g, z["grad"], rtol=1e-4, atol=1e-5 * np.abs(z["grad"]).max())


def test_oracle_dot_product_adjoint():
    """<J dv, w> == <dv, J^T w> on a small grid (no reference needed)."""
    z = load_golden("fwd_small")
    ctx = dict(ctx_of(z), nt=160)
    f = O.OracleFWI(ctx, 1)
    rng = np.random.default_rng(0)
    v0 = vnorm(z["v"][:1]).astype(np.float64) + rng.uniform(0, 0.05, (1, 1, 16, 16))
    v0[0, 0, 7, 9] = v0.min() - 0.05   # unique minimum: the sponge term is differentiable
    dv = rng.standard_normal(v0.shape) * 5e-3   # large enough that fp32 forward noise is small
    w = rng.standard_normal((1, f.g.ns, f.nrec, f.g.ng)).astype(np.float32)
    s0, c = f.forward(v0.astype(np.float32), keep_history=True)
    g = f.finalize(c, *f.adjoint(c, w))
    eps = 1.0
    sp, _ = f.forward((v0 + eps * dv).astype(np.float32))
    sm, _ = f.forward((v0 - eps * dv).astype(np.float32))
    lhs = np.sum((sp.astype(np.float64) - sm) / (2 * eps) * w)
    rhs = np.sum(g.astype(np.float64) * dv)
    assert abs(lhs - rhs) / abs(rhs) < 2e-2, (lhs, rhs)
