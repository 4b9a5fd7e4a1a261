"""The FWI plan's production tuning and its calling contract (include/red_diffeq_fwi.h).

* configs[4]'s chunked kernels run with the plan's automatic tuning: two concurrent launch chains and
  several shots of one region per workgroup (k_fwd_tw / k_adj_tw shot loop with the next shot's loads
  pipelined, the gk partials added with a no-return fp64 atomic).  These tests pin exactly those
  settings -- 16 shots per workgroup with an uneven last group, two and three chains, graph replays,
  and the full 740 x 3240 grid with the defaults -- bitwise against one shot per workgroup on one
  chain, which test_gpu_fwi.py pins to the oracle (reference pde.py:61-86).
* One call in flight per plan: calls from two streams, and from two host threads, on one plan give
  the results of calls made one after the other.
"""
import threading

import numpy as np
import pytest
import torch

from conftest import vnorm
from oracle import oracle as O
from test_gpu_fwi import _shot_sum, bits_equal, make_fwi

pytestmark = pytest.mark.gpu


def _run_tuned(plan, v, B, dseis, T, fspw, aspw, chains, reps=2):
    """Chunked forward (history) + adjoint with the given wide tuning; `reps` calls (the first
    captures the graphs, the rest replay them), each equal to the first bit for bit.  Returns
    (seis, per-shot gA [B, ns, Hp, Wp], gbeta [B, ns], gk sum [B]) of the last call."""
    plan.set_persistent(False)
    plan.set_variant(wide_chunked=True)
    plan.set_tuning(T, T, chains)
    plan.set_wide_adj_steps(0)
    plan.set_wide_fwd_shots(fspw)
    plan.set_wide_adj_shots(aspw)
    sz = plan.sizes(B)
    outs = []
    for _ in range(reps):
        coeffs, _ = plan.coeffs(v, 0)
        seis, hist = plan.forward(coeffs, B, keep_history=True)
        gA, gk, gb = plan.adjoint(coeffs, hist, dseis, B)
        plan.status()
        del hist
        outs.append((seis.cpu().numpy(), gA.view(B, plan.ns, sz.Hp, sz.ld)[..., :sz.Wp].cpu().numpy(),
                     gb.view(B, -1).cpu().numpy(), gk.view(B, -1).sum(1).cpu().numpy()))
        del seis, gA, gk, gb
    for o in outs[1:]:
        for a_, b_ in zip(o[:3], outs[0][:3]):
            assert bits_equal(a_, b_)
        assert np.array_equal(o[3], outs[0][3])
    return outs[-1]


def _reset(plan):
    plan.set_wide_fwd_shots(0)
    plan.set_wide_adj_shots(0)
    plan.set_tuning(4, 4, 0)


def test_wide_16_shots_per_workgroup_two_chains_bitexact(cuda):
    """35 shots (>= 17, so a workgroup runs 16 shots and the last group is uneven: one
    chain 16 + 16 + 3; two chains 16 + 1 and 16 + 2; three chains 11 / 12 / 12), explicit 16 and the
    automatic choice, graph capture and replay: seismograms, gA and gbeta equal one shot per workgroup
    on one chain bit for bit, gk (fp64 adds in launch order) to 1e-12; and those equal the oracle's
    (gA / gbeta bitwise, gk at rtol 1e-7).  A shot-index defect at shot >= 5 of the loop (LDS reused
    across shots, a next-shot prefetch into a live register) would show here."""
    from red_diffeq.utils.synthetic import make_model
    ns = 35
    ctx = dict(n_grid=71, nt=158, dx=10.0, dt=0.001, nbc=20, f=15.0, sz=10, gz=10, ng=71, ns=ns)
    vn = vnorm(make_model("curvefault", 36, 71, seed=21, batch=1))
    fwi = make_fwi(dict(ctx))
    v = torch.from_numpy(vn).to(cuda)
    plan = fwi._plan(36, 71, v.device)
    B = 1
    sz = plan.sizes(B)
    rng = np.random.default_rng(35)
    dseis_np = rng.standard_normal((B, ns, sz.nrec, plan.ng)).astype(np.float32)
    dseis = torch.from_numpy(dseis_np).to(cuda)
    try:
        for T in (4, 3):
            ref = _run_tuned(plan, v, B, dseis, T, 1, 1, 1)
            for fspw, aspw, chains, want in ((16, 16, 1, (1, 16, 16, 35)), (16, 16, 2, (2, 16, 16, 17)),
                                             (16, 16, 3, (3, 11, 11, 11)), (0, 0, 0, None), (8, 16, 2, None)):
                plan.set_tuning(T, T, chains)
                plan.set_wide_fwd_shots(fspw)
                plan.set_wide_adj_shots(aspw)
                info = plan.wide_info(B)
                if want is not None:
                    assert (info["chains"], info["fwd_spw"], info["adj_spw"], info["chain0_shots"]) == want, info
                got = _run_tuned(plan, v, B, dseis, T, fspw, aspw, chains)
                for name, a_, b_ in zip(("seis", "gA", "gbeta"), got[:3], ref[:3]):
                    assert bits_equal(a_, b_), (T, fspw, aspw, chains, info, name)
                np.testing.assert_allclose(got[3], ref[3], rtol=1e-12)
            if T == 4:
                f = O.OracleFWI(dict(ctx), B)
                so, c = f.forward(vn, keep_history=True)
                oA, oK, ob = f.adjoint(c, dseis_np)
                assert bits_equal(ref[0], so)
                assert bits_equal(_shot_sum(ref[1]), oA)
                assert bits_equal(ref[2], ob)
                np.testing.assert_allclose(ref[3], oK, rtol=1e-7)
    finally:
        _reset(plan)


def test_configs4_grid_default_tuning_bitexact(cuda):
    """the full configs[4] grid (500 x 3000 model, nbc 120: 740 x 3240 padded, 3000
    receivers), 16 shots, nt = 150, with the plan's DEFAULT tuning -- automatic shots per workgroup,
    automatic chains (two), wide adjoint depth 5, forward depth 4 -- and with one chain (where the
    automatic choice is 16 shots per workgroup for both kernels), against one shot per workgroup on
    one chain (the setting test_marmousi_scale_grid_vs_oracle pins to the oracle): seismograms, gA,
    gbeta bitwise; gk to 1e-12."""
    from red_diffeq.utils.synthetic import make_model
    nz, nx, ns = 500, 3000, 16
    ctx = dict(n_grid=nx, nt=150, dx=10.0, dt=0.001, nbc=120, f=15.0, sz=10, gz=10, ng=nx, ns=ns)
    vn = vnorm(make_model("curvefault", nz, nx, seed=5, batch=1))
    fwi = make_fwi(dict(ctx))
    v = torch.from_numpy(vn).to(cuda)
    plan = fwi._plan(nz, nx, v.device)
    B = 1
    sz = plan.sizes(B)
    assert (sz.Hp, sz.Wp) == (740, 3240)
    dseis = torch.from_numpy(np.random.default_rng(16).standard_normal((B, ns, sz.nrec, plan.ng))
                             .astype(np.float32)).to(cuda)
    try:
        info = plan.launch_info(B)
        assert not info["fwd_persistent"] and not info["adj_persistent"] and info["adj_T"] == 5
        assert plan.wide_info(B) == {"chains": 2, "fwd_spw": 8, "adj_spw": 8, "chain0_shots": 8}
        default = _run_tuned(plan, v, B, dseis, 4, 0, 0, 0)
        plan.set_tuning(4, 4, 1)
        assert plan.wide_info(B) == {"chains": 1, "fwd_spw": 16, "adj_spw": 16, "chain0_shots": 16}
        one_chain = _run_tuned(plan, v, B, dseis, 4, 0, 0, 1)
        ref = _run_tuned(plan, v, B, dseis, 4, 1, 1, 1, reps=1)
        for got, what in ((default, "default"), (one_chain, "one chain, 16 per workgroup")):
            for name, a_, b_ in zip(("seis", "gA", "gbeta"), got[:3], ref[:3]):
                assert bits_equal(a_, b_), (what, name)
            np.testing.assert_allclose(got[3], ref[3], rtol=1e-12)
    finally:
        _reset(plan)


def _openfwi_plan(cuda, ns=5, nt=400):
    from red_diffeq.utils.synthetic import make_model
    ctx = dict(n_grid=70, nt=nt, dx=10.0, dt=0.001, nbc=120, f=15.0, sz=10, gz=10, ng=70, ns=ns)
    vn = vnorm(make_model("curvefault", 70, 70, seed=3, batch=1))
    fwi = make_fwi(dict(ctx))
    v = torch.from_numpy(vn).to(cuda)
    return fwi, fwi._plan(70, 70, v.device), v


@pytest.mark.parametrize("persistent", [True, False])
def test_plan_calls_from_two_streams_do_not_overlap(cuda, persistent):
    """One call in flight per plan: a forward and an adjoint enqueued on stream A and, without any
    host synchronisation, the same calls on stream B (other buffers).  The persistent launches each
    take the whole chip and share the plan's arrival counters, so overlapping them would leave one
    grid non-resident (status 2) or corrupt the slot assignment; the plan orders B's calls after A's.
    Both results equal a call made alone, bit for bit, and the status word stays clear."""
    fwi, plan, v = _openfwi_plan(cuda)
    B = 1
    plan.set_persistent(persistent)
    plan.set_tuning(4, 4, 0)
    info = plan.launch_info(B)
    assert info["fwd_persistent"] == persistent and info["adj_persistent"] == persistent
    sz = plan.sizes(B)
    dseis = torch.from_numpy(np.random.default_rng(2).standard_normal((B, plan.ns, sz.nrec, plan.ng))
                             .astype(np.float32)).to(cuda)
    coeffs, _ = plan.coeffs(v, 0)
    seis0, hist0 = plan.forward(coeffs, B, keep_history=True)
    g0 = plan.adjoint(coeffs, hist0, dseis, B)
    plan.status()
    want = [seis0.cpu().numpy()] + [t.cpu().numpy() for t in g0]
    del hist0
    sA, sB = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    got = []
    for _ in range(2):                      # the plan's stream alternates A, B, A, B
        for s in (sA, sB):
            with torch.cuda.stream(s):
                seis, hist = plan.forward(coeffs, B, keep_history=True)
                g = plan.adjoint(coeffs, hist, dseis, B)
                got.append((s, seis, hist) + tuple(g))
    torch.cuda.synchronize()
    assert plan.debug_words()[0] == 0
    plan.status()
    for s, seis, hist, *g in got:
        assert bits_equal(seis.cpu().numpy(), want[0])
        for a_, b_ in zip(g, want[1:]):
            assert np.array_equal(a_.cpu().numpy(), b_)


def test_plan_calls_from_two_threads(cuda):
    """Two host threads share one plan (its graph cache, chain streams and events are guarded by the
    plan's mutex), each on its own stream, several calls each, chunked kernels with two launch chains
    (graph capture racing with replay): every result equals a call made alone, bit for bit."""
    fwi, plan, v = _openfwi_plan(cuda, ns=4, nt=200)
    B = 1
    plan.set_persistent(False)
    plan.set_tuning(4, 4, 2)
    coeffs, _ = plan.coeffs(v, 0)
    want = plan.forward(coeffs, B, keep_history=False)[0].cpu().numpy()
    torch.cuda.synchronize()
    errors, results = [], []

    def worker():
        try:
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                for _ in range(6):
                    results.append(plan.forward(coeffs, B, keep_history=False)[0])
            s.synchronize()
        except Exception as e:          # surfaced in the main thread
            errors.append(e)

    th = [threading.Thread(target=worker) for _ in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    torch.cuda.synchronize()
    assert not errors, errors
    assert len(results) == 12
    for r in results:
        assert bits_equal(r.cpu().numpy(), want)
    plan.status()


def test_sweep_delay_changes_timing_only(cuda):
    """rdq_fwi_set_sweep_delay (the persistent kernels' wait between an epoch's publish and its first
    hand-off pass) moves only the timing: seismograms and the adjoint accumulators are bitwise those of
    no delay, for the defaults, 0.25 us and a 5 us delay (many epochs then find their granules at once)."""
    fwi, plan, v = _openfwi_plan(cuda, ns=8, nt=300)
    B = 1
    assert plan.launch_info(B)["fwd_persistent"] and plan.launch_info(B)["adj_persistent"]
    sz = plan.sizes(B)
    dseis = torch.from_numpy(np.random.default_rng(4).standard_normal((B, plan.ns, sz.nrec, plan.ng))
                             .astype(np.float32)).to(cuda)
    coeffs, _ = plan.coeffs(v, 0)
    outs = []
    try:
        for d in ((0, 0), (15, 0), (25, 25), (500, 500)):
            plan.set_sweep_delay(*d)
            seis, hist = plan.forward(coeffs, B, keep_history=True)
            g = plan.adjoint(coeffs, hist, dseis, B)
            plan.status()
            outs.append([seis.cpu().numpy()] + [t.cpu().numpy() for t in g])
            del hist
    finally:
        plan.set_sweep_delay(15, 0)                       # the defaults
    for o in outs[1:]:
        for a_, b_ in zip(o, outs[0]):
            assert np.array_equal(a_.view(np.uint8), b_.view(np.uint8))
