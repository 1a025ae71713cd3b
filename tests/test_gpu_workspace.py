"""Workspace and argument-normalisation regressions:

* the few-point division chain of kzgx_prove_range writes only the m = n - len
  quotient coefficients the caller allocated (no device write past ws->q);
* a workspace slot is rebound after an event recorded by the call that last
  used it, so the streams that used it may be destroyed in between;
* evaluation points are residues mod r (x and x + r are one point, as in
  NTL's ZZ_p, src/trusted_setup.cpp:214-219);
* kzgx_set_fixed_base_budget needs the SRS in place.
"""
import gc

import numpy as np
import pytest

import kzg_ref as K

pytestmark = pytest.mark.gpu


def limbs(vals, nl=4):
    import corc
    return corc.ints_to_limbs(vals, nl)


def pt(curve, row, inf=False):
    import corc
    return None if inf else corc.array_to_points(curve, row[None, :])[0]


def _range_proof_exp(C, tau, P, xs):
    """[q(tau)]G1, q = (P - I) / Z (reference create_proof, trusted_setup.cpp:203-228)"""
    r = C.r
    if len(P) <= len(xs):
        return None
    q = list(P)
    for x in xs:  # P div Z by one synthetic division per linear factor
        out = [0] * (len(q) - 1)
        acc = 0
        for k in range(len(q) - 1, 0, -1):
            acc = (acc * x + q[k]) % r
            out[k - 1] = acc
        q = out
    return K.commit_via_tau(C, tau, q)


@pytest.mark.parametrize("n,len_", [(6, 3), (7, 4), (5, 3), (9, 4)])
def test_prove_range_division_chain_stays_in_bounds(n, len_):
    """the division chain used to write up to m + len - 1
    coefficients into d_q, which holds m.  A first, longer opening grows ws->q
    and fills it; a short one must leave every word past its m coefficients
    untouched, and stay exact."""
    import kzgx
    C = K.BN254
    tau = K.default_tau(C)
    ctx = kzgx.Context("BN254")
    try:
        ctx.gen_srs(tau, 64)
        big = K.random_scalars(C, 48, seed=0xA1)
        ctx.prove_range(limbs(big), limbs([5, 9, 11]))  # ws->q: 45 coefficients
        cap = 45 * 32
        before = ctx.debug_ws_read("q", cap)
        P = K.random_scalars(C, n, seed=0xB0 + n)
        xs = [2 + 3 * k for k in range(len_)]
        out, inf = ctx.prove_range(limbs(P), limbs(xs))
        after = ctx.debug_ws_read("q", cap)
        m = n - len_
        assert np.array_equal(before[m * 32:], after[m * 32:]), "write past the m quotient coefficients"
        assert pt("BN254", out, inf) == _range_proof_exp(C, tau, P, xs)
    finally:
        ctx.close()


def test_workspace_rebinding_after_streams_are_destroyed():
    """8 streams bind the 8 workspace slots and are then
    destroyed; 4 new streams must rebind slots without touching the dead
    stream handles, and stay exact"""
    import torch
    import kzgx
    C = K.BN254
    tau = K.default_tau(C)
    ctx = kzgx.Context("BN254")
    try:
        n, B = 129, 2
        ctx.gen_srs(tau, n + 1)
        dev = torch.device("cuda", 0)
        polys = [K.random_scalars(C, n, seed=1300 + s) for s in range(12)]
        d_c = [torch.from_numpy(np.concatenate([limbs(p)] * B).view(np.int64)).to(dev) for p in polys]
        outs = [torch.zeros((B, 8), dtype=torch.int64, device=dev) for _ in polys]
        infs = [torch.zeros((B,), dtype=torch.int32, device=dev) for _ in polys]
        torch.cuda.synchronize(dev)
        old = [torch.cuda.Stream(device=dev) for _ in range(8)]
        for s, st in enumerate(old):
            ctx.msm_batch_device(d_c[s].data_ptr(), n, B, n, outs[s].data_ptr(), infs[s].data_ptr(), st.cuda_stream)
        torch.cuda.synchronize(dev)
        del old, st
        gc.collect()
        new = [torch.cuda.Stream(device=dev) for _ in range(4)]
        for k, st in enumerate(new):
            s = 8 + k
            ctx.msm_batch_device(d_c[s].data_ptr(), n, B, n, outs[s].data_ptr(), infs[s].data_ptr(), st.cuda_stream)
        torch.cuda.synchronize(dev)
        for s in range(12):
            exp = K.commit_via_tau(C, tau, polys[s])
            o = outs[s].cpu().numpy().view(np.uint64)
            for b in range(B):
                assert pt("BN254", o[b], bool(infs[s][b].item())) == exp, s
    finally:
        ctx.close()


def test_prove_range_points_are_residues_mod_r():
    """x + r is the point x (ZZ_p); a pair {x, x + r} is a
    repeated point (KZGX_ERR_DIV_ZERO), and a lone x + r opens like x"""
    import kzgx
    C = K.BN254
    tau = K.default_tau(C)
    ctx = kzgx.Context("BN254")
    try:
        ctx.gen_srs(tau, 40)
        P = K.random_scalars(C, 30, seed=0xC3)
        a, ia = ctx.prove_range(limbs(P), limbs([7, 12]))
        b, ib = ctx.prove_range(limbs(P), limbs([7 + C.r, 12]))
        assert ia == ib and np.array_equal(a, b)
        assert pt("BN254", a, ia) == _range_proof_exp(C, tau, P, [7, 12])
        with pytest.raises(kzgx.KzgxError) as e:
            ctx.prove_range(limbs(P), limbs([7, 12, 7 + C.r]))
        assert e.value.status == -8
    finally:
        ctx.close()


def test_fixed_base_budget_needs_the_srs():
    """no table can be sized before the SRS exists"""
    import kzgx
    C = K.BN254
    ctx = kzgx.Context("BN254")
    try:
        with pytest.raises(kzgx.KzgxError) as e:
            ctx.set_fixed_base_budget(1 << 30, 100)
        assert e.value.status == -4  # KZGX_ERR_NO_SRS
        ctx.gen_srs(K.default_tau(C), 100)
        c = ctx.set_fixed_base_budget(kzgx.fixed_base_bytes("BN254", 10, 100), 1 << 20)  # clamped to 100 points
        assert c == 10 and ctx.fixed_base_info()[:2] == (10, 100)
    finally:
        ctx.close()
