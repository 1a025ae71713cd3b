"""The default table (kzgx_set_default_table, Ctx::fixed_def): odd multiples
over the first 4097 SRS points at the widest window c <= 12 that fits 4.5% of
the HBM (BN254 c = 12, BLS12-381 c = 11 on an MI355X), built with the SRS,
read by the MSMs that fit in it -- every single create_commit / create_proof
of degree <= 4096 (the reference's benchmark calls,
benchmark/benchmark.cpp:40-66) through the one-launch path, larger batches
through the batched kernel.  Checked against the known-tau identity
commit = [P(tau)]G1 / proof = [q(tau)]G1 (oracle), at the sizes around the
table's edges, on both curves, with a degenerate SRS, and with the table off
or too short (Pippenger)."""
import numpy as np
import pytest

import kzg_ref as K

pytestmark = pytest.mark.gpu

CURVES = [("BN254", K.BN254), ("BLS12381", K.BLS12381)]


def limbs(vals, nl=4):
    import corc
    return corc.ints_to_limbs(vals, nl)


def pt(curve, row, inf=False):
    import corc
    return None if inf else corc.array_to_points(curve, row[None, :])[0]


@pytest.fixture(scope="module")
def lat_ctx():
    import kzgx
    made = {}

    def get(name, C):
        if name not in made:
            ctx = kzgx.Context(name)
            ctx.gen_srs(K.default_tau(C), 4200)
            made[name] = ctx
        return made[name]

    yield get
    for c in made.values():
        c.close()


@pytest.mark.parametrize("name,C", CURVES)
def test_default_table_is_built_by_default(name, C, lat_ctx):
    import kzgx
    import torch
    ctx = lat_ctx(name, C)
    c, n, b = ctx.default_table_info()
    total = torch.cuda.get_device_properties(0).total_memory
    budget = total // 1000 * 45
    assert n == 4097 and 7 <= c <= 12
    assert b == kzgx.fixed_base_bytes(name, c, 4097) <= budget
    if c < 12:  # the widest that fits (the free-memory cap aside)
        assert kzgx.fixed_base_bytes(name, c + 1, 4097) > budget or torch.cuda.mem_get_info()[0] < (8 << 30)
    assert ctx.fixed_base_info()[0] == 0  # the main (throughput) table stays opt-in


@pytest.mark.parametrize("name,C", CURVES)
@pytest.mark.parametrize("n", [1, 2, 129, 4096, 4097, 4098])
def test_single_commit_matches_oracle(name, C, n, lat_ctx):
    """n <= 4097: the latency table; 4098: past its prefix (Pippenger)"""
    ctx = lat_ctx(name, C)
    tau = K.default_tau(C)
    P = K.random_scalars(C, n, seed=7100 + n)
    if n >= 3:
        P[0], P[1], P[-1] = 0, C.r - 1, 2
    out, inf = ctx.msm(limbs(P))
    assert pt(name, out, inf) == K.commit_via_tau(C, tau, P)


@pytest.mark.parametrize("name,C", CURVES)
@pytest.mark.parametrize("batch", [2, 16, 17, 64])
def test_small_batches(name, C, batch, lat_ctx):
    """<= 16 MSMs take the one-launch path, more the batched table kernel
    (c >= 10) or the batched Pippenger"""
    ctx = lat_ctx(name, C)
    tau = K.default_tau(C)
    n = 300
    polys = [K.random_scalars(C, n, seed=7300 + b) for b in range(batch)]
    polys[0] = [0] * n  # the zero polynomial -> infinity
    out, inf = ctx.msm_batch(np.concatenate([limbs(P) for P in polys]), n, batch)
    for b in range(batch):
        assert pt(name, out[b], inf[b]) == K.commit_via_tau(C, tau, polys[b]), b


@pytest.mark.parametrize("name,C", CURVES)
@pytest.mark.parametrize("n,batch", [(4097, 2), (2000, 3), (513, 16)])
def test_small_batches_two_level_fold(name, C, n, batch, lat_ctx):
    """the one-launch kernel's two fold levels (more than 128 wavefront
    partials per MSM) with per-MSM counters past the first MSM's"""
    ctx = lat_ctx(name, C)
    tau = K.default_tau(C)
    polys = [K.random_scalars(C, n, seed=7400 + 13 * b + n) for b in range(batch)]
    polys[-1][n // 2] = 0
    out, inf = ctx.msm_batch(np.concatenate([limbs(P) for P in polys]), n, batch)
    for b in range(batch):
        assert pt(name, out[b], inf[b]) == K.commit_via_tau(C, tau, polys[b]), b


@pytest.mark.parametrize("name,C", CURVES)
@pytest.mark.parametrize("tau", [1, 2])
def test_degenerate_setup_cooperative_levels(name, C, tau):
    """tau = 1: every SRS point is G, so wavefront partials are small
    multiples of G and the cooperative fold levels meet equal x (doubling)
    and P = -Q; tau = 2 the same with distinct points"""
    import kzgx
    ctx = kzgx.Context(name)
    try:
        ctx.gen_srs(tau, 1600)
        for n in (129, 1500):
            P = [1] * n if tau == 1 else K.random_scalars(C, n, seed=7800 + n)
            out, inf = ctx.msm(limbs(P))
            assert pt(name, out, inf) == K.commit_via_tau(C, tau, P), n
        P = [1, C.r - 1] * 700  # sums to zero
        out, inf = ctx.msm(limbs(P))
        assert pt(name, out, inf) == K.commit_via_tau(C, tau, P)
    finally:
        ctx.close()


@pytest.mark.parametrize("name,C", CURVES)
def test_single_proofs(name, C, lat_ctx):
    """create_proof(poly, z, 1) at degree 128 and 4096: quotient + table MSM"""
    ctx = lat_ctx(name, C)
    tau = K.default_tau(C)
    for n in (129, 4097):
        P = K.random_scalars(C, n, seed=7500 + n)
        z = 12345 + n
        zs = np.array([[z, 0, 0, 0]], dtype=np.uint64)
        out, inf, y = ctx.prove_single_batch(limbs(P), zs)
        assert pt(name, out[0], inf[0]) == K.commit_via_tau(C, tau, K.proof_quotient(C, P, z, 1))


@pytest.mark.parametrize("name,C", CURVES)
def test_default_table_off_and_degenerate(name, C):
    """c = 0 turns it off (Pippenger); tau = 0 (every SRS point but the
    first infinite) still exact through the table"""
    import kzgx
    ctx = kzgx.Context(name)
    try:
        ctx.gen_srs(0, 200)
        c0, n0, _ = ctx.default_table_info()
        assert n0 == 200 and c0 >= 7
        P = K.random_scalars(C, 150, seed=7700)
        out, inf = ctx.msm(limbs(P))
        assert pt(name, out, inf) == K.commit_via_tau(C, 0, P)
        ctx.set_default_table(0)
        assert ctx.default_table_info() == (0, 0, 0)
        out2, inf2 = ctx.msm(limbs(P))
        assert pt(name, out2, inf2) == K.commit_via_tau(C, 0, P)
        ctx.set_default_table(7, 100)  # rebuilt at once over the installed SRS
        assert ctx.default_table_info()[:2] == (7, 100)
        out3, inf3 = ctx.msm(limbs(P[:90]))
        assert pt(name, out3, inf3) == K.commit_via_tau(C, 0, P[:90])
        ctx.set_default_table(-1)  # back to the budget's choice (4097 points, clamped to the SRS)
        assert ctx.default_table_info()[:2] == (c0, 200)
        outb, infb = ctx.msm_batch(np.concatenate([limbs(P[:90])] * 20), 90, 20)
        for b in range(20):
            assert pt(name, outb[b], infb[b]) == K.commit_via_tau(C, 0, P[:90]), b
    finally:
        ctx.close()


def _quotient(C, P, z):
    """synthetic division: q_(k-1) = h_k = sum_(i >= k) p_i z^(i - k), y = h_0"""
    h, q = 0, [0] * max(len(P) - 1, 0)
    for k in range(len(P) - 1, -1, -1):
        h = (P[k] + h * z) % C.r
        if k >= 1:
            q[k - 1] = h
    return q, h


@pytest.mark.parametrize("name,C", CURVES)
def test_single_opening_quotient_one_workgroup(name, C):
    """create_proof(poly, z, 1) at the sizes of the one-workgroup quotient
    (k_quotient_wg: 512 <= n <= 2^14, batch <= 4) and either side of it, with
    full-width opening points: proof = [q(tau)]G1 and y = P(z)"""
    import kzgx
    ctx = kzgx.Context(name)
    try:
        tau = K.default_tau(C)
        ctx.gen_srs(tau, 16400)
        for n, batch in ((511, 1), (512, 1), (1025, 3), (4097, 4), (5000, 2), (16384, 1), (16385, 1)):
            P = K.random_scalars(C, n, seed=7900 + n)
            zs = K.random_scalars(C, batch, seed=7950 + n)
            out, inf, y = ctx.prove_single_batch(limbs(P), limbs(zs))
            for b in range(batch):
                q, yv = _quotient(C, P, zs[b])
                assert int(sum(int(y[b, i]) << (64 * i) for i in range(4))) == yv, (n, b)
                assert pt(name, out[b], inf[b]) == K.commit_via_tau(C, tau, q), (n, b)
    finally:
        ctx.close()


@pytest.mark.parametrize("name,C", CURVES)
def test_default_table_shared_across_contexts(name, C):
    """8 contexts over one SRS hold ONE default table,
    each of their commits exact; a context over another SRS builds its own;
    the last context to go frees it"""
    import kzgx
    tau = K.default_tau(C) + 4242  # an SRS no other test's context holds
    n0, b0 = kzgx.shared_tables(0)
    ctxs = []
    try:
        for _ in range(8):
            ctx = kzgx.Context(name)
            ctx.gen_srs(tau, 700)
            ctxs.append(ctx)
        c, npts, b = ctxs[0].default_table_info()
        assert npts == 700 and c >= 7
        assert kzgx.shared_tables(0) == (n0 + 1, b0 + b)
        for k, ctx in enumerate(ctxs):
            assert ctx.default_table_info() == (c, npts, b)
            P = K.random_scalars(C, 129 + 70 * k, seed=8100 + k)
            out, inf = ctx.msm(limbs(P))
            assert pt(name, out, inf) == K.commit_via_tau(C, tau, P), k
        other = kzgx.Context(name)
        ctxs.append(other)
        other.gen_srs(tau + 1, 700)
        assert kzgx.shared_tables(0)[0] == n0 + 2
        P = K.random_scalars(C, 400, seed=8200)
        out, inf = other.msm(limbs(P))
        assert pt(name, out, inf) == K.commit_via_tau(C, tau + 1, P)
        # dropping all but one holder keeps the table; the survivor is exact
        for ctx in ctxs[:7]:
            ctx.close()
        ctxs = ctxs[7:]
        assert kzgx.shared_tables(0)[0] == n0 + 2
        out, inf = ctxs[0].msm(limbs(P))
        assert pt(name, out, inf) == K.commit_via_tau(C, tau, P)
    finally:
        for ctx in ctxs:
            ctx.close()
    assert kzgx.shared_tables(0) == (n0, b0)
