"""GPU parity: the HIP path (through the C ABI) against the CPU oracle.

Bit-exact: affine (x, y) of a group element is unique, so every comparison is
exact equality of canonical integers.  Sizes are chosen so the oracle side
finishes in seconds; full-size cases use the MSM-independent identity
commit == [P(tau)]G1."""
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


@pytest.mark.parametrize("name,C", CURVES)
def test_gen_srs_matches_oracle(name, C, ctx_factory, oracle_c):
    ctx = ctx_factory(name)
    tau = K.default_tau(C)
    ctx.gen_srs(tau, 97, start=5)
    got = ctx.get_srs(97)
    ref = oracle_c.gen_srs(name, tau, 102)[5:]
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("name,C", CURVES)
@pytest.mark.parametrize("n", [1, 2, 3, 17, 129, 600])
def test_msm_matches_naive(name, C, n, ctx_factory, oracle_c):
    ctx = ctx_factory(name)
    tau = K.default_tau(C)
    srs = oracle_c.gen_srs(name, tau, max(n, 2))
    ctx.load_srs(srs)
    sc = K.random_scalars(C, n, seed=1000 + n)
    if n >= 3:
        sc[0], sc[1], sc[2] = 0, 1, C.r - 1
    S = limbs(sc)
    out, inf = ctx.msm(S)
    ref = oracle_c.msm_naive(name, srs, S)
    assert pt(name, out, inf) == ref


@pytest.mark.parametrize("name,C", CURVES)
def test_msm_batch_identity(name, C, ctx_factory):
    ctx = ctx_factory(name)
    tau = K.default_tau(C)
    n, batch = 4097, 6
    ctx.gen_srs(tau, 5000)
    polys = [K.random_scalars(C, n, seed=77 + b) for b in range(batch)]
    polys[1] = [0] * n                       # zero polynomial -> infinity
    polys[2] = [5] + [0] * (n - 1)           # constant
    S = np.concatenate([limbs(p) for p in polys])
    out, inf = ctx.msm_batch(S, n, batch)
    for b in range(batch):
        assert pt(name, out[b], inf[b]) == K.commit_via_tau(C, tau, polys[b]), b


@pytest.mark.parametrize("name,C", CURVES)
@pytest.mark.parametrize("batch", [255, 256])
def test_msm_batch_fold_forms(name, C, batch, ctx_factory):
    """Pippenger's bucket fold switches form at 256 MSMs per call (workgroup
    fold with inline affine conversion below, wavefront fold + finish kernel
    from there): both sides of the switch, every MSM checked"""
    ctx = ctx_factory(name)
    tau = K.default_tau(C)
    n = 65
    ctx.gen_srs(tau, n)
    rng = np.random.default_rng(0xF01D + batch)
    S = rng.integers(0, 2**63, size=(batch, n, 4), dtype=np.uint64)
    S[..., 3] &= np.uint64((1 << 59) - 1)  # < 2^251 < r: canonical
    S[7] = 0                               # zero polynomial -> infinity
    S[9, 1:] = 0                           # constant polynomial
    out, inf = ctx.msm_batch(S.reshape(batch * n, 4), n, batch)
    for b in range(batch):
        coeffs = [sum(int(S[b, i, k]) << (64 * k) for k in range(4)) for i in range(n)]
        assert pt(name, out[b], inf[b]) == K.commit_via_tau(C, tau, coeffs), b


@pytest.mark.parametrize("name,C", CURVES)
@pytest.mark.parametrize("tau", [0, 1, 2, -1])
def test_degenerate_srs(name, C, tau, ctx_factory, oracle_c):
    """tau = 0 gives infinite SRS points, tau = +-1 repeats points (bucket doublings)."""
    ctx = ctx_factory(name)
    t = tau % C.r
    n = 300
    srs = oracle_c.gen_srs(name, t, n)
    ctx.load_srs(srs)
    sc = K.random_scalars(C, n, seed=5)
    sc[7] = sc[3]
    out, inf = ctx.msm(limbs(sc))
    assert pt(name, out, inf) == K.commit_via_tau(C, t, sc)


@pytest.mark.parametrize("name,C", CURVES)
def test_empty_msm_is_infinity(name, C, ctx_factory):
    ctx = ctx_factory(name)
    ctx.gen_srs(K.default_tau(C), 8)
    out, inf = ctx.msm_batch(np.zeros((0, 4), dtype=np.uint64), 0, 2)
    assert inf.all() and not out.any()


@pytest.mark.parametrize("name,C", CURVES)
@pytest.mark.parametrize("n", [1, 2, 5, 64, 65, 130, 4097])
def test_single_opening_proofs(name, C, n, ctx_factory):
    ctx = ctx_factory(name)
    tau = K.default_tau(C)
    ctx.gen_srs(tau, max(n + 1, 8))
    P = K.random_scalars(C, n, seed=n)
    zs = [0, 1, 7, n + 3, C.r - 2]
    out, inf, y = ctx.prove_single_batch(limbs(P), limbs(zs))
    for j, z in enumerate(zs):
        q = K.proof_quotient(C, P, z, 1) if z < 2**31 else None
        yv = K.poly_eval(C, P, z)
        assert int(sum(int(y[j, i]) << (64 * i) for i in range(4))) == yv
        # q(tau) = (P(tau) - P(z)) / (tau - z)
        qt = (K.poly_eval(C, P, tau) - yv) * pow((tau - z) % C.r, -1, C.r) % C.r
        exp = K.scalar_mul(C, (C.gx, C.gy), qt)
        assert pt(name, out[j], inf[j]) == exp, (n, z)
        if q is not None and n < 200:
            assert pt(name, out[j], inf[j]) == K.commit_via_tau(C, tau, q)


@pytest.mark.parametrize("name,C", CURVES)
def test_prove_batch_distinct_polys(name, C, ctx_factory):
    ctx = ctx_factory(name)
    tau = K.default_tau(C)
    n, batch = 513, 5
    ctx.gen_srs(tau, n + 1)
    polys = [K.random_scalars(C, n, seed=300 + b) for b in range(batch)]
    zs = [b * 11 for b in range(batch)]
    coeffs = np.stack([limbs(p) for p in polys])
    out, inf, y = ctx.prove_single_batch(coeffs, limbs(zs), shared=False)
    for b in range(batch):
        q = K.proof_quotient(C, polys[b], zs[b], 1)
        assert pt(name, out[b], inf[b]) == K.commit_via_tau(C, tau, q)


@pytest.mark.parametrize("name,C", CURVES)
@pytest.mark.parametrize("n", [1, 2, 9, 100, 257])
def test_poly_eval_and_interpolate(name, C, n, ctx_factory, oracle_c):
    ctx = ctx_factory(name)
    P = K.random_scalars(C, n, seed=n + 9)
    xs = [i + 3 for i in range(n)]
    ys = ctx.poly_eval(limbs(P), limbs(xs))
    assert oracle_c.limbs_to_ints(ys) == [K.poly_eval(C, P, x) for x in xs]
    coeffs = ctx.interpolate(limbs(xs), ys)
    got = oracle_c.limbs_to_ints(coeffs)
    assert got == P + [0] * (n - len(P))
    # arbitrary nodes + values (signed-char style residues)
    xs2 = K.random_scalars(C, n, seed=4 * n)
    ys2 = [(-(i % 200)) % C.r for i in range(n)]
    got2 = oracle_c.limbs_to_ints(ctx.interpolate(limbs(xs2), limbs(ys2)))
    ref2 = oracle_c.interpolate(name, xs2, ys2)
    assert K.normalize(got2) == ref2


@pytest.mark.parametrize("name,C", CURVES)
def test_interpolate_duplicate_node_raises(name, C, ctx_factory):
    import kzgx
    ctx = ctx_factory(name)
    with pytest.raises(kzgx.KzgxError):
        ctx.interpolate(limbs([1, 2, 1]), limbs([3, 4, 5]))


@pytest.mark.parametrize("name,C", CURVES)
def test_g1_sum(name, C, ctx_factory, oracle_c):
    ctx = ctx_factory(name)
    srs = oracle_c.gen_srs(name, 3, 6)
    out, inf = ctx.g1_sum(srs)
    exp = K.scalar_mul(C, (C.gx, C.gy), 1 + 3 + 9 + 27 + 81 + 243)
    assert pt(name, out, inf) == exp


@pytest.mark.parametrize("name,C", CURVES)
def test_g1_sum_device(name, C, ctx_factory, oracle_c):
    """kzgx_g1_sum_device (the sharded commit's on-device fold): device
    points + uint32 infinity flags, enqueued on a torch stream"""
    import torch
    ctx = ctx_factory(name)
    srs = oracle_c.gen_srs(name, 3, 6)
    dev = torch.device("cuda", 0)
    pts = torch.from_numpy(np.ascontiguousarray(srs).view(np.int64)).to(dev)
    flags = torch.tensor([0, 1, 0, 0, 1, 0], dtype=torch.int32, device=dev)  # drop 3^1 and 3^4
    out = torch.zeros((2 * ctx.w64,), dtype=torch.int64, device=dev)
    oinf = torch.ones((1,), dtype=torch.int32, device=dev)
    st = torch.cuda.Stream(device=dev)
    torch.cuda.synchronize(dev)
    ctx.g1_sum_device(pts.data_ptr(), flags.data_ptr(), 6, out.data_ptr(), oinf.data_ptr(), st.cuda_stream)
    st.synchronize()
    exp = K.scalar_mul(C, (C.gx, C.gy), 1 + 9 + 27 + 243)
    assert pt(name, out.cpu().numpy().view(np.uint64), bool(oinf.item())) == exp
    # all flagged -> infinity; no flags pointer -> plain sum
    flags.fill_(1)
    ctx.g1_sum_device(pts.data_ptr(), flags.data_ptr(), 6, out.data_ptr(), oinf.data_ptr(), st.cuda_stream)
    st.synchronize()
    assert bool(oinf.item())
    ctx.g1_sum_device(pts.data_ptr(), None, 6, out.data_ptr(), oinf.data_ptr(), st.cuda_stream)
    st.synchronize()
    exp = K.scalar_mul(C, (C.gx, C.gy), 1 + 3 + 9 + 27 + 81 + 243)
    assert pt(name, out.cpu().numpy().view(np.uint64), bool(oinf.item())) == exp


@pytest.mark.parametrize("name,C", CURVES)
@pytest.mark.parametrize("n", [0, 1, 2, 3, 5, 9, 64, 100, 257])
def test_vanishing(name, C, n, ctx_factory, oracle_c):
    ctx = ctx_factory(name)
    xs = K.random_scalars(C, n, seed=n)
    got = oracle_c.limbs_to_ints(ctx.vanishing(limbs(xs)))
    assert got == K.linear_roots(C, xs)


@pytest.mark.parametrize("name,C", CURVES)
@pytest.mark.parametrize("c,seg", [(10, 1), (11, 7), (12, 1000), (13, 64)])
def test_msm_window_and_segment_variants(name, C, c, seg):
    """every supported window width / segment length gives the same group element"""
    import kzgx
    ctx = kzgx.Context(name)
    try:
        ctx.set_window_bits(c)
        ctx.set_segment(seg)
        tau = K.default_tau(C)
        ctx.gen_srs(tau, 700)
        n, batch = 700, 3
        polys = [K.random_scalars(C, n, seed=c * 100 + b) for b in range(batch)]
        S = np.concatenate([limbs(p) for p in polys])
        out, inf = ctx.msm_batch(S, n, batch)
        for b in range(batch):
            assert pt(name, out[b], inf[b]) == K.commit_via_tau(C, tau, polys[b])
        with pytest.raises(kzgx.KzgxError):
            ctx.set_window_bits(10)  # table already built
    finally:
        ctx.close()


@pytest.mark.parametrize("name,C", CURVES)
@pytest.mark.parametrize("n", [16384, 16385, 20000, 70001, 131072, 140001])
def test_large_single_msm_chunked(name, C, n, ctx_factory):
    """single large MSMs: one Pippenger below 2^17 points (segments shrink to
    spread it), from 2^17 a chunked batch + XYZZ tree sum"""
    ctx = ctx_factory(name)
    tau = K.default_tau(C)
    ctx.gen_srs(tau, n + 3)
    sc = K.random_scalars(C, n, seed=n)
    sc[n // 2] = 0
    out, inf = ctx.msm(limbs(sc))
    assert pt(name, out, inf) == K.commit_via_tau(C, tau, sc)


@pytest.mark.parametrize("name,C", CURVES)
def test_prove_range_duplicate_point_raises(name, C, ctx_factory, oracle_c):
    """kzgx_prove_range with a repeated opening point: the reference's
    interpolation (NTL polyfit) fails on it, so does the opening
    (KZGX_ERR_DIV_ZERO), even though P div Z alone would be defined"""
    import kzgx
    ctx = ctx_factory(name)
    ctx.load_srs(oracle_c.gen_srs(name, 5, 40))
    with pytest.raises(kzgx.KzgxError) as e:
        ctx.prove_range(limbs(list(range(1, 30))), limbs([3, 7, 3]))
    assert e.value.status == -8  # KZGX_ERR_DIV_ZERO


@pytest.mark.parametrize("name,C", CURVES)
@pytest.mark.parametrize("npts", [2, 5])
def test_prove_range_long_polynomial_few_points(name, C, npts, oracle_c):
    """few points on a long polynomial: degree 2^16 opened at
    2 / 5 points goes through the division chain (one chip-wide synthetic
    division per point), not the quadratic Newton route; exact against the
    known-tau identity, and bounded in time"""
    import time
    import kzgx
    tau = K.default_tau(C)
    n = (1 << 16) + 1
    P = K.random_scalars(C, n, seed=0xD1 + npts)
    xs = [3 + 17 * k for k in range(npts)]
    ctx = kzgx.Context(name)
    try:
        ctx.gen_srs(tau, n)
        ctx.prove_range(limbs(P[:1000]), limbs(xs))  # warm
        t0 = time.perf_counter()
        out, inf = ctx.prove_range(limbs(P), limbs(xs))
        dt = time.perf_counter() - t0
        # [q(tau)]G1 with q = P div Z: q(tau) = (P(tau) - I(tau)) / Z(tau)
        r = C.r
        ptau = K.poly_eval(C, P, tau)
        Z = 1
        for x in xs:
            Z = Z * (tau - x) % r
        # I(tau) by Lagrange over the points
        I = 0
        for i, xi in enumerate(xs):
            num, den = 1, 1
            for j, xj in enumerate(xs):
                if j != i:
                    num = num * (tau - xj) % r
                    den = den * (xi - xj) % r
            I = (I + K.poly_eval(C, P, xi) * num * pow(den, -1, r)) % r
        qt = (ptau - I) * pow(Z, -1, r) % r
        assert pt(name, out, inf) == K.scalar_mul(C, (C.gx, C.gy), qt)
        assert dt < 2.0, dt
    finally:
        ctx.close()


@pytest.mark.parametrize("name,C", CURVES)
def test_small_batch_window_matches_main_window(name, C, ctx_factory):
    """Batches of <= kzgx_set_small_batch MSMs run on the window-10 table
    (msm.hip, the single-call latency path); larger ones, and every batch
    with it off, on the context's window-12 table.  Both must give [P(tau)]G1
    for every MSM, at the threshold (16) and one past it, with the digit
    edge cases (0, 1, r - 1) and a zero polynomial in the batch."""
    ctx = ctx_factory(name)
    tau = K.default_tau(C)
    n = 4097
    ctx.gen_srs(tau, 5000)
    polys = [K.random_scalars(C, n, seed=500 + b) for b in range(17)]
    polys[0][:3] = [0, 1, C.r - 1]
    polys[3] = [0] * n
    S = np.concatenate([limbs(p) for p in polys])
    exp = [K.commit_via_tau(C, tau, p) for p in polys]
    for small in (16, 0):
        ctx.set_small_batch(small)
        for batch in (1, 16, 17):
            out, inf = ctx.msm_batch(S, n, batch)
            for b in range(batch):
                got = pt(name, out[b], inf[b])
                assert got == exp[b], (small, batch, b)
    with pytest.raises(Exception):
        ctx.set_small_batch(1 << 20)
