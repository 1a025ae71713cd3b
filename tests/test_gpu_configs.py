"""GPU parity at the BASELINE.json configurations and at the exact kernel
instantiations the headline bench runs.

  * configs[1] / bench.py default: degree-4096 BN254 commits + single-opening
    proofs, batch 1024, fixed-base table c = 16 (k_fixed_accum<BN254G1, 16>),
    16 points per thread, commits and proofs on two streams sharing one
    context;
  * configs[2]: one degree-4096 polynomial opened at x = 0..4095 as ONE
    4096-wide batch, on the c = 16 table and on Pippenger; plus the
    reference-semantics multi-proof create_proof(poly, 0, N) of
    benchmark/benchmark.cpp:73-82 for N in {128, 2048, 4096};
  * configs[4]: one 2^20 + 1 coefficient commitment (chunked Pippenger), and
    the same commitment sharded over 2 and 8 contexts (kzgx_msm_g1_sharded);
  * the c = 16 / 17 window instantiations on both curves against the naive
    per-term MSM of the reference's polyeval_G1 (src/trusted_setup.cpp:149-174)
    on the digit edge cases.

Checks are bit-exact: [P(tau)]G1 for commits, [q(tau)]G1 with
q(tau) = (P(tau) - P(z)) / (tau - z) for single openings, the C oracle's
quotient (orc_quotient: evaluate + interpolate + long division, the
reference's create_proof algorithm) for multi-point openings."""
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


def g_mul(curve, C, s):
    import corc
    return corc.scalar_mul(curve, (C.gx, C.gy), s % C.r)


def digit_edge_scalars(C, c, n, seed):
    sc = K.random_scalars(C, n, seed=seed)
    H = 1 << (c - 1)
    sc[0], sc[1], sc[2] = 0, 1, C.r - 1
    sc[3] = sum(H << (c * w) for w in range(250 // c)) % C.r          # every digit = +H
    sc[4] = (1 << 253) - 1                                             # carries through every window
    sc[5] = sum((H + 1) << (c * w) for w in range(250 // c)) % C.r    # every digit = -H+1 with carry
    sc[6] = C.r - 2
    sc[7] = sc[3]                                                      # a repeated scalar
    return sc


@pytest.mark.parametrize("name,C", CURVES)
@pytest.mark.parametrize("c", [16, 17])
def test_headline_window_bits(name, C, c):
    """k_fixed_accum<C, 16> (the bench default) and <C, 17> (its fallback
    neighbour) on both curves, against the naive per-term MSM."""
    import corc
    import kzgx
    ctx = kzgx.Context(name)
    try:
        n = 64
        srs = corc.gen_srs(name, K.default_tau(C), n)
        ctx.load_srs(srs)
        ctx.set_fixed_base(c, n)
        assert ctx.fixed_base_info()[:2] == (c, n)
        sc = digit_edge_scalars(C, c, n, seed=1600 + c)
        S = limbs(sc)
        for n_use in (n, 1, 7, 33):
            out, inf = ctx.msm(S[:n_use])
            assert pt(name, out, inf) == corc.msm_naive(name, srs[:n_use], S[:n_use]), n_use
        # a batch through the bench's points-per-thread setting
        ctx.set_fixed_points_per_thread(16)
        B = 5
        scb = [digit_edge_scalars(C, c, n, seed=2000 + b) for b in range(B)]
        out, inf = ctx.msm_batch(np.concatenate([limbs(s) for s in scb]), n, B)
        for b in range(B):
            assert pt(name, out[b], inf[b]) == corc.msm_naive(name, srs, limbs(scb[b])), b
    finally:
        ctx.close()


@pytest.fixture(scope="module")
def bn254_c16():
    """the bench's context: BN254, SRS 5000 from the fixed tau, c = 16 table
    over the 4097-point prefix (171.8 GB), 16 points per thread"""
    import kzgx
    C = K.BN254
    ctx = kzgx.Context("BN254")
    ctx.gen_srs(K.default_tau(C), 5000)
    ctx.set_fixed_base(16, 4097)
    ctx.set_fixed_points_per_thread(16)
    assert ctx.fixed_base_info()[:2] == (16, 4097)
    yield ctx
    ctx.close()


def _proof_scalar(C, tau, ptau, pz, z):
    return (ptau - pz) * pow((tau - z) % C.r, -1, C.r) % C.r


def test_bench_shape_two_streams(bn254_c16):
    """bench.py's default step, exactly: 1024 commits (n = 4097) on one
    stream and 1024 single-opening proofs (n = 4097, z = b) on another, both
    on one context's c = 16 table; every one of the 2048 results checked."""
    import corc
    import torch
    name, C = "BN254", K.BN254
    ctx = bn254_c16
    tau = K.default_tau(C)
    n, B = 4097, 1024
    rng = np.random.default_rng(0x4B5A47)
    coeffs = rng.integers(0, 2**63, size=(B, n, 4), dtype=np.uint64)
    coeffs[..., 3] &= np.uint64((1 << 59) - 1)  # < 2^251 < r: canonical
    coeffs[3] = 0                                # zero polynomial -> infinity
    coeffs[5, 1:] = 0                            # constant polynomial
    zs = np.zeros((B, 4), dtype=np.uint64)
    zs[:, 0] = np.arange(B, dtype=np.uint64)
    dev = torch.device("cuda", 0)
    d_c = torch.from_numpy(coeffs.view(np.int64)).to(dev)
    d_z = torch.from_numpy(zs.view(np.int64)).to(dev)
    d_co = torch.zeros((B, 8), dtype=torch.int64, device=dev)
    d_ci = torch.zeros((B,), dtype=torch.int32, device=dev)
    d_po = torch.zeros((B, 8), dtype=torch.int64, device=dev)
    d_pi = torch.zeros((B,), dtype=torch.int32, device=dev)
    s1, s2 = torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)
    torch.cuda.synchronize(dev)
    for _ in range(2):  # twice: the second pass reuses the per-stream workspaces
        ctx.prove_single_batch_device(d_c.data_ptr(), n, n, d_z.data_ptr(), B, d_po.data_ptr(), d_pi.data_ptr(),
                                      None, s2.cuda_stream)
        ctx.msm_batch_device(d_c.data_ptr(), n, B, n, d_co.data_ptr(), d_ci.data_ptr(), s1.cuda_stream)
    torch.cuda.synchronize(dev)
    co, ci = d_co.cpu().numpy().view(np.uint64), d_ci.cpu().numpy()
    po, pi = d_po.cpu().numpy().view(np.uint64), d_pi.cpu().numpy()
    for b in range(B):
        ptau = corc.poly_eval(name, coeffs[b], tau)
        assert pt(name, co[b], ci[b]) == g_mul(name, C, ptau), ("commit", b)
        pz = corc.poly_eval(name, coeffs[b], b)
        assert pt(name, po[b], pi[b]) == g_mul(name, C, _proof_scalar(C, tau, ptau, pz, b)), ("proof", b)


def _cfg3_check(name, C, ctx, tau):
    import corc
    import torch
    n = 4097
    coeffs = limbs(K.random_scalars(C, n, seed=0xCF63))
    B = 4096
    zs = np.zeros((B, 4), dtype=np.uint64)
    zs[:, 0] = np.arange(B, dtype=np.uint64)
    dev = torch.device("cuda", 0)
    d_c = torch.from_numpy(coeffs.view(np.int64)).to(dev)
    d_z = torch.from_numpy(zs.view(np.int64)).to(dev)
    d_po = torch.zeros((B, 8), dtype=torch.int64, device=dev)
    d_pi = torch.zeros((B,), dtype=torch.int32, device=dev)
    d_y = torch.zeros((B, 4), dtype=torch.int64, device=dev)
    torch.cuda.synchronize(dev)
    ctx.prove_single_batch_device(d_c.data_ptr(), n, 0, d_z.data_ptr(), B, d_po.data_ptr(), d_pi.data_ptr(),
                                  d_y.data_ptr(), ctx.stream)
    ctx.sync()
    po, pi = d_po.cpu().numpy().view(np.uint64), d_pi.cpu().numpy()
    ys = corc.limbs_to_ints(d_y.cpu().numpy().view(np.uint64))
    ptau = corc.poly_eval(name, coeffs, tau)
    for z in range(B):
        pz = corc.poly_eval(name, coeffs, z)
        assert ys[z] == pz, ("y", z)
        assert pt(name, po[z], pi[z]) == g_mul(name, C, _proof_scalar(C, tau, ptau, pz, z)), ("proof", z)


def test_cfg3_4096_openings_table(bn254_c16):
    """configs[2]: 4096 single-point openings of one degree-4096 polynomial
    as one batch on the c = 16 fixed-base table"""
    _cfg3_check("BN254", K.BN254, bn254_c16, K.default_tau(K.BN254))


def test_cfg3_4096_openings_pippenger():
    """configs[2] on the default (table-less) Pippenger path"""
    import kzgx
    C = K.BN254
    ctx = kzgx.Context("BN254")
    try:
        ctx.gen_srs(K.default_tau(C), 5000)
        _cfg3_check("BN254", C, ctx, K.default_tau(C))
    finally:
        ctx.close()


@pytest.mark.parametrize("name,C", CURVES)
@pytest.mark.parametrize("N", [128, 2048, 4096])
def test_reference_multi_proof(name, C, N):
    """create_proof(poly, 0, N) on a 4096-coefficient polynomial
    (benchmark/benchmark.cpp:73-82: a 4096-char string -> degree <= 4095):
    one proof opening x = 0..N-1.  N = 4096 >= 4096 coefficients gives
    q = 0 and the proof at infinity."""
    import corc
    import kzgx
    ctx = kzgx.Context(name)
    try:
        tau = K.default_tau(C)
        ctx.gen_srs(tau, 5000)
        P = K.random_scalars(C, 4096, seed=0xB0 + N)
        xs = np.zeros((N, 4), dtype=np.uint64)
        xs[:, 0] = np.arange(N, dtype=np.uint64)
        out, inf = ctx.prove_range(limbs(P), xs)
        q = corc.quotient(name, P, 0, N)
        if N >= 4096:
            assert q == [] and inf
        exp = K.commit_via_tau(C, tau, q)
        assert pt(name, out, inf) == exp
    finally:
        ctx.close()


@pytest.fixture(scope="module")
def cfg5_poly():
    C = K.BN254
    n = (1 << 20) + 1
    rng = np.random.default_rng(0x4B5A47)
    S = rng.integers(0, 2**63, size=(n, 4), dtype=np.uint64)
    S[:, 3] &= np.uint64((1 << 59) - 1)
    S[17] = 0
    import corc
    ptau = corc.poly_eval("BN254", S, K.default_tau(C))
    return S, g_mul("BN254", C, ptau)


def test_cfg5_commit_single(cfg5_poly):
    """configs[4] on one context: a 2^20 + 1 term MSM (chunked Pippenger)"""
    import kzgx
    S, exp = cfg5_poly
    n = S.shape[0]
    ctx = kzgx.Context("BN254")
    try:
        ctx.gen_srs(K.default_tau(K.BN254), n)
        out, inf = ctx.msm(S)
        assert pt("BN254", out, inf) == exp
    finally:
        ctx.close()


@pytest.mark.parametrize("shards", [2, 8])
def test_cfg5_commit_sharded(cfg5_poly, shards):
    """configs[4] sharded: contiguous SRS slices over `shards` contexts (one
    GPU on the box, so all on device 0), partial MSMs on their own streams,
    device-side fold on the first context"""
    import kzgx
    S, exp = cfg5_poly
    n = S.shape[0]
    tau = K.default_tau(K.BN254)
    starts = [n * k // shards for k in range(shards)]
    sizes = [(n * (k + 1) // shards) - starts[k] for k in range(shards)]
    ctxs = [kzgx.Context("BN254") for _ in range(shards)]
    try:
        for c, s0, m in zip(ctxs, starts, sizes):
            c.gen_srs(tau, m, start=s0)
        out, inf = kzgx.msm_g1_sharded(ctxs, starts, S)
        assert pt("BN254", out, inf) == exp
        # the same context twice is rejected (its staging would be shared)
        with pytest.raises(kzgx.KzgxError) as e:
            kzgx.msm_g1_sharded([ctxs[0], ctxs[0]], [0, sizes[0]], S[: 2 * sizes[0]])
        assert e.value.status == -1
    finally:
        for c in ctxs:
            c.close()


def test_benchmark_common_degree_2_23():
    """benchmark.cpp --benchmark-common (:123-136): a 10,429,000-point setup
    and its largest commit, degree 2^23 (8,388,609 coefficients), through the
    table-less chunked Pippenger (2049 chunks), against [P(tau)]G1"""
    import corc
    import kzgx
    C = K.BN254
    tau = K.default_tau(C)
    n = (1 << 23) + 1
    rng = np.random.default_rng(0xC0)
    S = rng.integers(0, 2**63, size=(n, 4), dtype=np.uint64)
    S[:, 3] &= np.uint64((1 << 59) - 1)
    S[n // 3] = 0
    exp = g_mul("BN254", C, corc.poly_eval("BN254", S, tau))
    ctx = kzgx.Context("BN254")
    try:
        ctx.gen_srs(tau, 10429000)
        out, inf = ctx.msm(S)
        assert pt("BN254", out, inf) == exp
    finally:
        ctx.close()


def test_more_streams_than_workspaces():
    """a context keeps workspaces for 8 streams; a 9th..12th distinct stream
    rebinds the least recently bound one after a device synchronisation
    (kzg_gpu.h) -- results stay exact, calls never fail"""
    import torch
    import kzgx
    C = K.BN254
    tau = K.default_tau(C)
    ctx = kzgx.Context("BN254")
    try:
        n, B = 257, 3
        ctx.gen_srs(tau, n + 1)
        dev = torch.device("cuda", 0)
        streams = [torch.cuda.Stream(device=dev) for _ in range(12)]
        polys = [K.random_scalars(C, n, seed=900 + s) for s in range(len(streams))]
        d_c = [torch.from_numpy(np.concatenate([limbs(p)] * B).view(np.int64)).to(dev) for p in polys]
        outs = [torch.zeros((B, 8), dtype=torch.int64, device=dev) for _ in streams]
        infs = [torch.zeros((B,), dtype=torch.int32, device=dev) for _ in streams]
        torch.cuda.synchronize(dev)
        for rep in range(2):
            for s, st in enumerate(streams):
                ctx.msm_batch_device(d_c[s].data_ptr(), n, B, n, outs[s].data_ptr(), infs[s].data_ptr(),
                                     st.cuda_stream)
        torch.cuda.synchronize(dev)
        for s in range(len(streams)):
            exp = K.commit_via_tau(C, tau, polys[s])
            o = outs[s].cpu().numpy().view(np.uint64)
            for b in range(B):
                assert pt("BN254", o[b], bool(infs[s][b].item())) == exp
    finally:
        ctx.close()
