"""GPU parity at the BASELINE.json configurations and at the exact kernel
instantiations the headline bench runs.

  * every throughput line of bench.py (configs[1] cfg2, configs[2] cfg3,
    configs[3] cfg4) at its exact launch shape (bench.WORKLOAD_SHAPES: curve,
    window, batch, points per thread, streams), through the bench's own step
    and checker, every output checked;
  * configs[2] on Pippenger too, plus the reference-semantics multi-proof
    create_proof(poly, 0, N) of benchmark/benchmark.cpp:73-82 for N in
    {128, 2048, 4096};
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
    """k_fixed_accum<C, 17> (the BN254 bench default, cfg2 / cfg3) and
    <C, 16> (the BLS12-381 default, cfg4, and BN254's fallback when c = 17
    does not fit) on both curves, against the naive per-term MSM."""
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


def _proof_scalar(C, tau, ptau, pz, z):
    return (ptau - pz) * pow((tau - z) % C.r, -1, C.r) % C.r


def _bench():
    import os
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    if root not in sys.path:
        sys.path.insert(0, root)
    import bench
    return bench


@pytest.mark.parametrize("workload", ["cfg2", "cfg3", "cfg4"])
def test_bench_shape(workload):
    """each throughput line of bench.py exactly as it runs: the curve, window,
    batch, points per thread and streams of bench.WORKLOAD_SHAPES, the
    bench's own inputs and step (bench.make_step: commits and proofs on two
    streams of one context), run twice (the second pass reuses the per-stream
    workspaces), then EVERY output checked with bench.check_step (commit =
    [P(tau)]G1, proof = [q(tau)]G1, y = P(z)).  One table at a time: the
    BN254 c = 17 table is 257.8 GB, the BLS12-381 c = 16 one 240.6 GB."""
    import torch
    import kzgx
    bench = _bench()
    shape = bench.WORKLOAD_SHAPES[workload]
    curve = shape["curve"]
    C = K.BN254 if curve == "BN254" else K.BLS12381
    tau = K.default_tau(C)
    n = bench.DEGREE + 1
    B = shape["batch"]
    ctx = kzgx.Context(curve)
    try:
        ctx.gen_srs(tau, bench.SRS_POINTS)
        ctx.set_fixed_base(shape["fixed_bits"], n)
        assert ctx.fixed_base_info()[:2] == (shape["fixed_bits"], n)
        ctx.set_fixed_points_per_thread(shape["points_per_thread"])
        coeffs, zs = bench.bench_inputs(C, workload, B, n)
        if workload != "cfg3":
            coeffs[3] = 0          # zero polynomial: commit and proof at infinity
            coeffs[5, 1:] = 0      # constant polynomial: proof at infinity
            coeffs[7, :] = coeffs[6, :]  # a repeated polynomial
        dev = torch.device("cuda", 0)
        bufs = bench.StepBuffers(torch, dev, coeffs, zs, ctx.w64)
        streams = [torch.cuda.Stream(device=dev) for _ in range(2)]
        step = bench.make_step(ctx, workload, n, bufs, streams)
        torch.cuda.synchronize(dev)
        for _ in range(2):
            step()
        torch.cuda.synchronize(dev)
        checked, ok, bad = bench.check_step(curve, C, tau, workload, coeffs, zs, bufs, ctx.w64)
        assert checked == (2 * B if workload == "cfg3" else 3 * B)
        assert ok == checked, bad
    finally:
        ctx.close()


@pytest.mark.parametrize("workload", ["cfg2", "cfg3"])
def test_bench_step_pippenger(workload):
    """the same bench steps on the default (table-less) Pippenger path, what
    create_commit / create_proof run without precompute(): every output"""
    import torch
    import kzgx
    bench = _bench()
    C = K.BN254
    tau = K.default_tau(C)
    n = bench.DEGREE + 1
    B = 1024 if workload == "cfg2" else 4096
    ctx = kzgx.Context("BN254")
    try:
        ctx.gen_srs(tau, bench.SRS_POINTS)
        coeffs, zs = bench.bench_inputs(C, workload, B, n)
        dev = torch.device("cuda", 0)
        bufs = bench.StepBuffers(torch, dev, coeffs, zs, ctx.w64)
        streams = [torch.cuda.Stream(device=dev) for _ in range(2)]
        step = bench.make_step(ctx, workload, n, bufs, streams)
        torch.cuda.synchronize(dev)
        step()
        torch.cuda.synchronize(dev)
        checked, ok, bad = bench.check_step("BN254", C, tau, workload, coeffs, zs, bufs, ctx.w64)
        assert ok == checked, bad
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
    from bench import random_fr
    # full-range scalars in [0, r) (c = 16's top window filled, as the
    # 262 145-point BIG cases of test_gpu_pippenger_buckets.py), plus 0,
    # r - 1 and the top bit alone
    S = random_fr(np.random.default_rng(0x4B5A47), (n,), C.r)
    S[17] = 0
    for k, v in ((18, C.r - 1), (19, 1 << 253)):
        S[k] = [(v >> (64 * i)) & 0xFFFFFFFFFFFFFFFF for i in range(4)]
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
