"""GPU parity of the fixed-base (precomputed multiples) MSM path.

kzgx_set_fixed_base precomputes M[w][i][j] = (j+1) 2^(c w) SRS[i]; MSMs over
the covered SRS prefix then run as plain table sums (msm_fixed.hip).  Every
result is checked bit-exactly against the CPU oracle: the naive per-term MSM
of the reference's polyeval_G1 (src/trusted_setup.cpp:149-174) at small
sizes, the MSM-independent identity commit == [P(tau)]G1 at full size.

These tests make their own contexts (the table is per context and large)."""
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


@pytest.fixture
def fresh_ctx():
    import kzgx
    made = []

    def get(curve):
        c = kzgx.Context(curve)
        made.append(c)
        return c

    yield get
    for c in made:
        c.close()


@pytest.mark.parametrize("name,C", CURVES)
@pytest.mark.parametrize("c", [4, 8, 10, 12])
def test_fixed_msm_matches_naive(name, C, c, fresh_ctx, oracle_c):
    ctx = fresh_ctx(name)
    n = 300
    srs = oracle_c.gen_srs(name, K.default_tau(C), n)
    ctx.load_srs(srs)
    ctx.set_fixed_base(c, n)
    cc, nt, nbytes = ctx.fixed_base_info()
    assert (cc, nt) == (c, n) and nbytes > 0
    sc = K.random_scalars(C, n, seed=31 + c)
    # digit edge cases: zero, one, r - 1, every digit = +-H boundary, top window carries
    H = 1 << (c - 1)
    sc[0], sc[1], sc[2] = 0, 1, C.r - 1
    sc[3] = sum(H << (c * w) for w in range(250 // c)) % C.r
    sc[4] = (1 << 253) - 1
    sc[5] = sum((H + 1) << (c * w) for w in range(250 // c)) % C.r
    S = limbs(sc)
    for n_use in (n, 1, 2, 65, 257):
        out, inf = ctx.msm(S[:n_use])
        assert pt(name, out, inf) == oracle_c.msm_naive(name, srs[:n_use], S[:n_use]), n_use


@pytest.mark.parametrize("name,C", CURVES)
def test_fixed_noncanonical_scalars(name, C, fresh_ctx, oracle_c):
    """Scalars >= r (outside the ABI contract) still give s P = (s mod r) P."""
    ctx = fresh_ctx(name)
    n = 40
    srs = oracle_c.gen_srs(name, K.default_tau(C), n)
    ctx.load_srs(srs)
    ctx.set_fixed_base(8, n)
    sc = [C.r, C.r + 5, (1 << 256) - 1, 2 * C.r + 1] + K.random_scalars(C, n - 4, seed=9)
    S = limbs(sc)
    out, inf = ctx.msm(S)
    assert pt(name, out, inf) == K.commit_via_tau(C, K.default_tau(C), [v % C.r for v in sc])


@pytest.mark.parametrize("name,C", CURVES)
@pytest.mark.parametrize("tau", [0, 1, 2, -1])
def test_fixed_degenerate_srs(name, C, tau, fresh_ctx, oracle_c):
    """tau = 0: infinite SRS points (skipped); tau = +-1: repeated points, so
    the accumulator meets P == Q (doubling) and P == -Q (cancellation)."""
    ctx = fresh_ctx(name)
    t = tau % C.r
    n = 200
    srs = oracle_c.gen_srs(name, t, n)
    ctx.load_srs(srs)
    ctx.set_fixed_base(8, n)
    sc = K.random_scalars(C, n, seed=5)
    sc[7] = sc[3]
    sc[9] = (C.r - sc[3]) % C.r
    out, inf = ctx.msm(limbs(sc))
    assert pt(name, out, inf) == K.commit_via_tau(C, t, sc)
    # a sum that cancels exactly: s P_0 + (r - s) P_0 style via repeated points
    if tau in (1, -1):
        z = [0] * n
        z[0], z[1] = 12345, (C.r - 12345) if tau == 1 else 12345
        out, inf = ctx.msm(limbs(z))
        assert inf and pt(name, out, inf) is None


@pytest.mark.parametrize("ppt", [1, 3, 8, 64])
def test_fixed_points_per_thread(ppt, fresh_ctx, oracle_c):
    name, C = CURVES[0]
    ctx = fresh_ctx(name)
    n = 700
    srs = oracle_c.gen_srs(name, K.default_tau(C), n)
    ctx.load_srs(srs)
    ctx.set_fixed_base(10, n)
    ctx.set_fixed_points_per_thread(ppt)
    sc = K.random_scalars(C, n, seed=ppt)
    S = limbs(sc)
    out, inf = ctx.msm(S)
    assert pt(name, out, inf) == oracle_c.msm_naive(name, srs, S)


def test_fixed_coverage_and_fallback(fresh_ctx, oracle_c):
    """MSMs longer than the table fall back to Pippenger; the table follows
    SRS changes; c = 0 turns it off."""
    name, C = CURVES[0]
    ctx = fresh_ctx(name)
    tau = K.default_tau(C)
    srs = oracle_c.gen_srs(name, tau, 500)
    ctx.load_srs(srs)
    ctx.set_fixed_base(8, 300)
    assert ctx.fixed_base_info()[1] == 300
    sc = K.random_scalars(C, 500, seed=3)
    S = limbs(sc)
    for n_use in (300, 301, 500):
        out, inf = ctx.msm(S[:n_use])
        assert pt(name, out, inf) == oracle_c.msm_naive(name, srs[:n_use], S[:n_use]), n_use
    # a new SRS rebuilds the table (clamped to the SRS size)
    ctx.gen_srs(tau + 1, 200)
    c, nt, _ = ctx.fixed_base_info()
    assert (c, nt) == (8, 200)
    out, inf = ctx.msm(S[:200])
    assert pt(name, out, inf) == K.commit_via_tau(C, tau + 1, sc[:200])
    ctx.set_fixed_base(0)
    assert ctx.fixed_base_info() == (0, 0, 0)
    out, inf = ctx.msm(S[:200])
    assert pt(name, out, inf) == K.commit_via_tau(C, tau + 1, sc[:200])
    with pytest.raises(Exception):
        ctx.set_fixed_base(5, 100)  # unsupported window
    with pytest.raises(Exception):
        ctx.set_fixed_base(8, 0)


@pytest.mark.parametrize("name,C,c", [("BN254", K.BN254, 13), ("BLS12381", K.BLS12381, 12)])
def test_fixed_degree4096_batch(name, C, c, fresh_ctx):
    """BASELINE configs[1]/[3] size: degree-4096 commits and single-opening
    proofs on the fixed-base path, against [P(tau)]G1 / [q(tau)]G1."""
    ctx = fresh_ctx(name)
    tau = K.default_tau(C)
    n, batch = 4097, 5
    ctx.gen_srs(tau, 5000)
    ctx.set_fixed_base(c, n)
    polys = [K.random_scalars(C, n, seed=177 + b) for b in range(batch)]
    polys[1] = [0] * n
    polys[2] = [5] + [0] * (n - 1)
    S = np.concatenate([limbs(p) for p in polys])
    out, inf = ctx.msm_batch(S, n, batch)
    for b in range(batch):
        assert pt(name, out[b], inf[b]) == K.commit_via_tau(C, tau, polys[b]), b
    zs = [0, 1, 7, C.r - 1]
    pout, pinf, _ = ctx.prove_single_batch(limbs(polys[0]), limbs(zs))
    for j, z in enumerate(zs):
        q = K.proof_quotient(C, polys[0], z, 1)
        assert pt(name, pout[j], pinf[j]) == K.commit_via_tau(C, tau, q), z


@pytest.mark.parametrize("name,C", CURVES)
@pytest.mark.parametrize("batch", [1, 3])
def test_fixed_large_single_msm(name, C, batch, fresh_ctx):
    """few large MSMs on the fixed-base path (configs[4] shape, scaled down):
    automatic points-per-thread fills the GPU, each wavefront folds its 64
    partials, one workgroup sums the rest; identity commit == [P(tau)]G1"""
    ctx = fresh_ctx(name)
    tau = K.default_tau(C)
    n = 70001
    ctx.gen_srs(tau, n)
    ctx.set_fixed_base(7, n)
    polys = [K.random_scalars(C, n, seed=900 + b) for b in range(batch)]
    polys[0][5] = 0
    S = np.concatenate([limbs(P) for P in polys])
    out, inf = ctx.msm_batch(S, n, batch)
    for b in range(batch):
        exp = K.commit_via_tau(C, tau, polys[b])
        assert pt(name, out[b], inf[b]) == exp


@pytest.mark.parametrize("name,C", CURVES)
@pytest.mark.parametrize("tau_kind,batch", [("default", 1), ("default", 2), ("default", 5), ("zero", 1)])
def test_fixed_flat_terms(name, C, tau_kind, batch, fresh_ctx):
    """few large MSMs with >= 32 digit terms per resident lane take the
    flattened-term kernel (k_fixed_accum_flat): threads start inside a point
    (carry-only recoding of its lower windows), every thread ends on a term
    boundary, and tau = 0 makes every SRS point but the first infinity (all of
    its terms skipped).  c = 4: 64 windows, 100 003 points -> 33 terms per
    thread; scalars with digit edge cases sit on both sides of thread
    boundaries.  The reduction: batches 1 and 2 take the three fold launches
    (k_fold_level, 768 / 384 first-level wavefronts per MSM), batch 5 the
    one-launch arrival-counter form (k_fixed_fold3: 144 per MSM, not a
    multiple of 64)."""
    ctx = fresh_ctx(name)
    tau = K.default_tau(C) if tau_kind == "default" else 0
    n, c = 100003, 4
    ctx.gen_srs(tau, n)
    ctx.set_fixed_base(c, n)
    assert ctx.fixed_base_info()[:2] == (c, n)
    H = 1 << (c - 1)
    polys = []
    for b in range(batch):
        P = K.random_scalars(C, n, seed=4400 + b)
        for j, i in enumerate((0, 1, 2, 3, 4, 5, 6, 7, 50000, 99999, n - 1)):
            P[i] = [2, 1, C.r - 1, sum(H << (c * w) for w in range(63)) % C.r, (1 << 253) - 1,
                    sum((H + 1) << (c * w) for w in range(62)) % C.r, 0, 0, C.r - 1, 1, 3][j]
        polys.append(P)
    S = np.concatenate([limbs(P) for P in polys])
    out, inf = ctx.msm_batch(S, n, batch)
    for b in range(batch):
        assert pt(name, out[b], inf[b]) == K.commit_via_tau(C, tau, polys[b]), b


@pytest.mark.parametrize("name,C", CURVES)
@pytest.mark.parametrize("c", [7, 8, 12, 13])
def test_fixed_table_layouts_agree(name, C, c, fresh_ctx, oracle_c):
    """Window-major M[w][i][j] and point-major M[i][w][j] tables
    (kzgx_set_fixed_base_layout; automatic = point-major for c <= 12) give
    the oracle's sums on every kernel that reads them: the latency kernel
    (one small MSM), the batched kernel (a batch of 20) and the flattened-term
    kernel (one MSM with >= 8 terms per resident lane)."""
    ctx = fresh_ctx(name)
    tau = K.default_tau(C)
    n_small, n_big = 300, 50001 if c <= 8 else 4097
    ctx.gen_srs(tau, n_big)
    sc = K.random_scalars(C, n_big, seed=1300 + c)
    sc[1], sc[2] = 0, C.r - 1
    S = limbs(sc)
    polys = [K.random_scalars(C, n_small, seed=1400 + b) for b in range(20)]
    SB = np.concatenate([limbs(P) for P in polys])
    exp_small = oracle_c.msm_naive(name, oracle_c.gen_srs(name, tau, n_small), S[:n_small])
    exp_big = K.commit_via_tau(C, tau, sc)
    for layout, want_pm in ((-1, c <= 12), (0, False), (1, True)):
        ctx.set_fixed_base_layout(layout)
        ctx.set_fixed_base(c, n_big)
        assert ctx.fixed_base_point_major() == want_pm, layout
        out, inf = ctx.msm(S[:n_small])
        assert pt(name, out, inf) == exp_small, (layout, "latency")
        out, inf = ctx.msm_batch(SB, n_small, 20)
        for b in (0, 7, 19):
            assert pt(name, out[b], inf[b]) == K.commit_via_tau(C, tau, polys[b]), (layout, "batch", b)
        out, inf = ctx.msm(S)
        assert pt(name, out, inf) == exp_big, (layout, "large")
    with pytest.raises(Exception):
        ctx.set_fixed_base_layout(2)


def test_fixed_base_budget_picks_the_widest_fitting_window():
    """kzgx_set_fixed_base_budget: the widest c whose table fits the budget
    (kzgx_fixed_base_bytes), none below c = 7 (Pippenger stays); exact MSMs
    either way"""
    import kzgx
    import kzg_ref as K
    C = K.BN254
    tau = K.default_tau(C)
    ctx = kzgx.Context("BN254")
    try:
        ctx.gen_srs(tau, 300)
        n = 257
        b12 = kzgx.fixed_base_bytes("BN254", 12, n)
        b13 = kzgx.fixed_base_bytes("BN254", 13, n)
        c = ctx.set_fixed_base_budget(b13 - 1, n)
        assert c == 12 and ctx.fixed_base_info()[:3] == (12, n, b12)
        P = K.random_scalars(C, n, seed=77)
        out, inf = ctx.msm(np.array([[(v >> (64 * i)) & (2**64 - 1) for i in range(4)] for v in P], dtype=np.uint64))
        exp = K.commit_via_tau(C, tau, P)
        got = None if inf else (sum(int(out[i]) << (64 * i) for i in range(4)), sum(int(out[4 + i]) << (64 * i) for i in range(4)))
        assert got == exp
        c = ctx.set_fixed_base_budget(kzgx.fixed_base_bytes("BN254", 7, n) - 1, n)
        assert c == 0 and ctx.fixed_base_info()[0] == 0
        out, inf = ctx.msm(np.array([[(v >> (64 * i)) & (2**64 - 1) for i in range(4)] for v in P], dtype=np.uint64))
        got = None if inf else (sum(int(out[i]) << (64 * i) for i in range(4)), sum(int(out[4 + i]) << (64 * i) for i in range(4)))
        assert got == exp
    finally:
        ctx.close()


def test_microbench_mad_u64_is_a_hardware_ceiling():
    """kzgx_microbench_mad_u64: lane-ops/s of v_mad_u64_u32 issue on the whole
    GPU; profiles/r01_micro_valu.txt measured 3.19e13 (256 CUs, 2.4 GHz peak
    clock: <= 256 x 4 SIMD x 16 lanes x 2.4e9 = 3.9e13)"""
    import kzgx
    import kzg_ref as K
    ctx = kzgx.Context("BN254")
    try:
        ctx.gen_srs(K.default_tau(K.BN254), 8)
        r = ctx.microbench_mad_u64()
        assert 1.0e13 < r < 4.0e13, r
    finally:
        ctx.close()


def test_clock_measurements_read_a_plausible_core_clock():
    """kzgx_microbench_mad_u64_clock and kzgx_clock_probe: the core clock from
    core-clock vs wall-clock counters (MI355X: up to 2.4 GHz, DVFS lowers it
    under load); the probe's wall time is the spin asked for"""
    import torch
    import kzgx
    import kzg_ref as K
    ctx = kzgx.Context("BN254")
    try:
        ctx.gen_srs(K.default_tau(K.BN254), 8)
        r, ghz = ctx.microbench_mad_u64_clock()
        assert 1.0e13 < r < 4.0e13, r
        assert 0.5 < ghz < 3.0, ghz
        buf = torch.zeros(3, dtype=torch.int64, device="cuda:0")
        ctx.clock_probe(buf.data_ptr(), 2000)
        torch.cuda.synchronize()
        core, wall, khz = (int(v) for v in buf.cpu().tolist())
        assert khz > 0 and abs(wall / khz - 2.0) < 0.1, (wall, khz)  # 2000 us of wall ticks
        assert 0.5 < core / wall * khz * 1e-6 < 3.0, (core, wall, khz)
        with pytest.raises(kzgx.KzgxError):
            ctx.clock_probe(buf.data_ptr(), 0)
    finally:
        ctx.close()


@pytest.mark.parametrize("name,C", CURVES)
@pytest.mark.parametrize("c", [7, 16, 17])
def test_odd_digit_edges(name, C, c, fresh_ctx):
    """Regular odd digits (fixed_accum.hpp): even scalars run as r - k with
    every digit negated, 0 becomes r (terms summing to O), and the extreme
    windows -- u's window bits all zero (digit 1 - 2^c) or all one (digit
    2^c - 1), the top digit at its largest -- index the first and last
    odd multiple.  Batched kernel (batch 20) and latency kernel (batch 1)."""
    ctx = fresh_ctx(name)
    tau = K.default_tau(C)
    n = 40
    ctx.gen_srs(tau, n)
    ctx.set_fixed_base(c, n)
    W = (C.r.bit_length() + c - 1) // c
    ones = sum(((1 << c) - 1) << (c * w) for w in range(W - 1))  # u windows all ones
    edge = [0, 1, 2, 3, C.r - 1, C.r - 2, C.r - 3, 2 * ones + 1, (2 * ones + 1) % C.r,
            (1 << (C.r.bit_length() - 1)) + 1, C.r - (2 * ones + 1) % C.r, 5, 1 << 200]
    polys = []
    for b in range(20):
        P = K.random_scalars(C, n, seed=5100 + b)
        for j, v in enumerate(edge):
            P[(j + b) % n] = v % C.r
        polys.append(P)
    S = np.concatenate([limbs(P) for P in polys])
    out, inf = ctx.msm_batch(S, n, len(polys))
    for b in range(len(polys)):
        assert pt(name, out[b], inf[b]) == K.commit_via_tau(C, tau, polys[b]), b
    ctx.set_fixed_points_per_thread(0)
    out1, inf1 = ctx.msm(limbs(polys[3]))
    assert pt(name, out1, inf1) == K.commit_via_tau(C, tau, polys[3])
