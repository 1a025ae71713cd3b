"""GPU parity of the table-less Pippenger MSM (csrc/msm.hip) on bucket
distributions that exercise every merge path of the round-2 design:

* one giant bucket (all scalars equal): every segment is a spanning head, so
  the bucket's partials chain across many workgroups (k_msm_merge's
  segmented scan + k_msm_wg_fixup's multi-workgroup walk);
* cancelling entries in one bucket (s and r - s on equal points, tau = 1):
  partials that sum to infinity inside the merge and the fold;
* a single MSM (the segment length shrinks to 8: long head chains from the
  top window's few small digits take the segmented-scan merge);
* every window width with segment lengths that force chains of each kind.

The reference is the MSM-independent identity commit == [P(tau)]G1 (and the
naive oracle MSM for small n), so every comparison is bit-exact."""
import numpy as np
import pytest

import kzg_ref as K

pytestmark = pytest.mark.gpu

CURVES = [("BN254", K.BN254), ("BLS12381", K.BLS12381)]


def limbs(vals):
    import corc
    return corc.ints_to_limbs(vals, 4)


def as_point(curve_name, row, inf):
    import corc
    return None if inf else corc.array_to_points(curve_name, row[None, :])[0]


@pytest.mark.parametrize("name,C", CURVES)
@pytest.mark.parametrize("n,seg", [(4097, 128), (20000, 8), (3000, 1)])
def test_one_giant_bucket(name, C, n, seg):
    """all scalars equal: one digit per window, so each window's entries sit
    in one bucket that spans many segments and workgroups"""
    import kzgx
    ctx = kzgx.Context(name)
    try:
        ctx.set_segment(seg)
        tau = K.default_tau(C)
        ctx.gen_srs(tau, n + 1)
        s = K.random_scalars(C, 1, seed=n)[0]
        sc = [s] * n
        out, inf = ctx.msm(limbs(sc))
        assert as_point(name, out, inf) == K.commit_via_tau(C, tau, sc)
        # two batched MSMs of the same shape: per-MSM buckets stay separate
        sc2 = [(s * 3 + 1) % C.r] * n
        S = np.concatenate([limbs(sc), limbs(sc2)])
        outb, infb = ctx.msm_batch(S, n, 2)
        assert as_point(name, outb[0], infb[0]) == K.commit_via_tau(C, tau, sc)
        assert as_point(name, outb[1], infb[1]) == K.commit_via_tau(C, tau, sc2)
    finally:
        ctx.close()


@pytest.mark.parametrize("name,C", CURVES)
@pytest.mark.parametrize("seg", [1, 8, 128])
def test_cancelling_buckets(name, C, seg, oracle_c):
    """tau = 1: every SRS point is G, so scalars s and r - s land their digits
    in the same buckets with opposite signs and the partials cancel"""
    import kzgx
    ctx = kzgx.Context(name)
    try:
        ctx.set_segment(seg)
        n = 600
        srs = oracle_c.gen_srs(name, 1, n)
        ctx.load_srs(srs)
        base = K.random_scalars(C, n // 2, seed=11)
        sc = []
        for v in base:
            sc += [v, (C.r - v) % C.r]
        out, inf = ctx.msm(limbs(sc))
        assert inf and not out.any()
        # one extra term survives: the sum is exactly that term
        sc[5] = (sc[5] + 7) % C.r
        out, inf = ctx.msm(limbs(sc))
        assert as_point(name, out, inf) == K.scalar_mul(C, (C.gx, C.gy), 7)
    finally:
        ctx.close()


@pytest.mark.parametrize("name,C", CURVES)
@pytest.mark.parametrize("c", [10, 11, 12, 13])
def test_single_msm_small_segments(name, C, c):
    """one degree-4096 commitment: the segment length shrinks to 8 for a
    single MSM, the top window's small digits make buckets of ~n/4 entries
    whose head chains take the segmented-scan merge"""
    import kzgx
    ctx = kzgx.Context(name)
    try:
        ctx.set_window_bits(c)
        tau = K.default_tau(C)
        n = 4097
        ctx.gen_srs(tau, n + 1)
        sc = K.random_scalars(C, n, seed=c)
        out, inf = ctx.msm(limbs(sc))
        assert as_point(name, out, inf) == K.commit_via_tau(C, tau, sc)
    finally:
        ctx.close()


@pytest.mark.parametrize("name,C", CURVES)
def test_sparse_and_small_scalars(name, C):
    """mostly-zero scalars and scalars < 2^c: few, short buckets; empty
    segments and empty workgroups in the accumulation grid"""
    import kzgx
    ctx = kzgx.Context(name)
    try:
        tau = K.default_tau(C)
        n = 5000
        ctx.gen_srs(tau, n + 1)
        rng = np.random.default_rng(3)
        sc = [0] * n
        for i in rng.choice(n, 37, replace=False):
            sc[int(i)] = int(rng.integers(1, 1 << 11))
        sc[-1] = C.r - 1
        out, inf = ctx.msm(limbs(sc))
        assert as_point(name, out, inf) == K.commit_via_tau(C, tau, sc)
    finally:
        ctx.close()


# ---- the wide-window single-MSM path (msm.hip msm_big, round 5) ----------------
# An SRS of >= 2^16 points gets a wide-window table at setup: c = 14 below
# 2^18 points, 16 from there; single MSMs of >= 2^16 points
# take it (global counting sort, LDS histograms of 2^(c-1) buckets, the
# batched accumulation / merges, latency.hip's bucket reduction).
BIG = [(65536 + 7, 14), (131072 + 3, 14), (262144 + 1, 16)]


@pytest.mark.parametrize("name,C", CURVES)
@pytest.mark.parametrize("srs_n,cbits", BIG)
def test_big_window_random_and_edges(name, C, srs_n, cbits):
    """random scalars with zeros, r - 1, 1 and 2^k values mixed in, at the
    SRS size and one below; and the shortest MSM that takes the path"""
    import kzgx
    ctx = kzgx.Context(name)
    try:
        tau = K.default_tau(C)
        ctx.gen_srs(tau, srs_n)
        for n in (srs_n, srs_n - 1, 65536):
            sc = K.random_scalars(C, n, seed=n + cbits)
            for j in range(0, n, 997):
                sc[j] = 0
            sc[1], sc[2], sc[3], sc[n - 1] = C.r - 1, 1, 1 << 200, (1 << 255) % C.r
            out, inf = ctx.msm(limbs(sc))
            assert as_point(name, out, inf) == K.commit_via_tau(C, tau, sc), n
    finally:
        ctx.close()


@pytest.mark.parametrize("name,C", CURVES)
@pytest.mark.parametrize("srs_n,cbits", BIG)
def test_big_window_one_giant_bucket(name, C, srs_n, cbits):
    """all scalars equal: every window's entries in one bucket spanning
    thousands of segments and many merge workgroups"""
    import kzgx
    ctx = kzgx.Context(name)
    try:
        tau = K.default_tau(C)
        ctx.gen_srs(tau, srs_n)
        s = K.random_scalars(C, 1, seed=cbits)[0]
        sc = [s] * srs_n
        out, inf = ctx.msm(limbs(sc))
        assert as_point(name, out, inf) == K.commit_via_tau(C, tau, sc)
        # the top bucket (digit 2^(c-1) in every window below the top)
        top = sum((1 << (cbits - 1)) << (cbits * w) for w in range(256 // cbits)) % C.r
        sc = [top] * 65536
        out, inf = ctx.msm(limbs(sc))
        assert as_point(name, out, inf) == K.commit_via_tau(C, tau, sc)
    finally:
        ctx.close()


@pytest.mark.parametrize("name,C", CURVES)
def test_big_window_degenerate_setups(name, C):
    """tau = 1 (every point G: s and r - s cancel bucket by bucket; one extra
    term survives) and tau = 0 (every point but the first is infinite)"""
    import kzgx
    n = 65536 + 2
    ctx = kzgx.Context(name)
    try:
        ctx.gen_srs(1, n)
        base = K.random_scalars(C, n // 2, seed=5)
        sc = []
        for v in base:
            sc += [v, (C.r - v) % C.r]
        out, inf = ctx.msm(limbs(sc))
        assert inf and not out.any()
        sc[77] = (sc[77] + 5) % C.r
        out, inf = ctx.msm(limbs(sc))
        assert as_point(name, out, inf) == K.commit_via_tau(C, 1, sc)
    finally:
        ctx.close()
    ctx = kzgx.Context(name)
    try:
        ctx.gen_srs(0, n)
        sc = K.random_scalars(C, n, seed=6)
        out, inf = ctx.msm(limbs(sc))
        assert as_point(name, out, inf) == K.commit_via_tau(C, 0, sc)
    finally:
        ctx.close()
