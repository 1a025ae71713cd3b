"""kzgx_msm_g1_sharded: one commitment over several contexts holding
contiguous SRS slices (the one-process form of SURVEY 8e's sharded commit),
bit-exact with one MSM over the whole SRS and with [P(tau)]G1.  The box has
one GPU, so the shards are contexts on device 0; the fold and the slice
bookkeeping are what is under test (each context has its own stream)."""
import numpy as np
import pytest

import kzg_ref as K

pytestmark = pytest.mark.gpu

CURVES = [("BN254", K.BN254), ("BLS12381", K.BLS12381)]


def limbs(vals):
    return np.array([[(v >> (64 * i)) & 0xFFFFFFFFFFFFFFFF for i in range(4)] for v in vals], dtype=np.uint64)


def point(C, xy, inf):
    if inf:
        return None
    w = 4 if C is K.BN254 else 6
    return (sum(int(xy[i]) << (64 * i) for i in range(w)), sum(int(xy[w + i]) << (64 * i) for i in range(w)))


@pytest.mark.parametrize("name,C", CURVES)
def test_msm_g1_sharded(name, C):
    import kzgx
    tau = K.default_tau(C)
    sizes = [100, 37, 250]
    starts = [0, 100, 137]
    ctxs = [kzgx.Context(name) for _ in sizes]
    whole = kzgx.Context(name)
    try:
        for c, s0, m in zip(ctxs, starts, sizes):
            c.gen_srs(tau, m, start=s0)
        whole.gen_srs(tau, sum(sizes))
        for n in (387, 300, 137, 90, 1):
            P = K.random_scalars(C, n, seed=n)
            xy, inf = kzgx.msm_g1_sharded(ctxs, starts, limbs(P))
            got = point(C, xy, inf)
            assert got == point(C, *whole.msm(limbs(P)))
            assert got == K.commit_via_tau(C, tau, P)
        # a sum that cancels across shards: c at point 0, and at point 100 of tau = 1
        ones = [kzgx.Context(name) for _ in range(2)]
        try:
            ones[0].gen_srs(1, 100)
            ones[1].gen_srs(1, 50, start=100)
            sc = [0] * 150
            sc[0], sc[120] = 5, C.r - 5
            xy, inf = kzgx.msm_g1_sharded(ones, [0, 100], limbs(sc))
            assert inf
        finally:
            for c in ones:
                c.close()
        # slices must be contiguous from 0 and cover n
        with pytest.raises(kzgx.KzgxError) as e:
            kzgx.msm_g1_sharded(ctxs, [0, 99, 137], limbs([1] * 10))
        assert e.value.status == -1
        with pytest.raises(kzgx.KzgxError) as e:
            kzgx.msm_g1_sharded(ctxs, starts, limbs([1] * 388))
        assert e.value.status == -5
    finally:
        for c in ctxs + [whole]:
            c.close()
