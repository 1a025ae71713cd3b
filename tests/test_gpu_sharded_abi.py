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


@pytest.mark.parametrize("name,C", CURVES)
@pytest.mark.parametrize("count", [1, 2, 3, 8, 64, 65, 130])
def test_g1_sum_packed_device(name, C, count):
    """kzgx_g1_sum_packed_device: the sharded commitment's one-wave fold over
    packed records (x || y || infinity word), against the oracle sum; with
    infinite records, a record equal to another (doubling) and one cancelling
    another (P + (-P))."""
    import torch
    import kzgx
    tau = K.default_tau(C)
    w = 4 if C is K.BN254 else 6
    ctx = kzgx.Context(name)
    try:
        ctx.gen_srs(tau, 4)
        rng = np.random.default_rng(count)
        ks = [int(rng.integers(1, 1 << 62)) for _ in range(count)]
        if count >= 3:
            ks[1] = ks[0]                  # equal records: the fold doubles
            ks[2] = C.r - ks[0] if count > 3 else ks[2]  # P and -P cancel
        infs = [count > 4 and j % 5 == 4 for j in range(count)]
        rec = np.zeros((count, 2 * w + 1), dtype=np.uint64)
        exp = None
        for j, (k, inf) in enumerate(zip(ks, infs)):
            if inf:
                rec[j, -1] = 1
                continue
            x, y = K.scalar_mul(C, (C.gx, C.gy), k)
            for i in range(w):
                rec[j, i] = (x >> (64 * i)) & 0xFFFFFFFFFFFFFFFF
                rec[j, w + i] = (y >> (64 * i)) & 0xFFFFFFFFFFFFFFFF
            exp = K.point_add(C, exp, (x, y))
        d_rec = torch.from_numpy(rec.view(np.int64)).cuda()
        d_out = torch.full((2 * w + 1,), -1, dtype=torch.int64, device="cuda")
        ctx.g1_sum_packed_device(d_rec.data_ptr(), count, d_out.data_ptr())
        torch.cuda.synchronize()
        out = d_out.cpu().numpy().view(np.uint64)
        got = None if out[-1] else point(C, out[: 2 * w], False)
        assert int(out[-1]) in (0, 1)
        assert got == exp
    finally:
        ctx.close()


def test_init_device_twice():
    """kzgx_init_device (kzg::init's device bring-up) is idempotent per process."""
    import kzgx
    for curve in ("BN254", "BLS12381", "BN254"):
        assert kzgx.lib().kzgx_init_device(kzgx.CURVES[curve], 0) == 0


@pytest.mark.parametrize("name,C", CURVES)
def test_partial_records_fold(name, C):
    """The sharded commitment's round-6 exchange: every shard's MSM left
    projective (kzgx_msm_g1_partial_device: one XYZZ record, no inversion),
    the records folded with one inversion (kzgx_g1_sum_partials_device) --
    against [P(tau)]G1.  Shards on every MSM path: the wide-window Pippenger
    (>= 2^16 points), the main fixed table's flattened kernel, the default
    table's one-launch kernel (lifted affine result), and an empty shard."""
    import torch
    import kzgx
    tau = K.default_tau(C)
    w = 4 if C is K.BN254 else 6
    sizes = [70001, 3000, 60000, 0]
    starts = [0, 70001, 73001, 133001]
    n = sum(sizes)
    P = K.random_scalars(C, n, seed=9100)
    P[5], P[70001 + 7] = 0, C.r - 1
    ctxs = []
    try:
        for s0, m in zip(starts, sizes):
            c = kzgx.Context(name)
            ctxs.append(c)
            if m:
                c.gen_srs(tau, m, start=s0)
        ctxs[2].set_default_table(0)
        ctxs[2].set_fixed_base(8, 60000)  # the main table (15.7 GB): flattened few-MSM kernel
        rw = ctxs[0].partial_record_words
        assert rw == (18 if C is K.BN254 else 28)
        recs = torch.full((len(sizes), rw), -1, dtype=torch.int64, device="cuda")
        for k, (c, s0, m) in enumerate(zip(ctxs, starts, sizes)):
            d_s = torch.from_numpy(limbs(P[s0:s0 + m]).view(np.int64).reshape(-1) if m else np.zeros(4, np.int64)).cuda()
            if m:
                c.msm_partial_device(d_s.data_ptr(), m, recs[k].data_ptr())
            else:
                ctxs[0].msm_partial_device(d_s.data_ptr(), 0, recs[k].data_ptr())
            torch.cuda.synchronize()
        d_out = torch.full((2 * w + 1,), -1, dtype=torch.int64, device="cuda")
        ctxs[0].g1_sum_partials_device(recs.data_ptr(), len(sizes), d_out.data_ptr())
        torch.cuda.synchronize()
        out = d_out.cpu().numpy().view(np.uint64)
        assert int(out[-1]) == 0
        assert point(C, out[: 2 * w], False) == K.commit_via_tau(C, tau, P)
        # each record alone is its shard's commitment (the fold of one record
        # is its affine conversion); a record and its negation cancel
        for k, (s0, m) in enumerate(zip(starts, sizes)):
            ctxs[0].g1_sum_partials_device(recs[k].data_ptr(), 1, d_out.data_ptr())
            torch.cuda.synchronize()
            out = d_out.cpu().numpy().view(np.uint64)
            exp = K.commit_via_tau(C, tau, [0] * s0 + P[s0:s0 + m]) if m else None
            assert (None if out[-1] else point(C, out[: 2 * w], False)) == exp, k
        neg = [(C.r - v) % C.r for v in P[70001:73001]]
        d_s = torch.from_numpy(limbs(neg).view(np.int64).reshape(-1)).cuda()
        ctxs[1].msm_partial_device(d_s.data_ptr(), 3000, recs[2].data_ptr())
        torch.cuda.synchronize()  # ctxs[1]'s stream wrote it; the fold runs on ctxs[0]'s
        ctxs[0].g1_sum_partials_device(recs[1:].data_ptr(), 2, d_out.data_ptr())  # records 1 and -1
        torch.cuda.synchronize()
        assert int(d_out.cpu().numpy()[-1]) == 1
    finally:
        for c in ctxs:
            c.close()
