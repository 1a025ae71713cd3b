"""Multi-process CPU test of the sharded-commit path (configs[4]) with the
gloo backend, world_size 2 and 3: the same driver as bench.py's GPU path,
with the CPU oracle standing in for the per-rank GPU MSM and fold."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import kzg_ref as K
import kzgx_dist


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n, results):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    C = K.BN254
    tau = 0xC0FFEE
    coeffs = K.random_scalars(C, n, 7)

    def partial(start, count):
        # oracle naive MSM over [tau^(start+i)]G1 (the rank's own SRS slice)
        acc = None
        for i in range(count):
            base = K.scalar_mul(C, (C.gx, C.gy), pow(tau, start + i, C.r))
            acc = K.point_add(C, acc, K.scalar_mul(C, base, coeffs[start + i]))
        xy = np.zeros(8, dtype=np.uint64)
        if acc is not None:
            for j in range(4):
                xy[j] = (acc[0] >> (64 * j)) & 0xFFFFFFFFFFFFFFFF
                xy[4 + j] = (acc[1] >> (64 * j)) & 0xFFFFFFFFFFFFFFFF
        return xy, acc is None

    def fold(pts, infs):
        acc = None
        for row, inf in zip(pts, infs):
            if not inf:
                acc = K.point_add(C, acc, (sum(int(row[j]) << (64 * j) for j in range(4)),
                                           sum(int(row[4 + j]) << (64 * j) for j in range(4))))
        return acc, acc is None

    got, _ = kzgx_dist.sharded_commit(n, world, rank, 4, partial, kzgx_dist.torch_all_gather(dist), fold)
    results[rank] = got

    # the device-resident driver (bench.py's configs[4] step) on CPU tensors:
    # packed records, all-gathered into one (world, 2 W64 + 1) tensor, folded
    # as records (the format kzgx_g1_sum_packed_device reads)
    import torch

    def partial_t(start, count):
        xy, inf = partial(start, count)
        return torch.from_numpy(kzgx_dist.pack_point(xy, inf, 4))

    def fold_t(recs):
        assert recs.dtype == torch.int64 and recs.shape == (world, 9)
        pts, infs = kzgx_dist.unpack_points(recs.numpy(), 4)
        acc, inf = fold(pts, infs)
        xy = np.zeros(8, dtype=np.uint64)
        if acc is not None:
            for j in range(4):
                xy[j] = (acc[0] >> (64 * j)) & 0xFFFFFFFFFFFFFFFF
                xy[4 + j] = (acc[1] >> (64 * j)) & 0xFFFFFFFFFFFFFFFF
        return torch.from_numpy(kzgx_dist.pack_point(xy, inf, 4))

    packed = kzgx_dist.sharded_commit_tensor(n, world, rank, 4, partial_t, fold_t, dist, torch)
    xy, inf = kzgx_dist.unpack_points(packed.numpy(), 4)
    results[("t", rank)] = None if inf[0] else (sum(int(xy[0, j]) << (64 * j) for j in range(4)),
                                                 sum(int(xy[0, 4 + j]) << (64 * j) for j in range(4)))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_commit_gloo(world):
    n = 11
    mgr = mp.Manager()
    results = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), n, results), nprocs=world, join=True)
    C = K.BN254
    exp = K.commit_via_tau(C, 0xC0FFEE, K.random_scalars(C, n, 7))
    assert all(results[r] == exp for r in range(world))
    assert all(results[("t", r)] == exp for r in range(world))


def test_shard_range_partitions():
    for n in (0, 1, 7, 1 << 20 | 1):
        for world in (1, 2, 3, 8):
            spans = [kzgx_dist.shard_range(n, world, r) for r in range(world)]
            assert sum(c for _, c in spans) == n
            pos = 0
            for s, c in spans:
                assert s == pos
                pos += c
    with pytest.raises(ValueError):
        kzgx_dist.shard_range(5, 2, 2)
