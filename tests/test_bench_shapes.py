"""bench.py's launch shapes are pinned here: tests/test_gpu_configs.py
runs exactly these shapes (bench.WORKLOAD_SHAPES through bench.make_step), so
a changed bench default must change this file too (the tests
and the bench defaults had drifted apart)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PINNED = {
    "cfg2": {"curve": "BN254", "batch": 2048, "fixed_bits": 17, "points_per_thread": 22, "streams": 2},
    "cfg3": {"curve": "BN254", "batch": 4096, "fixed_bits": 17, "points_per_thread": 16, "streams": 1},
    "cfg4": {"curve": "BLS12381", "batch": 2048, "fixed_bits": 16, "points_per_thread": 65, "streams": 2},
}


def test_bench_shapes_pinned():
    sys.path.insert(0, ROOT)
    import bench
    assert bench.WORKLOAD_SHAPES == PINNED
    assert bench.DEGREE == 4096 and bench.SRS_POINTS == 5000


def test_bench_inputs_shapes():
    sys.path.insert(0, ROOT)
    import bench
    import kzg_ref as K
    C = K.BN254
    c, z = bench.bench_inputs(C, "cfg2", 8, 33)
    assert c.shape == (8, 33, 4) and z.shape == (8, 4)
    assert list(z[:, 0]) == list(range(8))
    c, z = bench.bench_inputs(C, "cfg3", 8, 33)
    assert c.shape == (1, 33, 4)
    ints = [sum(int(w) << (64 * i) for i, w in enumerate(row)) for row in c[0]]
    assert all(0 <= v < C.r for v in ints)


def test_cfg5_fixed_bits_choice():
    """configs[4]: a rank's shard of <= 2^18 + 1 points gets the c = 10
    fixed-base table unless --fixed-bits says otherwise (bench.cfg5_fixed_bits;
    kzgx_dist.shard_range gives the shard sizes of the 2^20 + 1 coefficients)"""
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "kzg-commitments_amd", "python"))
    import bench
    import kzgx_dist
    n = (1 << 20) + 1
    want = {1: 0, 2: 0, 4: 10, 8: 10}
    for world, c in want.items():
        counts = [kzgx_dist.shard_range(n, world, r)[1] for r in range(world)]
        assert sum(counts) == n
        assert {bench.cfg5_fixed_bits(-1, k) for k in counts} == {c}, world
    assert bench.cfg5_fixed_bits(0, 131073) == 0
    assert bench.cfg5_fixed_bits(8, (1 << 20) + 1) == 8
