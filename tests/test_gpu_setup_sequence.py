"""Round-5 setup path, the way the reference benchmark drives it
(benchmark/benchmark.cpp:19-38: one trusted_setup per degree, each destroyed
before the next): G1 + G2 generation from the comb tables, the per-window
small-SRS Pippenger table, the adaptive batch-affine default table, pooled
context streams and the cached table block.  Every context's commit and
proof (default table, one-launch path) and a table-off commit (Pippenger,
which builds the small-batch table on first use) are checked against the
known-tau identity commit = [P(tau)]G1."""
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
def test_setup_sequence_commit_proof(name, C):
    import kzgx
    tau = K.default_tau(C)
    for deg in (128, 256, 512, 4096):
        ctx = kzgx.Context(name)
        try:
            ctx.gen_srs(tau, deg + 1)
            ctx.gen_srs_g2(tau, deg + 1)
            sc = K.random_scalars(C, deg + 1, seed=deg)
            P = limbs(sc)
            out, inf = ctx.msm(P)
            assert as_point(name, out, inf) == K.commit_via_tau(C, tau, sc), deg
            z0 = np.zeros((1, 4), dtype=np.uint64)
            pxy, pinf, y = ctx.prove_single_batch(P, z0)
            assert ctx.verify_proof(out, bool(inf), pxy[0], bool(pinf[0]), z0, y), deg
            # the table-off path (Pippenger, small-batch window table built lazily)
            ctx.set_default_table(0)
            out2, inf2 = ctx.msm(P)
            assert as_point(name, out2, inf2) == K.commit_via_tau(C, tau, sc), deg
        finally:
            ctx.close()
