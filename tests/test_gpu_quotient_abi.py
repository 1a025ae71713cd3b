"""kzgx_quotient_single_batch (host pointers): q = (P - P(z)) / (X - z) and
y = P(z), the quotient step of create_proof(poly, z, 1)
(trusted_setup.cpp:214-225), against the oracle's proof_quotient; shared and
per-opening polynomials, n = 1 (constant P: empty quotient), z = 0 and r - 1."""
import numpy as np
import pytest

import kzg_ref as K

pytestmark = pytest.mark.gpu

CURVES = [("BN254", K.BN254), ("BLS12381", K.BLS12381)]


def limbs(vals):
    return np.array([[(v >> (64 * i)) & 0xFFFFFFFFFFFFFFFF for i in range(4)] for v in vals], dtype=np.uint64)


def ints(rows):
    return [sum(int(r[i]) << (64 * i) for i in range(4)) for r in rows]


def trim(q):
    q = list(q)
    while q and q[-1] == 0:
        q.pop()
    return q


@pytest.mark.parametrize("name,C", CURVES)
def test_quotient_single_batch(name, C, ctx_factory):
    ctx = ctx_factory(name)
    zs = [0, 1, 5, C.r - 1, 123456789]
    for n in (1, 2, 33, 300):
        P = K.random_scalars(C, n, seed=7 * n)
        q, y = ctx.quotient_single_batch(limbs(P), limbs(zs))
        for j, z in enumerate(zs):
            assert ints(y[j:j + 1])[0] == K.poly_eval(C, P, z)
            assert trim(ints(q[j])) == trim(K.proof_quotient(C, P, z, 1))
    # one polynomial per opening
    n = 40
    Ps = [K.random_scalars(C, n, seed=100 + j) for j in range(len(zs))]
    q, y = ctx.quotient_single_batch(np.stack([limbs(P) for P in Ps]), limbs(zs), shared=False)
    for j, z in enumerate(zs):
        assert ints(y[j:j + 1])[0] == K.poly_eval(C, Ps[j], z)
        assert trim(ints(q[j])) == trim(K.proof_quotient(C, Ps[j], z, 1))


@pytest.mark.parametrize("name,C", [("BN254", K.BN254), ("BLS12381", K.BLS12381)])
@pytest.mark.parametrize("n", [8192, 65536, 70001, 1 << 20])
def test_quotient_single_large(name, C, n):
    """one opening of a long polynomial (n >= 2^13) takes the chip-wide three-phase
    quotient (k_qbig_*): q and y against the C oracle's quotient (n <= 70001)
    or the identity q(tau) = (P(tau) - P(z)) / (tau - z) through the proof"""
    import corc
    import kzgx
    ctx = kzgx.Context(name)
    try:
        rng = np.random.default_rng(n)
        S = rng.integers(0, 2**63, size=(n, 4), dtype=np.uint64)
        S[:, 3] &= np.uint64((1 << 59) - 1)
        z = 0x1234567 + n
        zs = np.array([[z, 0, 0, 0]], dtype=np.uint64)
        y_exp = corc.poly_eval(name, S, z)
        if n <= 70001:
            q, y = ctx.quotient_single_batch(S, zs)
            assert int(sum(int(y[0, i]) << (64 * i) for i in range(4))) == y_exp
            q_exp = corc.quotient(name, corc.limbs_to_ints(S), z, 1)
            assert corc.limbs_to_ints(q.reshape(-1, 4)) == q_exp
        tau = K.default_tau(C)
        ctx.gen_srs(tau, n + 1)
        out, inf, y = ctx.prove_single_batch(S, zs)
        assert int(sum(int(y[0, i]) << (64 * i) for i in range(4))) == y_exp
        qt = (corc.poly_eval(name, S, tau) - y_exp) * pow((tau - z) % C.r, -1, C.r) % C.r
        assert corc.array_to_points(name, out[0][None, :])[0] == corc.scalar_mul(name, (C.gx, C.gy), qt)
    finally:
        ctx.close()
