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
