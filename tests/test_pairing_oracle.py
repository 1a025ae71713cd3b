"""CPU tests of the verify-half oracle (oracle/pairing_ref.py) and of the
build-time G2 / pairing constants (kzg-commitments_amd/csrc/gen_consts.py).

Pins: twist orders (exactly one sextic twist has order divisible by r, and
its generator has order r), pairing bilinearity and non-degeneracy, and the
pairing-form verify_proof (reference src/trusted_setup.cpp:230-254) agreeing
with the MSM-free known-tau identity on accept and reject cases."""
import importlib.util
import os
import struct

import pytest

import kzg_ref as K
import pairing_ref as PR

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CURVES = [K.BN254, K.BLS12381]


def gen_consts():
    spec = importlib.util.spec_from_file_location(
        "gen_consts", os.path.join(ROOT, "kzg-commitments_amd", "csrc", "gen_consts.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


@pytest.mark.parametrize("C", CURVES, ids=lambda c: c.name)
def test_twist_and_generator(C):
    assert PR.self_check(C)
    T = PR.twist(C)
    assert T.kind == ("D" if C.name == "BN254" else "M")
    assert T.order % C.r == 0


@pytest.mark.parametrize("C", CURVES, ids=lambda c: c.name)
def test_build_constants_match_oracle(C):
    """the device constants (G2 generator, twist b', Frobenius) are derived
    independently at build time; they must equal the oracle's"""
    g = gen_consts()
    d = g.g2_data(C.name)
    assert d["gen"] == PR.g2_generator(C)
    assert d["b2"] == PR.twist(C).b2
    assert d["d_type"] == (PR.twist(C).kind == "D")
    p = C.p
    # Frobenius on the twist: pi(Q) untwisted == (x^p, y^p) of the untwisted Q
    if d["d_type"]:
        Q = PR.g2_generator(C)
        q1 = (PR.f2mul(p, (Q[0][0], (-Q[0][1]) % p), d["twx"]), PR.f2mul(p, (Q[1][0], (-Q[1][1]) % p), d["twy"]))
        e = PR.untwist(C, Q)
        e1 = PR.untwist(C, q1)
        assert e1[0] == e[0].frob() and e1[1] == e[1].frob()
    # hard-part digits reassemble (p^4 - p^2 + 1) / r
    assert sum(v * p ** i for i, v in enumerate(d["digits"])) == (p ** 4 - p ** 2 + 1) // C.r


@pytest.mark.parametrize("C", CURVES, ids=lambda c: c.name)
def test_pairing_bilinear_nondegenerate(C):
    G1, G2 = (C.gx, C.gy), PR.g2_generator(C)
    e = PR.pairing(C, G1, G2)
    assert not e.is_one()
    assert e.pow(C.r).is_one()
    a, b = 0xDEADBEEF, 0x1337
    assert PR.pairing(C, K.scalar_mul(C, G1, a), PR.g2_mul(C, G2, b)) == e.pow(a * b)
    assert PR.pairing(C, None, G2).is_one() and PR.pairing(C, G1, None).is_one()


@pytest.mark.parametrize("C", CURVES, ids=lambda c: c.name)
def test_verify_proof_pairing_vs_tau(C):
    tau, n = K.default_tau(C), 8
    s1, s2 = K.gen_srs(C, tau, n), PR.gen_srs_g2(C, tau, n)
    P = K.random_scalars(C, 6, seed=11)
    com = K.commit_via_tau(C, tau, P)
    pts = K.evaluate_points(C, P, 1, 2)
    prf = K.create_proof(C, s1, P, 1, 2, tau=tau)
    assert PR.verify_proof(C, s1, s2, com, prf, pts) is True
    bad = [(x, (y + 1) % C.r) for x, y in pts]
    assert PR.verify_proof(C, s1, s2, com, prf, bad) is False
    assert K.verify_proof_tau(C, tau, n, com, prf, bad) is False
    assert PR.verify_proof(C, s1, s2, com, prf, [(x, x) for x in range(n)]) is False
    with pytest.raises(ValueError):
        PR.verify_proof(C, s1, s2, com, prf, [])


@pytest.mark.parametrize("C", CURVES, ids=lambda c: c.name)
def test_setup_file_layout(C):
    """export_setup layout (trusted_setup.cpp:256-287): u64 n, then n x
    (u32 len, G1 octet), then n x (u32 len, G2 octet)"""
    tau, n = 12345, 3
    s1, s2 = K.gen_srs(C, tau, n), PR.gen_srs_g2(C, tau, n)
    blob = PR.export_setup(C, s1, s2)
    mb = C.modbytes
    assert struct.unpack("<Q", blob[:8])[0] == n
    assert len(blob) == 8 + n * (4 + 2 * mb + 1) + n * (4 + 4 * mb + 1)
    off = 8 + n * (4 + 2 * mb + 1)
    for k in range(n):
        ln = struct.unpack("<I", blob[off:off + 4])[0]
        assert ln == 4 * mb + 1
        assert PR.ecp2_from_octet(C, blob[off + 4:off + 4 + ln]) == s2[k]
        off += 4 + ln
