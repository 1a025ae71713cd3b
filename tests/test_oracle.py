"""CPU tests: the oracle against the golden fixtures and the reference's own
known behaviours (testing/testing.cpp).  No GPU needed.

The Python oracle (oracle/kzg_ref.py) and the C oracle (oracle/kzg_oracle.c)
are checked against each other and against tests/golden/*.json."""
import hashlib
import json
import os

import numpy as np
import pytest

import corc
import kzg_ref as K

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CURVES = ["BN254", "BLS12381"]


def golden(name):
    with open(os.path.join(GOLD, name + ".json")) as f:
        return json.load(f)


def pt(j):
    return None if j is None else (int(j[0], 16), int(j[1], 16))


def case_points(C, case):
    raw = case["input"]
    if raw["kind"] == "string":
        return K.blob_from_string(C, bytes.fromhex(raw["hex"]), raw["offset"])
    if raw["kind"] == "bytes":
        data = bytes.fromhex(raw["hex"])
        return K.blob_from_bytes(C, data, 0, len(data), raw["chunk_size"])
    with open(os.path.join(GOLD, raw["file"])) as f:
        bts = K.pad_chunks(C, K.from_hex(f.read()))
    assert len(bts) == raw["n_bytes_padded"]
    return K.blob_from_bytes(C, bts, 0, len(bts), C.max_chunk_bytes)


def coeff_sha(P):
    return hashlib.sha256(b"".join(c.to_bytes(32, "little") for c in P)).hexdigest()


@pytest.mark.parametrize("name", CURVES)
def test_curve_constants(name):
    C = K.CURVES[name]
    assert K.self_check(C)
    g = golden(name)
    assert int(g["p"], 16) == C.p and int(g["r"], 16) == C.r
    assert C.order_bytes == 32 and C.max_chunk_bytes == 31  # kzg.h:31, trusted_setup.cpp:18


def test_bn254_is_miracl_nogami_not_alt_bn128():
    C = K.BN254
    u = -(2**62 + 2**55 + 1)
    assert C.p == 36 * u**4 + 36 * u**3 + 24 * u**2 + 6 * u + 1
    assert C.b == 2 and (C.gx, C.gy) == (C.p - 1, 1)
    assert C.p != 0x30644E72E131A029B85045B68181585D97816A916871CA8D3C208C16D87CFD47


@pytest.mark.parametrize("name", CURVES)
def test_srs_matches_golden(name, oracle_c):
    C = K.CURVES[name]
    g = golden(name)
    tau = int(g["tau"], 16)
    assert tau == K.default_tau(C)
    srs = oracle_c.gen_srs(name, tau, 5000)
    assert hashlib.sha256(srs.tobytes()).hexdigest() == g["srs_5000_sha256"]
    pts = oracle_c.array_to_points(name, srs)
    for i, P in g["srs_sample"].items():
        assert pts[int(i)] == pt(P)


@pytest.mark.parametrize("name", CURVES)
def test_golden_cases(name, oracle_c):
    """interpolation, degree guard, commits and proofs of every golden case"""
    C = K.CURVES[name]
    g = golden(name)
    tau = int(g["tau"], 16)
    for case in g["cases"]:
        if "input" not in case:
            P = K.random_scalars(C, case["n_coeffs"], case["synthetic_seed"])
            assert coeff_sha(P) == case["coeffs_sha256"]
            assert K.commit_via_tau(C, tau, P) == pt(case["commit"])
            continue
        pts = case_points(C, case)
        xs, ys = [x for x, _ in pts], [y for _, y in pts]
        P = oracle_c.interpolate(name, xs, ys)
        assert coeff_sha(P) == case["coeffs_sha256"], case["name"]
        if len(P) <= 160:
            assert P == K.interpolate(C, pts)
            assert K.serialize_poly(C, P).hex() == case["poly_serialized"]
            assert K.deserialize_poly(C, bytes.fromhex(case["poly_serialized"])) == P
        if case.get("commit_throws"):
            with pytest.raises(ValueError):
                K.create_commit(C, [None] * case["setup"], P)
            continue
        assert K.commit_via_tau(C, tau, P) == pt(case["commit"])
        assert K.serialize_ecp(C, pt(case["commit"])).hex() == case["commit_serialized"]
        for pr in case["proofs"]:
            q = oracle_c.quotient(name, P, pr["chunk_offset"], pr["chunk_length"])
            assert coeff_sha(q) == pr["q_sha256"]
            assert K.commit_via_tau(C, tau, q) == pt(pr["proof"])


@pytest.mark.parametrize("name", CURVES)
def test_naive_msm_matches_golden_small(name, oracle_c):
    """the C restatement of polyeval_G1 (per-term scalar mult + add) on the small cases"""
    C = K.CURVES[name]
    g = golden(name)
    tau = int(g["tau"], 16)
    srs = oracle_c.gen_srs(name, tau, 160)
    for case in g["cases"]:
        if "coeffs" not in case or case.get("commit_throws"):
            continue
        P = [int(c, 16) for c in case["coeffs"]]
        got = oracle_c.msm_naive(name, srs[: max(len(P), 1)], oracle_c.ints_to_limbs(P, 4))
        assert got == pt(case["commit"]), case["name"]
        for pr in case["proofs"]:
            q = oracle_c.quotient(name, P, pr["chunk_offset"], pr["chunk_length"])
            if not q:
                assert pr["proof"] is None
                continue
            got = oracle_c.msm_naive(name, srs[: len(q)], oracle_c.ints_to_limbs(q, 4))
            assert got == pt(pr["proof"])


@pytest.mark.parametrize("name", CURVES)
def test_verify_round_trips(name):
    """known-tau restatement of verify_proof on the reference's small verify/refute cases"""
    C = K.CURVES[name]
    tau = K.default_tau(C)
    srs_len = 11
    P = K.interpolate(C, K.blob_from_string(C, b"CEBIDAGFJH"))
    cm = K.commit_via_tau(C, tau, P)
    proof = K.create_proof(C, None, P, 2, 3, tau)
    assert K.verify_proof_tau(C, tau, srs_len, cm, proof, K.blob_from_string(C, b"BID", 2))
    for s, off in ((b"CDEF", 0), (b"CD", 12), (b"BHSDJCSHJDVBZ", 0)):  # testing.cpp:216-219
        assert not K.verify_proof_tau(C, tau, srs_len, cm, proof, K.blob_from_string(C, s, off))
    with pytest.raises(ValueError):
        K.verify_proof_tau(C, tau, srs_len, cm, proof, [])  # empty_verify_test
    # degree-1 test (setup 2): refute2 has 2 points >= setup size -> false, no throw
    P1 = K.interpolate(C, K.blob_from_string(C, b"K"))
    cm1 = K.commit_via_tau(C, tau, P1)
    pr1 = K.create_proof(C, None, P1, 0, 1, tau)
    assert K.verify_proof_tau(C, tau, 2, cm1, pr1, K.blob_from_string(C, b"K", 0))
    assert not K.verify_proof_tau(C, tau, 2, cm1, pr1, K.blob_from_string(C, b"k", 0))
    assert not K.verify_proof_tau(C, tau, 2, cm1, pr1, K.blob_from_string(C, b"jj", 2))


def test_reference_argument_checks():
    C = K.BN254
    with pytest.raises(ValueError):
        K.gen_srs(C, 5, 0)  # invalid_setup_test
    with pytest.raises(ValueError):
        K.gen_srs(C, 5, 1)
    P = K.interpolate(C, K.blob_from_string(C, b"some data here"))
    with pytest.raises(ValueError):
        K.proof_quotient(C, P, 5, 0)  # empty_proof_test
    data = b"ysudYUGdghv675d\x00"
    with pytest.raises(ValueError):
        K.blob_from_bytes(C, data, 0, len(data), 3)  # chunks do not divide data
    with pytest.raises(ValueError):
        K.blob_from_bytes(C, data, 0, 32, 32)  # chunk > MAX_CHUNK_BYTES
    with pytest.raises(ValueError):
        K.create_proof_bytes(C, None, P, 0, 5, 4, tau=3)  # invalid byte length
    with pytest.raises(ValueError):
        K.create_proof_bytes(C, None, P, 2, 8, 4, tau=3)  # invalid byte offset


def test_blob_encodings():
    C = K.BN254
    pts = K.blob_from_string(C, bytes([0x41, 0x80, 0xFF]), 5)
    assert pts == [(5, 0x41), (6, C.r - 128), (7, C.r - 1)]  # (signed char) s[i]
    pts = K.blob_from_bytes(C, bytes(range(1, 9)), 8, 8, 4)
    assert pts == [(2, 0x04030201), (3, 0x08070605)]  # little-endian chunks, x = byte_offset / chunk
    assert K.from_hex("0a1\n") == bytes([0x0A, 0x01])  # odd length: strtol("1\n") = 1
    assert len(K.pad_chunks(C, bytes(31))) == 62  # always pads (testing.cpp:64-66)


def test_serialization_formats():
    C = K.BN254
    s = K.serialize_ecp(C, (C.gx, C.gy))
    assert s[:4] == (65).to_bytes(4, "little") and s[4] == 4 and len(s) == 69
    assert K.deserialize_ecp(C, s) == (C.gx, C.gy)
    assert K.deserialize_ecp(C, K.serialize_ecp(C, None)) is None
    P = [0, 1, 255, 256, C.r - 1]
    b = K.serialize_poly(C, P)
    assert b[:8] == (4).to_bytes(8, "little") and b[8] == 0 and b[9:11] == bytes([1, 1])
    assert K.deserialize_poly(C, b) == P
    assert K.serialize_poly(C, []) == (-1).to_bytes(8, "little", signed=True)


@pytest.mark.parametrize("name", CURVES)
def test_c_oracle_matches_python_oracle(name, oracle_c):
    C = K.CURVES[name]
    tau = 0x1234567
    srs = oracle_c.gen_srs(name, tau, 20)
    assert oracle_c.array_to_points(name, srs) == K.gen_srs(C, tau, 20)
    sc = K.random_scalars(C, 20, 11)
    assert oracle_c.msm_naive(name, srs, oracle_c.ints_to_limbs(sc, 4)) == K.commit_via_tau(C, tau, sc)
    assert oracle_c.msm_naive(name, srs[:0], np.zeros((0, 4), dtype=np.uint64)) is None
