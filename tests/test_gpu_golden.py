"""GPU vs the committed golden fixtures, through the C ABI (Python binding):
the SRS, interpolation of every reference input, commits, single- and
multi-point openings, and the synthetic benchmark-config polynomials."""
import hashlib
import json
import os

import numpy as np
import pytest

import kzg_ref as K

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CURVES = ["BN254", "BLS12381"]


def golden(name):
    with open(os.path.join(GOLD, name + ".json")) as f:
        return json.load(f)


def limbs(vals):
    return np.array([[(v >> (64 * i)) & 0xFFFFFFFFFFFFFFFF for i in range(4)] for v in vals],
                    dtype=np.uint64).reshape(-1, 4)


def ints(arr):
    return [sum(int(r[i]) << (64 * i) for i in range(len(r))) for r in np.asarray(arr).reshape(len(arr), -1)]


def pt(ctx, row, inf):
    if inf:
        return None
    w = ctx.w64
    return [hex(ints(row[None, :w])[0]), hex(ints(row[None, w:])[0])]


def case_points(C, case):
    raw = case["input"]
    if raw["kind"] == "string":
        return K.blob_from_string(C, bytes.fromhex(raw["hex"]), raw["offset"])
    if raw["kind"] == "bytes":
        data = bytes.fromhex(raw["hex"])
        return K.blob_from_bytes(C, data, 0, len(data), raw["chunk_size"])
    with open(os.path.join(GOLD, raw["file"])) as f:
        bts = K.pad_chunks(C, K.from_hex(f.read()))
    return K.blob_from_bytes(C, bts, 0, len(bts), C.max_chunk_bytes)


@pytest.fixture(scope="module")
def setups():
    import kzgx
    made = {}
    for name in CURVES:
        g = golden(name)
        ctx = kzgx.Context(name)
        ctx.gen_srs(int(g["tau"], 16), 5000)
        made[name] = (ctx, g)
    yield made
    for ctx, _ in made.values():
        ctx.close()


@pytest.mark.parametrize("name", CURVES)
def test_srs(name, setups):
    ctx, g = setups[name]
    srs = ctx.get_srs(5000)
    assert hashlib.sha256(srs.tobytes()).hexdigest() == g["srs_5000_sha256"]


@pytest.mark.parametrize("name", CURVES)
def test_reference_inputs(name, setups):
    ctx, g = setups[name]
    C = K.CURVES[name]
    for case in g["cases"]:
        if "input" not in case:
            continue
        pts = case_points(C, case)
        coeffs = ctx.interpolate(limbs([x for x, _ in pts]), limbs([y for _, y in pts]))
        P = K.normalize(ints(coeffs))
        assert hashlib.sha256(b"".join(c.to_bytes(32, "little") for c in P)).hexdigest() == case["coeffs_sha256"]
        if case.get("commit_throws"):
            assert len(P) >= case["setup"]
            continue
        out, inf = ctx.msm(limbs(P))
        assert pt(ctx, out, inf) == case["commit"], case["name"]
        for pr in case["proofs"]:
            xs = [pr["chunk_offset"] + i for i in range(pr["chunk_length"])]
            if pr["chunk_length"] == 1:
                o, f, _ = ctx.prove_single_batch(limbs(P), limbs(xs))
                got = pt(ctx, o[0], f[0])
            else:
                o, f = ctx.prove_range(limbs(P), limbs(xs))
                got = pt(ctx, o, f)
            assert got == pr["proof"], (case["name"], pr["chunk_offset"], pr["chunk_length"])


@pytest.mark.parametrize("name", CURVES)
def test_synthetic_configs(name, setups):
    ctx, g = setups[name]
    C = K.CURVES[name]
    for case in g["cases"]:
        if "synthetic_seed" not in case:
            continue
        P = K.random_scalars(C, case["n_coeffs"], case["synthetic_seed"])
        out, inf = ctx.msm(limbs(P))
        assert pt(ctx, out, inf) == case["commit"]
        zs = [p["z"] for p in case["single_proofs"]]
        o, f, y = ctx.prove_single_batch(limbs(P), limbs(zs))
        for j, p in enumerate(case["single_proofs"]):
            assert pt(ctx, o[j], f[j]) == p["proof"]
            assert hex(ints(y[j:j + 1])[0]) == p["y"]


@pytest.mark.parametrize("name", CURVES)
def test_multi_open_edges(name, setups):
    """multi-point openings: deg P < len (q = 0 -> infinity), offsets past the
    data, and the reference multi-proof shape (len up to the degree)"""
    ctx, g = setups[name]
    C = K.CURVES[name]
    tau = int(g["tau"], 16)
    P = K.random_scalars(C, 300, 99)
    for off, ln in ((0, 300), (0, 301), (250, 100), (5, 140), (17, 2)):
        o, f = ctx.prove_range(limbs(P), limbs([off + i for i in range(ln)]))
        q = K.proof_quotient(C, P, off, ln)
        exp = K.commit_via_tau(C, tau, q)
        assert pt(ctx, o, f) == (None if exp is None else [hex(exp[0]), hex(exp[1])]), (off, ln)
