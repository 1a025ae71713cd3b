"""GPU: the C++ drop-in facade (include/kzg.h) driven by tests/cpp/test_kzg.cpp,
a port of the reference's testing/testing.cpp, with every commitment, proof
and serialized polynomial compared byte-for-byte with the golden fixtures."""
import json
import os
import subprocess

import pytest

import kzg_ref as K

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "cpp", "test_kzg")
GOLD = os.path.join(ROOT, "tests", "golden")


@pytest.mark.parametrize("curve_id,name", [(0, "BN254"), (1, "BLS12381")])
def test_cpp_api_against_golden(curve_id, name):
    assert os.path.exists(BIN), "run __graft_entry__.build()"
    with open(os.path.join(GOLD, name + ".json")) as f:
        g = json.load(f)
    C = K.CURVES[name]
    res = subprocess.run([BIN, str(curve_id), g["tau"], GOLD], capture_output=True, text=True, timeout=600)
    out = res.stdout.splitlines()
    assert res.returncode == 0, res.stdout[-3000:] + res.stderr[-2000:]
    assert not [l for l in out if l.startswith("FAILED")]
    cases = {c["name"]: c for c in g["cases"]}
    seen = {"COMMIT": 0, "PROOF": 0, "POLY": 0}
    for line in out:
        parts = line.split("\t")
        tag = parts[0]
        if tag == "COMMIT":
            assert parts[2] == cases[parts[1]]["commit_serialized"], parts[1]
        elif tag == "PROOF":
            case = cases[parts[1]]
            off, ln = int(parts[2]), int(parts[3])
            pr = [p for p in case["proofs"] if (p["chunk_offset"], p["chunk_length"]) == (off, ln)]
            assert pr, (parts[1], off, ln)
            P = pr[0]["proof"]
            exp = K.serialize_ecp(C, None if P is None else (int(P[0], 16), int(P[1], 16))).hex()
            assert parts[4] == exp, (parts[1], off, ln)
        elif tag == "POLY":
            assert parts[2] == cases[parts[1]]["poly_serialized"], parts[1]
        else:
            continue
        seen[tag] += 1
    assert seen["COMMIT"] >= 11 and seen["PROOF"] >= 15 and seen["POLY"] >= 9, seen
