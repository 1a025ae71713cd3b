#!/usr/bin/env python3
"""Generate the golden fixtures tests/golden/{BN254,BLS12381}.json.

Inputs are the reference's own test data (testing/testing.cpp strings,
testing/blob1.txt, testing/blob2.txt, the README.md example) plus seeded
synthetic polynomials for the benchmark configs.  Expected outputs come from
the oracle (oracle/kzg_ref.py) with a fixed tau; commits and proofs use the
MSM-independent identity [P(tau)]G1 / [q(tau)]G1, cross-checked against the
naive per-term MSM (polyeval_G1 restatement) wherever that is cheap.

The reference itself cannot run here, so these vectors pin
our implementation to the oracle; the oracle is pinned by the curve
self-checks and the identity above.  This script reads /root/reference
(inputs only); the fixtures it writes are self-contained so the GPU box never
needs the reference.

    python tests/golden/make_golden.py [--ref /root/reference]
"""
import argparse
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import corc  # noqa: E402
import kzg_ref as K  # noqa: E402

# testing/testing.cpp:224 and :233 (150 and 149 characters)
HIGH_150 = ("fa37JncCHryDsbzayy4cBWDxS22JjzhMaiRrV41mtzxlYvKWrO72tK0LK0e1zLOZ2nOXpPIhMFSv8kP07U20o0J90xA0GWXIIwo7J4o"
            "gHFZQxwQ2RQ0DRJKRETPVzxlFrXL8b7mtKLHIGhIh5JuWcF")
HIGH_149 = ("wrgJKdE3t5bECALy3eKIwYxEF3V7Z8KTx0nFe1IX5tjH22F5gXOa5LnIMIQuOiNJj8YL8rqDiZSkZfoEDAmGTXXqqvkCd5WKE2fMtVXa2zKa"
            "e6opGY4i6bYuUG67LaSXd5tUbO4bNPB0TxnkWrSaQ")


def coeff_bytes(P):
    return b"".join(c.to_bytes(32, "little") for c in P)


def pt_json(P):
    return None if P is None else [hex(P[0]), hex(P[1])]


def interp(C, name, pts):
    xs = [x for x, _ in pts]
    ys = [y for _, y in pts]
    if len(pts) > 400:
        return corc.interpolate(name, xs, ys)  # C oracle (checked against Python below on smaller cases)
    P = K.interpolate(C, pts)
    assert P == corc.interpolate(name, xs, ys)
    return P


def case_from_points(C, name, tau, label, pts, setup, proofs, naive_check, raw=None):
    P = interp(C, name, pts)
    case = {"name": label, "setup": setup, "n_points": len(pts), "deg": K.deg(P),
            "coeffs_sha256": hashlib.sha256(coeff_bytes(P)).hexdigest()}
    if raw is not None:
        case["input"] = raw
    if len(P) <= 160:
        case["coeffs"] = [hex(c) for c in P]
        case["poly_serialized"] = K.serialize_poly(C, P).hex()
    if K.deg(P) + 1 >= setup:
        case["commit_throws"] = True
    else:
        cm = K.commit_via_tau(C, tau, P)
        if naive_check:
            srs = corc.array_to_points(name, corc.gen_srs(name, tau, max(len(P), 2)))
            assert K.polyeval_g1(C, srs, P) == cm, label
        case["commit"] = pt_json(cm)
        case["commit_serialized"] = K.serialize_ecp(C, cm).hex()
    pr = []
    for off, ln in proofs:
        q = K.proof_quotient(C, P, off, ln)
        w = K.commit_via_tau(C, tau, q)
        if naive_check and q:
            srs = corc.array_to_points(name, corc.gen_srs(name, tau, max(len(q), 2)))
            assert K.polyeval_g1(C, srs, q) == w, (label, off, ln)
        pr.append({"chunk_offset": off, "chunk_length": ln, "q_deg": K.deg(q), "proof": pt_json(w),
                   "q_sha256": hashlib.sha256(coeff_bytes(q)).hexdigest()})
    case["proofs"] = pr
    return case, P


def synthetic(C, name, tau, label, n, seed, proofs, setup=5000):
    P = K.random_scalars(C, n, seed)
    case = {"name": label, "setup": setup, "synthetic_seed": seed, "n_coeffs": n,
            "coeffs_sha256": hashlib.sha256(coeff_bytes(P)).hexdigest(),
            "commit": pt_json(K.commit_via_tau(C, tau, P))}
    pr = []
    for z in proofs:
        yz = K.poly_eval(C, P, z)
        qt = (K.poly_eval(C, P, tau) - yz) * pow((tau - z) % C.r, -1, C.r) % C.r
        pr.append({"z": z, "y": hex(yz), "proof": pt_json(K.scalar_mul(C, (C.gx, C.gy), qt))})
    case["single_proofs"] = pr
    return case


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--curves", default="BN254,BLS12381")
    args = ap.parse_args()
    corc.build()
    with open(os.path.join(args.ref, "testing", "blob1.txt")) as f:
        blob1_hex = f.read()
    with open(os.path.join(args.ref, "testing", "blob2.txt")) as f:
        blob2_hex = f.read()
    # the reference's hex files are copied as data fixtures (inputs only)
    for nm, txt in (("blob1.txt", blob1_hex), ("blob2.txt", blob2_hex)):
        with open(os.path.join(HERE, nm), "w") as f:
            f.write(txt)

    for name in args.curves.split(","):
        C = K.CURVES[name]
        K.self_check(C)
        tau = K.default_tau(C)
        srs5000 = corc.gen_srs(name, tau, 5000)
        sample_idx = [0, 1, 2, 3, 127, 128, 149, 4096, 4999]
        pys = {i: K.scalar_mul(C, (C.gx, C.gy), pow(tau, i, C.r)) for i in sample_idx}
        got = corc.array_to_points(name, srs5000)
        for i in sample_idx:
            assert got[i] == pys[i]
        out = {
            "curve": name, "p": hex(C.p), "r": hex(C.r), "b": C.b, "gx": hex(C.gx), "gy": hex(C.gy),
            "modbytes": C.modbytes, "max_chunk_bytes": C.max_chunk_bytes, "tau": hex(tau),
            "tau_source": "sha256('kzg-mi355x-tau') mod r",
            "srs_5000_sha256": hashlib.sha256(srs5000.tobytes()).hexdigest(),
            "srs_sample": {str(i): pt_json(pys[i]) for i in sample_idx},
            "cases": [],
        }
        cases = out["cases"]
        M = C.max_chunk_bytes
        # ---- testing/testing.cpp ----
        for label, s, setup, proofs in [
            ("poly_degree_1_test K", b"K", 2, [(0, 1)]),                       # :165-190
            ("poly_degree_1_test AB", b"AB", 2, []),                           # throws at commit
            ("poly_degree_10_test 11 chars", b"CEBIDKAGFJH", 11, []),          # :195 throws
            ("poly_degree_10_test", b"CEBIDAGFJH", 11, [(2, 3)]),              # :204-214
            ("high_poly_degree_test 150", HIGH_150.encode(), 150, []),         # :224 throws
            ("high_poly_degree_test 149", HIGH_149.encode(), 150, [(49, 57)]),  # :233-240
            ("empty_verify_test", b"some data here", 128, [(7, 2)]),           # :139-151
            ("README example", b"hello there my name is bob", 128, [(0, 5), (15, 7), (23, 3)]),  # README.md:37
            ("signed chars", bytes([0x80, 0xFF, 0x7F, 0x00, 0x41]), 16, [(1, 2)]),  # blob.cpp:13 (char)
        ]:
            c, _ = case_from_points(C, name, tau, label, K.blob_from_string(C, s), setup, proofs, True,
                                    raw={"kind": "string", "hex": s.hex(), "offset": 0})
            cases.append(c)
        data = b"ysudYUGdghv675d\x00"  # testing.cpp:257 (sizeof includes the NUL)
        for cs, (bo, bl) in ((1, (3, 9)), (2, (2, 10)), (4, (4, 8))):  # :264-289
            pts = K.blob_from_bytes(C, data, 0, len(data), cs)
            c, _ = case_from_points(C, name, tau, "chunking_test chunk %d" % cs, pts, 128,
                                    [(bo // cs, bl // cs)], True,
                                    raw={"kind": "bytes", "hex": data.hex(), "chunk_size": cs})
            c["byte_proof"] = {"byte_offset": bo, "byte_length": bl, "chunk_size": cs}
            cases.append(c)
        # ---- eth_blob_test: testing.cpp:53-102 ----
        for label, txt, proofs in (("eth_blob_test blob2", blob2_hex, [(0, 1), (10, 4), (62, 4)]),
                                   ("eth_blob_test blob1", blob1_hex, [(7, 1), (100, 4), (4224, 4)])):
            bts = K.pad_chunks(C, K.from_hex(txt))
            pts = K.blob_from_bytes(C, bts, 0, len(bts), M)
            c, _ = case_from_points(C, name, tau, label, pts, 5000, proofs, False,
                                    raw={"kind": "hexfile", "file": "blob1.txt" if "blob1" in label else "blob2.txt",
                                         "n_bytes_padded": len(bts)})
            cases.append(c)
        # ---- benchmark configs: degree 128 and 4096 synthetic ----
        cases.append(synthetic(C, name, tau, "cfg1 degree 128", 129, 0x4B5A47, [0, 1, 128]))
        cases.append(synthetic(C, name, tau, "cfg2 degree 4096", 4097, 0x4B5A47 + 1, [0, 7, 4095]))
        with open(os.path.join(HERE, name + ".json"), "w") as f:
            json.dump(out, f, indent=1)
        print("wrote", name, len(cases), "cases")


if __name__ == "__main__":
    main()
