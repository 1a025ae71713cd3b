#!/usr/bin/env python3
"""Verify-half timings on one MI355X: trusted_setup::
verify_proof latency at degree 4096 for 1..2048 opened points, batched
pairing throughput, and batched single-point verify throughput
(kzgx_verify_single_batch, host buffers in and out).  Reference numbers: README.md:130-144 (BN254, unstated CPU,
1 thread): single verify ~3.1 ms, 2048-point verify 1599 ms.

    python scripts/bench_verify.py [--curve BN254] [--pairings 4096]
Prints one JSON line."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kzg-commitments_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))  # checker only (known-tau verify)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--curve", default="BN254")
    ap.add_argument("--pairings", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--verifies", type=int, default=32768)
    args = ap.parse_args()
    import kzg_ref as K
    import kzgx

    C = K.CURVES[args.curve]
    w = kzgx.BASE_LIMBS[args.curve]
    tau = K.default_tau(C)
    ctx = kzgx.Context(args.curve)
    ctx.gen_srs(tau, 5000)
    ctx.gen_srs_g2(tau, 5000)
    P = K.random_scalars(C, 4097, 0x5EED)
    S = np.array([[(v >> (64 * i)) & 0xFFFFFFFFFFFFFFFF for i in range(4)] for v in P], dtype=np.uint64)
    com, cinf = ctx.msm(S)
    res = {"metric": "verify_proof latency + pairing throughput", "curve": args.curve, "degree": 4096,
           "verify_ms": {}, "checked": {}}
    for npts in (1, 16, 256, 2048):
        xs = list(range(7, 7 + npts))
        xa = np.array([[x, 0, 0, 0] for x in xs], dtype=np.uint64)
        ys = ctx.poly_eval(S, xa)
        prf, pinf = ctx.prove_range(S, xa)
        ok = ctx.verify_proof(com, cinf, prf, pinf, xa, ys)  # warm-up + correctness
        t0 = time.perf_counter()
        for _ in range(args.reps):
            ok = ctx.verify_proof(com, cinf, prf, pinf, xa, ys)
        res["verify_ms"][str(npts)] = (time.perf_counter() - t0) / args.reps * 1e3
        bad = ys.copy()
        bad[0, 0] ^= np.uint64(1)
        res["checked"][str(npts)] = bool(ok) and not ctx.verify_proof(com, cinf, prf, pinf, xa, bad)
    # batched pairings: e([k]G1, G2), k = 1..n
    n = args.pairings
    g1 = ctx.get_srs(1)
    g2 = ctx.get_srs_g2(1)
    A = np.repeat(g1, n, axis=0)
    B = np.repeat(g2, n, axis=0)
    out = ctx.pairing(A[:64], B[:64])  # warm-up
    t0 = time.perf_counter()
    out = ctx.pairing(A, B)
    dt = time.perf_counter() - t0
    res["pairings"] = n
    res["pairings_per_s"] = n / dt
    res["pairing_batch_ms"] = dt * 1e3
    res["pairings_consistent"] = bool((out == out[0]).all())
    # batched single-point verifies: one polynomial opened at n points
    nv = args.verifies
    zs = np.zeros((nv, 4), dtype=np.uint64)
    zs[:, 0] = np.arange(nv, dtype=np.uint64) + 1
    prf, pinf, yv = ctx.prove_single_batch(S, zs)
    cc = np.repeat(com[None, :], nv, axis=0)
    ok = ctx.verify_single_batch(cc[:64], prf[:64], zs[:64], yv[:64])  # warm-up
    t0 = time.perf_counter()
    ok = ctx.verify_single_batch(cc, prf, zs, yv)
    dt = time.perf_counter() - t0
    res["single_verifies"] = nv
    res["single_verifies_per_s"] = nv / dt
    res["single_verifies_all_ok"] = bool(ok.all())
    # wave-per-opening vs lane-per-opening kernels over batch sizes
    sweep = {}
    for m in (1, 16, 256, 1024, 4096, 16384):
        if m > nv:
            break
        row = {}
        for mode, wmax in (("wave", 1 << 30), ("lane", 0)):
            ctx.set_verify_wave_max(wmax)
            ok = ctx.verify_single_batch(cc[:m], prf[:m], zs[:m], yv[:m])  # warm-up (+ tables)
            reps = 5 if m <= 256 else 2
            t0 = time.perf_counter()
            for _ in range(reps):
                ok = ctx.verify_single_batch(cc[:m], prf[:m], zs[:m], yv[:m])
            dt = (time.perf_counter() - t0) / reps
            row[mode] = {"ms": dt * 1e3, "per_s": m / dt, "all_ok": bool(ok.all())}
        sweep[str(m)] = row
    ctx.set_verify_wave_max(8192)
    res["single_verify_sweep"] = sweep
    res["reference_readme_ms"] = {"verify_1": 3.109, "verify_2048": 1599.394, "source": "README.md:130-144 (BN254)"}
    print(json.dumps(res), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
