#!/usr/bin/env python3
"""Single-call latencies through the C ABI (host buffers in and out), the
shape of the reference's benchmark/benchmark.cpp:46-52 / :73-82 timed
regions: one create_commit, one create_proof(poly, 0, 1) and one
create_proof(poly, 0, N) at degree 4096.  Exploration tool; bench.py carries
the numbers that are reported."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kzg-commitments_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import kzgx  # noqa: E402
import kzg_ref as K  # noqa: E402


def timeit(f, reps=5):
    f()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t0)
    return min(ts) * 1e3, float(np.median(ts)) * 1e3


def main():
    fixed = int(sys.argv[1]) if len(sys.argv) > 1 else 0
    C = K.BN254
    ctx = kzgx.Context("BN254")
    tau = K.default_tau(C)
    ctx.gen_srs(tau, 5000)
    if fixed:
        ctx.set_fixed_base(fixed, 4097)
    P = np.array(K.random_scalars(C, 4097, seed=1), dtype=object)
    S = np.array([[(int(v) >> (64 * i)) & 0xFFFFFFFFFFFFFFFF for i in range(4)] for v in P], dtype=np.uint64)
    res = {"fixed_bits": fixed}
    res["commit_ms"] = timeit(lambda: ctx.msm(S))
    z = np.zeros((1, 4), dtype=np.uint64)
    res["proof1_ms"] = timeit(lambda: ctx.prove_single_batch(S, z))
    for N in (128, 512, 2048, 4096):
        xs = np.zeros((N, 4), dtype=np.uint64)
        xs[:, 0] = np.arange(N, dtype=np.uint64)
        res["proofN_ms_%d" % N] = timeit(lambda: ctx.prove_range(S[:4096], xs), reps=3)
    for b in (1, 8, 64, 1024):
        SB = np.tile(S, (b, 1))
        res["msm_batch_ms_%d" % b] = timeit(lambda: ctx.msm_batch(SB, 4097, b), reps=3)
    print(json.dumps(res))
    ctx.close()


if __name__ == "__main__":
    main()
