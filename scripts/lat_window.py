"""Single create_commit latency (host buffers, degree 4096, BN254) on the
Pippenger path at each supported window (the small-batch window table off),
and batches of 4..256 MSMs: the single-MSM reduction chain shortens with
fewer buckets while the accumulation grows.  Prints one JSON line per
window.  profiles/r03_latency_window.json."""
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

C = K.BN254
tau = K.default_tau(C)
vals = K.random_scalars(C, 4097, 5)
P = np.array([[(v >> (64 * i)) & 0xFFFFFFFFFFFFFFFF for i in range(4)] for v in vals], dtype=np.uint64)
exp = K.commit_via_tau(C, tau, vals)
for c in [int(x) for x in os.environ.get("LAT_WINDOWS", "9,10,11,12,13").split(",")]:
    ctx = kzgx.Context("BN254")  # the window is fixed before the SRS (its window table depends on it)
    ctx.set_window_bits(c)
    ctx.set_small_batch(0)  # this window's own table at every batch size
    ctx.gen_srs(tau, 5000)
    for _ in range(3):
        out, inf = ctx.msm(P)
    got = None if inf else (sum(int(out[i]) << (64 * i) for i in range(4)), sum(int(out[4 + i]) << (64 * i) for i in range(4)))
    ts = []
    for _ in range(15):
        t0 = time.perf_counter()
        ctx.msm(P)
        ts.append(time.perf_counter() - t0)
    rec = {"window_bits": c, "commit_ms_median": 1e3 * float(np.median(ts)), "ok": got == exp}
    for bsz in [int(x) for x in os.environ.get("LAT_BATCHES", "4,16,64,256").split(",") if x]:
        Pb = np.ascontiguousarray(np.broadcast_to(P, (bsz,) + P.shape))
        ctx.msm_batch(Pb, 4097, bsz)
        tb = []
        for _ in range(5):
            t0 = time.perf_counter()
            ctx.msm_batch(Pb, 4097, bsz)
            tb.append(time.perf_counter() - t0)
        rec["batch_%d_ms" % bsz] = 1e3 * float(np.median(tb))
    print(json.dumps(rec), flush=True)
    ctx.close()
