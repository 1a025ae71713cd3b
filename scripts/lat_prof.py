"""Single create_commit / create_proof calls (host buffers), for a rocprofv3
kernel trace: 10 Pippenger commits, then 10 table commits (c=16 table over
the 4097-point prefix, automatic points per thread)."""
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
ctx = kzgx.Context("BN254")
ctx.gen_srs(K.default_tau(C), 5000)
P = np.array([[(v >> (64 * i)) & 0xFFFFFFFFFFFFFFFF for i in range(4)] for v in K.random_scalars(C, 4097, 5)],
             dtype=np.uint64)
for tag in os.environ.get("LAT_TAGS", "pippenger,table").split(","):
    if tag == "table":
        ctx.set_fixed_base(16, 4097)
        ctx.set_fixed_points_per_thread(0)
    for _ in range(3):
        ctx.msm(P)
    ts = []
    for _ in range(10):
        t0 = time.perf_counter()
        ctx.msm(P)
        ts.append(time.perf_counter() - t0)
    print(tag, "commit median ms %.3f" % (1e3 * float(np.median(ts))), flush=True)
if os.environ.get("LAT_PROOF"):
    # single create_proof(poly, z, 1) calls on the Pippenger path (table off)
    ctx.set_fixed_base(0, 0)
    zs = np.array([[12345, 0, 0, 0]], dtype=np.uint64)
    for _ in range(3):
        ctx.prove_single_batch(P, zs)
    ts = []
    for _ in range(10):
        t0 = time.perf_counter()
        ctx.prove_single_batch(P, zs)
        ts.append(time.perf_counter() - t0)
    print("pippenger proof median ms %.3f" % (1e3 * float(np.median(ts))), flush=True)
