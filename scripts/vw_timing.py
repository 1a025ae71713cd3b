"""One single-point verify_proof with the kernel's wall-clock stamps
(build variant KZGX_VW_TIMING) plus the host-side call latency."""
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
tau = K.default_tau(C)
ctx.gen_srs(tau, 4100)
ctx.gen_srs_g2(tau, 4100)
P = np.array([[(v >> (64 * i)) & 0xFFFFFFFFFFFFFFFF for i in range(4)] for v in K.random_scalars(C, 4097, 5)],
             dtype=np.uint64)
z0 = np.zeros((1, 4), dtype=np.uint64)
cxy, cinf = ctx.msm(P)
pxy, pinf, y = ctx.prove_single_batch(P, z0)
for _ in range(3):
    ok = ctx.verify_proof(cxy, cinf, pxy[0], bool(pinf[0]), z0, y)
ts = []
for _ in range(7):
    t0 = time.perf_counter()
    ok = ctx.verify_proof(cxy, cinf, pxy[0], bool(pinf[0]), z0, y)
    ts.append(time.perf_counter() - t0)
print("verify ok", ok, "median ms %.3f" % (1e3 * float(np.median(ts))), flush=True)
