"""A/B timing of one large fixed-base MSM (the per-GPU shard of a sharded
cfg5 commit): python scripts/flat_small.py N C -> one JSON line with the
median call time (host buffers).  Run with and without KZGX_NO_FIXED_FLAT."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kzg-commitments_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))  # checker only
import kzg_ref as K  # noqa: E402
import kzgx  # noqa: E402

n, c = int(sys.argv[1]), int(sys.argv[2])
C = K.BN254
tau = K.default_tau(C)
ctx = kzgx.Context("BN254")
ctx.gen_srs(tau, n)
ctx.set_fixed_base(c, n)
rng = np.random.default_rng(7)
S = rng.integers(0, 2**63, size=(n, 4), dtype=np.uint64)
S[:, 3] &= np.uint64((1 << 59) - 1)
out, inf = ctx.msm(S)
ts = []
for _ in range(15):
    t0 = time.perf_counter()
    ctx.msm(S)
    ts.append(time.perf_counter() - t0)
import corc  # noqa: E402
exp = K.scalar_mul(C, (C.gx, C.gy), corc.poly_eval("BN254", S, tau))
got = None if inf else corc.array_to_points("BN254", out[None, :])[0]
print(json.dumps({"n": n, "c": c, "flat": "KZGX_NO_FIXED_FLAT" not in os.environ,
                  "median_ms": sorted(ts)[len(ts) // 2] * 1e3, "ok": got == exp}))
ctx.close()
