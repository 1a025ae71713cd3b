"""Single large MSMs on the table-less Pippenger path (host buffers, medians
of 5): the per-rank partial of the sharded degree-2^20 commit (2^19 points
on 2 ranks) and the benchmark-common sizes.  KZGX_* knobs apply."""
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
ctx.set_default_table(0)
ctx.gen_srs(K.default_tau(C), (1 << 20) + 1)
rng = np.random.default_rng(5)
P = rng.integers(0, 2**63, size=((1 << 20) + 1, 4), dtype=np.uint64)
P[:, 3] &= np.uint64((1 << 59) - 1)
for n in (1 << 14, 1 << 17, (1 << 19) + 1, (1 << 20) + 1):
    ctx.msm(P[:n])
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        ctx.msm(P[:n])
        ts.append(time.perf_counter() - t0)
    print("pippenger n=%8d %.3f ms" % (n, 1e3 * float(np.median(ts))), flush=True)
