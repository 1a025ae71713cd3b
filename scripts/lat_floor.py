"""Where a single host-buffer call's time goes (table-less default path):
the floor of a call that launches nothing (kzgx_sync), a 1-point MSM, and the
degree sweep of create_commit / create_proof(poly, z, 1), medians of 15.
Wrap in `rocprofv3 --kernel-trace --stats` for the per-kernel part."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kzg-commitments_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import kzgx  # noqa: E402
import kzg_ref as K  # noqa: E402


def med(f, reps=15):
    for _ in range(3):
        f()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t0)
    return 1e3 * float(np.median(ts))


C = K.BN254
ctx = kzgx.Context("BN254")
if os.environ.get("LAT_NO_DEFAULT_TABLE"):  # the table-off (Pippenger) path
    ctx.set_default_table(0)
ctx.gen_srs(K.default_tau(C), 5000)
P = np.array([[(v >> (64 * i)) & 0xFFFFFFFFFFFFFFFF for i in range(4)] for v in K.random_scalars(C, 4097, 5)],
             dtype=np.uint64)
z0 = np.zeros((1, 4), dtype=np.uint64)
z0[0, 0] = 12345
print("sync_ms %.4f" % med(ctx.sync), flush=True)


def clock_after(f):
    """core GHz seen by a one-wave probe enqueued right after one call f():
    the clock a single call runs at on an otherwise idle GPU"""
    import torch
    buf = torch.zeros(3, dtype=torch.int64, device="cuda")
    f()
    ctx.clock_probe(buf.data_ptr(), 200)
    ctx.sync()
    core, wall, khz = (int(v) for v in buf.cpu().tolist())
    return core / wall * khz * 1e-6 if wall else None


print("clock_ghz after a commit: %.3f" % clock_after(lambda: ctx.msm(P)), flush=True)
for n in (1, 2, 129, 257, 1025, 4097):
    print("commit n=%5d ms %.4f   proof ms %.4f" % (n, med(lambda: ctx.msm(P[:n])),
                                                      med(lambda: ctx.prove_single_batch(P[:n], z0))), flush=True)
