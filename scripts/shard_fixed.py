"""One rank's partial MSM of the sharded degree-2^20 commit (BASELINE
configs[4]) on the fixed-base table path against the wide-window Pippenger
path.  Rank 0's shard (131 073 points at world 8) on one context holding
only that SRS slice, as each rank of the driver's run does; for each window
c the shard's fixed-base table is built (setup, outside the timed region),
then the projective partial (kzgx_msm_g1_partial_device) is timed with HIP
events on its stream (median of 7 after 2 warm runs) and its affine value
checked against [P_shard(tau)]G1.  c = 0 is the table-less wide-window path.

    python3 scripts/shard_fixed.py [world] [c ...]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kzg-commitments_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import kzgx  # noqa: E402
import kzgx_dist  # noqa: E402
import kzg_ref as K  # noqa: E402
import corc  # noqa: E402  (checker only: P(tau) by Horner)
from bench import random_fr  # noqa: E402

world = int(sys.argv[1]) if len(sys.argv) > 1 else 8
windows = [int(a) for a in sys.argv[2:]] or [0, 9, 10, 11]
C = K.BN254
tau = K.default_tau(C)
n = (1 << 20) + 1
s0, cnt = kzgx_dist.shard_range(n, world, 0)
P = random_fr(np.random.default_rng(0x4B5A47), (n,), C.r)[s0:s0 + cnt].copy()
corc.build()
want = K.scalar_mul(C, (C.gx, C.gy), corc.poly_eval("BN254", P, tau) * pow(tau, s0, C.r) % C.r)


def timed(fn, st, reps=7, warm=2):
    ts = []
    for k in range(warm + reps):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record(st)
        fn()
        b.record(st)
        b.synchronize()
        if k >= warm:
            ts.append(a.elapsed_time(b))
    return float(np.median(ts)), float(min(ts))


ctx = kzgx.Context("BN254")
try:
    ctx.set_default_table(0)
    ctx.gen_srs(tau, cnt, s0)
    d_s = torch.from_numpy(P.view(np.int64)).cuda()
    rec = torch.zeros((ctx.partial_record_words,), dtype=torch.int64, device="cuda")
    out = torch.zeros((2 * ctx.w64 + 1,), dtype=torch.int64, device="cuda")
    st = torch.cuda.Stream()
    for c in windows:
        t0 = time.perf_counter()
        ctx.set_fixed_base(c, cnt if c else 0)
        torch.cuda.synchronize()
        setup_s = time.perf_counter() - t0
        info = ctx.fixed_base_info()
        med, mn = timed(lambda: ctx.msm_partial_device(d_s.data_ptr(), cnt, rec.data_ptr(), st.cuda_stream), st)
        ctx.g1_sum_partials_device(rec.data_ptr(), 1, out.data_ptr(), st.cuda_stream)
        st.synchronize()
        o = out.cpu().numpy().view(np.uint64)
        got = None if o[8] else (sum(int(o[j]) << (64 * j) for j in range(4)),
                                 sum(int(o[4 + j]) << (64 * j) for j in range(4)))
        print(json.dumps({"world": world, "rank": 0, "points": cnt, "fixed_bits": c,
                          "table_gb": info[2] / 1e9, "setup_s": setup_s, "partial_ms": med, "partial_min_ms": mn,
                          "checked": got == want,
                          "path": "fixed-base table" if c else "wide-window Pippenger"}), flush=True)
        assert got == want
finally:
    ctx.close()
