"""Single large MSMs on the table-less path (no default / fixed table):
device-resident scalars, HIP events on the call's stream, median of 7, every
result checked against [P(tau)]G1.  Sizes: the 8-way shard of the sharded
degree-2^20 commit (131 073 points on an SRS of that size, as each rank
holds), 2^17, the 2-way shard (2^19 + 1) and the whole degree-2^20 commit
(2^20 + 1).  From 2^16 points the wide-window path runs (msm.hip msm_big:
c = 14 / 15 / 16 by SRS size); KZGX_BIG_MIN=0 restores the round-4 chunked
c = 12 Pippenger for A/B.  Prints one JSON line per size."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kzg-commitments_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import torch  # noqa: E402,F401
import kzgx  # noqa: E402
import kzg_ref as K  # noqa: E402
import corc  # noqa: E402  (checker only: Horner of P at tau)

C = K.BN254
tau = K.default_tau(C)
sys.path.insert(0, ROOT)
from bench import random_fr  # noqa: E402

NMAX = (1 << 20) + 1
# uniform in [0, r) (round 6; round 5 drew 251-bit scalars, whose top window
# is empty -- real scalars put up to r's top bits there, and a window whose
# top digit takes few values concentrates entries in a few buckets)
P = random_fr(np.random.default_rng(5), (NMAX,), C.r)
corc.build()


def run(srs_n, n):
    ctx = kzgx.Context("BN254")
    try:
        ctx.set_default_table(0)
        if os.environ.get("KZGX_SEG"):  # A/B: entries per accumulation thread (default 128)
            ctx.set_segment(int(os.environ["KZGX_SEG"]))
        ctx.gen_srs(tau, srs_n)
        d_s = torch.from_numpy(P[:n].copy().view(np.int64)).cuda()
        d_o = torch.zeros((8,), dtype=torch.int64, device="cuda")
        d_i = torch.zeros((1,), dtype=torch.int32, device="cuda")
        st = torch.cuda.Stream()
        ts = []
        for rep in range(9):
            a = torch.cuda.Event(enable_timing=True)
            b = torch.cuda.Event(enable_timing=True)
            a.record(st)
            ctx.msm_batch_device(d_s.data_ptr(), n, 1, n, d_o.data_ptr(), d_i.data_ptr(), st.cuda_stream)
            b.record(st)
            b.synchronize()
            if rep >= 2:
                ts.append(a.elapsed_time(b))
        out = d_o.cpu().numpy().view(np.uint64)
        inf = bool(d_i.cpu().item())
        got = None if inf else (sum(int(out[j]) << (64 * j) for j in range(4)),
                                sum(int(out[4 + j]) << (64 * j) for j in range(4)))
        exp = K.scalar_mul(C, (C.gx, C.gy), corc.poly_eval("BN254", P[:n], tau))
        rec = {"srs_points": srs_n, "n": n, "median_ms": float(np.median(ts)), "min_ms": float(min(ts)),
               "per_s": 1e3 / float(np.median(ts)), "checked": got == exp,
               "path": "chunked c=12" if os.environ.get("KZGX_BIG_MIN") == "0" else "wide-window",
               "big_window": os.environ.get("KZGX_BIG_WINDOW", "auto"), "seg": os.environ.get("KZGX_SEG", "128")}
        print(json.dumps(rec), flush=True)
        assert got == exp
    finally:
        ctx.close()


SIZES = ((131073, 131073), ((1 << 17), (1 << 17)), ((1 << 19) + 1, (1 << 19) + 1), (NMAX, NMAX))
# optional argv: the sizes to run (e.g. "1048577")
pick = [int(a) for a in sys.argv[1:]]
for srs_n, n in SIZES:
    if not pick or n in pick:
        run(srs_n, n)
