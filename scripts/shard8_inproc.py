"""The 8-way sharded degree-2^20 commit (BASELINE configs[4]) in one process
on one GPU: 8 contexts hold the 8 contiguous SRS slices each rank of the
driver's 8-GPU run holds (kzgx_dist.shard_range), so each context's partial
MSM is one rank's critical-path work, timed alone on its own stream with HIP
events (median of 7 after 2 warm runs).  Then the fold of the 8 projective
records (kzgx_g1_sum_partials_device) the same way, and the result against
[P(tau)]G1.  predicted_step_ms = max partial + fold (+ the all-gather, not
measurable on one GPU: 8 records of 144 B).  KZGX_BIG_WINDOW pins the
wide-window c (12..16; default by SRS size: 14 below 2^18 points).

    python3 scripts/shard8_inproc.py [world]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kzg-commitments_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import torch  # noqa: E402
import kzgx  # noqa: E402
import kzgx_dist  # noqa: E402
import kzg_ref as K  # noqa: E402
import corc  # noqa: E402  (checker only: P(tau) by Horner)

world = int(sys.argv[1]) if len(sys.argv) > 1 else 8
C = K.BN254
tau = K.default_tau(C)
n = (1 << 20) + 1
sys.path.insert(0, ROOT)
from bench import random_fr  # noqa: E402  (uniform in [0, r): the bench's cfg5 scalars)

P = random_fr(np.random.default_rng(0x4B5A47), (n,), C.r)
corc.build()


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


ctxs, scal, streams = [], [], []
try:
    for r in range(world):
        s0, cnt = kzgx_dist.shard_range(n, world, r)
        c = kzgx.Context("BN254")
        c.set_default_table(0)
        c.gen_srs(tau, cnt, s0)
        ctxs.append(c)
        scal.append(torch.from_numpy(P[s0:s0 + cnt].copy().view(np.int64)).cuda())
        streams.append(torch.cuda.Stream())
    rw = ctxs[0].partial_record_words
    recs = torch.zeros((world, rw), dtype=torch.int64, device="cuda")
    out = torch.zeros((9,), dtype=torch.int64, device="cuda")
    parts = []
    for r in range(world):
        cnt = kzgx_dist.shard_range(n, world, r)[1]
        med, mn = timed(lambda r=r, cnt=cnt: ctxs[r].msm_partial_device(scal[r].data_ptr(), cnt, recs[r].data_ptr(),
                                                                          streams[r].cuda_stream), streams[r])
        parts.append({"rank": r, "points": cnt, "partial_ms": med, "partial_min_ms": mn})
    fmed, fmin = timed(lambda: ctxs[0].g1_sum_partials_device(recs.data_ptr(), world, out.data_ptr(),
                                                              streams[0].cuda_stream), streams[0])
    o = out.cpu().numpy().view(np.uint64)
    got = None if o[8] else (sum(int(o[j]) << (64 * j) for j in range(4)), sum(int(o[4 + j]) << (64 * j) for j in range(4)))
    ok = got == K.scalar_mul(C, (C.gx, C.gy), corc.poly_eval("BN254", P, tau))
    # every shard at once on the one GPU (not the per-rank figure: 8 shards share the chip)
    def all_at_once():
        for r in range(world):
            cnt = kzgx_dist.shard_range(n, world, r)[1]
            ctxs[r].msm_partial_device(scal[r].data_ptr(), cnt, recs[r].data_ptr(), streams[r].cuda_stream)
        for r in range(1, world):
            ev = torch.cuda.Event()
            ev.record(streams[r])
            streams[0].wait_event(ev)
        ctxs[0].g1_sum_partials_device(recs.data_ptr(), world, out.data_ptr(), streams[0].cuda_stream)
    amed, _ = timed(all_at_once, streams[0])
    pmax = max(p["partial_ms"] for p in parts)
    print(json.dumps({"world": world, "n": n, "big_window": os.environ.get("KZGX_BIG_WINDOW", "auto"),
                      "per_rank": parts, "fold_ms": fmed, "fold_min_ms": fmin,
                      "predicted_step_ms": pmax + fmed, "predicted_commits_per_s": 1e3 / (pmax + fmed),
                      "all_shards_one_gpu_ms": amed, "checked": bool(ok),
                      "note": "partial_ms: one context's projective partial MSM alone on its stream (one rank's "
                              "work); fold_ms: kzgx_g1_sum_partials_device over the world records; the 8-GPU "
                              "step adds the RCCL all-gather of world x %d B" % (rw * 8)}), flush=True)
    assert ok
finally:
    for c in ctxs:
        c.close()
