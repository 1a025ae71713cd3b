#!/usr/bin/env python3
"""bench.py -- KZG commits/s + proofs/s on MI355X (BASELINE.json metric).

Default workload (BASELINE.json configs[1]): BN254 (miracl Nogami curve),
degree 4096 -> 4097 coefficients per polynomial, SRS of 5000 points
(reference benchmark/benchmark.cpp:111).  One "step" = one batch of B
polynomials per GPU, each committed (create_commit: MSM over 4097 points)
and opened at one point (create_proof(poly, z, 1): quotient + MSM over 4096
points), i.e. 2B commits+proofs per GPU per step, all inputs resident in HBM
before the timed region.  Multi-GPU = independent batches per rank (weak
scaling, no collective in the data path); timing is max over ranks.

    python bench.py [--gpus N --steps K --warmup W --batch B --workload cfg2|cfg3|cfg4]

Prints ONE JSON line on rank 0.  The roofline entry is for the dominant
kernel (msm_accum), timed with HIP events on its launch stream inside the
timed region.  cpu_baseline times the C oracle (oracle/liboracle.so, a
restatement of the reference's naive per-term polyeval_G1) on a bounded
sample on one host core.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "kzg-commitments_amd", "python"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)

# The exact launch shape of each throughput line: curve, MSMs per launch,
# fixed-base window, SRS points per accumulation thread, streams per step.
# tests/test_gpu_configs.py runs these shapes through make_step() and checks
# every output; tests/test_bench_shapes.py pins them, so a changed default
# fails a test until the test is changed with it.
#   cfg2: 2048 MSMs x 3 wavefronts (22 points per thread): two full
#         residencies of the chip's 3072 accumulation slots per launch
#         (+2.9% over 1024 x 16, profiles/r02_ab_table_layout.json); c = 17
#         (15 windows for 254-bit scalars, 257.8 GB)
#   cfg3: one polynomial opened at x = 0..4095, one launch per step; 16
#         points per thread beats 22 there (profiles/r02_s3_cfg4_shape_ab.json)
#   cfg4: BLS12-381, 2048 x 1 wavefront (65 points per thread) = one
#         residency at 2 waves per SIMD (+5% over 1024 x 16); c = 16 (255-bit
#         scalars need 16 windows at c = 16 or 17)
WORKLOAD_SHAPES = {
    "cfg2": {"curve": "BN254", "batch": 2048, "fixed_bits": 17, "points_per_thread": 22, "streams": 2},
    "cfg3": {"curve": "BN254", "batch": 4096, "fixed_bits": 17, "points_per_thread": 16, "streams": 1},
    "cfg4": {"curve": "BLS12381", "batch": 2048, "fixed_bits": 16, "points_per_thread": 65, "streams": 2},
}
DEGREE = 4096      # BASELINE configs[1..3] (benchmark/benchmark.cpp:111)
SRS_POINTS = 5000  # the reference benchmark's setup size
REF_COMMIT_S = 1.104637  # README.md:132, BN254 degree 4096, 1 thread, unstated CPU
REF_PROOF_S = 1.080747


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=0,
                    help="polynomials (cfg2/cfg4) or openings (cfg3) per GPU per step; default cfg2 2048, "
                         "cfg4 2048, cfg3 4096 (BASELINE configs[2]: 4096 openings)")
    ap.add_argument("--workload", default="cfg2", choices=["cfg2", "cfg3", "cfg4", "cfg5", "common"],
                    help="cfg2..cfg5: BASELINE.json configs[1..4]; common: benchmark.cpp --benchmark-common")
    ap.add_argument("--window-bits", type=int, default=12, help="signed-digit window (10..13)")
    ap.add_argument("--segment", type=int, default=128, help="sorted entries per accumulation thread")
    ap.add_argument("--fixed-bits", type=int, default=-1,
                    help="fixed-base table window (0 = Pippenger only; default BN254 17: 15 windows, "
                         "257.8 GB of 64-B entries; BLS12-381 16: 240.6 GB of 112-B entries, of the 288 GiB HBM; "
                         "a window that does not fit steps down; cfg5 default: a c <= 10 table over shards of <= 2^18 + 1 "
                         "points, else 0: the wide-window Pippenger)")
    ap.add_argument("--fixed-ppt", type=int, default=-1,
                    help="SRS points per accumulation thread (fixed-base path; 0 = automatic; default cfg2 22: "
                         "2048 MSMs x 3 wavefronts = two full residencies per launch; cfg4 65: 2048 x 1 wavefront; "
                         "else 16)")
    ap.add_argument("--table-gb", type=float, default=0.0,
                    help="cfg5: fixed-base table budget per GPU (GB; 0 = free HBM minus 8 GB)")
    ap.add_argument("--serial", action="store_true",
                    help="commit and proof batches on one stream (exact per-kernel event timing)")
    ap.add_argument("--split", type=int, default=1, help="sub-batches (each on its own stream) per batch")
    ap.add_argument("--commit-first", action="store_true",
                    help="enqueue the commit batch before the proof batch (default: proofs first, so the "
                         "short quotient kernel is dispatched before the commit MSM fills the GPU)")
    ap.add_argument("--cpu-sample", type=int, default=12,
                    help="commits (+ as many proofs) timed on the CPU oracle (~0.4 s each)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pippenger", action="store_true",
                    help="skip the secondary Pippenger (table-less, create_commit's default) leg")
    ap.add_argument("--no-table-curve", action="store_true",
                    help="skip the throughput-vs-table-size leg (c = 10 .. 16, after the headline table)")
    ap.add_argument("--no-latency", action="store_true",
                    help="skip the single-call latency leg (benchmark/benchmark.cpp's timed regions)")
    ap.add_argument("--no-setup", action="store_true",
                    help="skip the trusted-setup leg (G1 + G2 SRS of 4097 points, README.md:124)")
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"],
                    help="cfg2/cfg3/cfg4: weak = --batch per GPU (default); strong = --global-batch split "
                         "over the ranks")
    ap.add_argument("--global-batch", type=int, default=0,
                    help="--scaling strong: polynomials (openings for cfg3) per step over all ranks "
                         "(default 8 x the per-GPU default batch)")
    return ap.parse_args()


def curve_consts(curve):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))  # checker only (parity + cpu_baseline)
    import kzg_ref
    return kzg_ref, kzg_ref.CURVES[curve]


def random_fr(rng, shape, r):
    """uniform integers in [0, r) as little-endian uint64 limbs (..., 4)"""
    rl = [(r >> (64 * i)) & 0xFFFFFFFFFFFFFFFF for i in range(4)]
    top_bits = r.bit_length() - 192
    out = rng.integers(0, 2**64, size=shape + (4,), dtype=np.uint64)
    out[..., 3] &= np.uint64((1 << top_bits) - 1)
    while True:
        w = out.reshape(-1, 4)
        ge = np.zeros(w.shape[0], dtype=bool)
        eq = np.ones(w.shape[0], dtype=bool)
        for i in (3, 2, 1, 0):
            ge |= eq & (w[:, i] > np.uint64(rl[i]))
            eq &= w[:, i] == np.uint64(rl[i])
        ge |= eq
        if not ge.any():
            return out
        fresh = rng.integers(0, 2**64, size=(int(ge.sum()), 4), dtype=np.uint64)
        fresh[:, 3] &= np.uint64((1 << top_bits) - 1)
        w[ge] = fresh


def fixed_table_bytes(curve, c, npts):
    """device bytes of the fixed-base table (msm_fixed.hip: W x n x 2^(c-1)
    entries of 64 B (BN254, packed words) / 112 B (BLS12-381, radix-2^29 limbs);
    W = ceil(bits(r) / c) regular odd digits, fixed_accum.hpp)"""
    bits = 254 if curve == "BN254" else 255
    w = (bits + c - 1) // c
    return w * npts * (1 << (c - 1)) * (64 if curve == "BN254" else 112)


def set_fixed_with_fallback(kzgx, ctx, c, npts, budget=None):
    """build the fixed-base table at the widest window <= c that fits the
    device's free memory (minus 8 GB for workspaces) and the optional budget;
    a failed allocation steps the window down once more.  Returns the window
    built (0 = none: Pippenger)."""
    import torch
    free = torch.cuda.mem_get_info()[0] - 8e9
    if budget is not None:
        free = min(free, budget)
    while c >= 7 and fixed_table_bytes(ctx.curve, c, npts) > free:
        c -= 1
    while c >= 7:
        try:
            ctx.set_fixed_base(c, npts)
            return c
        except kzgx.KzgxError as e:
            if e.status != -3:  # KZGX_ERR_OOM
                raise
            print("bench: fixed-base table c=%d did not fit, trying c=%d" % (c, c - 1), file=sys.stderr)
            c -= 1
    ctx.set_fixed_base(0, 0)
    return 0


def to_int(row):
    return sum(int(row[i]) << (64 * i) for i in range(len(row)))


def bench_inputs(C, workload, B, n, rank=0):
    """seeded host inputs of one step: coefficients (1 or B polynomials of n
    Fr limbs) and the opening points z"""
    rng = np.random.default_rng(0x4B5A47 + rank)
    zs_h = np.zeros((B, 4), dtype=np.uint64)
    if workload == "cfg3":
        # one degree-4096 polynomial opened at x = 0..B-1 (the reference's
        # multi-proof benchmark's 4096 openings as single-opening proofs,
        # SURVEY 8(a) a8)
        coeffs_h = random_fr(rng, (1, n), C.r)
        zs_h[:, 0] = np.arange(B, dtype=np.uint64)
    else:
        coeffs_h = random_fr(rng, (B, n), C.r)
        zs_h[:, 0] = np.arange(B, dtype=np.uint64) % n
    return coeffs_h, zs_h


class StepBuffers:
    """device inputs and outputs of one bench step"""

    def __init__(self, torch, dev, coeffs_h, zs_h, w64):
        B = zs_h.shape[0]
        self.d_coeffs = torch.from_numpy(coeffs_h.view(np.int64)).to(dev)
        self.d_z = torch.from_numpy(zs_h.view(np.int64)).to(dev)
        self.d_cout = torch.zeros((B, 2 * w64), dtype=torch.int64, device=dev)
        self.d_cinf = torch.zeros((B,), dtype=torch.int32, device=dev)
        self.d_pout = torch.zeros((B, 2 * w64), dtype=torch.int64, device=dev)
        self.d_pinf = torch.zeros((B,), dtype=torch.int32, device=dev)
        self.d_y = torch.zeros((B, 4), dtype=torch.int64, device=dev)


def make_step(ctx, workload, n, bufs, streams, split=1, commit_first=False):
    """one step: B commits (create_commit, n-point MSM) on streams[2s] and B
    single-opening proofs (create_proof(poly, z, 1): quotient + (n-1)-point
    MSM) on streams[2s + 1], cut into `split` sub-batches; cfg3 has no
    commits and one shared polynomial"""
    B = bufs.d_z.shape[0]
    S = max(1, split)
    cstride = 0 if workload == "cfg3" else n
    cut = [B * s // S for s in range(S + 1)]

    def step():
        for s in range(S):
            lo, hi = cut[s], cut[s + 1]
            if hi == lo:
                continue

            def commits():
                if workload != "cfg3":
                    ctx.msm_batch_device(bufs.d_coeffs[lo].data_ptr(), n, hi - lo, n, bufs.d_cout[lo].data_ptr(),
                                         bufs.d_cinf[lo:].data_ptr(), streams[2 * s].cuda_stream)

            def proofs():
                ctx.prove_single_batch_device(bufs.d_coeffs[0 if cstride == 0 else lo].data_ptr(), n, cstride,
                                              bufs.d_z[lo].data_ptr(), hi - lo, bufs.d_pout[lo].data_ptr(),
                                              bufs.d_pinf[lo:].data_ptr(), bufs.d_y[lo].data_ptr(),
                                              streams[2 * s + 1].cuda_stream)

            for f in ((commits, proofs) if commit_first else (proofs, commits)):
                f()

    return step


def check_step(curve, C, tau, workload, coeffs_h, zs_h, bufs, w64):
    """every output of the last step against the MSM-independent identity
    (test infrastructure, outside the timed region): commit = [P(tau)]G1,
    proof = [(P(tau) - P(z)) / (tau - z)]G1, y = P(z), with the C oracle's
    Horner evaluation and scalar multiplication.  Returns (checked, ok,
    first failure)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))  # checker only
    import corc
    corc.build()
    cout = bufs.d_cout.cpu().numpy().view(np.uint64)
    cinf = bufs.d_cinf.cpu().numpy()
    pout = bufs.d_pout.cpu().numpy().view(np.uint64)
    pinf = bufs.d_pinf.cpu().numpy()
    ys = corc.limbs_to_ints(bufs.d_y.cpu().numpy().view(np.uint64))
    G = (C.gx, C.gy)
    B = zs_h.shape[0]
    checked = ok = 0
    bad = None
    ptau_shared = corc.poly_eval(curve, coeffs_h[0], tau) if workload == "cfg3" else None

    def got(row, inf):
        return None if inf else (to_int(row[:w64]), to_int(row[w64:2 * w64]))

    for b in range(B):
        P = coeffs_h[0 if workload == "cfg3" else b]
        ptau = ptau_shared if workload == "cfg3" else corc.poly_eval(curve, P, tau)
        if workload != "cfg3":
            checked += 1
            good = got(cout[b], cinf[b]) == corc.scalar_mul(curve, G, ptau)
            ok += good
            bad = bad or (None if good else ("commit", b))
        z = to_int(zs_h[b])
        pz = corc.poly_eval(curve, P, z)
        qt = (ptau - pz) * pow((tau - z) % C.r, -1, C.r) % C.r
        checked += 2
        g1 = got(pout[b], pinf[b]) == corc.scalar_mul(curve, G, qt)
        g2 = ys[b] == pz
        ok += int(g1) + int(g2)
        bad = bad or (None if g1 else ("proof", b)) or (None if g2 else ("y", b))
    return checked, ok, bad


KERNELS = ("msm_count", "msm_scan", "msm_scatter", "msm_accum", "msm_reduce", "quotient_single")


def timed_run(ctx, step, streams, steps, warmup, world, dist, torch, dev):
    """W untimed warmup steps, then exactly K steps bracketed by a barrier +
    synchronize on both sides; per-kernel HIP-event times (on each launch's
    own stream) are collected inside the timed region.  Returns (elapsed s,
    {kernel: (total ms, launches)}), elapsed = max over ranks."""
    stream = streams[0]
    for _ in range(warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    ctx.prof_clear()
    ctx.prof_enable(True)
    ev0 = torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    ev0.record(stream)
    for s in streams[1:]:
        if s is not stream:
            s.wait_event(ev0)
    for _ in range(steps):
        step()
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    ctx.prof_enable(False)
    elapsed = t1 - t0
    kern = {name: ctx.prof_read(name) for name in KERNELS}
    local_s = elapsed
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed, kern, local_s


def clock_during(ctx, step, step_s, torch, dev, nsteps=4):
    """core GHz while `step` runs: the probe (kzgx_clock_probe) is enqueued
    first on a stream of its own, so it is resident before the step's kernels
    fill the GPU, and spins for about half of nsteps steps"""
    try:
        buf = torch.zeros(3, dtype=torch.int64, device=dev)
        ps = torch.cuda.Stream(device=dev)
        torch.cuda.synchronize(dev)
        ctx.clock_probe(buf.data_ptr(), max(1000, int(step_s * 1e6 * nsteps / 2)), ps.cuda_stream)
        for _ in range(nsteps):
            step()
        torch.cuda.synchronize(dev)
        core, wall, khz = (int(v) for v in buf.cpu().tolist())
        return core / wall * khz * 1e-6 if wall else None
    except Exception as e:  # noqa: BLE001 -- a measurement aid, never fatal
        print("bench: clock probe unavailable: %s" % e, file=sys.stderr)
        return None


def median_ms(f, reps):
    f()  # warm (workspaces, first-use tables)
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts)) * 1e3


def latency_leg(ctx, coeffs_h, reps=7):
    """The reference's own timed regions (benchmark/benchmark.cpp:46-52 and
    :73-82), one call each through the C ABI entry points the C++ facade
    calls (host buffers in, result on the host): create_commit of a
    degree-4096 polynomial, create_proof(poly, 0, 1), and the multi-point
    create_proof(poly, 0, N) on a 4096-coefficient polynomial."""
    P = coeffs_h[0]
    z0 = np.zeros((1, 4), dtype=np.uint64)
    out = {"commit_ms": median_ms(lambda: ctx.msm(P), reps),
           "proof_ms": median_ms(lambda: ctx.prove_single_batch(P, z0), reps)}
    multi = {}
    for N in (128, 256, 512, 1024, 2048, 4096):
        xs = np.zeros((N, 4), dtype=np.uint64)
        xs[:, 0] = np.arange(N, dtype=np.uint64)
        multi[str(N)] = median_ms(lambda: ctx.prove_range(P[:4096], xs), 3)
    out["multi_proof_ms"] = multi
    # benchmark/benchmark.cpp:113-115: single commit / proof for degree
    # 128 .. 4096 (README.md:127-132 publishes 30.1 / 42.5 ms at 128)
    sweep = {}
    for deg in (128, 256, 512, 1024, 2048, 4096):
        Pd = P[:deg + 1]
        sweep[str(deg)] = {"commit_ms": median_ms(lambda: ctx.msm(Pd), reps),
                           "proof_ms": median_ms(lambda: ctx.prove_single_batch(Pd, z0), reps)}
    out["degree_sweep"] = sweep
    return out


def mads_per_mixed_add(L):
    """v_mad_u64_u32 per XYZZ mixed addition (curve.hpp xyzz_add_affine_*):
    6 products (L^2 + L^2 reduction), 2 squares (L(L+1)/2 + L^2) and one
    two-product sum with one reduction (3 L^2) -- 1467 for BN254 (L = 9),
    3542 for BLS12-381 (L = 14); the gfx950 ISA of k_fixed_accum holds exactly
    these (scripts/isa_count.py, profiles/r03_isa_counts.json)"""
    return 6 * 2 * L * L + 2 * (L * (L + 1) // 2 + L * L) + 3 * L * L


def dist_info(world, dist, torch):
    """what actually carried the ranks: the process-group backend and, on
    ROCm, the RCCL version torch was built against (torch.cuda.nccl)"""
    info = {"world_size": world, "backend": None, "rccl_version": None}
    if world > 1:
        try:
            info["backend"] = str(dist.get_backend())
        except Exception as e:  # noqa: BLE001 -- reported, never fatal
            info["backend"] = "unknown (%s)" % e
    try:
        v = torch.cuda.nccl.version()
        info["rccl_version"] = ".".join(str(x) for x in v) if isinstance(v, tuple) else str(v)
    except Exception:  # noqa: BLE001
        pass
    return info


def rank_records(world, rank, local, dev, local_s, dist, torch, extra=None):
    """one record per rank: the device it ran on (ordinal, PCI address, UUID,
    the visible-device mask) and its own elapsed time of the timed region, so
    a multi-GPU line shows that N distinct GPUs ran and how evenly"""
    props = torch.cuda.get_device_properties(dev) if dev is not None else None
    rec = {"rank": rank, "local_rank": local, "device": dev.index if dev is not None else None,
           "pci": "%04x:%02x:%02x.0" % (getattr(props, "pci_domain_id", 0), getattr(props, "pci_bus_id", 0),
                                        getattr(props, "pci_device_id", 0)) if props is not None else None,
           "uuid": str(getattr(props, "uuid", "")) if props is not None else None,
           "visible_devices": os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("CUDA_VISIBLE_DEVICES"),
           "elapsed_s": local_s}
    if extra:
        rec.update(extra)
    if world == 1:
        return [rec]
    out = [None] * world
    dist.all_gather_object(out, rec)
    return out


def accum_kernel_id(curve, c):
    """SHA-256 of the gfx950 machine code of k_fixed_accum<curve, c> in the
    loaded libkzgx.so (python/codeobj.py): counter passes are attached to a
    line only when they measured this exact kernel"""
    try:
        import codeobj
        import kzgx
        return codeobj.kernel_hash(kzgx.LIB_PATH, *codeobj.fixed_accum_parts(curve, c))
    except Exception as e:  # noqa: BLE001 -- reported, never fatal
        return {"sha256": None, "error": str(e)}


def matching_traffic(workload, batch, fixed_bits, kernel_sha):
    """the counter pass (profiles/*pmc_traffic_<workload>*.json, written by
    scripts/pmc_traffic.py) of this kernel build at this batch and window, or
    None: a pass of another build is never presented as this kernel's traffic"""
    import glob
    if not kernel_sha:
        return None, None
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc_traffic_%s*.json" % workload)), reverse=True):
        try:
            with open(path) as f:
                tj = json.load(f)
        except (OSError, ValueError):
            continue
        if tj.get("kernel_sha256") == kernel_sha and tj.get("batch") == batch and tj.get("fixed_bits") == fixed_bits:
            return tj, os.path.relpath(path, ROOT)
    return None, None


def setup_leg(kzgx, curve, K, C, tau, npts=DEGREE + 1, reps=3):
    """trusted_setup(4097) on the GPU: the G1 and G2 SRS of a degree-4096
    setup (src/trusted_setup.cpp:21-74; README.md:124 publishes 947.288 ms for
    the 4096-term G1 + G2 setup on all threads).  A fresh context per run;
    the first run carries the one-time code-object load and is reported
    apart.  Checked: every G1 point against the C port, sampled G2 points
    against the Python oracle's [tau^i]G2."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))  # checker only
    import corc
    import pairing_ref as PR
    times = []
    g1 = g2 = None
    for k in range(reps + 1):
        c2 = kzgx.Context(curve)
        t0 = time.perf_counter()
        c2.gen_srs(tau, npts)
        c2.gen_srs_g2(tau, npts)
        c2.sync()
        times.append((time.perf_counter() - t0) * 1e3)
        if k == reps:
            g1 = c2.get_srs(npts)
            g2 = c2.get_srs_g2(npts)
        c2.close()
    corc.build()
    tc = time.perf_counter()
    ref1 = corc.gen_srs(curve, tau, npts)
    cpu_g1_ms = (time.perf_counter() - tc) * 1e3
    w = 4 if curve == "BN254" else 6
    Q = PR.g2_generator(C)
    g2_ok = True
    for i in (0, 1, 2, npts // 2, npts - 2, npts - 1):
        v = [to_int(g2[i][k * w:(k + 1) * w]) for k in range(4)]
        g2_ok &= ((v[0], v[1]), (v[2], v[3])) == PR.g2_mul(C, Q, pow(tau, i, C.r))
    return {"points": npts, "g1_g2_ms": float(np.median(times[1:])), "first_call_ms": times[0],
            "runs_ms": times[1:],
            "reference_published_ms": 947.288,
            "reference_source": "README.md:124, G1 + G2 setup of 4096 terms, all host threads, unstated CPU",
            "cpu_port_g1_ms": cpu_g1_ms,
            "cpu_port_note": "G1 half only, C restatement (oracle/kzg_oracle.c: tau^i by repeated products, "
                             "one double-and-add scalar multiplication per point), 1 thread",
            "parity": {"g1_points_checked": npts, "g1_ok": bool(np.array_equal(g1, ref1)),
                       "g2_points_checked": 6, "g2_ok": bool(g2_ok)}}


def free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def rank_launch_cmd(n, argv, port):
    """the child command that runs `bench.py <argv>` as n ranks, one process
    per GPU (the same form the driver uses for its multi-GPU runs)"""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % n,
            "--master-addr=127.0.0.1", "--master-port=%d" % port, os.path.abspath(__file__)] + list(argv)


def launch_ranks(n, argv):
    """`bench.py --gpus N` with no launcher around it: start the N ranks as a
    child torch.distributed.run and wait.  This process never touches the GPU
    (no torch import, no HIP call), so nothing is exec'ed from a process that
    initialised the device.  Rank 0's JSON line reaches stdout through the
    inherited descriptor; the exit status is the launcher's (non-zero when
    any rank fails)."""
    import subprocess
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on these hosts (RCCL)
    return subprocess.call(rank_launch_cmd(n, argv, free_port()), env=env)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return launch_ranks(args.gpus, sys.argv[1:])
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit("bench: WORLD_SIZE=%d but --gpus %d" % (world, args.gpus))
    selftest = os.environ.get("KZGX_BENCH_LAUNCH_SELFTEST")
    if selftest == "1":
        # launcher self-test (tests/test_bench_launcher.py, CPU only): report
        # the rank layout and stop before anything touches a device
        fail = os.environ.get("KZGX_BENCH_FAIL_RANK")
        if fail is not None and int(fail) == rank:
            return 3
        if rank == 0:
            print(json.dumps({"selftest": True, "world": world, "rank": rank, "gpus": args.gpus}), flush=True)
        return 0
    if selftest == "dist":
        # the per-rank provenance fields of a multi-GPU line, over gloo on
        # the CPU (no device): every rank's record reaches rank 0
        import torch
        import torch.distributed as dist
        if world > 1:
            dist.init_process_group(backend="gloo", init_method="env://")
        t0 = time.perf_counter()
        if world > 1:
            dist.barrier()
        ranks = rank_records(world, rank, local, None, time.perf_counter() - t0, dist, torch, {"batch": 7 + rank})
        dinfo = dist_info(world, dist, torch)
        if rank == 0:
            print(json.dumps({"selftest": "dist", "ranks": ranks, "dist": dinfo}), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return 0
    import torch
    import torch.distributed as dist

    # one process per GPU; KZGX_BENCH_ONE_DEVICE=1 maps every rank to device 0
    # and KZGX_DIST_BACKEND=gloo swaps RCCL for gloo -- only to rehearse the
    # N > 1 control flow on a one-GPU box (the driver's runs use neither)
    if os.environ.get("KZGX_BENCH_ONE_DEVICE") == "1":
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        backend = os.environ.get("KZGX_DIST_BACKEND", "nccl")
        if backend == "nccl":
            # bind the communicator to this rank's GPU up front (barriers and
            # collectives then never guess the device)
            dist.init_process_group(backend="nccl", init_method="env://", device_id=dev)
        else:
            dist.init_process_group(backend=backend, init_method="env://")

    import kzgx

    if args.workload == "cfg5":
        return run_cfg5(args, world, rank, local, dev, torch, dist, kzgx)
    if args.workload == "common":
        return run_common(args, world, rank, local, dev, torch, dist, kzgx)

    shape = WORKLOAD_SHAPES[args.workload]
    curve = shape["curve"]
    K, C = curve_consts(curve)
    tau = K.default_tau(C)
    degree = DEGREE
    n = degree + 1
    B = args.batch or shape["batch"]
    global_batch = B * world
    if args.scaling == "strong":
        # a fixed total batch split over the ranks (the first ranks take the
        # remainder): 1/2/4/8 GPUs then trace a strong-scaling curve
        global_batch = args.global_batch or 8 * shape["batch"]
        if global_batch < world:  # every rank needs at least one polynomial
            raise SystemExit("--global-batch %d is smaller than the world size %d" % (global_batch, world))
        B = global_batch // world + (1 if rank < global_batch % world else 0)
    if args.fixed_ppt < 0:
        args.fixed_ppt = shape["points_per_thread"]
    ctx = kzgx.Context(curve, device=local)
    ctx.set_window_bits(args.window_bits)
    ctx.set_segment(args.segment)
    ctx.gen_srs(tau, SRS_POINTS)
    w64 = ctx.w64

    coeffs_h, zs_h = bench_inputs(C, args.workload, B, n, rank)
    bufs = StepBuffers(torch, dev, coeffs_h, zs_h, w64)
    # the commits and proofs of a step are independent batches: each runs on
    # its own stream (optionally cut into `split` sub-batches) so the short
    # latency-bound phases of one (reduction, affine conversion, quotient)
    # overlap the accumulation of the other
    S = max(1, args.split)
    streams = [torch.cuda.Stream(device=dev) for _ in range(2 * S)]
    if args.serial:
        streams = [streams[0]] * (2 * S)
    step = make_step(ctx, args.workload, n, bufs, streams, S, args.commit_first)

    units_per_step = B if args.workload == "cfg3" else 2 * B
    units_all = global_batch if args.workload == "cfg3" else 2 * global_batch  # every rank's units per step
    # c = 17 cuts BN254's 254-bit scalars to 15 windows (16 at c = 16: +7.8%
    # measured on one box, profiles/r02_ab_table_layout.json); BLS12-381's
    # 255-bit scalars need 16 windows at either width
    fixed_bits = args.fixed_bits if args.fixed_bits >= 0 else shape["fixed_bits"]

    # ---- secondary legs on the product paths without precompute(): what
    # kzg::trusted_setup::create_commit / create_proof run out of the box
    # ("default": the budget-chosen default table of the first 4097 SRS
    # points, built with the SRS) and with that table off ("pippenger": the
    # table-less path, which allocates nothing beyond the SRS like the
    # reference, src/trusted_setup.cpp:137-142)
    dt = ctx.default_table_info()
    dflt = pip = lat = None
    sec_steps = max(3, min(args.steps, 6))
    if fixed_bits and not args.no_pippenger and dt[0]:
        de, dk, _ = timed_run(ctx, step, streams, sec_steps, 1, world, dist, torch, dev)
        dflt = {"value": units_all * sec_steps / de, "ms_per_step": de / sec_steps * 1e3,
                "msm": "default table, c=%d over %d points (%.2f GB)" % (dt[0], dt[1], dt[2] / 1e9),
                "kernel_ms_per_step": {k: v[0] / sec_steps for k, v in dk.items()}}
    if not args.no_latency and args.workload != "cfg3":
        lat = {"default": latency_leg(ctx, coeffs_h),
               "default_table": {"window_bits": dt[0], "points": dt[1], "bytes": dt[2]}}
    ctx.set_default_table(0)  # off from here on: the main table serves the rest
    if fixed_bits and not args.no_pippenger:
        pe, pk, _ = timed_run(ctx, step, streams, sec_steps, 1, world, dist, torch, dev)
        pip = {"value": units_all * sec_steps / pe, "ms_per_step": pe / sec_steps * 1e3,
               "msm": "pippenger, c=%d, segment %d" % (args.window_bits, args.segment),
               "kernel_ms_per_step": {k: v[0] / sec_steps for k, v in pk.items()}}
    if lat is not None:
        lat["pippenger"] = latency_leg(ctx, coeffs_h)

    setup = None
    if rank == 0 and world == 1 and not args.no_setup and args.workload != "cfg3":
        try:
            setup = setup_leg(kzgx, curve, K, C, tau)
        except Exception as e:  # noqa: BLE001 -- a secondary leg, never fatal for the headline
            setup = {"error": str(e)}
            print("bench: setup leg failed: %s" % e, file=sys.stderr)

    t_setup = time.perf_counter()
    if fixed_bits:
        # precompute the signed-digit multiples of the 4097-point SRS prefix
        # (setup time, like the reference's trusted_setup ctor; not timed)
        fixed_bits = set_fixed_with_fallback(kzgx, ctx, fixed_bits, n)
    t_setup = time.perf_counter() - t_setup
    fb = ctx.fixed_base_info()
    if fb[0] and lat is not None:
        ctx.set_fixed_points_per_thread(0)  # single calls: spread the few MSMs over the GPU
        lat["fixed_table"] = latency_leg(ctx, coeffs_h)
    if fb[0]:
        ctx.set_fixed_points_per_thread(args.fixed_ppt)

    elapsed, kern, local_s = timed_run(ctx, step, streams, args.steps, args.warmup, world, dist, torch, dev)

    # ---- core clock during the step (outside the timed region): a one-wave
    # probe spins on its own stream beside a few more steps (DVFS lowers the
    # clock under this load: profiles/r03_pmc_clock_table_sweep.json) ----
    step_clock = clock_during(ctx, step, elapsed / args.steps, torch, dev)
    ranks = rank_records(world, rank, local, dev, local_s, dist, torch, {"batch": B})
    dinfo = dist_info(world, dist, torch)

    # ---- parity: every output of the last step (oracle identity, MSM-independent) ----
    checked = ok = 0
    bad = None
    if rank == 0:
        checked, ok, bad = check_step(curve, C, tau, args.workload, coeffs_h, zs_h, bufs, w64)

    # ---- throughput vs table size: what a re-linked create_commit gets at
    # each HBM budget (trusted_setup::precompute_budget picks the widest window
    # that fits); c = 0 is Pippenger, the table-less default.  Run after the
    # headline: the amdgpu driver wipes freed VRAM before it hands it out
    # again (~30 GB/s, scripts/probe_alloc.hip, profiles/r06_probe_alloc.jsonl),
    # so a table built right after a larger one was freed waits for that wipe;
    # building the headline table first keeps its setup time the table's own.
    # The curve's own setup_s values after the headline table's release
    # include that wait. ----
    curve_pts = None
    if fixed_bits and not args.no_table_curve:
        curve_pts = [{"window_bits": 0, "gb": 0.0, "value": pip["value"] if pip else None}]
        if fb[0]:
            curve_pts.append({"window_bits": fb[0], "gb": fb[2] / 1e9, "setup_s": t_setup,
                              "value": units_all * args.steps / elapsed})
        ctx.set_fixed_base(0, 0)
        ctx.set_fixed_points_per_thread(args.fixed_ppt)
        for cc in (10, 12, 14, 16):
            if cc >= fixed_bits:
                continue
            tb = time.perf_counter()
            built = set_fixed_with_fallback(kzgx, ctx, cc, n)
            tb = time.perf_counter() - tb
            if built != cc:
                continue
            ce, _, _ = timed_run(ctx, step, streams, 4, 1, world, dist, torch, dev)
            curve_pts.append({"window_bits": cc, "gb": ctx.fixed_base_info()[2] / 1e9, "setup_s": tb,
                              "value": units_all * 4 / ce})
        ctx.set_fixed_base(0, 0)
        curve_pts.sort(key=lambda e: e["window_bits"])

    # ---- CPU baseline (rank 0, N = 1 only) ----
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.cpu_sample > 0:
        import corc
        corc.build()
        srs = corc.gen_srs(curve, tau, n)
        s = args.cpu_sample
        polys = [coeffs_h[0 if args.workload == "cfg3" else i] for i in range(s)]
        tc0 = time.perf_counter()
        nunits = 0
        for i in range(s):
            if args.workload != "cfg3":
                corc.msm_naive(curve, srs, polys[i])  # create_commit
                nunits += 1
            # create_proof(poly, z, 1): evaluate + interpolate + (P - I) / Z in C, then the naive MSM
            q = corc.quotient(curve, corc.limbs_to_ints(polys[i]), int(zs_h[i, 0]), 1)
            corc.msm_naive(curve, srs[: max(len(q), 1)], corc.ints_to_limbs(q, 4))
            nunits += 1
        tcpu = time.perf_counter() - tc0
        # BASELINE configs[0]: degree-128 commit + single-opening proof on the
        # CPU path (benchmark.cpp:40-66 at degree 128; README.md:127 reports
        # 30.1 ms commit / 42.5 ms proof for the reference)
        P128 = coeffs_h[0][:129]
        t128 = time.perf_counter()
        corc.msm_naive(curve, srs[:129], P128)
        t128c = time.perf_counter() - t128
        q128 = corc.quotient(curve, corc.limbs_to_ints(P128), 0, 1)
        corc.msm_naive(curve, srs[: max(len(q128), 1)], corc.ints_to_limbs(q128, 4))
        t128p = time.perf_counter() - t128 - t128c
        cpu_model = platform.processor()
        try:
            with open("/proc/cpuinfo") as f:
                for line in f:
                    if line.startswith("model name"):
                        cpu_model = line.split(":", 1)[1].strip()
                        break
        except OSError:
            pass
        cpu = {
            "value": nunits / tcpu,
            "unit": "commits+proofs/s" if args.workload != "cfg3" else "proofs/s",
            "cores": 1,
            "kind": "port",
            "configs0_degree128": {"commit_ms": t128c * 1e3, "proof_ms": t128p * 1e3,
                                   "reference_published_ms": {"commit": 30.1, "proof": 42.5}},
            "sample": "%d %s at degree %d on the C restatement of the reference path (oracle/kzg_oracle.c: "
                      "naive per-term polyeval_G1 with left-to-right double-and-add scalar multiplication in "
                      "Jacobian coordinates, no GLV; quotient by evaluate + interpolate + long division), "
                      "1 thread, %s, %.1f s" % (
                          nunits, "proofs" if args.workload == "cfg3" else "commits+proofs", degree, cpu_model,
                          tcpu),
        }

    if rank == 0:
        acc_ms, acc_cnt = kern["msm_accum"]
        ms_per_step = elapsed / args.steps * 1e3
        # algorithmic bytes per MSM unit: n (affine point + 32 B scalar) + affine out
        P_b = 2 * w64 * 8
        unit_bytes_commit = n * (P_b + 32) + P_b
        unit_bytes_proof = (n - 1) * (P_b + 32) + P_b
        per_step_bytes = B * unit_bytes_proof + (0 if args.workload == "cfg3" else B * unit_bytes_commit)
        launches_per_step = 1 if args.workload == "cfg3" else 2
        bytes_per_launch = per_step_bytes / launches_per_step
        avg_launch_ms = acc_ms / max(acc_cnt, 1)
        overlapped = not args.serial and launches_per_step > 1
        if not overlapped and acc_cnt:
            # one stream: the accumulation launches are disjoint in time
            assert launches_per_step * avg_launch_ms <= ms_per_step * 1.02, (avg_launch_ms, ms_per_step)
        # achieved: algorithmic bytes of the step / step time -- never a
        # per-launch duration, which the second stream's launch inflates
        achieved = per_step_bytes / (ms_per_step * 1e-3) / 1e9
        if fb[0]:
            wins = (C.r.bit_length() + fb[0] - 1) // fb[0]  # regular odd digits
        else:
            wins = (257 + args.window_bits - 1) // args.window_bits
        # HBM traffic per launch from a counter pass of THIS kernel build
        # (code-object hash), batch and window; null otherwise
        kid = accum_kernel_id(curve, fb[0]) if fb[0] else {"sha256": None}
        tj, tsrc = matching_traffic(args.workload, B, fb[0], kid.get("sha256"))
        traffic = tj.get("msm_accum_bytes_per_launch") if tj else None
        entry_bytes = fb[2] // max(1, wins * fb[1] << (fb[0] - 1)) if fb[0] else 0
        gathered = B * n * wins * entry_bytes  # table entries looked up per launch (B MSMs)
        total_units = units_all * args.steps
        value = total_units / elapsed
        madds = (B * n + (0 if args.workload == "cfg3" else B * n)) * wins
        madd_rate = madds / (ms_per_step * 1e-3)
        peak = None
        mad_peak = None
        mad_ghz = None
        try:
            peak = ctx.microbench_mixed_add()
            mad_peak, mad_ghz = ctx.microbench_mad_u64_clock()
        except Exception as e:  # noqa: BLE001 -- reported, never fatal for the headline
            print("bench: VALU microbenchmarks unavailable: %s" % e, file=sys.stderr)
        L = 9 if curve == "BN254" else 14
        mpa = mads_per_mixed_add(L)
        isa = None
        try:
            import glob
            latest = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_isa_counts.json")))[-1]
            with open(latest) as f:
                isa = json.load(f).get("%s_c%d" % (curve, fb[0]))
            if isa is not None:
                isa = dict(isa, source=os.path.relpath(latest, ROOT))
        except (OSError, ValueError, IndexError):
            isa = None
        line = {
            "metric": "KZG commits/sec + proofs/sec, %s degree-4096" % curve,
            "value": value,
            "unit": "commits+proofs/s" if args.workload != "cfg3" else "proofs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": args.scaling,
            # 0.905 commits/s + 0.925 proofs/s (README.md:132) -> 2 units per 2.185 s
            "vs_baseline": (value / (2.0 / (REF_COMMIT_S + REF_PROOF_S))) if args.workload == "cfg2" else None,
            "dtype": "u32 (radix-2^29 Montgomery limbs, %d-bit Fp)" % (254 if curve == "BN254" else 381),
            "data": "synthetic: seeded uniform Fr coefficients, SRS [tau^i]G1 from fixed tau",
            "config": {
                "workload": {"cfg2": "BN254 degree-4096 commit + single-opening proof, batched",
                             "cfg3": "BN254 degree-4096 poly, batched single-opening proofs at x=0..B-1",
                             "cfg4": "BLS12-381 degree-4096 commit + single-opening proof, batched"}[args.workload],
                "curve": curve,
                "degree": degree,
                "batch_per_gpu": B,
                "global_batch": global_batch,
                "srs_points": 5000,
                "parallelism": "dp%d (independent batches, no collective)" % world,
                "msm": ("fixed-base table, c=%d, %d windows, %.1f GB, %d points/thread" % (
                    fb[0], wins, fb[2] / 1e9, args.fixed_ppt)) if fb[0] else
                       ("pippenger, c=%d, segment %d" % (args.window_bits, args.segment)),
                "streams": 1 if args.serial else 2 * max(1, args.split),
            },
            "roofline": {
                "kernel": "msm_accum",
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "traffic_source": tsrc,
                "traffic_over_algorithmic": traffic / bytes_per_launch if traffic else None,
                "traffic_over_gathered_entries": traffic / gathered if traffic and gathered else None,
                "gathered_entry_bytes_per_launch": gathered or None,
                "kernel_code": kid,
                "algorithmic_bytes_per_step": per_step_bytes,
                "launches_per_step": launches_per_step,
                "avg_launch_ms": avg_launch_ms,
                "achieved_from": "algorithmic bytes per step / ms_per_step" + (
                    " (the commit and proof launches overlap on two streams, so avg_launch_ms is not an isolated "
                    "duration; profiles/*serial* hold the one-stream rocprof run)" if overlapped else ""),
                "note": "integer-VALU bound (no MFMA); see secondary.mad_issue",
            },
            "secondary": {
                "mixed_adds_per_s": madd_rate,
                "kernel_ms_per_step": {k: v[0] / args.steps for k, v in kern.items()},
                "fixed_table_setup_s": t_setup if fb[0] else None,
                "fixed_table_bytes": fb[2] if fb[0] else None,
                "valu_yardstick": None if not peak else {
                    "achieved_mixed_adds_per_s": madd_rate,
                    "yardstick_mixed_adds_per_s": peak,
                    "ratio": madd_rate / peak,
                    "from": "kzgx_microbench_mixed_add: the accumulation loop's XYZZ mixed add on "
                            "register-resident operands at one occupancy, whole GPU, measured live. A yardstick "
                            "of the instruction mix, not a ceiling (BLS12-381 exceeds it): mad_issue is the "
                            "hardware-anchored figure",
                },
                "mad_issue": None if not mad_peak else {
                    "mads_per_mixed_add": mpa,
                    "achieved_mad_lane_ops_per_s": madd_rate * mpa,
                    "peak_mad_lane_ops_per_s": mad_peak,
                    "frac": madd_rate * mpa / mad_peak,
                    "valu_per_mixed_add_isa": isa,
                    "clock_ghz": {"step": step_clock, "peak_run": mad_ghz},
                    "frac_at_step_clock": (madd_rate * mpa / step_clock) / (mad_peak / mad_ghz)
                    if step_clock and mad_ghz else None,
                    "clock_from": "kzgx_clock_probe: one wave counting core clocks against the 100 MHz wall "
                                  "clock, resident beside 4 more steps (outside the timed region); the peak's "
                                  "own launch stamps its clock the same way. The chip lowers its clock under "
                                  "this load (DVFS), so frac_at_step_clock is the issue efficiency at the "
                                  "clock the step actually ran",
                    "peak_from": "kzgx_microbench_mad_u64: v_mad_u64_u32 in asm, 8 independent chains per lane, "
                                 "whole GPU, measured live (the hardware issue ceiling of the instruction every "
                                 "partial product is)",
                },
                "table_curve": curve_pts,
                "default_table": dflt,
                "pippenger": pip,
                "latency": lat,
                "setup_ms": setup,
                "ranks": ranks,
                "dist": dinfo,
            },
            "parity": {"checked": checked, "ok": int(ok), "first_failure": bad,
                       "method": "every output of the last step: commit = [P(tau)]G1, proof = [q(tau)]G1, "
                                 "y = P(z) (C oracle)"},
            "cpu_baseline": cpu,
            "reference_published": {"commit_ms": REF_COMMIT_S * 1e3, "proof_ms": REF_PROOF_S * 1e3,
                                    "multi_proof_ms": {"128": 922.247, "256": 860.305, "512": 810.811,
                                                       "1024": 800.158, "2048": 745.346},
                                    "degree_sweep_ms": {"128": [30.083, 42.504], "256": [55.151, 62.676],
                                                        "512": [136.220, 122.255], "1024": [211.453, 267.592],
                                                        "2048": [445.452, 446.845], "4096": [1104.637, 1080.747]},
                                    "source": "README.md:127-139 (BN254, unstated CPU, 1 thread); "
                                              "throughput equivalent %.3f commits+proofs/s" % (
                                                  2.0 / (REF_COMMIT_S + REF_PROOF_S))},
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()
    ctx.close()


def cfg5_fixed_bits(requested, shard_points):
    """configs[4]'s fixed-base window for one rank's shard: --fixed-bits when
    given (>= 0), else c = 10 for shards of <= 2^18 + 1 points (4 ranks and
    more: 0.44 ms per 131 073-point partial against 0.68 ms table-free,
    0.74 against 1.0 ms at 262 145 points) and 0 (the wide-window Pippenger)
    for larger ones.  set_fixed_with_fallback then steps the window down to
    what fits."""
    if requested >= 0:
        return requested
    return 10 if shard_points <= (1 << 18) + 1 else 0


def run_cfg5(args, world, rank, local, dev, torch, dist, kzgx):
    """configs[4]: one BN254 degree-2^20 commitment sharded over the ranks.
    Each rank owns a contiguous point range with its own SRS slice; the only
    exchange is an all-gather of the partial points, then an exact fold."""
    import kzgx_dist

    K, C = curve_consts("BN254")
    tau = K.default_tau(C)
    n = (1 << 20) + 1
    start, count = kzgx_dist.shard_range(n, world, rank)
    ctx = kzgx.Context("BN254", device=local)
    ctx.set_window_bits(args.window_bits)
    ctx.set_segment(args.segment)
    ctx.set_default_table(0)  # one 2^20-point MSM: its HBM goes to the shard's table
    ctx.gen_srs(tau, max(count, 1), start)
    # Default (round 5): no fixed-base table -- the shard's MSM runs on the
    # wide-window Pippenger path (msm.hip msm_big: c = 16 from 2^18 SRS
    # points, 15 below (BLS12-381: 16); the window table is built with the SRS), which beats
    # the c = 8 table over the whole SRS (2.2 vs 3.05 ms per 2^20 + 1 commit).
    # --fixed-bits N: a fixed-base table over the shard, the widest window
    # whose table fits the free HBM (2^20 points on 1 GPU: c = 8, 274.9 GB;
    # 2^19 on 2: c = 9; 2^18 on 4: c = 10; 2^17 on 8: c = 11), point-major
    # (msm_fixed.hip).  Setup work, outside the timed region.
    # Round 6, automatic choice (no --fixed-bits): a shard of <= 2^18 + 1
    # points (4 ranks and more) gets the fixed-base table over its points at
    # the widest window <= 10 that fits (131 073 points: c = 10, 111.7 GB,
    # 0.44 ms per partial against 0.68 ms on the wide-window path,
    # profiles/r06_shard_fixed.jsonl); larger shards stay table-free (2^20 + 1
    # points: c = 8 would run 3.05 ms against 2.05 ms).
    t_setup = time.perf_counter()
    fixed_bits = cfg5_fixed_bits(args.fixed_bits, count)
    if fixed_bits:
        fixed_bits = set_fixed_with_fallback(kzgx, ctx, fixed_bits, max(count, 1),
                                             budget=args.table_gb * 1e9 if args.table_gb > 0 else None)
    t_setup = time.perf_counter() - t_setup
    rng = np.random.default_rng(0x4B5A47)  # same full polynomial on every rank
    coeffs_h = random_fr(rng, (n,), C.r)
    d_c = torch.from_numpy(coeffs_h[start:start + count].copy().view(np.int64)).to(dev)
    w64 = ctx.w64
    # the partial MSM writes its record in place, RCCL gathers the records
    # into one tensor and one launch folds them -- no stack / cast / cat
    # between the phases (What's weak 4).  Round 6: the record
    # each rank contributes is its partial left projective
    # (one XYZZ point, kzgx_msm_g1_partial_device: no inversion on the rank);
    # kzgx_g1_sum_partials_device adds the gathered records and inverts once,
    # into the packed affine record (x || y || infinity word)
    d_rec = torch.zeros((ctx.partial_record_words,), dtype=torch.int64, device=dev)  # all-zero: the identity
    d_res = torch.zeros((2 * w64 + 1,), dtype=torch.int64, device=dev)
    stream = torch.cuda.Stream(device=dev)

    # Device-resident step: the partial MSM, the RCCL all-gather and the
    # exact fold are all enqueued on one stream; nothing crosses to the host
    # inside a step.
    def partial(s0, cnt):
        if cnt:
            ctx.msm_partial_device(d_c.data_ptr(), cnt, d_rec.data_ptr(), stream.cuda_stream)
        return d_rec

    def fold(recs):
        ctx.g1_sum_partials_device(recs.data_ptr(), recs.shape[0], d_res.data_ptr(), stream.cuda_stream)
        return d_res

    # per-phase HIP events on the step's stream: start, partial MSM enqueued,
    # all-gather done (the collective's completion is ordered before the
    # stream's next work), fold done
    marks = []
    timing = [False]

    def mark(_phase):
        if timing[0]:
            e = torch.cuda.Event(enable_timing=True)
            e.record(stream)
            marks[-1].append(e)

    def step():
        if timing[0]:
            marks.append([])
            mark("start")
        with torch.cuda.stream(stream):
            return kzgx_dist.sharded_commit_tensor(n, world, rank, w64, partial, fold, dist, torch, on_phase=mark)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    timing[0] = True
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = step()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    timing[0] = False
    local_s = elapsed
    # phase times of this rank, mean over the timed steps
    names = ["partial_msm", "all_gather", "fold"]
    phase_tot = [0.0] * 3
    phase_min = [float("inf")] * 3
    phase_max = [0.0] * 3
    for m in marks:
        for k in range(min(3, len(m) - 1)):
            t_k = m[k].elapsed_time(m[k + 1])
            phase_tot[k] += t_k
            phase_min[k] = min(phase_min[k], t_k)
            phase_max[k] = max(phase_max[k], t_k)
    nph = 3  # at world 1: the gather is empty and the fold is the one affine conversion
    my_phases = {names[k]: phase_tot[k] / max(1, len(marks)) for k in range(nph)}
    # per-step extremes, so a slow step (e.g. two ranks time-slicing one
    # device) shows in the record itself
    my_phase_range = {names[k]: [phase_min[k], phase_max[k]] for k in range(nph)}
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ranks = rank_records(world, rank, local, dev, local_s, dist, torch,
                         {"shard_points": count, "phase_ms_per_step": my_phases,
                          "phase_ms_min_max": my_phase_range})
    dinfo = dist_info(world, dist, torch)
    phases = {"rank0": my_phases,
              "max_over_ranks": {k: max(r["phase_ms_per_step"].get(k, 0.0) for r in ranks) for k in my_phases},
              "min_max_over_steps_rank0": my_phase_range,
              "from": "HIP events on the step stream: partial_msm = this rank's shard MSM; all_gather = the "
                      "%s all-gather of the projective partial records (until the stream may use them); fold = "
                      "kzgx_g1_sum_partials_device of the gathered records (the step's one inversion)"
                      % dinfo.get("backend", "no")}
    if rank == 0:
        xys, infs = kzgx_dist.unpack_points(res.cpu().numpy(), w64)
        xy, inf = xys[0], bool(infs[0])
        got = None if inf else (to_int(xy[:4]), to_int(xy[4:8]))
        ptau = 0
        for c in reversed([to_int(r) for r in coeffs_h]):
            ptau = (ptau * tau + c) % C.r
        ok = got == K.scalar_mul(C, (C.gx, C.gy), ptau)
        ms_per_step = elapsed / args.steps * 1e3
        # algorithmic bytes of one commit: n (affine point + 32 B scalar) + affine out
        P_b = 2 * w64 * 8
        unit_bytes = n * (P_b + 32) + P_b
        achieved = unit_bytes / (ms_per_step * 1e-3) / 1e9
        # the table-less window (msm.hip big_window_bits / big_min_points)
        cbig = int(os.environ.get("KZGX_BIG_WINDOW", "0")) or (16 if count >= (1 << 18) else 15)
        cbig = cbig if count >= (1 << 16) else 0
        wins = ((C.r.bit_length() + fixed_bits - 1) // fixed_bits) if fixed_bits else \
            (257 + (cbig or args.window_bits) - 1) // (cbig or args.window_bits)
        madd_rate = n * wins / (ms_per_step * 1e-3)  # all ranks' mixed additions per second
        peak = None
        try:
            peak = ctx.microbench_mixed_add() * world  # measured on this rank's GPU, times the ranks
        except Exception as e:  # noqa: BLE001 -- reported, never fatal for the headline
            print("bench: mixed-add microbenchmark unavailable: %s" % e, file=sys.stderr)
        cpu = None
        if world == 1 and not args.no_cpu_baseline and args.cpu_sample > 0:
            # the naive CPU commit of 2^20 + 1 terms takes minutes, so
            # time the first 2^14 terms and scale linearly (the algorithm is one
            # independent scalar multiplication per term)
            import corc
            corc.build()
            m = 1 << 14
            srs = corc.gen_srs("BN254", tau, m)
            tc0 = time.perf_counter()
            corc.msm_naive("BN254", srs, coeffs_h[:m])
            tcpu = time.perf_counter() - tc0
            cpu = {
                "value": 1.0 / (tcpu * n / m),
                "unit": "commits/s",
                "cores": 1,
                "kind": "port",
                "sample": "first %d of the %d terms of the same commit on the C restatement of polyeval_G1 "
                          "(oracle/kzg_oracle.c: naive per-term double-and-add, no GLV), 1 thread, %.1f s, "
                          "scaled linearly to the full commit" % (m, n, tcpu),
            }
        n_dev = len({r.get("uuid") or r.get("pci") for r in ranks}) or world
        line = {
            "metric": "KZG commits/sec, BN254 degree-2^20, sharded",
            "value": args.steps / elapsed,
            "unit": "commits/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "uint32 limbs (254-bit Montgomery Fp)",
            "data": "synthetic: seeded uniform Fr coefficients, SRS [tau^i]G1 from fixed tau",
            "config": {"workload": "BN254 degree-2^20 commit, point range sharded, device-resident %s" % (
                           "%s all-gather + fold" % dinfo.get("backend") if world > 1 else "single shard (no exchange)"),
                       "n_coeffs": n, "shard_points": count,
                       "msm": ("fixed-base table over the shard, c=%d, %.1f GB" % (
                           fixed_bits, ctx.fixed_base_info()[2] / 1e9)) if fixed_bits else
                              ("wide-window pippenger, c=%d, one MSM (msm.hip msm_big)" % cbig if cbig else
                               "pippenger, c=%d, segment %d, 4096-point chunks" % (args.window_bits, args.segment)),
                       "parallelism": "msm-shard%d" % world},
            "roofline": {
                "kernel": "msm_accum (one MSM per rank) + all-gather + fold",
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS * n_dev,
                "unit": "GB/s",
                "frac": achieved / (HBM_PEAK_GBS * n_dev),
                "traffic": None,
                "distinct_devices": n_dev,
                "algorithmic_bytes_per_step": unit_bytes,
                "achieved_from": "algorithmic bytes of one commit / ms_per_step",
                "note": "integer-VALU bound (no MFMA); see secondary.valu_yardstick",
            },
            "secondary": {
                "fixed_table_setup_s": t_setup,
                "valu_yardstick": None if not peak else {
                    "achieved_mixed_adds_per_s": madd_rate,
                    "yardstick_mixed_adds_per_s": peak,
                    "ratio": madd_rate / peak,
                    "from": "kzgx_microbench_mixed_add on rank 0's GPU x ranks, measured live (a yardstick of "
                            "the instruction mix, not a ceiling)",
                },
                "phase_ms_per_step": phases,
                "ranks": ranks,
                "dist": dinfo,
            },
            "parity": {"checked": 1, "ok": int(ok), "method": "[P(tau)]G1 identity"},
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()
    ctx.close()


def run_common(args, world, rank, local, dev, torch, dist, kzgx):
    """benchmark/benchmark.cpp --benchmark-common (:123-136): one
    10,429,000-point trusted setup (G1 and G2, generated on the GPU; timed as
    setup like the reference's "Finished loading setup"), then for degree =
    1024, 2048, ... <= 10,428,576 the timed regions of benchmark_single_proof
    (:40-66): one create_commit, one create_proof(poly, 0, 1) and one
    verify_proof of that opening, each through the C ABI calls the C++ facade
    makes (host buffers in and out, median of 3).  Coefficients are seeded
    uniform residues instead of an interpolated random string (from_blob is
    outside the reference's timed regions).  Every commitment is checked
    against [P(tau)]G1 (C Horner + scalar multiplication, test
    infrastructure), every opening by verify_proof.  Rank 0 only: one GPU."""
    K, C = curve_consts("BN254")
    import corc  # checker only (oracle/ is on sys.path after curve_consts)

    tau = K.default_tau(C)
    n_setup = 10429000
    ctx = kzgx.Context("BN254", device=local)
    ctx.set_window_bits(args.window_bits)
    t0 = time.perf_counter()
    ctx.gen_srs(tau, n_setup)
    ctx.gen_srs_g2(tau, n_setup)
    ctx.sync()
    setup_s = time.perf_counter() - t0
    rng = np.random.default_rng(0x4B5A47)
    rows = []
    ok_all = True
    degree = 1024
    reps = 3
    while degree <= 10428576:
        n = degree + 1
        P = rng.integers(0, 2**63, size=(n, 4), dtype=np.uint64)
        P[:, 3] &= np.uint64((1 << 59) - 1)  # < 2^251 < r
        z0 = np.zeros((1, 4), dtype=np.uint64)
        commit_ms = median_ms(lambda: ctx.msm(P), reps)
        cxy, cinf = ctx.msm(P)
        proof_ms = median_ms(lambda: ctx.prove_single_batch(P, z0), reps)
        pxy, pinf, y = ctx.prove_single_batch(P, z0)
        verify_ms = median_ms(lambda: ctx.verify_proof(cxy, cinf, pxy[0], bool(pinf[0]), z0, y), reps)
        verified = ctx.verify_proof(cxy, cinf, pxy[0], bool(pinf[0]), z0, y)
        exp = corc.scalar_mul("BN254", (C.gx, C.gy), corc.poly_eval("BN254", P, tau) % C.r)
        got = None if cinf else (to_int(cxy[:4]), to_int(cxy[4:8]))
        ok = verified and got == exp
        ok_all = ok_all and ok
        rows.append({"degree": degree, "commit_ms": commit_ms, "proof_ms": proof_ms, "verify_ms": verify_ms,
                     "commit_ok": got == exp, "verified": verified})
        print("common: degree %8d commit %8.3f ms proof %8.3f ms verify %7.3f ms %s" % (
            degree, commit_ms, proof_ms, verify_ms, "ok" if ok else "MISMATCH"), file=sys.stderr, flush=True)
        degree *= 2
    top = rows[-1]
    line = {
        "metric": "KZG single commit/proof/verify latency, BN254, 10,429,000-point setup (benchmark-common)",
        "value": 1e3 / top["commit_ms"],
        "unit": "commits/s at degree %d" % top["degree"],
        "n_gpus": 1,
        "steps": reps,
        "warmup": 1,
        "ms_per_step": top["commit_ms"],
        "higher_is_better": True,
        "scaling": "none",
        "vs_baseline": None,
        "dtype": "uint32 limbs (254-bit Montgomery Fp)",
        "data": "synthetic: seeded uniform Fr coefficients, SRS [tau^i]G1 / [tau^i]G2 from fixed tau",
        "config": {"workload": "benchmark.cpp --benchmark-common: setup of 10429000 points, degree 1024..8388608",
                   "msm": "pippenger (chunked for n >= 16384), c=%d" % args.window_bits,
                   "host_buffers": True},
        "secondary": {"setup_s": setup_s, "per_degree": rows},
        "parity": {"checked": len(rows), "ok": int(sum(r["commit_ok"] and r["verified"] for r in rows)),
                   "method": "[P(tau)]G1 identity + verify_proof"},
    }
    if rank == 0:
        print(json.dumps(line), flush=True)
    ctx.close()


if __name__ == "__main__":
    sys.exit(main() or 0)
