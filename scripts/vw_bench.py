"""Latency of the wave-wide Fp12 ops of the verify path (verify_wave.hip
k_vw_bench via kzgx_debug_vw_bench) and of one verify_proof of a single point
(host buffers, median of 15), both curves.  Prints one JSON line per curve.

    python3 scripts/vw_bench.py"""
import ctypes
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

OPS = ["cyclo_sqr", "mul", "sqr", "mul_line", "frob", "inv", "inv_wave", "csqr_product_ws", "csqr_fold_ws", "csqr_ws"]


def main():
    L = kzgx.lib()
    fn = L.kzgx_debug_vw_bench
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_uint, ctypes.POINTER(ctypes.c_double)]
    for name in ("BN254", "BLS12381"):
        C = K.CURVES[name]
        ctx = kzgx.Context(name)
        try:
            rec = {"curve": name, "op_us": {}, "op_clk": {}}
            for k, op in enumerate(OPS):
                res = (ctypes.c_double * 2)()
                iters = 4 if op.startswith("inv") else 64
                fn(ctx.h, k, iters, res)  # warm
                assert fn(ctx.h, k, iters, res) == 0
                rec["op_us"][op] = res[0] / 1e3
                rec["op_clk"][op] = res[1]
            tau = K.default_tau(C)
            ctx.gen_srs(tau, 4100)
            ctx.gen_srs_g2(tau, 4100)
            P = np.array([[(v >> (64 * i)) & 0xFFFFFFFFFFFFFFFF for i in range(4)]
                          for v in K.random_scalars(C, 4097, 5)], dtype=np.uint64)
            z0 = np.zeros((1, 4), dtype=np.uint64)
            cxy, cinf = ctx.msm(P)
            pxy, pinf, y = ctx.prove_single_batch(P, z0)
            ts = []
            for _ in range(18):
                t0 = time.perf_counter()
                ok = ctx.verify_proof(cxy, cinf, pxy[0], bool(pinf[0]), z0, y)
                ts.append(time.perf_counter() - t0)
                assert ok
            rec["verify_proof_ms_median"] = 1e3 * float(np.median(ts[3:]))
            print(json.dumps(rec), flush=True)
        finally:
            ctx.close()


if __name__ == "__main__":
    main()
