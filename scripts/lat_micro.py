"""Single-lane latency of the tail primitives (kzgx_debug_latency): ns and
core clocks per dependent operation, both curves."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kzg-commitments_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import kzgx  # noqa: E402
import kzg_ref as K  # noqa: E402

lib = kzgx.lib()
lib.kzgx_debug_latency.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_uint, ctypes.POINTER(ctypes.c_double)]
OPS = [("mont_mul", 4000), ("inv_fermat", 40), ("inv_euclid", 40), ("xyzz_add", 400), ("mixed_add", 400),
       ("to_affine", 40), ("inv_euclid_salu", 40), ("to_affine_salu", 40),
       ("inv_euclid_wave", 40), ("to_affine_wave", 40)]
for name, C in [("BN254", K.BN254), ("BLS12381", K.BLS12381)]:
    ctx = kzgx.Context(name, device=0)
    ctx.gen_srs(K.default_tau(C), 4)
    for op, (nm, it) in enumerate(OPS):
        r = (ctypes.c_double * 2)()
        rc = lib.kzgx_debug_latency(ctx.h, op, it, r)
        assert rc == 0, rc
        print(f"{name} {nm:11s} {r[0] / 1e3:9.3f} us {r[1]:11.0f} clk")
    ctx.close()
