"""Group-cooperative point operations (csrc/coop.hpp) against the lone-lane
forms: P + Q, P + P (the doubling branch), P + (-P) (infinity) and 2Q on
SRS-derived XYZZ points, both curves (kzgx_debug_coop_test)."""
import ctypes

import pytest

import kzg_ref as K

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["BN254", "BLS12381"])
def test_coop_ops_match_lone_lane(name):
    import kzgx
    lib = kzgx.lib()
    fn = lib.kzgx_debug_coop_test
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint)]
    C = K.CURVES[name]
    ctx = kzgx.Context(name)
    try:
        ctx.gen_srs(K.default_tau(C), 3000)
        bad = ctypes.c_uint(0xFFFFFFFF)
        assert fn(ctx.h, ctypes.byref(bad)) == 0
        assert bad.value == 0, f"failing cases mask {bad.value:#x}"
    finally:
        ctx.close()
