"""ctypes binding of oracle/liboracle.so (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it.
Encodings: integers <-> little-endian uint64 limb arrays (numpy)."""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
CURVE_ID = {"BN254": 0, "BLS12381": 1}
BASE_LIMBS = {"BN254": 4, "BLS12381": 6}

_lib = None


def build(force: bool = False) -> str:
    src = [os.path.join(HERE, f) for f in ("kzg_oracle.c", "oracle_field.h")]
    if force or not os.path.exists(LIB_PATH) or any(
            os.path.getmtime(s) > os.path.getmtime(LIB_PATH) for s in src):
        subprocess.check_call(["make", "-s", "-C", HERE, "-B", "liboracle.so"])
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = ctypes.CDLL(LIB_PATH)
        u64p = ctypes.POINTER(ctypes.c_uint64)
        for name, args in {
            "orc_gen_srs": [ctypes.c_int, u64p, ctypes.c_size_t, u64p],
            "orc_msm_naive": [ctypes.c_int, u64p, u64p, ctypes.c_size_t, u64p],
            "orc_scalar_mul": [ctypes.c_int, u64p, u64p, u64p],
            "orc_on_curve": [ctypes.c_int, u64p],
            "orc_poly_eval": [ctypes.c_int, u64p, ctypes.c_size_t, u64p, u64p],
            "orc_interpolate": [ctypes.c_int, u64p, u64p, ctypes.c_size_t, u64p],
            "orc_quotient": [ctypes.c_int, u64p, ctypes.c_size_t, ctypes.c_long, ctypes.c_long,
                             u64p, ctypes.POINTER(ctypes.c_size_t)],
        }.items():
            fn = getattr(_lib, name)
            fn.argtypes = args
            fn.restype = ctypes.c_int
    return _lib


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))


def ints_to_limbs(vals, nl: int) -> np.ndarray:
    out = np.zeros((len(vals), nl), dtype=np.uint64)
    for i, v in enumerate(vals):
        for j in range(nl):
            out[i, j] = (v >> (64 * j)) & 0xFFFFFFFFFFFFFFFF
    return out


def limbs_to_ints(arr) -> list:
    arr = np.asarray(arr, dtype=np.uint64)
    res = []
    if arr.size == 0:
        return res
    for row in arr.reshape(arr.shape[0], -1):
        v = 0
        for j, w in enumerate(row):
            v |= int(w) << (64 * j)
        res.append(v)
    return res


def points_to_array(curve: str, pts) -> np.ndarray:
    nl = BASE_LIMBS[curve]
    out = np.zeros((len(pts), 2 * nl), dtype=np.uint64)
    for i, P in enumerate(pts):
        if P is not None:
            out[i, :nl] = ints_to_limbs([P[0]], nl)[0]
            out[i, nl:] = ints_to_limbs([P[1]], nl)[0]
    return out


def array_to_points(curve: str, arr) -> list:
    nl = BASE_LIMBS[curve]
    arr = np.asarray(arr, dtype=np.uint64).reshape(-1, 2 * nl)
    xs = limbs_to_ints(arr[:, :nl])
    ys = limbs_to_ints(arr[:, nl:])
    return [None if (x == 0 and y == 0) else (x, y) for x, y in zip(xs, ys)]


def gen_srs(curve: str, tau: int, n: int) -> np.ndarray:
    nl = BASE_LIMBS[curve]
    out = np.zeros((n, 2 * nl), dtype=np.uint64)
    t = ints_to_limbs([tau], 4)
    rc = lib().orc_gen_srs(CURVE_ID[curve], _p(t), n, _p(out))
    if rc != 0:
        raise ValueError("orc_gen_srs failed %d" % rc)
    return out


def msm_naive(curve: str, srs: np.ndarray, scalars: np.ndarray):
    """Returns the affine point (x, y) or None (infinity)."""
    nl = BASE_LIMBS[curve]
    srs = np.ascontiguousarray(srs, dtype=np.uint64)
    sc = np.ascontiguousarray(scalars, dtype=np.uint64).reshape(-1, 4)
    out = np.zeros(2 * nl, dtype=np.uint64)
    inf = lib().orc_msm_naive(CURVE_ID[curve], _p(srs), _p(sc), sc.shape[0], _p(out))
    if inf < 0:
        raise ValueError("bad curve")
    return None if inf else array_to_points(curve, out[None, :])[0]


def interpolate(curve: str, xs, ys) -> list:
    n = len(xs)
    X = ints_to_limbs(xs, 4)
    Y = ints_to_limbs(ys, 4)
    out = np.zeros((max(n, 1), 4), dtype=np.uint64)
    rc = lib().orc_interpolate(CURVE_ID[curve], _p(X), _p(Y), n, _p(out))
    if rc != 0:
        raise ZeroDivisionError("duplicate node")
    c = limbs_to_ints(out[:n])
    while c and c[-1] == 0:
        c.pop()
    return c


def quotient(curve: str, coeffs, off: int, length: int) -> list:
    P = ints_to_limbs(coeffs, 4) if coeffs else np.zeros((1, 4), dtype=np.uint64)
    out = np.zeros((max(len(coeffs), 1), 4), dtype=np.uint64)
    nq = ctypes.c_size_t(0)
    rc = lib().orc_quotient(CURVE_ID[curve], _p(P), len(coeffs), off, length, _p(out), ctypes.byref(nq))
    if rc == -2:
        raise ValueError("chunk_length must be 1 or greater")
    if rc != 0:
        raise ZeroDivisionError("quotient failed %d" % rc)
    return limbs_to_ints(out[:nq.value])


def scalar_mul(curve: str, P, k: int):
    """k P for an affine P = (x, y) (None = infinity); the C oracle's
    double-and-add (orc_scalar_mul)."""
    if P is None:
        return None
    nl = BASE_LIMBS[curve]
    xy = points_to_array(curve, [P])[0].copy()
    kk = ints_to_limbs([k], 4)[0].copy()
    out = np.zeros(2 * nl, dtype=np.uint64)
    inf = lib().orc_scalar_mul(CURVE_ID[curve], _p(xy), _p(kk), _p(out))
    if inf < 0:
        raise ValueError("bad curve")
    return None if inf else array_to_points(curve, out[None, :])[0]


def poly_eval(curve: str, coeff_limbs: np.ndarray, x: int) -> int:
    """P(x) mod r by Horner in C; coeff_limbs: n x 4 canonical limbs"""
    P = np.ascontiguousarray(coeff_limbs, dtype=np.uint64).reshape(-1, 4)
    xx = ints_to_limbs([x], 4)[0].copy()
    y = np.zeros(4, dtype=np.uint64)
    lib().orc_poly_eval(CURVE_ID[curve], _p(P), P.shape[0], _p(xx), _p(y))
    return limbs_to_ints(y[None, :])[0]
