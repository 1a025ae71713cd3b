"""ctypes binding of libkzgx.so (the C ABI in include/kzg_gpu.h).

Host-side plumbing for tests and bench.py: numpy arrays in, numpy arrays out.
There is no fallback: if libkzgx.so is missing or no gfx950 device is visible,
every entry point raises.  Scalars are (n, 4) uint64 arrays (little-endian
limbs, canonical mod r); points are (n, 2 * W64) uint64 arrays (x || y,
canonical), W64 = 4 (BN254) or 6 (BLS12-381), infinity = all zeros.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("KZGX_LIB", os.path.join(PKG_DIR, "libkzgx.so"))
CURVES = {"BN254": 0, "BLS12381": 1}
BASE_LIMBS = {"BN254": 4, "BLS12381": 6}

# exported C symbols (must match include/kzg_gpu.h)
EXPORTS = [
    "kzgx_strerror", "kzgx_base_limbs", "kzgx_init_device", "kzgx_create", "kzgx_destroy", "kzgx_sync", "kzgx_curve",
    "kzgx_srs_size", "kzgx_stream", "kzgx_prof_enable", "kzgx_prof_read", "kzgx_prof_clear", "kzgx_set_window_bits", "kzgx_set_segment",
    "kzgx_set_fixed_base", "kzgx_fixed_base_info", "kzgx_fixed_base_bytes", "kzgx_set_fixed_base_budget",
    "kzgx_set_fixed_base_layout", "kzgx_fixed_base_layout", "kzgx_set_default_table", "kzgx_default_table_info",
    "kzgx_microbench_mad_u64", "kzgx_microbench_mad_u64_clock", "kzgx_clock_probe", "kzgx_set_fixed_points_per_thread", "kzgx_set_small_batch", "kzgx_microbench_mixed_add", "kzgx_load_srs_g1", "kzgx_gen_srs_g1", "kzgx_get_srs_g1", "kzgx_msm_g1",
    "kzgx_msm_g1_batch", "kzgx_msm_g1_batch_device", "kzgx_quotient_single_batch_device",
    "kzgx_prove_single_batch", "kzgx_prove_single_batch_device", "kzgx_prove_range", "kzgx_poly_eval",
    "kzgx_poly_interpolate", "kzgx_poly_vanishing", "kzgx_g1_validate", "kzgx_g1_sum", "kzgx_g1_sum_device", "kzgx_g1_sum_packed_device",
    "kzgx_gen_srs_g2", "kzgx_load_srs_g2", "kzgx_get_srs_g2", "kzgx_srs_g2_size", "kzgx_g2_validate",
    "kzgx_msm_g2", "kzgx_pairing", "kzgx_verify_proof", "kzgx_verify_single_batch",
    "kzgx_verify_single_batch_device", "kzgx_set_verify_wave_max", "kzgx_msm_g1_sharded",
    "kzgx_quotient_single_batch", "kzgx_shared_tables", "kzgx_release_cached_memory",
    "kzgx_partial_record_words", "kzgx_msm_g1_partial_device", "kzgx_g1_sum_partials_device",
]

_lib = None
u64p = ctypes.POINTER(ctypes.c_uint64)
intp = ctypes.POINTER(ctypes.c_int)
vp = ctypes.c_void_p
sz = ctypes.c_size_t


class KzgxError(RuntimeError):
    def __init__(self, status: int, where: str):
        self.status = status
        super().__init__("%s: %s (%d)" % (where, lib().kzgx_strerror(status).decode(), status))


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError("libkzgx.so not built (run __graft_entry__.build())")
        # One HIP runtime per process: PyTorch ships its own libamdhip64 with
        # the same soname as /opt/rocm's.  Loaded first, torch's copy is the
        # one libkzgx.so binds to; loaded second (after libkzgx pulled in
        # /opt/rocm's), torch finds no devices.  Device pointers from torch
        # tensors are then valid in both.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = ctypes.CDLL(LIB_PATH)
        sig = {
            "kzgx_strerror": (ctypes.c_char_p, [ctypes.c_int]),
            "kzgx_base_limbs": (ctypes.c_int, [ctypes.c_int]),
            "kzgx_init_device": (ctypes.c_int, [ctypes.c_int, ctypes.c_int]),
            "kzgx_create": (ctypes.c_int, [ctypes.POINTER(vp), ctypes.c_int, ctypes.c_int]),
            "kzgx_destroy": (None, [vp]),
            "kzgx_sync": (ctypes.c_int, [vp]),
            "kzgx_curve": (ctypes.c_int, [vp]),
            "kzgx_srs_size": (sz, [vp]),
            "kzgx_stream": (vp, [vp]),
            "kzgx_prof_enable": (ctypes.c_int, [vp, ctypes.c_int]),
            "kzgx_prof_read": (ctypes.c_int, [vp, ctypes.c_char_p, ctypes.POINTER(ctypes.c_double), intp]),
            "kzgx_prof_clear": (ctypes.c_int, [vp]),
            "kzgx_set_window_bits": (ctypes.c_int, [vp, ctypes.c_int]),
            "kzgx_set_segment": (ctypes.c_int, [vp, ctypes.c_uint]),
            "kzgx_set_fixed_base": (ctypes.c_int, [vp, ctypes.c_int, sz]),
            "kzgx_fixed_base_info": (ctypes.c_int, [vp, intp, ctypes.POINTER(sz), ctypes.POINTER(sz)]),
            "kzgx_fixed_base_bytes": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, sz, ctypes.POINTER(sz)]),
            "kzgx_set_fixed_base_budget": (ctypes.c_int, [vp, sz, sz, intp]),
            "kzgx_set_fixed_base_layout": (ctypes.c_int, [vp, ctypes.c_int]),
            "kzgx_set_default_table": (ctypes.c_int, [vp, ctypes.c_int, sz]),
            "kzgx_default_table_info": (ctypes.c_int, [vp, intp, ctypes.POINTER(sz), ctypes.POINTER(sz)]),
            "kzgx_fixed_base_layout": (ctypes.c_int, [vp, intp]),
            "kzgx_microbench_mad_u64": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_double)]),
            "kzgx_microbench_mad_u64_clock": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_double),
                                                             ctypes.POINTER(ctypes.c_double)]),
            "kzgx_clock_probe": (ctypes.c_int, [vp, vp, ctypes.c_uint, vp]),
            "kzgx_set_fixed_points_per_thread": (ctypes.c_int, [vp, ctypes.c_uint]),
            "kzgx_set_small_batch": (ctypes.c_int, [vp, ctypes.c_uint]),
            "kzgx_microbench_mixed_add": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_double)]),
            "kzgx_load_srs_g1": (ctypes.c_int, [vp, u64p, sz]),
            "kzgx_gen_srs_g1": (ctypes.c_int, [vp, u64p, sz, sz]),
            "kzgx_get_srs_g1": (ctypes.c_int, [vp, u64p, sz]),
            "kzgx_msm_g1": (ctypes.c_int, [vp, u64p, sz, u64p, intp]),
            "kzgx_msm_g1_batch": (ctypes.c_int, [vp, u64p, sz, sz, u64p, intp]),
            "kzgx_msm_g1_batch_device": (ctypes.c_int, [vp, vp, sz, sz, sz, vp, vp, vp]),
            "kzgx_quotient_single_batch_device": (ctypes.c_int, [vp, vp, sz, sz, vp, sz, vp, sz, vp, vp]),
            "kzgx_prove_single_batch": (ctypes.c_int, [vp, u64p, sz, sz, u64p, sz, u64p, intp, u64p]),
            "kzgx_prove_single_batch_device": (ctypes.c_int, [vp, vp, sz, sz, vp, sz, vp, vp, vp, vp]),
            "kzgx_prove_range": (ctypes.c_int, [vp, u64p, sz, u64p, sz, u64p, intp]),
            "kzgx_poly_eval": (ctypes.c_int, [vp, u64p, sz, u64p, sz, u64p]),
            "kzgx_poly_interpolate": (ctypes.c_int, [vp, u64p, u64p, sz, u64p]),
            "kzgx_poly_vanishing": (ctypes.c_int, [vp, u64p, sz, u64p]),
            "kzgx_g1_validate": (ctypes.c_int, [vp, u64p, intp]),
            "kzgx_g1_sum": (ctypes.c_int, [vp, u64p, intp, sz, u64p, intp]),
            "kzgx_g1_sum_device": (ctypes.c_int, [vp, vp, vp, sz, vp, vp, vp]),
            "kzgx_g1_sum_packed_device": (ctypes.c_int, [vp, vp, sz, vp, vp]),
            "kzgx_gen_srs_g2": (ctypes.c_int, [vp, u64p, sz, sz]),
            "kzgx_load_srs_g2": (ctypes.c_int, [vp, u64p, sz]),
            "kzgx_get_srs_g2": (ctypes.c_int, [vp, u64p, sz]),
            "kzgx_srs_g2_size": (sz, [vp]),
            "kzgx_g2_validate": (ctypes.c_int, [vp, u64p, sz, intp]),
            "kzgx_msm_g2": (ctypes.c_int, [vp, u64p, sz, u64p, intp]),
            "kzgx_pairing": (ctypes.c_int, [vp, u64p, intp, u64p, intp, sz, u64p]),
            "kzgx_verify_proof": (ctypes.c_int, [vp, u64p, ctypes.c_int, u64p, ctypes.c_int, u64p, u64p, sz, intp]),
            "kzgx_verify_single_batch": (ctypes.c_int, [vp, u64p, intp, u64p, intp, u64p, u64p, sz, intp]),
            "kzgx_verify_single_batch_device": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, vp, sz, vp, vp]),
            "kzgx_set_verify_wave_max": (ctypes.c_int, [vp, sz]),
            "kzgx_quotient_single_batch": (ctypes.c_int, [vp, u64p, sz, sz, u64p, sz, u64p, u64p]),
            "kzgx_msm_g1_sharded": (ctypes.c_int, [ctypes.POINTER(vp), ctypes.POINTER(sz), sz, u64p, sz, u64p, intp]),
            "kzgx_shared_tables": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(sz), ctypes.POINTER(sz)]),
            "kzgx_release_cached_memory": (ctypes.c_int, [ctypes.c_int]),
            "kzgx_partial_record_words": (ctypes.c_int, [ctypes.c_int]),
            "kzgx_msm_g1_partial_device": (ctypes.c_int, [vp, vp, sz, vp, vp]),
            "kzgx_g1_sum_partials_device": (ctypes.c_int, [vp, vp, sz, vp, vp]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(u64p)


def _chk(rc, where):
    if rc != 0:
        raise KzgxError(rc, where)


def as_scalars(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.uint64).reshape(-1, 4)


def msm_g1_sharded(ctxs, starts, scalars):
    """kzgx_msm_g1_sharded: one commitment over contexts holding contiguous SRS
    slices (context k's slice starts at point starts[k]); -> (xy, is_inf)"""
    sc = as_scalars(scalars)
    n = sc.shape[0]
    hs = (vp * len(ctxs))(*[c.h for c in ctxs])
    st = (sz * len(ctxs))(*starts)
    out = np.zeros(2 * ctxs[0].w64, dtype=np.uint64)
    oi = ctypes.c_int(0)
    _chk(lib().kzgx_msm_g1_sharded(hs, st, len(ctxs), _p(sc) if n else None, n, _p(out), ctypes.byref(oi)),
         "kzgx_msm_g1_sharded")
    return out, bool(oi.value)


def init_device(curve: str, device: int):
    """kzgx_init_device: HIP, every code object and the generator tables, once
    per (curve, device)."""
    _chk(lib().kzgx_init_device(CURVES[curve], device), "kzgx_init_device")


def shared_tables(device: int = 0):
    """kzgx_shared_tables: (count, bytes) of the default tables shared on a device"""
    c, b = sz(0), sz(0)
    _chk(lib().kzgx_shared_tables(device, ctypes.byref(c), ctypes.byref(b)), "kzgx_shared_tables")
    return c.value, b.value


def release_cached_memory(device: int = 0):
    """kzgx_release_cached_memory: hand the device's cached table block back"""
    _chk(lib().kzgx_release_cached_memory(device), "kzgx_release_cached_memory")


def fixed_base_bytes(curve: str, c: int, n_points: int) -> int:
    """device bytes of a fixed-base table (host arithmetic, no device)"""
    b = sz(0)
    _chk(lib().kzgx_fixed_base_bytes(CURVES[curve], c, n_points, ctypes.byref(b)), "kzgx_fixed_base_bytes")
    return b.value


class Context:
    """One device context (SRS + stream + workspaces), kzgx_ctx*."""

    def __init__(self, curve: str = "BN254", device: int = 0):
        self.curve = curve
        self.w64 = BASE_LIMBS[curve]
        h = vp()
        _chk(lib().kzgx_create(ctypes.byref(h), CURVES[curve], device), "kzgx_create")
        self.h = h
        self.device = device

    def set_default_table(self, c: int, n_points: int = 4097):
        """kzgx_set_default_table: c = -1 the budget-chosen window, 0 off"""
        _chk(lib().kzgx_set_default_table(self.h, c, n_points if c else 0), "kzgx_set_default_table")

    def default_table_info(self):
        c, n, b = ctypes.c_int(0), ctypes.c_size_t(0), ctypes.c_size_t(0)
        _chk(lib().kzgx_default_table_info(self.h, ctypes.byref(c), ctypes.byref(n), ctypes.byref(b)),
             "kzgx_default_table_info")
        return c.value, n.value, b.value

    def debug_ws_read(self, name: str, nbytes: int) -> np.ndarray:
        """bytes of one workspace buffer of the context stream (test hook:
        kzgx_debug_ws_read, declared outside kzg_gpu.h)"""
        L = lib()
        fn = L.kzgx_debug_ws_read
        fn.restype = ctypes.c_int
        fn.argtypes = [vp, ctypes.c_char_p, vp, sz]
        a = np.zeros(nbytes, dtype=np.uint8)
        _chk(fn(self.h, name.encode(), a.ctypes.data, nbytes), "kzgx_debug_ws_read")
        return a

    def close(self):
        if getattr(self, "h", None):
            lib().kzgx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def stream(self) -> int:
        return lib().kzgx_stream(self.h)

    def sync(self):
        _chk(lib().kzgx_sync(self.h), "kzgx_sync")

    def prof_enable(self, on: bool = True):
        _chk(lib().kzgx_prof_enable(self.h, 1 if on else 0), "kzgx_prof_enable")

    def prof_read(self, name: str):
        ms = ctypes.c_double(0)
        cnt = ctypes.c_int(0)
        _chk(lib().kzgx_prof_read(self.h, name.encode(), ctypes.byref(ms), ctypes.byref(cnt)), "kzgx_prof_read")
        return ms.value, cnt.value

    def set_window_bits(self, c: int):
        _chk(lib().kzgx_set_window_bits(self.h, c), "kzgx_set_window_bits")

    def set_small_batch(self, max_batch: int):
        """table-less batches of <= max_batch MSMs use the window-10 table (0 = never)"""
        _chk(lib().kzgx_set_small_batch(self.h, max_batch), "kzgx_set_small_batch")

    def set_segment(self, k: int):
        _chk(lib().kzgx_set_segment(self.h, k), "kzgx_set_segment")

    def set_fixed_base(self, c: int, n_points: int = 0):
        """Precompute the signed-digit multiples table for the first n_points
        SRS points (c = 0: off).  Built now if an SRS is installed."""
        _chk(lib().kzgx_set_fixed_base(self.h, c, n_points), "kzgx_set_fixed_base")

    def set_fixed_base_layout(self, layout: int):
        """-1 automatic, 0 window-major, 1 point-major (next table build)"""
        _chk(lib().kzgx_set_fixed_base_layout(self.h, layout), "kzgx_set_fixed_base_layout")

    def fixed_base_point_major(self) -> bool:
        pm = ctypes.c_int(0)
        _chk(lib().kzgx_fixed_base_layout(self.h, ctypes.byref(pm)), "kzgx_fixed_base_layout")
        return bool(pm.value)

    def fixed_base_info(self):
        c = ctypes.c_int(0)
        n = sz(0)
        b = sz(0)
        _chk(lib().kzgx_fixed_base_info(self.h, ctypes.byref(c), ctypes.byref(n), ctypes.byref(b)),
             "kzgx_fixed_base_info")
        return c.value, n.value, b.value

    def set_fixed_base_budget(self, budget_bytes: int, n_points: int) -> int:
        """widest table window whose table fits budget_bytes and free device
        memory (0: none built, Pippenger); returns the window built"""
        c = ctypes.c_int(0)
        _chk(lib().kzgx_set_fixed_base_budget(self.h, int(budget_bytes), n_points, ctypes.byref(c)),
             "kzgx_set_fixed_base_budget")
        return c.value

    def microbench_mad_u64(self) -> float:
        """v_mad_u64_u32 lane operations / s (hardware issue ceiling)"""
        r = ctypes.c_double(0)
        _chk(lib().kzgx_microbench_mad_u64(self.h, ctypes.byref(r)), "kzgx_microbench_mad_u64")
        return r.value

    def microbench_mad_u64_clock(self):
        """(v_mad_u64_u32 lane operations / s, core GHz the ceiling ran at)"""
        r = ctypes.c_double(0)
        g = ctypes.c_double(0)
        _chk(lib().kzgx_microbench_mad_u64_clock(self.h, ctypes.byref(r), ctypes.byref(g)),
             "kzgx_microbench_mad_u64_clock")
        return r.value, g.value

    def clock_probe(self, d_out: int, spin_us: int, stream: int = 0):
        """enqueue the core-clock probe on stream; d_out: device address of 3 uint64"""
        _chk(lib().kzgx_clock_probe(self.h, ctypes.c_void_p(stream or None), spin_us, ctypes.c_void_p(d_out)),
             "kzgx_clock_probe")

    def set_fixed_points_per_thread(self, p: int):
        _chk(lib().kzgx_set_fixed_points_per_thread(self.h, p), "kzgx_set_fixed_points_per_thread")

    def microbench_mixed_add(self) -> float:
        """mixed additions / s of the accumulation loop at full occupancy"""
        r = ctypes.c_double(0)
        _chk(lib().kzgx_microbench_mixed_add(self.h, ctypes.byref(r)), "kzgx_microbench_mixed_add")
        return r.value

    def prof_clear(self):
        _chk(lib().kzgx_prof_clear(self.h), "kzgx_prof_clear")

    # ---- SRS ----
    @property
    def srs_size(self) -> int:
        return lib().kzgx_srs_size(self.h)

    def load_srs(self, xy: np.ndarray):
        xy = np.ascontiguousarray(xy, dtype=np.uint64).reshape(-1, 2 * self.w64)
        _chk(lib().kzgx_load_srs_g1(self.h, _p(xy), xy.shape[0]), "kzgx_load_srs_g1")

    def gen_srs(self, tau: int, n: int, start: int = 0):
        t = np.array([(tau >> (64 * i)) & 0xFFFFFFFFFFFFFFFF for i in range(4)], dtype=np.uint64)
        _chk(lib().kzgx_gen_srs_g1(self.h, _p(t), start, n), "kzgx_gen_srs_g1")

    def get_srs(self, n: int | None = None) -> np.ndarray:
        n = self.srs_size if n is None else n
        out = np.zeros((n, 2 * self.w64), dtype=np.uint64)
        _chk(lib().kzgx_get_srs_g1(self.h, _p(out), n), "kzgx_get_srs_g1")
        return out

    # ---- MSM ----
    def msm_batch(self, scalars: np.ndarray, n: int, batch: int):
        sc = np.ascontiguousarray(scalars, dtype=np.uint64).reshape(-1)
        assert sc.size >= n * batch * 4
        out = np.zeros((batch, 2 * self.w64), dtype=np.uint64)
        inf = np.zeros(batch, dtype=np.int32)
        _chk(lib().kzgx_msm_g1_batch(self.h, _p(sc) if n else None, n, batch, _p(out),
                                     inf.ctypes.data_as(intp)), "kzgx_msm_g1_batch")
        return out, inf.astype(bool)

    def msm(self, scalars: np.ndarray):
        sc = as_scalars(scalars)
        out, inf = self.msm_batch(sc, sc.shape[0], 1)
        return out[0], bool(inf[0])

    def quotient_single_batch(self, coeffs, zs, shared: bool = True):
        """q_j = (P_j - P_j(z_j)) / (X - z_j) and y_j = P_j(z_j) (host buffers);
        coeffs: n x 4 (shared) or batch x n x 4 words -> (q: batch x (n-1) x 4, y: batch x 4)"""
        c = np.ascontiguousarray(coeffs, dtype=np.uint64)
        z = as_scalars(zs)
        batch = z.shape[0]
        n = c.shape[-2] if c.ndim == 3 else c.reshape(-1, 4).shape[0]
        stride = 0 if shared else n
        q = np.zeros((batch, max(n - 1, 0), 4), dtype=np.uint64)
        y = np.zeros((batch, 4), dtype=np.uint64)
        _chk(lib().kzgx_quotient_single_batch(self.h, _p(c) if n else None, n, stride, _p(z), batch,
                                              _p(q) if n > 1 else None, _p(y)), "kzgx_quotient_single_batch")
        return q, y

    def msm_batch_device(self, d_scalars: int, n: int, batch: int, stride: int, d_out: int, d_inf: int,
                         stream: int | None = None):
        _chk(lib().kzgx_msm_g1_batch_device(self.h, d_scalars, n, batch, stride, d_out, d_inf, stream),
             "kzgx_msm_g1_batch_device")

    # ---- proofs ----
    def prove_single_batch(self, coeffs: np.ndarray, zs: np.ndarray, shared: bool = True):
        """coeffs: (n, 4) shared polynomial (shared=True) or (batch, n, 4)."""
        zs = as_scalars(zs)
        batch = zs.shape[0]
        c = np.ascontiguousarray(coeffs, dtype=np.uint64)
        n = c.shape[-2] if c.ndim >= 2 else 0
        stride = 0 if shared else n
        out = np.zeros((batch, 2 * self.w64), dtype=np.uint64)
        inf = np.zeros(batch, dtype=np.int32)
        y = np.zeros((batch, 4), dtype=np.uint64)
        _chk(lib().kzgx_prove_single_batch(self.h, _p(c) if n else None, n, stride, _p(zs), batch, _p(out),
                                           inf.ctypes.data_as(intp), _p(y)), "kzgx_prove_single_batch")
        return out, inf.astype(bool), y

    def prove_single_batch_device(self, d_coeffs, n, stride, d_z, batch, d_out, d_inf, d_y=None, stream=None):
        _chk(lib().kzgx_prove_single_batch_device(self.h, d_coeffs, n, stride, d_z, batch, d_out, d_inf, d_y,
                                                  stream), "kzgx_prove_single_batch_device")

    def quotient_single_device(self, d_coeffs, n, stride, d_z, batch, d_q, q_stride, d_y=None, stream=None):
        _chk(lib().kzgx_quotient_single_batch_device(self.h, d_coeffs, n, stride, d_z, batch, d_q, q_stride, d_y,
                                                     stream), "kzgx_quotient_single_batch_device")

    def prove_range(self, coeffs: np.ndarray, xs: np.ndarray):
        """multi-point opening: MSM of (P - I) / Z for the points xs"""
        c = as_scalars(coeffs) if len(coeffs) else np.zeros((0, 4), dtype=np.uint64)
        x = as_scalars(xs)
        out = np.zeros(2 * self.w64, dtype=np.uint64)
        inf = ctypes.c_int(0)
        _chk(lib().kzgx_prove_range(self.h, _p(c) if c.shape[0] else None, c.shape[0], _p(x), x.shape[0], _p(out),
                                    ctypes.byref(inf)), "kzgx_prove_range")
        return out, bool(inf.value)

    # ---- poly ----
    def poly_eval(self, coeffs: np.ndarray, xs: np.ndarray) -> np.ndarray:
        c = as_scalars(coeffs) if len(coeffs) else np.zeros((0, 4), dtype=np.uint64)
        x = as_scalars(xs)
        y = np.zeros_like(x)
        _chk(lib().kzgx_poly_eval(self.h, _p(c) if c.shape[0] else None, c.shape[0], _p(x), x.shape[0], _p(y)),
             "kzgx_poly_eval")
        return y

    def interpolate(self, xs: np.ndarray, ys: np.ndarray) -> np.ndarray:
        x = as_scalars(xs)
        y = as_scalars(ys)
        out = np.zeros_like(x)
        _chk(lib().kzgx_poly_interpolate(self.h, _p(x), _p(y), x.shape[0], _p(out)), "kzgx_poly_interpolate")
        return out

    def vanishing(self, xs: np.ndarray) -> np.ndarray:
        x = as_scalars(xs)
        out = np.zeros((x.shape[0] + 1, 4), dtype=np.uint64)
        _chk(lib().kzgx_poly_vanishing(self.h, _p(x) if x.shape[0] else None, x.shape[0], _p(out)),
             "kzgx_poly_vanishing")
        return out

    def g1_validate(self, xy: np.ndarray) -> bool:
        xy = np.ascontiguousarray(xy, dtype=np.uint64).reshape(2 * self.w64)
        ok = ctypes.c_int(0)
        _chk(lib().kzgx_g1_validate(self.h, _p(xy), ctypes.byref(ok)), "kzgx_g1_validate")
        return bool(ok.value)

    def g1_sum(self, pts: np.ndarray, inf=None):
        pts = np.ascontiguousarray(pts, dtype=np.uint64).reshape(-1, 2 * self.w64)
        f = None if inf is None else np.ascontiguousarray(inf, dtype=np.int32)
        out = np.zeros(2 * self.w64, dtype=np.uint64)
        oi = ctypes.c_int(0)
        _chk(lib().kzgx_g1_sum(self.h, _p(pts), None if f is None else f.ctypes.data_as(intp), pts.shape[0],
                               _p(out), ctypes.byref(oi)), "kzgx_g1_sum")
        return out, bool(oi.value)

    def g1_sum_device(self, d_xy: int, d_inf: int | None, count: int, d_out: int, d_out_inf: int,
                      stream: int | None = None):
        """Fold of count device-resident canonical points (uint32 infinity flags) on stream."""
        _chk(lib().kzgx_g1_sum_device(self.h, d_xy, d_inf, count, d_out, d_out_inf, stream), "kzgx_g1_sum_device")

    def g1_sum_packed_device(self, d_rec: int, count: int, d_out: int, stream: int | None = None):
        """Fold of count packed records (2 W64 uint64 x || y, then a uint64 infinity word) into one
        record at d_out, on stream (the sharded commitment's exchange format)."""
        _chk(lib().kzgx_g1_sum_packed_device(self.h, d_rec, count, d_out, stream), "kzgx_g1_sum_packed_device")

    @property
    def partial_record_words(self) -> int:
        """uint64 words of one projective partial record (kzgx_partial_record_words)"""
        return lib().kzgx_partial_record_words(CURVES[self.curve])

    def msm_partial_device(self, d_scalars: int, n: int, d_rec: int, stream: int | None = None):
        """kzgx_msm_g1_partial_device: sum_i s_i SRS_i as one XYZZ record at d_rec (no inversion)."""
        _chk(lib().kzgx_msm_g1_partial_device(self.h, d_scalars, n, d_rec, stream), "kzgx_msm_g1_partial_device")

    def g1_sum_partials_device(self, d_rec: int, count: int, d_out: int, stream: int | None = None):
        """kzgx_g1_sum_partials_device: count XYZZ records -> one packed affine record at d_out."""
        _chk(lib().kzgx_g1_sum_partials_device(self.h, d_rec, count, d_out, stream), "kzgx_g1_sum_partials_device")

    def init_device(self):
        """kzgx_init_device for this context's curve and device (ADVICE r05:
        the module-level init_device(curve, device) takes them explicitly)."""
        init_device(self.curve, self.device)

    # ---- verify half: G2 setup, polyeval_G2, pairing ----
    # G2 points: (n, 4 * W64) uint64 = x.re || x.im || y.re || y.im; Fp12: (12 * W64,)
    @property
    def srs2_size(self) -> int:
        return lib().kzgx_srs_g2_size(self.h)

    def gen_srs_g2(self, tau: int, n: int, start: int = 0):
        t = np.array([(tau >> (64 * i)) & 0xFFFFFFFFFFFFFFFF for i in range(4)], dtype=np.uint64)
        _chk(lib().kzgx_gen_srs_g2(self.h, _p(t), start, n), "kzgx_gen_srs_g2")

    def load_srs_g2(self, xy: np.ndarray):
        xy = np.ascontiguousarray(xy, dtype=np.uint64).reshape(-1, 4 * self.w64)
        _chk(lib().kzgx_load_srs_g2(self.h, _p(xy), xy.shape[0]), "kzgx_load_srs_g2")

    def get_srs_g2(self, n: int | None = None) -> np.ndarray:
        n = self.srs2_size if n is None else n
        out = np.zeros((n, 4 * self.w64), dtype=np.uint64)
        _chk(lib().kzgx_get_srs_g2(self.h, _p(out), n), "kzgx_get_srs_g2")
        return out

    def g2_validate(self, xy: np.ndarray) -> np.ndarray:
        xy = np.ascontiguousarray(xy, dtype=np.uint64).reshape(-1, 4 * self.w64)
        ok = np.zeros(xy.shape[0], dtype=np.int32)
        _chk(lib().kzgx_g2_validate(self.h, _p(xy), xy.shape[0], ok.ctypes.data_as(intp)), "kzgx_g2_validate")
        return ok.astype(bool)

    def msm_g2(self, scalars: np.ndarray):
        sc = as_scalars(scalars) if len(scalars) else np.zeros((0, 4), dtype=np.uint64)
        out = np.zeros(4 * self.w64, dtype=np.uint64)
        inf = ctypes.c_int(0)
        _chk(lib().kzgx_msm_g2(self.h, _p(sc) if sc.shape[0] else None, sc.shape[0], _p(out), ctypes.byref(inf)),
             "kzgx_msm_g2")
        return out, bool(inf.value)

    def pairing(self, g1: np.ndarray, g2: np.ndarray, g1_inf=None, g2_inf=None) -> np.ndarray:
        a = np.ascontiguousarray(g1, dtype=np.uint64).reshape(-1, 2 * self.w64)
        b = np.ascontiguousarray(g2, dtype=np.uint64).reshape(-1, 4 * self.w64)
        assert a.shape[0] == b.shape[0]
        fa = None if g1_inf is None else np.ascontiguousarray(g1_inf, dtype=np.int32)
        fb = None if g2_inf is None else np.ascontiguousarray(g2_inf, dtype=np.int32)
        out = np.zeros((a.shape[0], 12 * self.w64), dtype=np.uint64)
        _chk(lib().kzgx_pairing(self.h, _p(a), None if fa is None else fa.ctypes.data_as(intp), _p(b),
                                None if fb is None else fb.ctypes.data_as(intp), a.shape[0], _p(out)),
             "kzgx_pairing")
        return out

    def verify_proof(self, commit, commit_inf: bool, proof, proof_inf: bool, xs, ys) -> bool:
        c = np.ascontiguousarray(commit, dtype=np.uint64).reshape(2 * self.w64)
        p = np.ascontiguousarray(proof, dtype=np.uint64).reshape(2 * self.w64)
        x = as_scalars(xs) if len(xs) else np.zeros((0, 4), dtype=np.uint64)
        y = as_scalars(ys) if len(ys) else np.zeros((0, 4), dtype=np.uint64)
        ok = ctypes.c_int(0)
        _chk(lib().kzgx_verify_proof(self.h, _p(c), int(commit_inf), _p(p), int(proof_inf),
                                     _p(x) if x.shape[0] else None, _p(y) if y.shape[0] else None, x.shape[0],
                                     ctypes.byref(ok)), "kzgx_verify_proof")
        return bool(ok.value)

    def verify_single_batch(self, commits, proofs, zs, ys, commit_inf=None, proof_inf=None) -> np.ndarray:
        c = np.ascontiguousarray(commits, dtype=np.uint64).reshape(-1, 2 * self.w64)
        p = np.ascontiguousarray(proofs, dtype=np.uint64).reshape(-1, 2 * self.w64)
        z, y = as_scalars(zs), as_scalars(ys)
        n = c.shape[0]
        assert p.shape[0] == n and z.shape[0] == n and y.shape[0] == n
        fc = None if commit_inf is None else np.ascontiguousarray(commit_inf, dtype=np.int32)
        fp = None if proof_inf is None else np.ascontiguousarray(proof_inf, dtype=np.int32)
        ok = np.zeros(n, dtype=np.int32)
        _chk(lib().kzgx_verify_single_batch(self.h, _p(c), None if fc is None else fc.ctypes.data_as(intp), _p(p),
                                            None if fp is None else fp.ctypes.data_as(intp), _p(z), _p(y), n,
                                            ok.ctypes.data_as(intp)), "kzgx_verify_single_batch")
        return ok.astype(bool)

    def set_verify_wave_max(self, max_count: int) -> None:
        """batches of <= max_count openings run a wave per opening (0: a lane each)"""
        _chk(lib().kzgx_set_verify_wave_max(self.h, max_count), "kzgx_set_verify_wave_max")

    def verify_single_batch_device(self, d_commits, d_commit_inf, d_proofs, d_proof_inf, d_z, d_y, count, d_ok,
                                   stream=None):
        _chk(lib().kzgx_verify_single_batch_device(self.h, d_commits, d_commit_inf, d_proofs, d_proof_inf, d_z, d_y,
                                                   count, d_ok, stream), "kzgx_verify_single_batch_device")
