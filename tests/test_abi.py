"""CPU tests of the drop-in boundary: libkzgx.so loads and exports every
symbol include/kzg_gpu.h declares; the ctypes binding mirrors the header;
without a gfx950 device the library refuses to run (no CPU fallback)."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "kzg_gpu.h")
LIB = os.path.join(ROOT, "kzg-commitments_amd", "libkzgx.so")


def declared():
    with open(HEADER) as f:
        txt = f.read()
    return sorted(set(re.findall(r"\b(kzgx_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    assert os.path.exists(LIB), "run __graft_entry__.build() first"
    lib = ctypes.CDLL(LIB)
    names = declared()
    assert len(names) >= 20
    for n in names:
        assert hasattr(lib, n), n
    dyn = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True).stdout
    for n in names:
        assert re.search(r"\bT %s\b" % n, dyn), n


def test_python_binding_matches_header():
    import kzgx
    assert sorted(kzgx.EXPORTS) == declared()


def test_strerror_and_constants():
    lib = ctypes.CDLL(LIB)
    lib.kzgx_strerror.restype = ctypes.c_char_p
    assert lib.kzgx_strerror(0) == b"ok"
    assert b"degree" in lib.kzgx_strerror(-5)
    assert lib.kzgx_base_limbs(0) == 4 and lib.kzgx_base_limbs(1) == 6 and lib.kzgx_base_limbs(7) == -1


def test_no_device_means_no_compute():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    import kzgx
    with pytest.raises(kzgx.KzgxError) as e:
        kzgx.Context("BN254")
    assert e.value.status == -7  # KZGX_ERR_NO_DEVICE


def test_init_device_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    import kzgx
    assert kzgx.lib().kzgx_init_device(0, 0) == -7  # KZGX_ERR_NO_DEVICE
    assert kzgx.lib().kzgx_init_device(9, 0) == -1  # unknown curve, before any device query


def test_bad_arguments_rejected_before_device():
    import kzgx
    h = ctypes.c_void_p()
    assert kzgx.lib().kzgx_create(ctypes.byref(h), 9, 0) == -1  # unknown curve
    assert kzgx.lib().kzgx_create(None, 0, 0) == -1


def test_fixed_base_bytes_matches_the_table_layout():
    """kzgx_fixed_base_bytes (host arithmetic, no device): W x n x 2^(c-1)
    entries of 64 B (BN254) / 112 B (BLS12-381), W = ceil((bits(r)+1)/c) --
    the sizes include/kzg.h quotes"""
    import kzgx
    assert kzgx.fixed_base_bytes("BN254", 17, 4097) == 15 * 4097 * (1 << 16) * 64      # 257.8 GB
    assert kzgx.fixed_base_bytes("BN254", 16, 4097) == 16 * 4097 * (1 << 15) * 64      # 137.5 GB
    assert kzgx.fixed_base_bytes("BN254", 12, 4097) == 22 * 4097 * (1 << 11) * 64      # 11.8 GB
    assert kzgx.fixed_base_bytes("BLS12381", 16, 4097) == 16 * 4097 * (1 << 15) * 112  # 240.6 GB
    with pytest.raises(kzgx.KzgxError):
        kzgx.fixed_base_bytes("BN254", 18, 4097)
