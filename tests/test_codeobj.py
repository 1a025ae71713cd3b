"""The kernel identity behind roofline.traffic: the bench
attaches a counter pass only when its code-object hash equals the hash of
k_fixed_accum in the loaded libkzgx.so.  CPU only (ELF parsing)."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kzg-commitments_amd", "python"))
LIB = os.path.join(ROOT, "kzg-commitments_amd", "libkzgx.so")


@pytest.mark.skipif(not os.path.exists(LIB), reason="libkzgx.so not built")
@pytest.mark.parametrize("curve,c", [("BN254", 17), ("BN254", 16), ("BLS12381", 16)])
def test_accum_kernel_hash_names_one_kernel(curve, c):
    import codeobj
    h = codeobj.kernel_hash(LIB, *codeobj.fixed_accum_parts(curve, c))
    assert len(h["symbols"]) == 1 and "k_fixed_accum" in h["symbols"][0]
    assert h["sha256"] and len(h["sha256"]) == 64 and h["bytes"] > 1000
    other = codeobj.kernel_hash(LIB, *codeobj.fixed_accum_parts(curve, c - 1))
    assert other["sha256"] != h["sha256"]


def test_traffic_needs_the_same_kernel(tmp_path, monkeypatch):
    sys.path.insert(0, ROOT)
    import bench
    prof = tmp_path / "profiles"
    prof.mkdir()
    (prof / "r99_pmc_traffic_cfg2.json").write_text(json.dumps(
        {"kernel_sha256": "ab" * 32, "batch": 2048, "fixed_bits": 17, "msm_accum_bytes_per_launch": 123}))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    tj, src = bench.matching_traffic("cfg2", 2048, 17, "ab" * 32)
    assert tj["msm_accum_bytes_per_launch"] == 123 and src.endswith("r99_pmc_traffic_cfg2.json")
    assert bench.matching_traffic("cfg2", 2048, 17, "cd" * 32) == (None, None)
    assert bench.matching_traffic("cfg2", 1024, 17, "ab" * 32) == (None, None)
    assert bench.matching_traffic("cfg2", 2048, 17, None) == (None, None)


def test_pc_relative_offsets_do_not_change_the_identity():
    """a call's s_getpc_b64 + s_add_u32 / s_addc_u32 literals move when other
    code moves; they are masked, every other word is kept"""
    import struct
    import codeobj

    def code(lit_lo, lit_hi, tail):
        words = [0xBF800000, 0xBE901C00, 0x8010FF10, lit_lo, 0x8211FF11, lit_hi, tail, 0xBF800000, 0xBF800000]
        return struct.pack("<%dI" % len(words), *words)

    a = codeobj.mask_pc_relative(code(0xFFFFEC9C, 0xFFFFFFFF, 0x7E000280))
    b = codeobj.mask_pc_relative(code(0x00001234, 0x00000000, 0x7E000280))
    c = codeobj.mask_pc_relative(code(0x00001234, 0x00000000, 0x7E000281))
    assert a == b and a != c
