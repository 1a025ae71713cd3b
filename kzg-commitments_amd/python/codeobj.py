"""Identify the machine code of one kernel inside libkzgx.so.

Counter passes (rocprofv3 --pmc) are expensive and run on the GPU box; the
bench attaches their result to a line only when the kernel they measured is
the kernel loaded now.  The identity is a SHA-256 over the gfx950 machine
code of the named kernel symbol(s): libkzgx.so's `.hip_fatbin` section holds
one clang offload bundle per translation unit, each with an amdgcn ELF per
target; the kernel's bytes are its symbol's [st_value, st_value + st_size)
in that ELF's .text.  Pure parsing (no HIP call): usable on the CPU, in the
bench, and by the scripts that write profiles/r04_pmc_traffic_*.json.
"""
from __future__ import annotations

import hashlib
import struct

BUNDLE_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _sections(elf: bytes):
    """{name: (offset, size, addr)} of an ELF64 little-endian image"""
    if elf[:4] != b"\x7fELF" or elf[4] != 2:
        raise ValueError("not an ELF64 image")
    shoff, = struct.unpack_from("<Q", elf, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", elf, 0x3A)
    hdrs = []
    for k in range(shnum):
        name, typ, flags, addr, off, size, link, info, align, entsize = struct.unpack_from(
            "<IIQQQQIIQQ", elf, shoff + k * shentsize)
        hdrs.append((name, typ, addr, off, size, link, entsize))
    stroff = hdrs[shstrndx][3]
    out = {}
    for name, typ, addr, off, size, link, entsize in hdrs:
        end = elf.index(b"\0", stroff + name)
        out[elf[stroff + name:end].decode()] = (off, size, addr, typ, link, entsize)
    return out


def device_images(so_path: str, target: str = "gfx950"):
    """the amdgcn ELF images for `target` embedded in a host shared object"""
    with open(so_path, "rb") as f:
        host = f.read()
    secs = _sections(host)
    if ".hip_fatbin" not in secs:
        raise ValueError("%s has no .hip_fatbin section" % so_path)
    off, size = secs[".hip_fatbin"][:2]
    blob = host[off:off + size]
    images = []
    pos = 0
    while True:
        b = blob.find(BUNDLE_MAGIC, pos)
        if b < 0:
            break
        n, = struct.unpack_from("<Q", blob, b + 24)
        p = b + 32
        for _ in range(n):
            eoff, esize, tlen = struct.unpack_from("<QQQ", blob, p)
            triple = blob[p + 24:p + 24 + tlen].decode()
            p += 24 + tlen
            if triple.startswith("hip") and triple.endswith(target) and esize:
                images.append(blob[b + eoff:b + eoff + esize])
        pos = b + len(BUNDLE_MAGIC)
    return images


def kernel_symbols(elf: bytes):
    """[(name, bytes)] of every function symbol with a size in an amdgcn ELF"""
    secs = _sections(elf)
    symoff, symsize, _, _, link, entsize = secs[".symtab"]
    names = list(secs.keys())
    strtab_off = secs[names[link]][0]
    text_off, text_size, text_addr = secs[".text"][:3]
    out = []
    for k in range(symsize // entsize):
        st_name, st_info, st_other, st_shndx, st_value, st_size = struct.unpack_from(
            "<IBBHQQ", elf, symoff + k * entsize)
        if (st_info & 0xF) != 2 or st_size == 0:  # STT_FUNC with a body
            continue
        end = elf.index(b"\0", strtab_off + st_name)
        name = elf[strtab_off + st_name:end].decode()
        lo = text_off + (st_value - text_addr)
        out.append((name, elf[lo:lo + st_size]))
    return out


def mask_pc_relative(code: bytes) -> bytes:
    """the code with the PC-relative offsets of its calls and constant
    addresses zeroed: `s_getpc_b64 s[n:n+1]` (SOP1, op 0x1c) followed by
    `s_add_u32` / `s_addc_u32` with a 32-bit literal (SOP2, src1 = 0xff).
    Those literals move whenever any other function of the code object moves
    (a kernel's calls to its out-of-line rare paths), so without this a change
    elsewhere in the translation unit would change the kernel's identity."""
    b = bytearray(code)
    for i in range(0, len(b) - 20, 4):
        w, = struct.unpack_from("<I", b, i)
        if (w & 0xFF80FF00) != 0xBE801C00:
            continue
        for k in (4, 12):
            w2, = struct.unpack_from("<I", b, i + k)
            if (w2 >> 30) == 2 and ((w2 >> 8) & 0xFF) == 0xFF:
                b[i + k + 4:i + k + 8] = b"\0\0\0\0"
    return bytes(b)


def kernel_hash(so_path: str, *name_parts: str, target: str = "gfx950") -> dict:
    """SHA-256 over the machine code of every function whose mangled name
    contains all of name_parts (sorted by name), with the symbols hashed and
    PC-relative offsets masked (mask_pc_relative)"""
    h = hashlib.sha256()
    found = []
    for img in device_images(so_path, target):
        for name, code in kernel_symbols(img):
            if all(s in name for s in name_parts):
                found.append((name, code))
    found.sort()
    for name, code in found:
        h.update(name.encode() + b"\0")
        h.update(mask_pc_relative(code))
    return {"sha256": h.hexdigest() if found else None, "symbols": [n for n, _ in found],
            "bytes": sum(len(c) for _, c in found), "hash": "sha256 of name + code, PC-relative offsets masked"}


def fixed_accum_parts(curve: str, c: int):
    """name parts selecting exactly k_fixed_accum<curve G1, c, ...> (the
    batched fixed-base accumulation kernel of the throughput lines)"""
    g1 = {"BN254": "7BN254G1", "BLS12381": "10BLS12381G1"}[curve]
    return ("13k_fixed_accumINS_%sELi%dE" % (g1, c),)
