#!/usr/bin/env python3
"""Per-kernel register / scratch usage of the built gfx950 code objects.

    python3 scripts/kernel_resources.py [kzg-commitments_amd/build/*.o] [--filter SUBSTR] [--json]

Extracts the device ELF from each object's .hip_fatbin (llvm-objcopy +
clang-offload-bundler) and reads the .num_vgpr / .num_agpr /
.private_seg_size symbols of every kernel.  Scratch (private segment) in a
hot loop means spills; the accumulation kernels must show none (DESIGN.md
section 3)."""
from __future__ import annotations

import argparse
import glob
import json
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def device_elf(obj, tmp):
    fat = os.path.join(tmp, os.path.basename(obj) + ".fatbin")
    elf = os.path.join(tmp, os.path.basename(obj) + ".elf")
    subprocess.run([LLVM + "/llvm-objcopy", "--dump-section=.hip_fatbin=" + fat, obj], check=True,
                   capture_output=True)
    subprocess.run([LLVM + "/clang-offload-bundler", "--unbundle", "--type=o", "--input=" + fat,
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--output=" + elf], check=True, capture_output=True)
    return elf


def resources(elf):
    out = subprocess.run([LLVM + "/llvm-readelf", "-s", elf], check=True, capture_output=True, text=True).stdout
    res = {}
    for ln in out.splitlines():
        m = re.search(r"\s([0-9a-f]+)\s+0\s+NOTYPE\s+LOCAL\s+DEFAULT\s+ABS\s+(\S+)\.(num_vgpr|num_agpr|private_seg_size|numbered_sgpr)$", ln)
        if m:
            res.setdefault(m.group(2), {})[m.group(3)] = int(m.group(1), 16)
    return res


def demangle(names):
    p = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True)
    return p.stdout.splitlines() if p.returncode == 0 else names


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("objs", nargs="*")
    ap.add_argument("--filter", default="")
    ap.add_argument("--json", action="store_true")
    ap.add_argument("--scratch-only", action="store_true")
    a = ap.parse_args()
    objs = a.objs or sorted(glob.glob(os.path.join(os.path.dirname(__file__), "..", "kzg-commitments_amd", "build",
                                                   "*.o")))
    rows = []
    with tempfile.TemporaryDirectory() as tmp:
        for o in objs:
            try:
                elf = device_elf(o, tmp)
            except subprocess.CalledProcessError:
                continue  # host-only object
            for k, v in resources(elf).items():
                rows.append((os.path.basename(o), k, v))
    names = demangle([r[1] for r in rows])
    out = []
    for (o, k, v), dn in zip(rows, names):
        if a.filter and a.filter not in dn:
            continue
        if a.scratch_only and not v.get("private_seg_size"):
            continue
        out.append({"object": o, "kernel": dn, **v})
    if a.json:
        print(json.dumps(out, indent=1))
    else:
        for r in out:
            print("%-14s vgpr %3s agpr %3s sgpr %3s scratch %5s  %s" % (
                r["object"], r.get("num_vgpr"), r.get("num_agpr"), r.get("numbered_sgpr"), r.get("private_seg_size"),
                r["kernel"][:150]))


if __name__ == "__main__":
    sys.exit(main())
