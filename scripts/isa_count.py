#!/usr/bin/env python3
"""Count the VALU instructions of a kernel's hot loop in gfx950 assembly.

    hipcc -O3 -std=c++17 --offload-arch=gfx950 --cuda-device-only -S -o x.s csrc/msm_fixed.hip
    python3 scripts/isa_count.py x.s 'k_fixed_accumINS_7BN254G1ELi17E' [--per N]

Finds the kernel whose symbol contains the given substring, then the loop
(a backward branch to an earlier label) holding the most v_mad_u64_u32, and
prints a histogram of the instructions between that label and the branch.
Loop bodies of the accumulation kernels hold one mixed addition on the common
path plus the rare special cases (doubling, infinity), so the script also
reports the counts of the straight-line blocks on the fall-through path
(`--path`): from the loop head, follow fall-through and forward branches'
not-taken edges to the back edge.  --per N divides the totals by N (e.g. the
number of mixed additions per iteration).

Used for bench.py's secondary.mad_issue (v_mad_u64_u32 per mixed addition)
and DESIGN.md section 7:

    python3 scripts/isa_count.py --profile profiles/r03_isa_counts.json
"""
from __future__ import annotations

import argparse
import collections
import json
import re
import sys

LABEL = re.compile(r"^(\.LBB\d+_\d+|\.L[\w$.]+):")
BRANCH = re.compile(r"^\s*(s_cbranch_\w+|s_branch)\s+(\.LBB\d+_\d+)")


def kernel_body(lines, needle):
    start = None
    for i, ln in enumerate(lines):
        if start is None:
            m = re.match(r"^([A-Za-z_][\w$.]*):", ln)
            if m and needle in m.group(1):
                start = i
        elif ln.startswith(".Lfunc_end"):
            return lines[start:i]
    if start is None:
        raise SystemExit("kernel with %r not found" % needle)
    return lines[start:]


def mnemonic(ln):
    s = ln.strip()
    if not s or s.startswith(";") or s.startswith(".") or s.endswith(":"):
        return None
    return s.split()[0]


def histogram(body):
    h = collections.Counter()
    for ln in body:
        m = mnemonic(ln)
        if m:
            h[m] += 1
    return h


def hot_loop(body):
    labels = {}
    for i, ln in enumerate(body):
        m = LABEL.match(ln)
        if m:
            labels[m.group(1)] = i
    best = None
    for i, ln in enumerate(body):
        m = BRANCH.match(ln)
        if m and m.group(2) in labels and labels[m.group(2)] < i:
            lo = labels[m.group(2)]
            mads = sum(1 for x in body[lo:i] if "v_mad_u64_u32" in x)
            # most mads; among equal counts the tightest loop (an outer loop
            # around the term loop holds the same mads)
            if best is None or mads > best[0] or (mads == best[0] and i - lo < best[2] - best[1]):
                best = (mads, lo, i)
    if best is None:
        raise SystemExit("no loop found")
    return best[1], best[2]


def common_path(body, lo, hi):
    """the per-term common path: the accumulation loops compute the mixed
    addition's products, then test (one limb first) whether the rare case
    (the table point equals the accumulator: doubling) needs a full check;
    `s_cbranch_execz <loop label>` skips that check and the doubling when no
    lane needs it.  The common path is the loop from its first line to the
    first conditional back edge after a basic block of >= 100
    v_mad_u64_u32 (the products)"""
    labels = {}
    for i in range(lo, hi + 1):
        m = LABEL.match(body[i])
        if m:
            labels[m.group(1)] = i
    block_mads = 0
    seen_products = False
    for i in range(lo, hi + 1):
        ln = body[i]
        if LABEL.match(ln) or BRANCH.match(ln):
            seen_products = seen_products or block_mads >= 100
            block_mads = 0
        elif "v_mad_u64_u32" in ln:
            block_mads += 1
        m = BRANCH.match(ln)
        if (seen_products and m and m.group(1) != "s_branch" and m.group(2) in labels
                and labels[m.group(2)] < i):
            return body[lo:i + 1]
    return body[lo:hi + 1]


def fallthrough_path(body, lo, hi):
    """instructions on the not-taken path of every forward conditional branch
    from the loop head to the back edge (unconditional forward jumps are
    followed)"""
    labels = {}
    for i in range(lo, hi + 1):
        m = LABEL.match(body[i])
        if m:
            labels[m.group(1)] = i
    out = []
    i = lo
    seen = set()
    while i <= hi and i not in seen:
        seen.add(i)
        ln = body[i]
        m = BRANCH.match(ln)
        if m and m.group(1) == "s_branch" and m.group(2) in labels and labels[m.group(2)] > i:
            i = labels[m.group(2)]
            continue
        out.append(ln)
        i += 1
    return out


def marked_path(body, lo, hi, per_point):
    """(line, weight) pairs of one term's steady-state path through the loop
    [lo, hi], in a build with -DKZGX_ISA_MARKERS (curve.hpp KZGX_MARK): a
    forward branch whose first guarded block holds ';KZGX_RARE' is taken
    (the rare body is skipped), one whose first block holds
    ';KZGX_PER_POINT' guards the point change, counted with weight
    1 / per_point; every other forward branch falls through (its body runs
    on the common path).  Unconditional forward jumps are followed."""
    labels = {}
    for i in range(lo, hi + 1):
        m = LABEL.match(body[i])
        if m:
            labels[m.group(1)] = i

    def first_block(i):
        """the guarded region's lines outside every region nested in it (an
        asm marker may be scheduled anywhere in its block, not only first)"""
        tgt = labels[BRANCH.match(body[i]).group(2)]
        out = []
        j = i + 1
        while j < tgt:
            m = BRANCH.match(body[j])
            if m and m.group(2) in labels and j < labels[m.group(2)] <= tgt:
                j = labels[m.group(2)]  # skip the nested region
                continue
            out.append(body[j])
            j += 1
        return out

    out = []
    i = lo
    while i <= hi:
        ln = body[i]
        m = BRANCH.match(ln)
        if m and m.group(2) in labels and labels[m.group(2)] > i:
            tgt = labels[m.group(2)]
            head = first_block(i)
            if m.group(1) == "s_branch":
                i = tgt
                continue
            if any("KZGX_RARE" in x for x in head):
                out.append((ln, 1.0))
                i = tgt
                continue
            if any("KZGX_PER_POINT" in x for x in head):
                out.append((ln, 1.0))
                out.extend((x, 1.0 / per_point) for x in body[i + 1:tgt])
                i = tgt
                continue
        out.append((ln, 1.0))
        i += 1
    return out


def weighted_histogram(pairs):
    h = collections.Counter()
    for ln, wgt in pairs:
        m = mnemonic(ln)
        if m:
            h[m] += wgt
    return h


VALU_PREFIX = "v_"


def summarize(h, per):
    valu = sum(v for k, v in h.items() if k.startswith(VALU_PREFIX))
    res = {
        "v_mad_u64_u32": h.get("v_mad_u64_u32", 0) / per,
        "valu": valu / per,
        "salu": sum(v for k, v in h.items() if k.startswith("s_")) / per,
        "top": {k: v / per for k, v in h.most_common(24)},
    }
    return res


KERNELS = {  # bench.py's secondary.mad_issue key -> (kernel instantiation, windows per point)
    "BN254_c16": ("k_fixed_accumINS_7BN254G1ELi16E", 16),
    "BN254_c17": ("k_fixed_accumINS_7BN254G1ELi17E", 15),
    "BLS12381_c16": ("k_fixed_accumINS_10BLS12381G1ELi16E", 16),
}

PROBE = """#include "fixed_accum.hpp"
namespace kzgx {
template __global__ void k_fixed_accum<BN254G1, 16>(const uint32_t*, uint32_t, size_t, const uint32_t*, TabStrides,
                                                    const uint8_t*, uint32_t, uint32_t, uint32_t*);
template __global__ void k_fixed_accum<BN254G1, 17>(const uint32_t*, uint32_t, size_t, const uint32_t*, TabStrides,
                                                    const uint8_t*, uint32_t, uint32_t, uint32_t*);
template __global__ void k_fixed_accum<BLS12381G1, 16>(const uint32_t*, uint32_t, size_t, const uint32_t*,
                                                       TabStrides, const uint8_t*, uint32_t, uint32_t, uint32_t*);
}
"""


def emit_profile(out_path):
    """compile the k_fixed_accum instantiations of the throughput lines with
    the rare-path markers (-DKZGX_ISA_MARKERS) to gfx950 assembly and write
    the steady-state instructions per term: the common path of one mixed
    addition and its fetch / unpack / digit work, plus the point change
    divided by the windows per point"""
    import os
    import subprocess
    import tempfile
    root = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
    csrc = os.path.join(root, "kzg-commitments_amd", "csrc")
    with tempfile.TemporaryDirectory() as tmp:
        src = os.path.join(tmp, "probe.hip")
        with open(src, "w") as f:
            f.write(PROBE)
        asm = os.path.join(tmp, "probe.s")
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only",
                        "-DKZGX_ISA_MARKERS", "-I", csrc, "-S", "-o", asm, src], check=True, capture_output=True)
        with open(asm) as f:
            lines = f.read().splitlines()
    res = {"generated_by": "python3 scripts/isa_count.py --profile " + os.path.relpath(out_path, root),
           "unit": "instructions per table term in steady state: the loop's path with the rare bodies "
                   "(accumulator at infinity, equal x) skipped and the point change (scalar load, odd "
                   "recoding prep, table row) divided by the W windows per point; built with "
                   "-DKZGX_ISA_MARKERS (asm comments at those branches, curve.hpp KZGX_MARK)"}
    for key, (needle, W) in KERNELS.items():
        body = kernel_body(lines, needle)
        lo, hi = hot_loop(body)
        h = weighted_histogram(marked_path(body, lo, hi, W))
        valu = sum(v for k, v in h.items() if k.startswith(VALU_PREFIX))
        mads = h.get("v_mad_u64_u32", 0)
        res[key] = {"v_mad_u64_u32": round(mads, 2), "valu": round(valu, 2),
                    "salu": round(sum(v for k, v in h.items() if k.startswith("s_")), 2),
                    "s_nop": round(h.get("s_nop", 0), 2), "non_mad_valu": round(valu - mads, 2),
                    "v_mov": round(sum(v for k, v in h.items() if k.startswith("v_mov")), 2)}
    with open(out_path, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


def main():
    if len(sys.argv) == 3 and sys.argv[1] == "--profile":
        return emit_profile(sys.argv[2])
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("kernel")
    ap.add_argument("--per", type=float, default=1.0)
    ap.add_argument("--json", action="store_true")
    a = ap.parse_args()
    with open(a.asm) as f:
        lines = f.read().splitlines()
    body = kernel_body(lines, a.kernel)
    lo, hi = hot_loop(body)
    loop = body[lo:hi + 1]
    path = fallthrough_path(body, lo, hi)
    common = common_path(body, lo, hi)
    out = {"kernel": a.kernel, "loop_lines": hi - lo, "loop": summarize(histogram(loop), a.per),
           "path": summarize(histogram(path), a.per), "common": summarize(histogram(common), a.per)}
    if a.json:
        print(json.dumps(out))
    else:
        for k in ("loop", "path", "common"):
            s = out[k]
            print("%s: v_mad_u64_u32 %.0f  VALU %.0f  SALU %.0f" % (k, s["v_mad_u64_u32"], s["valu"], s["salu"]))
            print("   ", ", ".join("%s %.0f" % kv for kv in s["top"].items()))


if __name__ == "__main__":
    sys.exit(main())
