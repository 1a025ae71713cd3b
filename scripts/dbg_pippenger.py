"""Debug: run one table-less Pippenger MSM and check every stage's workspace
(bucket offsets, sorted entries, bucket sums) against Python EC arithmetic."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kzg-commitments_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import kzgx  # noqa: E402
import kzg_ref as K  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "BN254"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 17
C = K.BN254 if name == "BN254" else K.BLS12381
CB = 12
W = (257 + CB - 1) // CB
NB = 1 << (CB - 1)
L = 9 if name == "BN254" else 14
XW = 4 * L
p = C.p

ctx = kzgx.Context(name, device=0)
tau = K.default_tau(C)
ctx.gen_srs(tau, max(n, 2))
srs = ctx.get_srs(max(n, 2))
sc = K.random_scalars(C, n, seed=1000 + n)
limbs = np.array([[(v >> (64 * i)) & 0xFFFFFFFFFFFFFFFF for i in range(4)] for v in sc], dtype=np.uint64)
out, inf = ctx.msm(limbs)
w64 = ctx.w64


def to_int(row):
    return sum(int(row[i]) << (64 * i) for i in range(len(row)))


got = None if inf else (to_int(out[:w64]), to_int(out[w64:2 * w64]))
pts = [(to_int(srs[i, :w64]), to_int(srs[i, w64:2 * w64])) for i in range(n)]
exp = K.commit_via_tau(C, tau, sc)
print("final ok:", got == exp)

lib = kzgx.lib()
lib.kzgx_debug_ws_read.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_void_p, ctypes.c_size_t]


def read(nm, count, dtype):
    a = np.zeros(count, dtype=dtype)
    rc = lib.kzgx_debug_ws_read(ctx.h, nm.encode(), a.ctypes.data, a.nbytes)
    assert rc == 0, (nm, rc)
    return a


off = read("offsets", NB + 1, np.uint32).astype(np.int64)
E = int(off[NB])


def digits(s):
    out_, carry = [], 0
    for w in range(W):
        raw = ((s >> (CB * w)) & ((1 << CB) - 1)) + carry
        if raw > NB:
            carry = 1
            out_.append(raw - (1 << CB))
        else:
            carry = 0
            out_.append(raw)
    return out_


exp_b = [[] for _ in range(NB)]
for i, s in enumerate(sc):
    for w, d in enumerate(digits(s)):
        if d:
            exp_b[abs(d) - 1].append((w, i, d < 0))
ent = read("entries", E, np.uint32)
bad = 0
for k in range(NB):
    got_b = sorted(((int(e) & 0x7fffffff) // max(n, 2), (int(e) & 0x7fffffff) % max(n, 2), bool(e >> 31))
                   for e in ent[off[k]:off[k + 1]])
    if got_b != sorted(exp_b[k]):
        bad += 1
        if bad < 4:
            print("bucket", k, "entries differ", got_b[:4], sorted(exp_b[k])[:4])
print("E", E, "expected", sum(len(x) for x in exp_b), "buckets with wrong entries:", bad)


def mul(P, s):
    return K.scalar_mul(C, P, s % C.r)


def add(P, Q):
    return K.point_add(C, P, Q) if hasattr(K, "point_add") else K.ec_add(C, P, Q)


bs = read("bsum", NB * XW, np.uint32).reshape(NB, XW)


def limbs29(v):
    return sum(int(v[i]) << (29 * i) for i in range(L))


def xyzz_affine(row):
    X, Y, ZZ, ZZZ = (limbs29(row[j * L:(j + 1) * L]) for j in range(4))
    if ZZ % p == 0:
        return None
    return (X * pow(ZZ, -1, p) % p, Y * pow(ZZZ, -1, p) % p)


wrong = 0
for k in range(NB):
    if off[k + 1] == off[k]:
        continue
    acc = None
    for (w, i, neg) in exp_b[k]:
        s = (1 << (CB * w)) * (-1 if neg else 1)
        acc = add(acc, mul(pts[i], s))
    g = xyzz_affine(bs[k])
    if g != acc:
        wrong += 1
        if wrong < 6:
            print("bucket", k, "size", off[k + 1] - off[k], "bsum wrong")
print("buckets with wrong sums:", wrong, "of", int(np.sum(off[1:] > off[:-1])))

# per-segment partials of the wrong buckets
Kseg = 128
while Kseg > 8 and n * W // Kseg < 131072:
    Kseg //= 2
smax = (n * W + Kseg - 1) // Kseg
st = read("sstate", smax, np.uint8)
tk = read("tailk", smax, np.uint32)
hd = read("heads", smax * XW, np.uint32).reshape(smax, XW)
tl = read("tails", smax * XW, np.uint32).reshape(smax, XW)
ent_pts = []
for e in ent:
    e = int(e)
    w, i = (e & 0x7fffffff) // max(n, 2), (e & 0x7fffffff) % max(n, 2)
    ent_pts.append(mul(pts[i], (1 << (CB * w)) * (-1 if e >> 31 else 1)))
print("K", Kseg, "smax", smax)
for k in range(NB):
    if off[k + 1] == off[k]:
        continue
    s0, s1 = off[k] // Kseg, (off[k + 1] - 1) // Kseg
    if s0 == s1:
        continue
    acc = None
    for q in range(off[k], off[k + 1]):
        acc = add(acc, ent_pts[q])
    g = xyzz_affine(bs[k])
    # expected tail (entries in s0) and heads
    tail_exp = None
    for q in range(off[k], min(off[k + 1], (s0 + 1) * Kseg)):
        tail_exp = add(tail_exp, ent_pts[q])
    print("bucket", k, "entries", off[k], off[k + 1], "segs", s0, s1, "ok" if g == acc else "WRONG",
          "tailk[s0]", int(tk[s0]), "tail ok", xyzz_affine(tl[s0]) == tail_exp,
          "states", [int(st[s]) for s in range(s0, s1 + 1)])
    for s in range(s0 + 1, s1 + 1):
        h_exp = None
        for q in range(max(off[k], s * Kseg), min(off[k + 1], (s + 1) * Kseg)):
            h_exp = add(h_exp, ent_pts[q])
        print("   head", s, "ok", xyzz_affine(hd[s]) == h_exp)
    if g != acc:
        print("   bsum equals tail only:", g == tail_exp, " is None:", g is None)
nwg = (smax + 127) // 128
gm = read("gmeta", 2 * nwg, np.uint32)
print("gtailk", [hex(int(v)) for v in gm[:nwg]], "gflag", [int(v) for v in gm[nwg:]])
for k in range(NB):
    if off[k + 1] - off[k] >= 2:
        s0, s1 = off[k] // Kseg, (off[k + 1] - 1) // Kseg
        if s0 != s1:
            g = xyzz_affine(bs[k])
            th = add(xyzz_affine(tl[s0]), xyzz_affine(hd[s0 + 1]))
            print("bucket", k, "bsum == tail+head(gpu partials):", g == th, "raw bsum ZZ limbs", list(bs[k][2 * L:2 * L + 3]))
