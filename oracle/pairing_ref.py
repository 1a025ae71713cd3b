"""CPU oracle (TEST INFRASTRUCTURE ONLY) for the verify half of the reference:
G2, the optimal ate pairing and the pairing-based verify_proof.

Only ``tests/`` may import this module, and only as the checker; the product
path (libkzgx.so) never calls it.

What it restates
----------------
* ``trusted_setup::verify_proof`` (reference src/trusted_setup.cpp:230-254):
  v1 = e(proof, [Z(tau)]G2), v2 = e(C - [I(tau)]G1, G2_0), return v1 == v2,
  with Z, I from ``linear_roots_and_polyfit`` (src/util.cpp:172-178).
* ``polyeval_G2`` (src/trusted_setup.cpp:176-201): naive sum c_i [tau^i]G2.
* the G2 half of the SRS (``generate_elements_range``, :123-135) and of the
  setup file (``export_setup`` :256-287, loader :76-121).
* miracl-core ``PAIR_ate`` + ``PAIR_fexp`` (un-vendored dependency, version
  unpinned): the optimal ate pairing.  BN254 (miracl's Nogami
  curve): loop 6u+2 with u < 0, two Frobenius lines.  BLS12-381: loop |x|,
  x < 0.  The final exponentiation is the exact (p^12 - 1)/r, so the pairing
  value is unique for a given curve, twist and Fp12 basis.

This oracle computes everything from definitions, in a deliberately
different way from the HIP kernels: the G2 point is untwisted into E(Fp12)
(Fp12 as Fp[w]/(w^12 - 2 w^6 + 2), i.e. w^6 = xi = 1 + i), the Miller loop
runs in affine Fp12 coordinates with exact inversions, and Frobenius is
plain exponentiation by p.  ``to_tower`` maps the result into the
Fp2 -> Fp6 -> Fp12 tower basis the GPU uses.

Twists (derived here, see ``twist_check``): both curves use Fp2 = Fp[i],
i^2 = -1, xi = 1 + i.  BN254 is a D-type sextic twist y^2 = x^3 + 2/xi,
BLS12-381 an M-type twist y^2 = x^3 + 4 xi -- in each case the only one of
the two candidates whose group order is divisible by r.

Parity status: verify_proof's boolean is independent of the pairing
variant and of the G2 generator (bilinearity + non-degeneracy), and it is
cross-checked against the MSM-free known-tau identity of
``kzg_ref.verify_proof_tau``.  The G2 generator of BLS12-381 is the standard
one (on-curve and order-r checked in ``self_check``).  miracl's BN254 G2
generator constants cannot be verified here (no miracl sources), so this
build derives one deterministically (``_derive_g2_gen``); exported G2 bytes
for BN254 are therefore "parity unpinned" against the reference binary.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass

import kzg_ref as K


# --------------------------------------------------------------------------
# Fp2 = Fp[i] / (i^2 + 1)
# --------------------------------------------------------------------------
def f2add(p, a, b):
    return ((a[0] + b[0]) % p, (a[1] + b[1]) % p)


def f2sub(p, a, b):
    return ((a[0] - b[0]) % p, (a[1] - b[1]) % p)


def f2neg(p, a):
    return ((-a[0]) % p, (-a[1]) % p)


def f2mul(p, a, b):
    return ((a[0] * b[0] - a[1] * b[1]) % p, (a[0] * b[1] + a[1] * b[0]) % p)


def f2inv(p, a):
    n = (a[0] * a[0] + a[1] * a[1]) % p
    ni = pow(n, -1, p)
    return (a[0] * ni % p, (-a[1]) * ni % p)


def f2pow(p, a, e):
    r = (1, 0)
    while e:
        if e & 1:
            r = f2mul(p, r, a)
        a = f2mul(p, a, a)
        e >>= 1
    return r


def f2sqrt(p, a):
    """square root in Fp2 for p = 3 mod 4 (None if a is a non-residue)"""
    if a == (0, 0):
        return (0, 0)
    a1 = f2pow(p, a, (p - 3) // 4)
    alpha = f2mul(p, f2mul(p, a1, a1), a)
    a0 = f2mul(p, f2pow(p, alpha, p), alpha)
    if a0 == (p - 1, 0):
        return None
    x0 = f2mul(p, a1, a)
    if alpha == (p - 1, 0):
        x = f2mul(p, (0, 1), x0)
    else:
        x = f2mul(p, f2pow(p, f2add(p, (1, 0), alpha), (p - 1) // 2), x0)
    assert f2mul(p, x, x) == a
    return x


XI = (1, 1)


# --------------------------------------------------------------------------
# curves: twist data
# --------------------------------------------------------------------------
def _trace(C):
    if C.name == "BN254":
        return 6 * K._U ** 2 + 1
    return K._BLS_X + 1


def _twist_order(C):
    p, r, t = C.p, C.r, _trace(C)
    t2 = t * t - 2 * p
    f2 = (4 * p * p - t2 * t2) // 3
    import math
    f = math.isqrt(f2)
    assert f * f == f2
    cands = [p * p + 1 - (s1 * 3 * f + s2 * t2) // 2 for s1 in (1, -1) for s2 in (1, -1)]
    cands = sorted({n for n in cands if n % r == 0})
    assert len(cands) == 1
    return cands[0]


@dataclass(frozen=True)
class Twist:
    kind: str      # "D": y^2 = x^3 + b/xi ; "M": y^2 = x^3 + b xi
    b2: tuple
    order: int     # #E'(Fp2)
    h2: int        # cofactor order / r


def twist(C) -> Twist:
    p = C.p
    n2 = _twist_order(C)
    if C.name == "BN254":
        return Twist("D", f2mul(p, (C.b, 0), f2inv(p, XI)), n2, n2 // C.r)
    return Twist("M", f2mul(p, (C.b, 0), XI), n2, n2 // C.r)


# ---- G2 affine arithmetic (None = infinity) --------------------------------
def g2_on_curve(C, Q):
    if Q is None:
        return True
    p = C.p
    x, y = Q
    return f2sub(p, f2mul(p, y, y), f2add(p, f2mul(p, f2mul(p, x, x), x), twist(C).b2)) == (0, 0)


def g2_neg(C, Q):
    return None if Q is None else (Q[0], f2neg(C.p, Q[1]))


def g2_add(C, P, Q):
    p = C.p
    if P is None:
        return Q
    if Q is None:
        return P
    if P[0] == Q[0]:
        if f2add(p, P[1], Q[1]) == (0, 0):
            return None
        lam = f2mul(p, f2mul(p, (3, 0), f2mul(p, P[0], P[0])), f2inv(p, f2mul(p, (2, 0), P[1])))
    else:
        lam = f2mul(p, f2sub(p, Q[1], P[1]), f2inv(p, f2sub(p, Q[0], P[0])))
    x3 = f2sub(p, f2sub(p, f2mul(p, lam, lam), P[0]), Q[0])
    y3 = f2sub(p, f2mul(p, lam, f2sub(p, P[0], x3)), P[1])
    return (x3, y3)


def g2_mul_raw(C, Q, k):
    R = None
    if k < 0:
        Q, k = g2_neg(C, Q), -k
    for bit in bin(k)[2:] if k else "":
        R = g2_add(C, R, R)
        if bit == "1":
            R = g2_add(C, R, Q)
    return R


def g2_mul(C, Q, k):
    """[k]Q for Q of order r (k reduced mod r, like PAIR_G2mul)"""
    return g2_mul_raw(C, Q, k % C.r)


# standard BLS12-381 G2 generator (x = x0 + x1 i, y = y0 + y1 i)
_BLS_G2 = (
    (0x024AA2B2F08F0A91260805272DC51051C6E47AD4FA403B02B4510B647AE3D1770BAC0326A805BBEFD48056C8C121BDB8,
     0x13E02B6052719F607DACD3A088274F65596BD0D09920B61AB5DA61BBDC7F5049334CF11213945D57E5AC7D055D042B7E),
    (0x0CE5D527727D6E118CC9CDC6DA2E351AADFD9BAA8CBDD3A76D429A695160D12C923AC9CC3BACA289E193548608B82801,
     0x0606C4A02EA734CC32ACD2B02BC28B99CB3E287E85A763AF267492AB572E99AB3F370D275CEC1DA1AAA9075FF05F79BE),
)


def _derive_g2_gen(C):
    """Deterministic G2 generator: the first x = k + i (k = 1, 2, ...) with
    x^3 + b' a square in Fp2, y the root with the smaller (imag, real) pair,
    times the twist cofactor."""
    p = C.p
    T = twist(C)
    k = 1
    while True:
        x = (k % p, 1)
        y = f2sqrt(p, f2add(p, f2mul(p, f2mul(p, x, x), x), T.b2))
        if y is not None:
            ny = f2neg(p, y)
            if (ny[1], ny[0]) < (y[1], y[0]):
                y = ny
            Q = g2_mul_raw(C, (x, y), T.h2)
            if Q is not None:
                return Q
        k += 1


_G2_CACHE = {}


def g2_generator(C):
    if C.name not in _G2_CACHE:
        _G2_CACHE[C.name] = _BLS_G2 if C.name == "BLS12381" else _derive_g2_gen(C)
    return _G2_CACHE[C.name]


def self_check(C):
    """twist order divisible by r, generator on the twist with order r"""
    Q = g2_generator(C)
    assert g2_on_curve(C, Q)
    assert g2_mul_raw(C, Q, C.r) is None
    assert g2_mul_raw(C, Q, C.r - 1) == g2_neg(C, Q)
    return True


# --------------------------------------------------------------------------
# Fp12 = Fp[w] / (w^12 - 2 w^6 + 2)   (w^6 = xi = 1 + i, i = w^6 - 1)
# --------------------------------------------------------------------------
class F12:
    __slots__ = ("c", "p")

    def __init__(self, p, c):
        self.p = p
        self.c = [v % p for v in c]

    @staticmethod
    def one(p):
        return F12(p, [1] + [0] * 11)

    @staticmethod
    def from_fp(p, a):
        return F12(p, [a] + [0] * 11)

    @staticmethod
    def from_fp2(p, a):
        # a0 + a1 i = a0 + a1 (w^6 - 1)
        c = [0] * 12
        c[0] = a[0] - a[1]
        c[6] = a[1]
        return F12(p, c)

    def __eq__(self, o):
        return self.c == o.c

    def __add__(self, o):
        return F12(self.p, [a + b for a, b in zip(self.c, o.c)])

    def __sub__(self, o):
        return F12(self.p, [a - b for a, b in zip(self.c, o.c)])

    def __neg__(self):
        return F12(self.p, [-a for a in self.c])

    def __mul__(self, o):
        p = self.p
        t = [0] * 23
        for i, a in enumerate(self.c):
            if a:
                for j, b in enumerate(o.c):
                    t[i + j] += a * b
        for k in range(22, 11, -1):  # w^k = 2 w^(k-6) - 2 w^(k-12)
            v = t[k]
            if v:
                t[k - 6] += 2 * v
                t[k - 12] -= 2 * v
        return F12(p, t[:12])

    def is_one(self):
        return self.c == [1] + [0] * 11

    def inv(self):
        """extended Euclid over Fp[w] against the modulus polynomial"""
        p = self.p

        def deg(a):
            d = len(a) - 1
            while d >= 0 and a[d] % p == 0:
                d -= 1
            return d

        def pdivmod(a, b):
            a = [x % p for x in a]
            db = deg(b)
            ib = pow(b[db], -1, p)
            q = [0] * max(len(a) - db, 1)
            for k in range(deg(a), db - 1, -1):
                c = a[k] * ib % p
                if c:
                    q[k - db] = c
                    for j in range(db + 1):
                        a[k - db + j] = (a[k - db + j] - c * b[j]) % p
            return q, a

        def psub(a, b):
            n = max(len(a), len(b))
            return [((a[i] if i < len(a) else 0) - (b[i] if i < len(b) else 0)) % p for i in range(n)]

        def pmul(a, b):
            t = [0] * (len(a) + len(b))
            for i, x in enumerate(a):
                for j, y in enumerate(b):
                    t[i + j] = (t[i + j] + x * y) % p
            return t

        modulus = [2, 0, 0, 0, 0, 0, (-2) % p, 0, 0, 0, 0, 0, 1]
        r0, r1 = modulus, list(self.c)
        s0, s1 = [0], [1]
        while deg(r1) > 0:
            q, rem = pdivmod(r0, r1)
            r0, r1 = r1, rem
            s0, s1 = s1, psub(s0, pmul(q, s1))
        assert deg(r1) == 0, "not invertible"
        c = pow(r1[0], -1, p)
        out = [(x * c) % p for x in s1]
        # reduce mod the modulus
        _, out = pdivmod(out + [0] * 13, modulus)
        res = F12(p, (out + [0] * 12)[:12])
        assert (res * self).is_one()
        return res

    def pow(self, e):
        r = F12.one(self.p)
        a = self
        while e:
            if e & 1:
                r = r * a
            a = a * a
            e >>= 1
        return r

    def frob(self):
        return self.pow(self.p)


def _w(p):
    return F12(p, [0, 1] + [0] * 10)


def untwist(C, Q):
    p = C.p
    x, y = F12.from_fp2(p, Q[0]), F12.from_fp2(p, Q[1])
    w = _w(p)
    w2 = w * w
    w3 = w2 * w
    if twist(C).kind == "D":
        return (x * w2, y * w3)
    w2i, w3i = w2.inv(), w3.inv()
    return (x * w2i, y * w3i)


# ---- E(Fp12) affine (None = infinity) ---------------------------------------
def _e12_add(p, P, Q):
    if P is None:
        return Q
    if Q is None:
        return P
    if P[0] == Q[0]:
        if (P[1] + Q[1]).c == [0] * 12:
            return None
        lam = F12.from_fp(p, 3) * P[0] * P[0] * (F12.from_fp(p, 2) * P[1]).inv()
    else:
        lam = (Q[1] - P[1]) * (Q[0] - P[0]).inv()
    x3 = lam * lam - P[0] - Q[0]
    return (x3, lam * (P[0] - x3) - P[1])


def _line(p, T, Q, Px, Py):
    """l_{T,Q}(P): the line through T and Q (tangent if T == Q) at P"""
    if T[0] == Q[0]:
        if (T[1] + Q[1]).c == [0] * 12:
            return Px - T[0]  # vertical
        lam = F12.from_fp(p, 3) * T[0] * T[0] * (F12.from_fp(p, 2) * T[1]).inv()
    else:
        lam = (Q[1] - T[1]) * (Q[0] - T[0]).inv()
    return (Py - T[1]) - lam * (Px - T[0])


def _miller(p, Q, n, Px, Py):
    f = F12.one(p)
    T = Q
    for bit in bin(n)[3:]:
        f = f * f * _line(p, T, T, Px, Py)
        T = _e12_add(p, T, T)
        if bit == "1":
            f = f * _line(p, T, Q, Px, Py)
            T = _e12_add(p, T, Q)
    return f, T


def miller_loop(C, P, Q):
    """optimal ate Miller function value (before the final exponentiation)"""
    p = C.p
    if P is None or Q is None:
        return F12.one(p)
    Qe = untwist(C, Q)
    Px, Py = F12.from_fp(p, P[0]), F12.from_fp(p, P[1])
    if C.name == "BN254":
        s = 6 * K._U + 2
        f, T = _miller(p, Qe, abs(s), Px, Py)
        if s < 0:
            f = f.inv()
            T = (T[0], -T[1])
        Q1 = (Qe[0].frob(), Qe[1].frob())
        Q2 = (Q1[0].frob(), Q1[1].frob())
        nQ2 = (Q2[0], -Q2[1])
        f = f * _line(p, T, Q1, Px, Py)
        T = _e12_add(p, T, Q1)
        f = f * _line(p, T, nQ2, Px, Py)
        return f
    s = K._BLS_X
    f, _ = _miller(p, Qe, abs(s), Px, Py)
    if s < 0:
        f = f.inv()
    return f


def final_exp(C, f):
    return f.pow((C.p ** 12 - 1) // C.r)


def pairing(C, P, Q):
    """e(P, Q) for P in G1, Q in G2 (PAIR_ate + PAIR_fexp)"""
    return final_exp(C, miller_loop(C, P, Q))


def to_tower(C, f):
    """flat Fp12 -> tower coordinates [c0.a0, c0.a1, c0.a2, c1.a0, c1.a1, c1.a2],
    each Fp2 as (re, im): Fp12 = Fp6[w]/(w^2 - v), Fp6 = Fp2[v]/(v^3 - xi)"""
    p = C.p
    out = []
    for half in (0, 1):
        for j in range(3):
            k = 2 * j + half
            im = f.c[k + 6]
            re = (f.c[k] + im) % p
            out.append((re, im))
    return out


# --------------------------------------------------------------------------
# KZG verify half (trusted_setup.cpp:123-135, 176-201, 230-254)
# --------------------------------------------------------------------------
def gen_srs_g2(C, tau: int, n: int):
    Q = g2_generator(C)
    out, s = [], 1
    for _ in range(n):
        out.append(g2_mul(C, Q, s))
        s = s * tau % C.r
    return out


def polyeval_g2(C, srs2, P):
    """naive sum c_i [tau^i]G2 (trusted_setup.cpp:176-201)"""
    P = K.normalize(P)
    acc = None
    for i, c in enumerate(P):
        acc = g2_add(C, acc, g2_mul(C, srs2[i], c))
    return acc


def verify_proof(C, srs1, srs2, commit, proof, points):
    """trusted_setup::verify_proof, pairing form (trusted_setup.cpp:230-254)"""
    if len(points) < 1:
        raise ValueError("expected_data size must be 1 or greater")
    if len(points) >= len(srs1):
        return False
    I = K.interpolate(C, points)
    Z = K.linear_roots(C, [x for x, _ in points])
    p1 = polyeval_g2(C, srs2, Z)
    v1 = pairing(C, proof, p1)
    p2 = K.point_add(C, K.point_neg(C, K.polyeval_g1(C, srs1, I)), commit)
    v2 = pairing(C, p2, srs2[0])
    return v1 == v2


# ---- setup file (trusted_setup.cpp:76-121, 256-287) ------------------------
def ecp2_octet(C, Q) -> bytes:
    """ECP2_toOctet(..., false): 0x04 || x || y, each Fp2 as (imag, real)
    big-endian MODBYTES each -- miracl-core's current FP2_toBytes order
    (recalled; version-dependent and not verifiable here).  Infinity:
    ECP2_inf = (0, 1)."""
    mb = C.modbytes

    def fp2b(a):
        return a[1].to_bytes(mb, "big") + a[0].to_bytes(mb, "big")

    if Q is None:
        return b"\x04" + fp2b((0, 0)) + fp2b((1, 0))
    return b"\x04" + fp2b(Q[0]) + fp2b(Q[1])


def ecp2_from_octet(C, o: bytes):
    mb = C.modbytes
    if len(o) != 4 * mb + 1 or o[0] != 4:
        raise ValueError("bad G2 octet")
    v = [int.from_bytes(o[1 + k * mb:1 + (k + 1) * mb], "big") for k in range(4)]
    x, y = (v[1], v[0]), (v[3], v[2])
    if x == (0, 0) and y == (1, 0):
        return None
    if not g2_on_curve(C, (x, y)):
        raise ValueError("bad G2 octet")
    return (x, y)


def export_setup(C, srs1, srs2) -> bytes:
    out = [struct.pack("<Q", len(srs1))]
    for P in srs1:
        o = K.ecp_octet(C, P)
        out.append(struct.pack("<I", len(o)) + o)
    for Q in srs2:
        o = ecp2_octet(C, Q)
        out.append(struct.pack("<I", len(o)) + o)
    return b"".join(out)
