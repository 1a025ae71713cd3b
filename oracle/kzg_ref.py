"""CPU oracle (TEST INFRASTRUCTURE ONLY) -- pure-Python restatement of the
reference KZG path of uncommitted6453/kzg-commitments.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this module, and only as the checker.  The
product path (``libkzgx.so``) never calls it.

Parity status
-------------
The reference cannot be built or run here (its miracl-core and NTL
submodules are empty) and its own tests hold no
known-answer vectors: every check there is a round trip against a random SRS.
This oracle is therefore pinned by
  * the curve constants: p and r re-derived from the BN parameter u
    (BN254) / the BLS parameter x (BLS12-381), G on the curve, r*G = O
    (``self_check``),
  * an MSM-independent identity: with a known tau, commit == [P(tau)]G1 and
    every proof == [q(tau)]G1 (``commit_via_tau``),
  * the reference's own fixtures (testing/blob1.txt, blob2.txt, the test
    strings of testing/testing.cpp) and its known throw / no-throw
    behaviours, replayed in tests/test_oracle.py.
Reference-produced output bytes do not exist for this path, so byte-level
parity against the reference binary itself is "parity unpinned" beyond the
above; affine (x, y) of a group element is unique, so any exact
implementation of the same math is bit-exact.
"""
from __future__ import annotations

import hashlib
import struct
from dataclasses import dataclass


# --------------------------------------------------------------------------
# curves (config/curve_BN254/kzg_config.h:4-13, config/curve_BLS12381/...)
# --------------------------------------------------------------------------
@dataclass(frozen=True)
class Curve:
    name: str
    p: int          # base field modulus
    r: int          # group order == scalar field modulus (NTL ZZ_p::init(r))
    b: int          # y^2 = x^3 + b
    gx: int
    gy: int
    modbytes: int   # MODBYTES_CURVE

    @property
    def order_bytes(self) -> int:      # kzg::CURVE_ORDER_BYTES, trusted_setup.cpp:18
        return (self.r.bit_length() + 7) // 8

    @property
    def max_chunk_bytes(self) -> int:  # MAX_CHUNK_BYTES, kzg.h:31
        return self.order_bytes - 1


_U = -(2**62 + 2**55 + 1)                      # miracl BN254 (Nogami) parameter
_BN_P = 36 * _U**4 + 36 * _U**3 + 24 * _U**2 + 6 * _U + 1
_BN_R = 36 * _U**4 + 36 * _U**3 + 18 * _U**2 + 6 * _U + 1
BN254 = Curve("BN254", _BN_P, _BN_R, 2, _BN_P - 1, 1, 32)

_BLS_X = -0xD201000000010000
_BLS_P = (_BLS_X - 1) ** 2 * (_BLS_X**4 - _BLS_X**2 + 1) // 3 + _BLS_X
_BLS_R = _BLS_X**4 - _BLS_X**2 + 1
BLS12381 = Curve(
    "BLS12381", _BLS_P, _BLS_R, 4,
    0x17F1D3A73197D7942695638C4FA9AC0FC3688C4F9774B905A14E3A3F171BAC586C55E83FF97A1AEFFB3AF00ADB22C6BB,
    0x08B3F481E3AAA0F1A09E30ED741D8AE4FCF5E095D5D00AF600DB18CB2C04B3EDD03CC744A2888AE40CAA232946C5E7E1,
    48,
)
CURVES = {"BN254": BN254, "BLS12381": BLS12381}

INF = None  # point at infinity (affine representation)


# --------------------------------------------------------------------------
# G1 arithmetic (stands in for miracl ECP / PAIR_G1mul / ECP_add)
# Jacobian (X, Y, Z), a = 0.
# --------------------------------------------------------------------------
def _jdbl(C, P):
    X, Y, Z = P
    if Z == 0 or Y == 0:
        return (1, 1, 0)
    p = C.p
    A = X * X % p
    B = Y * Y % p
    CC = B * B % p
    D = 2 * ((X + B) ** 2 - A - CC) % p
    E = 3 * A % p
    X3 = (E * E - 2 * D) % p
    Y3 = (E * (D - X3) - 8 * CC) % p
    Z3 = 2 * Y * Z % p
    return (X3, Y3, Z3)


def _jadd(C, P, Q):
    if P[2] == 0:
        return Q
    if Q[2] == 0:
        return P
    p = C.p
    X1, Y1, Z1 = P
    X2, Y2, Z2 = Q
    Z1Z1 = Z1 * Z1 % p
    Z2Z2 = Z2 * Z2 % p
    U1 = X1 * Z2Z2 % p
    U2 = X2 * Z1Z1 % p
    S1 = Y1 * Z2 * Z2Z2 % p
    S2 = Y2 * Z1 * Z1Z1 % p
    if U1 == U2:
        if S1 == S2:
            return _jdbl(C, P)
        return (1, 1, 0)
    H = (U2 - U1) % p
    I = (2 * H) ** 2 % p
    J = H * I % p
    rr = 2 * (S2 - S1) % p
    V = U1 * I % p
    X3 = (rr * rr - J - 2 * V) % p
    Y3 = (rr * (V - X3) - 2 * S1 * J) % p
    Z3 = ((Z1 + Z2) ** 2 - Z1Z1 - Z2Z2) * H % p
    return (X3, Y3, Z3)


def to_jac(P):
    return (1, 1, 0) if P is None else (P[0], P[1], 1)


def to_affine(C, P):
    if P[2] == 0:
        return None
    zi = pow(P[2], -1, C.p)
    zi2 = zi * zi % C.p
    return (P[0] * zi2 % C.p, P[1] * zi2 * zi % C.p)


def point_add(C, P, Q):
    return to_affine(C, _jadd(C, to_jac(P), to_jac(Q)))


def point_neg(C, P):
    return None if P is None else (P[0], (-P[1]) % C.p)


def scalar_mul(C, P, k):
    """Left-to-right double-and-add; equals PAIR_G1mul(P, k) as a group element."""
    k %= C.r
    R = (1, 1, 0)
    Pj = to_jac(P)
    for bit in bin(k)[2:] if k else "":
        R = _jdbl(C, R)
        if bit == "1":
            R = _jadd(C, R, Pj)
    return to_affine(C, R)


def on_curve(C, P):
    if P is None:
        return True
    x, y = P
    return (y * y - x * x * x - C.b) % C.p == 0


def self_check(C):
    """Curve constants pinned: G on curve, r*G = O, (r-1)*G = -G."""
    G = (C.gx, C.gy)
    assert on_curve(C, G)
    # scalar_mul reduces k mod r, so check the order via (r-1)G == -G
    R = _jac_mul_raw(C, G, C.r - 1)
    assert to_affine(C, R) == point_neg(C, G)
    R2 = _jadd(C, R, to_jac(G))
    assert R2[2] == 0
    return True


def _jac_mul_raw(C, P, k):
    R = (1, 1, 0)
    Pj = to_jac(P)
    for bit in bin(k)[2:]:
        R = _jdbl(C, R)
        if bit == "1":
            R = _jadd(C, R, Pj)
    return R


# --------------------------------------------------------------------------
# SRS  (trusted_setup.cpp:21-74, generate_elements_range :123-135)
# The reference draws tau from std::random_device (util.cpp:62-76); the oracle
# takes it as a parameter so goldens are reproducible.
# --------------------------------------------------------------------------
def default_tau(C) -> int:
    return int.from_bytes(hashlib.sha256(b"kzg-mi355x-tau").digest(), "big") % C.r


def gen_srs(C, tau: int, n: int):
    if n < 2:                                   # trusted_setup.cpp:22-24
        raise ValueError("num_coeff must be at least 2")
    G = (C.gx, C.gy)
    out = []
    s = 1
    for _ in range(n):
        out.append(scalar_mul(C, G, s))
        s = s * tau % C.r
    return out


# --------------------------------------------------------------------------
# blob (blob.cpp:3-48)
# --------------------------------------------------------------------------
def blob_from_string(C, s: bytes, offset: int = 0):
    """x = i + offset, y = (signed char) s[i]  (blob.cpp:7-18)."""
    pts = []
    for i, ch in enumerate(s):
        v = ch - 256 if ch >= 128 else ch
        pts.append(((i + offset) % C.r, v % C.r))
    return pts


def blob_from_bytes(C, data: bytes, byte_offset: int, byte_length: int, chunk_size: int):
    """Little-endian chunks (blob.cpp:20-48).  Reads data[0 ...]: ``data``
    already points at the byte range, byte_offset only sets x."""
    if chunk_size > C.max_chunk_bytes:
        raise ValueError("chunk_size must be at most MAX_CHUNK_BYTES.")
    if chunk_size < 1:  # reference: integer division by zero (UB); we reject
        raise ValueError("chunk_size must be at least 1")
    if _cmod(byte_offset, chunk_size) != 0:
        raise ValueError("byte_offset is not a multiple of chunk_size.")
    if _cmod(byte_length, chunk_size) != 0:
        raise ValueError("byte_length is not a multiple of chunk_size.")
    chunk_offset = _cdiv(byte_offset, chunk_size)
    chunk_length = _cdiv(byte_length, chunk_size)
    pts = []
    for i in range(max(chunk_length, 0)):
        chunk = data[i * chunk_size:(i + 1) * chunk_size]
        pts.append(((chunk_offset + i) % C.r, int.from_bytes(chunk, "little") % C.r))
    return pts


def _cdiv(a, b):  # C integer division (truncation toward zero)
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b >= 0) else -q


def _cmod(a, b):
    return a - b * _cdiv(a, b)


# --------------------------------------------------------------------------
# polynomials over Z_r (NTL ZZ_pX semantics: little-endian coeff list,
# normalized -> no trailing zero; deg(0) = -1)
# --------------------------------------------------------------------------
def normalize(P):
    P = list(P)
    while P and P[-1] == 0:
        P.pop()
    return P


def deg(P) -> int:
    return len(normalize(P)) - 1


def poly_eval(C, P, x):
    acc = 0
    for c in reversed(P):
        acc = (acc * x + c) % C.r
    return acc


def poly_mul(C, A, B):
    if not A or not B:
        return []
    out = [0] * (len(A) + len(B) - 1)
    for i, a in enumerate(A):
        if a:
            for j, b in enumerate(B):
                out[i + j] = (out[i + j] + a * b) % C.r
    return normalize(out)


def poly_sub(C, A, B):
    n = max(len(A), len(B))
    return normalize([((A[i] if i < len(A) else 0) - (B[i] if i < len(B) else 0)) % C.r
                      for i in range(n)])


def poly_divmod(C, A, B):
    """NTL DivRem over Z_r (quotient used by operator/ in trusted_setup.cpp:225)."""
    A = normalize(A)
    B = normalize(B)
    if not B:
        raise ZeroDivisionError("division by zero polynomial")
    if len(A) < len(B):
        return [], A
    inv_lead = pow(B[-1], -1, C.r)
    rem = list(A)
    q = [0] * (len(A) - len(B) + 1)
    for k in range(len(q) - 1, -1, -1):
        c = rem[k + len(B) - 1] * inv_lead % C.r
        q[k] = c
        if c:
            for j, b in enumerate(B):
                rem[k + j] = (rem[k + j] - c * b) % C.r
    return normalize(q), normalize(rem[:len(B) - 1])


def linear_roots(C, xs):
    """Z = prod (X - x_i)  (build_linear_roots_tree, util.cpp:269-284)."""
    Z = [1]
    for x in xs:
        # multiply by (X - x)
        nz = [0] * (len(Z) + 1)
        for k, c in enumerate(Z):
            nz[k + 1] = (nz[k + 1] + c) % C.r
            nz[k] = (nz[k] - x * c) % C.r
        Z = nz
    return Z


def interpolate(C, points):
    """Unique interpolant of degree < N through N points with distinct x
    (polyfit / polyfit_R, util.cpp:172-184, 213-248; same polynomial as the
    reference's subproduct-tree method, computed by Lagrange)."""
    n = len(points)
    if n == 0:
        return []
    r = C.r
    xs = [p[0] % r for p in points]
    ys = [p[1] % r for p in points]
    if len(set(xs)) != n:
        raise ZeroDivisionError("duplicate interpolation node")
    Z = linear_roots(C, xs)
    # a_i = y_i / Z'(x_i)
    dZ = [(k * Z[k]) % r for k in range(1, len(Z))]
    denoms = [poly_eval(C, dZ, x) for x in xs]
    invs = _batch_inv(r, denoms)
    a = [y * iv % r for y, iv in zip(ys, invs)]
    # c_k = sum_i a_i * (Z / (X - x_i))_k, synthetic division vectorized over i
    coef = [0] * n
    q = [0] * n
    for k in range(n - 1, -1, -1):
        zk1 = Z[k + 1]
        s = 0
        for i in range(n):
            qi = (zk1 + xs[i] * q[i]) % r
            q[i] = qi
            s += a[i] * qi
        coef[k] = s % r
    return normalize(coef)


def _batch_inv(r, vals):
    pref = []
    acc = 1
    for v in vals:
        pref.append(acc)
        acc = acc * v % r
    inv = pow(acc, -1, r)
    out = [0] * len(vals)
    for i in range(len(vals) - 1, -1, -1):
        out[i] = pref[i] * inv % r
        inv = inv * vals[i] % r
    return out


def evaluate_points(C, P, offset: int, length: int):
    """evaluate_polynomial_points (util.cpp:186-211): x = offset..offset+len-1."""
    return [((x) % C.r, poly_eval(C, P, x % C.r)) for x in range(offset, offset + length)]


# --------------------------------------------------------------------------
# KZG API mirror (trusted_setup.cpp)
# --------------------------------------------------------------------------
def polyeval_g1(C, srs, P):
    """Naive per-term MSM exactly as trusted_setup.cpp:149-174."""
    P = normalize(P)
    if not P:
        return None                                   # :150-154
    acc = (1, 1, 0)
    for i, c in enumerate(P):                          # :156-171
        term = scalar_mul(C, srs[i], c)
        acc = _jadd(C, acc, to_jac(term))
    return to_affine(C, acc)


def commit_via_tau(C, tau, P):
    """MSM-independent check: [P(tau)]G1."""
    return scalar_mul(C, (C.gx, C.gy), poly_eval(C, normalize(P), tau))


def create_commit(C, srs, P, tau=None):
    """trusted_setup.cpp:137-142 (degree guard :138-139)."""
    if deg(P) + 1 >= len(srs):
        raise ValueError("polynomial degree be at most one less than the setup size (num_coeffs)")
    if tau is not None:
        return commit_via_tau(C, tau, P)
    return polyeval_g1(C, srs, P)


def proof_quotient(C, P, chunk_offset: int, chunk_length: int):
    """q = (P - I) / Z  (trusted_setup.cpp:214-225)."""
    if chunk_length < 1:
        raise ValueError("chunk_length must be 1 or greater")
    pts = evaluate_points(C, P, chunk_offset, chunk_length)
    I = interpolate(C, pts)
    Z = linear_roots(C, [x for x, _ in pts])
    q, _ = poly_divmod(C, poly_sub(C, P, I), Z)
    return q


def create_proof(C, srs, P, chunk_offset, chunk_length, tau=None):
    """trusted_setup.cpp:214-228 (MSM of q, :227)."""
    q = proof_quotient(C, P, chunk_offset, chunk_length)
    if tau is not None:
        return commit_via_tau(C, tau, q)
    return polyeval_g1(C, srs, q)


def create_proof_bytes(C, srs, P, byte_offset, byte_length, chunk_size, tau=None):
    """trusted_setup.cpp:203-212."""
    if chunk_size > C.max_chunk_bytes:
        raise ValueError("chunk_size must at most MAX_CHUNK_BYTES.")
    if chunk_size < 1:
        raise ValueError("chunk_size must be at least 1")
    if _cmod(byte_offset, chunk_size) != 0:
        raise ValueError("byte_offset is not a multiple of chunk_size.")
    if _cmod(byte_length, chunk_size) != 0:
        raise ValueError("byte_length is not a multiple of chun_size.")
    return create_proof(C, srs, P, _cdiv(byte_offset, chunk_size),
                        _cdiv(byte_length, chunk_size), tau)


def verify_proof_tau(C, tau, srs_len, commit, proof, points):
    """Known-tau restatement of verify_proof (trusted_setup.cpp:230-254).

    e(proof, [Z(tau)]G2) == e(C - [I(tau)]G1, G2)  <=>  [Z(tau)]proof == C - [I(tau)]G1
    by bilinearity and non-degeneracy; used only as the test oracle."""
    if len(points) < 1:
        raise ValueError("expected_data size must be 1 or greater")
    if len(points) >= srs_len:
        return False
    I = interpolate(C, points)
    Z = linear_roots(C, [x for x, _ in points])
    lhs = scalar_mul(C, proof, poly_eval(C, Z, tau)) if proof is not None else None
    rhs = point_add(C, commit, point_neg(C, scalar_mul(C, (C.gx, C.gy), poly_eval(C, I, tau))))
    return lhs == rhs


# --------------------------------------------------------------------------
# wire formats (util.cpp:78-170, trusted_setup.cpp:256-287)
# --------------------------------------------------------------------------
def ecp_octet(C, P) -> bytes:
    """ECP_toOctet(..., false): 0x04 || X || Y big-endian (util.cpp:82).
    Infinity: miracl ECP_inf is (x=0, y=1, z=0), ECP_affine leaves it, so the
    octet is 04 || 0 || 1 (not verifiable here)."""
    mb = C.modbytes
    if P is None:
        return b"\x04" + (0).to_bytes(mb, "big") + (1).to_bytes(mb, "big")
    return b"\x04" + P[0].to_bytes(mb, "big") + P[1].to_bytes(mb, "big")


def serialize_ecp(C, P) -> bytes:
    o = ecp_octet(C, P)
    return struct.pack("<I", len(o)) + o


def deserialize_ecp(C, data: bytes):
    """deserialize_ECP (util.cpp:98-115): any octet that is not a valid
    on-curve point decodes to infinity."""
    ln = struct.unpack("<I", data[:4])[0]
    o = data[4:4 + ln]
    mb = C.modbytes
    if ln != 2 * mb + 1 or o[0] != 4:
        return None
    x = int.from_bytes(o[1:1 + mb], "big")
    y = int.from_bytes(o[1 + mb:], "big")
    if x >= C.p or y >= C.p or not on_curve(C, (x, y)):
        return None
    return (x, y)


def serialize_poly(C, P) -> bytes:
    """serialize_ZZ_pX (util.cpp:118-140): i64 deg, per coeff u8 NumBytes + LE bytes."""
    P = normalize(P)
    out = bytearray(struct.pack("<q", len(P) - 1))
    for c in P:
        nb = (c.bit_length() + 7) // 8
        out.append(nb)
        out += c.to_bytes(nb, "little")
    return bytes(out)


def deserialize_poly(C, data: bytes):
    d = struct.unpack("<q", data[:8])[0]
    off = 8
    P = []
    for _ in range(d + 1):
        nb = data[off]
        off += 1
        P.append(int.from_bytes(data[off:off + nb], "little") % C.r)
        off += nb
    return normalize(P)


# --------------------------------------------------------------------------
# test helpers mirroring testing/testing.cpp
# --------------------------------------------------------------------------
def strtol16(s: str) -> int:
    """strtol(s, NULL, 16) on a <=2-char substring (testing.cpp:406-413)."""
    i = 0
    while i < len(s) and s[i] in " \t\n\v\f\r":
        i += 1
    neg = False
    if i < len(s) and s[i] in "+-":
        neg = s[i] == "-"
        i += 1
    if i + 1 < len(s) and s[i] == "0" and s[i + 1] in "xX" and i + 2 < len(s) and s[i + 2] in "0123456789abcdefABCDEF":
        i += 2
    v = 0
    while i < len(s) and s[i] in "0123456789abcdefABCDEF":
        v = v * 16 + int(s[i], 16)
        i += 1
    return (-v if neg else v) & 0xFF  # pushed into vector<uint8_t>


def from_hex(s: str) -> bytes:
    return bytes(strtol16(s[i:i + 2]) for i in range(0, len(s), 2))


def pad_chunks(C, data: bytes) -> bytes:
    """Zero pad exactly as testing.cpp:64-66 (always pads, a full chunk if aligned)."""
    m = C.max_chunk_bytes
    return data + b"\x00" * (m - len(data) % m)


def splitmix64(seed: int):
    """Deterministic scalar generator shared with the C oracle and bench."""
    x = seed & 0xFFFFFFFFFFFFFFFF
    while True:
        x = (x + 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
        z = x
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
        yield z ^ (z >> 31)


def random_scalars(C, n: int, seed: int):
    """n scalars in [0, r): 4 splitmix64 words LE, top word masked to the
    bit-length of r, rejection sampled."""
    g = splitmix64(seed)
    nb = C.r.bit_length()
    out = []
    while len(out) < n:
        v = 0
        for w in range(4):
            v |= next(g) << (64 * w)
        v &= (1 << nb) - 1
        if v < C.r:
            out.append(v)
    return out
