#!/usr/bin/env python3
"""Generate curve_consts.h: Montgomery constants for the device field code.

Curves: miracl-core BN254 (Nogami; config/curve_BN254/kzg_config.h) and
BLS12-381 (config/curve_BLS12381/kzg_config.h).  p and r are re-derived from
the curve parameters (u / x) rather than typed in, and the generators are
checked on the curve.  Limbs are 32-bit little-endian (device word size)."""
import os

U = -(2**62 + 2**55 + 1)
BN_P = 36 * U**4 + 36 * U**3 + 24 * U**2 + 6 * U + 1
BN_R = 36 * U**4 + 36 * U**3 + 18 * U**2 + 6 * U + 1
X = -0xD201000000010000
BLS_P = (X - 1) ** 2 * (X**4 - X**2 + 1) // 3 + X
BLS_R = X**4 - X**2 + 1
BLS_GX = 0x17F1D3A73197D7942695638C4FA9AC0FC3688C4F9774B905A14E3A3F171BAC586C55E83FF97A1AEFFB3AF00ADB22C6BB
BLS_GY = 0x08B3F481E3AAA0F1A09E30ED741D8AE4FCF5E095D5D00AF600DB18CB2C04B3EDD03CC744A2888AE40CAA232946C5E7E1

assert (1 - ((BN_P - 1) ** 3 + 2)) % BN_P == 0
assert (BLS_GY**2 - BLS_GX**3 - 4) % BLS_P == 0


def limbs(v, n):
    return [(v >> (32 * i)) & 0xFFFFFFFF for i in range(n)]


def arr(v, n):
    return "{" + ", ".join("0x%08xu" % w for w in limbs(v, n)) + "}"


def field(name, m, n):
    R = 1 << (32 * n)
    inv = (-pow(m, -1, 1 << 32)) % (1 << 32)
    lines = [
        "struct %s {" % name,
        "  static constexpr int N = %d;" % n,
        "  static constexpr int BITS = %d;" % m.bit_length(),
        "  static constexpr uint32_t INV = 0x%08xu;  // -m^-1 mod 2^32" % inv,
        "  static constexpr uint32_t P[N] = %s;" % arr(m, n),
        "  static constexpr uint32_t P2[N] = %s;  // 2m" % arr(2 * m, n),
        "  static constexpr uint32_t R2[N] = %s;  // R^2 mod m" % arr(R * R % m, n),
        "  static constexpr uint32_t ONE[N] = %s;  // R mod m" % arr(R % m, n),
        "  static constexpr uint32_t PM2[N] = %s;  // m - 2 (Fermat exponent)" % arr(m - 2, n),
        "};",
    ]
    return "\n".join(lines)


def limbs29(v, n):
    return [(v >> (29 * i)) & ((1 << 29) - 1) for i in range(n)]


def arr29(v, n):
    assert v < (1 << (29 * n))
    return "{" + ", ".join("0x%08xu" % w for w in limbs29(v, n)) + "}"


def field29(name, m, L):
    """radix-2^29 Montgomery constants (R = 2^(29 L)) for field29.hpp"""
    R = 1 << (29 * L)
    assert R >= 64 * m, "lazy-reduction headroom"
    inv = (-pow(m, -1, 1 << 29)) % (1 << 29)
    lines = [
        "struct %s {" % name,
        "  static constexpr int L = %d;  // 29-bit limbs" % L,
        "  static constexpr uint32_t INV = 0x%08xu;  // -m^-1 mod 2^29" % inv,
        "  static constexpr uint32_t P[L] = %s;" % arr29(m, L),
    ]
    for k in (2, 4, 6, 8, 10, 16):
        lines.append("  static constexpr uint32_t P%d[L] = %s;  // %dm" % (k, arr29(k * m, L), k))
    # 2m with every limb borrowed up into [2^29 - 1, 2^30): K - a needs no
    # carry for any a < m with normalized limbs (lazy negation, field29.hpp)
    t = limbs29(2 * m, L)
    b = [t[0] + (1 << 29)] + [t[i] + (1 << 29) - 1 for i in range(1, L - 1)] + [t[L - 1] - 1]
    assert sum(v << (29 * i) for i, v in enumerate(b)) == 2 * m and all(v < (1 << 30) for v in b)
    assert b[L - 1] >= (m - 1) >> (29 * (L - 1)) and all(v >= (1 << 29) - 1 for v in b[:L - 1])
    lines.append("  static constexpr uint32_t P2B[L] = {%s};  // 2m, limbs borrowed into [2^29-1, 2^30)" %
                 ", ".join("0x%08xu" % v for v in b))
    t = limbs29(8 * m, L)
    b = [t[0] + (1 << 29)] + [t[i] + (1 << 29) - 1 for i in range(1, L - 1)] + [t[L - 1] - 1]
    assert sum(v << (29 * i) for i, v in enumerate(b)) == 8 * m and all(v < (1 << 30) for v in b)
    # limb-wise >= every normalized a < 4m: middle limbs >= 2^29 - 1, top limb
    # >= the top limb of 4m - 1 >= a's top limb
    assert b[L - 1] >= (4 * m - 1) >> (29 * (L - 1)) and all(v >= (1 << 29) - 1 for v in b[:L - 1])
    lines.append("  static constexpr uint32_t P8B[L] = {%s};  // 8m, limbs borrowed into [2^29-1, 2^30)" %
                 ", ".join("0x%08xu" % v for v in b))
    lines += [
        "  static constexpr uint32_t R2[L] = %s;  // R^2 mod m" % arr29(R * R % m, L),
        "  static constexpr uint32_t R3[L] = %s;  // R^3 mod m" % arr29(R * R * R % m, L),
        "  static constexpr uint32_t ONE[L] = %s;  // R mod m" % arr29(R % m, L),
        "  // low limb of k m, k = 0..3 (zero filter for values < 4m)",
        "  static constexpr uint32_t LOW[4] = {0u, 0x%08xu, 0x%08xu, 0x%08xu};" % tuple(
            (k * m) & ((1 << 29) - 1) for k in (1, 2, 3)),
        "};",
    ]
    return "\n".join(lines)


def mont(v, m, n):
    return v * (1 << (32 * n)) % m


def mont29(v, m, L):
    return v * (1 << (29 * L)) % m


# --------------------------------------------------------------------------
# G2 / pairing constants (verify path: trusted_setup.cpp:123-135, 176-201,
# 230-254).  Fp2 = Fp[i]/(i^2+1), xi = 1 + i, Fp6 = Fp2[v]/(v^3 - xi),
# Fp12 = Fp6[w]/(w^2 - v).  The twist type is selected by group order: the
# sextic twist whose order is divisible by r (BN254: D-type y^2 = x^3 + b/xi,
# BLS12-381: M-type y^2 = x^3 + b xi).
# --------------------------------------------------------------------------
def _f2mul(p, a, b):
    return ((a[0] * b[0] - a[1] * b[1]) % p, (a[0] * b[1] + a[1] * b[0]) % p)


def _f2pow(p, a, e):
    r = (1, 0)
    while e:
        if e & 1:
            r = _f2mul(p, r, a)
        a = _f2mul(p, a, a)
        e >>= 1
    return r


def _f2inv(p, a):
    ni = pow((a[0] * a[0] + a[1] * a[1]) % p, -1, p)
    return (a[0] * ni % p, (-a[1]) * ni % p)


def _f2add(p, a, b):
    return ((a[0] + b[0]) % p, (a[1] + b[1]) % p)


def _f2sqrt(p, a):
    a1 = _f2pow(p, a, (p - 3) // 4)
    alpha = _f2mul(p, _f2mul(p, a1, a1), a)
    if _f2mul(p, _f2pow(p, alpha, p), alpha) == (p - 1, 0):
        return None
    x0 = _f2mul(p, a1, a)
    if alpha == (p - 1, 0):
        return _f2mul(p, (0, 1), x0)
    return _f2mul(p, _f2pow(p, _f2add(p, (1, 0), alpha), (p - 1) // 2), x0)


def _twist(p, r, b, trace):
    import math
    t2 = trace * trace - 2 * p
    f = math.isqrt((4 * p * p - t2 * t2) // 3)
    orders = {p * p + 1 - (s1 * 3 * f + s2 * t2) // 2 for s1 in (1, -1) for s2 in (1, -1)}
    orders = [n for n in orders if n % r == 0]
    assert len(orders) == 1
    return orders[0]


def _g2_smul(p, Q, k):
    def add(P, Q):
        if P is None:
            return Q
        if Q is None:
            return P
        if P[0] == Q[0]:
            if _f2add(p, P[1], Q[1]) == (0, 0):
                return None
            lam = _f2mul(p, _f2mul(p, (3, 0), _f2mul(p, P[0], P[0])), _f2inv(p, _f2mul(p, (2, 0), P[1])))
        else:
            lam = _f2mul(p, ((Q[1][0] - P[1][0]) % p, (Q[1][1] - P[1][1]) % p),
                         _f2inv(p, ((Q[0][0] - P[0][0]) % p, (Q[0][1] - P[0][1]) % p)))
        l2 = _f2mul(p, lam, lam)
        x3 = ((l2[0] - P[0][0] - Q[0][0]) % p, (l2[1] - P[0][1] - Q[0][1]) % p)
        t = _f2mul(p, lam, ((P[0][0] - x3[0]) % p, (P[0][1] - x3[1]) % p))
        return (x3, ((t[0] - P[1][0]) % p, (t[1] - P[1][1]) % p))

    R = None
    for bit in bin(k)[2:]:
        R = add(R, R)
        if bit == "1":
            R = add(R, Q)
    return R


BLS_G2 = ((0x024AA2B2F08F0A91260805272DC51051C6E47AD4FA403B02B4510B647AE3D1770BAC0326A805BBEFD48056C8C121BDB8,
           0x13E02B6052719F607DACD3A088274F65596BD0D09920B61AB5DA61BBDC7F5049334CF11213945D57E5AC7D055D042B7E),
          (0x0CE5D527727D6E118CC9CDC6DA2E351AADFD9BAA8CBDD3A76D429A695160D12C923AC9CC3BACA289E193548608B82801,
           0x0606C4A02EA734CC32ACD2B02BC28B99CB3E287E85A763AF267492AB572E99AB3F370D275CEC1DA1AAA9075FF05F79BE))


def g2_data(name):
    """twist, G2 generator, Frobenius constants, loop and hard-part digits"""
    if name == "BN254":
        p, r, b, trace = BN_P, BN_R, 2, 6 * U * U + 1
    else:
        p, r, b, trace = BLS_P, BLS_R, 4, X + 1
    order = _twist(p, r, b, trace)
    xi = (1, 1)
    d_type = name == "BN254"
    b2 = _f2mul(p, (b, 0), _f2inv(p, xi)) if d_type else _f2mul(p, (b, 0), xi)
    if name == "BLS12381":
        gen = BLS_G2
    else:  # deterministic: first x = k + i on the twist, smaller root, cofactor cleared
        k = 1
        while True:
            x = (k, 1)
            y = _f2sqrt(p, _f2add(p, _f2mul(p, _f2mul(p, x, x), x), b2))
            if y is not None:
                ny = ((-y[0]) % p, (-y[1]) % p)
                if (ny[1], ny[0]) < (y[1], y[0]):
                    y = ny
                gen = _g2_smul(p, (x, y), order // r)
                if gen is not None:
                    break
            k += 1
    assert _g2_smul(p, gen, r) is None
    frob = [_f2pow(p, xi, kk * (p - 1) // 6) for kk in range(6)]
    twx = _f2pow(p, xi, (p - 1) // 3)
    twy = _f2pow(p, xi, (p - 1) // 2)
    loop = 6 * U + 2 if name == "BN254" else X
    hard = (p ** 4 - p ** 2 + 1) // r
    digits = []
    for _ in range(4):
        digits.append(hard % p)
        hard //= p
    assert hard == 0
    z = U if name == "BN254" else X
    k3 = (X - 1) ** 2 // 3 if name == "BLS12381" else 0
    return dict(p=p, b2=b2, gen=gen, frob=frob, twx=twx, twy=twy, loop=loop, digits=digits, d_type=d_type, z=z, k3=k3)


def pairing_struct(name, L, nw):
    d = g2_data(name)
    p = d["p"]

    def m29(v):
        return arr29(mont29(v, p, L), L)

    def f2(a):
        return "{%s, %s}" % (m29(a[0]), m29(a[1]))

    lines = [
        "struct %sPair {" % name,
        "  static constexpr bool D_TWIST = %s;  // D: y^2 = x^3 + b/xi, M: y^2 = x^3 + b xi" % (
            "true" if d["d_type"] else "false"),
        "  static constexpr uint32_t B2[2][%d] = %s;  // twist b' (radix-2^29 Montgomery)" % (L, f2(d["b2"])),
        "  static constexpr uint32_t G2X[2][%d] = %s;" % (L, f2(d["gen"][0])),
        "  static constexpr uint32_t G2Y[2][%d] = %s;" % (L, f2(d["gen"][1])),
        "  // Fp12 Frobenius: coefficient of w^k picks up xi^(k (p-1)/6)",
        "  static constexpr uint32_t FROB[6][2][%d] = {%s};" % (L, ", ".join(f2(g) for g in d["frob"])),
        "  // twist Frobenius (D-type): x -> conj(x) xi^((p-1)/3), y -> conj(y) xi^((p-1)/2)",
        "  static constexpr uint32_t TWX[2][%d] = %s;" % (L, f2(d["twx"])),
        "  static constexpr uint32_t TWY[2][%d] = %s;" % (L, f2(d["twy"])),
        "  // Miller loop count |%s| (LOOP_BITS bits, two 64-bit words)" % ("6u+2" if name == "BN254" else "x"),
        "  static constexpr uint64_t LOOP[2] = {0x%016xull, 0x%016xull};" % (abs(d["loop"]) & (2**64 - 1), abs(d["loop"]) >> 64),
        "  static constexpr int LOOP_BITS = %d;" % abs(d["loop"]).bit_length(),
        "  static constexpr bool LOOP_NEG = %s;" % ("true" if d["loop"] < 0 else "false"),
        "  static constexpr int NW = %d;" % nw,
        "  // (p^4 - p^2 + 1)/r = sum_i HARD[i] p^i (canonical words)",
        "  static constexpr uint32_t HARD[4][%d] = {%s};" % (nw, ", ".join(arr(v, nw) for v in d["digits"])),
        "  static constexpr int HARD_BITS = %d;" % max(v.bit_length() for v in d["digits"]),
        "  // curve parameter z (BN: u, BLS: x) for the hard part of the final exponentiation",
        "  static constexpr bool IS_BN = %s;" % ("true" if name == "BN254" else "false"),
        "  static constexpr uint64_t Z_ABS = 0x%016xull;" % abs(d["z"]),
        "  static constexpr bool Z_NEG = %s;" % ("true" if d["z"] < 0 else "false"),
        "  // BLS12: (p^4 - p^2 + 1)/r = K3 (x + p)(x^2 + p^2 - 1) + 1, K3 = (x - 1)^2 / 3",
        "  static constexpr uint64_t K3[2] = {0x%016xull, 0x%016xull};" % (d["k3"] & (2**64 - 1), d["k3"] >> 64),
        "  static constexpr int K3_BITS = %d;" % d["k3"].bit_length(),
        "};",
    ]
    return "\n".join(lines)


def main():
    out = [
        "// GENERATED by gen_consts.py -- do not edit.",
        "#pragma once",
        "#include <stdint.h>",
        "namespace kzgx {",
        field("BN254Fp", BN_P, 8),
        field("BN254Fr", BN_R, 8),
        field("BLS12381Fp", BLS_P, 12),
        field("BLS12381Fr", BLS_R, 8),
        field29("BN254Fp29", BN_P, 9),
        field29("BLS12381Fp29", BLS_P, 14),
        # the scalar fields in radix 2^29: their inversion by f29_inv_uniform
        # (poly.hip fe_inv_wave, the interpolation weights)
        field29("BN254Fr29", BN_R, 9),
        field29("BLS12381Fr29", BLS_R, 9),
        "struct BN254G1 {",
        "  using Fp = BN254Fp;",
        "  using Fp29 = BN254Fp29;",
        "  using Fr = BN254Fr;",
        "  static constexpr int ID = 0;",
        "  static constexpr uint32_t BSMALL = 2;  // y^2 = x^3 + 2",
        "  static constexpr int SCALAR_BITS = %d;" % BN_R.bit_length(),
        "  static constexpr uint32_t GX[8] = %s;  // Montgomery" % arr(mont(BN_P - 1, BN_P, 8), 8),
        "  static constexpr uint32_t GY[8] = %s;" % arr(mont(1, BN_P, 8), 8),
        "  static constexpr uint32_t B[8] = %s;" % arr(mont(2, BN_P, 8), 8),
        "  static constexpr uint32_t GX29[9] = %s;  // radix-2^29 Montgomery" % arr29(mont29(BN_P - 1, BN_P, 9), 9),
        "  static constexpr uint32_t GY29[9] = %s;" % arr29(mont29(1, BN_P, 9), 9),
        "};",
        "struct BLS12381G1 {",
        "  using Fp = BLS12381Fp;",
        "  using Fp29 = BLS12381Fp29;",
        "  using Fr = BLS12381Fr;",
        "  static constexpr int ID = 1;",
        "  static constexpr uint32_t BSMALL = 4;  // y^2 = x^3 + 4",
        "  static constexpr int SCALAR_BITS = %d;" % BLS_R.bit_length(),
        "  static constexpr uint32_t GX[12] = %s;" % arr(mont(BLS_GX, BLS_P, 12), 12),
        "  static constexpr uint32_t GY[12] = %s;" % arr(mont(BLS_GY, BLS_P, 12), 12),
        "  static constexpr uint32_t B[12] = %s;" % arr(mont(4, BLS_P, 12), 12),
        "  static constexpr uint32_t GX29[14] = %s;" % arr29(mont29(BLS_GX, BLS_P, 14), 14),
        "  static constexpr uint32_t GY29[14] = %s;" % arr29(mont29(BLS_GY, BLS_P, 14), 14),
        "};",
        pairing_struct("BN254", 9, 8),
        pairing_struct("BLS12381", 14, 12),
        "}  // namespace kzgx",
        "",
    ]
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "curve_consts.h")
    text = "\n".join(out)
    # unchanged constants leave the header (and its mtime) alone: every object
    # includes it, so a rewrite would make build() recompile everything
    if os.path.exists(path):
        with open(path) as f:
            if f.read() == text:
                return
    with open(path, "w") as f:
        f.write(text)


if __name__ == "__main__":
    main()
