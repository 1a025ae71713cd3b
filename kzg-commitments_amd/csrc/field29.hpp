// Base-field (Fp) arithmetic for the G1 hot path on gfx950: radix-2^29
// Montgomery with lazy reduction.
//
// Why radix 2^29 (measured, scripts/micro_valu.hip, profiles/r01_micro_valu.txt):
// on gfx950 v_mad_u64_u32 issues at about the cost of any other 64-bit /
// carry-out VALU op (~4.5-5 SIMD cycles per wave-instruction), so the cost of
// a 32-bit-limb CIOS product is dominated by the carry glue around each mad
// (v_lshl_add_u64 + v_mov pairs: ~600 instructions per product).  With 29-bit
// limbs every partial product fits a single v_mad_u64_u32 that accumulates
// into a 64-bit column sum with >= 2 bits of headroom per column (product
// scanning / FIPS), so a product is one mad per partial product plus a shift
// and a mask per column: 1.6x faster per multiplication.
//
// Lazy reduction: R = 2^(29 L) >= 64 m (BN254: L = 9, R/m ~ 222; BLS12-381:
// L = 14), so a Montgomery product of inputs a, b with a b < (R/m) m^2 comes
// out < 2m with no final subtraction.  Additions and subtractions are plain
// carry-propagated limb arithmetic with a multiple of m added to keep
// subtractions non-negative; curve.hpp documents the bound of every value.
// Only equality tests and the final output need a full reduction.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "curve_consts.h"

#ifndef KZGX_DEV
#define KZGX_DEV __device__ __forceinline__
#endif

namespace kzgx {

constexpr uint32_t M29 = (1u << 29) - 1;

template <class F>
struct F29 {
  uint32_t v[F::L];
};

template <class F>
KZGX_DEV F29<F> f29_const(const uint32_t (&c)[F::L]) {
  F29<F> r;
#pragma unroll
  for (int i = 0; i < F::L; i++) r.v[i] = c[i];
  return r;
}

template <class F>
KZGX_DEV F29<F> f29_zero() {
  F29<F> r;
#pragma unroll
  for (int i = 0; i < F::L; i++) r.v[i] = 0;
  return r;
}

template <class F>
KZGX_DEV F29<F> f29_one() {
  return f29_const<F>(F::ONE);
}

template <class F>
KZGX_DEV bool f29_is_zero_exact(const F29<F>& a) {
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < F::L; i++) o |= a.v[i];
  return o == 0;
}

// a + b, carry propagated (no modular reduction; caller tracks the bound)
template <class F>
KZGX_DEV F29<F> f29_add(const F29<F>& a, const F29<F>& b) {
  F29<F> r;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < F::L; i++) {
    uint32_t s = a.v[i] + b.v[i] + c;
    r.v[i] = s & M29;
    c = s >> 29;
  }
  return r;
}

// a + K - b where K = k m >= b (so the result is non-negative)
template <class F>
KZGX_DEV F29<F> f29_sub(const F29<F>& a, const F29<F>& b, const uint32_t (&K)[F::L]) {
  F29<F> r;
  int32_t c = 0;
#pragma unroll
  for (int i = 0; i < F::L; i++) {
    int32_t s = (int32_t)(a.v[i] + K[i]) - (int32_t)b.v[i] + c;
    r.v[i] = (uint32_t)s & M29;
    c = s >> 29;  // arithmetic shift: -1, 0 or 1
  }
  return r;
}

// Modulus limb j as an opaque uniform value (BN254).  Left as a literal, a
// limb that is a power of two (BN254: 2^25) is strength-reduced to a 64-bit
// shift plus a 64-bit add -- two VALU issues where v_mad_u64_u32 with an SGPR
// operand is one.  The asm is pure (not volatile), so it is hoisted out of
// loops.
template <class F>
KZGX_DEV uint32_t f29_pl(int j) {
#ifndef KZGX_SGPR_PL_ALL
  // BLS12-381 (14 limbs): pinning its limbs in SGPRs spills SGPRs to
  // scratch in every point-addition kernel (111 SGPR spills, 172 B/lane of
  // scratch in the mixed-add loop, -Rpass-analysis=kernel-resource-usage);
  // left as literals they cost no scratch
  if (F::L > 9) return F::P[j];
#endif
  uint32_t r;
  asm("" : "=s"(r) : "0"(F::P[j]));
  return r;
}

// acc += x y as one v_mad_u64_u32.  With KZGX_ASM_MAD each column is a
// single dependent chain (the compiler cannot re-associate it into two
// chains that then need a 64-bit merge per column); otherwise plain C.
KZGX_DEV void mad_vv(uint64_t& acc, uint32_t x, uint32_t y) {
  acc += (uint64_t)x * y;
#ifdef KZGX_ASM_MAD
  asm("" : "+v"(acc));
#endif
}
KZGX_DEV void mad_vs(uint64_t& acc, uint32_t x, uint32_t y_uniform) {
  acc += (uint64_t)x * y_uniform;
#ifdef KZGX_ASM_MAD
  asm("" : "+v"(acc));
#endif
}

// Latency-first Montgomery product for code that runs as a lone wave (the
// verify path): the same value and bounds as f29_mul, arranged for a short
// dependency chain instead of few instructions.  f29_mul threads every
// partial product of every column through ONE accumulator (a ~2L^2-long
// dependent mad chain: fine when other waves fill the SIMD, ~15 cycles per
// mad when the wave is alone).  Here the 2L - 1 column sums are independent
// chains of <= L mads, and only the reduction digits form a chain (L steps
// of digit, mad, shift).  Column bound: 2L products < 2^58 plus a carry,
// < 2^63 for both curves.
template <class F>
KZGX_DEV F29<F> f29_mul_lat(const F29<F>& a, const F29<F>& b) {
  constexpr int L = F::L;
  uint64_t col[2 * L];
#pragma unroll
  for (int k = 0; k < 2 * L - 1; k++) {
    uint64_t s = 0;
#pragma unroll
    for (int i = 0; i < L; i++) {
      const int j = k - i;
      if (j >= 0 && j < L) s += (uint64_t)a.v[i] * b.v[j];
    }
    col[k] = s;
  }
  col[2 * L - 1] = 0;
#pragma unroll
  for (int k = 0; k < L; k++) {
    const uint32_t q = ((uint32_t)col[k] * F::INV) & M29;
    // modulus limbs as opaque uniform values (f29_pl): one v_mad_u64_u32
    // each, never strength-reduced to shifts and adds
    col[k + 1] += (col[k] + (uint64_t)q * f29_pl<F>(0)) >> 29;
#pragma unroll
    for (int j = 1; j < L; j++) col[k + j] += (uint64_t)q * f29_pl<F>(j);
  }
  F29<F> t;
  uint64_t c = 0;
#pragma unroll
  for (int k = L; k < 2 * L - 1; k++) {
    const uint64_t s = col[k] + c;
    t.v[k - L] = (uint32_t)s & M29;
    c = s >> 29;
  }
  t.v[L - 1] = (uint32_t)c;
  return t;
}

// (a b + c d) / R, latency-first (f29_mul2's value and bounds): column
// sums 2L products + L reduction terms < 2^58 each, < 2^64 for both curves
template <class F>
KZGX_DEV F29<F> f29_mul2_lat(const F29<F>& a, const F29<F>& b, const F29<F>& c, const F29<F>& d) {
  constexpr int L = F::L;
  uint64_t col[2 * L];
#pragma unroll
  for (int k = 0; k < 2 * L - 1; k++) {
    uint64_t s = 0;
#pragma unroll
    for (int i = 0; i < L; i++) {
      const int j = k - i;
      if (j >= 0 && j < L) s += (uint64_t)a.v[i] * b.v[j] + (uint64_t)c.v[i] * d.v[j];
    }
    col[k] = s;
  }
  col[2 * L - 1] = 0;
#pragma unroll
  for (int k = 0; k < L; k++) {
    const uint32_t q = ((uint32_t)col[k] * F::INV) & M29;
    col[k + 1] += (col[k] + (uint64_t)q * f29_pl<F>(0)) >> 29;
#pragma unroll
    for (int j = 1; j < L; j++) col[k + j] += (uint64_t)q * f29_pl<F>(j);
  }
  F29<F> t;
  uint64_t cy = 0;
#pragma unroll
  for (int k = L; k < 2 * L - 1; k++) {
    const uint64_t s = col[k] + cy;
    t.v[k - L] = (uint32_t)s & M29;
    cy = s >> 29;
  }
  t.v[L - 1] = (uint32_t)cy;
  return t;
}

// Montgomery product a b / R mod m, product scanning; output < 2m when
// a b < (R / m) m^2 (see header).  A translation unit that defines
// KZGX_FIELD_LATENCY before including this header (verify_wave.hip: one
// wave per pairing) gets the latency-first form for every f29_mul /
// f29_sqr, including those inside the tower and curve code.
template <class F>
KZGX_DEV F29<F> f29_mul(const F29<F>& a, const F29<F>& b) {
#ifdef KZGX_FIELD_LATENCY
  return f29_mul_lat<F>(a, b);
#endif
  constexpr int L = F::L;
  uint32_t q[L];
  F29<F> t;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 2 * L - 1; k++) {
#pragma unroll
    for (int i = 0; i < L; i++) {
      const int j = k - i;
      if (j >= 0 && j < L) mad_vv(acc, a.v[i], b.v[j]);
    }
#pragma unroll
    for (int i = 0; i < L; i++) {
      const int j = k - i;
      if (i < k && j >= 1 && j < L) mad_vs(acc, q[i], f29_pl<F>(j));
    }
    if (k < L) {
      q[k] = ((uint32_t)acc * F::INV) & M29;
      mad_vs(acc, q[k], f29_pl<F>(0));
    } else {
      t.v[k - L] = (uint32_t)acc & M29;
    }
    acc >>= 29;
  }
  t.v[L - 1] = (uint32_t)acc;
  return t;
}

// (a b + c d) / R mod m with ONE reduction (sum of products before REDC).
// Column sums stay below 2^64: 2L products + L reduction terms < 2^58 each.
// Output < 2m when a b + c d < (R / m) m^2.
template <class F>
KZGX_DEV F29<F> f29_mul2(const F29<F>& a, const F29<F>& b, const F29<F>& c, const F29<F>& d) {
#ifdef KZGX_FIELD_LATENCY
  return f29_mul2_lat<F>(a, b, c, d);
#endif
  constexpr int L = F::L;
  uint32_t q[L];
  F29<F> t;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 2 * L - 1; k++) {
#pragma unroll
    for (int i = 0; i < L; i++) {
      const int j = k - i;
      if (j >= 0 && j < L) {
        mad_vv(acc, a.v[i], b.v[j]);
        mad_vv(acc, c.v[i], d.v[j]);
      }
    }
#pragma unroll
    for (int i = 0; i < L; i++) {
      const int j = k - i;
      if (i < k && j >= 1 && j < L) mad_vs(acc, q[i], f29_pl<F>(j));
    }
    if (k < L) {
      q[k] = ((uint32_t)acc * F::INV) & M29;
      mad_vs(acc, q[k], f29_pl<F>(0));
    } else {
      t.v[k - L] = (uint32_t)acc & M29;
    }
    acc >>= 29;
  }
  t.v[L - 1] = (uint32_t)acc;
  return t;
}

// acc += x y with the sum pinned to one dependent chain (the asm is an
// opaque identity on acc: the compiler can neither re-associate the column
// into two chains nor merge them back with a 64-bit add)
KZGX_DEV void mad_chain(uint64_t& acc, uint32_t x, uint32_t y) {
#if defined(KZGX_MAD_S100)
  asm("v_mad_u64_u32 %0, s[100:101], %1, %2, %0" : "+v"(acc) : "v"(x), "v"(y) : "s100", "s101");
#elif defined(KZGX_MAD_VCC)
  asm("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(acc) : "v"(x), "v"(y) : "vcc");
#else
  acc += (uint64_t)x * y;
  asm("" : "+v"(acc));
#endif
}
// the same with a wave-uniform second factor (a modulus limb in an SGPR)
KZGX_DEV void mad_chain_s(uint64_t& acc, uint32_t x, uint32_t y_uniform) {
#if defined(KZGX_MAD_S100)
  asm("v_mad_u64_u32 %0, s[100:101], %1, %2, %0" : "+v"(acc) : "v"(x), "v"(y_uniform) : "s100", "s101");
#elif defined(KZGX_MAD_VCC)
  asm("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(acc) : "v"(x), "v"(y_uniform) : "vcc");
#else
  acc += (uint64_t)x * y_uniform;
  asm("" : "+v"(acc));
#endif
}

// compile-time loop: f(std::integral_constant<int, K>) for K in [K0, K1)
template <int K0, int K1, class Fn>
KZGX_DEV void static_for(Fn&& f) {
  if constexpr (K0 < K1) {
    f(std::integral_constant<int, K0>{});
    static_for<K0 + 1, K1>(f);
  }
}

// One Montgomery product's column state for the chained forms below: the
// 64-bit column accumulator and the reduction digits so far.
template <class F>
struct MontChain {
  uint64_t acc;
  uint32_t q[F::L];
};

// column K of a b into the chain
template <class F, int K>
KZGX_DEV void mc_prod(MontChain<F>& c, const F29<F>& a, const F29<F>& b) {
#pragma unroll
  for (int i = 0; i < F::L; i++) {
    const int j = K - i;
    if (j >= 0 && j < F::L) mad_chain(c.acc, a.v[i], b.v[j]);
  }
}

// column K of a^2 (dd = 2a limb-wise)
template <class F, int K>
KZGX_DEV void mc_sqr(MontChain<F>& c, const F29<F>& a, const F29<F>& dd) {
#pragma unroll
  for (int i = 0; i < F::L; i++) {
    const int j = K - i;
    if (j > i && j < F::L) mad_chain(c.acc, a.v[i], dd.v[j]);
  }
  if constexpr ((K & 1) == 0 && (K >> 1) < F::L) mad_chain(c.acc, a.v[K >> 1], a.v[K >> 1]);
}

// the reduction terms of column K, then its digit (K < L) or output limb,
// then the carry into column K + 1
template <class F, int K>
KZGX_DEV void mc_reduce(MontChain<F>& c, F29<F>& r, const uint32_t (&pl)[F::L]) {
  constexpr int L = F::L;
#pragma unroll
  for (int i = 0; i < L; i++) {
    const int j = K - i;
    if (i < K && j >= 1 && j < L) mad_chain_s(c.acc, c.q[i], pl[j]);
  }
  if constexpr (K < L) {
    c.q[K] = ((uint32_t)c.acc * F::INV) & M29;
    mad_chain_s(c.acc, c.q[K], pl[0]);
  } else {
    r.v[K - L] = (uint32_t)c.acc & M29;
  }
  c.acc >>= 29;
  if constexpr (K == 2 * L - 2) r.v[L - 1] = (uint32_t)c.acc;
}

// the modulus limbs of the chained products, once per call: BN254 as the
// opaque uniform (SGPR) values of f29_pl -- the mads read them as their
// SGPR operand, where opaque VGPR copies were rematerialised with 14 v_mov
// per table term (steady-state non-mad VALU 761.9 -> 743.9,
// scripts/isa_count.py; cfg2 +0.9% interleaved, profiles/r04_ab_pl_sgpr_cfg2.json);
// BLS12-381 keeps opaque VGPR copies (f29_pl leaves its 14 limbs literal to
// avoid SGPR spills).  KZGX_PL_VGPR / KZGX_PL_SGPR force one form (A/B).
template <class F>
struct PLimbs {
  uint32_t v[F::L];
  KZGX_DEV PLimbs() {
#if defined(KZGX_PL_SGPR)
    constexpr bool sg = true;
#elif defined(KZGX_PL_VGPR)
    constexpr bool sg = false;
#else
    constexpr bool sg = F::L <= 9;
#endif
#pragma unroll
    for (int j = 0; j < F::L; j++) {
      if constexpr (sg)
        v[j] = f29_pl<F>(j);
      else
        asm("" : "=v"(v[j]) : "0"(F::P[j]));
    }
  }
};

// ---- Paired chains (KZGX_MAD_PAIR) ----
// The scheduler runs each of two independent column chains for several
// columns before it switches to the other, so consecutive mads read each
// other's result: every one waits out the mad's latency and carries the
// `s_nop 0` that gfx950's hazard rule puts between two dependent 64-bit VALU
// results (hipcc -S).  Here one asm statement advances both chains by one mad,
// so the two mads of a step are independent and the next step's first mad
// is one instruction behind its producer (the one wait state the rule asks).
// The unused carry-out goes to a scratch SGPR pair.
KZGX_DEV void mad_pair(uint64_t& a0, uint32_t x0, uint32_t y0, uint64_t& a1, uint32_t x1, uint32_t y1) {
  uint64_t cc;
  asm("v_mad_u64_u32 %0, %2, %3, %4, %0\n\tv_mad_u64_u32 %1, %2, %5, %6, %1"
      : "+v"(a0), "+v"(a1), "=&s"(cc)
      : "v"(x0), "v"(y0), "v"(x1), "v"(y1));
}

// column K of a0 b0 and of a1 b1, in lockstep
template <class F, int K>
KZGX_DEV void mc_prod2(MontChain<F>& c0, const F29<F>& a0, const F29<F>& b0, MontChain<F>& c1, const F29<F>& a1,
                       const F29<F>& b1) {
#pragma unroll
  for (int i = 0; i < F::L; i++) {
    const int j = K - i;
    if (j >= 0 && j < F::L) mad_pair(c0.acc, a0.v[i], b0.v[j], c1.acc, a1.v[i], b1.v[j]);
  }
}

// column K of a0^2 and of a1^2 (dd = 2a limb-wise), in lockstep
template <class F, int K>
KZGX_DEV void mc_sqr2(MontChain<F>& c0, const F29<F>& a0, const F29<F>& dd0, MontChain<F>& c1, const F29<F>& a1,
                      const F29<F>& dd1) {
#pragma unroll
  for (int i = 0; i < F::L; i++) {
    const int j = K - i;
    if (j > i && j < F::L) mad_pair(c0.acc, a0.v[i], dd0.v[j], c1.acc, a1.v[i], dd1.v[j]);
  }
  if constexpr ((K & 1) == 0 && (K >> 1) < F::L)
    mad_pair(c0.acc, a0.v[K >> 1], a0.v[K >> 1], c1.acc, a1.v[K >> 1], a1.v[K >> 1]);
}

// mc_reduce of two chains in lockstep
template <class F, int K>
KZGX_DEV void mc_reduce2(MontChain<F>& c0, F29<F>& r0, MontChain<F>& c1, F29<F>& r1, const uint32_t (&pl)[F::L]) {
  constexpr int L = F::L;
#pragma unroll
  for (int i = 0; i < L; i++) {
    const int j = K - i;
    if (i < K && j >= 1 && j < L) mad_pair(c0.acc, c0.q[i], pl[j], c1.acc, c1.q[i], pl[j]);
  }
  if constexpr (K < L) {
    c0.q[K] = ((uint32_t)c0.acc * F::INV) & M29;
    c1.q[K] = ((uint32_t)c1.acc * F::INV) & M29;
    mad_pair(c0.acc, c0.q[K], pl[0], c1.acc, c1.q[K], pl[0]);
  } else {
    r0.v[K - L] = (uint32_t)c0.acc & M29;
    r1.v[K - L] = (uint32_t)c1.acc & M29;
  }
  c0.acc >>= 29;
  c1.acc >>= 29;
  if constexpr (K == 2 * L - 2) {
    r0.v[L - 1] = (uint32_t)c0.acc;
    r1.v[L - 1] = (uint32_t)c1.acc;
  }
}

// ---- Three chains in lockstep ----
// gfx950 wants two wait states between a v_mad_u64_u32 and a VALU that reads
// its result (hipcc -S: an `s_nop 0` wherever only one instruction separates
// them, so two chains in lockstep still pay one pad per pair of mads).  With
// three independent chains advanced round-robin every mad is two instructions
// behind its producer: no pad at all.  Each pad costs about a quarter of a mad
// issue at three waves per SIMD (scripts/micro_chain.hip,
// profiles/r03_micro_chain.txt).
KZGX_DEV void mad_tri(uint64_t& a0, uint32_t x0, uint32_t y0, uint64_t& a1, uint32_t x1, uint32_t y1, uint64_t& a2,
                      uint32_t x2, uint32_t y2) {
  uint64_t cc;
  asm("v_mad_u64_u32 %0, %3, %4, %5, %0\n\tv_mad_u64_u32 %1, %3, %6, %7, %1\n\tv_mad_u64_u32 %2, %3, %8, %9, %2"
      : "+v"(a0), "+v"(a1), "+v"(a2), "=&s"(cc)
      : "v"(x0), "v"(y0), "v"(x1), "v"(y1), "v"(x2), "v"(y2));
}
// the same, the third chain starting from zero (a fresh column of a split
// accumulator: src2 is the inline constant 0, no register to clear)
KZGX_DEV void mad_tri_z(uint64_t& a0, uint32_t x0, uint32_t y0, uint64_t& a1, uint32_t x1, uint32_t y1, uint64_t& a2,
                        uint32_t x2, uint32_t y2) {
  uint64_t cc;
  asm("v_mad_u64_u32 %0, %3, %4, %5, %0\n\tv_mad_u64_u32 %1, %3, %6, %7, %1\n\tv_mad_u64_u32 %2, %3, %8, %9, 0"
      : "+v"(a0), "+v"(a1), "=&v"(a2), "=&s"(cc)
      : "v"(x0), "v"(y0), "v"(x1), "v"(y1), "v"(x2), "v"(y2));
}

// column K of three products, in lockstep
template <class F, int K>
KZGX_DEV void mc_prod3(MontChain<F>& c0, const F29<F>& a0, const F29<F>& b0, MontChain<F>& c1, const F29<F>& a1,
                       const F29<F>& b1, MontChain<F>& c2, const F29<F>& a2, const F29<F>& b2) {
#pragma unroll
  for (int i = 0; i < F::L; i++) {
    const int j = K - i;
    if (j >= 0 && j < F::L) mad_tri(c0.acc, a0.v[i], b0.v[j], c1.acc, a1.v[i], b1.v[j], c2.acc, a2.v[i], b2.v[j]);
  }
}

// mc_reduce of three chains in lockstep
template <class F, int K>
KZGX_DEV void mc_reduce3(MontChain<F>& c0, F29<F>& r0, MontChain<F>& c1, F29<F>& r1, MontChain<F>& c2, F29<F>& r2,
                         const uint32_t (&pl)[F::L]) {
  constexpr int L = F::L;
#pragma unroll
  for (int i = 0; i < L; i++) {
    const int j = K - i;
    if (i < K && j >= 1 && j < L) mad_tri(c0.acc, c0.q[i], pl[j], c1.acc, c1.q[i], pl[j], c2.acc, c2.q[i], pl[j]);
  }
  if constexpr (K < L) {
    c0.q[K] = ((uint32_t)c0.acc * F::INV) & M29;
    c1.q[K] = ((uint32_t)c1.acc * F::INV) & M29;
    c2.q[K] = ((uint32_t)c2.acc * F::INV) & M29;
    mad_tri(c0.acc, c0.q[K], pl[0], c1.acc, c1.q[K], pl[0], c2.acc, c2.q[K], pl[0]);
  } else {
    r0.v[K - L] = (uint32_t)c0.acc & M29;
    r1.v[K - L] = (uint32_t)c1.acc & M29;
    r2.v[K - L] = (uint32_t)c2.acc & M29;
  }
  c0.acc >>= 29;
  c1.acc >>= 29;
  c2.acc >>= 29;
  if constexpr (K == 2 * L - 2) {
    r0.v[L - 1] = (uint32_t)c0.acc;
    r1.v[L - 1] = (uint32_t)c1.acc;
    r2.v[L - 1] = (uint32_t)c2.acc;
  }
}

// r0 = a0 b0 / R, r1 = a1 b1 / R, r2 = a2 b2 / R: three chains in lockstep
template <class F>
KZGX_DEV void f29_mul_x3(const F29<F>& a0, const F29<F>& b0, const F29<F>& a1, const F29<F>& b1, const F29<F>& a2,
                         const F29<F>& b2, F29<F>& r0, F29<F>& r1, F29<F>& r2) {
  const PLimbs<F> pl;
  MontChain<F> c0, c1, c2;
  c0.acc = c1.acc = c2.acc = 0;
  static_for<0, 2 * F::L - 1>([&](auto kc) {
    constexpr int k = decltype(kc)::value;
    mc_prod3<F, k>(c0, a0, b0, c1, a1, b1, c2, a2, b2);
    mc_reduce3<F, k>(c0, r0, c1, r1, c2, r2, pl.v);
  });
}

// f29_sqr_x2 with the two chains in lockstep (mad_pair) whatever
// KZGX_MAD_PAIR says: for latency-bound callers (few waves per SIMD), where
// a lone chain pays every hazard pad
template <class F>
KZGX_DEV void f29_sqr_x2_pair(const F29<F>& a0, const F29<F>& a1, F29<F>& r0, F29<F>& r1) {
  F29<F> d0, d1;
#pragma unroll
  for (int i = 0; i < F::L; i++) {
    d0.v[i] = a0.v[i] << 1;
    d1.v[i] = a1.v[i] << 1;
  }
  const PLimbs<F> pl;
  MontChain<F> c0, c1;
  c0.acc = c1.acc = 0;
  static_for<0, 2 * F::L - 1>([&](auto kc) {
    constexpr int k = decltype(kc)::value;
    mc_sqr2<F, k>(c0, a0, d0, c1, a1, d1);
    mc_reduce2<F, k>(c0, r0, c1, r1, pl.v);
  });
}

// r0 = (a b + c d) / R with one reduction, r1 = e f / R.  The products run as
// three chains in lockstep (c d into a second accumulator of r0 that starts
// from zero every column and is merged before the column's reduction), the
// reductions as a pair.  Same bounds as f29_mul2 / f29_mul.
template <class F>
KZGX_DEV void f29_mul2_mul(const F29<F>& a, const F29<F>& b, const F29<F>& c, const F29<F>& d, const F29<F>& e,
                           const F29<F>& f, F29<F>& r0, F29<F>& r1) {
  const PLimbs<F> pl;
  MontChain<F> c0, c1;
  c0.acc = c1.acc = 0;
  static_for<0, 2 * F::L - 1>([&](auto kc) {
    constexpr int K = decltype(kc)::value;
    constexpr int i0 = K < F::L ? 0 : K - F::L + 1;  // first term of column K
    uint64_t side;
    mad_tri_z(c0.acc, a.v[i0], b.v[K - i0], c1.acc, e.v[i0], f.v[K - i0], side, c.v[i0], d.v[K - i0]);
#pragma unroll
    for (int i = i0 + 1; i < F::L; i++) {
      const int j = K - i;
      if (j >= 0) mad_tri(c0.acc, a.v[i], b.v[j], c1.acc, e.v[i], f.v[j], side, c.v[i], d.v[j]);
    }
    c0.acc += side;
    mc_reduce2<F, K>(c0, r0, c1, r1, pl.v);
  });
}

// Independent Montgomery products computed side by side, every column of
// every product ONE dependent v_mad_u64_u32 chain that starts from the
// previous column's carry: a shift per column and no merge of two partial
// chains (the compiler splits a lone product's columns into two chains for
// latency and pays a 64-bit add per column to join them).  The chains of the
// different products are independent: with KZGX_MAD_PAIR they advance in
// lockstep (mad_pair), otherwise the scheduler interleaves them.
// Same output bounds as f29_mul / f29_sqr / f29_mul2.
template <class F>
KZGX_DEV void f29_mul_x2(const F29<F>& a0, const F29<F>& b0, const F29<F>& a1, const F29<F>& b1, F29<F>& r0,
                         F29<F>& r1) {
  const PLimbs<F> pl;
  MontChain<F> c0, c1;
  c0.acc = c1.acc = 0;
  static_for<0, 2 * F::L - 1>([&](auto kc) {
    constexpr int k = decltype(kc)::value;
#ifdef KZGX_MAD_PAIR
    mc_prod2<F, k>(c0, a0, b0, c1, a1, b1);
    mc_reduce2<F, k>(c0, r0, c1, r1, pl.v);
#else
    mc_prod<F, k>(c0, a0, b0);
    mc_prod<F, k>(c1, a1, b1);
    mc_reduce<F, k>(c0, r0, pl.v);
    mc_reduce<F, k>(c1, r1, pl.v);
#endif
  });
}

template <class F>
KZGX_DEV void f29_sqr_x2(const F29<F>& a0, const F29<F>& a1, F29<F>& r0, F29<F>& r1) {
  F29<F> d0, d1;
#pragma unroll
  for (int i = 0; i < F::L; i++) {
    d0.v[i] = a0.v[i] << 1;
    d1.v[i] = a1.v[i] << 1;
  }
  const PLimbs<F> pl;
  MontChain<F> c0, c1;
  c0.acc = c1.acc = 0;
  static_for<0, 2 * F::L - 1>([&](auto kc) {
    constexpr int k = decltype(kc)::value;
#ifdef KZGX_MAD_PAIR
    mc_sqr2<F, k>(c0, a0, d0, c1, a1, d1);
    mc_reduce2<F, k>(c0, r0, c1, r1, pl.v);
#else
    mc_sqr<F, k>(c0, a0, d0);
    mc_sqr<F, k>(c1, a1, d1);
    mc_reduce<F, k>(c0, r0, pl.v);
    mc_reduce<F, k>(c1, r1, pl.v);
#endif
  });
}

// a b / R as f29_mul, each column one chain
template <class F>
KZGX_DEV F29<F> f29_mul_chain(const F29<F>& a, const F29<F>& b) {
  const PLimbs<F> pl;
  MontChain<F> h;
  h.acc = 0;
  F29<F> r;
  static_for<0, 2 * F::L - 1>([&](auto kc) {
    constexpr int k = decltype(kc)::value;
    mc_prod<F, k>(h, a, b);
    mc_reduce<F, k>(h, r, pl.v);
  });
  return r;
}

// a^2 / R as f29_sqr, each column one chain
template <class F>
KZGX_DEV F29<F> f29_sqr_chain(const F29<F>& a) {
  F29<F> dd;
#pragma unroll
  for (int i = 0; i < F::L; i++) dd.v[i] = a.v[i] << 1;
  const PLimbs<F> pl;
  MontChain<F> h;
  h.acc = 0;
  F29<F> r;
  static_for<0, 2 * F::L - 1>([&](auto kc) {
    constexpr int k = decltype(kc)::value;
    mc_sqr<F, k>(h, a, dd);
    mc_reduce<F, k>(h, r, pl.v);
  });
  return r;
}

// (a b + c d) / R as f29_mul2, each column one chain
template <class F>
KZGX_DEV F29<F> f29_mul2_chain(const F29<F>& a, const F29<F>& b, const F29<F>& c, const F29<F>& d) {
  const PLimbs<F> pl;
  MontChain<F> h;
  h.acc = 0;
  F29<F> r;
  static_for<0, 2 * F::L - 1>([&](auto kc) {
    constexpr int k = decltype(kc)::value;
    mc_prod<F, k>(h, a, b);
    mc_prod<F, k>(h, c, d);
    mc_reduce<F, k>(h, r, pl.v);
  });
  return r;
}

// r0 = (a0 b0 + c0 d0) / R (one reduction), r1 = a1 b1 / R, r2 = a2 b2 / R
template <class F>
KZGX_DEV void f29_mul2_x3(const F29<F>& a0, const F29<F>& b0, const F29<F>& c0, const F29<F>& d0, const F29<F>& a1,
                          const F29<F>& b1, const F29<F>& a2, const F29<F>& b2, F29<F>& r0, F29<F>& r1, F29<F>& r2) {
  const PLimbs<F> pl;
  MontChain<F> h0, h1, h2;
  h0.acc = h1.acc = h2.acc = 0;
  static_for<0, 2 * F::L - 1>([&](auto kc) {
    constexpr int k = decltype(kc)::value;
    mc_prod<F, k>(h0, a0, b0);
    mc_prod<F, k>(h0, c0, d0);
    mc_prod<F, k>(h1, a1, b1);
    mc_prod<F, k>(h2, a2, b2);
    mc_reduce<F, k>(h0, r0, pl.v);
    mc_reduce<F, k>(h1, r1, pl.v);
    mc_reduce<F, k>(h2, r2, pl.v);
  });
}

// Montgomery square: cross products once, against a doubled operand
template <class F>
KZGX_DEV F29<F> f29_sqr(const F29<F>& a) {
#ifdef KZGX_FIELD_LATENCY
  return f29_mul_lat<F>(a, a);
#endif
  constexpr int L = F::L;
  uint32_t q[L], d[L];
#pragma unroll
  for (int i = 0; i < L; i++) d[i] = a.v[i] << 1;
  F29<F> t;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 2 * L - 1; k++) {
#pragma unroll
    for (int i = 0; i < L; i++) {
      const int j = k - i;
      if (j > i && j < L) mad_vv(acc, a.v[i], d[j]);
    }
    if ((k & 1) == 0 && (k >> 1) < L) mad_vv(acc, a.v[k >> 1], a.v[k >> 1]);
#pragma unroll
    for (int i = 0; i < L; i++) {
      const int j = k - i;
      if (i < k && j >= 1 && j < L) mad_vs(acc, q[i], f29_pl<F>(j));
    }
    if (k < L) {
      q[k] = ((uint32_t)acc * F::INV) & M29;
      mad_vs(acc, q[k], f29_pl<F>(0));
    } else {
      t.v[k - L] = (uint32_t)acc & M29;
    }
    acc >>= 29;
  }
  t.v[L - 1] = (uint32_t)acc;
  return t;
}

// 2m - a for a < m with normalized limbs, no carry chain: one v_sub per
// limb.  The result (< 2m) has limbs in [0, 2^30), NOT normalized; it may
// only feed f29_mul / f29_mul2 as one operand (column sums: L 2^59 products
// + the reduction terms stay < 2^64 for both curves), f29_add / f29_sub
// (int32 carries absorb limbs < 2^30) or a reduction.
template <class F>
KZGX_DEV F29<F> f29_neg_lazy(const F29<F>& a) {
  F29<F> r;
#pragma unroll
  for (int i = 0; i < F::L; i++) r.v[i] = F::P2B[i] - a.v[i];
  return r;
}

// a + 2 b limb-wise, no carry: for normalized a, b the limbs are < 3 2^29.
// Only for a f29_sub subtrahend (its int32 carries absorb limbs < 2^31).
template <class F>
KZGX_DEV F29<F> f29_add_2x_lazy(const F29<F>& a, const F29<F>& b) {
  F29<F> r;
#pragma unroll
  for (int i = 0; i < F::L; i++) r.v[i] = a.v[i] + 2u * b.v[i];
  return r;
}

// 8m - a for normalized a < 4m, no carry chain: one v_sub per limb (P8B's
// limbs dominate a's limb-wise, see gen_consts.py), result < 8m with limbs
// in [0, 2^30).  For a product operand whose partner has normalized limbs
// (f29_mul2's column bound holds with one such operand).
template <class F>
KZGX_DEV F29<F> f29_neg8_lazy(const F29<F>& a) {
  F29<F> r;
#pragma unroll
  for (int i = 0; i < F::L; i++) r.v[i] = F::P8B[i] - a.v[i];
  return r;
}

// carry-normalize limbs (< 2^31 each) without changing the value
template <class F>
KZGX_DEV F29<F> f29_normalize(const F29<F>& a) {
  F29<F> r;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < F::L; i++) {
    const uint32_t s = a.v[i] + c;
    r.v[i] = i + 1 < F::L ? (s & M29) : s;
    c = s >> 29;
  }
  return r;
}

// a - K if a >= K (K a multiple of m)
template <class F>
KZGX_DEV F29<F> f29_csub(const F29<F>& a, const uint32_t (&K)[F::L]) {
  F29<F> r;
  int32_t c = 0;
#pragma unroll
  for (int i = 0; i < F::L; i++) {
    int32_t s = (int32_t)a.v[i] - (int32_t)K[i] + c;
    r.v[i] = (uint32_t)s & M29;
    c = s >> 29;
  }
  const bool keep = c < 0;  // borrow out: a < K
#pragma unroll
  for (int i = 0; i < F::L; i++) r.v[i] = keep ? a.v[i] : r.v[i];
  return r;
}

// full reduction of a < 16 m to [0, m)
template <class F>
KZGX_DEV F29<F> f29_reduce(const F29<F>& a) {
  F29<F> r = f29_csub<F>(a, F::P8);
  r = f29_csub<F>(r, F::P4);
  r = f29_csub<F>(r, F::P2);
  return f29_csub<F>(r, F::P);
}

// a == 0 mod m for a < 2m, with a one-limb filter in front of the full test
template <class F>
KZGX_DEV bool f29_is_zero_lt2m(const F29<F>& a) {
  const uint32_t v0 = a.v[0];
  if (v0 != 0u && v0 != F::LOW[1]) return false;
  return f29_is_zero_exact<F>(f29_csub<F>(a, F::P));
}

template <class F>
KZGX_DEV bool f29_is_zero(const F29<F>& a) {
  return f29_is_zero_exact<F>(f29_reduce<F>(a));
}

template <class F>
KZGX_DEV F29<F> f29_to_mont(const F29<F>& a) {
  return f29_mul<F>(a, f29_const<F>(F::R2));
}

template <class F>
KZGX_DEV F29<F> f29_from_mont(const F29<F>& a) {
  F29<F> one = f29_zero<F>();
  one.v[0] = 1;
  return f29_reduce<F>(f29_mul<F>(a, one));
}

// canonical little-endian 32-bit words (NW of them) <-> radix-2^29 limbs
template <class F, int NW>
KZGX_DEV F29<F> f29_from_words(const uint32_t (&w)[NW]) {
  F29<F> r;
#pragma unroll
  for (int i = 0; i < F::L; i++) {
    const int bit = 29 * i, wd = bit >> 5, sh = bit & 31;
    uint32_t lo = wd < NW ? w[wd] : 0u;
    uint32_t hi = wd + 1 < NW ? w[wd + 1] : 0u;
    r.v[i] = (sh == 0 ? lo : __builtin_amdgcn_alignbit(hi, lo, sh)) & M29;
  }
  return r;
}

template <class F, int NW>
KZGX_DEV void f29_to_words(const F29<F>& a, uint32_t (&w)[NW]) {
#pragma unroll
  for (int j = 0; j < NW; j++) {
    const int bit = 32 * j, li = bit / 29, sh = bit % 29;
    uint64_t v = li < F::L ? (uint64_t)(a.v[li] >> sh) : 0u;
    int have = 29 - sh;
    if (li + 1 < F::L) v |= (uint64_t)a.v[li + 1] << have;
    if (li + 2 < F::L && have + 29 < 32) v |= (uint64_t)a.v[li + 2] << (have + 29);
    w[j] = (uint32_t)v;
  }
}

// a^(m-2), left-to-right sliding window of width 3 over the exponent words
// PM2 (NW 32-bit words): 4 odd powers a, a^3, a^5, a^7 (36 VGPRs on BN254;
// a 16-entry fixed window spilled to scratch on the latency-bound paths that
// use this, k_*_finish and k_xyzz_sum), ~254 squarings + ~64 products.
template <class F, int NW>
__device__ __noinline__ F29<F> f29_inv(const F29<F>& a, const uint32_t (&pm2)[NW]) {
  F29<F> odd[4];
  odd[0] = a;
  const F29<F> a2 = f29_sqr<F>(a);
  odd[1] = f29_mul<F>(odd[0], a2);
  odd[2] = f29_mul<F>(odd[1], a2);
  odd[3] = f29_mul<F>(odd[2], a2);
  auto bit = [&](int i) -> uint32_t { return (pm2[i >> 5] >> (i & 31)) & 1u; };
  // the window [i .. j] (j >= i - 2, ending in a set bit) as an odd value < 8
  auto window = [&](int i, int& j) -> F29<F> {
    j = i - 2 < 0 ? 0 : i - 2;
    while (!bit(j)) j++;
    uint32_t w = 0;
    for (int k = i; k >= j; k--) w = (w << 1) | bit(k);
    const int idx = (int)(w >> 1);
    F29<F> m = odd[0];
#pragma unroll
    for (int k = 1; k < 4; k++)
      if (k == idx) m = odd[k];
    return m;
  };
  int i = 32 * NW - 1;
  while (i >= 0 && !bit(i)) i--;
  int j = 0;
  F29<F> acc = window(i, j);  // m - 2 > 0: the top window exists
  i = j - 1;
  while (i >= 0) {
    if (!bit(i)) {
      acc = f29_sqr<F>(acc);
      i--;
      continue;
    }
    const F29<F> m = window(i, j);
    for (int k = i; k >= j; k--) acc = f29_sqr<F>(acc);
    acc = f29_mul<F>(acc, m);
    i = j - 1;
  }
  return acc;
}

// a^-1 for a Montgomery-form a < 16 m (0 -> 0): binary GCD with 60-bit
// approximations (Pornin, "Optimized Binary GCD for Modular Inversion",
// 2020, algorithm 2, k = 30).  Variable time: every value these paths invert
// (commitment / proof coordinates, pairing values) is public.
//
// Why: on the single-MSM tails this runs in ONE lane, where every dependent
// VALU instruction costs ~8 core clocks (scripts/lat_micro.py: a BN254
// Montgomery product is ~2000 clocks, the Fermat chain ~417 000).  Here the
// bit-serial work runs on two 60-bit words (the low 29 and the top 31 bits of
// the operands) and the full-width limbs are touched once per 29 steps.
//
// State, in radix-2^29 limbs: y = the canonical Montgomery representative,
// a = y, b = m, u = 1, v = 0, keeping a = u y and b = v y (mod m).  Each pass
// runs 29 binary-GCD steps on the approximations, collecting the signed
// matrix (f0 g0; f1 g1) (|f| + |g| <= 2^29), then
//   a <- |a f0 + b g0| / 2^29, b <- |a f1 + b g1| / 2^29 (exact divisions),
//   u <- (u f0 + v g0) / 2^29 mod m, v <- (u f1 + v g1) / 2^29 mod m
// (signs folded into f, g; the mod-m halvings are Montgomery steps with
// INV = -m^-1 mod 2^29), until a = 0; then b = 1 and v = y^-1.  BN254:
// 13 passes on average (16 at most over 3000 random inputs), BLS12-381 19
// (21).  The Montgomery form of the result, (y / R)^-1 R = v R^2, is two
// products by R^2 mod m.
//
// U (wave-uniform): the caller guarantees the first active lane holds the
// value every lane needs -- a single lane's tail (lane 0 of the latency
// path's fold) -- and the input is read from that lane, so the whole GCD
// state is uniform: the bit-serial inner loop runs on the scalar ALU, and
// with lanes 0-3 active the four linear combinations of a pass run one per
// lane (combine4).  Never with a different value per lane (the batched
// finish kernels).
template <class F, int NW, bool U = false, bool RAW = false>
__device__ __noinline__ F29<F> f29_inv_vt(const F29<F>& in_, const uint32_t (&)[NW]) {
  constexpr int L = F::L;
  constexpr int K = 29;
  F29<F> in = in_;
  if constexpr (U) {
#pragma unroll
    for (int j = 0; j < L; j++) in.v[j] = __builtin_amdgcn_readfirstlane(in.v[j]);
  }
  F29<F> a = f29_reduce<F>(in), b = f29_const<F>(F::P), u = f29_zero<F>(), v = f29_zero<F>();
  if (f29_is_zero_exact<F>(a)) return a;
  u.v[0] = 1;
  auto approx = [](const F29<F>& x, int i, int o) -> uint64_t {
    // bits [29 i + o, 29 i + o + 31) of x, over limbs i, i + 1, i + 2
    uint32_t w0 = 0, w1 = 0, w2 = 0;
#pragma unroll
    for (int j = 0; j < L; j++) {
      w0 = j == i ? x.v[j] : w0;
      w1 = j == i + 1 ? x.v[j] : w1;
      w2 = j == i + 2 ? x.v[j] : w2;
    }
    const uint64_t w = (uint64_t)w0 | ((uint64_t)w1 << 29) | ((uint64_t)w2 << 58);
    return (((w >> o) & 0x7fffffffull) << K) | x.v[0];
  };
  // (x f + y g) / 2^29 as signed limbs (the low 29 bits of the sum are zero);
  // returns the sign and leaves |.| in r
  auto combine = [](const F29<F>& x, const F29<F>& y, int32_t f, int32_t g, F29<F>& r) -> bool {
    int64_t c = (int64_t)(int32_t)x.v[0] * f + (int64_t)(int32_t)y.v[0] * g;
    c >>= K;
#pragma unroll
    for (int j = 1; j < L; j++) {
      c += (int64_t)(int32_t)x.v[j] * f + (int64_t)(int32_t)y.v[j] * g;
      r.v[j - 1] = (uint32_t)c & M29;
      c >>= K;
    }
    r.v[L - 1] = (uint32_t)c;
    const bool neg = c < 0;
    if (neg) {  // r <- -r
      int64_t d = 0;
#pragma unroll
      for (int j = 0; j < L; j++) {
        d -= (int64_t)(int32_t)r.v[j];
        r.v[j] = j + 1 < L ? (uint32_t)d & M29 : (uint32_t)d;
        d >>= K;
      }
    }
    return neg;
  };
  // (x f + y g) / 2^29 mod m, x, y in [0, m): Montgomery halving, result in
  // (-m, 2m), then brought to [0, m)
  auto combine_mod = [](const F29<F>& x, const F29<F>& y, int32_t f, int32_t g) -> F29<F> {
    F29<F> r;
    int64_t c = (int64_t)(int32_t)x.v[0] * f + (int64_t)(int32_t)y.v[0] * g;
    const uint32_t q = ((uint32_t)c * F::INV) & M29;
    c += (int64_t)q * F::P[0];
    c >>= K;
#pragma unroll
    for (int j = 1; j < L; j++) {
      c += (int64_t)(int32_t)x.v[j] * f + (int64_t)(int32_t)y.v[j] * g + (int64_t)q * F::P[j];
      r.v[j - 1] = (uint32_t)c & M29;
      c >>= K;
    }
    r.v[L - 1] = (uint32_t)c;
    const uint32_t mask = c < 0 ? M29 : 0u;  // negative: + m
    int64_t d = 0;
#pragma unroll
    for (int j = 0; j < L; j++) {
      d += (int64_t)(int32_t)r.v[j] + (F::P[j] & mask);
      r.v[j] = j + 1 < L ? (uint32_t)d & M29 : (uint32_t)d;
      d >>= K;
    }
    return f29_csub<F>(r, F::P);
  };
  // U: lane k < 4 computes one of a' = |a f0 + b g0| / 2^29 (k = 0),
  // b' = |a f1 + b g1| / 2^29 (1), u' = (u f0 + v g0) / 2^29 mod m (2),
  // v' = (u f1 + v g1) / 2^29 mod m (3) -- the exact division and the
  // Montgomery halving as one routine (q = 0 on lanes 0 and 1) -- then lanes
  // 2 and 3 take the sign of lanes 0 and 1 (x -> m - x), and the four
  // results return to uniform registers (readlane)
  auto combine4 = [](F29<F>& a, F29<F>& b, F29<F>& u, F29<F>& v, int32_t f0, int32_t g0, int32_t f1, int32_t g1) {
    const uint32_t lane = __lane_id();
    const bool hi = (lane & 1) != 0, md = (lane & 2) != 0;
    const int32_t f = hi ? f1 : f0, g = hi ? g1 : g0;
    F29<F> r;
    int64_t c = (int64_t)(int32_t)(md ? u.v[0] : a.v[0]) * f + (int64_t)(int32_t)(md ? v.v[0] : b.v[0]) * g;
    const uint32_t q = md ? ((uint32_t)c * F::INV) & M29 : 0u;
    c += (int64_t)q * F::P[0];
    c >>= K;
#pragma unroll
    for (int j = 1; j < L; j++) {
      c += (int64_t)(int32_t)(md ? u.v[j] : a.v[j]) * f + (int64_t)(int32_t)(md ? v.v[j] : b.v[j]) * g +
           (int64_t)q * F::P[j];
      r.v[j - 1] = (uint32_t)c & M29;
      c >>= K;
    }
    r.v[L - 1] = (uint32_t)c;
    const bool neg = c < 0;
    // negative: lanes 0, 1 take |r| = -r, lanes 2, 3 add m (r in (-m, 2m))
    int64_t d = 0;
#pragma unroll
    for (int j = 0; j < L; j++) {
      const int64_t rj = (int64_t)(int32_t)r.v[j];
      d += neg ? (md ? rj + (int64_t)F::P[j] : -rj) : rj;
      r.v[j] = j + 1 < L ? (uint32_t)d & M29 : (uint32_t)d;
      d >>= K;
    }
    if (md) r = f29_csub<F>(r, F::P);  // [0, m)
    // lanes 2, 3: the sign lanes 0, 1 folded into f, g in the per-lane form
    const int sgn = __shfl((int)neg, (int)(lane & 1), 64);
    if (md && sgn && !f29_is_zero_exact<F>(r)) r = f29_sub<F>(f29_zero<F>(), r, F::P);  // m - r
#pragma unroll
    for (int j = 0; j < L; j++) {
      a.v[j] = __builtin_amdgcn_readlane(r.v[j], 0);
      b.v[j] = __builtin_amdgcn_readlane(r.v[j], 1);
      u.v[j] = __builtin_amdgcn_readlane(r.v[j], 2);
      v.v[j] = __builtin_amdgcn_readlane(r.v[j], 3);
    }
  };
  // 3x the most passes seen: a bound every lane reaches even on a bad input
  for (int pass = 0; pass < 3 * (2 * 29 * L / K + 2) && !f29_is_zero_exact<F>(a); pass++) {
    // n = max(len(a), len(b), 60); the approximations keep bits [0, 29) and
    // [n - 31, n)
    uint32_t top = 0;
    int h = 0;
#pragma unroll
    for (int j = 0; j < L; j++) {
      const uint32_t o = a.v[j] | b.v[j];
      h = o ? j : h;
      top = o ? o : top;
    }
    int n = 29 * h + 32 - __clz(top);
    n = n < 60 ? 60 : n;
    const int p = n - 31, i = p / 29, o = p - 29 * i;
    uint64_t ab = approx(a, i, o), bb = approx(b, i, o);
    int32_t f0 = 1, g0 = 0, f1 = 0, g1 = 1;
    int rem = K;
    while (rem > 0) {
      if (ab & 1) {
        if (ab < bb) {
          const uint64_t t = ab;
          ab = bb;
          bb = t;
          int32_t s = f0;
          f0 = f1;
          f1 = s;
          s = g0;
          g0 = g1;
          g1 = s;
        }
        ab -= bb;
        f0 -= f1;
        g0 -= g1;
      }
      int z = ab ? __builtin_ctzll(ab) : rem;
      z = z < rem ? z : rem;
      ab >>= z;
      f1 = (int32_t)((uint32_t)f1 << z);
      g1 = (int32_t)((uint32_t)g1 << z);
      rem -= z;
    }
    if constexpr (U) {
      // the four combinations side by side, one per lane (lanes 0-3), in one
      // instruction stream -- a lone wave pays per instruction, not per lane
      // -- when lanes 0-3 are active (callers from a one-thread region fall
      // through to the sequential form)
      if ((__builtin_amdgcn_read_exec() & 0xFull) == 0xFull) {
        combine4(a, b, u, v, f0, g0, f1, g1);
        continue;
      }
    }
    F29<F> a2, b2;
    if (combine(a, b, f0, g0, a2)) {
      f0 = -f0;
      g0 = -g0;
    }
    if (combine(a, b, f1, g1, b2)) {
      f1 = -f1;
      g1 = -g1;
    }
    const F29<F> u2 = combine_mod(u, v, f0, g0);
    v = combine_mod(u, v, f1, g1);
    u = u2;
    a = a2;
    b = b2;
  }
  // RAW: (y / R)^-1 as a plain residue, v R = one product by R^2; else its
  // Montgomery form v R^2 = one product by R^3 (was two by R^2)
  if constexpr (RAW) return f29_mul<F>(v, f29_const<F>(F::R2));
  return f29_mul<F>(v, f29_const<F>(F::R3));
}

// a^-1 of the first active lane's a (see U above)
template <class F, int NW>
KZGX_DEV F29<F> f29_inv_uniform(const F29<F>& a, const uint32_t (&m)[NW]) {
  return f29_inv_vt<F, NW, true>(a, m);
}
// the same inverse of the Montgomery value a (= A R) as the plain residue
// A^-1 (not its Montgomery form A^-1 R): one product fewer
template <class F, int NW>
KZGX_DEV F29<F> f29_inv_uniform_raw(const F29<F>& a, const uint32_t (&m)[NW]) {
  return f29_inv_vt<F, NW, true, true>(a, m);
}

// the inversion the finish / pairing paths use (KZGX_INV_FERMAT: the
// constant-time exponentiation, for A/B runs)
template <class F, int NW>
KZGX_DEV F29<F> f29_inv_fast(const F29<F>& a, const uint32_t (&m)[NW], const uint32_t (&pm2)[NW]) {
#ifdef KZGX_INV_FERMAT
  (void)m;
  return f29_inv<F, NW>(a, pm2);
#else
  (void)pm2;
  return f29_inv_vt<F, NW>(a, m);
#endif
}

template <class F>
KZGX_DEV F29<F> f29_load(const uint32_t* p) {
  F29<F> r;
#pragma unroll
  for (int i = 0; i < F::L; i++) r.v[i] = p[i];
  return r;
}

template <class F>
KZGX_DEV void f29_store(uint32_t* p, const F29<F>& a) {
#pragma unroll
  for (int i = 0; i < F::L; i++) p[i] = a.v[i];
}

}  // namespace kzgx
