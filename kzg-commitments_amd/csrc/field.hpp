// Device-side multi-precision Montgomery arithmetic for gfx950.
//
// Limbs are 32-bit (the VALU word).  Products use v_mad_u64_u32 through the
// (uint64_t)a * b + c idiom; carry chains use __builtin_addc / __builtin_subc
// (v_add_co_u32 / v_addc_co_u32).  Everything is fully unrolled so a field
// element lives in N VGPRs.  Values are kept fully reduced in [0, m).
//
// Replaces the role of miracl-core's FP (un-vendored) on the
// commit/prove hot path (src/trusted_setup.cpp:149-174).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "curve_consts.h"

#define KZGX_DEV __device__ __forceinline__

namespace kzgx {

template <class FP>
struct Fe {
  uint32_t v[FP::N];
};

template <class FP>
KZGX_DEV Fe<FP> fe_const(const uint32_t (&c)[FP::N]) {
  Fe<FP> r;
#pragma unroll
  for (int i = 0; i < FP::N; i++) r.v[i] = c[i];
  return r;
}

template <class FP>
KZGX_DEV Fe<FP> fe_zero() {
  Fe<FP> r;
#pragma unroll
  for (int i = 0; i < FP::N; i++) r.v[i] = 0;
  return r;
}

template <class FP>
KZGX_DEV Fe<FP> fe_one() {
  return fe_const<FP>(FP::ONE);
}

template <class FP>
KZGX_DEV bool fe_is_zero(const Fe<FP>& a) {
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < FP::N; i++) o |= a.v[i];
  return o == 0;
}

template <class FP>
KZGX_DEV bool fe_eq(const Fe<FP>& a, const Fe<FP>& b) {
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < FP::N; i++) o |= a.v[i] ^ b.v[i];
  return o == 0;
}

// r = a + b mod m
template <class FP>
KZGX_DEV Fe<FP> fe_add(const Fe<FP>& a, const Fe<FP>& b) {
  constexpr int N = FP::N;
  Fe<FP> s, t;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < N; i++) s.v[i] = __builtin_addc(a.v[i], b.v[i], c, &c);
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < N; i++) t.v[i] = __builtin_subc(s.v[i], FP::P[i], br, &br);
  // keep s if (no carry out and borrow) i.e. s < m
  const bool keep = (c == 0) && (br != 0);
#pragma unroll
  for (int i = 0; i < N; i++) s.v[i] = keep ? s.v[i] : t.v[i];
  return s;
}

// r = a - b mod m
template <class FP>
KZGX_DEV Fe<FP> fe_sub(const Fe<FP>& a, const Fe<FP>& b) {
  constexpr int N = FP::N;
  Fe<FP> s, t;
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < N; i++) s.v[i] = __builtin_subc(a.v[i], b.v[i], br, &br);
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < N; i++) t.v[i] = __builtin_addc(s.v[i], FP::P[i], c, &c);
#pragma unroll
  for (int i = 0; i < N; i++) s.v[i] = br ? t.v[i] : s.v[i];
  return s;
}

template <class FP>
KZGX_DEV Fe<FP> fe_neg(const Fe<FP>& a) {
  return fe_sub<FP>(fe_zero<FP>(), a);
}

template <class FP>
KZGX_DEV Fe<FP> fe_dbl(const Fe<FP>& a) {
  return fe_add<FP>(a, a);
}

// Montgomery product a b R^-1 mod m, CIOS (coarsely integrated operand scanning).
template <class FP>
KZGX_DEV Fe<FP> fe_mul(const Fe<FP>& a, const Fe<FP>& b) {
  constexpr int N = FP::N;
  uint32_t t[N + 2];
#pragma unroll
  for (int i = 0; i < N + 2; i++) t[i] = 0;
#pragma unroll
  for (int i = 0; i < N; i++) {
    uint32_t carry = 0;
    const uint32_t bi = b.v[i];
#pragma unroll
    for (int j = 0; j < N; j++) {
      uint64_t v = (uint64_t)a.v[j] * bi + (uint64_t)t[j] + carry;
      t[j] = (uint32_t)v;
      carry = (uint32_t)(v >> 32);
    }
    uint64_t v = (uint64_t)t[N] + carry;
    t[N] = (uint32_t)v;
    t[N + 1] = (uint32_t)(v >> 32);
    const uint32_t mq = t[0] * FP::INV;
    v = (uint64_t)mq * FP::P[0] + t[0];
    carry = (uint32_t)(v >> 32);
#pragma unroll
    for (int j = 1; j < N; j++) {
      v = (uint64_t)mq * FP::P[j] + (uint64_t)t[j] + carry;
      t[j - 1] = (uint32_t)v;
      carry = (uint32_t)(v >> 32);
    }
    v = (uint64_t)t[N] + carry;
    t[N - 1] = (uint32_t)v;
    t[N] = t[N + 1] + (uint32_t)(v >> 32);
  }
  Fe<FP> r, s;
#pragma unroll
  for (int i = 0; i < N; i++) r.v[i] = t[i];
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < N; i++) s.v[i] = __builtin_subc(r.v[i], FP::P[i], br, &br);
  const bool keep = (t[N] == 0) && (br != 0);
#pragma unroll
  for (int i = 0; i < N; i++) r.v[i] = keep ? r.v[i] : s.v[i];
  return r;
}

template <class FP>
KZGX_DEV Fe<FP> fe_sqr(const Fe<FP>& a) {
  return fe_mul<FP>(a, a);
}

// canonical -> Montgomery
template <class FP>
KZGX_DEV Fe<FP> fe_to_mont(const Fe<FP>& a) {
  return fe_mul<FP>(a, fe_const<FP>(FP::R2));
}

// Montgomery -> canonical
template <class FP>
KZGX_DEV Fe<FP> fe_from_mont(const Fe<FP>& a) {
  Fe<FP> one = fe_zero<FP>();
  one.v[0] = 1;
  return fe_mul<FP>(a, one);
}

// a^(m-2) (Fermat inverse), fixed 4-bit window over the constant exponent.
// inv(0) = 0.
template <class FP>
__device__ __noinline__ Fe<FP> fe_inv(const Fe<FP>& a) {
  constexpr int N = FP::N;
  Fe<FP> tbl[16];
  tbl[0] = fe_one<FP>();
  tbl[1] = a;
#pragma unroll
  for (int i = 2; i < 16; i++) tbl[i] = fe_mul<FP>(tbl[i - 1], a);
  Fe<FP> acc = fe_one<FP>();
  for (int nib = 8 * N - 1; nib >= 0; nib--) {
#pragma unroll
    for (int s = 0; s < 4; s++) acc = fe_sqr<FP>(acc);
    const uint32_t d = (FP::PM2[nib >> 3] >> (4 * (nib & 7))) & 15u;
    // table index is wave-uniform (constant exponent) -> no divergence
    Fe<FP> m;
#pragma unroll
    for (int k = 0; k < 16; k++)
      if (k == (int)d) m = tbl[k];
    acc = fe_mul<FP>(acc, m);
  }
  return acc;
}

// loads / stores of N-limb elements from 32-bit arrays
template <class FP>
KZGX_DEV Fe<FP> fe_load(const uint32_t* p) {
  Fe<FP> r;
  if constexpr (FP::N % 4 == 0) {
#pragma unroll
    for (int i = 0; i < FP::N / 4; i++) {
      uint4 q = reinterpret_cast<const uint4*>(p)[i];
      r.v[4 * i] = q.x;
      r.v[4 * i + 1] = q.y;
      r.v[4 * i + 2] = q.z;
      r.v[4 * i + 3] = q.w;
    }
  } else {
#pragma unroll
    for (int i = 0; i < FP::N; i++) r.v[i] = p[i];
  }
  return r;
}

template <class FP>
KZGX_DEV void fe_store(uint32_t* p, const Fe<FP>& a) {
  if constexpr (FP::N % 4 == 0) {
#pragma unroll
    for (int i = 0; i < FP::N / 4; i++)
      reinterpret_cast<uint4*>(p)[i] = make_uint4(a.v[4 * i], a.v[4 * i + 1], a.v[4 * i + 2], a.v[4 * i + 3]);
  } else {
#pragma unroll
    for (int i = 0; i < FP::N; i++) p[i] = a.v[i];
  }
}

}  // namespace kzgx
