// Wave-per-opening verify on gfx950: the two-pairing product check of
// verify_proof (reference src/trusted_setup.cpp:230-254) with every Fp12
// product spread over a 64-lane wave, the G2 line tables it consumes, and
// the wave-parallel G2 chain for a variable second argument.  Split from
// pairing.hip to keep each translation unit's compile time bounded.
#include <hip/hip_runtime.h>

// every Fp product in this translation unit (wave ops, tower, curve) takes
// the latency-first form (field29.hpp f29_mul_lat): these kernels run as one
// wave per pairing, where a product's dependency chain is the cost
// (KZGX_VW_CHAIN: the chained form, A/B)
#ifndef KZGX_VW_CHAIN
#define KZGX_FIELD_LATENCY
#endif
#include "coop.hpp"
#include "pairing_common.hpp"
#include "kzgx_setup.hpp"

namespace kzgx {

// ---- wave-parallel single verify (latency path) ----------------------------------
// One 64-lane wave per opening instead of one lane: the same product of two
// Miller loops and one final exponentiation as k_verify_single, with every
// Fp12 product spread over the wave.  Fp12 is kept in the w basis
// (a = sum_k a_k w^k, a_k in Fp2, w^6 = xi; tower c_h.c_j is w^(2j+h)) in
// LDS: a dense product is 36 Fp2 products, one per lane, then 12 lanes fold
// the columns; a line product is 18 Fp2 products and 3-term folds.
// Both G2 arguments are fixed by the setup (G2[0], G2[1] = [tau]G2), so
// their line coefficients are precomputed once (k_vlines) and only scaled
// by the G1 argument's coordinates per opening; the G1 argument -D is used
// in XYZZ form (the line is multiplied by the Fp factor ZZ ZZZ, which the
// final exponentiation removes).  [y]G comes from a table of
// d 2^(8w) G (k_vtab: 32 windows x 255 digits) summed by a 5-level tree;
// [z]pi is double-and-add over z's bit length (z is a point index in the
// reference's use, trusted_setup.cpp:230-254).
#ifdef KZGX_VW_TIMING
#define VW_STAMP(i) \
  if (threadIdx.x == 0) vw_ts[i] = wall_clock64()
__device__ uint64_t vw_ts[16];
#else
#define VW_STAMP(i)
#endif

template <class C>
struct VWave {
  using P = typename PairOf<C>::T;
  static constexpr int L = C::Fp29::L;
  static constexpr int E2 = 2 * L;    // words per Fp2
  static constexpr int E12 = 12 * L;  // words per Fp12 (6 Fp2)
  static constexpr int LW = 3 * E2;   // words per line (w0, w1, w3 coefficients)
  static constexpr int adds_below_top() {
    int n = 0;
    for (int i = 0; i < P::LOOP_BITS - 1; i++) n += (int)((P::LOOP[i >> 6] >> (i & 63)) & 1ull);
    return n;
  }
  static constexpr int NL = (P::LOOP_BITS - 1) + adds_below_top() + (P::D_TWIST ? 2 : 0);
  static constexpr int TAB = 32 * 255;  // [y]G table entries
  static constexpr int AW = affine_words<C>();
  // positions of the w0, w1, w3 coefficients in the w basis
  static constexpr int POS0 = P::D_TWIST ? 0 : 3, POS1 = P::D_TWIST ? 1 : 2, POS3 = P::D_TWIST ? 3 : 0;
  static constexpr int NSLOT = 15;  // 0..8: the final exponentiation's program, 9..14: the second wave's
  // LDS carve (words)
  static constexpr int O_LINES = 0;                        // [2][NL][LW] scaled lines
  static constexpr int O_SLOT = O_LINES + 2 * NL * LW;     // [NSLOT][E12]
  // product parts at a 16-byte stride PL >= L, so a part is written and
  // read back with 128-bit LDS accesses (the folds read 7-18 parts per lane)
  static constexpr int PL = (L + 3) & ~3;
  static constexpr int O_PROD = O_SLOT + NSLOT * E12;      // [108][PL] product parts; G1 phase: [32][4L] XYZZ tree
  static constexpr int PROD_W = (108 * PL > 32 * 4 * L) ? 108 * PL : 32 * 4 * L;
  static constexpr int O_SCALE = O_PROD + PROD_W;          // [2][3][L] scale factors
  static constexpr int O_FLAG = O_SCALE + 6 * L;           // [16]
  // the second wave's product parts during the two-wave Miller loop
  static constexpr int O_PROD2 = (O_FLAG + 16 + 3) & ~3;   // [108][PL]
  // one opening's inputs, copied in at the kernel's start (the host entry
  // point passes them in mapped pinned memory: one PCIe round trip, not one
  // per access): commit (2N) | proof (2N) | z (8) | y (8) | commit_inf | proof_inf
  static constexpr int NW = C::Fp::N;
  static constexpr int I_C = 0, I_P = 2 * NW, I_Z = 4 * NW, I_Y = 4 * NW + 8, I_CINF = 4 * NW + 16, I_PINF = I_CINF + 1;
  static constexpr int O_IN = O_PROD2 + 108 * PL;
  static constexpr int WORDS = O_IN + I_PINF + 1;
};

// the wave kernel's LDS (dynamic; V::WORDS words), addressed by word offset
// so that the non-inlined helpers still issue LDS (ds_*) instructions
extern __shared__ __attribute__((aligned(16))) uint32_t vw_smem[];

template <class C>
KZGX_DEV F29<typename C::Fp29> vw_ld(const uint32_t* p) {
  F29<typename C::Fp29> r;
#pragma unroll
  for (int i = 0; i < C::Fp29::L; i++) r.v[i] = p[i];
  return r;
}
template <class C>
KZGX_DEV void vw_st(uint32_t* p, const F29<typename C::Fp29>& a) {
#pragma unroll
  for (int i = 0; i < C::Fp29::L; i++) p[i] = a.v[i];
}
template <class C>
KZGX_DEV Fp2<C> vw_ld2(const uint32_t* p) {
  return Fp2<C>{vw_ld<C>(p), vw_ld<C>(p + C::Fp29::L)};
}
template <class C>
KZGX_DEV void vw_st2(uint32_t* p, const Fp2<C>& a) {
  vw_st<C>(p, a.a);
  vw_st<C>(p + C::Fp29::L, a.b);
}

// line coefficients of the Miller loop for a fixed Q, in consumption order:
// (w0c, w1c, w3c) with the line at P = w0c yP, w1c xP, w3c (line_dbl /
// line_add with the P factors left out)
template <class C>
KZGX_DEV void vl_dbl(G2J<C>& T, uint32_t* out) {
  constexpr int E2 = VWave<C>::E2;
  const Fp2<C> A = f2_sqr<C>(T.X);
  const Fp2<C> B = f2_sqr<C>(T.Y);
  const Fp2<C> E = f2_add<C>(f2_dbl<C>(A), A);
  const Fp2<C> ZZ = f2_sqr<C>(T.Z);
  const Fp2<C> Z3 = f2_dbl<C>(f2_mul<C>(T.Y, T.Z));
  vw_st2<C>(out, f2_mul<C>(Z3, ZZ));
  vw_st2<C>(out + E2, f2_neg<C>(f2_mul<C>(E, ZZ)));
  vw_st2<C>(out + 2 * E2, f2_sub<C>(f2_mul<C>(E, T.X), f2_dbl<C>(B)));
  T = g2_dbl<C>(T);
}
template <class C>
KZGX_DEV void vl_add(G2J<C>& T, const G2A<C>& q, uint32_t* out) {
  constexpr int E2 = VWave<C>::E2;
  const Fp2<C> Z1Z1 = f2_sqr<C>(T.Z);
  const Fp2<C> U2 = f2_mul<C>(q.x, Z1Z1);
  const Fp2<C> S2 = f2_mul<C>(q.y, f2_mul<C>(T.Z, Z1Z1));
  const Fp2<C> H = f2_sub<C>(U2, T.X);
  const Fp2<C> rr = f2_dbl<C>(f2_sub<C>(S2, T.Y));
  const Fp2<C> Z3 = f2_dbl<C>(f2_mul<C>(T.Z, H));
  vw_st2<C>(out, Z3);
  vw_st2<C>(out + E2, f2_neg<C>(rr));
  vw_st2<C>(out + 2 * E2, f2_sub<C>(f2_mul<C>(rr, q.x), f2_mul<C>(q.y, Z3)));
  T = g2_add_mixed<C>(T, q);
}

// lanes 0, 1: the line tables of Q0 = G2[0] and Q1 = G2[1]; qfin[q] = finite
template <class C>
__global__ __launch_bounds__(64) void k_vlines(const uint32_t* __restrict__ g2_01, uint32_t* __restrict__ lines,
                                               uint32_t* __restrict__ qfin) {
  using P = typename PairOf<C>::T;
  using V = VWave<C>;
  const int q = threadIdx.x;
  if (q >= 2) return;
  G2A<C> Q;
  const bool fin = g2_from_canon<C>(g2_01 + q * 4 * C::Fp::N, Q);
  qfin[q] = fin ? 1u : 0u;
  if (!fin) return;
  uint32_t* out = lines + (size_t)q * V::NL * V::LW;
  int s = 0;
  G2J<C> T = g2_from_affine<C>(Q);
  for (int i = P::LOOP_BITS - 2; i >= 0; i--) {
    vl_dbl<C>(T, out + (s++) * V::LW);
    if ((P::LOOP[i >> 6] >> (i & 63)) & 1ull) vl_add<C>(T, Q, out + (s++) * V::LW);
  }
  if (P::LOOP_NEG) T.Y = f2_neg<C>(T.Y);
  if (P::D_TWIST) {
    const G2A<C> q1 = twist_frob<C>(Q);
    G2A<C> q2 = twist_frob<C>(q1);
    q2.y = f2_neg<C>(q2.y);
    vl_add<C>(T, q1, out + (s++) * V::LW);
    vl_add<C>(T, q2, out + (s++) * V::LW);
  }
}

// entry (w, d - 1) = d 2^(8 w) G for d in 1..255 (affine Montgomery)
template <class C>
__global__ __launch_bounds__(64) void k_vtab(const uint32_t* __restrict__ g1_0, uint32_t* __restrict__ tab) {
  using V = VWave<C>;
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (uint32_t)V::TAB) return;
  const uint32_t w = t / 255, d = t % 255 + 1;
  Affine<C> g;
  (void)affine_from_canonical<C>(g1_0, g);
  uint32_t e[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  e[w >> 2] = d << (8 * (w & 3));
  Affine<C> a;
  if (!xyzz_to_affine<C>(g1_mul_words<C>(g, e), a)) a.x = a.y = f29_zero<typename C::Fp29>();
  affine_store<C>(tab + (size_t)t * V::AW, a);
}

// Lazy signed combination sum_j c_j p_j of values with limbs < 2^31 and
// small integer c_j: one signed 64-bit accumulator per limb (one
// v_mad_i64_i32 per limb and term), then lin_fin reduces the value v
// (|v| < 2^20 m) to [0, 2m) in one step: the quotient q = floor(v/m) is
// estimated in double precision from the top three limb sums, and v - q m is
// carry-normalized once.  The estimate's error (dropped limbs < 2^-20 m,
// rounding < 2^-40) is far below the 2^-12 bias, so q is floor(v/m) or one
// less: the result lies in (0, 2m).  This replaces a carry pass per sign, a
// subtraction and a chain of conditional subtractions (~240 dependent
// instructions on the lone wave) with ~40.
template <class F>
struct LinAcc {
  int64_t v[F::L];
};
constexpr double lin_pow29(int k) {
  double s = 1.0;
  for (int i = 0; i < k; i++) s *= 536870912.0;
  return s;
}
template <class F>
constexpr double lin_modulus() {
  double s = 0.0;
  for (int i = F::L - 1; i >= 0; i--) s = s * 536870912.0 + (double)F::P[i];
  return s;
}
template <class F>
struct LinInvM {  // 2^(29 l) / m for the top three limbs
  static constexpr double T0 = lin_pow29(F::L - 1) / lin_modulus<F>();
  static constexpr double T1 = lin_pow29(F::L - 2) / lin_modulus<F>();
  static constexpr double T2 = lin_pow29(F::L - 3) / lin_modulus<F>();
};
template <class F>
KZGX_DEV void lin_init(LinAcc<F>& a) {
#pragma unroll
  for (int l = 0; l < F::L; l++) a.v[l] = 0;
}
template <class F>
KZGX_DEV void lin_add(LinAcc<F>& a, const uint32_t* p, int c) {
#pragma unroll
  for (int l = 0; l < F::L; l++) a.v[l] += (int64_t)(int32_t)p[l] * (int64_t)c;
}
template <class F>
KZGX_DEV void lin_add(LinAcc<F>& a, const F29<F>& p, int c) {
  lin_add<F>(a, p.v, c);
}
template <class F>
KZGX_DEV F29<F> lin_fin(const LinAcc<F>& a) {
  constexpr int L = F::L;
  const double x = (double)a.v[L - 1] * LinInvM<F>::T0 + (double)a.v[L - 2] * LinInvM<F>::T1 +
                   (double)a.v[L - 3] * LinInvM<F>::T2;
  // |q| < 2^20: one v_mad_i64_i32 per limb, off the carry chain
  const int32_t q = (int32_t)__builtin_floor(x - 0x1p-12);
  F29<F> r;
  int64_t c = 0;
#pragma unroll
  for (int l = 0; l < L; l++) {
    const int64_t s = (a.v[l] - (int64_t)q * (int64_t)(int32_t)F::P[l]) + c;
    if (l + 1 < L) {
      r.v[l] = (uint32_t)s & M29;
      c = s >> 29;  // arithmetic
    } else {
      r.v[l] = (uint32_t)s;
    }
  }
  return r;
}

// The fold of an output split over two adjacent lanes (lane ^ 1): each
// accumulates its share of the terms, then a += the partner's accumulator by
// DPP (quad_perm [1, 0, 3, 2]: a VALU operand modifier, no LDS), so the
// lin_fin lane's dependent limb-sum chains are half as long.
KZGX_DEV uint32_t dpp_xor1(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);
}
template <class F>
KZGX_DEV void lin_pair_sum(LinAcc<F>& a) {
#pragma unroll
  for (int l = 0; l < F::L; l++) {
    const uint64_t u = (uint64_t)a.v[l];
    const uint64_t o = ((uint64_t)dpp_xor1((uint32_t)(u >> 32)) << 32) | dpp_xor1((uint32_t)u);
    a.v[l] += (int64_t)o;
  }
}

// Karatsuba parts of an Fp2 product x y: 0 = xa ya, 1 = xb yb,
// 2 = (xa + xb)(ya + yb); the product is (p0 - p1, p2 - p0 - p1) and xi
// times it (2 p0 - p2, p2 - 2 p1)
template <class C>
KZGX_DEV F29<typename C::Fp29> vw_part(const Fp2<C>& X, const Fp2<C>& Y, int part) {
  using F = typename C::Fp29;
  F29<F> o0 = X.a, o1 = Y.a;
  if (part == 1) {
    o0 = X.b;
    o1 = Y.b;
  } else if (part == 2) {
    o0 = f29_add<F>(X.a, X.b);  // < 4m: the product stays < 16 m^2
    o1 = f29_add<F>(Y.a, Y.b);
  }
  return f29_mul<F>(o0, o1);
}
// add d (x product) or d (xi x product) of parts q[0..2], component im
template <class F>
KZGX_DEV void lin_add_f2(LinAcc<F>& acc, const uint32_t* q, int im, bool xi, int d) {
  constexpr int L = F::L;
  // coefficients of (p0, p1, p2): re (1, -1, 0), im (-1, -1, 1); xi: re (2, 0, -1), im (0, -2, 1)
  const int c0 = xi ? (im ? 0 : 2) : (im ? -1 : 1);
  const int c1 = xi ? (im ? -2 : 0) : -1;
  const int c2 = xi ? (im ? 1 : -1) : (im ? 1 : 0);
  lin_add<F>(acc, q, d * c0);
  lin_add<F>(acc, q + L, d * c1);
  lin_add<F>(acc, q + 2 * L, d * c2);
}

// product parts (16-byte aligned, stride VWave::PL): 128-bit LDS accesses
template <class C>
KZGX_DEV void vw_stp(uint32_t* p, const F29<typename C::Fp29>& a) {
  constexpr int L = C::Fp29::L;
#pragma unroll
  for (int i = 0; i + 4 <= L; i += 4)
    *reinterpret_cast<uint4*>(p + i) = make_uint4(a.v[i], a.v[i + 1], a.v[i + 2], a.v[i + 3]);
#pragma unroll
  for (int i = L & ~3; i < L; i++) p[i] = a.v[i];
}
template <class F>
KZGX_DEV void lin_addp(LinAcc<F>& a, const uint32_t* p, int c) {
  constexpr int L = F::L;
  uint32_t w[L];
#pragma unroll
  for (int i = 0; i + 4 <= L; i += 4) {
    const uint4 q = *reinterpret_cast<const uint4*>(p + i);
    w[i] = q.x;
    w[i + 1] = q.y;
    w[i + 2] = q.z;
    w[i + 3] = q.w;
  }
#pragma unroll
  for (int i = L & ~3; i < L; i++) w[i] = p[i];
#pragma unroll
  for (int l = 0; l < L; l++) a.v[l] += (int64_t)(int32_t)w[l] * (int64_t)c;
}
// lin_add_f2 over a part triple at stride PL
template <class F, int PL>
KZGX_DEV void lin_add_f2p(LinAcc<F>& acc, const uint32_t* q, int im, bool xi, int d) {
  const int c0 = xi ? (im ? 0 : 2) : (im ? -1 : 1);
  const int c1 = xi ? (im ? -2 : 0) : -1;
  const int c2 = xi ? (im ? 1 : -1) : (im ? 1 : 0);
  lin_addp<F>(acc, q, d * c0);
  lin_addp<F>(acc, q + PL, d * c1);
  lin_addp<F>(acc, q + 2 * PL, d * c2);
}

// The ops' synchronisation: a workgroup barrier (WS = false: every wave of
// the block runs the same op sequence), or (WS = true: each wave runs its own
// sequence on its own slots and product parts, vw_hard_bn2) only this wave's
// LDS accesses completed and a compiler barrier -- a wave's lanes exchange
// through LDS with no other wave involved
template <bool WS>
KZGX_DEV void vw_sync() {
  if constexpr (WS) __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  else __syncthreads();
}
template <bool WS>
KZGX_DEV int vw_lane() {
  return WS ? (int)(threadIdx.x & 63) : (int)threadIdx.x;
}

// ---- Fp12 (w basis) in LDS, wave-cooperative; every op ends with a barrier
// dst = a b (dst may alias a or b): the 36 Fp2 products a_i b_j as 108 Fp
// (Karatsuba) parts, two independent products per lane (54 lanes), then lane
// (k, im) < 12 folds the six products landing on w^k (xi for the wrapped
// ones) lazily
template <class C, bool WS = false>
KZGX_DEV void vw_mul(uint32_t dst_o, uint32_t a_o, uint32_t b_o, uint32_t prod_o) {
  uint32_t *dst = vw_smem + dst_o, *prod = vw_smem + prod_o;
  const uint32_t *a = vw_smem + a_o, *b = vw_smem + b_o;
  using F = typename C::Fp29;
  constexpr int E2 = VWave<C>::E2, L = VWave<C>::L, PL = VWave<C>::PL;
  const int lane = vw_lane<WS>();
  // the 108 parts over the block: two per lane on one wave, one per lane
  // when the kernel runs two waves (k_verify_wave / k_pair2_wave) in step
  const int nt = (!WS && (int)blockDim.x >= 108) ? 108 : 54;
  if (lane < nt) {
#pragma unroll 1
    for (int t = lane; t < 108; t += nt) {
      const int pr = t / 3;
      vw_stp<C>(prod + t * PL, vw_part<C>(vw_ld2<C>(a + (pr / 6) * E2), vw_ld2<C>(b + (pr % 6) * E2), t % 3));
    }
  }
  vw_sync<WS>();
  if (lane < 24) {
    // c_k = sum_{i+j=k} p_ij + xi sum_{i+j=k+6} p_ij; lanes 2 o, 2 o + 1
    // take i = h, h + 2, h + 4 (h = lane & 1) of output o = (k, im)
    const int o = lane >> 1, h = lane & 1, k = o >> 1, im = o & 1;
    LinAcc<F> acc;
    lin_init<F>(acc);
#pragma unroll
    for (int i2 = 0; i2 < 3; i2++) {
      const int i = 2 * i2 + h;
      const bool wrap = i > k;
      const int j = wrap ? k + 6 - i : k - i;
      lin_add_f2p<F, PL>(acc, prod + (i * 6 + j) * 3 * PL, im, wrap, 1);
    }
    lin_pair_sum<F>(acc);
    if (!h) vw_st<C>(dst + k * E2 + im * L, lin_fin<F>(acc));
  }
  vw_sync<WS>();
}

// f = f l for a scaled line l = (l0, l1, l3) at positions (POS0, POS1, POS3):
// 18 Fp2 products f_i l_t as 54 Fp (Karatsuba) parts, one per lane, then
// lane (k, im) < 12 folds the three products landing on w^k (xi for the
// wrapped ones) lazily
template <class C, bool WS = false>
KZGX_DEV void vw_mul_line(uint32_t f_o, uint32_t line_o, uint32_t prod_o, int lane) {
  using F = typename C::Fp29;
  using V = VWave<C>;
  constexpr int E2 = V::E2, L = V::L, PL = V::PL;
  uint32_t *f = vw_smem + f_o, *prod = vw_smem + prod_o;
  const uint32_t* line = vw_smem + line_o;
  if (lane < 54) {
    const int i = lane / 9, t = (lane / 3) % 3;
    vw_stp<C>(prod + lane * PL, vw_part<C>(vw_ld2<C>(f + i * E2), vw_ld2<C>(line + t * E2), lane % 3));
  }
  vw_sync<WS>();
  if (lane < 12) {
    // (three terms: a two-lane split measured slower, 2.29 vs 1.98 us)
    const int k = lane >> 1, im = lane & 1;
    LinAcc<F> acc;
    lin_init<F>(acc);
#pragma unroll
    for (int t = 0; t < 3; t++) {
      const int pos = t == 0 ? V::POS0 : t == 1 ? V::POS1 : V::POS3;
      int i = k - pos;
      const bool wrap = i < 0;
      if (wrap) i += 6;
      lin_add_f2p<F, PL>(acc, prod + (i * 9 + t * 3) * PL, im, wrap, 1);
    }
    vw_st<C>(f + k * E2 + im * L, lin_fin<F>(acc));
  }
  vw_sync<WS>();
}

// dst = a^2 for any a: the 21 products a_i a_j (i <= j) as 63 Fp
// (Karatsuba) parts, one per lane; lane (k, im) < 12 folds the pairs with
// i + j = k and, times xi, i + j = k + 6 (cross terms doubled)
template <class C>
KZGX_DEV int vw_pair_index(int i, int j) {
  return i * 6 - (i * (i - 1)) / 2 + (j - i);
}
template <class C, bool WS = false>
KZGX_DEV void vw_sqr(uint32_t dst_o, uint32_t a_o, uint32_t prod_o, int lane) {
  using F = typename C::Fp29;
  constexpr int E2 = VWave<C>::E2, L = VWave<C>::L, PL = VWave<C>::PL;
  uint32_t *dst = vw_smem + dst_o, *prod = vw_smem + prod_o;
  const uint32_t* a = vw_smem + a_o;
  if (lane < 63) {
    int idx = lane / 3, i = 0;
    while (idx >= 6 - i) {
      idx -= 6 - i;
      i++;
    }
    vw_stp<C>(prod + lane * PL, vw_part<C>(vw_ld2<C>(a + i * E2), vw_ld2<C>(a + (i + idx) * E2), lane % 3));
  }
  vw_sync<WS>();
  if (lane < 24) {
    // c_k = sum_i a_i a_{(k - i) mod 6} (xi for the wrapped ones): one
    // uniform pass over i, reading the unordered pair's parts -- a cross
    // pair (i, j) is met at i and at j, so it counts twice (the lanes'
    // divergent walk over i <= j executed the union: twice the loads).
    // Lanes 2 o, 2 o + 1 of output o = (k, im) take i = h, h + 2, h + 4.
    const int o = lane >> 1, h = lane & 1, k = o >> 1, im = o & 1;
    LinAcc<F> acc;
    lin_init<F>(acc);
#pragma unroll
    for (int i2 = 0; i2 < 3; i2++) {
      const int i = 2 * i2 + h;
      const bool wrap = i > k;
      const int j = wrap ? k + 6 - i : k - i;
      const int lo = i < j ? i : j, hi = i < j ? j : i;
      lin_add_f2p<F, PL>(acc, prod + 3 * vw_pair_index<C>(lo, hi) * PL, im, wrap, 1);
    }
    lin_pair_sum<F>(acc);
    if (!h) vw_st<C>(dst + k * E2 + im * L, lin_fin<F>(acc));
  }
  vw_sync<WS>();
}

// Granger-Scott squaring of a cyclotomic element (f12_cyclo_sqr) with one Fp
// product per lane.  In the w basis the three Fp4 squarings pair (a_j, a_{j+3}),
// j = 0, 1, 2: fp4_sqr(x, y) needs t = x y and u = (x + y)(x + xi y), each
// an Fp2 Karatsuba product of 3 Fp products -> 18 lanes.  The operands are
// formed lazily: limb-wise sums of the loaded coefficients (xi y and the
// sums inside a Karatsuba part folded in), 2m added limb-wise under the one
// negative term, then a single carry pass -- values < 10 m, products
// < 80 m^2 < (R/m) m^2.  Then, with c0_j = u - t - xi t and c1_j = 2 t:
//   a0' = 3 c0_0 - 2 a0   a2' = 3 c0_1 - 2 a2   a4' = 3 c0_2 - 2 a4
//   a3' = 3 c1_0 + 2 a3   a5' = 3 c1_1 + 2 a5   a1' = 3 xi c1_2 + 2 a1
// In parts p (of t) and q (of u):
//   c0.re = q0 - q1 - 3 p0 + p1 + p2      c0.im = q2 - q0 - q1 + p0 + 3 p1 - 2 p2
//   c1.re = 2 p0 - 2 p1                   c1.im = 2 p2 - 2 p0 - 2 p1
//   (xi c1).re = 4 p0 - 2 p2              (xi c1).im = 2 p2 - 4 p1
// folded in one lazy sum per output component (3 x the parts, +-2 a_k).
template <class F>
KZGX_DEV F29<F> vw_norm(const uint32_t (&o)[F::L]) {
  F29<F> r;
  uint32_t c = 0;
#pragma unroll
  for (int l = 0; l < F::L; l++) {
    const uint32_t t = o[l] + c;
    r.v[l] = l + 1 < F::L ? (t & M29) : t;
    c = t >> 29;
  }
  return r;
}
// PH (measurement only, k_vw_bench): 1 = the product round alone, 2 = the
// fold round alone, 3 = the op
// one carry step for every limb at once (no chain): limbs < 2^32 in, limbs
// < 2^29 + 8 out (the top limb absorbs), the value unchanged.  f29_mul's
// column sums stay < 2^62 with such limbs; the product's bound depends only
// on the values (< 10 m here).
template <class F>
KZGX_DEV F29<F> vw_norm1(const uint32_t (&o)[F::L]) {
  F29<F> r;
  r.v[0] = o[0] & M29;
#pragma unroll
  for (int l = 1; l < F::L; l++) r.v[l] = (l + 1 < F::L ? (o[l] & M29) : o[l]) + (o[l - 1] >> 29);
  return r;
}
// L limbs from LDS with 64-bit accesses: ODD = the first limb sits at an odd
// word (slots and coefficients start at even words; the imaginary part of an
// Fp2 at +L)
template <int L, bool ODD>
KZGX_DEV void vw_ld_limbs(const uint32_t* p, uint32_t (&v)[L]) {
  constexpr int S = ODD ? 1 : 0;
  if (ODD) v[0] = p[0];
#pragma unroll
  for (int i = 0; S + 2 * i + 1 < L; i++) {
    const uint2 t = *reinterpret_cast<const uint2*>(p + S + 2 * i);
    v[S + 2 * i] = t.x;
    v[S + 2 * i + 1] = t.y;
  }
  if ((L - S) & 1) v[L - 1] = p[L - 1];
}

template <class C, bool WS = false, int PH = 3>
KZGX_DEV void vw_cyclo_sqr(uint32_t dst_o, uint32_t a_o, uint32_t prod_o) {
  using F = typename C::Fp29;
  constexpr int E2 = VWave<C>::E2, L = VWave<C>::L, PL = VWave<C>::PL;
  uint32_t *dst = vw_smem + dst_o, *prod = vw_smem + prod_o;
  const uint32_t* a = vw_smem + a_o;
  const int lane = vw_lane<WS>();
  if ((PH & 1) && lane < 18) {
    const int j = lane / 6, which = (lane / 3) & 1, part = lane % 3;
    const uint32_t *xp = a + j * E2, *yp = a + (j + 3) * E2;
    // part 0: (re, re), 1: (im, im), 2: (re + im, re + im) of
    // t: (x, y);  u: (x + y, x + xi y), x + xi y = (xa + ya - yb, xb + ya + yb)
    const uint32_t e0 = part != 1 ? ~0u : 0u, e1 = part != 0 ? ~0u : 0u, w = which ? ~0u : 0u;
    const uint32_t y2 = part == 2 ? ~0u : 0u, yn = part == 0 ? ~0u : 0u, yp1 = part == 1 ? ~0u : 0u;
    uint32_t o0[L], o1[L], XA[L], XB[L], YA[L], YB[L];
    vw_ld_limbs<L, false>(xp, XA);
    vw_ld_limbs<L, (L & 1) != 0>(xp + L, XB);
    vw_ld_limbs<L, false>(yp, YA);
    vw_ld_limbs<L, (L & 1) != 0>(yp + L, YB);
#pragma unroll
    for (int l = 0; l < L; l++) {
      const uint32_t xa = XA[l], xb = XB[l], ya = YA[l], yb = YB[l];
      const uint32_t sx = (xa & e0) + (xb & e1), sy = (ya & e0) + (yb & e1);
      o0[l] = sx + (sy & w);
      const uint32_t u1 = sx + ya + (ya & y2) + ((F::P2B[l] - yb) & yn) + (yb & yp1);
      o1[l] = which ? u1 : sy;
    }
    vw_stp<C>(prod + lane * PL, f29_mul<F>(vw_norm1<F>(o0), vw_norm1<F>(o1)));
  }
  vw_sync<WS>();
  if ((PH & 2) && lane < 24) {
    // lanes 2 o, 2 o + 1 of output o = (k, im): the t parts / the u parts and 2 a_k
    const int o = lane >> 1, h = lane & 1, k = o >> 1, im = o & 1;
    const int j = (k & 1) ? (k == 3 ? 0 : k == 5 ? 1 : 2) : (k >> 1);
    const uint32_t* q = prod + j * 6 * PL;
    int cp0, cp1, cp2, cq0 = 0, cq1 = 0, cq2 = 0;
    if (!(k & 1)) {
      cp0 = im ? 1 : -3;
      cp1 = im ? 3 : 1;
      cp2 = im ? -2 : 1;
      cq0 = im ? -1 : 1;
      cq1 = -1;
      cq2 = im ? 1 : 0;
    } else if (k != 1) {
      cp0 = im ? -2 : 2;
      cp1 = -2;
      cp2 = im ? 2 : 0;
    } else {
      cp0 = im ? 0 : 4;
      cp1 = im ? -4 : 0;
      cp2 = im ? 2 : -2;
    }
    // one instruction stream for both halves (selected addresses and
    // coefficients: an if / else on h would run both sides masked); the
    // h = 0 lane adds a_k with coefficient 0
    LinAcc<F> acc;
    lin_init<F>(acc);
    const uint32_t* qh = q + 3 * h * PL;
    lin_addp<F>(acc, qh, 3 * (h ? cq0 : cp0));
    lin_addp<F>(acc, qh + PL, 3 * (h ? cq1 : cp1));
    lin_addp<F>(acc, qh + 2 * PL, 3 * (h ? cq2 : cp2));
    lin_add<F>(acc, a + k * E2 + im * L, h ? ((k & 1) ? 2 : -2) : 0);
    lin_pair_sum<F>(acc);
    if (!h) vw_st<C>(dst + k * E2 + im * L, lin_fin<F>(acc));
  }
  vw_sync<WS>();
}

template <class C, bool WS = false>
KZGX_DEV void vw_copy(uint32_t dst_o, uint32_t a_o) {
  uint32_t* dst = vw_smem + dst_o;
  const uint32_t* a = vw_smem + a_o;
  // (at most two waves copy: k_pair2_fused's third wave has left by then)
  const int step = WS ? 64 : ((int)blockDim.x < 128 ? (int)blockDim.x : 128);
  for (int w = vw_lane<WS>(); w < VWave<C>::E12; w += step) dst[w] = a[w];
  vw_sync<WS>();
}

template <class C, bool WS = false>
KZGX_DEV void vw_conj(uint32_t dst_o, uint32_t a_o, int lane) {
  uint32_t* dst = vw_smem + dst_o;
  const uint32_t* a = vw_smem + a_o;
  using F = typename C::Fp29;
  constexpr int L = VWave<C>::L;
  if (lane < 12) {
    const int k = lane >> 1;
    const F29<F> v = vw_ld<C>(a + lane * L);
    vw_st<C>(dst + lane * L, (k & 1) ? fp_neg<F>(v) : v);
  }
  vw_sync<WS>();
}

// dst = a^p: coefficient k is conj(a_k) g_k (g_k = P::FROB[k]); lane (k, t)
// < 24 forms one of the four Fp products of conj(a_k) g_k, lane (k, im) < 12
// folds re = a.re g.re + a.im g.im, im = a.re g.im - a.im g.re
template <class C, bool WS = false>
KZGX_DEV void vw_frob(uint32_t dst_o, uint32_t a_o, uint32_t prod_o) {
  uint32_t* dst = vw_smem + dst_o;
  const uint32_t* a = vw_smem + a_o;
  uint32_t* prod = vw_smem + prod_o;
  using P = typename PairOf<C>::T;
  using F = typename C::Fp29;
  constexpr int E2 = VWave<C>::E2, L = VWave<C>::L, PL = VWave<C>::PL;
  const int lane = vw_lane<WS>();
  if (lane < 24) {
    const int k = lane >> 2, t = lane & 3;
    // t: 0 a.re g.re, 1 a.im g.im, 2 a.re g.im, 3 a.im g.re
    F29<F> g;
#pragma unroll
    for (int l = 0; l < L; l++) {
      uint32_t v = 0;
#pragma unroll
      for (int kk = 0; kk < 6; kk++) v = k == kk ? P::FROB[kk][(t == 1 || t == 2) ? 1 : 0][l] : v;
      g.v[l] = v;
    }
    // the chained product form (f29_mul_chain): measured 2.90 vs 3.38 us per
    // Frobenius against the latency-first form (profiles/r05_vw_ops_ab.json)
    vw_stp<C>(prod + lane * PL, f29_mul_chain<F>(vw_ld<C>(a + k * E2 + ((t & 1) ? L : 0)), g));
  }
  vw_sync<WS>();
  if (lane < 12) {
    const int k = lane >> 1, im = lane & 1;
    const uint32_t* q = prod + k * 4 * PL;
    LinAcc<F> acc;
    lin_init<F>(acc);
    lin_addp<F>(acc, q + (im ? 2 : 0) * PL, 1);
    lin_addp<F>(acc, q + (im ? 3 : 1) * PL, im ? -1 : 1);
    vw_st<C>(dst + k * E2 + im * L, lin_fin<F>(acc));
  }
  vw_sync<WS>();
}

// one lane: the tower inverse
template <class C>
KZGX_TW void vw_inv(uint32_t dst_o, uint32_t a_o) {
  uint32_t* dst = vw_smem + dst_o;
  const uint32_t* a = vw_smem + a_o;
  constexpr int E2 = VWave<C>::E2;
  if (threadIdx.x == 0) {
    Fp12<C> x;
    x.c0.c0 = vw_ld2<C>(a + 0 * E2);
    x.c1.c0 = vw_ld2<C>(a + 1 * E2);
    x.c0.c1 = vw_ld2<C>(a + 2 * E2);
    x.c1.c1 = vw_ld2<C>(a + 3 * E2);
    x.c0.c2 = vw_ld2<C>(a + 4 * E2);
    x.c1.c2 = vw_ld2<C>(a + 5 * E2);
    const Fp12<C> r = f12_inv<C>(x);
    vw_st2<C>(dst + 0 * E2, r.c0.c0);
    vw_st2<C>(dst + 1 * E2, r.c1.c0);
    vw_st2<C>(dst + 2 * E2, r.c0.c1);
    vw_st2<C>(dst + 3 * E2, r.c1.c1);
    vw_st2<C>(dst + 4 * E2, r.c0.c2);
    vw_st2<C>(dst + 5 * E2, r.c1.c2);
  }
  __syncthreads();
}

// dst = a^-1 by the whole wave (replaces the one-lane tower inverse, ~140 us
// on BN254 -- a hundred dependent Fp products in one lane): with conj the
// p^6-Frobenius (odd coefficients negated),
//   a^-1 = conj(a) / N,   N = a conj(a) = n0 + n1 v + n2 v^2 in Fp6 (v = w^2),
//   N^-1 = (A + B v + C v^2) / F,  A = n0^2 - xi n1 n2,  B = xi n2^2 - n0 n1,
//   C = n1^2 - n0 n2,  F = n0 A + xi (n2 B + n1 C) in Fp2,
//   F^-1 = conj2(F) / (F.re^2 + F.im^2), one Fp inversion (wave-uniform).
// Rounds of Karatsuba parts, one per lane, with lazy folds; ta, tb are two
// free slots (ta = conj(a); tb = N, then A, B, C in its odd positions, then
// N^-1 in its even positions).
template <class C>
KZGX_TW void vw_inv_wave(uint32_t dst_o, uint32_t a_o, uint32_t ta_o, uint32_t tb_o, uint32_t prod_o) {
  using F = typename C::Fp29;
  constexpr int E2 = VWave<C>::E2, L = VWave<C>::L, PL = VWave<C>::PL;
  uint32_t* prod = vw_smem + prod_o;
  uint32_t* tb = vw_smem + tb_o;
  uint32_t* sc = prod + 64 * L;  // scratch past the parts: F (2L), t (L), F^-1 (2L)
  const int lane = threadIdx.x;
  vw_conj<C>(ta_o, a_o, lane);
  vw_mul<C>(tb_o, a_o, ta_o, prod_o);
  // (n0, n1, n2) = tb[0], tb[2], tb[4]
  // round A: n0^2, n1 n2, n2^2, n0 n1, n1^2, n0 n2
  if (lane < 18) {
    const int pr = lane / 3;
    const int x = pr == 0 ? 0 : pr == 1 ? 2 : pr == 2 ? 4 : pr == 3 ? 0 : pr == 4 ? 2 : 0;
    const int y = pr == 0 ? 0 : pr == 1 ? 4 : pr == 2 ? 4 : pr == 3 ? 2 : pr == 4 ? 2 : 4;
    vw_stp<C>(prod + lane * PL, vw_part<C>(vw_ld2<C>(tb + x * E2), vw_ld2<C>(tb + y * E2), lane % 3));
  }
  __syncthreads();
  if (lane < 6) {  // A, B, C -> tb[1], tb[3], tb[5]
    const int c = lane >> 1, im = lane & 1;
    LinAcc<F> acc;
    lin_init<F>(acc);
    if (c == 0) {
      lin_add_f2p<F, PL>(acc, prod + 0 * 3 * PL, im, false, 1);
      lin_add_f2p<F, PL>(acc, prod + 1 * 3 * PL, im, true, -1);
    } else if (c == 1) {
      lin_add_f2p<F, PL>(acc, prod + 2 * 3 * PL, im, true, 1);
      lin_add_f2p<F, PL>(acc, prod + 3 * 3 * PL, im, false, -1);
    } else {
      lin_add_f2p<F, PL>(acc, prod + 4 * 3 * PL, im, false, 1);
      lin_add_f2p<F, PL>(acc, prod + 5 * 3 * PL, im, false, -1);
    }
    vw_st<C>(tb + (2 * c + 1) * E2 + im * L, lin_fin<F>(acc));
  }
  __syncthreads();
  // round B: n0 A, n2 B, n1 C -> F = n0 A + xi (n2 B + n1 C)
  if (lane < 9) {
    const int pr = lane / 3;
    const int x = pr == 0 ? 0 : pr == 1 ? 4 : 2;
    vw_stp<C>(prod + lane * PL, vw_part<C>(vw_ld2<C>(tb + x * E2), vw_ld2<C>(tb + (2 * pr + 1) * E2), lane % 3));
  }
  __syncthreads();
  if (lane < 2) {
    LinAcc<F> acc;
    lin_init<F>(acc);
    lin_add_f2p<F, PL>(acc, prod, lane, false, 1);
    lin_add_f2p<F, PL>(acc, prod + 3 * PL, lane, true, 1);
    lin_add_f2p<F, PL>(acc, prod + 6 * PL, lane, true, 1);
    vw_st<C>(sc + lane * L, lin_fin<F>(acc));
  }
  __syncthreads();
  // round C: t = F.re^2 + F.im^2
  if (lane < 2) {
    const F29<F> v = vw_ld<C>(sc + lane * L);
    vw_stp<C>(prod + lane * PL, f29_mul<F>(v, v));
  }
  __syncthreads();
  if (lane == 0) {
    LinAcc<F> acc;
    lin_init<F>(acc);
    lin_addp<F>(acc, prod, 1);
    lin_addp<F>(acc, prod + PL, 1);
    vw_st<C>(sc + 2 * L, lin_fin<F>(acc));
  }
  __syncthreads();
  // t^-1 by the whole wave (lane 0's value, binary GCD on the scalar ALU)
  const F29<F> ti = f29_inv_uniform<F, C::Fp::N>(vw_ld<C>(sc + 2 * L), C::Fp::P);
  // F^-1 = (F.re t^-1, -F.im t^-1)
  if (lane < 2) {
    const F29<F> v = f29_mul<F>(vw_ld<C>(sc + lane * L), ti);
    vw_st<C>(sc + 3 * L + lane * L, lane ? fp_neg<F>(v) : v);
  }
  __syncthreads();
  // round E: A F^-1, B F^-1, C F^-1 -> tb = [A', 0, B', 0, C', 0]
  if (lane < 9) {
    const int pr = lane / 3;
    vw_stp<C>(prod + lane * PL, vw_part<C>(vw_ld2<C>(tb + (2 * pr + 1) * E2), vw_ld2<C>(sc + 3 * L), lane % 3));
  }
  __syncthreads();
  if (lane < 12) {
    const int k = lane >> 1, im = lane & 1;
    F29<F> v = f29_zero<F>();
    if (!(k & 1)) {
      LinAcc<F> acc;
      lin_init<F>(acc);
      lin_add_f2p<F, PL>(acc, prod + (k >> 1) * 3 * PL, im, false, 1);
      v = lin_fin<F>(acc);
    }
    vw_st<C>(tb + k * E2 + im * L, v);
  }
  __syncthreads();
  vw_mul<C>(dst_o, ta_o, tb_o, prod_o);
}

// final exponentiation as a small program over Fp12 slots (the chains of
// final_exp), run by one loop so that every wave-wide op is inlined once and
// no call (with its register save / restore through scratch) sits between
// rounds.
enum : uint8_t { VW_MUL, VW_CSQR, VW_CONJ, VW_FROB, VW_INV, VW_POWZ, VW_POWS, VW_POWK3, VW_SYNC, VW_END };
// BN254 easy part f^(p^6 - 1)(p^2 + 1) -> g (slot 1), both waves in step
__constant__ uint8_t vw_fe_bn[][4] = {{VW_INV, 2, 0, 0},  {VW_CONJ, 1, 0, 0}, {VW_MUL, 1, 1, 2},
                                      {VW_FROB, 2, 1, 0}, {VW_FROB, 2, 2, 0}, {VW_MUL, 1, 2, 1}};
// BN254 hard part in u, a = g^u, b = a^u, c = b^u:
//   f = conj(c^36 b^30 a^18 g^2) (conj(c^36 b^18 a^12) g)^p (b^6 g)^(p^2) g^(p^3),
// on two waves, each on its own program and slots with per-wave syncs
// (VW_SYNC: both waves meet).  Wave 0 runs the chain of exponentiations by u
// (3 x 62 cyclotomic squarings, the critical path); wave 1 meanwhile builds
// every factor that does not involve c -- during b = a^u the a-chain
// (a^6, a^12, a^18 = a^12 a^6, shared as in round 5), g^2 and g^(p^3); during
// c = b^u the b-chain (b^6, b^12, b^18, b^30), X1 = b^30 a^18 g^2,
// X2 = b^18 a^12 and X34 = (b^6 g)^(p^2) g^(p^3) -- so after c only c^36, two
// products per wave and one more product remain:
//   T1 = conj(c^36 X1) X34 (wave 0),  T2 = (conj(c^36 X2) g)^p (wave 1),  f = T1 T2.
// Slots: 1 g, 4 a, 5 b, 6 c, 7 c^36, 8 T1, 9-14 wave 1's (10 X1, 11 X2, 12 X34, 13 T2).
__constant__ uint8_t vw_hard_bn[2][34][4] = {
    {{VW_POWZ, 4, 1, 0}, {VW_SYNC, 0, 0, 0}, {VW_POWZ, 5, 4, 0}, {VW_SYNC, 0, 0, 0}, {VW_POWZ, 6, 5, 0},
     {VW_SYNC, 0, 0, 0}, {VW_POWS, 7, 6, 36}, {VW_SYNC, 0, 0, 0}, {VW_MUL, 8, 7, 10}, {VW_CONJ, 8, 8, 0},
     {VW_MUL, 8, 8, 12}, {VW_SYNC, 0, 0, 0}, {VW_MUL, 0, 8, 13}, {VW_SYNC, 0, 0, 0}, {VW_END, 0, 0, 0}},
    {{VW_SYNC, 0, 0, 0},
     // a^3 -> 9, a^6 -> 10, a^12 -> 11, a^18 -> 10, g^2 -> 9, a^18 g^2 -> 10, g^(p^3) -> 12
     {VW_CSQR, 9, 4, 0}, {VW_MUL, 9, 9, 4}, {VW_CSQR, 10, 9, 0}, {VW_CSQR, 11, 10, 0}, {VW_MUL, 10, 11, 10},
     {VW_CSQR, 9, 1, 0}, {VW_MUL, 10, 10, 9}, {VW_FROB, 12, 1, 0}, {VW_FROB, 12, 12, 0}, {VW_FROB, 12, 12, 0},
     {VW_SYNC, 0, 0, 0},
     // b^3 -> 9, b^6 -> 13, b^12 -> 9, b^18 -> 14, b^30 -> 9, X1 -> 10, X2 -> 11, (b^6 g)^(p^2) -> 13, X34 -> 12
     {VW_CSQR, 9, 5, 0}, {VW_MUL, 9, 9, 5}, {VW_CSQR, 13, 9, 0}, {VW_CSQR, 9, 13, 0}, {VW_MUL, 14, 9, 13},
     {VW_MUL, 9, 14, 9}, {VW_MUL, 10, 9, 10}, {VW_MUL, 11, 14, 11}, {VW_MUL, 13, 13, 1}, {VW_FROB, 13, 13, 0},
     {VW_FROB, 13, 13, 0}, {VW_MUL, 12, 13, 12},
     {VW_SYNC, 0, 0, 0}, {VW_SYNC, 0, 0, 0},
     {VW_MUL, 13, 7, 11}, {VW_CONJ, 13, 13, 0}, {VW_MUL, 13, 13, 1}, {VW_FROB, 13, 13, 0},
     {VW_SYNC, 0, 0, 0}, {VW_SYNC, 0, 0, 0}, {VW_END, 0, 0, 0}}};
// easy part, then BLS12: t = g^K3, t2 = t^(x + p), t3 = t2^(x^2 + p^2 - 1), f = t3 g
__constant__ uint8_t vw_fe_bls[][4] = {
    {VW_INV, 2, 0, 0},  {VW_CONJ, 1, 0, 0}, {VW_MUL, 1, 1, 2},  {VW_FROB, 2, 1, 0}, {VW_FROB, 2, 2, 0},
    {VW_MUL, 1, 2, 1},  {VW_POWK3, 2, 1, 0}, {VW_POWZ, 3, 2, 0}, {VW_FROB, 2, 2, 0}, {VW_MUL, 3, 3, 2},
    {VW_POWZ, 4, 3, 0}, {VW_POWZ, 5, 4, 0}, {VW_FROB, 2, 3, 0}, {VW_FROB, 2, 2, 0}, {VW_MUL, 5, 5, 2},
    {VW_CONJ, 2, 3, 0}, {VW_MUL, 5, 5, 2},  {VW_MUL, 0, 5, 1}};

// run nops ops of prog (WS: this wave's own program, per-wave syncs, VW_SYNC
// a workgroup barrier; else every wave in step)
template <class C, bool WS>
KZGX_TW void vw_fe_run(const uint8_t (*prog)[4], int nops, uint32_t slots, uint32_t prod) {
  using P = typename PairOf<C>::T;
  constexpr int E = VWave<C>::E12;
  const int lane = vw_lane<WS>();
  for (int k = 0; k < nops; k++) {
    // the op as uniform (SGPR) values: the program pointer reaches this
    // non-inlined function in VGPRs, and a switch on a per-lane value would
    // put the barrier of VW_SYNC under an exec mask (skipped only while the
    // compiler happens to branch around empty-exec blocks)
    uint32_t op[4];
#pragma unroll
    for (int j = 0; j < 4; j++) op[j] = __builtin_amdgcn_readfirstlane((uint32_t)prog[k][j]);
    const uint32_t d = slots + op[1] * E, a = slots + op[2] * E, b = slots + op[3] * E;
    switch (op[0]) {
      case VW_END: return;
      case VW_SYNC: __syncthreads(); break;
      case VW_MUL: vw_mul<C, WS>(d, a, b, prod); break;
      case VW_CSQR: vw_cyclo_sqr<C, WS>(d, a, prod); break;
      case VW_CONJ: vw_conj<C, WS>(d, a, lane); break;
      case VW_FROB: vw_frob<C, WS>(d, a, prod); break;
      case VW_INV:
        if constexpr (!WS) vw_inv_wave<C>(d, a, slots + 7 * E, slots + 8 * E, prod);
        break;
      default: {  // d = a^e (cyclotomic a, top bit of e set), d != a
        uint64_t e0 = op[3], e1 = 0;
        int bits = 32 - __builtin_clz((uint32_t)op[3] | 1u);
        if (op[0] == VW_POWZ) {
          e0 = P::Z_ABS;
          bits = 64 - __builtin_clzll(P::Z_ABS);
        } else if (op[0] == VW_POWK3) {
          e0 = P::K3[0];
          e1 = P::K3[1];
          bits = P::K3_BITS;
        }
        vw_copy<C, WS>(d, a);
#pragma unroll 1
        for (int i = bits - 2; i >= 0; i--) {
          vw_cyclo_sqr<C, WS>(d, d, prod);
          if (((i < 64 ? e0 >> i : e1 >> (i - 64)) & 1ull)) vw_mul<C, WS>(d, d, a, prod);
        }
        if (op[0] == VW_POWZ && P::Z_NEG) vw_conj<C, WS>(d, d, lane);
      }
    }
  }
}

// The final exponentiation of slot 0 into slot 0.  BN254 needs the block's
// two waves (k_verify_wave / k_pair2_wave launch 128 threads): the easy part
// in step, then the hard part on one program per wave (vw_hard_bn).
template <class C>
KZGX_TW void vw_final_exp(uint32_t slots, uint32_t prod) {
  using P = typename PairOf<C>::T;
  if constexpr (P::IS_BN) {
    vw_fe_run<C, false>(vw_fe_bn, (int)(sizeof(vw_fe_bn) / 4), slots, prod);
    // the wave index as a uniform (SGPR) value: each wave's program, and so
    // every branch around its barriers, is then uniform control flow
    const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    vw_fe_run<C, true>(vw_hard_bn[w], 34, slots, w ? (uint32_t)VWave<C>::O_PROD2 : prod);
  } else {
    vw_fe_run<C, false>(vw_fe_bls, (int)(sizeof(vw_fe_bls) / 4), slots, prod);
  }
}

// Miller loops of both pairings, one per wave (the kernel runs two waves):
// wave q squares its own f_q and multiplies in pairing q's lines, so a step
// costs one squaring and one line product on the critical path instead of a
// squaring and two line products; then f = f_0 f_1.  Line s is a doubling
// line (square first, except at the top bit), an addition line (after a
// doubling line of a set bit), or (BN) one of the two Frobenius lines after
// the conjugation.  Both waves run the same op sequence, so their barriers
// pair up; an unused pairing (use_mask bit clear) runs on zeroed lines and
// its f_q is replaced by 1 before the product.
template <class C>
KZGX_TW void vw_miller(uint32_t f, int use_mask, uint32_t prod) {
  using P = typename PairOf<C>::T;
  using V = VWave<C>;
  constexpr int NLOOP = V::NL - (P::D_TWIST ? 2 : 0);
  const int q = (int)(threadIdx.x >> 6), lane = (int)(threadIdx.x & 63);
  const uint32_t fq = f + (uint32_t)q * V::E12;
  const uint32_t pq = q ? (uint32_t)V::O_PROD2 : prod;
  int i = P::LOOP_BITS - 2;
  bool add_next = false;
#pragma unroll 1
  for (int s = 0; s < V::NL; s++) {
    if (s < NLOOP) {
      if (add_next) {
        add_next = false;
        i--;
      } else {
        if (i != P::LOOP_BITS - 2) vw_sqr<C>(fq, fq, pq, lane);  // f = 1 before the first line
        add_next = (P::LOOP[i >> 6] >> (i & 63)) & 1ull;
        if (!add_next) i--;
      }
    } else if (s == NLOOP && P::LOOP_NEG) {
      vw_conj<C>(fq, fq, lane);
    }
    vw_mul_line<C>(fq, V::O_LINES + (q * V::NL + s) * V::LW, pq, lane);
  }
  if (NLOOP == V::NL && P::LOOP_NEG) vw_conj<C>(fq, fq, lane);
  // f_q = 1 for an unused pairing (uniform per wave), then f = f_0 f_1
  if (!((use_mask >> q) & 1) && lane < 12) {
    using F = typename C::Fp29;
    vw_st<C>(vw_smem + fq + lane * V::L, lane == 0 ? f29_one<F>() : f29_zero<F>());
  }
  __syncthreads();
  vw_mul<C>(f, f, f + V::E12, prod);
}

// vw_miller with per-wave syncs only (k_pair2_fused): wave q runs pairing
// q's loop on its own slots and product parts, so neither waits at the
// other's barriers; with `wait`, wave 0 takes line s only once the LDS word
// at ready_o (the producer wave's count of published lines) exceeds s
// (ready_o + 1 set: it gave up waiting).  Then
// the workgroup barrier and f = f_0 f_1.
template <class C>
KZGX_TW void vw_miller_ws(uint32_t f, int use_mask, uint32_t prod, uint32_t ready_o, bool wait) {
  using P = typename PairOf<C>::T;
  using V = VWave<C>;
  constexpr int NLOOP = V::NL - (P::D_TWIST ? 2 : 0);
  const int q = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)), lane = (int)(threadIdx.x & 63);
  const uint32_t fq = f + (uint32_t)q * V::E12;
  const uint32_t pq = q ? (uint32_t)V::O_PROD2 : prod;
  const bool w0 = wait && q == 0;
  volatile const uint32_t* ready = vw_smem + ready_o;
  int i = P::LOOP_BITS - 2;
  bool add_next = false;
#pragma unroll 1
  for (int s = 0; s < V::NL; s++) {
    if (s < NLOOP) {
      if (add_next) {
        add_next = false;
        i--;
      } else {
        if (i != P::LOOP_BITS - 2) vw_sqr<C, true>(fq, fq, pq, lane);
        add_next = (P::LOOP[i >> 6] >> (i & 63)) & 1ull;
        if (!add_next) i--;
      }
    } else if (s == NLOOP && P::LOOP_NEG) {
      vw_conj<C, true>(fq, fq, lane);
    }
    if (w0) {
      // bounded (~0.5 s): a producer that never delivers marks the result
      // for the two-launch rerun instead of holding the GPU
      uint32_t spins = 0;
      while ((uint32_t)__builtin_amdgcn_readfirstlane((int)*ready) <= (uint32_t)s) {
        __builtin_amdgcn_s_sleep(2);
        if (++spins == (1u << 22)) {
          if (lane == 0) vw_smem[ready_o + 1] = 1u;
          break;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    }
    vw_mul_line<C, true>(fq, V::O_LINES + (q * V::NL + s) * V::LW, pq, lane);
  }
  if (NLOOP == V::NL && P::LOOP_NEG) vw_conj<C, true>(fq, fq, lane);
  if (!((use_mask >> q) & 1) && lane < 12) {
    using F = typename C::Fp29;
    vw_st<C>(vw_smem + fq + lane * V::L, lane == 0 ? f29_one<F>() : f29_zero<F>());
  }
  __syncthreads();
  vw_mul<C>(f, f, f + V::E12, prod);
}

// The same line table for a variable Q with the G2 chain spread over a wave
// (k_vlines runs it on one lane: ~25 dependent Fp2 operations per step).
// Each step is a few rounds of independent Fp2 products, one Karatsuba part
// per lane, folded lazily (LinAcc):
//   doubling (dbl-2009-l + tangent):  [X^2, Y^2, Z^2, YZ] -> [2YZ ZZ, E ZZ, E X, B^2,
//                                     (X+B)^2, E^2] -> [E (D - X3)]
//   addition (madd-2007-bl + chord): [Z^2] -> [qx Z1Z1, Z Z1Z1] -> [qy ZZZ, H^2, Z H]
//                                     -> [H I, X I, r^2, r qx, qy Z3] -> [Y J, r (V - X3)]
// Any Jacobian representative gives the lines up to Fp2 factors, which the
// final exponentiation removes.  T = O or H = 0 (impossible for Q of order
// r) sets redo[q]; k_vlines_redo then recomputes that table on one lane.
template <class C>
struct VLine {
  static constexpr int L = C::Fp29::L, E2 = 2 * L;
  // Fp2 slots
  enum { X, Y, Z, QX, QY, Q1X, Q1Y, Q2X, Q2Y, A, B, ZZ, YZ, D, CC, Z1Z1, U2, ZZZ, H, R, Z3, I, J, V, NS };
  static constexpr int PROD = NS * E2;  // 18 parts of L words
  static constexpr int FLAG = PROD + 18 * L;
  static constexpr int WORDS = FLAG + 4;
};

template <class C, int OFF = 0>
KZGX_DEV uint32_t* vl_slot(int k) {
  return vw_smem + OFF + k * VLine<C>::E2;
}
// lanes < 3 n: part (lane % 3) of product lane / 3, operands from `ops`
template <class C, int OFF, bool WS, class Ops>
KZGX_DEV void vl_parts(int n, Ops ops) {
  const int lane = vw_lane<WS>();
  if (lane < 3 * n) {
    Fp2<C> x, y;
    ops(lane / 3, x, y);
    vw_st<C>(vw_smem + OFF + VLine<C>::PROD + lane * VLine<C>::L, vw_part<C>(x, y, lane % 3));
  }
  vw_sync<WS>();
}
template <class C, int OFF = 0>
KZGX_DEV const uint32_t* vl_prod(int k) {
  return vw_smem + OFF + VLine<C>::PROD + 3 * k * VLine<C>::L;
}
template <class C, int OFF = 0>
KZGX_DEV const uint32_t* vl_comp(int slot, int im) {
  return vw_smem + OFF + slot * VLine<C>::E2 + im * VLine<C>::L;
}

template <class C, int OFF = 0, bool WS = false>
KZGX_DEV void vl_dbl_wave(uint32_t* out) {
  using F = typename C::Fp29;
  using S = VLine<C>;
  constexpr int L = S::L, E2 = S::E2;
  const int lane = vw_lane<WS>();
  // round 1: A = X^2, B = Y^2, ZZ = Z^2, YZ = Y Z
  vl_parts<C, OFF, WS>(4, [&](int k, Fp2<C>& x, Fp2<C>& y) {
    const int a = k == 0 ? S::X : k == 1 ? S::Y : k == 2 ? S::Z : S::Y;
    const int b = k == 3 ? S::Z : a;
    x = vw_ld2<C>(vl_slot<C, OFF>(a));
    y = vw_ld2<C>(vl_slot<C, OFF>(b));
  });
  if (lane < 8) {
    const int k = lane >> 1, im = lane & 1;
    LinAcc<F> acc;
    lin_init<F>(acc);
    lin_add_f2<F>(acc, vl_prod<C, OFF>(k), im, false, 1);
    const int dst = k == 0 ? S::A : k == 1 ? S::B : k == 2 ? S::ZZ : S::YZ;
    vw_st<C>(vl_slot<C, OFF>(dst) + im * L, lin_fin<F>(acc));
  }
  vw_sync<WS>();
  // round 2: 2YZ ZZ, E ZZ, E X, B^2, (X + B)^2, E^2 with E = 3A
  vl_parts<C, OFF, WS>(6, [&](int k, Fp2<C>& x, Fp2<C>& y) {
    const Fp2<C> a = vw_ld2<C>(vl_slot<C, OFF>(S::A));
    const Fp2<C> E = f2_add<C>(f2_dbl<C>(a), a);
    if (k == 0) {
      x = f2_dbl<C>(vw_ld2<C>(vl_slot<C, OFF>(S::YZ)));
      y = vw_ld2<C>(vl_slot<C, OFF>(S::ZZ));
    } else if (k == 1) {
      x = E;
      y = vw_ld2<C>(vl_slot<C, OFF>(S::ZZ));
    } else if (k == 2) {
      x = E;
      y = vw_ld2<C>(vl_slot<C, OFF>(S::X));
    } else if (k == 3) {
      x = y = vw_ld2<C>(vl_slot<C, OFF>(S::B));
    } else if (k == 4) {
      x = y = f2_add<C>(vw_ld2<C>(vl_slot<C, OFF>(S::X)), vw_ld2<C>(vl_slot<C, OFF>(S::B)));
    } else {
      x = y = E;
    }
  });
  // w0c = P0, w1c = -P1, w3c = P2 - 2B, C = P3, D = 2 P4 - 2A - 2 P3,
  // X3 = P5 - 2D = P5 - 4 P4 + 4A + 4 P3, Z3 = 2 YZ
  if (lane < 14) {
    const int w = lane >> 1, im = lane & 1;
    LinAcc<F> acc;
    lin_init<F>(acc);
    switch (w) {
      case 0: lin_add_f2<F>(acc, vl_prod<C, OFF>(0), im, false, 1); break;
      case 1: lin_add_f2<F>(acc, vl_prod<C, OFF>(1), im, false, -1); break;
      case 2:
        lin_add_f2<F>(acc, vl_prod<C, OFF>(2), im, false, 1);
        lin_add<F>(acc, vl_comp<C, OFF>(S::B, im), -2);
        break;
      case 3: lin_add_f2<F>(acc, vl_prod<C, OFF>(3), im, false, 1); break;
      case 4:
        lin_add_f2<F>(acc, vl_prod<C, OFF>(4), im, false, 2);
        lin_add<F>(acc, vl_comp<C, OFF>(S::A, im), -2);
        lin_add_f2<F>(acc, vl_prod<C, OFF>(3), im, false, -2);
        break;
      case 5:
        lin_add_f2<F>(acc, vl_prod<C, OFF>(5), im, false, 1);
        lin_add_f2<F>(acc, vl_prod<C, OFF>(4), im, false, -4);
        lin_add<F>(acc, vl_comp<C, OFF>(S::A, im), 4);
        lin_add_f2<F>(acc, vl_prod<C, OFF>(3), im, false, 4);
        break;
      default: lin_add<F>(acc, vl_comp<C, OFF>(S::YZ, im), 2); break;
    }
    const F29<F> v = lin_fin<F>(acc);
    if (w < 3) {
      vw_st<C>(out + w * E2 + im * L, v);
    } else {
      const int dst = w == 3 ? S::CC : w == 4 ? S::D : w == 5 ? S::X : S::Z;
      vw_st<C>(vl_slot<C, OFF>(dst) + im * L, v);
    }
  }
  vw_sync<WS>();
  // round 3: Y3 = E (D - X3) - 8 C
  vl_parts<C, OFF, WS>(1, [&](int, Fp2<C>& x, Fp2<C>& y) {
    const Fp2<C> a = vw_ld2<C>(vl_slot<C, OFF>(S::A));
    x = f2_add<C>(f2_dbl<C>(a), a);
    y = f2_sub<C>(vw_ld2<C>(vl_slot<C, OFF>(S::D)), vw_ld2<C>(vl_slot<C, OFF>(S::X)));
  });
  if (lane < 2) {
    LinAcc<F> acc;
    lin_init<F>(acc);
    lin_add_f2<F>(acc, vl_prod<C, OFF>(0), lane, false, 1);
    lin_add<F>(acc, vl_comp<C, OFF>(S::CC, lane), -8);
    vw_st<C>(vl_slot<C, OFF>(S::Y) + lane * L, lin_fin<F>(acc));
  }
  vw_sync<WS>();
  if (lane == 0 && f2_is_zero<C>(vw_ld2<C>(vl_slot<C, OFF>(S::Z)))) vw_smem[OFF + S::FLAG] = 1u;  // T = O
  vw_sync<WS>();
}

// T += q (q = slots qx, qy) and the chord line into out
template <class C, int OFF = 0, bool WS = false>
KZGX_DEV void vl_add_wave(int qx, int qy, uint32_t* out) {
  using F = typename C::Fp29;
  using S = VLine<C>;
  constexpr int L = S::L, E2 = S::E2;
  const int lane = vw_lane<WS>();
  auto fin1 = [&](int k, int dst, int d) {  // lanes 2k, 2k+1: slot dst = d * product k
    if ((lane >> 1) == k) {
      LinAcc<F> acc;
      lin_init<F>(acc);
      lin_add_f2<F>(acc, vl_prod<C, OFF>(k), lane & 1, false, d);
      vw_st<C>(vl_slot<C, OFF>(dst) + (lane & 1) * L, lin_fin<F>(acc));
    }
  };
  // Z1Z1 = Z^2
  vl_parts<C, OFF, WS>(1, [&](int, Fp2<C>& x, Fp2<C>& y) { x = y = vw_ld2<C>(vl_slot<C, OFF>(S::Z)); });
  fin1(0, S::Z1Z1, 1);
  vw_sync<WS>();
  // U2 = qx Z1Z1, ZZZ = Z Z1Z1
  vl_parts<C, OFF, WS>(2, [&](int k, Fp2<C>& x, Fp2<C>& y) {
    x = vw_ld2<C>(vl_slot<C, OFF>(k == 0 ? qx : S::Z));
    y = vw_ld2<C>(vl_slot<C, OFF>(S::Z1Z1));
  });
  fin1(0, S::U2, 1);
  fin1(1, S::ZZZ, 1);
  vw_sync<WS>();
  if (lane < 2) {  // H = U2 - X
    const int im = lane;
    vw_st<C>(vl_slot<C, OFF>(S::H) + im * L, fp_sub<F>(vw_ld<C>(vl_comp<C, OFF>(S::U2, im)), vw_ld<C>(vl_comp<C, OFF>(S::X, im))));
  }
  vw_sync<WS>();
  // S2 = qy ZZZ, HH = H^2, ZH = Z H
  vl_parts<C, OFF, WS>(3, [&](int k, Fp2<C>& x, Fp2<C>& y) {
    x = vw_ld2<C>(vl_slot<C, OFF>(k == 0 ? qy : k == 1 ? S::H : S::Z));
    y = vw_ld2<C>(vl_slot<C, OFF>(k == 0 ? S::ZZZ : S::H));
  });
  // r = 2 (S2 - Y), I = 4 HH, Z3 = 2 ZH
  if (lane < 6) {
    const int w = lane >> 1, im = lane & 1;
    LinAcc<F> acc;
    lin_init<F>(acc);
    lin_add_f2<F>(acc, vl_prod<C, OFF>(w), im, false, w == 1 ? 4 : 2);
    if (w == 0) lin_add<F>(acc, vl_comp<C, OFF>(S::Y, im), -2);
    vw_st<C>(vl_slot<C, OFF>(w == 0 ? S::R : w == 1 ? S::I : S::Z3) + im * L, lin_fin<F>(acc));
  }
  vw_sync<WS>();
  if (lane == 0 && f2_is_zero<C>(vw_ld2<C>(vl_slot<C, OFF>(S::H)))) vw_smem[OFF + S::FLAG] = 1u;  // T = +-q
  // J = H I, V = X I, r^2, r qx, qy Z3
  vl_parts<C, OFF, WS>(5, [&](int k, Fp2<C>& x, Fp2<C>& y) {
    const int a = k == 0 ? S::H : k == 1 ? S::X : k == 4 ? qy : S::R;
    const int b = k <= 1 ? S::I : k == 2 ? S::R : k == 3 ? qx : S::Z3;
    x = vw_ld2<C>(vl_slot<C, OFF>(a));
    y = vw_ld2<C>(vl_slot<C, OFF>(b));
  });
  // J, V; X3 = r^2 - J - 2V; line: w0c = Z3, w1c = -r, w3c = r qx - qy Z3
  if (lane < 12) {
    const int w = lane >> 1, im = lane & 1;
    LinAcc<F> acc;
    lin_init<F>(acc);
    switch (w) {
      case 0: lin_add_f2<F>(acc, vl_prod<C, OFF>(0), im, false, 1); break;
      case 1: lin_add_f2<F>(acc, vl_prod<C, OFF>(1), im, false, 1); break;
      case 2:
        lin_add_f2<F>(acc, vl_prod<C, OFF>(2), im, false, 1);
        lin_add_f2<F>(acc, vl_prod<C, OFF>(0), im, false, -1);
        lin_add_f2<F>(acc, vl_prod<C, OFF>(1), im, false, -2);
        break;
      case 3: lin_add<F>(acc, vl_comp<C, OFF>(S::Z3, im), 1); break;
      case 4: lin_add<F>(acc, vl_comp<C, OFF>(S::R, im), -1); break;
      default:
        lin_add_f2<F>(acc, vl_prod<C, OFF>(3), im, false, 1);
        lin_add_f2<F>(acc, vl_prod<C, OFF>(4), im, false, -1);
        break;
    }
    const F29<F> v = lin_fin<F>(acc);
    if (w < 3)
      vw_st<C>(vl_slot<C, OFF>(w == 0 ? S::J : w == 1 ? S::V : S::D) + im * L, v);  // D holds X3 for now
    else
      vw_st<C>(out + (w - 3) * E2 + im * L, v);
  }
  vw_sync<WS>();
  // Y3 = r (V - X3) - 2 Y J
  vl_parts<C, OFF, WS>(2, [&](int k, Fp2<C>& x, Fp2<C>& y) {
    if (k == 0) {
      x = vw_ld2<C>(vl_slot<C, OFF>(S::R));
      y = f2_sub<C>(vw_ld2<C>(vl_slot<C, OFF>(S::V)), vw_ld2<C>(vl_slot<C, OFF>(S::D)));
    } else {
      x = vw_ld2<C>(vl_slot<C, OFF>(S::Y));
      y = vw_ld2<C>(vl_slot<C, OFF>(S::J));
    }
  });
  if (lane < 6) {  // new T: X = X3, Y = Y3, Z = Z3
    const int w = lane >> 1, im = lane & 1;
    F29<F> v;
    if (w == 0) {
      v = vw_ld<C>(vl_comp<C, OFF>(S::D, im));
    } else if (w == 1) {
      LinAcc<F> acc;
      lin_init<F>(acc);
      lin_add_f2<F>(acc, vl_prod<C, OFF>(0), im, false, 1);
      lin_add_f2<F>(acc, vl_prod<C, OFF>(1), im, false, -2);
      v = lin_fin<F>(acc);
    } else {
      v = vw_ld<C>(vl_comp<C, OFF>(S::Z3, im));
    }
    vw_st<C>(vl_slot<C, OFF>(w) + im * L, v);  // slots X, Y, Z are 0, 1, 2
  }
  vw_sync<WS>();
}

// block q: the line table of Q_q (canonical) into lines + q NL LW
template <class C>
__global__ __launch_bounds__(64) void k_vlines_wave(const uint32_t* __restrict__ g2, uint32_t* __restrict__ lines,
                                                    uint32_t* __restrict__ qfin, uint32_t* __restrict__ redo) {
  using P = typename PairOf<C>::T;
  using V = VWave<C>;
  using S = VLine<C>;
  const int q = blockIdx.x;
  uint32_t* out = lines + (size_t)q * V::NL * V::LW;
  if (threadIdx.x == 0) {
    G2A<C> Q;
    const bool fin = g2_from_canon<C>(g2 + q * 4 * C::Fp::N, Q);
    qfin[q] = fin ? 1u : 0u;
    redo[q] = 0u;
    vw_smem[S::FLAG] = fin ? 0u : 2u;
    vw_st2<C>(vl_slot<C>(S::X), Q.x);
    vw_st2<C>(vl_slot<C>(S::Y), Q.y);
    vw_st2<C>(vl_slot<C>(S::Z), f2_one<C>());
    vw_st2<C>(vl_slot<C>(S::QX), Q.x);
    vw_st2<C>(vl_slot<C>(S::QY), Q.y);
    if (P::D_TWIST) {
      const G2A<C> q1 = twist_frob<C>(Q);
      G2A<C> q2 = twist_frob<C>(q1);
      q2.y = f2_neg<C>(q2.y);
      vw_st2<C>(vl_slot<C>(S::Q1X), q1.x);
      vw_st2<C>(vl_slot<C>(S::Q1Y), q1.y);
      vw_st2<C>(vl_slot<C>(S::Q2X), q2.x);
      vw_st2<C>(vl_slot<C>(S::Q2Y), q2.y);
    }
  }
  __syncthreads();
  if (vw_smem[S::FLAG] == 2u) return;  // Q = O: no table (uniform)
  int s = 0;
  for (int i = P::LOOP_BITS - 2; i >= 0; i--) {
    vl_dbl_wave<C>(out + (s++) * V::LW);
    if ((P::LOOP[i >> 6] >> (i & 63)) & 1ull) vl_add_wave<C>(S::QX, S::QY, out + (s++) * V::LW);
  }
  if (P::LOOP_NEG && threadIdx.x < 2) {
    using F = typename C::Fp29;
    uint32_t* y = vl_slot<C>(S::Y) + threadIdx.x * S::L;
    vw_st<C>(y, fp_neg<F>(vw_ld<C>(y)));
  }
  __syncthreads();
  if (P::D_TWIST) {
    vl_add_wave<C>(S::Q1X, S::Q1Y, out + (s++) * V::LW);
    vl_add_wave<C>(S::Q2X, S::Q2Y, out + (s++) * V::LW);
  }
  if (threadIdx.x == 0 && vw_smem[S::FLAG]) redo[q] = 1u;
}

// single-lane recompute of the tables flagged by k_vlines_wave
template <class C>
__global__ __launch_bounds__(64) void k_vlines_redo(const uint32_t* __restrict__ g2, uint32_t* __restrict__ lines,
                                                    const uint32_t* __restrict__ redo) {
  using P = typename PairOf<C>::T;
  using V = VWave<C>;
  const int q = threadIdx.x;
  if (q >= 2 || !redo[q]) return;
  G2A<C> Q;
  (void)g2_from_canon<C>(g2 + q * 4 * C::Fp::N, Q);
  uint32_t* out = lines + (size_t)q * V::NL * V::LW;
  int s = 0;
  G2J<C> T = g2_from_affine<C>(Q);
  for (int i = P::LOOP_BITS - 2; i >= 0; i--) {
    vl_dbl<C>(T, out + (s++) * V::LW);
    if ((P::LOOP[i >> 6] >> (i & 63)) & 1ull) vl_add<C>(T, Q, out + (s++) * V::LW);
  }
  if (P::LOOP_NEG) T.Y = f2_neg<C>(T.Y);
  if (P::D_TWIST) {
    const G2A<C> q1 = twist_frob<C>(Q);
    G2A<C> q2 = twist_frob<C>(q1);
    q2.y = f2_neg<C>(q2.y);
    vl_add<C>(T, q1, out + (s++) * V::LW);
    vl_add<C>(T, q2, out + (s++) * V::LW);
  }
}

// the product of the two pairings (P_q, Q_q), q = 0, 1, from the line tables
// of Q_0, Q_1 (k_vlines) and the per-pairing scale factors and use flags the
// caller left in LDS (scale: [q][yP, xP, 1] up to an Fp factor; flag[q]);
// *ok_out = (product after the final exponentiation == 1)
template <class C>
KZGX_DEV void vw_pair_tail(const uint32_t* __restrict__ vlines, uint32_t* __restrict__ ok_out) {
  using F = typename C::Fp29;
  using V = VWave<C>;
  constexpr int L = V::L, E2 = V::E2;
  uint32_t* lines = vw_smem + V::O_LINES;
  uint32_t* scale = vw_smem + V::O_SCALE;
  uint32_t* flag = vw_smem + V::O_FLAG;
  const int lane = threadIdx.x;
  const bool use0 = flag[0] != 0, use1 = flag[1] != 0;
  // ---- scale the precomputed lines (zeros for an unused pairing: its
  // wave's Miller loop then runs on zeros, vw_miller)
  for (int t = lane; t < 2 * V::NL * 3; t += blockDim.x) {
    const int q = t / (3 * V::NL), c = t % 3;
    const uint32_t* src = vlines + (size_t)t * E2;  // [q][s][c] order matches t
    const bool use = q ? use1 : use0;
    vw_st2<C>(lines + t * E2, use ? f2_mul_fp<C>(vw_ld2<C>(src), vw_ld<C>(scale + (q * 3 + c) * L)) : f2_zero<C>());
  }
  // f_0 = f_1 = 1 (slots 0 and 1, one per wave)
  constexpr uint32_t f = V::O_SLOT, pr = V::O_PROD;
  if ((lane & 63) < 12)
    vw_st<C>(vw_smem + f + (lane >> 6) * V::E12 + (lane & 63) * L, (lane & 63) == 0 ? f29_one<F>() : f29_zero<F>());
  __syncthreads();
  VW_STAMP(3);
#ifdef KZGX_VW_TIMING
  // which SIMD each of the two waves runs on (HW_ID bits 5:4; CU 11:8)
  if ((threadIdx.x & 63) == 0) vw_ts[10 + (threadIdx.x >> 6)] = __builtin_amdgcn_s_getreg((31 << 11) | 4);
#endif
  vw_miller<C>(f, (use0 ? 1 : 0) | (use1 ? 2 : 0), pr);
  VW_STAMP(4);
  vw_final_exp<C>(V::O_SLOT, pr);
  VW_STAMP(8);
  // ---- f == 1 ?
  if (lane < 12) {
    const F29<F> v = f29_reduce<F>(vw_ld<C>(vw_smem + f + lane * L));
    const F29<F> want = lane == 0 ? f29_reduce<F>(f29_one<F>()) : f29_zero<F>();
    uint32_t diff = 0;
    for (int i = 0; i < L; i++) diff |= v.v[i] ^ want.v[i];
    flag[2 + lane] = diff;
  }
  __syncthreads();
  if (lane == 0) {
    uint32_t bad = 0;
    for (int i = 0; i < 12; i++) bad |= flag[2 + i];
    *ok_out = bad == 0 ? 1u : 0u;
#ifdef KZGX_VW_TIMING
    if (blockIdx.x == 0)
      printf("vw_ts tree %llu d %llu scale %llu miller %llu final_exp %llu (x10ns)\n",
             (unsigned long long)(vw_ts[1] - vw_ts[0]), (unsigned long long)(vw_ts[2] - vw_ts[1]),
             (unsigned long long)(vw_ts[3] - vw_ts[2]), (unsigned long long)(vw_ts[4] - vw_ts[3]),
             (unsigned long long)(vw_ts[8] - vw_ts[4]));
    if (blockIdx.x == 0)
      printf("vw_hwid wave0 simd %u cu %u  wave1 simd %u cu %u\n", (unsigned)((vw_ts[10] >> 4) & 3),
             (unsigned)((vw_ts[10] >> 8) & 15), (unsigned)((vw_ts[11] >> 4) & 3), (unsigned)((vw_ts[11] >> 8) & 15));
#endif
  }
}

// block (one wave) per opening; same contract as k_verify_single
template <class C>
__global__ __launch_bounds__(128) void k_verify_wave(const uint32_t* __restrict__ commits,
                                                    const uint32_t* __restrict__ commit_inf,
                                                    const uint32_t* __restrict__ proofs,
                                                    const uint32_t* __restrict__ proof_inf,
                                                    const uint32_t* __restrict__ zs, const uint32_t* __restrict__ ys,
                                                    uint32_t count, const uint32_t* __restrict__ g1_0,
                                                    const uint32_t* __restrict__ vtab, const uint32_t* __restrict__ vlines,
                                                    const uint32_t* __restrict__ qfin, uint32_t* __restrict__ ok) {
  using F = typename C::Fp29;
  using V = VWave<C>;
  constexpr int N = C::Fp::N, L = V::L;
  uint32_t* prod = vw_smem + V::O_PROD;
  uint32_t* scale = vw_smem + V::O_SCALE;
  uint32_t* flag = vw_smem + V::O_FLAG;
  const uint32_t k = blockIdx.x;
  const int lane = threadIdx.x;
  if (k >= count) return;  // uniform over the block
  VW_STAMP(0);
  // the opening's inputs into LDS, one word per thread (inputs may live in
  // mapped host memory: every later read is then an LDS read)
  uint32_t* in = vw_smem + V::O_IN;
  static_assert(V::I_PINF < 128, "k_verify_wave: one input word per thread");
  if (lane < V::I_P) in[lane] = commits[(size_t)k * 2 * N + lane];
  else if (lane < V::I_Z) in[lane] = proofs[(size_t)k * 2 * N + lane - V::I_P];
  else if (lane < V::I_Y) in[lane] = zs[(size_t)k * 8 + lane - V::I_Z];
  else if (lane < V::I_CINF) in[lane] = ys[(size_t)k * 8 + lane - V::I_Y];
  else if (lane == V::I_CINF) in[lane] = commit_inf ? commit_inf[k] : 0u;
  else if (lane == V::I_PINF) in[lane] = proof_inf ? proof_inf[k] : 0u;
  __syncthreads();
  // ---- [y]G on wave 0: lane w takes window w's table entry, then a tree of
  // group-cooperative additions (coop.hpp, 8 lanes each: 2 + 1 + 1 + 1 + 1
  // dependent additions, ~4.4 us each against ~8 us for a lone lane's),
  // synchronised per wave; meanwhile one lane of wave 1 forms
  // D' = C + [z]pi and pairing 1's scale factors.  Then D = D' - [y]G.
  Affine<C> g;
  const bool gf = affine_from_canonical<C>(g1_0, g);
  // cooperative scratch: the line area, written only after the prologue
  uint32_t* sc = vw_smem + V::O_LINES;
  uint32_t* dp = vw_smem + V::O_SLOT + 2 * V::E12;  // D' then D (XYZZ), a free slot until the Miller loop
  if (lane < 64) {
    if (lane < 32) {
      const uint32_t d = (in[V::I_Y + (lane >> 2)] >> (8 * (lane & 3))) & 255u;
      Xyzz<C> p = xyzz_inf<C>();
      if (gf && d) p = xyzz_from_affine<C>(affine_load<C>(vtab + ((size_t)lane * 255 + d - 1) * V::AW));
      xyzz_store<C>(prod + lane * 4 * L, p);
    }
    coop_fence();
    const int grp = lane >> 3, j = lane & 7;
    uint32_t* my = sc + grp * COOP_SLOTS * L;
#pragma unroll 1
    for (int h = 16; h >= 1; h >>= 1) {
#pragma unroll 1
      for (int r = grp; r < h; r += 8) {
        const Xyzz<C> R = coop_add<C>(xyzz_load<C>(prod + r * 4 * L), xyzz_load<C>(prod + (r + h) * 4 * L), my, j);
        if (j == 0) xyzz_store<C>(prod + r * 4 * L, R);
      }
      coop_fence();
    }
  } else if (lane == 64) {
    Affine<C> c, pi;
    const bool cf = affine_from_canonical<C>(in + V::I_C, c) && !in[V::I_CINF];
    const bool pf = affine_from_canonical<C>(in + V::I_P, pi) && !in[V::I_PINF];
    Xyzz<C> d = cf ? xyzz_from_affine<C>(c) : xyzz_inf<C>();
    if (pf) {
      int top = -1;
      for (int b = 255; b >= 0 && top < 0; b--)
        if ((in[V::I_Z + (b >> 5)] >> (b & 31)) & 1u) top = b;
      Xyzz<C> zp = xyzz_inf<C>();
      for (int b = top; b >= 0; b--) {
        zp = xyzz_dbl<C>(zp);
        if ((in[V::I_Z + (b >> 5)] >> (b & 31)) & 1u) zp = xyzz_add_affine<C>(zp, pi);
      }
      d = xyzz_add<C>(d, zp);
    }
    xyzz_store<C>(dp, d);
    // pairing 1: (pi, G2[1]) with (y, x, 1)
    vw_st<C>(scale + 3 * L, pi.y);
    vw_st<C>(scale + 4 * L, pi.x);
    vw_st<C>(scale + 5 * L, f29_one<F>());
    flag[1] = (pf && qfin[1]) ? 1u : 0u;
  }
  __syncthreads();
  VW_STAMP(1);
  // ---- D = D' - [y]G (group 0, cooperative), then pairing 0's line factors
  // for (-D, G2[0]): (-Y ZZ, X ZZZ, ZZ ZZZ), one product per lane
  if (lane < 8) {
    const Xyzz<C> R = coop_add<C>(xyzz_load<C>(dp), xyzz_neg<C>(xyzz_load<C>(prod)), sc, lane);
    if (lane == 0) xyzz_store<C>(dp, R);
    coop_fence();
    if (lane < 3) {
      const Xyzz<C> d = xyzz_load<C>(dp);
      const F29<F> x = lane == 0 ? d.Y : lane == 1 ? d.X : d.ZZ;
      const F29<F> y = lane == 0 ? d.ZZ : d.ZZZ;
      const F29<F> v = f29_mul<F>(x, y);
      vw_st<C>(scale + lane * L, lane == 0 ? fp_neg<F>(v) : v);
      if (lane == 0) flag[0] = (!xyzz_is_inf<C>(d) && qfin[0]) ? 1u : 0u;
    }
  }
  __syncthreads();
  VW_STAMP(2);
  vw_pair_tail<C>(vlines, ok + k);
}

// one wave: e(P_0, Q_0) e(-P_1, Q_1) == 1 for canonical affine G1 points
// p = (P_0, P_1) and the line tables of (Q_0, Q_1); the pairing-equation form
// of verify_proof with more than one point (e(pi, [Z(tau)]G2) ==
// e(C - [I(tau)]G1, G2[0]))
template <class C>
__global__ __launch_bounds__(128) void k_pair2_wave(const uint32_t* __restrict__ p, const uint32_t* __restrict__ p_inf,
                                                   const uint32_t* __restrict__ q_inf,
                                                   const uint32_t* __restrict__ vlines,
                                                   const uint32_t* __restrict__ qfin, uint32_t* __restrict__ ok) {
  using F = typename C::Fp29;
  using V = VWave<C>;
  constexpr int N = C::Fp::N, L = V::L;
  uint32_t* scale = vw_smem + V::O_SCALE;
  uint32_t* flag = vw_smem + V::O_FLAG;
  if (threadIdx.x == 0) {
    for (int q = 0; q < 2; q++) {
      Affine<C> a;
      const bool fin = affine_from_canonical<C>(p + q * 2 * N, a) && !(p_inf && p_inf[q]);
      vw_st<C>(scale + (q * 3 + 0) * L, q ? fp_neg<F>(a.y) : a.y);
      vw_st<C>(scale + (q * 3 + 1) * L, a.x);
      vw_st<C>(scale + (q * 3 + 2) * L, f29_one<F>());
      flag[q] = (fin && qfin[q] && !(q_inf && q_inf[q])) ? 1u : 0u;
    }
  }
  __syncthreads();
  vw_pair_tail<C>(vlines, ok);
}

// verify_proof with more than one point in one workgroup of three waves:
// e(P_0, Q_0) e(-P_1, Q_1) == 1 with Q_0 = [Z(tau)]G2 (canonical, variable)
// and Q_1 = G2[0], whose line table the setup built (verify_wave_prepare,
// table 0).  Wave 2 runs Q_0's G2 chain (vl_dbl_wave / vl_add_wave with
// per-wave syncs in its own LDS region), scales each line by P_0's (yP, xP)
// into wave 0's line slots and publishes it (the LDS word READY counts the
// lines out); wave 0 squares and multiplies the lines in as they arrive,
// wave 1 runs Q_1's loop from the table (vw_miller_ws).  So the chain and
// the Miller loop overlap instead of running as two launches (k_vlines_wave,
// then k_pair2_wave).  The producer leaves after its last line (a finished
// wave no longer counts at the workgroup barriers); the two waves then take
// the final exponentiation as k_pair2_wave.  A degenerate chain (T = O or
// T = +-Q, impossible for Q of order r) gives *ok = 2: the caller reruns
// the two-launch path, whose k_vlines_redo recomputes it on one lane.
template <class C>
struct Fused {
  static constexpr int OFF = (VWave<C>::WORDS + 3) & ~3;  // the producer's VLine region
  static constexpr int READY = OFF + VLine<C>::WORDS;  // lines published; READY + 1: wave 0 gave up waiting
  static constexpr int WORDS = READY + 2;
  static_assert(WORDS * 4 <= 160 * 1024, "one workgroup's LDS");
};

template <class C>
__global__ __launch_bounds__(192) void k_pair2_fused(const uint32_t* __restrict__ p, const uint32_t* __restrict__ p_inf,
                                                    const uint32_t* __restrict__ q0,
                                                    const uint32_t* __restrict__ q0_inf,
                                                    const uint32_t* __restrict__ tab_lines,
                                                    const uint32_t* __restrict__ tab_qfin, uint32_t* __restrict__ ok) {
  using P = typename PairOf<C>::T;
  using F = typename C::Fp29;
  using V = VWave<C>;
  using S = VLine<C>;
  constexpr int N = C::Fp::N, L = V::L, E2 = V::E2, OFF = Fused<C>::OFF, READY = Fused<C>::READY;
  uint32_t* scale = vw_smem + V::O_SCALE;
  uint32_t* flag = vw_smem + V::O_FLAG;
  uint32_t* lines = vw_smem + V::O_LINES;
  const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)), lane = (int)(threadIdx.x & 63);
  if (threadIdx.x == 0) {
    for (int q = 0; q < 2; q++) {
      Affine<C> a;
      const bool fin = affine_from_canonical<C>(p + q * 2 * N, a) && !(p_inf && p_inf[q]);
      vw_st<C>(scale + (q * 3 + 0) * L, q ? fp_neg<F>(a.y) : a.y);
      vw_st<C>(scale + (q * 3 + 1) * L, a.x);
      vw_st<C>(scale + (q * 3 + 2) * L, f29_one<F>());
      flag[q] = fin ? 1u : 0u;
    }
    flag[1] = flag[1] && tab_qfin[0];
    vw_smem[READY] = 0u;
    vw_smem[READY + 1] = 0u;
  }
  if (threadIdx.x == 128) {
    G2A<C> Q;
    const bool fin = g2_from_canon<C>(q0, Q) && !(q0_inf && *q0_inf);
    vw_smem[OFF + S::FLAG] = fin ? 0u : 2u;
    vw_st2<C>(vl_slot<C, OFF>(S::X), Q.x);
    vw_st2<C>(vl_slot<C, OFF>(S::Y), Q.y);
    vw_st2<C>(vl_slot<C, OFF>(S::Z), f2_one<C>());
    vw_st2<C>(vl_slot<C, OFF>(S::QX), Q.x);
    vw_st2<C>(vl_slot<C, OFF>(S::QY), Q.y);
    if (P::D_TWIST) {
      const G2A<C> q1 = twist_frob<C>(Q);
      G2A<C> q2 = twist_frob<C>(q1);
      q2.y = f2_neg<C>(q2.y);
      vw_st2<C>(vl_slot<C, OFF>(S::Q1X), q1.x);
      vw_st2<C>(vl_slot<C, OFF>(S::Q1Y), q1.y);
      vw_st2<C>(vl_slot<C, OFF>(S::Q2X), q2.x);
      vw_st2<C>(vl_slot<C, OFF>(S::Q2Y), q2.y);
    }
  }
  __syncthreads();
  const bool use0 = flag[0] != 0 && vw_smem[OFF + S::FLAG] == 0u, use1 = flag[1] != 0;
  if (w == 2) {  // the producer: Q_0's lines, scaled, one at a time
    if (!use0) return;
    int s = 0;
    auto publish = [&]() {
      uint32_t* out = lines + s * V::LW;
      if (lane < 2) vw_st2<C>(out + lane * E2, f2_mul_fp<C>(vw_ld2<C>(out + lane * E2), vw_ld<C>(scale + lane * L)));
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      s++;
      if (lane == 0) *(volatile uint32_t*)(vw_smem + READY) = (uint32_t)s;
    };
#pragma unroll 1
    for (int i = P::LOOP_BITS - 2; i >= 0; i--) {
      vl_dbl_wave<C, OFF, true>(lines + s * V::LW);
      publish();
      if ((P::LOOP[i >> 6] >> (i & 63)) & 1ull) {
        vl_add_wave<C, OFF, true>(S::QX, S::QY, lines + s * V::LW);
        publish();
      }
    }
    if (P::LOOP_NEG && lane < 2) {
      uint32_t* y = vl_slot<C, OFF>(S::Y) + lane * S::L;
      vw_st<C>(y, fp_neg<F>(vw_ld<C>(y)));
    }
    vw_sync<true>();
    if (P::D_TWIST) {
      vl_add_wave<C, OFF, true>(S::Q1X, S::Q1Y, lines + s * V::LW);
      publish();
      vl_add_wave<C, OFF, true>(S::Q2X, S::Q2Y, lines + s * V::LW);
      publish();
    }
    return;
  }
  // wave 1: Q_1's table lines scaled by -P_1; wave 0 (Q_0 unused): zeros
  if (w == 1) {
    for (int t = lane; t < V::NL * 3; t += 64) {
      const int c = t % 3;
      vw_st2<C>(lines + (V::NL * 3 + t) * E2,
                use1 ? f2_mul_fp<C>(vw_ld2<C>(tab_lines + (size_t)t * E2), vw_ld<C>(scale + (3 + c) * L))
                     : f2_zero<C>());
    }
  } else if (!use0) {
    for (int t = lane; t < V::NL * 3; t += 64) vw_st2<C>(lines + t * E2, f2_zero<C>());
  }
  constexpr uint32_t f = V::O_SLOT, pr = V::O_PROD;
  if (lane < 12) vw_st<C>(vw_smem + f + w * V::E12 + lane * L, lane == 0 ? f29_one<F>() : f29_zero<F>());
  vw_sync<true>();
  vw_miller_ws<C>(f, (use0 ? 1 : 0) | (use1 ? 2 : 0), pr, READY, use0);
  vw_final_exp<C>(V::O_SLOT, pr);
  if (threadIdx.x < 12) {
    const F29<F> v = f29_reduce<F>(vw_ld<C>(vw_smem + f + threadIdx.x * L));
    const F29<F> want = threadIdx.x == 0 ? f29_reduce<F>(f29_one<F>()) : f29_zero<F>();
    uint32_t diff = 0;
    for (int i = 0; i < L; i++) diff |= v.v[i] ^ want.v[i];
    flag[2 + threadIdx.x] = diff;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t bad = 0;
    for (int i = 0; i < 12; i++) bad |= flag[2 + i];
    *ok = (vw_smem[OFF + S::FLAG] == 1u || vw_smem[READY + 1] != 0u) ? 2u : (bad == 0 ? 1u : 0u);
  }
}

// Debug / measurement (kzgx_debug_vw_bench, not in kzg_gpu.h): the latency
// of one wave-wide Fp12 op, iterated `iters` times on arbitrary values < m
// in LDS: 0 cyclotomic squaring, 1 dense product, 2 squaring, 3 line
// product, 4 Frobenius, 5 one-lane inverse, 6 wave inverse.  out[0] = wall-clock ticks
// (100 MHz), out[1] = core clocks (s_memtime).
template <class C>
__global__ __launch_bounds__(64) void k_vw_bench(int op, uint32_t iters, uint64_t* __restrict__ out) {
  using V = VWave<C>;
  constexpr int L = V::L;
  const uint32_t lane = threadIdx.x;
  constexpr uint32_t s0 = V::O_SLOT, s1 = V::O_SLOT + V::E12;
  // arbitrary values below m: pseudo-random low limbs, a small top limb
  for (uint32_t w = lane; w < (uint32_t)V::O_PROD; w += 64) {
    const uint32_t h = (w + 1) * 2654435761u;
    vw_smem[w] = (w % L == L - 1) ? (h >> 24) : (h >> 3);
  }
  __syncthreads();
  const uint64_t w0 = wall_clock64(), c0 = clock64();
#pragma unroll 1
  for (uint32_t it = 0; it < iters; it++) {
    switch (op) {
      case 0: vw_cyclo_sqr<C>(s0, s0, V::O_PROD); break;
      case 1: vw_mul<C>(s0, s0, s1, V::O_PROD); break;
      case 2: vw_sqr<C>(s0, s0, V::O_PROD, lane); break;
      case 3: vw_mul_line<C>(s0, V::O_LINES, V::O_PROD, lane); break;
      case 4: vw_frob<C>(s0, s0, V::O_PROD); break;
      case 5: vw_inv<C>(s1, s0); break;
      case 6: vw_inv_wave<C>(s1, s0, s1 + V::E12, s1 + 2 * V::E12, V::O_PROD); break;
      case 7: vw_cyclo_sqr<C, true, 1>(s0, s0, V::O_PROD); break;  // product round, per-wave sync
      case 8: vw_cyclo_sqr<C, true, 2>(s0, s0, V::O_PROD); break;  // fold round, per-wave sync
      default: vw_cyclo_sqr<C, true, 3>(s0, s0, V::O_PROD); break;  // 9: the op, per-wave sync
    }
  }
  const uint64_t w1 = wall_clock64(), c1 = clock64();
  if (lane == 0) {
    out[0] = w1 - w0;
    out[1] = c1 - c0;
  }
}

int vw_bench(int curve, int op, uint32_t iters, double* ns_per_op, double* clk_per_op, hipStream_t st) {
  uint64_t* d = nullptr;
  KZGX_TRY_HIP(hipMalloc((void**)&d, 16));
  if (curve == KZGX_CURVE_BN254)
    hipLaunchKernelGGL(k_vw_bench<BN254G1>, dim3(1), dim3(64), VWave<BN254G1>::WORDS * 4, st, op, iters, d);
  else
    hipLaunchKernelGGL(k_vw_bench<BLS12381G1>, dim3(1), dim3(64), VWave<BLS12381G1>::WORDS * 4, st, op, iters, d);
  uint64_t h[2] = {0, 0};
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) e = hipMemcpyAsync(h, d, 16, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  (void)hipFree(d);
  if (e != hipSuccess) return hip_fail(e);
  *ns_per_op = 10.0 * (double)h[0] / iters;
  *clk_per_op = (double)h[1] / iters;
  return KZGX_OK;
}

// wave path: [y]G table | line tables | Q flags, in one device buffer
template <class C>
static constexpr size_t vw_tab_words() {
  return (size_t)VWave<C>::TAB * VWave<C>::AW;
}
template <class C>
static constexpr size_t vw_buf_words() {
  return vw_tab_words<C>() + (size_t)2 * VWave<C>::NL * VWave<C>::LW + 4;
}

size_t verify_wave_bytes(int curve) {
  return 4 * (curve == KZGX_CURVE_BN254 ? vw_buf_words<BN254G1>() : vw_buf_words<BLS12381G1>());
}

// at setup (both SRS halves present): the [y]G table (a copy of the
// generator's comb when G1[0] is the generator) and the line tables of
// G2[0], G2[1] from the wave-parallel G2 chain (k_vlines_wave; a degenerate
// chain is recomputed on one lane)
template <class C>
static int verify_wave_prepare_impl(const uint32_t* d_g1_0, const uint32_t* d_g2_01, const uint32_t* g1_comb,
                                    uint32_t* d_buf, hipStream_t st) {
  uint32_t* lines = d_buf + vw_tab_words<C>();
  uint32_t* qfin = lines + (size_t)2 * VWave<C>::NL * VWave<C>::LW;
  if (g1_comb) {
    KZGX_TRY(vtab_prepare(C::ID == 0 ? KZGX_CURVE_BN254 : KZGX_CURVE_BLS12381, d_g1_0, g1_comb, d_buf, st));
  } else {
    hipLaunchKernelGGL(k_vtab<C>, dim3((VWave<C>::TAB + 63) / 64), dim3(64), 0, st, d_g1_0, d_buf);
  }
  hipLaunchKernelGGL(k_vlines_wave<C>, dim3(2), dim3(64), VLine<C>::WORDS * 4, st, d_g2_01, lines, qfin, qfin + 2);
  hipLaunchKernelGGL(k_vlines_redo<C>, dim3(1), dim3(64), 0, st, d_g2_01, lines, qfin + 2);
  KZGX_TRY_HIP(hipGetLastError());
  return KZGX_OK;
}

int verify_wave_prepare(Ctx* ctx, const uint32_t* d_g1_0, const uint32_t* d_g2_01, const uint32_t* g1_comb,
                        uint32_t* d_buf, hipStream_t st) {
  ProfScope p(ctx, st, "verify_wave_prepare");
  return ctx->curve == KZGX_CURVE_BN254 ? verify_wave_prepare_impl<BN254G1>(d_g1_0, d_g2_01, g1_comb, d_buf, st)
                                        : verify_wave_prepare_impl<BLS12381G1>(d_g1_0, d_g2_01, g1_comb, d_buf, st);
}

template <class C>
static int verify_wave_impl(const uint32_t* d_commits, const uint32_t* d_commit_inf, const uint32_t* d_proofs,
                            const uint32_t* d_proof_inf, const uint32_t* d_z, const uint32_t* d_y, size_t count,
                            const uint32_t* d_g1_0, const uint32_t* d_buf, uint32_t* d_ok, hipStream_t st) {
  const uint32_t* lines = d_buf + vw_tab_words<C>();
  const uint32_t* qfin = lines + (size_t)2 * VWave<C>::NL * VWave<C>::LW;
  hipLaunchKernelGGL(k_verify_wave<C>, dim3((unsigned)count), dim3(128), VWave<C>::WORDS * 4, st, d_commits, d_commit_inf, d_proofs,
                     d_proof_inf, d_z, d_y, (uint32_t)count, d_g1_0, d_buf, lines, qfin, d_ok);
  KZGX_TRY_HIP(hipGetLastError());
  return KZGX_OK;
}

int verify_wave_batch(Ctx* ctx, const uint32_t* d_commits, const uint32_t* d_commit_inf, const uint32_t* d_proofs,
                      const uint32_t* d_proof_inf, const uint32_t* d_z, const uint32_t* d_y, size_t count,
                      const uint32_t* d_g1_0, const uint32_t* d_buf, uint32_t* d_ok, hipStream_t st) {
  if (count == 0) return KZGX_OK;
  ProfScope p(ctx, st, "verify_wave");
  return ctx->curve == KZGX_CURVE_BN254
             ? verify_wave_impl<BN254G1>(d_commits, d_commit_inf, d_proofs, d_proof_inf, d_z, d_y, count, d_g1_0,
                                         d_buf, d_ok, st)
             : verify_wave_impl<BLS12381G1>(d_commits, d_commit_inf, d_proofs, d_proof_inf, d_z, d_y, count, d_g1_0,
                                            d_buf, d_ok, st);
}

template <class C>
static int pair2_wave_impl(const uint32_t* d_p, const uint32_t* d_p_inf, const uint32_t* d_q, const uint32_t* d_q_inf,
                           uint32_t* d_lines, uint32_t* d_ok, hipStream_t st) {
  uint32_t* qfin = d_lines + (size_t)2 * VWave<C>::NL * VWave<C>::LW;
  hipLaunchKernelGGL(k_vlines_wave<C>, dim3(2), dim3(64), VLine<C>::WORDS * 4, st, d_q, d_lines, qfin, qfin + 2);
  hipLaunchKernelGGL(k_vlines_redo<C>, dim3(1), dim3(64), 0, st, d_q, d_lines, qfin + 2);
  hipLaunchKernelGGL(k_pair2_wave<C>, dim3(1), dim3(128), VWave<C>::WORDS * 4, st, d_p, d_p_inf, d_q_inf, d_lines,
                     qfin, d_ok);
  KZGX_TRY_HIP(hipGetLastError());
  return KZGX_OK;
}

template <class C>
static int pair2_fused_impl(const uint32_t* d_p, const uint32_t* d_p_inf, const uint32_t* d_q, const uint32_t* d_q_inf,
                            const uint32_t* d_buf, uint32_t* d_ok, hipStream_t st) {
  const uint32_t* lines = d_buf + vw_tab_words<C>();
  const uint32_t* qfin = lines + (size_t)2 * VWave<C>::NL * VWave<C>::LW;
  hipLaunchKernelGGL(k_pair2_fused<C>, dim3(1), dim3(192), Fused<C>::WORDS * 4, st, d_p, d_p_inf, d_q, d_q_inf, lines,
                     qfin, d_ok);
  KZGX_TRY_HIP(hipGetLastError());
  return KZGX_OK;
}

int pair2_fused(Ctx* ctx, const uint32_t* d_p, const uint32_t* d_p_inf, const uint32_t* d_q, const uint32_t* d_q_inf,
                const uint32_t* d_vw, uint32_t* d_ok, hipStream_t st) {
  ProfScope p(ctx, st, "pair2_fused");
  return ctx->curve == KZGX_CURVE_BN254 ? pair2_fused_impl<BN254G1>(d_p, d_p_inf, d_q, d_q_inf, d_vw, d_ok, st)
                                        : pair2_fused_impl<BLS12381G1>(d_p, d_p_inf, d_q, d_q_inf, d_vw, d_ok, st);
}

size_t pair2_wave_scratch_bytes(int curve) {
  return 4 * (curve == KZGX_CURVE_BN254 ? (size_t)2 * VWave<BN254G1>::NL * VWave<BN254G1>::LW + 4
                                        : (size_t)2 * VWave<BLS12381G1>::NL * VWave<BLS12381G1>::LW + 4);
}

int pair2_wave(Ctx* ctx, const uint32_t* d_p, const uint32_t* d_p_inf, const uint32_t* d_q, const uint32_t* d_q_inf,
               uint32_t* d_scratch, uint32_t* d_ok, hipStream_t st) {
  ProfScope p(ctx, st, "pair2_wave");
  return ctx->curve == KZGX_CURVE_BN254 ? pair2_wave_impl<BN254G1>(d_p, d_p_inf, d_q, d_q_inf, d_scratch, d_ok, st)
                                        : pair2_wave_impl<BLS12381G1>(d_p, d_p_inf, d_q, d_q_inf, d_scratch, d_ok, st);
}

}  // namespace kzgx

namespace kzgx {
// device bring-up (kzgx_setup.hpp): one launch loads this code object
__global__ void k_warm_verify_wave() {}
int warm_verify_wave(hipStream_t st) {
  hipLaunchKernelGGL(k_warm_verify_wave, dim3(1), dim3(64), 0, st);
  KZGX_TRY_HIP(hipGetLastError());
  return KZGX_OK;
}
}  // namespace kzgx
