// Device side of the fixed-base G1 MSM (msm_fixed.hip): the packed table
// entry layout, signed-digit recoding and the batched accumulation kernel
// k_fixed_accum.  A header so scripts/micro_madd.hip can time the very
// kernel the bench runs, with either mixed-addition variant.
#pragma once
#include <hip/hip_runtime.h>

#include "curve.hpp"

namespace kzgx {

// Table point layout, per curve (KZGX_FIXED_L29 = 0 / 1 forces one for both):
//  * packed: x || y as canonical-width 32-bit words, 64 B (BN254) / 96 B
//    (BLS12-381), unpacked to radix-2^29 limbs per term;
//  * radix-2^29: the limbs the accumulation consumes, padded to 80 B / 112 B.
// Measured on MI355X (profiles/r02_pmc_fetch_calibration.json): every DRAM
// read is a 128-B request; an 80-B BN254 entry costs 1.5 lines and a 64-B
// one exactly one, so packed moves 33% fewer bytes (8.7 vs 13.0 GB per
// 1024-MSM launch), needs 20% less HBM and is 1% faster -- and lets c = 17
// (15 windows) fit.  BLS12-381 keeps the radix-2^29 entries: its 14-limb
// unpack does not hide, 112-B entries are 2% faster than 96-B ones
// (profiles/r02_ab_table_layout.json).
template <class C>
constexpr bool fixed_l29() {
#ifdef KZGX_FIXED_L29
  return KZGX_FIXED_L29 != 0;
#else
  return C::Fp29::L > 9;
#endif
}
template <class C>
constexpr int packed_words() {
  return fixed_l29<C>() ? affine_words<C>() : 2 * C::Fp::N;
}

// Where entry (i, w, j) of the table lives: word (i is + w ws + j PW).
//  * window-major M[w][i][j] (is = H PW, ws = n_t H PW): a wavefront's lanes
//    (consecutive points, one window) read within one window slice;
//  * point-major M[i][w][j] (is = W H PW, ws = H PW): the W windows of a point
//    are adjacent, so one thread's consecutive terms (k_fixed_accum_flat walks
//    a point's windows in order) stay within W H PW words -- 148 KB at c = 7
//    -- instead of jumping a whole window slice (4.3 GB at cfg5) per term.
struct TabStrides {
  size_t is, ws;  // words
};

template <class C, int CB>
struct FixedWin {
  // regular odd digits (below) of a scalar k < r < 2^SCALAR_BITS need
  // W c >= SCALAR_BITS: the top digit 2 (u >> c (W - 1)) + 1, u = k >> 1 <
  // 2^(SCALAR_BITS - 1), then indexes one of the H table entries
  static constexpr int W = (C::SCALAR_BITS + CB - 1) / CB;
  static constexpr uint32_t H = 1u << (CB - 1);
};

template <class C>
KZGX_DEV Affine<C> packed_load(const uint32_t* __restrict__ p) {
  if (fixed_l29<C>()) return affine_load<C>(p);
  using F = typename C::Fp29;
  constexpr int N = C::Fp::N;
  uint32_t wx[N], wy[N];
#pragma unroll
  for (int k = 0; k < N / 4; k++) {
    uint4 a = reinterpret_cast<const uint4*>(p)[k];
    uint4 b = reinterpret_cast<const uint4*>(p + N)[k];
    wx[4 * k] = a.x; wx[4 * k + 1] = a.y; wx[4 * k + 2] = a.z; wx[4 * k + 3] = a.w;
    wy[4 * k] = b.x; wy[4 * k + 1] = b.y; wy[4 * k + 2] = b.z; wy[4 * k + 3] = b.w;
  }
  Affine<C> r;
  r.x = f29_from_words<F, N>(wx);
  r.y = f29_from_words<F, N>(wy);
  return r;
}

template <class C>
KZGX_DEV void packed_store(uint32_t* __restrict__ p, const Affine<C>& a) {
  if (fixed_l29<C>()) {
    affine_store<C>(p, a);
    return;
  }
  using F = typename C::Fp29;
  constexpr int N = C::Fp::N;
  uint32_t wx[N], wy[N];
  f29_to_words<F, N>(a.x, wx);
  f29_to_words<F, N>(a.y, wy);
#pragma unroll
  for (int k = 0; k < N / 4; k++) {
    reinterpret_cast<uint4*>(p)[k] = make_uint4(wx[4 * k], wx[4 * k + 1], wx[4 * k + 2], wx[4 * k + 3]);
    reinterpret_cast<uint4*>(p + N)[k] = make_uint4(wy[4 * k], wy[4 * k + 1], wy[4 * k + 2], wy[4 * k + 3]);
  }
}

// s mod r for any 256-bit s (the ABI asks for canonical scalars; this keeps a
// non-canonical one exact for points of order r instead of overflowing the
// top digit).  Common case: one compare of the top word.
template <class C>
KZGX_DEV void scalar_reduce(uint32_t (&s)[8]) {
  using R = typename C::Fr;
  while (s[7] >= R::P[7]) {
    uint32_t d[8];
    int64_t br = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) {
      int64_t v = (int64_t)s[k] - (int64_t)R::P[k] + br;
      d[k] = (uint32_t)v;
      br = v >> 32;
    }
    if (br < 0) break;  // s < r
#pragma unroll
    for (int k = 0; k < 8; k++) s[k] = d[k];
  }
}

// --------------------------------------------------------------------------
// MSM
// --------------------------------------------------------------------------
// shift the 256-bit scalar right by CB (static register indexing only)
template <int CB>
KZGX_DEV void shr_scalar(uint32_t (&s)[8]) {
#pragma unroll
  for (int k = 0; k < 7; k++) s[k] = __builtin_amdgcn_alignbit(s[k + 1], s[k], CB);
  s[7] >>= CB;
}

// Regular odd signed digits (Joye-Tunstall "regular recoding").  For an odd
// k with u = k >> 1:
//   d_w = 2 ((u >> c w) mod 2^c) + 1 - 2^c   (w < W - 1),
//   d_{W-1} = 2 (u >> c (W - 1)) + 1,
// sum_w d_w 2^(c w) = k, and every digit is odd: never zero.  The table then
// holds the odd multiples M[w][i][j] = (2 j + 1) 2^(c w) P_i, j = (|d| - 1) / 2
// < H, and every term is one mixed addition -- no zero-digit branch, whose
// accumulator merge cost ~36 register copies per term.  An even k is
// replaced by r - k (odd; r is odd) with every digit negated:
// (r - k) P = -k P for P of order r.  k = 0 becomes r: its terms sum to O
// through exact additions.  Digit w reads bits [c w, c w + c) of u alone
// (no carry), so a thread may start at any window.
//
// odd_prepare: canonical s (scalar_reduce first) -> u = k' >> 1 in s, and the
// sign flip (1 when k was even)
template <class C>
KZGX_DEV uint32_t odd_prepare(uint32_t (&s)[8]) {
  using R = typename C::Fr;
  const uint32_t flip = (s[0] & 1u) ^ 1u;
  // s = flip ? r - s : s, branch-free (r - s >= 0 for canonical s)
  const uint32_t m = 0u - flip;
  int64_t br = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const int64_t v = (int64_t)(R::P[k] & m) - (int64_t)(s[k] & m) + (int64_t)(s[k] & ~m) + br;
    s[k] = (uint32_t)v;
    br = v >> 32;
  }
  shr_scalar<1>(s);
  return flip;
}

// table entry index j and sign of the digit whose window bits are the low CB
// bits of s (top: the remaining bits, top digit of the scalar)
template <int CB>
KZGX_DEV void odd_digit(uint32_t s0, bool top, uint32_t flip, uint32_t& j, uint32_t& neg) {
  constexpr uint32_t H = 1u << (CB - 1);
  const uint32_t m = s0 & ((1u << CB) - 1u);
  const uint32_t hi = m >> (CB - 1);  // 1: d > 0
  j = top ? s0 : ((m ^ (hi - 1u)) & (H - 1u));
  neg = (top ? 0u : hi ^ 1u) ^ flip;
}

// thread t of MSM b sums the W digit terms of points i = t, t + T, t + 2T, ...
// (a wavefront reads 64 consecutive scalars per point step)
template <class C>
struct PackedPt {
  uint4 q[packed_words<C>() / 4];
};

template <class C>
KZGX_DEV PackedPt<C> packed_fetch(const uint32_t* __restrict__ p) {
  PackedPt<C> r;
#pragma unroll
  for (int k = 0; k < packed_words<C>() / 4; k++) r.q[k] = reinterpret_cast<const uint4*>(p)[k];
  return r;
}

template <class C>
KZGX_DEV Affine<C> packed_unpack(const PackedPt<C>& r) {
  using F = typename C::Fp29;
  Affine<C> a;
  if (fixed_l29<C>()) {
    constexpr int L = F::L;
    uint32_t w[packed_words<C>()];
#pragma unroll
    for (int k = 0; k < packed_words<C>() / 4; k++) {
      w[4 * k] = r.q[k].x; w[4 * k + 1] = r.q[k].y; w[4 * k + 2] = r.q[k].z; w[4 * k + 3] = r.q[k].w;
    }
#pragma unroll
    for (int i = 0; i < L; i++) {
      a.x.v[i] = w[i];
      a.y.v[i] = w[L + i];
    }
    return a;
  }
  constexpr int N = C::Fp::N;
  uint32_t wx[N], wy[N];
#pragma unroll
  for (int k = 0; k < N / 4; k++) {
    const uint4 p = r.q[k], q = r.q[N / 4 + k];
    wx[4 * k] = p.x; wx[4 * k + 1] = p.y; wx[4 * k + 2] = p.z; wx[4 * k + 3] = p.w;
    wy[4 * k] = q.x; wy[4 * k + 1] = q.y; wy[4 * k + 2] = q.z; wy[4 * k + 3] = q.w;
  }
  a.x = f29_from_words<F, N>(wx);
  a.y = f29_from_words<F, N>(wy);
  return a;
}

// waves per SIMD the accumulation kernel is register-budgeted for
#ifndef KZGX_FIXED_WAVES_BN
#define KZGX_FIXED_WAVES_BN 3
#endif
#ifndef KZGX_FIXED_WAVES_BLS
#define KZGX_FIXED_WAVES_BLS 2
#endif
template <class C>
constexpr int fixed_accum_waves() {
  return C::Fp29::L <= 9 ? KZGX_FIXED_WAVES_BN : KZGX_FIXED_WAVES_BLS;
}

KZGX_DEV void scalar_load(const uint32_t* __restrict__ src, uint32_t (&s)[8]) {
  const uint4 lo = reinterpret_cast<const uint4*>(src)[0];
  const uint4 hi = reinterpret_cast<const uint4*>(src)[1];
  s[0] = lo.x; s[1] = lo.y; s[2] = lo.z; s[3] = lo.w;
  s[4] = hi.x; s[5] = hi.y; s[6] = hi.z; s[7] = hi.w;
}

// y or 2m - y (a negative digit: -(x, y) = (x, 2m - y), f29_neg_lazy), as
// per-limb selects: no branch, so no register merge after it
template <class C>
KZGX_DEV void affine_cond_neg(Affine<C>& a, uint32_t neg) {
  using F = typename C::Fp29;
#pragma unroll
  for (int i = 0; i < F::L; i++) a.y.v[i] = neg ? F::P2B[i] - a.y.v[i] : a.y.v[i];
}

// Batched fixed-base accumulation.  Thread t of MSM b sums the W odd-digit
// terms (odd_digit) of points i = t, t + T, t + 2T, ... into one XYZZ
// accumulator with mixed additions (variant V, curve.hpp); a wavefront reads
// 64 consecutive scalars per point step.  Every term is one addition (odd
// digits are never zero), and the control flow is uniform across the
// wavefront: the first n / T points of every lane run as one loop whose trip
// count and window index live in scalar registers (the point change is a
// uniform branch), and the lanes with one more point run it afterwards.  The
// loop body is then straight-line code around the addition, so the
// accumulator and the in-flight table entry stay in their loop registers
// (the divergent zero-digit branch and per-lane trip counts of round 3 cost
// ~135 register copies per term).  The table lookup of the next term is in
// flight during each addition; the next point's scalar is loaded a whole
// point ahead.
//
// inf (null when no SRS point of the prefix is infinite): an infinite point
// P_i contributes O whatever its scalar, so its terms are replaced by those
// of scalar 0 on the finite point fin0 -- odd digits of r, which sum to
// r P_fin0 = O through exact additions.  Selects at the point change, no
// branch in the loop.
template <class C, int CB, int V = madd_variant<C>()>
__global__ __launch_bounds__(64, fixed_accum_waves<C>()) void k_fixed_accum(
    const uint32_t* __restrict__ scalars, uint32_t n, size_t stride_words, const uint32_t* __restrict__ tab,
    TabStrides ts, const uint8_t* __restrict__ inf, uint32_t fin0, uint32_t T, uint32_t* __restrict__ part) {
  constexpr int XW = xyzz_words<C>();
  constexpr int PW = packed_words<C>();
  constexpr int W = FixedWin<C, CB>::W;
  const uint32_t b = blockIdx.y;
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= T) return;  // T is a multiple of 64: whole wavefronts
  Xyzz<C> acc = xyzz_inf<C>();
  const uint32_t nmin = n / T;                                  // points of every lane
  const bool extra = t < n - nmin * T;                          // one more point
  if (nmin > 0 || extra) {
    const uint32_t* sc = scalars + (size_t)b * stride_words;
    const uint32_t last = n - 1;
    uint32_t i = t;
    uint32_t s[8], sn[8];
    // point i's table row and its scalar in s: u and the sign flip (an
    // infinite point becomes scalar 0 on point fin0)
    const uint32_t* prow;
    uint32_t flip;
    auto point = [&](uint32_t ii) __attribute__((always_inline)) {
      if (inf != nullptr) {  // uniform
        const bool z = inf[ii] != 0;
#pragma unroll
        for (int k = 0; k < 8; k++) s[k] = z ? 0u : s[k];
        ii = z ? fin0 : ii;
      }
      scalar_reduce<C>(s);
      flip = odd_prepare<C>(s);
      prow = tab + (size_t)ii * ts.is;
    };
    scalar_load(sc + (size_t)(i < last ? i : last) * 8, s);
    point(i < last ? i : last);
    {
      const uint32_t i2 = i + T < last ? i + T : last;
      scalar_load(sc + (size_t)i2 * 8, sn);
    }
    // entry (w, j) of term (i, w) from the low bits of s (s consumed by CB
    // bits); w is uniform
    auto fetch = [&](int w, uint32_t& neg) __attribute__((always_inline)) {
      uint32_t j;
      odd_digit<CB>(s[0], w == W - 1, flip, j, neg);
      shr_scalar<CB>(s);
      return packed_fetch<C>(prow + (size_t)w * ts.ws + (size_t)j * PW);
    };
    uint32_t nq;
    PackedPt<C> pq = fetch(0, nq);
    int w = 0;
    // one term: add the queued entry, queue the next term's lookup
    auto step = [&]() __attribute__((always_inline)) {
      Affine<C> cur = packed_unpack<C>(pq);
      const uint32_t neg = nq;
      if (w == W - 1) {  // uniform: the next term is window 0 of the next point
        KZGX_MARK("KZGX_PER_POINT");
        w = 0;
        i += T;
#pragma unroll
        for (int k = 0; k < 8; k++) s[k] = sn[k];
        point(i < last ? i : last);
        const uint32_t i2 = i + T < last ? i + T : last;
        scalar_load(sc + (size_t)i2 * 8, sn);
      } else {
        w++;
      }
      pq = fetch(w, nq);
      affine_cond_neg<C>(cur, neg);
      acc = xyzz_add_affine_v<C, V>(acc, cur);
    };
    const uint32_t E = nmin * (uint32_t)W;
#pragma unroll 1
    for (uint32_t e = 0; e < E; e++) step();
    if (extra) {
#pragma unroll 1
      for (int e = 0; e < W; e++) step();
    }
  }
  xyzz_store<C>(part + ((size_t)b * T + t) * XW, acc);
}

}  // namespace kzgx
