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
  // signed digits of a scalar < r need W c >= bits(r) + 1: the top digit
  // then absorbs the final carry without overflowing H
  static constexpr int W = (C::SCALAR_BITS + 1 + CB - 1) / CB;
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

// next signed digit from the low CB bits of s (consumed), carry in/out
template <int CB>
KZGX_DEV int next_digit(uint32_t (&s)[8], uint32_t& carry) {
  uint32_t raw = (s[0] & ((1u << CB) - 1u)) + carry;
  shr_scalar<CB>(s);
  carry = raw > (1u << (CB - 1)) ? 1u : 0u;
  return (int)raw - (int)(carry << CB);
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

typedef __attribute__((address_space(1))) const void* kzgx_gptr_t;
typedef __attribute__((address_space(3))) void* kzgx_lptr_t;

KZGX_DEV void scalar_load(const uint32_t* __restrict__ src, uint32_t (&s)[8]) {
  const uint4 lo = reinterpret_cast<const uint4*>(src)[0];
  const uint4 hi = reinterpret_cast<const uint4*>(src)[1];
  s[0] = lo.x; s[1] = lo.y; s[2] = lo.z; s[3] = lo.w;
  s[4] = hi.x; s[5] = hi.y; s[6] = hi.z; s[7] = hi.w;
}

// The digit terms of one accumulation thread, in order: points i = t,
// t + T, t + 2T, ... (a wavefront reads 64 consecutive scalars per point
// step), windows w = 0 .. W - 1 of each.  next() recodes the next signed
// digit (0: no addition; every term of an infinite SRS point is 0) and
// returns its table entry.  inf may be null: no SRS point is infinite (the
// table build checks), and no flag is read.
template <class C, int CB>
struct FixedTerms {
  static constexpr int PW = packed_words<C>();
  static constexpr int W = FixedWin<C, CB>::W;
  static constexpr uint32_t H = FixedWin<C, CB>::H;
  const uint32_t* sc;
  const uint8_t* inf;
  const uint32_t* tab;
  TabStrides ts;
  uint32_t i, T;
  int w;
  uint32_t s[8], carry;
  bool skip;

  KZGX_DEV void load() {
    scalar_load(sc + (size_t)i * 8, s);
    scalar_reduce<C>(s);
    carry = 0;
    skip = inf != nullptr && inf[i] != 0;
    w = 0;
  }
  // only while terms remain
  KZGX_DEV const uint32_t* next(int& d) {
    if (w == W) {
      i += T;
      load();
    }
    const int dd = next_digit<CB>(s, carry);
    d = skip ? 0 : dd;
    const uint32_t* p = tab + (size_t)i * ts.is + (size_t)w * ts.ws + (size_t)((d < 0 ? -d : d) - (d != 0)) * PW;
    w++;
    return p;
  }
};

#ifndef KZGX_FIXED_PF
#define KZGX_FIXED_PF 1
#endif

// thread t of MSM b sums its terms (FixedTerms) into one XYZZ accumulator
// with mixed additions (variant V, curve.hpp).  Software pipeline: the
// table lookups of the next PF terms are in flight during each addition.
template <class C, int CB, int V = madd_variant<C>(), int PF = KZGX_FIXED_PF>
__global__ __launch_bounds__(64, fixed_accum_waves<C>()) void k_fixed_accum(
    const uint32_t* __restrict__ scalars, uint32_t n, size_t stride_words, const uint32_t* __restrict__ tab,
    TabStrides ts, const uint8_t* __restrict__ inf, uint32_t T, uint32_t* __restrict__ part) {
  constexpr int XW = xyzz_words<C>();
  using G = FixedTerms<C, CB>;
  const uint32_t b = blockIdx.y;
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= T) return;
  Xyzz<C> acc = xyzz_inf<C>();
  const uint32_t npts = t < n ? (n - 1 - t) / T + 1 : 0;
  const int E = (int)npts * G::W;
  if constexpr (PF == 0) {
    // LDS ring: the next term's entry goes global -> LDS directly
    // (global_load_lds_dwordx4, per-lane source, lane-linear destination),
    // so no VGPR holds an in-flight entry; the current one is read back
    // with ds_read_b128 at the top of each addition
    constexpr int NCH = G::PW / 4;
    __shared__ uint4 ring[2][NCH][64];
    const uint32_t lane = threadIdx.x & 63;
    if (E > 0) {
      G g;
      g.sc = scalars + (size_t)b * stride_words;
      g.inf = inf;
      g.tab = tab;
      g.ts = ts;
      g.i = t;
      g.T = T;
      g.load();
      auto issue = [&](int slot, const uint32_t* src) {
#pragma unroll
        for (int k = 0; k < NCH; k++)
          __builtin_amdgcn_global_load_lds((kzgx_gptr_t)(src + 4 * k), (kzgx_lptr_t)&ring[slot][k][0], 16, 0, 0);
      };
      int dn = 0;
      issue(0, g.next(dn));
#pragma unroll 1
      for (int e = 0; e < E; e++) {
        const int slot = e & 1;
        PackedPt<C> pk;
#pragma unroll
        for (int k = 0; k < NCH; k++) pk.q[k] = ring[slot][k][lane];
        Affine<C> cur = packed_unpack<C>(pk);
        const int d = dn;
        if (e + 1 < E) issue(slot ^ 1, g.next(dn));
        if (d != 0) {
          if (d < 0) cur.y = f29_neg_lazy<typename C::Fp29>(cur.y);
          acc = xyzz_add_affine_v<C, V>(acc, cur);
        }
      }
    }
  } else {
   if (E > 0) {
    G g;
    g.sc = scalars + (size_t)b * stride_words;
    g.inf = inf;
    g.tab = tab;
    g.ts = ts;
    g.i = t;
    g.T = T;
    g.load();
    int dq[PF];
    PackedPt<C> pq[PF];
#pragma unroll
    for (int k = 0; k < PF; k++) {
      dq[k] = 0;
      if (k < E) pq[k] = packed_fetch<C>(g.next(dq[k]));
    }
    // one term: add the queued entry, queue the lookup PF terms ahead
    auto step = [&](int e) {
      Affine<C> cur = packed_unpack<C>(pq[0]);
      const int d = dq[0];
#pragma unroll
      for (int k = 0; k + 1 < PF; k++) {
        pq[k] = pq[k + 1];
        dq[k] = dq[k + 1];
      }
      dq[PF - 1] = 0;
      if (e + PF < E) pq[PF - 1] = packed_fetch<C>(g.next(dq[PF - 1]));
      if (d != 0) {
        // -T = (x, 2m - y): one v_sub per limb (f29_neg_lazy; the
        // mixed add only multiplies y and feeds it to carry-absorbing subs)
        if (d < 0) cur.y = f29_neg_lazy<typename C::Fp29>(cur.y);
        acc = xyzz_add_affine_v<C, V>(acc, cur);
      }
    };
    // (a two-term body, for the allocator to alternate the accumulator
    // between two register sets instead of copying it back, spilled: 368 B
    // of scratch on BN254, 704 B on BLS12-381)
#pragma unroll 1
    for (int e = 0; e < E; e++) step(e);
   }
  }
  xyzz_store<C>(part + ((size_t)b * T + t) * XW, acc);
}

}  // namespace kzgx
