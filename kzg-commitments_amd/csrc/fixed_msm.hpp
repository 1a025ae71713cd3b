// The per-window half of the fixed-base G1 MSM (msm_fixed.hip holds the
// table build, the reductions and the dispatch): the accumulation kernels
// templated on the window -- the one-launch latency kernel
// k_fixed_accum_lat, the flattened few-large-MSM kernel k_fixed_accum_flat,
// and fixed_accum.hpp's batched k_fixed_accum -- and fixed_msm_win, the host
// routine that picks among them.  Instantiated per (curve, window group) in
// separate translation units (msm_fixed_inst.hip, compiled once per group by
// the Makefile) so a parallel build compiles them side by side.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "curve.hpp"
#include "fixed_accum.hpp"
#include "kzgx_internal.hpp"

namespace kzgx {

// msm_fixed.hip: k_fixed_reduce (one wavefront per MSM over T partials) and
// k_fixed_finish (XYZZ -> canonical affine, or the XYZZ copy) launches
template <class C>
void fixed_reduce_launch(const uint32_t* part, uint32_t T, uint32_t batch, uint32_t* sums, hipStream_t st);
template <class C>
void fixed_finish_launch(const uint32_t* sums, uint32_t batch, uint32_t* out, uint32_t* out_inf, uint32_t* xyzz_out,
                         hipStream_t st);

template <class C>
inline TabStrides fixed_strides(bool point_major, int W, size_t n, uint64_t H) {
  constexpr size_t PW = packed_words<C>();
  if (point_major) return TabStrides{(size_t)W * H * PW, H * PW};
  return TabStrides{H * PW, n * H * PW};
}

template <class C>
inline TabStrides tab_strides(const FixedTable& ft) {
  return fixed_strides<C>(ft.point_major, ft.W, ft.n_t, 1ull << (ft.c - 1));
}

// the infinity flags the accumulation kernels read, or null when none is set
inline const uint8_t* fixed_inf(const FixedTable& ft) { return ft.any_inf ? ft.inf : nullptr; }

// the MSM over table ft at window CB (explicitly instantiated per (curve,
// window) in the msm_fixed_inst.hip objects; msm_fixed.hip dispatches on ft.c)
template <class C, int CB>
int fixed_msm_win(Ctx* ctx, FixedTable& ft, const uint32_t* d_scalars, size_t n, size_t batch, size_t stride_words,
                  uint32_t* d_out, uint32_t* d_out_inf, hipStream_t st, uint32_t* xyzz_out);

#ifdef KZGX_FIXED_INST
// --------------------------------------------------------------------------
// latency path (a few MSMs of <= 2^14 points): every step below runs on
// mostly idle CUs, so the time of one call is the longest dependent chain of
// point additions, each ~5 us (mixed) / ~8 us (XYZZ) in one lane
// (scripts/lat_micro.py).  The chain is cut to
//   WG mixed additions (a thread owns one point and WG of its W windows)
//   + 6 shuffle additions (wavefront fold inside the accumulation kernel)
//   + Q / 64 - 1 + log2(min(Q, 64)) additions (one wavefront per MSM over the
//     Q <= 256 wavefront partials, which then converts to affine in lane 0)
// instead of W mixed additions + two 64:1 fold levels + a separate finish.
// --------------------------------------------------------------------------
// lane l and lane l ^ off both add the pair, the lower lane's value first:
// the same operands in the same order give bit-identical XYZZ values in both
// lanes (the addition is not symmetric in representation: swapping the
// operands negates P, hence Y3 and ZZZ3), which xyzz_coop_level's butterfly
// layout relies on when it reads one point's fields from different lanes
template <class C>
KZGX_DEV Xyzz<C> xyzz_shfl_xor_add(const Xyzz<C>& acc, int off) {
  constexpr int L = C::Fp29::L;
  const bool hi = (threadIdx.x & (unsigned)off) != 0;
  Xyzz<C> o, a, b;
#pragma unroll
  for (int k = 0; k < L; k++) {
    o.X.v[k] = __shfl_xor(acc.X.v[k], off, 64);
    o.Y.v[k] = __shfl_xor(acc.Y.v[k], off, 64);
    o.ZZ.v[k] = __shfl_xor(acc.ZZ.v[k], off, 64);
    o.ZZZ.v[k] = __shfl_xor(acc.ZZZ.v[k], off, 64);
    a.X.v[k] = hi ? o.X.v[k] : acc.X.v[k];
    a.Y.v[k] = hi ? o.Y.v[k] : acc.Y.v[k];
    a.ZZ.v[k] = hi ? o.ZZ.v[k] : acc.ZZ.v[k];
    a.ZZZ.v[k] = hi ? o.ZZZ.v[k] : acc.ZZZ.v[k];
    b.X.v[k] = hi ? acc.X.v[k] : o.X.v[k];
    b.Y.v[k] = hi ? acc.Y.v[k] : o.Y.v[k];
    b.ZZ.v[k] = hi ? acc.ZZ.v[k] : o.ZZ.v[k];
    b.ZZZ.v[k] = hi ? acc.ZZZ.v[k] : o.ZZZ.v[k];
  }
  return xyzz_add_impl<C>(a, b);
}

// ---- the last four fold levels as cooperative additions ------------------
// A lone wave pays for every instruction it issues whatever the number of
// lanes doing useful work, so the last levels of a shuffle tree (8, 4, 2, 1
// additions) leave most lanes idle while one addition's ~14 dependent
// products run in sequence.  Here a group of 8 lanes computes one addition:
// its independent products side by side, in 4 rounds --
//   (U1, U2, S1, S2, ZZ1 ZZ2, ZZZ1 ZZZ2), (P^2, R^2), (P PP, U1 PP, ZZ12 PP),
//   (ZZZ12 PPP, R (Q - X3), S1 PPP)
// -- with the operands moved between lanes by ds_bpermute (__shfl).  Same
// formulas and value bounds as xyzz_add_impl (add-2008-s; Y3 as a difference
// of two products, < 4m), so the sum is the same group element.  Infinity
// on either side or equal x (P^2 = 0) in any active group sends the whole
// level to xyzz_add_impl with the full operands (exact special cases).
template <class C>
KZGX_DEV F29<typename C::Fp29> xyzz_field(const Xyzz<C>& p, uint32_t f) {
  F29<typename C::Fp29> r;
#pragma unroll
  for (int k = 0; k < C::Fp29::L; k++)
    r.v[k] = f == 0 ? p.X.v[k] : f == 1 ? p.Y.v[k] : f == 2 ? p.ZZ.v[k] : p.ZZZ.v[k];
  return r;
}

template <class F>
KZGX_DEV F29<F> f29_shfl(const F29<F>& v, uint32_t src) {
  F29<F> r;
#pragma unroll
  for (int k = 0; k < F::L; k++) r.v[k] = __shfl(v.v[k], (int)src, 64);
  return r;
}

template <class F>
KZGX_DEV F29<F> f29_sel(bool c, const F29<F>& a, const F29<F>& b) {
  F29<F> r;
#pragma unroll
  for (int k = 0; k < F::L; k++) r.v[k] = c ? a.v[k] : b.v[k];
  return r;
}

// values V[j], j < 2 half (half <= 8), as held on entry:
//   bfly: the xor-butterfly state after the off = 32 and 16 shuffle levels
//         (V[j] in lanes j, j + 16, j + 32, j + 48; lane k offers field k >> 4)
//   else: a previous level's result (V[j] in group j; lane 8 j + s offers
//         field s & 3)
// returns V[g] + V[g + half] in every lane of group g = lane / 8 < half
// (garbage in the other groups).  Every lane of the wave must call it.
template <class C>
KZGX_PT Xyzz<C> xyzz_coop_level(const Xyzz<C>& mine, uint32_t lane, uint32_t half, bool bfly) {
  using F = typename C::Fp29;
  const uint32_t g = lane >> 3, s = lane & 7, g8 = lane & ~7u;
  const bool act = g < half;
  const uint32_t a = act ? g : 0, b = act ? g + half : half;
  const F29<F> prov = xyzz_field<C>(mine, bfly ? (lane >> 4) : (lane & 3));
  auto src = [&](uint32_t j, uint32_t f) -> uint32_t { return bfly ? j + 16 * f : 8 * j + f; };
  auto full = [&](uint32_t j) -> Xyzz<C> {
    Xyzz<C> r;
    r.X = f29_shfl<F>(prov, src(j, 0));
    r.Y = f29_shfl<F>(prov, src(j, 1));
    r.ZZ = f29_shfl<F>(prov, src(j, 2));
    r.ZZZ = f29_shfl<F>(prov, src(j, 3));
    return r;
  };
  const int inf_self = xyzz_is_inf<C>(mine) ? 1 : 0;
  const int inf_ab = __shfl(inf_self, (int)src(a, 0), 64) | __shfl(inf_self, (int)src(b, 0), 64);
  if (__any(act && inf_ab)) return xyzz_add<C>(full(a), full(b));
  // round 1: s = 0..5 -> U1 = X_a ZZ_b, U2 = X_b ZZ_a, S1 = Y_a ZZZ_b,
  // S2 = Y_b ZZZ_a, ZZ_a ZZ_b, ZZZ_a ZZZ_b (s = 6, 7 repeat s = 0)
  const bool sb = s == 1 || s == 3;
  const uint32_t xf = s == 2 || s == 3 ? 1u : s == 4 ? 2u : s == 5 ? 3u : 0u;
  const uint32_t yf = s == 2 || s == 3 || s == 5 ? 3u : 2u;
  const F29<F> p1 = f29_mul<F>(f29_shfl<F>(prov, src(sb ? b : a, xf)), f29_shfl<F>(prov, src(sb ? a : b, yf)));
  // round 2: even lanes P = U2 - U1, PP = P^2; odd lanes R = S2 - S1, RR = R^2
  const uint32_t k2 = (s & 1) * 2;
  const F29<F> D = f29_sub<F>(f29_shfl<F>(p1, g8 + k2 + 1), f29_shfl<F>(p1, g8 + k2), F::P2);  // < 4m
  const F29<F> p2 = f29_sqr<F>(D);
  // round 3: s = 0 PPP = P PP, 1 Q = U1 PP, 2 ZZ3 = ZZ1 ZZ2 PP
  const F29<F> PP = f29_shfl<F>(p2, g8);
  if (__any(act && f29_is_zero_lt2m<F>(PP))) return xyzz_add<C>(full(a), full(b));  // equal x
  const F29<F> t3 = f29_shfl<F>(p1, g8 + (s == 2 ? 4u : 0u));
  const F29<F> p3 = f29_mul<F>(f29_sel<F>(s == 0, D, t3), PP);
  // round 4: s = 0 ZZZ3 = ZZZ1 ZZZ2 PPP, 1 R (Q - X3), 2 S1 PPP
  const F29<F> RR = f29_shfl<F>(p2, g8 + 1);
  const F29<F> PPP = f29_shfl<F>(p3, g8);
  const F29<F> Qv = f29_shfl<F>(p3, g8 + 1);
  Xyzz<C> r;
  r.X = f29_sub<F>(RR, f29_add<F>(PPP, f29_add<F>(Qv, Qv)), F::P6);  // < 8m
  const F29<F> t4 = f29_shfl<F>(p1, g8 + (s == 0 ? 5u : 2u));
  const F29<F> p4 = f29_mul<F>(f29_sel<F>(s == 1, D, t4), f29_sel<F>(s == 1, f29_sub<F>(Qv, r.X, F::P8), PPP));
  r.ZZ = f29_shfl<F>(p3, g8 + 2);
  r.ZZZ = f29_shfl<F>(p4, g8);
  r.Y = f29_sub<F>(f29_shfl<F>(p4, g8 + 1), f29_shfl<F>(p4, g8 + 2), F::P2);  // R (Q - X3) - S1 PPP, < 4m
  return r;
}

// a full 64-lane xor-butterfly sum (every lane holds a partial): two
// shuffle levels, then the four cooperative ones; the sum lands in lanes 0-7
// (coop = false: six shuffle levels, the sum in every lane)
template <class C>
KZGX_PT Xyzz<C> xyzz_wave_sum(Xyzz<C> acc, uint32_t lane, bool coop) {
  if (!coop) {
#pragma unroll 1
    for (int off = 32; off >= 1; off >>= 1) acc = xyzz_shfl_xor_add<C>(acc, off);
    return acc;
  }
  acc = xyzz_shfl_xor_add<C>(acc, 32);
  acc = xyzz_shfl_xor_add<C>(acc, 16);
  acc = xyzz_coop_level<C>(acc, lane, 8, true);
#pragma unroll 1
  for (uint32_t h = 4; h >= 1; h >>= 1) acc = xyzz_coop_level<C>(acc, lane, h, false);
  return acc;
}

template <class C>
KZGX_DEV Xyzz<C> lat_fold(const uint32_t* __restrict__ p, uint32_t Q, uint32_t lane, bool coop);
template <class C>
KZGX_DEV void lat_store_affine(const Xyzz<C>& acc, uint32_t b, uint32_t lane, uint32_t* __restrict__ out,
                               uint32_t* __restrict__ out_inf);

// thread (g, i): point i < n_pad of MSM b, windows [g WG, min(W, (g + 1) WG));
// wavefront partial q = (g n_pad + i) / 64 -> part[b][q].  NG = 1: the last
// of the Q wavefronts folds all Q partials; NG > 1 (Q > 128): the last
// wavefront of each group of 64 folds its group into part2[b][group], and the
// last of the NG group folders folds those (two fold levels of <= 64
// partials each instead of one wavefront summing Q / 64 partials per lane).
// cnt[b (NG + 1)]: the final arrival counter, then one per group.
template <class C, int CB>
__global__ __launch_bounds__(64) void k_fixed_accum_lat(const uint32_t* __restrict__ scalars, uint32_t n,
                                                        uint32_t n_pad, size_t stride_words,
                                                        const uint32_t* __restrict__ tab, TabStrides ts,
                                                        const uint8_t* __restrict__ inf, int WG, uint32_t Q,
                                                        uint32_t* __restrict__ part, uint32_t* __restrict__ cnt,
                                                        uint32_t* __restrict__ out, uint32_t* __restrict__ out_inf,
                                                        int coop, uint32_t NG, uint32_t* __restrict__ part2) {
  constexpr int PW = packed_words<C>();
  constexpr int XW = xyzz_words<C>();
  constexpr int W = FixedWin<C, CB>::W;
  const uint32_t b = blockIdx.y;
  const uint32_t t = blockIdx.x * 64 + threadIdx.x;  // < G n_pad: grid is exact
  const uint32_t g = t / n_pad, i = t - g * n_pad;
  const int w0 = (int)g * WG, w1 = w0 + WG < W ? w0 + WG : W;
  Xyzz<C> acc = xyzz_inf<C>();
  if (i < n && !(inf != nullptr && inf[i] != 0)) {
    const uint32_t* sc = scalars + (size_t)b * stride_words + (size_t)i * 8;
    uint32_t s[8];
    {
      const uint4 lo = reinterpret_cast<const uint4*>(sc)[0];
      const uint4 hi = reinterpret_cast<const uint4*>(sc)[1];
      s[0] = lo.x; s[1] = lo.y; s[2] = lo.z; s[3] = lo.w;
      s[4] = hi.x; s[5] = hi.y; s[6] = hi.z; s[7] = hi.w;
    }
    scalar_reduce<C>(s);
    const uint32_t flip = odd_prepare<C>(s);
    const uint32_t* base = tab + (size_t)i * ts.is;
#pragma unroll 1
    for (int w = 0; w < w0; w++) shr_scalar<CB>(s);  // odd digits carry nothing: skip the lower windows
#pragma unroll 1
    for (int w = w0; w < w1; w++) {
      uint32_t j, neg;
      odd_digit<CB>(s[0], w == W - 1, flip, j, neg);
      shr_scalar<CB>(s);
      Affine<C> cur = packed_unpack<C>(packed_fetch<C>(base + (size_t)w * ts.ws + (size_t)j * PW));
      affine_cond_neg<C>(cur, neg);
      acc = xyzz_add_affine_impl<C>(acc, cur);
    }
  }
  acc = xyzz_wave_sum<C>(acc, threadIdx.x, coop != 0);  // lane 0 holds the wavefront's sum
  // the last of MSM b's Q wavefronts to finish folds the Q partials (one
  // launch per call instead of two): release the partial, count it in
  // (device-scope atomic), and the wavefront that counts the Q-th acquires
  // the others and runs the fold
  const uint32_t q = t / 64, lane = threadIdx.x;
  uint32_t* cb = cnt + (size_t)b * (NG + 1);
  const uint32_t grp = q >> 6;
  uint32_t prev = 0;
  if (lane == 0) {
    xyzz_store<C>(part + ((size_t)b * Q + q) * XW, acc);
    __threadfence();
    prev = atomicAdd(NG > 1 ? cb + 1 + grp : cb, 1u);
  }
  prev = __shfl(prev, 0, 64);
  if (NG > 1) {
    const uint32_t gsz = Q - grp * 64 < 64 ? Q - grp * 64 : 64;
    if (prev + 1 != gsz) return;
    __threadfence();
    const Xyzz<C> gs = lat_fold<C>(part + ((size_t)b * Q + grp * 64) * XW, gsz, lane, coop != 0);
    if (lane == 0) {
      cb[1 + grp] = 0;  // every arrival of the group is in
      xyzz_store<C>(part2 + ((size_t)b * NG + grp) * XW, gs);
      __threadfence();
      prev = atomicAdd(cb, 1u);
    }
    prev = __shfl(prev, 0, 64);
    if (prev + 1 != NG) return;
    __threadfence();
    lat_store_affine<C>(lat_fold<C>(part2 + (size_t)b * NG * XW, NG, lane, coop != 0), b, lane, out, out_inf);
  } else {
    if (prev + 1 != Q) return;
    __threadfence();
    lat_store_affine<C>(lat_fold<C>(part + (size_t)b * Q * XW, Q, lane, coop != 0), b, lane, out, out_inf);
  }
  if (lane == 0) cb[0] = 0;  // ready for the next call (stream order)
}

// the sum of Q partials p[0..Q) by one wavefront, in lane 0: lane sums
// partials lane, lane + 64, ... < Q, then a butterfly (cooperative last
// levels) or a shuffle tree over the lanes that hold any
template <class C>
KZGX_DEV Xyzz<C> lat_fold(const uint32_t* __restrict__ p, uint32_t Q, uint32_t lane, bool coop) {
  constexpr int XW = xyzz_words<C>();
  Xyzz<C> acc = lane < Q ? xyzz_load<C>(p + (size_t)lane * XW) : xyzz_inf<C>();
#pragma unroll 1
  for (uint32_t k = lane + 64; k < Q; k += 64) acc = xyzz_add_impl<C>(acc, xyzz_load<C>(p + (size_t)k * XW));
  if (coop && Q > 16) return xyzz_wave_sum<C>(acc, lane, true);  // the full butterfly (lanes >= Q: identity)
  int off = 32;
  while (off > 1 && (uint32_t)off >= Q) off >>= 1;  // lanes >= Q hold the identity
#pragma unroll 1
  for (; off >= 1; off >>= 1) acc = xyzz_shfl_xor_add<C>(acc, off);
  return acc;
}

// MSM b's sum (lane 0's) converted by the whole wavefront on lane 0's value
// (uniform: the inversion's bit-serial loop on the scalar ALU, its linear
// combinations one per lane) and stored by lane 0
template <class C>
KZGX_DEV void lat_store_affine(const Xyzz<C>& acc, uint32_t b, uint32_t lane, uint32_t* __restrict__ out,
                               uint32_t* __restrict__ out_inf) {
  Xyzz<C> s;
#pragma unroll
  for (int k = 0; k < C::Fp29::L; k++) {
    s.X.v[k] = __builtin_amdgcn_readfirstlane(acc.X.v[k]);
    s.Y.v[k] = __builtin_amdgcn_readfirstlane(acc.Y.v[k]);
    s.ZZ.v[k] = __builtin_amdgcn_readfirstlane(acc.ZZ.v[k]);
    s.ZZZ.v[k] = __builtin_amdgcn_readfirstlane(acc.ZZZ.v[k]);
  }
  constexpr int N = C::Fp::N;
  uint32_t wx[N], wy[N];
  const bool fin = xyzz_to_canonical_lane<C>(s, wx, wy);
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < N; k++) {
      out[(size_t)b * 2 * N + k] = wx[k];
      out[(size_t)b * 2 * N + N + k] = wy[k];
    }
    out_inf[b] = fin ? 0u : 1u;
  }
}

// --------------------------------------------------------------------------
// few large MSMs (cfg5: one 2^20-point commit over a table shard).  The
// point-strided k_fixed_accum gives each thread ceil(n / T) whole points, so
// with 2^20 points over the 196 608 resident lanes some SIMDs carry 3 waves x
// 6 points while the average is 5.3: the busiest SIMD is 12.5% over the mean
// (measured: 83% of the mixed-add peak).  Here the n W digit terms are
// flattened point-major (term e = i W + w) and thread t owns the Q
// consecutive terms [t Q, t Q + Q): every thread does Q or fewer additions.
// A thread that starts inside point i runs the digit recoding of i's lower
// windows for their carry only.  The lookup of the next term is in flight
// during the addition of the current one.  lane_parts: every thread stores
// its partial (part[b][t], for k_fixed_fold3); else the wavefront folds its
// 64 partials with 6 shuffle additions before one lane stores (round 5: the
// first 64:1 level of the reduction without a launch -- but 6 full additions
// on every one of the ~3 resident waves per SIMD, ~90 us of a 131 073-point
// shard's 0.4 ms accumulation).
// --------------------------------------------------------------------------
template <class C, int CB>
__global__ __launch_bounds__(64, fixed_accum_waves<C>()) void k_fixed_accum_flat(
    const uint32_t* __restrict__ scalars, uint32_t n, size_t stride_words, const uint32_t* __restrict__ tab,
    TabStrides ts, const uint8_t* __restrict__ inf, uint32_t Q, uint32_t T, uint32_t* __restrict__ part,
    uint32_t lane_parts) {
  constexpr int PW = packed_words<C>();
  constexpr int XW = xyzz_words<C>();
  constexpr int W = FixedWin<C, CB>::W;
  const uint32_t b = blockIdx.y;
  const uint32_t t = blockIdx.x * 64 + threadIdx.x;  // < T: the grid is exact
  const uint32_t* sc = scalars + (size_t)b * stride_words;
  const size_t e_end = (size_t)n * W;
  size_t e = (size_t)t * Q;
  const size_t e1 = e + Q < e_end ? e + Q : e_end;
  Xyzz<C> acc = xyzz_inf<C>();
  if (e < e1) {
    // generator state: point i, window w, the remaining bits of u (odd
    // digits, fixed_accum.hpp) and the sign flip of the point's scalar
    uint32_t i = (uint32_t)(e / W);
    int w = (int)(e - (size_t)i * W);
    uint32_t s[8], flip = 0;
    bool skip = false;  // infinity SRS point: all its terms are the identity
    auto load = [&](uint32_t ii) {
      scalar_load(sc + (size_t)ii * 8, s);
      scalar_reduce<C>(s);
      flip = odd_prepare<C>(s);
      skip = inf != nullptr && inf[ii] != 0;
    };
    load(i);
#pragma unroll 1
    for (int k = 0; k < w; k++) shr_scalar<CB>(s);  // no carry: the lower windows are skipped outright
    // the table entry of the current term (i, w); consumes its window bits
    struct Term {
      PackedPt<C> p;
      uint32_t neg;
      bool skip;
    };
    auto fetch = [&]() {
      Term r;
      uint32_t j;
      odd_digit<CB>(s[0], w == W - 1, flip, j, r.neg);
      shr_scalar<CB>(s);
      r.skip = skip;
      r.p = packed_fetch<C>(tab + (size_t)i * ts.is + (size_t)w * ts.ws + (size_t)j * PW);
      return r;
    };
    auto advance = [&]() {
      if (++w == W) {
        w = 0;
        load(++i);
      }
    };
    Term t0 = fetch();
    // two lookups in flight: terms e + 1 and e + 2 load during the addition
    // of term e (one wave in three is ready to issue while the other two wait
    // on random table lines)
    Term t1 = t0;
    if (e + 1 < e1) {
      advance();
      t1 = fetch();
    }
#pragma unroll 1
    for (; e < e1; e++) {
      Affine<C> cur = packed_unpack<C>(t0.p);
      const uint32_t neg = t0.neg;
      const bool sk = t0.skip;
      t0 = t1;
      if (e + 2 < e1) {
        advance();
        t1 = fetch();
      }
      if (!sk) {
        affine_cond_neg<C>(cur, neg);
        acc = xyzz_add_affine_impl<C>(acc, cur);
      }
    }
  }
  if (lane_parts) {
    xyzz_store<C>(part + ((size_t)b * T + t) * XW, acc);
    return;
  }
#pragma unroll 1
  for (int off = 32; off >= 1; off >>= 1) acc = xyzz_shfl_xor_add<C>(acc, off);
  if (threadIdx.x == 0) xyzz_store<C>(part + ((size_t)b * (T / 64) + t / 64) * XW, acc);
}

// One fold level as its own launch (the default; KZGX_FOLD3_SPLIT=0 runs
// k_fixed_fold3's arrival counters and device-scope fences): wavefront g
// folds in[g per, g per + per) into out[g]; with fin, group g = MSM b's last
// level, stored as the XYZZ record or converted to affine
template <class C>
__global__ __launch_bounds__(64) void k_fold_level(const uint32_t* __restrict__ in, uint32_t per,
                                                   uint32_t* __restrict__ out, int fin, uint32_t* __restrict__ fout,
                                                   uint32_t* __restrict__ fout_inf, uint32_t* __restrict__ xyzz_out) {
  constexpr int XW = xyzz_words<C>();
  const uint32_t g = blockIdx.x, lane = threadIdx.x;
  const uint32_t* src = in + (size_t)g * per * XW;
  Xyzz<C> s;
  if (per == 256) {
    auto ld = [&](int k) { return xyzz_load<C>(src + (size_t)(lane + 64 * k) * XW); };
    s = xyzz_wave_sum<C>(xyzz_add_impl<C>(xyzz_add_impl<C>(ld(0), ld(1)), xyzz_add_impl<C>(ld(2), ld(3))), lane, true);
  } else {
    s = lat_fold<C>(src, per, lane, true);
  }
  if (!fin) {
    if (lane == 0) xyzz_store<C>(out + (size_t)g * XW, s);
    return;
  }
  if (xyzz_out) {
    if (lane == 0) xyzz_store<C>(xyzz_out + (size_t)g * XW, s);
    return;
  }
  lat_store_affine<C>(s, g, lane, fout, fout_inf);
}

// The flat path's reduction in one launch (three fold levels, arrival
// counters as k_fixed_accum_lat): wavefront q < P1 of MSM b folds partials
// [q per, q per + per) (lat_fold: strided sums, then the butterfly with
// cooperative last levels) into part2[b][q]; the last wavefront of each
// group of 64 to arrive folds its group's sums into part3[b][grp]; the last
// of the NG group folders folds those into the result -- the XYZZ record
// (xyzz_out) or the canonical affine point.  Three levels of <= 64 partials
// on mostly idle SIMDs, each a few dependent additions, instead of a 6-level
// shuffle fold in every accumulating wavefront plus two reduce launches
// (131 073-point shard at c = 10: 0.22 ms of reduction in round 5).
// cnt[b (NG + 1)]: the final counter, then one per group; each is zeroed by
// the wavefront that consumes it (stream order makes the next call see 0).
template <class C>
__global__ __launch_bounds__(64) void k_fixed_fold3(const uint32_t* __restrict__ part, uint32_t per, uint32_t P1,
                                                    uint32_t NG, uint32_t* __restrict__ part2,
                                                    uint32_t* __restrict__ part3, uint32_t* __restrict__ cnt,
                                                    uint32_t* __restrict__ out, uint32_t* __restrict__ out_inf,
                                                    uint32_t* __restrict__ xyzz_out) {
  constexpr int XW = xyzz_words<C>();
  const uint32_t b = blockIdx.y, q = blockIdx.x, lane = threadIdx.x;
  const uint32_t* src = part + ((size_t)b * P1 * per + (size_t)q * per) * XW;
  Xyzz<C> s;
  if (per == 256 || per == 512) {
    // the lane's 4 (8) strided partials as a tree of independent additions
    // (depth 2 (3)) instead of a chain of 3 (7)
    auto ld = [&](int k) { return xyzz_load<C>(src + (size_t)(lane + 64 * k) * XW); };
    s = xyzz_add_impl<C>(xyzz_add_impl<C>(ld(0), ld(1)), xyzz_add_impl<C>(ld(2), ld(3)));
    if (per == 512) s = xyzz_add_impl<C>(s, xyzz_add_impl<C>(xyzz_add_impl<C>(ld(4), ld(5)), xyzz_add_impl<C>(ld(6), ld(7))));
    s = xyzz_wave_sum<C>(s, lane, true);
  } else {
    s = lat_fold<C>(src, per, lane, true);
  }
  uint32_t* cb = cnt + (size_t)b * (NG + 1);
  const uint32_t grp = q >> 6;
  uint32_t prev = 0;
  if (lane == 0) {
    xyzz_store<C>(part2 + ((size_t)b * P1 + q) * XW, s);
    __threadfence();
    prev = atomicAdd(cb + 1 + grp, 1u);
  }
  prev = __shfl(prev, 0, 64);
  const uint32_t gsz = P1 - grp * 64 < 64 ? P1 - grp * 64 : 64;
  if (prev + 1 != gsz) return;
  __threadfence();
  s = lat_fold<C>(part2 + ((size_t)b * P1 + grp * 64) * XW, gsz, lane, true);
  if (lane == 0) {
    cb[1 + grp] = 0;  // every arrival of the group is in
    xyzz_store<C>(part3 + ((size_t)b * NG + grp) * XW, s);
    __threadfence();
    prev = atomicAdd(cb, 1u);
  }
  prev = __shfl(prev, 0, 64);
  if (prev + 1 != NG) return;
  __threadfence();
  s = lat_fold<C>(part3 + (size_t)b * NG * XW, NG, lane, true);
  if (lane == 0) cb[0] = 0;
  if (xyzz_out) {
    if (lane == 0) xyzz_store<C>(xyzz_out + (size_t)b * XW, s);
    return;
  }
  lat_store_affine<C>(s, b, lane, out, out_inf);
}

template <class C, int CB>
int fixed_msm_win(Ctx* ctx, FixedTable& ft, const uint32_t* d_scalars, size_t n, size_t batch, size_t stride_words,
                  uint32_t* d_out, uint32_t* d_out_inf, hipStream_t st, uint32_t* xyzz_out) {
  const size_t XB = xyzz_words<C>() * sizeof(uint32_t);
  // latency path: a few MSMs of <= 2^14 points (k_fixed_accum_lat)
  static const bool lat_off = std::getenv("KZGX_NO_FIXED_LAT") != nullptr;
  const size_t n_pad = (n + 63) / 64 * 64;
  if (batch <= 16 && !xyzz_out && n_pad <= 16384 && ft.pts_per_thread == 0 && !lat_off) {
    constexpr int W = FixedWin<C, CB>::W;
    // G window groups of WG windows over up to 2^14 threads per MSM
    // (KZGX_LAT_THREADS: the single-MSM count, A/B; 2^16 measured slower:
    // degree 4096 0.233 vs 0.202 ms, profiles/r04_lat_ab_coop_threads.txt):
    // degree 4096 takes 3 groups of 8 windows (195 wavefront partials,
    // folded in two levels), degree 128 one window per thread
    static const size_t lat_threads = std::getenv("KZGX_LAT_THREADS") ? std::strtoul(std::getenv("KZGX_LAT_THREADS"), nullptr, 10) : 16384;
    const size_t per_msm = std::max<size_t>(std::min<size_t>(lat_threads, 16384), lat_threads / batch);
    int G = (int)std::min<size_t>(W, std::max<size_t>(1, per_msm / n_pad));
    int WG = (W + G - 1) / G;
    // between 64 and 128 partials, one more window per thread when that
    // leaves <= 64 partials (a fold with no strided level: a mixed addition
    // instead of an XYZZ one on the chain; degree 128 / 256 commits -2.5 us,
    // profiles/r04_lat_ab_q64_qwg8.txt; KZGX_LAT_Q64=0 turns it off, A/B)
    static const bool q64 = !(std::getenv("KZGX_LAT_Q64") && std::getenv("KZGX_LAT_Q64")[0] == '0');
    if (q64 && n_pad * G / 64 > 64 && n_pad * G / 64 <= 128) {
      const int G2 = (int)(64 * 64 / n_pad);
      if (G2 >= 1 && (W + G2 - 1) / G2 <= WG + 1) WG = (W + G2 - 1) / G2;
    }
    G = (W + WG - 1) / WG;
    const uint32_t Q = (uint32_t)(n_pad * G / 64);
    const uint32_t NG = Q > 128 ? (Q + 63) / 64 : 1;  // <= 16
    WsLease wsp = ctx->ws_for(st);
    if (!wsp) return KZGX_ERR_ARG;
    KZGX_TRY(dev_alloc(ctx, (void**)&wsp->fpart, batch * (Q + NG) * XB, &wsp->fpart_b));
    constexpr size_t kCnt = 16 * 17;  // batch <= 16 MSMs x (NG <= 16 groups + 1)
    if (!wsp->lat_cnt) {  // per-MSM arrival counters, zero between calls
      KZGX_TRY_HIP(hipMalloc((void**)&wsp->lat_cnt, kCnt * sizeof(uint32_t)));
      KZGX_TRY_HIP(hipMemsetAsync(wsp->lat_cnt, 0, kCnt * sizeof(uint32_t), st));
    }
    if (NG > 16 || batch * (NG + 1) > kCnt) return KZGX_ERR_ARG;  // unreachable: Q <= 2^16 / 64
    // KZGX_NO_LAT_COOP: the last fold levels as plain shuffle additions (A/B)
    static const bool coop_off = std::getenv("KZGX_NO_LAT_COOP") != nullptr;
    ProfScope p(ctx, st, "msm_accum");
    hipLaunchKernelGGL((k_fixed_accum_lat<C, CB>), dim3(Q, (unsigned)batch), dim3(64), 0, st, d_scalars, (uint32_t)n,
                       (uint32_t)n_pad, stride_words, ft.d, tab_strides<C>(ft), fixed_inf(ft), WG, Q, wsp->fpart,
                       wsp->lat_cnt, d_out, d_out_inf, coop_off ? 0 : 1, NG, wsp->fpart + batch * Q * XB / 4);
    KZGX_TRY_HIP(hipGetLastError());
    return KZGX_OK;
  }
  // points per thread: 16 for batches (one MSM ~ 5 wavefronts at degree
  // 4096, T = 320 partials); for a few large MSMs, enough threads to fill
  // the 256 CUs x 4 SIMDs x 3 waves of resident slots
  constexpr size_t kSlots = 256 * 4 * 3 * 64;
  // few large MSMs (>= 8 terms per resident lane): flattened terms, balanced
  // to one addition per thread (k_fixed_accum_flat), T a multiple of 64^2
  static const bool flat_off = std::getenv("KZGX_NO_FIXED_FLAT") != nullptr;
  // instantiated for c <= 12 only: from c = 13 a table with 8 x 196 608 terms
  // (BN254: >= 78 644 points x 20 windows x 4096 entries x 64 B = 422 GB) does
  // not fit in HBM, so the path could never run (and each instantiation costs
  // compile time)
  if constexpr (CB <= 12) {
    constexpr int W = FixedWin<C, CB>::W;
    const size_t terms = n * (size_t)W;
    if (batch <= 16 && ft.pts_per_thread == 0 && !flat_off && terms * batch >= 8 * kSlots) {
      // KZGX_FLAT_TMULT: threads per resident-lane slot (A/B)
      static const size_t tmult = std::getenv("KZGX_FLAT_TMULT") ? std::strtoul(std::getenv("KZGX_FLAT_TMULT"), nullptr, 10) : 1;
      const uint32_t T = (uint32_t)std::max<size_t>(4096, kSlots * (tmult ? tmult : 1) / batch / 4096 * 4096);
      const uint32_t Q = (uint32_t)((terms + T - 1) / T);
      WsLease wsp = ctx->ws_for(st);
      if (!wsp) return KZGX_ERR_ARG;
      MsmWs& ws = *wsp;
      // round 6: per-lane partials and the one-launch three-level fold
      // (k_fixed_fold3); KZGX_FLAT_WAVEFOLD=1 keeps round 5's in-wave fold
      // and reduce launches (A/B)
      static const bool wavefold = std::getenv("KZGX_FLAT_WAVEFOLD") && std::getenv("KZGX_FLAT_WAVEFOLD")[0] == '1';
      constexpr size_t kCnt = 16 * 17;  // the lat path's counter block
      // per: partials per first-level wavefront (KZGX_FOLD3_PER, A/B: 64 / 128 / 256)
      static const uint32_t per = std::getenv("KZGX_FOLD3_PER") ? (uint32_t)std::strtoul(std::getenv("KZGX_FOLD3_PER"), nullptr, 10) : 256u;
      const uint32_t P1 = T / per, NG = (P1 + 63) / 64;  // T is a multiple of 4096
      if (!wavefold && (per == 64 || per == 128 || per == 256 || per == 512) && batch * (NG + 1) <= kCnt) {
        KZGX_TRY(dev_alloc(ctx, (void**)&ws.fpart, batch * (size_t)T * XB, &ws.fpart_b));
        KZGX_TRY(dev_alloc(ctx, (void**)&ws.fsum, batch * (size_t)(P1 + NG) * XB, &ws.fsum_b));
        if (!ws.lat_cnt) {  // arrival counters, zero between calls
          KZGX_TRY_HIP(hipMalloc((void**)&ws.lat_cnt, kCnt * sizeof(uint32_t)));
          KZGX_TRY_HIP(hipMemsetAsync(ws.lat_cnt, 0, kCnt * sizeof(uint32_t), st));
        }
        {
          ProfScope p(ctx, st, "msm_accum");
          hipLaunchKernelGGL((k_fixed_accum_flat<C, CB>), dim3(T / 64, (unsigned)batch), dim3(64), 0, st, d_scalars,
                             (uint32_t)n, stride_words, ft.d, tab_strides<C>(ft), fixed_inf(ft), Q, T, ws.fpart, 1u);
        }
        ProfScope p(ctx, st, "msm_reduce");
        // three launches by default: measured 15-20 us faster than
        // k_fixed_fold3's one launch on the same box (131 073 points, c = 10:
        // 0.438-0.458 vs 0.461-0.480 ms, profiles/r06_shard_fixed.jsonl) --
        // the arrival pattern's device-scope release fences write back the
        // L2 that still holds the accumulation's 28 MB of partials, where a
        // kernel boundary does it once.  KZGX_FOLD3_SPLIT=0: k_fixed_fold3 (A/B)
        static const bool split = !(std::getenv("KZGX_FOLD3_SPLIT") && std::getenv("KZGX_FOLD3_SPLIT")[0] == '0');
        if (split && per == 256 && P1 % 64 == 0) {
          uint32_t* f1 = ws.fsum;
          uint32_t* f2 = ws.fsum + batch * (size_t)P1 * xyzz_words<C>();
          hipLaunchKernelGGL(k_fold_level<C>, dim3(batch * P1), dim3(64), 0, st, ws.fpart, 256u, f1, 0, nullptr,
                             nullptr, nullptr);
          hipLaunchKernelGGL(k_fold_level<C>, dim3(batch * NG), dim3(64), 0, st, f1, 64u, f2, 0, nullptr, nullptr,
                             nullptr);
          hipLaunchKernelGGL(k_fold_level<C>, dim3(batch), dim3(64), 0, st, f2, NG, nullptr, 1, d_out, d_out_inf,
                             xyzz_out);
          KZGX_TRY_HIP(hipGetLastError());
          return KZGX_OK;
        }
        hipLaunchKernelGGL(k_fixed_fold3<C>, dim3(P1, (unsigned)batch), dim3(64), 0, st, ws.fpart, per, P1, NG,
                           ws.fsum, ws.fsum + batch * (size_t)P1 * xyzz_words<C>(), ws.lat_cnt, d_out, d_out_inf,
                           xyzz_out);
        KZGX_TRY_HIP(hipGetLastError());
        return KZGX_OK;
      }
      KZGX_TRY(dev_alloc(ctx, (void**)&ws.fpart, batch * (T / 64) * XB, &ws.fpart_b));
      KZGX_TRY(dev_alloc(ctx, (void**)&ws.fsum, batch * (T / 4096) * XB, &ws.fsum_b));
      {
        ProfScope p(ctx, st, "msm_accum");
        hipLaunchKernelGGL((k_fixed_accum_flat<C, CB>), dim3(T / 64, (unsigned)batch), dim3(64), 0, st, d_scalars,
                           (uint32_t)n, stride_words, ft.d, tab_strides<C>(ft), fixed_inf(ft), Q, T, ws.fpart, 0u);
      }
      ProfScope p(ctx, st, "msm_reduce");
      // T / 64 wavefront partials per MSM: one more 64:1 level, then one
      // wavefront per MSM over the T / 4096 left, then a thread per MSM
      const size_t g2 = batch * (T / 4096);
      fixed_reduce_launch<C>(ws.fpart, 64u, (uint32_t)g2, ws.fsum, st);
      fixed_reduce_launch<C>(ws.fsum, T / 4096, (uint32_t)batch, ws.fpart, st);
      fixed_finish_launch<C>(ws.fpart, (uint32_t)batch, d_out, d_out_inf, xyzz_out, st);
      KZGX_TRY_HIP(hipGetLastError());
      return KZGX_OK;
    }
  }
  uint32_t P0 = ft.pts_per_thread;
  // automatic: 16 points per thread from 64 MSMs; BLS12-381 from 2048 MSMs
  // 65 (one residency at two waves per SIMD, the cfg4 shape: +2.4% on the
  // default table's batches, profiles/r04_ab_ppt_auto.json; BN254 22 vs 16
  // measured +0.3%, kept); else enough threads to fill the chip.
  // KZGX_PPT_AUTO_BIG: the count from 1024 MSMs (A/B)
  static const uint32_t ppt_env = std::getenv("KZGX_PPT_AUTO_BIG") ? (uint32_t)std::strtoul(std::getenv("KZGX_PPT_AUTO_BIG"), nullptr, 10) : 0u;
  if (P0 == 0) {
    if (ppt_env && batch >= 1024) P0 = ppt_env;
    else if (C::Fp29::L > 9 && batch >= 2048) P0 = 65;
    else P0 = batch >= 64 ? 16u : (uint32_t)std::max<size_t>(1, (n * batch + kSlots - 1) / kSlots);
  }
  uint32_t T = (uint32_t)(64 * ((n + 64 * (size_t)P0 - 1) / (64 * (size_t)P0)));
  // few large MSMs: 64:1 wavefront folds until at most 128 partials per MSM
  // remain, then one wavefront per MSM folds those and a thread per MSM
  // converts -- instead of one wavefront per MSM summing T partials in
  // sequence.  Beyond 64 x 128 partials T is padded to a multiple of 64^2
  // (the extra threads own no points: identity partials) for a second 64:1
  // level.
  const bool wave_red = batch <= 16 && T > 1024;
  if (wave_red && T > 64 * 128) T = (T + 4095) / 4096 * 4096;
  WsLease wsp = ctx->ws_for(st);
  if (!wsp) return KZGX_ERR_ARG;
  MsmWs& ws = *wsp;
  KZGX_TRY(dev_alloc(ctx, (void**)&ws.fpart, batch * T * XB, &ws.fpart_b));
  KZGX_TRY(dev_alloc(ctx, (void**)&ws.fsum, batch * (wave_red ? T / 64 : 1) * XB, &ws.fsum_b));
  {
    ProfScope p(ctx, st, "msm_accum");
    hipLaunchKernelGGL((k_fixed_accum<C, CB>), dim3(T / 64, (unsigned)batch), dim3(64), 0, st, d_scalars,
                       (uint32_t)n, stride_words, ft.d, tab_strides<C>(ft), fixed_inf(ft), ft.fin0, T, ws.fpart);
  }
  if (wave_red) {
    ProfScope p(ctx, st, "msm_reduce");
    // level 1: 64:1 into fsum (T / 64 per MSM)
    const size_t g1 = batch * (T / 64);
    fixed_reduce_launch<C>(ws.fpart, 64u, (uint32_t)g1, ws.fsum, st);
    const uint32_t* lvl = ws.fsum;
    size_t per = T / 64;
    if (per > 128) {  // level 2: 64:1 back into fpart (T is a multiple of 64^2 here)
      const size_t g2 = batch * (T / 4096);
      fixed_reduce_launch<C>(ws.fsum, 64u, (uint32_t)g2, ws.fpart, st);
      lvl = ws.fpart;
      per = T / 4096;
    }
    // last level: one wavefront per MSM over its `per` partials, into the
    // buffer the last level did not read, then a thread per MSM converts
    uint32_t* fin = lvl == ws.fsum ? ws.fpart : ws.fsum;
    fixed_reduce_launch<C>(lvl, (uint32_t)per, (uint32_t)batch, fin, st);
    fixed_finish_launch<C>(fin, (uint32_t)batch, d_out, d_out_inf, xyzz_out, st);
    KZGX_TRY_HIP(hipGetLastError());
    return KZGX_OK;
  }
  {
    ProfScope p(ctx, st, "msm_reduce");
    fixed_reduce_launch<C>(ws.fpart, T, (uint32_t)batch, ws.fsum, st);
    fixed_finish_launch<C>(ws.fsum, (uint32_t)batch, d_out, d_out_inf, xyzz_out, st);
  }
  KZGX_TRY_HIP(hipGetLastError());
  return KZGX_OK;
}

#endif  // KZGX_FIXED_INST
}  // namespace kzgx
