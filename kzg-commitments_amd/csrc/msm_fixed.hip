// Fixed-base G1 MSM with a precomputed table of signed-digit multiples
// (Brickell-Gordon-McCurley-Wilson style) for gfx950 -- the fast path behind
// kzg::trusted_setup::create_commit / create_proof / verify_commit when the
// SRS prefix is small enough to precompute
// (reference: trusted_setup::polyeval_G1, src/trusted_setup.cpp:149-174, a
// naive per-term PAIR_G1mul + ECP_add loop).
//
// The SRS is fixed for the lifetime of a trusted_setup, so the work that
// does not depend on the scalars is paid once, at setup time:
//
//   M[w][i][j] = (j + 1) 2^(c w) P_i      w < W, i < n_t, j < H = 2^(c-1)
// stored window-major, or point-major for small c (TabStrides, fixed_accum.hpp)
//
// stored affine, Montgomery form (64-B packed words on BN254, 112-B radix-2^29
// limbs on BLS12-381, see fixed_l29).  A scalar s_i with signed c-bit digits
// d_w (|d_w| <= H) then
// contributes sum_w sign(d_w) M[w][i][|d_w| - 1], so an MSM is a plain sum
// of n W table points: no bucket sort, no bucket reduction, no doublings.
// Each thread sums the W terms of ~P points into one XYZZ accumulator with
// mixed additions (the only heavy instruction stream: 8M + 2S per term, the
// table lookup for the next term in flight underneath), one wavefront per
// MSM folds the partials, and one thread per MSM converts to affine.
//
// Size: W n_t H points; BN254 c = 17 (W = 15) for the 4097-point prefix of
// the degree-4096 benchmark is 257.8 GB -- sized for the 288 GB of HBM3E.
// Every step is an exact group operation, so the affine output is bit-exact
// with any other correct evaluation of sum c_i [tau^i]G1.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "curve.hpp"
#include "fixed_accum.hpp"
#include "kzgx_internal.hpp"
#include "kzgx_setup.hpp"

namespace kzgx {

int fixed_windows(int curve, int c) {  // FixedWin<C, c>::W (regular odd digits)
  const int bits = curve == KZGX_CURVE_BN254 ? BN254G1::SCALAR_BITS : BLS12381G1::SCALAR_BITS;
  return (bits + c - 1) / c;
}

// --------------------------------------------------------------------------
// table construction (setup time)
// --------------------------------------------------------------------------
// window bases B[w][i] = 2^(c w) P_i, packed; thread per SRS point
template <class C>
__global__ __launch_bounds__(64) void k_fixed_bases(const uint32_t* __restrict__ canon, uint32_t n, int W, int c,
                                                    uint32_t* __restrict__ bases, uint8_t* __restrict__ inf) {
  constexpr int PW = packed_words<C>();
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Affine<C> a;
  const bool finite = affine_from_canonical<C>(canon + (size_t)i * 2 * C::Fp::N, a);
  inf[i] = finite ? 0 : 1;
  for (int w = 0; w < W; w++) {
    packed_store<C>(bases + ((size_t)w * n + i) * PW, a);
    if (finite && w + 1 < W) {
      Xyzz<C> p = xyzz_from_affine<C>(a);
      for (int s = 0; s < c; s++) p = xyzz_dbl<C>(p);
      xyzz_to_affine<C>(p, a);  // 2^(cw) P_i != O: P_i has order r > 2^(cw)
    }
  }
}

// the same bases from the Pippenger window table when it has the fixed
// table's window (T[w][i] = 2^(c w) P_i, msm.hip k_table_build): a copy into
// the packed layout instead of each point's chain of c (W - 1) doublings and
// W - 1 inversions (2.4 ms for any SRS size, latency-bound)
template <class C>
__global__ __launch_bounds__(256) void k_fixed_bases_from_table(const uint32_t* __restrict__ table,
                                                                const uint8_t* __restrict__ inf_src, uint32_t n,
                                                                uint32_t n_rows, int W, uint32_t* __restrict__ bases,
                                                                uint8_t* __restrict__ inf) {
  constexpr int PW = packed_words<C>();
  constexpr int AW = affine_words<C>();
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= (uint64_t)W * n) return;
  const uint32_t w = (uint32_t)(g / n), i = (uint32_t)(g % n);
  packed_store<C>(bases + g * PW, affine_load<C>(table + ((size_t)w * n_rows + i) * AW));
  if (w == 0) inf[i] = inf_src[i];
}

// M(w, i, j0 + j) = (2 (j0 + j) + 1) B[w][i], j < J (the odd multiples the
// regular odd digits index, fixed_accum.hpp); thread per (w, i, block),
// written at the table's strides (TabStrides)
template <class C>
__global__ __launch_bounds__(64) void k_fixed_multiples(const uint32_t* __restrict__ bases,
                                                        const uint8_t* __restrict__ inf, uint32_t n, int W, uint32_t H,
                                                        uint32_t J, uint64_t g0, uint64_t cnt, TabStrides ts,
                                                        uint32_t* __restrict__ tab) {
  constexpr int PW = packed_words<C>();
  const uint64_t gl = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t nblk = H / J;
  if (gl >= cnt) return;
  const uint64_t g = g0 + gl;  // < W n nblk
  const uint32_t blk = (uint32_t)(g % nblk);
  const uint64_t wi = g / nblk;  // w * n + i
  const uint32_t i = (uint32_t)(wi % n);
  const uint32_t w = (uint32_t)(wi / n);
  uint32_t* out = tab + (uint64_t)i * ts.is + (uint64_t)w * ts.ws + (uint64_t)blk * J * PW;
  if (inf[i]) {  // never read: the MSM skips infinite SRS points
    for (uint32_t j = 0; j < J * PW; j++) out[j] = 0;
    return;
  }
  const Affine<C> B = packed_load<C>(bases + wi * PW);
  Affine<C> B2;  // 2 B (!= O: B has order r > 2)
  xyzz_to_affine<C>(xyzz_dbl<C>(xyzz_from_affine<C>(B)), B2);
  const uint32_t k0 = 2 * blk * J + 1;
  // acc = k0 B, left-to-right double-and-add
  Xyzz<C> acc = xyzz_from_affine<C>(B);
  for (int bit = 30 - __builtin_clz(k0); bit >= 0; bit--) {
    acc = xyzz_dbl<C>(acc);
    if ((k0 >> bit) & 1u) acc = xyzz_add_affine<C>(acc, B);
  }
  for (uint32_t j = 0; j < J; j++) {
    if (j) acc = xyzz_add_affine<C>(acc, B2);
    Affine<C> a;
    xyzz_to_affine<C>(acc, a);  // (k0 + 2 j) B != O since k0 + 2 j < 2 H <= 2^17 < r
    packed_store<C>(out + (size_t)j * PW, a);
  }
}

// one wavefront per MSM: strided sums of the T partials, then a shuffle tree
template <class C>
__global__ __launch_bounds__(256) void k_fixed_reduce(const uint32_t* __restrict__ part, uint32_t T, uint32_t batch,
                                                      uint32_t* __restrict__ sums) {
  constexpr int XW = xyzz_words<C>();
  constexpr int L = C::Fp29::L;
  const uint32_t b = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
  const uint32_t lane = threadIdx.x & 63;
  if (b >= batch) return;  // whole wavefronts
  Xyzz<C> acc = xyzz_inf<C>();
  for (uint32_t k = lane; k < T; k += 64) acc = xyzz_add_impl<C>(acc, xyzz_load<C>(part + ((size_t)b * T + k) * XW));
  for (int off = 32; off >= 1; off >>= 1) {
    Xyzz<C> o;
#pragma unroll
    for (int k = 0; k < L; k++) {
      o.X.v[k] = __shfl_down(acc.X.v[k], off, 64);
      o.Y.v[k] = __shfl_down(acc.Y.v[k], off, 64);
      o.ZZ.v[k] = __shfl_down(acc.ZZ.v[k], off, 64);
      o.ZZZ.v[k] = __shfl_down(acc.ZZZ.v[k], off, 64);
    }
    acc = xyzz_add_impl<C>(acc, o);
  }
  if (lane == 0) xyzz_store<C>(sums + (size_t)b * XW, acc);
}

// thread per MSM: XYZZ -> canonical affine + infinity flag, or copy the XYZZ
// point out (chunked callers sum partials themselves)
template <class C>
__global__ __launch_bounds__(64) void k_fixed_finish(const uint32_t* __restrict__ sums, uint32_t batch,
                                                     uint32_t* __restrict__ out, uint32_t* __restrict__ out_inf,
                                                     uint32_t* __restrict__ xyzz_out) {
  constexpr int XW = xyzz_words<C>();
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= batch) return;
  const Xyzz<C> p = xyzz_load<C>(sums + (size_t)b * XW);
  if (xyzz_out) {
    xyzz_store<C>(xyzz_out + (size_t)b * XW, p);
    return;
  }
  Affine<C> a;
  const bool fin = xyzz_to_affine<C>(p, a);
  affine_to_canonical<C>(out + (size_t)b * 2 * C::Fp::N, a, fin);
  out_inf[b] = fin ? 0u : 1u;
}

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
  Affine<C> a;
  const bool fin = xyzz_to_affine_lane<C>(s, a);
  if (lane == 0) {
    affine_to_canonical<C>(out + (size_t)b * 2 * C::Fp::N, a, fin);
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
// during the addition of the current one, and the wavefront folds its 64
// partials with 6 shuffle additions before one lane stores (the first 64:1
// level of the reduction, without a launch).
// --------------------------------------------------------------------------
template <class C, int CB>
__global__ __launch_bounds__(64, fixed_accum_waves<C>()) void k_fixed_accum_flat(
    const uint32_t* __restrict__ scalars, uint32_t n, size_t stride_words, const uint32_t* __restrict__ tab,
    TabStrides ts, const uint8_t* __restrict__ inf, uint32_t Q, uint32_t T, uint32_t* __restrict__ part) {
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
#pragma unroll 1
  for (int off = 32; off >= 1; off >>= 1) acc = xyzz_shfl_xor_add<C>(acc, off);
  if (threadIdx.x == 0) xyzz_store<C>(part + ((size_t)b * (T / 64) + t / 64) * XW, acc);
}

// --------------------------------------------------------------------------
// host side
// --------------------------------------------------------------------------
constexpr uint32_t FIXED_J = 16;  // multiples per table-build thread

// Table layout (TabStrides): point-major for c <= KZGX_FIXED_PM_MAX_C (the
// few-large-MSM tables, walked point by point by k_fixed_accum_flat),
// window-major above (profiles/r03_cfg5_table_layout.json,
// r03_ab_point_major_cfg2.json).  kzgx_set_fixed_base_layout or
// KZGX_FIXED_POINT_MAJOR=0/1 force one.
#ifndef KZGX_FIXED_PM_MAX_C
#define KZGX_FIXED_PM_MAX_C 12
#endif
static bool fixed_point_major(int c, int layout_req) {
  // an explicit kzgx_set_fixed_base_layout(0/1) wins; the environment knob
  // (A/B runs) only overrides the automatic choice
  if (layout_req >= 0) return layout_req != 0;
  static const char* e = std::getenv("KZGX_FIXED_POINT_MAJOR");
  if (e && *e) return std::atoi(e) != 0;
  return c <= KZGX_FIXED_PM_MAX_C;
}

template <class C>
static TabStrides fixed_strides(bool point_major, int W, size_t n, uint64_t H) {
  constexpr size_t PW = packed_words<C>();
  if (point_major) return TabStrides{(size_t)W * H * PW, H * PW};
  return TabStrides{H * PW, n * H * PW};
}

template <class C>
static TabStrides tab_strides(const FixedTable& ft) {
  return fixed_strides<C>(ft.point_major, ft.W, ft.n_t, 1ull << (ft.c - 1));
}

// the infinity flags the accumulation kernels read, or null when none is set
static const uint8_t* fixed_inf(const FixedTable& ft) { return ft.any_inf ? ft.inf : nullptr; }

// the per-device cached table block (kzgx_api.hip)
hipError_t table_malloc(void** p, size_t bytes);
void table_free(void* p, size_t bytes);

template <class C>
static int fixed_build_impl(Ctx* ctx, FixedTable& ft, const uint32_t* d_canon, size_t n) {
  const int c = ft.c_req;
  const int W = fixed_windows(ctx->curve, c);
  const uint64_t H = 1ull << (c - 1);
  const size_t PB = packed_words<C>() * sizeof(uint32_t);
  const size_t bytes = (size_t)W * n * H * PB;
  // drop the old table (and its infinity flags) first: the new one may need
  // most of the device
  if (ft.d || ft.inf) {
    KZGX_TRY_HIP(hipDeviceSynchronize());
    fixed_free_table(ft);
  }
  // any failure below leaves no table (and no half-built allocation) behind
  struct Guard {
    FixedTable& ft;
    uint32_t* bases = nullptr;
    uint8_t* inf = nullptr;
    bool ok = false;
    ~Guard() {
      if (bases) (void)hipFree(bases);
      if (!ok) {
        if (inf) (void)hipFree(inf);
        fixed_free_table(ft);
      }
    }
  } g{ft};
  KZGX_TRY_HIP(table_malloc((void**)&ft.d, bytes));
  ft.bytes = bytes;
  KZGX_TRY_HIP(hipMalloc((void**)&g.bases, (size_t)W * n * PB));
  KZGX_TRY_HIP(hipMalloc((void**)&g.inf, n));
  uint32_t* d_bases = g.bases;
  uint8_t* d_inf = g.inf;
  hipStream_t st = ctx->stream;
  if (ctx->d_table && ctx->c == c && W <= ctx->W && n <= ctx->n_srs)
    hipLaunchKernelGGL(k_fixed_bases_from_table<C>, dim3((unsigned)(((uint64_t)W * n + 255) / 256)), dim3(256), 0, st,
                       ctx->d_table, ctx->d_inf, (uint32_t)n, (uint32_t)ctx->n_srs, W, d_bases, d_inf);
  else
    hipLaunchKernelGGL(k_fixed_bases<C>, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, st, d_canon, (uint32_t)n, W, c,
                       d_bases, d_inf);
  ft.point_major = fixed_point_major(c, ft.layout_req);
  const TabStrides ts = fixed_strides<C>(ft.point_major, W, n, H);
  // KZGX_TABLE_BUILD_SERIAL=1: the round-4 builder (one inversion per entry),
  // for A/B runs of the batch-affine one (setup.hip)
  static const bool serial = std::getenv("KZGX_TABLE_BUILD_SERIAL") && std::getenv("KZGX_TABLE_BUILD_SERIAL")[0] == '1';
  if (!serial) {
    ProfScope p(ctx, st, "fixed_build");
    KZGX_TRY(fixed_multiples_batch(ctx->curve, d_bases, d_inf, (uint32_t)n, W, (uint32_t)H, ts.is, ts.ws, ft.d, st));
  } else {
    const uint32_t J = (uint32_t)(H < FIXED_J ? H : FIXED_J);
    const uint64_t tasks = (uint64_t)W * n * (H / J);
    // bounded launches of <= 2^22 threads each, synchronised per slice so one
    // setup never queues seconds of work behind a single dispatch
    const uint64_t slice = 1ull << 22;
    for (uint64_t s0 = 0; s0 < tasks; s0 += slice) {
      const uint64_t cnt = tasks - s0 < slice ? tasks - s0 : slice;
      {
        ProfScope p(ctx, st, "fixed_build");
        hipLaunchKernelGGL(k_fixed_multiples<C>, dim3((unsigned)((cnt + 63) / 64)), dim3(64), 0, st, d_bases, d_inf,
                           (uint32_t)n, W, (uint32_t)H, J, s0, cnt, ts, ft.d);
      }
      KZGX_TRY_HIP(hipGetLastError());
      KZGX_TRY_HIP(hipStreamSynchronize(st));
    }
  }
  // whether any SRS point of the prefix is infinite: when none is (every SRS
  // but a degenerate tau = 0 one), the accumulation kernels get no flag array
  // and read no flag per point
  {
    std::vector<uint8_t> h(n);
    KZGX_TRY_HIP(hipMemcpyAsync(h.data(), d_inf, n, hipMemcpyDeviceToHost, st));
    KZGX_TRY_HIP(hipStreamSynchronize(st));
    ft.any_inf = std::any_of(h.begin(), h.end(), [](uint8_t v) { return v != 0; });
    const auto f = std::find(h.begin(), h.end(), (uint8_t)0);
    ft.fin0 = f == h.end() ? UINT32_MAX : (uint32_t)(f - h.begin());
  }
  g.ok = true;
  ft.inf = d_inf;
  ft.c = c;
  ft.W = W;
  ft.n_t = n;
  return KZGX_OK;
}

int fixed_build_table(Ctx* ctx, FixedTable& ft, const uint32_t* d_canon, size_t n_srs) {
  if (ft.c_req == 0 || ft.n_req == 0) return KZGX_OK;
  const size_t n = ft.n_req < n_srs ? ft.n_req : n_srs;
  return ctx->curve == KZGX_CURVE_BN254 ? fixed_build_impl<BN254G1>(ctx, ft, d_canon, n)
                                        : fixed_build_impl<BLS12381G1>(ctx, ft, d_canon, n);
}

// the default table: a fixed window, or (c_req < 0) the widest c <= 12 whose
// table fits KZGX_DEFAULT_TABLE_PERMILLE of the device memory and the free
// memory less 4 GiB; none if even c = 7 does not
static int fixed_build_default(Ctx* ctx, const uint32_t* d_canon, size_t n_srs) {
  FixedTable& ft = ctx->fixed_def;
  if (ft.c_req >= 0) return fixed_build_table(ctx, ft, d_canon, n_srs);
  if (ft.n_req == 0) return KZGX_OK;
  fixed_free_table(ft);  // its memory counts as free for the choice
  const size_t n = ft.n_req < n_srs ? ft.n_req : n_srs;
  size_t free_b = 0, total_b = 0;
  KZGX_TRY_HIP(hipMemGetInfo(&free_b, &total_b));
  const size_t margin = (size_t)4 << 30;
  size_t budget = total_b / 1000 * KZGX_DEFAULT_TABLE_PERMILLE;
  if (free_b < margin) return KZGX_OK;
  if (budget > free_b - margin) budget = free_b - margin;
  for (int c = 12; c >= 7; c--) {
    if (fixed_table_bytes(ctx->curve, c, n) > budget) continue;
    ft.c_req = c;
    const int rc = fixed_build_table(ctx, ft, d_canon, n_srs);
    ft.c_req = -1;  // the next SRS picks again
    return rc == KZGX_ERR_OOM ? KZGX_OK : rc;  // no room after all: no default table
  }
  return KZGX_OK;
}

int fixed_build(Ctx* ctx, const uint32_t* d_canon, size_t n_srs) {
  KZGX_TRY(fixed_build_table(ctx, ctx->fixed, d_canon, n_srs));
  // the default table is an acceleration cache: if it cannot be built (any
  // status) the SRS stays loaded and the MSMs take Pippenger
  if (fixed_build_default(ctx, d_canon, n_srs) != KZGX_OK) {
    (void)hipGetLastError();
    (void)hipStreamSynchronize(ctx->stream);
    fixed_free_table(ctx->fixed_def);
  }
  return KZGX_OK;
}

int fixed_rebuild_default(Ctx* ctx, const uint32_t* d_canon, size_t n_srs) {
  return fixed_build_default(ctx, d_canon, n_srs);
}

void fixed_free(Ctx* ctx) { fixed_free_table(ctx->fixed); }

void fixed_free_table(FixedTable& ft) {
  if (ft.d) table_free(ft.d, ft.bytes);
  if (ft.inf) (void)hipFree(ft.inf);
  ft.d = nullptr;
  ft.inf = nullptr;
  ft.bytes = 0;
  ft.n_t = 0;
  ft.c = 0;
  ft.fin0 = UINT32_MAX;
}

template <class C, int CB>
static int fixed_msm_impl(Ctx* ctx, FixedTable& ft, const uint32_t* d_scalars, size_t n, size_t batch,
                          size_t stride_words, uint32_t* d_out, uint32_t* d_out_inf, hipStream_t st,
                          uint32_t* xyzz_out) {
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
    if (batch <= 16 && !xyzz_out && ft.pts_per_thread == 0 && !flat_off && terms * batch >= 8 * kSlots) {
      // KZGX_FLAT_TMULT: threads per resident-lane slot (A/B)
      static const size_t tmult = std::getenv("KZGX_FLAT_TMULT") ? std::strtoul(std::getenv("KZGX_FLAT_TMULT"), nullptr, 10) : 1;
      const uint32_t T = (uint32_t)std::max<size_t>(4096, kSlots * (tmult ? tmult : 1) / batch / 4096 * 4096);
      const uint32_t Q = (uint32_t)((terms + T - 1) / T);
      WsLease wsp = ctx->ws_for(st);
      if (!wsp) return KZGX_ERR_ARG;
      MsmWs& ws = *wsp;
      KZGX_TRY(dev_alloc(ctx, (void**)&ws.fpart, batch * (T / 64) * XB, &ws.fpart_b));
      KZGX_TRY(dev_alloc(ctx, (void**)&ws.fsum, batch * (T / 4096) * XB, &ws.fsum_b));
      {
        ProfScope p(ctx, st, "msm_accum");
        hipLaunchKernelGGL((k_fixed_accum_flat<C, CB>), dim3(T / 64, (unsigned)batch), dim3(64), 0, st, d_scalars,
                           (uint32_t)n, stride_words, ft.d, tab_strides<C>(ft), fixed_inf(ft), Q, T, ws.fpart);
      }
      ProfScope p(ctx, st, "msm_reduce");
      // T / 64 wavefront partials per MSM: one more 64:1 level, then one
      // wavefront per MSM over the T / 4096 left, then a thread per MSM
      const size_t g2 = batch * (T / 4096);
      hipLaunchKernelGGL(k_fixed_reduce<C>, dim3((unsigned)((g2 + 3) / 4)), dim3(256), 0, st, ws.fpart, 64u,
                         (uint32_t)g2, ws.fsum);
      hipLaunchKernelGGL(k_fixed_reduce<C>, dim3((unsigned)((batch + 3) / 4)), dim3(256), 0, st, ws.fsum,
                         T / 4096, (uint32_t)batch, ws.fpart);
      hipLaunchKernelGGL(k_fixed_finish<C>, dim3((unsigned)((batch + 63) / 64)), dim3(64), 0, st, ws.fpart,
                         (uint32_t)batch, d_out, d_out_inf, nullptr);
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
  const bool wave_red = batch <= 16 && T > 1024 && !xyzz_out;
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
    hipLaunchKernelGGL(k_fixed_reduce<C>, dim3((unsigned)((g1 + 3) / 4)), dim3(256), 0, st, ws.fpart, 64u,
                       (uint32_t)g1, ws.fsum);
    const uint32_t* lvl = ws.fsum;
    size_t per = T / 64;
    if (per > 128) {  // level 2: 64:1 back into fpart (T is a multiple of 64^2 here)
      const size_t g2 = batch * (T / 4096);
      hipLaunchKernelGGL(k_fixed_reduce<C>, dim3((unsigned)((g2 + 3) / 4)), dim3(256), 0, st, ws.fsum, 64u,
                         (uint32_t)g2, ws.fpart);
      lvl = ws.fpart;
      per = T / 4096;
    }
    // last level: one wavefront per MSM over its `per` partials, into the
    // buffer the last level did not read, then a thread per MSM converts
    uint32_t* fin = lvl == ws.fsum ? ws.fpart : ws.fsum;
    hipLaunchKernelGGL(k_fixed_reduce<C>, dim3((unsigned)((batch + 3) / 4)), dim3(256), 0, st, lvl, (uint32_t)per,
                       (uint32_t)batch, fin);
    hipLaunchKernelGGL(k_fixed_finish<C>, dim3((unsigned)((batch + 63) / 64)), dim3(64), 0, st, fin,
                       (uint32_t)batch, d_out, d_out_inf, nullptr);
    KZGX_TRY_HIP(hipGetLastError());
    return KZGX_OK;
  }
  {
    ProfScope p(ctx, st, "msm_reduce");
    hipLaunchKernelGGL(k_fixed_reduce<C>, dim3((unsigned)((batch + 3) / 4)), dim3(256), 0, st, ws.fpart, T,
                       (uint32_t)batch, ws.fsum);
    hipLaunchKernelGGL(k_fixed_finish<C>, dim3((unsigned)((batch + 63) / 64)), dim3(64), 0, st, ws.fsum,
                       (uint32_t)batch, d_out, d_out_inf, xyzz_out);
  }
  KZGX_TRY_HIP(hipGetLastError());
  return KZGX_OK;
}

template <class C>
static int fixed_msm_c(Ctx* ctx, FixedTable& ft, const uint32_t* d_scalars, size_t n, size_t batch,
                       size_t stride_words, uint32_t* d_out, uint32_t* d_out_inf, hipStream_t st, uint32_t* xyzz_out) {
  switch (ft.c) {
#define KZGX_FIXED_CASE(cb) \
  case cb: return fixed_msm_impl<C, cb>(ctx, ft, d_scalars, n, batch, stride_words, d_out, d_out_inf, st, xyzz_out);
    KZGX_FIXED_CASE(4)
    KZGX_FIXED_CASE(7)
    KZGX_FIXED_CASE(8)
    KZGX_FIXED_CASE(9)
    KZGX_FIXED_CASE(10)
    KZGX_FIXED_CASE(11)
    KZGX_FIXED_CASE(12)
    KZGX_FIXED_CASE(13)
    KZGX_FIXED_CASE(14)
    KZGX_FIXED_CASE(15)
    KZGX_FIXED_CASE(16)
    KZGX_FIXED_CASE(17)
#undef KZGX_FIXED_CASE
    default: return KZGX_ERR_INTERNAL;
  }
}

size_t fixed_table_bytes(int curve, int c, size_t n) {
  if (c <= 0) return 0;
  const size_t pb = curve == KZGX_CURVE_BN254 ? packed_words<BN254G1>() * 4 : packed_words<BLS12381G1>() * 4;
  return (size_t)fixed_windows(curve, c) * n * ((size_t)1 << (c - 1)) * pb;
}

bool fixed_bits_supported(int c) {
  return c == 0 || c == 4 || (c >= 7 && c <= 17);
}

// (a prefix of infinite points only -- a loaded all-infinity SRS -- has no
// finite point to carry the identity terms of k_fixed_accum: Pippenger)
bool fixed_table_usable(const FixedTable& ft, size_t n) {
  return ft.d && ft.n_t > 0 && n <= ft.n_t && ft.fin0 != UINT32_MAX;
}
bool fixed_usable(const Ctx* ctx, size_t n) { return fixed_table_usable(ctx->fixed, n); }

int fixed_msm_table(Ctx* ctx, FixedTable& ft, const uint32_t* d_scalars, size_t n, size_t batch, size_t stride_words,
                    uint32_t* d_out, uint32_t* d_out_inf, hipStream_t st, uint32_t* xyzz_out) {
  return ctx->curve == KZGX_CURVE_BN254
             ? fixed_msm_c<BN254G1>(ctx, ft, d_scalars, n, batch, stride_words, d_out, d_out_inf, st, xyzz_out)
             : fixed_msm_c<BLS12381G1>(ctx, ft, d_scalars, n, batch, stride_words, d_out, d_out_inf, st, xyzz_out);
}

int fixed_msm(Ctx* ctx, const uint32_t* d_scalars, size_t n, size_t batch, size_t stride_words, uint32_t* d_out,
              uint32_t* d_out_inf, hipStream_t st, uint32_t* xyzz_out) {
  return fixed_msm_table(ctx, ctx->fixed, d_scalars, n, batch, stride_words, d_out, d_out_inf, st, xyzz_out);
}

// --------------------------------------------------------------------------
// measured VALU peak of the accumulation loop (the denominator of the bench's
// valu_roofline): k_fixed_accum's inlined XYZZ mixed addition, with the same
// launch bounds (waves per SIMD), over operands that stay in L1 (a 64-point
// table: no HBM stream, no digit logic), whole GPU, ITER additions per thread
// --------------------------------------------------------------------------
template <class C>
__global__ __launch_bounds__(64, fixed_accum_waves<C>()) void k_microbench_madd(const uint32_t* __restrict__ pts,
                                                                                uint32_t iters,
                                                                                uint32_t* __restrict__ sink) {
  constexpr int PW = affine_words<C>();
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  Xyzz<C> acc = xyzz_from_affine<C>(affine_load<C>(pts + (size_t)(t & 63) * PW));
#pragma unroll 1
  for (uint32_t k = 0; k < iters; k++) {
    Affine<C> a = affine_load<C>(pts + (size_t)((t + 1 + k) & 63) * PW);
    acc = xyzz_add_affine_impl<C>(acc, a);
  }
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < C::Fp29::L; i++) o ^= acc.X.v[i] ^ acc.ZZ.v[i];
  if (o == 0x9e3779b9u) sink[t] = o;  // keeps the chain live; practically never stores
}

// mixed additions per second: 64 distinct multiples of the SRS's first point
// (built with the table kernels' own arithmetic), then a timed launch
template <class C>
static int microbench_madd_impl(Ctx* ctx, double* rate) {
  if (ctx->n_srs == 0) return KZGX_ERR_NO_SRS;
  constexpr int PW = affine_words<C>();
  hipStream_t st = ctx->stream;
  uint32_t *d_pts = nullptr, *d_sink = nullptr;
  const uint32_t waves = 256 * 4 * fixed_accum_waves<C>() * 4;  // four full residencies
  const uint32_t iters = 192;
  KZGX_TRY_HIP(hipMalloc((void**)&d_pts, 64 * PW * 4));
  struct Free {
    uint32_t** a;
    uint32_t** b;
    ~Free() {
      if (*a) (void)hipFree(*a);
      if (*b) (void)hipFree(*b);
    }
  } fr{&d_pts, &d_sink};
  KZGX_TRY_HIP(hipMalloc((void**)&d_sink, (size_t)waves * 64 * 4));
  // T[0][i] holds the SRS points in the 80 / 112 B radix-2^29 layout; the
  // first 64 points (or repeats of them) are distinct curve points
  for (uint32_t i = 0; i < 64; i++)
    KZGX_TRY_HIP(hipMemcpyAsync(d_pts + (size_t)i * PW, ctx->d_table + (size_t)(i % ctx->n_srs) * PW, PW * 4,
                                hipMemcpyDeviceToDevice, st));
  hipLaunchKernelGGL(k_microbench_madd<C>, dim3(waves), dim3(64), 0, st, d_pts, 8u, d_sink);  // warm
  hipEvent_t a, b;
  KZGX_TRY_HIP(hipEventCreate(&a));
  KZGX_TRY_HIP(hipEventCreate(&b));
  KZGX_TRY_HIP(hipEventRecord(a, st));
  hipLaunchKernelGGL(k_microbench_madd<C>, dim3(waves), dim3(64), 0, st, d_pts, iters, d_sink);
  KZGX_TRY_HIP(hipEventRecord(b, st));
  KZGX_TRY_HIP(hipEventSynchronize(b));
  float ms = 0;
  hipError_t e = hipEventElapsedTime(&ms, a, b);
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  KZGX_TRY_HIP(e);
  KZGX_TRY_HIP(hipGetLastError());
  *rate = (double)waves * 64 * iters / (ms * 1e-3);
  return KZGX_OK;
}

// v_mad_u64_u32 issue ceiling: 8 independent accumulator chains per lane,
// 256 mads per chain per iteration, 8 waves per SIMD (the instruction
// exactly, in asm; scripts/micro_valu.hip, profiles/r01_micro_valu.txt)
__global__ __launch_bounds__(256) void k_microbench_mad64(uint32_t iters, uint32_t* __restrict__ sink,
                                                          uint64_t* __restrict__ stamp) {
  // block 0's first lane counts core clocks against the constant-rate wall
  // clock over its run: every block is resident at once, so that is the
  // clock the ceiling was measured at
  uint64_t w0 = 0, c0 = 0;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    w0 = wall_clock64();
    c0 = clock64();
  }
  uint64_t acc[8];
  const uint32_t a = threadIdx.x + 1, b = blockIdx.x + 3;
#pragma unroll
  for (int k = 0; k < 8; k++) acc[k] = k;
#pragma unroll 1
  for (uint32_t it = 0; it < iters; it++) {
#pragma unroll
    for (int r = 0; r < 32; r++) {
#pragma unroll
      for (int k = 0; k < 8; k++) {
        uint64_t sc;
        asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc[k]), "=s"(sc) : "v"(a), "v"(b));
      }
    }
  }
  uint64_t o = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) o ^= acc[k];
  if ((uint32_t)o == 0x9e3779b9u) sink[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)o;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    const uint64_t c1 = clock64(), w1 = wall_clock64();
    stamp[0] = c1 - c0;
    stamp[1] = w1 - w0;
  }
}

int microbench_mad_u64(Ctx* ctx, double* rate, double* ghz) {
  hipStream_t st = ctx->stream;
  const uint32_t blocks = 256 * 8, iters = 64;
  uint32_t* d_sink = nullptr;
  KZGX_TRY_HIP(hipMalloc((void**)&d_sink, (size_t)blocks * 256 * 4 + 16));
  uint64_t* d_stamp = reinterpret_cast<uint64_t*>(d_sink + (size_t)blocks * 256);
  hipLaunchKernelGGL(k_microbench_mad64, dim3(blocks), dim3(256), 0, st, 2u, d_sink, d_stamp);  // warm
  hipEvent_t a, b;
  KZGX_TRY_HIP(hipEventCreate(&a));
  KZGX_TRY_HIP(hipEventCreate(&b));
  KZGX_TRY_HIP(hipEventRecord(a, st));
  hipLaunchKernelGGL(k_microbench_mad64, dim3(blocks), dim3(256), 0, st, iters, d_sink, d_stamp);
  KZGX_TRY_HIP(hipEventRecord(b, st));
  KZGX_TRY_HIP(hipEventSynchronize(b));
  float ms = 0;
  hipError_t e = hipEventElapsedTime(&ms, a, b);
  uint64_t h[2] = {0, 0};
  if (e == hipSuccess) e = hipMemcpy(h, d_stamp, sizeof h, hipMemcpyDeviceToHost);
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  (void)hipFree(d_sink);
  KZGX_TRY_HIP(e);
  KZGX_TRY_HIP(hipGetLastError());
  *rate = (double)blocks * 256 * iters * 256 / (ms * 1e-3);
  if (ghz) {
    int khz = 0;
    KZGX_TRY_HIP(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, ctx->device));
    *ghz = h[1] ? (double)h[0] / (double)h[1] * khz * 1e-6 : 0.0;
  }
  return KZGX_OK;
}

// The core clock while other work runs: one lane spins for spin_us of the
// constant-rate wall clock and counts core clocks meanwhile.  The DVFS clock
// is one per device (MI355X_MICROARCH.md, DVFS give-back), so a probe
// resident beside a kernel reads that kernel's clock; it holds one wave slot.
// out: core clocks, wall ticks, wall clock rate in kHz.
__global__ __launch_bounds__(64) void k_clock_probe(uint64_t ticks, uint32_t khz, uint64_t* __restrict__ out) {
  if (threadIdx.x != 0) return;
  const uint64_t w0 = wall_clock64(), c0 = clock64();
  uint64_t w = w0;
  while (w - w0 < ticks) w = wall_clock64();
  const uint64_t c1 = clock64();
  out[0] = c1 - c0;
  out[1] = w - w0;
  out[2] = khz;
}

int clock_probe(Ctx* ctx, hipStream_t st, uint32_t spin_us, uint64_t* d_out) {
  int khz = 0;
  KZGX_TRY_HIP(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, ctx->device));
  const uint64_t ticks = (uint64_t)spin_us * (uint64_t)khz / 1000;
  hipLaunchKernelGGL(k_clock_probe, dim3(1), dim3(64), 0, st ? st : ctx->stream, ticks, (uint32_t)khz, d_out);
  KZGX_TRY_HIP(hipGetLastError());
  return KZGX_OK;
}

int microbench_mixed_add(Ctx* ctx, double* rate) {
  return ctx->curve == KZGX_CURVE_BN254 ? microbench_madd_impl<BN254G1>(ctx, rate)
                                        : microbench_madd_impl<BLS12381G1>(ctx, rate);
}

// --------------------------------------------------------------------------
// single-lane latency of the primitives on the latency-bound tails (the
// finish kernels and the last reduction levels of one MSM): a dependent chain
// of ITER operations in one lane of one wavefront, timed with the shader's
// constant-rate wall clock and its core-clock counter inside the kernel
// (no launch overhead).  op: 0 Montgomery product, 1 Fermat inversion,
// 2 binary-Euclid inversion, 3 XYZZ addition, 4 mixed addition, 5 XYZZ ->
// affine conversion, 6 / 7 the same as 2 / 5 on the scalar ALU (one lane's
// value made wave-uniform), 8 / 9 the same with the whole wavefront active
// (the linear combinations one per lane).
// --------------------------------------------------------------------------
template <class C>
__global__ __launch_bounds__(64) void k_debug_latency(const uint32_t* __restrict__ pts, int op, uint32_t iters,
                                                      uint64_t* __restrict__ out) {
  using F = typename C::Fp29;
  constexpr int PW = affine_words<C>();
  if (threadIdx.x != 0 && op < 8) return;  // 8, 9: the whole wavefront on one value
  const Affine<C> p = affine_load<C>(pts), q = affine_load<C>(pts + PW);
  F29<F> a = p.x;
  Xyzz<C> acc = xyzz_from_affine<C>(p);
  const Xyzz<C> qx = xyzz_add_affine_impl<C>(xyzz_from_affine<C>(q), q);  // 2q, Z != 1
  const uint64_t w0 = wall_clock64(), c0 = clock64();
#pragma unroll 1
  for (uint32_t k = 0; k < iters; k++) {
    if (op == 0) a = f29_mul<F>(a, p.y);
    else if (op == 1) a = f29_inv<F, C::Fp::N>(a, C::Fp::PM2);
    else if (op == 2) a = f29_inv_vt<F, C::Fp::N>(a, C::Fp::P);
    else if (op == 3) acc = xyzz_add_impl<C>(acc, qx);
    else if (op == 4) acc = xyzz_add_affine_impl<C>(acc, q);
    else if (op == 6 || op == 8) a = f29_inv_uniform<F, C::Fp::N>(a, C::Fp::P);
    else if (op == 7 || op == 9) {
      Affine<C> r;
      (void)xyzz_to_affine_impl<C, true>(acc, r);
      acc.X = r.y;
    } else {
      Affine<C> r;
      (void)xyzz_to_affine_impl<C>(acc, r);
      acc.X = r.y;  // next input depends on this output
    }
  }
  const uint64_t w1 = wall_clock64(), c1 = clock64();
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < F::L; i++) o ^= a.v[i] ^ acc.X.v[i] ^ acc.ZZ.v[i];
  if (threadIdx.x != 0) return;
  out[0] = w1 - w0;
  out[1] = c1 - c0;
  out[2] = o;
}

template <class C>
static int debug_latency_impl(Ctx* ctx, int op, uint32_t iters, double* res) {
  if (ctx->n_srs < 2) return KZGX_ERR_NO_SRS;
  constexpr int PW = affine_words<C>();
  hipStream_t st = ctx->stream;
  uint32_t* d_pts = nullptr;
  uint64_t* d_out = nullptr;
  KZGX_TRY_HIP(hipMalloc((void**)&d_pts, 2 * PW * 4));
  if (hipMalloc((void**)&d_out, 3 * 8) != hipSuccess) {
    (void)hipFree(d_pts);
    return KZGX_ERR_HIP;
  }
  (void)hipMemcpyAsync(d_pts, ctx->d_table, 2 * PW * 4, hipMemcpyDeviceToDevice, st);
  hipLaunchKernelGGL(k_debug_latency<C>, dim3(1), dim3(64), 0, st, d_pts, op, 1u, d_out);  // warm
  hipLaunchKernelGGL(k_debug_latency<C>, dim3(1), dim3(64), 0, st, d_pts, op, iters, d_out);
  uint64_t h[3] = {0, 0, 0};
  hipError_t e = hipMemcpyAsync(h, d_out, sizeof h, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  (void)hipFree(d_pts);
  (void)hipFree(d_out);
  KZGX_TRY_HIP(e);
  int khz = 0;
  KZGX_TRY_HIP(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, ctx->device));
  res[0] = (double)h[0] / iters / (khz * 1e3) * 1e9;  // ns per operation
  res[1] = (double)h[1] / iters;                      // core clocks per operation
  return KZGX_OK;
}

int debug_latency(Ctx* ctx, int op, uint32_t iters, double* res) {
  if (op < 0 || op > 9 || iters == 0) return KZGX_ERR_ARG;
  return ctx->curve == KZGX_CURVE_BN254 ? debug_latency_impl<BN254G1>(ctx, op, iters, res)
                                        : debug_latency_impl<BLS12381G1>(ctx, op, iters, res);
}

}  // namespace kzgx

namespace kzgx {
// device bring-up (kzgx_setup.hpp): one launch loads this code object
__global__ void k_warm_msm_fixed() {}
int warm_msm_fixed(hipStream_t st) {
  hipLaunchKernelGGL(k_warm_msm_fixed, dim3(1), dim3(64), 0, st);
  KZGX_TRY_HIP(hipGetLastError());
  return KZGX_OK;
}
}  // namespace kzgx
