// Lone-wave kernels outside the verify path: work that is one dependent
// chain on one wave (the sharded commitment's fold, the bucket reduction of
// the wide-window Pippenger MSM).
//
// k_g1_fold_packed: the exact fold of the sharded commitment (BASELINE
// configs[4], python/kzgx_dist.py): the N ranks' partial points, all-gathered
// as packed records (x || y || infinity word), summed by one wave -- lane k
// takes record k (strided above 64), a shuffle tree adds the lanes' XYZZ
// sums, and the whole wave converts lane 0's total to affine with the
// wave-uniform inversion (f29_inv_uniform) -- written back as one packed
// record.  Replaces torch.stack / .to / .contiguous / torch.cat around the
// one-lane k_g1_sum ("What's weak" 4).
// This object must be compiled with memory clauses off (the Makefile's
// -mllvm -amdgpu-max-memory-clause=1, which also defines KZGX_MEMCLAUSE_OFF):
// with hipcc's default clause formation the inlined additions next to
// clause-formed loads give wrong sums
#ifndef KZGX_MEMCLAUSE_OFF
#error "latency.hip needs -mllvm -amdgpu-max-memory-clause=1 -DKZGX_MEMCLAUSE_OFF (see the Makefile)"
#endif
#include <hip/hip_runtime.h>

#include <cstdlib>

// The product form: the chained (throughput) form by default -- measured
// faster here than the latency-first f29_mul_lat (2^20 + 1 points 2.579 vs
// 2.603 ms, 131 073: 0.691 vs 0.724 ms, profiles/r05_big_msm_*): an XYZZ
// addition has enough independent products that one lane's chain of them
// is issue-bound either way.  KZGX_LATENCY_LAT selects f29_mul_lat (A/B).
#ifdef KZGX_LATENCY_LAT
#define KZGX_FIELD_LATENCY
#endif
#include "coop.hpp"
#include "msm_merge.hpp"
#include "curve.hpp"
#include "kzgx_internal.hpp"
#include "kzgx_setup.hpp"

namespace kzgx {

__global__ void k_warm_latency() {}
int warm_latency(hipStream_t st) {
  hipLaunchKernelGGL(k_warm_latency, dim3(1), dim3(64), 0, st);
  KZGX_TRY_HIP(hipGetLastError());
  return KZGX_OK;
}

// packed record: 2 N canonical words (x || y, little-endian 32-bit words)
// followed by a 64-bit infinity word (nonzero = infinity); stride 2 N + 2 words
template <class C>
__global__ __launch_bounds__(64) void k_g1_fold_packed(const uint32_t* __restrict__ rec, uint32_t count,
                                                       uint32_t* __restrict__ out) {
  constexpr int N = C::Fp::N, L = C::Fp29::L;
  constexpr int RW = 2 * N + 2;
  const uint32_t lane = threadIdx.x;
  Xyzz<C> acc = xyzz_inf<C>();
  for (uint32_t k = lane; k < count; k += 64) {
    const uint32_t* r = rec + (size_t)k * RW;
    Affine<C> a;
    const bool fin = affine_from_canonical<C>(r, a) && (r[2 * N] | r[2 * N + 1]) == 0u;
    if (fin) acc = xyzz_add_affine_impl<C>(acc, a);
  }
  for (int off = 32; off >= 1; off >>= 1) {
    if (count <= (uint32_t)off) continue;  // uniform: no lane >= off holds a record
    Xyzz<C> o;
#pragma unroll
    for (int k = 0; k < L; k++) {
      o.X.v[k] = __shfl_xor(acc.X.v[k], off, 64);
      o.Y.v[k] = __shfl_xor(acc.Y.v[k], off, 64);
      o.ZZ.v[k] = __shfl_xor(acc.ZZ.v[k], off, 64);
      o.ZZZ.v[k] = __shfl_xor(acc.ZZZ.v[k], off, 64);
    }
    acc = xyzz_add_impl<C>(acc, o);
  }
  // every lane holds a representative of the total; lane 0's is converted
  // by the whole wave (wave-uniform binary GCD on the scalar ALU)
  Affine<C> a;
  const bool fin = xyzz_to_affine_impl<C, true>(acc, a);
  if (lane == 0) {
    affine_to_canonical<C>(out, a, fin);
    out[2 * N] = fin ? 0u : 1u;
    out[2 * N + 1] = 0u;
  }
}

// The fold of projective partial records (the sharded commitment's exchange
// format since round 6, kzgx_msm_g1_partial_device): record k is one XYZZ
// point as the library holds it (4 coordinates of radix-2^29 Montgomery
// limbs, xyzz_words words; ZZ = 0 is infinity), so no rank converts its
// partial to affine -- the fold's one wave-uniform inversion is the only
// one of the step.  Output: one packed affine record, as k_g1_fold_packed.
template <class C>
KZGX_DEV Xyzz<C> xyzz_shfl_down_w(const Xyzz<C>& p, int off);

// Group-cooperative (coop.hpp: 8 lanes per addition, ~1/3 of a lone lane's
// latency): group g sums records g, g + 8, ...; a 3-level tree over the
// groups; the whole wave then converts group 0's sum (one wave-uniform
// inversion).  For the 2-8 records of a sharded step the chain is three
// cooperative additions and the inversion.
template <class C>
__global__ __launch_bounds__(64) void k_g1_fold_xyzz(const uint32_t* __restrict__ rec, uint32_t count,
                                                     uint32_t* __restrict__ out) {
  constexpr int N = C::Fp::N, L = C::Fp29::L;
  constexpr int XW = xyzz_words<C>();
  __shared__ uint32_t sc[8 * COOP_SLOTS * L];
  const uint32_t lane = threadIdx.x, g = lane >> 3;
  const int j = (int)(lane & 7);
  uint32_t* my = sc + g * COOP_SLOTS * L;
  Xyzz<C> acc = g < count ? xyzz_load<C>(rec + (size_t)g * XW) : xyzz_inf<C>();
  for (uint32_t k = g + 8; k < count; k += 8) acc = coop_add<C>(acc, xyzz_load<C>(rec + (size_t)k * XW), my, j);
#pragma unroll 1
  for (uint32_t o = 4; o >= 1; o >>= 1) {
    if (count <= o) continue;  // uniform: groups >= o hold only the identity
    const Xyzz<C> x = xyzz_shfl_down_w<C>(acc, (int)(8 * o));
    if (g < o) acc = coop_add<C>(acc, x, my, j);
  }
  uint32_t wx[N], wy[N];
  const bool fin = xyzz_to_canonical_lane<C>(acc, wx, wy);  // lane 0's value (group 0: the sum)
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < N; k++) {
      out[k] = wx[k];
      out[N + k] = wy[k];
    }
    out[2 * N] = fin ? 0u : 1u;
    out[2 * N + 1] = 0u;
  }
}

// an affine point (canonical, + infinity flag) as a projective record: the
// partial of an MSM path that ends in affine form
template <class C>
__global__ __launch_bounds__(64) void k_affine_to_xyzz(const uint32_t* __restrict__ xy,
                                                       const uint32_t* __restrict__ inf, uint32_t* __restrict__ rec) {
  if (threadIdx.x != 0) return;
  Affine<C> a;
  const bool fin = affine_from_canonical<C>(xy, a) && *inf == 0u;
  xyzz_store<C>(rec, fin ? xyzz_from_affine<C>(a) : xyzz_inf<C>());
}

int g1_fold_xyzz(int curve, const uint32_t* d_rec, size_t count, uint32_t* d_out, hipStream_t st) {
  if (curve == KZGX_CURVE_BN254)
    hipLaunchKernelGGL(k_g1_fold_xyzz<BN254G1>, dim3(1), dim3(64), 0, st, d_rec, (uint32_t)count, d_out);
  else
    hipLaunchKernelGGL(k_g1_fold_xyzz<BLS12381G1>, dim3(1), dim3(64), 0, st, d_rec, (uint32_t)count, d_out);
  KZGX_TRY_HIP(hipGetLastError());
  return KZGX_OK;
}

int affine_to_xyzz(int curve, const uint32_t* d_xy, const uint32_t* d_inf, uint32_t* d_rec, hipStream_t st) {
  if (curve == KZGX_CURVE_BN254)
    hipLaunchKernelGGL(k_affine_to_xyzz<BN254G1>, dim3(1), dim3(64), 0, st, d_xy, d_inf, d_rec);
  else
    hipLaunchKernelGGL(k_affine_to_xyzz<BLS12381G1>, dim3(1), dim3(64), 0, st, d_xy, d_inf, d_rec);
  KZGX_TRY_HIP(hipGetLastError());
  return KZGX_OK;
}

size_t xyzz_record_words(int curve) {
  return curve == KZGX_CURVE_BN254 ? (size_t)xyzz_words<BN254G1>() : (size_t)xyzz_words<BLS12381G1>();
}

// ---- bucket reduction of one wide-window Pippenger MSM (msm.hip, big path) ----
// V = sum_k (k + 1) B_k over nb = 2^(c-1) buckets (c = 14..16), the chain
// that follows the accumulation.  Its depth is ~log2(nb) doublings plus
// ~2 log2(nb) additions whatever the schedule, and a lone wave issues one
// XYZZ addition in ~7 us (its ~2400 VALU instructions), so the schedule is
// made wide: every level runs on as many waves as it has elements.
//   k_lat_bucket_sums: thread t owns J = 2 buckets: R_t = B_{2t} + 2 B_{2t+1},
//                      T_t = B_{2t} + B_{2t+1}  (nb / 2 threads)
//   k_lat_fold1:       256-thread workgroup g over pairs t = 256 g + l:
//                      V_g = sum_l R_l + J sum_l l T_l (suffix sums S_l of T
//                      by a wave scan + the higher waves' totals, a tree),
//                      T_g = sum_l T_l
//   k_lat_fold2:       one wave over the NG = nb / 512 groups: V = sum_g V_g
//                      + 256 J sum_g g T_g the same way, then the wave-uniform
//                      affine conversion
// (k_msm_bucket_fold_wg's algebra: sum_t t T_t = sum_{t >= 1} S_t.)
constexpr uint32_t BIG_RED_J = 2;
constexpr uint32_t BIG_F1 = 256;  // pairs per fold-1 workgroup

template <class C, uint32_t J>
__global__ __launch_bounds__(256) void k_lat_bucket_sums(const uint32_t* __restrict__ offsets, uint32_t nb,
                                                         const uint32_t* __restrict__ bsum, uint32_t* __restrict__ rt) {
  constexpr int XW = xyzz_words<C>();
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nb / J) return;
  const uint32_t* off = offsets + (size_t)t * J;
  const uint32_t* src = bsum + (size_t)t * J * XW;
  Xyzz<C> run = xyzz_inf<C>(), sum = xyzz_inf<C>();
  for (int j = (int)J - 1; j >= 0; j--) {
    if (off[j + 1] > off[j]) run = xyzz_add_impl<C>(run, xyzz_load<C>(src + (size_t)j * XW));  // empty: never written
    sum = xyzz_add_impl<C>(sum, run);
  }
  xyzz_store<C>(rt + (size_t)t * 2 * XW, sum);
  xyzz_store<C>(rt + (size_t)t * 2 * XW + XW, run);
}

template <class C>
KZGX_DEV Xyzz<C> xyzz_shfl_down_w(const Xyzz<C>& p, int off) {
  Xyzz<C> o;
#pragma unroll
  for (int k = 0; k < C::Fp29::L; k++) {
    o.X.v[k] = __shfl_down(p.X.v[k], off, 64);
    o.Y.v[k] = __shfl_down(p.Y.v[k], off, 64);
    o.ZZ.v[k] = __shfl_down(p.ZZ.v[k], off, 64);
    o.ZZZ.v[k] = __shfl_down(p.ZZZ.v[k], off, 64);
  }
  return o;
}

template <class C>
KZGX_DEV Xyzz<C> xyzz_dbl_pow2(Xyzz<C> p, uint32_t m) {  // m p, m a power of two
#pragma unroll 1
  for (; m > 1; m >>= 1) p = xyzz_dbl_impl<C>(p);
  return p;
}

// inclusive suffix sums over the wave's lanes < n (lanes >= n: infinity)
template <class C>
KZGX_DEV Xyzz<C> wave_suffix(Xyzz<C> S, uint32_t lane, uint32_t n) {
#pragma unroll 1
  for (uint32_t o = 1; o < n; o <<= 1) {
    const Xyzz<C> x = xyzz_shfl_down_w<C>(S, (int)o);
    if (lane + o < n) S = xyzz_add_impl<C>(S, x);
  }
  return S;
}
// sum over the wave's lanes < n, landing in lane 0
template <class C>
KZGX_DEV Xyzz<C> wave_total(Xyzz<C> U, uint32_t n) {
#pragma unroll 1
  for (uint32_t o = 32; o >= 1; o >>= 1)
    if (o < n) U = xyzz_add_impl<C>(U, xyzz_shfl_down_w<C>(U, (int)o));
  return U;
}

// workgroups g < NG: V_g = sum_l R_l + J sum_l l T_l over the group's 256
// pairs.  Workgroups NG + g: T'_g = 512 T_g (J BIG_F1 = 512), the group
// total scaled for the second level, on its own CU so that its 9 doublings
// run beside V_g's chain instead of after it (k_lat_fold2 then needs none).
template <class C>
__global__ __launch_bounds__(BIG_F1) void k_lat_fold1(const uint32_t* __restrict__ rt, uint32_t NG,
                                                      uint32_t* __restrict__ vt) {
  constexpr int XW = xyzz_words<C>();
  constexpr uint32_t NW = BIG_F1 / 64;
  static_assert(NW == 4, "k_lat_fold1: four waves");
  __shared__ uint32_t lds[NW * XW];
  const uint32_t l = threadIdx.x, lane = l & 63, wv = l >> 6;
  if (blockIdx.x >= NG) {
    const uint32_t g = blockIdx.x - NG;
    Xyzz<C> T = wave_total<C>(xyzz_load<C>(rt + ((size_t)g * BIG_F1 + l) * 2 * XW + XW), 64);
    if (lane == 0) xyzz_store<C>(lds + wv * XW, T);
    __syncthreads();
    if (l != 0) return;
    T = xyzz_add_impl<C>(xyzz_add_impl<C>(T, xyzz_load<C>(lds + XW)),
                         xyzz_add_impl<C>(xyzz_load<C>(lds + 2 * XW), xyzz_load<C>(lds + 3 * XW)));
    xyzz_store<C>(vt + (size_t)g * 2 * XW + XW, xyzz_dbl_pow2<C>(T, BIG_RED_J * BIG_F1));
    return;
  }
  const uint32_t* src = rt + ((size_t)blockIdx.x * BIG_F1 + l) * 2 * XW;
  const Xyzz<C> R = xyzz_load<C>(src);
  Xyzz<C> S = wave_suffix<C>(xyzz_load<C>(src + XW), lane, 64);
  if (lane == 0) xyzz_store<C>(lds + wv * XW, S);
  __syncthreads();
#pragma unroll 1
  for (uint32_t w = wv + 1; w < NW; w++) S = xyzz_add_impl<C>(S, xyzz_load<C>(lds + w * XW));
  __syncthreads();  // lds is reused below
  Xyzz<C> U = R;
  if (l > 0) U = xyzz_add_impl<C>(U, xyzz_dbl_pow2<C>(S, BIG_RED_J));
  U = wave_total<C>(U, 64);
  if (lane == 0) xyzz_store<C>(lds + wv * XW, U);
  __syncthreads();
  // (U0 + U1) + (U2 + U3): waves 0 and 2 in parallel, then thread 0
  if (l == 128) xyzz_store<C>(lds + 2 * XW, xyzz_add_impl<C>(U, xyzz_load<C>(lds + 3 * XW)));
  if (l == 0) U = xyzz_add_impl<C>(U, xyzz_load<C>(lds + XW));
  __syncthreads();
  if (l != 0) return;
  xyzz_store<C>(vt + (size_t)blockIdx.x * 2 * XW, xyzz_add_impl<C>(U, xyzz_load<C>(lds + 2 * XW)));
}

template <class C>
__global__ __launch_bounds__(64) void k_lat_fold2(const uint32_t* __restrict__ vt, uint32_t NG,
                                                  uint32_t* __restrict__ out, uint32_t* __restrict__ out_inf) {
  constexpr int XW = xyzz_words<C>();
  const uint32_t lane = threadIdx.x;
  Xyzz<C> V = xyzz_inf<C>(), S = xyzz_inf<C>();
  if (lane < NG) {
    V = xyzz_load<C>(vt + (size_t)lane * 2 * XW);
    S = xyzz_load<C>(vt + (size_t)lane * 2 * XW + XW);  // already 512 T_g
  }
  S = wave_suffix<C>(S, lane, NG);
  if (lane > 0 && lane < NG) V = xyzz_add_impl<C>(V, S);
  V = wave_total<C>(V, NG);
  Xyzz<C> v;
#pragma unroll
  for (int k = 0; k < C::Fp29::L; k++) {
    v.X.v[k] = __builtin_amdgcn_readfirstlane(V.X.v[k]);
    v.Y.v[k] = __builtin_amdgcn_readfirstlane(V.Y.v[k]);
    v.ZZ.v[k] = __builtin_amdgcn_readfirstlane(V.ZZ.v[k]);
    v.ZZZ.v[k] = __builtin_amdgcn_readfirstlane(V.ZZZ.v[k]);
  }
  Affine<C> a;
  const bool fin = xyzz_to_affine_impl<C, true>(v, a);
  if (lane != 0) return;
  affine_to_canonical<C>(out, a, fin);
  *out_inf = fin ? 0u : 1u;
}

size_t big_reduce_rt_bytes(int curve, uint32_t nb) {
  const size_t xb = 4 * (curve == KZGX_CURVE_BN254 ? xyzz_words<BN254G1>() : xyzz_words<BLS12381G1>());
  const size_t T1 = nb / BIG_RED_J;
  return (T1 + T1 / 16 + 4) * 2 * xb;  // the pairs, then the fold levels' outputs
}

// ---- group-cooperative fold levels (coop.hpp): the top of the reduction ----
// A level reduces N (R_t, T_t) pairs, V = sum_t R_t + 2^JLOG t T_t, 32 pairs
// per 256-thread workgroup (one 8-lane group per pair):
//   workgroups b < NGo:  V_b = sum_l R_l + 2^JLOG l T_l over its pairs
//                        (suffix sums S_l by group shuffles + the higher
//                        waves' totals; sum_l l T_l = sum_{l >= 1} S_l)
//   workgroups NGo + b:  T'_b = 2^(5 + JLOG) sum_l T_l, beside V_b's chain,
// so the next level sees pairs (V_b, T'_b) with JLOG = 0.  Every point op is
// one cooperative addition / doubling (~1/3 of a lone lane's latency).
// the fold's point ops: cooperative, or (LONE, A/B and debugging) every
// lane of the group running the lone-lane form
template <class C, bool LONE>
KZGX_DEV Xyzz<C> cadd(const Xyzz<C>& a, const Xyzz<C>& b, uint32_t* sc, int j) {
  if constexpr (LONE) return xyzz_add_impl<C>(a, b);
  else return coop_add<C>(a, b, sc, j);
}
template <class C, bool LONE>
KZGX_DEV Xyzz<C> cdbl(const Xyzz<C>& a, uint32_t* sc, int j) {
  if constexpr (LONE) return xyzz_dbl_impl<C>(a);
  else return coop_dbl<C>(a, sc, j);
}

template <class C, int JLOG, bool LONE>
__global__ __launch_bounds__(256) void k_coop_fold(const uint32_t* __restrict__ in, uint32_t N, uint32_t NGo,
                                                   uint32_t* __restrict__ out) {
  using F = typename C::Fp29;
  constexpr int XW = xyzz_words<C>(), L = F::L;
  __shared__ uint32_t sc[32 * COOP_SLOTS * L];
  __shared__ uint32_t wt[4 * XW];
  const uint32_t t = threadIdx.x, wv = t >> 6, g = t >> 3, gw = (t & 63) >> 3;
  const int j = (int)(t & 7);
  uint32_t* my = sc + g * COOP_SLOTS * L;
  const bool tpath = blockIdx.x >= NGo;
  const uint32_t b = tpath ? blockIdx.x - NGo : blockIdx.x;
  const uint32_t idx = b * 32 + g;
  const uint32_t* src = in + (size_t)idx * 2 * XW;
  if (tpath) {
    Xyzz<C> T = idx < N ? xyzz_load<C>(src + XW) : xyzz_inf<C>();
#pragma unroll 1
    for (int o = 4; o >= 1; o >>= 1) T = cadd<C, LONE>(T, xyzz_shfl_down_w<C>(T, 8 * o), my, j);
    if ((t & 63) == 0) xyzz_store<C>(wt + wv * XW, T);
    __syncthreads();
    if (t >= 16) return;
    // groups 0 and 1 of wave 0: (wt0 + wt1), (wt2 + wt3); then group 0 adds
    T = cadd<C, LONE>(xyzz_load<C>(wt + (2 * g) * XW), xyzz_load<C>(wt + (2 * g + 1) * XW), my, j);
    T = cadd<C, LONE>(T, xyzz_shfl_down_w<C>(T, 8), my, j);
#pragma unroll 1
    for (int d = 0; d < 5 + JLOG; d++) T = cdbl<C, LONE>(T, my, j);
    if (t == 0) xyzz_store<C>(out + (size_t)b * 2 * XW + XW, T);
    return;
  }
  const Xyzz<C> R = idx < N ? xyzz_load<C>(src) : xyzz_inf<C>();
  Xyzz<C> S = idx < N ? xyzz_load<C>(src + XW) : xyzz_inf<C>();
#pragma unroll 1
  for (uint32_t o = 1; o < 8; o <<= 1) {
    const Xyzz<C> x = xyzz_shfl_down_w<C>(S, (int)(8 * o));
    if (gw + o < 8) S = cadd<C, LONE>(S, x, my, j);
  }
  if ((t & 63) == 0) xyzz_store<C>(wt + wv * XW, S);
  __syncthreads();
#pragma unroll 1
  for (uint32_t w = wv + 1; w < 4; w++) S = cadd<C, LONE>(S, xyzz_load<C>(wt + w * XW), my, j);
  __syncthreads();  // wt is reused below
  Xyzz<C> U = R;
  if (g > 0) {
#pragma unroll 1
    for (int d = 0; d < JLOG; d++) S = cdbl<C, LONE>(S, my, j);
    U = cadd<C, LONE>(U, S, my, j);
  }
#pragma unroll 1
  for (int o = 4; o >= 1; o >>= 1) U = cadd<C, LONE>(U, xyzz_shfl_down_w<C>(U, 8 * o), my, j);
  if ((t & 63) == 0) xyzz_store<C>(wt + wv * XW, U);
  __syncthreads();
  if (t < 8 || (t >= 128 && t < 136)) {  // group 0 of waves 0 and 2
    const Xyzz<C> o = xyzz_load<C>(wt + (wv + 1) * XW);
    U = cadd<C, LONE>(U, o, my, j);
    if (t == 128) xyzz_store<C>(wt + 2 * XW, U);
  }
  __syncthreads();
  if (t >= 8) return;
  U = cadd<C, LONE>(U, xyzz_load<C>(wt + 2 * XW), my, j);
  if (t == 0) xyzz_store<C>(out + (size_t)b * 2 * XW, U);
}

// the last level's V (pair 0's R slot) -> canonical affine, by one wave; or
// (xyzz_out) V itself, for a caller that adds it to more points before the
// one inversion (the sharded commitment's partial records)
template <class C>
__global__ __launch_bounds__(64) void k_coop_finish(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                    uint32_t* __restrict__ out_inf, uint32_t* __restrict__ xyzz_out) {
  const Xyzz<C> V = xyzz_load<C>(in);
  if (xyzz_out) {
    if (threadIdx.x == 0) xyzz_store<C>(xyzz_out, V);
    return;
  }
  constexpr int N = C::Fp::N;
  uint32_t wx[N], wy[N];
  const bool fin = xyzz_to_canonical_lane<C>(V, wx, wy);
  if (threadIdx.x != 0) return;
#pragma unroll
  for (int k = 0; k < N; k++) {
    out[k] = wx[k];
    out[N + k] = wy[k];
  }
  *out_inf = fin ? 0u : 1u;
}

// self-test of coop.hpp against the lone-lane forms (kzgx_debug_coop_test):
// group k takes table points a0, a1, a2 = tab[3k..3k+2] (affine Montgomery),
// P = 2 a0 (XYZZ, ZZ != 1), Q = 2 a1 + a2, and checks coop_add(P, Q),
// coop_add(P, P), coop_add(P, -P) and coop_dbl(Q) against xyzz_add_impl /
// xyzz_dbl_impl in affine form; bit c of *bad set on a mismatch in case c
template <class C>
__global__ __launch_bounds__(256) void k_coop_selftest(const uint32_t* __restrict__ tab, uint32_t groups,
                                                      uint32_t* __restrict__ bad) {
  using F = typename C::Fp29;
  constexpr int AW = affine_words<C>();
  __shared__ uint32_t sc[32 * COOP_SLOTS * F::L];
  const uint32_t t = threadIdx.x, g = t >> 3;
  const int j = (int)(t & 7);
  const uint32_t k = blockIdx.x * 32 + g;
  if (blockIdx.x * 32 >= groups) return;
  const uint32_t kk = k < groups ? k : 0;
  const Affine<C> a0 = affine_load<C>(tab + (size_t)(3 * kk) * AW);
  const Affine<C> a1 = affine_load<C>(tab + (size_t)(3 * kk + 1) * AW);
  const Affine<C> a2 = affine_load<C>(tab + (size_t)(3 * kk + 2) * AW);
  const Xyzz<C> P = xyzz_dbl_impl<C>(xyzz_from_affine<C>(a0));
  const Xyzz<C> Q = xyzz_add_affine_impl<C>(xyzz_dbl_impl<C>(xyzz_from_affine<C>(a1)), a2);
  uint32_t* my = sc + g * COOP_SLOTS * F::L;
  Xyzz<C> got[4], want[4];
  got[0] = coop_add<C>(P, Q, my, j);
  want[0] = xyzz_add_impl<C>(P, Q);
  got[1] = coop_add<C>(P, P, my, j);
  want[1] = xyzz_dbl_impl<C>(P);
  got[2] = coop_add<C>(P, xyzz_neg<C>(P), my, j);
  want[2] = xyzz_inf<C>();
  got[3] = coop_dbl<C>(Q, my, j);
  want[3] = xyzz_dbl_impl<C>(Q);
  // case 4: the fold's in-wave suffix scan (shuffles between groups, groups
  // dropping out), cooperative against every lane running the lone form
  {
    const uint32_t gw = (t & 63) >> 3;
    Xyzz<C> S = Q, Sl = Q;
#pragma unroll 1
    for (uint32_t o = 1; o < 8; o <<= 1) {
      const Xyzz<C> x = xyzz_shfl_down_w<C>(S, (int)(8 * o));
      const Xyzz<C> xl = xyzz_shfl_down_w<C>(Sl, (int)(8 * o));
      if (gw + o < 8) {
        S = coop_add<C>(S, x, my, j);
        Sl = xyzz_add_impl<C>(Sl, xl);
      }
    }
    got[3] = coop_dbl<C>(Q, my, j);
    want[3] = xyzz_dbl_impl<C>(Q);
    got[2] = S;
    want[2] = Sl;
  }
  if (k >= groups) return;
  uint32_t b = 0;
#pragma unroll 1
  for (int c = 0; c < 4; c++) {
    Affine<C> x, y;
    const bool fx = xyzz_to_affine_impl<C>(got[c], x), fy = xyzz_to_affine_impl<C>(want[c], y);
    bool same = fx == fy;
    if (fx && fy)
      for (int i = 0; i < F::L; i++) same = same && x.x.v[i] == y.x.v[i] && x.y.v[i] == y.y.v[i];
    if (!same) b |= 1u << c;
  }
  if (b) atomicOr(bad, b);
}

int coop_selftest(int curve, const uint32_t* d_tab, uint32_t n_pts, uint32_t* d_bad, hipStream_t st) {
  const uint32_t groups = n_pts / 3;
  if (groups == 0) return KZGX_ERR_ARG;
  if (curve == KZGX_CURVE_BN254)
    hipLaunchKernelGGL(k_coop_selftest<BN254G1>, dim3((groups + 31) / 32), dim3(256), 0, st, d_tab, groups, d_bad);
  else
    hipLaunchKernelGGL(k_coop_selftest<BLS12381G1>, dim3((groups + 31) / 32), dim3(256), 0, st, d_tab, groups, d_bad);
  KZGX_TRY_HIP(hipGetLastError());
  return KZGX_OK;
}

// A/B-only kernels (the lone-lane fold forms behind KZGX_COOP_LONE and
// KZGX_BIG_LONEFOLD) are compiled only into variant builds
// (make variant VFLAGS=-DKZGX_AB_VARIANTS): the dispatcher never reaches
// them otherwise, and they were a third of this object's compile time
template <class C, int JLOG>
static void coop_level(const uint32_t* in, uint32_t N, uint32_t NG, uint32_t* out, hipStream_t st) {
#ifdef KZGX_AB_VARIANTS
  static const bool lone = std::getenv("KZGX_COOP_LONE") != nullptr;
  if (lone) {
    hipLaunchKernelGGL((k_coop_fold<C, JLOG, true>), dim3(2 * NG), dim3(256), 0, st, in, N, NG, out);
    return;
  }
#endif
  hipLaunchKernelGGL((k_coop_fold<C, JLOG, false>), dim3(2 * NG), dim3(256), 0, st, in, N, NG, out);
}

// rt holds T1 pairs (R_t, T_t) weighted V = sum_t R_t + 2^jlog t T_t
template <class C>
static int coop_levels(uint32_t* d_rt, uint32_t T1, int jlog, uint32_t* d_out, uint32_t* d_out_inf, hipStream_t st,
                       uint32_t* xyzz_out) {
  constexpr int XW = xyzz_words<C>();
  uint32_t* in = d_rt;
  uint32_t* nxt = d_rt + (size_t)T1 * 2 * XW;
  uint32_t N = T1;
  bool first = true;
  for (;;) {
    const uint32_t NG = (N + 31) / 32;
    const int jl = first ? jlog : 0;
    if (jl == 2)
      coop_level<C, 2>(in, N, NG, nxt, st);
    else if (jl == 1)
      coop_level<C, 1>(in, N, NG, nxt, st);
    else
      coop_level<C, 0>(in, N, NG, nxt, st);
    first = false;
    in = nxt;
    nxt += (size_t)NG * 2 * XW;
    N = NG;
    if (N == 1) break;
  }
  hipLaunchKernelGGL(k_coop_finish<C>, dim3(1), dim3(64), 0, st, in, d_out, d_out_inf, xyzz_out);
  KZGX_TRY_HIP(hipGetLastError());
  return KZGX_OK;
}

template <class C>
static int big_reduce_impl(const uint32_t* d_offsets, uint32_t nb, const uint32_t* d_bsum, uint32_t* d_rt,
                           uint32_t* d_out, uint32_t* d_out_inf, hipStream_t st, uint32_t* xyzz_out) {
  const uint32_t T1 = nb / BIG_RED_J, NG = T1 / BIG_F1;
  if (NG < 1 || T1 % BIG_F1) return KZGX_ERR_INTERNAL;  // nb >= 512
#ifdef KZGX_AB_VARIANTS
  static const bool lone = std::getenv("KZGX_BIG_LONEFOLD") != nullptr;
  if (lone && !xyzz_out && NG <= 64) {  // k_lat_fold2: one wave over the NG groups
    uint32_t* vt = d_rt + (size_t)T1 * 2 * xyzz_words<C>();
    hipLaunchKernelGGL((k_lat_bucket_sums<C, BIG_RED_J>), dim3((T1 + 255) / 256), dim3(256), 0, st, d_offsets, nb,
                       d_bsum, d_rt);
    hipLaunchKernelGGL(k_lat_fold1<C>, dim3(2 * NG), dim3(BIG_F1), 0, st, d_rt, NG, vt);
    hipLaunchKernelGGL(k_lat_fold2<C>, dim3(1), dim3(64), 0, st, vt, NG, d_out, d_out_inf);
    KZGX_TRY_HIP(hipGetLastError());
    return KZGX_OK;
  }
#endif
  // 4 buckets per bucket-sum thread: half the pairs for the cooperative
  // levels (the first level then holds 2 waves per SIMD, not 4)
  const uint32_t T4 = nb / 4;
  hipLaunchKernelGGL((k_lat_bucket_sums<C, 4>), dim3((T4 + 255) / 256), dim3(256), 0, st, d_offsets, nb, d_bsum,
                     d_rt);
  return coop_levels<C>(d_rt, T4, 2, d_out, d_out_inf, st, xyzz_out);
}

// ---- bucket-aligned segments (msm.hip k_big2_*): partials -> (R_t, T_t) ----
KZGX_DEV uint32_t lat_seg_bucket(const uint32_t* __restrict__ seg_off, uint32_t nb, uint32_t j) {
  uint32_t lo = 0, hi = nb;  // seg_off[lo] <= j < seg_off[hi]
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (seg_off[mid] <= j)
      lo = mid;
    else
      hi = mid;
  }
  return lo;
}
// stride of a bucket's live partials after the pre-sum passes: the smallest
// 8^p with ceil(s / 8^p) <= BIG_MAXSEG
constexpr uint32_t LAT_MAXSEG = 64;  // msm.hip BIG_MAXSEG
KZGX_DEV uint32_t lat_seg_stride(uint32_t s) {
  uint32_t st = 1;
  while ((s + st - 1) / st > LAT_MAXSEG) st *= 8;
  return st;
}

// pre-sum pass p (1, 2, ...) for buckets with more than LAT_MAXSEG segment
// partials (skewed scalars): the partials at stride 8^(p-1) are summed 8 to
// 1 into the positions that are multiples of 8^p.  No-op unless *flag.
template <class C>
__global__ __launch_bounds__(256) void k_lat_long(const uint32_t* __restrict__ seg_off, uint32_t nb, uint32_t sp,
                                                  const uint32_t* __restrict__ flag, uint32_t* __restrict__ part) {
  constexpr int XW = xyzz_words<C>();
  if (!*flag) return;
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= seg_off[nb]) return;
  const uint32_t k = lat_seg_bucket(seg_off, nb, j);
  const uint32_t s = seg_off[k + 1] - seg_off[k];
  if ((s + sp - 1) / sp <= LAT_MAXSEG) return;
  const uint32_t i = j - seg_off[k];
  if (i % (8 * sp)) return;
  uint32_t* base = part + (size_t)seg_off[k] * XW;
  Xyzz<C> acc = xyzz_load<C>(base + (size_t)i * XW);
  for (uint32_t m = 1; m < 8 && i + m * sp < s; m++) acc = xyzz_add_impl<C>(acc, xyzz_load<C>(base + (size_t)(i + m * sp) * XW));
  xyzz_store<C>(base + (size_t)i * XW, acc);
}

template <class C>
KZGX_DEV Xyzz<C> xyzz_shfl_xor_w(const Xyzz<C>& p, int m) {
  Xyzz<C> o;
#pragma unroll
  for (int k = 0; k < C::Fp29::L; k++) {
    o.X.v[k] = __shfl_xor(p.X.v[k], m, 64);
    o.Y.v[k] = __shfl_xor(p.Y.v[k], m, 64);
    o.ZZ.v[k] = __shfl_xor(p.ZZ.v[k], m, 64);
    o.ZZZ.v[k] = __shfl_xor(p.ZZZ.v[k], m, 64);
  }
  return o;
}

// G lanes per bucket, 2 G per pair t: B_k = the sum of bucket k's partials
// (lane-strided, then a G-lane shuffle tree), T_t = B_2t + B_2t+1 (lane 0
// stores), R_t = T_t + B_2t+1 (lane G stores)
template <class C, uint32_t G>
__global__ __launch_bounds__(256) void k_lat_seg_sums(const uint32_t* __restrict__ seg_off, uint32_t nb,
                                                      const uint32_t* __restrict__ part, uint32_t* __restrict__ rt) {
  constexpr int XW = xyzz_words<C>();
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t t = gid / (2 * G), q = gid % (2 * G);
  if (t >= nb / 2) return;  // whole pair groups
  const uint32_t k = 2 * t + q / G, sub = q % G;
  const uint32_t s0 = seg_off[k], s = seg_off[k + 1] - s0;
  const uint32_t sp = lat_seg_stride(s), c = (s + sp - 1) / sp;
  Xyzz<C> acc = xyzz_inf<C>();
  for (uint32_t i = sub; i < c; i += G) acc = xyzz_add_impl<C>(acc, xyzz_load<C>(part + (size_t)(s0 + i * sp) * XW));
#pragma unroll 1
  for (uint32_t m = 1; m < G; m <<= 1) acc = xyzz_add_impl<C>(acc, xyzz_shfl_xor_w<C>(acc, (int)m));
  const Xyzz<C> T = xyzz_add_impl<C>(acc, xyzz_shfl_xor_w<C>(acc, (int)G));
  if (q == 0) xyzz_store<C>(rt + (size_t)t * 2 * XW + XW, T);
  if (q == G) xyzz_store<C>(rt + (size_t)t * 2 * XW, xyzz_add_impl<C>(T, acc));
}

template <class C>
static int big_reduce_seg_impl(const uint32_t* d_seg_off, uint32_t* d_part, uint32_t nb, uint32_t s_ub,
                               const uint32_t* d_flag, uint32_t* d_rt, uint32_t* d_out, uint32_t* d_out_inf,
                               hipStream_t st, uint32_t* xyzz_out) {
  const uint32_t T1 = nb / BIG_RED_J, NG = T1 / BIG_F1;
  if (NG < 1 || T1 % BIG_F1) return KZGX_ERR_INTERNAL;
  uint32_t* vt = d_rt + (size_t)T1 * 2 * xyzz_words<C>();
  // pre-sum passes: as many as the largest possible bucket (s_ub partials)
  // could need; each exits at once unless some bucket has > LAT_MAXSEG
  for (uint64_t sp = 1; (s_ub + sp - 1) / sp > LAT_MAXSEG; sp *= 8)
    hipLaunchKernelGGL(k_lat_long<C>, dim3((s_ub + 255) / 256), dim3(256), 0, st, d_seg_off, nb, (uint32_t)sp, d_flag,
                       d_part);
  // lanes per bucket: 8 when buckets hold more than ~8 partials on average
  if (s_ub / nb > 8)
    hipLaunchKernelGGL((k_lat_seg_sums<C, 8>), dim3((nb * 8 + 255) / 256), dim3(256), 0, st, d_seg_off, nb, d_part,
                       d_rt);
  else
    hipLaunchKernelGGL((k_lat_seg_sums<C, 4>), dim3((nb * 4 + 255) / 256), dim3(256), 0, st, d_seg_off, nb, d_part,
                       d_rt);
  // the fold: group-cooperative levels (variant builds: KZGX_BIG_LONEFOLD,
  // the lone-lane k_lat_fold1 / k_lat_fold2, A/B)
#ifdef KZGX_AB_VARIANTS
  static const bool lone = std::getenv("KZGX_BIG_LONEFOLD") != nullptr;
  if (lone && !xyzz_out && NG <= 64) {  // k_lat_fold2: one wave over the NG groups
    hipLaunchKernelGGL(k_lat_fold1<C>, dim3(2 * NG), dim3(BIG_F1), 0, st, d_rt, NG, vt);
    hipLaunchKernelGGL(k_lat_fold2<C>, dim3(1), dim3(64), 0, st, vt, NG, d_out, d_out_inf);
    KZGX_TRY_HIP(hipGetLastError());
    return KZGX_OK;
  }
#else
  (void)vt;
#endif
  return coop_levels<C>(d_rt, T1, 1, d_out, d_out_inf, st, xyzz_out);
}

int big_reduce_seg(int curve, const uint32_t* d_seg_off, uint32_t* d_part, uint32_t nb, uint32_t s_ub,
                   const uint32_t* d_flag, uint32_t* d_rt, uint32_t* d_out, uint32_t* d_out_inf, hipStream_t st,
                   uint32_t* xyzz_out) {
  return curve == KZGX_CURVE_BN254
             ? big_reduce_seg_impl<BN254G1>(d_seg_off, d_part, nb, s_ub, d_flag, d_rt, d_out, d_out_inf, st, xyzz_out)
             : big_reduce_seg_impl<BLS12381G1>(d_seg_off, d_part, nb, s_ub, d_flag, d_rt, d_out, d_out_inf, st,
                                               xyzz_out);
}

int big_reduce(int curve, const uint32_t* d_offsets, uint32_t nb, const uint32_t* d_bsum, uint32_t* d_rt,
               uint32_t* d_out, uint32_t* d_out_inf, hipStream_t st, uint32_t* xyzz_out) {
  return curve == KZGX_CURVE_BN254
             ? big_reduce_impl<BN254G1>(d_offsets, nb, d_bsum, d_rt, d_out, d_out_inf, st, xyzz_out)
             : big_reduce_impl<BLS12381G1>(d_offsets, nb, d_bsum, d_rt, d_out, d_out_inf, st, xyzz_out);
}

// the large-MSM path's segment merge with the XYZZ addition inlined
// (k_msm_merge<C, true>): exact only with memory clauses off (DESIGN.md
// section 7), which this translation unit is compiled with; msm.hip's batched
// path keeps the called form
int big_merge_inline(int curve, const uint32_t* heads, const uint32_t* tails, const uint32_t* tailk,
                     const uint8_t* sstate, uint32_t smax, uint32_t nb, uint32_t nwg, uint32_t* bsum, uint32_t* ghead,
                     uint32_t* gtail, uint32_t* gtailk, uint32_t* gflag, hipStream_t st) {
  if (curve == KZGX_CURVE_BN254)
    hipLaunchKernelGGL((k_msm_merge<BN254G1, true>), dim3(nwg, 1), dim3(ACC_WG), 0, st, heads, tails, tailk, sstate,
                       smax, nb, nwg, bsum, ghead, gtail, gtailk, gflag);
  else
    hipLaunchKernelGGL((k_msm_merge<BLS12381G1, true>), dim3(nwg, 1), dim3(ACC_WG), 0, st, heads, tails, tailk,
                       sstate, smax, nb, nwg, bsum, ghead, gtail, gtailk, gflag);
  KZGX_TRY_HIP(hipGetLastError());
  return KZGX_OK;
}

int g1_fold_packed(int curve, const uint32_t* d_rec, size_t count, uint32_t* d_out, hipStream_t st) {
  if (curve == KZGX_CURVE_BN254)
    hipLaunchKernelGGL(k_g1_fold_packed<BN254G1>, dim3(1), dim3(64), 0, st, d_rec, (uint32_t)count, d_out);
  else
    hipLaunchKernelGGL(k_g1_fold_packed<BLS12381G1>, dim3(1), dim3(64), 0, st, d_rec, (uint32_t)count, d_out);
  KZGX_TRY_HIP(hipGetLastError());
  return KZGX_OK;
}

}  // namespace kzgx
