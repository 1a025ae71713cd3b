// SRS generation and small G1 helpers for gfx950.
//
// kzgx_gen_srs_g1 replaces the G1 half of trusted_setup(int)
// (src/trusted_setup.cpp:21-74, worker generate_elements_range :123-135),
// which computes power(s, i) per index and one PAIR_G1mul per point on
// hardware_concurrency() std::threads.  Here every GPU thread derives
// tau^(start+i) by square-and-multiply and runs its own fixed-base
// double-and-add in XYZZ coordinates.
#include <hip/hip_runtime.h>

#include "curve.hpp"
#include "kzgx_internal.hpp"
#include "kzgx_setup.hpp"

namespace kzgx {

template <class C>
__global__ __launch_bounds__(256) void k_gen_srs(const uint32_t* __restrict__ tau_canon, uint64_t start, uint32_t n,
                                                 uint32_t* __restrict__ out) {
  using F = typename C::Fp29;
  using FR = typename C::Fr;
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  // e = tau^(start + i) mod r
  const Fe<FR> tm = fe_to_mont<FR>(fe_load<FR>(tau_canon));
  const uint64_t ex = start + i;
  Fe<FR> e = fe_one<FR>();
  for (int b = 63; b >= 0; b--) {
    e = fe_sqr<FR>(e);
    if ((ex >> b) & 1ull) e = fe_mul<FR>(e, tm);
  }
  e = fe_from_mont<FR>(e);
  Affine<C> g;
  g.x = f29_const<F>(C::GX29);
  g.y = f29_const<F>(C::GY29);
  Xyzz<C> acc = xyzz_inf<C>();
  for (int b = 8 * FR::N * 4 - 1; b >= 0; b--) {
    acc = xyzz_dbl<C>(acc);
    if ((e.v[b >> 5] >> (b & 31)) & 1u) acc = xyzz_add_affine<C>(acc, g);
  }
  Affine<C> a;
  const bool fin = xyzz_to_affine<C>(acc, a);
  affine_to_canonical<C>(out + (size_t)i * 2 * C::Fp::N, a, fin);
}

// out = sum of count canonical affine points (zero or flagged = infinity)
template <class C>
__global__ void k_g1_sum(const uint32_t* __restrict__ xy, const uint32_t* __restrict__ inf, uint32_t count,
                         uint32_t* __restrict__ out, uint32_t* __restrict__ out_inf) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  Xyzz<C> acc = xyzz_inf<C>();
  for (uint32_t i = 0; i < count; i++) {
    Affine<C> a;
    const bool finite = affine_from_canonical<C>(xy + (size_t)i * 2 * C::Fp::N, a);
    if ((inf && inf[i]) || !finite) continue;
    acc = xyzz_add_affine<C>(acc, a);
  }
  Affine<C> r;
  bool fin = xyzz_to_affine<C>(acc, r);
  affine_to_canonical<C>(out, r, fin);
  *out_inf = fin ? 0u : 1u;
}

int gen_srs_points(Ctx* ctx, const uint32_t* d_tau, size_t start, size_t n, uint32_t* d_out, hipStream_t st) {
  dim3 blk(256), grd((unsigned)((n + 255) / 256));
  if (ctx->curve == KZGX_CURVE_BN254)
    hipLaunchKernelGGL(k_gen_srs<BN254G1>, grd, blk, 0, st, d_tau, (uint64_t)start, (uint32_t)n, d_out);
  else
    hipLaunchKernelGGL(k_gen_srs<BLS12381G1>, grd, blk, 0, st, d_tau, (uint64_t)start, (uint32_t)n, d_out);
  KZGX_TRY_HIP(hipGetLastError());
  return KZGX_OK;
}

int g1_sum(Ctx* ctx, const uint32_t* d_xy, const uint32_t* d_inf, size_t count, uint32_t* d_out, uint32_t* d_out_inf,
           hipStream_t st) {
  if (ctx->curve == KZGX_CURVE_BN254)
    hipLaunchKernelGGL(k_g1_sum<BN254G1>, dim3(1), dim3(64), 0, st, d_xy, d_inf, (uint32_t)count, d_out, d_out_inf);
  else
    hipLaunchKernelGGL(k_g1_sum<BLS12381G1>, dim3(1), dim3(64), 0, st, d_xy, d_inf, (uint32_t)count, d_out, d_out_inf);
  KZGX_TRY_HIP(hipGetLastError());
  return KZGX_OK;
}

}  // namespace kzgx

namespace kzgx {

// 1 if the canonical affine point is a valid curve point (coordinates < m,
// y^2 = x^3 + b), else 0; infinity (all zero) is not a valid octet point
template <class C>
__global__ void k_g1_validate(const uint32_t* __restrict__ xy, uint32_t* __restrict__ ok) {
  using F = typename C::Fp29;
  constexpr int N = C::Fp::N;
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  bool lt = true;
  for (int c = 0; c < 2; c++) {
    int cmp = 0;  // coordinate vs modulus, most significant word first
    for (int i = N - 1; i >= 0 && cmp == 0; i--) {
      const uint32_t a = xy[c * N + i], m = C::Fp::P[i];
      cmp = a < m ? -1 : (a > m ? 1 : 0);
    }
    lt = lt && cmp < 0;
  }
  Affine<C> a;
  const bool finite = affine_from_canonical<C>(xy, a);
  uint32_t bw[N];
  for (int i = 0; i < N; i++) bw[i] = i == 0 ? C::BSMALL : 0u;
  const F29<F> b = f29_to_mont<F>(f29_from_words<F, N>(bw));
  const F29<F> y2 = f29_sqr<F>(a.y);
  const F29<F> x3 = f29_mul<F>(f29_sqr<F>(a.x), a.x);
  const F29<F> d = f29_sub<F>(y2, f29_add<F>(x3, b), F::P4);  // < 6m
  *ok = (lt && finite && f29_is_zero<F>(d)) ? 1u : 0u;
}

int g1_validate(Ctx* ctx, const uint32_t* d_xy, uint32_t* d_ok, hipStream_t st) {
  if (ctx->curve == KZGX_CURVE_BN254)
    hipLaunchKernelGGL(k_g1_validate<BN254G1>, dim3(1), dim3(64), 0, st, d_xy, d_ok);
  else
    hipLaunchKernelGGL(k_g1_validate<BLS12381G1>, dim3(1), dim3(64), 0, st, d_xy, d_ok);
  KZGX_TRY_HIP(hipGetLastError());
  return KZGX_OK;
}

}  // namespace kzgx

namespace kzgx {
// device bring-up (kzgx_setup.hpp): one launch loads this code object
__global__ void k_warm_srs() {}
int warm_srs(hipStream_t st) {
  hipLaunchKernelGGL(k_warm_srs, dim3(1), dim3(64), 0, st);
  KZGX_TRY_HIP(hipGetLastError());
  return KZGX_OK;
}
}  // namespace kzgx
