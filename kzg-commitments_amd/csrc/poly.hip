// Scalar-field (Fr) polynomial kernels for gfx950 -- the companion ops of
// the prove path (reference: src/trusted_setup.cpp:214-225 and
// src/util.cpp:172-284, NTL ZZ_pX arithmetic).
//
//  * k_quotient_single: q = (P - P(z)) / (X - z) and y = P(z) for a batch of
//    openings, one wavefront per opening.  The recurrence
//    q_{k-1} = p_k + z q_k is split into 64 lane chunks: local Horner sums,
//    a 6-step wave scan of the carries (c_g += z^(L 2^s) c_{g+2^s}), then each
//    lane replays its chunk from its carry-in.  Depth 2L + 6 mulmods instead
//    of n.
//  * k_poly_eval: Horner, one thread per evaluation point.
//  * interpolation (polyfit): Z = prod (X - x_i) by a product tree, weights
//    a_i = y_i / prod_{j != i}(x_i - x_j), power moments m_t = sum_i a_i x_i^t,
//    and c_k = sum_{j > k} z_j m_{j-k-1}; every sum is a wavefront reduction.
//    Result = the unique interpolant, identical to NTL's subproduct-tree fit.
//
// Canonical inputs are multiplied by Montgomery-form constants with fe_mul,
// which yields canonical results (a * bR * R^-1 = ab), so no conversions are
// needed on the streaming paths.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include <algorithm>

#include <utility>

#include "field.hpp"
#include "field29.hpp"
#include "kzgx_internal.hpp"
#include "kzgx_setup.hpp"

namespace kzgx {

template <class FR>
KZGX_DEV Fe<FR> fe_shfl_down(const Fe<FR>& a, int d) {
  Fe<FR> r;
#pragma unroll
  for (int i = 0; i < FR::N; i++) r.v[i] = __shfl_down(a.v[i], d, 64);
  return r;
}

template <class FR>
KZGX_DEV Fe<FR> fe_shfl(const Fe<FR>& a, uint32_t src) {
  Fe<FR> r;
#pragma unroll
  for (int i = 0; i < FR::N; i++) r.v[i] = __shfl(a.v[i], (int)src, 64);
  return r;
}

template <class FR>
KZGX_DEV Fe<FR> fe_shfl_xor(const Fe<FR>& a, int m) {
  Fe<FR> r;
#pragma unroll
  for (int i = 0; i < FR::N; i++) r.v[i] = __shfl_xor(a.v[i], m, 64);
  return r;
}

template <class FR>
KZGX_DEV Fe<FR> wave_sum(Fe<FR> a) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) a = fe_add<FR>(a, fe_shfl_xor<FR>(a, m));
  return a;
}

// the scalar field's radix-2^29 twin (gen_consts.py)
template <class FR>
struct Fr29Of;
template <>
struct Fr29Of<BN254Fr> {
  using T = BN254Fr29;
};
template <>
struct Fr29Of<BLS12381Fr> {
  using T = BLS12381Fr29;
};

// a^-1 (inv(0) = 0) of lane 0's Montgomery value for the whole wave (every
// lane calls): the canonical value in radix 2^29 and Montgomery-29 form,
// Pornin's binary GCD with the bit-serial loop on the scalar ALU and the
// four linear combinations on four lanes (field29.hpp f29_inv_uniform_raw,
// ~30 us), back to a 32-bit-limb Montgomery value.  Variable time: public
// values only (the interpolation nodes).
template <class FR>
KZGX_DEV Fe<FR> fe_inv_wave(const Fe<FR>& a) {
  using F = typename Fr29Of<FR>::T;
  constexpr int N = FR::N;
  const Fe<FR> c = fe_from_mont<FR>(a);
  uint32_t w[N];
#pragma unroll
  for (int k = 0; k < N; k++) w[k] = __builtin_amdgcn_readfirstlane(c.v[k]);
  const F29<F> x = f29_mul<F>(f29_from_words<F, N>(w), f29_const<F>(F::R2));  // c R29
  const F29<F> i = f29_inv_uniform_raw<F, N>(x, FR::P);                      // c^-1, plain
  uint32_t o[N];
  f29_to_words<F, N>(f29_reduce<F>(i), o);
  Fe<FR> r;
#pragma unroll
  for (int k = 0; k < N; k++) r.v[k] = o[k];
  return fe_to_mont<FR>(r);
}

template <class FR>
KZGX_DEV Fe<FR> wave_prod(Fe<FR> a) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) a = fe_mul<FR>(a, fe_shfl_xor<FR>(a, m));
  return a;
}

// left-to-right square-and-multiply from the exponent's top set bit (the
// exponents here are chunk lengths, 3-10 bits: squaring the leading ones
// would be most of the work on the single-opening latency path)
template <class FR>
KZGX_DEV Fe<FR> fe_pow_u32(const Fe<FR>& base_m, uint32_t e) {
  if (e == 0) return fe_one<FR>();
  Fe<FR> acc = base_m;
  for (int b = 30 - __builtin_clz(e); b >= 0; b--) {
    acc = fe_sqr<FR>(acc);
    if ((e >> b) & 1u) acc = fe_mul<FR>(acc, base_m);
  }
  return acc;
}

// --------------------------------------------------------------------------
// single-opening quotient (create_proof(poly, z, 1), trusted_setup.cpp:214-225)
// --------------------------------------------------------------------------
template <class FR>
__global__ __launch_bounds__(256) void k_quotient_single(const uint32_t* __restrict__ coeffs, uint32_t n,
                                                         size_t cstride, const uint32_t* __restrict__ zs,
                                                         uint32_t batch, uint32_t* __restrict__ q, size_t qstride,
                                                         uint32_t* __restrict__ ys) {
  constexpr int N = FR::N;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t j = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (j >= batch) return;  // whole wavefront
  const uint32_t* P = coeffs + (size_t)j * cstride;
  const Fe<FR> zm = fe_to_mont<FR>(fe_load<FR>(zs + (size_t)j * N));
  const uint32_t L = (n + 63) / 64;
  const uint32_t lo = min(lane * L, n), hi = min(lo + L, n);
  // phase 1: local_g = sum_{k in chunk} p_k z^(k - lo)
  Fe<FR> h = fe_zero<FR>();
  for (uint32_t k = hi; k-- > lo;) h = fe_add<FR>(fe_load<FR>(P + (size_t)k * N), fe_mul<FR>(h, zm));
  // phase 2: c_g = sum_{u >= g} local_u z^(L (u - g))
  Fe<FR> c = h;
  Fe<FR> zp = fe_pow_u32<FR>(zm, L);
#pragma unroll
  for (int s = 0; s < 6; s++) {
    Fe<FR> o = fe_shfl_down<FR>(c, 1 << s);
    if (lane + (1u << s) < 64) c = fe_add<FR>(c, fe_mul<FR>(o, zp));  // canonical * Montgomery = canonical
    zp = fe_sqr<FR>(zp);
  }
  Fe<FR> cin = fe_shfl_down<FR>(c, 1);
  if (lane == 63) cin = fe_zero<FR>();
  // phase 3: replay the chunk from its carry-in, emitting q_{k-1}
  h = cin;
  uint32_t* Q = q + (size_t)j * qstride;
  for (uint32_t k = hi; k-- > lo;) {
    h = fe_add<FR>(fe_load<FR>(P + (size_t)k * N), fe_mul<FR>(h, zm));
    if (k >= 1)
      fe_store<FR>(Q + (size_t)(k - 1) * N, h);
    else if (ys)
      fe_store<FR>(ys + (size_t)j * N, h);
  }
  if (n == 0 && lane == 0 && ys) fe_store<FR>(ys + (size_t)j * N, fe_zero<FR>());
}

// Mid-size single openings (batch <= 4, 2^9 <= n <= 2^14): the three phases
// in ONE workgroup of NWV wavefronts per opening, so one launch and no global
// round trips.  Thread t owns [t L, t L + L), L = ceil(n / (64 NWV)):
//   local Horner; a wavefront suffix scan of (c, pw) with multiplier z^L, pw
//   = z^(L (63 - lane)) as a suffix product in the same 6 steps; the NWV
//   wavefront totals H_w through LDS, each wavefront scanning them itself
//   (log2 NWV steps, multiplier Z = z^(64 L), the scan's last power) into
//   C_w = h at the top of wavefront w and y = h_0; carry-in c_{t+1} + C_w pw;
//   replay.  NWV = 8 (two wavefronts per SIMD of the CU) by default: 4 is one
//   per SIMD with twice the chunk (9 us slower at degree 4096), 16 shares each
//   SIMD four ways and lost to the chip-wide kernel outright.
template <class FR, int NWV>
__global__ __launch_bounds__(64 * NWV) void k_quotient_wg(const uint32_t* __restrict__ coeffs, uint32_t n,
                                                          size_t cstride, const uint32_t* __restrict__ zs,
                                                          uint32_t* __restrict__ q, size_t qstride,
                                                          uint32_t* __restrict__ ys) {
  constexpr int N = FR::N;
  __shared__ uint32_t sh[NWV * N];
  const uint32_t j = blockIdx.x, t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const uint32_t* P = coeffs + (size_t)j * cstride;
  const Fe<FR> zm = fe_to_mont<FR>(fe_load<FR>(zs + (size_t)j * N));
  const uint32_t L = (n + 64 * NWV - 1) / (64 * NWV);
  const uint32_t lo = min(t * L, n), hi = min(lo + L, n);
  Fe<FR> h = fe_zero<FR>();
  for (uint32_t k = hi; k-- > lo;) h = fe_add<FR>(fe_load<FR>(P + (size_t)k * N), fe_mul<FR>(h, zm));
  const Fe<FR> zL = fe_pow_u32<FR>(zm, L);
  Fe<FR> c = h, zp = zL, pw = lane < 63 ? zL : fe_one<FR>();
#pragma unroll
  for (int s = 0; s < 6; s++) {
    const Fe<FR> o = fe_shfl_down<FR>(c, 1 << s), po = fe_shfl_down<FR>(pw, 1 << s);
    if (lane + (1u << s) < 64) {
      c = fe_add<FR>(c, fe_mul<FR>(o, zp));  // canonical * Montgomery = canonical
      pw = fe_mul<FR>(pw, po);
    }
    zp = fe_sqr<FR>(zp);
  }
  // zp = z^(64 L); c at lane 0 = the wavefront's total H_w
  if (lane == 0) fe_store<FR>(sh + wv * N, c);
  __syncthreads();
  Fe<FR> S = lane < NWV ? fe_load<FR>(sh + lane * N) : fe_zero<FR>();
  Fe<FR> Zp = zp;
#pragma unroll
  for (int s = 0; (1 << s) < NWV; s++) {
    const Fe<FR> o = fe_shfl_down<FR>(S, 1 << s);
    if (lane + (1u << s) < NWV) S = fe_add<FR>(S, fe_mul<FR>(o, Zp));
    Zp = fe_sqr<FR>(Zp);
  }
  // S at lane v = h at the bottom of wavefront v's span; C_w = S_(w+1)
  const Fe<FR> Cw = fe_shfl<FR>(S, wv + 1 < NWV ? wv + 1 : NWV);  // lane NWV holds zero
  const Fe<FR> cn = fe_shfl_down<FR>(c, 1);
  h = fe_mul<FR>(Cw, pw);
  if (lane < 63) h = fe_add<FR>(h, cn);
  uint32_t* Q = q + (size_t)j * qstride;
  for (uint32_t k = hi; k-- > lo;) {
    h = fe_add<FR>(fe_load<FR>(P + (size_t)k * N), fe_mul<FR>(h, zm));
    if (k >= 1)
      fe_store<FR>(Q + (size_t)(k - 1) * N, h);
    else if (ys)
      fe_store<FR>(ys + (size_t)j * N, h);
  }
}

// Large single openings (batch <= 4, n >= 2^13): the same three phases spread
// over the whole chip instead of one wavefront.  Lane t of the grid owns
// coefficients [t L, t L + L) (zeros past n); with h_k = sum_{i >= k} p_i z^(i-k)
// (q_{k-1} = h_k, y = h_0):
//   k_qbig_local : lane-local Horner, then a wavefront suffix scan with
//                  multiplier z^L -> c_t (the wavefront-local h at t L) and
//                  the wavefront total H_g;
//   k_qbig_scan  : one workgroup scans the G totals with multiplier z^(64 L)
//                  -> C_g = h at the top of wavefront g, and y;
//   k_qbig_replay: lane carry-in c_{t+1} + z^(L (63 - l)) C_g, then the
//                  chunk replayed, emitting q.
template <class FR>
__global__ __launch_bounds__(256) void k_qbig_local(const uint32_t* __restrict__ P, uint32_t n,
                                                    const uint32_t* __restrict__ z, uint32_t L,
                                                    uint32_t* __restrict__ cl, uint32_t* __restrict__ H) {
  constexpr int N = FR::N;
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t lane = threadIdx.x & 63;
  const Fe<FR> zm = fe_to_mont<FR>(fe_load<FR>(z));
  const uint64_t lo64 = (uint64_t)t * L;
  const uint32_t lo = (uint32_t)(lo64 < n ? lo64 : n), hi = (uint32_t)(lo64 + L < n ? lo64 + L : n);
  Fe<FR> h = fe_zero<FR>();
  for (uint32_t k = hi; k-- > lo;) h = fe_add<FR>(fe_load<FR>(P + (size_t)k * N), fe_mul<FR>(h, zm));
  Fe<FR> c = h;
  Fe<FR> zp = fe_pow_u32<FR>(zm, L);
#pragma unroll
  for (int s = 0; s < 6; s++) {
    Fe<FR> o = fe_shfl_down<FR>(c, 1 << s);
    if (lane + (1u << s) < 64) c = fe_add<FR>(c, fe_mul<FR>(o, zp));
    zp = fe_sqr<FR>(zp);
  }
  fe_store<FR>(cl + (size_t)t * N, c);
  if (lane == 0) fe_store<FR>(H + (size_t)(t >> 6) * N, c);
}

template <class FR>
__global__ __launch_bounds__(256) void k_qbig_scan(const uint32_t* __restrict__ H, uint32_t G,
                                                   const uint32_t* __restrict__ z, uint32_t L,
                                                   uint32_t* __restrict__ Cg, uint32_t* __restrict__ y) {
  constexpr int N = FR::N;
  __shared__ uint32_t sh[256 * N];
  const uint32_t t = threadIdx.x;
  const Fe<FR> zm = fe_to_mont<FR>(fe_load<FR>(z));
  const Fe<FR> Z = fe_pow_u32<FR>(zm, 64u * L);  // one wavefront's span
  const uint32_t per = (G + 255) / 256;
  const uint32_t g0 = min(t * per, G), g1 = min(g0 + per, G);
  Fe<FR> u = fe_zero<FR>();
  for (uint32_t g = g1; g-- > g0;) u = fe_add<FR>(fe_load<FR>(H + (size_t)g * N), fe_mul<FR>(u, Z));
  // S_t = sum_{t' >= t} u_t' Z^(per (t' - t)), Hillis-Steele over LDS
  Fe<FR> S = u;
  Fe<FR> Zp = fe_pow_u32<FR>(Z, per);
  for (uint32_t d = 1; d < 256; d <<= 1) {
    fe_store<FR>(sh + t * N, S);
    __syncthreads();
    if (t + d < 256) S = fe_add<FR>(S, fe_mul<FR>(fe_load<FR>(sh + (t + d) * N), Zp));
    __syncthreads();
    Zp = fe_sqr<FR>(Zp);
  }
  fe_store<FR>(sh + t * N, S);
  __syncthreads();
  Fe<FR> K = t + 1 < 256 ? fe_load<FR>(sh + (t + 1) * N) : fe_zero<FR>();
  // K = h at the top of this thread's range (ranges start at multiples of
  // per; only the last non-empty one can be short, and it has no successor)
  for (uint32_t g = g1; g-- > g0;) {
    fe_store<FR>(Cg + (size_t)g * N, K);
    K = fe_add<FR>(fe_load<FR>(H + (size_t)g * N), fe_mul<FR>(K, Z));
  }
  if (t == 0 && y) fe_store<FR>(y, K);
}

template <class FR>
__global__ __launch_bounds__(256) void k_qbig_replay(const uint32_t* __restrict__ P, uint32_t n,
                                                     const uint32_t* __restrict__ z, uint32_t L,
                                                     const uint32_t* __restrict__ cl, const uint32_t* __restrict__ Cg,
                                                     uint32_t* __restrict__ q) {
  constexpr int N = FR::N;
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t lo64 = (uint64_t)t * L;
  if (lo64 >= n) return;
  const uint32_t lo = (uint32_t)lo64, hi = (uint32_t)(lo64 + L < n ? lo64 + L : n);
  const Fe<FR> zm = fe_to_mont<FR>(fe_load<FR>(z));
  Fe<FR> h = fe_mul<FR>(fe_load<FR>(Cg + (size_t)(t >> 6) * N), fe_pow_u32<FR>(zm, L * (63u - lane)));
  if (lane < 63) h = fe_add<FR>(h, fe_load<FR>(cl + (size_t)(t + 1) * N));
  for (uint32_t k = hi; k-- > lo;) {
    h = fe_add<FR>(fe_load<FR>(P + (size_t)k * N), fe_mul<FR>(h, zm));
    if (k >= 1) fe_store<FR>(q + (size_t)(k - 1) * N, h);
  }
}

// --------------------------------------------------------------------------
// evaluation at m points (evaluate_polynomial_points, util.cpp:186-211)
// --------------------------------------------------------------------------
template <class FR>
__global__ __launch_bounds__(256) void k_poly_eval(const uint32_t* __restrict__ coeffs, uint32_t n,
                                                   const uint32_t* __restrict__ xs, uint32_t m,
                                                   uint32_t* __restrict__ ys) {
  constexpr int N = FR::N;
  uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= m) return;
  const Fe<FR> xm = fe_to_mont<FR>(fe_load<FR>(xs + (size_t)j * N));
  Fe<FR> h = fe_zero<FR>();
  for (uint32_t k = n; k-- > 0;) h = fe_add<FR>(fe_load<FR>(coeffs + (size_t)k * N), fe_mul<FR>(h, xm));
  fe_store<FR>(ys + (size_t)j * N, h);
}

// --------------------------------------------------------------------------
// interpolation (polyfit, util.cpp:172-184 / polyfit_R :213-248)
// --------------------------------------------------------------------------
template <class FR>
__global__ void k_to_mont(const uint32_t* __restrict__ in, uint32_t* __restrict__ out, uint32_t n) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) fe_store<FR>(out + (size_t)i * FR::N, fe_to_mont<FR>(fe_load<FR>(in + (size_t)i * FR::N)));
}

template <class FR>
__global__ void k_from_mont(const uint32_t* __restrict__ in, uint32_t* __restrict__ out, uint32_t n) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) fe_store<FR>(out + (size_t)i * FR::N, fe_from_mont<FR>(fe_load<FR>(in + (size_t)i * FR::N)));
}

// level 0 of the product tree: slot i = (X - x_i), 2 coefficients
template <class FR>
__global__ void k_tree_leaves(const uint32_t* __restrict__ xm, uint32_t n, uint32_t* __restrict__ lvl) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  fe_store<FR>(lvl + (size_t)(2 * i) * FR::N, fe_neg<FR>(fe_load<FR>(xm + (size_t)i * FR::N)));
  fe_store<FR>(lvl + (size_t)(2 * i + 1) * FR::N, fe_one<FR>());
}

// level l -> l+1: slot j = slot 2j * slot 2j+1.  Input slots hold s+1
// coefficients (s = 2^l nodes, fewer in the last slot: its degree is
// cnt = min(s, n - j s)); one wavefront per output coefficient.
template <class FR>
__global__ __launch_bounds__(256) void k_tree_mul(const uint32_t* __restrict__ in, uint32_t s, uint32_t n,
                                                  uint32_t* __restrict__ out, uint32_t nslots_out) {
  constexpr int N = FR::N;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t gw = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const uint32_t S = 2 * s;  // nodes per output slot
  const uint64_t j = gw / (S + 1), k = gw % (S + 1);
  if (j >= nslots_out) return;
  const uint32_t base = (uint32_t)j * S;
  const uint32_t da = min(s, n - base);                        // degree of left factor
  const uint32_t db = base + s < n ? min(s, n - base - s) : 0;  // degree of right (0 -> constant 1)
  const bool has_b = base + s < n;
  const uint32_t* A = in + (size_t)(2 * j) * (s + 1) * N;
  const uint32_t* B = in + (size_t)(2 * j + 1) * (s + 1) * N;
  Fe<FR> acc = fe_zero<FR>();
  if (k <= da + db) {
    if (has_b) {
      const uint32_t i0 = k > db ? (uint32_t)k - db : 0, i1 = min((uint32_t)k, da);
      for (uint32_t i = i0 + lane; i <= i1; i += 64)
        acc = fe_add<FR>(acc, fe_mul<FR>(fe_load<FR>(A + (size_t)i * N), fe_load<FR>(B + (size_t)(k - i) * N)));
    } else if (lane == 0) {
      acc = fe_load<FR>(A + (size_t)k * N);
    }
  }
  acc = wave_sum<FR>(acc);
  if (lane == 0) fe_store<FR>(out + ((size_t)j * (S + 1) + k) * N, acc);
}

// a_i = y_i / prod_{j != i} (x_i - x_j); one wavefront per node; flags duplicates
template <class FR>
__global__ __launch_bounds__(256) void k_interp_weights(const uint32_t* __restrict__ xm, const uint32_t* __restrict__ ym,
                                                        uint32_t n, uint32_t* __restrict__ a, uint32_t* err) {
  constexpr int N = FR::N;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t i = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= n) return;
  const Fe<FR> xi = fe_load<FR>(xm + (size_t)i * N);
  Fe<FR> p = fe_one<FR>();
  for (uint32_t j = lane; j < n; j += 64)
    if (j != i) p = fe_mul<FR>(p, fe_sub<FR>(xi, fe_load<FR>(xm + (size_t)j * N)));
  p = wave_prod<FR>(p);  // in every lane (xor butterfly)
  // the nodes are public (opening points): the variable-time inverse, by the
  // whole wave (round 5: a Fermat chain in lane 0, 1.65 ms at 128 points)
  const Fe<FR> pi = fe_inv_wave<FR>(p);
  if (lane == 0) {
    if (fe_is_zero<FR>(p)) atomicOr(err, 1u);
    fe_store<FR>(a + (size_t)i * N, fe_mul<FR>(fe_load<FR>(ym + (size_t)i * N), pi));
  }
}

// partial moments: part[it][t] = sum_{i in tile it} a_i x_i^t, t in [t0, t0+TT)
constexpr int MOM_TT = 64;
template <class FR>
__global__ __launch_bounds__(256) void k_moments(const uint32_t* __restrict__ xm, const uint32_t* __restrict__ a,
                                                 uint32_t n, uint32_t* __restrict__ part) {
  constexpr int N = FR::N;
  __shared__ uint32_t red[4][MOM_TT][N];
  const uint32_t t0 = blockIdx.x * MOM_TT;
  const uint32_t it = blockIdx.y;
  const uint32_t i = it * 256 + threadIdx.x;
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  Fe<FR> x = fe_zero<FR>(), v = fe_zero<FR>();
  if (i < n) {
    x = fe_load<FR>(xm + (size_t)i * N);
    // v = a_i x_i^t0: x_i^t0 via square-and-multiply
    v = fe_mul<FR>(fe_load<FR>(a + (size_t)i * N), fe_pow_u32<FR>(x, t0));
  }
  for (int tt = 0; tt < MOM_TT; tt++) {
    Fe<FR> s = wave_sum<FR>(v);
    if (lane == 0) {
#pragma unroll
      for (int w = 0; w < N; w++) red[wave][tt][w] = s.v[w];
    }
    v = fe_mul<FR>(v, x);
  }
  __syncthreads();
  if (threadIdx.x < MOM_TT && t0 + threadIdx.x < n) {
    Fe<FR> s = fe_zero<FR>();
    for (int w = 0; w < 4; w++) {
      Fe<FR> o;
#pragma unroll
      for (int q = 0; q < N; q++) o.v[q] = red[w][threadIdx.x][q];
      s = fe_add<FR>(s, o);
    }
    fe_store<FR>(part + ((size_t)it * n + t0 + threadIdx.x) * N, s);
  }
}

template <class FR>
__global__ void k_moments_sum(const uint32_t* __restrict__ part, uint32_t n, uint32_t ntiles, uint32_t* __restrict__ m) {
  uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  Fe<FR> s = fe_zero<FR>();
  for (uint32_t it = 0; it < ntiles; it++) s = fe_add<FR>(s, fe_load<FR>(part + ((size_t)it * n + t) * FR::N));
  fe_store<FR>(m + (size_t)t * FR::N, s);
}

// c_k = sum_{j=k+1}^{n} z_j m_{j-k-1}; one wavefront per coefficient; canonical out
template <class FR>
__global__ __launch_bounds__(256) void k_interp_coeffs(const uint32_t* __restrict__ Z, const uint32_t* __restrict__ m,
                                                       uint32_t n, uint32_t* __restrict__ coeffs) {
  constexpr int N = FR::N;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t k = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (k >= n) return;
  Fe<FR> acc = fe_zero<FR>();
  for (uint32_t j = k + 1 + lane; j <= n; j += 64)
    acc = fe_add<FR>(acc, fe_mul<FR>(fe_load<FR>(Z + (size_t)j * N), fe_load<FR>(m + (size_t)(j - k - 1) * N)));
  acc = wave_sum<FR>(acc);
  if (lane == 0) fe_store<FR>(coeffs + (size_t)k * N, fe_from_mont<FR>(acc));
}

// --------------------------------------------------------------------------
// host side
// --------------------------------------------------------------------------
template <class FR>
static int quotient_single_impl(Ctx* ctx, const uint32_t* d_coeffs, size_t n, size_t cstride, const uint32_t* d_z, size_t batch,
                                uint32_t* d_q, size_t qstride, uint32_t* d_y, hipStream_t st) {
  if (batch == 0) return KZGX_OK;
  ProfScope prof(ctx, st, "quotient_single");
  // from QBIG_N coefficients a single opening spreads over the chip: a
  // degree-4096 create_proof(poly, z, 1) 0.69-0.73 ms with the one-wavefront
  // kernel, 0.60-0.67 ms chip-wide (profiles/r03_latency_window.json;
  // KZGX_QBIG_N overrides, for A/B)
  static const size_t QBIG_N = [] {
    const char* e = std::getenv("KZGX_QBIG_N");
    return e && *e ? (size_t)std::strtoull(e, nullptr, 10) : (size_t)1u << 11;
  }();
  constexpr size_t QBIG_LANES = 1u << 18;  // 4096 wavefronts: 4 per SIMD
  // one workgroup per opening from QWG_MIN to 2^14 coefficients
  // (k_quotient_wg; KZGX_QWG_MIN overrides, 0 = never, for A/B)
  static const size_t QWG_MIN = [] {
    const char* e = std::getenv("KZGX_QWG_MIN");
    return e && *e ? (size_t)std::strtoull(e, nullptr, 10) : (size_t)512;
  }();
  if (batch <= 4 && QWG_MIN && n >= QWG_MIN && n <= (1u << 14)) {
    // 8 wavefronts (two per SIMD, half the chunk length): degree-4096 proof
    // -9 us against 4 (profiles/r04_lat_ab_q64_qwg8.txt); KZGX_QWG_WAVES=4
    // selects 4 (A/B)
    static const bool w8 = !(std::getenv("KZGX_QWG_WAVES") && std::strtoul(std::getenv("KZGX_QWG_WAVES"), nullptr, 10) == 4);
    if (w8)
      hipLaunchKernelGGL((k_quotient_wg<FR, 8>), dim3((unsigned)batch), dim3(512), 0, st, d_coeffs, (uint32_t)n,
                         cstride, d_z, d_q, qstride, d_y);
    else
      hipLaunchKernelGGL((k_quotient_wg<FR, 4>), dim3((unsigned)batch), dim3(256), 0, st, d_coeffs, (uint32_t)n,
                         cstride, d_z, d_q, qstride, d_y);
    KZGX_TRY_HIP(hipGetLastError());
    return KZGX_OK;
  }
  if (batch <= 4 && n >= QBIG_N) {
    constexpr int N = FR::N;
    const uint32_t L = (uint32_t)std::max<size_t>(8, (n + QBIG_LANES - 1) / QBIG_LANES);
    const size_t T = (n + L - 1) / L;
    const size_t Tw = (T + 255) / 256 * 256;  // whole workgroups
    const size_t G = Tw / 64;
    WsLease ws = ctx->ws_for(st);
    if (!ws) return KZGX_ERR_ARG;
    KZGX_TRY(dev_alloc(ctx, (void**)&ws->qbig, (Tw + 2 * G) * N * sizeof(uint32_t), &ws->qbig_b));
    uint32_t* cl = ws->qbig;
    uint32_t* H = cl + Tw * N;
    uint32_t* Cg = H + G * N;
    for (size_t j = 0; j < batch; j++) {
      const uint32_t* P = d_coeffs + j * cstride;
      const uint32_t* z = d_z + j * N;
      hipLaunchKernelGGL(k_qbig_local<FR>, dim3((unsigned)(Tw / 256)), dim3(256), 0, st, P, (uint32_t)n, z, L, cl, H);
      hipLaunchKernelGGL(k_qbig_scan<FR>, dim3(1), dim3(256), 0, st, H, (uint32_t)G, z, L, Cg,
                         d_y ? d_y + j * N : nullptr);
      if (n > 1)
        hipLaunchKernelGGL(k_qbig_replay<FR>, dim3((unsigned)(Tw / 256)), dim3(256), 0, st, P, (uint32_t)n, z, L,
                           cl, Cg, d_q + j * qstride);
    }
    KZGX_TRY_HIP(hipGetLastError());
    return KZGX_OK;
  }
  hipLaunchKernelGGL(k_quotient_single<FR>, dim3((unsigned)((batch + 3) / 4)), dim3(256), 0, st, d_coeffs,
                     (uint32_t)n, cstride, d_z, (uint32_t)batch, d_q, qstride, d_y);
  KZGX_TRY_HIP(hipGetLastError());
  return KZGX_OK;
}

int quotient_single(Ctx* ctx, const uint32_t* d_coeffs, size_t n, size_t coeff_stride_words, const uint32_t* d_z,
                    size_t batch, uint32_t* d_q, size_t q_stride_words, uint32_t* d_y, hipStream_t st) {
  return ctx->curve == KZGX_CURVE_BN254
             ? quotient_single_impl<BN254Fr>(ctx, d_coeffs, n, coeff_stride_words, d_z, batch, d_q, q_stride_words, d_y, st)
             : quotient_single_impl<BLS12381Fr>(ctx, d_coeffs, n, coeff_stride_words, d_z, batch, d_q, q_stride_words, d_y,
                                                st);
}

template <class FR>
static int poly_eval_impl(const uint32_t* d_coeffs, size_t n, const uint32_t* d_x, size_t m, uint32_t* d_y,
                          hipStream_t st) {
  if (m == 0) return KZGX_OK;
  hipLaunchKernelGGL(k_poly_eval<FR>, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, st, d_coeffs, (uint32_t)n, d_x,
                     (uint32_t)m, d_y);
  KZGX_TRY_HIP(hipGetLastError());
  return KZGX_OK;
}

int poly_eval(Ctx* ctx, const uint32_t* d_coeffs, size_t n, const uint32_t* d_x, size_t m, uint32_t* d_y,
              hipStream_t st) {
  return ctx->curve == KZGX_CURVE_BN254 ? poly_eval_impl<BN254Fr>(d_coeffs, n, d_x, m, d_y, st)
                                        : poly_eval_impl<BLS12381Fr>(d_coeffs, n, d_x, m, d_y, st);
}

template <class FR>
static int interpolate_impl(Ctx* ctx, const uint32_t* d_x, const uint32_t* d_y, size_t n, uint32_t* d_coeffs, hipStream_t st) {
  constexpr int N = FR::N;
  const size_t eb = N * sizeof(uint32_t);
  if (n == 0) return KZGX_OK;
  // workspace: xm, ym, a, m (n each), Z-tree ping/pong (<= 2n + nslots), partials, err
  size_t tiles = (n + 255) / 256;
  size_t lvl_elems = 2 * n + 2;  // each level stores nslots * (s+1) <= n + nslots <= 2n coefficients
  uint32_t *xm, *ym, *a, *mm, *L0, *L1, *part, *err;
  size_t total = (4 * n + 2 * lvl_elems + tiles * n) * eb + 256;
  char* base;
  KZGX_TRY(dev_alloc(ctx, &ctx->d_poly_ws, total, &ctx->poly_ws_b));
  base = (char*)ctx->d_poly_ws;
  xm = (uint32_t*)base;
  ym = xm + n * N;
  a = ym + n * N;
  mm = a + n * N;
  L0 = mm + n * N;
  L1 = L0 + lvl_elems * N;
  part = L1 + lvl_elems * N;
  err = part + tiles * n * N;
  KZGX_TRY_HIP(hipMemsetAsync(err, 0, 4, st));
  const unsigned g1 = (unsigned)((n + 255) / 256);
  hipLaunchKernelGGL(k_to_mont<FR>, dim3(g1), dim3(256), 0, st, d_x, xm, (uint32_t)n);
  hipLaunchKernelGGL(k_to_mont<FR>, dim3(g1), dim3(256), 0, st, d_y, ym, (uint32_t)n);
  // product tree
  hipLaunchKernelGGL(k_tree_leaves<FR>, dim3(g1), dim3(256), 0, st, xm, (uint32_t)n, L0);
  uint32_t* cur = L0;
  uint32_t* nxt = L1;
  size_t s = 1;
  while (s < n) {
    size_t nslots_out = (n + 2 * s - 1) / (2 * s);
    size_t waves = nslots_out * (2 * s + 1);
    hipLaunchKernelGGL(k_tree_mul<FR>, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, st, cur, (uint32_t)s,
                       (uint32_t)n, nxt, (uint32_t)nslots_out);
    uint32_t* t = cur;
    cur = nxt;
    nxt = t;
    s *= 2;
  }
  // cur: one slot of s+1 coefficients, Z has degree n (entries above n unused)
  hipLaunchKernelGGL(k_interp_weights<FR>, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, st, xm, ym, (uint32_t)n, a,
                     err);
  hipLaunchKernelGGL(k_moments<FR>, dim3((unsigned)((n + MOM_TT - 1) / MOM_TT), (unsigned)tiles), dim3(256), 0, st,
                     xm, a, (uint32_t)n, part);
  hipLaunchKernelGGL(k_moments_sum<FR>, dim3(g1), dim3(256), 0, st, part, (uint32_t)n, (uint32_t)tiles, mm);
  hipLaunchKernelGGL(k_interp_coeffs<FR>, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, st, cur, mm, (uint32_t)n,
                     d_coeffs);
  KZGX_TRY_HIP(hipGetLastError());
  uint32_t h_err = 0;
  KZGX_TRY_HIP(hipMemcpyAsync(&h_err, err, 4, hipMemcpyDeviceToHost, st));
  KZGX_TRY_HIP(hipStreamSynchronize(st));
  return h_err ? KZGX_ERR_DIV_ZERO : KZGX_OK;
}

template <class FR>
static uint32_t* vanishing_mont(const uint32_t* d_x, size_t n, uint32_t* ws, hipStream_t st);

template <class FR>
static int vanishing_impl(Ctx* ctx, const uint32_t* d_x, size_t n, uint32_t* d_Z, hipStream_t st) {
  constexpr int N = FR::N;
  const size_t eb = N * sizeof(uint32_t);
  KZGX_TRY(dev_alloc(ctx, &ctx->d_poly_ws, (n + 2 * (2 * n + 2)) * eb, &ctx->poly_ws_b));
  uint32_t* Z = vanishing_mont<FR>(d_x, n, (uint32_t*)ctx->d_poly_ws, st);
  hipLaunchKernelGGL(k_from_mont<FR>, dim3((unsigned)((n + 1 + 255) / 256)), dim3(256), 0, st, Z, d_Z,
                     (uint32_t)(n + 1));
  KZGX_TRY_HIP(hipGetLastError());
  return KZGX_OK;
}

int poly_vanishing(Ctx* ctx, const uint32_t* d_x, size_t n, uint32_t* d_Z, hipStream_t st) {
  return ctx->curve == KZGX_CURVE_BN254 ? vanishing_impl<BN254Fr>(ctx, d_x, n, d_Z, st)
                                        : vanishing_impl<BLS12381Fr>(ctx, d_x, n, d_Z, st);
}

// the multi-point verify's scalar-field and G2 workspaces for up to n points
// (interpolate_impl's layout, the larger of its two users), made at setup so
// the first verify_proof(poly, 0, N) grows nothing
int verify_ws_reserve(Ctx* ctx, size_t n) {
  static_assert(BN254Fr::N == 8 && BLS12381Fr::N == 8, "Fr elements of 8 words");
  const size_t eb = 8 * sizeof(uint32_t);
  const size_t tiles = (n + 255) / 256, lvl = 2 * n + 2;
  KZGX_TRY(dev_alloc(ctx, &ctx->d_poly_ws, (4 * n + 2 * lvl + tiles * n) * eb + 256, &ctx->poly_ws_b));
  return g2_ws_reserve(ctx, n + 1);
}

int poly_interpolate(Ctx* ctx, const uint32_t* d_x, const uint32_t* d_y, size_t n, uint32_t* d_coeffs,
                     hipStream_t st) {
  return ctx->curve == KZGX_CURVE_BN254 ? interpolate_impl<BN254Fr>(ctx, d_x, d_y, n, d_coeffs, st)
                                        : interpolate_impl<BLS12381Fr>(ctx, d_x, d_y, n, d_coeffs, st);
}

// --------------------------------------------------------------------------
// multi-point opening: q = (P - I) / Z  (trusted_setup.cpp:225, NTL sub + div)
// --------------------------------------------------------------------------
// out[j] = in[n_in - 1 - j] for j < cnt (zero where the source index is
// negative): the reversal X^(n_in - 1) A(1 / X), truncated to cnt terms
template <class FR>
__global__ void k_fr_rev(const uint32_t* __restrict__ in, uint32_t n_in, uint32_t* __restrict__ out, uint32_t cnt) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= cnt) return;
  fe_store<FR>(out + (size_t)j * FR::N, j < n_in ? fe_load<FR>(in + (size_t)(n_in - 1 - j) * FR::N) : fe_zero<FR>());
}

// truncated product, one wavefront per output coefficient:
//   out[k] = (neg ? -1 : 1) sum_{i + j = k - shift} A_i B_j,   k in [k0, k1)
// A_i (i < na) and B_j (j < nb); one operand canonical and the other in
// Montgomery form gives a canonical result (both Montgomery: Montgomery).
template <class FR>
__global__ __launch_bounds__(256) void k_conv(const uint32_t* __restrict__ A, uint32_t na,
                                              const uint32_t* __restrict__ B, uint32_t nb, uint32_t* __restrict__ out,
                                              uint32_t k0, uint32_t k1, uint32_t shift, int neg) {
  constexpr int N = FR::N;
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t k = k0 + blockIdx.x * 4 + (threadIdx.x >> 6);
  if (k >= k1) return;  // whole wavefront
  const uint32_t t = k - shift;
  const uint32_t i0 = t + 1 > nb ? t + 1 - nb : 0, i1 = min(t, na - 1);
  Fe<FR> acc = fe_zero<FR>();
  for (uint32_t i = i0 + lane; i <= i1; i += 64)
    acc = fe_add<FR>(acc, fe_mul<FR>(fe_load<FR>(A + (size_t)i * N), fe_load<FR>(B + (size_t)(t - i) * N)));
  acc = wave_sum<FR>(acc);
  if (lane == 0) fe_store<FR>(out + (size_t)k * N, neg ? fe_neg<FR>(acc) : acc);
}

template <class FR>
static void launch_conv(const uint32_t* A, size_t na, const uint32_t* B, size_t nb, uint32_t* out, size_t k0, size_t k1,
                        size_t shift, bool neg, hipStream_t st) {
  if (k1 <= k0) return;
  hipLaunchKernelGGL(k_conv<FR>, dim3((unsigned)((k1 - k0 + 3) / 4)), dim3(256), 0, st, A, (uint32_t)na, B,
                     (uint32_t)nb, out, (uint32_t)k0, (uint32_t)k1, (uint32_t)shift, neg ? 1 : 0);
}

// vanishing polynomial Z = prod (X - x_i) in Montgomery form (product tree
// over the context's scratch); returns the slot holding Z's n + 1
// coefficients.  ws must hold n + 2 (2 n + 2) elements.
template <class FR>
static uint32_t* vanishing_mont(const uint32_t* d_x, size_t n, uint32_t* ws, hipStream_t st) {
  constexpr int N = FR::N;
  const size_t lvl_elems = 2 * n + 2;
  uint32_t* xm = ws;
  uint32_t* L0 = xm + n * N;
  uint32_t* L1 = L0 + lvl_elems * N;
  const unsigned g1 = (unsigned)((n + 255) / 256);
  hipLaunchKernelGGL(k_to_mont<FR>, dim3(g1), dim3(256), 0, st, d_x, xm, (uint32_t)n);
  hipLaunchKernelGGL(k_tree_leaves<FR>, dim3(g1), dim3(256), 0, st, xm, (uint32_t)n, L0);
  uint32_t* cur = L0;
  uint32_t* nxt = L1;
  for (size_t s = 1; s < n; s *= 2) {
    size_t nslots_out = (n + 2 * s - 1) / (2 * s);
    size_t waves = nslots_out * (2 * s + 1);
    hipLaunchKernelGGL(k_tree_mul<FR>, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, st, cur, (uint32_t)s,
                       (uint32_t)n, nxt, (uint32_t)nslots_out);
    std::swap(cur, nxt);
  }
  return cur;
}

// Multi-point quotient without interpolation.  For the points x_0..x_{N-1},
// I = P mod Z (I agrees with P on every x_i and deg I < N), so the
// reference's (P - I) / Z (trusted_setup.cpp:225, NTL sub + div) is exactly
// the polynomial quotient P div Z.  With m = n - N quotient coefficients and
// rev_k(A) = X^k A(1/X):
//   rev_{m-1}(q) = rev_{n-1}(P) * rev_N(Z)^-1  mod X^m
// (the remainder term carries a factor X^m).  rev_N(Z) has constant term 1
// (Z is monic), so its inverse mod X^m comes from Newton's iteration
//   S_{2l} = S_l - S_l ((rev Z) S_l - 1)   mod X^{2l},
// every step two truncated products of one wavefront per output coefficient
// (BN254's r - 1 has 2-adicity 2: no NTT domain, and at these sizes the
// parallel schoolbook products are a fraction of the MSM anyway).
//
// For few points on a long polynomial the Newton route costs ~1.8 m^2
// products while dividing by the len linear factors one after the other
// (floor division by monic factors composes: P div (X - x_0) div (X - x_1)
// ... = P div Z) costs len synthetic divisions of O(n) each, on the chip-wide
// single-opening quotient (quotient_single_impl: k_qbig_* from 2^13
// coefficients).  The division chain is sequential, so Newton (fully
// parallel) stays for len comparable to m.
template <class FR>
static bool prove_range_by_division(size_t n, size_t len) {
  const size_t m = n - len;
  return len <= 4 || (double)m * (double)m > 64.0 * (double)len * (double)n;
}

template <class FR>
static int prove_range_poly_impl(Ctx* ctx, const uint32_t* d_P, size_t n, const uint32_t* d_x, size_t len,
                                 uint32_t* d_q, size_t* nq_out, hipStream_t st) {
  constexpr int N = FR::N;
  const size_t eb = N * 4;
  *nq_out = 0;
  if (n <= len) return KZGX_OK;  // deg P < len: I = P, q = 0 (NTL normalizes to the zero polynomial)
  const size_t m = n - len;
  if (prove_range_by_division<FR>(n, len)) {
    // Intermediate quotients ping-pong between two scratch halves of n - 1
    // coefficients each; only the last division (m coefficients) writes d_q,
    // which the caller sizes for exactly m.
    KZGX_TRY(dev_alloc(ctx, &ctx->d_poly_ws2, 2 * (n - 1) * eb, &ctx->poly_ws2_b));
    uint32_t* half[2] = {(uint32_t*)ctx->d_poly_ws2, (uint32_t*)ctx->d_poly_ws2 + (n - 1) * N};
    const uint32_t* cur = d_P;
    size_t ncur = n;
    for (size_t i = 0; i < len; i++) {
      uint32_t* dst = i + 1 == len ? d_q : half[i & 1];
      KZGX_TRY(quotient_single_impl<FR>(ctx, cur, ncur, 0, d_x + i * N, 1, dst, 0, nullptr, st));
      cur = dst;
      ncur--;
    }
    *nq_out = m;
    return KZGX_OK;
  }
  // workspace: tree (len + 2 (2 len + 2)), Rz, S, E, Prev, Qrev (m each)
  const size_t tree = len + 2 * (2 * len + 2);
  KZGX_TRY(dev_alloc(ctx, &ctx->d_poly_ws2, (tree + 5 * m) * eb, &ctx->poly_ws2_b));
  uint32_t* base = (uint32_t*)ctx->d_poly_ws2;
  uint32_t* Zm = vanishing_mont<FR>(d_x, len, base, st);
  uint32_t* Rz = base + tree * N;
  uint32_t* S = Rz + m * N;
  uint32_t* E = S + m * N;
  uint32_t* Prev = E + m * N;
  uint32_t* Qrev = Prev + m * N;
  const size_t nrz = std::min(len + 1, m);
  const unsigned gm = (unsigned)((m + 255) / 256);
  hipLaunchKernelGGL(k_fr_rev<FR>, dim3((unsigned)((nrz + 255) / 256)), dim3(256), 0, st, Zm, (uint32_t)(len + 1), Rz,
                     (uint32_t)nrz);
  hipLaunchKernelGGL(k_fr_rev<FR>, dim3(gm), dim3(256), 0, st, d_P, (uint32_t)n, Prev, (uint32_t)m);
  // S = 1 (Montgomery) mod X^1, then Newton to m terms
  hipLaunchKernelGGL(k_fr_rev<FR>, dim3(1), dim3(64), 0, st, Zm + len * N, 1u, S, 1u);  // Z_len = 1 (monic)
  for (size_t l = 1; l < m;) {
    const size_t l2 = std::min(2 * l, m);
    // E_k = ((rev Z) S)_k for k in [l, l2): the coefficients of (rev Z) S - 1 that are not yet zero
    launch_conv<FR>(S, l, Rz, nrz, E, l, l2, 0, false, st);
    // S_k = -(S (E X^l))_k = -sum_i S_i E_{k-i} for k in [l, l2)
    launch_conv<FR>(S, l, E + l * N, l2 - l, S, l, l2, l, true, st);
    l = l2;
  }
  // rev(q) = rev(P) S mod X^m (canonical * Montgomery = canonical), then q
  launch_conv<FR>(Prev, m, S, m, Qrev, 0, m, 0, false, st);
  hipLaunchKernelGGL(k_fr_rev<FR>, dim3(gm), dim3(256), 0, st, Qrev, (uint32_t)m, d_q, (uint32_t)m);
  KZGX_TRY_HIP(hipGetLastError());
  *nq_out = m;
  return KZGX_OK;
}

int prove_range_poly(Ctx* ctx, const uint32_t* d_P, size_t n, const uint32_t* d_x, size_t len, uint32_t* d_q,
                     size_t* nq, hipStream_t st) {
  return ctx->curve == KZGX_CURVE_BN254 ? prove_range_poly_impl<BN254Fr>(ctx, d_P, n, d_x, len, d_q, nq, st)
                                        : prove_range_poly_impl<BLS12381Fr>(ctx, d_P, n, d_x, len, d_q, nq, st);
}

}  // namespace kzgx

namespace kzgx {
// device bring-up (kzgx_setup.hpp): one launch loads this code object
__global__ void k_warm_poly() {}
int warm_poly(hipStream_t st) {
  hipLaunchKernelGGL(k_warm_poly, dim3(1), dim3(64), 0, st);
  KZGX_TRY_HIP(hipGetLastError());
  return KZGX_OK;
}
}  // namespace kzgx
