// Mixed-addition throughput microbenchmark for gfx950 (the accumulation loop
// of k_fixed_accum without the table stream): each variant of the XYZZ mixed
// addition runs ITERS dependent additions per thread over 64 L1-resident
// affine points, whole GPU, at the accumulation kernel's occupancy.  Every
// variant's final accumulators are reduced and compared with variant 0
// (same formulas, so the same field values).  Also: the dependent-issue
// latency of v_mad_u64_u32 chains.
//
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -o scripts/micro_madd scripts/micro_madd.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#pragma clang diagnostic ignored "-Wunused-result"
#pragma clang diagnostic ignored "-Wunused-value"

#include "../kzg-commitments_amd/csrc/curve.hpp"
#include "../kzg-commitments_amd/csrc/fixed_accum.hpp"

using namespace kzgx;

#ifndef WAVES_BN
#define WAVES_BN 3
#endif
#ifndef WAVES_BLS
#define WAVES_BLS 2
#endif

template <class C>
constexpr int waves_of() {
  return C::Fp29::L <= 9 ? WAVES_BN : WAVES_BLS;
}

// pts[i] = (i + 1) G, radix-2^29 Montgomery affine, thread per point
template <class C>
__global__ void k_points(uint32_t* pts) {
  using F = typename C::Fp29;
  const int i = threadIdx.x;
  Affine<C> g;
  g.x = f29_const<F>(C::GX29);
  g.y = f29_const<F>(C::GY29);
  Xyzz<C> acc = xyzz_from_affine<C>(g);
  for (int k = 0; k < i; k++) acc = xyzz_add_affine<C>(acc, g);
  Affine<C> a;
  xyzz_to_affine<C>(acc, a);
  affine_store<C>(pts + i * affine_words<C>(), a);
}

template <class C, int V>
__global__ __launch_bounds__(64, waves_of<C>()) void k_madd(const uint32_t* __restrict__ pts, uint32_t iters,
                                                           uint32_t* __restrict__ out) {
  using F = typename C::Fp29;
  constexpr int PW = affine_words<C>();
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  Xyzz<C> acc = xyzz_from_affine<C>(affine_load<C>(pts + (size_t)(t & 63) * PW));
#pragma unroll 1
  for (uint32_t k = 0; k < iters; k++) {
    Affine<C> a = affine_load<C>(pts + (size_t)((t + 1 + k) & 63) * PW);
    if (k & 1) a.y = f29_neg_lazy<F>(a.y);
    acc = xyzz_add_affine_v<C, V>(acc, a);
  }
  if (out) {
    constexpr int L = F::L;
    const F29<F> v[4] = {f29_reduce<F>(acc.X), f29_reduce<F>(acc.Y), f29_reduce<F>(acc.ZZ), f29_reduce<F>(acc.ZZZ)};
    for (int c = 0; c < 4; c++)
      for (int i = 0; i < L; i++) out[((size_t)t * 4 + c) * L + i] = v[c].v[i];
  }
}

// table of W x n x H packed entries, every one a copy of one of the 64
// points (any curve points do: both variants sum the same entries)
template <class C>
__global__ void k_fill(uint32_t* __restrict__ tab, size_t entries, const uint32_t* __restrict__ pts) {
  for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < entries; e += (size_t)gridDim.x * blockDim.x)
    packed_store<C>(tab + e * packed_words<C>(), affine_load<C>(pts + (e & 63) * affine_words<C>()));
}

// k_fixed_accum itself (the bench's kernel, fixed_accum.hpp) at the bench's
// batch and points per thread, window CB (a table that fits the micro),
// classic vs nway mixed addition; partial sums compared word for word
template <class C, int CB, int PF>
static int run_accum(const char* name, uint32_t B, uint32_t ppt) {
  constexpr int W = FixedWin<C, CB>::W;
  constexpr size_t H = FixedWin<C, CB>::H;
  constexpr int PW = packed_words<C>();
  const uint32_t n = 4097;
  const uint32_t T = 64 * ((n + 64 * ppt - 1) / (64 * ppt));
  const size_t entries = (size_t)W * n * H;
  uint32_t *d_pts, *d_tab, *d_sc, *d_p0, *d_p1;
  uint8_t* d_inf;
  hipMalloc(&d_pts, 64 * affine_words<C>() * 4);
  hipLaunchKernelGGL(k_points<C>, dim3(1), dim3(64), 0, 0, d_pts);
  // MICRO_CONTIG=1: the table as one physically contiguous allocation (fewer,
  // larger page-table fragments: the TLB-reach probe)
  if (getenv("MICRO_CONTIG")) {
    if (hipExtMallocWithFlags((void**)&d_tab, entries * PW * 4, hipDeviceMallocContiguous) != hipSuccess) {
      printf("{\"contiguous_alloc\": \"failed\", \"bytes\": %zu}\n", entries * PW * 4);
      return 2;
    }
  } else if (hipMalloc(&d_tab, entries * PW * 4) != hipSuccess) {
    return 2;
  }
  hipLaunchKernelGGL(k_fill<C>, dim3(65536), dim3(256), 0, 0, d_tab, entries, d_pts);
  std::vector<uint32_t> sc((size_t)B * n * 8);
  uint64_t x = 0x9E3779B97F4A7C15ull;
  for (size_t i = 0; i < sc.size(); i++) {
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    sc[i] = (uint32_t)x;
    if (i % 8 == 7) sc[i] &= 0x0fffffffu;  // < 2^252 < r
  }
  hipMalloc(&d_sc, sc.size() * 4);
  hipMemcpy(d_sc, sc.data(), sc.size() * 4, hipMemcpyHostToDevice);
  hipMalloc(&d_inf, n);
  hipMemset(d_inf, 0, n);
  const size_t pw = (size_t)B * T * xyzz_words<C>();
  hipMalloc(&d_p0, pw * 4);
  hipMalloc(&d_p1, pw * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  // window-major layout (msm_fixed.hip, TabStrides)
  const TabStrides ts{(size_t)FixedWin<C, CB>::H * PW, (size_t)n * FixedWin<C, CB>::H * PW};
  double ms[3];
  for (int v = 0; v < 3; v++) {
    for (int rep = 0; rep < 3; rep++) {
      hipEventRecord(e0, 0);
      if (v == 0)
        hipLaunchKernelGGL((k_fixed_accum<C, CB, 0>), dim3(T / 64, B), dim3(64), 0, 0, d_sc, n, (size_t)n * 8, d_tab,
                           ts, nullptr, 0u, T, d_p0);
      else if (v == 1)
        hipLaunchKernelGGL((k_fixed_accum<C, CB, 1>), dim3(T / 64, B), dim3(64), 0, 0, d_sc, n, (size_t)n * 8, d_tab,
                           ts, nullptr, 0u, T, d_p1);
      else  // loads and digit recoding only: the memory path's own rate
        hipLaunchKernelGGL((k_fixed_accum<C, CB, 2>), dim3(T / 64, B), dim3(64), 0, 0, d_sc, n, (size_t)n * 8, d_tab,
                           ts, nullptr, 0u, T, d_p0 + 0 * pw);
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      float m = 0;
      hipEventElapsedTime(&m, e0, e1);
      ms[v] = m;
    }
  }
  // rerun classic into d_p0 (the probe overwrote it)
  hipLaunchKernelGGL((k_fixed_accum<C, CB, 0>), dim3(T / 64, B), dim3(64), 0, 0, d_sc, n, (size_t)n * 8, d_tab, ts,
                     d_inf, 0u, T, d_p0);
  std::vector<uint32_t> h0(pw), h1(pw);
  hipMemcpy(h0.data(), d_p0, pw * 4, hipMemcpyDeviceToHost);
  hipMemcpy(h1.data(), d_p1, pw * 4, hipMemcpyDeviceToHost);
  const bool same = memcmp(h0.data(), h1.data(), pw * 4) == 0;
  const double madds = (double)B * n * W;
  printf("{\"kernel\": \"k_fixed_accum<%s,%d,PF=%d>\", \"waves\": %d, \"batch\": %u, \"ppt\": %u, \"ms\": {\"classic\": %.3f, "
         "\"nway\": %.3f}, \"madd_per_s\": {\"classic\": %.4e, \"nway\": %.4e}, \"nway_over_classic\": %.4f, "
         "\"same_partials\": %s, \"loads_only_terms_per_s\": %.4e}\n",
         name, CB, PF, fixed_accum_waves<C>(), B, ppt, ms[0], ms[1], madds / (ms[0] * 1e-3), madds / (ms[1] * 1e-3), ms[0] / ms[1],
         same ? "true" : "false", madds / (ms[2] * 1e-3));
  hipFree(d_pts); hipFree(d_tab); hipFree(d_sc); hipFree(d_inf); hipFree(d_p0); hipFree(d_p1);
  return same ? 0 : 1;
}

// NCH independent dependent chains of v_mad_u64_u32 per lane
template <int NCH>
__global__ __launch_bounds__(64) void k_chain(uint32_t* out, int iters) {
  uint64_t acc[NCH];
  uint32_t a = threadIdx.x + 1, b = blockIdx.x + 3;
  for (int k = 0; k < NCH; k++) acc[k] = k;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int r = 0; r < 64 / NCH; r++) {
#pragma unroll
      for (int k = 0; k < NCH; k++) {
        uint64_t sc;
        asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc[k]), "=s"(sc) : "v"(a), "v"(b));
      }
    }
  }
  uint64_t s = 0;
  for (int k = 0; k < NCH; k++) s += acc[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s;
}

template <class C>
static int run_curve(const char* name) {
  using F = typename C::Fp29;
  constexpr int L = F::L;
  uint32_t* d_pts;
  hipMalloc(&d_pts, 64 * affine_words<C>() * 4);
  hipLaunchKernelGGL(k_points<C>, dim3(1), dim3(64), 0, 0, d_pts);
  const uint32_t waves = 256 * 4 * waves_of<C>() * 4;
  const uint32_t iters = 192;
  const size_t nthr = (size_t)waves * 64;
  uint32_t *d_o0, *d_o1;
  hipMalloc(&d_o0, nthr * 4 * L * 4);
  hipMalloc(&d_o1, nthr * 4 * L * 4);
  hipLaunchKernelGGL((k_madd<C, 0>), dim3(waves), dim3(64), 0, 0, d_pts, 64u, d_o0);
  hipLaunchKernelGGL((k_madd<C, 1>), dim3(waves), dim3(64), 0, 0, d_pts, 64u, d_o1);
  std::vector<uint32_t> h0(nthr * 4 * L), h1(nthr * 4 * L);
  hipMemcpy(h0.data(), d_o0, h0.size() * 4, hipMemcpyDeviceToHost);
  hipMemcpy(h1.data(), d_o1, h1.size() * 4, hipMemcpyDeviceToHost);
  const bool same = memcmp(h0.data(), h1.data(), h0.size() * 4) == 0;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  double rate[2];
  for (int v = 0; v < 2; v++) {
    for (int rep = 0; rep < 2; rep++) {
      hipEventRecord(e0, 0);
      if (v == 0) hipLaunchKernelGGL((k_madd<C, 0>), dim3(waves), dim3(64), 0, 0, d_pts, iters, nullptr);
      else hipLaunchKernelGGL((k_madd<C, 1>), dim3(waves), dim3(64), 0, 0, d_pts, iters, nullptr);
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      rate[v] = (double)nthr * iters / (ms * 1e-3);
    }
  }
  printf("{\"curve\": \"%s\", \"waves_per_simd\": %d, \"madd_per_s\": {\"impl\": %.4e, \"nway\": %.4e}, "
         "\"nway_over_impl\": %.4f, \"same_values\": %s}\n",
         name, waves_of<C>(), rate[0], rate[1], rate[1] / rate[0], same ? "true" : "false");
  hipFree(d_pts);
  hipFree(d_o0);
  hipFree(d_o1);
  return same ? 0 : 1;
}

template <int NCH>
static void run_chain(int waves_per_simd) {
  uint32_t* d;
  const int blocks = 256 * 4 * waves_per_simd;
  hipMalloc(&d, blocks * 64 * 4);
  const int iters = 256;
  hipLaunchKernelGGL(k_chain<NCH>, dim3(blocks), dim3(64), 0, 0, d, 1);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0, 0);
  hipLaunchKernelGGL(k_chain<NCH>, dim3(blocks), dim3(64), 0, 0, d, iters);
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  const double wave_ops = (double)blocks * iters * 64;  // per wave: iters x 64 mads
  const double simd_cyc = 256.0 * 4 * 2.4e9 * (ms * 1e-3);
  printf("{\"mad_chain\": %d, \"waves_per_simd\": %d, \"simd_cycles_per_mad\": %.2f}\n", NCH, waves_per_simd,
         simd_cyc / wave_ops);
  hipFree(d);
}

int main() {
  int bad = 0;
  bad |= run_curve<BN254G1>("BN254");
  bad |= run_curve<BLS12381G1>("BLS12381");
  bad |= run_accum<BN254G1, 12, 1>("BN254", 2048, 22);
  bad |= run_accum<BN254G1, 12, 0>("BN254", 2048, 22);
  bad |= run_accum<BLS12381G1, 12, 1>("BLS12381", 2048, 65);
  bad |= run_accum<BLS12381G1, 12, 0>("BLS12381", 2048, 65);
  if (getenv("MICRO_C14")) bad |= run_accum<BN254G1, 14, 1>("BN254", 2048, 22);
  if (getenv("MICRO_CSWEEP")) {  // table window sweep: HBM gather (c = 8, 12) vs a cache-resident table (c = 2, 4)
    bad |= run_accum<BN254G1, 2, 1>("BN254", 2048, 22);
    bad |= run_accum<BN254G1, 4, 1>("BN254", 2048, 22);
    bad |= run_accum<BN254G1, 8, 1>("BN254", 2048, 22);
  }
  if (getenv("MICRO_CHAINS")) {
    for (int w : {1, 2, 3, 4}) {
      run_chain<1>(w);
      run_chain<2>(w);
      run_chain<4>(w);
    }
  }
  return bad;
}
