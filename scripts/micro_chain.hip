// Dependent-chain cost of v_mad_u64_u32 on gfx950: how many independent
// mad chains a wave must keep in flight, at 1-4 waves per SIMD, before the
// SIMD issues mads at its ceiling.  Evidence for the paired-chain products of
// field29.hpp ("Where the issue slots go").
//   hipcc -O3 --offload-arch=gfx950 -o scripts/mb/micro_chain scripts/micro_chain.hip
//
// Every kernel issues REP mads per iteration per lane, in NCH dependent chains
// advanced round-robin inside one asm statement (so the order is exact):
//   NCH = 1: each mad reads the previous one's result; an `s_nop 0` follows
//            every mad, the pad the compiler's hazard recognizer puts between
//            two dependent 64-bit VALU results (hipcc -S of field29.hpp);
//   NCH = 2, 4: consecutive mads are independent, no pad.
#include <hip/hip_runtime.h>

#include <cstdio>

#define REP 64

template <int NCH>
__global__ void __launch_bounds__(256) k_chain(uint32_t* out, int iters) {
  uint64_t a0 = threadIdx.x, a1 = 1, a2 = 2, a3 = 3;
  const uint32_t x = threadIdx.x + 1, y = blockIdx.x + 3;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int r = 0; r < REP / 4; r++) {
      uint64_t sc;
      if constexpr (NCH == 1) {
        asm volatile(
            "v_mad_u64_u32 %0, %1, %2, %3, %0\n\ts_nop 0\n\t"
            "v_mad_u64_u32 %0, %1, %2, %3, %0\n\ts_nop 0\n\t"
            "v_mad_u64_u32 %0, %1, %2, %3, %0\n\ts_nop 0\n\t"
            "v_mad_u64_u32 %0, %1, %2, %3, %0\n\ts_nop 0"
            : "+v"(a0), "=s"(sc)
            : "v"(x), "v"(y));
      } else if constexpr (NCH == 2) {
        asm volatile(
            "v_mad_u64_u32 %0, %2, %3, %4, %0\n\t"
            "v_mad_u64_u32 %1, %2, %3, %4, %1\n\t"
            "v_mad_u64_u32 %0, %2, %3, %4, %0\n\t"
            "v_mad_u64_u32 %1, %2, %3, %4, %1"
            : "+v"(a0), "+v"(a1), "=s"(sc)
            : "v"(x), "v"(y));
      } else {
        asm volatile(
            "v_mad_u64_u32 %0, %4, %5, %6, %0\n\t"
            "v_mad_u64_u32 %1, %4, %5, %6, %1\n\t"
            "v_mad_u64_u32 %2, %4, %5, %6, %2\n\t"
            "v_mad_u64_u32 %3, %4, %5, %6, %3"
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "=s"(sc)
            : "v"(x), "v"(y));
      }
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(a0 + a1 + a2 + a3);
}

// the same single chain with the pad left to the mad's own latency (no
// s_nop: how much of the pad's cost is the pad itself)
__global__ void __launch_bounds__(256) k_chain1_nopad(uint32_t* out, int iters) {
  uint64_t a0 = threadIdx.x;
  const uint32_t x = threadIdx.x + 1, y = blockIdx.x + 3;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int r = 0; r < REP / 4; r++) {
      uint64_t sc;
      asm volatile(
          "v_mad_u64_u32 %0, %1, %2, %3, %0\n\t"
          "v_mad_u64_u32 %0, %1, %2, %3, %0\n\t"
          "v_mad_u64_u32 %0, %1, %2, %3, %0\n\t"
          "v_mad_u64_u32 %0, %1, %2, %3, %0"
          : "+v"(a0), "=s"(sc)
          : "v"(x), "v"(y));
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)a0;
}

template <class K>
static void run(const char* name, K kern, int waves_per_simd, uint32_t* d) {
  const int cus = 256, iters = 4096;
  // 256-thread blocks = 4 wavefronts = one per SIMD of a CU
  dim3 grid(cus * waves_per_simd), block(256);
  hipLaunchKernelGGL(kern, grid, block, 0, 0, d, 16);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(kern, grid, block, 0, 0, d, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  double ops = (double)grid.x * 256 * iters * REP;
  printf("%-22s waves/SIMD %d  %8.3f ms  %.3e mad lane-ops/s\n", name, waves_per_simd, ms, ops / (ms * 1e-3));
}

int main() {
  uint32_t* d;
  hipMalloc(&d, 256 * 8 * 256 * sizeof(uint32_t));
  for (int w = 1; w <= 4; w++) {
    run("1 chain + s_nop", k_chain<1>, w, d);
    run("1 chain, no pad", k_chain1_nopad, w, d);
    run("2 chains", k_chain<2>, w, d);
    run("4 chains", k_chain<4>, w, d);
  }
  hipFree(d);
  return 0;
}
