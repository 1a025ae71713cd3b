// Where the waves of one workgroup run, and what that costs a latency-bound
// chain: every wave of a block runs the same dependent 64-bit mad chain
// (ITERS steps) and records its SIMD (HW_ID bits 5:4), CU (11:8) and its
// elapsed core clocks.  Block sizes 64 / 128 / 256, grids of 1 and 48 blocks.
//
//   hipcc -O3 --offload-arch=gfx950 -o scripts/probe_simd scripts/probe_simd.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

__global__ void k_probe(uint32_t iters, uint64_t* out) {
  const uint32_t w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  uint64_t acc = threadIdx.x + 1;
  const uint64_t t0 = clock64();
  for (uint32_t i = 0; i < iters; i++) acc = acc * 0x9E3779B97F4A7C15ull + (acc >> 29);
  const uint64_t t1 = clock64();
  if ((threadIdx.x & 63) == 0) {
    out[3 * w] = __builtin_amdgcn_s_getreg((31 << 11) | 4);
    out[3 * w + 1] = t1 - t0;
    out[3 * w + 2] = acc;
  }
}

int main() {
  uint64_t* d = nullptr;
  if (hipMalloc(&d, 3 * 8 * 4096) != hipSuccess) return 1;
  const unsigned sizes[3] = {64, 128, 256};
  for (unsigned grid : {1u, 48u}) {
    for (unsigned bs : sizes) {
      hipLaunchKernelGGL(k_probe, dim3(grid), dim3(bs), 0, 0, 1000u, d);
      hipLaunchKernelGGL(k_probe, dim3(grid), dim3(bs), 0, 0, 200000u, d);
      uint64_t h[3 * 4096];
      const unsigned waves = grid * bs / 64;
      if (hipMemcpy(h, d, 3 * 8 * waves, hipMemcpyDeviceToHost) != hipSuccess) return 1;
      printf("{\"grid\": %u, \"block\": %u, \"waves\": [", grid, bs);
      for (unsigned i = 0; i < waves && i < 16; i++)
        printf("%s{\"simd\": %u, \"cu\": %u, \"se\": %u, \"clk\": %llu}", i ? ", " : "", (unsigned)((h[3 * i] >> 4) & 3),
               (unsigned)((h[3 * i] >> 8) & 15), (unsigned)((h[3 * i] >> 13) & 3), (unsigned long long)h[3 * i + 1]);
      printf("]}\n");
    }
  }
  return 0;
}
