// Calibration of rocprofv3 FETCH_SIZE for the fixed-base table's access
// pattern (does the guide's x2 correction, stated for wide
// coalesced streaming reads, hold for random 80-B gathers?).
//
// Kernels, each launched alone on a table far larger than the 256 MiB
// Infinity Cache (so every gather misses on-die caches):
//   k_stream  : coalesced 16-B/lane streaming read of S bytes (the guide's
//               calibrated case: FETCH_SIZE should read S / 2)
//   k_gather<EW>: G random entries of EW words (EW = 20: the 80-B radix-2^29
//               layout, 16: the 64-B packed layout), each entry read as EW/4
//               dwordx4 loads by one lane, entries EW*4-byte aligned
// The program prints the algorithmic bytes of each launch; rocprofv3 --pmc
// FETCH_SIZE gives the counter per dispatch.  Build:
//   hipcc -O3 --offload-arch=gfx950 -o scripts/micro_gather scripts/micro_gather.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e = (x);                                                           \
    if (e != hipSuccess) {                                                        \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                 \
      std::exit(1);                                                               \
    }                                                                             \
  } while (0)

__global__ void k_stream(const uint4* __restrict__ p, size_t n16, uint32_t* __restrict__ sink) {
  uint32_t o = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
    const uint4 v = p[i];
    o ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (o == 0x9e3779b9u) sink[threadIdx.x] = o;
}

__device__ __forceinline__ uint64_t mix(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}

template <int EW>
__global__ void k_gather(const uint32_t* __restrict__ tab, uint64_t entries, uint64_t gathers,
                         uint32_t* __restrict__ sink) {
  uint32_t o = 0;
  for (uint64_t g = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; g < gathers; g += (uint64_t)gridDim.x * blockDim.x) {
    const uint4* e = reinterpret_cast<const uint4*>(tab + (mix(g) % entries) * EW);
#pragma unroll
    for (int k = 0; k < EW / 4; k++) {
      const uint4 v = e[k];
      o ^= v.x ^ v.y ^ v.z ^ v.w;
    }
  }
  if (o == 0x9e3779b9u) sink[threadIdx.x] = o;
}

int main(int argc, char** argv) {
  const double table_gb = argc > 1 ? std::atof(argv[1]) : 32.0;
  const uint64_t gathers = argc > 2 ? std::strtoull(argv[2], nullptr, 10) : (64ull << 20);
  const size_t bytes = (size_t)(table_gb * 1e9) / 80 * 80;
  uint32_t *tab = nullptr, *sink = nullptr;
  CHECK(hipMalloc((void**)&tab, bytes));
  CHECK(hipMalloc((void**)&sink, 4096));
  CHECK(hipMemset(tab, 0x5a, bytes));
  CHECK(hipDeviceSynchronize());
  const dim3 grid(256 * 8 * 4), blk(256);
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  float ms = 0;
  // 1. streaming read of the whole table
  CHECK(hipEventRecord(a));
  hipLaunchKernelGGL(k_stream, grid, blk, 0, 0, reinterpret_cast<const uint4*>(tab), bytes / 16, sink);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  CHECK(hipEventElapsedTime(&ms, a, b));
  std::printf("k_stream bytes %zu time_ms %.3f GBps %.1f\n", bytes, ms, bytes / (ms * 1e6));
  // 2. 80-B gathers (radix-2^29 table entries)
  CHECK(hipEventRecord(a));
  hipLaunchKernelGGL(k_gather<20>, grid, blk, 0, 0, tab, (uint64_t)(bytes / 80), gathers, sink);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  CHECK(hipEventElapsedTime(&ms, a, b));
  std::printf("k_gather<20> gathers %llu bytes %llu time_ms %.3f\n", (unsigned long long)gathers,
              (unsigned long long)(gathers * 80), ms);
  // 3. 64-B gathers (packed entries, 64-B aligned)
  CHECK(hipEventRecord(a));
  hipLaunchKernelGGL(k_gather<16>, grid, blk, 0, 0, tab, (uint64_t)(bytes / 64), gathers, sink);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  CHECK(hipEventElapsedTime(&ms, a, b));
  std::printf("k_gather<16> gathers %llu bytes %llu time_ms %.3f\n", (unsigned long long)gathers,
              (unsigned long long)(gathers * 64), ms);
  CHECK(hipFree(tab));
  CHECK(hipFree(sink));
  return 0;
}
