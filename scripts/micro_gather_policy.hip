// Load-policy sweep for the fixed-base table's gathers:
// does any load form gfx950 offers turn a random 64-B entry read into a
// 64-B DRAM request instead of a 128-B line fill?
//
// One kernel per policy, each gathering G random 64-B-aligned entries of a
// table far larger than the 256 MiB Infinity Cache, every entry read by one
// lane as four 16-B loads (exactly what fixed_accum.hpp's packed_fetch does):
//   default   : plain global_load_dwordx4 (the product's form)
//   nt_builtin: __builtin_nontemporal_load (the compiler's streaming form)
//   asm_<bits>: global_load_dwordx4 with the gfx950 cache-policy bits
//               sc0 / sc1 / nt in every combination
//   buffer    : raw buffer loads (aux 0; aux 2 = nt, aux 1 = sc0 on gfx950)
// Each launch prints its algorithmic bytes and time; rocprofv3 --pmc
// TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum gives
// the DRAM request sizes per dispatch (scripts/gpu.sh profbin / pmc steps).
// Loads only: no store touches the scalar cache.
//   hipcc -O3 --offload-arch=gfx950 -o scripts/micro_gather_policy scripts/micro_gather_policy.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                  \
  do {                                                            \
    hipError_t e = (x);                                           \
    if (e != hipSuccess) {                                        \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); \
      std::exit(1);                                               \
    }                                                             \
  } while (0)

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint64_t mix(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}

enum Policy { P_DEFAULT, P_NT_BUILTIN, P_SC0, P_SC1, P_NT, P_SC0_SC1, P_SC0_NT, P_SC1_NT, P_SC0_SC1_NT, P_BUF, P_BUF_SLC, P_BUF_GLC };

template <int P>
__device__ __forceinline__ v4u load16(const v4u* p, __amdgpu_buffer_rsrc_t rsrc, uint32_t off) {
  v4u v;
  if constexpr (P == P_DEFAULT) {
    v = *p;
  } else if constexpr (P == P_NT_BUILTIN) {
    v = __builtin_nontemporal_load(p);
  } else if constexpr (P == P_BUF) {
    v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, off, 0, 0);
  } else if constexpr (P == P_BUF_SLC) {
    v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, off, 0, 2);
  } else if constexpr (P == P_BUF_GLC) {
    v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, off, 0, 1);
  } else {
#define KZGX_GLD(BITS) asm volatile("global_load_dwordx4 %0, %1, off " BITS "\n s_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory")
    if constexpr (P == P_SC0) KZGX_GLD("sc0");
    if constexpr (P == P_SC1) KZGX_GLD("sc1");
    if constexpr (P == P_NT) KZGX_GLD("nt");
    if constexpr (P == P_SC0_SC1) KZGX_GLD("sc0 sc1");
    if constexpr (P == P_SC0_NT) KZGX_GLD("sc0 nt");
    if constexpr (P == P_SC1_NT) KZGX_GLD("sc1 nt");
    if constexpr (P == P_SC0_SC1_NT) KZGX_GLD("sc0 sc1 nt");
#undef KZGX_GLD
  }
  return v;
}

template <int P>
__global__ __launch_bounds__(256) void k_gather(const uint32_t* __restrict__ tab, uint64_t entries, uint64_t gathers,
                                                uint32_t* __restrict__ sink) {
  uint32_t o = 0;
  // buffer resource over the first 4 GiB window the buffer offsets can reach
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)tab, 0, 0xffffffff, 0x00020000);
  const uint64_t ent = P >= P_BUF ? (entries < (1ull << 26) ? entries : (1ull << 26)) : entries;
  for (uint64_t g = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; g < gathers;
       g += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t e = mix(g) % ent;
    const v4u* p = reinterpret_cast<const v4u*>(tab + e * 16);
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const v4u v = load16<P>(p + k, rsrc, (uint32_t)(e * 64 + 16 * k));
      o ^= v.x ^ v.y ^ v.z ^ v.w;
    }
  }
  if (o == 0x9e3779b9u) sink[threadIdx.x] = o;
}

template <int P>
static void run(const char* name, const uint32_t* tab, size_t bytes, uint64_t gathers, uint32_t* sink) {
  const dim3 grid(256 * 8 * 4), blk(256);
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  CHECK(hipEventRecord(a));
  hipLaunchKernelGGL(k_gather<P>, grid, blk, 0, 0, tab, (uint64_t)(bytes / 64), gathers, sink);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  const uint64_t ent = P >= P_BUF ? ((bytes / 64) < (1ull << 26) ? bytes / 64 : (1ull << 26)) : bytes / 64;
  std::printf("{\"policy\": \"%s\", \"gathers\": %llu, \"entries\": %llu, \"algorithmic_bytes\": %llu, "
              "\"time_ms\": %.3f, \"gather_GBps\": %.1f}\n",
              name, (unsigned long long)gathers, (unsigned long long)ent, (unsigned long long)(gathers * 64), ms,
              gathers * 64 / (ms * 1e6));
  std::fflush(stdout);
  CHECK(hipEventDestroy(a));
  CHECK(hipEventDestroy(b));
}

int main(int argc, char** argv) {
  const double table_gb = argc > 1 ? std::atof(argv[1]) : 16.0;
  const uint64_t gathers = argc > 2 ? std::strtoull(argv[2], nullptr, 10) : (32ull << 20);
  const size_t bytes = (size_t)(table_gb * 1e9) / 64 * 64;
  uint32_t *tab = nullptr, *sink = nullptr;
  CHECK(hipMalloc((void**)&tab, bytes));
  CHECK(hipMalloc((void**)&sink, 4096));
  CHECK(hipMemset(tab, 0x5a, bytes));
  CHECK(hipDeviceSynchronize());
  run<P_DEFAULT>("default", tab, bytes, gathers, sink);
  run<P_NT_BUILTIN>("nt_builtin", tab, bytes, gathers, sink);
  run<P_SC0>("asm_sc0", tab, bytes, gathers, sink);
  run<P_SC1>("asm_sc1", tab, bytes, gathers, sink);
  run<P_NT>("asm_nt", tab, bytes, gathers, sink);
  run<P_SC0_SC1>("asm_sc0_sc1", tab, bytes, gathers, sink);
  run<P_SC0_NT>("asm_sc0_nt", tab, bytes, gathers, sink);
  run<P_SC1_NT>("asm_sc1_nt", tab, bytes, gathers, sink);
  run<P_SC0_SC1_NT>("asm_sc0_sc1_nt", tab, bytes, gathers, sink);
  run<P_BUF>("buffer", tab, bytes, gathers, sink);
  run<P_BUF_SLC>("buffer_nt", tab, bytes, gathers, sink);
  run<P_BUF_GLC>("buffer_sc0", tab, bytes, gathers, sink);
  run<P_DEFAULT>("default_again", tab, bytes, gathers, sink);
  CHECK(hipFree(tab));
  CHECK(hipFree(sink));
  return 0;
}
