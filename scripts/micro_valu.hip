// VALU microbenchmark for gfx950: issue cost of the integer instructions the
// field arithmetic is built from, and throughput of candidate Montgomery
// multipliers.  Evidence for DESIGN.md section "field arithmetic".
//   hipcc -O3 --offload-arch=gfx950 -o micro_valu scripts/micro_valu.hip
#include <hip/hip_runtime.h>

#include <cstdio>

#include "../kzg-commitments_amd/csrc/field.hpp"

using namespace kzgx;

#define REP 256

// 8 independent chains per lane, REP iterations each, inline asm so the
// instruction mix is exact
__global__ void k_mad64(uint32_t* out, int iters) {
  uint64_t acc[8];
  uint32_t a = threadIdx.x + 1, b = blockIdx.x + 3;
  for (int k = 0; k < 8; k++) acc[k] = k;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int r = 0; r < REP / 8; r++) {
#pragma unroll
      for (int k = 0; k < 8; k++) {
        uint64_t sc;
        asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc[k]), "=s"(sc) : "v"(a), "v"(b));
      }
    }
  }
  uint64_t s = 0;
  for (int k = 0; k < 8; k++) s += acc[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s;
}

__global__ void k_mullo(uint32_t* out, int iters) {
  uint32_t acc[8];
  uint32_t a = threadIdx.x + 1;
  for (int k = 0; k < 8; k++) acc[k] = k + 7;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int r = 0; r < REP / 8; r++) {
#pragma unroll
      for (int k = 0; k < 8; k++) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(acc[k]) : "v"(a));
    }
  }
  uint32_t s = 0;
  for (int k = 0; k < 8; k++) s += acc[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_mulhi(uint32_t* out, int iters) {
  uint32_t acc[8];
  uint32_t a = threadIdx.x + 1;
  for (int k = 0; k < 8; k++) acc[k] = k + 7;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int r = 0; r < REP / 8; r++) {
#pragma unroll
      for (int k = 0; k < 8; k++) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(acc[k]) : "v"(a));
    }
  }
  uint32_t s = 0;
  for (int k = 0; k < 8; k++) s += acc[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_addco(uint32_t* out, int iters) {
  uint32_t acc[8];
  uint32_t a = threadIdx.x + 1;
  for (int k = 0; k < 8; k++) acc[k] = k + 7;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int r = 0; r < REP / 8; r++) {
#pragma unroll
      for (int k = 0; k < 8; k++) {
        uint64_t sc;
        asm volatile("v_add_co_u32 %0, %1, %0, %2" : "+v"(acc[k]), "=s"(sc) : "v"(a));
      }
    }
  }
  uint32_t s = 0;
  for (int k = 0; k < 8; k++) s += acc[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_lshladd(uint32_t* out, int iters) {
  uint64_t acc[8];
  uint64_t a = threadIdx.x + 1;
  for (int k = 0; k < 8; k++) acc[k] = k + 7;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int r = 0; r < REP / 8; r++) {
#pragma unroll
      for (int k = 0; k < 8; k++) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(acc[k]) : "v"(a));
    }
  }
  uint64_t s = 0;
  for (int k = 0; k < 8; k++) s += acc[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s;
}

__global__ void k_mov(uint32_t* out, int iters) {
  uint32_t acc[8];
  for (int k = 0; k < 8; k++) acc[k] = k + threadIdx.x;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int r = 0; r < REP / 8; r++) {
#pragma unroll
      for (int k = 0; k < 8; k++) asm volatile("v_mov_b32 %0, %1" : "=v"(acc[k]) : "v"(acc[(k + 1) & 7]));
    }
  }
  uint32_t s = 0;
  for (int k = 0; k < 8; k++) s += acc[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}


// generic 32-bit binary op, 8 independent chains: "OP acc, acc, a"
#define K_BIN32(NAME, ASM)                                                              \
  __global__ void NAME(uint32_t* out, int iters) {                                      \
    uint32_t acc[8];                                                                    \
    uint32_t a = threadIdx.x + 1;                                                       \
    for (int k = 0; k < 8; k++) acc[k] = k + 7;                                         \
    for (int it = 0; it < iters; it++) {                                                \
      _Pragma("unroll") for (int r = 0; r < REP / 8; r++) {                             \
        _Pragma("unroll") for (int k = 0; k < 8; k++) asm volatile(ASM : "+v"(acc[k]) : "v"(a)); \
      }                                                                                 \
    }                                                                                   \
    uint32_t s = 0;                                                                     \
    for (int k = 0; k < 8; k++) s += acc[k];                                            \
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;                                     \
  }
K_BIN32(k_add32, "v_add_u32 %0, %0, %1")
K_BIN32(k_sub32, "v_sub_u32 %0, %0, %1")
K_BIN32(k_and32, "v_and_b32 %0, %0, %1")
K_BIN32(k_ashr32, "v_ashrrev_i32 %0, %1, %0")
K_BIN32(k_align32, "v_alignbit_b32 %0, %0, %1, 11")
K_BIN32(k_add3, "v_add3_u32 %0, %0, %1, %0")
K_BIN32(k_mul24, "v_mul_u32_u24 %0, %0, %1")
K_BIN32(k_mad24, "v_mad_u32_u24 %0, %0, %1, %0")

__global__ void k_lshr64(uint32_t* out, int iters) {
  uint64_t acc[8];
  for (int k = 0; k < 8; k++) acc[k] = k + 7 + threadIdx.x;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int r = 0; r < REP / 8; r++) {
#pragma unroll
      for (int k = 0; k < 8; k++) asm volatile("v_lshrrev_b64 %0, 1, %0" : "+v"(acc[k]));
    }
  }
  uint64_t s = 0;
  for (int k = 0; k < 8; k++) s += acc[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s;
}

__global__ void k_mov64(uint32_t* out, int iters) {
  uint64_t acc[8];
  for (int k = 0; k < 8; k++) acc[k] = k + threadIdx.x;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int r = 0; r < REP / 8; r++) {
#pragma unroll
      for (int k = 0; k < 8; k++) asm volatile("v_mov_b64 %0, %1" : "=v"(acc[k]) : "v"(acc[(k + 1) & 7]));
    }
  }
  uint64_t s = 0;
  for (int k = 0; k < 8; k++) s += acc[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s;
}

// REP field multiplications per iteration, 4 independent chains per lane
template <class FP>
__global__ void k_fe_mul(uint32_t* out, int iters) {
  Fe<FP> a[4], b;
  for (int i = 0; i < FP::N; i++) b.v[i] = (threadIdx.x * 2654435761u + i * 40503u) & 0x0fffffffu;
  for (int k = 0; k < 4; k++)
    for (int i = 0; i < FP::N; i++) a[k].v[i] = (threadIdx.x * 7u + i * 13u + k) & 0x0fffffffu;
  for (int it = 0; it < iters; it++) {
    for (int r = 0; r < REP / 4; r++) {
#pragma unroll
      for (int k = 0; k < 4; k++) a[k] = fe_mul<FP>(a[k], b);
    }
  }
  uint32_t s = 0;
  for (int k = 0; k < 4; k++)
    for (int i = 0; i < FP::N; i++) s ^= a[k].v[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// candidate: radix-2^29 limbs, product scanning (FIPS), 64-bit column accumulator;
// every partial product is one v_mad_u64_u32, no carry chains; output < 2p
template <int L>
struct R29 {
  uint32_t v[L];
};
__device__ __constant__ uint32_t P29_BN[9];
template <int L, uint32_t INV29>
__device__ __forceinline__ R29<L> mul29(const R29<L>& a, const R29<L>& b, const uint32_t (&p)[L]) {
  constexpr uint32_t M = (1u << 29) - 1;
  uint32_t m[L];
  R29<L> t;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 2 * L - 1; k++) {
#pragma unroll
    for (int i = 0; i < L; i++) {
      const int j = k - i;
      if (j >= 0 && j < L) acc += (uint64_t)a.v[i] * b.v[j];
    }
#pragma unroll
    for (int i = 0; i < L; i++) {
      const int j = k - i;
      if (i < k && j >= 1 && j < L) acc += (uint64_t)m[i] * p[j];
    }
    if (k < L) {
      m[k] = ((uint32_t)acc * INV29) & M;
      acc += (uint64_t)m[k] * p[0];
    } else {
      t.v[k - L] = (uint32_t)acc & M;
    }
    acc >>= 29;
  }
  t.v[L - 1] = (uint32_t)acc;
  return t;
}

__global__ void k_mul29(uint32_t* out, int iters) {
  constexpr uint32_t p[9] = {0x00000013u, 0x18000000u, 0x000004e9u, 0x02000000u, 0x00008612u, 0x06c00000u, 0x0006e8d1u, 0x10480000u, 0x00252364u};  // BN254 p, radix 2^29
  R29<9> a[4], b;
  for (int i = 0; i < 9; i++) b.v[i] = (threadIdx.x * 2654435761u + i * 40503u) & 0x0fffffffu;
  for (int k = 0; k < 4; k++)
    for (int i = 0; i < 9; i++) a[k].v[i] = (threadIdx.x * 7u + i * 13u + k) & 0x0fffffffu;
  for (int it = 0; it < iters; it++) {
    for (int r = 0; r < REP / 4; r++) {
#pragma unroll
      for (int k = 0; k < 4; k++) a[k] = mul29<9, 0x179435e5u>(a[k], b, p);
    }
  }
  uint32_t s = 0;
  for (int k = 0; k < 4; k++)
    for (int i = 0; i < 9; i++) s ^= a[k].v[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <class K>
static double run(K kern, const char* name, double ops_per_thread_iter, int iters, int blocks, int threads,
                  uint32_t* d_out) {
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, d_out, 1);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, d_out, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  double lane_ops = ops_per_thread_iter * iters * (double)blocks * threads;
  double per_s = lane_ops / (ms * 1e-3);
  // wave-instructions per SIMD-cycle at 2.4 GHz: 256 CUs x 4 SIMD
  double simd_cyc = 256.0 * 4 * 2.4e9 * (ms * 1e-3);
  double cyc_per_wave_op = simd_cyc / (lane_ops / 64.0);
  printf("%-16s %9.3f ms  %10.3e lane-ops/s  %6.2f SIMD-cycles per wave-op\n", name, ms, per_s, cyc_per_wave_op);
  return per_s;
}

int main() {
  uint32_t* d_out;
  const int blocks = 256 * 8, threads = 256;
  hipMalloc(&d_out, blocks * threads * 4);
  run(k_mad64, "v_mad_u64_u32", REP, 64, blocks, threads, d_out);
  run(k_mullo, "v_mul_lo_u32", REP, 64, blocks, threads, d_out);
  run(k_mulhi, "v_mul_hi_u32", REP, 64, blocks, threads, d_out);
  run(k_addco, "v_add_co_u32", REP, 256, blocks, threads, d_out);
  run(k_lshladd, "v_lshl_add_u64", REP, 256, blocks, threads, d_out);
  run(k_mov, "v_mov_b32", REP, 256, blocks, threads, d_out);
  run(k_add32, "v_add_u32", REP, 256, blocks, threads, d_out);
  run(k_sub32, "v_sub_u32", REP, 256, blocks, threads, d_out);
  run(k_and32, "v_and_b32", REP, 256, blocks, threads, d_out);
  run(k_ashr32, "v_ashrrev_i32", REP, 256, blocks, threads, d_out);
  run(k_align32, "v_alignbit_b32", REP, 256, blocks, threads, d_out);
  run(k_add3, "v_add3_u32", REP, 256, blocks, threads, d_out);
  run(k_mul24, "v_mul_u32_u24", REP, 256, blocks, threads, d_out);
  run(k_mad24, "v_mad_u32_u24", REP, 256, blocks, threads, d_out);
  run(k_lshr64, "v_lshrrev_b64", REP, 256, blocks, threads, d_out);
  run(k_mov64, "v_mov_b64", REP, 256, blocks, threads, d_out);
  run(k_fe_mul<BN254Fp>, "fe_mul BN254", REP, 4, blocks, threads, d_out);
  run(k_fe_mul<BLS12381Fp>, "fe_mul BLS12381", REP, 2, blocks, threads, d_out);
  run(k_mul29, "mul29 (9 limbs)", REP, 4, blocks, threads, d_out);
  return 0;
}
