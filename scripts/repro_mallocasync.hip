// The ordering rules around stream-ordered allocations (hipMallocAsync) on a
// non-blocking stream, the setting of the round-1 "product-tree levels read
// back as zeros" observation.  Each case writes a
// buffer with a slow kernel on the non-blocking stream and reads it back:
//   ordered   - hipMemcpyAsync on the same stream + hipStreamSynchronize
//   nullcopy  - hipMemcpy (legacy null stream), no sync: a non-blocking stream
//               is not ordered against the null stream
//   plainmalloc - the nullcopy pattern on a hipMalloc buffer allocated after
//               the kernel launch (hipMalloc may synchronise the device)
//   reuse     - free a small async allocation, allocate a larger one on the
//               same stream, write it on a second stream without an event
// A case that reads stale data prints stale > 0.
//
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -o scripts/mb/repro_mallocasync scripts/repro_mallocasync.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#pragma clang diagnostic ignored "-Wunused-result"
#pragma clang diagnostic ignored "-Wunused-value"

__global__ void k_slow_fill(uint32_t* p, size_t n, uint32_t v, int spin) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  uint32_t x = v;
  for (int k = 0; k < spin; k++) x = x * 1664525u + 1013904223u;  // delay
  if (i < n) p[i] = v + ((x == 0x12345678u && spin < 0) ? 1u : 0u);  // keeps the delay loop
}

static size_t stale(const std::vector<uint32_t>& h, uint32_t v) {
  size_t s = 0;
  for (uint32_t x : h) s += x != v;
  return s;
}

int main() {
  const size_t n = 1 << 24;
  const int spin = 200000;
  hipStream_t s, s2;
  hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
  std::vector<uint32_t> h(n);
  const dim3 g((n + 255) / 256), b(256);

  {  // ordered
    uint32_t* d;
    hipMallocAsync((void**)&d, n * 4, s);
    hipLaunchKernelGGL(k_slow_fill, g, b, 0, s, d, n, 7u, spin);
    hipMemcpyAsync(h.data(), d, n * 4, hipMemcpyDeviceToHost, s);
    hipStreamSynchronize(s);
    printf("{\"case\": \"ordered\", \"stale\": %zu}\n", stale(h, 7u));
    hipFreeAsync(d, s);
    hipStreamSynchronize(s);
  }
  {  // nullcopy
    uint32_t* d;
    hipMallocAsync((void**)&d, n * 4, s);
    hipMemsetAsync(d, 0, n * 4, s);
    hipStreamSynchronize(s);
    hipLaunchKernelGGL(k_slow_fill, g, b, 0, s, d, n, 9u, spin);
    hipMemcpy(h.data(), d, n * 4, hipMemcpyDeviceToHost);
    printf("{\"case\": \"nullcopy\", \"stale\": %zu}\n", stale(h, 9u));
    hipStreamSynchronize(s);
    hipFreeAsync(d, s);
    hipStreamSynchronize(s);
  }
  {  // plainmalloc: same as nullcopy, with a hipMalloc between launch and copy
    uint32_t* d;
    hipMallocAsync((void**)&d, n * 4, s);
    hipMemsetAsync(d, 0, n * 4, s);
    hipStreamSynchronize(s);
    hipLaunchKernelGGL(k_slow_fill, g, b, 0, s, d, n, 11u, spin);
    uint32_t* e;
    hipMalloc((void**)&e, 1 << 20);
    hipMemcpy(h.data(), d, n * 4, hipMemcpyDeviceToHost);
    printf("{\"case\": \"plainmalloc\", \"stale\": %zu}\n", stale(h, 11u));
    hipStreamSynchronize(s);
    hipFree(e);
    hipFreeAsync(d, s);
    hipStreamSynchronize(s);
  }
  {  // reuse across streams without an event
    uint32_t *a, *c;
    hipMallocAsync((void**)&a, n * 2, s);
    hipLaunchKernelGGL(k_slow_fill, dim3((n / 2 + 255) / 256), b, 0, s, a, n / 2, 3u, spin);
    hipFreeAsync(a, s);
    hipMallocAsync((void**)&c, n * 4, s);
    hipLaunchKernelGGL(k_slow_fill, g, b, 0, s2, c, n, 5u, 0);  // s2 is not ordered after s
    hipStreamSynchronize(s2);
    hipStreamSynchronize(s);
    hipMemcpy(h.data(), c, n * 4, hipMemcpyDeviceToHost);
    printf("{\"case\": \"reuse\", \"stale\": %zu, \"same_address\": %d}\n", stale(h, 5u), (int)(a == c));
    hipFreeAsync(c, s);
    hipStreamSynchronize(s);
  }
  printf("{\"hip\": \"%s\"}\n", hipGetErrorString(hipDeviceSynchronize()));
  return 0;
}
