// Allocation-stall probe.  Times hipMalloc / hipFree of
// multi-GB blocks in the sequences the library's setup paths issue:
//   fresh      : the first N-GB hipMalloc of the process
//   after_free : the same hipMalloc right after hipFree of an M-GB block that
//                a kernel has written (a table that was built and dropped)
//   after_wait : the same, with a pause between the free and the malloc
//   reuse      : what the library does instead (keep the block, no free)
// Every hipMalloc is followed by a memset of the whole block (the table build
// writes all of it) so the pages are really backed; the memset is timed too.
// One JSON line per measurement on stdout.
//
//   hipcc -O2 --offload-arch=gfx950 scripts/probe_alloc.hip -o scripts/probe_alloc
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      std::printf("{\"error\": \"%s\", \"line\": %d}\n", hipGetErrorString(e_), __LINE__); \
      std::exit(1);                                                                   \
    }                                                                                 \
  } while (0)

static size_t free_gb() {
  size_t f = 0, t = 0;
  (void)hipMemGetInfo(&f, &t);
  return f >> 30;
}

// hipMalloc + memset of `gb` GB; returns the pointer, prints the timings
static void* alloc_touch(const char* tag, size_t gb) {
  void* p = nullptr;
  const size_t fg = free_gb();
  double t0 = now_ms();
  CK(hipMalloc(&p, gb << 30));
  double t1 = now_ms();
  CK(hipMemsetD32((hipDeviceptr_t)p, 0x5a5a5a5a, (gb << 30) / 4));
  CK(hipDeviceSynchronize());
  double t2 = now_ms();
  std::printf("{\"case\": \"%s\", \"gb\": %zu, \"free_gb_before\": %zu, \"malloc_ms\": %.3f, \"memset_ms\": %.3f}\n", tag,
              gb, fg, t1 - t0, t2 - t1);
  std::fflush(stdout);
  return p;
}

static void free_timed(const char* tag, void* p, size_t gb) {
  double t0 = now_ms();
  CK(hipFree(p));
  double t1 = now_ms();
  std::printf("{\"case\": \"%s\", \"gb\": %zu, \"free_ms\": %.3f}\n", tag, gb, t1 - t0);
  std::fflush(stdout);
}

int main(int argc, char** argv) {
  CK(hipSetDevice(0));
  CK(hipFree(nullptr));
  // 1. the default-table size (BN254 c = 12: 11.8 GB): fresh, then right
  //    after freeing the same size, three times, then after a 2 s pause
  void* a = alloc_touch("fresh_12", 12);
  for (int i = 0; i < 3; i++) {
    free_timed("free_12", a, 12);
    a = alloc_touch("after_free_12", 12);
  }
  free_timed("free_12", a, 12);
  std::this_thread::sleep_for(std::chrono::seconds(2));
  a = alloc_touch("after_wait2s_12", 12);
  free_timed("free_12", a, 12);
  // 2. a small block right after a large free (does the stall scale with the
  //    freed bytes or the requested ones?)
  void* b = alloc_touch("fresh_137", 137);
  free_timed("free_137", b, 137);
  a = alloc_touch("after_free137_12", 12);
  free_timed("free_12", a, 12);
  // 3. the opt-in table sequence: c = 16 (137 GB) dropped, c = 17 (258 GB) built
  b = alloc_touch("fresh_137", 137);
  free_timed("free_137", b, 137);
  void* c = alloc_touch("after_free137_258", 258);
  free_timed("free_258", c, 258);
  std::this_thread::sleep_for(std::chrono::seconds(8));
  c = alloc_touch("after_wait8s_258", 258);
  free_timed("free_258", c, 258);
  // 4. without a memset of the freed block (was it the written bytes?)
  void* d = nullptr;
  double t0 = now_ms();
  CK(hipMalloc(&d, (size_t)137 << 30));
  double t1 = now_ms();
  CK(hipFree(d));
  double t2 = now_ms();
  std::printf("{\"case\": \"untouched_137\", \"malloc_ms\": %.3f, \"free_ms\": %.3f}\n", t1 - t0, t2 - t1);
  c = alloc_touch("after_free_untouched137_258", 258);
  free_timed("free_258", c, 258);
  return 0;
}
