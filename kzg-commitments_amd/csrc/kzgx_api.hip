// C ABI of libkzgx.so (declared in include/kzg_gpu.h).  Thin host layer:
// argument checks, staging copies for the host-pointer entry points, and
// dispatch into the HIP kernels of msm.hip / poly.hip / srs.hip.  No compute
// happens on the host and there is no CPU fallback: without a gfx950 device
// kzgx_create fails with KZGX_ERR_NO_DEVICE.
#include <hip/hip_runtime.h>

#include <map>
#include <mutex>

#include <array>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "curve_consts.h"
#include "kzgx_internal.hpp"
#include "kzgx_setup.hpp"

// a generated G2 SRS of at most this many points gets its polyeval_G2 window
// table at setup (kzgx_gen_srs_g2); larger ones on first use
#ifndef KZGX_G2TAB_EAGER_MAX
#define KZGX_G2TAB_EAGER_MAX 16385
#endif

struct kzgx_ctx {
  kzgx::Ctx c;
  uint32_t* d_srs_canon = nullptr;  // installed SRS, canonical affine
  size_t srs_canon_b = 0;
  uint32_t* d_srs2_canon = nullptr;  // installed G2 SRS, canonical affine (x.re, x.im, y.re, y.im)
  size_t srs2_canon_b = 0;
  size_t n_srs2 = 0;
  // wave-per-opening verify: tables derived from G1[0], G2[0..1] (built on
  // first use, dropped when either SRS changes)
  uint32_t* d_vw = nullptr;
  size_t vw_b = 0;
  bool vw_ready = false;
  size_t vw_max = 8192;  // batches up to this size take the wave path
  // windowed multiples of the G2 SRS for polyeval_G2 (built on first use)
  uint32_t* d_g2tab = nullptr;
  size_t g2tab_b = 0;
  size_t g2tab_n = 0;  // points covered; 0 = stale

  // pinned, device-mapped host staging for the host-pointer entry points
  // (kzgx_msm_g1_batch, kzgx_prove_single_batch): inputs are copied into it
  // and read by the kernels in place (small) or DMA'd from it (large); the
  // last kernel of a call writes its results straight into it, so a call
  // makes no device-to-host copy and synchronises once
  uint8_t* h_pin = nullptr;
  uint8_t* d_pin = nullptr;  // device address of h_pin
  size_t pin_b = 0;

  // verify_proof's side stream (from the device pool, on first use): the G2
  // half ([Z(tau)]G2) runs there beside the G1 half (I, [I(tau)]G1, C - it)
  hipStream_t side = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
};

namespace kzgx {

int hip_fail(hipError_t e) { return e == hipErrorOutOfMemory ? KZGX_ERR_OOM : KZGX_ERR_HIP; }

// Freed table blocks are cached per device for later tables.  A
// trusted_setup per degree (the reference benchmark,
// benchmark/benchmark.cpp:19-38) otherwise frees one default table and
// allocates the next.  Why that matters: the amdgpu driver wipes released
// VRAM before it hands it out again, at ~30 GB/s, and work on a block that
// lands on freed memory waits for that wipe (137 GB freed -> the next large
// hipMalloc 4.1-4.9 s, 0.3 ms on clean memory; scripts/probe_alloc.hip,
// profiles/r06_probe_alloc.jsonl).  So a freed block of 64 MB .. 32 GB is kept (up to 32 GB per device in all,
// oldest evicted first), a request takes the smallest cached block that
// fits it with at most 2x + 64 MB slack, and a request nothing fits gets a
// fresh allocation beside the cached blocks -- freeing them first would put
// it on memory that is being wiped.  The cache is released on an allocation
// failure, when the last context of the device is destroyed, and by
// kzgx_release_cached_memory; KZGX_NO_TABLE_CACHE=1 turns it off.
namespace {
struct TableBlock {
  void* p = nullptr;
  size_t bytes = 0;
};
constexpr size_t CACHE_MIN = (size_t)64 << 20;
constexpr size_t CACHE_CAP = (size_t)32 << 30;
std::mutex g_table_mu;
std::vector<TableBlock> g_table_cache[64];  // oldest first
size_t g_cache_bytes[64];
std::map<void*, size_t> g_block_bytes;  // true size of each block table_malloc handed out
int g_live_ctx[64];  // live contexts per device (guarded by g_table_mu)
bool table_cache_off() {
  static const bool off = std::getenv("KZGX_NO_TABLE_CACHE") && std::getenv("KZGX_NO_TABLE_CACHE")[0] == '1';
  return off;
}
int current_device() {
  int dev = 0;
  return hipGetDevice(&dev) == hipSuccess && dev >= 0 && dev < 64 ? dev : -1;
}
void cache_release_locked(int dev) {
  for (auto& b : g_table_cache[dev]) {
    g_block_bytes.erase(b.p);
    (void)hipFree(b.p);
  }
  g_table_cache[dev].clear();
  g_cache_bytes[dev] = 0;
}
}  // namespace

void table_cache_release() {
  const int dev = current_device();
  if (dev < 0) return;
  std::lock_guard<std::mutex> lk(g_table_mu);
  cache_release_locked(dev);
}

// a context created (+1) or destroyed (-1) on `dev`; the last one to go
// releases the device's cached blocks (nothing else would)
void ctx_live_add(int dev, int delta) {
  if (dev < 0 || dev >= 64) return;
  std::lock_guard<std::mutex> lk(g_table_mu);
  g_live_ctx[dev] += delta;
  if (g_live_ctx[dev] <= 0) {
    g_live_ctx[dev] = 0;
    cache_release_locked(dev);
  }
}

// bytes held by the current device's cached blocks: memory a table build may
// count as free (table_malloc reuses them or releases them on failure)
size_t table_cache_bytes() {
  const int dev = current_device();
  if (dev < 0) return 0;
  std::lock_guard<std::mutex> lk(g_table_mu);
  return g_cache_bytes[dev];
}

hipError_t table_malloc(void** p, size_t bytes) {
  const int dev = current_device();
  if (dev >= 0) {
    std::lock_guard<std::mutex> lk(g_table_mu);
    auto& c = g_table_cache[dev];
    int best = -1;
    for (int k = 0; k < (int)c.size(); k++)
      if (c[k].bytes >= bytes && c[k].bytes <= 2 * bytes + CACHE_MIN && (best < 0 || c[k].bytes < c[best].bytes))
        best = k;
    if (best >= 0) {
      *p = c[best].p;
      g_cache_bytes[dev] -= c[best].bytes;
      c.erase(c.begin() + best);
      return hipSuccess;
    }
  }
  hipError_t e = hipMalloc(p, bytes);
  if (e == hipErrorOutOfMemory && dev >= 0) {  // the cached blocks may be what is missing
    (void)hipGetLastError();
    {
      std::lock_guard<std::mutex> lk(g_table_mu);
      cache_release_locked(dev);
    }
    e = hipMalloc(p, bytes);
  }
  if (e == hipSuccess) {
    std::lock_guard<std::mutex> lk(g_table_mu);
    g_block_bytes[*p] = bytes;
  }
  return e;
}

void table_free(void* p, size_t bytes) {
  if (!p) return;
  const int dev = current_device();
  std::lock_guard<std::mutex> lk(g_table_mu);
  const auto it = g_block_bytes.find(p);
  if (it != g_block_bytes.end()) bytes = it->second;  // the block's own size (it may have served a smaller table)
  // blocks of 64 MB .. 32 GB: an opt-in table of hundreds of GB is freed at once
  if (table_cache_off() || bytes < CACHE_MIN || bytes > CACHE_CAP || dev < 0) {
    if (it != g_block_bytes.end()) g_block_bytes.erase(it);
    (void)hipFree(p);
    return;
  }
  auto& c = g_table_cache[dev];
  c.push_back(TableBlock{p, bytes});
  g_cache_bytes[dev] += bytes;
  while (g_cache_bytes[dev] > CACHE_CAP && !c.empty()) {  // oldest first
    g_cache_bytes[dev] -= c.front().bytes;
    g_block_bytes.erase(c.front().p);
    (void)hipFree(c.front().p);
    c.erase(c.begin());
  }
}

// Shared default tables: contexts on one
// device whose SRS starts with the same points (compared word for word, not
// by a hash) and that pick the same window share one default table, counted
// by reference.  kzgx_msm_g1_sharded-style callers and repeated trusted
// setups then hold one 11.8 GB table, not one per context.
namespace {
struct SharedTable {
  int id = 0;
  int device = 0, curve = 0;
  uint32_t* d_key = nullptr;  // device copy of the canonical SRS prefix the table was built from
  size_t key_words = 0;
  FixedTable t;  // owner's view of the table (d, inf, c, W, n_t, ...)
  int refs = 0;
};
std::vector<SharedTable> g_shared;  // guarded by g_table_mu
int g_shared_next = 1;

// *differ = (a[0..words) != b[0..words)), both on the device, compared by a
// kernel that stores into a mapped host word: the setup path makes no
// device-to-host copy (a 32 KB one stalled 6-18 ms now and then inside the
// reference benchmark's 512-term setup, profiles/r06_kzg_bench_trace_setup.txt)
__global__ void k_words_differ(const uint32_t* __restrict__ a, const uint32_t* __restrict__ b, size_t words,
                               volatile uint32_t* __restrict__ flag) {
  for (size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x; k < words; k += (size_t)gridDim.x * blockDim.x)
    if (a[k] != b[k]) *flag = 1u;  // every writer stores the same value
}
int words_differ(const uint32_t* a, const uint32_t* b, size_t words, hipStream_t st, bool* differ) {
  thread_local uint32_t* h_flag = nullptr;  // mapped pinned word, kept for the thread
  thread_local uint32_t* d_flag = nullptr;
  if (!h_flag) {
    KZGX_TRY_HIP(hipHostMalloc((void**)&h_flag, 64, hipHostMallocMapped | hipHostMallocCoherent));
    KZGX_TRY_HIP(hipHostGetDevicePointer((void**)&d_flag, h_flag, 0));
  }
  *(volatile uint32_t*)h_flag = 0u;
  const unsigned blocks = (unsigned)std::min<size_t>((words + 255) / 256, 1024);
  hipLaunchKernelGGL(k_words_differ, dim3(blocks ? blocks : 1), dim3(256), 0, st, a, b, words, d_flag);
  KZGX_TRY_HIP(hipGetLastError());
  KZGX_TRY_HIP(hipStreamSynchronize(st));
  *differ = *(volatile uint32_t*)h_flag != 0u;
  return KZGX_OK;
}
}  // namespace

bool table_share_attach(int device, int curve, int c_req, const uint32_t* d_canon, size_t key_words, hipStream_t st,
                        FixedTable& ft) {
  std::lock_guard<std::mutex> lk(g_table_mu);
  for (auto& e : g_shared) {
    if (e.device != device || e.curve != curve || (c_req > 0 && e.t.c != c_req) || e.key_words != key_words) continue;
    bool differ = true;
    if (words_differ(e.d_key, d_canon, key_words, st, &differ) != KZGX_OK || differ) continue;
    const uint32_t ppt = ft.pts_per_thread;
    const int c_keep = ft.c_req;
    const size_t n_keep = ft.n_req;
    const int layout_keep = ft.layout_req;
    ft = e.t;
    ft.pts_per_thread = ppt;
    ft.c_req = c_keep;
    ft.n_req = n_keep;
    ft.layout_req = layout_keep;
    ft.shared = e.id;
    e.refs++;
    return true;
  }
  return false;
}

// ft (just built from d_canon's first key_words words) becomes shareable; a
// failure to keep the key just leaves it unshared
void table_share_register(int device, int curve, const uint32_t* d_canon, size_t key_words, hipStream_t st,
                          FixedTable& ft) {
  uint32_t* d_key = nullptr;
  if (hipMalloc((void**)&d_key, key_words * 4) != hipSuccess) {
    (void)hipGetLastError();
    return;
  }
  if (hipMemcpyAsync(d_key, d_canon, key_words * 4, hipMemcpyDeviceToDevice, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess) {
    (void)hipFree(d_key);
    return;
  }
  std::lock_guard<std::mutex> lk(g_table_mu);
  SharedTable e;
  e.id = g_shared_next++;
  e.device = device;
  e.curve = curve;
  e.d_key = d_key;
  e.key_words = key_words;
  e.t = ft;
  e.refs = 1;
  ft.shared = e.id;
  g_shared.push_back(std::move(e));
}

// drop ft's reference; the last one frees the table (into the block cache)
void table_share_release(FixedTable& ft) {
  void* d = nullptr;
  uint8_t* inf = nullptr;
  uint32_t* key = nullptr;
  size_t bytes = 0;
  {
    std::lock_guard<std::mutex> lk(g_table_mu);
    for (size_t k = 0; k < g_shared.size(); k++) {
      if (g_shared[k].id != ft.shared) continue;
      if (--g_shared[k].refs == 0) {
        d = g_shared[k].t.d;
        inf = g_shared[k].t.inf;
        key = g_shared[k].d_key;
        bytes = g_shared[k].t.bytes;
        g_shared.erase(g_shared.begin() + (long)k);
      }
      break;
    }
  }
  if (d) table_free(d, bytes);
  if (inf) (void)hipFree(inf);
  if (key) (void)hipFree(key);
}

void shared_tables_info(int device, size_t* count, size_t* bytes) {
  std::lock_guard<std::mutex> lk(g_table_mu);
  size_t c = 0, b = 0;
  for (auto& e : g_shared)
    if (e.device == device) c++, b += e.t.bytes;
  *count = c;
  *bytes = b;
}

int dev_alloc(Ctx* ctx, void** p, size_t bytes, size_t* cap) {
  (void)ctx;
  if (bytes == 0) bytes = 16;
  if (*p && bytes <= *cap) return KZGX_OK;
  if (*p) {
    KZGX_TRY_HIP(hipDeviceSynchronize());
    KZGX_TRY_HIP(hipFree(*p));
    *p = nullptr;
    *cap = 0;
  }
  // round up to limit re-allocation churn
  size_t want = bytes + bytes / 8;
  hipError_t e = hipMalloc(p, want);
  if (e != hipSuccess) {
    *p = nullptr;
    table_cache_release();  // a cached table block may be what is missing
    e = hipMalloc(p, bytes);
    if (e != hipSuccess) {
      *p = nullptr;
      return hip_fail(e);
    }
    want = bytes;
  }
  *cap = want;
  return KZGX_OK;
}

}  // namespace kzgx

using kzgx::Ctx;

namespace {

int activate(kzgx_ctx* ctx) {
  if (!ctx) return KZGX_ERR_ARG;
  KZGX_TRY_HIP(hipSetDevice(ctx->c.device));
  return KZGX_OK;
}

hipStream_t pick(kzgx_ctx* ctx, void* stream) { return stream ? (hipStream_t)stream : ctx->c.stream; }

int stage(kzgx_ctx* ctx, int slot, size_t bytes, void** out) {
  KZGX_TRY(kzgx::dev_alloc(&ctx->c, &ctx->c.d_stage[slot], bytes, &ctx->c.stage_b[slot]));
  *out = ctx->c.d_stage[slot];
  return KZGX_OK;
}

size_t point_words(const kzgx_ctx* ctx) { return 2 * (size_t)ctx->c.base_words(); }

// the context's pinned mapped staging of at least `bytes` (grow-only)
int pin_stage(kzgx_ctx* ctx, size_t bytes) {
  if (ctx->h_pin && bytes <= ctx->pin_b) return KZGX_OK;
  if (ctx->h_pin) {
    KZGX_TRY_HIP(hipStreamSynchronize(ctx->c.stream));
    (void)hipHostFree(ctx->h_pin);
    ctx->h_pin = ctx->d_pin = nullptr;
    ctx->pin_b = 0;
  }
  const size_t want = std::max<size_t>(bytes + bytes / 8, (size_t)1 << 20);
  void* h = nullptr;
  KZGX_TRY_HIP(hipHostMalloc(&h, want, hipHostMallocMapped | hipHostMallocCoherent));
  void* d = nullptr;
  const hipError_t e = hipHostGetDevicePointer(&d, h, 0);
  if (e != hipSuccess) {
    (void)hipHostFree(h);
    return kzgx::hip_fail(e);
  }
  ctx->h_pin = static_cast<uint8_t*>(h);
  ctx->d_pin = static_cast<uint8_t*>(d);
  ctx->pin_b = want;
  return KZGX_OK;
}

// kernels read inputs up to this size straight from the mapped staging
// (PCIe reads, no copy launch); larger inputs are DMA'd to device memory
constexpr size_t PIN_DIRECT_MAX = (size_t)256 << 10;

size_t align256(size_t b) { return (b + 255) & ~(size_t)255; }

// x mod r for a 4 x 64-bit little-endian value: the reference converts its
// evaluation points into ZZ_p (src/trusted_setup.cpp:214-219), so x and x + r
// are the same point.  Argument normalisation only (a handful of compares and
// subtractions per point), done before the repeated-point check.
template <class FR>
std::array<uint64_t, 4> fr_reduce(const uint64_t* x) {
  uint64_t r[4], v[4] = {x[0], x[1], x[2], x[3]};
  for (int i = 0; i < 4; i++) r[i] = (uint64_t)FR::P[2 * i] | ((uint64_t)FR::P[2 * i + 1] << 32);
  for (;;) {
    int i = 3;
    while (i >= 0 && v[i] == r[i]) i--;
    if (i >= 0 && v[i] < r[i]) break;  // v < r (i < 0: v == r, reduces to 0)
    unsigned __int128 borrow = 0;
    for (int k = 0; k < 4; k++) {
      const unsigned __int128 d = (unsigned __int128)v[k] - r[k] - borrow;
      v[k] = (uint64_t)d;
      borrow = (d >> 64) & 1;
    }
  }
  return {v[0], v[1], v[2], v[3]};
}

// gfx950 device check shared by kzgx_create and kzgx_init_device
int device_ok(int device) {
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return KZGX_ERR_NO_DEVICE;
  if (device < 0 || device >= ndev) return KZGX_ERR_ARG;
  hipDeviceProp_t prop;
  KZGX_TRY_HIP(hipGetDeviceProperties(&prop, device));
  if (std::string(prop.gcnArchName).find("gfx950") == std::string::npos) return KZGX_ERR_NO_DEVICE;
  return KZGX_OK;
}

int setup_finish(kzgx_ctx* ctx);

}  // namespace

extern "C" {

const char* kzgx_strerror(int s) {
  switch (s) {
    case KZGX_OK: return "ok";
    case KZGX_ERR_ARG: return "invalid argument";
    case KZGX_ERR_HIP: return "HIP runtime error";
    case KZGX_ERR_OOM: return "device out of memory";
    case KZGX_ERR_NO_SRS: return "no SRS loaded";
    case KZGX_ERR_DEGREE: return "polynomial degree be at most one less than the setup size (num_coeffs)";
    case KZGX_ERR_INTERNAL: return "internal error";
    case KZGX_ERR_NO_DEVICE: return "no gfx950 (MI355X) device available";
    case KZGX_ERR_DIV_ZERO: return "division by zero (duplicate interpolation point)";
    default: return "unknown status";
  }
}

int kzgx_base_limbs(int curve) {
  return curve == KZGX_CURVE_BN254 ? 4 : curve == KZGX_CURVE_BLS12381 ? 6 : -1;
}

// Context streams are pooled per device: creating one costs 1.5-2 ms (the
// first few of a process up to 8.5 ms, each new hardware queue), and the
// reference benchmark builds one trusted_setup per degree
// (profiles/r05_kzg_bench_trace: the 128-term setup's stream creation was a
// third of its time).  Destroyed contexts return theirs after a sync.
namespace {
std::mutex g_stream_mu;
std::vector<hipStream_t> g_stream_pool[64];
constexpr size_t STREAM_POOL_MAX = 4;
hipError_t stream_take(int device, hipStream_t* s) {
  if (device >= 0 && device < 64) {
    std::lock_guard<std::mutex> lk(g_stream_mu);
    if (!g_stream_pool[device].empty()) {
      *s = g_stream_pool[device].back();
      g_stream_pool[device].pop_back();
      return hipSuccess;
    }
  }
  return hipStreamCreateWithFlags(s, hipStreamNonBlocking);
}
void stream_give(int device, hipStream_t s) {
  if (!s) return;
  if (device >= 0 && device < 64) {
    std::lock_guard<std::mutex> lk(g_stream_mu);
    if (g_stream_pool[device].size() < STREAM_POOL_MAX) {
      g_stream_pool[device].push_back(s);
      return;
    }
  }
  (void)hipStreamDestroy(s);
}
}  // namespace

int kzgx_init_device(int curve, int device) {
  if (curve != KZGX_CURVE_BN254 && curve != KZGX_CURVE_BLS12381) return KZGX_ERR_ARG;
  KZGX_TRY(device_ok(device));
  KZGX_TRY_HIP(hipSetDevice(device));
  // the streams of the first contexts (kzg::init's default context, the
  // first trusted_setup), created here, outside the timed regions
  hipStream_t spare[3] = {nullptr, nullptr, nullptr};  // (+1: verify_proof's side stream)
  for (auto& s2 : spare) KZGX_TRY_HIP(stream_take(device, &s2));
  for (auto s2 : spare) stream_give(device, s2);
  hipStream_t st = nullptr;
  KZGX_TRY_HIP(stream_take(device, &st));
  struct StreamGuard {
    hipStream_t s;
    int d;
    ~StreamGuard() {
      (void)hipStreamSynchronize(s);
      stream_give(d, s);
    }
  } sg{st, device};
  // every code object of the library, once (the first launch of any kernel
  // of a translation unit loads its whole object)
  int (*const warm[])(hipStream_t) = {
      kzgx::warm_setup,      kzgx::warm_msm,        kzgx::warm_msm_fixed,   kzgx::warm_poly,
      kzgx::warm_srs,        kzgx::warm_pairing,    kzgx::warm_verify_wave, kzgx::warm_latency,
      kzgx::warm_fixed_bn_a, kzgx::warm_fixed_bn_b, kzgx::warm_fixed_bn_c,  kzgx::warm_fixed_bn_d,
      kzgx::warm_fixed_bls_a, kzgx::warm_fixed_bls_b, kzgx::warm_fixed_bls_c, kzgx::warm_fixed_bls_d};
  for (auto f : warm) KZGX_TRY(f(st));
  // the generator comb tables (per process, per device and curve)
  kzgx::GenTables g;
  KZGX_TRY(kzgx::gen_tables_get(curve, device, st, &g));
  // the pinned-allocation path of the host-pointer calls
  void* h = nullptr;
  KZGX_TRY_HIP(hipHostMalloc(&h, 4096, hipHostMallocMapped | hipHostMallocCoherent));
  (void)hipHostFree(h);
  KZGX_TRY_HIP(hipStreamSynchronize(st));
  return KZGX_OK;
}

int kzgx_create(kzgx_ctx** out, int curve, int device) {
  if (!out || (curve != KZGX_CURVE_BN254 && curve != KZGX_CURVE_BLS12381)) return KZGX_ERR_ARG;
  *out = nullptr;
  KZGX_TRY(device_ok(device));
  kzgx_ctx* ctx = new (std::nothrow) kzgx_ctx();
  if (!ctx) return KZGX_ERR_OOM;
  ctx->c.curve = curve;
  ctx->c.device = device;
  if (const char* e = getenv("KZGX_WINDOW_BITS")) {
    int c = atoi(e);
    if (kzgx::window_bits_supported(c)) ctx->c.c = c;
  }
  ctx->c.W = (257 + ctx->c.c - 1) / ctx->c.c;
  hipError_t e = hipSetDevice(device);
  if (e == hipSuccess) e = stream_take(device, &ctx->c.stream);
  if (e != hipSuccess) {
    delete ctx;
    return kzgx::hip_fail(e);
  }
  kzgx::ctx_live_add(device, +1);
  *out = ctx;
  return KZGX_OK;
}

int kzgx_release_cached_memory(int device) {
  if (device < 0 || device >= 64) return KZGX_ERR_ARG;
  int prev = 0;
  KZGX_TRY_HIP(hipGetDevice(&prev));
  KZGX_TRY_HIP(hipSetDevice(device));
  kzgx::table_cache_release();
  return hipSetDevice(prev) == hipSuccess ? KZGX_OK : KZGX_ERR_HIP;
}

int kzgx_shared_tables(int device, size_t* count, size_t* bytes) {
  if (!count || !bytes || device < 0 || device >= 64) return KZGX_ERR_ARG;
  kzgx::shared_tables_info(device, count, bytes);
  return KZGX_OK;
}

void kzgx_destroy(kzgx_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->c.device);
  (void)hipStreamSynchronize(ctx->c.stream);
  (void)kzgx_prof_clear(ctx);
  Ctx& c = ctx->c;
  void* bufs[] = {c.d_table, c.d_table_small, c.d_table_big, c.d_inf, c.d_stage[0], c.d_stage[1], c.d_stage[2], c.d_stage[3],
                  c.d_poly_ws, c.d_poly_ws2, ctx->d_srs_canon, ctx->d_srs2_canon, c.d_g2_ws, ctx->d_vw, ctx->d_g2tab,
                  c.d_lift};
  for (void* p : bufs)
    if (p) (void)hipFree(p);
  kzgx::fixed_free(&c);
  kzgx::fixed_free_table(c.fixed_def);
  for (auto& w : c.ws) {
    void* wb[] = {w.counts, w.offsets, w.cursors, w.entries, w.bsum,  w.heads,
                  w.tails,  w.tailk,   w.rt,      w.q,       w.parts, w.fpart, w.fsum, w.gpart, w.gmeta, w.sstate, w.qbig,
                  w.lat_cnt};
    for (void* p : wb)
      if (p) (void)hipFree(p);
    if (w.done) (void)hipEventDestroy(w.done);
  }
  if (ctx->h_pin) (void)hipHostFree(ctx->h_pin);
  if (c.small_ev) (void)hipEventDestroy(c.small_ev);
  if (ctx->side) {
    (void)hipStreamSynchronize(ctx->side);
    stream_give(c.device, ctx->side);
  }
  if (ctx->ev_fork) (void)hipEventDestroy(ctx->ev_fork);
  if (ctx->ev_join) (void)hipEventDestroy(ctx->ev_join);
  (void)hipStreamSynchronize(c.stream);
  stream_give(c.device, c.stream);
  kzgx::ctx_live_add(c.device, -1);
  delete ctx;
}

int kzgx_sync(kzgx_ctx* ctx) {
  KZGX_TRY(activate(ctx));
  KZGX_TRY_HIP(hipStreamSynchronize(ctx->c.stream));
  return KZGX_OK;
}

void* kzgx_stream(kzgx_ctx* ctx) { return ctx ? (void*)ctx->c.stream : nullptr; }

int kzgx_prof_enable(kzgx_ctx* ctx, int on) {
  KZGX_TRY(activate(ctx));
  ctx->c.prof_on = on != 0;
  return KZGX_OK;
}

int kzgx_prof_read(kzgx_ctx* ctx, const char* name, double* total_ms, int* count) {
  KZGX_TRY(activate(ctx));
  if (!name || !total_ms || !count) return KZGX_ERR_ARG;
  double tot = 0;
  int cnt = 0;
  std::vector<kzgx::ProfRec> keep;
  for (auto& r : ctx->c.prof) {
    if (std::strcmp(r.name, name) != 0) {
      keep.push_back(r);
      continue;
    }
    KZGX_TRY_HIP(hipEventSynchronize(r.b));
    float ms = 0;
    KZGX_TRY_HIP(hipEventElapsedTime(&ms, r.a, r.b));
    tot += ms;
    cnt++;
    (void)hipEventDestroy(r.a);
    (void)hipEventDestroy(r.b);
  }
  ctx->c.prof.swap(keep);
  *total_ms = tot;
  *count = cnt;
  return KZGX_OK;
}

int kzgx_prof_clear(kzgx_ctx* ctx) {
  KZGX_TRY(activate(ctx));
  for (auto& r : ctx->c.prof) {
    (void)hipEventSynchronize(r.b);
    (void)hipEventDestroy(r.a);
    (void)hipEventDestroy(r.b);
  }
  ctx->c.prof.clear();
  return KZGX_OK;
}

int kzgx_set_window_bits(kzgx_ctx* ctx, int c) {
  KZGX_TRY(activate(ctx));
  if (!kzgx::window_bits_supported(c)) return KZGX_ERR_ARG;
  if (ctx->c.n_srs != 0) return KZGX_ERR_ARG;  // the fixed-base table depends on c
  ctx->c.c = c;
  ctx->c.W = (257 + c - 1) / c;
  return KZGX_OK;
}

int kzgx_set_small_batch(kzgx_ctx* ctx, unsigned max_batch) {
  KZGX_TRY(activate(ctx));
  if (max_batch > 65535) return KZGX_ERR_ARG;
  ctx->c.small_batch = max_batch;
  return KZGX_OK;
}

int kzgx_set_segment(kzgx_ctx* ctx, unsigned k) {
  KZGX_TRY(activate(ctx));
  if (k < 1 || k > 4096) return KZGX_ERR_ARG;
  ctx->c.seg_k = k;
  return KZGX_OK;
}

int kzgx_set_fixed_base(kzgx_ctx* ctx, int c, size_t n_points) {
  KZGX_TRY(activate(ctx));
  if (!kzgx::fixed_bits_supported(c)) return KZGX_ERR_ARG;
  if (c != 0 && n_points == 0) return KZGX_ERR_ARG;
  KZGX_TRY_HIP(hipStreamSynchronize(ctx->c.stream));
  kzgx::fixed_free(&ctx->c);
  ctx->c.fixed.c_req = c;
  ctx->c.fixed.n_req = c ? n_points : 0;
  if (c != 0 && ctx->c.n_srs != 0)
    KZGX_TRY(kzgx::fixed_build_table(&ctx->c, ctx->c.fixed, ctx->d_srs_canon, ctx->c.n_srs));  // the default table stays
  return KZGX_OK;
}

int kzgx_set_default_table(kzgx_ctx* ctx, int c, size_t n_points) {
  KZGX_TRY(activate(ctx));
  if (c != -1 && !kzgx::fixed_bits_supported(c)) return KZGX_ERR_ARG;
  if (c != 0 && n_points == 0) return KZGX_ERR_ARG;
  KZGX_TRY_HIP(hipStreamSynchronize(ctx->c.stream));
  kzgx::fixed_free_table(ctx->c.fixed_def);
  ctx->c.fixed_def.c_req = c;
  ctx->c.fixed_def.n_req = c ? n_points : 0;
  if (c != 0 && ctx->c.n_srs != 0) KZGX_TRY(kzgx::fixed_rebuild_default(&ctx->c, ctx->d_srs_canon, ctx->c.n_srs));
  return KZGX_OK;
}

int kzgx_default_table_info(const kzgx_ctx* ctx, int* c, size_t* n_points, size_t* bytes) {
  if (!ctx) return KZGX_ERR_ARG;
  if (c) *c = ctx->c.fixed_def.c;
  if (n_points) *n_points = ctx->c.fixed_def.n_t;
  if (bytes) *bytes = ctx->c.fixed_def.bytes;
  return KZGX_OK;
}

int kzgx_set_fixed_base_layout(kzgx_ctx* ctx, int layout) {
  KZGX_TRY(activate(ctx));
  if (layout < -1 || layout > 1) return KZGX_ERR_ARG;
  ctx->c.fixed.layout_req = layout;
  return KZGX_OK;
}

int kzgx_fixed_base_layout(const kzgx_ctx* ctx, int* point_major) {
  if (!ctx || !point_major) return KZGX_ERR_ARG;
  *point_major = ctx->c.fixed.point_major ? 1 : 0;
  return KZGX_OK;
}

int kzgx_fixed_base_info(const kzgx_ctx* ctx, int* c, size_t* n_points, size_t* bytes) {
  if (!ctx) return KZGX_ERR_ARG;
  if (c) *c = ctx->c.fixed.c;
  if (n_points) *n_points = ctx->c.fixed.n_t;
  if (bytes) *bytes = ctx->c.fixed.bytes;
  return KZGX_OK;
}

int kzgx_fixed_base_bytes(int curve, int c, size_t n_points, size_t* bytes) {
  if (!bytes || (curve != KZGX_CURVE_BN254 && curve != KZGX_CURVE_BLS12381) || !kzgx::fixed_bits_supported(c))
    return KZGX_ERR_ARG;
  *bytes = kzgx::fixed_table_bytes(curve, c, n_points);
  return KZGX_OK;
}

int kzgx_set_fixed_base_budget(kzgx_ctx* ctx, size_t budget_bytes, size_t n_points, int* c_out) {
  KZGX_TRY(activate(ctx));
  if (!c_out || n_points == 0) return KZGX_ERR_ARG;
  *c_out = 0;
  // the budget is sized against the free HBM after the SRS and its window
  // tables exist, and for the points that will actually be tabled
  if (ctx->c.n_srs == 0) return KZGX_ERR_NO_SRS;
  if (n_points > ctx->c.n_srs) n_points = ctx->c.n_srs;
  KZGX_TRY_HIP(hipStreamSynchronize(ctx->c.stream));
  kzgx::fixed_free(&ctx->c);  // the old table's memory counts as free
  size_t free_b = 0, total_b = 0;
  KZGX_TRY_HIP(hipMemGetInfo(&free_b, &total_b));
  free_b += kzgx::table_cache_bytes();  // reused or released by table_malloc
  const size_t margin = (size_t)4 << 30;
  const size_t avail = free_b > margin ? free_b - margin : 0;
  const size_t cap = budget_bytes < avail ? budget_bytes : avail;
  for (int c = 17; c >= 7; c--) {
    if (kzgx::fixed_table_bytes(ctx->c.curve, c, n_points) > cap) continue;
    const int rc = kzgx_set_fixed_base(ctx, c, n_points);
    if (rc == KZGX_OK) {
      *c_out = c;
      return KZGX_OK;
    }
    if (rc != KZGX_ERR_OOM) {
      ctx->c.fixed.c_req = 0;  // no half-requested window left for the next SRS upload
      ctx->c.fixed.n_req = 0;
      return rc;
    }
  }
  ctx->c.fixed.c_req = 0;
  ctx->c.fixed.n_req = 0;
  return KZGX_OK;
}

int kzgx_microbench_mad_u64(kzgx_ctx* ctx, double* lane_ops_per_s) {
  KZGX_TRY(activate(ctx));
  if (!lane_ops_per_s) return KZGX_ERR_ARG;
  KZGX_TRY_HIP(hipStreamSynchronize(ctx->c.stream));
  return kzgx::microbench_mad_u64(&ctx->c, lane_ops_per_s, nullptr);
}

int kzgx_microbench_mad_u64_clock(kzgx_ctx* ctx, double* lane_ops_per_s, double* core_ghz) {
  KZGX_TRY(activate(ctx));
  if (!lane_ops_per_s || !core_ghz) return KZGX_ERR_ARG;
  KZGX_TRY_HIP(hipStreamSynchronize(ctx->c.stream));
  return kzgx::microbench_mad_u64(&ctx->c, lane_ops_per_s, core_ghz);
}

int kzgx_clock_probe(kzgx_ctx* ctx, void* stream, unsigned spin_us, void* d_out) {
  KZGX_TRY(activate(ctx));
  if (!d_out || spin_us == 0 || spin_us > 10000000u) return KZGX_ERR_ARG;
  return kzgx::clock_probe(&ctx->c, pick(ctx, stream), spin_us, static_cast<uint64_t*>(d_out));
}

int kzgx_microbench_mixed_add(kzgx_ctx* ctx, double* adds_per_s) {
  KZGX_TRY(activate(ctx));
  if (!adds_per_s) return KZGX_ERR_ARG;
  KZGX_TRY_HIP(hipStreamSynchronize(ctx->c.stream));
  return kzgx::microbench_mixed_add(&ctx->c, adds_per_s);
}

int kzgx_set_fixed_points_per_thread(kzgx_ctx* ctx, unsigned p) {
  KZGX_TRY(activate(ctx));
  if (p > 1024) return KZGX_ERR_ARG;  // 0 = automatic
  ctx->c.fixed.pts_per_thread = p;
  return KZGX_OK;
}

int kzgx_curve(const kzgx_ctx* ctx) { return ctx ? ctx->c.curve : -1; }

size_t kzgx_srs_size(const kzgx_ctx* ctx) { return ctx ? ctx->c.n_srs : 0; }

int kzgx_load_srs_g1(kzgx_ctx* ctx, const uint64_t* xy, size_t n) {
  KZGX_TRY(activate(ctx));
  ctx->vw_ready = false;
  if (!xy || n == 0) return KZGX_ERR_ARG;
  const size_t bytes = n * point_words(ctx) * 4;
  KZGX_TRY(kzgx::dev_alloc(&ctx->c, (void**)&ctx->d_srs_canon, bytes, &ctx->srs_canon_b));
  KZGX_TRY_HIP(hipMemcpyAsync(ctx->d_srs_canon, xy, bytes, hipMemcpyHostToDevice, ctx->c.stream));
  KZGX_TRY(kzgx::srs_upload(&ctx->c, ctx->d_srs_canon, n));
  KZGX_TRY_HIP(hipStreamSynchronize(ctx->c.stream));
  return setup_finish(ctx);
}

int kzgx_gen_srs_g1(kzgx_ctx* ctx, const uint64_t* tau, size_t start, size_t n) {
  KZGX_TRY(activate(ctx));
  ctx->vw_ready = false;
  if (!tau || n == 0 || n > 0x7fffffffu) return KZGX_ERR_ARG;
  const size_t bytes = n * point_words(ctx) * 4;
  KZGX_TRY(kzgx::dev_alloc(&ctx->c, (void**)&ctx->d_srs_canon, bytes, &ctx->srs_canon_b));
  void* d_tau;
  KZGX_TRY(stage(ctx, 0, 32, &d_tau));
  KZGX_TRY_HIP(hipMemcpyAsync(d_tau, tau, 32, hipMemcpyHostToDevice, ctx->c.stream));
  kzgx::GenTables g;
  KZGX_TRY(kzgx::gen_tables_get(ctx->c.curve, ctx->c.device, ctx->c.stream, &g));
  KZGX_TRY(kzgx::gen_srs_g1_comb(ctx->c.curve, (const uint32_t*)d_tau, start, n, g.g1_comb, ctx->d_srs_canon,
                                 ctx->c.stream));
  KZGX_TRY(kzgx::srs_upload(&ctx->c, ctx->d_srs_canon, n));
  KZGX_TRY_HIP(hipStreamSynchronize(ctx->c.stream));
  return setup_finish(ctx);
}

int kzgx_get_srs_g1(kzgx_ctx* ctx, uint64_t* xy, size_t n) {
  KZGX_TRY(activate(ctx));
  if (!xy) return KZGX_ERR_ARG;
  if (ctx->c.n_srs == 0) return KZGX_ERR_NO_SRS;
  if (n > ctx->c.n_srs) return KZGX_ERR_ARG;
  KZGX_TRY_HIP(hipMemcpyAsync(xy, ctx->d_srs_canon, n * point_words(ctx) * 4, hipMemcpyDeviceToHost, ctx->c.stream));
  KZGX_TRY_HIP(hipStreamSynchronize(ctx->c.stream));
  return KZGX_OK;
}

int kzgx_msm_g1_batch_device(kzgx_ctx* ctx, const void* d_scalars, size_t n, size_t batch, size_t scalar_stride,
                             void* d_out_xy, void* d_out_is_inf, void* stream) {
  KZGX_TRY(activate(ctx));
  if (batch == 0) return KZGX_OK;
  if (!d_out_xy || !d_out_is_inf || (n > 0 && !d_scalars) || batch > 65535) return KZGX_ERR_ARG;
  if (ctx->c.n_srs == 0) return KZGX_ERR_NO_SRS;
  if (n > ctx->c.n_srs) return KZGX_ERR_DEGREE;
  if (batch > 1 && scalar_stride < n) return KZGX_ERR_ARG;
  hipStream_t st = pick(ctx, stream);
  if (n == 0) {  // zero polynomial: ECP_inf (trusted_setup.cpp:150-154)
    KZGX_TRY_HIP(hipMemsetAsync(d_out_xy, 0, batch * point_words(ctx) * 4, st));
    std::vector<uint32_t> ones(batch, 1u);
    KZGX_TRY_HIP(hipMemcpyAsync(d_out_is_inf, ones.data(), batch * 4, hipMemcpyHostToDevice, st));
    KZGX_TRY_HIP(hipStreamSynchronize(st));
    return KZGX_OK;
  }
  return kzgx::msm_batch(&ctx->c, (const uint32_t*)d_scalars, n, batch, scalar_stride * 8, (uint32_t*)d_out_xy,
                         (uint32_t*)d_out_is_inf, st);
}

int kzgx_msm_g1_batch(kzgx_ctx* ctx, const uint64_t* scalars, size_t n, size_t batch, uint64_t* out_xy,
                      int* out_is_inf) {
  KZGX_TRY(activate(ctx));
  if (batch == 0) return KZGX_OK;
  if (!out_xy || !out_is_inf || (n > 0 && !scalars)) return KZGX_ERR_ARG;
  if (ctx->c.n_srs == 0) return KZGX_ERR_NO_SRS;
  if (n > ctx->c.n_srs) return KZGX_ERR_DEGREE;
  const size_t sb = n * batch * 32, ob = batch * point_words(ctx) * 4;
  // pinned layout: [results | flags | scalars]; results are written by the
  // last kernel into mapped host memory (no D2H copy).  Scalars up to
  // PIN_DIRECT_MAX are read by the kernels from the pinned copy; larger
  // ones are DMA'd straight from the caller's buffer (no host copy, and the
  // pinned buffer stays small: ADVICE r04)
  const bool direct = sb <= PIN_DIRECT_MAX;
  const size_t o_off = 0, i_off = align256(ob), s_off = i_off + align256(batch * 4);
  KZGX_TRY(pin_stage(ctx, s_off + (direct ? sb : 0)));
  void* d_s = nullptr;
  if (n) {
    if (direct) {
      std::memcpy(ctx->h_pin + s_off, scalars, sb);
      d_s = ctx->d_pin + s_off;
    } else {
      KZGX_TRY(stage(ctx, 0, sb, &d_s));
      KZGX_TRY_HIP(hipMemcpyAsync(d_s, scalars, sb, hipMemcpyHostToDevice, ctx->c.stream));
    }
  }
  KZGX_TRY(kzgx_msm_g1_batch_device(ctx, d_s, n, batch, n, ctx->d_pin + o_off, ctx->d_pin + i_off, nullptr));
  KZGX_TRY_HIP(hipStreamSynchronize(ctx->c.stream));
  std::memcpy(out_xy, ctx->h_pin + o_off, ob);
  const uint32_t* inf = reinterpret_cast<const uint32_t*>(ctx->h_pin + i_off);
  for (size_t b = 0; b < batch; b++) out_is_inf[b] = (int)inf[b];
  return KZGX_OK;
}

int kzgx_msm_g1(kzgx_ctx* ctx, const uint64_t* scalars, size_t n, uint64_t* out_xy, int* out_is_inf) {
  return kzgx_msm_g1_batch(ctx, scalars, n, 1, out_xy, out_is_inf);
}

int kzgx_quotient_single_batch_device(kzgx_ctx* ctx, const void* d_coeffs, size_t n, size_t coeff_stride,
                                      const void* d_z, size_t batch, void* d_q, size_t q_stride, void* d_y,
                                      void* stream) {
  KZGX_TRY(activate(ctx));
  if (batch == 0) return KZGX_OK;
  if (!d_z || (n > 0 && !d_coeffs) || (n > 1 && !d_q) || n > 0xffffffffu) return KZGX_ERR_ARG;
  if (batch > 1 && coeff_stride != 0 && coeff_stride < n) return KZGX_ERR_ARG;
  return kzgx::quotient_single(&ctx->c, (const uint32_t*)d_coeffs, n, coeff_stride * 8, (const uint32_t*)d_z, batch,
                               (uint32_t*)d_q, q_stride * 8, (uint32_t*)d_y, pick(ctx, stream));
}

int kzgx_quotient_single_batch(kzgx_ctx* ctx, const uint64_t* coeffs, size_t n, size_t coeff_stride,
                               const uint64_t* zs, size_t batch, uint64_t* q_out, uint64_t* y_out) {
  KZGX_TRY(activate(ctx));
  if (batch == 0) return KZGX_OK;
  if (!zs || (n > 0 && !coeffs) || (n > 1 && !q_out) || n > 0xffffffffu) return KZGX_ERR_ARG;
  if (batch > 1 && coeff_stride != 0 && coeff_stride < n) return KZGX_ERR_ARG;
  const size_t nc = coeff_stride == 0 ? n : (batch - 1) * coeff_stride + n;  // coefficient rows read
  const size_t nq = n > 1 ? n - 1 : 0;
  void *d_c = nullptr, *d_z, *d_q = nullptr, *d_y;
  if (nc) KZGX_TRY(stage(ctx, 0, nc * 32, &d_c));
  KZGX_TRY(stage(ctx, 1, batch * 32, &d_z));
  if (nq) KZGX_TRY(stage(ctx, 2, batch * nq * 32, &d_q));
  KZGX_TRY(stage(ctx, 3, batch * 32, &d_y));
  hipStream_t st = ctx->c.stream;
  if (nc) KZGX_TRY_HIP(hipMemcpyAsync(d_c, coeffs, nc * 32, hipMemcpyHostToDevice, st));
  KZGX_TRY_HIP(hipMemcpyAsync(d_z, zs, batch * 32, hipMemcpyHostToDevice, st));
  KZGX_TRY(kzgx::quotient_single(&ctx->c, (const uint32_t*)d_c, n, coeff_stride * 8, (const uint32_t*)d_z, batch,
                                 (uint32_t*)d_q, nq * 8, (uint32_t*)d_y, st));
  if (nq) KZGX_TRY_HIP(hipMemcpyAsync(q_out, d_q, batch * nq * 32, hipMemcpyDeviceToHost, st));
  if (y_out) KZGX_TRY_HIP(hipMemcpyAsync(y_out, d_y, batch * 32, hipMemcpyDeviceToHost, st));
  KZGX_TRY_HIP(hipStreamSynchronize(st));
  return KZGX_OK;
}

int kzgx_prove_single_batch_device(kzgx_ctx* ctx, const void* d_coeffs, size_t n, size_t coeff_stride,
                                   const void* d_z, size_t batch, void* d_out_xy, void* d_out_is_inf, void* d_y,
                                   void* stream) {
  KZGX_TRY(activate(ctx));
  if (batch == 0) return KZGX_OK;
  if (ctx->c.n_srs == 0) return KZGX_ERR_NO_SRS;
  const size_t nq = n > 0 ? n - 1 : 0;
  if (nq > ctx->c.n_srs) return KZGX_ERR_DEGREE;
  hipStream_t st = pick(ctx, stream);
  kzgx::WsLease ws = ctx->c.ws_for(st);
  if (!ws) return KZGX_ERR_ARG;
  void* d_q = nullptr;
  if (nq) {
    KZGX_TRY(kzgx::dev_alloc(&ctx->c, (void**)&ws->q, nq * batch * 32, &ws->q_b));
    d_q = ws->q;
  }
  KZGX_TRY(kzgx_quotient_single_batch_device(ctx, d_coeffs, n, coeff_stride, d_z, batch, d_q, nq, d_y, st));
  return kzgx_msm_g1_batch_device(ctx, d_q, nq, batch, nq, d_out_xy, d_out_is_inf, st);
}

int kzgx_prove_range(kzgx_ctx* ctx, const uint64_t* coeffs, size_t n, const uint64_t* xs, size_t len,
                     uint64_t* out_xy, int* out_is_inf) {
  KZGX_TRY(activate(ctx));
  if (!xs || !out_xy || !out_is_inf || len == 0 || (n > 0 && !coeffs) || len > (1u << 24)) return KZGX_ERR_ARG;
  if (ctx->c.n_srs == 0) return KZGX_ERR_NO_SRS;
  while (n > 0 && (coeffs[4 * (n - 1)] | coeffs[4 * (n - 1) + 1] | coeffs[4 * (n - 1) + 2] | coeffs[4 * (n - 1) + 3]) == 0)
    n--;  // NTL keeps polynomials normalized
  if (n > len && n - len > ctx->c.n_srs) return KZGX_ERR_DEGREE;
  // the points as residues mod r (x and x + r are one point, as in ZZ_p)
  std::vector<uint64_t> xr(4 * len);
  for (size_t i = 0; i < len; i++) {
    const auto v = ctx->c.curve == KZGX_CURVE_BN254 ? fr_reduce<kzgx::BN254Fr>(xs + 4 * i)
                                                    : fr_reduce<kzgx::BLS12381Fr>(xs + 4 * i);
    std::copy(v.begin(), v.end(), xr.begin() + 4 * i);
  }
  {
    // repeated points: the reference's interpolation (NTL polyfit) fails on
    // them, so does this call (P div Z alone would still be defined)
    std::vector<std::array<uint64_t, 4>> sorted(len);
    for (size_t i = 0; i < len; i++) sorted[i] = {xr[4 * i + 3], xr[4 * i + 2], xr[4 * i + 1], xr[4 * i]};
    std::sort(sorted.begin(), sorted.end());
    if (std::adjacent_find(sorted.begin(), sorted.end()) != sorted.end()) return KZGX_ERR_DIV_ZERO;
  }
  hipStream_t st = ctx->c.stream;
  kzgx::WsLease ws = ctx->c.ws_for(st);
  if (!ws) return KZGX_ERR_ARG;
  void *d_c = nullptr, *d_x, *d_o;
  if (n) KZGX_TRY(stage(ctx, 0, n * 32, &d_c));
  KZGX_TRY(stage(ctx, 1, len * 32, &d_x));
  KZGX_TRY(stage(ctx, 2, point_words(ctx) * 4 + 16, &d_o));
  if (n) KZGX_TRY_HIP(hipMemcpyAsync(d_c, coeffs, n * 32, hipMemcpyHostToDevice, st));
  KZGX_TRY_HIP(hipMemcpyAsync(d_x, xr.data(), len * 32, hipMemcpyHostToDevice, st));
  size_t nq = 0;
  if (n > len) {
    KZGX_TRY(kzgx::dev_alloc(&ctx->c, (void**)&ws->q, (n - len) * 32, &ws->q_b));
    KZGX_TRY(kzgx::prove_range_poly(&ctx->c, (const uint32_t*)d_c, n, (const uint32_t*)d_x, len, ws->q, &nq, st));
  }
  uint32_t* d_oi = (uint32_t*)((char*)d_o + point_words(ctx) * 4);
  KZGX_TRY(kzgx_msm_g1_batch_device(ctx, ws->q, nq, 1, nq, d_o, d_oi, st));
  uint32_t oi = 0;
  KZGX_TRY_HIP(hipMemcpyAsync(out_xy, d_o, point_words(ctx) * 4, hipMemcpyDeviceToHost, st));
  KZGX_TRY_HIP(hipMemcpyAsync(&oi, d_oi, 4, hipMemcpyDeviceToHost, st));
  KZGX_TRY_HIP(hipStreamSynchronize(st));
  *out_is_inf = (int)oi;
  return KZGX_OK;
}

int kzgx_prove_single_batch(kzgx_ctx* ctx, const uint64_t* coeffs, size_t n, size_t coeff_stride,
                            const uint64_t* zs, size_t batch, uint64_t* out_xy, int* out_is_inf, uint64_t* out_y) {
  KZGX_TRY(activate(ctx));
  if (batch == 0) return KZGX_OK;
  if (!zs || !out_xy || !out_is_inf || (n > 0 && !coeffs)) return KZGX_ERR_ARG;
  if (batch > 1 && coeff_stride != 0 && coeff_stride < n) return KZGX_ERR_ARG;
  if (ctx->c.n_srs == 0) return KZGX_ERR_NO_SRS;
  const size_t npolys = coeff_stride == 0 ? 1 : batch;
  const size_t cb = (npolys - 1) * coeff_stride * 32 + n * 32;
  const size_t ob = batch * point_words(ctx) * 4;
  // pinned layout: [results | flags | y | z | coefficients]; outputs are
  // written by the kernels into mapped host memory (no D2H copies)
  const bool direct = cb <= PIN_DIRECT_MAX;  // as kzgx_msm_g1_batch
  const size_t o_off = 0, i_off = align256(ob), y_off = i_off + align256(batch * 4),
               z_off = y_off + align256(batch * 32), c_off = z_off + align256(batch * 32);
  KZGX_TRY(pin_stage(ctx, c_off + (direct ? cb : 0)));
  std::memcpy(ctx->h_pin + z_off, zs, batch * 32);
  void* d_c = nullptr;
  if (n) {
    if (direct) {
      std::memcpy(ctx->h_pin + c_off, coeffs, cb);
      d_c = ctx->d_pin + c_off;
    } else {
      KZGX_TRY(stage(ctx, 0, cb, &d_c));
      KZGX_TRY_HIP(hipMemcpyAsync(d_c, coeffs, cb, hipMemcpyHostToDevice, ctx->c.stream));
    }
  }
  KZGX_TRY(kzgx_prove_single_batch_device(ctx, d_c, n, coeff_stride, ctx->d_pin + z_off, batch, ctx->d_pin + o_off,
                                          ctx->d_pin + i_off, ctx->d_pin + y_off, nullptr));
  KZGX_TRY_HIP(hipStreamSynchronize(ctx->c.stream));
  std::memcpy(out_xy, ctx->h_pin + o_off, ob);
  const uint32_t* inf = reinterpret_cast<const uint32_t*>(ctx->h_pin + i_off);
  for (size_t b = 0; b < batch; b++) out_is_inf[b] = (int)inf[b];
  if (out_y) std::memcpy(out_y, ctx->h_pin + y_off, batch * 32);
  return KZGX_OK;
}

int kzgx_poly_eval(kzgx_ctx* ctx, const uint64_t* coeffs, size_t n, const uint64_t* xs, size_t m, uint64_t* ys) {
  KZGX_TRY(activate(ctx));
  if (m == 0) return KZGX_OK;
  if (!xs || !ys || (n > 0 && !coeffs) || n > 0xffffffffu || m > 0xffffffffu) return KZGX_ERR_ARG;
  void *d_c = nullptr, *d_x, *d_y;
  if (n) KZGX_TRY(stage(ctx, 0, n * 32, &d_c));
  KZGX_TRY(stage(ctx, 1, m * 32, &d_x));
  KZGX_TRY(stage(ctx, 2, m * 32, &d_y));
  if (n) KZGX_TRY_HIP(hipMemcpyAsync(d_c, coeffs, n * 32, hipMemcpyHostToDevice, ctx->c.stream));
  KZGX_TRY_HIP(hipMemcpyAsync(d_x, xs, m * 32, hipMemcpyHostToDevice, ctx->c.stream));
  KZGX_TRY(kzgx::poly_eval(&ctx->c, (const uint32_t*)d_c, n, (const uint32_t*)d_x, m, (uint32_t*)d_y, ctx->c.stream));
  KZGX_TRY_HIP(hipMemcpyAsync(ys, d_y, m * 32, hipMemcpyDeviceToHost, ctx->c.stream));
  KZGX_TRY_HIP(hipStreamSynchronize(ctx->c.stream));
  return KZGX_OK;
}

int kzgx_poly_interpolate(kzgx_ctx* ctx, const uint64_t* xs, const uint64_t* ys, size_t n, uint64_t* coeffs) {
  KZGX_TRY(activate(ctx));
  if (n == 0) return KZGX_OK;
  if (!xs || !ys || !coeffs || n > (1u << 24)) return KZGX_ERR_ARG;
  void *d_x, *d_y, *d_c;
  KZGX_TRY(stage(ctx, 0, n * 32, &d_x));
  KZGX_TRY(stage(ctx, 1, n * 32, &d_y));
  KZGX_TRY(stage(ctx, 2, n * 32, &d_c));
  KZGX_TRY_HIP(hipMemcpyAsync(d_x, xs, n * 32, hipMemcpyHostToDevice, ctx->c.stream));
  KZGX_TRY_HIP(hipMemcpyAsync(d_y, ys, n * 32, hipMemcpyHostToDevice, ctx->c.stream));
  int rc = kzgx::poly_interpolate(&ctx->c, (const uint32_t*)d_x, (const uint32_t*)d_y, n, (uint32_t*)d_c,
                                  ctx->c.stream);
  if (rc != KZGX_OK) return rc;
  KZGX_TRY_HIP(hipMemcpyAsync(coeffs, d_c, n * 32, hipMemcpyDeviceToHost, ctx->c.stream));
  KZGX_TRY_HIP(hipStreamSynchronize(ctx->c.stream));
  return KZGX_OK;
}

int kzgx_poly_vanishing(kzgx_ctx* ctx, const uint64_t* xs, size_t n, uint64_t* z_out) {
  KZGX_TRY(activate(ctx));
  if (!z_out) return KZGX_ERR_ARG;
  if (n == 0) {  // empty product = 1
    std::memset(z_out, 0, 32);
    z_out[0] = 1;
    return KZGX_OK;
  }
  if (!xs || n > (1u << 24)) return KZGX_ERR_ARG;
  void *d_x, *d_z;
  KZGX_TRY(stage(ctx, 0, n * 32, &d_x));
  KZGX_TRY(stage(ctx, 1, (n + 1) * 32, &d_z));
  KZGX_TRY_HIP(hipMemcpyAsync(d_x, xs, n * 32, hipMemcpyHostToDevice, ctx->c.stream));
  KZGX_TRY(kzgx::poly_vanishing(&ctx->c, (const uint32_t*)d_x, n, (uint32_t*)d_z, ctx->c.stream));
  KZGX_TRY_HIP(hipMemcpyAsync(z_out, d_z, (n + 1) * 32, hipMemcpyDeviceToHost, ctx->c.stream));
  KZGX_TRY_HIP(hipStreamSynchronize(ctx->c.stream));
  return KZGX_OK;
}

int kzgx_g1_validate(kzgx_ctx* ctx, const uint64_t* xy, int* ok) {
  KZGX_TRY(activate(ctx));
  if (!xy || !ok) return KZGX_ERR_ARG;
  const size_t pb = point_words(ctx) * 4;
  void* d_p;
  KZGX_TRY(stage(ctx, 0, pb + 16, &d_p));
  uint32_t* d_ok = (uint32_t*)((char*)d_p + pb);
  KZGX_TRY_HIP(hipMemcpyAsync(d_p, xy, pb, hipMemcpyHostToDevice, ctx->c.stream));
  KZGX_TRY(kzgx::g1_validate(&ctx->c, (const uint32_t*)d_p, d_ok, ctx->c.stream));
  uint32_t v = 0;
  KZGX_TRY_HIP(hipMemcpyAsync(&v, d_ok, 4, hipMemcpyDeviceToHost, ctx->c.stream));
  KZGX_TRY_HIP(hipStreamSynchronize(ctx->c.stream));
  *ok = (int)v;
  return KZGX_OK;
}

int kzgx_g1_sum(kzgx_ctx* ctx, const uint64_t* xy, const int* is_inf, size_t count, uint64_t* out_xy,
                int* out_is_inf) {
  KZGX_TRY(activate(ctx));
  if (!out_xy || !out_is_inf || (count > 0 && !xy)) return KZGX_ERR_ARG;
  const size_t pb = point_words(ctx) * 4;
  void *d_p, *d_f, *d_o;
  KZGX_TRY(stage(ctx, 0, count * pb + 16, &d_p));
  KZGX_TRY(stage(ctx, 1, count * 4 + 16, &d_f));
  KZGX_TRY(stage(ctx, 2, pb + 16, &d_o));
  std::vector<uint32_t> f(count);
  for (size_t i = 0; i < count; i++) f[i] = is_inf ? (uint32_t)(is_inf[i] != 0) : 0u;
  if (count) {
    KZGX_TRY_HIP(hipMemcpyAsync(d_p, xy, count * pb, hipMemcpyHostToDevice, ctx->c.stream));
    KZGX_TRY_HIP(hipMemcpyAsync(d_f, f.data(), count * 4, hipMemcpyHostToDevice, ctx->c.stream));
  }
  uint32_t* d_oi = (uint32_t*)((char*)d_o + pb);
  KZGX_TRY(kzgx::g1_sum(&ctx->c, (const uint32_t*)d_p, (const uint32_t*)d_f, count, (uint32_t*)d_o, d_oi,
                        ctx->c.stream));
  uint32_t oi = 0;
  KZGX_TRY_HIP(hipMemcpyAsync(out_xy, d_o, pb, hipMemcpyDeviceToHost, ctx->c.stream));
  KZGX_TRY_HIP(hipMemcpyAsync(&oi, d_oi, 4, hipMemcpyDeviceToHost, ctx->c.stream));
  KZGX_TRY_HIP(hipStreamSynchronize(ctx->c.stream));
  *out_is_inf = (int)oi;
  return KZGX_OK;
}

int kzgx_g1_sum_device(kzgx_ctx* ctx, const void* d_xy, const void* d_inf, size_t count, void* d_out_xy,
                       void* d_out_inf, void* stream) {
  KZGX_TRY(activate(ctx));
  if (!d_out_xy || !d_out_inf || (count > 0 && !d_xy) || count > 0xffffffffu) return KZGX_ERR_ARG;
  return kzgx::g1_sum(&ctx->c, (const uint32_t*)d_xy, (const uint32_t*)d_inf, count, (uint32_t*)d_out_xy,
                      (uint32_t*)d_out_inf, pick(ctx, stream));
}

int kzgx_g1_sum_packed_device(kzgx_ctx* ctx, const void* d_records, size_t count, void* d_out_record, void* stream) {
  KZGX_TRY(activate(ctx));
  if (!d_out_record || (count > 0 && !d_records) || count > 0xffffffu) return KZGX_ERR_ARG;
  return kzgx::g1_fold_packed(ctx->c.curve, (const uint32_t*)d_records, count, (uint32_t*)d_out_record,
                              pick(ctx, stream));
}

int kzgx_partial_record_words(int curve) {
  if (curve != KZGX_CURVE_BN254 && curve != KZGX_CURVE_BLS12381) return -1;
  return (int)(kzgx::xyzz_record_words(curve) / 2);
}

int kzgx_msm_g1_partial_device(kzgx_ctx* ctx, const void* d_scalars, size_t n, void* d_out_record, void* stream) {
  KZGX_TRY(activate(ctx));
  if (!d_out_record || (n > 0 && !d_scalars)) return KZGX_ERR_ARG;
  if (ctx->c.n_srs == 0) return KZGX_ERR_NO_SRS;
  if (n > ctx->c.n_srs) return KZGX_ERR_DEGREE;
  hipStream_t st = pick(ctx, stream);
  if (n == 0) {  // the identity: ZZ = 0
    KZGX_TRY_HIP(hipMemsetAsync(d_out_record, 0, kzgx::xyzz_record_words(ctx->c.curve) * 4, st));
    return KZGX_OK;
  }
  return kzgx::msm_partial_xyzz(&ctx->c, (const uint32_t*)d_scalars, n, (uint32_t*)d_out_record, st);
}

int kzgx_g1_sum_partials_device(kzgx_ctx* ctx, const void* d_records, size_t count, void* d_out_record, void* stream) {
  KZGX_TRY(activate(ctx));
  if (!d_out_record || (count > 0 && !d_records) || count > 0xffffffu) return KZGX_ERR_ARG;
  return kzgx::g1_fold_xyzz(ctx->c.curve, (const uint32_t*)d_records, count, (uint32_t*)d_out_record,
                            pick(ctx, stream));
}

int kzgx_msm_g1_sharded(kzgx_ctx* const* ctxs, const size_t* starts, size_t nctx, const uint64_t* scalars,
                        size_t n, uint64_t* out_xy, int* out_is_inf) {
  if (!ctxs || !starts || nctx == 0 || (n > 0 && !scalars) || !out_xy || !out_is_inf) return KZGX_ERR_ARG;
  std::vector<size_t> cnt(nctx, 0);
  for (size_t k = 0; k < nctx; k++) {
    kzgx_ctx* c = ctxs[k];
    if (!c || c->c.curve != ctxs[0]->c.curve) return KZGX_ERR_ARG;
    for (size_t j = 0; j < k; j++)
      if (ctxs[j] == c) return KZGX_ERR_ARG;  // shards share per-context staging: one slice per context
    if (c->c.n_srs == 0) return KZGX_ERR_NO_SRS;
    if (starts[k] != (k == 0 ? 0 : starts[k - 1] + ctxs[k - 1]->c.n_srs)) return KZGX_ERR_ARG;  // contiguous
    cnt[k] = starts[k] >= n ? 0 : std::min(n - starts[k], c->c.n_srs);
  }
  if (starts[nctx - 1] + ctxs[nctx - 1]->c.n_srs < n) return KZGX_ERR_DEGREE;
  const size_t pb = point_words(ctxs[0]) * 4;
  // projective partial records (round 6): no shard converts its partial to
  // affine; the fold's one inversion is the step's only one
  const size_t rb = kzgx::xyzz_record_words(ctxs[0]->c.curve) * 4;
  kzgx_ctx* c0 = ctxs[0];
  // the fold's inputs live on ctxs[0]'s device: nctx partial records
  // (all-zero = infinity: empty shards contribute nothing)
  void *d_gather, *d_res;
  KZGX_TRY(activate(c0));
  KZGX_TRY(stage(c0, 2, nctx * rb + 16, &d_gather));
  KZGX_TRY(stage(c0, 3, pb + 16, &d_res));
  KZGX_TRY_HIP(hipMemsetAsync(d_gather, 0, nctx * rb, c0->c.stream));
  hipEvent_t zeroed;
  KZGX_TRY_HIP(hipEventCreateWithFlags(&zeroed, hipEventDisableTiming));
  std::vector<hipEvent_t> done;
  struct EvGuard {
    std::vector<hipEvent_t>* v;
    hipEvent_t z;
    ~EvGuard() {
      for (auto e : *v) (void)hipEventDestroy(e);
      (void)hipEventDestroy(z);
    }
  } evg{&done, zeroed};
  KZGX_TRY_HIP(hipEventRecord(zeroed, c0->c.stream));
  // every shard's partial MSM on its own context's stream, then a
  // device-to-device (peer) copy of the partial point to ctxs[0]: no host
  // round trip between the partial MSMs and the fold
  for (size_t k = 0; k < nctx; k++) {
    if (!cnt[k]) continue;
    kzgx_ctx* c = ctxs[k];
    KZGX_TRY(activate(c));
    void *d_s, *d_o;
    KZGX_TRY(stage(c, 0, cnt[k] * 32, &d_s));
    KZGX_TRY(stage(c, 1, rb + 16, &d_o));
    KZGX_TRY_HIP(hipMemcpyAsync(d_s, scalars + starts[k] * 4, cnt[k] * 32, hipMemcpyHostToDevice, c->c.stream));
    KZGX_TRY(kzgx::msm_partial_xyzz(&c->c, (const uint32_t*)d_s, cnt[k], (uint32_t*)d_o, c->c.stream));
    KZGX_TRY_HIP(hipStreamWaitEvent(c->c.stream, zeroed, 0));
    KZGX_TRY_HIP(hipMemcpyPeerAsync((char*)d_gather + k * rb, c0->c.device, d_o, c->c.device, rb, c->c.stream));
    hipEvent_t e;
    KZGX_TRY_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    done.push_back(e);
    KZGX_TRY_HIP(hipEventRecord(e, c->c.stream));
  }
  KZGX_TRY(activate(c0));
  for (auto e : done) KZGX_TRY_HIP(hipStreamWaitEvent(c0->c.stream, e, 0));
  uint32_t* d_oi = (uint32_t*)((char*)d_res + pb);  // the packed record's infinity word
  KZGX_TRY(kzgx::g1_fold_xyzz(c0->c.curve, (const uint32_t*)d_gather, nctx, (uint32_t*)d_res, c0->c.stream));
  uint32_t oi = 0;
  KZGX_TRY_HIP(hipMemcpyAsync(out_xy, d_res, pb, hipMemcpyDeviceToHost, c0->c.stream));
  KZGX_TRY_HIP(hipMemcpyAsync(&oi, d_oi, 4, hipMemcpyDeviceToHost, c0->c.stream));
  KZGX_TRY_HIP(hipStreamSynchronize(c0->c.stream));
  *out_is_inf = (int)oi;
  return KZGX_OK;
}

/* ---- verify half: G2 SRS, polyeval_G2, pairing, verify_proof ---------------- */
namespace {
// the G2 SRS's windowed table for n points (rebuilt when the SRS changed or
// more points are needed); nullptr (plain per-term path) if it cannot be had
const uint32_t* g2_table(kzgx_ctx* ctx, size_t n, hipStream_t st) {
  if (ctx->g2tab_n >= n) return ctx->d_g2tab;
  const size_t all = ctx->n_srs2;
  ctx->g2tab_n = 0;
  if (kzgx::dev_alloc(&ctx->c, (void**)&ctx->d_g2tab, kzgx::g2_table_bytes(ctx->c.curve, all), &ctx->g2tab_b) !=
          KZGX_OK ||
      kzgx::g2_table_build(&ctx->c, ctx->d_srs2_canon, all, ctx->d_g2tab, st) != KZGX_OK ||
      hipStreamSynchronize(st) != hipSuccess)
    return nullptr;
  ctx->g2tab_n = all;
  return ctx->d_g2tab;
}

// the wave verify's setup-derived buffer ([y]G table, the line tables of
// G2[0] and G2[1]), built on first use after a setup
int vw_ensure(kzgx_ctx* ctx, hipStream_t st) {
  if (ctx->vw_ready) return KZGX_OK;
  KZGX_TRY(kzgx::dev_alloc(&ctx->c, (void**)&ctx->d_vw, kzgx::verify_wave_bytes(ctx->c.curve), &ctx->vw_b));
  kzgx::GenTables g;
  KZGX_TRY(kzgx::gen_tables_get(ctx->c.curve, ctx->c.device, st, &g));
  KZGX_TRY(kzgx::verify_wave_prepare(&ctx->c, ctx->d_srs_canon, ctx->d_srs2_canon, g.g1_comb, ctx->d_vw, st));
  KZGX_TRY_HIP(hipStreamSynchronize(st));  // one-time; later calls may come on other streams
  ctx->vw_ready = true;
  return KZGX_OK;
}

int side_ready(kzgx_ctx* ctx) {
  if (!ctx->side) KZGX_TRY_HIP(stream_take(ctx->c.device, &ctx->side));
  if (!ctx->ev_fork) KZGX_TRY_HIP(hipEventCreateWithFlags(&ctx->ev_fork, hipEventDisableTiming));
  if (!ctx->ev_join) KZGX_TRY_HIP(hipEventCreateWithFlags(&ctx->ev_join, hipEventDisableTiming));
  return KZGX_OK;
}

// KZGX_PAIR2_SPLIT=1: the multi-point verify's pairing as round 6's two
// launches (k_vlines_wave, then k_pair2_wave) instead of k_pair2_fused (A/B)
bool split_pair2() {
  static const bool on = std::getenv("KZGX_PAIR2_SPLIT") && std::getenv("KZGX_PAIR2_SPLIT")[0] == '1';
  return on;
}

}  // namespace

size_t kzgx_srs_g2_size(const kzgx_ctx* ctx) { return ctx ? ctx->n_srs2 : 0; }

int kzgx_gen_srs_g2(kzgx_ctx* ctx, const uint64_t* tau, size_t start, size_t n) {
  KZGX_TRY(activate(ctx));
  ctx->vw_ready = false;
  ctx->g2tab_n = 0;
  if (!tau || n == 0 || n > 0x7fffffffu) return KZGX_ERR_ARG;
  const size_t bytes = n * 2 * point_words(ctx) * 4;
  KZGX_TRY(kzgx::dev_alloc(&ctx->c, (void**)&ctx->d_srs2_canon, bytes, &ctx->srs2_canon_b));
  void* d_tau;
  KZGX_TRY(stage(ctx, 0, 32, &d_tau));
  KZGX_TRY_HIP(hipMemcpyAsync(d_tau, tau, 32, hipMemcpyHostToDevice, ctx->c.stream));
  kzgx::GenTables g;
  KZGX_TRY(kzgx::gen_tables_get(ctx->c.curve, ctx->c.device, ctx->c.stream, &g));
  KZGX_TRY(kzgx::gen_srs_g2_comb(ctx->c.curve, (const uint32_t*)d_tau, start, n, g.g2_comb, ctx->d_srs2_canon,
                                 ctx->c.stream));
  // polyeval_G2's window table from the same comb (one comb evaluation per
  // entry, ~1 ms at 4097 points) so no verify_proof(poly, 0, N) pays the
  // 4.3-ms doubling chains of building it from the points (k_g2_tab, still
  // the path of a loaded G2 SRS); large SRSs keep it for first use
  const bool eager = n <= KZGX_G2TAB_EAGER_MAX;
  if (eager) {
    KZGX_TRY(kzgx::dev_alloc(&ctx->c, (void**)&ctx->d_g2tab, kzgx::g2_table_bytes(ctx->c.curve, n), &ctx->g2tab_b));
    KZGX_TRY(kzgx::g2_table_comb(ctx->c.curve, (const uint32_t*)d_tau, start, n, g.g2_comb, ctx->d_g2tab,
                                 ctx->c.stream));
  }
  KZGX_TRY_HIP(hipStreamSynchronize(ctx->c.stream));
  ctx->g2tab_n = eager ? n : 0;
  ctx->n_srs2 = n;
  return setup_finish(ctx);
}

int kzgx_load_srs_g2(kzgx_ctx* ctx, const uint64_t* xy, size_t n) {
  KZGX_TRY(activate(ctx));
  ctx->vw_ready = false;
  ctx->g2tab_n = 0;
  if (!xy || n == 0) return KZGX_ERR_ARG;
  const size_t bytes = n * 2 * point_words(ctx) * 4;
  KZGX_TRY(kzgx::dev_alloc(&ctx->c, (void**)&ctx->d_srs2_canon, bytes, &ctx->srs2_canon_b));
  KZGX_TRY_HIP(hipMemcpyAsync(ctx->d_srs2_canon, xy, bytes, hipMemcpyHostToDevice, ctx->c.stream));
  KZGX_TRY_HIP(hipStreamSynchronize(ctx->c.stream));
  ctx->n_srs2 = n;
  return setup_finish(ctx);
}

int kzgx_get_srs_g2(kzgx_ctx* ctx, uint64_t* xy, size_t n) {
  KZGX_TRY(activate(ctx));
  if (!xy) return KZGX_ERR_ARG;
  if (ctx->n_srs2 == 0) return KZGX_ERR_NO_SRS;
  if (n > ctx->n_srs2) return KZGX_ERR_ARG;
  KZGX_TRY_HIP(
      hipMemcpyAsync(xy, ctx->d_srs2_canon, n * 2 * point_words(ctx) * 4, hipMemcpyDeviceToHost, ctx->c.stream));
  KZGX_TRY_HIP(hipStreamSynchronize(ctx->c.stream));
  return KZGX_OK;
}

int kzgx_g2_validate(kzgx_ctx* ctx, const uint64_t* xy, size_t count, int* ok) {
  KZGX_TRY(activate(ctx));
  if (count == 0) return KZGX_OK;
  if (!xy || !ok) return KZGX_ERR_ARG;
  const size_t pb = 2 * point_words(ctx) * 4;
  void *d_p, *d_ok;
  KZGX_TRY(stage(ctx, 0, count * pb, &d_p));
  KZGX_TRY(stage(ctx, 1, count * 4, &d_ok));
  KZGX_TRY_HIP(hipMemcpyAsync(d_p, xy, count * pb, hipMemcpyHostToDevice, ctx->c.stream));
  KZGX_TRY(kzgx::g2_validate(&ctx->c, (const uint32_t*)d_p, count, (uint32_t*)d_ok, ctx->c.stream));
  std::vector<uint32_t> v(count);
  KZGX_TRY_HIP(hipMemcpyAsync(v.data(), d_ok, count * 4, hipMemcpyDeviceToHost, ctx->c.stream));
  KZGX_TRY_HIP(hipStreamSynchronize(ctx->c.stream));
  for (size_t k = 0; k < count; k++) ok[k] = (int)v[k];
  return KZGX_OK;
}

int kzgx_msm_g2(kzgx_ctx* ctx, const uint64_t* scalars, size_t n, uint64_t* out_xy, int* out_is_inf) {
  KZGX_TRY(activate(ctx));
  if (!out_xy || !out_is_inf || (n > 0 && !scalars) || n > (1u << 24)) return KZGX_ERR_ARG;
  if (ctx->n_srs2 == 0) return KZGX_ERR_NO_SRS;
  if (n > ctx->n_srs2) return KZGX_ERR_DEGREE;
  const size_t pb = 2 * point_words(ctx) * 4;
  void *d_s = nullptr, *d_o;
  if (n) KZGX_TRY(stage(ctx, 0, n * 32, &d_s));
  KZGX_TRY(stage(ctx, 1, pb + 16, &d_o));
  if (n) KZGX_TRY_HIP(hipMemcpyAsync(d_s, scalars, n * 32, hipMemcpyHostToDevice, ctx->c.stream));
  uint32_t* d_oi = (uint32_t*)((char*)d_o + pb);
  KZGX_TRY(kzgx::msm_g2(&ctx->c, (const uint32_t*)d_s, ctx->d_srs2_canon, n, (uint32_t*)d_o, d_oi, ctx->c.stream,
                        n ? g2_table(ctx, n, ctx->c.stream) : nullptr));
  uint32_t oi = 0;
  KZGX_TRY_HIP(hipMemcpyAsync(out_xy, d_o, pb, hipMemcpyDeviceToHost, ctx->c.stream));
  KZGX_TRY_HIP(hipMemcpyAsync(&oi, d_oi, 4, hipMemcpyDeviceToHost, ctx->c.stream));
  KZGX_TRY_HIP(hipStreamSynchronize(ctx->c.stream));
  *out_is_inf = (int)oi;
  return KZGX_OK;
}

int kzgx_pairing(kzgx_ctx* ctx, const uint64_t* g1_xy, const int* g1_inf, const uint64_t* g2_xy, const int* g2_inf,
                 size_t count, uint64_t* out) {
  KZGX_TRY(activate(ctx));
  if (count == 0) return KZGX_OK;
  if (!g1_xy || !g2_xy || !out || count > (1u << 20)) return KZGX_ERR_ARG;
  const size_t p1 = point_words(ctx) * 4, p2 = 2 * p1, fb = 6 * p1;
  void *d_1, *d_2, *d_f, *d_o;
  KZGX_TRY(stage(ctx, 0, count * p1, &d_1));
  KZGX_TRY(stage(ctx, 1, count * p2, &d_2));
  KZGX_TRY(stage(ctx, 2, count * 8, &d_f));
  KZGX_TRY(stage(ctx, 3, count * fb, &d_o));
  std::vector<uint32_t> f(2 * count);
  for (size_t k = 0; k < count; k++) {
    f[k] = g1_inf ? (uint32_t)(g1_inf[k] != 0) : 0u;
    f[count + k] = g2_inf ? (uint32_t)(g2_inf[k] != 0) : 0u;
  }
  KZGX_TRY_HIP(hipMemcpyAsync(d_1, g1_xy, count * p1, hipMemcpyHostToDevice, ctx->c.stream));
  KZGX_TRY_HIP(hipMemcpyAsync(d_2, g2_xy, count * p2, hipMemcpyHostToDevice, ctx->c.stream));
  KZGX_TRY_HIP(hipMemcpyAsync(d_f, f.data(), count * 8, hipMemcpyHostToDevice, ctx->c.stream));
  KZGX_TRY(kzgx::pairing_batch(&ctx->c, (const uint32_t*)d_1, (const uint32_t*)d_f, (const uint32_t*)d_2,
                               (const uint32_t*)d_f + count, count, (uint32_t*)d_o, ctx->c.stream));
  KZGX_TRY_HIP(hipMemcpyAsync(out, d_o, count * fb, hipMemcpyDeviceToHost, ctx->c.stream));
  KZGX_TRY_HIP(hipStreamSynchronize(ctx->c.stream));
  return KZGX_OK;
}

int kzgx_verify_proof(kzgx_ctx* ctx, const uint64_t* commit_xy, int commit_inf, const uint64_t* proof_xy,
                      int proof_inf, const uint64_t* xs, const uint64_t* ys, size_t npoints, int* ok) {
  KZGX_TRY(activate(ctx));
  if (!commit_xy || !proof_xy || !ok || (npoints > 0 && (!xs || !ys)) || npoints > (1u << 24)) return KZGX_ERR_ARG;
  if (npoints < 1) return KZGX_ERR_ARG;  // "expected_data size must be 1 or greater"
  if (ctx->c.n_srs == 0) return KZGX_ERR_NO_SRS;
  *ok = 0;
  if (npoints >= ctx->c.n_srs) return KZGX_OK;  // trusted_setup.cpp:235-236
  if (ctx->n_srs2 < npoints + 1) return KZGX_ERR_NO_SRS;
  if (npoints == 1) {  // I = y, Z = X - x: the single-opening product check
    const int cf = commit_inf != 0, pf = proof_inf != 0;
    return kzgx_verify_single_batch(ctx, commit_xy, &cf, proof_xy, &pf, xs, ys, 1, ok);
  }
  hipStream_t st = ctx->c.stream;
  const size_t n = npoints;
  const size_t p1 = point_words(ctx) * 4, p2 = 2 * p1, fb = 6 * p1;
  // one device block: x | y | I | Z | G1 in (commit, proof) | G1 work | G2 in | flags | Fp12 out
  const size_t o_x = 0, o_y = o_x + n * 32, o_I = o_y + n * 32, o_Z = o_I + n * 32, o_g1 = o_Z + (n + 1) * 32;
  const size_t o_w = o_g1 + 4 * p1, o_g2 = o_w + 2 * p1, o_f = o_g2 + 2 * p2, o_o = o_f + 64;
  const size_t o_ln = (o_o + 2 * fb + 255) & ~(size_t)255;
  void* d;
  KZGX_TRY(stage(ctx, 3, o_ln + kzgx::pair2_wave_scratch_bytes(ctx->c.curve), &d));
  char* b = (char*)d;
  uint32_t* g1 = (uint32_t*)(b + o_g1);  // [proof, p2, commit, msm(I)]
  uint32_t* fl = (uint32_t*)(b + o_f);   // [proof_inf, p2_inf, p1_inf, srs2_0_inf, commit_inf, msmI_inf]
  uint32_t hf[8] = {(uint32_t)(proof_inf != 0), 0, 0, 0, (uint32_t)(commit_inf != 0), 0, 0, 0};
  KZGX_TRY_HIP(hipMemcpyAsync(b + o_x, xs, n * 32, hipMemcpyHostToDevice, st));
  KZGX_TRY_HIP(hipMemcpyAsync(b + o_y, ys, n * 32, hipMemcpyHostToDevice, st));
  KZGX_TRY_HIP(hipMemcpyAsync(g1, proof_xy, p1, hipMemcpyHostToDevice, st));
  KZGX_TRY_HIP(hipMemcpyAsync((char*)g1 + 2 * p1, commit_xy, p1, hipMemcpyHostToDevice, st));
  KZGX_TRY_HIP(hipMemcpyAsync(fl, hf, sizeof(hf), hipMemcpyHostToDevice, st));
  // Z and I (linear_roots_and_polyfit, util.cpp:172-178): Z first, then the
  // G2 half (p1 = [Z(tau)]G2, ~0.9 ms of lone-lane G2 chains) forks onto the
  // side stream while this stream takes the G1 half (I, [I(tau)]G1, C - it)
  KZGX_TRY(kzgx::poly_vanishing(&ctx->c, (const uint32_t*)(b + o_x), n, (uint32_t*)(b + o_Z), st));
  KZGX_TRY(side_ready(ctx));
  hipStream_t sd = ctx->side;
  KZGX_TRY_HIP(hipEventRecord(ctx->ev_fork, st));
  KZGX_TRY_HIP(hipStreamWaitEvent(sd, ctx->ev_fork, 0));
  uint32_t* g2 = (uint32_t*)(b + o_g2);
  const int rg2 =
      kzgx::msm_g2(&ctx->c, (const uint32_t*)(b + o_Z), ctx->d_srs2_canon, n + 1, g2, fl + 2, sd, g2_table(ctx, n + 1, sd));
  // (joined before any return below: the side work writes into this call's staging)
  const hipError_t jr = hipEventRecord(ctx->ev_join, sd);
  auto join = [&]() { return hipStreamWaitEvent(st, ctx->ev_join, 0); };
  if (rg2 != KZGX_OK || jr != hipSuccess) {
    (void)hipStreamSynchronize(sd);
    return rg2 != KZGX_OK ? rg2 : kzgx::hip_fail(jr);
  }
  int rg1 = kzgx::poly_interpolate(&ctx->c, (const uint32_t*)(b + o_x), (const uint32_t*)(b + o_y), n,
                                   (uint32_t*)(b + o_I), st);
  // p2 = C - [I(tau)]G1
  if (rg1 == KZGX_OK)
    rg1 = kzgx::msm_batch(&ctx->c, (const uint32_t*)(b + o_I), n, 1, n * 8, (uint32_t*)((char*)g1 + 3 * p1), fl + 5, st);
  if (rg1 == KZGX_OK)
    rg1 = kzgx::g1_sub(&ctx->c, (const uint32_t*)((char*)g1 + 2 * p1), fl + 4, (const uint32_t*)((char*)g1 + 3 * p1),
                       fl + 5, (uint32_t*)((char*)g1 + p1), fl + 1, st);
  KZGX_TRY_HIP(join());
  if (rg1 != KZGX_OK) {
    (void)hipStreamSynchronize(st);
    return rg1;
  }
  // the second pairing's G2 input = G2[0] (the two-launch path reads it here)
  KZGX_TRY_HIP(hipMemcpyAsync((char*)g2 + p2, ctx->d_srs2_canon, p2, hipMemcpyDeviceToDevice, st));
  // e(proof, p1) == e(p2, G2[0])  <=>  e(proof, p1) e(-p2, G2[0]) == 1 (one wave, one final
  // exponentiation; the booleans of the reference's FP12_equals)
  uint32_t* d_ok = (uint32_t*)(b + o_o);
  uint32_t v = 2;
  if (!split_pair2()) {  // one launch: [Z(tau)]G2's lines overlap the Miller loop
    KZGX_TRY(vw_ensure(ctx, st));
    KZGX_TRY(kzgx::pair2_fused(&ctx->c, g1, fl, g2, fl + 2, ctx->d_vw, d_ok, st));
    KZGX_TRY_HIP(hipMemcpyAsync(&v, d_ok, 4, hipMemcpyDeviceToHost, st));
    KZGX_TRY_HIP(hipStreamSynchronize(st));
  }
  if (v == 2) {  // (a degenerate line chain, or KZGX_PAIR2_SPLIT): two launches
    KZGX_TRY(kzgx::pair2_wave(&ctx->c, g1, fl, g2, fl + 2, (uint32_t*)(b + o_ln), d_ok, st));
    KZGX_TRY_HIP(hipMemcpyAsync(&v, d_ok, 4, hipMemcpyDeviceToHost, st));
    KZGX_TRY_HIP(hipStreamSynchronize(st));
  }
  *ok = v ? 1 : 0;
  return KZGX_OK;
}

int kzgx_verify_single_batch_device(kzgx_ctx* ctx, const void* d_commits, const void* d_commit_inf,
                                    const void* d_proofs, const void* d_proof_inf, const void* d_z, const void* d_y,
                                    size_t count, void* d_ok, void* stream) {
  KZGX_TRY(activate(ctx));
  if (count == 0) return KZGX_OK;
  if (!d_commits || !d_proofs || !d_z || !d_y || !d_ok || count > (1u << 26)) return KZGX_ERR_ARG;
  if (ctx->c.n_srs == 0 || ctx->n_srs2 < 2) return KZGX_ERR_NO_SRS;
  hipStream_t st = pick(ctx, stream);
  if (count <= ctx->vw_max) {
    KZGX_TRY(vw_ensure(ctx, st));
    return kzgx::verify_wave_batch(&ctx->c, (const uint32_t*)d_commits, (const uint32_t*)d_commit_inf,
                                   (const uint32_t*)d_proofs, (const uint32_t*)d_proof_inf, (const uint32_t*)d_z,
                                   (const uint32_t*)d_y, count, ctx->d_srs_canon, ctx->d_vw, (uint32_t*)d_ok, st);
  }
  return kzgx::verify_single_batch(&ctx->c, (const uint32_t*)d_commits, (const uint32_t*)d_commit_inf,
                                   (const uint32_t*)d_proofs, (const uint32_t*)d_proof_inf, (const uint32_t*)d_z,
                                   (const uint32_t*)d_y, count, ctx->d_srs_canon, ctx->d_srs2_canon,
                                   (uint32_t*)d_ok, st);
}

int kzgx_set_verify_wave_max(kzgx_ctx* ctx, size_t max_count) {
  if (!ctx) return KZGX_ERR_ARG;
  ctx->vw_max = max_count;
  return KZGX_OK;
}

int kzgx_verify_single_batch(kzgx_ctx* ctx, const uint64_t* commits_xy, const int* commit_inf,
                             const uint64_t* proofs_xy, const int* proof_inf, const uint64_t* zs, const uint64_t* ys,
                             size_t count, int* ok) {
  KZGX_TRY(activate(ctx));
  if (count == 0) return KZGX_OK;
  if (!commits_xy || !proofs_xy || !zs || !ys || !ok || count > (1u << 26)) return KZGX_ERR_ARG;
  const size_t pb = point_words(ctx) * 4;
  if (count <= ctx->vw_max && count * (2 * pb + 76) <= PIN_DIRECT_MAX) {
    // the wave path (single verify_proof calls): inputs and the result in
    // the context's mapped pinned staging -- the kernel copies each opening's
    // inputs into LDS in one round trip and writes its boolean straight into
    // host memory, so the call makes no copy at all (it made five H2D and
    // one D2H copies from pageable memory, ~10 us each)
    const size_t o_ok = 0, o_c = align256(count * 4), o_p = o_c + align256(count * pb);
    const size_t o_z = o_p + align256(count * pb), o_y = o_z + count * 32, o_f = align256(o_y + count * 32);
    KZGX_TRY(pin_stage(ctx, o_f + count * 8));
    uint8_t* h = ctx->h_pin;
    std::memcpy(h + o_c, commits_xy, count * pb);
    std::memcpy(h + o_p, proofs_xy, count * pb);
    std::memcpy(h + o_z, zs, count * 32);
    std::memcpy(h + o_y, ys, count * 32);
    uint32_t* hf = reinterpret_cast<uint32_t*>(h + o_f);
    for (size_t k = 0; k < count; k++) {
      hf[k] = commit_inf ? (uint32_t)(commit_inf[k] != 0) : 0u;
      hf[count + k] = proof_inf ? (uint32_t)(proof_inf[k] != 0) : 0u;
    }
    uint8_t* d = ctx->d_pin;
    KZGX_TRY(kzgx_verify_single_batch_device(ctx, d + o_c, d + o_f, d + o_p, d + o_f + count * 4, d + o_z, d + o_y,
                                             count, d + o_ok, nullptr));
    KZGX_TRY_HIP(hipStreamSynchronize(ctx->c.stream));
    const uint32_t* v = reinterpret_cast<const uint32_t*>(h + o_ok);
    for (size_t k = 0; k < count; k++) ok[k] = (int)v[k];
    return KZGX_OK;
  }
  void *d_c, *d_p, *d_s, *d_f;
  KZGX_TRY(stage(ctx, 0, count * pb, &d_c));
  KZGX_TRY(stage(ctx, 1, count * pb, &d_p));
  KZGX_TRY(stage(ctx, 2, count * 64, &d_s));
  KZGX_TRY(stage(ctx, 3, count * 12, &d_f));
  std::vector<uint32_t> fl(2 * count);
  for (size_t k = 0; k < count; k++) {
    fl[k] = commit_inf ? (uint32_t)(commit_inf[k] != 0) : 0u;
    fl[count + k] = proof_inf ? (uint32_t)(proof_inf[k] != 0) : 0u;
  }
  hipStream_t st = ctx->c.stream;
  KZGX_TRY_HIP(hipMemcpyAsync(d_c, commits_xy, count * pb, hipMemcpyHostToDevice, st));
  KZGX_TRY_HIP(hipMemcpyAsync(d_p, proofs_xy, count * pb, hipMemcpyHostToDevice, st));
  KZGX_TRY_HIP(hipMemcpyAsync(d_s, zs, count * 32, hipMemcpyHostToDevice, st));
  KZGX_TRY_HIP(hipMemcpyAsync((char*)d_s + count * 32, ys, count * 32, hipMemcpyHostToDevice, st));
  KZGX_TRY_HIP(hipMemcpyAsync(d_f, fl.data(), count * 8, hipMemcpyHostToDevice, st));
  uint32_t* d_ok = (uint32_t*)d_f + 2 * count;
  KZGX_TRY(kzgx_verify_single_batch_device(ctx, d_c, d_f, d_p, (uint32_t*)d_f + count, d_s,
                                           (char*)d_s + count * 32, count, d_ok, nullptr));
  std::vector<uint32_t> v(count);
  KZGX_TRY_HIP(hipMemcpyAsync(v.data(), d_ok, count * 4, hipMemcpyDeviceToHost, st));
  KZGX_TRY_HIP(hipStreamSynchronize(st));
  for (size_t k = 0; k < count; k++) ok[k] = (int)v[k];
  return KZGX_OK;
}

}  // extern "C"

namespace {
// Once both SRS halves are present (the end of trusted_setup(int) or of a
// setup-file load): the verify tables (kzgx_verify_proof's [y]G table and the
// line tables of G2[0], G2[1]) and the call workspaces are made here, so the
// first commit / proof / verify on a new setup pays no allocation or table
// build (the reference's benchmark times each first call,
// benchmark/benchmark.cpp:40-66).  KZGX_LAZY_SETUP=1 leaves them to first use.
int setup_finish(kzgx_ctx* ctx) {
  static const bool lazy = std::getenv("KZGX_LAZY_SETUP") && std::getenv("KZGX_LAZY_SETUP")[0] == '1';
  if (lazy || ctx->c.n_srs == 0 || ctx->n_srs2 < 2) return KZGX_OK;
  hipStream_t st = ctx->c.stream;
  kzgx::GenTables g;
  KZGX_TRY(kzgx::gen_tables_get(ctx->c.curve, ctx->c.device, st, &g));
  KZGX_TRY(kzgx::dev_alloc(&ctx->c, (void**)&ctx->d_vw, kzgx::verify_wave_bytes(ctx->c.curve), &ctx->vw_b));
  KZGX_TRY(kzgx::verify_wave_prepare(&ctx->c, ctx->d_srs_canon, ctx->d_srs2_canon, g.g1_comb, ctx->d_vw, st));
  // staging of the host-pointer calls, sized for degree-4096 single calls
  KZGX_TRY(pin_stage(ctx, (size_t)1 << 20));
  void* d;
  for (int s = 0; s < 4; s++) KZGX_TRY(stage(ctx, s, (size_t)256 << 10, &d));
  KZGX_TRY_HIP(hipStreamSynchronize(st));
  ctx->vw_ready = true;
  // the multi-point verify's workspaces at the reference benchmark's largest
  // opening count (4096 points, benchmark/benchmark.cpp:85-99)
  {
    const size_t nv = std::min<size_t>(ctx->n_srs2 - 1, 4096);
    const size_t p1 = point_words(ctx) * 4, fb = 6 * p1;
    const size_t o_o = 3 * nv * 32 + (nv + 1) * 32 + 6 * p1 + 4 * 2 * p1 + 64;
    KZGX_TRY(stage(ctx, 3, ((o_o + 2 * fb + 255) & ~(size_t)255) + kzgx::pair2_wave_scratch_bytes(ctx->c.curve), &d));
    KZGX_TRY(kzgx::verify_ws_reserve(&ctx->c, nv));
  }
  // the single-call workspaces (quotient, latency partials, arrival
  // counters, Pippenger buffers): one zero proof at the largest default
  // degree and one at degree 128 size them
  const size_t nmax = std::min<size_t>(ctx->c.n_srs, 4097);
  std::vector<uint64_t> zc(4 * nmax, 0), zz(4, 0), xy(2 * point_words(ctx), 0), y(4, 0);
  int inf = 0;
  for (size_t n : {nmax, std::min<size_t>(nmax, 129)}) {
    KZGX_TRY(kzgx_prove_single_batch(ctx, zc.data(), n, 0, zz.data(), 1, xy.data(), &inf, y.data()));
    KZGX_TRY(kzgx_msm_g1(ctx, zc.data(), n, xy.data(), &inf));
  }
  return KZGX_OK;
}
}  // namespace

// Debug only (not part of include/kzg_gpu.h): copy a Pippenger workspace
// buffer of the context's default stream to the host, after a device sync.
// Looks the workspace up without binding or refreshing one.
extern "C" int kzgx_debug_ws_read(kzgx_ctx* ctx, const char* name, void* host, size_t bytes) {
  KZGX_TRY(activate(ctx));
  kzgx::MsmWs* w = ctx->c.ws_find(ctx->c.stream);
  if (!w || !name || !host) return KZGX_ERR_ARG;
  const void* src = nullptr;
  size_t cap = 0;
  const std::string s(name);
  if (s == "offsets") src = w->offsets, cap = w->offsets_b;
  else if (s == "entries") src = w->entries, cap = w->entries_b;
  else if (s == "bsum") src = w->bsum, cap = w->bsum_b;
  else if (s == "sstate") src = w->sstate, cap = w->sstate_b;
  else if (s == "tailk") src = w->tailk, cap = w->tailk_b;
  else if (s == "heads") src = w->heads, cap = w->heads_b;
  else if (s == "tails") src = w->tails, cap = w->tails_b;
  else if (s == "counts") src = w->counts, cap = w->counts_b;
  else if (s == "cursors") src = w->cursors, cap = w->cursors_b;
  else if (s == "gmeta") src = w->gmeta, cap = w->gmeta_b;
  else if (s == "gpart") src = w->gpart, cap = w->gpart_b;
  else if (s == "q") src = w->q, cap = w->q_b;
  if (!src || bytes > cap) return KZGX_ERR_ARG;
  KZGX_TRY_HIP(hipDeviceSynchronize());
  KZGX_TRY_HIP(hipMemcpy(host, src, bytes, hipMemcpyDeviceToHost));
  return KZGX_OK;
}

// debug: single-lane dependent-chain latency of one primitive (msm_fixed.hip
// k_debug_latency); res[0] = ns per operation, res[1] = core clocks
extern "C" int kzgx_debug_latency(kzgx_ctx* ctx, int op, unsigned iters, double* res) {
  KZGX_TRY(activate(ctx));
  if (!res) return KZGX_ERR_ARG;
  KZGX_TRY_HIP(hipStreamSynchronize(ctx->c.stream));
  return kzgx::debug_latency(&ctx->c, op, iters, res);
}

// debug: latency of one wave-wide Fp12 op of the verify path
// (verify_wave.hip k_vw_bench): res[0] = ns per op, res[1] = core clocks
namespace kzgx {
int coop_selftest(int curve, const uint32_t* d_tab, uint32_t n_pts, uint32_t* d_bad, hipStream_t st);  // latency.hip
}
// coop.hpp's cooperative point operations against the lone-lane forms on the
// loaded SRS (window 0 of the Pippenger table); *bad = bit mask of failing cases
extern "C" int kzgx_debug_coop_test(kzgx_ctx* ctx, unsigned* bad) {
  KZGX_TRY(activate(ctx));
  if (!bad || ctx->c.n_srs < 3) return KZGX_ERR_ARG;
  uint32_t* d_bad = nullptr;
  KZGX_TRY_HIP(hipMalloc((void**)&d_bad, 4));
  int rc = hipMemsetAsync(d_bad, 0, 4, ctx->c.stream) == hipSuccess ? KZGX_OK : KZGX_ERR_HIP;
  if (rc == KZGX_OK)
    rc = kzgx::coop_selftest(ctx->c.curve, ctx->c.d_table, (uint32_t)(ctx->c.n_srs < 3 * 4096 ? ctx->c.n_srs : 3 * 4096),
                             d_bad, ctx->c.stream);
  if (rc == KZGX_OK && hipMemcpyAsync(bad, d_bad, 4, hipMemcpyDeviceToHost, ctx->c.stream) != hipSuccess) rc = KZGX_ERR_HIP;
  if (rc == KZGX_OK && hipStreamSynchronize(ctx->c.stream) != hipSuccess) rc = KZGX_ERR_HIP;
  (void)hipFree(d_bad);
  return rc;
}

extern "C" int kzgx_debug_vw_bench(kzgx_ctx* ctx, int op, unsigned iters, double* res) {
  KZGX_TRY(activate(ctx));
  if (!res || iters == 0) return KZGX_ERR_ARG;
  KZGX_TRY_HIP(hipStreamSynchronize(ctx->c.stream));
  return kzgx::vw_bench(ctx->c.curve, op, iters, &res[0], &res[1], ctx->c.stream);
}
