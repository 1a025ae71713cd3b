// Internal (host-side) declarations shared by the libkzgx translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <vector>

#include "../../include/kzg_gpu.h"

#ifndef KZGX_ACCUM_WAVES
#define KZGX_ACCUM_WAVES 3  // min waves per SIMD for k_msm_accum (VGPR budget)
#endif

#ifndef KZGX_BS_WAVES
#define KZGX_BS_WAVES 2  // min waves per SIMD for k_msm_bucket_sums
#endif

#ifndef KZGX_WINDOW_BITS
#define KZGX_WINDOW_BITS 12  // default signed-digit window (10..13 supported)
#endif

#define KZGX_TRY(expr)                 \
  do {                                 \
    int _rc = (expr);                  \
    if (_rc != KZGX_OK) return _rc;    \
  } while (0)

#define KZGX_TRY_HIP(expr)                              \
  do {                                                  \
    hipError_t _e = (expr);                             \
    if (_e != hipSuccess) return ::kzgx::hip_fail(_e);  \
  } while (0)

namespace kzgx {

int hip_fail(hipError_t e);

struct MsmWs {
  uint32_t *counts = nullptr, *offsets = nullptr, *cursors = nullptr, *entries = nullptr;
  uint32_t *bsum = nullptr, *heads = nullptr, *tails = nullptr, *tailk = nullptr, *rt = nullptr, *q = nullptr,
           *parts = nullptr, *fpart = nullptr, *fsum = nullptr, *gpart = nullptr, *gmeta = nullptr, *qbig = nullptr;
  uint8_t* sstate = nullptr;
  uint32_t* lat_cnt = nullptr;  // [64] arrival counters of the one-launch latency path (msm_fixed.hip)
  size_t counts_b = 0, offsets_b = 0, cursors_b = 0, entries_b = 0, bsum_b = 0, heads_b = 0, tails_b = 0, tailk_b = 0,
         rt_b = 0, q_b = 0, parts_b = 0, fpart_b = 0, fsum_b = 0, gpart_b = 0, gmeta_b = 0, sstate_b = 0, qbig_b = 0;
  hipStream_t owner = nullptr;  // workspaces are per stream so calls on
  bool used = false;            // different streams may run concurrently
  uint64_t bound_at = 0;        // Ctx::ws_clock when bound to owner
  hipEvent_t done = nullptr;    // recorded on the owner stream after the last call that used this slot
  bool done_recorded = false;
};

struct Ctx;
// A workspace bound to a stream for the length of one call.  Its destructor
// records the slot's `done` event on that stream after everything the call
// enqueued, so rebinding the slot later waits on the event -- never on the
// old owner stream's handle, which the caller may have destroyed since.
class WsLease {
 public:
  WsLease(Ctx* c, MsmWs* w, hipStream_t st) : c_(c), w_(w), st_(st) {}
  WsLease(const WsLease&) = delete;
  WsLease& operator=(const WsLease&) = delete;
  ~WsLease();
  MsmWs* operator->() const { return w_; }
  MsmWs& operator*() const { return *w_; }
  bool operator!() const { return w_ == nullptr; }
  MsmWs* get() const { return w_; }

 private:
  Ctx* c_;
  MsmWs* w_;
  hipStream_t st_;
};

constexpr int KZGX_MAX_STREAMS = 8;

// precomputed odd multiples of the SRS prefix (msm_fixed.hip, indexed by
// the regular odd digits of fixed_accum.hpp):
// M[w][i][j] = (2 j + 1) 2^(c w) P_i, packed affine, w < W, i < n_t, j < 2^(c-1)
struct FixedTable {
  int c_req = 0;        // requested window bits (0 = off)
  size_t n_req = 0;     // requested SRS prefix length
  uint32_t pts_per_thread = 0;  // 0 = automatic (fixed_msm_impl)
  int c = 0, W = 0;     // built table
  size_t n_t = 0;
  int layout_req = -1;       // -1 automatic, 0 window-major, 1 point-major
  bool point_major = false;  // built: M[i][w][j] instead of M[w][i][j] (msm_fixed.hip)
  uint32_t* d = nullptr;
  size_t bytes = 0;
  uint8_t* inf = nullptr;  // [n_t] infinite SRS points (skipped)
  bool any_inf = true;     // some flag of inf is set (else the kernels get no flags)
  uint32_t fin0 = UINT32_MAX;  // first finite point of the prefix (k_fixed_accum's identity terms)
  int shared = 0;  // registry id of a shared default table (kzgx_api.hip), 0 = owned by this context
};

// per-device table memory (kzgx_api.hip): the cached block of the last freed
// default-size table, and the registry of default tables shared by contexts
// with the same device, curve, window and SRS prefix
hipError_t table_malloc(void** p, size_t bytes);
void table_free(void* p, size_t bytes);
void table_cache_release();
size_t table_cache_bytes();
bool table_share_attach(int device, int curve, int c_req, const uint32_t* d_canon, size_t key_words, hipStream_t st,
                        FixedTable& ft);
void table_share_register(int device, int curve, const uint32_t* d_canon, size_t key_words, hipStream_t st,
                          FixedTable& ft);
void table_share_release(FixedTable& ft);
void shared_tables_info(int device, size_t* count, size_t* bytes);

// optional per-kernel timing with HIP events on the launch stream
struct ProfRec {
  const char* name;
  hipEvent_t a, b;
};

// the default table (Ctx::fixed_def): odd multiples of the first 4097 SRS
// points (degree-4096 calls and below) at the widest window c <= 12 whose
// table fits KZGX_DEFAULT_TABLE_PERMILLE of the device's memory -- 45 per
// mille = 13 GB of an MI355X: BN254 c = 12 (11.8 GB), BLS12-381 c = 11
// (9.7 GB).  -1 = that automatic choice, 0 = none, c = a fixed window.
#ifndef KZGX_DEFAULT_TABLE_BITS
#define KZGX_DEFAULT_TABLE_BITS -1
#endif
#ifndef KZGX_DEFAULT_TABLE_POINTS
#define KZGX_DEFAULT_TABLE_POINTS 4097
#endif
#ifndef KZGX_DEFAULT_TABLE_PERMILLE
#define KZGX_DEFAULT_TABLE_PERMILLE 45
#endif
// batches larger than Ctx::small_batch use the default table from this
// window on (below it the batched Pippenger is as fast or faster).  cfg2
// shape, BN254: c = 10 138k-141k / 11 148k-151k / 12 161k-164k against
// Pippenger's 130k per second; cfg4 shape, BLS12-381: c = 10 63k-64k /
// 12 75k against 64k (profiles/r04_default_table_windows.json)
#ifndef KZGX_DEFAULT_TABLE_BATCH_MIN_C_BN
#define KZGX_DEFAULT_TABLE_BATCH_MIN_C_BN 10
#endif
#ifndef KZGX_DEFAULT_TABLE_BATCH_MIN_C_BLS
#define KZGX_DEFAULT_TABLE_BATCH_MIN_C_BLS 11
#endif

// batches of at most this many MSMs use the small-window table (msm.hip)
#ifndef KZGX_SMALL_BATCH
#define KZGX_SMALL_BATCH 16
#endif

struct Ctx {
  int curve = 0;
  int device = 0;
  hipStream_t stream = nullptr;
  int c = KZGX_WINDOW_BITS;  // window bits
  int W = 0;                 // windows
  uint32_t seg_k = 128;      // entries per accumulation thread
  size_t n_srs = 0;
  uint32_t* d_table = nullptr;  // [W][n_srs] affine Montgomery points
  size_t table_bytes = 0;
  // small-batch window table (msm.hip, msm_batch_c): [W_s][n_small] at
  // window KZGX_SMALL_WINDOW_BITS over the first n_small SRS points
  uint32_t* d_table_small = nullptr;
  size_t table_small_bytes = 0;
  size_t n_small = 0;
  hipEvent_t small_ev = nullptr;  // recorded after the small table's build (small_table_ready)
  // wide-window table of the large single MSMs (msm.hip, msm_big):
  // [W_big][n_srs] at c_big bits, built with an SRS of >= 2^16 points
  uint32_t* d_table_big = nullptr;
  size_t table_big_bytes = 0;
  int c_big = 0;  // 0: none / stale
  size_t small_batch = KZGX_SMALL_BATCH;  // largest batch that uses it (0: never)
  uint8_t* d_inf = nullptr;  // [n_srs]
  size_t inf_bytes = 0;
  MsmWs ws[KZGX_MAX_STREAMS];
  FixedTable fixed;
  // the default table: odd multiples at a bounded window over the first SRS
  // points, built with the SRS, read by the MSMs the main table does not
  // serve (msm.hip msm_batch; kzgx_set_default_table); c_req -1 = the
  // window is picked from the memory budget at each build
  FixedTable fixed_def{KZGX_DEFAULT_TABLE_BITS, KZGX_DEFAULT_TABLE_POINTS};
  // the workspace bound to stream st (claimed on first use; every lookup
  // refreshes its use stamp).  With more than KZGX_MAX_STREAMS distinct
  // streams the least recently USED slot is rebound once the work of its
  // last call has drained: hipEventSynchronize of the slot's own event,
  // recorded by the lease after that call's last enqueue (other streams and
  // contexts keep running, and the old owner stream may already be
  // destroyed).  A null lease only if that synchronisation fails.
  uint64_t ws_clock = 0;
  MsmWs* ws_find(hipStream_t st) {
    for (auto& w : ws)
      if (w.used && w.owner == st) return &w;
    return nullptr;
  }
  WsLease ws_for(hipStream_t st) {
    if (MsmWs* w = ws_find(st)) {
      w->bound_at = ++ws_clock;
      return WsLease(this, w, st);
    }
    for (auto& w : ws)
      if (!w.used) {
        w.used = true;
        w.owner = st;
        w.bound_at = ++ws_clock;
        return WsLease(this, &w, st);
      }
    MsmWs* lru = &ws[0];
    for (auto& w : ws)
      if (w.bound_at < lru->bound_at) lru = &w;
    if (lru->done_recorded && hipEventSynchronize(lru->done) != hipSuccess) return WsLease(this, nullptr, st);
    lru->done_recorded = false;
    lru->owner = st;
    lru->bound_at = ++ws_clock;
    return WsLease(this, lru, st);
  }
  // end of a call's use of w on st (WsLease destructor)
  void ws_release(MsmWs* w, hipStream_t st) {
    if (!w->done && hipEventCreateWithFlags(&w->done, hipEventDisableTiming) != hipSuccess) {
      w->done = nullptr;
      (void)hipStreamSynchronize(st);  // no event: drain now, while st is known to be alive
      return;
    }
    w->done_recorded = hipEventRecord(w->done, st) == hipSuccess;
    if (!w->done_recorded) (void)hipStreamSynchronize(st);
  }
  bool prof_on = false;
  std::vector<ProfRec> prof;
  void* d_poly_ws = nullptr;  // scratch for the Fr polynomial kernels
  size_t poly_ws_b = 0;
  void* d_poly_ws2 = nullptr;  // scratch of the multi-point opening pipeline
  size_t poly_ws2_b = 0;
  void* d_g2_ws = nullptr;  // G2 MSM terms (pairing.hip)
  size_t g2_ws_b = 0;
  uint32_t* d_lift = nullptr;  // msm_partial_xyzz's affine result before the lift
  size_t lift_b = 0;
  // staging for host-pointer entry points
  void* d_stage[4] = {nullptr, nullptr, nullptr, nullptr};
  size_t stage_b[4] = {0, 0, 0, 0};
  int base_words() const { return curve == KZGX_CURVE_BN254 ? 8 : 12; }
};

inline WsLease::~WsLease() {
  if (w_) c_->ws_release(w_, st_);
}

// bracket one launch with events when profiling is enabled
struct ProfScope {
  Ctx* ctx;
  hipStream_t st;
  ProfRec rec;
  ProfScope(Ctx* c, hipStream_t s, const char* name) : ctx(c), st(s) {
    rec.name = nullptr;
    if (!ctx->prof_on) return;
    rec.name = name;
    (void)hipEventCreate(&rec.a);
    (void)hipEventCreate(&rec.b);
    (void)hipEventRecord(rec.a, st);
  }
  ~ProfScope() {
    if (!rec.name) return;
    (void)hipEventRecord(rec.b, st);
    ctx->prof.push_back(rec);
  }
};

// grow-only device allocation (frees the old block)
int dev_alloc(Ctx* ctx, void** p, size_t bytes, size_t* cap);

bool window_bits_supported(int c);
bool fixed_bits_supported(int c);
int fixed_windows(int curve, int c);
int fixed_build(Ctx* ctx, const uint32_t* d_canon, size_t n_srs);  // the main and the default table
int fixed_build_table(Ctx* ctx, FixedTable& ft, const uint32_t* d_canon, size_t n_srs);
int fixed_rebuild_default(Ctx* ctx, const uint32_t* d_canon, size_t n_srs);
void fixed_free(Ctx* ctx);  // the main table
void fixed_free_table(FixedTable& ft);
bool fixed_usable(const Ctx* ctx, size_t n);
bool fixed_table_usable(const FixedTable& ft, size_t n);
int fixed_msm_table(Ctx* ctx, FixedTable& ft, const uint32_t* d_scalars, size_t n, size_t batch, size_t stride_words,
                    uint32_t* d_out, uint32_t* d_out_inf, hipStream_t st, uint32_t* xyzz_out);
int fixed_msm(Ctx* ctx, const uint32_t* d_scalars, size_t n, size_t batch, size_t stride_words, uint32_t* d_out,
              uint32_t* d_out_inf, hipStream_t st, uint32_t* xyzz_out);
int srs_upload(Ctx* ctx, const uint32_t* d_canon, size_t n);
// mixed additions / s of the fixed-base accumulation loop on L1-resident operands (msm_fixed.hip)
int microbench_mixed_add(Ctx* ctx, double* rate);
int microbench_mad_u64(Ctx* ctx, double* rate, double* ghz);
int clock_probe(Ctx* ctx, hipStream_t st, uint32_t spin_us, uint64_t* d_out);
size_t fixed_table_bytes(int curve, int c, size_t n);
int debug_latency(Ctx* ctx, int op, uint32_t iters, double* res);  // ns, core clocks per op
// one workgroup sums count XYZZ points -> canonical affine (msm.hip)
int xyzz_sum(Ctx* ctx, const uint32_t* d_parts, size_t count, uint32_t* d_out, uint32_t* d_out_inf, hipStream_t st);
int msm_batch(Ctx* ctx, const uint32_t* d_scalars, size_t n, size_t batch, size_t stride_words, uint32_t* d_out,
              uint32_t* d_out_inf, hipStream_t st);
// one MSM as an XYZZ record, no affine conversion (msm.hip)
int msm_partial_xyzz(Ctx* ctx, const uint32_t* d_scalars, size_t n, uint32_t* d_rec, hipStream_t st);
int gen_srs_points(Ctx* ctx, const uint32_t* tau_canon_host, size_t start, size_t n, uint32_t* d_out_canon,
                   hipStream_t st);
int g1_validate(Ctx* ctx, const uint32_t* d_xy, uint32_t* d_ok, hipStream_t st);
int g1_sum(Ctx* ctx, const uint32_t* d_xy, const uint32_t* d_inf, size_t count, uint32_t* d_out, uint32_t* d_out_inf,
           hipStream_t st);

// scalar field (Fr) kernels, poly.hip
int quotient_single(Ctx* ctx, const uint32_t* d_coeffs, size_t n, size_t coeff_stride_words, const uint32_t* d_z,
                    size_t batch, uint32_t* d_q, size_t q_stride_words, uint32_t* d_y, hipStream_t st);
int poly_eval(Ctx* ctx, const uint32_t* d_coeffs, size_t n, const uint32_t* d_x, size_t m, uint32_t* d_y,
              hipStream_t st);
int poly_vanishing(Ctx* ctx, const uint32_t* d_x, size_t n, uint32_t* d_Z, hipStream_t st);
int prove_range_poly(Ctx* ctx, const uint32_t* d_P, size_t n, const uint32_t* d_x, size_t len, uint32_t* d_q,
                     size_t* nq, hipStream_t st);
int poly_interpolate(Ctx* ctx, const uint32_t* d_x, const uint32_t* d_y, size_t n, uint32_t* d_coeffs,
                     hipStream_t st);
int verify_ws_reserve(Ctx* ctx, size_t n);  // poly.hip: workspaces of an n-point verify_proof
int g2_ws_reserve(Ctx* ctx, size_t n);      // pairing.hip: an n-point G2 MSM's workspace

// verify path: G2 SRS, polyeval_G2, pairing (pairing.hip)
int gen_srs_g2_points(Ctx* ctx, const uint32_t* d_tau, size_t start, size_t n, uint32_t* d_out, hipStream_t st);
// d_tab (optional): g2_table_build's windowed multiples of the G2 SRS
size_t g2_table_bytes(int curve, size_t n);
int g2_table_build(Ctx* ctx, const uint32_t* d_srs2, size_t n, uint32_t* d_tab, hipStream_t st);
int msm_g2(Ctx* ctx, const uint32_t* d_scalars, const uint32_t* d_srs2, size_t n, uint32_t* d_out,
           uint32_t* d_out_inf, hipStream_t st,
           const uint32_t* d_tab = nullptr);
int g2_validate(Ctx* ctx, const uint32_t* d_xy, size_t count, uint32_t* d_ok, hipStream_t st);
int pairing_batch(Ctx* ctx, const uint32_t* d_g1, const uint32_t* d_g1_inf, const uint32_t* d_g2,
                  const uint32_t* d_g2_inf, size_t count, uint32_t* d_out, hipStream_t st);
int verify_single_batch(Ctx* ctx, const uint32_t* d_commits, const uint32_t* d_commit_inf, const uint32_t* d_proofs,
                        const uint32_t* d_proof_inf, const uint32_t* d_z, const uint32_t* d_y, size_t count,
                        const uint32_t* d_g1_0, const uint32_t* d_g2_01, uint32_t* d_ok, hipStream_t st);
// wave-per-opening verify (pairing.hip): setup-derived tables, then the batch
size_t verify_wave_bytes(int curve);
// g1_comb: the generator's comb (kzgx_setup.hpp GenTables), copied into the
// buffer when G1[0] is the generator; null: computed from G1[0]
int verify_wave_prepare(Ctx* ctx, const uint32_t* d_g1_0, const uint32_t* d_g2_01, const uint32_t* g1_comb,
                        uint32_t* d_buf, hipStream_t st);
int verify_wave_batch(Ctx* ctx, const uint32_t* d_commits, const uint32_t* d_commit_inf, const uint32_t* d_proofs,
                      const uint32_t* d_proof_inf, const uint32_t* d_z, const uint32_t* d_y, size_t count,
                      const uint32_t* d_g1_0, const uint32_t* d_buf, uint32_t* d_ok, hipStream_t st);
// one wave: *ok = e(P_0, Q_0) e(-P_1, Q_1) == 1 (p: 2 canonical affine G1
// points, q: 2 canonical G2 points, inf flags may be NULL; scratch of
// pair2_wave_scratch_bytes for the line tables)
size_t pair2_wave_scratch_bytes(int curve);
int pair2_wave(Ctx* ctx, const uint32_t* d_p, const uint32_t* d_p_inf, const uint32_t* d_q, const uint32_t* d_q_inf,
               uint32_t* d_scratch, uint32_t* d_ok, hipStream_t st);
// the same with Q_1 = G2[0] (d_vw: verify_wave_prepare's buffer) in one
// launch of three waves, Q_0's line chain overlapping the Miller loop; *ok = 2
// for a degenerate chain (rerun pair2_wave); d_q: Q_0 alone, d_q_inf: its flag
int pair2_fused(Ctx* ctx, const uint32_t* d_p, const uint32_t* d_p_inf, const uint32_t* d_q, const uint32_t* d_q_inf,
                const uint32_t* d_vw, uint32_t* d_ok, hipStream_t st);
int g1_sub(Ctx* ctx, const uint32_t* d_a, const uint32_t* d_a_inf, const uint32_t* d_b, const uint32_t* d_b_inf,
           uint32_t* d_out, uint32_t* d_out_inf, hipStream_t st);

}  // namespace kzgx
