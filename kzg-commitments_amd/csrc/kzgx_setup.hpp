// Pieces shared across translation units that are not the batched hot
// path: device bring-up, the per-process generator tables, comb SRS
// generation and the batch-affine table builder (setup.hip), and the
// lone-wave kernels compiled with the latency-first product (latency.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace kzgx {

// One trivial launch per translation unit: the first launch of any kernel of
// a code object loads that whole object onto the device, so kzgx_init_device
// (the reference's kzg::init, src/kzg.h:33-38, called outside the timed
// regions of benchmark/benchmark.cpp:104) pays every load up front.
int warm_setup(hipStream_t st);
int warm_msm(hipStream_t st);
int warm_msm_fixed(hipStream_t st);
int warm_poly(hipStream_t st);
int warm_srs(hipStream_t st);
int warm_pairing(hipStream_t st);
int warm_verify_wave(hipStream_t st);
int warm_latency(hipStream_t st);
// the fixed-base MSM's per-window objects (msm_fixed_inst.hip, one per group)
int warm_fixed_bn_a(hipStream_t st);
int warm_fixed_bn_b(hipStream_t st);
int warm_fixed_bn_c(hipStream_t st);
int warm_fixed_bn_d(hipStream_t st);
int warm_fixed_bls_a(hipStream_t st);
int warm_fixed_bls_b(hipStream_t st);
int warm_fixed_bls_c(hipStream_t st);
int warm_fixed_bls_d(hipStream_t st);

// Per-process tables of the curve generators, one per (device, curve), built
// once (kzgx_init_device, or the first setup that needs them) and kept until
// process exit:
//   g1_comb[w][d - 1] = d 2^(8 w) G,   w < 32, d = 1..255, affine Montgomery
//                       (affine_words per entry; the [y]G table of verify)
//   g2_comb[w][d - 1] = d 2^(8 w) G2,  same layout, G2A<C> per entry
struct GenTables {
  uint32_t* g1_comb = nullptr;
  uint32_t* g2_comb = nullptr;
};
constexpr int GEN_COMB_ENTRIES = 32 * 255;
int gen_tables_get(int curve, int device, hipStream_t st, GenTables* out);

// [tau^(start + i)] G1 / G2 for i < n from the comb tables: 32 lanes per
// point each take one 8-bit window's entry, a 5-level shuffle tree sums
// them, and lane 0 converts to canonical affine (replaces a 256-bit
// double-and-add per point: generate_elements_range, trusted_setup.cpp:123-135)
int gen_srs_g1_comb(int curve, const uint32_t* d_tau, size_t start, size_t n, const uint32_t* g1_comb,
                    uint32_t* d_out, hipStream_t st);
int gen_srs_g2_comb(int curve, const uint32_t* d_tau, size_t start, size_t n, const uint32_t* g2_comb,
                    uint32_t* d_out, hipStream_t st);

// The odd multiples (2 j + 1) B[w][i], j < H, of every window base into the
// fixed-base table at strides (is, ws) words, by batch-affine chains: each
// thread owns `per` consecutive entries of one (w, i) as 8 interleaved chains
// stepping by 16 B, and one inversion serves the 8 additions of a step
// (Montgomery's trick) instead of one per entry.
int fixed_multiples_batch(int curve, const uint32_t* d_bases, const uint8_t* d_inf, uint32_t n, int W, uint32_t H,
                          size_t is, size_t ws, uint32_t* d_tab, hipStream_t st);

// the verify path's [y]G table for the setup's G1[0] (canonical): a copy of
// g1_comb when G1[0] is the curve generator, else computed
int vtab_prepare(int curve, const uint32_t* d_g1_0, const uint32_t* g1_comb, uint32_t* d_vtab, hipStream_t st);

// the sharded commitment's fold (latency.hip): count packed records
// (x || y canonical words, then a 64-bit infinity word) summed into one
int g1_fold_packed(int curve, const uint32_t* d_rec, size_t count, uint32_t* d_out, hipStream_t st);
// polyeval_G2's windowed table (pairing.hip k_g2_terms_w) of a generated G2
// SRS [tau^(start+i)]G2, i < n: G2_TAB_WINDOWS entries per point from the
// generator's comb (setup.hip k_g2_tab_comb): entry (i, w) = 2^(G2_TAB_BITS w)
// [tau^(start+i)]G2
#ifndef KZGX_G2_TAB_BITS
#define KZGX_G2_TAB_BITS 8
#endif
constexpr int G2_TAB_BITS = KZGX_G2_TAB_BITS;
static_assert(G2_TAB_BITS == 4 || G2_TAB_BITS == 8 || G2_TAB_BITS == 16, "digits must tile a 32-bit word");
constexpr int G2_TAB_WINDOWS = 256 / G2_TAB_BITS;
int g2_table_comb(int curve, const uint32_t* d_tau, size_t start, size_t n, const uint32_t* g2_comb, uint32_t* d_tab,
                  hipStream_t st);
// the same over projective partial records (one XYZZ point, xyzz_record_words
// words each: the partials stay projective, the fold inverts once), and the
// lift of an affine point (+ flag) into such a record
size_t xyzz_record_words(int curve);
int g1_fold_xyzz(int curve, const uint32_t* d_rec, size_t count, uint32_t* d_out, hipStream_t st);
int affine_to_xyzz(int curve, const uint32_t* d_xy, const uint32_t* d_inf, uint32_t* d_rec, hipStream_t st);

// latency of one wave-wide Fp12 op of the verify path (verify_wave.hip
// k_vw_bench; kzgx_debug_vw_bench)
int vw_bench(int curve, int op, uint32_t iters, double* ns_per_op, double* clk_per_op, hipStream_t st);

// the bucket reduction of one wide-window Pippenger MSM (latency.hip):
// sum_k (k + 1) B_k over nb >= 4096 buckets (bsum, occupancy from offsets)
// -> canonical affine out / out_inf, or (xyzz_out) the XYZZ sum itself;
// d_rt: big_reduce_rt_bytes of scratch
size_t big_reduce_rt_bytes(int curve, uint32_t nb);
int big_reduce(int curve, const uint32_t* d_offsets, uint32_t nb, const uint32_t* d_bsum, uint32_t* d_rt,
               uint32_t* d_out, uint32_t* d_out_inf, hipStream_t st, uint32_t* xyzz_out = nullptr);
// the same from bucket-aligned segment partials (msm.hip k_big2_*): bucket k
// owns part[seg_off[k] .. seg_off[k + 1]); s_ub bounds seg_off[nb]; *d_flag:
// some bucket has more than 64 partials (pre-sum passes run); part is
// overwritten
int big_reduce_seg(int curve, const uint32_t* d_seg_off, uint32_t* d_part, uint32_t nb, uint32_t s_ub,
                   const uint32_t* d_flag, uint32_t* d_rt, uint32_t* d_out, uint32_t* d_out_inf, hipStream_t st,
                   uint32_t* xyzz_out = nullptr);

}  // namespace kzgx
