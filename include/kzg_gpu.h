/* kzg_gpu.h -- C ABI of the MI355X KZG engine (libkzgx.so).
 *
 * This is the drop-in boundary under the reference's C++ API
 * (kzg::trusted_setup, /root/reference/src/kzg.h:182-290).  The reference has
 * no FFI of its own; these entry points replace, one for one:
 *
 *   kzgx_msm_g1*            trusted_setup::polyeval_G1  src/trusted_setup.cpp:149-174
 *                           (private, declared src/kzg.h:187) -- the G1 MSM
 *                           behind create_commit (:137-142), verify_commit
 *                           (:144-147), create_proof (:227), verify_proof (:246)
 *   kzgx_quotient_single*   q = (P - I) / Z for one opening, trusted_setup.cpp:214-225
 *                           (chunk_length == 1: I = P(z), Z = X - z)
 *   kzgx_prove_single_batch create_proof(poly, z, 1) for many (poly, z) pairs
 *   kzgx_poly_eval          evaluate_polynomial_points, src/util.cpp:186-211
 *   kzgx_poly_interpolate   polyfit / linear_roots_and_polyfit, src/util.cpp:172-184
 *   kzgx_gen_srs_g1*        trusted_setup(int) G1 part, trusted_setup.cpp:21-74,123-135
 *   kzgx_load_srs_g1        trusted_setup(const string&) G1 part, trusted_setup.cpp:76-101
 *
 * Conventions
 *   - plain pointers and sizes only; no torch / HIP types in signatures
 *     (streams are passed as void*, NULL = the context's own stream);
 *   - scalars / Fr elements: 4 x uint64 little-endian, canonical (< r);
 *   - G1 points: canonical affine x || y, each coordinate W64 = 4 (BN254) or
 *     6 (BLS12-381) uint64 little-endian limbs; infinity is x = y = 0 (never
 *     on either curve since b != 0) and is also flagged in *_is_inf outputs;
 *   - "_device" entry points take device pointers and enqueue work
 *     asynchronously on the given stream; the others take host pointers and
 *     block until the result is on the host;
 *   - every function returns KZGX_OK (0) or a negative status; kzgx_strerror
 *     names it.  The C++ facade (include/kzg.h) maps statuses onto the
 *     reference's exception types.
 *   - one context per thread (contexts are not internally locked).
 *   - a context keeps MSM workspaces for up to 8 streams at once, so calls
 *     on different streams run concurrently; a 9th distinct stream takes
 *     over the least recently bound workspace after a device-wide
 *     synchronisation (correct, but serialising: reuse streams).
 */
#ifndef KZG_GPU_H
#define KZG_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KZGX_OK 0
#define KZGX_ERR_ARG -1        /* invalid argument (std::invalid_argument) */
#define KZGX_ERR_HIP -2        /* HIP runtime failure */
#define KZGX_ERR_OOM -3        /* device allocation failed */
#define KZGX_ERR_NO_SRS -4     /* no SRS loaded */
#define KZGX_ERR_DEGREE -5     /* more coefficients than SRS points */
#define KZGX_ERR_INTERNAL -6
#define KZGX_ERR_NO_DEVICE -7  /* no usable gfx950 device */
#define KZGX_ERR_DIV_ZERO -8   /* duplicate interpolation node (NTL: division by zero) */

#define KZGX_CURVE_BN254 0     /* miracl-core BN254 (Nogami), config/curve_BN254 */
#define KZGX_CURVE_BLS12381 1  /* BLS12-381, config/curve_BLS12381 */

typedef struct kzgx_ctx kzgx_ctx;

const char* kzgx_strerror(int status);
/* uint64 limbs per base-field coordinate (4 or 6), or -1 */
int kzgx_base_limbs(int curve);

/* Device bring-up for `curve` on `device`, meant to run once, outside any
 * timed region: HIP initialisation, every kernel code object of the library
 * loaded, and the per-process generator tables (comb tables of G1 and G2,
 * used by SRS generation and verify) built.  Replaces the device-independent
 * kzg::init of the reference (src/kzg.h:33-38, kzg.cpp init; its benchmark
 * calls it before timing, benchmark/benchmark.cpp:104).  Optional: without
 * it the first setup pays the same work. */
int kzgx_init_device(int curve, int device);
int kzgx_create(kzgx_ctx** out, int curve, int device);
void kzgx_destroy(kzgx_ctx* ctx);
int kzgx_sync(kzgx_ctx* ctx);
int kzgx_curve(const kzgx_ctx* ctx);
size_t kzgx_srs_size(const kzgx_ctx* ctx);
/* the context's own HIP stream (hipStream_t), used when stream == NULL */
void* kzgx_stream(kzgx_ctx* ctx);

/* per-kernel timing: when enabled, every launch of a named kernel
 * ("msm_count", "msm_scan", "msm_scatter", "msm_accum", "msm_reduce",
 * "quotient_single") is bracketed by HIP events on its launch stream;
 * kzgx_prof_read sums (and then drops) the records of one name. */
int kzgx_prof_enable(kzgx_ctx* ctx, int on);
int kzgx_prof_read(kzgx_ctx* ctx, const char* name, double* total_ms, int* count);
int kzgx_prof_clear(kzgx_ctx* ctx);

/* tuning: signed-digit window bits (10..13; default 12 or $KZGX_WINDOW_BITS),
 * settable only before the SRS is loaded; entries per accumulation thread */
int kzgx_set_window_bits(kzgx_ctx* ctx, int c);
int kzgx_set_segment(kzgx_ctx* ctx, unsigned k);
/* tuning: table-less MSM batches of at most max_batch MSMs (default 16; 0 =
 * never) over the first 65536 SRS points run at window 10 on a second window
 * table built with the SRS: a single commit's bucket reduction is a chain of
 * dependent additions as deep as the bucket count, so the shorter window
 * answers one call sooner (BN254 degree 4096: 0.545 vs 0.712 ms) */
int kzgx_set_small_batch(kzgx_ctx* ctx, unsigned max_batch);

/* fixed-base precomputation (the SRS is fixed for a trusted_setup's
 * lifetime): store M[w][i][j] = (j+1) 2^(c w) SRS[i] for the first n_points
 * SRS points, w < ceil((bits(r)+1)/c), j < 2^(c-1), affine (BN254: 64-B
 * packed words; BLS12-381: 112-B radix-2^29 limbs).  Every MSM with
 * n <= n_points then runs as a plain sum of table points (no bucket sort /
 * reduction).  Built now if an SRS is installed, else when one is; rebuilt
 * on every SRS change.  c = 0 turns it off (Pippenger for every MSM).
 * c in {4, 7..17}; BN254 c = 17 over 4097 points (15 windows) takes
 * 257.8 GB of device memory, c = 16 137.5 GB. */
int kzgx_set_fixed_base(kzgx_ctx* ctx, int c, size_t n_points);
/* table layout for the next build: -1 = automatic (the default: point-major
 * M[i][w][j] for c <= 12, where the few-large-MSM kernel walks one point's
 * windows in order; window-major M[w][i][j] above), 0 = window-major,
 * 1 = point-major.  Results are identical; only speed differs (DESIGN.md
 * section 3).  Extension with no reference counterpart. */
int kzgx_set_fixed_base_layout(kzgx_ctx* ctx, int layout);
/* the default table (extension, no reference counterpart): odd multiples at
 * window c over the first n_points SRS points, built with every SRS load.
 * c = -1 (the default) picks the widest c <= 12 whose table fits 4.5% of the
 * device memory and its free memory less 4 GiB: over 4097 points BN254
 * c = 12 (11.8 GB), BLS12-381 c = 11 (9.7 GB) on an MI355X.  MSMs that fit in
 * it and that the main table (kzgx_set_fixed_base) does not serve take it:
 * batches of at most kzgx_set_small_batch MSMs (single create_commit /
 * create_proof calls) its one-launch path, larger batches its batched
 * kernel when c >= 10 (BN254) / 11 (BLS12-381), below which the batched
 * Pippenger is as fast.  c = 0 turns it off (every such MSM then runs the
 * table-less Pippenger, as the reference allocates nothing beyond the SRS);
 * c in {4, 7..17} fixes the window.  Rebuilt at once when an SRS is
 * installed. */
int kzgx_set_default_table(kzgx_ctx* ctx, int c, size_t n_points);
int kzgx_default_table_info(const kzgx_ctx* ctx, int* c, size_t* n_points, size_t* bytes);
/* Contexts on one device whose SRS begins with the same n_points points (word
 * for word) share one default table, counted by reference: the last context
 * using it frees it.  *count / *bytes: the shared default tables live on
 * `device` and their device bytes.  Extension, no reference counterpart. */
int kzgx_shared_tables(int device, size_t* count, size_t* bytes);
/* Freed table blocks of 64 MB .. 32 GB are kept per device (32 GB in all)
 * for later table builds, since the driver wipes released VRAM before reuse
 * ("SRS").  They are released when the last context of
 * the device is destroyed, on an allocation failure, or by this call. */
int kzgx_release_cached_memory(int device);
/* layout of the built table: *point_major = 1 (M[i][w][j]) or 0 (M[w][i][j]) */
int kzgx_fixed_base_layout(const kzgx_ctx* ctx, int* point_major);
/* built table: window bits (0 = none), points covered, device bytes */
int kzgx_fixed_base_info(const kzgx_ctx* ctx, int* c, size_t* n_points, size_t* bytes);
/* device bytes a table of window c over n_points would take (no context) */
int kzgx_fixed_base_bytes(int curve, int c, size_t n_points, size_t* bytes);
/* bounded-memory precompute: the widest supported window c <= 17 whose
 * table over n_points fits budget_bytes AND the device's free memory
 * (less a 4 GiB margin for workspaces); builds it (as kzgx_set_fixed_base)
 * and returns it in *c_out, or installs no table (*c_out = 0: every MSM on
 * Pippenger) when even c = 7 does not fit.  n_points is clamped to the
 * installed SRS; KZGX_ERR_NO_SRS before one is loaded (the free-memory
 * check needs the SRS and its window tables in place).  Extension with no
 * reference counterpart: trusted_setup::precompute_budget. */
int kzgx_set_fixed_base_budget(kzgx_ctx* ctx, size_t budget_bytes, size_t n_points, int* c_out);
/* SRS points summed per accumulation thread on the fixed-base path
 * (0 = automatic, the default: 16 for batches of >= 64 MSMs, else enough
 * threads to fill the GPU, with a wavefront-level fold for single MSMs) */
int kzgx_set_fixed_points_per_thread(kzgx_ctx* ctx, unsigned p);
/* measurement: mixed additions per second of the MSM accumulation loop
 * (the XYZZ mixed add k_fixed_accum inlines, same waves per SIMD) on
 * L1-resident operands over the whole GPU -- the VALU ceiling the bench's
 * valu_roofline divides by.  Needs an SRS (its first points are the operands). */
int kzgx_microbench_mixed_add(kzgx_ctx* ctx, double* adds_per_s);
/* measurement: the hardware issue ceiling of v_mad_u64_u32 (lane
 * operations per second; 8 independent chains per lane, whole GPU) -- the
 * denominator of the bench's mad_issue roofline */
int kzgx_microbench_mad_u64(kzgx_ctx* ctx, double* lane_ops_per_s);
/* the same, plus the core clock (GHz) the ceiling ran at: one lane of the
 * launch counts core clocks against the constant-rate wall clock */
int kzgx_microbench_mad_u64_clock(kzgx_ctx* ctx, double* lane_ops_per_s, double* core_ghz);
/* measurement: enqueue on stream (NULL = the context's) a one-wavefront
 * probe that spins for spin_us of wall time and writes three uint64 to the
 * device buffer d_out: core clocks elapsed, wall ticks elapsed, wall clock
 * rate (kHz).  Enqueued beside a running batch it reads that batch's clock
 * (the DVFS clock is one per device); it occupies one wave slot. */
int kzgx_clock_probe(kzgx_ctx* ctx, void* stream, unsigned spin_us, void* d_out);

/* ---- SRS ---------------------------------------------------------------- */
/* upload n canonical affine points as the G1 SRS (replaces any previous one) */
int kzgx_load_srs_g1(kzgx_ctx* ctx, const uint64_t* xy, size_t n);
/* generate [tau^(start+i)] G1, i < n, on the GPU and install it as the SRS */
int kzgx_gen_srs_g1(kzgx_ctx* ctx, const uint64_t* tau, size_t start, size_t n);
/* copy the installed SRS back (canonical affine) */
int kzgx_get_srs_g1(kzgx_ctx* ctx, uint64_t* xy, size_t n);

/* ---- MSM (polyeval_G1) ---------------------------------------------------- */
/* out = sum_{i<n} scalars[i] * SRS[i].  n == 0 gives infinity. */
int kzgx_msm_g1(kzgx_ctx* ctx, const uint64_t* scalars, size_t n, uint64_t* out_xy, int* out_is_inf);
/* batch of independent MSMs over the same SRS prefix: scalars[b*n + i] */
int kzgx_msm_g1_batch(kzgx_ctx* ctx, const uint64_t* scalars, size_t n, size_t batch, uint64_t* out_xy,
                      int* out_is_inf);
/* device pointers; scalar_stride = distance between consecutive MSMs in
 * scalars; out_xy: batch x 2 x W64 limbs; out_is_inf: batch x uint32 */
int kzgx_msm_g1_batch_device(kzgx_ctx* ctx, const void* d_scalars, size_t n, size_t batch, size_t scalar_stride,
                             void* d_out_xy, void* d_out_is_inf, void* stream);

/* ---- single-opening proofs (create_proof(poly, z, 1)) --------------------- */
/* q_j = (P_j - P_j(z_j)) / (X - z_j) (n-1 coefficients), y_j = P_j(z_j).
 * coeff_stride == 0 -> every opening uses the same polynomial. */
int kzgx_quotient_single_batch_device(kzgx_ctx* ctx, const void* d_coeffs, size_t n, size_t coeff_stride,
                                      const void* d_z, size_t batch, void* d_q, size_t q_stride, void* d_y,
                                      void* stream);
/* the same with host pointers (the q = (P - I) / Z step of create_proof,
 * trusted_setup.cpp:225, batched): q_out holds batch x (n - 1) scalars,
 * y_out (may be NULL) batch scalars; coeff_stride in scalars (0: shared P) */
int kzgx_quotient_single_batch(kzgx_ctx* ctx, const uint64_t* coeffs, size_t n, size_t coeff_stride,
                               const uint64_t* zs, size_t batch, uint64_t* q_out, uint64_t* y_out);
/* quotient + MSM per opening; host pointers.  out_y may be NULL. */
int kzgx_prove_single_batch(kzgx_ctx* ctx, const uint64_t* coeffs, size_t n, size_t coeff_stride,
                            const uint64_t* zs, size_t batch, uint64_t* out_xy, int* out_is_inf, uint64_t* out_y);
/* device pipeline: quotients into the workspace, then one batched MSM */
int kzgx_prove_single_batch_device(kzgx_ctx* ctx, const void* d_coeffs, size_t n, size_t coeff_stride,
                                   const void* d_z, size_t batch, void* d_out_xy, void* d_out_is_inf, void* d_y,
                                   void* stream);

/* ---- multi-point opening (create_proof(poly, off, len), any len >= 1) ------ */
/* proof = MSM of q = (P - I) / Z, I the interpolant of P at the len points
 * xs, Z = prod (X - xs[i]) (trusted_setup.cpp:214-227); all on the GPU.
 * P is normalized first; deg P < len gives q = 0 -> infinity. */
int kzgx_prove_range(kzgx_ctx* ctx, const uint64_t* coeffs, size_t n, const uint64_t* xs, size_t len,
                     uint64_t* out_xy, int* out_is_inf);

/* ---- scalar-field polynomial ops ----------------------------------------- */
/* ys[j] = P(xs[j]), j < m */
int kzgx_poly_eval(kzgx_ctx* ctx, const uint64_t* coeffs, size_t n, const uint64_t* xs, size_t m, uint64_t* ys);
/* unique interpolant of degree < n through (xs[i], ys[i]); coeffs: n entries */
int kzgx_poly_interpolate(kzgx_ctx* ctx, const uint64_t* xs, const uint64_t* ys, size_t n, uint64_t* coeffs);

/* Z = prod (X - xs[i]) (build_linear_roots_tree, src/util.cpp:269-284); z_out: n+1 entries */
int kzgx_poly_vanishing(kzgx_ctx* ctx, const uint64_t* xs, size_t n, uint64_t* z_out);

/* ---- G1 helpers ------------------------------------------------------------ */
/* *ok = 1 iff xy is a canonical on-curve affine point (ECP_fromOctet's check,
 * used by deserialize_ECP, src/util.cpp:98-115) */
int kzgx_g1_validate(kzgx_ctx* ctx, const uint64_t* xy, int* ok);
/* out = sum of count affine points (is_inf may be NULL); host pointers */
int kzgx_g1_sum(kzgx_ctx* ctx, const uint64_t* xy, const int* is_inf, size_t count, uint64_t* out_xy, int* out_is_inf);
/* The same on device pointers, enqueued on stream (NULL = the context's):
 * d_xy count canonical affine points (2 W64 words each), d_inf count uint32
 * infinity flags (may be NULL), d_out_xy one point, d_out_inf one uint32.
 * The fold of the sharded commit's gathered partials without a
 * host round trip. */
int kzgx_g1_sum_device(kzgx_ctx* ctx, const void* d_xy, const void* d_inf, size_t count, void* d_out_xy,
                       void* d_out_inf, void* stream);
/* The same fold over packed records, the exchange format of the sharded
 * commitment (python/kzgx_dist.py): record k is 2 W64 uint64 (x || y,
 * canonical little-endian) followed by one uint64 infinity word (nonzero =
 * infinity); the sum is written as one record.  One launch, one wave
 * (strided sums, a shuffle tree, a wave-uniform inversion).  Device
 * pointers; stream as kzgx_msm_g1_batch_device. */
int kzgx_g1_sum_packed_device(kzgx_ctx* ctx, const void* d_records, size_t count, void* d_out_record, void* stream);
/* Projective partials (round 6): the sharded commitment's per-rank MSM left
 * as one XYZZ point (X, Y, ZZ, ZZZ in the library's radix-2^29 Montgomery
 * limbs; ZZ = 0 is infinity) -- an exchange format between ranks running this
 * library, kzgx_partial_record_words(curve) uint64 words (BN254 18,
 * BLS12-381 28) -- so no rank inverts; kzgx_g1_sum_partials_device adds
 * count such records and converts the sum once, into one packed affine
 * record (as kzgx_g1_sum_packed_device).  Device pointers; stream as
 * kzgx_msm_g1_batch_device.  n = 0 gives the identity record. */
int kzgx_partial_record_words(int curve);
int kzgx_msm_g1_partial_device(kzgx_ctx* ctx, const void* d_scalars, size_t n, void* d_out_record, void* stream);
int kzgx_g1_sum_partials_device(kzgx_ctx* ctx, const void* d_records, size_t count, void* d_out_record, void* stream);
/* One commitment sharded over several contexts, typically one per GPU (the
 * one-process form of SURVEY 8e's sharded commit; bench.py's configs[4] runs
 * the one-process-per-GPU form over RCCL).  Context k holds the SRS slice
 * starting at point starts[k] (kzgx_gen_srs_g1(ctx, tau, starts[k], n_k) or
 * kzgx_load_srs_g1); the slices must be contiguous from 0 (starts[k + 1] ==
 * starts[k] + |SRS_k|, else KZGX_ERR_ARG) and cover n (else
 * KZGX_ERR_DEGREE).  Every context runs the partial MSM of its slice of
 * scalars[0..n) on its own stream, concurrently; the projective partials are
 * then folded exactly on ctxs[0] (affine result, bit-exact with one MSM). */
int kzgx_msm_g1_sharded(kzgx_ctx* const* ctxs, const size_t* starts, size_t nctx, const uint64_t* scalars,
                        size_t n, uint64_t* out_xy, int* out_is_inf);

/* ---- verify half: G2 setup, polyeval_G2, pairing ----------------------------
 * G2 points are canonical affine on the sextic twist (BN254: D-type
 * y^2 = x^3 + 2/(1+i); BLS12-381: M-type y^2 = x^3 + 4(1+i)), Fp2 = Fp[i],
 * i^2 = -1, stored as x.re || x.im || y.re || y.im (4 x W64 limbs); all zero
 * = infinity.  Fp12 values are 12 canonical Fp elements in tower order
 * (Fp6 = Fp2[v]/(v^3 - (1+i)), Fp12 = Fp6[w]/(w^2 - v)):
 * c0.c0, c0.c1, c0.c2, c1.c0, c1.c1, c1.c2, each (re, im). */
/* generate [tau^(start+i)] G2, i < n (G2 half of generate_elements_range,
 * src/trusted_setup.cpp:123-135) and install it */
int kzgx_gen_srs_g2(kzgx_ctx* ctx, const uint64_t* tau, size_t start, size_t n);
/* install n canonical affine G2 points (G2 half of the setup-file loader,
 * src/trusted_setup.cpp:103-118) */
int kzgx_load_srs_g2(kzgx_ctx* ctx, const uint64_t* xy, size_t n);
int kzgx_get_srs_g2(kzgx_ctx* ctx, uint64_t* xy, size_t n);
size_t kzgx_srs_g2_size(const kzgx_ctx* ctx);
/* ok[k] = 1 iff point k is canonical and on the twist (ECP2_fromOctet) */
int kzgx_g2_validate(kzgx_ctx* ctx, const uint64_t* xy, size_t count, int* ok);
/* out = sum_{i<n} scalars[i] [tau^i]G2 (polyeval_G2, src/trusted_setup.cpp:176-201) */
int kzgx_msm_g2(kzgx_ctx* ctx, const uint64_t* scalars, size_t n, uint64_t* out_xy, int* out_is_inf);
/* out[k] = e(P_k, Q_k): optimal ate pairing + final exponentiation
 * (miracl PAIR_ate + PAIR_fexp, src/trusted_setup.cpp:240-250); inf flags may be NULL */
int kzgx_pairing(kzgx_ctx* ctx, const uint64_t* g1_xy, const int* g1_inf, const uint64_t* g2_xy, const int* g2_inf,
                 size_t count, uint64_t* out);
/* trusted_setup::verify_proof (src/trusted_setup.cpp:230-254): *ok =
 * e(proof, [Z(tau)]G2) == e(C - [I(tau)]G1, G2[0]) for the npoints opened
 * points (xs, ys); npoints >= |SRS G1| gives *ok = 0; npoints == 0 is
 * KZGX_ERR_ARG; needs a G2 setup of >= npoints + 1 points.  npoints == 1
 * runs as kzgx_verify_single_batch with one opening (same boolean). */
int kzgx_verify_proof(kzgx_ctx* ctx, const uint64_t* commit_xy, int commit_inf, const uint64_t* proof_xy,
                      int proof_inf, const uint64_t* xs, const uint64_t* ys, size_t npoints, int* ok);
/* batch of single-point verifies (verify_proof with one opened point each):
 * ok[k] = e(proof_k, [tau - z_k]G2) == e(commit_k - [y_k]G1, G2), evaluated as
 * one two-Miller-loop product and one final exponentiation per opening (a
 * wave or a lane each, see kzgx_set_verify_wave_max).  Needs G1[0] = G and
 * G2[0..1]; inf arrays may be NULL. */
int kzgx_verify_single_batch(kzgx_ctx* ctx, const uint64_t* commits_xy, const int* commit_inf,
                             const uint64_t* proofs_xy, const int* proof_inf, const uint64_t* zs, const uint64_t* ys,
                             size_t count, int* ok);
/* device pointers (inf flags uint32, may be NULL), ok: count x uint32 */
int kzgx_verify_single_batch_device(kzgx_ctx* ctx, const void* d_commits, const void* d_commit_inf,
                                    const void* d_proofs, const void* d_proof_inf, const void* d_z, const void* d_y,
                                    size_t count, void* d_ok, void* stream);
/* Batches of at most max_count openings (default 4096) run one 64-lane wave
 * per opening (Fp12 products spread over the wave, setup-derived line and
 * [y]G tables built on first use); larger batches run one lane per opening.
 * Both give the same booleans; 0 forces the lane-per-opening kernel. */
int kzgx_set_verify_wave_max(kzgx_ctx* ctx, size_t max_count);

#ifdef __cplusplus
}
#endif

#endif /* KZG_GPU_H */
