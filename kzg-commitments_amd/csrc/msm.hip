// Batched Pippenger G1 MSM for gfx950 -- the hot path behind
// kzg::trusted_setup::create_commit / create_proof / verify_commit
// (reference: trusted_setup::polyeval_G1, src/trusted_setup.cpp:149-174,
// a naive per-term PAIR_G1mul + ECP_add loop).
//
// Design (MI355X-first):
//  * fixed-base windows: at SRS load every point P_i is expanded into W
//    window copies T[w][i] = 2^(c w) P_i (affine, Montgomery, HBM resident),
//    so all windows of an MSM share ONE set of 2^(c-1) signed-digit buckets and
//    there is no per-window doubling chain;
//  * per MSM b: signed c-bit digits -> (point, sign) entries counting-sorted by
//    bucket (LDS histograms + one global atomic per (workgroup, bucket));
//  * bucket accumulation is load balanced: every thread owns exactly K
//    consecutive sorted entries and does K mixed XYZZ additions; runs that
//    cross a segment boundary leave head/tail partials that the reduction
//    kernel merges;
//  * the reduction (one workgroup per MSM) finishes the buckets, forms
//    sum (k+1) B_k with an LDS suffix scan + tree, and converts to affine.
// Every step is an exact group operation, so the affine output is bit-exact
// with any other correct evaluation of sum c_i [tau^i]G1.
#include <hip/hip_runtime.h>

#include "curve.hpp"
#include "kzgx_internal.hpp"

namespace kzgx {

// --------------------------------------------------------------------------
// SRS upload / fixed-base table
// --------------------------------------------------------------------------
// canonical affine (x||y, 2N words per point) -> Montgomery into T[0];
// all-zero input marks infinity.
template <class C>
__global__ void k_srs_to_mont(const uint32_t* __restrict__ canon, uint32_t* __restrict__ table, uint8_t* __restrict__ inf,
                              uint32_t n) {
  constexpr int AW = affine_words<C>();
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Affine<C> a;
  const bool finite = affine_from_canonical<C>(canon + (size_t)i * 2 * C::Fp::N, a);
  inf[i] = finite ? 0 : 1;
  affine_store<C>(table + (size_t)i * AW, a);
}

// T[w][i] = 2^c T[w-1][i] for w = 1..W-1
template <class C>
__global__ void k_table_build(uint32_t* __restrict__ table, const uint8_t* __restrict__ inf, uint32_t n, int W, int c) {
  using F = typename C::Fp29;
  constexpr int AW = affine_words<C>();
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Affine<C> a = affine_load<C>(table + (size_t)i * AW);
  const bool is_inf = inf[i] != 0;
  for (int w = 1; w < W; w++) {
    if (!is_inf) {
      Xyzz<C> p = xyzz_from_affine<C>(a);
      for (int s = 0; s < c; s++) p = xyzz_dbl<C>(p);
      if (!xyzz_to_affine<C>(p, a)) {
        a.x = f29_zero<F>();
        a.y = f29_zero<F>();
      }
    }
    affine_store<C>(table + ((size_t)w * n + i) * AW, a);
  }
}

// --------------------------------------------------------------------------
// signed-digit recoding
// --------------------------------------------------------------------------
template <int CB>
struct Win {
  static constexpr int W = (257 + CB - 1) / CB;  // covers any 256-bit integer
  static constexpr uint32_t NB = 1u << (CB - 1);
};

// digit w of the scalar (8 canonical LE words); returns signed digit, updates carry
template <int CB>
KZGX_DEV int digit_at(const uint32_t (&s)[8], int w, uint32_t& carry) {
  const int bit = CB * w;
  const int word = bit >> 5;
  const int sh = bit & 31;
  uint32_t raw = 0;
  if (word < 8) {
    raw = s[word] >> sh;
    if (sh + CB > 32 && word + 1 < 8) raw |= s[word + 1] << (32 - sh);
  }
  raw &= (1u << CB) - 1u;
  raw += carry;
  if (raw > Win<CB>::NB) {
    carry = 1;
    return (int)raw - (1 << CB);
  }
  carry = 0;
  return (int)raw;
}

KZGX_DEV void load_scalar(const uint32_t* p, uint32_t (&s)[8]) {
  uint4 a = reinterpret_cast<const uint4*>(p)[0];
  uint4 b = reinterpret_cast<const uint4*>(p)[1];
  s[0] = a.x; s[1] = a.y; s[2] = a.z; s[3] = a.w;
  s[4] = b.x; s[5] = b.y; s[6] = b.z; s[7] = b.w;
}

// pass 1: per-MSM bucket histogram
template <int CB>
__global__ __launch_bounds__(256) void k_msm_count(const uint32_t* __restrict__ scalars, uint32_t n, size_t stride_words,
                                                   const uint8_t* __restrict__ inf, uint32_t* __restrict__ counts,
                                                   uint32_t point_base, uint32_t point_stride) {
  constexpr int W = Win<CB>::W;
  constexpr uint32_t NB = Win<CB>::NB;
  __shared__ uint32_t hist[NB];
  const uint32_t b = blockIdx.y;
  for (uint32_t k = threadIdx.x; k < NB; k += blockDim.x) hist[k] = 0;
  __syncthreads();
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && !inf[point_base + b * point_stride + i]) {
    uint32_t s[8];
    load_scalar(scalars + b * stride_words + (size_t)i * 8, s);
    uint32_t carry = 0;
#pragma unroll
    for (int w = 0; w < W; w++) {
      int d = digit_at<CB>(s, w, carry);
      if (d != 0) atomicAdd(&hist[(d < 0 ? -d : d) - 1], 1u);
    }
  }
  __syncthreads();
  for (uint32_t k = threadIdx.x; k < NB; k += blockDim.x) {
    uint32_t h = hist[k];
    if (h) atomicAdd(&counts[(size_t)b * NB + k], h);
  }
}

// pass 2: exclusive scan of the histogram -> offsets[b][0..NB], cursors
__global__ __launch_bounds__(256) void k_msm_scan(const uint32_t* __restrict__ counts, uint32_t* __restrict__ offsets,
                                                  uint32_t* __restrict__ cursors, uint32_t nb) {
  __shared__ uint32_t part[256];
  const uint32_t b = blockIdx.x;
  const uint32_t t = threadIdx.x;
  const uint32_t per = nb / 256;  // nb is a multiple of 256
  const uint32_t* cnt = counts + (size_t)b * nb;
  uint32_t local = 0;
  for (uint32_t j = 0; j < per; j++) local += cnt[t * per + j];
  part[t] = local;
  __syncthreads();
  for (uint32_t d = 1; d < 256; d <<= 1) {
    uint32_t v = (t >= d) ? part[t - d] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  uint32_t run = part[t] - local;  // exclusive prefix
  uint32_t* off = offsets + (size_t)b * (nb + 1);
  uint32_t* cur = cursors + (size_t)b * nb;
  for (uint32_t j = 0; j < per; j++) {
    off[t * per + j] = run;
    cur[t * per + j] = run;
    run += cnt[t * per + j];
  }
  if (t == 255) off[nb] = run;
}

// pass 3: scatter (table index | sign) entries into bucket order
template <int CB>
__global__ __launch_bounds__(256) void k_msm_scatter(const uint32_t* __restrict__ scalars, uint32_t n,
                                                     size_t stride_words, const uint8_t* __restrict__ inf,
                                                     uint32_t* __restrict__ cursors, uint32_t* __restrict__ entries,
                                                     size_t emax, uint32_t n_srs, uint32_t point_base,
                                                     uint32_t point_stride) {
  constexpr int W = Win<CB>::W;
  constexpr uint32_t NB = Win<CB>::NB;
  __shared__ uint32_t lcount[NB];
  __shared__ uint32_t lbase[NB];
  const uint32_t b = blockIdx.y;
  for (uint32_t k = threadIdx.x; k < NB; k += blockDim.x) lcount[k] = 0;
  __syncthreads();
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  int dig[W];
  uint32_t rank[W];
  const uint32_t ig = point_base + b * point_stride + i;  // SRS index of this scalar
  const bool live = i < n && !inf[ig];
  if (live) {
    uint32_t s[8];
    load_scalar(scalars + b * stride_words + (size_t)i * 8, s);
    uint32_t carry = 0;
#pragma unroll
    for (int w = 0; w < W; w++) {
      int d = digit_at<CB>(s, w, carry);
      dig[w] = d;
      rank[w] = d != 0 ? atomicAdd(&lcount[(d < 0 ? -d : d) - 1], 1u) : 0u;
    }
  }
  __syncthreads();
  for (uint32_t k = threadIdx.x; k < NB; k += blockDim.x) {
    uint32_t h = lcount[k];
    lbase[k] = h ? atomicAdd(&cursors[(size_t)b * NB + k], h) : 0u;
  }
  __syncthreads();
  if (live) {
    uint32_t* out = entries + b * emax;
#pragma unroll
    for (int w = 0; w < W; w++) {
      int d = dig[w];
      if (d != 0) {
        uint32_t k = (uint32_t)((d < 0 ? -d : d) - 1);
        out[lbase[k] + rank[w]] = ((uint32_t)w * n_srs + ig) | (d < 0 ? 0x80000000u : 0u);
      }
    }
  }
}

// pass 4: balanced bucket accumulation, K entries per thread
constexpr uint32_t NO_TAIL = 0xffffffffu;

template <class C>
__global__ __launch_bounds__(256, KZGX_ACCUM_WAVES) void k_msm_accum(const uint32_t* __restrict__ entries, size_t emax,
                                                   const uint32_t* __restrict__ offsets, uint32_t nb,
                                                   const uint32_t* __restrict__ table, uint32_t K, size_t smax,
                                                   uint32_t* __restrict__ bsum, uint32_t* __restrict__ heads,
                                                   uint32_t* __restrict__ tails, uint32_t* __restrict__ tailk) {
  constexpr int PW = affine_words<C>();
  constexpr int XW = xyzz_words<C>();
  const uint32_t b = blockIdx.y;
  const uint32_t seg = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t* off = offsets + (size_t)b * (nb + 1);
  const uint32_t E = off[nb];
  const uint32_t start = seg * K;
  if (start >= E) return;
  const uint32_t end = min(start + K, E);
  // bucket k with off[k] <= start < off[k+1]
  uint32_t lo = 0, hi = nb;  // invariant off[lo] <= start < off[hi]
  while (hi - lo > 1) {
    uint32_t mid = (lo + hi) >> 1;
    if (off[mid] <= start)
      lo = mid;
    else
      hi = mid;
  }
  uint32_t k = lo;
  uint32_t next = off[k + 1];
  bool before = off[k] < start;
  const uint32_t* ent = entries + b * emax;
  Xyzz<C> acc = xyzz_inf<C>();
  for (uint32_t p = start; p < end; ++p) {
    if (p == next) {
      // bucket k ended inside this segment
      uint32_t* dst = before ? heads + ((size_t)b * smax + seg) * XW : bsum + ((size_t)b * nb + k) * XW;
      xyzz_store<C>(dst, acc);
      acc = xyzz_inf<C>();
      before = false;
      do {
        k++;
        next = off[k + 1];
      } while (next == p);
    }
    const uint32_t e = ent[p];
    Affine<C> a = affine_load<C>(table + (size_t)(e & 0x7fffffffu) * PW);
    if (e >> 31) a = affine_neg<C>(a);
    acc = xyzz_add_affine_impl<C>(acc, a);
  }
  uint32_t* dst;
  uint32_t tk = NO_TAIL;
  if (before) {
    dst = heads + ((size_t)b * smax + seg) * XW;
  } else if (next > end) {
    dst = tails + ((size_t)b * smax + seg) * XW;
    tk = k;
  } else {
    dst = bsum + ((size_t)b * nb + k) * XW;
  }
  xyzz_store<C>(dst, acc);
  tailk[(size_t)b * smax + seg] = tk;
}

// pass 4b: buckets that straddle segments.  The segment holding the start
// of such a bucket stored its partial as a tail (tailk = bucket); the later
// segments of the bucket stored heads.  One thread per segment with a tail
// sums tail + heads into bsum, so the bucket pass below is branch-free.
template <class C>
__global__ __launch_bounds__(256) void k_msm_fixup(const uint32_t* __restrict__ offsets, uint32_t nb, uint32_t K,
                                                   size_t smax, const uint32_t* __restrict__ heads,
                                                   const uint32_t* __restrict__ tails,
                                                   const uint32_t* __restrict__ tailk, uint32_t* __restrict__ bsum) {
  constexpr int XW = xyzz_words<C>();
  const uint32_t b = blockIdx.y;
  const uint32_t seg = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t* off = offsets + (size_t)b * (nb + 1);
  if ((size_t)seg * K >= off[nb]) return;
  const uint32_t k = tailk[(size_t)b * smax + seg];
  if (k == NO_TAIL) return;
  const uint32_t e1 = off[k + 1];
  Xyzz<C> acc = xyzz_load<C>(tails + ((size_t)b * smax + seg) * XW);
  for (uint32_t s = seg + 1; (size_t)s * K < e1; s++) acc = xyzz_add<C>(acc, xyzz_load<C>(heads + ((size_t)b * smax + s) * XW));
  xyzz_store<C>(bsum + ((size_t)b * nb + k) * XW, acc);
}

// pass 5a: finish the buckets and their first-level weighted sums.
// Thread t of MSM b owns buckets [t J, t J + J) (J = RED_J) and emits
//   R_t = sum_j (j+1) B_{tJ+j}   and   T_t = sum_j B_{tJ+j}
// so that sum_k (k+1) B_k = sum_t R_t + J sum_t t T_t.
constexpr uint32_t RED_J = 8;

template <class C>
__global__ __launch_bounds__(256, KZGX_BS_WAVES) void k_msm_bucket_sums(const uint32_t* __restrict__ offsets, uint32_t nb,
                                                                        const uint32_t* __restrict__ bsum,
                                                                        uint32_t* __restrict__ rt) {
  constexpr int XW = xyzz_words<C>();
  const uint32_t b = blockIdx.y;
  const uint32_t T1 = nb / RED_J;
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= T1) return;
  const uint32_t* off = offsets + (size_t)b * (nb + 1) + t * RED_J;
  const uint32_t* src = bsum + ((size_t)b * nb + t * RED_J) * XW;
  Xyzz<C> run = xyzz_inf<C>(), sum = xyzz_inf<C>();
  for (int j = (int)RED_J - 1; j >= 0; j--) {
    Xyzz<C> bk = xyzz_inf<C>();
    if (off[j + 1] > off[j]) bk = xyzz_load<C>(src + (size_t)j * XW);  // empty buckets were never written
    run = xyzz_add_impl<C>(run, bk);
    sum = xyzz_add_impl<C>(sum, run);
  }
  uint32_t* dst = rt + ((size_t)b * T1 + t) * 2 * XW;
  xyzz_store<C>(dst, sum);
  xyzz_store<C>(dst + XW, run);
}

// pass 5b: fold the T1 (R_t, T_t) pairs of every MSM to its value
//   V = sum_t R_t + s sum_t t T_t        (s = RED_J initially)
// 8:1 per level: group g = {8g .. 8g+7} becomes
//   R'_g = sum_i R_{8g+i} + s sum_i i T_{8g+i},   T'_g = sum_i T_{8g+i},
// with s' = 8 s, which preserves V.  A 256-thread block folds 2048 / T1
// MSMs in place in rt; at every level the live groups of all its MSMs are
// packed onto the lowest threads so the shrinking levels occupy one
// wavefront instead of one per MSM.  The thread of the last group converts
// the MSM value to canonical affine (or stores the XYZZ point to xyzz_out
// for chunked single MSMs, summed by k_xyzz_sum).
template <class C>
__global__ __launch_bounds__(256) void k_msm_fold(uint32_t* __restrict__ rt, uint32_t T1, uint32_t batch,
                                                  uint32_t* __restrict__ out, uint32_t* __restrict__ out_inf,
                                                  uint32_t* __restrict__ xyzz_out) {
  constexpr int XW = xyzz_words<C>();
  const uint32_t mpb = 2048u / T1;  // MSMs per block (T1 in [64, 512])
  const uint32_t tid = threadIdx.x;
  uint32_t cnt = T1, stride = 1, s = RED_J;
  while (cnt > 1) {
    const uint32_t G = cnt >= 8 ? 8 : cnt;
    const uint32_t groups = cnt / G;
    if (tid < groups * mpb) {
      const uint32_t b = blockIdx.x * mpb + tid / groups;
      const uint32_t g = tid % groups;
      if (b < batch) {
        uint32_t* base = rt + ((size_t)b * T1 + (size_t)g * G * stride) * 2 * XW;
        const size_t step = (size_t)stride * 2 * XW;
        Xyzz<C> u = xyzz_inf<C>(), v = xyzz_inf<C>(), r = xyzz_inf<C>();
        for (int i = (int)G - 1; i >= 1; i--) {
          u = xyzz_add<C>(u, xyzz_load<C>(base + i * step + XW));
          v = xyzz_add<C>(v, u);  // v = sum_i i T_i
          r = xyzz_add<C>(r, xyzz_load<C>(base + i * step));
        }
        for (uint32_t m = s; m > 1; m >>= 1) v = xyzz_dbl<C>(v);
        r = xyzz_add<C>(r, xyzz_load<C>(base));
        const Xyzz<C> R = xyzz_add<C>(r, v);
        if (groups > 1) {
          xyzz_store<C>(base, R);
          xyzz_store<C>(base + XW, xyzz_add<C>(xyzz_load<C>(base + XW), u));
        } else if (xyzz_out) {
          xyzz_store<C>(xyzz_out + (size_t)b * XW, R);
        } else {
          Affine<C> a;
          const bool fin = xyzz_to_affine<C>(R, a);
          affine_to_canonical<C>(out + (size_t)b * 2 * C::Fp::N, a, fin);
          out_inf[b] = fin ? 0u : 1u;
        }
      }
    }
    __syncthreads();
    cnt = groups;
    stride *= G;
    s *= G;
  }
}

// sum of count XYZZ points -> canonical affine (one 256-thread workgroup:
// strided per-thread sums, then an LDS tree)
template <class C>
__global__ __launch_bounds__(256) void k_xyzz_sum(const uint32_t* __restrict__ pts, uint32_t count,
                                                  uint32_t* __restrict__ out, uint32_t* __restrict__ out_inf) {
  constexpr int XW = xyzz_words<C>();
  extern __shared__ uint32_t lds[];
  const uint32_t t = threadIdx.x;
  Xyzz<C> acc = xyzz_inf<C>();
  for (uint32_t i = t; i < count; i += blockDim.x) acc = xyzz_add<C>(acc, xyzz_load<C>(pts + (size_t)i * XW));
  xyzz_store<C>(lds + t * XW, acc);
  __syncthreads();
  for (uint32_t h = blockDim.x / 2; h >= 1; h >>= 1) {
    if (t < h) {
      acc = xyzz_add<C>(acc, xyzz_load<C>(lds + (t + h) * XW));
      xyzz_store<C>(lds + t * XW, acc);
    }
    __syncthreads();
  }
  if (t == 0) {
    Affine<C> a;
    bool fin = xyzz_to_affine<C>(acc, a);
    affine_to_canonical<C>(out, a, fin);
    *out_inf = fin ? 0u : 1u;
  }
}

// --------------------------------------------------------------------------
// host side
// --------------------------------------------------------------------------
template <class C>
int srs_upload_impl(Ctx* ctx, const uint32_t* d_canon, size_t n) {
  const int W = ctx->W;
  const size_t pw = affine_words<C>() * sizeof(uint32_t);
  KZGX_TRY(dev_alloc(ctx, (void**)&ctx->d_table, (size_t)W * n * pw, &ctx->table_bytes));
  KZGX_TRY(dev_alloc(ctx, (void**)&ctx->d_inf, n, &ctx->inf_bytes));
  dim3 blk(256), grd((unsigned)((n + 255) / 256));
  hipLaunchKernelGGL(k_srs_to_mont<C>, grd, blk, 0, ctx->stream, d_canon, ctx->d_table, ctx->d_inf, (uint32_t)n);
  hipLaunchKernelGGL(k_table_build<C>, grd, blk, 0, ctx->stream, ctx->d_table, ctx->d_inf, (uint32_t)n, W, ctx->c);
  KZGX_TRY_HIP(hipGetLastError());
  ctx->n_srs = n;
  return fixed_build(ctx, d_canon, n);
}

template <class C, int CB>
int msm_batch_impl(Ctx* ctx, const uint32_t* d_scalars, size_t n, size_t batch, size_t stride_words, uint32_t* d_out,
                   uint32_t* d_out_inf, hipStream_t st, uint32_t point_base, uint32_t point_stride,
                   uint32_t* xyzz_out) {
  constexpr int W = Win<CB>::W;
  constexpr uint32_t NB = Win<CB>::NB;
  const uint32_t K = ctx->seg_k;
  const size_t emax = (size_t)n * W;
  const size_t smax = (emax + K - 1) / K;
  const size_t XB = xyzz_words<C>() * sizeof(uint32_t);
  MsmWs* wsp = ctx->ws_for(st);
  if (!wsp) return KZGX_ERR_ARG;  // too many concurrent streams on one context
  MsmWs& ws = *wsp;
  KZGX_TRY(dev_alloc(ctx, (void**)&ws.counts, batch * NB * 4, &ws.counts_b));
  KZGX_TRY(dev_alloc(ctx, (void**)&ws.offsets, batch * (NB + 1) * 4, &ws.offsets_b));
  KZGX_TRY(dev_alloc(ctx, (void**)&ws.cursors, batch * NB * 4, &ws.cursors_b));
  KZGX_TRY(dev_alloc(ctx, (void**)&ws.entries, batch * emax * 4, &ws.entries_b));
  KZGX_TRY(dev_alloc(ctx, (void**)&ws.bsum, batch * NB * XB, &ws.bsum_b));
  KZGX_TRY(dev_alloc(ctx, (void**)&ws.heads, batch * smax * XB, &ws.heads_b));
  KZGX_TRY(dev_alloc(ctx, (void**)&ws.tails, batch * smax * XB, &ws.tails_b));
  KZGX_TRY(dev_alloc(ctx, (void**)&ws.tailk, batch * smax * 4, &ws.tailk_b));
  KZGX_TRY(dev_alloc(ctx, (void**)&ws.rt, batch * (NB / RED_J) * 2 * XB, &ws.rt_b));
  KZGX_TRY_HIP(hipMemsetAsync(ws.counts, 0, batch * NB * 4, st));
  dim3 blk(256);
  dim3 gs((unsigned)((n + 255) / 256), (unsigned)batch);
  {
    ProfScope p(ctx, st, "msm_count");
    hipLaunchKernelGGL(k_msm_count<CB>, gs, blk, 0, st, d_scalars, (uint32_t)n, stride_words, ctx->d_inf, ws.counts,
                       point_base, point_stride);
  }
  {
    ProfScope p(ctx, st, "msm_scan");
    hipLaunchKernelGGL(k_msm_scan, dim3((unsigned)batch), blk, 0, st, ws.counts, ws.offsets, ws.cursors, NB);
  }
  {
    ProfScope p(ctx, st, "msm_scatter");
    hipLaunchKernelGGL(k_msm_scatter<CB>, gs, blk, 0, st, d_scalars, (uint32_t)n, stride_words, ctx->d_inf,
                       ws.cursors, ws.entries, emax, (uint32_t)ctx->n_srs, point_base, point_stride);
  }
  {
    ProfScope p(ctx, st, "msm_accum");
    dim3 ga((unsigned)((smax + 255) / 256), (unsigned)batch);
    hipLaunchKernelGGL(k_msm_accum<C>, ga, blk, 0, st, ws.entries, emax, ws.offsets, NB, ctx->d_table, K, smax,
                       ws.bsum, ws.heads, ws.tails, ws.tailk);
  }
  {
    ProfScope p(ctx, st, "msm_reduce");
    const uint32_t T1 = NB / RED_J;
    static_assert(NB / RED_J >= 64 && NB / RED_J <= 512, "k_msm_fold packs 2048 / T1 MSMs per block");
    hipLaunchKernelGGL(k_msm_fixup<C>, dim3((unsigned)((smax + 255) / 256), (unsigned)batch), blk, 0, st, ws.offsets,
                       NB, K, smax, ws.heads, ws.tails, ws.tailk, ws.bsum);
    hipLaunchKernelGGL(k_msm_bucket_sums<C>, dim3((T1 + 255) / 256, (unsigned)batch), blk, 0, st, ws.offsets, NB,
                       ws.bsum, ws.rt);
    const uint32_t mpb = 2048u / T1;
    hipLaunchKernelGGL(k_msm_fold<C>, dim3((unsigned)((batch + mpb - 1) / mpb)), blk, 0, st, ws.rt, T1,
                       (uint32_t)batch, d_out, d_out_inf, xyzz_out);
  }
  KZGX_TRY_HIP(hipGetLastError());
  return KZGX_OK;
}

int srs_upload(Ctx* ctx, const uint32_t* d_canon, size_t n) {
  return ctx->curve == KZGX_CURVE_BN254 ? srs_upload_impl<BN254G1>(ctx, d_canon, n)
                                        : srs_upload_impl<BLS12381G1>(ctx, d_canon, n);
}

template <class C>
static int msm_batch_c(Ctx* ctx, const uint32_t* d_scalars, size_t n, size_t batch, size_t stride_words,
                       uint32_t* d_out, uint32_t* d_out_inf, hipStream_t st, uint32_t point_base,
                       uint32_t point_stride, uint32_t* xyzz_out) {
  switch (ctx->c) {
    case 10: return msm_batch_impl<C, 10>(ctx, d_scalars, n, batch, stride_words, d_out, d_out_inf, st, point_base, point_stride, xyzz_out);
    case 11: return msm_batch_impl<C, 11>(ctx, d_scalars, n, batch, stride_words, d_out, d_out_inf, st, point_base, point_stride, xyzz_out);
    case 12: return msm_batch_impl<C, 12>(ctx, d_scalars, n, batch, stride_words, d_out, d_out_inf, st, point_base, point_stride, xyzz_out);
    case 13: return msm_batch_impl<C, 13>(ctx, d_scalars, n, batch, stride_words, d_out, d_out_inf, st, point_base, point_stride, xyzz_out);
    default: return KZGX_ERR_INTERNAL;
  }
}

bool window_bits_supported(int c) { return c >= 10 && c <= 13; }

// One large MSM is cut into chunks of MSM_CHUNK points that run as a batch
// of independent MSMs over consecutive SRS ranges (point_stride), each
// reduced to an XYZZ partial, then summed by one workgroup.  Every chunk has
// the bucket occupancy the batched path is tuned for, so a degree-2^20
// commitment fills the chip instead of waiting on 2^(c-1) very long buckets.
constexpr size_t MSM_CHUNK = 4096;

template <class C>
static int msm_single_chunked(Ctx* ctx, const uint32_t* d_scalars, size_t n, uint32_t* d_out, uint32_t* d_out_inf,
                              hipStream_t st) {
  const size_t XB = xyzz_words<C>() * sizeof(uint32_t);
  const size_t full = n / MSM_CHUNK, rest = n % MSM_CHUNK;
  const size_t parts = full + (rest ? 1 : 0);
  MsmWs* ws = ctx->ws_for(st);
  if (!ws) return KZGX_ERR_ARG;
  KZGX_TRY(dev_alloc(ctx, (void**)&ws->parts, parts * XB, &ws->parts_b));
  uint32_t* parts_buf = ws->parts;
  if (full)
    KZGX_TRY(msm_batch_c<C>(ctx, d_scalars, MSM_CHUNK, full, MSM_CHUNK * 8, d_out, d_out_inf, st, 0, MSM_CHUNK,
                            parts_buf));
  if (rest) {
    // the tail chunk: a batch of one over SRS points [full * CHUNK, n)
    KZGX_TRY(msm_batch_c<C>(ctx, d_scalars + full * MSM_CHUNK * 8, rest, 1, rest * 8, d_out, d_out_inf, st,
                            (uint32_t)(full * MSM_CHUNK), 0, parts_buf + full * xyzz_words<C>()));
  }
  {
    ProfScope p(ctx, st, "msm_reduce");
    hipLaunchKernelGGL(k_xyzz_sum<C>, dim3(1), dim3(256), 256 * XB, st, parts_buf, (uint32_t)parts, d_out, d_out_inf);
  }
  KZGX_TRY_HIP(hipGetLastError());
  return KZGX_OK;
}

int xyzz_sum(Ctx* ctx, const uint32_t* d_parts, size_t count, uint32_t* d_out, uint32_t* d_out_inf, hipStream_t st) {
  if (ctx->curve == KZGX_CURVE_BN254)
    hipLaunchKernelGGL(k_xyzz_sum<BN254G1>, dim3(1), dim3(256), 256 * xyzz_words<BN254G1>() * 4, st, d_parts,
                       (uint32_t)count, d_out, d_out_inf);
  else
    hipLaunchKernelGGL(k_xyzz_sum<BLS12381G1>, dim3(1), dim3(256), 256 * xyzz_words<BLS12381G1>() * 4, st, d_parts,
                       (uint32_t)count, d_out, d_out_inf);
  KZGX_TRY_HIP(hipGetLastError());
  return KZGX_OK;
}

int msm_batch(Ctx* ctx, const uint32_t* d_scalars, size_t n, size_t batch, size_t stride_words, uint32_t* d_out,
              uint32_t* d_out_inf, hipStream_t st) {
  const bool bn = ctx->curve == KZGX_CURVE_BN254;
  if (fixed_usable(ctx, n)) return fixed_msm(ctx, d_scalars, n, batch, stride_words, d_out, d_out_inf, st, nullptr);
  if (batch == 1 && n >= 4 * MSM_CHUNK)
    return bn ? msm_single_chunked<BN254G1>(ctx, d_scalars, n, d_out, d_out_inf, st)
              : msm_single_chunked<BLS12381G1>(ctx, d_scalars, n, d_out, d_out_inf, st);
  return bn ? msm_batch_c<BN254G1>(ctx, d_scalars, n, batch, stride_words, d_out, d_out_inf, st, 0, 0, nullptr)
            : msm_batch_c<BLS12381G1>(ctx, d_scalars, n, batch, stride_words, d_out, d_out_inf, st, 0, 0, nullptr);
}

}  // namespace kzgx
