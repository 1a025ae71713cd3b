// k_msm_merge (csrc/msm_merge.hpp, pass 4a of the batched Pippenger MSM)
// run on synthetic segment layouts with the XYZZ addition inlined
// (xyzz_add_impl) and as a call (xyzz_add): both must write the same bits.
// VERDICT r02 item 6 / ADVICE r02: decide whether the failure of the inlined
// form is a compiler defect or a source-level ordering bug.
//
// The layouts follow k_msm_accum's rules exactly (msm.hip pass 4): random
// bucket sizes (most short, a few spanning many segments, some empty),
// segments of K entries, per segment the state (HEAD, SPANS) and the tail
// bucket; heads and tails are valid XYZZ points.  Variant outputs compared:
// bsum (buckets the merge closes), ghead, gtail, gtailk, gflag.
//
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -o scripts/mb/repro_merge scripts/repro_merge.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#pragma clang diagnostic ignored "-Wunused-result"
#pragma clang diagnostic ignored "-Wunused-value"

#include "../kzg-commitments_amd/csrc/msm_merge.hpp"

using namespace kzgx;

template <class C>
__global__ void k_make(uint32_t* pts, int n) {
  using F = typename C::Fp29;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Affine<C> g;
  g.x = f29_const<F>(C::GX29);
  g.y = f29_const<F>(C::GY29);
  Xyzz<C> acc = xyzz_from_affine<C>(g);
  for (int k = 0; k < (i % 61); k++) acc = xyzz_add_affine<C>(acc, g);
  acc = xyzz_dbl<C>(acc);  // ZZ != 1
  xyzz_store<C>(pts + (size_t)i * xyzz_words<C>(), acc);
}

// the sequential merge restated without LDS: one thread per tail segment walks
// the heads in global memory (the expected bsum of every bucket closed inside
// a workgroup)
template <class C, bool INL>
__global__ void k_expect(const uint32_t* heads, const uint32_t* tails, const uint32_t* tailk, const uint8_t* sstate,
                         uint32_t smax, uint32_t* bsum) {
  constexpr int XW = xyzz_words<C>();
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= smax || tailk[s] == NO_TAIL) return;
  const uint32_t wg_end = (s / ACC_WG + 1) * ACC_WG;
  Xyzz<C> acc = xyzz_load<C>(tails + (size_t)s * XW);
  for (uint32_t u = s + 1; u < wg_end && u < smax; u++) {
    acc = merge_add<C, INL>(acc, xyzz_load<C>(heads + (size_t)u * XW));
    if (!(sstate[u] & SPANS)) {
      xyzz_store<C>(bsum + (size_t)tailk[s] * XW, acc);
      return;
    }
  }
}

struct Layout {
  uint32_t smax, nwg, nb;
  std::vector<uint8_t> state;
  std::vector<uint32_t> tailk;
};

static uint64_t rng_state = 0x9E3779B97F4A7C15ull;
static uint32_t rnd() {
  rng_state ^= rng_state << 13;
  rng_state ^= rng_state >> 7;
  rng_state ^= rng_state << 17;
  return (uint32_t)(rng_state >> 11);
}

// k_msm_accum's segment bookkeeping on indices only
static Layout make_layout(uint32_t nb, uint32_t K, int mode) {
  std::vector<uint32_t> size(nb);
  for (uint32_t k = 0; k < nb; k++) {
    uint32_t r = rnd() % 1000;
    if (mode == 0) size[k] = r < 100 ? 0 : (r < 990 ? 1 + rnd() % (3 * K) : K * (8 + rnd() % 40));
    else if (mode == 1) size[k] = 1 + rnd() % (K + 3);
    else size[k] = r < 500 ? 0 : (r < 995 ? 1 + rnd() % 4 : K * (2 + rnd() % 300));
  }
  std::vector<uint32_t> off(nb + 1, 0);
  for (uint32_t k = 0; k < nb; k++) off[k + 1] = off[k] + size[k];
  const uint32_t E = off[nb];
  Layout L;
  L.nb = nb;
  L.smax = (E + K - 1) / K;
  L.nwg = (L.smax + ACC_WG - 1) / ACC_WG;
  L.state.assign(L.smax, 0);
  L.tailk.assign(L.smax, NO_TAIL);
  for (uint32_t s = 0; s < L.smax; s++) {
    const uint32_t start = s * K, end = start + K < E ? start + K : E;
    uint32_t k = 0;
    while (!(off[k] <= start && start < off[k + 1])) k++;
    uint32_t next = off[k + 1];
    bool before = off[k] < start;
    uint8_t state = 0;
    uint32_t tk = NO_TAIL;
    for (uint32_t p = start; p < end; p++) {
      if (p == next) {
        if (before) {
          state = HEAD;
          before = false;
        }
        do {
          k++;
          next = off[k + 1];
        } while (next == p);
      }
    }
    if (before) state = HEAD | (next > end ? SPANS : 0);
    else if (next > end) tk = k;
    L.state[s] = state;
    L.tailk[s] = tk;
  }
  return L;
}

template <class C>
static int run(const char* name, uint32_t K, int mode) {
  constexpr int XW = xyzz_words<C>();
  const uint32_t nb = 2048;
  Layout L = make_layout(nb, K, mode);
  const int npts = 4096;
  uint32_t *d_pool, *d_heads, *d_tails, *d_tailk, *d_bsum[2], *d_gpart[2], *d_gmeta[2];
  uint8_t* d_st;
  hipMalloc(&d_pool, (size_t)npts * XW * 4);
  hipLaunchKernelGGL(k_make<C>, dim3(npts / 64), dim3(64), 0, 0, d_pool, npts);
  std::vector<uint32_t> pool((size_t)npts * XW);
  hipMemcpy(pool.data(), d_pool, pool.size() * 4, hipMemcpyDeviceToHost);
  std::vector<uint32_t> heads((size_t)L.smax * XW, 0), tails((size_t)L.smax * XW, 0);
  for (uint32_t s = 0; s < L.smax; s++) {
    if (L.state[s] & HEAD) memcpy(&heads[(size_t)s * XW], &pool[(size_t)(rnd() % npts) * XW], XW * 4);
    if (L.tailk[s] != NO_TAIL) memcpy(&tails[(size_t)s * XW], &pool[(size_t)(rnd() % npts) * XW], XW * 4);
  }
  hipMalloc(&d_heads, heads.size() * 4);
  hipMalloc(&d_tails, tails.size() * 4);
  hipMalloc(&d_tailk, L.smax * 4);
  hipMalloc(&d_st, L.smax);
  hipMemcpy(d_heads, heads.data(), heads.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(d_tails, tails.data(), tails.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(d_tailk, L.tailk.data(), L.smax * 4, hipMemcpyHostToDevice);
  hipMemcpy(d_st, L.state.data(), L.smax, hipMemcpyHostToDevice);
  const size_t bs = (size_t)nb * XW, gp = (size_t)L.nwg * 2 * XW, gm = (size_t)L.nwg * 2;
  for (int v = 0; v < 2; v++) {
    hipMalloc(&d_bsum[v], bs * 4);
    hipMalloc(&d_gpart[v], gp * 4);
    hipMalloc(&d_gmeta[v], gm * 4);
    hipMemset(d_bsum[v], 0, bs * 4);
    hipMemset(d_gpart[v], 0, gp * 4);
    hipMemset(d_gmeta[v], 0, gm * 4);
  }
  float ms[2] = {0, 0};
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int rep = 0; rep < 2; rep++)  // second pass timed
  for (int v = 0; v < 2; v++) {
    hipEventRecord(e0, 0);
    uint32_t* ghead = d_gpart[v];
    uint32_t* gtail = d_gpart[v] + (size_t)L.nwg * XW;
    uint32_t* gtailk = d_gmeta[v];
    uint32_t* gflag = d_gmeta[v] + L.nwg;
    if (v == 0)
      hipLaunchKernelGGL((k_msm_merge<C, false>), dim3(L.nwg, 1), dim3(ACC_WG), 0, 0, d_heads, d_tails, d_tailk, d_st,
                         L.smax, nb, L.nwg, d_bsum[v], ghead, gtail, gtailk, gflag);
    else if (const char* co = getenv("REPRO_CO")) {
      // the inlined kernel from a separately built code object
      // (scripts/repro_merge_mod.hip, e.g. pass-limited)
      hipModule_t mod;
      hipFunction_t fn;
      if (hipModuleLoad(&mod, co) != hipSuccess ||
          hipModuleGetFunction(&fn, mod, "_ZN4kzgx11k_msm_mergeINS_7BN254G1ELb1EEEvPKjS3_S3_PKhjjjPjS6_S6_S6_S6_") !=
              hipSuccess) {
        printf("cannot load %s\n", co);
        exit(3);
      }
      uint32_t smax = L.smax, nbv = nb, nwg = L.nwg;
      void* args[] = {&d_heads, &d_tails, &d_tailk, &d_st, &smax, &nbv, &nwg, &d_bsum[v], &ghead, &gtail, &gtailk, &gflag};
      hipModuleLaunchKernel(fn, L.nwg, 1, 1, ACC_WG, 1, 1, 0, 0, args, nullptr);
    } else
      hipLaunchKernelGGL((k_msm_merge<C, true>), dim3(L.nwg, 1), dim3(ACC_WG), 0, 0, d_heads, d_tails, d_tailk, d_st,
                         L.smax, nb, L.nwg, d_bsum[v], ghead, gtail, gtailk, gflag);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms[v], e0, e1);
  }
  uint32_t *d_ex[2];
  for (int v = 0; v < 2; v++) {
    hipMalloc(&d_ex[v], bs * 4);
    hipMemset(d_ex[v], 0, bs * 4);
  }
  hipLaunchKernelGGL((k_expect<C, false>), dim3((L.smax + 63) / 64), dim3(64), 0, 0, d_heads, d_tails, d_tailk, d_st,
                     L.smax, d_ex[0]);
  hipLaunchKernelGGL((k_expect<C, true>), dim3((L.smax + 63) / 64), dim3(64), 0, 0, d_heads, d_tails, d_tailk, d_st,
                     L.smax, d_ex[1]);
  hipError_t e = hipDeviceSynchronize();
  std::vector<uint32_t> b0(bs), b1(bs), p0(gp), p1(gp), m0(gm), m1(gm), x0(bs), x1(bs);
  hipMemcpy(x0.data(), d_ex[0], bs * 4, hipMemcpyDeviceToHost);
  hipMemcpy(x1.data(), d_ex[1], bs * 4, hipMemcpyDeviceToHost);
  hipFree(d_ex[0]);
  hipFree(d_ex[1]);
  hipMemcpy(b0.data(), d_bsum[0], bs * 4, hipMemcpyDeviceToHost);
  hipMemcpy(b1.data(), d_bsum[1], bs * 4, hipMemcpyDeviceToHost);
  hipMemcpy(p0.data(), d_gpart[0], gp * 4, hipMemcpyDeviceToHost);
  hipMemcpy(p1.data(), d_gpart[1], gp * 4, hipMemcpyDeviceToHost);
  hipMemcpy(m0.data(), d_gmeta[0], gm * 4, hipMemcpyDeviceToHost);
  hipMemcpy(m1.data(), d_gmeta[1], gm * 4, hipMemcpyDeviceToHost);
  int bad_b = 0, bad_p = 0, bad_m = 0, first_b = -1;
  for (uint32_t k = 0; k < nb; k++)
    if (memcmp(&b0[(size_t)k * XW], &b1[(size_t)k * XW], XW * 4)) {
      bad_b++;
      if (first_b < 0) first_b = (int)k;
    }
  int call_vs_expect = 0, inl_vs_expect = 0, expect_inl_vs_call = 0;
  for (uint32_t k = 0; k < nb; k++) {
    call_vs_expect += memcmp(&b0[(size_t)k * XW], &x0[(size_t)k * XW], XW * 4) != 0;
    inl_vs_expect += memcmp(&b1[(size_t)k * XW], &x0[(size_t)k * XW], XW * 4) != 0;
    expect_inl_vs_call += memcmp(&x1[(size_t)k * XW], &x0[(size_t)k * XW], XW * 4) != 0;
  }
  printf("{\"call_merge_vs_expected\": %d, \"inlined_merge_vs_expected\": %d, \"inlined_expected_vs_expected\": %d}\n",
         call_vs_expect, inl_vs_expect, expect_inl_vs_call);
  for (size_t i = 0; i < (size_t)L.nwg * 2; i++)
    if (memcmp(&p0[i * XW], &p1[i * XW], XW * 4)) bad_p++;
  for (size_t i = 0; i < gm; i++)
    if (m0[i] != m1[i]) bad_m++;
  int heads_n = 0, spans_n = 0, tails_n = 0;
  for (uint32_t s = 0; s < L.smax; s++) {
    heads_n += (L.state[s] & HEAD) != 0;
    spans_n += (L.state[s] & SPANS) != 0;
    tails_n += L.tailk[s] != NO_TAIL;
  }
  printf("{\"curve\": \"%s\", \"K\": %u, \"mode\": %d, \"segments\": %u, \"workgroups\": %u, \"heads\": %d, "
         "\"spans\": %d, \"tails\": %d, \"hip\": \"%s\", \"bsum_mismatch\": %d, \"first_bucket\": %d, "
         "\"gpart_mismatch\": %d, \"gmeta_mismatch\": %d, \"call_ms\": %.4f, \"inlined_ms\": %.4f}\n",
         name, K, mode, L.smax, L.nwg, heads_n, spans_n, tails_n, hipGetErrorString(e), bad_b, first_b, bad_p, bad_m, ms[0], ms[1]);
  fflush(stdout);
  hipFree(d_pool); hipFree(d_heads); hipFree(d_tails); hipFree(d_tailk); hipFree(d_st);
  for (int v = 0; v < 2; v++) {
    hipFree(d_bsum[v]);
    hipFree(d_gpart[v]);
    hipFree(d_gmeta[v]);
  }
  return bad_b || bad_p || bad_m;
}

int main() {
  int bad = 0;
#ifdef REPRO_FAST
  // one layout on one curve: the sequential path (mode 1), for bisection builds
  bad |= run<BN254G1>("BN254", 32, 1);
#else
  for (int mode = 0; mode < 3; mode++)
    for (uint32_t K : {8u, 32u, 128u}) {
      bad |= run<BN254G1>("BN254", K, mode);
      bad |= run<BLS12381G1>("BLS12381", K, mode);
    }
#endif
  return bad;
}
