// Pass 4a of the batched Pippenger MSM (msm.hip): the merge of bucket
// partials that cross accumulation segments.  A header so
// scripts/repro_merge.hip can run the very kernel on synthetic segment
// layouts with the addition inlined or called.
#pragma once
#include <hip/hip_runtime.h>

#include "curve.hpp"

namespace kzgx {

constexpr uint32_t NO_TAIL = 0xffffffffu;
constexpr uint32_t ACC_WG = 128;  // segments per merge workgroup
constexpr uint8_t HEAD = 1, SPANS = 2;

// pass 4a: merge the partials of buckets that cross segments, one workgroup
// per ACC_WG consecutive segments with their heads staged in LDS.  A head
// chain is the run of heads that continues one bucket: the tail's owner (or
// thread 0, for the bucket already open at the workgroup start) adds them.
// Short chains (the usual case: buckets shorter than K) are walked
// sequentially; if any chain is 8 or more segments long (a skewed bucket
// such as the top window's small digits, or a small K) the workgroup merges
// by a segmented suffix scan over LDS in 7 steps.  The additions here are
// calls (xyzz_add), not the inlined form: with xyzz_add_impl inlined, the
// ROCm 7.2 compiler's si-form-memory-clauses pass makes the register
// allocator drop the copies of the upper 8 bytes of each 16-byte tail load
// at the entry of the sequential walk, so the walk starts from a corrupted
// point (scripts/repro_merge.hip + scripts/merge_bisect.sh,
// profiles/r03_merge_bisect.txt).  -mllvm
// -amdgpu-max-memory-clause=1 makes the inlined form exact and 0-30% faster,
// but the merge is 3% of a Pippenger launch, so the call form stays.
// Only buckets that cross a
// workgroup boundary leave: its leading chain -> ghead (gflag HEAD, SPANS if
// the bucket runs past the workgroup), its trailing tail -> gtail / gtailk,
// merged by k_msm_wg_fixup.
template <class C, bool INL>
KZGX_DEV Xyzz<C> merge_add(const Xyzz<C>& a, const Xyzz<C>& b) {
  if constexpr (INL) return xyzz_add_impl<C>(a, b);
  else return xyzz_add<C>(a, b);
}

#ifndef KZGX_MERGE_INLINE
#define KZGX_MERGE_INLINE 0
#endif
template <class C, bool INL = KZGX_MERGE_INLINE != 0>
__global__ __launch_bounds__(ACC_WG) void k_msm_merge(const uint32_t* __restrict__ heads,
                                                      const uint32_t* __restrict__ tails,
                                                      const uint32_t* __restrict__ tailk,
                                                      const uint8_t* __restrict__ sstate, uint32_t smax, uint32_t nb,
                                                      uint32_t nwg, uint32_t* __restrict__ bsum,
                                                      uint32_t* __restrict__ ghead, uint32_t* __restrict__ gtail,
                                                      uint32_t* __restrict__ gtailk, uint32_t* __restrict__ gflag) {
  constexpr int XW = xyzz_words<C>();
  __shared__ uint4 lds_head4[ACC_WG * XW / 4];
  __shared__ uint8_t lds_state[ACC_WG];
  __shared__ uint8_t lds_g[ACC_WG];
  uint32_t* lds_head = reinterpret_cast<uint32_t*>(lds_head4);
  const uint32_t b = blockIdx.y;
  const uint32_t t = threadIdx.x;
  const uint32_t seg = blockIdx.x * ACC_WG + t;
  const size_t gi = (size_t)b * nwg + blockIdx.x;
  const size_t si = (size_t)b * smax + seg;
  uint8_t state = 0;
  uint32_t k = NO_TAIL;
  if (seg < smax) {
    state = sstate[si];
    k = tailk[si];
  }
  const bool has_tail = k != NO_TAIL;
  if (state & HEAD) xyzz_store<C>(lds_head + t * XW, xyzz_load<C>(heads + si * XW));
  lds_state[t] = state;
  if (t == 0) gtailk[gi] = NO_TAIL;  // overwritten below by a crossing tail
  __syncthreads();
  // chain length (heads it sums, capped at 8) from head index u0
  auto chain_len = [&](uint32_t u0) {
    uint32_t c = 0;
    for (uint32_t u = u0; u < ACC_WG && c < 8; u++) {
      c++;
      if (!(lds_state[u] & SPANS)) break;
    }
    return c;
  };
  bool long_chain = false;
  if (has_tail && chain_len(t + 1) >= 8) long_chain = true;
  if (t == 0 && (state & HEAD) && chain_len(0) >= 8) long_chain = true;
#ifdef KZGX_MERGE_SEQ_ONLY
  long_chain = false;
#endif
  if (__syncthreads_or(long_chain)) {
    // y_u = sum of the heads u .. (chain end or workgroup end); g_u = the
    // chain runs past the workgroup.  Step D adds y_{u+D} while the chain
    // from u still continues past u + D - 1.
    uint8_t g = (state & SPANS) ? 1 : 0;
    lds_g[t] = g;
    Xyzz<C> y = xyzz_inf<C>();
    if (state & HEAD) y = xyzz_load<C>(lds_head + t * XW);
    __syncthreads();
#pragma unroll 1
    for (uint32_t D = 1; D < ACC_WG; D <<= 1) {
      const bool need = g && t + D < ACC_WG;
      Xyzz<C> o;
      uint8_t go = 0;
      if (need) {
        o = xyzz_load<C>(lds_head + (t + D) * XW);
        go = lds_g[t + D];
      }
      __syncthreads();
      if (need) {
        y = merge_add<C, INL>(y, o);
        g = go;
        xyzz_store<C>(lds_head + t * XW, y);
        lds_g[t] = g;
      }
      __syncthreads();
    }
    if (has_tail) {
      Xyzz<C> acc = xyzz_load<C>(tails + si * XW);
      bool past = true;
      if (t + 1 < ACC_WG) {
        acc = merge_add<C, INL>(acc, xyzz_load<C>(lds_head + (t + 1) * XW));
        past = lds_g[t + 1] != 0;
      }
      if (!past) {
        xyzz_store<C>(bsum + ((size_t)b * nb + k) * XW, acc);
      } else {
        xyzz_store<C>(gtail + gi * XW, acc);
        gtailk[gi] = k;
      }
    }
    if (t == 0) {
      uint32_t f = 0;
      if (state & HEAD) {
        f = HEAD | (lds_g[0] ? SPANS : 0);
        xyzz_store<C>(ghead + gi * XW, y);
      }
      gflag[gi] = f;
    }
    return;
  }
  if (has_tail) {
    // the next segment starts inside bucket k, so it holds a head
    Xyzz<C> acc = xyzz_load<C>(tails + si * XW);
    uint32_t u = t + 1;
    bool closed = false;
    for (; u < ACC_WG; u++) {
      acc = merge_add<C, INL>(acc, xyzz_load<C>(lds_head + u * XW));
      if (!(lds_state[u] & SPANS)) {
        closed = true;
        break;
      }
    }
    if (closed) {
      xyzz_store<C>(bsum + ((size_t)b * nb + k) * XW, acc);
    } else {
      xyzz_store<C>(gtail + gi * XW, acc);
      gtailk[gi] = k;
    }
  }
  if (t == 0) {
    uint32_t f = 0;
    if (state & HEAD) {
      Xyzz<C> h = xyzz_load<C>(lds_head);
      uint32_t u = 0;
      f = HEAD;
      while (lds_state[u] & SPANS) {
        if (u + 1 == ACC_WG) {
          f |= SPANS;
          break;
        }
        u++;
        h = merge_add<C, INL>(h, xyzz_load<C>(lds_head + u * XW));
      }
      xyzz_store<C>(ghead + gi * XW, h);
    }
    gflag[gi] = f;
  }
}

}  // namespace kzgx
