// Group-cooperative XYZZ point operations: 8 lanes of a wave compute ONE
// addition (or doubling) together, one field product per lane per round.
//
// Why: a chain of dependent point additions run by a lone wave costs ~10 us
// per addition (its ~2400 VALU instructions issue one after another, most of
// them waiting on the previous one).  The tops of the bucket-reduction trees
// are such chains with lanes to spare.  An addition's 14 products form 4
// rounds of independent products, so 8 lanes finish it in 4 product
// latencies (~1/3 of the time), a doubling in 3.
//
// Contract: every lane of an aligned 8-lane group calls with the same
// operands (points replicated over the group) and gets the same result; `sc`
// is the group's LDS scratch of COOP_SLOTS * L words.  The operations are
// exactly xyzz_add_impl / xyzz_dbl_impl's (curve.hpp: same formulas, same
// value bounds), the products spread over the lanes; results are the same
// group elements (representatives may differ).  Exchange between rounds goes
// through LDS within the wave: a wave's LDS accesses complete in program
// order, and the fences (coop_fence) keep the compiler from reordering them.
#pragma once
#include "curve.hpp"

namespace kzgx {

constexpr int COOP_G = 8;       // lanes per group
constexpr int COOP_SLOTS = 40;  // 5 banks of 8 products

template <class F>
KZGX_DEV void f29_lds_st(uint32_t* p, const F29<F>& a) {
#pragma unroll
  for (int i = 0; i < F::L; i++) p[i] = a.v[i];
}
template <class F>
KZGX_DEV F29<F> f29_lds_ld(const uint32_t* p) {
  F29<F> a;
#pragma unroll
  for (int i = 0; i < F::L; i++) a.v[i] = p[i];
  return a;
}
// workgroup scope: an s_waitcnt on the LDS counter and a compiler barrier
// (a wavefront-scope fence lowers to nothing, and nothing then stops the
// scheduler from lifting the next round's LDS reads above this round's writes)
KZGX_DEV void coop_fence() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup"); }

template <class F>
KZGX_DEV F29<F> f29_sel(bool c, const F29<F>& a, const F29<F>& b) {
  F29<F> r;
#pragma unroll
  for (int i = 0; i < F::L; i++) r.v[i] = c ? a.v[i] : b.v[i];
  return r;
}

// 2P (dbl-2008-s-1 as xyzz_dbl_impl): round 1 V = U^2, xx = X^2 (U = 2Y);
// round 2 W = U V, S = X V, MM = M M, ZZ3 = V ZZ (M = 3 xx); round 3
// Y3 = M (S - X3) - W Y, ZZZ3 = W ZZZ (X3 = MM - 2S)
template <class C>
KZGX_DEV Xyzz<C> coop_dbl(const Xyzz<C>& p, uint32_t* sc, int j) {
  using F = typename C::Fp29;
  constexpr int L = F::L;
  if (xyzz_is_inf<C>(p)) return p;
  uint32_t* b1 = sc;
  uint32_t* b2 = sc + 8 * L;
  uint32_t* b3 = sc + 16 * L;
  const F29<F> U = f29_add<F>(p.Y, p.Y);  // < 8m
  f29_lds_st<F>(b1 + j * L, f29_sqr<F>(f29_sel<F>(j == 0, U, p.X)));
  coop_fence();
  const F29<F> V = f29_lds_ld<F>(b1);
  const F29<F> xx = f29_lds_ld<F>(b1 + L);
  const F29<F> M = f29_add<F>(f29_add<F>(xx, xx), xx);  // < 6m
  {
    const F29<F> A = j == 0 ? U : j == 1 ? p.X : j == 2 ? M : V;
    const F29<F> B = j <= 1 ? V : j == 2 ? M : p.ZZ;
    f29_lds_st<F>(b2 + j * L, f29_mul<F>(A, B));
  }
  coop_fence();
  const F29<F> W = f29_lds_ld<F>(b2);
  const F29<F> S = f29_lds_ld<F>(b2 + L);
  const F29<F> X3 = f29_sub<F>(f29_lds_ld<F>(b2 + 2 * L), f29_add<F>(S, S), F::P4);  // < 6m
  {
    const F29<F> A = f29_sel<F>(j == 0, M, W);
    const F29<F> B = f29_sel<F>(j == 0, f29_sub<F>(S, X3, F::P8), p.ZZZ);
    const F29<F> Cc = f29_sel<F>(j == 0, W, f29_zero<F>());
    const F29<F> D = f29_sel<F>(j == 0, f29_sub<F>(f29_zero<F>(), p.Y, F::P4), f29_zero<F>());
    f29_lds_st<F>(b3 + j * L, f29_mul2<F>(A, B, Cc, D));  // Y3 < 2m; ZZZ3 < 2m
  }
  coop_fence();
  Xyzz<C> r;
  r.X = X3;
  r.Y = f29_lds_ld<F>(b3);
  r.ZZ = f29_lds_ld<F>(b2 + 3 * L);
  r.ZZZ = f29_lds_ld<F>(b3 + L);
  coop_fence();  // the scratch is reused by the group's next operation
  return r;
}

// P + Q (add-2008-s as xyzz_add_impl): round 1 U1, U2, S1, S2, ZZ1 ZZ2,
// ZZZ1 ZZZ2; round 2 PP = P^2, RR = R^2 (P = U2 - U1, R = S2 - S1); round 3
// PPP = P PP, Q = U1 PP, ZZ3 = ZZ12 PP; round 4 Y3 = R (Q - X3) - S1 PPP,
// ZZZ3 = ZZZ12 PPP (X3 = RR - PPP - 2Q)
template <class C>
KZGX_DEV Xyzz<C> coop_add(const Xyzz<C>& p, const Xyzz<C>& q, uint32_t* sc, int j) {
  using F = typename C::Fp29;
  constexpr int L = F::L;
  if (xyzz_is_inf<C>(p)) return q;
  if (xyzz_is_inf<C>(q)) return p;
  uint32_t* b1 = sc;
  uint32_t* b2 = sc + 8 * L;
  uint32_t* b3 = sc + 16 * L;
  uint32_t* b4 = sc + 24 * L;
  uint32_t* bx = sc + 32 * L;
  {
    const F29<F> A = j == 0 ? p.X : j == 1 ? q.X : j == 2 ? p.Y : j == 3 ? q.Y : j == 4 ? p.ZZ : p.ZZZ;
    const F29<F> B = j == 0 ? q.ZZ : j == 1 ? p.ZZ : j == 2 ? q.ZZZ : j == 3 ? p.ZZZ : j == 4 ? q.ZZ : q.ZZZ;
    f29_lds_st<F>(b1 + j * L, f29_mul<F>(A, B));
  }
  coop_fence();
  {
    const int ia = (j & 1) ? 3 : 1;  // lane 0: P = U2 - U1, lane 1: R = S2 - S1
    const F29<F> x = f29_sub<F>(f29_lds_ld<F>(b1 + ia * L), f29_lds_ld<F>(b1 + (ia - 1) * L), F::P2);  // < 4m
    f29_lds_st<F>(bx + j * L, x);
    f29_lds_st<F>(b2 + j * L, f29_sqr<F>(x));
  }
  coop_fence();
  const F29<F> PP = f29_lds_ld<F>(b2);
  if (f29_is_zero_lt2m<F>(PP)) {  // equal x (uniform over the group): double or cancel
    coop_fence();
    if (f29_is_zero<F>(f29_lds_ld<F>(bx + L))) return coop_dbl<C>(p, sc, j);
    return xyzz_inf<C>();
  }
  {
    const F29<F> A = j == 0 ? f29_lds_ld<F>(bx) : f29_lds_ld<F>(b1 + (j == 1 ? 0 : 4) * L);
    f29_lds_st<F>(b3 + j * L, f29_mul<F>(A, PP));
  }
  coop_fence();
  const F29<F> PPP = f29_lds_ld<F>(b3);
  const F29<F> Q = f29_lds_ld<F>(b3 + L);
  const F29<F> X3 = f29_sub<F>(f29_lds_ld<F>(b2 + L), f29_add<F>(PPP, f29_add<F>(Q, Q)), F::P6);
  {
    const F29<F> A = j == 0 ? f29_lds_ld<F>(bx + L) : f29_lds_ld<F>(b1 + 5 * L);
    const F29<F> B = f29_sel<F>(j == 0, f29_sub<F>(Q, X3, F::P8), PPP);
    const F29<F> Cc = f29_sel<F>(j == 0, f29_sub<F>(f29_zero<F>(), f29_lds_ld<F>(b1 + 2 * L), F::P2), f29_zero<F>());
    const F29<F> D = f29_sel<F>(j == 0, PPP, f29_zero<F>());
    f29_lds_st<F>(b4 + j * L, f29_mul2<F>(A, B, Cc, D));  // Y3 < 2m; ZZZ3 < 2m
  }
  coop_fence();
  Xyzz<C> r;
  r.X = X3;
  r.Y = f29_lds_ld<F>(b4);
  r.ZZ = f29_lds_ld<F>(b3 + 2 * L);
  r.ZZZ = f29_lds_ld<F>(b4 + L);
  coop_fence();
  return r;
}

}  // namespace kzgx
