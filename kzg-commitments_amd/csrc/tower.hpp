// Extension-field tower and G2 arithmetic for the verify path on gfx950:
// Fp2 = Fp[i]/(i^2 + 1), Fp6 = Fp2[v]/(v^3 - xi), Fp12 = Fp6[w]/(w^2 - v),
// xi = 1 + i (both curves), over the radix-2^29 Montgomery Fp of
// field29.hpp.
//
// Replaces miracl-core's FP2 / FP4 / FP12 / ECP2 (un-vendored)
// behind trusted_setup::verify_proof, polyeval_G2 and the G2 half of the
// setup (src/trusted_setup.cpp:123-135, 176-201, 230-254).
//
// This is cold code (a handful of pairings per verify, one G2 MSM of N+1
// terms), so it trades speed for a simple invariant: every stored Fp value
// is < 2m.  Sums are reduced back below 2m with one conditional subtraction;
// products of two values < 2m are < 2m without one (field29.hpp).  Operations
// are real calls (__noinline__) to keep code size and compile time bounded.
#pragma once
#include "curve.hpp"

#define KZGX_TW __device__ __noinline__
// Fp2 products: inlined into their (non-inlined) Fp6 / G2 callers by
// default -- a call per Fp2 product costs more in argument copies and
// callee-saved spills than the product itself on single-lane pairing code
#ifndef KZGX_F2_NOINLINE
#define KZGX_TW2 __device__ __forceinline__
#else
#define KZGX_TW2 __device__ __noinline__
#endif

namespace kzgx {

template <class C>
struct PairOf;
template <>
struct PairOf<BN254G1> {
  using T = BN254Pair;
};
template <>
struct PairOf<BLS12381G1> {
  using T = BLS12381Pair;
};

// ---- Fp with the < 2m invariant ---------------------------------------------
template <class F>
KZGX_DEV F29<F> fp_add(const F29<F>& a, const F29<F>& b) {
  return f29_csub<F>(f29_add<F>(a, b), F::P2);
}
template <class F>
KZGX_DEV F29<F> fp_sub(const F29<F>& a, const F29<F>& b) {
  return f29_csub<F>(f29_sub<F>(a, b, F::P2), F::P2);  // a + 2m - b in (0, 4m)
}
template <class F>
KZGX_DEV F29<F> fp_neg(const F29<F>& a) {
  return fp_sub<F>(f29_zero<F>(), a);
}

// canonical little-endian words <-> Montgomery (< m)
template <class C>
KZGX_DEV F29<typename C::Fp29> fp_from_canon(const uint32_t* w) {
  using F = typename C::Fp29;
  constexpr int N = C::Fp::N;
  uint32_t t[N];
#pragma unroll
  for (int i = 0; i < N; i++) t[i] = w[i];
  return f29_reduce<F>(f29_to_mont<F>(f29_from_words<F, N>(t)));
}
template <class C>
KZGX_DEV void fp_to_canon(const F29<typename C::Fp29>& a, uint32_t* w) {
  using F = typename C::Fp29;
  constexpr int N = C::Fp::N;
  uint32_t t[N];
  f29_to_words<F, N>(f29_from_mont<F>(a), t);
#pragma unroll
  for (int i = 0; i < N; i++) w[i] = t[i];
}
// canonical words < m ?
template <class C>
KZGX_DEV bool canon_lt_m(const uint32_t* w) {
  constexpr int N = C::Fp::N;
  int cmp = 0;
  for (int i = N - 1; i >= 0 && cmp == 0; i--) cmp = w[i] < C::Fp::P[i] ? -1 : (w[i] > C::Fp::P[i] ? 1 : 0);
  return cmp < 0;
}

// ---- Fp2 ----------------------------------------------------------------------
template <class C>
struct Fp2 {
  F29<typename C::Fp29> a, b;  // a + b i
};

template <class C>
KZGX_DEV Fp2<C> f2_const(const uint32_t (&c)[2][C::Fp29::L]) {
  using F = typename C::Fp29;
  Fp2<C> r;
  r.a = f29_const<F>(c[0]);
  r.b = f29_const<F>(c[1]);
  return r;
}
template <class C>
KZGX_DEV Fp2<C> f2_zero() {
  using F = typename C::Fp29;
  return Fp2<C>{f29_zero<F>(), f29_zero<F>()};
}
template <class C>
KZGX_DEV Fp2<C> f2_one() {
  using F = typename C::Fp29;
  return Fp2<C>{f29_one<F>(), f29_zero<F>()};
}
template <class C>
KZGX_DEV Fp2<C> f2_add(const Fp2<C>& x, const Fp2<C>& y) {
  using F = typename C::Fp29;
  return Fp2<C>{fp_add<F>(x.a, y.a), fp_add<F>(x.b, y.b)};
}
template <class C>
KZGX_DEV Fp2<C> f2_sub(const Fp2<C>& x, const Fp2<C>& y) {
  using F = typename C::Fp29;
  return Fp2<C>{fp_sub<F>(x.a, y.a), fp_sub<F>(x.b, y.b)};
}
template <class C>
KZGX_DEV Fp2<C> f2_neg(const Fp2<C>& x) {
  using F = typename C::Fp29;
  return Fp2<C>{fp_neg<F>(x.a), fp_neg<F>(x.b)};
}
template <class C>
KZGX_DEV Fp2<C> f2_conj(const Fp2<C>& x) {
  using F = typename C::Fp29;
  return Fp2<C>{x.a, fp_neg<F>(x.b)};
}
template <class C>
KZGX_DEV Fp2<C> f2_dbl(const Fp2<C>& x) {
  return f2_add<C>(x, x);
}
template <class C>
KZGX_TW2 Fp2<C> f2_mul(const Fp2<C>& x, const Fp2<C>& y) {
  using F = typename C::Fp29;
  const F29<F> t0 = f29_mul<F>(x.a, y.a);
  const F29<F> t1 = f29_mul<F>(x.b, y.b);
  // (xa + xb)(ya + yb): operands < 4m, product < 16 m^2 -> < 2m
  const F29<F> t2 = f29_mul<F>(f29_add<F>(x.a, x.b), f29_add<F>(y.a, y.b));
  return Fp2<C>{fp_sub<F>(t0, t1), fp_sub<F>(fp_sub<F>(t2, t0), t1)};
}
template <class C>
KZGX_TW2 Fp2<C> f2_sqr(const Fp2<C>& x) {
  using F = typename C::Fp29;
  // (a + b)(a - b), 2 a b
  const F29<F> c0 = f29_mul<F>(f29_add<F>(x.a, x.b), fp_sub<F>(x.a, x.b));
  const F29<F> c1 = f29_mul<F>(f29_add<F>(x.a, x.a), x.b);
  return Fp2<C>{c0, c1};
}
template <class C>
KZGX_DEV Fp2<C> f2_mul_fp(const Fp2<C>& x, const F29<typename C::Fp29>& s) {
  using F = typename C::Fp29;
  return Fp2<C>{f29_mul<F>(x.a, s), f29_mul<F>(x.b, s)};
}
// x (1 + i)
template <class C>
KZGX_DEV Fp2<C> f2_mul_xi(const Fp2<C>& x) {
  using F = typename C::Fp29;
  return Fp2<C>{fp_sub<F>(x.a, x.b), fp_add<F>(x.a, x.b)};
}
template <class C>
KZGX_TW Fp2<C> f2_inv(const Fp2<C>& x) {
  using F = typename C::Fp29;
  const F29<F> t = fp_add<F>(f29_sqr<F>(x.a), f29_sqr<F>(x.b));
  const F29<F> ti = f29_inv_fast<F, C::Fp::N>(t, C::Fp::P, C::Fp::PM2);
  return Fp2<C>{f29_mul<F>(x.a, ti), fp_neg<F>(f29_mul<F>(x.b, ti))};
}
template <class C>
KZGX_DEV bool f2_is_zero(const Fp2<C>& x) {
  using F = typename C::Fp29;
  return f29_is_zero<F>(x.a) && f29_is_zero<F>(x.b);
}
template <class C>
KZGX_DEV Fp2<C> f2_from_canon(const uint32_t* w) {  // a words || b words
  return Fp2<C>{fp_from_canon<C>(w), fp_from_canon<C>(w + C::Fp::N)};
}
template <class C>
KZGX_DEV void f2_to_canon(const Fp2<C>& x, uint32_t* w) {
  fp_to_canon<C>(x.a, w);
  fp_to_canon<C>(x.b, w + C::Fp::N);
}

// ---- Fp6 ----------------------------------------------------------------------
template <class C>
struct Fp6 {
  Fp2<C> c0, c1, c2;
};
template <class C>
KZGX_DEV Fp6<C> f6_zero() {
  return Fp6<C>{f2_zero<C>(), f2_zero<C>(), f2_zero<C>()};
}
template <class C>
KZGX_DEV Fp6<C> f6_add(const Fp6<C>& x, const Fp6<C>& y) {
  return Fp6<C>{f2_add<C>(x.c0, y.c0), f2_add<C>(x.c1, y.c1), f2_add<C>(x.c2, y.c2)};
}
template <class C>
KZGX_DEV Fp6<C> f6_sub(const Fp6<C>& x, const Fp6<C>& y) {
  return Fp6<C>{f2_sub<C>(x.c0, y.c0), f2_sub<C>(x.c1, y.c1), f2_sub<C>(x.c2, y.c2)};
}
template <class C>
KZGX_DEV Fp6<C> f6_neg(const Fp6<C>& x) {
  return Fp6<C>{f2_neg<C>(x.c0), f2_neg<C>(x.c1), f2_neg<C>(x.c2)};
}
// x v  (v^3 = xi)
template <class C>
KZGX_DEV Fp6<C> f6_mul_v(const Fp6<C>& x) {
  return Fp6<C>{f2_mul_xi<C>(x.c2), x.c0, x.c1};
}
template <class C>
KZGX_TW Fp6<C> f6_mul(const Fp6<C>& a, const Fp6<C>& b) {
  const Fp2<C> t0 = f2_mul<C>(a.c0, b.c0);
  const Fp2<C> t1 = f2_mul<C>(a.c1, b.c1);
  const Fp2<C> t2 = f2_mul<C>(a.c2, b.c2);
  Fp6<C> r;
  r.c0 = f2_add<C>(
      t0, f2_mul_xi<C>(f2_sub<C>(f2_sub<C>(f2_mul<C>(f2_add<C>(a.c1, a.c2), f2_add<C>(b.c1, b.c2)), t1), t2)));
  r.c1 = f2_add<C>(f2_sub<C>(f2_sub<C>(f2_mul<C>(f2_add<C>(a.c0, a.c1), f2_add<C>(b.c0, b.c1)), t0), t1),
                   f2_mul_xi<C>(t2));
  r.c2 = f2_add<C>(f2_sub<C>(f2_sub<C>(f2_mul<C>(f2_add<C>(a.c0, a.c2), f2_add<C>(b.c0, b.c2)), t0), t2), t1);
  return r;
}
template <class C>
KZGX_TW Fp6<C> f6_inv(const Fp6<C>& a) {
  const Fp2<C> A = f2_sub<C>(f2_sqr<C>(a.c0), f2_mul_xi<C>(f2_mul<C>(a.c1, a.c2)));
  const Fp2<C> B = f2_sub<C>(f2_mul_xi<C>(f2_sqr<C>(a.c2)), f2_mul<C>(a.c0, a.c1));
  const Fp2<C> Cc = f2_sub<C>(f2_sqr<C>(a.c1), f2_mul<C>(a.c0, a.c2));
  const Fp2<C> F = f2_add<C>(f2_mul<C>(a.c0, A), f2_mul_xi<C>(f2_add<C>(f2_mul<C>(a.c2, B), f2_mul<C>(a.c1, Cc))));
  const Fp2<C> Fi = f2_inv<C>(F);
  return Fp6<C>{f2_mul<C>(A, Fi), f2_mul<C>(B, Fi), f2_mul<C>(Cc, Fi)};
}

// ---- Fp12 ---------------------------------------------------------------------
template <class C>
struct Fp12 {
  Fp6<C> c0, c1;  // c0 + c1 w
};
template <class C>
KZGX_DEV Fp12<C> f12_one() {
  Fp12<C> r;
  r.c0 = f6_zero<C>();
  r.c1 = f6_zero<C>();
  r.c0.c0 = f2_one<C>();
  return r;
}
template <class C>
KZGX_TW Fp12<C> f12_mul(const Fp12<C>& a, const Fp12<C>& b) {
  const Fp6<C> t0 = f6_mul<C>(a.c0, b.c0);
  const Fp6<C> t1 = f6_mul<C>(a.c1, b.c1);
  Fp12<C> r;
  r.c0 = f6_add<C>(t0, f6_mul_v<C>(t1));
  r.c1 = f6_sub<C>(f6_sub<C>(f6_mul<C>(f6_add<C>(a.c0, a.c1), f6_add<C>(b.c0, b.c1)), t0), t1);
  return r;
}
template <class C>
KZGX_TW Fp12<C> f12_sqr(const Fp12<C>& a) {
  // (a0 + a1 w)^2 = (a0 + a1)(a0 + v a1) - t - v t + 2 t w,  t = a0 a1
  const Fp6<C> t = f6_mul<C>(a.c0, a.c1);
  Fp12<C> r;
  r.c0 = f6_sub<C>(f6_sub<C>(f6_mul<C>(f6_add<C>(a.c0, a.c1), f6_add<C>(a.c0, f6_mul_v<C>(a.c1))), t),
                   f6_mul_v<C>(t));
  r.c1 = f6_add<C>(t, t);
  return r;
}
template <class C>
KZGX_DEV Fp12<C> f12_conj(const Fp12<C>& a) {
  return Fp12<C>{a.c0, f6_neg<C>(a.c1)};
}
template <class C>
KZGX_TW Fp12<C> f12_inv(const Fp12<C>& a) {
  const Fp6<C> t = f6_sub<C>(f6_mul<C>(a.c0, a.c0), f6_mul_v<C>(f6_mul<C>(a.c1, a.c1)));
  const Fp6<C> ti = f6_inv<C>(t);
  return Fp12<C>{f6_mul<C>(a.c0, ti), f6_neg<C>(f6_mul<C>(a.c1, ti))};
}
// a^p: the coefficient of w^k (k = 2 j + h for c_h.c_j) is conjugated and
// multiplied by xi^(k (p-1)/6)
template <class C>
KZGX_TW Fp12<C> f12_frob(const Fp12<C>& a) {
  using P = typename PairOf<C>::T;
  Fp12<C> r;
  r.c0.c0 = f2_mul<C>(f2_conj<C>(a.c0.c0), f2_const<C>(P::FROB[0]));
  r.c0.c1 = f2_mul<C>(f2_conj<C>(a.c0.c1), f2_const<C>(P::FROB[2]));
  r.c0.c2 = f2_mul<C>(f2_conj<C>(a.c0.c2), f2_const<C>(P::FROB[4]));
  r.c1.c0 = f2_mul<C>(f2_conj<C>(a.c1.c0), f2_const<C>(P::FROB[1]));
  r.c1.c1 = f2_mul<C>(f2_conj<C>(a.c1.c1), f2_const<C>(P::FROB[3]));
  r.c1.c2 = f2_mul<C>(f2_conj<C>(a.c1.c2), f2_const<C>(P::FROB[5]));
  return r;
}
// tower order: c0.c0, c0.c1, c0.c2, c1.c0, c1.c1, c1.c2, each (re, im)
template <class C>
KZGX_DEV void f12_to_canon(const Fp12<C>& a, uint32_t* w) {
  constexpr int N = C::Fp::N;
  f2_to_canon<C>(a.c0.c0, w + 0 * N);
  f2_to_canon<C>(a.c0.c1, w + 2 * N);
  f2_to_canon<C>(a.c0.c2, w + 4 * N);
  f2_to_canon<C>(a.c1.c0, w + 6 * N);
  f2_to_canon<C>(a.c1.c1, w + 8 * N);
  f2_to_canon<C>(a.c1.c2, w + 10 * N);
}

// ---- G2: twist points, Jacobian (x = X/Z^2, y = Y/Z^3), Z = 0 at infinity ----
template <class C>
struct G2A {
  Fp2<C> x, y;
};
template <class C>
struct G2J {
  Fp2<C> X, Y, Z;
};
template <class C>
KZGX_DEV G2J<C> g2_inf() {
  return G2J<C>{f2_one<C>(), f2_one<C>(), f2_zero<C>()};
}
template <class C>
KZGX_DEV bool g2_is_inf(const G2J<C>& p) {
  return f2_is_zero<C>(p.Z);
}
template <class C>
KZGX_DEV G2J<C> g2_from_affine(const G2A<C>& a) {
  return G2J<C>{a.x, a.y, f2_one<C>()};
}
// dbl-2009-l (a = 0)
template <class C>
KZGX_TW G2J<C> g2_dbl(const G2J<C>& p) {
  if (g2_is_inf<C>(p)) return p;
  const Fp2<C> A = f2_sqr<C>(p.X);
  const Fp2<C> B = f2_sqr<C>(p.Y);
  const Fp2<C> Cc = f2_sqr<C>(B);
  const Fp2<C> D = f2_dbl<C>(f2_sub<C>(f2_sub<C>(f2_sqr<C>(f2_add<C>(p.X, B)), A), Cc));
  const Fp2<C> E = f2_add<C>(f2_dbl<C>(A), A);
  G2J<C> r;
  r.X = f2_sub<C>(f2_sqr<C>(E), f2_dbl<C>(D));
  const Fp2<C> C8 = f2_dbl<C>(f2_dbl<C>(f2_dbl<C>(Cc)));
  r.Y = f2_sub<C>(f2_mul<C>(E, f2_sub<C>(D, r.X)), C8);
  r.Z = f2_dbl<C>(f2_mul<C>(p.Y, p.Z));
  return r;
}
// p + q, q affine (madd-2007-bl), complete over the special cases
template <class C>
KZGX_TW G2J<C> g2_add_mixed(const G2J<C>& p, const G2A<C>& q) {
  if (g2_is_inf<C>(p)) return g2_from_affine<C>(q);
  const Fp2<C> Z1Z1 = f2_sqr<C>(p.Z);
  const Fp2<C> U2 = f2_mul<C>(q.x, Z1Z1);
  const Fp2<C> S2 = f2_mul<C>(q.y, f2_mul<C>(p.Z, Z1Z1));
  const Fp2<C> H = f2_sub<C>(U2, p.X);
  const Fp2<C> rr = f2_dbl<C>(f2_sub<C>(S2, p.Y));
  if (f2_is_zero<C>(H)) {
    if (f2_is_zero<C>(rr)) return g2_dbl<C>(p);
    return g2_inf<C>();
  }
  const Fp2<C> HH = f2_sqr<C>(H);
  const Fp2<C> I = f2_dbl<C>(f2_dbl<C>(HH));
  const Fp2<C> J = f2_mul<C>(H, I);
  const Fp2<C> V = f2_mul<C>(p.X, I);
  G2J<C> r;
  r.X = f2_sub<C>(f2_sub<C>(f2_sqr<C>(rr), J), f2_dbl<C>(V));
  r.Y = f2_sub<C>(f2_mul<C>(rr, f2_sub<C>(V, r.X)), f2_dbl<C>(f2_mul<C>(p.Y, J)));
  r.Z = f2_sub<C>(f2_sub<C>(f2_sqr<C>(f2_add<C>(p.Z, H)), Z1Z1), HH);
  return r;
}
// p + q (add-2007-bl), complete over the special cases
template <class C>
KZGX_TW G2J<C> g2_add(const G2J<C>& p, const G2J<C>& q) {
  if (g2_is_inf<C>(p)) return q;
  if (g2_is_inf<C>(q)) return p;
  const Fp2<C> Z1Z1 = f2_sqr<C>(p.Z);
  const Fp2<C> Z2Z2 = f2_sqr<C>(q.Z);
  const Fp2<C> U1 = f2_mul<C>(p.X, Z2Z2);
  const Fp2<C> U2 = f2_mul<C>(q.X, Z1Z1);
  const Fp2<C> S1 = f2_mul<C>(p.Y, f2_mul<C>(q.Z, Z2Z2));
  const Fp2<C> S2 = f2_mul<C>(q.Y, f2_mul<C>(p.Z, Z1Z1));
  const Fp2<C> H = f2_sub<C>(U2, U1);
  const Fp2<C> rr = f2_dbl<C>(f2_sub<C>(S2, S1));
  if (f2_is_zero<C>(H)) {
    if (f2_is_zero<C>(rr)) return g2_dbl<C>(p);
    return g2_inf<C>();
  }
  const Fp2<C> I = f2_sqr<C>(f2_dbl<C>(H));
  const Fp2<C> J = f2_mul<C>(H, I);
  const Fp2<C> V = f2_mul<C>(U1, I);
  G2J<C> r;
  r.X = f2_sub<C>(f2_sub<C>(f2_sqr<C>(rr), J), f2_dbl<C>(V));
  r.Y = f2_sub<C>(f2_mul<C>(rr, f2_sub<C>(V, r.X)), f2_dbl<C>(f2_mul<C>(S1, J)));
  r.Z = f2_mul<C>(f2_sub<C>(f2_sub<C>(f2_sqr<C>(f2_add<C>(p.Z, q.Z)), Z1Z1), Z2Z2), H);
  return r;
}
template <class C>
KZGX_TW bool g2_to_affine(const G2J<C>& p, G2A<C>& out) {
  if (g2_is_inf<C>(p)) {
    out.x = f2_zero<C>();
    out.y = f2_zero<C>();
    return false;
  }
  const Fp2<C> zi = f2_inv<C>(p.Z);
  const Fp2<C> zi2 = f2_sqr<C>(zi);
  out.x = f2_mul<C>(p.X, zi2);
  out.y = f2_mul<C>(p.Y, f2_mul<C>(zi2, zi));
  return true;
}
// canonical affine G2 point: x.re, x.im, y.re, y.im (N words each); all
// zero = infinity.  Returns false for infinity.
template <class C>
KZGX_DEV bool g2_from_canon(const uint32_t* w, G2A<C>& a) {
  constexpr int N = C::Fp::N;
  uint32_t o = 0;
  for (int i = 0; i < 4 * N; i++) o |= w[i];
  a.x = f2_from_canon<C>(w);
  a.y = f2_from_canon<C>(w + 2 * N);
  return o != 0;
}
template <class C>
KZGX_DEV void g2_to_canon(const G2A<C>& a, bool finite, uint32_t* w) {
  constexpr int N = C::Fp::N;
  if (!finite) {
    for (int i = 0; i < 4 * N; i++) w[i] = 0;
    return;
  }
  f2_to_canon<C>(a.x, w);
  f2_to_canon<C>(a.y, w + 2 * N);
}

}  // namespace kzgx
