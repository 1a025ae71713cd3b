// G1 arithmetic on y^2 = x^3 + b (a = 0) for gfx950.
//
// Bucket accumulators use extended Jacobian "XYZZ" coordinates
// (x = X/ZZ, y = Y/ZZZ, ZZ^3 = ZZZ^2): a mixed add with an affine SRS point
// costs 8M + 2S and a full add 12M + 2S, with no inversion.  ZZ == 0 marks
// infinity.  All formulas are complete over the special cases (P == Q ->
// doubling, P == -Q -> infinity), so the result is the exact group element
// whatever the SRS (tau = 0 / 1 / -1 included).
//
// Replaces miracl-core's ECP_add / PAIR_G1mul on the hot path
// (src/trusted_setup.cpp:161-170).
#pragma once
#include "field.hpp"

// Point operations are real calls (not inlined): each is 8-14 inlined field
// products, and inlining them into every kernel call site multiplies code
// size (and compile time) without helping the scheduler.
#define KZGX_PT __device__ __noinline__

namespace kzgx {

template <class C>
struct Affine;
template <class C>
struct Xyzz;
template <class C>
KZGX_PT Xyzz<C> xyzz_dbl_affine(const Affine<C>& a);
template <class C>
KZGX_PT Xyzz<C> xyzz_dbl(const Xyzz<C>& p);
template <class C>
KZGX_PT Xyzz<C> xyzz_add_affine(const Xyzz<C>& p, const Affine<C>& a);
template <class C>
KZGX_PT Xyzz<C> xyzz_add(const Xyzz<C>& p, const Xyzz<C>& q);
template <class C>
KZGX_PT bool xyzz_to_affine(const Xyzz<C>& p, Affine<C>& out);

template <class C>
struct Affine {
  Fe<typename C::Fp> x, y;
};

template <class C>
struct Xyzz {
  Fe<typename C::Fp> X, Y, ZZ, ZZZ;
};

template <class C>
KZGX_DEV Xyzz<C> xyzz_inf() {
  using F = typename C::Fp;
  Xyzz<C> r;
  r.X = fe_one<F>();
  r.Y = fe_one<F>();
  r.ZZ = fe_zero<F>();
  r.ZZZ = fe_zero<F>();
  return r;
}

template <class C>
KZGX_DEV bool xyzz_is_inf(const Xyzz<C>& p) {
  return fe_is_zero<typename C::Fp>(p.ZZ);
}

template <class C>
KZGX_DEV Xyzz<C> xyzz_from_affine(const Affine<C>& a) {
  using F = typename C::Fp;
  Xyzz<C> r;
  r.X = a.x;
  r.Y = a.y;
  r.ZZ = fe_one<F>();
  r.ZZZ = fe_one<F>();
  return r;
}

// doubling of an affine point (mdbl-2008-s-1)
template <class C>
KZGX_DEV Xyzz<C> xyzz_dbl_affine_impl(const Affine<C>& a) {
  using F = typename C::Fp;
  Xyzz<C> r;
  Fe<F> U = fe_dbl<F>(a.y);
  Fe<F> V = fe_sqr<F>(U);
  Fe<F> W = fe_mul<F>(U, V);
  Fe<F> S = fe_mul<F>(a.x, V);
  Fe<F> xx = fe_sqr<F>(a.x);
  Fe<F> M = fe_add<F>(fe_dbl<F>(xx), xx);
  Fe<F> X3 = fe_sub<F>(fe_sqr<F>(M), fe_dbl<F>(S));
  r.Y = fe_sub<F>(fe_mul<F>(M, fe_sub<F>(S, X3)), fe_mul<F>(W, a.y));
  r.X = X3;
  r.ZZ = V;
  r.ZZZ = W;
  return r;
}

// doubling (dbl-2008-s-1, a = 0)
template <class C>
KZGX_DEV Xyzz<C> xyzz_dbl_impl(const Xyzz<C>& p) {
  using F = typename C::Fp;
  if (xyzz_is_inf<C>(p)) return p;
  Xyzz<C> r;
  Fe<F> U = fe_dbl<F>(p.Y);
  Fe<F> V = fe_sqr<F>(U);
  Fe<F> W = fe_mul<F>(U, V);
  Fe<F> S = fe_mul<F>(p.X, V);
  Fe<F> xx = fe_sqr<F>(p.X);
  Fe<F> M = fe_add<F>(fe_dbl<F>(xx), xx);
  Fe<F> X3 = fe_sub<F>(fe_sqr<F>(M), fe_dbl<F>(S));
  r.Y = fe_sub<F>(fe_mul<F>(M, fe_sub<F>(S, X3)), fe_mul<F>(W, p.Y));
  r.X = X3;
  r.ZZ = fe_mul<F>(V, p.ZZ);
  r.ZZZ = fe_mul<F>(W, p.ZZZ);
  return r;
}

// p + a, a affine (madd-2008-s); a must not be infinity
template <class C>
KZGX_DEV Xyzz<C> xyzz_add_affine_impl(const Xyzz<C>& p, const Affine<C>& a) {
  using F = typename C::Fp;
  if (xyzz_is_inf<C>(p)) return xyzz_from_affine<C>(a);
  Fe<F> U2 = fe_mul<F>(a.x, p.ZZ);
  Fe<F> S2 = fe_mul<F>(a.y, p.ZZZ);
  Fe<F> P = fe_sub<F>(U2, p.X);
  Fe<F> R = fe_sub<F>(S2, p.Y);
  if (fe_is_zero<F>(P)) {
    if (fe_is_zero<F>(R)) return xyzz_dbl_affine<C>(a);
    return xyzz_inf<C>();
  }
  Fe<F> PP = fe_sqr<F>(P);
  Fe<F> PPP = fe_mul<F>(P, PP);
  Fe<F> Q = fe_mul<F>(p.X, PP);
  Xyzz<C> r;
  r.X = fe_sub<F>(fe_sub<F>(fe_sqr<F>(R), PPP), fe_dbl<F>(Q));
  r.Y = fe_sub<F>(fe_mul<F>(R, fe_sub<F>(Q, r.X)), fe_mul<F>(p.Y, PPP));
  r.ZZ = fe_mul<F>(p.ZZ, PP);
  r.ZZZ = fe_mul<F>(p.ZZZ, PPP);
  return r;
}

// p + q (add-2008-s)
template <class C>
KZGX_DEV Xyzz<C> xyzz_add_impl(const Xyzz<C>& p, const Xyzz<C>& q) {
  using F = typename C::Fp;
  if (xyzz_is_inf<C>(p)) return q;
  if (xyzz_is_inf<C>(q)) return p;
  Fe<F> U1 = fe_mul<F>(p.X, q.ZZ);
  Fe<F> U2 = fe_mul<F>(q.X, p.ZZ);
  Fe<F> S1 = fe_mul<F>(p.Y, q.ZZZ);
  Fe<F> S2 = fe_mul<F>(q.Y, p.ZZZ);
  Fe<F> P = fe_sub<F>(U2, U1);
  Fe<F> R = fe_sub<F>(S2, S1);
  if (fe_is_zero<F>(P)) {
    if (fe_is_zero<F>(R)) return xyzz_dbl<C>(p);
    return xyzz_inf<C>();
  }
  Fe<F> PP = fe_sqr<F>(P);
  Fe<F> PPP = fe_mul<F>(P, PP);
  Fe<F> Q = fe_mul<F>(U1, PP);
  Xyzz<C> r;
  r.X = fe_sub<F>(fe_sub<F>(fe_sqr<F>(R), PPP), fe_dbl<F>(Q));
  r.Y = fe_sub<F>(fe_mul<F>(R, fe_sub<F>(Q, r.X)), fe_mul<F>(S1, PPP));
  r.ZZ = fe_mul<F>(fe_mul<F>(p.ZZ, q.ZZ), PP);
  r.ZZZ = fe_mul<F>(fe_mul<F>(p.ZZZ, q.ZZZ), PPP);
  return r;
}

template <class C>
KZGX_DEV Xyzz<C> xyzz_neg(const Xyzz<C>& p) {
  Xyzz<C> r = p;
  r.Y = fe_neg<typename C::Fp>(p.Y);
  return r;
}

// k * p for a small non-negative integer k (double-and-add, MSB first)
template <class C>
KZGX_PT Xyzz<C> xyzz_mul_small(const Xyzz<C>& p, uint32_t k) {
  Xyzz<C> acc = xyzz_inf<C>();
  for (int b = 31; b >= 0; b--) {
    acc = xyzz_dbl<C>(acc);
    if ((k >> b) & 1u) acc = xyzz_add<C>(acc, p);
  }
  return acc;
}

// XYZZ -> affine (Montgomery).  Returns false for infinity.
template <class C>
KZGX_DEV bool xyzz_to_affine_impl(const Xyzz<C>& p, Affine<C>& out) {
  using F = typename C::Fp;
  if (xyzz_is_inf<C>(p)) {
    out.x = fe_zero<F>();
    out.y = fe_zero<F>();
    return false;
  }
  Fe<F> t = fe_mul<F>(p.ZZ, p.ZZZ);
  Fe<F> i = fe_inv<F>(t);           // 1 / (ZZ ZZZ)
  Fe<F> izz = fe_mul<F>(i, p.ZZZ);   // 1 / ZZ
  Fe<F> izzz = fe_mul<F>(i, p.ZZ);   // 1 / ZZZ
  out.x = fe_mul<F>(p.X, izz);
  out.y = fe_mul<F>(p.Y, izzz);
  return true;
}

// non-inlined entry points (cold paths and non-critical kernels)
template <class C>
KZGX_PT Xyzz<C> xyzz_dbl_affine(const Affine<C>& a) {
  return xyzz_dbl_affine_impl<C>(a);
}

template <class C>
KZGX_PT Xyzz<C> xyzz_dbl(const Xyzz<C>& p) {
  return xyzz_dbl_impl<C>(p);
}

template <class C>
KZGX_PT Xyzz<C> xyzz_add_affine(const Xyzz<C>& p, const Affine<C>& a) {
  return xyzz_add_affine_impl<C>(p, a);
}

template <class C>
KZGX_PT Xyzz<C> xyzz_add(const Xyzz<C>& p, const Xyzz<C>& q) {
  return xyzz_add_impl<C>(p, q);
}

template <class C>
KZGX_PT bool xyzz_to_affine(const Xyzz<C>& p, Affine<C>& out) {
  return xyzz_to_affine_impl<C>(p, out);
}

// point <-> 32-bit word arrays (Montgomery affine: x || y, 2N words)
template <class C>
KZGX_DEV Affine<C> affine_load(const uint32_t* p) {
  using F = typename C::Fp;
  Affine<C> a;
  a.x = fe_load<F>(p);
  a.y = fe_load<F>(p + F::N);
  return a;
}

template <class C>
KZGX_DEV void affine_store(uint32_t* p, const Affine<C>& a) {
  using F = typename C::Fp;
  fe_store<F>(p, a.x);
  fe_store<F>(p + F::N, a.y);
}

template <class C>
KZGX_DEV Xyzz<C> xyzz_load(const uint32_t* p) {
  using F = typename C::Fp;
  Xyzz<C> r;
  r.X = fe_load<F>(p);
  r.Y = fe_load<F>(p + F::N);
  r.ZZ = fe_load<F>(p + 2 * F::N);
  r.ZZZ = fe_load<F>(p + 3 * F::N);
  return r;
}

template <class C>
KZGX_DEV void xyzz_store(uint32_t* p, const Xyzz<C>& a) {
  using F = typename C::Fp;
  fe_store<F>(p, a.X);
  fe_store<F>(p + F::N, a.Y);
  fe_store<F>(p + 2 * F::N, a.ZZ);
  fe_store<F>(p + 3 * F::N, a.ZZZ);
}

}  // namespace kzgx
