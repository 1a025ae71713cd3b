// G1 arithmetic on y^2 = x^3 + b (a = 0) for gfx950, over the radix-2^29
// lazily reduced base field of field29.hpp.
//
// Bucket accumulators use extended Jacobian "XYZZ" coordinates
// (x = X/ZZ, y = Y/ZZZ, ZZ^3 = ZZZ^2): a mixed add with an affine SRS point
// costs 8M + 2S and a full add 12M + 2S, with no inversion.  ZZ == 0 (exact
// zero limbs) marks infinity; every path that yields infinity writes it
// exactly.  The formulas are complete over the special cases (P == Q ->
// doubling, P == -Q -> infinity), so the result is the exact group element
// whatever the SRS (tau = 0 / 1 / -1 included).
//
// Value bounds (m = field modulus; products are < 2m, see field29.hpp):
//   affine x, y (table / inputs)     < m   (canonical Montgomery)
//   XYZZ X < 8m, Y < 4m, ZZ, ZZZ < 2m   (invariant kept by every op below)
// Each subtraction adds the smallest multiple of m that keeps it
// non-negative; every product's operands satisfy a b < 222 m^2 (BN254, the
// tighter of the two curves).
//
// Replaces miracl-core's ECP_add / PAIR_G1mul on the hot path
// (src/trusted_setup.cpp:161-170).
#pragma once
#include "field.hpp"
#include "field29.hpp"

// Cold or non-critical point operations are real calls (not inlined):
// inlining them into every call site multiplies code size (and compile
// time) without helping the scheduler.  The hot loop uses the _impl forms.
#define KZGX_PT __device__ __noinline__

// Assembly comments that scripts/isa_count.py uses to find the rare paths
// (first term after infinity, equal x) and the per-point work of the
// accumulation loops.  Only with -DKZGX_ISA_MARKERS (the counting build): an
// asm statement is a scheduling barrier, so production code has none.
#ifdef KZGX_ISA_MARKERS
#define KZGX_MARK(s) asm volatile(";" s)
#else
#define KZGX_MARK(s)
#endif

// -Y1 in the mixed add's Y3: carry-free 8m - Y1 (f29_neg8_lazy) or the
// carried 4m - Y1.  The lazy form saves ~25 VALU instructions but makes the
// compiler spill around the rare P == +-a branch of the fixed-base kernel.
#ifdef KZGX_LAZY_NEG_Y1
#define KZGX_NEG_Y1(y) f29_neg8_lazy<F>(y)
#else
#define KZGX_NEG_Y1(y) f29_sub<F>(f29_zero<F>(), (y), F::P4)
#endif

// scheduling fence between the product groups of the chained mixed addition
// (keeps the scheduler from overlapping groups, which raises register
// pressure past the accumulation kernels' budget)
#ifdef KZGX_NO_GROUP_FENCE
#define KZGX_GROUP_FENCE() ((void)0)
#else
#define KZGX_GROUP_FENCE() __builtin_amdgcn_sched_barrier(0)
#endif

// the full XYZZ addition with its products as lockstep chains (1) or one
// product at a time (0, the default: the lockstep form measured no change in
// single-call latency -- 0.746 / 0.296 ms Pippenger / table commit against
// 0.741 / 0.301 -- nor in the batched Pippenger leg, profiles/r03_add_tri_latency.txt)
#ifndef KZGX_ADD_TRI
#define KZGX_ADD_TRI 0
#endif

namespace kzgx {

template <class C>
struct Affine {
  F29<typename C::Fp29> x, y;
};

template <class C>
struct Xyzz {
  F29<typename C::Fp29> X, Y, ZZ, ZZZ;
};

// words per stored affine point / XYZZ point (16-byte aligned)
template <class C>
constexpr int affine_words() {
  return (2 * C::Fp29::L + 3) & ~3;
}
template <class C>
constexpr int xyzz_words() {
  return 4 * C::Fp29::L;
}

template <class C>
KZGX_PT Xyzz<C> xyzz_dbl(const Xyzz<C>& p);
template <class C>
KZGX_PT Xyzz<C> xyzz_dbl_affine(const Affine<C>& a);

template <class C>
KZGX_DEV Xyzz<C> xyzz_inf() {
  using F = typename C::Fp29;
  Xyzz<C> r;
  r.X = f29_one<F>();
  r.Y = f29_one<F>();
  r.ZZ = f29_zero<F>();
  r.ZZZ = f29_zero<F>();
  return r;
}

template <class C>
KZGX_DEV bool xyzz_is_inf(const Xyzz<C>& p) {
  return f29_is_zero_exact<typename C::Fp29>(p.ZZ);
}

template <class C>
KZGX_DEV Xyzz<C> xyzz_from_affine(const Affine<C>& a) {
  using F = typename C::Fp29;
  Xyzz<C> r;
  r.X = a.x;
  r.Y = a.y;
  r.ZZ = f29_one<F>();
  r.ZZZ = f29_one<F>();
  return r;
}

// doubling of an affine point (mdbl-2008-s-1); x, y < 2m
template <class C>
KZGX_DEV Xyzz<C> xyzz_dbl_affine_impl(const Affine<C>& a) {
  using F = typename C::Fp29;
  Xyzz<C> r;
  F29<F> U = f29_add<F>(a.y, a.y);                      // < 4m
  F29<F> V = f29_sqr<F>(U);                             // < 2m
  F29<F> W = f29_mul<F>(U, V);
  F29<F> S = f29_mul<F>(a.x, V);
  F29<F> xx = f29_sqr<F>(a.x);
  F29<F> M = f29_add<F>(f29_add<F>(xx, xx), xx);        // < 6m
  F29<F> X3 = f29_sub<F>(f29_sqr<F>(M), f29_add<F>(S, S), F::P4);  // < 6m
  // M (S - X3) - W y as one reduction: + W (4m - y) = - W y mod m; < 60m^2 + 8m^2
  F29<F> Y3 = f29_mul2<F>(M, f29_sub<F>(S, X3, F::P8), W, f29_sub<F>(f29_zero<F>(), a.y, F::P4));  // < 2m
  r.X = X3;
  r.Y = Y3;
  r.ZZ = V;
  r.ZZZ = W;
  return r;
}

// doubling (dbl-2008-s-1, a = 0); no 2-torsion in the prime-order subgroup
template <class C>
KZGX_DEV Xyzz<C> xyzz_dbl_impl(const Xyzz<C>& p) {
  using F = typename C::Fp29;
  if (xyzz_is_inf<C>(p)) return p;
  Xyzz<C> r;
  F29<F> U = f29_add<F>(p.Y, p.Y);                      // < 8m
  F29<F> V = f29_sqr<F>(U);                             // < 2m (64 m^2)
  F29<F> W = f29_mul<F>(U, V);
  F29<F> S = f29_mul<F>(p.X, V);
  F29<F> xx = f29_sqr<F>(p.X);
  F29<F> M = f29_add<F>(f29_add<F>(xx, xx), xx);        // < 6m
  F29<F> X3 = f29_sub<F>(f29_sqr<F>(M), f29_add<F>(S, S), F::P4);  // < 6m
  F29<F> Y3 = f29_mul2<F>(M, f29_sub<F>(S, X3, F::P8), W, f29_sub<F>(f29_zero<F>(), p.Y, F::P4));  // < 2m
  r.X = X3;
  r.Y = Y3;
  r.ZZ = f29_mul<F>(V, p.ZZ);
  r.ZZZ = f29_mul<F>(W, p.ZZZ);
  return r;
}

// p + a, a affine and finite (madd-2008-s), one product at a time (the
// compiler splits each column into two mad chains and merges them: kept for
// A/B against xyzz_add_affine_nway, scripts/micro_madd.hip)
template <class C>
KZGX_DEV Xyzz<C> xyzz_add_affine_classic(const Xyzz<C>& p, const Affine<C>& a) {
  using F = typename C::Fp29;
#ifdef KZGX_LAZY_NEG_Y1
  if (xyzz_is_inf<C>(p)) {  // keep Y normalized (a.y may be a lazy negation)
    Xyzz<C> r = xyzz_from_affine<C>(a);
    r.Y = f29_normalize<F>(a.y);
    return r;
  }
#else
  if (xyzz_is_inf<C>(p)) {
    KZGX_MARK("KZGX_RARE");
    return xyzz_from_affine<C>(a);
  }
#endif
  F29<F> U2 = f29_mul<F>(a.x, p.ZZ);                    // < 2m
  F29<F> S2 = f29_mul<F>(a.y, p.ZZZ);                   // < 2m
  F29<F> P = f29_sub<F>(U2, p.X, F::P8);                // < 10m
  F29<F> R = f29_sub<F>(S2, p.Y, F::P4);                // < 6m
  F29<F> PP = f29_sqr<F>(P);                            // < 2m
  if (f29_is_zero_lt2m<F>(PP)) {                        // x equal: double or cancel
    KZGX_MARK("KZGX_RARE");
    if (f29_is_zero<F>(R)) return xyzz_dbl_affine_impl<C>(a);  // inline: no call frame in the hot loop
    return xyzz_inf<C>();
  }
  F29<F> PPP = f29_mul<F>(P, PP);
  F29<F> Q = f29_mul<F>(p.X, PP);
  Xyzz<C> r;
  // PPP + 2Q < 6m without carries (limbs < 3 2^29): f29_sub absorbs them
  r.X = f29_sub<F>(f29_sqr<F>(R), f29_add_2x_lazy<F>(PPP, Q), F::P6);       // < 8m
  // R (Q - X3) - Y1 PPP with one reduction: < 60m^2 + 16m^2 -> < 2m.  8m - Y1
  // is carry-free (limbs < 2^30; Y1 < 4m normalized: every path writes Y
  // normalized); the column sums hold with it as the one lazy operand.
  r.Y = f29_mul2<F>(R, f29_sub<F>(Q, r.X, F::P8), KZGX_NEG_Y1(p.Y), PPP);
  r.ZZ = f29_mul<F>(p.ZZ, PP);
  r.ZZZ = f29_mul<F>(p.ZZZ, PPP);
  return r;
}

// p + a as xyzz_add_affine_classic (same formulas, same value bounds, the
// same field values), with every product's columns as single mad chains
// (field29.hpp, "chained forms": no per-column merge of two partial
// chains).  KZGX_NWAY_PAIRS: independent products side by side --
// (U2, S2), (PPP, Q), (ZZ3, ZZZ3) -- otherwise one product at a time.
// The order keeps few values live: P^2 before (PPP, Q), R^2 after it, Y3
// before ZZ3 / ZZZ3.
#ifndef KZGX_NWAY_PAIRS
#define KZGX_NWAY_PAIRS 1
#endif
template <class C>
KZGX_DEV Xyzz<C> xyzz_add_affine_nway(const Xyzz<C>& p, const Affine<C>& a) {
  using F = typename C::Fp29;
#ifdef KZGX_LAZY_NEG_Y1
  if (xyzz_is_inf<C>(p)) {
    Xyzz<C> r = xyzz_from_affine<C>(a);
    r.Y = f29_normalize<F>(a.y);
    return r;
  }
#else
  if (xyzz_is_inf<C>(p)) {
    KZGX_MARK("KZGX_RARE");
    return xyzz_from_affine<C>(a);
  }
#endif
  F29<F> U2, S2;
#ifdef KZGX_NWAY_TRI
  // (U2, S2), (P^2, R^2), (PPP, Q, ZZ3) three in lockstep, (Y3, ZZZ3) with
  // Y3's two products and ZZZ3's as three chains (field29.hpp "three chains")
  f29_mul_x2<F>(a.x, p.ZZ, a.y, p.ZZZ, U2, S2);
  const F29<F> P = f29_sub<F>(U2, p.X, F::P8);  // < 10m
  const F29<F> R = f29_sub<F>(S2, p.Y, F::P4);  // < 6m
  F29<F> PP, RR;
  f29_sqr_x2<F>(P, R, PP, RR);                   // < 2m each
  if (f29_is_zero_lt2m<F>(PP)) {
    KZGX_MARK("KZGX_RARE");
    if (f29_is_zero<F>(R)) return xyzz_dbl_affine_impl<C>(a);
    return xyzz_inf<C>();
  }
  F29<F> PPP, Q;
  Xyzz<C> r;
  f29_mul_x3<F>(P, PP, p.X, PP, p.ZZ, PP, PPP, Q, r.ZZ);
  r.X = f29_sub<F>(RR, f29_add_2x_lazy<F>(PPP, Q), F::P6);  // < 8m
  f29_mul2_mul<F>(R, f29_sub<F>(Q, r.X, F::P8), KZGX_NEG_Y1(p.Y), PPP, p.ZZZ, PPP, r.Y, r.ZZZ);
  return r;
#else
#if KZGX_NWAY_PAIRS
  f29_mul_x2<F>(a.x, p.ZZ, a.y, p.ZZZ, U2, S2);
#else
  U2 = f29_mul_chain<F>(a.x, p.ZZ);
  S2 = f29_mul_chain<F>(a.y, p.ZZZ);
#endif
  const F29<F> P = f29_sub<F>(U2, p.X, F::P8);          // < 10m
  const F29<F> R = f29_sub<F>(S2, p.Y, F::P4);          // < 6m
  const F29<F> PP = f29_sqr_chain<F>(P);                // < 2m
  if (f29_is_zero_lt2m<F>(PP)) {  // x equal: double or cancel
    KZGX_MARK("KZGX_RARE");
    if (f29_is_zero<F>(R)) return xyzz_dbl_affine_impl<C>(a);
    return xyzz_inf<C>();
  }
  F29<F> PPP, Q;
#if KZGX_NWAY_PAIRS
  f29_mul_x2<F>(P, PP, p.X, PP, PPP, Q);
#else
  PPP = f29_mul_chain<F>(P, PP);
  Q = f29_mul_chain<F>(p.X, PP);
#endif
  const F29<F> RR = f29_sqr_chain<F>(R);
  Xyzz<C> r;
  r.X = f29_sub<F>(RR, f29_add_2x_lazy<F>(PPP, Q), F::P6);  // < 8m
  // Y3 = R (Q - X3) + (-Y1) PPP with one reduction
  r.Y = f29_mul2_chain<F>(R, f29_sub<F>(Q, r.X, F::P8), KZGX_NEG_Y1(p.Y), PPP);
#if KZGX_NWAY_PAIRS
  f29_mul_x2<F>(p.ZZ, PP, p.ZZZ, PPP, r.ZZ, r.ZZZ);
#else
  r.ZZ = f29_mul_chain<F>(p.ZZ, PP);
  r.ZZZ = f29_mul_chain<F>(p.ZZZ, PPP);
#endif
  return r;
#endif
}

// the mixed addition every accumulation loop inlines: 0 = classic (one
// product at a time), 1 = grouped independent products (nway).  Per curve
// (KZGX_MADD_VARIANT overrides both): chosen by the interleaved A/B of the
// bench kernels in DESIGN.md section 3.
#ifdef KZGX_MADD_VARIANT
#define KZGX_MADD_VARIANT_BN KZGX_MADD_VARIANT
#define KZGX_MADD_VARIANT_BLS KZGX_MADD_VARIANT
#endif
#ifndef KZGX_MADD_VARIANT_BN
#define KZGX_MADD_VARIANT_BN 1
#endif
#ifndef KZGX_MADD_VARIANT_BLS
#define KZGX_MADD_VARIANT_BLS 1
#endif
template <class C>
constexpr int madd_variant() {
  return C::Fp29::L <= 9 ? KZGX_MADD_VARIANT_BN : KZGX_MADD_VARIANT_BLS;
}
template <class C, int V>
KZGX_DEV Xyzz<C> xyzz_add_affine_v(const Xyzz<C>& p, const Affine<C>& a) {
  if constexpr (V == 0) {
    return xyzz_add_affine_classic<C>(p, a);
  } else if constexpr (V == 1) {
    return xyzz_add_affine_nway<C>(p, a);
  } else {  // V == 2: no arithmetic, the operand only consumed (memory-path probe for scripts/micro_madd.hip)
    Xyzz<C> r = p;
#pragma unroll
    for (int i = 0; i < C::Fp29::L; i++) {
      r.X.v[i] ^= a.x.v[i];
      r.Y.v[i] ^= a.y.v[i];
    }
    return r;
  }
}
template <class C>
KZGX_DEV Xyzz<C> xyzz_add_affine_impl(const Xyzz<C>& p, const Affine<C>& a) {
  return xyzz_add_affine_v<C, madd_variant<C>()>(p, a);
}

// p + q (add-2008-s)
template <class C>
KZGX_DEV Xyzz<C> xyzz_add_impl(const Xyzz<C>& p, const Xyzz<C>& q) {
  using F = typename C::Fp29;
  if (xyzz_is_inf<C>(p)) return q;
  if (xyzz_is_inf<C>(q)) return p;
#if KZGX_ADD_TRI
  // the same formulas and bounds as below, the products three chains in
  // lockstep (field29.hpp "three chains"): (U1, U2, S1), (S2, ZZ1 ZZ2,
  // ZZZ1 ZZZ2), (P^2, R^2) paired, (PPP, Q, ZZ3), then Y3 with ZZZ3
  {
    F29<F> U1, U2, S1, S2, ZZ12, ZZZ12;
    f29_mul_x3<F>(p.X, q.ZZ, q.X, p.ZZ, p.Y, q.ZZZ, U1, U2, S1);
    f29_mul_x3<F>(q.Y, p.ZZZ, p.ZZ, q.ZZ, p.ZZZ, q.ZZZ, S2, ZZ12, ZZZ12);
    const F29<F> P = f29_sub<F>(U2, U1, F::P2);  // < 4m
    const F29<F> R = f29_sub<F>(S2, S1, F::P2);  // < 4m
    F29<F> PP, RR;
    f29_sqr_x2_pair<F>(P, R, PP, RR);
    if (f29_is_zero_lt2m<F>(PP)) {
      if (f29_is_zero<F>(R)) return xyzz_dbl_impl<C>(p);
      return xyzz_inf<C>();
    }
    F29<F> PPP, Q;
    Xyzz<C> r;
    f29_mul_x3<F>(P, PP, U1, PP, ZZ12, PP, PPP, Q, r.ZZ);
    r.X = f29_sub<F>(RR, f29_add<F>(PPP, f29_add<F>(Q, Q)), F::P6);
    f29_mul2_mul<F>(R, f29_sub<F>(Q, r.X, F::P8), f29_sub<F>(f29_zero<F>(), S1, F::P2), PPP, ZZZ12, PPP, r.Y,
                    r.ZZZ);  // Y3 < 2m
    return r;
  }
#endif
  F29<F> U1 = f29_mul<F>(p.X, q.ZZ);
  F29<F> U2 = f29_mul<F>(q.X, p.ZZ);
  F29<F> S1 = f29_mul<F>(p.Y, q.ZZZ);
  F29<F> S2 = f29_mul<F>(q.Y, p.ZZZ);
  F29<F> P = f29_sub<F>(U2, U1, F::P2);                 // < 4m
  F29<F> R = f29_sub<F>(S2, S1, F::P2);                 // < 4m
  F29<F> PP = f29_sqr<F>(P);
  if (f29_is_zero_lt2m<F>(PP)) {
    if (f29_is_zero<F>(R)) return xyzz_dbl_impl<C>(p);  // inline: no call frame in callers' loops
    return xyzz_inf<C>();
  }
  F29<F> PPP = f29_mul<F>(P, PP);
  F29<F> Q = f29_mul<F>(U1, PP);
  Xyzz<C> r;
  r.X = f29_sub<F>(f29_sqr<F>(R), f29_add<F>(PPP, f29_add<F>(Q, Q)), F::P6);
  r.Y = f29_mul2<F>(R, f29_sub<F>(Q, r.X, F::P8), f29_sub<F>(f29_zero<F>(), S1, F::P2), PPP);  // < 2m
  r.ZZ = f29_mul<F>(f29_mul<F>(p.ZZ, q.ZZ), PP);
  r.ZZZ = f29_mul<F>(f29_mul<F>(p.ZZZ, q.ZZZ), PPP);
  return r;
}

// XYZZ -> affine, canonical Montgomery (< m).  Returns false for infinity.
// UNIFORM: one lane's conversion (the first active lane's point), its
// inversion on the scalar ALU (f29_inv_uniform)
template <class C, bool UNIFORM = false>
KZGX_DEV bool xyzz_to_affine_impl(const Xyzz<C>& p, Affine<C>& out) {
  using F = typename C::Fp29;
  if (xyzz_is_inf<C>(p)) {
    out.x = f29_zero<F>();
    out.y = f29_zero<F>();
    return false;
  }
  F29<F> t = f29_mul<F>(p.ZZ, p.ZZZ);
  F29<F> i;  // 1 / (ZZ ZZZ)
  if constexpr (UNIFORM) i = f29_inv_uniform<F, C::Fp::N>(t, C::Fp::P);
  else i = f29_inv_fast<F, C::Fp::N>(t, C::Fp::P, C::Fp::PM2);
  F29<F> izz = f29_mul<F>(i, p.ZZZ);               // 1 / ZZ
  F29<F> izzz = f29_mul<F>(i, p.ZZ);               // 1 / ZZZ
  out.x = f29_reduce<F>(f29_mul<F>(p.X, izz));
  out.y = f29_reduce<F>(f29_mul<F>(p.Y, izzz));
  return true;
}

template <class C>
KZGX_DEV Xyzz<C> xyzz_neg(const Xyzz<C>& p) {
  using F = typename C::Fp29;
  Xyzz<C> r = p;
  r.Y = f29_sub<F>(f29_zero<F>(), p.Y, F::P4);
  return r;
}

template <class C>
KZGX_DEV Affine<C> affine_neg(const Affine<C>& a) {
  using F = typename C::Fp29;
  Affine<C> r = a;
  r.y = f29_sub<F>(f29_zero<F>(), a.y, F::P);  // m - y, in (0, m]
  return r;
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

// one lane's conversion (only the calling lane active, or every active lane
// holding the same point)
template <class C>
KZGX_PT bool xyzz_to_affine_lane(const Xyzz<C>& p, Affine<C>& out) {
  return xyzz_to_affine_impl<C, true>(p, out);
}

// XYZZ -> the canonical affine words written at out (x || y, C::Fp::N words
// each, zeros for infinity), for the final result of a latency path: one
// lane's point converted by the whole wave (uniform inversion, as
// xyzz_to_affine_lane).  The inverse comes out as the plain residue
// i = 1 / (ZZ ZZZ) (f29_inv_uniform_raw), so 1/ZZ = i ZZZ / R and
// x = X (1/ZZ) / R are already canonical: against xyzz_to_affine_lane +
// affine_to_canonical, one product by R^2 and the two from-Montgomery
// products leave the chain.  Every lane computes; the caller lets one store.
template <class C>
KZGX_PT bool xyzz_to_canonical_lane(const Xyzz<C>& p, uint32_t (&wx)[C::Fp::N], uint32_t (&wy)[C::Fp::N]) {
  using F = typename C::Fp29;
  constexpr int N = C::Fp::N;
  if (xyzz_is_inf<C>(p)) {
#pragma unroll
    for (int k = 0; k < N; k++) wx[k] = wy[k] = 0u;
    return false;
  }
  const F29<F> i = f29_inv_uniform_raw<F, N>(f29_mul<F>(p.ZZ, p.ZZZ), C::Fp::P);
  const F29<F> izz = f29_mul<F>(i, p.ZZZ);   // 1 / ZZ, plain
  const F29<F> izzz = f29_mul<F>(i, p.ZZ);   // 1 / ZZZ, plain
  f29_to_words<F, N>(f29_reduce<F>(f29_mul<F>(p.X, izz)), wx);
  f29_to_words<F, N>(f29_reduce<F>(f29_mul<F>(p.Y, izzz)), wy);
  return true;
}

// ---- storage ---------------------------------------------------------------
// table / workspace affine point: x (L words) || y (L words), padded to
// affine_words<C>() so every point starts 16-byte aligned
template <class C>
KZGX_DEV Affine<C> affine_load(const uint32_t* p) {
  constexpr int L = C::Fp29::L;
  constexpr int AW = affine_words<C>();
  uint32_t w[AW];
#pragma unroll
  for (int i = 0; i < AW / 4; i++) {
    uint4 q = reinterpret_cast<const uint4*>(p)[i];
    w[4 * i] = q.x;
    w[4 * i + 1] = q.y;
    w[4 * i + 2] = q.z;
    w[4 * i + 3] = q.w;
  }
  Affine<C> a;
#pragma unroll
  for (int i = 0; i < L; i++) {
    a.x.v[i] = w[i];
    a.y.v[i] = w[L + i];
  }
  return a;
}

template <class C>
KZGX_DEV void affine_store(uint32_t* p, const Affine<C>& a) {
  constexpr int L = C::Fp29::L;
  constexpr int AW = affine_words<C>();
  uint32_t w[AW];
#pragma unroll
  for (int i = 0; i < AW; i++) w[i] = 0;
#pragma unroll
  for (int i = 0; i < L; i++) {
    w[i] = a.x.v[i];
    w[L + i] = a.y.v[i];
  }
#pragma unroll
  for (int i = 0; i < AW / 4; i++)
    reinterpret_cast<uint4*>(p)[i] = make_uint4(w[4 * i], w[4 * i + 1], w[4 * i + 2], w[4 * i + 3]);
}

template <class C>
KZGX_DEV Xyzz<C> xyzz_load(const uint32_t* p) {
  constexpr int L = C::Fp29::L;
  uint32_t w[4 * L];
#pragma unroll
  for (int i = 0; i < L; i++) {
    uint4 q = reinterpret_cast<const uint4*>(p)[i];
    w[4 * i] = q.x;
    w[4 * i + 1] = q.y;
    w[4 * i + 2] = q.z;
    w[4 * i + 3] = q.w;
  }
  Xyzz<C> r;
#pragma unroll
  for (int i = 0; i < L; i++) {
    r.X.v[i] = w[i];
    r.Y.v[i] = w[L + i];
    r.ZZ.v[i] = w[2 * L + i];
    r.ZZZ.v[i] = w[3 * L + i];
  }
  return r;
}

template <class C>
KZGX_DEV void xyzz_store(uint32_t* p, const Xyzz<C>& a) {
  constexpr int L = C::Fp29::L;
  uint32_t w[4 * L];
#pragma unroll
  for (int i = 0; i < L; i++) {
    w[i] = a.X.v[i];
    w[L + i] = a.Y.v[i];
    w[2 * L + i] = a.ZZ.v[i];
    w[3 * L + i] = a.ZZZ.v[i];
  }
#pragma unroll
  for (int i = 0; i < L; i++)
    reinterpret_cast<uint4*>(p)[i] = make_uint4(w[4 * i], w[4 * i + 1], w[4 * i + 2], w[4 * i + 3]);
}

// canonical little-endian 32-bit-word affine point (x || y, N words each;
// all-zero = infinity) <-> radix-2^29 Montgomery.  Returns false for infinity.
template <class C>
KZGX_DEV bool affine_from_canonical(const uint32_t* p, Affine<C>& a) {
  using F = typename C::Fp29;
  constexpr int N = C::Fp::N;
  uint32_t wx[N], wy[N];
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < N; i++) {
    wx[i] = p[i];
    wy[i] = p[N + i];
    o |= wx[i] | wy[i];
  }
  a.x = f29_reduce<F>(f29_to_mont<F>(f29_from_words<F, N>(wx)));
  a.y = f29_reduce<F>(f29_to_mont<F>(f29_from_words<F, N>(wy)));
  return o != 0;
}

// affine (Montgomery, < m) -> canonical words; infinity writes zeros
template <class C>
KZGX_DEV void affine_to_canonical(uint32_t* p, const Affine<C>& a, bool finite) {
  using F = typename C::Fp29;
  constexpr int N = C::Fp::N;
  uint32_t wx[N], wy[N];
  f29_to_words<F, N>(f29_from_mont<F>(a.x), wx);
  f29_to_words<F, N>(f29_from_mont<F>(a.y), wy);
#pragma unroll
  for (int i = 0; i < N; i++) {
    p[i] = finite ? wx[i] : 0u;
    p[N + i] = finite ? wy[i] : 0u;
  }
}

}  // namespace kzgx
