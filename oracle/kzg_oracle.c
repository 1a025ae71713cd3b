/* CPU oracle (TEST INFRASTRUCTURE ONLY) -- plain-C restatement of the
 * reference KZG hot path of uncommitted6453/kzg-commitments.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load
 * liboracle.so, as the checker / the timed "port" CPU baseline; the product
 * (libkzgx.so) never links or calls it.
 *
 * Parity status: the reference is unbuildable here (miracl-core + NTL are
 * empty submodules) and holds no known-answer vectors, so this port is
 * pinned by the Python oracle's goldens (tests/golden/), which are in turn
 * pinned by curve-constant self checks and the MSM-independent identity
 * commit == [P(tau)]G1 (see oracle/kzg_ref.py header).
 *
 * What it restates (file:line into /root/reference):
 *   orc_msm_naive   trusted_setup::polyeval_G1, src/trusted_setup.cpp:149-174
 *                   (one full scalar multiplication per term + ECP_add)
 *   orc_gen_srs     trusted_setup(int), src/trusted_setup.cpp:21-74,123-135
 *                   (G1 part; tau given instead of std::random_device)
 *   orc_poly_eval   NTL eval / evaluate_polynomial_points, src/util.cpp:186-211
 *   orc_interpolate polyfit / linear_roots_and_polyfit, src/util.cpp:172-184
 *   orc_quotient    q = (P - I) / Z, src/trusted_setup.cpp:214-225
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define NL 4
#define PFX f4_
#include "oracle_field.h"
#undef NL
#undef PFX
#define NL 6
#define PFX f6_
#include "oracle_field.h"
#undef NL
#undef PFX

/* curve ids: 0 = miracl BN254 (Nogami, y^2 = x^3 + 2), 1 = BLS12-381 */
static const char* BN_P_HEX = "2523648240000001BA344D80000000086121000000000013A700000000000013";
static const char* BN_R_HEX = "2523648240000001BA344D8000000007FF9F800000000010A10000000000000D";
static const char* BN_GX_HEX = "2523648240000001BA344D80000000086121000000000013A700000000000012";
static const char* BN_GY_HEX = "01";
static const char* BLS_P_HEX =
    "1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB";
static const char* BLS_R_HEX = "73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001";
static const char* BLS_GX_HEX =
    "17F1D3A73197D7942695638C4FA9AC0FC3688C4F9774B905A14E3A3F171BAC586C55E83FF97A1AEFFB3AF00ADB22C6BB";
static const char* BLS_GY_HEX =
    "08B3F481E3AAA0F1A09E30ED741D8AE4FCF5E095D5D00AF600DB18CB2C04B3EDD03CC744A2888AE40CAA232946C5E7E1";

static void hex_to_limbs(const char* h, uint64_t* out, int nl) {
  memset(out, 0, nl * 8);
  int len = (int)strlen(h);
  for (int i = 0; i < len; i++) {
    char c = h[len - 1 - i];
    uint64_t v = (c >= '0' && c <= '9') ? (uint64_t)(c - '0') : (uint64_t)((c | 32) - 'a' + 10);
    out[i / 16] |= v << (4 * (i % 16));
  }
}

typedef struct {
  int ready;
  f4_field_t fr;
  f4_field_t fp4;
  f6_field_t fp6;
  int nlp;                 /* base-field limbs: 4 or 6 */
  uint64_t gx[6], gy[6];   /* Montgomery */
  uint64_t b[6];           /* Montgomery curve constant */
} orc_curve_t;

static orc_curve_t CURVES[2];

static orc_curve_t* get_curve(int id) {
  if (id < 0 || id > 1) return NULL;
  orc_curve_t* c = &CURVES[id];
  if (c->ready) return c;
  uint64_t m[6], gx[6], gy[6], b[6];
  memset(b, 0, sizeof b);
  if (id == 0) {
    hex_to_limbs(BN_P_HEX, m, 4);
    f4_field_init(&c->fp4, m);
    hex_to_limbs(BN_R_HEX, m, 4);
    f4_field_init(&c->fr, m);
    c->nlp = 4;
    hex_to_limbs(BN_GX_HEX, gx, 4);
    hex_to_limbs(BN_GY_HEX, gy, 4);
    b[0] = 2;
    f4_to_mont(&c->fp4, c->gx, gx);
    f4_to_mont(&c->fp4, c->gy, gy);
    f4_to_mont(&c->fp4, c->b, b);
  } else {
    hex_to_limbs(BLS_P_HEX, m, 6);
    f6_field_init(&c->fp6, m);
    hex_to_limbs(BLS_R_HEX, m, 4);
    f4_field_init(&c->fr, m);
    c->nlp = 6;
    hex_to_limbs(BLS_GX_HEX, gx, 6);
    hex_to_limbs(BLS_GY_HEX, gy, 6);
    b[0] = 4;
    f6_to_mont(&c->fp6, c->gx, gx);
    f6_to_mont(&c->fp6, c->gy, gy);
    f6_to_mont(&c->fp6, c->b, b);
  }
  c->ready = 1;
  return c;
}

int orc_base_limbs(int curve) {
  orc_curve_t* c = get_curve(curve);
  return c ? c->nlp : -1;
}

/* ---------------------------------------------------------------------- */
/* G1 helpers dispatching on limb count                                    */
/* ---------------------------------------------------------------------- */
typedef union {
  f4_jac_t j4;
  f6_jac_t j6;
} jac_u;

static void pt_from_affine_canon(orc_curve_t* c, jac_u* R, const uint64_t* xy) {
  int nl = c->nlp;
  uint64_t x[6], y[6];
  if (nl == 4) {
    f4_to_mont(&c->fp4, x, xy);
    f4_to_mont(&c->fp4, y, xy + 4);
    f4_from_affine(&c->fp4, &R->j4, x, y);
  } else {
    f6_to_mont(&c->fp6, x, xy);
    f6_to_mont(&c->fp6, y, xy + 6);
    f6_from_affine(&c->fp6, &R->j6, x, y);
  }
}

static int pt_to_affine_canon(orc_curve_t* c, uint64_t* xy, const jac_u* P) {
  int nl = c->nlp;
  uint64_t x[6], y[6];
  int inf;
  if (nl == 4) {
    inf = f4_to_affine(&c->fp4, x, y, &P->j4);
    f4_from_mont(&c->fp4, xy, x);
    f4_from_mont(&c->fp4, xy + 4, y);
  } else {
    inf = f6_to_affine(&c->fp6, x, y, &P->j6);
    f6_from_mont(&c->fp6, xy, x);
    f6_from_mont(&c->fp6, xy + 6, y);
  }
  return inf;
}

static void pt_mul(orc_curve_t* c, jac_u* R, const jac_u* P, const uint64_t* k) {
  if (c->nlp == 4)
    f4_jmul(&c->fp4, &R->j4, &P->j4, k);
  else
    f6_jmul(&c->fp6, &R->j6, &P->j6, k);
}

static void pt_add(orc_curve_t* c, jac_u* R, const jac_u* P, const jac_u* Q) {
  if (c->nlp == 4)
    f4_jadd(&c->fp4, &R->j4, &P->j4, &Q->j4);
  else
    f6_jadd(&c->fp6, &R->j6, &P->j6, &Q->j6);
}

static void pt_inf(orc_curve_t* c, jac_u* R) { memset(R, 0, sizeof *R); (void)c; }

static void pt_gen(orc_curve_t* c, jac_u* R) {
  if (c->nlp == 4)
    f4_from_affine(&c->fp4, &R->j4, c->gx, c->gy);
  else
    f6_from_affine(&c->fp6, &R->j6, c->gx, c->gy);
}

/* is the canonical affine point on the curve (or the all-zero infinity)? */
int orc_on_curve(int curve, const uint64_t* xy) {
  orc_curve_t* c = get_curve(curve);
  if (!c) return -1;
  int nl = c->nlp;
  uint64_t x[6], y[6], l[6], r[6];
  int allzero = 1;
  for (int i = 0; i < 2 * nl; i++) allzero &= xy[i] == 0;
  if (allzero) return 1;
  if (nl == 4) {
    if (f4_geq(xy, c->fp4.m) || f4_geq(xy + 4, c->fp4.m)) return 0;
    f4_to_mont(&c->fp4, x, xy);
    f4_to_mont(&c->fp4, y, xy + 4);
    f4_fmul(&c->fp4, l, y, y);
    f4_fmul(&c->fp4, r, x, x);
    f4_fmul(&c->fp4, r, r, x);
    f4_fadd(&c->fp4, r, r, c->b);
    return memcmp(l, r, 32) == 0;
  }
  if (f6_geq(xy, c->fp6.m) || f6_geq(xy + 6, c->fp6.m)) return 0;
  f6_to_mont(&c->fp6, x, xy);
  f6_to_mont(&c->fp6, y, xy + 6);
  f6_fmul(&c->fp6, l, y, y);
  f6_fmul(&c->fp6, r, x, x);
  f6_fmul(&c->fp6, r, r, x);
  f6_fadd(&c->fp6, r, r, c->b);
  return memcmp(l, r, 48) == 0;
}

/* k * P for a canonical affine P; returns 1 if the result is infinity */
int orc_scalar_mul(int curve, const uint64_t* xy, const uint64_t* k, uint64_t* out) {
  orc_curve_t* c = get_curve(curve);
  if (!c) return -1;
  jac_u P, R;
  pt_from_affine_canon(c, &P, xy);
  pt_mul(c, &R, &P, k);
  return pt_to_affine_canon(c, out, &R);
}

/* SRS [tau^i] G1, i < n (trusted_setup.cpp:21-74 / :123-135, G1 part).
 * out: n points, canonical affine x || y (nlp limbs each); infinity = zeros. */
int orc_gen_srs(int curve, const uint64_t* tau, size_t n, uint64_t* out) {
  orc_curve_t* c = get_curve(curve);
  if (!c) return -1;
  if (n < 2) return -2; /* trusted_setup.cpp:22-24 */
  uint64_t s[4] = {1, 0, 0, 0};
  uint64_t t_m[4], s_m[4];
  f4_to_mont(&c->fr, t_m, tau);
  f4_to_mont(&c->fr, s_m, s);
  jac_u G, R;
  pt_gen(c, &G);
  for (size_t i = 0; i < n; i++) {
    f4_from_mont(&c->fr, s, s_m); /* s = tau^i, canonical */
    pt_mul(c, &R, &G, s);
    pt_to_affine_canon(c, out + i * 2 * c->nlp, &R);
    f4_fmul(&c->fr, s_m, s_m, t_m);
  }
  return 0;
}

/* Naive MSM exactly as trusted_setup::polyeval_G1 (src/trusted_setup.cpp:149-174):
 * one full scalar multiplication per term, then an addition.  n == 0 (the
 * zero polynomial, deg -1) gives infinity (:150-154).  Returns 1 if the
 * result is infinity, 0 otherwise. */
int orc_msm_naive(int curve, const uint64_t* srs, const uint64_t* scalars, size_t n, uint64_t* out) {
  orc_curve_t* c = get_curve(curve);
  if (!c) return -1;
  jac_u acc, P, T;
  pt_inf(c, &acc);
  for (size_t i = 0; i < n; i++) {
    pt_from_affine_canon(c, &P, srs + i * 2 * c->nlp);
    pt_mul(c, &T, &P, scalars + 4 * i);
    pt_add(c, &acc, &acc, &T);
  }
  return pt_to_affine_canon(c, out, &acc);
}

/* ---------------------------------------------------------------------- */
/* scalar-field polynomial ops (NTL ZZ_pX semantics, canonical 4-limb)     */
/* ---------------------------------------------------------------------- */
static size_t norm_len(const uint64_t* P, size_t n) {
  while (n > 0 && f4_is_zero(P + 4 * (n - 1))) n--;
  return n;
}

/* y = P(x) by Horner (NTL eval; util.cpp:190) */
int orc_poly_eval(int curve, const uint64_t* P, size_t n, const uint64_t* x, uint64_t* y) {
  orc_curve_t* c = get_curve(curve);
  if (!c) return -1;
  uint64_t acc[4] = {0, 0, 0, 0}, xm[4], cm[4];
  f4_to_mont(&c->fr, xm, x);
  for (size_t i = n; i-- > 0;) {
    f4_fmul(&c->fr, acc, acc, xm);
    f4_to_mont(&c->fr, cm, P + 4 * i);
    f4_fadd(&c->fr, acc, acc, cm);
  }
  f4_from_mont(&c->fr, y, acc);
  return 0;
}

/* Lagrange interpolation through n points with distinct x (the unique
 * polynomial polyfit_R builds via its subproduct tree, util.cpp:213-248).
 * coeffs_out gets n coefficients (not normalized).  Returns -3 on a
 * duplicate node (NTL would raise a division-by-zero error). */
int orc_interpolate(int curve, const uint64_t* xs, const uint64_t* ys, size_t n, uint64_t* coeffs_out) {
  orc_curve_t* c = get_curve(curve);
  if (!c) return -1;
  f4_field_t* f = &c->fr;
  if (n == 0) return 0;
  uint64_t(*X)[4] = malloc(n * 32);
  uint64_t(*Z)[4] = calloc(n + 1, 32);
  uint64_t(*A)[4] = malloc(n * 32);
  uint64_t(*Q)[4] = calloc(n, 32);
  uint64_t(*Cf)[4] = calloc(n, 32);
  int rc = 0;
  for (size_t i = 0; i < n; i++) f4_to_mont(f, X[i], xs + 4 * i);
  /* Z = prod (X - x_i), Montgomery domain; in place, k downward:
   * Z'[k+1] += Z[k], Z'[k] = -x Z[k]  gives  Z' = (X - x) Z */
  memcpy(Z[0], f->one, 32);
  for (size_t i = 0; i < n; i++) {
    for (size_t k = i + 1; k-- > 0;) {
      uint64_t t[4];
      f4_fmul(f, t, Z[k], X[i]);
      f4_fadd(f, Z[k + 1], Z[k + 1], Z[k]);
      f4_fsub(f, Z[k], (uint64_t[4]){0, 0, 0, 0}, t);
    }
  }
  /* a_i = y_i / Z'(x_i) */
  for (size_t i = 0; i < n && rc == 0; i++) {
    uint64_t acc[4] = {0, 0, 0, 0};
    for (size_t k = n; k >= 1; k--) { /* Z' = sum k Z[k] X^(k-1) */
      uint64_t kk[4] = {k, 0, 0, 0}, km[4], t[4];
      f4_fmul(f, acc, acc, X[i]);
      f4_to_mont(f, km, kk);
      f4_fmul(f, t, km, Z[k]);
      f4_fadd(f, acc, acc, t);
    }
    if (f4_is_zero(acc)) {
      rc = -3;
      break;
    }
    uint64_t inv[4], ym[4];
    f4_finv(f, inv, acc);
    f4_to_mont(f, ym, ys + 4 * i);
    f4_fmul(f, A[i], ym, inv);
  }
  if (rc == 0) {
    /* coef_k = sum_i a_i (Z / (X - x_i))_k, synthetic division per node */
    for (size_t k = n; k-- > 0;) {
      uint64_t s[4] = {0, 0, 0, 0};
      for (size_t i = 0; i < n; i++) {
        uint64_t t[4];
        f4_fmul(f, t, X[i], Q[i]);
        f4_fadd(f, Q[i], Z[k + 1], t);
        f4_fmul(f, t, A[i], Q[i]);
        f4_fadd(f, s, s, t);
      }
      memcpy(Cf[k], s, 32);
    }
    for (size_t k = 0; k < n; k++) f4_from_mont(f, coeffs_out + 4 * k, Cf[k]);
  }
  free(X);
  free(Z);
  free(A);
  free(Q);
  free(Cf);
  return rc;
}

/* q = (P - I) / Z for the points x = off .. off+len-1 (trusted_setup.cpp:214-225).
 * P: np canonical coefficients.  q_out must hold max(np, 1) coefficients;
 * *nq receives the normalized quotient length.  Returns -2 if len < 1. */
int orc_quotient(int curve, const uint64_t* P, size_t np, long off, long len, uint64_t* q_out, size_t* nq) {
  orc_curve_t* c = get_curve(curve);
  if (!c) return -1;
  if (len < 1) return -2;
  f4_field_t* f = &c->fr;
  size_t n = (size_t)len;
  uint64_t* xs = malloc(n * 32);
  uint64_t* ys = malloc(n * 32);
  uint64_t* I = calloc(n, 32);
  for (size_t i = 0; i < n; i++) {
    long v = off + (long)i;
    uint64_t a[4] = {(uint64_t)(v < 0 ? -v : v), 0, 0, 0};
    if (v < 0)
      f4_sub_raw(xs + 4 * i, f->m, a);
    else
      memcpy(xs + 4 * i, a, 32);
    orc_poly_eval(curve, P, np, xs + 4 * i, ys + 4 * i);
  }
  int rc = orc_interpolate(curve, xs, ys, n, I);
  size_t npn = norm_len(P, np);
  *nq = 0;
  if (rc == 0 && npn > n) {
    /* R = P - I (Montgomery), then long division by monic Z */
    size_t m = npn;
    uint64_t(*R)[4] = calloc(m, 32);
    uint64_t(*Z)[4] = calloc(n + 1, 32);
    for (size_t k = 0; k < m; k++) {
      uint64_t pm[4], im[4] = {0, 0, 0, 0};
      f4_to_mont(f, pm, P + 4 * k);
      if (k < n) f4_to_mont(f, im, I + 4 * k);
      f4_fsub(f, R[k], pm, im);
    }
    memcpy(Z[0], f->one, 32);
    for (size_t i = 0; i < n; i++) { /* Z *= (X - x_i) */
      uint64_t xm[4];
      f4_to_mont(f, xm, xs + 4 * i);
      for (size_t k = i + 1; k-- > 0;) {
        uint64_t t[4];
        f4_fmul(f, t, Z[k], xm);
        f4_fadd(f, Z[k + 1], Z[k + 1], Z[k]);
        f4_fsub(f, Z[k], (uint64_t[4]){0, 0, 0, 0}, t);
      }
    }
    size_t nqq = m - n;
    for (size_t k = nqq; k-- > 0;) {
      uint64_t qk[4];
      memcpy(qk, R[k + n], 32); /* Z monic */
      for (size_t j = 0; j <= n; j++) {
        uint64_t t[4];
        f4_fmul(f, t, qk, Z[j]);
        f4_fsub(f, R[k + j], R[k + j], t);
      }
      f4_from_mont(f, q_out + 4 * k, qk);
    }
    *nq = norm_len(q_out, nqq);
    free(R);
    free(Z);
  }
  free(xs);
  free(ys);
  free(I);
  return rc;
}
