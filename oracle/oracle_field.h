/* CPU oracle (TEST INFRASTRUCTURE ONLY): multi-precision Montgomery field +
 * short-Weierstrass G1 arithmetic, instantiated once per limb count.
 * Included by kzg_oracle.c with NL (64-bit limbs) and PFX (name prefix)
 * defined.  Stands in for miracl-core's FP / ECP (un-vendored, see
 * SURVEY.md section 8c); restates the group law, not miracl's code. */
#ifndef NL
#error "define NL before including oracle_field.h"
#endif

#define CAT2(a, b) a##b
#define CAT(a, b) CAT2(a, b)
#define F(name) CAT(PFX, name)

typedef struct {
  uint64_t m[NL];   /* modulus */
  uint64_t r2[NL];  /* R^2 mod m, R = 2^(64 NL) */
  uint64_t one[NL]; /* R mod m */
  uint64_t n0;      /* -m^-1 mod 2^64 */
} F(field_t);

static int F(geq)(const uint64_t* a, const uint64_t* b) {
  for (int i = NL - 1; i >= 0; i--) {
    if (a[i] != b[i]) return a[i] > b[i];
  }
  return 1;
}

static uint64_t F(add_raw)(uint64_t* c, const uint64_t* a, const uint64_t* b) {
  unsigned __int128 t = 0;
  for (int i = 0; i < NL; i++) {
    t += (unsigned __int128)a[i] + b[i];
    c[i] = (uint64_t)t;
    t >>= 64;
  }
  return (uint64_t)t;
}

static uint64_t F(sub_raw)(uint64_t* c, const uint64_t* a, const uint64_t* b) {
  uint64_t borrow = 0;
  for (int i = 0; i < NL; i++) {
    unsigned __int128 t = (unsigned __int128)a[i] - b[i] - borrow;
    c[i] = (uint64_t)t;
    borrow = (uint64_t)(t >> 64) & 1;
  }
  return borrow;
}

static void F(fadd)(const F(field_t) * f, uint64_t* c, const uint64_t* a, const uint64_t* b) {
  uint64_t t[NL];
  uint64_t carry = F(add_raw)(t, a, b);
  if (carry || F(geq)(t, f->m)) F(sub_raw)(t, t, f->m);
  memcpy(c, t, sizeof t);
}

static void F(fsub)(const F(field_t) * f, uint64_t* c, const uint64_t* a, const uint64_t* b) {
  uint64_t t[NL];
  if (F(sub_raw)(t, a, b)) F(add_raw)(t, t, f->m);
  memcpy(c, t, sizeof t);
}

/* CIOS Montgomery product, c = a b R^-1 mod m (inputs < m). */
static void F(fmul)(const F(field_t) * f, uint64_t* c, const uint64_t* a, const uint64_t* b) {
  uint64_t t[NL + 2];
  memset(t, 0, sizeof t);
  for (int i = 0; i < NL; i++) {
    unsigned __int128 acc = 0;
    for (int j = 0; j < NL; j++) {
      acc = (unsigned __int128)a[j] * b[i] + t[j] + (uint64_t)(acc >> 64);
      t[j] = (uint64_t)acc;
    }
    acc = (unsigned __int128)t[NL] + (uint64_t)(acc >> 64);
    t[NL] = (uint64_t)acc;
    t[NL + 1] = (uint64_t)(acc >> 64);
    uint64_t mq = t[0] * f->n0;
    acc = (unsigned __int128)mq * f->m[0] + t[0];
    for (int j = 1; j < NL; j++) {
      acc = (unsigned __int128)mq * f->m[j] + t[j] + (uint64_t)(acc >> 64);
      t[j - 1] = (uint64_t)acc;
    }
    acc = (unsigned __int128)t[NL] + (uint64_t)(acc >> 64);
    t[NL - 1] = (uint64_t)acc;
    t[NL] = t[NL + 1] + (uint64_t)(acc >> 64);
  }
  if (t[NL] || F(geq)(t, f->m)) F(sub_raw)(t, t, f->m);
  memcpy(c, t, NL * sizeof(uint64_t));
}

static int F(is_zero)(const uint64_t* a) {
  uint64_t o = 0;
  for (int i = 0; i < NL; i++) o |= a[i];
  return o == 0;
}

static void F(field_init)(F(field_t) * f, const uint64_t* m) {
  memcpy(f->m, m, sizeof f->m);
  uint64_t inv = 1; /* Newton: inv = m0^-1 mod 2^64 */
  for (int i = 0; i < 6; i++) inv *= 2 - m[0] * inv;
  f->n0 = (uint64_t)0 - inv;
  /* R mod m and R^2 mod m by repeated doubling of 1 */
  uint64_t x[NL];
  memset(x, 0, sizeof x);
  x[0] = 1;
  for (int i = 0; i < 128 * NL; i++) {
    if (i == 64 * NL) memcpy(f->one, x, sizeof x);
    F(fadd)(f, x, x, x);
  }
  memcpy(f->r2, x, sizeof x);
}

static void F(to_mont)(const F(field_t) * f, uint64_t* c, const uint64_t* a) { F(fmul)(f, c, a, f->r2); }

static void F(from_mont)(const F(field_t) * f, uint64_t* c, const uint64_t* a) {
  uint64_t one[NL];
  memset(one, 0, sizeof one);
  one[0] = 1;
  F(fmul)(f, c, a, one);
}

/* a^e (Montgomery domain), e given as NL limbs, plain binary */
static void F(fpow)(const F(field_t) * f, uint64_t* c, const uint64_t* a, const uint64_t* e) {
  uint64_t acc[NL];
  memcpy(acc, f->one, sizeof acc);
  for (int i = 64 * NL - 1; i >= 0; i--) {
    F(fmul)(f, acc, acc, acc);
    if ((e[i / 64] >> (i % 64)) & 1) F(fmul)(f, acc, acc, a);
  }
  memcpy(c, acc, sizeof acc);
}

static void F(finv)(const F(field_t) * f, uint64_t* c, const uint64_t* a) {
  uint64_t e[NL], two[NL];
  memset(two, 0, sizeof two);
  two[0] = 2;
  F(sub_raw)(e, f->m, two);
  F(fpow)(f, c, a, e);
}

/* ---- G1, Jacobian (X, Y, Z), a = 0; Z == 0 is infinity ---- */
typedef struct {
  uint64_t x[NL], y[NL], z[NL];
} F(jac_t);

static void F(jdbl)(const F(field_t) * f, F(jac_t) * R, const F(jac_t) * P) {
  if (F(is_zero)(P->z) || F(is_zero)(P->y)) {
    memset(R, 0, sizeof *R);
    return;
  }
  uint64_t A[NL], B[NL], C[NL], D[NL], E[NL], t[NL], X3[NL], Y3[NL], Z3[NL];
  F(fmul)(f, A, P->x, P->x);
  F(fmul)(f, B, P->y, P->y);
  F(fmul)(f, C, B, B);
  F(fadd)(f, t, P->x, B);
  F(fmul)(f, t, t, t);
  F(fsub)(f, t, t, A);
  F(fsub)(f, t, t, C);
  F(fadd)(f, D, t, t);
  F(fadd)(f, E, A, A);
  F(fadd)(f, E, E, A);
  F(fmul)(f, X3, E, E);
  F(fsub)(f, X3, X3, D);
  F(fsub)(f, X3, X3, D);
  F(fsub)(f, t, D, X3);
  F(fmul)(f, Y3, E, t);
  F(fadd)(f, C, C, C);
  F(fadd)(f, C, C, C);
  F(fadd)(f, C, C, C);
  F(fsub)(f, Y3, Y3, C);
  F(fmul)(f, Z3, P->y, P->z);
  F(fadd)(f, Z3, Z3, Z3);
  memcpy(R->x, X3, sizeof X3);
  memcpy(R->y, Y3, sizeof Y3);
  memcpy(R->z, Z3, sizeof Z3);
}

static void F(jadd)(const F(field_t) * f, F(jac_t) * R, const F(jac_t) * P, const F(jac_t) * Q) {
  if (F(is_zero)(P->z)) {
    *R = *Q;
    return;
  }
  if (F(is_zero)(Q->z)) {
    *R = *P;
    return;
  }
  uint64_t Z1Z1[NL], Z2Z2[NL], U1[NL], U2[NL], S1[NL], S2[NL], H[NL], I[NL], J[NL], rr[NL], V[NL], t[NL];
  F(fmul)(f, Z1Z1, P->z, P->z);
  F(fmul)(f, Z2Z2, Q->z, Q->z);
  F(fmul)(f, U1, P->x, Z2Z2);
  F(fmul)(f, U2, Q->x, Z1Z1);
  F(fmul)(f, S1, P->y, Q->z);
  F(fmul)(f, S1, S1, Z2Z2);
  F(fmul)(f, S2, Q->y, P->z);
  F(fmul)(f, S2, S2, Z1Z1);
  if (memcmp(U1, U2, sizeof U1) == 0) {
    if (memcmp(S1, S2, sizeof S1) == 0) {
      F(jdbl)(f, R, P);
    } else {
      memset(R, 0, sizeof *R);
    }
    return;
  }
  F(fsub)(f, H, U2, U1);
  F(fadd)(f, I, H, H);
  F(fmul)(f, I, I, I);
  F(fmul)(f, J, H, I);
  F(fsub)(f, rr, S2, S1);
  F(fadd)(f, rr, rr, rr);
  F(fmul)(f, V, U1, I);
  F(jac_t) out;
  F(fmul)(f, out.x, rr, rr);
  F(fsub)(f, out.x, out.x, J);
  F(fsub)(f, out.x, out.x, V);
  F(fsub)(f, out.x, out.x, V);
  F(fsub)(f, t, V, out.x);
  F(fmul)(f, out.y, rr, t);
  F(fmul)(f, t, S1, J);
  F(fadd)(f, t, t, t);
  F(fsub)(f, out.y, out.y, t);
  F(fadd)(f, t, P->z, Q->z);
  F(fmul)(f, t, t, t);
  F(fsub)(f, t, t, Z1Z1);
  F(fsub)(f, t, t, Z2Z2);
  F(fmul)(f, out.z, t, H);
  *R = out;
}

/* affine (Montgomery) -> Jacobian; all-zero affine encodes infinity */
static void F(from_affine)(const F(field_t) * f, F(jac_t) * R, const uint64_t* x, const uint64_t* y) {
  if (F(is_zero)(x) && F(is_zero)(y)) {
    memset(R, 0, sizeof *R);
    return;
  }
  memcpy(R->x, x, NL * 8);
  memcpy(R->y, y, NL * 8);
  memcpy(R->z, f->one, NL * 8);
}

/* Jacobian -> affine (Montgomery); returns 1 for infinity (x = y = 0) */
static int F(to_affine)(const F(field_t) * f, uint64_t* x, uint64_t* y, const F(jac_t) * P) {
  if (F(is_zero)(P->z)) {
    memset(x, 0, NL * 8);
    memset(y, 0, NL * 8);
    return 1;
  }
  uint64_t zi[NL], zi2[NL];
  F(finv)(f, zi, P->z);
  F(fmul)(f, zi2, zi, zi);
  F(fmul)(f, x, P->x, zi2);
  F(fmul)(f, zi2, zi2, zi);
  F(fmul)(f, y, P->y, zi2);
  return 0;
}

/* R = k P, left-to-right double-and-add over the plain integer k (4 limbs) */
static void F(jmul)(const F(field_t) * f, F(jac_t) * R, const F(jac_t) * P, const uint64_t* k) {
  F(jac_t) acc;
  memset(&acc, 0, sizeof acc);
  int top = 255;
  while (top >= 0 && !((k[top / 64] >> (top % 64)) & 1)) top--;
  for (int i = top; i >= 0; i--) {
    F(jdbl)(f, &acc, &acc);
    if ((k[i / 64] >> (i % 64)) & 1) F(jadd)(f, &acc, &acc, P);
  }
  *R = acc;
}

#undef F
#undef CAT
#undef CAT2
