// Pieces shared by pairing.hip (lane-per-pairing kernels, G2 setup and MSM)
// and verify_wave.hip (wave-per-opening verify): the twist Frobenius and a
// G1 double-and-add.
#pragma once
#include <hip/hip_runtime.h>

#include "kzgx_internal.hpp"
#include "tower.hpp"

namespace kzgx {

// pi(q) on the D-type twist: (conj(x) xi^((p-1)/3), conj(y) xi^((p-1)/2))
template <class C>
KZGX_DEV G2A<C> twist_frob(const G2A<C>& q) {
  using P = typename PairOf<C>::T;
  G2A<C> r;
  r.x = f2_mul<C>(f2_conj<C>(q.x), f2_const<C>(P::TWX));
  r.y = f2_mul<C>(f2_conj<C>(q.y), f2_const<C>(P::TWY));
  return r;
}

// [k] P for a canonical 256-bit scalar (XYZZ double-and-add, complete)
template <class C>
KZGX_TW Xyzz<C> g1_mul_words(const Affine<C>& p, const uint32_t (&e)[8]) {
  Xyzz<C> acc = xyzz_inf<C>();
  for (int b = 255; b >= 0; b--) {
    acc = xyzz_dbl<C>(acc);
    if ((e[b >> 5] >> (b & 31)) & 1u) acc = xyzz_add_affine<C>(acc, p);
  }
  return acc;
}

}  // namespace kzgx
