// One window group of the fixed-base MSM's per-window code (fixed_msm.hpp),
// compiled once per group by the Makefile with
//   -DKZGX_INST_CURVE=BN254G1|BLS12381G1 -DKZGX_INST_TAG=<name>
//   -DKZGX_INST_WINDOWS="KZGX_W(c) KZGX_W(c) ..."
// so the 24 (curve, window) instantiations -- each three accumulation
// kernels of a full XYZZ addition inlined -- compile in parallel objects
// instead of one 12-minute translation unit ("build").
#define KZGX_FIXED_INST 1
#include "fixed_msm.hpp"

#ifndef KZGX_INST_CURVE
#error "KZGX_INST_CURVE / KZGX_INST_WINDOWS / KZGX_INST_TAG come from the Makefile"
#endif

#define KZGX_CAT2(a, b) a##b
#define KZGX_CAT(a, b) KZGX_CAT2(a, b)

namespace kzgx {

#define KZGX_W(cb)                                                                                               \
  template int fixed_msm_win<KZGX_INST_CURVE, cb>(Ctx*, FixedTable&, const uint32_t*, size_t, size_t, size_t, uint32_t*, \
                                                  uint32_t*, hipStream_t, uint32_t*);
KZGX_INST_WINDOWS
#undef KZGX_W

// device bring-up (kzgx_setup.hpp): one launch loads this code object
__global__ void KZGX_CAT(k_warm_fixed_, KZGX_INST_TAG)() {}
int KZGX_CAT(warm_fixed_, KZGX_INST_TAG)(hipStream_t st) {
  hipLaunchKernelGGL(KZGX_CAT(k_warm_fixed_, KZGX_INST_TAG), dim3(1), dim3(64), 0, st);
  KZGX_TRY_HIP(hipGetLastError());
  return KZGX_OK;
}

}  // namespace kzgx
