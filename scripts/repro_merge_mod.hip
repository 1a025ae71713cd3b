// k_msm_merge<BN254G1, true> alone, for device-only builds loaded with
// hipModuleLoad by scripts/repro_merge.hip (REPRO_CO=path): a pass-limited
// build (-mllvm -opt-bisect-limit=N) of this translation unit changes the
// inlined merge kernel and nothing else.
#include "../kzg-commitments_amd/csrc/msm_merge.hpp"

template __global__ void kzgx::k_msm_merge<kzgx::BN254G1, true>(const uint32_t*, const uint32_t*, const uint32_t*,
                                                                 const uint8_t*, uint32_t, uint32_t, uint32_t,
                                                                 uint32_t*, uint32_t*, uint32_t*, uint32_t*,
                                                                 uint32_t*);
