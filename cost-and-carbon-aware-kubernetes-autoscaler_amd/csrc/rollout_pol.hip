// rollout_pol.hip — the fused closed loop's instantiations of rollout.hip's
// kernel template (rollout_kernel<1, 8, POL>: features -> MFMA MLP -> action
// -> step, the whole horizon in one launch), compiled in parallel with
// rollout.hip.
#define CCKA_ROLLOUT_PART 1
#include "rollout.hip"

namespace ccka {

// the fused closed loop: the whole horizon in one launch, one 256-thread block
// (4 waves, one per SIMD) per 256 scenarios
hipError_t launch_rollout_policy(const KParams& p, size_t lds, int pol, hipStream_t s) {
  const unsigned grid = (unsigned)((p.N + 255) / 256);
  if (p.D != 1 || p.maxn > 8 || (pol != 1 && pol != 2)) return hipErrorInvalidValue;
  if (pol == 1) hipLaunchKernelGGL((rollout_kernel<1, 8, 1>), dim3(grid), dim3(256), lds, s, p);
  else hipLaunchKernelGGL((rollout_kernel<1, 8, 2>), dim3(grid), dim3(256), lds, s, p);
  return hipGetLastError();
}

}  // namespace ccka
