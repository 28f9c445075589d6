// rollout_sk16.hip — the lane-skewed schedule's instantiations for eight and
// sixteen deployments (rollout_kernel<8|16, 16, 0, 1>, rollout.hip; launched by
// launch_rollout_sk, rollout_sk.hip), in their own unit so that they compile in
// parallel with the smaller ones.
#define CCKA_ROLLOUT_PART 1
#include "rollout.hip"

namespace ccka {

hipError_t launch_rollout_sk16(const KParams& p, int block, size_t lds, hipStream_t s) {
  const unsigned grid = (unsigned)((p.N + block - 1) / block);
  int dmax, nmax;
  kernel_dims(p.D, p.maxn, &dmax, &nmax);
  if (dmax == 8)
    hipLaunchKernelGGL((rollout_kernel<8, 16, 0, 1>), dim3(grid), dim3(block), lds, s, p);
  else if (dmax == 16)
    hipLaunchKernelGGL((rollout_kernel<16, 16, 0, 1>), dim3(grid), dim3(block), lds, s, p);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

}  // namespace ccka
