// rollout_multi.hip — the general kernel's lockstep instantiations for four or
// more deployments (rollout_kernel<4|8|12|16, 8|16>). The kernel template is
// rollout.hip's; this unit only instantiates it, so the instantiations compile
// in parallel with rollout.hip's.
#define CCKA_ROLLOUT_PART 1
#include "rollout.hip"

namespace ccka {

hipError_t launch_rollout_multi(const KParams& p, int block, size_t lds, hipStream_t s) {
  const unsigned grid = (unsigned)((p.N + block - 1) / block);
  int dmax, nmax;
  kernel_dims(p.D, p.maxn, &dmax, &nmax);
  if (dmax == 4 && nmax == 8)
    hipLaunchKernelGGL((rollout_kernel<4, 8>), dim3(grid), dim3(block), lds, s, p);
  else if (dmax == 4)
    hipLaunchKernelGGL((rollout_kernel<4, 16>), dim3(grid), dim3(block), lds, s, p);
  else if (dmax == 8)
    hipLaunchKernelGGL((rollout_kernel<8, 16>), dim3(grid), dim3(block), lds, s, p);
  else if (dmax == 12)
    hipLaunchKernelGGL((rollout_kernel<12, 16>), dim3(grid), dim3(block), lds, s, p);
  else if (dmax == 16)
    hipLaunchKernelGGL((rollout_kernel<16, 16>), dim3(grid), dim3(block), lds, s, p);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

}  // namespace ccka
