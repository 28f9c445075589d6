// rollout_sk416.hip — the lane-skewed schedule's four-deployment, 16-slot
// instantiation (rollout_kernel<4, 16, 0, 1>, rollout.hip), in its own unit:
// it is compiled with the lane-local provisioning branch (SK_LANE_F2), which
// never runs here (its per-lane NodeClaim columns, 180 KB, do not fit in LDS,
// and the host enables it nowhere). With the branch present the register
// allocator places this instantiation's spills off the hot loops: 214 -> 176 ms
// at 1e5 x 1440 (bench --deployments 4, same results; tools/sk_ab.py).
#define CCKA_ROLLOUT_PART 1
#define SK_LANE_F2 1
#include "rollout.hip"

namespace ccka {

hipError_t launch_rollout_sk416(const KParams& p, int block, size_t lds, hipStream_t s) {
  const unsigned grid = (unsigned)((p.N + block - 1) / block);
  hipLaunchKernelGGL((rollout_kernel<4, 16, 0, 1>), dim3(grid), dim3(block), lds, s, p);
  return hipGetLastError();
}

}  // namespace ccka
