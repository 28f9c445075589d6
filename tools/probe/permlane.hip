// permlane.hip — semantics of v_permlane32_swap_b32 (__builtin_amdgcn_permlane32_swap) on gfx950
// (diagnostic): lane l passes (X = 100 + l, Y = 200 + l); prints what lanes 0,
// 1, 32, 33 get back in each element. Build: hipcc -O3 --offload-arch=gfx950
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned* out) {
  const unsigned l = threadIdx.x;
  const auto r = __builtin_amdgcn_permlane32_swap(100u + l, 200u + l, false, false);
  out[l * 2] = r[0];
  out[l * 2 + 1] = r[1];
}
int main() {
  unsigned* d;
  hipMalloc(&d, 128 * 4);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  unsigned h[128];
  hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
  for (int l : {0, 1, 31, 32, 33, 63}) printf("lane %2d: first %u second %u\n", l, h[2 * l], h[2 * l + 1]);
  return 0;
}
