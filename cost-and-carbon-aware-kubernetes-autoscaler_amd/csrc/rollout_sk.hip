// rollout_sk.hip — the general kernel on the lane-skewed schedule
// (rollout_kernel<DMAX, MAXN, 0, 1>, rollout.hip): worlds of two to four HPA /
// static deployments run their quiet steps per lane and their full steps in
// per-wave batches of stalled lanes (the single-deployment kernel's event
// batching, rollout_d1.hip, for several deployments). sk_eligible
// (ccka_abi.cpp) checks the preconditions.
#define CCKA_ROLLOUT_PART 1
#include "rollout.hip"

namespace ccka {

// [T][D][NL] -> [NL][T][DP] through an LDS tile of 64 columns x TT steps x DP
// (TT * DP = 32: each column's part of the tile is one 128-byte run of the
// output): reads of 64 consecutive columns, writes of whole runs
template <int DP>
__global__ void __launch_bounds__(256) trace_nt_kernel(const int32_t* __restrict__ in, int32_t* __restrict__ out,
                                                       int64_t NL, int64_t T, int D) {
  constexpr int TT = 32 / DP;
  __shared__ int32_t tile[64 * 32];  // [col][tt][d]
  const int64_t c0 = (int64_t)blockIdx.x * 64, t0 = (int64_t)blockIdx.y * TT;
  const int tid = threadIdx.x;
  for (int x = tid; x < TT * DP * 64; x += 256) {
    const int c = x & 63, r = x >> 6, tt = r / DP, d = r % DP;
    const int64_t col = c0 + c, t = t0 + tt;
    int32_t v = 0;
    if (d < D && col < NL && t < T) v = in[(t * D + d) * NL + col];
    tile[c * 32 + tt * DP + d] = v;
  }
  __syncthreads();
  for (int x = tid; x < 64 * 32; x += 256) {
    const int c = x >> 5, k = x & 31, tt = k / DP;
    const int64_t col = c0 + c, t = t0 + tt;
    if (col < NL && t < T) out[(col * T + t0) * DP + k] = tile[x];
  }
}

hipError_t launch_trace_nt(const int32_t* in, int32_t* out, int64_t NL, int64_t T, int32_t D, int32_t DP,
                           hipStream_t s) {
  if (NL <= 0 || T <= 0 || D < 1 || D > DP) return hipErrorInvalidValue;
  const dim3 grid((unsigned)((NL + 63) / 64), (unsigned)((T * DP + 31) / 32));
  switch (DP) {
    case 2: hipLaunchKernelGGL(trace_nt_kernel<2>, grid, dim3(256), 0, s, in, out, NL, T, D); break;
    case 4: hipLaunchKernelGGL(trace_nt_kernel<4>, grid, dim3(256), 0, s, in, out, NL, T, D); break;
    case 8: hipLaunchKernelGGL(trace_nt_kernel<8>, grid, dim3(256), 0, s, in, out, NL, T, D); break;
    case 16: hipLaunchKernelGGL(trace_nt_kernel<16>, grid, dim3(256), 0, s, in, out, NL, T, D); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_rollout_sk(const KParams& p, int block, size_t lds, hipStream_t s) {
  const unsigned grid = (unsigned)((p.N + block - 1) / block);
  int dmax, nmax;
  kernel_dims(p.D, p.maxn, &dmax, &nmax);
  if (dmax == 2 && nmax == 8)
    hipLaunchKernelGGL((rollout_kernel<2, 8, 0, 1>), dim3(grid), dim3(block), lds, s, p);
#ifdef CCKA_SK_ONE  // variant builds (tools/build_variants.py): <2, 8> only, compiled in a minute
  else
    return hipErrorInvalidValue;
#else
  else if (dmax == 2)
    hipLaunchKernelGGL((rollout_kernel<2, 16, 0, 1>), dim3(grid), dim3(block), lds, s, p);
  else if (dmax == 4 && nmax == 8)
    hipLaunchKernelGGL((rollout_kernel<4, 8, 0, 1>), dim3(grid), dim3(block), lds, s, p);
  else if (dmax == 4)  // rollout_sk416.hip
    return launch_rollout_sk416(p, block, lds, s);
  else
    return hipErrorInvalidValue;
#endif
  return hipGetLastError();
}

}  // namespace ccka
