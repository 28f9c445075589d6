// sweep.hip — BASELINE config 4: policy sweep of parameter grids over shared
// load traces. Per-grid sums of the rollout results (fixed-order, so
// deterministic) and the cost / gCO2 / SLO-minutes Pareto frontier
// (local non-dominated candidates, exchanged with an RCCL
// all-gather in ccka_abi.cpp, then the same filter on every rank).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kparams.h"

namespace ccka {

// one workgroup per grid: strided partial sums in a fixed order, then a
// fixed-shape tree over the workgroup
__global__ void __launch_bounds__(256) grid_stats_kernel(GridSrc g, ccka_grid_stats* out) {
  __shared__ long long s_cost[256], s_slo[256];
  __shared__ double s_g[256], s_e[256];
  const int tid = threadIdx.x;
  const int64_t lo = (int64_t)blockIdx.x * g.grid_size;
  long long c = 0, sl = 0;
  double gc = 0.0, en = 0.0;
  for (int64_t k = tid; k < g.grid_size; k += blockDim.x) {
    c += g.cost[lo + k];
    sl += g.slo[lo + k];
    gc += g.gco2[lo + k];
    en += g.energy[lo + k];
  }
  s_cost[tid] = c;
  s_slo[tid] = sl;
  s_g[tid] = gc;
  s_e[tid] = en;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (tid < w) {
      s_cost[tid] += s_cost[tid + w];
      s_slo[tid] += s_slo[tid + w];
      s_g[tid] += s_g[tid + w];
      s_e[tid] += s_e[tid + w];
    }
    __syncthreads();
  }
  if (tid == 0) {
    ccka_grid_stats o;
    o.grid = g.first_grid + blockIdx.x;
    o.scenarios = g.grid_size;
    o.cost_uphmin = s_cost[0];
    o.slo_minutes = s_slo[0];
    o.gco2 = s_g[0];
    o.energy_wmin = s_e[0];
    out[blockIdx.x] = o;
  }
}

__device__ __forceinline__ bool dominates(const ccka_grid_stats& a, const ccka_grid_stats& b) {
  const bool le = a.cost_uphmin <= b.cost_uphmin && a.gco2 <= b.gco2 && a.slo_minutes <= b.slo_minutes;
  const bool lt = a.cost_uphmin < b.cost_uphmin || a.gco2 < b.gco2 || a.slo_minutes < b.slo_minutes;
  return le && lt;
}

// flags[i] = 1 iff entry i is dominated by any other entry (one thread per entry)
__global__ void __launch_bounds__(256) pareto_mark_kernel(const ccka_grid_stats* in, int n_host,
                                                          const int32_t* n_dev, uint8_t* flags) {
  const int n = n_dev ? *n_dev : n_host;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const ccka_grid_stats me = in[i];
  uint8_t dom = 0;
  for (int j = 0; j < n && !dom; ++j)
    if (j != i && dominates(in[j], me)) dom = 1;
  flags[i] = dom;
}

// ordered compaction of the non-dominated entries (one workgroup, block scan)
__global__ void __launch_bounds__(1024) pareto_compact_kernel(const ccka_grid_stats* in, int n_host,
                                                              const int32_t* n_dev, const uint8_t* flags,
                                                              ccka_grid_stats* out, int32_t* count) {
  __shared__ int s_scan[1024];
  __shared__ int s_base;
  const int n = n_dev ? *n_dev : n_host;
  const int tid = threadIdx.x;
  if (tid == 0) s_base = 0;
  __syncthreads();
  for (int base = 0; base < n; base += blockDim.x) {
    const int i = base + tid;
    const int keep = (i < n && !flags[i]) ? 1 : 0;
    s_scan[tid] = keep;
    __syncthreads();
    for (int off = 1; off < (int)blockDim.x; off <<= 1) {  // inclusive Hillis-Steele scan
      const int v = tid >= off ? s_scan[tid - off] : 0;
      __syncthreads();
      s_scan[tid] += v;
      __syncthreads();
    }
    if (keep) out[s_base + s_scan[tid] - 1] = in[i];
    __syncthreads();
    if (tid == blockDim.x - 1) s_base += s_scan[tid];
    __syncthreads();
  }
  if (tid == 0) *count = s_base;
}

// valid prefixes of the all-gathered [ranks][cap] buffers, in rank order
// (ranks own ascending grid ranges, so the union stays sorted by grid id)
__global__ void __launch_bounds__(256) pareto_union_kernel(const ccka_grid_stats* gathered, const int64_t* counts,
                                                           int ranks, int cap, ccka_grid_stats* out, int32_t* n_dev) {
  int off = 0;
  for (int q = 0; q < ranks; ++q) {
    const int c = (int)counts[q];
    for (int k = threadIdx.x; k < c; k += blockDim.x) out[off + k] = gathered[(int64_t)q * cap + k];
    off += c;
  }
  if (threadIdx.x == 0) *n_dev = off;
}

hipError_t launch_grid_stats(const GridSrc& g, ccka_grid_stats* out, hipStream_t s) {
  hipLaunchKernelGGL(grid_stats_kernel, dim3((unsigned)g.n_grids), dim3(256), 0, s, g, out);
  return hipGetLastError();
}

hipError_t launch_pareto(const ccka_grid_stats* in, int n, const int32_t* n_dev, uint8_t* flags,
                         ccka_grid_stats* out, int32_t* count_dev, hipStream_t s) {
  // n is the capacity bound when the live count is device-resident
  hipLaunchKernelGGL(pareto_mark_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, in, n, n_dev, flags);
  hipLaunchKernelGGL(pareto_compact_kernel, dim3(1), dim3(1024), 0, s, in, n, n_dev, flags, out, count_dev);
  return hipGetLastError();
}

hipError_t launch_pareto_union(const ccka_grid_stats* gathered, const int64_t* counts, int ranks, int cap,
                               ccka_grid_stats* out, int32_t* n_dev, hipStream_t s) {
  hipLaunchKernelGGL(pareto_union_kernel, dim3(1), dim3(256), 0, s, gathered, counts, ranks, cap, out, n_dev);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Copy ceiling (bench.py's roofline denominator beside the 8 TB/s peak): a
// plain streaming device copy, 16 bytes per lane (dwordx4), one element per
// thread with the grid covering the buffer, nontemporal on both sides. The
// fastest of the variants tools/probe/copyprobe.hip measured on MI355X (6.5
// TB/s read + write; grid-stride loops with 4-8 accesses in flight per lane:
// 4.4-4.8 TB/s). Profiling aid, not part of the rollout.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) copy16_kernel(const int4* __restrict__ in, int4* __restrict__ out, int64_t n) {
  typedef int i32x4 __attribute__((ext_vector_type(4)));
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) __builtin_nontemporal_store(__builtin_nontemporal_load((const i32x4*)(in + i)), (i32x4*)(out + i));
}

hipError_t launch_copy16(const void* in, void* out, int64_t bytes, int cus, hipStream_t s) {
  (void)cus;
  const int64_t n = bytes / 16;
  const int64_t grid = (n + 255) / 256;
  if (grid > 0x7fffffffLL) return hipErrorInvalidValue;
  hipLaunchKernelGGL(copy16_kernel, dim3((unsigned)grid), dim3(256), 0, s, (const int4*)in, (int4*)out, n);
  return hipGetLastError();
}

}  // namespace ccka
