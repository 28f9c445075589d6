// Device copy ceiling probe: variants of a 16-B-per-lane streaming copy,
// GB/s of read + write over a 2 GiB buffer, median of 7 launches each.
// build: hipcc --offload-arch=gfx950 -O3 -o tools/probe/copyprobe tools/probe/copyprobe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef int i32x4 __attribute__((ext_vector_type(4)));

// one element per thread, grid covers the buffer
template <bool NT>
__global__ void __launch_bounds__(256) flat1(const i32x4* __restrict__ in, i32x4* __restrict__ out, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  if constexpr (NT) __builtin_nontemporal_store(__builtin_nontemporal_load(in + i), out + i);
  else out[i] = in[i];
}

// U elements per thread, consecutive blocks of 256*U elements
template <int U, bool NT>
__global__ void __launch_bounds__(256) flatU(const i32x4* __restrict__ in, i32x4* __restrict__ out, int64_t n) {
  const int64_t b = (int64_t)blockIdx.x * 256 * U + threadIdx.x;
  i32x4 v[U];
#pragma unroll
  for (int k = 0; k < U; ++k) {
    const int64_t i = b + k * 256;
    if (i < n) v[k] = NT ? __builtin_nontemporal_load(in + i) : in[i];
  }
#pragma unroll
  for (int k = 0; k < U; ++k) {
    const int64_t i = b + k * 256;
    if (i < n) {
      if constexpr (NT) __builtin_nontemporal_store(v[k], out + i);
      else out[i] = v[k];
    }
  }
}

// grid-stride, U in flight
template <int U, bool NT>
__global__ void __launch_bounds__(256) stride(const i32x4* __restrict__ in, i32x4* __restrict__ out, int64_t n) {
  const int64_t s = (int64_t)gridDim.x * 256;
  int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  for (; i + (U - 1) * s < n; i += U * s) {
    i32x4 v[U];
#pragma unroll
    for (int k = 0; k < U; ++k) v[k] = NT ? __builtin_nontemporal_load(in + i + k * s) : in[i + k * s];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      if constexpr (NT) __builtin_nontemporal_store(v[k], out + i + k * s);
      else out[i + k * s] = v[k];
    }
  }
  for (; i < n; i += s) out[i] = in[i];
}

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } \
  } while (0)

int main() {
  const int64_t bytes = 1ll << 31, n = bytes / 16;
  i32x4 *a, *b;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&b, bytes));
  CK(hipMemset(a, 1, bytes));
  CK(hipMemset(b, 0, bytes));
  hipDeviceProp_t pr;
  CK(hipGetDeviceProperties(&pr, 0));
  const int cus = pr.multiProcessorCount;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto run = [&](const char* name, auto launch) {
    std::vector<float> ms;
    for (int r = 0; r < 9; ++r) {
      hipEventRecord(e0);
      launch();
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float m = 0;
      hipEventElapsedTime(&m, e0, e1);
      if (r >= 2) ms.push_back(m);
    }
    std::sort(ms.begin(), ms.end());
    const float med = ms[ms.size() / 2];
    printf("%-28s %8.3f ms  %7.0f GB/s (read+write)\n", name, med, 2.0 * bytes / (med * 1e-3) / 1e9);
  };
  const unsigned g1 = (unsigned)((n + 255) / 256);
  run("flat1", [&] { hipLaunchKernelGGL(flat1<false>, dim3(g1), dim3(256), 0, 0, a, b, n); });
  run("flat1 nt", [&] { hipLaunchKernelGGL(flat1<true>, dim3(g1), dim3(256), 0, 0, a, b, n); });
  run("flat4", [&] { hipLaunchKernelGGL((flatU<4, false>), dim3((g1 + 3) / 4), dim3(256), 0, 0, a, b, n); });
  run("flat4 nt", [&] { hipLaunchKernelGGL((flatU<4, true>), dim3((g1 + 3) / 4), dim3(256), 0, 0, a, b, n); });
  run("flat8", [&] { hipLaunchKernelGGL((flatU<8, false>), dim3((g1 + 7) / 8), dim3(256), 0, 0, a, b, n); });
  for (int m : {8, 16, 32, 64}) {
    char nm[64];
    snprintf(nm, sizeof nm, "stride4 x%d/CU", m);
    run(nm, [&] { hipLaunchKernelGGL((stride<4, false>), dim3(cus * m), dim3(256), 0, 0, a, b, n); });
    snprintf(nm, sizeof nm, "stride8 nt x%d/CU", m);
    run(nm, [&] { hipLaunchKernelGGL((stride<8, true>), dim3(cus * m), dim3(256), 0, 0, a, b, n); });
    snprintf(nm, sizeof nm, "stride8 x%d/CU", m);
    run(nm, [&] { hipLaunchKernelGGL((stride<8, false>), dim3(cus * m), dim3(256), 0, 0, a, b, n); });
  }
  CK(hipDeviceSynchronize());
  return 0;
}
