// Shader-clock probe under a bf16 MFMA load: every wave of a 256-CU grid runs
// back-to-back v_mfma_f32_32x32x16_bf16 on 4 accumulators; wave 0 of block 0
// samples s_memtime (shader clock) and s_memrealtime (100 MHz) around it.
// Prints the shader clock and the achieved dense bf16 rate.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ void __launch_bounds__(256, 1) probe(int iters, unsigned long long* t, float* sink) {
  const int lane = threadIdx.x & 63;
  bf16x8 a = {(short)lane, 1, 2, 3, 4, 5, 6, 7}, b = {1, 2, 3, 4, 5, 6, 7, (short)lane};
  f32x16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
  unsigned long long m0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < iters; ++i) {
    c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c3, 0, 0, 0);
  }
  float s = 0.f;
  for (int k = 0; k < 16; ++k) s += c0[k] + c1[k] + c2[k] + c3[k];
  unsigned long long m1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (blockIdx.x == 0 && threadIdx.x == 0) { t[0] = m1 - m0; t[1] = r1 - r0; }
  if (s == 12345.f) sink[0] = s;
}

int main() {
  int dev = 0, cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  unsigned long long* t; float* sink;
  hipMalloc(&t, 16); hipMalloc(&sink, 4);
  const int iters = 400000;
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  probe<<<cus, 256>>>(100, t, sink);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  probe<<<cus, 256>>>(iters, t, sink);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0; hipEventElapsedTime(&ms, e0, e1);
  unsigned long long h[2]; hipMemcpy(h, t, 16, hipMemcpyDeviceToHost);
  const double flops = (double)cus * 4 * iters * 4 * 32.0 * 32 * 16 * 2;
  printf("{\"cus\": %d, \"shader_clock_ghz\": %.3f, \"ms\": %.3f, \"tflops\": %.1f, \"cycles_per_mfma\": %.2f}\n", cus,
         (double)h[0] / (double)h[1] * 0.1, ms, flops / (ms * 1e-3) / 1e12, (double)h[0] / (iters * 4.0));
  return 0;
}
