// mlp.hip — BASELINE config 5: the learned MLP control policy
// (state 64 -> 256 -> 256 -> 8, ReLU) batched over millions of cluster states
// with bf16 MFMA on gfx950 (v_mfma_f32_32x32x16_bf16, fp32 accumulation).
//
// Orientation: every layer computes the TRANSPOSED activation tile
// (hidden units on rows, 32 cluster states on columns = lanes):
//   H1^T = W1^T X^T,  H2^T = W2^T H1^T,  Y^T = W3^T H2^T.
// A 32x32 accumulator of one layer then IS the B operand of the next
// (column on the lane, rows in registers): registers 8s..8s+7, converted to
// bf16, are k-step s of the next product with the permuted k order
// k = 16s + 8(j>>2) + 4h + (j&3) (j = element, h = lane half). The host lays
// the weight fragments out in exactly that order (ccka_abi.cpp,
// mlp_fragments), so no activation ever moves between lanes or through LDS.
//
// Residency: W1 fragments (32 KB) live in each wave's registers, W2 (128 KB)
// and W3 (16 KB, rows 8..31 zero) fragments plus the biases in LDS; one
// persistent 4-wave workgroup per CU, each wave streaming 32-state tiles of X
// from HBM with the next tile's loads in flight during the current tile's
// 176 MFMAs.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kparams.h"

namespace ccka {

namespace {

typedef mlp_bf16x8 bf16x8;
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int WAVE = 64;

typedef short short2v __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));

// registers 8s..8s+7 as one bf16 operand fragment with ReLU: pairs rounded to
// nearest even (v_cvt_pk_bf16_f32), then ReLU on the bf16 bit patterns as
// packed int16 max with 0 (v_pk_max_i16: every negative value, -0 included,
// has the sign bit set) -- the same bits as rounding relu(x)
__device__ __forceinline__ bf16x8 relu_pack(const f32x16& a, int s) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; j += 2) {
    const bf16x2v b = __builtin_convertvector((f32x2){a[8 * s + j], a[8 * s + j + 1]}, bf16x2v);
    const short2v v = __builtin_elementwise_max(__builtin_bit_cast(short2v, b), (short2v){0, 0});
    r[j] = v.x;
    r[j + 1] = v.y;
  }
  return r;
}

// accumulator initialised with the bias of its rows: row = (reg&3) + 8(reg>>2) + 4h
__device__ __forceinline__ f32x16 bias_tile(const float* b, int h) {
  f32x16 a;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(b + 8 * g + 4 * h);
    a[4 * g + 0] = v[0];
    a[4 * g + 1] = v[1];
    a[4 * g + 2] = v[2];
    a[4 * g + 3] = v[3];
  }
  return a;
}

__device__ __forceinline__ f32x16 mfma(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

}  // namespace

__global__ void __launch_bounds__(256, 1) mlp_kernel(MlpParams p) {
  __shared__ __attribute__((aligned(16))) float s_b1[MLP_HID], s_b2[MLP_HID], s_b3[32];
  __shared__ bf16x8 s_w3[(MLP_HID / 16) * WAVE];                  // 16 KiB
  __shared__ bf16x8 s_w2[MLP_HID / 32 * (MLP_HID / 16) * WAVE];  // 128 KiB
  const int tid = threadIdx.x, lane = tid & (WAVE - 1), wave = tid / WAVE;
  const int r = lane & 31, h = lane >> 5;
  for (int x = tid; x < MLP_HID / 32 * (MLP_HID / 16) * WAVE; x += blockDim.x) s_w2[x] = p.w2f[x];
  for (int x = tid; x < (MLP_HID / 16) * WAVE; x += blockDim.x) s_w3[x] = p.w3f[x];
  for (int x = tid; x < MLP_HID; x += blockDim.x) { s_b1[x] = p.b1[x]; s_b2[x] = p.b2[x]; }
  if (tid < 32) s_b3[tid] = tid < MLP_OUT ? p.b3[tid] : 0.0f;
  // layer-1 weight fragments stay in registers for the whole kernel
  bf16x8 w1[MLP_HID / 32][MLP_IN / 16];
#pragma unroll
  for (int n = 0; n < MLP_HID / 32; ++n)
#pragma unroll
    for (int s = 0; s < MLP_IN / 16; ++s) {
      w1[n][s] = p.w1f[(n * (MLP_IN / 16) + s) * WAVE + lane];
      asm volatile("" : "+a"(w1[n][s]));  // accumulation registers: MFMA reads its A operand from them
    }
  __syncthreads();

  const int64_t ntiles = (p.N + 31) / 32;
  const int64_t nw = (int64_t)gridDim.x * (blockDim.x / WAVE);
  int64_t tile = (int64_t)blockIdx.x * (blockDim.x / WAVE) + wave;
  // X^T fragments (B operand of layer 1): state r, features 16s + 8h .. +7
  auto load_x = [&](int64_t tl, bf16x8* xf) {
    const int64_t row = tl * 32 + r;
    const bool ok = tl < ntiles && row < p.N;
    const bf16x8* src = reinterpret_cast<const bf16x8*>(p.x + (ok ? row : 0) * MLP_IN + 8 * h);
#pragma unroll
    for (int s = 0; s < MLP_IN / 16; ++s) {
      const bf16x8 v = src[2 * s];
      xf[s] = ok ? v : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
  };
  bf16x8 xf[MLP_IN / 16], xn[MLP_IN / 16];
  load_x(tile, xf);
  for (; tile < ntiles; tile += nw) {
    load_x(tile + nw, xn);  // next tile in flight during this tile's MFMAs
    // ---- layer 1: H1^T = relu(W1^T X^T + b1) ----
    // row blocks software-pipelined: block n+1's MFMAs are issued before
    // block n's ReLU/bf16 epilogue, which then runs in their shadow
    bf16x8 hf[MLP_HID / 16];
    f32x16 acur = bias_tile(s_b1, h);
#pragma unroll
    for (int s = 0; s < MLP_IN / 16; ++s) acur = mfma(w1[0][s], xf[s], acur);
#pragma unroll
    for (int n = 0; n < MLP_HID / 32; ++n) {
      f32x16 anext;
      if (n + 1 < MLP_HID / 32) {
        anext = bias_tile(s_b1 + 32 * (n + 1), h);
#pragma unroll
        for (int s = 0; s < MLP_IN / 16; ++s) anext = mfma(w1[n + 1][s], xf[s], anext);
      }
      hf[2 * n] = relu_pack(acur, 0);
      hf[2 * n + 1] = relu_pack(acur, 1);
      if (n + 1 < MLP_HID / 32) acur = anext;
    }
    // ---- layer 2: H2^T = relu(W2^T H1^T + b2) ----
    f32x16 a2[MLP_HID / 32];
#pragma unroll
    for (int n = 0; n < MLP_HID / 32; ++n) a2[n] = bias_tile(s_b2 + 32 * n, h);
    // W2 fragments software-pipelined one k-step ahead (LDS latency hidden
    // behind the current k-step's 8 MFMAs); the barriers keep exactly two
    // k-steps of fragments in registers (the scheduler would otherwise hoist
    // all 128 fragment reads and spill)
    bf16x8 wf[MLP_HID / 32], wn[MLP_HID / 32];
#pragma unroll
    for (int n = 0; n < MLP_HID / 32; ++n) wf[n] = s_w2[n * (MLP_HID / 16) * WAVE + lane];
#pragma unroll
    for (int kk = 0; kk < MLP_HID / 16; ++kk) {
      if (kk + 1 < MLP_HID / 16) {
#pragma unroll
        for (int n = 0; n < MLP_HID / 32; ++n) wn[n] = s_w2[(n * (MLP_HID / 16) + kk + 1) * WAVE + lane];
      }
      asm volatile("" ::: "memory");
#pragma unroll
      for (int n = 0; n < MLP_HID / 32; ++n) a2[n] = mfma(wf[n], hf[kk], a2[n]);
#pragma unroll
      for (int n = 0; n < MLP_HID / 32; ++n) wf[n] = wn[n];
    }
    // ---- layer 3: Y^T = W3^T H2^T + b3 (rows 8..31 of W3^T are zero) ----
    // interleaved with layer 2's epilogue: k-steps 2n, 2n+1 need only block n
    f32x16 a3 = bias_tile(s_b3, h);
#pragma unroll
    for (int n = 0; n < MLP_HID / 32; ++n) {
      const bf16x8 g0 = relu_pack(a2[n], 0), g1 = relu_pack(a2[n], 1);
      a3 = mfma(s_w3[(2 * n) * WAVE + lane], g0, a3);
      a3 = mfma(s_w3[(2 * n + 1) * WAVE + lane], g1, a3);
    }
    // registers 0..3 hold outputs 4h..4h+3 of state r
    const int64_t row = tile * 32 + r;
    if (row < p.N) *reinterpret_cast<f32x4*>(p.y + row * MLP_OUT + 4 * h) = f32x4{a3[0], a3[1], a3[2], a3[3]};
#pragma unroll
    for (int s = 0; s < MLP_IN / 16; ++s) xf[s] = xn[s];
  }
}

// Synthetic cluster states: Irwin-Hall sums of Philox words (~N(0,1)), bf16.
__device__ __forceinline__ void philox_s(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0,
                                         uint32_t k1, uint32_t out[4]) {
#pragma unroll
  for (int q = 0; q < 10; ++q) {
    const uint32_t lo0 = 0xD2511F53u * c0, hi0 = __umulhi(0xD2511F53u, c0);
    const uint32_t lo1 = 0xCD9E8D57u * c2, hi1 = __umulhi(0xCD9E8D57u, c2);
    const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

__global__ void __launch_bounds__(256) mlp_gen_states_kernel(uint16_t* x, int64_t count, uint64_t seed) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= count) return;
  uint32_t u[4];
  philox_s((uint32_t)e, (uint32_t)(e >> 32), 0x5EEDu, 0x57A7Eu, (uint32_t)seed, (uint32_t)(seed >> 32), u);
  const float v = ((float)(u[0] >> 16) + (float)(u[1] >> 16) + (float)(u[2] >> 16) + (float)(u[3] >> 16) - 131070.0f) *
                  (1.0f / 37837.0f);
  x[e] = __builtin_bit_cast(uint16_t, (__bf16)v);
}

hipError_t launch_mlp(const MlpParams& p, int cus, hipStream_t s) {
  hipLaunchKernelGGL(mlp_kernel, dim3((unsigned)cus), dim3(256), 0, s, p);
  return hipGetLastError();
}

hipError_t launch_mlp_gen_states(uint16_t* x, int64_t count, uint64_t seed, hipStream_t s) {
  hipLaunchKernelGGL(mlp_gen_states_kernel, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, s, x, count, seed);
  return hipGetLastError();
}

}  // namespace ccka
