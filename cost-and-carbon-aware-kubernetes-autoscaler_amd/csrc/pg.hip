// pg.hip — differentiable control for the learned policy (BASELINE config 5,
// "differentiable-control rollout"): a score-function (likelihood-ratio)
// gradient of the closed loop's objective with respect to the MLP weights.
//
// The rollout's dynamics are integer and piecewise constant, so the objective
// J = cost + w_c gCO2 + w_s SLO has no useful pathwise derivative. The policy
// is made stochastic instead: at every step each scenario samples one of the
// 8 action bins from softmax(y) (counter-based Philox, reproducible), and
//   grad E[J] = E[(J - b) sum_t grad log pi(a_t | x_t)],
// whose per-row factor is the softmax cross-entropy gradient
// g_y = c (e_a - softmax(y)) with c = (J - b) / N. The MLP backward then runs
// on bf16 MFMA with fp32 accumulation:
//   pg_rows_kernel   recomputes H1, H2, y per 32-state tile (the forward's
//                    transposed formulation), forms g_y, and back-propagates
//                    dH2^T = W3 g_y^T (masked by H2 > 0) and dH1^T = W2 dH2^T
//                    (masked by H1 > 0) with the same in-register operand
//                    chaining; it stores X^T, H1^T, H2^T, dH1^T, dH2^T, g_y^T
//                    row-blocked ([row / 16][unit][16]: a unit's 16 rows of a
//                    block in one 32-byte run), transposed through LDS so each
//                    store instruction writes whole 512-byte runs
//   pg_wgrad_kernel  C[a][b] = sum_m A[a][m] B[b][m] over millions of rows:
//                    one 8-wave workgroup per CU owns a chunk of rows and the
//                    whole output, 16 rows per MFMA k-step; an operand fragment
//                    (32 units x 16 rows) is ONE contiguous 1 KB run of the
//                    row-blocked arrays; row-split partials summed in a fixed
//                    order (deterministic)
// dW1 = X^T dH1, dW2 = H1^T dH2, dW3 = H2^T g_y, db = the same with a ones row.
// Anchor: the controller chooses "the cheapest and cleanest number of pods and
// node types that still meet the SLO" (CS218_Project_Proposal.pdf p.1) and the
// dashboards plot cost / carbon / SLO trade-offs (p.5). SEMANTICS 5.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "kparams.h"

namespace ccka {

namespace {

typedef mlp_bf16x8 bf16x8;
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short short2v __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));

constexpr int WAVE = 64;

__device__ __forceinline__ f32x16 mfma(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int k = 0; k < 16; ++k) z[k] = 0.f;
  return z;
}

// registers 8s..8s+7 -> bf16 (round to nearest even), then ReLU on the bits
// (as mlp.hip's relu_pack: the forward's exact H1 / H2 operands)
typedef uint32_t u32x4_ __attribute__((ext_vector_type(4)));
__device__ __forceinline__ bf16x8 relu_pack(const f32x16& a, int s) {
  u32x4_ o;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    const bf16x2v b = __builtin_convertvector((f32x2){a[8 * s + 2 * w], a[8 * s + 2 * w + 1]}, bf16x2v);
    const short2v v = __builtin_elementwise_max(__builtin_bit_cast(short2v, b), (short2v){0, 0});
    o[w] = __builtin_bit_cast(uint32_t, v);
  }
  return __builtin_bit_cast(bf16x8, o);
}

// registers 8s..8s+7 -> bf16, zeroed where the activation h is 0 (ReLU'(h) = 0),
// whole dwords at a time (each half masked by a 32-bit test of h's half)
__device__ __forceinline__ bf16x8 mask_pack(const f32x16& a, int s, const bf16x8& h) {
  const u32x4_ hv = __builtin_bit_cast(u32x4_, h);
  u32x4_ o;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    const bf16x2v b = __builtin_convertvector((f32x2){a[8 * s + 2 * w], a[8 * s + 2 * w + 1]}, bf16x2v);
    const uint32_t m = ((hv[w] & 0xFFFFu) != 0u ? 0x0000FFFFu : 0u) | ((hv[w] >> 16) != 0u ? 0xFFFF0000u : 0u);
    o[w] = __builtin_bit_cast(uint32_t, b) & m;
  }
  return __builtin_bit_cast(bf16x8, o);
}

// fragment f (64 lanes x 16 B) of a fragment array through a buffer resource:
// the lane offset is one VGPR and the fragment offset an SGPR, so no 64-bit
// address per fragment is kept live across the tile loop
__device__ __forceinline__ bf16x8 frag(__amdgpu_buffer_rsrc_t r, int lane16, int f) {
  return __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(r, lane16, f * (WAVE * 16), 0));
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t frag_rsrc(const mlp_bf16x8* p, int nfrag) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, 0, nfrag * WAVE * 16, 0x00020000);
}

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


// Row-blocked work arrays: element (unit u, row m) of a U-unit array sits at
// ((m / 16) * U + u) * 16 + m % 16, so the 16 rows of a block are contiguous
// per unit and a wgrad operand fragment (32 units x 16 rows) is one 1 KB run.
__device__ __forceinline__ int64_t rb_off(int64_t m, int U, int u) { return ((m >> 4) * U + u) * 16 + (m & 15); }

// One 16-unit fragment of this wave's 32-row tile into a row-blocked array.
// Lane (row r, half h) holds units o(j, h), j = 0..7, of row r, as two runs of
// four (o(0..3, h), o(4..7, h)): two 8-byte LDS writes into the wave's
// [row][unit] image (rows TR_ROW elements apart: 40 B, so the writes of lanes
// 0-15 hit distinct banks). ds_read_b64_tr_b16 reads it back transposed: lane
// (group g, i) gets unit i of rows 8g..8g+3 and, with a second read, 8g+4..8g+7
// (16 B: 8 consecutive rows of one unit), and each store instruction writes
// two 512-byte runs (units u0..u0+15 of rows 0-15 and of rows 16-31). The read
// crosses lanes, so every lane takes part (EXEC all ones); only units < U are
// stored.
constexpr int TR_ROW = 20;
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2_ __attribute__((ext_vector_type(2)));
template <int NF, class O>
__device__ __forceinline__ void store_rows(uint16_t* __restrict__ arr, int U, int u0, int64_t tile, const bf16x8* v,
                                           uint16_t* s_tr, int lane, O o) {
  // NF consecutive 16-unit fragments (units u0 + 16 f ...) share one pass: all
  // writes, one wave barrier, all transposed reads, all stores
  const int r = lane & 31, h = lane >> 5;
#pragma unroll
  for (int f = 0; f < NF; ++f) {
    const u32x4_ d = __builtin_bit_cast(u32x4_, v[f]);
    uint16_t* img = s_tr + f * 32 * TR_ROW;
    *reinterpret_cast<u32x2_*>(img + r * TR_ROW + o(0, h)) = u32x2_{d[0], d[1]};
    *reinterpret_cast<u32x2_*>(img + r * TR_ROW + o(4, h)) = u32x2_{d[2], d[3]};
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
  const int g = lane >> 4, i = lane & 15, q = i >> 2, pp = i & 3;
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  u32x4_ w[NF];
#pragma unroll
  for (int f = 0; f < NF; ++f) {
    const uint16_t* a0 = s_tr + f * 32 * TR_ROW + (8 * g + q) * TR_ROW + 4 * pp;
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(uintptr_t)(uint32_t)(uintptr_t)a0);
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(uintptr_t)(uint32_t)(uintptr_t)(a0 + 4 * TR_ROW));
    const u32x2_ wl = __builtin_bit_cast(u32x2_, lo), wh = __builtin_bit_cast(u32x2_, hi);
    w[f] = u32x4_{wl[0], wl[1], wh[0], wh[1]};
  }
#pragma unroll
  for (int f = 0; f < NF; ++f)
    if (u0 + 16 * f + i < U) *reinterpret_cast<u32x4_*>(arr + rb_off(tile * 32 + 8 * g, U, u0 + 16 * f + i)) = w[f];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
}
// hidden-unit fragment q (the accumulator row order, kin) / input fragment s
// (units 16 s + 8 h + j) / action fragment (h = 0: actions 0..7)
__device__ __forceinline__ int o_kin(int j, int h) { return 8 * (j >> 2) + 4 * h + (j & 3); }
__device__ __forceinline__ int o_lin(int j, int h) { return 8 * h + j; }

__device__ __forceinline__ void philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1,
                                       uint32_t out[4]) {
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

}  // namespace

// ---------------------------------------------------------------------------
// Stochastic policy step (SEMANTICS 5): p = softmax(y) in binary32 (max
// subtracted, expf); u = Philox(seed; global id, step) as a 24-bit uniform in
// [0, 1); the action is the first a with u * sum(p) < p_0 + ... + p_a (the
// last one if rounding leaves none). Action a maps to the HPA target
// 40 + 10 (a & 3) % and the carbon weight (a >> 2) $/kgCO2.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) policy_sample_kernel(PgSampleParams q) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= q.n) return;
  const float* y = q.y + i * MLP_OUT;
  float p[MLP_OUT];
  float mx = y[0];
#pragma unroll
  for (int a = 1; a < MLP_OUT; ++a) mx = fmaxf(mx, y[a]);
  float sum = 0.f;
#pragma unroll
  for (int a = 0; a < MLP_OUT; ++a) {
    p[a] = expf(y[a] - mx);
    sum += p[a];
  }
  const int64_t g = q.first_id + i;
  const uint64_t seed = *q.seed;
  uint32_t u4[4];
  philox((uint32_t)g, (uint32_t)(g >> 32), (uint32_t)q.t, 0x5A3B1E7u, (uint32_t)seed, (uint32_t)(seed >> 32), u4);
  const float u = (float)(u4[0] >> 8) * (1.0f / 16777216.0f) * sum;
  int act = MLP_OUT - 1;  // the last action when rounding leaves u above every partial sum
  float acc = 0.f;
  bool found = false;
#pragma unroll
  for (int a = 0; a < MLP_OUT; ++a) {
    acc += p[a];
    if (!found && u < acc) { act = a; found = true; }
  }
  q.act[i] = (uint8_t)act;
  q.target[i] = (int16_t)(40 + 10 * (act & 3));
  q.cw[i] = (double)(act >> 2);
  if (q.rec_target) {
    q.rec_target[i] = q.target[i];
    q.rec_cw[i] = q.cw[i];
  }
}

// ---------------------------------------------------------------------------
// Forward recompute + backward of one 32-row tile per wave (persistent grid).
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256, 1) pg_rows_kernel(PgRowsParams p) {
  constexpr int KS1 = MLP_IN / 16, KS2 = MLP_HID / 16, NB = MLP_HID / 32;
  __shared__ __attribute__((aligned(16))) float s_b[2 * MLP_HID + 32];
  __shared__ bf16x8 s_w2[NB * KS2 * WAVE];  // forward W2 fragments, 128 KiB
  __shared__ __attribute__((aligned(16))) uint16_t s_trans[4][4 * 32 * TR_ROW];  // per wave: up to 4 fragments' [row][unit]
  const int tid = threadIdx.x, lane = tid & (WAVE - 1), wave = tid / WAVE;
  uint16_t* const s_tr = s_trans[wave];
  const int r = lane & 31, h = lane >> 5;
  for (int x = tid; x < NB * KS2 * WAVE; x += blockDim.x) s_w2[x] = p.w2f[x];
  for (int x = tid; x < 2 * MLP_HID + 32; x += blockDim.x) s_b[x] = p.bias[x];
  __syncthreads();
  const __amdgpu_buffer_rsrc_t r1 = frag_rsrc(p.w1f, NB * KS1), r3 = frag_rsrc(p.w3f, KS2);
  const __amdgpu_buffer_rsrc_t r2b = frag_rsrc(p.w2b, NB * KS2), r3b = frag_rsrc(p.w3b, NB);
  const int l16 = lane * 16;
  const int64_t ntiles = p.Mpad / 32;
  const int64_t nw = (int64_t)gridDim.x * (blockDim.x / WAVE);
  for (int64_t tl = (int64_t)blockIdx.x * (blockDim.x / WAVE) + wave; tl < ntiles; tl += nw) {
    const int64_t m = tl * 32 + r;  // this lane's row (state)
    const bool ok = m < p.M;
    // Stores trail by one block: a phase's weight fragments for block n are
    // loaded BEFORE the stores of block n - 1, so waiting for them does not
    // wait for those stores (vector-memory operations retire in issue order).
    // ---- X^T fragments (B operand of layer 1), stored for dW1; row factors ----
    bf16x8 xf[KS1];
    {
      const bf16x8* src = reinterpret_cast<const bf16x8*>(p.x + (ok ? m : 0) * MLP_IN + 8 * h);
#pragma unroll
      for (int s = 0; s < KS1; ++s) {
        const bf16x8 v = src[2 * s];
        xf[s] = ok ? v : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
      }
    }
    const float cf = ok ? p.coef[(p.row0 + m) % p.n_scen] : 0.f;
    const int act = ok ? (int)p.act[m] : -1;
    // ---- layer 1: H1^T = relu(bf16(W1^T X^T + b1)) ----
    bf16x8 h1[KS2];
#pragma unroll
    for (int n = 0; n < NB; ++n) {
      bf16x8 wv[KS1];
#pragma unroll
      for (int s = 0; s < KS1; ++s) wv[s] = frag(r1, l16, n * KS1 + s);
      __builtin_amdgcn_sched_barrier(0);
      if (n == 0) {
        store_rows<KS1>(p.xT, MLP_IN, 0, tl, xf, s_tr, lane, o_lin);
      } else {
        store_rows<2>(p.h1T, MLP_HID, 32 * (n - 1), tl, h1 + 2 * n - 2, s_tr, lane, o_kin);
      }
      __builtin_amdgcn_sched_barrier(0);
      f32x16 c = bias_tile(s_b + 32 * n, h);
#pragma unroll
      for (int s = 0; s < KS1; ++s) c = mfma(wv[s], xf[s], c);
      h1[2 * n] = relu_pack(c, 0);
      h1[2 * n + 1] = relu_pack(c, 1);
      __builtin_amdgcn_sched_barrier(0);
    }
    // ---- layer 2: H2^T = relu(bf16(W2^T H1^T + b2)); layer 3: Y^T = W3^T H2^T + b3 ----
    bf16x8 h2[KS2];
    f32x16 yv = bias_tile(s_b + 2 * MLP_HID, h);
#pragma unroll
    for (int n = 0; n < NB; ++n) {
      const bf16x8 w30 = frag(r3, l16, 2 * n), w31 = frag(r3, l16, 2 * n + 1);
      __builtin_amdgcn_sched_barrier(0);
      const bf16x8* prev = n == 0 ? h1 + 2 * (NB - 1) : h2 + 2 * (n - 1);
      uint16_t* parr = n == 0 ? p.h1T : p.h2T;
      const int pu = 32 * (n == 0 ? NB - 1 : n - 1);
      store_rows<2>(parr, MLP_HID, pu, tl, prev, s_tr, lane, o_kin);
      __builtin_amdgcn_sched_barrier(0);
      f32x16 c = bias_tile(s_b + MLP_HID + 32 * n, h);
#pragma unroll
      for (int kk = 0; kk < KS2; ++kk) c = mfma(s_w2[(n * KS2 + kk) * WAVE + lane], h1[kk], c);
      h2[2 * n] = relu_pack(c, 0);
      h2[2 * n + 1] = relu_pack(c, 1);
      yv = mfma(w30, h2[2 * n], yv);
      yv = mfma(w31, h2[2 * n + 1], yv);
      __builtin_amdgcn_sched_barrier(0);
    }
    // ---- g_y = c (e_a - softmax(y)): logits 4h..4h+3 of row m in registers 0..3 ----
    float mx = fmaxf(fmaxf(yv[0], yv[1]), fmaxf(yv[2], yv[3]));
    mx = fmaxf(mx, __shfl_xor(mx, 32));
    float e[4], se = 0.f;
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      e[a] = expf(yv[a] - mx);
      se += e[a];
    }
    se += __shfl_xor(se, 32);
    float gy[4];
#pragma unroll
    for (int a = 0; a < 4; ++a) gy[a] = cf * ((4 * h + a == act ? 1.f : 0.f) - e[a] / se);
    // B operand of dH2^T = W3 g_y^T (k = action, padded to 16): half 0 holds
    // actions 0..7 of its row, half 1 zeros
    float g8[8];
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      const float o = __shfl_xor(gy[a], 32);
      g8[a] = h == 0 ? gy[a] : 0.f;
      g8[4 + a] = h == 0 ? o : 0.f;
    }
    u32x4_ gw;
#pragma unroll
    for (int w = 0; w < 4; ++w)
      gw[w] = __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){g8[2 * w], g8[2 * w + 1]}, bf16x2v));
    const bf16x8 gyf = __builtin_bit_cast(bf16x8, gw);
    __builtin_amdgcn_sched_barrier(0);
    // ---- dH2^T = (W3 g_y^T) masked by H2 > 0 ----
    bf16x8 dh2[KS2];
#pragma unroll
    for (int n = 0; n < NB; ++n) {
      const bf16x8 wb = frag(r3b, l16, n);
      __builtin_amdgcn_sched_barrier(0);
      if (n == 0) {
        store_rows<2>(p.h2T, MLP_HID, 32 * (NB - 1), tl, h2 + 2 * NB - 2, s_tr, lane, o_kin);
        store_rows<1>(p.gyT, MLP_OUT, 0, tl, &gyf, s_tr, lane, o_lin);  // half 1 holds zeros (units 8..15, not stored)
      } else {
        store_rows<2>(p.dh2T, MLP_HID, 32 * (n - 1), tl, dh2 + 2 * n - 2, s_tr, lane, o_kin);
      }
      __builtin_amdgcn_sched_barrier(0);
      const f32x16 c = mfma(wb, gyf, zero16());
      dh2[2 * n] = mask_pack(c, 0, h2[2 * n]);
      dh2[2 * n + 1] = mask_pack(c, 1, h2[2 * n + 1]);
      __builtin_amdgcn_sched_barrier(0);
    }
    // ---- dH1^T = (W2 dH2^T) masked by H1 > 0, one 32-row block at a time ----
    bf16x8 dd[2] = {dh2[2 * NB - 2], dh2[2 * NB - 1]};  // the block stored next
#pragma unroll
    for (int n = 0; n < NB; ++n) {
      bf16x8 wv[KS2];
#pragma unroll
      for (int kk = 0; kk < KS2; ++kk) wv[kk] = frag(r2b, l16, n * KS2 + kk);
      __builtin_amdgcn_sched_barrier(0);
      uint16_t* parr = n == 0 ? p.dh2T : p.dh1T;
      const int pu = 32 * (n == 0 ? NB - 1 : n - 1);
      store_rows<2>(parr, MLP_HID, pu, tl, dd, s_tr, lane, o_kin);
      __builtin_amdgcn_sched_barrier(0);
      f32x16 c = zero16();
#pragma unroll
      for (int kk = 0; kk < KS2; ++kk) c = mfma(wv[kk], dh2[kk], c);
      dd[0] = mask_pack(c, 0, h1[2 * n]);
      dd[1] = mask_pack(c, 1, h1[2 * n + 1]);
      __builtin_amdgcn_sched_barrier(0);
    }
    store_rows<2>(p.dh1T, MLP_HID, 32 * (NB - 1), tl, dd, s_tr, lane, o_kin);
  }
}

// ---------------------------------------------------------------------------
// C[a][b] = sum_m A[a][m] B[b][m] (A: KA units, B: KB units, row-blocked bf16
// arrays; units past KA / KB read as zero) and, with q.bpart, the bias
// gradient sum_m B[b][m] as one more MFMA per column tile against a constant
// A fragment (row 0 all ones), so the bias never re-reads B. One 8-wave
// workgroup per CU (q.splits of them; two waves per SIMD) owns a contiguous
// chunk of rows and the WHOLE output: the (KA/32) x (KB/32) tiles are split
// into eight wave blocks of RPW x CPW tiles whose fp32 accumulators stay in
// registers over the chunk, 16 rows per MFMA k-step. An operand fragment is
// one 1 KB run (lane (r, h): unit r of the slab, rows 8h..8h+7 of the block);
// the waves' shared fragments come from L1 / L2. Wave (row group g, column
// group) owns the bias of its column tile g (every column tile once: the
// instantiations have at least CPW row groups). The next k-step's fragments
// are in flight during this one's MFMAs. Each split's partials land in its
// block of the packed gradient layout; pg_reduce_kernel sums the blocks in
// split order (deterministic), all three GEMMs in one launch.
// ---------------------------------------------------------------------------
constexpr int WG_WAVES = 8;
template <int B, int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < N) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, N>(f);
  }
}
template <int RPW, int CPW, int PD = 2>
__global__ void __launch_bounds__(64 * WG_WAVES, 1) pg_wgrad_kernel(WgradParams q) {
  static_assert(RPW * CPW <= 8, "accumulators");
  // w wave-uniform in an SGPR (the loads' resources and offsets derive from it)
  const int lane = threadIdx.x & (WAVE - 1), w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / WAVE));
  const int r = lane & 31, h = lane >> 5;
  const int nrt = (q.KA + 31) / 32, nct = (q.KB + 31) / 32;
  const int wc = nct / CPW, wr = nrt / RPW;  // wave blocks per column / row of the tile grid
  if (w >= wr * wc) return;                 // wave-uniform; no barrier below
  const int g = w / wc, rt0 = g * RPW, ct0 = (w % wc) * CPW;
  const int64_t chunk = (q.Mpad / 16 + q.splits - 1) / q.splits * 16;
  // (a split past the last row still writes its zero partials)
  const int64_t m0 = min((int64_t)blockIdx.x * chunk, q.Mpad), m1 = min(m0 + chunk, q.Mpad);
  const int jb = q.bpart && g < CPW ? g : -1;  // the bias tile: column tile ct0 + jb
  const bf16x8 z = {0, 0, 0, 0, 0, 0, 0, 0};
  const short one = 0x3F80;  // bf16 1.0
  const bf16x8 ones = r == 0 ? bf16x8{one, one, one, one, one, one, one, one} : z;
  // one buffer resource per operand over this chunk's row blocks (base and
  // size through readfirstlane: a resource word the compiler left in a VGPR
  // would turn every load into a waterfall loop); a lane whose unit is past
  // KA / KB reads out of range (zero)
  auto chunk_rsrc = [&](const uint16_t* base, int U) {
    const uint64_t a = (uint64_t)(base + (m0 >> 4) * U * 16);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)a);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32));
    const int bytes = __builtin_amdgcn_readfirstlane((int)(((m1 - m0) >> 4) * U * 32));
    return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0, bytes, 0x00020000);
  };
  const __amdgpu_buffer_rsrc_t rsa = chunk_rsrc(q.A, q.KA), rsb = chunk_rsrc(q.B, q.KB);
  int oa[RPW], ob[CPW];
#pragma unroll
  for (int i = 0; i < RPW; ++i) {
    const int u = (rt0 + i) * 32 + r;
    oa[i] = u < q.KA ? u * 32 + 16 * h : 0x40000000;
  }
#pragma unroll
  for (int j = 0; j < CPW; ++j) {
    const int u = (ct0 + j) * 32 + r;
    ob[j] = u < q.KB ? u * 32 + 16 * h : 0x40000000;
  }
  const int sa = q.KA * 32, sb = q.KB * 32;  // bytes per row block
  f32x16 c[RPW][CPW], cb = zero16();
#pragma unroll
  for (int i = 0; i < RPW; ++i)
#pragma unroll
    for (int j = 0; j < CPW; ++j) c[i][j] = zero16();
  bf16x8 xa[PD][RPW], xb[PD][CPW];  // PD k-steps of fragments: this one's and PD - 1 in flight
  auto load = [&](int blk, auto S) {  // row block blk of the chunk into buffer S
#pragma unroll
    for (int i = 0; i < RPW; ++i)
      xa[S][i] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rsa, oa[i], blk * sa, 0));
#pragma unroll
    for (int j = 0; j < CPW; ++j)
      xb[S][j] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rsb, ob[j], blk * sb, 0));
  };
  const int nblk = (int)((m1 - m0) >> 4);
  static_for<0, PD>([&](auto S) {
    if (nblk > decltype(S)::value) load(decltype(S)::value, S);
  });
  // this k-step's fragments in buffer S, the next PD - 1 in flight in the
  // others; buffer S is refilled (PD k-steps ahead) once its MFMAs have read
  // it. PD k-steps per trip keep the buffer index a compile-time constant (a
  // runtime-indexed register array would live in scratch memory)
  auto kstep = [&](int blk, auto S) {
#pragma unroll
    for (int j = 0; j < CPW; ++j) {
#pragma unroll
      for (int i = 0; i < RPW; ++i) c[i][j] = mfma(xa[S][i], xb[S][j], c[i][j]);
      if (j == jb) cb = mfma(ones, xb[S][j], cb);  // wave-uniform branch
    }
    __builtin_amdgcn_sched_barrier(0);
    if (blk + PD < nblk) load(blk + PD, S);
  };
  for (int blk = 0; blk < nblk; blk += PD) {
    static_for<0, PD>([&](auto S) {
      if (blk + decltype(S)::value < nblk) kstep(blk + decltype(S)::value, S);
    });
  }
  // accumulator register k: row a0 + (k&3) + 8(k>>2) + 4h, column b0 + r
  float* out = q.part + (int64_t)blockIdx.x * q.pstride;
#pragma unroll
  for (int i = 0; i < RPW; ++i)
#pragma unroll
    for (int j = 0; j < CPW; ++j)
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int a = (rt0 + i) * 32 + (k & 3) + 8 * (k >> 2) + 4 * h, b = (ct0 + j) * 32 + r;
        if (a < q.KA && b < q.KB) out[(int64_t)a * q.KB + b] = c[i][j][k];
      }
  if (jb >= 0 && h == 0) {  // row 0 of the bias tile: register 0 of the lower half
    const int b = (ct0 + jb) * 32 + r;
    if (b < q.KB) q.bpart[(int64_t)blockIdx.x * q.pstride + b] = cb[0];
  }
}

// The same GEMM with the operand fragments staged once per workgroup: every
// k-step's nrt + nct distinct fragments (<= 16 KB) are loaded by the 8 waves
// together (wave w loads fragments w and w + 8) into registers PG_PF k-steps
// ahead, written to an LDS double buffer one k-step ahead, and each wave reads
// its RPW + CPW fragments from LDS: global / L1 traffic is the unique 16 KB per
// k-step instead of the waves' 48 KB (dW2), one barrier per k-step.
#ifndef PG_PF
#define PG_PF 8  // (A/B at 250k x 60: 2 / 4 / 8 k-steps 23.23 / 22.97 / 22.40 ms per gradient, unstaged 23.39)
#endif
// f(integral_constant<E>) for E = B .. N - 1 (compile-time register indices)
template <int RPW, int CPW>
__global__ void __launch_bounds__(64 * WG_WAVES, 1) pg_wgrad_lds_kernel(WgradParams q) {
  static_assert(RPW * CPW <= 8, "accumulators");
  constexpr int PF = PG_PF;  // k-steps in flight in registers (power of two)
  static_assert(PF >= 2 && (PF & (PF - 1)) == 0, "PG_PF");
  __shared__ bf16x8 sf[2][16][WAVE];  // [buffer][fragment][lane]: 32 KB
  const int lane = threadIdx.x & (WAVE - 1), w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / WAVE));
  const int r = lane & 31, h = lane >> 5;
  const int nrt = (q.KA + 31) / 32, nct = (q.KB + 31) / 32, nf = nrt + nct;  // <= 16 (launch_pg_wgrad)
  const int wc = nct / CPW, wr = nrt / RPW;
  const bool comp = w < wr * wc;  // this wave accumulates (all 8 load)
  const int g = comp ? w / wc : 0, rt0 = g * RPW, ct0 = comp ? (w % wc) * CPW : 0;
  const int64_t chunk = (q.Mpad / 16 + q.splits - 1) / q.splits * 16;
  const int64_t m0 = min((int64_t)blockIdx.x * chunk, q.Mpad), m1 = min(m0 + chunk, q.Mpad);
  const int jb = comp && q.bpart && g < CPW ? g : -1;
  const bf16x8 z = {0, 0, 0, 0, 0, 0, 0, 0};
  const short one = 0x3F80;
  const bf16x8 ones = r == 0 ? bf16x8{one, one, one, one, one, one, one, one} : z;
  auto chunk_rsrc = [&](const uint16_t* base, int U) {
    const uint64_t a = (uint64_t)(base + (m0 >> 4) * U * 16);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)a);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32));
    const int bytes = __builtin_amdgcn_readfirstlane((int)(((m1 - m0) >> 4) * U * 32));
    return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0, bytes, 0x00020000);
  };
  const __amdgpu_buffer_rsrc_t rsa = chunk_rsrc(q.A, q.KA), rsb = chunk_rsrc(q.B, q.KB);
  // the two fragments this wave loads (f = w, w + 8; none past nf): operand,
  // lane offset (a unit past KA / KB reads out of range: zero) and row-block stride
  int lf[2];
  bool la[2], lv[2];
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    const int f = w + 8 * e;
    lv[e] = f < nf;
    la[e] = f < nrt;
    const int u = (la[e] ? f : f - nrt) * 32 + r;
    lf[e] = (u < (la[e] ? q.KA : q.KB)) ? u * 32 + 16 * h : 0x40000000;
  }
  const int sa = q.KA * 32, sb = q.KB * 32;
  const int nblk = (int)((m1 - m0) >> 4);
  bf16x8 G[PF][2];
  auto gload = [&](int blk, auto E) {
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      G[E][e] = z;
      if (lv[e] && blk < nblk)  // wave-uniform
        G[E][e] = __builtin_bit_cast(bf16x8, la[e] ? __builtin_amdgcn_raw_buffer_load_b128(rsa, lf[e], blk * sa, 0)
                                                    : __builtin_amdgcn_raw_buffer_load_b128(rsb, lf[e], blk * sb, 0));
    }
  };
  auto lwrite = [&](int buf, auto E) {
#pragma unroll
    for (int e = 0; e < 2; ++e)
      if (lv[e]) sf[buf][w + 8 * e][lane] = G[E][e];
  };
  f32x16 c[RPW][CPW], cb = zero16();
#pragma unroll
  for (int i = 0; i < RPW; ++i)
#pragma unroll
    for (int j = 0; j < CPW; ++j) c[i][j] = zero16();
  // prologue: k-steps 0 .. PF - 1 in flight, k-step 0 in LDS buffer 0
  static_for<0, PF>([&](auto E) { gload(decltype(E)::value, E); });
  lwrite(0, std::integral_constant<int, 0>{});
  __syncthreads();
  // k-step blk: its fragments in LDS buffer blk & 1, k-steps blk + 1 .. blk + PF - 1
  // in registers (G[(blk + k) % PF]); k-step blk + 1 goes to the other buffer (its
  // readers of k-step blk - 1 passed the last barrier), G[blk % PF] is refilled
  // with k-step blk + PF. PF trips per loop keep every G index a constant.
  auto kstep = [&](int blk, auto E) {
    constexpr int e0 = decltype(E)::value, e1 = (e0 + 1) % PF;
    const int bufc = blk & 1;
    if (blk + 1 < nblk) lwrite(bufc ^ 1, std::integral_constant<int, e1>{});
    gload(blk + PF, E);
    if (comp) {  // wave-uniform
      bf16x8 xa[RPW], xb[CPW];
#pragma unroll
      for (int i = 0; i < RPW; ++i) xa[i] = sf[bufc][rt0 + i][lane];
#pragma unroll
      for (int j = 0; j < CPW; ++j) xb[j] = sf[bufc][nrt + ct0 + j][lane];
#pragma unroll
      for (int j = 0; j < CPW; ++j) {
#pragma unroll
        for (int i = 0; i < RPW; ++i) c[i][j] = mfma(xa[i], xb[j], c[i][j]);
        if (j == jb) cb = mfma(ones, xb[j], cb);
      }
    }
    __syncthreads();
  };
  for (int blk = 0; blk < nblk; blk += PF) {
    static_for<0, PF>([&](auto E) {
      if (blk + decltype(E)::value < nblk) kstep(blk + decltype(E)::value, E);
    });
  }
  if (!comp) return;
  float* out = q.part + (int64_t)blockIdx.x * q.pstride;
#pragma unroll
  for (int i = 0; i < RPW; ++i)
#pragma unroll
    for (int j = 0; j < CPW; ++j)
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int a = (rt0 + i) * 32 + (k & 3) + 8 * (k >> 2) + 4 * h, b = (ct0 + j) * 32 + r;
        if (a < q.KA && b < q.KB) out[(int64_t)a * q.KB + b] = c[i][j][k];
      }
  if (jb >= 0 && h == 0) {
    const int b = (ct0 + jb) * 32 + r;
    if (b < q.KB) q.bpart[(int64_t)blockIdx.x * q.pstride + b] = cb[0];
  }
}

// out = sum of the splits' partials in split order (acc: added to out, the
// running sum over row chunks in chunk order)
__global__ void __launch_bounds__(256) pg_reduce_kernel(const float* __restrict__ part, float* __restrict__ out,
                                                        int64_t n, int splits, int acc) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  // split order as one chain of additions; the loads of 16 splits issue
  // together ahead of their adds (one dependent load per add measured 103 us
  // per launch for 256 x 86k floats)
  float s = 0.f;
  int k = 0;
  for (; k + 16 <= splits; k += 16) {
    float v[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = part[(int64_t)(k + j) * n + i];
#pragma unroll
    for (int j = 0; j < 16; ++j) s += v[j];
  }
  for (; k < splits; ++k) s += part[(int64_t)k * n + i];
  out[i] = acc ? out[i] + s : s;
}

__global__ void __launch_bounds__(256) pg_fill_kernel(uint16_t* __restrict__ x, int64_t n, int64_t valid, uint16_t v) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) x[i] = i < valid ? v : (uint16_t)0;
}

hipError_t launch_policy_sample(const PgSampleParams& q, hipStream_t s) {
  hipLaunchKernelGGL(policy_sample_kernel, dim3((unsigned)((q.n + 255) / 256)), dim3(256), 0, s, q);
  return hipGetLastError();
}

hipError_t launch_pg_rows(const PgRowsParams& p, int cus, hipStream_t s) {
  hipLaunchKernelGGL(pg_rows_kernel, dim3((unsigned)cus), dim3(256), 0, s, p);
  return hipGetLastError();
}

hipError_t launch_pg_wgrad(const WgradParams& q, hipStream_t s) {
  // eight wave blocks over the output tiles
  const int nrt = (q.KA + 31) / 32, nct = (q.KB + 31) / 32;
  const dim3 grid((unsigned)q.splits), block(64 * WG_WAVES);
// k-steps of operand fragments per wave in flight + 1 (variant builds),
// measured per launch at 250k x 60 (two launches per gradient): dW3 (one row
// and one column tile per wave) PD 2 / 4 / 8: 0.742 / 0.653 / 0.668 ms; dW1
// (two row tiles per wave) PD 2 / 3 / 4: 0.899 / 0.936 / 1.007 ms
#ifndef PG_PD1  // dW1
#define PG_PD1 2
#endif
#ifndef PG_PD3  // dW3
#define PG_PD3 4
#endif
#ifndef PG_WGRAD_LDS  // A/B of the operand staging (variant builds)
#define PG_WGRAD_LDS 1
#endif
  // dW2 (16 distinct fragments per k-step, each wave reading 6: 48 KB through
  // L1 per k-step unstaged) stages them in LDS: 4.8 -> 2.5 ms per gradient at
  // 250k x 60; dW1 / dW3 (10 / 9 distinct, 3 / 2 per wave) measured 1.9 / 1.3 ms
  // unstaged against 1.9 / 1.6 ms staged (profiles/round6/config5_grad_kernel_stats*.csv)
  if (PG_WGRAD_LDS && nrt == 8 && nct == 8) {
    hipLaunchKernelGGL((pg_wgrad_lds_kernel<2, 4>), grid, block, 0, s, q);  // dW2 (+ db2)
    return hipGetLastError();
  }
  if (nrt == 8 && nct == 8) hipLaunchKernelGGL((pg_wgrad_kernel<2, 4>), grid, block, 0, s, q);       // dW2 (+ db2)
  else if (nrt == 2 && nct == 8) hipLaunchKernelGGL((pg_wgrad_kernel<2, 1, PG_PD1>), grid, block, 0, s, q);  // dW1 (+ db1)
  else if (nrt == 8 && nct == 1) hipLaunchKernelGGL((pg_wgrad_kernel<1, 1, PG_PD3>), grid, block, 0, s, q);  // dW3 (+ db3)
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t launch_pg_reduce(const float* part, float* out, int64_t n, int splits, int acc, hipStream_t s) {
  hipLaunchKernelGGL(pg_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, part, out, n, splits, acc);
  return hipGetLastError();
}

hipError_t launch_pg_fill(uint16_t* x, int64_t n, int64_t valid, uint16_t v, hipStream_t s) {
  hipLaunchKernelGGL(pg_fill_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, x, n, valid, v);
  return hipGetLastError();
}

}  // namespace ccka
