// d1_common.h — device helpers shared by the single-deployment engines:
// rollout_d1.hip (one wave per scenario batch, event steps per wave) and
// rollout_pool.hip (event steps pooled per workgroup). Internal linkage: each
// translation unit gets its own copy.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ccka.h"
#include "kparams.h"

namespace ccka {
namespace {

constexpr int WAVE = 64;

__device__ __forceinline__ int capbit1(int c) { return c == 0 ? CCKA_CAP_SPOT : CCKA_CAP_OD; }

// Opaque copy of a kernel argument: the value then lives in a register for the
// whole loop (spilled to a VGPR lane if need be) instead of being re-read from
// the kernarg segment with an s_load + lgkmcnt wait at each use.
template <class V>
__device__ __forceinline__ V opq(V v) {
  asm volatile("" : "+s"(v));
  return v;
}
// global-memory pointer made opaque the same way, keeping its address space
// (a generic pointer would turn every access into a flat_* instruction)
#define GLOBAL_AS __attribute__((address_space(1)))
template <class V>
__device__ __forceinline__ GLOBAL_AS V* opq_ptr(V* v) {
  uint64_t x = (uint64_t)v;
  asm volatile("" : "+s"(x));
  return (GLOBAL_AS V*)x;
}

// down-window entries of a window (entry k is (k + 1) steps old): bit k set
// while (k + 1) * 60 < window_s
__device__ __forceinline__ int wmask(int window_s) {
  int m = 0;
#pragma unroll
  for (int k = 0; k < CCKA_HIST; ++k) m |= ((k + 1) * CCKA_STEP_SECONDS < window_s) ? (1 << k) : 0;
  return m;
}

// packed int16 history rings: entry k (k steps old, 0 = this step) sits in
// half k&1 of word k>>1
template <int W = 4>
__device__ __forceinline__ void ring_push(uint32_t* r, int v) {
#pragma unroll
  for (int w = W - 1; w > 0; --w) r[w] = __builtin_amdgcn_alignbit(r[w], r[w - 1], 16);
  r[0] = (r[0] << 16) | ((uint32_t)v & 0xFFFFu);
}
// four equal records at once (one step of 15 s decisions): a two-word shift
template <int W>
__device__ __forceinline__ void ring_push4(uint32_t* r, int v) {
#pragma unroll
  for (int w = W - 1; w > 1; --w) r[w] = r[w - 2];
  r[1] = r[0] = ((uint32_t)v & 0xFFFFu) * 0x10001u;
}

typedef short short2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ short2v as_s2(uint32_t x) { return __builtin_bit_cast(short2v, x); }
// (m & a) | (~m & b): v_bfi_b32
__device__ __forceinline__ uint32_t bfi(uint32_t m, uint32_t a, uint32_t b) { return (m & a) | (~m & b); }

// floor(a / b) for 0 <= a < 2^31, 1 <= b < 2^30, given rb = 1/(float)b
// (v_rcp_f32), without a branch: the f32 estimate is within one of the
// quotient while the quotient is below 2^20, and one remainder test corrects
// it. `bad` is set when those preconditions fail (the caller then recomputes
// exactly); lanes whose inputs are meaningless get a meaningless quotient and
// no fault.
__device__ __forceinline__ int fdiv_nb(int a, int b, float rb, bool& bad) {
  int q = (int)((float)a * rb);
  const int r = (int)((uint32_t)a - (uint32_t)q * (uint32_t)b);
  q += (r >= b ? 1 : 0) - (r < 0 ? 1 : 0);
  bad = bad || (uint32_t)q >= (1u << 20) || (uint32_t)b >= (1u << 30);
  return q;
}

// trajectory record through a buffer resource: the hardware drops a store
// whose offset lies past num_records, so an out-of-range offset masks a lane's
// store without an exec-mask branch, and num_records = 0 turns every store
// off when no trajectory is kept
constexpr int D1_NOSTORE = 0x7FFFFFF0;
__device__ __forceinline__ void d1_store_rec(__amdgpu_buffer_rsrc_t r, int voff, const int4& v) {
  typedef int i32x4 __attribute__((ext_vector_type(4)));
  const i32x4 x = {v.x, v.y, v.z, v.w};
  __builtin_amdgcn_raw_buffer_store_b128(x, r, voff, 0, 0);
}

// Argmin-table reads of the event step through the scalar data cache: a
// vector load would wait for every older vector-memory operation of the wave
// (trajectory stores and sample loads still in flight: they complete in issue
// order), a scalar load only for older scalar ones. The active lanes'
// addresses are taken four at a time (v_readlane), loaded with s_load_dwordx2
// and handed back to their lanes.
#define CONST_AS __attribute__((address_space(4)))
__device__ __forceinline__ int2 d1_tload(const GLOBAL_AS int2* ptr) {
  const uint64_t a = (uint64_t)ptr;
  const int alo = (int)(uint32_t)a, ahi = (int)(uint32_t)(a >> 32);
  const int me = (int)(threadIdx.x & (WAVE - 1));
  uint64_t m = __ballot(1);
  int ox = 0, oy = 0;
  while (m) {
    int l[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      l[k] = m ? __ffsll((long long)m) - 1 : l[0];
      m &= m - 1;  // (0 stays 0)
    }
    uint64_t v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint64_t ak = (uint64_t)(uint32_t)__builtin_amdgcn_readlane(alo, l[k]) |
                          (uint64_t)(uint32_t)__builtin_amdgcn_readlane(ahi, l[k]) << 32;
      v[k] = *(const CONST_AS uint64_t*)ak;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      ox = me == l[k] ? (int)(uint32_t)v[k] : ox;
      oy = me == l[k] ? (int)(uint32_t)(v[k] >> 32) : oy;
    }
  }
  return make_int2(ox, oy);
}

}  // namespace
}  // namespace ccka
