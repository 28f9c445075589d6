// isa_rates.hip — measured issue cost and dependent latency (shader cycles)
// of the VALU instructions the rollout kernels are built from, one wave on
// one SIMD (and two waves sharing a SIMD), on gfx950. Diagnostic tool only.
// Build: hipcc -O3 --offload-arch=gfx950 -o isa_rates isa_rates.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define REP8(x) x x x x x x x x
#define REP64(x) REP8(REP8(x))

// dependent chain: each instruction reads the previous result
#define DEP(NAME, ASM)                                                              \
  __global__ void dep_##NAME(uint64_t* out, uint32_t seed) {                      \
    uint32_t a = seed + threadIdx.x, b = seed * 3u + 1u;                           \
    uint64_t w = (uint64_t)a << 32 | b;                                              \
    (void)w;                                                                          \
    uint64_t t0 = __builtin_amdgcn_s_memtime();                                      \
    for (int it = 0; it < 16; ++it) { REP64(ASM) }                                   \
    uint64_t t1 = __builtin_amdgcn_s_memtime();                                      \
    if (threadIdx.x == 0) out[blockIdx.x * 4 + threadIdx.y] = t1 - t0;              \
    if (a == 0x12345 && b == 7) out[1000] = a + (uint32_t)w;                         \
  }
// 8 independent chains interleaved
#define IND(NAME, ASM8)                                                             \
  __global__ void ind_##NAME(uint64_t* out, uint32_t seed) {                      \
    uint32_t a0 = seed + threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, \
             a6 = a0 + 6, a7 = a0 + 7, b = seed * 3u + 1u;                           \
    uint64_t t0 = __builtin_amdgcn_s_memtime();                                      \
    for (int it = 0; it < 16; ++it) { REP8(ASM8) }                                   \
    uint64_t t1 = __builtin_amdgcn_s_memtime();                                      \
    if (threadIdx.x == 0) out[blockIdx.x * 4 + threadIdx.y] = t1 - t0;              \
    if ((a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7) == 0x12345) out[1000] = b;          \
  }

#define I8(op) op(a0) op(a1) op(a2) op(a3) op(a4) op(a5) op(a6) op(a7)

#define A_ADD asm volatile("v_add_u32 %0, %0, %1" : "+v"(a) : "v"(b));
#define A_MULLO asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a) : "v"(b));
#define A_MULHI asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a) : "v"(b));
#define A_MUL24 asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a) : "v"(b));
#define A_MAD64 asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(w) : "v"(a), "v"(b) : "vcc");
#define A_CVT asm volatile("v_cvt_f32_u32 %0, %0" : "+v"(a));
#define A_RCP asm volatile("v_rcp_f32 %0, %0" : "+v"(a));
#define A_FMUL asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a) : "v"(b));
#define A_DMUL asm volatile("v_mul_f64 %0, %0, %0" : "+v"(w));
#define A_DFMA asm volatile("v_fma_f64 %0, %0, %0, %0" : "+v"(w));
#define A_CND asm volatile("v_cmp_gt_u32 vcc, %0, %1\n v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a) : "v"(b) : "vcc");
#define A_MIN asm volatile("v_min_u32 %0, %0, %1" : "+v"(a) : "v"(b));
#define A_LSHLOR asm volatile("v_lshl_or_b32 %0, %0, 1, %1" : "+v"(a) : "v"(b));
#define A_PKADD asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a) : "v"(b));
#define A_ADD64 asm volatile("v_lshl_add_u64 %0, %0, 0, %0" : "+v"(w));
#define A_BFE asm volatile("v_bfe_u32 %0, %0, 3, 5" : "+v"(a));
#define A_CMPX asm volatile("v_cmp_gt_u32 vcc, %0, %1" :: "v"(a), "v"(b) : "vcc");
#define A_SADD asm volatile("s_add_u32 s40, s40, s41" ::: "s40", "s41", "scc");

DEP(add, A_ADD) DEP(mullo, A_MULLO) DEP(mulhi, A_MULHI) DEP(mul24, A_MUL24) DEP(mad64, A_MAD64)
DEP(cvt, A_CVT) DEP(rcp, A_RCP) DEP(fmul, A_FMUL) DEP(dmul, A_DMUL) DEP(dfma, A_DFMA) DEP(cnd, A_CND)
DEP(min, A_MIN) DEP(lshlor, A_LSHLOR) DEP(pkadd, A_PKADD) DEP(add64, A_ADD64) DEP(bfe, A_BFE)
DEP(cmp, A_CMPX) DEP(sadd, A_SADD)

#define O_ADD(x) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(b));
#define O_MULLO(x) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x) : "v"(b));
#define O_MUL24(x) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(x) : "v"(b));
#define O_CVT(x) asm volatile("v_cvt_f32_u32 %0, %0" : "+v"(x));
#define O_RCP(x) asm volatile("v_rcp_f32 %0, %0" : "+v"(x));
#define O_MIN(x) asm volatile("v_min_u32 %0, %0, %1" : "+v"(x) : "v"(b));
#define O_CND(x) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x) : "v"(b) : "vcc");
IND(add, I8(O_ADD)) IND(mullo, I8(O_MULLO)) IND(mul24, I8(O_MUL24)) IND(cvt, I8(O_CVT))
IND(rcp, I8(O_RCP)) IND(min, I8(O_MIN)) IND(cnd, I8(O_CND))

typedef void (*kfn)(uint64_t*, uint32_t);
static void run(const char* name, kfn f, int ninstr, uint64_t* d) {
  for (int waves = 1; waves <= 8; waves *= 2) {
    // one workgroup of `waves` waves on one CU: 4 SIMDs, so waves 5..8 double up
    hipLaunchKernelGGL(f, dim3(1), dim3(64, waves > 4 ? 4 : waves, waves > 4 ? 2 : 1), 0, 0, d, 1u);
    hipDeviceSynchronize();
    uint64_t h[8];
    hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    hipLaunchKernelGGL(f, dim3(1), dim3(64, waves > 4 ? 4 : waves, waves > 4 ? 2 : 1), 0, 0, d, 1u);
    hipDeviceSynchronize();
    hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    printf("%-10s waves=%d  %.2f cycles/instr\n", name, waves, (double)h[0] / ninstr);
  }
}

int main() {
  uint64_t* d;
  hipMalloc(&d, 8192 * 8);
  hipMemset(d, 0, 8192 * 8);
  const int N = 16 * 64;
  printf("-- dependent chains (latency-bound), 1 wave / 2 waves per SIMD --\n");
#define R(n) run("dep_" #n, dep_##n, N, d);
  R(add) R(mullo) R(mulhi) R(mul24) R(mad64) R(cvt) R(rcp) R(fmul) R(dmul) R(dfma) R(min) R(lshlor) R(pkadd)
  R(add64) R(bfe) R(cmp) R(sadd)
  printf("cnd = cmp + cndmask pair:\n");
  R(cnd)
  printf("-- 8 independent chains (issue-bound) --\n");
#define RI(n) run("ind_" #n, ind_##n, N, d);
  RI(add) RI(mullo) RI(mul24) RI(cvt) RI(rcp) RI(min) RI(cnd)
  return 0;
}
