// rollout.hip — MI355X (gfx950) batched policy-rollout engine.
//
// One lane = one cluster scenario stepped through the whole horizon
// (docs/SEMANTICS.md). Decision semantics restate the upstream controllers the
// reference drives: the peak/off-peak NodePool switch
// (demo_20_offpeak_configure.sh:59-81, demo_21_peak_configure.sh:56-77,
// demo_19_reset_policies.sh:68-75), the burst Deployments
// (demo_30_burst_configure.sh:57-141) and PDB (demo_10_setup_configure.sh:47-56),
// HPA (k8s 1.34, .env:4), KEDA (.env:10-12), Karpenter 1.8.1 (05_karpenter.sh:20).
//
// Data layout in HBM (structure of arrays, coalesced per step):
//   load[t][d][n]  int32   read once per (step, deployment): 256 B per wave
//   traj[t][n]     16 B    written once per step (optional): 1 KiB per wave
//   params/results SoA     read/written once per scenario
// LDS per workgroup: the catalog (48 B/type), the per-type pod capacity of the
// single-deployment fast path, the price tile(s) of the current hour for the
// regions the workgroup covers, and per-wave NodeClaim scratch.
//
// Karpenter provisioning is wave-cooperative: lanes that need a NodeClaim are
// served one after another (ballot), and for each of them all 64 lanes scan a
// strided slice of the catalog in LDS and reduce with cross-lane shuffles
// (max-fit and the lexicographic (score, type, zone, cap) argmin).
//
// Floating point: binary64, no contraction (pragma below + -ffp-contract=off),
// operation order identical to the spec, so results are bit-identical to the
// CPU oracle.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ccka.h"
#include "kparams.h"

#pragma clang fp contract(off)

namespace ccka {

#define CONSTANT __attribute__((address_space(4)))
typedef const CONSTANT ccka_world CWorld;

constexpr int WAVE = 64;
constexpr int CLAIM_FIXED = 7;  // pool, cap, zone, slot, s_cpu, s_mem, s_pods

__device__ __forceinline__ int rdl(int v, int lane) { return __builtin_amdgcn_readlane(v, lane); }
__device__ __forceinline__ uint32_t rdlu(uint32_t v, int lane) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, lane);
}
__device__ __forceinline__ double rdld(double v, int lane) {
  long long b = __double_as_longlong(v);
  int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffLL), lane);
  int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ long long rdll(long long v, int lane) {
  int lo = __builtin_amdgcn_readlane((int)(v & 0xffffffffLL), lane);
  int hi = __builtin_amdgcn_readlane((int)(v >> 32), lane);
  return ((long long)hi << 32) | (unsigned int)lo;
}
__device__ __forceinline__ int wave_max(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o));
  return v;
}
__device__ __forceinline__ void wave_argmin(double& s, int& idx) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double s2 = __shfl_xor(s, o);
    const int i2 = __shfl_xor(idx, o);
    if (s2 < s || (s2 == s && i2 < idx)) { s = s2; idx = i2; }
  }
}
__device__ __forceinline__ int capbit(int c) { return c == 0 ? CCKA_CAP_SPOT : CCKA_CAP_OD; }

// ---------------------------------------------------------------------------
// Philox-4x32-10 and the synthetic load generator (SEMANTICS.md §4)
// ---------------------------------------------------------------------------
__device__ __forceinline__ void philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                       uint32_t k0, uint32_t k1, uint32_t out[4]) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t lo0 = 0xD2511F53u * c0, hi0 = __umulhi(0xD2511F53u, c0);
    const uint32_t lo1 = 0xCD9E8D57u * c2, hi1 = __umulhi(0xCD9E8D57u, c2);
    const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

#ifndef CCKA_ROLLOUT_PART  // the other rollout_*.hip units include this file for the kernel template only
__global__ void __launch_bounds__(256) gen_load_kernel(GenParams g) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int d = blockIdx.y;
  if (i >= g.n) return;
  const uint64_t s = (uint64_t)(g.first_id + i);
  const uint32_t slo = (uint32_t)s, shi = (uint32_t)(s >> 32);
  const uint32_t k0 = (uint32_t)g.seed, k1 = (uint32_t)(g.seed >> 32);
  uint32_t u[4], v[4];
  philox(0xFFFFFFFFu, slo, shi, (uint32_t)d, k0, k1, u);
  philox(0xFFFFFFFEu, slo, shi, (uint32_t)d, k0, k1, v);
  const int64_t base = g.base_lo + (int64_t)(u[0] % (uint32_t)(g.base_hi - g.base_lo + 1));
  const int64_t amp = g.amp_lo + (int64_t)(u[1] % (uint32_t)(g.amp_hi - g.amp_lo + 1));
  const int phase = (int)(u[2] % 1440u);
  const bool burst = (int)(u[3] % 1000u) < g.burst_prob;
  const int bstart = (int)(v[0] % 1440u);
  for (int t = 0; t < g.T; ++t) {
    uint32_t e4[4];
    philox((uint32_t)t, slo, shi, (uint32_t)d, k0, k1, e4);
    const int64_t e = (int64_t)(e4[0] >> 16) + (int64_t)(e4[1] >> 16) + (int64_t)(e4[2] >> 16) +
                      (int64_t)(e4[3] >> 16) - 131072;
    int64_t val = base * (65536000LL + amp * (int64_t)g.sinq[(t + phase) % 1440]) / 65536000LL;
    val = val * (37837000LL + (int64_t)g.noise * e) / 37837000LL;
    if (burst && t >= bstart && t < bstart + g.burst_len) val = val * g.burst_mult / 1000;
    if (val < 0) val = 0;
    if (val > 0x7fffffff) val = 0x7fffffff;
    g.out[((int64_t)t * g.D + d) * g.n + i] = (int32_t)val;
  }
}
#endif

// ---------------------------------------------------------------------------
// Rollout kernel
// ---------------------------------------------------------------------------
// node info word: bit0 used | bits1-2 pool | bits3-12 type | bits13-14 zone | bit15 cap
__device__ __forceinline__ int ni_used(uint32_t x) { return x & 1u; }
__device__ __forceinline__ int ni_pool(uint32_t x) { return (x >> 1) & 3u; }
__device__ __forceinline__ int ni_type(uint32_t x) { return (x >> 3) & 1023u; }
__device__ __forceinline__ int ni_zone(uint32_t x) { return (x >> 13) & 3u; }
__device__ __forceinline__ int ni_cap(uint32_t x) { return (x >> 15) & 1u; }
__device__ __forceinline__ uint32_t ni_make(int pool, int type, int zone, int cap) {
  return 1u | (uint32_t)pool << 1 | (uint32_t)type << 3 | (uint32_t)zone << 13 | (uint32_t)cap << 15;
}

struct Lds {
  ccka_itype* types;   // [K]
  int* cap1;           // [K] pod capacity of deployment 0 from empty (D == 1 path)
  int* tile;           // current hour: region rl at tile + rl * rstride
  int rstride;         // ints per region: one hour's tile, or all 24 (all_hours)
  int* claims;         // [waves][MAXN][CLAIM_FIXED + DMAX]
  int K, Z, rmin;
};

__device__ __forceinline__ int tprice(const Lds& L, int rl, int k, int z, int c) {
  return L.tile[rl * L.rstride + (k * L.Z + z) * 2 + c];
}

// largest pod count of deployment d that fits on type k given sums; -1 if the
// type cannot hold the sums. (SEMANTICS §3.E fit rule)
template <int DMAX>
__device__ __forceinline__ int type_fit(const Lds& L, int k, int s_cpu, int s_mem, int s_pods, int rc,
                                        int rm) {
  if (DMAX == 1) {
    const int c = L.cap1[k];
    return c >= s_pods ? c - s_pods : -1;  // exact: floor((A - p*r)/r) = floor(A/r) - p
  }
  const ccka_itype& ty = L.types[k];
  if (s_cpu > ty.alloc_cpu_m || s_mem > ty.alloc_mem_mi || s_pods > ty.max_pods) return -1;
  int f = ty.max_pods - s_pods;
  if (rc > 0) f = min(f, (ty.alloc_cpu_m - s_cpu) / rc);
  if (rm > 0) f = min(f, (ty.alloc_mem_mi - s_mem) / rm);
  return f;
}

template <int DMAX>
__device__ __forceinline__ bool type_holds(const Lds& L, int k, int s_cpu, int s_mem, int s_pods) {
  if (DMAX == 1) return L.cap1[k] >= s_pods;
  const ccka_itype& ty = L.types[k];
  return s_cpu <= ty.alloc_cpu_m && s_mem <= ty.alloc_mem_mi && s_pods <= ty.max_pods;
}

__device__ __forceinline__ bool type_offered(const Lds& L, int rl, int k, uint32_t zm, uint32_t cm) {
  for (int z = 0; z < L.Z; ++z) {
    if (!(zm >> z & 1u)) continue;
    if ((cm & CCKA_CAP_SPOT) && tprice(L, rl, k, z, 0) > 0) return true;
    if ((cm & CCKA_CAP_OD) && tprice(L, rl, k, z, 1) > 0) return true;
  }
  return false;
}

// NodePool spec.limits: a new node of type k keeps the pool's CPU (millicores)
// and memory (MiB) capacity within the limits (-1: none)
__device__ __forceinline__ bool limit_ok(const Lds& L, int k, int use, int limit, int usem, int limitm) {
  return (limit < 0 || use + L.types[k].vcpu * 1000 <= limit) && (limitm < 0 || usem + L.types[k].mem_mi <= limitm);
}

// wave-cooperative j (max additional pods of d over candidate types). All
// arguments are wave-uniform.
template <int DMAX>
__device__ int wave_claim_j(const Lds& L, int rl, uint32_t zm, uint32_t cm, int s_cpu, int s_mem,
                            int s_pods, int rc, int rm, int use, int limit, int usem, int limitm, int lane) {
  int best = 0;
  for (int k = lane; k < L.K; k += WAVE) {
    if (!limit_ok(L, k, use, limit, usem, limitm)) continue;
    const int f = type_fit<DMAX>(L, k, s_cpu, s_mem, s_pods, rc, rm);
    if (f <= best) continue;
    if (!type_offered(L, rl, k, zm, cm)) continue;
    best = f;
  }
  return wave_max(best);
}

// wave-cooperative launch decision; returns packed idx (k*Z+z)*2+c or -1.
template <int DMAX>
__device__ int wave_launch(const Lds& L, int rl, uint32_t zm, uint32_t cm, int s_cpu, int s_mem,
                           int s_pods, int use, int limit, int usem, int limitm, double wc1000, double ci_gpwh,
                           int lane) {
  bool spot_only = false;
  if (cm & CCKA_CAP_SPOT) {
    bool any = false;
    for (int k = lane; k < L.K && !any; k += WAVE) {
      if (!type_holds<DMAX>(L, k, s_cpu, s_mem, s_pods) || !limit_ok(L, k, use, limit, usem, limitm)) continue;
      for (int z = 0; z < L.Z; ++z)
        if ((zm >> z & 1u) && tprice(L, rl, k, z, 0) > 0) { any = true; break; }
    }
    spot_only = __ballot(any) != 0;
  }
  double bs = __builtin_inf();
  int bi = 0x7fffffff;
  for (int k = lane; k < L.K; k += WAVE) {
    if (!type_holds<DMAX>(L, k, s_cpu, s_mem, s_pods) || !limit_ok(L, k, use, limit, usem, limitm)) continue;
    const double carbon = L.types[k].p_ref_w * ci_gpwh;
    for (int z = 0; z < L.Z; ++z) {
      if (!(zm >> z & 1u)) continue;
      for (int c = 0; c < 2; ++c) {
        if (!(cm & (uint32_t)capbit(c))) continue;
        if (spot_only && c != 0) continue;
        const int pr = tprice(L, rl, k, z, c);
        if (pr <= 0) continue;
        const double score = (double)pr + wc1000 * carbon;
        if (score < bs) { bs = score; bi = (k * L.Z + z) * 2 + c; }
      }
    }
  }
  wave_argmin(bs, bi);
  return bi == 0x7fffffff ? -1 : bi;
}

// 32-bit fast path of util = int32(usage*100 / (ready*req)) (exact: taken only
// when both operands fit in 31 bits; the int64 divide is a long software
// sequence on the GPU)
__device__ __forceinline__ int util_div(long long usage, long long den) {
  const long long num = usage * 100;
  if (num < 0x7fffffffLL && den < 0x7fffffffLL) return (int)((unsigned)num / (unsigned)den);
  return (int)(num / den);
}

// HPA proposal of one decision with a metric (replica_calculator.go
// GetResourceReplicas, SEMANTICS 3.C): usage (already clamped by the pod CPU
// limit) over `ready` pods, `cur` replicas; u = the utilisation. Phase C and
// the skewed schedule's record rebuild share it (the same binary64 operations).
__device__ __forceinline__ int hpa_prop(long long usage, int cur, int ready, int req, int target, double lo,
                                        double hi, int& u) {
  u = util_div(usage, (long long)ready * req);
  const double ratio = (double)u / (double)target;
  if (cur - ready > 0 && ratio > 1.0) {
    const int nu = util_div(usage, (long long)cur * req);
    const double nr = (double)nu / (double)target;
    if ((lo <= nr && nr <= hi) || nr < 1.0) return cur;
    return max(cur, (int)ceil(nr * (double)cur));
  }
  if (lo <= ratio && ratio <= hi) return cur;
  return (int)ceil(ratio * (double)ready);
}

// HPA behavior rules of one direction, hoisted into registers. wmask bit k:
// a record k+1 steps old is inside the policy period / stabilisation window.
struct Rule {
  int sel, n, stab_mask;
  int type[2], value[2], pmask[2];
};

// Hot deployment fields, hoisted out of the step loop into registers. Loaded
// once through a generic pointer: the compiler must keep them in registers
// (it cannot re-issue the loads across the loop's stores), so the loop runs
// with no scalar-memory waits (SMEM and LDS share lgkmcnt).
struct Dep {
  int scaler, minr, req_cpu, req_mem, limit, pdb, kmin, kmax, kcool;
  long long kthr, kact;
  double lo, hi;
  Rule up, dn;
};

__device__ __forceinline__ int window_mask(int window_s) {
  int m = 0;
#pragma unroll
  for (int k = 0; k < CCKA_HIST; ++k) m |= ((k + 1) * CCKA_STEP_SECONDS < window_s) ? (1 << k) : 0;
  return m;
}

__device__ __forceinline__ Rule load_rule(const ccka_hpa_rules* r, bool up) {
  Rule o;
  o.sel = r->select;
  o.n = r->n_policies;
  o.stab_mask = window_mask(r->stab_window_s);
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    o.type[q] = r->policies[q].type;
    o.value[q] = r->policies[q].value;
    o.pmask[q] = window_mask(r->policies[q].period_s);
  }
  return o;
}

__device__ __forceinline__ Dep load_dep(const ccka_deployment* d) {
  Dep o;
  o.scaler = d->scaler;
  o.minr = d->min_replicas;
  o.req_cpu = d->req_cpu_m;
  o.req_mem = d->req_mem_mi;
  o.limit = d->limit_cpu_m;
  o.pdb = d->pdb_member;
  o.kmin = d->keda_min;
  o.kmax = d->keda_max;
  o.kcool = d->keda_cooldown_s;
  o.kthr = d->keda_threshold;
  o.kact = d->keda_activation;
  o.lo = 1.0 - d->tolerance;
  o.hi = 1.0 + d->tolerance;
  o.up = load_rule(&d->up, true);
  o.dn = load_rule(&d->down, false);
  return o;
}

// Percent policy factor 1 +/- value/100 exactly as the spec writes it, made
// where it is used: the asm redefines the value, so the compiler cannot hoist
// the binary64 factors out of the step loop (four of them held across it
// spilled to scratch in the occupancy-2 instantiation)
__device__ __forceinline__ double pct_factor(int value, bool up) {
  asm volatile("" : "+v"(value));
  return up ? 1.0 + (double)value / 100.0 : 1.0 - (double)value / 100.0;
}

// rate limit of one direction (convertDesiredReplicasWithBehaviorRate)
__device__ __forceinline__ int rate_limit(const Rule& R, bool up, int cur, const int* delta) {
  if (R.sel == CCKA_SELECT_DISABLED) return cur;
  const bool min_sel = R.sel == CCKA_SELECT_MIN;
  long long res = (up == min_sel) ? 0x7fffffffLL : -0x80000000LL;
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    if (q >= R.n) break;
    int added = 0, removed = 0;
#pragma unroll
    for (int k = 0; k < CCKA_HIST; ++k)
      if (R.pmask[q] >> k & 1) {
        added += max(delta[k], 0);
        removed += max(-delta[k], 0);
      }
    const long long pst = (long long)cur - added + removed;
    long long pr;
    if (R.type[q] == CCKA_HPA_PODS) pr = up ? pst + R.value[q] : pst - R.value[q];
    // Percent: 1 +/- value/100 computed exactly as the spec writes it (on use:
    // rare, and no registers held across the step loop)
    else if (up) pr = (int)ceil((double)pst * pct_factor(R.value[q], true));
    else pr = (int)((double)pst * pct_factor(R.value[q], false));
    res = (up == min_sel) ? min(res, pr) : max(res, pr);
  }
  return (int)res;
}

// ---- closed-loop policy rollout: state persistence and features ----
// one 32-bit word per SoA row of the state block (8-byte values take two rows)
template <class T>
__device__ __forceinline__ void st_xfer(T& v, int32_t* st, int& k, int64_t N, int64_t i, bool save) {
  if constexpr (sizeof(T) == 8) {
    int32_t w2[2];
    if (save) {
      __builtin_memcpy(w2, &v, 8);
      st[(int64_t)k * N + i] = w2[0];
      st[(int64_t)(k + 1) * N + i] = w2[1];
    } else {
      w2[0] = st[(int64_t)k * N + i];
      w2[1] = st[(int64_t)(k + 1) * N + i];
      __builtin_memcpy(&v, w2, 8);
    }
    k += 2;
  } else if constexpr (sizeof(T) == 4) {
    int32_t x;
    if (save) { __builtin_memcpy(&x, &v, 4); st[(int64_t)k * N + i] = x; }
    else { x = st[(int64_t)k * N + i]; __builtin_memcpy(&v, &x, 4); }
    k += 1;
  } else {
    if (save) st[(int64_t)k * N + i] = v ? 1 : 0;
    else v = st[(int64_t)k * N + i] != 0;
    k += 1;
  }
}

// float -> bf16 bits, round to nearest even (finite inputs)
__device__ __forceinline__ uint16_t f2bf(float f) {
  uint32_t b;
  __builtin_memcpy(&b, &f, 4);
  return (uint16_t)((b + 0x7FFFu + ((b >> 16) & 1u)) >> 16);
}

// decision-history entries inside a window / period: entry k is (k + 1) * sync_s old
__device__ __forceinline__ int hist_n(int window_s, int sync_s) { return window_s > sync_s ? (window_s - 1) / sync_s : 0; }

// replicas added / removed by the scaler over the n newest HBM history entries
__device__ __forceinline__ void hist_sums(const int2* ring, int hpos, int hlen, int64_t stride, int n, int* add,
                                          int* rem) {
  int a = 0, r = 0, idx = hpos;
  for (int k = 0; k < n; ++k) {
    idx = idx == 0 ? hlen - 1 : idx - 1;
    const int dl = ring[(int64_t)idx * stride].y;
    a += max(dl, 0);
    r += max(-dl, 0);
  }
  *add = a;
  *rem = r;
}

// rate limit of one direction over the HBM history (one policy at a time:
// few live registers on this rare path)
__device__ int rate_long(const ccka_hpa_rules* R, bool up, int cur, int sync_s, const int2* ring, int hpos, int hlen,
                         int64_t stride) {
  if (R->select == CCKA_SELECT_DISABLED) return cur;
  const bool min_sel = R->select == CCKA_SELECT_MIN;
  long long res = (up == min_sel) ? 0x7fffffffLL : -0x80000000LL;
  for (int q = 0; q < R->n_policies; ++q) {
    const ccka_hpa_policy& P = R->policies[q];
    int add, rem;
    hist_sums(ring, hpos, hlen, stride, min(hist_n(P.period_s, sync_s), hlen), &add, &rem);
    const long long pst = (long long)cur - add + rem;
    long long pr;
    if (P.type == CCKA_HPA_PODS) pr = up ? pst + P.value : pst - P.value;
    else if (up) pr = (int)ceil((double)pst * pct_factor(P.value, true));
    else pr = (int)((double)pst * pct_factor(P.value, false));
    res = (up == min_sel) ? min(res, pr) : max(res, pr);
  }
  return (int)res;
}

// HPA behavior (stabilisation + rate limits) over the HBM decision history:
// windows up to 3600 s, up to 4 policies per direction, hpa_sync_s sub-steps
// (SEMANTICS 3.C). Entry k of this (deployment, scenario) lives at
// ring[((hpos - 1 - k) mod hlen) * stride].
__device__ int behavior_long(const ccka_hpa_rules* up, const ccka_hpa_rules* dn, int dstab, int sync_s, int cur,
                             int proposal, int minr, int mx, const int2* ring, int hpos, int hlen, int64_t stride) {
  const int nu = min(hist_n(up->stab_window_s, sync_s), hlen), nd = min(hist_n(dstab, sync_s), hlen);
  int upr = proposal, dnr = proposal, idx = hpos;
  for (int k = 0; k < max(nu, nd); ++k) {
    idx = idx == 0 ? hlen - 1 : idx - 1;
    const int rx = ring[(int64_t)idx * stride].x;
    if (rx) {
      if (k < nu) upr = min(upr, rx - 1);
      if (k < nd) dnr = max(dnr, rx - 1);
    }
  }
  int rc = max(cur, upr);
  rc = min(rc, dnr);
  int lo = minr, hi = mx;
  if (rc > cur) hi = min(hi, max(rate_long(up, true, cur, sync_s, ring, hpos, hlen, stride), cur));
  else if (rc < cur) lo = max(lo, min(rate_long(dn, false, cur, sync_s, ring, hpos, hlen, stride), cur));
  return rc < lo ? lo : (rc > hi ? hi : rc);
}

// W2 fragments the fused loop's MLP reads ahead of their MFMA (A/B macro)
#ifndef MLP_W2PF
#define MLP_W2PF 2
#endif
#ifndef MLP_BPF
#define MLP_BPF 1
#endif
// ---- the learned policy inside the step loop (fused closed loop, POL > 0) ----
// The MLP of mlp.hip (H1^T = W1^T X^T, H2^T = W2^T H1^T, Y^T = W3^T H2^T on
// v_mfma_f32_32x32x16_bf16, each accumulator chained as the next layer's B
// operand) evaluated on one 32-state tile, with the MFMAs issued in exactly
// mlp_kernel's accumulation order, so the outputs are bit-identical to the
// standalone kernel's. W2 fragments and the biases from LDS, W1 / W3 fragments
// from L2.
namespace {
typedef mlp_bf16x8 pbf16x8;
typedef float pf32x16 __attribute__((ext_vector_type(16)));
typedef float pf32x4 __attribute__((ext_vector_type(4)));
typedef short pshort2v __attribute__((ext_vector_type(2)));
typedef float pf32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 pbf16x2v __attribute__((ext_vector_type(2)));

__device__ __forceinline__ pf32x16 pmfma(const pbf16x8& a, const pbf16x8& b, const pf32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ pbf16x8 prelu_pack(const pf32x16& a, int s) {
  pbf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; j += 2) {
    const pbf16x2v b = __builtin_convertvector((pf32x2){a[8 * s + j], a[8 * s + j + 1]}, pbf16x2v);
    const pshort2v v = __builtin_elementwise_max(__builtin_bit_cast(pshort2v, b), (pshort2v){0, 0});
    r[j] = v.x;
    r[j + 1] = v.y;
  }
  return r;
}
__device__ __forceinline__ pf32x16 pbias_tile(const float* b, int h) {
  pf32x16 a;
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const pf32x4 v = *reinterpret_cast<const pf32x4*>(b + 8 * g + 4 * h);
    a[4 * g + 0] = v[0];
    a[4 * g + 1] = v[1];
    a[4 * g + 2] = v[2];
    a[4 * g + 3] = v[3];
  }
  return a;
}
// Y^T of one 32-state tile (xf: its X^T fragments); registers 0..3 of the
// result = outputs 4h..4h+3 of the lane's column state. W1 fragments come
// from L2 one row block ahead (their latency hides under the block's MFMAs
// and epilogue), W2 / W3 fragments and the biases from LDS.
// w1b0: W1's first row block, loaded by the caller ahead of the tile; the
// call reloads it into w1b0 during its second layer for the next tile
__device__ __forceinline__ pf32x16 mlp_tile(const pbf16x8 (&xf)[MLP_IN / 16], const pbf16x8* __restrict__ w1f,
                                            pbf16x8 (&w1b0)[MLP_IN / 16], const pbf16x8* s_w2, const pbf16x8* s_w3,
                                            const float* s_b, int lane, int h) {
  constexpr int KS1 = MLP_IN / 16, KS2 = MLP_HID / 16, NB = MLP_HID / 32;
  pbf16x8 hh[KS2];
  pbf16x8 wc[KS1], wn[KS1];
#pragma unroll
  for (int s = 0; s < KS1; ++s) wc[s] = w1b0[s];
  // the next block's bias tile (the accumulator's initial value) is read from
  // LDS before this block's epilogue, which covers its latency (MLP_BPF)
  pf32x16 cb = pbias_tile(s_b, h);
#pragma unroll
  for (int n = 0; n < NB; ++n) {
    if (n + 1 < NB) {
#pragma unroll
      for (int s = 0; s < KS1; ++s) wn[s] = w1f[((n + 1) * KS1 + s) * 64 + lane];
    }
    pf32x16 c = MLP_BPF ? cb : pbias_tile(s_b + 32 * n, h);
#pragma unroll
    for (int s = 0; s < KS1; ++s) c = pmfma(wc[s], xf[s], c);
    if (MLP_BPF) cb = pbias_tile(n + 1 < NB ? s_b + 32 * (n + 1) : s_b + MLP_HID, h);
    hh[2 * n] = prelu_pack(c, 0);
    hh[2 * n + 1] = prelu_pack(c, 1);
#pragma unroll
    for (int s = 0; s < KS1; ++s) wc[s] = wn[s];
    __builtin_amdgcn_sched_barrier(0);  // bounded live ranges: the rollout state shares the register file
  }
#pragma unroll
  for (int s = 0; s < KS1; ++s) w1b0[s] = w1f[s * 64 + lane];  // the next tile's (L2 latency under layer 2)
  pf32x16 y = pbias_tile(s_b + 2 * MLP_HID, h);
  // W2 fragments from LDS MLP_W2PF MFMAs ahead (one wave per SIMD: nothing
  // else hides an LDS read issued just before its MFMA)
  constexpr int PF = MLP_W2PF;
  // the read-ahead ring is indexed by kk % PF for fragment m * KS2 + kk: that
  // is the fragment's own slot only while PF divides KS2
  static_assert(KS2 % PF == 0, "MLP_W2PF must divide MLP_HID / 16");
  pbf16x8 wq[PF];
#pragma unroll
  for (int j = 0; j < PF; ++j) wq[j] = s_w2[j * 64 + lane];
#pragma unroll
  for (int m = 0; m < NB; ++m) {
    pf32x16 c = MLP_BPF ? cb : pbias_tile(s_b + MLP_HID + 32 * m, h);
    const pbf16x8 w3a = s_w3[(2 * m) * 64 + lane], w3b = s_w3[(2 * m + 1) * 64 + lane];  // used after the chain
#pragma unroll
    for (int kk = 0; kk < KS2; ++kk) {
      const pbf16x8 w = wq[kk % PF];
      const int nx = m * KS2 + kk + PF;  // the fragment PF ahead (across m-blocks)
      if (nx < NB * KS2) wq[kk % PF] = s_w2[nx * 64 + lane];
      c = pmfma(w, hh[kk], c);
    }
    if (MLP_BPF && m + 1 < NB) cb = pbias_tile(s_b + MLP_HID + 32 * (m + 1), h);
    y = pmfma(w3a, prelu_pack(c, 0), y);
    y = pmfma(w3b, prelu_pack(c, 1), y);
    __builtin_amdgcn_sched_barrier(0);
  }
  return y;
}
// v_permlane32_swap_b32: x's lanes 32..63 <-> y's lanes 0..31
// (tools/probe/permlane.hip documents the lanes). Only for operands held in
// separate scalars: ROCm 7.2 lowers a swap of two elements of one MFMA
// accumulator vector with both operands in the same register, so the outputs
// cross the lane halves by __shfl_xor instead.
__device__ __forceinline__ void pswap32(uint32_t& x, uint32_t& y) {
  const auto r = __builtin_amdgcn_permlane32_swap(x, y, false, false);
  x = r[0];
  y = r[1];
}
__device__ __forceinline__ void pol_philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0,
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
}  // namespace

// Diagnostic phase stamps (tools/build_variants.py NAME="r@rollout.hip:-DGK_STAMPS",
// tools/gk_stamps.py): s_memtime deltas per phase of the step loop
// accumulated per wave, at wave-uniform points
#ifdef GK_STAMPS
constexpr bool kGKS = true;
#else
constexpr bool kGKS = false;
#endif
#define GK_STAMP(k)                                             \
  do {                                                          \
    if constexpr (kGKS) {                                       \
      const unsigned long long now_ = __builtin_amdgcn_s_memtime(); \
      gst[k] += now_ - glast;                                   \
      glast = now_;                                             \
    }                                                           \
  } while (0)

// POL: 0 = rule-based rollout (steps [t0, t1), resumable); 1 / 2 = the fused
// closed loop over the whole horizon: before every step the scenario's
// features, the MLP (MFMA, both 32-lane halves of the wave as two tiles) and
// the action (1: policy_act_kernel's mapping, 2: policy_sample_kernel's
// sampling) -- one launch instead of 4T + 1, the state never leaves registers.
// SK: lane-skewed schedule (two to four deployments, round 6): each lane keeps its
// own step counter; a step whose outcome is fixed by the state of the lane's
// last full step and the step's load samples (every HPA keeps its replica
// count, no readiness / hour / peak-window / consolidation boundary, nothing
// pending) is a *quiet step* (threshold compares, accounting, the record);
// every other step stalls the lane, and the wave runs the full step for all
// its stalled lanes together (the single-deployment kernel's event batching,
// rollout_d1.hip, for D <= 4 deployments). Host-checked preconditions
// (sk_eligible in ccka_abi.cpp): HPA / static deployments, one decision per
// step over the register rings, every hour's price tiles in LDS, no detail,
// drift, replacement or multi-node consolidation, the whole horizon in one
// launch. Trajectory records scenario-major [N][T].
#ifndef SK_OCC2  // skewed instantiations at two waves per SIMD (variant builds)
#define SK_OCC2 0
#endif
template <int DMAX, int MAXN, int POL = 0, int SK = 0>
__global__ void __launch_bounds__(256, ((POL == 0 && DMAX == 1 && MAXN <= 8) || (SK && SK_OCC2)) ? 2 : 1)
    rollout_kernel(KParams p) {
  static_assert(POL == 0 || (DMAX == 1 && MAXN <= 8), "fused closed loop: one deployment, <= 8 slots");
  static_assert(SK == 0 || POL == 0, "the skewed schedule is the rule-based rollout's");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  // world through the constant address space for rare (profile-switch) reads;
  // hot fields are hoisted into registers below
  CWorld* w = (CWorld*)p.w;
  const ccka_world* gw = p.w;
  const int K = p.K, Z = p.Z, D = p.D, NP = p.P, NN = p.maxn;
  const int tid = threadIdx.x, lane = tid & (WAVE - 1), wid = tid >> 6;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + tid;
  const bool active = i < p.N;
  DetailDev* const det = !SK && active && p.detail ? p.detail + i : nullptr;  // (SK worlds: no detail)

  Lds L;
  L.K = K;
  L.Z = Z;
  L.types = reinterpret_cast<ccka_itype*>(smem);
  L.cap1 = reinterpret_cast<int*>(smem + p.lds_off_cap1);
  L.tile = reinterpret_cast<int*>(smem + p.lds_off_tile);
  L.claims = reinterpret_cast<int*>(smem + p.lds_off_claims) + wid * MAXN * (CLAIM_FIXED + DMAX);
  int* s_rng = reinterpret_cast<int*>(smem + p.lds_off_misc);
  double* s_ci = reinterpret_cast<double*>(smem + p.lds_off_ci);  // [span][24][gpwmin, gpwh]

  // ---- stage the catalog, the region range of this block ----
  static_assert(sizeof(ccka_itype) == 48, "catalog entries are staged as three 16-byte words");
  for (int k = tid; k < K; k += blockDim.x) {
    // three 16-byte words (a struct copy would go through a private temporary)
    const int4* src = reinterpret_cast<const int4*>(p.types + k);
    const int4 a = src[0], b = src[1], c = src[2];
    int4* dst = reinterpret_cast<int4*>(L.types + k);
    dst[0] = a;
    dst[1] = b;
    dst[2] = c;
    if (DMAX == 1) {  // vcpu, alloc_cpu_m, alloc_mem_mi, max_pods are the first word
      const int rc = w->deploy[0].req_cpu_m, rm = w->deploy[0].req_mem_mi;
      int f = a.w;
      if (rc > 0) f = min(f, a.y / rc);
      if (rm > 0) f = min(f, a.z / rm);
      L.cap1[k] = f;
    }
  }
  const int my_r = active ? (p.region ? (int)p.region[i] : 0) : 0x7fffffff;
  if (tid == 0) { s_rng[0] = 0x7fffffff; }
  __syncthreads();
  if (active) atomicMin(&s_rng[0], my_r);
  __syncthreads();
  L.rmin = s_rng[0] == 0x7fffffff ? 0 : s_rng[0];
  const int rl = active ? my_r - L.rmin : 0;
  // price-tile row of this lane's region and hour: every hour staged
  // (all_hours): tile_base + (rl * 24 + hour) * tile_ints, so lanes at
  // different hours (SK) read their own; else the staged hour's tile of rl
  int rlx = rl;
  const int tile_ints = K * Z * 2;
  int* const tile_base = L.tile;
  for (int x = tid; x < p.span * 24; x += blockDim.x) {
    const int rg = min(L.rmin + x / 24, p.R - 1);
    s_ci[x * 2 + 0] = p.ci_gpwmin[rg * 24 + x % 24];
    s_ci[x * 2 + 1] = p.ci_gpwh[rg * 24 + x % 24];
  }
  __syncthreads();
  L.rstride = tile_ints;
  if (p.all_hours) {
    // small catalogs: stage every hour's tiles once -> no barrier in the step loop
    for (int rr = 0; rr < p.span; ++rr) {
      const int rg = L.rmin + rr;
      if (rg >= p.R) break;
      const int* src = p.price + (int64_t)rg * 24 * tile_ints;
      for (int x = tid; x < 24 * tile_ints; x += blockDim.x) tile_base[rr * 24 * tile_ints + x] = src[x];
    }
    __syncthreads();
  }

  // fused closed loop: W2 (128 KiB) and W3 (16 KiB) fragments and the biases in LDS
  constexpr int NW2 = (MLP_HID / 32) * (MLP_HID / 16) * 64, NW3 = (MLP_HID / 16) * 64;
  const pbf16x8* s_w2 = reinterpret_cast<const pbf16x8*>(smem + p.lds_off_mlp);
  const pbf16x8* s_w3 = s_w2 + NW2;
  const float* s_mb = reinterpret_cast<const float*>(s_w3 + NW3);
  if constexpr (POL != 0) {
    pbf16x8* dw = reinterpret_cast<pbf16x8*>(smem + p.lds_off_mlp);
    for (int x = tid; x < NW2; x += blockDim.x) dw[x] = p.w2f[x];
    for (int x = tid; x < NW3; x += blockDim.x) dw[NW2 + x] = p.w3f[x];
    float* db = const_cast<float*>(s_mb);
    for (int x = tid; x < 2 * MLP_HID + 32; x += blockDim.x) db[x] = p.mlp_b[x];
    __syncthreads();
  }

  // ---- hoisted world fields ----
  Dep dep[DMAX];
#pragma unroll
  for (int d = 0; d < DMAX; ++d) dep[d] = load_dep(&gw->deploy[d < D ? d : 0]);
  int pbudget[CCKA_MAX_POOLS], plimit[CCKA_MAX_POOLS];
#pragma unroll
  for (int q = 0; q < CCKA_MAX_POOLS; ++q) {
    pbudget[q] = gw->pools[q].budget_pct;
    plimit[q] = gw->pools[q].limit_cpu_m;
  }
  const int pdb_pct = gw->pdb_min_available_pct;
  // (SK worlds have none of the three: their code folds away)
  const bool gdrift = !SK && (gw->disrupt_ext & CCKA_DISRUPT_DRIFT) != 0;
  const bool greplace = !SK && (gw->disrupt_ext & CCKA_DISRUPT_REPLACE) != 0;
  const bool gmulti = !SK && (gw->disrupt_ext & CCKA_DISRUPT_MULTI) != 0;
  const int slo_util = gw->slo_util_pct;
  const int base_nodes = gw->base_nodes, base_type = gw->base_type;

  // ---- per-scenario parameters ----
  const double cw = active && p.cw ? p.cw[i] : gw->carbon_weight;
  double wc1000 = cw * 1000.0;  // the fused closed loop sets it every step
  int pwi = 0;                  // ... and its argmin-table weight index (16 * weight)
  const int reset_ca = active && p.reset_ca ? (int)p.reset_ca[i] : gw->reset_ca_s;
  const int pswitch = active && p.pswitch ? (int)p.pswitch[i] : gw->peak_switch;

  int target[DMAX], maxr[DMAX], dnmask[DMAX];
  uint32_t capsel[DMAX];
  int replicas[DMAX], last_active[DMAX], placed[DMAX], rpods[DMAX];
  int rec[DMAX][CCKA_HIST], delta[DMAX][CCKA_HIST];
  uint32_t recv[DMAX];
#pragma unroll
  for (int d = 0; d < DMAX; ++d) {
    const ccka_deployment& dp = gw->deploy[d < D ? d : 0];
    target[d] = dp.target_util_pct;
    maxr[d] = dp.max_replicas;
    int dstab = dp.down.stab_window_s;
    if (active && dp.scaler == CCKA_SCALER_HPA) {
      if (p.target) target[d] = p.target[i];
      if (p.maxr) maxr[d] = p.maxr[i];
      if (p.down_stab) dstab = p.down_stab[i];
    }
    dnmask[d] = window_mask(dstab);
    capsel[d] = active && p.cap_sel ? (uint32_t)p.cap_sel[i] : dp.cap_sel;
    replicas[d] = d < D ? dp.replicas0 : 0;
    last_active[d] = 0;
    placed[d] = 0;
    rpods[d] = 0;
    recv[d] = 0;
#pragma unroll
    for (int k = 0; k < CCKA_HIST; ++k) { rec[d][k] = 0; delta[d][k] = 0; }
  }
  // pools: current policy, consolidateAfter, zone and capacity-type masks
  int ppol[CCKA_MAX_POOLS], pca[CCKA_MAX_POOLS], puse[CCKA_MAX_POOLS];
  uint32_t pzm[CCKA_MAX_POOLS], pcm[CCKA_MAX_POOLS];
#pragma unroll
  for (int q = 0; q < CCKA_MAX_POOLS; ++q) {
    ppol[q] = 0; pca[q] = 0; pzm[q] = 0; pcm[q] = 0; puse[q] = 0;
    if (q < NP) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        auto& x = s == 0 ? w->pools[q].base : w->pools[q].profile[CCKA_PROFILE_RESET];
        if (x.policy != CCKA_POLICY_KEEP) ppol[q] = x.policy;
        if (x.consolidate_after_s >= 0) pca[q] = s == 1 ? reset_ca : x.consolidate_after_s;
        if (x.zone_mask) pzm[q] = x.zone_mask;
        if (x.cap_mask) pcm[q] = x.cap_mask;
      }
    }
  }
  // node slots; `used` / `rdy` are bitmasks over slots. nprice caches the
  // slot's offering price for the current hour, ncap (D == 1) its pod capacity.
  uint32_t ninfo[MAXN];
  uint32_t nsrc[MAXN];  // replacement node: bit m = it replaces slot m (SEMANTICS 3.G2, 3.G3)
  int nready[MAXN], nlast[MAXN], nprice[MAXN], ncap[MAXN];
  int npods[MAXN][DMAX];
#pragma unroll
  for (int n = 0; n < MAXN; ++n) {
    ninfo[n] = 0; nready[n] = 0; nlast[n] = 0; nprice[n] = 0; ncap[n] = 0; nsrc[n] = 0;
#pragma unroll
    for (int d = 0; d < DMAX; ++d) npods[n][d] = 0;
  }  // slots tainted karpenter.sh/disrupted: sources of an in-flight pre-spun
  // replacement and those replacements (SEMANTICS 3.G0/G2)
  auto taint_mask = [&]() {
    uint32_t m = 0;
#pragma unroll
    for (int n = 0; n < MAXN; ++n)
      if (nsrc[n]) m |= (1u << n) | nsrc[n];
    return m;
  };

  uint32_t used = 0, rdy = 0;
  // memory capacity (MiB) of pool q's nodes: recounted where a limits.memory
  // applies (rare) instead of a register per pool
  auto pool_mem = [&](int q) {
    int m = 0;
#pragma unroll
    for (int n = 0; n < MAXN; ++n)
      if (((used >> n) & 1u) && ni_pool(ninfo[n]) == q) m += L.types[ni_type(ninfo[n])].mem_mi;
    return m;
  };
  const uint32_t slot_mask = NN >= 32 ? 0xFFFFFFFFu : ((1u << NN) - 1u);
  int next_ready = 0x7fffffff;  // earliest ready_step among not-ready nodes
  int nsp = 0, nod = 0;         // Karpenter nodes by capacity type
  // exact skip of the disruption phase: re-evaluate only when something it
  // depends on changed (g_dirty) or a node crosses its consolidateAfter /
  // readiness threshold (g_wake)
  bool g_dirty = true;
  int g_wake = 0;

  int profile = -1;
  long long cost = 0, pend_min = 0, burn = 0, base_price = 0;
  long long energy_nw = 0, e_hour = 0;  // exact nanowatt-minutes (SEMANTICS §3.H)
  double gco2 = 0.0, ci_gpwmin = 0.0, ci_gpwh = 0.0;
  int slo = 0, nmin_spot = 0, nmin_od = 0, launches = 0, deletions = 0, peak_nodes = 0;
  uint32_t last_choice = 0xFFFFFFFFu, hash = 2166136261u;
  const ccka_itype bt = p.types[base_type];
  const long long base_nw =
      (long long)base_nodes * (bt.idle_nw + bt.dyn_nw_per_m * (long long)(gw->base_util * (double)bt.alloc_cpu_m));
  const int ps = gw->peak_start_min, pe = gw->peak_end_min;
  const int delay = gw->provision_delay_steps;
  int hpos = 0;  // HBM history write position (p.hlen > 0)

  // load samples are software-pipelined one step ahead: the HBM latency of
  // step t+1's coalesced read hides behind step t's decision work
  int Lnext[DMAX];
  // load column: the scenario's own trace, or its shared trace (policy sweeps)
  const int64_t lcol = !active ? 0 : (p.trace_mod > 0 ? (p.first_id + i) % p.trace_mod : i);
  const int32_t* lptr = p.load + lcol;
  const int64_t lstride = p.NL;
  int hour = -1;

  // ---- persisted state (closed-loop policy rollout): the loop-carried
  // variables in one fixed order, loaded before the first step of a resumed
  // launch and saved after its last ----
  auto state_io = [&](bool save) {
    int32_t* st = p.state;
    const int64_t sN = p.N;
    int k = 0;
#pragma unroll
    for (int d = 0; d < DMAX; ++d) {
      st_xfer(replicas[d], st, k, sN, i, save);
      st_xfer(last_active[d], st, k, sN, i, save);
      st_xfer(placed[d], st, k, sN, i, save);
      st_xfer(rpods[d], st, k, sN, i, save);
      st_xfer(recv[d], st, k, sN, i, save);
#pragma unroll
      for (int h = 0; h < CCKA_HIST; ++h) {
        st_xfer(rec[d][h], st, k, sN, i, save);
        st_xfer(delta[d][h], st, k, sN, i, save);
      }
    }
#pragma unroll
    for (int q = 0; q < CCKA_MAX_POOLS; ++q) {
      st_xfer(ppol[q], st, k, sN, i, save);
      st_xfer(pca[q], st, k, sN, i, save);
      st_xfer(puse[q], st, k, sN, i, save);
      st_xfer(pzm[q], st, k, sN, i, save);
      st_xfer(pcm[q], st, k, sN, i, save);
    }
#pragma unroll
    for (int n = 0; n < MAXN; ++n) {
      st_xfer(ninfo[n], st, k, sN, i, save);
      st_xfer(nsrc[n], st, k, sN, i, save);
      st_xfer(nready[n], st, k, sN, i, save);
      st_xfer(nlast[n], st, k, sN, i, save);
      st_xfer(nprice[n], st, k, sN, i, save);
      st_xfer(ncap[n], st, k, sN, i, save);
#pragma unroll
      for (int d = 0; d < DMAX; ++d) st_xfer(npods[n][d], st, k, sN, i, save);
    }
    st_xfer(used, st, k, sN, i, save);
    st_xfer(rdy, st, k, sN, i, save);
    st_xfer(next_ready, st, k, sN, i, save);
    st_xfer(nsp, st, k, sN, i, save);
    st_xfer(nod, st, k, sN, i, save);
    st_xfer(g_dirty, st, k, sN, i, save);
    st_xfer(g_wake, st, k, sN, i, save);
    st_xfer(profile, st, k, sN, i, save);
    st_xfer(cost, st, k, sN, i, save);
    st_xfer(pend_min, st, k, sN, i, save);
    st_xfer(burn, st, k, sN, i, save);
    st_xfer(base_price, st, k, sN, i, save);
    st_xfer(energy_nw, st, k, sN, i, save);
    st_xfer(e_hour, st, k, sN, i, save);
    st_xfer(gco2, st, k, sN, i, save);
    st_xfer(ci_gpwmin, st, k, sN, i, save);
    st_xfer(ci_gpwh, st, k, sN, i, save);
    st_xfer(slo, st, k, sN, i, save);
    st_xfer(nmin_spot, st, k, sN, i, save);
    st_xfer(nmin_od, st, k, sN, i, save);
    st_xfer(launches, st, k, sN, i, save);
    st_xfer(deletions, st, k, sN, i, save);
    st_xfer(peak_nodes, st, k, sN, i, save);
    st_xfer(last_choice, st, k, sN, i, save);
    st_xfer(hash, st, k, sN, i, save);
    st_xfer(hpos, st, k, sN, i, save);
    st_xfer(hour, st, k, sN, i, save);
    // k is a compile-time constant here (every loop above is unrolled): the
    // trap is folded away while the sequence and state_words() agree, and
    // stops the kernel before a lane writes past its rows if they ever differ
    if (k != state_words(DMAX, MAXN)) __builtin_trap();
  };
  const int t0 = p.t0, t1 = p.t1;
  if (p.state && p.state_load) {
    if (active) state_io(false);
    // the hour's price tiles (block-uniform: every lane is at the same minute)
    const int h0 = ((gw->start_minute + t0) % 1440) / 60;
    if (p.all_hours) {
      rlx = rl * 24 + max(hour, 0);  // the restored hour's row
    } else {
      for (int rr = 0; rr < p.span; ++rr) {
        const int rg = L.rmin + rr;
        if (rg >= p.R) break;
        const int* src = p.price + ((int64_t)rg * 24 + h0) * tile_ints;
        for (int x = tid; x < tile_ints; x += blockDim.x) tile_base[rr * tile_ints + x] = src[x];
      }
      __syncthreads();
    }
    // inactive lanes follow the block's hour sequence (the restage barrier is block-uniform)
    if (!active) hour = t0 > 0 ? ((gw->start_minute + t0 - 1) % 1440) / 60 : -1;
  }
#pragma unroll
  for (int d = 0; d < DMAX; ++d) Lnext[d] = lptr[((int64_t)min(t0, p.T - 1) * D + (d < D ? d : 0)) * lstride];
  int minute = (gw->start_minute + t0) % 1440;

  // policy features of step tq from the state after step tq - 1 (SEMANTICS 5):
  // integers scaled by powers of two (exact in fp32), rounded to bf16 -- the
  // oracle computes the same bits; packed in pairs (feature 2k in the low half
  // of word k, the memory order of a [64] bf16 row)
  auto feat_words = [&](int tq, uint32_t (&fw)[32]) {
    int reps = 0, rd = 0;
#pragma unroll
    for (int d = 0; d < DMAX; ++d)
      if (d < D) { reps += replicas[d]; rd += rpods[d]; }
    const int mf = (gw->start_minute + tq) % 1440, hf = mf / 60;
    const bool pk = pswitch && (ps <= pe ? (mf >= ps && mf < pe) : (mf >= ps || mf < pe));
    uint16_t f[64];
    f[0] = f2bf(1.0f);
    f[1] = f2bf((float)reps * 0.0625f);
    f[2] = f2bf((float)rd * 0.0625f);
    f[3] = f2bf((float)(reps - rd) * 0.0625f);
    // the sample of step min(tq, T - 1): Lnext[0] holds it at the top of step
    // tq and after the last one (no second load of the same word)
    f[4] = f2bf((float)Lnext[0] * (1.0f / 1024.0f));
    f[5] = f2bf((float)nsp);
    f[6] = f2bf((float)nod);
    f[7] = f2bf(pk ? 1.0f : 0.0f);
    f[8] = f2bf((float)s_ci[(rl * 24 + hf) * 2 + 1]);
    f[9] = f2bf((float)burn * (1.0f / 65536.0f));
#pragma unroll
    for (int hh = 0; hh < 24; ++hh) f[10 + hh] = hh == hf ? (uint16_t)0x3F80 : (uint16_t)0;  // bf16 1.0 / 0
#pragma unroll
    for (int n = 0; n < 16; ++n) {
      int pods = 0, code = 0;
      if (n < MAXN && (used >> n & 1u)) {
#pragma unroll
        for (int d = 0; d < DMAX; ++d) pods += d < D ? npods[n < MAXN ? n : 0][d] : 0;
        code = 1 + ni_cap(ninfo[n < MAXN ? n : 0]) + ((rdy >> n & 1u) ? 0 : 2);
      }
      f[34 + n] = f2bf((float)pods * 0.0625f);
      if (n < 14) f[50 + n] = f2bf((float)code);
    }
#pragma unroll
    for (int k = 0; k < 32; ++k) fw[k] = (uint32_t)f[2 * k] | (uint32_t)f[2 * k + 1] << 16;
  };
  auto store_feat = [&](uint16_t* row, const uint32_t (&fw)[32]) {
    uint4* dst = reinterpret_cast<uint4*>(row);
#pragma unroll
    for (int q = 0; q < 8; ++q) dst[q] = make_uint4(fw[4 * q], fw[4 * q + 1], fw[4 * q + 2], fw[4 * q + 3]);
  };

  // ---- SK: the lane-skewed schedule's state ----
#ifndef SK_S_V  // A/B of the quiet steps per pass (variant builds): 32 samples held per lane
// (two deployments x 8 / 16 / 32 quiet steps per pass: 31.4 / 29.0 / 31.3 ms at 1e5 x 1440)
#define SK_S_V (32 / DMAX > 2 ? 32 / DMAX : 2)
#endif
  constexpr int SKS = SK ? (SK_S_V) : 1;  // quiet steps per iteration and lane
  constexpr int SKD = SK ? DMAX : 1;
  constexpr int UQ = 0x7fffffff;  // "any usage" threshold
#ifndef SK_LANE_F2  // lane-local provisioning on the skewed schedule (variant builds)
#define SK_LANE_F2 0
#endif
#ifndef SK_K_V  // full-step cadence in passes (variant builds)
#define SK_K_V 1
#endif
  int skpass = 0;    // passes (wave-uniform)
  int tl = t0;       // the lane's next step
  bool ev = true;    // ... runs the full step
  int nxt = 0;       // first step that needs the full step again
  int tq = t0;       // quiet steps [tq, tl) not yet flushed into the per-step sums
  // per deployment, from the lane's last full step: the step keeps the replica
  // count iff usage < q_ulim and (usage >= q_pge or t <= q_hold); usage >=
  // q_slo is an SLO miss
  int q_ulim[SKD], q_pge[SKD], q_hold[SKD], q_slo[SKD], q_rcap[SKD];  // q_rcap: ready pods * CPU limit
  float q_R[SKD];          // max over ready slots of pods / allocatable CPU (saturation bound)
  long long q_W[SKD];      // sum over ready slots of dyn_nw_per_m * pods
  uint32_t q_usum[SKD];    // sum of the quiet steps' upp since the flush
  uint32_t q_ran = 0;      // bit d: the deployment's HPA runs with a metric
  uint32_t q_atmax = 0;    // bit d: at maxReplicas (a quiet step's proposal may exceed cur)
  uint32_t q_rawm[SKD];    // ring entries pushed by quiet steps as raw usages (proposal != cur)
  // the tolerance band as utilisations, per deployment (constant: the
  // scenario's target): lo <= fl(u / target) <= hi <=> ulo <= u <= uhi;
  // packed ulo | uhi << 16
  uint32_t q_band[SKD];
  long long q_sidle = 0, q_corr = 0;  // base + idle energy per step; saturated-step corrections
  int q_pend = 0, q_reps = 0, q_w0 = 0;
  bool q_sloall = false;   // pods pending: every step misses the SLO
  int Lq[SKS][SKD];        // the next quiet steps' load samples
  // diagnostic schedule counters (SK_STATS variant builds only, tools/sk_stats.py):
  // stalls by the reason of the lane's last full step's nxt (0 disruption
  // pending, 1 pods not placed, 2 consolidation wake, 3 node ready, 4 hour /
  // peak boundary), 5 HPA outside its thresholds, 6 live lane-passes, 7 lane
  // full steps, 8 lane quiet steps, 9 wave full-step runs, 10 wave passes
#ifdef SK_STATS
  constexpr bool kSKS = SK != 0;
#else
  constexpr bool kSKS = false;
#endif
  uint32_t sks_c[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};  // 11: lanes served by provisioning
  int sks_why = 0;
#pragma unroll
  for (int d = 0; d < SKD; ++d) {
    q_ulim[d] = 0; q_pge[d] = 0; q_hold[d] = 0; q_slo[d] = UQ; q_rcap[d] = UQ;
    q_R[d] = 0.f; q_W[d] = 0; q_usum[d] = 0; q_rawm[d] = 0; q_band[d] = 0;
#pragma unroll
    for (int s = 0; s < SKS; ++s) Lq[s][d] = 0;
    if constexpr (SK) {
      if (d < D && dep[d].scaler == CCKA_SCALER_HPA && target[d] > 0) {
        const int tg = target[d];
        int ulo = max(0, (int)floor(dep[d].lo * (double)tg) - 2);
        while ((double)ulo / (double)tg < dep[d].lo) ++ulo;
        int uhi = (int)floor(dep[d].hi * (double)tg) + 2;
        while ((double)uhi / (double)tg > dep[d].hi) --uhi;
        q_band[d] = (uint32_t)ulo | (uint32_t)uhi << 16;
      }
    }
  }
  // per-step sums of the quiet steps [tq, tl) (SEMANTICS 3.H: integer sums, any order)
  auto sk_flush = [&]() {
    const int nq = tl - tq;
    if (nq > 0) {
      long long e = (long long)nq * q_sidle + q_corr;
#pragma unroll
      for (int d = 0; d < SKD; ++d) e += (long long)q_usum[d] * q_W[d];
      cost += (long long)nq * (burn + base_price);
      energy_nw += e;
      e_hour += e;
      pend_min += (long long)nq * q_pend;
      nmin_spot += nq * nsp;
      nmin_od += nq * nod;
      // the history rings: a quiet step pushed its proposal (cur) into the
      // decision records, or, where the proposal differs from cur, its raw
      // usage (q_rawm): converted here under the replica / ready counts the
      // quiet steps ran with (unchanged since the last full step); their zero
      // replica changes enter the change ring here, min(nq, 8) at once
      const int m = min(nq, CCKA_HIST);
#pragma unroll
      for (int d = 0; d < SKD; ++d) {
        if (d >= D || dep[d].scaler != CCKA_SCALER_HPA) continue;
        if (q_rawm[d]) {
#pragma unroll
          for (int k = 0; k < CCKA_HIST; ++k) {
            if (q_rawm[d] >> k & 1u) {
              int u;
              rec[d][k] = hpa_prop(rec[d][k], replicas[d], rpods[d], dep[d].req_cpu, target[d], dep[d].lo, dep[d].hi, u);
            }
          }
        }
#pragma unroll
        for (int b = 4; b >= 1; b >>= 1) {
          const bool sh = (m & b) != 0;
#pragma unroll
          for (int k = CCKA_HIST - 1; k >= 0; --k) delta[d][k] = sh ? (k >= b ? delta[d][k - (k >= b ? b : 0)] : 0) : delta[d][k];
        }
        if (m & 8) {
#pragma unroll
          for (int k = 0; k < CCKA_HIST; ++k) delta[d][k] = 0;
        }
      }
    }
    q_corr = 0;
#pragma unroll
    for (int d = 0; d < SKD; ++d) { q_usum[d] = 0; q_rawm[d] = 0; }
    tq = tl;
  };
  // exact dynamic energy of one step (SEMANTICS 3.H) for the given upp
  auto sk_dyn = [&](const uint32_t (&upp)[SKD]) -> long long {
    long long e = 0;
#pragma unroll
    for (int n = 0; n < MAXN; ++n) {
      if (!((used & rdy) >> n & 1u)) continue;
      const ccka_itype& ty = L.types[ni_type(ninfo[n])];
      long long use = 0;
#pragma unroll
      for (int d = 0; d < SKD; ++d) if (d < D) use += (long long)npods[n][d] * upp[d];
      e += ty.dyn_nw_per_m * min(use, (long long)ty.alloc_cpu_m);
    }
    return e;
  };
  // the quiet steps' caches after a full step at t (state final for the step)
  auto sk_caches = [&](int t, bool peak) {
    int pend = 0, reps = 0;
    const bool unplaced = g_dirty;
    q_ran = 0;
    q_atmax = 0;
    // the slots' type fields, read once and unconditionally (an unused slot
    // reads type 0 and contributes nothing): the LDS reads issue together
    long long sidle = base_nw;
    long long Wd[SKD];
    float Rd[SKD];
#pragma unroll
    for (int d = 0; d < SKD; ++d) { Wd[d] = 0; Rd[d] = 0.f; }
#pragma unroll
    for (int n = 0; n < MAXN; ++n) {
      const ccka_itype& ty = L.types[ni_type(ninfo[n])];
      const long long idle = ty.idle_nw, dyn = ty.dyn_nw_per_m;
      const int acpu = ty.alloc_cpu_m;
      const bool u = (used >> n & 1u) != 0, r = ((used & rdy) >> n & 1u) != 0;
      sidle += u ? idle : 0;
      const float ra = acpu > 0 ? __builtin_amdgcn_rcpf((float)acpu) : 1e30f;  // (a bound: the check keeps a margin)
#pragma unroll
      for (int d = 0; d < SKD; ++d) {
        const int k = d < D ? npods[n][d] : 0;
        Wd[d] += r ? dyn * (long long)k : 0;
        Rd[d] = r ? fmaxf(Rd[d], (float)k * ra) : Rd[d];
      }
    }
    q_sidle = sidle;
#pragma unroll
    for (int d = 0; d < SKD; ++d) {
      if (d >= D) continue;
      const Dep& dp = dep[d];
      const int cur = replicas[d], rd = rpods[d];
      pend += cur - rd;
      reps += cur;
      q_W[d] = Wd[d];
      q_R[d] = Rd[d];
      q_rcap[d] = dp.limit > 0 ? (int)min((long long)rd * dp.limit, (long long)UQ) : UQ;
      int ulim = UQ, pge = 0, slo_thr = UQ, hold = UQ;
      if (dp.scaler == CCKA_SCALER_HPA) {
        const int minr = dp.minr, mx = maxr[d], tg = target[d];
        const bool hpa_path = !(cur == 0 && minr != 0);
        if (hpa_path && (cur > mx || cur < minr)) {
          ulim = 0;  // the clamp moves the count: never quiet
        } else if (hpa_path && rd > 0) {
          q_ran |= 1u << d;
          q_atmax |= (cur >= mx ? 1u : 0u) << d;
          const int ulo = (int)(q_band[d] & 0xFFFFu), uhi = (int)(q_band[d] >> 16);
          // smallest usage with floor(100 usage / den) >= u (u >= 0)
          auto umin = [](long long u, long long den) -> int {
            return u <= 0 ? 0 : (int)min((u * den + 99) / 100, (long long)UQ);
          };
          const long long dreq = (long long)rd * dp.req_cpu;
          int lim;
          if (cur > rd) {
            // unready pods: util <= target proposes ceil(util * ready / target) < cur
            // below the band; util > target counts every replica (nu): keep iff nu <= uhi
            pge = umin(ulo, dreq);
            lim = max(umin((long long)tg + 1, dreq), umin((long long)uhi + 1, (long long)cur * dp.req_cpu));
            slo_thr = 0;
          } else {
            // below the band the proposal ceil(fl(fl(u / tg) * cur)) reaches cur
            // from the smallest u with u * cur > (cur - 1) * tg on (the binary64
            // rounding can move that only at an exact multiple, checked with the
            // spec's own arithmetic); monotone in u, capped at the band
            const uint32_t x = (uint32_t)(cur - 1) * (uint32_t)tg;  // < 2^31: cur, tg < 2^15
            int us = (int)(x / (uint32_t)cur) + 1;
            if (__builtin_expect((uint32_t)(us - 1) * (uint32_t)cur == x, 0) &&
                (int)ceil(((double)(us - 1) / (double)tg) * (double)cur) >= cur)
              --us;
            us = min(us, ulo);
            pge = umin(us, dreq);
            lim = umin((long long)uhi + 1, dreq);
            slo_thr = umin((long long)slo_util + 1, dreq);
          }
          ulim = cur >= mx ? UQ : lim;
          if (cur <= minr) {
            hold = UQ;  // a lower proposal cannot go below minReplicas = cur
          } else {
            // newest down-window record >= cur: held while it stays inside the window
            const int nw = __popc((uint32_t)dnmask[d]);
            hold = -0x40000000;
#pragma unroll
            for (int k = CCKA_HIST - 1; k >= 0; --k)
              if (k < nw && (recv[d] >> k & 1u) && rec[d][k] >= cur) hold = t - k + nw;
          }
        }
      }
      q_ulim[d] = ulim;
      q_pge[d] = pge;
      q_slo[d] = slo_thr;
      q_hold[d] = hold;
    }
    q_pend = pend;
    q_reps = reps;
    q_sloall = pend > 0;
    q_w0 = 0xFFFF | (int)((peak ? 1u : 0u) << 16);
    // first step that needs the full step again: a node becomes ready, the
    // next clock hour or peak-window boundary, a ready node that the
    // disruption gate admits becomes a consolidation candidate, or the next
    // step while the disruption phase has work (g_dirty). Pods left pending
    // by this step stay pending until one of these: the scheduler and
    // Karpenter (phases E, F1, F2) placed or claimed all they could this step,
    // and with the same nodes, prices and pools they do the same again.
    const int mn = minute;
    int nx = min(next_ready, t + 60 - mn % 60);
    if (pswitch) {
      const int dps = (ps - mn + 1439) % 1440 + 1, dpe = (pe - mn + 1439) % 1440 + 1;
      nx = min(nx, t + min(dps, dpe));
    }
    {
      // the gate of phase G (several deployments: a necessary condition for a
      // deletion): a candidate that is empty, or of a WhenEmptyOrUnderutilized
      // pool with its pods' CPU / memory / count within the free resources of
      // the other ready slots of the capacity types its deployments admit. A
      // candidate the gate rejects leaves the evaluation nothing to do (the
      // evaluation at any step is exact, skipping it only when it would act
      // on nothing), so only gate-admitted candidates wake the lane.
      auto node_use = [&](int n, int& c, int& m, int& pods) {
        c = 0; m = 0; pods = 0;
#pragma unroll
        for (int e = 0; e < SKD; ++e) {
          const int k = e < D ? npods[n][e] : 0;
          c += k * dep[e].req_cpu;
          m += k * dep[e].req_mem;
          pods += k;
        }
      };
      // per ready slot: its free CPU / memory / pod count (the type's allocatable
      // minus its pods' requests), summed by capacity type; branch-free, every
      // slot's type read unconditionally so that the LDS reads issue together
      int fcs[MAXN], fms[MAXN], fps[MAXN];
      int gwk = 0x7fffffff;
      int ac0 = 0, ac1 = 0, am0 = 0, am1 = 0, ap0 = 0, ap1 = 0;
#pragma unroll
      for (int n = 0; n < MAXN; ++n) {
        const ccka_itype& ty = L.types[ni_type(ninfo[n])];
        int c, m, pods;
        node_use(n, c, m, pods);
        const bool r = ((used & rdy) >> n & 1u) != 0, od = ni_cap(ninfo[n]) != 0;
        fcs[n] = ty.alloc_cpu_m - c;
        fms[n] = ty.alloc_mem_mi - m;
        fps[n] = ty.max_pods - pods;
        ac0 += (r && !od) ? fcs[n] : 0; ac1 += (r && od) ? fcs[n] : 0;
        am0 += (r && !od) ? fms[n] : 0; am1 += (r && od) ? fms[n] : 0;
        ap0 += (r && !od) ? fps[n] : 0; ap1 += (r && od) ? fps[n] : 0;
      }
#pragma unroll
      for (int n = 0; n < MAXN; ++n) {
        const uint32_t x = ninfo[n];
        int ca = 0, pol = 0;
#pragma unroll
        for (int q = 0; q < CCKA_MAX_POOLS; ++q)
          if (q == ni_pool(x)) { ca = pca[q]; pol = ppol[q]; }
        // a slot that is not yet a candidate (one already is: evaluated with this state)
        const int thr = max(nready[n], nlast[n] + (ca + CCKA_STEP_SECONDS - 1) / CCKA_STEP_SECONDS);
        int c, m, pods;
        node_use(n, c, m, pods);
        uint32_t cs = 0;
#pragma unroll
        for (int e = 0; e < SKD; ++e) cs |= (e < D && npods[n][e] > 0) ? capsel[e] : 0u;
        const bool s0 = (cs & capbit(0)) != 0, s1 = (cs & capbit(1)) != 0;
        int vc = (s0 ? ac0 : 0) + (s1 ? ac1 : 0), vm = (s0 ? am0 : 0) + (s1 ? am1 : 0);
        int vp = (s0 ? ap0 : 0) + (s1 ? ap1 : 0);
        const bool own = (cs & capbit(ni_cap(x))) != 0;  // not a receiver of its own pods
        vc -= own ? fcs[n] : 0;
        vm -= own ? fms[n] : 0;
        vp -= own ? fps[n] : 0;
        const bool pass = pods == 0 || (pol == CCKA_WHEN_EMPTY_OR_UNDERUTILIZED && c <= vc && m <= vm && pods <= vp);
        if (((used & rdy) >> n & 1u) && thr > t && pass) gwk = min(gwk, thr);
      }
      // the disruption phase's own wake (exact for the same reason): the next
      // full step evaluates it only when the gate may admit a candidate or
      // something it depends on moved (g_dirty)
      g_wake = gwk;
      nx = min(nx, gwk);
    }
    if (unplaced) nx = t + 1;
    if constexpr (kSKS) {
      bool unpl = false;
#pragma unroll
      for (int d = 0; d < SKD; ++d) unpl = unpl || (d < D && placed[d] != replicas[d]);
      // 1: pending pods (no longer a stall reason: counts full steps due to the rest while pods wait)
      sks_why = g_dirty ? 0 : nx == next_ready ? 3 : nx == t + 60 - mn % 60 ? 4 : unpl ? 1 : 2;
    }
    nxt = nx;
  };

  unsigned long long gst[11] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, glast = kGKS ? __builtin_amdgcn_s_memtime() : 0ull;
  for (int tt = t0;;) {
    int t = tt;
    bool stepl = active;  // this lane runs the full step of t in this pass
    if constexpr (SK) {
      const bool live = active && tl < t1;
      if (__ballot(live) == 0) break;
      t = tl;
      stepl = live && ev;
      // full steps every SK_K_V passes (more stalled lanes per run), or at once
      // when no live lane can step quietly
      if constexpr (SK_K_V > 1) {
        const bool due = (++skpass % SK_K_V) == 0 || __ballot(live && !ev) == 0;
        stepl = stepl && due;
      }
      GK_STAMP(7);  // SK: the quiet samples issued, loop top
      if constexpr (kSKS) {
        sks_c[6] += live ? 1 : 0;
        sks_c[7] += stepl ? 1 : 0;
        const unsigned long long bs = __ballot(stepl), bl = __ballot(live);
        const bool lead = lane == __ffsll((long long)bl) - 1;
        sks_c[9] += (lead && bs) ? 1 : 0;
        sks_c[10] += lead ? 1 : 0;
      }
    } else {
      if (tt >= t1) break;
    }
    if (!SK || __ballot(stepl) != 0) {
    const bool active = stepl;  // the rest of the step is this lane's only when it runs it
    if constexpr (SK) {
      if (active) {
        sk_flush();
        minute = (gw->start_minute + t) % 1440;
      }
    }
    if constexpr (POL != 0) {
      // ---- the learned policy chooses step t's HPA target and carbon weight ----
      pbf16x8 w1b0[MLP_IN / 16];  // W1's first row block, in flight under the features
#pragma unroll
      for (int s = 0; s < MLP_IN / 16; ++s) w1b0[s] = p.w1f[s * 64 + lane];
      uint32_t fw[32];
      feat_words(t, fw);
      if (p.feat_rec && active) store_feat(p.feat_rec + ((int64_t)t * p.N + i) * 64, fw);
      // X^T operands of the wave's two 32-state tiles (tile a: the states of
      // lanes 0..31, tile b: lanes 32..63; lane (r, h) holds features
      // 16s + 8h .. +7 of state r of the tile): one lane-half swap per word pair
      pbf16x8 xa[MLP_IN / 16], xb[MLP_IN / 16];
#pragma unroll
      for (int s = 0; s < MLP_IN / 16; ++s) {
        uint32_t wa[4], wb[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          wa[j] = fw[8 * s + j];
          wb[j] = fw[8 * s + 4 + j];
          pswap32(wa[j], wb[j]);
        }
        xa[s] = __builtin_bit_cast(pbf16x8, make_uint4(wa[0], wa[1], wa[2], wa[3]));
        xb[s] = __builtin_bit_cast(pbf16x8, make_uint4(wb[0], wb[1], wb[2], wb[3]));
      }
      const int hl = lane >> 5;
      GK_STAMP(7);  // features, X^T operands
      pf32x16 ya, yb;
      if (ablated(p.ablate, 32)) {  // profiling only: the loop without its MLP
#pragma unroll
        for (int k = 0; k < 16; ++k) ya[k] = yb[k] = 0.f;
      } else {
        ya = mlp_tile(xa, p.w1f, w1b0, s_w2, s_w3, s_mb, lane, hl);
        GK_STAMP(8);  // MLP tile a
        yb = mlp_tile(xb, p.w1f, w1b0, s_w2, s_w3, s_mb, lane, hl);
        GK_STAMP(9);  // MLP tile b
      }
      // this lane's state's 8 outputs
      float y[MLP_OUT] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k = 0; k < (POL == 1 ? 2 : 4); ++k) {  // the deterministic mapping reads y0, y1 only
        // lanes < 32 own state l of tile a: outputs k (own), 4 + k (lane l + 32);
        // lanes >= 32 own state l of tile b: outputs k (lane l - 32), 4 + k (own)
        const float oa = __shfl_xor(ya[k], 32), ob = __shfl_xor(yb[k], 32);
        y[k] = hl ? ob : ya[k];
        y[4 + k] = hl ? yb[k] : oa;
      }
      int tg;
      double c;
      if constexpr (POL == 1) {  // policy_act_kernel
        const float q0 = rintf(y[0] * 16.0f), q1 = rintf(y[1] * 16.0f);
        tg = 60 + (int)fminf(fmaxf(q0, -40.0f), 35.0f);
        c = (double)(int)fminf(fmaxf(q1, 0.0f), 64.0f) / 16.0;
      } else {  // policy_sample_kernel
        float pr[MLP_OUT];
        float mx = y[0];
#pragma unroll
        for (int a = 1; a < MLP_OUT; ++a) mx = fmaxf(mx, y[a]);
        float sum = 0.f;
#pragma unroll
        for (int a = 0; a < MLP_OUT; ++a) {
          pr[a] = expf(y[a] - mx);
          sum += pr[a];
        }
        const int64_t g = p.first_id + i;
        const uint64_t seed = *p.pol_seed;
        uint32_t u4[4];
        pol_philox((uint32_t)g, (uint32_t)(g >> 32), (uint32_t)t, 0x5A3B1E7u, (uint32_t)seed, (uint32_t)(seed >> 32), u4);
        const float u = (float)(u4[0] >> 8) * (1.0f / 16777216.0f) * sum;
        int act = MLP_OUT - 1;
        float acc = 0.f;
        bool found = false;
#pragma unroll
        for (int a = 0; a < MLP_OUT; ++a) {
          acc += pr[a];
          if (!found && u < acc) { act = a; found = true; }
        }
        tg = 40 + 10 * (act & 3);
        c = (double)(act >> 2);
        if (active) p.pol_act[(int64_t)t * p.N + i] = (uint8_t)act;
      }
      if (active) {
#pragma unroll
        for (int d = 0; d < DMAX; ++d)
          if (d < D && dep[d].scaler == CCKA_SCALER_HPA) target[d] = tg;
        wc1000 = c * 1000.0;
        pwi = (int)(c * 16.0);
        if (p.rec_target) {
          p.rec_target[(int64_t)t * p.N + i] = (int16_t)tg;
          p.rec_cw[(int64_t)t * p.N + i] = c;
        }
      }
    }
    GK_STAMP(10);  // the fused loop's action
    int Lcur[DMAX];
#pragma unroll
    for (int d = 0; d < DMAX; ++d) {
      if constexpr (SK) {  // this lane's step
        Lcur[d] = p.load_nt ? p.load_nt[(lcol * (int64_t)p.T + min(t, p.T - 1)) * DMAX + d]
                            : lptr[((int64_t)min(t, p.T - 1) * D + (d < D ? d : 0)) * lstride];
      } else {
        Lcur[d] = Lnext[d];
        // unconditional (clamped) load: lets the compiler count vmcnt exactly
        // instead of draining every outstanding store at the loop back-edge
        const int tn = t + 1 < p.T ? t + 1 : t;
        Lnext[d] = lptr[((int64_t)tn * D + (d < D ? d : 0)) * lstride];
      }
    }
    const int h = minute / 60;
    if (h != hour) {  // block-uniform: this hour's price tiles
      hour = h;
      if (SK || p.all_hours) {
        rlx = rl * 24 + h;
      } else {
        __syncthreads();
        for (int rr = 0; rr < p.span; ++rr) {
          const int rg = L.rmin + rr;
          if (rg >= p.R) break;
          const int* src = p.price + ((int64_t)rg * 24 + h) * tile_ints;
          for (int x = tid; x < tile_ints; x += blockDim.x) tile_base[rr * tile_ints + x] = src[x];
        }
        __syncthreads();
      }
      if (active) {
        // carbon of the hour that just ended
        if (t > 0) gco2 += (double)e_hour * (ci_gpwmin * 1e-9);
        e_hour = 0;
        if (det) {  // the same hourly charge per pool and for the base node group
          for (int q = 0; q < NP; ++q) {
            if (t > 0) det->d.pool_gco2[q] += (double)det->e_hour[q] * (ci_gpwmin * 1e-9);
            det->e_hour[q] = 0;
          }
          if (t > 0) det->d.base_gco2 += (double)det->base_e_hour * (ci_gpwmin * 1e-9);
          det->base_e_hour = 0;
        }
        ci_gpwmin = s_ci[(rl * 24 + h) * 2 + 0];
        ci_gpwh = s_ci[(rl * 24 + h) * 2 + 1];
        base_price = (long long)base_nodes * tprice(L, rlx, base_type, 0, 1);
        burn = 0;
        if (greplace) g_dirty = true;  // replacement offers depend on this hour's prices
#pragma unroll
        for (int n = 0; n < MAXN; ++n) {
          if (used >> n & 1u) {
            nprice[n] = tprice(L, rlx, ni_type(ninfo[n]), ni_zone(ninfo[n]), ni_cap(ninfo[n]));
            burn += nprice[n];
          }
        }
      }
    }
    uint32_t flags = 0;
    int step_last_type = 0xFFFF;
    int util_valid[DMAX], util[DMAX], pend[DMAX];
    bool kact_any[DMAX];
#pragma unroll
    for (int d = 0; d < DMAX; ++d) { util_valid[d] = 0; util[d] = 0; pend[d] = 0; kact_any[d] = false; }

    GK_STAMP(0);  // samples, the hour's tiles
    if (active) {
      // ---- B. readiness transitions (nominated pods start running) ----
      if (t >= next_ready) {
        next_ready = 0x7fffffff;
#pragma unroll
        for (int n = 0; n < MAXN; ++n) {
          if ((used & ~rdy) >> n & 1u) {
            if (nready[n] <= t) {
              rdy |= 1u << n;
#pragma unroll
              for (int d = 0; d < DMAX; ++d) rpods[d] += npods[n][d];
            } else {
              next_ready = min(next_ready, nready[n]);
            }
          }
        }
        g_dirty = true;
      }
      // ---- A. profile ----
      const bool in_win = ps <= pe ? (minute >= ps && minute < pe) : (minute >= ps || minute < pe);
      const bool peak = pswitch && in_win;
      const int prof = peak ? CCKA_PROFILE_PEAK : CCKA_PROFILE_OFFPEAK;
      if (peak) flags |= 1u;
      if (prof != profile) {
        profile = prof;
        g_dirty = true;
#pragma unroll
        for (int q = 0; q < CCKA_MAX_POOLS; ++q) {
          if (q >= NP) continue;
          auto& x = w->pools[q].profile[prof];
          if (x.policy != CCKA_POLICY_KEEP) ppol[q] = x.policy;
          if (x.consolidate_after_s >= 0) pca[q] = x.consolidate_after_s;
          if (x.zone_mask) pzm[q] = x.zone_mask;
          if (x.cap_mask) pcm[q] = x.cap_mask;
        }
      }
      GK_STAMP(1);  // readiness, profile
      // ---- C. scalers: nsub decisions on the step's metric sample ----
      for (int sub = 0; sub < (SK ? 1 : p.nsub); ++sub) {  // SK: one decision per step
      if (sub > 0) {
#pragma unroll
        for (int d = 0; d < DMAX; ++d) { util_valid[d] = 0; util[d] = 0; kact_any[d] = false; }
      }
#pragma unroll
      for (int d = 0; d < DMAX; ++d) {
        if (d >= D) continue;
        const Dep& dp = dep[d];
        const int Lv = Lcur[d];
        if (dp.scaler != CCKA_SCALER_HPA && dp.scaler != CCKA_SCALER_KEDA) continue;  // static / trigger
        if (SK && dp.scaler != CCKA_SCALER_HPA) continue;  // (SK worlds have none)
        const int ready = rpods[d];
        const int cur = replicas[d];
        int desired = cur, proposal = cur;
        bool ran = false, hpa_path = false;
        int minr = dp.minr, mx = maxr[d];
        bool do_behavior = false;
        if (dp.scaler == CCKA_SCALER_HPA) {
          hpa_path = true;
          if (cur == 0 && minr != 0) { hpa_path = false; }
          else if (cur > mx) desired = mx;
          else if (cur < minr) desired = minr;
          else if (ready > 0) {
            long long usage = Lv;
            if (dp.limit > 0) usage = min(usage, (long long)ready * dp.limit);
            int u;
            proposal = hpa_prop(usage, cur, ready, dp.req_cpu, target[d], dp.lo, dp.hi, u);
            util_valid[d] = 1;
            util[d] = u;
            do_behavior = true;
          }
        } else {  // KEDA: own trigger + the KEDA_TRIGGER entries right after d
          bool act = (long long)Lv > dp.kact;
          bool chain = true;
#pragma unroll
          for (int e = 0; e < DMAX; ++e) {
            if (e > d) {
              chain = chain && e < D && dep[e].scaler == CCKA_SCALER_KEDA_TRIGGER;
              if (chain) act |= (long long)Lcur[e] > dep[e].kact;
            }
          }
          kact_any[d] = act;
          if (act) last_active[d] = t;
          if (cur == 0) desired = act ? 1 : 0;
          else if (!act && dp.kmin == 0 && (t - last_active[d]) * CCKA_STEP_SECONDS >= dp.kcool)
            desired = 0;
          else {
            hpa_path = true;
            minr = max(dp.kmin, 1);
            mx = dp.kmax;
            if (cur > mx) desired = mx;
            else if (cur < minr) desired = minr;
            else {
              const double r = (double)Lv / ((double)dp.kthr * (double)cur);
              proposal = (dp.lo <= r && r <= dp.hi) ? cur : (int)ceil((double)Lv / (double)dp.kthr);
              bool ch = true;
#pragma unroll
              for (int e = 0; e < DMAX; ++e) {
                if (e > d) {
                  ch = ch && e < D && dep[e].scaler == CCKA_SCALER_KEDA_TRIGGER;
                  if (ch) {
                    const double re = (double)Lcur[e] / ((double)dep[e].kthr * (double)cur);
                    const int pe = (dp.lo <= re && re <= dp.hi) ? cur : (int)ceil((double)Lcur[e] / (double)dep[e].kthr);
                    proposal = max(proposal, pe);
                  }
                }
              }
              do_behavior = true;
            }
          }
        }
        if (do_behavior && !ablated(p.ablate, 8) && !SK && p.hlen) {
          ran = true;
          const ccka_deployment& gd = gw->deploy[d];
          const int dstab = p.down_stab && dp.scaler == CCKA_SCALER_HPA ? (int)p.down_stab[i] : gd.down.stab_window_s;
          desired = behavior_long(&gd.up, &gd.down, dstab, p.sync_s, cur, proposal, minr, mx, p.hist + (int64_t)d * p.N + i,
                                  hpos, p.hlen, (int64_t)D * p.N);
        } else if (do_behavior && !ablated(p.ablate, 8)) {
          ran = true;
          // stabilisation over the valid records inside each window
          const uint32_t upm = recv[d] & (uint32_t)dp.up.stab_mask;
          const uint32_t dnm = recv[d] & (uint32_t)dnmask[d];
          int upr = proposal, dnr = proposal;
#pragma unroll
          for (int k = 0; k < CCKA_HIST; ++k) {
            if (upm >> k & 1u) upr = min(upr, rec[d][k]);
            if (dnm >> k & 1u) dnr = max(dnr, rec[d][k]);
          }
          int rc = max(cur, upr);
          rc = min(rc, dnr);
          int lo = minr, hi = mx;
          if (rc > cur) hi = min(hi, max(rate_limit(dp.up, true, cur, delta[d]), cur));
          else if (rc < cur) lo = max(lo, min(rate_limit(dp.dn, false, cur, delta[d]), cur));
          desired = rc < lo ? lo : (rc > hi ? hi : rc);
        }
        if (!SK && p.hlen) {  // HBM history: this decision at hpos
          int2 e;
          e.x = ran ? proposal + 1 : 0;
          e.y = (hpa_path && desired != cur) ? desired - cur : 0;
          p.hist[((int64_t)hpos * D + d) * p.N + i] = e;
        } else {
          // shift history rings; entry 0 = this step
#pragma unroll
          for (int k = CCKA_HIST - 1; k > 0; --k) { rec[d][k] = rec[d][k - 1]; delta[d][k] = delta[d][k - 1]; }
          rec[d][0] = ran ? proposal : 0;
          recv[d] = ((recv[d] << 1) | (ran ? 1u : 0u)) & 0xFFu;
          delta[d][0] = (hpa_path && desired != cur) ? desired - cur : 0;
        }
        if (desired != cur) g_dirty = true;  // PDB expectation changed
        replicas[d] = desired;
      }
      if (!SK && p.hlen) hpos = hpos + 1 == p.hlen ? 0 : hpos + 1;
      }  // sub-steps
      GK_STAMP(2);  // scalers
      // ---- D. ReplicaSet reconcile (nominated first, then running; high slot first) ----
#pragma unroll
      for (int d = 0; d < DMAX; ++d) {
        if (d >= D) continue;
        int excess = placed[d] - replicas[d];
        if (excess > 0) {
          g_dirty = true;
          placed[d] = replicas[d];
#pragma unroll
          for (int pass = 0; pass < 2; ++pass) {
            const uint32_t m = pass == 0 ? (used & ~rdy) : rdy;
#pragma unroll
            for (int n = MAXN - 1; n >= 0; --n) {
              if ((m >> n & 1u) && npods[n][d] > 0 && excess > 0) {
                const int k = min(npods[n][d], excess);
                npods[n][d] -= k;
                excess -= k;
                nlast[n] = t;
                if (pass == 1) rpods[d] -= k;
              }
            }
          }
        }
      }
      // ---- E. kube-scheduler (ready) / F1. nomination (in-flight) ----
      // nodes tainted karpenter.sh/disrupted (a source whose pre-spun
      // replacement is in flight, and that replacement) take no other pods
      const uint32_t tnt = (greplace || gdrift || gmulti) ? taint_mask() : 0u;
      // (a 16-deployment body is too large to unroll: the loop stays rolled there)
      constexpr int kUnrollE = DMAX <= 4 ? DMAX : 1;
#pragma unroll kUnrollE
      for (int d = 0; d < DMAX; ++d) {
        if (d >= D) continue;
        int pd = replicas[d] - placed[d];
        if (pd > 0) {
#pragma unroll
          for (int pass = 0; pass < 2; ++pass) {
            const uint32_t m = (pass == 0 ? rdy : (used & ~rdy)) & ~tnt;
#pragma unroll
            for (int n = 0; n < MAXN; ++n) {
              const uint32_t x = ninfo[n];
              if (pd > 0 && (m >> n & 1u) && (capbit(ni_cap(x)) & capsel[d])) {
                int f;
                if (DMAX == 1) {
                  f = ncap[n] - npods[n][0];
                } else {
                  int sc = 0, sm = 0, sp = 0;
#pragma unroll
                  for (int e = 0; e < DMAX; ++e) {
                    if (e >= D) continue;
                    sc += npods[n][e] * dep[e].req_cpu;
                    sm += npods[n][e] * dep[e].req_mem;
                    sp += npods[n][e];
                  }
                  f = max(type_fit<DMAX>(L, ni_type(x), sc, sm, sp, dep[d].req_cpu, dep[d].req_mem), 0);
                }
                const int k = min(f, pd);
                if (k > 0) {
                  npods[n][d] += k;
                  pd -= k;
                  placed[d] += k;
                  nlast[n] = t;
                  // nominations onto not-ready nodes cannot validate a
                  // consolidation candidate before readiness (which dirties)
                  if (pass == 0) { rpods[d] += k; g_dirty = true; }
                }
              }
            }
          }
        }
        pend[d] = pd;
      }
    }

    GK_STAMP(3);  // reconcile, scheduler
    // ---- F2. Karpenter provisioning ----
    if (POL > 0 && p.ptable) {
      // the fused closed loop on a single-deployment world without pool limits:
      // claims of min(J, pending) pods in slot order from the first pool (in
      // Karpenter's order) whose capacity types the deployment admits and
      // whose J (largest pod count any offered type holds) is > 0, each launch
      // one read of the argmin table (table_kernel: region-hour, zone mask,
      // capacity mask, carbon weight, pods) -- the same choice as the
      // wave-cooperative scans below, lane-local (rollout_d1_kernel's F2)
      uint32_t fm = ~used & slot_mask;
      int pd = pend[0];
      if (active && pd > 0 && fm && !ablated(p.ablate, 2)) {
        const int rh = my_r * 24 + hour;
        int q = -1, J = 0, zi = 0;
        uint32_t cm = 0;
        for (int qq = 0; qq < NP && q < 0; ++qq) {
          const uint32_t c = pcm[qq] & capsel[0];
          const int z = c ? p.pzmi[pzm[qq] & 15] : -1;
          const int j = z >= 0 ? p.pjtab[(rh * p.pNZI + z) * 3 + (int)(c - 1)] : 0;
          if (j > 0) { q = qq; J = j; cm = c; zi = z; }
        }
        if (q >= 0) {
          const int2* row = p.ptable + ((((int64_t)rh * p.pNZI + zi) * 3 + (cm - 1)) * p.pNW + pwi) * p.pJT;
          while (pd > 0 && fm) {
            const int slot = __ffs((int)fm) - 1;
            fm &= fm - 1;
            const int k = min(J, pd);
            const int2 e = row[k];  // never empty: k <= J
            const int price = e.x, bk = e.y & 1023, bz = e.y >> 10 & 3, bc = e.y >> 12 & 1, cap = e.y >> 16;
            const bool now_ready = delay == 0;
#pragma unroll
            for (int n = 0; n < MAXN; ++n) {
              if (n == slot) {
                ninfo[n] = ni_make(q, bk, bz, bc);
                nready[n] = t + delay;
                nlast[n] = t;
                nprice[n] = price;
                ncap[n] = cap;
                npods[n][0] = k;
              }
            }
            placed[0] += k;
            if (now_ready) rpods[0] += k;
            used |= 1u << slot;
            if (now_ready) rdy |= 1u << slot;
            else next_ready = min(next_ready, t + delay);
#pragma unroll
            for (int qq = 0; qq < CCKA_MAX_POOLS; ++qq)
              if (qq == q) puse[qq] += L.types[bk].vcpu * 1000;
            if (bc == 0) nsp++; else nod++;
            burn += price;
            launches++;
            if (det) det->d.pool_launches[q]++;
            last_choice = (uint32_t)bk | (uint32_t)bz << 12 | (uint32_t)bc << 14 | (uint32_t)q << 16;
            hash = (hash ^ last_choice) * 16777619u;
            step_last_type = bk;
            flags |= 2u;
            if (now_ready) g_dirty = true;
            pd -= k;
          }
        }
      }
    } else if (SK && SK_LANE_F2 && p.lds_lclaims >= 0) {
      // lane-local F2 (variant builds, SK_LANE_F2; measured 1-4 % slower than the
      // cooperative scans on 2 / 4 deployments x 8 / 16 slots): every
      // lane that needs NodeClaims builds and launches them itself, by the
      // cooperative path's rules in the same order (claims of this step in
      // creation order, the first admitting pool with j > 0, the launch argmin
      // over (score, type, zone, capacity type) in index order), so the lanes
      // of a run provision in parallel instead of one after another; each
      // lane's claims in its own LDS column [claim][field][lane]
      int anyp = 0;
#pragma unroll
      for (int d = 0; d < DMAX; ++d) anyp |= pend[d] > 0;
      const uint32_t free_mask = ~used & slot_mask;
      if (active && anyp && free_mask != 0) {
        if constexpr (kSKS) sks_c[11]++;
        uint32_t lfree = free_mask;
        int use0[CCKA_MAX_POOLS], usenow[CCKA_MAX_POOLS];
#pragma unroll
        for (int q = 0; q < CCKA_MAX_POOLS; ++q) { use0[q] = puse[q]; usenow[q] = puse[q]; }
        auto mem_now = [&](int q) { return w->pools[q].limit_mem_mi >= 0 ? pool_mem(q) : 0; };
        constexpr int CW = CLAIM_FIXED + DMAX;
        int* const CLb = reinterpret_cast<int*>(smem + p.lds_lclaims);
        const int nthr = (int)blockDim.x;
        auto CLA = [&](int c, int f) -> int& { return CLb[(c * CW + f) * nthr + tid]; };
        // j: most pods of the deployment any candidate type holds on top of the sums
        auto claim_j = [&](uint32_t zm, uint32_t cm, int s_cpu, int s_mem, int s_pods, int rc, int rm, int use, int limit,
                           int usem, int limitm) {
          int best = 0;
          for (int k = 0; k < L.K; ++k) {
            if (!limit_ok(L, k, use, limit, usem, limitm)) continue;
            const int f = type_fit<DMAX>(L, k, s_cpu, s_mem, s_pods, rc, rm);
            if (f <= best) continue;
            if (!type_offered(L, rlx, k, zm, cm)) continue;
            best = f;
          }
          return best;
        };
        int ncl = 0;
        for (int oi = 0; oi < D; ++oi) {
          const int d = p.prov[oi];
          int rem = 0, rc = 0, rm = 0;
          uint32_t csel = 0;
#pragma unroll
          for (int e = 0; e < DMAX; ++e)
            if (e == d) { rem = pend[e]; csel = capsel[e]; rc = dep[e].req_cpu; rm = dep[e].req_mem; }
          if (rem <= 0) continue;
          for (int c = 0; c < ncl && rem > 0; ++c) {
            const int cpool = CLA(c, 0);
            const uint32_t cm = (uint32_t)CLA(c, 1) & csel;
            if (!cm) continue;
            int climit = 0;
#pragma unroll
            for (int q = 0; q < CCKA_MAX_POOLS; ++q) if (q == cpool) climit = plimit[q];
            int u0 = 0;
#pragma unroll
            for (int q = 0; q < CCKA_MAX_POOLS; ++q) if (q == cpool) u0 = use0[q];
            const int j = claim_j((uint32_t)CLA(c, 2), cm, CLA(c, 4), CLA(c, 5), CLA(c, 6), rc, rm, u0, climit,
                                  mem_now(cpool), w->pools[cpool].limit_mem_mi);
            if (j <= 0) continue;
            const int k = min(j, rem);
            CLA(c, 1) = (int)cm;
            CLA(c, 4) += k * rc;
            CLA(c, 5) += k * rm;
            CLA(c, 6) += k;
            CLA(c, CLAIM_FIXED + d) += k;
            rem -= k;
          }
          while (rem > 0 && lfree) {
            const int slot = __ffs((int)lfree) - 1;
            int chosen = -1, jj = 0;
            uint32_t czm = 0, ccm = 0;
            for (int q = 0; q < NP && chosen < 0; ++q) {
              uint32_t zq = 0, cq = 0;
              int u0 = 0, lq = 0;
#pragma unroll
              for (int qq = 0; qq < CCKA_MAX_POOLS; ++qq)
                if (qq == q) { zq = pzm[qq]; cq = pcm[qq]; u0 = use0[qq]; lq = plimit[qq]; }
              const uint32_t cm = cq & csel;
              if (!cm) continue;
              const int j = claim_j(zq, cm, 0, 0, 0, rc, rm, u0, lq, mem_now(q), w->pools[q].limit_mem_mi);
              if (j > 0) { chosen = q; jj = j; czm = zq; ccm = cm; }
            }
            if (chosen < 0) break;
            const int k = min(jj, rem);
            CLA(ncl, 0) = chosen;
            CLA(ncl, 1) = (int)ccm;
            CLA(ncl, 2) = (int)czm;
            CLA(ncl, 3) = slot;
            CLA(ncl, 4) = k * rc;
            CLA(ncl, 5) = k * rm;
            CLA(ncl, 6) = k;
#pragma unroll
            for (int e = 0; e < DMAX; ++e) CLA(ncl, CLAIM_FIXED + e) = e == d ? k : 0;
            ncl++;
            lfree &= ~(1u << slot);
            rem -= k;
          }
        }
        // launch in creation order (wave_launch's rule, lane-local)
        for (int c = 0; c < ncl; ++c) {
          const int cpool = CLA(c, 0);
          const uint32_t zm = (uint32_t)CLA(c, 2), cm = (uint32_t)CLA(c, 1);
          const int s_cpu = CLA(c, 4), s_mem = CLA(c, 5), s_pods = CLA(c, 6);
          int climit = 0, unow = 0;
#pragma unroll
          for (int q = 0; q < CCKA_MAX_POOLS; ++q) if (q == cpool) { climit = plimit[q]; unow = usenow[q]; }
          const int usem = mem_now(cpool), limitm = w->pools[cpool].limit_mem_mi;
          bool spot_only = false;
          if (cm & CCKA_CAP_SPOT) {
            for (int k = 0; k < L.K && !spot_only; ++k) {
              if (!type_holds<DMAX>(L, k, s_cpu, s_mem, s_pods) || !limit_ok(L, k, unow, climit, usem, limitm)) continue;
              for (int z = 0; z < L.Z; ++z)
                if ((zm >> z & 1u) && tprice(L, rlx, k, z, 0) > 0) { spot_only = true; break; }
            }
          }
          double bs = __builtin_inf();
          int bi = 0x7fffffff;
          for (int k = 0; k < L.K; ++k) {
            if (!type_holds<DMAX>(L, k, s_cpu, s_mem, s_pods) || !limit_ok(L, k, unow, climit, usem, limitm)) continue;
            const double carbon = L.types[k].p_ref_w * ci_gpwh;
            for (int z = 0; z < L.Z; ++z) {
              if (!(zm >> z & 1u)) continue;
              for (int cc = 0; cc < 2; ++cc) {
                if (!(cm & (uint32_t)capbit(cc))) continue;
                if (spot_only && cc != 0) continue;
                const int pr = tprice(L, rlx, k, z, cc);
                if (pr <= 0) continue;
                const double score = (double)pr + wc1000 * carbon;
                if (score < bs) { bs = score; bi = (k * L.Z + z) * 2 + cc; }
              }
            }
          }
          if (bi == 0x7fffffff) continue;
          const int bc = bi & 1, bz = (bi >> 1) % Z, bk = (bi >> 1) / Z;
          const int vcpu_m = L.types[bk].vcpu * 1000;
#pragma unroll
          for (int q = 0; q < CCKA_MAX_POOLS; ++q) if (q == cpool) usenow[q] += vcpu_m;
          const int slot = CLA(c, 3);
          const uint32_t choice = (uint32_t)bk | (uint32_t)bz << 12 | (uint32_t)bc << 14 | (uint32_t)cpool << 16;
          const bool now_ready = delay == 0;
          const int price = tprice(L, rlx, bk, bz, bc);
          const int cap = DMAX == 1 ? L.cap1[bk] : 0;
#pragma unroll
          for (int n = 0; n < MAXN; ++n) {
            if (n == slot) {
              ninfo[n] = ni_make(cpool, bk, bz, bc);
              nready[n] = t + delay;
              nlast[n] = t;
              nprice[n] = price;
              ncap[n] = cap;
#pragma unroll
              for (int e = 0; e < DMAX; ++e) {
                const int k = e < D ? CLA(c, CLAIM_FIXED + e) : 0;
                npods[n][e] = k;
                placed[e] += k;
                if (now_ready) rpods[e] += k;
              }
            }
          }
          used |= 1u << slot;
          if (now_ready) rdy |= 1u << slot;
          else next_ready = min(next_ready, t + delay);
#pragma unroll
          for (int q = 0; q < CCKA_MAX_POOLS; ++q)
            if (q == cpool) puse[q] += vcpu_m;
          if (bc == 0) nsp++; else nod++;
          burn += price;
          launches++;
          last_choice = choice;
          hash = (hash ^ choice) * 16777619u;
          step_last_type = bk;
          flags |= 2u;
          if (now_ready) g_dirty = true;
        }
      }
    } else {
      int anyp = 0;
#pragma unroll
      for (int d = 0; d < DMAX; ++d) anyp |= pend[d] > 0;
      const uint32_t free_mask = ~used & slot_mask;
      unsigned long long need = __ballot(active && anyp && free_mask != 0 && !ablated(p.ablate, 2));
      while (need) {
        const int ld = __ffsll((long long)need) - 1;
        if constexpr (kSKS) sks_c[11] += lane == ld ? 1 : 0;
        need &= need - 1;
        // broadcast the leader's state
        const int lrl = rdl(rlx, ld);
        const double lwc = rdld(wc1000, ld);
        const double lci = rdld(ci_gpwh, ld);
        uint32_t lfree = rdlu(free_mask, ld);
        int use0[CCKA_MAX_POOLS], usenow[CCKA_MAX_POOLS];
        // pool memory in use (limits.memory only): lane ld's slots, launches of
        // this step included (they update its slots as they happen)
        auto mem_now = [&](int q) { return w->pools[q].limit_mem_mi >= 0 ? rdl(pool_mem(q), ld) : 0; };
        uint32_t lzm[CCKA_MAX_POOLS], lcm[CCKA_MAX_POOLS];
#pragma unroll
        for (int q = 0; q < CCKA_MAX_POOLS; ++q) {
          use0[q] = rdl(puse[q], ld);
          usenow[q] = use0[q];
          lzm[q] = rdlu(pzm[q], ld);
          lcm[q] = rdlu(pcm[q], ld);
        }
        int* CL = L.claims;
        const int CW = CLAIM_FIXED + DMAX;
        int ncl = 0;
        for (int oi = 0; oi < D; ++oi) {
          const int d = p.prov[oi];
          int pd_self = 0, rc = 0, rm = 0;
          uint32_t csel_self = 0;
#pragma unroll
          for (int e = 0; e < DMAX; ++e)
            if (e == d) { pd_self = pend[e]; csel_self = capsel[e]; rc = dep[e].req_cpu; rm = dep[e].req_mem; }
          int rem = rdl(pd_self, ld);
          if (rem <= 0) continue;
          const uint32_t csel = rdlu(csel_self, ld);
          for (int c = 0; c < ncl && rem > 0; ++c) {
            int* cl = CL + c * CW;
            const int cpool = cl[0];
            const uint32_t cm = (uint32_t)cl[1] & csel;
            if (!cm) continue;
            int climit = 0;
#pragma unroll
            for (int q = 0; q < CCKA_MAX_POOLS; ++q) if (q == cpool) climit = plimit[q];
            const int j = wave_claim_j<DMAX>(L, lrl, (uint32_t)cl[2], cm, cl[4], cl[5], cl[6], rc, rm,
                                             use0[cpool], climit, mem_now(cpool), w->pools[cpool].limit_mem_mi, lane);
            if (j <= 0) continue;
            const int k = min(j, rem);
            __builtin_amdgcn_wave_barrier();
            cl[1] = (int)cm;
            cl[4] += k * rc;
            cl[5] += k * rm;
            cl[6] += k;
            cl[CLAIM_FIXED + d] += k;
            __builtin_amdgcn_wave_barrier();
            rem -= k;
          }
          while (rem > 0 && lfree) {
            const int slot = __ffs((int)lfree) - 1;
            int chosen = -1, jj = 0;
            for (int q = 0; q < NP; ++q) {
              const uint32_t cm = lcm[q] & csel;
              if (!cm) continue;
              const int j = wave_claim_j<DMAX>(L, lrl, lzm[q], cm, 0, 0, 0, rc, rm, use0[q], plimit[q], mem_now(q),
                                               w->pools[q].limit_mem_mi, lane);
              if (j > 0) { chosen = q; jj = j; break; }
            }
            if (chosen < 0) break;
            const int k = min(jj, rem);
            int* cl = CL + ncl * CW;
            __builtin_amdgcn_wave_barrier();
            cl[0] = chosen;
            cl[1] = (int)(lcm[chosen] & csel);
            cl[2] = (int)lzm[chosen];
            cl[3] = slot;
            cl[4] = k * rc;
            cl[5] = k * rm;
            cl[6] = k;
            for (int e = 0; e < DMAX; ++e) cl[CLAIM_FIXED + e] = e == d ? k : 0;
            __builtin_amdgcn_wave_barrier();
            ncl++;
            lfree &= ~(1u << slot);
            rem -= k;
          }
        }
        // launch in creation order
        for (int c = 0; c < ncl; ++c) {
          const int* cl = CL + c * CW;
          const int cpool = cl[0];
          int climit = 0;
#pragma unroll
          for (int q = 0; q < CCKA_MAX_POOLS; ++q) if (q == cpool) climit = plimit[q];
          const int bi = wave_launch<DMAX>(L, lrl, (uint32_t)cl[2], (uint32_t)cl[1], cl[4], cl[5],
                                           cl[6], usenow[cpool], climit, mem_now(cpool), w->pools[cpool].limit_mem_mi,
                                           lwc, lci, lane);
          if (bi < 0) continue;
          const int bc = bi & 1, bz = (bi >> 1) % Z, bk = (bi >> 1) / Z;
          const int vcpu_m = L.types[bk].vcpu * 1000;
          usenow[cpool] += vcpu_m;
          const int slot = cl[3];
          if (lane == ld) {
            const uint32_t choice = (uint32_t)bk | (uint32_t)bz << 12 | (uint32_t)bc << 14 | (uint32_t)cpool << 16;
            const bool now_ready = t + delay <= t;
            const int price = tprice(L, lrl, bk, bz, bc);
            const int cap = DMAX == 1 ? L.cap1[bk] : 0;
#pragma unroll
            for (int n = 0; n < MAXN; ++n) {
              if (n == slot) {
                ninfo[n] = ni_make(cpool, bk, bz, bc);
                nready[n] = t + delay;
                nlast[n] = t;
                nprice[n] = price;
                ncap[n] = cap;
#pragma unroll
                for (int e = 0; e < DMAX; ++e) {
                  const int k = e < D ? cl[CLAIM_FIXED + e] : 0;
                  npods[n][e] = k;
                  placed[e] += k;
                  if (now_ready) rpods[e] += k;
                }
              }
            }
            used |= 1u << slot;
            if (now_ready) rdy |= 1u << slot;
            else next_ready = min(next_ready, t + delay);
#pragma unroll
            for (int q = 0; q < CCKA_MAX_POOLS; ++q)
              if (q == cpool) puse[q] += vcpu_m;
            if (bc == 0) nsp++; else nod++;
            burn += price;
            launches++;
            if (det) det->d.pool_launches[cpool]++;
            last_choice = choice;
            hash = (hash ^ choice) * 16777619u;
            step_last_type = bk;
            flags |= 2u;
            if (now_ready) g_dirty = true;
          }
        }
        __builtin_amdgcn_wave_barrier();
      }
    }

    GK_STAMP(4);  // provisioning
    if (active) {
      // ---- G. disruption (skipped exactly when nothing it depends on moved) ----
      const bool g_eval = (g_dirty || t >= g_wake) && !ablated(p.ablate, 1);
      // One deployment without drift / replacement / multi-node consolidation:
      // an exact gate first (the single-deployment kernel's). The phase acts
      // only on a ready candidate past its consolidateAfter that is empty, or
      // of a WhenEmptyOrUnderutilized pool with its pods fitting the other
      // compatible ready slots (their free capacity F minus its own >= its
      // pods; the budget and the PDB only restrict further); with none, the
      // evaluation would change nothing, so only the next wake step is kept.
      bool g_gate = true;
      // several deployments: the gate's free-resource sums by capacity type
      // (valid for the search below until its first deletion)
      bool gsum = false;
      int ac0 = 0, ac1 = 0, am0 = 0, am1 = 0, ap0 = 0, ap1 = 0;
      if constexpr (DMAX == 1) {
        if (g_eval && !gdrift && !greplace && !gmulti) {
          int F = 0;
          uint32_t cm1 = 0, el = 0;
#pragma unroll
          for (int n = 0; n < MAXN; ++n) {
            const uint32_t x = ninfo[n];
            const bool r = (used & rdy) >> n & 1u;
            const bool c = r && (capbit(ni_cap(x)) & capsel[0]);
            cm1 |= (c ? 1u : 0u) << n;
            F += c ? ncap[n] - npods[n][0] : 0;
            int ca = 0, pol = 0;
#pragma unroll
            for (int q = 0; q < CCKA_MAX_POOLS; ++q)
              if (q == ni_pool(x)) { ca = pca[q]; pol = ppol[q]; }
            const bool cand = r && (t - nlast[n]) * CCKA_STEP_SECONDS >= ca &&
                              (npods[n][0] == 0 || pol == CCKA_WHEN_EMPTY_OR_UNDERUTILIZED);
            el |= (cand ? 1u : 0u) << n;
          }
          bool any = false;
#pragma unroll
          for (int n = 0; n < MAXN; ++n) {
            const int pods = npods[n][0];
            const int fo = F - ((cm1 >> n & 1u) ? ncap[n] - pods : 0);
            any |= (el >> n & 1u) && (pods == 0 || fo >= pods);
          }
          g_gate = any;
        }
      } else {
        // Several deployments (same cases): a necessary condition for a
        // deletion. A non-empty candidate's pods move onto ready nodes of a
        // capacity type one of its deployments admits, so their CPU, memory and
        // pod count must fit those nodes' free resources (the candidate's own
        // excluded); with no candidate that is empty or passes these sums, the
        // sequential search would reject every one.
        if (g_eval && !gdrift && !greplace && !gmulti) {
          auto node_use = [&](int n, int& c, int& m, int& pods) {
            c = 0; m = 0; pods = 0;
#pragma unroll
            for (int e = 0; e < DMAX; ++e) {
              const int k = e < D ? npods[n][e] : 0;
              c += k * dep[e].req_cpu;
              m += k * dep[e].req_mem;
              pods += k;
            }
          };
          gsum = true;  // free resources by capacity type
#pragma unroll
          for (int n = 0; n < MAXN; ++n) {
            if (!(rdy >> n & 1u)) continue;
            int c, m, pods;
            node_use(n, c, m, pods);
            const ccka_itype& ty = L.types[ni_type(ninfo[n])];
            const bool od = ni_cap(ninfo[n]) != 0;
            const int fc = ty.alloc_cpu_m - c, fmm = ty.alloc_mem_mi - m, fp = ty.max_pods - pods;
            ac0 += od ? 0 : fc; ac1 += od ? fc : 0;
            am0 += od ? 0 : fmm; am1 += od ? fmm : 0;
            ap0 += od ? 0 : fp; ap1 += od ? fp : 0;
          }
          bool any = false;
#pragma unroll
          for (int n = 0; n < MAXN; ++n) {
            if (!(rdy >> n & 1u)) continue;
            const uint32_t x = ninfo[n];
            int ca = 0, pol = 0;
#pragma unroll
            for (int q = 0; q < CCKA_MAX_POOLS; ++q)
              if (q == ni_pool(x)) { ca = pca[q]; pol = ppol[q]; }
            if ((t - nlast[n]) * CCKA_STEP_SECONDS < ca) continue;
            int c, m, pods;
            node_use(n, c, m, pods);
            if (pods == 0) { any = true; continue; }
            if (pol != CCKA_WHEN_EMPTY_OR_UNDERUTILIZED) continue;
            uint32_t cs = 0;  // capacity types some deployment with pods here admits
#pragma unroll
            for (int e = 0; e < DMAX; ++e) cs |= (e < D && npods[n][e] > 0) ? capsel[e] : 0u;
            const bool s0 = (cs & capbit(0)) != 0, s1 = (cs & capbit(1)) != 0;
            int vc = (s0 ? ac0 : 0) + (s1 ? ac1 : 0), vm = (s0 ? am0 : 0) + (s1 ? am1 : 0);
            int vp = (s0 ? ap0 : 0) + (s1 ? ap1 : 0);
            if (cs & capbit(ni_cap(x))) {  // not a receiver of its own pods
              const ccka_itype& ty = L.types[ni_type(x)];
              vc -= ty.alloc_cpu_m - c;
              vm -= ty.alloc_mem_mi - m;
              vp -= ty.max_pods - pods;
            }
            any |= c <= vc && m <= vm && pods <= vp;
          }
          g_gate = any;
        }
      }
      if (g_eval && !g_gate) g_dirty = false;
      if (g_eval && g_gate) {
        bool budget_hit = false, any_deleted = false;
        long long allowed = 0x3fffffffffffffffLL;
        if (pdb_pct >= 0) {
          long long rdyp = 0, reps = 0;
#pragma unroll
          for (int d = 0; d < DMAX; ++d) {
            if (d >= D || !dep[d].pdb) continue;
            reps += replicas[d];
            rdyp += rpods[d];
          }
          allowed = max(rdyp - ((long long)pdb_pct * reps + 99) / 100, 0LL);
        }
        // a freed slot's pending replacement becomes an ordinary node
        auto unlink = [&](int b) {
#pragma unroll
          for (int m = 0; m < MAXN; ++m) nsrc[m] &= ~(1u << b);
        };
        auto free_slot = [&](int b) {
#pragma unroll
          for (int n = 0; n < MAXN; ++n) {
            if (n == b) {
              if (ni_cap(ninfo[n]) == 0) nsp--; else nod--;
#pragma unroll
              for (int qq = 0; qq < CCKA_MAX_POOLS; ++qq)
                if (qq == ni_pool(ninfo[n])) puse[qq] -= L.types[ni_type(ninfo[n])].vcpu * 1000;
              burn -= nprice[n];
              ninfo[n] = 0; nready[n] = 0; nlast[n] = 0; nprice[n] = 0; ncap[n] = 0; nsrc[n] = 0;
#pragma unroll
              for (int d = 0; d < DMAX; ++d) npods[n][d] = 0;
            }
          }
          used &= ~(1u << b);
          rdy &= ~(1u << b);
          unlink(b);
        };
        // cheapest single offering (price, k, z, c) that holds the sums under a
        // pool's zone / capacity-type masks and CPU limit
        auto find_offer = [&](uint32_t zm, uint32_t cm, int use, int limit, int usem, int limitm, int s_cpu, int s_mem,
                              int s_pods, int& bk, int& bz, int& bc, int& bpr) {
          bk = -1; bz = 0; bc = 0; bpr = 0;
          for (int k = 0; k < L.K; ++k) {
            if (type_fit<DMAX>(L, k, s_cpu, s_mem, s_pods, 0, 0) < 0) continue;
            if (!limit_ok(L, k, use, limit, usem, limitm)) continue;
            for (int z = 0; z < L.Z; ++z) {
              if (!(zm >> z & 1u)) continue;
#pragma unroll
              for (int c = 0; c < 2; ++c) {
                if (!(cm & capbit(c))) continue;
                const int pr = tprice(L, rlx, k, z, c);
                if (pr > 0 && (bk < 0 || pr < bpr)) { bk = k; bz = z; bc = c; bpr = pr; }
              }
            }
          }
        };
        // the F2 launch rule for one NodeClaim, per lane (SEMANTICS 3.F): spot
        // offerings only when spot is allowed and any is feasible; argmin of
        // (score, k, z, c), score = price + carbon weight * 1000 * p_ref_w * ci
        auto lane_launch = [&](uint32_t zm, uint32_t cm, int use, int limit, int usem, int limitm, int s_cpu,
                               int s_mem, int s_pods, int& bk, int& bz, int& bc, int& bpr) {
          bk = -1; bz = 0; bc = 0; bpr = 0;
          bool spot_only = false;
          if (cm & CCKA_CAP_SPOT) {
            for (int k = 0; k < L.K && !spot_only; ++k) {
              if (type_fit<DMAX>(L, k, s_cpu, s_mem, s_pods, 0, 0) < 0) continue;
              if (!limit_ok(L, k, use, limit, usem, limitm)) continue;
              for (int z = 0; z < L.Z; ++z)
                if ((zm >> z & 1u) && tprice(L, rlx, k, z, 0) > 0) { spot_only = true; break; }
            }
          }
          double bs = 0.0;
          for (int k = 0; k < L.K; ++k) {
            if (type_fit<DMAX>(L, k, s_cpu, s_mem, s_pods, 0, 0) < 0) continue;
            if (!limit_ok(L, k, use, limit, usem, limitm)) continue;
            const double carbon = L.types[k].p_ref_w * ci_gpwh;
            for (int z = 0; z < L.Z; ++z) {
              if (!(zm >> z & 1u)) continue;
#pragma unroll
              for (int c = 0; c < 2; ++c) {
                if (!(cm & capbit(c)) || (spot_only && c != 0)) continue;
                const int pr = tprice(L, rlx, k, z, c);
                if (pr <= 0) continue;
                const double score = (double)pr + wc1000 * carbon;
                if (bk < 0 || score < bs) { bk = k; bz = z; bc = c; bpr = pr; bs = score; }
              }
            }
          }
        };
        // a pre-spun replacement node for the slots in `srcm` (no pods until it takes over)
        auto launch_replacement = [&](int q, int slot, uint32_t srcm, int bk, int bz, int bc, int bpr) {
          const bool now_ready = delay == 0;
#pragma unroll
          for (int n = 0; n < MAXN; ++n) {
            if (n == slot) {
              ninfo[n] = ni_make(q, bk, bz, bc);
              nready[n] = t + delay;
              nlast[n] = t;
              nprice[n] = bpr;
              ncap[n] = DMAX == 1 ? L.cap1[bk] : 0;
              nsrc[n] = srcm;
#pragma unroll
              for (int e = 0; e < DMAX; ++e) npods[n][e] = 0;
            }
          }
          used |= 1u << slot;
          if (now_ready) rdy |= 1u << slot;
          else next_ready = min(next_ready, t + delay);
#pragma unroll
          for (int qq = 0; qq < CCKA_MAX_POOLS; ++qq)
            if (qq == q) puse[qq] += L.types[bk].vcpu * 1000;
          if (bc == 0) nsp++; else nod++;
          burn += bpr;
          launches++;
          if (det) det->d.pool_launches[q]++;
          last_choice = (uint32_t)bk | (uint32_t)bz << 12 | (uint32_t)bc << 14 | (uint32_t)q << 16;
          hash = (hash ^ last_choice) * 16777619u;
          step_last_type = bk;
          flags |= 2u | 32u;
        };
        // ---- G2. single-node replacement consolidation (SEMANTICS 3.G2): the
        // first candidate in (pods asc, price desc, slot asc) order that is
        // on-demand, has pods, is not being replaced and has a strictly cheaper
        // single offering gets a pre-spun replacement; one per pool per step
        auto try_replace = [&](int q, int qca, int budget, int& deleted) {
          uint32_t srcm = 0, pq = 0;
#pragma unroll
          for (int n = 0; n < MAXN; ++n) {
            srcm |= nsrc[n];
            pq |= (ni_pool(ninfo[n]) == q && ni_cap(ninfo[n]) == 1 ? 1u : 0u) << n;
          }
          uint32_t cand = rdy & pq & ~srcm;
          while (deleted < budget) {
            int best = -1, bpods = 0, bprice = 0;
#pragma unroll
            for (int n = 0; n < MAXN; ++n) {
              if (!(cand >> n & 1u)) continue;
              if ((t - nlast[n]) * CCKA_STEP_SECONDS < qca) continue;
              int pods = 0;
#pragma unroll
              for (int d = 0; d < DMAX; ++d) pods += d < D ? npods[n][d] : 0;
              if (pods == 0) continue;
              const int pr = nprice[n];
              if (best < 0 || pods < bpods || (pods == bpods && pr > bprice)) { best = n; bpods = pods; bprice = pr; }
            }
            if (best < 0) break;
            const uint32_t fr = ~used & slot_mask;
            if (!fr) break;
            const int slot = __builtin_ctz(fr);
            long long pdb_pods = 0;
            int s_cpu = 0, s_mem = 0, s_pods = 0;
            uint32_t cm = 0, zm = 0;
            int use = 0, limit = 0, usem = 0;
            const int limitm = w->pools[q].limit_mem_mi;
            if (limitm >= 0) usem = pool_mem(q);
#pragma unroll
            for (int qq = 0; qq < CCKA_MAX_POOLS; ++qq)
              if (qq == q) { cm = pcm[qq]; zm = pzm[qq]; use = puse[qq]; limit = plimit[qq]; }
#pragma unroll
            for (int d = 0; d < DMAX; ++d) {
              int bp = 0;
#pragma unroll
              for (int n = 0; n < MAXN; ++n) if (n == best) bp = npods[n][d];
              if (d >= D || bp <= 0) continue;
              if (dep[d].pdb) pdb_pods += bp;
              cm &= capsel[d];
              s_cpu += bp * dep[d].req_cpu;
              s_mem += bp * dep[d].req_mem;
              s_pods += bp;
            }
            cand &= ~(1u << best);
            if (pdb_pods > allowed || !cm) continue;
            int bk, bz, bc, bpr;
            find_offer(zm, cm, use, limit, usem, limitm, s_cpu, s_mem, s_pods, bk, bz, bc, bpr);
            if (bk < 0 || bpr >= bprice) continue;
            launch_replacement(q, slot, 1u << best, bk, bz, bc, bpr);
            deleted++;
            break;
          }
        };
        // ---- G3. multi-node consolidation (SEMANTICS 3.G3): Karpenter's firstN
        // binary search over the prefix (>= 2 candidates, consolidation order)
        // that can leave together with at most one strictly cheaper
        // replacement; the winning prefix is re-evaluated with commit = true
        // (one evaluation site keeps the unrolled slot loops emitted once)
        auto try_multi = [&](int q, int qca, int budget, int& deleted) -> bool {
          if (deleted >= budget) return false;
          const uint32_t tn = taint_mask();
          uint32_t cset = 0;
          int cpods[MAXN];
#pragma unroll
          for (int n = 0; n < MAXN; ++n) {
            int pods = 0;
#pragma unroll
            for (int d = 0; d < DMAX; ++d) pods += d < D ? npods[n][d] : 0;
            cpods[n] = pods;
            const bool c = ((rdy & ~tn) >> n & 1u) && ni_pool(ninfo[n]) == q &&
                           (t - nlast[n]) * CCKA_STEP_SECONDS >= qca && pods > 0;
            cset |= (c ? 1u : 0u) << n;
          }
          // rank in (pods asc, price desc, slot asc) order; ordl nibble r = slot of rank r
          unsigned long long ordl = 0;
#pragma unroll
          for (int n = 0; n < MAXN; ++n) {
            int rk = 0;
#pragma unroll
            for (int m = 0; m < MAXN; ++m) {
              const bool before = cpods[m] < cpods[n] ||
                                  (cpods[m] == cpods[n] && (nprice[m] > nprice[n] || (nprice[m] == nprice[n] && m < n)));
              rk += ((cset >> m & 1u) && before) ? 1 : 0;
            }
            if (cset >> n & 1u) ordl |= (unsigned long long)n << (4 * rk);
          }
          const int nc = min(__popc(cset), budget - deleted);
          int lo = 1, hi = nc - 1, bestk = 0, mid = 0;
          bool acted = false;
          while (true) {
            int k;
            bool commit = false;
            if (lo <= hi) { mid = (lo + hi) / 2; k = mid + 1; }
            else if (bestk) { k = bestk; commit = true; }
            else break;
            // ---- evaluate the first k candidates ----
            uint32_t set = 0;
            for (int r = 0; r < k; ++r) set |= 1u << ((ordl >> (4 * r)) & 15u);
            long long pdbp = 0, psum = 0;
            bool all_spot = true;
            int tpods[MAXN][DMAX];
#pragma unroll
            for (int n = 0; n < MAXN; ++n) {
#pragma unroll
              for (int d = 0; d < DMAX; ++d) tpods[n][d] = npods[n][d];
              if (set >> n & 1u) {
                psum += nprice[n];
                all_spot = all_spot && ni_cap(ninfo[n]) == 0;
#pragma unroll
                for (int d = 0; d < DMAX; ++d) if (d < D && dep[d].pdb) pdbp += npods[n][d];
              }
            }
            bool ok = pdbp <= allowed;
            uint32_t touched = 0;
            const uint32_t recv = rdy & ~tn & ~set;
            for (int r = 0; r < k && ok; ++r) {
              const int c = (int)((ordl >> (4 * r)) & 15u);
              int cp[DMAX];
#pragma unroll
              for (int d = 0; d < DMAX; ++d) {
                cp[d] = 0;
#pragma unroll
                for (int n = 0; n < MAXN; ++n) if (n == c) cp[d] = tpods[n][d];
              }
#pragma unroll
              for (int d = 0; d < DMAX; ++d) {
                if (d >= D) continue;
                int need_d = cp[d];
#pragma unroll
                for (int m = 0; m < MAXN; ++m) {
                  const uint32_t x = ninfo[m];
                  if (need_d > 0 && (recv >> m & 1u) && (capbit(ni_cap(x)) & capsel[d])) {
                    int f;
                    if (DMAX == 1) {
                      f = ncap[m] - tpods[m][0];
                    } else {
                      int sc = 0, sm = 0, sp = 0;
#pragma unroll
                      for (int e = 0; e < DMAX; ++e) {
                        if (e >= D) continue;
                        sc += tpods[m][e] * dep[e].req_cpu;
                        sm += tpods[m][e] * dep[e].req_mem;
                        sp += tpods[m][e];
                      }
                      f = max(type_fit<DMAX>(L, ni_type(x), sc, sm, sp, dep[d].req_cpu, dep[d].req_mem), 0);
                    }
                    const int kk = min(f, need_d);
                    if (kk > 0) { tpods[m][d] += kk; need_d -= kk; touched |= 1u << m; }
                  }
                }
                cp[d] = need_d;
              }
#pragma unroll
              for (int n = 0; n < MAXN; ++n)
                if (n == c) {
#pragma unroll
                  for (int d = 0; d < DMAX; ++d) tpods[n][d] = cp[d];
                }
            }
            // leftover pods need one new node, strictly cheaper than the set
            int s_cpu = 0, s_mem = 0, s_pods = 0;
            uint32_t cm = 0, zm = 0;
            int use = 0, limit = 0, usem = 0;
            const int limitm = w->pools[q].limit_mem_mi;
#pragma unroll
            for (int qq = 0; qq < CCKA_MAX_POOLS; ++qq)
              if (qq == q) { cm = pcm[qq]; zm = pzm[qq]; use = puse[qq]; limit = plimit[qq]; }
#pragma unroll
            for (int n = 0; n < MAXN; ++n) {
              if (!(set >> n & 1u)) continue;
#pragma unroll
              for (int d = 0; d < DMAX; ++d) {
                if (d >= D || tpods[n][d] <= 0) continue;
                cm &= capsel[d];
                s_cpu += tpods[n][d] * dep[d].req_cpu;
                s_mem += tpods[n][d] * dep[d].req_mem;
                s_pods += tpods[n][d];
              }
            }
            int bk = -1, bz = 0, bc = 0, bpr = 0;
            const uint32_t fr = ~used & slot_mask;
            if (ok && s_pods > 0) {
              if (all_spot) cm &= ~(uint32_t)CCKA_CAP_SPOT;
              ok = cm != 0 && fr != 0;
              if (ok) {
                if (limitm >= 0) usem = pool_mem(q);
                find_offer(zm, cm, use, limit, usem, limitm, s_cpu, s_mem, s_pods, bk, bz, bc, bpr);
                ok = bk >= 0 && (long long)bpr < psum;
              }
            }
            if (!commit) {
              if (ok) { bestk = k; lo = mid + 1; }
              else hi = mid - 1;
              continue;
            }
            // ---- commit: moves, emptied candidates leave now, the rest await the replacement ----
            uint32_t srcm = 0;
#pragma unroll
            for (int n = 0; n < MAXN; ++n) {
#pragma unroll
              for (int d = 0; d < DMAX; ++d) npods[n][d] = tpods[n][d];
              if (touched >> n & 1u) nlast[n] = t;
            }
#pragma unroll
            for (int n = 0; n < MAXN; ++n) {
              if (!(set >> n & 1u)) continue;
              int left = 0;
#pragma unroll
              for (int d = 0; d < DMAX; ++d) left += d < D ? npods[n][d] : 0;
              if (left > 0) srcm |= 1u << n;
            }
            uint32_t gone = set & ~srcm;
            while (gone) {
              const int n = __builtin_ctz(gone);
              gone &= gone - 1u;
              free_slot(n);
              deletions++;
              flags |= 4u;
            }
            if (s_pods > 0) launch_replacement(q, __builtin_ctz(fr), srcm, bk, bz, bc, bpr);
            flags |= 64u;
            allowed -= pdbp;
            deleted += k;
            any_deleted = true;
            acted = true;
            break;
          }
          return acted;
        };
        // ---- G1. ready replacements take over their sources' pods (SEMANTICS 3.G0, 3.G2, 3.G3):
        // replacements in slot order, each one's sources in slot order ----
        if (greplace || gdrift || gmulti) {
          uint32_t rm = 0;
#pragma unroll
          for (int m = 0; m < MAXN; ++m) rm |= ((nsrc[m] != 0) && (rdy >> m & 1u) ? 1u : 0u) << m;
          while (rm) {
            const int m = __builtin_ctz(rm);
            rm &= rm - 1u;
            uint32_t sm = 0, xm = 0;
#pragma unroll
            for (int n = 0; n < MAXN; ++n) if (n == m) { sm = nsrc[n]; nsrc[n] = 0; xm = ninfo[n]; }
            rm &= ~sm;
            while (sm) {
              const int src = __builtin_ctz(sm);
              sm &= sm - 1u;
              int sp[DMAX];
#pragma unroll
              for (int d = 0; d < DMAX; ++d) {
                sp[d] = 0;
#pragma unroll
                for (int n = 0; n < MAXN; ++n) if (n == src) sp[d] = npods[n][d];
              }
#pragma unroll
              for (int d = 0; d < DMAX; ++d) {
                if (d >= D) continue;
                int k = 0;
                if (capbit(ni_cap(xm)) & capsel[d]) {
#pragma unroll
                  for (int n = 0; n < MAXN; ++n) {
                    if (n == m) {
                      int f;
                      if (DMAX == 1) {
                        f = ncap[n] - npods[n][0];
                      } else {
                        int sc = 0, smm = 0, spp = 0;
#pragma unroll
                        for (int e = 0; e < DMAX; ++e) {
                          if (e >= D) continue;
                          sc += npods[n][e] * dep[e].req_cpu;
                          smm += npods[n][e] * dep[e].req_mem;
                          spp += npods[n][e];
                        }
                        f = max(type_fit<DMAX>(L, ni_type(xm), sc, smm, spp, dep[d].req_cpu, dep[d].req_mem), 0);
                      }
                      k = min(f, sp[d]);
                      npods[n][d] += k;
                    }
                  }
                }
                rpods[d] -= sp[d] - k;
                placed[d] -= sp[d] - k;
              }
              free_slot(src);
              deletions++;
            }
#pragma unroll
            for (int n = 0; n < MAXN; ++n) if (n == m) nlast[n] = t;
            any_deleted = true;
            flags |= 4u;
          }
        }
        // the PDB allowance counts after the takeovers (evictions change it)
        if (pdb_pct >= 0) {
          long long rdyp = 0, reps = 0;
#pragma unroll
          for (int d = 0; d < DMAX; ++d) {
            if (d >= D || !dep[d].pdb) continue;
            reps += replicas[d];
            rdyp += rpods[d];
          }
          allowed = max(rdyp - ((long long)pdb_pct * reps + 99) / 100, 0LL);
        }
        // drifted nodes (SEMANTICS 3.G0): zone / capacity type outside the
        // pool's current requirements
        uint32_t dmask = 0;
        if (gdrift) {
#pragma unroll
          for (int n = 0; n < MAXN; ++n) {
            const uint32_t x = ninfo[n];
            uint32_t zm = 0, cm = 0;
#pragma unroll
            for (int qq = 0; qq < CCKA_MAX_POOLS; ++qq)
              if (qq == ni_pool(x)) { zm = pzm[qq]; cm = pcm[qq]; }
            if ((used >> n & 1u) && (!(zm >> ni_zone(x) & 1u) || !(cm & capbit(ni_cap(x))))) dmask |= 1u << n;
          }
        }
        for (int q = 0; q < NP; ++q) {
          int npool = 0, qbudget = 0, qca = 0, qpol = 0;
#pragma unroll
          for (int qq = 0; qq < CCKA_MAX_POOLS; ++qq)
            if (qq == q) { qbudget = pbudget[qq]; qca = pca[qq]; qpol = ppol[qq]; }
#pragma unroll
          for (int n = 0; n < MAXN; ++n) npool += ((used >> n & 1u) && ni_pool(ninfo[n]) == q) ? 1 : 0;
          if (npool == 0) continue;
          const int budget = (qbudget * npool + 99) / 100;
          int deleted = 0;
          // ---- G0. drift: slot order, shares the pool budget, no consolidateAfter ----
          if (dmask) {
            uint32_t pq = 0;
#pragma unroll
            for (int n = 0; n < MAXN; ++n) pq |= (ni_pool(ninfo[n]) == q ? 1u : 0u) << n;
            uint32_t srcm = 0;  // nodes whose pre-spun replacement is in flight wait for it
#pragma unroll
            for (int n = 0; n < MAXN; ++n) srcm |= nsrc[n];
            uint32_t cand = dmask & rdy & pq & ~srcm;
            while (cand && deleted < budget) {
              const int best = __builtin_ctz(cand);
              cand &= cand - 1u;
              int bp[DMAX];
              long long pdb_pods = 0;
#pragma unroll
              for (int d = 0; d < DMAX; ++d) {
                bp[d] = 0;
#pragma unroll
                for (int n = 0; n < MAXN; ++n) if (n == best) bp[d] = npods[n][d];
                if (d < D && dep[d].pdb) pdb_pods += bp[d];
              }
              if (pdb_pods > allowed) continue;
              // pods move first-fit onto ready, non-drifted nodes; the rest are
              // evicted (Pending until E/F of a later step)
              const uint32_t recv = rdy & ~dmask & ~taint_mask();
              int left[DMAX];
#pragma unroll
              for (int d = 0; d < DMAX; ++d) {
                left[d] = 0;
                if (d >= D) continue;
                int need_d = bp[d];
#pragma unroll
                for (int n = 0; n < MAXN; ++n) {
                  const uint32_t x = ninfo[n];
                  if (need_d > 0 && (recv >> n & 1u) && (capbit(ni_cap(x)) & capsel[d])) {
                    int f;
                    if (DMAX == 1) {
                      f = ncap[n] - npods[n][0];
                    } else {
                      int sc = 0, sm = 0, sp = 0;
#pragma unroll
                      for (int e = 0; e < DMAX; ++e) {
                        if (e >= D) continue;
                        sc += npods[n][e] * dep[e].req_cpu;
                        sm += npods[n][e] * dep[e].req_mem;
                        sp += npods[n][e];
                      }
                      f = max(type_fit<DMAX>(L, ni_type(x), sc, sm, sp, dep[d].req_cpu, dep[d].req_mem), 0);
                    }
                    const int k = min(f, need_d);
                    if (k > 0) { npods[n][d] += k; need_d -= k; nlast[n] = t; }
                  }
                }
                left[d] = need_d;
              }
              // pods that found no room: a pre-spun replacement under the new
              // requirements takes them when ready (G1); without a free slot
              // or an offering they are evicted and the node goes now
              int s_cpu = 0, s_mem = 0, s_pods = 0;
              uint32_t cm = 0, zm = 0;
              int use = 0, limit = 0, usem = 0;
              const int limitm = w->pools[q].limit_mem_mi;
              if (limitm >= 0) usem = pool_mem(q);
#pragma unroll
              for (int qq = 0; qq < CCKA_MAX_POOLS; ++qq)
                if (qq == q) { cm = pcm[qq]; zm = pzm[qq]; use = puse[qq]; limit = plimit[qq]; }
#pragma unroll
              for (int d = 0; d < DMAX; ++d) {
                if (d >= D || left[d] <= 0) continue;
                cm &= capsel[d];
                s_cpu += left[d] * dep[d].req_cpu;
                s_mem += left[d] * dep[d].req_mem;
                s_pods += left[d];
              }
              const uint32_t fr = ~used & slot_mask;
              int bk = -1, bz = 0, bc = 0, bpr = 0;
              // an ordinary provisioning decision: the F2 launch rule
              if (s_pods > 0 && fr && cm)
                lane_launch(zm, cm, use, limit, usem, limitm, s_cpu, s_mem, s_pods, bk, bz, bc, bpr);
              if (bk >= 0) {
#pragma unroll
                for (int n = 0; n < MAXN; ++n)
                  if (n == best) {
#pragma unroll
                    for (int d = 0; d < DMAX; ++d) npods[n][d] = d < D ? left[d] : 0;
                  }
                launch_replacement(q, __builtin_ctz(fr), 1u << best, bk, bz, bc, bpr);
                allowed -= pdb_pods;
                deleted++;
                flags |= 16u;
                continue;
              }
#pragma unroll
              for (int d = 0; d < DMAX; ++d) {
                rpods[d] -= left[d];
                placed[d] -= left[d];
              }
              free_slot(best);
              dmask &= ~(1u << best);
              allowed -= pdb_pods;
              deleted++;
              deletions++;
              any_deleted = true;
              flags |= 4u | 16u;
            }
          }
          if (DMAX == 1) {
            // identical pods: a candidate's pods fit first-fit on the other
            // compatible ready nodes iff their free capacities add up, so one
            // scan over the slots ranks every valid candidate (no rescans per
            // rejection); the winner is the first valid one in (pods asc, price
            // desc, slot asc) order, exactly as the spec's sequential search.
            uint32_t pm = 0, cm1 = 0;
#pragma unroll
            for (int n = 0; n < MAXN; ++n) {
              const uint32_t x = ninfo[n];
              if (ni_pool(x) == q) pm |= 1u << n;
              if (capbit(ni_cap(x)) & capsel[0]) cm1 |= 1u << n;
            }
            pm &= used;
            cm1 &= used;
            {
              const uint32_t tn = taint_mask();
              pm &= ~tn;   // no source of an in-flight replacement is a candidate
              cm1 &= ~tn;  // nor a receiver of moved pods
            }
            while (true) {
              if (deleted >= budget) { budget_hit = true; break; }
              int F = 0;
#pragma unroll
              for (int n = 0; n < MAXN; ++n) if ((rdy & cm1) >> n & 1u) F += ncap[n] - npods[n][0];
              int best = -1, bpods = 0, bprice = 0;
#pragma unroll
              for (int n = 0; n < MAXN; ++n) {
                if (!((pm & rdy) >> n & 1u)) continue;
                if ((t - nlast[n]) * CCKA_STEP_SECONDS < qca) continue;
                const int pods = npods[n][0];
                bool ok = pods == 0;
                if (!ok && qpol == CCKA_WHEN_EMPTY_OR_UNDERUTILIZED) {
                  const int fo = F - ((cm1 >> n & 1u) ? ncap[n] - pods : 0);
                  ok = fo >= pods && (!dep[0].pdb || (long long)pods <= allowed);
                }
                if (!ok) continue;
                const int pr = nprice[n];
                if (best < 0 || pods < bpods || (pods == bpods && pr > bprice)) { best = n; bpods = pods; bprice = pr; }
              }
              if (best < 0) break;
              int need_d = bpods;
#pragma unroll
              for (int n = 0; n < MAXN; ++n) {
                if (need_d > 0 && n != best && ((rdy & cm1) >> n & 1u)) {
                  const int k = min(ncap[n] - npods[n][0], need_d);
                  if (k > 0) { npods[n][0] += k; need_d -= k; nlast[n] = t; }
                }
              }
#pragma unroll
              for (int n = 0; n < MAXN; ++n) {
                if (n == best) {
                  if (ni_cap(ninfo[n]) == 0) nsp--; else nod--;
#pragma unroll
                  for (int qq = 0; qq < CCKA_MAX_POOLS; ++qq)
                    if (qq == q) puse[qq] -= L.types[ni_type(ninfo[n])].vcpu * 1000;
                  ninfo[n] = 0; nready[n] = 0; nlast[n] = 0; nprice[n] = 0; ncap[n] = 0; nsrc[n] = 0;
                  npods[n][0] = 0;
                }
              }
              burn -= bprice;
              used &= ~(1u << best);
              unlink(best);
              rdy &= ~(1u << best);
              pm &= ~(1u << best);
              cm1 &= ~(1u << best);
              if (dep[0].pdb) allowed -= bpods;
              deleted++;
              deletions++;
              any_deleted = true;
              flags |= 4u;
            }
            {
              const bool g3 = gmulti && qpol == CCKA_WHEN_EMPTY_OR_UNDERUTILIZED && try_multi(q, qca, budget, deleted);
              if (greplace && !g3 && qpol == CCKA_WHEN_EMPTY_OR_UNDERUTILIZED) try_replace(q, qca, budget, deleted);
            }
            continue;
          }
          uint32_t rejected = taint_mask();  // tainted nodes: neither candidates nor receivers
          const uint32_t tn_g = rejected;
          while (true) {
            if (deleted >= budget) { budget_hit = true; break; }
            int best = -1, bpods = 0, bprice = 0;
#pragma unroll
            for (int n = 0; n < MAXN; ++n) {
              const uint32_t x = ninfo[n];
              if (!((rdy & ~rejected) >> n & 1u) || ni_pool(x) != q) continue;
              if ((t - nlast[n]) * CCKA_STEP_SECONDS < qca) continue;
              int pods = 0;
#pragma unroll
              for (int d = 0; d < DMAX; ++d) pods += d < D ? npods[n][d] : 0;
              if (pods > 0 && qpol != CCKA_WHEN_EMPTY_OR_UNDERUTILIZED) continue;
              const int pr = nprice[n];
              if (best < 0 || pods < bpods || (pods == bpods && pr > bprice)) { best = n; bpods = pods; bprice = pr; }
            }
            if (best < 0) break;
            bool ok = true;
            long long pdb_pods = 0;
            if (DMAX == 1) {
              // identical pods: first-fit succeeds iff the other compatible
              // ready nodes' free capacities add up to the candidate's pods
              if (bpods > 0) {
                if (dep[0].pdb) pdb_pods = bpods;
                if (pdb_pods > allowed) ok = false;
                int free_sum = 0;
#pragma unroll
                for (int n = 0; n < MAXN; ++n)
                  if (n != best && ((rdy & ~tn_g) >> n & 1u) && (capbit(ni_cap(ninfo[n])) & capsel[0]))
                    free_sum += ncap[n] - npods[n][0];
                if (free_sum < bpods) ok = false;
              }
              if (!ok) { rejected |= 1u << best; continue; }
              int need_d = bpods;
#pragma unroll
              for (int n = 0; n < MAXN; ++n) {
                if (need_d > 0 && n != best && ((rdy & ~tn_g) >> n & 1u) && (capbit(ni_cap(ninfo[n])) & capsel[0])) {
                  const int k = min(ncap[n] - npods[n][0], need_d);
                  if (k > 0) { npods[n][0] += k; need_d -= k; nlast[n] = t; }
                }
              }
            } else {
              // the gate's necessary sums first (the state they were taken from
              // until this evaluation's first deletion): a candidate they reject
              // fails the first-fit trial below as well
              if (gsum && !any_deleted && bpods > 0) {
                int c = 0, m = 0;
                uint32_t cs = 0, xb = 0;
#pragma unroll
                for (int n = 0; n < MAXN; ++n)
                  if (n == best) {
                    xb = ninfo[n];
#pragma unroll
                    for (int e = 0; e < DMAX; ++e) {
                      const int k = e < D ? npods[n][e] : 0;
                      c += k * dep[e].req_cpu;
                      m += k * dep[e].req_mem;
                      cs |= k > 0 ? capsel[e] : 0u;
                    }
                  }
                const bool s0 = (cs & capbit(0)) != 0, s1 = (cs & capbit(1)) != 0;
                int vc = (s0 ? ac0 : 0) + (s1 ? ac1 : 0), vm = (s0 ? am0 : 0) + (s1 ? am1 : 0);
                int vp = (s0 ? ap0 : 0) + (s1 ? ap1 : 0);
                if (cs & capbit(ni_cap(xb))) {
                  const ccka_itype& ty = L.types[ni_type(xb)];
                  vc -= ty.alloc_cpu_m - c;
                  vm -= ty.alloc_mem_mi - m;
                  vp -= ty.max_pods - bpods;
                }
                if (!(c <= vc && m <= vm && bpods <= vp)) { rejected |= 1u << best; continue; }
              }
              int tpods[MAXN][DMAX];
              int tlast[MAXN];
#pragma unroll
              for (int n = 0; n < MAXN; ++n) {
                tlast[n] = nlast[n];
#pragma unroll
                for (int d = 0; d < DMAX; ++d) tpods[n][d] = npods[n][d];
              }
              if (bpods > 0) {
                int bp[DMAX];
#pragma unroll
                for (int d = 0; d < DMAX; ++d) {
                  bp[d] = 0;
#pragma unroll
                  for (int n = 0; n < MAXN; ++n) if (n == best) bp[d] = npods[n][d];
                  if (d < D && dep[d].pdb) pdb_pods += bp[d];
                }
                if (pdb_pods > allowed) ok = false;
#pragma unroll
                for (int d = 0; d < DMAX; ++d) {
                  if (d >= D || !ok) continue;
                  int need_d = bp[d];
#pragma unroll
                  for (int n = 0; n < MAXN; ++n) {
                    const uint32_t x = ninfo[n];
                    if (need_d > 0 && n != best && ((rdy & ~tn_g) >> n & 1u) && (capbit(ni_cap(x)) & capsel[d])) {
                      int sc = 0, sm = 0, sp = 0;
#pragma unroll
                      for (int e = 0; e < DMAX; ++e) {
                        if (e >= D) continue;
                        sc += tpods[n][e] * dep[e].req_cpu;
                        sm += tpods[n][e] * dep[e].req_mem;
                        sp += tpods[n][e];
                      }
                      const int f = max(type_fit<DMAX>(L, ni_type(x), sc, sm, sp, dep[d].req_cpu, dep[d].req_mem), 0);
                      const int k = min(f, need_d);
                      if (k > 0) { tpods[n][d] += k; need_d -= k; tlast[n] = t; }
                    }
                  }
                  if (need_d > 0) ok = false;
                }
              }
              if (!ok) { rejected |= 1u << best; continue; }
#pragma unroll
              for (int n = 0; n < MAXN; ++n) {
                nlast[n] = tlast[n];
#pragma unroll
                for (int d = 0; d < DMAX; ++d) npods[n][d] = tpods[n][d];
              }
            }
            // remove the node (its pods moved between ready nodes: running counts unchanged)
#pragma unroll
            for (int n = 0; n < MAXN; ++n) {
              if (n == best) {
                if (ni_cap(ninfo[n]) == 0) nsp--; else nod--;
#pragma unroll
                for (int qq = 0; qq < CCKA_MAX_POOLS; ++qq)
                  if (qq == q) puse[qq] -= L.types[ni_type(ninfo[n])].vcpu * 1000;
                ninfo[n] = 0; nready[n] = 0; nlast[n] = 0; nprice[n] = 0; ncap[n] = 0; nsrc[n] = 0;
#pragma unroll
                for (int d = 0; d < DMAX; ++d) npods[n][d] = 0;
              }
            }
            burn -= bprice;
            used &= ~(1u << best);
              unlink(best);
            rdy &= ~(1u << best);
            allowed -= pdb_pods;
            deleted++;
            deletions++;
            any_deleted = true;
            flags |= 4u;
          }
          {
            const bool g3 = gmulti && qpol == CCKA_WHEN_EMPTY_OR_UNDERUTILIZED && try_multi(q, qca, budget, deleted);
            if (greplace && !g3 && qpol == CCKA_WHEN_EMPTY_OR_UNDERUTILIZED) try_replace(q, qca, budget, deleted);
          }
        }
        bool pending_repl = false;
#pragma unroll
        for (int n = 0; n < MAXN; ++n) pending_repl |= nsrc[n] != 0;
        g_dirty = budget_hit || any_deleted || dmask != 0 || pending_repl;
      }
      if (g_eval) {
        // next step at which a node becomes a new candidate (consolidatable and ready)
        int wake = 0x7fffffff;
#pragma unroll
        for (int n = 0; n < MAXN; ++n) {
          if (used >> n & 1u) {
            int ca = 0;
#pragma unroll
            for (int q = 0; q < CCKA_MAX_POOLS; ++q) if (q == ni_pool(ninfo[n])) ca = pca[q];
            const int thr = max(nready[n], nlast[n] + (ca + CCKA_STEP_SECONDS - 1) / CCKA_STEP_SECONDS);
            if (thr > t) wake = min(wake, thr);
          }
        }
        g_wake = wake;
      }
      GK_STAMP(5);  // disruption
      // ---- H. accounting ----
      long long upp[DMAX];
#pragma unroll
      for (int d = 0; d < DMAX; ++d) {
        upp[d] = 0;
        if (d >= D) continue;
        const int rd = rpods[d];
        if (rd > 0) {
          long long usage = Lcur[d];
          if (dep[d].limit > 0) usage = min(usage, (long long)rd * dep[d].limit);
          upp[d] = (long long)((uint32_t)max(usage, 0LL) / (uint32_t)rd);  // usage <= INT32_MAX
        }
      }
      long long e_step = base_nw;
#pragma unroll
      for (int n = 0; n < MAXN; ++n) {
        if (!(used >> n & 1u) || ablated(p.ablate, 4)) continue;
        const ccka_itype& ty = L.types[ni_type(ninfo[n])];
        long long use = 0;
        if (rdy >> n & 1u) {
#pragma unroll
          for (int d = 0; d < DMAX; ++d) if (d < D) use += (long long)npods[n][d] * upp[d];
          use = min(use, (long long)ty.alloc_cpu_m);
        }
        const long long en = ty.idle_nw + ty.dyn_nw_per_m * use;
        e_step += en;
        if (det) {
          const int q = ni_pool(ninfo[n]);
          det->d.pool_cost_uphmin[q] += nprice[n];
          det->d.pool_energy_nwmin[q] += en;
          det->e_hour[q] += en;
          if (ni_cap(ninfo[n]) == 0) det->d.pool_node_min_spot[q]++;
          else det->d.pool_node_min_od[q]++;
        }
      }
      if (det) {
        det->d.base_cost_uphmin += base_price;
        det->d.base_energy_nwmin += base_nw;
        det->base_e_hour += base_nw;
        for (int q = 0; q < NP; ++q) {
          int cnt = 0;
#pragma unroll
          for (int n = 0; n < MAXN; ++n) cnt += ((used >> n) & 1u) && ni_pool(ninfo[n]) == q ? 1 : 0;
          det->d.pool_peak_nodes[q] = max(det->d.pool_peak_nodes[q], cnt);
        }
      }
      cost += burn + base_price;
      energy_nw += e_step;
      e_hour += e_step;
      int pending = 0, reps = 0;
      bool viol = false;
#pragma unroll
      for (int d = 0; d < DMAX; ++d) {
        if (d >= D) continue;
        pending += replicas[d] - rpods[d];
        reps += replicas[d];
        if (dep[d].scaler == CCKA_SCALER_HPA && util_valid[d] && util[d] > slo_util) viol = true;
        if (dep[d].scaler == CCKA_SCALER_KEDA && kact_any[d] && replicas[d] == 0) viol = true;
      }
      if (pending > 0) viol = true;
      if (viol) { slo++; flags |= 8u; }
      pend_min += pending;
      nmin_spot += nsp;
      nmin_od += nod;
      peak_nodes = max(peak_nodes, nsp + nod);
      if (p.traj) {
        ccka_traj_rec rcd;
        rcd.replicas = reps;
        rcd.pending = pending;
        rcd.nodes_spot = (uint16_t)nsp;
        rcd.nodes_od = (uint16_t)nod;
        rcd.last_type = (uint16_t)step_last_type;
        rcd.flags = (uint16_t)flags;
        // SK: scenario-major [N][T] (a lane's steps fill whole lines however far the lanes drift apart)
        const int64_t ri = SK ? i * (int64_t)p.T + t : (int64_t)t * p.N + i;
        *reinterpret_cast<int4*>(&p.traj[ri]) = *reinterpret_cast<int4*>(&rcd);
      }
    }
    GK_STAMP(6);  // accounting, record
    if constexpr (SK) {
      if (active) {
        sk_caches(t, (flags & 1u) != 0);
        tl = t + 1;
        tq = tl;
        ev = false;
      }
      GK_STAMP(9);  // SK: the quiet steps' caches
    }
    }  // the full step
    if constexpr (SK) {
      // this pass's quiet-step samples, steps tl .. tl + SKS - 1 (loaded after
      // the full steps: held across them they would spill): from the
      // scenario-major copy, one contiguous run per lane ([NL][T][DMAX]), or
      // gathered from [T][D][N]
      if (p.load_nt) {
        const int32_t* b = p.load_nt + lcol * (int64_t)p.T * DMAX;
#pragma unroll
        for (int s = 0; s < SKS; ++s) {
          const int ts = min(tl + s, p.T - 1);
          if constexpr (DMAX == 2) {
            const int2 v = *reinterpret_cast<const int2*>(b + (int64_t)ts * 2);
            Lq[s][0] = v.x;
            Lq[s][1] = v.y;
          } else {
#pragma unroll
            for (int q = 0; q < DMAX / 4; ++q) {
              const int4 v = *reinterpret_cast<const int4*>(b + (int64_t)ts * DMAX + 4 * q);
              Lq[s][4 * q] = v.x;
              Lq[s][4 * q + 1] = v.y;
              Lq[s][4 * q + 2] = v.z;
              Lq[s][4 * q + 3] = v.w;
            }
          }
        }
      } else {
#pragma unroll
        for (int s = 0; s < SKS; ++s) {
          const int ts = min(tl + s, p.T - 1);
#pragma unroll
          for (int d = 0; d < SKD; ++d) Lq[s][d] = lptr[((int64_t)ts * D + (d < D ? d : 0)) * lstride];
        }
      }
      // ---- quiet steps: up to SKS per iteration and lane ----
      // (a rolled loop over a shifting sample window: the unrolled one is SKS
      // copies of the sub-step, code that the full steps' evict from the
      // instruction cache every pass)
#ifdef SK_QUNROLL
#pragma unroll
#else
#pragma unroll 1
#endif
      for (int s = 0; s < SKS; ++s) {
        if (active && !ev && tl < t1) {
          const int tc = tl;
          bool ok = tc < nxt;
          int us[SKD];
          bool ge[SKD];
#pragma unroll
          for (int d = 0; d < SKD; ++d) {
            us[d] = 0;
            ge[d] = false;
            if (d >= D) continue;
            us[d] = min(Lq[0][d], q_rcap[d]);  // usage clamped by the pods' CPU limit
            if (dep[d].scaler != CCKA_SCALER_HPA) continue;
            ge[d] = us[d] >= q_pge[d];
            ok = ok && (uint32_t)us[d] < (uint32_t)q_ulim[d] && (ge[d] || tc <= q_hold[d]);
          }
          if (ok) {
            bool slo_b = q_sloall;
            uint32_t upp[SKD];
            float sat = 0.f;
#pragma unroll
            for (int d = 0; d < SKD; ++d) {
              upp[d] = 0u;
              if (d >= D) continue;
              // upp = floor(usage / ready): a binary32 reciprocal estimate and one
              // remainder correction, exact while upp < 2^20 (else the division)
              const int rd = max(rpods[d], 1);
              const uint32_t a = (uint32_t)max(us[d], 0);
              uint32_t q = (uint32_t)((float)a * __builtin_amdgcn_rcpf((float)rd));
              const int rm = (int)(a - q * (uint32_t)rd);
              q = q + (rm >= rd ? 1u : 0u) - (rm < 0 ? 1u : 0u);
              if (__builtin_expect(q >= (1u << 20), 0)) q = a / (uint32_t)rd;
              upp[d] = rpods[d] > 0 ? q : 0u;
              q_usum[d] += upp[d];
              sat += (float)upp[d] * q_R[d];
              if (dep[d].scaler != CCKA_SCALER_HPA) continue;
              const bool ran = (q_ran >> d & 1u) != 0;
              // the proposal is cur from q_pge on below maxReplicas; else the raw
              // usage goes into the record, its proposal computed at the flush
              const bool raw = !ge[d] || (q_atmax >> d & 1u) != 0;
              if (ge[d]) q_hold[d] = max(q_hold[d], tc + __popc((uint32_t)dnmask[d]));
              slo_b = slo_b || us[d] >= q_slo[d];
#pragma unroll
              for (int k = CCKA_HIST - 1; k > 0; --k) rec[d][k] = rec[d][k - 1];
              rec[d][0] = ran ? (raw ? us[d] : replicas[d]) : 0;
              q_rawm[d] = ((q_rawm[d] << 1) | ((ran && raw) ? 1u : 0u)) & 0xFFu;
              recv[d] = ((recv[d] << 1) | (ran ? 1u : 0u)) & 0xFFu;
            }
            if (__builtin_expect(sat >= 0.9999f, 0)) {  // a node may saturate: the exact per-node sum
              long long lin = 0;
#pragma unroll
              for (int d = 0; d < SKD; ++d) lin += (long long)upp[d] * q_W[d];
              q_corr += sk_dyn(upp) - lin;
            }
            slo += slo_b ? 1 : 0;
            if (p.traj) {
              const int4 r = make_int4(q_reps, q_pend, (nsp & 0xFFFF) | nod << 16, q_w0 | (slo_b ? (8 << 16) : 0));
              *reinterpret_cast<int4*>(&p.traj[i * (int64_t)p.T + tc]) = r;
            }
            tl = tc + 1;
            if constexpr (kSKS) sks_c[8]++;
#pragma unroll
            for (int q = 0; q + 1 < SKS; ++q) {
#pragma unroll
              for (int d = 0; d < SKD; ++d) Lq[q][d] = Lq[q + 1][d];
            }
          } else {
            ev = true;
            if constexpr (kSKS) {
              if (tc >= nxt) {
#pragma unroll
                for (int r = 0; r < 5; ++r) sks_c[r] += sks_why == r ? 1 : 0;
              } else {
                sks_c[5]++;
              }
            }
          }
        }
      }
      GK_STAMP(8);  // SK: quiet steps
    } else {
      ++tt;
      minute = minute == 1439 ? 0 : minute + 1;
    }
  }
  if constexpr (kGKS) {
    if (p.stamps && lane == (__ffsll((long long)__ballot(1)) - 1)) {
#pragma unroll
      for (int k = 0; k < 11; ++k) atomicAdd(&p.stamps[k], gst[k]);
      atomicAdd(&p.stamps[11], 1ull);  // waves
    }
  }
  if constexpr (kSKS) {
    if (p.stamps) {
#pragma unroll
      for (int k = 0; k < 12; ++k) atomicAdd(&p.stamps[k], (unsigned long long)sks_c[k]);
    }
  }
  if (!active) return;
  if constexpr (SK) sk_flush();  // the quiet steps since the last full step
  if (p.state) state_io(true);
  if (p.feat || p.feat_rec) {  // policy features of step t1 (SEMANTICS 5)
    uint32_t fw[32];
    feat_words(t1, fw);
    if (p.feat) store_feat(p.feat + i * 64, fw);
    if (POL != 0 && p.feat_rec) store_feat(p.feat_rec + ((int64_t)t1 * p.N + i) * 64, fw);
  }
  if (t1 == p.T) gco2 += (double)e_hour * (ci_gpwmin * 1e-9);  // the last hour's carbon (run outputs only)
  if (det && t1 == p.T) {
    for (int q = 0; q < NP; ++q) {
      det->d.pool_gco2[q] += (double)det->e_hour[q] * (ci_gpwmin * 1e-9);
      int cnt = 0;
#pragma unroll
      for (int n = 0; n < MAXN; ++n) cnt += ((used >> n) & 1u) && ni_pool(ninfo[n]) == q ? 1 : 0;
      det->d.pool_final_nodes[q] = cnt;
    }
    det->d.base_gco2 += (double)det->base_e_hour * (ci_gpwmin * 1e-9);
#pragma unroll
    for (int d = 0; d < DMAX; ++d)
      if (d < D) {
        det->d.desired[d] = replicas[d];
        det->d.ready[d] = rpods[d];
        det->d.pending[d] = replicas[d] - rpods[d];
      }
  }
  int reps = 0;
#pragma unroll
  for (int d = 0; d < DMAX; ++d) reps += d < D ? replicas[d] : 0;
  p.cost[i] = cost;
  p.energy[i] = (double)energy_nw * 1e-9;
  p.gco2[i] = gco2;
  p.slo[i] = slo;
  p.pend_min[i] = pend_min;
  p.nmin_spot[i] = nmin_spot;
  p.nmin_od[i] = nmin_od;
  p.launches[i] = launches;
  p.deletions[i] = deletions;
  p.peak_nodes[i] = peak_nodes;
  p.final_reps[i] = reps;
  p.final_nodes[i] = __popc(used);
  p.last_choice[i] = last_choice;
  p.hash[i] = hash;
}

#ifndef CCKA_ROLLOUT_PART
// ---------------------------------------------------------------------------
// Totals: fixed-order block partials, then one ordered final pass.
// ---------------------------------------------------------------------------
struct Part {
  long long v[11];  // ccka_totals' int64 block (energy and gCO2 in fixed point) + overflow flag
};

// a + b into a, setting the flag instead of wrapping (signed int64)
__device__ __forceinline__ void add_chk(long long& a, long long b, long long& ovf) {
  long long r;
  if (__builtin_add_overflow(a, b, &r)) ovf = 1;
  a = r;
}
// llrint(x * scale), flagged when it is not representable (|x * scale| >= 2^63)
__device__ __forceinline__ long long fix_chk(double x, double scale, long long& ovf) {
  const double y = x * scale;
  if (!(y > -9.2233720368547758e18 && y < 9.2233720368547758e18)) {
    ovf = 1;
    return 0;
  }
  return __double2ll_rn(y);
}

__global__ void __launch_bounds__(256) totals_partial(TotParams q) {
  __shared__ Part sp[256];
  const int tid = threadIdx.x;
  Part a;
#pragma unroll
  for (int k = 0; k < 11; ++k) a.v[k] = 0;
  long long& ovf = a.v[10];
  const int64_t chunk = (q.N + gridDim.x - 1) / gridDim.x;
  const int64_t lo = (int64_t)blockIdx.x * chunk, hi = min(lo + chunk, q.N);
  for (int64_t i = lo + tid; i < hi; i += blockDim.x) {
    a.v[0] += 1;
    add_chk(a.v[1], q.cost[i], ovf);
    a.v[2] += q.slo[i];  // int32 per scenario: < 2^31 * N, no overflow below N = 2^32
    add_chk(a.v[3], q.pend_min[i], ovf);
    a.v[4] += q.nmin_spot[i];
    a.v[5] += q.nmin_od[i];
    a.v[6] += q.launches[i];
    a.v[7] += q.deletions[i];
    add_chk(a.v[8], fix_chk(q.energy[i], 1e6, ovf), ovf);  // llrint, as ccka_oracle_totals
    add_chk(a.v[9], fix_chk(q.gco2[i], 1e6, ovf), ovf);
  }
  sp[tid] = a;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (tid < s) {
#pragma unroll
      for (int k = 0; k < 10; ++k) add_chk(sp[tid].v[k], sp[tid + s].v[k], sp[tid].v[10]);
      sp[tid].v[10] |= sp[tid + s].v[10];
    }
    __syncthreads();
  }
  if (tid == 0) q.parts[blockIdx.x] = sp[0];
}

__global__ void totals_final(TotParams q, int nparts) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  Part a;
  for (int k = 0; k < 11; ++k) a.v[k] = 0;
  for (int b = 0; b < nparts; ++b) {
    for (int k = 0; k < 10; ++k) add_chk(a.v[k], q.parts[b].v[k], a.v[10]);
    a.v[10] |= q.parts[b].v[10];
  }
  ccka_totals* o = q.out;
  o->scenarios = a.v[0];
  o->cost_uphmin = a.v[1];
  o->slo_minutes = a.v[2];
  o->pending_pod_minutes = a.v[3];
  o->node_min_spot = a.v[4];
  o->node_min_od = a.v[5];
  o->launches = a.v[6];
  o->deletions = a.v[7];
  o->energy_uwmin = a.v[8];
  o->gco2_ug = a.v[9];
  o->energy_wmin = (double)a.v[8] * 1e-6;
  o->gco2 = (double)a.v[9] * 1e-6;
  *q.ovf = a.v[10];
}

// ---------------------------------------------------------------------------
// launchers (called from ccka_abi.cpp)
// ---------------------------------------------------------------------------
hipError_t launch_gen_load(const GenParams& g, hipStream_t s) {
  dim3 grid((unsigned)((g.n + 255) / 256), (unsigned)g.D);
  hipLaunchKernelGGL(gen_load_kernel, grid, dim3(256), 0, s, g);
  return hipGetLastError();
}

hipError_t launch_rollout(const KParams& p, int block, size_t lds, hipStream_t s) {
  const unsigned grid = (unsigned)((p.N + block - 1) / block);
#ifdef CCKA_DEV_POL_ONLY  // development builds of the fused loop alone (compile time)
  (void)grid; (void)lds; (void)s;
  return hipErrorInvalidValue;
#else
  // the smallest instantiation that holds the world (kernel_dims); four or
  // more deployments: rollout_multi.hip
  int dmax, nmax;
  kernel_dims(p.D, p.maxn, &dmax, &nmax);
  if (dmax >= 4) return launch_rollout_multi(p, block, lds, s);
  if (dmax == 1 && nmax == 8)
    hipLaunchKernelGGL((rollout_kernel<1, 8>), dim3(grid), dim3(block), lds, s, p);
  else if (dmax == 1)
    hipLaunchKernelGGL((rollout_kernel<1, 16>), dim3(grid), dim3(block), lds, s, p);
  else if (dmax == 2 && nmax == 8)
    hipLaunchKernelGGL((rollout_kernel<2, 8>), dim3(grid), dim3(block), lds, s, p);
  else
    hipLaunchKernelGGL((rollout_kernel<2, 16>), dim3(grid), dim3(block), lds, s, p);
  return hipGetLastError();
#endif
}

hipError_t launch_totals(const TotParams& q, int nparts, hipStream_t s) {
  hipLaunchKernelGGL(totals_partial, dim3(nparts), dim3(256), 0, s, q);
  hipLaunchKernelGGL(totals_final, dim3(1), dim3(64), 0, s, q, nparts);
  return hipGetLastError();
}

#endif  // CCKA_ROLLOUT_PART

}  // namespace ccka
