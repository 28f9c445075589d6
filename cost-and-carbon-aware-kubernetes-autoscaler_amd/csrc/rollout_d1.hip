// rollout_d1.hip — MI355X (gfx950) rollout engine for single-deployment HPA
// worlds (BASELINE configs 2-4: one Deployment per cluster scenario).
//
// Same semantics as rollout_kernel (docs/SEMANTICS.md), re-planned for the
// common case so that a quiet step (no scale event) costs a few dozen VALU
// instructions:
//   * Karpenter launch choice (SEMANTICS §3.F, the argmin over cost + carbon
//     weight, spot-first): with one deployment and no pool CPU limits it is a
//     pure function of (region, hour, zone mask, capacity mask, carbon weight,
//     pod count). table_kernel evaluates it once per rollout for every key
//     with wavefront prefix-argmin scans over the catalog sorted by pod
//     capacity; a launch is then one L2-resident load instead of a
//     wave-serialised catalog scan per lane.
//   * HPA utilisation (upstream replica_calculator.go) is a 32-bit integer
//     division; the 10 % tolerance test is an integer interval on util derived
//     exactly from the binary64 ratio test. The binary64 proposal arithmetic
//     runs only on scale events.
//   * HPA history rings (stabilisation window, rate periods) are packed int16.
//   * Disruption (Karpenter WhenEmpty / WhenEmptyOrUnderutilized) keeps a
//     per-slot "consolidatable from step" and is evaluated only when state
//     changed or a node crossed that threshold; with identical pods the
//     first-fit re-packing test reduces to a sum of free capacities.
// Results are bit-identical to the CPU oracle (tests/test_gpu_parity.py).
//
// Reference anchors: the NodePool profile patches demo_19_reset_policies.sh:68-75,
// demo_20_offpeak_configure.sh:59-81, demo_21_peak_configure.sh:56-77; pods
// demo_30_burst_configure.sh:57-141; PDB demo_10_setup_configure.sh:47-56.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ccka.h"
#include "d1_common.h"
#include "kparams.h"

#pragma clang fp contract(off)

namespace ccka {

namespace {

// ---------------------------------------------------------------------------
// argmin tables
// ---------------------------------------------------------------------------
struct Best {
  double s;   // score
  int k;      // catalog index (tie-break)
  int info;   // packed k | z<<10 | c<<12 (cap1 added on write)
  int price;
};

__device__ __forceinline__ bool better(double s2, int k2, double s, int k) {
  return s2 < s || (s2 == s && k2 < k);
}

__device__ __forceinline__ void take_if_better(Best& a, const Best& b) {
  if (better(b.s, b.k, a.s, a.k)) a = b;
}

__device__ __forceinline__ Best shfl_up_best(const Best& a, int off) {
  Best o;
  o.s = __shfl_up(a.s, off);
  o.k = __shfl_up(a.k, off);
  o.info = __shfl_up(a.info, off);
  o.price = __shfl_up(a.price, off);
  return o;
}

__device__ __forceinline__ Best readlane_best(const Best& a, int l) {
  Best o;
  const long long b = __double_as_longlong(a.s);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffLL), l);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  o.s = __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
  o.k = __builtin_amdgcn_readlane(a.k, l);
  o.info = __builtin_amdgcn_readlane(a.info, l);
  o.price = __builtin_amdgcn_readlane(a.price, l);
  return o;
}

}  // namespace

// One wave per key (region, hour, zone-mask index, capacity mask, carbon
// weight). Types are visited in pod-capacity-descending order, so the best
// offering among the first i types is the launch choice for every claim size
// n in (cap1[order[i+1]], cap1[order[i]]] (SEMANTICS §3.F: candidates hold the
// claim; spot offerings only, when spot is allowed and any is feasible; the
// lexicographic minimum of (score, k, z, c)). The per-chunk inclusive prefix
// argmin is a 6-round wavefront shuffle scan.
__global__ void __launch_bounds__(256) table_kernel(TableParams q) {
  const int lane = threadIdx.x & (WAVE - 1);
  const int64_t key = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / WAVE;
  const int64_t nkeys = (int64_t)q.R * 24 * q.NZI * 3 * q.NW;
  if (key >= nkeys) return;  // wave-uniform
  int64_t x = key;
  const int wi = (int)(x % q.NW); x /= q.NW;
  const int cmi = (int)(x % 3); x /= 3;
  const int zi = (int)(x % q.NZI); x /= q.NZI;
  const int rh = (int)x;  // r * 24 + h
  const uint32_t cm = (uint32_t)cmi + 1u, zm = q.zmasks[zi];
  const double wc = q.offer ? 0.0 : q.wc1000[wi];
  const double ci = q.ci_gpwh[rh];
  const int32_t* tile = q.price + (int64_t)rh * q.K * q.Z * 2;
  int2* out = q.table + key * q.JT;
  const double INF = __builtin_inf();
  Best cs{INF, 0x7fffffff, -1, 0}, ca{INF, 0x7fffffff, -1, 0};
  int jmax = 0;
  for (int base = 0; base < q.K; base += WAVE) {
    const int pos = base + lane;
    const bool v = pos < q.K;
    const int k = v ? q.order[pos] : 0;
    const int c1 = v ? q.cap1s[pos] : 0;
    const int c1n = pos + 1 < q.K ? q.cap1s[pos + 1] : 0;
    Best bs{INF, 0x7fffffff, -1, 0}, ba{INF, 0x7fffffff, -1, 0};
    if (v) {
      const double carbon = q.types[k].p_ref_w * ci;
      for (int z = 0; z < q.Z; ++z) {
        if (!(zm >> z & 1u)) continue;
        for (int c = 0; c < 2; ++c) {
          if (!(cm & (uint32_t)capbit1(c))) continue;
          const int pr = tile[(k * q.Z + z) * 2 + c];
          if (pr <= 0) continue;
          const double score = (double)pr + wc * carbon;
          const int info = k | z << 10 | c << 12;
          if (score < ba.s) { ba.s = score; ba.k = k; ba.info = info; ba.price = pr; }
          if (c == 0 && score < bs.s) { bs.s = score; bs.k = k; bs.info = info; bs.price = pr; }
        }
      }
      if (ba.info >= 0) jmax = max(jmax, c1);
    }
    // inclusive prefix argmin over the chunk
#pragma unroll
    for (int off = 1; off < WAVE; off <<= 1) {
      const Best os = shfl_up_best(bs, off), oa = shfl_up_best(ba, off);
      if (lane >= off) { take_if_better(bs, os); take_if_better(ba, oa); }
    }
    take_if_better(bs, cs);
    take_if_better(ba, ca);
    if (v && c1 > c1n) {
      // spot first when any spot offering holds n (the F launch rule); the
      // G2 offer rule takes the cheapest of all
      const Best& w = (!q.offer && bs.info >= 0) ? bs : ba;
      // the node's pod capacity is its type's, which may exceed the bracket's
      // c1 when a larger type wins the claim
      const int info = w.info >= 0 ? (w.info | q.cap1t[w.k] << 16) : -1;
      const int hi = min(c1, q.JT - 1);
      for (int n = c1n + 1; n <= hi; ++n) out[n] = make_int2(w.price, info);
    }
    cs = readlane_best(bs, WAVE - 1);
    ca = readlane_best(ba, WAVE - 1);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) jmax = max(jmax, __shfl_xor(jmax, o));
  if (lane == 0) {
    q.jtab[key / q.NW] = jmax;  // identical for every carbon weight of the key
    out[0] = make_int2(0, jmax);
  }
}

namespace {

// ---------------------------------------------------------------------------
// rollout helpers
// ---------------------------------------------------------------------------
// per-lane variant: the value is redefined by the asm, so no load is pending
// on it afterwards (the wait for the load happens here, not at its next use)
__device__ __forceinline__ int opqv(int v) {
  asm volatile("" : "+v"(v));
  return v;
}
__device__ __forceinline__ D1Rule opq_rule(const D1Rule& r) {
  D1Rule o;
  o.sel = opq(r.sel);
  o.n = opq(r.n);
  o.stab_mask = opq(r.stab_mask);
  o._pad = 0;
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    o.type[q] = opq(r.type[q]);
    o.value[q] = opq(r.value[q]);
    o.pmask[q] = opq(r.pmask[q]);
    o.factor[q] = opq(r.factor[q]);
  }
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    o.stab16[w] = opq(r.stab16[w]);
    o.pm16[0][w] = opq(r.pm16[0][w]);
    o.pm16[1][w] = opq(r.pm16[1][w]);
  }
  return o;
}

// convertDesiredReplicasWithBehaviorRate, one direction. The period sums of
// scale-up / scale-down deltas are packed int16 dot products of the delta
// ring (entries 1..8 steps old, i.e. the ring BEFORE this step's push) with
// the policy's period mask.
__device__ __forceinline__ int rate_limit1(const D1Rule& R, bool up, int cur, const uint32_t* del) {
  if (R.sel == CCKA_SELECT_DISABLED) return cur;
  const bool min_sel = R.sel == CCKA_SELECT_MIN;
  long long res = (up == min_sel) ? 0x7fffffffLL : -0x80000000LL;
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    if (q >= R.n) break;
    int added = 0, removed = 0;
    if (R.pmask[q]) {  // wave-uniform
      const short2v z = {0, 0};
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        const short2v d = as_s2(del[w]), m = as_s2((uint32_t)R.pm16[q][w]);
        added = __builtin_amdgcn_sdot2(__builtin_elementwise_max(d, z), m, added, false);
        removed = __builtin_amdgcn_sdot2(__builtin_elementwise_max(z - d, z), m, removed, false);
      }
    }
    const long long pst = (long long)cur - added + removed;
    long long pr;
    if (R.type[q] == CCKA_HPA_PODS) pr = up ? pst + R.value[q] : pst - R.value[q];
    else if (up) pr = (int)ceil((double)pst * R.factor[q]);
    else pr = (int)((double)pst * R.factor[q]);
    res = (up == min_sel) ? min(res, pr) : max(res, pr);
  }
  return (int)res;
}

}  // namespace

// STAMPS: diagnostic build only (never in a real run): per-phase s_memtime
// cycle totals summed over waves into p.stamps[12].
#define D1_STAMP(k)                                          \
  if constexpr (STAMPS) {                                    \
    __builtin_amdgcn_sched_barrier(0);                       \
    const uint64_t now_ = __builtin_amdgcn_s_memtime();      \
    __builtin_amdgcn_sched_barrier(0);                       \
    st_acc[k] += now_ - st_last;                             \
    st_last = now_;                                          \
  }

// ---------------------------------------------------------------------------
// Lane-skewed schedule (DESIGN.md "rollout_d1_kernel"):
// every lane (scenario) keeps its own step counter. Most lane-steps are
// quiet: the HPA keeps the replica count (desired == current, including the
// steps the stabilisation window or maxReplicas hold it) and no node becomes
// ready, no hour / peak-window boundary is crossed and no node becomes a new
// consolidation candidate. A quiet step is the HPA evaluation, the history
// push, the step's energy from cached sums and the trajectory record; a lane
// takes up to D1_S of them per iteration. Any other step is an event: the
// lane stalls and every D1_K iterations the wave runs the full step for all
// stalled lanes together (before that iteration's quiet steps), so the long
// event path runs once for many lanes instead of once per step for the union
// of every lane's events. Per-step constants (node cost, idle energy, pending
// pods, node-minutes) are added lazily at the next event.
//
// Load samples reach the lanes through a per-wave LDS ring of D1_RB trace
// rows (row t, lane l at [t % D1_RB][l]) filled by LDS-DMA
// (global_load_lds_dword, one row = the wave's scenarios at one step), D1_S
// rows per iteration and D1_VMN rows ahead of the lanes; a row is read only
// after D1_VMN younger DMA instructions were issued and `s_waitcnt
// vmcnt(D1_VMN)` retired it (every DMA instruction is one consecutive row).
// The ring is refilled only when every live lane has consumed the rows it
// overwrites.
// ---------------------------------------------------------------------------
constexpr int D1_RB = 64;   // ring rows (power of two)
constexpr int D1_K = 2;     // event cadence (iterations)
constexpr int D1_VMN = 4;   // rows in flight (vmcnt bound; <= 63)
constexpr int D1_S = 8;     // quiet steps per iteration and lane
// rows kept behind the slowest lane: the event step rebuilds the down-window
// records of its quiet steps from them (window <= CCKA_HIST steps)
constexpr int D1_BACK = CCKA_HIST;
// the initial fill (D1_VMN + 4 D1_S rows) plus the rows kept behind must fit,
// and the lanes must be able to spread over a few iterations' worth of rows
static_assert(D1_VMN + 4 * D1_S + D1_BACK <= D1_RB && D1_RB - D1_S - D1_BACK - D1_VMN >= 2 * D1_S,
              "ring too small for the DMA lead");
constexpr int D1_RING_BYTES = D1_RB * WAVE * 4;  // per wave
// Trajectory records go through a buffer resource over the wave's [lanes][T]
// record block (d1_store_rec, d1_common.h).
// wave priority raised outside the event runs (quiet steps and the loop): 4 %
// faster than none in round 3, whatever the level and direction (the gain is
// as much the s_setprio boundaries as the arbitration)
constexpr int D1_PRIO_HI = 3;
__device__ __forceinline__ void d1_dma_row(const int32_t* src, uint32_t lds_row) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dword %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(src), "s"(lds_row)
      : "memory");
}
__device__ __forceinline__ void d1_wait_rows() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(D1_VMN) : "memory"); }
__device__ __forceinline__ void d1_wait_all() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// logical block of dispatch block b among n (a bijection; 8 XCDs)
__device__ __forceinline__ uint32_t xcd_block(uint32_t b, uint32_t n) {
  const uint32_t x = b & 7u, k = b >> 3, q = n >> 3, r = n & 7u;
  return x * q + min(x, r) + k;
}

// NSUB: HPA decisions per step (1, or 4 = the Kubernetes default 15 s sync
// period, SEMANTICS 3.C sub-steps; upstream default behavior only). The down-
// stabilisation records then cover 4 decisions per step: HW packed words.
// HE: down-window records the ring keeps at one decision per step (8, or 4
// when no scenario's window exceeds 300 s: half the ring, rebuild and hold
// loops; launch_rollout_d1 picks it from the scenarios' largest window)
// G3: the DRIFT instantiation with multi-node consolidation (budgets of >= 2
// nodes; its trial copies of the slots would spill in the others)
// KEDA: the deployment is a single-trigger KEDA ScaledObject (SEMANTICS 3.C:
// activation, scale from / to zero after the cooldown, proposal
// ceil(metric / threshold) outside the tolerance band of the current count)
// with the default behavior, one decision per step
template <int MAXN, int MAXP, bool STAMPS, int OCC, bool BDEF, bool DRIFT = false, int NSUB = 1, int HE = 8,
          bool G3 = false, bool KEDA = false>
__global__ void __launch_bounds__(256, OCC) rollout_d1_kernel(D1Params p) {
  static_assert(NSUB == 1 || (NSUB == 4 && BDEF), "15 s sync: lean default path");
  static_assert(!KEDA || (BDEF && NSUB == 1 && !DRIFT), "KEDA: default behavior, one decision per step");
  static_assert(HE == 8 || (HE == 4 && NSUB == 1 && BDEF), "4-record ring: default behavior, one decision per step");
  static_assert(!G3 || (DRIFT && MAXP == 2), "G3: the DRIFT instantiation, two pools");
  constexpr int HW = NSUB == 1 ? HE / 2 : 10;  // history words (2 records each)
  // steps whose records the event step may rebuild: the window's entries
  constexpr int JR = NSUB == 1 ? HE : 5;
  uint64_t st_acc[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t st_last = STAMPS ? __builtin_amdgcn_s_memtime() : 0;
  // LDS: per instance type {idle_nw lo, idle_nw hi, dyn_nw_per_m, alloc_cpu_m}
  // (one ds_read_b128), then the load-sample rings of the block's waves
  extern __shared__ __attribute__((aligned(16))) int4 s_acc[];
  for (int x = threadIdx.x; x < p.K; x += blockDim.x) {
    const long long idle = p.acc[x * 3 + 0];
    s_acc[x] = make_int4((int)(idle & 0xffffffffLL), (int)(idle >> 32), (int)p.acc[x * 3 + 1], (int)p.acc[x * 3 + 2]);
  }
  // LDS copies of the price tiles [R][24][K][Z][2], ci [R][24] and J
  // [R][24][NZI][3] after the rings (launch_rollout_d1 sets lds_tab when they fit)
  const bool ldt = p.lds_tab;
  const uint32_t tab_off = ((uint32_t)p.K * 16u + 255u) / 256u * 256u + (blockDim.x / WAVE) * (uint32_t)D1_RING_BYTES;
  const int n_pr = p.R * 24 * p.K * p.Z * 2;
  const int n_pr8 = (n_pr + 1) & ~1;
  int* const s_price = reinterpret_cast<int*>(reinterpret_cast<char*>(s_acc) + tab_off);
  double* const s_ci = reinterpret_cast<double*>(s_price + n_pr8);
  int* const s_jtab = reinterpret_cast<int*>(s_ci + p.R * 24);
  if (ldt) {
    for (int x = threadIdx.x; x < n_pr; x += blockDim.x) s_price[x] = p.price[x];
    for (int x = threadIdx.x; x < p.R * 24; x += blockDim.x) s_ci[x] = p.ci_gpwmin[x];
    for (int x = threadIdx.x; x < p.R * 24 * p.NZI * 3; x += blockDim.x) s_jtab[x] = p.jtab[x];
  }
  __syncthreads();
  // lanes-per-wave mapping: wave w owns scenarios [w*lpw, (w+1)*lpw)
  const int lane = threadIdx.x & (WAVE - 1);
  // XCD-aware block order: blocks are dealt round-robin to the 8 XCDs, so
  // block b takes the (b / 8)-th block of XCD b % 8's contiguous scenario
  // range; trace rows shared by neighbouring blocks then sit in one XCD's L2
  // (one HBM fetch) instead of two
  const int64_t wv = (int64_t)xcd_block(blockIdx.x, gridDim.x) * (blockDim.x / WAVE) + (threadIdx.x / WAVE);
  const int64_t i = wv * p.lpw + lane;
  if (lane >= p.lpw || i >= p.N) return;  // no cross-lane operations below but ballots

  // ---- per-scenario parameters ----
  const int r = p.region ? (int)p.region[i] : 0;
  // (a KEDA ScaledObject has no utilisation target, and its replica bounds and
  // down window are its own: the scenario's target / max / window overrides
  // are the HPA's)
  const int target = KEDA ? 1 : (p.target ? (int)p.target[i] : p.target0);
  const int mx = KEDA ? opq(p.k_max) : (p.maxr ? (int)p.maxr[i] : p.maxr0);
  const int dwin = (!KEDA && p.down_stab) ? (int)p.down_stab[i] : p.dstab0;
  // records inside the down window: entries k < (W - 1) / sync (o_entries)
  const int nd = min(NSUB == 1 ? __popc(wmask(dwin)) : (dwin > 15 ? (dwin - 1) / 15 : 0), 2 * HW);
  const int dnmask = NSUB == 1 ? wmask(dwin) : 0;
  const int reset_ca = p.reset_ca ? (int)p.reset_ca[i] : p.reset_ca0;
  const int pswitch = p.pswitch ? (int)p.pswitch[i] : p.pswitch0;
  const int wi = p.wci ? (int)p.wci[i] : 0;
  const uint32_t capsel = p.cap_sel ? (uint32_t)p.cap_sel[i] : (uint32_t)p.capsel0;
  // KEDA: the HPA path's minimum is max(minReplicaCount, 1) (0 only by the cooldown)
  const int minr = KEDA ? max(opq(p.k_min), 1) : opq(p.minr), req = opq(p.req_cpu), limit = opq(p.limit);
  // KEDA trigger: threshold per replica, activation, cooldown in steps
  const int kthr = KEDA ? opq(p.k_thr) : 1, kact = KEDA ? opq(p.k_act) : 0, kcds = KEDA ? opq(p.k_cds) : 0;
  const bool kmin0 = KEDA && opq(p.k_min) == 0;
  const float rkthr = __builtin_amdgcn_rcpf((float)kthr);
  // 1-tol <= fl(util/target) <= 1+tol  <=>  ulo <= util <= uhi (fl(u/t) is monotone in u)
  int ulo = max(0, (int)floor(p.tol_lo * (double)target) - 2);
  while ((double)ulo / (double)target < p.tol_lo) ++ulo;
  int uhi = (int)floor(p.tol_hi * (double)target) + 2;
  while ((double)uhi / (double)target > p.tol_hi) --uhi;
  const float rtarget = __builtin_amdgcn_rcpf((float)target);

  // ---- kernel arguments used inside the step loop (opaque register copies) ----
  const int NP = opq(p.NP), NZI = opq(p.NZI), NW = opq(p.NW), JT = opq(p.JT);
  const int maxn = opq(p.maxn), ablate = CCKA_ABLATE_BUILD ? opq(p.ablate) : 0, pdb_member = opq(p.pdb_member);
  const int pdb_pct = opq(p.pdb_pct), slo_util = opq(p.slo_util), delay = opq(p.delay);
  const int base_nodes = opq(p.base_nodes), base_type = opq(p.base_type);
  const int K = opq(p.K), Z = opq(p.Z), T = opq(p.T);
  const int ps = opq(p.peak_start) % 1440, pe = opq(p.peak_end) % 1440;
  const int ps_raw = opq(p.peak_start), pe_raw = opq(p.peak_end);
  const int sm0 = opq(p.start_minute) % 1440;
  const long long base_nw = opq(p.base_nw);
  const GLOBAL_AS int32_t* const price = opq_ptr(p.price);
  const GLOBAL_AS double* const ci_gpwmin = opq_ptr(p.ci_gpwmin);
  const GLOBAL_AS int2* const table = opq_ptr(p.table);
  const GLOBAL_AS int2* const table2 = opq_ptr(p.table2);
  const int drift_on = opq(p.drift_on), replace = opq(p.replace), multi = G3 ? opq(p.multi) : 0;
  const GLOBAL_AS int32_t* const jtab = opq_ptr(p.jtab);
  GLOBAL_AS int4* const traj = opq_ptr(reinterpret_cast<int4*>(p.traj));
  // BDEF: the upstream default behavior as compile-time constants
  const D1Rule rup = [&] { if constexpr (BDEF) return d1_default_rule(true); else return opq_rule(p.up); }();
  const D1Rule rdn = [&] { if constexpr (BDEF) return d1_default_rule(false); else return opq_rule(p.dn); }();
  int budget[MAXP];
#pragma unroll
  for (int q = 0; q < MAXP; ++q) budget[q] = opq(p.budget[q]);

  // ---- NodePools: base spec then RESET (SEMANTICS §1) ----
  int ppol[MAXP], pcas[MAXP], pzi[MAXP], pJ[MAXP];
  uint32_t pcm[MAXP], pmask[MAXP];
#pragma unroll
  for (int q = 0; q < MAXP; ++q) {
    ppol[q] = 0; pcas[q] = 0; pzi[q] = -1; pcm[q] = 0; pJ[q] = 0; pmask[q] = 0;
    if (q < NP) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const D1Patch& x = p.patch[q][s];
        if (x.policy) ppol[q] = x.policy;
        if (x.cas >= 0) pcas[q] = s == 1 ? (reset_ca + CCKA_STEP_SECONDS - 1) / CCKA_STEP_SECONDS : x.cas;
        if (x.zi >= 0) pzi[q] = x.zi;
        if (x.cm) pcm[q] = (uint32_t)x.cm;
      }
    }
  }

  // consolidateAfter (steps) of a slot's pool: explicit selects on the pool
  // bits (an indexed pcas[] would be demoted to scratch memory), clamped to
  // 0xFFFF (with T <= 65535 a larger value never makes a node consolidatable
  // either). Each slot keeps its pool's value in scas[] and its
  // consolidatable-from step slc = last pod event + scas; it is a
  // consolidation candidate iff it is ready and slc <= t.
  auto cas_of = [&](uint32_t info) {
    const int m1 = -(int)(info >> 13 & 1u), m2 = -(int)(info >> 14 & 1u);
    const int lo = pcas[0] ^ ((pcas[0] ^ pcas[MAXP > 1 ? 1 : 0]) & m1);
    if constexpr (MAXP <= 2) {
      return lo;
    } else {
      const int hi = pcas[2] ^ ((pcas[2] ^ pcas[3]) & m1);
      return lo ^ ((lo ^ hi) & m2);
    }
  };
  auto casc = [](int c) { return min(c, 0xFFFF); };

  // ---- node slots (register arrays, fully unrolled loops) ----
  // Fields of a free slot are stale: every use is masked by `used` (or by
  // `rdy` / the candidate masks, subsets of it), except sallocr, which is
  // zero on every slot that is not ready (accounting reads it unmasked).
  uint32_t sinfo[MAXN];  // type | zone<<10 | cap<<12 | pool<<13
  int sready[MAXN], slc[MAXN], scas[MAXN], spods[MAXN], sprice[MAXN], scap[MAXN];
  uint32_t sdyn[MAXN];  // dyn_nw_per_m of the slot's type (SEMANTICS §3.H)
  int salloc[MAXN];     // alloc_cpu_m of the slot's type (< 2^24 by eligibility)
  int sallocr[MAXN];    // salloc once the node is ready, else 0 (read through alloc_ready)
#pragma unroll
  for (int n = 0; n < MAXN; ++n) {
    sinfo[n] = 0; sready[n] = 0; slc[n] = 0; scas[n] = 0; spods[n] = 0; sprice[n] = 0; scap[n] = 0;
    sdyn[n] = 0; salloc[n] = 0; sallocr[n] = 0;
  }
  uint32_t used = 0, rdy = 0, cmask = 0;  // cmask: slot capacity type matches the nodeSelector
  // allocatable CPU of slot n if ready, else 0: the one-decision-per-step
  // instantiations keep it in sallocr (deriving it measured 1-8 % slower
  // there, DRIFT included); the 15 s-sync and G3 ones derive it from `rdy`, so
  // sallocr is dead there (8 registers: spills 80 -> 44 B and 44 -> 16 B, the
  // upstream-defaults line 2.90 -> 2.61 ms; G3 320 -> 248 B, 7.41 -> 5.72 ms)
  // per-slot dynamic power and allocatable CPU of the slot's type: the G3
  // instantiation reads them from the LDS catalog (event paths only) instead
  // of keeping sdyn[] / salloc[] (16 registers: spill 160 -> 0 B, 244 -> 12 B
  // with 15 s sync; the multi-node consolidation line 4.50 -> 3.45 ms)
  auto dyn_of = [&](int n) -> uint32_t {
    if constexpr (G3) return (uint32_t)s_acc[sinfo[n] & 1023u].z;
    else return sdyn[n];
  };
  auto alloc_of = [&](int n) -> int {
    if constexpr (G3) return s_acc[sinfo[n] & 1023u].w;
    else return salloc[n];
  };
  constexpr bool kAllocR = NSUB == 1 && !G3;
  auto alloc_ready = [&](int n) -> uint32_t {
    if constexpr (kAllocR) return (uint32_t)sallocr[n];
    else return (rdy >> n & 1u) ? (uint32_t)alloc_of(n) : 0u;
  };
  // consolidateAfter (steps) of slot n's pool: the G3 instantiation derives it
  // from the pool bits instead of keeping scas[] (8 more registers: its spill
  // 248 -> 160 B, the multi-node consolidation line 5.69 -> 4.44 ms; in the
  // 15 s-sync + DRIFT one the same change measured 2 % slower)
  auto cas_slot = [&](int n) -> int {
    if constexpr (G3) return casc(cas_of(sinfo[n]));
    else return scas[n];
  };
  // DRIFT (SEMANTICS 3.G0): drifted slots, sources of an in-flight pre-spun
  // replacement and those replacements (tainted karpenter.sh/disrupted: no
  // pods placed on them, no consolidation; a replacement's source is
  // 1 + slot in sinfo bits 16..20)
  uint32_t dmask = 0, srcm = 0, repm = 0;
  auto taint = [&]() -> uint32_t { return DRIFT ? (srcm | repm) : 0u; };
  // slots of on-demand nodes (G2 candidates are on-demand)
  auto od_slots = [&]() {
    uint32_t m = 0;
#pragma unroll
    for (int n = MAXN - 1; n >= 0; --n) m = 2 * m + (sinfo[n] >> 12 & 1u);
    return m & used;
  };
  const uint32_t slot_mask = maxn >= 32 ? 0xFFFFFFFFu : ((1u << maxn) - 1u);

  int replicas = p.replicas0, placed = 0, rpods = 0;
  // HPA history, packed int16, entry k = k+1 steps old at decision time:
  // recommendations with invalid entries stored as the neutral element of the
  // max (hdn) and of the min (hup), and scale deltas. With the default
  // behavior only the down window reads history (no up window, 15 s periods).
  uint32_t hdn[HW], hup[4], hdel[4] = {0, 0, 0, 0};
  uint32_t dn16[HW];  // this scenario's down-stabilisation window as packed lane masks
#pragma unroll
  for (int w = 0; w < 4; ++w) hup[w] = 0x7FFF7FFFu;
#pragma unroll
  for (int w = 0; w < HW; ++w) {
    hdn[w] = 0x80008000u;
    dn16[w] = (2 * w < nd ? 0xFFFFu : 0u) | (2 * w + 1 < nd ? 0xFFFF0000u : 0u);
  }
  int next_ready = 0x7fffffff, nsp = 0, nod = 0;
  // KEDA: the cooldown runs out at kcd (the last active step + the cooldown;
  // last_active = 0 initially); the current replica count's tolerance band of
  // the metric: proposal = cur exactly on [q_klo, q_khi]
  int kcd = kcds, q_klo = 0, q_khi = -1, kb_cur = -1;
  bool q_kcd = false;  // the quiet steps must check the cooldown (replicas > 0, minReplicaCount 0)
  bool k_act_step = false;  // the step's trigger activity (the SLO reads it)
  // within(r), r = double(L) / (double(threshold) * double(cur)), is monotone
  // in L: the band's ends by the binary64 test itself around an estimate
  auto keda_band = [&](int cur) {
    if (!KEDA || cur == kb_cur) return;
    kb_cur = cur;
    if (cur <= 0) { q_klo = 0; q_khi = -1; return; }
    const double D = (double)kthr * (double)cur;
    long long lo = max((long long)floor(p.tol_lo * D) - 2, -1LL);
    while ((double)lo / D < p.tol_lo) ++lo;
    long long hi = (long long)floor(p.tol_hi * D) + 2;
    while ((double)hi / D > p.tol_hi) --hi;
    q_klo = (int)min(lo, 0x7fffffffLL);
    q_khi = (int)min(hi, 0x7ffffffeLL);
  };
  keda_band(p.replicas0);
  // free pod capacity of the compatible ready slots (kept incrementally)
  int Ffree = 0;
  // smallest pod capacity of any node launched so far (refreshed on deletion):
  // an under-utilised node can only be deleted when F >= its capacity
  int minscap = 0x7fffffff;
  int profile = -1, hour = -1;
  long long cost = 0, burn = 0, base_price = 0;
  int pend_min = 0;  // <= 32767 pods x T steps
  long long energy_nw = 0, e_hour = 0, Isum = 0;  // exact nanowatt-minutes; Isum: idle draw of used slots
  double gco2 = 0.0, ci_min = 0.0;
  int slo = 0, nmin_spot = 0, nmin_od = 0, launches = 0, deletions = 0, peak_nodes = 0;
  uint32_t last_choice = 0xFFFFFFFFu, hash = 2166136261u;

  // quiet-step caches, refreshed at the end of every event step
  unsigned long long Ssum = 0;  // sum over ready slots of dyn_nw_per_m * pods
  float Rmax = 0.f;             // max over ready slots of pods/alloc
  float q_rbd = 0.f, q_rbc = 0.f, q_rbp = 0.f;  // 1/(ready*req), 1/(cur*req), 1/ready pods
  bool q_peak = false;
  int q_rcap = 0;               // usage cap (ready*limit, or INT_MAX without a limit)
  int q_hold = -0x40000000;     // the down window holds a record >= cur up to this step
  (void)dnmask;
  // steps a record >= cur holds the replica count for (every decision of a
  // later step must see it: (nd - (NSUB - 1)) / NSUB whole steps), and the
  // steps whose records the event step rebuilds (they reach nd entries back)
  const int wl = NSUB == 1 ? nd : max(0, (nd - (NSUB - 1)) / NSUB);
  const int wr = NSUB == 1 ? nd : (nd + NSUB - 1) / NSUB;
  // LEAN 2 quiet step (default behavior): the HPA outcome of a quiet step is a
  // pair of integer compares on the step's usage. Between two event steps the
  // replica count, the ready pods and the node set are constant, so the
  // proposal is a monotone step function of usage and the step is quiet iff
  //   usage < q_ulim            (proposal <= cur, or any proposal at maxReplicas;
  //                              and usage < 2^20, the exact range of upp below)
  //   usage >= q_pge || t <= q_hold   (proposal >= cur, or a record >= cur is
  //                              still inside the down-stabilisation window)
  // The records themselves are not pushed: the next event step rebuilds the
  // ones inside the window from the trace rows still in the LDS ring. The
  // step's dynamic energy Ssum * upp is accumulated as sum(upp) and charged at
  // the next flush; SLO is usage >= q_slo.
  int q_ulim = 0, q_pge = 0, q_slo = 0, q_usat = 0, q_w0 = 0, q_w1 = 0, q_pendv = 0, q_nodes = 0;
  float q_hbp = 0.f;   // 0.5 / ready pods (upp = (usage + 0.5) / ready pods, truncated)
  uint32_t usum = 0;   // sum of upp over the quiet steps since the last flush
  bool q_met = false;  // the HPA has a metric (records are proposals, else invalid)

  auto refresh_J = [&](int rh) {
#pragma unroll
    for (int q = 0; q < MAXP; ++q) {
      const uint32_t cm = pcm[q] & capsel;
      const int64_t ji = ((int64_t)rh * NZI + pzi[q]) * 3 + (cm - 1);
      pJ[q] = (q < NP && cm && pzi[q] >= 0) ? (ldt ? s_jtab[ji] : jtab[ji]) : 0;
    }
  };

  // ---- C. HPA (replica_calculator.go + horizontal.go, SEMANTICS §3.C) ----
  // Evaluated without side effects (the history push is hpa_commit):
  // util = int32(usage*100 / (ready*req)) by an f32-reciprocal division with
  // an exact remainder correction; the tolerance band, the unready rule and
  // the SLO threshold are integer tests on util (exactly the binary64 tests
  // of the spec, see ulo/uhi). The proposal ceil(fl(fl(u/target)*base))
  // equals the exact integer ceiling unless u*base is a multiple of target
  // (|rounding error| < 1/target otherwise); only that case, and inputs
  // beyond the fast arithmetic's range, run the spec's expression (rare
  // branches). Then the stabilisation (packed min / max over the records
  // inside each window) and the rate limits; desired == cur exactly when
  // proposal == cur.
  struct HpaOut {
    int util, proposal, desired;
    bool ran, hpa_path;
  };
  // steps 4-5 for a decision that produced a proposal: the stabilisation
  // (packed min / max over the records inside each window), the rate limits
  // and the [minr, mx] clamp
  auto behave = [&](int proposal, int cur) -> int {
    int upr = proposal, dnr = proposal;
    if (rup.stab_mask) {  // wave-uniform
      short2v a = as_s2(bfi((uint32_t)rup.stab16[0], hup[0], 0x7FFF7FFFu));
#pragma unroll
      for (int w = 1; w < 4; ++w)
        a = __builtin_elementwise_min(a, as_s2(bfi((uint32_t)rup.stab16[w], hup[w], 0x7FFF7FFFu)));
      upr = min(upr, min((int)a.x, (int)a.y));
    }
    {
      short2v a = as_s2(bfi(dn16[0], hdn[0], 0x80008000u));
#pragma unroll
      for (int w = 1; w < HW; ++w) a = __builtin_elementwise_max(a, as_s2(bfi(dn16[w], hdn[w], 0x80008000u)));
      dnr = max(dnr, max((int)a.x, (int)a.y));
    }
    const int rc = min(max(cur, upr), dnr);
    int lo = minr, hi = mx;
    if constexpr (BDEF) {
      // up: max(Percent 100 -> ceil(2.0*cur), Pods 4 -> cur+4) over 15 s
      // periods (no 60 s history inside), never below cur; down: Percent 100
      // -> int(cur*0.0) = 0, never above cur
      hi = rc > cur ? min(hi, max(2 * cur, cur + 4)) : hi;
      lo = rc < cur ? max(lo, 0) : lo;
    } else {
      if (proposal != cur) {
        if (rc > cur) hi = min(hi, max(rate_limit1(rup, true, cur, hdel), cur));
        else if (rc < cur) lo = max(lo, min(rate_limit1(rdn, false, cur, hdel), cur));
      }
    }
    return rc < lo ? lo : (rc > hi ? hi : rc);
  };
  auto hpa_eval = [&](int L, int cur, int ready, float rbd, float rbc) -> HpaOut {
    HpaOut o;
    const bool metric = cur <= mx && cur >= minr && ready > 0 && !(cur == 0 && minr != 0);
    int util = 0, proposal = cur;
    {
      const int rcapv = ready * limit;  // limit <= 65535 (d1_check_world)
      const int usage = (limit > 0 && rcapv < L) ? rcapv : L;
      const int a = usage * 100;
      const int dreq = ready * req;     // < 2^31: ready <= 32767, req <= 65535
      const int dcur = cur * req;
      bool slow = usage < 0 || usage > 21474836;
      util = fdiv_nb(a, dreq, rbd, slow);
      int nu = 0;
      if (cur > ready) nu = fdiv_nb(a, dcur, rbc, slow);
      if (__builtin_expect(metric && slow, 0))  // exact 64-bit quotient
        util = (int)(((long long)usage * 100) / ((long long)ready * req));
      const bool unready_up = cur > ready && util > target;  // ratio > 1 <=> util > target
      int u = util, base = ready;
      if (unready_up) { u = nu; base = cur; }  // every replica counted, unready ones idle
      if (__builtin_expect(metric && slow && unready_up, 0))
        u = (int)(((long long)usage * 100) / ((long long)cur * req));
      const bool keep = (u >= ulo && u <= uhi) || (unready_up && u < target);  // within || nr < 1
      bool slow2 = (uint32_t)u > 0xFFFFu;
      const int x = u * base;  // < 2^31 when u <= 0xFFFF
      const int q = fdiv_nb(x, target, rtarget, slow2);
      const bool exactm = x == q * target;
      int c = q + (exactm ? 0 : 1);
      if (__builtin_expect(metric && !keep && (exactm || slow2), 0))  // binary64 as the spec writes it
        c = (int)ceil(((double)u / (double)target) * (double)base);
      const int pe2 = unready_up ? max(cur, c) : c;
      proposal = (metric && !keep) ? pe2 : cur;
    }
    o.util = util;
    o.proposal = proposal;
    o.ran = metric;
    o.hpa_path = !(cur == 0 && minr != 0);
    int desired = cur > mx ? mx : (cur < minr && o.hpa_path ? minr : cur);
    if (metric && !ablated(ablate, 8)) desired = behave(proposal, cur);
    o.desired = desired;
    return o;
  };
  // KEDA (SEMANTICS 3.C): activity, scale from / to zero, then the HPA steps
  // 1, 4, 5, 6 on the proposal ceil(L / threshold) outside the band
  auto keda_eval = [&](int L, int cur, int ts) -> HpaOut {
    HpaOut o{};
    const bool act = L > kact;
    const bool cool = !act && kmin0 && ts >= kcd;
    if (act) kcd = ts + kcds;
    k_act_step = act;
    o.util = 0;
    o.proposal = cur;
    o.ran = false;
    o.hpa_path = false;
    int desired = cur;
    if (cur == 0) {
      desired = act ? 1 : 0;
    } else if (cool) {
      desired = 0;
    } else {
      o.hpa_path = true;
      if (cur > mx) {
        desired = mx;
      } else if (cur < minr) {
        desired = minr;
      } else {
        int prop = cur;
        if (L < q_klo || L > q_khi) {
          // int32(ceil(double(L) / double(threshold))) is the exact integer
          // ceiling for 0 <= L and threshold < 2^22 (d1_check_world)
          bool slow = L < 0;
          const int q = fdiv_nb(max(L, 0), kthr, rkthr, slow);
          prop = q + (q * kthr != L ? 1 : 0);
          if (__builtin_expect(slow, 0)) prop = (int)ceil((double)L / (double)kthr);
        }
        o.proposal = prop;
        o.ran = true;
        desired = ablated(ablate, 8) ? cur : behave(prop, cur);
      }
    }
    o.desired = desired;
    return o;
  };
  // records clamp to int16 (replicas stay in [0, 32767]; min/max commute with clamping)
  auto hpa_commit = [&](const HpaOut& h, int cur) {
    const int rv = min(max(h.proposal, -D1_REC_SAT - 1), D1_REC_SAT);
    ring_push<HW>(hdn, h.ran ? rv : (int)0x8000);
    if constexpr (!BDEF) {
      ring_push(hup, h.ran ? rv : 0x7FFF);
      ring_push(hdel, (h.hpa_path && h.desired != cur) ? h.desired - cur : 0);
    }
  };
  // ---- H. per-node energy (SEMANTICS §3.H, exact integer nanowatt-minutes) ----
  // use = min(pods * upp, alloc) with sallocr = 0 on nodes not ready; pods <
  // 2^15 and upp < 2^16 keep every product in 32 bits (all operands uint32:
  // a mixed int/unsigned min() resolves to the double overload)
  auto upp_of = [&](int L, float rbp) {
    const int rcapv = rpods * limit;
    const int usage = max((limit > 0 && rcapv < L) ? rcapv : L, 0);
    bool slow = false;
    int upp = fdiv_nb(usage, max(rpods, 1), rbp, slow);
    if (__builtin_expect(slow, 0)) upp = usage / max(rpods, 1);
    return rpods > 0 ? upp : 0;
  };
  auto dyn_energy = [&](int upp) -> long long {
    if (__builtin_expect(upp <= 0xFFFF, 1)) {
      unsigned long long ed = 0;
#pragma unroll
      for (int n = 0; n < MAXN; ++n) {
        const uint32_t use = min((uint32_t)spods[n] * (uint32_t)upp, alloc_ready(n));  // both uint32: v_min_u32
        ed += (unsigned long long)dyn_of(n) * use;
      }
      return (long long)ed;
    }
    long long e = 0;
#pragma unroll
    for (int n = 0; n < MAXN; ++n) {
      const uint64_t prod = (uint64_t)(uint32_t)spods[n] * (uint64_t)(uint32_t)upp;
      const uint32_t al = alloc_ready(n);
      const uint32_t use = prod < (uint64_t)al ? (uint32_t)prod : al;
      e += (long long)((uint64_t)dyn_of(n) * use);
    }
    return e;
  };

  // ---- scheduler state ----
  int t = 0;      // this lane's next step
  int nxt = 0;    // first step that must take the event path (the first step always does)
  int npb = 0;    // next peak-window boundary step (pswitch lanes)
  int tq = 0;     // steps [tq, t) were quiet: their per-step constants are added at the next flush
  bool stall = false;
  // per-step constants of the quiet steps since the last event (SEMANTICS §3.H)
  auto flush = [&](int upto) {
    const int n = upto - tq;
    cost += (burn + base_price) * (long long)n;
    e_hour += (base_nw + Isum) * (long long)n;
    if constexpr (BDEF) {  // dynamic energy of the quiet steps (exact integers)
      e_hour += (long long)(Ssum * (unsigned long long)usum);
      usum = 0;
    }
    pend_min += (replicas - rpods) * n;
    nmin_spot += nsp * n;
    nmin_od += nod * n;
    tq = upto;
  };

  // load column: the scenario's own trace, or its shared trace (policy
  // sweeps); per-scenario traces are read wave-tiled when the host built that
  // copy (the wave's rows contiguous: no 128-B line shared with another wave)
  const int64_t wtb = [&] {  // the wave's first scenario (wave-uniform)
    const int64_t x = wv * p.lpw;
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(x >> 32));
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(x & 0xffffffffLL));
    return (int64_t)(((uint64_t)hi << 32) | lo);
  }();
  const int32_t* lp = p.load_w ? p.load_w + wtb * T + lane
                               : p.load + (p.trace_mod > 0 ? (p.first_id + i) % p.trace_mod : i);
  const long long lsl = opq(p.load_w ? (long long)p.lpw : (long long)p.NL);  // tiled rows: lpw wide (the last wave padded)
  // load-sample ring of this wave
  const uint32_t ring_off = (uint32_t)__builtin_amdgcn_readfirstlane(
      (int)(((uint32_t)p.K * 16u + 255u) / 256u * 256u + (threadIdx.x / WAVE) * (uint32_t)D1_RING_BYTES));
  // LDS byte address (the low word of the generic address of an LDS object)
  const uint32_t ring_lds = (uint32_t)(uintptr_t)s_acc + ring_off;
  const int* const ring = reinterpret_cast<const int*>(reinterpret_cast<const char*>(s_acc) + ring_off);
  // ring geometry (wave-uniform): rbn rows of rsw lanes; row of step x = x mod rbn
  constexpr int rsw = WAVE, rbn = D1_RB;
  auto rrow = [&](int x) { return x & (D1_RB - 1); };
  // ring index of (row r, this lane)
  auto ridx = [&](int r) { return r * rsw + lane; };
  // row r + q (0 <= q < rbn) wrapped
  auto rnext = [&](int r, int q) { return (r + q) & (D1_RB - 1); };
  int tf = 0;   // trace rows issued (wave-uniform)
  int tfr = 0;  // tf mod rbn (wave-uniform)
  const int32_t* lpf = lp;  // this lane's sample of row tf
  auto tf_adv = [&]() {
    ++tf;
    ++tfr;
    if (tfr == rbn) tfr = 0;
    lpf += lsl;
  };
  {
    const int n0 = min(T, D1_VMN + 4 * D1_S);
    while (tf < n0) {
      d1_dma_row(lpf, (uint32_t)__builtin_amdgcn_readfirstlane((int)(ring_lds + (uint32_t)tfr * (uint32_t)(rsw * 4))));
      tf_adv();
    }
    d1_wait_all();
  }
  int t_rdy = tf;  // rows < t_rdy have landed (wave-uniform)
  bool pf_ok = false;
  bool qadv = true;  // some lane stepped quietly in the last iteration (wave-uniform)
  int Lpf[D1_S];
#pragma unroll
  for (int q = 0; q < D1_S; ++q) Lpf[q] = 0;
  // trajectory records scenario-major on the device ([N][T]: a lane's records
  // are contiguous, so its consecutive steps fill whole lines however far the
  // lanes drift apart); ccka_get_trajectory returns them [T][N]
  const int64_t w0 = wtb;
  const int wlanes = (int)min((int64_t)p.lpw, p.N - w0);
  const __amdgpu_buffer_rsrc_t trs = __builtin_amdgcn_make_buffer_rsrc(
      traj ? (void*)(reinterpret_cast<int4*>(p.traj) + w0 * T) : (void*)p.load, 0, traj ? wlanes * T * 16 : 0,
      0x00020000);
  const int lb = lane * T * 16;  // this lane's record of step t at byte lb + 16 t

  for (int it = 0;; ++it) {
    const bool live = t < T;
    if (__ballot(live) == 0) break;  // wave-uniform
    d1_wait_rows();
    t_rdy = max(t_rdy, tf - D1_VMN);
    // ---- event steps of the stalled lanes: every D1_K iterations, or when no
    // lane stepped quietly in the last one. They run before this iteration's
    // quiet steps, so their loads do not wait for this iteration's records
    // (every load waits for all older memory operations), and a lane leaves
    // its event step straight into quiet steps ----
    const uint64_t sb = __ballot(stall);
    if constexpr (STAMPS) st_acc[9] += 1;
    if (sb != 0 && (it % D1_K == D1_K - 1 || !qadv)) {
      __builtin_amdgcn_s_setprio(0);
      if constexpr (STAMPS) { st_acc[10] += 1; st_acc[11] += __popcll(sb); }
      // the event step in phases, each a block over the stalled lanes (the
      // wave-uniform points between them carry the diagnostic stamps)
      const bool ev = stall;
      int L = 0, minute = 0, rh = 0, pd = 0, step_last_type = 0xFFFF;
      int4 rec;
      uint32_t flags = 0;
      bool g_acted = false, hchg = false, jchg = false;
      uint32_t emp_e = 0, weou_e = 0;  // empty slots / WhenEmptyOrUnderutilized slots after disruption
      HpaOut hp{};
      if (ev) {
        stall = false;
        const int tr = rrow(t);
        L = ring[ridx(tr)];
        if constexpr (BDEF) {
          // the down-window records of the quiet steps [tq, t), oldest first,
          // from their trace rows (the ring keeps >= 8 rows behind every lane)
          // and the state they ran with. A record >= cur is stored as cur: the
          // default behavior only ever compares it with a proposal and with cur
          // (<= maxReplicas), so its excess over cur never changes a decision.
          const int kq = min(t - tq, wr);
          if (kq > 0) {
            // entry j of the rebuilt window = the record of step t-1-j (j < kq);
            // the rows' samples are read first (independent LDS reads), held
            // proposals are computed only in waves where some lane has one
            const int cur16 = min(replicas, D1_REC_SAT);
            int us[JR], rv[JR];
            bool anylow = false;
#pragma unroll
            for (int j = 0; j < JR; ++j) {
              us[j] = KEDA ? ring[ridx(rnext(tr, rbn - 1 - j))] : min(ring[ridx(rnext(tr, rbn - 1 - j))], q_rcap);
              rv[j] = q_met ? cur16 : (int)0x8000;
              anylow |= (j < kq) & q_met & (us[j] < q_pge);
            }
            if (KEDA && anylow) {
              // held below cur (KEDA): the proposal ceil(L / threshold) < cur,
              // an exact integer ceiling (0 <= L < 2^20)
#pragma unroll
              for (int j = 0; j < JR; ++j) {
                bool sl = false;
                const bool low = (j < kq) & q_met & (us[j] < q_pge);
                const int q = fdiv_nb(max(us[j], 0), kthr, rkthr, sl);
                rv[j] = low ? min(q + (q * kthr != us[j] ? 1 : 0), D1_REC_SAT) : rv[j];
              }
            } else if (anylow) {
              // held below cur: util < ulo <= target, so no unready rule and the
              // proposal is ceil(util * ready / target) (binary64 at an exact
              // multiple, as the spec writes it); us < 2^20 and util < 2^15 keep
              // both f32 quotients exact after one correction
              const int dreq = rpods * req;
              const float rbd = __builtin_amdgcn_rcpf((float)dreq);
              bool anyex = false;
#pragma unroll
              for (int j = 0; j < JR; ++j) {
                bool sl = false;
                const bool low = (j < kq) & q_met & (us[j] < q_pge);
                const int util = fdiv_nb(us[j] * 100, dreq, rbd, sl);
                const int x = (int)__umul24((uint32_t)util, (uint32_t)rpods);
                const int q = fdiv_nb(x, target, rtarget, sl);
                const bool ex = x == q * target;
                anyex |= low & ex;
                rv[j] = low ? min(q + (ex ? 0 : 1), D1_REC_SAT) : rv[j];
                us[j] = (low & ex) ? util : -1;  // exact multiples: the spec's binary64 below
              }
              if (__builtin_expect(anyex, 0)) {
#pragma unroll
                for (int j = 0; j < JR; ++j)
                  if (us[j] >= 0)
                    rv[j] = min((int)ceil(((double)us[j] / (double)target) * (double)rpods), D1_REC_SAT);
              }
            }
#pragma unroll
            for (int j = JR - 1; j >= 0; --j)
              if (j < kq) {
                if constexpr (NSUB == 1) ring_push<HW>(hdn, rv[j]);
                else ring_push4<HW>(hdn, rv[j]);  // the step's NSUB equal records
              }
          }
        }
        flush(t);
        minute = (sm0 + t) % 1440;
        const int h = minute / 60;
        rh = r * 24 + h;
        if (h != hour) {  // this hour's prices and carbon intensity
          if (hour >= 0) {
            gco2 += (double)e_hour * (ci_min * 1e-9);  // carbon of the hour that ended
            energy_nw += e_hour;
          }
          e_hour = 0;
          hour = h;
          hchg = true;  // prices, carbon intensity and J are loaded before provisioning
        }
      }
      D1_STAMP(2);
      if (ev) {
        // ---- B. readiness ----
        if (t >= next_ready) {
          next_ready = 0x7fffffff;
#pragma unroll
          for (int n = 0; n < MAXN; ++n) {
            if ((used & ~rdy) >> n & 1u) {
              if (sready[n] <= t) {
                rdy |= 1u << n;
                rpods += spods[n];
                sallocr[n] = salloc[n];
                if ((cmask & ~taint()) >> n & 1u) Ffree += scap[n] - spods[n];
              }
              else next_ready = min(next_ready, sready[n]);
            }
          }
        }
        // ---- A. profile ----
        const bool in_win = ps_raw <= pe_raw ? (minute >= ps_raw && minute < pe_raw)
                                             : (minute >= ps_raw || minute < pe_raw);
        const bool peak = pswitch && in_win;
        const int prof = peak ? CCKA_PROFILE_PEAK : CCKA_PROFILE_OFFPEAK;
        if (peak) flags |= 1u;
        q_peak = peak;
        if (prof != profile) {
          profile = prof;
          int pold[MAXP];
#pragma unroll
          for (int q = 0; q < MAXP; ++q) pold[q] = pcas[q];
#pragma unroll
          for (int q = 0; q < MAXP; ++q) {
            if (q >= NP) break;
            const D1Patch& x = p.patch[q][prof + 1];
            if (x.policy) ppol[q] = x.policy;
            if (x.cas >= 0) pcas[q] = x.cas;
            if (x.zi >= 0) pzi[q] = x.zi;
            if (x.cm) pcm[q] = (uint32_t)x.cm;
          }
          // consolidateAfter may have changed: per-slot copies and thresholds
#pragma unroll
          for (int n = 0; n < MAXN; ++n)
            if (used >> n & 1u) {
              const int c = casc(cas_of(sinfo[n]));
              if constexpr (G3) {
                const int m1 = -(int)(sinfo[n] >> 13 & 1u);
                // the slot's value before this switch (G3 instantiations have MAXP = 2)
                const int o = pold[0] ^ ((pold[0] ^ pold[MAXP > 1 ? 1 : 0]) & m1);
                slc[n] += c - casc(o);
              } else {
                slc[n] += c - scas[n];
              }
              scas[n] = c;
            }
          jchg = true;
          if (DRIFT && drift_on) {  // the pools' requirements moved: which nodes left them
            uint32_t dm = 0;
#pragma unroll
            for (int n = 0; n < MAXN; ++n) {
              const uint32_t x = sinfo[n];
              uint32_t zm = 0, cm = 0;
#pragma unroll
              for (int q = 0; q < MAXP; ++q)
                if ((int)(x >> 13 & 3u) == q) { zm = pzi[q] >= 0 ? p.zml[pzi[q]] : 0u; cm = pcm[q]; }
              const bool drifted = !(zm >> (x >> 10 & 3u) & 1u) || !(cm & capbit1((int)(x >> 12 & 1u)));
              dm |= ((used >> n & 1u) && drifted ? 1u : 0u) << n;
            }
            dmask = dm;
          }
        }

      }
      D1_STAMP(3);
      if (ev) {
        // ---- C. HPA ----
        // NSUB decisions on the step's metric sample (the ready pods do not
        // change between them: the ReplicaSet acts after the last)
#pragma unroll
        for (int sub = 0; sub < NSUB; ++sub) {
          const int cur = replicas;
          if constexpr (KEDA) hp = keda_eval(L, cur, t);
          else
            hp = hpa_eval(L, cur, rpods, __builtin_amdgcn_rcpf((float)(rpods * req)),
                          __builtin_amdgcn_rcpf((float)(cur * req)));
          hpa_commit(hp, cur);
          replicas = hp.desired;
        }

        // ---- D. ReplicaSet reconcile (nominated first, then running; high slot first) ----
        if (placed > replicas) {
          int excess = placed - replicas;
          placed = replicas;
#pragma unroll
          for (int pass = 0; pass < 2; ++pass) {
            const uint32_t m = pass == 0 ? (used & ~rdy) : rdy;
            if (!m || excess <= 0) continue;  // skipped by the wave when no lane needs the pass
            int removed = 0, removed_c = 0;
#pragma unroll
            for (int n = MAXN - 1; n >= 0; --n) {  // branch-free: k = 0 leaves the slot untouched
              const int k = (m >> n & 1u) ? min(spods[n], excess) : 0;
              spods[n] -= k;
              excess -= k;
              removed += k;
              if (pass == 1) removed_c += ((cmask & ~taint()) >> n & 1u) ? k : 0;
              slc[n] = k > 0 ? t + cas_slot(n) : slc[n];
            }
            if (pass == 1) { rpods -= removed; Ffree += removed_c; }
          }
        }
        // ---- E. kube-scheduler (ready slots) / F1. nomination (in-flight slots) ----
        pd = replicas - placed;
        if (pd > 0) {
#pragma unroll
          for (int pass = 0; pass < 2; ++pass) {
            const uint32_t m = (pass == 0 ? rdy : (used & ~rdy)) & cmask & ~taint();
            if (!m || pd <= 0) continue;  // skipped by the wave when no lane needs the pass
            int added = 0;
#pragma unroll
            for (int n = 0; n < MAXN; ++n) {  // branch-free first fit
              const int fr = (m >> n & 1u) ? scap[n] - spods[n] : 0;
              const int k = min(fr, pd);  // fr, pd >= 0
              spods[n] += k;
              pd -= k;
              added += k;
              slc[n] = k > 0 ? t + cas_slot(n) : slc[n];
            }
            placed += added;
            if (pass == 0) { rpods += added; Ffree -= added; }
          }
        }
      }
      D1_STAMP(4);
      if (ev) {
        // ---- the hour's prices and carbon intensity, the pools' J: loaded only
        // here, after the phases that do not read them, since every load
        // waits for all older memory operations (this iteration's records) ----
        if (hchg) {
          const int64_t toff = (int64_t)rh * K * Z * 2;
          const GLOBAL_AS int32_t* tile = price + toff;
          const int* stile = s_price + toff;
          ci_min = ldt ? s_ci[rh] : ci_gpwmin[rh];
          base_price = (long long)base_nodes * (ldt ? stile[(base_type * Z) * 2 + 1] : tile[(base_type * Z) * 2 + 1]);
          burn = 0;
          // every slot's price in flight at once (unused slots read entry 0)
          int np[MAXN];
#pragma unroll
          for (int n = 0; n < MAXN; ++n) {
            const uint32_t x = sinfo[n];
            const int e = ((int)(x & 1023u) * Z + (int)(x >> 10 & 3u)) * 2 + (int)(x >> 12 & 1u);
            np[n] = ldt ? stile[e] : tile[e];
          }
#pragma unroll
          for (int n = 0; n < MAXN; ++n) {
            if (used >> n & 1u) {
              sprice[n] = np[n];
              burn += np[n];
            }
          }
        }
        if (hchg || jchg) refresh_J(rh);
        // ---- F2. Karpenter provisioning: claims of min(J, pending) pods ----
        {
          uint32_t fm = ~used & slot_mask;
          if (pd > 0 && fm && !ablated(ablate, 2)) {
            int q = -1, J = 0, zq = 0, cq = 0;
            uint32_t cm = 0;
#pragma unroll
            for (int qq = MAXP - 1; qq >= 0; --qq) {  // first pool in Karpenter order
              const uint32_t c = pcm[qq] & capsel;
              if (qq < NP && c && pJ[qq] > 0) { q = qq; J = pJ[qq]; cm = c; zq = pzi[qq]; cq = pcas[qq]; }
            }
            if (q >= 0) {
              const GLOBAL_AS int2* row = table + ((((int64_t)rh * NZI + zq) * 3 + (cm - 1)) * NW + wi) * JT;
              while (pd > 0 && fm) {
                const int slot = __ffs((int)fm) - 1;
                fm &= fm - 1;
                const int k = min(J, pd);
                const int2 e = d1_tload(row + k);  // never empty: k <= J
                const int info = e.y, price = e.x;
                const int bk = info & 1023, bz = info >> 10 & 3, bc = info >> 12 & 1, cap1 = info >> 16;
                const int rs = t + delay;
                const int4 ac = s_acc[bk];
#pragma unroll
                for (int n = 0; n < MAXN; ++n) {
                  if (n == slot) {
                    sinfo[n] = (uint32_t)(bk | bz << 10 | bc << 12 | q << 13);
                    sready[n] = rs;
                    slc[n] = t + casc(cq);
                    scas[n] = casc(cq);
                    spods[n] = k;
                    sprice[n] = price;
                    scap[n] = cap1;
                    sdyn[n] = (uint32_t)ac.z;
                    salloc[n] = ac.w;
                    sallocr[n] = delay == 0 ? ac.w : 0;
                  }
                }
                const uint32_t bit = 1u << slot;
                used |= bit;
                if (capbit1(bc) & capsel) cmask |= bit;
#pragma unroll
                for (int qq = 0; qq < MAXP; ++qq) if (qq == q) pmask[qq] |= bit;
                placed += k;
                minscap = min(minscap, cap1);
                Isum += ((long long)ac.y << 32) | (unsigned)ac.x;  // idle draw from launch on
                if (delay == 0) {
                  rdy |= bit;
                  rpods += k;
                  if (cmask & bit) Ffree += cap1 - k;
                }
                else next_ready = min(next_ready, rs);
                if (bc == 0) nsp++; else nod++;
                burn += price;
                launches++;
                last_choice = (uint32_t)bk | (uint32_t)bz << 12 | (uint32_t)bc << 14 | (uint32_t)q << 16;
                hash = (hash ^ last_choice) * 16777619u;
                step_last_type = bk;
                flags |= 2u;
                pd -= k;
              }
            }
          }
        }

      }
      D1_STAMP(5);
      if (ev) {
        // ---- G. disruption (SEMANTICS §3.G) ----
        // Candidates are the consolidatable slots (ready, idle >= consolidateAfter:
        // t >= slc). A deletion needs an empty candidate, or a candidate of a
        // WhenEmptyOrUnderutilized pool whose pods fit the other compatible ready
        // slots (F minus its own free space >= its pods, i.e. F >= its capacity),
        // which needs F >= the smallest node capacity. That gate costs a few
        // instructions per slot; the exact sequential evaluation runs only in the
        // lanes it admits (and only in waves where one does).
        uint32_t elig = 0, emp = 0;
#pragma unroll
        for (int n = MAXN - 1; n >= 0; --n) {  // slot masks built by doubling: 2 VALU per slot and mask
          elig = 2 * elig + (slc[n] <= t ? 1u : 0u);
          emp = 2 * emp + (spods[n] == 0 ? 1u : 0u);
        }
        elig &= rdy;
        emp &= used;
        uint32_t weou = 0;
#pragma unroll
        for (int q = 0; q < MAXP; ++q)
          if (q < NP && ppol[q] == CCKA_WHEN_EMPTY_OR_UNDERUTILIZED) weou |= pmask[q];
        weou_e = weou;
        // G2 (replacement consolidation): on-demand WEOU nodes with pods, not being replaced
        const uint32_t g2c = (DRIFT && replace) ? (weou & od_slots() & ~emp & ~srcm) : 0u;
        // G3 (multi-node consolidation): WEOU nodes with pods, untainted
        const uint32_t g3c = (DRIFT && G3 && multi) ? (weou & ~emp & ~taint()) : 0u;
        const uint32_t gate = elig & (emp | (Ffree >= minscap ? weou : (weou & ~cmask)) | g2c | g3c);
        // DRIFT: ready replacements take over (G1); drifted ready nodes not yet
        // being replaced are drift candidates (G0)
        const uint32_t tkm = DRIFT ? (repm & rdy) : 0u;
        const uint32_t dwork = DRIFT ? (dmask & rdy & ~srcm) : 0u;
        if ((gate || tkm || dwork) && !ablated(ablate, 1)) {
          bool any_del = false;
          // free capacity of the compatible ready untainted slots, from scratch
          auto ffree_now = [&]() {
            int f = 0;
            const uint32_t m = rdy & cmask & ~taint();
#pragma unroll
            for (int n = 0; n < MAXN; ++n) f += (m >> n & 1u) ? scap[n] - spods[n] : 0;
            Ffree = f;
          };
          auto masks_now = [&]() {
            uint32_t el = 0, em = 0;
#pragma unroll
            for (int n = MAXN - 1; n >= 0; --n) {
              el = 2 * el + (slc[n] <= t ? 1u : 0u);
              em = 2 * em + (spods[n] == 0 ? 1u : 0u);
            }
            elig = el & rdy;
            emp = em & used;
          };
          // a slot leaves the cluster (its pods are gone or moved already)
          auto drop_slot = [&](int b) {
            uint32_t binfo = 0;
            int bprice = 0;
#pragma unroll
            for (int n = 0; n < MAXN; ++n)
              if (n == b) {
                binfo = sinfo[n];
                bprice = sprice[n];
                sallocr[n] = 0;
                spods[n] = 0;
                sinfo[n] = 0;
              }
            if ((binfo >> 12 & 1u) == 0) nsp--; else nod--;
            burn -= bprice;
            const int4 ac = s_acc[binfo & 1023u];
            Isum -= ((long long)ac.y << 32) | (unsigned)ac.x;
            const uint32_t nb = ~(1u << b);
            used &= nb; rdy &= nb; cmask &= nb; dmask &= nb; srcm &= nb; repm &= nb;
#pragma unroll
            for (int qq = 0; qq < MAXP; ++qq) pmask[qq] &= nb;
            deletions++;
            any_del = true;
          };
          if constexpr (DRIFT) {
            if (tkm) {
              // G1: each ready replacement (slot order) takes its sources' pods
              // (sources in slot order; sinfo bits 16..23 = the source mask) up to
              // its free capacity; the rest are evicted; the sources are deleted
              uint32_t tk = tkm;
              while (tk) {
                const int m = __ffs((int)tk) - 1;
                tk &= tk - 1;
                uint32_t xm = 0;
                int capm = 0, podm = 0;
#pragma unroll
                for (int n = 0; n < MAXN; ++n)
                  if (n == m) { xm = sinfo[n]; sinfo[n] = xm & 0xFFFFu; capm = scap[n]; podm = spods[n]; }
                const bool okc = (capbit1((int)(xm >> 12 & 1u)) & capsel) != 0;
                uint32_t sm = xm >> 16 & 0xFFu;
                int got = 0;
                while (sm) {
                  const int src = __ffs((int)sm) - 1;
                  sm &= sm - 1;
                  int sp = 0;
#pragma unroll
                  for (int n = 0; n < MAXN; ++n) sp = n == src ? spods[n] : sp;
                  const int k = okc ? min(capm - podm - got, sp) : 0;
                  got += k;
                  rpods -= sp - k;
                  placed -= sp - k;
                  drop_slot(src);
                }
#pragma unroll
                for (int n = 0; n < MAXN; ++n)
                  if (n == m) { spods[n] += got; slc[n] = t + cas_slot(n); }
                repm &= ~(1u << m);
                flags |= 4u;
              }
              ffree_now();
              masks_now();
            }
          }
          // PDB evictions allowed (32-bit: pct <= 100 and replicas <= 32767)
          int allowed = 0x7fffffff;
          if (pdb_pct >= 0) {
            const int rdyp = pdb_member ? rpods : 0, reps = pdb_member ? replicas : 0;
            allowed = max(rdyp - (int)(((uint32_t)(pdb_pct * reps) + 99u) / 100u), 0);
          }
#pragma unroll
          for (int q = 0; q < MAXP; ++q) {
            if (q >= NP) break;
            const int npool = __popc(pmask[q]);
            if (npool == 0) continue;
            const int qbudget = (budget[q] * npool + 99) / 100;
            const bool weou_q = ppol[q] == CCKA_WHEN_EMPTY_OR_UNDERUTILIZED;
            int deleted = 0;
            if constexpr (DRIFT) {
              // G0: drifted ready nodes of the pool in slot order, sharing its budget
              uint32_t dc = dmask & rdy & ~srcm & pmask[q];
              bool acted = false;
              while (dc && deleted < qbudget) {
                const int best = __ffs((int)dc) - 1;
                dc &= dc - 1;
                int bp = 0;
#pragma unroll
                for (int n = 0; n < MAXN; ++n) bp = n == best ? spods[n] : bp;
                const int pdbp = pdb_member ? bp : 0;
                if (pdbp > allowed) continue;
                acted = true;
                // pods move first-fit onto ready, non-drifted, untainted compatible nodes
                const uint32_t recv = rdy & ~dmask & ~taint() & cmask;
                int need = bp;
#pragma unroll
                for (int n = 0; n < MAXN; ++n) {
                  const int fr = (recv >> n & 1u) ? scap[n] - spods[n] : 0;
                  const int k = min(fr, need);
                  spods[n] += k;
                  need -= k;
                  slc[n] = k > 0 ? t + cas_slot(n) : slc[n];
                }
                // the rest: a pre-spun replacement under the pool's current
                // requirements (the F launch rule: the argmin table row), else eviction
                const uint32_t fr = ~used & slot_mask;
                int2 e = make_int2(0, -1);
                uint32_t cmq = 0;
                int cq = 0;
                if (need > 0 && fr) {
                  int J = 0, zq = -1;
#pragma unroll
                  for (int qq = 0; qq < MAXP; ++qq)
                    if (qq == q) { J = pJ[qq]; zq = pzi[qq]; cmq = pcm[qq] & capsel; cq = pcas[qq]; }
                  if (cmq && zq >= 0 && need <= J)
                    e = d1_tload(table + ((((int64_t)rh * NZI + zq) * 3 + (cmq - 1)) * NW + wi) * JT + need);
                }
                if (e.y >= 0 && need > 0) {
                  const int info = e.y, price = e.x;
                  const int bk = info & 1023, bz = info >> 10 & 3, bc = info >> 12 & 1, cap1 = info >> 16;
                  const int slot = __ffs((int)fr) - 1;
                  const int rs = t + delay;
                  const int4 ac = s_acc[bk];
#pragma unroll
                  for (int n = 0; n < MAXN; ++n) {
                    if (n == slot) {
                      sinfo[n] = (uint32_t)(bk | bz << 10 | bc << 12 | q << 13) | (1u << (16 + best));
                      sready[n] = rs;
                      slc[n] = t + casc(cq);
                      scas[n] = casc(cq);
                      spods[n] = 0;
                      sprice[n] = price;
                      scap[n] = cap1;
                      sdyn[n] = (uint32_t)ac.z;
                      salloc[n] = ac.w;
                      sallocr[n] = delay == 0 ? ac.w : 0;
                    }
                    if (n == best) spods[n] = need;
                  }
                  const uint32_t bit = 1u << slot;
                  used |= bit;
                  if (capbit1(bc) & capsel) cmask |= bit;
#pragma unroll
                  for (int qq = 0; qq < MAXP; ++qq) if (qq == q) pmask[qq] |= bit;
                  if (delay == 0) rdy |= bit;
                  else next_ready = min(next_ready, rs);
                  minscap = min(minscap, cap1);
                  Isum += ((long long)ac.y << 32) | (unsigned)ac.x;
                  if (bc == 0) nsp++; else nod++;
                  burn += price;
                  launches++;
                  last_choice = (uint32_t)bk | (uint32_t)bz << 12 | (uint32_t)bc << 14 | (uint32_t)q << 16;
                  hash = (hash ^ last_choice) * 16777619u;
                  step_last_type = bk;
                  srcm |= 1u << best;
                  repm |= bit;
                  flags |= 2u | 16u | 32u;
                } else {
                  rpods -= need;
                  placed -= need;
                  drop_slot(best);
                  flags |= 4u | 16u;
                }
                allowed -= pdbp;
                deleted++;
              }
              if (acted) {
                g_acted = true;
                ffree_now();
                masks_now();
              }
            }
            while (deleted < qbudget) {
              const uint32_t cand = elig & pmask[q] & ~taint();
              const uint32_t ce = cand & emp;
              if (!ce && !(weou_q && (cand & ~emp) && (Ffree >= minscap || (cand & ~emp & ~cmask)))) break;
              int best = -1, bpods = 0, bprice = -1, bcap = 0;
              uint32_t binfo = 0;
              if (ce) {
                // empty candidates come first (pods asc): the highest price, then
                // the lowest slot; deleting one moves nothing
#pragma unroll
                for (int n = 0; n < MAXN; ++n) {
                  const bool c = (ce >> n & 1u) && sprice[n] > bprice;
                  best = c ? n : best;
                  bprice = c ? sprice[n] : bprice;
                  bcap = c ? scap[n] : bcap;
                  binfo = c ? sinfo[n] : binfo;
                }
              } else {
                // under-utilised candidates (pods asc, price desc, slot asc), valid
                // when their pods fit the other compatible ready slots (F minus
                // their own free space) and the PDB allows evicting them
                unsigned long long bkey = ~0ull;
#pragma unroll
                for (int n = 0; n < MAXN; ++n) {
                  const int pods = spods[n];
                  const int need = (cmask >> n & 1u) ? scap[n] : pods;
                  const bool ok = (cand >> n & 1u) && need <= Ffree && (!pdb_member || pods <= allowed);
                  const unsigned long long key = (unsigned long long)pods << 36 |
                                                 (unsigned long long)(0x7fffffff - sprice[n]) << 4 | (unsigned)n;
                  const bool c = ok && key < bkey;
                  bkey = c ? key : bkey;
                  bcap = c ? scap[n] : bcap;
                  binfo = c ? sinfo[n] : binfo;
                }
                if (bkey != ~0ull) {
                  best = (int)(bkey & 15u);
                  bpods = (int)(bkey >> 36);
                  bprice = 0x7fffffff - (int)((bkey >> 4) & 0x7fffffffull);
                  // move its pods first-fit onto the other compatible ready nodes
                  int need = bpods;
                  const uint32_t recv = rdy & cmask & ~(1u << best) & ~taint();
#pragma unroll
                  for (int n = 0; n < MAXN; ++n) {
                    const int fr = (recv >> n & 1u) ? scap[n] - spods[n] : 0;
                    const int k = min(fr, need);
                    spods[n] += k;
                    need -= k;
                    slc[n] = k > 0 ? t + cas_slot(n) : slc[n];
                  }
                }
              }
              if (best < 0) break;
              // delete the node (its pods moved between ready nodes: running counts unchanged)
#pragma unroll
              for (int n = 0; n < MAXN; ++n) {
                sallocr[n] = n == best ? 0 : sallocr[n];
                spods[n] = n == best ? 0 : spods[n];
              }
              if ((binfo >> 12 & 1u) == 0) nsp--; else nod--;
              burn -= bprice;
              const int4 ac = s_acc[binfo & 1023u];
              Isum -= ((long long)ac.y << 32) | (unsigned)ac.x;
              // F loses the node's free space and the moved pods: its whole capacity
              Ffree -= ((rdy & cmask) >> best & 1u) ? bcap : bpods;
              const uint32_t nb = ~(1u << best);
              used &= nb; rdy &= nb; cmask &= nb;
              if constexpr (DRIFT) dmask &= nb;
#pragma unroll
              for (int qq = 0; qq < MAXP; ++qq) pmask[qq] &= nb;
              if (pdb_member) allowed -= bpods;
              deleted++;
              deletions++;
              any_del = true;
              flags |= 4u;
              elig &= nb;
              emp &= nb;
              if (bpods > 0) {  // receivers got pods (and a new consolidatable-from step)
                uint32_t el = 0, em = 0;
#pragma unroll
                for (int n = MAXN - 1; n >= 0; --n) {
                  el = 2 * el + (slc[n] <= t ? 1u : 0u);
                  em = 2 * em + (spods[n] == 0 ? 1u : 0u);
                }
                elig = el & rdy;
                emp = em & used;
              }
            }
            // G3 (SEMANTICS 3.G3): Karpenter's firstN binary search over the
            // consolidation order (pods asc, price desc, slot asc) for the longest
            // prefix of >= 2 candidates that leaves together: their pods move
            // first-fit onto the other compatible ready untainted slots, the rest
            // needs one new node strictly cheaper than the set (the offer table,
            // no spot when every candidate is spot) in a free slot
            bool g3_acted = false;
            if constexpr (DRIFT && G3) {
              if (multi && weou_q && deleted < qbudget) {
                const uint32_t tn = taint();
                const uint32_t cset = elig & pmask[q] & ~emp & ~tn;
                const int nc = min(__popc(cset), qbudget - deleted);
                if (nc >= 2) {
                  uint32_t ord = 0;  // nibble r = slot of rank r
#pragma unroll
                  for (int n = 0; n < MAXN; ++n) {
                    int rk = 0;
#pragma unroll
                    for (int m = 0; m < MAXN; ++m) {
                      const bool before = spods[m] < spods[n] ||
                                          (spods[m] == spods[n] && (sprice[m] > sprice[n] || (sprice[m] == sprice[n] && m < n)));
                      rk += ((cset >> m & 1u) && before) ? 1 : 0;
                    }
                    ord |= (cset >> n & 1u) ? (uint32_t)n << (4 * rk) : 0u;
                  }
                  uint32_t cmq = 0;
                  int zq = -1, cq = 0;
#pragma unroll
                  for (int qq = 0; qq < MAXP; ++qq)
                    if (qq == q) { zq = pzi[qq]; cmq = pcm[qq] & capsel; cq = pcas[qq]; }
                  const uint32_t fr = ~used & slot_mask;
                  int lo = 1, hi = nc - 1, bestk = 0, mid = 0;
                  while (true) {
                    int k;
                    bool commit = false;
                    if (lo <= hi) { mid = (lo + hi) / 2; k = mid + 1; }
                    else if (bestk) { k = bestk; commit = true; }
                    else break;
                    uint32_t set = 0;
                    for (int r = 0; r < k; ++r) set |= 1u << (ord >> (4 * r) & 15u);
                    int tp[MAXN];
                    int pdbp = 0;
                    long long psum = 0;  // up to 8 hourly prices (int64 as in the oracle)
                    uint32_t anyod = 0;
#pragma unroll
                    for (int n = 0; n < MAXN; ++n) {
                      tp[n] = spods[n];
                      const bool in = set >> n & 1u;
                      pdbp += in ? spods[n] : 0;
                      psum += in ? sprice[n] : 0;
                      anyod |= in ? (sinfo[n] >> 12 & 1u) : 0u;
                    }
                    bool ok = !(pdb_member && pdbp > allowed);
                    uint32_t touched = 0;
                    const uint32_t recv = rdy & ~tn & ~set & cmask;
                    for (int r = 0; r < k; ++r) {
                      const int c = (int)(ord >> (4 * r) & 15u);
                      int need = 0;
#pragma unroll
                      for (int n = 0; n < MAXN; ++n) need = n == c ? tp[n] : need;
#pragma unroll
                      for (int m = 0; m < MAXN; ++m) {
                        const int f = (recv >> m & 1u) ? scap[m] - tp[m] : 0;
                        const int kk = min(f, need);
                        tp[m] += kk;
                        need -= kk;
                        touched |= (kk > 0 ? 1u : 0u) << m;
                      }
#pragma unroll
                      for (int n = 0; n < MAXN; ++n) tp[n] = n == c ? need : tp[n];
                    }
                    int sp = 0;
#pragma unroll
                    for (int n = 0; n < MAXN; ++n) sp += (set >> n & 1u) ? tp[n] : 0;
                    int2 e = make_int2(0, -1);
                    if (ok && sp > 0) {
                      const uint32_t cm = anyod ? cmq : (cmq & ~(uint32_t)CCKA_CAP_SPOT);
                      ok = cm != 0 && fr != 0 && zq >= 0 && sp < JT;
                      if (ok) e = d1_tload(table2 + (((int64_t)rh * NZI + zq) * 3 + (cm - 1)) * JT + sp);
                      ok = ok && e.y >= 0 && (long long)e.x < psum;
                    }
                    if (!commit) {
                      if (ok) { bestk = k; lo = mid + 1; }
                      else hi = mid - 1;
                      continue;
                    }
                    // commit: the moves, emptied candidates leave now, the others
                    // when the replacement is ready (G1)
                    uint32_t srcmask = 0;
#pragma unroll
                    for (int n = 0; n < MAXN; ++n) {
                      spods[n] = tp[n];
                      slc[n] = (touched >> n & 1u) ? t + cas_slot(n) : slc[n];
                      srcmask |= ((set >> n & 1u) && tp[n] > 0 ? 1u : 0u) << n;
                    }
                    uint32_t gone = set & ~srcmask;
                    while (gone) {
                      const int n = __ffs((int)gone) - 1;
                      gone &= gone - 1;
                      drop_slot(n);
                      flags |= 4u;
                    }
                    if (sp > 0) {
                      const int info = e.y, prc = e.x;
                      const int bk = info & 1023, bz = info >> 10 & 3, bc = info >> 12 & 1, cap1 = info >> 16;
                      const int slot = __ffs((int)fr) - 1;
                      const int rs = t + delay;
                      const int4 ac = s_acc[bk];
#pragma unroll
                      for (int n = 0; n < MAXN; ++n) {
                        if (n == slot) {
                          sinfo[n] = (uint32_t)(bk | bz << 10 | bc << 12 | q << 13) | (srcmask << 16);
                          sready[n] = rs;
                          slc[n] = t + casc(cq);
                          scas[n] = casc(cq);
                          spods[n] = 0;
                          sprice[n] = prc;
                          scap[n] = cap1;
                          sdyn[n] = (uint32_t)ac.z;
                          salloc[n] = ac.w;
                          sallocr[n] = delay == 0 ? ac.w : 0;
                        }
                      }
                      const uint32_t bit = 1u << slot;
                      used |= bit;
                      if (capbit1(bc) & capsel) cmask |= bit;
#pragma unroll
                      for (int qq = 0; qq < MAXP; ++qq) if (qq == q) pmask[qq] |= bit;
                      if (delay == 0) rdy |= bit;
                      else next_ready = min(next_ready, rs);
                      minscap = min(minscap, cap1);
                      Isum += ((long long)ac.y << 32) | (unsigned)ac.x;
                      if (bc == 0) nsp++; else nod++;
                      burn += prc;
                      launches++;
                      last_choice = (uint32_t)bk | (uint32_t)bz << 12 | (uint32_t)bc << 14 | (uint32_t)q << 16;
                      hash = (hash ^ last_choice) * 16777619u;
                      step_last_type = bk;
                      srcm |= srcmask;
                      repm |= bit;
                      flags |= 2u | 32u;
                    }
                    flags |= 64u;
                    if (pdb_member) allowed -= pdbp;
                    deleted += k;
                    any_del = true;
                    g_acted = true;
                    g3_acted = true;
                    ffree_now();
                    masks_now();
                    break;
                  }
                }
              }
            }
            if constexpr (DRIFT) {
              // G2: the first candidate (pods asc, price desc, slot asc) with a
              // strictly cheaper single offering for its pods gets a pre-spun
              // replacement (the offer table: price only); one per pool per step
              if (replace && weou_q && !g3_acted && deleted < qbudget) {
                uint32_t c2 = elig & pmask[q] & od_slots() & ~emp & ~srcm;
                while (c2) {
                  unsigned long long bkey = ~0ull;
#pragma unroll
                  for (int n = 0; n < MAXN; ++n) {
                    const unsigned long long key = (unsigned long long)spods[n] << 36 |
                                                   (unsigned long long)(0x7fffffff - sprice[n]) << 4 | (unsigned)n;
                    bkey = ((c2 >> n & 1u) && key < bkey) ? key : bkey;
                  }
                  const int best = (int)(bkey & 15u), bp = (int)(bkey >> 36);
                  const int bpr = 0x7fffffff - (int)((bkey >> 4) & 0x7fffffffull);
                  const uint32_t fr = ~used & slot_mask;
                  if (!fr) break;  // no free slot: the search ends
                  uint32_t cmq = 0;
                  int zq = -1, cq = 0;
#pragma unroll
                  for (int qq = 0; qq < MAXP; ++qq)
                    if (qq == q) { zq = pzi[qq]; cmq = pcm[qq] & capsel; cq = pcas[qq]; }
                  int2 e = make_int2(0, -1);
                  if (!(pdb_member && bp > allowed) && cmq && zq >= 0)
                    e = d1_tload(table2 + (((int64_t)rh * NZI + zq) * 3 + (cmq - 1)) * JT + bp);
                  if (e.y < 0 || e.x >= bpr) {  // PDB, no offer or not strictly cheaper
                    c2 &= ~(1u << best);
                    continue;
                  }
                  const int info = e.y, prc = e.x;
                  const int bk = info & 1023, bz = info >> 10 & 3, bc = info >> 12 & 1, cap1 = info >> 16;
                  const int slot = __ffs((int)fr) - 1;
                  const int rs = t + delay;
                  const int4 ac = s_acc[bk];
#pragma unroll
                  for (int n = 0; n < MAXN; ++n) {
                    if (n == slot) {
                      sinfo[n] = (uint32_t)(bk | bz << 10 | bc << 12 | q << 13) | (1u << (16 + best));
                      sready[n] = rs;
                      slc[n] = t + casc(cq);
                      scas[n] = casc(cq);
                      spods[n] = 0;
                      sprice[n] = prc;
                      scap[n] = cap1;
                      sdyn[n] = (uint32_t)ac.z;
                      salloc[n] = ac.w;
                      sallocr[n] = delay == 0 ? ac.w : 0;
                    }
                  }
                  const uint32_t bit = 1u << slot;
                  used |= bit;
                  if (capbit1(bc) & capsel) cmask |= bit;
#pragma unroll
                  for (int qq = 0; qq < MAXP; ++qq) if (qq == q) pmask[qq] |= bit;
                  if (delay == 0) rdy |= bit;
                  else next_ready = min(next_ready, rs);
                  minscap = min(minscap, cap1);
                  Isum += ((long long)ac.y << 32) | (unsigned)ac.x;
                  if (bc == 0) nsp++; else nod++;
                  burn += prc;
                  launches++;
                  last_choice = (uint32_t)bk | (uint32_t)bz << 12 | (uint32_t)bc << 14 | (uint32_t)q << 16;
                  hash = (hash ^ last_choice) * 16777619u;
                  step_last_type = bk;
                  srcm |= 1u << best;
                  repm |= bit;
                  flags |= 2u | 32u;
                  deleted++;
                  g_acted = true;
                  break;
                }
              }
            }
          }
          if (any_del) {  // capacity of the remaining nodes
            g_acted = true;
            minscap = 0x7fffffff;
#pragma unroll
            for (int n = 0; n < MAXN; ++n) minscap = (used >> n & 1u) ? min(minscap, scap[n]) : minscap;
          }
        }

        emp_e = emp;
      }
      D1_STAMP(6);
      if (ev) {
        // ---- H. accounting (energy from the cached sums unless a node saturates) ----
        {
          unsigned long long sv = 0;
          float rv = 0.f;
#pragma unroll
          for (int n = 0; n < MAXN; ++n) {
            const uint32_t pr = (rdy >> n & 1u) ? (uint32_t)spods[n] : 0u;
            sv += (unsigned long long)dyn_of(n) * pr;
            rv = fmaxf(rv, (float)pr * __builtin_amdgcn_rcpf((float)alloc_of(n)));  // 1/alloc only here
          }
          Ssum = sv;
          Rmax = rv;
        }
        q_rbp = __builtin_amdgcn_rcpf((float)rpods);
        const int upp = upp_of(L, q_rbp);
        long long e_step = base_nw + Isum;
        if ((float)upp * Rmax < 0.9999f) e_step += (long long)(Ssum * (unsigned long long)(uint32_t)upp);
        else e_step += dyn_energy(upp);
        cost += burn + base_price;
        e_hour += e_step;
        const int pending = replicas - rpods;
        // SLO: pending pods, an HPA's utilisation above the threshold, or an
        // active KEDA trigger with no replica
        const bool slo_s = KEDA ? (k_act_step && replicas == 0) : (hp.ran && hp.util > slo_util);
        if (pending > 0 || slo_s) { slo++; flags |= 8u; }
        pend_min += pending;
        nmin_spot += nsp;
        nmin_od += nod;
        peak_nodes = max(peak_nodes, nsp + nod);
        tq = t + 1;
        rec = make_int4(replicas, pending, (nsp & 0xFFFF) | nod << 16,
                        (step_last_type & 0xFFFF) | (int)(flags << 16));

        // ---- caches of the quiet steps that follow ----
        if constexpr (BDEF) {
          constexpr int UQ = 1 << 20;  // quiet usages: [0, 2^20)
          // smallest usage with floor(100 * usage / d) >= u (u >= 0), capped at UQ
          auto umin = [](int u, uint32_t d) -> int {
            const unsigned long long a = (unsigned long long)(uint32_t)u * d;
            return a > 100ull * UQ ? UQ : min((int)(((uint32_t)a + 99u) / 100u), UQ);
          };
          const bool hpa_path = !(replicas == 0 && minr != 0);
          bool met = replicas <= mx && replicas >= minr && rpods > 0 && hpa_path;
          const int dnm = replicas > mx ? mx : (replicas < minr && hpa_path ? minr : replicas);
          const bool pend = replicas > rpods;
          q_met = met;
          q_rcap = limit > 0 ? (int)__umul24((uint32_t)rpods, (uint32_t)limit) : 0x7fffffff;
          const uint32_t dreq = (uint32_t)rpods * (uint32_t)req;  // < 2^31
          int ulim = 0, pge = UQ, slo_thr = pend ? 0 : UQ;
          if (met) {
            // util = floor(100 usage / dreq); keep: ulo <= util <= uhi
            int uge = ulo;  // proposal >= cur from this util on
            int lim;        // proposal <= cur below this usage
            if (pend) {
              // unready pods (cur > ready): util <= target proposes ceil(util*ready/target)
              // < cur outside the band; util > target counts every replica (nu =
              // floor(100 usage / (cur*req))): keep iff nu <= uhi, else above cur
              lim = max(umin(target + 1, dreq), umin(uhi + 1, (uint32_t)replicas * (uint32_t)req));
            } else {
              // below the band the proposal ceil(util*cur/target) reaches cur from
              // us = floor((cur-1)*target/cur) + 1 on (binary64 at an exact multiple
              // may round one below that up to cur as well)
              bool sl = false;
              const int cq = fdiv_nb(target + replicas - 1, replicas, __builtin_amdgcn_rcpf((float)replicas), sl);
              int us = target - cq + 1;
              const int um = us - 1;  // < target, so um * cur < 2^30
              if (um >= 0) {
                const int xm = um * replicas;
                const int qm = fdiv_nb(xm, target, rtarget, sl);
                if (__builtin_expect(xm == qm * target, 0) &&
                    (int)ceil(((double)um / (double)target) * (double)replicas) >= replicas)
                  us = um;
              }
              uge = min(uge, max(us, 0));
              lim = umin(uhi + 1, dreq);
            }
            pge = umin(uge, dreq);
            ulim = replicas >= mx ? UQ : lim;
            if (!pend) slo_thr = umin(max(slo_util + 1, 0), dreq);
          } else if (dnm == replicas) {
            ulim = UQ;  // no metric, replicas in range: every step keeps them
          }
          if constexpr (KEDA) {
            // the ScaledObject's metric: quiet while the decision keeps the count
            // (replicas 0: while the trigger is inactive; in [minr, mx]: below
            // the band's top (any metric at mx), with proposal >= cur, i.e. in
            // the band or ceil(L / threshold) >= cur, from min(q_klo,
            // (cur - 1) * threshold + 1) on, or held by a record >= cur; the
            // cooldown is checked per step), no SLO miss but pending pods
            met = false;
            ulim = 0;
            pge = UQ;
            slo_thr = pend ? 0 : UQ;
            q_kcd = false;
            if (replicas == 0) {
              ulim = (int)min(max((long long)kact + 1, 0LL), (long long)UQ);
              pge = 0;
            } else if (replicas >= minr && replicas <= mx) {
              met = true;
              q_kcd = kmin0;
              keda_band(replicas);
              ulim = replicas >= mx ? UQ : (int)min((long long)q_khi + 1, (long long)UQ);
              const long long lc = (long long)(replicas - 1) * kthr + 1;
              pge = (int)max(0LL, min(min((long long)q_klo, lc), (long long)UQ));
            }
            q_met = met;
          }
          q_ulim = ulim;
          q_pge = pge;
          q_slo = slo_thr;
          // upp = floor(usage / ready) = trunc((usage + 0.5) / ready) in binary32 for
          // usage < 2^20 (the quotient stays 0.5/ready clear of an integer; the
          // correctly rounded reciprocal and the single fma rounding are far inside that)
          // (v_rcp_f32, <= 1 ulp: with the fma rounding the estimate is within
          // 0.19/ready of (usage + 0.5)/ready, which lies >= 0.5/ready from an integer)
          q_rbp = rpods > 0 ? __builtin_amdgcn_rcpf((float)rpods) : 0.f;
          q_hbp = 0.5f * q_rbp;
          // no node saturates while upp <= q_usat (pods*upp < alloc on every node)
          q_usat = Rmax > 0.f ? (int)fminf(0.9999f * __builtin_amdgcn_rcpf(Rmax), 1073741824.0f) - 1 : 0x7fffffff;
          q_pendv = replicas - rpods;
          q_nodes = (nsp & 0xFFFF) | nod << 16;
          q_w0 = 0xFFFF | (int)((q_peak ? 1u : 0u) << 16);
          q_w1 = q_w0 | (8 << 16);
        } else {
          q_rbd = __builtin_amdgcn_rcpf((float)(rpods * req));
          q_rbc = __builtin_amdgcn_rcpf((float)(replicas * req));
        }
        if constexpr (BDEF) {  // newest history record >= the new replica count
          int hit = -0x40000000;
#pragma unroll
          for (int k = 2 * HW - 1; k >= 0; --k) {
            const int e = (int)(short)(hdn[k >> 1] >> (16 * (k & 1)));
            hit = e >= replicas ? t - k / NSUB : hit;
          }
          q_hold = replicas <= minr ? 0x3fffffff : hit + wl;
          // without a metric: no records, nothing to hold
          if (!q_met) q_hold = 0x3fffffff;
        }
        // first step that needs the event path again: a node becomes ready,
        // an hour or peak-window boundary, a slot becomes a consolidation
        // candidate that the gate admits (state is unchanged until then, and a
        // disruption evaluation that acted on nothing acts on nothing again
        // with the same candidates), or the next step when disruption acted
        // (the budget may allow more)
        {
          const int th = t + 60 - minute % 60;  // the next clock-hour boundary
          int nx = min(next_ready, th);
          if (pswitch) {
            if (t >= npb) {  // the next peak-window boundary
              const int dps = (ps - minute + 1439) % 1440 + 1, dpe = (pe - minute + 1439) % 1440 + 1;
              npb = t + min(dps, dpe);
            }
            nx = min(nx, npb);
          }
          // empty slots and WhenEmptyOrUnderutilized pools as the disruption
          // phase left them (deletions only clear bits that rdy clears too)
          const uint32_t gm = rdy & (emp_e | (Ffree >= minscap ? weou_e : (weou_e & ~cmask)) |
                                     ((DRIFT && replace) ? (weou_e & od_slots() & ~emp_e & ~srcm) : 0u) |
                                     ((DRIFT && G3 && multi) ? (weou_e & ~emp_e & ~taint()) : 0u));
#pragma unroll
          for (int n = 0; n < MAXN; ++n) nx = ((gm >> n & 1u) && slc[n] > t) ? min(nx, slc[n]) : nx;
          if (g_acted || ablated(ablate, 15)) nx = t + 1;  // ablation runs: every step an event
          nxt = nx;
        }
      }
      if (ev) {
        d1_store_rec(trs, lb + t * 16, rec);
        ++t;
      }
      pf_ok = pf_ok && !ev;
      D1_STAMP(7);
    }
    __builtin_amdgcn_s_setprio(D1_PRIO_HI);
    // ---- ring refill: D1_S rows per iteration once every lane has consumed
    // what they overwrite; issued after the event steps, whose own loads
    // wait for every older vector-memory operation ----
    if (tf < T) {
      if (__ballot(t < T && t < tf + D1_S - rbn + D1_BACK) == 0) {
        const int n1 = min(T, tf + D1_S);
        while (tf < n1) {
          d1_dma_row(lpf, (uint32_t)__builtin_amdgcn_readfirstlane((int)(ring_lds + (uint32_t)tfr * (uint32_t)(rsw * 4))));
          tf_adv();
        }
        if (tf == T) {  // no younger DMA will retire the last rows
          d1_wait_all();
          t_rdy = T;
        }
      }
    }
    bool adv = false;
    if (!pf_ok) {  // a row landed after the prefetch (or the lane left an event step)
      const int tr = rrow(t);
#pragma unroll
      for (int q = 0; q < D1_S; ++q) Lpf[q] = ring[ridx(rnext(tr, q))];
    }

    D1_STAMP(8);
    // ---- quiet steps: up to D1_S per iteration and lane ----
    const int tlim = min(T, t_rdy);
#pragma unroll
    for (int sub = 0; sub < D1_S; ++sub) {
    if constexpr (BDEF) {
        const int L = Lpf[sub];
        // two usage compares decide the HPA (see q_ulim / q_pge); the rest is
        // accounting, the SLO test and the trajectory record, all predicated
        // on `go` (no branch but the rare saturation one). KEDA compares the
        // raw metric and checks the cooldown (an active step restarts it).
        const int usage = min(L, q_rcap);
        const int cv = KEDA ? L : usage;
        const bool ge = cv >= q_pge;
        bool ok = (t < nxt) & ((uint32_t)cv < (uint32_t)q_ulim) & (ge | (t <= q_hold));
        const bool kac = KEDA && L > kact;
        if constexpr (KEDA) ok = ok & (!q_kcd | kac | (t < kcd));
        const bool can = !stall & (t < tlim);
        const bool go = ok & can;
        stall = stall | (can & !ok);
        q_hold = (go & ge) ? max(q_hold, t + wl) : q_hold;
        if constexpr (KEDA) kcd = (go & kac) ? t + kcds : kcd;
        const int upp = (int)fmaf((float)usage, q_rbp, q_hbp);
        if (__builtin_expect(go & (upp > q_usat), 0)) {  // a node may saturate: exact per-node sum instead
          const long long corr = dyn_energy(upp) - (long long)(Ssum * (unsigned long long)(uint32_t)upp);
          e_hour += corr;
        }
        usum += go ? (uint32_t)upp : 0u;
        const bool slo_b = usage >= q_slo;
        slo += (go & slo_b) ? 1 : 0;
        d1_store_rec(trs, go ? lb + t * 16 : D1_NOSTORE, make_int4(replicas, q_pendv, q_nodes, slo_b ? q_w1 : q_w0));
        t += go ? 1 : 0;
        adv = adv | go;
    } else
    if (t < T && !stall && t < t_rdy) {
      // a lane still stepping in sub-step `sub` has advanced in every earlier one
      const int L = Lpf[sub];
      int4 rec;
      if (!(stall = t >= nxt)) {
        const HpaOut h = hpa_eval(L, replicas, rpods, q_rbd, q_rbc);
        stall = h.desired != replicas;
        if (!stall) {
          hpa_commit(h, replicas);
          const int upp = upp_of(L, q_rbp);
          if ((float)upp * Rmax < 0.9999f) e_hour += (long long)(Ssum * (unsigned long long)(uint32_t)upp);
          else e_hour += dyn_energy(upp);
          const int pending = replicas - rpods;
          const bool slo_b = pending > 0 || (h.ran && h.util > slo_util);
          slo += slo_b ? 1 : 0;
          const uint32_t flags = (q_peak ? 1u : 0u) | (slo_b ? 8u : 0u);
          rec = make_int4(replicas, pending, (nsp & 0xFFFF) | nod << 16, 0xFFFF | (int)(flags << 16));
          adv = true;
          d1_store_rec(trs, lb + t * 16, rec);
          ++t;
        }
      }
    }
    }
    qadv = __ballot(adv) != 0;
    D1_STAMP(1);
    // this lane's next samples (the LDS latency hides under the loop tail);
    // rows that have not landed yet are read again at the top
    pf_ok = t + (D1_S - 1) < t_rdy;
    {
      const int tr = rrow(t);
#pragma unroll
      for (int q = 0; q < D1_S; ++q) Lpf[q] = ring[ridx(rnext(tr, q))];
    }
    D1_STAMP(8);
  }
  d1_wait_all();  // no LDS-DMA may outlive the wave
  if constexpr (STAMPS) {
    if (lane == (__ffsll((long long)__ballot(1)) - 1)) {
      for (int k = 1; k < 12; ++k) atomicAdd(&p.stamps[k], (unsigned long long)st_acc[k]);
      atomicMax(&p.stamps[0], (unsigned long long)st_acc[9]);  // longest wave (iterations)
    }
  }
  flush(T);
  energy_nw += e_hour;
  gco2 += (double)e_hour * (ci_min * 1e-9);
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
  p.final_reps[i] = replicas;
  p.final_nodes[i] = __popc(used);
  p.last_choice[i] = last_choice;
  p.hash[i] = hash;
}

// [N][T] -> [T][N] trajectory records (ccka_get_trajectory after the
// single-deployment engine), steps [t0, t0 + tc) at a time into a bounded
// staging buffer: 32 x 32 tiles through LDS, 16-byte elements, both sides
// coalesced; the tiles are numbered on grid.x alone (no grid.y limit on N).
__global__ void __launch_bounds__(256) traj_transpose_kernel(const int4* __restrict__ in, int4* __restrict__ out,
                                                             int64_t N, int64_t T, int64_t t0, int64_t tc) {
  __shared__ int4 tile[32][33];
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
  const int64_t ntn = (N + 31) / 32;
  const int64_t tb = (int64_t)blockIdx.x / ntn * 32, n0 = (int64_t)blockIdx.x % ntn * 32;
#pragma unroll
  for (int k = 0; k < 32; k += 8) {
    const int64_t n = n0 + ty + k, t = tb + tx;
    if (n < N && t < tc) tile[ty + k][tx] = in[n * T + t0 + t];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 32; k += 8) {
    const int64_t t = tb + ty + k, n = n0 + tx;
    if (n < N && t < tc) out[t * N + n] = tile[tx][ty + k];
  }
}

hipError_t launch_traj_transpose(const ccka_traj_rec* in, ccka_traj_rec* out, int64_t N, int64_t T, int64_t t0,
                                 int64_t tc, hipStream_t s) {
  const int64_t blocks = (N + 31) / 32 * ((tc + 31) / 32);
  if (blocks <= 0) return hipSuccess;
  if (blocks > 0x7fffffffLL) return hipErrorInvalidValue;
  hipLaunchKernelGGL(traj_transpose_kernel, dim3((unsigned)blocks), dim3(256), 0, s,
                     reinterpret_cast<const int4*>(in), reinterpret_cast<int4*>(out), N, T, t0, tc);
  return hipGetLastError();
}

// [T][N] load trace -> wave-tiled [wave][T][lpw] (the single-deployment
// kernels' read layout: a wave's rows contiguous, every row lpw wide, the last
// wave's padded: one row stride for all), once per trace / lanes-per-wave
// change (ccka_abi.cpp d1_trace_tile); reads coalesced, writes in runs of lpw ints.
__global__ void __launch_bounds__(256) trace_tile_kernel(const int32_t* __restrict__ in, int32_t* __restrict__ out,
                                                         int64_t N, int64_t T, int64_t lpw) {
  const int64_t total = N * T, stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < total; x += stride) {
    const int64_t t = x / N, n = x - t * N;
    const int64_t w0 = n / lpw * lpw;
    out[w0 * T + t * lpw + (n - w0)] = in[x];
  }
}

hipError_t launch_trace_tile(const int32_t* in, int32_t* out, int64_t N, int64_t T, int32_t lpw, hipStream_t s) {
  if (N <= 0 || T <= 0 || lpw <= 0) return hipErrorInvalidValue;
  const int64_t b0 = (N * T + 255) / 256, blocks = b0 < 65536 ? b0 : 65536;
  hipLaunchKernelGGL(trace_tile_kernel, dim3((unsigned)blocks), dim3(256), 0, s, in, out, N, T, (int64_t)lpw);
  return hipGetLastError();
}

hipError_t launch_table(const TableParams& t, hipStream_t s) {
  const int64_t nkeys = (int64_t)t.R * 24 * t.NZI * 3 * t.NW;
  const unsigned grid = (unsigned)((nkeys * WAVE + 255) / 256);
  hipLaunchKernelGGL(table_kernel, dim3(grid), dim3(256), 0, s, t);
  return hipGetLastError();
}

hipError_t launch_rollout_d1(const D1Params& p, hipStream_t s) {
  const int B = 256;
  const int64_t waves = (p.N + p.lpw - 1) / p.lpw;
  const unsigned grid = (unsigned)((waves + B / WAVE - 1) / (B / WAVE));
  size_t lds = ((size_t)p.K * sizeof(int4) + 255) / 256 * 256 + (size_t)(B / WAVE) * D1_RING_BYTES;
  // price tiles, ci and J in LDS when two blocks per CU still fit (<= 80 KB each)
  const size_t npr = (size_t)p.R * 24 * p.K * p.Z * 2;
  const size_t tabB = ((npr + 1) & ~(size_t)1) * 4 + (size_t)p.R * 24 * 8 + (size_t)p.R * 24 * p.NZI * 3 * 4;
  D1Params q = p;
  q.lds_tab = 0;
  if (lds + tabB <= 80 * 1024) {
    q.lds_tab = 1;
    lds += tabB;
  }
  // OCC = resident waves per SIMD the register allocation targets
  const bool d = p.bdef != 0;
  if (p.keda) {  // a KEDA ScaledObject: default behavior, one decision per step, no drift (d1_prepare)
    if (p.he4) hipLaunchKernelGGL((rollout_d1_kernel<8, 2, false, 2, true, false, 1, 4, false, true>), dim3(grid), dim3(B), lds, s, q);
    else hipLaunchKernelGGL((rollout_d1_kernel<8, 2, false, 2, true, false, 1, 8, false, true>), dim3(grid), dim3(B), lds, s, q);
  } else if (p.nsub == 4) {  // 15 s HPA sync, default behavior (d1_check_world)
    if (p.multi) hipLaunchKernelGGL((rollout_d1_kernel<8, 2, false, 2, true, true, 4, 8, true>), dim3(grid), dim3(B), lds, s, q);
    else if (p.drift) hipLaunchKernelGGL((rollout_d1_kernel<8, 2, false, 2, true, true, 4>), dim3(grid), dim3(B), lds, s, q);
    else hipLaunchKernelGGL((rollout_d1_kernel<8, 2, false, 2, true, false, 4>), dim3(grid), dim3(B), lds, s, q);
  } else if (p.multi) {  // + multi-node consolidation (SEMANTICS 3.G3)
    if (d) hipLaunchKernelGGL((rollout_d1_kernel<8, 2, false, 2, true, true, 1, 8, true>), dim3(grid), dim3(B), lds, s, q);
    else hipLaunchKernelGGL((rollout_d1_kernel<8, 2, false, 2, false, true, 1, 8, true>), dim3(grid), dim3(B), lds, s, q);
  } else if (p.drift) {  // drift (SEMANTICS 3.G0): 8 slots, <= 2 pools (d1_disrupt_ok)
    if (d) hipLaunchKernelGGL((rollout_d1_kernel<8, 2, false, 2, true, true>), dim3(grid), dim3(B), lds, s, q);
    else hipLaunchKernelGGL((rollout_d1_kernel<8, 2, false, 2, false, true>), dim3(grid), dim3(B), lds, s, q);
  } else if (p.stamps) {
    if (d && p.he4) hipLaunchKernelGGL((rollout_d1_kernel<8, 2, true, 2, true, false, 1, 4>), dim3(grid), dim3(B), lds, s, q);
    else if (d) hipLaunchKernelGGL((rollout_d1_kernel<8, 2, true, 2, true>), dim3(grid), dim3(B), lds, s, q);
    else hipLaunchKernelGGL((rollout_d1_kernel<8, 2, true, 2, false>), dim3(grid), dim3(B), lds, s, q);
  } else if (p.maxn <= 8 && p.NP <= 2 && p.occ == 3) {
    hipLaunchKernelGGL((rollout_d1_kernel<8, 2, false, 3, false>), dim3(grid), dim3(B), lds, s, q);
  } else if (p.maxn <= 8 && p.NP <= 2) {
    if (d && p.he4) hipLaunchKernelGGL((rollout_d1_kernel<8, 2, false, 2, true, false, 1, 4>), dim3(grid), dim3(B), lds, s, q);
    else if (d) hipLaunchKernelGGL((rollout_d1_kernel<8, 2, false, 2, true>), dim3(grid), dim3(B), lds, s, q);
    else hipLaunchKernelGGL((rollout_d1_kernel<8, 2, false, 2, false>), dim3(grid), dim3(B), lds, s, q);
  } else if (p.maxn <= 8) {
    hipLaunchKernelGGL((rollout_d1_kernel<8, 4, false, 2, false>), dim3(grid), dim3(B), lds, s, q);
  } else if (p.NP <= 2) {
    hipLaunchKernelGGL((rollout_d1_kernel<16, 2, false, 1, false>), dim3(grid), dim3(B), lds, s, q);
  } else {
    hipLaunchKernelGGL((rollout_d1_kernel<16, 4, false, 1, false>), dim3(grid), dim3(B), lds, s, q);
  }
  return hipGetLastError();
}

}  // namespace ccka
