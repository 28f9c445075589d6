// rollout_pool.hip — MI355X (gfx950) single-deployment rollout with POOLED
// event steps (BASELINE configs 2-4, the headline path).
//
// Same semantics as rollout_d1_kernel and rollout_kernel (docs/SEMANTICS.md),
// bit-identical to the CPU oracle. rollout_d1_kernel runs a wave's event steps
// for the union of its stalled lanes every other iteration: ~16 of 64 lanes
// active per event instruction, and the event runs are most of its VALU
// (DESIGN.md "What bounds the kernel"). Here the full scenario state lives in
// LDS instead of registers, so any wave of the workgroup can run any
// scenario's event step:
//   * owner role (every wave, one lane per scenario): quiet steps from a small
//     register cache (the HPA thresholds, the record fields), up to PL_S per
//     iteration. A step that needs the event path stalls the lane; at the end
//     of the iteration its scenario id goes to the workgroup's LDS event queue
//     and the lane waits (away) until the step has been served.
//   * server role (any wave): when the queue holds >= p.pool_min entries, or
//     the wave has no lane left to step, the wave claims up to 64 queued
//     scenarios, loads their state from LDS, runs the full step for all of
//     them together (readiness, profile, HPA, ReplicaSet, kube-scheduler,
//     Karpenter provisioning, disruption, accounting), stores the state back
//     and publishes the quiet-step cache; the owner lane picks it up at the top
//     of a later iteration.
// One 512-thread workgroup per CU (8 waves, 2 per SIMD) holds ~400 scenarios'
// state (76-78 words each) in LDS; event runs now gather ~64 lanes.
//
// Scope: the upstream default HPA behavior (BDEF) with one decision per step,
// or the one-trigger KEDA ScaledObject, <= 8 slots, <= 2 pools, no drift /
// replacement / multi-node consolidation (launch_rollout_d1 sends those to
// rollout_d1_kernel).
//
// Reference anchors: demo_19_reset_policies.sh:68-75, demo_20_offpeak_configure.sh:59-81,
// demo_21_peak_configure.sh:56-77 (profile patches); demo_30_burst_configure.sh:57-141
// (pods); demo_10_setup_configure.sh:47-56 (PDB).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ccka.h"
#include "d1_common.h"
#include "kparams.h"

#pragma clang fp contract(off)

namespace ccka {

namespace {

constexpr int PL_MAXN = 8, PL_MAXP = 2;
constexpr int PL_BLOCK = PL_WAVES * WAVE;
constexpr int PL_S = 8;        // quiet steps per iteration and lane
constexpr int PL_QCAP = 512;   // event queue ring (>= scenarios per workgroup: 8 x 64)
// wave priority of the event runs (every waiting lane's critical path)
constexpr int PL_PRIO_HI = 3;

// LDS-resident scenario state: word w of local scenario li at [w][SB + li]
// (SoA: a run's lanes read one word of different scenarios per instruction)
namespace plw {
constexpr int SA = 0;      // [8] sinfo (type | zone << 10 | cap << 12 | pool << 13) | spods << 16
constexpr int SB = 8;      // [8] sready (clamped to 0xFFFF) | last pod event step << 16
constexpr int SP = 16;     // [8] sprice (the slot's offering at the current hour)
constexpr int MASK = 24;   // used | rdy << 8 | cmask << 16 | pmask[0] << 24
constexpr int PCAS = 25;   // consolidateAfter steps of pool 0 | pool 1 << 16 (clamped to 0xFFFF)
constexpr int POOL = 26;   // ppol0 | ppol1 << 4 | (pzi0 + 1) << 8 | (pzi1 + 1) << 12 | pcm0 << 16 | pcm1 << 18
                           // | (profile + 1) << 20 | (hour + 1) << 22 | peak_nodes << 27
constexpr int PJ = 27;     // J of pool 0 | pool 1 << 16
constexpr int REP = 28;    // replicas | placed << 16
constexpr int RP = 29;     // rpods | nsp << 16 | nod << 24
constexpr int NR = 30;     // next_ready (0xFFFF: none) | minscap << 16 (0xFFFF: none)
constexpr int FF = 31;     // Ffree
constexpr int COST = 32, BURN = 34, BASEP = 36, EN = 38, EH = 40, ISUM = 42, GCO2 = 44, CI = 46, SSUM = 48;  // 64-bit
constexpr int PEND = 50, SLO = 51, NSPM = 52, NODM = 53, LAU = 54, DEL = 55, LC = 56, HASH = 57;
constexpr int TQ = 58;     // tq | npb << 16
constexpr int QPGE = 59;   // q_pge (< 2^21) | q_kcd << 30 | q_met << 31 (the caches the quiet steps ran with)
constexpr int TEV = 60;    // owner -> server: the step to serve | its sample's window slot << 16 | window << 19
constexpr int USUM = 61;   // owner -> server: sum of upp over the quiet steps since the last event
constexpr int NXT = 62;    // server -> owner: nxt + 1 (0 while not served)
constexpr int QULIM = 63, QSLO = 64, QUSAT = 65, QHOLD = 66;  // server -> owner: quiet caches
constexpr int C0 = 67;     // target | mx << 16
constexpr int C1 = 68;     // ulo | uhi << 16
constexpr int C2 = 69;     // region | wci << 8 | capsel << 16 | pswitch << 18 | nd << 19
constexpr int KCD = 70;    // KEDA: end of the cooldown (owner <-> server)
constexpr int KLO = 71, KHI = 72, KBC = 73;  // KEDA: tolerance band of replica count KBC
constexpr int HDN = 74;    // [HW] packed int16 down-window records
}  // namespace plw

__device__ __forceinline__ int lds_ld(const int* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
__device__ __forceinline__ void lds_st(int* p, int v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
// every LDS operation this wave issued before has completed (LDS executes a
// wave's operations in order, so a flag stored after this is seen after the data)
__device__ __forceinline__ void lds_drain() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

}  // namespace

__host__ __device__ PoolLds pool_lds_layout(int K, int R, int Z, int NZI, int lds_tab, int sb, int hw) {
  auto up16 = [](uint32_t x) { return (x + 15u) & ~15u; };
  PoolLds o{};
  uint32_t off = up16((uint32_t)K * 16u);  // catalog {idle lo, idle hi, dyn, alloc}
  o.cap1 = off;
  off = up16(off + (uint32_t)K * 4u);
  o.tab = off;
  if (lds_tab) {
    const uint32_t npr = (uint32_t)R * 24u * (uint32_t)K * (uint32_t)Z * 2u;
    off = up16(off + ((npr + 1u) & ~1u) * 4u + (uint32_t)R * 24u * 8u + (uint32_t)R * 24u * (uint32_t)NZI * 3u * 4u);
  }
  o.win = off;  // [2][sb][8] the samples of each lane's last two iterations
  off += 2u * (uint32_t)sb * 32u;
  o.queue = off;
  off += PL_QCAP * 4u;
  o.rqueue = off;
  off += PL_QCAP * 4u;
  o.ctrl = off;
  off += 32u;
  o.state = off;
  off = up16(off + (uint32_t)(plw::HDN + hw) * (uint32_t)sb * 4u);
  o.total = off;
  return o;
}

// STATS: diagnostic build only (ccka_debug_ablate bit 16): per-wave counters
// summed into p.stamps[0..7]: iterations (max, sum), event runs, lanes served,
// and s_memtime cycles in the event runs, the quiet steps, idle waits and in all
template <int HE, bool KEDA, bool STATS>
__global__ void __launch_bounds__(PL_BLOCK, 1) rollout_pool_kernel(D1Params p) {
  using namespace plw;
  constexpr int MAXN = PL_MAXN, MAXP = PL_MAXP;
  constexpr int HW = HE / 2;  // history words (2 records each)
  constexpr int JR = HE;      // steps whose records an event step may rebuild
  extern __shared__ __attribute__((aligned(16))) int4 s_acc[];
  char* const lds = reinterpret_cast<char*>(s_acc);
  const int SBn = 8 * p.lpw;  // scenarios per workgroup (state stride)
  const PoolLds LY = pool_lds_layout(p.K, p.R, p.Z, p.NZI, p.lds_tab, SBn, HW);
  int* const s_cap1 = reinterpret_cast<int*>(lds + LY.cap1);
  int* const s_price = reinterpret_cast<int*>(lds + LY.tab);
  const int n_pr = p.R * 24 * p.K * p.Z * 2;
  double* const s_ci = reinterpret_cast<double*>(s_price + ((n_pr + 1) & ~1));
  int* const s_jtab = reinterpret_cast<int*>(s_ci + p.R * 24);
  int* const queue = reinterpret_cast<int*>(lds + LY.queue);
  int* const s_win = reinterpret_cast<int*>(lds + LY.win);
  int* const q_head = reinterpret_cast<int*>(lds + LY.ctrl);
  int* const q_tail = q_head + 1;
  int* const r_head = q_head + 3;
  int* const r_tail = q_head + 4;
  int* const n_done = q_head + 5;
  int* const rqueue = reinterpret_cast<int*>(lds + LY.rqueue);
  int* const st = reinterpret_cast<int*>(lds + LY.state);
  auto S = [&](int w, int li) -> int* { return st + w * SBn + li; };
  auto ld64 = [&](int w, int li) -> long long {
    return (long long)(((uint64_t)(uint32_t)*S(w + 1, li) << 32) | (uint32_t)*S(w, li));
  };
  auto st64 = [&](int w, int li, long long v) {
    *S(w, li) = (int)(uint32_t)(uint64_t)v;
    *S(w + 1, li) = (int)(uint32_t)((uint64_t)v >> 32);
  };
  auto ldd = [&](int w, int li) -> double { return __longlong_as_double(ld64(w, li)); };
  auto std_ = [&](int w, int li, double v) { st64(w, li, __double_as_longlong(v)); };

  const int tid = threadIdx.x;
  const int lane = tid & (WAVE - 1);
  const bool ldt = p.lds_tab;
  for (int x = tid; x < p.K; x += PL_BLOCK) {
    const long long idle = p.acc[x * 3 + 0];
    s_acc[x] = make_int4((int)(idle & 0xffffffffLL), (int)(idle >> 32), (int)p.acc[x * 3 + 1], (int)p.acc[x * 3 + 2]);
    s_cap1[x] = p.cap1t[x];
  }
  if (ldt) {
    for (int x = tid; x < n_pr; x += PL_BLOCK) s_price[x] = p.price[x];
    for (int x = tid; x < p.R * 24; x += PL_BLOCK) s_ci[x] = p.ci_gpwmin[x];
    for (int x = tid; x < p.R * 24 * p.NZI * 3; x += PL_BLOCK) s_jtab[x] = p.jtab[x];
  }

  // ---- world constants (opaque register copies) ----
  const int T = opq(p.T), lpw = opq(p.lpw);
  const int64_t blk_first = (int64_t)blockIdx.x * SBn;
  const int nblk = (int)min((int64_t)SBn, p.N - blk_first);  // scenarios of this workgroup
  // the event queue starts with every scenario's first step; the ready queue
  // (served scenarios waiting for a lane) empty
  for (int x = tid; x < PL_QCAP; x += PL_BLOCK) {
    queue[x] = x < nblk ? x + 1 : 0;
    rqueue[x] = 0;
  }
  if (tid == 0) {
    q_head[0] = 0;      // event queue head
    q_head[1] = nblk;   // event queue tail
    q_head[2] = 0;      // s_memtime (low word) of the last claim
    q_head[3] = 0;      // ready queue head
    q_head[4] = 0;      // ready queue tail
    q_head[5] = 0;      // scenarios finished
  }
  const int NP = opq(p.NP), NZI = opq(p.NZI), NW = opq(p.NW), JT = opq(p.JT);
  const int maxn = opq(p.maxn), pdb_member = opq(p.pdb_member);
  const int pdb_pct = opq(p.pdb_pct), slo_util = opq(p.slo_util), delay = opq(p.delay);
  const int base_nodes = opq(p.base_nodes), base_type = opq(p.base_type);
  const int K = opq(p.K), Z = opq(p.Z);
  const int ps = opq(p.peak_start) % 1440, pe = opq(p.peak_end) % 1440;
  const int ps_raw = opq(p.peak_start), pe_raw = opq(p.peak_end);
  const int sm0 = opq(p.start_minute) % 1440;
  const long long base_nw = opq(p.base_nw);
  const GLOBAL_AS int32_t* const price = opq_ptr(p.price);
  const GLOBAL_AS double* const ci_gpwmin = opq_ptr(p.ci_gpwmin);
  const GLOBAL_AS int2* const table = opq_ptr(p.table);
  const GLOBAL_AS int32_t* const jtab = opq_ptr(p.jtab);
  const int minr = KEDA ? max(opq(p.k_min), 1) : opq(p.minr), req = opq(p.req_cpu), limit = opq(p.limit);
  const int kthr = KEDA ? opq(p.k_thr) : 1, kact = KEDA ? opq(p.k_act) : 0, kcds = KEDA ? opq(p.k_cds) : 0;
  const bool kmin0 = KEDA && opq(p.k_min) == 0;
  const float rkthr = __builtin_amdgcn_rcpf((float)kthr);
  int budget[MAXP];
#pragma unroll
  for (int q = 0; q < MAXP; ++q) budget[q] = opq(p.budget[q]);
  const uint32_t slot_mask = maxn >= 32 ? 0xFFFFFFFFu : ((1u << maxn) - 1u);
  const int pool_min = opq(p.pool_min), pool_age = opq(p.pool_age), pool_idle = opq(p.pool_idle);
  auto casc = [](int c) { return min(c, 0xFFFF); };

  // ---- trace samples: a buffer resource over this workgroup's samples ----
  // wave-tiled copy [wave][T][lpw] (scenario li of wave w = li / lpw at
  // element w * lpw * T + t * lpw + li % lpw), or the [T][NL] trace (shared
  // traces: column (first_id + i) % trace_mod); one step stride either way
  const bool tiled = p.load_w != nullptr;
  const int sstride = tiled ? lpw : (int)opq(p.NL);
  const __amdgpu_buffer_rsrc_t lrs = __builtin_amdgcn_make_buffer_rsrc(
      tiled ? (void*)(p.load_w + blk_first * T) : (void*)p.load, 0,
      tiled ? (nblk + lpw - 1) / lpw * lpw * T * 4 : (int)min((int64_t)0x7FFFFFFF, p.NL * (int64_t)T * 4), 0x00020000);
  // element index of (scenario li, step 0)
  auto sample_base = [&](int li) -> int {
    if (tiled) {
      const int w = li / lpw;
      return w * lpw * T + (li - w * lpw);
    }
    const int64_t i = blk_first + li;
    return (int)(p.trace_mod > 0 ? (p.first_id + i) % p.trace_mod : i);
  };
  // trajectory records scenario-major [N][T] through the workgroup's range
  GLOBAL_AS int4* const traj = opq_ptr(reinterpret_cast<int4*>(p.traj));
  const __amdgpu_buffer_rsrc_t trs = __builtin_amdgcn_make_buffer_rsrc(
      traj ? (void*)(reinterpret_cast<int4*>(p.traj) + blk_first * T) : (void*)p.load, 0, traj ? nblk * T * 16 : 0,
      0x00020000);

  // ---- every scenario's initial state into LDS ----
  for (int li = tid; li < nblk; li += PL_BLOCK) {
    const int64_t i = blk_first + li;
    const int r = p.region ? (int)p.region[i] : 0;
    const int target = KEDA ? 1 : (p.target ? (int)p.target[i] : p.target0);
    const int mx = KEDA ? p.k_max : (p.maxr ? (int)p.maxr[i] : p.maxr0);
    const int dwin = (!KEDA && p.down_stab) ? (int)p.down_stab[i] : p.dstab0;
    const int nd = min(__popc(wmask(dwin)), 2 * HW);
    const int reset_ca = p.reset_ca ? (int)p.reset_ca[i] : p.reset_ca0;
    const int pswitch = p.pswitch ? (int)p.pswitch[i] : p.pswitch0;
    const int wi = p.wci ? (int)p.wci[i] : 0;
    const uint32_t capsel = p.cap_sel ? (uint32_t)p.cap_sel[i] : (uint32_t)p.capsel0;
    int ulo = max(0, (int)floor(p.tol_lo * (double)target) - 2);
    while ((double)ulo / (double)target < p.tol_lo) ++ulo;
    int uhi = (int)floor(p.tol_hi * (double)target) + 2;
    while ((double)uhi / (double)target > p.tol_hi) --uhi;
    *S(C0, li) = target | mx << 16;
    *S(C1, li) = ulo | uhi << 16;
    *S(C2, li) = r | wi << 8 | (int)(capsel & 3u) << 16 | (pswitch ? 1 : 0) << 18 | nd << 19;
    // NodePools: base spec then RESET (SEMANTICS §1)
    int ppol[MAXP], pcas[MAXP], pzi[MAXP];
    uint32_t pcm[MAXP];
#pragma unroll
    for (int q = 0; q < MAXP; ++q) {
      ppol[q] = 0; pcas[q] = 0; pzi[q] = -1; pcm[q] = 0;
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
#pragma unroll
    for (int n = 0; n < MAXN; ++n) { *S(SA + n, li) = 0; *S(SB + n, li) = 0; *S(SP + n, li) = 0; }
    *S(MASK, li) = 0;
    *S(PCAS, li) = casc(pcas[0]) | casc(pcas[1]) << 16;
    *S(POOL, li) = ppol[0] | ppol[1] << 4 | (pzi[0] + 1) << 8 | (pzi[1] + 1) << 12 | (int)pcm[0] << 16 |
                   (int)pcm[1] << 18;  // profile -1, hour -1, peak_nodes 0
    *S(PJ, li) = 0;
    *S(REP, li) = p.replicas0;  // placed 0
    *S(RP, li) = 0;
    *S(NR, li) = 0xFFFF | 0xFFFF << 16;
    *S(FF, li) = 0;
#pragma unroll
    for (int w = COST; w < PEND; ++w) *S(w, li) = 0;
    *S(PEND, li) = 0; *S(SLO, li) = 0; *S(NSPM, li) = 0; *S(NODM, li) = 0;
    *S(LAU, li) = 0; *S(DEL, li) = 0;
    *S(LC, li) = (int)0xFFFFFFFFu;
    *S(HASH, li) = (int)2166136261u;
    *S(TQ, li) = 0;
    *S(QPGE, li) = 0;
    *S(TEV, li) = 0; *S(USUM, li) = 0; *S(NXT, li) = 0;
    *S(KCD, li) = kcds;
    *S(KLO, li) = 0; *S(KHI, li) = -1; *S(KBC, li) = -1;
    if (KEDA && p.replicas0 > 0) {  // the tolerance band of the initial replica count
      const double D = (double)kthr * (double)p.replicas0;
      long long lo = max((long long)floor(p.tol_lo * D) - 2, -1LL);
      while ((double)lo / D < p.tol_lo) ++lo;
      long long hi = (long long)floor(p.tol_hi * D) + 2;
      while ((double)hi / D > p.tol_hi) --hi;
      *S(KLO, li) = (int)min(lo, 0x7fffffffLL);
      *S(KHI, li) = (int)min(hi, 0x7ffffffeLL);
      *S(KBC, li) = p.replicas0;
    } else if (KEDA) {
      *S(KBC, li) = p.replicas0;
    }
#pragma unroll
    for (int w = 0; w < HW; ++w) *S(HDN + w, li) = (int)0x80008000u;
    // the first step's sample (its event step reads slot 0 of window 0)
    s_win[li * 8] = (int)__builtin_amdgcn_raw_buffer_load_b32(lrs, sample_base(li) * 4, 0, 0);
  }
  __syncthreads();

  // ---- lane registers: the attached scenario's quiet-step cache ----
  // A lane steps whichever scenario it is attached to; a scenario leaves its
  // lane at an event step (the event queue) and joins the ready queue once
  // served, where any free lane picks it up: lanes never wait for a scenario.
  int sid = -1;        // attached local scenario (-1: free)
  int t = 0, nxt = 0;
  int q_ulim = 0, q_pge = 0, q_slo = 0, q_usat = 0, q_hold = 0, q_rcap = 0, q_pendv = 0, q_nodes = 0;
  int q_w0 = 0, replicas_q = 0, nd = 0;
  float q_rbp = 0.f, q_hbp = 0.f;
  bool q_kcd = false;
  int kcd = kcds;
  uint32_t usum = 0;
  int sloq = 0;    // SLO minutes of the quiet steps since the scenario was attached
  int sbase = 0;   // sample element of (sid, step 0)
  int lb = 0;      // record byte offset of (sid, step 0)
  int Lpf[PL_S];
#pragma unroll
  for (int q = 0; q < PL_S; ++q) Lpf[q] = 0;
  auto prefetch = [&](int tn) {
    const int vo = (sbase + tn * sstride) * 4;
#pragma unroll
    for (int q = 0; q < PL_S; ++q) Lpf[q] = __builtin_amdgcn_raw_buffer_load_b32(lrs, vo, q * sstride * 4, 0);
  };
  // a scenario's results (SEMANTICS §3.H: the quiet steps after its last
  // event, the last clock hour's carbon), `uq` / `sq` the quiet steps' sums
  auto finish = [&](int li, uint32_t uq, int sq) {
    const int64_t i = blk_first + li;
    const uint32_t wtq = (uint32_t)*S(TQ, li);
    const int n = T - (int)(wtq & 0xFFFFu);
    const uint32_t wrep = (uint32_t)*S(REP, li), wrp = (uint32_t)*S(RP, li);
    const int reps = (int)(wrep & 0xFFFFu), rpd = (int)(wrp & 0xFFFFu);
    const int nsp = (int)(wrp >> 16 & 0xFFu), nod = (int)(wrp >> 24);
    const long long cost = ld64(COST, li) + (ld64(BURN, li) + ld64(BASEP, li)) * (long long)n;
    long long e_hour = ld64(EH, li) + (base_nw + ld64(ISUM, li)) * (long long)n;
    e_hour += (long long)((unsigned long long)ld64(SSUM, li) * (unsigned long long)uq);
    const long long energy_nw = ld64(EN, li) + e_hour;
    const double gco2 = ldd(GCO2, li) + (double)e_hour * (ldd(CI, li) * 1e-9);
    p.cost[i] = cost;
    p.energy[i] = (double)energy_nw * 1e-9;
    p.gco2[i] = gco2;
    p.slo[i] = *S(SLO, li) + sq;
    p.pend_min[i] = *S(PEND, li) + (reps - rpd) * n;
    p.nmin_spot[i] = *S(NSPM, li) + nsp * n;
    p.nmin_od[i] = *S(NODM, li) + nod * n;
    p.launches[i] = *S(LAU, li);
    p.deletions[i] = *S(DEL, li);
    p.peak_nodes[i] = (int)((uint32_t)*S(POOL, li) >> 27);
    p.final_reps[i] = reps;
    p.final_nodes[i] = __popc((uint32_t)*S(MASK, li) & 0xFFu);
    p.last_choice[i] = (uint32_t)*S(LC, li);
    p.hash[i] = (uint32_t)*S(HASH, li);
  };

  // =======================================================================
  // the event step of up to 64 queued scenarios (lane j serves entry j)
  // =======================================================================
  auto serve = [&](const int h, const int c) {
    const bool ev = lane < c;
    int sl = 0;  // local scenario served by this lane
    if (ev) {
      int e = 0;
      do {
        e = __hip_atomic_exchange(&queue[(h + lane) & (PL_QCAP - 1)], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      } while (e == 0);  // reserved by an owner that has not written it yet
      sl = e - 1;
    }
    asm volatile("" ::: "memory");
    if (!ev) return;
    // ---- per-scenario constants ----
    const int ct0 = *S(C0, sl), ct1 = *S(C1, sl), ct2 = *S(C2, sl);
    const int target = ct0 & 0xFFFF, mx = (int)((uint32_t)ct0 >> 16);
    const int ulo = ct1 & 0xFFFF, uhi = (int)((uint32_t)ct1 >> 16);
    const int r = ct2 & 0xFF, wi = ct2 >> 8 & 0xFF;
    const uint32_t capsel = (uint32_t)(ct2 >> 16) & 3u;
    const bool pswitch = (ct2 >> 18 & 1) != 0;
    const int snd = ct2 >> 19 & 31;
    const float rtarget = __builtin_amdgcn_rcpf((float)target);
    uint32_t dn16[HW];
#pragma unroll
    for (int w = 0; w < HW; ++w) dn16[w] = (2 * w < snd ? 0xFFFFu : 0u) | (2 * w + 1 < snd ? 0xFFFF0000u : 0u);
    const int wl = snd, wr = snd;
    // ---- the step and its samples (this step's and the JR before it) ----
    // the step's sample and the JR before it, from the owner's windows of
    // its last two iterations (slot ws of window wp holds step ts)
    const uint32_t wtev = (uint32_t)*S(TEV, sl);
    const int ts = (int)(wtev & 0xFFFFu), ws = (int)(wtev >> 16 & 7u), wp = (int)(wtev >> 19 & 1u);
    const int* const wcur = s_win + (wp * SBn + sl) * 8;
    const int* const wprv = s_win + ((wp ^ 1) * SBn + sl) * 8;
    const int L = wcur[ws];
    int Lh[JR];
#pragma unroll
    for (int j = 0; j < JR; ++j) Lh[j] = j < ws ? wcur[ws - 1 - j] : wprv[8 + ws - 1 - j];
    // ---- state ----
    const uint32_t wpool = (uint32_t)*S(POOL, sl);
    int ppol[MAXP], pcas[MAXP], pzi[MAXP], pJ[MAXP];
    uint32_t pcm[MAXP], pmask[MAXP];
    ppol[0] = wpool & 15u; ppol[1] = wpool >> 4 & 15u;
    pzi[0] = (int)(wpool >> 8 & 15u) - 1; pzi[1] = (int)(wpool >> 12 & 15u) - 1;
    pcm[0] = wpool >> 16 & 3u; pcm[1] = wpool >> 18 & 3u;
    int profile = (int)(wpool >> 20 & 3u) - 1, hour = (int)(wpool >> 22 & 31u) - 1;
    int peak_nodes = (int)(wpool >> 27);
    {
      const uint32_t x = (uint32_t)*S(PCAS, sl);
      pcas[0] = x & 0xFFFFu; pcas[1] = x >> 16;
      const uint32_t y = (uint32_t)*S(PJ, sl);
      pJ[0] = y & 0xFFFFu; pJ[1] = y >> 16;
    }
    const uint32_t wmk = (uint32_t)*S(MASK, sl);
    uint32_t used = wmk & 0xFFu, rdy = wmk >> 8 & 0xFFu, cmask = wmk >> 16 & 0xFFu;
    pmask[0] = wmk >> 24;
    pmask[1] = used & ~pmask[0];
    auto cas_of = [&](uint32_t info) {
      const int m1 = -(int)(info >> 13 & 1u);
      return pcas[0] ^ ((pcas[0] ^ pcas[1]) & m1);
    };
    // node slots in registers; a slot's consolidateAfter, dynamic power and
    // allocatable CPU are its pool's / type's (derived, not carried)
    uint32_t sinfo[MAXN];
    int sready[MAXN], slc[MAXN], spods[MAXN], sprice[MAXN], scap[MAXN];
    auto cas_slot = [&](int n) -> int { return casc(cas_of(sinfo[n])); };
    auto dyn_of = [&](int n) -> uint32_t { return (uint32_t)s_acc[sinfo[n] & 1023u].z; };
    auto alloc_of = [&](int n) -> int { return s_acc[sinfo[n] & 1023u].w; };
    auto alloc_ready = [&](int n) -> uint32_t { return (rdy >> n & 1u) ? (uint32_t)alloc_of(n) : 0u; };
#pragma unroll
    for (int n = 0; n < MAXN; ++n) {
      const uint32_t a = (uint32_t)*S(SA + n, sl), b = (uint32_t)*S(SB + n, sl);
      sinfo[n] = a & 0xFFFFu;
      spods[n] = (int)(a >> 16);
      sready[n] = (int)(b & 0xFFFFu);
      slc[n] = (int)(b >> 16) + cas_slot(n);
      sprice[n] = *S(SP + n, sl);
      scap[n] = s_cap1[sinfo[n] & 1023u];
    }
    const uint32_t wrep = (uint32_t)*S(REP, sl), wrp = (uint32_t)*S(RP, sl), wnr = (uint32_t)*S(NR, sl);
    int replicas = (int)(wrep & 0xFFFFu), placed = (int)(wrep >> 16);
    int rpods = (int)(wrp & 0xFFFFu), nsp = (int)(wrp >> 16 & 0xFFu), nod = (int)(wrp >> 24);
    int next_ready = (wnr & 0xFFFFu) == 0xFFFFu ? 0x7fffffff : (int)(wnr & 0xFFFFu);
    int minscap = (wnr >> 16) == 0xFFFFu ? 0x7fffffff : (int)(wnr >> 16);
    int Ffree = *S(FF, sl);
    long long burn = ld64(BURN, sl), base_price = ld64(BASEP, sl), e_hour = ld64(EH, sl), Isum = ld64(ISUM, sl);
    // counters as this step's increments (added to the LDS state at the end)
    long long cost = 0;
    int pend_min = 0, slo = 0, nmin_spot = 0, nmin_od = 0, launches = 0, deletions = 0;
    const uint32_t wtq = (uint32_t)*S(TQ, sl);
    int tq = (int)(wtq & 0xFFFFu), npb = (int)(wtq >> 16);
    const uint32_t wqp = (uint32_t)*S(QPGE, sl);
    const int q_pge0 = (int)(wqp & 0x3FFFFFFFu);
    const bool q_met0 = (wqp >> 31) != 0;
    const uint32_t usum0 = (uint32_t)*S(USUM, sl);
    uint32_t hdn[HW];
#pragma unroll
    for (int w = 0; w < HW; ++w) hdn[w] = (uint32_t)*S(HDN + w, sl);
    int kcd_s = KEDA ? *S(KCD, sl) : 0, q_klo = 0, q_khi = -1, kb_cur = -1;
    if constexpr (KEDA) { q_klo = *S(KLO, sl); q_khi = *S(KHI, sl); kb_cur = *S(KBC, sl); }
    bool k_act_step = false;
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
    auto od_slots = [&]() {
      uint32_t m = 0;
#pragma unroll
      for (int n = MAXN - 1; n >= 0; --n) m = 2 * m + (sinfo[n] >> 12 & 1u);
      return m & used;
    };
    (void)od_slots;

    // ---- C. HPA helpers (as rollout_d1_kernel) ----
    struct HpaOut {
      int util, proposal, desired;
      bool ran, hpa_path;
    };
    auto behave = [&](int proposal, int cur) -> int {
      int dnr = proposal;
      {
        short2v a = as_s2(bfi(dn16[0], hdn[0], 0x80008000u));
#pragma unroll
        for (int w = 1; w < HW; ++w) a = __builtin_elementwise_max(a, as_s2(bfi(dn16[w], hdn[w], 0x80008000u)));
        dnr = max(dnr, max((int)a.x, (int)a.y));
      }
      const int rc = min(max(cur, proposal), dnr);
      int lo = minr, hi = mx;
      // up: max(Percent 100 -> ceil(2.0*cur), Pods 4 -> cur+4) over 15 s
      // periods (no 60 s history inside), never below cur; down: Percent 100
      // -> int(cur*0.0) = 0, never above cur
      hi = rc > cur ? min(hi, max(2 * cur, cur + 4)) : hi;
      lo = rc < cur ? max(lo, 0) : lo;
      return rc < lo ? lo : (rc > hi ? hi : rc);
    };
    auto hpa_eval = [&](int Lv, int cur, int ready, float rbd, float rbc) -> HpaOut {
      HpaOut o;
      const bool metric = cur <= mx && cur >= minr && ready > 0 && !(cur == 0 && minr != 0);
      int util = 0, proposal = cur;
      {
        const int rcapv = ready * limit;
        const int usage = (limit > 0 && rcapv < Lv) ? rcapv : Lv;
        const int a = usage * 100;
        const int dreq = ready * req;
        const int dcur = cur * req;
        bool slow = usage < 0 || usage > 21474836;
        util = fdiv_nb(a, dreq, rbd, slow);
        int nu = 0;
        if (cur > ready) nu = fdiv_nb(a, dcur, rbc, slow);
        if (__builtin_expect(metric && slow, 0)) util = (int)(((long long)usage * 100) / ((long long)ready * req));
        const bool unready_up = cur > ready && util > target;
        int u = util, base = ready;
        if (unready_up) { u = nu; base = cur; }
        if (__builtin_expect(metric && slow && unready_up, 0)) u = (int)(((long long)usage * 100) / ((long long)cur * req));
        const bool keep = (u >= ulo && u <= uhi) || (unready_up && u < target);
        bool slow2 = (uint32_t)u > 0xFFFFu;
        const int x = u * base;
        const int q = fdiv_nb(x, target, rtarget, slow2);
        const bool exactm = x == q * target;
        int cc = q + (exactm ? 0 : 1);
        if (__builtin_expect(metric && !keep && (exactm || slow2), 0)) cc = (int)ceil(((double)u / (double)target) * (double)base);
        const int pe2 = unready_up ? max(cur, cc) : cc;
        proposal = (metric && !keep) ? pe2 : cur;
      }
      o.util = util;
      o.proposal = proposal;
      o.ran = metric;
      o.hpa_path = !(cur == 0 && minr != 0);
      int desired = cur > mx ? mx : (cur < minr && o.hpa_path ? minr : cur);
      if (metric) desired = behave(proposal, cur);
      o.desired = desired;
      return o;
    };
    auto keda_eval = [&](int Lv, int cur, int tsv) -> HpaOut {
      HpaOut o{};
      const bool act = Lv > kact;
      const bool cool = !act && kmin0 && tsv >= kcd_s;
      if (act) kcd_s = tsv + kcds;
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
          if (Lv < q_klo || Lv > q_khi) {
            bool slow = Lv < 0;
            const int q = fdiv_nb(max(Lv, 0), kthr, rkthr, slow);
            prop = q + (q * kthr != Lv ? 1 : 0);
            if (__builtin_expect(slow, 0)) prop = (int)ceil((double)Lv / (double)kthr);
          }
          o.proposal = prop;
          o.ran = true;
          desired = behave(prop, cur);
        }
      }
      o.desired = desired;
      return o;
    };
    auto upp_of = [&](int Lv, float rbp) {
      const int rcapv = rpods * limit;
      const int usage = max((limit > 0 && rcapv < Lv) ? rcapv : Lv, 0);
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
          const uint32_t use = min((uint32_t)spods[n] * (uint32_t)upp, alloc_ready(n));
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
    auto refresh_J = [&](int rh) {
#pragma unroll
      for (int q = 0; q < MAXP; ++q) {
        const uint32_t cm = pcm[q] & capsel;
        const int64_t ji = ((int64_t)rh * NZI + pzi[q]) * 3 + (cm - 1);
        pJ[q] = (q < NP && cm && pzi[q] >= 0) ? (ldt ? s_jtab[ji] : jtab[ji]) : 0;
      }
    };

    // ---- the down-window records of the quiet steps [tq, ts), oldest first,
    // from their samples and the caches they ran with (rollout_d1_kernel) ----
    const int t = ts;
    {
      const int kq = min(t - tq, wr);
      if (kq > 0) {
        const int cur16 = min(replicas, D1_REC_SAT);
        const int q_rcap0 = limit > 0 ? (int)__umul24((uint32_t)rpods, (uint32_t)limit) : 0x7fffffff;
        int us[JR], rv[JR];
        bool anylow = false;
#pragma unroll
        for (int j = 0; j < JR; ++j) {
          us[j] = KEDA ? Lh[j] : min(Lh[j], q_rcap0);
          rv[j] = q_met0 ? cur16 : (int)0x8000;
          anylow |= (j < kq) & q_met0 & (us[j] < q_pge0);
        }
        if (KEDA && anylow) {
#pragma unroll
          for (int j = 0; j < JR; ++j) {
            bool sl2 = false;
            const bool low = (j < kq) & q_met0 & (us[j] < q_pge0);
            const int q = fdiv_nb(max(us[j], 0), kthr, rkthr, sl2);
            rv[j] = low ? min(q + (q * kthr != us[j] ? 1 : 0), D1_REC_SAT) : rv[j];
          }
        } else if (anylow) {
          const int dreq = rpods * req;
          const float rbd = __builtin_amdgcn_rcpf((float)dreq);
          bool anyex = false;
#pragma unroll
          for (int j = 0; j < JR; ++j) {
            bool sl2 = false;
            const bool low = (j < kq) & q_met0 & (us[j] < q_pge0);
            const int util = fdiv_nb(us[j] * 100, dreq, rbd, sl2);
            const int x = (int)__umul24((uint32_t)util, (uint32_t)rpods);
            const int q = fdiv_nb(x, target, rtarget, sl2);
            const bool ex = x == q * target;
            anyex |= low & ex;
            rv[j] = low ? min(q + (ex ? 0 : 1), D1_REC_SAT) : rv[j];
            us[j] = (low & ex) ? util : -1;
          }
          if (__builtin_expect(anyex, 0)) {
#pragma unroll
            for (int j = 0; j < JR; ++j)
              if (us[j] >= 0) rv[j] = min((int)ceil(((double)us[j] / (double)target) * (double)rpods), D1_REC_SAT);
          }
        }
#pragma unroll
        for (int j = JR - 1; j >= 0; --j)
          if (j < kq) ring_push<HW>(hdn, rv[j]);
      }
    }
    // flush: per-step constants of the quiet steps [tq, t) (SEMANTICS §3.H)
    {
      const int n = t - tq;
      cost += (burn + base_price) * (long long)n;
      e_hour += (base_nw + Isum) * (long long)n;
      e_hour += (long long)((unsigned long long)ld64(SSUM, sl) * (unsigned long long)usum0);
      pend_min += (replicas - rpods) * n;
      nmin_spot += nsp * n;
      nmin_od += nod * n;
      tq = t;
    }
    int pd = 0, step_last_type = 0xFFFF;
    uint32_t flags = 0;
    bool g_acted = false, hchg = false, jchg = false;
    uint32_t emp_e = 0, weou_e = 0;
    HpaOut hp{};
    const int minute = (sm0 + t) % 1440;
    const int hr = minute / 60;
    const int rh = r * 24 + hr;
    if (hr != hour) {  // this hour's prices and carbon intensity
      if (hour >= 0) {  // the carbon of the hour that ended
        std_(GCO2, sl, ldd(GCO2, sl) + (double)e_hour * (ldd(CI, sl) * 1e-9));
        st64(EN, sl, ld64(EN, sl) + e_hour);
      }
      e_hour = 0;
      hour = hr;
      hchg = true;
    }
    // ---- B. readiness ----
    if (t >= next_ready) {
      next_ready = 0x7fffffff;
#pragma unroll
      for (int n = 0; n < MAXN; ++n) {
        if ((used & ~rdy) >> n & 1u) {
          if (sready[n] <= t) {
            rdy |= 1u << n;
            rpods += spods[n];
            if (cmask >> n & 1u) Ffree += scap[n] - spods[n];
          } else {
            next_ready = min(next_ready, sready[n]);
          }
        }
      }
    }
    // ---- A. profile ----
    const bool in_win = ps_raw <= pe_raw ? (minute >= ps_raw && minute < pe_raw) : (minute >= ps_raw || minute < pe_raw);
    const bool peak = pswitch && in_win;
    const int prof = peak ? CCKA_PROFILE_PEAK : CCKA_PROFILE_OFFPEAK;
    if (peak) flags |= 1u;
    if (prof != profile) {
      profile = prof;
      const int pold0 = pcas[0], pold1 = pcas[1];
#pragma unroll
      for (int q = 0; q < MAXP; ++q) {
        if (q >= NP) break;
        const D1Patch& x = p.patch[q][prof + 1];
        if (x.policy) ppol[q] = x.policy;
        if (x.cas >= 0) pcas[q] = casc(x.cas);
        if (x.zi >= 0) pzi[q] = x.zi;
        if (x.cm) pcm[q] = (uint32_t)x.cm;
      }
      // consolidateAfter may have changed: per-slot copies and thresholds
#pragma unroll
      for (int n = 0; n < MAXN; ++n)
        if (used >> n & 1u) {
          const int m1 = -(int)(sinfo[n] >> 13 & 1u);
          slc[n] += cas_slot(n) - casc(pold0 ^ ((pold0 ^ pold1) & m1));  // the slot's value before the switch
        }
      jchg = true;
    }
    // ---- C. HPA / KEDA ----
    {
      const int cur = replicas;
      if constexpr (KEDA) hp = keda_eval(L, cur, t);
      else hp = hpa_eval(L, cur, rpods, __builtin_amdgcn_rcpf((float)(rpods * req)), __builtin_amdgcn_rcpf((float)(cur * req)));
      const int rv = min(max(hp.proposal, -D1_REC_SAT - 1), D1_REC_SAT);
      ring_push<HW>(hdn, hp.ran ? rv : (int)0x8000);
      replicas = hp.desired;
    }
    // ---- D. ReplicaSet reconcile (nominated first, then running; high slot first) ----
    if (placed > replicas) {
      int excess = placed - replicas;
      placed = replicas;
#pragma unroll
      for (int pass = 0; pass < 2; ++pass) {
        const uint32_t m = pass == 0 ? (used & ~rdy) : rdy;
        if (!m || excess <= 0) continue;
        int removed = 0, removed_c = 0;
#pragma unroll
        for (int n = MAXN - 1; n >= 0; --n) {
          const int k = (m >> n & 1u) ? min(spods[n], excess) : 0;
          spods[n] -= k;
          excess -= k;
          removed += k;
          if (pass == 1) removed_c += (cmask >> n & 1u) ? k : 0;
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
        const uint32_t m = (pass == 0 ? rdy : (used & ~rdy)) & cmask;
        if (!m || pd <= 0) continue;
        int added = 0;
#pragma unroll
        for (int n = 0; n < MAXN; ++n) {
          const int fr = (m >> n & 1u) ? scap[n] - spods[n] : 0;
          const int k = min(fr, pd);
          spods[n] += k;
          pd -= k;
          added += k;
          slc[n] = k > 0 ? t + cas_slot(n) : slc[n];
        }
        placed += added;
        if (pass == 0) { rpods += added; Ffree -= added; }
      }
    }
    // ---- the hour's prices and carbon intensity, the pools' J ----
    if (hchg) {
      const int64_t toff = (int64_t)rh * K * Z * 2;
      const GLOBAL_AS int32_t* tile = price + toff;
      const int* stile = s_price + toff;
      std_(CI, sl, ldt ? s_ci[rh] : ci_gpwmin[rh]);
      base_price = (long long)base_nodes * (ldt ? stile[(base_type * Z) * 2 + 1] : tile[(base_type * Z) * 2 + 1]);
      burn = 0;
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
      if (pd > 0 && fm) {
        int q = -1, J = 0, zq = 0, cq = 0;
        uint32_t cm = 0;
#pragma unroll
        for (int qq = MAXP - 1; qq >= 0; --qq) {
          const uint32_t c2 = pcm[qq] & capsel;
          if (qq < NP && c2 && pJ[qq] > 0) { q = qq; J = pJ[qq]; cm = c2; zq = pzi[qq]; cq = pcas[qq]; }
        }
        if (q >= 0) {
          const GLOBAL_AS int2* row = table + ((((int64_t)rh * NZI + zq) * 3 + (cm - 1)) * NW + wi) * JT;
          uint32_t last_choice = 0, hash = (uint32_t)*S(HASH, sl);
          while (pd > 0 && fm) {
            const int slot = __ffs((int)fm) - 1;
            fm &= fm - 1;
            const int k = min(J, pd);
            const int2 e = d1_tload(row + k);  // never empty: k <= J
            const int info = e.y, prc = e.x;
            const int bk = info & 1023, bz = info >> 10 & 3, bc = info >> 12 & 1, cap1 = info >> 16;
            const int rs = t + delay;
            const int4 ac = s_acc[bk];
#pragma unroll
            for (int n = 0; n < MAXN; ++n) {
              if (n == slot) {
                sinfo[n] = (uint32_t)(bk | bz << 10 | bc << 12 | q << 13);
                sready[n] = min(rs, 0xFFFF);
                slc[n] = t + casc(cq);
                spods[n] = k;
                sprice[n] = prc;
                scap[n] = cap1;
              }
            }
            const uint32_t bit = 1u << slot;
            used |= bit;
            if (capbit1(bc) & capsel) cmask |= bit;
#pragma unroll
            for (int qq = 0; qq < MAXP; ++qq) if (qq == q) pmask[qq] |= bit;
            placed += k;
            minscap = min(minscap, cap1);
            Isum += ((long long)ac.y << 32) | (unsigned)ac.x;
            if (delay == 0) {
              rdy |= bit;
              rpods += k;
              if (cmask & bit) Ffree += cap1 - k;
            } else {
              next_ready = min(next_ready, rs);
            }
            if (bc == 0) nsp++; else nod++;
            burn += prc;
            launches++;
            last_choice = (uint32_t)bk | (uint32_t)bz << 12 | (uint32_t)bc << 14 | (uint32_t)q << 16;
            hash = (hash ^ last_choice) * 16777619u;
            step_last_type = bk;
            flags |= 2u;
            pd -= k;
          }
          *S(LC, sl) = (int)last_choice;
          *S(HASH, sl) = (int)hash;
        }
      }
    }
    // ---- G. disruption (SEMANTICS §3.G) ----
    {
      uint32_t elig = 0, emp = 0;
#pragma unroll
      for (int n = MAXN - 1; n >= 0; --n) {
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
      const uint32_t gate = elig & (emp | (Ffree >= minscap ? weou : (weou & ~cmask)));
      if (gate) {
        bool any_del = false;
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
          while (deleted < qbudget) {
            const uint32_t cand = elig & pmask[q];
            const uint32_t ce = cand & emp;
            if (!ce && !(weou_q && (cand & ~emp) && (Ffree >= minscap || (cand & ~emp & ~cmask)))) break;
            int best = -1, bpods = 0, bprice = -1, bcap = 0;
            uint32_t binfo = 0;
            if (ce) {
#pragma unroll
              for (int n = 0; n < MAXN; ++n) {
                const bool cb = (ce >> n & 1u) && sprice[n] > bprice;
                best = cb ? n : best;
                bprice = cb ? sprice[n] : bprice;
                bcap = cb ? scap[n] : bcap;
                binfo = cb ? sinfo[n] : binfo;
              }
            } else {
              unsigned long long bkey = ~0ull;
#pragma unroll
              for (int n = 0; n < MAXN; ++n) {
                const int pods = spods[n];
                const int need = (cmask >> n & 1u) ? scap[n] : pods;
                const bool ok = (cand >> n & 1u) && need <= Ffree && (!pdb_member || pods <= allowed);
                const unsigned long long key = (unsigned long long)pods << 36 |
                                               (unsigned long long)(0x7fffffff - sprice[n]) << 4 | (unsigned)n;
                const bool cb = ok && key < bkey;
                bkey = cb ? key : bkey;
                bcap = cb ? scap[n] : bcap;
                binfo = cb ? sinfo[n] : binfo;
              }
              if (bkey != ~0ull) {
                best = (int)(bkey & 15u);
                bpods = (int)(bkey >> 36);
                bprice = 0x7fffffff - (int)((bkey >> 4) & 0x7fffffffull);
                int need = bpods;
                const uint32_t recv = rdy & cmask & ~(1u << best);
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
#pragma unroll
            for (int n = 0; n < MAXN; ++n) {
              spods[n] = n == best ? 0 : spods[n];
            }
            if ((binfo >> 12 & 1u) == 0) nsp--; else nod--;
            burn -= bprice;
            const int4 ac = s_acc[binfo & 1023u];
            Isum -= ((long long)ac.y << 32) | (unsigned)ac.x;
            Ffree -= ((rdy & cmask) >> best & 1u) ? bcap : bpods;
            const uint32_t nb = ~(1u << best);
            used &= nb; rdy &= nb; cmask &= nb;
#pragma unroll
            for (int qq = 0; qq < MAXP; ++qq) pmask[qq] &= nb;
            if (pdb_member) allowed -= bpods;
            deleted++;
            deletions++;
            any_del = true;
            flags |= 4u;
            elig &= nb;
            emp &= nb;
            if (bpods > 0) {
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
        }
        if (any_del) {
          g_acted = true;
          minscap = 0x7fffffff;
#pragma unroll
          for (int n = 0; n < MAXN; ++n) minscap = (used >> n & 1u) ? min(minscap, scap[n]) : minscap;
        }
      }
      emp_e = emp;
    }
    // ---- H. accounting ----
    unsigned long long Ssum = 0;
    float Rmax = 0.f;
#pragma unroll
    for (int n = 0; n < MAXN; ++n) {
      const uint32_t pr = (rdy >> n & 1u) ? (uint32_t)spods[n] : 0u;
      Ssum += (unsigned long long)dyn_of(n) * pr;
      Rmax = fmaxf(Rmax, (float)pr * __builtin_amdgcn_rcpf((float)alloc_of(n)));
    }
    {
      const float rbp = __builtin_amdgcn_rcpf((float)rpods);
      const int upp = upp_of(L, rbp);
      long long e_step = base_nw + Isum;
      if ((float)upp * Rmax < 0.9999f) e_step += (long long)(Ssum * (unsigned long long)(uint32_t)upp);
      else e_step += dyn_energy(upp);
      cost += burn + base_price;
      e_hour += e_step;
    }
    const int pending = replicas - rpods;
    const bool slo_s = KEDA ? (k_act_step && replicas == 0) : (hp.ran && hp.util > slo_util);
    if (pending > 0 || slo_s) { slo++; flags |= 8u; }
    pend_min += pending;
    nmin_spot += nsp;
    nmin_od += nod;
    peak_nodes = max(peak_nodes, nsp + nod);
    tq = t + 1;
    d1_store_rec(trs, sl * T * 16 + t * 16,
                 make_int4(replicas, pending, (nsp & 0xFFFF) | nod << 16, (step_last_type & 0xFFFF) | (int)(flags << 16)));

    // ---- caches of the quiet steps that follow ----
    constexpr int UQ = 1 << 20;  // quiet usages: [0, 2^20)
    auto umin = [](int u, uint32_t d) -> int {
      const unsigned long long a = (unsigned long long)(uint32_t)u * d;
      return a > 100ull * UQ ? UQ : min((int)(((uint32_t)a + 99u) / 100u), UQ);
    };
    const bool hpa_path = !(replicas == 0 && minr != 0);
    bool met = replicas <= mx && replicas >= minr && rpods > 0 && hpa_path;
    const int dnm = replicas > mx ? mx : (replicas < minr && hpa_path ? minr : replicas);
    const bool pend = replicas > rpods;
    const uint32_t dreq = (uint32_t)rpods * (uint32_t)req;
    int ulim = 0, pge = UQ, slo_thr = pend ? 0 : UQ;
    bool qkcd = false;
    if (met) {
      int uge = ulo;
      int lim;
      if (pend) {
        lim = max(umin(target + 1, dreq), umin(uhi + 1, (uint32_t)replicas * (uint32_t)req));
      } else {
        bool sl2 = false;
        const int cq = fdiv_nb(target + replicas - 1, replicas, __builtin_amdgcn_rcpf((float)replicas), sl2);
        int us = target - cq + 1;
        const int um = us - 1;
        if (um >= 0) {
          const int xm = um * replicas;
          const int qm = fdiv_nb(xm, target, rtarget, sl2);
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
      ulim = UQ;
    }
    if constexpr (KEDA) {
      met = false;
      ulim = 0;
      pge = UQ;
      slo_thr = pend ? 0 : UQ;
      if (replicas == 0) {
        ulim = (int)min(max((long long)kact + 1, 0LL), (long long)UQ);
        pge = 0;
      } else if (replicas >= minr && replicas <= mx) {
        met = true;
        qkcd = kmin0;
        keda_band(replicas);
        ulim = replicas >= mx ? UQ : (int)min((long long)q_khi + 1, (long long)UQ);
        const long long lc = (long long)(replicas - 1) * kthr + 1;
        pge = (int)max(0LL, min(min((long long)q_klo, lc), (long long)UQ));
      }
    }
    const float rbp2 = rpods > 0 ? __builtin_amdgcn_rcpf((float)rpods) : 0.f;
    (void)rbp2;
    const int usat = Rmax > 0.f ? (int)fminf(0.9999f * __builtin_amdgcn_rcpf(Rmax), 1073741824.0f) - 1 : 0x7fffffff;
    // newest history record >= the new replica count
    int qhold;
    {
      int hit = -0x40000000;
#pragma unroll
      for (int k = 2 * HW - 1; k >= 0; --k) {
        const int e = (int)(short)(hdn[k >> 1] >> (16 * (k & 1)));
        hit = e >= replicas ? t - k : hit;
      }
      qhold = replicas <= minr ? 0x3fffffff : hit + wl;
      if (!met) qhold = 0x3fffffff;
    }
    // first step that needs the event path again
    int nx;
    {
      const int th = t + 60 - minute % 60;
      nx = min(next_ready, th);
      if (pswitch) {
        if (t >= npb) {
          const int dps = (ps - minute + 1439) % 1440 + 1, dpe = (pe - minute + 1439) % 1440 + 1;
          npb = t + min(dps, dpe);
        }
        nx = min(nx, npb);
      }
      const uint32_t gm = rdy & (emp_e | (Ffree >= minscap ? weou_e : (weou_e & ~cmask)));
#pragma unroll
      for (int n = 0; n < MAXN; ++n) nx = ((gm >> n & 1u) && slc[n] > t) ? min(nx, slc[n]) : nx;
      if (g_acted) nx = t + 1;
    }

    // ---- state back to LDS ----
#pragma unroll
    for (int n = 0; n < MAXN; ++n) {
      *S(SA + n, sl) = (int)(sinfo[n] & 0xFFFFu) | spods[n] << 16;
      *S(SB + n, sl) = (sready[n] & 0xFFFF) | ((slc[n] - cas_slot(n)) & 0xFFFF) << 16;
      *S(SP + n, sl) = sprice[n];
    }
    *S(MASK, sl) = (int)(used | rdy << 8 | cmask << 16 | pmask[0] << 24);
    *S(PCAS, sl) = pcas[0] | pcas[1] << 16;
    *S(POOL, sl) = ppol[0] | ppol[1] << 4 | (pzi[0] + 1) << 8 | (pzi[1] + 1) << 12 | (int)pcm[0] << 16 |
                   (int)pcm[1] << 18 | (profile + 1) << 20 | (hour + 1) << 22 | peak_nodes << 27;
    *S(PJ, sl) = pJ[0] | pJ[1] << 16;
    *S(REP, sl) = replicas | placed << 16;
    *S(RP, sl) = rpods | nsp << 16 | nod << 24;
    *S(NR, sl) = min(next_ready, 0xFFFF) | min(minscap, 0xFFFF) << 16;
    *S(FF, sl) = Ffree;
    st64(COST, sl, ld64(COST, sl) + cost); st64(BURN, sl, burn); st64(BASEP, sl, base_price);
    st64(EH, sl, e_hour); st64(ISUM, sl, Isum);
    st64(SSUM, sl, (long long)Ssum);
    *S(PEND, sl) += pend_min; *S(SLO, sl) += slo; *S(NSPM, sl) += nmin_spot; *S(NODM, sl) += nmin_od;
    *S(LAU, sl) += launches; *S(DEL, sl) += deletions;
    *S(TQ, sl) = tq | npb << 16;
    *S(QPGE, sl) = pge | (qkcd ? 1 << 30 : 0) | (met ? (int)0x80000000u : 0);
#pragma unroll
    for (int w = 0; w < HW; ++w) *S(HDN + w, sl) = (int)hdn[w];
    if constexpr (KEDA) { *S(KCD, sl) = kcd_s; *S(KLO, sl) = q_klo; *S(KHI, sl) = q_khi; *S(KBC, sl) = kb_cur; }
    *S(QULIM, sl) = ulim;
    *S(QSLO, sl) = slo_thr;
    *S(QUSAT, sl) = usat;
    *S(QHOLD, sl) = qhold;
    *S(NXT, sl) = nx;
    // the horizon's last step: the results now; else the scenario is ready
    // for a lane (its cache published before its id)
    const bool last = t + 1 >= T;
    if (last) finish(sl, 0u, 0);
    const uint64_t rm = __ballot(!last), lm = __ballot(last);
    if (lm && lane == __ffsll((long long)(lm | rm)) - 1)
      __hip_atomic_fetch_add(n_done, __popcll(lm), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (rm) {
      const int first = __ffsll((long long)rm) - 1;
      int pos = 0;
      if (lane == first) pos = __hip_atomic_fetch_add(r_tail, __popcll(rm), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      pos = __builtin_amdgcn_readlane(pos, first);
      if (!last) {
        const int rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(rm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)rm, 0u));
        lds_drain();
        lds_st(&rqueue[(pos + rank) & (PL_QCAP - 1)], sl + 1);
      }
    }
  };

  // =======================================================================
  // main loop
  // =======================================================================
  // every wave leaves the loop once the workgroup's scenarios are finished;
  // the iteration bound is a safety net against a wedged queue (its results
  // would then be wrong, never a hung device)
  const int it_max = 64 * T + 65536;
  uint64_t sx_it = 0, sx_runs = 0, sx_lanes = 0, sx_cs = 0, sx_cq = 0, sx_ci = 0, sx_live = 0;
  uint64_t sx_e = 0, sx_s = 0, sx_at = 0, sx_pd = 0;
  const uint64_t sx_t0 = STATS ? __builtin_amdgcn_s_memtime() : 0;
  for (int it = 0; it < it_max; ++it) {
    if constexpr (STATS) ++sx_it;
    const bool live = sid >= 0;  // an attached scenario is before its horizon's end
    const uint64_t blive = __ballot(live);
    if constexpr (STATS) sx_live += __popcll(blive);
    // ---- quiet steps: up to PL_S per iteration and lane ----
    bool stall = false;
    const int t_it = t;  // the first step of this iteration's window
    uint64_t sx_a = STATS ? __builtin_amdgcn_s_memtime() : 0;
    if (blive) {
#pragma unroll
      for (int sub = 0; sub < PL_S; ++sub) {
        const int Lv = Lpf[sub];
        const int usage = min(Lv, q_rcap);
        const int cv = KEDA ? Lv : usage;
        const bool ge = cv >= q_pge;
        const int upp = (int)fmaf((float)usage, q_rbp, q_hbp);
        // quiet iff the HPA keeps the count, no event is due and no node
        // saturates (a saturating step takes the event path: its exact energy)
        bool ok = (t < nxt) & ((uint32_t)cv < (uint32_t)q_ulim) & (ge | (t <= q_hold)) & (upp <= q_usat);
        const bool kac = KEDA && Lv > kact;
        if constexpr (KEDA) ok = ok & (!q_kcd | kac | (t < kcd));
        const bool can = live & !stall & (t < T);
        const bool go = ok & can;
        stall = stall | (can & !ok);
        q_hold = (go & ge) ? max(q_hold, t + nd) : q_hold;
        if constexpr (KEDA) kcd = (go & kac) ? t + kcds : kcd;
        usum += go ? (uint32_t)upp : 0u;
        const bool slo_b = usage >= q_slo;
        sloq += (go & slo_b) ? 1 : 0;
        d1_store_rec(trs, go ? lb + t * 16 : D1_NOSTORE,
                     make_int4(replicas_q, q_pendv, q_nodes, slo_b ? (q_w0 | 8 << 16) : q_w0));
        t += go ? 1 : 0;
      }
    }
    if constexpr (STATS) { const uint64_t b = __builtin_amdgcn_s_memtime(); sx_cq += b - sx_a; sx_a = b; }
    // ---- the window this iteration stepped through (the server rebuilds the
    // down-window records of a scenario's quiet steps from its last two) ----
    if (live) {
      typedef int i32x4 __attribute__((ext_vector_type(4)));
      i32x4* const w = reinterpret_cast<i32x4*>(s_win + ((it & 1) * SBn + sid) * 8);
      w[0] = i32x4{Lpf[0], Lpf[1], Lpf[2], Lpf[3]};
      w[1] = i32x4{Lpf[4], Lpf[5], Lpf[6], Lpf[7]};
    }
    // ---- scenarios that reached the horizon's end leave with their results ----
    const bool fin = live && !stall && t >= T;
    const uint64_t bfin = __ballot(fin);
    if (bfin) {
      if (fin) { finish(sid, usum, sloq); sid = -1; }
      if (lane == __ffsll((long long)bfin) - 1)
        __hip_atomic_fetch_add(n_done, __popcll(bfin), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    // ---- stalled scenarios join the event queue and leave their lanes ----
    const uint64_t nm = __ballot(stall);
    if (nm) {
      const int first = __ffsll((long long)nm) - 1;
      int pos = 0;
      if (lane == first) pos = __hip_atomic_fetch_add(q_tail, __popcll(nm), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      pos = __builtin_amdgcn_readlane(pos, first);
      if (stall) {
        *S(TEV, sid) = t | (t - t_it) << 16 | (it & 1) << 19;
        *S(USUM, sid) = (int)usum;
        *S(SLO, sid) += sloq;
        if constexpr (KEDA) *S(KCD, sid) = kcd;
        const int rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(nm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)nm, 0u));
        lds_drain();
        lds_st(&queue[(pos + rank) & (PL_QCAP - 1)], sid + 1);
        sid = -1;
      }
    }
    if constexpr (STATS) { const uint64_t b = __builtin_amdgcn_s_memtime(); sx_e += b - sx_a; sx_a = b; }
    // ---- server role: serve a full batch, or whatever waits once the last
    // claim is pool_age cycles old (s_memtime) or this wave has nothing to step ----
    const uint64_t batt = __ballot(sid >= 0);
    {
      int qn = 0, aged = 0;
      if (lane == 0) {
        qn = lds_ld(q_tail) - lds_ld(q_head);
        aged = (int)((uint32_t)__builtin_amdgcn_s_memtime() - (uint32_t)lds_ld(q_head + 2)) > pool_age;
      }
      qn = __builtin_amdgcn_readfirstlane(qn);
      aged = __builtin_amdgcn_readfirstlane(aged);
      if (qn >= pool_min || (qn > 0 && (aged || (!batt && pool_idle)))) {
        int h = 0, c = 0;
        if (lane == 0) {
          for (;;) {
            h = lds_ld(q_head);
            c = min(WAVE, lds_ld(q_tail) - h);
            if (c <= 0) { c = 0; break; }
            int exp = h;
            if (__hip_atomic_compare_exchange_strong(q_head, &exp, h + c, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_WORKGROUP)) {
              lds_st(q_head + 2, (int)(uint32_t)__builtin_amdgcn_s_memtime());
              break;
            }
          }
        }
        h = __builtin_amdgcn_readfirstlane(h);
        c = __builtin_amdgcn_readfirstlane(c);
        if (c > 0) {
          __builtin_amdgcn_s_setprio(PL_PRIO_HI);
          if constexpr (STATS) { sx_runs += 1; sx_lanes += c; const uint64_t b = __builtin_amdgcn_s_memtime(); sx_s += b - sx_a; sx_a = b; }
          serve(h, c);
          if constexpr (STATS) { const uint64_t b = __builtin_amdgcn_s_memtime(); sx_cs += b - sx_a; sx_a = b; }
          __builtin_amdgcn_s_setprio(0);
        }
      }
    }
    if constexpr (STATS) { const uint64_t b = __builtin_amdgcn_s_memtime(); sx_s += b - sx_a; sx_a = b; }
    // ---- free lanes take served scenarios from the ready queue ----
    const uint64_t bfree = __ballot(sid < 0);
    {
      int rh = 0, k = 0;
      if (lane == 0) {
        for (;;) {
          rh = lds_ld(r_head);
          k = min(__popcll(bfree), lds_ld(r_tail) - rh);
          if (k <= 0) { k = 0; break; }
          int exp = rh;
          if (__hip_atomic_compare_exchange_strong(r_head, &exp, rh + k, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_WORKGROUP))
            break;
        }
      }
      rh = __builtin_amdgcn_readfirstlane(rh);
      k = __builtin_amdgcn_readfirstlane(k);
      if (k > 0) {
        const int rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(bfree >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bfree, 0u));
        if (sid < 0 && rank < k) {
          int e = 0;
          do {
            e = __hip_atomic_exchange(&rqueue[(rh + rank) & (PL_QCAP - 1)], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          } while (e == 0);  // reserved by a server that has not written it yet
          asm volatile("" ::: "memory");
          sid = e - 1;
          const uint32_t wtev = (uint32_t)*S(TEV, sid);
          t = (int)(wtev & 0xFFFFu) + 1;
          nxt = *S(NXT, sid);
          usum = 0;
          sloq = 0;
          q_ulim = *S(QULIM, sid);
          q_slo = *S(QSLO, sid);
          q_usat = *S(QUSAT, sid);
          q_hold = *S(QHOLD, sid);
          const uint32_t wqp = (uint32_t)*S(QPGE, sid);
          q_pge = (int)(wqp & 0x3FFFFFFFu);
          q_kcd = (wqp >> 30 & 1u) != 0;
          if constexpr (KEDA) kcd = *S(KCD, sid);
          const uint32_t wrep = (uint32_t)*S(REP, sid), wrp = (uint32_t)*S(RP, sid);
          replicas_q = (int)(wrep & 0xFFFFu);
          const int rp = (int)(wrp & 0xFFFFu);
          q_nodes = (int)(wrp >> 16 & 0xFFu) | (int)(wrp >> 24) << 16;
          q_pendv = replicas_q - rp;
          q_rcap = limit > 0 ? (int)__umul24((uint32_t)rp, (uint32_t)limit) : 0x7fffffff;
          q_rbp = rp > 0 ? __builtin_amdgcn_rcpf((float)rp) : 0.f;
          q_hbp = 0.5f * q_rbp;
          const bool pk = ((uint32_t)*S(POOL, sid) >> 20 & 3u) == (uint32_t)(CCKA_PROFILE_PEAK + 1);
          q_w0 = 0xFFFF | (int)((pk ? 1u : 0u) << 16);
          nd = (int)((uint32_t)*S(C2, sid) >> 19 & 31u);
          sbase = sample_base(sid);
          lb = sid * T * 16;
        }
      }
    }
    if constexpr (STATS) { const uint64_t b = __builtin_amdgcn_s_memtime(); sx_at += b - sx_a; sx_a = b; }
    // ---- the attached scenarios' next samples ----
    prefetch(t);
    // ---- done, or nothing to do for now ----
    int nd_all = 0;
    if (lane == 0) nd_all = lds_ld(n_done);
    nd_all = __builtin_amdgcn_readfirstlane(nd_all);
    if constexpr (STATS) { const uint64_t b = __builtin_amdgcn_s_memtime(); sx_pd += b - sx_a; sx_a = b; }
    if (nd_all >= nblk) break;
    if (!__ballot(sid >= 0)) {
      if constexpr (STATS) sx_a = __builtin_amdgcn_s_memtime();
      __builtin_amdgcn_s_sleep(4);
      if constexpr (STATS) sx_ci += __builtin_amdgcn_s_memtime() - sx_a;
    }
  }
  if constexpr (STATS) {
    if (lane == 0) {
      atomicMax(&p.stamps[0], (unsigned long long)sx_it);
      atomicAdd(&p.stamps[1], (unsigned long long)sx_it);
      atomicAdd(&p.stamps[2], (unsigned long long)sx_runs);
      atomicAdd(&p.stamps[3], (unsigned long long)sx_lanes);
      atomicAdd(&p.stamps[4], (unsigned long long)sx_cs);
      atomicAdd(&p.stamps[5], (unsigned long long)sx_cq);
      atomicAdd(&p.stamps[6], (unsigned long long)sx_ci);
      atomicAdd(&p.stamps[7], (unsigned long long)(__builtin_amdgcn_s_memtime() - sx_t0));
      atomicAdd(&p.stamps[8], (unsigned long long)sx_live);
      atomicAdd(&p.stamps[9], (unsigned long long)sx_e);
      atomicAdd(&p.stamps[10], (unsigned long long)sx_s);
      atomicAdd(&p.stamps[11], (unsigned long long)(sx_at + sx_pd));
    }
  }
}

hipError_t launch_rollout_pool(const D1Params& p, hipStream_t s) {
  const int sb = 8 * p.lpw;
  const int64_t grid = (p.N + sb - 1) / sb;
  const int hw = p.he4 ? 2 : 4;
  const PoolLds ly = pool_lds_layout(p.K, p.R, p.Z, p.NZI, p.lds_tab, sb, hw);
  if (p.stamps) {  // diagnostic counters (default-behavior worlds)
    if (p.he4) hipLaunchKernelGGL((rollout_pool_kernel<4, false, true>), dim3((unsigned)grid), dim3(PL_BLOCK), ly.total, s, p);
    else hipLaunchKernelGGL((rollout_pool_kernel<8, false, true>), dim3((unsigned)grid), dim3(PL_BLOCK), ly.total, s, p);
  } else if (p.keda) {
    if (p.he4) hipLaunchKernelGGL((rollout_pool_kernel<4, true, false>), dim3((unsigned)grid), dim3(PL_BLOCK), ly.total, s, p);
    else hipLaunchKernelGGL((rollout_pool_kernel<8, true, false>), dim3((unsigned)grid), dim3(PL_BLOCK), ly.total, s, p);
  } else {
    if (p.he4) hipLaunchKernelGGL((rollout_pool_kernel<4, false, false>), dim3((unsigned)grid), dim3(PL_BLOCK), ly.total, s, p);
    else hipLaunchKernelGGL((rollout_pool_kernel<8, false, false>), dim3((unsigned)grid), dim3(PL_BLOCK), ly.total, s, p);
  }
  return hipGetLastError();
}

}  // namespace ccka
