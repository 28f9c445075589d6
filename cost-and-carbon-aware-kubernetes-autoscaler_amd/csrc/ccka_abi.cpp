// ccka_abi.cpp — the C ABI of libccka.so (include/ccka.h).
//
// Owns the device buffers of one context, validates the world against the
// engine's limits, chooses the launch geometry (LDS budget per workgroup from
// the catalog, the price-tile span and the NodeClaim scratch) and drives the
// kernels in rollout.hip on the context's stream. Multi-GPU: one context per
// GPU; totals are summed with RCCL over xGMI (the only cross-GPU exchange:
// scenarios are independent).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdarg>
#include <map>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "../../include/ccka.h"
#include "kparams.h"

using namespace ccka;

struct ccka_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev_mid = nullptr, ev1 = nullptr;  // ev_mid: after the argmin tables
  std::string err;
  int cus = 0;
  char name[128] = {0};
  // world
  bool have_world = false;
  ccka_world hw{};
  ccka_world* d_world = nullptr;
  ccka_itype* d_types = nullptr;
  int32_t* d_price = nullptr;
  double* d_ci_gpwh = nullptr;
  double* d_ci_gpwmin = nullptr;
  int prov[CCKA_MAX_DEPLOY] = {0};
  // scenarios
  bool have_sc = false;
  int64_t N = 0, first_id = 0, n_traces = 0;
  std::vector<uint8_t> h_region;
  uint8_t* d_region = nullptr;
  int16_t* d_target = nullptr;
  int16_t* d_maxr = nullptr;
  int16_t* d_dstab = nullptr;
  int16_t* d_resetca = nullptr;
  uint8_t* d_pswitch = nullptr;
  double* d_cw = nullptr;
  uint8_t* d_capsel = nullptr;
  // traces / outputs
  int32_t* d_load = nullptr;
  int64_t load_count = 0;
  bool have_load = false;
  // wave-tiled copy of the trace for the single-deployment kernel (d1_trace_tile)
  int32_t* d_load_w = nullptr;
  int64_t load_w_count = 0;
  int32_t load_w_lpw = 0;  // lanes per wave it was tiled for (0: stale)
  // scenario-major copy [NL][T][DP] of the trace for the general kernel's
  // lane-skewed schedule (sk_trace); load_nt_dp = the DP it was built for (0: stale)
  int32_t* d_load_nt = nullptr;
  int64_t load_nt_count = 0;
  int32_t load_nt_dp = 0;
  bool trace_flat = false;  // ccka_debug_trace_flat: read [T][N] (A/B of the layout)
  void* d_res = nullptr;  // one allocation, SoA carve
  KParams kp{};
  ccka_traj_rec* d_traj = nullptr;
  int64_t traj_count = 0;
  bool traj_valid = false;
  bool traj_nt = false;              // device records are [N][T] (single-deployment engine)
  ccka_traj_rec* d_traj_t = nullptr;  // [T][N] staging blocks for ccka_get_trajectory
  int64_t traj_t_count = 0;
  void* d_parts = nullptr;
  ccka_totals* d_totals = nullptr;
  int32_t* d_sinq = nullptr;
  ncclComm_t comm = nullptr;
  double last_ms = 0.0;        // rollout kernel (HIP events on the engine stream)
  double last_table_ms = 0.0;  // argmin-table kernel of the same rollout
  bool ran = false;
  // single-deployment engine (rollout_d1.hip): world digest, argmin tables
  bool d1_world = false;     // the world qualifies (d1_check_world)
  bool d1_ready = false;     // scenario-dependent part prepared
  bool d1_ok = false;        // world + scenarios qualify
  bool sc_maxr_ok = true;
  int sc_dstab_max = -1;      // largest per-scenario down_stab_s override (-1: none given)
  // HPA decision history in HBM for long windows / sub-steps (general kernel)
  int2* d_hist = nullptr;
  int64_t hist_count = 0;
  uint32_t sc_capsel_or = 0;  // OR of the per-scenario cap_sel overrides (0: none given)
  int sc_pswitch_any = -1;    // any per-scenario peak_switch set (-1: none given)
  D1Params d1{};
  std::vector<uint32_t> zmasks;
  std::vector<double> h_cw;  // per-scenario carbon weights (empty: world default)
  long long* d_acc = nullptr;
  int32_t* d_order = nullptr;
  int32_t* d_cap1s = nullptr;
  int32_t* d_cap1t = nullptr;  // pod capacity per type (argmin-table entries)
  uint32_t* d_zmasks = nullptr;
  double* d_wc1000 = nullptr;
  uint8_t* d_wci = nullptr;
  int2* d_table = nullptr;
  int32_t* d_jtab = nullptr;
  int2* d_table2 = nullptr;   // G2 offer table (replacement consolidation in the single-deployment kernel)
  int32_t* d_jtab2 = nullptr;
  double* d_wc0 = nullptr;    // one zero carbon weight (the offer table's score is the price)
  int JT = 0, NW = 0;
  int engine_mode = 0;       // 0 auto, 1 general kernel only, 2 general kernel in lockstep (ccka_debug_engine)
  bool sk_coop_f2 = false;   // skewed schedule: keep the wave-cooperative provisioning (ccka_debug_engine 3)
#ifndef SK_LANE_F2
#define SK_LANE_F2 0
#endif
  bool sk_lane_f2 = SK_LANE_F2 != 0;  // lane-local provisioning compiled in (variant builds)
  unsigned long long* d_stamps = nullptr;
  int lpw = 0;               // scenarios per wave of the single-deployment kernel (0 = automatic)
  int occ = 0;               // its register-allocation occupancy target (0 = automatic)
  int pool_mode = 0;         // 1: pooled event steps (rollout_pool.hip, an A/B engine: measured slower) where eligible
  int pool_min = 48;         // queue length at which a wave serves it
  int pool_age = 20000;      // or any waiting entries once the last claim is this many cycles old
  int pool_idle = 1;         // or any waiting entries when none of its own lanes can step
  bool last_pooled = false;  // the last single-deployment rollout ran the pooled kernel
  int mlp_stamps = 0;        // diagnostic MLP phase stamps (ccka_debug_mlp_stamps)
  // policy sweep (config 4)
  ccka_grid_stats* d_gstats = nullptr;   // [grids] then [2 * grids] scratch
  ccka_grid_stats* d_gcand = nullptr;
  ccka_grid_stats* d_ggather = nullptr;
  int64_t* d_gcounts = nullptr;
  int32_t* d_gn = nullptr;
  uint8_t* d_gflags = nullptr;
  ccka_grid_stats* d_gfront = nullptr;   // the frontier (local or global)
  int64_t gcap = 0;
  int64_t pcap_ng = 0;
  int pcap_ranks = 0;
  // learned MLP policy (config 5)
  bool mlp_have_w = false;
  mlp_bf16x8* d_w1f = nullptr;
  mlp_bf16x8* d_w2f = nullptr;
  mlp_bf16x8* d_w3f = nullptr;
  // the standalone forward's fragments for v_mfma_f32_16x16x32_bf16 (mlp16_kernel)
  mlp_bf16x8* d_w1g = nullptr;
  mlp_bf16x8* d_w2g = nullptr;
  mlp_bf16x8* d_w3g = nullptr;
  int mlp_tile = 16;         // standalone forward: 16 (mlp16_kernel) or 32 (mlp_kernel; ccka_debug_mlp_tile)
  float* d_mb = nullptr;  // b1[256] b2[256] b3[8]
  uint16_t* d_mx = nullptr;
  float* d_my = nullptr;
  int64_t mlp_n = 0, mlp_cap = 0;
  int last_engine = 0;       // 1 general, 2 single-deployment
  // closed-loop policy rollout (config 5)
  int32_t* d_pol_state = nullptr;
  int64_t pol_state_count = 0;
  int16_t* d_pol_target = nullptr;
  double* d_pol_cw = nullptr;
  int64_t pol_n = 0;
  int16_t* d_rec_target = nullptr;
  double* d_rec_cw = nullptr;
  int64_t pol_rec_count = 0;
  bool pol_rec_valid = false;
  bool pol_feat_on = false;
  // the closed loop's launch sequence captured as one hipGraph, replayed while
  // its inputs (launch parameters, buffers, sizes) are unchanged
  hipGraphExec_t pol_graph = nullptr;
  std::vector<unsigned char> pol_graph_key;
  bool pol_graph_off = false;  // ccka_debug_policy_graph(0): launch the sequence directly
  bool pol_fused_off = false;  // ccka_debug_policy_fused(0): the launched loop even where the fused one applies
  bool pol_table_off = false;  // ccka_debug_policy_table(0): the fused loop's catalog scans instead of the tables
  int64_t pg_chunk = 0;        // ccka_debug_pg_chunk: rows per backward chunk (0: kPgChunkRows)
  int2* d_ptable = nullptr;    // the fused loop's argmin tables (65 policy carbon weights)
  int32_t* d_pjtab = nullptr;
  double* d_pwc = nullptr;
  int64_t ptable_count = 0;
  uint16_t* d_feat_rec = nullptr;
  int64_t pol_feat_count = 0;
  // differentiable control (ccka_policy_grad / ccka_mlp_backward, pg.hip)
  mlp_bf16x8* d_w2b = nullptr;   // A fragments of dH1^T = W2 dH2^T
  mlp_bf16x8* d_w3b = nullptr;   // A fragments of dH2^T = W3 g_y^T
  uint8_t* d_pg_act = nullptr;   // sampled actions [T][N] (or the rows of ccka_mlp_backward)
  int64_t pg_act_count = 0;
  float* d_pg_coef = nullptr;    // per-scenario (J - b) / N (or per row)
  uint64_t* d_pg_seed = nullptr; // the sampling key of the stochastic loop (outside the graph key)
  uint64_t pg_seed_host = 0;
  int64_t pg_coef_count = 0;
  uint16_t* d_pg_x = nullptr;    // ccka_mlp_backward's rows [M][64]
  int64_t pg_x_count = 0;
  uint16_t* d_pg_work = nullptr; // xT | h1T | h2T | dh1T | dh2T | gyT, each row-blocked [Mpad/16][units][16]
  int64_t pg_work_count = 0;
  float* d_pg_part = nullptr;    // weight-gradient row-split partials
  int64_t pg_part_count = 0;
  float* d_pg_grad = nullptr;    // dW1 | db1 | dW2 | db2 | dW3 | db3
  bool pg_valid = false;
  int64_t pg_T = 0;
  // per-scenario summary breakdown (ccka_set_detail)
  bool detail_on = false;
  bool detail_valid = false;
  DetailDev* d_detail = nullptr;
  int64_t detail_count = 0;
};

// staging records of ccka_get_trajectory's [N][T] -> [T][N] transpose (64 MiB)
constexpr int64_t kTrajStageRecs = int64_t(4) << 20;

static int fail(ccka_ctx* c, int code, const char* fmt, ...) __attribute__((format(printf, 3, 4)));
static int fail(ccka_ctx* c, int code, const char* fmt, ...) {
  if (c) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    c->err = buf;
  }
  return code;
}

#define HIPCHK(c, x)                                                              \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess)                                                         \
      return fail((c), CCKA_EHIP, "%s: %s", #x, hipGetErrorString(e_));          \
  } while (0)

template <class T>
static void dfree(T*& p) {
  if (p) { (void)hipFree((void*)p); p = nullptr; }
}

template <class T>
static int dupload(ccka_ctx* c, T*& dst, const T* src, size_t count) {
  dfree(dst);
  if (!src || count == 0) return CCKA_OK;
  if (hipMalloc((void**)&dst, sizeof(T) * count) != hipSuccess)
    return fail(c, CCKA_ENOMEM, "hipMalloc %zu bytes failed", sizeof(T) * count);
  HIPCHK(c, hipMemcpyAsync(dst, src, sizeof(T) * count, hipMemcpyHostToDevice, c->stream));
  return CCKA_OK;
}


// ---------------------------------------------------------------------------
// Single-deployment engine: eligibility and world digest.
// Conditions (anything else runs the general kernel): one HPA Deployment, no
// NodePool CPU limits (the launch choice is then independent of pool usage),
// replica counts and records within int16, tolerance in [0, 1), PDB percent
// <= 100, at most 65535 steps, at most
// D1_MAX_ZI distinct zone masks and D1_MAX_WC distinct carbon weights.
// ---------------------------------------------------------------------------
static int pod_cap(const ccka_itype& t, int rc, int rm) {
  int f = t.max_pods;
  if (rc > 0) f = std::min(f, t.alloc_cpu_m / rc);
  if (rm > 0) f = std::min(f, t.alloc_mem_mi / rm);
  return f;
}

// decisions of the register history rings (8 entries at one decision per
// step) cover the rules: the fast paths; otherwise the HBM history
static bool rules_fit_ring(const ccka_hpa_rules& r) {
  if (r.n_policies > 2 || r.stab_window_s > CCKA_HIST * CCKA_STEP_SECONDS) return false;
  for (int i = 0; i < r.n_policies; ++i)
    if (r.policies[i].period_s > CCKA_HIST * CCKA_STEP_SECONDS) return false;
  return true;
}

static int hist_entries(int window_s, int sync_s) { return window_s > sync_s ? (window_s - 1) / sync_s : 0; }

static D1Rule d1_rule(const ccka_hpa_rules& r, bool up) {
  auto wm = [](int w) {
    int m = 0;
    for (int k = 0; k < CCKA_HIST; ++k) m |= ((k + 1) * CCKA_STEP_SECONDS < w) ? (1 << k) : 0;
    return m;
  };
  D1Rule o{};
  o.sel = r.select;
  o.n = r.n_policies;
  o.stab_mask = wm(r.stab_window_s);
  for (int q = 0; q < 2; ++q) {
    o.type[q] = r.policies[q].type;
    o.value[q] = r.policies[q].value;
    o.pmask[q] = wm(r.policies[q].period_s);
    o.factor[q] = up ? (1.0 + (double)o.value[q] / 100.0) : (1.0 - (double)o.value[q] / 100.0);
  }
  for (int r = 0; r < 4; ++r) {
    auto bit = [](int m, int e) { return (m >> e) & 1; };
    o.stab16[r] = (bit(o.stab_mask, 2 * r) ? 0xFFFF : 0) | (bit(o.stab_mask, 2 * r + 1) ? (int32_t)0xFFFF0000 : 0);
    for (int q = 0; q < 2; ++q) {
      const int m = q < o.n ? o.pmask[q] : 0;
      o.pm16[q][r] = (bit(m, 2 * r) ? 1 : 0) | (bit(m, 2 * r + 1) ? 0x10000 : 0);
    }
  }
  return o;
}

// the rules as the kernel uses them equal the upstream default behavior
// (d1_default_rule; the down stabilisation window is per scenario, not here)
static bool d1_rule_is_default(const D1Rule& r, bool up) {
  const D1Rule d = d1_default_rule(up);
  if (r.sel != d.sel || r.n != d.n || (up && r.stab_mask != 0)) return false;
  for (int q = 0; q < r.n; ++q)
    if (r.type[q] != d.type[q] || r.value[q] != d.value[q] || r.pmask[q] != 0) return false;
  return true;
}

// longest down-stabilisation window the 15 s sync ring holds: 20 records,
// (W - 1) / 15 <= 20
constexpr int kD1Sync15MaxWindow = 315;

static int d1_check_world(ccka_ctx* c) {
  const ccka_world& w = c->hw;
  c->d1_world = false;
  c->d1_ready = false;
  const ccka_deployment& dp = w.deploy[0];
  // one HPA deployment, or one single-trigger KEDA ScaledObject (default
  // behavior, one decision per step: the KEDA instantiation)
  const bool keda = dp.scaler == CCKA_SCALER_KEDA;
  if (w.n_deploy != 1 || (dp.scaler != CCKA_SCALER_HPA && !keda)) return CCKA_OK;
  if (keda && (w.hpa_sync_s == 15 || w.max_nodes > 8 || w.n_pools > 2 || dp.keda_threshold < 1 || dp.keda_threshold >= (1 << 22) ||
               dp.keda_activation < INT32_MIN || dp.keda_activation >= INT32_MAX || dp.keda_min < 0 ||
               dp.keda_min > D1_REC_SAT || dp.keda_max < 0 || dp.keda_max > D1_REC_SAT))
    return CCKA_OK;
  // pool limits run on the general kernel; drift, replacement and multi-node
  // consolidation are checked per scenario set in d1_prepare (d1_disrupt_ok)
  for (int q = 0; q < w.n_pools; ++q)
    if (w.pools[q].limit_cpu_m >= 0 || w.pools[q].limit_mem_mi >= 0) return CCKA_OK;
  // one HPA decision per step over the 8-entry register rings, or the
  // Kubernetes default 15 s sync (four per step) with the default behavior
  // (checked below) over 20-entry rings
  const bool sync15 = w.hpa_sync_s == 15;
  if ((w.hpa_sync_s != 0 && w.hpa_sync_s != CCKA_STEP_SECONDS && !sync15) || !rules_fit_ring(dp.up) ||
      !rules_fit_ring(dp.down))
    return CCKA_OK;
  if (!(dp.tolerance >= 0.0 && dp.tolerance < 1.0) || dp.req_cpu_m < 1 || dp.req_cpu_m > 65535 ||
      dp.limit_cpu_m > 65535 ||
      dp.min_replicas < 0 || dp.max_replicas < 0 || dp.max_replicas > D1_REC_SAT || dp.replicas0 > D1_REC_SAT)
    return CCKA_OK;
  // 32-bit PDB arithmetic (pct x replicas) and pending-pod-minutes (pods x steps)
  if (w.pdb_min_available_pct > 100 || w.n_steps > 65535) return CCKA_OK;
  const int K = w.n_types;
  std::vector<int> cap1(K);
  int jmax = 0;
  for (int k = 0; k < K; ++k) {
    cap1[k] = std::max(0, pod_cap(w.types[k], dp.req_cpu_m, dp.req_mem_mi));
    if (cap1[k] > D1_REC_SAT || w.types[k].alloc_cpu_m >= (1 << 24) || w.types[k].idle_nw < 0 ||
        w.types[k].dyn_nw_per_m < 0 || w.types[k].dyn_nw_per_m > 0xFFFFFFFFLL)
      return CCKA_OK;
    jmax = std::max(jmax, cap1[k]);
  }
  // distinct zone masks of every patch that sets one
  std::vector<uint32_t> zm;
  auto zidx = [&](uint32_t m) -> int {
    if (!m) return -1;
    for (size_t i = 0; i < zm.size(); ++i) if (zm[i] == m) return (int)i;
    zm.push_back(m);
    return (int)zm.size() - 1;
  };
  D1Params& p = c->d1;
  p = D1Params{};
  for (int q = 0; q < w.n_pools; ++q) {
    const ccka_pool_patch* src[4] = {&w.pools[q].base, &w.pools[q].profile[CCKA_PROFILE_RESET],
                                     &w.pools[q].profile[CCKA_PROFILE_OFFPEAK], &w.pools[q].profile[CCKA_PROFILE_PEAK]};
    for (int s = 0; s < 4; ++s) {
      D1Patch& x = p.patch[q][s];
      x.policy = src[s]->policy;
      const int ca = src[s]->consolidate_after_s;
      x.cas = ca >= 0 ? (ca + CCKA_STEP_SECONDS - 1) / CCKA_STEP_SECONDS : -1;
      x.zi = zidx(src[s]->zone_mask & ((1u << w.n_zones) - 1u));
      x.cm = (int32_t)(src[s]->cap_mask & 3u);
    }
    p.budget[q] = w.pools[q].budget_pct;
  }
  if (zm.empty()) zm.push_back(1u);  // no pool ever selects a zone: J = 0 everywhere
  if ((int)zm.size() > D1_MAX_ZI) return CCKA_OK;
  // accounting coefficients and the catalog in pod-capacity-descending order
  std::vector<long long> acc((size_t)K * 3);
  std::vector<int32_t> order(K), cap1s(K);
  for (int k = 0; k < K; ++k) {
    acc[(size_t)k * 3 + 0] = w.types[k].idle_nw;
    acc[(size_t)k * 3 + 1] = w.types[k].dyn_nw_per_m;
    acc[(size_t)k * 3 + 2] = w.types[k].alloc_cpu_m;
    order[k] = k;
  }
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return cap1[a] > cap1[b]; });
  for (int k = 0; k < K; ++k) cap1s[k] = cap1[order[k]];
  int rc;
  if ((rc = dupload(c, c->d_acc, acc.data(), acc.size())) != CCKA_OK) return rc;
  if ((rc = dupload(c, c->d_order, order.data(), order.size())) != CCKA_OK) return rc;
  if ((rc = dupload(c, c->d_cap1s, cap1s.data(), cap1s.size())) != CCKA_OK) return rc;
  if ((rc = dupload(c, c->d_cap1t, cap1.data(), cap1.size())) != CCKA_OK) return rc;
  if ((rc = dupload(c, c->d_zmasks, zm.data(), zm.size())) != CCKA_OK) return rc;
  c->zmasks = zm;
  for (size_t z = 0; z < 16; ++z) p.zml[z] = z < zm.size() ? zm[z] : 0u;
  c->JT = jmax + 1;
  p.T = w.n_steps; p.K = K; p.Z = w.n_zones; p.R = w.n_regions; p.NP = w.n_pools; p.maxn = w.max_nodes;
  p.NZI = (int)zm.size(); p.JT = c->JT;
  p.start_minute = w.start_minute; p.peak_start = w.peak_start_min; p.peak_end = w.peak_end_min;
  p.pswitch0 = w.peak_switch; p.delay = w.provision_delay_steps;
  p.base_nodes = w.base_nodes; p.base_type = w.base_type; p.slo_util = w.slo_util_pct;
  p.pdb_pct = w.pdb_min_available_pct; p.pdb_member = dp.pdb_member ? 1 : 0;
  p.replicas0 = dp.replicas0; p.minr = dp.min_replicas; p.maxr0 = dp.max_replicas;
  p.target0 = dp.target_util_pct; p.req_cpu = dp.req_cpu_m; p.limit = dp.limit_cpu_m;
  p.dstab0 = dp.down.stab_window_s; p.reset_ca0 = w.reset_ca_s; p.capsel0 = (int32_t)dp.cap_sel;
  p.tol_lo = 1.0 - dp.tolerance;
  p.tol_hi = 1.0 + dp.tolerance;
  const ccka_itype& bt = w.types[w.base_type];
  p.base_nw = (long long)w.base_nodes *
              (bt.idle_nw + bt.dyn_nw_per_m * (long long)(w.base_util * (double)bt.alloc_cpu_m));
  p.up = d1_rule(dp.up, true);
  p.dn = d1_rule(dp.down, false);
  p.bdef = d1_rule_is_default(p.up, true) && d1_rule_is_default(p.dn, false);
  p.nsub = sync15 ? 4 : 1;
  if (sync15 && (!p.bdef || dp.down.stab_window_s > kD1Sync15MaxWindow)) return CCKA_OK;
  if (keda) {
    if (!p.bdef || dp.down.stab_window_s > CCKA_HIST * CCKA_STEP_SECONDS) return CCKA_OK;
    p.keda = 1;
    p.k_thr = (int32_t)dp.keda_threshold;
    p.k_act = (int32_t)dp.keda_activation;
    p.k_cds = dp.keda_cooldown_s > 0 ? (int32_t)std::min<int64_t>(((int64_t)dp.keda_cooldown_s + 59) / 60, 1 << 20) : 0;
    p.k_min = dp.keda_min;
    p.k_max = dp.keda_max;
  }
  c->d1_world = true;
  return CCKA_OK;
}

// Drift never acts when no scenario switches profile or OFFPEAK and PEAK
// resolve to the same masks for every pool.
static bool d1_drift_inert(const ccka_ctx* c) {
  const ccka_world& w = c->hw;
  if (!(w.disrupt_ext & CCKA_DISRUPT_DRIFT)) return true;
  const bool switching = c->sc_pswitch_any >= 0 ? c->sc_pswitch_any != 0 : w.peak_switch != 0;
  bool same = true;
  for (int q = 0; q < w.n_pools; ++q) {
    uint32_t zm = 0, cm = 0;
    for (const ccka_pool_patch* x : {&w.pools[q].base, &w.pools[q].profile[CCKA_PROFILE_RESET]}) {
      if (x->zone_mask) zm = x->zone_mask;
      if (x->cap_mask) cm = x->cap_mask;
    }
    // masks after the first profile (t = 0, either one) must never change
    // over the alternations that follow (merge: 0 keeps the previous mask)
    const ccka_pool_patch* pr[2] = {&w.pools[q].profile[CCKA_PROFILE_OFFPEAK],
                                    &w.pools[q].profile[CCKA_PROFILE_PEAK]};
    for (int first = 0; first < 2; ++first) {
      uint32_t z = zm, k = cm, z1 = 0, k1 = 0;
      for (int j = 0; j < 4; ++j) {
        const ccka_pool_patch* x = pr[(first + j) & 1];
        if (x->zone_mask) z = x->zone_mask;
        if (x->cap_mask) k = x->cap_mask;
        if (j == 0) { z1 = z; k1 = k; }
        else if (z != z1 || k != k1) same = false;
      }
    }
  }
  return !switching || same;
}

// The single-deployment kernel runs drift (SEMANTICS 3.G0) and single-node
// replacement consolidation (3.G2) itself in its DRIFT instantiation (8
// slots, <= 2 pools); multi-node consolidation runs on the general kernel
// unless provably inert. Replacement needs an on-demand node in a
// WhenEmptyOrUnderutilized pool: inert when no pool profile uses that policy
// or no scenario's nodeSelector admits on-demand; multi-node consolidation
// needs a WhenEmptyOrUnderutilized pool and a budget of >= 2 nodes.
static bool d1_disrupt_ok(const ccka_ctx* c, bool* drift, bool* replace, bool* multi) {
  const ccka_world& w = c->hw;
  *drift = !d1_drift_inert(c);
  *replace = false;
  *multi = false;
  if (*drift && !(w.max_nodes <= 8 && w.n_pools <= 2)) return false;
  bool weou = false;
  for (int q = 0; q < w.n_pools; ++q) {
    weou |= w.pools[q].base.policy == CCKA_WHEN_EMPTY_OR_UNDERUTILIZED;
    for (int s = 0; s < 3; ++s) weou |= w.pools[q].profile[s].policy == CCKA_WHEN_EMPTY_OR_UNDERUTILIZED;
  }
  if (w.disrupt_ext & CCKA_DISRUPT_REPLACE) {
    const uint32_t sel = c->sc_capsel_or ? c->sc_capsel_or : w.deploy[0].cap_sel;
    if (weou && (sel & CCKA_CAP_OD)) {
      if (!(w.max_nodes <= 8 && w.n_pools <= 2)) return false;
      *replace = true;
    }
  }
  if ((w.disrupt_ext & CCKA_DISRUPT_MULTI) && weou) {
    // Multi-node consolidation moves >= 2 nodes of a pool in one step: its
    // firstN search tries prefixes of at most budget - deleted candidates
    // (SEMANTICS 3.G3). With every pool's disruption budget at <= 1 node for
    // any node count the world allows (ceil(pct * max_nodes / 100) <= 1: the
    // reference's 10 % at 8 nodes) there is no prefix to try, so it never acts
    // and is not evaluated; larger budgets run it in the DRIFT instantiation.
    bool two = false;
    for (int q = 0; q < w.n_pools; ++q) two |= (w.pools[q].budget_pct * w.max_nodes + 99) / 100 >= 2;
    if (two) {
      if (!(w.max_nodes <= 8 && w.n_pools <= 2)) return false;
      *multi = true;
    }
  }
  return true;
}

// scenario-dependent part: distinct carbon weights, per-scenario index, tables
static int d1_prepare(ccka_ctx* c) {
  c->d1_ready = true;
  c->d1_ok = false;
  bool drift = false, replace = false, multi = false;
  // (a KEDA deployment ignores the per-scenario target / max / down-window
  // overrides: its bounds and rules are the ScaledObject's, SEMANTICS 3.C)
  const bool keda = c->d1.keda != 0;
  if (!c->d1_world || (!keda && !c->sc_maxr_ok) || !d1_disrupt_ok(c, &drift, &replace, &multi)) return CCKA_OK;
  if (keda && (drift || replace || multi)) return CCKA_OK;  // the KEDA instantiation has no DRIFT paths
  c->d1.drift = (drift || replace || multi) ? 1 : 0;  // the DRIFT instantiation carries all three
  c->d1.drift_on = drift ? 1 : 0;
  c->d1.replace = replace ? 1 : 0;
  c->d1.multi = multi ? 1 : 0;
  // beyond the register ring
  if (!keda && c->sc_dstab_max > (c->d1.nsub == 4 ? kD1Sync15MaxWindow : CCKA_HIST * CCKA_STEP_SECONDS))
    return CCKA_OK;
  // default behavior and no window beyond 300 s: the 4-record ring instantiation
  c->d1.he4 = (c->d1.nsub == 1 && c->d1.bdef && c->d1.dstab0 <= 300 && (keda || c->sc_dstab_max <= 300)) ? 1 : 0;
  const size_t n = (size_t)c->N;
  std::vector<double> wl;
  std::vector<uint8_t> wci;
  if (!c->h_cw.empty()) {
    std::map<uint64_t, int> seen;
    wci.resize(n);
    for (size_t i = 0; i < n; ++i) {
      uint64_t b;
      std::memcpy(&b, &c->h_cw[i], 8);
      auto it = seen.find(b);
      if (it == seen.end()) {
        if ((int)wl.size() >= D1_MAX_WC) return CCKA_OK;
        it = seen.emplace(b, (int)wl.size()).first;
        wl.push_back(c->h_cw[i]);
      }
      wci[i] = (uint8_t)it->second;
    }
  } else {
    wl.push_back(c->hw.carbon_weight);
  }
  std::vector<double> wc1000(wl.size());
  for (size_t k = 0; k < wl.size(); ++k) wc1000[k] = wl[k] * 1000.0;
  int rc;
  if ((rc = dupload(c, c->d_wc1000, wc1000.data(), wc1000.size())) != CCKA_OK) return rc;
  if ((rc = dupload(c, c->d_wci, wci.empty() ? nullptr : wci.data(), wci.size())) != CCKA_OK) return rc;
  c->NW = (int)wl.size();
  const ccka_world& w = c->hw;
  const size_t keys = (size_t)w.n_regions * 24 * c->zmasks.size() * 3;
  dfree(c->d_table);
  dfree(c->d_jtab);
  dfree(c->d_table2);
  dfree(c->d_jtab2);
  if (hipMalloc((void**)&c->d_table, keys * c->NW * c->JT * sizeof(int2)) != hipSuccess ||
      hipMalloc((void**)&c->d_jtab, keys * sizeof(int32_t)) != hipSuccess)
    return fail(c, CCKA_ENOMEM, "argmin table alloc (%zu keys x %d weights x %d)", keys, c->NW, c->JT);
  if (replace || multi) {  // the G2 / G3 offer table: cheapest offering holding n pods, by price
    const double zero = 0.0;
    if ((rc = dupload(c, c->d_wc0, &zero, 1)) != CCKA_OK) return rc;
    if (hipMalloc((void**)&c->d_table2, keys * c->JT * sizeof(int2)) != hipSuccess ||
        hipMalloc((void**)&c->d_jtab2, keys * sizeof(int32_t)) != hipSuccess)
      return fail(c, CCKA_ENOMEM, "offer table alloc (%zu keys x %d)", keys, c->JT);
  }
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->d1_ok = true;
  return CCKA_OK;
}

extern "C" {

int32_t ccka_abi_version(void) { return CCKA_ABI_VERSION; }

int32_t ccka_struct_sizes(int64_t* out, int32_t n) {
  const int64_t s[] = {sizeof(ccka_itype),    sizeof(ccka_pool),    sizeof(ccka_deployment),
                       sizeof(ccka_world),    sizeof(ccka_scenarios), sizeof(ccka_results),
                       sizeof(ccka_traj_rec), sizeof(ccka_totals),  sizeof(ccka_trace_gen),
                       sizeof(ccka_grid_stats), sizeof(ccka_detail)};
  const int32_t m = (int32_t)(sizeof s / sizeof s[0]);
  int32_t k = 0;
  for (; k < m && k < n; ++k) out[k] = s[k];
  return k;
}

const char* ccka_last_error(const ccka_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int ccka_open(ccka_ctx** out, int device_ordinal) {
  if (!out) return CCKA_EINVAL;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return CCKA_ENODEV;
  if (device_ordinal < 0 || device_ordinal >= ndev) return CCKA_ENODEV;
  if (hipSetDevice(device_ordinal) != hipSuccess) return CCKA_ENODEV;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device_ordinal) != hipSuccess) return CCKA_ENODEV;
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return CCKA_ENODEV;
  ccka_ctx* c = new (std::nothrow) ccka_ctx();
  if (!c) return CCKA_ENOMEM;
  c->device = device_ordinal;
  c->cus = prop.multiProcessorCount;
  std::snprintf(c->name, sizeof c->name, "%s (%s)", prop.name, prop.gcnArchName);
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess ||
      hipEventCreate(&c->ev_mid) != hipSuccess) {
    delete c;
    return CCKA_EHIP;
  }
  // sine table of the synthetic load generator (SEMANTICS.md §4)
  int32_t sinq[1440];
  for (int m = 0; m < 1440; ++m) sinq[m] = (int32_t)std::lround(65536.0 * std::sin(2.0 * M_PI * (double)m / 1440.0));
  if (dupload(c, c->d_sinq, sinq, 1440) != CCKA_OK || hipStreamSynchronize(c->stream) != hipSuccess) {
    ccka_close(c);
    return CCKA_EHIP;
  }
  *out = c;
  return CCKA_OK;
}

static void free_results(ccka_ctx* c) {
  dfree(c->d_res);
  dfree(c->d_traj);
  dfree(c->d_traj_t);
  c->traj_t_count = 0;
  dfree(c->d_parts);
  dfree(c->d_detail);
  c->traj_count = 0;
  c->traj_valid = false;
  c->detail_count = 0;
  c->detail_valid = false;
}

void ccka_close(ccka_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->comm) ncclCommDestroy(c->comm);
  dfree(c->d_world); dfree(c->d_types); dfree(c->d_price); dfree(c->d_ci_gpwh); dfree(c->d_ci_gpwmin);
  dfree(c->d_region); dfree(c->d_target); dfree(c->d_maxr); dfree(c->d_dstab); dfree(c->d_resetca);
  dfree(c->d_pswitch); dfree(c->d_cw); dfree(c->d_capsel); dfree(c->d_load); dfree(c->d_load_w); dfree(c->d_totals);
  dfree(c->d_load_nt);
  dfree(c->d_ptable); dfree(c->d_pjtab); dfree(c->d_pwc);
  dfree(c->d_sinq);
  dfree(c->d_acc); dfree(c->d_order); dfree(c->d_cap1s); dfree(c->d_cap1t); dfree(c->d_zmasks); dfree(c->d_wc1000);
  dfree(c->d_wci); dfree(c->d_table); dfree(c->d_jtab); dfree(c->d_stamps);
  dfree(c->d_table2); dfree(c->d_jtab2); dfree(c->d_wc0);
  dfree(c->d_gstats); dfree(c->d_gcand); dfree(c->d_ggather); dfree(c->d_gcounts); dfree(c->d_gn);
  dfree(c->d_gflags); dfree(c->d_gfront); dfree(c->d_hist);
  dfree(c->d_pol_state); dfree(c->d_pol_target); dfree(c->d_pol_cw); dfree(c->d_rec_target); dfree(c->d_rec_cw);
  dfree(c->d_feat_rec);
  dfree(c->d_w1f); dfree(c->d_w2f); dfree(c->d_w3f); dfree(c->d_mb); dfree(c->d_mx); dfree(c->d_my);
  dfree(c->d_w1g); dfree(c->d_w2g); dfree(c->d_w3g);
  dfree(c->d_w2b); dfree(c->d_w3b); dfree(c->d_pg_act); dfree(c->d_pg_coef); dfree(c->d_pg_seed); dfree(c->d_pg_x);
  dfree(c->d_pg_work); dfree(c->d_pg_part); dfree(c->d_pg_grad);
  free_results(c);
  if (c->ev0) (void)hipEventDestroy(c->ev0);
  if (c->ev1) (void)hipEventDestroy(c->ev1);
  if (c->ev_mid) (void)hipEventDestroy(c->ev_mid);
  if (c->pol_graph) (void)hipGraphExecDestroy(c->pol_graph);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

// autoscaling/v2 ranges: stabilizationWindowSeconds 0..3600, periodSeconds
// 1..1800 (0 accepted: an empty period), up to CCKA_HPA_MAX_POLICIES policies
static bool rules_ok(const ccka_hpa_rules& r) {
  if (r.select < 0 || r.select > 2 || r.n_policies < 0 || r.n_policies > CCKA_HPA_MAX_POLICIES) return false;
  if (r.stab_window_s < 0 || r.stab_window_s > CCKA_HPA_MAX_WINDOW_S) return false;
  for (int i = 0; i < r.n_policies; ++i) {
    const ccka_hpa_policy& p = r.policies[i];
    if ((p.type != CCKA_HPA_PODS && p.type != CCKA_HPA_PERCENT) || p.value < 0 || p.period_s < 1 ||
        p.period_s > CCKA_HPA_MAX_PERIOD_S)
      return false;
  }
  return true;
}



int ccka_set_world(ccka_ctx* c, const ccka_world* w) {
  if (!c || !w) return CCKA_EINVAL;
  (void)hipSetDevice(c->device);
  if (w->n_steps < 1 || w->n_steps > 65535) return fail(c, CCKA_EINVAL, "n_steps out of range");
  if (w->max_nodes < 1 || w->max_nodes > CCKA_MAX_NODES) return fail(c, CCKA_EINVAL, "max_nodes out of range");
  if (w->n_types < 1 || w->n_types > CCKA_MAX_TYPES || !w->types) return fail(c, CCKA_EINVAL, "catalog invalid");
  if (w->n_zones < 1 || w->n_zones > CCKA_MAX_ZONES) return fail(c, CCKA_EINVAL, "n_zones out of range");
  if (w->n_regions < 1 || w->n_regions > CCKA_MAX_REGIONS) return fail(c, CCKA_EINVAL, "n_regions out of range");
  if (w->n_pools < 1 || w->n_pools > CCKA_MAX_POOLS) return fail(c, CCKA_EINVAL, "n_pools out of range");
  if (w->n_deploy < 1 || w->n_deploy > CCKA_MAX_DEPLOY) return fail(c, CCKA_EINVAL, "n_deploy out of range");
  if (!w->price_uph || !w->ci_gpwh || !w->ci_gpwmin) return fail(c, CCKA_EINVAL, "tiles missing");
  if (w->disrupt_ext & ~(CCKA_DISRUPT_DRIFT | CCKA_DISRUPT_REPLACE | CCKA_DISRUPT_MULTI))
    return fail(c, CCKA_EINVAL, "unknown disrupt_ext bits");
  if (w->base_type < 0 || w->base_type >= w->n_types) return fail(c, CCKA_EINVAL, "base_type out of range");
  if (w->provision_delay_steps < 0 || w->start_minute < 0) return fail(c, CCKA_EINVAL, "negative timing");
  for (int k = 0; k < w->n_types; ++k) {
    const ccka_itype& t = w->types[k];
    if (t.vcpu < 0 || t.alloc_cpu_m <= 0 || t.alloc_mem_mi < 0 || t.max_pods < 0)
      return fail(c, CCKA_EINVAL, "catalog entry %d invalid", k);
  }
  for (int d = 0; d < w->n_deploy; ++d) {
    const ccka_deployment& dp = w->deploy[d];
    if (dp.scaler < 0 || dp.scaler > 3 || dp.cap_sel == 0 || dp.cap_sel > 3 || dp.req_cpu_m < 0 ||
        dp.req_mem_mi < 0 || dp.replicas0 < 0)
      return fail(c, CCKA_EINVAL, "deployment %d invalid", d);
    if (dp.scaler == CCKA_SCALER_HPA && (dp.req_cpu_m <= 0 || dp.target_util_pct <= 0))
      return fail(c, CCKA_EINVAL, "HPA deployment %d needs cpu request and target", d);
    if ((dp.scaler == CCKA_SCALER_KEDA || dp.scaler == CCKA_SCALER_KEDA_TRIGGER) && dp.keda_threshold <= 0)
      return fail(c, CCKA_EINVAL, "KEDA deployment %d needs threshold", d);
    if (dp.scaler == CCKA_SCALER_KEDA_TRIGGER &&
        (d == 0 || dp.replicas0 != 0 || dp.pdb_member ||
         (w->deploy[d - 1].scaler != CCKA_SCALER_KEDA && w->deploy[d - 1].scaler != CCKA_SCALER_KEDA_TRIGGER)))
      return fail(c, CCKA_EINVAL, "KEDA trigger %d must follow a KEDA deployment and own no pods", d);
    if (!rules_ok(dp.up) || !rules_ok(dp.down))
      return fail(c, CCKA_EINVAL, "deployment %d behavior outside autoscaling/v2 ranges (window <= %d s, period <= %d s, "
                  "<= %d policies)", d, CCKA_HPA_MAX_WINDOW_S, CCKA_HPA_MAX_PERIOD_S, CCKA_HPA_MAX_POLICIES);
  }
  if (w->hpa_sync_s != 0 && w->hpa_sync_s != 10 && w->hpa_sync_s != 15 && w->hpa_sync_s != 20 &&
      w->hpa_sync_s != 30 && w->hpa_sync_s != 60)
    return fail(c, CCKA_EINVAL, "hpa_sync_s must be 0, 10, 15, 20, 30 or 60");
  for (int q = 0; q < w->n_pools; ++q)
    if (w->pools[q].limit_mem_mi < -1) return fail(c, CCKA_EINVAL, "pool %d limit_mem_mi invalid", q);
  c->hw = *w;
  const int K = w->n_types, Z = w->n_zones, R = w->n_regions;
  int rc;
  if ((rc = dupload(c, c->d_types, w->types, (size_t)K)) != CCKA_OK) return rc;
  if ((rc = dupload(c, c->d_price, w->price_uph, (size_t)R * 24 * K * Z * 2)) != CCKA_OK) return rc;
  if ((rc = dupload(c, c->d_ci_gpwh, w->ci_gpwh, (size_t)R * 24)) != CCKA_OK) return rc;
  if ((rc = dupload(c, c->d_ci_gpwmin, w->ci_gpwmin, (size_t)R * 24)) != CCKA_OK) return rc;
  ccka_world dw = *w;
  dw.types = nullptr; dw.ci_gpwh = nullptr; dw.ci_gpwmin = nullptr; dw.price_uph = nullptr;
  if ((rc = dupload(c, c->d_world, &dw, 1)) != CCKA_OK) return rc;
  // provisioning order: req_cpu desc, req_mem desc, index asc
  const int D = w->n_deploy;
  for (int d = 0; d < D; ++d) c->prov[d] = d;
  std::stable_sort(c->prov, c->prov + D, [&](int a, int b) {
    const ccka_deployment &A = w->deploy[a], &B = w->deploy[b];
    if (A.req_cpu_m != B.req_cpu_m) return A.req_cpu_m > B.req_cpu_m;
    return A.req_mem_mi > B.req_mem_mi;
  });
  if ((rc = d1_check_world(c)) != CCKA_OK) return rc;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->have_world = true;
  c->have_load = false;
  c->traj_valid = false;
  c->ran = false;
  return CCKA_OK;
}

static int alloc_results(ccka_ctx* c) {
  free_results(c);
  const int64_t N = c->N;
  // 8-byte fields first, then 4-byte fields; each array 256-B aligned
  auto up = [](int64_t b) { return (b + 255) & ~(int64_t)255; };
  const int64_t b8 = up(N * 8), b4 = up(N * 4);
  const int64_t total = 4 * b8 + 10 * b4;
  if (hipMalloc(&c->d_res, (size_t)total) != hipSuccess) return fail(c, CCKA_ENOMEM, "results alloc");
  char* p = (char*)c->d_res;
  KParams& k = c->kp;
  k.cost = (int64_t*)p; p += b8;
  k.energy = (double*)p; p += b8;
  k.gco2 = (double*)p; p += b8;
  k.pend_min = (int64_t*)p; p += b8;
  k.slo = (int32_t*)p; p += b4;
  k.nmin_spot = (int32_t*)p; p += b4;
  k.nmin_od = (int32_t*)p; p += b4;
  k.launches = (int32_t*)p; p += b4;
  k.deletions = (int32_t*)p; p += b4;
  k.peak_nodes = (int32_t*)p; p += b4;
  k.final_reps = (int32_t*)p; p += b4;
  k.final_nodes = (int32_t*)p; p += b4;
  k.last_choice = (uint32_t*)p; p += b4;
  k.hash = (uint32_t*)p; p += b4;
  if (hipMalloc(&c->d_parts, (1024 * 11 + 1) * sizeof(long long)) != hipSuccess) return fail(c, CCKA_ENOMEM, "parts alloc");
  if (!c->d_totals && hipMalloc((void**)&c->d_totals, sizeof(ccka_totals)) != hipSuccess)
    return fail(c, CCKA_ENOMEM, "totals alloc");
  return CCKA_OK;
}

int ccka_set_scenarios(ccka_ctx* c, const ccka_scenarios* sc) {
  if (!c || !sc) return CCKA_EINVAL;
  if (!c->have_world) return fail(c, CCKA_ESTATE, "set_world first");
  if (sc->n < 1 || sc->n > (int64_t)1 << 31) return fail(c, CCKA_EINVAL, "scenario count out of range");
  if (sc->n_traces < 0 || sc->n_traces > (int64_t)1 << 31 || sc->first_id < 0)
    return fail(c, CCKA_EINVAL, "n_traces / first_id out of range");
  (void)hipSetDevice(c->device);
  const size_t n = (size_t)sc->n;
  if (sc->region) {
    for (size_t i = 0; i < n; ++i)
      if (sc->region[i] >= c->hw.n_regions) return fail(c, CCKA_EINVAL, "region %u out of range", sc->region[i]);
    c->h_region.assign(sc->region, sc->region + n);
  } else {
    c->h_region.clear();
  }
  if (sc->cap_sel)
    for (size_t i = 0; i < n; ++i)
      if (sc->cap_sel[i] == 0 || sc->cap_sel[i] > 3) return fail(c, CCKA_EINVAL, "cap_sel invalid");
  if (sc->target_util_pct)
    for (size_t i = 0; i < n; ++i)
      if (sc->target_util_pct[i] <= 0) return fail(c, CCKA_EINVAL, "target_util_pct must be > 0");
  c->sc_dstab_max = -1;
  if (sc->down_stab_s)
    for (size_t i = 0; i < n; ++i) {
      if (sc->down_stab_s[i] < 0 || sc->down_stab_s[i] > CCKA_HPA_MAX_WINDOW_S)
        return fail(c, CCKA_EINVAL, "down_stab_s outside 0..%d s", CCKA_HPA_MAX_WINDOW_S);
      c->sc_dstab_max = std::max<int>(c->sc_dstab_max, sc->down_stab_s[i]);
    }
  int rc;
  if ((rc = dupload(c, c->d_region, sc->region, n)) != CCKA_OK) return rc;
  if ((rc = dupload(c, c->d_target, sc->target_util_pct, n)) != CCKA_OK) return rc;
  if ((rc = dupload(c, c->d_maxr, sc->max_replicas, n)) != CCKA_OK) return rc;
  if ((rc = dupload(c, c->d_dstab, sc->down_stab_s, n)) != CCKA_OK) return rc;
  if ((rc = dupload(c, c->d_resetca, sc->reset_ca_s, n)) != CCKA_OK) return rc;
  if ((rc = dupload(c, c->d_pswitch, sc->peak_switch, n)) != CCKA_OK) return rc;
  if ((rc = dupload(c, c->d_cw, sc->carbon_weight, n)) != CCKA_OK) return rc;
  if ((rc = dupload(c, c->d_capsel, sc->cap_sel, n)) != CCKA_OK) return rc;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->h_cw.clear();
  if (sc->carbon_weight) c->h_cw.assign(sc->carbon_weight, sc->carbon_weight + n);
  c->sc_capsel_or = 0;
  if (sc->cap_sel)
    for (size_t i = 0; i < n; ++i) c->sc_capsel_or |= sc->cap_sel[i];
  c->sc_pswitch_any = -1;
  if (sc->peak_switch) {
    c->sc_pswitch_any = 0;
    for (size_t i = 0; i < n; ++i) c->sc_pswitch_any |= sc->peak_switch[i] != 0;
  }
  c->sc_maxr_ok = true;
  if (sc->max_replicas)
    for (size_t i = 0; i < n; ++i)
      if (sc->max_replicas[i] < 0) { c->sc_maxr_ok = false; break; }
  c->d1_ready = false;
  c->N = sc->n;
  c->first_id = sc->first_id;
  c->n_traces = sc->n_traces;
  if ((rc = alloc_results(c)) != CCKA_OK) return rc;
  dfree(c->d_load);
  dfree(c->d_load_w);
  c->load_w_count = 0;
  c->load_w_lpw = 0;
  c->load_nt_dp = 0;
  c->have_load = false;
  c->have_sc = true;
  c->ran = false;
  return CCKA_OK;
}

static int64_t load_cols(const ccka_ctx* c) { return c->n_traces > 0 ? c->n_traces : c->N; }

static int ensure_load(ccka_ctx* c) {
  const int64_t cnt = (int64_t)c->hw.n_steps * c->hw.n_deploy * load_cols(c);
  if (c->d_load && c->load_count == cnt) return CCKA_OK;
  dfree(c->d_load);
  if (hipMalloc((void**)&c->d_load, (size_t)cnt * 4) != hipSuccess)
    return fail(c, CCKA_ENOMEM, "load alloc %lld ints", (long long)cnt);
  c->load_count = cnt;
  return CCKA_OK;
}

// The pooled single-deployment kernel (rollout_pool.hip) takes the worlds with
// the default HPA behavior or one KEDA trigger, one decision per step, <= 8
// slots and <= 2 pools, no drift / replacement / multi-node consolidation,
// when the workgroup's scenario state fits the 160 KiB of LDS (price tiles
// staged too when they fit) and its trace resource spans < 2 GiB; the others
// keep rollout_d1_kernel.
static bool d1_pool_plan(const ccka_ctx* c, D1Params& p) {
  if (!c->pool_mode || !p.bdef || p.nsub != 1 || p.drift || p.maxn > 8 || p.NP > 2 || (p.ablate & ~16) ||
      (p.stamps && p.keda) || c->occ > 2 || p.lpw < 1 || p.lpw > 64)
    return false;
  if (!p.load_w && p.NL * (int64_t)p.T * 4 >= (1LL << 31)) return false;
  const int hw = p.he4 ? 2 : 4;
  for (int tab = 1; tab >= 0; --tab) {
    if (pool_lds_layout(p.K, p.R, p.Z, p.NZI, tab, PL_WAVES * p.lpw, hw).total <= 160u * 1024u) {
      p.lds_tab = tab;
      return true;
    }
  }
  return false;
}

// scenarios per wave of the single-deployment kernel: a wave's cost is the
// union of its lanes' event paths, so when the batch is smaller than one full
// round of resident waves (two per SIMD at this kernel's register budget)
// spread it over all of them
static int32_t d1_lpw(const ccka_ctx* c) {
  if (c->lpw > 0) return c->lpw;
  const int64_t slots = 2LL * 4 * c->cus;  // resident waves: 2 per SIMD, 4 SIMDs per CU
  return (int32_t)std::min<int64_t>(64, std::max<int64_t>(32, (c->N + slots - 1) / slots));
}

// The single-deployment kernel reads a per-scenario trace wave-tiled
// ([wave][T][lanes]): with [T][N] a wave's 196-byte row shares its first and
// last 128-byte lines with the neighbouring waves, which run up to hundreds of
// steps apart (lane skew), so the L2 has evicted those lines before the
// neighbour reads them. Built lazily by the first single-deployment rollout of
// a trace and lanes-per-wave value (never by the policy loop or the general
// kernel, which read [T][N]), beside the [T][N] trace; without the memory for
// it the kernel reads [T][N] (same results). The policy loop frees it.
static int d1_trace_tile(ccka_ctx* c) {
  if (!c->d1_world || c->hw.n_deploy != 1 || c->n_traces > 0 || !c->have_load) return CCKA_OK;
  const int32_t lpw = d1_lpw(c);
  if (c->load_w_lpw == lpw && c->d_load_w) return CCKA_OK;
  const int64_t cnt = (int64_t)c->hw.n_steps * ((c->N + lpw - 1) / lpw * lpw);  // rows lpw wide
  if (!c->d_load_w || c->load_w_count != cnt) {
    dfree(c->d_load_w);
    c->load_w_count = 0;
    if (hipMalloc((void**)&c->d_load_w, (size_t)cnt * 4) != hipSuccess) {
      (void)hipGetLastError();
      c->d_load_w = nullptr;
      return CCKA_OK;
    }
    c->load_w_count = cnt;
  }
  HIPCHK(c, launch_trace_tile(c->d_load, c->d_load_w, c->N, c->hw.n_steps, lpw, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->load_w_lpw = lpw;
  return CCKA_OK;
}

// the skewed schedule's scenario-major trace copy (built once per trace: N*T*DP*4
// bytes; without memory for it the kernel gathers from [T][D][N], same results)
static int sk_trace(ccka_ctx* c) {
  int dmax, nmax;
  kernel_dims(c->hw.n_deploy, c->hw.max_nodes, &dmax, &nmax);
  if (c->load_nt_dp == dmax && c->d_load_nt) return CCKA_OK;
  const int64_t NL = load_cols(c), cnt = NL * c->hw.n_steps * dmax;
  if (!c->d_load_nt || c->load_nt_count != cnt) {
    dfree(c->d_load_nt);
    c->load_nt_count = 0;
    if (hipMalloc((void**)&c->d_load_nt, (size_t)cnt * 4) != hipSuccess) {
      (void)hipGetLastError();
      c->d_load_nt = nullptr;
      return CCKA_OK;
    }
    c->load_nt_count = cnt;
  }
  HIPCHK(c, launch_trace_nt(c->d_load, c->d_load_nt, NL, c->hw.n_steps, c->hw.n_deploy, dmax, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->load_nt_dp = dmax;
  return CCKA_OK;
}

int ccka_set_load(ccka_ctx* c, const int32_t* load, int64_t count) {
  if (!c || !load) return CCKA_EINVAL;
  if (!c->have_sc) return fail(c, CCKA_ESTATE, "set_scenarios first");
  (void)hipSetDevice(c->device);
  int rc;
  if ((rc = ensure_load(c)) != CCKA_OK) return rc;
  if (count != c->load_count) return fail(c, CCKA_EINVAL, "load count %lld != T*D*N %lld", (long long)count, (long long)c->load_count);
  c->load_w_lpw = 0;
  c->load_nt_dp = 0;
  HIPCHK(c, hipMemcpyAsync(c->d_load, load, (size_t)count * 4, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->have_load = true;
  return CCKA_OK;
}

int ccka_gen_load(ccka_ctx* c, const ccka_trace_gen* g) {
  if (!c || !g) return CCKA_EINVAL;
  if (!c->have_sc) return fail(c, CCKA_ESTATE, "set_scenarios first");
  if (g->base_hi < g->base_lo || g->amp_hi_pm < g->amp_lo_pm || g->burst_len < 0)
    return fail(c, CCKA_EINVAL, "trace generator ranges invalid");
  (void)hipSetDevice(c->device);
  int rc;
  if ((rc = ensure_load(c)) != CCKA_OK) return rc;
  GenParams gp{};
  gp.out = c->d_load;
  gp.sinq = c->d_sinq;
  // shared traces are keyed by trace index, per-scenario traces by global id
  gp.n = load_cols(c);
  gp.first_id = c->n_traces > 0 ? 0 : c->first_id;
  gp.seed = g->seed;
  gp.T = c->hw.n_steps;
  gp.D = c->hw.n_deploy;
  gp.base_lo = g->base_lo; gp.base_hi = g->base_hi;
  gp.amp_lo = g->amp_lo_pm; gp.amp_hi = g->amp_hi_pm;
  gp.noise = g->noise_pm; gp.burst_prob = g->burst_prob_pm;
  gp.burst_mult = g->burst_mult_pm; gp.burst_len = g->burst_len;
  c->load_w_lpw = 0;
  c->load_nt_dp = 0;
  HIPCHK(c, launch_gen_load(gp, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->have_load = true;
  return CCKA_OK;
}

int ccka_get_load(ccka_ctx* c, int32_t* load, int64_t count) {
  if (!c || !load) return CCKA_EINVAL;
  if (!c->have_load) return fail(c, CCKA_ESTATE, "no load on device");
  if (count != c->load_count) return fail(c, CCKA_EINVAL, "load count mismatch");
  (void)hipSetDevice(c->device);
  HIPCHK(c, hipMemcpyAsync(load, c->d_load, (size_t)count * 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return CCKA_OK;
}

static int plan_launch(ccka_ctx* c, int* block, size_t* lds) {
  const ccka_world& w = c->hw;
  const int B = 256;
  int span = 1;
  if (!c->h_region.empty()) {
    for (int64_t b = 0; b < c->N; b += B) {
      const int64_t e = std::min<int64_t>(c->N, b + B);
      int lo = 255, hi = 0;
      for (int64_t i = b; i < e; ++i) { lo = std::min<int>(lo, c->h_region[i]); hi = std::max<int>(hi, c->h_region[i]); }
      span = std::max(span, hi - lo + 1);
    }
  }
  int dmax, nmax;
  kernel_dims(w.n_deploy, w.max_nodes, &dmax, &nmax);
  auto up16 = [](size_t x) { return (x + 15) & ~(size_t)15; };
  const size_t K = (size_t)w.n_types;
  size_t off = up16(K * sizeof(ccka_itype));
  KParams& k = c->kp;
  k.lds_off_cap1 = (int32_t)off;
  off = up16(off + K * 4);
  k.lds_off_tile = (int32_t)off;
  const size_t tile_bytes = (size_t)span * K * w.n_zones * 2 * 4;
  // stage all 24 hourly tiles when they fit comfortably (no barrier in the step
  // loop); otherwise one hour at a time, restaged at each hour boundary
  k.all_hours = (off + 24 * tile_bytes + 8 * 1024) <= 64 * 1024 ? 1 : 0;
  off = up16(off + (k.all_hours ? 24 : 1) * tile_bytes);
  k.lds_off_claims = (int32_t)off;
  off = up16(off + (size_t)(B / 64) * nmax * (7 + dmax) * 4);
  k.lds_off_misc = (int32_t)off;
  off += 16;
  k.lds_off_ci = (int32_t)off;
  off = up16(off + (size_t)span * 24 * 2 * sizeof(double));
  if (off > 160 * 1024) return fail(c, CCKA_EINVAL, "LDS budget %zu B exceeds 160 KiB (catalog %zu types, span %d)", off, K, span);
  k.span = span;
  *block = B;
  *lds = off;
  return CCKA_OK;
}

// the general kernel's parameters for a whole-horizon rollout: buffers,
// launch geometry, HPA history, detail (shared by ccka_rollout_async and
// ccka_policy_rollout)
static int setup_general(ccka_ctx* c, int32_t trajectory, int* block_out, size_t* lds_out) {
  const ccka_world& w = c->hw;
  int block = 256;
  size_t lds = 0;
  int rc;
  if ((rc = plan_launch(c, &block, &lds)) != CCKA_OK) return rc;
  *block_out = block;
  *lds_out = lds;
  KParams& k = c->kp;
  k.w = c->d_world;
  k.types = c->d_types;
  k.price = c->d_price;
  k.ci_gpwh = c->d_ci_gpwh;
  k.ci_gpwmin = c->d_ci_gpwmin;
  k.load = c->d_load;
  k.region = c->d_region;
  k.target = c->d_target;
  k.maxr = c->d_maxr;
  k.down_stab = c->d_dstab;
  k.reset_ca = c->d_resetca;
  k.pswitch = c->d_pswitch;
  k.cw = c->d_cw;
  k.cap_sel = c->d_capsel;
  k.traj = nullptr;
  if (trajectory) {
    const int64_t cnt = (int64_t)w.n_steps * c->N;
    if (c->traj_count != cnt) {
      dfree(c->d_traj);
      if (hipMalloc((void**)&c->d_traj, (size_t)cnt * sizeof(ccka_traj_rec)) != hipSuccess)
        return fail(c, CCKA_ENOMEM, "trajectory alloc");
      c->traj_count = cnt;
    }
    k.traj = c->d_traj;
  }
  k.detail = nullptr;
  if (c->detail_on) {
    if (c->detail_count != c->N) {
      dfree(c->d_detail);
      if (hipMalloc((void**)&c->d_detail, (size_t)c->N * sizeof(DetailDev)) != hipSuccess)
        return fail(c, CCKA_ENOMEM, "detail alloc");
      c->detail_count = c->N;
    }
    HIPCHK(c, hipMemsetAsync(c->d_detail, 0, (size_t)c->N * sizeof(DetailDev), c->stream));
    k.detail = c->d_detail;
  }
  // HPA decisions: one per step over the register rings, or nsub per step /
  // long windows / > 2 policies over the HBM history (SEMANTICS 3.C)
  k.sync_s = w.hpa_sync_s > 0 ? w.hpa_sync_s : CCKA_STEP_SECONDS;
  k.nsub = CCKA_STEP_SECONDS / k.sync_s;
  {
    bool fit = k.nsub == 1 && c->sc_dstab_max <= CCKA_HIST * CCKA_STEP_SECONDS;
    int hl = 0;
    for (int d = 0; d < w.n_deploy; ++d) {
      const ccka_deployment& dp = w.deploy[d];
      if (dp.scaler != CCKA_SCALER_HPA && dp.scaler != CCKA_SCALER_KEDA) continue;
      fit = fit && rules_fit_ring(dp.up) && rules_fit_ring(dp.down);
      int dstab = dp.down.stab_window_s;
      if (dp.scaler == CCKA_SCALER_HPA && c->sc_dstab_max >= 0) dstab = std::max(dstab, c->sc_dstab_max);
      hl = std::max({hl, hist_entries(dp.up.stab_window_s, k.sync_s), hist_entries(dstab, k.sync_s)});
      for (const ccka_hpa_rules* r : {&dp.up, &dp.down})
        for (int q = 0; q < r->n_policies; ++q) hl = std::max(hl, hist_entries(r->policies[q].period_s, k.sync_s));
    }
    k.hlen = fit ? 0 : std::max(hl, 1);
    k.hist = nullptr;
    if (k.hlen) {
      const int64_t cnt = (int64_t)k.hlen * w.n_deploy * c->N;
      if (c->hist_count < cnt) {
        dfree(c->d_hist);
        c->hist_count = 0;
        if (hipMalloc((void**)&c->d_hist, (size_t)cnt * sizeof(int2)) != hipSuccess)
          return fail(c, CCKA_ENOMEM, "HPA history alloc (%lld entries)", (long long)cnt);
        c->hist_count = cnt;
      }
      HIPCHK(c, hipMemsetAsync(c->d_hist, 0, (size_t)cnt * sizeof(int2), c->stream));
      k.hist = c->d_hist;
    }
  }
  k.lds_lclaims = -1;
  k.t0 = 0;
  k.t1 = w.n_steps;
  k.state = nullptr;
  k.state_load = 0;
  k.feat = nullptr;
  k.N = c->N;
  k.NL = load_cols(c);
  k.trace_mod = c->n_traces;
  k.first_id = c->first_id;
  k.T = w.n_steps;
  k.D = w.n_deploy;
  k.K = w.n_types;
  k.Z = w.n_zones;
  k.R = w.n_regions;
  k.P = w.n_pools;
  k.maxn = w.max_nodes;
  for (int d = 0; d < CCKA_MAX_DEPLOY; ++d) k.prov[d] = c->prov[d];
  return CCKA_OK;
}

// The general kernel's lane-skewed schedule (rollout_sk.hip) holds for worlds
// of two or more deployments that are HPA-scaled or static, with one HPA
// decision per step over the register history rings, every hour's price tiles
// in LDS, no detail breakdown and no drift / replacement / multi-node
// consolidation (rollout.hip, rollout_kernel's SK notes).
static bool sk_eligible(const ccka_ctx* c) {
  const ccka_world& w = c->hw;
  const KParams& k = c->kp;
  if (w.n_deploy < 2 || c->engine_mode == 2 || c->detail_on) return false;
  // up to four deployments: beyond, the per-lane state of the skewed schedule
  // spills (8 x 16 slots: 5.6 KB per lane) and the lockstep kernel is faster
  // (8 deployments 475 vs 307 ms, 12: 1039 vs 695 ms at 1e5 x 1440)
  int dmax, nmax;
  kernel_dims(w.n_deploy, w.max_nodes, &dmax, &nmax);
  if (dmax > 4) return false;
  if (k.nsub != 1 || k.hlen != 0 || !k.all_hours || (k.ablate & ~16) != 0) return false;  // 16: diagnostic counters
  if (w.disrupt_ext & (CCKA_DISRUPT_DRIFT | CCKA_DISRUPT_REPLACE | CCKA_DISRUPT_MULTI)) return false;
  for (int d = 0; d < w.n_deploy; ++d) {
    const int sc = w.deploy[d].scaler;
    if (sc != CCKA_SCALER_HPA && sc != CCKA_SCALER_STATIC) return false;
    if (sc == CCKA_SCALER_HPA && w.deploy[d].target_util_pct <= 0) return false;
  }
  return true;
}

int ccka_rollout_async(ccka_ctx* c, int32_t trajectory) {
  if (!c) return CCKA_EINVAL;
  if (!c->have_world || !c->have_sc) return fail(c, CCKA_ESTATE, "world/scenarios not set");
  if (!c->have_load) return fail(c, CCKA_ESTATE, "no load traces (ccka_set_load / ccka_gen_load)");
  (void)hipSetDevice(c->device);
  const ccka_world& w = c->hw;
  int block = 256;
  size_t lds = 0;
  int rc;
  if ((rc = setup_general(c, trajectory, &block, &lds)) != CCKA_OK) return rc;
  KParams& k = c->kp;
  if (c->engine_mode == 0 && c->d1_world && !c->d1_ready && (rc = d1_prepare(c)) != CCKA_OK) return rc;
  if (c->engine_mode == 0 && c->d1_world && c->d1_ok && !c->detail_on) {
    // single-deployment engine: argmin tables for this rollout, then the rollout
    TableParams tp{};
    tp.price = c->d_price; tp.ci_gpwh = c->d_ci_gpwh; tp.types = c->d_types;
    tp.order = c->d_order; tp.cap1s = c->d_cap1s; tp.cap1t = c->d_cap1t; tp.zmasks = c->d_zmasks; tp.wc1000 = c->d_wc1000;
    tp.table = c->d_table; tp.jtab = c->d_jtab;
    tp.K = w.n_types; tp.Z = w.n_zones; tp.R = w.n_regions; tp.NZI = (int)c->zmasks.size();
    tp.NW = c->NW; tp.JT = c->JT;
    D1Params& p = c->d1;
    p.load = c->d_load; p.price = c->d_price; p.ci_gpwmin = c->d_ci_gpwmin; p.acc = c->d_acc;
    p.table = c->d_table; p.jtab = c->d_jtab;
    p.region = c->d_region; p.target = c->d_target; p.maxr = c->d_maxr; p.down_stab = c->d_dstab;
    p.reset_ca = c->d_resetca; p.pswitch = c->d_pswitch; p.wci = c->d_wci; p.cap_sel = c->d_capsel;
    p.cost = k.cost; p.energy = k.energy; p.gco2 = k.gco2; p.slo = k.slo; p.pend_min = k.pend_min;
    p.nmin_spot = k.nmin_spot; p.nmin_od = k.nmin_od; p.launches = k.launches; p.deletions = k.deletions;
    p.peak_nodes = k.peak_nodes; p.final_reps = k.final_reps; p.final_nodes = k.final_nodes;
    p.last_choice = k.last_choice; p.hash = k.hash; p.traj = k.traj;
    p.N = c->N;
    p.NL = k.NL;
    p.trace_mod = k.trace_mod;
    p.first_id = k.first_id;
    p.NW = c->NW;
    p.occ = c->occ > 0 ? c->occ : 2;  // higher targets spill (measured slower: tools/occ.py)
    p.lpw = d1_lpw(c);
    p.load_w = nullptr;
    if (!c->trace_flat) {
      if ((rc = d1_trace_tile(c)) != CCKA_OK) return rc;
      if (c->load_w_lpw == p.lpw && c->d_load_w && p.trace_mod == 0) p.load_w = c->d_load_w;
    }
    p.ablate = k.ablate;
    p.stamps = nullptr;
    if (k.ablate & 16) {  // diagnostic phase stamps (single-deployment engine, 8 slots, 2 pools)
      if (!c->d_stamps && hipMalloc((void**)&c->d_stamps, 12 * sizeof(unsigned long long)) != hipSuccess)
        return fail(c, CCKA_ENOMEM, "stamps alloc");
      HIPCHK(c, hipMemsetAsync(c->d_stamps, 0, 12 * sizeof(unsigned long long), c->stream));
      p.stamps = c->d_stamps;
    }
    HIPCHK(c, hipEventRecord(c->ev0, c->stream));
    HIPCHK(c, launch_table(tp, c->stream));
    p.table2 = nullptr;
    if (p.replace || p.multi) {  // the G2 / G3 offer table (price only)
      TableParams t2 = tp;
      t2.wc1000 = c->d_wc0;
      t2.NW = 1;
      t2.offer = 1;
      t2.table = c->d_table2;
      t2.jtab = c->d_jtab2;
      HIPCHK(c, launch_table(t2, c->stream));
      p.table2 = c->d_table2;
    }
    HIPCHK(c, hipEventRecord(c->ev_mid, c->stream));
    p.cap1t = c->d_cap1t;
    p.pool_min = c->pool_min;
    p.pool_age = c->pool_age;
    p.pool_idle = c->pool_idle;
    D1Params q = p;
    c->last_pooled = d1_pool_plan(c, q);
    if (c->last_pooled) HIPCHK(c, launch_rollout_pool(q, c->stream));
    else HIPCHK(c, launch_rollout_d1(p, c->stream));
    HIPCHK(c, hipEventRecord(c->ev1, c->stream));
    c->last_engine = 2;
    c->traj_nt = true;
  } else {
    k.ptable = nullptr;  // the argmin-table launches are the policy loops' (weights k / 16)
    k.pjtab = nullptr;
    k.stamps = nullptr;
    if (k.ablate & 16) {  // diagnostic phase stamps (read by ccka_debug_stamps; GK_STAMPS builds)
      if (!c->d_stamps && hipMalloc((void**)&c->d_stamps, 12 * sizeof(unsigned long long)) != hipSuccess)
        return fail(c, CCKA_ENOMEM, "stamps alloc");
      HIPCHK(c, hipMemsetAsync(c->d_stamps, 0, 12 * sizeof(unsigned long long), c->stream));
      k.stamps = c->d_stamps;
    }
    const bool sk = sk_eligible(c);
    k.load_nt = nullptr;
    if (sk) {
      if ((rc = sk_trace(c)) != CCKA_OK) return rc;
      if (c->load_nt_dp) k.load_nt = c->d_load_nt;
      // lane-local provisioning for small catalogs: one LDS column of NodeClaims
      // per lane ([claim][field][lane] ints) when it fits beside the rest
      int dmax, nmax;
      kernel_dims(w.n_deploy, w.max_nodes, &dmax, &nmax);
      const size_t col = ((lds + 15) & ~(size_t)15), need = (size_t)nmax * (7 + dmax) * block * 4;
      if (!c->sk_coop_f2 && c->sk_lane_f2 && w.n_types <= 64 && col + need <= 160 * 1024) {
        k.lds_lclaims = (int32_t)col;
        lds = col + need;
      }
    }
    HIPCHK(c, hipEventRecord(c->ev0, c->stream));
    HIPCHK(c, hipEventRecord(c->ev_mid, c->stream));
    if (sk) HIPCHK(c, launch_rollout_sk(k, block, lds, c->stream));
    else HIPCHK(c, launch_rollout(k, block, lds, c->stream));
    HIPCHK(c, hipEventRecord(c->ev1, c->stream));
    c->last_engine = sk ? 5 : 1;
    c->traj_nt = sk;  // the skewed schedule writes scenario-major records
  }
  c->traj_valid = trajectory != 0;
  c->detail_valid = c->detail_on;
  c->ran = true;
  return CCKA_OK;
}

int ccka_set_detail(ccka_ctx* c, int32_t on) {
  if (!c) return CCKA_EINVAL;
  c->detail_on = on != 0;
  return CCKA_OK;
}

int ccka_get_detail(ccka_ctx* c, ccka_detail* out, int64_t count) {
  if (!c || !out) return CCKA_EINVAL;
  if (!c->ran || !c->detail_valid) return fail(c, CCKA_ESTATE, "last rollout recorded no detail (ccka_set_detail)");
  if (count != c->N) return fail(c, CCKA_EINVAL, "detail count %lld != %lld scenarios", (long long)count, (long long)c->N);
  (void)hipSetDevice(c->device);
  HIPCHK(c, hipMemcpy2DAsync(out, sizeof(ccka_detail), c->d_detail, sizeof(DetailDev), sizeof(ccka_detail), (size_t)count,
                             hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return CCKA_OK;
}

int ccka_sync(ccka_ctx* c) {
  if (!c) return CCKA_EINVAL;
  (void)hipSetDevice(c->device);
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (c->ran) {
    float ms = 0.f, tab = 0.f;
    HIPCHK(c, hipEventElapsedTime(&ms, c->ev_mid, c->ev1));
    HIPCHK(c, hipEventElapsedTime(&tab, c->ev0, c->ev_mid));
    c->last_ms = ms;
    c->last_table_ms = tab;
  }
  return CCKA_OK;
}

int ccka_rollout(ccka_ctx* c, int32_t trajectory) {
  int rc = ccka_rollout_async(c, trajectory);
  if (rc != CCKA_OK) return rc;
  return ccka_sync(c);
}

static int mlp_alloc(ccka_ctx* c, int64_t n);

// ---- closed-loop learned control policy (config 5) ----

// The closed loop (SEMANTICS 5). pg == nullptr: the deterministic policy
// (policy_act_kernel); otherwise each step samples an action bin from
// softmax(y) (policy_sample_kernel) and the features and actions of every
// step are kept for the score-function gradient (ccka_policy_grad).
// The fused loop's Karpenter launches on a single-deployment world without
// pool limits (d1_check_world) read argmin tables instead of scanning the
// catalog: table_kernel over every carbon weight the policy can emit (k / 16,
// k = 0..64; the sampled policy's 0 and 1 are k = 0 and 16), rebuilt per loop
// on the stream (prices and carbon intensity are the world's). Leaves
// k->ptable null when the world does not qualify.
static int policy_tables(ccka_ctx* c, KParams* k) {
  const ccka_world& w = c->hw;
  if (!c->d1_world || w.n_zones > 4 || c->zmasks.empty()) return CCKA_OK;
  constexpr int NWP = 65;
  const int64_t keys = (int64_t)w.n_regions * 24 * (int64_t)c->zmasks.size() * 3;
  const int64_t cnt = keys * NWP * c->JT;
  if (c->ptable_count != cnt) {
    dfree(c->d_ptable);
    dfree(c->d_pjtab);
    c->ptable_count = 0;
    if (hipMalloc((void**)&c->d_ptable, (size_t)cnt * sizeof(int2)) != hipSuccess ||
        hipMalloc((void**)&c->d_pjtab, (size_t)keys * sizeof(int32_t)) != hipSuccess) {
      // no memory for the tables: the fused loop scans the catalog instead (same choices)
      (void)hipGetLastError();
      dfree(c->d_ptable);
      dfree(c->d_pjtab);
      return CCKA_OK;
    }
    c->ptable_count = cnt;
  }
  if (!c->d_pwc) {
    double wc[NWP];
    for (int x = 0; x < NWP; ++x) wc[x] = (double)x / 16.0 * 1000.0;  // the kernel's c * 1000.0
    int rc;
    if ((rc = dupload(c, c->d_pwc, wc, (size_t)NWP)) != CCKA_OK) return rc;
  }
  TableParams tp{};
  tp.price = c->d_price; tp.ci_gpwh = c->d_ci_gpwh; tp.types = c->d_types;
  tp.order = c->d_order; tp.cap1s = c->d_cap1s; tp.cap1t = c->d_cap1t; tp.zmasks = c->d_zmasks; tp.wc1000 = c->d_pwc;
  tp.table = c->d_ptable; tp.jtab = c->d_pjtab;
  tp.K = w.n_types; tp.Z = w.n_zones; tp.R = w.n_regions; tp.NZI = (int)c->zmasks.size();
  tp.NW = NWP; tp.JT = c->JT;
  HIPCHK(c, launch_table(tp, c->stream));
  k->ptable = c->d_ptable;
  k->pjtab = c->d_pjtab;
  k->pNZI = tp.NZI;
  k->pJT = c->JT;
  k->pNW = NWP;
  const uint32_t zall = (1u << w.n_zones) - 1u;
  for (uint32_t m = 0; m < 16; ++m) {
    k->pzmi[m] = -1;
    for (size_t z = 0; z < c->zmasks.size(); ++z)
      if ((m & zall) && c->zmasks[z] == (m & zall)) k->pzmi[m] = (int32_t)z;
  }
  return CCKA_OK;
}

static int policy_loop(ccka_ctx* c, int32_t trajectory, int32_t record, const ccka_pg_params* pg) {
  if (!c) return CCKA_EINVAL;
  c->pg_valid = false;  // the recorded features / actions are about to be overwritten
  if (!c->have_world || !c->have_sc) return fail(c, CCKA_ESTATE, "world/scenarios not set");
  // the single-deployment kernel's tiled trace copy (N*T*4 bytes) and the
  // skewed schedule's scenario-major one are not read here: released for the
  // loop's own arrays, rebuilt by the next rollout
  dfree(c->d_load_w);
  c->load_w_count = 0;
  c->load_w_lpw = 0;
  dfree(c->d_load_nt);
  c->load_nt_count = 0;
  c->load_nt_dp = 0;
  if (!c->have_load) return fail(c, CCKA_ESTATE, "no load traces (ccka_set_load / ccka_gen_load)");
  if (!c->mlp_have_w) return fail(c, CCKA_ESTATE, "MLP weights not set (ccka_mlp_set_weights)");
  (void)hipSetDevice(c->device);
  const ccka_world& w = c->hw;
  const int64_t N = c->N;
  const int T = w.n_steps;
  int block = 256;
  size_t lds = 0;
  int rc;
  if ((rc = setup_general(c, trajectory, &block, &lds)) != CCKA_OK) return rc;
  KParams& k = c->kp;
  int dmax, nmax;
  kernel_dims(w.n_deploy, w.max_nodes, &dmax, &nmax);
  const int64_t words = state_words(dmax, nmax);
  if (c->pol_state_count < words * N) {
    dfree(c->d_pol_state);
    c->pol_state_count = 0;
    if (hipMalloc((void**)&c->d_pol_state, (size_t)(words * N) * 4) != hipSuccess)
      return fail(c, CCKA_ENOMEM, "policy state alloc (%lld words)", (long long)(words * N));
    c->pol_state_count = words * N;
  }
  if (c->pol_n < N) {
    dfree(c->d_pol_target);
    dfree(c->d_pol_cw);
    c->pol_n = 0;
    if (hipMalloc((void**)&c->d_pol_target, (size_t)N * 2) != hipSuccess ||
        hipMalloc((void**)&c->d_pol_cw, (size_t)N * 8) != hipSuccess)
      return fail(c, CCKA_ENOMEM, "policy action alloc");
    c->pol_n = N;
  }
  c->pol_rec_valid = false;
  if (record) {
    if (c->pol_rec_count < (int64_t)T * N) {
      dfree(c->d_rec_target);
      dfree(c->d_rec_cw);
      c->pol_rec_count = 0;
      if (hipMalloc((void**)&c->d_rec_target, (size_t)T * N * 2) != hipSuccess ||
          hipMalloc((void**)&c->d_rec_cw, (size_t)T * N * 8) != hipSuccess)
        return fail(c, CCKA_ENOMEM, "policy action record alloc");
      c->pol_rec_count = (int64_t)T * N;
    }
  }
  const bool feat_on = c->pol_feat_on || pg;
  if (pg) {
    if (c->pg_act_count < (int64_t)T * N) {
      dfree(c->d_pg_act);
      c->pg_act_count = 0;
      if (hipMalloc((void**)&c->d_pg_act, (size_t)T * N) != hipSuccess)
        return fail(c, CCKA_ENOMEM, "policy-gradient action record alloc");
      c->pg_act_count = (int64_t)T * N;
    }
  }
  if (feat_on) {
    if (c->pol_feat_count < (int64_t)(T + 1) * N * 64) {
      dfree(c->d_feat_rec);
      c->pol_feat_count = 0;
      if (hipMalloc((void**)&c->d_feat_rec, (size_t)(T + 1) * N * 64 * 2) != hipSuccess)
        return fail(c, CCKA_ENOMEM, "policy feature record alloc");
      c->pol_feat_count = (int64_t)(T + 1) * N * 64;
    }
  }
  if ((rc = mlp_alloc(c, N)) != CCKA_OK) return rc;
  if (pg) {
    if (!c->d_pg_seed && hipMalloc((void**)&c->d_pg_seed, sizeof(uint64_t)) != hipSuccess)
      return fail(c, CCKA_ENOMEM, "seed alloc");
    // the seed is data, not part of a captured sequence: a new seed replays the graph
    c->pg_seed_host = pg->seed;
    HIPCHK(c, hipMemcpyAsync(c->d_pg_seed, &c->pg_seed_host, sizeof(uint64_t), hipMemcpyHostToDevice, c->stream));
  }
  // ---- the fused loop (rollout_kernel<1, 8, POL>): one deployment, <= 8 node
  // slots and the MLP's W2 fragments + biases beside the kernel's LDS ----
  {
    const size_t mlp_lds = (size_t)((MLP_HID / 32) * (MLP_HID / 16) + MLP_HID / 16) * 64 * 16 + (2 * MLP_HID + 32) * 4;
    const size_t off = (lds + 15) & ~(size_t)15;
    if (!c->pol_fused_off && dmax == 1 && nmax == 8 && off + mlp_lds <= 160 * 1024) {
      k.t0 = 0;
      k.t1 = T;
      k.state = nullptr;
      k.state_load = 0;
      k.feat = c->d_mx;  // the last step's features become the MLP states
      k.w1f = c->d_w1f;
      k.w2f = c->d_w2f;
      k.w3f = c->d_w3f;
      k.mlp_b = c->d_mb;
      k.pol_seed = pg ? c->d_pg_seed : nullptr;
      k.rec_target = record ? c->d_rec_target : nullptr;
      k.rec_cw = record ? c->d_rec_cw : nullptr;
      k.pol_act = pg ? c->d_pg_act : nullptr;
      k.feat_rec = feat_on ? c->d_feat_rec : nullptr;
      k.lds_off_mlp = (int32_t)off;
      // the fused-only fields leave the persistent parameter block on every path
      auto clear_fused = [&]() {
        k.ptable = nullptr;
        k.pjtab = nullptr;
        k.feat = nullptr;
        k.w1f = k.w2f = k.w3f = nullptr;
        k.mlp_b = nullptr;
        k.pol_seed = nullptr;
        k.rec_target = nullptr;
        k.rec_cw = nullptr;
        k.pol_act = nullptr;
        k.feat_rec = nullptr;
      };
      k.stamps = nullptr;
      if (k.ablate & 16) {  // diagnostic phase stamps (GK_STAMPS builds; ccka_debug_stamps)
        if (!c->d_stamps && hipMalloc((void**)&c->d_stamps, 12 * sizeof(unsigned long long)) != hipSuccess) {
          clear_fused();
          return fail(c, CCKA_ENOMEM, "stamps alloc");
        }
        HIPCHK(c, hipMemsetAsync(c->d_stamps, 0, 12 * sizeof(unsigned long long), c->stream));
        k.stamps = c->d_stamps;
      }
      hipError_t le = hipEventRecord(c->ev0, c->stream);
      k.ptable = nullptr;
      if (le == hipSuccess && !c->pol_table_off && (rc = policy_tables(c, &k)) != CCKA_OK) {
        clear_fused();
        return rc;
      }
      if (le == hipSuccess) le = hipEventRecord(c->ev_mid, c->stream);
      if (le == hipSuccess) le = launch_rollout_policy(k, off + mlp_lds, pg ? 2 : 1, c->stream);
      clear_fused();
      HIPCHK(c, le);
      HIPCHK(c, hipEventRecord(c->ev1, c->stream));
      c->last_engine = 4;
      c->traj_nt = false;
      c->traj_valid = trajectory != 0;
      c->detail_valid = c->detail_on;
      c->pol_rec_valid = record != 0;
      c->ran = true;
      return ccka_sync(c);
    }
  }
  MlpParams mp{};
  mp.x = c->d_mx;
  mp.y = c->d_my;
  mp.w1f = c->d_w1f;
  mp.w2f = c->d_w2f;
  mp.w3f = c->d_w3f;
  mp.b1 = c->d_mb;
  mp.b2 = c->d_mb + MLP_HID;
  mp.b3 = c->d_mb + 2 * MLP_HID;
  mp.N = N;
  mp.stamps = nullptr;
  // the policy's actions replace the scenarios' target / carbon-weight overrides
  k.target = c->d_pol_target;
  k.cw = c->d_pol_cw;
  k.state = c->d_pol_state;
  k.feat = c->d_mx;
  auto keep_feat = [&](int t) -> int {
    if (!feat_on) return CCKA_OK;
    HIPCHK(c, hipMemcpyAsync(c->d_feat_rec + (size_t)t * N * 64, c->d_mx, (size_t)N * 64 * 2, hipMemcpyDeviceToDevice,
                             c->stream));
    return CCKA_OK;
  };
  PgSampleParams q0{};
  if (pg) {
    q0.y = c->d_my;
    q0.target = c->d_pol_target;
    q0.cw = c->d_pol_cw;
    q0.n = N;
    q0.first_id = c->first_id;
    q0.seed = c->d_pg_seed;
  }
  // the whole loop: state initialisation (t = 0, features of step 0), then
  // per step MLP -> actions -> one rollout step (+ the features kept)
  auto enqueue = [&]() -> int {
    k.t0 = 0;
    k.t1 = 0;
    k.state_load = 0;
    HIPCHK(c, launch_rollout(k, block, lds, c->stream));
    if ((rc = keep_feat(0)) != CCKA_OK) return rc;
    for (int t = 0; t < T; ++t) {
      HIPCHK(c, launch_mlp(mp, c->cus, c->stream));
      if (pg) {
        PgSampleParams q = q0;
        q.act = c->d_pg_act + (size_t)t * N;
        q.rec_target = record ? c->d_rec_target + (size_t)t * N : nullptr;
        q.rec_cw = record ? c->d_rec_cw + (size_t)t * N : nullptr;
        q.t = t;
        HIPCHK(c, launch_policy_sample(q, c->stream));
      } else {
        HIPCHK(c, launch_policy_act(c->d_my, c->d_pol_target, c->d_pol_cw,
                                    record ? c->d_rec_target + (size_t)t * N : nullptr,
                                    record ? c->d_rec_cw + (size_t)t * N : nullptr, N, c->stream));
      }
      k.t0 = t;
      k.t1 = t + 1;
      k.state_load = 1;
      HIPCHK(c, launch_rollout(k, block, lds, c->stream));
      if ((rc = keep_feat(t + 1)) != CCKA_OK) return rc;
    }
    return CCKA_OK;
  };
  // (launches by the wave-cooperative catalog scans: the argmin-table path is
  // the fused kernel's, whose register budget has room for it)
  k.ptable = nullptr;
  // graph key: every input of the sequence (parameter blocks by value: their
  // device pointers and sizes)
  std::vector<unsigned char> key;
  auto put = [&](const void* v, size_t n) {
    const unsigned char* b = static_cast<const unsigned char*>(v);
    key.insert(key.end(), b, b + n);
  };
  {
    KParams k0 = k;
    k0.t0 = k0.t1 = k0.state_load = 0;
    put(&k0, sizeof k0);
    put(&mp, sizeof mp);
    put(&q0, sizeof q0);
    const int64_t misc[10] = {N, T, block, (int64_t)lds, record, feat_on, pg != nullptr, c->cus,
                              (int64_t)(uintptr_t)c->d_feat_rec, (int64_t)(uintptr_t)c->d_rec_target};
    put(misc, sizeof misc);
    const void* ptrs[3] = {c->d_rec_cw, c->d_pg_act, c->stream};
    put(ptrs, sizeof ptrs);
  }
  HIPCHK(c, hipEventRecord(c->ev0, c->stream));
  HIPCHK(c, hipEventRecord(c->ev_mid, c->stream));
  if (c->pol_graph_off) {
    if ((rc = enqueue()) != CCKA_OK) return rc;
  } else {
    if (!c->pol_graph || key != c->pol_graph_key) {
      if (c->pol_graph) {
        (void)hipGraphExecDestroy(c->pol_graph);
        c->pol_graph = nullptr;
      }
      hipGraph_t g = nullptr;
      HIPCHK(c, hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal));
      const int erc = enqueue();
      const hipError_t ce = hipStreamEndCapture(c->stream, &g);
      if (erc != CCKA_OK) {
        if (g) (void)hipGraphDestroy(g);
        return erc;
      }
      HIPCHK(c, ce);
      const hipError_t ie = hipGraphInstantiate(&c->pol_graph, g, nullptr, nullptr, 0);
      (void)hipGraphDestroy(g);
      HIPCHK(c, ie);
      c->pol_graph_key = key;
    }
    HIPCHK(c, hipGraphLaunch(c->pol_graph, c->stream));
  }
  HIPCHK(c, hipEventRecord(c->ev1, c->stream));
  // back to whole-horizon rollouts with the scenarios' own overrides
  k.ptable = nullptr;
  k.pjtab = nullptr;
  k.target = c->d_target;
  k.cw = c->d_cw;
  k.state = nullptr;
  k.feat = nullptr;
  k.t0 = 0;
  k.t1 = T;
  k.state_load = 0;
  c->last_engine = 3;
  c->traj_nt = false;
  c->traj_valid = trajectory != 0;
  c->detail_valid = c->detail_on;
  c->pol_rec_valid = record != 0;
  c->ran = true;
  return ccka_sync(c);
}

int ccka_policy_rollout(ccka_ctx* c, int32_t trajectory, int32_t record) {
  return policy_loop(c, trajectory, record, nullptr);
}

// ---- differentiable control: the MLP backward (pg.hip) ----
// rows m = 0..M-1 of x [M][64] bf16 / act [M] / coef[m % n_scen] -> d_pg_grad
// (dW1 | db1 | dW2 | db2 | dW3 | db3, fp32, the layouts of ccka_mlp_set_weights)
static constexpr int64_t kGradFloats = 64 * 256 + 256 + 256 * 256 + 256 + 256 * 8 + 8;
// Rows per backward chunk: the work arrays hold 1,096 bf16 units per row
// (2.2 KB), so all N*T rows of a large loop do not fit at once (1e7 x 60 would
// need 1.3 TB). Chunks of kPgChunkRows rows run one after another, each
// chunk's gradient added to the running sum in chunk order: the result depends
// only on M, never on the memory available (deterministic); M <= one chunk is
// the unchunked computation.
constexpr int64_t kPgChunkRows = 1LL << 23;
constexpr int64_t kPgSplits = 256;  // weight-gradient row splits per chunk (at most; 512 measured 21.8 -> 22.6 ms)
static int64_t pg_chunk_rows(const ccka_ctx* c) { return c->pg_chunk > 0 ? c->pg_chunk : kPgChunkRows; }

static int pg_backward(ccka_ctx* c, const uint16_t* x, const uint8_t* act, const float* coef, int64_t n_scen,
                       int64_t M) {
  if (!c->mlp_have_w) return fail(c, CCKA_ESTATE, "MLP weights not set (ccka_mlp_set_weights)");
  if (M < 1 || n_scen < 1) return fail(c, CCKA_EINVAL, "no rows");
  const int64_t rows = 64 + 4 * MLP_HID + 8;  // xT h1T h2T dh1T dh2T gyT
  const int64_t CH = pg_chunk_rows(c);
  const int64_t cap = (std::min(M, CH) + 31) / 32 * 32;
  if (c->pg_work_count < rows * cap) {
    dfree(c->d_pg_work);
    c->pg_work_count = 0;
    if (hipMalloc((void**)&c->d_pg_work, (size_t)(rows * cap) * 2) != hipSuccess)
      return fail(c, CCKA_ENOMEM, "policy-gradient work alloc (%lld rows x %lld)", (long long)rows, (long long)cap);
    c->pg_work_count = rows * cap;
  }
  if (!c->d_pg_grad && hipMalloc((void**)&c->d_pg_grad, (size_t)kGradFloats * 4) != hipSuccess)
    return fail(c, CCKA_ENOMEM, "gradient alloc");
  // the three weight-gradient GEMMs over all rows, each with its bias gradient
  // (the row sums of its B operand) folded in: dW1 | db1, dW2 | db2, dW3 | db3
  const int64_t o_b1 = 64 * 256, o_w2 = o_b1 + 256, o_b2 = o_w2 + 256 * 256, o_w3 = o_b2 + 256, o_b3 = o_w3 + 256 * 8;
  for (int64_t r0 = 0; r0 < M; r0 += CH) {
    const int64_t Mc = std::min(CH, M - r0);
    const int64_t Mpad = (Mc + 31) / 32 * 32;
    uint16_t* xT = c->d_pg_work;
    uint16_t* h1T = xT + 64 * Mpad;
    uint16_t* h2T = h1T + MLP_HID * Mpad;
    uint16_t* dh1T = h2T + MLP_HID * Mpad;
    uint16_t* dh2T = dh1T + MLP_HID * Mpad;
    uint16_t* gyT = dh2T + MLP_HID * Mpad;
    PgRowsParams rp{};
    rp.x = x + r0 * MLP_IN;
    rp.act = act + r0;
    rp.coef = coef;
    rp.w1f = c->d_w1f;
    rp.w2f = c->d_w2f;
    rp.w3f = c->d_w3f;
    rp.w2b = c->d_w2b;
    rp.w3b = c->d_w3b;
    rp.bias = c->d_mb;
    rp.xT = xT; rp.h1T = h1T; rp.h2T = h2T; rp.dh1T = dh1T; rp.dh2T = dh2T; rp.gyT = gyT;
    rp.M = Mc;
    rp.Mpad = Mpad;
    rp.n_scen = n_scen;
    rp.row0 = r0;
    HIPCHK(c, launch_pg_rows(rp, c->cus, c->stream));
    struct G { const uint16_t* a; int ka; const uint16_t* b; int kb; int64_t off, boff; };
    const G gs[3] = {{xT, 64, dh1T, MLP_HID, 0, o_b1}, {h1T, MLP_HID, dh2T, MLP_HID, o_w2, o_b2},
                     {h2T, MLP_HID, gyT, MLP_OUT, o_w3, o_b3}};
    // one workgroup per split owns a share of the chunk's rows and the whole
    // output (pg.hip); the split count is a function of Mpad alone (256 = the
    // MI355X's CU count, not the device's), so the gradient's summation order
    // and bits do not depend on the GPU or its partition mode
    const int splits = (int)std::max<int64_t>(1, std::min<int64_t>(kPgSplits, Mpad / 256));
    // each split's partials in the packed gradient order (w1 | b1 | w2 | b2 |
    // w3 | b3): one reduction for the three GEMMs
    const int64_t need = (int64_t)splits * kGradFloats;
    if (c->pg_part_count < need) {
      dfree(c->d_pg_part);
      c->pg_part_count = 0;
      if (hipMalloc((void**)&c->d_pg_part, (size_t)need * 4) != hipSuccess)
        return fail(c, CCKA_ENOMEM, "gradient partials alloc");
      c->pg_part_count = need;
    }
    for (const G& g : gs) {
      WgradParams q{};
      q.A = g.a;
      q.B = g.b;
      q.part = c->d_pg_part + g.off;
      q.bpart = c->d_pg_part + g.boff;
      q.Mpad = Mpad;
      q.pstride = kGradFloats;
      q.KA = g.ka;
      q.KB = g.kb;
      q.splits = splits;
      HIPCHK(c, launch_pg_wgrad(q, c->stream));
    }
    HIPCHK(c, launch_pg_reduce(c->d_pg_part, c->d_pg_grad, kGradFloats, splits, r0 > 0 ? 1 : 0, c->stream));
  }
  return CCKA_OK;
}

static int pg_copy_grads(ccka_ctx* c, ccka_mlp_grads* out) {
  if (!out) return CCKA_OK;
  const int64_t o_b1 = 64 * 256, o_w2 = o_b1 + 256, o_b2 = o_w2 + 256 * 256, o_w3 = o_b2 + 256, o_b3 = o_w3 + 256 * 8;
  const struct { float* dst; int64_t off, n; } m[6] = {{out->w1, 0, 64 * 256}, {out->b1, o_b1, 256},
                                                      {out->w2, o_w2, 256 * 256}, {out->b2, o_b2, 256},
                                                      {out->w3, o_w3, 256 * 8}, {out->b3, o_b3, 8}};
  for (const auto& x : m)
    if (x.dst) HIPCHK(c, hipMemcpyAsync(x.dst, c->d_pg_grad + x.off, (size_t)x.n * 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return CCKA_OK;
}

int ccka_mlp_backward(ccka_ctx* c, const uint16_t* x, const uint8_t* actions, const float* coef, int64_t m,
                      ccka_mlp_grads* out) {
  if (!c || !x || !actions || !coef || !out || m < 1) return CCKA_EINVAL;
  (void)hipSetDevice(c->device);
  if (c->pg_x_count < m * MLP_IN) {
    dfree(c->d_pg_x);
    c->pg_x_count = 0;
    if (hipMalloc((void**)&c->d_pg_x, (size_t)m * MLP_IN * 2) != hipSuccess)
      return fail(c, CCKA_ENOMEM, "backward rows alloc");
    c->pg_x_count = m * MLP_IN;
  }
  if (c->pg_act_count < m) {
    dfree(c->d_pg_act);
    c->pg_act_count = 0;
    if (hipMalloc((void**)&c->d_pg_act, (size_t)m) != hipSuccess) return fail(c, CCKA_ENOMEM, "action alloc");
    c->pg_act_count = m;
  }
  if (c->pg_coef_count < m) {
    dfree(c->d_pg_coef);
    c->pg_coef_count = 0;
    if (hipMalloc((void**)&c->d_pg_coef, (size_t)m * 4) != hipSuccess) return fail(c, CCKA_ENOMEM, "coef alloc");
    c->pg_coef_count = m;
  }
  for (int64_t i = 0; i < m; ++i)
    if (actions[i] >= MLP_OUT) return fail(c, CCKA_EINVAL, "action %d of row %lld out of range", actions[i], (long long)i);
  HIPCHK(c, hipMemcpyAsync(c->d_pg_x, x, (size_t)m * MLP_IN * 2, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(c->d_pg_act, actions, (size_t)m, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(c->d_pg_coef, coef, (size_t)m * 4, hipMemcpyHostToDevice, c->stream));
  c->pg_valid = false;  // the recorded samples of ccka_policy_grad are gone
  int rc;
  if ((rc = pg_backward(c, c->d_pg_x, c->d_pg_act, c->d_pg_coef, m, m)) != CCKA_OK) return rc;
  return pg_copy_grads(c, out);
}

int ccka_policy_grad(ccka_ctx* c, const ccka_pg_params* pg, ccka_mlp_grads* out, double* objective_mean) {
  if (!c || !pg) return CCKA_EINVAL;
  if (!(pg->w_carbon >= 0.0) || !(pg->w_slo >= 0.0)) return fail(c, CCKA_EINVAL, "objective weights must be >= 0");
  (void)hipSetDevice(c->device);
  int rc;
  if ((rc = policy_loop(c, 0, 1, pg)) != CCKA_OK) return rc;
  const int64_t N = c->N;
  const int64_t T = c->hw.n_steps;
  // J_i = cost $ + w_c gCO2 kg + w_s SLO minutes; coef_i = (J_i - b) / N
  std::vector<int64_t> cost((size_t)N);
  std::vector<double> g((size_t)N);
  std::vector<int32_t> slo((size_t)N);
  HIPCHK(c, hipMemcpyAsync(cost.data(), c->kp.cost, (size_t)N * 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(g.data(), c->kp.gco2, (size_t)N * 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(slo.data(), c->kp.slo, (size_t)N * 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  std::vector<double> J((size_t)N);
  double sum = 0.0;
  for (int64_t i = 0; i < N; ++i) {
    J[(size_t)i] = (double)cost[(size_t)i] / 6e7 + pg->w_carbon * (g[(size_t)i] * 1e-3) + pg->w_slo * (double)slo[(size_t)i];
    sum += J[(size_t)i];
  }
  const double mean = sum / (double)N, b = pg->baseline ? mean : 0.0;
  std::vector<float> coef((size_t)N);
  for (int64_t i = 0; i < N; ++i) coef[(size_t)i] = (float)((J[(size_t)i] - b) / (double)N);
  if (objective_mean) *objective_mean = mean;
  if (c->pg_coef_count < N) {
    dfree(c->d_pg_coef);
    c->pg_coef_count = 0;
    if (hipMalloc((void**)&c->d_pg_coef, (size_t)N * 4) != hipSuccess) return fail(c, CCKA_ENOMEM, "coef alloc");
    c->pg_coef_count = N;
  }
  HIPCHK(c, hipMemcpyAsync(c->d_pg_coef, coef.data(), (size_t)N * 4, hipMemcpyHostToDevice, c->stream));
  // rows (t, i) -> m = t N + i: the recorded features [T+1][N][64] (steps 0..T-1) and actions [T][N]
  if ((rc = pg_backward(c, c->d_feat_rec, c->d_pg_act, c->d_pg_coef, N, T * N)) != CCKA_OK) return rc;
  c->pg_valid = true;
  c->pg_T = T;
  return pg_copy_grads(c, out);
}

// Internal (tests): the backward's unit-major work arrays of the last
// ccka_mlp_backward / ccka_policy_grad: xT | h1T | h2T | dh1T | dh2T | gyT,
// each row-blocked [Mpad/16][units][16] bf16; *mpad receives Mpad.
int ccka_debug_pg_work(ccka_ctx* c, uint16_t* out, int64_t count, int64_t* mpad) {
  if (!c || !out || !mpad || !c->d_pg_work) return CCKA_EINVAL;
  const int64_t rows = 64 + 4 * MLP_HID + 8;
  if (count < c->pg_work_count) return fail(c, CCKA_EINVAL, "need %lld", (long long)c->pg_work_count);
  (void)hipSetDevice(c->device);
  *mpad = c->pg_work_count / rows;
  HIPCHK(c, hipMemcpy(out, c->d_pg_work, (size_t)c->pg_work_count * 2, hipMemcpyDeviceToHost));
  return CCKA_OK;
}

int ccka_get_policy_samples(ccka_ctx* c, uint8_t* actions, float* coef, int64_t count) {
  if (!c || !actions || !coef) return CCKA_EINVAL;
  if (!c->pg_valid) return fail(c, CCKA_ESTATE, "no ccka_policy_grad samples");
  if (count != c->pg_T * c->N) return fail(c, CCKA_EINVAL, "sample count mismatch");
  (void)hipSetDevice(c->device);
  HIPCHK(c, hipMemcpyAsync(actions, c->d_pg_act, (size_t)count, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(coef, c->d_pg_coef, (size_t)c->N * 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return CCKA_OK;
}

int ccka_get_policy_actions(ccka_ctx* c, int16_t* target, double* cw, int64_t count) {
  if (!c || !target || !cw) return CCKA_EINVAL;
  if (!c->pol_rec_valid) return fail(c, CCKA_ESTATE, "last run recorded no policy actions");
  if (count != (int64_t)c->hw.n_steps * c->N) return fail(c, CCKA_EINVAL, "action count != T x N");
  (void)hipSetDevice(c->device);
  HIPCHK(c, hipMemcpyAsync(target, c->d_rec_target, (size_t)count * 2, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(cw, c->d_rec_cw, (size_t)count * 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return CCKA_OK;
}

// Internal test hooks (not part of include/ccka.h): record the policy
// features of every step ([T + 1][N][64] bf16) and read them back.
int ccka_debug_policy_features(ccka_ctx* c, int32_t enable) {
  if (!c) return CCKA_EINVAL;
  c->pol_feat_on = enable != 0;
  return CCKA_OK;
}

int ccka_debug_get_policy_features(ccka_ctx* c, uint16_t* out, int64_t count) {
  if (!c || !out) return CCKA_EINVAL;
  if (!(c->pol_feat_on || c->pg_valid) || !c->pol_rec_valid) return fail(c, CCKA_ESTATE, "no recorded features");
  if (count != (int64_t)(c->hw.n_steps + 1) * c->N * 64) return fail(c, CCKA_EINVAL, "feature count mismatch");
  (void)hipSetDevice(c->device);
  HIPCHK(c, hipMemcpyAsync(out, c->d_feat_rec, (size_t)count * 2, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return CCKA_OK;
}

int ccka_last_kernel_ms(ccka_ctx* c, double* ms) {
  if (!c || !ms) return CCKA_EINVAL;
  if (!c->ran) return fail(c, CCKA_ESTATE, "no rollout yet");
  *ms = c->last_ms;
  return CCKA_OK;
}

int ccka_get_results(ccka_ctx* c, ccka_results* o) {
  if (!c || !o) return CCKA_EINVAL;
  if (!c->ran) return fail(c, CCKA_ESTATE, "no rollout yet");
  (void)hipSetDevice(c->device);
  const size_t n = (size_t)c->N;
  const KParams& k = c->kp;
  struct { void* dst; const void* src; size_t sz; } m[] = {
      {o->cost_uphmin, k.cost, 8}, {o->energy_wmin, k.energy, 8}, {o->gco2, k.gco2, 8},
      {o->slo_minutes, k.slo, 4}, {o->pending_pod_minutes, k.pend_min, 8},
      {o->node_min_spot, k.nmin_spot, 4}, {o->node_min_od, k.nmin_od, 4},
      {o->launches, k.launches, 4}, {o->deletions, k.deletions, 4}, {o->peak_nodes, k.peak_nodes, 4},
      {o->final_replicas, k.final_reps, 4}, {o->final_nodes, k.final_nodes, 4},
      {o->last_choice, k.last_choice, 4}, {o->choice_hash, k.hash, 4}};
  for (auto& x : m)
    if (x.dst) HIPCHK(c, hipMemcpyAsync(x.dst, x.src, n * x.sz, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return CCKA_OK;
}

int ccka_get_trajectory(ccka_ctx* c, ccka_traj_rec* out, int64_t count) {
  if (!c || !out) return CCKA_EINVAL;
  if (!c->traj_valid) return fail(c, CCKA_ESTATE, "last rollout had no trajectory");
  if (count != c->traj_count) return fail(c, CCKA_EINVAL, "trajectory count mismatch");
  (void)hipSetDevice(c->device);
  if (!c->traj_nt) {  // already [T][N]
    HIPCHK(c, hipMemcpyAsync(out, c->d_traj, (size_t)count * sizeof(ccka_traj_rec), hipMemcpyDeviceToHost,
                             c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return CCKA_OK;
  }
  // the single-deployment engine keeps [N][T] on the device: transpose tc
  // steps at a time into a bounded staging buffer (>= one step of N records,
  // else kTrajStageRecs) and copy each block of steps to its place in out
  const int64_t N = c->N, T = count / N;
  const int64_t cap = std::max<int64_t>(N, std::min<int64_t>(count, kTrajStageRecs));
  if (c->traj_t_count < cap) {
    dfree(c->d_traj_t);
    c->traj_t_count = 0;
    if (hipMalloc((void**)&c->d_traj_t, (size_t)cap * sizeof(ccka_traj_rec)) != hipSuccess)
      return fail(c, CCKA_ENOMEM, "trajectory staging alloc (%lld records)", (long long)cap);
    c->traj_t_count = cap;
  }
  const int64_t tc = std::max<int64_t>(1, c->traj_t_count / N);
  for (int64_t t0 = 0; t0 < T; t0 += tc) {
    const int64_t n = std::min(tc, T - t0);
    HIPCHK(c, launch_traj_transpose(c->d_traj, c->d_traj_t, N, T, t0, n, c->stream));
    HIPCHK(c, hipMemcpyAsync(out + t0 * N, c->d_traj_t, (size_t)(n * N) * sizeof(ccka_traj_rec),
                             hipMemcpyDeviceToHost, c->stream));
  }
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return CCKA_OK;
}

int ccka_trajectory_layout(ccka_ctx* c, int32_t* layout) {
  if (!c || !layout) return CCKA_EINVAL;
  if (!c->traj_valid) return fail(c, CCKA_ESTATE, "last rollout had no trajectory");
  *layout = c->traj_nt ? CCKA_TRAJ_NT : CCKA_TRAJ_TN;
  return CCKA_OK;
}

int ccka_get_trajectory_native(ccka_ctx* c, ccka_traj_rec* out, int64_t count, int32_t* layout) {
  if (!c || !out) return CCKA_EINVAL;
  if (!c->traj_valid) return fail(c, CCKA_ESTATE, "last rollout had no trajectory");
  if (count != c->traj_count) return fail(c, CCKA_EINVAL, "trajectory count mismatch");
  (void)hipSetDevice(c->device);
  if (layout) *layout = c->traj_nt ? CCKA_TRAJ_NT : CCKA_TRAJ_TN;
  HIPCHK(c, hipMemcpyAsync(out, c->d_traj, (size_t)count * sizeof(ccka_traj_rec), hipMemcpyDeviceToHost,
                           c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return CCKA_OK;
}

int ccka_get_totals(ccka_ctx* c, ccka_totals* out) {
  if (!c || !out) return CCKA_EINVAL;
  if (!c->ran) return fail(c, CCKA_ESTATE, "no rollout yet");
  (void)hipSetDevice(c->device);
  TotParams q{};
  const KParams& k = c->kp;
  q.cost = k.cost; q.energy = k.energy; q.gco2 = k.gco2; q.slo = k.slo; q.pend_min = k.pend_min;
  q.nmin_spot = k.nmin_spot; q.nmin_od = k.nmin_od; q.launches = k.launches; q.deletions = k.deletions;
  q.parts = (Part*)c->d_parts;
  q.ovf = (long long*)c->d_parts + 1024 * 11;
  q.out = c->d_totals;
  q.N = c->N;
  const int nparts = (int)std::min<int64_t>(1024, (c->N + 255) / 256);
  long long ovf = 0;
  HIPCHK(c, launch_totals(q, nparts, c->stream));
  HIPCHK(c, hipMemcpyAsync(out, c->d_totals, sizeof(ccka_totals), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(&ovf, q.ovf, sizeof ovf, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (ovf) return fail(c, CCKA_EOVERFLOW, "a fixed-point total exceeds int64 (ccka.h: ccka_totals)");
  return CCKA_OK;
}

// ---- the totals exchange, host halves (ccka.h: ccka_totals_pack / _finish) ----
int ccka_totals_pack(const ccka_totals* in, int32_t nranks, int64_t* block, int32_t n) {
  if (!in || !block || n != CCKA_TOTALS_BLOCK || nranks < 1) return CCKA_EINVAL;
  const int64_t* f = &in->scenarios;  // the leading CCKA_TOTALS_INT64 int64 fields
  static_assert(offsetof(ccka_totals, gco2_ug) == (CCKA_TOTALS_INT64 - 1) * sizeof(int64_t), "int64 block");
  const int64_t lim = INT64_MAX / nranks;
  int64_t risk = 0;
  for (int k = 0; k < CCKA_TOTALS_INT64; ++k) {
    block[k] = f[k];
    risk |= (f[k] > lim || f[k] < -lim) ? 1 : 0;
  }
  block[CCKA_TOTALS_INT64] = risk;
  return CCKA_OK;
}

int ccka_totals_finish(const int64_t* block, int32_t n, ccka_totals* out) {
  if (!block || !out || n != CCKA_TOTALS_BLOCK) return CCKA_EINVAL;
  if (block[CCKA_TOTALS_INT64] != 0) return CCKA_EOVERFLOW;
  int64_t* f = &out->scenarios;
  for (int k = 0; k < CCKA_TOTALS_INT64; ++k) f[k] = block[k];
  out->energy_wmin = (double)out->energy_uwmin * 1e-6;
  out->gco2 = (double)out->gco2_ug * 1e-6;
  return CCKA_OK;
}

int ccka_comm_unique_id(uint8_t* id128) {
  if (!id128) return CCKA_EINVAL;
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return CCKA_ERCCL;
  static_assert(sizeof(ncclUniqueId) == 128, "RCCL unique id size");
  std::memcpy(id128, &id, 128);
  return CCKA_OK;
}

int ccka_comm_init(ccka_ctx* c, const uint8_t* id128, int32_t nranks, int32_t rank) {
  if (!c || !id128 || nranks < 1 || rank < 0 || rank >= nranks) return CCKA_EINVAL;
  (void)hipSetDevice(c->device);
  ncclUniqueId id;
  std::memcpy(&id, id128, 128);
  if (c->comm) { ncclCommDestroy(c->comm); c->comm = nullptr; }
  const ncclResult_t r = ncclCommInitRank(&c->comm, nranks, id, rank);
  if (r != ncclSuccess) return fail(c, CCKA_ERCCL, "ncclCommInitRank: %s", ncclGetErrorString(r));
  return CCKA_OK;
}

int ccka_allreduce_totals(ccka_ctx* c, ccka_totals* io) {
  if (!c || !io) return CCKA_EINVAL;
  if (!c->comm) return fail(c, CCKA_ESTATE, "ccka_comm_init first");
  (void)hipSetDevice(c->device);
  int nranks = 1;
  if (ncclCommCount(c->comm, &nranks) != ncclSuccess) return fail(c, CCKA_ERCCL, "ncclCommCount failed");
  int64_t block[CCKA_TOTALS_BLOCK];
  if (ccka_totals_pack(io, nranks, block, CCKA_TOTALS_BLOCK) != CCKA_OK) return fail(c, CCKA_EINVAL, "totals pack");
  // the block goes through the device totals buffer (96 B >= 88 B)
  static_assert(sizeof(ccka_totals) >= CCKA_TOTALS_BLOCK * sizeof(int64_t), "totals block fits");
  if (!c->d_totals && hipMalloc((void**)&c->d_totals, sizeof(ccka_totals)) != hipSuccess)
    return fail(c, CCKA_ENOMEM, "totals alloc");
  int64_t* d_block = (int64_t*)c->d_totals;
  HIPCHK(c, hipMemcpyAsync(d_block, block, sizeof block, hipMemcpyHostToDevice, c->stream));
  // one in-place all-reduce (exact, order-independent); the doubles are
  // re-derived from the sums, so every rank count gives the same bits
  const ncclResult_t r = ncclAllReduce(d_block, d_block, CCKA_TOTALS_BLOCK, ncclInt64, ncclSum, c->comm, c->stream);
  if (r != ncclSuccess) return fail(c, CCKA_ERCCL, "ncclAllReduce: %s", ncclGetErrorString(r));
  HIPCHK(c, hipMemcpyAsync(block, d_block, sizeof block, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  const int st = ccka_totals_finish(block, CCKA_TOTALS_BLOCK, io);
  if (st != CCKA_OK) return fail(c, st, "a summed total exceeds int64 at %d ranks (ccka.h: ccka_totals)", nranks);
  return CCKA_OK;
}

int ccka_comm_info(ccka_ctx* c, int32_t* nranks, int32_t* rank) {
  if (!c) return CCKA_EINVAL;
  if (!c->comm) return fail(c, CCKA_ESTATE, "ccka_comm_init first");
  int n = 0, r = 0;
  if (ncclCommCount(c->comm, &n) != ncclSuccess || ncclCommUserRank(c->comm, &r) != ncclSuccess)
    return fail(c, CCKA_ERCCL, "ncclCommCount / ncclCommUserRank failed");
  if (nranks) *nranks = n;
  if (rank) *rank = r;
  return CCKA_OK;
}

// ---------------------------------------------------------------------------
// Policy sweep (BASELINE config 4)
// ---------------------------------------------------------------------------
static int sweep_grids(ccka_ctx* c, int64_t grid_size, int64_t* n_grids) {
  if (!c->ran) return fail(c, CCKA_ESTATE, "no rollout yet");
  if (grid_size < 1 || c->N % grid_size || c->first_id % grid_size)
    return fail(c, CCKA_EINVAL, "batch (first_id %lld, n %lld) does not hold whole grids of %lld",
                (long long)c->first_id, (long long)c->N, (long long)grid_size);
  const int64_t ng = c->N / grid_size;
  if (ng > (1 << 24)) return fail(c, CCKA_EINVAL, "too many grids");
  if (c->gcap < ng) {
    dfree(c->d_gstats);
    if (hipMalloc((void**)&c->d_gstats, sizeof(ccka_grid_stats) * ng) != hipSuccess)
      return fail(c, CCKA_ENOMEM, "grid buffers");
    c->gcap = ng;
  }
  GridSrc g{};
  g.cost = c->kp.cost; g.gco2 = c->kp.gco2; g.slo = c->kp.slo; g.energy = c->kp.energy;
  g.grid_size = grid_size;
  g.first_grid = c->first_id / grid_size;
  g.n_grids = ng;
  HIPCHK(c, launch_grid_stats(g, c->d_gstats, c->stream));
  *n_grids = ng;
  return CCKA_OK;
}

int ccka_get_grid_stats(ccka_ctx* c, int64_t grid_size, ccka_grid_stats* out, int64_t n_grids) {
  if (!c || !out) return CCKA_EINVAL;
  (void)hipSetDevice(c->device);
  int64_t ng = 0;
  int rc;
  if ((rc = sweep_grids(c, grid_size, &ng)) != CCKA_OK) return rc;
  if (n_grids != ng) return fail(c, CCKA_EINVAL, "n_grids %lld != %lld", (long long)n_grids, (long long)ng);
  HIPCHK(c, hipMemcpyAsync(out, c->d_gstats, sizeof(ccka_grid_stats) * ng, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return CCKA_OK;
}

// Pareto buffers for `ng` local grids and `nranks` ranks: the local candidates
// (ng), the all-gathered candidate rows [nranks][ng] followed by their union
// (nranks * ng), the final frontier and the dominance flags (nranks * ng each:
// the global frontier can hold every rank's candidates), the per-rank counts
// (+ the local one) and two device-side sizes.
static int pareto_bufs(ccka_ctx* c, int64_t ng, int nranks) {
  const int64_t tot = ng * nranks;
  if (c->pcap_ng < ng || c->pcap_ranks < nranks) {
    dfree(c->d_gcand); dfree(c->d_gflags); dfree(c->d_gn); dfree(c->d_ggather); dfree(c->d_gcounts);
    dfree(c->d_gfront);
    if (hipMalloc((void**)&c->d_gcand, sizeof(ccka_grid_stats) * ng) != hipSuccess ||
        hipMalloc((void**)&c->d_gfront, sizeof(ccka_grid_stats) * tot) != hipSuccess ||
        hipMalloc((void**)&c->d_gflags, (size_t)tot) != hipSuccess ||
        hipMalloc((void**)&c->d_gn, 2 * sizeof(int32_t)) != hipSuccess ||
        hipMalloc((void**)&c->d_ggather, sizeof(ccka_grid_stats) * tot * 2) != hipSuccess ||
        hipMalloc((void**)&c->d_gcounts, sizeof(int64_t) * (nranks + 1)) != hipSuccess) {
      c->pcap_ng = c->pcap_ranks = 0;
      return fail(c, CCKA_ENOMEM, "pareto buffers (%lld grids x %d ranks)", (long long)ng, nranks);
    }
    c->pcap_ng = ng;
    c->pcap_ranks = nranks;
  }
  return CCKA_OK;
}

// Global filter over the exchanged candidates, identical on every rank: the
// valid prefixes of gathered[nranks][ng] (counts[q] each, rank order = grid
// order) are compacted, then filtered again into d_gfront / d_gn[0].
static int pareto_merge(ccka_ctx* c, int64_t ng, int nranks) {
  ccka_grid_stats* uni = c->d_ggather + ng * nranks;
  HIPCHK(c, launch_pareto_union(c->d_ggather, c->d_gcounts, nranks, (int)ng, uni, c->d_gn + 1, c->stream));
  HIPCHK(c, launch_pareto(uni, (int)(ng * nranks), c->d_gn + 1, c->d_gflags, c->d_gfront, c->d_gn, c->stream));
  return CCKA_OK;
}

static int pareto_copy_out(ccka_ctx* c, ccka_grid_stats* out, int32_t capacity, int32_t* n_out) {
  int32_t n = 0;
  HIPCHK(c, hipMemcpyAsync(&n, c->d_gn, sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  *n_out = n;
  if (n > capacity) return fail(c, CCKA_EINVAL, "frontier has %d grids, capacity %d", n, capacity);
  if (n > 0) {
    HIPCHK(c, hipMemcpyAsync(out, c->d_gfront, sizeof(ccka_grid_stats) * n, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
  }
  return CCKA_OK;
}

int ccka_pareto_frontier(ccka_ctx* c, int64_t grid_size, ccka_grid_stats* out, int32_t capacity, int32_t* n_out) {
  if (!c || !n_out || capacity < 0 || (capacity > 0 && !out)) return CCKA_EINVAL;
  (void)hipSetDevice(c->device);
  int64_t ng = 0;
  int rc;
  if ((rc = sweep_grids(c, grid_size, &ng)) != CCKA_OK) return rc;
  int nranks = 1;
  if (c->comm && ncclCommCount(c->comm, &nranks) != ncclSuccess)
    return fail(c, CCKA_ERCCL, "ncclCommCount failed");
  if ((rc = pareto_bufs(c, ng, nranks)) != CCKA_OK) return rc;
  if (!c->comm) {
    // local frontier only: non-dominated grids of this batch, in grid order
    HIPCHK(c, launch_pareto(c->d_gstats, (int)ng, nullptr, c->d_gflags, c->d_gfront, c->d_gn, c->stream));
    return pareto_copy_out(c, out, capacity, n_out);
  }
  // local candidates, then the exchange: every rank's candidates (fixed
  // capacity = grids per rank, every rank holds the same number) and counts
  HIPCHK(c, launch_pareto(c->d_gstats, (int)ng, nullptr, c->d_gflags, c->d_gcand, c->d_gn, c->stream));
  int64_t* cnt_local = c->d_gcounts + nranks;
  // int32 count -> int64 slot (device copy keeps the exchange on the stream)
  HIPCHK(c, hipMemsetAsync(cnt_local, 0, sizeof(int64_t), c->stream));
  HIPCHK(c, hipMemcpyAsync(cnt_local, c->d_gn, sizeof(int32_t), hipMemcpyDeviceToDevice, c->stream));
  ncclGroupStart();
  ncclResult_t r1 = ncclAllGather(cnt_local, c->d_gcounts, 1, ncclInt64, c->comm, c->stream);
  ncclResult_t r2 = ncclAllGather(c->d_gcand, c->d_ggather, (size_t)ng * sizeof(ccka_grid_stats), ncclUint8,
                                  c->comm, c->stream);
  ncclResult_t r3 = ncclGroupEnd();
  if (r1 != ncclSuccess || r2 != ncclSuccess || r3 != ncclSuccess)
    return fail(c, CCKA_ERCCL, "ncclAllGather (pareto candidates) failed");
  if ((rc = pareto_merge(c, ng, nranks)) != CCKA_OK) return rc;
  return pareto_copy_out(c, out, capacity, n_out);
}

// ---------------------------------------------------------------------------
// Learned MLP policy (BASELINE config 5)
// ---------------------------------------------------------------------------
// MFMA fragment order of the weights (see mlp.hip). Lane l: r = l & 31, h = l >> 5.
// Layer 1 A operand (natural k): element j = W1[16s + 8h + j][32n + r].
// Layers 2/3 A operand, k-step kk, in the k order of the chained accumulator:
// element j <-> input unit 32(kk>>1) + 16(kk&1) + 8(j>>2) + 4h + (j&3).
static int kin(int kk, int j, int h) { return 32 * (kk >> 1) + 16 * (kk & 1) + 8 * (j >> 2) + 4 * h + (j & 3); }
// 16x16x32 (mlp16_kernel), lane l: i = l & 15 (output row of the tile), g = l >> 4.
// Layer 1 A operand (natural k): element e = W1[32s + 8g + e][16o + i].
// Layers 2/3, k-step s, chained order: element e <-> input unit 32s + 16(e>>2) + 4g + (e&3).
static int kin16(int s, int e, int g) { return 32 * s + 16 * (e >> 2) + 4 * g + (e & 3); }

int ccka_mlp_set_weights(ccka_ctx* c, int32_t in_dim, int32_t hidden, int32_t out_dim, const uint16_t* w1,
                         const float* b1, const uint16_t* w2, const float* b2, const uint16_t* w3, const float* b3) {
  if (!c || !w1 || !b1 || !w2 || !b2 || !w3 || !b3) return CCKA_EINVAL;
  if (in_dim != MLP_IN || hidden != MLP_HID || out_dim != MLP_OUT)
    return fail(c, CCKA_EINVAL, "MLP shape %dx%dx%d unsupported (64 -> 256 -> 256 -> 8)", in_dim, hidden, out_dim);
  (void)hipSetDevice(c->device);
  std::vector<uint16_t> f1((size_t)8 * 4 * 64 * 8), f2((size_t)8 * 16 * 64 * 8), f3((size_t)16 * 64 * 8, 0);
  for (int n = 0; n < 8; ++n)
    for (int st = 0; st < 4; ++st)
      for (int l = 0; l < 64; ++l)
        for (int j = 0; j < 8; ++j) {
          const int r = l & 31, h = l >> 5;
          f1[(((size_t)n * 4 + st) * 64 + l) * 8 + j] = w1[(size_t)(16 * st + 8 * h + j) * MLP_HID + 32 * n + r];
        }
  for (int n = 0; n < 8; ++n)
    for (int kk = 0; kk < 16; ++kk)
      for (int l = 0; l < 64; ++l)
        for (int j = 0; j < 8; ++j) {
          const int r = l & 31, h = l >> 5;
          f2[(((size_t)n * 16 + kk) * 64 + l) * 8 + j] = w2[(size_t)kin(kk, j, h) * MLP_HID + 32 * n + r];
        }
  for (int kk = 0; kk < 16; ++kk)
    for (int l = 0; l < 64; ++l)
      for (int j = 0; j < 8; ++j) {
        const int r = l & 31, h = l >> 5;
        if (r < MLP_OUT) f3[((size_t)kk * 64 + l) * 8 + j] = w3[(size_t)kin(kk, j, h) * MLP_OUT + r];
      }
  // backward (pg.hip): dH1^T = W2 dH2^T with dH2^T chained in the same permuted
  // k order (rows = H1 units), dH2^T = W3 g_y^T with k = action padded to 16
  std::vector<uint16_t> f2b((size_t)8 * 16 * 64 * 8), f3b((size_t)8 * 64 * 8, 0);
  for (int n = 0; n < 8; ++n)
    for (int kk = 0; kk < 16; ++kk)
      for (int l = 0; l < 64; ++l)
        for (int j = 0; j < 8; ++j) {
          const int r = l & 31, h = l >> 5;
          f2b[(((size_t)n * 16 + kk) * 64 + l) * 8 + j] = w2[(size_t)(32 * n + r) * MLP_HID + kin(kk, j, h)];
        }
  for (int n = 0; n < 8; ++n)
    for (int l = 0; l < 64; ++l)
      for (int j = 0; j < 8; ++j) {
        const int r = l & 31, h = l >> 5;
        if (h == 0) f3b[((size_t)n * 64 + l) * 8 + j] = w3[(size_t)(32 * n + r) * MLP_OUT + j];
      }
  std::vector<uint16_t> g1((size_t)16 * 2 * 64 * 8), g2((size_t)16 * 8 * 64 * 8), g3((size_t)8 * 64 * 8, 0);
  for (int o = 0; o < 16; ++o)
    for (int st = 0; st < 2; ++st)
      for (int l = 0; l < 64; ++l)
        for (int e = 0; e < 8; ++e) {
          const int i = l & 15, g = l >> 4;
          g1[(((size_t)o * 2 + st) * 64 + l) * 8 + e] = w1[(size_t)(32 * st + 8 * g + e) * MLP_HID + 16 * o + i];
        }
  for (int o = 0; o < 16; ++o)
    for (int st = 0; st < 8; ++st)
      for (int l = 0; l < 64; ++l)
        for (int e = 0; e < 8; ++e) {
          const int i = l & 15, g = l >> 4;
          g2[(((size_t)o * 8 + st) * 64 + l) * 8 + e] = w2[(size_t)kin16(st, e, g) * MLP_HID + 16 * o + i];
        }
  for (int st = 0; st < 8; ++st)
    for (int l = 0; l < 64; ++l)
      for (int e = 0; e < 8; ++e) {
        const int i = l & 15, g = l >> 4;
        if (i < MLP_OUT) g3[((size_t)st * 64 + l) * 8 + e] = w3[(size_t)kin16(st, e, g) * MLP_OUT + i];
      }
  std::vector<float> bias(MLP_HID * 2 + 32);  // b3 zero-padded to one 32-row tile
  std::memcpy(bias.data(), b1, MLP_HID * 4);
  std::memcpy(bias.data() + MLP_HID, b2, MLP_HID * 4);
  std::memcpy(bias.data() + 2 * MLP_HID, b3, MLP_OUT * 4);
  int rc;
  if ((rc = dupload(c, c->d_w1f, (const mlp_bf16x8*)f1.data(), f1.size() / 8)) != CCKA_OK) return rc;
  if ((rc = dupload(c, c->d_w2f, (const mlp_bf16x8*)f2.data(), f2.size() / 8)) != CCKA_OK) return rc;
  if ((rc = dupload(c, c->d_w3f, (const mlp_bf16x8*)f3.data(), f3.size() / 8)) != CCKA_OK) return rc;
  if ((rc = dupload(c, c->d_mb, bias.data(), bias.size())) != CCKA_OK) return rc;
  if ((rc = dupload(c, c->d_w2b, (const mlp_bf16x8*)f2b.data(), f2b.size() / 8)) != CCKA_OK) return rc;
  if ((rc = dupload(c, c->d_w3b, (const mlp_bf16x8*)f3b.data(), f3b.size() / 8)) != CCKA_OK) return rc;
  if ((rc = dupload(c, c->d_w1g, (const mlp_bf16x8*)g1.data(), g1.size() / 8)) != CCKA_OK) return rc;
  if ((rc = dupload(c, c->d_w2g, (const mlp_bf16x8*)g2.data(), g2.size() / 8)) != CCKA_OK) return rc;
  if ((rc = dupload(c, c->d_w3g, (const mlp_bf16x8*)g3.data(), g3.size() / 8)) != CCKA_OK) return rc;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->mlp_have_w = true;
  return CCKA_OK;
}

static int mlp_alloc(ccka_ctx* c, int64_t n) {
  if (n < 1 || n > ((int64_t)1 << 34)) return fail(c, CCKA_EINVAL, "state count out of range");
  if (c->mlp_cap < n) {
    dfree(c->d_mx);
    dfree(c->d_my);
    c->mlp_cap = 0;
    c->mlp_n = 0;
    if (hipMalloc((void**)&c->d_mx, (size_t)n * MLP_IN * 2) != hipSuccess ||
        hipMalloc((void**)&c->d_my, (size_t)n * MLP_OUT * 4) != hipSuccess)
      return fail(c, CCKA_ENOMEM, "MLP state/action buffers (%lld states)", (long long)n);
    c->mlp_cap = n;
  }
  c->mlp_n = n;
  return CCKA_OK;
}

int ccka_mlp_set_states(ccka_ctx* c, const uint16_t* x, int64_t n) {
  if (!c || !x) return CCKA_EINVAL;
  (void)hipSetDevice(c->device);
  int rc;
  if ((rc = mlp_alloc(c, n)) != CCKA_OK) return rc;
  HIPCHK(c, hipMemcpyAsync(c->d_mx, x, (size_t)n * MLP_IN * 2, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return CCKA_OK;
}

int ccka_mlp_gen_states(ccka_ctx* c, int64_t n, uint64_t seed) {
  if (!c) return CCKA_EINVAL;
  (void)hipSetDevice(c->device);
  int rc;
  if ((rc = mlp_alloc(c, n)) != CCKA_OK) return rc;
  HIPCHK(c, launch_mlp_gen_states(c->d_mx, n * MLP_IN, seed, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return CCKA_OK;
}

int ccka_mlp_forward_async(ccka_ctx* c) {
  if (!c) return CCKA_EINVAL;
  if (!c->mlp_have_w || !c->mlp_n) return fail(c, CCKA_ESTATE, "MLP weights / states not set");
  (void)hipSetDevice(c->device);
  MlpParams p{};
  p.x = c->d_mx;
  p.y = c->d_my;
  p.w1f = c->d_w1f;
  p.w2f = c->d_w2f;
  p.w3f = c->d_w3f;
  p.b1 = c->d_mb;
  p.b2 = c->d_mb + MLP_HID;
  p.b3 = c->d_mb + 2 * MLP_HID;
  p.N = c->mlp_n;
  p.stamps = nullptr;
  if (c->mlp_tile == 16) {
    p.w1g = c->d_w1g;
    p.w2g = c->d_w2g;
    p.w3g = c->d_w3g;
  }
  if (c->mlp_stamps) {
    if (!c->d_stamps && hipMalloc((void**)&c->d_stamps, 12 * sizeof(unsigned long long)) != hipSuccess)
      return fail(c, CCKA_ENOMEM, "stamps alloc");
    HIPCHK(c, hipMemsetAsync(c->d_stamps, 0, 12 * sizeof(unsigned long long), c->stream));
    p.stamps = c->d_stamps;
  }
  HIPCHK(c, hipEventRecord(c->ev0, c->stream));
  HIPCHK(c, hipEventRecord(c->ev_mid, c->stream));
  HIPCHK(c, launch_mlp(p, c->cus, c->stream));
  HIPCHK(c, hipEventRecord(c->ev1, c->stream));
  c->ran = true;
  return CCKA_OK;
}

// Internal measurement hook (bench.py config 5): `launches` back-to-back MLP
// launches with an event pair around each one; *avg_ms = the mean kernel
// duration (what rocprofv3 --kernel-trace averages), *span_ms = first start
// to last end (launch gaps included).
int ccka_debug_mlp_batch(ccka_ctx* c, int32_t launches, double* avg_ms, double* span_ms) {
  if (!c || !avg_ms || !span_ms || launches < 1 || launches > 4096) return CCKA_EINVAL;
  if (!c->mlp_have_w || !c->mlp_n) return fail(c, CCKA_ESTATE, "MLP weights / states not set");
  (void)hipSetDevice(c->device);
  std::vector<hipEvent_t> ev((size_t)launches * 2);
  for (auto& e : ev) HIPCHK(c, hipEventCreate(&e));
  MlpParams p{};
  p.x = c->d_mx;
  p.y = c->d_my;
  p.w1f = c->d_w1f;
  p.w2f = c->d_w2f;
  p.w3f = c->d_w3f;
  p.b1 = c->d_mb;
  p.b2 = c->d_mb + MLP_HID;
  p.b3 = c->d_mb + 2 * MLP_HID;
  p.N = c->mlp_n;
  p.stamps = nullptr;
  if (c->mlp_tile == 16) {
    p.w1g = c->d_w1g;
    p.w2g = c->d_w2g;
    p.w3g = c->d_w3g;
  }
  int rc = CCKA_OK;
  // the context's own pair spans the batch (ccka_sync / ccka_last_kernel_ms)
  HIPCHK(c, hipEventRecord(c->ev0, c->stream));
  HIPCHK(c, hipEventRecord(c->ev_mid, c->stream));
  for (int k = 0; k < launches && rc == CCKA_OK; ++k) {
    if (hipEventRecord(ev[2 * k], c->stream) != hipSuccess || launch_mlp(p, c->cus, c->stream) != hipSuccess ||
        hipEventRecord(ev[2 * k + 1], c->stream) != hipSuccess)
      rc = fail(c, CCKA_EHIP, "MLP batch launch %d", k);
  }
  double sum = 0.0;
  float span = 0.f;
  if (rc == CCKA_OK && hipEventRecord(c->ev1, c->stream) != hipSuccess) rc = fail(c, CCKA_EHIP, "event record");
  if (rc == CCKA_OK && hipStreamSynchronize(c->stream) != hipSuccess) rc = fail(c, CCKA_EHIP, "MLP batch sync");
  for (int k = 0; k < launches && rc == CCKA_OK; ++k) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, ev[2 * k], ev[2 * k + 1]) != hipSuccess) rc = fail(c, CCKA_EHIP, "event time");
    sum += ms;
  }
  if (rc == CCKA_OK && hipEventElapsedTime(&span, ev[0], ev[2 * launches - 1]) != hipSuccess)
    rc = fail(c, CCKA_EHIP, "event time");
  for (auto& e : ev) (void)hipEventDestroy(e);
  if (rc != CCKA_OK) return rc;
  *avg_ms = sum / launches;
  *span_ms = span;
  c->ran = true;
  return CCKA_OK;
}

int ccka_mlp_forward(ccka_ctx* c) {
  int rc = ccka_mlp_forward_async(c);
  if (rc != CCKA_OK) return rc;
  return ccka_sync(c);
}

int ccka_mlp_get_actions(ccka_ctx* c, float* y, int64_t n) {
  if (!c || !y) return CCKA_EINVAL;
  if (n != c->mlp_n) return fail(c, CCKA_EINVAL, "action count mismatch");
  (void)hipSetDevice(c->device);
  HIPCHK(c, hipMemcpyAsync(y, c->d_my, (size_t)n * MLP_OUT * 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return CCKA_OK;
}

// Internal profiling hook (not part of include/ccka.h): phase-ablation mask
// for timing attribution only; results of an ablated run are meaningless.
// Internal: the device copy ceiling, GB/s of read + write of a `bytes`-byte
// dwordx4 streaming copy (launch_copy16), the median of `reps` launches timed
// with HIP events on the engine's stream after one warm-up launch.
int ccka_debug_copy_gbs(ccka_ctx* c, int64_t bytes, int32_t reps, double* gbs) {
  if (!c || !gbs || bytes < (1 << 20) || reps < 1 || reps > 64) return CCKA_EINVAL;
  (void)hipSetDevice(c->device);
  bytes &= ~(int64_t)4095;
  void *a = nullptr, *b = nullptr;
  if (hipMalloc(&a, (size_t)bytes) != hipSuccess || hipMalloc(&b, (size_t)bytes) != hipSuccess) {
    if (a) (void)hipFree(a);
    return fail(c, CCKA_ENOMEM, "copy probe alloc (2 x %lld bytes)", (long long)bytes);
  }
  int rc = CCKA_OK;
  std::vector<float> ms((size_t)reps);
  hipEvent_t e0 = nullptr, e1 = nullptr;  // own events: ccka_last_kernel_ms keeps the rollout's
  if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess)
    rc = fail(c, CCKA_EHIP, "copy probe events");
  if (rc == CCKA_OK && (hipMemsetAsync(a, 1, (size_t)bytes, c->stream) != hipSuccess ||
      launch_copy16(a, b, bytes, c->cus, c->stream) != hipSuccess))
    rc = fail(c, CCKA_EHIP, "copy probe warm-up");
  for (int k = 0; k < reps && rc == CCKA_OK; ++k) {
    if (hipEventRecord(e0, c->stream) != hipSuccess || launch_copy16(a, b, bytes, c->cus, c->stream) != hipSuccess ||
        hipEventRecord(e1, c->stream) != hipSuccess || hipEventSynchronize(e1) != hipSuccess ||
        hipEventElapsedTime(&ms[(size_t)k], e0, e1) != hipSuccess)
      rc = fail(c, CCKA_EHIP, "copy probe launch %d", k);
  }
  (void)hipStreamSynchronize(c->stream);
  if (e0) (void)hipEventDestroy(e0);
  if (e1) (void)hipEventDestroy(e1);
  (void)hipFree(a);
  (void)hipFree(b);
  if (rc != CCKA_OK) return rc;
  std::sort(ms.begin(), ms.end());
  *gbs = 2.0 * (double)bytes / ((double)ms[(size_t)reps / 2] * 1e-3) / 1e9;
  return CCKA_OK;
}

int ccka_debug_ablate(ccka_ctx* c, int32_t mask) {
  if (!c) return CCKA_EINVAL;
  c->kp.ablate = mask;
  return CCKA_OK;
}

// Internal (not in include/ccka.h): 0 = choose the engine automatically,
// 1 = always the general kernel (tests compare both engines), 2 = the general
// kernel in lockstep (no lane-skewed schedule for several deployments), 3 =
// automatic with the skewed schedule's provisioning on the wave-cooperative scans.
int ccka_debug_engine(ccka_ctx* c, int32_t mode) {
  if (!c || mode < 0 || mode > 3) return CCKA_EINVAL;
  // 3: automatic, with the skewed schedule's wave-cooperative provisioning (A/B of the lane-local one)
  c->sk_coop_f2 = mode == 3;
  c->engine_mode = mode == 3 ? 0 : mode;
  return CCKA_OK;
}

// Internal: which engine ran last (1 general, 2 single-deployment, 3 the
// launched closed loop, 4 the fused closed loop, 5 the general kernel on the
// lane-skewed schedule) and the
// duration of its argmin-table kernel.
int ccka_debug_last_engine(ccka_ctx* c, int32_t* engine, double* table_ms) {
  if (!c) return CCKA_EINVAL;
  if (engine) *engine = c->last_engine;
  if (table_ms) *table_ms = c->last_table_ms;
  return CCKA_OK;
}

// Internal: scenarios per wave of the single-deployment kernel (1..64; 0 = automatic).
// Internal: 0 = enqueue the closed loop's launches directly instead of
// replaying its captured hipGraph (1, the default)
// Internal: rows per policy-gradient backward chunk (multiple of 32; 0 = the
// default 2^23), to exercise the chunked sum at test sizes.
int ccka_debug_pg_chunk(ccka_ctx* c, int64_t rows) {
  if (!c || rows < 0 || rows % 32) return CCKA_EINVAL;
  c->pg_chunk = rows;
  return CCKA_OK;
}

// Internal: 0 = the fused loop scans the catalog for its launches (A/B of the
// argmin tables; same results).
int ccka_debug_policy_table(ccka_ctx* c, int32_t on) {
  if (!c) return CCKA_EINVAL;
  c->pol_table_off = on == 0;
  return CCKA_OK;
}

int ccka_debug_policy_fused(ccka_ctx* c, int32_t on) {
  if (!c) return CCKA_EINVAL;
  c->pol_fused_off = on == 0;
  return CCKA_OK;
}

int ccka_debug_policy_graph(ccka_ctx* c, int32_t on) {
  if (!c) return CCKA_EINVAL;
  c->pol_graph_off = on == 0;
  return CCKA_OK;
}

int ccka_debug_lpw(ccka_ctx* c, int32_t lpw) {
  if (!c || lpw < 0 || lpw > 64) return CCKA_EINVAL;
  c->lpw = lpw;
  return CCKA_OK;
}

// Internal: 1 = the single-deployment kernel reads the [T][N] trace instead of
// its wave-tiled copy (layout A/B; results are the same).
int ccka_debug_trace_flat(ccka_ctx* c, int32_t on) {
  if (!c) return CCKA_EINVAL;
  c->trace_flat = on != 0;
  return CCKA_OK;
}

// Internal: pooled event steps of the single-deployment engine (mode 1; 0 =
// rollout_d1_kernel everywhere, the default: DESIGN.md "Pooled event steps,
// built and measured") and the queue length at which a
// wave serves the queue (1..64; 0 = the default 48); `last` (nullable): whether
// the last single-deployment rollout ran the pooled kernel.
int ccka_debug_pool(ccka_ctx* c, int32_t mode, int32_t min_queue, int32_t* last) {
  if (!c || mode < -1 || mode > 1 || min_queue < 0 || min_queue > 64) return CCKA_EINVAL;
  if (mode >= 0) c->pool_mode = mode;
  if (min_queue > 0) c->pool_min = min_queue;
  if (last) *last = c->last_pooled ? 1 : 0;
  return CCKA_OK;
}

// Internal: the other serving rules of the pooled kernel (age in s_memtime
// cycles since the last claim, >= 0; idle: serve when no own lane can step).
int ccka_debug_pool_policy(ccka_ctx* c, int32_t age, int32_t idle) {
  if (!c || age < 0 || idle < 0 || idle > 1) return CCKA_EINVAL;
  c->pool_age = age;
  c->pool_idle = idle;
  return CCKA_OK;
}

// Internal: occupancy target of the single-deployment kernel (2, 3; 0 = automatic).
int ccka_debug_occ(ccka_ctx* c, int32_t occ) {
  if (!c || occ < 0 || occ > 3 || occ == 1) return CCKA_EINVAL;
  c->occ = occ;
  return CCKA_OK;
}

// Internal: per-phase cycle totals of the last stamped rollout (ablate bit 16).
// Internal: diagnostic phase stamps of the MLP kernel (read with ccka_debug_stamps).
// Internal: the standalone forward's MFMA tile (16: mlp16_kernel, 32: mlp_kernel).
int ccka_debug_mlp_tile(ccka_ctx* c, int32_t tile) {
  if (!c || (tile != 16 && tile != 32)) return CCKA_EINVAL;
  c->mlp_tile = tile;
  return CCKA_OK;
}

int ccka_debug_mlp_stamps(ccka_ctx* c, int32_t enable) {
  if (!c) return CCKA_EINVAL;
  c->mlp_stamps = enable != 0;
  return CCKA_OK;
}

int ccka_debug_stamps(ccka_ctx* c, unsigned long long* out8) {
  if (!c || !out8 || !c->d_stamps) return CCKA_EINVAL;
  HIPCHK(c, hipMemcpy(out8, c->d_stamps, 12 * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  return CCKA_OK;
}

// Internal (not in include/ccka.h): the cross-rank half of
// ccka_pareto_frontier on caller-supplied exchange buffers, i.e. what every
// rank runs after the RCCL all-gather: `gathered` [nranks][cap] candidate rows
// (rank q's first counts[q] valid, each sorted by grid id, ranks in grid
// order), merged and filtered into the global frontier. Lets a single GPU
// exercise the multi-rank merge path.
int ccka_debug_pareto_merge(ccka_ctx* c, const ccka_grid_stats* gathered, const int64_t* counts, int32_t nranks,
                            int64_t cap, ccka_grid_stats* out, int32_t capacity, int32_t* n_out) {
  if (!c || !gathered || !counts || !n_out || nranks < 1 || cap < 1 || capacity < 0 || (capacity > 0 && !out))
    return CCKA_EINVAL;
  for (int q = 0; q < nranks; ++q)
    if (counts[q] < 0 || counts[q] > cap) return fail(c, CCKA_EINVAL, "count of rank %d out of range", q);
  (void)hipSetDevice(c->device);
  int rc;
  if ((rc = pareto_bufs(c, cap, nranks)) != CCKA_OK) return rc;
  HIPCHK(c, hipMemcpyAsync(c->d_ggather, gathered, sizeof(ccka_grid_stats) * cap * nranks, hipMemcpyHostToDevice,
                           c->stream));
  HIPCHK(c, hipMemcpyAsync(c->d_gcounts, counts, sizeof(int64_t) * nranks, hipMemcpyHostToDevice, c->stream));
  if ((rc = pareto_merge(c, cap, nranks)) != CCKA_OK) return rc;
  return pareto_copy_out(c, out, capacity, n_out);
}

int ccka_device_info(ccka_ctx* c, char* name, int32_t name_len, int32_t* cu_count) {
  if (!c) return CCKA_EINVAL;
  if (name && name_len > 0) std::snprintf(name, (size_t)name_len, "%s", c->name);
  if (cu_count) *cu_count = c->cus;
  return CCKA_OK;
}

}  // extern "C"
