/*
 * ccka.h — C ABI of the MI355X policy-rollout engine (libccka.so).
 *
 * Drop-in boundary for the reference's decision path. In the reference the
 * decision path is reached through Kubernetes objects: `kubectl patch
 * nodepool` merge patches on spec.disruption
 * (demo_20_offpeak_configure.sh:59-60, demo_21_peak_configure.sh:56-57,
 * demo_19_reset_policies.sh:68-75), RFC 6902 patches on
 * /spec/template/spec/requirements (demo_20_offpeak_configure.sh:64-81,96;
 * demo_21_peak_configure.sh:60-77,88) and `kubectl apply` of the burst
 * Deployments and PDB (demo_30_burst_configure.sh:78-143,
 * demo_10_setup_configure.sh:47-56), reconciled by upstream HPA/KEDA/Karpenter.
 * Here those objects are ingested by the host (ccka_host.h) into the POD
 * structs below and the decisions for millions of independent cluster
 * scenarios are evaluated on the GPU. Semantics: docs/SEMANTICS.md.
 *
 * Conventions: plain C, explicit widths, no allocation escapes the ABI.
 * The caller owns every host buffer; the library owns device buffers inside
 * the context. Calls are blocking (stream-synchronous at return) unless the
 * name ends in _async. One context per device and per host thread.
 * Return 0 on success or a negative ccka_status; message via ccka_last_error.
 */
#ifndef CCKA_H
#define CCKA_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CCKA_ABI_VERSION 5

#define CCKA_STEP_SECONDS 60
#define CCKA_MAX_TYPES 1024
#define CCKA_MAX_ZONES 4
#define CCKA_MAX_REGIONS 16
#define CCKA_MAX_POOLS 4
#define CCKA_MAX_DEPLOY 16
#define CCKA_MAX_NODES 16
#define CCKA_HIST 8              /* register history ring depth (decisions) of the fast paths */
#define CCKA_HPA_MAX_POLICIES 4   /* scaling policies per direction */
#define CCKA_HPA_MAX_WINDOW_S 3600 /* stabilizationWindowSeconds upper bound (autoscaling/v2) */
#define CCKA_HPA_MAX_PERIOD_S 1800 /* policy periodSeconds upper bound (autoscaling/v2) */
#define CCKA_HPA_HIST_MAX 360     /* decision history entries: 3600 s / the shortest sync (10 s) */
#define CCKA_HOURS 24

enum ccka_status {
  CCKA_OK = 0,
  CCKA_EINVAL = -1,   /* invalid argument / world fails validation */
  CCKA_ENOMEM = -2,   /* device or host allocation failed */
  CCKA_EHIP = -3,     /* HIP runtime error */
  CCKA_ERCCL = -4,    /* RCCL error */
  CCKA_EPARITY = -5,  /* self-check mismatch */
  CCKA_ESTATE = -6,   /* call order (e.g. rollout before set_world) */
  CCKA_ENODEV = -7,   /* no usable gfx950 device */
  CCKA_EOVERFLOW = -8 /* a fixed-point total would leave int64 (ccka_totals) */
};

/* capacity-type bits (karpenter.sh/capacity-type); offering index c: 0 spot, 1 on-demand */
enum { CCKA_CAP_SPOT = 1, CCKA_CAP_OD = 2 };
/* NodePool spec.disruption.consolidationPolicy */
enum { CCKA_POLICY_KEEP = 0, CCKA_WHEN_EMPTY = 1, CCKA_WHEN_EMPTY_OR_UNDERUTILIZED = 2 };
/* CCKA_SCALER_KEDA_TRIGGER: an extra trigger of the KEDA deployment that
 * precedes it (a chain KEDA, TRIGGER, TRIGGER...). It owns no pods; its load
 * column is that trigger's metric and keda_threshold / keda_activation its
 * targets (multi-trigger ScaledObject; SEMANTICS 3.C). */
/* ccka_world.disrupt_ext */
#define CCKA_DISRUPT_DRIFT 1    /* drift on a zone / capacity-type requirement change */
#define CCKA_DISRUPT_REPLACE 2  /* single-node replacement consolidation (on-demand ->
                                   strictly cheaper offering, pre-spun replacement) */
#define CCKA_DISRUPT_MULTI 4    /* multi-node consolidation: >= 2 nodes of a
                                   WhenEmptyOrUnderutilized pool leave together, with at
                                   most one cheaper replacement (SEMANTICS 3.G3) */
enum { CCKA_SCALER_STATIC = 0, CCKA_SCALER_HPA = 1, CCKA_SCALER_KEDA = 2, CCKA_SCALER_KEDA_TRIGGER = 3 };
enum { CCKA_PROFILE_RESET = 0, CCKA_PROFILE_OFFPEAK = 1, CCKA_PROFILE_PEAK = 2 };
/* HPA behavior */
enum { CCKA_SELECT_MAX = 0, CCKA_SELECT_MIN = 1, CCKA_SELECT_DISABLED = 2 };
enum { CCKA_HPA_PODS = 1, CCKA_HPA_PERCENT = 2 };

/* One EC2 instance type of the catalog (the ~800-entry catalog Karpenter's AWS
 * provider discovers at runtime, 05_karpenter.sh:64-75). The power model
 *  is precomputed by the host: energy is accounted in exact
 * integer nanowatt-minutes (docs/SEMANTICS.md §3.H). 48 bytes. */
typedef struct ccka_itype {
  int32_t vcpu;
  int32_t alloc_cpu_m;    /* allocatable millicores (after kube-reserved)      */
  int32_t alloc_mem_mi;   /* allocatable MiB                                   */
  int32_t max_pods;
  int64_t idle_nw;        /* llround(vcpu*Wmin*PUE * 1e9)                      */
  int64_t dyn_nw_per_m;   /* llround(vcpu*(Wmax-Wmin)*PUE * 1e9 / alloc_cpu_m) */
  double p_ref_w;         /* p_idle + 0.5*p_dyn in W (launch-score power)      */
  int32_t mem_mi;         /* memory capacity MiB (NodePool spec.limits.memory) */
  int32_t _pad;
} ccka_itype;

/* A NodePool patch profile (merge semantics: 0 / -1 = keep). */
typedef struct ccka_pool_patch {
  int32_t policy;               /* CCKA_POLICY_*                     */
  int32_t consolidate_after_s;  /* -1 keep                           */
  uint32_t zone_mask;           /* topology.kubernetes.io/zone In .. */
  uint32_t cap_mask;            /* karpenter.sh/capacity-type In ..  */
} ccka_pool_patch;

typedef struct ccka_pool {
  int32_t limit_cpu_m;          /* spec.limits.cpu in millicores, -1 none */
  int32_t budget_pct;           /* disruption budget nodes %, default 10  */
  ccka_pool_patch base;         /* the NodePool as created                */
  ccka_pool_patch profile[3];   /* RESET, OFFPEAK, PEAK                   */
  int32_t limit_mem_mi;         /* spec.limits.memory in MiB, -1 none     */
  int32_t _pad;
} ccka_pool;

typedef struct ccka_hpa_policy {
  int32_t type;       /* CCKA_HPA_PODS / CCKA_HPA_PERCENT */
  int32_t value;
  int32_t period_s;   /* 1..CCKA_HPA_MAX_PERIOD_S */
} ccka_hpa_policy;

typedef struct ccka_hpa_rules {
  int32_t select;       /* CCKA_SELECT_* */
  int32_t n_policies;   /* 0..CCKA_HPA_MAX_POLICIES */
  int32_t stab_window_s;/* 0..CCKA_HPA_MAX_WINDOW_S */
  int32_t _pad;
  ccka_hpa_policy policies[CCKA_HPA_MAX_POLICIES];
} ccka_hpa_rules;

typedef struct ccka_deployment {
  int32_t scaler;           /* CCKA_SCALER_* */
  int32_t replicas0;
  int32_t min_replicas;
  int32_t max_replicas;
  int32_t target_util_pct;  /* HPA averageUtilization */
  int32_t req_cpu_m;
  int32_t req_mem_mi;
  int32_t limit_cpu_m;
  uint32_t cap_sel;         /* nodeSelector capacity-type bits, 3 = none */
  int32_t pdb_member;       /* selected by the PDB */
  int32_t keda_cooldown_s;
  int32_t keda_min;
  int32_t keda_max;
  int32_t _pad;
  int64_t keda_threshold;   /* AverageValue target per replica (metric units) */
  int64_t keda_activation;  /* activationThreshold */
  double tolerance;         /* 0.1 */
  ccka_hpa_rules up;
  ccka_hpa_rules down;
} ccka_deployment;

/* Everything batch-uniform. Array pointers are HOST pointers. */
typedef struct ccka_world {
  int32_t n_steps;
  int32_t start_minute;
  int32_t provision_delay_steps;
  int32_t max_nodes;            /* Karpenter node slots per scenario (<= 16) */

  int32_t n_types;
  int32_t n_regions;
  int32_t n_zones;
  int32_t n_pools;
  const ccka_itype* types;      /* [n_types]                         */
  const double* ci_gpwh;        /* [n_regions][24]                   */
  const double* ci_gpwmin;      /* [n_regions][24]                   */
  const int32_t* price_uph;     /* [n_regions][24][n_types][n_zones][2] */

  ccka_pool pools[CCKA_MAX_POOLS];
  int32_t n_deploy;
  int32_t base_nodes;
  int32_t base_type;
  int32_t slo_util_pct;
  ccka_deployment deploy[CCKA_MAX_DEPLOY];

  double base_util;
  double carbon_weight;         /* $/kgCO2 (default; per-scenario override) */
  int32_t pdb_min_available_pct;/* -1 none */
  int32_t peak_start_min;
  int32_t peak_end_min;
  int32_t peak_switch;          /* 1: peak/off-peak switch on            */
  int32_t reset_ca_s;           /* consolidateAfter of the RESET profile */
  int32_t disrupt_ext;          /* CCKA_DISRUPT_* bits: Karpenter disruption
                                   beyond WhenEmpty / WhenEmptyOrUnderutilized
                                   deletes (SEMANTICS 3.G0, 3.G2) */
  int32_t hpa_sync_s;           /* HPA / KEDA decision period (kube-controller-manager
                                   --horizontal-pod-autoscaler-sync-period): 0 or 60 =
                                   one decision per 60-s step; 10, 15, 20, 30 = 60/s
                                   decisions per step on the step's metric sample
                                   (SEMANTICS 3.C) */
  int32_t _pad2;
} ccka_world;

/* Per-scenario parameters, SoA, host pointers. NULL ⇒ world default. */
typedef struct ccka_scenarios {
  int64_t n;
  int64_t first_id;             /* global id of element 0 (trace RNG key) */
  int64_t n_traces;             /* 0: one load trace per scenario ([T][D][n]);
                                   > 0: a shared trace set [T][D][n_traces], scenario
                                   with global id g reads trace g mod n_traces (policy
                                   sweeps: every parameter grid over the same traces) */
  const uint8_t* region;
  const int16_t* target_util_pct;
  const int16_t* max_replicas;
  const int16_t* down_stab_s;
  const int16_t* reset_ca_s;
  const uint8_t* peak_switch;
  const double* carbon_weight;
  const uint8_t* cap_sel;       /* nodeSelector override for every deployment */
} ccka_scenarios;

/* Per-scenario results, SoA, caller-owned host arrays (NULL ⇒ skipped). */
typedef struct ccka_results {
  int64_t* cost_uphmin;         /* µ$/h·min; dollars = v/6e7 */
  double* energy_wmin;          /* W·min; kWh = v/6e4        */
  double* gco2;
  int32_t* slo_minutes;
  int64_t* pending_pod_minutes;
  int32_t* node_min_spot;
  int32_t* node_min_od;
  int32_t* launches;
  int32_t* deletions;
  int32_t* peak_nodes;
  int32_t* final_replicas;
  int32_t* final_nodes;
  uint32_t* last_choice;
  uint32_t* choice_hash;
} ccka_results;

/* Per-scenario breakdown behind the demo_41 summary (ccka_set_detail): the
 * run's cost / energy / carbon / node-minutes per NodePool and for the base
 * managed node group (01_cluster.sh:24-30), and per Deployment the final
 * DESIRED (spec.replicas after the scaler) / READY (pods on ready nodes,
 * status.readyReplicas) / pending, the columns of demo_30_burst_observe.sh:10-11.
 * Pool p's sums cover the Karpenter nodes of that pool; totals = base + pools
 * (exact for the integer fields; gCO2 is charged per clock hour per group, as
 * the run total is, SEMANTICS 3.H). 392 bytes. */
typedef struct ccka_detail {
  int64_t pool_cost_uphmin[CCKA_MAX_POOLS];
  int64_t pool_energy_nwmin[CCKA_MAX_POOLS];  /* nanowatt-minutes, exact */
  double pool_gco2[CCKA_MAX_POOLS];
  int32_t pool_node_min_spot[CCKA_MAX_POOLS];
  int32_t pool_node_min_od[CCKA_MAX_POOLS];
  int32_t pool_final_nodes[CCKA_MAX_POOLS];
  int32_t pool_peak_nodes[CCKA_MAX_POOLS];
  int32_t pool_launches[CCKA_MAX_POOLS];
  int32_t desired[CCKA_MAX_DEPLOY];
  int32_t ready[CCKA_MAX_DEPLOY];
  int32_t pending[CCKA_MAX_DEPLOY];
  int64_t base_cost_uphmin;
  int64_t base_energy_nwmin;
  double base_gco2;
} ccka_detail;

/* Trajectory record, one per (step, scenario). 16 bytes. ccka_get_trajectory
 * returns them step-major [T][N]; on the device they stay in the layout the
 * engine wrote (ccka_trajectory_layout): the single-deployment engine and the
 * general engine's lane-skewed schedule (worlds of several HPA / static
 * deployments) write scenario-major [N][T] (each scenario's horizon
 * contiguous), the general engine in lockstep step-major [T][N]. */
enum { CCKA_TRAJ_TN = 0, CCKA_TRAJ_NT = 1 };
typedef struct ccka_traj_rec {
  int32_t replicas;
  int32_t pending;
  uint16_t nodes_spot;
  uint16_t nodes_od;
  uint16_t last_type;
  uint16_t flags;
} ccka_traj_rec;

/* Whole-batch totals (packed for one all-reduce). Every summed field is an
 * int64, so sums are exact and independent of the summation order, the device
 * tree and the rank count: energy and gCO2 are summed in fixed point, each
 * scenario's value rounded once (llrint: to nearest, ties to even). The two
 * doubles are derived from them after every sum (ccka_get_totals,
 * ccka_totals_finish), so they too are bit-identical at any rank count.
 * Units and headroom: energy in microwatt-minutes (a config-3 scenario, one
 * day on up to 8 nodes, is ~8.6e9 uW.min, so int64 holds ~1e9 such scenarios
 * summed over all ranks), gCO2 in micrograms (~5.7e7 ug per such scenario at
 * 400 g/kWh: ~1.6e11 scenarios). A sum that would leave int64 is reported as
 * CCKA_EOVERFLOW (ccka_get_totals, ccka_totals_finish,
 * ccka_allreduce_totals), never wrapped. */
typedef struct ccka_totals {
  int64_t scenarios;
  int64_t cost_uphmin;
  int64_t slo_minutes;
  int64_t pending_pod_minutes;
  int64_t node_min_spot;
  int64_t node_min_od;
  int64_t launches;
  int64_t deletions;
  int64_t energy_uwmin;         /* sum of llrint(energy_wmin[i] * 1e6): microwatt-minutes */
  int64_t gco2_ug;              /* sum of llrint(gco2[i] * 1e6): micrograms               */
  double energy_wmin;           /* energy_uwmin * 1e-6 */
  double gco2;                  /* gco2_ug * 1e-6      */
} ccka_totals;
#define CCKA_TOTALS_INT64 10    /* leading int64 fields of ccka_totals */
/* The exchanged block: the CCKA_TOTALS_INT64 fields plus one overflow guard
 * word (the count of ranks whose own values could make the sum leave int64). */
#define CCKA_TOTALS_BLOCK 11

/* Per-grid sums of a policy sweep (BASELINE config 4): grid g = the scenarios
 * with global ids [g*grid_size, (g+1)*grid_size). 48 bytes. */
typedef struct ccka_grid_stats {
  int64_t grid;
  int64_t scenarios;
  int64_t cost_uphmin;
  int64_t slo_minutes;
  double gco2;
  double energy_wmin;
} ccka_grid_stats;

/* Synthetic load-trace generator (docs/SEMANTICS.md §4). */
typedef struct ccka_trace_gen {
  uint64_t seed;
  int32_t base_lo, base_hi;       /* millicores */
  int32_t amp_lo_pm, amp_hi_pm;   /* diurnal amplitude, permille */
  int32_t noise_pm;               /* noise sigma, permille */
  int32_t burst_prob_pm;
  int32_t burst_mult_pm;
  int32_t burst_len;              /* steps */
} ccka_trace_gen;

typedef struct ccka_ctx ccka_ctx;

/* ---- lifetime -------------------------------------------------------- */
int32_t ccka_abi_version(void);
/* sizes of the ABI structs, for binding self-checks: fills out[0..n) in the
 * order itype, pool, deployment, world, scenarios, results, traj_rec, totals,
 * trace_gen, grid_stats, detail; returns the count written. */
int32_t ccka_struct_sizes(int64_t* out, int32_t n);
int ccka_open(ccka_ctx** out, int device_ordinal);
void ccka_close(ccka_ctx* ctx);
const char* ccka_last_error(const ccka_ctx* ctx);

/* ---- inputs ---------------------------------------------------------- */
/* Validate and upload the world (catalog, tiles, pools, deployments). */
int ccka_set_world(ccka_ctx* ctx, const ccka_world* world);
/* Upload per-scenario parameters (resets any previous batch). */
int ccka_set_scenarios(ccka_ctx* ctx, const ccka_scenarios* sc);
/* Upload host load traces, layout [T][D][N] int32. For a single-deployment
 * world with per-scenario traces the device also keeps a wave-tiled copy
 * (another T*N*4 bytes; the single-deployment kernel's read layout, built
 * by the first rollout after each new trace; without the memory for it that
 * kernel reads [T][N]). Worlds that run on the general kernel's lane-skewed
 * schedule keep a scenario-major copy [N][T][DP] instead (DP = 2/4/8/16 >=
 * the deployments; built the same way). ccka_policy_rollout and
 * ccka_policy_grad release both copies for their own arrays: the next rollout
 * rebuilds its copy (one transpose kernel, ~0.4 ms for 1e5 x 1440 x 1). */
int ccka_set_load(ccka_ctx* ctx, const int32_t* load, int64_t count);
/* Generate load traces on the device (same values as the host generator;
 * the same wave-tiled copy as ccka_set_load). */
int ccka_gen_load(ccka_ctx* ctx, const ccka_trace_gen* gen);
/* Copy the device-resident traces back ([T][D][N]). */
int ccka_get_load(ccka_ctx* ctx, int32_t* load, int64_t count);

/* ---- rollout --------------------------------------------------------- */
/* Run the whole horizon for every scenario. trajectory != 0 also writes one
 * trajectory record per (step, scenario) on the device, in the engine's own
 * layout (ccka_trajectory_layout: [N][T] from the single-deployment engine,
 * whose kernel time ccka_last_kernel_ms reports with those writes included;
 * [T][N] from the general engine). Results stay on the device until
 * ccka_get_results / ccka_get_trajectory / ccka_get_totals. */
int ccka_rollout(ccka_ctx* ctx, int32_t trajectory);
int ccka_rollout_async(ccka_ctx* ctx, int32_t trajectory);
int ccka_sync(ccka_ctx* ctx);
/* Duration of the last rollout kernel(s), from HIP events on the engine's
 * stream (milliseconds). */
int ccka_last_kernel_ms(ccka_ctx* ctx, double* ms);
int ccka_get_results(ccka_ctx* ctx, ccka_results* out);
/* The records in [T][N] order (count = T*N). From an [N][T] device layout the
 * engine transposes blocks of steps on the device through a bounded staging
 * buffer (max(N, 4 Mi) records) and copies each block into place. */
int ccka_get_trajectory(ccka_ctx* ctx, ccka_traj_rec* out, int64_t count);
/* Device layout of the last rollout's records (CCKA_TRAJ_TN / CCKA_TRAJ_NT). */
int ccka_trajectory_layout(ccka_ctx* ctx, int32_t* layout);
/* The records exactly as the device holds them (no transpose); *layout (nullable)
 * receives CCKA_TRAJ_TN / CCKA_TRAJ_NT. */
int ccka_get_trajectory_native(ccka_ctx* ctx, ccka_traj_rec* out, int64_t count, int32_t* layout);
int ccka_get_totals(ccka_ctx* ctx, ccka_totals* out);
/* on != 0: later rollouts also record the per-scenario ccka_detail (the
 * summary path: the run takes the general kernel; results are unchanged). */
int ccka_set_detail(ccka_ctx* ctx, int32_t on);
/* Copy the last rollout's details [count == n scenarios]; CCKA_ESTATE when it
 * ran without ccka_set_detail. */
int ccka_get_detail(ccka_ctx* ctx, ccka_detail* out, int64_t count);

/* ---- policy sweep (BASELINE config 4) -------------------------------- */
/* Per-grid sums of the last rollout's results. The batch must hold whole
 * grids (first_id and n multiples of grid_size); out[n / grid_size]. Sums are
 * taken on the device in a fixed order (deterministic). */
int ccka_get_grid_stats(ccka_ctx* ctx, int64_t grid_size, ccka_grid_stats* out, int64_t n_grids);
/* Cost / gCO2 / SLO-minutes Pareto frontier of the batch's grids (all three
 * minimised; equal vectors do not dominate each other). With a communicator
 * (ccka_comm_init) each rank's non-dominated grids are exchanged with an RCCL
 * all-gather over xGMI and every rank filters the union the same way, so all
 * ranks return the identical global frontier, sorted by grid id. Writes at most
 * `capacity` entries; *n_out = frontier size (CCKA_EINVAL if it exceeds
 * capacity). Every rank must hold the same number of grids. */
int ccka_pareto_frontier(ccka_ctx* ctx, int64_t grid_size, ccka_grid_stats* out, int32_t capacity,
                         int32_t* n_out);

/* ---- learned MLP control policy (BASELINE config 5) ------------------- */
/* Weights of the state(64) -> 256 -> 256 -> actions(8) ReLU policy: bf16 bit
 * patterns, row-major [in][out]; biases fp32. Only that shape is supported. */
int ccka_mlp_set_weights(ccka_ctx* ctx, int32_t in_dim, int32_t hidden, int32_t out_dim,
                         const uint16_t* w1, const float* b1, const uint16_t* w2, const float* b2,
                         const uint16_t* w3, const float* b3);
/* Cluster states [n][in_dim] bf16: uploaded, or synthesised on the device. */
int ccka_mlp_set_states(ccka_ctx* ctx, const uint16_t* x, int64_t n);
int ccka_mlp_gen_states(ccka_ctx* ctx, int64_t n, uint64_t seed);
/* actions = policy(states) on the device (bf16 MFMA, fp32 accumulation). The
 * standalone forward runs the 16x16x32 MFMA kernel; the policy loops keep the
 * 32x32x16 accumulation order. On the same states the two differ only in fp32
 * summation order (|dy| ~ 1e-3), which after the policy's rint can move an
 * action: for a loop's final states, ccka_debug_mlp_tile(ctx, 32) (internal)
 * makes the forward reproduce the loop's outputs bit for bit. */
int ccka_mlp_forward(ccka_ctx* ctx);
int ccka_mlp_forward_async(ccka_ctx* ctx);
/* Copy the actions [n][out_dim] fp32 back. */
int ccka_mlp_get_actions(ccka_ctx* ctx, float* y, int64_t n);

/* Closed-loop policy rollout (config 5): the learned policy in the loop.
 * Before every step t the engine writes each scenario's 64 policy features
 * (bf16, SEMANTICS 5), runs the MLP on all of them (bf16 MFMA, the weights of
 * ccka_mlp_set_weights) and maps each scenario's actions to step t's scaler
 * parameters: HPA target utilisation 60 + rint(16 y0) clamped to 20..95 % and
 * Karpenter carbon weight rint(16 y1)/16 clamped to 0..4 $/kgCO2 (they replace
 * the scenarios' target_util_pct / carbon_weight overrides). World, scenarios
 * and load as ccka_rollout; results / trajectory / totals / detail read back
 * the same way. record != 0 keeps the actions of every step.
 * The loop runs on the context's MLP state and action buffers: afterwards
 * the MLP state count is N and the states are the last step's features (as
 * if ccka_mlp_set_states had been called with them), so a later
 * ccka_mlp_forward evaluates those; states set before are replaced.
 * ccka_policy_grad does the same. */
int ccka_policy_rollout(ccka_ctx* ctx, int32_t trajectory, int32_t record);
/* The recorded actions: target [T][N] int16 (%), cw [T][N] double ($/kg). */
int ccka_get_policy_actions(ccka_ctx* ctx, int16_t* target, double* cw, int64_t count);

/* ---- differentiable control (config 5) -------------------------------- */
/* The closed loop with a stochastic policy: at every step each scenario samples
 * an action bin a from softmax(y) (y = the MLP's 8 outputs; Philox keyed by
 * seed, global id and step), a -> HPA target 40 + 10*(a & 3) % and Karpenter
 * carbon weight (a >> 2) $/kgCO2 (SEMANTICS 5). The objective of scenario i is
 * J_i = cost_i [$] + w_carbon * gCO2_i [kg] + w_slo * SLO-minutes_i, and
 * ccka_policy_grad returns the score-function (likelihood-ratio) estimate
 *   dE[J]/dW = (1/N) sum_i (J_i - b) sum_t d log pi(a_it | x_it) / dW,
 * b = mean J when baseline != 0 (else 0): the MLP backward over all N*T
 * (step, scenario) rows on bf16 MFMA with fp32 accumulation. Proposal anchor:
 * the controller picks "the cheapest and cleanest" pods / node types that meet
 * the SLO (CS218_Project_Proposal.pdf p.1); cost/carbon/SLO trade-offs (p.5). */
typedef struct ccka_pg_params {
  uint64_t seed;        /* Philox key of the action sampling */
  double w_carbon;      /* $ per kgCO2 in the objective (>= 0) */
  double w_slo;         /* $ per SLO-violation minute (>= 0) */
  int32_t baseline;     /* 1: advantages J - mean(J) */
  int32_t _pad;
} ccka_pg_params;
/* Gradient outputs: caller-owned fp32 host arrays in the layouts of
 * ccka_mlp_set_weights (w1 [64][256], b1 [256], w2 [256][256], b2 [256],
 * w3 [256][8], b3 [8]); NULL members are skipped. */
typedef struct ccka_mlp_grads {
  float* w1;
  float* b1;
  float* w2;
  float* b2;
  float* w3;
  float* b3;
} ccka_mlp_grads;
/* One stochastic closed-loop rollout (world, scenarios, load and weights as
 * ccka_policy_rollout; results / actions read back the same way) and the
 * gradient of E[J]; *objective_mean (nullable) = mean J of the batch.
 * Device memory: the loop's features, 128 B per (step, scenario) row, plus
 * the backward's work arrays for one chunk of at most 2^23 rows (2,192 B per
 * row, ~18 GB); chunks run in order and their gradients add up in that order,
 * so the result depends on N*T only, on any GPU (1e7 x 60 rows: ~78 GB of
 * features + ~18 GB of work arrays, ~96 GB in all; the single-deployment
 * kernel's tiled trace copy, N*T*4 B, is released for the loop). */
int ccka_policy_grad(ccka_ctx* ctx, const ccka_pg_params* params, ccka_mlp_grads* out, double* objective_mean);
/* The sampled action bins [T][N] and the per-scenario factors (J_i - b) / N of
 * the last ccka_policy_grad (count = T*N). */
int ccka_get_policy_samples(ccka_ctx* ctx, uint8_t* actions, float* coef, int64_t count);
/* The MLP backward alone on m given rows: x [m][64] bf16, action bins [m] (< 8),
 * coef [m]: the gradient of sum_m coef[m] * log softmax(policy(x_m))[a_m]. */
int ccka_mlp_backward(ccka_ctx* ctx, const uint16_t* x, const uint8_t* actions, const float* coef, int64_t m,
                      ccka_mlp_grads* out);

/* ---- multi-GPU (RCCL over xGMI) -------------------------------------- */
/* Fill a 128-byte RCCL unique id (rank 0 only; distribute it out of band). */
int ccka_comm_unique_id(uint8_t* id128);
int ccka_comm_init(ccka_ctx* ctx, const uint8_t* id128, int32_t nranks, int32_t rank);
/* In-place sum of the packed totals across ranks: ccka_totals_pack, one RCCL
 * all-reduce (sum) of the CCKA_TOTALS_BLOCK int64 words, ccka_totals_finish
 * (bit-identical at any rank count; CCKA_EOVERFLOW on every rank when the
 * sum could leave int64). */
int ccka_allreduce_totals(ccka_ctx* ctx, ccka_totals* inout);
/* Rank count and this context's rank as the RCCL communicator reports them
 * (ncclCommCount / ncclCommUserRank); CCKA_ESTATE without ccka_comm_init. */
int ccka_comm_info(ccka_ctx* ctx, int32_t* nranks, int32_t* rank);

/* Host-side halves of the totals exchange (no context, no GPU): the block
 * a rank contributes to the sum, and the totals of a summed block. A rank
 * whose fields exceed INT64_MAX / nranks in magnitude sets the guard word, so
 * after the sum every rank sees the same guard and ccka_totals_finish returns
 * CCKA_EOVERFLOW on all of them (no rank leaves the collective early). Any
 * transport that sums int64 words (RCCL here, gloo in the CPU tests) can carry
 * the block. n must be CCKA_TOTALS_BLOCK. */
int ccka_totals_pack(const ccka_totals* in, int32_t nranks, int64_t* block, int32_t n);
int ccka_totals_finish(const int64_t* block, int32_t n, ccka_totals* out);

/* ---- introspection ---------------------------------------------------- */
/* Name and compute-unit count of the context's device. */
int ccka_device_info(ccka_ctx* ctx, char* name, int32_t name_len, int32_t* cu_count);

#ifdef __cplusplus
}
#endif
#endif /* CCKA_H */
