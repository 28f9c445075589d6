// kparams.h — kernel argument blocks shared by rollout.hip and ccka_abi.cpp.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ccka.h"

namespace ccka {

// ccka_detail plus the per-group energy of the current clock hour (carbon is
// charged per hour, SEMANTICS 3.H); zeroed before the launch
struct DetailDev {
  ccka_detail d;
  int64_t e_hour[CCKA_MAX_POOLS];
  int64_t base_e_hour;
};

// Words per scenario of the general kernel's persisted state block (the
// closed loop): the st_xfer sequence of state_io in rollout.hip, one row per
// 32-bit value and two per 64-bit value. Host (allocation) and kernel (a
// check folded away at compile time when the sequence matches) both use it.
__host__ __device__ constexpr int64_t state_words(int dmax, int nmax) {
  return (int64_t)dmax * (5 + 2 * CCKA_HIST) + 5 * CCKA_MAX_POOLS + (int64_t)nmax * (6 + dmax) + 36;
}

constexpr int MLP_IN = 64, MLP_HID = 256, MLP_OUT = 8;
typedef short mlp_bf16x8 __attribute__((ext_vector_type(8)));

// Profiling-only phase switches (ccka_debug_ablate bits 1/2/4/8/32: skip
// disruption / provisioning / the detail breakdown / the HPA behavior / the
// fused loop's MLP). Compiled in only by variant builds
// (tools/build_variants.py name=-DCCKA_ABLATE_BUILD=1, tools/ablate.py); the
// shipping kernels fold every switch away.
#ifndef CCKA_ABLATE_BUILD
#define CCKA_ABLATE_BUILD 0
#endif
__host__ __device__ constexpr bool ablated(int mask, int bits) { return CCKA_ABLATE_BUILD && (mask & bits) != 0; }

struct KParams {
  const ccka_world* w;  // device copy (pools, deployments, scalars)
  const ccka_itype* types;
  const int32_t* price;  // [R][24][K][Z][2]
  const double* ci_gpwh;
  const double* ci_gpwmin;
  const int32_t* load;  // [T][D][N]
  const int32_t* load_nt;  // nullable: the same samples scenario-major [NL][T][DMAX] (SK; deployments >= D zero)
  // per-scenario overrides (nullable)
  const uint8_t* region;
  const int16_t* target;
  const int16_t* maxr;
  const int16_t* down_stab;
  const int16_t* reset_ca;
  const uint8_t* pswitch;
  const double* cw;
  const uint8_t* cap_sel;
  // results
  int64_t* cost;
  double* energy;
  double* gco2;
  int32_t* slo;
  int64_t* pend_min;
  int32_t* nmin_spot;
  int32_t* nmin_od;
  int32_t* launches;
  int32_t* deletions;
  int32_t* peak_nodes;
  int32_t* final_reps;
  int32_t* final_nodes;
  uint32_t* last_choice;
  uint32_t* hash;
  ccka_traj_rec* traj;  // nullable
  DetailDev* detail;    // nullable: per-scenario summary breakdown (ccka_set_detail)
  int2* hist;           // HBM decision history [hlen][D][N] {rec + 1 (0: none), delta}; hlen 0: register rings
  int32_t hlen, nsub, sync_s, _hpad;
  // closed-loop policy rollout (ccka_policy_rollout): steps [t0, t1) of the
  // horizon per launch; the scenario state persists in HBM between launches
  // ([word][N] int32, SoA: coalesced), and the launch leaves the policy
  // features of step t1 ([N][64] bf16, SEMANTICS 5)
  int32_t t0, t1;
  int32_t* state;        // nullable: no persistence (whole horizon in one launch)
  int32_t state_load;    // 1: resume from `state` (else initialise from the world)
  uint16_t* feat;        // nullable
  int64_t N;
  int64_t NL;           // load columns: N, or the shared trace count
  int64_t trace_mod;    // 0: column = scenario; else column = (first_id + i) % trace_mod
  int64_t first_id;
  int32_t T, D, K, Z, R, P, maxn, span, all_hours;
  int32_t lds_off_cap1, lds_off_tile, lds_off_claims, lds_off_misc, lds_off_ci;
  int32_t lds_lclaims;  // SK: per-lane NodeClaim columns for the lane-local F2 (-1: the cooperative scans)
  int32_t _kpad;
  int32_t ablate;  // profiling-only phase switches (0 in every real run)
  unsigned long long* stamps;  // diagnostic phase cycle totals (GK_STAMPS builds only; nullptr otherwise)
  int32_t prov[CCKA_MAX_DEPLOY];
  // fused closed loop (rollout_kernel<1, 8, POL>): the MLP runs inside the step
  // loop (SEMANTICS 5); POL 1 = deterministic actions, 2 = sampled (the
  // differentiable-control loop). W2 fragments and the biases in LDS at
  // lds_off_mlp; W1 / W3 fragments from L2.
  const mlp_bf16x8* w1f;
  const mlp_bf16x8* w2f;
  const mlp_bf16x8* w3f;
  const float* mlp_b;        // b1 | b2 | b3 (zero-padded to 32)
  const uint64_t* pol_seed;  // POL 2: the Philox key (device word)
  int16_t* rec_target;       // [T][N] nullable: the actions of every step
  double* rec_cw;
  uint8_t* pol_act;          // POL 2: sampled action bins [T][N]
  uint16_t* feat_rec;        // nullable: features of steps 0..T [T+1][N][64]
  int32_t lds_off_mlp, _ppad;
  // fused loop on a single-deployment world without pool limits: provisioning
  // by the argmin tables of table_kernel over the policy's 65 carbon weights
  // (k / 16, k = 0..64) instead of the wave-cooperative catalog scans
  const int2* ptable;        // nullable: [R*24][NZI][3][65][JT]
  const int32_t* pjtab;      // [R*24][NZI][3] J (largest pod count of an offered type)
  int32_t pNZI, pJT, pNW, _ppad2;
  int32_t pzmi[16];          // zone mask -> zone-mask index of the tables (-1: none)
};

struct GenParams {
  int32_t* out;
  const int32_t* sinq;
  int64_t n, first_id;
  uint64_t seed;
  int32_t T, D;
  int32_t base_lo, base_hi, amp_lo, amp_hi, noise, burst_prob, burst_mult, burst_len;
};

struct Part;
struct TotParams {
  const int64_t* cost;
  const double* energy;
  const double* gco2;
  const int32_t* slo;
  const int64_t* pend_min;
  const int32_t* nmin_spot;
  const int32_t* nmin_od;
  const int32_t* launches;
  const int32_t* deletions;
  Part* parts;
  ccka_totals* out;
  long long* ovf;  // set when a fixed-point sum would leave int64
  int64_t N;
};

constexpr int kPartBytes = 11 * 8;

// kernel instantiation chosen for (D, max_nodes): DMAX x MAXN
inline void kernel_dims(int D, int maxn, int* dmax, int* nmax) {
  // (12: the reference's own 12 burst Deployments, demo_30_burst_configure.sh, without
  // four empty deployment columns of per-lane state)
  *dmax = D == 1 ? 1 : D <= 2 ? 2 : D <= 4 ? 4 : D <= 8 ? 8 : D <= 12 ? 12 : 16;
  *nmax = maxn <= 8 && *dmax <= 4 ? 8 : 16;
}

hipError_t launch_gen_load(const GenParams& g, hipStream_t s);
hipError_t launch_rollout(const KParams& p, int block, size_t lds, hipStream_t s);
hipError_t launch_totals(const TotParams& q, int nparts, hipStream_t s);
hipError_t launch_rollout_policy(const KParams& p, size_t lds, int pol, hipStream_t s);
// four or more deployments, lockstep (rollout_multi.hip)
hipError_t launch_rollout_multi(const KParams& p, int block, size_t lds, hipStream_t s);
// two to four deployments on the lane-skewed schedule (rollout_sk.hip)
hipError_t launch_rollout_sk(const KParams& p, int block, size_t lds, hipStream_t s);
hipError_t launch_rollout_sk416(const KParams& p, int block, size_t lds, hipStream_t s);  // <4, 16> (rollout_sk416.hip)
// [T][D][NL] -> [NL][T][DP] (DP >= D, a power of two <= 16; padded with 0) for the skewed schedule
hipError_t launch_trace_nt(const int32_t* in, int32_t* out, int64_t NL, int64_t T, int32_t D, int32_t DP,
                           hipStream_t s);

// ---------------------------------------------------------------------------
// Single-deployment HPA engine (rollout_d1.hip): every BASELINE config 2-4
// workload. The host digests the world into this block (ccka_abi.cpp,
// d1_eligible / d1_prepare); the Karpenter launch choice comes from the
// per-rollout argmin tables built by launch_table.
// ---------------------------------------------------------------------------
constexpr int D1_MAX_ZI = 8;   // distinct NodePool zone masks
constexpr int D1_MAX_WC = 8;   // distinct carbon weights
constexpr int D1_REC_SAT = 32767;

struct D1Rule {
  int32_t sel, n, stab_mask, _pad;
  int32_t type[2], value[2], pmask[2];
  double factor[2];   // Percent: 1 +/- value/100 (binary64, as the spec writes it)
  // the same windows as packed int16 lane masks over the 8-entry history
  // (word r holds entries 2r, 2r+1): stab16 = 0xFFFF per entry in the
  // stabilisation window, pm16 = 1 per entry inside policy q's period
  int32_t stab16[4];
  int32_t pm16[2][4];
};

// Upstream default HPA behavior (autoscaling/v2 defaults): scale-up
// max(Percent 100, Pods 4) per 15 s without stabilisation, scale-down
// Percent 100 per 15 s (its window is per scenario). 15 s periods hold no
// 60 s history entry, so pmask = 0. The single-deployment kernel has an
// instantiation with these rules as compile-time constants (no rule registers).
constexpr D1Rule d1_default_rule(bool up) {
  D1Rule r{};
  r.sel = CCKA_SELECT_MAX;
  r.n = up ? 2 : 1;
  r.type[0] = CCKA_HPA_PERCENT;
  r.value[0] = 100;
  r.factor[0] = up ? 1.0 + 100.0 / 100.0 : 1.0 - 100.0 / 100.0;
  if (up) {
    r.type[1] = CCKA_HPA_PODS;
    r.value[1] = 4;
    r.factor[1] = 1.0 + 4.0 / 100.0;
  }
  return r;
}

// one profile patch of one pool, pre-digested: policy 0 / cas -1 / zi -1 / cm 0 = keep
struct D1Patch {
  int32_t policy, cas, zi, cm;  // cas = ceil(consolidate_after_s / 60) steps
};

struct D1Params {
  const int32_t* load;       // [T][N]
  const int32_t* load_w;     // the same trace wave-tiled [wave][T][lanes] (nullptr: read `load`)
  const int32_t* price;      // [R][24][K][Z][2]
  const double* ci_gpwmin;   // [R][24]
  const long long* acc;      // [K][3] idle_nw, dyn_nw_per_m, alloc_cpu_m
  const int2* table;         // [R][24][NZI][3][NW][JT] {price, info}; info -1 = none
  const int32_t* jtab;       // [R][24][NZI][3] max pods of one new claim
  // per-scenario overrides (nullable)
  const uint8_t* region;
  const int16_t* target;
  const int16_t* maxr;
  const int16_t* down_stab;
  const int16_t* reset_ca;
  const uint8_t* pswitch;
  const uint8_t* wci;        // carbon-weight index (NW distinct values)
  const uint8_t* cap_sel;
  // results (same buffers as KParams)
  int64_t* cost;
  double* energy;
  double* gco2;
  int32_t* slo;
  int64_t* pend_min;
  int32_t* nmin_spot;
  int32_t* nmin_od;
  int32_t* launches;
  int32_t* deletions;
  int32_t* peak_nodes;
  int32_t* final_reps;
  int32_t* final_nodes;
  uint32_t* last_choice;
  uint32_t* hash;
  ccka_traj_rec* traj;  // nullable
  int64_t N;
  int64_t NL, trace_mod, first_id;  // load columns / shared-trace mapping (as KParams)
  int32_t lpw;  // scenarios per wave (<= 64; fewer lanes = less divergence per wave)
  int32_t occ;   // register-allocation occupancy target of the instantiation (2 or 3)
  int32_t bdef;  // 1: up/dn are the upstream default behavior (d1_default_rule)
  int32_t T, K, Z, R, NP, maxn, NZI, NW, JT;
  int32_t start_minute, peak_start, peak_end, pswitch0, delay;
  int32_t base_nodes, base_type, slo_util, pdb_pct, pdb_member;
  int32_t replicas0, minr, maxr0, target0, req_cpu, limit, dstab0, reset_ca0, capsel0;
  double tol_lo, tol_hi;
  long long base_nw;
  int32_t ablate;  // profiling-only phase switches (0 in every real run)
  unsigned long long* stamps;  // diagnostic per-phase cycle totals (nullptr in every real run)
  D1Rule up, dn;
  int32_t budget[CCKA_MAX_POOLS];
  D1Patch patch[CCKA_MAX_POOLS][4];  // base, RESET, OFFPEAK, PEAK
  int32_t drift;                     // 1: the DRIFT instantiation (drift and/or replacement)
  uint32_t zml[16];                  // zone mask of each zone-mask index (patch zi)
  int32_t drift_on;                  // 1: Karpenter drift (SEMANTICS 3.G0) acts
  int32_t replace;                   // 1: replacement consolidation offers (SEMANTICS 3.G2)
  const int2* table2;                // [R][24][NZI][3][JT] cheapest offering by price (the G2 offer rule)
  int32_t lds_tab;                   // set by launch_rollout_d1: price tiles, ci and J staged in LDS
  int32_t nsub;                      // HPA decisions per step: 1, or 4 (15 s sync, default behavior)
  int32_t he4;                       // every down window <= 300 s (a 4-record ring suffices)
  int32_t multi;                     // 1: multi-node consolidation (SEMANTICS 3.G3) acts (DRIFT instantiation)
  // KEDA ScaledObject deployment (SEMANTICS 3.C, one trigger; the KEDA
  // instantiation: default behavior, one decision per step, no drift)
  int32_t keda;
  int32_t k_thr;   // AverageValue threshold per replica, 1 .. 2^22 - 1
  int32_t k_act;   // activationThreshold (int32; < INT32_MAX)
  int32_t k_cds;   // cooldownPeriod in whole steps: ceil(cooldown_s / 60), >= 0
  int32_t k_min;   // minReplicaCount
  int32_t k_max;   // maxReplicaCount
  // pooled event steps (rollout_pool.hip)
  const int32_t* cap1t;  // [K] pod capacity per type (the slots' capacity is their type's)
  int32_t pool_min;      // a wave serves the queue once it holds this many scenarios,
  int32_t pool_age;      // or any once the last claim is this many cycles old,
  int32_t pool_idle;     // or any when none of its own lanes can step (1)
  int32_t _ppad;
};

// rollout_pool_kernel: one 8-wave workgroup per CU, the scenario state in LDS
constexpr int PL_WAVES = 8;
struct PoolLds {
  uint32_t cap1, tab, win, queue, rqueue, ctrl, state, total;  // byte offsets into the dynamic LDS, total size
};
__host__ __device__ PoolLds pool_lds_layout(int K, int R, int Z, int NZI, int lds_tab, int sb, int hw);
hipError_t launch_rollout_pool(const D1Params& p, hipStream_t s);

// argmin-table builder: one wave per (region, hour, zone-mask, cap-mask, carbon weight)
struct TableParams {
  const int32_t* price;      // [R][24][K][Z][2]
  const double* ci_gpwh;     // [R][24]
  const ccka_itype* types;   // [K]
  const int32_t* order;      // [K] types by pod capacity desc, index asc
  const int32_t* cap1s;      // [K] pod capacity of order[i]
  const int32_t* cap1t;      // [K] pod capacity of type k (the launched node's, SEMANTICS 3.E/F)
  const uint32_t* zmasks;    // [NZI]
  const double* wc1000;      // [NW] carbon weight * 1000
  int2* table;
  int32_t* jtab;
  int32_t K, Z, R, NZI, NW, JT;
  int32_t offer;  // 1: the G2 offer rule (price only, no spot-first preference; NW = 1)
};

hipError_t launch_table(const TableParams& t, hipStream_t s);
hipError_t launch_trace_tile(const int32_t* in, int32_t* out, int64_t N, int64_t T, int32_t lpw, hipStream_t s);

// ---------------------------------------------------------------------------
// Policy sweep (config 4): per-grid sums and the Pareto frontier (sweep.hip)
// ---------------------------------------------------------------------------
struct GridSrc {
  const int64_t* cost;
  const double* gco2;
  const int32_t* slo;
  const double* energy;
  int64_t grid_size, first_grid, n_grids;
};
hipError_t launch_grid_stats(const GridSrc& g, ccka_grid_stats* out, hipStream_t s);
// streaming 16-byte-per-lane device copy (the measured copy ceiling of bench.py)
hipError_t launch_copy16(const void* in, void* out, int64_t bytes, int cus, hipStream_t s);
// non-dominated entries of in[0..n) (n may be device-resident: *n_dev if n < 0),
// compacted in input order into out; count into *count_dev
hipError_t launch_pareto(const ccka_grid_stats* in, int n, const int32_t* n_dev, uint8_t* flags,
                         ccka_grid_stats* out, int32_t* count_dev, hipStream_t s);
// concatenate the valid prefixes of an all-gathered [ranks][cap] buffer
hipError_t launch_pareto_union(const ccka_grid_stats* gathered, const int64_t* counts, int ranks, int cap,
                               ccka_grid_stats* out, int32_t* n_dev, hipStream_t s);

// ---------------------------------------------------------------------------
// Learned MLP policy (config 5, mlp.hip)
// ---------------------------------------------------------------------------
struct MlpParams {
  const uint16_t* x;          // [N][64] bf16
  float* y;                   // [N][8]
  const mlp_bf16x8* w1f;      // [8 row tiles][4 k-steps][64 lanes] A fragments of layer 1
  const mlp_bf16x8* w2f;      // [8][16][64] (k order of the chained accumulator)
  const mlp_bf16x8* w3f;      // [16][64], rows 8..31 zero
  const float *b1, *b2, *b3;
  int64_t N;
  unsigned long long* stamps;  // diagnostic phase stamps (nullptr in every real run)
  // set: mlp16_kernel (v_mfma_f32_16x16x32_bf16) with these fragment arrays
  const mlp_bf16x8* w1g;      // [16 row tiles][2 k-steps][64 lanes]
  const mlp_bf16x8* w2g;      // [16][8][64] (k order of the chained 16x16 accumulators)
  const mlp_bf16x8* w3g;      // [8][64], rows 8..15 zero
};
hipError_t launch_mlp(const MlpParams& p, int cus, hipStream_t s);
hipError_t launch_mlp_gen_states(uint16_t* x, int64_t count, uint64_t seed, hipStream_t s);
// policy actions -> the step's scaler parameters (SEMANTICS 5); rec_* nullable
hipError_t launch_policy_act(const float* y, int16_t* target, double* cw, int16_t* rec_target, double* rec_cw,
                             int64_t n, hipStream_t s);
hipError_t launch_rollout_d1(const D1Params& p, hipStream_t s);

// ---------------------------------------------------------------------------
// Differentiable control: score-function policy gradient (pg.hip)
// ---------------------------------------------------------------------------
// one stochastic policy step: action ~ softmax(y) (Philox(seed; id, t)), mapped
// to the step's HPA target and carbon weight (SEMANTICS 5)
struct PgSampleParams {
  const float* y;        // [n][8]
  uint8_t* act;          // [n]
  int16_t* target;       // [n]
  double* cw;            // [n]
  int16_t* rec_target;   // nullable [n]
  double* rec_cw;        // nullable [n]
  int64_t n, first_id;
  const uint64_t* seed;  // device word: the Philox key (read at run time, so a
                         // captured loop replays with any seed)
  int32_t t, _pad;
};
hipError_t launch_policy_sample(const PgSampleParams& q, hipStream_t s);
// forward recompute + backward per 32-row tile: unit-major [unit][Mpad] bf16 outputs
struct PgRowsParams {
  const uint16_t* x;        // [M][64] bf16
  const uint8_t* act;       // [M]
  const float* coef;        // [n_scen]
  const mlp_bf16x8* w1f;    // forward fragments (as MlpParams)
  const mlp_bf16x8* w2f;
  const mlp_bf16x8* w3f;
  const mlp_bf16x8* w2b;    // [8 row blocks][16 k-steps][64]: A fragments of dH1^T = W2 dH2^T
  const mlp_bf16x8* w3b;    // [8][64]: A fragments of dH2^T = W3 g_y^T (k = action, padded to 16)
  const float* bias;        // b1 | b2 | b3 (zero-padded), as MlpParams
  // row-blocked [Mpad/16][64|256|256|256|256|8][16] (element (u, m) at ((m/16) U + u) 16 + m%16)
  uint16_t *xT, *h1T, *h2T, *dh1T, *dh2T, *gyT;
  int64_t M, Mpad, n_scen;
  int64_t row0;  // global index of row 0 (row chunks): row m's factor is coef[(row0 + m) % n_scen]
};
hipError_t launch_pg_rows(const PgRowsParams& p, int cus, hipStream_t s);
// C[KA][KB] = sum_m A[a][m] B[b][m] over row-blocked bf16 operands (fp32 result)
struct WgradParams {
  const uint16_t* A;  // [Mpad/16][KA][16]
  const uint16_t* B;  // [Mpad/16][KB][16]
  float* part;        // split s's [KA][KB] at part + s * pstride
  float* bpart;       // nullable: split s's [KB] column sums of B (the bias gradient) at bpart + s * pstride
  int64_t Mpad;
  int64_t pstride;    // floats between two splits' partials
  int32_t KA, KB, splits, _pad;
};
// per-split partials of A B^T summed over the split's rows (+ the row sums of B)
hipError_t launch_pg_wgrad(const WgradParams& q, hipStream_t s);
// out[i] (+)= sum over splits of part[s * n + i], in split order
hipError_t launch_pg_reduce(const float* part, float* out, int64_t n, int splits, int acc, hipStream_t s);
hipError_t launch_pg_fill(uint16_t* x, int64_t n, int64_t valid, uint16_t v, hipStream_t s);
// [N][T] (single-deployment engine, device side) -> steps [t0, t0 + tc) of the
// [T][N] order ccka_get_trajectory returns, into out[tc][N]
hipError_t launch_traj_transpose(const ccka_traj_rec* in, ccka_traj_rec* out, int64_t N, int64_t T, int64_t t0,
                                 int64_t tc, hipStream_t s);

}  // namespace ccka
