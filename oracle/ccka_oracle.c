/*
 * ccka_oracle.c — TEST INFRASTRUCTURE: CPU restatement of docs/SEMANTICS.md.
 *
 * This file is the checker for the HIP engine and the timed CPU baseline
 * ("kind": "port" in bench.py). It is deliberately written as plain,
 * array-based C that follows the spec line by line; it shares no code with
 * the engine (only the POD declarations of include/ccka.h).
 *
 * Reference anchors (the reference is bash + manifests; the arithmetic is the
 * upstream controllers it drives, see SEMANTICS.md "Parity status"):
 *   profiles      demo_19_reset_policies.sh:68-75, demo_20_offpeak_configure.sh:59-81,
 *                 demo_21_peak_configure.sh:56-77 (captured run lines 188-209)
 *   pods          demo_30_burst_configure.sh:57-141 (nodeSelector :104-105,
 *                 requests/limits :134-140), PDB demo_10_setup_configure.sh:47-56
 *   base nodes    01_cluster.sh:24-30, .env:5-8
 *   HPA           upstream k8s 1.34 (.env:4) horizontal.go / replica_calculator.go
 *   Karpenter     upstream 1.8.1 (05_karpenter.sh:20) provisioner + disruption
 *   KEDA          never installed (.env:10-12), ScaledObject semantics
 *
 * Build: gcc -O3 -march=native -ffp-contract=off -fPIC -shared -pthread
 * (see oracle/Makefile). No contraction, no fast-math: every double operation
 * below is one IEEE binary64 operation in the order SEMANTICS.md states.
 */
#include "ccka_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <stddef.h>
#include <string.h>

#define O_BIG 0x3fffffffffffffffLL

/* ------------------------------------------------------------------------ */
/* Philox-4x32-10                                                            */
/* ------------------------------------------------------------------------ */
void ccka_oracle_philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                        uint32_t k0, uint32_t k1, uint32_t* out4) {
  uint32_t c[4] = {c0, c1, c2, c3};
  uint32_t k[2] = {k0, k1};
  for (int r = 0; r < 10; ++r) {
    uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    uint32_t n0 = hi1 ^ c[1] ^ k[0];
    uint32_t n1 = lo1;
    uint32_t n2 = hi0 ^ c[3] ^ k[1];
    uint32_t n3 = lo0;
    c[0] = n0; c[1] = n1; c[2] = n2; c[3] = n3;
    k[0] += 0x9E3779B9u;
    k[1] += 0xBB67AE85u;
  }
  out4[0] = c[0]; out4[1] = c[1]; out4[2] = c[2]; out4[3] = c[3];
}

void ccka_oracle_sin_table(int32_t* out) {
  for (int m = 0; m < 1440; ++m)
    out[m] = (int32_t)lround(65536.0 * sin(2.0 * M_PI * (double)m / 1440.0));
}

void ccka_oracle_gen_load(const ccka_trace_gen* g, int32_t T, int32_t D, int64_t n,
                          int64_t first_id, int32_t* out) {
  int32_t sinq[1440];
  ccka_oracle_sin_table(sinq);
  const uint32_t k0 = (uint32_t)g->seed, k1 = (uint32_t)(g->seed >> 32);
  for (int64_t i = 0; i < n; ++i) {
    const uint64_t s = (uint64_t)(first_id + i);
    const uint32_t slo = (uint32_t)s, shi = (uint32_t)(s >> 32);
    for (int32_t d = 0; d < D; ++d) {
      uint32_t u[4], v[4];
      ccka_oracle_philox(0xFFFFFFFFu, slo, shi, (uint32_t)d, k0, k1, u);
      ccka_oracle_philox(0xFFFFFFFEu, slo, shi, (uint32_t)d, k0, k1, v);
      const int64_t base = g->base_lo + (int64_t)(u[0] % (uint32_t)(g->base_hi - g->base_lo + 1));
      const int64_t amp = g->amp_lo_pm + (int64_t)(u[1] % (uint32_t)(g->amp_hi_pm - g->amp_lo_pm + 1));
      const int32_t phase = (int32_t)(u[2] % 1440u);
      const int burst = (int32_t)(u[3] % 1000u) < g->burst_prob_pm;
      const int32_t bstart = (int32_t)(v[0] % 1440u);
      for (int32_t t = 0; t < T; ++t) {
        uint32_t e4[4];
        ccka_oracle_philox((uint32_t)t, slo, shi, (uint32_t)d, k0, k1, e4);
        const int64_t e = (int64_t)(e4[0] >> 16) + (int64_t)(e4[1] >> 16) +
                          (int64_t)(e4[2] >> 16) + (int64_t)(e4[3] >> 16) - 131072;
        int64_t val = base * (65536000LL + amp * (int64_t)sinq[(t + phase) % 1440]) / 65536000LL;
        val = val * (37837000LL + (int64_t)g->noise_pm * e) / 37837000LL;
        if (burst && t >= bstart && t < bstart + g->burst_len) val = val * g->burst_mult_pm / 1000;
        if (val < 0) val = 0;
        if (val > 0x7fffffff) val = 0x7fffffff;
        out[((int64_t)t * D + d) * n + i] = (int32_t)val;
      }
    }
  }
}

/* ------------------------------------------------------------------------ */
/* HPA pieces                                                                */
/* ------------------------------------------------------------------------ */
static int o_within(double x, double tol) { return (1.0 - tol) <= x && x <= (1.0 + tol); }

int32_t ccka_oracle_hpa_resource_proposal(int32_t cur, int32_t ready, int64_t usage_m,
                                          int32_t req_m, int32_t target_pct, double tol,
                                          int32_t* util_out) {
  if (ready <= 0 || req_m <= 0) {
    if (util_out) *util_out = -1;
    return cur;
  }
  const int32_t util = (int32_t)((usage_m * 100) / ((int64_t)ready * req_m));
  if (util_out) *util_out = util;
  const double ratio = (double)util / (double)target_pct;
  const int32_t unready = cur - ready;
  if (unready > 0 && ratio > 1.0) {
    /* upstream: unready pods count as 0 usage when scaling up */
    const int32_t nutil = (int32_t)((usage_m * 100) / ((int64_t)cur * req_m));
    const double nr = (double)nutil / (double)target_pct;
    if (o_within(nr, tol) || nr < 1.0) return cur;
    int32_t p = (int32_t)ceil(nr * (double)cur);
    if (p < cur) p = cur;
    return p;
  }
  if (o_within(ratio, tol)) return cur;
  return (int32_t)ceil(ratio * (double)ready);
}

int32_t ccka_oracle_keda_proposal(int32_t cur, int64_t metric, int64_t threshold, double tol) {
  const double r = (double)metric / ((double)threshold * (double)cur);
  if (o_within(r, tol)) return cur;
  return (int32_t)ceil((double)metric / (double)threshold);
}

/* history entry k holds the decision (k + 1) * sync_s seconds ago; a record
 * counts inside a window / period W iff its age < W (upstream's
 * timestamp.Add(W).After(now)) */
static int o_entries(int32_t window_s, int32_t sync_s) { return window_s > sync_s ? (window_s - 1) / sync_s : 0; }

/* replicas changed by the scaler within a policy period: (added, deleted) */
static void o_period_sums(const ccka_hpa_policy* p, int32_t sync_s, const int32_t* deltas, int n, int64_t* added,
                          int64_t* deleted) {
  *added = *deleted = 0;
  const int m = o_entries(p->period_s, sync_s) < n ? o_entries(p->period_s, sync_s) : n;
  for (int k = 0; k < m; ++k) {
    if (deltas[k] > 0) *added += deltas[k];
    if (deltas[k] < 0) *deleted += -deltas[k];
  }
}

static int32_t o_rate_up(int32_t cur, const ccka_hpa_rules* up, int32_t sync_s, const int32_t* deltas, int n) {
  if (up->select == CCKA_SELECT_DISABLED) return cur;
  int64_t res = up->select == CCKA_SELECT_MIN ? INT32_MAX : INT32_MIN;
  for (int i = 0; i < up->n_policies; ++i) {
    const ccka_hpa_policy* p = &up->policies[i];
    int64_t added, deleted;
    o_period_sums(p, sync_s, deltas, n, &added, &deleted);
    const int64_t ps = cur - added + deleted;
    int64_t prop;
    if (p->type == CCKA_HPA_PODS) prop = ps + p->value;
    else prop = (int32_t)ceil((double)ps * (1.0 + (double)p->value / 100.0));
    if (up->select == CCKA_SELECT_MIN) { if (prop < res) res = prop; }
    else { if (prop > res) res = prop; }
  }
  return (int32_t)res;
}

static int32_t o_rate_down(int32_t cur, const ccka_hpa_rules* dn, int32_t sync_s, const int32_t* deltas, int n) {
  if (dn->select == CCKA_SELECT_DISABLED) return cur;
  /* Max selects the policy allowing the biggest change: the minimum count */
  int64_t res = dn->select == CCKA_SELECT_MIN ? INT32_MIN : INT32_MAX;
  for (int i = 0; i < dn->n_policies; ++i) {
    const ccka_hpa_policy* p = &dn->policies[i];
    int64_t added, deleted;
    o_period_sums(p, sync_s, deltas, n, &added, &deleted);
    const int64_t ps = cur - added + deleted;
    int64_t prop;
    if (p->type == CCKA_HPA_PODS) prop = ps - p->value;
    else prop = (int32_t)((double)ps * (1.0 - (double)p->value / 100.0));
    if (dn->select == CCKA_SELECT_MIN) { if (prop > res) res = prop; }
    else { if (prop < res) res = prop; }
  }
  return (int32_t)res;
}

int32_t ccka_oracle_hpa_behavior_n(int32_t cur, int32_t proposal, int32_t min_r, int32_t max_r,
                                   const ccka_hpa_rules* up, const ccka_hpa_rules* down, int32_t sync_s,
                                   const int32_t* recs, const uint8_t* rec_valid, const int32_t* deltas, int32_t n) {
  /* stabilizeRecommendationWithBehaviors */
  int32_t upr = proposal, dnr = proposal;
  const int nu = o_entries(up->stab_window_s, sync_s), nd = o_entries(down->stab_window_s, sync_s);
  const int m = (nu > nd ? nu : nd) < n ? (nu > nd ? nu : nd) : n;
  for (int k = 0; k < m; ++k) {
    if (!rec_valid[k]) continue;
    if (k < nu && recs[k] < upr) upr = recs[k];
    if (k < nd && recs[k] > dnr) dnr = recs[k];
  }
  int32_t rec = cur;
  if (rec < upr) rec = upr;
  if (rec > dnr) rec = dnr;
  /* convertDesiredReplicasWithBehaviorRate */
  int32_t lo = min_r, hi = max_r;
  if (rec > cur) {
    int32_t lim = o_rate_up(cur, up, sync_s, deltas, n);
    if (lim < cur) lim = cur;
    if (hi > lim) hi = lim;
  } else if (rec < cur) {
    int32_t lim = o_rate_down(cur, down, sync_s, deltas, n);
    if (lim > cur) lim = cur;
    if (lo < lim) lo = lim;
  }
  if (rec < lo) return lo;
  if (rec > hi) return hi;
  return rec;
}

int32_t ccka_oracle_hpa_behavior(int32_t cur, int32_t proposal, int32_t min_r, int32_t max_r,
                                 const ccka_hpa_rules* up, const ccka_hpa_rules* down,
                                 const int32_t* recs, const uint8_t* rec_valid,
                                 const int32_t* deltas) {
  return ccka_oracle_hpa_behavior_n(cur, proposal, min_r, max_r, up, down, CCKA_STEP_SECONDS, recs, rec_valid, deltas,
                                    CCKA_HIST);
}

/* ------------------------------------------------------------------------ */
/* Scenario state                                                            */
/* ------------------------------------------------------------------------ */
typedef struct {
  int used, pool, type, zone, cap, ready_step, last_event;
  uint32_t srcm; /* replacement node: bit n = it replaces slot n (0: none) */
  int pods[CCKA_MAX_DEPLOY];
} o_node;

typedef struct {
  int policy, ca_s;
  uint32_t zone_mask, cap_mask;
} o_pool;

typedef struct {
  int replicas;
  int32_t rec[CCKA_HPA_HIST_MAX]; /* entry k: the decision (k + 1) * sync_s ago */
  uint8_t rec_valid[CCKA_HPA_HIST_MAX];
  int32_t delta[CCKA_HPA_HIST_MAX];
  int hn; /* entries any window or period of this deployment reaches */
  int last_active;
} o_dep;

typedef struct {
  int pool, slot;
  uint32_t cap, zone;
  int64_t s_cpu, s_mem, s_pods;
  int pods[CCKA_MAX_DEPLOY];
} o_claim;

static void o_patch(o_pool* p, const ccka_pool_patch* pp) {
  if (pp->policy != CCKA_POLICY_KEEP) p->policy = pp->policy;
  if (pp->consolidate_after_s >= 0) p->ca_s = pp->consolidate_after_s;
  if (pp->zone_mask) p->zone_mask = pp->zone_mask;
  if (pp->cap_mask) p->cap_mask = pp->cap_mask;
}

static int64_t o_usage(int64_t L, int64_t ready, int32_t limit) {
  if (limit <= 0) return L;
  const int64_t cap = ready * limit;
  return L < cap ? L : cap;
}

/* max additional pods of (rc, rm) on capacity (ac, am, ap) holding (uc, um, up);
 * -1 when the capacity cannot hold what it already has. */
static int64_t o_fit(int64_t ac, int64_t am, int64_t ap, int64_t uc, int64_t um, int64_t up,
                     int32_t rc, int32_t rm) {
  if (uc > ac || um > am || up > ap) return -1;
  int64_t f = ap - up;
  if (rc > 0) { int64_t c = (ac - uc) / rc; if (c < f) f = c; }
  if (rm > 0) { int64_t m = (am - um) / rm; if (m < f) f = m; }
  return f;
}

static int o_capidx_bit(int c) { return c == 0 ? CCKA_CAP_SPOT : CCKA_CAP_OD; }

typedef struct {
  const ccka_world* w;
  int T, D, K, Z, N;     /* N = maxnodes */
  int prov[CCKA_MAX_DEPLOY];
} o_env;

static int32_t o_price(const o_env* e, int r, int h, int k, int z, int c) {
  return e->w->price_uph[((((int64_t)r * 24 + h) * e->K + k) * e->Z + z) * 2 + c];
}

/* node usage of a slot */
static void o_node_use(const o_env* e, const o_node* nd, int64_t* uc, int64_t* um, int64_t* up) {
  int64_t c = 0, m = 0, p = 0;
  for (int d = 0; d < e->D; ++d) {
    c += (int64_t)nd->pods[d] * e->w->deploy[d].req_cpu_m;
    m += (int64_t)nd->pods[d] * e->w->deploy[d].req_mem_mi;
    p += nd->pods[d];
  }
  *uc = c; *um = m; *up = p;
}

static int64_t o_node_fit(const o_env* e, const o_node* nd, int d) {
  const ccka_itype* ty = &e->w->types[nd->type];
  int64_t uc, um, up;
  o_node_use(e, nd, &uc, &um, &up);
  int64_t f = o_fit(ty->alloc_cpu_m, ty->alloc_mem_mi, ty->max_pods, uc, um, up,
                    e->w->deploy[d].req_cpu_m, e->w->deploy[d].req_mem_mi);
  return f < 0 ? 0 : f;
}

/* resources of a pool's nodes: CPU capacity (millicores) and memory capacity (MiB) */
typedef struct {
  int64_t cpu, mem;
} o_use;

/* NodePool spec.limits: a new node of type ty keeps the pool within its CPU
 * and memory limits (SEMANTICS 3.F) */
static int o_limits_ok(const ccka_pool* pl, o_use u, const ccka_itype* ty) {
  if (pl->limit_cpu_m >= 0 && u.cpu + (int64_t)ty->vcpu * 1000 > pl->limit_cpu_m) return 0;
  if (pl->limit_mem_mi >= 0 && u.mem + (int64_t)ty->mem_mi > pl->limit_mem_mi) return 0;
  return 1;
}

/* type candidate for a claim: holds sums, limits, offered in masks */
static int o_type_ok(const o_env* e, int r, int h, int k, uint32_t zm, uint32_t cm,
                     o_use pool_use, const ccka_pool* pl) {
  const ccka_itype* ty = &e->w->types[k];
  if (!o_limits_ok(pl, pool_use, ty)) return 0;
  for (int z = 0; z < e->Z; ++z) {
    if (!(zm >> z & 1u)) continue;
    for (int c = 0; c < 2; ++c)
      if ((cm & (uint32_t)o_capidx_bit(c)) && o_price(e, r, h, k, z, c) > 0) return 1;
  }
  return 0;
}

static int64_t o_claim_j(const o_env* e, int r, int h, const o_claim* cl, uint32_t cm, int d,
                         o_use pool_use, const ccka_pool* pl) {
  int64_t best = 0;
  for (int k = 0; k < e->K; ++k) {
    if (!o_type_ok(e, r, h, k, cl->zone, cm, pool_use, pl)) continue;
    const ccka_itype* ty = &e->w->types[k];
    const int64_t f = o_fit(ty->alloc_cpu_m, ty->alloc_mem_mi, ty->max_pods, cl->s_cpu, cl->s_mem,
                            cl->s_pods, e->w->deploy[d].req_cpu_m, e->w->deploy[d].req_mem_mi);
    if (f > best) best = f;
  }
  return best;
}

typedef struct {
  o_pool pools[CCKA_MAX_POOLS];
  o_node nodes[CCKA_MAX_NODES];
  int profile;
  int64_t cost, pend_min;
  int64_t energy_nw, e_hour; /* nanowatt-minutes: total, current clock hour */
  double gco2;
  int slo, nmin_spot, nmin_od, launches, deletions, peak_nodes;
  uint32_t last_choice, hash;
  int pool_launches[CCKA_MAX_POOLS];
  o_dep dep[CCKA_MAX_DEPLOY]; /* last: only the first D are initialised */
} o_state;

/* Karpenter drift: the node's zone or capacity type no longer satisfies its
 * pool's (patched) requirements. */
/* free a slot; a pending replacement of it becomes an ordinary node */
static void o_free(o_node* nodes, int NN, int n) {
  memset(&nodes[n], 0, sizeof(o_node));
  for (int m = 0; m < NN; ++m)
    nodes[m].srcm &= ~(1u << n);
}

/* cheapest single offering (price, k, z, c) holding the sums under zone mask
 * zm, capacity mask cm and the pool CPU limit; -1 if none (SEMANTICS 3.G2) */
static int o_offer(const o_env* e, int r, int h, uint32_t zm, uint32_t cm, o_use use, const ccka_pool* pl,
                   int64_t sc, int64_t sm, int64_t sp, int* bz, int* bc, int32_t* bp) {
  int bk = -1;
  for (int k = 0; k < e->K; ++k) {
    const ccka_itype* ty = &e->w->types[k];
    if (o_fit(ty->alloc_cpu_m, ty->alloc_mem_mi, ty->max_pods, sc, sm, sp, 0, 0) < 0) continue;
    if (!o_limits_ok(pl, use, ty)) continue;
    for (int z = 0; z < e->Z; ++z) {
      if (!(zm >> z & 1u)) continue;
      for (int cc = 0; cc < 2; ++cc) {
        if (!(cm & (uint32_t)o_capidx_bit(cc))) continue;
        const int32_t pr = o_price(e, r, h, k, z, cc);
        if (pr > 0 && (bk < 0 || pr < *bp)) { bk = k; *bz = z; *bc = cc; *bp = pr; }
      }
    }
  }
  return bk;
}

/* The launch choice of a NodeClaim with sums (sc, sm, sp) (SEMANTICS 3.F):
 * candidates hold the sums, fit the pool limit and have an offering with
 * z in zm, c in cm, price > 0; if spot is allowed and any spot offering is
 * feasible only spot offerings compete; the lexicographic minimum of
 * (score, k, z, c), score = price + carbon_weight*1000*(p_ref_w*ci). -1 if none. */
static int o_launch_choice(const o_env* e, int r, int h, uint32_t zm, uint32_t cm, o_use use, const ccka_pool* pl,
                           int64_t sc, int64_t sm, int64_t sp, double wc1000, int* bz, int* bc, int32_t* bp) {
  const ccka_world* w = e->w;
  int spot_only = 0;
  if (cm & CCKA_CAP_SPOT) {
    for (int k = 0; k < e->K && !spot_only; ++k) {
      const ccka_itype* ty = &w->types[k];
      if (o_fit(ty->alloc_cpu_m, ty->alloc_mem_mi, ty->max_pods, sc, sm, sp, 0, 0) < 0) continue;
      if (!o_limits_ok(pl, use, ty)) continue;
      for (int z = 0; z < e->Z; ++z)
        if ((zm >> z & 1u) && o_price(e, r, h, k, z, 0) > 0) { spot_only = 1; break; }
    }
  }
  int bk = -1;
  double bs = 0.0;
  for (int k = 0; k < e->K; ++k) {
    const ccka_itype* ty = &w->types[k];
    if (o_fit(ty->alloc_cpu_m, ty->alloc_mem_mi, ty->max_pods, sc, sm, sp, 0, 0) < 0) continue;
    if (!o_limits_ok(pl, use, ty)) continue;
    for (int z = 0; z < e->Z; ++z) {
      if (!(zm >> z & 1u)) continue;
      for (int cc = 0; cc < 2; ++cc) {
        if (!(cm & (uint32_t)o_capidx_bit(cc))) continue;
        if (spot_only && cc != 0) continue;
        const int32_t pr = o_price(e, r, h, k, z, cc);
        if (pr <= 0) continue;
        const double score = (double)pr + wc1000 * (ty->p_ref_w * w->ci_gpwh[r * 24 + h]);
        if (bk < 0 || score < bs) { bk = k; *bz = z; *bc = cc; *bp = pr; bs = score; }
      }
    }
  }
  return bk;
}

/* a pre-spun replacement for the slots in srcm, no pods until it takes over */
static void o_launch_repl(o_state* st, int slot, int p, int bk, int bz, int bc, int ready, int t, uint32_t srcm) {
  o_node* nd = &st->nodes[slot];
  memset(nd, 0, sizeof *nd);
  nd->used = 1;
  nd->pool = p;
  nd->type = bk;
  nd->zone = bz;
  nd->cap = bc;
  nd->ready_step = ready;
  nd->last_event = t;
  nd->srcm = srcm;
  st->launches++;
  st->pool_launches[p]++;
  st->last_choice = (uint32_t)bk | (uint32_t)bz << 12 | (uint32_t)bc << 14 | (uint32_t)p << 16;
  st->hash = (st->hash ^ st->last_choice) * 16777619u;
}

/* Karpenter taints a disruption candidate karpenter.sh/disrupted:NoSchedule
 * while its replacement is in flight: neither the source nor the pre-spun
 * replacement (sized for the source's pods, SEMANTICS 3.G0/G2) receives other
 * pods until the takeover, and the source is no consolidation candidate. */
static int o_tainted(const o_node* nodes, int NN, int n) {
  if (nodes[n].srcm) return 1;
  for (int m = 0; m < NN; ++m)
    if (nodes[m].used && (nodes[m].srcm >> n & 1u)) return 1;
  return 0;
}

static o_use o_pool_use(const o_state* st, const ccka_world* w, int NN, int p) {
  o_use u = {0, 0};
  for (int m = 0; m < NN; ++m)
    if (st->nodes[m].used && st->nodes[m].pool == p) {
      u.cpu += (int64_t)w->types[st->nodes[m].type].vcpu * 1000;
      u.mem += w->types[st->nodes[m].type].mem_mi;
    }
  return u;
}

static int o_drifted(const o_state* st, const o_node* nd) {
  const o_pool* pl = &st->pools[nd->pool];
  return !(pl->zone_mask >> nd->zone & 1u) || !(pl->cap_mask & (uint32_t)o_capidx_bit(nd->cap));
}

/* G3 trial (docs/SEMANTICS.md 3.G3): the first k candidates of `order` leave
 * the cluster together. Their pods move first-fit (candidates in order,
 * deployments in index order, receivers in slot order: ready, untainted,
 * outside the set, capacity-type compatible) on a copy of the slots; what does
 * not fit needs one new node: the cheapest offering (price, k, z, c) holding
 * the leftover sums under the pool's zone mask, capacity types
 * pool.cap_mask & the leftovers' nodeSelectors (no spot when every candidate is
 * spot) and limits, strictly cheaper than the candidates together, in a free
 * slot. Returns 1 when the set consolidates; *bk < 0: no new node needed. */
static int o_g3_try(const o_env* e, const o_state* st, int r, int h, int p, const int* order, int k,
                    const uint32_t* capsel, int64_t allowed, int t, o_node* trial, int* bk, int* bz, int* bc,
                    int32_t* bp, int* slot, int64_t* pdb_out) {
  const ccka_world* w = e->w;
  const int D = e->D, NN = e->N;
  uint32_t set = 0;
  int all_spot = 1;
  int64_t pdb_pods = 0, price_sum = 0;
  for (int i = 0; i < k; ++i) {
    const o_node* nd = &st->nodes[order[i]];
    set |= 1u << order[i];
    all_spot &= nd->cap == 0;
    price_sum += o_price(e, r, h, nd->type, nd->zone, nd->cap);
    for (int d = 0; d < D; ++d) if (w->deploy[d].pdb_member) pdb_pods += nd->pods[d];
  }
  *pdb_out = pdb_pods;
  if (pdb_pods > allowed) return 0;
  memcpy(trial, st->nodes, sizeof(o_node) * (size_t)NN);
  for (int i = 0; i < k; ++i) {
    o_node* cn = &trial[order[i]];
    for (int d = 0; d < D; ++d) {
      int need = cn->pods[d];
      for (int m = 0; m < NN && need > 0; ++m) {
        o_node* nd = &trial[m];
        if ((set >> m & 1u) || !nd->used || nd->ready_step > t) continue;
        if (o_tainted(st->nodes, NN, m)) continue;
        if (!((uint32_t)o_capidx_bit(nd->cap) & capsel[d])) continue;
        const int64_t f = o_node_fit(e, nd, d);
        const int kk = (int)(f < need ? f : need);
        if (kk > 0) { nd->pods[d] += kk; need -= kk; nd->last_event = t; }
      }
      cn->pods[d] = need;
    }
  }
  int64_t sc = 0, sm = 0, sp = 0;
  uint32_t cm = st->pools[p].cap_mask;
  for (int i = 0; i < k; ++i)
    for (int d = 0; d < D; ++d) {
      const int left = trial[order[i]].pods[d];
      if (left <= 0) continue;
      cm &= capsel[d];
      sc += (int64_t)left * w->deploy[d].req_cpu_m;
      sm += (int64_t)left * w->deploy[d].req_mem_mi;
      sp += left;
    }
  *bk = -1;
  *slot = -1;
  if (sp == 0) return 1;  /* delete only */
  if (all_spot) cm &= ~(uint32_t)CCKA_CAP_SPOT;
  if (!cm) return 0;
  for (int m = 0; m < NN; ++m) if (!st->nodes[m].used) { *slot = m; break; }
  if (*slot < 0) return 0;
  const o_use use = o_pool_use(st, w, NN, p);
  *bk = o_offer(e, r, h, st->pools[p].zone_mask, cm, use, &w->pools[p], sc, sm, sp, bz, bc, bp);
  return *bk >= 0 && (int64_t)*bp < price_sum;
}

static uint16_t o_bf16(float f) {
  uint32_t b;
  memcpy(&b, &f, 4);
  return (uint16_t)((b + 0x7FFFu + ((b >> 16) & 1u)) >> 16);
}

/* The 64 policy features of a scenario before step t1 (docs/SEMANTICS.md 5),
 * bit-identical to the engine's (integers scaled by powers of two, fp32, bf16
 * round-to-nearest-even). */
static void o_features(const o_env* e, const o_state* st, const int32_t* load, int64_t nl, int64_t col, int r,
                       int pswitch, int t1, uint16_t* f) {
  const ccka_world* w = e->w;
  const int D = e->D, NN = e->N, T = e->T;
  int reps = 0, rd = 0;
  for (int d = 0; d < D; ++d) {
    reps += st->dep[d].replicas;
    for (int n = 0; n < NN; ++n)
      if (st->nodes[n].used && st->nodes[n].ready_step <= t1 - 1) rd += st->nodes[n].pods[d];
  }
  const int tf = t1 < T ? t1 : T - 1;
  const int mf = (w->start_minute + t1) % 1440, hf = mf / 60;
  const int ps = w->peak_start_min, pe = w->peak_end_min;
  const int in_win = ps <= pe ? (mf >= ps && mf < pe) : (mf >= ps || mf < pe);
  int64_t burn = 0;
  int nsp = 0, nod = 0;
  const int hp = t1 > 0 ? ((w->start_minute + t1 - 1) % 1440) / 60 : 0;
  for (int n = 0; n < NN; ++n) {
    const o_node* nd = &st->nodes[n];
    if (!nd->used) continue;
    burn += o_price(e, r, hp, nd->type, nd->zone, nd->cap);
    if (nd->cap == 0) nsp++; else nod++;
  }
  float v[34];
  v[0] = 1.0f;
  v[1] = (float)reps * 0.0625f;
  v[2] = (float)rd * 0.0625f;
  v[3] = (float)(reps - rd) * 0.0625f;
  v[4] = (float)load[((int64_t)tf * D) * nl + col] * (1.0f / 1024.0f);
  v[5] = (float)nsp;
  v[6] = (float)nod;
  v[7] = (pswitch && in_win) ? 1.0f : 0.0f;
  v[8] = (float)w->ci_gpwh[r * 24 + hf];
  v[9] = (float)burn * (1.0f / 65536.0f);
  for (int h = 0; h < 24; ++h) v[10 + h] = h == hf ? 1.0f : 0.0f;
  for (int j = 0; j < 34; ++j) f[j] = o_bf16(v[j]);
  for (int n = 0; n < 16; ++n) {
    int pods = 0, code = 0;
    if (n < NN && st->nodes[n].used) {
      for (int d = 0; d < D; ++d) pods += st->nodes[n].pods[d];
      code = 1 + st->nodes[n].cap + (st->nodes[n].ready_step <= t1 - 1 ? 0 : 2);
    }
    f[34 + n] = o_bf16((float)pods * 0.0625f);
    if (n < 14) f[50 + n] = o_bf16((float)code);
  }
}

/* det (optional): the per-pool / base-group / per-deployment breakdown of
 * ccka_detail, accounted exactly as the run totals (SEMANTICS 3.H) */
/* act_t / act_cw (optional, [T][nsc]): the closed-loop policy's per-step HPA
 * target utilisation and carbon weight (SEMANTICS 5); feat (optional,
 * [T + 1][nsc][64]): the policy features before every step and after the last */
static void o_run_one(const o_env* e, const ccka_scenarios* sc, const int32_t* load, int64_t i,
                      int64_t nsc, ccka_results* out, ccka_traj_rec* traj, ccka_detail* det,
                      const int16_t* act_t, const double* act_cw, uint16_t* feat) {
  const ccka_world* w = e->w;
  const int D = e->D, NN = e->N;
  o_state st;
  memset(&st, 0, offsetof(o_state, dep));
  memset(st.dep, 0, (size_t)D * sizeof(o_dep));
  /* HPA / KEDA decisions per step (SEMANTICS 3.C sub-steps) */
  const int32_t sync_s = w->hpa_sync_s > 0 ? w->hpa_sync_s : CCKA_STEP_SECONDS;
  const int nsub = CCKA_STEP_SECONDS / sync_s;
  /* load column: the scenario's own trace, or its shared trace (policy sweeps) */
  const int64_t nl = sc->n_traces > 0 ? sc->n_traces : nsc;
  const int64_t col = sc->n_traces > 0 ? (sc->first_id + i) % sc->n_traces : i;
  const int r = sc->region ? sc->region[i] : 0;
  const int reset_ca = sc->reset_ca_s ? sc->reset_ca_s[i] : w->reset_ca_s;
  const int pswitch = sc->peak_switch ? sc->peak_switch[i] : w->peak_switch;
  const double cw = sc->carbon_weight ? sc->carbon_weight[i] : w->carbon_weight;
  double wc1000 = cw * 1000.0;
  int target[CCKA_MAX_DEPLOY], maxr[CCKA_MAX_DEPLOY];
  uint32_t capsel[CCKA_MAX_DEPLOY];
  ccka_hpa_rules downr[CCKA_MAX_DEPLOY];
  for (int d = 0; d < D; ++d) {
    const ccka_deployment* dp = &w->deploy[d];
    target[d] = dp->target_util_pct;
    maxr[d] = dp->max_replicas;
    downr[d] = dp->down;
    capsel[d] = sc->cap_sel ? sc->cap_sel[i] : dp->cap_sel;
    if (dp->scaler == CCKA_SCALER_HPA) {
      if (sc->target_util_pct) target[d] = sc->target_util_pct[i];
      if (sc->max_replicas) maxr[d] = sc->max_replicas[i];
      if (sc->down_stab_s) downr[d].stab_window_s = sc->down_stab_s[i];
    }
    st.dep[d].replicas = dp->replicas0;
    st.dep[d].last_active = 0;
    int hn = o_entries(dp->up.stab_window_s, sync_s);
    const int hd = o_entries(downr[d].stab_window_s, sync_s);
    if (hd > hn) hn = hd;
    for (int q = 0; q < dp->up.n_policies; ++q)
      if (o_entries(dp->up.policies[q].period_s, sync_s) > hn) hn = o_entries(dp->up.policies[q].period_s, sync_s);
    for (int q = 0; q < dp->down.n_policies; ++q)
      if (o_entries(dp->down.policies[q].period_s, sync_s) > hn) hn = o_entries(dp->down.policies[q].period_s, sync_s);
    st.dep[d].hn = hn < CCKA_HPA_HIST_MAX ? hn : CCKA_HPA_HIST_MAX;
  }
  for (int p = 0; p < w->n_pools; ++p) {
    memset(&st.pools[p], 0, sizeof(o_pool));
    o_patch(&st.pools[p], &w->pools[p].base);
    ccka_pool_patch rp = w->pools[p].profile[CCKA_PROFILE_RESET];
    if (rp.consolidate_after_s >= 0) rp.consolidate_after_s = reset_ca;
    o_patch(&st.pools[p], &rp);
  }
  st.profile = -1;
  st.hash = 2166136261u;
  st.last_choice = 0xFFFFFFFFu;
  const ccka_itype* bt = &w->types[w->base_type];
  const int64_t base_nw = (int64_t)w->base_nodes *
                          (bt->idle_nw + bt->dyn_nw_per_m * (int64_t)(w->base_util * (double)bt->alloc_cpu_m));
  int prev_h = -1;
  const int ps = w->peak_start_min, pe = w->peak_end_min;
  int64_t pool_eh[CCKA_MAX_POOLS] = {0}, base_eh = 0; /* detail: energy of the current clock hour */
  if (det) memset(det, 0, sizeof *det);

  for (int t = 0; t < w->n_steps; ++t) {
    if (feat) o_features(e, &st, load, nl, col, r, pswitch, t, feat + ((int64_t)t * nsc + i) * 64);
    if (act_t) {  /* this step's policy action */
      for (int d = 0; d < D; ++d)
        if (w->deploy[d].scaler == CCKA_SCALER_HPA) target[d] = act_t[(int64_t)t * nsc + i];
      wc1000 = act_cw[(int64_t)t * nsc + i] * 1000.0;
    }
    const int minute = (w->start_minute + t) % 1440;
    const int h = minute / 60;
    /* carbon is charged per clock hour (SEMANTICS §3.H) */
    if (prev_h >= 0 && h != prev_h) {
      st.gco2 += (double)st.e_hour * (w->ci_gpwmin[r * 24 + prev_h] * 1e-9);
      st.e_hour = 0;
      if (det) {
        for (int p = 0; p < w->n_pools; ++p) {
          det->pool_gco2[p] += (double)pool_eh[p] * (w->ci_gpwmin[r * 24 + prev_h] * 1e-9);
          pool_eh[p] = 0;
        }
        det->base_gco2 += (double)base_eh * (w->ci_gpwmin[r * 24 + prev_h] * 1e-9);
        base_eh = 0;
      }
    }
    prev_h = h;
    uint16_t flags = 0;
    uint16_t step_last_type = 0xFFFF;
    /* ---- A. profile ---- */
    int in_win = ps <= pe ? (minute >= ps && minute < pe) : (minute >= ps || minute < pe);
    const int peak = pswitch && in_win;
    const int prof = peak ? CCKA_PROFILE_PEAK : CCKA_PROFILE_OFFPEAK;
    if (peak) flags |= 1;
    if (prof != st.profile) {
      for (int p = 0; p < w->n_pools; ++p) o_patch(&st.pools[p], &w->pools[p].profile[prof]);
      st.profile = prof;
    }
    /* ---- C. scalers: nsub decisions on the step's metric sample ---- */
    int util_valid[CCKA_MAX_DEPLOY], util[CCKA_MAX_DEPLOY], keda_act[CCKA_MAX_DEPLOY] = {0};
    int64_t Lt[CCKA_MAX_DEPLOY];
    for (int sub = 0; sub < nsub; ++sub)
    for (int d = 0; d < D; ++d) {
      const ccka_deployment* dp = &w->deploy[d];
      o_dep* ds = &st.dep[d];
      const int64_t L = load[((int64_t)t * D + d) * nl + col];
      Lt[d] = L;
      util_valid[d] = 0;
      util[d] = 0;
      int ready = 0;
      for (int n = 0; n < NN; ++n)
        if (st.nodes[n].used && st.nodes[n].ready_step <= t) ready += st.nodes[n].pods[d];
      const int cur = ds->replicas;
      int desired = cur;
      int ran = 0;           /* HPA normal path ran: store rec */
      int32_t proposal = cur;
      int hpa_path = 0;      /* desired produced by the HPA (records delta) */
      int minr = dp->min_replicas, mx = maxr[d];
      if (dp->scaler == CCKA_SCALER_HPA) {
        hpa_path = 1;
        if (cur == 0 && minr != 0) { desired = 0; hpa_path = 0; }
        else if (cur > mx) desired = mx;
        else if (cur < minr) desired = minr;
        else if (ready == 0) { desired = cur; }
        else {
          int32_t u = 0;
          const int64_t usage = o_usage(L, ready, dp->limit_cpu_m);
          proposal = ccka_oracle_hpa_resource_proposal(cur, ready, usage, dp->req_cpu_m, target[d],
                                                       dp->tolerance, &u);
          util_valid[d] = 1;
          util[d] = u;
          desired = ccka_oracle_hpa_behavior_n(cur, proposal, minr, mx, &dp->up, &downr[d], sync_s, ds->rec,
                                               ds->rec_valid, ds->delta, ds->hn);
          ran = 1;
        }
      } else if (dp->scaler == CCKA_SCALER_KEDA) {
        /* triggers: this deployment's own + the KEDA_TRIGGER entries after it;
         * active if any trigger is, proposal = max over triggers (upstream HPA
         * with several external metrics) */
        int nt = 1;
        while (d + nt < D && w->deploy[d + nt].scaler == CCKA_SCALER_KEDA_TRIGGER) ++nt;
        int active = 0;
        for (int j = 0; j < nt; ++j)
          active |= load[((int64_t)t * D + d + j) * nl + col] > w->deploy[d + j].keda_activation;
        keda_act[d] = active;
        if (active) ds->last_active = t;
        if (cur == 0) desired = active ? 1 : 0;
        else if (!active && dp->keda_min == 0 &&
                 (int64_t)(t - ds->last_active) * CCKA_STEP_SECONDS >= dp->keda_cooldown_s)
          desired = 0;
        else {
          hpa_path = 1;
          minr = dp->keda_min > 1 ? dp->keda_min : 1;
          mx = dp->keda_max;
          if (cur > mx) desired = mx;
          else if (cur < minr) desired = minr;
          else {
            proposal = ccka_oracle_keda_proposal(cur, L, dp->keda_threshold, dp->tolerance);
            for (int j = 1; j < nt; ++j) {
              const int32_t pj = ccka_oracle_keda_proposal(cur, load[((int64_t)t * D + d + j) * nl + col],
                                                           w->deploy[d + j].keda_threshold, dp->tolerance);
              if (pj > proposal) proposal = pj;
            }
            desired = ccka_oracle_hpa_behavior_n(cur, proposal, minr, mx, &dp->up, &dp->down, sync_s, ds->rec,
                                                 ds->rec_valid, ds->delta, ds->hn);
            ran = 1;
          }
        }
      }
      if (dp->scaler == CCKA_SCALER_HPA || dp->scaler == CCKA_SCALER_KEDA) {
        /* shift the history: entry 0 becomes this decision */
        if (ds->hn > 0) {
          for (int k = ds->hn - 1; k > 0; --k) {
            ds->rec[k] = ds->rec[k - 1];
            ds->rec_valid[k] = ds->rec_valid[k - 1];
            ds->delta[k] = ds->delta[k - 1];
          }
          ds->rec[0] = ran ? proposal : 0;
          ds->rec_valid[0] = (uint8_t)ran;
          ds->delta[0] = (hpa_path && desired != cur) ? desired - cur : 0;
        }
        ds->replicas = desired;
      }
    }
    /* ---- D. ReplicaSet reconcile ---- */
    for (int d = 0; d < D; ++d) {
      int total = 0;
      for (int n = 0; n < NN; ++n) if (st.nodes[n].used) total += st.nodes[n].pods[d];
      int excess = total - st.dep[d].replicas;
      for (int pass = 0; pass < 2 && excess > 0; ++pass) {
        for (int n = NN - 1; n >= 0 && excess > 0; --n) {
          o_node* nd = &st.nodes[n];
          if (!nd->used) continue;
          const int rdy = nd->ready_step <= t;
          if ((pass == 0 && rdy) || (pass == 1 && !rdy)) continue;
          if (nd->pods[d] <= 0) continue;
          const int k = nd->pods[d] < excess ? nd->pods[d] : excess;
          nd->pods[d] -= k;
          excess -= k;
          nd->last_event = t;
        }
      }
    }
    /* ---- E. kube-scheduler (ready) and F1. nomination (in-flight) ---- */
    int pend[CCKA_MAX_DEPLOY];
    for (int pass = 0; pass < 2; ++pass) {
      for (int d = 0; d < D; ++d) {
        int total = 0;
        for (int n = 0; n < NN; ++n) if (st.nodes[n].used) total += st.nodes[n].pods[d];
        int p = st.dep[d].replicas - total;
        for (int n = 0; n < NN && p > 0; ++n) {
          o_node* nd = &st.nodes[n];
          if (!nd->used) continue;
          const int rdy = nd->ready_step <= t;
          if ((pass == 0 && !rdy) || (pass == 1 && rdy)) continue;
          if (!((uint32_t)o_capidx_bit(nd->cap) & capsel[d])) continue;
          if (o_tainted(st.nodes, NN, n)) continue;
          const int64_t f = o_node_fit(e, nd, d);
          const int k = (int)(f < p ? f : p);
          if (k > 0) { nd->pods[d] += k; p -= k; nd->last_event = t; }
        }
        pend[d] = p;
      }
    }
    /* ---- F2. provisioning ---- */
    {
      o_use pool_use[CCKA_MAX_POOLS];
      memset(pool_use, 0, sizeof pool_use);
      int slot_taken[CCKA_MAX_NODES];
      for (int n = 0; n < NN; ++n) {
        slot_taken[n] = st.nodes[n].used;
        if (st.nodes[n].used) {
          pool_use[st.nodes[n].pool].cpu += (int64_t)w->types[st.nodes[n].type].vcpu * 1000;
          pool_use[st.nodes[n].pool].mem += w->types[st.nodes[n].type].mem_mi;
        }
      }
      o_claim claims[CCKA_MAX_NODES];
      int ncl = 0;
      for (int oi = 0; oi < D; ++oi) {
        const int d = e->prov[oi];
        int rem = pend[d];
        if (rem <= 0) continue;
        const ccka_deployment* dp = &w->deploy[d];
        for (int c = 0; c < ncl && rem > 0; ++c) {
          o_claim* cl = &claims[c];
          const uint32_t cm = cl->cap & capsel[d];
          if (!cm) continue;
          const int64_t j = o_claim_j(e, r, h, cl, cm, d, pool_use[cl->pool], &w->pools[cl->pool]);
          if (j <= 0) continue;
          const int k = (int)(j < rem ? j : rem);
          cl->cap = cm;
          cl->pods[d] += k;
          cl->s_cpu += (int64_t)k * dp->req_cpu_m;
          cl->s_mem += (int64_t)k * dp->req_mem_mi;
          cl->s_pods += k;
          rem -= k;
        }
        while (rem > 0) {
          int slot = -1;
          for (int n = 0; n < NN; ++n) if (!slot_taken[n]) { slot = n; break; }
          if (slot < 0) break;
          int chosen = -1;
          int64_t jj = 0;
          o_claim nc;
          memset(&nc, 0, sizeof nc);
          for (int p = 0; p < w->n_pools; ++p) {
            const uint32_t cm = st.pools[p].cap_mask & capsel[d];
            if (!cm) continue;
            nc.pool = p;
            nc.cap = cm;
            nc.zone = st.pools[p].zone_mask;
            const int64_t j = o_claim_j(e, r, h, &nc, cm, d, pool_use[p], &w->pools[p]);
            if (j > 0) { chosen = p; jj = j; break; }
          }
          if (chosen < 0) break;
          const int k = (int)(jj < rem ? jj : rem);
          nc.pool = chosen;
          nc.cap = st.pools[chosen].cap_mask & capsel[d];
          nc.zone = st.pools[chosen].zone_mask;
          nc.slot = slot;
          nc.pods[d] = k;
          nc.s_cpu = (int64_t)k * dp->req_cpu_m;
          nc.s_mem = (int64_t)k * dp->req_mem_mi;
          nc.s_pods = k;
          slot_taken[slot] = 1;
          claims[ncl++] = nc;
          rem -= k;
        }
      }
      /* launch in creation order */
      for (int c = 0; c < ncl; ++c) {
        o_claim* cl = &claims[c];
        int bz = 0, bc = 0;
        int32_t bpr = 0;
        const int bk = o_launch_choice(e, r, h, cl->zone, cl->cap, pool_use[cl->pool], &w->pools[cl->pool], cl->s_cpu, cl->s_mem,
                                       cl->s_pods, wc1000, &bz, &bc, &bpr);
        if (bk < 0) { continue; /* dropped: slot stays free */ }
        o_node* nd = &st.nodes[cl->slot];
        memset(nd, 0, sizeof *nd);
        nd->used = 1;
        nd->pool = cl->pool;
        nd->type = bk;
        nd->zone = bz;
        nd->cap = bc;
        nd->ready_step = t + w->provision_delay_steps;
        nd->last_event = t;
        for (int d = 0; d < D; ++d) nd->pods[d] = cl->pods[d];
        pool_use[cl->pool].cpu += (int64_t)w->types[bk].vcpu * 1000;
        pool_use[cl->pool].mem += w->types[bk].mem_mi;
        st.launches++;
        st.pool_launches[cl->pool]++;
        st.last_choice = (uint32_t)bk | (uint32_t)bz << 12 | (uint32_t)bc << 14 | (uint32_t)cl->pool << 16;
        st.hash = (st.hash ^ st.last_choice) * 16777619u;
        step_last_type = (uint16_t)bk;
        flags |= 2;
      }
    }
    /* ---- G. disruption ---- */
    {
      /* G1. replacements that are ready take over their sources' pods
       * (docs/SEMANTICS.md 3.G2, 3.G3): replacements in slot order, each one's
       * sources in slot order; pods that no longer fit are evicted; the
       * sources are deleted */
      for (int m = 0; (w->disrupt_ext & (CCKA_DISRUPT_DRIFT | CCKA_DISRUPT_REPLACE | CCKA_DISRUPT_MULTI)) && m < NN;
           ++m) {
        o_node* rn = &st.nodes[m];
        if (!rn->used || !rn->srcm || rn->ready_step > t) continue;
        const uint32_t sm = rn->srcm;
        rn->srcm = 0;
        for (int n = 0; n < NN; ++n) {
          if (!(sm >> n & 1u)) continue;
          for (int d = 0; d < D; ++d) {
            if (!((uint32_t)o_capidx_bit(rn->cap) & capsel[d])) continue;
            const int64_t f = o_node_fit(e, rn, d);
            const int k = (int)(f < st.nodes[n].pods[d] ? f : st.nodes[n].pods[d]);
            if (k > 0) rn->pods[d] += k;
          }
          o_free(st.nodes, NN, n);
          st.deletions++;
        }
        rn->last_event = t;
        flags |= 4;
      }
      int64_t allowed = O_BIG;
      if (w->pdb_min_available_pct >= 0) {
        int64_t rdy = 0, reps = 0;
        for (int d = 0; d < D; ++d) {
          if (!w->deploy[d].pdb_member) continue;
          reps += st.dep[d].replicas;
          for (int n = 0; n < NN; ++n)
            if (st.nodes[n].used && st.nodes[n].ready_step <= t) rdy += st.nodes[n].pods[d];
        }
        const int64_t desired_healthy = (w->pdb_min_available_pct * reps + 99) / 100;
        allowed = rdy - desired_healthy;
        if (allowed < 0) allowed = 0;
      }
      for (int p = 0; p < w->n_pools; ++p) {
        int npool = 0;
        for (int n = 0; n < NN; ++n) if (st.nodes[n].used && st.nodes[n].pool == p) npool++;
        if (npool == 0) continue;
        const int budget = (w->pools[p].budget_pct * npool + 99) / 100;
        int deleted = 0;
        /* G0. drift (docs/SEMANTICS.md 3.G0): ready nodes whose zone or
         * capacity type left the pool's requirements after the patch of
         * demo_20_offpeak_configure.sh:64-81 / demo_21_peak_configure.sh:60-77,
         * slot order, sharing this pool's budget; no consolidateAfter wait */
        for (int n = 0; (w->disrupt_ext & CCKA_DISRUPT_DRIFT) && n < NN && deleted < budget; ++n) {
          o_node* dn = &st.nodes[n];
          if (!dn->used || dn->pool != p || dn->ready_step > t || !o_drifted(&st, dn)) continue;
          int src = 0;  /* its pre-spun replacement is in flight: wait for it */
          for (int m = 0; m < NN; ++m) src |= (st.nodes[m].srcm >> n) & 1u;
          if (src) continue;
          int64_t pdb_pods = 0;
          for (int d = 0; d < D; ++d) if (w->deploy[d].pdb_member) pdb_pods += dn->pods[d];
          if (pdb_pods > allowed) continue;
          /* pods move first-fit onto ready, non-drifted nodes; the rest are
           * evicted and Pending until F places or provisions them */
          int left[CCKA_MAX_DEPLOY];
          for (int d = 0; d < D; ++d) {
            int need = dn->pods[d];
            for (int m = 0; m < NN && need > 0; ++m) {
              o_node* nd = &st.nodes[m];
              if (m == n || !nd->used || nd->ready_step > t || o_drifted(&st, nd)) continue;
              if (o_tainted(st.nodes, NN, m)) continue;
              if (!((uint32_t)o_capidx_bit(nd->cap) & capsel[d])) continue;
              const int64_t f = o_node_fit(e, nd, d);
              const int k = (int)(f < need ? f : need);
              if (k > 0) { nd->pods[d] += k; need -= k; nd->last_event = t; }
            }
            left[d] = need;
          }
          /* pods that found no room: a pre-spun replacement under the new
           * requirements takes them when ready (G1); without a free slot or
           * an offering they are evicted and the node goes now */
          {
            int64_t sc = 0, sm = 0, sp = 0;
            uint32_t cm = st.pools[p].cap_mask;
            for (int d = 0; d < D; ++d) {
              if (left[d] <= 0) continue;
              cm &= capsel[d];
              sc += (int64_t)left[d] * w->deploy[d].req_cpu_m;
              sm += (int64_t)left[d] * w->deploy[d].req_mem_mi;
              sp += left[d];
            }
            int slot = -1;
            for (int m = 0; m < NN; ++m) if (!st.nodes[m].used) { slot = m; break; }
            const o_use use = o_pool_use(&st, w, NN, p);
            int bz = 0, bc = 0, bk = -1;
            int32_t bp = 0;
            if (sp > 0 && slot >= 0 && cm)  /* an ordinary provisioning decision: the F2 rule */
              bk = o_launch_choice(e, r, h, st.pools[p].zone_mask, cm, use, &w->pools[p], sc, sm, sp,
                                   wc1000, &bz, &bc, &bp);
            if (bk >= 0) {
              for (int d = 0; d < D; ++d) dn->pods[d] = left[d];
              o_launch_repl(&st, slot, p, bk, bz, bc, t + w->provision_delay_steps, t, 1u << n);
              step_last_type = (uint16_t)bk;
              allowed -= pdb_pods;
              deleted++;
              flags |= 2 | 16 | 32;
              continue;
            }
          }
          o_free(st.nodes, NN, n);
          allowed -= pdb_pods;
          deleted++;
          st.deletions++;
          flags |= 4 | 16;
        }
        int rejected[CCKA_MAX_NODES] = {0};
        while (deleted < budget) {
          int best = -1, bpods = 0;
          int32_t bprice = 0;
          for (int n = 0; n < NN; ++n) {
            const o_node* nd = &st.nodes[n];
            if (!nd->used || nd->pool != p || nd->ready_step > t || rejected[n]) continue;
            if ((int64_t)(t - nd->last_event) * CCKA_STEP_SECONDS < st.pools[p].ca_s) continue;
            if (o_tainted(st.nodes, NN, n)) continue;
            int pods = 0;
            for (int d = 0; d < D; ++d) pods += nd->pods[d];
            if (pods > 0 && st.pools[p].policy != CCKA_WHEN_EMPTY_OR_UNDERUTILIZED) continue;
            const int32_t pr = o_price(e, r, h, nd->type, nd->zone, nd->cap);
            if (best < 0 || pods < bpods || (pods == bpods && pr > bprice)) {
              best = n; bpods = pods; bprice = pr;
            }
          }
          if (best < 0) break;
          int ok = 1;
          int64_t pdb_pods = 0;
          o_node trial[CCKA_MAX_NODES];
          memcpy(trial, st.nodes, sizeof(o_node) * (size_t)NN);
          if (bpods > 0) {
            for (int d = 0; d < D; ++d) if (w->deploy[d].pdb_member) pdb_pods += trial[best].pods[d];
            if (pdb_pods > allowed) ok = 0;
            for (int d = 0; d < D && ok; ++d) {
              int need = trial[best].pods[d];
              for (int n = 0; n < NN && need > 0; ++n) {
                o_node* nd = &trial[n];
                if (n == best || !nd->used || nd->ready_step > t) continue;
                if (o_tainted(trial, NN, n)) continue;
                if (!((uint32_t)o_capidx_bit(nd->cap) & capsel[d])) continue;
                const int64_t f = o_node_fit(e, nd, d);
                const int k = (int)(f < need ? f : need);
                if (k > 0) { nd->pods[d] += k; need -= k; nd->last_event = t; }
              }
              if (need > 0) ok = 0;
            }
          }
          if (!ok) { rejected[best] = 1; continue; }
          memcpy(st.nodes, trial, sizeof(o_node) * (size_t)NN);
          o_free(st.nodes, NN, best);
          allowed -= pdb_pods;
          deleted++;
          st.deletions++;
          flags |= 4;
        }
        /* G3. multi-node consolidation (docs/SEMANTICS.md 3.G3): Karpenter's
         * firstN binary search over the candidate prefix (>= 2 nodes) that can
         * leave together, with at most one cheaper replacement */
        int g3_acted = 0;
        if ((w->disrupt_ext & CCKA_DISRUPT_MULTI) && st.pools[p].policy == CCKA_WHEN_EMPTY_OR_UNDERUTILIZED &&
            deleted < budget) {
          int order[CCKA_MAX_NODES], nc = 0;
          uint32_t taken = 0;
          for (;;) {
            int best = -1, bpods = 0;
            int32_t bprice = 0;
            for (int n = 0; n < NN; ++n) {
              const o_node* nd = &st.nodes[n];
              if ((taken >> n & 1u) || !nd->used || nd->pool != p || nd->ready_step > t) continue;
              if ((int64_t)(t - nd->last_event) * CCKA_STEP_SECONDS < st.pools[p].ca_s) continue;
              if (o_tainted(st.nodes, NN, n)) continue;
              int pods = 0;
              for (int d = 0; d < D; ++d) pods += nd->pods[d];
              if (pods == 0) continue;
              const int32_t pr = o_price(e, r, h, nd->type, nd->zone, nd->cap);
              if (best < 0 || pods < bpods || (pods == bpods && pr > bprice)) { best = n; bpods = pods; bprice = pr; }
            }
            if (best < 0) break;
            taken |= 1u << best;
            order[nc++] = best;
          }
          if (nc > budget - deleted) nc = budget - deleted;
          int lo = 1, hi = nc - 1, bestk = 0;
          o_node trial[CCKA_MAX_NODES];
          int bk = -1, bz = 0, bc = 0, slot = -1;
          int32_t bp = 0;
          int64_t pdb_pods = 0;
          while (lo <= hi) {
            const int mid = (lo + hi) / 2;
            if (o_g3_try(e, &st, r, h, p, order, mid + 1, capsel, allowed, t, trial, &bk, &bz, &bc, &bp, &slot,
                         &pdb_pods)) {
              bestk = mid + 1;
              lo = mid + 1;
            } else {
              hi = mid - 1;
            }
          }
          if (bestk) {
            (void)o_g3_try(e, &st, r, h, p, order, bestk, capsel, allowed, t, trial, &bk, &bz, &bc, &bp, &slot,
                           &pdb_pods);
            memcpy(st.nodes, trial, sizeof(o_node) * (size_t)NN);
            uint32_t srcm = 0;
            for (int i = 0; i < bestk; ++i) {
              const int n = order[i];
              int pods = 0;
              for (int d = 0; d < D; ++d) pods += st.nodes[n].pods[d];
              if (pods > 0) {
                srcm |= 1u << n;  /* leaves when the replacement is ready */
              } else {
                o_free(st.nodes, NN, n);
                st.deletions++;
                flags |= 4;
              }
            }
            if (bk >= 0) {
              o_launch_repl(&st, slot, p, bk, bz, bc, t + w->provision_delay_steps, t, srcm);
              step_last_type = (uint16_t)bk;
              flags |= 2 | 32;
            }
            flags |= 64;
            allowed -= pdb_pods;
            deleted += bestk;
            g3_acted = 1;
          }
        }
        /* G2. single-node replacement consolidation (docs/SEMANTICS.md 3.G2):
         * the first candidate (same order, on-demand, with pods, not already
         * being replaced) that has a strictly cheaper single offering for its
         * pods gets a pre-spun replacement; one per pool per step */
        int rej2[CCKA_MAX_NODES] = {0};
        while ((w->disrupt_ext & CCKA_DISRUPT_REPLACE) && !g3_acted &&
               st.pools[p].policy == CCKA_WHEN_EMPTY_OR_UNDERUTILIZED && deleted < budget) {
          int best = -1, bpods = 0;
          int32_t bprice = 0;
          for (int n = 0; n < NN; ++n) {
            const o_node* nd = &st.nodes[n];
            if (!nd->used || nd->pool != p || nd->ready_step > t || rej2[n] || nd->cap != 1) continue;
            if ((int64_t)(t - nd->last_event) * CCKA_STEP_SECONDS < st.pools[p].ca_s) continue;
            int src = 0;
            for (int m = 0; m < NN; ++m) src |= (st.nodes[m].srcm >> n) & 1u;
            if (src) continue;
            int pods = 0;
            for (int d = 0; d < D; ++d) pods += nd->pods[d];
            if (pods == 0) continue;
            const int32_t pr = o_price(e, r, h, nd->type, nd->zone, nd->cap);
            if (best < 0 || pods < bpods || (pods == bpods && pr > bprice)) { best = n; bpods = pods; bprice = pr; }
          }
          if (best < 0) break;
          int slot = -1;
          for (int n = 0; n < NN; ++n) if (!st.nodes[n].used) { slot = n; break; }
          if (slot < 0) break;
          const o_node* cn = &st.nodes[best];
          int64_t pdb_pods = 0, s_cpu = 0, s_mem = 0, s_pods = 0;
          uint32_t cm = st.pools[p].cap_mask;
          for (int d = 0; d < D; ++d) {
            if (cn->pods[d] <= 0) continue;
            if (w->deploy[d].pdb_member) pdb_pods += cn->pods[d];
            cm &= capsel[d];
            s_cpu += (int64_t)cn->pods[d] * w->deploy[d].req_cpu_m;
            s_mem += (int64_t)cn->pods[d] * w->deploy[d].req_mem_mi;
            s_pods += cn->pods[d];
          }
          if (pdb_pods > allowed || !cm) { rej2[best] = 1; continue; }
          const o_use use = o_pool_use(&st, w, NN, p);
          int bz = 0, bc = 0;
          int32_t bp = 0;
          const int bk = o_offer(e, r, h, st.pools[p].zone_mask, cm, use, &w->pools[p], s_cpu, s_mem, s_pods, &bz, &bc, &bp);
          if (bk < 0 || bp >= bprice) { rej2[best] = 1; continue; }
          o_launch_repl(&st, slot, p, bk, bz, bc, t + w->provision_delay_steps, t, 1u << best);
          step_last_type = (uint16_t)bk;
          flags |= 2 | 32;
          deleted++;
          break;
        }
      }
    }
    /* ---- H. accounting ---- */
    {
      int64_t cost = (int64_t)w->base_nodes * o_price(e, r, h, w->base_type, 0, 1);
      int ready_d[CCKA_MAX_DEPLOY];
      int64_t upp[CCKA_MAX_DEPLOY];
      for (int d = 0; d < D; ++d) {
        int rd = 0;
        for (int n = 0; n < NN; ++n)
          if (st.nodes[n].used && st.nodes[n].ready_step <= t) rd += st.nodes[n].pods[d];
        ready_d[d] = rd;
        upp[d] = 0;
        if (rd > 0) {
          int64_t u = o_usage(Lt[d], rd, w->deploy[d].limit_cpu_m);
          if (u < 0) u = 0;
          upp[d] = u / rd;
        }
      }
      int64_t e_step = base_nw;
      int nsp = 0, nod = 0;
      for (int n = 0; n < NN; ++n) {
        const o_node* nd = &st.nodes[n];
        if (!nd->used) continue;
        const ccka_itype* ty = &w->types[nd->type];
        cost += o_price(e, r, h, nd->type, nd->zone, nd->cap);
        int64_t use = 0;
        if (nd->ready_step <= t) {
          for (int d = 0; d < D; ++d) use += (int64_t)nd->pods[d] * upp[d];
          if (use > ty->alloc_cpu_m) use = ty->alloc_cpu_m;
        }
        e_step += ty->idle_nw + ty->dyn_nw_per_m * use;
        if (nd->cap == 0) nsp++; else nod++;
        if (det) {
          det->pool_cost_uphmin[nd->pool] += o_price(e, r, h, nd->type, nd->zone, nd->cap);
          det->pool_energy_nwmin[nd->pool] += ty->idle_nw + ty->dyn_nw_per_m * use;
          pool_eh[nd->pool] += ty->idle_nw + ty->dyn_nw_per_m * use;
          if (nd->cap == 0) det->pool_node_min_spot[nd->pool]++; else det->pool_node_min_od[nd->pool]++;
        }
      }
      if (det) {
        det->base_cost_uphmin += (int64_t)w->base_nodes * o_price(e, r, h, w->base_type, 0, 1);
        det->base_energy_nwmin += base_nw;
        base_eh += base_nw;
        for (int p = 0; p < w->n_pools; ++p) {
          int cnt = 0;
          for (int n = 0; n < NN; ++n) cnt += st.nodes[n].used && st.nodes[n].pool == p;
          if (cnt > det->pool_peak_nodes[p]) det->pool_peak_nodes[p] = cnt;
        }
      }
      st.cost += cost;
      st.energy_nw += e_step;
      st.e_hour += e_step;
      int pending = 0, viol = 0, reps = 0;
      for (int d = 0; d < D; ++d) {
        pending += st.dep[d].replicas - ready_d[d];
        reps += st.dep[d].replicas;
        const ccka_deployment* dp = &w->deploy[d];
        if (dp->scaler == CCKA_SCALER_HPA && util_valid[d] && util[d] > w->slo_util_pct) viol = 1;
        if (dp->scaler == CCKA_SCALER_KEDA && keda_act[d] && st.dep[d].replicas == 0) viol = 1;
      }
      if (pending > 0) viol = 1;
      if (viol) { st.slo++; flags |= 8; }
      st.pend_min += pending;
      st.nmin_spot += nsp;
      st.nmin_od += nod;
      if (nsp + nod > st.peak_nodes) st.peak_nodes = nsp + nod;
      if (traj) {
        ccka_traj_rec* tr = &traj[(int64_t)t * nsc + i];
        tr->replicas = reps;
        tr->pending = pending;
        tr->nodes_spot = (uint16_t)nsp;
        tr->nodes_od = (uint16_t)nod;
        tr->last_type = step_last_type;
        tr->flags = flags;
      }
    }
  }
  if (feat) o_features(e, &st, load, nl, col, r, pswitch, w->n_steps, feat + ((int64_t)w->n_steps * nsc + i) * 64);
  if (prev_h >= 0) st.gco2 += (double)st.e_hour * (w->ci_gpwmin[r * 24 + prev_h] * 1e-9);
  if (det && prev_h >= 0) {
    for (int p = 0; p < w->n_pools; ++p) {
      det->pool_gco2[p] += (double)pool_eh[p] * (w->ci_gpwmin[r * 24 + prev_h] * 1e-9);
      int cnt = 0;
      for (int n = 0; n < NN; ++n) cnt += st.nodes[n].used && st.nodes[n].pool == p;
      det->pool_final_nodes[p] = cnt;
      det->pool_launches[p] = st.pool_launches[p];
    }
    det->base_gco2 += (double)base_eh * (w->ci_gpwmin[r * 24 + prev_h] * 1e-9);
    for (int d = 0; d < D; ++d) {
      int rd = 0;
      for (int n = 0; n < NN; ++n)
        if (st.nodes[n].used && st.nodes[n].ready_step <= w->n_steps - 1) rd += st.nodes[n].pods[d];
      det->desired[d] = st.dep[d].replicas;
      det->ready[d] = rd;
      det->pending[d] = st.dep[d].replicas - rd;
    }
  }
  int reps = 0, nodes = 0;
  for (int d = 0; d < D; ++d) reps += st.dep[d].replicas;
  for (int n = 0; n < NN; ++n) nodes += st.nodes[n].used;
  if (out->cost_uphmin) out->cost_uphmin[i] = st.cost;
  if (out->energy_wmin) out->energy_wmin[i] = (double)st.energy_nw * 1e-9;
  if (out->gco2) out->gco2[i] = st.gco2;
  if (out->slo_minutes) out->slo_minutes[i] = st.slo;
  if (out->pending_pod_minutes) out->pending_pod_minutes[i] = st.pend_min;
  if (out->node_min_spot) out->node_min_spot[i] = st.nmin_spot;
  if (out->node_min_od) out->node_min_od[i] = st.nmin_od;
  if (out->launches) out->launches[i] = st.launches;
  if (out->deletions) out->deletions[i] = st.deletions;
  if (out->peak_nodes) out->peak_nodes[i] = st.peak_nodes;
  if (out->final_replicas) out->final_replicas[i] = reps;
  if (out->final_nodes) out->final_nodes[i] = nodes;
  if (out->last_choice) out->last_choice[i] = st.last_choice;
  if (out->choice_hash) out->choice_hash[i] = st.hash;
}

typedef struct {
  const o_env* e;
  const ccka_scenarios* sc;
  const int32_t* load;
  ccka_results* out;
  ccka_traj_rec* traj;
  ccka_detail* detail;
  const int16_t* act_t;
  const double* act_cw;
  uint16_t* feat;
  int64_t lo, hi;
} o_job;

static void* o_worker(void* arg) {
  o_job* j = (o_job*)arg;
  for (int64_t i = j->lo; i < j->hi; ++i) o_run_one(j->e, j->sc, j->load, i, j->sc->n, j->out, j->traj, j->detail ? &j->detail[i] : NULL, j->act_t,
                                                 j->act_cw, j->feat);
  return NULL;
}

int ccka_oracle_rollout(const ccka_world* w, const ccka_scenarios* sc, const int32_t* load,
                        ccka_results* out, ccka_traj_rec* traj, int32_t n_threads) {
  return ccka_oracle_rollout_policy(w, sc, load, out, traj, NULL, NULL, NULL, NULL, n_threads);
}

int ccka_oracle_rollout_detail(const ccka_world* w, const ccka_scenarios* sc, const int32_t* load,
                               ccka_results* out, ccka_traj_rec* traj, ccka_detail* detail, int32_t n_threads) {
  return ccka_oracle_rollout_policy(w, sc, load, out, traj, detail, NULL, NULL, NULL, n_threads);
}

int ccka_oracle_rollout_policy(const ccka_world* w, const ccka_scenarios* sc, const int32_t* load,
                               ccka_results* out, ccka_traj_rec* traj, ccka_detail* detail, const int16_t* act_target,
                               const double* act_cw, uint16_t* feat, int32_t n_threads) {
  if ((act_target == NULL) != (act_cw == NULL)) return CCKA_EINVAL;
  if (!w || !sc || !load || !out || w->n_deploy < 1 || w->n_deploy > CCKA_MAX_DEPLOY ||
      w->max_nodes < 1 || w->max_nodes > CCKA_MAX_NODES || w->n_types < 1 || w->n_zones < 1 ||
      w->n_zones > CCKA_MAX_ZONES || w->n_pools < 1 || w->n_pools > CCKA_MAX_POOLS)
    return CCKA_EINVAL;
  o_env e;
  e.w = w;
  e.T = w->n_steps;
  e.D = w->n_deploy;
  e.K = w->n_types;
  e.Z = w->n_zones;
  e.N = w->max_nodes;
  /* provisioning order: req_cpu desc, req_mem desc, index asc (insertion sort, stable) */
  for (int d = 0; d < e.D; ++d) e.prov[d] = d;
  for (int a = 1; a < e.D; ++a) {
    const int x = e.prov[a];
    int b = a - 1;
    while (b >= 0) {
      const ccka_deployment* P = &w->deploy[e.prov[b]];
      const ccka_deployment* X = &w->deploy[x];
      const int before = X->req_cpu_m > P->req_cpu_m ||
                         (X->req_cpu_m == P->req_cpu_m && X->req_mem_mi > P->req_mem_mi);
      if (!before) break;
      e.prov[b + 1] = e.prov[b];
      --b;
    }
    e.prov[b + 1] = x;
  }
  if (n_threads < 1) n_threads = 1;
  if ((int64_t)n_threads > sc->n) n_threads = (int32_t)(sc->n > 0 ? sc->n : 1);
  pthread_t th[256];
  o_job jobs[256];
  if (n_threads > 256) n_threads = 256;
  for (int k = 0; k < n_threads; ++k) {
    jobs[k].e = &e;
    jobs[k].sc = sc;
    jobs[k].load = load;
    jobs[k].out = out;
    jobs[k].traj = traj;
    jobs[k].detail = detail;
    jobs[k].act_t = act_target;
    jobs[k].act_cw = act_cw;
    jobs[k].feat = feat;
    jobs[k].lo = sc->n * k / n_threads;
    jobs[k].hi = sc->n * (k + 1) / n_threads;
  }
  if (n_threads == 1) {
    o_worker(&jobs[0]);
  } else {
    for (int k = 0; k < n_threads; ++k) pthread_create(&th[k], NULL, o_worker, &jobs[k]);
    for (int k = 0; k < n_threads; ++k) pthread_join(th[k], NULL);
  }
  return CCKA_OK;
}

/* a += b, flagging instead of wrapping */
static void o_add(int64_t* a, int64_t b, int* ovf) {
  int64_t r;
  if (__builtin_add_overflow(*a, b, &r)) *ovf = 1;
  *a = r;
}
/* llrint(x * scale), flagged when not representable */
static int64_t o_fix(double x, double scale, int* ovf) {
  const double y = x * scale;
  if (!(y > -9.2233720368547758e18 && y < 9.2233720368547758e18)) {
    *ovf = 1;
    return 0;
  }
  return llrint(y);
}

int ccka_oracle_totals(const ccka_results* r, int64_t n, ccka_totals* o) {
  int ovf = 0;
  memset(o, 0, sizeof *o);
  o->scenarios = n;
  for (int64_t i = 0; i < n; ++i) {
    o_add(&o->cost_uphmin, r->cost_uphmin[i], &ovf);
    o_add(&o->slo_minutes, r->slo_minutes[i], &ovf);
    o_add(&o->pending_pod_minutes, r->pending_pod_minutes[i], &ovf);
    o_add(&o->node_min_spot, r->node_min_spot[i], &ovf);
    o_add(&o->node_min_od, r->node_min_od[i], &ovf);
    o_add(&o->launches, r->launches[i], &ovf);
    o_add(&o->deletions, r->deletions[i], &ovf);
    /* fixed point, as the device totals: microwatt-minutes, micrograms */
    o_add(&o->energy_uwmin, o_fix(r->energy_wmin[i], 1e6, &ovf), &ovf);
    o_add(&o->gco2_ug, o_fix(r->gco2[i], 1e6, &ovf), &ovf);
  }
  o->energy_wmin = (double)o->energy_uwmin * 1e-6;
  o->gco2 = (double)o->gco2_ug * 1e-6;
  return ovf ? CCKA_EOVERFLOW : CCKA_OK;
}
