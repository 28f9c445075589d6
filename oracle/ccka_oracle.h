/*
 * ccka_oracle.h — TEST INFRASTRUCTURE. CPU restatement of docs/SEMANTICS.md.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library, and only as the checker / the timed CPU baseline. The
 * product (libccka.so, the ccka CLI) never links or calls it.
 *
 * Parity status: the decision rules restate upstream controllers the
 * reference drives but does not vendor (k8s 1.34 HPA, Karpenter 1.8.1, KEDA):
 * "parity unpinned" w.r.t. the reference, pinned by the known-answer tests in
 * tests/test_oracle_kat.py. The policy inputs are pinned by the payloads the
 * reference scripts emit (tests/golden/reference_capture/).
 */
#ifndef CCKA_ORACLE_H
#define CCKA_ORACLE_H
#include "../include/ccka.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Full rollout of sc->n scenarios. load is [T][D][sc->n]; traj (optional) is
 * [T][sc->n]. n_threads contiguous scenario shards (pthreads). */
int ccka_oracle_rollout(const ccka_world* w, const ccka_scenarios* sc, const int32_t* load,
                        ccka_results* out, ccka_traj_rec* traj, int32_t n_threads);

/* The same, also filling detail[sc->n] (ccka_detail, per pool / base group /
 * deployment) when detail is non-NULL. */
int ccka_oracle_rollout_detail(const ccka_world* w, const ccka_scenarios* sc, const int32_t* load,
                               ccka_results* out, ccka_traj_rec* traj, ccka_detail* detail, int32_t n_threads);

/* Closed-loop policy replay (SEMANTICS 5): act_target / act_cw ([T][sc->n])
 * set every step's HPA target utilisation and carbon weight; feat (optional,
 * [T + 1][sc->n][64] bf16) receives the policy features before every step and
 * after the last. */
int ccka_oracle_rollout_policy(const ccka_world* w, const ccka_scenarios* sc, const int32_t* load,
                               ccka_results* out, ccka_traj_rec* traj, ccka_detail* detail, const int16_t* act_target,
                               const double* act_cw, uint16_t* feat, int32_t n_threads);

/* Serial totals over results (fixed scenario order); CCKA_EOVERFLOW when a
 * fixed-point sum would leave int64. */
int ccka_oracle_totals(const ccka_results* r, int64_t n, ccka_totals* out);

/* HPA replica calculator, CPU utilisation target (SEMANTICS §3.C step 3).
 * Returns the proposal; *util_out = utilisation (or -1 if metrics missing). */
int32_t ccka_oracle_hpa_resource_proposal(int32_t cur, int32_t ready, int64_t usage_m,
                                          int32_t req_m, int32_t target_pct, double tol,
                                          int32_t* util_out);
/* KEDA AverageValue external-metric proposal (SEMANTICS §3.C KEDA). */
int32_t ccka_oracle_keda_proposal(int32_t cur, int64_t metric, int64_t threshold, double tol);
/* HPA behavior (stabilisation + rate limits) for one decision: history given as
 * recs/valid/deltas of the previous CCKA_HIST steps (index k = step t-1-k). */
int32_t ccka_oracle_hpa_behavior(int32_t cur, int32_t proposal, int32_t min_r, int32_t max_r,
                                 const ccka_hpa_rules* up, const ccka_hpa_rules* down,
                                 const int32_t* recs, const uint8_t* rec_valid,
                                 const int32_t* deltas);

/* The same with a decision history of n entries, entry k = the decision
 * (k + 1) * sync_s seconds ago (windows up to CCKA_HPA_MAX_WINDOW_S, up to
 * CCKA_HPA_MAX_POLICIES policies per direction). */
int32_t ccka_oracle_hpa_behavior_n(int32_t cur, int32_t proposal, int32_t min_r, int32_t max_r,
                                   const ccka_hpa_rules* up, const ccka_hpa_rules* down, int32_t sync_s,
                                   const int32_t* recs, const uint8_t* rec_valid, const int32_t* deltas, int32_t n);

/* Synthetic traces (SEMANTICS §4): out is [T][D][n]. */
void ccka_oracle_sin_table(int32_t* out1440);
void ccka_oracle_gen_load(const ccka_trace_gen* g, int32_t T, int32_t D, int64_t n,
                          int64_t first_id, int32_t* out);
/* Philox-4x32-10 block, exposed for cross-checks. */
void ccka_oracle_philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                        uint32_t k0, uint32_t k1, uint32_t* out4);

#ifdef __cplusplus
}
#endif
#endif
