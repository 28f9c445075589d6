/*
 * ccka_host.h — C ABI of libccka_host.so: the manifest-in / summary-out side
 * of the drop-in (no GPU needed).
 *
 * It replaces the kubectl round-trips of the reference's decision path:
 *   ccka_host_apply         `kubectl apply -f`            demo_30_burst_configure.sh:143,
 *                                                          demo_10_setup_configure.sh (PDB, RBAC)
 *   ccka_host_patch         `kubectl patch --type=merge|json`
 *                                                          demo_20_offpeak_configure.sh:59-60,96;
 *                                                          demo_21_peak_configure.sh:56-57,88;
 *                                                          demo_19_reset_policies.sh:68-75
 *   ccka_host_get_json      `kubectl get nodepool -o json` (the read-back of apply_and_verify,
 *                                                          demo_20_offpeak_configure.sh:102)
 *   ccka_host_policy_patch  write_req_patch + the merge patches (demo_20 :59-81, demo_21 :56-77,
 *                           demo_19 :68-75), byte-identical to what the scripts send
 *   ccka_host_burst_manifest demo_30_burst_configure.sh:78-141 heredoc, byte-identical
 *   ccka_host_build_world   the stored objects -> ccka_world for libccka (ccka.h)
 *   ccka_host_label         `kubectl label nodepool ... --overwrite` (demo_10_setup_configure.sh:61-62)
 *   ccka_host_summary       the missing demo_41_observe_cost_nodes.sh (README.md:57)
 * Environment names follow the scripts: NP_SPOT, NP_OD, OFFPEAK_ZONES,
 * PEAK_ZONES, NAMESPACE, COUNT, REPLICAS (demo_00_env.sh, demo_30 :7-8),
 * with the same ${VAR:-default} rules, read at ccka_host_open.
 *
 * Strings out: the call writes at most `cap` bytes including the NUL and
 * returns the length written (>= 0), or a negative ccka_status.
 */
#ifndef CCKA_HOST_H
#define CCKA_HOST_H

#include <stdint.h>

#include "ccka.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ccka_host ccka_host;

int ccka_host_open(ccka_host** out);
void ccka_host_close(ccka_host* h);
const char* ccka_host_last_error(const ccka_host* h);

int ccka_host_apply(ccka_host* h, const char* yaml);
int ccka_host_patch(ccka_host* h, const char* kind, const char* name, const char* type,
                    const char* patch);
int ccka_host_get_json(ccka_host* h, const char* kind, const char* name, char* out, int64_t cap);

/* Kyverno guard policies of 04_kyverno.sh:24-75 (enforce mode, auto-gen for
 * pod controllers) as an admission pre-filter on ccka_host_apply: a denied
 * document is not stored and apply returns CCKA_EINVAL with kubectl's denial
 * text in ccka_host_last_error (the admitted documents of the same call are
 * stored). Off by default: the reference disables the stage (README.md:42). */
#define CCKA_ADMIT_REQUIRE_REQUESTS_LIMITS 1u /* require-requests-limits      :24-42 */
#define CCKA_ADMIT_CRITICAL_NO_SPOT 2u        /* critical-no-spot-without-pdb :44-72 */
int ccka_host_set_admission(ccka_host* h, uint32_t policies);
/* dry run: JSON array of {kind,name,policy,rule,message,path} violations of
 * every document in `yaml` under `policies`; length written (excl. NUL) */
int ccka_host_admission_review(ccka_host* h, uint32_t policies, const char* yaml, char* out, int64_t cap);

/* profile: CCKA_PROFILE_*; json_patch 0 -> the merge patch, 1 -> the
 * requirements JSON Patch (fallback 1: /spec/template path) */
int ccka_host_policy_patch(ccka_host* h, int32_t profile, const char* pool, int32_t json_patch,
                           int32_t fallback, char* out, int64_t cap);
/* index >= 1: that Deployment; 0: the PodDisruptionBudget; -1: the base NodePools */
int ccka_host_burst_manifest(ccka_host* h, int32_t index, char* out, int64_t cap);

/* catalog: "tiny" (12 types) or "small" (16). The world's array pointers
 * stay valid until the next build or ccka_host_close. */
int ccka_host_build_world(ccka_host* h, const char* catalog, int32_t n_steps, int32_t max_nodes,
                          ccka_world* out);
/* kubectl label <kind> <name> <labels> [--overwrite]: labels is a
 * whitespace-separated list of "key=value" (set) and "key-" (remove); a key
 * that already holds a different value fails unless overwrite (kubectl's
 * message). The reference labels its NodePools carbon.simulated=low|medium and
 * autoscale.strategy=cost|slo "for grouping in OpenCost/dashboards"; the world
 * builder carries them as each pool's group in the summary and export. */
int ccka_host_label(ccka_host* h, const char* kind, const char* name, const char* labels, int32_t overwrite);

/* demo_41-style summary of scenario 0 (results arrays of length >= 1; traj and
 * detail may be NULL). Sections: the NodePools' disruption settings and
 * requirements at the last step (demo_20_offpeak_observe.sh:9-20 views) with
 * their labels; the Deployments as NAME READY DESIRED CAPACITY
 * (demo_30_burst_observe.sh:10-11 custom columns); nodes; with detail, cost /
 * energy / gCO2 / node-minutes per NodePool and the base node group, and per
 * carbon.simulated group; run totals. */
int ccka_host_summary(ccka_host* h, const ccka_world* w, const ccka_results* r,
                      const ccka_traj_rec* traj, const ccka_detail* detail, char* out, int64_t cap);

/* Trajectory export, the downstream wire format of the reference's observe
 * path (kube-state-metrics scraped into Prometheus/AMP for Grafana and
 * OpenCost: 06_opencost.sh:318-341,404-432, demo_40_watch_config.sh:51-72).
 * Scenarios [s0, s0 + n) of a trajectory laid out [n_steps][traj_n] and of
 * results arrays indexed by scenario (global id = first_id + scenario).
 *   CCKA_EXPORT_PROMETHEUS: text exposition format, one sample per step at
 *     start_unix_ms + 60000 t: kube_deployment_spec_replicas,
 *     kube_deployment_status_replicas_available / _unavailable, ccka_nodes
 *     {capacity_type}, ccka_policy_profile, ccka_step_event{event}; run
 *     totals at the last step (cost, energy, carbon, SLO minutes, pending
 *     pod-minutes, node-minutes, launches, deletions) and the OpenCost-style
 *     allocation ccka_pod_cost_dollars_per_hour = cost / available pod-hours.
 *   CCKA_EXPORT_CSV: scenario,step,minute,replicas,pending,nodes_spot,
 *     nodes_od,last_type,flags.
 * *needed = bytes required including the terminating NUL; CCKA_EINVAL (with
 * *needed set) when out is NULL or cap is smaller. */
enum { CCKA_EXPORT_PROMETHEUS = 1, CCKA_EXPORT_CSV = 2 };
int ccka_host_export(ccka_host* h, int32_t format, const ccka_world* w, const ccka_traj_rec* traj,
                     int64_t traj_n, const ccka_results* r, int64_t s0, int64_t n, int64_t first_id,
                     int64_t start_unix_ms, char* out, int64_t cap, int64_t* needed);
/* Prometheus text of the per-pool breakdown of detail[0..n) at the last
 * step: ccka_nodepool_{cost_dollars,energy_kwh,carbon_grams,launches}_total,
 * ccka_nodepool_nodes, ccka_nodepool_node_minutes_total{capacity_type}, each
 * labelled nodepool / carbon_simulated / autoscale_strategy (the base managed
 * node group as nodepool="base-managed"), and
 * kube_deployment_status_replicas_ready. Buffer rules as ccka_host_export. */
int ccka_host_export_detail(ccka_host* h, const ccka_world* w, const ccka_detail* detail, int64_t n,
                            int64_t first_id, int64_t start_unix_ms, char* out, int64_t cap, int64_t* needed);

#ifdef __cplusplus
}
#endif
#endif
