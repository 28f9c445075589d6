// host_abi.cpp — C ABI of libccka_host.so (include/ccka_host.h).
#include <cstdio>
#include <cstring>
#include <exception>
#include <string>

#include "../../include/ccka_host.h"
#include "model.h"
#include "policy.h"

using namespace ccka::host;

struct ccka_host {
  PolicyEnv env;
  ManifestStore store;
  Tables tables;
  WorldMeta meta;
  std::string err;
};

static int put(ccka_host* h, const std::string& s, char* out, int64_t cap) {
  if (!out || cap <= 0) return CCKA_EINVAL;
  if ((int64_t)s.size() + 1 > cap) {
    h->err = "output buffer too small: need " + std::to_string(s.size() + 1);
    return CCKA_EINVAL;
  }
  std::memcpy(out, s.data(), s.size());
  out[s.size()] = 0;
  return (int)s.size();
}

template <class F>
static int guarded(ccka_host* h, F&& f) {
  if (!h) return CCKA_EINVAL;
  try {
    return f();
  } catch (const std::exception& e) {
    h->err = e.what();
    return CCKA_EINVAL;
  }
}

extern "C" {

int ccka_host_open(ccka_host** out) {
  if (!out) return CCKA_EINVAL;
  *out = new (std::nothrow) ccka_host();
  if (!*out) return CCKA_ENOMEM;
  (*out)->env = PolicyEnv::from_environment();
  return CCKA_OK;
}

void ccka_host_close(ccka_host* h) { delete h; }

const char* ccka_host_last_error(const ccka_host* h) { return h ? h->err.c_str() : "null handle"; }

int ccka_host_apply(ccka_host* h, const char* yaml) {
  return guarded(h, [&] { h->store.apply(yaml ? yaml : ""); return CCKA_OK; });
}

int ccka_host_patch(ccka_host* h, const char* kind, const char* name, const char* type, const char* patch) {
  return guarded(h, [&] {
    if (!kind || !name || !type || !patch) return (int)CCKA_EINVAL;
    h->store.patch(kind, name, type, patch);
    return (int)CCKA_OK;
  });
}

int ccka_host_get_json(ccka_host* h, const char* kind, const char* name, char* out, int64_t cap) {
  return guarded(h, [&] {
    const Value* v = h->store.get(kind ? kind : "", name ? name : "");
    if (!v) { h->err = "not found"; return (int)CCKA_EINVAL; }
    return put(h, to_json(*v), out, cap);
  });
}

int ccka_host_policy_patch(ccka_host* h, int32_t profile, const char* pool, int32_t json_patch,
                           int32_t fallback, char* out, int64_t cap) {
  return guarded(h, [&] {
    if (profile < 0 || profile > 2 || !pool) return (int)CCKA_EINVAL;
    const Profile p = (Profile)profile;
    if (json_patch && p == Profile::Reset) { h->err = "reset sends no JSON patch"; return (int)CCKA_EINVAL; }
    return put(h, json_patch ? requirements_patch(p, h->env, pool, fallback != 0)
                             : disruption_merge_patch(p, h->env, pool), out, cap);
  });
}

int ccka_host_burst_manifest(ccka_host* h, int32_t index, char* out, int64_t cap) {
  return guarded(h, [&] {
    if (index >= 1) return put(h, burst_deployment_yaml(h->env, index), out, cap);
    if (index == 0) return put(h, pdb_yaml(h->env), out, cap);
    return put(h, default_nodepools_yaml(h->env), out, cap);
  });
}

int ccka_host_build_world(ccka_host* h, const char* catalog, int32_t n_steps, int32_t max_nodes,
                          ccka_world* out) {
  return guarded(h, [&] {
    if (!out || n_steps < 1 || max_nodes < 1 || max_nodes > CCKA_MAX_NODES) return (int)CCKA_EINVAL;
    h->tables = builtin_tables(catalog ? catalog : "tiny");
    h->meta = build_world(h->store, h->env, h->tables, n_steps, max_nodes, out);
    return (int)CCKA_OK;
  });
}

int ccka_host_summary(ccka_host* h, const ccka_world* w, const ccka_results* r,
                      const ccka_traj_rec* traj, char* out, int64_t cap) {
  return guarded(h, [&] {
    if (!w || !r) return (int)CCKA_EINVAL;
    std::string s;
    char b[512];
    const int T = w->n_steps;
    s += "# ccka summary: node pools, cost and carbon (demo_41_observe_cost_nodes)\n";
    std::snprintf(b, sizeof b, "horizon: %d steps x %d s   pools: %d   deployments: %d   catalog: %d types\n\n",
                  T, CCKA_STEP_SECONDS, w->n_pools, w->n_deploy, w->n_types);
    s += b;
    s += "# NodePools (Karpenter order)\n";
    for (int q = 0; q < w->n_pools; ++q) {
      const char* nm = q < (int)h->meta.pool_names.size() ? h->meta.pool_names[(size_t)q].c_str() : "?";
      std::snprintf(b, sizeof b, "  %-18s cap=%s%s zones=0x%x budget=%d%%\n", nm,
                    (w->pools[q].base.cap_mask & CCKA_CAP_SPOT) ? "spot," : "",
                    (w->pools[q].base.cap_mask & CCKA_CAP_OD) ? "on-demand" : "", w->pools[q].base.zone_mask,
                    w->pools[q].budget_pct);
      s += b;
    }
    if (traj) {
      const ccka_traj_rec& last = traj[T - 1];
      std::snprintf(b, sizeof b, "\n# Final step: replicas=%d pending=%d nodes spot=%u on-demand=%u\n",
                    last.replicas, last.pending, last.nodes_spot, last.nodes_od);
      s += b;
    }
    s += "\n# Deployments (NAME DESIRED CAPACITY)\n";
    for (int d = 0; d < w->n_deploy; ++d) {
      const char* nm = d < (int)h->meta.deploy_names.size() ? h->meta.deploy_names[(size_t)d].c_str() : "?";
      const uint32_t c = w->deploy[d].cap_sel;
      std::snprintf(b, sizeof b, "  %-18s %-5d %s\n", nm, w->deploy[d].replicas0,
                    c == CCKA_CAP_SPOT ? "spot" : c == CCKA_CAP_OD ? "on-demand" : "any");
      s += b;
    }
    const uint32_t lc = r->last_choice ? r->last_choice[0] : 0xFFFFFFFFu;
    s += "\n# Nodes\n";
    std::snprintf(b, sizeof b, "  node-minutes spot=%d on-demand=%d   peak nodes=%d   launches=%d deletions=%d\n",
                  r->node_min_spot[0], r->node_min_od[0], r->peak_nodes[0], r->launches[0], r->deletions[0]);
    s += b;
    if (lc != 0xFFFFFFFFu) {
      const int k = (int)(lc & 0xFFF), z = (int)((lc >> 12) & 3), c = (int)((lc >> 14) & 3), q = (int)(lc >> 16);
      std::snprintf(b, sizeof b, "  last launch: %s zone=%c capacity=%s pool=%s\n",
                    k < (int)h->tables.names.size() ? h->tables.names[(size_t)k].c_str() : "?", 'a' + z,
                    c == 0 ? "spot" : "on-demand",
                    q < (int)h->meta.pool_names.size() ? h->meta.pool_names[(size_t)q].c_str() : "?");
      s += b;
    }
    s += "\n# Cost and carbon\n";
    std::snprintf(b, sizeof b, "  cost=$%.4f   energy=%.4f kWh   carbon=%.2f gCO2\n", (double)r->cost_uphmin[0] / 6e7,
                  r->energy_wmin[0] / 6e4, r->gco2[0]);
    s += b;
    std::snprintf(b, sizeof b, "  SLO violation minutes=%d   pending pod-minutes=%lld\n", r->slo_minutes[0],
                  (long long)r->pending_pod_minutes[0]);
    s += b;
    return put(h, s, out, cap);
  });
}

}  // extern "C"
