// host_abi.cpp — C ABI of libccka_host.so (include/ccka_host.h).
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <exception>
#include <string>

#include "../../include/ccka_host.h"
#include "admission.h"
#include "model.h"
#include "policy.h"

using namespace ccka::host;

// printf-style append of any length (no fixed line buffer: long names are
// never truncated)
static void appendf(std::string& o, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
static void appendf(std::string& o, const char* fmt, ...) {
  char b[256];
  va_list ap;
  va_start(ap, fmt);
  const int n = std::vsnprintf(b, sizeof b, fmt, ap);
  va_end(ap);
  if (n < 0) return;
  if ((size_t)n < sizeof b) {
    o.append(b, (size_t)n);
    return;
  }
  const size_t at = o.size();
  o.resize(at + (size_t)n + 1);
  va_start(ap, fmt);
  std::vsnprintf(&o[at], (size_t)n + 1, fmt, ap);
  va_end(ap);
  o.resize(at + (size_t)n);
}

// Prometheus text exposition label value: backslash, double quote and line
// feed escaped (exposition format 0.0.4)
static std::string prom_esc(const std::string& v) {
  std::string r;
  r.reserve(v.size());
  for (char ch : v) {
    if (ch == '\\') r += "\\\\";
    else if (ch == '"') r += "\\\"";
    else if (ch == '\n') r += "\\n";
    else r += ch;
  }
  return r;
}

struct ccka_host {
  PolicyEnv env;
  ManifestStore store;
  Tables tables;
  WorldMeta meta;
  std::string err;
  uint32_t admission = 0;  // Kyverno policies enforced at apply (CCKA_ADMIT_*)
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
  return guarded(h, [&] { h->store.apply(yaml ? yaml : "", h->admission); return CCKA_OK; });
}

int ccka_host_set_admission(ccka_host* h, uint32_t policies) {
  return guarded(h, [&] {
    if (policies & ~(uint32_t)(CCKA_ADMIT_REQUIRE_REQUESTS_LIMITS | CCKA_ADMIT_CRITICAL_NO_SPOT)) {
      h->err = "unknown admission policy bits";
      return (int)CCKA_EINVAL;
    }
    h->admission = policies;
    return (int)CCKA_OK;
  });
}

int ccka_host_admission_review(ccka_host* h, uint32_t policies, const char* yaml, char* out, int64_t cap) {
  return guarded(h, [&] {
    Value arr = Value::array();
    for (const Value& doc : parse_yaml_documents(yaml ? yaml : "")) {
      if (!doc.is_map()) continue;
      for (const Violation& v : admission_review(doc, policies)) {
        Value o = Value::object();
        const Value* k = doc.get("kind");
        const Value* n = doc.at({"metadata", "name"});
        o.set("kind", Value::str(k ? k->as_string() : ""));
        o.set("name", Value::str(n ? n->as_string() : ""));
        o.set("policy", Value::str(v.policy));
        o.set("rule", Value::str(v.rule));
        o.set("message", Value::str(v.message));
        o.set("path", Value::str(v.path));
        arr.seq.push_back(o);
      }
    }
    return put(h, to_json(arr), out, cap);
  });
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

int ccka_host_label(ccka_host* h, const char* kind, const char* name, const char* labels, int32_t overwrite) {
  return guarded(h, [&] {
    if (!kind || !name || !labels) return (int)CCKA_EINVAL;
    h->store.label(kind, name, labels, overwrite != 0);
    return (int)CCKA_OK;
  });
}

// NodePool disruption / requirements as configured at the run's last step:
// the pool as created, the RESET profile (consolidateAfter per scenario 0),
// then the peak or off-peak profile in force (merge semantics, SEMANTICS 3.A)
static ccka_pool_patch pool_at_end(const ccka_world* w, int q, bool peak) {
  ccka_pool_patch cur = w->pools[q].base;
  ccka_pool_patch rp = w->pools[q].profile[CCKA_PROFILE_RESET];
  if (rp.consolidate_after_s >= 0) rp.consolidate_after_s = w->reset_ca_s;
  const ccka_pool_patch* steps[2] = {&rp, &w->pools[q].profile[peak ? CCKA_PROFILE_PEAK : CCKA_PROFILE_OFFPEAK]};
  for (const ccka_pool_patch* x : steps) {
    if (x->policy != CCKA_POLICY_KEEP) cur.policy = x->policy;
    if (x->consolidate_after_s >= 0) cur.consolidate_after_s = x->consolidate_after_s;
    if (x->zone_mask) cur.zone_mask = x->zone_mask;
    if (x->cap_mask) cur.cap_mask = x->cap_mask;
  }
  return cur;
}

static bool peak_at(const ccka_world* w, int t) {
  const int minute = (w->start_minute + t) % 1440, ps = w->peak_start_min, pe = w->peak_end_min;
  const bool in = ps <= pe ? (minute >= ps && minute < pe) : (minute >= ps || minute < pe);
  return w->peak_switch && in;
}

static std::string duration_text(int s) {
  if (s % 3600 == 0 && s) return std::to_string(s / 3600) + "h";
  if (s % 60 == 0 && s) return std::to_string(s / 60) + "m";
  return std::to_string(s) + "s";
}

int ccka_host_summary(ccka_host* h, const ccka_world* w, const ccka_results* r, const ccka_traj_rec* traj,
                      const ccka_detail* det, char* out, int64_t cap) {
  return guarded(h, [&] {
    if (!w || !r) return (int)CCKA_EINVAL;
    const WorldMeta& M = h->meta;
    auto pool_name = [&](int q) { return q < (int)M.pool_names.size() ? M.pool_names[(size_t)q] : std::string("?"); };
    auto label_or = [](const std::vector<std::string>& v, int i, const char* dflt) {
      return i < (int)v.size() && !v[(size_t)i].empty() ? v[(size_t)i] : std::string(dflt);
    };
    std::string s;
    const int T = w->n_steps;
    s += "# ccka summary: node pools, cost and carbon (demo_41_observe_cost_nodes)\n";
    appendf(s, "horizon: %d steps x %d s   pools: %d   deployments: %d   catalog: %d types\n\n",
                  T, CCKA_STEP_SECONDS, w->n_pools, w->n_deploy, w->n_types);
    // ---- NodePools: demo_20_offpeak_observe.sh:9-20 views at the last step
    const bool peak = traj ? (traj[T - 1].flags & 1u) != 0 : peak_at(w, T - 1);
    appendf(s, "[Observe] Disruption settings (last step, %s profile)\n", peak ? "peak" : "off-peak");
    for (int q = 0; q < w->n_pools; ++q) {
      const ccka_pool_patch e = pool_at_end(w, q, peak);
      appendf(s, "== %s ==\nconsolidationPolicy=%s  consolidateAfter=%s\n", pool_name(q).c_str(),
                    e.policy == CCKA_WHEN_EMPTY ? "WhenEmpty" : "WhenEmptyOrUnderutilized",
                    duration_text(e.consolidate_after_s).c_str());
      s += "topology.kubernetes.io/zone=In: ";
      for (int z = 0; z < w->n_zones; ++z)
        if (e.zone_mask >> z & 1u) s += M.zone_prefix + (char)('a' + z) + " ";
      s += "\nkarpenter.sh/capacity-type=In: ";
      if (e.cap_mask & CCKA_CAP_SPOT) s += "spot ";
      if (e.cap_mask & CCKA_CAP_OD) s += "on-demand ";
      appendf(s, "\nlabels: autoscale.strategy=%s carbon.simulated=%s   budget: nodes %d%%",
                    label_or(M.pool_strategy, q, "<none>").c_str(), label_or(M.pool_carbon, q, "<none>").c_str(),
                    w->pools[q].budget_pct);
      if (w->pools[q].limit_cpu_m >= 0) {
        appendf(s, "   limits: cpu %dm", w->pools[q].limit_cpu_m);
      }
      s += "\n";
    }
    // ---- Deployments: demo_30_burst_observe.sh:10-11 custom columns
    s += "\n# Summary of deployments (last step)\n";
    appendf(s, "%-24s %-7s %-8s %s\n", "NAME", "READY", "DESIRED", "CAPACITY");
    for (int d = 0; d < w->n_deploy; ++d) {
      if (w->deploy[d].scaler == CCKA_SCALER_KEDA_TRIGGER) continue;  // a trigger, not a Deployment
      const std::string nm = d < (int)M.deploy_names.size() ? M.deploy_names[(size_t)d] : "?";
      // kubectl omits status.readyReplicas at 0 -> "<none>"
      std::string ready = "<none>", desired = std::to_string(w->deploy[d].replicas0) + "*";
      if (det) {
        if (det->ready[d] > 0) ready = std::to_string(det->ready[d]);
        desired = std::to_string(det->desired[d]);
      }
      appendf(s, "%-24s %-7s %-8s %s\n", nm.c_str(), ready.c_str(), desired.c_str(),
                    label_or(M.deploy_capacity, d, "<none>").c_str());
    }
    if (!det) s += "(* manifest replicas: run with the detail breakdown for the rollout's values)\n";
    if (traj) {
      const ccka_traj_rec& last = traj[T - 1];
      appendf(s, "pods: desired=%d pending=%d   nodes: spot=%u on-demand=%u\n", last.replicas,
                    last.pending, last.nodes_spot, last.nodes_od);
    }
    // ---- nodes
    const uint32_t lc = r->last_choice ? r->last_choice[0] : 0xFFFFFFFFu;
    s += "\n# Nodes\n";
    appendf(s, "  node-minutes spot=%d on-demand=%d   peak nodes=%d   launches=%d deletions=%d\n",
                  r->node_min_spot[0], r->node_min_od[0], r->peak_nodes[0], r->launches[0], r->deletions[0]);
    if (lc != 0xFFFFFFFFu) {
      const int k = (int)(lc & 0xFFF), z = (int)((lc >> 12) & 3), c = (int)((lc >> 14) & 3), q = (int)(lc >> 16);
      appendf(s, "  last launch: %s zone=%s%c capacity=%s pool=%s\n",
                    k < (int)h->tables.names.size() ? h->tables.names[(size_t)k].c_str() : "?", M.zone_prefix.c_str(),
                    'a' + z, c == 0 ? "spot" : "on-demand", pool_name(q).c_str());
    }
    // ---- cost and carbon by pool and by carbon.simulated group
    if (det) {
      s += "\n# Cost and carbon by node pool\n";
      appendf(s, "%-24s %-8s %10s %10s %15s %8s %11s %12s %12s\n", "NODEPOOL", "CARBON", "NODEMIN-S",
                    "NODEMIN-OD", "NODES(END/PEAK)", "LAUNCHES", "COST($)", "ENERGY(kWh)", "gCO2");
      std::vector<std::pair<std::string, double>> gcost, gkwh, gco2;
      auto add = [](std::vector<std::pair<std::string, double>>& v, const std::string& k, double x) {
        for (auto& e : v)
          if (e.first == k) { e.second += x; return; }
        v.push_back({k, x});
      };
      for (int q = 0; q < w->n_pools; ++q) {
        const std::string grp = label_or(M.pool_carbon, q, "<none>");
        const double usd = (double)det->pool_cost_uphmin[q] / 6e7, kwh = (double)det->pool_energy_nwmin[q] * 1e-9 / 6e4;
        appendf(s, "%-24s %-8s %10d %10d %15s %8d %11.4f %12.4f %12.2f\n", pool_name(q).c_str(),
                      grp.c_str(), det->pool_node_min_spot[q], det->pool_node_min_od[q],
                      (std::to_string(det->pool_final_nodes[q]) + "/" + std::to_string(det->pool_peak_nodes[q])).c_str(),
                      det->pool_launches[q], usd, kwh, det->pool_gco2[q]);
        add(gcost, grp, usd);
        add(gkwh, grp, kwh);
        add(gco2, grp, det->pool_gco2[q]);
      }
      const double busd = (double)det->base_cost_uphmin / 6e7, bkwh = (double)det->base_energy_nwmin * 1e-9 / 6e4;
      appendf(s, "%-24s %-8s %10s %10d %15s %8s %11.4f %12.4f %12.2f\n", "(base managed nodes)", "<none>",
                    "-", w->base_nodes * T, (std::to_string(w->base_nodes) + "/" + std::to_string(w->base_nodes)).c_str(),
                    "-", busd, bkwh, det->base_gco2);
      add(gcost, "<none>", busd);
      add(gkwh, "<none>", bkwh);
      add(gco2, "<none>", det->base_gco2);
      s += "\n# By carbon.simulated group (demo_10_setup_configure.sh:61-62 labels)\n";
      appendf(s, "%-10s %11s %12s %12s\n", "GROUP", "COST($)", "ENERGY(kWh)", "gCO2");
      for (size_t g = 0; g < gcost.size(); ++g) {
        appendf(s, "%-10s %11.4f %12.4f %12.2f\n", gcost[g].first.c_str(), gcost[g].second,
                      gkwh[g].second, gco2[g].second);
      }
    }
    s += "\n# Cost and carbon (run total)\n";
    appendf(s, "  cost=$%.4f   energy=%.4f kWh   carbon=%.2f gCO2\n", (double)r->cost_uphmin[0] / 6e7,
                  r->energy_wmin[0] / 6e4, r->gco2[0]);
    appendf(s, "  SLO violation minutes=%d   pending pod-minutes=%lld\n", r->slo_minutes[0],
                  (long long)r->pending_pod_minutes[0]);
    return put(h, s, out, cap);
  });
}

int ccka_host_export(ccka_host* h, int32_t format, const ccka_world* w, const ccka_traj_rec* traj,
                     int64_t traj_n, const ccka_results* r, int64_t s0, int64_t n, int64_t first_id,
                     int64_t start_unix_ms, char* out, int64_t cap, int64_t* needed) {
  return guarded(h, [&] {
    if (needed) *needed = 0;
    if (!w || !traj || !r || n < 0 || s0 < 0 || s0 + n > traj_n || w->n_steps < 1 ||
        (format != CCKA_EXPORT_PROMETHEUS && format != CCKA_EXPORT_CSV))
      return (int)CCKA_EINVAL;
    const int T = w->n_steps;
    const int start = ((w->start_minute % 1440) + 1440) % 1440;
    auto rec = [&](int t, int64_t s) -> const ccka_traj_rec& { return traj[(int64_t)t * traj_n + s0 + s]; };
    std::string o;
    if (format == CCKA_EXPORT_CSV) {
      o.reserve((size_t)(n * T * 40 + 128));
      o += "scenario,step,minute,replicas,pending,nodes_spot,nodes_od,last_type,flags\n";
      for (int64_t s = 0; s < n; ++s)
        for (int t = 0; t < T; ++t) {
          const ccka_traj_rec& x = rec(t, s);
          appendf(o, "%lld,%d,%d,%d,%d,%u,%u,%u,%u\n", (long long)(first_id + s0 + s), t,
                        (start + t) % 1440, x.replicas, x.pending, x.nodes_spot, x.nodes_od, x.last_type, x.flags);
        }
    } else {
      o.reserve((size_t)(n * T * 7 * 110 + 4096));
      const std::string ns = prom_esc(h->env.ns);
      const std::string dep = w->n_deploy == 1 && !h->meta.deploy_names.empty() ? prom_esc(h->meta.deploy_names[0])
                              : w->n_deploy == 1                                 ? std::string("deployment-0")
                                                                                 : std::string("all");
      auto family = [&](const char* name, const char* type, const char* help) {
        appendf(o, "# HELP %s %s\n# TYPE %s %s\n", name, help, name, type);
      };
      auto ts = [&](int t) { return (long long)(start_unix_ms + (int64_t)t * CCKA_STEP_SECONDS * 1000); };
      auto dep_series = [&](const char* name, const char* type, const char* help, auto value) {
        family(name, type, help);
        for (int64_t s = 0; s < n; ++s)
          for (int t = 0; t < T; ++t) {
            appendf(o, "%s{namespace=\"%s\",deployment=\"%s\",scenario=\"%lld\"} %lld %lld\n", name,
                          ns.c_str(), dep.c_str(), (long long)(first_id + s0 + s), (long long)value(rec(t, s)), ts(t));
          }
      };
      dep_series("kube_deployment_spec_replicas", "gauge", "Number of desired pods for a deployment.",
                 [](const ccka_traj_rec& x) { return (long long)x.replicas; });
      dep_series("kube_deployment_status_replicas_available", "gauge",
                 "The number of available (running) replicas per deployment.",
                 [](const ccka_traj_rec& x) { return (long long)x.replicas - x.pending; });
      dep_series("kube_deployment_status_replicas_unavailable", "gauge",
                 "The number of unavailable (pending) replicas per deployment.",
                 [](const ccka_traj_rec& x) { return (long long)x.pending; });
      family("ccka_nodes", "gauge", "Karpenter nodes of the scenario by capacity type.");
      for (int c = 0; c < 2; ++c)
        for (int64_t s = 0; s < n; ++s)
          for (int t = 0; t < T; ++t) {
            const ccka_traj_rec& x = rec(t, s);
            appendf(o, "ccka_nodes{scenario=\"%lld\",capacity_type=\"%s\"} %u %lld\n",
                          (long long)(first_id + s0 + s), c == 0 ? "spot" : "on-demand",
                          c == 0 ? (unsigned)x.nodes_spot : (unsigned)x.nodes_od, ts(t));
          }
      family("ccka_policy_profile", "gauge", "1 while the peak NodePool profile is applied, 0 off-peak.");
      for (int64_t s = 0; s < n; ++s)
        for (int t = 0; t < T; ++t) {
          appendf(o, "ccka_policy_profile{scenario=\"%lld\"} %u %lld\n", (long long)(first_id + s0 + s),
                        rec(t, s).flags & 1u, ts(t));
        }
      family("ccka_step_event", "gauge", "1 when the step launched a node, deleted a node or violated the SLO.");
      static const char* ev[3] = {"launch", "deletion", "slo_violation"};
      for (int e = 0; e < 3; ++e)
        for (int64_t s = 0; s < n; ++s)
          for (int t = 0; t < T; ++t) {
            appendf(o, "ccka_step_event{scenario=\"%lld\",event=\"%s\"} %u %lld\n",
                          (long long)(first_id + s0 + s), ev[e], (rec(t, s).flags >> (e + 1)) & 1u, ts(t));
          }
      // run totals at the last step
      auto total = [&](const char* name, const char* type, const char* help, const char* extra, auto value) {
        family(name, type, help);
        for (int64_t s = 0; s < n; ++s) {
          appendf(o, "%s{scenario=\"%lld\"%s} %.17g %lld\n", name, (long long)(first_id + s0 + s), extra,
                        (double)value(s0 + s), ts(T - 1));
        }
      };
      if (r->cost_uphmin)
        total("ccka_cost_dollars_total", "counter", "Node cost of the run (cloud prices, per-minute billing).", "",
              [&](int64_t i) { return (double)r->cost_uphmin[i] / 6e7; });
      if (r->energy_wmin)
        total("ccka_energy_kwh_total", "counter", "Node energy of the run.", "",
              [&](int64_t i) { return r->energy_wmin[i] / 6e4; });
      if (r->gco2)
        total("ccka_carbon_grams_total", "counter", "Operational carbon of the run (hourly grid intensity).", "",
              [&](int64_t i) { return r->gco2[i]; });
      if (r->slo_minutes)
        total("ccka_slo_violation_minutes_total", "counter", "Minutes with pending pods or utilisation above the SLO.",
              "", [&](int64_t i) { return (double)r->slo_minutes[i]; });
      if (r->pending_pod_minutes)
        total("ccka_pending_pod_minutes_total", "counter", "Pending pod-minutes of the run.", "",
              [&](int64_t i) { return (double)r->pending_pod_minutes[i]; });
      if (r->node_min_spot && r->node_min_od) {
        family("ccka_node_minutes_total", "counter", "Karpenter node-minutes of the run by capacity type.");
        for (int c = 0; c < 2; ++c)
          for (int64_t s = 0; s < n; ++s) {
            appendf(o, "ccka_node_minutes_total{scenario=\"%lld\",capacity_type=\"%s\"} %d %lld\n",
                          (long long)(first_id + s0 + s), c == 0 ? "spot" : "on-demand",
                          c == 0 ? r->node_min_spot[s0 + s] : r->node_min_od[s0 + s], ts(T - 1));
          }
      }
      if (r->launches)
        total("ccka_launches_total", "counter", "NodeClaims launched.", "",
              [&](int64_t i) { return (double)r->launches[i]; });
      if (r->deletions)
        total("ccka_deletions_total", "counter", "Nodes removed by consolidation.", "",
              [&](int64_t i) { return (double)r->deletions[i]; });
      if (r->cost_uphmin) {
        // OpenCost-style allocation: the run's node cost over its running pod-hours
        family("ccka_pod_cost_dollars_per_hour", "gauge",
               "Node cost allocated per running pod-hour (cost / available pod-hours).");
        for (int64_t s = 0; s < n; ++s) {
          long long pod_min = 0;
          for (int t = 0; t < T; ++t) pod_min += (long long)rec(t, s).replicas - rec(t, s).pending;
          if (pod_min <= 0) continue;
          appendf(o,
                        "ccka_pod_cost_dollars_per_hour{namespace=\"%s\",deployment=\"%s\",scenario=\"%lld\"} %.17g %lld\n",
                        ns.c_str(), dep.c_str(), (long long)(first_id + s0 + s),
                        ((double)r->cost_uphmin[s0 + s] / 6e7) / ((double)pod_min / 60.0), ts(T - 1));
        }
      }
    }
    if (needed) *needed = (int64_t)o.size() + 1;
    if (!out || (int64_t)o.size() + 1 > cap) {
      h->err = "output buffer too small: need " + std::to_string(o.size() + 1);
      return (int)CCKA_EINVAL;
    }
    std::memcpy(out, o.data(), o.size());
    out[o.size()] = 0;
    return (int)CCKA_OK;
  });
}

int ccka_host_export_detail(ccka_host* h, const ccka_world* w, const ccka_detail* det, int64_t n, int64_t first_id,
                            int64_t start_unix_ms, char* out, int64_t cap, int64_t* needed) {
  return guarded(h, [&] {
    if (needed) *needed = 0;
    if (!w || !det || n < 0 || w->n_steps < 1) return (int)CCKA_EINVAL;
    const WorldMeta& M = h->meta;
    const long long ts = (long long)(start_unix_ms + (int64_t)(w->n_steps - 1) * CCKA_STEP_SECONDS * 1000);
    std::string o;
    auto family = [&](const char* name, const char* type, const char* help) {
      appendf(o, "# HELP %s %s\n# TYPE %s %s\n", name, help, name, type);
    };
    auto lab = [&](const std::vector<std::string>& v, int q) { return q < (int)v.size() ? prom_esc(v[(size_t)q]) : std::string(); };
    // one sample per (scenario, group); group P = the base managed node group
    auto pool_series = [&](const char* name, const char* type, const char* help, auto value) {
      family(name, type, help);
      for (int64_t s = 0; s < n; ++s)
        for (int q = 0; q <= w->n_pools; ++q) {
          const bool base = q == w->n_pools;
          const std::string np = base ? std::string("base-managed") : (q < (int)M.pool_names.size() ? prom_esc(M.pool_names[(size_t)q]) : "?");
          appendf(o,
                        "%s{scenario=\"%lld\",nodepool=\"%s\",carbon_simulated=\"%s\",autoscale_strategy=\"%s\"} %.17g %lld\n",
                        name, (long long)(first_id + s), np.c_str(), base ? "" : lab(M.pool_carbon, q).c_str(),
                        base ? "" : lab(M.pool_strategy, q).c_str(), value(det[s], q, base), ts);
        }
    };
    pool_series("ccka_nodepool_cost_dollars_total", "counter", "Node cost of the run per NodePool (base: managed node group).",
                [](const ccka_detail& d, int q, bool base) { return (double)(base ? d.base_cost_uphmin : d.pool_cost_uphmin[q]) / 6e7; });
    pool_series("ccka_nodepool_energy_kwh_total", "counter", "Node energy of the run per NodePool.",
                [](const ccka_detail& d, int q, bool base) {
                  return (double)(base ? d.base_energy_nwmin : d.pool_energy_nwmin[q]) * 1e-9 / 6e4;
                });
    pool_series("ccka_nodepool_carbon_grams_total", "counter", "Operational carbon of the run per NodePool.",
                [](const ccka_detail& d, int q, bool base) { return base ? d.base_gco2 : d.pool_gco2[q]; });
    pool_series("ccka_nodepool_nodes", "gauge", "Nodes of the NodePool at the last step.",
                [&](const ccka_detail& d, int q, bool base) { return (double)(base ? w->base_nodes : d.pool_final_nodes[q]); });
    pool_series("ccka_nodepool_launches_total", "counter", "NodeClaims launched per NodePool.",
                [](const ccka_detail& d, int q, bool base) { return base ? 0.0 : (double)d.pool_launches[q]; });
    family("ccka_nodepool_node_minutes_total", "counter", "Karpenter node-minutes per NodePool and capacity type.");
    for (int64_t s = 0; s < n; ++s)
      for (int q = 0; q < w->n_pools; ++q)
        for (int c = 0; c < 2; ++c) {
          appendf(o,
                        "ccka_nodepool_node_minutes_total{scenario=\"%lld\",nodepool=\"%s\",carbon_simulated=\"%s\","
                        "capacity_type=\"%s\"} %d %lld\n",
                        (long long)(first_id + s), q < (int)M.pool_names.size() ? prom_esc(M.pool_names[(size_t)q]).c_str() : "?",
                        lab(M.pool_carbon, q).c_str(), c == 0 ? "spot" : "on-demand",
                        c == 0 ? det[s].pool_node_min_spot[q] : det[s].pool_node_min_od[q], ts);
        }
    family("kube_deployment_status_replicas_ready", "gauge", "The number of ready replicas per deployment (last step).");
    for (int64_t s = 0; s < n; ++s)
      for (int d = 0; d < w->n_deploy; ++d) {
        if (w->deploy[d].scaler == CCKA_SCALER_KEDA_TRIGGER) continue;
        appendf(o, "kube_deployment_status_replicas_ready{namespace=\"%s\",deployment=\"%s\",scenario=\"%lld\"} %d %lld\n",
                      prom_esc(h->env.ns).c_str(), d < (int)M.deploy_names.size() ? prom_esc(M.deploy_names[(size_t)d]).c_str() : "?",
                      (long long)(first_id + s), det[s].ready[d], ts);
      }
    if (needed) *needed = (int64_t)o.size() + 1;
    if (!out || (int64_t)o.size() + 1 > cap) {
      h->err = "output buffer too small: need " + std::to_string(o.size() + 1);
      return (int)CCKA_EINVAL;
    }
    std::memcpy(out, o.data(), o.size());
    out[o.size()] = 0;
    return (int)CCKA_OK;
  });
}

}  // extern "C"
