// model.cpp — see model.h.
#include "model.h"

#include "admission.h"

#include <algorithm>
#include <cmath>
#include <cstring>

namespace ccka::host {

// ------------------------------------------------------------------ store
static std::string kind_of(const Value& v) { return v.get("kind") ? v.get("kind")->as_string() : ""; }
static std::string name_of(const Value& v) {
  const Value* n = v.at({"metadata", "name"});
  return n ? n->as_string() : "";
}

Value* ManifestStore::find(const std::string& kind, const std::string& name) {
  for (auto& o : objs_)
    if (kind_of(o) == kind && name_of(o) == name) return &o;
  return nullptr;
}

const Value* ManifestStore::get(const std::string& kind, const std::string& name) const {
  for (auto& o : objs_)
    if (kind_of(o) == kind && name_of(o) == name) return &o;
  return nullptr;
}

std::vector<const Value*> ManifestStore::all(const std::string& kind) const {
  std::vector<const Value*> out;
  for (auto& o : objs_)
    if (kind_of(o) == kind) out.push_back(&o);
  return out;
}

void ManifestStore::apply(const std::string& yaml_text, uint32_t admission) {
  std::string denied;
  for (auto& doc : parse_yaml_documents(yaml_text)) {
    if (!doc.is_map()) continue;
    const std::string k = kind_of(doc), n = name_of(doc);
    if (k.empty() || n.empty()) throw ParseError("apply: document without kind/metadata.name");
    const std::vector<Violation> v = admission_review(doc, admission);
    if (!v.empty()) {
      denied += (denied.empty() ? "" : "\n") + ("Error from server: error when creating \"" + n + "\": ") +
                denial_message(doc, v);
      continue;
    }
    if (Value* cur = find(k, n)) *cur = doc;
    else objs_.push_back(doc);
  }
  if (!denied.empty()) throw ParseError(denied);
}

void ManifestStore::patch(const std::string& kind, const std::string& name, const std::string& type,
                          const std::string& text) {
  Value* o = find(kind, name);
  if (!o) throw ParseError("Error from server (NotFound): " + kind + " \"" + name + "\" not found");
  const Value p = parse_json(text);
  Value copy = *o;  // kubectl patches are atomic
  if (type == "merge") apply_merge_patch(copy, p);
  else if (type == "json") apply_json_patch(copy, p);
  else throw ParseError("patch type must be merge or json");
  *o = std::move(copy);
}

// apimachinery validation (IsQualifiedName / IsValidLabelValue): a name is
// at most 63 characters of [A-Za-z0-9._-], alphanumeric at both ends; a key
// is an optional DNS-subdomain prefix (<= 253 characters, lowercase
// alphanumerics, '-' and '.') and '/' before such a name; a value is empty or
// such a name
static bool label_name_ok(const std::string& v) {
  if (v.empty() || v.size() > 63) return false;
  auto alnum = [](char c) { return std::isalnum((unsigned char)c) != 0; };
  if (!alnum(v.front()) || !alnum(v.back())) return false;
  for (char c : v)
    if (!alnum(c) && c != '-' && c != '_' && c != '.') return false;
  return true;
}
static bool label_key_ok(const std::string& k) {
  const size_t sl = k.find('/');
  if (sl == std::string::npos) return label_name_ok(k);
  const std::string pre = k.substr(0, sl), nm = k.substr(sl + 1);
  if (pre.empty() || pre.size() > 253 || !label_name_ok(nm)) return false;
  for (char c : pre)
    if (!(std::islower((unsigned char)c) || std::isdigit((unsigned char)c) || c == '-' || c == '.')) return false;
  return std::isalnum((unsigned char)pre.front()) && std::isalnum((unsigned char)pre.back());
}

void ManifestStore::label(const std::string& kind, const std::string& name, const std::string& labels,
                          bool overwrite) {
  Value* o = find(kind, name);
  if (!o) throw ParseError("Error from server (NotFound): " + kind + " \"" + name + "\" not found");
  Value copy = *o;
  Value* md = copy.get("metadata");
  if (!md || !md->is_map()) throw ParseError("label: object without metadata");
  Value* ls = md->get("labels");
  if (!ls) ls = &md->set("labels", Value::object());
  if (!ls->is_map()) throw ParseError("label: metadata.labels is not a map");
  size_t i = 0;
  int n = 0;
  while (i < labels.size()) {
    while (i < labels.size() && std::isspace((unsigned char)labels[i])) ++i;
    size_t j = i;
    while (j < labels.size() && !std::isspace((unsigned char)labels[j])) ++j;
    if (j == i) break;
    const std::string tok = labels.substr(i, j - i);
    i = j;
    ++n;
    const size_t eq = tok.find('=');
    if (eq == std::string::npos) {
      if (tok.size() < 2 || tok.back() != '-') throw ParseError("error: at least one label update is required");
      ls->erase(tok.substr(0, tok.size() - 1));
      continue;
    }
    const std::string key = tok.substr(0, eq), val = tok.substr(eq + 1);
    if (key.empty()) throw ParseError("error: invalid label spec: " + tok);
    if (!label_key_ok(key) || !(val.empty() || label_name_ok(val)))
      throw ParseError("error: invalid label spec: " + tok +
                       " (keys and values: <= 63 characters of [A-Za-z0-9._-], alphanumeric at both ends)");
    if (const Value* cur = ls->get(key); cur && cur->as_string() != val && !overwrite)
      throw ParseError("error: '" + key + "' already has a value (" + cur->as_string() +
                       "), and --overwrite is false");
    ls->set(key, Value::str(val));
  }
  if (!n) throw ParseError("error: at least one label update is required");
  *o = std::move(copy);
}

// ------------------------------------------------------------------ tables
int Tables::index(const std::string& n) const {
  for (size_t k = 0; k < names.size(); ++k)
    if (names[k] == n) return (int)k;
  return -1;
}

static uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ULL;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
  return x ^ (x >> 31);
}
static double unit(uint64_t h) { return (double)(h >> 11) * (1.0 / 9007199254740992.0); }

Tables builtin_tables(const std::string& which, double ci, uint64_t seed) {
  // {family, GiB per vCPU, $/h of .large in micro-dollars}
  struct Fam { const char* f; int gib; int64_t uph; };
  const Fam fams[] = {{"m6i", 4, 96000}, {"c6i", 2, 85000}, {"r6i", 8, 126000}, {"m7i", 4, 100800}};
  const struct { const char* s; int v; int pods; } sizes[] = {
      {"large", 2, 29}, {"xlarge", 4, 58}, {"2xlarge", 8, 58}, {"4xlarge", 16, 234}};
  const int nfam = which == "tiny" ? 3 : 4;
  if (which != "tiny" && which != "small") throw ParseError("unknown builtin catalog " + which);
  Tables T;
  T.regions = 1;
  T.zones = 3;
  std::vector<int64_t> od;
  for (int f = 0; f < nfam; ++f) {
    for (auto& sz : sizes) {
      T.names.push_back(std::string(fams[f].f) + "." + sz.s);
      ccka_itype t{};
      const int64_t v = sz.v;
      int64_t res = 60 + (v >= 2 ? 10 : 0) + std::min<int64_t>(std::max<int64_t>(v - 2, 0), 2) * 5 +
                    std::max<int64_t>(v - 4, 0) * 25 / 10;
      t.vcpu = (int32_t)v;
      t.alloc_cpu_m = (int32_t)(v * 1000 - res);
      const int64_t mem_mi = (int64_t)v * fams[f].gib * 1024;
      t.alloc_mem_mi = (int32_t)((mem_mi * 925) / 1000 - (11 * sz.pods + 255) - 100);
      t.max_pods = sz.pods;
      const double p_idle = (double)v * 0.74 * 1.135, p_dyn = (double)v * (3.5 - 0.74) * 1.135;
      t.idle_nw = std::llround(p_idle * 1e9);
      t.dyn_nw_per_m = std::llround(p_dyn * 1e9 / (double)t.alloc_cpu_m);
      t.p_ref_w = p_idle + 0.5 * p_dyn;
      t.mem_mi = (int32_t)mem_mi;
      T.types.push_back(t);
      od.push_back(fams[f].uph * v / 2);
    }
  }
  const int K = (int)T.types.size(), Z = T.zones;
  T.price.assign((size_t)24 * K * Z * 2, 0);
  for (int h = 0; h < 24; ++h)
    for (int k = 0; k < K; ++k)
      for (int z = 0; z < Z; ++z) {
        // spot = OD x U[0.25, 0.7] per (type, zone) x (1 +/- 10 %) per hour
        const double disc = 0.25 + 0.45 * unit(splitmix64(seed ^ ((uint64_t)k << 8) ^ (uint64_t)z));
        const double wig = 1.0 + 0.1 * (2.0 * unit(splitmix64(seed * 31 + (uint64_t)(h * 4096 + k * 8 + z))) - 1.0);
        const size_t base = (((size_t)h * K + k) * Z + z) * 2;
        T.price[base + 0] = (int32_t)std::llround((double)od[(size_t)k] * disc * wig);
        T.price[base + 1] = (int32_t)od[(size_t)k];
      }
  for (int h = 0; h < 24; ++h) {
    const double c = ci * (1.0 + 0.3 * std::sin(2.0 * M_PI * (h - 13) / 24.0));
    T.ci_gpwh.push_back(c / 1000.0);
    T.ci_gpwmin.push_back(c / 60000.0);
  }
  return T;
}

// ------------------------------------------------------------------ world
uint32_t zone_bit(const std::string& zone) {
  if (zone.empty()) return 0;
  const char c = zone.back();
  if (c < 'a' || c > 'd') throw ParseError("zone " + zone + " outside the a..d range");
  return 1u << (c - 'a');
}

std::string default_nodepools_yaml(const PolicyEnv& env) {
  auto pool = [](const std::string& name, const char* caps) {
    return "apiVersion: karpenter.sh/v1\nkind: NodePool\nmetadata:\n  name: " + name +
           "\nspec:\n  template:\n    spec:\n      nodeClassRef:\n        group: karpenter.k8s.aws\n"
           "        kind: EC2NodeClass\n        name: default-class\n      requirements:\n"
           "        - key: topology.kubernetes.io/zone\n          operator: In\n"
           "          values: [\"us-east-2a\", \"us-east-2b\", \"us-east-2c\"]\n"
           "        - key: karpenter.sh/capacity-type\n          operator: In\n          values: " +
           std::string(caps) +
           "\n  disruption:\n    consolidationPolicy: WhenEmptyOrUnderutilized\n    consolidateAfter: 0s\n"
           "    budgets:\n      - nodes: \"10%\"\n";
  };
  return pool(env.np_spot, "[\"spot\", \"on-demand\"]") + "---\n" + pool(env.np_od, "[\"on-demand\"]");
}

static int policy_code(const std::string& s) {
  if (s == "WhenEmpty") return CCKA_WHEN_EMPTY;
  if (s == "WhenEmptyOrUnderutilized") return CCKA_WHEN_EMPTY_OR_UNDERUTILIZED;
  throw ParseError("unknown consolidationPolicy " + s);
}

static thread_local std::string g_zone_prefix_seen;  // region prefix of the last zone name parsed (summary names)

static void requirements_masks(const Value* reqs, uint32_t* zm, uint32_t* cm) {
  if (!reqs || !reqs->is_seq()) return;
  for (auto& r : reqs->seq) {
    const std::string key = r.get("key") ? r.get("key")->as_string() : "";
    const std::string op = r.get("operator") ? r.get("operator")->as_string() : "";
    const Value* vals = r.get("values");
    if (op != "In" || !vals || !vals->is_seq()) continue;
    uint32_t m = 0;
    for (auto& v : vals->seq) {
      const std::string s = v.as_string();
      if (key == "topology.kubernetes.io/zone") {
        m |= zone_bit(s);
        if (!s.empty()) g_zone_prefix_seen = s.substr(0, s.size() - 1);
      }
      else if (key == "karpenter.sh/capacity-type") m |= s == "spot" ? CCKA_CAP_SPOT : s == "on-demand" ? CCKA_CAP_OD : 0;
    }
    if (key == "topology.kubernetes.io/zone") *zm = m;
    if (key == "karpenter.sh/capacity-type") *cm = m;
  }
}

static ccka_pool_patch patch_from(const std::string& merge, const std::string& json) {
  ccka_pool_patch p{CCKA_POLICY_KEEP, -1, 0, 0};
  if (!merge.empty()) {
    const Value m = parse_json(merge);
    if (const Value* pol = m.at({"spec", "disruption", "consolidationPolicy"})) p.policy = policy_code(pol->as_string());
    if (const Value* ca = m.at({"spec", "disruption", "consolidateAfter"})) p.consolidate_after_s = (int32_t)duration_s(ca->as_string());
  }
  if (!json.empty()) {
    const Value j = parse_json(json);
    for (auto& op : j.seq)
      if (const Value* v = op.get("value")) requirements_masks(v, &p.zone_mask, &p.cap_mask);
  }
  return p;
}

static ccka_hpa_rules rules_from(const Value* b, bool up, int default_stab) {
  ccka_hpa_rules r{};
  r.select = CCKA_SELECT_MAX;
  r.stab_window_s = default_stab;
  if (up) {  // autoscaling/v2 defaults
    r.n_policies = 2;
    r.policies[0] = {CCKA_HPA_PERCENT, 100, 15};
    r.policies[1] = {CCKA_HPA_PODS, 4, 15};
  } else {
    r.n_policies = 1;
    r.policies[0] = {CCKA_HPA_PERCENT, 100, 15};
  }
  if (!b || !b->is_map()) return r;
  if (const Value* s = b->get("stabilizationWindowSeconds")) r.stab_window_s = (int32_t)s->as_int();
  if (const Value* s = b->get("selectPolicy")) {
    const std::string v = s->as_string();
    r.select = v == "Min" ? CCKA_SELECT_MIN : v == "Disabled" ? CCKA_SELECT_DISABLED : CCKA_SELECT_MAX;
  }
  if (const Value* ps = b->get("policies"); ps && ps->is_seq()) {
    r.n_policies = 0;
    for (auto& p : ps->seq) {
      if (r.n_policies == CCKA_HPA_MAX_POLICIES)
        throw ParseError("HPA behavior: more than " + std::to_string(CCKA_HPA_MAX_POLICIES) + " policies per direction");
      const std::string ty = p.get("type") ? p.get("type")->as_string() : "";
      r.policies[r.n_policies].type = ty == "Pods" ? CCKA_HPA_PODS : CCKA_HPA_PERCENT;
      r.policies[r.n_policies].value = (int32_t)(p.get("value") ? p.get("value")->as_int() : 0);
      r.policies[r.n_policies].period_s = (int32_t)(p.get("periodSeconds") ? p.get("periodSeconds")->as_int() : 15);
      ++r.n_policies;
    }
  }
  return r;
}

static bool labels_match(const Value* selector, const Value* labels) {
  if (!selector || !selector->is_map()) return false;
  for (auto& kv : selector->map) {
    const Value* l = labels ? labels->get(kv.first) : nullptr;
    if (!l || l->as_string() != kv.second.as_string()) return false;
  }
  return true;
}

WorldMeta build_world(const ManifestStore& store, const PolicyEnv& env, const Tables& T, int n_steps,
                      int max_nodes, ccka_world* w) {
  std::memset(w, 0, sizeof *w);
  WorldMeta meta;
  g_zone_prefix_seen.clear();
  // ---- NodePools, Karpenter order: weight desc, name asc
  auto pools = store.all("NodePool");
  if (pools.empty()) throw ParseError("no NodePool objects");
  if (pools.size() > CCKA_MAX_POOLS) throw ParseError("more than 4 NodePools");
  std::stable_sort(pools.begin(), pools.end(), [](const Value* a, const Value* b) {
    const Value* wa = a->at({"spec", "weight"});
    const Value* wb = b->at({"spec", "weight"});
    const int64_t x = wa ? wa->as_int() : 0, y = wb ? wb->as_int() : 0;
    if (x != y) return x > y;
    return name_of(*a) < name_of(*b);
  });
  w->n_pools = (int32_t)pools.size();
  for (size_t q = 0; q < pools.size(); ++q) {
    const Value& np = *pools[q];
    const std::string name = name_of(np);
    meta.pool_names.push_back(name);
    const Value* cl = np.at({"metadata", "labels", "carbon.simulated"});
    const Value* sl = np.at({"metadata", "labels", "autoscale.strategy"});
    meta.pool_carbon.push_back(cl ? cl->as_string() : "");
    meta.pool_strategy.push_back(sl ? sl->as_string() : "");
    ccka_pool& P = w->pools[q];
    P.limit_cpu_m = -1;
    P.limit_mem_mi = -1;
    if (const Value* l = np.at({"spec", "limits", "cpu"})) P.limit_cpu_m = (int32_t)cpu_millis(l->as_string());
    if (const Value* l = np.at({"spec", "limits", "memory"})) {
      const int64_t m = mem_mib(l->as_string());
      if (m < 0 || m > 0x7fffffff) throw ParseError("NodePool " + name + ": limits.memory out of range");
      P.limit_mem_mi = (int32_t)m;
    }
    P.budget_pct = 10;
    if (const Value* b = np.at({"spec", "disruption", "budgets", "0", "nodes"})) {
      const std::string s = b->as_string();
      if (s.empty() || s.back() != '%') throw ParseError("NodePool " + name + ": only percentage budgets are modelled");
      P.budget_pct = std::atoi(s.c_str());
    }
    ccka_pool_patch base{CCKA_WHEN_EMPTY_OR_UNDERUTILIZED, 0, 0, CCKA_CAP_OD};
    if (const Value* pol = np.at({"spec", "disruption", "consolidationPolicy"})) base.policy = policy_code(pol->as_string());
    if (const Value* ca = np.at({"spec", "disruption", "consolidateAfter"})) base.consolidate_after_s = (int32_t)duration_s(ca->as_string());
    const Value* reqs = np.at({"spec", "template", "spec", "requirements"});
    if (!reqs) reqs = np.at({"spec", "template", "requirements"});  // v1beta-style fallback path
    base.zone_mask = (1u << T.zones) - 1u;
    requirements_masks(reqs, &base.zone_mask, &base.cap_mask);
    P.base = base;
    const bool spot = name == env.np_spot, od = name == env.np_od;
    // demo_19 hard-codes its two pool names
    if (name == "spot-preferred" || name == "on-demand-slo")
      P.profile[CCKA_PROFILE_RESET] = patch_from(disruption_merge_patch(Profile::Reset, env, name), "");
    else
      P.profile[CCKA_PROFILE_RESET] = {CCKA_POLICY_KEEP, -1, 0, 0};
    for (Profile pr : {Profile::OffPeak, Profile::Peak}) {
      P.profile[(int)pr] = (spot || od) ? patch_from(disruption_merge_patch(pr, env, name),
                                                     requirements_patch(pr, env, name))
                                        : ccka_pool_patch{CCKA_POLICY_KEEP, -1, 0, 0};
    }
  }
  // ---- Deployments
  auto deps = store.all("Deployment");
  if (deps.empty()) throw ParseError("no Deployment objects");
  if (deps.size() > CCKA_MAX_DEPLOY) throw ParseError("more than 16 Deployments per scenario");
  w->n_deploy = (int32_t)deps.size();
  const Value* pdb = nullptr;
  auto pdbs = store.all("PodDisruptionBudget");
  if (pdbs.size() > 1) throw ParseError("at most one PodDisruptionBudget is modelled");
  w->pdb_min_available_pct = -1;
  if (!pdbs.empty()) {
    pdb = pdbs[0];
    const Value* ma = pdb->at({"spec", "minAvailable"});
    const std::string s = ma ? ma->as_string() : "";
    if (s.empty() || s.back() != '%') throw ParseError("PDB: only percentage minAvailable is modelled");
    w->pdb_min_available_pct = std::atoi(s.c_str());
  }
  for (size_t d = 0; d < deps.size(); ++d) {
    const Value& dv = *deps[d];
    const std::string name = name_of(dv);
    meta.deploy_names.push_back(name);
    const Value* capl = dv.at({"metadata", "labels", "capacity"});
    meta.deploy_capacity.push_back(capl ? capl->as_string() : "");
    ccka_deployment& D = w->deploy[d];
    D.scaler = CCKA_SCALER_STATIC;
    D.replicas0 = (int32_t)(dv.at({"spec", "replicas"}) ? dv.at({"spec", "replicas"})->as_int() : 1);
    D.min_replicas = D.max_replicas = D.replicas0;
    D.tolerance = 0.1;
    const Value* sel = dv.at({"spec", "template", "spec", "nodeSelector", "karpenter.sh/capacity-type"});
    const std::string cs = sel ? sel->as_string() : "";
    D.cap_sel = cs == "spot" ? CCKA_CAP_SPOT : cs == "on-demand" ? CCKA_CAP_OD : (CCKA_CAP_SPOT | CCKA_CAP_OD);
    const Value* c0 = dv.at({"spec", "template", "spec", "containers", "0", "resources"});
    if (c0) {
      if (const Value* q = c0->at({"requests", "cpu"})) D.req_cpu_m = (int32_t)cpu_millis(q->as_string());
      if (const Value* q = c0->at({"requests", "memory"})) D.req_mem_mi = (int32_t)mem_mib(q->as_string());
      if (const Value* q = c0->at({"limits", "cpu"})) D.limit_cpu_m = (int32_t)cpu_millis(q->as_string());
    }
    D.pdb_member = pdb && labels_match(pdb->at({"spec", "selector", "matchLabels"}),
                                       dv.at({"spec", "template", "metadata", "labels"}));
    D.up = rules_from(nullptr, true, 0);
    D.down = rules_from(nullptr, false, 300);
  }
  auto dep_index = [&](const Value* ref) -> int {
    const std::string n = ref ? ref->as_string() : "";
    for (size_t d = 0; d < meta.deploy_names.size(); ++d)
      if (meta.deploy_names[d] == n) return (int)d;
    throw ParseError("scale target " + n + " not found");
  };
  // ---- HPAs (autoscaling/v2, CPU Utilization)
  for (const Value* h : store.all("HorizontalPodAutoscaler")) {
    ccka_deployment& D = w->deploy[dep_index(h->at({"spec", "scaleTargetRef", "name"}))];
    D.scaler = CCKA_SCALER_HPA;
    D.min_replicas = (int32_t)(h->at({"spec", "minReplicas"}) ? h->at({"spec", "minReplicas"})->as_int() : 1);
    D.max_replicas = (int32_t)h->at({"spec", "maxReplicas"})->as_int();
    D.target_util_pct = 80;
    if (const Value* ms = h->at({"spec", "metrics"}); ms && ms->is_seq())
      for (auto& m : ms->seq)
        if (const Value* u = m.at({"resource", "target", "averageUtilization"})) D.target_util_pct = (int32_t)u->as_int();
    D.up = rules_from(h->at({"spec", "behavior", "scaleUp"}), true, 0);
    D.down = rules_from(h->at({"spec", "behavior", "scaleDown"}), false, 300);
  }
  // ---- KEDA ScaledObjects (AverageValue triggers); triggers[1..] become
  // CCKA_SCALER_KEDA_TRIGGER entries placed right after their deployment
  auto trig_params = [](const Value* md, int64_t* thr, int64_t* act) {
    for (const char* k : {"value", "threshold", "targetValue", "queueLength"})
      if (const Value* v = md->get(k)) *thr = (int64_t)std::llround(std::atof(v->as_string().c_str()));
    for (const char* k : {"activationThreshold", "activationValue", "activationTargetValue", "activationQueueLength"})
      if (const Value* v = md->get(k)) *act = (int64_t)std::llround(std::atof(v->as_string().c_str()));
  };
  std::vector<std::vector<std::pair<int64_t, int64_t>>> extra(deps.size());
  size_t n_extra = 0;
  for (const Value* so : store.all("ScaledObject")) {
    const int di = dep_index(so->at({"spec", "scaleTargetRef", "name"}));
    ccka_deployment& D = w->deploy[di];
    D.scaler = CCKA_SCALER_KEDA;
    D.keda_min = (int32_t)(so->at({"spec", "minReplicaCount"}) ? so->at({"spec", "minReplicaCount"})->as_int() : 0);
    D.keda_max = (int32_t)(so->at({"spec", "maxReplicaCount"}) ? so->at({"spec", "maxReplicaCount"})->as_int() : 100);
    D.keda_cooldown_s = (int32_t)(so->at({"spec", "cooldownPeriod"}) ? so->at({"spec", "cooldownPeriod"})->as_int() : 300);
    const Value* md = so->at({"spec", "triggers", "0", "metadata"});
    if (!md) throw ParseError("ScaledObject without triggers[0].metadata");
    trig_params(md, &D.keda_threshold, &D.keda_activation);
    const Value* trs = so->at({"spec", "triggers"});
    for (size_t j = 1; trs && trs->is_seq() && j < trs->seq.size(); ++j) {
      const Value* mj = trs->seq[j].get("metadata");
      if (!mj) throw ParseError("ScaledObject trigger without metadata");
      int64_t thr = 0, act = 0;
      trig_params(mj, &thr, &act);
      extra[di].push_back({thr, act});
      ++n_extra;
    }
    const Value* beh = so->at({"spec", "advanced", "horizontalPodAutoscalerConfig", "behavior"});
    D.up = rules_from(beh ? beh->get("scaleUp") : nullptr, true, 0);
    D.down = rules_from(beh ? beh->get("scaleDown") : nullptr, false, 300);
  }
  if (n_extra) {
    if (deps.size() + n_extra > CCKA_MAX_DEPLOY) throw ParseError("more than 16 Deployments + extra KEDA triggers");
    std::vector<ccka_deployment> out;
    std::vector<std::string> names, caps;
    for (size_t d = 0; d < deps.size(); ++d) {
      out.push_back(w->deploy[d]);
      names.push_back(meta.deploy_names[d]);
      caps.push_back(meta.deploy_capacity[d]);
      for (size_t j = 0; j < extra[d].size(); ++j) {
        ccka_deployment T{};
        T.scaler = CCKA_SCALER_KEDA_TRIGGER;
        T.cap_sel = w->deploy[d].cap_sel;
        T.tolerance = 0.1;
        T.keda_threshold = extra[d][j].first;
        T.keda_activation = extra[d][j].second;
        T.up = rules_from(nullptr, true, 0);
        T.down = rules_from(nullptr, false, 300);
        out.push_back(T);
        names.push_back(meta.deploy_names[d] + "/trigger-" + std::to_string(j + 1));
        caps.push_back(meta.deploy_capacity[d]);
      }
    }
    for (size_t d = 0; d < out.size(); ++d) w->deploy[d] = out[d];
    w->n_deploy = (int32_t)out.size();
    meta.deploy_names = names;
    meta.deploy_capacity = caps;
  }
  if (!g_zone_prefix_seen.empty()) meta.zone_prefix = g_zone_prefix_seen;
  // ---- catalog, tiles, cluster defaults
  w->n_steps = n_steps;
  w->start_minute = 0;
  w->provision_delay_steps = 1;
  w->max_nodes = max_nodes;
  w->n_types = (int32_t)T.types.size();
  w->n_regions = T.regions;
  w->n_zones = T.zones;
  w->types = T.types.data();
  w->ci_gpwh = T.ci_gpwh.data();
  w->ci_gpwmin = T.ci_gpwmin.data();
  w->price_uph = T.price.data();
  w->base_nodes = 3;  // 01_cluster.sh:24-30, .env:5-8: 3 x m6i.large
  w->base_type = T.index("m6i.large") >= 0 ? T.index("m6i.large") : 0;
  w->slo_util_pct = 150;
  w->base_util = 0.0;
  w->carbon_weight = 0.0;
  w->peak_start_min = 960;  // 4-9 PM, report p.2
  w->peak_end_min = 1260;
  w->peak_switch = 1;
  w->reset_ca_s = 30;
  w->disrupt_ext = 0;  // opt-in (ccka replay --drift)
  return meta;
}

}  // namespace ccka::host
