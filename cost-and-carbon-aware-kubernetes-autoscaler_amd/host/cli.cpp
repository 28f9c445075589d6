// cli.cpp — the `ccka` command: a drop-in for the reference's decision path.
//
//   ccka patch <reset|offpeak|peak> --pool NAME [--json] [--fallback]
//       the exact payload demo_19 / demo_20 / demo_21 hand to `kubectl patch`
//   ccka manifest <burst [--index I] | pdb | nodepools>
//       the demo_30 Deployments / demo_10 PDB / our base NodePools (YAML)
//   ccka replay [--nodepools F] [--apply F]... [--patch KIND NAME TYPE FILE]... [--label KIND NAME LABELS]...
//               [--catalog tiny|small] [--steps T] [--max-nodes N] [--load-m M]
//               [--device D] [--json OUT] [--prom OUT] [--csv OUT] [--start-unix-ms MS]
//       ingest the manifests, build the world, roll one cluster forward on the
//       MI355X through libccka (ccka.h) and print the demo_41-style summary
//       (the reference's missing demo_41_observe_cost_nodes.sh, README.md:57);
//       --prom / --csv write the trajectory as Prometheus text exposition / CSV
//       (ccka_host_export, the series the reference's observe path scrapes).
// Environment: NP_SPOT NP_OD OFFPEAK_ZONES PEAK_ZONES NAMESPACE COUNT REPLICAS.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/ccka.h"
#include "../../include/ccka_host.h"

static std::string slurp(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) {
    std::fprintf(stderr, "ccka: cannot read %s\n", path.c_str());
    std::exit(2);
  }
  std::stringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

static int usage() {
  std::fprintf(stderr,
               "usage: ccka version\n"
               "       ccka patch <reset|offpeak|peak> --pool NAME [--json] [--fallback]\n"
               "       ccka manifest <burst [--index I] | pdb | nodepools>\n"
               "       ccka replay [--nodepools F] [--apply F]... [--patch KIND NAME TYPE FILE]...\n"
               "                   [--label KIND NAME 'k=v ...']...\n"
               "                   [--catalog tiny|small] [--steps T] [--max-nodes N] [--load-m M]\n"
               "                   [--device D] [--json OUT] [--prom OUT] [--csv OUT] [--start-unix-ms MS]\n"
               "                   [--drift] [--replace] [--multi] [--kyverno] [--hpa-sync S]\n");
  return 2;
}

static void die_host(ccka_host* h, const char* what) {
  std::fprintf(stderr, "[err] %s: %s\n", what, ccka_host_last_error(h));
  std::exit(1);
}

int main(int argc, char** argv) {
  if (argc < 2) return usage();
  const std::string cmd = argv[1];
  ccka_host* h = nullptr;
  if (ccka_host_open(&h) != CCKA_OK) return 1;
  static char buf[1 << 20];

  if (cmd == "version") {
    std::printf("ccka abi %d\n", ccka_abi_version());
    return 0;
  }
  if (cmd == "patch") {
    if (argc < 3) return usage();
    const std::string prof = argv[2];
    const int p = prof == "reset" ? CCKA_PROFILE_RESET : prof == "offpeak" ? CCKA_PROFILE_OFFPEAK
                  : prof == "peak" ? CCKA_PROFILE_PEAK : -1;
    if (p < 0) return usage();
    std::string pool;
    int json = 0, fb = 0;
    for (int a = 3; a < argc; ++a) {
      if (!std::strcmp(argv[a], "--pool") && a + 1 < argc) pool = argv[++a];
      else if (!std::strcmp(argv[a], "--json")) json = 1;
      else if (!std::strcmp(argv[a], "--fallback")) fb = 1;
      else return usage();
    }
    if (pool.empty()) return usage();
    const int n = ccka_host_policy_patch(h, p, pool.c_str(), json, fb, buf, sizeof buf);
    if (n < 0) die_host(h, "patch");
    std::fwrite(buf, 1, (size_t)n, stdout);
    return 0;
  }
  if (cmd == "manifest") {
    if (argc < 3) return usage();
    const std::string what = argv[2];
    std::vector<int> idx;
    if (what == "pdb") idx.push_back(0);
    else if (what == "nodepools") idx.push_back(-1);
    else if (what == "burst") {
      int one = 0;
      for (int a = 3; a < argc; ++a)
        if (!std::strcmp(argv[a], "--index") && a + 1 < argc) one = std::atoi(argv[++a]);
      const char* c = std::getenv("COUNT");
      const int count = (c && *c) ? std::atoi(c) : 12;
      if (one) idx.push_back(one);
      else for (int i = 1; i <= count; ++i) idx.push_back(i);
    } else {
      return usage();
    }
    for (size_t k = 0; k < idx.size(); ++k) {
      const int n = ccka_host_burst_manifest(h, idx[k], buf, sizeof buf);
      if (n < 0) die_host(h, "manifest");
      if (k) std::fputs("---\n", stdout);
      std::fwrite(buf, 1, (size_t)n, stdout);
    }
    return 0;
  }
  if (cmd != "replay") return usage();

  std::string nodepools, catalog = "tiny", json_out, prom_out, csv_out;
  long long start_ms = 0;
  std::vector<std::string> applies;
  std::vector<std::vector<std::string>> patches, labels;
  int steps = 1440, max_nodes = 16, device = 0, drift = 0, replace = 0, multi = 0, kyverno = 0, hpa_sync = 0;
  long load_m = 100;
  for (int a = 2; a < argc; ++a) {
    auto next = [&]() -> std::string {
      if (a + 1 >= argc) std::exit(usage());
      return argv[++a];
    };
    if (!std::strcmp(argv[a], "--nodepools")) nodepools = next();
    else if (!std::strcmp(argv[a], "--apply")) applies.push_back(next());
    else if (!std::strcmp(argv[a], "--patch")) {
      std::vector<std::string> p;
      for (int k = 0; k < 4; ++k) p.push_back(next());
      patches.push_back(p);
    } else if (!std::strcmp(argv[a], "--label")) {
      std::vector<std::string> p;
      for (int k = 0; k < 3; ++k) p.push_back(next());
      labels.push_back(p);
    } else if (!std::strcmp(argv[a], "--catalog")) catalog = next();
    else if (!std::strcmp(argv[a], "--steps")) steps = std::atoi(next().c_str());
    else if (!std::strcmp(argv[a], "--max-nodes")) max_nodes = std::atoi(next().c_str());
    else if (!std::strcmp(argv[a], "--load-m")) load_m = std::atol(next().c_str());
    else if (!std::strcmp(argv[a], "--device")) device = std::atoi(next().c_str());
    else if (!std::strcmp(argv[a], "--json")) json_out = next();
    else if (!std::strcmp(argv[a], "--prom")) prom_out = next();
    else if (!std::strcmp(argv[a], "--csv")) csv_out = next();
    else if (!std::strcmp(argv[a], "--start-unix-ms")) start_ms = std::atoll(next().c_str());
    else if (!std::strcmp(argv[a], "--drift")) drift = 1;
    else if (!std::strcmp(argv[a], "--replace")) replace = 1;
    else if (!std::strcmp(argv[a], "--multi")) multi = 1;
    else if (!std::strcmp(argv[a], "--kyverno")) kyverno = 1;
    else if (!std::strcmp(argv[a], "--hpa-sync")) hpa_sync = std::atoi(next().c_str());
    else return usage();
  }
  // manifests in: base NodePools, then every applied file; default demand is
  // the demo_30 burst + the demo_10 PDB when no Deployment was applied
  // 04_kyverno.sh guard policies as the admission pre-filter (opt-in)
  if (kyverno && ccka_host_set_admission(h, CCKA_ADMIT_REQUIRE_REQUESTS_LIMITS | CCKA_ADMIT_CRITICAL_NO_SPOT) != CCKA_OK)
    die_host(h, "kyverno");
  if (!nodepools.empty()) {
    if (ccka_host_apply(h, slurp(nodepools).c_str()) != CCKA_OK) die_host(h, nodepools.c_str());
  } else {
    ccka_host_burst_manifest(h, -1, buf, sizeof buf);
    if (ccka_host_apply(h, buf) != CCKA_OK) die_host(h, "base nodepools");
  }
  for (auto& f : applies)
    if (ccka_host_apply(h, slurp(f).c_str()) != CCKA_OK) die_host(h, f.c_str());
  for (auto& p : patches)
    if (ccka_host_patch(h, p[0].c_str(), p[1].c_str(), p[2].c_str(), slurp(p[3]).c_str()) != CCKA_OK)
      die_host(h, "patch");
  if (ccka_host_get_json(h, "Deployment", "burst-web-1", buf, sizeof buf) < 0 && applies.empty()) {
    const char* c = std::getenv("COUNT");
    const int count = (c && *c) ? std::atoi(c) : 12;
    for (int i = 1; i <= count; ++i) {
      ccka_host_burst_manifest(h, i, buf, sizeof buf);
      if (ccka_host_apply(h, buf) != CCKA_OK) die_host(h, "burst");
    }
    ccka_host_burst_manifest(h, 0, buf, sizeof buf);
    if (ccka_host_apply(h, buf) != CCKA_OK) die_host(h, "pdb");
    // demo_10_setup_configure.sh:61-62 (`kubectl label nodepool ... --overwrite || true`)
    const char* sp = std::getenv("NP_SPOT");
    const char* od = std::getenv("NP_OD");
    (void)ccka_host_label(h, "NodePool", sp && *sp ? sp : "spot-preferred", "autoscale.strategy=cost carbon.simulated=low", 1);
    (void)ccka_host_label(h, "NodePool", od && *od ? od : "on-demand-slo", "autoscale.strategy=slo carbon.simulated=medium", 1);
  }
  for (auto& l : labels)  // kubectl label --overwrite
    if (ccka_host_label(h, l[0].c_str(), l[1].c_str(), l[2].c_str(), 1) != CCKA_OK) die_host(h, "label");
  ccka_world w;
  if (ccka_host_build_world(h, catalog.c_str(), steps, max_nodes, &w) != CCKA_OK) die_host(h, "build world");
  // Karpenter drift on the zone switch / replacement consolidation (SEMANTICS 3.G0, 3.G2)
  w.disrupt_ext = (drift ? CCKA_DISRUPT_DRIFT : 0) | (replace ? CCKA_DISRUPT_REPLACE : 0) |
                  (multi ? CCKA_DISRUPT_MULTI : 0);
  // kube-controller-manager --horizontal-pod-autoscaler-sync-period (upstream default 15 s;
  // 0 = one decision per 60-s step, SEMANTICS 3.C)
  w.hpa_sync_s = hpa_sync;

  // decisions: one cluster on the GPU
  ccka_ctx* ctx = nullptr;
  int rc = ccka_open(&ctx, device);
  if (rc != CCKA_OK) {
    std::fprintf(stderr, "[err] ccka_open(%d) failed (%d): no gfx950 device\n", device, rc);
    return 1;
  }
  auto chk = [&](int r, const char* what) {
    if (r != CCKA_OK) {
      std::fprintf(stderr, "[err] %s: %s\n", what, ccka_last_error(ctx));
      std::exit(1);
    }
  };
  chk(ccka_set_world(ctx, &w), "ccka_set_world");
  ccka_scenarios sc{};
  sc.n = 1;
  chk(ccka_set_scenarios(ctx, &sc), "ccka_set_scenarios");
  std::vector<int32_t> load((size_t)steps * w.n_deploy, (int32_t)load_m);
  chk(ccka_set_load(ctx, load.data(), (int64_t)load.size()), "ccka_set_load");
  chk(ccka_set_detail(ctx, 1), "ccka_set_detail");
  chk(ccka_rollout(ctx, 1), "ccka_rollout");
  ccka_detail det;
  chk(ccka_get_detail(ctx, &det, 1), "ccka_get_detail");
  int64_t cost, pend;
  double energy, gco2;
  int32_t slo, nsp, nod, lau, del, peak, frep, fnod;
  uint32_t lc, hash;
  ccka_results r{&cost, &energy, &gco2, &slo, &pend, &nsp, &nod, &lau, &del, &peak, &frep, &fnod, &lc, &hash};
  chk(ccka_get_results(ctx, &r), "ccka_get_results");
  std::vector<ccka_traj_rec> traj((size_t)steps);
  chk(ccka_get_trajectory(ctx, traj.data(), (int64_t)steps), "ccka_get_trajectory");
  const int n = ccka_host_summary(h, &w, &r, traj.data(), &det, buf, sizeof buf);
  if (n < 0) die_host(h, "summary");
  std::fwrite(buf, 1, (size_t)n, stdout);
  if (!json_out.empty()) {
    FILE* f = std::fopen(json_out.c_str(), "w");
    if (!f) return 1;
    std::fprintf(f,
                 "{\"cost_uphmin\": %lld, \"energy_wmin\": %.17g, \"gco2\": %.17g, \"slo_minutes\": %d, "
                 "\"pending_pod_minutes\": %lld, \"node_min_spot\": %d, \"node_min_od\": %d, \"launches\": %d, "
                 "\"deletions\": %d, \"peak_nodes\": %d, \"final_replicas\": %d, \"final_nodes\": %d, "
                 "\"last_choice\": %u, \"choice_hash\": %u, \"detail\": {",
                 (long long)cost, energy, gco2, slo, (long long)pend, nsp, nod, lau, del, peak, frep, fnod, lc, hash);
    auto arr64 = [&](const char* k, const int64_t* v, int m, bool last = false) {
      std::fprintf(f, "\"%s\": [", k);
      for (int i = 0; i < m; ++i) std::fprintf(f, "%s%lld", i ? ", " : "", (long long)v[i]);
      std::fprintf(f, "]%s", last ? "" : ", ");
    };
    auto arr32 = [&](const char* k, const int32_t* v, int m) {
      std::fprintf(f, "\"%s\": [", k);
      for (int i = 0; i < m; ++i) std::fprintf(f, "%s%d", i ? ", " : "", v[i]);
      std::fprintf(f, "], ");
    };
    const int P = w.n_pools, D = w.n_deploy;
    arr64("pool_cost_uphmin", det.pool_cost_uphmin, P);
    arr64("pool_energy_nwmin", det.pool_energy_nwmin, P);
    std::fprintf(f, "\"pool_gco2\": [");
    for (int i = 0; i < P; ++i) std::fprintf(f, "%s%.17g", i ? ", " : "", det.pool_gco2[i]);
    std::fprintf(f, "], ");
    arr32("pool_node_min_spot", det.pool_node_min_spot, P);
    arr32("pool_node_min_od", det.pool_node_min_od, P);
    arr32("pool_final_nodes", det.pool_final_nodes, P);
    arr32("pool_peak_nodes", det.pool_peak_nodes, P);
    arr32("pool_launches", det.pool_launches, P);
    arr32("desired", det.desired, D);
    arr32("ready", det.ready, D);
    arr32("pending", det.pending, D);
    std::fprintf(f, "\"base_cost_uphmin\": %lld, \"base_energy_nwmin\": %lld, \"base_gco2\": %.17g}}\n",
                 (long long)det.base_cost_uphmin, (long long)det.base_energy_nwmin, det.base_gco2);
    std::fclose(f);
  }
  for (int fmt : {CCKA_EXPORT_PROMETHEUS, CCKA_EXPORT_CSV}) {
    const std::string& path = fmt == CCKA_EXPORT_PROMETHEUS ? prom_out : csv_out;
    if (path.empty()) continue;
    int64_t need = 0;
    ccka_host_export(h, fmt, &w, traj.data(), 1, &r, 0, 1, 0, start_ms, nullptr, 0, &need);
    std::vector<char> text((size_t)(need > 0 ? need : 1));
    if (ccka_host_export(h, fmt, &w, traj.data(), 1, &r, 0, 1, 0, start_ms, text.data(), need, &need) != CCKA_OK)
      die_host(h, "export");
    FILE* f = std::fopen(path.c_str(), "w");
    if (!f) return 1;
    std::fputs(text.data(), f);
    if (fmt == CCKA_EXPORT_PROMETHEUS) {  // the per-pool breakdown (carbon.simulated groups)
      ccka_host_export_detail(h, &w, &det, 1, 0, start_ms, nullptr, 0, &need);
      std::vector<char> t2((size_t)(need > 0 ? need : 1));
      if (ccka_host_export_detail(h, &w, &det, 1, 0, start_ms, t2.data(), need, &need) != CCKA_OK)
        die_host(h, "export detail");
      std::fputs(t2.data(), f);
    }
    std::fclose(f);
  }
  ccka_close(ctx);
  ccka_host_close(h);
  return 0;
}
