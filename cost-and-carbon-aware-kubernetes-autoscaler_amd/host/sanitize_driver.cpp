// sanitize_driver.cpp — TEST INFRASTRUCTURE: the host library (manifest
// ingest, kubectl apply / patch emulation, payload generators, world builder,
// summary, export, admission) and the CPU oracle built with
// -fsanitize=address,undefined (`make -C host sanitize`), driven over every
// input given on the command line. tests/test_sanitize.py runs it on the
// reference-captured payloads and a hypothesis-generated corpus; any
// AddressSanitizer / UndefinedBehaviorSanitizer report aborts the process.
//
//   sanitize_driver yaml FILE...      apply each file (errors are fine, faults are not),
//                                     read back JSON, review admission
//   sanitize_driver json FILE...      merge-patch and JSON-patch a stored NodePool with each file
//   sanitize_driver world             payload generators, world build, oracle rollout of the
//                                     replay world (drift + replacement on), summary, export
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/ccka.h"
#include "../../include/ccka_host.h"
#include "../../oracle/ccka_oracle.h"

static std::string slurp(const char* path) {
  std::ifstream f(path, std::ios::binary);
  std::stringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

static std::vector<char> buf(1 << 22);

static int run_yaml(ccka_host* h, const char* path) {
  const std::string text = slurp(path);
  int rc = ccka_host_apply(h, text.c_str());
  (void)ccka_host_last_error(h);
  for (const char* kind : {"NodePool", "Deployment", "PodDisruptionBudget", "HorizontalPodAutoscaler",
                           "ScaledObject"})
    for (const char* name : {"spot-preferred", "on-demand-slo", "burst-web-1", "burst-pdb", "x"})
      (void)ccka_host_get_json(h, kind, name, buf.data(), (int64_t)buf.size());
  (void)ccka_host_admission_review(h, CCKA_ADMIT_REQUIRE_REQUESTS_LIMITS | CCKA_ADMIT_CRITICAL_NO_SPOT, text.c_str(),
                                   buf.data(), (int64_t)buf.size());
  return rc;
}

static void run_json(ccka_host* h, const char* path) {
  const std::string text = slurp(path);
  for (const char* type : {"merge", "json"})
    for (const char* name : {"spot-preferred", "on-demand-slo"})
      (void)ccka_host_patch(h, "NodePool", name, type, text.c_str());
  (void)ccka_host_get_json(h, "NodePool", "spot-preferred", buf.data(), (int64_t)buf.size());
}

static int run_world(ccka_host* h) {
  for (int p = 0; p <= 2; ++p)
    for (const char* pool : {"spot-preferred", "on-demand-slo"})
      for (int js = 0; js < 2; ++js)
        for (int fb = 0; fb < 2; ++fb) (void)ccka_host_policy_patch(h, p, pool, js, fb, buf.data(), 4096);
  for (int i = -1; i <= 12; ++i) {
    if (ccka_host_burst_manifest(h, i, buf.data(), (int64_t)buf.size()) < 0) return 1;
    if (ccka_host_apply(h, buf.data()) != CCKA_OK) return 2;
  }
  ccka_world w;
  (void)ccka_host_label(h, "NodePool", "spot-preferred", "autoscale.strategy=cost carbon.simulated=low", 1);
  (void)ccka_host_label(h, "NodePool", "on-demand-slo", "carbon.simulated=medium x=y x- bad", 0);
  if (ccka_host_build_world(h, "tiny", 360, 16, &w) != CCKA_OK) return 3;
  w.disrupt_ext = CCKA_DISRUPT_DRIFT | CCKA_DISRUPT_REPLACE;
  const int64_t n = 3, T = w.n_steps, D = w.n_deploy;
  std::vector<int32_t> load((size_t)(T * D * n));
  ccka_trace_gen g{};
  g.seed = 20251205;
  g.base_lo = 500; g.base_hi = 5000; g.amp_lo_pm = 200; g.amp_hi_pm = 800; g.noise_pm = 50;
  g.burst_prob_pm = 500; g.burst_mult_pm = 3000; g.burst_len = 30;
  ccka_oracle_gen_load(&g, (int32_t)T, (int32_t)D, n, 0, load.data());
  ccka_scenarios sc{};
  sc.n = n;
  std::vector<int64_t> cost(n), ppm(n);
  std::vector<double> en(n), co2(n);
  std::vector<int32_t> i32[8];
  for (auto& v : i32) v.assign((size_t)n, 0);
  std::vector<uint32_t> lc(n), hs(n);
  ccka_results r{cost.data(), en.data(), co2.data(), i32[0].data(), ppm.data(), i32[1].data(), i32[2].data(),
                 i32[3].data(), i32[4].data(), i32[5].data(), i32[6].data(), i32[7].data(), lc.data(), hs.data()};
  std::vector<ccka_traj_rec> traj((size_t)(T * n));
  std::vector<ccka_detail> det((size_t)n);
  if (ccka_oracle_rollout_detail(&w, &sc, load.data(), &r, traj.data(), det.data(), 2) != CCKA_OK) return 4;
  ccka_totals tot;
  if (ccka_oracle_totals(&r, n, &tot) != CCKA_OK) return 8;
  if (ccka_host_summary(h, &w, &r, traj.data(), det.data(), buf.data(), (int64_t)buf.size()) < 0) return 5;
  if (ccka_host_summary(h, &w, &r, nullptr, nullptr, buf.data(), (int64_t)buf.size()) < 0) return 5;
  int64_t need = 0;
  for (int f : {CCKA_EXPORT_PROMETHEUS, CCKA_EXPORT_CSV})
    if (ccka_host_export(h, f, &w, traj.data(), n, &r, 0, n, 0, 1700000000000LL, buf.data(), (int64_t)buf.size(),
                         &need) != CCKA_OK)
      return 6;
  if (ccka_host_export_detail(h, &w, det.data(), n, 0, 1700000000000LL, buf.data(), (int64_t)buf.size(), &need) !=
      CCKA_OK)
    return 7;
  std::printf("world ok: %lld scenarios x %lld steps, launches %lld deletions %lld\n", (long long)n, (long long)T,
              (long long)tot.launches, (long long)tot.deletions);
  return 0;
}

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  ccka_host* h = nullptr;
  if (ccka_host_open(&h) != CCKA_OK) return 1;
  const std::string mode = argv[1];
  int rc = 0, ok = 0;
  if (mode == "yaml") {
    for (int a = 2; a < argc; ++a) ok += run_yaml(h, argv[a]) == CCKA_OK;
    std::printf("yaml: %d of %d documents sets applied\n", ok, argc - 2);
  } else if (mode == "json") {
    if (ccka_host_burst_manifest(h, -1, buf.data(), (int64_t)buf.size()) >= 0) (void)ccka_host_apply(h, buf.data());
    for (int a = 2; a < argc; ++a) run_json(h, argv[a]);
    std::printf("json: %d patches\n", argc - 2);
  } else if (mode == "world") {
    rc = run_world(h);
  } else {
    rc = 2;
  }
  ccka_host_close(h);
  return rc;
}
