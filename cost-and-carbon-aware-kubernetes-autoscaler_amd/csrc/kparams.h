// kparams.h — kernel argument blocks shared by rollout.hip and ccka_abi.cpp.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ccka.h"

namespace ccka {

struct KParams {
  const ccka_world* w;  // device copy (pools, deployments, scalars)
  const ccka_itype* types;
  const int32_t* price;  // [R][24][K][Z][2]
  const double* ci_gpwh;
  const double* ci_gpwmin;
  const int32_t* load;  // [T][D][N]
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
  int64_t N;
  int32_t T, D, K, Z, R, P, maxn, span, all_hours;
  int32_t lds_off_cap1, lds_off_tile, lds_off_claims, lds_off_misc, lds_off_ci;
  int32_t ablate;  // profiling-only phase switches (0 in every real run)
  int32_t prov[CCKA_MAX_DEPLOY];
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
  int64_t N;
};

constexpr int kPartBytes = 8 * 8 + 2 * 8;

// kernel instantiation chosen for (D, max_nodes): DMAX x MAXN
inline void kernel_dims(int D, int maxn, int* dmax, int* nmax) {
  if (D == 1 && maxn <= 8) { *dmax = 1; *nmax = 8; }
  else if (D == 1) { *dmax = 1; *nmax = 16; }
  else if (D <= 4) { *dmax = 4; *nmax = 16; }
  else { *dmax = 16; *nmax = 16; }
}

hipError_t launch_gen_load(const GenParams& g, hipStream_t s);
hipError_t launch_rollout(const KParams& p, int block, size_t lds, hipStream_t s);
hipError_t launch_totals(const TotParams& q, int nparts, hipStream_t s);

}  // namespace ccka
