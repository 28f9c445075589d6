"""Shared helpers: run the HIP engine and the CPU oracle on identical inputs and
compare bit-exactly (integers, instance choices, trajectories) and within
1e-9 relative error (fp64 energy / gCO2; in practice these are bit-exact too:
both sides evaluate the same binary64 operations without contraction)."""
from __future__ import annotations

import numpy as np

import pyoracle as po

INT_FIELDS = ["cost_uphmin", "slo_minutes", "pending_pod_minutes", "node_min_spot", "node_min_od",
              "launches", "deletions", "peak_nodes", "final_replicas", "final_nodes", "last_choice",
              "choice_hash"]
FP_FIELDS = ["energy_wmin", "gco2"]
FP_RTOL = 1e-9  # north_star: <= 1e-9 relative error for fp64 cost / gCO2 totals


def run_engine(engine, spec, scen, load=None, gen=None, traj=False):
    engine.set_world(spec)
    engine.set_scenarios(scen)
    if load is not None:
        engine.set_load(load)
    else:
        engine.gen_load(gen)
    engine.rollout(trajectory=traj)
    res = engine.results()
    tr = engine.trajectory() if traj else None
    return res, tr


def compare(res_gpu, res_cpu, tr_gpu=None, tr_cpu=None, exact_fp=True):
    for f in INT_FIELDS:
        a, b = res_gpu[f], res_cpu[f]
        bad = np.nonzero(a != b)[0]
        assert bad.size == 0, f"{f}: {bad.size} mismatches, first idx {bad[:5]} gpu {a[bad[:5]]} cpu {b[bad[:5]]}"
    for f in FP_FIELDS:
        a, b = res_gpu[f], res_cpu[f]
        if exact_fp:
            bad = np.nonzero(a != b)[0]
            assert bad.size == 0, f"{f}: {bad.size} not bit-exact, first {bad[:5]} {a[bad[:5]]} {b[bad[:5]]}"
        rel = np.abs(a - b) / np.maximum(np.abs(b), 1e-300)
        assert rel.max() <= FP_RTOL, f"{f}: max rel err {rel.max()}"
    if tr_gpu is not None:
        for f in tr_gpu.dtype.names:
            bad = np.argwhere(tr_gpu[f] != tr_cpu[f])
            assert bad.size == 0, f"traj.{f}: {len(bad)} mismatches, first (t, i) {bad[:5].tolist()}"


def oracle(spec, scen, load, traj=False, threads=8):
    return po.rollout(spec, scen, load, traj=traj, threads=threads)
