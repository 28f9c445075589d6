"""GPU parity of the policy sweep (BASELINE config 4): shared load traces,
per-grid sums and the cost / gCO2 / SLO Pareto frontier, against the CPU oracle
and its numpy restatement of the frontier (oracle/pyoracle.py)."""
import numpy as np
import pytest

import pyoracle as po
from ccka import configs
from parity import compare, oracle, run_engine

pytestmark = pytest.mark.gpu
THREADS = 16


def _sweep(engine, grid_lo, n_grids, n_traces, T):
    spec = configs.config2_world(n_steps=T)
    sc = configs.config4_scenarios(grid_lo, n_grids, n_traces)
    load = po.gen_load(configs.config4_trace_gen(), T, 1, n_traces)  # keyed by trace index
    rg, tg = run_engine(engine, spec, sc, load=load, traj=True)
    return spec, sc, load, rg, tg


def test_shared_traces_parity(engine):
    spec, sc, load, rg, tg = _sweep(engine, 37, 24, 48, 480)
    assert engine.last_engine()[0] == 2
    rc, tc = oracle(spec, sc, load, traj=True, threads=THREADS)
    compare(rg, rc, tg, tc)


def test_device_generated_shared_traces(engine):
    spec = configs.config2_world(n_steps=240)
    sc = configs.config4_scenarios(5, 8, 64)
    engine.set_world(spec)
    engine.set_scenarios(sc)
    engine.gen_load(configs.config4_trace_gen())
    got = engine.get_load()
    assert got.shape == (240, 1, 64)
    assert np.array_equal(got, po.gen_load(configs.config4_trace_gen(), 240, 1, 64))


def test_grid_stats_and_pareto(engine):
    n_traces = 32
    spec, sc, load, rg, _ = _sweep(engine, 64, 96, n_traces, 600)
    rc, _ = oracle(spec, sc, load, threads=THREADS)
    got = engine.grid_stats(n_traces)
    want = po.grid_stats(rc, n_traces, sc.first_id)
    for f in ("grid", "scenarios", "cost_uphmin", "slo_minutes"):
        assert np.array_equal(got[f], want[f]), f
    for f in ("gco2", "energy_wmin"):
        assert np.allclose(got[f], want[f], rtol=1e-12, atol=0), f
    front = engine.pareto(n_traces)
    # the device frontier is exactly the numpy frontier of the device's grid sums ...
    idx = po.pareto({k: got[k] for k in got.dtype.names})
    assert np.array_equal(front["grid"], got["grid"][idx])
    assert np.array_equal(front, got[idx])
    # ... and of the oracle's
    assert np.array_equal(front["grid"], want["grid"][po.pareto(want)])
    assert 1 <= len(front) < len(got)


def test_pareto_rejects_partial_grids(engine):
    spec, sc, load, rg, _ = _sweep(engine, 0, 4, 16, 60)
    from ccka import abi
    with pytest.raises(abi.CckaError):
        engine.grid_stats(24)
