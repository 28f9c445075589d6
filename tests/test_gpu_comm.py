"""The RCCL exchange paths of libccka on one GPU: a one-rank
communicator through ccka_comm_unique_id / ccka_comm_init, the totals
all-reduce, the Pareto all-gather + merge, and the cross-rank merge itself on
synthetic multi-rank exchange buffers, each against the single-rank result or
the numpy restatement of the frontier (oracle/pyoracle.py)."""
import numpy as np
import pytest

import pyoracle as po
from ccka import abi, configs
from ccka.engine import GRID_DTYPE, Engine
from parity import run_engine

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    e = Engine(0)
    yield e
    e.close()


def test_comm_state_errors_before_init(eng):
    with pytest.raises(abi.CckaError):
        eng.comm_info()
    with pytest.raises(abi.CckaError):
        eng.allreduce_totals(abi.Totals())


def test_one_rank_allreduce_is_identity(eng):
    spec = configs.config2_world(n_steps=240)
    sc = configs.hpa_scenarios(3000, first_id=777)
    run_engine(eng, spec, sc, gen=configs.trace_gen())
    t = eng.totals()
    eng.comm_init()
    assert eng.comm_info() == (1, 0)
    got = eng.allreduce_totals(t)
    for f, _ in abi.Totals._fields_:
        assert getattr(got, f) == getattr(t, f), f
    assert got.scenarios == 3000


def test_pareto_with_communicator_equals_local(eng):
    n_traces = 16
    spec = configs.config2_world(n_steps=360)
    sc = configs.config4_scenarios(40, 48, n_traces)
    load = po.gen_load(configs.config4_trace_gen(), 360, 1, n_traces)
    fresh = Engine(0)  # no communicator: the local frontier
    try:
        run_engine(fresh, spec, sc, load=load)
        want = fresh.pareto(n_traces)
    finally:
        fresh.close()
    run_engine(eng, spec, sc, load=load)
    if not eng.lib.ccka_comm_info(eng.ctx, None, None) == 0:
        eng.comm_init()
    got = eng.pareto(n_traces)  # all-gather over the one-rank communicator + merge
    assert np.array_equal(got, want)
    stats = eng.grid_stats(n_traces)
    assert np.array_equal(got, stats[po.pareto({k: stats[k] for k in stats.dtype.names})])


def _random_grids(rng, g0, n):
    a = np.zeros(n, GRID_DTYPE)
    a["grid"] = np.arange(g0, g0 + n)
    a["scenarios"] = 16
    a["cost_uphmin"] = rng.integers(0, 40, n)
    a["slo_minutes"] = rng.integers(0, 40, n)
    a["gco2"] = rng.integers(0, 40, n).astype(np.float64) * 0.5
    a["energy_wmin"] = rng.random(n)
    return a


@pytest.mark.parametrize("nranks", [2, 3, 8])
def test_cross_rank_merge_equals_frontier_of_concatenation(eng, nranks):
    rng = np.random.default_rng(nranks)
    cap = 64
    rows = [_random_grids(rng, q * cap, cap) for q in range(nranks)]
    gathered = np.zeros((nranks, cap), GRID_DTYPE)
    counts = []
    for q, r in enumerate(rows):  # each rank contributes its local frontier
        loc = r[po.pareto({k: r[k] for k in r.dtype.names})]
        gathered[q, :len(loc)] = loc
        gathered[q, len(loc):]["grid"] = -1  # garbage beyond the count must be ignored
        counts.append(len(loc))
    got = eng.debug_pareto_merge(gathered, counts)
    allg = np.concatenate(rows)
    want = allg[po.pareto({k: allg[k] for k in allg.dtype.names})]
    assert np.array_equal(got, want)
    assert np.all(np.diff(got["grid"]) > 0)


def test_cross_rank_merge_keeps_all_when_nothing_dominates(eng):
    # every candidate of every rank survives: the frontier is larger than one
    # rank's grid count (the global buffer holds nranks x grids)
    nranks, cap = 4, 8
    g = np.zeros((nranks, cap), GRID_DTYPE)
    k = np.arange(nranks * cap)
    g["grid"] = k.reshape(nranks, cap)
    g["cost_uphmin"] = k.reshape(nranks, cap)
    g["slo_minutes"] = (nranks * cap - k).reshape(nranks, cap)
    got = eng.debug_pareto_merge(g, [cap] * nranks)
    assert len(got) == nranks * cap
    with pytest.raises(abi.CckaError):
        eng.debug_pareto_merge(g, [cap] * nranks, capacity=cap)
