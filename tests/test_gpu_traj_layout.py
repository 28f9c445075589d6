"""Trajectory layout contract (include/ccka.h): the single-deployment engine
keeps its records scenario-major [N][T] on the device (ccka_trajectory_layout
= CCKA_TRAJ_NT); ccka_get_trajectory returns [T][N] through a bounded staging
buffer, block by block of steps. Past 2^21 scenarios a one-step block is all
the staging buffer holds, so every block boundary is exercised; the transpose
tiles sit on grid.x alone (a grid.y of ceil(N/32) would exceed 65535)."""
import numpy as np
import pytest

import pyoracle as po
from ccka import abi, configs
from parity import run_engine

pytestmark = pytest.mark.gpu


def test_large_n_readback_matches_native_and_oracle(engine):
    n, T = (1 << 21) + 4099, 4
    spec = configs.config2_world(n_steps=T)
    sc = configs.hpa_scenarios(n)
    rg, tg = run_engine(engine, spec, sc, gen=configs.trace_gen(), traj=True)
    assert engine.last_engine()[0] == 2  # the single-deployment engine
    native, lay = engine.trajectory_native()
    assert lay == abi.TRAJ_NT and native.shape == (n, T)
    assert np.array_equal(tg, native.T)
    # a prefix and the tail against the oracle (same device-generated traces)
    load = engine.get_load()
    for lo, hi in ((0, 20_000), (n - 5_000, n)):
        sub = sc.slice(lo, hi)
        rc, tc = po.rollout(spec, sub, np.ascontiguousarray(load[:, :, lo:hi]), traj=True, threads=8)
        assert np.array_equal(tg[:, lo:hi], tc)
        for k in rc:
            assert np.array_equal(rg[k][lo:hi], rc[k]), k


def test_general_engine_layout_is_step_major(engine):
    # the general engine (per-scenario detail requested) writes [T][N]
    spec = configs.config2_world(n_steps=120)
    sc = configs.hpa_scenarios(3000)
    engine.set_detail(True)
    try:
        _, tg = run_engine(engine, spec, sc, gen=configs.trace_gen(), traj=True)
        native, lay = engine.trajectory_native()
    finally:
        engine.set_detail(False)
    assert lay == abi.TRAJ_TN and np.array_equal(native, tg)
