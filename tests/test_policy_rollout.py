"""Closed-loop learned control policy (BASELINE config 5; SEMANTICS 5): the
MLP decides every step's HPA target utilisation and Karpenter carbon weight
from the scenario state. Parity is split where the arithmetic allows it:
the features and the rollout under the recorded actions are bit-exact against
the CPU oracle; the MLP itself is checked against a PyTorch fp32 reference
(the actions derived from it agree except within rounding of an action
boundary); the action mapping is reproduced in numpy."""
import numpy as np
import pytest

import pyoracle as po
from ccka import abi, configs
from parity import compare

THREADS = 16


def _case(n=512, T=180, drift=0, world=None):
    spec = (world or configs.config2_world)(n_steps=T)
    spec.drift = drift
    sc = configs.hpa_scenarios(n, first_id=99)
    load = po.gen_load(configs.trace_gen(5), T, 1, n, first_id=99)
    return spec, sc, load


def test_action_mapping_bounds():
    y = np.array([[0.0, 0.0], [0.03125, 0.03125], [0.09375, -1.0], [10.0, 10.0], [-10.0, 0.2]], np.float32)
    t, c = po.policy_act(np.pad(y, ((0, 0), (0, 6))))
    assert t.tolist() == [60, 60, 62, 95, 20]  # rint(0.5) = 0, rint(1.5) = 2 (half to even)
    assert c.tolist() == [0.0, 0.0, 0.0, 4.0, 0.1875]


def test_oracle_replay_matches_fixed_overrides():
    """Constant actions reproduce the ordinary rollout with the same per-scenario
    overrides (the replay path is the rollout, not a second model)."""
    spec, sc, load = _case(n=200, T=120)
    tg = np.asarray(sc.target_util_pct, np.int16)
    cw = np.full(sc.n, 0.5)
    at = np.broadcast_to(tg, (spec.n_steps, sc.n)).copy()
    ac = np.broadcast_to(cw, (spec.n_steps, sc.n)).copy()
    r1, t1, f1 = po.rollout_policy(spec, sc, load, at, ac, traj=True, threads=8, features=True)
    sc.carbon_weight = cw
    r0, t0 = po.rollout(spec, sc, load, traj=True, threads=8)
    compare(r1, r0, t1, t0)
    # features: bias, hour one-hot, and the replica count match the trajectory
    bf = configs.from_bf16_bits(f1)
    assert (bf[:, :, 0] == 1.0).all() and (bf[:, :, 10:34].sum(-1) == 1.0).all()
    assert np.array_equal(bf[1:, :, 1] * 16, t0["replicas"].astype(np.float32))


@pytest.mark.gpu
@pytest.mark.parametrize("drift", [0, 1, "cheap_large"])
def test_closed_loop_policy_parity(engine, drift):
    import torch
    from test_gpu_mlp import torch_ref
    if drift == "cheap_large":  # table launches of a type larger than the claim (SEMANTICS 3.F)
        spec, sc, load = _case(world=configs.cheap_large_world)
    else:
        spec, sc, load = _case(drift=drift)
    ws, bs = configs.mlp_weights(11)
    wb = [configs.to_bf16_bits(w) for w in ws]
    engine.set_world(spec)
    engine.set_scenarios(sc)
    engine.set_load(load)
    engine.mlp_set_weights(wb, bs)
    engine.debug_policy_features(True)
    try:
        engine.policy_rollout(trajectory=True, record=True)
        rg = engine.results()
        tg = engine.trajectory()
        at, ac = engine.policy_actions()
        fg = engine.debug_get_policy_features()
    finally:
        engine.debug_policy_features(False)
    assert engine.last_engine()[0] == 4  # the fused loop (one launch, MLP inside the step loop)
    assert at.std() > 0 and len(np.unique(at)) >= 3  # the policy really steers
    # 1. the rollout under the recorded actions and every step's features: bit-exact
    rc, tc, fc = po.rollout_policy(spec, sc, load, at, ac, traj=True, threads=THREADS, features=True)
    compare(rg, rc, tg, tc)
    bad = np.argwhere(fg != fc)
    assert bad.size == 0, f"features differ at (t, i, f) {bad[:5].tolist()}"
    # 2. the MLP on those features vs PyTorch fp32, through the action mapping
    torch.manual_seed(0)
    steps = [0, spec.n_steps // 2, spec.n_steps - 1]
    for t in steps:
        y = torch_ref(fg[t], wb, bs)
        want_t, want_c = po.policy_act(y)
        # a mismatch is allowed only where the reference sits on a rounding boundary
        near = (np.abs(np.abs(y[:, 0] * 16 - np.floor(y[:, 0] * 16)) - 0.5) < 0.05) | \
               (np.abs(np.abs(y[:, 1] * 16 - np.floor(y[:, 1] * 16)) - 0.5) < 0.05)
        ok = (want_t == at[t]) & (want_c == ac[t])
        assert (ok | near).all(), f"step {t}: {np.count_nonzero(~(ok | near))} actions off"
        assert ok.mean() > 0.98


@pytest.mark.gpu
@pytest.mark.parametrize("drift", [0, 1])
def test_closed_loop_fused_equals_launched(engine, drift):
    """The fused loop (rollout_kernel<1, 8, 1>: features, MLP and actions inside
    the step loop, one launch) against the launched loop (resumable general
    kernel + mlp_kernel + policy_act_kernel per step, as a captured hipGraph:
    first call = capture, second = replay, then direct launches): results,
    trajectories, actions, every step's features and the final MLP states are
    bit-identical; new scenarios force a fresh capture."""
    import ctypes as C
    spec, sc, load = _case(drift=drift)
    ws, bs = configs.mlp_weights(11)
    engine.set_world(spec)
    engine.set_scenarios(sc)
    engine.set_load(load)
    engine.mlp_set_weights([configs.to_bf16_bits(w) for w in ws], bs)
    fn = engine.lib.ccka_debug_policy_graph
    fn.argtypes = [C.c_void_p, C.c_int32]
    fu = engine.lib.ccka_debug_policy_fused
    fu.argtypes = [C.c_void_p, C.c_int32]
    runs = []
    engine.debug_policy_features(True)
    try:
        for fused, graph in ((1, 1), (0, 1), (0, 1), (0, 0)):
            fu(engine.ctx, fused)
            fn(engine.ctx, graph)
            engine.policy_rollout(trajectory=True, record=True)
            assert engine.last_engine()[0] == (4 if fused else 3)
            runs.append((engine.results(), engine.trajectory(), engine.policy_actions(),
                         engine.debug_get_policy_features()))
    finally:
        fu(engine.ctx, 1)
        fn(engine.ctx, 1)
        engine.debug_policy_features(False)
    for r, t, (at, ac), f in runs[1:]:
        compare(r, runs[0][0], t, runs[0][1])
        assert np.array_equal(at, runs[0][2][0]) and np.array_equal(ac, runs[0][2][1])
        assert np.array_equal(f, runs[0][3])
    # the MLP states left behind are the last step's features (ccka.h)
    engine.mlp_n = sc.n
    engine.mlp_forward()
    y_last = engine.mlp_actions()
    fu(engine.ctx, 0)
    try:
        engine.policy_rollout(trajectory=False, record=False)
        engine.mlp_forward()
        assert np.array_equal(engine.mlp_actions(), y_last)
    finally:
        fu(engine.ctx, 1)
    sc2 = configs.hpa_scenarios(sc.n, first_id=777)
    engine.set_scenarios(sc2)
    engine.set_load(load)
    engine.policy_rollout(trajectory=False, record=True)
    at2, ac2 = engine.policy_actions()
    rc = po.rollout_policy(spec, sc2, load, at2, ac2, threads=THREADS)[0]
    compare(engine.results(), rc)


def _policy_hooks(engine):
    import ctypes as C
    hooks = {}
    for name in ("ccka_debug_policy_fused", "ccka_debug_policy_table", "ccka_debug_policy_graph"):
        fn = getattr(engine.lib, name)
        fn.argtypes = [C.c_void_p, C.c_int32]
        hooks[name.rsplit("_", 1)[1]] = fn
    return hooks


@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["pool_limit", "no_table"])
@pytest.mark.parametrize("pol", [1, 2])
def test_fused_loop_catalog_scans_equal_launched(engine, variant, pol):
    """The fused loop on its catalog-scan path (no argmin tables: a world with
    NodePool CPU limits, which d1_check_world refuses, or the tables turned
    off with ccka_debug_policy_table(0)) against the launched loop, for the
    deterministic policy (POL 1) and the sampled one of the policy gradient
    (POL 2): results, trajectories, actions / sampled bins, every step's
    features and, for POL 2, the gradient are bit-identical; POL 1 also equals
    the oracle's replay of its actions."""
    spec, sc, load = _case(n=384, T=120)
    if variant == "pool_limit":
        for p in spec.pools:
            p.limit_cpu_m = 6000
    ws, bs = configs.mlp_weights(11)
    engine.set_world(spec)
    engine.set_scenarios(sc)
    engine.set_load(load)
    engine.mlp_set_weights([configs.to_bf16_bits(w) for w in ws], bs)
    h = _policy_hooks(engine)
    runs = []
    engine.debug_policy_features(True)
    try:
        h["table"](engine.ctx, 0 if variant == "no_table" else 1)
        for fused in (1, 0):
            h["fused"](engine.ctx, fused)
            if pol == 1:
                engine.policy_rollout(trajectory=True, record=True)
                extra = engine.policy_actions()
                tr = engine.trajectory()
            else:
                g, obj = engine.policy_grad(seed=3, w_carbon=0.05, w_slo=0.01)
                extra = engine.policy_samples() + (obj,)
                extra = extra + tuple(np.array(g[k]) for k in sorted(g))
                tr = None
            assert engine.last_engine()[0] == (4 if fused else 3)
            runs.append((engine.results(), tr, extra, engine.debug_get_policy_features()))
    finally:
        h["fused"](engine.ctx, 1)
        h["table"](engine.ctx, 1)
        engine.debug_policy_features(False)
    (r0, t0, x0, f0), (r1, t1, x1, f1) = runs
    compare(r1, r0, t1, t0)
    assert all(np.array_equal(a, b) for a, b in zip(x0, x1))
    assert np.array_equal(f0, f1)
    if pol == 1:
        at, ac = x0
        assert at.std() > 0
        ref = po.rollout_policy(spec, sc, load, at, ac, traj=True, threads=THREADS)
        compare(r0, ref[0], t0, ref[1])
