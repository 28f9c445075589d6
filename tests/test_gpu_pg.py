"""Differentiable control (BASELINE config 5, "differentiable-control rollout";
SEMANTICS 5): the score-function gradient of the closed loop's objective.

* The MLP backward (bf16 MFMA, fp32 accumulation) against PyTorch fp32
  autograd of the same forward (bf16-rounded activations with an identity
  gradient through the rounding, as the kernel's operands): the kernel also
  rounds g_y, dH2 and dH1 to bf16 for its MFMAs, so the tolerance is bf16's.
* ccka_policy_grad is that backward applied to the loop's own rows: the
  recorded features, sampled action bins and per-scenario factors reproduce its
  gradient bit for bit through ccka_mlp_backward; the rollout under the
  sampled actions is bit-exact against the CPU oracle; the sampled bins follow
  softmax(y) and the bin -> (target, carbon weight) table.
* A few plain gradient steps lower the objective on config 2.
Parity of the sampled decisions themselves is unpinned (the reference has no
learned policy); the proposal's objective is the anchor
(CS218_Project_Proposal.pdf p.1, p.5)."""
import numpy as np
import pytest
import torch

import pyoracle as po
from ccka import configs
from parity import compare

pytestmark = pytest.mark.gpu


def torch_grads(x_bits, actions, coef, ws_bits, bs):
    """d/dW of sum_m coef[m] * log_softmax(policy(x_m))[a_m] in fp32 autograd."""
    bf = lambda a: torch.from_numpy(configs.from_bf16_bits(a))  # noqa: E731
    x = bf(x_bits)
    w = [bf(wb).clone().requires_grad_(True) for wb in ws_bits]
    b = [torch.from_numpy(np.asarray(v, np.float32)).clone().requires_grad_(True) for v in bs]

    def rnd(h):  # the kernel's bf16 operand, identity gradient
        return h + (h.to(torch.bfloat16).float() - h).detach()

    h1 = torch.relu(rnd(x @ w[0] + b[0]))
    h2 = torch.relu(rnd(h1 @ w[1] + b[1]))
    y = h2 @ w[2] + b[2]
    lp = torch.log_softmax(y, dim=1)
    a = torch.from_numpy(np.asarray(actions, np.int64))
    loss = (torch.from_numpy(np.asarray(coef, np.float32)) * lp[torch.arange(len(a)), a]).sum()
    loss.backward()
    return {"w1": w[0].grad.numpy(), "w2": w[1].grad.numpy(), "w3": w[2].grad.numpy(),
            "b1": b[0].grad.numpy(), "b2": b[1].grad.numpy(), "b3": b[2].grad.numpy()}


def rel_err(got, want):
    return float(np.linalg.norm(got - want) / max(np.linalg.norm(want), 1e-30))


@pytest.mark.parametrize("m", [1, 31, 32 * 37 + 5, 20000])
def test_mlp_backward_matches_torch_autograd(engine, m):
    rng = np.random.default_rng(m)
    ws, bs = configs.mlp_weights(11)
    wb = [configs.to_bf16_bits(w) for w in ws]
    engine.mlp_set_weights(wb, bs)
    x = configs.to_bf16_bits(rng.standard_normal((m, 64)).astype(np.float32))
    act = rng.integers(0, 8, size=m).astype(np.uint8)
    coef = rng.standard_normal(m).astype(np.float32) / m
    got = engine.mlp_backward(x, act, coef)
    want = torch_grads(x, act, coef, wb, bs)
    for k in want:
        assert got[k].shape == want[k].shape
        e = rel_err(got[k], want[k])
        assert e <= 2e-2, f"{k}: relative error {e:.3e}"


@pytest.mark.parametrize("chunk", [4096, 32 * 37])
def test_mlp_backward_row_chunks(engine, chunk):
    """Row chunks (the backward of N*T rows too many for one work buffer runs
    in chunks of 2^23 rows, each chunk's gradient added in chunk order): with a
    small chunk size forced, 20,000 rows in 5 / 17 chunks give the autograd
    gradient within the same bf16 tolerance and the unchunked kernel's within
    fp32 summation-order rounding; repeated runs are bit-identical."""
    import ctypes as C
    rng = np.random.default_rng(7)
    m = 20000
    ws, bs = configs.mlp_weights(11)
    wb = [configs.to_bf16_bits(w) for w in ws]
    engine.mlp_set_weights(wb, bs)
    x = configs.to_bf16_bits(rng.standard_normal((m, 64)).astype(np.float32))
    act = rng.integers(0, 8, size=m).astype(np.uint8)
    coef = rng.standard_normal(m).astype(np.float32) / m
    whole = engine.mlp_backward(x, act, coef)
    fn = engine.lib.ccka_debug_pg_chunk
    fn.argtypes = [C.c_void_p, C.c_int64]
    assert fn(engine.ctx, chunk) == 0
    try:
        got = engine.mlp_backward(x, act, coef)
        again = engine.mlp_backward(x, act, coef)
    finally:
        fn(engine.ctx, 0)
    want = torch_grads(x, act, coef, wb, bs)
    for k in want:
        assert rel_err(got[k], want[k]) <= 2e-2, k
        assert rel_err(got[k], whole[k]) <= 1e-5, k
        assert np.array_equal(got[k], again[k]), k


def test_mlp_backward_single_row_structure(engine):
    """One row with coef 1: every gradient is a rank-1 outer product; a
    fragment or k-order error would break it far beyond bf16 rounding."""
    ws, bs = configs.mlp_weights(5)
    wb = [configs.to_bf16_bits(w) for w in ws]
    engine.mlp_set_weights(wb, bs)
    x = configs.to_bf16_bits(np.random.default_rng(1).standard_normal((1, 64)).astype(np.float32))
    for a in (0, 3, 7):
        got = engine.mlp_backward(x, np.array([a], np.uint8), np.array([1.0], np.float32))
        want = torch_grads(x, [a], [1.0], wb, bs)
        for k in want:
            assert rel_err(got[k], want[k]) <= 2e-2, k
        # d/dy of log softmax sums to zero over the actions
        assert abs(float(got["b3"].sum())) <= 1e-2 * float(np.abs(got["b3"]).sum())


def _loop_case(n=1024, T=120):
    spec = configs.config2_world(n_steps=T)
    sc = configs.hpa_scenarios(n, first_id=7)
    load = po.gen_load(configs.trace_gen(5), T, 1, n, first_id=7)
    return spec, sc, load


def test_policy_grad_is_the_backward_of_its_own_rows(engine):
    spec, sc, load = _loop_case()
    ws, bs = configs.mlp_weights(11)
    wb = [configs.to_bf16_bits(w) for w in ws]
    engine.set_world(spec)
    engine.set_scenarios(sc)
    engine.set_load(load)
    engine.mlp_set_weights(wb, bs)
    g, obj = engine.policy_grad(seed=123, w_carbon=0.5, w_slo=0.01)
    act, coef = engine.policy_samples()
    feats = engine.debug_get_policy_features()
    tg, cw = engine.policy_actions()
    rg = engine.results()
    # the objective and the factors (J - mean J) / N from the results
    J = rg["cost_uphmin"] / 6e7 + 0.5 * rg["gco2"] * 1e-3 + 0.01 * rg["slo_minutes"]
    assert obj == pytest.approx(J.mean(), rel=1e-12)
    assert np.allclose(coef, ((J - J.mean()) / sc.n).astype(np.float32), rtol=1e-6, atol=1e-12)
    # the bin table: target 40 + 10 (a & 3) %, carbon weight a >> 2
    assert np.array_equal(tg, 40 + 10 * (act.astype(np.int16) & 3))
    assert np.array_equal(cw, (act >> 2).astype(np.float64))
    assert len(np.unique(act)) == 8
    # the same rows through the standalone backward: bit-identical gradient
    T, n = spec.n_steps, sc.n
    rows_x = feats[:T].reshape(T * n, 64)
    rows_c = np.tile(coef, T)
    g2 = engine.mlp_backward(rows_x, act.reshape(-1), rows_c)
    for k in g:
        assert np.array_equal(g[k], g2[k]), k
    # and within bf16 tolerance of PyTorch autograd on those rows
    want = torch_grads(rows_x, act.reshape(-1), rows_c, wb, bs)
    for k in want:
        assert rel_err(g[k], want[k]) <= 2e-2, k
    # the rollout under the sampled actions and every step's features: bit-exact
    # against the oracle
    rc, _, fc = po.rollout_policy(spec, sc, load, tg, cw, threads=16, features=True)
    compare(rg, rc)
    assert np.array_equal(feats, fc)


def test_policy_sampling_follows_softmax_and_seed(engine):
    from test_gpu_mlp import torch_ref
    spec, sc, load = _loop_case(n=4096, T=30)
    ws, bs = configs.mlp_weights(11)
    ws[2] = ws[2] * 4.0  # sharper logits: a non-uniform policy
    wb = [configs.to_bf16_bits(w) for w in ws]
    engine.set_world(spec)
    engine.set_scenarios(sc)
    engine.set_load(load)
    engine.mlp_set_weights(wb, bs)
    engine.policy_grad(seed=9)
    a1, _ = engine.policy_samples()
    feats = engine.debug_get_policy_features()
    engine.policy_grad(seed=9)
    a2, _ = engine.policy_samples()
    assert np.array_equal(a1, a2)  # counter-based: same seed, same samples
    engine.policy_grad(seed=10)
    a3, _ = engine.policy_samples()
    assert (a1 != a3).mean() > 0.2
    # empirical bin frequencies vs the mean softmax probabilities of the rows
    y = torch_ref(feats[:spec.n_steps].reshape(-1, 64), wb, bs)
    pr = torch.softmax(torch.from_numpy(y), dim=1).numpy()
    f = np.bincount(a1.reshape(-1), minlength=8) / a1.size
    assert np.abs(f - pr.mean(0)).max() < 0.01, (f, pr.mean(0))
    # each sample against the oracle's Philox draw: u lies in its bin of the
    # cumulative softmax (PyTorch's y may differ from the kernel's in the last
    # bits, so a draw within 1e-4 of a bin edge may land in the neighbour)
    for t in (0, spec.n_steps - 1):
        u = po.policy_uniform(9, sc.first_id + np.arange(sc.n), t)
        cum = np.cumsum(pr[t * sc.n:(t + 1) * sc.n], axis=1)
        a = a1[t].astype(np.int64)
        lo = np.where(a > 0, cum[np.arange(sc.n), np.maximum(a - 1, 0)], 0.0)
        hi = cum[np.arange(sc.n), a]
        inside = (u >= lo - 1e-4) & (u < hi + 1e-4)
        assert inside.all(), np.nonzero(~inside)[0][:10]
        assert ((u >= lo) & (u < hi)).mean() > 0.999


def test_gradient_steps_lower_the_objective(engine):
    """Plain gradient descent on E[J] (config 2, 2048 scenarios x 120 steps,
    cost + 0.02 $ per SLO-minute): the mean objective after a few steps is
    below the first one's."""
    spec, sc, load = _loop_case(n=2048, T=120)
    ws, bs = configs.mlp_weights(11)
    engine.set_world(spec)
    engine.set_scenarios(sc)
    engine.set_load(load)
    objs = []
    lr = 0.5
    for it in range(6):
        engine.mlp_set_weights([configs.to_bf16_bits(w) for w in ws], bs)
        g, obj = engine.policy_grad(seed=1000 + it, w_slo=0.02)
        objs.append(obj)
        ws = [ws[0] - lr * g["w1"], ws[1] - lr * g["w2"], ws[2] - lr * g["w3"]]
        bs = [bs[0] - lr * g["b1"], bs[1] - lr * g["b2"], bs[2] - lr * g["b3"]]
    assert min(objs[-2:]) < objs[0], objs
