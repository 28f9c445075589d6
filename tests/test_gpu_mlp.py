"""GPU numerics of the bf16 MFMA MLP control policy (BASELINE config 5)
against a plain PyTorch fp32 reference of the same op. The reference rounds the
hidden activations to bf16 exactly where the kernel does (the MFMA operands of
the next layer); accumulation is fp32 on both sides."""
import numpy as np
import pytest
import torch

from ccka import configs

pytestmark = pytest.mark.gpu


def torch_ref(x_bits, ws_bits, bs):
    bf = lambda a: torch.from_numpy(configs.from_bf16_bits(a))  # noqa: E731
    x = bf(x_bits)
    w1, w2, w3 = (bf(w) for w in ws_bits)
    b1, b2, b3 = (torch.from_numpy(b) for b in bs)
    h1 = torch.relu(x @ w1 + b1).to(torch.bfloat16).float()
    h2 = torch.relu(h1 @ w2 + b2).to(torch.bfloat16).float()
    return (h2 @ w3 + b3).numpy()


@pytest.mark.parametrize("n", [32 * 37 + 5, 32 * 38 + 7, 64 * 256 * 4 + 33, 31, 1])
def test_mlp_exact_integer_data(engine, n):
    """Small integers: every product, sum and bf16 activation is exact, so any
    fragment-layout / k-order error shows up as an exact mismatch. Sizes: a
    ragged last tile, an odd number of tiles (a wave's pair half empty), more
    tiles than resident waves, and single-tile batches."""
    rng = np.random.default_rng(3)
    x = rng.integers(-1, 2, size=(n, 64)).astype(np.float32)
    w1 = rng.integers(-1, 2, size=(64, 256)).astype(np.float32)
    w2 = (rng.integers(-1, 2, size=(256, 256)) * (rng.random((256, 256)) < 0.02)).astype(np.float32)
    w3 = rng.integers(-2, 3, size=(256, 8)).astype(np.float32)
    bs = [rng.integers(-3, 4, size=k).astype(np.float32) for k in (256, 256, 8)]
    wb = [configs.to_bf16_bits(w) for w in (w1, w2, w3)]
    xb = configs.to_bf16_bits(x)
    engine.mlp_set_weights(wb, bs)
    engine.mlp_set_states(xb)
    engine.mlp_forward()
    got = engine.mlp_actions()
    want = torch_ref(xb, wb, bs)
    assert np.array_equal(got, want)


def test_mlp_random_data_tolerance(engine):
    ws, bs = configs.mlp_weights(11)
    wb = [configs.to_bf16_bits(w) for w in ws]
    n = 20000
    xb = configs.to_bf16_bits(np.random.default_rng(7).standard_normal((n, 64)).astype(np.float32))
    engine.mlp_set_weights(wb, bs)
    engine.mlp_set_states(xb)
    engine.mlp_forward()
    got = engine.mlp_actions()
    want = torch_ref(xb, wb, bs)
    # fp32 accumulation order differs; a bf16 activation may round to the
    # neighbouring value when the sums differ in the last fp32 bit
    err = np.abs(got - want)
    assert err.max() <= 2e-2 * max(1.0, float(np.abs(want).max())), err.max()
    assert err.mean() <= 1e-3, err.mean()


def test_mlp_device_states(engine):
    ws, bs = configs.mlp_weights(11)
    engine.mlp_set_weights([configs.to_bf16_bits(w) for w in ws], bs)
    engine.mlp_gen_states(4096, seed=7)
    engine.mlp_forward()
    y = engine.mlp_actions()
    assert np.isfinite(y).all() and y.std() > 0
