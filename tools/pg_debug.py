"""Diagnostic: the policy-gradient backward's intermediate unit-major arrays
against PyTorch (which stage disagrees). Profiling/debug aid only."""
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cost-and-carbon-aware-kubernetes-autoscaler_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
from ccka import configs  # noqa: E402
from ccka.engine import Engine  # noqa: E402
from test_gpu_pg import rel_err, torch_grads  # noqa: E402

eng = Engine(0)
ws, bs = configs.mlp_weights(11)
wb = [configs.to_bf16_bits(w) for w in ws]
eng.mlp_set_weights(wb, bs)
for m in (1, 40, 5000):
    rng = np.random.default_rng(m)
    x = configs.to_bf16_bits(rng.standard_normal((m, 64)).astype(np.float32))
    act = rng.integers(0, 8, size=m).astype(np.uint8)
    coef = (rng.standard_normal(m) / m).astype(np.float32)
    got = eng.mlp_backward(x, act, coef)
    want = torch_grads(x, act, coef, wb, bs)
    print(m, {k: round(rel_err(got[k], want[k]), 4) for k in want}, flush=True)
    rows = 64 + 4 * 256 + 9
    mp_guess = (m + 31) // 32 * 32
    buf = np.zeros(rows * mp_guess + 64, np.uint16)
    mp = C.c_int64()
    fn = eng.lib.ccka_debug_pg_work
    fn.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.POINTER(C.c_int64)]
    rc = fn(eng.ctx, buf.ctypes.data, buf.size, C.byref(mp))
    if rc:
        print("work fetch rc", rc)
        continue
    Mp = mp.value
    wk = buf[:rows * Mp].reshape(rows, Mp)
    f = lambda a: configs.from_bf16_bits(a)  # noqa: E731
    xT, h1T, h2T, dh1T, dh2T, gyT = (wk[0:64], wk[64:320], wk[320:576], wk[576:832], wk[832:1088], wk[1088:1096])
    xf = torch.from_numpy(f(x))
    W = [torch.from_numpy(f(w)) for w in wb]
    B = [torch.from_numpy(b) for b in bs]
    h1 = torch.relu(xf @ W[0] + B[0]).to(torch.bfloat16).float()
    h2 = torch.relu(h1 @ W[1] + B[1]).to(torch.bfloat16).float()
    y = h2 @ W[2] + B[2]
    p = torch.softmax(y, 1)
    gy = torch.from_numpy(coef)[:, None] * (torch.nn.functional.one_hot(torch.from_numpy(act.astype(np.int64)), 8) - p)
    dh2 = (gy @ W[2].T) * (h2 > 0)
    dh1 = (dh2 @ W[1].T) * (h1 > 0)
    for name, got_a, want_a in (("xT", xT, xf), ("h1T", h1T, h1), ("h2T", h2T, h2), ("gyT", gyT, gy),
                                ("dh2T", dh2T, dh2), ("dh1T", dh1T, dh1)):
        g = f(got_a[:, :m]).T
        print("  ", name, round(rel_err(g, want_a.numpy()), 4), flush=True)
    if m == 5000:
        # the matrix the kernel applied: dh2_got[s][u] = sum_a M[u][a] gy[s][a] on unmasked entries
        g = f(dh2T[:, :m]).T
        gyn = gy.numpy()
        W3 = W[2].numpy()
        mask = (h2 > 0).numpy()
        for u in (0, 1, 4, 5, 8, 16, 17, 33, 100):
            sel = mask[:, u]
            M, *_ = np.linalg.lstsq(gyn[sel], g[sel, u], rcond=None)
            print("   unit", u, "applied", np.round(M, 3).tolist(), "W3", np.round(W3[u], 3).tolist(), flush=True)
        nomask = (gy @ W[2].T).numpy()
        print("   vs unmasked", round(rel_err(g, nomask), 4), "masked-entry nonzero frac",
              float((g[~mask] != 0).mean()), "unmasked-entry zero frac", float((g[mask] == 0).mean()), flush=True)
        want2 = nomask * mask
        bad = np.abs(g - want2) > 0.02 * np.abs(want2).max()
        print("   bad entries", int(bad.sum()), "of", bad.size, "units with bad", np.unique(np.nonzero(bad)[1])[:40].tolist())
        print("   states with bad", np.unique(np.nonzero(bad)[0])[:20].tolist())
