"""A/B of the standalone MLP forward's MFMA tile (mlp_kernel 32x32x16 vs
mlp16_kernel 16x16x32) on config 5 (1e7 states), interleaved in one process:
mean kernel ms over 20 back-to-back launches (HIP events), TFLOP/s, and the
largest output difference between the two (fp32 summation orders differ).
usage: [VARIANT=name] python tools/mlp_ab.py [n]"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cost-and-carbon-aware-kubernetes-autoscaler_amd"))
from ccka import configs  # noqa: E402
from ccka.engine import Engine  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
lib = os.environ.get("VARIANT")
e = Engine(0, lib_path=os.path.join(ROOT, "cost-and-carbon-aware-kubernetes-autoscaler_amd", "csrc", "build", "variants",
                                    lib, "libccka.so")) if lib else Engine(0)
ws, bs = configs.mlp_weights(11)
e.mlp_set_weights([configs.to_bf16_bits(w) for w in ws], bs)
e.mlp_gen_states(n, seed=7)
tile = e.lib.ccka_debug_mlp_tile
tile.argtypes = [C.c_void_p, C.c_int32]
batch = e.lib.ccka_debug_mlp_batch
batch.argtypes = [C.c_void_p, C.c_int32, C.POINTER(C.c_double), C.POINTER(C.c_double)]
flops = 2 * (64 * 256 + 256 * 256 + 256 * 8) * n
out = {}
for rnd in range(3):
    for t in (32, 16):
        assert tile(e.ctx, t) == 0
        avg, span = C.c_double(), C.c_double()
        assert batch(e.ctx, 50 if rnd == 0 else 20, C.byref(avg), C.byref(span)) == 0
        if rnd == 0:
            e.mlp_forward()
            out[t] = e.mlp_actions().copy()
        else:
            print(f"tile {t}: {avg.value:.4f} ms  {flops / avg.value / 1e9:.0f} TFLOP/s "
                  f"({flops / avg.value / 1e9 / 2500:.1%} of 2.5 PF)", flush=True)
d = np.abs(out[16] - out[32])
print(f"max |y16 - y32| = {d.max():.3g}, mean {d.mean():.3g}, bit-identical {np.mean(out[16] == out[32]):.3f}")
