"""Phase cycles of the MLP policy kernel (config 5): layer 1 vs layers 2+3,
per 64-state pair and wave, against the MFMA floor of each phase
(32 cycles per v_mfma_f32_32x32x16_bf16)."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cost-and-carbon-aware-kubernetes-autoscaler_amd"))
from ccka import configs  # noqa: E402
from ccka.engine import Engine  # noqa: E402

N = 10_000_000
eng = Engine(0)
ws, bs = configs.mlp_weights()
eng.mlp_set_weights([configs.to_bf16_bits(w) for w in ws], bs)
eng.mlp_gen_states(N)
eng.mlp_forward()
plain = []
for _ in range(10):
    eng.mlp_forward()
    plain.append(eng.kernel_ms())
eng.lib.ccka_debug_mlp_stamps.argtypes = [C.c_void_p, C.c_int32]
eng.lib.ccka_debug_stamps.argtypes = [C.c_void_p, C.POINTER(C.c_ulonglong)]
eng.lib.ccka_debug_mlp_stamps(eng.ctx, 1)
stamped = []
for _ in range(10):
    eng.mlp_forward()
    stamped.append(eng.kernel_ms())
buf = (C.c_ulonglong * 12)()
eng.lib.ccka_debug_stamps(eng.ctx, buf)
eng.lib.ccka_debug_mlp_stamps(eng.ctx, 0)
pairs = (N + 63) // 64
l1, l23 = buf[0] / pairs, buf[1] / pairs
print(f"layer 1: {l1:8.0f} cycles/pair (MFMA floor {64 * 32}), layers 2+3: {l23:8.0f} (floor {288 * 32}), "
      f"wave {buf[2] / 1024:.0f} cycles at {buf[2] / buf[3] * 0.1:.3f} GHz, "
      f"kernel {min(stamped):.3f}..{max(stamped):.3f} ms stamped, {min(plain):.3f}..{max(plain):.3f} ms plain")
print("plain  ", " ".join(f"{x:.3f}" for x in plain))
print("stamped", " ".join(f"{x:.3f}" for x in stamped))
eng.lib.ccka_debug_mlp_stamps(eng.ctx, 0)
alt = []
for k in range(20):
    eng.lib.ccka_debug_mlp_stamps(eng.ctx, k & 1)
    eng.mlp_forward()
    alt.append(eng.kernel_ms())
print("alternating plain/stamped", " ".join(f"{x:.3f}" for x in alt))
eng.lib.ccka_debug_mlp_stamps(eng.ctx, 0)
b2b = []
for k in range(20):
    eng.mlp_forward_async()
for k in range(20):
    eng.mlp_forward_async()
    eng.sync()
    b2b.append(eng.kernel_ms())
print("plain after 20 back-to-back launches", " ".join(f"{x:.3f}" for x in b2b))
