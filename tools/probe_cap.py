"""Probe: single-deployment engine vs oracle on a catalog whose larger type is
cheaper than the smaller one (the launch winner's pod capacity exceeds the
claim's capacity bracket). Diagnostic only."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cost-and-carbon-aware-kubernetes-autoscaler_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import pyoracle as po  # noqa: E402
from ccka import configs  # noqa: E402
from ccka.engine import Engine  # noqa: E402
from ccka.world import WorldSpec, catalog_small, carbon_intensity, price_tiles, reference_pools, deployment  # noqa: E402
from ccka import abi  # noqa: E402
from parity import compare  # noqa: E402

cat = catalog_small()
price = price_tiles(cat, 1, 3, 7)
# make every 4xlarge very cheap (spot and on-demand): it wins every claim
for k, n in enumerate(cat.names):
    if n.endswith(".4xlarge"):
        price[:, :, k, :, :] = np.maximum(price[:, :, k, :, :] // 20, 1)
spec = WorldSpec(catalog=cat, ci=carbon_intensity(1, 7), price=price, pools=reference_pools(),
                 deploys=[deployment(abi.SCALER_HPA)], n_steps=600)
sc = configs.hpa_scenarios(2000)
load = po.gen_load(configs.trace_gen(), spec.n_steps, 1, sc.n)
eng = Engine(0)
eng.set_world(spec)
eng.set_scenarios(sc)
eng.set_load(load)
eng.rollout(trajectory=True)
rg, tg = eng.results(), eng.trajectory()
print("engine", eng.last_engine())
rc, tc = po.rollout(spec, sc, load, traj=True, threads=8)
print("types chosen", sorted(set((rc["last_choice"] & 0xFFF).tolist())))
try:
    compare(rg, rc, tg, tc)
    print("PARITY OK")
except AssertionError as e:
    print("PARITY FAIL", e)
