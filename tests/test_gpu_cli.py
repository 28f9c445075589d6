"""GPU: the drop-in CLI (`ccka replay`, manifests in -> summary out) against the
oracle on the world the host library builds from the same manifests
(BASELINE config 1: demo_20/21/30 replay, 12 burst Deployments, 3 base nodes)."""
import json
import os
import subprocess

import numpy as np
import pytest

import pyoracle as po
from ccka.host import CLI, Host
from ccka.world import ScenarioSet
from parity import INT_FIELDS

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("load_m,catalog,drift", [(100, "tiny", 0), (450, "small", 0), (450, "small", 1),
                                                            (450, "small", 3)])
def test_cli_replay_matches_oracle(tmp_path, load_m, catalog, drift):
    out = tmp_path / "r.json"
    env = {k: v for k, v in os.environ.items() if k not in ("COUNT", "REPLICAS", "NP_SPOT", "NP_OD")}
    prom = tmp_path / "r.prom"
    txt = subprocess.run([CLI, "replay", "--catalog", catalog, "--load-m", str(load_m), "--json", str(out),
                          "--prom", str(prom)] + (["--drift"] if drift & 1 else [])
                         + (["--replace"] if drift & 2 else []),
                         env=env, check=True, capture_output=True, text=True, timeout=120).stdout
    assert "cost=$" in txt and "spot-preferred" in txt
    got = json.load(open(out))
    h = Host()
    h.apply(h.manifest(-1))
    for i in range(1, 13):
        h.apply(h.manifest(i))
    h.apply(h.manifest(0))
    w = h.build_world(catalog, 1440, 16)
    w.disrupt_ext = drift
    load = np.full((1440, 12, 1), load_m, np.int32)
    want, _ = po.rollout_world(w, ScenarioSet(1), load)
    for f in INT_FIELDS:
        assert got[f] == int(want[f][0]), f
    for f in ("energy_wmin", "gco2"):
        assert got[f] == float(want[f][0]), f
    # the exported run totals are the same results
    lines = [ln for ln in open(prom).read().splitlines() if ln.startswith("ccka_launches_total{")]
    assert len(lines) == 1 and float(lines[0].split()[1]) == got["launches"]
