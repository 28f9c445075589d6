"""BASELINE.json workload configurations.

Per-scenario parameters are pure functions of the GLOBAL scenario id
(splitmix64), so any sharding of scenarios over ranks yields identical
per-scenario inputs and therefore identical results.
"""
from __future__ import annotations

import numpy as np

from . import abi
from .world import (ScenarioSet, WorldSpec, burst_deployments, carbon_intensity, catalog_small,
                    catalog_synth, catalog_tiny, deployment, price_tiles, reference_pools)

SEED = 20251205


def splitmix32(ids: np.ndarray, salt: int) -> np.ndarray:
    """uint32 hash of uint64 ids (splitmix64 finaliser), vectorised."""
    with np.errstate(over="ignore"):
        z = (ids.astype(np.uint64) + np.uint64(salt) * np.uint64(0x9E3779B97F4A7C15))
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return (z >> np.uint64(32)).astype(np.uint32)


def trace_gen(seed: int = SEED) -> abi.TraceGen:
    """config 2 load: base U[500,5000] m, diurnal amplitude U[0.2,0.8], 5 % noise,
    p=0.5 burst x3 for 30 min."""
    g = abi.TraceGen()
    g.seed = seed
    g.base_lo, g.base_hi = 500, 5000
    g.amp_lo_pm, g.amp_hi_pm = 200, 800
    g.noise_pm = 50
    g.burst_prob_pm, g.burst_mult_pm, g.burst_len = 500, 3000, 30
    return g


def hpa_scenarios(n: int, first_id: int = 0, n_regions: int = 1, region_block: int | None = None,
                  carbon=None) -> ScenarioSet:
    ids = np.arange(first_id, first_id + n, dtype=np.uint64)
    tgt = np.array([50, 60, 70, 80], np.int16)[splitmix32(ids, 1) % 4]
    mx = (20 + splitmix32(ids, 2) % 81).astype(np.int16)
    # demo_30_burst_configure.sh:59-71: odd deployments select spot, even on-demand
    cap = np.where(ids % 2 == 0, abi.CAP_SPOT, abi.CAP_OD).astype(np.uint8)
    if region_block:
        reg = np.minimum(ids // np.uint64(region_block), n_regions - 1).astype(np.uint8)
    else:
        reg = np.zeros(n, np.uint8)
    cw = None
    if carbon is not None:
        cw = np.asarray(carbon, np.float64)[splitmix32(ids, 3) % len(carbon)]
    return ScenarioSet(n, first_id, region=reg, target_util_pct=tgt, max_replicas=mx,
                       cap_sel=cap, carbon_weight=cw)


def config2_world(n_steps: int = 1440, max_nodes: int = 8) -> WorldSpec:
    """1e5 clusters x 1 deployment x 1440 one-minute steps, HPA + peak/off-peak."""
    cat = catalog_small()
    return WorldSpec(catalog=cat, ci=carbon_intensity(1, SEED), price=price_tiles(cat, 1, 3, SEED),
                     pools=reference_pools(), deploys=[deployment(abi.SCALER_HPA)],
                     n_steps=n_steps, max_nodes=max_nodes)


def cheap_large_world(n_steps: int = 600, max_nodes: int = 8) -> WorldSpec:
    """config 2 with every 4xlarge offering at 1/20 of its price: a claim of a
    few pods launches a type far larger than it needs, so a launched node's pod
    capacity (its type's) exceeds the claim's capacity bracket (regression
    world for the argmin tables, SEMANTICS 3.F)."""
    cat = catalog_small()
    price = price_tiles(cat, 1, 3, SEED)
    for k, name in enumerate(cat.names):
        if name.endswith(".4xlarge"):
            price[:, :, k] = np.maximum(price[:, :, k] // 20, 1)
    return WorldSpec(catalog=cat, ci=carbon_intensity(1, SEED), price=price, pools=reference_pools(),
                     deploys=[deployment(abi.SCALER_HPA)], n_steps=n_steps, max_nodes=max_nodes)


def config3_world(n_steps: int = 1440, max_nodes: int = 8) -> WorldSpec:
    """8 regions x ~800-type catalog, Karpenter argmin with carbon weight."""
    cat = catalog_synth(800, SEED)
    return WorldSpec(catalog=cat, ci=carbon_intensity(8, SEED),
                     price=price_tiles(cat, 8, 3, SEED, avail=0.9),
                     pools=reference_pools(), deploys=[deployment(abi.SCALER_HPA)],
                     n_steps=n_steps, max_nodes=max_nodes)


CONFIG3_REGION_BLOCK = 125_000
CONFIG3_CARBON = (0.0, 0.5, 1.0, 2.0)


def config3_scenarios(n: int, first_id: int = 0) -> ScenarioSet:
    return hpa_scenarios(n, first_id, 8, CONFIG3_REGION_BLOCK, CONFIG3_CARBON)


def config1_world() -> WorldSpec:
    """Replay of demo_20/21/30: 12 burst Deployments x 5 replicas on a 3-node
    cluster, reset -> off-peak at t=0 -> peak 16:00-21:00, T=1440."""
    cat = catalog_tiny()
    return WorldSpec(catalog=cat, ci=carbon_intensity(1, SEED), price=price_tiles(cat, 1, 3, SEED),
                     pools=reference_pools(), deploys=burst_deployments(12, 5), n_steps=1440,
                     max_nodes=16)


# ---------------------------------------------------------------------------
# config 4: policy sweep, 4096 grids x 1024 shared load traces
# ---------------------------------------------------------------------------
CONFIG4_GRIDS = 4096
CONFIG4_TRACES = 1024
CONFIG4_CA = (30, 60, 120, 300)
CONFIG4_CARBON = (0.0, 0.5, 1.0, 2.0)


def config4_grid_params(grids: np.ndarray) -> dict:
    """16 target utilisations (40..85 %) x 8 down-stabilisation windows (0..420 s)
    x 4 consolidateAfter x 4 carbon weights x peak switch on/off = 4096 grids."""
    g = np.asarray(grids, np.int64)
    return {
        "target_util_pct": (40 + 3 * (g % 16)).astype(np.int16),
        "down_stab_s": (60 * ((g // 16) % 8)).astype(np.int16),
        "reset_ca_s": np.asarray(CONFIG4_CA, np.int16)[(g // 128) % 4],
        "carbon_weight": np.asarray(CONFIG4_CARBON, np.float64)[(g // 512) % 4],
        "peak_switch": (1 - (g // 2048) % 2).astype(np.uint8),
    }


def config4_scenarios(grid_lo: int, n_grids: int, n_traces: int = CONFIG4_TRACES) -> ScenarioSet:
    """Grids [grid_lo, grid_lo + n_grids) x n_traces shared traces; scenario
    global id = grid * n_traces + trace (shard by grid: SURVEY.md 8(e))."""
    first = grid_lo * n_traces
    ids = np.arange(first, first + n_grids * n_traces, dtype=np.int64)
    prm = config4_grid_params(ids // n_traces)
    trace = ids % n_traces
    cap = np.where(trace % 2 == 0, abi.CAP_SPOT, abi.CAP_OD).astype(np.uint8)
    return ScenarioSet(len(ids), first, n_traces, cap_sel=cap, **prm)


def config4_trace_gen() -> abi.TraceGen:
    return trace_gen(SEED + 1)


# ---------------------------------------------------------------------------
# config 5: learned MLP control policy 64 -> 256 -> 256 -> 8 (bf16)
# ---------------------------------------------------------------------------
MLP_SHAPE = (64, 256, 256, 8)


def mlp_weights(seed: int = 11):
    """Xavier-uniform weights (fp32), zero-mean small biases; row-major [in][out]."""
    rng = np.random.default_rng(seed)
    dims = MLP_SHAPE
    ws, bs = [], []
    for a, b in zip(dims[:-1], dims[1:]):
        lim = np.sqrt(6.0 / (a + b))
        ws.append(rng.uniform(-lim, lim, size=(a, b)).astype(np.float32))
        bs.append(rng.uniform(-0.05, 0.05, size=b).astype(np.float32))
    return ws, bs


def to_bf16_bits(a: np.ndarray) -> np.ndarray:
    """float32 -> bf16 bit patterns (round to nearest even), as uint16."""
    u = np.ascontiguousarray(a, np.float32).view(np.uint32).astype(np.uint64)
    r = (u + 0x7FFF + ((u >> 16) & 1)) >> 16
    return r.astype(np.uint16)


def from_bf16_bits(b: np.ndarray) -> np.ndarray:
    return (np.asarray(b, np.uint32) << 16).view(np.float32)
