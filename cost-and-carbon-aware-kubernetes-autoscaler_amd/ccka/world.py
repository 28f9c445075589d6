"""World / scenario builders (host side).

The policy defaults below are the values the reference's scripts emit
(pinned by tests/golden/reference_capture, see tests/test_golden_capture.py):

* pools ``spot-preferred`` / ``on-demand-slo``           demo_00_env.sh:18-19
* zones off-peak ``us-east-2a`` / peak ``us-east-2c``    demo_00_env.sh:22-23
* RESET WhenEmpty/30s on both pools                      demo_19_reset_policies.sh:68-75
* OFFPEAK spot WhenEmptyOrUnderutilized (keep ca),
  OD WhenEmpty/60s                                       demo_20_offpeak_configure.sh:59-60
* PEAK both WhenEmpty/120s                               demo_21_peak_configure.sh:56-57
* capacity types spot pool {spot,on-demand}, OD pool
  {on-demand}, identical in both profiles                demo_20_offpeak_configure.sh:74-78
* burst pods 200m/128Mi requests, 500m limit, nodeSelector
  alternating spot / on-demand, replicas 5               demo_30_burst_configure.sh:57-140
* PDB minAvailable 50%                                   demo_10_setup_configure.sh:47-56
* base managed group 3 x m6i.large                       01_cluster.sh:24-30, .env:5-8

The catalog, price tiles and carbon-intensity traces are synthetic (the
reference discovers them at run time through Karpenter's AWS provider,
05_karpenter.sh:64-75; there is no network here).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

import numpy as np

from . import abi

# power model defaults (cloud-carbon-footprint AWS coefficients)
W_MIN_PER_VCPU = 0.74
W_MAX_PER_VCPU = 3.5
PUE = 1.135
DEFAULT_CI = 400.0  # gCO2/kWh, .env:14 "dummy ~400 g/kWh"

NP_SPOT = "spot-preferred"
NP_OD = "on-demand-slo"


def llround(x: float) -> int:
    """C llround: nearest integer, halves away from zero."""
    import math
    return int(math.copysign(math.floor(abs(x) + 0.5), x))


def zone_bit(zone: str) -> int:
    """'us-east-2a' -> bit 0, 'b' -> bit 1, ..."""
    return 1 << (ord(zone.strip()[-1]) - ord("a"))


def zone_mask(zones) -> int:
    m = 0
    for z in zones:
        m |= zone_bit(z)
    return m


def hpa_rules(select=abi.SELECT_MAX, policies=(), stab=0):
    r = abi.HpaRules()
    r.select = select
    r.n_policies = len(policies)
    r.stab_window_s = stab
    for i, (ty, val, per) in enumerate(policies):
        r.policies[i].type = ty
        r.policies[i].value = val
        r.policies[i].period_s = per
    return r


def default_up():  # autoscaling/v2 defaults: max(+4 pods, +100%) per 15 s, no stabilisation
    return hpa_rules(abi.SELECT_MAX, [(abi.HPA_PERCENT, 100, 15), (abi.HPA_PODS, 4, 15)], 0)


def default_down(stab=300):  # 100% per 15 s, 300 s stabilisation
    return hpa_rules(abi.SELECT_MAX, [(abi.HPA_PERCENT, 100, 15)], stab)


@dataclass
class Catalog:
    names: list
    vcpu: np.ndarray
    mem_gib: np.ndarray
    max_pods: np.ndarray
    od_uph: np.ndarray  # on-demand price, micro-dollars per hour

    @property
    def k(self):
        return len(self.names)

    def alloc(self):
        """EKS/Karpenter default kube-reserved + eviction + VM overhead."""
        v = self.vcpu.astype(np.int64)
        res = np.zeros_like(v)
        # cpu reservation: 6% of core 1, 1% of core 2, 0.5% cores 3-4, 0.25% beyond (millicores)
        res += 60
        res += np.where(v >= 2, 10, 0)
        res += np.clip(v - 2, 0, 2) * 5
        res += np.clip(v - 4, 0, None) * 25 // 10
        alloc_cpu = v * 1000 - res
        mem_mi = (self.mem_gib * 1024).astype(np.int64)
        alloc_mem = (mem_mi * 925) // 1000 - (11 * self.max_pods.astype(np.int64) + 255) - 100
        return alloc_cpu.astype(np.int32), alloc_mem.astype(np.int32)

    def itypes(self):
        ac, am = self.alloc()
        arr = (abi.ItType * self.k)()
        for i in range(self.k):
            v = int(self.vcpu[i])
            t = arr[i]
            t.vcpu = v
            t.alloc_cpu_m = int(ac[i])
            t.alloc_mem_mi = int(am[i])
            t.max_pods = int(self.max_pods[i])
            p_idle = float(v) * W_MIN_PER_VCPU * PUE
            p_dyn = float(v) * (W_MAX_PER_VCPU - W_MIN_PER_VCPU) * PUE
            t.idle_nw = llround(p_idle * 1e9)
            t.dyn_nw_per_m = llround(p_dyn * 1e9 / float(t.alloc_cpu_m))
            t.p_ref_w = p_idle + 0.5 * p_dyn
            t.mem_mi = int(self.mem_gib[i] * 1024)
        return arr

    def index(self, name):
        return self.names.index(name)


_SIZES = [("large", 2), ("xlarge", 4), ("2xlarge", 8), ("4xlarge", 16)]
_ENI_PODS = {2: 29, 4: 58, 8: 58, 16: 234}


def catalog_small() -> Catalog:
    """16 real-ish us-east-2 types: {m6i, c6i, r6i, m7i} x {large..4xlarge}."""
    fam = [("m6i", 4, 96000), ("c6i", 2, 85000), ("r6i", 8, 126000), ("m7i", 4, 100800)]
    names, vcpu, mem, pods, od = [], [], [], [], []
    for f, gib_per_vcpu, uph_large in fam:
        for s, v in _SIZES:
            names.append(f"{f}.{s}")
            vcpu.append(v)
            mem.append(v * gib_per_vcpu)
            pods.append(_ENI_PODS[v])
            od.append(uph_large * v // 2)
    return Catalog(names, np.array(vcpu, np.int32), np.array(mem, np.float64),
                   np.array(pods, np.int32), np.array(od, np.int64))


def catalog_tiny() -> Catalog:
    """config 1 catalog: m6i/c6i/r6i x {large, xlarge, 2xlarge, 4xlarge} (12 types)."""
    c = catalog_small()
    keep = [i for i, n in enumerate(c.names) if not n.startswith("m7i")]
    return Catalog([c.names[i] for i in keep], c.vcpu[keep], c.mem_gib[keep], c.max_pods[keep],
                   c.od_uph[keep])


def catalog_synth(k: int = 800, seed: int = 20251205) -> Catalog:
    """~800-type synthetic catalog: vCPU in
    {1..192}, 2/4/8 GiB per vCPU, OD price = vCPU x base x family multiplier.
    m6i.large is forced to index 0 so the base node group is present."""
    rng = np.random.default_rng(seed)
    vcpus = [1, 2, 4, 8, 16, 32, 48, 64, 96, 128, 192]
    ratios = [2, 4, 8]
    names = ["m6i.large"]
    vcpu, mem, pods, od = [2], [8.0], [29], [96000]
    fam = 0
    while len(names) < k:
        mult = 0.8 + 0.5 * rng.random()
        ratio = ratios[fam % 3]
        for v in vcpus:
            if len(names) >= k:
                break
            names.append(f"x{fam:02d}{'cmr'[fam % 3]}.{v}xl")
            vcpu.append(v)
            mem.append(float(v * ratio))
            pods.append(min(737, 8 + 14 * v if v < 16 else 234 if v < 48 else 737))
            base = {2: 21250, 4: 24000, 8: 31500}[ratio]
            od.append(int(v * base * mult))
        fam += 1
    return Catalog(names, np.array(vcpu, np.int32), np.array(mem, np.float64),
                   np.array(pods, np.int32), np.array(od, np.int64))


def price_tiles(cat: Catalog, n_regions: int, n_zones: int = 3, seed: int = 20251205,
                avail: float = 1.0) -> np.ndarray:
    """int32 [R][24][K][Z][2] micro-$/h; c=0 spot, c=1 on-demand; <=0 = not offered."""
    rng = np.random.default_rng(seed + 17)
    K = cat.k
    reg_mult = 1.0 + 0.08 * np.arange(n_regions)
    od = (cat.od_uph[None, :] * reg_mult[:, None])  # [R][K]
    disc = rng.uniform(0.25, 0.7, size=(n_regions, K, n_zones))
    noise = rng.normal(0.0, 1.0, size=(n_regions, 24, K, n_zones))
    spot = od[:, None, :, None] * disc[:, None, :, :] * (1.0 + 0.1 * noise)
    spot = np.clip(spot, 0.2 * od[:, None, :, None], 0.95 * od[:, None, :, None])
    tile = np.zeros((n_regions, 24, K, n_zones, 2), np.int32)
    tile[..., 0] = np.rint(spot).astype(np.int32)
    tile[..., 1] = np.rint(np.broadcast_to(od[:, None, :, None], spot.shape)).astype(np.int32)
    if avail < 1.0:
        miss = rng.random(size=(n_regions, K, n_zones)) > avail
        tile[..., 0] = np.where(miss[:, None, :, :], 0, tile[..., 0])
    return tile


def carbon_intensity(n_regions: int, seed: int = 20251205, means=None) -> np.ndarray:
    """gCO2/kWh [R][24]: mean_r*(1+0.3 sin(2pi(h-13)/24))*(1+0.05 eps); region 0
    defaults to the reference's 400 g/kWh (.env:14)."""
    rng = np.random.default_rng(seed + 29)
    if means is None:
        means = [DEFAULT_CI] + list(np.linspace(50, 700, max(n_regions - 1, 0)))
    means = np.asarray(means[:n_regions], np.float64)
    h = np.arange(24)
    ci = means[:, None] * (1.0 + 0.3 * np.sin(2 * np.pi * (h[None, :] - 13) / 24.0))
    ci = ci * (1.0 + 0.05 * rng.normal(size=ci.shape))
    return np.clip(ci, 5.0, None)


def patch(policy=abi.POLICY_KEEP, ca=-1, zones=0, caps=0):
    p = abi.PoolPatch()
    p.policy, p.consolidate_after_s, p.zone_mask, p.cap_mask = policy, ca, zones, caps
    return p


def reference_pools(offpeak_zones=("us-east-2a",), peak_zones=("us-east-2c",),
                    all_zones=("us-east-2a", "us-east-2b", "us-east-2c")):
    """The two NodePools in Karpenter order (weight desc, name asc): index 0 =
    on-demand-slo, 1 = spot-preferred. Base spec is ours (the reference never
    creates the pools, demo_00_env.sh:17); profiles are the captured patches."""
    allz = zone_mask(all_zones)
    off, pk = zone_mask(offpeak_zones), zone_mask(peak_zones)
    od = abi.Pool()
    od.limit_cpu_m, od.budget_pct, od.limit_mem_mi = -1, 10, -1
    od.base = patch(abi.WHEN_EMPTY_OR_UNDERUTILIZED, 0, allz, abi.CAP_OD)
    od.profile[abi.PROFILE_RESET] = patch(abi.WHEN_EMPTY, 30)
    od.profile[abi.PROFILE_OFFPEAK] = patch(abi.WHEN_EMPTY, 60, off, abi.CAP_OD)
    od.profile[abi.PROFILE_PEAK] = patch(abi.WHEN_EMPTY, 120, pk, abi.CAP_OD)
    sp = abi.Pool()
    sp.limit_cpu_m, sp.budget_pct, sp.limit_mem_mi = -1, 10, -1
    sp.base = patch(abi.WHEN_EMPTY_OR_UNDERUTILIZED, 0, allz, abi.CAP_SPOT | abi.CAP_OD)
    sp.profile[abi.PROFILE_RESET] = patch(abi.WHEN_EMPTY, 30)
    sp.profile[abi.PROFILE_OFFPEAK] = patch(abi.WHEN_EMPTY_OR_UNDERUTILIZED, -1, off,
                                            abi.CAP_SPOT | abi.CAP_OD)
    sp.profile[abi.PROFILE_PEAK] = patch(abi.WHEN_EMPTY, 120, pk, abi.CAP_SPOT | abi.CAP_OD)
    return [od, sp]


def deployment(scaler=abi.SCALER_HPA, replicas0=5, min_r=1, max_r=100, target=70,
               req_cpu=200, req_mem=128, limit_cpu=500, cap_sel=abi.CAP_SPOT, pdb=1,
               down_stab=300, keda_threshold=500, keda_activation=0, keda_cooldown=300,
               keda_min=0, keda_max=100, tol=0.1, up=None, down=None):
    d = abi.Deployment()
    d.scaler, d.replicas0, d.min_replicas, d.max_replicas = scaler, replicas0, min_r, max_r
    d.target_util_pct, d.req_cpu_m, d.req_mem_mi, d.limit_cpu_m = target, req_cpu, req_mem, limit_cpu
    d.cap_sel, d.pdb_member = cap_sel, pdb
    d.keda_cooldown_s, d.keda_min, d.keda_max = keda_cooldown, keda_min, keda_max
    d.keda_threshold, d.keda_activation, d.tolerance = keda_threshold, keda_activation, tol
    d.up = up if up is not None else default_up()
    d.down = down if down is not None else default_down(down_stab)
    return d


def keda_trigger(threshold, activation=0):
    """An extra ScaledObject trigger of the KEDA deployment listed just before it
    (CCKA_SCALER_KEDA_TRIGGER: owns no pods; its load column is the metric)."""
    return deployment(abi.SCALER_KEDA_TRIGGER, replicas0=0, min_r=0, max_r=0, pdb=0,
                      keda_threshold=threshold, keda_activation=activation)


def burst_deployments(count=12, replicas=5):
    """demo_30_burst_configure.sh:57-151: odd -> spot, even -> on-demand, static replicas."""
    out = []
    for i in range(1, count + 1):
        cap = abi.CAP_SPOT if i % 2 == 1 else abi.CAP_OD
        out.append(deployment(abi.SCALER_STATIC, replicas, replicas, replicas, 70, 200, 128, 500,
                              cap, 1))
    return out


@dataclass
class WorldSpec:
    catalog: Catalog
    ci: np.ndarray                 # [R][24] gCO2/kWh
    price: np.ndarray              # [R][24][K][Z][2] int32
    pools: list
    deploys: list
    n_steps: int = 1440
    start_minute: int = 0
    provision_delay_steps: int = 1
    max_nodes: int = 8
    base_nodes: int = 3
    base_type: str = "m6i.large"
    base_util: float = 0.0
    slo_util_pct: int = 150
    pdb_pct: int = 50
    peak_start: int = 960
    peak_end: int = 1260
    peak_switch: int = 1
    reset_ca_s: int = 30
    carbon_weight: float = 0.0
    drift: int = 0                 # CCKA_DISRUPT_DRIFT
    replace: int = 0               # CCKA_DISRUPT_REPLACE
    multi: int = 0                 # CCKA_DISRUPT_MULTI
    hpa_sync_s: int = 0            # HPA decision period: 0/60 = once per step; 10/15/20/30 = sub-steps
    _keep: list = field(default_factory=list, repr=False)

    @property
    def n_regions(self):
        return self.price.shape[0]

    @property
    def n_zones(self):
        return self.price.shape[3]

    def to_c(self) -> abi.World:
        w = abi.World()
        types = self.catalog.itypes()
        ci = np.ascontiguousarray(self.ci, np.float64)
        gpwh = np.ascontiguousarray(ci / 1000.0)
        gpwmin = np.ascontiguousarray(ci / 60000.0)
        price = np.ascontiguousarray(self.price, np.int32)
        self._keep = [types, gpwh, gpwmin, price]
        w.n_steps = self.n_steps
        w.start_minute = self.start_minute
        w.provision_delay_steps = self.provision_delay_steps
        w.max_nodes = self.max_nodes
        w.n_types = self.catalog.k
        w.n_regions = self.n_regions
        w.n_zones = self.n_zones
        w.n_pools = len(self.pools)
        w.types = C.cast(types, C.POINTER(abi.ItType))
        w.ci_gpwh = gpwh.ctypes.data_as(C.POINTER(C.c_double))
        w.ci_gpwmin = gpwmin.ctypes.data_as(C.POINTER(C.c_double))
        w.price_uph = price.ctypes.data_as(C.POINTER(C.c_int32))
        for i, p in enumerate(self.pools):
            w.pools[i] = p
        w.n_deploy = len(self.deploys)
        for i, d in enumerate(self.deploys):
            w.deploy[i] = d
        w.base_nodes = self.base_nodes
        w.base_type = self.catalog.index(self.base_type)
        w.slo_util_pct = self.slo_util_pct
        w.base_util = self.base_util
        w.carbon_weight = self.carbon_weight
        w.pdb_min_available_pct = self.pdb_pct
        w.peak_start_min = self.peak_start
        w.peak_end_min = self.peak_end
        w.peak_switch = self.peak_switch
        w.reset_ca_s = self.reset_ca_s
        w.disrupt_ext = ((abi.DISRUPT_DRIFT if self.drift else 0) | (abi.DISRUPT_REPLACE if self.replace else 0)
                         | (abi.DISRUPT_MULTI if self.multi else 0))
        w.hpa_sync_s = self.hpa_sync_s
        return w


@dataclass
class ScenarioSet:
    n: int
    first_id: int = 0
    n_traces: int = 0  # > 0: scenario with global id g reads shared trace g % n_traces
    region: np.ndarray | None = None
    target_util_pct: np.ndarray | None = None
    max_replicas: np.ndarray | None = None
    down_stab_s: np.ndarray | None = None
    reset_ca_s: np.ndarray | None = None
    peak_switch: np.ndarray | None = None
    carbon_weight: np.ndarray | None = None
    cap_sel: np.ndarray | None = None

    _DT = {"region": (np.uint8, C.c_uint8), "target_util_pct": (np.int16, C.c_int16),
           "max_replicas": (np.int16, C.c_int16), "down_stab_s": (np.int16, C.c_int16),
           "reset_ca_s": (np.int16, C.c_int16), "peak_switch": (np.uint8, C.c_uint8),
           "carbon_weight": (np.float64, C.c_double), "cap_sel": (np.uint8, C.c_uint8)}

    def to_c(self) -> abi.Scenarios:
        s = abi.Scenarios()
        s.n, s.first_id, s.n_traces = self.n, self.first_id, self.n_traces
        keep = []
        for name, (npt, ct) in self._DT.items():
            a = getattr(self, name)
            if a is None:
                continue
            a = np.ascontiguousarray(a, npt)
            assert a.shape == (self.n,), (name, a.shape)
            keep.append(a)
            setattr(s, name, a.ctypes.data_as(C.POINTER(ct)))
        self._keep = keep
        return s

    def slice(self, lo, hi):
        kw = {k: (None if getattr(self, k) is None else getattr(self, k)[lo:hi]) for k in self._DT}
        return ScenarioSet(hi - lo, self.first_id + lo, self.n_traces, **kw)


def alloc_results(n: int):
    """numpy arrays + ctypes Results pointing at them."""
    arrays = {name: np.zeros(n, dt) for name, _, dt in abi.RESULT_FIELDS}
    r = abi.Results()
    for name, ct, _ in abi.RESULT_FIELDS:
        setattr(r, name, arrays[name].ctypes.data_as(C.POINTER(ct)))
    return arrays, r


TRAJ_DTYPE = np.dtype([("replicas", "<i4"), ("pending", "<i4"), ("nodes_spot", "<u2"),
                       ("nodes_od", "<u2"), ("last_type", "<u2"), ("flags", "<u2")])
