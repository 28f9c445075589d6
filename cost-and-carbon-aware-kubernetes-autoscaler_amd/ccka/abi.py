"""ctypes mirror of include/ccka.h (the C ABI of libccka.so).

Field order, widths and padding follow the header exactly; ``check_sizes``
compares them against ``ccka_struct_sizes()`` exported by the library.
"""
from __future__ import annotations

import ctypes as C
import os

ABI_VERSION = 5
STEP_SECONDS = 60
MAX_TYPES = 1024
MAX_ZONES = 4
MAX_REGIONS = 16
MAX_POOLS = 4
MAX_DEPLOY = 16
MAX_NODES = 16
HIST = 8
HPA_MAX_POLICIES = 4
HPA_MAX_WINDOW_S = 3600
HPA_MAX_PERIOD_S = 1800
HPA_HIST_MAX = 360

CAP_SPOT, CAP_OD = 1, 2
POLICY_KEEP, WHEN_EMPTY, WHEN_EMPTY_OR_UNDERUTILIZED = 0, 1, 2
SCALER_STATIC, SCALER_HPA, SCALER_KEDA, SCALER_KEDA_TRIGGER = 0, 1, 2, 3
DISRUPT_DRIFT, DISRUPT_REPLACE, DISRUPT_MULTI = 1, 2, 4
PROFILE_RESET, PROFILE_OFFPEAK, PROFILE_PEAK = 0, 1, 2
SELECT_MAX, SELECT_MIN, SELECT_DISABLED = 0, 1, 2
HPA_PODS, HPA_PERCENT = 1, 2

STATUS = {0: "OK", -1: "EINVAL", -2: "ENOMEM", -3: "EHIP", -4: "ERCCL",
          -5: "EPARITY", -6: "ESTATE", -7: "ENODEV"}


class ItType(C.Structure):
    _fields_ = [("vcpu", C.c_int32), ("alloc_cpu_m", C.c_int32), ("alloc_mem_mi", C.c_int32),
                ("max_pods", C.c_int32), ("idle_nw", C.c_int64), ("dyn_nw_per_m", C.c_int64),
                ("p_ref_w", C.c_double), ("mem_mi", C.c_int32), ("_pad", C.c_int32)]


class PoolPatch(C.Structure):
    _fields_ = [("policy", C.c_int32), ("consolidate_after_s", C.c_int32),
                ("zone_mask", C.c_uint32), ("cap_mask", C.c_uint32)]


class Pool(C.Structure):
    _fields_ = [("limit_cpu_m", C.c_int32), ("budget_pct", C.c_int32), ("base", PoolPatch),
                ("profile", PoolPatch * 3), ("limit_mem_mi", C.c_int32), ("_pad", C.c_int32)]


class HpaPolicy(C.Structure):
    _fields_ = [("type", C.c_int32), ("value", C.c_int32), ("period_s", C.c_int32)]


class HpaRules(C.Structure):
    _fields_ = [("select", C.c_int32), ("n_policies", C.c_int32), ("stab_window_s", C.c_int32),
                ("_pad", C.c_int32), ("policies", HpaPolicy * HPA_MAX_POLICIES)]


class Deployment(C.Structure):
    _fields_ = [("scaler", C.c_int32), ("replicas0", C.c_int32), ("min_replicas", C.c_int32),
                ("max_replicas", C.c_int32), ("target_util_pct", C.c_int32),
                ("req_cpu_m", C.c_int32), ("req_mem_mi", C.c_int32), ("limit_cpu_m", C.c_int32),
                ("cap_sel", C.c_uint32), ("pdb_member", C.c_int32), ("keda_cooldown_s", C.c_int32),
                ("keda_min", C.c_int32), ("keda_max", C.c_int32), ("_pad", C.c_int32),
                ("keda_threshold", C.c_int64), ("keda_activation", C.c_int64),
                ("tolerance", C.c_double), ("up", HpaRules), ("down", HpaRules)]


class World(C.Structure):
    _fields_ = [("n_steps", C.c_int32), ("start_minute", C.c_int32),
                ("provision_delay_steps", C.c_int32), ("max_nodes", C.c_int32),
                ("n_types", C.c_int32), ("n_regions", C.c_int32), ("n_zones", C.c_int32),
                ("n_pools", C.c_int32),
                ("types", C.POINTER(ItType)), ("ci_gpwh", C.POINTER(C.c_double)),
                ("ci_gpwmin", C.POINTER(C.c_double)), ("price_uph", C.POINTER(C.c_int32)),
                ("pools", Pool * MAX_POOLS), ("n_deploy", C.c_int32), ("base_nodes", C.c_int32),
                ("base_type", C.c_int32), ("slo_util_pct", C.c_int32),
                ("deploy", Deployment * MAX_DEPLOY),
                ("base_util", C.c_double), ("carbon_weight", C.c_double),
                ("pdb_min_available_pct", C.c_int32), ("peak_start_min", C.c_int32),
                ("peak_end_min", C.c_int32), ("peak_switch", C.c_int32),
                ("reset_ca_s", C.c_int32), ("disrupt_ext", C.c_int32), ("hpa_sync_s", C.c_int32),
                ("_pad2", C.c_int32)]


class Scenarios(C.Structure):
    _fields_ = [("n", C.c_int64), ("first_id", C.c_int64), ("n_traces", C.c_int64),
                ("region", C.POINTER(C.c_uint8)), ("target_util_pct", C.POINTER(C.c_int16)),
                ("max_replicas", C.POINTER(C.c_int16)), ("down_stab_s", C.POINTER(C.c_int16)),
                ("reset_ca_s", C.POINTER(C.c_int16)), ("peak_switch", C.POINTER(C.c_uint8)),
                ("carbon_weight", C.POINTER(C.c_double)), ("cap_sel", C.POINTER(C.c_uint8))]


RESULT_FIELDS = [
    ("cost_uphmin", C.c_int64, "int64"), ("energy_wmin", C.c_double, "float64"),
    ("gco2", C.c_double, "float64"), ("slo_minutes", C.c_int32, "int32"),
    ("pending_pod_minutes", C.c_int64, "int64"), ("node_min_spot", C.c_int32, "int32"),
    ("node_min_od", C.c_int32, "int32"), ("launches", C.c_int32, "int32"),
    ("deletions", C.c_int32, "int32"), ("peak_nodes", C.c_int32, "int32"),
    ("final_replicas", C.c_int32, "int32"), ("final_nodes", C.c_int32, "int32"),
    ("last_choice", C.c_uint32, "uint32"), ("choice_hash", C.c_uint32, "uint32"),
]


class Results(C.Structure):
    _fields_ = [(name, C.POINTER(ct)) for name, ct, _ in RESULT_FIELDS]


class TrajRec(C.Structure):
    _fields_ = [("replicas", C.c_int32), ("pending", C.c_int32), ("nodes_spot", C.c_uint16),
                ("nodes_od", C.c_uint16), ("last_type", C.c_uint16), ("flags", C.c_uint16)]


class Totals(C.Structure):
    _fields_ = [("scenarios", C.c_int64), ("cost_uphmin", C.c_int64), ("slo_minutes", C.c_int64),
                ("pending_pod_minutes", C.c_int64), ("node_min_spot", C.c_int64),
                ("node_min_od", C.c_int64), ("launches", C.c_int64), ("deletions", C.c_int64),
                ("energy_uwmin", C.c_int64), ("gco2_ug", C.c_int64),
                ("energy_wmin", C.c_double), ("gco2", C.c_double)]


class PgParams(C.Structure):
    """ccka_pg_params: the stochastic closed loop's sampling key and objective weights."""
    _fields_ = [("seed", C.c_uint64), ("w_carbon", C.c_double), ("w_slo", C.c_double),
                ("baseline", C.c_int32), ("_pad", C.c_int32)]


class MlpGrads(C.Structure):
    """ccka_mlp_grads: fp32 host gradient arrays (layouts of ccka_mlp_set_weights)."""
    _fields_ = [(n, C.POINTER(C.c_float)) for n in ("w1", "b1", "w2", "b2", "w3", "b3")]


GRAD_SHAPES = {"w1": (64, 256), "b1": (256,), "w2": (256, 256), "b2": (256,), "w3": (256, 8), "b3": (8,)}


class GridStats(C.Structure):
    _fields_ = [("grid", C.c_int64), ("scenarios", C.c_int64), ("cost_uphmin", C.c_int64),
                ("slo_minutes", C.c_int64), ("gco2", C.c_double), ("energy_wmin", C.c_double)]


class Detail(C.Structure):
    """ccka_detail: per-pool / base-group / per-deployment breakdown (ccka_set_detail)."""
    _fields_ = [("pool_cost_uphmin", C.c_int64 * MAX_POOLS), ("pool_energy_nwmin", C.c_int64 * MAX_POOLS),
                ("pool_gco2", C.c_double * MAX_POOLS), ("pool_node_min_spot", C.c_int32 * MAX_POOLS),
                ("pool_node_min_od", C.c_int32 * MAX_POOLS), ("pool_final_nodes", C.c_int32 * MAX_POOLS),
                ("pool_peak_nodes", C.c_int32 * MAX_POOLS), ("pool_launches", C.c_int32 * MAX_POOLS),
                ("desired", C.c_int32 * MAX_DEPLOY), ("ready", C.c_int32 * MAX_DEPLOY),
                ("pending", C.c_int32 * MAX_DEPLOY), ("base_cost_uphmin", C.c_int64),
                ("base_energy_nwmin", C.c_int64), ("base_gco2", C.c_double)]


def detail_dtype():
    """numpy structured dtype laid out exactly as ccka_detail (arrays of it are
    passed to ccka_get_detail / the oracle as a flat buffer)."""
    import numpy as np
    kinds = {C.c_int64: "<i8", C.c_int32: "<i4", C.c_double: "<f8"}
    fields = []
    for name, ct in Detail._fields_:
        if hasattr(ct, "_length_"):
            fields.append((name, kinds[ct._type_], (ct._length_,)))
        else:
            fields.append((name, kinds[ct]))
    dt = np.dtype(fields)
    assert dt.itemsize == C.sizeof(Detail)
    return dt


class TraceGen(C.Structure):
    _fields_ = [("seed", C.c_uint64), ("base_lo", C.c_int32), ("base_hi", C.c_int32),
                ("amp_lo_pm", C.c_int32), ("amp_hi_pm", C.c_int32), ("noise_pm", C.c_int32),
                ("burst_prob_pm", C.c_int32), ("burst_mult_pm", C.c_int32),
                ("burst_len", C.c_int32)]


STRUCT_ORDER = [ItType, Pool, Deployment, World, Scenarios, Results, TrajRec, Totals, TraceGen,
                GridStats, Detail]

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
ENGINE_LIB = os.path.join(os.path.dirname(PKG_DIR), "csrc", "build", "libccka.so")


class CckaError(RuntimeError):
    pass


def check(rc: int, what: str, lib=None, ctx=None) -> None:
    if rc != 0:
        msg = ""
        if lib is not None and ctx is not None:
            try:
                msg = lib.ccka_last_error(ctx).decode()
            except Exception:  # pragma: no cover
                msg = ""
        raise CckaError(f"{what} failed: {STATUS.get(rc, rc)} {msg}")


_ENGINE = None


def load_engine(path: str | None = None):
    """Load libccka.so (the HIP engine). Fails loudly if it is missing: there is
    no CPU fallback in the product path."""
    global _ENGINE
    if _ENGINE is not None and path is None:
        return _ENGINE
    p = path or ENGINE_LIB
    if not os.path.exists(p):
        raise CckaError(f"HIP engine library not built: {p} (run __graft_entry__.build())")
    lib = C.CDLL(p)
    vp = C.c_void_p
    sig = {
        "ccka_abi_version": (C.c_int32, []),
        "ccka_struct_sizes": (C.c_int32, [C.POINTER(C.c_int64), C.c_int32]),
        "ccka_open": (C.c_int, [C.POINTER(vp), C.c_int]),
        "ccka_close": (None, [vp]),
        "ccka_last_error": (C.c_char_p, [vp]),
        "ccka_set_world": (C.c_int, [vp, C.POINTER(World)]),
        "ccka_set_scenarios": (C.c_int, [vp, C.POINTER(Scenarios)]),
        "ccka_set_load": (C.c_int, [vp, C.POINTER(C.c_int32), C.c_int64]),
        "ccka_gen_load": (C.c_int, [vp, C.POINTER(TraceGen)]),
        "ccka_get_load": (C.c_int, [vp, C.POINTER(C.c_int32), C.c_int64]),
        "ccka_rollout": (C.c_int, [vp, C.c_int32]),
        "ccka_rollout_async": (C.c_int, [vp, C.c_int32]),
        "ccka_sync": (C.c_int, [vp]),
        "ccka_last_kernel_ms": (C.c_int, [vp, C.POINTER(C.c_double)]),
        "ccka_get_results": (C.c_int, [vp, C.POINTER(Results)]),
        "ccka_get_trajectory": (C.c_int, [vp, C.POINTER(TrajRec), C.c_int64]),
        "ccka_trajectory_layout": (C.c_int, [vp, C.POINTER(C.c_int32)]),
        "ccka_get_trajectory_native": (C.c_int, [vp, C.POINTER(TrajRec), C.c_int64, C.POINTER(C.c_int32)]),
        "ccka_get_totals": (C.c_int, [vp, C.POINTER(Totals)]),
        "ccka_set_detail": (C.c_int, [vp, C.c_int32]),
        "ccka_policy_rollout": (C.c_int, [vp, C.c_int32, C.c_int32]),
        "ccka_get_policy_actions": (C.c_int, [vp, C.c_void_p, C.c_void_p, C.c_int64]),
        "ccka_get_detail": (C.c_int, [vp, C.c_void_p, C.c_int64]),
        "ccka_policy_grad": (C.c_int, [vp, C.POINTER(PgParams), C.POINTER(MlpGrads), C.POINTER(C.c_double)]),
        "ccka_get_policy_samples": (C.c_int, [vp, C.POINTER(C.c_uint8), C.POINTER(C.c_float), C.c_int64]),
        "ccka_mlp_backward": (C.c_int, [vp, C.POINTER(C.c_uint16), C.POINTER(C.c_uint8), C.POINTER(C.c_float),
                                        C.c_int64, C.POINTER(MlpGrads)]),
        "ccka_comm_unique_id": (C.c_int, [C.POINTER(C.c_uint8)]),
        "ccka_comm_init": (C.c_int, [vp, C.POINTER(C.c_uint8), C.c_int32, C.c_int32]),
        "ccka_allreduce_totals": (C.c_int, [vp, C.POINTER(Totals)]),
        "ccka_comm_info": (C.c_int, [vp, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
        "ccka_totals_pack": (C.c_int, [C.POINTER(Totals), C.c_int32, C.POINTER(C.c_int64), C.c_int32]),
        "ccka_totals_finish": (C.c_int, [C.POINTER(C.c_int64), C.c_int32, C.POINTER(Totals)]),
        "ccka_device_info": (C.c_int, [vp, C.c_char_p, C.c_int32, C.POINTER(C.c_int32)]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _ENGINE = lib
    return lib


EXPORTED = [
    "ccka_abi_version", "ccka_struct_sizes", "ccka_open", "ccka_close", "ccka_last_error",
    "ccka_set_world", "ccka_set_scenarios", "ccka_set_load", "ccka_gen_load", "ccka_get_load",
    "ccka_rollout", "ccka_rollout_async", "ccka_sync", "ccka_last_kernel_ms", "ccka_get_results",
    "ccka_get_trajectory", "ccka_get_totals", "ccka_comm_unique_id", "ccka_comm_init",
    "ccka_allreduce_totals", "ccka_comm_info", "ccka_device_info", "ccka_get_grid_stats", "ccka_pareto_frontier",
    "ccka_mlp_set_weights", "ccka_mlp_set_states", "ccka_mlp_gen_states", "ccka_mlp_forward",
    "ccka_mlp_forward_async", "ccka_mlp_get_actions", "ccka_set_detail", "ccka_get_detail",
    "ccka_policy_rollout", "ccka_get_policy_actions", "ccka_trajectory_layout", "ccka_get_trajectory_native",
    "ccka_policy_grad", "ccka_get_policy_samples", "ccka_mlp_backward", "ccka_totals_pack", "ccka_totals_finish",
]
TOTALS_INT64, TOTALS_BLOCK = 10, 11  # CCKA_TOTALS_INT64, CCKA_TOTALS_BLOCK
EOVERFLOW = -8
TRAJ_TN, TRAJ_NT = 0, 1  # device layouts of the trajectory records (ccka_trajectory_layout)


def check_sizes(lib) -> None:
    buf = (C.c_int64 * 16)()
    n = lib.ccka_struct_sizes(buf, 16)
    want = [C.sizeof(s) for s in STRUCT_ORDER]
    got = list(buf[:n])
    if got != want:
        raise CckaError(f"ABI struct size mismatch: lib {got} vs python {want}")
