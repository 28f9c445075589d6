"""Python handle on libccka.so (the HIP rollout engine) through its C ABI.

There is no CPU fallback: constructing an Engine without the built library or
without a GPU raises.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import abi
from .world import TRAJ_DTYPE, ScenarioSet, WorldSpec, alloc_results


GRID_DTYPE = np.dtype([("grid", "<i8"), ("scenarios", "<i8"), ("cost_uphmin", "<i8"),
                       ("slo_minutes", "<i8"), ("gco2", "<f8"), ("energy_wmin", "<f8")])


def _grid_array(a, n) -> np.ndarray:
    return np.frombuffer(bytes(a)[:n * C.sizeof(abi.GridStats)], GRID_DTYPE).copy()


class Engine:
    def __init__(self, device: int = 0, lib_path: str | None = None):
        self.lib = abi.load_engine(lib_path)
        abi.check_sizes(self.lib)
        self.ctx = C.c_void_p()
        abi.check(self.lib.ccka_open(C.byref(self.ctx), device), "ccka_open")
        self.n = 0
        self.T = 0
        self.D = 0

    def _chk(self, rc, what):
        abi.check(rc, what, self.lib, self.ctx)

    def close(self):
        if self.ctx:
            self.lib.ccka_close(self.ctx)
            self.ctx = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_world(self, spec: WorldSpec):
        w = spec.to_c()
        self._chk(self.lib.ccka_set_world(self.ctx, C.byref(w)), "ccka_set_world")
        self.T = spec.n_steps
        self.D = len(spec.deploys)

    def set_scenarios(self, sc: ScenarioSet):
        s = sc.to_c()
        self._chk(self.lib.ccka_set_scenarios(self.ctx, C.byref(s)), "ccka_set_scenarios")
        self.n = sc.n
        self.load_cols = sc.n_traces if sc.n_traces > 0 else sc.n

    def set_load(self, load: np.ndarray):
        a = np.ascontiguousarray(load, np.int32)
        self._chk(self.lib.ccka_set_load(self.ctx, a.ctypes.data_as(C.POINTER(C.c_int32)), a.size),
                  "ccka_set_load")

    def gen_load(self, gen: abi.TraceGen):
        self._chk(self.lib.ccka_gen_load(self.ctx, C.byref(gen)), "ccka_gen_load")

    def get_load(self) -> np.ndarray:
        a = np.zeros((self.T, self.D, self.load_cols), np.int32)
        self._chk(self.lib.ccka_get_load(self.ctx, a.ctypes.data_as(C.POINTER(C.c_int32)), a.size),
                  "ccka_get_load")
        return a

    def rollout(self, trajectory: bool = False):
        self._chk(self.lib.ccka_rollout(self.ctx, int(trajectory)), "ccka_rollout")

    def rollout_async(self, trajectory: bool = False):
        self._chk(self.lib.ccka_rollout_async(self.ctx, int(trajectory)), "ccka_rollout_async")

    def sync(self):
        self._chk(self.lib.ccka_sync(self.ctx), "ccka_sync")

    def kernel_ms(self) -> float:
        v = C.c_double()
        self._chk(self.lib.ccka_last_kernel_ms(self.ctx, C.byref(v)), "ccka_last_kernel_ms")
        return v.value

    def results(self) -> dict:
        arrays, r = alloc_results(self.n)
        self._chk(self.lib.ccka_get_results(self.ctx, C.byref(r)), "ccka_get_results")
        return arrays

    def trajectory(self) -> np.ndarray:
        a = np.zeros((self.T, self.n), TRAJ_DTYPE)
        self._chk(self.lib.ccka_get_trajectory(self.ctx, a.ctypes.data_as(C.POINTER(abi.TrajRec)),
                                               a.size), "ccka_get_trajectory")
        return a

    def trajectory_native(self):
        """(records, layout): the device records without a transpose, shaped
        [N][T] (abi.TRAJ_NT, the single-deployment engine) or [T][N]."""
        lay = C.c_int32()
        self._chk(self.lib.ccka_trajectory_layout(self.ctx, C.byref(lay)), "ccka_trajectory_layout")
        shape = (self.n, self.T) if lay.value == abi.TRAJ_NT else (self.T, self.n)
        a = np.zeros(shape, TRAJ_DTYPE)
        self._chk(self.lib.ccka_get_trajectory_native(self.ctx, a.ctypes.data_as(C.POINTER(abi.TrajRec)), a.size,
                                                      None), "ccka_get_trajectory_native")
        return a, lay.value

    @staticmethod
    def _grads():
        g = {k: np.zeros(v, np.float32) for k, v in abi.GRAD_SHAPES.items()}
        s = abi.MlpGrads(*[g[k].ctypes.data_as(C.POINTER(C.c_float)) for k in ("w1", "b1", "w2", "b2", "w3", "b3")])
        return g, s

    def policy_grad(self, seed: int, w_carbon: float = 0.0, w_slo: float = 0.0, baseline: bool = True):
        """One stochastic closed-loop rollout and the score-function gradient
        of E[J] (ccka_policy_grad): (grads dict, mean objective)."""
        g, s = self._grads()
        prm = abi.PgParams(seed, w_carbon, w_slo, int(bool(baseline)), 0)
        obj = C.c_double()
        self._chk(self.lib.ccka_policy_grad(self.ctx, C.byref(prm), C.byref(s), C.byref(obj)), "ccka_policy_grad")
        return g, obj.value

    def policy_samples(self):
        """(actions [T][N] uint8, coef [N] fp32) of the last policy_grad."""
        a = np.zeros((self.T, self.n), np.uint8)
        cf = np.zeros(self.n, np.float32)
        self._chk(self.lib.ccka_get_policy_samples(self.ctx, a.ctypes.data_as(C.POINTER(C.c_uint8)),
                                                   cf.ctypes.data_as(C.POINTER(C.c_float)), a.size),
                  "ccka_get_policy_samples")
        return a, cf

    def mlp_backward(self, x_bits: np.ndarray, actions: np.ndarray, coef: np.ndarray):
        """Gradient of sum_m coef[m] log softmax(policy(x_m))[a_m] (ccka_mlp_backward)."""
        x = np.ascontiguousarray(x_bits, np.uint16)
        a = np.ascontiguousarray(actions, np.uint8)
        cf = np.ascontiguousarray(coef, np.float32)
        g, s = self._grads()
        self._chk(self.lib.ccka_mlp_backward(self.ctx, x.ctypes.data_as(C.POINTER(C.c_uint16)),
                                             a.ctypes.data_as(C.POINTER(C.c_uint8)),
                                             cf.ctypes.data_as(C.POINTER(C.c_float)), len(a), C.byref(s)),
                  "ccka_mlp_backward")
        return g

    def totals(self) -> abi.Totals:
        t = abi.Totals()
        self._chk(self.lib.ccka_get_totals(self.ctx, C.byref(t)), "ccka_get_totals")
        return t

    def set_detail(self, on: bool = True):
        """Record the per-pool / base-group / per-deployment breakdown
        (ccka_detail) in later rollouts (the summary path)."""
        self._chk(self.lib.ccka_set_detail(self.ctx, int(bool(on))), "ccka_set_detail")

    def detail(self) -> np.ndarray:
        a = np.zeros(self.n, abi.detail_dtype())
        self._chk(self.lib.ccka_get_detail(self.ctx, a.ctypes.data, a.size), "ccka_get_detail")
        return a

    # ---- closed-loop learned policy (config 5) ----
    def policy_rollout(self, trajectory: bool = False, record: bool = False):
        """ccka_policy_rollout: the MLP policy (mlp_set_weights) decides every
        step's HPA target and carbon weight from the scenario state."""
        self._chk(self.lib.ccka_policy_rollout(self.ctx, int(trajectory), int(record)), "ccka_policy_rollout")

    def policy_actions(self):
        """The recorded actions: (target [T][N] int16, carbon weight [T][N] float64)."""
        tg = np.zeros((self.T, self.n), np.int16)
        cw = np.zeros((self.T, self.n), np.float64)
        self._chk(self.lib.ccka_get_policy_actions(self.ctx, tg.ctypes.data, cw.ctypes.data, tg.size),
                  "ccka_get_policy_actions")
        return tg, cw

    def debug_policy_features(self, enable: bool = True):
        """Internal test hook: record the policy features of every step."""
        fn = self.lib.ccka_debug_policy_features
        fn.argtypes = [C.c_void_p, C.c_int32]
        self._chk(fn(self.ctx, int(enable)), "ccka_debug_policy_features")

    def debug_get_policy_features(self) -> np.ndarray:
        fn = self.lib.ccka_debug_get_policy_features
        fn.argtypes = [C.c_void_p, C.c_void_p, C.c_int64]
        a = np.zeros((self.T + 1, self.n, 64), np.uint16)
        self._chk(fn(self.ctx, a.ctypes.data, a.size), "ccka_debug_get_policy_features")
        return a

    # ---- policy sweep (config 4) ----
    def grid_stats(self, grid_size: int) -> np.ndarray:
        ng = self.n // grid_size
        a = (abi.GridStats * ng)()
        self._chk(self.lib.ccka_get_grid_stats(self.ctx, C.c_int64(grid_size), a, C.c_int64(ng)),
                  "ccka_get_grid_stats")
        return _grid_array(a, ng)

    def pareto(self, grid_size: int, capacity: int | None = None) -> np.ndarray:
        cap = capacity if capacity is not None else max(1, self.n // grid_size) * 8
        a = (abi.GridStats * cap)()
        n = C.c_int32()
        self._chk(self.lib.ccka_pareto_frontier(self.ctx, C.c_int64(grid_size), a, cap, C.byref(n)),
                  "ccka_pareto_frontier")
        return _grid_array(a, n.value)

    # ---- multi-GPU (RCCL over xGMI) ----
    def comm_init(self, uid: bytes | None = None, nranks: int = 1, rank: int = 0):
        """RCCL communicator of this context; uid = None creates a fresh id
        (one-rank communicator, or rank 0 before distributing it)."""
        buf = (C.c_uint8 * 128)()
        if uid is None:
            self._chk(self.lib.ccka_comm_unique_id(buf), "ccka_comm_unique_id")
        else:
            buf = (C.c_uint8 * 128).from_buffer_copy(uid)
        self._chk(self.lib.ccka_comm_init(self.ctx, buf, nranks, rank), "ccka_comm_init")

    def comm_info(self):
        n, r = C.c_int32(), C.c_int32()
        self._chk(self.lib.ccka_comm_info(self.ctx, C.byref(n), C.byref(r)), "ccka_comm_info")
        return n.value, r.value

    def allreduce_totals(self, t: abi.Totals) -> abi.Totals:
        out = abi.Totals.from_buffer_copy(t)
        self._chk(self.lib.ccka_allreduce_totals(self.ctx, C.byref(out)), "ccka_allreduce_totals")
        return out

    def debug_pareto_merge(self, gathered: np.ndarray, counts, capacity: int | None = None) -> np.ndarray:
        """Internal: the cross-rank merge of ccka_pareto_frontier on given
        exchange buffers (gathered: GRID_DTYPE [nranks][cap])."""
        g = np.ascontiguousarray(gathered, GRID_DTYPE)
        nranks, cap = g.shape
        cnt = np.ascontiguousarray(counts, np.int64)
        assert cnt.shape == (nranks,)
        outcap = capacity if capacity is not None else nranks * cap
        a = (abi.GridStats * outcap)()
        n = C.c_int32()
        fn = self.lib.ccka_debug_pareto_merge
        fn.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32, C.c_int64, C.c_void_p, C.c_int32,
                       C.POINTER(C.c_int32)]
        self._chk(fn(self.ctx, g.ctypes.data, cnt.ctypes.data, nranks, cap, a, outcap, C.byref(n)),
                  "ccka_debug_pareto_merge")
        return _grid_array(a, n.value)

    # ---- learned MLP policy (config 5) ----
    def mlp_set_weights(self, ws, bs):
        """ws: bf16 bit arrays (uint16) [in][out]; bs: float32 biases."""
        w = [np.ascontiguousarray(x, np.uint16) for x in ws]
        b = [np.ascontiguousarray(x, np.float32) for x in bs]
        u16 = C.POINTER(C.c_uint16)
        f32 = C.POINTER(C.c_float)
        self._chk(self.lib.ccka_mlp_set_weights(
            self.ctx, w[0].shape[0], w[0].shape[1], w[2].shape[1],
            w[0].ctypes.data_as(u16), b[0].ctypes.data_as(f32), w[1].ctypes.data_as(u16),
            b[1].ctypes.data_as(f32), w[2].ctypes.data_as(u16), b[2].ctypes.data_as(f32)),
            "ccka_mlp_set_weights")
        self.mlp_out = w[2].shape[1]

    def mlp_set_states(self, x: np.ndarray):
        a = np.ascontiguousarray(x, np.uint16)
        self._chk(self.lib.ccka_mlp_set_states(self.ctx, a.ctypes.data_as(C.POINTER(C.c_uint16)),
                                               C.c_int64(a.shape[0])), "ccka_mlp_set_states")
        self.mlp_n = a.shape[0]

    def mlp_gen_states(self, n: int, seed: int = 7):
        self._chk(self.lib.ccka_mlp_gen_states(self.ctx, C.c_int64(n), C.c_uint64(seed)),
                  "ccka_mlp_gen_states")
        self.mlp_n = n

    def mlp_forward(self):
        self._chk(self.lib.ccka_mlp_forward(self.ctx), "ccka_mlp_forward")

    def mlp_forward_async(self):
        self._chk(self.lib.ccka_mlp_forward_async(self.ctx), "ccka_mlp_forward_async")

    def mlp_actions(self) -> np.ndarray:
        y = np.zeros((self.mlp_n, getattr(self, "mlp_out", 8)), np.float32)
        self._chk(self.lib.ccka_mlp_get_actions(self.ctx, y.ctypes.data_as(C.POINTER(C.c_float)),
                                                C.c_int64(self.mlp_n)), "ccka_mlp_get_actions")
        return y

    def set_engine(self, mode: int):
        """Internal: 0 = automatic engine choice, 1 = general kernel only, 2 = the
        general kernel in lockstep (no lane-skewed schedule for several deployments)."""
        self.lib.ccka_debug_engine.argtypes = [C.c_void_p, C.c_int32]
        self._chk(self.lib.ccka_debug_engine(self.ctx, mode), "ccka_debug_engine")

    def debug_pool(self, mode: int = -1, min_queue: int = 0) -> int:
        """Internal: pooled event steps of the single-deployment engine (1 on,
        0 off, -1 unchanged) and the queue length at which a wave serves the
        queue (0 unchanged); returns whether the last such rollout was pooled."""
        fn = self.lib.ccka_debug_pool
        fn.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.POINTER(C.c_int32)]
        last = C.c_int32(0)
        self._chk(fn(self.ctx, mode, min_queue, C.byref(last)), "ccka_debug_pool")
        return last.value

    def debug_pool_policy(self, age: int, idle: int = 1):
        """Internal: the pooled kernel's other serving rules (see ccka_abi.cpp)."""
        fn = self.lib.ccka_debug_pool_policy
        fn.argtypes = [C.c_void_p, C.c_int32, C.c_int32]
        self._chk(fn(self.ctx, age, idle), "ccka_debug_pool_policy")

    def last_engine(self):
        """Internal: (engine, table_ms) of the last rollout; engine 1 = general
        kernel, 2 = single-deployment kernel (rollout_d1.hip), 3 / 4 = the
        launched / fused closed loop, 5 = the general kernel on the lane-skewed
        schedule (rollout_sk.hip)."""
        e, ms = C.c_int32(), C.c_double()
        self._chk(self.lib.ccka_debug_last_engine(self.ctx, C.byref(e), C.byref(ms)),
                  "ccka_debug_last_engine")
        return e.value, ms.value

    def device_info(self):
        name = C.create_string_buffer(256)
        cus = C.c_int32()
        self._chk(self.lib.ccka_device_info(self.ctx, name, 256, C.byref(cus)), "ccka_device_info")
        return name.value.decode(), cus.value
