"""ctypes binding of libccka_host.so (include/ccka_host.h): manifest ingest,
kubectl apply/patch emulation, the reference scripts' payload generators, and
the manifest -> ccka_world builder. No GPU needed."""
from __future__ import annotations

import ctypes as C
import os

from . import abi

HOST_LIB = os.path.join(os.path.dirname(abi.PKG_DIR), "host", "build", "libccka_host.so")
CLI = os.path.join(os.path.dirname(abi.PKG_DIR), "host", "build", "ccka")

_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        if not os.path.exists(HOST_LIB):
            raise abi.CckaError(f"host library not built: {HOST_LIB}")
        L = C.CDLL(HOST_LIB)
        vp = C.c_void_p
        sig = {
            "ccka_host_open": (C.c_int, [C.POINTER(vp)]),
            "ccka_host_close": (None, [vp]),
            "ccka_host_last_error": (C.c_char_p, [vp]),
            "ccka_host_apply": (C.c_int, [vp, C.c_char_p]),
            "ccka_host_patch": (C.c_int, [vp, C.c_char_p, C.c_char_p, C.c_char_p, C.c_char_p]),
            "ccka_host_get_json": (C.c_int, [vp, C.c_char_p, C.c_char_p, C.c_char_p, C.c_int64]),
            "ccka_host_policy_patch": (C.c_int, [vp, C.c_int32, C.c_char_p, C.c_int32, C.c_int32,
                                                 C.c_char_p, C.c_int64]),
            "ccka_host_burst_manifest": (C.c_int, [vp, C.c_int32, C.c_char_p, C.c_int64]),
            "ccka_host_build_world": (C.c_int, [vp, C.c_char_p, C.c_int32, C.c_int32,
                                                C.POINTER(abi.World)]),
            "ccka_host_summary": (C.c_int, [vp, C.POINTER(abi.World), C.POINTER(abi.Results),
                                            C.POINTER(abi.TrajRec), C.c_void_p, C.c_char_p, C.c_int64]),
            "ccka_host_label": (C.c_int, [vp, C.c_char_p, C.c_char_p, C.c_char_p, C.c_int32]),
            "ccka_host_export_detail": (C.c_int, [vp, C.POINTER(abi.World), C.c_void_p, C.c_int64, C.c_int64,
                                                  C.c_int64, C.c_char_p, C.c_int64, C.POINTER(C.c_int64)]),
            "ccka_host_export": (C.c_int, [vp, C.c_int32, C.POINTER(abi.World), C.POINTER(abi.TrajRec),
                                           C.c_int64, C.POINTER(abi.Results), C.c_int64, C.c_int64,
                                           C.c_int64, C.c_int64, C.c_char_p, C.c_int64,
                                           C.POINTER(C.c_int64)]),
            "ccka_host_set_admission": (C.c_int, [vp, C.c_uint32]),
            "ccka_host_admission_review": (C.c_int, [vp, C.c_uint32, C.c_char_p, C.c_char_p, C.c_int64]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _LIB = L
    return _LIB


HOST_EXPORTED = ["ccka_host_open", "ccka_host_close", "ccka_host_last_error", "ccka_host_apply",
                 "ccka_host_patch", "ccka_host_get_json", "ccka_host_policy_patch",
                 "ccka_host_burst_manifest", "ccka_host_build_world", "ccka_host_summary",
                 "ccka_host_export", "ccka_host_set_admission", "ccka_host_admission_review",
                 "ccka_host_label", "ccka_host_export_detail"]

# Kyverno guard policies (04_kyverno.sh:24-75), ccka_host.h CCKA_ADMIT_*
ADMIT_REQUIRE_REQUESTS_LIMITS = 1
ADMIT_CRITICAL_NO_SPOT = 2
ADMIT_ALL = ADMIT_REQUIRE_REQUESTS_LIMITS | ADMIT_CRITICAL_NO_SPOT

EXPORT_PROMETHEUS = 1
EXPORT_CSV = 2


class Host:
    """One manifest store. Environment (NP_SPOT, OFFPEAK_ZONES, ...) is read at open."""

    def __init__(self):
        self.L = lib()
        self.h = C.c_void_p()
        abi.check(self.L.ccka_host_open(C.byref(self.h)), "ccka_host_open")
        self._buf = C.create_string_buffer(1 << 20)

    def close(self):
        if self.h:
            self.L.ccka_host_close(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _err(self, what):
        raise abi.CckaError(f"{what}: {self.L.ccka_host_last_error(self.h).decode()}")

    def _str(self, n, what):
        if n < 0:
            self._err(what)
        return self._buf.raw[:n].decode()

    def apply(self, yaml_text: str):
        if self.L.ccka_host_apply(self.h, yaml_text.encode()) != 0:
            self._err("apply")

    def set_admission(self, policies: int):
        if self.L.ccka_host_set_admission(self.h, policies) != 0:
            self._err("set_admission")

    def admission_review(self, yaml_text: str, policies: int = ADMIT_ALL) -> list:
        """Dry run: the violations of every document, [{kind, name, policy, rule, message, path}]."""
        import json
        return json.loads(self._str(self.L.ccka_host_admission_review(self.h, policies, yaml_text.encode(),
                                                                      self._buf, len(self._buf)),
                                    "admission_review"))

    def patch(self, kind, name, ptype, text):
        if self.L.ccka_host_patch(self.h, kind.encode(), name.encode(), ptype.encode(), text.encode()) != 0:
            self._err("patch")

    def get_json(self, kind, name) -> str:
        return self._str(self.L.ccka_host_get_json(self.h, kind.encode(), name.encode(), self._buf,
                                                   len(self._buf)), "get_json")

    def policy_patch(self, profile: int, pool: str, json_patch: bool, fallback=False) -> str:
        return self._str(self.L.ccka_host_policy_patch(self.h, profile, pool.encode(), int(json_patch),
                                                       int(fallback), self._buf, len(self._buf)),
                         "policy_patch")

    def manifest(self, index: int) -> str:
        return self._str(self.L.ccka_host_burst_manifest(self.h, index, self._buf, len(self._buf)),
                         "manifest")

    def build_world(self, catalog="tiny", n_steps=1440, max_nodes=16) -> abi.World:
        w = abi.World()
        if self.L.ccka_host_build_world(self.h, catalog.encode(), n_steps, max_nodes, C.byref(w)) != 0:
            self._err("build_world")
        return w

    def label(self, kind, name, labels: str, overwrite=True):
        """kubectl label <kind> <name> k=v ... [--overwrite] ("k-" removes)."""
        if self.L.ccka_host_label(self.h, kind.encode(), name.encode(), labels.encode(), int(overwrite)) != 0:
            self._err("label")

    def summary(self, world, results, traj=None, detail=None) -> str:
        """demo_41 summary of scenario 0; `detail` = ccka_detail records (abi.detail_dtype())."""
        tp = traj.ctypes.data_as(C.POINTER(abi.TrajRec)) if traj is not None else None
        if detail is not None:
            import numpy as np
            detail = np.ascontiguousarray(detail, abi.detail_dtype())
        dp = detail.ctypes.data if detail is not None else None
        return self._str(self.L.ccka_host_summary(self.h, C.byref(world), C.byref(results), tp, dp,
                                                  self._buf, len(self._buf)), "summary")

    def export_detail(self, world, detail, first_id=0, start_unix_ms=0) -> str:
        """Per-pool Prometheus series of the ccka_detail records (ccka_host_export_detail)."""
        import numpy as np
        detail = np.ascontiguousarray(detail, abi.detail_dtype())
        need = C.c_int64(0)
        args = (self.h, C.byref(world), detail.ctypes.data, detail.size, first_id, start_unix_ms)
        if self.L.ccka_host_export_detail(*args, None, 0, C.byref(need)) != 0 and need.value <= 0:
            self._err("export_detail")
        buf = C.create_string_buffer(need.value)
        if self.L.ccka_host_export_detail(*args, buf, need.value, C.byref(need)) != 0:
            self._err("export_detail")
        return buf.value.decode()

    def export(self, world, results: dict, traj, fmt=EXPORT_PROMETHEUS, s0=0, n=None, first_id=0,
               start_unix_ms=0) -> str:
        """Trajectory export (ccka_host_export): Prometheus text exposition or CSV for
        scenarios [s0, s0 + n) of `traj` ([n_steps][traj_n] TRAJ_DTYPE) and the per-scenario
        `results` arrays (any subset of abi.RESULT_FIELDS; missing families are omitted)."""
        import numpy as np
        traj = np.ascontiguousarray(traj)
        traj_n = traj.shape[1]
        n = traj_n - s0 if n is None else n
        r = abi.Results()
        keep = []
        for name, ct, dt in abi.RESULT_FIELDS:
            if name in results:
                a = np.ascontiguousarray(results[name], dt)
                keep.append(a)
                setattr(r, name, a.ctypes.data_as(C.POINTER(ct)))
        tp = traj.ctypes.data_as(C.POINTER(abi.TrajRec))
        need = C.c_int64(0)
        args = (self.h, fmt, C.byref(world), tp, traj_n, C.byref(r), s0, n, first_id, start_unix_ms)
        if self.L.ccka_host_export(*args, None, 0, C.byref(need)) != 0 and need.value <= 0:
            self._err("export")
        buf = C.create_string_buffer(need.value)
        if self.L.ccka_host_export(*args, buf, need.value, C.byref(need)) != 0:
            self._err("export")
        return buf.raw[:need.value - 1].decode()
