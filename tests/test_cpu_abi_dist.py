"""CPU-side checks: the C ABI libraries load and export every declared symbol,
the ctypes mirrors match the C struct layouts, the product path refuses to run
without a GPU (no CPU fallback), and the multi-rank path (scenario sharding +
totals all-reduce) reproduces the single-rank totals with world_size 2 over
gloo."""
import ctypes as C
import os
import re
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import pyoracle as po
from ccka import abi, configs, dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared(header):
    txt = open(os.path.join(ROOT, "include", header)).read()
    return sorted(set(re.findall(r"^\w[\w\s\*]*?\b(ccka_\w+)\s*\(", txt, re.M)))


def test_engine_library_exports_header_symbols():
    lib = C.CDLL(abi.ENGINE_LIB)
    syms = declared("ccka.h")
    assert "ccka_rollout" in syms and "ccka_allreduce_totals" in syms
    for s in syms:
        assert hasattr(lib, s), s
    assert sorted(abi.EXPORTED) == syms


def test_host_library_exports_header_symbols():
    from ccka.host import HOST_EXPORTED, lib
    L = lib()
    syms = declared("ccka_host.h")
    for s in syms:
        assert hasattr(L, s), s
    assert sorted(HOST_EXPORTED) == syms


def test_struct_layouts_match():
    lib = abi.load_engine()
    abi.check_sizes(lib)
    assert lib.ccka_abi_version() == abi.ABI_VERSION


def test_no_cpu_fallback_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    lib = abi.load_engine()
    ctx = C.c_void_p()
    assert lib.ccka_open(C.byref(ctx), 0) == -7  # CCKA_ENODEV
    from ccka.engine import Engine
    with pytest.raises(abi.CckaError):
        Engine(0)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, n_per_rank, T, q):
    import torch.distributed as tdist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    tdist.init_process_group("gloo", rank=rank, world_size=world)
    first, n = dist.shard(n_per_rank, rank)
    spec = configs.config2_world(n_steps=T)
    sc = configs.hpa_scenarios(n, first_id=first)
    load = po.gen_load(configs.trace_gen(), T, 1, n, first_id=first)
    res, _ = po.rollout(spec, sc, load, threads=2)
    tot = dist.reduce_totals(po.totals(res, n))
    if rank == 0:
        q.put({f: getattr(tot, f) for f in dist.INT_TOTALS + dist.FP_TOTALS})
    tdist.destroy_process_group()


def test_two_rank_gloo_sharding_matches_single_rank():
    n_per_rank, T = 300, 240
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, n_per_rank, T, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    spec = configs.config2_world(n_steps=T)
    sc = configs.hpa_scenarios(2 * n_per_rank)
    load = po.gen_load(configs.trace_gen(), T, 1, 2 * n_per_rank)
    res, _ = po.rollout(spec, sc, load, threads=4)
    want = po.totals(res, 2 * n_per_rank)
    # every field bit-identical to the single-rank totals: the int64 block is
    # an exact sum, and the doubles derive from it
    for f in dist.INT_TOTALS + dist.FP_TOTALS:
        assert got[f] == getattr(want, f), f


def test_per_scenario_params_are_functions_of_global_id():
    a = configs.hpa_scenarios(1000)
    b = configs.hpa_scenarios(400, first_id=600)
    for f in ("target_util_pct", "max_replicas", "cap_sel", "region"):
        assert np.array_equal(getattr(a, f)[600:], getattr(b, f)), f
