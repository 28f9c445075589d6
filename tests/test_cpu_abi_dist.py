"""CPU-side checks: the C ABI libraries load and export every declared symbol,
the ctypes mirrors match the C struct layouts, the product path refuses to run
without a GPU (no CPU fallback), and the multi-rank path (scenario sharding +
totals all-reduce) reproduces the single-rank totals with world_size 2 over
gloo through libccka's own halves of the exchange (ccka_totals_pack /
ccka_totals_finish); fixed-point totals have headroom and report overflow
instead of wrapping."""
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
    # a rank whose totals could overflow the sum: every rank sees the guard
    big = po.totals(res, n)
    if rank == 1:
        big.energy_uwmin = (1 << 63) - 1 - 10
    try:
        dist.reduce_totals(big)
        ovf = False
    except OverflowError:
        ovf = True
    q.put((rank, ovf, {f: getattr(tot, f) for f in dist.INT_TOTALS + dist.FP_TOTALS}))
    tdist.destroy_process_group()


def test_two_rank_gloo_sharding_matches_single_rank():
    n_per_rank, T = 300, 240
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, n_per_rank, T, q)) for r in range(2)]
    for p in procs:
        p.start()
    outs = [q.get(timeout=240) for _ in range(2)]
    got = [o[2] for o in outs if o[0] == 0][0]
    assert [o[1] for o in outs] == [True, True]  # both ranks refuse the overflowing sum
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


def _synthetic_results(n, energy_wmin, gco2=1.0):
    from ccka import abi as A
    arr = {}
    for name, _, dt in A.RESULT_FIELDS:
        arr[name] = np.zeros(n, dt)
    arr["energy_wmin"][:] = energy_wmin
    arr["gco2"][:] = gco2
    return arr


def test_energy_total_has_headroom_past_the_nanowatt_unit():
    # 2e6 config-3-sized scenarios (8,590 W.min each, profiles/round3/bench_config3.json):
    # 1.7e19 nW.min would wrap int64; the microwatt-minute sum is exact
    n, e = 2_000_000, 8590.125
    t = po.totals(_synthetic_results(n, e), n)
    assert t.energy_uwmin == n * 8_590_125_000
    assert n * int(e * 1e9) > (1 << 63) - 1
    assert t.energy_wmin == float(n * 8_590_125_000) * 1e-6


def test_totals_overflow_is_reported_not_wrapped():
    with pytest.raises(OverflowError):
        po.totals(_synthetic_results(1000, 1e13), 1000)  # 1e16 W.min: beyond int64 in uW.min
    # the host halves of the exchange: a rank's value above INT64_MAX / nranks sets the guard
    t = abi.Totals()
    t.energy_uwmin = (1 << 62)
    blk = dist.pack_totals(t, 1)
    assert blk[abi.TOTALS_BLOCK - 1] == 0
    assert dist.finish_totals(blk).energy_uwmin == 1 << 62
    blk = dist.pack_totals(t, 2)
    assert blk[abi.TOTALS_BLOCK - 1] == 1
    with pytest.raises(OverflowError):
        dist.finish_totals(blk)


def test_pack_finish_round_trip_derives_doubles():
    t = abi.Totals()
    for k, f in enumerate(dist.INT_TOTALS):
        setattr(t, f, 1000 * k + 7)
    blk = dist.pack_totals(t, 8)
    assert blk[:abi.TOTALS_INT64] == [getattr(t, f) for f in dist.INT_TOTALS]
    out = dist.finish_totals([8 * v for v in blk])  # as if 8 equal ranks were summed
    for f in dist.INT_TOTALS:
        assert getattr(out, f) == 8 * getattr(t, f)
    assert out.energy_wmin == float(out.energy_uwmin) * 1e-6
    assert out.gco2 == float(out.gco2_ug) * 1e-6
