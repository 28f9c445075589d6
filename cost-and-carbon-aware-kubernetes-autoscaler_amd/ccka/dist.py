"""Multi-GPU helpers: scenario sharding and the totals exchange.

Scenarios are independent: rank r owns the contiguous global
ids [r*N, (r+1)*N) (weak scaling); per-scenario inputs are pure functions of
the global id, so results do not depend on the rank count. The only exchange
is a sum of the packed totals: ccka_allreduce_totals (RCCL over xGMI) inside
libccka, or `reduce_totals` below through torch.distributed (RCCL on GPU,
gloo on CPU tests).
"""
from __future__ import annotations

from . import abi

# the int64 block of ccka_totals (CCKA_TOTALS_INT64): energy and gCO2 in fixed
# point, so the sum is exact at any rank count; the doubles derive from it
INT_TOTALS = ["scenarios", "cost_uphmin", "slo_minutes", "pending_pod_minutes", "node_min_spot",
              "node_min_od", "launches", "deletions", "energy_uwmin", "gco2_ug"]
FP_TOTALS = ["energy_wmin", "gco2"]


def shard(n_per_rank: int, rank: int) -> tuple[int, int]:
    """(first global id, count) of a rank's scenarios."""
    return rank * n_per_rank, n_per_rank


def pack_totals(t: abi.Totals, nranks: int) -> list[int]:
    """libccka's ccka_totals_pack: the CCKA_TOTALS_BLOCK int64 words this rank
    contributes (the int64 fields + the overflow guard)."""
    import ctypes as C

    lib = abi.load_engine()
    blk = (C.c_int64 * abi.TOTALS_BLOCK)()
    abi.check(lib.ccka_totals_pack(C.byref(t), nranks, blk, abi.TOTALS_BLOCK), "ccka_totals_pack")
    return list(blk)


def finish_totals(block) -> abi.Totals:
    """libccka's ccka_totals_finish on a summed block: the totals with the
    doubles re-derived (as ccka_allreduce_totals after its all-reduce);
    OverflowError when the guard word says the sum left int64."""
    import ctypes as C

    lib = abi.load_engine()
    blk = (C.c_int64 * abi.TOTALS_BLOCK)(*[int(v) for v in block])
    out = abi.Totals()
    st = lib.ccka_totals_finish(blk, abi.TOTALS_BLOCK, C.byref(out))
    if st == abi.EOVERFLOW:
        raise OverflowError("ccka_totals_finish: a summed total exceeds int64")
    abi.check(st, "ccka_totals_finish")
    return out


def reduce_totals(t: abi.Totals, device=None) -> abi.Totals:
    """Sum a Totals struct over the default process group with libccka's own
    halves of ccka_allreduce_totals (ccka_totals_pack -> an int64 sum over
    torch.distributed: RCCL on GPU, gloo in the CPU tests -> ccka_totals_finish),
    exact and bit-identical at any rank count."""
    import torch
    import torch.distributed as dist

    blk = torch.tensor(pack_totals(t, dist.get_world_size()), dtype=torch.int64, device=device)
    dist.all_reduce(blk)
    return finish_totals(blk.tolist())


def unique_id_exchange(eng, rank: int) -> bytes:
    """Rank 0 creates the RCCL unique id via the C ABI; broadcast it."""
    import ctypes as C

    import torch.distributed as dist

    uid = (C.c_uint8 * 128)()
    if rank == 0:
        abi.check(eng.lib.ccka_comm_unique_id(uid), "ccka_comm_unique_id")
    obj = [bytes(uid)]
    dist.broadcast_object_list(obj, src=0)
    return obj[0]
