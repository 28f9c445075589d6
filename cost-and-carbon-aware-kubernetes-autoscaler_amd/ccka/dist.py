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
              "node_min_od", "launches", "deletions", "energy_nwmin", "gco2_ug"]
FP_TOTALS = ["energy_wmin", "gco2"]


def shard(n_per_rank: int, rank: int) -> tuple[int, int]:
    """(first global id, count) of a rank's scenarios."""
    return rank * n_per_rank, n_per_rank


def finish_totals(t: abi.Totals) -> abi.Totals:
    """Re-derive the doubles from the summed fixed-point fields (as
    ccka_allreduce_totals does after its all-reduce)."""
    t.energy_wmin = float(t.energy_nwmin) * 1e-9
    t.gco2 = float(t.gco2_ug) * 1e-6
    return t


def reduce_totals(t: abi.Totals, device=None) -> abi.Totals:
    """Sum a Totals struct over the default process group: the same exchange
    as ccka_allreduce_totals (one all-reduce of the int64 block, exact at any
    rank count, then the doubles re-derived)."""
    import torch
    import torch.distributed as dist

    ints = torch.tensor([getattr(t, f) for f in INT_TOTALS], dtype=torch.int64, device=device)
    dist.all_reduce(ints)
    out = abi.Totals()
    for f, v in zip(INT_TOTALS, ints.tolist()):
        setattr(out, f, int(v))
    return finish_totals(out)


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
