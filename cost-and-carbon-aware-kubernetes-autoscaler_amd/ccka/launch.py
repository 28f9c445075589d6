"""One process per GPU: the rank launcher behind `bench.py --gpus N`.

The parent never touches a GPU (it does not import torch): it starts N fresh
child processes of the same command, each with RANK / LOCAL_RANK / WORLD_SIZE /
MASTER_ADDR / MASTER_PORT in its environment (the variables torchrun sets, so
a child cannot tell the two launchers apart), waits for all of them and exits
with the first non-zero status. A child that fails takes the others down
(killed by PID, never by pattern), so a rank stuck in a collective cannot
outlive its peers.
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys
import time

RANK_VARS = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def rank_env(rank: int, world: int, port: int, base: dict | None = None) -> dict:
    env = dict(os.environ if base is None else base)
    env.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    # dmabuf IPC only on this driver (RCCL / cross-process buffers)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return env


def spawn_ranks(world: int, argv: list[str], poll_s: float = 0.2, port: int | None = None) -> int:
    """Run `python argv...` as `world` rank processes; returns the exit status."""
    if world < 1:
        raise ValueError("world must be >= 1")
    port = port or free_port()
    procs = [subprocess.Popen([sys.executable] + list(argv), env=rank_env(r, world, port))
             for r in range(world)]
    status = 0
    live = list(procs)
    while live:
        for p in list(live):
            rc = p.poll()
            if rc is None:
                continue
            live.remove(p)
            if rc != 0 and status == 0:
                status = rc if rc > 0 else 128 - rc
                for q in live:  # a failed rank: stop its peers (exact PIDs)
                    q.terminate()
        time.sleep(poll_s)
    for p in procs:
        p.wait()
    return status


def is_rank_process() -> bool:
    """True when launched as one rank (by spawn_ranks or torchrun)."""
    return "WORLD_SIZE" in os.environ and "RANK" in os.environ
