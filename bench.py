#!/usr/bin/env python3
"""Benchmark: policy-evaluated cluster-steps/s of the HIP rollout engine.

Workload (BASELINE.json configs[1]): 1e5 clusters x 1 deployment x 1440
one-minute steps, HPA + peak/off-peak policy, synthetic load, per GPU
(weak scaling: rank r owns global scenarios [r*N, (r+1)*N)). One "step" of
this benchmark = one full rollout of that batch (1.44e8 cluster-steps per GPU).
Inputs (load traces, parameters) are generated on the device before timing and
stay resident in HBM.

Prints ONE JSON line (rank 0). Fields beyond the driver contract:
  roofline      HBM roofline of the rollout kernel (HIP-event duration)
  cpu_baseline  the CPU oracle (plain C, same semantics) on a bounded sample
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "cost-and-carbon-aware-kubernetes-autoscaler_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--n", type=int, default=100_000, help="scenarios per GPU")
    ap.add_argument("--T", type=int, default=1440)
    ap.add_argument("--mode", choices=["trajectory", "summary"], default="trajectory")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="target CPU baseline duration")
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch

    dist = None
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    from ccka import configs
    from ccka.engine import Engine

    eng = Engine(local)
    spec = configs.config2_world(n_steps=args.T)
    sc = configs.hpa_scenarios(args.n, first_id=rank * args.n)
    eng.set_world(spec)
    eng.set_scenarios(sc)
    eng.gen_load(configs.trace_gen())
    traj = args.mode == "trajectory"

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
        eng.sync()

    for _ in range(args.warmup):
        eng.rollout(trajectory=traj)
    barrier()
    t0 = time.perf_counter()
    kms = []
    for _ in range(args.steps):
        eng.rollout_async(trajectory=traj)
        eng.sync()
        kms.append(eng.kernel_ms())
    barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    totals = eng.totals()
    if dist is not None:
        # the only cross-GPU exchange: packed totals, RCCL all-reduce inside libccka
        import ctypes as C

        from ccka import dist as cdist

        uid = (C.c_uint8 * 128).from_buffer_copy(cdist.unique_id_exchange(eng, rank))
        eng._chk(eng.lib.ccka_comm_init(eng.ctx, uid, world, rank), "ccka_comm_init")
        eng._chk(eng.lib.ccka_allreduce_totals(eng.ctx, C.byref(totals)), "ccka_allreduce_totals")

    T, N, K = args.T, args.n, args.steps
    steps_total = world * N * T * K
    value = steps_total / elapsed
    avg_ms = sum(kms) / len(kms)
    # algorithmic bytes per launch: load [T][N] int32 read once, trajectory 16 B
    # per cluster-step written once, per-scenario params (region u8, target i16,
    # max i16, cap_sel u8 = 6 B) read once, results (4x8 + 10x4 = 72 B) written once
    bytes_launch = N * T * 4 + (N * T * 16 if traj else 0) + N * 6 + N * 72
    achieved = bytes_launch / (avg_ms * 1e-3) / 1e9
    traffic = measured_traffic(args.mode, N, T)
    out = {
        "metric": "policy-evaluated cluster-steps/sec",
        "value": value,
        "unit": "cluster-steps/s",
        "n_gpus": world,
        "steps": K,
        "warmup": args.warmup,
        "ms_per_step": elapsed / K * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int32+f64",
        "data": "synthetic (on-device Philox load traces, seed 20251205)",
        "config": {"workload": "config2: 1e5 clusters x 1 deployment x 1440 one-minute steps, "
                               "HPA + peak/off-peak, 16-type catalog",
                   "scenarios_per_gpu": N, "steps_per_rollout": T, "mode": args.mode,
                   "parallelism": f"scenario-sharded x{world}"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": "rollout_kernel<1,8>", "kernel_ms_avg": avg_ms,
                     "bytes_per_launch": bytes_launch},
        "totals": {"cost_usd": totals.cost_uphmin / 6e7, "energy_kwh": totals.energy_wmin / 6e4,
                   "gco2_kg": totals.gco2 / 1e3, "slo_minutes": totals.slo_minutes,
                   "launches": totals.launches, "deletions": totals.deletions},
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline(eng, spec, sc, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


def measured_traffic(mode, n, T):
    """HBM bytes per launch of the rollout kernel measured by rocprofv3 PMC
    passes of this same command (tools/prof_round.sh; L2 memory-side request
    counters TCC_EA0_RDREQ_{32,64,128}B x size + TCC_EA0_WRREQ_64B x 64), kept
    under profiles/. None when no profile matches this workload."""
    import glob

    name = "config2_traj_summary.json" if mode == "trajectory" else "config2_summary_summary.json"
    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "round*", name)))
    if not paths or (n, T) != (100_000, 1440):
        return None
    return json.load(open(paths[-1])).get("traffic_bytes")


def cpu_baseline(eng, spec, sc, target_s):
    """The CPU oracle (plain C restatement, gcc -O3, pthreads over contiguous
    scenario shards) on the same workload: the same global ids and the same
    device-generated traces (copied to the host, untimed). The full batch is
    rolled out repeatedly until ~target_s of CPU time; the median run is
    reported. A 1-thread figure on a prefix of the batch is added beside it."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as po

    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    load = eng.get_load()
    T = spec.n_steps

    def run(n, th):
        sub = sc.slice(0, n)
        ld = np.ascontiguousarray(load[:, :, :n])
        t0 = time.perf_counter()
        po.rollout(spec, sub, ld, threads=th)
        return time.perf_counter() - t0

    times = [run(sc.n, threads)]
    while sum(times) < target_s and len(times) < 25:
        times.append(run(sc.n, threads))
    times.sort()
    med = times[len(times) // 2]
    n1 = min(sc.n, 8192)
    t1 = run(n1, 1)
    return {"value": sc.n * T / med, "unit": "cluster-steps/s", "cores": threads, "kind": "port",
            "sample": f"full batch {sc.n} scenarios x {T} steps, median of {len(times)} runs "
                      f"({med:.3f} s each) on {threads} threads",
            "value_1thread": n1 * T / t1, "sample_1thread": f"{n1} scenarios x {T} steps, {t1:.2f} s"}


if __name__ == "__main__":
    main()
