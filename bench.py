#!/usr/bin/env python3
"""Benchmark: policy-evaluated cluster-steps/s of the HIP rollout engine.

Default workload = BASELINE.json configs[1] (config 2): 1e5 clusters x 1
deployment x 1440 one-minute steps, HPA + peak/off-peak, per GPU (weak
scaling: rank r owns global scenarios [r*N, (r+1)*N)). One "step" of this
benchmark = one full rollout of that batch (1.44e8 cluster-steps per GPU).
Inputs (load traces, parameters) are generated on the device before timing and
stay resident in HBM.

Other BASELINE configs (reported the same way, selected with --config):
  3  1e6 scenarios x 1440 steps over 8 regions, ~800-type catalog, carbon-
     weighted Karpenter argmin; the 1e6 are split over the ranks (strong scaling)
  4  policy sweep: 4096 parameter grids x 1024 shared load traces x 1440 steps,
     grids sharded over the ranks (weak in grids per rank = 4096/N), per-grid
     sums + cost/gCO2/SLO Pareto frontier exchanged with RCCL all-gather
  5  learned MLP policy 64->256->256->8, bf16 MFMA, 1e7 states per GPU

Prints ONE JSON line (rank 0). Fields beyond the driver contract:
  roofline      of the dominant kernel (HIP-event duration on the engine stream)
  cpu_baseline  the CPU oracle (plain C, same semantics) on a bounded sample
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "cost-and-carbon-aware-kubernetes-autoscaler_amd"))

HBM_PEAK_GBS = 8000.0      # MI355X HBM3E peak (MI355X_MICROARCH.md)
BF16_DENSE_TFLOPS = 2500.0  # MI355X dense bf16 MFMA peak (no sparsity)
MLP_FLOPS_PER_STATE = 2 * (64 * 256 + 256 * 256 + 256 * 8)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=None,
                    help="untimed warmup steps (default: 50 for config 5, whose 1 ms launches need ~50 ms "
                         "of sustained load before the shader clock settles; 2 otherwise)")
    ap.add_argument("--config", type=int, choices=[2, 3, 4, 5], default=2)
    ap.add_argument("--n", type=int, default=None, help="scenarios (states) per GPU, overrides the config")
    ap.add_argument("--T", type=int, default=1440)
    ap.add_argument("--mode", choices=["trajectory", "summary", "policy", "grad"], default=None,
                    help="config 5: 'policy' = the closed-loop policy rollout (MLP in the loop every step); "
                         "'grad' = the differentiable-control step: a stochastic closed-loop rollout plus the "
                         "score-function gradient of E[cost + w gCO2 + w SLO] (ccka_policy_grad)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="target CPU baseline duration")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--drift", action="store_true",
                    help="configs 2-4 with Karpenter drift at the zone switch (SEMANTICS 3.G0; general kernel)")
    ap.add_argument("--replace", action="store_true",
                    help="configs 2-4 with single-node replacement consolidation (SEMANTICS 3.G2)")
    ap.add_argument("--multi", action="store_true",
                    help="configs 2-4 with multi-node consolidation (SEMANTICS 3.G3, Karpenter's default for "
                         "WhenEmptyOrUnderutilized pools)")
    ap.add_argument("--deployments", type=int, default=1,
                    help="config 2 with this many HPA deployments sharing each cluster's nodes (the general "
                         "kernel's multi-deployment layouts; 8 node slots up to 2 deployments, else 16; from 5 on "
                         "the demo_30 burst shape: alternating spot / on-demand deployments of 5 replicas, "
                         "max 10 each, no per-scenario overrides)")
    ap.add_argument("--lockstep", action="store_true",
                    help="--deployments: the general kernel in lockstep instead of its lane-skewed schedule (A/B)")
    ap.add_argument("--mlp-tile", type=int, choices=(16, 32), default=16,
                    help="config 5 forward: mlp16_kernel (16x16x32 MFMA, default) or mlp_kernel (32x32x16)")
    ap.add_argument("--keda", action="store_true",
                    help="configs 2-3 with a KEDA ScaledObject queue worker instead of the HPA deployment "
                         "(SURVEY A.2 defaults: scale from / to zero, cooldown 300 s, min 0, max 100; threshold "
                         "500 per replica, activation 0; docs/SEMANTICS.md 3.C)")
    ap.add_argument("--budget", type=int, default=None,
                    help="NodePool disruption budget in %% of the pool's nodes (default: the reference's 10)")
    ap.add_argument("--hpa-sync", type=int, default=0, choices=[0, 10, 15, 20, 30, 60],
                    help="HPA decision period in seconds (Kubernetes default 15: four decisions per one-minute "
                         "step; 0 = one per step)")
    ap.add_argument("--no-graph", action="store_true",
                    help="config 5 --mode policy/grad with --launched: enqueue the loop's launches directly instead "
                         "of replaying its captured hipGraph")
    ap.add_argument("--launched", action="store_true",
                    help="config 5 --mode policy/grad: the launched loop (general kernel + MLP + action kernels per "
                         "step) instead of the fused one-launch loop")
    ap.add_argument("--trace-flat", action="store_true",
                    help="single-deployment kernel: read the [T][N] load trace instead of its wave-tiled copy "
                         "(layout A/B; same results)")
    ap.add_argument("--spawn", action="store_true",
                    help="run the ranks as fresh child processes even at --gpus 1 (the launcher path)")
    args = ap.parse_args()
    if args.deployments > 1 and (args.config != 2 or args.keda):
        ap.error("--deployments applies to config 2 with HPA deployments only (not with --keda)")

    # one process per GPU: without a launcher's rank environment, this process
    # only starts the N rank processes (it never touches a GPU itself)
    from ccka import launch

    if not launch.is_rank_process() and (args.gpus > 1 or args.spawn):
        sys.exit(launch.spawn_ranks(args.gpus, [os.path.abspath(__file__)] + sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
    import torch

    dist = None
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    from ccka import abi, configs
    from ccka import dist as cdist
    from ccka.engine import Engine

    eng = Engine(local)

    rccl = {}

    def comm_init():
        """RCCL communicator of libccka (also at one rank: the same exchange
        code runs); records the rank count the communicator reports."""
        if world > 1:
            uid = (C.c_uint8 * 128).from_buffer_copy(cdist.unique_id_exchange(eng, rank))
        else:
            uid = (C.c_uint8 * 128)()
            eng._chk(eng.lib.ccka_comm_unique_id(uid), "ccka_comm_unique_id")
        eng._chk(eng.lib.ccka_comm_init(eng.ctx, uid, world, rank), "ccka_comm_init")
        nr, rk = C.c_int32(), C.c_int32()
        eng._chk(eng.lib.ccka_comm_info(eng.ctx, C.byref(nr), C.byref(rk)), "ccka_comm_info")
        rccl.update(nranks=nr.value, rank=rk.value)

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
        eng.sync()

    cfg = args.config
    if args.warmup is None:
        args.warmup = 50 if cfg == 5 and args.mode != "policy" else (1 if cfg == 5 else 2)
    T = args.T
    spec = sc = None
    policy = cfg == 5 and args.mode in ("policy", "grad")
    grad = cfg == 5 and args.mode == "grad"
    if policy:
        # closed loop: every step featurize -> MLP (bf16 MFMA) -> actions -> one rollout step
        N = args.n or (250_000 if grad else 1_000_000)
        T = args.T if args.T != 1440 else 60
        spec = configs.config2_world(n_steps=T)
        sc = configs.hpa_scenarios(N, first_id=rank * N)
        ws, bs = configs.mlp_weights(11)
        eng.mlp_set_weights([configs.to_bf16_bits(w) for w in ws], bs)
        eng.set_world(spec)
        eng.set_scenarios(sc)
        eng.gen_load(configs.trace_gen())
        traj = False
        fn = eng.lib.ccka_debug_policy_graph
        fn.argtypes = [C.c_void_p, C.c_int32]
        eng._chk(fn(eng.ctx, 0 if args.no_graph else 1), "ccka_debug_policy_graph")
        fu = eng.lib.ccka_debug_policy_fused
        fu.argtypes = [C.c_void_p, C.c_int32]
        eng._chk(fu(eng.ctx, 0 if args.launched else 1), "ccka_debug_policy_fused")

        grad_obj = []

        def step_fn():
            if grad:  # one policy-gradient step's data: rollout + MLP backward over N x T rows
                grad_obj.append(eng.policy_grad(seed=len(grad_obj) + 1, w_carbon=0.05, w_slo=0.01)[1])
            else:
                eng.policy_rollout(trajectory=False)
    elif cfg == 5:
        N = args.n or 10_000_000
        ws, bs = configs.mlp_weights(11)
        eng.mlp_set_weights([configs.to_bf16_bits(w) for w in ws], bs)
        eng.mlp_gen_states(N, seed=7 + rank)
        mt = eng.lib.ccka_debug_mlp_tile
        mt.argtypes = [C.c_void_p, C.c_int32]
        eng._chk(mt(eng.ctx, args.mlp_tile), "ccka_debug_mlp_tile")
        step_fn = eng.mlp_forward_async
        traj = False
    else:
        if cfg == 2:
            N = args.n or 100_000
            spec = configs.config2_world(n_steps=T)
            sc = configs.hpa_scenarios(N, first_id=rank * N)
            gen = configs.trace_gen()
            traj = (args.mode or "trajectory") == "trajectory"
        elif cfg == 3:
            total = args.n or 1_000_000
            N = total // world
            spec = configs.config3_world(n_steps=T)
            sc = configs.config3_scenarios(N, first_id=rank * N)
            gen = configs.trace_gen()
            traj = (args.mode or "summary") == "trajectory"
        else:
            grids = configs.CONFIG4_GRIDS // world
            ntr = configs.CONFIG4_TRACES
            N = grids * ntr
            spec = configs.config2_world(n_steps=T)
            sc = configs.config4_scenarios(rank * grids, grids, ntr)
            gen = configs.config4_trace_gen()
            traj = (args.mode or "summary") == "trajectory"
        if args.deployments > 1:  # several HPA deployments per cluster (demo_30's burst shape)
            if args.deployments <= 4:
                spec.deploys = [configs.deployment(abi.SCALER_HPA, replicas0=3, max_r=30,
                                                   req_cpu=(200, 300, 250, 400)[d % 4], target=(70, 60, 80, 50)[d % 4])
                                for d in range(args.deployments)]
            else:
                # demo_30_burst_configure.sh:57-151: odd (1-based) deployments select spot, even
                # on-demand, 5 replicas each; each keeps its own capacity type and bounds
                spec.deploys = [configs.deployment(abi.SCALER_HPA, replicas0=5, max_r=10,
                                                   cap_sel=abi.CAP_SPOT if d % 2 == 0 else abi.CAP_OD,
                                                   req_cpu=(200, 300, 250, 400)[d % 4], target=(70, 60, 80, 50)[d % 4])
                                for d in range(args.deployments)]
                sc.cap_sel = None
                sc.max_replicas = None
                sc.target_util_pct = None
            spec.max_nodes = 8 if args.deployments <= 2 else 16
        if args.keda:  # the queue-worker side of the path: one ScaledObject per scenario
            spec.deploys = [configs.deployment(abi.SCALER_KEDA, replicas0=0, keda_threshold=500, keda_activation=0,
                                               keda_cooldown=300, keda_min=0, keda_max=100)]
        spec.drift = int(args.drift)
        spec.replace = int(args.replace)
        spec.multi = int(args.multi)
        spec.hpa_sync_s = args.hpa_sync
        if args.budget is not None:
            for pool in spec.pools:
                pool.budget_pct = args.budget
        eng.set_world(spec)
        eng.set_scenarios(sc)
        if args.lockstep:
            eng.set_engine(2)
        if args.trace_flat:
            tf = eng.lib.ccka_debug_trace_flat
            tf.argtypes = [C.c_void_p, C.c_int32]
            eng._chk(tf(eng.ctx, 1), "ccka_debug_trace_flat")
        eng.gen_load(gen)
        if cfg == 4:
            comm_init()
        frontier = []

        def step_fn():
            eng.rollout_async(trajectory=traj)
            if cfg == 4:  # per-grid sums + Pareto frontier (RCCL all-gather at N > 1)
                frontier.append(len(eng.pareto(configs.CONFIG4_TRACES)))

    for _ in range(args.warmup):
        step_fn()
        if cfg != 5:
            eng.sync()
    eng.sync()
    barrier()
    t0 = time.perf_counter()
    kms = []
    if policy:
        for _ in range(args.steps):
            step_fn()
            kms.append(eng.kernel_ms())
    elif cfg == 5:
        # back-to-back launches, one sync: the policy kernel is ~1 ms, and a
        # host round trip per launch lets the shader clock sag between them;
        # an event pair around every launch gives the mean kernel duration
        # (the figure rocprofv3's kernel trace averages)
        avg, span = C.c_double(), C.c_double()
        fn = eng.lib.ccka_debug_mlp_batch
        fn.argtypes = [C.c_void_p, C.c_int32, C.POINTER(C.c_double), C.POINTER(C.c_double)]
        eng._chk(fn(eng.ctx, args.steps, C.byref(avg), C.byref(span)), "ccka_debug_mlp_batch")
        kms = [avg.value]
    else:
        for _ in range(args.steps):
            step_fn()
            eng.sync()
            kms.append(eng.kernel_ms())
    barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    K = args.steps
    avg_ms = sum(kms) / len(kms)
    engine_id, table_ms = eng.last_engine() if cfg != 5 or policy else (0, 0.0)

    if policy:
        value = world * N * T * K / elapsed
        # dominant MFMA work: one MLP batch over the N states per rollout step
        # (+ for the gradient: the forward recomputed and the backward over
        # the N x T rows: dH2 = W3 g, dH1 = W2 dH2, dW1..3, db)
        flops = MLP_FLOPS_PER_STATE * N * T * (1 if not grad else 2) + \
            (2 * (256 * 8 + 256 * 256 + 64 * 256 + 256 * 256 + 256 * 8) * N * T if grad else 0)
        if grad:  # the loop's events do not cover the backward: the whole step's wall time
            avg_ms = elapsed / K * 1e3
        achieved = flops / (avg_ms * 1e-3) / 1e12
        out = {
            "metric": "policy-evaluated cluster-steps/sec (closed-loop MLP control policy)" if not grad else
                      "policy-gradient cluster-steps/sec (stochastic closed loop + score-function MLP backward)",
            "value": value, "unit": "cluster-steps/s", "n_gpus": world, "steps": K,
            "warmup": args.warmup, "ms_per_step": elapsed / K * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "bf16 MLP (fp32 accumulate) + int64/f64 rollout",
            "data": "synthetic (on-device Philox traces, Xavier-uniform weights seed 11)",
            "config": {"workload": (f"config5 closed loop: {N} clusters x {T} steps, every step featurize -> "
                                    "MLP 64->256->256->8 -> HPA target + carbon weight -> rollout step") if not grad
                       else (f"config5 differentiable control: {N} clusters x {T} steps, stochastic policy "
                             "(8 action bins, softmax sampling), objective cost + 0.05 $/kg gCO2 + 0.01 $/SLO-min, "
                             f"score-function gradient over {N * T} (step, cluster) rows"),
                       "clusters_per_gpu": N, "steps": T, "parallelism": f"data-parallel x{world}",
                       "launch": ("fused: one launch per loop (features, MLP on MFMA and actions inside the "
                                  "rollout's step loop, rollout_kernel<1,8,POL>)") if not args.launched else
                                 ("launched: direct" if args.no_graph else "launched: hipGraph (captured loop, replayed)")},
            "roofline": {"bound": "mfma", "achieved": achieved, "peak": BF16_DENSE_TFLOPS, "unit": "TFLOP/s",
                         "frac": achieved / BF16_DENSE_TFLOPS, "traffic": None,
                         "kernel": (("whole loop: rollout_kernel<1,8,1> (fused)" if not args.launched else
                                     "whole loop (mlp_kernel + policy_act_kernel + rollout_kernel per step)")
                                    if not grad else "whole step (closed loop + pg_rows_kernel + pg_wgrad_kernel)"),
                         "loop_ms_avg": avg_ms, "flops_per_loop": flops},
        }
        if grad:
            out["objective_mean_usd"] = grad_obj[-1]
    elif cfg == 5:
        value = world * N * K / elapsed
        flops = MLP_FLOPS_PER_STATE * N
        achieved = flops / (avg_ms * 1e-3) / 1e12
        out = {
            "metric": "policy-evaluated cluster-states/sec (MLP control policy)",
            "value": value, "unit": "cluster-states/s", "n_gpus": world, "steps": K,
            "warmup": args.warmup, "ms_per_step": elapsed / K * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "bf16 (fp32 accumulate)",
            "data": "synthetic (on-device Philox states, Xavier-uniform weights seed 11)",
            "config": {"workload": "config5: MLP 64->256->256->8 over 1e7 cluster states per GPU",
                       "states_per_gpu": N, "parallelism": f"data-parallel x{world}"},
            "roofline": {"bound": "mfma", "achieved": achieved, "peak": BF16_DENSE_TFLOPS,
                         "unit": "TFLOP/s", "frac": achieved / BF16_DENSE_TFLOPS, "traffic": None,
                         "kernel": "mlp16_kernel" if args.mlp_tile == 16 else "mlp_kernel", "kernel_ms_avg": avg_ms,
                         "flops_per_launch": flops},
        }
        if rank == 0 and world == 1 and not args.no_cpu:
            out["cpu_baseline"] = cpu_baseline_mlp(args.cpu_seconds)
    else:
        local_totals = eng.totals()
        totals = abi.Totals.from_buffer_copy(local_totals)
        if cfg != 4:
            comm_init()
        # the cross-GPU exchange of the totals: RCCL all-reduce inside libccka
        eng._chk(eng.lib.ccka_allreduce_totals(eng.ctx, C.byref(totals)), "ccka_allreduce_totals")
        steps_total = (N * world if cfg != 3 else N * world) * T * K
        value = steps_total / elapsed
        # algorithmic bytes per launch: load [T][N] int32 read once (config 4:
        # the 1024 shared traces), trajectory 16 B per cluster-step written once
        # (trajectory mode), per-scenario params (6 B) read and results (72 B)
        # written once
        load_cols = (configs.CONFIG4_TRACES if cfg == 4 else N) * len(spec.deploys)
        bytes_launch = load_cols * T * 4 + (N * T * 16 if traj else 0) + N * 6 + N * 72
        achieved = bytes_launch / (avg_ms * 1e-3) / 1e9
        traffic, traffic_src = (None, None) if (args.drift or args.replace or args.multi or args.keda or
                                                args.deployments > 1 or
                                                args.hpa_sync not in (0, 60) or args.budget is not None or
                                                args.trace_flat) else measured_traffic(cfg, traj, N, T)
        workloads = {
            2: "config2: 1e5 clusters x 1 deployment x 1440 one-minute steps, HPA + peak/off-peak, "
               "16-type catalog",
            3: "config3: 1e6 scenarios x 1440 steps over 8 regions, 800-type catalog, carbon-weighted "
               "Karpenter argmin (scenarios split over the ranks)",
            4: "config4: policy sweep 4096 grids x 1024 shared traces x 1440 steps, per-grid sums + "
               "cost/gCO2/SLO Pareto frontier (RCCL all-gather)",
        }
        out = {
            "metric": "policy-evaluated cluster-steps/sec",
            "value": value, "unit": "cluster-steps/s", "n_gpus": world, "steps": K,
            "warmup": args.warmup, "ms_per_step": elapsed / K * 1e3, "higher_is_better": True,
            "scaling": "strong" if cfg == 3 else "weak", "vs_baseline": None, "dtype": "int32+int64+f64",
            "data": "synthetic (on-device Philox load traces, seed 20251205)",
            "config": {"workload": (workloads[cfg].replace("HPA", "KEDA ScaledObject (scale to zero)") if args.keda
                                    else workloads[cfg].replace("1 deployment", f"{args.deployments} HPA deployments "
                                                                f"sharing {spec.max_nodes} node slots"
                                                                + (" (demo_30 burst shape: alternating spot / "
                                                                   "on-demand, 5 replicas, max 10)"
                                                                   if args.deployments > 4 else ""))
                                    if args.deployments > 1 else workloads[cfg]) + (" + Karpenter drift at the zone switch" if args.drift else "")
                       + (" + replacement consolidation" if args.replace else "")
                       + (" + multi-node consolidation" if args.multi else "")
                       + (f" + HPA sync every {args.hpa_sync} s" if args.hpa_sync not in (0, 60) else "")
                       + (f", disruption budget {args.budget} %" if args.budget is not None else "")
,
                       "scenarios_per_gpu": N, "steps_per_rollout": T,
                       "mode": "trajectory" if traj else "summary",
                       "schedule": ("lane-skewed" if engine_id == 5 else "lockstep" if engine_id == 1 else "lane-skewed (single deployment)"
                                    if engine_id == 2 else None),
                       "trace_layout": "[T][N] (shared traces)" if cfg == 4 else "[T][N]" if args.trace_flat else
                       "[T][D][N]" if engine_id in (1, 5) else "wave-tiled [wave][T][lanes] (built by the first rollout)",
                       "parallelism": f"scenario-sharded x{world}", "rccl_nranks": rccl.get("nranks")},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS,
                         "traffic": traffic,
                         # not measured in this run: copied from the committed profile named here
                         "traffic_source": traffic_src,
                         "kernel": "rollout_d1_kernel<8,2>" if engine_id == 2 else
                                   "rollout_kernel<%d,%d,0,1> (lane-skewed)" % general_dims(len(spec.deploys), spec.max_nodes)
                                   if engine_id == 5 else
                                   "rollout_kernel<%d,%d>" % general_dims(len(spec.deploys), spec.max_nodes),
                         "kernel_ms_avg": avg_ms, "argmin_table_ms": table_ms,
                         "bytes_per_launch": bytes_launch},
            # the kernel is issue-bound, not HBM-bound: its measured issue-side
            # utilisation (profiled) and the measured copy ceiling
            # (profiled on the single-deployment kernel only)
            "issue": profiled_issue(cfg) if engine_id == 2 and not (args.drift or args.replace or args.multi or
                                                                   args.keda or args.hpa_sync not in (0, 60)) else None,
            "totals": {"cost_usd": totals.cost_uphmin / 6e7, "energy_kwh": totals.energy_wmin / 6e4,
                       "gco2_kg": totals.gco2 / 1e3, "slo_minutes": totals.slo_minutes,
                       "launches": totals.launches, "deletions": totals.deletions},
        }
        if cfg == 4:
            out["pareto_frontier_grids"] = frontier[-1] if frontier else None
        if rank == 0:
            cbw = copy_bandwidth(eng)
            out["roofline"]["copy_gbs"] = cbw
            out["roofline"]["copy_kernel"] = "copy16_kernel: 2 GiB dwordx4 nontemporal copy, one element per thread, median of 5 (tools/probe/copyprobe.hip)"
            out["roofline"]["frac_of_copy"] = achieved / cbw
        if rank == 0 and world == 1 and not args.no_cpu:
            out["cpu_baseline"], out["parity"], out["parity_detail"] = cpu_baseline(
                eng, spec, sc, args.cpu_seconds, traj, local_totals)
        elif world > 1 and not args.no_cpu:
            # every rank: an untimed prefix of its own shard against the oracle
            ok, det = rank_parity(eng, spec, sc, traj)
            flags = [None] * world
            dist.all_gather_object(flags, (rank, ok, det))
            if rank == 0:
                out["parity"] = all(f[1] for f in flags)
                out["parity_detail"] = {"per_rank": [f[2] for f in flags],
                                        "rule": "per rank: the first scenarios of its shard, results (and "
                                                "trajectory) bit-exact vs the CPU oracle on the same traces"}
    if rank == 0:
        print(json.dumps(out), flush=True)
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


def general_dims(d, maxn):
    """The general kernel's register layout for d deployments and maxn node
    slots (kernel_dims in csrc/kparams.h)."""
    dmax = 1 if d == 1 else 2 if d <= 2 else 4 if d <= 4 else 8 if d <= 8 else 12 if d <= 12 else 16
    return dmax, 8 if maxn <= 8 and dmax <= 4 else 16


def measured_traffic(cfg, traj, n, T):
    """HBM bytes per launch of the rollout kernel measured by rocprofv3 PMC
    passes of this same command (tools/prof_round.sh; TCC_EA0 read/write
    request counters, see profiles/), or None when no profile matches."""
    import glob

    if (cfg, n, T) != (2, 100_000, 1440):
        return None, None
    name = "config2_traj_summary.json" if traj else "config2_summary_summary.json"
    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "round*", name)))
    if not paths:
        return None, None
    d = json.load(open(paths[-1]))
    return d.get("traffic_bytes"), {"file": os.path.relpath(paths[-1], ROOT), "head": d.get("source_head"),
                                    "how": "rocprofv3 TCC_EA0 request counters, separate --pmc passes "
                                           "(tools/prof_round.sh); copied, not measured in this run"}


def copy_bandwidth(eng, nbytes=1 << 31, reps=5):
    """Measured device copy ceiling (GB/s of read + write): libccka's
    copy16_kernel, a 2 GiB streaming copy with 16 bytes per lane per access
    (dwordx4), timed with HIP events on the engine stream; the practical HBM
    ceiling the rollout's achieved bytes are also compared against (SURVEY.md
    8(d))."""
    gbs = C.c_double()
    fn = eng.lib.ccka_debug_copy_gbs
    fn.argtypes = [C.c_void_p, C.c_int64, C.c_int32, C.POINTER(C.c_double)]
    eng._chk(fn(eng.ctx, nbytes, reps, C.byref(gbs)), "ccka_debug_copy_gbs")
    return gbs.value


def profiled_issue(cfg):
    """Issue-side utilisation of the rollout kernel for this config from the
    committed rocprofv3 PMC pass (tools/prof_issue.sh -> profiles/round*/
    issue_config234.json): VALU / SALU issue fractions of SIMD cycles, mean
    active lanes per VALU instruction, clock. None when no profile exists."""
    import glob

    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "round*", "issue_config234.json")))
    if not paths:
        return None
    j = json.load(open(paths[-1]))
    d = j.get(f"config{cfg}")
    if d:
        d = dict(d, issue_source={"file": os.path.relpath(paths[-1], ROOT), "head": j.get("source_head"),
                                  "how": "rocprofv3 SQ PMC pass (tools/prof_issue.sh); copied, not measured in "
                                         "this run"})
    return d


def host_cpu():
    """Host CPU facts for the baseline: usable cores (affinity), nproc, the
    cgroup CPU quota when one is set, and the /proc/cpuinfo model name."""
    info = {"nproc": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)), "cpu_model": None,
            "cgroup_cpus": None}
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                info["cpu_model"] = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            info["cgroup_cpus"] = int(q) / int(per)
    except (OSError, ValueError):
        pass
    return info


def oracle_native():
    """Build the CPU oracle with -march=native for THIS host (the prebuilt one
    is x86-64-v3 so that it loads on any box); returns (module, march)."""
    import subprocess

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as po

    try:
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "native"], check=True, timeout=180,
                       stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)
        po.use_library(po.NATIVE_LIB)
        return po, "native"
    except Exception as e:  # the portable build still measures the same code
        print(f"bench: -march=native oracle build failed ({e}); using the x86-64-v3 build", file=sys.stderr)
        return po, "x86-64-v3"


def cpu_baseline(eng, spec, sc, target_s, traj, gpu_totals):
    """The CPU oracle (plain C restatement, gcc -O3 -march=native, pthreads
    over contiguous scenario shards, one per usable host core) on the same
    workload: the same global ids and the same device-generated traces (copied
    to the host, untimed). Whole batches up to ~target_s of CPU time (a bounded
    prefix when one batch would take longer); the median run is reported, plus
    a 1-thread figure on a prefix.

    Before timing, one untimed oracle run over the same batch (the whole
    config-2 batch; a 1e5-scenario prefix of larger ones) is compared with the
    GPU rollout field by field, with its trajectory when the rollout wrote one,
    and with the device totals: the returned parity flag."""
    po, march = oracle_native()
    cpu = host_cpu()
    # every core this process may run on: the affinity set, capped by the
    # cgroup CPU quota when one is set (more threads than the quota only
    # time-slice; the nproc-thread figure is reported beside it)
    threads = max(1, cpu["affinity"])
    if cpu["cgroup_cpus"]:
        threads = max(1, min(threads, int(cpu["cgroup_cpus"])))
    load = eng.get_load()
    T = spec.n_steps
    n = min(sc.n, 100_000)

    def inputs(m):
        sub = sc.slice(0, m)
        ld = load if sc.n_traces else np.ascontiguousarray(load[:, :, :m])
        return sub, ld

    # ---- parity at the benchmark size (untimed) ----
    sub, ld = inputs(n)
    ref, ref_tr = po.rollout(spec, sub, ld, traj=traj, threads=threads)
    got = eng.results()
    bad = [k for k in ref if not np.array_equal(got[k][:n], ref[k])]
    checked = ["results"]
    if traj:
        gtr = eng.trajectory()
        if not np.array_equal(gtr[:, :n], ref_tr):
            bad.append("trajectory")
        checked.append("trajectory")
        del gtr, ref_tr
    if n == sc.n:
        want = po.totals(ref, n)
        for f, _ in abi_totals_fields():
            # every total is an exact int64 sum (energy / gCO2 in fixed point) or
            # derived from one: bit-identical whatever the summation order
            if getattr(gpu_totals, f) != getattr(want, f):
                bad.append(f"totals.{f}")
        checked.append("totals")
    parity = not bad
    detail = {"scenarios": n, "of": sc.n, "steps": T, "checked": checked, "mismatched": bad,
              "rule": "per-scenario results and trajectory bit-exact (integers, instance choices, fp64 "
                      "energy/gCO2); totals bit-exact (int64 sums, energy/gCO2 in fixed point)"}

    def run(m, th):
        s2, l2 = inputs(m)
        t0 = time.perf_counter()
        po.rollout(spec, s2, l2, threads=th)
        return time.perf_counter() - t0

    times = [run(n, threads)]
    while sum(times) < target_s and len(times) < 25:
        times.append(run(n, threads))
    times.sort()
    med = times[len(times) // 2]
    n1 = min(sc.n, 8192)
    t1 = run(n1, 1)
    tn = None
    if cpu["nproc"] and cpu["nproc"] != threads:
        tn = min(run(n, cpu["nproc"]) for _ in range(3))
    base = {"value": n * T / med, "unit": "cluster-steps/s", "cores": threads, "kind": "port",
            "sample": f"{n} of {sc.n} scenarios x {T} steps, median of {len(times)} runs "
                      f"({med:.3f} s each) on {threads} threads",
            "value_1thread": n1 * T / t1, "sample_1thread": f"{n1} scenarios x {T} steps, {t1:.2f} s",
            "nproc": cpu["nproc"], "cpu_model": cpu["cpu_model"], "cgroup_cpus": cpu["cgroup_cpus"],
            "value_nproc_threads": None if tn is None else n * T / tn,
            "build": f"gcc -O3 -march={march} -ffp-contract=off"}
    return base, parity, detail


def rank_parity(eng, spec, sc, traj, n=10_000):
    """Untimed check of this rank's shard prefix (global ids first_id ..
    first_id + n) against the CPU oracle on the same device-generated traces:
    every per-scenario result and, in trajectory mode, every record."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as po

    n = min(n, sc.n)
    load = eng.get_load()
    ld = load if sc.n_traces else np.ascontiguousarray(load[:, :, :n])
    ref, ref_tr = po.rollout(spec, sc.slice(0, n), ld, traj=traj, threads=max(1, min(16, os.cpu_count() or 1)))
    got = eng.results()
    bad = [k for k in ref if not np.array_equal(got[k][:n], ref[k])]
    if traj and not np.array_equal(eng.trajectory()[:, :n], ref_tr):
        bad.append("trajectory")
    return not bad, {"first_id": int(sc.first_id), "scenarios": n, "mismatched": bad}


def abi_totals_fields():
    from ccka import abi

    return abi.Totals._fields_


def cpu_baseline_mlp(target_s):
    """PyTorch fp32 on the host cores (the numerics reference of the kernel's
    tests) on a bounded sample of states."""
    import torch

    from ccka import configs

    cpu = host_cpu()
    # the rollout baseline's rule: affinity capped by the cgroup CPU quota
    # (256 threads on a 16-CPU quota only time-slice the GEMMs)
    threads = max(1, cpu["affinity"])
    if cpu["cgroup_cpus"]:
        threads = max(1, min(threads, int(cpu["cgroup_cpus"])))
    torch.set_num_threads(threads)
    ws, bs = configs.mlp_weights(11)
    w = [torch.from_numpy(configs.from_bf16_bits(configs.to_bf16_bits(x))) for x in ws]
    b = [torch.from_numpy(x) for x in bs]
    n = 200_000
    x = torch.randn(n, 64).to(torch.bfloat16).float()

    def run():
        t0 = time.perf_counter()
        h1 = torch.relu(x @ w[0] + b[0]).to(torch.bfloat16).float()
        h2 = torch.relu(h1 @ w[1] + b[1]).to(torch.bfloat16).float()
        _ = h2 @ w[2] + b[2]
        return time.perf_counter() - t0

    times = [run()]
    while sum(times) < target_s and len(times) < 25:
        times.append(run())
    times.sort()
    med = times[len(times) // 2]
    return {"value": n / med, "unit": "cluster-states/s", "cores": threads, "kind": "port",
            "sample": f"{n} states, PyTorch fp32 (bf16-rounded activations), median of {len(times)} runs",
            "nproc": cpu["nproc"], "cpu_model": cpu["cpu_model"], "cgroup_cpus": cpu["cgroup_cpus"]}


if __name__ == "__main__":
    main()
