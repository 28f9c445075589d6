#!/usr/bin/env bash
# The profiles beside tools/refresh_d1.sh's single-deployment set (one GPU call):
# the read-traffic split of config 2 (L2 hit / miss counters with the shipped
# wave-tiled trace and with the [T][N] trace, FETCH_SIZE and bench line of the
# [T][N] trace), the upstream-defaults line, and the config-5 lines (MLP, the
# closed loop at 1e7 with its kernel trace, the policy gradient with its kernel
# trace). Output: gpurun_out/r2b/ (tools/save_profiles.sh copies it).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/r2b; mkdir -p $out/tcc
tools/gpu_step.sh pgt 300 python -u -m pytest tests/test_gpu_pg.py tests/test_policy_rollout.py -m gpu -x -q \
  --timeout 120 --timeout-method thread || exit $?
pmc() {  # <name> <counters> [bench args]: one PMC pass over one config-2 rollout
  local name="$1" set="$2"; shift 2
  timeout -s KILL 120 rocprofv3 --pmc $set -d "$out/tcc/$name" -o run --output-format csv -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu "$@" > "$out/tcc/$name.log" 2>&1
}
pmc hit_tiled "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE" || exit $?
pmc hit_flat "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE" --trace-flat || exit $?
pmc rd_flat "TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B GRBM_GUI_ACTIVE" --trace-flat || exit $?
pmc fetch_flat "FETCH_SIZE" --trace-flat || exit $?
pmc rd_summary "TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B GRBM_GUI_ACTIVE" --mode summary || exit $?
tools/gpu_step.sh b2f 300 python bench.py --config 2 --no-cpu --trace-flat || exit $?
grep '^{' gpurun_out/b2f.log | tail -1 > $out/bench_config2_trace_flat.json || exit 1
tools/gpu_step.sh b2all 300 python bench.py --config 2 --hpa-sync 15 --drift --replace --multi --no-cpu || exit $?
grep '^{' gpurun_out/b2all.log | tail -1 > $out/bench_config2_sync15_drift_replace_multi.json || exit 1
tools/gpu_step.sh b5 300 python bench.py --config 5 || exit $?
grep '^{' gpurun_out/b5.log | tail -1 > $out/bench_config5.json || exit 1
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d "$out/c5p7" -o run --output-format csv -- \
  python3 bench.py --config 5 --mode policy --n 10000000 --steps 2 --warmup 1 --no-cpu > "$out/c5p7.log" 2>&1 || exit $?
grep '^{' "$out/c5p7.log" | tail -1 > $out/bench_config5_policy_1e7_under_rocprof.json || exit 1
tools/gpu_step.sh b5p7 300 python bench.py --config 5 --mode policy --n 10000000 --steps 3 --warmup 1 || exit $?
grep '^{' gpurun_out/b5p7.log | tail -1 > $out/bench_config5_policy_1e7.json || exit 1
tools/gpu_step.sh b5p 300 python bench.py --config 5 --mode policy || exit $?
grep '^{' gpurun_out/b5p.log | tail -1 > $out/bench_config5_policy.json || exit 1
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d "$out/c5g" -o run --output-format csv -- \
  python3 bench.py --config 5 --mode grad --steps 3 --warmup 1 --no-cpu > "$out/c5g.log" 2>&1 || exit $?
tools/gpu_step.sh b5g 300 python bench.py --config 5 --mode grad || exit $?
grep '^{' gpurun_out/b5g.log | tail -1 > $out/bench_config5_grad.json || exit 1
tools/gpu_step.sh b5g7 400 python bench.py --config 5 --mode grad --n 10000000 --steps 2 --warmup 1 || exit $?
grep '^{' gpurun_out/b5g7.log | tail -1 > $out/bench_config5_grad_1e7.json || exit 1
tools/gpu_step.sh lsplit 300 python tools/loop_split.py 10000000 60 || exit $?
cp gpurun_out/lsplit.log $out/loop_split_1e7.txt
echo extra-done
