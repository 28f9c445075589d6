#!/usr/bin/env bash
# Run ONE GPU step under its own time limit; log to gpurun_out/<name>.log.
# Exit status 0/1 (success / ordinary test failure) lets the caller continue;
# anything else (abort, segfault, timeout) must end the GPU call.
# usage: tools/gpu_step.sh <name> <seconds> <command...>
name="$1"; secs="$2"; shift 2
mkdir -p gpurun_out
echo "[gpu_step] $name: $*" | tee -a gpurun_out/steps.log
timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
rc=$?
echo "[gpu_step] $name rc=$rc" | tee -a gpurun_out/steps.log
tail -n 5 "gpurun_out/$name.log"
exit $rc
