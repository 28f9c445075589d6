#!/usr/bin/env bash
# the skewed kernel's time against the scenario count: one round of waves (65,536 = 1,024 SIMDs x 64 lanes)
# against 1e5 (1,563 waves: two rounds) -- the gain a lane-refill schedule could take
cd "$GRAFT_REPO_ROOT" || exit 1
for n in 16384 32768 65536 100000 131072; do
  tools/gpu_step.sh n$n 200 python -u tools/sk_stats.py --lib main $n 1440 || exit $?
done
