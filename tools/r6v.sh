#!/usr/bin/env bash
# round-6 SK variant A/B: tools/r6v.sh "<timing variants>" "<stamp variants>"
cd "$GRAFT_REPO_ROOT" || exit 1
for v in $1; do tools/gpu_step.sh t_$v 120 python -u tools/sk_stats.py --lib $v 100000 1440 || exit $?; done
for v in $2; do tools/gpu_step.sh g_$v 120 python -u tools/sk_stats.py --stamps --lib $v 100000 1440 || exit $?; done
