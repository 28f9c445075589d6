cd "$GRAFT_REPO_ROOT" || exit 1
tools/gpu_step.sh g_sum 120 python -u tools/sk_stats.py --summary --stamps --lib skrg 100000 1440 || exit $?
