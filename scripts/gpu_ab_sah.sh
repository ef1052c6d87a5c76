#!/bin/bash
# SAH-optimal wide collapse: -m gpu suite on sah8, then C3 and C2 A/B vs the greedy-collapse library, walk statistics
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
BENCH_ARGS="--scene C3" bash scripts/ab_lib.sh || exit $?
REPS=1 AB="base|base| sah8|sah8|" BENCH_ARGS="--scene C2" bash scripts/ab_r03.sh || exit $?
timeout -k 10 300 python -u scripts/bvh_stats.py > gpurun_out/bvh_stats_sah.txt 2>&1 || exit 1
grep "8-wide" gpurun_out/bvh_stats_sah.txt
