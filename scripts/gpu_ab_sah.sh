#!/bin/bash
# wide-tree variants: -m gpu suite for each non-base library, C3 A/B, C2 A/B, walk statistics of the default library
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
BENCH_ARGS="--scene C3" bash scripts/ab_lib.sh || exit $?
REPS=1 AB="${AB_C2:-base|base| sah8|sah8|}" BENCH_ARGS="--scene C2" bash scripts/ab_r03.sh || exit $?
timeout -k 10 300 python -u scripts/bvh_stats.py > gpurun_out/bvh_stats_sah.txt 2>&1 || exit 1
grep "8-wide" gpurun_out/bvh_stats_sah.txt
