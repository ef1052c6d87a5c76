#!/bin/bash
# Round-5 session AE: refit / update workgroups of 256 threads against 128 and 64 (lib_b128, lib_b64) -- the
# refit and moving-geometry tests on the default build, then C5 frame rates both ways, two interleaved rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
AB_TESTS="tests/test_gpu_wide.py tests/test_gpu_parity.py" BENCH_ARGS="--scene C5" STEPS=240 REPS=2 bash scripts/ab_r05.sh || exit 1
echo "session ae done"
