#!/bin/bash
# Round-5 session X: piece-major wide-node copy for the per-lane walks (RS_WIDE_SOA) -- parity / wide-tree
# tests on the default (piece-major) build, then C3 and C2 frame rates against the record-major build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_wide.py \
  > gpurun_out/x_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|assert|Error" gpurun_out/x_tests.log | head; tail -30 gpurun_out/x_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/x_tests.log | tail -2
AB_TESTS=tests/test_gpu_wide.py BENCH_ARGS="--scene C3" STEPS=15 REPS=2 bash scripts/ab_r05.sh || exit 1
BENCH_ARGS="--scene C2" STEPS=60 REPS=2 AB_TESTS=tests/test_gpu_wide.py bash scripts/ab_r05.sh || exit 1
echo "session x done"
