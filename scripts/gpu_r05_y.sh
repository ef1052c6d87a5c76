#!/bin/bash
# Round-5 session Y: the sorted initial pass keeping phase A's candidate weights for phase C (RS_SORT_STORE_W)
# instead of drawing every candidate again -- parity tests on the default build, then C3 frame rates against
# the recompute build (lib_recompute), two interleaved rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_mgpu.py \
  > gpurun_out/y_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|assert|Error" gpurun_out/y_tests.log | head; tail -30 gpurun_out/y_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/y_tests.log | tail -2
AB_TESTS=tests/test_gpu_wide.py BENCH_ARGS="--scene C3" STEPS=15 REPS=2 bash scripts/ab_r05.sh || exit 1
echo "session y done"
