#!/bin/bash
# Round-5 session AB: the sorted initial pass's phase A with the next candidate's light pick in flight (RS_SORT_PICK_AHEAD)
# -- parity tests on the default build, then C3 and C4-on-one-GPU frame rates against
# the build without it (lib_noahead), two interleaved rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_mgpu.py \
  > gpurun_out/ab_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|assert|Error" gpurun_out/ab_tests.log | head; tail -30 gpurun_out/ab_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/ab_tests.log | tail -2
AB_TESTS=tests/test_gpu_wide.py BENCH_ARGS="--scene C3" STEPS=15 REPS=2 bash scripts/ab_r05.sh || exit 1
BENCH_ARGS="--scene C3 --width 3840 --height 2160" STEPS=6 REPS=1 AB_TESTS=tests/test_gpu_wide.py bash scripts/ab_r05.sh || exit 1
echo "session ab done"
