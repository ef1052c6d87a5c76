#!/bin/bash
# Round-5 session AM: C2's initial pass with the pixel's surface point parked in LDS and le re-read from the G-buffer
# (RS_INIT_PARK; lib_nopark = without) -- parity tests on the default build, C2 both ways, three interleaved rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_mgpu.py \
  "tests/test_gpu_workloads.py::test_c2_full_1080p" > gpurun_out/am_tests.log 2>&1 \
  || { echo "tests failed"; grep -E "FAILED|assert|Error" gpurun_out/am_tests.log | head; exit 1; }
grep -E "passed|failed" gpurun_out/am_tests.log | tail -1
AB_TESTS="tests/test_gpu_wide.py" BENCH_ARGS="--scene C2" STEPS=60 REPS=3 bash scripts/ab_r05.sh || exit 1
echo "session am done"
