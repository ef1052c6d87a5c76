#!/bin/bash
# Round-5 session AF: the refits' leaf loads issued before their stores (refit_leaf / wide_leaf_slots; lib_head = without) -- the
# refit and moving-geometry tests on the default build, then C5 frame rates both ways, two interleaved rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_wide.py tests/test_gpu_parity.py "tests/test_gpu_workloads.py::test_c5_moving_lights_sequence" tests/test_gpu_mgpu.py > gpurun_out/af_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|assert|Error" gpurun_out/af_tests.log | head; exit 1; }
grep -E "passed|failed" gpurun_out/af_tests.log | tail -1
AB_TESTS="tests/test_gpu_wide.py" BENCH_ARGS="--scene C5" STEPS=240 REPS=2 bash scripts/ab_r05.sh || exit 1
echo "session af done"
