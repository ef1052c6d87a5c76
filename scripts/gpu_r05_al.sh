#!/bin/bash
# Round-5 session AL: a third geometry copy for pipelined updates (RS_GEO_COPIES=3; lib_copies2 = the round-4
# pair) -- every -m gpu test on the default build, then C5 both ways, two interleaved rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/al_tests.log 2>&1 \
  || { echo "tests failed"; grep -E "FAILED|assert|Error" gpurun_out/al_tests.log | head; tail -5 gpurun_out/al_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/al_tests.log | tail -1
AB_TESTS="tests/test_gpu_wide.py" BENCH_ARGS="--scene C5" STEPS=240 REPS=2 bash scripts/ab_r05.sh || exit 1
echo "session al done"
