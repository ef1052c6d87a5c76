#!/bin/bash
# Round-4 GPU session: selected / all GPU tests, smoke, bench; stops at the first failure or fatal exit.
#   TESTS="tests/test_gpu_wide.py ..."  (default: every -m gpu test), NO_TESTS=1, NO_SMOKE=1, NO_BENCH=1,
#   BENCH_ARGS="--scene C3 --no-cpu-baseline --no-extras"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v -s -rf --timeout 300 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  echo "pytest_gpu rc=$rc"; grep -E "passed|failed|error" gpurun_out/pytest_gpu.log | tail -3
  [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
fi
if [ -z "$NO_SMOKE" ]; then
  timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
  echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log
  [ $rc -ne 0 ] && exit $rc
fi
if [ -z "$NO_BENCH" ]; then
  timeout -k 10 900 python -u bench.py ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?
  echo "bench rc=$rc"; tail -3 gpurun_out/bench.err; head -c 400 gpurun_out/bench.json
  [ $rc -ne 0 ] && exit $rc
fi
exit 0
