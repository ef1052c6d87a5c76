#!/bin/bash
# Round-3 GPU session: parity tests, smoke, default bench line; stops at the first failure or fatal exit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; *) [ "$1" -gt 128 ] && return 0; return 1;; esac; }
{ rocminfo 2>/dev/null | grep -m2 -E "Marketing Name|gfx950"; nproc; lscpu | grep -m1 "Model name"; \
  python -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'OMP', os.environ.get('OMP_NUM_THREADS'))"; \
  cat /sys/fs/cgroup/cpu.max 2>/dev/null; } > gpurun_out/device.txt
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  echo "pytest_gpu rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
  [ $rc -ne 0 ] && exit $rc
  timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
  echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
  [ $rc -ne 0 ] && exit $rc
fi
if [ -z "$NO_BENCH" ]; then
  timeout -k 10 900 python -u bench.py ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?
  echo "bench rc=$rc"; tail -3 gpurun_out/bench.err; head -c 600 gpurun_out/bench.json
  [ $rc -ne 0 ] && exit $rc
fi
exit 0
