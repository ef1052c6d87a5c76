#!/bin/bash
# One GPU-box session: parity tests, smoke, short bench, rocprofv3 kernel stats.
# Stops at the first GPU fault / abort / timeout (exit 124/134/137/139); continues past plain test failures.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
STEPS=${STEPS:-10}
fatal() { case "$1" in 124|134|137|139) return 0;; *) [ "$1" -gt 128 ] && return 0; return 1;; esac; }
rocminfo 2>/dev/null | grep -m2 -E "Marketing Name|gfx950" > gpurun_out/device.txt; nproc >> gpurun_out/device.txt
lscpu | grep -m1 "Model name" >> gpurun_out/device.txt
timeout -k 10 600 python -m pytest tests -m gpu -q -rf ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest_gpu rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
if fatal $rc; then echo "fatal pytest rc"; exit $rc; fi
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps $STEPS --warmup 2 ${BENCH_ARGS} > gpurun_out/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -2 gpurun_out/bench.log
if [ $rc -ne 0 ]; then exit $rc; fi
if [ -n "$PROFILE" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run -- \
     python "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 1 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1; rc=$?
  echo "rocprof rc=$rc"; tail -2 "$GRAFT_REPO_ROOT/gpurun_out/prof.log"
fi
exit 0
