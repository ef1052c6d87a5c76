#!/bin/bash
# PMC HBM-traffic passes (one counter group per run, kernel-trace only besides --pmc).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d "$R/gpurun_out/pmc_$C" -o run -- \
     python "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > "$R/gpurun_out/pmc_$C.log" 2>&1; rc=$?
  echo "pmc $C rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
