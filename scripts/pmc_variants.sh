#!/bin/bash
# One PMC pass (default WRITE_SIZE) per _variants/*.so over a short bench.py run, one frame in flight,
# lockstep pinned: per-kernel counter values land in gpurun_out/pmcv_<variant>/
export RESTIR_TRAVERSAL=${RESTIR_TRAVERSAL:-lockstep}
export RESTIR_RUNAHEAD=${RESTIR_RUNAHEAD:-0}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for so in $R/restir-embree_amd/_variants/${VARIANTS:-*}.so; do
  n=$(basename $so .so)
  RESTIR_LIB=$so timeout -k 10 200 rocprofv3 --pmc ${PMC:-WRITE_SIZE} --output-format csv -d "$R/gpurun_out/pmcv_$n" -o run -- \
     python "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > "$R/gpurun_out/pmcv_$n.log" 2>&1; rc=$?
  echo "pmc $n rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
