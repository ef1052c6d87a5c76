#!/bin/bash
# PMC HBM-traffic passes (one counter group per run, kernel-trace only besides --pmc).  The traversal
# kind is pinned (RESTIR_TRAVERSAL, default lockstep) so AUTO's tuning frames do not mix both kinds.
export RESTIR_TRAVERSAL=${RESTIR_TRAVERSAL:-lockstep}
# one frame in flight: counters are read per dispatch, and overlapping frames would add their traffic
export RESTIR_RUNAHEAD=${RESTIR_RUNAHEAD:-0}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY"; do
  D=${C%% *}
  timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d "$R/gpurun_out/pmc_$D" -o run -- \
     python "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > "$R/gpurun_out/pmc_$D.log" 2>&1; rc=$?
  echo "pmc $C rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
