#!/bin/bash
# Diagnostic PMC passes (SQ issue/wait, caches) on the bench workload; one counter group per run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; mkdir -p gpurun_out/diag
cd /tmp && export TMPDIR=/tmp
rocprofv3 -L > "$R/gpurun_out/diag/counters_list.txt" 2>&1
i=0
while read -r GROUP; do
  [ -z "$GROUP" ] && continue
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $GROUP --output-format csv -d "$R/gpurun_out/diag/p$i" -o run -- \
     python "$R/bench.py" --steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > "$R/gpurun_out/diag/p$i.log" 2>&1; rc=$?
  echo "pass $i ($GROUP) rc=$rc"
  [ $rc -ne 0 ] && { tail -5 "$R/gpurun_out/diag/p$i.log"; exit $rc; }
done <<'GROUPS'
SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_SALU SQ_BUSY_CYCLES
SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE
TCC_HIT_sum TCC_MISS_sum
TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum
GROUPS
exit 0
