#!/bin/bash
# SQ instruction-mix counters for k_gbuffer_initial under the parameter points of
# scripts/initial_breakdown.py (CFGS, default all 8); one counter group per rocprofv3 run
# (PMC_SETS: newline-separated groups).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; OUT=$R/gpurun_out/${DIAG_OUT:-diag2}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
SETS="${PMC_SETS:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY}"
for cfg in ${CFGS:-0 1 2 3 4 5 6 7}; do
i=0
while read -r SET; do
  [ -z "$SET" ] && continue
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $SET --output-format csv -d "$OUT/c${cfg}_p$i" -o run -- \
     python "$R/scripts/initial_breakdown.py" --frames 2 --only $cfg > "$OUT/c${cfg}_p$i.log" 2>&1; rc=$?
  echo "cfg $cfg pass $i rc=$rc"
  [ $rc -ne 0 ] && { tail -5 "$OUT/c${cfg}_p$i.log"; exit $rc; }
done <<< "$SETS"
done
exit 0
