#!/bin/bash
# SQ instruction-mix counters for k_gbuffer_initial under two parameter points of
# scripts/initial_breakdown.py (0 = metric, 7 = G-buffer + 1 sample); one counter group per run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; mkdir -p gpurun_out/diag2
cd /tmp && export TMPDIR=/tmp
for cfg in 0 7; do
i=0
while read -r GROUP; do
  [ -z "$GROUP" ] && continue
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $GROUP --output-format csv -d "$R/gpurun_out/diag2/c${cfg}_p$i" -o run -- \
     python "$R/scripts/initial_breakdown.py" --frames 2 --only $cfg > "$R/gpurun_out/diag2/c${cfg}_p$i.log" 2>&1; rc=$?
  echo "cfg $cfg pass $i ($GROUP) rc=$rc"
  [ $rc -ne 0 ] && { tail -5 "$R/gpurun_out/diag2/c${cfg}_p$i.log"; exit $rc; }
done <<'GROUPS'
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAVE_CYCLES
SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_FLAT SQ_INSTS_LDS SQ_WAIT_ANY GRBM_GUI_ACTIVE
GROUPS
done
exit 0
