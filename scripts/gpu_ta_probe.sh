#!/bin/bash
# Vector-memory pipeline counters (TA/TD/TCP + SQ VMEM) of the C3 initial pass for each _variants/*.so:
# one --pmc pass per library, one frame in flight, per-lane walks pinned.  Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
C="SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD SQ_VMEM_TA_ADDR_FIFO_FULL SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TD_TD_BUSY TD_TC_STALL GRBM_GUI_ACTIVE GRBM_COUNT TCP_TOTAL_CACHE_ACCESSES TCP_TCC_READ_REQ TCP_PENDING_STALL_CYCLES TCP_TCP_TA_DATA_STALL_CYCLES"
for so in $R/restir-embree_amd/_variants/${VARIANTS:-*}.so; do
  n=$(basename $so .so)
  RESTIR_LIB=$so RESTIR_RUNAHEAD=0 RESTIR_TRAVERSAL=${TRAV:-lane} timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv \
     -d "$R/gpurun_out/ta_$n" -o run -- python3 "$R/bench.py" --scene ${SCENE:-C3} --steps 3 --warmup 1 --no-cpu-baseline --no-extras \
     > "$R/gpurun_out/ta_$n.log" 2>&1 || { echo "pmc $n failed"; tail -5 "$R/gpurun_out/ta_$n.log"; exit 1; }
  echo "pmc $n ok"
done
