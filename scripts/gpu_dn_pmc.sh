#!/bin/bash
# Denoiser PMC passes (one counter group per run, kernel-trace only besides --pmc) over scripts/denoise_probe.py
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
i=0
for C in "FETCH_SIZE" "WRITE_SIZE" \
         "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS" \
         "GRBM_GUI_ACTIVE TA_TA_BUSY TD_TD_BUSY TCP_TOTAL_CACHE_ACCESSES TCP_TCC_READ_REQ SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_ACTIVE_INST_VALU"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d "$R/gpurun_out/dnpmc_$i" -o run -- \
     python3 "$R/scripts/denoise_probe.py" --iters 3 > "$R/gpurun_out/dnpmc_$i.log" 2>&1; rc=$?
  echo "pmc pass $i ($C) rc=$rc"
  [ $rc -ne 0 ] && { tail -5 "$R/gpurun_out/dnpmc_$i.log"; exit $rc; }
done
exit 0
