#!/bin/bash
# Round-4 profiles on the GPU box (after scripts/gpu_r04.sh): BVH walk statistics, rocprofv3 kernel-trace
# stats of C2 and C3 (frames in flight, and one frame in flight = the kernel averages bench.py's
# kernel_roofline uses), then one --pmc pass per counter group with one frame in flight and the scene's
# traversal kind pinned: FETCH_SIZE, WRITE_SIZE, SQ_* (issue / wait) and the vector-memory pipeline group
# (TA/TD/TCP busy and requests).  scripts/pmc_summary.py turns the passes into profiles/r04_pmc_<cfg>.json.
# Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out
timeout -k 10 300 python3 scripts/bvh_stats.py > gpurun_out/bvh_stats.txt 2>&1 || { echo "bvh_stats failed"; tail -5 gpurun_out/bvh_stats.txt; exit 1; }
echo "bvh_stats ok"
cd /tmp && export TMPDIR=/tmp
TA="SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU SQ_WAVES TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TD_TD_BUSY TD_TC_STALL GRBM_GUI_ACTIVE GRBM_COUNT TCP_TOTAL_CACHE_ACCESSES TCP_TCC_READ_REQ TCP_PENDING_STALL_CYCLES TCP_TCP_TA_DATA_STALL_CYCLES"
for cfg in ${CFGS:-C2 C3}; do
  trav=lockstep; [ $cfg = C3 ] && trav=lane
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$cfg" -o run -- \
     python3 "$R/bench.py" --scene $cfg --steps 10 --warmup 2 --no-cpu-baseline --no-extras > "$R/gpurun_out/prof_$cfg.json" 2> "$R/gpurun_out/prof_$cfg.err" \
     || { echo "rocprof $cfg failed"; tail -5 "$R/gpurun_out/prof_$cfg.err"; exit 1; }
  echo "stats $cfg ok"
  RESTIR_RUNAHEAD=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof0_$cfg" -o run -- \
     python3 "$R/bench.py" --scene $cfg --steps 10 --warmup 2 --no-cpu-baseline --no-extras > "$R/gpurun_out/prof0_$cfg.json" 2> "$R/gpurun_out/prof0_$cfg.err" \
     || { echo "rocprof runahead-0 $cfg failed"; tail -5 "$R/gpurun_out/prof0_$cfg.err"; exit 1; }
  echo "stats (run-ahead 0) $cfg ok"
  [ -n "$NO_PMC" ] && continue
  for C in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY" "$TA"; do
    D=${C%% *}
    RESTIR_RUNAHEAD=0 RESTIR_TRAVERSAL=$trav timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv \
       -d "$R/gpurun_out/pmc_${cfg}_$D" -o run -- \
       python3 "$R/bench.py" --scene $cfg --steps 3 --warmup 1 --no-cpu-baseline --no-extras > "$R/gpurun_out/pmc_${cfg}_$D.log" 2>&1 \
       || { echo "pmc $cfg $D failed"; tail -5 "$R/gpurun_out/pmc_${cfg}_$D.log"; exit 1; }
    echo "pmc $cfg $D ok"
  done
done
