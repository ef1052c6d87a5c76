#!/bin/bash
# Round-2 profiles on the GPU box: rocprofv3 kernel-trace stats of the bench (C2 headline, C3) and the
# PMC passes (one counter group per run, --pmc + kernel trace only) that profiles/r02_pmc_<cfg>.json
# summarises.  One frame in flight (RESTIR_RUNAHEAD=0) and a pinned traversal kind for the PMC runs so
# counters are per dispatch of one kind.  Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for cfg in ${CFGS:-C2 C3}; do
  trav=lockstep; [ $cfg = C3 ] && trav=lane
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$cfg" -o run -- \
     python3 "$R/bench.py" --scene $cfg --steps 10 --warmup 2 --no-cpu-baseline --no-extras > "$R/gpurun_out/prof_$cfg.log" 2>&1 \
     || { echo "rocprof $cfg failed"; tail -5 "$R/gpurun_out/prof_$cfg.log"; exit 1; }
  echo "stats $cfg ok"
  # every launch with one frame in flight: the kernel averages bench.py's kernel_roofline.kernel_ms uses
  RESTIR_RUNAHEAD=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof0_$cfg" -o run -- \
     python3 "$R/bench.py" --scene $cfg --steps 10 --warmup 2 --no-cpu-baseline --no-extras > "$R/gpurun_out/prof0_$cfg.json" 2> "$R/gpurun_out/prof0_$cfg.err" \
     || { echo "rocprof runahead-0 $cfg failed"; tail -5 "$R/gpurun_out/prof0_$cfg.err"; exit 1; }
  echo "stats (run-ahead 0) $cfg ok"
  [ -n "$NO_PMC" ] && continue
  for C in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY"; do
    D=${C%% *}
    RESTIR_RUNAHEAD=0 RESTIR_TRAVERSAL=$trav timeout -k 10 300 rocprofv3 --pmc $C --output-format csv \
       -d "$R/gpurun_out/pmc_${cfg}_$D" -o run -- \
       python3 "$R/bench.py" --scene $cfg --steps 3 --warmup 1 --no-cpu-baseline --no-extras > "$R/gpurun_out/pmc_${cfg}_$D.log" 2>&1 \
       || { echo "pmc $cfg $C failed"; tail -5 "$R/gpurun_out/pmc_${cfg}_$D.log"; exit 1; }
    echo "pmc $cfg $D ok"
  done
done
