#!/bin/bash
# One GPU-box session (gpurun): the steps named on the command line, in order, stopping at the first failure or
# fatal exit (every GPU step under its own time limit).  Replaces the per-session scripts of rounds 3-5 (their
# outcomes are in profiles/r05_sessions.txt and git history).
#
#   bash scripts/gpu_session.sh tests smoke bench prof pmc ab band
#
#   tests   -m gpu tests -> gpurun_out/pytest_gpu.log.  TESTS (default: tests), PYTEST_ARGS, KEEP_GOING=1 (no -x)
#   smoke   __graft_entry__.smoke() -> gpurun_out/smoke.log
#   bench   bench.py $BENCH_ARGS -> gpurun_out/bench${TAG}.json (+ .err)
#   prof    rocprofv3 --kernel-trace --stats of bench.py per config (CFGS, default "C2 C3"), frames in flight and
#           one frame in flight (RESTIR_RUNAHEAD=0) -> gpurun_out/prof{,0}_<cfg>/
#   pmc     one rocprofv3 --pmc pass per counter group per config (one frame in flight) -> gpurun_out/pmc_<cfg>$PMC_TAG_<group>/
#           (scripts/pmc_summary.py turns them into profiles/rNN_pmc_<cfg>$PMC_TAG.json); PMC_ENV: extra VAR=value settings
#   ab      A/B of prebuilt libraries restir-embree_amd/_ab/lib_*.so: AB_TESTS against each non-base one, then
#           bench.py (--steps STEPS, BENCH_ARGS) for each, REPS times interleaved
#   abenv   bench.py (--steps STEPS, BENCH_ARGS) under each environment of ENVS ("A=1 B=2;C=3;" -- ';'-separated
#           sets, an empty set = the defaults), REPS times interleaved
#   band    scripts/band_probe.py $BAND_ARGS -> gpurun_out/band${TAG}.txt
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out

step_tests() {
  local x="-x"; [ -n "$KEEP_GOING" ] && x=""
  timeout -k 10 ${TESTS_LIMIT:-1000} python -u -m pytest ${TESTS:-tests} -m gpu $x -v -s -rf --timeout 400 \
      --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1; local rc=$?
  echo "tests rc=$rc"; grep -E "passed|failed|error" gpurun_out/pytest_gpu.log | tail -3
  [ $rc -ne 0 ] && { grep -E "^FAILED|Error|assert " gpurun_out/pytest_gpu.log | head -20; return $rc; }
  return 0
}
step_smoke() {
  timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; local rc=$?
  echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log
  return $rc
}
step_bench() {
  timeout -k 10 ${BENCH_LIMIT:-900} python -u bench.py ${BENCH_ARGS} > gpurun_out/bench${TAG}.json 2> gpurun_out/bench${TAG}.err
  local rc=$?
  echo "bench rc=$rc"; tail -3 gpurun_out/bench${TAG}.err; head -c 600 gpurun_out/bench${TAG}.json; echo
  return $rc
}
step_prof() {
  ( cd /tmp && export TMPDIR=/tmp
    for cfg in ${CFGS:-C2 C3}; do
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$cfg" -o run -- \
        python3 "$R/bench.py" --scene $cfg --steps ${PROF_STEPS:-10} --warmup 2 --no-cpu-baseline --no-extras \
        > "$R/gpurun_out/prof_$cfg.json" 2> "$R/gpurun_out/prof_$cfg.err" || { echo "rocprof $cfg failed"; tail -5 "$R/gpurun_out/prof_$cfg.err"; exit 1; }
      echo "prof $cfg ok"
      RESTIR_RUNAHEAD=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof0_$cfg" -o run -- \
        python3 "$R/bench.py" --scene $cfg --steps ${PROF_STEPS:-10} --warmup 2 --no-cpu-baseline --no-extras \
        > "$R/gpurun_out/prof0_$cfg.json" 2> "$R/gpurun_out/prof0_$cfg.err" || { echo "rocprof run-ahead 0 $cfg failed"; tail -5 "$R/gpurun_out/prof0_$cfg.err"; exit 1; }
      echo "prof (run-ahead 0) $cfg ok"
    done )
}
step_pmc() {
  local TA="SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU SQ_WAVES TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TD_TD_BUSY TD_TC_STALL GRBM_GUI_ACTIVE GRBM_COUNT TCP_TOTAL_CACHE_ACCESSES TCP_TCC_READ_REQ TCP_PENDING_STALL_CYCLES TCP_TCP_TA_DATA_STALL_CYCLES"
  ( cd /tmp && export TMPDIR=/tmp
    [ -n "$PMC_ENV" ] && export $PMC_ENV
    for cfg in ${CFGS:-C2 C3}; do
      local trav=lockstep; [ $cfg = C3 ] && trav=lane
      for C in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY" "$TA"; do
        local D=${C%% *}
        RESTIR_RUNAHEAD=0 RESTIR_TRAVERSAL=$trav timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv \
          -d "$R/gpurun_out/pmc_${cfg}${PMC_TAG}_$D" -o run -- \
          python3 "$R/bench.py" --scene $cfg --steps 3 --warmup 1 --no-cpu-baseline --no-extras > "$R/gpurun_out/pmc_${cfg}${PMC_TAG}_$D.log" 2>&1 \
          || { echo "pmc $cfg $D failed"; tail -5 "$R/gpurun_out/pmc_${cfg}${PMC_TAG}_$D.log"; exit 1; }
        echo "pmc $cfg $D ok"
      done
    done )
}
step_ab() {
  for so in restir-embree_amd/_ab/*.so; do
    local n=$(basename $so .so); [ "$n" = lib_base ] && continue
    [ -z "$AB_TESTS" ] && continue
    RESTIR_LIB=$PWD/$so timeout -k 10 400 python -u -m pytest $AB_TESTS -m gpu -x -q --timeout 200 \
      --timeout-method thread > gpurun_out/ab_pytest_$n.log 2>&1 || { echo "$n: gpu tests failed"; tail -30 gpurun_out/ab_pytest_$n.log; return 1; }
    echo "$n: $(tail -1 gpurun_out/ab_pytest_$n.log)"
  done
  for rep in $(seq ${REPS:-2}); do
    for so in restir-embree_amd/_ab/*.so; do
      local n=$(basename $so .so)
      RESTIR_LIB=$PWD/$so timeout -k 10 240 python bench.py --steps ${STEPS:-30} --warmup 5 --no-cpu-baseline --no-extras ${BENCH_ARGS} \
        > gpurun_out/ab_$n.log 2>&1; local rc=$?
      [ $rc -ne 0 ] && { echo "$n rc=$rc"; tail -3 gpurun_out/ab_$n.log; return $rc; }
      python3 - "$n" gpurun_out/ab_$n.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
kr = d.get('kernel_roofline', {})
print(f"{sys.argv[1]:>14s} fps={d['value']:8.2f} {kr.get('kernel', '')}_ms={kr.get('kernel_ms', 0):.3f} " +
      " ".join(f"{k}={v:.3f}" for k, v in d.get('pass_ms_one_frame_in_flight', {}).items() if v > 0.01), flush=True)
PY
    done
  done
}
step_abenv() {
  local IFS_OLD="$IFS"
  for rep in $(seq ${REPS:-2}); do
    IFS=';'; local sets=($ENVS); IFS="$IFS_OLD"
    for e in "${sets[@]}"; do
      local tag=$(echo "${e:-default}" | tr ' =/' '_-_' | cut -c1-80)
      env $e timeout -k 10 240 python bench.py --steps ${STEPS:-30} --warmup 5 --no-cpu-baseline --no-extras ${BENCH_ARGS} \
        > gpurun_out/abenv_$tag.log 2>&1; local rc=$?
      [ $rc -ne 0 ] && { echo "$tag rc=$rc"; tail -3 gpurun_out/abenv_$tag.log; return $rc; }
      python3 - "$tag" gpurun_out/abenv_$tag.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
kr = d.get('kernel_roofline', {})
print(f"{sys.argv[1]:>40s} fps={d['value']:8.2f} {kr.get('kernel', '')}_ms={kr.get('kernel_ms', 0):.3f}", flush=True)
PY
    done
  done
}
step_band() {
  timeout -k 10 ${BAND_LIMIT:-600} python3 -u scripts/band_probe.py ${BAND_ARGS} > gpurun_out/band${TAG}.txt 2>&1; local rc=$?
  echo "band rc=$rc"; tail -${BAND_TAIL:-12} gpurun_out/band${TAG}.txt
  return $rc
}

for s in "$@"; do
  "step_$s" || { echo "session: step $s failed"; exit 1; }
done
echo "session done: $*"
