#!/bin/bash
# Round-5 A/B of prebuilt libraries restir-embree_amd/_ab/lib_*.so: the selected -m gpu tests (AB_TESTS, default the
# parity suite) against each non-base one, then bench.py (BENCH_ARGS, e.g. --scene C3) for each, REPS times
# interleaved, one line per run with the per-pass times of one frame in flight.  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for so in restir-embree_amd/_ab/*.so; do
  n=$(basename $so .so); [ "$n" = lib_base ] && continue
  RESTIR_LIB=$PWD/$so timeout -k 10 400 python -u -m pytest ${AB_TESTS:-tests/test_gpu_parity.py} -m gpu -x -q --timeout 200 \
    --timeout-method thread > gpurun_out/ab_pytest_$n.log 2>&1 || { echo "$n: gpu tests failed"; tail -30 gpurun_out/ab_pytest_$n.log; exit 1; }
  echo "$n: $(tail -1 gpurun_out/ab_pytest_$n.log)"
done
for rep in $(seq ${REPS:-2}); do
for so in restir-embree_amd/_ab/*.so; do
  n=$(basename $so .so)
  RESTIR_LIB=$PWD/$so timeout -k 10 240 python bench.py --steps ${STEPS:-30} --warmup 5 --no-cpu-baseline --no-extras ${BENCH_ARGS} > gpurun_out/ab_$n.log 2>&1; rc=$?
  [ $rc -ne 0 ] && { echo "$n rc=$rc"; tail -3 gpurun_out/ab_$n.log; exit $rc; }
  python - "$n" gpurun_out/ab_$n.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
kr = d.get('kernel_roofline', {})
print(f"{sys.argv[1]:>14s} fps={d['value']:8.2f} {kr.get('kernel', '')}_ms={kr.get('kernel_ms', 0):.3f} " +
      " ".join(f"{k}={v:.3f}" for k, v in d.get('pass_ms_one_frame_in_flight', {}).items() if v > 0.01), flush=True)
PY
done; done
