#!/bin/bash
# A/B of prebuilt libraries in restir-embree_amd/_ab/*.so: the -m gpu suite against each non-base one
# (RESTIR_LIB override), then bench.py on BENCH_ARGS (e.g. --scene C3) for each, twice, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for so in restir-embree_amd/_ab/*.so; do
  n=$(basename $so .so); [ "$n" = base ] && continue
  RESTIR_LIB=$PWD/$so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/ab_pytest_$n.log 2>&1 || { echo "$n: gpu tests failed"; tail -30 gpurun_out/ab_pytest_$n.log; exit 1; }
  echo "$n: $(tail -1 gpurun_out/ab_pytest_$n.log)"
done
for rep in 1 2; do
for so in restir-embree_amd/_ab/*.so; do
  n=$(basename $so .so)
  RESTIR_LIB=$PWD/$so timeout -k 10 180 python bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --no-extras ${BENCH_ARGS} > gpurun_out/ab_$n.log 2>&1; rc=$?
  [ $rc -ne 0 ] && { echo "$n rc=$rc"; tail -3 gpurun_out/ab_$n.log; exit $rc; }
  python - "$n" gpurun_out/ab_$n.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(f"{sys.argv[1]:>14s} fps={d['value']:8.2f} Mrays/s={d['mrays_per_s']:9.1f} " + " ".join(f"{k}={v:.3f}" for k, v in d['pass_ms_one_frame_in_flight'].items() if v > 0.01))
PY
done; done
