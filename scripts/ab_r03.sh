#!/bin/bash
# A/B of library builds and environment settings: `name|lib|env` entries in AB (space separated), bench.py on
# BENCH_ARGS for each, REPS times interleaved.  TESTS=1 first runs the -m gpu suite on the default library.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 180 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  echo "pytest rc=$rc: $(tail -1 gpurun_out/pytest_gpu.log)"
  [ $rc -ne 0 ] && { tail -40 gpurun_out/pytest_gpu.log; exit $rc; }
fi
for rep in $(seq 1 ${REPS:-2}); do
for e in $AB; do
  IFS='|' read -r n lib envs <<< "$e"
  L=""; [ -n "$lib" ] && L="RESTIR_LIB=$PWD/restir-embree_amd/_ab/$lib.so"
  env $L $envs timeout -k 10 240 python bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --no-extras ${BENCH_ARGS} > gpurun_out/ab_$n.log 2>&1; rc=$?
  [ $rc -ne 0 ] && { echo "$n rc=$rc"; tail -5 gpurun_out/ab_$n.log; exit $rc; }
  python - "$n" gpurun_out/ab_$n.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(f"{sys.argv[1]:>10s} fps={d['value']:8.2f} Mrays/s={d['mrays_per_s']:9.1f} " + " ".join(f"{k}={v:.3f}" for k, v in d['pass_ms_one_frame_in_flight'].items() if v > 0.01), flush=True)
PY
done; done
