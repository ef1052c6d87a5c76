#!/bin/bash
# A/B: bench.py with each _variants/*.so (RESTIR_LIB override); prints fps and pass times.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
for so in restir-embree_amd/_variants/${VARIANTS:-*}.so; do
  n=$(basename $so .so)
  RESTIR_LIB=$PWD/$so timeout -k 10 120 python bench.py --steps ${STEPS:-30} --warmup 3 --no-cpu-baseline --no-extras ${BENCH_ARGS} > gpurun_out/ab_$n.log 2>&1; rc=$?
  [ $rc -ne 0 ] && { echo "$n rc=$rc"; tail -3 gpurun_out/ab_$n.log; exit $rc; }
  python - "$n" gpurun_out/ab_$n.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(f"{sys.argv[1]:>14s} fps={d['value']:8.2f} Mrays/s={d['mrays_per_s']:9.1f} " + " ".join(f"{k}={v:.3f}" for k, v in d['pass_ms_one_frame_in_flight'].items() if v > 0.01))
PY
done; done
