#!/bin/bash
# LDS top-of-tree cache A/B: BVH + frame parity tests on the default build, then C3 / C2 benches of the
# RS_WIDE_TOP variants interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ab_top_tests.log 2>&1
rc=$?; echo "parity tests rc=$rc: $(tail -1 gpurun_out/ab_top_tests.log)"; [ $rc -ne 0 ] && { tail -30 gpurun_out/ab_top_tests.log; exit 1; }
for rep in 1 2; do
for v in top0 top73 top9; do
  for sc in C3 C2; do
    RESTIR_LIB=$PWD/restir-embree_amd/_ab/$v.so timeout -k 10 240 python bench.py --scene $sc --steps 20 --warmup 3 --no-cpu-baseline --no-extras > gpurun_out/ab_${v}_$sc.log 2>&1 || { echo "$v $sc failed"; tail -5 gpurun_out/ab_${v}_$sc.log; exit 1; }
    python - "$v $sc" gpurun_out/ab_${v}_$sc.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(f"{sys.argv[1]:>10s} fps={d['value']:8.2f} " + " ".join(f"{k}={v:.3f}" for k, v in d['pass_ms_one_frame_in_flight'].items() if v > 0.01), flush=True)
PY
  done
done; done
