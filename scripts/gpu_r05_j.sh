#!/bin/bash
# Round-5 session J: pooled stream-ordered builder scratch + sized wave sorts -- wide / parity / mgpu tests,
# the C3 build probe, the C3 bench line (scene_build_ms), and C2's bands with time refinement.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_wide.py tests/test_gpu_parity.py \
  tests/test_gpu_mgpu.py > gpurun_out/j_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" gpurun_out/j_tests.log | head -20; tail -20 gpurun_out/j_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/j_tests.log | tail -2
timeout -k 10 300 python scripts/build_probe.py --scene C3 --repeat 4 > gpurun_out/j_build_C3.txt 2>&1 || { echo "build probe failed"; tail -5 gpurun_out/j_build_C3.txt; exit 1; }
cat gpurun_out/j_build_C3.txt
VARIANTS="base" SCENES="C3" STEPS=20 bash scripts/gpu_ab_env.sh || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/ab_C3_base.full.json')); print('bench C3 scene_build_ms', d['config']['scene_build_ms'])"
for rf in 0 2; do
  timeout -k 10 400 python scripts/band_probe.py --scene C2 --balanced --all-ranks 8 --steps 150 --refine $rf \
    > gpurun_out/band_all_C2_j_refine$rf.txt 2>&1 || { echo "band probe refine $rf failed"; tail -5 gpurun_out/band_all_C2_j_refine$rf.txt; exit 1; }
  python3 - gpurun_out/band_all_C2_j_refine$rf.txt "refine $rf" <<'PY'
import re, sys
t = [float(m.group(1)) for m in re.finditer(r"wall ([0-9.]+) ms/frame", open(sys.argv[1]).read())]
print(f"{sys.argv[2]:12s} bands: max {max(t):.4f} mean {sum(t) / len(t):.4f} ms  {['%.4f' % x for x in t]}", flush=True)
PY
done
echo "session j done"
