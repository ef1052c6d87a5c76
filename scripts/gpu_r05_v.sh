#!/bin/bash
# Round-5 session V: the persistent sorted pass restricted to full frames without row-cost recording -- tests,
# C3 default vs off, C4's eight bands at 4K both ways.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "sorted" tests/test_gpu_mgpu.py \
  "tests/test_gpu_workloads.py::test_c4_eight_bands_4k_bit_identical" > gpurun_out/v_tests.log 2>&1 \
  || { echo "tests failed"; grep -E "FAILED|assert|Error" gpurun_out/v_tests.log | head; tail -30 gpurun_out/v_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/v_tests.log | tail -2
VARIANTS="base RESTIR_PERSIST_SORTED=off" SCENES="C3" STEPS=15 bash scripts/gpu_ab_env.sh || exit 1
for v in base RESTIR_PERSIST_SORTED=off; do
  envs=""; [ "$v" != base ] && envs="$v"
  env $envs timeout -k 10 600 python scripts/band_probe.py --scene C3 --width 3840 --height 2160 --balanced --all-ranks 8 --steps 12 \
    > gpurun_out/band_all_C4_v_${v//=/-}.txt 2>&1 || { echo "C4 band probe $v failed"; tail -5 gpurun_out/band_all_C4_v_${v//=/-}.txt; exit 1; }
  python3 - gpurun_out/band_all_C4_v_${v//=/-}.txt "$v" <<'PY'
import re, sys
txt = open(sys.argv[1]).read()
t = [float(m.group(1)) for m in re.finditer(r"wall ([0-9.]+) ms/frame", txt)]
print(f"C4 {sys.argv[2]:28s} bands: max {max(t):.3f} mean {sum(t) / len(t):.3f} ms  {['%.3f' % x for x in t]}", flush=True)
PY
done
echo "session v done"
