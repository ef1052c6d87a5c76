#!/bin/bash
# Round-5 session AH: the wide-node quantisation with exact power-of-two multiplications instead of double divisions,
# its slot loops unrolled (no scratch: session AH2)
# (rs_wide.h wide_axis; lib_head = before) -- wide-tree / refit tests, the update probe, C5 and C3 frame rates both ways.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_wide.py tests/test_gpu_parity.py \
  "tests/test_gpu_workloads.py::test_c5_moving_lights_sequence" tests/test_gpu_mgpu.py > gpurun_out/ah_tests.log 2>&1 \
  || { echo "tests failed"; grep -E "FAILED|assert|Error" gpurun_out/ah_tests.log | head; exit 1; }
grep -E "passed|failed" gpurun_out/ah_tests.log | tail -1
for so in base head; do
  RESTIR_LIB=$PWD/restir-embree_amd/_ab/lib_$so.so timeout -k 10 300 python scripts/update_probe.py --updates 50 2>&1 | grep "per update" | sed "s/^/$so: /" || exit 1
done
AB_TESTS="tests/test_gpu_wide.py" BENCH_ARGS="--scene C5" STEPS=240 REPS=2 bash scripts/ab_r05.sh || exit 1
AB_TESTS="tests/test_gpu_wide.py" BENCH_ARGS="--scene C3" STEPS=15 REPS=1 bash scripts/ab_r05.sh || exit 1
echo "session ah done"
