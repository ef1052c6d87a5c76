#!/bin/bash
# Round-5 session R: the sorted initial pass by persistent waves (RESTIR_PERSIST_SORTED) -- bit identity, then
# C3 (and C4 on one GPU) A/B, two interleaved rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "persistent_sorted or sorted_initial" \
  > gpurun_out/r_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|assert|Error" gpurun_out/r_tests.log | head; tail -30 gpurun_out/r_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/r_tests.log | tail -2
for r in 1 2; do
  VARIANTS="base RESTIR_PERSIST_SORTED=on" SCENES="C3" STEPS=15 bash scripts/gpu_ab_env.sh || exit 1
done
echo "session r done"
