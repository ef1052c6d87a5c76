#!/bin/bash
# Round-5 session B: the persistent-wave initial pass (RESTIR_PERSIST=on) through the parity suite, then A/B against
# the default launch on C2 and C3 (two interleaved rounds).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
RESTIR_PERSIST=on timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/pytest_persist.log 2>&1 || { echo "persist: parity tests failed"; tail -30 gpurun_out/pytest_persist.log; exit 1; }
echo "persist parity: $(tail -1 gpurun_out/pytest_persist.log)"
for rep in 1 2; do
  VARIANTS="base RESTIR_PERSIST=on" SCENES="C2 C3" STEPS=30 bash scripts/gpu_ab_env.sh || exit 1
done
