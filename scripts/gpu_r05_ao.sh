#!/bin/bash
# Round-5 session AO: phase B of the sorted pass forming its rays from the stored sample point (12 B, RS_SORT_STORE_RAY=2,
# lib_pt12) instead of the stored (direction, tfar) (16 B) -- parity tests on lib_pt12, C3 both ways, two rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
AB_TESTS="tests/test_gpu_parity.py tests/test_gpu_mgpu.py" BENCH_ARGS="--scene C3" STEPS=15 REPS=2 bash scripts/ab_r05.sh || exit 1
echo "session ao done"
