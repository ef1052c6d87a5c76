#!/bin/bash
# Round-5 session AK: the sorted initial pass's chunk and register budget re-checked with phase A's stored results
# (lib_c14w6: 14-candidate chunks at 6 waves per SIMD; lib_w6: 16 at 6) -- C3 both ways, two interleaved rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
AB_TESTS="tests/test_gpu_parity.py" BENCH_ARGS="--scene C3" STEPS=15 REPS=2 bash scripts/ab_r05.sh || exit 1
echo "session ak done"
