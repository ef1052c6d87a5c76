#!/bin/bash
# Round-5 session AN (timing diagnostic): what the counter RNG's 32-bit multiplies cost -- lib_cheaprng replaces the
# hash by a multiply-free one (RS_DIAG_CHEAP_RNG=1; different random numbers, so no parity), C2 and C3 both ways.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
AB_TESTS="tests/test_gpu_wide.py -k gpu_equals_host" BENCH_ARGS="--scene C2" STEPS=60 REPS=2 bash scripts/ab_r05.sh || exit 1
AB_TESTS="tests/test_gpu_wide.py -k gpu_equals_host" BENCH_ARGS="--scene C3" STEPS=15 REPS=1 bash scripts/ab_r05.sh || exit 1
echo "session an done"
