#!/bin/bash
# Round-5 session AP (timing study): the counter RNG's hash with two full-rate 24-bit multiplies (RS_DIAG_CHEAP_RNG=2,
# lib_hash24; scripts/rng_quality.py: avalanche bias as the product's lowbias32) -- C2 and C3 both ways.  Different
# random numbers, so no parity against the oracle (which keeps lowbias32).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
AB_TESTS="tests/test_gpu_wide.py -k gpu_equals_host" BENCH_ARGS="--scene C2" STEPS=60 REPS=3 bash scripts/ab_r05.sh || exit 1
AB_TESTS="tests/test_gpu_wide.py -k gpu_equals_host" BENCH_ARGS="--scene C3" STEPS=15 REPS=1 bash scripts/ab_r05.sh || exit 1
echo "session ap done"
