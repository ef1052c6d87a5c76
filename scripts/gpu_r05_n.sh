#!/bin/bash
# Round-5 session N: the initial pass's wave budgets re-tuned on the final tree -- C2 (lockstep: RS_INITIAL_WAVES 4 / 5
# / 6) and C3 (per-lane: RS_INITIAL_WAVES_LANE 5 / 6 / 7), two interleaved rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do
  VARIANTS="base RESTIR_LIB=restir-embree_amd/_ab/lib_iw4.so RESTIR_LIB=restir-embree_amd/_ab/lib_iw6.so" SCENES="C2" STEPS=30 bash scripts/gpu_ab_env.sh || exit 1
  VARIANTS="base RESTIR_LIB=restir-embree_amd/_ab/lib_iwl5.so RESTIR_LIB=restir-embree_amd/_ab/lib_iwl7.so" SCENES="C3" STEPS=12 bash scripts/gpu_ab_env.sh || exit 1
done
echo "session n done"
