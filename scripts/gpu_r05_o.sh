#!/bin/bash
# Round-5 session O: the current library against the session-J build (commit 8605dce) on one box -- C3 and C2
# pass times, two interleaved rounds (the C3 temporal pass read 1.08 ms in sessions D/J and 1.33 in session N).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do
  VARIANTS="base RESTIR_LIB=restir-embree_amd/_ab/lib_j.so" SCENES="C3 C2" STEPS=20 bash scripts/gpu_ab_env.sh || exit 1
done
echo "session o done"
