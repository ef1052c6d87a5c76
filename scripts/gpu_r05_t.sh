#!/bin/bash
# Round-5 session T: the persistent sorted pass at 2 / 3 resident workgroups per CU against the one-launch pass,
# C3 (1080p) and C4's scene at 4K on one GPU, two interleaved rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do
  VARIANTS="base RESTIR_PERSIST_SORTED=on,RESTIR_PERSIST_SORTED_WGS=3 RESTIR_PERSIST_SORTED=on,RESTIR_PERSIST_SORTED_WGS=2" \
    SCENES="C3" STEPS=15 bash scripts/gpu_ab_env.sh || exit 1
  VARIANTS="base RESTIR_PERSIST_SORTED=on,RESTIR_PERSIST_SORTED_WGS=3" SCENES="C4" STEPS=6 bash scripts/gpu_ab_env.sh || exit 1
done
echo "session t done"
