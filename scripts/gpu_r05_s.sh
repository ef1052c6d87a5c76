#!/bin/bash
# Round-5 session S: the persistent sorted pass with fewer resident workgroups per CU than the kernel's occupancy
# (room for the previous frame's passes in flight) -- C3 A/B, two interleaved rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do
  VARIANTS="base RESTIR_PERSIST_SORTED=on RESTIR_PERSIST_SORTED=on,RESTIR_PERSIST_SORTED_WGS=4 RESTIR_PERSIST_SORTED=on,RESTIR_PERSIST_SORTED_WGS=3" \
    SCENES="C3" STEPS=15 bash scripts/gpu_ab_env.sh || exit 1
done
echo "session s done"
