#!/bin/bash
# scripts/initial_breakdown.py configs (ONLY=list of indices) for each _variants/*.so (diagnostic builds)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export RESTIR_TRAVERSAL=${RESTIR_TRAVERSAL:-lockstep}
for so in restir-embree_amd/_variants/${VARIANTS:-*}.so; do
  for i in ${ONLY:-0 6}; do
    RESTIR_LIB=$PWD/$so timeout -k 10 120 python scripts/initial_breakdown.py --only $i --frames ${FRAMES:-10} 2>/dev/null | grep gbuffer || { echo "$so failed"; exit 1; }
  done
done
