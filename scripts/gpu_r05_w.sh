#!/bin/bash
# Round-5 session W: where C2's initial pass spends its time (scripts/initial_breakdown.py: primary ray / area
# sampling / shadow rays / BRDF ray, by parameter variations), on the final tree.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/initial_breakdown.py --scene ${SCENE:-C2} --frames ${FRAMES:-20} > gpurun_out/w_breakdown_${SCENE:-C2}.txt 2>&1 \
  || { echo "breakdown failed"; tail -20 gpurun_out/w_breakdown_${SCENE:-C2}.txt; exit 1; }
cat gpurun_out/w_breakdown_${SCENE:-C2}.txt
echo "session w done"
