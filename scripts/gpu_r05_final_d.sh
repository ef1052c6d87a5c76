#!/bin/bash
# Round-5 closing session D (final tree after sessions W-AJ): every -m gpu test, smoke, and the default bench.py line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/gpu_r04.sh || exit 1
cp gpurun_out/bench.json gpurun_out/r05_bench_final.json
echo "final D done"
