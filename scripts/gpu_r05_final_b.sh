#!/bin/bash
# Round-5 closing session, part B: rocprofv3 kernel statistics (frames in flight and one frame in flight) and
# the PMC passes of C2 and C3 (scripts/gpu_profile_r04.sh), then the 1080p denoise sub-line under the profiler.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out
bash scripts/gpu_profile_r04.sh || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_dn" -o run -- \
  python3 "$R/scripts/bench_denoise.py" --no-cpu > "$R/gpurun_out/prof_dn.json" 2> "$R/gpurun_out/prof_dn.err" || { echo "denoise profile failed"; tail -5 "$R/gpurun_out/prof_dn.err"; exit 1; }
echo "final B done"
