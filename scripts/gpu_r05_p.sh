#!/bin/bash
# Round-5 session P: kernel trace of one C2 1/8 band (rank 4 of 8, frames in flight) -- the launches of a band
# frame and their durations (scripts/trace_overlap.py summarises the overlap).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/p_bandtrace" -o run -- \
  python3 "$R/scripts/band_probe.py" --scene C2 --balanced --only-n 8 --steps 200 > "$R/gpurun_out/p_bandtrace.log" 2>&1 \
  || { echo "band trace failed"; tail -5 "$R/gpurun_out/p_bandtrace.log"; exit 1; }
grep -v amdgpu "$R/gpurun_out/p_bandtrace.log" | tail -3
echo "session p done"
