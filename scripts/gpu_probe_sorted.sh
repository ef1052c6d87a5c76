#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/probe_sorted" -o run -- \
  python3 "$R/scripts/sorted_rays_probe.py" ${PROBE_ARGS} > "$R/gpurun_out/probe_sorted.log" 2>&1 || { tail -20 "$R/gpurun_out/probe_sorted.log"; exit 1; }
cat "$R/gpurun_out/probe_sorted.log" | tail -10
python3 - "$R/gpurun_out/probe_sorted/run_kernel_trace.csv" <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "k_debug_trace" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
for r in rows:
    print(f"k_debug_trace {(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6:.3f} ms")
PY
