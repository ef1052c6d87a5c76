#!/bin/bash
# per-kernel average durations of a short bench run (rocprofv3 --kernel-trace --stats), one frame in flight
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
cd /tmp && export TMPDIR=/tmp
RESTIR_RUNAHEAD=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/kt_${TAG:-x}" -o run -- \
  python3 "$R/bench.py" ${BENCH_ARGS:---scene C3} --steps 8 --warmup 2 --no-cpu-baseline --no-extras > "$R/gpurun_out/kt_${TAG:-x}.json" 2>/dev/null || exit 1
python3 - "$R/gpurun_out/kt_${TAG:-x}/run_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if float(r["AverageNs"]) > 20000:
        print(f"{r['Name'].split('(')[0][:60]:60s} calls {r['Calls']:>4s} avg {float(r['AverageNs'])/1e6:8.3f} ms")
PY
