#!/bin/bash
# Round-5 session AC: kernel statistics of the C5 sequence (rocprofv3 --kernel-trace --stats over bench.py --scene C5)
# -- where C5's frame time goes beyond C2's (initial pass, temporal, refit and light tables).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ac_prof -o ac -- python3 bench.py --scene C5 --steps 240 --warmup 5 --no-cpu-baseline --no-extras \
  > gpurun_out/ac_bench.log 2>&1 || { echo "profile failed"; tail -20 gpurun_out/ac_bench.log; exit 1; }
f=$(find gpurun_out/ac_prof -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/ac_C5_kernel_stats.csv
python3 - gpurun_out/ac_C5_kernel_stats.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:16]:
    print(f"{r['Name'][:70]:70s} calls={r['Calls']:>5s} avg_us={float(r['AverageNs'])/1e3:8.3f} share={float(r['TotalDurationNs'])/tot:.3f}")
PY
tail -1 gpurun_out/ac_bench.log | cut -c1-200
echo "session ac done"
