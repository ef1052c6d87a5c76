#!/bin/bash
# Round-5 session AG: what one C5 geometry update costs alone (scripts/update_probe.py) and, under a kernel trace
# with RESTIR_UPDATE_SPLIT=1, which of the fused update kernel's three jobs is the long one.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python scripts/update_probe.py --updates 50 > gpurun_out/ag_probe.txt 2>&1 || { echo "probe failed"; tail -5 gpurun_out/ag_probe.txt; exit 1; }
grep "per update" gpurun_out/ag_probe.txt
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
RESTIR_UPDATE_SPLIT=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ag_prof -o ag -- python3 scripts/update_probe.py --updates 50 \
  > gpurun_out/ag_prof.log 2>&1 || { echo "profile failed"; tail -5 gpurun_out/ag_prof.log; exit 1; }
python3 - gpurun_out/ag_prof/ag_kernel_trace.csv <<'PY'
import csv, sys, statistics
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
upd = [r for r in rows if "k_scene_update" in r["Kernel_Name"]]
for j in range(3):
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in upd[j::3][4:]]
    print(f"k_scene_update job {j} ({['light tables', 'binary refit tail', 'wide refit tail'][j]}): median {statistics.median(d):.1f} us over {len(d)}")
other = {}
for r in rows:
    n = r["Kernel_Name"].split("(")[0]
    if "k_scene_update" in n: continue
    other.setdefault(n, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for n, d in sorted(other.items(), key=lambda kv: -sum(kv[1]))[:6]:
    print(f"{n[:60]:60s} calls={len(d)} median_us={statistics.median(d):.1f}")
PY
echo "session ag done"
