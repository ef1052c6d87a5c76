#!/bin/bash
# cache counters of the C3 shadow-ray walks (queued pass: k_q_trace is nothing but walks)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
cd /tmp && export TMPDIR=/tmp
export RESTIR_QUEUE=on RESTIR_RUNAHEAD=0 RESTIR_TRAVERSAL=lane
for C in "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" "SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU"; do
  D=${C%% *}
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d "$R/gpurun_out/pmct_$D" -o run -- \
     python3 "$R/bench.py" --scene C3 --steps 2 --warmup 1 --no-cpu-baseline --no-extras > "$R/gpurun_out/pmct_$D.log" 2>&1 \
     || { echo "pmc $C failed"; tail -5 "$R/gpurun_out/pmct_$D.log"; exit 1; }
  python3 - "$R/gpurun_out/pmct_$D/run_counter_collection.csv" <<'PY'
import csv, sys, collections
v = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"].split("(")[0].replace("void ", "")
    if "k_q_" in k or "k_temporal" in k or "k_spatial" in k:
        v[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), x in sorted(v.items()):
    print(f"{k[:28]:28s} {c:32s} {sum(x)/len(x):.4g}")
PY
done
