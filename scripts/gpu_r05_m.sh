#!/bin/bash
# Round-5 session M: band boundaries on whole 8-row wave tiles -- the multi-GPU tests, then C2's eight 1/8 bands
# (cost balanced; then two rounds of time refinement) and C4's eight bands at 4K, each rank timed alone.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_mgpu.py \
  "tests/test_gpu_workloads.py::test_c4_eight_bands_4k_bit_identical" > gpurun_out/m_tests.log 2>&1 \
  || { echo "tests failed"; grep -E "FAILED|Error|assert" gpurun_out/m_tests.log | head; tail -20 gpurun_out/m_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/m_tests.log | tail -2
summ() {
python3 - "$1" "$2" <<'PY'
import re, sys
txt = open(sys.argv[1]).read()
rounds = re.findall(r"\[round (\d+)\] bands \[([^\]]*)\]: max ([0-9.]+) mean ([0-9.]+)", txt)
if rounds:
    for r, rows, mx, mn in rounds:
        print(f"{sys.argv[2]:14s} round {r}: rows [{rows}] max {mx} mean {mn} ms", flush=True)
else:
    t = [float(m.group(1)) for m in re.finditer(r"wall ([0-9.]+) ms/frame", txt)]
    rows = [int(m.group(1)) for m in re.finditer(r"rows=(\d+)", txt)]
    print(f"{sys.argv[2]:14s} bands: max {max(t):.4f} mean {sum(t) / len(t):.4f} ms  rows {rows}  {['%.4f' % x for x in t]}", flush=True)
PY
}
for rf in 0 2; do
  timeout -k 10 400 python scripts/band_probe.py --scene C2 --balanced --all-ranks 8 --steps 150 --refine $rf \
    > gpurun_out/band_all_C2_m_refine$rf.txt 2>&1 || { echo "C2 band probe refine $rf failed"; tail -5 gpurun_out/band_all_C2_m_refine$rf.txt; exit 1; }
  summ gpurun_out/band_all_C2_m_refine$rf.txt "C2 refine $rf"
done
timeout -k 10 600 python scripts/band_probe.py --scene C3 --width 3840 --height 2160 --balanced --all-ranks 8 --steps 12 --refine 2 \
  > gpurun_out/band_all_C4_m.txt 2>&1 || { echo "C4 band probe failed"; tail -5 gpurun_out/band_all_C4_m.txt; exit 1; }
summ gpurun_out/band_all_C4_m.txt "C4 refine 2"
echo "session m done"
