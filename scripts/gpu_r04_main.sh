#!/bin/bash
# Round-4 GPU session: the -m gpu suite, then band / occupancy / host-overhead probes (each step under its own
# time limit; stops at a test failure; probes print one summary line each into gpurun_out/main_*.txt).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > gpurun_out/main_pytest.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -2 gpurun_out/main_pytest.log
  [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/main_pytest.log | head -20; exit $rc; }
  grep "\[parity\]\|\[rccl-stub\]\|\[wide\]" gpurun_out/main_pytest.log | sed 's/^tests[^ ]* //' > gpurun_out/main_parity_stats.txt
fi
P() { timeout -k 10 150 "$@" 2>&1 | grep -v amdgpu.ids; }
{
for L in default ${LIBS}; do
  E=""; [ $L != default ] && E="RESTIR_LIB=$L"
  echo "== lib $L"
  P env $E python scripts/band_probe.py --scene C2 --balanced --only-n 8 --steps 300
done
P python scripts/band_probe.py --scene C2 --balanced --steps 200
P python scripts/host_overhead.py --steps 2000
P python scripts/host_overhead.py --steps 2000 --mgpu 1
P env RESTIR_RUNAHEAD=0 python scripts/initial_breakdown.py --scene C3 --frames 5
} > gpurun_out/main_probes.txt
cat gpurun_out/main_probes.txt
