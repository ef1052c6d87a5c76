#!/bin/bash
# Round-5 session A: the new / changed -m gpu tests (240-frame C5 and C3 4K vs the oracle, time-based rebalance,
# wide refit with NaN / inf), then the initial-pass breakdown and the C2 band probe of every rank at N = 8.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_workloads.py::test_c5_1080p tests/test_gpu_workloads.py::test_c3_4k_frame \
  tests/test_gpu_mgpu.py tests/test_gpu_wide.py -m gpu -x -v -s --timeout 600 --timeout-method thread \
  > gpurun_out/pytest_a.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/pytest_a.log | tail -2
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/pytest_a.log | head -20; exit $rc; }
timeout -k 10 300 python scripts/initial_breakdown.py --scene C2 > gpurun_out/breakdown_C2.txt 2>&1 || exit 1
grep C2 gpurun_out/breakdown_C2.txt
timeout -k 10 400 python scripts/band_probe.py --scene C2 --balanced --all-ranks 8 --steps 150 > gpurun_out/band_all_C2.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/band_all_C2.txt | tail -3
