#!/bin/bash
# Round-5 session I: wave-parallel small-segment builds and the code-object preload -- BVH / wide-tree / parity tests, the C3 build timed over repeated
# builds and traced; the denoiser tests with k_conv3 back as the default.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_wide.py tests/test_gpu_parity.py \
  >  gpurun_out/i_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" gpurun_out/i_tests.log | head -20; tail -20 gpurun_out/i_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/i_tests.log | tail -2
timeout -k 10 300 python scripts/build_probe.py --scene C3 --repeat 4 > gpurun_out/i_build_C3.txt 2>&1 || { echo "build probe failed"; tail -5 gpurun_out/i_build_C3.txt; exit 1; }
cat gpurun_out/i_build_C3.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/i_buildtrace" -o run -- \
  python3 "$R/scripts/build_probe.py" --scene C3 --repeat 3 > "$R/gpurun_out/i_buildtrace.log" 2>&1 || { echo "build trace failed"; tail -5 "$R/gpurun_out/i_buildtrace.log"; exit 1; }
echo "session i done"
