#!/bin/bash
# Denoiser GPU round: tests, timing probe, bench sub-line, rocprofv3 kernel stats (csv).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_denoise.py -q -s --timeout 120 --timeout-method thread > gpurun_out/dn_tests.log 2>&1
echo "tests rc=$?" >> gpurun_out/dn_tests.log
timeout -k 10 300 python -u scripts/bench_denoise.py > gpurun_out/dn_bench.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
# profiled: bench.py's own denoise leg (the C2 frame's accumulator and G-buffer), so the per-layer durations
# match the bench line's (MFMA power, hence clocks, depends on the data: random inputs run ~10 % slower)
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/dn_prof" -o dn -- \
    python3 "$GRAFT_REPO_ROOT/scripts/bench_denoise.py" --no-cpu > "$GRAFT_REPO_ROOT/gpurun_out/dn_prof.log" 2>&1
cd "$GRAFT_REPO_ROOT" && python3 scripts/dn_trace_layers.py > gpurun_out/dn_probe.log 2>&1
