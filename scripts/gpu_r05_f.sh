#!/bin/bash
# Round-5 session F: the pipelined denoiser convolution on every 2..4-n-tile layer -- bit identity vs
# k_conv3, per-layer A/B (RESTIR_DN_PIPE=0 / 1), then rocprofv3 kernel trace and one SQ --pmc pass per arm.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_denoise.py \
  > gpurun_out/f_denoise_tests.log 2>&1 || { echo "denoise tests failed"; tail -40 gpurun_out/f_denoise_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/f_denoise_tests.log | tail -2
for r in 1 2; do for v in 0 1; do
  RESTIR_DN_PIPE=$v timeout -k 10 300 python scripts/bench_denoise.py --no-cpu > gpurun_out/f_dn_pipe${v}_r$r.json 2> gpurun_out/f_dn_pipe${v}_r$r.err \
    || { echo "bench_denoise pipe=$v failed"; tail -20 gpurun_out/f_dn_pipe${v}_r$r.err; exit 1; }
  python3 - gpurun_out/f_dn_pipe${v}_r$r.json "pipe=$v r$r" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
lm = d.get("layer_ms", {})
print(f"{sys.argv[2]}: execute {d.get('execute_ms_hip_events')} ms  " + " ".join(f"{k}={v}" for k, v in lm.items()), flush=True)
PY
done; done
cd /tmp && export TMPDIR=/tmp
for v in 0 1; do
  RESTIR_DN_PIPE=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/f_dntrace_$v" -o run -- \
    python3 "$R/scripts/bench_denoise.py" --no-cpu > "$R/gpurun_out/f_dntrace_$v.log" 2>&1 || { echo "trace $v failed"; tail -5 "$R/gpurun_out/f_dntrace_$v.log"; exit 1; }
  echo "trace $v ok"
  RESTIR_DN_PIPE=$v timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT \
    --output-format csv -d "$R/gpurun_out/f_dnpmc_$v" -o run -- python3 "$R/scripts/bench_denoise.py" --no-cpu > "$R/gpurun_out/f_dnpmc_$v.log" 2>&1 \
    || { echo "pmc $v failed"; tail -5 "$R/gpurun_out/f_dnpmc_$v.log"; exit 1; }
  echo "pmc $v ok"
done
echo "session f done"
