#!/bin/bash
# Round-5 session Q: k_conv3's all-chunks-loaded form for the coarse layers -- bit identity and the float64
# per-layer parity (test_gpu_denoise.py), then the denoise sub-line's layers, RESTIR_DN_ALLC=0 / 1, two rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_denoise.py \
  > gpurun_out/q_denoise_tests.log 2>&1 || { echo "denoise tests failed"; grep -E "FAILED|assert" gpurun_out/q_denoise_tests.log | head; tail -30 gpurun_out/q_denoise_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/q_denoise_tests.log | tail -2
for r in 1 2; do for v in 0 1; do
  RESTIR_DN_ALLC=$v timeout -k 10 300 python scripts/bench_denoise.py --no-cpu > gpurun_out/q_dn_allc${v}_r$r.json 2> gpurun_out/q_dn_allc${v}_r$r.err \
    || { echo "bench_denoise allc=$v failed"; tail -20 gpurun_out/q_dn_allc${v}_r$r.err; exit 1; }
  python3 - gpurun_out/q_dn_allc${v}_r$r.json "allc=$v r$r" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
lm = d.get("layer_ms", {})
print(f"{sys.argv[2]}: execute {d.get('execute_ms_hip_events')} ms  " + " ".join(f"{k}={v}" for k, v in lm.items()), flush=True)
PY
done; done
echo "session q done"
