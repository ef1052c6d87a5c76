#!/bin/bash
# Round-5 session E: the pipelined denoiser convolution (k_conv3p) -- bit identity vs k_conv3, the float64
# per-layer parity, the denoise sub-line A/B; the band margin split A/B and the band bit-identity tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_denoise.py \
  > gpurun_out/e_denoise_tests.log 2>&1 || { echo "denoise tests failed"; tail -40 gpurun_out/e_denoise_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/e_denoise_tests.log | tail -2
for r in 1 2; do for v in 0 1; do
  RESTIR_DN_PIPE=$v timeout -k 10 300 python scripts/bench_denoise.py --no-cpu > gpurun_out/e_dn_pipe${v}_r$r.json 2> gpurun_out/e_dn_pipe${v}_r$r.err \
    || { echo "bench_denoise pipe=$v failed"; tail -20 gpurun_out/e_dn_pipe${v}_r$r.err; exit 1; }
  python3 - gpurun_out/e_dn_pipe${v}_r$r.json "pipe=$v r$r" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
lm = d.get("layer_ms", {})
print(f"{sys.argv[2]}: execute {d.get('execute_ms_hip_events')} ms  " + " ".join(f"{k}={v}" for k, v in lm.items()), flush=True)
PY
done; done
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_mgpu.py \
  "tests/test_gpu_workloads.py::test_c4_eight_bands_4k_bit_identical" > gpurun_out/e_band_tests.log 2>&1 \
  || { echo "band tests failed"; tail -40 gpurun_out/e_band_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/e_band_tests.log | tail -2
for v in base RESTIR_MARGIN_SPLIT=off; do
  envs=""; [ "$v" != base ] && envs="$v"
  tag=$(echo "$v" | tr '/=.' '__-')
  env $envs timeout -k 10 400 python scripts/band_probe.py --scene C2 --balanced --all-ranks 8 --steps 150 \
    > gpurun_out/band_all_C2_e_$tag.txt 2>&1 || { echo "band probe $v failed"; tail -5 gpurun_out/band_all_C2_e_$tag.txt; exit 1; }
  python3 - gpurun_out/band_all_C2_e_$tag.txt "$v" <<'PY'
import re, sys
t = [float(m.group(1)) for m in re.finditer(r"wall ([0-9.]+) ms/frame", open(sys.argv[1]).read())]
print(f"{sys.argv[2]:30s} bands: max {max(t):.4f} mean {sum(t) / len(t):.4f} ms  {['%.4f' % x for x in t]}", flush=True)
PY
done
echo "session e done"
