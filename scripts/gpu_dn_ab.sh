#!/bin/bash
# Denoiser A/B of library variants in restir-embree_amd/_ab/ (bench_denoise.py --no-cpu, per-layer ms)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
for v in ${VARIANTS:-dnbase}; do
  RESTIR_LIB=$PWD/restir-embree_amd/_ab/$v.so timeout -k 10 120 python -u scripts/bench_denoise.py --no-cpu > gpurun_out/dnab_$v.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/dnab_$v.log; exit 1; }
  python - "$v" gpurun_out/dnab_$v.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(f"{sys.argv[1]:>8s} {d['execute_ms_hip_events']:.3f} ms " + " ".join(f"{k.replace('_conv','')}={v*1e3:.0f}" for k, v in d['layer_ms'].items()), flush=True)
PY
done; done
