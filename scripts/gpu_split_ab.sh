#!/bin/bash
# Candidate-split cost weights (RS_SPLIT_BRDF_W variants in _ab/): bit-identity of the split pass, then
# every rank of C2's N=8 bands per variant (max / mean of the per-rank band times).  Build the variants
# first: scripts/build_variant.sh w2 "-DRS_SPLIT_BRDF_W=2" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${LIBS:-w3}; do
  RESTIR_LIB=restir-embree_amd/_ab/lib_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "initial_split" --timeout 200 --timeout-method thread > gpurun_out/pt_$v.log 2>&1 || { echo "parity $v failed"; tail -20 gpurun_out/pt_$v.log; exit 1; }
  echo "parity $v: $(tail -1 gpurun_out/pt_$v.log)"
done
for rep in 1 2; do
  for v in base ${LIBS:-w3}; do
    envs=""; [ "$v" != base ] && envs="RESTIR_LIB=restir-embree_amd/_ab/lib_$v.so"
    env $envs timeout -k 10 300 python scripts/band_probe.py --scene C2 --balanced --steps 200 --all-ranks 8 > gpurun_out/split_$v.txt 2>&1 || { echo "probe $v failed"; tail -5 gpurun_out/split_$v.txt; exit 1; }
    python - gpurun_out/split_$v.txt "$v" <<'PY'
import re, sys
t = [float(m.group(1)) for m in re.finditer(r"wall ([0-9.]+) ms/frame", open(sys.argv[1]).read())]
r = [int(m.group(1)) for m in re.finditer(r"rows=(\d+)", open(sys.argv[1]).read())]
print(f"{sys.argv[2]:6s} max {max(t):.4f} mean {sum(t)/len(t):.4f} ranks {' '.join(f'{x:.4f}' for x in t)} rows {r}")
PY
  done
done
