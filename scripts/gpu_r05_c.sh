#!/bin/bash
# Round-5 session C: every -m gpu test on the current tree, then C2's eight 1/8 bands timed one by one with the
# candidate-split spatial pass (default for such launches) and without it, and with the 2-wave initial split.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
NO_BENCH=1 NO_SMOKE=1 bash scripts/gpu_r04.sh || exit 1
for v in base RESTIR_SPATIAL_SPLIT=off RESTIR_LIB=restir-embree_amd/_ab/lib_split2.so; do
  envs=""; [ "$v" != base ] && envs="$v"
  tag=$(echo "$v" | tr '/=.' '__-')
  env $envs timeout -k 10 400 python scripts/band_probe.py --scene C2 --balanced --all-ranks 8 --steps 150 \
    > gpurun_out/band_all_C2_$tag.txt 2>&1 || { echo "band probe $v failed"; tail -5 gpurun_out/band_all_C2_$tag.txt; exit 1; }
  python3 - gpurun_out/band_all_C2_$tag.txt "$v" <<'PY'
import re, sys
t = [float(m.group(1)) for m in re.finditer(r"wall ([0-9.]+) ms/frame", open(sys.argv[1]).read())]
print(f"{sys.argv[2]:45s} bands: max {max(t):.4f} mean {sum(t) / len(t):.4f} ms  {['%.4f' % x for x in t]}", flush=True)
PY
done
# the persistent initial pass with workgroup-granular tile pulls (RS_PERSIST_WG) against the default launch
RESTIR_PERSIST=on timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/pytest_persist_wg.log 2>&1 || { echo "persist-wg: parity tests failed"; tail -30 gpurun_out/pytest_persist_wg.log; exit 1; }
echo "persist-wg parity: $(tail -1 gpurun_out/pytest_persist_wg.log)"
for rep in 1 2; do
  VARIANTS="base RESTIR_PERSIST=on" SCENES="C2" STEPS=30 bash scripts/gpu_ab_env.sh || exit 1
done
