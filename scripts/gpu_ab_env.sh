#!/bin/bash
# A/B of environment switches on the GPU box: optional tests first (TESTS=...), then for each scene in
# SCENES and each setting in VARIANTS ("NAME=val,NAME2=val" or "base") a short bench.py line; prints fps and
# the one-frame-in-flight pass times.  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v -s -rf --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/pytest_gpu.log | tail -2
  [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
fi
for sc in ${SCENES:-C2 C3}; do
  for v in ${VARIANTS:-base}; do
    envs=""; [ "$v" != base ] && envs=$(echo $v | tr ',' ' ')
    tag=$(echo "$v" | tr '/,=' '_~-')
    env $envs timeout -k 10 300 python bench.py --scene $sc --no-cpu-baseline --no-extras --steps ${STEPS:-20} --full-out gpurun_out/ab_${sc}_$tag.full.json > gpurun_out/ab_${sc}_$tag.json 2> gpurun_out/ab_${sc}_$tag.err || { echo "bench $sc $v failed"; tail -5 gpurun_out/ab_${sc}_$tag.err; exit 1; }
    python - gpurun_out/ab_${sc}_$tag.full.json "$sc $v" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
p = d.get("pass_ms_one_frame_in_flight") or {}
print(f"{sys.argv[2]:40s} fps={d['value']:8.2f} trav={d['config']['traversal']} " + " ".join(f"{k[:-3]}={v:.3f}" for k, v in p.items() if v > 0.005))
PY
  done
done
