#!/bin/bash
# Round-5 session D: parity / workload / multi-GPU tests with the temporal and spatial canonical-ray skips, the C2
# 1/8 bands one by one (default; initial split off; 6-wave initial budget), and the C2 / C3 / C5 bench lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TESTS="tests/test_gpu_parity.py tests/test_gpu_workloads.py tests/test_gpu_mgpu.py" NO_BENCH=1 NO_SMOKE=1 bash scripts/gpu_r04.sh || exit 1
for v in base RESTIR_SPLIT=off RESTIR_LIB=restir-embree_amd/_ab/lib_w6.so; do
  envs=""; [ "$v" != base ] && envs="$v"
  tag=$(echo "$v" | tr '/=.' '__-')
  env $envs timeout -k 10 400 python scripts/band_probe.py --scene C2 --balanced --all-ranks 8 --steps 150 \
    > gpurun_out/band_all_C2_d_$tag.txt 2>&1 || { echo "band probe $v failed"; tail -5 gpurun_out/band_all_C2_d_$tag.txt; exit 1; }
  python3 - gpurun_out/band_all_C2_d_$tag.txt "$v" <<'PY'
import re, sys
t = [float(m.group(1)) for m in re.finditer(r"wall ([0-9.]+) ms/frame", open(sys.argv[1]).read())]
print(f"{sys.argv[2]:45s} bands: max {max(t):.4f} mean {sum(t) / len(t):.4f} ms  {['%.4f' % x for x in t]}", flush=True)
PY
done
VARIANTS="base" SCENES="C2 C3 C5" STEPS=30 bash scripts/gpu_ab_env.sh || exit 1
timeout -k 10 300 python scripts/initial_breakdown.py --scene C2 --frames 6 > gpurun_out/breakdown_C2.txt 2>&1 || exit 1
timeout -k 10 400 python scripts/initial_breakdown.py --scene C3 --frames 4 > gpurun_out/breakdown_C3.txt 2>&1 || exit 1
grep -h "initial_ms" gpurun_out/breakdown_C2.txt gpurun_out/breakdown_C3.txt
