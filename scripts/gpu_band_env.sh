#!/bin/bash
# C2's 1/8 band (scripts/band_probe.py --only-n 8) under environment switches: "NAME=v,NAME2=v" or base
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${VARIANTS:-base}; do
  envs=""; [ "$v" != base ] && envs=$(echo $v | tr ',' ' ')
  env $envs timeout -k 10 200 python scripts/band_probe.py --scene ${SCENE:-C2} --balanced --steps ${STEPS:-200} --only-n ${N:-8} > gpurun_out/bandenv.txt 2>&1 || { echo "probe $v failed"; tail -5 gpurun_out/bandenv.txt; exit 1; }
  echo "$v :: $(grep -v amdgpu.ids gpurun_out/bandenv.txt | tail -1)"
done
