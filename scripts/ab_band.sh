#!/bin/bash
# A/B of _variants/*.so on one rank's band (scripts/band_probe.py --balanced): per-variant wall ms/frame
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
for so in restir-embree_amd/_variants/${VARIANTS:-*}.so; do
  n=$(basename $so .so)
  for N in ${NS:-4 8}; do
    RESTIR_LIB=$PWD/$so timeout -k 10 120 python scripts/band_probe.py ${BAL---balanced} --only-n $N --steps ${STEPS:-300} ${PROBE_ARGS} > gpurun_out/abb_${n}_$N.log 2>&1 || { echo "$n N=$N failed"; tail -3 gpurun_out/abb_${n}_$N.log; exit 1; }
    echo "$n $(grep -o 'N=[0-9] rank.*wall [0-9.]* ms/frame' gpurun_out/abb_${n}_$N.log | sed 's/rank=.*wall/wall/')"
  done
done; done
