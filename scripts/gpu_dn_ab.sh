#!/bin/bash
# denoiser A/B of prebuilt libraries (restir-embree_amd/_ab/*.so): parity tests on each, then the timing probe, interleaved twice
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for so in restir-embree_amd/_ab/*.so; do
  n=$(basename $so .so); [ "$n" = base ] && continue
  RESTIR_LIB=$PWD/$so timeout -k 10 300 python -u -m pytest tests/test_gpu_denoise.py -x -q --timeout 120 --timeout-method thread > gpurun_out/dn_ab_tests_$n.log 2>&1 \
    || { echo "$n: denoiser tests failed"; tail -30 gpurun_out/dn_ab_tests_$n.log; exit 1; }
  echo "$n: $(tail -1 gpurun_out/dn_ab_tests_$n.log)"
done
for rep in 1 2; do for so in restir-embree_amd/_ab/*.so; do
  n=$(basename $so .so)
  RESTIR_LIB=$PWD/$so timeout -k 10 120 python -u scripts/denoise_probe.py > gpurun_out/dn_ab_$n.log 2>&1 || { tail -5 gpurun_out/dn_ab_$n.log; exit 1; }
  echo "$n"; tail -2 gpurun_out/dn_ab_$n.log
done; done
