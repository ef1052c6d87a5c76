#!/bin/bash
# gpu_r03.sh followed by the denoiser timing probe (per-layer ms)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_r03.sh || exit $?
timeout -k 10 120 python -u scripts/denoise_probe.py > gpurun_out/dn_probe.log 2>&1; rc=$?
echo "dn_probe rc=$rc"; tail -3 gpurun_out/dn_probe.log
exit $rc
