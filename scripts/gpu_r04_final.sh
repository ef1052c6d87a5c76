#!/bin/bash
# Round-4 closing session: every -m gpu test, smoke, rocprofv3 stats + PMC (C2, C3), the bench line, and the
# band probes (C2 and C4 at N = 1/2/4/8).  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
NO_BENCH=1 bash scripts/gpu_r04.sh || exit 1
bash scripts/gpu_profile_r04.sh || exit 1
NO_TESTS=1 NO_SMOKE=1 bash scripts/gpu_r04.sh || exit 1
timeout -k 10 300 python scripts/band_probe.py --scene C2 --balanced --steps 200 > gpurun_out/band_C2.txt 2>&1 || exit 1
timeout -k 10 400 python scripts/band_probe.py --scene C3 --width 3840 --height 2160 --balanced --steps 16 > gpurun_out/band_C4.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/band_C2.txt gpurun_out/band_C4.txt
