set -o pipefail
mkdir -p gpurun_out
for k in 3 4; do
timeout -k 10 150 python scripts/band_probe.py --scene C2 --steps 200 --balanced --inflight $k > gpurun_out/band_c2_if$k.log 2>&1 || exit 1
done
timeout -k 10 150 python scripts/band_probe.py --scene C2 --steps 200 --balanced --inflight 2 --split off > gpurun_out/band_c2_if2_off.log 2>&1 || exit 1
timeout -k 10 150 python scripts/band_probe.py --scene C2 --steps 200 --balanced --inflight 2 --split on > gpurun_out/band_c2_if2_on.log 2>&1 || exit 1
