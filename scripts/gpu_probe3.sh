set -o pipefail
mkdir -p gpurun_out
for k in 1 2; do
timeout -k 10 150 python scripts/band_probe.py --scene C2 --steps 200 --balanced --inflight $k > gpurun_out/band_c2_if$k.log 2>&1 || exit 1
done
timeout -k 10 150 python scripts/band_probe.py --scene C2 --steps 100 --balanced --inflight 2 --all-ranks 8 > gpurun_out/band_c2_if2_all.log 2>&1 || exit 1
