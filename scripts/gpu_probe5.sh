set -o pipefail
mkdir -p gpurun_out
for d in 0 1 2 3 4; do
timeout -k 10 150 python scripts/band_probe.py --scene C2 --steps 200 --balanced --ahead $d > gpurun_out/band_ahead$d.log 2>&1 || exit 1
grep "N=" gpurun_out/band_ahead$d.log | cut -c1-100
done
