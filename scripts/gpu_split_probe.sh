set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "split or traversal or c2_metric" > gpurun_out/t_split.log 2>&1 || { tail -30 gpurun_out/t_split.log; exit 1; }
tail -3 gpurun_out/t_split.log
for m in off on; do timeout -k 10 150 python scripts/band_probe.py --scene C2 --steps 100 --split $m > gpurun_out/band_c2_$m.log 2>&1 || exit 1; done
timeout -k 10 150 python scripts/band_probe.py --scene C2 --steps 100 --all-ranks 8 --split on > gpurun_out/band_c2r_on.log 2>&1 || exit 1
timeout -k 10 200 python scripts/band_probe.py --scene C3 --steps 10 --split on > gpurun_out/band_c3_on.log 2>&1 || exit 1
