set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_tiles.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "tiles or split or c2_metric or temporal" > gpurun_out/t_tiles.log 2>&1 || { tail -40 gpurun_out/t_tiles.log; exit 1; }
tail -3 gpurun_out/t_tiles.log
timeout -k 10 150 python scripts/band_probe.py --scene C2 --steps 100 --all-ranks 8 --balanced > gpurun_out/band_c2_bal.log 2>&1 || exit 1
timeout -k 10 150 python scripts/band_probe.py --scene C2 --steps 100 --balanced > gpurun_out/band_c2_bal_n.log 2>&1 || exit 1
