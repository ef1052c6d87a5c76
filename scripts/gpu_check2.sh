# full GPU tests, then benches for C2/C3/C5 and the N-band probe (stops at the first failure)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for sc in C2 C5 C3; do
  timeout -k 10 300 python bench.py --scene $sc --no-cpu-baseline > gpurun_out/bench_$sc.log 2>&1 || { tail -5 gpurun_out/bench_$sc.log; exit 1; }
  tail -1 gpurun_out/bench_$sc.log | cut -c1-400
done
timeout -k 10 150 python scripts/band_probe.py --scene C2 --steps 200 --balanced > gpurun_out/band_ra.log 2>&1 || exit 1
grep "N=" gpurun_out/band_ra.log | cut -c1-110
