# GPU tests + C2/C3 benches (quick check after a change); stops at the first failure
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for sc in ${SCENES:-C2 C3}; do
  timeout -k 10 300 python bench.py --scene $sc --no-cpu-baseline --steps ${STEPS:-20} > gpurun_out/bench_$sc.log 2>&1 || { tail -5 gpurun_out/bench_$sc.log; exit 1; }
  python - gpurun_out/bench_$sc.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"{d['config']['workload'][:3]} fps={d['value']:8.2f} Mrays/s={d['mrays_per_s']:9.1f} trav={d['config']['traversal']} " + " ".join(f"{k}={v:.3f}" for k, v in d['pass_ms'].items() if v > 0.01))
PY
done
