#!/bin/bash
# Round-5 session AJ: pipelined geometry updates on a high-priority stream (RESTIR_UPDATE_STREAM, default on) with the
# round-4 wide-node encoder -- tests, then C5: default, RESTIR_UPDATE_STREAM=0, and
# lib_head (the same library before the stream), two interleaved rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_wide.py tests/test_gpu_parity.py \
  "tests/test_gpu_workloads.py::test_c5_moving_lights_sequence" tests/test_gpu_mgpu.py > gpurun_out/aj_tests.log 2>&1 \
  || { echo "tests failed"; grep -E "FAILED|assert|Error" gpurun_out/aj_tests.log | head; exit 1; }
grep -E "passed|failed" gpurun_out/aj_tests.log | tail -1
for rep in 1 2; do
  for v in base nostream head; do
    so=restir-embree_amd/_ab/lib_base.so; envs=""
    [ $v = head ] && so=restir-embree_amd/_ab/lib_head.so
    [ $v = nostream ] && envs="RESTIR_UPDATE_STREAM=0"
    env $envs RESTIR_LIB=$PWD/$so timeout -k 10 240 python bench.py --scene C5 --steps 240 --warmup 5 --no-cpu-baseline --no-extras \
      > gpurun_out/aj_$v.log 2>&1 || { echo "$v failed"; tail -3 gpurun_out/aj_$v.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/aj_$v.log').read().strip().splitlines()[-1]); print('$v', d['value'])"
  done
done
echo "session aj done"
