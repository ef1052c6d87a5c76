#!/bin/bash
# Round-5 session G: k_conv3p timing ablations (B-fragment DMA / halo DMA skipped: analysis builds, wrong
# results) beside the default and k_conv3; the C3 scene build timed over repeated builds and traced.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out
for v in "RESTIR_DN_PIPE=0" "RESTIR_DN_PIPE=1" "RESTIR_DN_PIPE=1 RESTIR_LIB=restir-embree_amd/_ab/lib_dnab1.so" \
         "RESTIR_DN_PIPE=1 RESTIR_LIB=restir-embree_amd/_ab/lib_dnab2.so" "RESTIR_DN_PIPE=1 RESTIR_LIB=restir-embree_amd/_ab/lib_dnab3.so"; do
  tag=$(echo "$v" | tr ' /=.' '____')
  env $v timeout -k 10 300 python scripts/bench_denoise.py --no-cpu > gpurun_out/g_dn_$tag.json 2> gpurun_out/g_dn_$tag.err \
    || { echo "bench_denoise $v failed"; tail -20 gpurun_out/g_dn_$tag.err; exit 1; }
  python3 - gpurun_out/g_dn_$tag.json "$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
lm = d.get("layer_ms", {})
print(f"{sys.argv[2][-40:]:40s}: execute {d.get('execute_ms_hip_events')} ms  " + " ".join(f"{k}={v}" for k, v in lm.items() if k.startswith(('dec_conv1', 'dec_conv2', 'enc_conv0', 'enc_conv1'))), flush=True)
PY
done
timeout -k 10 300 python scripts/build_probe.py --scene C3 --repeat 4 > gpurun_out/g_build_C3.txt 2>&1 || { echo "build probe failed"; tail -5 gpurun_out/g_build_C3.txt; exit 1; }
cat gpurun_out/g_build_C3.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/g_buildtrace" -o run -- \
  python3 "$R/scripts/build_probe.py" --scene C3 --repeat 3 > "$R/gpurun_out/g_buildtrace.log" 2>&1 || { echo "build trace failed"; tail -5 "$R/gpurun_out/g_buildtrace.log"; exit 1; }
echo "session g done"
