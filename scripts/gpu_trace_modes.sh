R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tm -o tm -- python $R/scripts/trace_bench_modes.py ${SCENE:-C3} > $R/gpurun_out/tm.log 2>&1 || { tail -5 $R/gpurun_out/tm.log; exit 1; }
python $R/scripts/trace_bench_modes.py --report $R/gpurun_out/tm/tm_kernel_trace.csv
