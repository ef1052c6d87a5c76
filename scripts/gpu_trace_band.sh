set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/trband -o tb -- python $R/scripts/band_probe.py --scene C2 --steps 50 --balanced --only-n 8 --ahead 2 > $R/gpurun_out/trband.log 2>&1
