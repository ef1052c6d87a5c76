# kernel trace of one rank's band (scripts/band_probe.py), plus the same band with one frame in flight
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
N=${N:-8}
timeout -k 10 120 python $R/scripts/band_probe.py --scene C2 --steps 200 --balanced --only-n $N --ahead 0 > $R/gpurun_out/band_ahead0.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/trband -o tb -- python $R/scripts/band_probe.py --scene C2 --steps 100 --balanced --only-n $N --ahead 2 > $R/gpurun_out/trband.log 2>&1
