#!/bin/bash
# Round-5 session L: band bounds from row costs spread over a wave's 8 rows (default) against the whole wave's
# time on its top row (lib_lump), C2's eight bands, interleaved in one session.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do for v in base RESTIR_LIB=restir-embree_amd/_ab/lib_lump.so; do
  envs=""; [ "$v" != base ] && envs="$v"
  tag=$(echo "$v" | tr '/=.' '___')_$r
  env $envs timeout -k 10 400 python scripts/band_probe.py --scene C2 --balanced --all-ranks 8 --steps 150 \
    > gpurun_out/band_all_C2_l_$tag.txt 2>&1 || { echo "band probe $v failed"; tail -5 gpurun_out/band_all_C2_l_$tag.txt; exit 1; }
  python3 - gpurun_out/band_all_C2_l_$tag.txt "$v r$r" <<'PY'
import re, sys
txt = open(sys.argv[1]).read()
t = [float(m.group(1)) for m in re.finditer(r"wall ([0-9.]+) ms/frame", txt)]
rows = [int(m.group(1)) for m in re.finditer(r"rows=(\d+)", txt)]
print(f"{sys.argv[2][-30:]:30s} bands: max {max(t):.4f} mean {sum(t) / len(t):.4f} ms  rows {rows}  {['%.4f' % x for x in t]}", flush=True)
PY
done; done
echo "session l done"
