#!/bin/bash
# Round-5 session K: band bounds from row costs spread over each wave's 8 rows -- C2's eight 1/8 bands (cost
# balanced, then two rounds of time refinement) and C4's eight bands at 4K, each rank timed alone.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
summ() {
python3 - "$1" "$2" <<'PY'
import re, sys
txt = open(sys.argv[1]).read()
for blk in re.split(r"(?=\[round \d+\])", txt) if "[round" in txt else [txt]:
    t = [float(m.group(1)) for m in re.finditer(r"wall ([0-9.]+) ms/frame", blk)]
    if t:
        print(f"{sys.argv[2]:16s} bands: max {max(t):.4f} mean {sum(t) / len(t):.4f} ms  {['%.4f' % x for x in t]}", flush=True)
PY
}
for rf in 0 2; do
  timeout -k 10 400 python scripts/band_probe.py --scene C2 --balanced --all-ranks 8 --steps 150 --refine $rf \
    > gpurun_out/band_all_C2_k_refine$rf.txt 2>&1 || { echo "C2 band probe refine $rf failed"; tail -5 gpurun_out/band_all_C2_k_refine$rf.txt; exit 1; }
  summ gpurun_out/band_all_C2_k_refine$rf.txt "C2 refine $rf"
done
timeout -k 10 600 python scripts/band_probe.py --scene C3 --width 3840 --height 2160 --balanced --all-ranks 8 --steps 12 --refine 2 \
  > gpurun_out/band_all_C4_k.txt 2>&1 || { echo "C4 band probe failed"; tail -5 gpurun_out/band_all_C4_k.txt; exit 1; }
summ gpurun_out/band_all_C4_k.txt "C4 refine 2"
echo "session k done"
