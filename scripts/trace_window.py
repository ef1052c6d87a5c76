"""Per-kernel average durations over the TIMED frames of a bench.py run, from a rocprofv3 kernel trace
(rocprofv3 --kernel-trace --stats ... -- python bench.py --steps K ...).  The --stats summary averages every
launch, including the traversal-tuning frames (which run alone, without frames in flight, and so are
shorter); the last K launches of a pass kernel are the timed frames', which bench.py's HIP-event
`roofline.kernel_ms` measures.  Usage: python scripts/trace_window.py TRACE.csv K [OUT.json]"""
import csv
import json
import sys
from collections import defaultdict


def main():
    path, k = sys.argv[1], int(sys.argv[2])
    rows = list(csv.DictReader(open(path)))
    by = defaultdict(list)
    for r in sorted(rows, key=lambda r: int(r["Start_Timestamp"])):
        name = r["Kernel_Name"]
        if not name.startswith("void rs::k_") and not name.startswith("rs::k_reduce"):
            continue
        by[name.split("(")[0]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    out = {}
    for name, d in by.items():
        last = d[-k:]
        out[name] = {"launches": len(d), "timed_launches": len(last), "timed_avg_ms": round(sum(last) / len(last), 4),
                     "all_avg_ms": round(sum(d) / len(d), 4)}
    res = {"trace": path, "timed_frames": k, "kernels": out}
    print(json.dumps(res, indent=1))
    if len(sys.argv) > 3:
        json.dump(res, open(sys.argv[3], "w"), indent=1)


if __name__ == "__main__":
    main()
