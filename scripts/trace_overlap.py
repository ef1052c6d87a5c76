"""Analysis of a rocprofv3 --kernel-trace CSV (tooling): per kernel name the launches and mean / median duration,
and over the steady-state window (the last `--window` fraction of the trace) how many kernels run concurrently
(time fractions with >= 1, 2, 3 kernels), the summed kernel time / wall ratio, and per frame-sized window the
kernel time per kernel type.  Usage: python scripts/trace_overlap.py trace.csv [--window 0.8] [--match substr]"""
import argparse
import csv
import statistics
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--window", type=float, default=0.8, help="fraction of the trace (from the end) analysed")
    ap.add_argument("--match", default="", help="only kernels whose name contains this")
    a = ap.parse_args()
    rows = []
    with open(a.csv) as f:
        for r in csv.DictReader(f):
            if a.match and a.match not in r["Kernel_Name"]:
                continue
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], int(r.get("Grid_Size_X", 0) or 0),
                         int(r.get("Grid_Size_Y", 0) or 0), int(r.get("Workgroup_Size_X", 0) or 0)))
    rows.sort()
    t0, t1 = rows[0][0], max(r[1] for r in rows)
    ws = t1 - (t1 - t0) * a.window
    win = [r for r in rows if r[0] >= ws]
    by = defaultdict(list)
    for s, e, n, gx, gy, bx in win:
        short = n.split("(")[0].replace("void ", "")[:60]
        by[(short, gx, gy, bx)].append((e - s) / 1e3)
    wall = (max(r[1] for r in win) - min(r[0] for r in win)) / 1e3
    print(f"window {wall:.1f} us, {len(win)} kernels")
    for k, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        print(f"  {k[0]:60s} grid {k[1]}x{k[2]} wg {k[3]:4d}: n {len(v):5d} mean {statistics.mean(v):8.2f} us "
              f"median {statistics.median(v):8.2f} us  sum {sum(v) / wall:6.3f} x wall")
    ev = []
    for s, e, *_ in win:
        ev.append((s, 1)); ev.append((e, -1))
    ev.sort()
    cur, last, acc = 0, ev[0][0], defaultdict(float)
    for t, d in ev:
        acc[cur] += t - last
        cur += d
        last = t
    tot = sum(acc.values())
    print("concurrency: " + ", ".join(f">={k}: {100 * sum(v for c, v in acc.items() if c >= k) / tot:.1f} %" for k in (1, 2, 3, 4)))


if __name__ == "__main__":
    main()
