"""Groups the rocprofv3 --pmc rows of scripts/valu_budget.py's initial-pass launches by variant and prints the mean
per launch of every counter (the untimed warm-up launches of each variant skipped).

  python scripts/valu_budget_summary.py gpurun_out/valu_pmc_*/run_counter_collection.csv [--frames 8] [--warmup 2]
"""
import argparse
import collections
import csv
import json
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from valu_budget import VARIANTS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv", nargs="+")
    ap.add_argument("--frames", type=int, default=8)
    ap.add_argument("--warmup", type=int, default=2)
    a = ap.parse_args()
    out = collections.defaultdict(dict)
    for path in a.csv:
        per = collections.defaultdict(lambda: collections.defaultdict(float))   # dispatch -> counter -> value
        order = []
        with open(path) as f:
            for row in csv.DictReader(f):
                if "k_gbuffer" not in row["Kernel_Name"]:
                    continue
                d = int(row["Dispatch_Id"])
                if d not in per:
                    order.append(d)
                per[d][row["Counter_Name"]] += float(row["Counter_Value"])
        order.sort()
        if len(order) != a.frames * len(VARIANTS):
            print(f"{path}: {len(order)} initial-pass launches, expected {a.frames * len(VARIANTS)}", file=sys.stderr)
        for v, (name, _) in enumerate(VARIANTS):
            ds = order[v * a.frames + a.warmup:(v + 1) * a.frames]
            for c in per[ds[0]] if ds else []:
                out[name][c] = sum(per[d][c] for d in ds) / len(ds)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
