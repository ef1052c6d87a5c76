"""Summarise per-dispatch SQ counters of one kernel from rocprofv3 --pmc CSV directories.
Usage: python scripts/pmc_table.py gpurun_out/diag3 [kernel-substring]"""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
kname = sys.argv[2] if len(sys.argv) > 2 else "k_gbuffer_initial"
rows = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(root, "c*_p*", "**", "*counter_collection.csv"), recursive=True):
    cfg = os.path.relpath(f, root).split(os.sep)[0].split("_")[0]
    for r in csv.DictReader(open(f)):
        if kname in r["Kernel_Name"]:
            rows[cfg][r["Counter_Name"]].append(float(r["Counter_Value"]))
names = sorted({n for c in rows.values() for n in c})
print("cfg " + " ".join(f"{n[3:]:>16s}" for n in names) + "   valu/wave")
for cfg in sorted(rows, key=lambda c: int(c[1:])):
    v = {n: sum(x) / len(x) for n, x in rows[cfg].items()}
    print(f"{cfg:3s} " + " ".join(f"{v.get(n, 0):16.4g}" for n in names) +
          f"   {v.get('SQ_INSTS_VALU', 0) / max(1, v.get('SQ_WAVES', 1)):9.0f}")
