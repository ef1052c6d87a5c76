"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (gpurun_out/pmc_*/run_counter_collection.csv)
into profiles/pmc_traffic.json.  Units and gfx950 correction per MI355X_MICROARCH.md §HBM:
FETCH_SIZE/WRITE_SIZE are KiB; FETCH_SIZE reads 1/2 of a wide streaming read's bytes on gfx950, so
hbm_bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (the x2 is calibrated for 16-B/lane streaming loads only;
the uncorrected figure is kept beside it)."""
import collections
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out")
config = sys.argv[2] if len(sys.argv) > 2 else "C2_1920x1080"
out = sys.argv[3] if len(sys.argv) > 3 else os.path.join(ROOT, "profiles", "pmc_traffic.json")
px = 1920 * 1080
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    with open(os.path.join(src, f"pmc_{c}", "run_counter_collection.csv")) as f:
        for row in csv.DictReader(f):
            # "void rs::k_gbuffer_initial<0>(...)" -> "k_gbuffer_initial" (<0> lockstep / <1> lane kind)
            k = row["Kernel_Name"].split("(")[0].replace("rs::", "").replace("void ", "").split("<")[0]
            if k.startswith("k_gbuffer_initial") or k.startswith("k_spatial") or k.startswith("k_temporal") \
                    or k.startswith("k_shade"):
                vals[k][c].append(float(row["Counter_Value"]))
res = {"config": config, "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate runs), "
                                    "bench.py --steps 3 --warmup 1", "kernels": {}}
for k, d in vals.items():
    fe = sum(d["FETCH_SIZE"]) / len(d["FETCH_SIZE"])
    wr = sum(d["WRITE_SIZE"]) / len(d["WRITE_SIZE"])
    res["kernels"][k] = {"launches": len(d["FETCH_SIZE"]), "fetch_kib": round(fe, 1), "write_kib": round(wr, 1),
                         "hbm_bytes_corrected": int((2 * fe + wr) * 1024),
                         "hbm_bytes_uncorrected": int((fe + wr) * 1024),
                         "bytes_per_px_corrected": round((2 * fe + wr) * 1024 / px, 2)}
if "k_gbuffer_initial" in res["kernels"]:
    res["k_gbuffer_initial_bytes_per_launch"] = res["kernels"]["k_gbuffer_initial"]["hbm_bytes_corrected"]
# one frame = one launch of each pass kernel (C2: initial + spatial)
res["frame_bytes"] = sum(v["hbm_bytes_corrected"] for v in res["kernels"].values())
# instruction-issue pass (SQ counters; SQ_WAVE_CYCLES / SQ_ACTIVE_INST_* / SQ_WAIT_* are quad-cycles)
sq_csv = os.path.join(src, "pmc_SQ_WAVES", "run_counter_collection.csv")
if os.path.exists(sq_csv):
    sq = collections.defaultdict(lambda: collections.defaultdict(list))
    with open(sq_csv) as f:
        for row in csv.DictReader(f):
            k = row["Kernel_Name"].split("(")[0].replace("rs::", "").replace("void ", "").split("<")[0]
            sq[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for k, d in sq.items():
        if k in res["kernels"]:
            res["kernels"][k]["sq"] = {c: round(sum(v) / len(v), 1) for c, v in d.items()}
    if "k_gbuffer_initial" in sq:
        g = res["kernels"]["k_gbuffer_initial"]["sq"]
        res["k_gbuffer_initial_valu_per_launch"] = g.get("SQ_INSTS_VALU")
        res["k_gbuffer_initial_salu_per_launch"] = g.get("SQ_INSTS_SALU")
    res["source"] += "; SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY (one run)"
res["traversal"] = os.environ.get("RESTIR_TRAVERSAL", "lockstep")
with open(out, "w") as f:
    json.dump(res, f, indent=1)
print(json.dumps(res, indent=1))
