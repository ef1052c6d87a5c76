"""Summarise rocprofv3 --pmc passes (gpurun_out/pmc_<cfg>_{FETCH_SIZE,WRITE_SIZE,SQ_WAVES}/) into
profiles/<round>_pmc_<cfg>.json (round from $ROUND, default r03): per pass kernel the per-launch mean HBM bytes and SQ counters, and per
frame (one launch of every pass kernel) the HBM bytes and VALU wave-instructions that bench.py reports.
Units and gfx950 correction per MI355X_MICROARCH.md §HBM: FETCH_SIZE/WRITE_SIZE are KiB; FETCH_SIZE
reads 1/2 of a wide streaming read's bytes on gfx950, so hbm_bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024
(the x2 is calibrated for 16-B/lane streaming loads; the uncorrected figure is kept beside it).

    python scripts/pmc_summary.py C2 [W H]"""
import collections
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
cfg = sys.argv[1] if len(sys.argv) > 1 else "C2"
W, H = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (1920, 1080)
src = os.path.join(ROOT, "gpurun_out")
ROUND = os.environ.get("ROUND", "r03")
TAG = os.environ.get("PMC_TAG", "")            # gpu_session.sh pmc PMC_TAG (with its PMC_ENV)
out = os.path.join(ROOT, "profiles", f"{ROUND}_pmc_{cfg}{TAG}.json")
px = W * H
PASS = ("k_gbuffer_initial", "k_visibility", "k_temporal", "k_spatial", "k_shade")


def kname(row):
    # "void rs::k_gbuffer_initial<0>(...)" -> "k_gbuffer_initial" (<0> lockstep / <1> lane kind)
    k = row["Kernel_Name"].split("(")[0].replace("rs::", "").replace("void ", "").split("<")[0]
    return k.replace("_split", "").replace("_sorted", "").replace("_pq", "")


vals = collections.defaultdict(lambda: collections.defaultdict(list))
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    with open(os.path.join(src, f"pmc_{cfg}{TAG}_{c}", "run_counter_collection.csv")) as f:
        for row in csv.DictReader(f):
            k = kname(row)
            if k in PASS:
                vals[k][c].append(float(row["Counter_Value"]))
res = {"config": f"{cfg}_{W}x{H}", "source": f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE / --pmc SQ_* (separate "
       f"runs), RESTIR_RUNAHEAD=0 {os.environ.get('PMC_ENV', '')}, bench.py --scene {cfg} --steps 3 --warmup 1 "
                 f"(scripts/gpu_session.sh pmc)",
       "kernels": {}}
for k, d in vals.items():
    fe = sum(d["FETCH_SIZE"]) / len(d["FETCH_SIZE"])
    wr = sum(d["WRITE_SIZE"]) / len(d["WRITE_SIZE"])
    res["kernels"][k] = {"launches": len(d["FETCH_SIZE"]), "fetch_kib": round(fe, 1), "write_kib": round(wr, 1),
                         "hbm_bytes_corrected": int((2 * fe + wr) * 1024),
                         "hbm_bytes_uncorrected": int((fe + wr) * 1024),
                         "bytes_per_px_corrected": round((2 * fe + wr) * 1024 / px, 2)}
sq_csv = os.path.join(src, f"pmc_{cfg}{TAG}_SQ_WAVES", "run_counter_collection.csv")
if os.path.exists(sq_csv):   # SQ_WAVE_CYCLES / SQ_ACTIVE_INST_* / SQ_WAIT_* are quad-cycles
    sq = collections.defaultdict(lambda: collections.defaultdict(list))
    with open(sq_csv) as f:
        for row in csv.DictReader(f):
            sq[kname(row)][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for k, d in sq.items():
        if k in res["kernels"]:
            res["kernels"][k]["sq"] = {c: round(sum(v) / len(v), 1) for c, v in d.items()}
ta_csv = os.path.join(src, f"pmc_{cfg}{TAG}_SQ_INSTS_VMEM_RD", "run_counter_collection.csv")
if os.path.exists(ta_csv):   # vector-memory pipeline group: per-launch means, and derived ratios
    ta = collections.defaultdict(lambda: collections.defaultdict(list))
    with open(ta_csv) as f:
        for row in csv.DictReader(f):
            ta[kname(row)][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for k, d in ta.items():
        if k not in res["kernels"]:
            continue
        m = {c: sum(v) / len(v) for c, v in d.items()}
        # GRBM_GUI_ACTIVE is summed over the 8 XCDs (MI355X_MICROARCH.md, DVFS item): per-XCD active cycles
        g = max(1.0, m.get("GRBM_GUI_ACTIVE", 0.0) / 8.0)
        res["kernels"][k]["vmem"] = {c: round(v, 1) for c, v in m.items()}
        # TA/TD busy are summed over the 256 CUs' units: per-unit fraction of the kernel's active cycles
        cus = 256.0
        res["kernels"][k]["vmem_derived"] = {
            "ta_busy_frac": round(m.get("TA_TA_BUSY", 0.0) / cus / g, 4),
            "td_busy_frac": round(m.get("TD_TD_BUSY", 0.0) / cus / g, 4),
            "valu_issue_frac": round(m.get("SQ_INSTS_VALU", 0.0) / (1024.0 * g / 2.0), 4),
            "cache_accesses_per_vmem_rd": round(m.get("TCP_TOTAL_CACHE_ACCESSES", 0.0) / max(1.0, m.get("SQ_INSTS_VMEM_RD", 0.0)), 2),
            "tcp_tcc_read_req": m.get("TCP_TCC_READ_REQ"),
            "wait_any_over_wave_cycles": round(m.get("SQ_WAIT_ANY", 0.0) / max(1.0, m.get("SQ_WAVE_CYCLES", 0.0)), 4),
            "note": "busy fractions: TA_TA_BUSY / TD_TD_BUSY / 256 CUs / (GRBM_GUI_ACTIVE / 8 XCDs); VALU issue: "
                    "SQ_INSTS_VALU / (1024 SIMDs x active cycles / 2 cycles per wave64 instruction); cache accesses per "
                    "vector load instruction = TCP_TOTAL_CACHE_ACCESSES / SQ_INSTS_VMEM_RD"}
# one frame = one launch of each pass kernel present
res["frame_bytes"] = sum(v["hbm_bytes_corrected"] for v in res["kernels"].values())
res["frame_valu"] = sum(v.get("sq", {}).get("SQ_INSTS_VALU", 0.0) for v in res["kernels"].values()) or None
res["frame_salu"] = sum(v.get("sq", {}).get("SQ_INSTS_SALU", 0.0) for v in res["kernels"].values()) or None
with open(out, "w") as f:
    json.dump(res, f, indent=1)
print(json.dumps(res, indent=1))
