"""Summarise the denoiser's rocprofv3 --pmc passes (scripts/gpu_dn_pmc.sh: gpurun_out/dnpmc_{1..4}/) into
profiles/<round>_pmc_denoise.json: per convolution (dispatches mapped to layers by their order inside each
execute: auto-exposure bins, auto-exposure final, input transform, the 16 convolutions) the per-launch
mean HBM bytes (gfx950 FETCH_SIZE correction as scripts/pmc_summary.py: (2 FETCH + WRITE) KiB), the SQ /
vector-memory counters, and derived fractions:
  mfma_busy_frac   = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs)
  valu_issue_frac  = SQ_INSTS_VALU / (1024 SIMDs x active cycles / 2)
  ta / td busy     = TA_TA_BUSY, TD_TD_BUSY / 256 CUs / active cycles
  lds_conflict_per_lds_instr = SQ_LDS_BANK_CONFLICT / SQ_INSTS_LDS (extra LDS cycles per LDS instruction)
    python scripts/dn_pmc_summary.py [W H]"""
import collections
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
W, H = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (1920, 1080)
ROUND = os.environ.get("ROUND", "r03")
LAYERS = ["enc_conv0", "enc_conv1", "enc_conv2", "enc_conv3", "enc_conv4", "enc_conv5a", "enc_conv5b",
          "dec_conv4a", "dec_conv4b", "dec_conv3a", "dec_conv3b", "dec_conv2a", "dec_conv2b",
          "dec_conv1a", "dec_conv1b", "dec_conv0"]
NAMES = ["ae_bins", "ae_final", "input_transform"] + LAYERS


def per_layer(i):
    rows = list(csv.DictReader(open(os.path.join(ROOT, "gpurun_out", f"dnpmc_{i}", "run_counter_collection.csv"))))
    disp = collections.OrderedDict()
    for r in rows:
        d = disp.setdefault(int(r["Dispatch_Id"]), {"name": r["Kernel_Name"], "grid": int(r["Grid_Size"]), "c": {}})
        d["c"][r["Counter_Name"]] = float(r["Counter_Value"])
    seq = [d for _, d in sorted(disp.items()) if "rs::dn::" in d["name"]]
    starts = [k for k, d in enumerate(seq) if "k_dn_ae_bins" in d["name"]]
    execs = [seq[s:s + len(NAMES)] for s in starts if s + len(NAMES) <= len(seq)][-3:]   # after warm-up
    out = {}
    for j, n in enumerate(NAMES):
        ds = [e[j] for e in execs]
        out[n] = {"kernel": ds[0]["name"].split("(")[0].replace("void ", ""), "grid": ds[0]["grid"],
                  **{c: sum(d["c"].get(c, 0.0) for d in ds) / len(ds) for c in ds[0]["c"]}}
    return out


res = {"config": f"denoise_{W}x{H}", "source": "rocprofv3 --pmc, four separate runs of scripts/denoise_probe.py "
       "(--iters 3: 3 warm-up + 3 timed executes; the last 3 executes averaged), scripts/gpu_dn_pmc.sh", "layers": {}}
passes = [per_layer(i) for i in (1, 2, 3, 4)]
tot = 0
for n in NAMES:
    m = {}
    for p in passes:
        m.update({k: v for k, v in p[n].items()})
    fe, wr = m.get("FETCH_SIZE", 0.0), m.get("WRITE_SIZE", 0.0)
    g = max(1.0, m.get("GRBM_GUI_ACTIVE", 0.0) / 8.0)
    lay = {"kernel": m["kernel"], "grid": m["grid"], "fetch_kib": round(fe, 1), "write_kib": round(wr, 1),
           "hbm_bytes_corrected": int((2 * fe + wr) * 1024), "hbm_bytes_uncorrected": int((fe + wr) * 1024),
           "counters": {k: round(v, 1) for k, v in m.items() if k.isupper()}}
    lay["derived"] = {
        "active_cycles_per_xcd": round(g, 1),
        "mfma_busy_frac": round(m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (1024.0 * g), 4),
        "valu_issue_frac": round(m.get("SQ_INSTS_VALU", 0.0) / (1024.0 * g / 2.0), 4),
        "ta_busy_frac": round(m.get("TA_TA_BUSY", 0.0) / 256.0 / g, 4),
        "td_busy_frac": round(m.get("TD_TD_BUSY", 0.0) / 256.0 / g, 4),
        "lds_conflict_per_lds_instr": round(m.get("SQ_LDS_BANK_CONFLICT", 0.0) / max(1.0, m.get("SQ_INSTS_LDS", 0.0)), 3),
        "wait_any_over_wave_cycles": round(m.get("SQ_WAIT_ANY", 0.0) / max(1.0, m.get("SQ_WAVE_CYCLES", 0.0)), 4),
        "hbm_gbs_at_active_cycles": round((2 * fe + wr) * 1024 / (g / 2.4e9) / 1e9, 1)}
    tot += lay["hbm_bytes_corrected"]
    res["layers"][n] = lay
res["execute_hbm_bytes_corrected"] = tot
out = os.path.join(ROOT, "profiles", f"{ROUND}_pmc_denoise.json")
with open(out, "w") as f:
    json.dump(res, f, indent=1)
for n, l in res["layers"].items():
    d = l["derived"]
    print(f"{n:16s} {l['hbm_bytes_corrected']/1e6:8.1f} MB  mfma {d['mfma_busy_frac']:.3f} valu {d['valu_issue_frac']:.3f} "
          f"ta {d['ta_busy_frac']:.3f} td {d['td_busy_frac']:.3f} ldsconf {d['lds_conflict_per_lds_instr']:.2f} "
          f"wait {d['wait_any_over_wave_cycles']:.3f} {d['hbm_gbs_at_active_cycles']:.0f} GB/s")
print("execute HBM MB", tot / 1e6)
