"""Per-layer SQ counters of the denoiser from a rocprofv3 --pmc run of scripts/bench_denoise.py
(csrc/rs_denoise.hip): the execute's dispatches in order are [AE bins, AE final, input transform, 16
convolutions], so conv dispatches are assigned to layers by their position in that sequence.  Prints per layer
the mean over executes of: duration, effective clock (GRBM_GUI_ACTIVE / 8 XCDs / duration), MFMA busy
(SQ_VALU_MFMA_BUSY_CYCLES / (CUs x 4 SIMDs x GRBM/8)), LDS waits per wave-cycle, LDS bank conflicts per LDS
instruction.

    python scripts/dn_pmc_layers.py gpurun_out/f_dnpmc_1/run_counter_collection.csv [--json out.json]"""
import collections
import csv
import json
import sys

LAYERS = ["enc_conv0", "enc_conv1", "enc_conv2", "enc_conv3", "enc_conv4", "enc_conv5a", "enc_conv5b", "dec_conv4a",
          "dec_conv4b", "dec_conv3a", "dec_conv3b", "dec_conv2a", "dec_conv2b", "dec_conv1a", "dec_conv1b", "dec_conv0"]
CUS = 256


def main():
    path = sys.argv[1]
    disp = collections.OrderedDict()
    for row in csv.DictReader(open(path)):
        d = disp.setdefault(int(row["Dispatch_Id"]), {"name": row["Kernel_Name"], "t0": int(row["Start_Timestamp"]),
                                                     "t1": int(row["End_Timestamp"]), "c": {}})
        d["c"][row["Counter_Name"]] = d["c"].get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
    seq = [d for _, d in sorted(disp.items()) if "k_conv3" in d["name"]]
    if len(seq) % 16:
        sys.exit(f"{len(seq)} convolution dispatches: not a multiple of 16")
    per = collections.defaultdict(list)
    for i, d in enumerate(seq[16:]):           # skip the first execute (code loading)
        per[LAYERS[i % 16]].append(d)
    out = {}
    for name in LAYERS:
        ds = per[name]
        m = lambda k: sum(d["c"].get(k, 0.0) for d in ds) / len(ds)   # noqa: E731
        dur = sum(d["t1"] - d["t0"] for d in ds) / len(ds) * 1e-9
        grbm = m("GRBM_GUI_ACTIVE") / 8
        o = {"kernel": ds[0]["name"].split("(")[0].replace("void ", ""), "us": round(dur * 1e6, 2),
             "clock_ghz": round(grbm / dur / 1e9, 3) if dur else None,
             "mfma_busy": round(m("SQ_VALU_MFMA_BUSY_CYCLES") / (CUS * 4 * grbm), 4) if grbm else None,
             "lds_wait_over_wave_cycles": round(m("SQ_WAIT_INST_LDS") / m("SQ_WAVE_CYCLES"), 4) if m("SQ_WAVE_CYCLES") else None,
             "wait_any_over_wave_cycles": round(m("SQ_WAIT_ANY") / m("SQ_WAVE_CYCLES"), 4) if m("SQ_WAVE_CYCLES") else None,
             "lds_conflict_per_lds_instr": round(m("SQ_LDS_BANK_CONFLICT") / m("SQ_INSTS_LDS"), 4) if m("SQ_INSTS_LDS") else None,
             "waves": m("SQ_WAVES")}
        out[name] = o
        print(f"{name:11s} {o['kernel'][:40]:40s} {o['us']:8.2f} us  clk {o['clock_ghz']}  mfma {o['mfma_busy']}  "
              f"ldswait {o['lds_wait_over_wave_cycles']}  waitany {o['wait_any_over_wave_cycles']}  "
              f"conf/lds {o['lds_conflict_per_lds_instr']}")
    if "--json" in sys.argv:
        json.dump(out, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
