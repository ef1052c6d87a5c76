"""Per-convolution durations of the denoiser from a rocprofv3 kernel trace (scripts/gpu_dn.sh's
gpurun_out/dn_prof/dn_kernel_trace.csv): each execute is k_dn_input followed by the 16 k_conv3 dispatches in
network order, so the i-th k_conv3 after an input transform is layer i.  Prints / writes the mean and median
ns per layer over the traced executes -- the rocprofv3 side of bench.py's per-layer HIP-event figures
(the kernel-stats CSV pools layers that share a template instance).
    python scripts/dn_trace_layers.py [trace.csv] [out.json]"""
import csv
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NAMES = ["enc_conv0", "enc_conv1", "enc_conv2", "enc_conv3", "enc_conv4", "enc_conv5a", "enc_conv5b", "dec_conv4a",
         "dec_conv4b", "dec_conv3a", "dec_conv3b", "dec_conv2a", "dec_conv2b", "dec_conv1a", "dec_conv1b", "dec_conv0"]
src = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "dn_prof", "dn_kernel_trace.csv")
rows = sorted(csv.DictReader(open(src)), key=lambda r: int(r["Start_Timestamp"]))
per = {n: [] for n in NAMES}
layer = None
for r in rows:
    name = r["Kernel_Name"]
    if "k_dn_input" in name:
        layer = 0
    elif "k_conv3" in name and layer is not None and layer < 16:
        per[NAMES[layer]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        layer += 1
out = {"source": os.path.relpath(src, ROOT), "executes": len(per[NAMES[0]]),
       "layers": {n: {"mean_ns": round(statistics.mean(v), 1), "median_ns": statistics.median(v)} for n, v in per.items() if v}}
print(json.dumps(out, indent=1))
if len(sys.argv) > 2:
    json.dump(out, open(sys.argv[2], "w"), indent=1)
