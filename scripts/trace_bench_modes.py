"""Diagnostic: isolated BVH query cost per traversal mode (rs_debug_trace) on a scene's primary rays
(closest hit) and one shadow ray per pixel to a random emissive triangle (any hit), 8x8-tile order.
Dispatch order per rep: modes 0 2 (closest: lockstep, per-lane), 1 3 (any hit); one mode-0 dispatch first.
Time with: rocprofv3 --kernel-trace -d gpurun_out/tm -o tm -- python scripts/trace_bench_modes.py C3
then scripts/trace_bench_modes.py --report gpurun_out/tm/tm_kernel_trace.csv"""
import csv
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "restir-embree_amd"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
MODES = (0, 2, 1, 3)
NAMES = {0: "closest lockstep", 2: "closest per-lane", 1: "any lockstep", 3: "any per-lane"}


def report(path):
    rows = [r for r in csv.DictReader(open(path)) if "k_debug_trace" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[1:]                                  # the mode-0 dispatch that finds the shadow-ray origins
    dur = {}
    for i, r in enumerate(rows):
        m = MODES[i % len(MODES)]
        dur.setdefault(m, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    for m in MODES:
        print(f"{NAMES[m]:>18s}: {np.median(dur[m]):8.3f} ms (median of {len(dur[m])})")


def main():
    import torch  # noqa: F401
    from restir_amd import Renderer, scenes
    from trace_bench import primary_rays
    from bvh_stats import shadow_rays
    which = sys.argv[1] if len(sys.argv) > 1 else "C3"
    W, H = 1920, 1080
    sc = scenes.sponza_like() if which == "C3" else scenes.cornell_many_lights(1024)
    r = Renderer(W, H, device=0)
    gs = r.load_scene(sc)
    o, d = primary_rays(sc.camera, W, H)
    t, prim = r._debug_trace(gs, o, d, 0.01, 3.0e38, 0)
    hit = prim >= 0
    p, sd, tf = shadow_rays(sc, o, d, t, hit)
    for rep in range(3):
        for m in MODES:
            if m in (0, 2):
                r._debug_trace(gs, o, d, 0.01, 3.0e38, m)
            else:
                r._debug_trace(gs, p, sd, 0.01, tf, m)
    print(f"rays={o.shape[0]} primary hit={hit.mean():.3f}")


if __name__ == "__main__":
    if sys.argv[1:2] == ["--report"]:
        report(sys.argv[2])
    else:
        main()
