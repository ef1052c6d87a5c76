"""Where do GPU and oracle frames still differ?  Renders one frame of a workload on the GPU (several kernel
variants) and in the oracle, and reports the differing pixels per stage: G-buffer, the initial pass alone (no
reuse), the full frame; for a few differing pixels the G element and reservoirs on both sides.

  python scripts/parity_probe.py --scene C3 --width 3840 --height 2160 --frame 0
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "restir-embree_amd"), os.path.join(ROOT, "tests")]

import oracle_lib as O  # noqa: E402
from restir_amd import params as P, scenes  # noqa: E402
from restir_amd.renderer import Renderer  # noqa: E402


def workload(name):
    if name == "C3":
        sc = scenes.sponza_like()
        return sc, P.c3_params, lambda f: scenes.orbit_camera(sc.camera, f, 240, 0.3)
    sc = scenes.cornell_many_lights(1024)
    if name == "C2":
        return sc, P.metric_params, lambda f: sc.camera
    return sc, P.c3_params, lambda f: scenes.orbit_camera(sc.camera, f, 240, 0.3)


def gpu_frames(sc, prm, cam, W, H, frames, env=None, trav=None):
    old = {k: os.environ.get(k) for k in (env or {})}
    os.environ.update(env or {})
    try:
        g = Renderer(W, H)
        if trav:
            g.set_traversal(trav)
        gs = g.load_scene(sc)
        out = None
        for f in range(frames + 1):
            out = g.produce_restir(gs, cam(f), prm, f).copy()
        res = (out, g.gbuffer().copy(), g.reservoirs().copy())
        gs.close()
        g.close()
        return res
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="C3")
    ap.add_argument("--width", type=int, default=3840)
    ap.add_argument("--height", type=int, default=2160)
    ap.add_argument("--frame", type=int, default=0)
    a = ap.parse_args()
    sc, prm, cam = workload(a.scene)
    W, H = a.width, a.height
    o, os_ = O.OracleRenderer(W, H), O.OracleScene(sc)
    stages = {"initial_only": prm(do_spatial=0, do_temporal=0), "full": prm()}
    for name, pp in stages.items():
        ref = None
        for f in range(a.frame + 1):
            ref = o.render(os_, cam(f), pp, f)
        rg, rr = o.gbuffer().copy(), o.reservoirs().copy()
        variants = {"default": ({}, None), "unsorted": ({"RESTIR_SORT": "off", "RESTIR_SORT_SPATIAL": "off",
                                                          "RESTIR_SORT_TEMPORAL": "off"}, None),
                    "lockstep": ({}, "lockstep")}
        for vn, (env, trav) in variants.items():
            img, gb, res = gpu_frames(sc, pp, cam, W, H, a.frame, env, trav)
            dpx = np.argwhere(np.any(img != ref, -1))
            dg = np.argwhere(np.any(gb != rg, -1))
            dr = np.argwhere(np.any(res != rr, -1))
            print(f"[{name}/{vn}] frame {a.frame} {W}x{H}: frame px differing {len(dpx)}, G elements {len(dg)}, "
                  f"reservoirs {len(dr)}", flush=True)
            if len(dg):
                ch = np.nonzero(np.any(gb != rg, axis=(0, 1)))[0]
                print(f"    G channels differing: {ch.tolist()}; first px {dg[:4].tolist()}")
            for y, x in dr[:4]:
                print(f"    px ({x},{y}) gpu R {res[y, x].tolist()}\n               ora R {rr[y, x].tolist()}")
                print(f"               G {gb[y, x].tolist()}")
            for y, x in dpx[:4]:
                print(f"    px ({x},{y}) gpu {img[y, x].tolist()} ora {ref[y, x].tolist()}")


if __name__ == "__main__":
    main()
