"""Diagnostic: the initial pass's time at 1080p under parameter variations, to split its cost into
primary ray / area sampling / shadow rays / BRDF ray.  Not a parity test; prints one line per config.
Usage (GPU box): python scripts/initial_breakdown.py [--scene C2|C3] [--frames N]   (RESTIR_LIB selects a variant .so)"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "restir-embree_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=10)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--only", type=int, default=-1, help="run only config #N")
    ap.add_argument("--scene", default="C2")
    a = ap.parse_args()
    import torch
    from restir_amd import Renderer, scenes
    from restir_amd.params import metric_params, c3_params

    torch.cuda.set_stream(torch.cuda.Stream())
    r = Renderer(a.width, a.height, device=0, stream=torch.cuda.current_stream().cuda_stream)
    sc = scenes.sponza_like() if a.scene == "C3" else scenes.cornell_many_lights(1024)
    base = c3_params if a.scene == "C3" else metric_params
    r.set_traversal("lane" if a.scene == "C3" else "lockstep")   # pinned: AUTO's tuning frames alternate kinds
    gs = r.load_scene(sc)
    cfgs = [
        ("A32 B1 (metric)", {}),
        ("A32 B0", dict(m_brdf=0)),
        ("A0 B1", dict(m_area=0)),
        ("A1 B0", dict(m_area=1, m_brdf=0)),
        ("A8 B1", dict(m_area=8)),
        ("A16 B1", dict(m_area=16)),
        ("A32 B1 vis-pass (no shadow rays in initial)", dict(do_visibility_pass=1)),
        ("A32 B0 vis-pass (G-buffer + 32 samples, no rays)", dict(m_brdf=0, do_visibility_pass=1)),
        ("A1 B0 vis-pass (G-buffer + 1 sample)", dict(m_area=1, m_brdf=0, do_visibility_pass=1)),
    ]
    lib = os.path.basename(os.environ.get("RESTIR_LIB", "default"))
    for i, (name, kw) in enumerate(cfgs):
        if a.only >= 0 and i != a.only:
            continue
        prm = base(**kw)
        for f in range(3):
            r.produce_restir(gs, sc.camera, prm, f, copy_out=False, timed=True)
        tot, rays = 0.0, 0
        for f in range(a.frames):
            r.produce_restir(gs, sc.camera, prm, 3 + f, copy_out=False, timed=True)
            tot += r.last_times.gbuffer_initial_ms
            rays += int(r.last_times.rays)
        print(f"{a.scene} {lib:>10s} {name:48s} gbuffer_initial_ms={tot / a.frames:.3f} rays/frame={rays // a.frames}",
              flush=True)


if __name__ == "__main__":
    main()
