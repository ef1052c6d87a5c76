"""Diagnostic (GPU box): wall time of rs_debug_trace per-lane queries (modes 2 closest / 3 any-hit) on C3's
primary rays and one shadow ray per pixel (scripts/bvh_stats.py's ray set), with the scene's current
walk (8-wide by default, RESTIR_WIDE=off: skip pointers).  Host copies included; compare like with like."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "restir-embree_amd"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
from trace_bench import primary_rays  # noqa: E402
from bvh_stats import shadow_rays  # noqa: E402


def main():
    import torch  # noqa: F401
    from restir_amd import Renderer, scenes
    W, H = 1920, 1080
    sc = scenes.sponza_like()
    r = Renderer(W, H, device=0)
    gs = r.load_scene(sc)
    o, d = primary_rays(sc.camera, W, H)
    t, prim = r.debug_trace(gs, o, d, 0.01, 3.0e38, any_hit=False)
    so, sd, tf = shadow_rays(sc, o, d, t, prim >= 0)
    for name, args in (("primary closest", (o, d, 0.01, 3.0e38, False)), ("shadow any", (so, sd, 0.01, tf, True))):
        for mode in ("lockstep", "lane"):
            ts = []
            for _ in range(4):
                t0 = time.perf_counter()
                r.debug_trace(gs, *args[:4], any_hit=args[4], lockstep=(mode == "lockstep"))
                ts.append(time.perf_counter() - t0)
            print(f"{os.environ.get('RESTIR_WIDE', 'wide'):5s} {name:16s} {mode:8s} {1e3 * min(ts[1:]):8.2f} ms", flush=True)


def wide_stats():
    import torch  # noqa: F401
    from restir_amd import Renderer, scenes
    W, H = 1920, 1080
    sc = scenes.sponza_like()
    r = Renderer(W, H, device=0)
    gs = r.load_scene(sc)
    o, d = primary_rays(sc.camera, W, H)
    t, prim = r.debug_trace(gs, o, d, 0.01, 3.0e38, any_hit=False)
    so, sd, tf = shadow_rays(sc, o, d, t, prim >= 0)
    for name, args in (("primary", (o, d, 0.01, 3.0e38, False, np.ones(len(o), bool))), ("shadow", (so, sd, 0.01, tf, True, prim >= 0))):
        t0 = time.perf_counter()
        f, tr, lost = r.debug_trace(gs, *args[:4], any_hit=args[4], wide_stats=True)
        t1 = time.perf_counter()
        f, tr, lost = r.debug_trace(gs, *args[:4], any_hit=args[4], wide_stats=True)
        print(f"stats query {1e3 * (time.perf_counter() - t1):.2f} ms (first {1e3 * (t1 - t0):.2f})")
        a = args[5]
        wf = np.where(a, f, 0)[: (f.size // 64) * 64].reshape(-1, 64).max(1)
        print(f"max fetches {f[a].max()}, max tris {tr[a].max()}")
        for mode in (8, 9, 10):
            ts = []
            for _ in range(3):
                t0 = time.perf_counter()
                r._debug_trace(gs, *args[:4], mode)
                ts.append(time.perf_counter() - t0)
            print(f"  mode {mode}: {1e3 * min(ts[1:]):.2f} ms")
        print(f"wide {name:8s} fetches mean={f[a].mean():6.2f} p95={np.percentile(f[a], 95):5.0f} wave-max={wf.mean():6.1f} "
              f"tris={tr[a].mean():5.2f} lost={float((lost[a] > 0).mean()):.5f}", flush=True)


if __name__ == "__main__":
    wide_stats() if "--stats" in sys.argv else main()
