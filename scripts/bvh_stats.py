"""Diagnostic: BVH walk statistics on the GPU BVHs (rs_debug_trace stats modes: the skip-pointer walk's node
visits and the 8-wide walk's node fetches) for the scenes' primary
rays (closest hit) and one shadow ray per pixel to a random point on a random emissive triangle
(any hit), in 8x8-tile (wave) order.  Prints mean / p95 node visits and triangle tests per ray and
the per-wave maximum (what a per-lane walk pays).  Usage (GPU box): python scripts/bvh_stats.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "restir-embree_amd"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))


def primary_rays(cam, W, H):
    """Camera rays of a W x H frame in the kernels' wave order (8x8 tiles, row-major within a tile, tiles row-major)."""
    eye, at, fov = np.array(cam.eye, np.float64), np.array(cam.at, np.float64), cam.fov_y
    fwd = at - eye
    fwd /= np.linalg.norm(fwd)
    up = np.array([0.0, 0.0, 1.0])
    right = np.cross(fwd, up)
    right /= np.linalg.norm(right)
    upv = np.cross(right, fwd)
    focal = (H / 2.0) / np.tan(np.radians(fov) / 2.0)
    ty, tx, iy, ix = np.meshgrid(np.arange(H // 8), np.arange(W // 8), np.arange(8), np.arange(8), indexing="ij")
    x = (tx * 8 + ix).ravel().astype(np.float64)
    y = (ty * 8 + iy).ravel().astype(np.float64)
    d = (x - W / 2)[:, None] * right + (H / 2 - y)[:, None] * upv + focal * fwd
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    o = np.broadcast_to(eye, d.shape)
    return o.astype(np.float32), d.astype(np.float32)


def shadow_rays(sc, o, d, t, hit, seed=1):
    n = o.shape[0]
    p = o + d * np.where(hit, t, 0.0)[:, None]
    tri_p = np.asarray(sc.positions, np.float64).reshape(-1, 3, 3)
    emis = np.nonzero(sc.emissive_mask())[0]
    rng = np.random.default_rng(seed)
    e = emis[rng.integers(0, len(emis), n)]
    r1, r2 = rng.random(n), rng.random(n)
    sr = np.sqrt(r1)
    q = tri_p[e, 0] * (1 - sr)[:, None] + tri_p[e, 1] * (sr * (1 - r2))[:, None] + tri_p[e, 2] * (sr * r2)[:, None]
    sd = q - p
    dist = np.linalg.norm(sd, axis=1)
    sd = sd / np.maximum(dist, 1e-20)[:, None]
    return p.astype(np.float32), sd.astype(np.float32), np.where(hit, dist - 0.001, -1.0).astype(np.float32)


def report_wide(name, fetches, tris, lost, active):
    f, tr = fetches[active], tris[active]
    wf = np.where(active, fetches, 0)[: (fetches.size // 64) * 64].reshape(-1, 64).max(1)
    print(f"  {name:8s} rays={active.sum():8d} 8-wide node fetches mean={f.mean():6.1f} p95={np.percentile(f, 95):6.0f} "
          f"wave-max mean={wf.mean():6.1f} | tri tests mean={tr.mean():5.2f} | stack overflows {int((lost[active] > 0).sum())}")


def report(name, visits, tris, active):
    v, tr = visits[active], tris[active]
    wv = np.where(active, visits, 0)[: (visits.size // 64) * 64].reshape(-1, 64).max(1)
    print(f"  {name:8s} rays={active.sum():8d} visits mean={v.mean():6.1f} p95={np.percentile(v, 95):6.0f} "
          f"wave-max mean={wv.mean():6.1f} | tri tests mean={tr.mean():5.2f} p95={np.percentile(tr, 95):4.0f}")


def main():
    import torch  # noqa: F401
    from restir_amd import Renderer, scenes

    W, H = 1920, 1080
    for name, sc in (("C2", scenes.cornell_many_lights(1024)), ("C3", scenes.sponza_like())):
        r = Renderer(W, H, device=0)
        gs = r.load_scene(sc)
        o, d = primary_rays(sc.camera, W, H)
        t, prim = r.debug_trace(gs, o, d, 0.01, 3.0e38, any_hit=False)
        hit = prim >= 0
        print(f"{name}: {sc.n_tris} tris, primary hit {hit.mean():.3f}")
        vis, tri = r.debug_trace(gs, o, d, 0.01, 3.0e38, any_hit=False, stats=True)
        report("primary", vis, tri, np.ones_like(hit))
        so, sd, tf = shadow_rays(sc, o, d, t, hit)
        vis, tri = r.debug_trace(gs, so, sd, 0.01, tf, any_hit=True, stats=True)
        report("shadow", vis, tri, hit)
        fe, tr, lost = r.debug_trace(gs, o, d, 0.01, 3.0e38, any_hit=False, wide_stats=True)
        report_wide("primary", fe, tr, lost, np.ones_like(hit))
        fe, tr, lost = r.debug_trace(gs, so, sd, 0.01, tf, any_hit=True, wide_stats=True)
        report_wide("shadow", fe, tr, lost, hit)


if __name__ == "__main__":
    main()
