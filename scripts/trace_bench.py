"""Diagnostic: isolated BVH query cost on C2 1080p through rs_debug_trace -- primary rays (closest hit)
and one shadow ray per pixel (any hit) to a random point on a random emissive triangle, in 8x8-tile
order (the pass kernels' wave shape), lockstep and per-lane.  Time it with
  rocprofv3 --kernel-trace --stats -d gpurun_out/tb -o tb -- python scripts/trace_bench.py
(k_debug_trace dispatches in order: for rep: closest-lockstep, closest-lane, any-lockstep, any-lane)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "restir-embree_amd"))


def primary_rays(cam, W, H):
    eye, at, fov = np.array(cam.eye, np.float64), np.array(cam.at, np.float64), cam.fov_y
    fwd = at - eye
    fwd /= np.linalg.norm(fwd)
    up = np.array([0.0, 0.0, 1.0])
    right = np.cross(fwd, up)
    right /= np.linalg.norm(right)
    upv = np.cross(right, fwd)
    focal = (H / 2.0) / np.tan(np.radians(fov) / 2.0)
    # 8x8 tiles, row-major within a tile, tiles row-major (wave = one tile)
    ty, tx, iy, ix = np.meshgrid(np.arange(H // 8), np.arange(W // 8), np.arange(8), np.arange(8), indexing="ij")
    x = (tx * 8 + ix).ravel().astype(np.float64)
    y = (ty * 8 + iy).ravel().astype(np.float64)
    d = (x - W / 2)[:, None] * right + (H / 2 - y)[:, None] * upv + focal * fwd
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    o = np.broadcast_to(eye, d.shape)
    return o.astype(np.float32), d.astype(np.float32)


def main():
    import torch  # noqa: F401  (HIP runtime init as in the product)
    from restir_amd import Renderer, scenes

    W, H = 1920, 1080
    sc = scenes.cornell_many_lights(1024)
    r = Renderer(W, H, device=0)
    gs = r.load_scene(sc)
    o, d = primary_rays(sc.camera, W, H)
    n = o.shape[0]
    t, prim = r.debug_trace(gs, o, d, 0.01, 3.0e38, any_hit=False)
    hit = prim >= 0
    p = o + d * np.where(hit, t, 0.0)[:, None]
    tri_p = np.asarray(sc.positions, np.float64).reshape(-1, 3, 3)
    emis = np.nonzero(sc.emissive_mask())[0]
    rng = np.random.default_rng(1)
    e = emis[rng.integers(0, len(emis), n)]
    r1, r2 = rng.random(n), rng.random(n)
    sr = np.sqrt(r1)
    q = (tri_p[e, 0] * (1 - sr)[:, None] + tri_p[e, 1] * (sr * (1 - r2))[:, None] + tri_p[e, 2] * (sr * r2)[:, None])
    sd = q - p
    dist = np.linalg.norm(sd, axis=1)
    sd = sd / np.maximum(dist, 1e-20)[:, None]
    sdir = sd.astype(np.float32)
    tfar = np.where(hit, dist - 0.001, -1.0).astype(np.float32)
    for rep in range(3):
        r.debug_trace(gs, o, d, 0.01, 3.0e38, any_hit=False, lockstep=True)
        r.debug_trace(gs, o, d, 0.01, 3.0e38, any_hit=False, lockstep=False)
        r.debug_trace(gs, p.astype(np.float32), sdir, 0.01, tfar, any_hit=True, lockstep=True)
        r.debug_trace(gs, p.astype(np.float32), sdir, 0.01, tfar, any_hit=True, lockstep=False)
    print(f"rays={n} primary hit={hit.mean():.3f}")


if __name__ == "__main__":
    main()
