"""Probe for the queued initial pass: C3 shadow rays (G-buffer positions -> area samples on the lamps)
traced in pixel-tile order (what the initial pass does now) vs sorted by target cell within 16x16-pixel
tiles, with the lockstep and the per-lane walk (rs_debug_trace modes 1 / 3).  Run under
rocprofv3 --kernel-trace: the k_debug_trace durations, in call order, are the answer.
    python scripts/sorted_rays_probe.py [W H cand]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "restir-embree_amd")]
import numpy as np

from restir_amd import params as P, scenes
from restir_amd.renderer import Renderer

W, H, A = (int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (960, 540, 8)
sc = scenes.sponza_like()
r = Renderer(W, H)
s = r.load_scene(sc)
r.set_traversal("lane")
r.produce_restir(s, sc.camera, P.c3_params(), 0)
g = r.gbuffer()
pos = g[..., 0:3].reshape(-1, 3)
valid = (g[..., 12:15].max(-1) <= 0).reshape(-1) & (np.abs(pos).sum(-1) > 0)
rng = np.random.default_rng(1)
em = np.nonzero(sc.emissive_mask())[0]
tri = sc.positions[em].reshape(-1, 3, 3).astype(np.float64)
area = 0.5 * np.linalg.norm(np.cross(tri[:, 1] - tri[:, 0], tri[:, 2] - tri[:, 0]), axis=1)
cdf = np.cumsum(area) / area.sum()
n_px = W * H
# rays in the initial pass's order: 8x8 tiles, candidate-major within a tile (a wave = one candidate of
# 64 pixels)
ty, tx = np.meshgrid(np.arange(H // 8), np.arange(W // 8), indexing="ij")
ly, lx = np.meshgrid(np.arange(8), np.arange(8), indexing="ij")
px = ((ty.reshape(-1, 1) * 8 + ly.reshape(1, -1)) * W + (tx.reshape(-1, 1) * 8 + lx.reshape(1, -1)))   # (tiles, 64)
pix = np.repeat(px[:, None, :], A, axis=1).reshape(-1)                   # tile, cand, lane
k = np.searchsorted(cdf, rng.random(pix.size))
k = np.minimum(k, len(em) - 1)
r1, r2 = rng.random(pix.size), rng.random(pix.size)
sr = np.sqrt(r1)
b = np.stack([1 - sr, sr * (1 - r2), sr * r2], 1)
tgt = (tri[k] * b[:, :, None]).sum(1)
o = pos[pix].astype(np.float64)
d = tgt - o
dist = np.linalg.norm(d, axis=1)
keep = valid[pix] & (dist > 0.02)
o, d, dist, tgt, pix = o[keep], d[keep], dist[keep], tgt[keep], pix[keep]
d /= dist[:, None]
tn = np.full(len(o), np.float32(np.finfo(np.float32).tiny + 0.01), np.float32)
tf = (dist - 0.001).astype(np.float32)
print(f"{len(o)} rays", flush=True)
# sorted: within 16x16 pixel tiles by a 5-bit-per-axis Morton code of the target
lo, hi = sc.positions.reshape(-1, 3).min(0), sc.positions.reshape(-1, 3).max(0)
q = np.clip(((tgt - lo) / (hi - lo) * 32).astype(np.int64), 0, 31)
def part1by2(v):
    v = v & 0x3FF
    v = (v | (v << 16)) & 0x030000FF
    v = (v | (v << 8)) & 0x0300F00F
    v = (v | (v << 4)) & 0x030C30C3
    v = (v | (v << 2)) & 0x09249249
    return v
morton = part1by2(q[:, 0]) | (part1by2(q[:, 1]) << 1) | (part1by2(q[:, 2]) << 2)
tile16 = (pix // W // 16) * ((W + 15) // 16) + (pix % W) // 16
order_sorted = np.lexsort((morton, tile16))
orders = {"pixel_tile": np.arange(len(o)), "sorted16": order_sorted}
for name, idx in orders.items():
    for mode_name, lockstep in (("lockstep", True), ("lane", False)):
        for rep in range(2):
            t0 = time.perf_counter()
            _, occ = r.debug_trace(s, o[idx].astype(np.float32), d[idx].astype(np.float32), tn[idx], tf[idx],
                                   any_hit=True, lockstep=lockstep)
            print(f"{name:10s} {mode_name:8s} rep {rep}: wall {1e3 * (time.perf_counter() - t0):.1f} ms, "
                  f"occluded {occ.mean():.3f}", flush=True)
