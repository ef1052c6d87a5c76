"""Which occlusion (any-hit) rays does the GPU answer differently from the oracle?  Renders one initial-pass-only
frame of a workload on both, takes the pixels whose reservoirs differ, records every shadow ray the oracle traces
from those pixels' surface points (or_record_rays), traces them again on the GPU (lockstep and per-lane walks)
and in the oracle (binary and 8-wide trees), and for each disagreement lists the triangles Moller-Trumbore accepts
on the segment (brute force over the scene, the kernels' float operation order) and where the hit point lies
relative to each such triangle's box.

  python scripts/anyhit_probe.py --scene C3 --width 3840 --height 2160
"""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "restir-embree_amd"), os.path.join(ROOT, "tests")]

import oracle_lib as O  # noqa: E402
from restir_amd import params as P, scenes  # noqa: E402
from restir_amd.renderer import Renderer  # noqa: E402

F = np.float32


def mt_all(pos, o, d, tnear, tfar):
    """Moller-Trumbore (rs_scene.h tri_test's operation order) of one ray against every triangle: accepted mask, t."""
    v0, v1, v2 = pos[:, 0:3], pos[:, 3:6], pos[:, 6:9]
    e1, e2 = (v1 - v0).astype(F), (v2 - v0).astype(F)

    def cross(a, b):
        return np.stack([a[..., 1] * b[..., 2] - b[..., 1] * a[..., 2], a[..., 2] * b[..., 0] - b[..., 2] * a[..., 0],
                         a[..., 0] * b[..., 1] - b[..., 0] * a[..., 1]], -1).astype(F)

    def dot(a, b):
        t = (a * b).astype(F)
        return ((t[..., 0] + t[..., 1]).astype(F) + t[..., 2]).astype(F)

    dd = np.broadcast_to(d, e2.shape).astype(F)
    p = cross(dd, e2)
    det = dot(e1, p)
    with np.errstate(all="ignore"):
        inv = (F(1) / det).astype(F)
        sv = (o - v0).astype(F)
        u = (dot(sv, p) * inv).astype(F)
        q = cross(sv, e1)
        v = (dot(dd, q) * inv).astype(F)
        t = (dot(e2, q) * inv).astype(F)
        ok = (det != 0) & (u >= 0) & (u <= 1) & (v >= 0) & ((u + v).astype(F) <= 1) & (t >= tnear) & (t <= tfar)
    return ok, t, u, v


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="C3")
    ap.add_argument("--width", type=int, default=3840)
    ap.add_argument("--height", type=int, default=2160)
    ap.add_argument("--frame", type=int, default=0)
    a = ap.parse_args()
    W, H = a.width, a.height
    if a.scene == "C3":
        sc = scenes.sponza_like()
        cam = scenes.orbit_camera(sc.camera, a.frame, 240, 0.3)
        prm = P.c3_params(do_spatial=0, do_temporal=0)
    else:
        sc = scenes.cornell_many_lights(1024)
        cam = scenes.orbit_camera(sc.camera, a.frame, 240, 0.3)
        prm = P.metric_params(do_spatial=0)
    g = Renderer(W, H)
    gs = g.load_scene(sc)
    g.produce_restir(gs, cam, prm, a.frame)
    rg, gg = g.reservoirs().copy(), g.gbuffer().copy()
    L = O.lib()
    L.or_record_rays.argtypes = [ctypes.c_int, O._f32p, O._f32p, ctypes.c_int]
    L.or_recorded_rays.restype = ctypes.c_int
    o = O.OracleRenderer(W, H)
    osw, osb = O.OracleScene(sc, wide=True), O.OracleScene(sc, wide=False)
    o.render(osw, cam, prm, a.frame)
    ro, go = o.reservoirs().copy(), o.gbuffer().copy()
    dpx = np.argwhere(np.any(rg != ro, -1))
    print(f"{a.scene} {W}x{H} frame {a.frame} initial only: reservoirs differ at {len(dpx)} px, G at "
          f"{int(np.any(gg != go, -1).sum())} px", flush=True)
    if not len(dpx):
        return
    pts = np.ascontiguousarray(np.stack([go[y, x, 0:3] for y, x in dpx[:16]]), F)
    cap = 4096
    buf = np.zeros((cap, 9), F)
    L.or_record_rays(len(pts), O._ptr(pts), O._ptr(buf), cap)
    o.render(osw, cam, prm, a.frame)
    n = min(cap, L.or_recorded_rays())
    L.or_record_rays(0, O._ptr(pts), O._ptr(buf), cap)
    rays = buf[:n]
    org, dirs = np.ascontiguousarray(rays[:, 0:3]), np.ascontiguousarray(rays[:, 3:6])
    tn, tf, res = np.ascontiguousarray(rays[:, 6]), np.ascontiguousarray(rays[:, 7]), rays[:, 8].astype(int)
    out = {"ora_wide_rec": res, "ora_wide": np.asarray(osw.trace_any(org, dirs, tn, tf)).astype(int),
           "ora_bin": np.asarray(osb.trace_any(org, dirs, tn, tf)).astype(int),
           "gpu_lockstep": g.debug_trace(gs, org, dirs, tn, tf, any_hit=True, lockstep=True)[1].astype(int),
           "gpu_lane": g.debug_trace(gs, org, dirs, tn, tf, any_hit=True, lockstep=False)[1].astype(int)}
    print(f"{n} shadow rays recorded from {len(pts)} pixels; occluded: " +
          ", ".join(f"{k} {int(v.sum())}" for k, v in out.items()), flush=True)
    ref = out["ora_bin"]
    bad = sorted({int(i) for k, v in out.items() for i in np.nonzero(v != ref)[0]})
    pos = sc.positions.astype(F)
    for i in bad[:8]:
        print(f"  ray {i}: " + " ".join(f"{k}={int(v[i])}" for k, v in out.items()) +
              f" o={org[i].tolist()} d={dirs[i].tolist()} tnear={float(tn[i])!r} tfar={float(tf[i])!r}")
        ok, t, u, v = mt_all(pos, org[i], dirs[i], tn[i], tf[i])
        for k in np.nonzero(ok)[0][:6]:
            tri = pos[k].reshape(3, 3)
            lo, hi = tri.min(0), tri.max(0)
            ph = (org[i] + dirs[i] * t[k]).astype(F)
            out_by = np.maximum(lo - ph, ph - hi)
            print(f"     accepts tri {k}: t={float(t[k])!r} u={float(u[k])!r} v={float(v[k])!r} hit point {ph.tolist()} "
                  f"outside its box by {out_by.tolist()} (box {lo.tolist()} .. {hi.tolist()})")


if __name__ == "__main__":
    main()
