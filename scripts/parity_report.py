"""Prints GPU-vs-oracle parity statistics per configuration (numbers quoted in DESIGN.md).
Run on the GPU box: python scripts/parity_report.py > gpurun_out/parity.txt"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "restir-embree_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402

import oracle_lib as O  # noqa: E402
from restir_amd import Renderer, params as P, scenes  # noqa: E402


def stats(a, b):
    diff = np.linalg.norm(a.astype(np.float64) - b, axis=-1)
    den = np.maximum(np.linalg.norm(b.astype(np.float64), axis=-1), 1e-3)
    rel = diff / den
    return dict(exact=float((a == b).all(-1).mean()), within_1e4=float((rel <= 1e-4).mean()),
                within_1e6=float((rel <= 1e-6).mean()), mean_rel=float(rel.mean()), max_rel=float(rel.max()),
                n_px=int(rel.size), n_gt_1e2=int((rel > 1e-2).sum()))


def run(name, sc, W, H, prm, frames=1, cam=None):
    g = Renderer(W, H)
    gs = g.load_scene(sc)
    o = O.OracleRenderer(W, H)
    os_ = O.OracleScene(sc)
    for f in range(frames):
        c = cam(f) if cam else sc.camera
        a = g.produce_restir(gs, c, prm, f).copy()
        t0 = time.time()
        b = o.render(os_, c, prm, f)
        dt = time.time() - t0
        s = stats(a, b)
        print(f"{name:34s} f{f} {W}x{H}: " + " ".join(f"{k}={v:.6g}" if isinstance(v, float) else f"{k}={v}"
                                                    for k, v in s.items()) + f" gpu_rays={g.last_times.rays} oracle_rays={o.rays} oracle_s={dt:.2f}")


if __name__ == "__main__":
    c1, c2 = scenes.cornell_box(8), scenes.cornell_many_lights(1024)
    run("C1 defaults", c1, 256, 256, P.default_params())
    run("C2 metric point", c2, 480, 270, P.metric_params())
    for m in ("constant", "debias_contrib", "debias_z", "balance", "pairwise"):
        run(f"C1 spatial {m}", c1, 128, 96, P.default_params(m_area=4, do_spatial=1, spatial_neighbors=4, spatial_mis=m))
    run("C1 temporal+spatial orbit", c1, 160, 120, P.c3_params(m_area=8), frames=4,
        cam=lambda f: scenes.orbit_camera(c1.camera, f, 24, 0.3))
    sp = scenes.sponza_like(target_tris=120_000, n_lamps=1024)
    run("C3-like temporal+spatial", sp, 192, 108, P.c3_params(), frames=3,
        cam=lambda f: scenes.orbit_camera(sp.camera, f, 240, 0.3))
