"""Diagnostic (GPU box, 1 GPU): C2's (or C3's, --scene C3) initial pass broken into its parts by varying the workload -- the VALU
budget of DESIGN §4.  Renders the C2 frame (1920x1080, lockstep walks, one frame in flight) for
each variant in turn and prints the initial pass's mean time (HIP events, rs_get_timing_totals) and rays per frame:

  A32B1      the metric point (A = 32 area candidates, B = 1 BRDF candidate)
  A16B1      half the area candidates            -> per area candidate (pair of shadow rays = one walk)
  A32B0      no BRDF candidate                   -> the BRDF candidate (closest hit + shadow ray)
  A32B1vis   doVisibilityPass: no shadow rays in the initial pass -> the shadow walks
  A0B0       G-buffer only (primary ray + G element + empty reservoir)

Run it under `rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES ...` for instruction counts: the variants'
launches come in the order above, --frames each (the first --warmup of them untimed); scripts/valu_budget_summary.py
groups the counter rows by variant.

  python scripts/valu_budget.py [--frames 8] [--warmup 2]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "restir-embree_amd"))

from restir_amd import params as P, scenes  # noqa: E402
from restir_amd.renderer import Renderer  # noqa: E402

VARIANTS = [("A32B1", {}), ("A16B1", {"m_area": 16}), ("A32B0", {"m_brdf": 0}),
            ("A32B1vis", {"do_visibility_pass": 1}), ("A0B0", {"m_area": 0, "m_brdf": 0})]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=8)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--scene", default="C2", help="C2 (lockstep walks) or C3 (per-lane walks, sorted pass)")
    a = ap.parse_args()
    sc = scenes.cornell_many_lights(1024) if a.scene == "C2" else scenes.sponza_like()
    r = Renderer(1920, 1080)
    r.set_traversal("lockstep" if a.scene == "C2" else "lane")
    r.set_run_ahead(0)
    gs = r.load_scene(sc)
    f = 0
    for name, kw in VARIANTS:
        prm = P.metric_params(**kw)
        for i in range(a.frames):
            if i == a.warmup:
                r.synchronize()
                r.timing_totals(reset=True)
            r.produce_restir(gs, sc.camera, prm, f, copy_out=False, timed=False)
            f += 1
        r.synchronize()
        t, n = r.timing_totals(reset=True)
        print(f"{name:10s} frames {n}: initial {t.gbuffer_initial_ms / max(n, 1):.4f} ms, visibility "
              f"{t.visibility_ms / max(n, 1):.4f}, spatial {t.spatial_ms / max(n, 1):.4f}, rays/frame "
              f"{t.rays / max(n, 1) / 1e6:.2f} M", flush=True)
    gs.close()
    r.close()


if __name__ == "__main__":
    main()
