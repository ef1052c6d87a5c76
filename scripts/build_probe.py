"""Scene build timing (rs_scene_create's BVH build, restir_capi.hip build_bvh): builds the named scene
`--repeat` times in one process and prints build_ms each time -- the first build carries the one-time
costs (kernel code-object loading, first allocations), the later ones are the steady state.  Run it under
`rocprofv3 --kernel-trace --stats` for the per-kernel split.

    python scripts/build_probe.py --scene C3 --repeat 4"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "restir-embree_amd"))

ap = argparse.ArgumentParser()
ap.add_argument("--scene", default="C3")
ap.add_argument("--repeat", type=int, default=4)
a = ap.parse_args()

import torch  # noqa: E402
from restir_amd import Renderer, scenes  # noqa: E402

torch.cuda.set_device(0)
sc = scenes.by_name(a.scene)
t0 = time.perf_counter()
r = Renderer(64, 48)
print(f"context create wall {(time.perf_counter() - t0) * 1e3:.1f} ms", flush=True)
for i in range(a.repeat):
    t0 = time.perf_counter()
    gs = r.load_scene(sc)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) * 1e3
    print(f"{a.scene} build {i}: build_ms {gs.build_ms:.2f} (HIP events around build_bvh), load_scene wall {wall:.1f} ms,"
          f" {gs.n_tris} triangles, {gs.n_nodes} nodes, wide {gs.wide_tree_nodes()}", flush=True)
    gs.close()
r.close()
