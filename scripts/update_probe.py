"""Timing of the per-update geometry work (rs_scene_update_positions: binary + wide refits, light tables) on
C5's scene, alone on the device: `--updates` updates back to back, synchronised, wall ms per update printed.
Run it under `rocprofv3 --kernel-trace --stats` (with RESTIR_UPDATE_SPLIT=1 the fused update kernel's three
jobs are separate launches) for the per-kernel split.
    python scripts/update_probe.py --updates 50"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "restir-embree_amd"))

ap = argparse.ArgumentParser()
ap.add_argument("--updates", type=int, default=50)
a = ap.parse_args()

import torch  # noqa: E402
from restir_amd import Renderer, scenes  # noqa: E402

torch.cuda.set_device(0)
sc = scenes.by_name("C2")
r = Renderer(64, 48)
gs = r.load_scene(sc)
pos = [scenes.moving_light_positions(sc, f, 240) for f in range(8)]
for f in range(4):
    gs.update_positions(pos[f % 8])
torch.cuda.synchronize()
t0 = time.perf_counter()
for f in range(a.updates):
    gs.update_positions(pos[f % 8])
torch.cuda.synchronize()
print(f"C5 scene update: {(time.perf_counter() - t0) * 1e3 / a.updates:.3f} ms wall per update ({a.updates} back to back)",
      flush=True)
gs.close()
r.close()
