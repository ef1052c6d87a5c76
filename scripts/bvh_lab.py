"""Driver for scripts/bvh_lab.cpp (analysis tooling): dumps a scene (C3 sponza_like by default), builds
the lab, runs builder / leaf / order variants and prints one line each."""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "restir-embree_amd"))
from restir_amd import scenes  # noqa: E402


def dump(sc, path):
    em = np.nonzero(sc.emissive_mask())[0].astype(np.int32)
    with open(path, "wb") as f:
        np.array([sc.n_tris, em.size], np.int32).tofile(f)
        sc.camera.as_array().astype(np.float32).tofile(f)
        np.ascontiguousarray(sc.positions, np.float32).tofile(f)
        em.tofile(f)


def main():
    exe = "/tmp/bvh_lab"
    src = os.path.join(ROOT, "scripts", "bvh_lab.cpp")
    if not os.path.exists(exe) or os.path.getmtime(exe) < os.path.getmtime(src):
        subprocess.check_call(["g++", "-O3", "-march=native", "-fopenmp", "-std=c++17", "-o", exe, src])
    name = os.environ.get("SCENE", "C3")
    if name == "moved":   # tests/test_gpu_parity.py::test_update_positions_refit_matches_fresh_scene[c3]
        sc = scenes.sponza_like(target_tris=30_000, n_lamps=128)
        sc.positions = scenes.moving_light_positions(sc, 130, 240, amplitude=0.4)
    else:
        sc = scenes.by_name(name)
    path = f"/tmp/bvh_lab_{name}.bin"
    dump(sc, path)
    W, H = os.environ.get("LAB_W", "480"), os.environ.get("LAB_H", "272")
    runs = [a.split(",") for a in sys.argv[1:]] or [["ploc"], ["sweep"], ["sbvh"]]
    for r in runs:
        subprocess.run([exe, path, r[0], W, H, *r[1:]], check=False)


if __name__ == "__main__":
    main()
