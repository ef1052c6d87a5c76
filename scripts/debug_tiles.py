import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "restir-embree_amd"), os.path.join(ROOT, "tests")]
import numpy as np, torch
from restir_amd import Renderer, params as P, scenes
from test_gpu_tiles import _emulate
sc = scenes.cornell_many_lights(1024)
W, H = 128, 72
for name, prm, cams in [("metric", P.metric_params(), [sc.camera]),
                        ("nospatial", P.metric_params(do_spatial=0), [sc.camera]),
                        ("spatial_k0", P.metric_params(spatial_neighbors=0), [sc.camera])]:
    tiles = _emulate(sc, W, H, prm, 4, cams, margin=0)
    full = Renderer(W, H, stream=torch.cuda.current_stream().cuda_stream)
    ref = full.produce_restir(full.load_scene(sc), cams[0], prm, 0)
    bad = np.any(tiles[0] != ref, axis=-1)
    rows = np.flatnonzero(bad.any(1))
    print(name, "mismatched px", int(bad.sum()), "rows", rows[:40].tolist())
