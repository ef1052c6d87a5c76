"""Diagnostic: C3 row bands on one GPU -- reproj_outside counts per band and equality with the full frame."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "restir-embree_amd"), os.path.join(ROOT, "tests")]
import numpy as np
import torch
from restir_amd import params as P, scenes
from restir_amd.renderer import Renderer
from restir_amd.distributed import GpuTileBackend, band_rows, halo_rows

W, H, N = int(sys.argv[1]), int(sys.argv[2]), 8
margin = int(sys.argv[3]) if len(sys.argv) > 3 else 64
sc = scenes.sponza_like()
prm = P.c3_params()
cams = [scenes.orbit_camera(sc.camera, f, 240, 0.3) for f in range(3)]
torch.cuda.set_stream(torch.cuda.Stream())
st = torch.cuda.current_stream().cuda_stream
full = Renderer(W, H, stream=st)
fs = full.load_scene(sc)
ref, gb = [], []
for f, c in enumerate(cams):
    ref.append(full.produce_restir(fs, c, prm, f).copy())
    gb.append(full.gbuffer())
bes = [GpuTileBackend(Renderer(W, H, stream=st)) for _ in range(N)]
hs = [be.load_scene(sc) for be in bes]
h = halo_rows(prm)
for f, cam in enumerate(cams):
    for r, be in enumerate(bes):
        y0, y1 = band_rows(H, r, N)
        be.begin(hs[r], cam, prm, f, y0, y1, max(margin, h), h)
    for be in bes:
        be.temporal()
    for p in range(prm.spatial_passes):
        torch.cuda.synchronize()
        for r, be in enumerate(bes):
            if r > 0:
                be.halo_tensor(0).copy_(bes[r - 1].halo_tensor(3))
            if r < N - 1:
                be.halo_tensor(1).copy_(bes[r + 1].halo_tensor(2))
        torch.cuda.synchronize()
        for be in bes:
            be.spatial(p)
    bands = [be.finish(timed=True).cpu().numpy().reshape(-1, W, 3) for be in bes]
    outside = [int(be.last_times.reproj_outside) for be in bes]
    img = np.concatenate(bands, 0)
    diff = np.nonzero(np.any(img != ref[f], -1))
    print(f"frame {f}: outside={outside} differing px={diff[0].size}", list(zip(diff[0][:10], diff[1][:10])))
    g = gb[f]
    miss = (np.abs(g[..., 0:3]).sum(-1) == 0)
    print(f"   miss pixels (pos==0) in the full frame: {int(miss.sum())}; emissive: {int((g[..., 12:15].max(-1) > 0).sum())}")
