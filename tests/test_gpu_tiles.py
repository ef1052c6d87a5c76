"""GPU test of the tile stages (rs_tile_*) used by the multi-GPU path: N contexts on one device play
N ranks; halo rows move device-to-device through the same zero-copy tensor views the RCCL exchange
uses (restir_amd.distributed.GpuTileBackend).  The assembled frame must equal the single-context
frame bit for bit."""
import os
import numpy as np
import pytest

from restir_amd import params as P
from restir_amd import scenes
from restir_amd.distributed import GpuTileBackend, band_rows, halo_rows
from restir_amd.renderer import Renderer

pytestmark = pytest.mark.gpu


def _emulate(sc, W, H, prm, n_ranks, cams, margin):
    import torch
    torch.cuda.set_stream(torch.cuda.Stream())      # a real (non-null) stream shared with the contexts
    st = torch.cuda.current_stream().cuda_stream
    bes = [GpuTileBackend(Renderer(W, H, stream=st)) for _ in range(n_ranks)]
    hs = [be.load_scene(sc) for be in bes]
    h = halo_rows(prm)
    out = []
    for f, cam in enumerate(cams):
        for r, be in enumerate(bes):
            y0, y1 = band_rows(H, r, n_ranks)
            be.begin(hs[r], cam, prm, f, y0, y1, max(margin, h), h)
        for be in bes:
            be.temporal()
        if prm.do_spatial:
            for p in range(prm.spatial_passes):
                torch.cuda.synchronize()
                for r, be in enumerate(bes):
                    if r > 0:
                        be.halo_tensor(0).copy_(bes[r - 1].halo_tensor(3))
                    if r < n_ranks - 1:
                        be.halo_tensor(1).copy_(bes[r + 1].halo_tensor(2))
                torch.cuda.synchronize()
                for be in bes:
                    be.spatial(p)
        bands = [be.finish().cpu().numpy().reshape(-1, W, 3) for be in bes]
        out.append(np.concatenate(bands, 0))
    return out


@pytest.mark.parametrize("n_ranks", [2, 4])
def test_tiles_bit_identical_to_full_frame(n_ranks):
    sc = scenes.cornell_many_lights(128)
    W, H = 96, 64
    prm = P.default_params(m_area=6, do_spatial=1, spatial_neighbors=4, spatial_passes=2, do_temporal=1)
    cams = [scenes.orbit_camera(sc.camera, f, 48, 0.2) for f in range(3)]
    tiles = _emulate(sc, W, H, prm, n_ranks, cams, margin=H)
    full = Renderer(W, H)
    fs = full.load_scene(sc)
    for f, cam in enumerate(cams):
        ref = full.produce_restir(fs, cam, prm, f)
        assert np.array_equal(tiles[f], ref), f"frame {f}"


def test_metric_point_tiles():
    sc = scenes.cornell_many_lights(1024)
    W, H = 128, 72
    prm = P.metric_params()
    tiles = _emulate(sc, W, H, prm, 4, [sc.camera], margin=0)
    full = Renderer(W, H)
    ref = full.produce_restir(full.load_scene(sc), sc.camera, prm, 0)
    assert np.array_equal(tiles[0], ref)


# ---------------------------------------------------------------- real processes, real GPU contexts
def _gpu_worker(rank, world, port, W, H, out_path, rebalance, async_gather=False):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "restir-embree_amd"), os.path.join(root, "tests")]
    import torch
    import torch.distributed as dist
    from restir_amd import params as P, scenes
    from restir_amd.distributed import TiledRenderer
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    torch.cuda.set_stream(torch.cuda.Stream())
    sc = scenes.cornell_many_lights(256)
    prm = P.c3_params(m_area=8, spatial_passes=2)
    tr = TiledRenderer(W, H, rank, world, device=0, stream=torch.cuda.current_stream().cuda_stream,
                       temporal_margin=H, async_gather=async_gather)
    tr.be.r.set_traversal("lockstep")      # no AUTO tuning frames (they run alone): frames use the lanes
    s = tr.load_scene(sc)
    if rebalance:   # bands from the GPU's own per-row wave times (unequal in general)
        bands = tr.rebalance(lambda i: tr.render(s, sc.camera, prm, i), n_frames=2, min_rows=6)
        assert bands[0][0] == 0 and bands[-1][1] == H and len(bands) == world
    frames = []
    for f in range(3):
        fr = tr.render(s, scenes.orbit_camera(sc.camera, f, 24, 0.25), prm, f)
        tr.wait()
        if rank == 0:
            frames.append(fr.cpu().numpy().copy())
    if rank == 0:
        np.save(out_path, np.stack(frames))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,rebalance,async_gather", [(2, False, False), (3, True, True)])
def test_multiprocess_tiles_on_gpu_match_full_frame(world, rebalance, async_gather, tmp_path):
    """TiledRenderer + GpuTileBackend in 2-3 real processes (one HIP context each on the same GPU; halo
    exchange and gather over gloo, staged through host memory because RCCL refuses two ranks on one
    device; the 3-rank case with bench.py's async gather: per-lane process groups and framebuffers):
    the gathered frames equal a single-context full frame bit for bit."""
    import socket
    import torch.multiprocessing as mp
    from restir_amd import params as P, scenes
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    W, H = 48, 40
    out = str(tmp_path / "frames.npy")
    mp.spawn(_gpu_worker, args=(world, port, W, H, out, rebalance, async_gather), nprocs=world, join=True)
    got = np.load(out)
    sc = scenes.cornell_many_lights(256)
    prm = P.c3_params(m_area=8, spatial_passes=2)
    g = Renderer(W, H)
    gs = g.load_scene(sc)
    for f in range(3):
        ref = g.produce_restir(gs, scenes.orbit_camera(sc.camera, f, 24, 0.25), prm, f)
        assert np.array_equal(got[f], ref), f"frame {f}"
