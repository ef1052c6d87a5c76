"""CPU test of the multi-GPU path's orchestration (restir_amd/distributed.py) with the gloo backend:
row-band sharding, reservoir halo exchange (batch_isend_irecv) before every spatial pass, framebuffer
gather.  Each rank renders its band with the oracle's tile stages; the gathered frame must equal the
full-frame oracle frame bit for bit (the per-pixel counter RNG is keyed by the full-frame index)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _cfg(n_frames=3):
    from restir_amd import params as P, scenes
    sc = scenes.cornell_box(8)
    prm = P.default_params(m_area=4, do_spatial=1, spatial_neighbors=4, spatial_passes=2, do_temporal=1)
    cams = [scenes.orbit_camera(sc.camera, f, 24, 0.25) for f in range(n_frames)]
    return sc, prm, cams


def _worker(rank, world, port, W, H, out_path, rebalance=False, margin=None):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "restir-embree_amd"), os.path.join(root, "tests")]
    import torch.distributed as dist
    import oracle_lib as O
    from restir_amd.distributed import TiledRenderer
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    O.lib().or_set_num_threads(2)
    sc, prm, cams = _cfg(3 if margin is None else 8)
    tr = TiledRenderer(W, H, rank, world, backend=O.OracleTileBackend(W, H),
                       temporal_margin=H if margin is None else margin)
    s = tr.load_scene(sc)
    if rebalance:
        bands = tr.rebalance(lambda i: tr.render(s, cams[0], prm, i), n_frames=1, min_rows=6)
        assert bands != [(r * H // world, (r + 1) * H // world) for r in range(world)], bands
    frames = []
    for f, cam in enumerate(cams):
        fr = tr.render(s, cam, prm, f)
        if rank == 0:
            frames.append(fr.numpy().copy())
    if rank == 0:
        np.save(out_path, np.stack(frames))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,rebalance,margin", [(2, False, None), (3, False, None), (3, True, None), (3, False, 5)])
def test_tiled_frames_match_full_frame(world, rebalance, margin, tmp_path):
    """Equal bands and cost-balanced (unequal) bands both gather the full frame bit for bit -- also with a
    G-buffer margin of only the spatial halo (5 rows), where the temporal pass's reprojections (moving
    camera; miss pixels at (0,0,0) project into other bands) rebuild the elements beyond the tile."""
    import oracle_lib as O
    W, H = 40, 36
    out = str(tmp_path / "frames.npy")
    mp.spawn(_worker, args=(world, _free_port(), W, H, out, rebalance, margin), nprocs=world, join=True)
    got = np.load(out)
    sc, prm, cams = _cfg(3 if margin is None else 8)
    r = O.OracleRenderer(W, H)
    s = O.OracleScene(sc)
    for f, cam in enumerate(cams):
        ref = r.render(s, cam, prm, f)
        assert np.array_equal(got[f], ref), f"frame {f}: max diff {np.abs(got[f] - ref).max()}"


def test_balanced_bands():
    from restir_amd.distributed import balanced_bands
    assert balanced_bands(np.ones(100), 4) == [(0, 25), (25, 50), (50, 75), (75, 100)]
    b = balanced_bands(np.r_[np.ones(50), 3 * np.ones(50)], 2)
    assert b == [(0, 67), (67, 100)], b                     # 50 + 17*3 = 101 vs 99
    assert balanced_bands(np.zeros(10), 2) == [(0, 5), (5, 10)]  # no costs: equal bands
    b = balanced_bands(np.r_[np.zeros(90), np.ones(10)], 4, min_rows=5)
    assert all(y1 - y0 >= 5 for y0, y1 in b) and b[0][0] == 0 and b[-1][1] == 100
    with pytest.raises(ValueError):
        balanced_bands(np.ones(10), 4, min_rows=3)


def test_halo_rows_and_bands():
    from restir_amd.distributed import band_rows, halo_rows
    from restir_amd import params as P
    assert [band_rows(1080, r, 8) for r in (0, 7)] == [(0, 135), (945, 1080)]
    assert sum(b - a for a, b in (band_rows(1081, r, 8) for r in range(8))) == 1081
    assert halo_rows(P.metric_params()) == 5          # floor(sqrt(30))
    assert halo_rows(P.default_params()) == 0         # no spatial reuse -> nothing to exchange
    # float32 semantics (the device's sqrtf): 24.999998f -> sqrtf rounds to 5.0, so 5 rows, not 4
    assert halo_rows(P.metric_params(spatial_radius=24.999998)) == 5
    assert halo_rows(P.metric_params(spatial_radius=24.9)) == 4


def test_oracle_tiles_halo_margin_rebuild_bit_identical():
    """Tile stages with a G-buffer margin of only the spatial halo under a moving camera (the miss pixels
    around the box have position (0,0,0), which projects into other bands): the temporal pass rebuilds the
    G elements beyond a tile's rows (counted: the path runs), so 4 in-process bands (halo copies between
    the stages, as the RCCL exchange does) give the full frame bit for bit over 5 frames."""
    import oracle_lib as O
    from restir_amd import params as P, scenes
    from restir_amd.distributed import band_rows, halo_rows
    O.lib().or_set_num_threads(4)
    sc = scenes.cornell_many_lights(64)
    W, H, N = 96, 72, 4
    prm = P.c3_params(m_area=4)
    cams = [scenes.orbit_camera(sc.camera, f, 40, 0.6) for f in range(5)]
    bes = [O.OracleTileBackend(W, H) for _ in range(N)]
    hs = [be.load_scene(sc) for be in bes]
    h = halo_rows(prm)
    full, fs = O.OracleRenderer(W, H), O.OracleScene(sc)
    for f, cam in enumerate(cams):
        for r, be in enumerate(bes):
            y0, y1 = band_rows(H, r, N)
            be.begin(hs[r], cam, prm, f, y0, y1, h, h)
        for be in bes:
            be.temporal()
        for p in range(prm.spatial_passes):
            for r, be in enumerate(bes):
                if r > 0:
                    be.halo_tensor(0).copy_(bes[r - 1].halo_tensor(3))
                if r < N - 1:
                    be.halo_tensor(1).copy_(bes[r + 1].halo_tensor(2))
            for be in bes:
                be.spatial(p)
        img = np.concatenate([be.finish().numpy().reshape(-1, W, 3) for be in bes], 0)
        ref = full.render(fs, cam, prm, f)
        assert np.array_equal(img, ref), f"frame {f}: {int(np.any(img != ref, -1).sum())} pixels differ"
    assert sum(int(O.lib().or_ctx_rebuilt(be.r.h)) for be in bes) > 0
