"""GPU parity at the BASELINE.json workloads (configs C1-C5), not reduced stand-ins.

Every frame goes through the C ABI (librestir_amd.so) and is compared with the oracle on the same seeded
inputs.  Since round 6 the kernels and the oracle share their transcendental functions (csrc/rs_libm.h: one
fixed sequence of IEEE operations instead of ocml vs glibc) and the closest-hit walks test boxes with a margin
(rs_wide.h box_epsilon), so the frames are bit-identical (np.array_equal) at C1, C2 1920x1080, C3 480x270 and the
first 64+ frames of C5.  What remains is an any-hit edge case: Moller-Trumbore accepts a shadow ray's hit on a
triangle edge that coincides with a face of the triangle's box while the slab test of that box rejects the ray
(by rounding), so whether the occluder is found depends on the tree (GPU PLOC vs the oracle's SAH tree) -- about
1 ray in 1e9 (C3 at 3840x2160: 1 seed pixel per frame; scripts/anyhit_probe.py).  Those frames are checked with
a pixel-count bound on top of the tolerance (per-pixel relative L2 <= 1e-4 on >= 99.5 % of pixels, mean
<= 1e-4).  The statistics are printed (-s) and recorded in DESIGN.md §5.

  C1  Cornell box, 8 emissive quads, 512x512, reference defaults
  C2  Cornell + 1024 emissive quads, full 1920x1080, metric point (A=32 B=1, k=4 CONSTANT, temporal off)
  C3  Sponza-like (250 k tris, 4096 emissive tris), 480x270, 2 temporal+spatial frames, orbiting camera;
      and at the metric's full 1920x1080, 3 orbit frames
  C5  C2's scene with 1024 lights, 32 consecutive orbit frames with moving lights (temporal + spatial,
      confidence cap 20 reached after 20 frames and held across the rest of the sequence); and the full
      240-frame sequence at 1920x1080
  C3  also one frame pair at C4's 3840x2160 against the oracle
  C4  C3 at 3840x2160 split in 8 row bands rendered by 8 contexts on one GPU (the RCCL halo exchange
      emulated by device copies) with G-buffer margins of only the spatial halo: bit-identical to one
      context's full frame (the temporal pass rebuilds the few G elements a reprojection needs beyond
      a tile's rows)
"""
import numpy as np
import pytest

import oracle_lib as O
from restir_amd import params as P
from restir_amd import scenes
from restir_amd.renderer import Renderer

pytestmark = pytest.mark.gpu

PIX_TOL, PIX_FRAC, MEAN_TOL = 1e-4, 0.995, 1e-4


def _stats(gpu, ref):
    diff = np.linalg.norm(gpu.astype(np.float64) - ref, axis=-1)
    den = np.maximum(np.linalg.norm(ref.astype(np.float64), axis=-1), 1e-3)
    rel = diff / den
    return float((rel <= PIX_TOL).mean()), float(rel.mean()), float(rel.max())


def _check(gpu, ref, what, exact=True, max_diff=0):
    assert np.isfinite(gpu).all(), what
    frac, mean, mx = _stats(gpu, ref)
    ndiff = int(np.any(gpu != ref, axis=-1).sum())
    print(f"[parity] {what}: differing pixels {ndiff} of {gpu.shape[0] * gpu.shape[1]}, within 1e-4 = "
          f"{100 * frac:.4f} %, mean rel L2 = {mean:.3g}, max = {mx:.3g}", flush=True)
    assert frac >= PIX_FRAC and mean <= MEAN_TOL, f"{what}: frac_ok={frac:.5f} mean_rel={mean:.3g} max_rel={mx:.3g}"
    if exact:
        assert ndiff == 0, f"{what}: {ndiff} pixels differ from the oracle"
    else:
        assert ndiff <= max_diff, f"{what}: {ndiff} pixels differ from the oracle (bound {max_diff})"


def test_c1_512():
    sc = scenes.cornell_box(8)
    W = H = 512
    g = Renderer(W, H)
    gs = g.load_scene(sc)
    o, os_ = O.OracleRenderer(W, H), O.OracleScene(sc)
    for f in range(2):
        _check(g.produce_restir(gs, sc.camera, P.default_params(), f).copy(),
               o.render(os_, sc.camera, P.default_params(), f), f"C1 512x512 frame {f}")


def test_c2_full_1080p():
    sc = scenes.cornell_many_lights(1024)
    W, H = 1920, 1080
    prm = P.metric_params()
    g = Renderer(W, H)
    gs = g.load_scene(sc)
    a = g.produce_restir(gs, sc.camera, prm, 0, timed=True).copy()
    rays = int(g.last_times.rays)
    o = O.OracleRenderer(W, H)
    b = o.render(O.OracleScene(sc), sc.camera, prm, 0)
    _check(a, b, "C2 1920x1080")
    # the device skips the re-traced final p-hat / shade rays the oracle still traces
    print(f"[rays] C2 1080p: device {rays}, oracle {o.rays}")
    assert 0.9 * o.rays <= rays <= o.rays, (rays, o.rays)


def test_c3_full_scene_temporal():
    sc = scenes.sponza_like()
    assert sc.n_tris >= 245_000 and int(sc.emissive_mask().sum()) == 4096
    W, H = 480, 270
    prm = P.c3_params()
    cam = lambda f: scenes.orbit_camera(sc.camera, f, 240, 0.3)
    g = Renderer(W, H)
    gs = g.load_scene(sc)
    o, os_ = O.OracleRenderer(W, H), O.OracleScene(sc)
    for f in range(2):
        _check(g.produce_restir(gs, cam(f), prm, f).copy(), o.render(os_, cam(f), prm, f), f"C3 480x270 frame {f}")


def test_c3_full_1080p():
    """C3 at the resolution the metric is quoted on: 3 orbit frames (temporal + spatial) of the full scene at
    1920x1080 against the oracle (~9 s per frame on 16 host threads)."""
    sc = scenes.sponza_like()
    W, H = 1920, 1080
    prm = P.c3_params()
    cam = lambda f: scenes.orbit_camera(sc.camera, f, 240, 0.3)
    g = Renderer(W, H)
    gs = g.load_scene(sc)
    o, os_ = O.OracleRenderer(W, H), O.OracleScene(sc)
    for f in range(3):
        # (frames 0 and 1 bit-identical; frame 2 carries one any-hit edge-case pixel, see the module docstring)
        _check(g.produce_restir(gs, cam(f), prm, f).copy(), o.render(os_, cam(f), prm, f), f"C3 1920x1080 frame {f}",
               exact=f < 2, max_diff=16)


def test_c5_moving_lights_sequence():
    sc = scenes.cornell_many_lights(1024)
    W, H = 480, 270
    prm = P.c3_params()
    g = Renderer(W, H)
    gs = g.load_scene(sc)
    o = O.OracleRenderer(W, H)
    n = 32
    worst = 1.0
    for f in range(n):
        pos = scenes.moving_light_positions(sc, f, 240)
        gs.update_positions(pos)
        cam = scenes.orbit_camera(sc.camera, f, 240, 0.3)
        a = g.produce_restir(gs, cam, prm, f).copy()
        moved = scenes.Scene(pos, sc.normals, sc.tri_material, sc.materials, sc.camera)
        b = o.render(O.OracleScene(moved), cam, prm, f)
        _check(a, b, f"C5 frame {f}")
        worst = min(worst, _stats(a, b)[0])
    # M-capping across the sequence: after 20+ temporal frames the confidences sit at the cap (20)
    # (pixels with a reservoir: emissive / miss pixels keep an empty one with confidence 0)
    conf = g.reservoirs()[..., 11]
    has = conf > 0
    assert has.mean() > 0.3 and conf.max() == prm.confidence_cap
    assert (conf[has] == prm.confidence_cap).mean() >= 0.99
    ro = o.reservoirs()[..., 11]
    assert np.array_equal(conf, ro)
    print(f"[parity] C5 {n} frames: worst frame {100 * worst:.4f} % of pixels within 1e-4")


def test_c4_eight_bands_4k_bit_identical():
    import torch
    from restir_amd.distributed import GpuTileBackend, band_rows, halo_rows
    sc = scenes.sponza_like()
    W, H, N = 3840, 2160, 8
    prm = P.c3_params()
    cams = [scenes.orbit_camera(sc.camera, f, 240, 0.3) for f in range(3)]
    torch.cuda.set_stream(torch.cuda.Stream())
    st = torch.cuda.current_stream().cuda_stream
    full = Renderer(W, H, stream=st)
    fs = full.load_scene(sc)
    ref = [full.produce_restir(fs, c, prm, f).copy() for f, c in enumerate(cams)]
    bes = [GpuTileBackend(Renderer(W, H, stream=st)) for _ in range(N)]
    hs = [be.load_scene(sc) for be in bes]
    h = halo_rows(prm)
    margin = h                                    # TiledRenderer's default: the halo rows only
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
        rebuilt = [int(be.last_times.reproj_outside) for be in bes]
        assert np.array_equal(np.concatenate(bands, 0), ref[f]), f"C4 frame {f}"
        print(f"[parity] C4 3840x2160 frame {f}, 8 bands, margin {margin}: bit-identical to the full frame "
              f"(G elements rebuilt beyond the tiles: {rebuilt})")


def _energy_rel(gpu, ref):
    """sum |gpu - ref| / sum |ref| over the frame (L2 per pixel): the frame's relative radiance error, which -- unlike
    the per-pixel mean -- a dark pixel's flip cannot dominate (its 1e-3 denominator floor turns a 0.1 difference into
    a relative error of 100)"""
    d = np.linalg.norm(gpu.astype(np.float64) - ref, axis=-1).sum()
    return float(d / max(np.linalg.norm(ref.astype(np.float64), axis=-1).sum(), 1e-30))


def test_c5_1080p():
    """C5 at the shape BASELINE names: the C2 scene at 1920x1080 with the lights moving every frame, the camera
    orbiting, temporal (cap 20) + spatial reuse, ALL 240 frames of the sequence against the oracle rendering each
    moved scene: bit-identical through frame 63 and in most frames after (see the assertions).  Every frame's figures go to
    gpurun_out/c5_240_stats.txt (profiles/r06_c5_240_stats.txt)."""
    import os
    sc = scenes.cornell_many_lights(1024)
    W, H = 1920, 1080
    prm = P.c3_params()
    g = Renderer(W, H)
    gs = g.load_scene(sc)
    o = O.OracleRenderer(W, H)
    n = 240
    rows, fr = [], []
    for f in range(n):
        pos = scenes.moving_light_positions(sc, f, 240)
        gs.update_positions(pos)
        cam = scenes.orbit_camera(sc.camera, f, 240, 0.3)
        a = g.produce_restir(gs, cam, prm, f).copy()
        moved = scenes.Scene(pos, sc.normals, sc.tri_material, sc.materials, sc.camera)
        b = o.render(O.OracleScene(moved), cam, prm, f)
        assert np.isfinite(a).all(), f
        frac, mean, mx = _stats(a, b)
        er = _energy_rel(a, b)
        rel = np.linalg.norm(a.astype(np.float64) - b, axis=-1) / np.maximum(np.linalg.norm(b, axis=-1), 1e-3)
        lum = np.linalg.norm(b, axis=-1)
        dark = lum < 1e-2
        # how much of the per-pixel mean the dark pixels carry
        dark_share = float(rel[dark].sum() / max(rel.sum(), 1e-30))
        fr.append(frac)
        rows.append((f, frac, mean, mx, er, dark_share, int((rel > PIX_TOL).sum()), int(np.any(a != b, axis=-1).sum())))
        print(f"[parity] C5 1080p frame {f}: within 1e-4 {100 * frac:.4f} %, mean rel {mean:.3g}, max {mx:.3g}, "
              f"energy rel {er:.3g}, dark-pixel share of the mean {dark_share:.2f}", flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/c5_240_stats.txt", "w") as fh:
        fh.write("frame frac_within_1e-4 mean_rel max_rel energy_rel dark_share_of_mean pixels_out pixels_differing\n")
        for r in rows:
            fh.write(f"{r[0]} {r[1]:.6f} {r[2]:.4g} {r[3]:.4g} {r[4]:.4g} {r[5]:.3f} {r[6]} {r[7]}\n")
    worst = min(fr)
    print(f"[parity] C5 1080p {n} frames: worst frame {100 * worst:.4f} % (frame {int(np.argmin(fr))}), "
          f"mean of the last 16 {100 * float(np.mean(fr[-16:])):.4f} %, worst energy rel {max(r[4] for r in rows):.3g}")
    bad = [r for r in rows if not (r[1] >= PIX_FRAC and r[2] <= MEAN_TOL and r[4] <= MEAN_TOL)]
    assert not bad, bad[:5]
    # bit-identical through the first 64 frames and in >= 3/4 of all; the any-hit edge cases (module docstring) enter
    # at a few frames (measured: 80 and 119, each one seed pixel) and fade from the capped history: <= 0.1 % of the
    # pixels and a relative energy error <= 1e-7 in any frame (measured worst: 503 px, 1.0e-9)
    assert all(r[7] == 0 for r in rows[:64]), [r for r in rows[:64] if r[7]][:3]
    assert sum(r[7] == 0 for r in rows) >= 180, sum(r[7] == 0 for r in rows)
    assert all(r[7] <= 0.001 * W * H and r[4] <= 1e-7 for r in rows), [r for r in rows if r[7] > 0.001 * W * H or r[4] > 1e-7][:3]


def test_c3_4k_frame():
    """C3's scene at C4's 3840x2160 against the oracle (C4 was only a self-comparison of bands vs the
    GPU's full frame): two orbit frames -- the first without, the second with temporal history -- temporal + spatial
    reuse, the oracle on the host (~40 s per frame on 16 threads)."""
    sc = scenes.sponza_like()
    W, H = 3840, 2160
    prm = P.c3_params()
    cam = lambda f: scenes.orbit_camera(sc.camera, f, 240, 0.3)
    g = Renderer(W, H)
    gs = g.load_scene(sc)
    o, os_ = O.OracleRenderer(W, H), O.OracleScene(sc)
    for f in range(2):
        a = g.produce_restir(gs, cam(f), prm, f).copy()
        b = o.render(os_, cam(f), prm, f)
        _check(a, b, f"C3 3840x2160 frame {f}", exact=False, max_diff=64)
        print(f"[parity] C3 3840x2160 frame {f}: energy rel {_energy_rel(a, b):.3g}", flush=True)
