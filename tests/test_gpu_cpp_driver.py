"""GPU test of the C++ host mirror (include/restir.hpp) through its headless driver
(restir-embree_amd/tools/restir_render.cpp, the reference's tutorial_3 -> Producer loop without UI):
it renders frames with temporal + spatial reuse and writes the last frame as a PFM."""
import os
import subprocess

import numpy as np
import pytest

from restir_amd.renderer import decode_image

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOL = os.path.join(ROOT, "restir-embree_amd", "restir_render")


def test_cpp_driver_renders(tmp_path):
    assert os.path.exists(TOOL), "build restir-embree_amd (make) first"
    out = tmp_path / "frame.pfm"
    p = subprocess.run([TOOL, "--w", "64", "--h", "48", "--frames", "3", "--area", "4", "--spatial", "4",
                        "--temporal", "--out", str(out)], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stdout + p.stderr
    img = decode_image(out)
    assert img.shape == (48, 64, 3) and np.isfinite(img).all()
    assert img.max() > 0.0                         # the light and lit walls


def test_cpp_driver_denoised_display(tmp_path):
    """restir.hpp initOIDN + `denoise` (pg/simpleguidx11.cpp:52-75, :277-280): the exported display is the
    tonemapped denoised accumulator (weights from a .tza written by restir_amd.tza)."""
    from restir_amd import tza
    w = tmp_path / "w.tza"
    w.write_bytes(tza.write_tza(tza.random_unet_weights(seed=2)))
    png = tmp_path / "den.png"
    p = subprocess.run([TOOL, "--w", "64", "--h", "48", "--frames", "2", "--area", "4", "--denoise", str(w),
                        "--png", str(png)], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stdout + p.stderr
    img = decode_image(png)
    assert img.shape == (48, 64, 4) and img[..., 3].min() == 255
    p = subprocess.run([TOOL, "--w", "64", "--h", "48", "--frames", "1", "--denoise", str(tmp_path / "missing.tza")],
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 1 and "cannot open" in p.stderr


def test_cpp_driver_bench_pipelined_host_framebuffer():
    """restir_render --bench: produceRestir with frame_data in host memory every frame, pipelined (the
    readback of frame f overlaps frame f+1) and synchronous; one JSON line with both rates."""
    import json
    p = subprocess.run([TOOL, "--bench", "--w", "96", "--h", "64", "--frames", "12", "--area", "4", "--spatial", "4"],
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stdout + p.stderr
    d = json.loads(p.stdout.strip().splitlines()[-1])
    assert d["value"] > 0 and d["sync_value"] > 0 and d["frame_bytes"] == 96 * 64 * 12


def test_frame_readback_matches_synchronous_copy():
    """rs_frame_readback / rs_frame_wait (async copy on the context's copy stream, ordered after the frame;
    the lane's next frame waits for it) return the same framebuffer as rs_render_frame's synchronous copy,
    also while later frames are already rendering on other lanes."""
    import ctypes
    from restir_amd import params as P, scenes
    from restir_amd.renderer import Renderer
    sc = scenes.cornell_many_lights(128)
    W, H = 80, 48
    prm = P.c3_params(m_area=6)
    a, b = Renderer(W, H), Renderer(W, H)
    ga, gb = a.load_scene(sc), b.load_scene(sc)
    a.set_traversal("lockstep")
    b.set_traversal("lockstep")
    want = [a.produce_restir(ga, scenes.orbit_camera(sc.camera, f, 24, 0.2), prm, f).copy() for f in range(6)]
    L = b.lib
    bufs = [np.zeros((H, W, 3), np.float32) for _ in range(6)]
    tickets = []
    for f in range(6):
        b.produce_restir(gb, scenes.orbit_camera(sc.camera, f, 24, 0.2), prm, f, copy_out=False, timed=False)
        t = ctypes.c_uint64()
        assert L.rs_frame_readback(b.h, bufs[f].ctypes.data_as(ctypes.POINTER(ctypes.c_float)), ctypes.byref(t)) == 0
        tickets.append(t.value)
    for f in range(6):
        assert L.rs_frame_wait(b.h, tickets[f]) == 0
        assert np.array_equal(bufs[f], want[f]), f


def test_cpp_driver_multi_gpu_ranks_bit_identical():
    """A C++ host renders tiled frames through restir::MultiGpuRenderer (rs_mgpu_create_local +
    rs_mgpu_render_frame): 3 row bands with temporal + spatial reuse, bit-identical to one context."""
    import json
    p = subprocess.run([TOOL, "--w", "80", "--h", "60", "--frames", "4", "--area", "4", "--spatial", "4", "--temporal",
                        "--ranks", "3", "--compare"], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stdout + p.stderr
    d = json.loads(p.stdout.strip().splitlines()[-1])
    assert d == {"ranks": 3, "frames": 4, "compared": True, "bit_identical": True}
