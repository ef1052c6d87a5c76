"""CPU test of the native multi-GPU orchestration (restir-embree_amd/csrc/rs_mgpu_core.h -- the stage
sequence, halo exchange and gather rs_mgpu_render_frame runs): tests/cpp/mgpu_core_harness.cpp drives it
with the oracle's tile stages as ranks and host memcpy as the transport; the gathered frames equal the
oracle's full frames bit for bit.  The band-balancing rule is checked against restir_amd.distributed."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

import oracle_lib as O
from restir_amd import params as P
from restir_amd import scenes

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "cpp", "mgpu_core_harness.cpp")
HDR = os.path.join(ROOT, "restir-embree_amd", "csrc", "rs_mgpu_core.h")
SO = os.path.join(ROOT, "oracle", "_build", "libmgpu_core_harness.so")


def _harness():
    O.build()
    if not os.path.exists(SO) or os.path.getmtime(SO) < max(os.path.getmtime(SRC), os.path.getmtime(HDR)):
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-o", SO, SRC,
                               "-L" + os.path.dirname(O.LIB_PATH), "-lrestir_oracle",
                               "-Wl,-rpath," + os.path.dirname(O.LIB_PATH)])
    O.lib()                                       # the oracle first (the harness resolves or_tile_* from it)
    L = ctypes.CDLL(SO)
    vp = ctypes.c_void_p
    L.harness_frame.argtypes = [ctypes.POINTER(vp), ctypes.POINTER(vp), ctypes.c_int, ctypes.POINTER(ctypes.c_int32),
                                ctypes.c_int, ctypes.POINTER(ctypes.c_float), vp, ctypes.c_int, ctypes.c_float,
                                ctypes.c_int, ctypes.c_uint32, ctypes.POINTER(ctypes.c_float),
                                ctypes.POINTER(ctypes.c_int)]
    L.harness_balanced.argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                   ctypes.POINTER(ctypes.c_int32)]
    L.harness_balanced_grain.argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_int, ctypes.POINTER(ctypes.c_int32)]
    L.harness_halo.argtypes = [ctypes.c_float]
    L.harness_plan_check.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_int32), ctypes.c_int, ctypes.c_int,
                                     ctypes.c_int, ctypes.c_int, ctypes.c_char_p, ctypes.c_int]
    return L


@pytest.mark.parametrize("n,which", [(2, "c1"), (3, "c3"), (4, "c2")])
def test_native_orchestration_matches_full_frames(n, which):
    L = _harness()
    O.lib().or_set_num_threads(4)
    W, H = 64, 48
    if which == "c1":
        sc, prm = scenes.cornell_box(8), P.default_params(m_area=4, do_spatial=1, spatial_passes=2, do_temporal=1)
    elif which == "c2":
        sc, prm = scenes.cornell_many_lights(128), P.metric_params(m_area=8)
    else:
        sc, prm = scenes.sponza_like(target_tris=20_000, n_lamps=64), P.c3_params(m_area=4)
    cams = [scenes.orbit_camera(sc.camera, f, 24, 0.3) for f in range(3)]
    ranks = [O.OracleRenderer(W, H) for _ in range(n)]
    oscs = [O.OracleScene(sc) for _ in range(n)]
    ctxs = (ctypes.c_void_p * n)(*[r.h for r in ranks])
    scs = (ctypes.c_void_p * n)(*[s.h for s in oscs])
    rng = np.random.default_rng(n)
    while True:                                             # unequal bands, each >= the 5-row halo
        cuts = np.sort(rng.choice(np.arange(6, H - 5), n - 1, replace=False))
        bounds = np.array([0, *cuts, H], np.int32)
        if np.diff(bounds).min() >= 6:
            break
    full_ref = O.OracleRenderer(W, H)
    ref_scene = O.OracleScene(sc)
    for f, cam in enumerate(cams):
        out = np.zeros((H, W, 3), np.float32)
        ex = ctypes.c_int(0)
        cam7 = np.ascontiguousarray(cam.as_array(), np.float32)
        rc = L.harness_frame(ctxs, scs, n, bounds.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), W,
                             cam7.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), ctypes.cast(ctypes.byref(prm), ctypes.c_void_p),
                             prm.spatial_passes, prm.spatial_radius, prm.do_spatial, f,
                             out.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), ctypes.byref(ex))
        assert rc == 0
        assert ex.value == (2 * (n - 1) * prm.spatial_passes if prm.do_spatial else 0)
        ref = full_ref.render(ref_scene, cam, prm, f)
        assert np.array_equal(out, ref), f"{which} n={n} frame {f}: {int(np.any(out != ref, -1).sum())} px differ"


def test_native_orchestration_rejects_bands_thinner_than_halo():
    L = _harness()
    W, H, n = 32, 24, 3
    sc, prm = scenes.cornell_box(8), P.metric_params(m_area=2)
    ranks = [O.OracleRenderer(W, H) for _ in range(n)]
    oscs = [O.OracleScene(sc) for _ in range(n)]
    bounds = np.array([0, 10, 13, H], np.int32)             # a 3-row band, halo 5
    out = np.zeros((H, W, 3), np.float32)
    cam7 = np.ascontiguousarray(sc.camera.as_array(), np.float32)
    rc = L.harness_frame((ctypes.c_void_p * n)(*[r.h for r in ranks]), (ctypes.c_void_p * n)(*[s.h for s in oscs]), n,
                         bounds.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), W,
                         cam7.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), ctypes.cast(ctypes.byref(prm), ctypes.c_void_p),
                         1, 30.0, 1, 0, out.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), None)
    assert rc == -1


def test_native_band_balancing_matches_python():
    from restir_amd.distributed import balanced_bands, halo_rows
    L = _harness()
    rng = np.random.default_rng(3)
    for H, world, mr in [(100, 4, 1), (1080, 8, 5), (64, 3, 6), (37, 2, 5)]:
        for costs in (rng.uniform(0, 1, H), np.r_[np.zeros(H // 2), np.ones(H - H // 2)], np.zeros(H),
                      np.linspace(1, 9, H) ** 2):
            out = np.zeros(world + 1, np.int32)
            c = np.ascontiguousarray(costs, np.float64)
            assert L.harness_balanced(c.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), H, world, mr,
                                      out.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))) == 0
            py = balanced_bands(costs, world, mr)
            assert [(int(out[i]), int(out[i + 1])) for i in range(world)] == py, (H, world, mr)
    for r in (30.0, 24.999998, 24.9, 25.0, 0.5, 0.0):
        assert L.harness_halo(r) == halo_rows(P.metric_params(spatial_radius=r))


def test_band_balancing_on_wave_tiles():
    """rs_mgpu_rebalance's split on whole 8-row wave tiles (rs_mgpu_core.h balanced_bounds_grain) equals the
    Python restatement (distributed.balanced_bands(grain=8)); boundaries are multiples of 8 with >= min_rows rows,
    and heights that are not a multiple of 8 (or too few units) fall back to the row-exact split."""
    from restir_amd.distributed import balanced_bands
    L = _harness()
    rng = np.random.default_rng(5)
    for H, world, mr in [(1080, 8, 5), (2160, 8, 5), (1080, 2, 8), (48, 4, 5), (100, 4, 1), (37, 2, 5), (64, 8, 5)]:
        for costs in (rng.uniform(0, 1, H), np.r_[np.zeros(H // 2), np.ones(H - H // 2)], np.zeros(H),
                      np.linspace(1, 9, H) ** 2):
            out = np.zeros(world + 1, np.int32)
            c = np.ascontiguousarray(costs, np.float64)
            assert L.harness_balanced_grain(c.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), H, world, mr, 8,
                                            out.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))) == 0
            py = balanced_bands(costs, world, mr, grain=8)
            assert [(int(out[i]), int(out[i + 1])) for i in range(world)] == py, (H, world, mr)
            assert all(y1 - y0 >= mr for y0, y1 in py)
            if H % 8 == 0 and world * -(-mr // 8) <= H // 8:
                assert all(y0 % 8 == 0 for y0, _ in py), py


@pytest.mark.parametrize("world", [2, 3, 4, 5, 6, 7, 8])
@pytest.mark.parametrize("bands", ["equal", "rebalanced"])
def test_rccl_transfer_plans_pair_up(world, bands):
    """The RCCL branch's pairing (rs_mgpu_core.h halo_plan / gather_plan through issue_plan, the code
    rs_mgpu.hip posts to ncclSend/ncclRecv) recorded per rank on a fake link: every send has exactly one recv
    of equal bytes from the same peer on the same lane communicator, at 1080p and 4K with equal and
    cost-rebalanced bands, for each of the 3 run-ahead lanes."""
    from restir_amd.distributed import balanced_bands
    L = _harness()
    rng = np.random.default_rng(world)
    for W, H in ((1920, 1080), (3840, 2160)):
        if bands == "equal":
            b = [r * H // world for r in range(world + 1)]
        else:
            cost = rng.uniform(0.2, 3.0, H) * np.linspace(0.3, 2.5, H)
            b = [0] + [e for _, e in balanced_bands(cost, world, 8)]
        bounds = np.ascontiguousarray(b, np.int32)
        for lane in range(3):
            msg = ctypes.create_string_buffer(256)
            n = L.harness_plan_check(world, bounds.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), W, H, 5, lane, msg, 256)
            assert n > 0, (n, msg.value.decode())
            # 4 halo ops per interior boundary (send + recv each way) + 2 gather ops per non-root rank
            assert n == 4 * (world - 1) + 2 * (world - 1)


def test_rccl_plan_checker_rejects_broken_plans():
    L = _harness()
    assert L.harness_plan_check_negative() == 0
