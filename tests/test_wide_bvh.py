"""CPU tests of the 8-wide tree of the per-lane walks (restir-embree_amd/csrc/rs_wide.h, collapsed from the
PLOC tree after every build, walked by rs_scene.h wide_walk): breadth-first layout, every triangle in
exactly one leaf slot, outward-quantised child boxes that are exact floats, and -- with the walk's box test
restated on the CPU with the same float operations -- closest hits (t, triangle, tie rule) and any-hit
answers identical to brute force over all triangles, for random, axis-parallel and on-plane rays
(tests/cpp/wide_harness.cpp)."""
import ctypes
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "cpp", "wide_harness.cpp")
HDR = os.path.join(ROOT, "restir-embree_amd", "csrc", "rs_wide.h")
SO = os.path.join(ROOT, "oracle", "_build", "libwide_harness.so")


def _lib():
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    if not os.path.exists(SO) or os.path.getmtime(SO) < max(os.path.getmtime(SRC), os.path.getmtime(HDR)):
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-shared", "-fPIC", "-o", SO, SRC])
    L = ctypes.CDLL(SO)
    L.wide_check.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.POINTER(ctypes.c_int), ctypes.c_char_p, ctypes.c_int,
                             ctypes.c_int]
    L.wide_query.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.c_int]
    return L


@pytest.mark.parametrize("collapse", [0, 1, 2, 3], ids=["greedy", "sah", "sah-hostsah", "hostsah-coincident"])
@pytest.mark.parametrize("n,seed", [(1, 1), (2, 2), (7, 3), (9, 4), (64, 5), (1000, 6), (20000, 7)])
def test_wide_tree_structure_and_conservative_boxes(n, seed, collapse):
    L = _lib()
    msg = ctypes.create_string_buffer(256)
    depth = ctypes.c_int(-1)
    nn = L.wide_check(n, seed, ctypes.byref(depth), msg, 256, collapse)
    assert nn > 0, msg.value.decode()
    assert depth.value >= 0 and (n <= 8 or depth.value >= 1)


@pytest.mark.parametrize("collapse", [0, 1, 2, 3], ids=["greedy", "sah", "sah-hostsah", "hostsah-coincident"])
@pytest.mark.parametrize("n,seed", [(1, 11), (5, 12), (300, 13), (5000, 14)])
def test_wide_walk_matches_brute_force(n, seed, collapse):
    L = _lib()
    hits = ctypes.c_int(0)
    rc = L.wide_query(n, seed, 4000, ctypes.byref(hits), collapse)
    assert rc == 4000, f"ray {-rc - 1000} differs from brute force"
    assert n < 100 or hits.value > 100


def test_nonfinite_geometry_builds_no_wide_tree():
    """non-finite vertices leave the scene without a wide tree (the walks take the skip pointers)
    instead of failing the load or sorting NaN centroids (tests/test_gpu_wide.py checks the GPU builder)."""
    import numpy as np
    L = _lib()
    L.wide_build_host.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                  ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
    rng = np.random.default_rng(2)
    for bad in (np.nan, np.inf, -np.inf):
        pos = rng.uniform(-1, 1, (300, 9)).astype(np.float32)
        pos[123, 5] = bad
        words = np.zeros((300, 20), np.uint32)
        prims = np.zeros(300, np.int32)
        npr, dep = ctypes.c_int(), ctypes.c_int()
        assert L.wide_build_host(pos.ctypes.data, 300, words.ctypes.data, 300, prims.ctypes.data, ctypes.byref(npr),
                                 ctypes.byref(dep)) == -2
