"""GPU tests of the 8-wide tree of the per-lane walks (csrc/rs_wide_build.hip builds it on the device, csrc/rs_refit.h
refits it when the positions move; the reference's counterpart is Embree's rtcCommitScene, pg/Scene.cpp:15):

  * the GPU build equals the host restatement (rs_wide.h build_sah_host + SAH-optimal collapse, through
    tests/cpp/wide_harness.cpp) word for word -- node records, quantised planes and leaf-triangle order -- on the
    BASELINE scenes (C2's 2 k and C3's 248 k triangles) and on edge cases (one to three triangles, hundreds of
    coincident triangles: the degenerate-centroid split, random soups);
  * after rs_scene_update_positions the tree stays live with its topology, every dequantised child box contains
    the exact box of what is below it (numpy, from the new positions), and the per-lane wide walk returns the
    same closest / any hits as the binary lockstep walk (bit-identical) for random rays;
  * the C3 scene with moving lamps renders 8 temporal + spatial frames on the live wide tree within the frame
    tolerance of the oracle rendering the moved scene.
"""
import ctypes

import numpy as np
import pytest

import oracle_lib as O
from restir_amd import params as P
from restir_amd import scenes
from restir_amd.renderer import Renderer

import test_wide_bvh

pytestmark = pytest.mark.gpu


def _host_tree(pos):
    L = test_wide_bvh._lib()
    L.wide_build_host.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                  ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
    pos = np.ascontiguousarray(pos, np.float32)
    n = pos.shape[0]
    cap = max(1, n)
    words = np.zeros((cap, 20), np.uint32)
    prims = np.zeros(n, np.int32)
    npr, dep = ctypes.c_int(), ctypes.c_int()
    nn = L.wide_build_host(pos.ctypes.data, n, words.ctypes.data, cap, prims.ctypes.data, ctypes.byref(npr), ctypes.byref(dep))
    if nn == -2:
        return None
    assert nn > 0, nn
    return words[:nn], prims[:npr.value], dep.value


def _scene_from_positions(pos):
    base = scenes.cornell_box(8)
    n = pos.shape[0]
    nrm = np.tile(np.array([0, 0, 1] * 3, np.float32), (n, 1))
    return scenes.Scene(np.ascontiguousarray(pos, np.float32), nrm, np.zeros(n, np.uint32), base.materials[:1], base.camera)


def _soup(n, seed, dup=0):
    rng = np.random.default_rng(seed)
    c = rng.uniform(-1, 1, (n, 1, 3)).astype(np.float32) * np.array([4, 2, 1.5], np.float32)
    p = (c + rng.normal(scale=0.05, size=(n, 3, 3)).astype(np.float32)).reshape(n, 9)
    if dup:
        p[:dup] = p[0]                   # coincident triangles: every centroid equal in a > 256-triangle node
    return p


def _nonfinite():
    p = _soup(800, 5)
    p[17, 4] = np.nan                    # one NaN and one infinite coordinate
    p[401, 0] = np.inf
    return _scene_from_positions(p)


def _chain(n, ratio):
    """n triangles side by side along x, each `ratio` x the size of the previous: a binned / swept SAH split peels
    off the largest triangle at every level, so the source tree is a chain of depth n - 1 (the SAH-optimal 8-wide
    collapse of 100 such triangles needs exactly 8 levels; of 110, more than the walk's group stack holds)"""
    pos, x = [], 0.0
    for i in range(n):
        sz = ratio ** i
        pos.append([x, 0.0, 0.0, x + sz, 0.0, 0.0, x, sz, 0.0])
        x += sz
    return np.array(pos, np.float32)


CASES = {
    "c2": lambda: scenes.cornell_many_lights(1024),
    "c3": lambda: scenes.sponza_like(),
    "one": lambda: _scene_from_positions(_soup(1, 1)),
    "three": lambda: _scene_from_positions(_soup(3, 2)),
    "soup5k": lambda: _scene_from_positions(_soup(5000, 3)),
    "coincident": lambda: _scene_from_positions(_soup(1500, 4, dup=700)),
    "nonfinite": _nonfinite,             # the wide tree is optional -- the scene loads without one
    "depth8": lambda: _scene_from_positions(_chain(100, 1.5)),   # exactly the walk's stack depth
}


@pytest.mark.parametrize("case", list(CASES))
def test_wide_tree_gpu_equals_host(case):
    sc = CASES[case]()
    g = Renderer(8, 8)
    gs = g.load_scene(sc)
    got = gs.wide_tree()
    want = _host_tree(sc.positions)
    if want is None:
        assert got is None
        if case == "nonfinite":          # the scene still loads and its skip-pointer walks agree
            rng = np.random.default_rng(3)
            o = rng.uniform(-4, 4, (2000, 3)).astype(np.float32)
            d = rng.normal(size=(2000, 3)).astype(np.float32)
            d /= np.linalg.norm(d, axis=1, keepdims=True)
            for any_hit in (False, True):
                tl, pl = g.debug_trace(gs, o, d, 0.01, 3.0e38, any_hit=any_hit, lockstep=False)
                tk, pk = g.debug_trace(gs, o, d, 0.01, 3.0e38, any_hit=any_hit, lockstep=True)
                assert np.array_equal(pl, pk) and np.array_equal(tl, tk)
                if not any_hit:
                    assert (pl >= 0).any() and not np.isin(pl, [17, 401]).any()   # non-finite triangles: never hit
        return
    assert got is not None, f"{case}: the GPU built no wide tree"
    gw, gp, gd = got
    hw, hp, hd = want
    assert gd == hd and gw.shape == hw.shape, (case, gd, hd, gw.shape, hw.shape)
    bad = np.nonzero((gw != hw).any(axis=1))[0]
    assert bad.size == 0, f"{case}: {bad.size} of {len(hw)} nodes differ, first {bad[:5]}"
    assert np.array_equal(gp, hp), f"{case}: leaf-triangle order differs"
    print(f"[wide] {case}: {len(gw)} nodes, depth {gd}, build {gs.build_ms:.1f} ms (binary + wide tree)")


def _decode(words):
    """(ni, nv, child_base, tri_base, lo (N, 8, 3), hi (N, 8, 3)) of rs_wide.h's node words (float64 planes)."""
    w = words.astype(np.uint64)
    o = words[:, 0:3].copy().view(np.float32).astype(np.float64)
    e = np.stack([(w[:, 3] >> (8 * a)) & 0xFF for a in range(3)], 1).astype(np.int64) - 127
    ni = ((w[:, 3] >> 24) & 0xF).astype(np.int64)
    nv = (w[:, 3] >> 28).astype(np.int64)
    s = np.ldexp(1.0, e)                                     # (N, 3)

    def planes(w0):                                          # 6 words = x[0..3] x[4..7] y.. z.. -> (N, 8, 3)
        b = np.stack([(words[:, w0 + k][:, None] >> (8 * np.arange(4, dtype=np.uint32))) & 0xFF for k in range(6)], 1)
        b = b.reshape(-1, 3, 8).transpose(0, 2, 1).astype(np.float64)
        return b
    lo = o[:, None, :] + planes(6) * s[:, None, :]
    hi = o[:, None, :] + planes(12) * s[:, None, :]
    return ni, nv, words[:, 4].astype(np.int64), words[:, 5].astype(np.int64), lo, hi


def _check_conservative(words, prims, pos):
    ni, nv, cb, tb, lo, hi = _decode(words)
    p = pos.reshape(-1, 3, 3).astype(np.float64)
    tlo, thi = p.min(1), p.max(1)
    # a triangle with a non-finite coordinate can never be hit: the refit gives it a point box at the origin (or, for
    # a NaN the min/max order skips, the box of its finite coordinates); either way no containment is owed for it
    bad = ~np.isfinite(p).all(axis=(1, 2))
    N = len(words)
    blo = np.full((N, 3), np.inf)
    bhi = np.full((N, 3), -np.inf)
    for j in range(N - 1, -1, -1):                           # breadth-first: children after parents
        for i in range(nv[j]):
            if i < ni[j]:
                c = cb[j] + i
                clo, chi = blo[c], bhi[c]
            else:
                t = prims[tb[j] + i - ni[j]]
                if bad[t]:
                    continue
                clo, chi = tlo[t], thi[t]
            assert (lo[j, i] <= clo).all() and (hi[j, i] >= chi).all(), (j, i, lo[j, i], clo, hi[j, i], chi)
            blo[j] = np.minimum(blo[j], clo)
            bhi[j] = np.maximum(bhi[j], chi)


def test_wide_refit_after_updates():
    sc = scenes.sponza_like(target_tris=30_000, n_lamps=128)
    g = Renderer(8, 8)
    gs = g.load_scene(sc)
    w0, p0, d0 = gs.wide_tree()
    rng = np.random.default_rng(9)
    n = 6000
    lo, hi = sc.positions.reshape(-1, 3).min(0), sc.positions.reshape(-1, 3).max(0)
    for f in range(4):
        pos = scenes.moving_light_positions(sc, 17 * f + 5, 240, amplitude=0.2)
        if f == 3:                                           # the whole scene moves too
            pos = pos + np.float32(0.37)
        gs.update_positions(pos)
        w, p, d = gs.wide_tree()
        assert d == d0 and w.shape == w0.shape and np.array_equal(p, p0)
        assert np.array_equal(w[:, 3] >> 24, w0[:, 3] >> 24) and np.array_equal(w[:, 4:6], w0[:, 4:6])   # topology
        _check_conservative(w, p, pos)
        o = rng.uniform(lo, hi, (n, 3)).astype(np.float32) + (np.float32(0.37) if f == 3 else 0)
        dr = rng.normal(size=(n, 3)).astype(np.float32)
        dr /= np.linalg.norm(dr, axis=1, keepdims=True)
        for any_hit in (False, True):
            tl, pl = g.debug_trace(gs, o, dr, 0.01, 3.0e38, any_hit=any_hit, lockstep=False)   # wide per-lane
            tk, pk = g.debug_trace(gs, o, dr, 0.01, 3.0e38, any_hit=any_hit, lockstep=True)    # binary lockstep
            assert np.array_equal(pl, pk) and np.array_equal(tl, tk), (f, any_hit)
        fetches, _, lost = g.debug_trace(gs, o, dr, 0.01, 3.0e38, any_hit=True, wide_stats=True)
        assert ((fetches > 0) & (fetches != 0xFFFF)).all() and (lost == 0).all()

    # an update that moves vertices to NaN / inf on a live wide tree.  Those triangles get point boxes
    # (never hittable anyway), every other node keeps exact outward planes, and the wide per-lane walk still
    # equals the binary lockstep walk for the finite triangles that moved in the same update.
    # the whole scene shifts as well, so a node that kept its previous planes would miss its moved finite triangles
    pos = scenes.moving_light_positions(sc, 77, 240, amplitude=0.2) + np.float32(0.11)
    plain = np.nonzero(~sc.emissive_mask())[0]               # not an emitter: the light tables stay finite
    t_nan, t_inf = int(plain[1234]), int(plain[len(plain) // 2])
    pos[t_nan, 4] = np.nan
    pos[t_inf, 0] = np.inf
    gs.update_positions(pos)
    w, p, d = gs.wide_tree()
    assert d == d0 and w.shape == w0.shape
    _check_conservative(w, p, pos)
    o = rng.uniform(lo, hi, (n, 3)).astype(np.float32) + np.float32(0.11)
    dr = rng.normal(size=(n, 3)).astype(np.float32)
    dr /= np.linalg.norm(dr, axis=1, keepdims=True)
    for any_hit in (False, True):
        tl, pl = g.debug_trace(gs, o, dr, 0.01, 3.0e38, any_hit=any_hit, lockstep=False)
        tk, pk = g.debug_trace(gs, o, dr, 0.01, 3.0e38, any_hit=any_hit, lockstep=True)
        assert np.array_equal(pl, pk) and np.array_equal(tl, tk), ("nonfinite update", any_hit)
        if not any_hit:
            assert (pl >= 0).any() and not np.isin(pl, [t_nan, t_inf]).any()


def test_c3_moving_lamps_on_live_wide_tree():
    """C3's lamps move for 8 frames (rs_scene_update_positions: light tables + binary and 8-wide
    refit every frame) with the per-lane wide walk live; frames vs the oracle rendering the moved scene."""
    sc = scenes.sponza_like()
    W, H = 480, 270
    prm = P.c3_params()
    g = Renderer(W, H)
    g.set_traversal("lane")
    gs = g.load_scene(sc)
    o = O.OracleRenderer(W, H)
    for f in range(8):
        pos = scenes.moving_light_positions(sc, 9 * f, 240, amplitude=0.1)
        gs.update_positions(pos)
        assert gs.wide_tree() is not None
        cam = scenes.orbit_camera(sc.camera, f, 240, 0.3)
        a = g.produce_restir(gs, cam, prm, f).copy()
        moved = scenes.Scene(pos, sc.normals, sc.tri_material, sc.materials, sc.camera)
        b = o.render(O.OracleScene(moved), cam, prm, f)
        diff = np.linalg.norm(a.astype(np.float64) - b, axis=-1)
        rel = diff / np.maximum(np.linalg.norm(b.astype(np.float64), axis=-1), 1e-3)
        frac, mean = float((rel <= 1e-4).mean()), float(rel.mean())
        print(f"[parity] C3 moving lamps frame {f}: {100 * frac:.4f} % within 1e-4, mean {mean:.3g}")
        assert frac >= 0.995 and mean <= 1e-4, (f, frac, mean)


def test_deep_tree_falls_back_to_skip_walks():
    """a scene whose SAH-optimal collapse does not fit the walk's 8-level group stack (_chain(110)) loads
    without a wide tree; rs_scene_walk_info says why (too_deep), the host restatement agrees (no plan within depth 8),
    and the per-lane walks -- on the skip pointers now -- return the lockstep walks' and the oracle's hits bit for
    bit.  The 100-triangle chain (depth exactly 8) keeps its tree (CASES["depth8"] above)."""
    pos = _chain(110, 1.5)
    assert _host_tree(pos) is None
    sc = _scene_from_positions(pos)
    g = Renderer(8, 8)
    gs = g.load_scene(sc)
    assert gs.walk_info() == {"wide_nodes": 0, "wide_depth": -1, "status": "too_deep"}, gs.walk_info()
    assert gs.wide_tree() is None
    ok = g.load_scene(_scene_from_positions(_chain(100, 1.5)))
    info = ok.walk_info()
    assert info["status"] == "live" and info["wide_depth"] == 8 and info["wide_nodes"] > 0, info
    # rays aimed at a random point of a random triangle from a scale-relative distance (every size class is hit;
    # a fifth of them in random directions)
    rng = np.random.default_rng(4)
    n = 8000
    tri = rng.integers(0, len(pos), n)
    p3 = pos.reshape(-1, 3, 3).astype(np.float64)
    b = rng.dirichlet((1.0, 1.0, 1.0), n)
    tgt = np.einsum("nk,nkc->nc", b, p3[tri])
    size = p3[tri, 1, 0] - p3[tri, 0, 0]
    o = (tgt + rng.normal(size=(n, 3)) * size[:, None] * 2.0).astype(np.float32)
    d = tgt - o.astype(np.float64)
    d[::5] = rng.normal(size=d[::5].shape)
    d = (d / np.linalg.norm(d, axis=1, keepdims=True)).astype(np.float32)   # normalised in float64: no overflow
    os_ = O.OracleScene(sc)
    tr, pr = os_.trace_closest(o, d, 0.0, 3.0e38)
    assert (pr >= 0).mean() > 0.5, (pr >= 0).mean()
    tf = np.where(tr > 0, tr * np.float32(0.999), np.float32(3.0e38)).astype(np.float32)
    tf[::3] = np.where(tr[::3] > 0, tr[::3] * np.float32(1.001), np.float32(3.0e38))
    anyr = os_.trace_any(o, d, np.zeros(n, np.float32), tf)
    for lockstep in (False, True):
        t, prim = g.debug_trace(gs, o, d, 0.0, 3.0e38, any_hit=False, lockstep=lockstep)
        assert np.array_equal(prim, pr) and np.array_equal(t, tr), lockstep
        _, anyg = g.debug_trace(gs, o, d, np.zeros(n, np.float32), tf, any_hit=True, lockstep=lockstep)
        assert np.array_equal(anyg, anyr), lockstep
