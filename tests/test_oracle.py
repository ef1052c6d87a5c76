"""CPU tests: the oracle (CPU restatement) pinned against the golden vectors generated from the
reference's vendored third-party code (Boost 1.86 ibeta, glm 0.9.9), plus its own invariants.

The oracle is test infrastructure (oracle/restir_oracle.c); see DESIGN.md "Oracle" for what is
pinned and what is parity-unpinned."""
import ctypes
import json
import math
import os

import numpy as np
import pytest

import oracle_lib as O
from restir_amd import params as P
from restir_amd import scenes

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _kat(name):
    with open(os.path.join(GOLD, name)) as f:
        return json.load(f)


# ---------------------------------------------------------------- Boost-pinned Phong normalisation
def test_ibeta_matches_boost():
    L = O.lib()
    for x, a, b, v in _kat("ibeta_kat.json")["ibeta"]:
        r = L.or_ibeta(x, a, b)
        if v == 0:
            assert r == 0.0
        else:
            assert abs(r - v) / abs(v) < 1e-11, (x, a, b, v, r)


def _calc_I_M_correctly_rounded(L, c, n):
    """calc_I_M (pg/MaterialPhong.cpp:224-244) in the reference's float operation order, every libm call
    (lgammaf, expf, powf) replaced by Python's double-precision math rounded once to float32 -- the correctly
    rounded float results -- and the Boost-pinned ibeta (test_ibeta_matches_boost)."""
    f = np.float32
    c, n = f(c), f(n)
    s2 = min(max(f(f(1) - c * c), f(0)), f(1))
    halfn = f(f(0.5) * n)
    neg = c
    if n >= f(1e-18):
        neg = f(neg * f(halfn * f(L.or_ibeta(float(s2), float(halfn), 0.5))))
    lg = lambda v: f(math.lgamma(float(v)))                                    # noqa: E731
    gq = f(math.exp(float(f(lg(halfn + f(0.5)) - lg(halfn + f(1))))))
    pw = f(math.pow(float(s2), float(halfn)))
    two_pi, root_pi = f(6.28318530717958647692), f(1.772453850905516027)
    return f(f(f(two_pi * c) + f(f(root_pi * gq) * f(pw - neg))) / f(n + f(2)))


def test_calc_I_M_vs_boost():
    """calc_I_M (pg/MaterialPhong.cpp:228-244) with the genuine boost::math::beta.  The oracle (and the kernels,
    rs_libm.h) evaluate lgammaf / expf / powf correctly rounded: bit-exact against the independent correctly
    rounded restatement above at all 130 points.  The KAT itself was generated with glibc's lgammaf / expf /
    powf; glibc's lgammaf is off by an ulp at some arguments, and the formula's cancellation (pow(s^2, n/2) -
    negterm at grazing angles and high exponents) magnifies that: the KAT agrees bit for bit at 114 of the 130
    points and within 3.1e-5 relative at the other 16 (n = 128, n.v = 0: 446 ulps)."""
    L = O.lib()
    kat = _kat("ibeta_kat.json")["calc_I_M"]
    exact = 0
    for c, n, v in kat:
        got = np.float32(L.or_calc_I_M(c, n))
        assert got == _calc_I_M_correctly_rounded(L, c, n), (c, n)
        assert abs(float(got) - v) <= 3.1e-5 * abs(v), (c, n, got, v)
        exact += got == np.float32(v)
    assert exact >= 114, exact


# ---------------------------------------------------------------- glm-pinned camera / reprojection
def test_camera_matrices_and_rays_bit_exact_vs_glm():
    L = O.lib()
    for c in _kat("glm_kat.json")["cameras"]:
        cam = np.array(c["cam"], np.float32)
        out = np.zeros(36, np.float32)
        for px, py, *dw in c["rays"]:
            L.or_camera_kat(O._ptr(cam), c["W"], c["H"], px, py, O._ptr(out))
            assert np.array_equal(out[:16], np.array(c["view"], np.float32))
            assert np.array_equal(out[16:32], np.array(c["inv_view"], np.float32))
            assert out[32] == np.float32(c["focal"])
            assert np.array_equal(out[33:36], np.array(dw, np.float32)), (px, py)


def test_reprojection_vs_glm():
    L = O.lib()
    for c in _kat("glm_kat.json")["cameras"]:
        cam = np.array(c["cam"], np.float32)
        for x, y, z, sx, sy in c["reproject"]:
            ws = np.array([x, y, z], np.float32)
            xy = np.zeros(2, np.int32)
            L.or_reproject_kat(O._ptr(cam), c["W"], c["H"], O._ptr(ws), O._ptr(xy, O._i32p))
            assert (int(xy[0]), int(xy[1])) == (sx, sy)


def test_disk_offset_truncation_semantics():
    """glm vec2 -> ivec2 conversion truncates toward zero (pg/ReSTIRIntegrator.cpp:338)."""
    for ox, oy, ix, iy in _kat("glm_kat.json")["disk_trunc"]:
        assert (int(np.float32(ox)), int(np.float32(oy))) == (ix, iy)


# ---------------------------------------------------------------- reference header-only code
# tests/golden/refheaders_kat.json: the reference's own Reservoir.h / Distribution.h / GBufferElement.h /
# utils.h compiled with its vendored glm (oracle/kat/gen_refheaders.cpp), U streams replayed.
def test_reservoir_add_sample_bit_exact_vs_reference():
    """Reservoir::addSample / capConfidence / hasSample / LightSample::isValid (pg/Reservoir.h:6-59): the
    oracle's res_update/res_take/res_cap consume the same draws, pick the same sample and accumulate
    the bit-identical w_sum and confidence."""
    L = O.lib()
    for case in _kat("refheaders_kat.json")["reservoir"]:
        w = np.array(case["w"], np.float32)
        conf = np.array(case["conf"], np.int32)
        u = np.array(case["u"], np.float32)
        n = len(w)
        wsum = np.zeros(1, np.float32)
        out = np.zeros(6, np.int32)
        taken = np.zeros(n, np.int32)
        L.or_kat_reservoir(O._ptr(w), O._ptr(conf, O._i32p), n, O._ptr(u), len(u), case["cap"], O._ptr(wsum),
                           O._ptr(out, O._i32p), O._ptr(taken, O._i32p))
        assert wsum[0] == np.float32(case["w_sum"])
        assert list(out) == [case["chosen"], case["draws"], case["confidence"], case["confidence_capped"],
                             case["has_sample"], case["valid"]], case
        assert list(np.nonzero(taken)[0]) == case["taken"]


def test_light_sample_is_valid_vs_reference():
    L = O.lib()
    for *v, ok in _kat("refheaders_kat.json")["light_sample_valid"]:
        a = np.array(v, np.float32)
        assert L.or_kat_light_sample_valid(O._ptr(a[0:3]), O._ptr(a[3:6]), O._ptr(a[6:9])) == ok, v


def test_cosine_distributions_vs_reference():
    """CosineWeightedDistribution / CosineLobeDistribution sample + getPdf (pg/Distribution.h:7-68) with
    the same (r1, r2) draws, incl. normals along the axes (Utils::orthogonal's branches), r1 = 0,
    r2 -> 1 and lobe exponents 0..1000.  The KAT ran the reference's header with glibc's sinf / cosf / powf,
    which are not correctly rounded at ~1.3 % / 0.13 % of arguments; the oracle (and the kernels) use
    rs_libm.h's correctly rounded ones (test_libm_correctly_rounded).  Directions and pdfs are bit-identical
    wherever the two libms agree (all but 2 of 192 and 4 of 144 rows); at the others a last-ulp angle moves a
    unit-vector component by <= 2e-7 absolute."""
    L = O.lib()
    kat = _kat("refheaders_kat.json")
    out = np.zeros(5, np.float32)
    exact = {"cosine_weighted": 0, "cosine_lobe": 0}
    for name in exact:
        for row in kat[name]:
            r = np.array(row, np.float32)
            if name == "cosine_weighted":
                L.or_kat_cosine(O._ptr(r[0:3]), r[3], r[4], O._ptr(r[9:12]), O._ptr(out))
                d, pdf = r[5:8], r[[8, 12]]
            else:
                L.or_kat_lobe(O._ptr(r[0:3]), r[3], r[4], r[5], O._ptr(r[10:13]), O._ptr(out))
                d, pdf = r[6:9], r[[9, 13]]
            exact[name] += bool(np.array_equal(out[:3], d) and np.array_equal(out[3:5], pdf))
            assert np.abs(out[:3] - d).max() <= 2e-7, row
            assert np.allclose(out[3:5], pdf, rtol=1e-6, atol=0), row
    assert exact["cosine_weighted"] >= 190 and exact["cosine_lobe"] >= 140, exact
    assert len(kat["cosine_weighted"]) >= 150 and len(kat["cosine_lobe"]) >= 100


def test_libm_correctly_rounded():
    """rs_libm.h (shared by the oracle and the kernels): powf / expf / lgammaf / sinf / cosf equal the float32
    rounding of numpy's / math's double-precision values on dense random grids over the path's argument
    ranges, and the double log / exp / log1p / lgamma of the incomplete beta are within 2 ulp / 2e-12."""
    L = O.lib()
    rng = np.random.default_rng(7)
    n = 200_000
    x = rng.uniform(0, 1, n).astype(np.float32)
    y = np.concatenate([rng.uniform(0, 1000, n // 2), rng.uniform(0, 4, n // 2)]).astype(np.float32)
    got = O.libm_f2("powf", x, y)
    assert np.array_equal(got, np.power(x.astype(np.float64), y.astype(np.float64)).astype(np.float32))
    e = rng.uniform(-100, 88, n).astype(np.float32)
    assert np.array_equal(O.libm_f1("expf", e), np.exp(e.astype(np.float64)).astype(np.float32))
    g = rng.uniform(0.5, 600, 20_000).astype(np.float32)
    ref = np.array([math.lgamma(float(v)) for v in g]).astype(np.float32)
    assert np.array_equal(O.libm_f1("lgammaf", g), ref)
    a = (rng.uniform(0, 1, n).astype(np.float32) * np.float32(2 * np.pi)).astype(np.float32)
    assert np.array_equal(O.libm_f1("sinf", a), np.sin(a.astype(np.float64)).astype(np.float32))
    assert np.array_equal(O.libm_f1("cosf", a), np.cos(a.astype(np.float64)).astype(np.float32))
    # special values of powf (C99 F.10.4.4)
    xs = np.array([0, 0, -2, -2, np.inf, 0.5, 2, 1, np.nan, -0.0, 0], np.float32)
    ys = np.array([2, -1, 3, 0.5, 2, np.inf, np.inf, np.nan, 0, 3, 0], np.float32)
    with np.errstate(all="ignore"):
        assert np.array_equal(O.libm_f2("powf", xs, ys), np.power(xs, ys), equal_nan=True)
    d = np.exp(rng.uniform(-700, 700, n))
    got = O.libm_d1("log", d)
    ref = np.log(d)
    assert np.all(np.abs(got - ref) <= 2 * np.spacing(np.abs(ref)))
    t = rng.uniform(-700, 700, n)
    assert np.all(np.abs(O.libm_d1("exp", t) - np.exp(t)) <= np.spacing(np.exp(t)))
    u = -rng.uniform(0, 1, n)
    assert np.all(np.abs(O.libm_d1("log1p", u) - np.log1p(u)) <= 2 * np.spacing(np.abs(np.log1p(u))))
    v = rng.uniform(1e-6, 600, 20_000)
    assert np.allclose(O.libm_d1("lgamma", v), [math.lgamma(q) for q in v], rtol=0, atol=2e-12)


def test_utils_inline_helpers_vs_reference():
    """Utils::powerHeuristic (= DirectMISIntegrator::powerHeuristic) and Utils::maxComponent (pg/utils.h:53-63)."""
    L = O.lib()
    kat = _kat("refheaders_kat.json")
    for a, b, v in kat["power_heuristic"]:
        assert np.float32(L.or_kat_power_heuristic(a, b)) == np.float32(v)
    for *xyz, v in kat["max_component"]:
        a = np.array(xyz, np.float32)
        assert np.float32(L.or_kat_max_component(O._ptr(a))) == np.float32(v)


def test_mis_weights_bit_exact_vs_reference():
    """ReSTIRIntegrator::m_area / m_brdf (pg/ReSTIRIntegrator.h:62-74, compiled from the reference header)
    over M_Area/M_Brdf in {0..32} x pdf pairs incl. both zero, one zero, tiny and huge; CenterSampler
    returns the pixel corner (0, 0) (pg/PixelSampler.h:12-17)."""
    L = O.lib()
    kat = _kat("refheaders_kat.json")
    out = np.zeros(2, np.float32)
    for a, b, pa, pb, wa, wb in kat["mis_area_brdf"]:
        L.or_kat_mis(a, b, pa, pb, O._ptr(out))       # M_Area = 0 gives inf / nan: compared as such
        assert np.array_equal(out, np.array([float(wa), float(wb)], np.float32), equal_nan=True), (a, b, pa, pb)
    assert kat["center_sampler"] == [0, 0]


def test_gbuffer_layout_vs_reference():
    """GBuffer::setAt (pg/GBufferElement.h:59-70) stores pixel (x, y) at y*W+x of each SoA array -- the
    row-major pixel index the oracle and the device G-buffer use; isValidForReSTIR <=> zero emission."""
    g = _kat("refheaders_kat.json")["gbuffer"]
    W = g["size"][0]
    where = {i: j for i, j, *_ in g["linear_index"]}
    for x, y, i, valid in g["set"]:
        assert where[i] == y * W + x
        assert valid == (0 if i == 2 else 1)
    assert g["sizeof_element"] == 72          # 69 B of payload, padded to 72


def test_reference_equivalent_ray_count():
    """The oracle's count of the rays the reference would trace (every rtcIntersect1 and every
    testOcclusion its code reaches, incl. zero-contribution shadow rays and re-evaluated final p-hats)
    against a closed form on a scene where every term is known: C1 defaults (A=1, B=1, no reuse) with the
    reference's Appendix-D model per non-emissive pixel = 1 primary + 1 BRDF ray + (A + B + 1) shadow
    rays for valid samples + 1 shade ray."""
    import oracle_lib as O
    sc = scenes.cornell_box(8)
    W, H = 48, 40
    r = O.OracleRenderer(W, H)
    r.render(O.OracleScene(sc), sc.camera, P.default_params(), 0)
    g = r.gbuffer()
    res = r.reservoirs()
    emissive = g[..., 12:15].max(-1) > 0
    n_px = W * H
    # upper bound: every non-emissive pixel traces 1 BRDF ray + A + B + final + shade shadow rays
    upper = n_px + int((~emissive).sum()) * (1 + 1 + 1 + 1 + 1)
    assert r.rays <= r.reference_rays <= upper
    # lower bound: primary rays + BRDF rays + the area candidate's shadow ray (always a valid sample)
    assert r.reference_rays >= n_px + 2 * int((~emissive).sum())
    # with M-capped reuse the reference traces many more rays than the restatement's skipped count
    r2 = O.OracleRenderer(W, H)
    r2.render(O.OracleScene(scenes.cornell_many_lights(64)), sc.camera, P.metric_params(), 0)
    assert r2.reference_rays > r2.rays


# ---------------------------------------------------------------- counter RNG
def test_rng_deterministic_and_uniform():
    L = O.lib()
    a = np.array([L.or_rng_u(123, 0, 1, p, n) for p in range(64) for n in range(64)], np.float64)
    b = np.array([L.or_rng_u(123, 0, 1, p, n) for p in range(64) for n in range(64)], np.float64)
    assert np.array_equal(a, b)
    assert a.min() >= 0.0 and a.max() < 1.0
    assert abs(a.mean() - 0.5) < 0.02
    assert abs(a.var() - 1 / 12) < 0.01
    # streams differ across pixel / frame / pass / seed
    base = L.or_rng_u(123, 0, 1, 7, 0)
    assert len({base, L.or_rng_u(123, 0, 1, 8, 0), L.or_rng_u(123, 1, 1, 7, 0), L.or_rng_u(123, 0, 2, 7, 0),
                L.or_rng_u(124, 0, 1, 7, 0)}) == 5


# ---------------------------------------------------------------- light CDF (pg/TriangleCDF.cpp)
def test_emissive_cdf():
    sc = scenes.cornell_many_lights(64, size=0.05)
    os_ = O.OracleScene(sc)
    assert os_.n_emissive == 128 == int(sc.emissive_mask().sum())
    cdf, pick, area = os_.cdf()
    assert np.all(np.diff(cdf) >= 0)
    assert abs(cdf[-1] - 1.0) < 1e-5
    assert abs(pick.sum() - 1.0) < 1e-5
    np.testing.assert_allclose(area, np.full(128, 0.5 * 0.05 * 0.05), rtol=1e-5)


# ---------------------------------------------------------------- oracle BVH vs brute force
def _brute_closest(sc, o, d, tnear, tfar):
    """numpy Moller-Trumbore over every triangle, float32, same operation order and tie rule."""
    f = np.float32
    P = sc.positions.astype(np.float32)
    v0, v1, v2 = P[:, 0:3], P[:, 3:6], P[:, 6:9]
    e1, e2 = v1 - v0, v2 - v0

    def dot(a, b):
        m = a * b
        return (m[..., 0] + m[..., 1]) + m[..., 2]

    def cross(x, y):
        return np.stack([x[..., 1] * y[..., 2] - y[..., 1] * x[..., 2], x[..., 2] * y[..., 0] - y[..., 2] * x[..., 0],
                         x[..., 0] * y[..., 1] - y[..., 0] * x[..., 1]], -1)

    ts = np.full(o.shape[0], -1.0, np.float32)
    prims = np.full(o.shape[0], -1, np.int32)
    with np.errstate(all="ignore"):
        for i in range(o.shape[0]):
            dd = np.broadcast_to(d[i], e2.shape).astype(np.float32)
            p = cross(dd, e2)
            det = dot(e1, p)
            inv = f(1.0) / det
            sv = (o[i] - v0).astype(np.float32)
            u = dot(sv, p) * inv
            q = cross(sv, e1)
            v = dot(dd, q) * inv
            t = dot(e2, q) * inv
            ok = (det != 0) & (u >= 0) & (u <= 1) & (v >= 0) & (u + v <= 1) & (t >= f(tnear)) & (t <= f(tfar))
            if ok.any():
                idx = np.flatnonzero(ok)
                best = idx[np.lexsort((idx, t[idx]))[0]]
                ts[i], prims[i] = t[best], best
    return ts, prims


@pytest.mark.parametrize("wide", [False, True])
def test_oracle_bvh_matches_brute_force(wide):
    """Both oracle walks (the binary stack walk and the 8-wide AVX2 walk of the CPU baseline) find the
    brute-force hits."""
    sc = scenes.cornell_many_lights(48)
    os_ = O.OracleScene(sc, wide=wide)
    assert os_.wide == wide
    rng = np.random.default_rng(3)
    n = 400
    o = rng.uniform([-0.9, -0.9, 0.1], [0.9, 0.9, 1.9], (n, 3)).astype(np.float32)
    d = rng.normal(size=(n, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    t, prim = os_.trace_closest(o, d, 0.01, 3.0e38)
    tb, pb = _brute_closest(sc, o, d, 0.01, 3.0e38)
    assert np.array_equal(prim, pb)
    assert np.array_equal(t, tb)
    # any-hit agrees with closest-hit on segment queries
    tf = np.where(tb > 0, tb * np.float32(0.5), np.float32(1.0)).astype(np.float32)
    anyh = os_.trace_any(o, d, np.full(n, 0.01, np.float32), tf)
    tb2, _ = _brute_closest_segment(sc, o, d, tf)
    assert np.array_equal(anyh.astype(bool), tb2 >= 0)


def _brute_closest_segment(sc, o, d, tf):
    ts = np.full(o.shape[0], -1.0, np.float32)
    prims = np.full(o.shape[0], -1, np.int32)
    for i in range(o.shape[0]):
        t, p = _brute_closest(sc, o[i:i + 1], d[i:i + 1], 0.01, float(tf[i]))
        ts[i], prims[i] = t[0], p[0]
    return ts, prims


# ---------------------------------------------------------------- oracle frame invariants
def _render(sc, W, H, prm, frames=1, threads=None, cam=None):
    if threads:
        O.lib().or_set_num_threads(threads)
    os_ = O.OracleScene(sc)
    r = O.OracleRenderer(W, H)
    img = None
    for f in range(frames):
        img = r.render(os_, cam(f) if cam else sc.camera, prm, f)
    return img, r


@pytest.mark.parametrize("name", ["cornell", "sponza"])
def test_oracle_wide_walk_frames_identical(name):
    """The CPU baseline's 8-wide walk renders the same frames as the binary walk (any tree, same hits)."""
    sc = scenes.cornell_many_lights(64) if name == "cornell" else scenes.sponza_like(target_tris=20_000, n_lamps=64)
    prm = P.default_params(m_area=8, m_brdf=1, do_spatial=1, spatial_neighbors=3, do_temporal=1)
    cam = lambda f: scenes.orbit_camera(sc.camera, f, 24, 0.3)
    imgs = []
    for wide in (False, True):
        os_ = O.OracleScene(sc, wide=wide)
        assert os_.wide == wide
        r = O.OracleRenderer(64, 48)
        imgs.append([r.render(os_, cam(f), prm, f).copy() for f in range(3)])
    for a, b in zip(*imgs):
        assert np.array_equal(a, b)


@pytest.mark.parametrize("mis", [0, 1, 2, 3, 4])
def test_oracle_deterministic_across_thread_counts(mis):
    """Per-pixel counter RNG: the frame does not depend on OpenMP scheduling (the reference's shared
    mt19937 does, pg/utils.cpp:175 -- SURVEY.md §2.3)."""
    sc = scenes.cornell_box(8)
    prm = P.default_params(m_area=4, do_spatial=1, spatial_neighbors=3, do_temporal=1, spatial_mis=mis)
    cam = lambda f: scenes.orbit_camera(sc.camera, f, 24, 0.2)
    a, _ = _render(sc, 48, 40, prm, frames=2, threads=1, cam=cam)
    b, _ = _render(sc, 48, 40, prm, frames=2, threads=8, cam=cam)
    O.lib().or_set_num_threads(os.cpu_count() or 1)
    assert np.array_equal(a, b)


def test_oracle_image_sanity_c1():
    sc = scenes.cornell_box(8)
    img, r = _render(sc, 64, 64, P.default_params())
    assert np.isfinite(img).all() and (img >= 0).all()
    g = r.gbuffer()
    miss = (g[..., 16] == 0)
    # miss pixels show the background colour (useSkybox=false path, pg/ReSTIRIntegrator.cpp:231)
    assert np.allclose(img[miss], 0.5)
    assert img[~miss].mean() > 0.05
    res = r.reservoirs()
    assert (res[..., 11] <= 20).all()            # confidence cap (pg/Reservoir.h:54-56)


def test_oracle_no_emitters_is_emission_only():
    sc = scenes.cornell_box(8)
    keep = ~sc.emissive_mask()
    sc2 = scenes.Scene(sc.positions[keep], sc.normals[keep], sc.tri_material[keep], sc.materials, sc.camera)
    img, r = _render(sc2, 32, 32, P.metric_params())
    g = r.gbuffer()
    assert np.array_equal(img, np.where(g[..., 16:17] == 0, np.float32(0.5), np.float32(0.0)).repeat(3, -1))


def test_oracle_rejects_skybox():
    sc = scenes.cornell_box(8)
    os_ = O.OracleScene(sc)
    r = O.OracleRenderer(8, 8)
    with pytest.raises(RuntimeError):
        r.render(os_, sc.camera, P.default_params(use_skybox=1), 0)


def test_params_struct_layout():
    assert ctypes.sizeof(P.FrameParams) == 88


def test_post_frame_restatement():
    """Oracle post-frame (accumulate / ACES / sRGB compress / mean-variance, pg/simpleguidx11.cpp:246-333,
    pg/utils.cpp:191-229) against an independent numpy float32 restatement of the same formulas."""
    from oracle_lib import OraclePost
    rng = np.random.default_rng(3)
    W, H = 13, 7
    frames = [rng.uniform(-0.2, 3.0, size=(H, W, 3)).astype(np.float32) for _ in range(4)]
    frames[0][0, 0] = [0.0, 1e-4, 0.0031]      # compress edge values / linear segment
    post = OraclePost(W, H)
    acc = np.zeros((H, W, 3), np.float32)
    f32 = np.float32

    def aces(x):
        v = (x * (f32(2.51) * x + f32(0.03))) / (x * (f32(2.43) * x + f32(0.59)) + f32(0.14))
        v = np.where(v < 0, f32(0), v)         # glm max(v, 0) select form
        return np.where(f32(1) < v, f32(1), v)  # glm min(v, 1)

    def compress(u):
        out = np.where(u <= 0, f32(0), np.where(u >= 1, f32(1), f32(0)))
        mid = (u > 0) & (u < 1)
        lin = mid & (u.astype(np.float64) <= 0.0031308)
        out = np.where(lin, u * f32(12.92), out)
        pw = f32(1.055) * np.power(u, f32(1.0) / f32(2.4), dtype=np.float32) - f32(0.055)
        return np.where(mid & ~lin, pw, out).astype(np.float32)

    for n, fr in enumerate(frames):
        a = f32(1.0) / f32(n + 1)
        acc = (acc * (f32(1) - a) + fr * a).astype(np.float32)
        disp, st = post.apply(fr, accumulate=True)
        assert st["acc_frames_used"] == n
        np.testing.assert_array_equal(post.acc, acc)
        ref = compress(aces(acc))
        np.testing.assert_allclose(disp[..., :3], ref, rtol=0, atol=2e-7)
        assert (disp[..., 3] == 1.0).all()
        m = ((acc[..., 0] + acc[..., 1] + acc[..., 2]) / f32(3)).astype(np.float32)
        mean = m.astype(np.float64).sum() / (W * H)
        var = (m * m).astype(np.float64).sum() / (W * H) - mean * mean
        assert abs(st["mean"] - mean) <= 1e-12 * max(1.0, abs(mean)) and abs(st["variance"] - var) <= 1e-9
    # no accumulation: accFrameCtr restarts, the accumulator becomes the frame
    post2 = OraclePost(W, H)
    for fr in frames[:2]:
        _, st = post2.apply(fr, accumulate=False, tonemap=False, gamma_correct=False)
        assert st["acc_frames_used"] == 0
        np.testing.assert_array_equal(post2.acc, fr)


@pytest.mark.parametrize("which", ["c1", "phong"])
def test_direct_mis_and_restir_converge_to_the_same_image(which):
    """§8f-3 ground truth: the MIS direct integrator (or_render_direct_mis) and ReSTIR's RIS (initial
    pass only -- unbiased) are two estimators of the same direct illumination; converged, their images
    agree.  Lambert Cornell box and a Phong scene (the lobe-sampling / I_M path).
    Excluded: surfaces facing down (normal.z < -0.5), which see the emitters' back faces (the lamps hang
    just below the ceiling).  There the reference's own estimators disagree: ReSTIR's p-hat uses a
    two-sided |cos theta_y| (pg/ReSTIRIntegrator.cpp:197) and counts back-face emission, the MIS light
    sample is one-sided (pg/DirectMISIntegrator.cpp:67) while its BRDF sample counts it through the
    ray-facing hit normal (pg/Intersection.h:93-98).  Both quirks are reproduced as they are."""
    if which == "c1":
        sc, prm, W, H = scenes.cornell_box(8), P.default_params(m_area=4), 48, 36
    else:
        sc, prm, W, H = scenes.sponza_like(target_tris=6_000, n_lamps=64), P.default_params(m_area=4), 48, 27
    o, os_ = O.OracleRenderer(W, H), O.OracleScene(sc)
    gt = o.render_direct_mis(os_, sc.camera, prm, 0, spp=256).astype(np.float64)
    again = o.render_direct_mis(os_, sc.camera, prm, 0, spp=256)
    assert np.array_equal(gt, again)                                     # deterministic
    assert not np.array_equal(o.render_direct_mis(os_, sc.camera, prm, 1, spp=1),
                              o.render_direct_mis(os_, sc.camera, prm, 2, spp=1))   # frame-keyed RNG
    n = 128
    acc = np.zeros((H, W, 3))
    for f in range(n):
        acc += o.render(os_, sc.camera, prm, f)
    acc /= n
    g = o.gbuffer()
    mask = (g[..., 12:15].sum(-1) == 0) & (g[..., 5] > -0.5) & (gt.sum(-1) > 0)
    assert mask.sum() > 0.4 * W * H
    s_gt, s_rs = gt.sum(-1)[mask].sum(), acc.sum(-1)[mask].sum()
    assert abs(s_rs / s_gt - 1.0) <= 0.02, (s_gt, s_rs)
    rel = np.abs(gt - acc).sum(-1)[mask] / np.maximum(gt.sum(-1)[mask], 1e-3)
    assert np.median(rel) < 0.15, float(np.median(rel))


def test_edge_hit_is_tree_independent():
    """A primary ray of C3 at 3840x2160 (pixel (1211, 1458), orbit frame 0) crosses the shared edge z = 0.158333 of
    triangles 65325 and 65388 at the same t.  Moller-Trumbore accepts both, but the point o + t d lies 2.5e-6 above
    65325's box, so before the box inflation (rs_wide.h box_epsilon, restated as or_box_epsilon) the 8-wide walk culled
    that box after finding 65388 while the binary walk found 65325 first: two trees, two hits.  Now both trees return
    the tie rule's answer (smaller t, then smaller index)."""
    sc = scenes.sponza_like()
    cam = scenes.orbit_camera(sc.camera, 0, 240, 0.3)
    out = np.zeros(36, np.float32)
    O.lib().or_camera_kat(O._ptr(cam.as_array()), 3840, 2160, 1211, 1458, O._ptr(out))
    o = np.array([cam.eye], np.float32)
    d = out[33:36][None].copy()
    tnear = np.float32(np.finfo(np.float32).tiny) + np.float32(0.01)
    hits = [O.OracleScene(sc, wide=w).trace_closest(o, d, tnear, 3.0e38) for w in (True, False)]
    assert hits[0][1][0] == hits[1][1][0] == 65325 and hits[0][0][0] == hits[1][0][0]
