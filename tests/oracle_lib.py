"""ctypes wrapper for the CPU oracle (oracle/restir_oracle.c).

TEST INFRASTRUCTURE ONLY: used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg as the checker / CPU baseline.  The product never imports this module.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "restir-embree_amd"))

from restir_amd.params import FrameParams  # noqa: E402

LIB_PATH = os.path.join(ROOT, "oracle", "_build", "librestir_oracle.so")
_lib = None

_f32p = ctypes.POINTER(ctypes.c_float)
_i32p = ctypes.POINTER(ctypes.c_int32)
_u32p = ctypes.POINTER(ctypes.c_uint32)


def _ptr(a, t=_f32p):
    return a.ctypes.data_as(t)


def build():
    srcs = [os.path.join(ROOT, "oracle", "restir_oracle.c"), os.path.join(ROOT, "restir-embree_amd", "csrc", "rs_libm.h")]
    if (not os.path.exists(LIB_PATH)) or os.path.getmtime(LIB_PATH) < max(os.path.getmtime(p) for p in srcs):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(LIB_PATH)
        L.or_scene_create.restype = ctypes.c_void_p
        L.or_scene_create.argtypes = [ctypes.c_uint32, _f32p, _f32p, _u32p, ctypes.c_uint32, _f32p, _i32p]
        L.or_scene_destroy.argtypes = [ctypes.c_void_p]
        L.or_scene_set_wide.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.or_ctx_create.restype = ctypes.c_void_p
        L.or_ctx_create.argtypes = [ctypes.c_int, ctypes.c_int]
        L.or_ctx_destroy.argtypes = [ctypes.c_void_p]
        L.or_ctx_set_cache_im.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.or_ctx_reset_history.argtypes = [ctypes.c_void_p]
        L.or_render_frame.restype = ctypes.c_int
        L.or_render_frame.argtypes = [ctypes.c_void_p, ctypes.c_void_p, _f32p, ctypes.POINTER(FrameParams),
                                      ctypes.c_uint32, _f32p, ctypes.POINTER(ctypes.c_uint64)]
        L.or_get_gbuffer.argtypes = [ctypes.c_void_p, ctypes.c_int, _f32p]
        L.or_scene_set_textures.restype = ctypes.c_int
        L.or_scene_set_textures.argtypes = [ctypes.c_void_p, _i32p, _f32p, _f32p, ctypes.c_uint32, ctypes.c_void_p]
        L.or_scene_set_sky.restype = ctypes.c_int
        L.or_scene_set_sky.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.or_render_direct_mis.restype = ctypes.c_int
        L.or_render_direct_mis.argtypes = [ctypes.c_void_p, ctypes.c_void_p, _f32p, ctypes.POINTER(FrameParams),
                                           ctypes.c_uint32, ctypes.c_int, _f32p, ctypes.POINTER(ctypes.c_uint64)]
        L.or_get_reservoirs.argtypes = [ctypes.c_void_p, _f32p]
        L.or_calc_I_M.restype = ctypes.c_float
        L.or_calc_I_M.argtypes = [ctypes.c_float, ctypes.c_float]
        L.or_ibeta.restype = ctypes.c_double
        L.or_ibeta.argtypes = [ctypes.c_double, ctypes.c_double, ctypes.c_double]
        L.or_camera_kat.argtypes = [_f32p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, _f32p]
        L.or_reproject_kat.argtypes = [_f32p, ctypes.c_int, ctypes.c_int, _f32p, _i32p]
        L.or_rng_u.restype = ctypes.c_float
        L.or_rng_u.argtypes = [ctypes.c_uint32] * 5
        L.or_scene_n_emissive.restype = ctypes.c_uint32
        L.or_scene_n_emissive.argtypes = [ctypes.c_void_p]
        L.or_scene_total_area.restype = ctypes.c_float
        L.or_scene_total_area.argtypes = [ctypes.c_void_p]
        L.or_scene_cdf.argtypes = [ctypes.c_void_p, _f32p, _f32p, _f32p]
        L.or_trace_closest.argtypes = [ctypes.c_void_p, ctypes.c_int, _f32p, _f32p, ctypes.c_float, ctypes.c_float,
                                       _f32p, _i32p]
        L.or_trace_any.argtypes = [ctypes.c_void_p, ctypes.c_int, _f32p, _f32p, _f32p, _f32p, _i32p]
        L.or_num_threads.restype = ctypes.c_int
        _f64p = ctypes.POINTER(ctypes.c_double)
        L.or_post_apply.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, _f32p, _f32p, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_int, _f32p, _f64p, _f64p]
        L.or_kat_reservoir.argtypes = [_f32p, _i32p, ctypes.c_int, _f32p, ctypes.c_int, ctypes.c_int, _f32p, _i32p,
                                       _i32p]
        L.or_kat_light_sample_valid.restype = ctypes.c_int
        L.or_kat_light_sample_valid.argtypes = [_f32p, _f32p, _f32p]
        L.or_kat_cosine.argtypes = [_f32p, ctypes.c_float, ctypes.c_float, _f32p, _f32p]
        L.or_kat_lobe.argtypes = [_f32p, ctypes.c_float, ctypes.c_float, ctypes.c_float, _f32p, _f32p]
        L.or_kat_power_heuristic.restype = ctypes.c_float
        L.or_kat_power_heuristic.argtypes = [ctypes.c_float, ctypes.c_float]
        L.or_kat_max_component.restype = ctypes.c_float
        L.or_kat_max_component.argtypes = [_f32p]
        L.or_ctx_ref_rays.restype = ctypes.c_uint64
        L.or_ctx_ref_rays.argtypes = [ctypes.c_void_p]
        L.or_ctx_rebuilt.restype = ctypes.c_uint64
        L.or_ctx_rebuilt.argtypes = [ctypes.c_void_p]
        L.or_kat_mis.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_float, ctypes.c_float, _f32p]
        L.or_libm_f1.argtypes = [ctypes.c_int, _f32p, _f32p, ctypes.c_int]
        L.or_libm_powf.argtypes = [_f32p, _f32p, _f32p, ctypes.c_int]
        L.or_libm_d1.argtypes = [ctypes.c_int, _f64p, _f64p, ctypes.c_int]
        _lib = L
    return _lib


def libm_f1(name, x):
    """rs_libm.h (shared by the oracle and the kernels): expf / lgammaf / sinf / cosf over a float32 array"""
    x = np.ascontiguousarray(x, np.float32)
    o = np.empty_like(x)
    lib().or_libm_f1(["expf", "lgammaf", "sinf", "cosf"].index(name), _ptr(x), _ptr(o), x.size)
    return o


def libm_f2(name, x, y):
    assert name == "powf"
    x, y = np.ascontiguousarray(x, np.float32), np.ascontiguousarray(y, np.float32)
    o = np.empty_like(x)
    lib().or_libm_powf(_ptr(x), _ptr(y), _ptr(o), x.size)
    return o


def libm_d1(name, x):
    """rs_libm.h's double log / exp / log1p / lgamma (the incomplete beta's)"""
    x = np.ascontiguousarray(x, np.float64)
    o = np.empty_like(x)
    p = ctypes.POINTER(ctypes.c_double)
    lib().or_libm_d1(["log", "exp", "log1p", "lgamma"].index(name), _ptr(x, p), _ptr(o, p), x.size)
    return o


class OraclePost:
    """Post-frame restatement (oracle or_post_apply) with the reference's accFrameCtr bookkeeping
    (pg/simpleguidx11.cpp:246-333): accumulate / tonemap / gamma, mean & variance of the accumulator."""

    def __init__(self, W: int, H: int):
        self.W, self.H = W, H
        self.acc = np.zeros((H, W, 3), np.float32)
        self.acc_frames = 0

    def apply(self, frame, accumulate=False, tonemap=True, gamma_correct=True, max_acc_frames=0):
        L = lib()
        frame = np.ascontiguousarray(frame, np.float32)
        disp = np.zeros((self.H, self.W, 4), np.float32)
        s, q = ctypes.c_double(), ctypes.c_double()
        used = self.acc_frames
        L.or_post_apply(self.W, 0, self.H, frame.ctypes.data_as(_f32p), self.acc.ctypes.data_as(_f32p), used,
                        int(tonemap), int(gamma_correct), disp.ctypes.data_as(_f32p), ctypes.byref(s),
                        ctypes.byref(q))
        self.acc_frames += 1
        max_acc = max_acc_frames if max_acc_frames > 0 else 300000
        if not (accumulate and self.acc_frames <= max_acc):
            self.acc_frames = 0
        n = self.W * self.H
        mean = s.value / n
        return disp, {"mean": mean, "variance": q.value / n - mean * mean, "sum": s.value, "sqr_sum": q.value,
                      "acc_frames_used": used}


class _TexDesc(ctypes.Structure):
    _fields_ = [("width", ctypes.c_uint32), ("height", ctypes.c_uint32), ("channels", ctypes.c_uint32),
                ("format", ctypes.c_int32), ("data", ctypes.c_void_p), ("srgb_expand", ctypes.c_int32)]


def _texdescs(textures):
    """or_texdesc array (+ the arrays it points into) for scenes.Texture objects."""
    keep, arr = [], (_TexDesc * max(1, len(textures)))()
    for i, t in enumerate(textures):
        a = np.asarray(t.data)
        if a.ndim == 2:
            a = a[:, :, None]
        fmt = 0 if a.dtype == np.uint8 else 1
        a = np.ascontiguousarray(a if fmt == 0 else a.astype(np.float32))
        keep.append(a)
        arr[i] = _TexDesc(a.shape[1], a.shape[0], a.shape[2], fmt, a.ctypes.data, int(t.srgb_expand))
    return arr, keep


class OracleScene:
    """wide: walk the 8-wide AVX2 tree (or_scene_set_wide; same hits as the binary tree, faster) --
    default on unless ORACLE_WIDE=0; False keeps the binary stack walk."""
    def __init__(self, scene, wide=None):
        L = lib()
        self.scene = scene
        self._pos = np.ascontiguousarray(scene.positions, dtype=np.float32)
        self._nrm = np.ascontiguousarray(scene.normals, dtype=np.float32)
        self._mat = np.ascontiguousarray(scene.tri_material, dtype=np.uint32)
        mf, mt = scene.material_arrays()
        self._mf, self._mt = np.ascontiguousarray(mf), np.ascontiguousarray(mt)
        self.h = L.or_scene_create(scene.n_tris, _ptr(self._pos), _ptr(self._nrm), _ptr(self._mat, _u32p),
                                   len(scene.materials), _ptr(self._mf), _ptr(self._mt, _i32p))
        textures = list(getattr(scene, "textures", []) or [])
        maps = np.array([[getattr(m, k, 0) for k in ("diffuse_map", "specular_map", "shininess_map", "normal_map")]
                         for m in scene.materials] or [[0, 0, 0, 0]], np.int32)
        if textures or maps.any():
            descs, keep = _texdescs(textures)
            uv = getattr(scene, "texcoords", None)
            tg = getattr(scene, "tangents", None)
            self._uv = None if uv is None else np.ascontiguousarray(uv, np.float32)
            self._tg = None if tg is None else np.ascontiguousarray(tg, np.float32)
            rc = L.or_scene_set_textures(self.h, _ptr(maps, _i32p), _ptr(self._uv) if self._uv is not None else None,
                                         _ptr(self._tg) if self._tg is not None else None, len(textures),
                                         ctypes.cast(descs, ctypes.c_void_p))
            if rc != 0:
                raise RuntimeError("or_scene_set_textures failed")
        if getattr(scene, "sky", None) is not None:
            descs, keep = _texdescs([scene.sky])
            if L.or_scene_set_sky(self.h, ctypes.cast(descs, ctypes.c_void_p)) != 0:
                raise RuntimeError("or_scene_set_sky failed")
        if wide is None:
            wide = os.environ.get("ORACLE_WIDE", "1") != "0"
        self.wide = bool(L.or_scene_set_wide(self.h, 1 if wide else 0))

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.or_scene_destroy(self.h)
            self.h = None

    @property
    def n_emissive(self):
        return int(lib().or_scene_n_emissive(self.h))

    def cdf(self):
        n = self.n_emissive
        c, p, a = (np.zeros(n, np.float32) for _ in range(3))
        lib().or_scene_cdf(self.h, _ptr(c), _ptr(p), _ptr(a))
        return c, p, a

    def trace_closest(self, o, d, tnear=0.0, tfar=3.0e38):
        o = np.ascontiguousarray(o, np.float32)
        d = np.ascontiguousarray(d, np.float32)
        n = o.shape[0]
        t = np.zeros(n, np.float32)
        prim = np.zeros(n, np.int32)
        lib().or_trace_closest(self.h, n, _ptr(o), _ptr(d), tnear, tfar, _ptr(t), _ptr(prim, _i32p))
        return t, prim

    def trace_any(self, o, d, tnear, tfar):
        o = np.ascontiguousarray(o, np.float32)
        d = np.ascontiguousarray(d, np.float32)
        tn = np.ascontiguousarray(tnear, np.float32)
        tf = np.ascontiguousarray(tfar, np.float32)
        n = o.shape[0]
        hit = np.zeros(n, np.int32)
        lib().or_trace_any(self.h, n, _ptr(o), _ptr(d), _ptr(tn), _ptr(tf), _ptr(hit, _i32p))
        return hit


class OracleRenderer:
    """Mirror of the product's frame API over the oracle: render(frame) -> framebuffer."""

    def __init__(self, width, height, cache_im=True):
        self.W, self.H = width, height
        self.h = lib().or_ctx_create(width, height)
        lib().or_ctx_set_cache_im(self.h, 1 if cache_im else 0)
        self.rays = 0

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.or_ctx_destroy(self.h)
            self.h = None

    def reset_history(self):
        lib().or_ctx_reset_history(self.h)

    def render(self, oscene: OracleScene, camera, params, frame_index=0):
        out = np.zeros((self.H, self.W, 3), np.float32)
        cam = np.ascontiguousarray(camera.as_array() if hasattr(camera, "as_array") else camera, np.float32)
        rays = ctypes.c_uint64(0)
        rc = lib().or_render_frame(self.h, oscene.h, _ptr(cam), ctypes.byref(params), frame_index, _ptr(out),
                                   ctypes.byref(rays))
        if rc != 0:
            raise RuntimeError(f"or_render_frame failed: {rc}")
        self.rays = int(rays.value)
        self.reference_rays = int(lib().or_ctx_ref_rays(self.h))
        return out

    def render_direct_mis(self, oscene, camera, params, frame_index=0, spp=1):
        """MIS direct-light ground truth (or_render_direct_mis): one frame of spp samples per pixel."""
        cam = camera.as_array() if hasattr(camera, "as_array") else np.asarray(camera, np.float32)
        out = np.zeros((self.H, self.W, 3), np.float32)
        rays = ctypes.c_uint64()
        rc = lib().or_render_direct_mis(self.h, oscene.h, _ptr(cam), ctypes.byref(params), frame_index, spp,
                                        _ptr(out), ctypes.byref(rays))
        if rc != 0:
            raise RuntimeError(f"or_render_direct_mis failed: {rc}")
        self.rays = int(rays.value)
        return out

    def gbuffer(self, prev=False):
        out = np.zeros((self.H, self.W, 19), np.float32)
        lib().or_get_gbuffer(self.h, 1 if prev else 0, _ptr(out))
        return out

    def reservoirs(self):
        out = np.zeros((self.H, self.W, 12), np.float32)
        lib().or_get_reservoirs(self.h, _ptr(out))
        return out


class OracleTileBackend:
    """Tile stages of the oracle (or_tile_*), same interface as restir_amd.distributed.GpuTileBackend,
    so the distributed orchestration can be checked on CPU with gloo."""

    def __init__(self, width, height):
        L = lib()
        vp = ctypes.c_void_p
        L.or_tile_begin.argtypes = [vp, vp, _f32p, ctypes.POINTER(FrameParams), ctypes.c_uint32, ctypes.c_int,
                                    ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.or_tile_halo_ptr.argtypes = [vp, ctypes.c_int, ctypes.POINTER(vp), ctypes.POINTER(ctypes.c_size_t)]
        L.or_tile_temporal.argtypes = [vp]
        L.or_tile_spatial.argtypes = [vp, ctypes.c_int]
        L.or_tile_finish.argtypes = [vp, _f32p, ctypes.POINTER(ctypes.c_uint64)]
        self.r = OracleRenderer(width, height)
        self.W, self.H = width, height
        self.last_times = None

    def load_scene(self, scene):
        return OracleScene(scene)

    # load-balancing hooks: the oracle records no wave times; a synthetic per-row cost (rising toward
    # the bottom rows, only for this rank's band) drives TiledRenderer.rebalance to unequal bands
    def track_row_costs(self, enable=True):
        self._track = enable

    def reset_history(self):
        self.r.reset_history()

    def row_costs(self, reset=True):
        c = np.zeros(self.H, np.float32)
        y0, y1 = getattr(self, "y0", 0), getattr(self, "y1", 0)
        c[y0:y1] = (np.arange(y0, y1, dtype=np.float32) + 1.0) ** 2
        return c

    def begin(self, scene, camera, params, frame, y0, y1, margin, halo):
        self.y0, self.y1 = y0, y1
        self._params = params
        cam = np.ascontiguousarray(camera.as_array() if hasattr(camera, "as_array") else camera, np.float32)
        rc = lib().or_tile_begin(self.r.h, scene.h, _ptr(cam), ctypes.byref(params), frame, y0, y1, margin, halo)
        if rc:
            raise RuntimeError(f"or_tile_begin failed {rc}")

    def halo_tensor(self, which):
        import torch
        p, n = ctypes.c_void_p(), ctypes.c_size_t()
        lib().or_tile_halo_ptr(self.r.h, which, ctypes.byref(p), ctypes.byref(n))
        if not p.value:
            return None
        arr = np.ctypeslib.as_array((ctypes.c_uint8 * n.value).from_address(p.value))
        return torch.from_numpy(arr)

    def temporal(self):
        lib().or_tile_temporal(self.r.h)

    def spatial(self, p):
        lib().or_tile_spatial(self.r.h, p)

    def finish(self, timed=False):
        import torch
        out = np.zeros((self.y1 - self.y0) * self.W * 3, np.float32)
        rays = ctypes.c_uint64(0)
        lib().or_tile_finish(self.r.h, _ptr(out), ctypes.byref(rays))
        self.rays = int(rays.value)
        self.reference_rays = int(lib().or_ctx_ref_rays(self.r.h))
        return torch.from_numpy(out)
