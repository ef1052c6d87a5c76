"""ctypes binding of librestir_amd.so (include/restir_c.h) with the reference's frame API.

Mirrors the reference's surface:
  * ``Renderer(width, height)``             ~ SimpleGuiDX11(width, height) + rtcNewDevice
  * ``Renderer.load_scene(scene | path)``    ~ Raytracer::LoadScene (pg/raytracer.cpp:34-38)
  * ``Renderer.produce_restir(camera, params, frame)`` ~ SimpleGuiDX11::produceRestir (pg/simpleguidx11.cpp:359)
  * ``Renderer.frame_data``                  ~ glm::vec3* frame_data (pg/simpleguidx11.h:152), (H, W, 3) f32
There is no CPU fallback: constructing a Renderer without the built library or without a HIP
device raises.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from .params import FrameParams

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(PKG_DIR, "librestir_amd.so")

RS_OK, RS_E_INVALID, RS_E_HIP, RS_E_UNSUPPORTED, RS_E_IO = 0, -1, -2, -3, -4

# Every symbol include/restir_c.h declares (checked by tests/test_capi_symbols.py).
EXPORTED_SYMBOLS = [
    "rs_context_create", "rs_context_destroy", "rs_last_error", "rs_scene_create", "rs_scene_load_obj",
    "rs_scene_destroy", "rs_scene_info", "rs_render_frame", "rs_get_frame_device_ptr", "rs_reset_history",
    "rs_synchronize", "rs_dump_gbuffer", "rs_dump_reservoirs", "rs_tile_begin", "rs_tile_halo_ptr",
    "rs_tile_temporal", "rs_tile_spatial", "rs_tile_finish", "rs_debug_trace", "rs_debug_wide_tree", "rs_scene_walk_info",
    "rs_context_set_traversal",
    "rs_context_get_traversal", "rs_get_timing_totals", "rs_scene_update_positions", "rs_post_frame",
    "rs_post_reset", "rs_scene_rebuild", "rs_render_direct_mis", "rs_scene_create_textured", "rs_scene_set_sky",
    "rs_scene_load_sky", "rs_image_decode", "rs_context_set_initial_split", "rs_context_get_initial_split",
    "rs_context_set_frame_ring", "rs_context_handoff_bytes", "rs_context_set_run_ahead", "rs_max_run_ahead", "rs_tile_stream", "rs_export_png",
    "rs_image_encode_png", "rs_context_track_row_costs", "rs_get_row_costs", "rs_frame_readback", "rs_frame_wait",
    "rs_host_alloc", "rs_host_free", "rs_mgpu_unique_id", "rs_mgpu_create", "rs_mgpu_create_local",
    "rs_mgpu_destroy", "rs_mgpu_set_bands", "rs_mgpu_get_bands", "rs_mgpu_rebalance", "rs_mgpu_render_frame",
    "rs_mgpu_frame_device_ptr", "rs_mgpu_reset_history", "rs_mgpu_allreduce", "rs_mgpu_get_stats",
    "rs_mgpu_set_rebalance_refine", "rs_mgpu_rebalance_times",
    "rs_denoiser_check_weights", "rs_denoiser_create", "rs_denoiser_create_from_file", "rs_denoiser_info_get",
    "rs_denoiser_execute", "rs_denoise_frame", "rs_context_set_denoiser", "rs_denoiser_set_timing",
    "rs_denoiser_last_ms", "rs_denoiser_layer_ms", "rs_denoiser_get_scale", "rs_denoiser_dump", "rs_denoiser_destroy",
]

# BVH traversal kinds (include/restir_c.h RS_TRAVERSAL_*)
TRAVERSAL_AUTO, TRAVERSAL_LOCKSTEP, TRAVERSAL_LANE = -1, 0, 1
TRAVERSAL_NAMES = {"auto": TRAVERSAL_AUTO, "lockstep": TRAVERSAL_LOCKSTEP, "lane": TRAVERSAL_LANE}
# candidate-split initial pass (include/restir_c.h RS_SPLIT_*)
SPLIT_AUTO, SPLIT_OFF, SPLIT_ON = -1, 0, 1
SPLIT_NAMES = {"auto": SPLIT_AUTO, "off": SPLIT_OFF, "on": SPLIT_ON}


class MeshDesc(ctypes.Structure):
    _fields_ = [("n_tris", ctypes.c_uint32), ("positions", ctypes.POINTER(ctypes.c_float)),
                ("normals", ctypes.POINTER(ctypes.c_float)), ("material", ctypes.c_uint32),
                ("texcoords", ctypes.POINTER(ctypes.c_float)), ("tangents", ctypes.POINTER(ctypes.c_float))]


class MaterialDesc(ctypes.Structure):
    _fields_ = [("diffuse", ctypes.c_float * 3), ("specular", ctypes.c_float * 3), ("emission", ctypes.c_float * 3),
                ("shininess", ctypes.c_float), ("type", ctypes.c_int32), ("diffuse_map", ctypes.c_int32),
                ("specular_map", ctypes.c_int32), ("shininess_map", ctypes.c_int32), ("normal_map", ctypes.c_int32)]


TEX_U8, TEX_F32 = 0, 1


class TextureDesc(ctypes.Structure):
    _fields_ = [("width", ctypes.c_uint32), ("height", ctypes.c_uint32), ("channels", ctypes.c_uint32),
                ("format", ctypes.c_int32), ("data", ctypes.c_void_p), ("srgb_expand", ctypes.c_int32)]


def texture_desc(tex):
    """(TextureDesc, keep-alive array) for a scenes.Texture or an (H, W, C) array."""
    arr = tex.data if hasattr(tex, "data") and not isinstance(tex, np.ndarray) else tex
    arr = np.asarray(arr)
    if arr.ndim == 2:
        arr = arr[:, :, None]
    if arr.dtype == np.uint8:
        fmt = TEX_U8
    else:
        arr, fmt = arr.astype(np.float32), TEX_F32
    arr = np.ascontiguousarray(arr)
    d = TextureDesc(arr.shape[1], arr.shape[0], arr.shape[2], fmt, arr.ctypes.data,
                    int(getattr(tex, "srgb_expand", 0)))
    return d, arr


class CameraDesc(ctypes.Structure):
    _fields_ = [("eye", ctypes.c_float * 3), ("at", ctypes.c_float * 3), ("fov_y_deg", ctypes.c_float)]


class PassTimes(ctypes.Structure):
    _fields_ = [("gbuffer_initial_ms", ctypes.c_float), ("visibility_ms", ctypes.c_float),
                ("temporal_ms", ctypes.c_float), ("spatial_ms", ctypes.c_float), ("shade_ms", ctypes.c_float),
                ("total_ms", ctypes.c_float), ("rays", ctypes.c_uint64), ("primary_rays", ctypes.c_uint64),
                ("reproj_outside", ctypes.c_uint64)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class PostParams(ctypes.Structure):
    _fields_ = [("accumulate", ctypes.c_int32), ("tonemap", ctypes.c_int32), ("gamma_correct", ctypes.c_int32),
                ("max_acc_frames", ctypes.c_int32), ("denoise", ctypes.c_int32)]


class PostStats(ctypes.Structure):
    _fields_ = [("mean", ctypes.c_double), ("variance", ctypes.c_double), ("sum", ctypes.c_double),
                ("sqr_sum", ctypes.c_double), ("pixels", ctypes.c_uint64), ("acc_frames_used", ctypes.c_uint32),
                ("reserved", ctypes.c_uint32)]


class ExportParams(ctypes.Structure):
    _fields_ = [("render_time_s", ctypes.c_float), ("write_sidecar", ctypes.c_int32)]


class TileDesc(ctypes.Structure):
    _fields_ = [("y0", ctypes.c_int32), ("y1", ctypes.c_int32), ("margin", ctypes.c_int32), ("halo", ctypes.c_int32)]


class RestirError(RuntimeError):
    pass


_lib = None


def load_library(path: str = LIB_PATH):
    """Load librestir_amd.so.  Raises if it has not been built (no silent fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    path = os.environ.get("RESTIR_LIB", path)     # A/B builds of the same ABI (scripts/ab_variants.sh)
    # One HIP runtime per process: PyTorch-ROCm ships its own libamdhip64.so.7 (same soname as
    # /opt/rocm's, which this library links).  Whichever is loaded first serves both, and torch cannot
    # initialise the device on a runtime other than its own -- so torch (when installed: it carries
    # the multi-GPU plumbing) is imported before this library is dlopen-ed.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(path):
        raise RestirError(f"{path} not found: build it with `make -C restir-embree_amd` (hipcc, gfx950)")
    L = ctypes.CDLL(path)
    vp, i32, u32 = ctypes.c_void_p, ctypes.c_int, ctypes.c_uint32
    fp = ctypes.POINTER(ctypes.c_float)
    L.rs_context_create.argtypes = [i32, i32, i32, vp, ctypes.POINTER(vp)]
    L.rs_context_destroy.argtypes = [vp]
    L.rs_context_destroy.restype = None
    L.rs_last_error.argtypes = [vp]
    L.rs_last_error.restype = ctypes.c_char_p
    L.rs_scene_create.argtypes = [vp, ctypes.POINTER(MeshDesc), u32, ctypes.POINTER(MaterialDesc), u32,
                                  ctypes.POINTER(vp)]
    L.rs_scene_load_obj.argtypes = [vp, ctypes.c_char_p, ctypes.POINTER(vp)]
    L.rs_scene_destroy.argtypes = [vp]
    L.rs_scene_destroy.restype = None
    L.rs_scene_info.argtypes = [vp, ctypes.POINTER(u32), ctypes.POINTER(u32), ctypes.POINTER(u32),
                                ctypes.POINTER(ctypes.c_float)]
    L.rs_render_frame.argtypes = [vp, vp, ctypes.POINTER(CameraDesc), ctypes.POINTER(FrameParams), u32, fp,
                                  ctypes.POINTER(PassTimes)]
    L.rs_get_frame_device_ptr.argtypes = [vp, ctypes.POINTER(vp)]
    L.rs_reset_history.argtypes = [vp]
    L.rs_synchronize.argtypes = [vp]
    L.rs_dump_gbuffer.argtypes = [vp, i32, fp]
    L.rs_dump_reservoirs.argtypes = [vp, fp]
    L.rs_tile_begin.argtypes = [vp, vp, ctypes.POINTER(CameraDesc), ctypes.POINTER(FrameParams), u32,
                                ctypes.POINTER(TileDesc)]
    L.rs_tile_halo_ptr.argtypes = [vp, i32, ctypes.POINTER(vp), ctypes.POINTER(ctypes.c_size_t)]
    L.rs_tile_temporal.argtypes = [vp]
    L.rs_tile_spatial.argtypes = [vp, i32]
    L.rs_tile_finish.argtypes = [vp, ctypes.POINTER(vp), ctypes.POINTER(PassTimes)]
    L.rs_debug_trace.argtypes = [vp, vp, u32, fp, fp, fp, fp, i32, fp, ctypes.POINTER(ctypes.c_int32)]
    L.rs_debug_wide_tree.argtypes = [vp, ctypes.POINTER(u32), ctypes.POINTER(u32), ctypes.POINTER(ctypes.c_int32), vp, vp]
    L.rs_scene_walk_info.argtypes = [vp, ctypes.POINTER(u32), ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32)]
    L.rs_context_set_traversal.argtypes = [vp, i32]
    ip = ctypes.POINTER(ctypes.c_int32)
    L.rs_context_get_traversal.argtypes = [vp, vp, ip, ip, ip]
    L.rs_context_set_initial_split.argtypes = [vp, i32]
    L.rs_context_get_initial_split.argtypes = [vp, ip, ip]
    L.rs_context_set_frame_ring.argtypes = [vp, i32]
    if hasattr(L, "rs_context_handoff_bytes"):   # (absent from round-5 builds, which A/Bs load)
        L.rs_context_handoff_bytes.argtypes = [vp, ctypes.POINTER(ctypes.c_uint64)]
    L.rs_context_set_run_ahead.argtypes = [vp, i32]
    L.rs_max_run_ahead.argtypes = []
    L.rs_max_run_ahead.restype = i32
    L.rs_tile_stream.argtypes = [vp, ctypes.POINTER(vp), ip]
    L.rs_export_png.argtypes = [vp, ctypes.c_char_p, ctypes.POINTER(ExportParams)]
    L.rs_image_encode_png.argtypes = [ctypes.c_char_p, u32, u32, u32, ctypes.POINTER(ctypes.c_uint8)]
    L.rs_context_track_row_costs.argtypes = [vp, i32]
    L.rs_get_row_costs.argtypes = [vp, fp, i32]
    L.rs_get_timing_totals.argtypes = [vp, ctypes.POINTER(PassTimes), ctypes.POINTER(u32), i32]
    L.rs_scene_update_positions.argtypes = [vp, fp, fp]
    L.rs_post_frame.argtypes = [vp, ctypes.POINTER(PostParams), ctypes.POINTER(vp), ctypes.POINTER(PostStats)]
    L.rs_post_reset.argtypes = [vp]
    L.rs_scene_rebuild.argtypes = [vp]
    L.rs_scene_create_textured.argtypes = [vp, ctypes.POINTER(MeshDesc), u32, ctypes.POINTER(MaterialDesc), u32,
                                           ctypes.POINTER(TextureDesc), u32, ctypes.POINTER(vp)]
    L.rs_scene_set_sky.argtypes = [vp, ctypes.POINTER(TextureDesc)]
    L.rs_scene_load_sky.argtypes = [vp, ctypes.c_char_p]
    L.rs_image_decode.argtypes = [ctypes.c_char_p, ctypes.POINTER(u32), ctypes.POINTER(u32), ctypes.POINTER(u32),
                                  ctypes.POINTER(i32), vp, ctypes.c_size_t]
    L.rs_render_direct_mis.argtypes = [vp, vp, ctypes.POINTER(CameraDesc), ctypes.POINTER(FrameParams), u32, u32, fp,
                                       ctypes.POINTER(PassTimes)]
    L.rs_frame_readback.argtypes = [vp, fp, ctypes.POINTER(ctypes.c_uint64)]
    L.rs_frame_wait.argtypes = [vp, ctypes.c_uint64]
    L.rs_host_alloc.argtypes = [vp, ctypes.c_size_t, ctypes.POINTER(vp)]
    L.rs_host_free.argtypes = [vp]
    L.rs_host_free.restype = None
    u8p = ctypes.POINTER(ctypes.c_uint8)
    i32p = ctypes.POINTER(ctypes.c_int32)
    L.rs_mgpu_unique_id.argtypes = [u8p]
    L.rs_mgpu_create.argtypes = [vp, i32, i32, u8p, ctypes.POINTER(vp)]
    L.rs_mgpu_create_local.argtypes = [ctypes.POINTER(vp), i32, ctypes.POINTER(vp)]
    L.rs_mgpu_destroy.argtypes = [vp]
    L.rs_mgpu_destroy.restype = None
    L.rs_mgpu_set_bands.argtypes = [vp, i32p]
    L.rs_mgpu_get_bands.argtypes = [vp, i32p]
    L.rs_mgpu_rebalance.argtypes = [vp, ctypes.POINTER(vp), ctypes.POINTER(CameraDesc), ctypes.POINTER(FrameParams),
                                    u32, i32, i32]
    L.rs_mgpu_render_frame.argtypes = [vp, ctypes.POINTER(vp), ctypes.POINTER(CameraDesc), ctypes.POINTER(FrameParams),
                                       u32, i32, fp, ctypes.POINTER(PassTimes)]
    L.rs_mgpu_frame_device_ptr.argtypes = [vp, ctypes.POINTER(vp)]
    L.rs_mgpu_reset_history.argtypes = [vp]
    L.rs_mgpu_allreduce.argtypes = [vp, ctypes.POINTER(ctypes.c_double), i32, i32]
    L.rs_mgpu_get_stats.argtypes = [vp, vp, i32]
    L.rs_mgpu_set_rebalance_refine.argtypes = [vp, i32]
    L.rs_mgpu_rebalance_times.argtypes = [vp, i32, ctypes.POINTER(ctypes.c_double)]
    L.rs_denoiser_check_weights.argtypes = [vp, ctypes.c_size_t, vp]
    L.rs_denoiser_create.argtypes = [vp, vp, ctypes.c_size_t, ctypes.POINTER(vp)]
    L.rs_denoiser_create_from_file.argtypes = [vp, ctypes.c_char_p, ctypes.POINTER(vp)]
    L.rs_denoiser_info_get.argtypes = [vp, vp]
    L.rs_denoiser_execute.argtypes = [vp, vp, vp, vp, vp, i32, i32, vp]
    L.rs_denoise_frame.argtypes = [vp, vp, vp, ctypes.POINTER(vp)]
    L.rs_context_set_denoiser.argtypes = [vp, vp]
    L.rs_denoiser_set_timing.argtypes = [vp, i32]
    L.rs_denoiser_last_ms.argtypes = [vp, fp]
    L.rs_denoiser_layer_ms.argtypes = [vp, fp]
    L.rs_denoiser_get_scale.argtypes = [vp, fp]
    L.rs_denoiser_dump.argtypes = [vp, i32, vp, ctypes.POINTER(ctypes.c_int32)]
    L.rs_denoiser_destroy.argtypes = [vp]
    L.rs_denoiser_destroy.restype = None
    _lib = L
    return L


def decode_image(path) -> np.ndarray:
    """The scene loader's image decoder (rs_image_decode; no GPU needed): (H, W, C) uint8 or float32."""
    L = load_library()
    w, h, c, f = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_int32()
    p = os.fsencode(path)
    rc = L.rs_image_decode(p, ctypes.byref(w), ctypes.byref(h), ctypes.byref(c), ctypes.byref(f), None, 0)
    if rc != RS_OK:
        raise RestirError(f"rs_image_decode({path}): {L.rs_last_error(None).decode()}")
    out = np.zeros((h.value, w.value, c.value), np.uint8 if f.value == TEX_U8 else np.float32)
    rc = L.rs_image_decode(p, ctypes.byref(w), ctypes.byref(h), ctypes.byref(c), ctypes.byref(f), out.ctypes.data,
                           out.nbytes)
    if rc != RS_OK:
        raise RestirError(f"rs_image_decode({path}): {L.rs_last_error(None).decode()}")
    return out


def encode_png(path, pixels) -> None:
    """Write (H, W[, C]) uint8 pixels (C = 1..4) as a PNG (rs_image_encode_png)."""
    a = np.ascontiguousarray(pixels, np.uint8)
    if a.ndim == 2:
        a = a[:, :, None]
    lib = load_library()
    if lib.rs_image_encode_png(os.fsencode(path), a.shape[1], a.shape[0], a.shape[2],
                               a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))) != RS_OK:
        raise RestirError(lib.rs_last_error(None).decode())


def camera_desc(camera) -> CameraDesc:
    c = CameraDesc()
    arr = camera.as_array() if hasattr(camera, "as_array") else np.asarray(camera, np.float32)
    for i in range(3):
        c.eye[i] = float(arr[i])
        c.at[i] = float(arr[3 + i])
    c.fov_y_deg = float(arr[6])
    return c


class Scene:
    """A scene uploaded to one context (Scene::Scene, pg/Scene.cpp:8-16; BVH built on the GPU)."""

    def __init__(self, renderer: "Renderer", handle):
        self.renderer = renderer
        self.h = handle
        n_tris, n_emis, n_nodes, ms = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_float()
        renderer._check(renderer.lib.rs_scene_info(handle, ctypes.byref(n_tris), ctypes.byref(n_emis),
                                                   ctypes.byref(n_nodes), ctypes.byref(ms)))
        self.n_tris, self.n_emissive, self.n_nodes, self.build_ms = n_tris.value, n_emis.value, n_nodes.value, ms.value

    def update_positions(self, positions, normals=None):
        """Move the geometry (rs_scene_update_positions): (T, 9) float32 positions in the scene's triangle
        order, optional (T, 9) normals; light CDF recomputed and BVH refit on the device, asynchronously
        (stream-ordered with the frames)."""
        pos = np.ascontiguousarray(positions, np.float32).reshape(-1)
        if pos.size != 9 * self.n_tris:
            raise ValueError(f"expected {self.n_tris} x 9 positions, got {pos.size}")
        fp = ctypes.POINTER(ctypes.c_float)
        nrm = None if normals is None else np.ascontiguousarray(normals, np.float32).reshape(-1)
        if nrm is not None and nrm.size != pos.size:
            raise ValueError("normals must match positions")
        r = self.renderer
        r._check(r.lib.rs_scene_update_positions(self.h, pos.ctypes.data_as(fp),
                                                 nrm.ctypes.data_as(fp) if nrm is not None else None))

    def set_sky(self, texture):
        """Equirect sky for params.use_skybox (rs_scene_set_sky); None removes it."""
        r = self.renderer
        if texture is None:
            r._check(r.lib.rs_scene_set_sky(self.h, None))
            return
        d, keep = texture_desc(texture)
        r._check(r.lib.rs_scene_set_sky(self.h, ctypes.byref(d)))
        del keep

    def load_sky(self, path):
        """Sky from a .hdr / .pfm / .ppm / .png file (rs_scene_load_sky)."""
        r = self.renderer
        r._check(r.lib.rs_scene_load_sky(self.h, os.fsencode(path)))

    def rebuild(self):
        """Full light-CDF + BVH rebuild from the current positions (rs_scene_rebuild; synchronous)."""
        r = self.renderer
        r._check(r.lib.rs_scene_rebuild(self.h))
        n_tris, n_emis, n_nodes, ms = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_float()
        r._check(r.lib.rs_scene_info(self.h, ctypes.byref(n_tris), ctypes.byref(n_emis), ctypes.byref(n_nodes),
                                     ctypes.byref(ms)))
        self.n_nodes, self.build_ms = n_nodes.value, ms.value

    WIDE_STATUS = {0: "live", 1: "nonfinite", 2: "too_deep", 3: "too_many", 4: "empty", 5: "off", 6: "error"}

    def walk_info(self) -> dict:
        """rs_scene_walk_info: the 8-wide tree's nodes and depth, or why the scene has none (status name)."""
        r = self.renderer
        nn, dp, st = ctypes.c_uint32(), ctypes.c_int32(), ctypes.c_int32()
        r._check(r.lib.rs_scene_walk_info(self.h, ctypes.byref(nn), ctypes.byref(dp), ctypes.byref(st)))
        return {"wide_nodes": int(nn.value), "wide_depth": int(dp.value), "status": self.WIDE_STATUS.get(st.value, st.value)}

    def wide_tree_nodes(self) -> int:
        """Nodes of the scene's 8-wide tree (0: none -- the per-lane walks take the skip pointers)."""
        r = self.renderer
        nn, nt, dp = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_int32()
        r._check(r.lib.rs_debug_wide_tree(self.h, ctypes.byref(nn), ctypes.byref(nt), ctypes.byref(dp), None, None))
        return int(nn.value)

    def wide_tree(self):
        """Test hook (rs_debug_wide_tree): the scene's 8-wide tree as (words (n_nodes, 20) uint32, leaf-triangle
        ids int32, depth), or None when the scene has none (its walks take the skip pointers)."""
        r = self.renderer
        nn, nt, dp = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_int32()
        r._check(r.lib.rs_debug_wide_tree(self.h, ctypes.byref(nn), ctypes.byref(nt), ctypes.byref(dp), None, None))
        if nn.value == 0:
            return None
        words = np.zeros((nn.value, 20), np.uint32)
        prims = np.zeros(nt.value, np.int32)
        r._check(r.lib.rs_debug_wide_tree(self.h, ctypes.byref(nn), ctypes.byref(nt), ctypes.byref(dp),
                                          words.ctypes.data_as(ctypes.c_void_p), prims.ctypes.data_as(ctypes.c_void_p)))
        return words, prims, dp.value

    def close(self):
        if self.h:
            self.renderer.lib.rs_scene_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Renderer:
    """One HIP device + its per-pixel buffers (G x2, reservoirs x3, framebuffer)."""

    def __init__(self, width: int, height: int, device: int = 0, stream: int | None = None):
        self.lib = load_library()
        self.W, self.H = int(width), int(height)
        self._tile_cache = None
        h = ctypes.c_void_p()
        rc = self.lib.rs_context_create(device, self.W, self.H, ctypes.c_void_p(stream) if stream else None,
                                        ctypes.byref(h))
        if rc != RS_OK:
            raise RestirError(f"rs_context_create failed ({rc}): {self.lib.rs_last_error(None).decode()}")
        self.h = h
        # hipStream_t the context renders on; None (or 0, the legacy null stream) -> a stream of its own
        self.stream = stream if stream else None
        self.frame_data = np.zeros((self.H, self.W, 3), np.float32)
        self.last_times = PassTimes()

    def _check(self, rc):
        if rc != RS_OK:
            msg = self.lib.rs_last_error(self.h).decode()
            raise RestirError(f"librestir_amd error {rc}: {msg}")
        return rc

    def close(self):
        # an attached denoiser stays valid: rs_context_destroy detaches it (its close() then frees only its
        # own memory); dropping the reference breaks the renderer <-> denoiser cycle
        self._denoiser = None
        if getattr(self, "h", None):
            self.lib.rs_context_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- scene-load ---------------------------------------------------------------------
    def load_scene(self, scene) -> Scene:
        if isinstance(scene, (str, os.PathLike)):
            out = ctypes.c_void_p()
            self._check(self.lib.rs_scene_load_obj(self.h, os.fsencode(scene), ctypes.byref(out)))
            return Scene(self, out)
        pos = np.ascontiguousarray(scene.positions, np.float32)
        nrm = np.ascontiguousarray(scene.normals, np.float32)
        tm = np.ascontiguousarray(scene.tri_material, np.uint32)
        # group consecutive triangles with equal material into meshes (keeps triangle order)
        cuts = np.flatnonzero(np.diff(tm)) + 1
        starts = np.concatenate([[0], cuts]).astype(np.int64)
        ends = np.concatenate([cuts, [tm.shape[0]]]).astype(np.int64)
        meshes = (MeshDesc * max(1, len(starts)))()
        fp = ctypes.POINTER(ctypes.c_float)
        uv = getattr(scene, "texcoords", None)
        tg = getattr(scene, "tangents", None)
        uv = None if uv is None else np.ascontiguousarray(uv, np.float32).reshape(-1, 6)
        tg = None if tg is None else np.ascontiguousarray(tg, np.float32).reshape(-1, 9)
        for i, (a, b) in enumerate(zip(starts, ends)):
            meshes[i].n_tris = int(b - a)
            meshes[i].positions = pos[a:b].ctypes.data_as(fp)
            meshes[i].normals = nrm[a:b].ctypes.data_as(fp)
            meshes[i].material = int(tm[a]) if b > a else 0
            if uv is not None:
                meshes[i].texcoords = uv[a:b].ctypes.data_as(fp)
            if tg is not None:
                meshes[i].tangents = tg[a:b].ctypes.data_as(fp)
        mats = (MaterialDesc * max(1, len(scene.materials)))()
        for i, m in enumerate(scene.materials):
            for j in range(3):
                mats[i].diffuse[j] = m.kd[j]
                mats[i].specular[j] = m.ks[j]
                mats[i].emission[j] = m.le[j]
            mats[i].shininess = m.shininess
            mats[i].type = m.type
            for k in ("diffuse_map", "specular_map", "shininess_map", "normal_map"):
                setattr(mats[i], k, int(getattr(m, k, 0)))
        out = ctypes.c_void_p()
        n_mesh = len(starts) if tm.shape[0] else 0
        textures = list(getattr(scene, "textures", []) or [])
        descs = [texture_desc(t) for t in textures]
        tex_arr = (TextureDesc * max(1, len(descs)))(*[d for d, _ in descs])
        self._check(self.lib.rs_scene_create_textured(self.h, meshes, n_mesh, mats, len(scene.materials), tex_arr,
                                                      len(descs), ctypes.byref(out)))
        sc = Scene(self, out)
        if getattr(scene, "sky", None) is not None:
            sc.set_sky(scene.sky)
        return sc

    # ---- render(frame) ------------------------------------------------------------------
    def produce_restir(self, scene: Scene, camera, params: FrameParams, frame_index: int = 0,
                       copy_out: bool = True, timed: bool = True) -> np.ndarray | None:
        cam = camera_desc(camera)
        out = self.frame_data.ctypes.data_as(ctypes.POINTER(ctypes.c_float)) if copy_out else None
        self._check(self.lib.rs_render_frame(self.h, scene.h, ctypes.byref(cam), ctypes.byref(params),
                                             int(frame_index), out, ctypes.byref(self.last_times) if timed else None))
        return self.frame_data if copy_out else None

    render = produce_restir

    def reset_history(self):
        self._check(self.lib.rs_reset_history(self.h))

    def synchronize(self):
        self._check(self.lib.rs_synchronize(self.h))

    def post_frame(self, accumulate: bool = False, tonemap: bool = True, gamma_correct: bool = True,
                   max_acc_frames: int = 0, stats: bool = True, denoise: bool = False):
        """Post-frame block of the reference's producer loop (rs_post_frame): accumulate, ACES + sRGB
        display, accumulator mean/variance; denoise (RenderParams::denoise) displays the denoised
        accumulator (needs set_denoiser).  Returns (display device pointer, PostStats or None)."""
        p = PostParams(int(accumulate), int(tonemap), int(gamma_correct), int(max_acc_frames), int(denoise))
        dptr, st = ctypes.c_void_p(), PostStats()
        self._check(self.lib.rs_post_frame(self.h, ctypes.byref(p), ctypes.byref(dptr),
                                           ctypes.byref(st) if stats else None))
        self._display_ptr = int(dptr.value or 0)
        return self._display_ptr, (st if stats else None)

    def export_png(self, path, render_time_s: float = 0.0, sidecar: bool = True):
        """SimpleGuiDX11::exportImage: the last post_frame's display as RGBA8 PNG (+ <path>.txt)."""
        p = ExportParams(float(render_time_s), 1 if sidecar else 0)
        self._check(self.lib.rs_export_png(self.h, os.fsencode(path), ctypes.byref(p)))

    def set_denoiser(self, denoiser):
        """rs_context_set_denoiser: the denoiser post_frame(denoise=True) runs (None clears it)."""
        self._denoiser = denoiser
        self._check(self.lib.rs_context_set_denoiser(self.h, denoiser.h if denoiser is not None else None))

    def post_reset(self):
        self._check(self.lib.rs_post_reset(self.h))

    def display_rgba(self) -> np.ndarray:
        """Host copy of the (H, W, 4) float32 display buffer written by post_frame (a zero-copy torch
        view of the device buffer, copied to the host)."""
        import torch
        if not getattr(self, "_display_ptr", 0):
            raise RestirError("display_rgba: call post_frame first")

        class _DeviceArray:
            def __init__(self, ptr, n):
                self.__cuda_array_interface__ = {"shape": (n,), "typestr": "<f4", "data": (ptr, False),
                                                 "version": 2, "strides": None}
        self.synchronize()
        t = torch.as_tensor(_DeviceArray(self._display_ptr, self.H * self.W * 4), device="cuda")
        return t.cpu().numpy().reshape(self.H, self.W, 4)

    def timing_totals(self, reset: bool = False):
        """(PassTimes with ms / ray totals, n_frames) over all frames finished since creation or the last
        reset -- no per-frame host sync needed (rs_get_timing_totals)."""
        t, n = PassTimes(), ctypes.c_uint32()
        self._check(self.lib.rs_get_timing_totals(self.h, ctypes.byref(t), ctypes.byref(n), 1 if reset else 0))
        return t, n.value

    def set_traversal(self, mode):
        """BVH traversal kind: "auto" (default), "lockstep" or "lane" (or the TRAVERSAL_* ints)."""
        m = TRAVERSAL_NAMES[mode] if isinstance(mode, str) else int(mode)
        self._check(self.lib.rs_context_set_traversal(self.h, m))

    def set_initial_split(self, mode):
        """Candidate-split initial pass: "auto" (default), "off" or "on" (or the SPLIT_* ints)."""
        m = SPLIT_NAMES[mode] if isinstance(mode, str) else int(mode)
        self._check(self.lib.rs_context_set_initial_split(self.h, m))

    def set_run_ahead(self, depth: int):
        """Frame pipelining depth 0..2: a frame's initial pass overlaps up to `depth` earlier frames."""
        self._check(self.lib.rs_context_set_run_ahead(self.h, int(depth)))

    def set_frame_ring(self, n: int):
        """1 (default) or 2 framebuffers alternating per frame (a reader may lag one frame)."""
        self._check(self.lib.rs_context_set_frame_ring(self.h, int(n)))

    def handoff_bytes(self) -> int:
        """rs_context_handoff_bytes: device bytes of the sorted initial pass's hand-off buffers (all lanes)."""
        v = ctypes.c_uint64()
        self._check(self.lib.rs_context_handoff_bytes(self.h, ctypes.byref(v)))
        return int(v.value)

    def track_row_costs(self, enable: bool = True):
        """Record per-row wave time in every pass (load balancing of tile-sharded frames)."""
        self._check(self.lib.rs_context_track_row_costs(self.h, 1 if enable else 0))

    def row_costs(self, reset: bool = True) -> np.ndarray:
        """(H,) float32 per-row wave time accumulated since the last reset (synchronises)."""
        out = np.zeros(self.H, np.float32)
        self._check(self.lib.rs_get_row_costs(self.h, out.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
                                              1 if reset else 0))
        return out

    def initial_split(self):
        """(requested mode, whether the last frame's initial pass ran split)."""
        m, last = ctypes.c_int32(), ctypes.c_int32()
        self._check(self.lib.rs_context_get_initial_split(self.h, ctypes.byref(m), ctypes.byref(last)))
        return m.value, bool(last.value)

    def traversal(self, scene: "Scene | None" = None):
        """(requested mode, kind the last frame ran with, kind AUTO settled on for `scene` or -1)."""
        m, k, s = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        self._check(self.lib.rs_context_get_traversal(self.h, scene.h if scene is not None else None,
                                                      ctypes.byref(m), ctypes.byref(k), ctypes.byref(s)))
        return m.value, k.value, s.value

    def frame_device_ptr(self) -> int:
        p = ctypes.c_void_p()
        self._check(self.lib.rs_get_frame_device_ptr(self.h, ctypes.byref(p)))
        return int(p.value or 0)

    # ---- dumps ----------------------------------------------------------------------------
    def gbuffer(self, prev: bool = False) -> np.ndarray:
        out = np.zeros((self.H, self.W, 19), np.float32)
        self._check(self.lib.rs_dump_gbuffer(self.h, 1 if prev else 0, out.ctypes.data_as(ctypes.POINTER(ctypes.c_float))))
        return out

    def reservoirs(self) -> np.ndarray:
        out = np.zeros((self.H, self.W, 12), np.float32)
        self._check(self.lib.rs_dump_reservoirs(self.h, out.ctypes.data_as(ctypes.POINTER(ctypes.c_float))))
        return out

    def render_direct_mis(self, scene: Scene, camera, params: FrameParams, frame_index: int = 0, spp: int = 1,
                          copy_out: bool = True, timed: bool = False) -> np.ndarray | None:
        """MIS direct-light ground truth (rs_render_direct_mis; DirectMISIntegrator, calcGI off): spp
        samples per pixel into the framebuffer.  Accumulate frames with post_frame(accumulate=True) for a
        converged reference.  timed=True fills last_times (shade_ms = the launch, rays)."""
        cam = camera_desc(camera)
        out = self.frame_data.ctypes.data_as(ctypes.POINTER(ctypes.c_float)) if copy_out else None
        self._check(self.lib.rs_render_direct_mis(self.h, scene.h, ctypes.byref(cam), ctypes.byref(params),
                                                  int(frame_index), int(spp), out,
                                                  ctypes.byref(self.last_times) if timed else None))
        return self.frame_data if copy_out else None

    def debug_trace(self, scene: Scene, o, d, tnear, tfar, any_hit: bool, lockstep: bool = True,
                    stats: bool = False, wide_stats: bool = False):
        """Raw BVH queries.  stats=True: per-lane skip-pointer walk statistics instead -- returns
        (visits, triangle_tests) int arrays per ray; wide_stats=True: the 8-wide walk's (node fetches,
        triangle tests, stack overflow flags)."""
        if wide_stats:
            t, prim = self._debug_trace(scene, o, d, tnear, tfar, 7 if any_hit else 6)
            p = prim.view(np.uint32)
            return (p >> 16).astype(np.int64), (p & 0xFFFF).astype(np.int64), t
        if stats:
            t, prim = self._debug_trace(scene, o, d, tnear, tfar, 5 if any_hit else 4)
            p = prim.view(np.uint32)
            return (p >> 16).astype(np.int64), (p & 0xFFFF).astype(np.int64)
        return self._debug_trace(scene, o, d, tnear, tfar, (1 if any_hit else 0) + (0 if lockstep else 2))

    def _debug_trace(self, scene: Scene, o, d, tnear, tfar, mode: int):
        o = np.ascontiguousarray(o, np.float32)
        d = np.ascontiguousarray(d, np.float32)
        n = o.shape[0]
        tn = np.ascontiguousarray(np.broadcast_to(np.asarray(tnear, np.float32), (n,)))
        tf = np.ascontiguousarray(np.broadcast_to(np.asarray(tfar, np.float32), (n,)))
        t = np.zeros(n, np.float32)
        prim = np.zeros(n, np.int32)
        fp = ctypes.POINTER(ctypes.c_float)
        self._check(self.lib.rs_debug_trace(self.h, scene.h, n, o.ctypes.data_as(fp), d.ctypes.data_as(fp),
                                            tn.ctypes.data_as(fp), tf.ctypes.data_as(fp), int(mode),
                                            t.ctypes.data_as(fp), prim.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))))
        return t, prim

    # ---- tile stages (multi-GPU) ------------------------------------------------------------
    def tile_begin(self, scene: Scene, camera, params: FrameParams, frame_index: int, y0: int, y1: int,
                   margin: int, halo: int):
        # per-frame host work is on the multi-GPU critical path: reuse the descriptors of a repeated
        # camera object / band instead of rebuilding them
        if self._tile_cache is None or self._tile_cache[0] is not camera or self._tile_cache[1] != (y0, y1, margin, halo):
            self._tile_cache = (camera, (y0, y1, margin, halo), camera_desc(camera), TileDesc(y0, y1, margin, halo))
        _, _, cam, t = self._tile_cache
        self._check(self.lib.rs_tile_begin(self.h, scene.h, ctypes.byref(cam), ctypes.byref(params),
                                           int(frame_index), ctypes.byref(t)))

    def tile_halo_ptr(self, which: int):
        p, n = ctypes.c_void_p(), ctypes.c_size_t()
        self._check(self.lib.rs_tile_halo_ptr(self.h, which, ctypes.byref(p), ctypes.byref(n)))
        return int(p.value or 0), int(n.value)

    def tile_stream(self):
        """(stream handle, lane index) of the frame in flight."""
        p, lane = ctypes.c_void_p(), ctypes.c_int32()
        self._check(self.lib.rs_tile_stream(self.h, ctypes.byref(p), ctypes.byref(lane)))
        return int(p.value or 0), lane.value

    def tile_temporal(self):
        self._check(self.lib.rs_tile_temporal(self.h))

    def tile_spatial(self, pass_index: int):
        self._check(self.lib.rs_tile_spatial(self.h, pass_index))

    def tile_finish(self, timed: bool = False):
        p = ctypes.c_void_p()
        self._check(self.lib.rs_tile_finish(self.h, ctypes.byref(p), ctypes.byref(self.last_times) if timed else None))
        return int(p.value or 0)
