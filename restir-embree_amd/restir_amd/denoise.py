"""Denoiser binding (rs_denoiser_*, csrc/rs_denoise.hip): the reference's Open Image Denoise "RT"
filter (pg/simpleguidx11.cpp:52-75 setup, :255-260 execute) as OIDN's UNet on the MI355X matrix cores.

    den = Denoiser(renderer, weights)            # oidnNewFilter("RT") + set("hdr", true) + commit
    out = den.execute(color, albedo, normal)     # oidnFilter.execute on (H, W, 3) float32 device tensors
    renderer.set_denoiser(den); renderer.post_frame(denoise=True)   # RenderParams::denoise display

`weights`: bytes of an OIDN tensor archive (.tza), a path to one, or a {name: array} dict (written to a
.tza in memory; restir_amd.tza).  OIDN's trained rt_hdr_alb_nrm.tza is not shipped with the reference.
"""
from __future__ import annotations

import ctypes
import math
import os

from .renderer import RS_OK, RestirError, load_library
from . import tza as _tza


class DenoiserInfo(ctypes.Structure):
    _fields_ = [("input_channels", ctypes.c_int32), ("channels", ctypes.c_int32 * 16),
                ("parameters", ctypes.c_uint64), ("mac_per_pixel", ctypes.c_double)]


class DenoiseParams(ctypes.Structure):
    _fields_ = [("input_scale", ctypes.c_float), ("hdr", ctypes.c_int32)]


def _blob(weights) -> bytes:
    if isinstance(weights, dict):
        return _tza.write_tza(weights)
    if isinstance(weights, (str, os.PathLike)):
        with open(weights, "rb") as f:
            return f.read()
    return bytes(weights)


def check_weights(weights) -> DenoiserInfo:
    """Parse + check an archive against the UNet topology on the host (no device work)."""
    L = load_library()
    b = _blob(weights)
    info = DenoiserInfo()
    buf = ctypes.create_string_buffer(b, len(b))
    if L.rs_denoiser_check_weights(buf, len(b), ctypes.byref(info)) != RS_OK:
        raise RestirError(L.rs_last_error(None).decode())
    return info


class Denoiser:
    def __init__(self, renderer, weights):
        self.r = renderer
        self.lib = renderer.lib
        b = _blob(weights)
        buf = ctypes.create_string_buffer(b, len(b))
        h = ctypes.c_void_p()
        self.r._check(self.lib.rs_denoiser_create(renderer.h, buf, len(b), ctypes.byref(h)))
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            self.lib.rs_denoiser_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def info(self) -> DenoiserInfo:
        i = DenoiserInfo()
        self.r._check(self.lib.rs_denoiser_info_get(self.h, ctypes.byref(i)))
        return i

    @staticmethod
    def _params(input_scale):
        s = float("nan") if input_scale is None else float(input_scale)
        return DenoiseParams(s, 1)

    def execute(self, color, albedo=None, normal=None, output=None, input_scale=None):
        """(H, W, 3) float32 torch device tensors -> denoised (H, W, 3) torch tensor (async on the
        renderer's stream; synchronise before reading)."""
        import torch
        H, W = int(color.shape[0]), int(color.shape[1])
        for t in (color, albedo, normal):
            if t is not None and (t.dtype != torch.float32 or not t.is_contiguous() or tuple(t.shape) != (H, W, 3)):
                raise RestirError("execute: images must be contiguous (H, W, 3) float32 device tensors")
        if output is None:
            output = torch.empty_like(color)
        p = self._params(input_scale)
        ptr = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None   # noqa: E731
        self.r._check(self.lib.rs_denoiser_execute(self.h, ptr(color), ptr(albedo), ptr(normal), ptr(output), W, H,
                                                   ctypes.byref(p)))
        return output

    def denoise_frame(self, input_scale=None) -> int:
        """The reference's per-frame call on the renderer's accumulator + G-buffer; device pointer of the
        (H, W, 3) output."""
        p = self._params(input_scale)
        out = ctypes.c_void_p()
        self.r._check(self.lib.rs_denoise_frame(self.r.h, self.h, ctypes.byref(p), ctypes.byref(out)))
        return int(out.value or 0)

    def frame_output(self, input_scale=None):
        """denoise_frame + host copy: (H, W, 3) float32 numpy array."""
        import torch
        ptr = self.denoise_frame(input_scale)
        n = self.r.H * self.r.W * 3

        class _DeviceArray:
            __cuda_array_interface__ = {"shape": (n,), "typestr": "<f4", "data": (ptr, False), "version": 2,
                                        "strides": None}
        self.r.synchronize()
        return torch.as_tensor(_DeviceArray(), device="cuda").cpu().numpy().reshape(self.r.H, self.r.W, 3)

    def dump(self, tensor: int):
        """Test hook (rs_denoiser_dump): float16 activation tensor `tensor` of the last execute with its zero
        border, (rows + 2, cols + 2, channel stride) numpy array, and its real channel count."""
        import numpy as np
        dims = (ctypes.c_int32 * 4)()
        self.r._check(self.lib.rs_denoiser_dump(self.h, int(tensor), None, dims))
        out = np.zeros((dims[0], dims[1], dims[2]), np.float16)
        self.r._check(self.lib.rs_denoiser_dump(self.h, int(tensor), out.ctypes.data_as(ctypes.c_void_p), dims))
        return out, int(dims[3])

    def set_timing(self, enable: bool = True):
        self.r._check(self.lib.rs_denoiser_set_timing(self.h, 1 if enable else 0))

    def last_ms(self) -> float:
        v = ctypes.c_float()
        self.r._check(self.lib.rs_denoiser_last_ms(self.h, ctypes.byref(v)))
        return v.value

    def layer_ms(self):
        """[input transform, 16 convolutions] ms of the last timed execute (HIP events on its stream)."""
        v = (ctypes.c_float * 17)()
        self.r._check(self.lib.rs_denoiser_layer_ms(self.h, v))
        return list(v)

    def scale(self) -> float:
        v = ctypes.c_float()
        self.r._check(self.lib.rs_denoiser_get_scale(self.h, ctypes.byref(v)))
        return v.value


def gflop_per_frame(info: DenoiserInfo, width: int, height: int) -> float:
    """Algorithmic GFLOP of one execute at the padded resolution (2 FLOP per MAC)."""
    hp, wp = math.ceil(height / 16) * 16, math.ceil(width / 16) * 16
    return 2.0 * info.mac_per_pixel * hp * wp / 1e9
