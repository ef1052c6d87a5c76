"""CPU fp32 reference of the denoiser -- TEST INFRASTRUCTURE ONLY.

Used by tests/ and bench.py's cpu_baseline leg as the checker / CPU baseline; the product
(restir-embree_amd/, librestir_amd.so) never imports it.

What the reference runs: every produced frame, SimpleGuiDX11::Producer executes an Open Image Denoise
"RT" filter on the accumulator with the current G-buffer's diffuse colour as albedo and its world-space
normal as normal, hdr = true, quality = High (pg/simpleguidx11.cpp:52-75 setup, :255-256 execute), and
shows the result instead of the accumulator when RenderParams::denoise is on
(pg/RenderParams.h:13, pg/simpleguidx11.cpp:273-280).

OIDN is NOT in /root/reference: only its two API headers and prebuilt Windows libraries
(template/src/libs/oidn-2.3.3.x64.windows), and its trained weights (the `oidn-weights` repository's
rt_hdr_alb_nrm.tza) are not shipped.  This module restates OIDN 2.3's published algorithm for that
filter -- parity UNPINNED against OIDN itself (no fixture or output of it exists here):
  * input: colour * inputScale (auto-exposure when unset), clamped to [0, 65504], through the PU
    transfer function normalised to 65504; albedo clamped to [0, 1]; normal clamped to [-1, 1] and
    mapped to [0, 1]; channels (colour, albedo, normal); image zero-padded to a multiple of 16;
  * the UNet: 3x3 convolutions (zero padding) + ReLU, 2x2 max pooling after enc_conv1..4, nearest 2x
    upsampling before dec_conv4a/3a/2a/1a, concatenation [upsampled, skip], dec_conv0 linear;
  * output: max(x, 0) through the inverse transfer function, divided by inputScale;
  * auto-exposure: key 0.18 over the geometric mean of the mean luminance of <= 16x16-pixel bins
    (bins with mean luminance <= 1e-8 skipped).
The GPU implementation (csrc/rs_denoise.hip) is checked against this module with the same weights.
`quantize=True` rounds weights and every stored activation to float16, as the GPU stores them, so the
two differ only by float32 accumulation order (tight tolerance); without it the comparison includes the
float16 storage error (looser tolerance) -- both stated in tests/test_gpu_denoise.py.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F

# PU (perceptually uniform) transfer function constants of OIDN's HDR path
PU_A, PU_B, PU_C = 1.41283765e+03, 1.64593172e+00, 4.31384981e-01
PU_D, PU_E, PU_F, PU_G = -2.94139609e-03, 1.92653254e-01, 6.26026094e-03, 9.98620152e-01
PU_Y0, PU_Y1 = 1.57945760e-06, 3.22087631e-02
PU_X0, PU_X1 = 2.23151711e-03, 3.70974749e-01
HDR_Y_MAX = 65504.0


def _f32(x):
    return np.asarray(x, dtype=np.float32)


def pu_forward(y):
    y = _f32(y)
    with np.errstate(divide="ignore", invalid="ignore"):
        a = np.float32(PU_A) * y
        b = np.float32(PU_B) * np.power(y, np.float32(PU_C)) + np.float32(PU_D)
        c = np.float32(PU_E) * np.log(y + np.float32(PU_F)) + np.float32(PU_G)
    return np.where(y <= np.float32(PU_Y0), a, np.where(y <= np.float32(PU_Y1), b, c)).astype(np.float32)


def pu_inverse(x):
    x = _f32(x)
    with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
        a = x / np.float32(PU_A)
        b = np.power((x - np.float32(PU_D)) / np.float32(PU_B), np.float32(1.0 / PU_C))
        c = np.exp((x - np.float32(PU_G)) / np.float32(PU_E)) - np.float32(PU_F)
    return np.where(x <= np.float32(PU_X0), a, np.where(x <= np.float32(PU_X1), b, c)).astype(np.float32)


NORM_SCALE = np.float32(1.0) / pu_forward(np.float32(HDR_Y_MAX))


def luminance(c):
    c = _f32(c)
    return (np.float32(0.212671) * c[..., 0] + np.float32(0.715160) * c[..., 1]
            + np.float32(0.072169) * c[..., 2]).astype(np.float32)


def autoexposure(color: np.ndarray) -> np.float32:
    """key / exp2(mean log2 L) over ceil(H/16) x ceil(W/16) bins (bin b spans [b*H/n, (b+1)*H/n))."""
    H, W = color.shape[:2]
    nbh, nbw = -(-H // 16), -(-W // 16)
    lum = luminance(color)
    s, n = np.float32(0.0), 0
    for i in range(nbh):
        y0, y1 = i * H // nbh, (i + 1) * H // nbh
        for j in range(nbw):
            x0, x1 = j * W // nbw, (j + 1) * W // nbw
            L = np.float32(lum[y0:y1, x0:x1].astype(np.float64).sum()) / np.float32((y1 - y0) * (x1 - x0))
            if L > np.float32(1e-8):
                s += np.float32(math.log2(L))
                n += 1
    return np.float32(0.18) / np.float32(2.0 ** (s / n)) if n else np.float32(1.0)


def _sanitize(x, lo, hi):
    x = np.nan_to_num(_f32(x), nan=0.0, posinf=hi, neginf=lo)
    return np.clip(x, lo, hi).astype(np.float32)


def preprocess(color, albedo, normal, scale, ic: int) -> np.ndarray:
    """(ic, Hp, Wp) float32 network input, zero outside the image."""
    H, W = color.shape[:2]
    Hp, Wp = -(-H // 16) * 16, -(-W // 16) * 16
    x = np.zeros((ic, Hp, Wp), np.float32)
    c = np.nan_to_num(_f32(color), nan=0.0) * np.float32(scale)
    c = np.clip(c, 0.0, HDR_Y_MAX).astype(np.float32)
    x[0:3, :H, :W] = (pu_forward(c) * NORM_SCALE).transpose(2, 0, 1)
    if ic >= 6:
        x[3:6, :H, :W] = _sanitize(albedo, 0.0, 1.0).transpose(2, 0, 1)
    if ic >= 9:
        n = _sanitize(normal, -1.0, 1.0)
        x[6:9, :H, :W] = (n * np.float32(0.5) + np.float32(0.5)).transpose(2, 0, 1)
    return x


def postprocess(y: np.ndarray, scale, H: int, W: int) -> np.ndarray:
    """(3, Hp, Wp) network output -> (H, W, 3) linear HDR radiance."""
    v = _f32(y[:3, :H, :W]).transpose(1, 2, 0)
    v = np.where(v > 0, v, np.float32(0.0)).astype(np.float32)
    out = pu_inverse(v / NORM_SCALE) / np.float32(scale)
    return np.nan_to_num(out, nan=0.0, posinf=0.0).astype(np.float32)


LAYERS = ["enc_conv0", "enc_conv1", "enc_conv2", "enc_conv3", "enc_conv4", "enc_conv5a", "enc_conv5b",
          "dec_conv4a", "dec_conv4b", "dec_conv3a", "dec_conv3b", "dec_conv2a", "dec_conv2b",
          "dec_conv1a", "dec_conv1b", "dec_conv0"]


def unet(weights: dict, x: torch.Tensor, quantize: bool = False) -> torch.Tensor:
    """OIDN's UNet on a (1, ic, Hp, Wp) tensor.  quantize: float16 weights and stored activations."""
    def q(t):
        return t.half().float() if quantize else t

    def conv(name, t, relu=True):
        w = q(torch.as_tensor(weights[name + ".weight"], dtype=torch.float32))
        b = torch.as_tensor(weights[name + ".bias"], dtype=torch.float32)
        y = F.conv2d(t, w, b, padding=1)
        return torch.relu(y) if relu else y

    pool = lambda t: F.max_pool2d(t, 2)                         # noqa: E731
    up = lambda t: F.interpolate(t, scale_factor=2, mode="nearest")   # noqa: E731
    x = q(x)
    t = q(conv("enc_conv0", x))
    p1 = q(pool(conv("enc_conv1", t)))
    p2 = q(pool(conv("enc_conv2", p1)))
    p3 = q(pool(conv("enc_conv3", p2)))
    p4 = q(pool(conv("enc_conv4", p3)))
    t = q(conv("enc_conv5a", p4))
    t = q(conv("enc_conv5b", t))
    t = q(conv("dec_conv4a", torch.cat([up(t), p3], 1)))
    t = q(conv("dec_conv4b", t))
    t = q(conv("dec_conv3a", torch.cat([up(t), p2], 1)))
    t = q(conv("dec_conv3b", t))
    t = q(conv("dec_conv2a", torch.cat([up(t), p1], 1)))
    t = q(conv("dec_conv2b", t))
    t = q(conv("dec_conv1a", torch.cat([up(t), x], 1)))
    t = q(conv("dec_conv1b", t))
    return conv("dec_conv0", t, relu=False)


# The GPU's activation tensors (rs_denoiser_dump index) and each convolution's sources / post-op / output
# tensor -- the same graph as `unet`, spelled per layer for the per-layer parity test.
NET = [
    ("enc_conv0", [(0, False)], "relu", 1), ("enc_conv1", [(1, False)], "pool", 2),
    ("enc_conv2", [(2, False)], "pool", 3), ("enc_conv3", [(3, False)], "pool", 4),
    ("enc_conv4", [(4, False)], "pool", 5), ("enc_conv5a", [(5, False)], "relu", 6),
    ("enc_conv5b", [(6, False)], "relu", 7), ("dec_conv4a", [(7, True), (4, False)], "relu", 8),
    ("dec_conv4b", [(8, False)], "relu", 9), ("dec_conv3a", [(9, True), (3, False)], "relu", 10),
    ("dec_conv3b", [(10, False)], "relu", 11), ("dec_conv2a", [(11, True), (2, False)], "relu", 12),
    ("dec_conv2b", [(12, False)], "relu", 13), ("dec_conv1a", [(13, True), (0, False)], "relu", 14),
    ("dec_conv1b", [(14, False)], "relu", 15), ("dec_conv0", [(15, False)], "linear", None),
]


def layer64(weights: dict, name: str, inputs, post: str, magnitude: bool = False) -> np.ndarray:
    """One convolution in float64 with float16-rounded weights: inputs = [(C, h, w) arrays, upsampled?]
    -> (O, h', w') float64 (before the float16 rounding the GPU stores).  magnitude: the same sums over
    |w| |x| plus |bias| (scale of a float32 accumulation's rounding error)."""
    xs = []
    for a, upsampled in inputs:
        t = torch.as_tensor(np.asarray(a, np.float64))[None]
        xs.append(F.interpolate(t, scale_factor=2, mode="nearest") if upsampled else t)
    x = torch.cat(xs, 1)
    w = torch.as_tensor(np.asarray(weights[name + ".weight"], np.float32)).half().double()
    b = torch.as_tensor(np.asarray(weights[name + ".bias"], np.float32)).double()
    if magnitude:
        x, w, b = x.abs(), w.abs(), b.abs()
    y = F.conv2d(x, w, b, padding=1)
    if post in ("relu", "pool") and not magnitude:
        y = torch.relu(y)
    if post == "pool":
        y = F.max_pool2d(y, 2)
    return y[0].numpy()


def denoise(color, albedo, normal, weights: dict, input_scale=None, quantize: bool = False,
            threads: int | None = None, return_network_output: bool = False):
    """The "RT" filter, hdr = true: (H, W, 3) float32 colour / albedo / normal -> (H, W, 3)."""
    if threads:
        torch.set_num_threads(threads)
    H, W = color.shape[:2]
    ic = int(np.asarray(weights["enc_conv0.weight"]).shape[1])
    scale = autoexposure(color) if input_scale is None else np.float32(input_scale)
    x = torch.from_numpy(preprocess(color, albedo, normal, scale, ic))[None]
    with torch.no_grad():
        y = unet(weights, x, quantize=quantize)[0].numpy()
    out = postprocess(y, scale, H, W)
    return (out, y, scale) if return_network_output else out
