"""Denoiser parity diagnostics: GPU vs the fp16-storage reference for weight subsets that isolate
parts of the UNet, errors in the network-output (PU) domain."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("restir-embree_amd", "oracle"):
    sys.path.insert(0, os.path.join(ROOT, p))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from restir_amd import Renderer, tza  # noqa: E402
from restir_amd.denoise import Denoiser  # noqa: E402
import denoise_ref as ref  # noqa: E402

H, W = 48, 64
rng = np.random.default_rng(1)
color = rng.lognormal(-0.5, 1.2, (H, W, 3)).astype(np.float32)
albedo = rng.uniform(0, 1, (H, W, 3)).astype(np.float32)
n = rng.standard_normal((H, W, 3)).astype(np.float32)
n /= np.linalg.norm(n, axis=-1, keepdims=True)
r = Renderer(64, 64)
base = tza.random_unet_weights(seed=7)


def xdom(y):
    return ref.pu_forward(y * np.float32(0.7)) * ref.NORM_SCALE


def run(name, w):
    d = Denoiser(r, w)
    dev = lambda a: torch.from_numpy(a).cuda()  # noqa: E731
    got = d.execute(dev(color), dev(albedo), dev(n), input_scale=0.7)
    torch.cuda.synchronize()
    got = got.cpu().numpy()
    q = ref.denoise(color, albedo, n, w, input_scale=0.7, quantize=True)
    f = ref.denoise(color, albedo, n, w, input_scale=0.7)
    gx, qx, fx = xdom(got), xdom(q), xdom(f)
    e = np.abs(gx - qx)
    iy, ix, ic = np.unravel_index(np.argmax(e), e.shape)
    print(f"{name:28s} |x| mean {np.abs(qx).mean():.3e}  gpu-refq max {e.max():.3e} mean {e.mean():.3e} "
          f"at ({iy},{ix},{ic})  refq-ref32 mean {np.abs(qx - fx).mean():.3e}  gpu-ref32 mean {np.abs(gx - fx).mean():.3e}")
    rows = e.mean(axis=(1, 2))
    cols = e.mean(axis=(0, 2))
    print("   row err (x1e4):", np.round(rows * 1e4, 1).tolist()[:48])
    print("   col err (x1e4):", np.round(cols * 1e4, 1).tolist()[:64])
    d.close()


def only(keep, w=base, zero_in=()):
    out = {}
    for k, v in w.items():
        layer = k.rsplit(".", 1)[0]
        out[k] = v if layer in keep else np.zeros_like(v)
    for k, sl in zero_in:
        out[k] = out[k].copy()
        out[k][sl] = 0
    return out


run("full", base)
run("IN->dec1a->dec1b->dec0", only({"dec_conv1a", "dec_conv1b", "dec_conv0"}))
run("IN->dec1a(+bias)", only({"dec_conv1a", "dec_conv1b", "dec_conv0"}))
run("enc0,enc1->dec2a..", only({"enc_conv0", "enc_conv1", "dec_conv2a", "dec_conv2b", "dec_conv1a", "dec_conv1b", "dec_conv0"},
                                zero_in=(("dec_conv1a.weight", (slice(None), slice(64, None))),)))
run("enc0..enc2,dec3b.. ", only({"enc_conv0", "enc_conv1", "enc_conv2", "dec_conv3a", "dec_conv3b", "dec_conv2a",
                                  "dec_conv2b", "dec_conv1a", "dec_conv1b", "dec_conv0"}))
