"""Denoiser timing probe: execute() at WxH with random OIDN-shaped weights; HIP-event ms per call,
algorithmic TFLOP/s (2 x MAC of the padded image) vs the 2.5 PFLOP/s dense f16 MFMA peak."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "restir-embree_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from restir_amd import Renderer, tza  # noqa: E402
from restir_amd.denoise import Denoiser, gflop_per_frame  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--width", type=int, default=1920)
ap.add_argument("--height", type=int, default=1080)
ap.add_argument("--iters", type=int, default=20)
a = ap.parse_args()
r = Renderer(64, 64)
d = Denoiser(r, tza.random_unet_weights(seed=1))
rng = np.random.default_rng(0)
H, W = a.height, a.width
col = torch.from_numpy(rng.lognormal(-0.5, 1.0, (H, W, 3)).astype(np.float32)).cuda()
alb = torch.rand(H, W, 3, device="cuda")
nrm = torch.nn.functional.normalize(torch.randn(H, W, 3, device="cuda"), dim=-1).contiguous()
out = torch.empty_like(col)
d.set_timing(True)
for _ in range(3):
    d.execute(col, alb, nrm, out)
torch.cuda.synchronize()
ms = []
t0 = time.perf_counter()
for _ in range(a.iters):
    d.execute(col, alb, nrm, out)
    ms.append(d.last_ms())
wall = (time.perf_counter() - t0) / a.iters * 1e3
gf = gflop_per_frame(d.info(), W, H)
m = float(np.median(ms))
print(f"denoise {W}x{H}: {m:.3f} ms/execute (HIP events, median of {a.iters}; wall {wall:.3f}), "
      f"{gf:.1f} GFLOP -> {gf / m:.1f} TFLOP/s = {gf / m / 2500:.3f} of 2.5 PF f16 dense")
lm = np.zeros(17)
for _ in range(5):
    d.execute(col, alb, nrm, out)
    lm += np.array(d.layer_ms())
lm /= 5
names = ["input+ae", "enc_conv0", "enc_conv1", "enc_conv2", "enc_conv3", "enc_conv4", "enc_conv5a", "enc_conv5b",
         "dec_conv4a", "dec_conv4b", "dec_conv3a", "dec_conv3b", "dec_conv2a", "dec_conv2b", "dec_conv1a",
         "dec_conv1b", "dec_conv0"]
print("per-layer ms (HIP events, mean of 5): " + ", ".join(f"{n} {v:.4f}" for n, v in zip(names, lm)))
