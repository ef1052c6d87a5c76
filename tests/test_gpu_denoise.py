"""GPU parity of the denoiser (csrc/rs_denoise.hip) against the reference
(oracle/denoise_ref.py) with the same weights.

Two levels:
  * per convolution (test_every_layer_matches_float64): each layer's float16 output tensor (rs_denoiser_dump)
    vs the layer recomputed in float64 from the GPU's own float16 inputs with float16-rounded weights, then
    rounded to float16 -- equal except where the float32-vs-float64 accumulation moves a value across a
    float16 rounding boundary: every element within 1 float16 ulp + 3e-5 x (sum of |w x| + |b|, the scale of
    a float32 accumulation's rounding error over <= 1440 terms), at most 2 % of them different at all; zero
    borders and zero channel padding checked too; the last layer's float32 output (with the inverse
    transfer function) within 2e-4 relative of the float64 result;
  * end to end vs the fp32 reference with float16 storage (`quantize=True`): in the network-output (PU)
    domain mean |err| <= 1e-3, max <= 2e-2.  With float16 storage the result depends on the accumulation
    order: two exact-storage references that differ only in float32 vs float64 accumulation already differ
    by 3.6e-4 mean / 2.0e-3 max on the 48x64 input (He-initialised weights are close to chaotic); the
    tolerance is ~3x that.
The weights are He-initialised random UNet weights (OIDN's trained weights are not shipped with the
reference), so what is pinned is the network, its fused pooling / upsampling / concatenation and the
pre/post-processing, not OIDN's output.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from restir_amd import Renderer, metric_params, scenes, tza  # noqa: E402
from restir_amd.denoise import Denoiser  # noqa: E402

import denoise_ref as ref  # noqa: E402  (oracle/, test infrastructure)


def _images(H, W, seed=0):
    rng = np.random.default_rng(seed)
    color = rng.lognormal(-0.5, 1.2, (H, W, 3)).astype(np.float32)
    albedo = rng.uniform(0, 1, (H, W, 3)).astype(np.float32)
    n = rng.standard_normal((H, W, 3)).astype(np.float32)
    n /= np.linalg.norm(n, axis=-1, keepdims=True)
    return color, albedo, n


def _err(got, want, scale=1.0):
    """(mean, max) |error| in the network-output (PU) domain of two denoised images."""
    to_x = lambda y: ref.pu_forward(np.float32(scale) * y) * ref.NORM_SCALE   # noqa: E731
    e = np.abs(to_x(got) - to_x(want))
    return float(e.mean()), float(e.max())


@pytest.fixture(scope="module")
def ctx():
    assert torch.cuda.is_available()
    r = Renderer(64, 48)
    w = tza.random_unet_weights(seed=7)
    d = Denoiser(r, w)
    yield r, d, w
    d.close()
    r.close()


def _run(d, color, albedo, normal, scale=None):
    dev = lambda a: torch.from_numpy(a).cuda()   # noqa: E731
    out = d.execute(dev(color), dev(albedo), dev(normal), input_scale=scale)
    torch.cuda.synchronize()
    return out.cpu().numpy()


@pytest.mark.parametrize("H,W", [(48, 64), (29, 37), (1, 1), (16, 16), (135, 240)])
def test_denoise_matches_reference(ctx, H, W):
    r, d, w = ctx
    color, albedo, normal = _images(H, W, seed=H * 1000 + W)
    got = _run(d, color, albedo, normal, scale=0.7)
    want_q = ref.denoise(color, albedo, normal, w, input_scale=0.7, quantize=True)
    want = ref.denoise(color, albedo, normal, w, input_scale=0.7)
    assert got.shape == (H, W, 3) and np.isfinite(got).all()
    mq, xq = _err(got, want_q, 0.7)
    m32, x32 = _err(got, want, 0.7)
    print(f"{H}x{W}: PU-domain |err| vs fp16-storage reference mean {mq:.2e} max {xq:.2e}; vs fp32 {m32:.2e} / {x32:.2e}")
    assert mq <= 1e-3 and xq <= 2e-2, (mq, xq)


@pytest.mark.parametrize("H,W", [(48, 64), (37, 83)])
def test_every_layer_matches_float64(ctx, H, W):
    r, d, w = ctx
    color, albedo, normal = _images(H, W, seed=31 + H)
    got = _run(d, color, albedo, normal, scale=0.9)
    t = {}
    for i in range(16):
        a, real = d.dump(i)
        assert not a[0].any() and not a[-1].any() and not a[:, 0].any() and not a[:, -1].any(), f"tensor {i}: border"
        assert not a[..., real:].any(), f"tensor {i}: channel padding"
        t[i] = a[1:-1, 1:-1, :real].astype(np.float64).transpose(2, 0, 1)
    # the network input tensor: the reference's preprocessing rounded to float16
    want_in = ref.preprocess(color, albedo, normal, np.float32(0.9), 9).astype(np.float16).astype(np.float64)
    assert np.abs(t[0] - want_in).max() <= np.abs(np.spacing(want_in.astype(np.float16))).max()
    for name, srcs, post, dst in ref.NET:
        y = ref.layer64(w, name, [(t[s], up) for s, up in srcs], post)
        if dst is None:        # dec_conv0 + output transform, float32 on the GPU
            want = ref.postprocess(y.astype(np.float32), np.float32(0.9), H, W)
            np.testing.assert_allclose(got, want, rtol=2e-4, atol=1e-6, err_msg=name)
            continue
        y16 = y.astype(np.float16)
        g16 = t[dst].astype(np.float16)
        assert g16.shape == y16.shape, name
        ulp = np.spacing(np.abs(y16)).astype(np.float64)
        mag = ref.layer64(w, name, [(t[s], up) for s, up in srcs], post, magnitude=True)
        bound = ulp * 1.0001 + 3e-5 * mag
        diff = np.abs(g16.astype(np.float64) - y16.astype(np.float64))
        off = diff > 0
        print(f"{name}: {off.mean() * 100:.3f} % of {diff.size} elements differ, max {float((diff / bound).max()):.3f} of the bound")
        assert (diff <= bound).all(), (name, float((diff / bound).max()))
        assert off.mean() <= 0.02, (name, float(off.mean()))


@pytest.mark.parametrize("H,W,grid", [(48, 64, "2"), (37, 83, "3"), (540, 960, None), (1080, 1920, None)])
def test_pipelined_conv_bit_identical(monkeypatch, H, W, grid):
    """k_conv3p (the persistent LDS-DMA pipeline, csrc/rs_denoise.hip) against k_conv3 on the layers it runs
    (dec_conv2a / 2b / 1a): the same k-steps in the same order on the same MFMA, so every tensor is bit-identical.
    A capped grid makes each workgroup walk several tiles (the stage pipeline across tile boundaries)."""
    r = Renderer(64, 48)
    w = tza.random_unet_weights(seed=11)
    color, albedo, normal = _images(H, W, seed=5 + H)
    outs = {}
    try:
        for pipe in ("0", "1"):                # 1: every layer k_conv3p applies to
            monkeypatch.setenv("RESTIR_DN_PIPE", pipe)
            if grid is not None:
                monkeypatch.setenv("RESTIR_DN_PIPE_GRID", grid)
            d = Denoiser(r, w)
            out = _run(d, color, albedo, normal, scale=0.8)
            outs[pipe] = (out, [d.dump(i)[0] for i in range(16)])
            d.close()
    finally:
        r.close()
    (o0, t0), (o1, t1) = outs["0"], outs["1"]
    for i in range(16):
        assert np.array_equal(t0[i].view(np.uint16), t1[i].view(np.uint16)), f"tensor {i}"
    assert np.array_equal(o0, o1)


def test_autoexposure_matches_reference(ctx):
    r, d, w = ctx
    for (H, W), seed in (((48, 64), 1), ((37, 91), 2), ((1080 // 4, 1920 // 4), 3)):
        color, albedo, normal = _images(H, W, seed)
        _run(d, color, albedo, normal)                    # input_scale unset: auto-exposure
        got = d.scale()
        want = float(ref.autoexposure(color))
        assert got == pytest.approx(want, rel=1e-4), (H, W, got, want)


def test_autoexposure_end_to_end(ctx):
    r, d, w = ctx
    color, albedo, normal = _images(40, 56, seed=5)
    got = _run(d, color, albedo, normal)
    want = ref.denoise(color, albedo, normal, w, quantize=True)
    m, x = _err(got, want, ref.autoexposure(color))
    assert m <= 1e-3 and x <= 2e-2, (m, x)


def test_half_archive_equals_float_archive(ctx):
    r, d, w = ctx
    wh = {k: v.astype(np.float16).astype(np.float32) for k, v in w.items()}
    d_f = Denoiser(r, tza.write_tza(wh, "f"))
    d_h = Denoiser(r, tza.write_tza(wh, "h"))
    color, albedo, normal = _images(32, 48, seed=9)
    a = _run(d_f, color, albedo, normal, scale=1.0)
    b = _run(d_h, color, albedo, normal, scale=1.0)
    np.testing.assert_array_equal(a, b)
    d_f.close()
    d_h.close()


def test_color_only_and_albedo_weights(ctx):
    r, _, _ = ctx
    for ic in (3, 6):
        w = tza.random_unet_weights(seed=11, ic=ic)
        d = Denoiser(r, w)
        color, albedo, normal = _images(24, 40, seed=ic)
        dev = lambda a: torch.from_numpy(a).cuda()   # noqa: E731
        out = d.execute(dev(color), dev(albedo) if ic >= 6 else None, None, input_scale=1.3)
        torch.cuda.synchronize()
        want = ref.denoise(color, albedo, normal, w, input_scale=1.3, quantize=True)
        m, x = _err(out.cpu().numpy(), want, 1.3)
        assert m <= 1e-3 and x <= 2e-2, (ic, m, x)
        d.close()


def test_denoise_frame_and_post_display():
    """The reference's per-frame use: accumulator + the frame's G-buffer kd / normal, and the display of
    the denoised accumulator with RenderParams::denoise (pg/simpleguidx11.cpp:246-292)."""
    W, H = 96, 64
    r = Renderer(W, H)
    sc = scenes.cornell_many_lights(64)
    s = r.load_scene(sc)
    w = tza.random_unet_weights(seed=21)
    d = Denoiser(r, w)
    prm = metric_params(m_area=8)
    frame = r.produce_restir(s, sc.camera, prm, 0).copy()
    r.post_frame(accumulate=False, stats=False)          # accumulator = the frame
    got = d.frame_output()
    g = r.gbuffer()                                      # per pixel: pos3 n3 kd3 ks3 Le3 ...
    normal, kd = g[..., 3:6], g[..., 6:9]
    want = ref.denoise(frame, kd, normal, w, quantize=True)
    m, x = _err(got, want, ref.autoexposure(frame))
    assert m <= 1e-3 and x <= 2e-2, (m, x)
    # post_frame(denoise=True): display = compress(aces(denoised))
    r.post_reset()
    r.produce_restir(s, sc.camera, prm, 1)
    r.set_denoiser(d)
    r.post_frame(accumulate=False, stats=False, denoise=True)
    disp = r.display_rgba()[..., :3]
    den = d.frame_output()                               # same inputs again: same output
    x = den
    a, b, c, dd, e = 2.51, 0.03, 2.43, 0.59, 0.14
    t = np.clip((x * (a * x + b)) / (x * (c * x + dd) + e), 0, 1)
    srgb = np.where(t <= 0.0031308, t * 12.92, 1.055 * np.power(t, 1 / 2.4) - 0.055)
    np.testing.assert_allclose(disp, srgb, atol=2e-5)
    r.set_denoiser(None)
    with pytest.raises(Exception):
        r.post_frame(denoise=True)                       # no denoiser set: loud error
    d.close()
    r.close()


def test_denoiser_lifetime_and_rejected_post_frame():
    """(1) a post_frame(denoise=True) that is rejected (no denoiser) leaves the accumulator and
    accFrameCtr as they were; (2) destroying the attached denoiser clears the context's post-frame denoiser
    (the next denoise=True call fails loudly instead of using freed memory); (3) destroying the context
    first detaches its denoisers: their calls fail with an error, and their close() is still safe."""
    W, H = 64, 48
    sc = scenes.cornell_many_lights(64)
    prm = metric_params(m_area=4)
    r = Renderer(W, H)
    s = r.load_scene(sc)
    r.produce_restir(s, sc.camera, prm, 0)
    _, st0 = r.post_frame(accumulate=True)
    assert st0.acc_frames_used == 0
    with pytest.raises(Exception):
        r.post_frame(accumulate=True, denoise=True)      # rejected before the accumulator is touched
    r.produce_restir(s, sc.camera, prm, 1)
    _, st1 = r.post_frame(accumulate=True)
    assert st1.acc_frames_used == 1, st1.acc_frames_used
    d = Denoiser(r, tza.random_unet_weights(seed=3))
    r.set_denoiser(d)
    r.post_frame(accumulate=True, denoise=True)
    d.close()                                            # attached: the context forgets it
    with pytest.raises(Exception):
        r.post_frame(accumulate=True, denoise=True)
    d2 = Denoiser(r, tza.random_unet_weights(seed=4))
    r.set_denoiser(d2)
    s.close()
    r.close()                                            # context first: d2 is detached, not freed
    import torch
    x = torch.zeros((H, W, 3), dtype=torch.float32, device="cuda")
    with pytest.raises(Exception):
        d2.execute(x, x, x)
    d2.close()
