"""CPU tests of the denoiser's host side: the tensor-archive format, the C ABI's
host-only weight check (topology, error messages), and properties of the fp32 reference
(oracle/denoise_ref.py) the GPU tests compare against.  No device work."""
import struct

import numpy as np
import pytest

from restir_amd import tza
from restir_amd.denoise import check_weights
from restir_amd.renderer import RestirError

import denoise_ref as ref  # oracle/ (test infrastructure)


@pytest.fixture(scope="module")
def weights():
    return tza.random_unet_weights(seed=3)


@pytest.mark.parametrize("dtype", ["f", "h"])
def test_tza_round_trip(weights, dtype):
    blob = tza.write_tza(weights, dtype)
    back = tza.read_tza(blob)
    assert list(back) == list(weights)
    for k, v in weights.items():
        want = v if dtype == "f" else v.astype(np.float16).astype(np.float32)
        np.testing.assert_array_equal(back[k], want)


def test_check_weights_reports_topology(weights):
    info = check_weights(tza.write_tza(weights))
    shapes = tza.unet_shapes(9)
    assert info.input_channels == 9
    assert list(info.channels) == [shapes[n][0] for n in ref.LAYERS]
    params = sum(o * i * 9 + o for o, i in shapes.values())
    assert info.parameters == params
    # MAC per padded input pixel: a layer at pooling level l runs on 1/4^l of the pixels
    levels = [0, 0, 1, 2, 3, 4, 4, 3, 3, 2, 2, 1, 1, 0, 0, 0]
    mac = sum(shapes[n][0] * shapes[n][1] * 9 / 4 ** lv for n, lv in zip(ref.LAYERS, levels))
    assert info.mac_per_pixel == pytest.approx(mac)
    assert 1.0e5 < mac < 1.5e5


def test_check_weights_other_input_sets():
    for ic in (3, 6):
        assert check_weights(tza.write_tza(tza.random_unet_weights(seed=1, ic=ic))).input_channels == ic


def test_check_weights_rejects_malformed(weights):
    blob = tza.write_tza(weights)
    with pytest.raises(RestirError, match="magic"):
        check_weights(b"\x00\x00" + blob[2:])
    with pytest.raises(RestirError, match="version"):
        check_weights(blob[:2] + b"\x03" + blob[3:])
    with pytest.raises(RestirError):
        check_weights(blob[:40])
    w = dict(weights)
    del w["dec_conv2b.bias"]
    with pytest.raises(RestirError, match="dec_conv2b.bias"):
        check_weights(tza.write_tza(w))
    w = dict(weights)
    w["dec_conv3a.weight"] = w["dec_conv3a.weight"][:, :100]
    with pytest.raises(RestirError, match="dec_conv3a"):
        check_weights(tza.write_tza(w))
    w = dict(weights)
    w["dec_conv0.weight"] = np.zeros((4, 32, 3, 3), np.float32)
    w["dec_conv0.bias"] = np.zeros(4, np.float32)
    with pytest.raises(RestirError, match="dec_conv0"):
        check_weights(tza.write_tza(w))
    # a table entry pointing past the end of the blob
    magic, major, minor, toff = struct.unpack_from("<HBBQ", blob, 0)
    bad = bytearray(blob)
    struct.pack_into("<Q", bad, 4, len(blob) + 100)
    with pytest.raises(RestirError, match="table"):
        check_weights(bytes(bad))


def test_pu_transfer_round_trip():
    y = np.concatenate([np.geomspace(1e-8, 65504, 2000), [0.0, ref.PU_Y0, ref.PU_Y1]]).astype(np.float32)
    x = ref.pu_forward(y)
    assert np.all(np.diff(x[:2000]) > 0)                              # monotone
    np.testing.assert_allclose(ref.pu_inverse(x), y, rtol=2e-5, atol=1e-12)
    assert float(ref.pu_forward(np.float32(65504.0)) * ref.NORM_SCALE) == pytest.approx(1.0, abs=1e-6)


def test_autoexposure_constant_and_bins():
    img = np.full((40, 50, 3), 2.0, np.float32)
    assert float(ref.autoexposure(img)) == pytest.approx(0.18 / 2.0, rel=1e-6)
    dark = np.zeros((40, 50, 3), np.float32)
    assert float(ref.autoexposure(dark)) == 1.0                        # every bin below eps
    half = img.copy()
    half[:, :25] = 0.0                                                 # bins at zero are skipped
    assert float(ref.autoexposure(half)) == pytest.approx(0.18 / 2.0, rel=1e-6)


def test_reference_shapes_and_quantised_close(weights):
    rng = np.random.default_rng(0)
    H, W = 21, 35
    color = rng.lognormal(0.0, 1.0, (H, W, 3)).astype(np.float32)
    albedo = rng.uniform(0, 1, (H, W, 3)).astype(np.float32)
    n = rng.standard_normal((H, W, 3)).astype(np.float32)
    n /= np.linalg.norm(n, axis=-1, keepdims=True)
    a = ref.denoise(color, albedo, n, weights)
    b = ref.denoise(color, albedo, n, weights, quantize=True)
    assert a.shape == (H, W, 3) and np.isfinite(a).all() and (a >= 0).all()
    rel = np.abs(a - b).sum() / np.abs(a).sum()
    assert rel < 2e-2, rel
