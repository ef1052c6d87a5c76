"""Scene-loader image decoders (rs_image_decode) -- CPU only, no device needed.

The reference decodes textures with FreeImage (pg/Texture.cpp:9-57), which is not available here.  The
decoders are pinned against PIL (an independent PNG decoder) and against numpy restatements of the
Radiance RGBE / PFM / PNM formats written by this test: bit-exact texels.
"""
import os
import struct

import numpy as np
import pytest
from PIL import Image

from restir_amd.renderer import RestirError, decode_image


def _rgbe_encode(img):
    """float32 (H, W, 3) -> RGBE bytes (Ward's float2rgbe) and the floats a decoder must return."""
    v = img.max(-1).astype(np.float64)
    m, e = np.frexp(v)
    scale = np.where(v > 1e-32, m * 256.0 / np.where(v > 0, v, 1), 0.0)
    rgb = np.clip(np.floor(img * scale[..., None]), 0, 255).astype(np.uint8)
    ex = np.where(v > 1e-32, e + 128, 0).astype(np.uint8)
    rgbe = np.concatenate([rgb, ex[..., None]], -1)
    f = np.where(rgbe[..., 3:4] > 0, np.ldexp(1.0, rgbe[..., 3:4].astype(np.int32) - 136), 0.0)
    dec = (rgbe[..., :3].astype(np.float64) * f).astype(np.float32)
    return rgbe, dec


def _rle_channel(a):
    out, i, n = bytearray(), 0, len(a)
    while i < n:
        j = i
        while j < n and j - i < 127 and a[j] == a[i]:
            j += 1
        if j - i >= 3:
            out += bytes([128 + (j - i), a[i]])
            i = j
            continue
        j = i
        while j < n and j - i < 128 and not (j + 2 < n and a[j] == a[j + 1] == a[j + 2]):
            j += 1
        out += bytes([j - i]) + bytes(a[i:j])
        i = j
    return out


def _write_hdr(path, rgbe, rle):
    H, W, _ = rgbe.shape
    with open(path, "wb") as f:
        f.write(b"#?RADIANCE\nFORMAT=32-bit_rle_rgbe\nEXPOSURE=1.0\n\n")
        f.write(f"-Y {H} +X {W}\n".encode())
        for y in range(H):
            if rle:
                f.write(bytes([2, 2, W >> 8, W & 255]))
                for c in range(4):
                    f.write(_rle_channel(rgbe[y, :, c].tolist()))
            else:
                f.write(rgbe[y].tobytes())


@pytest.mark.parametrize("mode", ["RGB", "RGBA", "L", "LA", "P", "PT"])
def test_png_matches_pil(tmp_path, mode):
    rng = np.random.default_rng(3)
    H, W = 37, 53                                 # odd sizes: row padding, every filter type
    base = rng.integers(0, 256, size=(H, W, 4), dtype=np.uint8)
    base[:, : W // 2] //= 16                     # smooth + noisy halves so the encoder picks mixed filters
    if mode in ("P", "PT"):
        im = Image.fromarray(base[..., :3]).quantize(colors=40)
        if mode == "PT":
            im.info["transparency"] = bytes(range(0, 240, 6))
    else:
        arr = {"RGB": base[..., :3], "RGBA": base, "L": base[..., 0], "LA": base[..., :2]}[mode]
        im = Image.fromarray(arr, mode=mode)
    p = tmp_path / f"t_{mode}.png"
    im.save(p, optimize=True)
    got = decode_image(p)
    ref_im = Image.open(p)
    if mode == "PT":
        want = np.asarray(ref_im.convert("RGBA"))
    elif mode == "P":
        want = np.asarray(ref_im.convert("RGB"))
    elif mode == "LA":                             # FreeImage loads gray+alpha as 32-bit RGBA
        want = np.asarray(ref_im.convert("RGBA"))
    else:
        want = np.asarray(ref_im)
    if want.ndim == 2:
        want = want[:, :, None]
    assert got.dtype == np.uint8 and got.shape == want.shape
    assert np.array_equal(got, want)


def test_png_unsupported_variants(tmp_path):
    p16 = tmp_path / "d16.png"
    Image.fromarray(np.arange(64, dtype=np.uint16).reshape(8, 8) * 900).save(p16)
    with pytest.raises(RestirError, match="8-bit"):
        decode_image(p16)
    with pytest.raises(RestirError):
        decode_image(tmp_path / "missing.png")


@pytest.mark.parametrize("rle", [False, True])
def test_radiance_hdr(tmp_path, rle):
    rng = np.random.default_rng(9)
    img = (rng.lognormal(0, 2, size=(13, 40, 3))).astype(np.float32)
    img[3, 5:30] = img[3, 5]                      # long runs for the RLE path
    img[7] = 0.0
    rgbe, want = _rgbe_encode(img)
    p = tmp_path / f"sky_{int(rle)}.hdr"
    _write_hdr(p, rgbe, rle)
    got = decode_image(p)
    assert got.dtype == np.float32 and got.shape == (13, 40, 3)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("little,color", [(True, True), (False, True), (True, False)])
def test_pfm(tmp_path, little, color):
    rng = np.random.default_rng(4)
    C = 3 if color else 1
    img = rng.normal(size=(9, 11, C)).astype(np.float32)
    p = tmp_path / "t.pfm"
    with open(p, "wb") as f:
        f.write(f"{'PF' if color else 'Pf'}\n11 9\n{-1.0 if little else 1.0}\n".encode())
        f.write(np.ascontiguousarray(img[::-1]).astype("<f4" if little else ">f4").tobytes())   # bottom row first
    got = decode_image(p)
    want = img if color else np.repeat(img, 3, -1)
    assert np.array_equal(got, want)


def test_pnm(tmp_path):
    rng = np.random.default_rng(5)
    rgb = rng.integers(0, 256, size=(6, 7, 3), dtype=np.uint8)
    gray = rng.integers(0, 256, size=(6, 7), dtype=np.uint8)
    p6, p5 = tmp_path / "t.ppm", tmp_path / "t.pgm"
    p6.write_bytes(b"P6\n# comment\n7 6\n255\n" + rgb.tobytes())
    p5.write_bytes(b"P5 7 6 255\n" + gray.tobytes())
    assert np.array_equal(decode_image(p6), rgb)
    assert np.array_equal(decode_image(p5), gray[:, :, None])


@pytest.mark.parametrize("channels", [1, 2, 3, 4])
def test_png_encoder_roundtrip(tmp_path, channels):
    """rs_image_encode_png (the exportImage writer) -> PIL and our decoder read back the same bytes."""
    from PIL import Image
    from restir_amd.renderer import encode_png
    rng = np.random.default_rng(channels)
    px = rng.integers(0, 256, (23, 37, channels), dtype=np.uint8)
    p = tmp_path / "e.png"
    encode_png(p, px)
    got = np.asarray(Image.open(p))
    assert np.array_equal(got.reshape(px.shape), px)
    dec = decode_image(p)
    if channels == 2:                     # the decoder expands gray+alpha to RGBA (g, g, g, a)
        assert np.array_equal(dec[..., 0], px[..., 0]) and np.array_equal(dec[..., 3], px[..., 1])
    else:
        assert np.array_equal(dec.reshape(px.shape), px)


# ---------------------------------------------------------------- JPEG (csrc/rs_jpeg.cpp)
# The reference's textures are all JPEG (data/room/room.mtl:11,21,32, ...), decoded by FreeImage's libjpeg.  The
# decoder restates libjpeg-turbo's default reconstruction and is pinned bit-exact to PIL's libjpeg-turbo.
# (FreeImage 3.18 bundles IJG libjpeg 9c, which upsamples 4:2:0 chroma through a 16x16 scaled IDCT instead of
# the triangle filter -- chroma may differ from it in the low bits; parity unpinned against FreeImage itself.)
import hashlib  # noqa: E402
import json  # noqa: E402

_REF = "/root/reference/template"
_HASHES = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "jpeg_reference_hashes.json")


def test_jpeg_reference_textures_bit_exact_to_libjpeg_turbo():
    """Every JPEG the reference ships (52 textures + 2 screenshots: baseline and progressive, 4:2:0, 4:4:4 and
    greyscale) decodes to the pixel arrays PIL's libjpeg-turbo gives (committed SHA-256,
    tests/golden/gen_jpeg_hashes.py)."""
    golden = json.load(open(_HASHES))["files"]
    if not os.path.isdir(_REF):
        pytest.skip("/root/reference not present (the hashes are checked where it is)")
    assert len(golden) >= 52
    kinds = set()
    for rel, g in sorted(golden.items()):
        a = decode_image(os.path.join(_REF, rel))
        a = a.reshape(g["shape"])
        assert hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest() == g["sha256"], rel
        kinds.add((g["mode"], g["progressive"]))
    assert {("RGB", False), ("RGB", True), ("L", False)} <= kinds


def _jpeg_image(h, w, mode, seed):
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w]
    base = np.stack([(xx * 255 // max(1, w - 1)), (yy * 255 // max(1, h - 1)), ((xx + yy) * 7) % 256], -1).astype(np.float64)
    img = np.clip(base + rng.normal(0, 25, base.shape), 0, 255).astype(np.uint8)
    return Image.fromarray(img[..., 0] if mode == "L" else img)


@pytest.mark.parametrize("mode,sub,prog,opt,restart,size", [
    ("RGB", 2, False, False, 0, (64, 48)),        # baseline 4:2:0
    ("RGB", 0, False, True, 0, (37, 23)),         # 4:4:4, optimised tables, partial blocks
    ("RGB", 1, False, False, 0, (50, 33)),        # 4:2:2 (h2v1 fancy upsampling)
    ("RGB", 2, True, False, 0, (97, 61)),         # progressive 4:2:0, odd size
    ("RGB", 0, True, True, 0, (40, 40)),          # progressive 4:4:4
    ("L", 0, False, False, 0, (31, 17)),          # greyscale baseline
    ("L", 0, True, False, 0, (65, 66)),           # greyscale progressive
    ("RGB", 2, False, False, 3, (80, 56)),        # restart interval (DRI)
    ("RGB", 2, True, False, 2, (72, 40)),         # progressive with restarts
    ("RGB", 2, False, False, 0, (1, 1)),
    ("RGB", 2, False, False, 0, (3, 2)),          # chroma width <= 2: plain replication
])
def test_jpeg_synthetic_bit_exact_to_libjpeg_turbo(tmp_path, mode, sub, prog, opt, restart, size):
    w, h = size
    im = _jpeg_image(h, w, mode, seed=w * 131 + h)
    kw = dict(quality=87, progressive=prog, optimize=opt)
    if mode == "RGB":
        kw["subsampling"] = sub
    if restart:
        kw["restart_marker_blocks"] = restart
    path = tmp_path / "t.jpg"
    im.save(path, "JPEG", **kw)
    want = np.asarray(Image.open(path))
    got = decode_image(str(path)).reshape(want.shape)
    assert np.array_equal(got, want), int((got != want).sum())


def test_jpeg_unsupported_variants_fail_loudly(tmp_path):
    im = _jpeg_image(16, 16, "RGB", 1).convert("CMYK")
    path = tmp_path / "cmyk.jpg"
    im.save(path, "JPEG")
    with pytest.raises(RestirError, match="3-component"):
        decode_image(str(path))
    bad = tmp_path / "trunc.jpg"
    bad.write_bytes(b"\xff\xd8\xff\xdb\x00")
    with pytest.raises(RestirError):
        decode_image(str(bad))


def _jpeg_segments(data):
    """(marker, offset of the length field, length) of every segment before the first SOS's entropy data."""
    out, p = [], 2
    while p + 4 <= len(data) and data[p] == 0xFF:
        m = data[p + 1]
        ln = (data[p + 2] << 8) | data[p + 3]
        out.append((m, p + 2, ln))
        if m == 0xDA:
            break
        p += 2 + ln
    return out


def test_jpeg_malformed_inputs_fail_cleanly(tmp_path):
    """an over-subscribed DHT must be rejected before any lookahead-table write (it used to write
    past the decoder's stack tables), an absurd SOF size must not commit gigabytes, and a garbage entropy
    stream must decode to something or fail -- never crash.  Every failure is a clean RestirError (-1)."""
    im = _jpeg_image(32, 32, "RGB", 7)
    path = tmp_path / "ok.jpg"
    im.save(path, "JPEG", quality=90)
    good = bytearray(path.read_bytes())
    segs = _jpeg_segments(good)

    # 1. over-subscribed code lengths: three 1-bit codes (total count unchanged, so the segment stays well-formed)
    bad = bytearray(good)
    m, off, ln = next(s for s in segs if s[0] == 0xC4)
    counts = off + 3                        # length (2) + table class/id (1)
    take = 3
    for i in range(15, 0, -1):
        d = min(take, bad[counts + i])
        bad[counts + i] -= d
        take -= d
        if not take:
            break
    assert take == 0
    bad[counts] += 3
    p1 = tmp_path / "oversub.jpg"
    p1.write_bytes(bytes(bad))
    with pytest.raises(RestirError, match="Huffman"):
        decode_image(str(p1))

    # 2. a 65535 x 65535 SOF in a file of a few hundred bytes
    bad = bytearray(good)
    m, off, ln = next(s for s in segs if s[0] in (0xC0, 0xC1, 0xC2))
    bad[off + 3:off + 7] = b"\xff\xff\xff\xff"
    p2 = tmp_path / "huge.jpg"
    p2.write_bytes(bytes(bad))
    with pytest.raises(RestirError, match="limit"):
        decode_image(str(p2))

    # 3. random entropy data after the SOS header (no 0xFF bytes, so no markers): any result, or a clean error
    m, off, ln = segs[-1]
    assert m == 0xDA
    start = off + ln
    rng = np.random.default_rng(3)
    for trial in range(8):
        junk = rng.integers(0, 255, size=len(good) - start - 2, dtype=np.uint8).tobytes()
        p3 = tmp_path / f"junk{trial}.jpg"
        p3.write_bytes(bytes(good[:start]) + junk + b"\xff\xd9")
        try:
            got = decode_image(str(p3))
            assert got.size == 32 * 32 * 3
        except RestirError:
            pass
    # 4. truncated right after the SOS header
    p4 = tmp_path / "cut.jpg"
    p4.write_bytes(bytes(good[:start + 3]))
    try:
        decode_image(str(p4))
    except RestirError:
        pass
