"""Tensor archives (.tza) -- the weight format of Open Image Denoise, which the reference's denoiser
loads its built-in "rt_hdr_alb_nrm" weights from (OIDN 2.3.3, pg/simpleguidx11.cpp:63-70).

Layout (little endian): u16 magic 0x41D7, u8 major version 2, u8 minor version 0, u64 table offset;
tensor data; at the table offset: u32 tensor count, then per tensor: u16 name length, name bytes,
u8 ndims, u32 dims[ndims], layout chars[ndims] ("oihw" for weights, "x" for biases), data type char
('f' float32 or 'h' float16), u64 data offset.  Restated from OIDN's published format; no OIDN file
ships with the reference, so the layout is unpinned against a real rt_*.tza -- librestir_amd.so's
parser (csrc/rs_denoise.hip) and this module are checked against each other.

The UNet topology (names and channel counts of OIDN's default "RT" network) lives in `unet_shapes`;
`random_unet_weights` makes He-initialised weights of that shape for tests and benchmarks (the trained
weights are not available here).
"""
from __future__ import annotations

import struct

import numpy as np

MAGIC = 0x41D7

# OIDN UNet (default size): encoder / decoder channel counts
EC1, EC2, EC3, EC4, EC5 = 32, 48, 64, 80, 96
DC4, DC3, DC2, DC1A, DC1B = 112, 96, 64, 64, 32


def unet_shapes(ic: int = 9, oc: int = 3) -> dict:
    """name -> (out_channels, in_channels) of every 3x3 convolution."""
    return {
        "enc_conv0": (EC1, ic), "enc_conv1": (EC1, EC1), "enc_conv2": (EC2, EC1),
        "enc_conv3": (EC3, EC2), "enc_conv4": (EC4, EC3), "enc_conv5a": (EC5, EC4),
        "enc_conv5b": (EC5, EC5), "dec_conv4a": (DC4, EC5 + EC3), "dec_conv4b": (DC4, DC4),
        "dec_conv3a": (DC3, DC4 + EC2), "dec_conv3b": (DC3, DC3), "dec_conv2a": (DC2, DC3 + EC1),
        "dec_conv2b": (DC2, DC2), "dec_conv1a": (DC1A, DC2 + ic), "dec_conv1b": (DC1B, DC1A),
        "dec_conv0": (oc, DC1B),
    }


def random_unet_weights(seed: int = 0, ic: int = 9, gain: float = 1.0, bias: float = 0.02) -> dict:
    """He-normal weights (std = gain * sqrt(2 / fan_in)) and small uniform biases, float32."""
    rng = np.random.default_rng(seed)
    w = {}
    for name, (o, i) in unet_shapes(ic).items():
        std = gain * np.sqrt(2.0 / (9 * i))
        w[name + ".weight"] = (rng.standard_normal((o, i, 3, 3)) * std).astype(np.float32)
        w[name + ".bias"] = rng.uniform(-bias, bias, o).astype(np.float32)
    return w


def write_tza(tensors: dict, dtype: str = "f") -> bytes:
    """Serialise {name: array} ('f' float32 or 'h' float16 payloads, 64-B aligned)."""
    if dtype not in ("f", "h"):
        raise ValueError("dtype must be 'f' or 'h'")
    npdt = np.float32 if dtype == "f" else np.float16
    data, table, off = bytearray(), [], 16
    for name, arr in tensors.items():
        a = np.ascontiguousarray(np.asarray(arr, dtype=npdt))
        pad = (-(off + len(data))) % 64
        data += b"\0" * pad
        table.append((name, a.shape, off + len(data)))
        data += a.tobytes()
    tab = bytearray(struct.pack("<I", len(table)))
    for name, shape, doff in table:
        nb = name.encode()
        layout = {4: "oihw", 1: "x"}.get(len(shape), "x" * len(shape))
        tab += struct.pack("<H", len(nb)) + nb + struct.pack("<B", len(shape))
        tab += struct.pack("<%dI" % len(shape), *shape) + layout.encode() + dtype.encode()
        tab += struct.pack("<Q", doff)
    table_off = 16 + len(data)
    return struct.pack("<HBBQ", MAGIC, 2, 0, table_off) + b"\0" * 4 + bytes(data) + bytes(tab)


def read_tza(blob: bytes) -> dict:
    """Parse a .tza into {name: float32 array}; raises ValueError on a malformed archive."""
    if len(blob) < 12:
        raise ValueError("tza: truncated header")
    magic, major, _minor, table_off = struct.unpack_from("<HBBQ", blob, 0)
    if magic != MAGIC:
        raise ValueError("tza: bad magic")
    if major != 2:
        raise ValueError("tza: unsupported version %d" % major)
    if table_off + 4 > len(blob):
        raise ValueError("tza: table offset out of range")
    (n,) = struct.unpack_from("<I", blob, table_off)
    p, out = table_off + 4, {}
    for _ in range(n):
        (ln,) = struct.unpack_from("<H", blob, p); p += 2
        name = blob[p:p + ln].decode(); p += ln
        (nd,) = struct.unpack_from("<B", blob, p); p += 1
        shape = struct.unpack_from("<%dI" % nd, blob, p); p += 4 * nd
        p += nd                                            # layout
        dt = chr(blob[p]); p += 1
        (doff,) = struct.unpack_from("<Q", blob, p); p += 8
        npdt = {"f": np.float32, "h": np.float16}.get(dt)
        if npdt is None:
            raise ValueError("tza: unsupported data type %r" % dt)
        cnt = int(np.prod(shape)) if nd else 1
        if doff + cnt * np.dtype(npdt).itemsize > len(blob):
            raise ValueError("tza: tensor %s out of range" % name)
        out[name] = np.frombuffer(blob, npdt, cnt, doff).reshape(shape).astype(np.float32)
    return out
