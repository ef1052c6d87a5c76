"""CPU study for a cheaper counter-RNG hash: avalanche bias of candidate 32-bit hashes, and the
correlation of the uniform draws of neighbouring pixels (key = hash of the pixel index) at equal slots.  The
product's hash (rs_device.h hash32 / oracle/restir_oracle.c) is lowbias32 (two 32-bit multiplies, quarter-rate
`v_mul_lo_u32` on gfx950); the candidates use only full-rate operations.  Prints one line per hash.
    python scripts/rng_quality.py [--n 200000]"""
import argparse

import numpy as np

M32 = np.uint64(0xFFFFFFFF)


def lowbias32(x):
    x = x.astype(np.uint64)
    x ^= x >> np.uint64(16); x = (x * np.uint64(0x7feb352d)) & M32
    x ^= x >> np.uint64(15); x = (x * np.uint64(0x846ca68b)) & M32
    x ^= x >> np.uint64(16)
    return x


def mul24(x, c):            # v_mul_u32_u24: low 32 bits of the 24 x 24-bit product
    return ((x & np.uint64(0xFFFFFF)) * np.uint64(c & 0xFFFFFF)) & M32


def hash24(x):              # two full-rate 24-bit multiplies, top bits folded down before each
    x = x.astype(np.uint64)
    x ^= x >> np.uint64(16); x = mul24(x, 0x7feb35) ^ (x >> np.uint64(24))
    x ^= x >> np.uint64(15); x = mul24(x, 0x846ca7) ^ (x >> np.uint64(24))
    x ^= x >> np.uint64(16)
    return x & M32


def wang(x):                # Thomas Wang's hash32shift (shifts and adds only; * 2057 = shift-add)
    x = x.astype(np.uint64)
    x = ((~x) + (x << np.uint64(15))) & M32
    x ^= x >> np.uint64(12)
    x = (x + (x << np.uint64(2))) & M32
    x ^= x >> np.uint64(4)
    x = (x * np.uint64(2057)) & M32
    x ^= x >> np.uint64(16)
    return x


def xorshift(x):            # the timing-only diagnostic (RS_DIAG_CHEAP_RNG): linear over GF(2)
    x = x.astype(np.uint64)
    x ^= (x << np.uint64(13)) & M32; x ^= x >> np.uint64(17); x ^= (x << np.uint64(5)) & M32; x ^= x >> np.uint64(16)
    return x


def avalanche_bias(h, n, rng):
    x = rng.integers(0, 2**32, size=n, dtype=np.uint64)
    hx = h(x)
    worst, tot = 0.0, 0.0
    for b in range(32):
        d = hx ^ h(x ^ np.uint64(1 << b))
        p = np.array([((d >> np.uint64(o)) & np.uint64(1)).mean() for o in range(32)])
        e = np.abs(p - 0.5)
        worst = max(worst, float(e.max())); tot += float(e.mean())
    return tot / 32, worst


def pixel_corr(h, n):
    # the product's draw: u = (hash(key ^ hash(slot + c)) >> 8) / 2^24, key = hash(... ^ pixel); neighbours p, p + 1
    key = h(h(np.arange(n, dtype=np.uint64) ^ np.uint64(0x1234567)) & M32)
    s = h(np.array([5 + 0x632be5ab], dtype=np.uint64) & M32)[0]
    u = (h(key ^ s) >> np.uint64(8)).astype(np.float64) / 2**24
    return float(np.corrcoef(u[:-1], u[1:])[0, 1]), float(abs(u.mean() - 0.5))


ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=200000)
a = ap.parse_args()
rng = np.random.default_rng(7)
for name, h in (("lowbias32 (product)", lowbias32), ("hash24 (2 x 24-bit mul)", hash24), ("wang hash32shift", wang),
                ("xorshift (diagnostic)", xorshift)):
    mb, wb = avalanche_bias(h, a.n, rng)
    c, m = pixel_corr(h, a.n)
    print(f"{name:26s} avalanche bias mean {mb:.4f} worst {wb:.4f}   neighbour-pixel corr {c:+.4f}  |mean-0.5| {m:.4f}",
          flush=True)
