"""Offline BVH quality model: node visits / triangle tests per ray for the GPU LBVH (Karras, leaves
<= 4, preorder skip layout) vs a binned-SAH tree, on the C2 scene's shadow rays.  Analysis tooling
only (not product, not test)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "restir-embree_amd"))
from restir_amd import scenes  # noqa: E402

LEAF_MAX = 4


def expand10(v):
    v = v.astype(np.uint64) & 0x3FF
    v = (v * 0x00010001) & 0xFF0000FF
    v = (v * 0x00000101) & 0x0F00F00F
    v = (v * 0x00000011) & 0xC30C30C3
    v = (v * 0x00000005) & 0x49249249
    return v


def lbvh(lo, hi):
    n = lo.shape[0]
    c = 0.5 * (lo + hi)
    cmin, cmax = c.min(0), c.max(0)
    ext = np.where(cmax - cmin > 0, cmax - cmin, 1)
    q = np.clip((((c - cmin) / ext) * 1024).astype(np.int64), 0, 1023)
    m = (expand10(q[:, 0]) << 2) | (expand10(q[:, 1]) << 1) | expand10(q[:, 2])
    keys = (m.astype(np.uint64) << np.uint64(32)) | np.arange(n, dtype=np.uint64)
    order = np.argsort(keys, kind="stable")
    keys = keys[order]

    def delta(i, j):
        if j < 0 or j >= n:
            return -1
        x = int(keys[i]) ^ int(keys[j])
        return 64 - x.bit_length()

    # node ids: internal 0..n-2, leaves n-1+j
    left = np.zeros(n - 1, np.int64)
    right = np.zeros(n - 1, np.int64)
    first = np.zeros(2 * n - 1, np.int64)
    last = np.zeros(2 * n - 1, np.int64)
    for j in range(n):
        first[n - 1 + j] = last[n - 1 + j] = j
    for i in range(n - 1):
        d = 1 if delta(i, i + 1) - delta(i, i - 1) >= 0 else -1
        dmin = delta(i, i - d)
        lmax = 2
        while delta(i, i + lmax * d) > dmin:
            lmax *= 2
        l = 0
        t = lmax // 2
        while t >= 1:
            if delta(i, i + (l + t) * d) > dmin:
                l += t
            t //= 2
        j = i + l * d
        dn = delta(i, j)
        s, t = 0, l
        while True:
            t = (t + 1) >> 1
            if delta(i, i + (s + t) * d) > dn:
                s += t
            if t <= 1:
                break
        g = i + s * d + min(d, 0)
        f, la = min(i, j), max(i, j)
        left[i] = (n - 1 + g) if f == g else g
        right[i] = (n - 1 + g + 1) if la == g + 1 else g + 1
        first[i], last[i] = f, la
    slo, shi = lo[order], hi[order]

    def build(node):
        if node >= n - 1 or last[node] - first[node] + 1 <= LEAF_MAX:
            a, b = first[node], last[node] + 1
            return ("leaf", slo[a:b].min(0), shi[a:b].max(0), list(range(a, b)))
        L, R = build(left[node]), build(right[node])
        return ("node", np.minimum(L[1], R[1]), np.maximum(L[2], R[2]), [L, R])
    return build(0), order


def sah_tree(lo, hi, idx=None):
    if idx is None:
        idx = np.arange(lo.shape[0])
    blo, bhi = lo[idx].min(0), hi[idx].max(0)
    if len(idx) <= LEAF_MAX:
        return ("leaf", blo, bhi, list(idx))
    c = 0.5 * (lo[idx] + hi[idx])
    best = None
    for ax in range(3):
        cl, ch = c[:, ax].min(), c[:, ax].max()
        if ch <= cl:
            continue
        nb = 16
        b = np.clip(((c[:, ax] - cl) / (ch - cl) * nb).astype(int), 0, nb - 1)
        for s in range(nb - 1):
            ml = b <= s
            if ml.all() or (~ml).all():
                continue

            def area(ii):
                e = hi[ii].max(0) - lo[ii].min(0)
                return 2 * (e[0] * e[1] + e[1] * e[2] + e[2] * e[0])
            cost = area(idx[ml]) * ml.sum() + area(idx[~ml]) * (~ml).sum()
            if best is None or cost < best[0]:
                best = (cost, ml)
    if best is None:
        h = len(idx) // 2
        ml = np.zeros(len(idx), bool)
        ml[:h] = True
    else:
        ml = best[1]
    L, R = sah_tree(lo, hi, idx[ml]), sah_tree(lo, hi, idx[~ml])
    return ("node", np.minimum(L[1], R[1]), np.maximum(L[2], R[2]), [L, R])


def flatten(tree):
    """preorder skip layout: list of (lo, hi, skip, tris or None)"""
    out = []

    def rec(t):
        i = len(out)
        out.append(None)
        if t[0] == "leaf":
            out[i] = (t[1], t[2], i + 1, t[3])
        else:
            rec(t[3][0])
            rec(t[3][1])
            out[i] = (t[1], t[2], len(out), None)
    rec(tree)
    lo = np.array([x[0] for x in out]); hi = np.array([x[1] for x in out])
    skip = np.array([x[2] for x in out]); leaf = [x[3] for x in out]
    return lo, hi, skip, leaf


def traverse_stats(flat, o, d, tfar):
    lo, hi, skip, leaf = flat
    n = len(skip)
    inv = 1.0 / np.where(d == 0, 1e-30, d)
    visits = np.zeros(o.shape[0], np.int64)
    tris = np.zeros(o.shape[0], np.int64)
    # vectorised over rays: per step each ray is at some node index
    i = np.zeros(o.shape[0], np.int64)
    active = np.ones(o.shape[0], bool)
    while active.any():
        a = np.flatnonzero(active)
        ni = i[a]
        t0 = (lo[ni] - o[a]) * inv[a]
        t1 = (hi[ni] - o[a]) * inv[a]
        tmin = np.maximum(np.minimum(t0, t1).max(1), 0.0)
        tmax = np.minimum(np.maximum(t0, t1).min(1), tfar[a])
        hit = tmin <= tmax
        visits[a] += 1
        is_leaf = np.array([leaf[k] is not None for k in ni])
        nl = np.array([len(leaf[k]) if leaf[k] is not None else 0 for k in ni])
        tris[a] += np.where(hit & is_leaf, nl, 0)
        nxt = np.where(hit & ~is_leaf, ni + 1, skip[ni])
        i[a] = nxt
        active[a] = nxt < n
    return visits, tris


def main():
    sc = scenes.cornell_many_lights(1024)
    P = sc.positions.reshape(-1, 3, 3)
    lo, hi = P.min(1), P.max(1)
    rng = np.random.default_rng(0)
    # shadow rays: from random floor/wall points to random points on random emissive triangles (segment)
    em = np.flatnonzero(sc.emissive_mask())
    nr = 4000
    org = np.stack([rng.uniform(-0.95, 0.95, nr), rng.uniform(-0.95, 0.95, nr), np.full(nr, 0.0)], 1)
    tri = P[rng.choice(em, nr)]
    r1, r2 = rng.random(nr), rng.random(nr)
    sr = np.sqrt(r1)
    tgt = tri[:, 0] * (1 - sr)[:, None] + tri[:, 1] * (sr * (1 - r2))[:, None] + tri[:, 2] * (sr * r2)[:, None]
    d = tgt - org
    dist = np.linalg.norm(d, axis=1)
    d /= dist[:, None]
    for name, tree in (("LBVH", lbvh(lo, hi)[0]), ("SAH", sah_tree(lo, hi))):
        flat = flatten(tree)
        v, t = traverse_stats(flat, org, d, dist - 0.001)
        print(f"{name}: nodes={len(flat[2])} visits/ray mean={v.mean():.1f} p90={np.percentile(v, 90):.0f} "
              f"tri tests/ray={t.mean():.1f}")


if __name__ == "__main__":
    main()


def ploc(lo, hi, radius=16):
    """PLOC (Meister & Bittner 2018) on Morton-ordered clusters; tie rule: smaller index."""
    n = lo.shape[0]
    c = 0.5 * (lo + hi)
    cmin, cmax = c.min(0), c.max(0)
    ext = np.where(cmax - cmin > 0, cmax - cmin, 1)
    q = np.clip((((c - cmin) / ext) * 1024).astype(np.int64), 0, 1023)
    m = (expand10(q[:, 0]) << 2) | (expand10(q[:, 1]) << 1) | expand10(q[:, 2])
    keys = (m.astype(np.uint64) << np.uint64(32)) | np.arange(n, dtype=np.uint64)
    order = np.argsort(keys, kind="stable")
    nodes = [("leaf", lo[k], hi[k], [int(k)]) for k in order]
    C = list(range(n))
    while len(C) > 1:
        k = len(C)
        blo = np.array([nodes[x][1] for x in C]); bhi = np.array([nodes[x][2] for x in C])
        N = np.zeros(k, np.int64)
        for i in range(k):
            a, b = max(0, i - radius), min(k, i + radius + 1)
            js = np.array([j for j in range(a, b) if j != i])
            e = np.maximum(bhi[js], bhi[i]) - np.minimum(blo[js], blo[i])
            area = e[:, 0] * e[:, 1] + e[:, 1] * e[:, 2] + e[:, 2] * e[:, 0]
            N[i] = js[np.argmin(area)]
        newC = []
        for i in range(k):
            j = N[i]
            if N[j] == i:
                if i < j:
                    L, R = nodes[C[i]], nodes[C[j]]
                    nodes.append(("node", np.minimum(L[1], R[1]), np.maximum(L[2], R[2]), [L, R]))
                    newC.append(len(nodes) - 1)
            else:
                newC.append(C[i])
        C = newC
    return nodes[C[0]]


def collapse(t, max_leaf=LEAF_MAX, c_trav=1.0, c_tri=1.0):
    """SAH collapse: returns (tree, cost, prims)."""
    def area(lo_, hi_):
        e = hi_ - lo_
        return 2 * (e[0] * e[1] + e[1] * e[2] + e[2] * e[0])
    if t[0] == "leaf":
        return t, c_tri * len(t[3]), t[3]
    L, cl, pl = collapse(t[3][0], max_leaf, c_trav, c_tri)
    R, cr, pr = collapse(t[3][1], max_leaf, c_trav, c_tri)
    A = max(area(t[1], t[2]), 1e-30)
    split = c_trav + (area(L[1], L[2]) * cl + area(R[1], R[2]) * cr) / A
    prims = pl + pr
    if len(prims) <= max_leaf and c_tri * len(prims) <= split:
        return ("leaf", t[1], t[2], prims), c_tri * len(prims), prims
    return ("node", t[1], t[2], [L, R]), split, prims


if __name__ == "__main__":
    sc = scenes.cornell_many_lights(1024)
    P = sc.positions.reshape(-1, 3, 3)
    lo, hi = P.min(1), P.max(1)
    rng = np.random.default_rng(0)
    em = np.flatnonzero(sc.emissive_mask())
    nr = 4000
    org = np.stack([rng.uniform(-0.95, 0.95, nr), rng.uniform(-0.95, 0.95, nr), np.full(nr, 0.0)], 1)
    tri = P[rng.choice(em, nr)]
    r1, r2 = rng.random(nr), rng.random(nr)
    sr = np.sqrt(r1)
    tgt = tri[:, 0] * (1 - sr)[:, None] + tri[:, 1] * (sr * (1 - r2))[:, None] + tri[:, 2] * (sr * r2)[:, None]
    d = tgt - org
    dist = np.linalg.norm(d, axis=1)
    d /= dist[:, None]
    for r in (8, 16):
        t = ploc(lo, hi, r)
        for ml in (1, 4, 8):
            flat = flatten(collapse(t, ml)[0])
            v, tt = traverse_stats(flat, org, d, dist - 0.001)
            print(f"PLOC r={r} leaf<={ml}: nodes={len(flat[2])} visits/ray={v.mean():.1f} p90={np.percentile(v, 90):.0f} tri tests={tt.mean():.1f}")
