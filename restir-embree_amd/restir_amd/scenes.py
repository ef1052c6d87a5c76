"""Synthetic scenes for the ReSTIR DI hot path (BASELINE.json configs C1-C5).

The reference ships no geometry (``*.obj`` is git-ignored), so every scene here
is procedural.  The layout mirrors what the reference's loader hands Embree
(pg/ModelLoader.cpp:218-321): de-indexed triangles (3 unique vertices per triangle,
``:297-299``), per-vertex normals (attribute slot 0, ``:280-282``) and one material per mesh
(``:213``) -- flattened here to one material index per triangle.  Emissive triangles are
those whose material has ``Ke.x+Ke.y+Ke.z > 0`` (pg/material.h:135-137); their order in the
triangle array is the emissive-id order (``triIdCtr``, pg/ModelLoader.cpp:291-305).

Materials are given in linear RGB (the loader's sRGB expansion of Kd/Ks, pg/ModelLoader.cpp:
80-97, is already applied).  The reference is Z-up (pg/camera.h:68).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

# pg/enums.h:3-11
NORMAL, LAMBERT, PHONG, MIRROR, DIELECTRIC, DIELECTRIC_TRANSPARENT, UNSUPPORTED = range(7)


@dataclass
class Material:
    kd: tuple = (0.0, 0.0, 0.0)
    ks: tuple = (0.0, 0.0, 0.0)
    le: tuple = (0.0, 0.0, 0.0)
    shininess: float = 1.0
    type: int = LAMBERT
    # texture slots (pg/material.cpp:105-134, pg/Intersection.h:26-39): 1-based index into Scene.textures
    diffuse_map: int = 0
    specular_map: int = 0
    shininess_map: int = 0
    normal_map: int = 0


@dataclass
class Texture:
    """Decoded texture (include/restir_c.h rs_texture_desc): (H, W, C) uint8 (texel = byte/255) or
    float32, top row first, C in {1, 3, 4} (float: 3 or 4).  srgb_expand: Texture::expand at load for
    colour maps (the OBJ loader sets it for map_Kd / map_Ks)."""
    data: np.ndarray
    srgb_expand: int = 0


@dataclass
class Camera:
    """Camera(eye, at, fov_y_deg) as built by tutorial_3 (pg/tutorials.cpp:35)."""
    eye: tuple
    at: tuple
    fov_y: float

    def as_array(self) -> np.ndarray:
        return np.array([*self.eye, *self.at, self.fov_y], dtype=np.float32)


@dataclass
class Scene:
    positions: np.ndarray        # (T, 9) float32, v0 v1 v2
    normals: np.ndarray          # (T, 9) float32, n0 n1 n2
    tri_material: np.ndarray     # (T,) uint32
    materials: list = field(default_factory=list)
    camera: Camera | None = None
    name: str = ""
    texcoords: np.ndarray | None = None   # (T, 6) float32 uv per vertex (attribute slot 1)
    tangents: np.ndarray | None = None    # (T, 9) float32 (attribute slot 3; normal maps)
    textures: list = field(default_factory=list)
    sky: Texture | None = None            # equirect sky (useSkybox)

    @property
    def n_tris(self) -> int:
        return int(self.positions.shape[0])

    def material_arrays(self):
        """(M,10) float32 [kd3 ks3 le3 shininess] and (M,) int32 type."""
        f = np.zeros((len(self.materials), 10), dtype=np.float32)
        t = np.zeros((len(self.materials),), dtype=np.int32)
        for i, m in enumerate(self.materials):
            f[i, 0:3] = m.kd
            f[i, 3:6] = m.ks
            f[i, 6:9] = m.le
            f[i, 9] = m.shininess
            t[i] = m.type
        return f, t

    def emissive_mask(self) -> np.ndarray:
        f, _ = self.material_arrays()
        le_sum = f[:, 6] + f[:, 7] + f[:, 8]
        return (le_sum > 0)[self.tri_material]


class _Builder:
    def __init__(self):
        self.pos: list[np.ndarray] = []
        self.nrm: list[np.ndarray] = []
        self.mat: list[np.ndarray] = []
        self.materials: list[Material] = []

    def material(self, m: Material) -> int:
        self.materials.append(m)
        return len(self.materials) - 1

    def tris(self, p: np.ndarray, n: np.ndarray, mat: int):
        p = np.asarray(p, dtype=np.float32).reshape(-1, 9)
        n = np.asarray(n, dtype=np.float32).reshape(-1, 9)
        self.pos.append(p)
        self.nrm.append(n)
        self.mat.append(np.full((p.shape[0],), mat, dtype=np.uint32))

    def quad(self, a, b, c, d, mat: int, normal=None):
        """Quad a-b-c-d (counter-clockwise seen from the normal side) as two triangles."""
        a, b, c, d = (np.asarray(v, dtype=np.float32) for v in (a, b, c, d))
        if normal is None:
            nn = np.cross(b - a, c - a)
            normal = nn / np.linalg.norm(nn)
        normal = np.asarray(normal, dtype=np.float32)
        p = np.stack([np.concatenate([a, b, c]), np.concatenate([a, c, d])])
        n = np.tile(normal, 6).reshape(2, 9)
        self.tris(p, n, mat)

    def quads(self, corners: np.ndarray, normals: np.ndarray, mat: int):
        """Vectorised quads: corners (Q,4,3) CCW, normals (Q,3)."""
        c = np.asarray(corners, dtype=np.float32)
        t0 = np.concatenate([c[:, 0], c[:, 1], c[:, 2]], axis=1)
        t1 = np.concatenate([c[:, 0], c[:, 2], c[:, 3]], axis=1)
        p = np.stack([t0, t1], axis=1).reshape(-1, 9)
        n = np.repeat(np.tile(np.asarray(normals, dtype=np.float32), (1, 3)), 2, axis=0)
        self.tris(p, n, mat)

    def box(self, lo, hi, mat: int, rot_z: float = 0.0, open_faces=()):
        lo = np.asarray(lo, dtype=np.float32)
        hi = np.asarray(hi, dtype=np.float32)
        c = 0.5 * (lo + hi)
        cs, sn = np.cos(rot_z), np.sin(rot_z)

        def R(v):
            v = np.asarray(v, dtype=np.float64) - c
            return np.array([cs * v[0] - sn * v[1] + c[0], sn * v[0] + cs * v[1] + c[1], v[2] + c[2]],
                            dtype=np.float32)

        def Rn(v):
            return np.array([cs * v[0] - sn * v[1], sn * v[0] + cs * v[1], v[2]], dtype=np.float32)

        x0, y0, z0 = lo
        x1, y1, z1 = hi
        faces = {
            "top": ([x0, y0, z1], [x1, y0, z1], [x1, y1, z1], [x0, y1, z1], [0, 0, 1]),
            "bottom": ([x0, y0, z0], [x0, y1, z0], [x1, y1, z0], [x1, y0, z0], [0, 0, -1]),
            "front": ([x0, y0, z0], [x1, y0, z0], [x1, y0, z1], [x0, y0, z1], [0, -1, 0]),
            "back": ([x1, y1, z0], [x0, y1, z0], [x0, y1, z1], [x1, y1, z1], [0, 1, 0]),
            "left": ([x0, y1, z0], [x0, y0, z0], [x0, y0, z1], [x0, y1, z1], [-1, 0, 0]),
            "right": ([x1, y0, z0], [x1, y1, z0], [x1, y1, z1], [x1, y0, z1], [1, 0, 0]),
        }
        for name, (a, b, cc, d, n) in faces.items():
            if name in open_faces:
                continue
            self.quad(R(a), R(b), R(cc), R(d), mat, normal=Rn(n))

    def build(self, camera: Camera, name: str) -> Scene:
        return Scene(positions=np.ascontiguousarray(np.concatenate(self.pos)),
                     normals=np.ascontiguousarray(np.concatenate(self.nrm)),
                     tri_material=np.ascontiguousarray(np.concatenate(self.mat)),
                     materials=list(self.materials), camera=camera, name=name)


def _cornell_shell(b: _Builder):
    """Box [-1,1]x[-1,1]x[0,2], open at y=-1 (the camera side); normals face inward."""
    white = b.material(Material(kd=(0.73, 0.73, 0.73), type=LAMBERT, shininess=1.0))
    red = b.material(Material(kd=(0.65, 0.05, 0.05), type=LAMBERT, shininess=1.0))
    green = b.material(Material(kd=(0.12, 0.45, 0.15), type=LAMBERT, shininess=1.0))
    glossy = b.material(Material(kd=(0.55, 0.55, 0.55), ks=(0.04, 0.04, 0.04), shininess=64.0, type=PHONG))
    b.quad([-1, -1, 0], [1, -1, 0], [1, 1, 0], [-1, 1, 0], white, normal=[0, 0, 1])       # floor
    b.quad([-1, -1, 2], [-1, 1, 2], [1, 1, 2], [1, -1, 2], white, normal=[0, 0, -1])      # ceiling
    b.quad([-1, 1, 0], [1, 1, 0], [1, 1, 2], [-1, 1, 2], white, normal=[0, -1, 0])        # back
    b.quad([-1, -1, 0], [-1, 1, 0], [-1, 1, 2], [-1, -1, 2], red, normal=[1, 0, 0])       # left
    b.quad([1, 1, 0], [1, -1, 0], [1, -1, 2], [1, 1, 2], green, normal=[-1, 0, 0])        # right
    b.box([-0.65, 0.0, 0.0], [-0.05, 0.6, 1.2], glossy, rot_z=0.3)                        # tall block
    b.box([0.05, -0.55, 0.0], [0.65, 0.05, 0.6], white, rot_z=-0.3)                       # short block


CORNELL_CAMERA = Camera(eye=(0.0, -3.9, 1.0), at=(0.0, 0.0, 1.0), fov_y=40.0)


def cornell_box(n_lights: int = 8) -> Scene:
    """C1: Cornell box with ``n_lights`` ceiling quads (2 tris each), Le = (17, 12, 4)."""
    b = _Builder()
    _cornell_shell(b)
    light = b.material(Material(le=(17.0, 12.0, 4.0), type=LAMBERT))
    side = int(np.ceil(np.sqrt(n_lights)))
    size = 0.18
    k = 0
    corners, normals = [], []
    for i in range(side):
        for j in range(side):
            if k >= n_lights:
                break
            cx = -0.45 + 0.9 * (i + 0.5) / side
            cy = -0.45 + 0.9 * (j + 0.5) / side
            z = 1.98
            h = size / 2
            corners.append([[cx - h, cy - h, z], [cx - h, cy + h, z], [cx + h, cy + h, z], [cx + h, cy - h, z]])
            normals.append([0, 0, -1])
            k += 1
    b.quads(np.array(corners), np.array(normals), light)
    return b.build(CORNELL_CAMERA, f"cornell_{n_lights}")


def textured_cornell(n_lights: int = 8, seed: int = 5, sky: bool = True) -> Scene:
    """§8f-2 test scene: C1 with material textures and an equirect sky (synthetic texels, seeded).
    Exercises every texture path of the reference: 8-bit RGB and RGBA diffuse maps (sRGB-expanded; the
    RGB map is shared by two materials, so it is expanded twice -- ModelLoader's TextureProxy quirk), a
    1-channel roughness map (the 3-byte read quirk, Ns = 2/r^2 - 2), a specular map, a normal map with
    tangents, planar uvs spanning negative values (REPEAT's abs(x % w)), a float RGB sky seen through the
    open front of the box."""
    sc = cornell_box(n_lights)
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:48, 0:64]
    checker = np.where(((xx // 8) + (yy // 8)) % 2 == 0, 220, 60).astype(np.uint8)
    checker = np.stack([checker, (xx * 4).astype(np.uint8), (255 - yy * 5).astype(np.uint8)], -1)
    rgba = rng.integers(0, 256, size=(32, 32, 4), dtype=np.uint8)
    rough = rng.integers(40, 200, size=(16, 24), dtype=np.uint8)[:, :, None]
    spec = rng.integers(0, 40, size=(20, 20, 3), dtype=np.uint8)
    ny, nx = np.mgrid[0:32, 0:32] / 32.0
    n = np.stack([0.3 * np.sin(6.28 * nx), 0.3 * np.cos(6.28 * ny), np.ones_like(nx)], -1)
    n /= np.linalg.norm(n, axis=-1, keepdims=True)
    nmap = np.clip((n * 0.5 + 0.5) * 255.0, 0, 255).astype(np.uint8)
    sc.textures = [Texture(checker, 1), Texture(rgba, 1), Texture(rough, 0), Texture(nmap, 0), Texture(spec, 1)]
    mats = [Material(**vars(m)) for m in sc.materials]
    mats[0].diffuse_map, mats[0].normal_map = 1, 4          # white: checker + normal map
    mats[1].diffuse_map = 2                                  # red: RGBA
    mats[2].diffuse_map = 1                                  # green: the checker again (expanded twice)
    mats[3].specular_map, mats[3].shininess_map = 5, 3      # glossy Phong block
    sc.materials = mats
    P = sc.positions.reshape(-1, 3, 3).astype(np.float64)
    u = 0.7 * (P[..., 0] + P[..., 1]) + 0.13
    v = 0.6 * P[..., 2] - 0.4
    sc.texcoords = np.stack([u, v], -1).reshape(-1, 6).astype(np.float32)
    t = np.tile(np.array([1.0, 1.0, 0.2]), (P.shape[0], 3, 1)) + rng.normal(0, 0.05, size=(P.shape[0], 3, 3))
    t /= np.linalg.norm(t, axis=-1, keepdims=True)
    sc.tangents = t.reshape(-1, 9).astype(np.float32)
    if sky:
        sy, sx = np.mgrid[0:16, 0:32]
        sc.sky = Texture(np.stack([0.2 + sx / 32.0, 0.5 + 0.5 * np.sin(sy / 3.0), 1.5 - sy / 16.0], -1).astype(np.float32))
    sc.name = f"textured_cornell_{n_lights}"
    return sc


def cornell_many_lights(n_lights: int = 1024, seed: int = 7, size: float = 0.02) -> Scene:
    """C2: Cornell box with ``n_lights`` emissive quads of ``size`` x ``size`` m (2*n_lights emissive
    triangles; SURVEY.md §8(d): 0.02 m quads).

    The reference has no point lights, so "1024 point lights" is encoded
    as 1024 small emissive quads: all but 16 placed uniformly on the ceiling (facing down), 16 on
    a 4x4 grid on the back wall (facing the camera).  Le ~ U[1,20]^3 with ``seed``; each light has
    its own material so its emission differs.
    """
    b = _Builder()
    _cornell_shell(b)
    rng = np.random.default_rng(seed)
    n_wall = min(16, n_lights)
    n_ceil = n_lights - n_wall
    le = rng.uniform(1.0, 20.0, size=(n_lights, 3)).astype(np.float32)
    h = size / 2
    xy = rng.uniform(-0.95 + h, 0.95 - h, size=(n_ceil, 2)).astype(np.float32)
    k = 0
    for i in range(n_ceil):
        cx, cy = float(xy[i, 0]), float(xy[i, 1])
        z = 1.985
        m = b.material(Material(le=tuple(float(v) for v in le[k]), type=LAMBERT))
        b.quad([cx - h, cy - h, z], [cx - h, cy + h, z], [cx + h, cy + h, z], [cx + h, cy - h, z], m, normal=[0, 0, -1])
        k += 1
    for i in range(n_wall):
        gx, gz = i % 4, i // 4
        cx = -0.6 + 1.2 * gx / 3.0
        cz = 0.6 + 1.0 * gz / 3.0
        y = 0.985
        m = b.material(Material(le=tuple(float(v) for v in le[k]), type=LAMBERT))
        b.quad([cx + h, y, cz - h], [cx - h, y, cz - h], [cx - h, y, cz + h], [cx + h, y, cz + h], m, normal=[0, -1, 0])
        k += 1
    return b.build(CORNELL_CAMERA, f"cornell_many_{n_lights}")


def sponza_like(target_tris: int = 250_000, n_lamps: int = 2048, seed: int = 11) -> Scene:
    """C3: procedural "Sponza-like" atrium with ~``target_tris`` triangles and 2*``n_lamps``
    emissive triangles (small lamp quads).  Phong materials with Ns in [8, 128], closed roof."""
    rng = np.random.default_rng(seed)
    b = _Builder()
    mats = []
    for _ in range(8):
        kd = tuple(float(v) for v in rng.uniform(0.2, 0.75, 3))
        ks = tuple(float(v) for v in rng.uniform(0.02, 0.2, 3))
        mats.append(b.material(Material(kd=kd, ks=ks, shininess=float(rng.uniform(8.0, 128.0)), type=PHONG)))
    L, Wd, Hh = 14.0, 6.0, 8.0   # atrium x in [-L, L], y in [-Wd, Wd], z in [0, Hh]
    # hall shell, subdivided so the floor/walls/roof carry a realistic triangle count
    def grid_quad(o, u, v, nu, nv, normal, mat):
        o, u, v = (np.asarray(a, dtype=np.float32) for a in (o, u, v))
        i, j = np.meshgrid(np.arange(nu), np.arange(nv), indexing="ij")
        i = i.reshape(-1, 1).astype(np.float32)
        j = j.reshape(-1, 1).astype(np.float32)
        a = o + (i / nu) * u + (j / nv) * v
        bb = o + ((i + 1) / nu) * u + (j / nv) * v
        c = o + ((i + 1) / nu) * u + ((j + 1) / nv) * v
        d = o + (i / nu) * u + ((j + 1) / nv) * v
        corners = np.stack([a, bb, c, d], axis=1)
        b.quads(corners, np.tile(np.asarray(normal, dtype=np.float32), (corners.shape[0], 1)), mat)

    grid_quad([-L, -Wd, 0], [2 * L, 0, 0], [0, 2 * Wd, 0], 96, 40, [0, 0, 1], mats[0])          # floor
    grid_quad([-L, Wd, Hh], [2 * L, 0, 0], [0, -2 * Wd, 0], 96, 40, [0, 0, -1], mats[1])        # roof
    grid_quad([-L, Wd, 0], [2 * L, 0, 0], [0, 0, Hh], 96, 24, [0, -1, 0], mats[2])              # +y wall
    grid_quad([L, -Wd, 0], [-2 * L, 0, 0], [0, 0, Hh], 96, 24, [0, 1, 0], mats[2])              # -y wall
    grid_quad([-L, -Wd, 0], [0, 2 * Wd, 0], [0, 0, Hh], 40, 24, [1, 0, 0], mats[3])             # -x wall
    grid_quad([L, Wd, 0], [0, -2 * Wd, 0], [0, 0, Hh], 40, 24, [-1, 0, 0], mats[3])             # +x wall

    def cylinder(cx, cy, z0, z1, r, seg, rings, mat):
        th = np.linspace(0, 2 * np.pi, seg + 1, dtype=np.float64)
        zs = np.linspace(z0, z1, rings + 1, dtype=np.float64)
        t0, t1 = th[:-1], th[1:]
        corners, normals = [], []
        for k in range(rings):
            za, zb = zs[k], zs[k + 1]
            a = np.stack([cx + r * np.cos(t0), cy + r * np.sin(t0), np.full_like(t0, za)], 1)
            bq = np.stack([cx + r * np.cos(t1), cy + r * np.sin(t1), np.full_like(t0, za)], 1)
            c = np.stack([cx + r * np.cos(t1), cy + r * np.sin(t1), np.full_like(t0, zb)], 1)
            d = np.stack([cx + r * np.cos(t0), cy + r * np.sin(t0), np.full_like(t0, zb)], 1)
            corners.append(np.stack([a, bq, c, d], 1))
            tm = 0.5 * (t0 + t1)
            normals.append(np.stack([np.cos(tm), np.sin(tm), np.zeros_like(tm)], 1))
        b.quads(np.concatenate(corners), np.concatenate(normals), mat)

    # two colonnades x two storeys of columns
    xs = np.linspace(-L + 1.5, L - 1.5, 12)
    for y in (-Wd + 1.8, Wd - 1.8):
        for x in xs:
            cylinder(x, y, 0.0, 3.8, 0.35, 32, 24, mats[4])
            cylinder(x, y, 4.2, 7.6, 0.25, 24, 16, mats[5])
    # arches: half-tori between neighbouring columns
    def arch(x0, x1, y, zbase, r_tube, seg, tube_seg, mat):
        R = 0.5 * (x1 - x0)
        cx = 0.5 * (x0 + x1)
        u = np.linspace(0, np.pi, seg + 1)
        v = np.linspace(0, 2 * np.pi, tube_seg + 1)
        corners, normals = [], []
        for i in range(seg):
            for j in range(tube_seg):
                pts = []
                for (uu, vv) in ((u[i], v[j]), (u[i + 1], v[j]), (u[i + 1], v[j + 1]), (u[i], v[j + 1])):
                    cxu = cx + R * np.cos(uu)
                    czu = zbase + R * np.sin(uu)
                    nx, nz = np.cos(uu), np.sin(uu)
                    pts.append([cxu + r_tube * np.cos(vv) * nx, y + r_tube * np.sin(vv), czu + r_tube * np.cos(vv) * nz])
                corners.append(pts)
                um, vm = 0.5 * (u[i] + u[i + 1]), 0.5 * (v[j] + v[j + 1])
                normals.append([np.cos(vm) * np.cos(um), np.sin(vm), np.cos(vm) * np.sin(um)])
        b.quads(np.array(corners), np.array(normals), mat)

    for y in (-Wd + 1.8, Wd - 1.8):
        for k in range(len(xs) - 1):
            arch(xs[k], xs[k + 1], y, 3.8, 0.18, 24, 12, mats[6])
    # drapes: wavy subdivided sheets hanging between upper columns
    cur = sum(p.shape[0] for p in b.pos)
    remaining = max(0, target_tris - cur - 2 * n_lamps)
    n_drapes = 2 * (len(xs) - 1)
    per = max(2, remaining // max(1, n_drapes))
    nu = max(4, int(np.sqrt(per / 2 * 2.0)))
    nv = max(2, per // (2 * nu))
    for side, y in enumerate((-Wd + 2.3, Wd - 2.3)):
        for k in range(len(xs) - 1):
            x0, x1 = xs[k] + 0.3, xs[k + 1] - 0.3
            i, j = np.meshgrid(np.arange(nu + 1), np.arange(nv + 1), indexing="ij")
            px = x0 + (x1 - x0) * i / nu
            pz = 7.0 - 2.6 * j / nv
            py = y + 0.15 * np.sin(2 * np.pi * 3 * i / nu) * (j / nv) * (1 if side == 0 else -1)
            P = np.stack([px, py, pz], -1)
            a, bq, c, d = P[:-1, :-1], P[1:, :-1], P[1:, 1:], P[:-1, 1:]
            corners = np.stack([a, bq, c, d], 2).reshape(-1, 4, 3)
            nn = np.cross(corners[:, 1] - corners[:, 0], corners[:, 3] - corners[:, 0])
            nn /= np.linalg.norm(nn, axis=1, keepdims=True)
            b.quads(corners, nn, mats[7])
    # lamps: small emissive quads facing down, hung in a grid under the roof and along the walls
    le = rng.uniform(5.0, 50.0, size=(n_lamps, 3))
    lx = rng.uniform(-L + 0.5, L - 0.5, n_lamps)
    ly = rng.uniform(-Wd + 0.5, Wd - 0.5, n_lamps)
    lz = rng.uniform(5.0, 7.8, n_lamps)
    h = 0.04
    for k in range(n_lamps):
        m = b.material(Material(le=tuple(float(v) for v in le[k]), type=LAMBERT))
        x, y, z = float(lx[k]), float(ly[k]), float(lz[k])
        b.quad([x - h, y - h, z], [x - h, y + h, z], [x + h, y + h, z], [x + h, y - h, z], m, normal=[0, 0, -1])
    cam = Camera(eye=(-L + 1.0, -0.5, 1.7), at=(L - 2.0, 0.6, 3.2), fov_y=66.0)
    return b.build(cam, f"sponza_like_{target_tris}")


def orbit_camera(base: Camera, frame: int, n_frames: int = 240, radius: float = 0.3) -> Camera:
    """C5: eye on a circle of ``radius`` around the base eye, looking at the base target."""
    a = 2.0 * np.pi * frame / n_frames
    ex = base.eye[0] + radius * np.cos(a)
    ey = base.eye[1]
    ez = base.eye[2] + radius * np.sin(a)
    return Camera(eye=(float(ex), float(ey), float(ez)), at=base.at, fov_y=base.fov_y)


def by_name(name: str) -> Scene:
    if name in ("C1", "cornell"):
        return cornell_box(8)
    if name in ("C2", "cornell_many"):
        return cornell_many_lights(1024)
    if name in ("C3", "sponza"):
        return sponza_like()
    raise KeyError(name)


def moving_light_positions(scene: Scene, frame: int, n_frames: int = 240, amplitude: float = 0.05) -> np.ndarray:
    """C5 "moving lights" (a build extension -- the reference cannot move geometry): every emissive quad
    (two consecutive emissive triangles) slides along its own plane, offset = amplitude *
    sin(2 pi frame / n_frames + phase_q) along the quad's first edge, phase_q = 2 pi frac(q * 0.618034).
    Returns the full (T, 9) float32 position array for Scene.update_positions / the oracle."""
    pos = np.array(scene.positions, dtype=np.float32, copy=True)
    emis = np.nonzero(scene.emissive_mask())[0]
    quads = emis.reshape(-1, 2) if emis.size % 2 == 0 else emis.reshape(-1, 1)
    v = pos[quads[:, 0]].reshape(-1, 3, 3).astype(np.float64)
    tangent = v[:, 1] - v[:, 0]
    tangent /= np.maximum(np.linalg.norm(tangent, axis=1, keepdims=True), 1e-12)
    q = np.arange(quads.shape[0], dtype=np.float64)
    phase = 2.0 * np.pi * np.modf(q * 0.618034)[0]
    off = amplitude * np.sin(2.0 * np.pi * frame / n_frames + phase)[:, None] * tangent      # (Q, 3)
    for j in range(quads.shape[1]):
        t = quads[:, j]
        pos[t] = (pos[t].reshape(-1, 3, 3) + off[:, None, :]).reshape(-1, 9).astype(np.float32)
    return pos


def write_obj(scene: Scene, obj_path: str) -> None:
    """Write ``scene`` as OBJ + MTL (``<obj>.mtl`` beside it) for rs_scene_load_obj / Raytracer::LoadScene.
    Kd / Ks are written sRGB-compressed so the loader's expansion (pg/ModelLoader.cpp:80-97) recovers the
    linear values; Ke, Ns and the material class (Pc) as they are; per-vertex normals; triangles in the
    scene's order (one usemtl run per material change)."""
    import os

    def comp(v):
        v = float(np.float32(v))
        return 0.0 if v <= 0 else (v * 12.92 if v <= 0.0031308 else 1.055 * v ** (1 / 2.4) - 0.055)

    mtl = os.path.splitext(obj_path)[0] + ".mtl"
    with open(mtl, "w") as f:
        for i, m in enumerate(scene.materials):
            f.write(f"newmtl m{i}\nPc {m.type}\nKd {' '.join(f'{comp(c):.9g}' for c in m.kd)}\n"
                    f"Ks {' '.join(f'{comp(c):.9g}' for c in m.ks)}\nKe {' '.join(f'{c:.9g}' for c in m.le)}\n"
                    f"Ns {m.shininess:.9g}\n")
    P = np.asarray(scene.positions, np.float32).reshape(-1, 3)
    N = np.asarray(scene.normals, np.float32).reshape(-1, 3)
    with open(obj_path, "w") as f:
        f.write(f"mtllib {os.path.basename(mtl)}\n")
        f.write("".join(f"v {x:.9g} {y:.9g} {z:.9g}\n" for x, y, z in P))
        f.write("".join(f"vn {x:.9g} {y:.9g} {z:.9g}\n" for x, y, z in N))
        cur = -1
        lines = []
        for t in range(scene.n_tris):
            if scene.tri_material[t] != cur:
                cur = int(scene.tri_material[t])
                lines.append(f"usemtl m{cur}\n")
            b = 3 * t + 1
            lines.append(f"f {b}//{b} {b + 1}//{b + 1} {b + 2}//{b + 2}\n")
        f.write("".join(lines))
