"""Sponza-proxy MESH (configs C2/C3/C5): a procedural atrium of ~262k triangles textured with the
reference's own Sponza JPEGs, rasterised by the HIP rasteriser (and the oracle) like any glTF scene.

The reference's Sponza.bin (geometry) is missing from its mount; its Sponza.gltf is present and gives, per
primitive, the material, the vertex / index counts and the POSITION bounds. This generator keeps what those
give: the layout of Sponza's atrium at the app's 0.01 scale (application.cpp:16; the node's 0.008 scale is
ignored, quirk Q4) -- a two-storey colonnade around an open court, galleries, a roof frame, hanging fabrics,
vases with plants, lamps -- the 25 materials with their baseColor / normal textures, and each material's
triangle count from the glTF (the budgets below sum to 262,267). Shapes are parametric surfaces (fluted
column shafts, arch bands, displaced cloth, lathed vases, leaf cards, tiled panels) wound counter-clockwise
seen from outside, like glTF, with planar / cylindrical uvs in world metres.

Deterministic (seed 0x5050). No file of the reference is read at run time: the textures come from the committed
256^2 fixture soc_real_time_renderer_amd/data/sponza/ or from the native-resolution set data/sponza_native/ (the
reference's 1024^2 image files, copied by __graft_entry__.build() in the container that has the reference; git-ignored,
shipped to the GPU box with the built libraries); tools/make_sponza_fixture.py makes both.
"""
from __future__ import annotations

import json
import math
import os
from typing import Dict, List, Optional

import numpy as np

DATA = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "data", "sponza")
NATIVE = os.path.join(os.path.dirname(DATA), "sponza_native")
SEED = 0x5050

# Sponza.gltf: triangles per material (sum over its primitives of indices.count / 3)
GLTF_TRIANGLES = {0: 31436, 1: 17688, 2: 18, 3: 3472, 4: 4086, 5: 796, 6: 10168, 7: 5876, 8: 2816, 9: 21, 10: 7088,
                  11: 880, 12: 23208, 13: 16496, 14: 16512, 15: 16512, 16: 11008, 17: 14336, 18: 18944, 19: 14336,
                  20: 32, 21: 19828, 22: 9184, 23: 3042, 24: 14484}

# atrium layout (world metres; the bounds of Sponza.gltf's accessors x 0.01)
X0, X1, Z0, Z1 = -19.2, 18.0, -11.8, 11.05
XI0, XI1 = -16.5, 15.5           # inner extent of the colonnades
ZC = 4.0                         # colonnade line |z|
COURT = 3.6                      # the open court |z| < COURT (no roof: the sky)


class _Mesh:
    def __init__(self):
        self.pos: List[np.ndarray] = []
        self.nrm: List[np.ndarray] = []
        self.uv: List[np.ndarray] = []
        self.idx: List[np.ndarray] = []
        self.mat: List[np.ndarray] = []
        self.nv = 0

    def add(self, P, N, UV, I, material):
        self.pos.append(np.asarray(P, np.float32).reshape(-1, 3))
        self.nrm.append(np.asarray(N, np.float32).reshape(-1, 3))
        self.uv.append(np.asarray(UV, np.float32).reshape(-1, 2))
        self.idx.append(np.asarray(I, np.int64).reshape(-1, 3) + self.nv)
        self.mat.append(np.full(len(self.idx[-1]), material, np.uint32))
        self.nv += len(self.pos[-1])

    def arrays(self):
        return (np.concatenate(self.pos), np.concatenate(self.nrm), np.concatenate(self.uv),
                np.concatenate(self.idx).astype(np.uint32), np.concatenate(self.mat))


def _surface(P: np.ndarray, UV: np.ndarray, outward: Optional[np.ndarray] = None, center=None):
    """Quad-grid surface from (nv+1, nu+1, 3) points: triangles wound so (b-a)x(c-a) points outward
    (`outward`: a direction, or `center`: away from a point); per-vertex normals from the grid tangents."""
    nv, nu = P.shape[0] - 1, P.shape[1] - 1
    du = np.gradient(P, axis=1)
    dv = np.gradient(P, axis=0)
    N = np.cross(du, dv)
    ln = np.linalg.norm(N, axis=-1, keepdims=True)
    N = N / np.maximum(ln, 1e-12)
    flip = False
    ref = (P - np.asarray(center)) if center is not None else np.broadcast_to(np.asarray(outward, np.float64), P.shape)
    # `outward` may also be a per-point array (e.g. towards an arch's centre)
    if np.sum(N * ref) < 0:
        N = -N
        flip = True
    j, i = np.meshgrid(np.arange(nv), np.arange(nu), indexing="ij")
    a = (j * (nu + 1) + i).ravel()
    b = a + 1
    c = a + (nu + 1)
    d = c + 1
    if not flip:   # du x dv outward: (a, b, d) and (a, d, c) are counter-clockwise seen from outside
        I = np.stack([np.stack([a, b, d], 1), np.stack([a, d, c], 1)], 1).reshape(-1, 3)
    else:
        I = np.stack([np.stack([a, d, b], 1), np.stack([a, c, d], 1)], 1).reshape(-1, 3)
    return P.reshape(-1, 3), N.reshape(-1, 3), UV.reshape(-1, 2), I


def _grid_counts(tris: int, aspect: float):
    """nu, nv with 2 nu nv ~= tris and nu / nv ~= aspect."""
    n = max(tris / 2.0, 1.0)
    nu = max(1, int(round(math.sqrt(n * aspect))))
    nv = max(1, int(round(n / nu)))
    return nu, nv


def panel(m: _Mesh, origin, eu, ev, normal, tris, material, tile=2.0, relief=0.0, freq=(3.0, 2.0), rng=None):
    """Tessellated rectangle origin + s eu + t ev, displaced along `normal` by a relief pattern."""
    eu, ev, normal = np.asarray(eu, np.float64), np.asarray(ev, np.float64), np.asarray(normal, np.float64)
    lu, lv = np.linalg.norm(eu), np.linalg.norm(ev)
    nu, nv = _grid_counts(tris, lu / lv)
    s, t = np.meshgrid(np.linspace(0, 1, nu + 1), np.linspace(0, 1, nv + 1))
    ph = rng.uniform(0, 2 * np.pi, 2) if rng is not None else (0.0, 0.0)
    h = relief * (np.sin(2 * np.pi * freq[0] * s + ph[0]) * np.cos(2 * np.pi * freq[1] * t + ph[1]))
    P = np.asarray(origin) + s[..., None] * eu + t[..., None] * ev + h[..., None] * normal / np.linalg.norm(normal)
    UV = np.stack([s * lu / tile, t * lv / tile], -1)
    m.add(*_surface(P, UV, outward=normal), material)


def column(m: _Mesh, x, z, y0, y1, r, tris, material, flutes=20, tile=1.5):
    """Fluted column shaft with an entasis, radius r (cylinder uvs)."""
    nu, nv = _grid_counts(tris, 2 * np.pi * r / (y1 - y0) * 2.0)
    nu = max(nu, 8)
    nv = max(1, tris // (2 * nu))
    a, t = np.meshgrid(np.linspace(0, 2 * np.pi, nu + 1), np.linspace(0, 1, nv + 1))
    rr = r * (1.0 - 0.08 * t) * (1.0 + 0.03 * np.cos(flutes * a))
    P = np.stack([x + rr * np.cos(a), y0 + t * (y1 - y0), z + rr * np.sin(a)], -1)
    UV = np.stack([a * r / tile, t * (y1 - y0) / tile], -1)
    center = np.stack([np.full_like(t, x), P[..., 1], np.full_like(t, z)], -1)
    m.add(*_surface(P, UV, center=center), material)


def ring(m: _Mesh, x, z, y, r, thick, tris, material, tile=1.0):
    """Torus ring (capitals, column bases, lamp rims)."""
    nu, nv = _grid_counts(tris, r / thick)
    nu, nv = max(nu, 8), max(nv, 3)
    a, b = np.meshgrid(np.linspace(0, 2 * np.pi, nu + 1), np.linspace(0, 2 * np.pi, nv + 1))
    rr = r + thick * np.cos(b)
    P = np.stack([x + rr * np.cos(a), y + thick * np.sin(b), z + rr * np.sin(a)], -1)
    center = np.stack([x + r * np.cos(a), np.full_like(a, y), z + r * np.sin(a)], -1)
    UV = np.stack([a * r / tile, b * thick / tile], -1)
    m.add(*_surface(P, UV, center=center), material)


def arch(m: _Mesh, xa, xb, z, y_spring, depth, band, tris, material, tile=1.5):
    """Semicircular arch band between xa and xb in the plane z (the intrados surface plus its face)."""
    r = (xb - xa) / 2.0
    cx = (xa + xb) / 2.0
    half = tris // 2
    nu, nv = _grid_counts(half, np.pi * r / depth)
    a, t = np.meshgrid(np.linspace(np.pi, 0, nu + 1), np.linspace(-depth / 2, depth / 2, nv + 1))
    P = np.stack([cx + r * np.cos(a), y_spring + r * np.sin(a), z + t], -1)          # intrados (faces the opening)
    toward_axis = np.stack([-np.cos(a), -np.sin(a), np.zeros_like(a)], -1)
    m.add(*_surface(P, np.stack([a * r / tile, t / tile], -1), outward=toward_axis), material)
    nu2, nv2 = _grid_counts(half, np.pi * r / band)
    a2, w = np.meshgrid(np.linspace(np.pi, 0, nu2 + 1), np.linspace(0, band, nv2 + 1))
    for side in (-1.0, 1.0):   # the two faces of the band
        P2 = np.stack([cx + (r + w) * np.cos(a2), y_spring + (r + w) * np.sin(a2), np.full_like(a2, z + side * depth / 2)], -1)
        m.add(*_surface(P2, np.stack([a2 * r / tile, w / tile], -1), outward=(0, 0, side)), material)


def lathe(m: _Mesh, x, z, y0, profile, tris, material, tile=0.8):
    """Surface of revolution of a radius profile r(t), t in [0, 1] over height profile[1]."""
    radii, height = profile
    nu, nv = _grid_counts(tris, 2.0)
    nu = max(nu, 8)
    nv = max(2, tris // (2 * nu))
    a, t = np.meshgrid(np.linspace(0, 2 * np.pi, nu + 1), np.linspace(0, 1, nv + 1))
    rr = np.interp(t, np.linspace(0, 1, len(radii)), radii)
    P = np.stack([x + rr * np.cos(a), y0 + t * height, z + rr * np.sin(a)], -1)
    center = np.stack([np.full_like(t, x), P[..., 1], np.full_like(t, z)], -1)
    m.add(*_surface(P, np.stack([a * 0.3 / tile, t * height / tile], -1), center=center), material)


def leaves(m: _Mesh, x, y, z, radius, tris, material, rng):
    """A plant: curved leaf cards (2 x 4 quads each) fanned around (x, z) from height y."""
    per = 16
    n = max(1, tris // per)
    for _ in range(n):
        az = rng.uniform(0, 2 * np.pi)
        el = rng.uniform(0.2, 1.2)
        ln = radius * rng.uniform(0.6, 1.0)
        wd = ln * 0.18
        s, t = np.meshgrid(np.linspace(0, 1, 3), np.linspace(0, 1, 5))
        d = np.array([np.cos(az) * np.cos(el), np.sin(el), np.sin(az) * np.cos(el)])
        side = np.array([-np.sin(az), 0.0, np.cos(az)])
        up = np.cross(side, d)
        curve = -0.25 * ln * t ** 2
        P = (np.array([x, y, z]) + t[..., None] * ln * d + (s[..., None] - 0.5) * wd * (1 - 0.6 * t[..., None]) * side +
             curve[..., None] * up)
        m.add(*_surface(P, np.stack([s, t], -1), outward=up), material)


def build(seed: int = SEED) -> Dict:
    """Mesh arrays {positions, normals, uvs (float32), indices (T, 3), materials (T,) (uint32)} and the per-material
    triangle counts, for the 25 Sponza materials."""
    rng = np.random.default_rng(seed)
    m = _Mesh()
    xs = [XI0 + 3.0 * i for i in range(11)]            # colonnade bays (3 m)
    # floor of the court and the aisles (material 22: tiled stone floor) and the outer walls (5: brick)
    panel(m, (X0, 0.0, Z1), (X1 - X0, 0, 0), (0, 0, Z0 - Z1), (0, 1, 0), GLTF_TRIANGLES[22], 22, tile=1.0,
          relief=0.004, freq=(60.0, 40.0), rng=rng)
    for (o, eu, ev, n) in (((X0, 0, Z1 - 0.6), (X1 - X0, 0, 0), (0, 14.3, 0), (0, 0, -1)),
                           ((X1, 0, Z0 + 0.6), (X0 - X1, 0, 0), (0, 14.3, 0), (0, 0, 1)),
                           ((X0 + 0.6, 0, Z0), (0, 0, Z1 - Z0), (0, 14.3, 0), (1, 0, 0)),
                           ((X1 - 0.6, 0, Z1), (0, 0, Z0 - Z1), (0, 14.3, 0), (-1, 0, 0))):
        panel(m, o, eu, ev, n, GLTF_TRIANGLES[5] // 4, 5, tile=2.0)
    # colonnades: ground-floor shafts (13), bases (8), first-floor shafts (7), capitals (6)
    cols = [(x, s * ZC) for x in xs for s in (-1, 1)]
    for (x, z) in cols:
        column(m, x, z, 0.35, 5.4, 0.42, GLTF_TRIANGLES[13] // len(cols), 13)
        ring(m, x, z, 0.2, 0.48, 0.2, GLTF_TRIANGLES[8] // len(cols), 8)
        column(m, x, z, 6.6, 11.6, 0.32, GLTF_TRIANGLES[7] // len(cols), 7, flutes=16)
        ring(m, x, z, 5.45, 0.46, 0.14, GLTF_TRIANGLES[6] // (2 * len(cols)), 6)
        ring(m, x, z, 11.6, 0.36, 0.12, GLTF_TRIANGLES[6] // (2 * len(cols)), 6)
    # arcades between the ground-floor columns (12) and the first-floor arches (10: details)
    for s in (-1, 1):
        for a, b in zip(xs[:-1], xs[1:]):
            arch(m, a + 0.42, b - 0.42, s * ZC, 4.0, 0.8, 0.5, GLTF_TRIANGLES[12] * 2 // 3 // 20, 12)
            arch(m, a + 0.32, b - 0.32, s * ZC, 9.6, 0.6, 0.35, GLTF_TRIANGLES[10] * 2 // 3 // 20, 10)
    # galleries (4: floors of the first storey, 11 / 9 / 2: small trims), roof frame (24)
    for s in (-1, 1):
        zin, zout = s * COURT, s * (Z1 if s > 0 else -Z0)
        panel(m, (X0, 6.5, zin), (X1 - X0, 0, 0), (0, 0, zout - zin), (0, 1, 0) if s < 0 else (0, 1, 0),
              GLTF_TRIANGLES[4] // 4, 4, tile=1.0)
        panel(m, (X0, 6.0, zout), (X1 - X0, 0, 0), (0, 0, zin - zout), (0, -1, 0), GLTF_TRIANGLES[4] // 4, 4, tile=1.0)
        panel(m, (X0, 5.4, s * (COURT - 0.05)), (X1 - X0, 0, 0), (0, 1.1, 0), (0, 0, -s), GLTF_TRIANGLES[11] // 2, 11,
              tile=1.0, relief=0.03, freq=(80.0, 3.0), rng=rng)
        panel(m, (X0, 11.8, zin), (X1 - X0, 0, 0), (0, 0, zout - zin), (0, -1, 0), GLTF_TRIANGLES[24] // 4, 24,
              tile=2.0)
        panel(m, (X0, 12.4, zin), (X1 - X0, 0, 0), (0, 0, zout - zin), (0, 1, 0), GLTF_TRIANGLES[24] // 4, 24,
              tile=2.0, relief=0.05, freq=(40.0, 10.0), rng=rng)
        panel(m, (X0, 12.4, s * (COURT - 0.2)), (X1 - X0, 0, 0), (0, 0.8, 0), (0, 0, -s), GLTF_TRIANGLES[9] + 200, 9,
              tile=1.0)
        panel(m, (X0, 7.0, s * (COURT + 0.1)), (X1 - X0, 0, 0), (0, 0.9, 0), (0, 0, -s), GLTF_TRIANGLES[2] + 200, 2,
              tile=1.0)
    # hanging fabrics between the first-floor columns (14, 15, 16) and along the aisle walls (17, 18, 19)
    fab = [14, 15, 16, 14, 15]
    for i, x in enumerate(xs[1:-1:2]):
        for s in (-1, 1):
            mt = fab[i % len(fab)]
            panel(m, (x - 1.2, 11.2, s * (ZC - 0.45)), (2.4, 0, 0), (0, -4.2, 0), (0, 0, -s),
                  GLTF_TRIANGLES[mt] // (2 * fab.count(mt)), mt, tile=2.4, relief=0.12, freq=(4.0, 1.0), rng=rng)
    for i, x in enumerate(xs[::2]):
        for s in (-1, 1):
            mt = (17, 18, 19)[i % 3]
            panel(m, (x - 1.3, 5.2, s * (Z1 - 0.7 if s > 0 else -Z0 - 0.7)), (2.6, 0, 0), (0, -4.6, 0), (0, 0, -s),
                  GLTF_TRIANGLES[mt] // 4, mt, tile=2.6, relief=0.15, freq=(5.0, 1.0), rng=rng)
    # lamps on the ground-floor columns: hanging vases (21) on chains (20)
    for x in xs[::2]:
        for s in (-1, 1):
            lathe(m, x, s * (ZC - 0.7), 2.6, ([0.05, 0.22, 0.28, 0.2, 0.08], 0.6), GLTF_TRIANGLES[21] // 12, 21)
            panel(m, (x - 0.02, 3.2, s * (ZC - 0.7)), (0.04, 0, 0), (0, 2.1, 0), (0, 0, -s), 2, 20, tile=0.1)
    # vases with plants along the court (1: vases, 0: leaves, 3: plant trims), lion reliefs (23) on the end walls
    vx = [-10.0, -7.0, -4.0, -1.0, 2.0, 5.0, 8.0, 11.0]
    for x in vx:
        for s in (-1, 1):
            z = s * 2.6
            lathe(m, x, z, 0.0, ([0.18, 0.32, 0.36, 0.28, 0.2, 0.26], 0.9), GLTF_TRIANGLES[1] // 16, 1)
            leaves(m, x, 0.85, z, 1.1, GLTF_TRIANGLES[0] // 16, 0, rng)
            ring(m, x, z, 0.88, 0.25, 0.05, GLTF_TRIANGLES[3] // 16, 3)
    for x, n in ((X0 + 0.62, 1.0), (X1 - 0.62, -1.0)):
        for z in (-2.0, 2.0):
            lathe_x = x + n * 0.05
            panel(m, (lathe_x, 1.0, z - 0.7), (0, 0, 1.4), (0, 1.6, 0), (n, 0, 0), GLTF_TRIANGLES[23] // 4, 23,
                  tile=1.4, relief=0.12, freq=(3.0, 2.0), rng=rng)
    # a canopy frame above the west end (inside the sun frustum: it casts a shadow into the map)
    panel(m, (-19.0, 27.0, 6.0), (3.5, 0, 0), (0, 0, -12.0), (0, 1, 0), 600, 24, tile=2.0)   # behind the C3 camera, facing the sun
    P, N, UV, I, M = m.arrays()
    return {"positions": P, "normals": N, "uvs": UV, "indices": I, "materials": M, "vertex_count": len(P)}


def texture_index(native: bool = False) -> dict:
    """{material: {"albedo": file, "normal": file}} of the committed 256^2 texture fixture, or of the native-resolution
    set (NATIVE: the reference's own image files, copied by __graft_entry__.build(); not in the history)."""
    root = NATIVE if native else DATA
    path = os.path.join(root, "materials.json")
    if native and not os.path.exists(path):
        raise FileNotFoundError(f"{path}: the native-resolution Sponza textures are made by __graft_entry__.build() "
                                "in a container that has the reference (tools/make_sponza_fixture.py --native)")
    with open(path) as fh:
        return {int(k): v for k, v in json.load(fh).items()}


def native_available() -> bool:
    """True when the native-resolution texture set is complete (its materials.json is written last)."""
    try:
        idx = texture_index(native=True)
    except FileNotFoundError:
        return False
    return all(os.path.exists(os.path.join(NATIVE, f)) for e in idx.values() for f in e.values())


def load_textures(size: Optional[int] = None, native: bool = False) -> Dict[int, dict]:
    """{material: {"albedo": RGBA8 array or None, "normal": RGBA8 array or None}} from the fixture (native=False) or
    the native-resolution set; `size` box-downsamples larger images (None: as stored). Alpha is forced to 255 for
    every image (the G-buffer pass reads colour only, g_buffer_generation.inl:189-194)."""
    from PIL import Image
    root = NATIVE if native else DATA
    out = {}
    for mid, t in texture_index(native).items():
        e = {}
        for k in ("albedo", "normal"):
            if t.get(k):
                im = Image.open(os.path.join(root, t[k])).convert("RGB").convert("RGBA")
                if size and im.size[0] > size:
                    im = im.resize((size, size), Image.BOX)
                e[k] = np.ascontiguousarray(np.asarray(im, np.uint8))
            else:
                e[k] = None
        out[mid] = e
    return out
