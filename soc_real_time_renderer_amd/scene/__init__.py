"""Synthetic frame inputs: the Sponza-proxy G-buffer + sun shadow map (scene_synth.c), the clouds noise
texture (decoded from the reference asset assets/Clouds/noise.png), and seeded random G-buffers for
unit tests. These stand in for the reference's raster producers, which are outside the hot path.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

from .. import _abi
from .._abi import Globals

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(os.path.dirname(HERE), "lib", "libsoc_scene.so")
NOISE_PATH = os.path.join(os.path.dirname(HERE), "data", "clouds_noise_64x64.u8")
SPONZA_PROXY = 0     # the analytic box atrium (ray-cast on the host): unit tests
TERRAIN = 1          # config C4: fBm terrain grid (seed 0x7E44) rasterised on the host
SPONZA_MESH = 2      # configs C2/C3/C5: the ~256k-triangle procedural atrium with the Sponza textures (sponza_mesh.py)

_LIB = None


def build() -> str:
    os.makedirs(os.path.dirname(LIB_PATH), exist_ok=True)
    subprocess.run(["gcc", "-O3", "-march=x86-64-v3", "-fopenmp", "-fPIC", "-shared", "-std=c11",
                    os.path.join(HERE, "scene_synth.c"), "-o", LIB_PATH, "-lm"], check=True)
    return LIB_PATH


def lib():
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            build()
        l = C.CDLL(LIB_PATH)
        G = C.POINTER(Globals)
        _abi.bind(l, {
            "soc_scene_gbuffer": (C.c_int, [C.c_int, G, C.c_int, C.c_int] + [C.c_void_p] * 5),
            "soc_scene_shadow": (C.c_int, [C.c_int, G, C.c_int, C.c_void_p]),
            "soc_scene_box_count": (C.c_int, [C.c_int]),
            "soc_scene_mesh_counts": (C.c_int, [C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
            "soc_scene_mesh": (C.c_int, [C.c_int, G] + [C.c_void_p] * 5),
            "soc_scene_material_count": (C.c_int, [C.c_int]),
            "soc_scene_terrain_heightmap": (C.c_int, [C.c_int, C.c_void_p]),
            "soc_scene_material_textures": (C.c_int, [C.c_int, G, C.c_int, C.c_void_p, C.c_void_p]),
        })
        _LIB = l
    return _LIB


def gbuffer(g: Globals, width: int, height: int, scene_id: int = SPONZA_PROXY) -> dict:
    """Host numpy G-buffer: albedo/emissive/normal/velocity (H,W,4) float16, depth (H,W) float32."""
    out = {k: np.zeros((height, width, 4), np.float16) for k in ("albedo", "emissive", "normal", "velocity")}
    out["depth"] = np.ones((height, width), np.float32)
    rc = lib().soc_scene_gbuffer(scene_id, C.byref(g), width, height, out["albedo"].ctypes.data,
                                 out["emissive"].ctypes.data, out["normal"].ctypes.data, out["depth"].ctypes.data,
                                 out["velocity"].ctypes.data)
    if rc:
        raise RuntimeError("soc_scene_gbuffer failed")
    return out


def shadow_map(g: Globals, size: int = 4096, scene_id: int = SPONZA_PROXY) -> np.ndarray:
    s = np.ones((size, size), np.float32)
    if lib().soc_scene_shadow(scene_id, C.byref(g), size, s.ctypes.data):
        raise RuntimeError("soc_scene_shadow failed")
    return s


def mesh(g: Globals, scene_id: int = SPONZA_PROXY) -> dict:
    """The scene as a triangle mesh for the rasteriser: positions/normals (V,3) f32, uvs (V,2) f32,
    indices (T,3) u32, materials (T,) u32."""
    nv, nt = C.c_int(), C.c_int()
    lib().soc_scene_mesh_counts(scene_id, C.byref(nv), C.byref(nt))
    V, T = nv.value, nt.value
    out = {"positions": np.zeros((V, 3), np.float32), "normals": np.zeros((V, 3), np.float32),
           "uvs": np.zeros((V, 2), np.float32), "indices": np.zeros((T, 3), np.uint32),
           "materials": np.zeros(T, np.uint32)}
    if lib().soc_scene_mesh(scene_id, C.byref(g), *(out[k].ctypes.data for k in
                                                    ("positions", "normals", "uvs", "indices", "materials"))):
        raise RuntimeError("soc_scene_mesh failed")
    return out


def material_textures(g: Globals, size: int, scene_id: int = SPONZA_PROXY):
    """(M, size, size, 4) uint8 albedo textures (linear values, UNORM) and (M, 3) emissive factors."""
    m = lib().soc_scene_material_count(scene_id)
    tex = np.zeros((m, size, size, 4), np.uint8)
    em = np.zeros((m, 3), np.float32)
    if lib().soc_scene_material_textures(scene_id, C.byref(g), size, tex.ctypes.data, em.ctypes.data):
        raise RuntimeError("soc_scene_material_textures failed")
    return tex, em


def terrain_heightmap(size: int = 1024) -> np.ndarray:
    """(size, size, 4) uint8 heightmap of the C4 terrain (R8G8B8A8_UNORM as renderer.cpp:155 loads it)."""
    out = np.zeros((size, size, 4), np.uint8)
    if lib().soc_scene_terrain_heightmap(size, out.ctypes.data):
        raise RuntimeError("soc_scene_terrain_heightmap failed")
    return out


def noise_texture() -> np.ndarray:
    """assets/Clouds/noise.png (64x64 grey, loaded as R8G8B8A8_UNORM by renderer.cpp:152) as RGBA8."""
    grey = np.fromfile(NOISE_PATH, dtype=np.uint8).reshape(64, 64)
    rgba = np.empty((64, 64, 4), np.uint8)
    rgba[..., 0] = rgba[..., 1] = rgba[..., 2] = grey
    rgba[..., 3] = 255
    return rgba


def random_gbuffer(width: int, height: int, seed: int = 0, sky_fraction: float = 0.15) -> dict:
    """Seeded random-but-plausible G-buffer for unit tests (depths in the NO range, unit normals, sky)."""
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:height, 0:width].astype(np.float32)
    # smooth depth field in view distance [0.5, 40] -> NDC z of the default projection
    dist = 0.5 + 39.5 * (0.5 + 0.25 * np.sin(xx / 7.0 + rng.uniform(0, 6)) + 0.25 * np.cos(yy / 5.0 + rng.uniform(0, 6)))
    dist += rng.uniform(-0.05, 0.05, size=dist.shape)
    n, f = 0.1, 1000.0
    z = (f + n) / (f - n) - (2 * f * n) / ((f - n) * dist)
    depth = z.astype(np.float32)
    sky = (yy < height * sky_fraction) | (rng.uniform(size=depth.shape) < 0.01)
    depth[sky] = 1.0
    nrm = rng.normal(size=(height, width, 3)).astype(np.float32)
    nrm /= np.linalg.norm(nrm, axis=2, keepdims=True)
    out = {
        "albedo": np.concatenate([rng.uniform(0.05, 0.95, (height, width, 3)), np.ones((height, width, 1))], 2),
        "emissive": np.concatenate([np.where(rng.uniform(size=(height, width, 1)) < 0.03,
                                             rng.uniform(0, 6, (height, width, 3)), 0.0), np.ones((height, width, 1))], 2),
        "normal": np.concatenate([nrm, np.ones((height, width, 1))], 2),
        "velocity": np.concatenate([rng.normal(0, 0.002, (height, width, 2)), np.zeros((height, width, 1)),
                                    np.ones((height, width, 1))], 2),
        "depth": depth,
    }
    for k in ("albedo", "emissive", "normal", "velocity"):
        out[k] = out[k].astype(np.float16)
    return out
