"""Host binding of the rasteriser passes (include/soc_rt.h "Rasterisation").

The reference draws its meshes with three raster pipelines: DepthPrepassTask (depth_prepass.inl:26-120),
GBufferGenerationTask (g_buffer_generation.inl:33-230) and SunShadowDrawTask (sun_shadow_draw.inl:27-91).
Here they are a visibility-buffer raster + resolve in libsoc_rt.so; this module only packs the mesh and
material structs (device pointers) and calls the C ABI. The same struct helpers accept numpy arrays so the
CPU oracle can be driven with host pointers.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import Optional, Sequence

import numpy as np
import torch

from . import _abi, _check, _gp, _ptr, _stream, img, lib
from ._abi import (CULL_BACK, CULL_FRONT, CULL_NONE, FMT_RGBA8_SRGB, FMT_RGBA8_UNORM, MATERIAL_MIPMAPPED,
                   MATERIAL_NORMAL_MAP, MATERIAL_NORMAL_TEXTURE, MATERIAL_PAIRED_TEXELS, MATERIAL_ZERO_VELOCITY, Material, Mesh,
                   SocImg)

__all__ = ["CULL_NONE", "CULL_FRONT", "CULL_BACK", "MATERIAL_ZERO_VELOCITY", "MeshBuffers", "MipTexture", "material",
           "normal_matrix", "materials_device", "raster_visibility", "raster_depth", "gbuffer_resolve",
           "SHADOW_BIAS_CONSTANT", "SHADOW_BIAS_SLOPE"]

# sun_shadow_draw.inl:47-50 / :81
SHADOW_BIAS_CONSTANT = 1.25
SHADOW_BIAS_SLOPE = 1.75

IDENTITY = np.eye(4, dtype=np.float32)


def normal_matrix(model) -> np.ndarray:
    """transpose(inverse(model)) (scene.cpp:69), column-major float32[16]."""
    m = np.asarray(model, np.float64).reshape(4, 4).T            # M (row-major) from the column-major flat
    # column-major flat of N = inverse(M)^T is the row-major flat of inverse(M)
    return np.ascontiguousarray(np.linalg.inv(m).astype(np.float32)).reshape(16)


def _colmajor(model) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(model, np.float32).reshape(16))


@dataclass
class MeshBuffers:
    """A mesh's vertex / index / material-index arrays (torch device tensors or numpy host arrays) and its
    soc_mesh struct. `model` is a column-major 4x4 (glm layout), identity by default."""
    positions: object
    normals: object
    uvs: object
    indices: object
    materials: object = None
    model: np.ndarray = field(default_factory=lambda: IDENTITY.reshape(16).copy())
    struct: Mesh = None

    def __post_init__(self):
        def addr(a):
            if a is None:
                return None
            if isinstance(a, torch.Tensor):
                assert a.is_contiguous()
                return a.data_ptr()
            assert a.flags["C_CONTIGUOUS"]
            return a.ctypes.data
        s = Mesh()
        s.positions, s.normals, s.uvs = addr(self.positions), addr(self.normals), addr(self.uvs)
        s.indices, s.materials = addr(self.indices), addr(self.materials)
        s.vertex_count = int(self.positions.shape[0])
        s.triangle_count = int(self.indices.shape[0])
        s.model_matrix[:] = _colmajor(self.model).tolist()
        s.normal_matrix[:] = normal_matrix(self.model).tolist()
        self.struct = s

    @classmethod
    def from_numpy(cls, positions, normals, uvs, indices, materials=None, model=None, device="cuda"):
        t = lambda a, dt: None if a is None else torch.from_numpy(np.ascontiguousarray(a, dt)).to(device)
        return cls(t(positions, np.float32), t(normals, np.float32), t(uvs, np.float32), t(indices, np.uint32),
                   t(materials, np.uint32), IDENTITY.reshape(16).copy() if model is None else _colmajor(model))

    def workspace(self, device="cuda") -> torch.Tensor:
        n = lib().soc_raster_workspace_size(self.struct.vertex_count, self.struct.triangle_count)
        return torch.empty(n, dtype=torch.uint8, device=device)


def mip_level_count(width: int, height: int) -> int:
    """floor(log2(max(W, H))) + 1 (texture.cpp:108)."""
    return int(lib().soc_mip_level_count(int(width), int(height)))


def mip_level_shapes(width: int, height: int):
    """(h, w) of every level of a chain: max(1, W >> k) x max(1, H >> k)."""
    return [(max(1, height >> k), max(1, width >> k)) for k in range(mip_level_count(width, height))]


class MipTexture:
    """An RGBA8 texture with its packed mip chain (include/soc_rt.h soc_generate_mips): `buf` is one flat uint8
    buffer (device tensor or host array) holding level 0 (tight rows) followed by levels 1.. . The reference
    builds the chain at upload (texture.cpp:184-246); build() does the same on the GPU."""

    def __init__(self, buf, width: int, height: int, srgb: bool = True):
        self.buf, self.width, self.height = buf, int(width), int(height)
        self.format = FMT_RGBA8_SRGB if srgb else FMT_RGBA8_UNORM

    @staticmethod
    def chain_bytes(width: int, height: int) -> int:
        return int(lib().soc_mip_chain_bytes(int(width), int(height), int(width) * 4))

    @classmethod
    def build(cls, level0, srgb: bool = True, device="cuda", stream=None) -> "MipTexture":
        """Upload an (H, W, 4) uint8 level 0 and generate levels 1.. with soc_generate_mips."""
        t = level0 if isinstance(level0, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(level0, np.uint8))
        H, W = int(t.shape[0]), int(t.shape[1])
        buf = torch.empty(cls.chain_bytes(W, H), dtype=torch.uint8, device=device)
        buf[:H * W * 4].copy_(t.reshape(-1))
        tex = cls(buf, W, H, srgb)
        _check(lib().soc_generate_mips(tex.img(), _stream(stream)), "generate_mips")
        return tex

    def img(self) -> SocImg:
        ptr = self.buf.data_ptr() if isinstance(self.buf, torch.Tensor) else self.buf.ctypes.data
        return SocImg(ptr, self.width, self.height, self.width * 4, self.format)

    def levels(self):
        """Host copies of every level, (h, w, 4) uint8."""
        raw = self.buf.cpu().numpy() if isinstance(self.buf, torch.Tensor) else np.asarray(self.buf)
        out, off = [], 0
        for h, w in mip_level_shapes(self.width, self.height):
            out.append(raw[off:off + h * w * 4].reshape(h, w, 4))
            off += h * w * 4
        return out


def material(albedo=None, emissive=None, albedo_factor=(1.0, 1.0, 1.0, 1.0), emissive_factor=(1.0, 1.0, 1.0, 1.0),
             flags=0, has_emissive: Optional[bool] = None, srgb=True, normal_map=None, normal_texture=None,
             max_anisotropy: float = 16.0) -> Material:
    """soc_material: albedo / emissive RGBA8 textures ((H, W, 4) uint8 tensors or arrays; sRGB like the
    reference's baseColor/emissive images, model.cpp:52-71) or None (white / no emissive); normal_texture: the
    glTF tangent-space normal image (RGBA8 UNORM, has_normal_image, g_buffer_generation.inl:197-211).
    MipTexture arguments make the material mip-mapped (SOC_MATERIAL_MIPMAPPED: trilinear, anisotropy up to
    max_anisotropy as the reference's sampler, texture.cpp:121-136); then every texture given must be one."""
    m = Material()
    fmt = FMT_RGBA8_SRGB if srgb else None
    given = [t for t in (albedo, emissive, normal_texture) if t is not None]
    mipped = any(isinstance(t, MipTexture) for t in given)
    if mipped and not all(isinstance(t, MipTexture) for t in given):
        raise ValueError("a mip-mapped material needs every RGBA8 texture as a MipTexture")
    tex_img = lambda t, f: t.img() if isinstance(t, MipTexture) else img(t, f)
    m.albedo = tex_img(albedo, fmt) if albedo is not None else img(None)
    m.emissive = tex_img(emissive, fmt) if emissive is not None else img(None)
    if mipped:
        m.flags |= MATERIAL_MIPMAPPED
        m.max_anisotropy = float(max_anisotropy)
    m.albedo_factor[:] = [float(v) for v in albedo_factor]
    m.emissive_factor[:] = [float(v) for v in emissive_factor]
    m.flags |= int(flags)
    m.has_emissive = int(emissive is not None if has_emissive is None else has_emissive)
    m.normal_map = img(normal_map) if normal_map is not None else img(None)
    if normal_map is not None:
        m.flags |= MATERIAL_NORMAL_MAP
    m.normal_image = tex_img(normal_texture, FMT_RGBA8_UNORM) if normal_texture is not None else img(None)
    if normal_texture is not None:
        m.flags |= MATERIAL_NORMAL_TEXTURE
    if (mipped and albedo is not None and normal_texture is not None and isinstance(albedo.buf, torch.Tensor)
            and isinstance(normal_texture.buf, torch.Tensor) and albedo.buf.is_cuda and normal_texture.buf.is_cuda
            and albedo.buf.device == normal_texture.buf.device
            and (albedo.width, albedo.height) == (normal_texture.width, normal_texture.height)):
        m.paired_texels = paired_texels(albedo, normal_texture)
        m.flags |= MATERIAL_PAIRED_TEXELS
    return m


def paired_texels(albedo: MipTexture, normal_texture: MipTexture, stream=None) -> int:
    """soc_pair_textures: the two device mip chains interleaved texel by texel (the G-buffer resolve then reads both
    textures of a tap row with one load). Returns its device address for soc_material.paired_texels (with
    SOC_MATERIAL_PAIRED_TEXELS). The buffer is kept on the normal texture, one per albedo it was paired with (the entry
    also holds the albedo, so its id is not reused): a normal texture shared by several materials, or a material built
    twice, never frees a buffer a live material points at, and the same pair is interleaved once."""
    if normal_texture.buf.device != albedo.buf.device:
        raise ValueError("paired_texels: albedo and normal texture on different devices")
    cache = getattr(normal_texture, "paired", None)
    if not isinstance(cache, dict):
        cache = normal_texture.paired = {}
    hit = cache.get(id(albedo))
    if hit is not None and hit[0] is albedo:
        return hit[1].data_ptr()
    n = int(lib().soc_paired_texels_bytes(albedo.width, albedo.height))
    buf = torch.empty(n, dtype=torch.uint8, device=albedo.buf.device)
    _check(lib().soc_pair_textures(albedo.img(), normal_texture.img(), C.c_void_p(buf.data_ptr()), _stream(stream)),
           "pair_textures")
    cache[id(albedo)] = (albedo, buf)
    return buf.data_ptr()


def materials_device(mats: Sequence[Material], device="cuda") -> torch.Tensor:
    """Device copy of a soc_material array (raw bytes)."""
    arr = (Material * len(mats))(*mats)
    raw = np.frombuffer(bytes(arr), dtype=np.uint8).copy()
    return torch.from_numpy(raw).to(device)


def raster_visibility(mesh: MeshBuffers, view_projection, cull, visibility: torch.Tensor, workspace: torch.Tensor,
                      clear=True, stream=None):
    """Depth prepass into an (H, W) int64/uint64 visibility buffer (depth bits << 32 | triangle key)."""
    H, W = visibility.shape
    vp = (C.c_float * 16)(*[float(v) for v in np.asarray(view_projection, np.float32).reshape(16)])
    _check(lib().soc_raster_visibility(C.byref(mesh.struct), vp, int(cull), _ptr(visibility), W, H, int(bool(clear)),
                                       _ptr(workspace), _stream(stream)), "raster_visibility")


def raster_depth(mesh: MeshBuffers, view_projection, cull, depth: torch.Tensor, workspace: torch.Tensor,
                 bias_constant=0.0, bias_slope=0.0, stream=None):
    """Depth-only raster into a D32 image (the sun shadow map with SHADOW_BIAS_*)."""
    vp = (C.c_float * 16)(*[float(v) for v in np.asarray(view_projection, np.float32).reshape(16)])
    _check(lib().soc_raster_depth(C.byref(mesh.struct), vp, int(cull), float(bias_constant), float(bias_slope),
                                  img(depth), _ptr(workspace), _stream(stream)), "raster_depth")


def gbuffer_resolve(g, mesh: MeshBuffers, d_materials: torch.Tensor, material_count: int, visibility: torch.Tensor,
                    depth, albedo, emissive, normal, velocity, workspace=None, stream=None):
    """workspace (MeshBuffers.workspace()): vertex stage once per vertex; None: per pixel (same bits)."""
    _check(lib().soc_gbuffer_resolve(_gp(g), C.byref(mesh.struct), _ptr(d_materials), int(material_count),
                                     _ptr(visibility), img(depth), img(albedo), img(emissive), img(normal), img(velocity),
                                     _ptr(workspace), _stream(stream)), "gbuffer_resolve")


def visibility_triangles(vis) -> np.ndarray:
    """Triangle id per pixel (-1 = empty) of a host visibility buffer (uint64/int64 array)."""
    low = (np.asarray(vis).view(np.uint64) & np.uint64(0xFFFFFFFF)).astype(np.int64)
    return np.where(low == 0xFFFFFFFF, -1, 0xFFFFFFFE - low)


def sponza_mesh_materials(tex_size: Optional[int] = None, device=None, mips: bool = False, host_mip_generator=None,
                          native: bool = False):
    """The 25 Sponza materials of the mesh proxy: baseColor (sRGB) and normal (UNORM) textures from the 256^2 fixture
    or (native=True) the reference's images at their own resolution, box-downsampled to tex_size when larger;
    no emissive image (Sponza has none); albedo factor 1 (GBufferGeneration ignores baseColorFactor,
    g_buffer_generation.inl:189-194). mips=True gives every texture its mip chain (the reference's upload,
    texture.cpp:184-246) and the anisotropic sampler: built on `device` by soc_generate_mips, or for host
    materials (device None) by `host_mip_generator(MipTexture)`. Returns (materials, textures kept alive)."""
    from .scene import sponza_mesh
    tex = sponza_mesh.load_textures(tex_size, native=native)
    keep, mats = [], []

    def prep(a, srgb):
        if a is None:
            return None
        if mips:
            if device is not None:
                return MipTexture.build(a, srgb, device)
            H, W = a.shape[:2]
            buf = np.zeros(MipTexture.chain_bytes(W, H), np.uint8)
            buf[:H * W * 4] = np.ascontiguousarray(a).reshape(-1)
            t = MipTexture(buf, W, H, srgb)
            if host_mip_generator is None:
                raise ValueError("host mip-mapped materials need a host_mip_generator")
            host_mip_generator(t)
            return t
        return torch.from_numpy(a).to(device) if device is not None else a

    for i in range(len(sponza_mesh.GLTF_TRIANGLES)):
        t = tex.get(i, {})
        a, n = prep(t.get("albedo"), True), prep(t.get("normal"), False)
        keep += [a, n]
        mats.append(material(albedo=a, normal_texture=n))
    return mats, keep


def scene_setup(g, scene_id: int, tex_size: Optional[int] = 512, device="cuda", mips: bool = True,
                native: bool = False) -> dict:
    """Device mesh, textures and material array of a synthetic scene: the Sponza-proxy mesh (sponza_mesh.py, the
    reference's Sponza textures), the box atrium (scene_synth.c: sRGB tiled textures, emissive lamps) or the terrain
    (the GPU-tessellated patch grid over a tex_size^2 heightmap, UNORM albedo, velocity 0 as draw_terrain.inl:221).
    native=True: the mesh proxy samples the native-resolution Sponza images (sponza_mesh.NATIVE)."""
    from . import scene as _scene
    if scene_id == _scene.SPONZA_MESH:
        from .scene import sponza_mesh
        m = sponza_mesh.build()
        mesh = MeshBuffers.from_numpy(m["positions"], m["normals"], m["uvs"], m["indices"], m["materials"],
                                      device=device)
        mats, keep = sponza_mesh_materials(tex_size, device, mips=mips, native=native)
        return {"mesh": mesh, "textures": keep, "normal_map": None, "materials": materials_device(mats, device),
                "material_count": len(mats), "host_mesh": m, "workspace": mesh.workspace(device)}
    tex, em = _scene.material_textures(g, tex_size, scene_id)
    terrain = scene_id == _scene.TERRAIN
    dtex = [torch.from_numpy(tex[i]).to(device) for i in range(len(tex))]
    nmap = None
    if terrain:
        # the terrain's normal map from its heightmap (HeightToNormalTask, renderer.cpp:158-190), and its mesh:
        # the patch grid tessellated on the GPU with heights from the same heightmap (draw_terrain.inl:138-191)
        hm = torch.from_numpy(_scene.terrain_heightmap(tex_size)).to(device)
        nmap = torch.empty((tex_size, tex_size, 4), dtype=torch.float16, device=device)
        height_to_normal(hm, nmap)
        mesh = terrain_tessellate(g, hm, device=device)
        torch.cuda.synchronize()
        m = {"positions": mesh.positions.cpu().numpy(), "normals": mesh.normals.cpu().numpy(),
             "uvs": mesh.uvs.cpu().numpy(), "indices": mesh.indices.cpu().numpy().view(np.uint32),
             "materials": mesh.materials.cpu().numpy().view(np.uint32)}
    else:
        m = _scene.mesh(g, scene_id)
        mesh = MeshBuffers.from_numpy(m["positions"], m["normals"], m["uvs"], m["indices"], m["materials"],
                                      device=device)
    mats = [material(albedo=dtex[i], emissive_factor=tuple(float(v) for v in em[i]) + (1.0,),
                     has_emissive=bool(em[i].any()), flags=MATERIAL_ZERO_VELOCITY if terrain else 0, srgb=not terrain,
                     normal_map=nmap)
            for i in range(len(tex))]
    return {"mesh": mesh, "textures": dtex, "normal_map": nmap, "materials": materials_device(mats, device),
            "material_count": len(mats), "host_mesh": m, "host_textures": tex, "emissive": em,
            "workspace": mesh.workspace(device)}


def render_gbuffer(g, sc: dict, width: int, height: int, shadow_size: int = 4096, device="cuda") -> dict:
    """The G-buffer (depth prepass + GBufferGeneration) and the sun shadow map (SunShadowDraw) of a scene_setup()
    scene, rendered once by the HIP rasteriser into device images (the inputs of the screen-space chain)."""
    f16 = dict(dtype=torch.float16, device=device)
    out = {k: torch.zeros((height, width, 4), **f16) for k in ("albedo", "emissive", "normal", "velocity")}
    out["depth"] = torch.ones((height, width), dtype=torch.float32, device=device)
    out["shadow"] = torch.ones((shadow_size, shadow_size), dtype=torch.float32, device=device)
    vis = torch.empty((height, width), dtype=torch.int64, device=device)
    raster_visibility(sc["mesh"], np.ctypeslib.as_array(g.camera_projection_view_matrix), CULL_FRONT, vis,
                      sc["workspace"])
    gbuffer_resolve(g, sc["mesh"], sc["materials"], sc["material_count"], vis, out["depth"], out["albedo"],
                    out["emissive"], out["normal"], out["velocity"], sc["workspace"])
    raster_depth(sc["mesh"], np.ctypeslib.as_array(g.sun_info.projection_view_matrix), CULL_BACK, out["shadow"],
                 sc["workspace"], SHADOW_BIAS_CONSTANT, SHADOW_BIAS_SLOPE)
    return out


TERRAIN_GRID = 100   # renderer.cpp:197


def terrain_tess_counts(grid_size: int = TERRAIN_GRID, tess_level: int = 3):
    v, t = C.c_int32(), C.c_int32()
    _check(lib().soc_terrain_tess_counts(int(grid_size), int(tess_level), C.byref(v), C.byref(t)), "terrain_tess_counts")
    return v.value, t.value


def terrain_tessellate(g, heightmap, grid_size: int = TERRAIN_GRID, tess_level: Optional[int] = None, device="cuda",
                       stream=None) -> MeshBuffers:
    """DrawTerrain's patch grid tessellated on the GPU (soc_terrain_tessellate): the terrain as a MeshBuffers
    whose heights come from `heightmap` ((H, W, 4) uint8 device tensor); level = globals' terrain_max_tess_level."""
    n = int(g.terrain_max_tess_level if tess_level is None else tess_level)
    V, T = terrain_tess_counts(grid_size, n)
    f32 = dict(dtype=torch.float32, device=device)
    pos, nrm, uv = torch.empty((V, 3), **f32), torch.empty((V, 3), **f32), torch.empty((V, 2), **f32)
    idx = torch.empty((T, 3), dtype=torch.int32, device=device)
    _check(lib().soc_terrain_tessellate(_gp(g), img(heightmap), int(grid_size), n, _ptr(pos), _ptr(nrm), _ptr(uv),
                                        _ptr(idx), _stream(stream)), "terrain_tessellate")
    mats = torch.zeros(T, dtype=torch.int32, device=device)
    return MeshBuffers(pos, nrm, uv, idx, mats)


def height_to_normal(heightmap, normal_target, stream=None):
    """HeightToNormalTask (height_to_normal.inl:52-83): (H, W, 4) uint8 heightmap -> (H, W, 4) f16 normals."""
    _check(lib().soc_height_to_normal(img(heightmap), img(normal_target), _stream(stream)), "height_to_normal")


def hiz_mip_count(width: int, height: int) -> int:
    """ceil(log2(max(W/2, H/2))) levels (generate_min_hiz.inl:36-37)."""
    import math
    return int(math.ceil(math.log2(max(width // 2, height // 2))))


def generate_hiz(g, depth, mips, op_max=False, counter=None, stream=None):
    """Min (or max) Hi-Z pyramid of a D32 depth into `mips` (list of (H/2>>i, W/2>>i) f32 tensors)."""
    if counter is None:
        counter = torch.zeros(1, dtype=torch.int32, device=depth.device)
    arr = (_abi.SocImg * len(mips))(*[img(m) for m in mips])
    _check(lib().soc_generate_hiz(_gp(g), img(depth), arr, len(mips), int(bool(op_max)), _ptr(counter), _stream(stream)),
           "generate_hiz")
