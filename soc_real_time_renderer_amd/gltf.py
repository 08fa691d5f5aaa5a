"""glTF 2.0 ingest for the rasteriser: Model::Model (model.cpp:15-466) restated.

Reads a .gltf (JSON) with its .bin buffers and image files into one raster.MeshBuffers-ready mesh and the
material list the G-buffer pass samples. Reference behaviour kept:
  * vertices: POSITION, NORMAL, TEXCOORD_0 as float32 (model.cpp:296-345); missing uvs are (0, 0);
  * indices: u8 / u16 / u32 widened to u32 (:347-381);
  * quirk Q4: the loop runs over scene.nodeIndices.size() but reads asset.nodes[i] (not
    nodes[nodeIndices[i]]), node transforms are ignored, and the vertex / index offsets restart at 0 for
    every node (:290-395), so each primitive's indices are rebased by the node-local vertex offset only;
  * materials: baseColor and emissive textures are sRGB, the others UNORM (:52-71); a material without a
    baseColor texture samples the white null texture (:188-203); emissive only with an emissive texture
    (g_buffer_generation.inl:189-191), factors ignored as the shader does.
Image decoding uses Pillow (present in this image); images are RGBA8, optionally box-downsampled to a
maximum size (the reference keeps full size plus a mip chain; the raster samples level 0 only).
"""
from __future__ import annotations

import json
import os
from typing import Optional

import numpy as np

_COMPONENT = {5121: np.uint8, 5123: np.uint16, 5125: np.uint32, 5126: np.float32}
_NCOMP = {"SCALAR": 1, "VEC2": 2, "VEC3": 3, "VEC4": 4}


def _accessor(doc, buffers, index):
    acc = doc["accessors"][index]
    view = doc["bufferViews"][acc["bufferView"]]
    dt = np.dtype(_COMPONENT[acc["componentType"]])
    n = _NCOMP[acc["type"]]
    start = view.get("byteOffset", 0) + acc.get("byteOffset", 0)
    stride = view.get("byteStride", 0) or dt.itemsize * n
    raw = buffers[view["buffer"]]
    if stride == dt.itemsize * n:
        a = np.frombuffer(raw, dtype=dt, count=acc["count"] * n, offset=start)
    else:
        rows = np.frombuffer(raw, dtype=np.uint8, count=stride * (acc["count"] - 1) + dt.itemsize * n, offset=start)
        a = np.lib.stride_tricks.as_strided(rows, (acc["count"], dt.itemsize * n), (stride, 1)).copy().view(dt)
    return a.reshape(acc["count"], n) if n > 1 else a.reshape(acc["count"])


def load_image(path: str, max_size: Optional[int] = None) -> np.ndarray:
    """RGBA8 (H, W, 4) of an image file, box-downsampled by powers of two to at most max_size."""
    from PIL import Image
    im = np.asarray(Image.open(path).convert("RGBA"), dtype=np.uint8)
    while max_size and max(im.shape[:2]) > max_size and im.shape[0] % 2 == 0 and im.shape[1] % 2 == 0:
        im = ((im[0::2, 0::2].astype(np.uint16) + im[1::2, 0::2] + im[0::2, 1::2] + im[1::2, 1::2] + 2) // 4).astype(np.uint8)
    return np.ascontiguousarray(im)


def load(path: str, max_texture: Optional[int] = None, images: Optional[dict] = None) -> dict:
    """Mesh arrays (positions, normals, uvs: float32; indices (T, 3) and materials (T,): uint32) and
    `materials`: a list of dicts {albedo, emissive (RGBA8 arrays or None), albedo_srgb, emissive_srgb}.
    `images` may map image uri -> RGBA8 array to bypass decoding."""
    base = os.path.dirname(os.path.abspath(path))
    with open(path) as f:
        doc = json.load(f)
    buffers = []
    for b in doc.get("buffers", []):
        with open(os.path.join(base, b["uri"]), "rb") as f:
            buffers.append(f.read())
    pos, nrm, uv, idx, mat = [], [], [], [], []
    total = 0
    for scene in doc.get("scenes", []):
        for i in range(len(scene.get("nodes", []))):   # Q4: nodes[i], not nodes[scene.nodes[i]]
            node = doc["nodes"][i]
            if "mesh" not in node:
                continue
            node_vertex_offset = 0                      # Q4: offsets restart per node
            for prim in doc["meshes"][node["mesh"]]["primitives"]:
                at = prim["attributes"]
                p = _accessor(doc, buffers, at["POSITION"]).astype(np.float32)
                n = _accessor(doc, buffers, at["NORMAL"]).astype(np.float32) if "NORMAL" in at else np.zeros_like(p)
                t = (_accessor(doc, buffers, at["TEXCOORD_0"]).astype(np.float32) if "TEXCOORD_0" in at
                     else np.zeros((len(p), 2), np.float32))
                ind = _accessor(doc, buffers, prim["indices"]).astype(np.uint32)
                pos.append(p); nrm.append(n); uv.append(t)
                # draw_indexed(first_index, vertex_offset = node-local offset): global index in the
                # concatenated vertex array = local index + node-local offset (renderer draw, :1103-1117)
                idx.append(ind.reshape(-1, 3) + np.uint32(node_vertex_offset))
                mat.append(np.full(len(ind) // 3, prim.get("material", 0), np.uint32))
                node_vertex_offset += len(p)
                total += len(p)
    tex_cache = {}

    def tex(ti):
        uri = doc["images"][doc["textures"][ti]["source"]]["uri"]
        if uri not in tex_cache:
            tex_cache[uri] = images[uri] if images and uri in images else load_image(os.path.join(base, uri), max_texture)
        return tex_cache[uri]

    materials = []
    for m in doc.get("materials", []):
        pbr = m.get("pbrMetallicRoughness", {})
        materials.append({
            "albedo": tex(pbr["baseColorTexture"]["index"]) if "baseColorTexture" in pbr else None,
            "emissive": tex(m["emissiveTexture"]["index"]) if "emissiveTexture" in m else None,
            # normalTexture: UNORM (model.cpp:52-71 makes only baseColor / emissive images sRGB), :217-224
            "normal": tex(m["normalTexture"]["index"]) if "normalTexture" in m else None,
            "albedo_srgb": True, "emissive_srgb": True,
        })
    if not materials:
        materials.append({"albedo": None, "emissive": None, "normal": None, "albedo_srgb": True, "emissive_srgb": True})
    return {"positions": np.ascontiguousarray(np.concatenate(pos)), "normals": np.ascontiguousarray(np.concatenate(nrm)),
            "uvs": np.ascontiguousarray(np.concatenate(uv)), "indices": np.ascontiguousarray(np.concatenate(idx)),
            "materials": np.ascontiguousarray(np.concatenate(mat)), "material_list": materials, "vertex_count": total}
