"""Sponza texture sets of the mesh proxy, made in the container that has /root/reference (the bench and the tests read
only what this writes):

- the committed 256^2 fixture (soc_real_time_renderer_amd/data/sponza/): the baseColor and normal images of the
  reference's 25 Sponza materials (assets/Sponza/glTF/Sponza.gltf, materials[i].pbrMetallicRoughness.baseColorTexture
  and normalTexture), decoded with Pillow, box-downsampled 1024^2 -> 256^2 and stored as JPEG (quality 92), plus
  materials.json mapping material index -> files (`python tools/make_sponza_fixture.py`);
- the native-resolution set (soc_real_time_renderer_amd/data/sponza_native/, git-ignored like the built libraries
  and shipped to the GPU box with them): the same 49 image files byte for byte (1024^2, one 4^2), written by
  __graft_entry__.build() through `native()` (`python tools/make_sponza_fixture.py --native`)."""
import json
import os
import shutil
import sys

SRC = "/root/reference/assets/Sponza/glTF"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DST = os.path.join(ROOT, "soc_real_time_renderer_amd", "data", "sponza")
NATIVE_DST = os.path.join(ROOT, "soc_real_time_renderer_amd", "data", "sponza_native")
SIZE = 256


def _material_images(doc):
    """(material index, "albedo" | "normal", image uri) of every material texture the G-buffer pass samples."""
    for i, m in enumerate(doc["materials"]):
        for key, ref in (("albedo", m.get("pbrMetallicRoughness", {}).get("baseColorTexture")),
                         ("normal", m.get("normalTexture"))):
            if ref:
                yield i, key, doc["images"][doc["textures"][ref["index"]]["source"]]["uri"]


def main():
    from PIL import Image
    os.makedirs(DST, exist_ok=True)
    doc = json.load(open(os.path.join(SRC, "Sponza.gltf")))
    index = {i: {} for i in range(len(doc["materials"]))}
    for i, key, uri in _material_images(doc):
        im = Image.open(os.path.join(SRC, uri)).convert("RGB")
        if im.size[0] > SIZE:
            im = im.resize((SIZE, SIZE), Image.BOX)
        name = f"m{i:02d}_{key}.jpg"
        im.save(os.path.join(DST, name), quality=92)
        index[i][key] = name
    with open(os.path.join(DST, "materials.json"), "w") as fh:
        json.dump(index, fh, indent=1, sort_keys=True)
    print("wrote", len(os.listdir(DST)), "files to", DST)


def native(src: str = SRC, dst: str = NATIVE_DST) -> bool:
    """Copy the material images at their native resolution into `dst` (+ materials.json). No-op when `dst` is already
    complete; False when the reference's glTF directory is absent (e.g. on the GPU box)."""
    gltf = os.path.join(src, "Sponza.gltf")
    if not os.path.exists(gltf):
        return False
    doc = json.load(open(gltf))
    index = {i: {} for i in range(len(doc["materials"]))}
    for i, key, uri in _material_images(doc):
        index[i][key] = f"m{i:02d}_{key}{os.path.splitext(uri)[1].lower()}"
    idx_path = os.path.join(dst, "materials.json")
    want = json.dumps(index, indent=1, sort_keys=True)
    if os.path.exists(idx_path) and open(idx_path).read() == want and \
            all(os.path.exists(os.path.join(dst, n)) for e in index.values() for n in e.values()):
        return True
    os.makedirs(dst, exist_ok=True)
    for i, key, uri in _material_images(doc):
        shutil.copyfile(os.path.join(src, uri), os.path.join(dst, index[i][key]))
    with open(idx_path, "w") as fh:   # written last: its presence marks a complete set
        fh.write(want)
    return True


if __name__ == "__main__":
    if "--native" in sys.argv[1:]:
        print("native set:", native())
    else:
        main()
