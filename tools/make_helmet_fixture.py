"""Config C1 fixtures of the reference's DamagedHelmet asset (assets/DamagedHelmet/glTF, data files), made in the
container that has /root/reference:

- the committed fixture (tests/golden/damaged_helmet/): glTF JSON + .bin copied, and its baseColor / emissive /
  normal JPEGs decoded with Pillow and box-downsampled to 256^2 RGBA8 (textures_256.npz)
  (`python tools/make_helmet_fixture.py`);
- the native-resolution images (tests/golden/damaged_helmet/native/: the three 2048^2 JPEGs byte for byte,
  git-ignored, shipped to the GPU box with the built libraries), written by __graft_entry__.build() through
  `native()` (`python tools/make_helmet_fixture.py --native`)."""
import os
import shutil
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = "/root/reference/assets/DamagedHelmet/glTF"
DST = os.path.join(ROOT, "tests", "golden", "damaged_helmet")
IMAGES = ("Default_albedo.jpg", "Default_emissive.jpg", "Default_normal.jpg")


def main():
    sys.path.insert(0, ROOT)
    from soc_real_time_renderer_amd.gltf import load_image
    os.makedirs(DST, exist_ok=True)
    for f in ("DamagedHelmet.gltf", "DamagedHelmet.bin"):
        shutil.copyfile(os.path.join(SRC, f), os.path.join(DST, f))
    np.savez_compressed(os.path.join(DST, "textures_256.npz"),
                        **{name: load_image(os.path.join(SRC, name), 256) for name in IMAGES})
    print("wrote", sorted(os.listdir(DST)))


def native(src: str = SRC, dst: str = os.path.join(DST, "native")) -> bool:
    """Copy the three material images at their native 2048^2 into `dst`; False when the reference is absent."""
    if not all(os.path.exists(os.path.join(src, n)) for n in IMAGES):
        return False
    os.makedirs(dst, exist_ok=True)
    for n in IMAGES:
        out = os.path.join(dst, n)
        if not os.path.exists(out) or os.path.getsize(out) != os.path.getsize(os.path.join(src, n)):
            shutil.copyfile(os.path.join(src, n), out)
    return True


if __name__ == "__main__":
    if "--native" in sys.argv[1:]:
        print("native images:", native())
    else:
        main()
