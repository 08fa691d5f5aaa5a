"""Config C1 fixture: the reference's DamagedHelmet asset (assets/DamagedHelmet/glTF, data files) copied as
glTF JSON + .bin, and its baseColor / emissive / normal JPEGs decoded with Pillow and box-downsampled to 256^2
RGBA8 (tests/golden/damaged_helmet/textures_256.npz). Run in the container that has /root/reference."""
import os
import shutil
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from soc_real_time_renderer_amd.gltf import load_image  # noqa: E402

SRC = "/root/reference/assets/DamagedHelmet/glTF"
DST = os.path.join(ROOT, "tests", "golden", "damaged_helmet")
os.makedirs(DST, exist_ok=True)
for f in ("DamagedHelmet.gltf", "DamagedHelmet.bin"):
    shutil.copyfile(os.path.join(SRC, f), os.path.join(DST, f))
np.savez_compressed(os.path.join(DST, "textures_256.npz"),
                    **{name: load_image(os.path.join(SRC, name), 256) for name in ("Default_albedo.jpg", "Default_emissive.jpg", "Default_normal.jpg")})
print("wrote", sorted(os.listdir(DST)))
