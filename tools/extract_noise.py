"""Decode the reference's clouds noise texture (assets/Clouds/noise.png, 64x64 8-bit grey; loaded as
R8G8B8A8_UNORM by src/graphics/renderer.cpp:152) into a raw 4096-byte fixture the GPU box can read
(the reference mount does not exist there). Run in the build container only."""
import sys

import numpy as np
from PIL import Image

src = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/assets/Clouds/noise.png"
dst = sys.argv[2] if len(sys.argv) > 2 else "soc_real_time_renderer_amd/data/clouds_noise_64x64.u8"
im = Image.open(src)
print(im.mode, im.size)
a = np.asarray(im.convert("RGBA"))
assert a.shape == (64, 64, 4)
assert (a[..., 0] == a[..., 1]).all() and (a[..., 0] == a[..., 2]).all(), "expected grey"
a[..., 0].astype(np.uint8).tofile(dst)
print("wrote", dst, a[..., 0].mean(), a[..., 0].min(), a[..., 0].max())
