"""Headless output: PNG writer (host, no GPU) and, on the GPU, framebuffer readback +
the per-frame GPU-metric JSON record with the reference's 12 group names (renderer.cpp:577-588)."""
import json

import numpy as np
import pytest
import torch

from helpers import SPONZA_CAMERA, globals_for
from soc_real_time_renderer_amd import raster, scene

GROUPS = ["Depth Prepass", "Composition", "Tone Mapping", "Bloom", "Depth Of Field", "Shadows", "Rendering G-Buffer",
          "Screen Space Reflections", "Ambient Occlusion", "Auto Exposure", "Sky Rendering", "Temporal Anti-Aliasing"]


@pytest.mark.parametrize("W,H", [(1, 1), (53, 37), (300, 220)])
def test_png_round_trip(soc, tmp_path, W, H):
    from PIL import Image
    img = np.random.default_rng(W).integers(0, 256, (H, W, 4)).astype(np.uint8)
    p = str(tmp_path / "f.png")
    soc.write_png(p, img)
    assert np.array_equal(np.array(Image.open(p)), img)


def test_png_rejects_bad_arguments(soc):
    with pytest.raises(soc.SocError):
        soc.write_png("/nonexistent-dir/x.png", np.zeros((2, 2, 4), np.uint8))


@pytest.mark.gpu
def test_framebuffer_and_metrics(soc, tmp_path):
    from PIL import Image
    W, H = 320, 180
    g = globals_for(W, H, camera=SPONZA_CAMERA, elapsed=10.0)
    sc = raster.scene_setup(g, scene.SPONZA_PROXY, tex_size=64)
    fr = soc.alloc_frame(W, H, "cuda", bloom_output=True)
    fr["noise"].copy_(torch.from_numpy(scene.noise_texture()))
    fr["shadow"] = torch.zeros((1024, 1024), dtype=torch.float32, device="cuda")
    vis = torch.zeros((H, W), dtype=torch.int64, device="cuda")
    r = soc.Renderer(fr, timing=True)
    r.set_raster_scene(sc["mesh"], sc["materials"], sc["material_count"], vis, sc["workspace"])
    for _ in range(2):
        r.execute(g)
    torch.cuda.synchronize()
    rec = json.loads(r.metrics_json(7))
    assert rec["frame"] == 7 and list(rec["groups"]) == GROUPS
    # a one-call frame folds the partial histograms in the resolve: the fold pass has no work, no record
    assert set(rec["passes"]) == set(r.pass_names()) - {"LuminanceHistogramFold"}
    assert rec["total_gpu_ms"] == pytest.approx(sum(rec["passes"].values()), rel=1e-4)
    assert rec["groups"]["Rendering G-Buffer"] > 0 and rec["groups"]["Screen Space Reflections"] == 0
    host = soc.read_image(fr["output"])
    assert np.array_equal(host, fr["output"].cpu().numpy())
    p = str(tmp_path / "frame.png")
    soc.write_png(p, host)
    assert np.array_equal(np.array(Image.open(p)), host)
    assert host[..., :3].std() > 1.0   # a rendered image, not a clear colour
    r.close()


def read_exr(path):
    """Minimal independent OpenEXR reader for the uncompressed scanline HALF files soc_write_exr writes."""
    import struct
    b = open(path, "rb").read()
    assert struct.unpack_from("<I", b, 0)[0] == 20000630 and b[4] == 2
    pos, attrs = 8, {}
    while b[pos] != 0:
        e = b.index(0, pos); name = b[pos:e].decode(); pos = e + 1
        e = b.index(0, pos); typ = b[pos:e].decode(); pos = e + 1
        n = struct.unpack_from("<i", b, pos)[0]; pos += 4
        attrs[name] = (typ, b[pos:pos + n]); pos += n
    pos += 1
    chans, v, p = [], attrs["channels"][1], 0
    while v[p] != 0:
        e = v.index(0, p); nm = v[p:e].decode(); p = e + 1
        assert struct.unpack_from("<i", v, p)[0] == 1        # HALF
        chans.append(nm); p += 16
    assert attrs["compression"][1] == b"\x00"
    x0, y0, x1, y1 = struct.unpack("<4i", attrs["dataWindow"][1])
    W, H = x1 - x0 + 1, y1 - y0 + 1
    offs = struct.unpack_from(f"<{H}Q", b, pos)
    img = np.zeros((H, W, 4), np.float16)
    for o in offs:
        y, n = struct.unpack_from("<ii", b, o)
        assert n == W * 2 * len(chans)
        row = np.frombuffer(b, np.float16, W * len(chans), o + 8).reshape(len(chans), W)
        for ci, nm in enumerate(chans):
            img[y, :, "RGBA".index(nm)] = row[ci]
    return chans, img


def test_write_exr_round_trip(soc, tmp_path):
    """soc_write_exr (f4's f16 framebuffer dump): a seeded RGBA16F image incl. HDR values, negatives, inf and NaN
    survives a write -> independent read bit-exact; sorted channel list; padded host rows accepted."""
    rng = np.random.default_rng(7)
    H, W = 13, 29
    a = (rng.standard_normal((H, W + 3, 4)) * 100).astype(np.float16)
    a[0, 0] = [np.inf, -np.inf, np.nan, 65504]
    view = a[:, :W]
    p = str(tmp_path / "f.exr")
    soc.write_exr(p, np.ascontiguousarray(view))
    chans, got = read_exr(p)
    assert chans == ["A", "B", "G", "R"]
    assert np.array_equal(got.view(np.uint16), np.ascontiguousarray(view).view(np.uint16))
    with pytest.raises(soc.SocError):
        soc.write_exr("/nonexistent-dir/x.exr", np.zeros((2, 2, 4), np.float16))
