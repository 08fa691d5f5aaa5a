"""Cross-check of the two independent CPU restatements of the reference GLSL.

oracle/soc_oracle.c (the checker every GPU parity test uses) against oracle/np_oracle.py (numpy, float64,
written from the GLSL without the C oracle's sampling contract or arithmetic order). A misreading of
/root/reference/src/graphics/tasks/*.inl in the C oracle -- which the HIP kernels, built to the C oracle's
contract, would share -- shows up here as a disagreement beyond the stated tolerances.

The numpy restatement samples with the Vulkan 8-bit sub-texel weight rule (np_oracle.SUBTEXEL_BITS = 8)
for the tight checks; `test_exact_weights_only_move_by_subtexel_rounding` shows that with exact float64
weights the only change is the sub-texel rounding. Tolerances (per output, stated in each test):

  bloom down/up, composition (RGBA16F)  |d| <= 1e-3 + 2e-3 |ref| on every channel
  TAA (RGBA16F)                          the same on >= 99.9 % of channels, max |d| <= 1e-2
  SSAO (R8)                              >= 99 % of pixels within 2/255; max = one tap flip (<= 11/255)
  SSAO blur (R8)                         within 1/255 (the /16 of float64 vs float32 sums at .5 ties)
  histogram bins                         identical on the fixtures; <= 0.1 % of pixels moved on scenes
  exposure                               |d| <= 1e-5 from the same bins
  tone map (RGBA8)                       within 1/255
  clouds (RGBA8)                         >= 99 % of channels within 2/255, max <= 16/255 (fp32 vs float64 over the
                                         24 x 10-step march through smoothstep(0.55, 0.6, noise): slope 20)
"""
import os

import numpy as np
import pytest

from conftest import ROOT

import np_oracle as npo  # noqa: E402

GOLDEN = [os.path.join(ROOT, "tests", "golden", f) for f in ("frame_64x36.npz", "frame_97x55.npz")]


@pytest.fixture(autouse=True)
def _subtexel8():
    old = npo.SUBTEXEL_BITS
    npo.SUBTEXEL_BITS = 8
    yield
    npo.SUBTEXEL_BITS = old


def _load(path, soc):
    d = np.load(path)
    g = soc.Globals.from_buffer_copy(d["in_globals"].tobytes())
    return d, g


def f16_ok(a, ref, frac=1.0, max_abs=None):
    a = np.asarray(a, np.float64)
    ref = np.asarray(ref, np.float64)
    d = np.abs(a - ref)
    ok = d <= 1e-3 + 2e-3 * np.abs(ref)
    assert ok.mean() >= frac, f"{(~ok).sum()} channels out of tolerance, max |d| {d.max()}"
    if max_abs is not None:
        assert d.max() <= max_abs, d.max()


def u8_diff(a, b):
    return np.abs(a.astype(np.int32) - b.astype(np.int32))


@pytest.mark.parametrize("path", GOLDEN, ids=["64x36", "97x55"])
def test_bloom(path, soc):
    d, g = _load(path, soc)
    H, W = d["in_depth"].shape
    f16_ok(npo.bloom_downsample(d["in_emissive"], (H // 2, W // 2)), d["out_bloom_down_half"][..., :3])
    f16_ok(npo.bloom_downsample(d["in_emissive"], (H, W)), d["out_bloom_down_same"][..., :3])
    f16_ok(npo.bloom_upsample(d["out_bloom_down_half"], (H, W)), d["out_bloom_up_double"][..., :3])


@pytest.mark.parametrize("path", GOLDEN, ids=["64x36", "97x55"])
def test_composition(path, soc):
    d, g = _load(path, soc)
    out = npo.composition(g, d["in_albedo"], d["in_emissive"], d["in_normal"], d["in_depth"], d["in_ssao_in"],
                          d["in_shadow"], d["in_clouds_in"])
    f16_ok(out, d["out_composition"])


@pytest.mark.parametrize("path", GOLDEN, ids=["64x36", "97x55"])
def test_ssao_and_blur(path, soc):
    d, g = _load(path, soc)
    H, W = d["in_depth"].shape
    diff = u8_diff(npo.ssao_generation(g, d["in_depth"], d["in_normal"], (H // 2, W // 2)), d["out_ssao"])
    assert (diff <= 2).mean() >= 0.99 and diff.max() <= 11, (diff > 2).mean()
    assert u8_diff(npo.ssao_blur(d["in_ssao_in"]), d["out_ssao_blur"]).max() <= 1


@pytest.mark.parametrize("path", GOLDEN, ids=["64x36", "97x55"])
def test_taa(path, soc):
    d, g = _load(path, soc)
    out = npo.temporal_antialiasing(g, d["in_color_in"], d["in_prev_in"], d["in_velocity"], d["in_velocity"],
                                    d["in_depth"])
    f16_ok(out, d["out_taa"], frac=0.999, max_abs=1e-2)


@pytest.mark.parametrize("path", GOLDEN, ids=["64x36", "97x55"])
def test_histogram_resolve_tonemap(path, soc):
    d, g = _load(path, soc)
    bins = npo.generate_luminance_histogram(g, d["in_color_in"])
    assert np.array_equal(bins, d["out_histogram"].astype(np.uint64))
    assert abs(npo.resolve_luminance_histogram(g, d["out_histogram"], 0.0) - float(d["out_exposure"][0])) <= 1e-5
    assert u8_diff(npo.tone_mapping(g, d["in_color_in"], -0.5), d["out_tonemap"]).max() <= 1


@pytest.mark.parametrize("path", GOLDEN, ids=["64x36", "97x55"])
def test_clouds(path, soc):
    d, g = _load(path, soc)
    diff = u8_diff(npo.cloud_rendering(g, d["in_depth"], d["in_noise"]), d["out_clouds"])
    assert (diff <= 2).mean() >= 0.99 and diff.max() <= 16, ((diff > 2).mean(), diff.max())


def test_exact_weights_only_move_by_subtexel_rounding(soc):
    """With exact float64 filter weights the TAA (history taps at arbitrary sub-texel positions) moves by at most
    half a 1/256 weight step times the local colour range (colours in [0, 5]: 5/512 ~ 0.01)."""
    d, g = _load(GOLDEN[0], soc)
    npo.SUBTEXEL_BITS = None
    out = npo.temporal_antialiasing(g, d["in_color_in"], d["in_prev_in"], d["in_velocity"], d["in_velocity"],
                                    d["in_depth"])
    diff = np.abs(out.astype(np.float64) - d["out_taa"].astype(np.float64))
    assert diff.max() <= 5.0 / 512 * 1.3


@pytest.mark.parametrize("scene_name", ["sponza", "terrain"])
def test_scene_frame_passes(scene_name, soc, oracle):
    """The realistic G-buffers (Sponza-proxy, C4 terrain) through both restatements, pass by pass: each pass of the
    numpy restatement gets the C oracle's inputs, so differences do not compound."""
    from helpers import sponza_inputs, terrain_inputs
    W, H = 96, 54
    g, gb = (sponza_inputs if scene_name == "sponza" else terrain_inputs)(W, H, shadow_size=256, elapsed=10.0,
                                                                          frame_counter=2)
    ssao = np.zeros((H // 2, W // 2), np.uint8)
    oracle.ssao_generation(g, gb["depth"], gb["normal"], ssao)
    diff = u8_diff(npo.ssao_generation(g, gb["depth"], gb["normal"], (H // 2, W // 2)), ssao)
    assert (diff <= 2).mean() >= 0.99 and diff.max() <= 11, ((diff > 2).mean(), diff.max())
    blur = np.zeros_like(ssao)
    oracle.ssao_blur(g, ssao, blur)
    assert u8_diff(npo.ssao_blur(ssao), blur).max() <= 1
    clouds = np.zeros((H, W, 4), np.uint8)
    oracle.cloud_rendering(g, gb["depth"], gb["noise"], clouds)
    diff = u8_diff(npo.cloud_rendering(g, gb["depth"], gb["noise"]), clouds)
    assert (diff <= 2).mean() >= 0.99 and diff.max() <= 16, ((diff > 2).mean(), diff.max())
    color = np.zeros((H, W, 4), np.float16)
    oracle.composition(g, color, gb["albedo"], gb["emissive"], gb["normal"], gb["depth"], blur, gb["shadow"], clouds)
    f16_ok(npo.composition(g, gb["albedo"], gb["emissive"], gb["normal"], gb["depth"], blur, gb["shadow"], clouds),
           color)
    ae = soc.AutoExposure()
    oracle.generate_luminance_histogram(g, color, ae)
    ref_bins = np.array(ae.histogram_buckets, np.int64)
    bins = npo.generate_luminance_histogram(g, color).astype(np.int64)
    assert np.abs(bins - ref_bins).sum() <= 2 * max(1, int(0.001 * W * H))
    oracle.resolve_luminance_histogram(g, ae)
    assert abs(npo.resolve_luminance_histogram(g, ref_bins, 0.0) - ae.exposure) <= 1e-5
    taa = np.zeros((H, W, 4), np.float16)
    prev = color[:, ::-1].copy()
    oracle.temporal_antialiasing(g, taa, color, prev, gb["velocity"], gb["velocity"], gb["depth"])
    f16_ok(npo.temporal_antialiasing(g, color, prev, gb["velocity"], gb["velocity"], gb["depth"]), taa,
           frac=0.999, max_abs=1e-2)
    tm = np.zeros((H, W, 4), np.uint8)
    oracle.tone_mapping(g, taa, ae, tm)
    assert u8_diff(npo.tone_mapping(g, taa, ae.exposure), tm).max() <= 1


def test_composition_with_lights(soc, oracle):
    """Composition with point and spot lights (calculate_point_light / calculate_spot_light,
    composition.inl:124-160): the light loops of both restatements."""
    from helpers import sponza_inputs
    W, H = 96, 54
    g, gb = sponza_inputs(W, H, shadow_size=256, elapsed=10.0, frame_counter=2)
    rng = np.random.default_rng(7)
    g.point_light_count = 5
    for i in range(5):
        L = g.point_lights[i]
        L.position[:] = [float(-14 + rng.uniform(-3, 8)), float(rng.uniform(0.5, 4)), float(rng.uniform(-3, 3))]
        L.color[:] = [float(c) for c in rng.uniform(0.2, 1.0, 3)]
        L.intensity = float(rng.uniform(0.5, 3.0))
    g.spot_light_count = 2
    for i in range(2):
        L = g.spot_lights[i]
        L.position[:] = [float(-12 + 3 * i), 3.0, 0.5]
        L.direction[:] = [0.3, -1.0, 0.1 * i]
        L.color[:] = [1.0, 0.9, 0.7]
        L.intensity = 2.0
        L.cut_off, L.outer_cut_off = float(np.cos(np.radians(20.0))), float(np.cos(np.radians(30.0)))
    ssao = np.full((H // 2, W // 2), 200, np.uint8)
    clouds = np.full((H, W, 4), 90, np.uint8)
    color = np.zeros((H, W, 4), np.float16)
    oracle.composition(g, color, gb["albedo"], gb["emissive"], gb["normal"], gb["depth"], ssao, gb["shadow"], clouds)
    f16_ok(npo.composition(g, gb["albedo"], gb["emissive"], gb["normal"], gb["depth"], ssao, gb["shadow"], clouds),
           color, frac=0.999)
