"""Known-answer tests pinning the CPU oracle to the reference's formulas (CPU only).

The reference ships no tests or golden vectors, so these KATs are derived by hand or in
float64 numpy from the reference source lines cited in each test.
"""
import ctypes as C
import math

import numpy as np
import pytest

from helpers import globals_for


# ------------------------------------------------------------------------------------------------ globals feed
def test_default_globals(soc):
    """renderer.cpp:72-133 defaults, incl. the inverted log-luminance range (quirk Q9)."""
    g = soc.globals_defaults(3840, 2160)
    assert g.ssao_bias == pytest.approx(0.025) and g.ssao_radius == pytest.approx(0.3) and g.ssao_kernel_size == 26
    assert list(g.ambient) == pytest.approx([0.1, 0.1, 0.1])
    assert g.ambient_occlussion_strength == pytest.approx(1.2) and g.emissive_bloom_strength == pytest.approx(2.0)
    assert g.log_min_luminance == pytest.approx(math.log2(0.214 / 2 ** -15), abs=1e-5)   # 12.77568
    assert g.log_max_luminance == pytest.approx(math.log2(0.214 / 2 ** 15), abs=1e-5)    # -17.22432
    assert (g.saturation, g.agxDs_linear_section, g.peak) == pytest.approx((1.0, 0.18, 1.0))
    assert g.compression == pytest.approx(0.15)
    assert g.sun_info.exponential_factor == -80.0 and g.sun_info.darkening_factor == 1.0
    d = np.array(g.sun_info.direction)
    assert d == pytest.approx([0.0, -math.cos(math.radians(4)), -math.sin(math.radians(4))], abs=1e-7)
    assert list(g.resolution) == [3840, 2160]


def np_mat(a):
    return np.array(a, np.float64).reshape(4, 4).T   # column-major float[16] -> row-major matrix


def test_glm_restatements(soc):
    lib = soc.lib()
    F16 = C.c_float * 16
    out = F16()
    lib.soc_mat4_perspective_rh_no(out, math.radians(90.0), 16 / 9, 0.1, 1000.0)
    P = np_mat(out)
    f = 1.0 / math.tan(math.radians(45.0))
    ref = np.array([[f / (16 / 9), 0, 0, 0], [0, f, 0, 0], [0, 0, -(1000.1) / 999.9, -2 * 1000 * 0.1 / 999.9],
                    [0, 0, -1, 0]])
    assert P == pytest.approx(ref, rel=1e-6, abs=1e-7)
    lib.soc_mat4_ortho_rh_no(out, -16, 16, -16, 16, -16, 16)
    O = np_mat(out)
    assert O == pytest.approx(np.diag([1 / 16, 1 / 16, -1 / 16, 1.0]), abs=1e-8)
    eye, ctr, up = (C.c_float * 3)(1, 2, 3), (C.c_float * 3)(4, 2, -1), (C.c_float * 3)(0, 1, 0)
    lib.soc_mat4_look_at_rh(out, eye, ctr, up)
    V = np_mat(out)
    fw = np.array([3, 0, -4], float) / 5
    s = np.cross(fw, [0, 1, 0]); s /= np.linalg.norm(s)
    u = np.cross(s, fw)
    refv = np.eye(4)
    refv[0, :3], refv[1, :3], refv[2, :3] = s, u, -fw
    refv[:3, 3] = [-s @ [1, 2, 3], -u @ [1, 2, 3], fw @ [1, 2, 3]]
    assert V == pytest.approx(refv, abs=1e-6)
    rng = np.random.default_rng(0)
    M = rng.normal(size=(4, 4)) + 4 * np.eye(4)
    src = F16(*M.T.reshape(-1).astype(np.float32))
    lib.soc_mat4_inverse(out, src)
    assert np_mat(out) == pytest.approx(np.linalg.inv(M.astype(np.float32).astype(np.float64)), rel=1e-4, abs=1e-5)


def test_jitter_sequence(soc):
    """R2 jitter, period 32, scaled by 1/W and 1/H and added to proj[3][0..1] (application.cpp:113-131)."""
    W, H = 1920, 1080
    g = soc.globals_defaults(W, H)
    cam = soc.make_camera((0, 1, 0))
    ji = C.c_uint32(0)
    a1, a2 = 1 / 1.32471795724474602596, 1 / 1.32471795724474602596 ** 2
    for i in range(40):
        soc.frame_update(g, cam, W, H, 0.016, ji)
        k = i % 32
        jx = ((0.5 + a1 * (k + 1)) % 1.0 - 0.5) / W
        jy = ((0.5 + a2 * (k + 1)) % 1.0 - 0.5) / H
        assert g.jitter[0] == pytest.approx(jx, abs=2e-7) and g.jitter[1] == pytest.approx(jy, abs=2e-7)
        assert g.camera_projection_matrix[12] == pytest.approx(g.jitter[0], abs=1e-9)
        assert g.camera_projection_matrix[5] < 0          # Y flip, camera.cpp:9
    assert g.frame_counter == 40 and g.elapsed_time == pytest.approx(40 * 0.016, rel=1e-5)


# ------------------------------------------------------------------------------------------------ numerics helpers
def test_f16_conversion_matches_numpy(oracle):
    rng = np.random.default_rng(1)
    vals = np.concatenate([rng.normal(0, 100, 4000), rng.normal(0, 1e-5, 2000), [65504, 65519.99, 65520, 70000, -0.0,
                                                                                   6.1e-5, 5.96e-8, 2.98e-8, 1e-9]]
                          ).astype(np.float32)
    for v in vals:
        assert oracle.lib().soc_oracle_f32_to_f16(float(v)) == np.float16(v).view(np.uint16), v
    for h in range(0, 65536, 97):
        a = oracle.lib().soc_oracle_f16_to_f32(h)
        b = float(np.uint16(h).view(np.float16))
        assert (math.isnan(a) and math.isnan(b)) or a == b


def test_deterministic_log2_accuracy(oracle):
    rng = np.random.default_rng(2)
    xs = np.concatenate([np.exp(rng.uniform(-80, 80, 20000)), [1.0, 2.0, 0.5, 1e-40, 3.4e38, 1.4142135]]).astype(np.float32)
    for x in xs[:5000]:
        got = oracle.log2(float(x))
        ref = math.log2(float(x))
        assert abs(got - ref) <= 4e-7 * max(1.0, abs(ref)), (x, got, ref)
    assert oracle.log2(0.0) == -math.inf
    assert math.isnan(oracle.log2(float("nan")))


def test_deterministic_noise_functions_correctly_rounded(oracle):
    """Quirk Q8: the SSAO hash's sin / cos / pow (soc_oracle.c det_sin / det_cos / det_pow, restated operation for
    operation by ssao.hip's random-vector table) against float64 numpy rounded to float32: correctly rounded on every
    sampled argument, over the hash's range (sin of |a| <= ~1e5, the noise's cos(pi x), pow(uv, 1.1) and
    pow(4.2 W, 1.5 + u / 10)); the GPU table equals these bits (GPU suite, frame_parity hash_differs = 0)."""
    L = oracle.lib()
    rng = np.random.default_rng(8)
    f32 = np.float32
    xs = np.concatenate([rng.uniform(-1.2e5, 1.2e5, 4000), rng.uniform(-8, 8, 2000), [0.0, -0.0, 1e-30, 3.1415927]]).astype(f32)
    for x in xs:
        assert L.soc_oracle_det_sin(float(x)) == f32(np.sin(np.float64(x))), x
        assert L.soc_oracle_det_cos(float(x)) == f32(np.cos(np.float64(x))), x
    for x, y in zip(rng.uniform(1e-4, 1.0, 3000).astype(f32), rng.uniform(1.0, 1.7, 3000).astype(f32)):
        assert L.soc_oracle_det_pow(float(x), float(y)) == f32(np.float64(x) ** np.float64(y)), (x, y)
    for w in (64, 512, 960, 1920, 2048, 3840, 8192):
        for u in (0.0001, 0.25, 0.5, 0.999):
            x, y = f32(w * 4.2), f32(f32(1.5) + f32(u) / f32(10.0))
            assert L.soc_oracle_det_pow(float(x), float(y)) == f32(np.float64(x) ** np.float64(y)), (w, u)
    assert L.soc_oracle_det_pow(1.0, 1.1) == 1.0


# ------------------------------------------------------------------------------------------------ histogram (Q9)
def test_luminance_bins_known_answers(soc, oracle):
    g = soc.globals_defaults(64, 64)
    lmin, lmax = g.log_min_luminance, g.log_max_luminance
    b = lambda L: oracle.luminance_bin(L, L, L, lmin, lmax)  # grey: luminance = L*(0.2126+0.7152+0.0722)
    assert oracle.luminance_bin(1.0, 1.0, 1.0, lmin, lmax) == 109      # survey §8a Q9
    assert oracle.luminance_bin(1e-3, 1e-3, 1e-3, lmin, lmax) == 193
    assert b(0.0) == 255                                                   # black -> +inf -> bin 255
    assert b(1e-4) == 255                                                  # below 1e-3 -> 0 -> bin 255
    assert b(1e5) == 0                                                     # super bright -> negative -> 0
    assert oracle.luminance_bin(float("nan"), 0, 0, lmin, lmax) == 0       # NaN -> i32 0
    assert oracle.luminance_bin(float("inf"), 0, 0, lmin, lmax) == 0
    # float64 restatement away from bin boundaries
    rng = np.random.default_rng(3)
    for L in np.exp(rng.uniform(-6, 9, 3000)):
        r = float(np.float32(L))
        lum = float(np.float32(np.float32(r) * np.float32(0.2126) + np.float32(r) * np.float32(0.7152)
                               + np.float32(r) * np.float32(0.0722)))
        if lum < 1e-3:
            continue
        mapped = (math.log2(lum) - lmin) / (lmax - lmin) * 254 + 1
        if abs(mapped - round(mapped)) < 1e-3:
            continue
        assert oracle.luminance_bin(r, r, r, lmin, lmax) == min(255, max(0, int(mapped))), L


def test_histogram_counts_and_resolve_formula(soc, oracle):
    W, H = 32, 16
    g = soc.globals_defaults(W, H)
    g.delta_time = 0.016
    img = np.ones((H, W, 4), np.float16)          # luminance 1.0 -> bin 109
    img[:4] = 0                                    # 128 black px -> bin 255
    ae = soc.AutoExposure()
    oracle.generate_luminance_histogram(g, img, ae)
    bins = np.array(ae.histogram_buckets)
    assert bins[109] == W * H - 128 and bins[255] == 128 and bins.sum() == W * H
    # resolve_luminance_histogram.inl:58-79 in float64
    s = 109 * (W * H - 128) + 255 * 128
    x = s / max(W * H - bins[0], 1)
    log2_mean = (x - 1) / 255 * (g.log_max_luminance - g.log_min_luminance) + g.log_min_luminance
    target = math.log2(g.target_luminance / 2 ** log2_mean)
    alpha = 1 - math.exp(-0.016)
    oracle.resolve_luminance_histogram(g, ae)
    assert ae.exposure == pytest.approx(alpha * target, abs=1e-5)
    assert sum(ae.histogram_buckets) == 0          # resolve clears the bins


def test_resolve_u32_wrap_vs_wide(soc, oracle):
    """u32 weighted sum wraps like the reference; the multi-GPU wide accumulator does not (§8e)."""
    g = soc.globals_defaults(64, 64)
    g.delta_time = 0.5
    ae1, ae2 = soc.AutoExposure(), soc.AutoExposure()
    for ae in (ae1, ae2):
        ae.histogram_buckets[200] = 40_000_000      # 200 * 4e7 = 8e9 > 2^32
    oracle.resolve_luminance_histogram(g, ae1, total_pixels=40_000_000, wide=False)
    oracle.resolve_luminance_histogram(g, ae2, total_pixels=40_000_000, wide=True)
    assert ae1.exposure != ae2.exposure


# ------------------------------------------------------------------------------------------------ passes
def test_bloom_weights_preserve_constants(soc, oracle):
    g = soc.globals_defaults(64, 36)
    src = np.full((36, 64, 4), 0.5, np.float16)
    for dst_shape in [(36, 64), (18, 32), (9, 16), (7, 11)]:
        dst = np.zeros(dst_shape + (4,), np.float16)
        oracle.bloom_downsample(g, src, dst)
        assert (dst[..., :3] == 0.5).all()
        up = np.zeros((36, 64, 4), np.float16)
        oracle.bloom_upsample(g, dst, up)
        assert (up[..., :3] == 0.5).all() and (up[..., 3] == 1.0).all()


def test_bloom_downsample_point_taps(soc, oracle):
    """Same-size downsample (emissive -> mip0): a single bright texel spreads with the 13-tap weights."""
    g = soc.globals_defaults(16, 16)
    src = np.zeros((16, 16, 4), np.float16)
    src[8, 8, :3] = 1.0
    dst = np.zeros_like(src)
    oracle.bloom_downsample(g, src, dst)
    d = dst[..., 0].astype(np.float32)
    assert d[8, 8] == 0.125                              # e
    assert d[8, 10] == 0.0625 and d[6, 8] == 0.0625      # b/d/f/h (texel at +-2)
    assert d[10, 10] == 0.03125                          # a/c/g/i
    assert d[9, 9] == 0.125 and d[7, 7] == 0.125         # j/k/l/m
    assert d.sum() == pytest.approx(1.0)


def test_ssao_blur_box(soc, oracle):
    g = soc.globals_defaults(32, 32)
    src = np.zeros((16, 16), np.uint8)
    src[8, 8] = 255
    dst = np.zeros_like(src)
    oracle.ssao_blur(g, src, dst)
    # taps -2..+1: pixel (x, y) sees (8, 8) when x-2 <= 8 <= x+1, i.e. x in 7..10
    nz = np.argwhere(dst > 0)
    assert set(map(tuple, nz)) == {(y, x) for y in range(7, 11) for x in range(7, 11)}
    assert (dst[7:11, 7:11] == 16).all()                 # rint(255/16/255*255) = 16


def test_composition_known_pixel(soc, oracle):
    """Non-sky pixel with shadow z > 1 (sun fully dark): (ambient*albedo)*ao^1.2 + 2*emissive."""
    W, H = 8, 8
    g = soc.globals_defaults(W, H)
    cam = soc.make_camera((0, 1, 0))
    soc.frame_update(g, cam, W, H, 0.016, C.c_uint32(0))
    depth = np.full((H, W), 0.95, np.float32)
    depth[0, 0] = 1.0
    albedo = np.full((H, W, 4), 0.5, np.float16)
    emis = np.full((H, W, 4), 0.25, np.float16)
    normal = np.zeros((H, W, 4), np.float16); normal[..., 1] = 1
    ssao = np.full((H // 2, W // 2), 128, np.uint8)
    shadow = np.full((16, 16), 1.0, np.float32)
    clouds = np.full((H, W, 4), 200, np.uint8)
    out = np.zeros((H, W, 4), np.float16)
    oracle.composition(g, out, albedo, emis, normal, depth, ssao, shadow, clouds)
    ao = (128 / 255) ** 1.2
    # sun term: world pos is ~y<=1, sun-space z ~ (40-1)/16 > 1 -> exp(-80*(z-1)) ~ 0
    expected = 0.1 * 0.5 * ao + 0.5
    assert float(out[4, 4, 0]) == pytest.approx(expected, abs=2e-3)
    assert float(out[0, 0, 0]) == pytest.approx(200 / 255, abs=1e-3)      # sky -> clouds texel
    assert (out[..., 3] == 1.0).all()


def test_taa_uses_plus_x_neighbour(soc, oracle):
    """Quirk Q7: the 'current colour' is neighbors[5] = the (+1, 0) texel; frame 0 -> accum 0."""
    W, H = 16, 8
    g = globals_for(W, H, frames=1)
    g.frame_counter = 5                     # accum = min(0.1, 5) = 0.1
    cur = np.full((H, W, 4), 0.25, np.float16)
    cur[4, 9] = 1.0                          # the +x neighbour of (4, 8)
    prev = cur.copy()
    prev[4, 8] = 0.5
    vel = np.zeros((H, W, 4), np.float16)
    depth = np.full((H, W), 0.9, np.float32)
    out = np.zeros_like(cur)
    oracle.temporal_antialiasing(g, out, cur, prev, vel, vel, depth)
    # colour = 1.0 (from x+1); history clamped to [min,max] of the 3x3 = [0.25, 1.0] -> 0.5
    assert float(out[4, 8, 0]) == pytest.approx(0.1 * 1.0 + 0.9 * 0.5, abs=1e-3)


def np_agx(rgb, exposure, compression=0.15, linear=0.18, peak=1.0, sat=1.0):
    def unproj(xy):
        x, y = xy
        return np.array([x / y, 1.0, (1 - x - y) / y])

    def prim(r, gg, b, w):
        R, G, B, Wt = map(unproj, (r, gg, b, w))
        temp = np.column_stack([[R[0], 1, R[2]], [G[0], 1, G[2]], [B[0], 1, B[2]]])
        s = np.linalg.inv(temp) @ Wt
        return np.column_stack([R * s[0], G * s[1], B * s[2]])
    xr, xg, xb, xw = (0.64, 0.33), (0.3, 0.6), (0.15, 0.06), (0.3127, 0.3290)
    sf = 1 / (1 - compression)
    mix = lambda a, b: tuple(np.array(a) * (1 - sf) + np.array(b) * sf)
    s2x = prim(xr, xg, xb, xw)
    a2x = prim(mix(xw, xr), mix(xw, xg), mix(xw, xb), xw)
    M = s2x @ np.linalg.inv(a2x)
    w = np.maximum(rgb, 0) * 2.0 ** exposure
    w = M @ w
    S = peak * linear
    C_ = peak / (peak - S)
    w = np.where(w < S, w, peak - (peak - S) * np.exp(-C_ * (w - S) / peak))
    w = np.clip(w, 0, 1)
    d = w @ np.array([0.2126729, 0.7151522, 0.0721750])
    w = np.clip(d * (1 - sat) + w * sat, 0, 1)
    return np.linalg.inv(M) @ w


def test_tone_mapping_matches_float64_agx(soc, oracle):
    g = soc.globals_defaults(4, 4)
    rng = np.random.default_rng(9)
    img = rng.uniform(0, 4, (4, 4, 4)).astype(np.float16)
    ae = soc.AutoExposure()
    ae.exposure = -0.7
    out = np.zeros((4, 4, 4), np.float32)
    oracle.tone_mapping(g, img, ae, out, soc.FMT_RGBA32F)
    for y in range(4):
        for x in range(4):
            ref = np_agx(img[y, x, :3].astype(np.float64), -0.7)
            assert out[y, x, :3] == pytest.approx(ref, abs=2e-5)


def test_clouds_non_sky_constant(soc, oracle):
    W, H = 32, 16
    g = globals_for(W, H)
    depth = np.full((H, W), 0.5, np.float32)
    noise = np.zeros((64, 64, 4), np.uint8)
    out = np.zeros((H, W, 4), np.uint8)
    oracle.cloud_rendering(g, depth, noise, out)
    assert (out[..., :3] == np.array([51, 102, 255])).all() and (out[..., 3] == 255).all()
