"""The clouds noise bilinear's float form (clouds.hip: bilerp_wide / bilerp_rows, round 6) against the integer form
(quad_bilerp_u, v_dot2_u32_u16): the f16 table entries 256 c0 and c1 - c0 are exact, and every product and partial sum
of the fp32 evaluation is an integer (or an integer / 256) below 2^24, so the float form is the integer bilinear / 256
bit for bit. CPU only: numpy fp32 arithmetic on the same operations (no rounding occurs in either)."""
import numpy as np


def _integer_form(c0, c1, c2, c3, wx, wy):
    top = c0 * (256 - wx) + c1 * wx          # v_dot2_u32_u16 of (c0, c1) with (256 - wx, wx)
    bot = c2 * (256 - wx) + c3 * wx
    return top * (256 - wy) + bot * wy       # 65536 x 255 x the bilinear at most: < 2^24


def _float_form(c0, c1, c2, c3, wx, wy):
    f16 = np.float16
    e0, d01 = f16(256 * c0).astype(np.float32), f16(c1 - c0).astype(np.float32)   # the table's f16 pairs
    e2, d23 = f16(256 * c2).astype(np.float32), f16(c3 - c2).astype(np.float32)
    wxf, wys = wx.astype(np.float32), wy.astype(np.float32) * np.float32(1.0 / 256.0)
    top = d01 * wxf + e0                     # v_fma_mix_f32: exact, so the fp32 product-then-sum is the same value
    bot = d23 * wxf + e2
    return (bot - top) * wys + top           # = the integer form / 256


def test_table_entries_exact_in_f16():
    c = np.arange(256, dtype=np.int64)
    assert (np.float16(256 * c).astype(np.int64) == 256 * c).all()
    d = np.arange(-255, 256, dtype=np.int64)
    assert (np.float16(d).astype(np.int64) == d).all()


def test_row_stage_exhaustive():
    # every (c0, c1, wx): top = 256 c0 + (c1 - c0) wx, in fp32, equals the integer row sum
    c0, c1, wx = np.meshgrid(np.arange(256), np.arange(256), np.arange(256), indexing="ij")
    c0, c1, wx = c0.ravel().astype(np.int64), c1.ravel().astype(np.int64), wx.ravel().astype(np.int64)
    top_f = np.float16(c1 - c0).astype(np.float32) * wx.astype(np.float32) + np.float16(256 * c0).astype(np.float32)
    assert (top_f.astype(np.int64) == c0 * (256 - wx) + c1 * wx).all()
    assert (top_f == np.round(top_f)).all()


def test_bilinear_random_and_corners():
    rng = np.random.default_rng(7)
    n = 2_000_000
    c = rng.integers(0, 256, size=(4, n))
    wx, wy = rng.integers(0, 256, size=n), rng.integers(0, 256, size=n)
    # the extremes: all-0 / all-255 texels, opposite corners, zero and full weights
    ext = np.array([[0, 255, 0, 255, 255, 0], [255, 0, 255, 0, 255, 0], [0, 255, 255, 0, 0, 255], [255, 0, 0, 255, 0, 255]])
    c = np.concatenate([c, np.repeat(ext, 4, axis=1)], axis=1)
    wx = np.concatenate([wx, np.tile([0, 255, 0, 255], 6)])
    wy = np.concatenate([wy, np.tile([0, 0, 255, 255], 6)])
    ref = _integer_form(*c, wx, wy)
    got = _float_form(*c, wx, wy)
    assert (got.astype(np.float64) * 256.0 == ref.astype(np.float64)).all()


def _fma32(x, y, z):
    # fp32 fma via float64: the product of two fp32 values and its sum with an integer below 2^24 are exact in float64
    # here, so one rounding to fp32 is the fused result
    return (x.astype(np.float64) * y.astype(np.float64) + z.astype(np.float64)).astype(np.float32)


def test_z_lerp_and_octave_constants_scale_exactly():
    """noise3's z lerp fma(f, b - a, a) on the float form's values (a / 256, b / 256) is the integer form's result / 256,
    and the octave constants x 256 (NoiseScale) give the same products: scaling by 2^8 commutes with every rounding."""
    rng = np.random.default_rng(11)
    n = 1_000_000
    a = rng.integers(0, 255 * 65536, size=n).astype(np.float32)
    b = rng.integers(0, 255 * 65536, size=n).astype(np.float32)
    f = rng.random(n, dtype=np.float32)
    whole = _fma32(f, b - a, a)
    scaled = _fma32(f, (b - a) / np.float32(256), a / np.float32(256))
    assert (scaled * np.float32(256) == whole).all()
    k = np.float32(1.0 / (255.0 * 65536.0))   # kNoiseNorm
    for w in (0.5, 0.25, 0.125, 0.0625):
        c = np.float32(w) * k
        assert ((whole * c) == ((whole / np.float32(256)) * (c * np.float32(256)))).all()
