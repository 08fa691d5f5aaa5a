"""np_oracle — a second, independent restatement of the screen-space passes in numpy (TEST INFRASTRUCTURE).

Written directly from the reference GLSL (/root/reference/src/graphics/tasks/*.inl, cited per function),
NOT from oracle/soc_oracle.c: it shares no code, no sampling contract and no arithmetic order with it.
Its purpose is to catch a misreading of the GLSL that the C oracle and the HIP kernels would share
(both follow the C oracle's contract). Differences by construction, which the cross-check tolerances
(tests/test_np_oracle.py) absorb:

* float64 everywhere the GLSL leaves the precision to the implementation (matrix products, dot,
  normalize, transcendentals); fp32 only where the GLSL's own fp32 rounding IS the result (the SSAO
  noise hash, ssao_generation.inl:139-141, whose sin argument reaches ~1e5);
* textures are sampled with the textbook bilinear filter (exact float64 weights, no 8-bit sub-texel
  quantisation), clamp-to-edge (Daxa-default linear sampler) or REPEAT (noise texture);
* stores: RGBA16F = numpy float16 (round to nearest even), UNORM8 = round(clamp(x, 0, 1) * 255).

Only tests/ import this module; nothing in the product path does.
"""
from __future__ import annotations

import math

import numpy as np

f64 = np.float64


# ------------------------------------------------------------------------------------------------
# globals (shared.inl:47-131) -> numpy
# ------------------------------------------------------------------------------------------------
def mat(m) -> np.ndarray:
    """glm column-major float[16] -> 4x4 float64 with M[row, col]."""
    return np.array(list(m), f64).reshape(4, 4).T


def vec(v) -> np.ndarray:
    return np.array(list(v), f64)


# ------------------------------------------------------------------------------------------------
# sampling (Vulkan linear filter, level 0)
# ------------------------------------------------------------------------------------------------
# Sub-texel precision of the filter weights: None = exact float64 weights (the textbook filter); 8 = the
# weights rounded to 1/256 of a texel (Vulkan subTexelPrecisionBits, 8 on AMD hardware). Set per call.
SUBTEXEL_BITS = None


def _axis(t, n, wrap):
    if SUBTEXEL_BITS:
        q = float(1 << SUBTEXEL_BITS)
        t = np.floor(t * q + 0.5) / q
    i0 = np.floor(t)
    w = t - i0
    i0 = i0.astype(np.int64)
    i1 = i0 + 1
    if wrap:
        return np.mod(i0, n), np.mod(i1, n), w
    return np.clip(i0, 0, n - 1), np.clip(i1, 0, n - 1), w


def bilinear(img: np.ndarray, u, v, wrap: bool = False) -> np.ndarray:
    """texture(sampler2D, (u, v)) of an (h, w[, c]) image as float64; result shape u.shape (+ (c,))."""
    a = np.asarray(img, f64)
    if a.ndim == 2:
        a = a[..., None]
    h, w = a.shape[:2]
    u = np.asarray(u, f64)
    v = np.asarray(v, f64)
    x0, x1, wx = _axis(u * w - 0.5, w, wrap)
    y0, y1, wy = _axis(v * h - 0.5, h, wrap)
    wx = wx[..., None]
    wy = wy[..., None]
    a00, a01, a10, a11 = a[y0, x0], a[y0, x1], a[y1, x0], a[y1, x1]
    top = a00 + (a01 - a00) * wx          # lerp form: equal texels give their value exactly
    bot = a10 + (a11 - a10) * wx
    r = top + (bot - top) * wy
    return r[..., 0] if np.asarray(img).ndim == 2 else r


def unorm8(img) -> np.ndarray:
    return np.asarray(img, f64) / 255.0


def to_unorm8(x) -> np.ndarray:
    return np.rint(np.clip(np.nan_to_num(np.asarray(x, f64), nan=0.0), 0.0, 1.0) * 255.0).astype(np.uint8)


def centres(W, H):
    """Fragment uv of a fullscreen-triangle pass: pixel centres, y = 0 the top row."""
    x = (np.arange(W, dtype=f64) + 0.5) / W
    y = (np.arange(H, dtype=f64) + 0.5) / H
    return np.meshgrid(x, y)


def normalize(v):
    return v / np.linalg.norm(v, axis=-1, keepdims=True)


def apply(M, v4):
    """M (4x4) times a (..., 4) array of column vectors."""
    return np.einsum("ij,...j->...i", M, v4)


def clamp(x, lo, hi):
    """GLSL clamp/min/max leave NaN operands undefined; taken as IEEE maxNum/minNum (a NaN operand yields the
    other one), which is what the GPU's v_max_f32 / v_min_f32 return. Matters for SSAO over the sky, whose
    cleared normal (0, 0, 0) normalises to NaN: the range check then clamps to 0 instead of propagating."""
    return np.fmin(np.fmax(x, lo), hi)


def smoothstep(e0, e1, x):
    t = clamp((x - e0) / (e1 - e0), 0.0, 1.0)
    return t * t * (3.0 - 2.0 * t)


# ------------------------------------------------------------------------------------------------
# Composition (composition.inl:110-225)
# ------------------------------------------------------------------------------------------------
def composition(g, albedo, emissive, normal, depth, ssao, shadow, clouds) -> np.ndarray:
    H, W = depth.shape
    u, v = centres(W, H)
    d = bilinear(depth, u, v)
    inv_proj, inv_view = mat(g.camera_inverse_projection_matrix), mat(g.camera_inverse_view_matrix)
    # get_world_position_from_depth, :114-122
    clip = np.stack([u * 2 - 1, v * 2 - 1, d, np.ones_like(d)], -1)
    vs = apply(inv_proj, clip)
    vs = vs / vs[..., 3:4]
    world = apply(inv_view, vs)[..., :3]
    # sun shadow (ESM), :166-173
    sun_pv = mat(g.sun_info.projection_matrix) @ mat(g.sun_info.view_matrix)
    sp = apply(sun_pv, np.concatenate([world, np.ones_like(d)[..., None]], -1))
    pc = sp[..., :3] / sp[..., 3:4]
    sd = bilinear(shadow, pc[..., 0] * 0.5 + 0.5, pc[..., 1] * 0.5 + 0.5)
    with np.errstate(over="ignore"):
        sun_shadow = np.clip(np.power(np.exp(g.sun_info.exponential_factor * (pc[..., 2] - sd)),
                                      g.sun_info.darkening_factor), 0.0, 1.0)
    # G-buffer reads, :198-201 (volumetric term is zeroed at :196)
    em = bilinear(emissive, u, v)[..., :3] * g.emissive_bloom_strength
    al = bilinear(albedo, u, v)[..., :3]
    nn = bilinear(normal, u, v)[..., :3]
    occ = np.power(bilinear(unorm8(ssao), u, v), g.ambient_occlussion_strength)
    sun_dir = vec(g.sun_info.direction)
    direct = (np.maximum(0.0, nn @ -sun_dir) * sun_shadow)[..., None] * np.ones(3)
    cam = vec(g.camera_position)
    view_dir = normalize(cam - world)
    for i in range(int(g.point_light_count)):      # calculate_point_light, :124-139
        L = g.point_lights[i]
        lp = vec(L.position)
        ld = normalize(lp - world)
        dist = np.linalg.norm(lp - world, axis=-1)
        att = 1.0 / (dist * dist)
        hw = normalize(ld + view_dir)
        diffuse = np.maximum(np.sum(nn * ld, -1), 0.0)
        nh = np.arccos(np.clip(np.sum(hw * nn, -1), -1.0, 1.0))
        direct += al * vec(L.color) * ((diffuse + np.exp(-(nh * nh))) * att * L.intensity)[..., None]
    for i in range(int(g.spot_light_count)):       # calculate_spot_light, :141-160
        L = g.spot_lights[i]
        lp = vec(L.position)
        ld = normalize(lp - world)
        theta = ld @ (-vec(L.direction) / np.linalg.norm(vec(L.direction)))
        inten = np.clip((theta - L.outer_cut_off) / (L.cut_off - L.outer_cut_off), 0.0, 1.0)
        dist = np.linalg.norm(lp - world, axis=-1)
        att = 1.0 / (dist * dist)
        hw = normalize(ld + view_dir)
        diffuse = np.maximum(np.sum(nn * ld, -1), 0.0)
        nh = np.arccos(np.clip(np.sum(hw * nn, -1), -1.0, 1.0))
        direct += al * vec(L.color) * ((diffuse + np.exp(-(nh * nh))) * att * L.intensity * inten)[..., None]
    color = (direct + vec(g.ambient)) * al * occ[..., None] + em          # :218
    sky = d == 1.0                                                          # :220-222
    color[sky] = bilinear(unorm8(clouds), u, v)[..., :3][sky]
    out = np.concatenate([color, np.ones_like(d)[..., None]], -1)
    return out.astype(np.float16)


# ------------------------------------------------------------------------------------------------
# SSAO (ssao_generation.inl:74-214) and blur (ssao_blur.inl:91-106)
# ------------------------------------------------------------------------------------------------
SSAO_KERNEL = np.array([
    (0.2196607, 0.9032637, 0.2254677), (0.05916681, 0.2201506, 0.1430302), (-0.4152246, 0.1320857, 0.7036734),
    (-0.3790807, 0.1454145, 0.100605), (0.3149606, -0.1294581, 0.7044517), (-0.1108412, 0.2162839, 0.1336278),
    (0.658012, -0.4395972, 0.2919373), (0.5377914, 0.3112189, 0.426864), (-0.2752537, 0.07625949, 0.1273409),
    (-0.1915639, -0.4973421, 0.3129629), (-0.2634767, 0.5277923, 0.1107446), (0.8242752, 0.02434147, 0.06049098),
    (0.06262707, -0.2128643, 0.03671562), (-0.1795662, -0.3543862, 0.07924347), (0.06039629, 0.24629, 0.4501176),
    (-0.7786345, -0.3814852, 0.2391262), (0.2792919, 0.2487278, 0.05185341), (0.1841383, 0.1696993, 0.8936281),
    (-0.3479781, 0.4725766, 0.719685), (-0.1365018, -0.2513416, 0.470937), (0.1280388, -0.563242, 0.3419276),
    (-0.4800232, -0.1899473, 0.2398808), (0.6389147, 0.1191014, 0.5271206), (0.1932822, -0.3692099, 0.6060588),
    (-0.3465451, -0.1654651, 0.6746758), (0.2448421, -0.1610962, 0.1289366)], np.float32)


def _rand32(cx, cy):
    """rand(c) = fract(sin(dot(c, (12.9898, 78.233))) * 43758.5453) in fp32, :139-141."""
    f = np.float32
    cx = cx.astype(f)
    cy = cy.astype(f)
    s = np.sin(cx * f(12.9898) + cy * f(78.233)).astype(f)
    y = (s * f(43758.5453)).astype(f)
    return (y - np.floor(y)).astype(f)


def _noise32(px, py, freq):
    """noise(p, freq), :143-155, in fp32 (the hash needs the GLSL's own fp32 rounding)."""
    f = np.float32
    px = px.astype(f)
    py = py.astype(f)
    unit = (f(2560.0) / f(freq)).astype(f) if isinstance(freq, np.ndarray) else f(f(2560.0) / f(freq))
    ix, iy = np.floor(px / unit), np.floor(py / unit)
    mx = (px - unit * np.floor(px / unit)).astype(f)        # GLSL mod(x, y) = x - y * floor(x / y)
    my = (py - unit * np.floor(py / unit)).astype(f)
    xx = (mx / unit).astype(f)
    yy = (my / unit).astype(f)
    xx = (f(0.5) * (f(1.0) - np.cos(f(3.14159265359) * xx))).astype(f)
    yy = (f(0.5) * (f(1.0) - np.cos(f(3.14159265359) * yy))).astype(f)
    a = _rand32(ix, iy)
    b = _rand32(ix + f(1), iy)
    c = _rand32(ix, iy + f(1))
    d = _rand32(ix + f(1), iy + f(1))
    x1 = a * (f(1) - xx) + b * xx
    x2 = c * (f(1) - xx) + d * xx
    return (x1 * (f(1) - yy) + x2 * yy).astype(f)


def ssao_random_vec(u, v, noise_w):
    """random_vec of :184-188 (x, y components; z = 0)."""
    f = np.float32
    u32, v32 = u.astype(f), v.astype(f)
    n1 = _noise32(u32, v32, f(noise_w * 2))
    freq2 = np.power(f(noise_w) * f(4.2), f(1.5) + u32 / f(10.0)).astype(f)
    n2 = _noise32(np.power(u32, f(1.1)), np.power(v32, f(1.1)), freq2)
    rv = np.stack([n1.astype(f64), n2.astype(f64), np.zeros(n1.shape)], -1)
    return normalize(rv)


def ssao_generation(g, depth, normal, out_shape) -> np.ndarray:
    h, w = out_shape
    u, v = centres(w, h)
    inv_proj, proj, view = mat(g.camera_inverse_projection_matrix), mat(g.camera_projection_matrix), mat(g.camera_view_matrix)

    def view_pos(uu, vv, dd):          # get_view_position_from_depth, :130-137
        vs = apply(inv_proj, np.stack([uu * 2 - 1, vv * 2 - 1, dd, np.ones_like(dd)], -1))
        return vs[..., :3] / vs[..., 3:4]

    frag = view_pos(u, v, bilinear(depth, u, v))                               # :177
    n = normalize(bilinear(normal, u, v)[..., :3]) @ view[:3, :3].T            # :178  mat3(view) * n
    rv = ssao_random_vec(u, v, normal.shape[1])                                 # :180-188
    t = normalize(rv - n * np.sum(rv * n, -1, keepdims=True))                   # :190
    b = np.cross(t, n)
    radius, bias = float(g.ssao_radius), float(g.ssao_bias)
    occ = np.zeros(u.shape)
    for i in range(int(g.ssao_kernel_size)):                                    # :195-210
        k = SSAO_KERNEL[i].astype(f64)
        s = frag + (t * k[0] + b * k[1] + n * k[2]) * radius
        off = apply(proj, np.concatenate([s, np.ones(u.shape)[..., None]], -1))
        ox, oy = off[..., 0] / off[..., 3] * 0.5 + 0.5, off[..., 1] / off[..., 3] * 0.5 + 0.5
        sz = view_pos(ox, oy, bilinear(depth, ox, oy))[..., 2]
        with np.errstate(divide="ignore"):
            rc = smoothstep(0.0, 1.0, radius / np.abs(frag[..., 2] - sz))
        occ += np.where(sz >= s[..., 2] + bias, 1.0, 0.0) * rc
    return to_unorm8(1.0 - occ / float(g.ssao_kernel_size))


def ssao_blur(ssao) -> np.ndarray:
    h, w = ssao.shape
    u, v = centres(w, h)
    img = unorm8(ssao)
    acc = np.zeros(u.shape)
    for x in range(-2, 2):
        for y in range(-2, 2):
            acc += bilinear(img, u + x / w, v + y / h)
    return to_unorm8(acc / 16.0)


# ------------------------------------------------------------------------------------------------
# Bloom (bloom_downsample.inl:107-141, bloom_upsample.inl:98-127)
# ------------------------------------------------------------------------------------------------
def bloom_downsample(higher, out_shape) -> np.ndarray:
    h, w = out_shape
    u, v = centres(w, h)
    sh, sw = higher.shape[:2]
    x, y = 1.0 / sw, 1.0 / sh

    def s(dx, dy):
        return bilinear(higher, u + dx * x, v + dy * y)[..., :3]

    e = s(0, 0)
    corners = s(-2, 2) + s(2, 2) + s(-2, -2) + s(2, -2)
    edges = s(0, 2) + s(-2, 0) + s(2, 0) + s(0, -2)
    inner = s(-1, 1) + s(1, 1) + s(-1, -1) + s(1, -1)
    rgb = e * 0.125 + corners * 0.03125 + edges * 0.0625 + inner * 0.125
    return rgb.astype(np.float16)


def bloom_upsample(lower, out_shape) -> np.ndarray:
    h, w = out_shape
    u, v = centres(w, h)
    lh, lw = lower.shape[:2]
    x, y = 1.0 / lw, 1.0 / lh

    def s(dx, dy):
        return bilinear(lower, u + dx * x, v + dy * y)[..., :3]

    rgb = (s(0, 0) * 4.0 + (s(0, 1) + s(-1, 0) + s(1, 0) + s(0, -1)) * 2.0 +
           (s(-1, 1) + s(1, 1) + s(-1, -1) + s(1, -1))) * (1.0 / 16.0)
    return rgb.astype(np.float16)


# ------------------------------------------------------------------------------------------------
# TAA (temporal_antialiasing.inl:137-190)
# ------------------------------------------------------------------------------------------------
GAUSS = np.array([1 / 16, 1 / 8, 1 / 16, 1 / 8, 1 / 4, 1 / 8, 1 / 16, 1 / 8, 1 / 16])


def temporal_antialiasing(g, color, prev, vel, pvel, depth) -> np.ndarray:
    H, W = depth.shape
    u, v = centres(W, H)
    rw, rh = float(g.resolution[0]), float(g.resolution[1])
    nb = [None] * 9
    blurred = np.zeros(u.shape + (4,))
    closest = np.ones(u.shape)
    du, dv = u.copy(), v.copy()
    mn = np.full(u.shape + (4,), 10.0e5)
    mx = np.full(u.shape + (4,), -10.0e5)
    for y in (1, 0, -1):
        for x in (1, 0, -1):
            idx = (y + 1) * 3 + (x + 1)
            su, sv = u + x / rw, v + y / rh
            nb[idx] = bilinear(color, su, sv)
            d = bilinear(depth, su, sv)
            closest = np.fmin(d, closest)
            hit = closest == d                                   # the LAST tie wins
            du = np.where(hit, su, du)
            dv = np.where(hit, sv, dv)
            mn = np.fmin(nb[idx], mn)
            mx = np.fmax(nb[idx], mx)
            blurred += GAUSS[idx] * nb[idx]
    c = nb[5]                                                    # quirk Q7: the (+1, 0) neighbour
    velocity = bilinear(vel, du, dv)[..., :2]
    accum = np.full(u.shape, min(0.1, float(g.frame_counter)))
    vu, vv = u - velocity[..., 0], v - velocity[..., 1]
    acc = bilinear(prev, vu, vv)
    outside = (vu < 0) | (vv < 0) | (vu > 1) | (vv > 1)
    accum[outside] = 1.0
    acc = clamp(acc, mn, mx)
    out = c * accum[..., None] + acc * (1 - accum[..., None])
    pv = bilinear(pvel, vu, vv)[..., :2]
    vlen = np.linalg.norm(pv - velocity, axis=-1)
    dis = np.clip((vlen - 0.001) * 10.0, 0.0, 1.0)[..., None]
    out = out * (1 - dis) + blurred * dis
    return out.astype(np.float16)


# ------------------------------------------------------------------------------------------------
# Auto exposure (generate_luminance_histogram.inl:59-78, resolve_luminance_histogram.inl:56-80)
# ------------------------------------------------------------------------------------------------
def luminance_bins(g, hdr) -> np.ndarray:
    """Per-pixel bin index (float64 dot / log2; i32() saturates, NaN -> 0)."""
    c = np.asarray(hdr, f64)[..., :3]
    lum = c @ np.array([0.2126, 0.7152, 0.0722])
    lum = np.where(lum < 1e-3, 0.0, lum)
    with np.errstate(divide="ignore", invalid="ignore"):
        lg = np.log2(lum)
        mapped = (lg - g.log_min_luminance) / (g.log_max_luminance - g.log_min_luminance) * (255.0 - 1.0) + 1.0
    i = np.where(np.isnan(mapped), 0.0, np.clip(np.trunc(np.nan_to_num(mapped, posinf=2.0 ** 31, neginf=-2.0 ** 31)),
                                                -2.0 ** 31, 2.0 ** 31 - 1))
    return np.clip(i, 0, 255).astype(np.int64)


def generate_luminance_histogram(g, hdr) -> np.ndarray:
    return np.bincount(luminance_bins(g, hdr).ravel(), minlength=256).astype(np.uint64)


def resolve_luminance_histogram(g, bins, exposure, total_pixels=None, wide=False) -> float:
    bins = np.asarray(bins, np.uint64)
    weighted = int(np.sum(bins * np.arange(256, dtype=np.uint64)))
    if not wide:
        weighted &= 0xFFFFFFFF                                   # u32 shared_buckets, :59-70
    total = float(g.resolution[0] * g.resolution[1]) if total_pixels is None else float(total_pixels)
    mean = float(weighted) / max(total - float(bins[0]), 1.0)
    log2_mean = (mean - 1.0) / (256.0 - 1.0) * (g.log_max_luminance - g.log_min_luminance) + g.log_min_luminance
    target = math.log2(g.target_luminance / 2.0 ** log2_mean)
    alpha = min(max(1.0 - math.exp(-g.delta_time * g.adjustment_speed), 0.0), 1.0)
    return exposure * (1.0 - alpha) + target * alpha


# ------------------------------------------------------------------------------------------------
# AgX-DS tone map (tone_mapping.inl:91-176)
# ------------------------------------------------------------------------------------------------
def _primaries(r, gr, b, w):
    def un(xy):
        return np.array([xy[0] / xy[1], 1.0, (1.0 - xy[0] - xy[1]) / xy[1]])
    R, G, B, Wt = un(r), un(gr), un(b), un(w)
    temp = np.array([[R[0], G[0], B[0]], [1.0, 1.0, 1.0], [R[2], G[2], B[2]]])   # columns = R, G, B
    s = np.linalg.inv(temp) @ Wt
    return np.stack([R * s[0], G * s[1], B * s[2]], 1)


def agx_matrix(compression):
    r, gr, b, w = (0.64, 0.33), (0.3, 0.6), (0.15, 0.06), (0.3127, 0.3290)
    srgb_to_xyz = _primaries(r, gr, b, w)
    sf = 1.0 / (1.0 - compression)

    def mix2(a, c):
        return (a[0] * (1 - sf) + c[0] * sf, a[1] * (1 - sf) + c[1] * sf)
    adjusted_to_xyz = _primaries(mix2(w, r), mix2(w, gr), mix2(w, b), w)
    return srgb_to_xyz @ np.linalg.inv(adjusted_to_xyz)


def tone_mapping(g, color, exposure) -> np.ndarray:
    """RGBA8_UNORM framebuffer of AgX_DS(color) (alpha 1)."""
    c = np.asarray(color, f64)[..., :3]
    wc = np.maximum(c, 0.0) * 2.0 ** exposure
    M = agx_matrix(g.compression)
    wc = wc @ M.T
    S = g.peak * g.agxDs_linear_section
    C_ = g.peak / (g.peak - S)
    with np.errstate(over="ignore"):
        ds = np.where(wc < S, wc, g.peak - (g.peak - S) * np.exp((-C_ * (wc - S)) / g.peak))
    wc = np.clip(ds, 0.0, 1.0)
    lum = wc @ np.array([0.2126729, 0.7151522, 0.0721750])
    wc = lum[..., None] * (1 - g.saturation) + wc * g.saturation
    wc = np.clip(wc, 0.0, 1.0)
    wc = wc @ np.linalg.inv(M).T
    out = np.concatenate([wc, np.ones(wc.shape[:-1] + (1,))], -1)
    return to_unorm8(out)


# ------------------------------------------------------------------------------------------------
# Atmosphere + volumetric clouds (cloud_rendering.inl:65-481)
# ------------------------------------------------------------------------------------------------
EARTH = 6371000.0
CLOUD_MIN, CLOUD_MAX = 1600.0, 2100.0
RAYLEIGH = np.array([0.27, 0.5, 1.0]) * 1e-5
MIE = np.full(3, 0.5e-6)
LN2 = math.log(2.0)


def _rsi(pos, d, radius):
    pod = np.sum(pos * d, -1)
    delta = pod * pod + radius * radius - np.sum(pos * pos, -1)
    ok = delta >= 0.0
    sq = np.sqrt(np.where(ok, delta, 0.0))
    return np.where(ok, -pod - sq, -1.0), np.where(ok, -pod + sq, -1.0)


def _bayer2(a):
    a = np.floor(a)
    x = a[..., 0] * 0.5 + a[..., 1] * (a[..., 1] * 0.75)
    return x - np.floor(x)


def _bayer(a, n):
    if n == 2:
        return _bayer2(a)
    return _bayer(0.5 * a, n // 2) * 0.25 + _bayer2(a)


def _noise3(noise, pos):
    p = np.floor(pos[..., 2])
    f = pos[..., 2] - p
    inv = 1.0 / 64.0
    zs = 17.0 * inv
    cu = pos[..., 0] * inv + p * zs
    cv = pos[..., 1] * inv + p * zs
    a = bilinear(noise, cu, cv, wrap=True)[..., 0]
    b = bilinear(noise, cu + zs, cv + zs, wrap=True)[..., 0]
    return a * (1 - f) + b * f


def _clouds(noise, p, cam, elapsed):
    h = np.linalg.norm(p + np.array([0.0, EARTH, 0.0]), axis=-1) - EARTH
    q = np.stack([p[..., 0] + cam[0], h, p[..., 2] + cam[2]], -1)
    inside = (h >= CLOUD_MIN) & (h <= CLOUD_MAX)
    t = -1.0 * 0.02 * elapsed
    mv = np.array([t, 0.0, t])
    cc = q * 0.001 + mv
    n = (_noise3(noise, cc) * 0.5 + _noise3(noise, cc * 2.0 + mv) * 0.25 + _noise3(noise, cc * 7.0 - mv) * 0.125 +
         _noise3(noise, (cc + mv) * 16.0) * 0.0625)
    hh = h - CLOUD_MIN
    thr = (1.0 - np.exp(-0.01 * hh)) * np.exp(-0.004 * hh)
    return np.where(inside, smoothstep(0.55, 0.6, n) * thr * 0.03, 0.0)


def _hg(x, gg):
    g2 = gg * gg
    return 0.25 * ((1.0 - g2) * np.power(1.0 + g2 - 2.0 * gg * x, -1.5))


def _sky_top(sun):
    od = 100000.0 / max(1.0 * 2.0 - 0.01, 0.01)
    odl = 100000.0 / max(sun[1] * 2.0 + 0.01, 0.01)
    tot = RAYLEIGH + MIE
    sv, av = tot * od, np.exp(-tot * od)
    sl, al = tot * odl, np.exp(-tot * odl)
    absorb_sun = (np.abs(al - av) + 1e-3) / (np.abs((sl - sv) * LN2) + 1e-3)
    return (MIE * od * 0.25 + RAYLEIGH * od * 0.375) * absorb_sun * 3.0


def _atmosphere(r, r0, psun, elapsed):
    i_sun, r_planet, r_atmos = 22.0, 6371e3, 6471e3
    k_rlh, k_mie, sh_rlh, sh_mie, g = np.array([5.5e-6, 13.0e-6, 22.4e-6]), 21e-6, 8e3, 1.2e3, 0.758
    r = normalize(r)
    r0b = np.broadcast_to(r0, r.shape)
    px, py = _rsi(r0b, r, r_atmos)
    valid = ~(px > py)
    py = np.minimum(py, _rsi(r0b, r, r_planet)[0])
    step = (py - px) / 16.0
    t = np.full(px.shape, float(elapsed))                    # quirk Q10: iTime starts at elapsed_time
    tot_r = np.zeros(r.shape)
    tot_m = np.zeros(r.shape)
    od_r = np.zeros(px.shape)
    od_m = np.zeros(px.shape)
    mu = r @ psun
    gg = g * g
    p_rlh = 3.0 / (16.0 * 3.141592) * (1.0 + mu * mu)
    p_mie = 3.0 / (8.0 * 3.141592) * ((1.0 - gg) * (mu * mu + 1.0)) / (np.power(1.0 + gg - 2.0 * mu * g, 1.5) * (2.0 + gg))
    for _ in range(16):
        ip = r0b + r * (t + step * 0.5)[..., None]
        ih = np.linalg.norm(ip, axis=-1) - r_planet
        s_r = np.exp(-ih / sh_rlh) * step
        s_m = np.exp(-ih / sh_mie) * step
        od_r += s_r
        od_m += s_m
        jstep = _rsi(ip, np.broadcast_to(psun, ip.shape), r_atmos)[1] / 8.0
        jt = np.zeros(px.shape)
        jr = np.zeros(px.shape)
        jm = np.zeros(px.shape)
        for _ in range(8):
            jp = ip + psun * (jt + jstep * 0.5)[..., None]
            jh = np.linalg.norm(jp, axis=-1) - r_planet
            jr += np.exp(-jh / sh_rlh) * jstep
            jm += np.exp(-jh / sh_mie) * jstep
            jt += jstep
        attn = np.exp(-(k_mie * (od_m + jm)[..., None] + k_rlh * (od_r + jr)[..., None]))
        tot_r += s_r[..., None] * attn
        tot_m += s_m[..., None] * attn
        t += step
    col = i_sun * (p_rlh[..., None] * k_rlh * tot_r + (p_mie * k_mie)[..., None] * tot_m)
    return np.where(valid[..., None], col, 0.0)


def _volumetric_clouds(noise, d, sun, color, dither, cam, elapsed):
    out = color.copy()
    up = d[..., 1] >= 0.0
    if not up.any():
        return out
    d, color, dither = d[up], color[up], dither[up]
    base = np.array([0.0, EARTH, 0.0])
    bottom = _rsi(np.broadcast_to(base, d.shape), d, EARTH + CLOUD_MIN)[1]
    top = _rsi(np.broadcast_to(base, d.shape), d, EARTH + CLOUD_MAX)[1]
    start, end = d * bottom[..., None], d * top[..., None]
    inc = (end - start) / 24.0
    pos = inc * dither[..., None] + start
    step_len = np.linalg.norm(inc, axis=-1)
    scattering = np.zeros(d.shape)
    trans = np.ones(d.shape[0])
    ldw = d @ sun
    phase = _hg(ldw, 0.8 * 0.8) * 0.5 + _hg(ldw, -0.5 * 0.8) * 0.5
    sky_light = _sky_top(sun)
    sun_color = np.full(3, 0.8)
    for _ in range(24):
        od = _clouds(noise, pos, cam, elapsed) * step_len
        act = od > 0.0
        if act.any():
            # getSunVisibility, :264-278
            incs = sun * (500.0 / 10.0)
            sp = incs * 0.5 + pos[act]
            tr = np.zeros(int(act.sum()))
            for _ in range(10):
                tr += _clouds(noise, sp, cam, elapsed)
                sp = sp + incs
            vis = np.exp(-tr * (500.0 / 10.0))
            o = od[act]
            integral = np.exp(-1.11 / LN2 * o) * (-1.0 / 1.11) + 1.0 / 1.11
            powder = 1.0 - np.exp(-(o * LN2) * 2.0)
            sunl = sun_color * (vis * powder * phase[act] * (math.pi * 0.5) * 3.0)[..., None]
            skyl = sky_light * 0.25 * (1.0 / math.pi)
            scattering[act] += (sunl + skyl) * (integral * math.pi)[..., None] * trans[act][..., None]
            trans[act] *= np.exp(-o)
        pos = pos + inc
    fade = np.clip(np.linalg.norm(start, axis=-1) * 0.00001 * 2.5, 0.0, 1.0)[..., None]
    out[up] = (color * trans[..., None] + scattering) * (1 - fade) + color * fade
    return out


def cloud_rendering(g, depth, noise) -> np.ndarray:
    """RGBA8 clouds target (quirk Q6: full resolution; non-sky pixels (0.2, 0.4, 1.0))."""
    H, W = depth.shape
    rw, rh = int(g.resolution[0]), int(g.resolution[1])
    px, py = np.meshgrid(np.arange(W, dtype=f64), np.arange(H, dtype=f64))
    ru, rv = px / (rw - 1.0), py / (rh - 1.0)
    inv_proj, inv_view = mat(g.camera_inverse_projection_matrix), mat(g.camera_inverse_view_matrix)
    vs = apply(inv_proj, np.stack([ru * 2 - 1, rv * 2 - 1, -np.ones_like(ru), np.zeros_like(ru)], -1))
    ws = apply(inv_view, np.stack([vs[..., 0], vs[..., 1], -np.ones_like(ru), np.zeros_like(ru)], -1))[..., :3]
    d = normalize(ws)
    sun = -vec(g.sun_info.direction)
    color = np.broadcast_to(np.array([0.2, 0.4, 1.0]), (H, W, 3)).copy()
    dep = bilinear(depth, ru, rv)
    sky = dep == 1.0
    if sky.any():
        cam = vec(g.camera_position)
        r0 = np.array([0.0, 6372e3, 0.0]) + cam
        dither = _bayer(np.stack([px[sky], py[sky]], -1), 16)
        c = _atmosphere(d[sky], r0, sun, float(g.elapsed_time))
        c = _volumetric_clouds(unorm8(noise), d[sky], sun, c, dither, cam, float(g.elapsed_time))
        c *= max(min(abs(sun[0]), abs(sun[2])) + sun[1], 0.0)
        color[sky] = c
    out = np.concatenate([color, np.ones((H, W, 1))], -1)
    return to_unorm8(out)
