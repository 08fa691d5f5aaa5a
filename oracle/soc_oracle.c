/*
 * soc_oracle.c — CPU restatement ("oracle") of the reference renderer's screen-space passes.
 *
 * TEST INFRASTRUCTURE ONLY: used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg, never by the product path. Parity vs the reference itself is UNPINNED (the Vulkan/Daxa
 * reference cannot run here and holds no golden vectors); this file is pinned by
 * hand-derived known-answer tests and cross-checked against a second, independent restatement of
 * the GLSL in numpy (oracle/np_oracle.py, float64, textbook filter) by tests/test_np_oracle.py.
 *
 * Every pass follows the GLSL of the reference line by line; the file:line of each restated shader
 * is cited at the function. Numerics: IEEE fp32, compiled with -ffp-contract=off (no implicit FMA),
 * libm transcendentals. Vulkan fixed-function behaviour is restated by the SAMPLING CONTRACT below
 * (DESIGN.md §3), which the HIP kernels implement too.
 *
 * Sampling contract (the reference's linear_sampler, renderer.cpp:599-604, CLAMP_TO_EDGE assumed;
 * the noise sampler, texture.cpp:114-128, REPEAT):
 *   t   = u * n - 0.5                      (two roundings)
 *   t   = min(max(t, -2), n + 1)           (clamp mode; NaN -> -2)
 *   fx  = floor(t * 256 + 0.5)             (8-bit sub-texel precision, Vulkan subTexelPrecisionBits)
 *   i   = fx >> 8,  w = (fx & 255) / 256
 *   clamp: i < 0 -> texel 0 exactly; i >= n-1 -> texel n-1 exactly; else lerp(i, i+1, w)
 *   repeat: i0 = i mod n, i1 = (i+1) mod n
 *   value = (a*(1-wx) + b*wx)*(1-wy) + (c*(1-wx) + d*wx)*wy
 *   UNORM8 texel -> float: u * (1/255);  float -> UNORM8: rint(clamp(x,0,1) * 255) (NaN -> 0)
 *   float -> RGBA16F: round-to-nearest-even.
 */
#include "soc_oracle.h"

#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------------------------------------ */
/* small vector / matrix helpers (GLSL semantics, column-major mat4 m[col*4+row])                     */
/* ------------------------------------------------------------------------------------------------ */
typedef struct { float x, y; } v2;
typedef struct { float x, y, z; } v3;
typedef struct { float x, y, z, w; } v4;

static inline v2 V2(float x, float y) { v2 r = {x, y}; return r; }
static inline v3 V3(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static inline v4 V4(float x, float y, float z, float w) { v4 r = {x, y, z, w}; return r; }
static inline v3 add3(v3 a, v3 b) { return V3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 sub3(v3 a, v3 b) { return V3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 mul3(v3 a, v3 b) { return V3(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline v3 muls3(v3 a, float s) { return V3(a.x * s, a.y * s, a.z * s); }
static inline v3 neg3(v3 a) { return V3(-a.x, -a.y, -a.z); }
static inline float dot3(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline float length3(v3 a) { return sqrtf(dot3(a, a)); }
static inline v3 normalize3(v3 a) { float l = length3(a); return V3(a.x / l, a.y / l, a.z / l); }
static inline v3 cross3(v3 a, v3 b) {
    return V3(a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y);
}
static inline v3 exp3(v3 a) { return V3(expf(a.x), expf(a.y), expf(a.z)); }
static inline float clampf(float x, float lo, float hi) { return fminf(fmaxf(x, lo), hi); }
static inline float mixf(float a, float b, float t) { return a * (1.0f - t) + b * t; }
static inline v3 mix3(v3 a, v3 b, float t) { return V3(mixf(a.x, b.x, t), mixf(a.y, b.y, t), mixf(a.z, b.z, t)); }
static inline float fractf(float x) { return x - floorf(x); }
static inline float smoothstepf(float e0, float e1, float x) {
    float t = clampf((x - e0) / (e1 - e0), 0.0f, 1.0f);
    return t * t * (3.0f - 2.0f * t);
}

/* GLSL mat4 * vec4: col0*v.x + col1*v.y + col2*v.z + col3*v.w */
static inline v4 mat4_mul_v4(const float* m, v4 v) {
    v4 r;
    r.x = m[0] * v.x + m[4] * v.y + m[8] * v.z + m[12] * v.w;
    r.y = m[1] * v.x + m[5] * v.y + m[9] * v.z + m[13] * v.w;
    r.z = m[2] * v.x + m[6] * v.y + m[10] * v.z + m[14] * v.w;
    r.w = m[3] * v.x + m[7] * v.y + m[11] * v.z + m[15] * v.w;
    return r;
}
/* GLSL mat4 * mat4 */
static void mat4_mul(float* out, const float* a, const float* b) {
    float t[16];
    for (int c = 0; c < 4; ++c)
        for (int r = 0; r < 4; ++r)
            t[c * 4 + r] = a[0 * 4 + r] * b[c * 4 + 0] + a[1 * 4 + r] * b[c * 4 + 1] + a[2 * 4 + r] * b[c * 4 + 2] +
                           a[3 * 4 + r] * b[c * 4 + 3];
    memcpy(out, t, sizeof t);
}
/* mat3(mat4) * vec3 */
static inline v3 mat3of4_mul_v3(const float* m, v3 v) {
    return V3(m[0] * v.x + m[4] * v.y + m[8] * v.z, m[1] * v.x + m[5] * v.y + m[9] * v.z,
              m[2] * v.x + m[6] * v.y + m[10] * v.z);
}
/* mat3 m[c*3+r] */
static inline v3 mat3_mul_v3(const float* m, v3 v) {
    return V3(m[0] * v.x + m[3] * v.y + m[6] * v.z, m[1] * v.x + m[4] * v.y + m[7] * v.z,
              m[2] * v.x + m[5] * v.y + m[8] * v.z);
}
static void mat3_mul(float* out, const float* a, const float* b) {
    float t[9];
    for (int c = 0; c < 3; ++c)
        for (int r = 0; r < 3; ++r) t[c * 3 + r] = a[0 * 3 + r] * b[c * 3 + 0] + a[1 * 3 + r] * b[c * 3 + 1] + a[2 * 3 + r] * b[c * 3 + 2];
    memcpy(out, t, sizeof t);
}
/* GLSL inverse(mat3) restated with glm's cofactor order (glm/detail/func_matrix.inl). */
static void mat3_inverse(float* o, const float* m) {
#define M(c, r) m[(c) * 3 + (r)]
    float det = M(0, 0) * (M(1, 1) * M(2, 2) - M(2, 1) * M(1, 2)) - M(1, 0) * (M(0, 1) * M(2, 2) - M(2, 1) * M(0, 2)) +
                M(2, 0) * (M(0, 1) * M(1, 2) - M(1, 1) * M(0, 2));
    float od = 1.0f / det;
    float t[9];
    t[0 * 3 + 0] = +(M(1, 1) * M(2, 2) - M(2, 1) * M(1, 2)) * od;
    t[1 * 3 + 0] = -(M(1, 0) * M(2, 2) - M(2, 0) * M(1, 2)) * od;
    t[2 * 3 + 0] = +(M(1, 0) * M(2, 1) - M(2, 0) * M(1, 1)) * od;
    t[0 * 3 + 1] = -(M(0, 1) * M(2, 2) - M(2, 1) * M(0, 2)) * od;
    t[1 * 3 + 1] = +(M(0, 0) * M(2, 2) - M(2, 0) * M(0, 2)) * od;
    t[2 * 3 + 1] = -(M(0, 0) * M(2, 1) - M(2, 0) * M(0, 1)) * od;
    t[0 * 3 + 2] = +(M(0, 1) * M(1, 2) - M(1, 1) * M(0, 2)) * od;
    t[1 * 3 + 2] = -(M(0, 0) * M(1, 2) - M(1, 0) * M(0, 2)) * od;
    t[2 * 3 + 2] = +(M(0, 0) * M(1, 1) - M(1, 0) * M(0, 1)) * od;
#undef M
    memcpy(o, t, sizeof t);
}

/* ------------------------------------------------------------------------------------------------ */
/* formats                                                                                           */
/* ------------------------------------------------------------------------------------------------ */
static inline uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

uint16_t soc_oracle_f32_to_f16(float f) {
    const uint32_t f32infty = 255u << 23, f16max = (127u + 16u) << 23;
    const uint32_t denorm_magic = ((127u - 15u) + (23u - 10u) + 1u) << 23;
    uint32_t u = f2u(f), sign = u & 0x80000000u, o;
    u ^= sign;
    if (u >= f16max) {
        o = (u > f32infty) ? 0x7e00u : 0x7c00u;
    } else if (u < (113u << 23)) {
        float fu = u2f(u) + u2f(denorm_magic);
        o = f2u(fu) - denorm_magic;
    } else {
        uint32_t mant_odd = (u >> 13) & 1u;
        u += ((uint32_t)(15 - 127) << 23) + 0xfffu;
        u += mant_odd;
        o = u >> 13;
    }
    return (uint16_t)(o | (sign >> 16));
}

float soc_oracle_f16_to_f32(uint16_t h) {
    uint32_t sign = (uint32_t)(h & 0x8000u) << 16, e = (h >> 10) & 0x1f, m = h & 0x3ffu;
    if (e == 0) {
        float v = (float)m * (1.0f / 16777216.0f); /* m * 2^-24 */
        return sign ? -v : v;
    }
    if (e == 31) return u2f(sign | 0x7f800000u | (m << 13));
    return u2f(sign | ((e + 112u) << 23) | (m << 13));
}

static inline int bpp(int fmt) {
    switch (fmt) {
    case SOC_FMT_RGBA16F: return 8;
    case SOC_FMT_D32F: return 4;
    case SOC_FMT_R8_UNORM: return 1;
    case SOC_FMT_RGBA8_UNORM:
    case SOC_FMT_RGBA8_SRGB: return 4;
    case SOC_FMT_RGBA32F: return 16;
    default: return 0;
    }
}

static inline float unorm8(uint8_t u) { return (float)u * (1.0f / 255.0f); }
static inline uint8_t to_unorm8(float x) { return (uint8_t)rintf(clampf(x, 0.0f, 1.0f) * 255.0f); }
static inline float srgb_encode(float c) {
    c = clampf(c, 0.0f, 1.0f);
    return c <= 0.0031308f ? c * 12.92f : 1.055f * powf(c, 1.0f / 2.4f) - 0.055f;
}
static inline float srgb_decode(float c) {
    return c <= 0.04045f ? c / 12.92f : powf((c + 0.055f) / 1.055f, 2.4f);
}

static inline v4 fetch(const soc_img* im, int x, int y) {
    const uint8_t* row = (const uint8_t*)im->data + (size_t)y * (size_t)im->pitch_bytes;
    switch (im->format) {
    case SOC_FMT_RGBA16F: {
        const uint16_t* p = (const uint16_t*)row + (size_t)x * 4;
        return V4(soc_oracle_f16_to_f32(p[0]), soc_oracle_f16_to_f32(p[1]), soc_oracle_f16_to_f32(p[2]),
                  soc_oracle_f16_to_f32(p[3]));
    }
    case SOC_FMT_D32F: return V4(((const float*)row)[x], 0.0f, 0.0f, 1.0f);
    case SOC_FMT_R8_UNORM: return V4(unorm8(row[x]), 0.0f, 0.0f, 1.0f);
    case SOC_FMT_RGBA8_UNORM: {
        const uint8_t* p = row + (size_t)x * 4;
        return V4(unorm8(p[0]), unorm8(p[1]), unorm8(p[2]), unorm8(p[3]));
    }
    case SOC_FMT_RGBA8_SRGB: {
        const uint8_t* p = row + (size_t)x * 4;
        return V4(srgb_decode(unorm8(p[0])), srgb_decode(unorm8(p[1])), srgb_decode(unorm8(p[2])), unorm8(p[3]));
    }
    case SOC_FMT_RGBA32F: {
        const float* p = (const float*)row + (size_t)x * 4;
        return V4(p[0], p[1], p[2], p[3]);
    }
    default: return V4(0, 0, 0, 0);
    }
}

static inline void store(const soc_img* im, int x, int y, v4 c) {
    uint8_t* row = (uint8_t*)im->data + (size_t)y * (size_t)im->pitch_bytes;
    switch (im->format) {
    case SOC_FMT_RGBA16F: {
        uint16_t* p = (uint16_t*)row + (size_t)x * 4;
        p[0] = soc_oracle_f32_to_f16(c.x); p[1] = soc_oracle_f32_to_f16(c.y);
        p[2] = soc_oracle_f32_to_f16(c.z); p[3] = soc_oracle_f32_to_f16(c.w);
        break;
    }
    case SOC_FMT_D32F: ((float*)row)[x] = c.x; break;
    case SOC_FMT_R8_UNORM: row[x] = to_unorm8(c.x); break;
    case SOC_FMT_RGBA8_UNORM: {
        uint8_t* p = row + (size_t)x * 4;
        p[0] = to_unorm8(c.x); p[1] = to_unorm8(c.y); p[2] = to_unorm8(c.z); p[3] = to_unorm8(c.w);
        break;
    }
    case SOC_FMT_RGBA8_SRGB: {
        uint8_t* p = row + (size_t)x * 4;
        p[0] = to_unorm8(srgb_encode(c.x)); p[1] = to_unorm8(srgb_encode(c.y));
        p[2] = to_unorm8(srgb_encode(c.z)); p[3] = to_unorm8(c.w);
        break;
    }
    case SOC_FMT_RGBA32F: {
        float* p = (float*)row + (size_t)x * 4;
        p[0] = c.x; p[1] = c.y; p[2] = c.z; p[3] = c.w;
        break;
    }
    default: break;
    }
}

/* ------------------------------------------------------------------------------------------------ */
/* sampling contract                                                                                 */
/* ------------------------------------------------------------------------------------------------ */
static inline void axis_clamp(float u, int n, int* i0, int* i1, float* w) {
    float t = u * (float)n;
    t = t - 0.5f;
    t = fminf(fmaxf(t, -2.0f), (float)n + 1.0f);
    int fx = (int)floorf(t * 256.0f + 0.5f);
    int i = fx >> 8;
    float f = (float)(fx & 255) * (1.0f / 256.0f);
    if (i < 0) { *i0 = *i1 = 0; *w = 0.0f; }
    else if (i >= n - 1) { *i0 = *i1 = n - 1; *w = 0.0f; }
    else { *i0 = i; *i1 = i + 1; *w = f; }
}

static inline void axis_repeat(float u, int n, int* i0, int* i1, float* w) {
    float t = u * (float)n;
    t = t - 0.5f;
    t = fminf(fmaxf(t, -4194304.0f), 4194304.0f);
    int fx = (int)floorf(t * 256.0f + 0.5f);
    int i = fx >> 8;
    *w = (float)(fx & 255) * (1.0f / 256.0f);
    int a = i % n; if (a < 0) a += n;
    *i0 = a;
    *i1 = (a + 1) % n;
}

static inline float lerp_w(float a, float b, float w) { return a * (1.0f - w) + b * w; }

static inline v4 bilerp(v4 a, v4 b, v4 c, v4 d, float wx, float wy) {
    v4 t = V4(lerp_w(a.x, b.x, wx), lerp_w(a.y, b.y, wx), lerp_w(a.z, b.z, wx), lerp_w(a.w, b.w, wx));
    v4 m = V4(lerp_w(c.x, d.x, wx), lerp_w(c.y, d.y, wx), lerp_w(c.z, d.z, wx), lerp_w(c.w, d.w, wx));
    return V4(lerp_w(t.x, m.x, wy), lerp_w(t.y, m.y, wy), lerp_w(t.z, m.z, wy), lerp_w(t.w, m.w, wy));
}

static inline v4 sample_clamp(const soc_img* im, float u, float v) {
    int x0, x1, y0, y1; float wx, wy;
    axis_clamp(u, im->width, &x0, &x1, &wx);
    axis_clamp(v, im->height, &y0, &y1, &wy);
    return bilerp(fetch(im, x0, y0), fetch(im, x1, y0), fetch(im, x0, y1), fetch(im, x1, y1), wx, wy);
}

static inline v4 sample_repeat(const soc_img* im, float u, float v) {
    int x0, x1, y0, y1; float wx, wy;
    axis_repeat(u, im->width, &x0, &x1, &wx);
    axis_repeat(v, im->height, &y0, &y1, &wy);
    return bilerp(fetch(im, x0, y0), fetch(im, x1, y0), fetch(im, x0, y1), fetch(im, x1, y1), wx, wy);
}

static int valid(const soc_img* im) {
    return im->data && im->width > 0 && im->height > 0 && bpp(im->format) > 0 &&
           im->pitch_bytes >= im->width * bpp(im->format);
}

int soc_oracle_num_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}

/* ------------------------------------------------------------------------------------------------ */
/* deterministic log2 (shared numeric contract with the HIP histogram kernel)        */
/* ------------------------------------------------------------------------------------------------ */
float soc_oracle_log2(float x) {
    if (x != x) return x;
    if (x < 0.0f) return u2f(0x7fc00000u);
    if (x == 0.0f) return -INFINITY;
    if (x == INFINITY) return INFINITY;
    uint32_t u = f2u(x);
    int e = 0;
    if (u < 0x00800000u) { x = x * 8388608.0f; u = f2u(x); e = -23; } /* subnormal */
    e += (int)(u >> 23) - 127;
    float m = u2f((u & 0x007fffffu) | 0x3f800000u); /* [1,2) */
    if (m > 1.41421356f) { m = m * 0.5f; e += 1; }  /* [0.707, 1.414] */
    float f = m - 1.0f;
    float s = f / (2.0f + f);
    float s2 = s * s;
    /* ln(1+f) = 2s (1 + s2/3 + s2^2/5 + s2^3/7 + s2^4/9 + s2^5/11) */
    float p = fmaf(s2, 1.0f / 11.0f, 1.0f / 9.0f);
    p = fmaf(s2, p, 1.0f / 7.0f);
    p = fmaf(s2, p, 1.0f / 5.0f);
    p = fmaf(s2, p, 1.0f / 3.0f);
    p = fmaf(s2, p, 1.0f);
    float ln = (2.0f * s) * p;
    return fmaf(ln, 1.44269504088896341f, (float)e);
}

/* generate_luminance_histogram.inl:64-69 with the explicit-fma luminance / remap of DESIGN.md §3.4 */
uint32_t soc_oracle_luminance_bin(float r, float g, float b, float log_min, float log_max) {
    float lum = fmaf(b, 0.0722f, fmaf(g, 0.7152f, r * 0.2126f));
    if (lum < 1e-3f) lum = 0.0f;
    float q = (soc_oracle_log2(lum) - log_min) / (log_max - log_min);
    float mapped = fmaf(q, (float)(SOC_AUTO_EXPOSURE_BIN_COUNT - 1) - 1.0f, 1.0f);
    /* clamp(i32(mapped), 0, 255), i32() truncates toward zero and saturates; NaN -> 0 */
    if (mapped >= 255.0f) return 255u;
    if (mapped > 0.0f) return (uint32_t)(int32_t)mapped;
    return 0u;
}

/* ------------------------------------------------------------------------------------------------ */
/* bloom (bloom_downsample.inl:107-141, bloom_upsample.inl:98-127)                                   */
/* ------------------------------------------------------------------------------------------------ */
int soc_oracle_bloom_downsample(const soc_globals* g, soc_img hi, soc_img lo) {
    (void)g;
    if (!valid(&hi) || !valid(&lo) || hi.format != SOC_FMT_RGBA16F || lo.format != SOC_FMT_RGBA16F) return SOC_E_INVALID_ARG;
    const float sx = 1.0f / (float)hi.width, sy = 1.0f / (float)hi.height;
#pragma omp parallel for schedule(static)
    for (int y = 0; y < lo.height; ++y) {
        for (int x = 0; x < lo.width; ++x) {
            const float u = ((float)x + 0.5f) / (float)lo.width, v = ((float)y + 0.5f) / (float)lo.height;
            const float X = sx, Y = sy;
            v4 a = sample_clamp(&hi, u - 2 * X, v + 2 * Y), b = sample_clamp(&hi, u, v + 2 * Y), c = sample_clamp(&hi, u + 2 * X, v + 2 * Y);
            v4 d = sample_clamp(&hi, u - 2 * X, v), e = sample_clamp(&hi, u, v), f = sample_clamp(&hi, u + 2 * X, v);
            v4 gg = sample_clamp(&hi, u - 2 * X, v - 2 * Y), h = sample_clamp(&hi, u, v - 2 * Y), i = sample_clamp(&hi, u + 2 * X, v - 2 * Y);
            v4 j = sample_clamp(&hi, u - X, v + Y), k = sample_clamp(&hi, u + X, v + Y);
            v4 l = sample_clamp(&hi, u - X, v - Y), m = sample_clamp(&hi, u + X, v - Y);
            float o[3];
            const float* A = &a.x; const float* B = &b.x; const float* C = &c.x; const float* D = &d.x;
            const float* E = &e.x; const float* F = &f.x; const float* G = &gg.x; const float* H = &h.x;
            const float* I = &i.x; const float* J = &j.x; const float* K = &k.x; const float* L = &l.x;
            const float* Mm = &m.x;
            for (int ch = 0; ch < 3; ++ch) {
                float r = E[ch] * 0.125f;
                r += (A[ch] + C[ch] + G[ch] + I[ch]) * 0.03125f;
                r += (B[ch] + D[ch] + F[ch] + H[ch]) * 0.0625f;
                r += (J[ch] + K[ch] + L[ch] + Mm[ch]) * 0.125f;
                o[ch] = r;
            }
            /* alpha is not written by the shader (undefined); the contract stores 1.0 */
            store(&lo, x, y, V4(o[0], o[1], o[2], 1.0f));
        }
    }
    return SOC_OK;
}

int soc_oracle_bloom_upsample(const soc_globals* g, soc_img lo, soc_img hi) {
    (void)g;
    if (!valid(&hi) || !valid(&lo) || hi.format != SOC_FMT_RGBA16F || lo.format != SOC_FMT_RGBA16F) return SOC_E_INVALID_ARG;
    const float X = 1.0f / (float)lo.width, Y = 1.0f / (float)lo.height;
#pragma omp parallel for schedule(static)
    for (int y = 0; y < hi.height; ++y) {
        for (int x = 0; x < hi.width; ++x) {
            const float u = ((float)x + 0.5f) / (float)hi.width, v = ((float)y + 0.5f) / (float)hi.height;
            v4 a = sample_clamp(&lo, u - X, v + Y), b = sample_clamp(&lo, u, v + Y), c = sample_clamp(&lo, u + X, v + Y);
            v4 d = sample_clamp(&lo, u - X, v), e = sample_clamp(&lo, u, v), f = sample_clamp(&lo, u + X, v);
            v4 gg = sample_clamp(&lo, u - X, v - Y), h = sample_clamp(&lo, u, v - Y), i = sample_clamp(&lo, u + X, v - Y);
            const float* A = &a.x; const float* B = &b.x; const float* C = &c.x; const float* D = &d.x;
            const float* E = &e.x; const float* F = &f.x; const float* G = &gg.x; const float* H = &h.x;
            const float* I = &i.x;
            float o[3];
            for (int ch = 0; ch < 3; ++ch) {
                float r = E[ch] * 4.0f;
                r += (B[ch] + D[ch] + F[ch] + H[ch]) * 2.0f;
                r += (A[ch] + C[ch] + G[ch] + I[ch]);
                r *= 1.0f / 16.0f;
                o[ch] = r;
            }
            /* CLEAR (0,0,0,1) + ONE/ONE blend: rgb overwritten (quirk Q5); alpha contract 1.0 */
            store(&hi, x, y, V4(o[0], o[1], o[2], 1.0f));
        }
    }
    return SOC_OK;
}

/* ------------------------------------------------------------------------------------------------ */
/* SSAO (ssao_generation.inl:74-214) and blur (ssao_blur.inl:91-106)                                 */
/* ------------------------------------------------------------------------------------------------ */
static const float k_ssao_kernel[SOC_SSAO_MAX_KERNEL][3] = {
    {0.2196607f, 0.9032637f, 0.2254677f},   {0.05916681f, 0.2201506f, 0.1430302f},  {-0.4152246f, 0.1320857f, 0.7036734f},
    {-0.3790807f, 0.1454145f, 0.100605f},   {0.3149606f, -0.1294581f, 0.7044517f},  {-0.1108412f, 0.2162839f, 0.1336278f},
    {0.658012f, -0.4395972f, 0.2919373f},   {0.5377914f, 0.3112189f, 0.426864f},    {-0.2752537f, 0.07625949f, 0.1273409f},
    {-0.1915639f, -0.4973421f, 0.3129629f}, {-0.2634767f, 0.5277923f, 0.1107446f},  {0.8242752f, 0.02434147f, 0.06049098f},
    {0.06262707f, -0.2128643f, 0.03671562f}, {-0.1795662f, -0.3543862f, 0.07924347f}, {0.06039629f, 0.24629f, 0.4501176f},
    {-0.7786345f, -0.3814852f, 0.2391262f}, {0.2792919f, 0.2487278f, 0.05185341f},  {0.1841383f, 0.1696993f, 0.8936281f},
    {-0.3479781f, 0.4725766f, 0.719685f},   {-0.1365018f, -0.2513416f, 0.470937f},  {0.1280388f, -0.563242f, 0.3419276f},
    {-0.4800232f, -0.1899473f, 0.2398808f}, {0.6389147f, 0.1191014f, 0.5271206f},   {0.1932822f, -0.3692099f, 0.6060588f},
    {-0.3465451f, -0.1654651f, 0.6746758f}, {0.2448421f, -0.1610962f, 0.1289366f}};

/* Deterministic sin / cos / pow of float arguments for the SSAO noise (quirk Q8: the hash fract(sin(a) * 43758.5453)
   turns a 1-ulp difference of sin into ~3e-3 of the hash, so the oracle and the GPU's random-vector table must evaluate
   sin identically, not merely accurately). Each is evaluated in double with IEEE add / mul / fma / div and rint only
   (no libm), and rounded to float once: an accurate sinf / cosf / powf (the correctly rounded result except where the
   double value lies within ~1e-16 of a float rounding boundary) whose bits do not depend on a math library. The GPU
   table (ssao.hip det_sin / det_cos / det_pow, same operation sequence) gives the same bits, which the GPU suite checks
   (frame_parity "hash_differs" = 0). Range reduction: Cody-Waite with the three-part pi/2 of fdlibm's __ieee754_rem_pio2
   (exact for |x| < 2^20 pi/2, far beyond the hash's |arg| <= ~1e5); kernels: Taylor series on |r| <= pi/4 to 1/21!. */
static const double k_pio2_1 = 1.57079632673412561417e+00, k_pio2_2 = 6.07710050630396597660e-11,
                    k_pio2_3 = 2.02226624879595063154e-21, k_2_pi = 6.36619772367581382433e-01;
static double det_sin_poly(double r) {
    const double r2 = r * r;
    double p = 1.9572941063391263e-20;
    p = fma(p, r2, -8.22063524662433e-18);
    p = fma(p, r2, 2.8114572543455206e-15);
    p = fma(p, r2, -7.647163731819816e-13);
    p = fma(p, r2, 1.6059043836821613e-10);
    p = fma(p, r2, -2.505210838544172e-08);
    p = fma(p, r2, 2.7557319223985893e-06);
    p = fma(p, r2, -0.0001984126984126984);
    p = fma(p, r2, 0.008333333333333333);
    p = fma(p, r2, -0.16666666666666666);
    return fma(r * r2, p, r);
}
static double det_cos_poly(double r) {
    const double r2 = r * r;
    double p = 4.110317623312165e-19;
    p = fma(p, r2, -1.5619206968586225e-16);
    p = fma(p, r2, 4.779477332387385e-14);
    p = fma(p, r2, -1.1470745597729725e-11);
    p = fma(p, r2, 2.08767569878681e-09);
    p = fma(p, r2, -2.755731922398589e-07);
    p = fma(p, r2, 2.48015873015873e-05);
    p = fma(p, r2, -0.001388888888888889);
    p = fma(p, r2, 0.041666666666666664);
    p = fma(p, r2, -0.5);
    return fma(r2, p, 1.0);
}
/* quadrant q of x (x = q pi/2 + r) and the reduced argument r */
static double det_reduce(float x, long long* q) {
    const double d = (double)x;
    const double k = rint(d * k_2_pi);
    double r = fma(-k, k_pio2_1, d);
    r = fma(-k, k_pio2_2, r);
    r = fma(-k, k_pio2_3, r);
    *q = (long long)k;
    return r;
}
static float det_sin(float x) {
    long long q;
    const double r = det_reduce(x, &q);
    const int k = (int)(q & 3);
    const double v = (k & 1) ? det_cos_poly(r) : det_sin_poly(r);
    return (float)((k & 2) ? -v : v);
}
static float det_cos(float x) {
    long long q;
    const double r = det_reduce(x, &q);
    const int k = (int)((q + 1) & 3);   /* cos x = sin(x + pi/2) */
    const double v = (k & 1) ? det_cos_poly(r) : det_sin_poly(r);
    return (float)((k & 2) ? -v : v);
}
/* pow(x, y) for finite x > 0 (the noise's uv and 4.2 W; GLSL pow is undefined for x < 0): exp(y ln x) in double,
   ln x = e ln2 + 2 atanh((m - 1) / (m + 1)) with m in [sqrt(1/2), sqrt(2)), exp by k ln2 + r, |r| <= ln2 / 2. */
static const double k_ln2_hi = 6.93147180369123816490e-01, k_ln2_lo = 1.90821492927058770002e-10,
                    k_inv_ln2 = 1.44269504088896338700e+00;
static float det_pow(float x, float y) {
    if (!(x > 0.0f) || !isfinite(x) || !isfinite(y)) return powf(x, y);   /* outside the hash's domain (not reached) */
    uint32_t b;
    memcpy(&b, &x, 4);
    int e = (int)((b >> 23) & 255u) - 127;
    if (e == -127) {   /* subnormal: scale by 2^32 first (exact) */
        float xs = x * 4294967296.0f;
        memcpy(&b, &xs, 4);
        e = (int)((b >> 23) & 255u) - 127 - 32;
    }
    const uint32_t mb = (b & 0x007fffffu) | 0x3f800000u;
    float mf;
    memcpy(&mf, &mb, 4);
    double m = (double)mf;
    if (m > 1.4142135623730951) { m *= 0.5; e += 1; }
    const double s = (m - 1.0) / (m + 1.0), s2 = s * s;
    double p = 0.04;   /* 1/25 */
    p = fma(p, s2, 0.043478260869565216);
    p = fma(p, s2, 0.047619047619047616);
    p = fma(p, s2, 0.05263157894736842);
    p = fma(p, s2, 0.058823529411764705);
    p = fma(p, s2, 0.06666666666666667);
    p = fma(p, s2, 0.07692307692307693);
    p = fma(p, s2, 0.09090909090909091);
    p = fma(p, s2, 0.1111111111111111);
    p = fma(p, s2, 0.14285714285714285);
    p = fma(p, s2, 0.2);
    p = fma(p, s2, 0.3333333333333333);
    const double lnm = 2.0 * fma(s * s2, p, s);
    const double lnx = fma((double)e, k_ln2_hi, fma((double)e, k_ln2_lo, lnm));
    const double z = (double)y * lnx;
    const double k = rint(z * k_inv_ln2);
    double r = fma(-k, k_ln2_hi, z);
    r = fma(-k, k_ln2_lo, r);
    double q = 8.896791392450574e-22;
    q = fma(q, r, 1.9572941063391263e-20);
    q = fma(q, r, 4.110317623312165e-19);
    q = fma(q, r, 8.22063524662433e-18);
    q = fma(q, r, 1.5619206968586225e-16);
    q = fma(q, r, 2.8114572543455206e-15);
    q = fma(q, r, 4.779477332387385e-14);
    q = fma(q, r, 7.647163731819816e-13);
    q = fma(q, r, 1.1470745597729725e-11);
    q = fma(q, r, 1.6059043836821613e-10);
    q = fma(q, r, 2.08767569878681e-09);
    q = fma(q, r, 2.505210838544172e-08);
    q = fma(q, r, 2.755731922398589e-07);
    q = fma(q, r, 2.7557319223985893e-06);
    q = fma(q, r, 2.48015873015873e-05);
    q = fma(q, r, 0.0001984126984126984);
    q = fma(q, r, 0.001388888888888889);
    q = fma(q, r, 0.008333333333333333);
    q = fma(q, r, 0.041666666666666664);
    q = fma(q, r, 0.16666666666666666);
    q = fma(q, r, 0.5);
    q = fma(q, r, 1.0);
    q = fma(q, r, 1.0);
    if (!(k > -1000.0 && k < 1000.0)) return (float)(k > 0.0 ? INFINITY : 0.0);
    const uint64_t sb = (uint64_t)((long long)k + 1023) << 52;
    double sc;
    memcpy(&sc, &sb, 8);
    return (float)(q * sc);
}

float soc_oracle_det_sin(float x) { return det_sin(x); }
float soc_oracle_det_cos(float x) { return det_cos(x); }
float soc_oracle_det_pow(float x, float y) { return det_pow(x, y); }

/* ssao_generation.inl:139-141 (sin: det_sin above) */
static inline float ssao_rand(v2 c) { return fractf(det_sin(c.x * 12.9898f + c.y * 78.233f) * 43758.5453f); }

/* ssao_generation.inl:143-155 */
static float ssao_noise(v2 p, float freq) {
    float unit = 2560.0f / freq;
    v2 q = V2(p.x / unit, p.y / unit);
    v2 ij = V2(floorf(q.x), floorf(q.y));
    /* mod(p, unit) = p - unit * floor(p / unit) */
    v2 xy = V2((p.x - unit * floorf(p.x / unit)) / unit, (p.y - unit * floorf(p.y / unit)) / unit);
    xy = V2(0.5f * (1.0f - det_cos(3.14159265359f * xy.x)), 0.5f * (1.0f - det_cos(3.14159265359f * xy.y)));
    float a = ssao_rand(V2(ij.x + 0.0f, ij.y + 0.0f));
    float b = ssao_rand(V2(ij.x + 1.0f, ij.y + 0.0f));
    float c = ssao_rand(V2(ij.x + 0.0f, ij.y + 1.0f));
    float d = ssao_rand(V2(ij.x + 1.0f, ij.y + 1.0f));
    float x1 = mixf(a, b, xy.x);
    float x2 = mixf(c, d, xy.x);
    return mixf(x1, x2, xy.y);
}

/* get_view_position_from_depth, ssao_generation.inl:128-135 */
static inline v3 view_position_from_depth(const float* inv_proj, v2 uv, float depth) {
    v4 c = V4(uv.x * 2.0f - 1.0f, uv.y * 2.0f - 1.0f, depth, 1.0f);
    v4 v = mat4_mul_v4(inv_proj, c);
    return V3(v.x / v.w, v.y / v.w, v.z / v.w);
}

/* rv_table: NULL (the reference's random vector, :184-188) or a (target.width x target.height) table of (x, y) random
   vectors to use instead (the conditional parity check: the GPU's table, i.e. the oracle's taps given the GPU's Q8 hash). */
static int ssao_generation(const soc_globals* g, soc_img depth, soc_img normal, soc_img target, const float* rv_table) {
    if (!g || !valid(&depth) || !valid(&normal) || !valid(&target) || depth.format != SOC_FMT_D32F ||
        normal.format != SOC_FMT_RGBA16F || target.format != SOC_FMT_R8_UNORM)
        return SOC_E_INVALID_ARG;
    const int ksize = g->ssao_kernel_size < SOC_SSAO_MAX_KERNEL ? g->ssao_kernel_size : SOC_SSAO_MAX_KERNEL;
    const float radius = g->ssao_radius, bias = g->ssao_bias;
    const float* ip = g->camera_inverse_projection_matrix;
    const float* P = g->camera_projection_matrix;
    const float* V = g->camera_view_matrix;
    /* textureSize(u_normal_image) (both tex_dim and noise_dim, :180-181) */
    const int ndx = normal.width;
#pragma omp parallel for schedule(dynamic, 4)
    for (int y = 0; y < target.height; ++y) {
        for (int x = 0; x < target.width; ++x) {
            const v2 uv = V2(((float)x + 0.5f) / (float)target.width, ((float)y + 0.5f) / (float)target.height);
            v3 frag = view_position_from_depth(ip, uv, sample_clamp(&depth, uv.x, uv.y).x);
            v4 nn = sample_clamp(&normal, uv.x, uv.y);
            v3 n = mat3of4_mul_v3(V, normalize3(V3(nn.x, nn.y, nn.z)));
            /* random_vec, :184-188 */
            v3 rv;
            if (rv_table) {
                const float* e = rv_table + 2 * ((size_t)y * (size_t)target.width + (size_t)x);
                rv = V3(e[0], e[1], 0.0f);
            } else {
                float n1 = ssao_noise(uv, (float)(ndx * 2));
                v2 puv = V2(det_pow(uv.x, 1.1f), det_pow(uv.y, 1.1f));
                float n2 = ssao_noise(puv, det_pow((float)ndx * 4.2f, 1.5f + uv.x / 10.0f));
                rv = normalize3(V3(n1, n2, 0.0f));
            }
            v3 t = normalize3(sub3(rv, muls3(n, dot3(rv, n))));
            v3 b = cross3(t, n);
            float occ = 0.0f;
            for (int i = 0; i < ksize; ++i) {
                const float* k = k_ssao_kernel[i];
                v3 s = add3(add3(muls3(t, k[0]), muls3(b, k[1])), muls3(n, k[2])); /* TBN * k */
                s = add3(frag, muls3(s, radius));
                v4 off = mat4_mul_v4(P, V4(s.x, s.y, s.z, 1.0f));
                float ox = off.x / off.w, oy = off.y / off.w;
                ox = ox * 0.5f + 0.5f;
                oy = oy * 0.5f + 0.5f;
                float sd = view_position_from_depth(ip, V2(ox, oy), sample_clamp(&depth, ox, oy).x).z;
                float range = smoothstepf(0.0f, 1.0f, radius / fabsf(frag.z - sd));
                occ += (sd >= s.z + bias ? 1.0f : 0.0f) * range;
            }
            occ = 1.0f - (occ / (float)g->ssao_kernel_size);
            store(&target, x, y, V4(occ, 0, 0, 1));
        }
    }
    return SOC_OK;
}

int soc_oracle_ssao_generation(const soc_globals* g, soc_img depth, soc_img normal, soc_img target) {
    return ssao_generation(g, depth, normal, target, NULL);
}

int soc_oracle_ssao_generation_rv(const soc_globals* g, soc_img depth, soc_img normal, const float* rv_table,
                                  soc_img target) {
    if (!rv_table) return SOC_E_INVALID_ARG;
    return ssao_generation(g, depth, normal, target, rv_table);
}

/* The oracle's per-pixel random vectors (x, y) of a (tw x th) SSAO target (the :184-188 expression above, uv at the
   target's pixel centres, noise frequency from the normal image's width), for comparing with a GPU table (Q8). */
int soc_oracle_ssao_random_vectors(int32_t normal_width, int32_t tw, int32_t th, float* out) {
    if (normal_width <= 0 || tw <= 0 || th <= 0 || !out) return SOC_E_INVALID_ARG;
#pragma omp parallel for schedule(static)
    for (int y = 0; y < th; ++y)
        for (int x = 0; x < tw; ++x) {
            const v2 uv = V2(((float)x + 0.5f) / (float)tw, ((float)y + 0.5f) / (float)th);
            float n1 = ssao_noise(uv, (float)(normal_width * 2));
            v2 puv = V2(det_pow(uv.x, 1.1f), det_pow(uv.y, 1.1f));
            float n2 = ssao_noise(puv, det_pow((float)normal_width * 4.2f, 1.5f + uv.x / 10.0f));
            v3 rv = normalize3(V3(n1, n2, 0.0f));
            out[2 * ((size_t)y * (size_t)tw + (size_t)x)] = rv.x;
            out[2 * ((size_t)y * (size_t)tw + (size_t)x) + 1] = rv.y;
        }
    return SOC_OK;
}

int soc_oracle_ssao_blur(const soc_globals* g, soc_img ssao, soc_img target) {
    (void)g;
    if (!valid(&ssao) || !valid(&target) || ssao.format != SOC_FMT_R8_UNORM || target.format != SOC_FMT_R8_UNORM)
        return SOC_E_INVALID_ARG;
    const float tx = 1.0f / (float)ssao.width, ty = 1.0f / (float)ssao.height;
#pragma omp parallel for schedule(static)
    for (int y = 0; y < target.height; ++y) {
        for (int x = 0; x < target.width; ++x) {
            const float u = ((float)x + 0.5f) / (float)target.width, v = ((float)y + 0.5f) / (float)target.height;
            float result = 0.0f;
            int n = 0;
            for (int dx = -2; dx < 2; ++dx)
                for (int dy = -2; dy < 2; ++dy) {
                    result += sample_clamp(&ssao, u + (float)dx * tx, v + (float)dy * ty).x;
                    n++;
                }
            store(&target, x, y, V4(result / (float)n, 0, 0, 1));
        }
    }
    return SOC_OK;
}

/* ------------------------------------------------------------------------------------------------ */
/* Composition (composition.inl:110-225)                                                             */
/* ------------------------------------------------------------------------------------------------ */
static v3 point_light(const soc_point_light* L, v3 frag_color, v3 normal, v3 pos, v3 cam) {
    v3 lp = V3(L->position[0], L->position[1], L->position[2]);
    v3 light_dir = normalize3(sub3(lp, pos));
    float distance = length3(sub3(lp, pos));
    float attenuation = 1.0f / (distance * distance);
    v3 view_dir = normalize3(sub3(cam, pos));
    v3 halfway = normalize3(add3(light_dir, view_dir));
    float diffuse = fmaxf(dot3(normal, light_dir), 0.0f);
    float nh = acosf(dot3(halfway, normal));
    float ex = nh * 1.0f;
    ex = -(ex * ex);
    v3 lc = V3(L->color[0], L->color[1], L->color[2]);
    return muls3(muls3(muls3(mul3(frag_color, lc), diffuse + expf(ex)), attenuation), L->intensity);
}

static v3 spot_light(const soc_spot_light* L, v3 frag_color, v3 normal, v3 pos, v3 cam) {
    v3 lp = V3(L->position[0], L->position[1], L->position[2]);
    v3 light_dir = normalize3(sub3(lp, pos));
    float theta = dot3(light_dir, normalize3(neg3(V3(L->direction[0], L->direction[1], L->direction[2]))));
    float epsilon = L->cut_off - L->outer_cut_off;
    float intensity = clampf((theta - L->outer_cut_off) / epsilon, 0.0f, 1.0f);
    float distance = length3(sub3(lp, pos));
    float attenuation = 1.0f / (distance * distance);
    v3 view_dir = normalize3(sub3(cam, pos));
    v3 halfway = normalize3(add3(light_dir, view_dir));
    float diffuse = fmaxf(dot3(normal, light_dir), 0.0f);
    float nh = acosf(dot3(halfway, normal));
    float ex = nh / 1.0f;
    ex = -(ex * ex);
    v3 lc = V3(L->color[0], L->color[1], L->color[2]);
    return muls3(muls3(muls3(muls3(mul3(frag_color, lc), diffuse + expf(ex)), attenuation), L->intensity), intensity);
}

int soc_oracle_composition(const soc_globals* g, soc_img target, soc_img albedo, soc_img emissive, soc_img normal,
                           soc_img depth, soc_img ssao, soc_img shadow, soc_img clouds) {
    if (!g || !valid(&target) || !valid(&albedo) || !valid(&emissive) || !valid(&normal) || !valid(&depth) ||
        !valid(&ssao) || !valid(&shadow) || !valid(&clouds))
        return SOC_E_INVALID_ARG;
    float sun_pv[16];
    mat4_mul(sun_pv, g->sun_info.projection_matrix, g->sun_info.view_matrix); /* (P * V) * v, :166 */
    const v3 sun_dir = V3(g->sun_info.direction[0], g->sun_info.direction[1], g->sun_info.direction[2]);
    const v3 cam = V3(g->camera_position[0], g->camera_position[1], g->camera_position[2]);
    const v3 ambient = V3(g->ambient[0], g->ambient[1], g->ambient[2]);
    const uint32_t npl = g->point_light_count < SOC_MAX_POINT_LIGHTS ? g->point_light_count : SOC_MAX_POINT_LIGHTS;
    const uint32_t nsl = g->spot_light_count < SOC_MAX_SPOT_LIGHTS ? g->spot_light_count : SOC_MAX_SPOT_LIGHTS;
#pragma omp parallel for schedule(static)
    for (int y = 0; y < target.height; ++y) {
        for (int x = 0; x < target.width; ++x) {
            const v2 uv = V2(((float)x + 0.5f) / (float)target.width, ((float)y + 0.5f) / (float)target.height);
            const float d = sample_clamp(&depth, uv.x, uv.y).x;
            /* get_world_position_from_depth, :114-122 */
            v4 c = V4(uv.x * 2.0f - 1.0f, uv.y * 2.0f - 1.0f, d, 1.0f);
            v4 vs = mat4_mul_v4(g->camera_inverse_projection_matrix, c);
            vs = V4(vs.x / vs.w, vs.y / vs.w, vs.z / vs.w, vs.w / vs.w);
            v4 ws = mat4_mul_v4(g->camera_inverse_view_matrix, vs);
            const v3 wp = V3(ws.x, ws.y, ws.z);
            v4 sp = mat4_mul_v4(sun_pv, V4(wp.x, wp.y, wp.z, 1.0f));
            v3 pc = V3(sp.x / sp.w, sp.y / sp.w, sp.z / sp.w);
            pc = V3(pc.x * 0.5f + 0.5f, pc.y * 0.5f + 0.5f, pc.z);
            const float sd = sample_clamp(&shadow, pc.x, pc.y).x;
            const float sun_shadow =
                clampf(powf(expf(g->sun_info.exponential_factor * (pc.z - sd)), g->sun_info.darkening_factor), 0.0f, 1.0f);
            /* volumetric fog (:176-195) is computed then zeroed at :196 — dead, omitted */
            v4 em = sample_clamp(&emissive, uv.x, uv.y);
            v3 e = muls3(V3(em.x, em.y, em.z), g->emissive_bloom_strength);
            v4 al = sample_clamp(&albedo, uv.x, uv.y);
            v3 a = V3(al.x, al.y, al.z);
            v4 nn = sample_clamp(&normal, uv.x, uv.y);
            v3 n = V3(nn.x, nn.y, nn.z);
            float occl = powf(sample_clamp(&ssao, uv.x, uv.y).x, g->ambient_occlussion_strength);
            float dd = fmaxf(0.0f, dot3(n, neg3(sun_dir))) * sun_shadow;
            v3 direct = V3(dd, dd, dd);
            for (uint32_t i = 0; i < npl; ++i) direct = add3(direct, point_light(&g->point_lights[i], a, n, wp, cam));
            for (uint32_t i = 0; i < nsl; ++i) direct = add3(direct, spot_light(&g->spot_lights[i], a, n, wp, cam));
            v3 color = add3(muls3(mul3(add3(direct, ambient), a), occl), e);
            if (d == 1.0f) {
                v4 cl = sample_clamp(&clouds, uv.x, uv.y);
                color = V3(cl.x, cl.y, cl.z);
            }
            store(&target, x, y, V4(color.x, color.y, color.z, 1.0f));
        }
    }
    return SOC_OK;
}

/* ------------------------------------------------------------------------------------------------ */
/* Luminance histogram (generate_luminance_histogram.inl:59-78) and resolve (:56-80)                 */
/* ------------------------------------------------------------------------------------------------ */
int soc_oracle_generate_luminance_histogram(const soc_globals* g, soc_img hdr, soc_auto_exposure* ae) {
    if (!g || !ae || !valid(&hdr)) return SOC_E_INVALID_ARG;
    const int W = g->resolution[0] < hdr.width ? g->resolution[0] : hdr.width;
    const int H = g->resolution[1] < hdr.height ? g->resolution[1] : hdr.height;
    uint64_t bins[SOC_AUTO_EXPOSURE_BIN_COUNT];
    memset(bins, 0, sizeof bins);
#pragma omp parallel
    {
        uint64_t local[SOC_AUTO_EXPOSURE_BIN_COUNT];
        memset(local, 0, sizeof local);
#pragma omp for schedule(static)
        for (int y = 0; y < H; ++y)
            for (int x = 0; x < W; ++x) {
                v4 c = fetch(&hdr, x, y); /* texelFetch */
                local[soc_oracle_luminance_bin(c.x, c.y, c.z, g->log_min_luminance, g->log_max_luminance)]++;
            }
#pragma omp critical
        for (int i = 0; i < SOC_AUTO_EXPOSURE_BIN_COUNT; ++i) bins[i] += local[i];
    }
    for (int i = 0; i < SOC_AUTO_EXPOSURE_BIN_COUNT; ++i) ae->histogram_buckets[i] += (uint32_t)bins[i];
    return SOC_OK;
}

int soc_oracle_resolve_luminance_histogram(const soc_globals* g, soc_auto_exposure* ae, uint64_t total_pixels,
                                           int32_t wide) {
    if (!g || !ae) return SOC_E_INVALID_ARG;
    const uint32_t bin0 = ae->histogram_buckets[0];
    float sum_f;
    if (wide) {
        uint64_t s = 0;
        for (uint32_t i = 0; i < SOC_AUTO_EXPOSURE_BIN_COUNT; ++i) s += (uint64_t)ae->histogram_buckets[i] * i;
        sum_f = (float)s;
    } else {
        /* shared_buckets[i] = bin_count * i (u32), tree reduction (u32 wrap), :58-70 */
        uint32_t sh[SOC_AUTO_EXPOSURE_BIN_COUNT];
        for (uint32_t i = 0; i < SOC_AUTO_EXPOSURE_BIN_COUNT; ++i) sh[i] = ae->histogram_buckets[i] * i;
        for (uint32_t th = SOC_AUTO_EXPOSURE_BIN_COUNT / 2; th > 0; th /= 2)
            for (uint32_t i = 0; i < th; ++i) sh[i] += sh[i + th];
        sum_f = (float)sh[0];
    }
    for (int i = 0; i < SOC_AUTO_EXPOSURE_BIN_COUNT; ++i) ae->histogram_buckets[i] = 0;
    float pixels;
    if (total_pixels) pixels = (float)total_pixels;
    else pixels = (float)(int32_t)((uint32_t)g->resolution[0] * (uint32_t)g->resolution[1]);
    float denom = fmaxf(pixels - (float)bin0, 1.0f);
    float x = sum_f / denom;
    /* remap(x, 1, 256, log_min, log_max) */
    float log2_mean = (x - 1.0f) / (256.0f - 1.0f) * (g->log_max_luminance - g->log_min_luminance) + g->log_min_luminance;
    float target = log2f(g->target_luminance / exp2f(log2_mean));
    float alpha = clampf(1.0f - expf(-g->delta_time * g->adjustment_speed), 0.0f, 1.0f);
    ae->exposure = mixf(ae->exposure, target, alpha);
    return SOC_OK;
}

/* ------------------------------------------------------------------------------------------------ */
/* TAA (temporal_antialiasing.inl:137-190)                                                           */
/* ------------------------------------------------------------------------------------------------ */
int soc_oracle_temporal_antialiasing(const soc_globals* g, soc_img target, soc_img cur, soc_img prev, soc_img vel,
                                     soc_img pvel, soc_img depth) {
    if (!g || !valid(&target) || !valid(&cur) || !valid(&prev) || !valid(&vel) || !valid(&pvel) || !valid(&depth))
        return SOC_E_INVALID_ARG;
    static const float gauss[9] = {1.0f / 16.0f, 1.0f / 8.0f, 1.0f / 16.0f, 1.0f / 8.0f, 1.0f / 4.0f,
                                   1.0f / 8.0f,  1.0f / 16.0f, 1.0f / 8.0f, 1.0f / 16.0f};
    const float pox = 1.0f / (float)g->resolution[0], poy = 1.0f / (float)g->resolution[1];
    const float accum0 = fminf(0.1f, (float)g->frame_counter);
#pragma omp parallel for schedule(static)
    for (int y = 0; y < target.height; ++y) {
        for (int x = 0; x < target.width; ++x) {
            const v2 uv = V2(((float)x + 0.5f) / (float)target.width, ((float)y + 0.5f) / (float)target.height);
            v4 nb[9];
            v4 blurred = V4(0, 0, 0, 0);
            float closest = 1.0f;
            v2 duv = uv;
            v4 mn = V4(10.0e5f, 10.0e5f, 10.0e5f, 10.0e5f), mx = V4(-10.0e5f, -10.0e5f, -10.0e5f, -10.0e5f);
            for (int oy = 1; oy > -2; --oy)
                for (int ox = 1; ox > -2; --ox) {
                    int idx = (oy + 1) * 3 + (ox + 1);
                    v2 s = V2(uv.x + pox * (float)ox, uv.y + poy * (float)oy);
                    nb[idx] = sample_clamp(&cur, s.x, s.y);
                    float dd = sample_clamp(&depth, s.x, s.y).x;
                    closest = fminf(dd, closest);
                    if (closest == dd) duv = s;
                    mn = V4(fminf(nb[idx].x, mn.x), fminf(nb[idx].y, mn.y), fminf(nb[idx].z, mn.z), fminf(nb[idx].w, mn.w));
                    mx = V4(fmaxf(nb[idx].x, mx.x), fmaxf(nb[idx].y, mx.y), fmaxf(nb[idx].z, mx.z), fmaxf(nb[idx].w, mx.w));
                    blurred = V4(blurred.x + gauss[idx] * nb[idx].x, blurred.y + gauss[idx] * nb[idx].y,
                                 blurred.z + gauss[idx] * nb[idx].z, blurred.w + gauss[idx] * nb[idx].w);
                }
            v4 color = nb[5]; /* quirk Q7: the (+1, 0) neighbour */
            v4 vv = sample_clamp(&vel, duv.x, duv.y);
            float accum = accum0;
            v2 vs = V2(uv.x - vv.x, uv.y - vv.y);
            v4 acc = sample_clamp(&prev, vs.x, vs.y);
            if (vs.x < 0.0f || vs.y < 0.0f || vs.x > 1.0f || vs.y > 1.0f) accum = 1.0f;
            acc = V4(clampf(acc.x, mn.x, mx.x), clampf(acc.y, mn.y, mx.y), clampf(acc.z, mn.z, mx.z), clampf(acc.w, mn.w, mx.w));
            v4 o = V4(color.x * accum + acc.x * (1.0f - accum), color.y * accum + acc.y * (1.0f - accum),
                      color.z * accum + acc.z * (1.0f - accum), color.w * accum + acc.w * (1.0f - accum));
            v4 pv = sample_clamp(&pvel, vs.x, vs.y);
            float dvx = pv.x - vv.x, dvy = pv.y - vv.y;
            float vlen = sqrtf(dvx * dvx + dvy * dvy);
            float dis = clampf((vlen - 0.001f) * 10.0f, 0.0f, 1.0f);
            o = V4(mixf(o.x, blurred.x, dis), mixf(o.y, blurred.y, dis), mixf(o.z, blurred.z, dis), mixf(o.w, blurred.w, dis));
            store(&target, x, y, o);
        }
    }
    return SOC_OK;
}

/* ------------------------------------------------------------------------------------------------ */
/* Tone mapping, AgX-DS (tone_mapping.inl:91-176)                                                    */
/* ------------------------------------------------------------------------------------------------ */
static v3 xyY_to_XYZ(v3 xyY) {
    float Y = xyY.z;
    float X = (xyY.x * Y) / xyY.y;
    float Z = ((1.0f - xyY.x - xyY.y) * Y) / xyY.y;
    return V3(X, Y, Z);
}
static v3 unproject(v2 xy) { return xyY_to_XYZ(V3(xy.x, xy.y, 1.0f)); }
static void primaries_to_matrix(float* out, v2 r, v2 gr, v2 b, v2 w) {
    v3 R = unproject(r), G = unproject(gr), B = unproject(b), Wt = unproject(w);
    float temp[9] = {R.x, 1.0f, R.z, G.x, 1.0f, G.z, B.x, 1.0f, B.z};
    float it[9];
    mat3_inverse(it, temp);
    v3 scale = mat3_mul_v3(it, Wt);
    v3 c0 = muls3(R, scale.x), c1 = muls3(G, scale.y), c2 = muls3(B, scale.z);
    float m[9] = {c0.x, c0.y, c0.z, c1.x, c1.y, c1.z, c2.x, c2.y, c2.z};
    memcpy(out, m, sizeof m);
}
static v2 mix2(v2 a, v2 b, float t) { return V2(mixf(a.x, b.x, t), mixf(a.y, b.y, t)); }

static float dual_section(float x, float linear, float peak) {
    float S = peak * linear;
    if (x < S) return x;
    float C = peak / (peak - S);
    return peak - (peak - S) * expf((-C * (x - S)) / peak);
}

int soc_oracle_tone_mapping(const soc_globals* g, soc_img color, const soc_auto_exposure* ae, soc_img target) {
    if (!g || !ae || !valid(&color) || !valid(&target)) return SOC_E_INVALID_ARG;
    const v2 xr = V2(0.64f, 0.33f), xg = V2(0.3f, 0.6f), xb = V2(0.15f, 0.06f), xw = V2(0.3127f, 0.3290f);
    float srgb_to_xyz[9], adjusted_to_xyz[9], xyz_to_adjusted[9], M[9], Minv[9];
    primaries_to_matrix(srgb_to_xyz, xr, xg, xb, xw);
    const float sf = 1.0f / (1.0f - g->compression);
    primaries_to_matrix(adjusted_to_xyz, mix2(xw, xr, sf), mix2(xw, xg, sf), mix2(xw, xb, sf), xw);
    mat3_inverse(xyz_to_adjusted, adjusted_to_xyz);
    mat3_mul(M, srgb_to_xyz, xyz_to_adjusted);
    mat3_inverse(Minv, M);
    const float expo = powf(2.0f, ae->exposure);
    const float lin = g->agxDs_linear_section, peak = g->peak, sat = g->saturation;
#pragma omp parallel for schedule(static)
    for (int y = 0; y < target.height; ++y) {
        for (int x = 0; x < target.width; ++x) {
            const float u = ((float)x + 0.5f) / (float)target.width, v = ((float)y + 0.5f) / (float)target.height;
            v4 c = sample_clamp(&color, u, v);
            v3 w = muls3(V3(fmaxf(c.x, 0.0f), fmaxf(c.y, 0.0f), fmaxf(c.z, 0.0f)), expo);
            w = mat3_mul_v3(M, w);
            w = V3(clampf(dual_section(w.x, lin, peak), 0.0f, 1.0f), clampf(dual_section(w.y, lin, peak), 0.0f, 1.0f),
                   clampf(dual_section(w.z, lin, peak), 0.0f, 1.0f));
            float ds = dot3(w, V3(0.2126729f, 0.7151522f, 0.0721750f));
            w = mix3(V3(ds, ds, ds), w, sat);
            w = V3(clampf(w.x, 0.0f, 1.0f), clampf(w.y, 0.0f, 1.0f), clampf(w.z, 0.0f, 1.0f));
            w = mat3_mul_v3(Minv, w);
            store(&target, x, y, V4(w.x, w.y, w.z, 1.0f));
        }
    }
    return SOC_OK;
}

/* ------------------------------------------------------------------------------------------------ */
/* Atmosphere + volumetric clouds (cloud_rendering.inl:65-481)                                       */
/* ------------------------------------------------------------------------------------------------ */
#define CL_EARTH_RADIUS 6371000.0f
#define CL_MIN_H 1600.0f
#define CL_MAX_H (500.0f + 1600.0f)
#define CL_SUN_BRIGHTNESS 3.0f

typedef struct {
    const soc_img* noise;
    const soc_globals* g;
    uint64_t* counters; /* per-thread tallies (tools/clouds_flops.py): [0] sky px, [1] dense steps, [2] get_clouds,
                           [3] noise taps, [4] get_clouds past the altitude test, [5] full atmosphere evaluations (not
                           the early exit of :359), [6] cloud marches (ray_direction.y >= 0, :311) */
} cloud_ctx;

static inline float bayer2(v2 a) {
    a = V2(floorf(a.x), floorf(a.y));
    return fractf(a.x * 0.5f + a.y * (a.y * 0.75f));
}
static inline float bayer4(v2 a) { return bayer2(V2(0.5f * a.x, 0.5f * a.y)) * 0.25f + bayer2(a); }
static inline float bayer8(v2 a) { return bayer4(V2(0.5f * a.x, 0.5f * a.y)) * 0.25f + bayer2(a); }
static inline float bayer16(v2 a) { return bayer8(V2(0.5f * a.x, 0.5f * a.y)) * 0.25f + bayer2(a); }

static inline v2 rsi(v3 p, v3 d, float radius) {
    float PoD = dot3(p, d);
    float r2 = radius * radius;
    float delta = PoD * PoD + r2 - dot3(p, p);
    if (delta < 0.0f) return V2(-1.0f, -1.0f);
    delta = sqrtf(delta);
    return V2(-PoD - delta, -PoD + delta);
}

static float get_3d_noise(cloud_ctx* cx, v3 pos) {
    float p = floorf(pos.z);
    float f = pos.z - p;
    const float inv = 1.0f / 64.0f;
    const float zs = 17.0f * inv;
    v2 coord = V2(pos.x * inv + p * zs, pos.y * inv + p * zs);
    float a = sample_repeat(cx->noise, coord.x, coord.y).x;
    float b = sample_repeat(cx->noise, coord.x + zs, coord.y + zs).x;
    cx->counters[3] += 2;
    return mixf(a, b, f);
}

static float get_clouds(cloud_ctx* cx, v3 p) {
    cx->counters[2]++;
    p = V3(p.x, length3(add3(p, V3(0.0f, CL_EARTH_RADIUS, 0.0f))) - CL_EARTH_RADIUS, p.z);
    p.x += cx->g->camera_position[0];
    p.z += cx->g->camera_position[2];
    if (p.y < CL_MIN_H || p.y > CL_MAX_H) return 0.0f;
    cx->counters[4]++;
    float time = -1.0f * 0.02f * cx->g->elapsed_time;
    v3 mv = V3(time, 0.0f, time);
    v3 cc = add3(muls3(p, 0.001f), mv);
    float noise = get_3d_noise(cx, cc) * 0.5f;
    noise += get_3d_noise(cx, add3(muls3(cc, 2.0f), mv)) * 0.25f;
    noise += get_3d_noise(cx, sub3(muls3(cc, 7.0f), mv)) * 0.125f;
    noise += get_3d_noise(cx, muls3(add3(cc, mv), 16.0f)) * 0.0625f;
    const float top = 0.004f, bottom = 0.01f;
    float hh = p.y - CL_MIN_H;
    float th = (1.0f - expf(-bottom * hh)) * expf(-top * hh);
    float clouds = smoothstepf(0.55f, 0.6f, noise);
    clouds *= th;
    return clouds * 0.03f;
}

static float get_sun_visibility(cloud_ctx* cx, v3 p, v3 sun) {
    const int steps = 10;
    const float rSteps = 500.0f / (float)steps;
    v3 inc = muls3(sun, rSteps);
    v3 pos = add3(muls3(inc, 0.5f), p);
    float tr = 0.0f;
    for (int i = 0; i < steps; i++, pos = add3(pos, inc)) tr += get_clouds(cx, pos);
    return expf(-tr * rSteps);
}

static inline float hg_phase(float x, float g) {
    float g2 = g * g;
    return 0.25f * ((1.0f - g2) * powf(1.0f + g2 - 2.0f * g * x, -1.5f));
}
static inline float phase_two_lobes(float x) {
    const float m = 0.5f, gm = 0.8f;
    float l1 = hg_phase(x, 0.8f * gm), l2 = hg_phase(x, -0.5f * gm);
    return mixf(l2, l1, m);
}

static v3 atmospheric_scattering_top(v3 sun) {
    const float ln2 = logf(2.0f);
    const v3 rayleigh = V3(0.27f * 1e-5f, 0.5f * 1e-5f, 1.0f * 1e-5f);
    const v3 mie = V3(0.5e-6f, 0.5e-6f, 0.5e-6f);
    const v3 total = add3(rayleigh, mie);
    float lDotU = dot3(sun, V3(0.0f, 1.0f, 0.0f));
    float od = 100000.0f / fmaxf(1.0f * 2.0f - 0.01f, 0.01f);
    float dl = lDotU * 2.0f;
    dl = fmaxf(dl + 0.01f, 0.01f);
    dl = 1.0f / dl;
    float odl = 100000.0f * dl;
    v3 sv = muls3(total, od), av = exp3(muls3(total, -od));
    v3 sl = muls3(total, odl), al = exp3(muls3(total, -odl));
    v3 num = sub3(al, av), den = muls3(sub3(sl, sv), ln2);
    v3 absorb_sun = V3((fabsf(num.x) + 1e-3f) / (fabsf(den.x) + 1e-3f), (fabsf(num.y) + 1e-3f) / (fabsf(den.y) + 1e-3f),
                       (fabsf(num.z) + 1e-3f) / (fabsf(den.z) + 1e-3f));
    v3 ms = muls3(muls3(mie, od), 0.25f);
    v3 rs = muls3(muls3(rayleigh, od), 0.375f);
    return muls3(mul3(add3(ms, rs), absorb_sun), CL_SUN_BRIGHTNESS);
}

static v3 volumetric_clouds(cloud_ctx* cx, v3 dir, v3 sun, v3 color, float dither, v3 sun_color) {
    const int steps = 24;
    const float iSteps = 1.0f / (float)steps;
    if (dir.y < 0.0f) return color;
    cx->counters[6]++;
    const float pi = acosf(-1.0f), rPi = 1.0f / pi, hPi = pi * 0.5f, rLOG2 = 1.0f / logf(2.0f);
    v3 c0 = muls3(V3(0.0f, 1.0f, 0.0f), CL_EARTH_RADIUS);
    float bottom = rsi(c0, dir, CL_EARTH_RADIUS + CL_MIN_H).y;
    float top = rsi(c0, dir, CL_EARTH_RADIUS + CL_MAX_H).y;
    v3 start = muls3(dir, bottom), end = muls3(dir, top);
    v3 inc = muls3(sub3(end, start), iSteps);
    v3 cp = add3(muls3(inc, dither), start);
    float stepLength = length3(inc);
    v3 scattering = V3(0, 0, 0);
    float transmittance = 1.0f;
    float phase = phase_two_lobes(dot3(sun, dir));
    v3 sky = atmospheric_scattering_top(sun);
    for (int i = 0; i < steps; i++, cp = add3(cp, inc)) {
        float od = get_clouds(cx, cp) * stepLength;
        if (od <= 0.0f) continue;
        cx->counters[1]++;
        /* get_volumetric_cloud_scattering, :290-299 */
        const float coeff = 1.11f;
        float ia = -coeff * rLOG2, ib = -1.0f / coeff, ic = 1.0f / coeff;
        float integral = expf(ia * od) * ib + ic;
        float beers = 1.0f - expf(-(od * logf(2.0f)) * 2.0f);
        float vis = get_sun_visibility(cx, cp, sun);
        /* (sunColor * vis * beers) * phase * hPi * sunBrightness — restated left to right */
        v3 sunl = muls3(muls3(muls3(muls3(muls3(sun_color, vis), beers), phase), hPi), CL_SUN_BRIGHTNESS);
        v3 skyl = muls3(muls3(sky, 0.25f), rPi);
        v3 sc = muls3(muls3(add3(sunl, skyl), integral), pi);
        scattering = add3(scattering, muls3(sc, transmittance));
        transmittance *= expf(-od);
    }
    v3 lit = add3(muls3(color, transmittance), scattering);
    return mix3(lit, color, clampf(length3(start) * 0.00001f * 2.5f, 0.0f, 1.0f));
}

static v3 atmosphere(cloud_ctx* cx, const soc_globals* g, v3 r, v3 r0, v3 pSun, float iSun, float rPlanet, float rAtmos, v3 kRlh,
                     float kMie, float shRlh, float shMie, float gg0) {
    const float PI = 3.141592f;
    r = normalize3(r);
    v2 p = rsi(r0, r, rAtmos);
    if (p.x > p.y) return V3(0, 0, 0);
    cx->counters[5]++;
    p.y = fminf(p.y, rsi(r0, r, rPlanet).x);
    float iStepSize = (p.y - p.x) / 16.0f;
    float iTime = g->elapsed_time; /* quirk Q10 */
    v3 totalRlh = V3(0, 0, 0), totalMie = V3(0, 0, 0);
    float iOdRlh = 0.0f, iOdMie = 0.0f;
    float mu = dot3(r, pSun);
    float mumu = mu * mu;
    float gg = gg0 * gg0;
    float pRlh = 3.0f / (16.0f * PI) * (1.0f + mumu);
    float pMie = 3.0f / (8.0f * PI) * ((1.0f - gg) * (mumu + 1.0f)) / (powf(1.0f + gg - 2.0f * mu * gg0, 1.5f) * (2.0f + gg));
    for (int i = 0; i < 16; i++) {
        v3 iPos = add3(r0, muls3(r, iTime + iStepSize * 0.5f));
        float iHeight = length3(iPos) - rPlanet;
        float odStepRlh = expf(-iHeight / shRlh) * iStepSize;
        float odStepMie = expf(-iHeight / shMie) * iStepSize;
        iOdRlh += odStepRlh;
        iOdMie += odStepMie;
        float jStepSize = rsi(iPos, pSun, rAtmos).y / 8.0f;
        float jTime = 0.0f, jOdRlh = 0.0f, jOdMie = 0.0f;
        for (int j = 0; j < 8; j++) {
            v3 jPos = add3(iPos, muls3(pSun, jTime + jStepSize * 0.5f));
            float jHeight = length3(jPos) - rPlanet;
            jOdRlh += expf(-jHeight / shRlh) * jStepSize;
            jOdMie += expf(-jHeight / shMie) * jStepSize;
            jTime += jStepSize;
        }
        float fm = kMie * (iOdMie + jOdMie);
        float fr = iOdRlh + jOdRlh;
        v3 attn = exp3(neg3(V3(fm + kRlh.x * fr, fm + kRlh.y * fr, fm + kRlh.z * fr)));
        totalRlh = add3(totalRlh, muls3(attn, odStepRlh));
        totalMie = add3(totalMie, muls3(attn, odStepMie));
        iTime += iStepSize;
    }
    v3 a = mul3(muls3(kRlh, pRlh), totalRlh);
    v3 b = muls3(totalMie, pMie * kMie);
    return muls3(add3(a, b), iSun);
}

static uint64_t g_cloud_counters[SOC_ORACLE_CLOUD_COUNTERS];

void soc_oracle_clouds_counters(uint64_t out[SOC_ORACLE_CLOUD_COUNTERS]) {
    memcpy(out, g_cloud_counters, sizeof g_cloud_counters);
}

int soc_oracle_cloud_rendering(const soc_globals* g, soc_img depth, soc_img noise, soc_img target) {
    if (!g || !valid(&depth) || !valid(&noise) || !valid(&target)) return SOC_E_INVALID_ARG;
    const int W = g->resolution[0] < target.width ? g->resolution[0] : target.width;
    const int H = g->resolution[1] < target.height ? g->resolution[1] : target.height;
    const v3 sun = V3(-g->sun_info.direction[0], -g->sun_info.direction[1], -g->sun_info.direction[2]);
    const v3 r0 = V3(0.0f + g->camera_position[0], 6372e3f + g->camera_position[1], 0.0f + g->camera_position[2]);
    const float sun_factor = fmaxf(fminf(fabsf(sun.x), fabsf(sun.z)) + sun.y, 0.0f);
    uint64_t c0 = 0, c1 = 0, c2 = 0, c3 = 0, c4 = 0, c5 = 0, c6 = 0;
#pragma omp parallel for schedule(dynamic, 2) reduction(+ : c0, c1, c2, c3, c4, c5, c6)
    for (int y = 0; y < H; ++y) {
        uint64_t cnt[SOC_ORACLE_CLOUD_COUNTERS] = {0};
        cloud_ctx cx = {&noise, g, cnt};
        for (int x = 0; x < W; ++x) {
            v2 ruv = V2((float)x / ((float)g->resolution[0] - 1.0f), (float)y / ((float)g->resolution[1] - 1.0f));
            v2 ndc = V2(ruv.x * 2.0f - 1.0f, ruv.y * 2.0f - 1.0f);
            v4 rvs = mat4_mul_v4(g->camera_inverse_projection_matrix, V4(ndc.x, ndc.y, -1.0f, 0.0f));
            v4 rws = mat4_mul_v4(g->camera_inverse_view_matrix, V4(rvs.x, rvs.y, -1.0f, 0.0f));
            v3 dir = normalize3(V3(rws.x, rws.y, rws.z));
            v3 color = V3(0.2f, 0.4f, 1.0f);
            float d = sample_clamp(&depth, ruv.x, ruv.y).x;
            if (d == 1.0f) {
                cnt[0]++;
                float dither = bayer16(V2((float)x, (float)y));
                color = atmosphere(&cx, g, dir, r0, sun, 22.0f, 6371e3f, 6471e3f, V3(5.5e-6f, 13.0e-6f, 22.4e-6f), 21e-6f, 8e3f,
                                   1.2e3f, 0.758f);
                color = volumetric_clouds(&cx, dir, sun, color, dither, V3(0.8f, 0.8f, 0.8f));
                color = muls3(color, sun_factor);
            }
            store(&target, x, y, V4(color.x, color.y, color.z, 1.0f));
        }
        c0 += cnt[0]; c1 += cnt[1]; c2 += cnt[2]; c3 += cnt[3]; c4 += cnt[4]; c5 += cnt[5]; c6 += cnt[6];
    }
    const uint64_t all[SOC_ORACLE_CLOUD_COUNTERS] = {c0, c1, c2, c3, c4, c5, c6, (uint64_t)W * (uint64_t)H};
    memcpy(g_cloud_counters, all, sizeof all);
    return SOC_OK;
}

/* ------------------------------------------------------------------------------------------------ */
/* Rasterisation: depth prepass / G-buffer / sun shadow                           */
/* Restates the fixed-function raster the reference pipelines configure (depth_prepass.inl:36-46,    */
/* g_buffer_generation.inl:50-60, sun_shadow_draw.inl:37-51) under the Vulkan rules: pixel-centre     */
/* sampling, top-left fill rule, depth clipping to [0, 1], LESS_OR_EQUAL in draw order, culling by    */
/* the sign of the framebuffer area (counter-clockwise front faces), depth bias m*slope + r*constant. */
/* Geometry at w <= 1e-6 is dropped (no near-plane clipping). Serial in draw order within each 32x32  */
/* tile (tiles are independent), so the result is the serial one.                                     */
/* ------------------------------------------------------------------------------------------------ */
typedef struct { float x, y, z, w; } rs_vtx;   /* homogeneous screen vertex: X, Y (pixels * w), z_c, w_c */
typedef struct {
    v3 r0, r1, r2;   /* sign-normalised edge functions E_i(p) = r_i . (px, py, 1) */
    float z0, z1, z2, w0, w1, w2, bias;
    int px0, px1, py0, py1, live;
} rs_tri;

static inline v4 mat_vec4(const float* m, float x, float y, float z, float w) {
    return V4(m[0] * x + m[4] * y + m[8] * z + m[12] * w, m[1] * x + m[5] * y + m[9] * z + m[13] * w,
              m[2] * x + m[6] * y + m[10] * z + m[14] * w, m[3] * x + m[7] * y + m[11] * z + m[15] * w);
}

/* 2DH rasterisation (Olano & Greer): no division per vertex, so geometry behind the eye needs no
   clipping; depth clipping per fragment (z_ndc in [0, 1]). X = (x_c/2 + w_c/2) W, Y likewise. */
static rs_vtx rs_clip_vertex(const float* pos, uint32_t v, const float* model, const float* vp, int W, int H) {
    v4 wp = mat_vec4(model, pos[3 * v], pos[3 * v + 1], pos[3 * v + 2], 1.0f);
    v4 c = mat_vec4(vp, wp.x, wp.y, wp.z, wp.w);
    rs_vtx o;
    o.x = (c.x * 0.5f + c.w * 0.5f) * (float)W;
    o.y = (c.y * 0.5f + c.w * 0.5f) * (float)H;
    o.z = c.z;
    o.w = c.w;
    return o;
}

static inline v3 rs_cross(v3 a, v3 b) { return V3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }

/* adjugate rows r_i of [v0 v1 v2], det = v0 . r0; facing = sign(det) (= the framebuffer area's sign when
   every w > 0; Vulkan a = -area/2 < 0 is clockwise = front, see soc_rt.h) */
static void rs_edges(rs_vtx A, rs_vtx B, rs_vtx C, v3* r0, v3* r1, v3* r2, float* det) {
    const v3 v0 = V3(A.x, A.y, A.w), v1 = V3(B.x, B.y, B.w), v2 = V3(C.x, C.y, C.w);
    *r0 = rs_cross(v1, v2);
    *r1 = rs_cross(v2, v0);
    *r2 = rs_cross(v0, v1);
    *det = v0.x * r0->x + v0.y * r0->y + v0.z * r0->z;
}

static rs_tri rs_setup(rs_vtx A, rs_vtx B, rs_vtx C, int cull, int W, int H, int depth_only, float bc, float bs) {
    rs_tri t;
    memset(&t, 0, sizeof t);
    v3 r0, r1, r2;
    float det;
    rs_edges(A, B, C, &r0, &r1, &r2, &det);
    if (!(det != 0.0f) || det != det) return t;
    if (cull == SOC_CULL_FRONT && det > 0.0f) return t;
    if (cull == SOC_CULL_BACK && det < 0.0f) return t;
    if (det < 0.0f) { r0 = neg3(r0); r1 = neg3(r1); r2 = neg3(r2); }
    t.r0 = r0; t.r1 = r1; t.r2 = r2;
    t.z0 = A.z; t.z1 = B.z; t.z2 = C.z;
    t.w0 = A.w; t.w1 = B.w; t.w2 = C.w;
    if (A.w > 1e-6f && B.w > 1e-6f && C.w > 1e-6f) {   /* bounding box of the projected vertices */
        float ax = A.x / A.w, ay = A.y / A.w, bx = B.x / B.w, by = B.y / B.w, cx = C.x / C.w, cy = C.y / C.w;
        float minx = fminf(ax, fminf(bx, cx)), maxx = fmaxf(ax, fmaxf(bx, cx));
        float miny = fminf(ay, fminf(by, cy)), maxy = fmaxf(ay, fmaxf(by, cy));
        /* one pixel of margin: the projected vertices are rounded, and coverage is decided by the edge
           functions alone (a centre on an edge may lie a rounding error outside the rounded box) */
        t.px0 = (int)floorf(fminf(fmaxf(minx - 1.5f, -1.0f), (float)W)); if (t.px0 < 0) t.px0 = 0;
        t.px1 = (int)ceilf(fminf(fmaxf(maxx + 0.5f, -1.0f), (float)W)); if (t.px1 > W - 1) t.px1 = W - 1;
        t.py0 = (int)floorf(fminf(fmaxf(miny - 1.5f, -1.0f), (float)H)); if (t.py0 < 0) t.py0 = 0;
        t.py1 = (int)ceilf(fminf(fmaxf(maxy + 0.5f, -1.0f), (float)H)); if (t.py1 > H - 1) t.py1 = H - 1;
    } else {                                           /* a vertex at or behind the eye: whole image */
        t.px0 = 0; t.px1 = W - 1; t.py0 = 0; t.py1 = H - 1;
    }
    if (t.px0 > t.px1 || t.py0 > t.py1) return t;
    if (depth_only) {   /* z_ndc = (sum z_i r_i) . p / |det| is affine in the pixel position */
        float adet = fabsf(det);
        float nx = A.z * r0.x + B.z * r1.x + C.z * r2.x, ny = A.z * r0.y + B.z * r1.y + C.z * r2.y;
        float m = fmaxf(fabsf(nx / adet), fabsf(ny / adet));
        float zmax = 0.0f;
        if (A.w > 0.0f) zmax = fmaxf(zmax, fabsf(A.z / A.w));
        if (B.w > 0.0f) zmax = fmaxf(zmax, fabsf(B.z / B.w));
        if (C.w > 0.0f) zmax = fmaxf(zmax, fabsf(C.z / C.w));
        uint32_t zb;
        memcpy(&zb, &zmax, 4);
        uint32_t e = (zb >> 23) & 255u;   /* r = 2^(E - 23), the D32F minimum resolvable difference */
        float r = (e == 0u || e == 255u) ? 0.0f : ldexpf(1.0f, (int)e - 127 - 23);
        t.bias = m * bs + r * bc;
    }
    t.live = 1;
    return t;
}

/* tie rule: an edge owns the centres exactly on it iff its normal points to +x (or +y when vertical);
   shared edges have exactly negated coefficients, so such a centre is covered once */
static inline int rs_owns(v3 r) { return r.x > 0.0f || (r.x == 0.0f && r.y > 0.0f); }
static inline float rs_edge(v3 r, float px, float py) { return r.x * px + r.y * py + r.z; }

static int rs_cover(const rs_tri* t, int x, int y, float* e0, float* e1, float* e2, float* z) {
    float fx = (float)x + 0.5f, fy = (float)y + 0.5f;
    *e0 = rs_edge(t->r0, fx, fy);
    *e1 = rs_edge(t->r1, fx, fy);
    *e2 = rs_edge(t->r2, fx, fy);
    if (*e0 < 0.0f || *e1 < 0.0f || *e2 < 0.0f) return 0;
    if (*e0 == 0.0f && !rs_owns(t->r0)) return 0;
    if (*e1 == 0.0f && !rs_owns(t->r1)) return 0;
    if (*e2 == 0.0f && !rs_owns(t->r2)) return 0;
    float num = *e0 * t->z0 + *e1 * t->z1 + *e2 * t->z2, den = *e0 * t->w0 + *e1 * t->w1 + *e2 * t->w2;
    if (!(den > 0.0f)) return 0;
    float zz = num / den;
    if (zz < 0.0f || zz > 1.0f) return 0;   /* depth clipping */
    *z = zz + 0.0f;
    return 1;
}

static int rs_check_mesh(const soc_mesh* m) {
    return m && m->positions && m->indices && m->vertex_count >= 0 && m->triangle_count >= 0;
}

/* Serial raster of the mesh in draw order, 32x32 tiles in parallel. depth_only: D32 target with bias;
   else: u64 visibility keys (depth bits << 32 | 0xFFFFFFFE - triangle, empty = 1.0 | 0xFFFFFFFF). */
static void rs_raster(const soc_mesh* mesh, const float* vp, int cull, int W, int H, int depth_only, float bc,
                      float bs, void* target, size_t pitch) {
    rs_vtx* sv = (rs_vtx*)malloc(sizeof(rs_vtx) * (size_t)(mesh->vertex_count > 0 ? mesh->vertex_count : 1));
#pragma omp parallel for
    for (int v = 0; v < mesh->vertex_count; ++v)
        sv[v] = rs_clip_vertex(mesh->positions, (uint32_t)v, mesh->model_matrix, vp, W, H);
    rs_tri* tris = (rs_tri*)malloc(sizeof(rs_tri) * (size_t)(mesh->triangle_count > 0 ? mesh->triangle_count : 1));
#pragma omp parallel for
    for (int i = 0; i < mesh->triangle_count; ++i) {
        const uint32_t* ix = mesh->indices + 3 * (size_t)i;
        tris[i] = rs_setup(sv[ix[0]], sv[ix[1]], sv[ix[2]], cull, W, H, depth_only, bc, bs);
    }
    const int TS = 32, tx_n = (W + TS - 1) / TS, ty_n = (H + TS - 1) / TS;
#pragma omp parallel for schedule(dynamic, 1)
    for (int tile = 0; tile < tx_n * ty_n; ++tile) {
        const int x0 = (tile % tx_n) * TS, y0 = (tile / tx_n) * TS;
        const int x1 = x0 + TS < W ? x0 + TS : W, y1 = y0 + TS < H ? y0 + TS : H;
        for (int y = y0; y < y1; ++y)
            for (int x = x0; x < x1; ++x) {
                if (depth_only) ((float*)((char*)target + (size_t)y * pitch))[x] = 1.0f;
                else ((uint64_t*)((char*)target + (size_t)y * pitch))[x] = ((uint64_t)0x3f800000u << 32) | 0xFFFFFFFFu;
            }
        for (int id = 0; id < mesh->triangle_count; ++id) {
            const rs_tri* t = &tris[id];
            if (!t->live || t->px1 < x0 || t->px0 >= x1 || t->py1 < y0 || t->py0 >= y1) continue;
            const int ya = t->py0 > y0 ? t->py0 : y0, yb = t->py1 < y1 - 1 ? t->py1 : y1 - 1;
            const int xa = t->px0 > x0 ? t->px0 : x0, xb = t->px1 < x1 - 1 ? t->px1 : x1 - 1;
            for (int y = ya; y <= yb; ++y)
                for (int x = xa; x <= xb; ++x) {
                    float e0, e1, e2, z;
                    if (!rs_cover(t, x, y, &e0, &e1, &e2, &z)) continue;
                    if (depth_only) {
                        float* d = (float*)((char*)target + (size_t)y * pitch) + x;
                        float zb = fminf(fmaxf(z + t->bias, 0.0f), 1.0f);
                        if (zb <= *d) *d = zb;                       /* LESS_OR_EQUAL */
                    } else {
                        uint64_t* d = (uint64_t*)((char*)target + (size_t)y * pitch) + x;
                        float cur = u2f((uint32_t)(*d >> 32));
                        if (z <= cur) {                              /* LESS_OR_EQUAL: later wins ties */
                            uint32_t zbits;
                            memcpy(&zbits, &z, 4);
                            *d = ((uint64_t)zbits << 32) | (uint64_t)(0xFFFFFFFEu - (uint32_t)id);
                        }
                    }
                }
        }
    }
    free(tris);
    free(sv);
}

int soc_oracle_raster_visibility(const soc_mesh* mesh, const float view_projection[16], int32_t cull,
                                 uint64_t* visibility, int32_t width, int32_t height) {
    if (!rs_check_mesh(mesh) || !view_projection || !visibility || width <= 0 || height <= 0) return SOC_E_INVALID_ARG;
    rs_raster(mesh, view_projection, cull, width, height, 0, 0.0f, 0.0f, visibility, (size_t)width * 8);
    return SOC_OK;
}

int soc_oracle_raster_depth(const soc_mesh* mesh, const float view_projection[16], int32_t cull, float bias_constant,
                            float bias_slope, soc_img depth) {
    if (!rs_check_mesh(mesh) || !view_projection || !valid(&depth) || depth.format != SOC_FMT_D32F) return SOC_E_INVALID_ARG;
    rs_raster(mesh, view_projection, cull, depth.width, depth.height, 1, bias_constant, bias_slope, depth.data,
              (size_t)depth.pitch_bytes);
    return SOC_OK;
}

/* REPEAT bilinear RGBA8 texture at level 0 (SRGB decoded per texel); no image samples white
   (the null texture, model.cpp:188). */
static v4 rs_sample_texture(const soc_img* tex, float u, float v) {
    if (!tex->data) return V4(1.0f, 1.0f, 1.0f, 1.0f);
    return sample_repeat(tex, u, v);
}

/* DrawTerrain patch tessellation (renderer.cpp:194-220, draw_terrain.inl:138-191; soc_rt.h
   soc_terrain_tessellate): the TES's uv bilinear in its operation order, the heightmap's .r bilinear clamp,
   the world point of the displaced vertex; shared vertices evaluated by the lowest patch holding them. */
int soc_oracle_terrain_tessellate(const soc_globals* g, soc_img heightmap, int32_t grid_size, int32_t tess_level,
                                  float* positions, float* normals, float* uvs, uint32_t* indices) {
    if (!g || !valid(&heightmap) || heightmap.format != SOC_FMT_RGBA8_UNORM || grid_size < 2 || tess_level < 1 ||
        !(tess_level & 1) || !positions || !normals || !uvs || !indices)
        return SOC_E_INVALID_ARG;
    const int n = tess_level, nv = (grid_size - 1) * n + 1;
    const float fn = (float)n, side = (float)(grid_size - 1);
    for (int gz = 0; gz < nv; ++gz)
        for (int gx = 0; gx < nv; ++gx) {
            const int k = gz * nv + gx;
            int pi = gx / n, pj = gz / n;
            if (pi > grid_size - 2) pi = grid_size - 2;
            if (pj > grid_size - 2) pj = grid_size - 2;
            const float tu = (float)(gz - pj * n) / fn, tv = (float)(gx - pi * n) / fn;
            const float i0 = (float)pi / side, i1 = (float)(pi + 1) / side, j0 = (float)pj / side, j1 = (float)(pj + 1) / side;
            const float u0x = (i0 - i0) * tu + i0, u0y = (j1 - j0) * tu + j0;
            const float u1x = (i1 - i1) * tu + i1, u1y = (j1 - j0) * tu + j0;
            const float ux = (u1x - u0x) * tv + u0x, uy = (u1y - u0y) * tv + u0y;
            const float h = sample_clamp(&heightmap, ux, uy).x;
            const float adj = (h - g->terrain_midpoint) * g->terrain_height_scale;
            positions[3 * k] = ux * g->terrain_scale[0] - g->terrain_offset[0];
            positions[3 * k + 1] = g->terrain_offset[1] + adj;
            positions[3 * k + 2] = uy * g->terrain_scale[1] - g->terrain_offset[2];
            normals[3 * k] = 0.0f; normals[3 * k + 1] = 1.0f; normals[3 * k + 2] = 0.0f;
            uvs[2 * k] = ux;
            uvs[2 * k + 1] = uy;
        }
    const int segs = nv - 1;
    for (int id = 0; id < 2 * segs * segs; ++id) {
        const int q = id >> 1, qi = q % segs, qj = q / segs;
        const uint32_t v00 = (uint32_t)(qj * nv + qi), v10 = v00 + 1, v01 = v00 + (uint32_t)nv, v11 = v01 + 1;
        indices[3 * id] = v00;
        indices[3 * id + 1] = (id & 1) ? v01 : v11;
        indices[3 * id + 2] = (id & 1) ? v11 : v10;
    }
    return SOC_OK;
}

/* ---- texture mip chains (texture.cpp:108, 184-246; soc_rt.h soc_generate_mips) ---- */
static int mip_levels(int w, int h) {
    int m = w > h ? w : h, n = 0;
    while (m > 0) { ++n; m >>= 1; }
    return n;
}
/* packed layout: level 0 = the image (any pitch), level k >= 1 tight, after the previous level */
static size_t mip_offset(int w, int h, int pitch, int k, int* wk, int* hk) {
    size_t off = 0;
    *wk = w;
    *hk = h;
    for (int j = 1; j <= k; ++j) {
        off += j == 1 ? (size_t)pitch * h : (size_t)4 * *wk * *hk;
        *wk = *wk > 1 ? *wk >> 1 : 1;
        *hk = *hk > 1 ? *hk >> 1 : 1;
    }
    return off;
}
static soc_img mip_level(const soc_img* tex, int k) {
    int wk, hk;
    size_t off = mip_offset(tex->width, tex->height, tex->pitch_bytes, k, &wk, &hk);
    soc_img im = {(char*)tex->data + off, wk, hk, k ? 4 * wk : tex->pitch_bytes, tex->format};
    return im;
}

/* vkCmdBlitImage LINEAR sample axis: destination texel x -> source coordinate (x + 0.5) n_src / n_dst, clamp to
   edge, the sampling contract's 8-bit weights */
static void blit_axis(int x, int n_src, int n_dst, int* i0, int* i1, float* w) {
    const float t = ((float)(2 * x + 1) * (float)n_src) / (float)(2 * n_dst) - 0.5f;
    const int fx = (int)floorf(t * 256.0f + 0.5f);
    int i = fx >> 8;
    float ww = (float)(fx & 255) * (1.0f / 256.0f);
    if (i < 0) { i = 0; ww = 0.0f; }
    else if (i >= n_src - 1) { i = n_src - 2; ww = 1.0f; }
    if (n_src == 1) { i = 0; ww = 0.0f; }
    *i0 = i;
    *i1 = i + 1 < n_src - 1 ? i + 1 : n_src - 1;
    *w = ww;
}

int soc_oracle_generate_mips(soc_img tex) {
    if (!tex.data || tex.width <= 0 || tex.height <= 0 || tex.pitch_bytes < tex.width * 4 ||
        (tex.format != SOC_FMT_RGBA8_UNORM && tex.format != SOC_FMT_RGBA8_SRGB))
        return SOC_E_INVALID_ARG;
    /* sRGB tables in double precision: decode per code; re-encode as a LINEAR blit does, encode then round: code k
     * from the boundary decode((k - 0.5) / 255) up (the decoded codes' midpoints biased near a boundary) */
    float dec[256], mid[256];
    for (int k = 0; k < 256; ++k) {
        const double c = k / 255.0, b = (k - 0.5) / 255.0;
        dec[k] = (float)(c <= 0.04045 ? c / 12.92 : pow((c + 0.055) / 1.055, 2.4));
        mid[k] = k ? (float)(b <= 0.04045 ? b / 12.92 : pow((b + 0.055) / 1.055, 2.4)) : 0.0f;
    }
    const int srgb = tex.format == SOC_FMT_RGBA8_SRGB, L = mip_levels(tex.width, tex.height);
    for (int k = 1; k < L; ++k) {
        const soc_img src = mip_level(&tex, k - 1), dst = mip_level(&tex, k);
        for (int y = 0; y < dst.height; ++y)
            for (int x = 0; x < dst.width; ++x) {
                int x0, x1, y0, y1;
                float wx, wy;
                blit_axis(x, src.width, dst.width, &x0, &x1, &wx);
                blit_axis(y, src.height, dst.height, &y0, &y1, &wy);
                const uint8_t* r0 = (const uint8_t*)src.data + (size_t)y0 * src.pitch_bytes;
                const uint8_t* r1 = (const uint8_t*)src.data + (size_t)y1 * src.pitch_bytes;
                uint8_t* o = (uint8_t*)dst.data + (size_t)y * dst.pitch_bytes + 4 * (size_t)x;
                for (int c = 0; c < 4; ++c) {
                    const uint8_t b[4] = {r0[4 * x0 + c], r0[4 * x1 + c], r1[4 * x0 + c], r1[4 * x1 + c]};
                    float v[4];
                    for (int q = 0; q < 4; ++q) v[q] = (srgb && c < 3) ? dec[b[q]] : unorm8(b[q]);
                    const float f = lerp_w(lerp_w(v[0], v[1], wx), lerp_w(v[2], v[3], wx), wy);
                    if (srgb && c < 3) {
                        int code = 0;
                        while (code < 255 && f >= mid[code + 1]) ++code;
                        o[c] = (uint8_t)code;
                    } else {
                        o[c] = to_unorm8(f);
                    }
                }
            }
    }
    return SOC_OK;
}

/* bilinear REPEAT sample of one chain level */
static v4 rs_sample_level(const soc_img* tex, int k, float u, float v) {
    const soc_img im = mip_level(tex, k);
    return sample_repeat(&im, u, v);
}

/* SOC_MATERIAL_MIPMAPPED sampling (soc_rt.h): trilinear + EXT_texture_filter_anisotropic's reference filter
   over the fine uv derivatives (texture.cpp:121-136: LINEAR/LINEAR/LINEAR, REPEAT, anisotropy 16) */
static v4 rs_sample_texture_mip(const soc_img* tex, float u, float v, float dudx, float dvdx, float dudy, float dvdy,
                                float max_aniso) {
    if (!tex->data) return V4(1.0f, 1.0f, 1.0f, 1.0f);
    const int L = mip_levels(tex->width, tex->height);
    const float W = (float)tex->width, H = (float)tex->height;
    const float ax = dudx * W, ay = dvdx * H, bx = dudy * W, by = dvdy * H;
    const float px = sqrtf(ax * ax + ay * ay), py = sqrtf(bx * bx + by * by);
    const float pmax = fmaxf(px, py), pmin = fminf(px, py);
    int n = 1;
    if (max_aniso > 1.0f && pmax > 0.0f && pmax <= 3.4e38f) {
        const float cap = floorf(max_aniso);
        n = (int)(pmin > 0.0f ? fminf(ceilf(pmax / pmin), cap) : cap);
    }
    int lq = 0;
    const float rho = pmax / (float)n;
    if (rho > 0.0f && rho <= 3.4e38f) {
        const float lam = fminf(fmaxf(soc_oracle_log2(rho), -64.0f), 64.0f);
        lq = (int)floorf(lam * 256.0f + 0.5f);
        if (lq < 0) lq = 0;
        if (lq > (L - 1) * 256) lq = (L - 1) * 256;
    }
    const int l0 = lq >> 8;
    const float f = (float)(lq & 255) * (1.0f / 256.0f);
    const int xmajor = px >= py;
    const float du = xmajor ? dudx : dudy, dv = xmajor ? dvdx : dvdy;
    v4 acc = V4(0.0f, 0.0f, 0.0f, 0.0f);
    for (int i = 1; i <= n; ++i) {
        float su = u, sv = v;
        if (n > 1) {
            const float t = (float)i / (float)(n + 1) - 0.5f;
            su = u + t * du;
            sv = v + t * dv;
        }
        v4 s0 = rs_sample_level(tex, l0, su, sv);
        if (lq & 255) {
            const v4 s1 = rs_sample_level(tex, l0 + 1, su, sv);
            s0 = V4(lerp_w(s0.x, s1.x, f), lerp_w(s0.y, s1.y, f), lerp_w(s0.z, s1.z, f), lerp_w(s0.w, s1.w, f));
        }
        acc = V4(acc.x + s0.x, acc.y + s0.y, acc.z + s0.z, acc.w + s0.w);
    }
    if (n == 1) return acc;
    const float fn = (float)n;
    return V4(acc.x / fn, acc.y / fn, acc.z / fn, acc.w / fn);
}

static v3 rs_normalize(v3 a) {
    float l = sqrtf(a.x * a.x + a.y * a.y + a.z * a.z);
    return V3(a.x / l, a.y / l, a.z / l);
}

/* GBufferGeneration from the visibility buffer: vertex stage g_buffer_generation.inl:169-178, fragment
   stage :189-225 incl. the normal-image TBN of :197-211 (metallic/roughness not modelled: composition does
   not read it). */
int soc_oracle_gbuffer_resolve(const soc_globals* g, const soc_mesh* mesh, const soc_material* materials,
                               int32_t material_count, const uint64_t* visibility, soc_img depth, soc_img albedo,
                               soc_img emissive, soc_img normal, soc_img velocity) {
    if (!g || !rs_check_mesh(mesh) || !mesh->normals || !mesh->uvs || !materials || material_count <= 0 || !visibility ||
        !valid(&depth) || !valid(&albedo) || !valid(&emissive) || !valid(&normal) || !valid(&velocity))
        return SOC_E_INVALID_ARG;
    const int W = depth.width, H = depth.height;
    const float* M = mesh->model_matrix;
    const float* vp = g->camera_projection_view_matrix;
    const float* pvp = g->camera_previous_projection_view_matrix;
    const float* nm = mesh->normal_matrix;
    const float n3[9] = {nm[0], nm[1], nm[2], nm[4], nm[5], nm[6], nm[8], nm[9], nm[10]};
#pragma omp parallel for schedule(static)
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            const uint64_t key = visibility[(size_t)y * W + x];
            const uint32_t low = (uint32_t)key;
            if (low == 0xFFFFFFFFu) {   /* clear values, g_buffer_generation.inl:78-100 */
                store(&depth, x, y, V4(1.0f, 0, 0, 0));
                store(&albedo, x, y, V4(0.2f, 0.4f, 1.0f, 1.0f));
                store(&emissive, x, y, V4(0, 0, 0, 1));
                store(&normal, x, y, V4(0, 0, 0, 1));
                store(&velocity, x, y, V4(0, 0, 0, 1));
                continue;
            }
            const uint32_t id = 0xFFFFFFFEu - low;
            const uint32_t ia = mesh->indices[3 * (size_t)id], ib = mesh->indices[3 * (size_t)id + 1],
                           ic = mesh->indices[3 * (size_t)id + 2];
            const rs_vtx A = rs_clip_vertex(mesh->positions, ia, M, vp, W, H);
            const rs_vtx B = rs_clip_vertex(mesh->positions, ib, M, vp, W, H);
            const rs_vtx C = rs_clip_vertex(mesh->positions, ic, M, vp, W, H);
            v3 r0, r1, r2;
            float det;
            rs_edges(A, B, C, &r0, &r1, &r2, &det);
            if (det < 0.0f) { r0 = neg3(r0); r1 = neg3(r1); r2 = neg3(r2); }
            const float fx = (float)x + 0.5f, fy = (float)y + 0.5f;
            const float e0 = rs_edge(r0, fx, fy), e1 = rs_edge(r1, fx, fy), e2 = rs_edge(r2, fx, fy);
            const float es = e0 + e1 + e2;
            const float b1 = e1 / es, b2 = e2 / es, b0 = 1.0f - b1 - b2;
            const float* uv = mesh->uvs;
            const float u = b0 * uv[2 * ia] + b1 * uv[2 * ib] + b2 * uv[2 * ic];
            const float v = b0 * uv[2 * ia + 1] + b1 * uv[2 * ib + 1] + b2 * uv[2 * ic + 1];
            const float* nr = mesh->normals;
            const v3 na = rs_normalize(mat3_mul_v3(n3, V3(nr[3 * ia], nr[3 * ia + 1], nr[3 * ia + 2])));
            const v3 nb = rs_normalize(mat3_mul_v3(n3, V3(nr[3 * ib], nr[3 * ib + 1], nr[3 * ib + 2])));
            const v3 nc = rs_normalize(mat3_mul_v3(n3, V3(nr[3 * ic], nr[3 * ic + 1], nr[3 * ic + 2])));
            uint32_t mi = mesh->materials ? mesh->materials[id] : 0u;
            if (mi > (uint32_t)(material_count - 1)) mi = (uint32_t)(material_count - 1);
            const soc_material* m = &materials[mi];
            v3 n;
            if ((m->flags & SOC_MATERIAL_NORMAL_MAP) && m->normal_map.data) {   /* draw_terrain.inl:206-219 */
                v4 t = sample_clamp(&m->normal_map, u, v);
                n = rs_normalize(V3(t.x, t.y, t.z));
            } else {
                n = rs_normalize(V3(b0 * na.x + b1 * nb.x + b2 * nc.x, b0 * na.y + b1 * nb.y + b2 * nc.y,
                                    b0 * na.z + b1 * nb.z + b2 * nc.z));
            }
            const int tbn = (m->flags & SOC_MATERIAL_NORMAL_TEXTURE) && m->normal_image.data;
            const int mipped = (m->flags & SOC_MATERIAL_MIPMAPPED) != 0;
            /* fine dFdx / dFdy: the same triangle's attributes at the two centres of the 2x2 quad per direction */
            v3 Q1 = V3(0, 0, 0), Q2 = V3(0, 0, 0);
            float gd[4] = {0.0f, 0.0f, 0.0f, 0.0f};   /* du/dx, dv/dx, du/dy, dv/dy */
            if (tbn || mipped) {
                v4 wp[3] = {V4(0, 0, 0, 0), V4(0, 0, 0, 0), V4(0, 0, 0, 0)};
                const uint32_t vi[3] = {ia, ib, ic};
                if (tbn)
                    for (int k = 0; k < 3; ++k) {
                        const float* p = mesh->positions + 3 * (size_t)vi[k];
                        wp[k] = mat_vec4(M, p[0], p[1], p[2], 1.0f);
                    }
                const float qx = (float)(x & ~1) + 0.5f, qy = (float)(y & ~1) + 0.5f;
                const float sxs[4] = {qx, qx + 1.0f, fx, fx}, sys[4] = {fy, fy, qy, qy + 1.0f};
                v3 P[4];
                float tu[4], tv[4];
                for (int k = 0; k < 4; ++k) {
                    const float a0 = rs_edge(r0, sxs[k], sys[k]), a1 = rs_edge(r1, sxs[k], sys[k]), a2 = rs_edge(r2, sxs[k], sys[k]);
                    const float as = a0 + a1 + a2;
                    const float c1 = a1 / as, c2 = a2 / as, c0 = 1.0f - c1 - c2;
                    P[k] = V3(c0 * wp[0].x + c1 * wp[1].x + c2 * wp[2].x, c0 * wp[0].y + c1 * wp[1].y + c2 * wp[2].y,
                              c0 * wp[0].z + c1 * wp[1].z + c2 * wp[2].z);
                    tu[k] = c0 * uv[2 * ia] + c1 * uv[2 * ib] + c2 * uv[2 * ic];
                    tv[k] = c0 * uv[2 * ia + 1] + c1 * uv[2 * ib + 1] + c2 * uv[2 * ic + 1];
                }
                Q1 = V3(P[1].x - P[0].x, P[1].y - P[0].y, P[1].z - P[0].z);
                Q2 = V3(P[3].x - P[2].x, P[3].y - P[2].y, P[3].z - P[2].z);
                gd[0] = tu[1] - tu[0]; gd[1] = tv[1] - tv[0]; gd[2] = tu[3] - tu[2]; gd[3] = tv[3] - tv[2];
            }
#define RS_TEX(img) (mipped ? rs_sample_texture_mip(&(img), u, v, gd[0], gd[1], gd[2], gd[3], m->max_anisotropy) \
                            : rs_sample_texture(&(img), u, v))
            if (tbn) {   /* g_buffer_generation.inl:197-211 */
                const v4 t = RS_TEX(m->normal_image);
                const v3 tn = V3(t.x * 2.0f - 1.0f, t.y * 2.0f - 1.0f, t.z * 2.0f - 1.0f);
                const float st1t = gd[1], st2t = gd[3];
                const v3 N = rs_normalize(n);
                const v3 T = rs_normalize(V3(Q1.x * st2t - Q2.x * st1t, Q1.y * st2t - Q2.y * st1t, Q1.z * st2t - Q2.z * st1t));
                const v3 B = rs_normalize(cross3(N, T));
                n = rs_normalize(V3(T.x * tn.x + B.x * tn.y + N.x * tn.z, T.y * tn.x + B.y * tn.y + N.y * tn.z,
                                    T.z * tn.x + B.z * tn.y + N.z * tn.z));
            }
            v3 em = V3(0, 0, 0);
            if (m->has_emissive) {
                v4 e = RS_TEX(m->emissive);
                em = V3(e.x * m->emissive_factor[0], e.y * m->emissive_factor[1], e.z * m->emissive_factor[2]);
            }
            const v4 al = RS_TEX(m->albedo);
#undef RS_TEX
            v4 vel = V4(0, 0, 0, 0);
            if (!(m->flags & SOC_MATERIAL_ZERO_VELOCITY)) {
                v4 cc[3], pc[3];
                const uint32_t vi[3] = {ia, ib, ic};
                for (int k = 0; k < 3; ++k) {
                    const float* p = mesh->positions + 3 * (size_t)vi[k];
                    v4 wp = mat_vec4(M, p[0], p[1], p[2], 1.0f);
                    cc[k] = mat_vec4(vp, wp.x, wp.y, wp.z, wp.w);
                    pc[k] = mat_vec4(pvp, wp.x, wp.y, wp.z, wp.w);
                }
                const float cx = b0 * cc[0].x + b1 * cc[1].x + b2 * cc[2].x, cy = b0 * cc[0].y + b1 * cc[1].y + b2 * cc[2].y;
                const float cw = b0 * cc[0].w + b1 * cc[1].w + b2 * cc[2].w;
                const float px = b0 * pc[0].x + b1 * pc[1].x + b2 * pc[2].x, py = b0 * pc[0].y + b1 * pc[1].y + b2 * pc[2].y;
                const float pw = b0 * pc[0].w + b1 * pc[1].w + b2 * pc[2].w;
                vel = V4(((cx / cw) * 0.5f + 0.5f) - ((px / pw) * 0.5f + 0.5f),
                         ((cy / cw) * 0.5f + 0.5f) - ((py / pw) * 0.5f + 0.5f), 0.0f, 1.0f);
            }
            store(&depth, x, y, V4(u2f((uint32_t)(key >> 32)), 0, 0, 0));
            store(&albedo, x, y, V4(al.x * m->albedo_factor[0] + em.x, al.y * m->albedo_factor[1] + em.y,
                                    al.z * m->albedo_factor[2] + em.z, 1.0f));
            store(&emissive, x, y, V4(em.x, em.y, em.z, 1.0f));
            store(&normal, x, y, V4(n.x, n.y, n.z, 1.0f));
            store(&velocity, x, y, vel);
        }
    return SOC_OK;
}

/* ------------------------------------------------------------------------------------------------ */
/* HeightToNormalTask, height_to_normal.inl:52-83                                                     */
/* ------------------------------------------------------------------------------------------------ */
int soc_oracle_height_to_normal(soc_img heightmap, soc_img target) {
    if (!valid(&heightmap) || !valid(&target) || heightmap.width != target.width || heightmap.height != target.height)
        return SOC_E_INVALID_ARG;
    const int W = heightmap.width, H = heightmap.height;
#pragma omp parallel for schedule(static)
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            /* clamp(pos + offset, 0, size - 1), :57-60 */
            int yu = y + 1 < H - 1 ? y + 1 : H - 1, yd = y - 1 > 0 ? y - 1 : 0;
            int xr = x + 1 < W - 1 ? x + 1 : W - 1, xl = x - 1 > 0 ? x - 1 : 0;
            float su = fetch(&heightmap, x, yu).x, sd = fetch(&heightmap, x, yd).x;
            float sr = fetch(&heightmap, xr, y).x, sl = fetch(&heightmap, xl, y).x;
            float fw = (float)W, fh = (float)H;
            v3 pu = V3((float)x / fw, su, (float)yu / fh), pd = V3((float)x / fw, sd, (float)yd / fh);
            v3 pr = V3((float)xr / fw, sr, (float)y / fh), pl = V3((float)xl / fw, sl, (float)y / fh);
            v3 vd = rs_normalize(sub3(pu, pd)), hd = rs_normalize(sub3(pr, pl));
            v3 n = rs_normalize(cross3(vd, hd));
            store(&target, x, y, V4(n.x, n.y, n.z, 1.0f));
        }
    return SOC_OK;
}

/* ------------------------------------------------------------------------------------------------ */
/* GenerateMin/MaxHIZTask, generate_hiz.glsl:17-98: the same 64x64-window reduction, serially. Every   */
/* window value is an exact min / max, so a per-window restatement over "virtual" mips (texels beyond  */
/* a mip's extent included, as the shader's LDS keeps them) gives the shader's results.               */
/* ------------------------------------------------------------------------------------------------ */
static inline float hz_op(int mx, float a, float b) { return mx ? fmaxf(a, b) : fminf(a, b); }

static void hz_store(const soc_img* mips, int count, int level, int x, int y, float v) {
    if (level >= count) return;
    const soc_img* d = &mips[level];
    if (x < d->width && y < d->height) ((float*)((char*)d->data + (size_t)y * d->pitch_bytes))[x] = v;
}

static float hz_load(const soc_img* im, int x, int y, int w, int h) {
    x = x < w - 1 ? x : w - 1;
    y = y < h - 1 ? y : h - 1;
    return ((const float*)((const char*)im->data + (size_t)y * im->pitch_bytes))[x];
}

/* one workgroup: window (gx, gy) of `src` (clamped to w x h) -> levels src_level+1 .. src_level+levels */
static void hz_window(const soc_img* src, int w, int h, int gx, int gy, int src_level, int levels, const soc_img* mips,
                      int count, int mx) {
    float a[32][32], b[32][32];   /* virtual level src_level+1 (32x32) and the following ones */
    for (int y = 0; y < 32; ++y)
        for (int x = 0; x < 32; ++x) {
            int ix = (gx * 32 + x) * 2, iy = (gy * 32 + y) * 2;
            float m = hz_op(mx, hz_op(mx, hz_load(src, ix, iy, w, h), hz_load(src, ix, iy + 1, w, h)),
                            hz_op(mx, hz_load(src, ix + 1, iy, w, h), hz_load(src, ix + 1, iy + 1, w, h)));
            a[y][x] = m;
            hz_store(mips, count, src_level + 1, gx * 32 + x, gy * 32 + y, m);
        }
    int n = 32;
    for (int i = 1; i < (levels > 2 ? levels : 2); ++i) {   /* the shader always writes the second level */
        n /= 2;
        for (int y = 0; y < n; ++y)
            for (int x = 0; x < n; ++x) {
                float m = hz_op(mx, hz_op(mx, a[2 * y][2 * x], a[2 * y][2 * x + 1]), hz_op(mx, a[2 * y + 1][2 * x], a[2 * y + 1][2 * x + 1]));
                b[y][x] = m;
                hz_store(mips, count, src_level + 1 + i, (gx * 32 >> i) + x, (gy * 32 >> i) + y, m);
            }
        memcpy(a, b, sizeof a);
        if (n == 1) break;
    }
}

int soc_oracle_generate_hiz(const soc_globals* g, soc_img depth, const soc_img* mips, int32_t mip_count, int32_t op_max) {
    if (!g || !mips || mip_count <= 0 || mip_count > 12 || !valid(&depth)) return SOC_E_INVALID_ARG;
    const int W = g->resolution[0], H = g->resolution[1];
    const int dx = (W + 63) / 64, dy = (H + 63) / 64;
    for (int gy = 0; gy < dy; ++gy)
        for (int gx = 0; gx < dx; ++gx) hz_window(&depth, depth.width, depth.height, gx, gy, -1, 6, mips, mip_count, op_max);
    /* the tail reads mip 5 at min(index, extent - 1) (:29-32): an extent of 0 (a frame under 64 texels across) reads
     * outside the image, undefined in the reference; the tail levels are then not written (hiz.hip does the same) */
    if (mip_count > 5 && (W >> 6) > 0 && (H >> 6) > 0)
        hz_window(&mips[5], W >> 6, H >> 6, 0, 0, 5, mip_count - 6, mips, mip_count, op_max);
    return SOC_OK;
}
