// soc_device.hpp — device-side helpers shared by the gfx950 pass kernels.
//
// Implements the SAMPLING CONTRACT of DESIGN.md §3 (the restatement of the reference's Vulkan
// linear_sampler / REPEAT sampler and image formats; gfx950 has no texture units, so filtering is
// VALU work here). Helpers that must be bit-identical to the oracle's arithmetic disable FMA
// contraction locally (`#pragma clang fp contract(off)`).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace soc {

// Flat work-group bound of the 256-lane kernels: their __launch_bounds__ and the bound their launchers check
// (soc_internal.hpp launch()).
constexpr int kWorkgroup = 256;

struct DImg {          // device view of a soc_img
    char* data;
    int w, h, pitch;
};

struct f4 { float x, y, z, w; };
struct f3 { float x, y, z; };

__device__ __forceinline__ f3 mk3(float x, float y, float z) { return f3{x, y, z}; }
__device__ __forceinline__ f3 operator+(f3 a, f3 b) { return f3{a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ f3 operator-(f3 a, f3 b) { return f3{a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ f3 operator*(f3 a, f3 b) { return f3{a.x * b.x, a.y * b.y, a.z * b.z}; }
__device__ __forceinline__ f3 operator*(f3 a, float s) { return f3{a.x * s, a.y * s, a.z * s}; }
__device__ __forceinline__ f3 operator-(f3 a) { return f3{-a.x, -a.y, -a.z}; }
__device__ __forceinline__ float dot3(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ float length3(f3 a) { return sqrtf(dot3(a, a)); }
__device__ __forceinline__ f3 normalize3(f3 a) { float l = length3(a); return f3{a.x / l, a.y / l, a.z / l}; }
__device__ __forceinline__ f3 cross3(f3 a, f3 b) {
    return f3{a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y};
}
__device__ __forceinline__ float clampf(float x, float lo, float hi) { return fminf(fmaxf(x, lo), hi); }
__device__ __forceinline__ float mixf(float a, float b, float t) { return a * (1.0f - t) + b * t; }
__device__ __forceinline__ float fractf(float x) { return x - floorf(x); }

// ---------------------------------------------------------------------------------------------
// formats
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ float h2f(uint16_t h) { return (float)__builtin_bit_cast(_Float16, h); }
__device__ __forceinline__ uint16_t f2h(float f) { return __builtin_bit_cast(uint16_t, (_Float16)f); }

__device__ __forceinline__ f4 unpack_h4(uint2 v) {
    return f4{h2f((uint16_t)(v.x & 0xffffu)), h2f((uint16_t)(v.x >> 16)), h2f((uint16_t)(v.y & 0xffffu)),
              h2f((uint16_t)(v.y >> 16))};
}
__device__ __forceinline__ uint2 pack_h4(f4 c) {
    return uint2{(uint32_t)f2h(c.x) | ((uint32_t)f2h(c.y) << 16), (uint32_t)f2h(c.z) | ((uint32_t)f2h(c.w) << 16)};
}

__device__ __forceinline__ float unorm8(uint32_t u) { return (float)u * (1.0f / 255.0f); }
__device__ __forceinline__ uint32_t to_unorm8(float x) { return (uint32_t)rintf(clampf(x, 0.0f, 1.0f) * 255.0f); }
__device__ __forceinline__ uint32_t pack_unorm8x4(f4 c) {
    return to_unorm8(c.x) | (to_unorm8(c.y) << 8) | (to_unorm8(c.z) << 16) | (to_unorm8(c.w) << 24);
}

template <typename T>
__device__ __forceinline__ const T* row_ptr(const DImg& im, int y) {
    return reinterpret_cast<const T*>(im.data + (size_t)y * (size_t)im.pitch);
}
template <typename T>
__device__ __forceinline__ T* row_ptr_w(const DImg& im, int y) {
    return reinterpret_cast<T*>(im.data + (size_t)y * (size_t)im.pitch);
}

__device__ __forceinline__ f4 fetch_h4(const DImg& im, int x, int y) { return unpack_h4(row_ptr<uint2>(im, y)[x]); }
__device__ __forceinline__ float fetch_f32(const DImg& im, int x, int y) { return row_ptr<float>(im, y)[x]; }
__device__ __forceinline__ float fetch_r8(const DImg& im, int x, int y) { return unorm8(row_ptr<uint8_t>(im, y)[x]); }
__device__ __forceinline__ f4 unpack_rgba8(uint32_t v) {
    return f4{unorm8(v & 0xffu), unorm8((v >> 8) & 0xffu), unorm8((v >> 16) & 0xffu), unorm8(v >> 24)};
}
__device__ __forceinline__ f4 fetch_rgba8(const DImg& im, int x, int y) { return unpack_rgba8(row_ptr<uint32_t>(im, y)[x]); }

// ---------------------------------------------------------------------------------------------
// sampling contract (clamp-to-edge, 8-bit sub-texel precision)
// ---------------------------------------------------------------------------------------------
// Returns the left tap i0 in [0, n-2] (0 when n == 1) and the weight of tap i0+1 (clamped to n-1).
// i < 0 maps to (0, w=0) and i >= n-1 to (n-2, w=1): both give the edge texel exactly, as the
// oracle's "coinciding taps" rule does.
struct Axis { int i0; int i1; float w; };

__device__ __forceinline__ Axis axis_clamp(float u, int n) {
#pragma clang fp contract(off)
    float t = u * (float)n;
    t = t - 0.5f;
    t = fminf(fmaxf(t, -2.0f), (float)n + 1.0f);
    int fx = (int)floorf(t * 256.0f + 0.5f);
    int i = fx >> 8;
    float w = (float)(fx & 255) * (1.0f / 256.0f);
    if (i < 0) { i = 0; w = 0.0f; }
    else if (i >= n - 1) { i = n - 2; w = 1.0f; }
    if (n == 1) { i = 0; w = 0.0f; }
    Axis a;
    a.i0 = i;
    a.i1 = min(i + 1, n - 1);
    a.w = w;
    return a;
}

// REPEAT addressing for a power-of-two extent n (mask = n-1).
__device__ __forceinline__ Axis axis_repeat_pow2(float u, int n, int mask) {
#pragma clang fp contract(off)
    float t = u * (float)n;
    t = t - 0.5f;
    t = fminf(fmaxf(t, -4194304.0f), 4194304.0f);
    int fx = (int)floorf(t * 256.0f + 0.5f);
    int i = fx >> 8;
    Axis a;
    a.w = (float)(fx & 255) * (1.0f / 256.0f);
    a.i0 = i & mask;
    a.i1 = (i + 1) & mask;
    return a;
}

__device__ __forceinline__ float lerp_w(float a, float b, float w) {
#pragma clang fp contract(off)
    return a * (1.0f - w) + b * w;
}
__device__ __forceinline__ float bilerp1(float a, float b, float c, float d, float wx, float wy) {
    return lerp_w(lerp_w(a, b, wx), lerp_w(c, d, wx), wy);
}
__device__ __forceinline__ f4 bilerp4(f4 a, f4 b, f4 c, f4 d, float wx, float wy) {
    return f4{bilerp1(a.x, b.x, c.x, d.x, wx, wy), bilerp1(a.y, b.y, c.y, d.y, wx, wy),
              bilerp1(a.z, b.z, c.z, d.z, wx, wy), bilerp1(a.w, b.w, c.w, d.w, wx, wy)};
}

// With n >= 2 texels across, axis_clamp's taps are i0 and i0 + 1 (i0 <= n - 2): each row's texel pair is one
// load of twice the texel size (4-byte aligned: the hardware's dword alignment), the same texels.
typedef uint32_t soc_u4a4 __attribute__((ext_vector_type(4))) __attribute__((aligned(4)));
typedef float soc_f2a4 __attribute__((ext_vector_type(2))) __attribute__((aligned(4)));
__device__ __forceinline__ f4 sample_h4(const DImg& im, float u, float v) {
    Axis ax = axis_clamp(u, im.w), ay = axis_clamp(v, im.h);
    const uint2* r0 = row_ptr<uint2>(im, ay.i0);
    const uint2* r1 = row_ptr<uint2>(im, ay.i1);
    if (im.w >= 2) {
        const soc_u4a4 p0 = *reinterpret_cast<const soc_u4a4*>(r0 + ax.i0);
        const soc_u4a4 p1 = *reinterpret_cast<const soc_u4a4*>(r1 + ax.i0);
        return bilerp4(unpack_h4(uint2{p0.x, p0.y}), unpack_h4(uint2{p0.z, p0.w}), unpack_h4(uint2{p1.x, p1.y}),
                       unpack_h4(uint2{p1.z, p1.w}), ax.w, ay.w);
    }
    return bilerp4(unpack_h4(r0[ax.i0]), unpack_h4(r0[ax.i1]), unpack_h4(r1[ax.i0]), unpack_h4(r1[ax.i1]), ax.w, ay.w);
}
__device__ __forceinline__ float sample_f32(const DImg& im, float u, float v) {
    Axis ax = axis_clamp(u, im.w), ay = axis_clamp(v, im.h);
    const float* r0 = row_ptr<float>(im, ay.i0);
    const float* r1 = row_ptr<float>(im, ay.i1);
    if (im.w >= 2) {
        const soc_f2a4 p0 = *reinterpret_cast<const soc_f2a4*>(r0 + ax.i0);
        const soc_f2a4 p1 = *reinterpret_cast<const soc_f2a4*>(r1 + ax.i0);
        return bilerp1(p0.x, p0.y, p1.x, p1.y, ax.w, ay.w);
    }
    return bilerp1(r0[ax.i0], r0[ax.i1], r1[ax.i0], r1[ax.i1], ax.w, ay.w);
}
__device__ __forceinline__ float sample_r8(const DImg& im, float u, float v) {
    Axis ax = axis_clamp(u, im.w), ay = axis_clamp(v, im.h);
    const uint8_t* r0 = row_ptr<uint8_t>(im, ay.i0);
    const uint8_t* r1 = row_ptr<uint8_t>(im, ay.i1);
    return bilerp1(unorm8(r0[ax.i0]), unorm8(r0[ax.i1]), unorm8(r1[ax.i0]), unorm8(r1[ax.i1]), ax.w, ay.w);
}
__device__ __forceinline__ f4 sample_rgba8(const DImg& im, float u, float v) {
    Axis ax = axis_clamp(u, im.w), ay = axis_clamp(v, im.h);
    return bilerp4(fetch_rgba8(im, ax.i0, ay.i0), fetch_rgba8(im, ax.i1, ay.i0), fetch_rgba8(im, ax.i0, ay.i1),
                   fetch_rgba8(im, ax.i1, ay.i1), ax.w, ay.w);
}

// An image as a buffer resource (wave-uniform descriptor) addressed with 32-bit byte offsets: one VALU
// multiply-add per address instead of the 64-bit pointer arithmetic of row_ptr. Images below 2 GiB
// (the C ABI checks the extents it launches with).
struct BufImg {
    __amdgpu_buffer_rsrc_t r;
    int pitch, w, h;
};
__device__ __forceinline__ BufImg buf_img(const DImg& im) {
    return BufImg{__builtin_amdgcn_make_buffer_rsrc(im.data, 0, im.pitch * im.h, 0x00020000), im.pitch, im.w, im.h};
}
__device__ __forceinline__ int buf_row(const BufImg& b, int y) { return __mul24(y, b.pitch); }

// sample_f32 / sample_r8 on a BufImg: the same taps, weights and arithmetic (same bits).
__device__ __forceinline__ float sample_f32(const BufImg& b, float u, float v) {
    typedef float f2u4 __attribute__((ext_vector_type(2))) __attribute__((aligned(4)));
    const Axis ax = axis_clamp(u, b.w), ay = axis_clamp(v, b.h);
    if (b.w < 2) {   // i1 == i0: the generic two-load form
        const float t0 = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(b.r, buf_row(b, ay.i0), 0, 0));
        const float t1 = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(b.r, buf_row(b, ay.i1), 0, 0));
        return bilerp1(t0, t0, t1, t1, ax.w, ay.w);
    }
    const int o = ax.i0 * 4;   // i1 == i0 + 1: one 8-B load per row
    const f2u4 r0 = __builtin_bit_cast(f2u4, __builtin_amdgcn_raw_buffer_load_b64(b.r, buf_row(b, ay.i0) + o, 0, 0));
    const f2u4 r1 = __builtin_bit_cast(f2u4, __builtin_amdgcn_raw_buffer_load_b64(b.r, buf_row(b, ay.i1) + o, 0, 0));
    return bilerp1(r0.x, r0.y, r1.x, r1.y, ax.w, ay.w);
}
__device__ __forceinline__ float sample_r8(const BufImg& b, float u, float v) {
    const Axis ax = axis_clamp(u, b.w), ay = axis_clamp(v, b.h);
    const int o0 = buf_row(b, ay.i0), o1 = buf_row(b, ay.i1);
    const uint32_t a = __builtin_amdgcn_raw_buffer_load_b8(b.r, o0 + ax.i0, 0, 0);
    const uint32_t c = __builtin_amdgcn_raw_buffer_load_b8(b.r, o0 + ax.i1, 0, 0);
    const uint32_t d = __builtin_amdgcn_raw_buffer_load_b8(b.r, o1 + ax.i0, 0, 0);
    const uint32_t e = __builtin_amdgcn_raw_buffer_load_b8(b.r, o1 + ax.i1, 0, 0);
    return bilerp1(unorm8(a), unorm8(c), unorm8(d), unorm8(e), ax.w, ay.w);
}

// sample_r8 at two coordinates of one row v whose taps span at most 8 bytes from the first tap's dword (a pixel pair
// reading a half-resolution image: 3 texels per row): one 8-B load per row for both samples instead of 8 byte loads,
// the same texels, weights and arithmetic (same bits); other spans, and a load that would pass the row's pitch, take
// the per-byte form.
__device__ __forceinline__ void sample_r8_pair(const BufImg& b, float u0, float u1, float v, float& s0, float& s1) {
    const Axis a0 = axis_clamp(u0, b.w), a1 = axis_clamp(u1, b.w), ay = axis_clamp(v, b.h);
    const int base = a0.i0 & ~3;
    if (a1.i0 >= a0.i0 && a1.i1 - base <= 7 && base + 8 <= b.pitch) {
        const uint64_t r0 = __builtin_bit_cast(uint64_t, __builtin_amdgcn_raw_buffer_load_b64(b.r, buf_row(b, ay.i0) + base, 0, 0));
        const uint64_t r1 = __builtin_bit_cast(uint64_t, __builtin_amdgcn_raw_buffer_load_b64(b.r, buf_row(b, ay.i1) + base, 0, 0));
        auto t = [&](uint64_t r, int i) { return unorm8((uint32_t)(r >> (8 * (i - base))) & 255u); };
        s0 = bilerp1(t(r0, a0.i0), t(r0, a0.i1), t(r1, a0.i0), t(r1, a0.i1), a0.w, ay.w);
        s1 = bilerp1(t(r0, a1.i0), t(r0, a1.i1), t(r1, a1.i0), t(r1, a1.i1), a1.w, ay.w);
        return;
    }
    s0 = sample_r8(b, u0, v);
    s1 = sample_r8(b, u1, v);
}

// Packed mip chain (soc_rt.h soc_generate_mips): level count and the byte offset / extent of level k.
__host__ __device__ __forceinline__ int mip_levels(int w, int h) {
    int m = w > h ? w : h, n = 0;
    while (m > 0) { ++n; m >>= 1; }
    return n;
}
__host__ __device__ __forceinline__ size_t mip_offset(int w, int h, int pitch, int k, int& wk, int& hk, int bpp = 4) {
    size_t off = 0;
    wk = w;
    hk = h;
    for (int j = 1; j <= k; ++j) {
        off += j == 1 ? (size_t)pitch * h : (size_t)bpp * wk * hk;
        wk = wk > 1 ? wk >> 1 : 1;
        hk = hk > 1 ? hk >> 1 : 1;
    }
    return off;
}

// GLSL mat4 * vec4 on a column-major float[16] (kernel-argument copy).
struct Mat4 { float m[16]; };
struct Mat3 { float m[9]; };

__device__ __forceinline__ f4 mul(const Mat4& M, f4 v) {
    const float* m = M.m;
    return f4{m[0] * v.x + m[4] * v.y + m[8] * v.z + m[12] * v.w, m[1] * v.x + m[5] * v.y + m[9] * v.z + m[13] * v.w,
              m[2] * v.x + m[6] * v.y + m[10] * v.z + m[14] * v.w, m[3] * v.x + m[7] * v.y + m[11] * v.z + m[15] * v.w};
}
__device__ __forceinline__ f3 mul3of4(const Mat4& M, f3 v) {
    const float* m = M.m;
    return f3{m[0] * v.x + m[4] * v.y + m[8] * v.z, m[1] * v.x + m[5] * v.y + m[9] * v.z, m[2] * v.x + m[6] * v.y + m[10] * v.z};
}
__device__ __forceinline__ f3 mul(const Mat3& M, f3 v) {
    const float* m = M.m;
    return f3{m[0] * v.x + m[3] * v.y + m[6] * v.z, m[1] * v.x + m[4] * v.y + m[7] * v.z, m[2] * v.x + m[5] * v.y + m[8] * v.z};
}

// XCD-aware tile order for a 2D grid. Workgroups are dispatched round-robin over the 8 XCDs by linear
// block id (id % 8); with swz != 0, XCD k's blocks take the contiguous row-major tile range
// [k n/8, (k+1) n/8), so neighbouring tiles whose halos / gather footprints overlap share one XCD's
// 4 MiB L2 instead of being spread over all eight. Placement only: every tile is still visited once.
__device__ __forceinline__ void xcd_tile(int swz, int& tx, int& ty) {
    const int gx = (int)gridDim.x, n = (int)(gridDim.x * gridDim.y);
    int id = (int)(blockIdx.y * gridDim.x + blockIdx.x);
    if (swz) {
        const int q = n >> 3, r = n & 7, k = id & 7;
        id = k * q + min(k, r) + (id >> 3);
    }
    ty = id / gx;
    tx = id - ty * gx;
}

// XCD-aware order with a compact footprint. The tiles are enumerated band by band (8 horizontal bands
// of ceil(gy / 8) tile rows), each band in column strips of `strip` tiles, each strip row by row; XCD k
// (workgroup id mod 8) takes the k-th contiguous eighth of that sequence. The workgroups in flight on
// one XCD then cover a near-square region, so its L2 holds their gather footprint. A bijection.
__device__ __forceinline__ void xcd_tile_strips(int strip, int& tx, int& ty) {
    const int gx = (int)gridDim.x, gy = (int)gridDim.y, n = gx * gy;
    const int id = (int)(blockIdx.y * gridDim.x + blockIdx.x);
    const int q = n >> 3, r = n & 7, k = id & 7;
    const int i = k * q + min(k, r) + (id >> 3);   // position in the band/strip sequence
    const int B = (gy + 7) >> 3;
    const int band = i / (B * gx), off = i - band * B * gx;
    const int rows = min(B, gy - band * B);
    const int s = off / (strip * rows), in = off - s * strip * rows;
    const int w = min(strip, gx - s * strip);
    const int ly = in / w;
    tx = s * strip + (in - ly * w);
    ty = band * B + ly;
}

// XCD-aware order in vertical bands: the tiles are enumerated in column strips of `strip` tiles over the
// full image height (left to right, each strip row by row); XCD k takes the k-th contiguous eighth, i.e. a
// vertical band of about gx / 8 tile columns. Every XCD then sees the same mix of rows (a sky band at the
// top of the frame no longer idles whole XCDs, as the horizontal bands of xcd_tile_strips do), and its
// workgroups in flight still cover a compact strip. A bijection.
__device__ __forceinline__ void xcd_tile_vbands(int strip, int& tx, int& ty) {
    const int gx = (int)gridDim.x, gy = (int)gridDim.y, n = gx * gy;
    const int id = (int)(blockIdx.y * gridDim.x + blockIdx.x);
    const int q = n >> 3, r = n & 7, k = id & 7;
    const int i = k * q + min(k, r) + (id >> 3);   // position in the strip sequence
    const int s = i / (strip * gy), in = i - s * strip * gy;
    const int w = min(strip, gx - s * strip);
    const int ly = in / w;
    tx = s * strip + (in - ly * w);
    ty = ly;
}
// swz: 0 row-major, 1 contiguous eighths, >= 2 horizontal bands of `swz`-tile strips, <= -2 vertical bands.
__device__ __forceinline__ void xcd_order(int swz, int& tx, int& ty) {
    if (swz >= 2) xcd_tile_strips(swz, tx, ty);
    else if (swz <= -2) xcd_tile_vbands(-swz, tx, ty);
    else xcd_tile(swz, tx, ty);
}

// Pixel-centre uv exactly as the oracle computes it: (x + 0.5) / n, correctly rounded.
__device__ __forceinline__ float centre_uv(int x, int n) { return ((float)x + 0.5f) / (float)n; }

// a / n correctly rounded without the IEEE division sequence, given rn = RN(1 / n) (host: recip_rn): one multiply and
// two fmas (Markstein's correction step). tools/check_div_rn.c verifies it exhaustively against the division for
// every a = x + 0.5 (x < n) and a = x (x <= n), n <= 16384; for larger n the host passes rn = 0 and the division runs.
__device__ __forceinline__ float div_rn(float a, float n, float rn) {
    if (rn == 0.0f) return a / n;   // wave-uniform
    const float q = a * rn;
    return __builtin_fmaf(__builtin_fmaf(-q, n, a), rn, q);
}
__device__ __forceinline__ float centre_uv_rn(int x, int n, float rn) { return div_rn((float)x + 0.5f, (float)n, rn); }

}  // namespace soc
