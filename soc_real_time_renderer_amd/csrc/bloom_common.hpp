// bloom_common.hpp — tap arithmetic of the bit-exact per-pass bloom kernels (bloom.hip). Every helper reproduces the
// oracle's rounding exactly.
#pragma once

#include "soc_internal.hpp"

namespace soc {
namespace {

constexpr int BX = 64, BY = 4;

// Clamp rule of the sampling contract applied to an 8-bit fixed-point texel coordinate.
__device__ __forceinline__ Axis axis_from_fixed(int fx, int n) {
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

// Float-uv -> fixed coordinate, identical arithmetic to axis_clamp / the oracle.
__device__ __forceinline__ int fixed_from_uv(float u, int n) {
#pragma clang fp contract(off)
    float t = u * (float)n;
    t = t - 0.5f;
    t = fminf(fmaxf(t, -2.0f), (float)n + 1.0f);
    return (int)floorf(t * 256.0f + 0.5f);
}

__device__ __forceinline__ f3 tap(const DImg& im, const Axis& ax, const Axis& ay) {
    const uint2* r0 = row_ptr<uint2>(im, ay.i0);
    const uint2* r1 = row_ptr<uint2>(im, ay.i1);
    f4 a = unpack_h4(r0[ax.i0]), b = unpack_h4(r0[ax.i1]), c = unpack_h4(r1[ax.i0]), d = unpack_h4(r1[ax.i1]);
    return f3{bilerp1(a.x, b.x, c.x, d.x, ax.w, ay.w), bilerp1(a.y, b.y, c.y, d.y, ax.w, ay.w),
              bilerp1(a.z, b.z, c.z, d.z, ax.w, ay.w)};
}

// Exact texel at clamped integer coordinates (a tap whose weights are 0/1).
__device__ __forceinline__ f3 point(const DImg& im, int x, int y) {
    x = min(max(x, 0), im.w - 1);
    y = min(max(y, 0), im.h - 1);
    f4 v = fetch_h4(im, x, y);
    return f3{v.x, v.y, v.z};
}

__device__ __forceinline__ void store_rgb1(const DImg& im, int x, int y, f3 c) {
    row_ptr_w<uint2>(im, y)[x] = pack_h4(f4{c.x, c.y, c.z, 1.0f});
}

// out = e*0.125 + (a+c+g+i)*0.03125 + (b+d+f+h)*0.0625 + (j+k+l+m)*0.125   (:137-140)
__device__ __forceinline__ float down13(float a, float b, float c, float d, float e, float f, float g, float h, float i,
                                        float j, float k, float l, float m) {
    // no contraction: the last add fused into the f16 store would become v_fma_mixlo_f16, a single
    // rounding to f16 where the oracle rounds to f32 first (1-ulp differences, double rounding)
#pragma clang fp contract(off)
    float r = e * 0.125f;
    r += (a + c + g + i) * 0.03125f;
    r += (b + d + f + h) * 0.0625f;
    r += (j + k + l + m) * 0.125f;
    return r;
}

// out = (e*4 + (b+d+f+h)*2 + (a+c+g+i)) / 16   (bloom_upsample.inl:122-125)
__device__ __forceinline__ float up9(float a, float b, float c, float d, float e, float f, float g, float h, float i) {
#pragma clang fp contract(off)
    float r = e * 4.0f;
    r += (b + d + f + h) * 2.0f;
    r += (a + c + g + i);
    r *= 1.0f / 16.0f;
    return r;
}

#define SOC_DOWN13(A, B, C, D, E, F, G, H, I, J, K, L, M)                                                   \
    f3{down13(A.x, B.x, C.x, D.x, E.x, F.x, G.x, H.x, I.x, J.x, K.x, L.x, M.x),                           \
       down13(A.y, B.y, C.y, D.y, E.y, F.y, G.y, H.y, I.y, J.y, K.y, L.y, M.y),                           \
       down13(A.z, B.z, C.z, D.z, E.z, F.z, G.z, H.z, I.z, J.z, K.z, L.z, M.z)}
#define SOC_UP9(A, B, C, D, E, F, G, H, I)                                                                  \
    f3{up9(A.x, B.x, C.x, D.x, E.x, F.x, G.x, H.x, I.x), up9(A.y, B.y, C.y, D.y, E.y, F.y, G.y, H.y, I.y), \
       up9(A.z, B.z, C.z, D.z, E.z, F.z, G.z, H.z, I.z)}

template <int C>
__device__ __forceinline__ float chan(uint2 v) {
    return C == 0 ? h2f((uint16_t)(v.x & 0xffffu)) : C == 1 ? h2f((uint16_t)(v.x >> 16)) : h2f((uint16_t)(v.y & 0xffffu));
}

__device__ __forceinline__ uint2 texel_clamped(const DImg& im, int x, int y) {
    x = min(max(x, 0), im.w - 1);
    y = min(max(y, 0), im.h - 1);
    return row_ptr<uint2>(im, y)[x];
}

__device__ __forceinline__ float lerp_c(float a, float b, float w) {
#pragma clang fp contract(off)
    return a * (1.0f - w) + b * w;
}

__device__ __forceinline__ void store_rgb1_c(const DImg& im, int x, int y, float r, float g, float b) {
    row_ptr_w<uint2>(im, y)[x] = pack_h4(f4{r, g, b, 1.0f});
}

// The two pixels (X0, y), (X0 + 1, y) of a quad row: one 16-B store when the row is 16-B aligned
// (X0 is even), so a wave writes 1 KiB contiguous per instruction.
__device__ __forceinline__ void store_quad_row(const DImg& im, int X0, int y, const float (&o)[2][3], bool vec) {
    if (y >= im.h) return;
    if (vec && X0 + 1 < im.w) {
        const uint2 a = pack_h4(f4{o[0][0], o[0][1], o[0][2], 1.0f}), b = pack_h4(f4{o[1][0], o[1][1], o[1][2], 1.0f});
        *reinterpret_cast<uint4*>(row_ptr_w<uint2>(im, y) + X0) = uint4{a.x, a.y, b.x, b.y};
        return;
    }
    if (X0 < im.w) store_rgb1_c(im, X0, y, o[0][0], o[0][1], o[0][2]);
    if (X0 + 1 < im.w) store_rgb1_c(im, X0 + 1, y, o[1][0], o[1][1], o[1][2]);
}

// Exact re-associations of lerp_c for the fixed weights of the register-window and fused kernels (no overflow or
// denormals occur for RGBA16F-origin data):
//  * w = 1/2: a*0.5 + b*0.5 == (a + b) * 0.5, both products being exact.
//  * w = 3/4 (1/4) on RGBA16F texels: a*0.25 + b*0.75 == (a + 3b) * 0.25, since 3b is exact for an
//    11-bit significand; half4_* return the unscaled a + 3b ("t", four times the lerp).
//  * vertical w = 3/4 (1/4) on two such t: h0*0.25 + round(h1*0.75) with h = t/4, i.e.
//    fma(t0, 1/16, round(t1 * 3/16)): the same two roundings as lerp_c.
__device__ __forceinline__ float mid(float a, float b) {
#pragma clang fp contract(off)
    return (a + b) * 0.5f;
}
__device__ __forceinline__ float t_w34(float a, float b) { return __builtin_fmaf(b, 3.0f, a); }   // 4*lerp(a,b,3/4)
__device__ __forceinline__ float t_w14(float a, float b) { return __builtin_fmaf(a, 3.0f, b); }   // 4*lerp(a,b,1/4)
__device__ __forceinline__ float v_w34(float t0, float t1) {
#pragma clang fp contract(off)
    const float p = t1 * 0.1875f;
    return __builtin_fmaf(t0, 0.0625f, p);
}
// The rounded product t * 3/16 shared by v_w34 (as t1) and v_w14 (as t0).
__device__ __forceinline__ float v_prod(float t) {
#pragma clang fp contract(off)
    return t * 0.1875f;
}
__device__ __forceinline__ float v_w14(float t0, float t1) {
#pragma clang fp contract(off)
    const float p = t0 * 0.1875f;
    return __builtin_fmaf(t1, 0.0625f, p);
}

}  // namespace
}  // namespace soc
