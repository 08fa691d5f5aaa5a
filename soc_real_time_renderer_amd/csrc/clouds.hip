// clouds.hip — CloudRenderingTask (src/graphics/tasks/cloud_rendering.inl:27-54, shader :92-481):
// Rayleigh/Mie single scattering (16 x 8 steps) + a 24-step volumetric cloud march with a 10-step
// sun-visibility march per dense step, on sky pixels only (depth == 1); other pixels get the constant
// (0.2, 0.4, 1.0). Output RGBA8_UNORM at full resolution (quirk Q6).
//
// VALU/transcendental-bound, not HBM-bound. Workgroups are 16x16 pixel tiles (4 waves of 16x4, so
// sky masks are wave-coherent); a tile with no sky pixel exits after its depth test. Tiles with sky
// stage the 64x64 noise texture into LDS as packed 2x2 quads (one ds_read_b32 returns the four texels
// of a bilinear REPEAT tap), 16 KiB per workgroup.
#include <cstdlib>
#include <type_traits>

#include "soc_internal.hpp"

// Profiling builds only (tools/kernel_variants.py): 1 = atmosphere only, 2 = cloud march only,
// 3 = cloud march without the sun-visibility march, 4 = classify only, 5 = classify only without the
// list atomic. The library is always built with 0.
// SOC_CLOUDS_EXITS (profiling only; 1 = the product): 0 evaluates every octave, 2 stops after the second (wrong results)
#ifndef SOC_CLOUDS_EXITS
#define SOC_CLOUDS_EXITS 1
#endif
#ifndef SOC_CLOUDS_PROFILE
#define SOC_CLOUDS_PROFILE 0
#endif

namespace soc {
namespace {

// The pass's transcendentals: the hardware approximations (default: v_exp_f32, v_sqrt_f32, v_log_f32, v_rcp_f32, ~1 ulp)
// or the library's accurate forms (SOC_CLOUDS_PRECISE=1: a parity-study build, tools/clouds_parity_probe.py, which
// measures what the approximations change against the oracle's libm).
#ifndef SOC_CLOUDS_PRECISE
#define SOC_CLOUDS_PRECISE 0
#endif
// SOC_CLOUDS_EXACT (default 1): the chain from the view ray to every noise tap (march geometry, step positions, altitude,
// noise coordinates, sub-texel fixed point) with the reference's operation order and roundings, so it selects the same
// texels and weights as the oracle (the file is compiled without implicit contraction; intended fmas are explicit).
// 0 = round 5's fused forms (fewer instructions, taps an ulp away). See noise3.
#ifndef SOC_CLOUDS_EXACT
#define SOC_CLOUDS_EXACT 1
#endif
__device__ __forceinline__ float cl_exp(float x) {
    if constexpr (SOC_CLOUDS_PRECISE != 0) return expf(x);
    else return __expf(x);
}
__device__ __forceinline__ float cl_exp2(float x) {
    if constexpr (SOC_CLOUDS_PRECISE != 0) return exp2f(x);
    else return __builtin_amdgcn_exp2f(x);
}
__device__ __forceinline__ float cl_sqrt(float x) {
    if constexpr (SOC_CLOUDS_PRECISE != 0) return sqrtf(x);
    else return __builtin_amdgcn_sqrtf(x);
}
__device__ __forceinline__ float cl_log2(float x) {
    if constexpr (SOC_CLOUDS_PRECISE != 0) return log2f(x);
    else return __builtin_amdgcn_logf(x);
}
__device__ __forceinline__ float cl_rcp(float x) {
    if constexpr (SOC_CLOUDS_PRECISE != 0) return 1.0f / x;
    else return __builtin_amdgcn_rcpf(x);
}

constexpr int kNoise = 64, kNoiseMask = 63;
// LDS quad table: 81 x 81 entries (64 + the 17-texel tap offset), so the second tap of get_3d_noise is
// the first tap's address plus a constant (an immediate ds_read offset) with no wrap arithmetic.
constexpr int kTap2 = 17, kTW = kNoise + kTap2, kTable = kTW * kTW;
// the quad tables padded to whole 16-B chunks (prebuilt in the workspace by clouds_od_lut, copied into LDS)
constexpr int kTableU32 = (kTable + 3) & ~3, kTableU2 = (kTable + 1) & ~1;
// the row table (RowF): one f16 pair per texel position of 82 rows (a quad's bottom row is the next row's entry)
constexpr int kRowTable = (kTW + 1) * kTW, kRowU32 = (kRowTable + 3) & ~3;
constexpr int kTableBuild = kRowU32 > kTableU32 ? kRowU32 : kTableU32;   // entries clouds_od_lut builds
constexpr float kEarthRadius = 6371000.0f, kMinH = 1600.0f, kMaxH = 500.0f + 1600.0f, kSunBrightness = 3.0f;
constexpr float kPi = 3.14159265358979f;   // acos(-1.0) in fp32
constexpr float kLn2 = 0.693147182f;       // log(2.0) in fp32

struct CloudParams {
    Mat4 inv_proj, inv_view;
    float sun[3];      // -sun_info.direction
    float cam[3];
    float res_x_m1, res_y_m1;  // resolution - 1
    float r_res_x_m1, r_res_y_m1;  // recip_rn(resolution - 1) for the ray uv x / (W - 1) (div_rn)
    float elapsed;
    float sun_factor;  // max(min(|sun.x|, |sun.z|) + sun.y, 0)
    int res_x, res_y;
};

// Q = uint32_t: LDS quads of 4 bytes (c0 c1 / c2 c3), filtered in integers (v_dot2_u32_u16); Q = uint2: the same quad
// in float form, two f16 pairs (256 c0 | (c1 - c0) << 16, 256 c2 | (c3 - c2) << 16) filtered by v_fma_mix_f32 (twice
// the LDS; every value and partial sum is an integer, or an integer / 256, below 2^24, so exact: the same bits as the
// integer form, scaled by 1 / 256, NoiseScale). On gfx950 the fp32 FMA issues at about twice the rate of the 32-bit
// integer, permute and dot-product opcodes (tools/microbench/valu_ops.hip), so the float form is the cheaper one.
template <typename Q>
struct CtxT {
    const Q* quads;   // LDS
    float cam_x, cam_z, time;
};
using Ctx = CtxT<uint32_t>;
using CtxW = CtxT<uint2>;
// noise3's value per unit of the noise (the u32 form's 65536 x 255 x bilinear; the f16 form's 256 x 255 x bilinear)
// Q = RowF: the float form with half the LDS: one f16 pair (256 c0 | (c1 - c0) << 16) per texel position of a row table,
// the quad's bottom row read from the entry kTW further (two 4-B LDS reads per tap instead of one 8-B read)
struct RowF {
    uint32_t h;
};
template <typename Q> struct NoiseScale { static constexpr float v = 1.0f; };
template <> struct NoiseScale<uint2> { static constexpr float v = 256.0f; };
template <> struct NoiseScale<RowF> { static constexpr float v = 256.0f; };

// The float-form table entry of quad texels (c0, c1, c2, c3) (bytes): 256 c0, c1 - c0, 256 c2, c3 - c2 as f16 (exact)
__device__ __forceinline__ uint2 wide_quad_entry(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3) {
    auto h = [](int v) { return (uint32_t)__builtin_bit_cast(uint16_t, (_Float16)(float)v); };
    return uint2{h(256 * (int)c0) | (h((int)c1 - (int)c0) << 16), h(256 * (int)c2) | (h((int)c3 - (int)c2) << 16)};
}
__device__ __forceinline__ uint32_t row_entry(uint32_t c0, uint32_t c1) {
    auto h = [](int v) { return (uint32_t)__builtin_bit_cast(uint16_t, (_Float16)(float)v); };
    return h(256 * (int)c0) | (h((int)c1 - (int)c0) << 16);
}
// (bilinear of the quad) / 256 from its float-form entry with wx = the x weight (0..255) and wys = the y weight / 256:
// top = 256 c0 + (c1 - c0) wx and bot are integers below 2^16, (bot - top) wy / 256 + top is the integer bilinear / 256
__device__ __forceinline__ float bilerp_wide(uint2 q, float wx, float wys) {
    const float top = __builtin_fmaf((float)__builtin_bit_cast(_Float16, (uint16_t)(q.x >> 16)), wx,
                                     (float)__builtin_bit_cast(_Float16, (uint16_t)(q.x & 0xffffu)));
    const float bot = __builtin_fmaf((float)__builtin_bit_cast(_Float16, (uint16_t)(q.y >> 16)), wx,
                                     (float)__builtin_bit_cast(_Float16, (uint16_t)(q.y & 0xffffu)));
    return __builtin_fmaf(bot - top, wys, top);
}
// the same from the row table's two entries (top row, bottom row)
__device__ __forceinline__ float bilerp_rows(RowF t, RowF b, float wx, float wys) {
    return bilerp_wide(uint2{t.h, b.h}, wx, wys);
}

__device__ __forceinline__ float bayer2(float ax, float ay) {
    ax = floorf(ax);
    ay = floorf(ay);
    return fractf(ax * 0.5f + ay * (ay * 0.75f));
}
__device__ __forceinline__ float bayer4(float x, float y) { return bayer2(0.5f * x, 0.5f * y) * 0.25f + bayer2(x, y); }
__device__ __forceinline__ float bayer8(float x, float y) { return bayer4(0.5f * x, 0.5f * y) * 0.25f + bayer2(x, y); }
__device__ __forceinline__ float bayer16(float x, float y) { return bayer8(0.5f * x, 0.5f * y) * 0.25f + bayer2(x, y); }

// The view-ray -> noise-tap chain restates the oracle's operation order without implicit contraction (SOC_CLOUDS_EXACT):
// these helpers carry `fp contract(off)` themselves (the rest of the file is compiled with contraction).
__device__ __forceinline__ float dot3_rn(f3 a, f3 b) {
#pragma clang fp contract(off)
    return a.x * b.x + a.y * b.y + a.z * b.z;
}
__device__ __forceinline__ float length3_rn(f3 a) { return sqrtf(dot3_rn(a, a)); }
__device__ __forceinline__ f3 normalize3_rn(f3 a) {
    const float l = length3_rn(a);
    return f3{a.x / l, a.y / l, a.z / l};
}
__device__ __forceinline__ f4 mul_rn(const Mat4& M, f4 v) {
#pragma clang fp contract(off)
    const float* m = M.m;
    return f4{m[0] * v.x + m[4] * v.y + m[8] * v.z + m[12] * v.w, m[1] * v.x + m[5] * v.y + m[9] * v.z + m[13] * v.w,
              m[2] * v.x + m[6] * v.y + m[10] * v.z + m[14] * v.w, m[3] * v.x + m[7] * v.y + m[11] * v.z + m[15] * v.w};
}
// sqrt(x) correctly rounded for a normal x > 0 (x = 0 gives 0): the hardware square root (within 1 ulp) and ocml's
// correction (the neighbour whose residual x - r s has the right sign), without the denormal scaling and class checks of
// sqrtf (the altitude's |p + R e_y|^2 ~ 4e13)
__device__ __forceinline__ float sqrt_rn(float x) {
    const float s = __builtin_amdgcn_sqrtf(x);
    const float dn = __uint_as_float(__float_as_uint(s) - 1u), up = __uint_as_float(__float_as_uint(s) + 1u);
    float r = __builtin_fmaf(-dn, s, x) <= 0.0f ? dn : s;
    r = __builtin_fmaf(-up, s, x) > 0.0f ? up : r;
    return r;
}

// rsi's discriminant (every caller that branches on it uses this one expression)
__device__ __forceinline__ float rsi_delta(f3 p, f3 d, float radius, float& PoD) {
#pragma clang fp contract(off)
    PoD = dot3_rn(p, d);
    const float r2 = radius * radius;
    return PoD * PoD + r2 - dot3_rn(p, p);
}
__device__ __forceinline__ float2 rsi(f3 p, f3 d, float radius) {
    float PoD;
    float delta = rsi_delta(p, d, radius, PoD);
    if (delta < 0.0f) return float2{-1.0f, -1.0f};
    delta = sqrtf(delta);
    return float2{-PoD - delta, -PoD + delta};
}

// texture(noise, uv).x under REPEAT + the sampling contract, from the LDS quad table. The two taps of
// get_3d_noise sit exactly 17 texels apart in u and v (zStretch = 17/64), so they share one axis
// computation. The bilinear blend of a tap is evaluated EXACTLY in integers on the raw bytes with the
// contract's 8-bit weights (v_dot2_u32_u16: c0 (256 - wx) + c1 wx per row, then the same across rows;
// at most 255 * 65536 < 2^24), i.e. without the fp32 rounding of the lerps; both are within the RGBA8
// tolerance of the pass.
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t udot2(uint32_t a, uint32_t b) {
    return __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, a), __builtin_bit_cast(u16x2, b), 0u, false);
}
// 65536 x bilinear of quad q (bytes c0 c1 / c2 c3) with packed weights wxp = (256 - wx) | wx << 16
__device__ __forceinline__ uint32_t quad_bilerp_u(uint32_t q, uint32_t wxp, uint32_t wyp) {
    const uint32_t top = udot2(__builtin_amdgcn_perm(q, q, 0x0c010c00u), wxp);   // c0 | c1 << 16
    const uint32_t bot = udot2(__builtin_amdgcn_perm(q, q, 0x0c030c02u), wxp);   // c2 | c3 << 16
    return udot2(top | (bot << 16), wyp);
}

__device__ __forceinline__ uint32_t quad_bilerp_u(uint2 q, uint32_t wxp, uint32_t wyp) {
    return udot2(udot2(q.x, wxp) | (udot2(q.y, wxp) << 16), wyp);
}

// (int)floorf(x) as one v_cvt_flr_i32_f32 (the compiler emits v_floor_f32 + v_cvt_i32_f32); the same value for
// every finite x in the int range, which the noise coordinates (|x| < 2^24) are.
__device__ __forceinline__ int floor_to_int(float x) {
    int r;
    asm("v_cvt_flr_i32_f32 %0, %1" : "=v"(r) : "v"(x));
    return r;
}

// Packed f32 pairs (v_pk_fma_f32 / v_pk_add_f32, tools/microbench/pk_rate.hip): element-wise the scalar operations.
typedef float f2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2v pfma(f2v a, f2v b, f2v c) { return __builtin_elementwise_fma(a, b, c); }

// One bilinear REPEAT tap of the noise .x at the fixed-point texel coordinate (fx, fy) (8 fractional bits), from the LDS
// quad table: 65536 x 255 x the bilinear (exact in integers).
template <typename Q>
__device__ __forceinline__ float noise_tap(const Q* quads, int fx, int fy) {
    const uint32_t wx = (uint32_t)fx & 255u, wy = (uint32_t)fy & 255u;
    const uint32_t ix = ((uint32_t)fx >> 8) & kNoiseMask, iy = ((uint32_t)fy >> 8) & kNoiseMask;
    if constexpr (std::is_same<Q, uint2>::value)
        return bilerp_wide(quads[iy * (uint32_t)kTW + ix], (float)wx, (float)wy * (1.0f / 256.0f));
    else if constexpr (std::is_same<Q, RowF>::value)
        return bilerp_rows(quads[iy * (uint32_t)kTW + ix], quads[(iy + 1u) * (uint32_t)kTW + ix], (float)wx,
                           (float)wy * (1.0f / 256.0f));
    else
        return (float)quad_bilerp_u(quads[iy * (uint32_t)kTW + ix], wx * 65535u + 256u, wy * 65535u + 256u);
}

// get_3d_noise, :219-233.
// SOC_CLOUDS_EXACT (default): the coordinates with the reference's (and the oracle's) roundings: coord = pos.xy / 64 +
// p 17/64 (both terms exact, so one fma is the same sum), the second tap at coord + 17/64 (rounded: near a binade edge
// it is not the first tap + 17 texels), and the sampling contract's fixed point t = RN(coord 64 - 0.5),
// fx = floor(RN(t 256 + 0.5)) (coord 64 and t 256 are exact, so each is one fma). A noise coordinate one ulp off moves a
// tap across a 1/256 sub-texel step in a few percent of the evaluations, and the smoothstep at 0.55..0.6 amplifies the
// density change: the fused form below put 6 % of C3's sky texels one RGBA8 level off the oracle's
// (tools/clouds_parity_probe.py). SOC_CLOUDS_EXACT=0 (round 5): 256 pos.x + 4352 p - 127.5 in one rounding, the
// second tap at +17 texels.
template <typename Q>
__device__ __forceinline__ float noise3(const CtxT<Q>& cx, f3 pos) {
    const float p = floorf(pos.z);
    const float f = pos.z - p;
    float a, b;
    if constexpr (SOC_CLOUDS_EXACT != 0) {
        const float pz = p * 0.265625f;   // p * zStretch: exact
        const float ux = __builtin_fmaf(pos.x, 0.015625f, pz), uy = __builtin_fmaf(pos.y, 0.015625f, pz);
        // the contract's t = RN(64 u - 0.5) is exact (|u| < 2^17) and 256 t is exact, so RN(256 t + 0.5) is the single
        // rounding RN(16384 u - 127.5): one fma
        const int fx = floor_to_int(__builtin_fmaf(ux, 16384.0f, -127.5f));
        const int fy = floor_to_int(__builtin_fmaf(uy, 16384.0f, -127.5f));
        const uint32_t ix = ((uint32_t)fx >> 8) & kNoiseMask, iy = ((uint32_t)fy >> 8) & kNoiseMask;
        const Q* t = cx.quads + (iy * (uint32_t)kTW + ix);
        // the second tap at coord + 17/64 taken as the first + 17 texels: u + 17/64 and 16384 (u + 17/64) - 127.5
        // are exact, or round as u's own terms do, except where a sum crosses into the next binade (there it may land
        // one sub-texel step away)
        if constexpr (std::is_same<Q, uint2>::value) {
            const float wx = (float)((uint32_t)fx & 255u), wys = (float)((uint32_t)fy & 255u) * (1.0f / 256.0f);
            a = bilerp_wide(t[0], wx, wys);
            b = bilerp_wide(t[kTap2 * kTW + kTap2], wx, wys);
        } else if constexpr (std::is_same<Q, RowF>::value) {
            const float wx = (float)((uint32_t)fx & 255u), wys = (float)((uint32_t)fy & 255u) * (1.0f / 256.0f);
            a = bilerp_rows(t[0], t[kTW], wx, wys);
            b = bilerp_rows(t[kTap2 * kTW + kTap2], t[(kTap2 + 1) * kTW + kTap2], wx, wys);
        } else {
            const uint32_t wxp = ((uint32_t)fx & 255u) * 65535u + 256u, wyp = ((uint32_t)fy & 255u) * 65535u + 256u;
            a = (float)quad_bilerp_u(t[0], wxp, wyp);
            b = (float)quad_bilerp_u(t[kTap2 * kTW + kTap2], wxp, wyp);
        }
        if constexpr (SOC_CLOUDS_EXACT >= 2) {
            // the second tap at RN(coord + 17/64), its own fixed point
            const int gx = floor_to_int(__builtin_fmaf(ux + 0.265625f, 16384.0f, -127.5f));
            const int gy = floor_to_int(__builtin_fmaf(uy + 0.265625f, 16384.0f, -127.5f));
            b = noise_tap(cx.quads, gx, gy);
        }
    } else {
        // fixed-point texel coordinate of the first tap: (u 64 - 0.5) 256 + 0.5 with u = pos.x / 64 + p 17/64,
        // i.e. 256 pos.x + 4352 p - 127.5 (one rounding instead of four)
        const float base = __builtin_fmaf(p, 4352.0f, -127.5f);
        const int fx = floor_to_int(__builtin_fmaf(pos.x, 256.0f, base));
        const int fy = floor_to_int(__builtin_fmaf(pos.y, 256.0f, base));
        const uint32_t wx = (uint32_t)fx & 255u, wy = (uint32_t)fy & 255u;
        const uint32_t wxp = wx * 65535u + 256u, wyp = wy * 65535u + 256u;
        const uint32_t ix = ((uint32_t)fx >> 8) & kNoiseMask, iy = ((uint32_t)fy >> 8) & kNoiseMask;
        const Q* t = cx.quads + (iy * (uint32_t)kTW + ix);
        const Q q0 = t[0], q1 = t[kTap2 * kTW + kTap2];
        if constexpr (std::is_same<Q, uint2>::value) {
            a = bilerp_wide(q0, (float)wx, (float)wy * (1.0f / 256.0f));
            b = bilerp_wide(q1, (float)wx, (float)wy * (1.0f / 256.0f));
        } else if constexpr (std::is_same<Q, RowF>::value) {
            a = bilerp_rows(q0, t[kTW], (float)wx, (float)wy * (1.0f / 256.0f));
            b = bilerp_rows(q1, t[(kTap2 + 1) * kTW + kTap2], (float)wx, (float)wy * (1.0f / 256.0f));
        } else {
            a = (float)quad_bilerp_u(q0, wxp, wyp);
            b = (float)quad_bilerp_u(q1, wxp, wyp);
        }
    }
    return __builtin_fmaf(f, b - a, a);   // x 1 / (255 65536) = the noise value (Q = uint2: x 1 / (255 256)); the caller
                                          // folds it into the octave weight
}
constexpr float kNoiseNorm = 1.0f / (255.0f * 65536.0f);

// |v| with the hardware square root (1 ulp). Every length in this pass is an Earth-scale distance
// (|v| ~ 6.4e6 m, ulp 0.5 m), far from the denormal range the full-precision sequence guards.
__device__ __forceinline__ float hw_length3(f3 v) { return cl_sqrt(dot3(v, v)); }
// The altitude's length with the correctly rounded square root under SOC_CLOUDS_EXACT: one ulp of |p + R e_y| is 0.5 m of
// altitude, which moves the y noise coordinate by ~0.13 sub-texel steps (the hardware square root's 1-ulp error flipped
// taps in ~1 of 8 evaluations)
__device__ __forceinline__ float alt_length3(f3 v) {
    if constexpr (SOC_CLOUDS_EXACT != 0) return sqrt_rn(dot3_rn(v, v));
    else return hw_length3(v);
}

// Altitude above the planet of a point given relative to the camera's ground point.
__device__ __forceinline__ float cloud_height(f3 p) { return alt_length3(f3{p.x, p.y + kEarthRadius, p.z}) - kEarthRadius; }

// get_clouds, :235-262, for a point whose altitude h is already known to lie inside the layer.
// The four octaves carry weights 1/2, 1/4, 1/8, 1/16 and each lies in [0, 1], so once the partial sum
// plus the largest possible remainder stays below the smoothstep's lower edge 0.55 the result is
// exactly 0 (smoothstep clamps to 0) and the remaining octaves are skipped. The 1e-4 margin covers the
// fp32 rounding of the remainder, so the early exits never change a result. (Round 4 measured two more exact exits
// -- after octave 1, and once the partial sum reaches the upper edge 0.6, where the smoothstep saturates -- on the C3
// and C4 frames: they fire on 0.5 % and 0-8 % of the evaluations and cost 1-2 % more time, profiles/r04_probe_clouds.txt.)
// a s + b and a s - b, each product and sum rounded (the GLSL expressions of get_clouds; no contraction)
__device__ __forceinline__ f3 madd_rn(f3 a, float s, f3 b) {
#pragma clang fp contract(off)
    return f3{a.x * s + b.x, a.y * s + b.y, a.z * s + b.z};
}
__device__ __forceinline__ f3 msub_rn(f3 a, float s, f3 b) {
#pragma clang fp contract(off)
    return f3{a.x * s - b.x, a.y * s - b.y, a.z * s - b.z};
}

template <typename C>
__device__ float clouds_at(const C& cx, f3 p, float h) {
    p = f3{p.x + cx.cam_x, h, p.z + cx.cam_z};
    const f3 mv = f3{cx.time, 0.0f, cx.time};
    const bool ex = SOC_CLOUDS_EXACT != 0;
    // mv.y == 0: the y terms' "+ 0" / "- 0" are dropped (they only map -0 to +0, and cc.y = 0.001 h > 0 for every caller,
    // which passes an h inside the layer), so cc.y and its multiples are the same bits without the three adds
    f3 cc;
    if (ex) {
        cc = madd_rn(p, 0.001f, mv);
        cc.y = p.y * 0.001f;
    } else {
        cc = p * 0.001f + mv;
    }
    // octave weight x noise normalisation as one constant per octave (powers of two apart: one fma per octave); the
    // float-form table's values are the integer form's / 256 and its constants x 256 (exact: the same products)
    using Q = typename std::remove_cv<typename std::remove_pointer<decltype(cx.quads)>::type>::type;
    constexpr float kS = NoiseScale<Q>::v;
    float n = noise3(cx, cc) * (0.5f * kNoiseNorm * kS);
    f3 c2 = cc * 2.0f + mv;   // 2 cc exact: one fma is the same sum
    if (ex) c2.y = cc.y * 2.0f;
    n = __builtin_fmaf(noise3(cx, c2), 0.25f * kNoiseNorm * kS, n);
    if (SOC_CLOUDS_EXITS == 2) return n;   // profiling only (wrong results): never the last two octaves
    if (SOC_CLOUDS_EXITS != 0 && n < 0.55f - 0.1875f - 1e-4f) return 0.0f;
    f3 c3;
    if (ex) {
        c3 = msub_rn(cc, 7.0f, mv);
        c3.y = cc.y * 7.0f;
    } else {
        c3 = cc * 7.0f - mv;
    }
    n = __builtin_fmaf(noise3(cx, c3), 0.125f * kNoiseNorm * kS, n);
    if (SOC_CLOUDS_EXITS != 0 && n < 0.55f - 0.0625f - 1e-4f) return 0.0f;
    // (cc + mv) 16 == fma(cc, 16, 16 mv) exactly: scaling by a power of two commutes with the rounding
    const f3 c4 = f3{__builtin_fmaf(cc.x, 16.0f, mv.x * 16.0f), ex ? cc.y * 16.0f : __builtin_fmaf(cc.y, 16.0f, mv.y * 16.0f),
                     __builtin_fmaf(cc.z, 16.0f, mv.z * 16.0f)};
    n = __builtin_fmaf(noise3(cx, c4), 0.0625f * kNoiseNorm * kS, n);
    const float hh = p.y - kMinH;
    const float th = (1.0f - cl_exp(-0.01f * hh)) * cl_exp(-0.004f * hh);
    const float t = clampf((n - 0.55f) * (1.0f / (0.6f - 0.55f)), 0.0f, 1.0f);
    const float clouds = t * t * (3.0f - 2.0f * t) * th;
    return clouds * 0.03f;
}

template <typename C>
__device__ __forceinline__ float get_clouds(const C& cx, f3 p) {
    const float h = cloud_height(p);
    if (h < kMinH || h > kMaxH) return 0.0f;
    return clouds_at(cx, p, h);
}

// getSunVisibility, :264-278. When the march starts out moving away from the planet centre
// ((p + R e_y) . sun > 0) the altitude grows monotonically along it (|a + t s|^2 is convex in t), so
// once a step leaves the top of the layer every later step returns 0, and stopping there leaves tr
// unchanged (tr + 0 == tr).
template <typename C>
__device__ float sun_visibility(const C& cx, f3 p, f3 sun) {
    const float rSteps = 500.0f / 10.0f;
    const f3 inc = sun * rSteps;
    f3 pos = inc * 0.5f + p;
    float tr = 0.0f;
    if (SOC_CLOUDS_PROFILE == 3) return 1.0f;
    const bool rising = dot3_rn(f3{p.x, p.y + kEarthRadius, p.z}, sun) > 0.0f;
    for (int i = 0; i < 10; i++, pos = pos + inc) {
        const float h = cloud_height(pos);
        if (h > kMaxH && rising) break;
        if (h >= kMinH && h <= kMaxH) tr += clouds_at(cx, pos, h);
    }
    return cl_exp(-tr * rSteps);
}

__device__ __forceinline__ float hg_phase(float x, float g) {
    const float g2 = g * g;
    return 0.25f * ((1.0f - g2) * powf(1.0f + g2 - 2.0f * g * x, -1.5f));
}

// calculate_atmospheric_scattering_top, :195-217
__device__ f3 scattering_top(f3 sun) {
    const f3 rayleigh = f3{0.27f * 1e-5f, 0.5f * 1e-5f, 1.0f * 1e-5f};
    const f3 mie = f3{0.5e-6f, 0.5e-6f, 0.5e-6f};
    const f3 total = rayleigh + mie;
    const float lDotU = dot3(sun, f3{0.0f, 1.0f, 0.0f});
    const float od = 100000.0f / fmaxf(1.0f * 2.0f - 0.01f, 0.01f);
    float dl = lDotU * 2.0f;
    dl = fmaxf(dl + 0.01f, 0.01f);
    dl = 1.0f / dl;
    const float odl = 100000.0f * dl;
    const f3 sv = total * od, sl = total * odl;
    const f3 av = f3{cl_exp(-total.x * od), cl_exp(-total.y * od), cl_exp(-total.z * od)};
    const f3 al = f3{cl_exp(-total.x * odl), cl_exp(-total.y * odl), cl_exp(-total.z * odl)};
    const f3 num = al - av, den = (sl - sv) * kLn2;
    const f3 absorb = f3{(fabsf(num.x) + 1e-3f) / (fabsf(den.x) + 1e-3f), (fabsf(num.y) + 1e-3f) / (fabsf(den.y) + 1e-3f),
                         (fabsf(num.z) + 1e-3f) / (fabsf(den.z) + 1e-3f)};
    const f3 ms = mie * od * 0.25f, rs = rayleigh * od * 0.375f;
    return (ms + rs) * absorb * kSunBrightness;
}

// The march of calculate_volumetric_clouds (:307-325): 24 steps between the bottom and top shells.
struct MarchGeom {
    f3 start, inc;
    float stepLength;
};
__device__ __forceinline__ MarchGeom march_geometry(f3 dir) {
    const f3 c0 = f3{0.0f, kEarthRadius, 0.0f};
    const float bottom = rsi(c0, dir, kEarthRadius + kMinH).y;
    const float top = rsi(c0, dir, kEarthRadius + kMaxH).y;
    MarchGeom g;
    g.start = dir * bottom;
    const f3 end = dir * top;
    g.inc = (end - g.start) * (1.0f / 24.0f);
    g.stepLength = length3_rn(g.inc);
    return g;
}

// Per-pixel constants of the scattering sum (:313-319).
struct MarchShade {
    float phase;
    f3 skyl;   // sky * 0.25 / pi
};
// skyl depends on the sun only: sky_light(sun) once per thread, then march_shade per pixel (same bits).
__device__ __forceinline__ f3 sky_light(f3 sun) { return scattering_top(sun) * 0.25f * (1.0f / kPi); }
__device__ __forceinline__ MarchShade march_shade(f3 dir, f3 sun, f3 skyl) {
    const float x = dot3(sun, dir);
    MarchShade m;
    m.phase = mixf(hg_phase(x, -0.5f * 0.8f), hg_phase(x, 0.8f * 0.8f), 0.5f);
    m.skyl = skyl;
    return m;
}

// Position of march step i (:321-333): cp = inc * dither + start, then cp += inc per step.
// SOC_CLOUDS_EXACT: the reference's accumulation (a pass over the steps carries cp along; a lane that needs step i alone
// repeats the i additions: a few dozen VALU against a sun march's ~1,500). 0: one fma per component,
// start + inc (i + dither) (i + dither is exact), which differs from the accumulated position by a few ulps.
// Every path (single-lane march, density, sunvis) uses these, so the pair path stays bit-identical to the single-lane march.
__device__ __forceinline__ f3 step_first_rn(const MarchGeom& mg, float dither) { return madd_rn(mg.inc, dither, mg.start); }
__device__ __forceinline__ f3 step_next(const MarchGeom& mg, float dither, int i, f3 cp) {
    if constexpr (SOC_CLOUDS_EXACT != 0) return cp + mg.inc;   // the position of step i + 1
    const float t = (float)(i + 1) + dither;
    return f3{__builtin_fmaf(mg.inc.x, t, mg.start.x), __builtin_fmaf(mg.inc.y, t, mg.start.y),
              __builtin_fmaf(mg.inc.z, t, mg.start.z)};
}
__device__ __forceinline__ f3 step_position(const MarchGeom& mg, float dither, int i) {
    if constexpr (SOC_CLOUDS_EXACT != 0) {
        f3 cp = step_first_rn(mg, dither);
        for (int k = 0; k < i; ++k) cp = cp + mg.inc;
        return cp;
    }
    const float t = (float)i + dither;
    return f3{__builtin_fmaf(mg.inc.x, t, mg.start.x), __builtin_fmaf(mg.inc.y, t, mg.start.y),
              __builtin_fmaf(mg.inc.z, t, mg.start.z)};
}

// One dense step of the scattering sum (:326-344), in the reference's order.
__device__ __forceinline__ void march_accumulate(const MarchShade& ms, f3 sun_color, float od, float vis, f3& scattering,
                                                 float& transmittance) {
    const float hPi = kPi * 0.5f, rLOG2 = 1.0f / kLn2;
    const float integral = cl_exp(-1.11f * rLOG2 * od) * (-1.0f / 1.11f) + 1.0f / 1.11f;
    const float beers = 1.0f - cl_exp(-(od * kLn2) * 2.0f);
    const f3 sunl = sun_color * vis * beers * ms.phase * hPi * kSunBrightness;
    scattering = scattering + (sunl + ms.skyl) * integral * kPi * transmittance;
    transmittance *= cl_exp(-od);
}

__device__ __forceinline__ f3 march_finish(const MarchGeom& mg, f3 color, f3 scattering, float transmittance) {
    const f3 lit = color * transmittance + scattering;
    const float m = clampf(length3(mg.start) * 0.00001f * 2.5f, 0.0f, 1.0f);
    return f3{mixf(lit.x, color.x, m), mixf(lit.y, color.y, m), mixf(lit.z, color.z, m)};
}

// calculate_volumetric_clouds, :307-347 (single-lane form: the no-workspace kernel and the overflow
// fallback of the pair path)
__device__ f3 volumetric_clouds(const Ctx& cx, f3 dir, f3 sun, f3 color, float dither, f3 sun_color) {
    if (dir.y < 0.0f) return color;
    const MarchGeom mg = march_geometry(dir);
    const MarchShade ms = march_shade(dir, sun, sky_light(sun));
    f3 scattering = f3{0.0f, 0.0f, 0.0f};
    float transmittance = 1.0f;
    f3 cp = step_position(mg, dither, 0);
    for (int i = 0; i < 24; cp = step_next(mg, dither, i, cp), i++) {
        const float od = get_clouds(cx, cp) * mg.stepLength;
        if (od <= 0.0f) continue;
        march_accumulate(ms, sun_color, od, sun_visibility(cx, cp, sun), scattering, transmittance);
    }
    return march_finish(mg, color, scattering, transmittance);
}

// atmosphere, :353-439 (primary ray starts at iTime = elapsed_time: quirk Q10)
constexpr float kRPlanet = 6371e3f, kRAtmos = 6471e3f, kShRlh = 8e3f, kShMie = 1.2e3f;
constexpr float kExpR = -1.44269504f / kShRlh, kExpM = -1.44269504f / kShMie;   // exp(-h/sh) = exp2(h * kExp)

// The secondary (sun) ray of a primary sample, :399-423: its (Rayleigh, Mie) optical depth. It depends on the sample
// only through A = |iPos|^2 and PoD = iPos.pSun (and C2 = |pSun|^2): |iPos + pSun t|^2 = A + t (B + t C2), B = 2 PoD,
// and rsi(iPos, pSun, rAtmos).y needs the same two dot products; exp(-h / sh) as exp2(|jPos| kExp - rPlanet kExp).
// Per step two fmas, a sqrt and the two exponentials.
__device__ __forceinline__ f2v secondary_od(float A, float PoD, float C2) {
    const float cR = -kRPlanet * kExpR, cM = -kRPlanet * kExpM;
    const float delta = PoD * PoD + kRAtmos * kRAtmos - A;
    const float jStep = (delta < 0.0f ? -1.0f : -PoD + cl_sqrt(delta)) / 8.0f;
    const float B = 2.0f * PoD, half = jStep * 0.5f;
    float jTime = 0.0f;
    f2v jOd = {0.0f, 0.0f};
    // two secondary steps per packed instruction (v_pk_fma_f32 / v_pk_add_f32), element-wise the same
    // operations, and the same sequential jTime and accumulation chains: the same bits
#pragma unroll 2
    for (int j = 0; j < 8; j += 2) {
        const float jT1 = jTime + jStep;
        const f2v t = f2v{jTime, jT1} + f2v{half, half};
        const f2v q = pfma(t, pfma(t, f2v{C2, C2}, f2v{B, B}), f2v{A, A});
        const f2v len = {cl_sqrt(q.x), cl_sqrt(q.y)};
        const f2v eR = pfma(len, f2v{kExpR, kExpR}, f2v{cR, cR}), eM = pfma(len, f2v{kExpM, kExpM}, f2v{cM, cM});
        jOd = pfma(f2v{cl_exp2(eR.x), cl_exp2(eM.x)}, f2v{jStep, jStep}, jOd);
        jOd = pfma(f2v{cl_exp2(eR.y), cl_exp2(eM.y)}, f2v{jStep, jStep}, jOd);
        jTime = jT1 + jStep;
    }
    return jOd;
}

// Optical-depth table of the secondary ray (round 4). By the symmetry above, secondary_od is a function of the sample's
// radius r = |iPos| and mu = PoD / r alone (for the frame's sun), the same for every sky pixel: the per-frame table holds
// (log2 odR, log2 odM) on a kOdR x kOdM grid over r in [rPlanet, rAtmos] and mu in [-1, 1], and a primary sample
// inside that shell reads
// its secondary depths by bilinear interpolation of the logs (the depths are nearly exponential in r) instead of
// marching the 8 secondary steps: 2 exponentials instead of 8 square roots and 16 exponentials. Against the march the
// secondary attenuation exp(-(kMie odM + kRlh odR)) differs by 2e-8 (median) and at most 6e-4 (grazing sun near the
// ground), 1.4e-5 for mu > 0.9 (the reference sun over the frame; tools/od_lut_check.py): within the pass's RGBA8
// tolerance (tests/test_gpu_parity.py test_clouds_od_table_against_marched_secondary_rays). Samples above the shell
// (the primary ray's 16 steps span the chord from the atmosphere's entry BEHIND the camera, so about half of an upward
// ray's samples lie above 100 km) read its top row (depth ~0: the march's own depths there are below 1e-2 m, 1e-7 of the
// exponent); samples below the ground march (see atmosphere()). Entries whose march is not
// finite (a sun ray through the planet, whose attenuation the reference takes to 0) are stored as NaN, and samples that
// read one march their secondary ray as before. SOC_CLOUDS_OD_LUT=0 marches every secondary ray (the single-lane kernel
// always does).
constexpr int kOdR = 256, kOdM = 512;
constexpr float kOdRScale = (float)(kOdR - 1) / (kRAtmos - kRPlanet), kOdMScale = (float)(kOdM - 1) * 0.5f;
struct OdLut {
    const float2* t;   // [kOdR][kOdM] (log2 odR, log2 odM); nullptr: no table
    float C2;
};

// Entry i of the quad tables stage_noise / stage_noise_wide build (the same bytes).
template <bool NOISE_R8>
__device__ __forceinline__ uint4 noise_quad_texels(const DImg& noise, int i) {
    const int ny = i / kTW, nx = (i - ny * kTW) & kNoiseMask;
    const int nyw = ny & kNoiseMask;
    const int nx1 = (nx + 1) & kNoiseMask, ny1 = (nyw + 1) & kNoiseMask;
    auto texel = [&](int tx, int ty) -> uint32_t {
        if (NOISE_R8) return row_ptr<uint8_t>(noise, ty)[tx];
        return row_ptr<uint32_t>(noise, ty)[tx] & 0xffu;
    };
    return uint4{texel(nx, nyw), texel(nx1, nyw), texel(nx, ny1), texel(nx1, ny1)};
}

// zero: the frame's 256-B counter block, cleared here (the lane's first kernel) instead of by a separate fill launch
// Blocks past the table's (lut_blocks) build the frame's noise quad tables (noise_quads: 4 bytes per entry, as
// stage_noise; noise_wide: the float-form f16 pairs, as stage_noise_wide; the padding entries zero) for the march kernels' LDS.
template <bool NOISE_R8>
__global__ __launch_bounds__(kWorkgroup) void clouds_od_lut(float2* __restrict__ lut, float C2, uint32_t* __restrict__ zero,
                                                     int lut_blocks, DImg noise, uint32_t* __restrict__ noise_quads,
                                                     uint2* __restrict__ noise_wide, uint32_t* __restrict__ noise_rows) {
    if ((int)blockIdx.x >= lut_blocks) {
        const int e = (int)(blockIdx.x - lut_blocks) * kWorkgroup + (int)threadIdx.x;
        if (e >= kTableBuild) return;
        uint4 t = uint4{0u, 0u, 0u, 0u};
        if (e < kTable) t = noise_quad_texels<NOISE_R8>(noise, e);
        if (e < kTableU32) noise_quads[e] = t.x | (t.y << 8) | (t.z << 16) | (t.w << 24);
        if (e < kTableU2) noise_wide[e] = e < kTable ? wide_quad_entry(t.x, t.y, t.z, t.w) : uint2{0u, 0u};
        if (e < kRowU32) {
            uint32_t r = 0u;
            if (e < kRowTable) {   // row e / kTW (wrapped), texels x and x + 1 (wrapped)
                const uint4 q = noise_quad_texels<NOISE_R8>(noise, e % kTW + ((e / kTW) & kNoiseMask) * kTW);
                r = row_entry(q.x, q.y);
            }
            noise_rows[e] = r;
        }
        return;
    }
    const int i = (int)(blockIdx.x * kWorkgroup + threadIdx.x);
    if (!lut) {
        if (i < 64) zero[i] = 0u;
        return;
    }
    if (i < 64) zero[i] = 0u;
    if (i >= kOdR * kOdM) return;
    const int ir = i / kOdM, im = i - ir * kOdM;
    const float r = kRPlanet + (float)ir * (1.0f / kOdRScale), mu = -1.0f + (float)im * (1.0f / kOdMScale);
    const f2v od = secondary_od(r * r, r * mu, C2);
    const float lo = 1e-30f;   // the top row (r = rAtmos: a zero-length ray)
    const bool ok = od.x < 3.0e38f && od.y < 3.0e38f && od.x >= 0.0f && od.y >= 0.0f;   // NaN / inf fail
    lut[i] = ok ? float2{cl_log2(fmaxf(od.x, lo)), cl_log2(fmaxf(od.y, lo))}
                : float2{__builtin_nanf(""), __builtin_nanf("")};
}

// The secondary depths of a sample from the table (bilinear in (r, mu), then exp2), or NaN where the table has none.
__device__ __forceinline__ f2v secondary_od_lut(const OdLut& L, float iLen, float PoD) {
    const float fr = fminf(fmaxf((iLen - kRPlanet) * kOdRScale, 0.0f), (float)(kOdR - 1));
    const float mu = PoD * cl_rcp(iLen);
    const float fm = fminf(fmaxf((mu + 1.0f) * kOdMScale, 0.0f), (float)(kOdM - 1));
    const int ir = min((int)fr, kOdR - 2), im = min((int)fm, kOdM - 2);
    const float wr = fr - (float)ir, wm = fm - (float)im;
    const float2* row = L.t + ir * kOdM + im;
    const float2 a = row[0], b = row[1], c = row[kOdM], d = row[kOdM + 1];
    const f2v top = pfma(f2v{wm, wm}, f2v{b.x - a.x, b.y - a.y}, f2v{a.x, a.y});
    const f2v bot = pfma(f2v{wm, wm}, f2v{d.x - c.x, d.y - c.y}, f2v{c.x, c.y});
    const f2v l = pfma(f2v{wr, wr}, bot - top, top);
    return f2v{cl_exp2(l.x), cl_exp2(l.y)};
}

constexpr float kAtmSun = 22.0f, kAtmMie = 21e-6f, kAtmG = 0.758f;
__device__ __forceinline__ f3 atm_krlh() { return f3{5.5e-6f, 13.0e-6f, 22.4e-6f}; }

// The phase-weighted sum of the atmosphere's in-scattering integrals (:435-438) for the normalised view ray r.
__device__ __forceinline__ f3 atmosphere_phase(f3 r, f3 pSun, f3 totalRlh, f3 totalMie) {
    const float PI = 3.141592f, g0 = kAtmG;
    const float mu = dot3(r, pSun), mumu = mu * mu, gg = g0 * g0;
    const float pRlh = 3.0f / (16.0f * PI) * (1.0f + mumu);
    const float pMie = 3.0f / (8.0f * PI) * ((1.0f - gg) * (mumu + 1.0f)) / (powf(1.0f + gg - 2.0f * mu * g0, 1.5f) * (2.0f + gg));
    return ((atm_krlh() * pRlh) * totalRlh + totalMie * (pMie * kAtmMie)) * kAtmSun;
}

// The in-scattering integrals totalRlh / totalMie of the normalised view ray r (:375-433); false when the ray misses the
// atmosphere (the colour is then 0).
__device__ __forceinline__ bool atmosphere_integrals(f3 r, f3 r0, f3 pSun, float iTime, const OdLut& L, f3& totalRlh,
                                                     f3& totalMie) {
    const float kMie = kAtmMie;
    const f3 kRlh = atm_krlh();
    float2 p = rsi(r0, r, kRAtmos);
    if (p.x > p.y) return false;
    p.y = fminf(p.y, rsi(r0, r, kRPlanet).x);
    const float iStep = (p.y - p.x) / 16.0f;
    totalRlh = f3{0, 0, 0};
    totalMie = f3{0, 0, 0};
    f2v iOd = {0.0f, 0.0f};   // (Rayleigh, Mie) optical depth of the primary ray, one packed pair
    const float C2 = dot3(pSun, pSun), cR = -kRPlanet * kExpR, cM = -kRPlanet * kExpM;
    for (int i = 0; i < 16; i++) {
        const f3 iPos = r0 + r * (iTime + iStep * 0.5f);
        const float A = dot3(iPos, iPos), PoD = dot3(iPos, pSun);
        const float iLen = cl_sqrt(A);
        // (odR, odM) and the accumulators as packed pairs: element-wise the scalar operations (the same bits)
        const f2v ea = pfma(f2v{iLen, iLen}, f2v{kExpR, kExpM}, f2v{cR, cM});
        const f2v od = f2v{cl_exp2(ea.x), cl_exp2(ea.y)} * f2v{iStep, iStep};
        const float odR = od.x, odM = od.y;
        iOd = iOd + od;
        f2v jOd;
        // below the planet's surface (a ray that hits the ground keeps stepping underground: its first sample is at
        // elapsed_time and its step spans the whole chord, quirk Q10) the depths grow without bound: marched
        if (L.t && iLen >= kRPlanet) {
            jOd = secondary_od_lut(L, iLen, PoD);
            if (!(jOd.x == jOd.x) || !(jOd.y == jOd.y)) jOd = secondary_od(A, PoD, C2);   // no table entry here
        } else {
            jOd = secondary_od(A, PoD, C2);
        }
        const f2v od_sum = iOd + jOd;
        const float fm = kMie * od_sum.y;
        const float fr = od_sum.x;
        const f3 attn = f3{cl_exp(-(fm + kRlh.x * fr)), cl_exp(-(fm + kRlh.y * fr)), cl_exp(-(fm + kRlh.z * fr))};
        totalRlh = totalRlh + attn * odR;
        totalMie = totalMie + attn * odM;
        iTime += iStep;
    }
    return true;
}

__device__ f3 atmosphere(f3 r, f3 r0, f3 pSun, float iTime, const OdLut& L) {
    r = normalize3(r);
    f3 totalRlh, totalMie;
    if (!atmosphere_integrals(r, r0, pSun, iTime, L, totalRlh, totalMie)) return f3{0.0f, 0.0f, 0.0f};
    return atmosphere_phase(r, pSun, totalRlh, totalMie);
}

// Sky-view table (round 4). The camera position r0, the sun and iTime are fixed for the frame, so the integrals are a
// function of the view direction alone, and by the mirror symmetry across the vertical plane through the sun, of the
// direction's elevation sine e = r.up and its azimuth away from the sun's, as u = sin(az / 2). They change branch where
// the ray grazes the planet (e = +-eh, eh = sqrt(1 - rPlanet^2 / |r0|^2)): below -eh the ray hits the ground ahead, within
// (-eh, eh) it misses (the reference's rsi returns -1 and the primary step spans the chord behind the camera), above +eh
// the line's ground hit lies behind (quirk Q10's min keeps it). One kSvT x kSvU table per branch, rows dense towards
// the grazing direction (e = boundary +- t^2 span, with a margin dl inside the branch so that the entries' own fp32
// branch test is unambiguous; the middle band linear in e); each pixel takes the branch from the same planet-intersection
// discriminant rsi computes, interpolates (totalRlh, totalMie) bilinearly and applies its exact phase functions. Against
// evaluating every pixel (float64 study over the C3 / C4 view frusta, tools/sky_table_check.py): at most 0.04 RGBA8
// levels. SOC_CLOUDS_SKY_TABLE=0 evaluates every pixel (the single-lane kernel always does).
constexpr int kSvT = 128, kSvU = 64, kSvEntries = 3 * kSvT * kSvU;
struct SkyTab {
    const float4* t;   // [3][kSvT][kSvU] x 2: (totalRlh.xyz, totalMie.x), (totalMie.yz, -, -); nullptr: no table
    float upx, upy, upz, shx, shy, shz, btx, bty, btz;   // frame: up = r0 / |r0|, the sun's horizontal direction, up x sh
    float eh, dl;
};
__device__ __forceinline__ f3 sv_dir(const SkyTab& st, int b, float t, float u) {
    const float eh = st.eh, dl = st.dl;
    const float e = b == 0 ? -(eh + dl) - t * t * (1.0f - eh - dl)
                  : b == 1 ? -(eh - dl) + t * 2.0f * (eh - dl) : (eh + dl) + t * t * (1.0f - eh - dl);
    const float c = 1.0f - 2.0f * u * u, sn = sqrtf(fmaxf(1.0f - c * c, 0.0f)), ce = sqrtf(fmaxf(1.0f - e * e, 0.0f));
    return f3{st.upx * e + ce * (c * st.shx + sn * st.btx), st.upy * e + ce * (c * st.shy + sn * st.bty),
              st.upz * e + ce * (c * st.shz + sn * st.btz)};
}
__global__ __launch_bounds__(kWorkgroup) void clouds_sky_table(float4* __restrict__ tab, CloudParams p, SkyTab st, OdLut L) {
    const int i = (int)(blockIdx.x * kWorkgroup + threadIdx.x);
    if (i >= kSvEntries) return;
    const int b = i / (kSvT * kSvU), rem = i - b * (kSvT * kSvU), ti = rem / kSvU, uj = rem - ti * kSvU;
    const f3 r = normalize3(sv_dir(st, b, (float)ti / (float)(kSvT - 1), (float)uj / (float)(kSvU - 1)));
    const f3 r0 = f3{0.0f + p.cam[0], 6372e3f + p.cam[1], 0.0f + p.cam[2]};
    f3 R = f3{0.0f, 0.0f, 0.0f}, M = R;
    if (!atmosphere_integrals(r, r0, f3{p.sun[0], p.sun[1], p.sun[2]}, p.elapsed, L, R, M)) R = M = f3{0.0f, 0.0f, 0.0f};
    tab[2 * i] = float4{R.x, R.y, R.z, M.x};
    tab[2 * i + 1] = float4{M.y, M.z, 0.0f, 0.0f};
}
__device__ f3 atmosphere_table(f3 r, f3 r0, f3 pSun, const SkyTab& st) {
    r = normalize3(r);
    const float2 pa = rsi(r0, r, kRAtmos);
    if (pa.x > pa.y) return f3{0.0f, 0.0f, 0.0f};
    // the branch atmosphere_integrals takes: rsi(r0, r, rPlanet)'s discriminant and the sign of r0.r
    float PoD;
    const float delta = rsi_delta(r0, r, kRPlanet, PoD);
    const int b = delta < 0.0f ? 1 : (PoD >= 0.0f ? 2 : 0);
    const f3 up = f3{st.upx, st.upy, st.upz};
    const float e = dot3(r, up), eh = st.eh, dl = st.dl;
    float t = b == 0 ? sqrtf(fmaxf((-(eh + dl) - e) / (1.0f - eh - dl), 0.0f))
            : b == 1 ? (e + (eh - dl)) / (2.0f * (eh - dl)) : sqrtf(fmaxf((e - (eh + dl)) / (1.0f - eh - dl), 0.0f));
    t = fminf(fmaxf(t, 0.0f), 1.0f);
    const f3 dh = f3{r.x - up.x * e, r.y - up.y * e, r.z - up.z * e};
    const float nh = length3(dh);
    const float c = nh > 0.0f ? fminf(fmaxf((dh.x * st.shx + dh.y * st.shy + dh.z * st.shz) / nh, -1.0f), 1.0f) : 1.0f;
    const float u = sqrtf(fmaxf((1.0f - c) * 0.5f, 0.0f));
    const float ft = t * (float)(kSvT - 1), fu = u * (float)(kSvU - 1);
    const int i0 = min((int)ft, kSvT - 2), j0 = min((int)fu, kSvU - 2);
    const float wt = ft - (float)i0, wu = fu - (float)j0;
    const float4* row = st.t + 2 * ((b * kSvT + i0) * kSvU + j0);
    auto lerp4 = [](float4 a, float4 c4, float w) {
        return float4{a.x + w * (c4.x - a.x), a.y + w * (c4.y - a.y), a.z + w * (c4.z - a.z), a.w + w * (c4.w - a.w)};
    };
    const float4 a0 = lerp4(row[0], row[2], wu), a1 = lerp4(row[1], row[3], wu);
    const float4 b0 = lerp4(row[2 * kSvU], row[2 * kSvU + 2], wu), b1 = lerp4(row[2 * kSvU + 1], row[2 * kSvU + 3], wu);
    const float4 v0 = lerp4(a0, b0, wt), v1 = lerp4(a1, b1, wt);
    return atmosphere_phase(r, pSun, f3{v0.x, v0.y, v0.z}, f3{v0.w, v1.x, v1.y});
}

constexpr int TX = 16, TY = 16;

// View ray of pixel (x, y): main(), :445-452 (ray_uv = pixel / (resolution - 1), not texel centres).
__device__ __forceinline__ f3 sky_dir(const CloudParams& p, int x, int y) {
    const float ru = div_rn((float)x, p.res_x_m1, p.r_res_x_m1), rv = div_rn((float)y, p.res_y_m1, p.r_res_y_m1);
    const float ndx = ru * 2.0f - 1.0f, ndy = rv * 2.0f - 1.0f;
    const f4 rvs = mul_rn(p.inv_proj, f4{ndx, ndy, -1.0f, 0.0f});
    const f4 rws = mul_rn(p.inv_view, f4{rvs.x, rvs.y, -1.0f, 0.0f});
    return normalize3_rn(f3{rws.x, rws.y, rws.z});
}

__device__ __forceinline__ f3 sky_atmosphere(const CloudParams& p, f3 dir, const OdLut& L = OdLut{nullptr, 0.0f}) {
    if (SOC_CLOUDS_PROFILE == 2 || SOC_CLOUDS_PROFILE == 3) return f3{0.1f, 0.2f, 0.3f};
    const f3 r0 = f3{0.0f + p.cam[0], 6372e3f + p.cam[1], 0.0f + p.cam[2]};
    return atmosphere(dir, r0, f3{p.sun[0], p.sun[1], p.sun[2]}, p.elapsed, L);
}

// Clouds over the atmosphere colour, sun factor, RGBA8 (main(), :466-477).
__device__ __forceinline__ uint32_t sky_clouds(const CloudParams& p, const uint32_t* quads, int x, int y, f3 dir, f3 color) {
    Ctx cx;
    cx.quads = quads;
    cx.cam_x = p.cam[0];
    cx.cam_z = p.cam[2];
    cx.time = -1.0f * 0.02f * p.elapsed;
    const float dither = bayer16((float)x, (float)y);
    if (SOC_CLOUDS_PROFILE != 1)
        color = volumetric_clouds(cx, dir, f3{p.sun[0], p.sun[1], p.sun[2]}, color, dither, f3{0.8f, 0.8f, 0.8f});
    color = color * p.sun_factor;
    return pack_unorm8x4(f4{color.x, color.y, color.z, 1.0f});
}

// Shading of one sky pixel (main(), :445-477).
__device__ __forceinline__ uint32_t shade_sky(const CloudParams& p, const uint32_t* quads, int x, int y) {
    const f3 dir = sky_dir(p, x, y);
    return sky_clouds(p, quads, x, y, dir, sky_atmosphere(p, dir));
}

// Stage the noise .x channel as 2x2 REPEAT quads (quad i = texels (x,y), (x+1,y), (x,y+1), (x+1,y+1)).
template <bool NOISE_R8>
__device__ __forceinline__ void stage_noise(const DImg& noise, uint32_t* quads, int tid, int nthreads) {
    for (int i = tid; i < kTable; i += nthreads) {
        const int ny = i / kTW, nx = (i - ny * kTW) & kNoiseMask;
        const int nyw = ny & kNoiseMask;
        const int nx1 = (nx + 1) & kNoiseMask, ny1 = (nyw + 1) & kNoiseMask;
        auto texel = [&](int tx, int ty) -> uint32_t {
            if (NOISE_R8) return row_ptr<uint8_t>(noise, ty)[tx];
            return row_ptr<uint32_t>(noise, ty)[tx] & 0xffu;
        };
        quads[i] = texel(nx, nyw) | (texel(nx1, nyw) << 8) | (texel(nx, ny1) << 16) | (texel(nx1, ny1) << 24);
    }
}

template <bool NOISE_R8>
__device__ __forceinline__ void stage_noise_wide(const DImg& noise, uint2* quads, int tid, int nthreads) {
    for (int i = tid; i < kTable; i += nthreads) {
        const int ny = i / kTW, nx = (i - ny * kTW) & kNoiseMask;
        const int nyw = ny & kNoiseMask;
        const int nx1 = (nx + 1) & kNoiseMask, ny1 = (nyw + 1) & kNoiseMask;
        auto texel = [&](int tx, int ty) -> uint32_t {
            if (NOISE_R8) return row_ptr<uint8_t>(noise, ty)[tx];
            return row_ptr<uint32_t>(noise, ty)[tx] & 0xffu;
        };
        quads[i] = wide_quad_entry(texel(nx, nyw), texel(nx1, nyw), texel(nx, ny1), texel(nx1, ny1));
    }
}

template <bool NOISE_R8>
__device__ __forceinline__ void stage_noise_rows(const DImg& noise, RowF* rows, int tid, int nthreads) {
    for (int i = tid; i < kRowTable; i += nthreads) {
        const int ny = (i / kTW) & kNoiseMask, nx = (i % kTW) & kNoiseMask, nx1 = (nx + 1) & kNoiseMask;
        auto texel = [&](int tx, int ty) -> uint32_t {
            if (NOISE_R8) return row_ptr<uint8_t>(noise, ty)[tx];
            return row_ptr<uint32_t>(noise, ty)[tx] & 0xffu;
        };
        rows[i] = RowF{row_entry(texel(nx, ny), texel(nx1, ny))};
    }
}

// Copy a prebuilt quad table (N16 16-B chunks) into LDS: each lane issues its loads in batches of 4 before their LDS
// stores (the per-texel staging loop took 4 byte loads per entry and waited on every round: 26 rounds for a
// 256-lane workgroup).
template <int N16>
__device__ __forceinline__ void stage_noise_table(const uint4* __restrict__ src, uint4* dst, int tid, int nthreads) {
    for (int k0 = tid; k0 < N16; k0 += 4 * nthreads) {
        const int k1 = k0 + nthreads, k2 = k1 + nthreads, k3 = k2 + nthreads;
        const uint4 a = src[k0];
        uint4 b = uint4{0u, 0u, 0u, 0u}, c = b, d = b;
        if (k1 < N16) b = src[k1];
        if (k2 < N16) c = src[k2];
        if (k3 < N16) d = src[k3];
        dst[k0] = a;
        if (k1 < N16) dst[k1] = b;
        if (k2 < N16) dst[k2] = c;
        if (k3 < N16) dst[k3] = d;
    }
}

__device__ __forceinline__ bool is_sky(const CloudParams& p, const DImg& depth, int x, int y) {
    return sample_f32(depth, div_rn((float)x, p.res_x_m1, p.r_res_x_m1), div_rn((float)y, p.res_y_m1, p.r_res_y_m1)) ==
           1.0f;   // textureLod(depth, ray_uv, 0), :458
}

// Single-kernel path (no workspace): 16x16 tiles, a tile without sky exits after its depth test.
template <bool NOISE_R8>
__global__ __launch_bounds__(kWorkgroup) void clouds_kernel(DImg depth, DImg noise, DImg target, CloudParams p) {
    __shared__ uint32_t quads[kTable];
    const int x = blockIdx.x * TX + threadIdx.x, y = blockIdx.y * TY + threadIdx.y;
    const int tid = threadIdx.y * TX + threadIdx.x;
    const bool inside = x < p.res_x && y < p.res_y && x < target.w && y < target.h;
    const bool sky = inside && is_sky(p, depth, x, y);
    if (!__syncthreads_or(sky)) {
        if (inside) row_ptr_w<uint32_t>(target, y)[x] = pack_unorm8x4(f4{0.2f, 0.4f, 1.0f, 1.0f});
        return;
    }
    stage_noise<NOISE_R8>(noise, quads, tid, TX * TY);
    __syncthreads();
    if (!inside) return;
    row_ptr_w<uint32_t>(target, y)[x] = sky ? shade_sky(p, quads, x, y) : pack_unorm8x4(f4{0.2f, 0.4f, 1.0f, 1.0f});
}

// Three-kernel path, stage 1 (classify). Every pixel first gets the constant non-sky colour (a sky pixel
// is overwritten by the march later in stream order); sky pixels are appended to a compact list.
// A workgroup covers 64x16 tiles, each wave a 32x8 quarter of one (every row of a wave one full 128-B line of
// depth and of the target), each lane 4 horizontal pixels (one 16-B store). Entries are ordered
// row-major inside a wave's quarter, so a wave of the march takes a compact 32x2 block. The list offset
// costs ONE atomic per workgroup that has sky: device-scope atomics on one address serialise across
// the XCDs (one per wave cost ~95 us at 4K).
// kClassifyTiles 64x16 tiles stacked vertically per workgroup (a 64x64 region): one list atomic per region instead of per
// tile. The atomics on the one counter serialise across the XCDs: at one per 64x16 tile they cost C4 34 of its 59 us
// (profiles/r04_probe_clouds_classify.txt).
constexpr int kClassifyTiles = 4;
// HOIST: every tile's depth samples issued before the first tile's stores (one memory round trip instead of four; the
// same samples). Faster alone (C3 299 -> 291 us, C4 541 -> 504 us CloudRendering) but in the frame only where the sky
// lane is the critical path (C4 +1.8 %; C3 -1.1 %, C2 -1 %: profiles/r05_ab_clouds_classify_hoist.txt), so the render
// graph selects it for a sky-bound frame (a high-priority sky lane) and the standalone pass by SOC_CLOUDS_CLASSIFY_HOIST.
template <bool HOIST>
__global__ __launch_bounds__(kWorkgroup) void clouds_classify(DImg depth, DImg target, CloudParams p, int vec_store,
                                                       uint32_t* __restrict__ counter, uint32_t* __restrict__ list) {
    __shared__ uint32_t wave_total[kClassifyTiles][4];
    __shared__ uint32_t wg_base;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int x0 = blockIdx.x * 64 + (wave & 1) * 32 + (lane & 7) * 4;
    const int W = min(p.res_x, target.w), H = min(p.res_y, target.h);
    const uint32_t other = pack_unorm8x4(f4{0.2f, 0.4f, 1.0f, 1.0f});
    const unsigned long long below = (1ull << lane) - 1ull;
    uint32_t masks = 0;   // bits 4k..4k+3: pixels (x0 + 0..3, y_k) of tile k are sky
    uint32_t before[kClassifyTiles];
    // HOIST: every tile's depth samples issued before the first tile's stores (rows clamped into the image; a row past
    // H is not used), so the 4 tiles cost one memory round trip instead of four
    float dk[kClassifyTiles][4];
    auto load_all = [&](auto sample) {
#pragma unroll
        for (int k = 0; k < kClassifyTiles; ++k) {
            const int y = min((blockIdx.y * kClassifyTiles + k) * 16 + (wave >> 1) * 8 + (lane >> 3), H - 1);
            const float ray_v = div_rn((float)y, p.res_y_m1, p.r_res_y_m1);
#pragma unroll
            for (int j = 0; j < 4; ++j) dk[k][j] = sample(div_rn((float)min(x0 + j, W - 1), p.res_x_m1, p.r_res_x_m1), ray_v);
        }
    };
    if (HOIST && depth.w >= 2) {   // sample_f32's row-pair form without its per-sample extent test (same texels, weights)
        load_all([&](float u, float v) {
            const Axis ax = axis_clamp(u, depth.w), ay = axis_clamp(v, depth.h);
            typedef float f2u4 __attribute__((ext_vector_type(2))) __attribute__((aligned(4)));
            const f2u4 r0 = *reinterpret_cast<const f2u4*>(row_ptr<float>(depth, ay.i0) + ax.i0);
            const f2u4 r1 = *reinterpret_cast<const f2u4*>(row_ptr<float>(depth, ay.i1) + ax.i0);
            return bilerp1(r0.x, r0.y, r1.x, r1.y, ax.w, ay.w);
        });
    } else if (HOIST) {
        load_all([&](float u, float v) { return sample_f32(depth, u, v); });
    }
#pragma unroll
    for (int k = 0; k < kClassifyTiles; ++k) {
        const int y = (blockIdx.y * kClassifyTiles + k) * 16 + (wave >> 1) * 8 + (lane >> 3);
        uint32_t mask = 0;   // bit j: pixel (x0 + j, y) is sky
        if (y < H) {
            if (!HOIST) {   // the round-4 order: this tile's samples, then its stores
                const float ray_v = div_rn((float)y, p.res_y_m1, p.r_res_y_m1);
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    dk[k][j] = sample_f32(depth, div_rn((float)min(x0 + j, W - 1), p.res_x_m1, p.r_res_x_m1), ray_v);
            }
            const float* d = dk[k];
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (x0 + j < W && d[j] == 1.0f) mask |= 1u << j;
            uint32_t* row = row_ptr_w<uint32_t>(target, y);
            if (vec_store && x0 + 3 < W) {
                *reinterpret_cast<uint4*>(row + x0) = uint4{other, other, other, other};
            } else {
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if (x0 + j < W) row[x0 + j] = other;
            }
        }
        uint32_t b4 = 0, total = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const unsigned long long b = __ballot((mask >> j) & 1u);
            b4 += (uint32_t)__builtin_popcountll(b & below);
            total += (uint32_t)__builtin_popcountll(b);
        }
        before[k] = b4;
        masks |= mask << (4 * k);
        if (lane == 0) wave_total[k][wave] = total;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t sum = 0;
        for (int k = 0; k < kClassifyTiles; ++k) sum += wave_total[k][0] + wave_total[k][1] + wave_total[k][2] + wave_total[k][3];
        if (SOC_CLOUDS_PROFILE == 5) wg_base = (blockIdx.y * gridDim.x + blockIdx.x) * (1024u * kClassifyTiles);
        else wg_base = sum ? atomicAdd(counter, sum) : 0u;
    }
    __syncthreads();
    if (!masks) return;
    // entries in tile order, then wave order, then the wave's row-major order (as one tile per workgroup gave)
    uint32_t tile_base = wg_base;
#pragma unroll
    for (int k = 0; k < kClassifyTiles; ++k) {
        const uint32_t mask = (masks >> (4 * k)) & 15u;
        const int y = (blockIdx.y * kClassifyTiles + k) * 16 + (wave >> 1) * 8 + (lane >> 3);
        uint32_t at = tile_base + before[k];
        for (int w = 0; w < wave; ++w) at += wave_total[k][w];
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if ((mask >> j) & 1u) list[at++] = ((uint32_t)y << 16) | (uint32_t)(x0 + j);
        tile_base += wave_total[k][0] + wave_total[k][1] + wave_total[k][2] + wave_total[k][3];
    }
}

// Three-kernel path, stage 2: the atmosphere of every listed sky pixel (no LDS, few registers, so many
// more lanes are resident than in the cloud march), kept in fp32 in the workspace.
template <bool TAB>
__global__ __launch_bounds__(kWorkgroup) __attribute__((amdgpu_waves_per_eu(8))) void clouds_atmosphere(CloudParams p, const uint32_t* __restrict__ counter,
                                                         const uint32_t* __restrict__ list, float4* __restrict__ atmos,
                                                         OdLut lut, SkyTab st) {
    const uint32_t count = *counter;
    const f3 r0 = f3{0.0f + p.cam[0], 6372e3f + p.cam[1], 0.0f + p.cam[2]}, sun = f3{p.sun[0], p.sun[1], p.sun[2]};
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < count; i += gridDim.x * 256u) {
        const uint32_t e = list[i];
        const f3 dir = sky_dir(p, (int)(e & 0xffffu), (int)(e >> 16));
        const f3 c = TAB && SOC_CLOUDS_PROFILE != 2 && SOC_CLOUDS_PROFILE != 3 ? atmosphere_table(dir, r0, sun, st)
                                                                             : sky_atmosphere(p, dir, lut);
        atmos[i] = float4{c.x, c.y, c.z, 0.0f};
    }
}

// ---- balanced cloud march: dense-step pairs ----------------------------------------------------
// The cost of a sky pixel is dominated by its dense steps (each adds a 10-step sun march), which vary
// from 0 to 24 between neighbouring screen regions; one pixel per lane leaves the kernel waiting on
// its heaviest waves. The march is therefore split at the dense steps:
//   density  one lane per sky pixel: the 24 primary steps -> dense-step mask; the pixel's
//            (pixel, step) pairs are appended to one of 8 sharded pair lists (one atomic per workgroup)
//   sunvis   one lane per pair: od and the sun visibility of that step (balanced work)
//   resolve  one lane per sky pixel: the reference's accumulation over its dense steps, in order
// Every position is re-derived with the same additions (cp = inc*dither + start, += inc), so od and vis
// are the bits the single-lane march computes. A workgroup whose pairs do not fit the list marks its
// pixels for the single-lane march in resolve.
constexpr int kShards = 8;
// clouds_sunvis workgroup: 512 lanes (the 26 KiB noise table caps residency at 6 workgroups per CU: 512 lanes give the
// full 8 waves per SIMD); its launch bound
constexpr uint32_t kSunvisLanes = 512;
constexpr uint32_t kInline = 0x80000000u;   // pix_mask flag: march this pixel in resolve

struct PairBufs {
    uint32_t* counts;     // [kShards] pair counts (workspace counter block)
    uint32_t* pairs;      // [kShards * cap] (list index << 5) | step
    float* od;            // [kShards * cap] od of each pair's step (clouds_density)
    float* vis;           // [kShards * cap] sun visibility of each pair's step (clouds_sunvis); od and vis in two dense
                          // arrays (round 5: one float2 array took each kernel's 4-byte writes at an 8-byte stride, so
                          // every written line was half written)
    uint32_t* pix_mask;   // [W*H] per list entry: dense-step mask | kInline
    uint32_t* batch_base; // [W*H/256] per 256-entry batch: physical index of its first pair | kInline
    float4* geom;         // [W*H] x 2 per list entry: (start, dither), (inc, stepLength) of its march (density
                          // writes it for upward rays when store_geom; sunvis and resolve read it instead of re-deriving
                          // it; store_geom == 0: they re-derive it from the list entry, the same bits)
    float* od_tmp;        // [od_blocks][24][256]: per density workgroup, the od of its current batch's dense steps until
                          // their pair slots are known; density then stores od in od[slot], and sunvis only adds vis
    const uint32_t* noise_quads;  // [kTableU32] the frame's noise quad table (clouds_od_lut), or nullptr: stage_noise
    const uint2* noise_wide;      // [kTableU2] the same quads in float form (stage_noise_wide)
    const uint32_t* noise_rows;   // [kRowU32] the row table (stage_noise_rows)
    uint32_t store_geom;  // tuning knob SOC_CLOUDS_GEOM
    uint32_t od_blocks;   // density workgroups the od scratch holds (the density grid is clamped to it)
    uint32_t n;           // list capacity (W*H)
    uint32_t cap;         // pairs per shard
};



// Rank of this lane among the lanes of its wave whose mask has step `st`.
__device__ __forceinline__ uint32_t mask_ballot_rank(uint32_t mask, uint32_t st, uint32_t lane) {
    const unsigned long long b = __ballot((mask >> st) & 1u);
    return (uint32_t)__builtin_popcountll(b & ((1ull << lane) - 1ull));
}
__device__ __forceinline__ uint32_t pair_offset(const uint32_t (*offs)[4], uint32_t st, uint32_t wave, uint32_t rank) {
    return offs[st][wave] + rank;
}
// Step-major slot offsets of a 256-lane batch: offs[s][w] = number of pairs of steps < s (all waves)
// plus those of step s in waves < w; offs[24][0] = total. Called by every lane of the workgroup
// (ballots per wave, then one lane scans the 24 x 4 counts).
__device__ __forceinline__ void batch_slots(uint32_t mask, uint32_t lane, uint32_t wave, uint32_t (*offs)[4],
                                            uint32_t& /*unused*/, uint32_t tid) {
    if (__ballot(mask != 0u) == 0ull) {   // no dense step in this wave (C4's below-horizon sky): 24 zero counts
        if (lane < 24) offs[lane][wave] = 0u;
    } else {
#pragma unroll 1
        for (uint32_t st = 0; st < 24; ++st) {
            const unsigned long long b = __ballot((mask >> st) & 1u);
            if (lane == 0) offs[st][wave] = (uint32_t)__builtin_popcountll(b);
        }
    }
    __syncthreads();
    // the exclusive scan of the 96 counts in (step, wave) order by wave 0: lane l < 48 takes counts 2l and 2l + 1, a wave
    // prefix sum of the pairs (6 shuffle steps) instead of one lane's 96 dependent LDS round trips (the same sums)
    if (tid < 64) {
        uint32_t* flat = &offs[0][0];
        const uint32_t c0 = lane < 48 ? flat[2 * lane] : 0u, c1 = lane < 48 ? flat[2 * lane + 1] : 0u;
        uint32_t incl = c0 + c1;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t o = (uint32_t)__shfl_up((int)incl, d, 64);
            if ((int)lane >= d) incl += o;
        }
        const uint32_t excl = incl - (c0 + c1);
        if (lane < 48) {
            flat[2 * lane] = excl;
            flat[2 * lane + 1] = excl + c0;
        }
        if (lane == 47) offs[24][0] = incl;
    }
    __syncthreads();
}

// The march geometry and dither of list entry i: stored by clouds_density (store_geom), or re-derived from the entry's
// pixel with the same functions (the same bits; a few dozen VALU against the ~1,500 of a pair's sun march, and no 32-B
// geometry read per pair).
__device__ __forceinline__ MarchGeom pair_geometry(const CloudParams& p, const uint32_t* __restrict__ list, const PairBufs& pb,
                                                   uint32_t i, float& dither) {
    if (pb.store_geom) {
        const float4 g0 = pb.geom[2 * i], g1 = pb.geom[2 * i + 1];
        dither = g0.w;
        return MarchGeom{f3{g0.x, g0.y, g0.z}, f3{g1.x, g1.y, g1.z}, g1.w};
    }
    const uint32_t e = list[i];
    const int x = (int)(e & 0xffffu), y = (int)(e >> 16);
    dither = bayer16((float)x, (float)y);
    return march_geometry(sky_dir(p, x, y));
}

// ROWS: the noise from the float-form row table (RowF: the same 26 KiB of LDS, half the bilinear's issue time)
template <bool NOISE_R8, int DB = 1, bool ROWS = false>
// 6 waves/SIMD: 80 VGPRs with 20 B of scratch, measured faster than 5 waves without a spill (profiles/r04_probe_clouds_scan.txt)
__global__ __launch_bounds__(kWorkgroup) __attribute__((amdgpu_waves_per_eu(6))) void clouds_density(
    DImg noise, CloudParams p, const uint32_t* __restrict__ counter, const uint32_t* __restrict__ list, PairBufs pb) {
    using Q = typename std::conditional<ROWS, RowF, uint32_t>::type;
    constexpr int kN16 = ROWS ? kRowU32 / 4 : kTableU32 / 4;
    __shared__ uint4 quads4[kN16];
    Q* quads = reinterpret_cast<Q*>(quads4);
    __shared__ uint32_t offs[25][4];
    __shared__ uint32_t wg_base;
    const uint32_t count = *counter;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (blockIdx.x * 256u >= count) return;
    const uint32_t* pre_tab = ROWS ? pb.noise_rows : pb.noise_quads;
    if (pre_tab) stage_noise_table<kN16>(reinterpret_cast<const uint4*>(pre_tab), quads4, tid, 256);
    else if constexpr (ROWS) stage_noise_rows<NOISE_R8>(noise, quads, tid, 256);
    else stage_noise<NOISE_R8>(noise, quads, tid, 256);
    __syncthreads();
    CtxT<Q> cx;
    cx.quads = quads;
    cx.cam_x = p.cam[0];
    cx.cam_z = p.cam[2];
    cx.time = -1.0f * 0.02f * p.elapsed;
    const uint32_t shard = blockIdx.x & (kShards - 1);
    float* const od_tmp = pb.od_tmp + (size_t)blockIdx.x * (24 * 256) + tid;   // this lane's od of dense step s at [s * 256]
    // workgroup-uniform trip count: every lane reaches the barriers of every round
    for (uint32_t first = blockIdx.x * 256u; first < count; first += gridDim.x * 256u) {
        const uint32_t i = first + tid;
        uint32_t mask = 0;
        if (i < count) {
            const uint32_t e = list[i];
            const int x = (int)(e & 0xffffu), y = (int)(e >> 16);
            const f3 dir = sky_dir(p, x, y);
            if (SOC_CLOUDS_PROFILE != 1 && !(dir.y < 0.0f)) {
                const MarchGeom mg = march_geometry(dir);
                const float dither = bayer16((float)x, (float)y);
                if (pb.store_geom) {
                    pb.geom[2 * i] = float4{mg.start.x, mg.start.y, mg.start.z, dither};
                    pb.geom[2 * i + 1] = float4{mg.inc.x, mg.inc.y, mg.inc.z, mg.stepLength};
                }
                f3 cp = step_position(mg, dither, 0);
                for (int s = 0; s < 24; cp = step_next(mg, dither, s, cp), s++) {
                    const float od = get_clouds(cx, cp) * mg.stepLength;
                    if (!(od <= 0.0f)) {
                        mask |= 1u << s;
                        od_tmp[s * 256] = od;
                    }
                }
            }
        }
        // pairs in step-major order within the batch (lanes of a sunvis wave then share the step and
        // march neighbouring rays); one atomic per batch on this workgroup's shard
        uint32_t slot_base;
        batch_slots(mask, lane, wave, offs, wg_base, tid);
        __shared__ uint32_t fail_from;
        if (tid == 0) {
            const uint32_t total = offs[24][0];
            uint32_t base = 0;
            bool fail = false;
            if (total) {
                base = atomicAdd(&pb.counts[shard], total);
                fail = base + total > pb.cap;
            }
            wg_base = fail ? kInline : shard * pb.cap + base;
            fail_from = fail ? base : pb.cap;
            pb.batch_base[first >> 8] = wg_base;
        }
        __syncthreads();
        slot_base = wg_base;
        // an overflowing batch leaves its reserved slots below the capacity empty: mark them
        for (uint32_t k = fail_from + tid; k < pb.cap && k < fail_from + offs[24][0]; k += 256u)
            pb.pairs[shard * pb.cap + k] = 0xffffffffu;
        if (i < count) pb.pix_mask[i] = mask | ((slot_base & kInline) ? kInline : 0u);
        if (!(slot_base & kInline) && __ballot(mask != 0u) != 0ull) {   // workgroup-uniform, then wave-uniform
            // uniform loop: the ballot of every step sees every lane of the wave. DB > 1: the lane's od scratch of DB
            // steps is read together (every lane, every step: its own scratch, always in bounds) before the stores, one
            // memory latency per DB steps instead of one per dense step (the same values)
            if constexpr (DB == 1) {
                for (uint32_t st = 0; st < 24; ++st) {
                    const uint32_t rank = mask_ballot_rank(mask, st, lane);
                    if ((mask >> st) & 1u) {
                        const uint32_t slot = slot_base + pair_offset(offs, st, wave, rank);
                        pb.pairs[slot] = (i << 5) | st;
                        pb.od[slot] = od_tmp[st * 256];   // this lane's own write
                    }
                }
            } else {
                static_assert(24 % DB == 0, "whole step batches");
                for (uint32_t s0 = 0; s0 < 24; s0 += DB) {
                    float odv[DB];
#pragma unroll
                    for (int b = 0; b < DB; ++b) odv[b] = od_tmp[(s0 + b) * 256];
#pragma unroll
                    for (int b = 0; b < DB; ++b) {
                        const uint32_t st = s0 + b;
                        const uint32_t rank = mask_ballot_rank(mask, st, lane);
                        if ((mask >> st) & 1u) {
                            const uint32_t slot = slot_base + pair_offset(offs, st, wave, rank);
                            pb.pairs[slot] = (i << 5) | st;
                            pb.od[slot] = odv[b];
                        }
                    }
                }
            }
        }
        __syncthreads();   // offs / wg_base are reused next round
    }
}

// 512-lane workgroups: the 26 KiB noise table per workgroup caps residency at 6 workgroups per CU, so 256 lanes
// give 6 waves per SIMD and 512 lanes give the full 8 (one table per 8 waves).
// ROWS: the float-form row table (RowF, 26 KiB: 8 waves per SIMD) instead of WIDE's quads (52 KiB: 6)
template <bool NOISE_R8, uint32_t kSunvisThreads, bool WIDE = false, bool PF = false, bool ROWS = false>
__global__ __launch_bounds__(kSunvisThreads) __attribute__((amdgpu_waves_per_eu(kSunvisThreads == 512 && !WIDE ? 8 : 6))) void clouds_sunvis(
    DImg noise, CloudParams p, const uint32_t* __restrict__ list, PairBufs pb) {
    static_assert(!(ROWS && WIDE), "one table form");
    using Q = typename std::conditional<ROWS, RowF, typename std::conditional<WIDE, uint2, uint32_t>::type>::type;
    constexpr int kN16 = ROWS ? kRowU32 / 4 : WIDE ? kTableU2 / 2 : kTableU32 / 4;
    __shared__ uint4 quads4[kN16];
    Q* quads = reinterpret_cast<Q*>(quads4);
    __shared__ uint32_t pre[kShards + 1];
    const uint32_t tid = threadIdx.x;
    if (tid == 0) {
        uint32_t acc = 0;
        for (int k = 0; k < kShards; ++k) {
            pre[k] = acc;
            acc += min(pb.counts[k], pb.cap);   // an overflowing workgroup wrote no pairs
        }
        pre[kShards] = acc;
    }
    __syncthreads();
    const uint32_t total = pre[kShards];
    if (blockIdx.x * kSunvisThreads >= total) return;
    const void* pre_tab = ROWS ? static_cast<const void*>(pb.noise_rows)
                               : WIDE ? static_cast<const void*>(pb.noise_wide) : static_cast<const void*>(pb.noise_quads);
    if (pre_tab) stage_noise_table<kN16>(static_cast<const uint4*>(pre_tab), quads4, tid, kSunvisThreads);
    else if constexpr (ROWS) stage_noise_rows<NOISE_R8>(noise, quads, tid, kSunvisThreads);
    else if constexpr (WIDE) stage_noise_wide<NOISE_R8>(noise, quads, tid, kSunvisThreads);
    else stage_noise<NOISE_R8>(noise, quads, tid, kSunvisThreads);
    __syncthreads();
    CtxT<Q> cx;
    cx.quads = quads;
    cx.cam_x = p.cam[0];
    cx.cam_z = p.cam[2];
    cx.time = -1.0f * 0.02f * p.elapsed;
    const f3 sun = f3{p.sun[0], p.sun[1], p.sun[2]};
    auto phys_of = [&](uint32_t v) {
        int k = 0;
        while (k + 1 < kShards && v >= pre[k + 1]) ++k;
        return (uint32_t)k * pb.cap + (v - pre[k]);
    };
    const uint32_t stride = gridDim.x * kSunvisThreads;
    // PF: the next pair's list word is loaded one iteration ahead (its latency overlaps this pair's sun march; the
    // geometry load that depends on it is the only wait left at the top of an iteration)
    uint32_t v0 = blockIdx.x * kSunvisThreads + tid;
    uint32_t phys_n = 0, pr_n = 0xffffffffu;
    if (PF && v0 < total) {
        phys_n = phys_of(v0);
        pr_n = pb.pairs[phys_n];
    }
    for (uint32_t v = v0; v < total; v += stride) {
        uint32_t phys, pr;
        if constexpr (PF) {
            phys = phys_n;
            pr = pr_n;
            if (v + stride < total) {
                phys_n = phys_of(v + stride);
                pr_n = pb.pairs[phys_n];
            }
        } else {
            phys = phys_of(v);
            pr = pb.pairs[phys];
        }
        if (pr == 0xffffffffu) continue;   // slot of an overflowed batch
        const uint32_t i = pr >> 5, step = pr & 31u;
        float dither;
        const MarchGeom mg = pair_geometry(p, list, pb, i, dither);
        const f3 cp = step_position(mg, dither, (int)step);
        // od of the step is already in od[phys] (clouds_density)
        const float vis = SOC_CLOUDS_PROFILE == 3 ? 1.0f : sun_visibility(cx, cp, sun);
        pb.vis[phys] = vis;
    }
}

// TAB: the atmosphere colour from the sky-view table here (no clouds_atmosphere launch, no per-pixel colour buffer);
// else read from the atmosphere kernel's output.
template <bool NOISE_R8, bool TAB = false, int RB = 1>
__global__ __launch_bounds__(kWorkgroup) __attribute__((amdgpu_waves_per_eu(5))) void clouds_resolve(DImg noise, DImg target, CloudParams p, const uint32_t* __restrict__ counter,
                                                      const uint32_t* __restrict__ list, const float4* __restrict__ atmos,
                                                      PairBufs pb, SkyTab st) {
    __shared__ uint32_t quads[kTable];
    __shared__ uint32_t offs[25][4];
    const uint32_t count = *counter;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (blockIdx.x * 256u >= count) return;
    const f3 sun = f3{p.sun[0], p.sun[1], p.sun[2]}, sun_color = f3{0.8f, 0.8f, 0.8f};
    const f3 skyl = sky_light(sun);
    uint32_t dummy = 0;
    for (uint32_t first = blockIdx.x * 256u; first < count; first += gridDim.x * 256u) {
        const uint32_t i = first + tid;
        const bool valid = i < count;
        const uint32_t flagged = valid ? pb.pix_mask[i] : 0u;
        const uint32_t mask = flagged & ~kInline;
        const uint32_t base = pb.batch_base[first >> 8];   // workgroup-uniform
        const bool inl = (base & kInline) != 0u;
        // the single-lane march of an overflowed batch needs the noise in LDS
        if (inl) {
            stage_noise<NOISE_R8>(noise, quads, tid, 256);
            __syncthreads();
        } else {
            batch_slots(mask, lane, wave, offs, dummy, tid);   // the slot layout of clouds_density
        }
        // a wave none of whose pixels has a dense step (C4: most of its sky lies below the horizon) has nothing to
        // accumulate: it skips the 24-step ballot loop
        const bool any_dense = __ballot(mask != 0u) != 0ull;
        uint32_t e = 0;
        f3 color = f3{0.0f, 0.0f, 0.0f}, dir = f3{0.0f, 1.0f, 0.0f};
        if (valid) {
            e = list[i];
            dir = sky_dir(p, (int)(e & 0xffffu), (int)(e >> 16));
            if (TAB) {
                color = atmosphere_table(dir, f3{0.0f + p.cam[0], 6372e3f + p.cam[1], 0.0f + p.cam[2]}, sun, st);
            } else {
                const float4 a = atmos[i];
                color = f3{a.x, a.y, a.z};
            }
        }
        const int x = (int)(e & 0xffffu), y = (int)(e >> 16);
        if (SOC_CLOUDS_PROFILE == 1) {
        } else if (inl) {
            if (valid) {
                Ctx cx;
                cx.quads = quads;
                cx.cam_x = p.cam[0];
                cx.cam_z = p.cam[2];
                cx.time = -1.0f * 0.02f * p.elapsed;
                color = volumetric_clouds(cx, dir, sun, color, bayer16((float)x, (float)y), sun_color);
            }
        } else {
            const bool march = valid && !(dir.y < 0.0f);
            MarchGeom mg{};
            MarchShade ms{};
            if (march) {
                if (pb.store_geom) {
                    const float4 g0 = pb.geom[2 * i], g1 = pb.geom[2 * i + 1];
                    mg = MarchGeom{f3{g0.x, g0.y, g0.z}, f3{g1.x, g1.y, g1.z}, g1.w};
                } else {
                    mg = march_geometry(dir);   // dir: this lane's own sky_dir, as clouds_density derived it
                }
                ms = march_shade(dir, sun, skyl);
            }
            f3 scattering = f3{0.0f, 0.0f, 0.0f};
            float transmittance = 1.0f;
            // steps in order; the ballot runs on every lane of the wave (uniform loop). RB > 1: the od / vis loads of RB
            // steps are issued together (a lane without that dense step loads slot 0 and discards it), then accumulated
            // in step order: one memory latency per RB steps instead of one per step (the same values, the same bits)
            if constexpr (RB == 1) {
                for (uint32_t st = 0; any_dense && st < 24; ++st) {
                    const uint32_t rank = mask_ballot_rank(mask, st, lane);
                    if (march && ((mask >> st) & 1u)) {
                        const uint32_t slot = base + offs[st][wave] + rank;
                        march_accumulate(ms, sun_color, pb.od[slot], pb.vis[slot], scattering, transmittance);
                    }
                }
            } else {
                static_assert(24 % RB == 0, "whole step batches");
                for (uint32_t s0 = 0; any_dense && s0 < 24; s0 += RB) {
                    float odv[RB], visv[RB];
                    uint32_t has = 0u;
#pragma unroll
                    for (int b = 0; b < RB; ++b) {
                        const uint32_t st = s0 + b;
                        const uint32_t rank = mask_ballot_rank(mask, st, lane);
                        const bool h = march && ((mask >> st) & 1u);
                        has |= (h ? 1u : 0u) << b;
                        const uint32_t slot = h ? base + offs[st][wave] + rank : 0u;
                        odv[b] = pb.od[slot];
                        visv[b] = pb.vis[slot];
                    }
#pragma unroll
                    for (int b = 0; b < RB; ++b)
                        if ((has >> b) & 1u) march_accumulate(ms, sun_color, odv[b], visv[b], scattering, transmittance);
                }
            }
            if (march) color = march_finish(mg, color, scattering, transmittance);
        }
        if (valid) {
            color = color * p.sun_factor;
            row_ptr_w<uint32_t>(target, y)[x] = pack_unorm8x4(f4{color.x, color.y, color.z, 1.0f});
        }
        __syncthreads();   // offs / quads are reused next round
    }
}

// Workgroups resident on the device for a kernel of `threads` lanes per workgroup (grid of one full wave set).
template <typename K>
int resident_blocks(K kernel, int threads = 256) {
    int dev = 0, cus = 256, per_cu = 0;
    (void)hipGetDevice(&dev);
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) == hipSuccess && prop.multiProcessorCount > 0) cus = prop.multiProcessorCount;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, threads, 0) != hipSuccess || per_cu < 1) per_cu = 2;
    return per_cu * cus;
}

}  // namespace
}  // namespace soc

using namespace soc;

namespace {
// Workspace: counters (256 B: [0] sky pixels, [8..15] pair counts per shard) | sky list (u32) |
// atmosphere (float4) | per-pixel dense mask (u32) | per-batch first pair (u32) | march geometry (2 float4) | pairs (u32) |
// od per pair (float) | vis per pair (float) | od scratch of the density workgroups (24 x 256 float each, at most kDensityBlocks) |
// the secondary-ray optical-depth table (kOdR x kOdM float2, 1 MiB).
// Pair capacity 2 per pixel of the image (8 shards).
// Per 256-entry batch of the list: the physical index of its first pair (or kInline).
// density workgroups the od scratch is sized for: the resident set (6 per CU on 256 CUs is 1536) times the largest grid
// multiplier used (2: a sky-bound frame's density grid), 24 KiB each (4096 held 48 MiB more than any grid uses)
constexpr size_t kDensityBlocks = 3072;
struct CloudWs {
    uint32_t* counter;
    uint32_t* list;
    float4* atmos;
    PairBufs pb;
    float2* od_lut;   // secondary-ray optical-depth table (kOdR x kOdM)
    uint32_t* noise_quads;   // [kTableU32] noise quad tables (clouds_od_lut)
    uint2* noise_wide;       // [kTableU2]
    uint32_t* noise_rows;    // [kRowU32]
    float4* sky_tab;  // sky-view table (kSvEntries x 2 float4)
    size_t bytes;
};
CloudWs cloud_ws_layout(void* base, size_t n) {
    auto al = [](size_t v) { return (v + 255) & ~(size_t)255; };
    char* b = static_cast<char*>(base);
    CloudWs w;
    size_t off = 256;
    w.counter = reinterpret_cast<uint32_t*>(b);
    w.list = reinterpret_cast<uint32_t*>(b + off);
    off = al(off + n * 4);
    w.atmos = reinterpret_cast<float4*>(b + off);
    off = al(off + n * 16);
    w.pb.counts = w.counter + 8;
    w.pb.pix_mask = reinterpret_cast<uint32_t*>(b + off);
    off = al(off + n * 4);
    w.pb.batch_base = reinterpret_cast<uint32_t*>(b + off);
    off = al(off + (n / 256 + 1) * 4);
    w.pb.geom = reinterpret_cast<float4*>(b + off);
    off = al(off + n * 32);
    w.pb.cap = (uint32_t)((2 * n + kShards - 1) / kShards);
    w.pb.pairs = reinterpret_cast<uint32_t*>(b + off);
    off = al(off + (size_t)kShards * w.pb.cap * 4);
    w.pb.od = reinterpret_cast<float*>(b + off);
    off = al(off + (size_t)kShards * w.pb.cap * 4);
    w.pb.vis = reinterpret_cast<float*>(b + off);
    off = al(off + (size_t)kShards * w.pb.cap * 4);
    w.pb.od_tmp = reinterpret_cast<float*>(b + off);
    w.pb.od_blocks = (uint32_t)std::min<size_t>(kDensityBlocks, (n + 255) / 256);
    w.pb.n = (uint32_t)n;
    off = al(off + (size_t)w.pb.od_blocks * 24 * 256 * 4);
    w.od_lut = reinterpret_cast<float2*>(b + off);
    off = al(off + (size_t)kOdR * kOdM * sizeof(float2));
    w.sky_tab = reinterpret_cast<float4*>(b + off);
    off = al(off + (size_t)kSvEntries * 2 * sizeof(float4));
    w.noise_quads = reinterpret_cast<uint32_t*>(b + off);
    off = al(off + (size_t)kTableU32 * 4);
    w.noise_wide = reinterpret_cast<uint2*>(b + off);
    off = al(off + (size_t)kTableU2 * 8);
    w.noise_rows = reinterpret_cast<uint32_t*>(b + off);
    off = al(off + (size_t)kRowU32 * 4);
    w.bytes = off;
    return w;
}
}  // namespace

extern "C" size_t soc_cloud_rendering_workspace_size(int32_t width, int32_t height) {
    if (width <= 0 || height <= 0) return 0;
    return cloud_ws_layout(nullptr, (size_t)width * (size_t)height).bytes;
}

extern "C" int soc_cloud_rendering(const soc_globals* g, soc_img depth, soc_img noise, soc_img target, void* workspace,
                                   soc_stream stream) {
    return soc::cloud_rendering_launch(g, depth, noise, target, workspace, stream, false);
}

int soc::cloud_rendering_launch(const soc_globals* g, soc_img depth, soc_img noise, soc_img target, void* workspace,
                                soc_stream stream, bool sky_bound) {
    static const char* P = "soc_cloud_rendering";
    if (!g) return set_error(SOC_E_INVALID_ARG, "%s: null globals", P);
    int rc = check_img(depth, SOC_FMT_D32F, P, "depth");
    if (!rc) rc = check_img(target, SOC_FMT_RGBA8_UNORM, P, "target");
    if (!rc) rc = check_img(noise, 0, P, "noise");
    if (rc) return rc;
    if (noise.format != SOC_FMT_R8_UNORM && noise.format != SOC_FMT_RGBA8_UNORM)
        return set_error(SOC_E_UNSUPPORTED, "%s: noise must be R8_UNORM or RGBA8_UNORM", P);
    if (noise.width != 64 || noise.height != 64)
        return set_error(SOC_E_SHAPE, "%s: noise texture must be 64x64 (assets/Clouds/noise.png)", P);
    CloudParams p;
    p.inv_proj = mat4(g->camera_inverse_projection_matrix);
    p.inv_view = mat4(g->camera_inverse_view_matrix);
    for (int i = 0; i < 3; ++i) {
        p.sun[i] = -g->sun_info.direction[i];
        p.cam[i] = g->camera_position[i];
    }
    p.res_x = g->resolution[0];
    p.res_y = g->resolution[1];
    p.res_x_m1 = (float)g->resolution[0] - 1.0f;
    p.res_y_m1 = (float)g->resolution[1] - 1.0f;
    p.r_res_x_m1 = recip_rn(g->resolution[0] - 1);
    p.r_res_y_m1 = recip_rn(g->resolution[1] - 1);
    p.elapsed = g->elapsed_time;
    p.sun_factor = fmaxf(fminf(fabsf(p.sun[0]), fabsf(p.sun[2])) + p.sun[1], 0.0f);
    const int W = std::min(target.width, p.res_x), H = std::min(target.height, p.res_y);
    if (W <= 0 || H <= 0) return SOC_OK;
    if (W > 65535 || H > 65535) return set_error(SOC_E_SHAPE, "%s: extent above 65535", P);
    hipStream_t s = hs(stream);
    const bool r8 = noise.format == SOC_FMT_R8_UNORM;
    if (!workspace) {
        dim3 blk(TX, TY), grd(ceil_div(W, TX), ceil_div(H, TY));
        if (r8) launch("clouds_kernel", kWorkgroup, clouds_kernel<true>, grd, blk, 0, s, dimg(depth), dimg(noise), dimg(target), p);
        else launch("clouds_kernel", kWorkgroup, clouds_kernel<false>, grd, blk, 0, s, dimg(depth), dimg(noise), dimg(target), p);
        return check_launch("cloud_rendering");
    }
    // the caller sized the workspace for the target extent (soc_cloud_rendering_workspace_size)
    CloudWs ws = cloud_ws_layout(workspace, (size_t)target.width * (size_t)target.height);
    ws.pb.store_geom = (uint32_t)tuning_knob("SOC_CLOUDS_GEOM", 1);
    uint32_t* counter = ws.counter;
    uint32_t* list = ws.list;
    // the frame's secondary-ray table (SOC_CLOUDS_OD_LUT=0: march every secondary ray, the single-lane kernel's bits);
    // its kernel also clears the counter block, else a fill does
    // The same kernel builds the frame's noise quad tables (SOC_CLOUDS_NOISE_TABLE=0: each march workgroup stages them
    // from the noise image texel by texel, the same bytes).
    OdLut lut{nullptr, 0.0f};
    const bool use_lut = SOC_CLOUDS_PROFILE < 4 && tuning_knob("SOC_CLOUDS_OD_LUT", 1);
    const bool noise_tab = tuning_knob("SOC_CLOUDS_NOISE_TABLE", 1) != 0;
    const float C2 = p.sun[0] * p.sun[0] + p.sun[1] * p.sun[1] + p.sun[2] * p.sun[2];   // dot3(pSun, pSun)
    if (use_lut) lut = OdLut{ws.od_lut, C2};
    ws.pb.noise_quads = noise_tab ? ws.noise_quads : nullptr;
    ws.pb.noise_wide = noise_tab ? ws.noise_wide : nullptr;
    ws.pb.noise_rows = noise_tab ? ws.noise_rows : nullptr;
    {
        const int lut_blocks = use_lut ? ceil_div(kOdR * kOdM, kWorkgroup) : 1;
        const int blocks_all = lut_blocks + (noise_tab ? ceil_div(kTableBuild, kWorkgroup) : 0);
        float2* lt = use_lut ? ws.od_lut : nullptr;
        if (noise.format == SOC_FMT_R8_UNORM)
            launch("clouds_od_lut", kWorkgroup, clouds_od_lut<true>, blocks_all, kWorkgroup, 0, s, lt, C2, counter, lut_blocks,
                   dimg(noise), ws.noise_quads, ws.noise_wide, ws.noise_rows);
        else
            launch("clouds_od_lut", kWorkgroup, clouds_od_lut<false>, blocks_all, kWorkgroup, 0, s, lt, C2, counter, lut_blocks,
                   dimg(noise), ws.noise_quads, ws.noise_wide, ws.noise_rows);
    }
    const int vec_store = (target.pitch_bytes % 16 == 0) && (reinterpret_cast<uintptr_t>(target.data) % 16 == 0);
    const bool hoist = sky_bound || tuning_knob("SOC_CLOUDS_CLASSIFY_HOIST", 0);
    if (hoist)
        launch("clouds_classify", kWorkgroup, clouds_classify<true>, dim3(ceil_div(W, 64), ceil_div(H, 16 * kClassifyTiles)),
               kWorkgroup, 0, s, dimg(depth), dimg(target), p, vec_store, counter, list);
    else
        launch("clouds_classify", kWorkgroup, clouds_classify<false>, dim3(ceil_div(W, 64), ceil_div(H, 16 * kClassifyTiles)),
               kWorkgroup, 0, s, dimg(depth), dimg(target), p, vec_store, counter, list);
    // One resident wave set per kernel, grid-stride over the list / pairs: the long per-item work is
    // balanced over all SIMDs instead of running as a second, partially filled round.
    static int res_atmos = 0, res_density = 0, res_sunvis = 0, res_sunvis_n = 0, res_sunvis_r = 0, res_resolve = 0;
    if (!res_atmos) {
        res_atmos = resident_blocks(clouds_atmosphere<false>);
        res_density = resident_blocks(clouds_density<false>);
        res_sunvis = resident_blocks(clouds_sunvis<false, kSunvisLanes, true>, kSunvisLanes);
        res_sunvis_n = resident_blocks(clouds_sunvis<false, kSunvisLanes, false, true>, kSunvisLanes);
        res_sunvis_r = resident_blocks(clouds_sunvis<false, kSunvisLanes, false, true, true>, kSunvisLanes);
        res_resolve = resident_blocks(clouds_resolve<false, true>);
    }
    const long long blocks = ((long long)W * H + 255) / 256;
    if (SOC_CLOUDS_PROFILE >= 4) return check_launch("cloud_rendering");
    // SOC_CLOUDS_GRID_MULT: the sun-visibility and resolve grids as this many times the resident wave set (1: one
    // persistent set; more: workgroups queue behind each other, so the dispatcher can place the main lane's workgroups
    // between them instead of on what a persistent set leaves). The same bits at any grid. Default 2: C3 1678 -> 1699 fps,
    // C2 5313 -> 5526, C4 unchanged; 3 measured C3 1644, C4 1342; 4 / 8: C3 1646 / 1629 (profiles/r05_ab_clouds_grid_mult.txt).
    const int gmul = std::max(1, tuning_knob("SOC_CLOUDS_GRID_MULT", 2));
    auto grid = [&](int res, long long items_blocks) { return (int)std::max(1LL, std::min<long long>(res, items_blocks)); };
    auto grid_m = [&](int res, long long items_blocks) {
        return (int)std::max(1LL, std::min<long long>((long long)res * gmul, items_blocks));
    };
    // Position of the atmosphere kernel in the lane (it feeds only the resolve): before the density march (0), before
    // the sun visibility (1) or after it (2). Default: after it above 1440p (C3 +0.7 %, C4 +5 % at 3840x2160: the
    // atmosphere's long transcendental run then overlaps the frame's TAA instead of its SSAO), first otherwise (C2
    // 1920x1080 -5 % after it); the same bits in every position (profiles/r03_ab_atmos_pos.txt, GPU identity test).
    const int apos_knob = tuning_knob("SOC_CLOUDS_ATMOS_POS", -1);
    const int apos = apos_knob >= 0 ? apos_knob : ((long long)W * H > 2560LL * 1440LL ? 2 : 0);
    // the frame's sky-view table (needs the secondary-ray table; SOC_CLOUDS_SKY_TABLE=0: every pixel evaluated)
    SkyTab st{};
    st.t = nullptr;
    if (lut.t && tuning_knob("SOC_CLOUDS_SKY_TABLE", 1)) {
        const double r0x = (double)(0.0f + p.cam[0]), r0y = (double)(6372e3f + p.cam[1]), r0z = (double)(0.0f + p.cam[2]);
        const double rl = std::sqrt(r0x * r0x + r0y * r0y + r0z * r0z);
        const double ux = r0x / rl, uy = r0y / rl, uz = r0z / rl;
        const double sx = p.sun[0], sy = p.sun[1], sz = p.sun[2], su = sx * ux + sy * uy + sz * uz;
        double hx = sx - su * ux, hy = sy - su * uy, hz = sz - su * uz, hl = std::sqrt(hx * hx + hy * hy + hz * hz);
        if (!(hl > 1e-9)) {   // sun at the zenith: any horizontal axis
            hx = uy; hy = -ux; hz = 0.0;
            hl = std::sqrt(hx * hx + hy * hy);
            if (!(hl > 1e-9)) { hx = 1.0; hy = 0.0; hz = 0.0; hl = 1.0; }
        }
        hx /= hl; hy /= hl; hz /= hl;
        const double bx = uy * hz - uz * hy, by = uz * hx - ux * hz, bz = ux * hy - uy * hx;
        const double q = (double)kRPlanet / rl;
        st.t = ws.sky_tab;
        st.upx = (float)ux; st.upy = (float)uy; st.upz = (float)uz;
        st.shx = (float)hx; st.shy = (float)hy; st.shz = (float)hz;
        st.btx = (float)bx; st.bty = (float)by; st.btz = (float)bz;
        st.eh = q < 1.0 ? (float)std::sqrt(1.0 - q * q) : 0.0f;
        st.dl = 3e-5f;   // margin inside each branch: the fp32 discriminant is ambiguous within ~1e-5 of the grazing elevation
        if (!(st.eh > 4.0f * st.dl)) st.t = nullptr;   // camera at or below the surface: no table
        if (st.t)
            launch("clouds_sky_table", kWorkgroup, clouds_sky_table, ceil_div(kSvEntries, kWorkgroup), kWorkgroup, 0, s, ws.sky_tab, p,
                   st, lut);
    }
    // with the table the resolve looks the atmosphere up itself (SOC_CLOUDS_ATMOS_FOLD=0: the atmosphere kernel from the table)
    const bool fold = st.t && tuning_knob("SOC_CLOUDS_ATMOS_FOLD", 1);
    auto atmos = [&]() {
        if (fold) return;
        if (st.t)
            launch("clouds_atmosphere", kWorkgroup, clouds_atmosphere<true>, grid(res_atmos, blocks), kWorkgroup, 0, s, p, counter,
                   list, ws.atmos, lut, st);
        else
            launch("clouds_atmosphere", kWorkgroup, clouds_atmosphere<false>, grid(res_atmos, blocks), kWorkgroup, 0, s, p, counter,
                   list, ws.atmos, lut, st);
    };
    auto resolve = [&](auto k) {
        launch("clouds_resolve", kWorkgroup, k, grid_m(res_resolve, blocks), kWorkgroup, 0, s, dimg(noise), dimg(target), p, counter,
               list, ws.atmos, ws.pb, st);
    };
    if (apos == 0) atmos();
    const DImg nz = dimg(noise);
    // the resolve's od / vis loads issued in batches of this many steps (1: one step at a time)
    const int rb = tuning_knob("SOC_CLOUDS_RESOLVE_BATCH", 4);
    // the density kernel's od scratch read back in batches of this many steps (1: one dense step at a time)
    const int db = tuning_knob("SOC_CLOUDS_DENSITY_BATCH", 8);
    // the sun-visibility kernel's next pair word loaded one iteration ahead
    const bool sv_pf = tuning_knob("SOC_CLOUDS_SUNVIS_PF", 1) != 0;
    // the sun-visibility kernel's noise table (SOC_CLOUDS_SUNVIS_WIDE): 2 (default) the float-form row table (RowF, 26 KiB
    // per 512-lane workgroup: 8 waves per SIMD, and room on the CU for the main lane's SSAO tile; C3 1728 -> 1799 fps),
    // 1 the float-form quads (52 KiB, 6 waves per SIMD), 0 the byte quads (integer form, 26 KiB). The same bits.
    const int sv_table = tuning_knob("SOC_CLOUDS_SUNVIS_WIDE", 2);
    const bool sv_wide = sv_table != 0;
    // one od scratch per workgroup; SOC_CLOUDS_DENSITY_MULT: the grid as this many times the resident set (as gmul).
    // Default 1: 2 measured C3 1710 -> 1697 fps, C4 1321 -> 1358 (profiles/r05_ab_clouds_density_mult.txt)
    const int dmul = sky_bound ? 2 : std::max(1, tuning_knob("SOC_CLOUDS_DENSITY_MULT", 1));
    const int density_grid = std::min((int)std::max(1LL, std::min<long long>((long long)res_density * dmul, blocks)),
                                      (int)ws.pb.od_blocks);
    // SOC_CLOUDS_DENSITY_ROWS (default 1): the density kernel's noise from the float-form row table (RowF; the same bits)
    const bool drows = tuning_knob("SOC_CLOUDS_DENSITY_ROWS", 1) != 0;
    if (r8) {
        if (drows) launch("clouds_density", kWorkgroup, clouds_density<true, 8, true>, density_grid, kWorkgroup, 0, s, nz, p, counter, list, ws.pb);
        else if (db == 4) launch("clouds_density", kWorkgroup, clouds_density<true, 4>, density_grid, kWorkgroup, 0, s, nz, p, counter, list, ws.pb);
        else if (db == 8) launch("clouds_density", kWorkgroup, clouds_density<true, 8>, density_grid, kWorkgroup, 0, s, nz, p, counter, list, ws.pb);
        else launch("clouds_density", kWorkgroup, clouds_density<true>, density_grid, kWorkgroup, 0, s, nz, p, counter, list, ws.pb);
        if (apos == 1) atmos();
        if (sv_table == 2)
            launch("clouds_sunvis", kSunvisLanes, clouds_sunvis<true, kSunvisLanes, false, true, true>, grid_m(res_sunvis_r, blocks), kSunvisLanes, 0, s, nz, p, list, ws.pb);
        else if (!sv_wide)
            launch("clouds_sunvis", kSunvisLanes, clouds_sunvis<true, kSunvisLanes, false, true>, grid_m(res_sunvis_n, blocks), kSunvisLanes, 0, s, nz, p, list, ws.pb);
        else if (sv_pf)
            launch("clouds_sunvis", kSunvisLanes, clouds_sunvis<true, kSunvisLanes, true, true>, grid_m(res_sunvis, blocks), kSunvisLanes, 0, s, nz, p, list, ws.pb);
        else
            launch("clouds_sunvis", kSunvisLanes, clouds_sunvis<true, kSunvisLanes, true>, grid_m(res_sunvis, blocks), kSunvisLanes, 0, s, nz, p, list, ws.pb);
        if (apos == 2) atmos();
        if (fold && rb == 4) resolve(clouds_resolve<true, true, 4>);
        else if (fold && rb == 8) resolve(clouds_resolve<true, true, 8>);
        else if (fold) resolve(clouds_resolve<true, true>);
        else resolve(clouds_resolve<true, false>);
    } else {
        if (drows) launch("clouds_density", kWorkgroup, clouds_density<false, 8, true>, density_grid, kWorkgroup, 0, s, nz, p, counter, list, ws.pb);
        else if (db == 4) launch("clouds_density", kWorkgroup, clouds_density<false, 4>, density_grid, kWorkgroup, 0, s, nz, p, counter, list, ws.pb);
        else if (db == 8) launch("clouds_density", kWorkgroup, clouds_density<false, 8>, density_grid, kWorkgroup, 0, s, nz, p, counter, list, ws.pb);
        else launch("clouds_density", kWorkgroup, clouds_density<false>, density_grid, kWorkgroup, 0, s, nz, p, counter, list, ws.pb);
        if (apos == 1) atmos();
        if (sv_table == 2)
            launch("clouds_sunvis", kSunvisLanes, clouds_sunvis<false, kSunvisLanes, false, true, true>, grid_m(res_sunvis_r, blocks), kSunvisLanes, 0, s, nz, p, list, ws.pb);
        else if (!sv_wide)
            launch("clouds_sunvis", kSunvisLanes, clouds_sunvis<false, kSunvisLanes, false, true>, grid_m(res_sunvis_n, blocks), kSunvisLanes, 0, s, nz, p, list, ws.pb);
        else if (sv_pf)
            launch("clouds_sunvis", kSunvisLanes, clouds_sunvis<false, kSunvisLanes, true, true>, grid_m(res_sunvis, blocks), kSunvisLanes, 0, s, nz, p, list, ws.pb);
        else
            launch("clouds_sunvis", kSunvisLanes, clouds_sunvis<false, kSunvisLanes, true>, grid_m(res_sunvis, blocks), kSunvisLanes, 0, s, nz, p, list, ws.pb);
        if (apos == 2) atmos();
        if (fold && rb == 4) resolve(clouds_resolve<false, true, 4>);
        else if (fold && rb == 8) resolve(clouds_resolve<false, true, 8>);
        else if (fold) resolve(clouds_resolve<false, true>);
        else resolve(clouds_resolve<false, false>);
    }
    return check_launch("cloud_rendering");
}
