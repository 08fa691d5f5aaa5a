// ssao.hip — SSAOGenerationTask (src/graphics/tasks/ssao_generation.inl:20-68, shader :128-214) and
// SSAOBlurTask (ssao_blur.inl:19-70, shader :91-106) as gfx950 kernels.
//
// SSAO: one lane per half-res output pixel, 32x8 pixel workgroups of 32x2-pixel waves (each tap row of
// a wave spans 64 full-res texels = two 128-B lines, so the 26 depth gathers of neighbouring lanes share
// L1/L2 lines; measured against 16x4 / 8x8 / 4x16 / 64x1 waves: 126 vs 132 / 144 / 158 / 135 us at 4K). Each tap is a bilinear D32 sample under
// the sampling contract, fetched as two 8-byte row pairs. The per-pixel random vector of :184-188 is
// a pure function of (uv, normal-image width): it is either evaluated inline or read from a table
// filled once per resolution by the SAME device function (soc_ssao_prepare_noise), so both give
// identical bits.
#include "soc_internal.hpp"

namespace soc {
namespace {

struct SsaoParams {
    Mat4 inv_proj;
    Mat4 proj;
    Mat4 view;
    float radius, bias, kernel_size_f;
    int ksize;     // loop bound, min(kernel_size, 26)
    int noise_w;   // textureSize(u_normal_image).x
    int swz;       // XCD-aware tile order (tuning knob SOC_SWZ_SSAO, see xcd_order; 0 = row-major)
    float rw, rh;  // recip_rn(target extent) for the pixel-centre uv (div_rn)
    // host-folded constants of the tap loop (make_params): the projection rows x, y, w scaled to texel space
    // (x 256 sub-texel steps on the sparse path), the texel-space centre and clamp bounds, 1 / kernel_size
    float pa[3][4];
    float c0x, c0y, tmx, tmy;
    float inv_ksize;
    float inv_radius;   // 1 / radius (the sparse path requires radius > 0)
};

// Deterministic sin / cos / pow of the noise (quirk Q8). The hash fract(sin(a) * 43758.5453) turns a 1-ulp difference of
// sin into ~3e-3 of the hash, and the device's sinf and the host libm's round differently on ~1 in 2 arguments, so both
// the random-vector table below and the oracle (soc_oracle.c det_sin / det_cos / det_pow) evaluate these functions with
// ONE operation sequence: double precision, IEEE add / mul / fma / div and rint only, rounded to float once (an accurate
// sinf: correctly rounded on every argument the CPU KAT samples). The table is filled once per resolution, so the double
// arithmetic costs nothing per frame. Cody-Waite reduction with fdlibm's three-part pi/2; Taylor kernels on |r| <= pi/4.
__device__ double det_sin_poly(double r) {
    const double r2 = r * r;
    double p = 1.9572941063391263e-20;
    p = __builtin_fma(p, r2, -8.22063524662433e-18);
    p = __builtin_fma(p, r2, 2.8114572543455206e-15);
    p = __builtin_fma(p, r2, -7.647163731819816e-13);
    p = __builtin_fma(p, r2, 1.6059043836821613e-10);
    p = __builtin_fma(p, r2, -2.505210838544172e-08);
    p = __builtin_fma(p, r2, 2.7557319223985893e-06);
    p = __builtin_fma(p, r2, -0.0001984126984126984);
    p = __builtin_fma(p, r2, 0.008333333333333333);
    p = __builtin_fma(p, r2, -0.16666666666666666);
    return __builtin_fma(r * r2, p, r);
}
__device__ double det_cos_poly(double r) {
    const double r2 = r * r;
    double p = 4.110317623312165e-19;
    p = __builtin_fma(p, r2, -1.5619206968586225e-16);
    p = __builtin_fma(p, r2, 4.779477332387385e-14);
    p = __builtin_fma(p, r2, -1.1470745597729725e-11);
    p = __builtin_fma(p, r2, 2.08767569878681e-09);
    p = __builtin_fma(p, r2, -2.755731922398589e-07);
    p = __builtin_fma(p, r2, 2.48015873015873e-05);
    p = __builtin_fma(p, r2, -0.001388888888888889);
    p = __builtin_fma(p, r2, 0.041666666666666664);
    p = __builtin_fma(p, r2, -0.5);
    return __builtin_fma(r2, p, 1.0);
}
// x = q pi/2 + r
__device__ double det_reduce(float x, long long& q) {
    const double d = (double)x;
    const double k = __builtin_rint(d * 6.36619772367581382433e-01);
    double r = __builtin_fma(-k, 1.57079632673412561417e+00, d);
    r = __builtin_fma(-k, 6.07710050630396597660e-11, r);
    r = __builtin_fma(-k, 2.02226624879595063154e-21, r);
    q = (long long)k;
    return r;
}
__device__ float det_sin(float x) {
    long long q;
    const double r = det_reduce(x, q);
    const int k = (int)(q & 3);
    const double v = (k & 1) ? det_cos_poly(r) : det_sin_poly(r);
    return (float)((k & 2) ? -v : v);
}
__device__ float det_cos(float x) {
    long long q;
    const double r = det_reduce(x, q);
    const int k = (int)((q + 1) & 3);   // cos x = sin(x + pi/2)
    const double v = (k & 1) ? det_cos_poly(r) : det_sin_poly(r);
    return (float)((k & 2) ? -v : v);
}
// pow(x, y) for finite x > 0 (uv and 4.2 W): exp(y ln x), ln x = e ln2 + 2 atanh((m - 1) / (m + 1)), m in
// [sqrt(1/2), sqrt(2)); exp by k ln2 + r
__device__ float det_pow(float x, float y) {
    if (!(x > 0.0f) || !__builtin_isfinite(x) || !__builtin_isfinite(y)) return powf(x, y);   // outside the noise's domain
    uint32_t b = __float_as_uint(x);
    int e = (int)((b >> 23) & 255u) - 127;
    if (e == -127) {   // subnormal: scale by 2^32 first (exact)
        b = __float_as_uint(x * 4294967296.0f);
        e = (int)((b >> 23) & 255u) - 127 - 32;
    }
    double m = (double)__uint_as_float((b & 0x007fffffu) | 0x3f800000u);
    if (m > 1.4142135623730951) {
        m *= 0.5;
        e += 1;
    }
    const double s = (m - 1.0) / (m + 1.0), s2 = s * s;
    double p = 0.04;   // 1/25
    p = __builtin_fma(p, s2, 0.043478260869565216);
    p = __builtin_fma(p, s2, 0.047619047619047616);
    p = __builtin_fma(p, s2, 0.05263157894736842);
    p = __builtin_fma(p, s2, 0.058823529411764705);
    p = __builtin_fma(p, s2, 0.06666666666666667);
    p = __builtin_fma(p, s2, 0.07692307692307693);
    p = __builtin_fma(p, s2, 0.09090909090909091);
    p = __builtin_fma(p, s2, 0.1111111111111111);
    p = __builtin_fma(p, s2, 0.14285714285714285);
    p = __builtin_fma(p, s2, 0.2);
    p = __builtin_fma(p, s2, 0.3333333333333333);
    const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
    const double lnm = 2.0 * __builtin_fma(s * s2, p, s);
    const double lnx = __builtin_fma((double)e, ln2_hi, __builtin_fma((double)e, ln2_lo, lnm));
    const double z = (double)y * lnx;
    const double k = __builtin_rint(z * 1.44269504088896338700e+00);
    double r = __builtin_fma(-k, ln2_hi, z);
    r = __builtin_fma(-k, ln2_lo, r);
    double q = 8.896791392450574e-22;
    q = __builtin_fma(q, r, 1.9572941063391263e-20);
    q = __builtin_fma(q, r, 4.110317623312165e-19);
    q = __builtin_fma(q, r, 8.22063524662433e-18);
    q = __builtin_fma(q, r, 1.5619206968586225e-16);
    q = __builtin_fma(q, r, 2.8114572543455206e-15);
    q = __builtin_fma(q, r, 4.779477332387385e-14);
    q = __builtin_fma(q, r, 7.647163731819816e-13);
    q = __builtin_fma(q, r, 1.1470745597729725e-11);
    q = __builtin_fma(q, r, 1.6059043836821613e-10);
    q = __builtin_fma(q, r, 2.08767569878681e-09);
    q = __builtin_fma(q, r, 2.505210838544172e-08);
    q = __builtin_fma(q, r, 2.755731922398589e-07);
    q = __builtin_fma(q, r, 2.7557319223985893e-06);
    q = __builtin_fma(q, r, 2.48015873015873e-05);
    q = __builtin_fma(q, r, 0.0001984126984126984);
    q = __builtin_fma(q, r, 0.001388888888888889);
    q = __builtin_fma(q, r, 0.008333333333333333);
    q = __builtin_fma(q, r, 0.041666666666666664);
    q = __builtin_fma(q, r, 0.16666666666666666);
    q = __builtin_fma(q, r, 0.5);
    q = __builtin_fma(q, r, 1.0);
    q = __builtin_fma(q, r, 1.0);
    if (!(k > -1000.0 && k < 1000.0)) return k > 0.0 ? __builtin_inff() : 0.0f;
    const double sc = __longlong_as_double((long long)((unsigned long long)((long long)k + 1023) << 52));
    return (float)(q * sc);
}

// ssao_generation.inl:139-141 (no FMA contraction: keeps the sin argument as the oracle's; sin: det_sin above)
__device__ __forceinline__ float ssao_rand(float cx, float cy) {
#pragma clang fp contract(off)
    return fractf(det_sin(cx * 12.9898f + cy * 78.233f) * 43758.5453f);
}

// ssao_generation.inl:143-155
__device__ float ssao_noise(float px, float py, float freq) {
#pragma clang fp contract(off)
    float unit = 2560.0f / freq;
    float ix = floorf(px / unit), iy = floorf(py / unit);
    float xx = (px - unit * floorf(px / unit)) / unit, yy = (py - unit * floorf(py / unit)) / unit;
    xx = 0.5f * (1.0f - det_cos(3.14159265359f * xx));
    yy = 0.5f * (1.0f - det_cos(3.14159265359f * yy));
    float a = ssao_rand(ix + 0.0f, iy + 0.0f);
    float b = ssao_rand(ix + 1.0f, iy + 0.0f);
    float c = ssao_rand(ix + 0.0f, iy + 1.0f);
    float d = ssao_rand(ix + 1.0f, iy + 1.0f);
    float x1 = a * (1.0f - xx) + b * xx;
    float x2 = c * (1.0f - xx) + d * xx;
    return x1 * (1.0f - yy) + x2 * yy;
}

// random_vec = normalize(vec3(noise(uv, W*2), noise(pow(uv,1.1), pow(W*4.2, 1.5 + uv.x/10)), 0)), :184-188
__device__ float2 ssao_random_vec(float u, float v, int noise_w) {
#pragma clang fp contract(off)
    float n1 = ssao_noise(u, v, (float)(noise_w * 2));
    float n2 = ssao_noise(det_pow(u, 1.1f), det_pow(v, 1.1f), det_pow((float)noise_w * 4.2f, 1.5f + u / 10.0f));
    float l = sqrtf(n1 * n1 + n2 * n2 + 0.0f * 0.0f);
    return float2{n1 / l, n2 / l};
}

__global__ __launch_bounds__(kWorkgroup) void ssao_noise_kernel(int tw, int th, int noise_w, float2* __restrict__ table) {
    const int x = blockIdx.x * 64 + threadIdx.x, y = blockIdx.y * 4 + threadIdx.y;
    if (x >= tw || y >= th) return;
    table[(size_t)y * tw + x] = ssao_random_vec(centre_uv(x, tw), centre_uv(y, th), noise_w);
}

typedef float f2a4 __attribute__((ext_vector_type(2))) __attribute__((aligned(4)));

// Bilinear D32 depth at (u, v) via the generic contract helper (centre tap).
__device__ __forceinline__ float depth_tap(const DImg& depth, float u, float v) {
    Axis ax = axis_clamp(u, depth.w), ay = axis_clamp(v, depth.h);
    f2a4 r0 = *reinterpret_cast<const f2a4*>(row_ptr<float>(depth, ay.i0) + ax.i0);
    f2a4 r1 = *reinterpret_cast<const f2a4*>(row_ptr<float>(depth, ay.i1) + ax.i0);
    return bilerp1(r0.x, r0.y, r1.x, r1.y, ax.w, ay.w);
}

__device__ __forceinline__ float fast_rcp(float x) { return __builtin_amdgcn_rcpf(x); }

// ssao_generation.inl:74-103 as compile-time constants (literal operands after unrolling)
struct KernelTable { float v[SOC_SSAO_MAX_KERNEL][3]; };
constexpr KernelTable kKernel = {{
    {0.2196607f, 0.9032637f, 0.2254677f},   {0.05916681f, 0.2201506f, 0.1430302f},  {-0.4152246f, 0.1320857f, 0.7036734f},
    {-0.3790807f, 0.1454145f, 0.100605f},   {0.3149606f, -0.1294581f, 0.7044517f},  {-0.1108412f, 0.2162839f, 0.1336278f},
    {0.658012f, -0.4395972f, 0.2919373f},   {0.5377914f, 0.3112189f, 0.426864f},    {-0.2752537f, 0.07625949f, 0.1273409f},
    {-0.1915639f, -0.4973421f, 0.3129629f}, {-0.2634767f, 0.5277923f, 0.1107446f},  {0.8242752f, 0.02434147f, 0.06049098f},
    {0.06262707f, -0.2128643f, 0.03671562f}, {-0.1795662f, -0.3543862f, 0.07924347f}, {0.06039629f, 0.24629f, 0.4501176f},
    {-0.7786345f, -0.3814852f, 0.2391262f}, {0.2792919f, 0.2487278f, 0.05185341f},  {0.1841383f, 0.1696993f, 0.8936281f},
    {-0.3479781f, 0.4725766f, 0.719685f},   {-0.1365018f, -0.2513416f, 0.470937f},  {0.1280388f, -0.563242f, 0.3419276f},
    {-0.4800232f, -0.1899473f, 0.2398808f}, {0.6389147f, 0.1191014f, 0.5271206f},   {0.1932822f, -0.3692099f, 0.6060588f},
    {-0.3465451f, -0.1654651f, 0.6746758f}, {0.2448421f, -0.1610962f, 0.1289366f}}};

// Affine form of one coordinate of the projected sample: c(k) = a0 + a1 kx + a2 ky + a3 kz.
struct Aff { float a0, a1, a2, a3; };
__device__ __forceinline__ float aff(const Aff& a, float kx, float ky, float kz) {
    return __builtin_fmaf(a.a3, kz, __builtin_fmaf(a.a2, ky, __builtin_fmaf(a.a1, kx, a.a0)));
}

// SSAO tap loop. The sample position s(k) = frag + (TBN k) r is affine in the kernel vector k, so the
// projected x', y', w' and the sample depth s.z are evaluated as per-pixel affine forms (3 FMAs each)
// with the texel-space scale of the sampling contract folded in (t = u W - 0.5 = x'/w' * W/2 + (W-1)/2).
// The bilinear depth tap follows the contract's clamp-to-edge / 8-bit sub-texel quantisation with t
// clamped to [0, n-1-1/256] (right-edge taps keep 1/256 of the inner texel). This regroups the
// reference's fp32 roundings; the result stays within the SSAO tolerance of DESIGN.md §5.
// 32x8-pixel workgroups of 32x2-pixel waves (each tap row of a wave spans two 128-B depth lines).
// D32 texel quad (x0, y0) .. (x0 + 1, y0 + 1) through the buffer descriptor: two 8-byte row loads.
struct GlobalQuad {
    __amdgpu_buffer_rsrc_t rsrc;
    int pitch;
    __device__ __forceinline__ void operator()(int x0, int y0, float& t0, float& t1, float& b0, float& b1) const {
        const int off = __mul24(y0, pitch) + x0 * 4;
        const f2a4 r0 = __builtin_bit_cast(f2a4, __builtin_amdgcn_raw_buffer_load_b64(rsrc, off, 0, 0));
        const f2a4 r1 = __builtin_bit_cast(f2a4, __builtin_amdgcn_raw_buffer_load_b64(rsrc, off, pitch, 0));
        t0 = r0.x; t1 = r0.y; b0 = r1.x; b1 = r1.y;
    }
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t depth_rsrc(const DImg& depth) {
    return __builtin_amdgcn_make_buffer_rsrc(depth.data, 0, depth.pitch * depth.h, 0x00020000);
}

// Packed f32 pairs (v_pk_fma_f32 / v_pk_mul_f32: two lanes' worth of f32 work per issue slot on gfx950,
// tools/microbench/pk_rate.hip); element-wise the same IEEE operations as the scalar forms, so the same bits.
typedef float f2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2v pfma(f2v a, f2v b, f2v c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f2v bc2(float x) { return f2v{x, x}; }
__device__ __forceinline__ f2v aff2(const Aff& a, f2v kx, f2v ky, f2v kz) {
    return pfma(bc2(a.a3), kz, pfma(bc2(a.a2), ky, pfma(bc2(a.a1), kx, bc2(a.a0))));
}

// The per-pixel part of SSAOGenerationTask (:176-194) before the tap loop: the view position, the view-space normal,
// the random-vector TBN and the tap loop's per-pixel affine forms. `skip`: a sky pixel (zero normal), written as 255.
struct SsaoPixel {
    bool skip;
    f3 frag;
    Aff ax, ay, aw, az, dzr;
    float A1, B1;
};

// The per-pixel fetches of the setup: the normal sample, the random vector, and (SsaoDepth) the centre depth tap.
struct SsaoFetch {
    f4 nn;
    float2 rv2;
};

template <bool TABLE>
__device__ __forceinline__ SsaoFetch ssao_fetch(int x, int y, float u, float v, const DImg& normal, const DImg& target,
                                                const float2* __restrict__ table, const SsaoParams& p) {
    SsaoFetch f;
    f.nn = sample_h4(normal, u, v);   // normal = mat3(view) * normalize(texture(normal, uv).rgb), :178
    f.rv2 = TABLE ? table[(size_t)y * target.w + x] : ssao_random_vec(u, v, p.noise_w);
    return f;
}

// ssao_fetch in two halves: the loads (issued early, their values not yet used) and the bilinear of the normal
// (sample_h4's taps and arithmetic: the same bits). Needs normal.w >= 2 and the table (the tiled kernel's case).
struct SsaoFetchRaw {
    soc_u4a4 p0, p1;
    Axis ax, ay;
    float2 rv2;
};
__device__ __forceinline__ SsaoFetchRaw ssao_fetch_issue(int x, int y, float u, float v, const DImg& normal,
                                                         const DImg& target, const float2* __restrict__ table) {
    SsaoFetchRaw r;
    r.ax = axis_clamp(u, normal.w);
    r.ay = axis_clamp(v, normal.h);
    r.p0 = *reinterpret_cast<const soc_u4a4*>(row_ptr<uint2>(normal, r.ay.i0) + r.ax.i0);
    r.p1 = *reinterpret_cast<const soc_u4a4*>(row_ptr<uint2>(normal, r.ay.i1) + r.ax.i0);
    r.rv2 = table[(size_t)y * target.w + x];
    return r;
}
__device__ __forceinline__ SsaoFetch ssao_fetch_finish(const SsaoFetchRaw& r) {
    SsaoFetch f;
    f.nn = bilerp4(unpack_h4(uint2{r.p0.x, r.p0.y}), unpack_h4(uint2{r.p0.z, r.p0.w}), unpack_h4(uint2{r.p1.x, r.p1.y}),
                   unpack_h4(uint2{r.p1.z, r.p1.w}), r.ax.w, r.ay.w);
    f.rv2 = r.rv2;
    return f;
}

// ssao_setup given the fetches; depth_at(u, v) returns the centre depth tap (depth_tap, or the same texels from LDS).
template <class DepthAt>
__device__ __forceinline__ SsaoPixel ssao_setup_from(float u, float v, const SsaoFetch& f, const DepthAt& depth_at,
                                                     const SsaoParams& p) {
    // no implicit contraction: every fused multiply-add below is an explicit fma, so the per-pixel arithmetic does not
    // depend on how the surrounding kernel is unrolled or scheduled (ssao_kernel and ssao_lds_kernel give the same bits)
#pragma clang fp contract(off)
    SsaoPixel px;
    const f4 nn = f.nn;
    // A zero normal (the G-buffer's clear value: sky) normalises to NaN; every sample's s.z + bias is then NaN,
    // no comparison adds occlusion, and the result is 1 - 0 / kernel_size = 255 whatever the taps read. Write
    // it without the 26 taps (the same bits as the full evaluation).
    px.skip = nn.x == 0.0f && nn.y == 0.0f && nn.z == 0.0f && p.kernel_size_f != 0.0f;   // (0 / 0 would be NaN -> 0)
    if (px.skip) return px;
    // frag_position = get_view_position_from_depth(in_uv, depth), :177: inv_proj (ndc, depth, 1) as fma chains, then
    // one reciprocal of w for the three divisions (the setup is a quarter of the pass's instructions; within the
    // SSAO tolerance of DESIGN.md §5)
    const float d = depth_at(u, v);
    const float* IP = p.inv_proj.m;
    const float ex = u * 2.0f - 1.0f, ey = v * 2.0f - 1.0f;
    auto ip_row = [&](int r) {
        return __builtin_fmaf(IP[8 + r], d, __builtin_fmaf(IP[4 + r], ey, __builtin_fmaf(IP[r], ex, IP[12 + r])));
    };
    const float iw = fast_rcp(ip_row(3));
    const f3 frag = f3{ip_row(0) * iw, ip_row(1) * iw, ip_row(2) * iw};
    px.frag = frag;
    // normal = mat3(view) * normalize(n): v_rsq instead of sqrt + three divisions (the zero normal left above)
    const float* V = p.view.m;
    const float nk = __builtin_amdgcn_rsqf(__builtin_fmaf(nn.z, nn.z, __builtin_fmaf(nn.y, nn.y, nn.x * nn.x)));
    const f3 nu = f3{nn.x * nk, nn.y * nk, nn.z * nk};
    const f3 n = f3{__builtin_fmaf(V[8], nu.z, __builtin_fmaf(V[4], nu.y, V[0] * nu.x)),
                    __builtin_fmaf(V[9], nu.z, __builtin_fmaf(V[5], nu.y, V[1] * nu.x)),
                    __builtin_fmaf(V[10], nu.z, __builtin_fmaf(V[6], nu.y, V[2] * nu.x))};

    const float2 rv2 = f.rv2;
    // tangent = normalize(rv - n dot(rv, n)) with rv.z = 0 (a zero vector gives NaN, as normalize does)
    const float rn = __builtin_fmaf(rv2.y, n.y, rv2.x * n.x);
    const f3 tu = f3{__builtin_fmaf(-n.x, rn, rv2.x), __builtin_fmaf(-n.y, rn, rv2.y), -n.z * rn};
    const float tk = __builtin_amdgcn_rsqf(__builtin_fmaf(tu.z, tu.z, __builtin_fmaf(tu.y, tu.y, tu.x * tu.x)));
    const f3 t = f3{tu.x * tk, tu.y * tk, tu.z * tk};
    const f3 b = cross3(t, n);

    const float* ip = p.inv_proj.m;
    const float r = p.radius;
    const f3 tr = t * r, br = b * r, nr = n * r;
    // s(k) = frag + tr kx + br ky + nr kz;  x' = P0 sx + P4 sy + P8 sz + P12, etc. (rows pre-scaled on the host:
    // SPARSE_IP's x / y forms carry the sub-texel scale 256 and the +0.5 of the rounding, so a tap's fixed-point
    // coordinate is one fma + clamp)
    auto proj_aff = [&](const float* m) {
        return Aff{__builtin_fmaf(m[2], frag.z, __builtin_fmaf(m[1], frag.y, __builtin_fmaf(m[0], frag.x, m[3]))),
                   __builtin_fmaf(m[2], tr.z, __builtin_fmaf(m[1], tr.y, m[0] * tr.x)),
                   __builtin_fmaf(m[2], br.z, __builtin_fmaf(m[1], br.y, m[0] * br.x)),
                   __builtin_fmaf(m[2], nr.z, __builtin_fmaf(m[1], nr.y, m[0] * nr.x))};
    };
    px.ax = proj_aff(p.pa[0]);
    px.ay = proj_aff(p.pa[1]);
    px.aw = proj_aff(p.pa[2]);
    px.az = Aff{frag.z + p.bias, tr.z, br.z, nr.z};     // s.z + bias
    // SPARSE_IP range test in units of the radius (r > 0, host-checked): with vw = ip11 d + ip15, vz = ip10 d + ip14,
    // D1 = frag.z vw - vz = d A + B and D2 = s.z vw - vz = D1 + (s.z - frag.z) vw; r vw / |D1| = vw / |D1 / r| and
    // sign(D2) = sign(D2 / r), so the tap needs vw, D1 / r (one fma each) and the per-pixel form (s.z - frag.z) / r
    const float ir = p.inv_radius;
    px.A1 = (frag.z * ip[11] - ip[10]) * ir;
    px.B1 = (frag.z * ip[15] - ip[14]) * ir;
    px.dzr = Aff{p.bias * ir, t.z, b.z, n.z};
    return px;
}

template <bool TABLE>
__device__ __forceinline__ SsaoPixel ssao_setup(int x, int y, const DImg& depth, const DImg& normal, const DImg& target,
                                                const float2* __restrict__ table, const SsaoParams& p) {
    const float u = centre_uv_rn(x, target.w, p.rw), v = centre_uv_rn(y, target.h, p.rh);
    return ssao_setup_from(u, v, ssao_fetch<TABLE>(x, y, u, v, normal, target, table, p),
                           [&](float uu, float vv) { return depth_tap(depth, uu, vv); }, p);
}

// One half-res pixel of SSAOGenerationTask (:176-214); `quad` fetches a tap's 2x2 D32 texels.
// PK (sparse inverse projection, full kernel only): the taps in pairs, the affine forms, weights, range test and
// smoothstep of both taps as packed f32 operations; per tap the same operations in the same order (bit-identical).
template <bool SPARSE_IP, bool FULL, class Quad, int UNROLL = SOC_SSAO_MAX_KERNEL, bool PK = false>
__device__ __forceinline__ void ssao_pixel_px(int x, int y, const SsaoPixel& px, const DImg& depth, const DImg& target,
                                              const SsaoParams& p, const Quad& quad);

template <bool TABLE, bool SPARSE_IP, bool FULL, class Quad, int UNROLL = SOC_SSAO_MAX_KERNEL, bool PK = false>
__device__ __forceinline__ void ssao_pixel(int x, int y, const DImg& depth, const DImg& normal, const DImg& target,
                                           const float2* __restrict__ table, const SsaoParams& p, const Quad& quad) {
    ssao_pixel_px<SPARSE_IP, FULL, Quad, UNROLL, PK>(x, y, ssao_setup<TABLE>(x, y, depth, normal, target, table, p), depth,
                                                    target, p, quad);
}

template <bool SPARSE_IP, bool FULL, class Quad, int UNROLL, bool PK>
__device__ __forceinline__ void ssao_pixel_px(int x, int y, const SsaoPixel& px, const DImg& depth, const DImg& target,
                                              const SsaoParams& p, const Quad& quad) {
#pragma clang fp contract(off)
    if (px.skip) {
        row_ptr_w<uint8_t>(target, y)[x] = 255;
        return;
    }
    const f3 frag = px.frag;
    const Aff ax = px.ax, ay = px.ay, aw = px.aw, az = px.az, dzr = px.dzr;
    const float A1 = px.A1, B1 = px.B1;
    const float* ip = p.inv_proj.m;
    const float r = p.radius;
    const int W = depth.w, H = depth.h;
    const float cx0 = p.c0x, cy0 = p.c0y, tmax_x = p.tmx, tmax_y = p.tmy;   // texel (or sub-texel) space
    float occ = 0.0f;
    if constexpr (PK && SPARSE_IP && FULL) {
        static_assert(SOC_SSAO_MAX_KERNEL % 2 == 0, "taps are paired");
        // the same per-tap operations as the scalar loop below, two taps per packed instruction (not unrolled: unrolling
        // 2 or 13 pairs measured 5x slower, profiles/r04_probe_ssao_unroll.txt)
#pragma unroll 1
        for (int i = 0; i < SOC_SSAO_MAX_KERNEL; i += 2) {
            const f2v kx = {kKernel.v[i][0], kKernel.v[i + 1][0]}, ky = {kKernel.v[i][1], kKernel.v[i + 1][1]},
                      kz = {kKernel.v[i][2], kKernel.v[i + 1][2]};
            const f2v ww = aff2(aw, kx, ky, kz);
            const f2v rw = {fast_rcp(ww.x), fast_rcp(ww.y)};
            const f2v X = pfma(aff2(ax, kx, ky, kz), rw, bc2(cx0)), Y = pfma(aff2(ay, kx, ky, kz), rw, bc2(cy0));
            const int fx0 = (int)__builtin_amdgcn_fmed3f(X.x, 0.5f, tmax_x), fx1 = (int)__builtin_amdgcn_fmed3f(X.y, 0.5f, tmax_x);
            const int fy0 = (int)__builtin_amdgcn_fmed3f(Y.x, 0.5f, tmax_y), fy1 = (int)__builtin_amdgcn_fmed3f(Y.y, 0.5f, tmax_y);
            const f2v wx = f2v{(float)(fx0 & 255), (float)(fx1 & 255)} * bc2(1.0f / 256.0f);
            const f2v wy = f2v{(float)(fy0 & 255), (float)(fy1 & 255)} * bc2(1.0f / 256.0f);
            float a0, a1, a2, a3, b0, b1, b2, b3;
            quad(fx0 >> 8, fy0 >> 8, a0, a1, a2, a3);
            quad(fx1 >> 8, fy1 >> 8, b0, b1, b2, b3);
            const float atop = __builtin_fmaf(wx.x, a1 - a0, a0), abot = __builtin_fmaf(wx.x, a3 - a2, a2);
            const float btop = __builtin_fmaf(wx.y, b1 - b0, b0), bbot = __builtin_fmaf(wx.y, b3 - b2, b2);
            const f2v dd = {__builtin_fmaf(wy.x, abot - atop, atop), __builtin_fmaf(wy.y, bbot - btop, btop)};
            const f2v vw = pfma(bc2(ip[11]), dd, bc2(ip[15]));
            const f2v d1 = pfma(dd, bc2(A1), bc2(B1));
            const f2v q = vw * f2v{fast_rcp(fabsf(d1.x)), fast_rcp(fabsf(d1.y))};
            const f2v rc = {__builtin_amdgcn_fmed3f(q.x, 0.0f, 1.0f), __builtin_amdgcn_fmed3f(q.y, 0.0f, 1.0f)};
            const f2v range = rc * rc * pfma(bc2(-2.0f), rc, bc2(3.0f));   // smoothstep(0, 1, x)
            const f2v d2 = pfma(aff2(dzr, kx, ky, kz), vw, d1);
            occ += (d2.x <= 0.0f) ? range.x : 0.0f;
            occ += (d2.y <= 0.0f) ? range.y : 0.0f;
        }
    } else {
#pragma unroll UNROLL
    for (int i = 0; i < SOC_SSAO_MAX_KERNEL; ++i) {
        if (FULL || i < p.ksize) {
            const float kx = kKernel.v[i][0], ky = kKernel.v[i][1], kz = kKernel.v[i][2];
            const float rw = fast_rcp(aff(aw, kx, ky, kz));
            float tx = 0.0f, ty = 0.0f;
            int fx, fy;
            if (SPARSE_IP) {   // 256 t + 0.5 directly, clamped to [0.5, 256 tmax + 0.5]; >= 0, so truncation floors
                fx = (int)__builtin_amdgcn_fmed3f(__builtin_fmaf(aff(ax, kx, ky, kz), rw, cx0), 0.5f, tmax_x);
                fy = (int)__builtin_amdgcn_fmed3f(__builtin_fmaf(aff(ay, kx, ky, kz), rw, cy0), 0.5f, tmax_y);
            } else {
                tx = __builtin_fmaf(aff(ax, kx, ky, kz), rw, cx0);
                ty = __builtin_fmaf(aff(ay, kx, ky, kz), rw, cy0);
                tx = __builtin_amdgcn_fmed3f(tx, 0.0f, tmax_x);   // clamp: one v_med3, no NaN quieting
                ty = __builtin_amdgcn_fmed3f(ty, 0.0f, tmax_y);
                // t >= 0, so truncation is the floor
                fx = (int)__builtin_fmaf(tx, 256.0f, 0.5f);
                fy = (int)__builtin_fmaf(ty, 256.0f, 0.5f);
            }
            const float wx = (float)(fx & 255) * (1.0f / 256.0f), wy = (float)(fy & 255) * (1.0f / 256.0f);
            float t0, t1, b0, b1;
            quad(fx >> 8, fy >> 8, t0, t1, b0, b1);
            const float top = __builtin_fmaf(wx, t1 - t0, t0);
            const float bot = __builtin_fmaf(wx, b1 - b0, b0);
            const float dd = __builtin_fmaf(wy, bot - top, top);
            float vz = 0.0f, vw;   // get_view_position_from_depth(offset.xy, depth).z
            if (SPARSE_IP) {
                vw = __builtin_fmaf(ip[11], dd, ip[15]);
            } else {
                const float ex = (tx + 0.5f) * (2.0f / (float)W) - 1.0f, ey = (ty + 0.5f) * (2.0f / (float)H) - 1.0f;
                vz = ip[2] * ex + ip[6] * ey + ip[10] * dd + ip[14];
                vw = ip[3] * ex + ip[7] * ey + ip[11] * dd + ip[15];
            }
            if (SPARSE_IP) {
                // vw > 0 for every stored depth (the host selects this path only then), so with sd = vz / vw:
                // r / |frag.z - sd| = r vw / |frag.z vw - vz| and sd >= s.z  <=>  s.z vw - vz <= 0 (one
                // reciprocal per tap instead of two), both scaled by 1 / r (above)
                const float d1 = __builtin_fmaf(dd, A1, B1);
                const float rc = __builtin_amdgcn_fmed3f(vw * fast_rcp(fabsf(d1)), 0.0f, 1.0f);
                const float range = rc * rc * __builtin_fmaf(-2.0f, rc, 3.0f);   // smoothstep(0, 1, x)
                occ += (__builtin_fmaf(aff(dzr, kx, ky, kz), vw, d1) <= 0.0f) ? range : 0.0f;
            } else {
                const float sd = vz * fast_rcp(vw);
                const float rc = __builtin_amdgcn_fmed3f(r * fast_rcp(fabsf(frag.z - sd)), 0.0f, 1.0f);   // >= 0
                const float range = rc * rc * __builtin_fmaf(-2.0f, rc, 3.0f);   // smoothstep(0, 1, x)
                occ += (sd >= aff(az, kx, ky, kz)) ? range : 0.0f;
            }
        }
    }
    }
    occ = 1.0f - occ * p.inv_ksize;
    row_ptr_w<uint8_t>(target, y)[x] = (uint8_t)to_unorm8(occ);
}

template <bool TABLE, bool SPARSE_IP, bool FULL>
__global__ __launch_bounds__(kWorkgroup) void ssao_kernel(DImg depth, DImg normal, DImg target, const float2* __restrict__ table,
                                                   SsaoParams p) {
    int bx, by;
    xcd_order(p.swz, bx, by);
    const int tid = threadIdx.x;
    const int x = bx * 32 + (tid & 31), y = by * 8 + (tid >> 5);
    if (x >= target.w || y >= target.h) return;
    ssao_pixel<TABLE, SPARSE_IP, FULL>(x, y, depth, normal, target, table, p, GlobalQuad{depth_rsrc(depth), depth.pitch});
}

// LDS-tiled taps. A workgroup of TXP x TYP half-res pixels (waves of 32 x 2) first stages the full-res depth tile
// its pixels cover plus a HALO-texel border in LDS (16-B loads, one pass); every tap whose 2x2 texels lie inside the
// tile reads them from LDS, the others (near geometry: the screen-space radius exceeds the halo) from the D32 image
// as before, exec-masked to those lanes. The same texels, so the same bits as ssao_kernel.
template <int TXP, int TYP, int HALO>
struct SsaoTile {
    static constexpr int TW = 2 * TXP + 2 * HALO, TH = 2 * TYP + 2 * HALO, THREADS = TXP * TYP;
};

// Profiling builds only (SOC_SSAO_PROBE, wrong results): 1 = every tap from the LDS tile (out-of-tile lanes read texel 0),
// 2 = no texel reads at all (constant texels). The library is built with 0.
#ifndef SOC_SSAO_PROBE
#define SOC_SSAO_PROBE 0
#endif
template <int TXP, int TYP, int HALO>
struct LdsQuad {
    const float* tile;
    int gx0, gy0;
    GlobalQuad g;
    __device__ __forceinline__ void operator()(int x0, int y0, float& t0, float& t1, float& b0, float& b1) const {
        constexpr int TW = SsaoTile<TXP, TYP, HALO>::TW, TH = SsaoTile<TXP, TYP, HALO>::TH;
        if (SOC_SSAO_PROBE == 2) {
            t0 = t1 = b0 = b1 = __int_as_float(0x3f7f0000 | (x0 & 255) | (y0 & 255) << 8);
            return;
        }
        const int lx = x0 - gx0, ly = y0 - gy0;
        const bool in = SOC_SSAO_PROBE == 1 || ((unsigned)lx < (unsigned)(TW - 1) && (unsigned)ly < (unsigned)(TH - 1));
        // ly * TW + lx as one full-rate v_mad_u32_u24 (the compiler otherwise selects v_mad_u64_u32 for it)
        uint32_t i;
        asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(i) : "v"(ly), "s"((uint32_t)TW), "v"(lx));
        if (SOC_SSAO_PROBE == 1) i = i % (uint32_t)(TW * (TH - 1) - 1);
        i = in ? i : 0u;
        t0 = tile[i];
        t1 = tile[i + 1];
        b0 = tile[i + TW];
        b1 = tile[i + TW + 1];
        if (!in) g(x0, y0, t0, t1, b0, b1);
    }
};

// Stage the workgroup's depth tile: rows clamped into the image; columns left of the image give a negative
// (out-of-range) offset, which the buffer load returns as 0. No tap reads a texel outside the image (taps clamp to
// [0, n - 2]). Every lane issues all its 16-B loads before its first LDS store (one memory latency, not one per load).
template <int TXP, int TYP, int HALO>
__device__ __forceinline__ void ssao_stage_tile(float4* tile4, __amdgpu_buffer_rsrc_t rsrc, const DImg& depth, int gx0, int gy0,
                                                int tid) {
    using T = SsaoTile<TXP, TYP, HALO>;
    constexpr int Q = T::TW / 4, N = Q * T::TH, K = (N + T::THREADS - 1) / T::THREADS;
    float4 v[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int i = tid + k * T::THREADS;
        if (N % T::THREADS == 0 || i < N) {
            const int r = i / Q, c = i - r * Q;
            const int gy = min(max(gy0 + r, 0), depth.h - 1);
            const int off = __mul24(gy, depth.pitch) + (gx0 + 4 * c) * 4;
            const auto w = __builtin_amdgcn_raw_buffer_load_b128(rsrc, off, 0, 0);
            v[k] = make_float4(__uint_as_float(w[0]), __uint_as_float(w[1]), __uint_as_float(w[2]), __uint_as_float(w[3]));
        }
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int i = tid + k * T::THREADS;
        if (N % T::THREADS == 0 || i < N) tile4[i] = v[k];
    }
}

// The default tile: 64 x 16 half-res pixels (1024 lanes), a 32-texel halo (tile sweep: profiles/r03_ssao_tile_sweep.txt);
// kSsaoTileLanes is the launch bound its launcher checks.
#ifndef SOC_SSAO_TILE_TX
#define SOC_SSAO_TILE_TX 64   // A/B builds: the tile's half-res extent and halo
#endif
#ifndef SOC_SSAO_TILE_TY
#define SOC_SSAO_TILE_TY 16
#endif
#ifndef SOC_SSAO_HALO
#define SOC_SSAO_HALO 32
#endif
constexpr int kSsaoTX = SOC_SSAO_TILE_TX, kSsaoTY = SOC_SSAO_TILE_TY, kSsaoHalo = SOC_SSAO_HALO, kSsaoTileLanes = kSsaoTX * kSsaoTY;

// EARLY (tuning knob SOC_SSAO_EARLY): 2 (default) stages the tile with every load of a lane issued before its first LDS
// store (ssao_stage_tile; the round-4 loop waited on each load in turn); 1 in addition fetches the pixel's normal texels
// and random vector before the workgroup barrier (their latency overlaps the staging) and reads its centre depth tap
// from the staged tile; 0 = the round-4 kernel. The same texels and arithmetic, so the same bits (GPU identity test).
// Measured alone (C3 / C4): 98.8 / 77.2 us (0), 97.8 / 74.5 (1), 97.0 / 73.5 (2); the frame unchanged
// (profiles/r05_probe_ssao_early.txt).
template <bool TABLE, bool SPARSE_IP, bool FULL, int TXP, int TYP, int HALO, int UNROLL, bool PK = false, int EARLY = 0>
__global__ __attribute__((amdgpu_flat_work_group_size(TXP * TYP, TXP * TYP)))
__attribute__((amdgpu_waves_per_eu(TXP * TYP >= 1024 ? 8 : TXP * TYP >= 512 ? 4 : 2)))
void ssao_lds_kernel(DImg depth, DImg normal, DImg target, const float2* __restrict__ table, SsaoParams p) {
    using T = SsaoTile<TXP, TYP, HALO>;
    __shared__ float4 tile4[T::TW * T::TH / 4];
    int bx, by;
    xcd_order(p.swz, bx, by);
    const int tid = threadIdx.x;
    const int gx0 = bx * 2 * TXP - HALO, gy0 = by * 2 * TYP - HALO;
    const __amdgpu_buffer_rsrc_t rsrc = depth_rsrc(depth);
    if constexpr (EARLY == 1) {
        const int w = tid >> 6, lane = tid & 63;
        const int x = bx * TXP + (w % (TXP / 32)) * 32 + (lane & 31), y = by * TYP + (w / (TXP / 32)) * 2 + (lane >> 5);
        const bool inside = x < target.w && y < target.h;
        const float u = centre_uv_rn(x, target.w, p.rw), v = centre_uv_rn(y, target.h, p.rh);
        static_assert(TABLE, "the early fetch reads the random-vector table");
        SsaoFetchRaw fr{};
        if (inside) fr = ssao_fetch_issue(x, y, u, v, normal, target, table);
        ssao_stage_tile<TXP, TYP, HALO>(tile4, rsrc, depth, gx0, gy0, tid);
        __syncthreads();
        if (!inside) return;
        const float* tile = reinterpret_cast<const float*>(tile4);
        const SsaoPixel px = ssao_setup_from(u, v, ssao_fetch_finish(fr), [&](float uu, float vv) {
            const Axis ax = axis_clamp(uu, depth.w), ay = axis_clamp(vv, depth.h);
            const int i = (ay.i0 - gy0) * T::TW + (ax.i0 - gx0);
            return bilerp1(tile[i], tile[i + 1], tile[i + T::TW], tile[i + T::TW + 1], ax.w, ay.w);
        }, p);
        const LdsQuad<TXP, TYP, HALO> quad{tile, gx0, gy0, GlobalQuad{rsrc, depth.pitch}};
        ssao_pixel_px<SPARSE_IP, FULL, LdsQuad<TXP, TYP, HALO>, UNROLL, PK>(x, y, px, depth, target, p, quad);
        return;
    }
    // stage the tile: rows clamped into the image; columns left of the image give a negative (out-of-range) offset,
    // which the buffer load returns as 0. No tap reads a texel outside the image (taps clamp to [0, n - 2]).
    if constexpr (EARLY == 2) {
        ssao_stage_tile<TXP, TYP, HALO>(tile4, rsrc, depth, gx0, gy0, tid);
    } else {
        constexpr int Q = T::TW / 4;
        for (int i = tid; i < Q * T::TH; i += T::THREADS) {
            const int r = i / Q, c = i - r * Q;
            const int gy = min(max(gy0 + r, 0), depth.h - 1);
            const int off = __mul24(gy, depth.pitch) + (gx0 + 4 * c) * 4;
            const auto v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, off, 0, 0);
            tile4[i] = make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]), __uint_as_float(v[3]));
        }
    }
    __syncthreads();
    const int w = tid >> 6, lane = tid & 63;
    const int x = bx * TXP + (w % (TXP / 32)) * 32 + (lane & 31), y = by * TYP + (w / (TXP / 32)) * 2 + (lane >> 5);
    if (x >= target.w || y >= target.h) return;
    const LdsQuad<TXP, TYP, HALO> quad{reinterpret_cast<const float*>(tile4), gx0, gy0, GlobalQuad{rsrc, depth.pitch}};
    ssao_pixel<TABLE, SPARSE_IP, FULL, LdsQuad<TXP, TYP, HALO>, UNROLL, PK>(x, y, depth, normal, target, table, p, quad);
}

// ---- the software-pipelined tap loop (round 6) --------------------------------------------------------------------
// ssao_lds_kernel's loop (not unrolled: unrolling let the compiler hoist every pair's loads, r04_probe_ssao_unroll)
// waited three times per tap pair: a scalar load of the pair's kernel vectors from the constant table (s_waitcnt
// lgkmcnt(0), which also drains the LDS queue), the LDS texel reads it had just issued, and, in a wave with any
// out-of-tile lane, that lane's global texel loads. Here the 13 pairs are unrolled by template recursion (kernel vectors
// as literal operands: no table load), each in two stages: ISSUE computes the pair's fixed-point tap coordinates and
// issues its texel reads (LDS tile, or the image for an out-of-tile lane), CONSUME filters them and adds the occlusion;
// pair p + 1 is issued before pair p is consumed, so each pair's LDS latency (and an out-of-tile lane's global latency)
// overlaps the previous pair's arithmetic. Per tap the same operations in the same order as the PK loop: the same bits.
struct TapPair {
    float v[8];   // tap 0: t0 t1 b0 b1, tap 1: t0 t1 b0 b1
    int f[4];     // fixed-point coordinates fx0, fx1, fy0, fy1 (their low bytes: the sub-texel weights)
    float w0, w1; // PERSP: the taps' w' (= -s.z), for the range test's sample depth
};

template <int I, bool PERSP, int TXP, int TYP, int HALO>
__device__ __forceinline__ TapPair ssao_issue_pair(const SsaoPixel& px, const SsaoParams& p, const LdsQuad<TXP, TYP, HALO>& quad) {
#pragma clang fp contract(off)
    const f2v kx = {kKernel.v[I][0], kKernel.v[I + 1][0]}, ky = {kKernel.v[I][1], kKernel.v[I + 1][1]},
              kz = {kKernel.v[I][2], kKernel.v[I + 1][2]};
    // the per-pixel affine forms as scalar fmas (their packed form needs every per-pixel coefficient duplicated into a
    // register pair: 18 more VGPRs, and this kernel's 8 waves per SIMD have 64; element-wise the same operations)
    const f2v ww = {aff(px.aw, kx.x, ky.x, kz.x), aff(px.aw, kx.y, ky.y, kz.y)};
    const f2v rw = {fast_rcp(ww.x), fast_rcp(ww.y)};
    const f2v X = {__builtin_fmaf(aff(px.ax, kx.x, ky.x, kz.x), rw.x, p.c0x), __builtin_fmaf(aff(px.ax, kx.y, ky.y, kz.y), rw.y, p.c0x)};
    const f2v Y = {__builtin_fmaf(aff(px.ay, kx.x, ky.x, kz.x), rw.x, p.c0y), __builtin_fmaf(aff(px.ay, kx.y, ky.y, kz.y), rw.y, p.c0y)};
    const int fx0 = (int)__builtin_amdgcn_fmed3f(X.x, 0.5f, p.tmx), fx1 = (int)__builtin_amdgcn_fmed3f(X.y, 0.5f, p.tmx);
    const int fy0 = (int)__builtin_amdgcn_fmed3f(Y.x, 0.5f, p.tmy), fy1 = (int)__builtin_amdgcn_fmed3f(Y.y, 0.5f, p.tmy);
    TapPair t;
    t.f[0] = fx0;
    t.f[1] = fx1;
    t.f[2] = fy0;
    t.f[3] = fy1;
    if (PERSP) {
        t.w0 = ww.x;
        t.w1 = ww.y;
    }
    quad(fx0 >> 8, fy0 >> 8, t.v[0], t.v[1], t.v[2], t.v[3]);
    quad(fx1 >> 8, fy1 >> 8, t.v[4], t.v[5], t.v[6], t.v[7]);
    return t;
}

template <int I, bool PERSP>
__device__ __forceinline__ void ssao_consume_pair(const TapPair& t, const SsaoPixel& px, const SsaoParams& p, float& occ) {
#pragma clang fp contract(off)
    const f2v kx = {kKernel.v[I][0], kKernel.v[I + 1][0]}, ky = {kKernel.v[I][1], kKernel.v[I + 1][1]},
              kz = {kKernel.v[I][2], kKernel.v[I + 1][2]};
    const float* ip = p.inv_proj.m;
    const f2v wx = f2v{(float)(t.f[0] & 255), (float)(t.f[1] & 255)} * bc2(1.0f / 256.0f);
    const f2v wy = f2v{(float)(t.f[2] & 255), (float)(t.f[3] & 255)} * bc2(1.0f / 256.0f);
    const float atop = __builtin_fmaf(wx.x, t.v[1] - t.v[0], t.v[0]), abot = __builtin_fmaf(wx.x, t.v[3] - t.v[2], t.v[2]);
    const float btop = __builtin_fmaf(wx.y, t.v[5] - t.v[4], t.v[4]), bbot = __builtin_fmaf(wx.y, t.v[7] - t.v[6], t.v[6]);
    const f2v dd = {__builtin_fmaf(wy.x, abot - atop, atop), __builtin_fmaf(wy.y, bbot - btop, btop)};
    const f2v vw = pfma(bc2(ip[11]), dd, bc2(ip[15]));
    const f2v d1 = {__builtin_fmaf(dd.x, px.A1, px.B1), __builtin_fmaf(dd.y, px.A1, px.B1)};
    // two scalar multiplies whose clamp is an output modifier (a packed multiply then two clamping v_max_f32 issue ~2.5x
    // the time: tools/microbench/valu_ops.hip); the same products
    const f2v rc = {__builtin_amdgcn_fmed3f(vw.x * fast_rcp(fabsf(d1.x)), 0.0f, 1.0f),
                    __builtin_amdgcn_fmed3f(vw.y * fast_rcp(fabsf(d1.y)), 0.0f, 1.0f)};
    const f2v range = rc * rc * pfma(bc2(-2.0f), rc, bc2(3.0f));   // smoothstep(0, 1, x)
    // (s.z + bias - frag.z) / r: the affine form, or PERSP (the projection's w row is (0, 0, -1, 0): w' = -s.z) one fma
    // from the tap's w' (within the SSAO tolerance: w' carries its own rounding)
    const float z0 = PERSP ? __builtin_fmaf(t.w0, -p.inv_radius, px.dzr.a0) : aff(px.dzr, kx.x, ky.x, kz.x);
    const float z1 = PERSP ? __builtin_fmaf(t.w1, -p.inv_radius, px.dzr.a0) : aff(px.dzr, kx.y, ky.y, kz.y);
    const f2v d2 = {__builtin_fmaf(z0, vw.x, d1.x), __builtin_fmaf(z1, vw.y, d1.y)};
    occ += (d2.x <= 0.0f) ? range.x : 0.0f;
    occ += (d2.y <= 0.0f) ? range.y : 0.0f;
}

// Pair PR consumed after pair PR + 1 is issued.
template <int PR, bool PERSP, int TXP, int TYP, int HALO>
__device__ __forceinline__ void ssao_pipe_step(const TapPair& cur, const SsaoPixel& px, const SsaoParams& p,
                                               const LdsQuad<TXP, TYP, HALO>& quad, float& occ) {
    constexpr int kPairs = SOC_SSAO_MAX_KERNEL / 2;
    if constexpr (PR + 1 < kPairs) {
        const TapPair nxt = ssao_issue_pair<2 * (PR + 1), PERSP>(px, p, quad);
        ssao_consume_pair<2 * PR, PERSP>(cur, px, p, occ);
        // keeps the stages in this order: the occlusion sum of pair PR is complete here and no later pair's texel read
        // moves above this point (without it the compiler sank every consume stage below the last issue stage: all 26
        // taps' texels live at once, 200 VGPRs spilled)
        asm volatile("" : "+v"(occ)::"memory");
        ssao_pipe_step<PR + 1, PERSP>(nxt, px, p, quad, occ);
    } else {
        ssao_consume_pair<2 * PR, PERSP>(cur, px, p, occ);
    }
}

// The LDS-tiled kernel (ssao_lds_kernel's tile, staging and per-pixel setup, EARLY = 2) with the pipelined tap loop;
// the sparse inverse projection and the full 26-tap kernel (the host selects it only then).
template <int TXP, int TYP, int HALO, bool PERSP>
__global__ __attribute__((amdgpu_flat_work_group_size(TXP * TYP, TXP * TYP)))
__attribute__((amdgpu_waves_per_eu(TXP * TYP >= 1024 ? 8 : TXP * TYP >= 512 ? 4 : 2)))
void ssao_pipe_kernel(DImg depth, DImg normal, DImg target, const float2* __restrict__ table, SsaoParams p) {
    static_assert(SOC_SSAO_MAX_KERNEL % 2 == 0, "taps are paired");
    using T = SsaoTile<TXP, TYP, HALO>;
    __shared__ float4 tile4[T::TW * T::TH / 4];
    int bx, by;
    xcd_order(p.swz, bx, by);
    const int tid = threadIdx.x;
    const int gx0 = bx * 2 * TXP - HALO, gy0 = by * 2 * TYP - HALO;
    const __amdgpu_buffer_rsrc_t rsrc = depth_rsrc(depth);
    ssao_stage_tile<TXP, TYP, HALO>(tile4, rsrc, depth, gx0, gy0, tid);
    __syncthreads();
    const int w = tid >> 6, lane = tid & 63;
    const int x = bx * TXP + (w % (TXP / 32)) * 32 + (lane & 31), y = by * TYP + (w / (TXP / 32)) * 2 + (lane >> 5);
    if (x >= target.w || y >= target.h) return;
    const SsaoPixel px = ssao_setup<true>(x, y, depth, normal, target, table, p);
    if (px.skip) {
        row_ptr_w<uint8_t>(target, y)[x] = 255;
        return;
    }
    const LdsQuad<TXP, TYP, HALO> quad{reinterpret_cast<const float*>(tile4), gx0, gy0, GlobalQuad{rsrc, depth.pitch}};
    float occ = 0.0f;
    SsaoPixel pxp = px;
    if (PERSP) pxp.dzr.a0 = (p.bias - px.frag.z) * p.inv_radius;
    ssao_pipe_step<0, PERSP>(ssao_issue_pair<0, PERSP>(pxp, p, quad), pxp, p, quad, occ);
    occ = 1.0f - occ * p.inv_ksize;
    row_ptr_w<uint8_t>(target, y)[x] = (uint8_t)to_unorm8(occ);
}

// ssao_blur.inl:91-106: 4x4 box at offsets -2..+1 (x outer, y inner), all taps on texel centres.
__global__ __launch_bounds__(kWorkgroup) void ssao_blur_kernel(DImg src, DImg dst) {
#pragma clang fp contract(off)
    const int x = blockIdx.x * 64 + threadIdx.x, y = blockIdx.y * 4 + threadIdx.y;
    if (x >= dst.w || y >= dst.h) return;
    float result = 0.0f;
#pragma unroll
    for (int dx = -2; dx < 2; ++dx)
#pragma unroll
        for (int dy = -2; dy < 2; ++dy) {
            int sx = min(max(x + dx, 0), src.w - 1), sy = min(max(y + dy, 0), src.h - 1);
            result += fetch_r8(src, sx, sy);
        }
    row_ptr_w<uint8_t>(dst, y)[x] = (uint8_t)to_unorm8(result / 16.0f);
}

// Generic blur for a target whose extent differs from the source (taps are real bilinear samples).
__global__ __launch_bounds__(kWorkgroup) void ssao_blur_generic(DImg src, DImg dst, float tx, float ty) {
#pragma clang fp contract(off)
    const int x = blockIdx.x * 64 + threadIdx.x, y = blockIdx.y * 4 + threadIdx.y;
    if (x >= dst.w || y >= dst.h) return;
    const float u = centre_uv(x, dst.w), v = centre_uv(y, dst.h);
    float result = 0.0f;
    for (int dx = -2; dx < 2; ++dx)
        for (int dy = -2; dy < 2; ++dy) result += sample_r8(src, u + (float)dx * tx, v + (float)dy * ty);
    row_ptr_w<uint8_t>(dst, y)[x] = (uint8_t)to_unorm8(result / 16.0f);
}

SsaoParams make_params(const soc_globals* g, const soc_img& normal) {
    SsaoParams p;
    p.inv_proj = mat4(g->camera_inverse_projection_matrix);
    p.proj = mat4(g->camera_projection_matrix);
    p.view = mat4(g->camera_view_matrix);
    p.radius = g->ssao_radius;
    p.bias = g->ssao_bias;
    p.kernel_size_f = (float)g->ssao_kernel_size;
    p.ksize = g->ssao_kernel_size < SOC_SSAO_MAX_KERNEL ? g->ssao_kernel_size : SOC_SSAO_MAX_KERNEL;
    p.noise_w = normal.width;
    p.swz = tuning_knob("SOC_SWZ_SSAO", -16);   // XCD vertical bands: HBM traffic 3.3x -> 1.25x algorithmic
    p.inv_ksize = 1.0f / p.kernel_size_f;
    p.inv_radius = 1.0f / p.radius;
    return p;
}

// The tap loop's uniform constants for a depth image of W x H (sip: the sparse-inverse-projection path, whose x / y
// forms count 1/256-texel steps with the rounding's +0.5 folded into the centre).
void fold_tap_constants(SsaoParams& p, int W, int H, bool sip) {
    const float fxs = sip ? 256.0f : 1.0f;
    const float scale[3] = {0.5f * (float)W * fxs, 0.5f * (float)H * fxs, 1.0f};
    const int rows[3] = {0, 1, 3};
    for (int k = 0; k < 3; ++k)
        for (int j = 0; j < 4; ++j) p.pa[k][j] = p.proj.m[4 * j + rows[k]] * scale[k];
    const float cx0 = 0.5f * (float)(W - 1), cy0 = 0.5f * (float)(H - 1);
    const float tmax_x = (float)(W - 1) - 1.0f / 256.0f, tmax_y = (float)(H - 1) - 1.0f / 256.0f;
    p.c0x = sip ? cx0 * 256.0f + 0.5f : cx0;
    p.c0y = sip ? cy0 * 256.0f + 0.5f : cy0;
    p.tmx = sip ? tmax_x * 256.0f + 0.5f : tmax_x;
    p.tmy = sip ? tmax_y * 256.0f + 0.5f : tmax_y;
}

}  // namespace
}  // namespace soc

using namespace soc;

extern "C" int soc_ssao_prepare_noise(soc_img normal, soc_img target, float* noise_table, soc_stream stream) {
    if (!noise_table) return set_error(SOC_E_INVALID_ARG, "soc_ssao_prepare_noise: null table");
    if (normal.width <= 0 || target.width <= 0 || target.height <= 0)
        return set_error(SOC_E_INVALID_ARG, "soc_ssao_prepare_noise: bad extents");
    dim3 blk(64, 4), grd(ceil_div(target.width, 64), ceil_div(target.height, 4));
    launch("ssao_noise_kernel", kWorkgroup, ssao_noise_kernel, grd, blk, 0, hs(stream), target.width, target.height, normal.width,
                                                   reinterpret_cast<float2*>(noise_table));
    return check_launch("ssao_prepare_noise");
}

extern "C" int soc_ssao_generation(const soc_globals* g, soc_img depth, soc_img normal, soc_img target,
                                   const float* noise_table, soc_stream stream) {
    if (!g) return set_error(SOC_E_INVALID_ARG, "soc_ssao_generation: null globals");
    int rc = check_img(depth, SOC_FMT_D32F, "soc_ssao_generation", "depth");
    if (!rc) rc = check_img(normal, SOC_FMT_RGBA16F, "soc_ssao_generation", "normal");
    if (!rc) rc = check_img(target, SOC_FMT_R8_UNORM, "soc_ssao_generation", "target");
    if (rc) return rc;
    if (depth.width < 2 || depth.height < 2)
        return set_error(SOC_E_SHAPE, "soc_ssao_generation: depth must be at least 2x2");
    if ((long long)depth.pitch_bytes * depth.height >= (1ll << 31) || depth.pitch_bytes >= (1 << 23))
        return set_error(SOC_E_SHAPE, "soc_ssao_generation: depth image exceeds the 2 GiB buffer-offset range");
    SsaoParams p = make_params(g, normal);
    p.rw = recip_rn(target.width);
    p.rh = recip_rn(target.height);
    const float* IP = g->camera_inverse_projection_matrix;
    // sparse inverse projection (the reference's perspective) whose w row stays positive over depths [-1, 1]
    const bool sip = IP[2] == 0.0f && IP[3] == 0.0f && IP[6] == 0.0f && IP[7] == 0.0f && IP[15] - IP[11] > 0.0f &&
                     IP[15] + IP[11] > 0.0f && p.radius > 0.0f && std::isfinite(p.inv_radius);
    fold_tap_constants(p, depth.width, depth.height, sip);
    const dim3 blk(256), grd(ceil_div(target.width, 32), ceil_div(target.height, 8));
    const float2* tb = reinterpret_cast<const float2*>(noise_table);
    hipStream_t st = hs(stream);
    DImg dd = dimg(depth), dn = dimg(normal), dt = dimg(target);
#define SOC_SSAO_LAUNCH(T, B, F) launch("ssao_kernel", kWorkgroup, ssao_kernel<T, B, F>, grd, blk, 0, st, dd, dn, dt, tb, p)
    const bool full = p.ksize == SOC_SSAO_MAX_KERNEL;
    // default: the LDS-tiled kernel (64 x 16 pixels, 32-texel halo) in the contiguous-eighths XCD order; SOC_SSAO_TILE=0
    // selects the plain gather kernel (the same bits: tests/test_gpu_parity.py)
    const bool tiled = tuning_knob("SOC_SSAO_TILE", 1) != 0;
    if (noise_table && sip && full && tiled) {
        SsaoParams pt = p;
        pt.swz = 1;
        const dim3 g(ceil_div(target.width, kSsaoTX), ceil_div(target.height, kSsaoTY));
        const int early = tuning_knob("SOC_SSAO_EARLY", 2);
        // SOC_SSAO_PIPE (default 1): the software-pipelined tap loop (ssao_pipe_kernel; the same bits)
        // the projection's w row (0, 0, -1, 0) (the reference's perspective; jitter moves only the x / y rows): the
        // range test's sample depth from the tap's w' (PERSP); SOC_SSAO_PIPE=2 forces the affine form
        const float* P = pt.proj.m;
        const int pipe = tuning_knob("SOC_SSAO_PIPE", 1);
        const bool persp = pipe == 1 && P[3] == 0.0f && P[7] == 0.0f && P[11] == -1.0f && P[15] == 0.0f;
        if (pipe && persp)
            launch("ssao_pipe_kernel", kSsaoTileLanes, ssao_pipe_kernel<kSsaoTX, kSsaoTY, kSsaoHalo, true>, g, kSsaoTileLanes, 0, st,
                   dd, dn, dt, tb, pt);
        else if (pipe)
            launch("ssao_pipe_kernel", kSsaoTileLanes, ssao_pipe_kernel<kSsaoTX, kSsaoTY, kSsaoHalo, false>, g, kSsaoTileLanes, 0, st,
                   dd, dn, dt, tb, pt);
        else if (early == 1)
            launch("ssao_lds_kernel", kSsaoTileLanes,
                   ssao_lds_kernel<true, true, true, kSsaoTX, kSsaoTY, kSsaoHalo, 2, true, 1>, g, kSsaoTileLanes, 0, st, dd,
                   dn, dt, tb, pt);
        else if (early == 2)
            launch("ssao_lds_kernel", kSsaoTileLanes,
                   ssao_lds_kernel<true, true, true, kSsaoTX, kSsaoTY, kSsaoHalo, 2, true, 2>, g, kSsaoTileLanes, 0, st, dd,
                   dn, dt, tb, pt);
        else
            launch("ssao_lds_kernel", kSsaoTileLanes, ssao_lds_kernel<true, true, true, kSsaoTX, kSsaoTY, kSsaoHalo, 2, true>,
                   g, kSsaoTileLanes, 0, st, dd, dn, dt, tb, pt);
    } else if (noise_table && sip && full) SOC_SSAO_LAUNCH(true, true, true);
    else if (noise_table && sip) SOC_SSAO_LAUNCH(true, true, false);
    else if (noise_table) SOC_SSAO_LAUNCH(true, false, false);
    else if (sip && full) SOC_SSAO_LAUNCH(false, true, true);
    else SOC_SSAO_LAUNCH(false, false, false);
#undef SOC_SSAO_LAUNCH
    return check_launch("ssao_generation");
}

extern "C" int soc_ssao_blur(const soc_globals* g, soc_img ssao, soc_img target, soc_stream stream) {
    (void)g;
    int rc = check_img(ssao, SOC_FMT_R8_UNORM, "soc_ssao_blur", "ssao");
    if (!rc) rc = check_img(target, SOC_FMT_R8_UNORM, "soc_ssao_blur", "target");
    if (rc) return rc;
    if (ssao.data == target.data) return set_error(SOC_E_INVALID_ARG, "soc_ssao_blur: source and target alias");
    dim3 blk(64, 4), grd(ceil_div(target.width, 64), ceil_div(target.height, 4));
    if (ssao.width == target.width && ssao.height == target.height && ssao.width <= 8192 && ssao.height <= 8192)
        launch("ssao_blur_kernel", kWorkgroup, ssao_blur_kernel, grd, blk, 0, hs(stream), dimg(ssao), dimg(target));
    else
        launch("ssao_blur_generic", kWorkgroup, ssao_blur_generic, grd, blk, 0, hs(stream), dimg(ssao), dimg(target), 1.0f / (float)ssao.width,
                                                       1.0f / (float)ssao.height);
    return check_launch("ssao_blur");
}
