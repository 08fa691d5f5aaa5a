// composition.hip — CompositionTask (src/graphics/tasks/composition.inl:29-79, shader :110-225) as a
// gfx950 kernel.
//
// HBM-bound stream: per pixel it reads depth (4 B), albedo/emissive/normal (8 B each), one bilinear
// half-res AO tap, one bilinear 4096^2 shadow-map tap and, on sky pixels only, the clouds texel; it
// writes 8 B of RGBA16F. Fast path: two horizontally adjacent pixels per lane so every G-buffer load
// and the store are 16 B per lane, a wave covering a 16x8 pixel block (one 128-B line per image row);
// the block shape keeps the shadow-map gathers of a wave in a compact 2D patch of the map (measured:
// 89 -> 75 us at 4K against 128x1 strips). Full-res taps are plain loads (a centre sample under the
// sampling contract is the texel itself). The dead volumetric-fog block (:176-196, zeroed at :196)
// is not computed.
#include <type_traits>

#include "bloom_w.hpp"
#include "luminance.hpp"
#include "soc_internal.hpp"

// Profiling builds only (tools/kernel_variants.py): 1 = no shadow-map tap, 2 = no AO tap, 3 = neither.
#ifndef SOC_COMP_PROFILE
#define SOC_COMP_PROFILE 0
#endif

namespace soc {
namespace {

struct CompParams {
    Mat4 inv_proj, inv_view, sun_pv;
    Mat4 sun_clip;        // sun_pv * inv_view * inv_proj: NDC (x, y, depth, 1) -> sun clip space
    float sun_dir[3], ambient[3], cam[3];
    float ef, df, emissive_strength, ao_strength;
    uint32_t npl, nsl;
    int swz;   // XCD-aware tile order (fast path)
    uint32_t* bins;        // fused histogram: 8 x 256 scratch copies (composition_pair<true>)
    float lmin, lrange;    // log_min_luminance, log_max - log_min
    BinFast bf;            // lum_bin_fast parameters
    const soc_globals* __restrict__ dg;  // device globals (lights), may be null when npl == nsl == 0
    int sky_external;      // 1: sky pixels (depth == 1) are written and binned by sky_compose_pair (second lane)
    float rw, rh;          // recip_rn(target extent) for the pixel-centre uv (div_rn)
};

__device__ __forceinline__ float fast_pow(float x, float y) {
    // pow(x, y) = exp2(y * log2(x)) on the native transcendental units (as the reference GPU does)
    return __builtin_amdgcn_exp2f(y * __builtin_amdgcn_logf(x));
}

// The light loops are written once over a lane type T: float (one pixel) or f2v (the lane's two pixels as packed
// f32 pairs, v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32), with the same operations in the same order, so both
// forms give the same bits per pixel. The light records are wave-uniform scalars, broadcast into both halves.
typedef float f2v __attribute__((ext_vector_type(2)));
template <class T> struct V3 { T x, y, z; };
__device__ __forceinline__ float bcv(float s, float) { return s; }
__device__ __forceinline__ f2v bcv(float s, f2v) { return f2v{s, s}; }
__device__ __forceinline__ float vfma(float a, float b, float c) { return __builtin_fmaf(a, b, c); }
__device__ __forceinline__ f2v vfma(f2v a, f2v b, f2v c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ float vrsq(float x) { return __builtin_amdgcn_rsqf(x); }
__device__ __forceinline__ f2v vrsq(f2v x) { return f2v{__builtin_amdgcn_rsqf(x.x), __builtin_amdgcn_rsqf(x.y)}; }
__device__ __forceinline__ float vsqrt(float x) { return __builtin_amdgcn_sqrtf(x); }
__device__ __forceinline__ f2v vsqrt(f2v x) { return f2v{__builtin_amdgcn_sqrtf(x.x), __builtin_amdgcn_sqrtf(x.y)}; }
__device__ __forceinline__ float vexp2(float x) { return __builtin_amdgcn_exp2f(x); }
__device__ __forceinline__ f2v vexp2(f2v x) { return f2v{__builtin_amdgcn_exp2f(x.x), __builtin_amdgcn_exp2f(x.y)}; }
__device__ __forceinline__ float vabs(float x) { return fabsf(x); }
__device__ __forceinline__ f2v vabs(f2v x) { return f2v{fabsf(x.x), fabsf(x.y)}; }
__device__ __forceinline__ float vmax0(float x) { return fmaxf(x, 0.0f); }
__device__ __forceinline__ f2v vmax0(f2v x) { return f2v{fmaxf(x.x, 0.0f), fmaxf(x.y, 0.0f)}; }
__device__ __forceinline__ float vclamp01(float x) { return clampf(x, 0.0f, 1.0f); }
__device__ __forceinline__ f2v vclamp01(f2v x) { return f2v{clampf(x.x, 0.0f, 1.0f), clampf(x.y, 0.0f, 1.0f)}; }
__device__ __forceinline__ float vneg_pi(float x, float r) { return x < 0.0f ? 3.14159265358979f - r : r; }
__device__ __forceinline__ f2v vneg_pi(f2v x, f2v r) {
    const f2v q = f2v{3.14159265358979f, 3.14159265358979f} - r;
    return f2v{x.x < 0.0f ? q.x : r.x, x.y < 0.0f ? q.y : r.y};
}
__device__ __forceinline__ float vnan_outside1(float x, float r) { return fabsf(x) > 1.0f ? __builtin_nanf("") : r; }
__device__ __forceinline__ f2v vnan_outside1(f2v x, f2v r) {
    return f2v{fabsf(x.x) > 1.0f ? __builtin_nanf("") : r.x, fabsf(x.y) > 1.0f ? __builtin_nanf("") : r.y};
}
__device__ __forceinline__ float vdiv(float a, float b) { return a / b; }
__device__ __forceinline__ f2v vdiv(f2v a, float b) { return f2v{a.x / b, a.y / b}; }
template <class T> __device__ __forceinline__ T vdot(const V3<T>& a, const V3<T>& b) {
    return vfma(a.z, b.z, vfma(a.y, b.y, a.x * b.x));
}

// acos on the native units: Abramowitz & Stegun 4.4.46, acos(a) = sqrt(1 - a) * P7(a) for a in [0, 1]
// (|error| <= 2e-8 rad), acos(x) = pi - acos(-x) below 0. Outside [-1, 1] the sqrt gives NaN, as acos does.
template <class T>
__device__ __forceinline__ T acos_fast(T x) {
    const T a = vabs(x);
    T r = bcv(-0.0012624911f, x);
    r = vfma(r, a, bcv(0.0066700901f, x));
    r = vfma(r, a, bcv(-0.0170881256f, x));
    r = vfma(r, a, bcv(0.0308918810f, x));
    r = vfma(r, a, bcv(-0.0501743046f, x));
    r = vfma(r, a, bcv(0.0889789874f, x));
    r = vfma(r, a, bcv(-0.2145988016f, x));
    r = vfma(r, a, bcv(1.5707963050f, x));
    r = r * vsqrt(bcv(1.0f, x) - a);
    return vneg_pi(x, r);
}

// exp(-acos(c)^2), the specular term of composition.inl:135-138, as one degree-10 polynomial in c (least squares on
// [-1, 1], fp32 Horner): |error| <= 1.1e-6 for c >= -0.9 and <= 2.6e-5 at c = -1, where the term itself is 5e-5 (acos is
// not analytic there; exp(-acos^2) is tiny). Ten FMAs instead of acos_fast's polynomial, square root and select plus
// the exponential: two transcendentals less per light and pixel. NaN outside [-1, 1], as acos (and acos_fast) give.
// SOC_COMP_SPEC_POLY=0 (build-time) keeps acos_fast + exp2.
#ifndef SOC_COMP_SPEC_POLY
#define SOC_COMP_SPEC_POLY 1
#endif
template <class T>
__device__ __forceinline__ T spec_exp_acos2(T c) {
    constexpr float k[11] = {0.08480516821146011f,  0.26642516255378723f,  0.33367738127708435f,   0.21618370711803436f,
                             0.07947526127099991f,  0.017337322235107422f, 0.0017174964305013418f, -0.00019129738211631775f,
                             0.0007113117026165128f, 0.00020575939561240375f, -0.00034820116707123816f};
    T r = bcv(k[10], c);
#pragma unroll
    for (int i = 9; i >= 0; --i) r = vfma(r, c, bcv(k[i], c));
    return vnan_outside1(c, r);
}

// The light loops of composition.inl:124-160, per light: L = light - pos, one rsqrt gives light_dir and the
// attenuation 1 / distance^2; dot(normalize(light_dir + view_dir), n) with one more rsqrt; the specular
// exp(-acos(x)^2) as one polynomial (spec_exp_acos2). The pixel's view_dir is hoisted out of the loop and the
// frag_color (albedo) factor out of the sum. Within the RGBA16F tolerance of the oracle's libm restatement.
// Light records are wave-uniform (scalar loads from the device globals).
template <class T>
__device__ __forceinline__ V3<T> light_sum(const soc_globals* __restrict__ dg, uint32_t npl, uint32_t nsl, const V3<T>& n,
                                           const V3<T>& pos, f3 cam) {
    const T z = pos.x;   // lane-type witness for the broadcasts
    const V3<T> vd0 = {bcv(cam.x, z) - pos.x, bcv(cam.y, z) - pos.y, bcv(cam.z, z) - pos.z};
    const T vk = vrsq(vdot(vd0, vd0));
    const V3<T> view_dir = {vd0.x * vk, vd0.y * vk, vd0.z * vk};
    V3<T> acc = {bcv(0.0f, z), bcv(0.0f, z), bcv(0.0f, z)};
    const T nlog2e = bcv(-1.44269504088896f, z);
    auto shade_light = [&](const float* lp, T& inv, V3<T>& ld) {
        const V3<T> l = {bcv(lp[0], z) - pos.x, bcv(lp[1], z) - pos.y, bcv(lp[2], z) - pos.z};
        inv = vrsq(vdot(l, l));
        ld = V3<T>{l.x * inv, l.y * inv, l.z * inv};
        const V3<T> h = {ld.x + view_dir.x, ld.y + view_dir.y, ld.z + view_dir.z};
        const T c = vdot(h, n) * vrsq(vdot(h, h));
        const T diffuse = vmax0(vdot(n, ld));
        if (SOC_COMP_SPEC_POLY) return (diffuse + spec_exp_acos2(c)) * (inv * inv);
        const T nh = acos_fast(c);
        return (diffuse + vexp2((nh * nh) * nlog2e)) * (inv * inv);
    };
    auto add = [&](const float* col, T s) {
        acc = V3<T>{vfma(bcv(col[0], z), s, acc.x), vfma(bcv(col[1], z), s, acc.y), vfma(bcv(col[2], z), s, acc.z)};
    };
// 2 lights per round (4: 108 VGPRs, 4 waves per SIMD); with the fused-histogram lights kernel held to 6 waves per SIMD
// (70 VGPRs, no spill): C3b 782 -> 799 fps (profiles/r05_ab_light_loop.txt)
#ifndef SOC_COMP_LIGHT_UNROLL
#define SOC_COMP_LIGHT_UNROLL 2
#endif
#pragma unroll SOC_COMP_LIGHT_UNROLL
    for (uint32_t i = 0; i < npl; ++i) {            // calculate_point_light, :124-139
        const soc_point_light& L = dg->point_lights[i];
        T inv;
        V3<T> ld;
        const T s = shade_light(L.position, inv, ld) * bcv(L.intensity, z);
        add(L.color, s);
    }
#pragma unroll 2
    for (uint32_t i = 0; i < nsl; ++i) {            // calculate_spot_light, :141-160
        const soc_spot_light& L = dg->spot_lights[i];
        T inv;
        V3<T> ld;
        const T b = shade_light(L.position, inv, ld);
        const float sdx = -L.direction[0], sdy = -L.direction[1], sdz = -L.direction[2];
        const float sk = __builtin_amdgcn_rsqf(__builtin_fmaf(sdz, sdz, __builtin_fmaf(sdy, sdy, sdx * sdx)));
        const T theta = vfma(ld.z, bcv(sdz, z), vfma(ld.y, bcv(sdy, z), ld.x * bcv(sdx, z))) * bcv(sk, z);
        const T intensity = vclamp01(vdiv(theta - bcv(L.outer_cut_off, z), L.cut_off - L.outer_cut_off));
        add(L.color, b * bcv(L.intensity, z) * intensity);
    }
    return acc;
}

// Shading of one pixel given its G-buffer values (composition.inl:164-224), in two parts around the light sum:
// shade_pre (sun ESM shadow, emissive, AO) and shade_post (lights, ambient, albedo, AO, emissive).
// The sun-space position is one projective transform of the NDC point: vs = inv_proj * ndc,
// ws = inv_view * (vs / vs.w), sp = sun_pv * ws, and pc = sp.xyz / sp.w, so the vs.w division cancels
// and sun_clip = sun_pv * inv_view * inv_proj (host fp32) gives pc directly (one rcp; within the
// RGBA16F tolerance). The world position itself is only formed for the light loops.
struct ShadePre {
    float direct;   // the sun term dot(n, -sun) * shadow (grey)
    float occl;
    f3 em;
};
template <typename ShadowImg = DImg>
__device__ __forceinline__ ShadePre shade_pre(const CompParams& p, float u, float v, float d, f3 emissive, f3 n, float ssao,
                                              const ShadowImg& shadow) {
    const f4 ndc = f4{u * 2.0f - 1.0f, v * 2.0f - 1.0f, d, 1.0f};
    // sun ESM shadow, :166-173
    const f4 sp = mul(p.sun_clip, ndc);
    const float rsw = __builtin_amdgcn_rcpf(sp.w);
    const float pcx = sp.x * rsw * 0.5f + 0.5f;
    const float pcy = sp.y * rsw * 0.5f + 0.5f;
    const float pcz = sp.z * rsw;
    const float sd = (SOC_COMP_PROFILE & 1) ? pcx * 0.001f : sample_f32(shadow, pcx, pcy);
    float e = __expf(p.ef * (pcz - sd));
    if (p.df != 1.0f) e = fast_pow(e, p.df);   // pow(x, 1.0) == x exactly
    const float sun_shadow = clampf(e, 0.0f, 1.0f);
    ShadePre s;
    s.em = emissive * p.emissive_strength;
    s.occl = fast_pow(ssao, p.ao_strength);
    s.direct = fmaxf(0.0f, dot3(n, -mk3(p.sun_dir[0], p.sun_dir[1], p.sun_dir[2]))) * sun_shadow;
    return s;
}
// get_world_position_from_depth, :114-122
__device__ __forceinline__ f3 world_pos(const CompParams& p, float u, float v, float d) {
    const f4 ndc = f4{u * 2.0f - 1.0f, v * 2.0f - 1.0f, d, 1.0f};
    f4 vs = mul(p.inv_proj, ndc);
    const float rw = __builtin_amdgcn_rcpf(vs.w);
    vs = f4{vs.x * rw, vs.y * rw, vs.z * rw, 1.0f};
    const f4 ws = mul(p.inv_view, vs);
    return f3{ws.x, ws.y, ws.z};
}
__device__ __forceinline__ f4 shade_post(const CompParams& p, const ShadePre& s, f3 albedo, const f3* lights) {
    f3 direct = f3{s.direct, s.direct, s.direct};
    if (lights)
        direct = f3{__builtin_fmaf(albedo.x, lights->x, direct.x), __builtin_fmaf(albedo.y, lights->y, direct.y),
                    __builtin_fmaf(albedo.z, lights->z, direct.z)};
    const f3 c = (direct + mk3(p.ambient[0], p.ambient[1], p.ambient[2])) * albedo * s.occl + s.em;
    return f4{c.x, c.y, c.z, 1.0f};
}
template <bool LIGHTS = true, typename ShadowImg = DImg>
__device__ __forceinline__ f4 shade(const CompParams& p, float u, float v, float d, f3 albedo, f3 emissive, f3 n,
                                    float ssao, const ShadowImg& shadow) {
    const ShadePre s = shade_pre(p, u, v, d, emissive, n, ssao, shadow);
    if (LIGHTS && (p.npl | p.nsl)) {
        const f3 wp = world_pos(p, u, v, d);
        const V3<float> ls = light_sum(p.dg, p.npl, p.nsl, V3<float>{n.x, n.y, n.z}, V3<float>{wp.x, wp.y, wp.z},
                                       mk3(p.cam[0], p.cam[1], p.cam[2]));
        const f3 l3 = f3{ls.x, ls.y, ls.z};
        return shade_post(p, s, albedo, &l3);
    }
    return shade_post(p, s, albedo, nullptr);
}

constexpr int BX = 64, BY = 4;

// Fast path: all full-res images share the target extent, width even, rows 16-B aligned.
// HIST: GenerateLuminanceHistogramTask fused in (generate_luminance_histogram.inl:59-78): the bins of the
// two stored RGBA16F pixels (the exact values the histogram pass would read back; lum_bin_fast with the
// exact fallback) are added into the wave's LDS histogram with one LDS atomic per lane (lane_bin_pair_mask: measured 90 -> 66 us
// at 4K on the textured mesh against the ballot-aggregated loop, whose rounds grow with the distinct bins of a wave and
// run on the VALU), which the workgroup flushes with one device atomic per
// non-zero bin (~3.6 distinct bins per 32x16 tile at 4K), saving the 8 B/px re-read of the colour.
// The flush goes to one of 8 scratch copies chosen by linear block id mod 8 (the XCD under round-robin
// dispatch): a single copy serialises the ~5k atomics of the hottest bin (measured 172 us vs 77 us),
// 8 copies cut that 8x. histogram_fold adds the copies into the AutoExposure bins and re-zeroes them.
// Measured at 4K (kernel trace): 68.4 us + a 4 us fold against 66-68 + 27.7 us for the two passes; frame
// 0.679 -> 0.660 ms. The render graph fuses by default (SOC_RENDERER_UNFUSED_HISTOGRAM: two passes).
// (An in-kernel fold by the last-arriving workgroup instead of the fold launch costs one same-address
// device atomic per workgroup: 16,200 of them serialise across the XCDs, 68 -> 207 us.)
// LIGHTS = false: no point / spot lights this frame (the reference default): the light loops are not
// compiled in, which keeps the kernel at a fraction of the registers (more waves, more loads in flight).
// BL (SOC_RENDERER_BLOOM_IN_COMPOSITION): the bloom chain's last upsample pair (mip1 -> [mip0] -> output, bloomw_up10s)
// is computed for the workgroup's 32 x 16 tile in LDS (Up10Tile, bloom_w.hpp: the same values per pixel, rounded to
// RGBA16F as the chain stores its output) while the G-buffer loads are in flight, and used as the emissive input, so
// the full-resolution bloom output is neither written by the chain nor read back here (16 B/px). `emissive` unused.
#ifndef SOC_COMP_LIGHT_WAVES
#define SOC_COMP_LIGHT_WAVES 6
#endif
template <bool HIST, bool LIGHTS, int NT = 0, bool BL = false>
__global__ __launch_bounds__(kWorkgroup) __attribute__((amdgpu_waves_per_eu(LIGHTS && !BL ? SOC_COMP_LIGHT_WAVES : 1))) void composition_pair(DImg target, DImg albedo, DImg emissive, DImg normal, DImg depth,
                                                        DImg ssao, DImg shadow, DImg clouds, CompParams p, DImg mip1) {
    static_assert(!BL || HIST, "the in-kernel bloom runs in the fused-histogram kernel (no early exit before its barriers)");
    // a wave covers 16x8 pixels (8 lanes x 2 pixels per row, 8 rows): every row segment is one
    // 128-B line of each G-buffer image, and the wave's shadow-map taps form a compact 2D patch
    // (a 128x1 strip maps to a line across the 4096^2 map and touches a new line per tap)
    // HIST: one 256-bin LDS histogram per wave, zeroed by its own wave (LDS operations of a wave are
    // ordered), so no barrier stands in front of the G-buffer loads
    __shared__ uint32_t sh[HIST ? 4 * kBins : 1];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (HIST) reinterpret_cast<uint4*>(sh + wave * kBins)[lane] = uint4{0u, 0u, 0u, 0u};
    int bx, by;
    xcd_order(p.swz, bx, by);
    const int x = bx * 32 + (wave & 1) * 16 + (lane & 7) * 2;
    const int y = by * 16 + (wave >> 1) * 8 + (lane >> 3);
    const bool inside = x < target.w && y < target.h;
    if (!HIST && !inside) return;
    uint2 outp[2] = {uint2{0u, 0u}, uint2{0u, 0u}};
    uint32_t own = 3u;   // bit k: this kernel writes (and bins) pixel k of the pair
    // buffer descriptors + 32-bit offsets (one multiply-add per image row instead of 64-bit pointer math)
    const BufImg bd = buf_img(depth), ba = buf_img(albedo), be = buf_img(emissive), bn = buf_img(normal);
    const BufImg bt = buf_img(target), bs = buf_img(shadow), bo = buf_img(ssao);
    const float v = centre_uv_rn(y, target.h, p.rh);
    // once-read streams non-temporal (NT & 1: keep L2 for the shadow-map / AO gathers); aux bit 1 = nt
    constexpr int ld_aux = (NT & 1) ? 2 : 0;
    float2 d2 = float2{0.0f, 0.0f};
    uint4 a4 = uint4{0u, 0u, 0u, 0u}, e4 = a4, n4 = a4;
    // NT & 4: both pixels' AO taps (3 half-res texels per row) as one 8-B load per row, issued with the G-buffer
    // loads (not after the depth test), for sky pixels too (in bounds, unused); the same bits as sample_r8
    float aop[2] = {0.0f, 0.0f};
    if (inside) {
        d2 = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(bd.r, buf_row(bd, y) + x * 4, 0, ld_aux));
        a4 = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(ba.r, buf_row(ba, y) + x * 8, 0, ld_aux));
        if (!BL) e4 = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(be.r, buf_row(be, y) + x * 8, 0, ld_aux));
        n4 = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(bn.r, buf_row(bn, y) + x * 8, 0, ld_aux));
        if (NT & 4) sample_r8_pair(bo, centre_uv_rn(x, target.w, p.rw), centre_uv_rn(x + 1, target.w, p.rw), v, aop[0], aop[1]);
    }
    if constexpr (BL) {   // every lane takes part in the tile's barriers; the pair's bloom as the chain stores it
        __shared__ Up10Tile<32, 16> bl;
        const int X0 = bx * 32, Y0 = by * 16;
        bl.build(mip1, X0, Y0, target.w, target.h, threadIdx.x);
        C3 o[2];
        bl.out(y - Y0, x - X0, o);
        const uint2 b0 = pack3(o[0]), b1 = pack3(o[1]);
        e4 = uint4{b0.x, b0.y, b1.x, b1.y};
    }
    if (inside) {
        // LIGHTS: the light sum of the lane's two pixels runs once, as packed pairs (light_sum<f2v>, the same bits per
        // pixel as light_sum<float>); a sky pixel of the pair rides along in the other half and is discarded
        ShadePre pre[2];
        f3 alb[2], nrm[2], wps[2];
        uint32_t lit = 0u;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const float u = centre_uv_rn(x + k, target.w, p.rw);
            const float d = k ? d2.y : d2.x;
            const f4 al = unpack_h4(k ? uint2{a4.z, a4.w} : uint2{a4.x, a4.y});
            const f4 em = unpack_h4(k ? uint2{e4.z, e4.w} : uint2{e4.x, e4.y});
            const f4 nn = unpack_h4(k ? uint2{n4.z, n4.w} : uint2{n4.x, n4.y});
            f4 c;
            if (LIGHTS) {   // the same pixel values for a sky pixel's discarded half
                nrm[k] = f3{nn.x, nn.y, nn.z};
                wps[k] = world_pos(p, u, v, d);
            }
            if (d == 1.0f && p.sky_external) {   // the second lane writes it (sky_compose_pair)
                own &= ~(1u << k);
                continue;
            }
            if (d == 1.0f) {
                const f4 cl = fetch_rgba8(clouds, x + k, y);
                c = f4{cl.x, cl.y, cl.z, 1.0f};
            } else {
                const float ao = (SOC_COMP_PROFILE & 2) ? u : (NT & 4) ? aop[k] : sample_r8(bo, u, v);
                if (LIGHTS) {
                    pre[k] = shade_pre(p, u, v, d, f3{em.x, em.y, em.z}, f3{nn.x, nn.y, nn.z}, ao, bs);
                    alb[k] = f3{al.x, al.y, al.z};
                    lit |= 1u << k;
                    continue;
                }
                c = shade<false>(p, u, v, d, f3{al.x, al.y, al.z}, f3{em.x, em.y, em.z}, f3{nn.x, nn.y, nn.z}, ao, bs);
            }
            outp[k] = pack_h4(c);
        }
        if (LIGHTS && lit) {
            const V3<f2v> n2 = {f2v{nrm[0].x, nrm[1].x}, f2v{nrm[0].y, nrm[1].y}, f2v{nrm[0].z, nrm[1].z}};
            const V3<f2v> w2 = {f2v{wps[0].x, wps[1].x}, f2v{wps[0].y, wps[1].y}, f2v{wps[0].z, wps[1].z}};
            const V3<f2v> ls = light_sum(p.dg, p.npl, p.nsl, n2, w2, mk3(p.cam[0], p.cam[1], p.cam[2]));
#pragma unroll
            for (int k = 0; k < 2; ++k)
                if (lit & (1u << k)) {
                    const f3 l3 = k ? f3{ls.x.y, ls.y.y, ls.z.y} : f3{ls.x.x, ls.y.x, ls.z.x};
                    outp[k] = pack_h4(shade_post(p, pre[k], alb[k], &l3));
                }
        }
        const uint4 o = uint4{outp[0].x, outp[0].y, outp[1].x, outp[1].y};
        typedef uint32_t v4w __attribute__((ext_vector_type(4)));
        const int to = buf_row(bt, y) + x * 8;
        if (own == 3u) {
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4w, o), bt.r, to, 0, (NT & 2) ? 2 : 0);
        } else {   // a sky pixel in the pair belongs to the second lane: 8-B stores of ours only
            typedef uint32_t v2w __attribute__((ext_vector_type(2)));
            if (own & 1u) __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2w, outp[0]), bt.r, to, 0, 0);
            if (own & 2u) __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2w, outp[1]), bt.r, to + 8, 0, 0);
        }
    }
    if (HIST) {
        const f4 c0 = unpack_h4(outp[0]), c1 = unpack_h4(outp[1]);
        uint32_t b0 = lum_bin_fast(c0.x, c0.y, c0.z, p.bf);
        uint32_t b1 = lum_bin_fast(c1.x, c1.y, c1.z, p.bf);
        if (b0 == kBinExact) b0 = lum_bin(c0.x, c0.y, c0.z, p.lmin, p.lrange);
        if (b1 == kBinExact) b1 = lum_bin(c1.x, c1.y, c1.z, p.lmin, p.lrange);
        lane_bin_pair_mask(sh + wave * kBins, b0, b1, inside ? own : 0u);
        __syncthreads();
        const uint32_t n = sh[threadIdx.x] + sh[kBins + threadIdx.x] + sh[2 * kBins + threadIdx.x] + sh[3 * kBins + threadIdx.x];
        if (n) atomicAdd(&p.bins[((blockIdx.y * gridDim.x + blockIdx.x) & 7u) * kBins + threadIdx.x], n);
    }
}

// The sky pixels of the colour image (composition.inl:220-222: depth == 1 -> color = clouds texel), written and
// binned on the renderer's second lane right after CloudRendering, so Composition (sky_external) does not wait
// for the clouds: the same tiling, texel fetch, f16 packing and bins as composition_pair's sky branch, hence
// the same bits. 8-B stores of the sky pixels only (Composition writes the others concurrently).
// CP (clouds rows 8-B aligned): a pair's two clouds texels in one 8-B load, issued once the depth shows a sky pixel in
// the pair (one dependent load level instead of two); else the per-pixel form. The same texels.
template <bool CP>
__global__ __launch_bounds__(kWorkgroup) void sky_compose_pair(DImg target, DImg depth, DImg clouds, CompParams p) {
    __shared__ uint32_t sh[4 * kBins];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    reinterpret_cast<uint4*>(sh + wave * kBins)[lane] = uint4{0u, 0u, 0u, 0u};
    const int bx = blockIdx.x, by = blockIdx.y;
    const int x = bx * 32 + (wave & 1) * 16 + (lane & 7) * 2;
    const int y = by * 16 + (wave >> 1) * 8 + (lane >> 3);
    const bool inside = x < target.w && y < target.h;
    uint32_t mine = 0u;
    uint2 outp[2] = {uint2{0u, 0u}, uint2{0u, 0u}};
    if (inside) {
        const float2 d2 = row_ptr<float2>(depth, y)[x >> 1];
        const bool s0 = d2.x == 1.0f, s1 = d2.y == 1.0f;
        if (!CP) {
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                if (!(k ? s1 : s0)) continue;
                const f4 cl = fetch_rgba8(clouds, x + k, y);
                outp[k] = pack_h4(f4{cl.x, cl.y, cl.z, 1.0f});
                row_ptr_w<uint2>(target, y)[x + k] = outp[k];
                mine |= 1u << k;
            }
        } else if (s0 || s1) {   // both clouds texels of the pair in one 8-B load (the pair's x is even)
            const uint2 cw = row_ptr<uint2>(clouds, y)[x >> 1];
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                if (!(k ? s1 : s0)) continue;
                const f4 cl = unpack_rgba8(k ? cw.y : cw.x);
                outp[k] = pack_h4(f4{cl.x, cl.y, cl.z, 1.0f});
                row_ptr_w<uint2>(target, y)[x + k] = outp[k];
                mine |= 1u << k;
            }
        }
    }
    const f4 c0 = unpack_h4(outp[0]), c1 = unpack_h4(outp[1]);
    uint32_t b0 = lum_bin_fast(c0.x, c0.y, c0.z, p.bf);
    uint32_t b1 = lum_bin_fast(c1.x, c1.y, c1.z, p.bf);
    if (b0 == kBinExact) b0 = lum_bin(c0.x, c0.y, c0.z, p.lmin, p.lrange);
    if (b1 == kBinExact) b1 = lum_bin(c1.x, c1.y, c1.z, p.lmin, p.lrange);
    lane_bin_pair_mask(sh + wave * kBins, b0, b1, mine);
    __syncthreads();
    const uint32_t n = sh[threadIdx.x] + sh[kBins + threadIdx.x] + sh[2 * kBins + threadIdx.x] + sh[3 * kBins + threadIdx.x];
    if (n) atomicAdd(&p.bins[((blockIdx.y * gridDim.x + blockIdx.x) & 7u) * kBins + threadIdx.x], n);
}

__global__ __launch_bounds__(kBins) void histogram_fold(uint32_t* __restrict__ scratch, uint32_t* __restrict__ bins) {
    const int i = threadIdx.x;
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        s += scratch[k * kBins + i];
        scratch[k * kBins + i] = 0u;
    }
    if (s) bins[i] += s;
}

// Generic path: every input is sampled under the sampling contract.
__global__ __launch_bounds__(kWorkgroup) void composition_generic(DImg target, DImg albedo, DImg emissive, DImg normal,
                                                           DImg depth, DImg ssao, DImg shadow, DImg clouds, CompParams p) {
    const int x = blockIdx.x * BX + threadIdx.x, y = blockIdx.y * BY + threadIdx.y;
    if (x >= target.w || y >= target.h) return;
    const float u = centre_uv(x, target.w), v = centre_uv(y, target.h);
    const float d = sample_f32(depth, u, v);
    f4 c;
    if (d == 1.0f) {
        const f4 cl = sample_rgba8(clouds, u, v);
        c = f4{cl.x, cl.y, cl.z, 1.0f};
    } else {
        const f4 al = sample_h4(albedo, u, v), em = sample_h4(emissive, u, v), nn = sample_h4(normal, u, v);
        c = shade(p, u, v, d, f3{al.x, al.y, al.z}, f3{em.x, em.y, em.z}, f3{nn.x, nn.y, nn.z}, sample_r8(ssao, u, v),
                  shadow);
    }
    row_ptr_w<uint2>(target, y)[x] = pack_h4(c);
}

bool aligned16(const soc_img& im) {
    return (reinterpret_cast<uintptr_t>(im.data) & 15u) == 0 && (im.pitch_bytes & 15) == 0;
}

}  // namespace
}  // namespace soc

using namespace soc;

namespace {
// bins != nullptr: the fused histogram variant if the pair path applies at the globals' resolution
// (returns 1 otherwise, having launched nothing)
// bloom_mip1 != nullptr (the render graph under SOC_RENDERER_BLOOM_IN_COMPOSITION): the bloom output is computed in the
// kernel from the chain's mip1 (composition_pair<..., BL>); needs the fused histogram and the pair path.
int composition_launch(const soc_globals* g, const soc_globals* d_globals, soc_img target, soc_img albedo, soc_img emissive,
                       soc_img normal, soc_img depth, soc_img ssao, soc_img shadow, soc_img clouds, uint32_t* bins,
                       uint32_t* scratch, soc_stream stream, bool fold = true, bool sky_external = false,
                       const soc_img* bloom_mip1 = nullptr) {
    static const char* P = "soc_composition";
    if (!g) return set_error(SOC_E_INVALID_ARG, "%s: null globals", P);
    int rc = check_img(target, SOC_FMT_RGBA16F, P, "target");
    if (!rc) rc = check_img(albedo, SOC_FMT_RGBA16F, P, "albedo");
    if (!rc) rc = check_img(emissive, SOC_FMT_RGBA16F, P, "emissive");
    if (!rc) rc = check_img(normal, SOC_FMT_RGBA16F, P, "normal");
    if (!rc) rc = check_img(depth, SOC_FMT_D32F, P, "depth");
    if (!rc) rc = check_img(ssao, SOC_FMT_R8_UNORM, P, "ssao");
    if (!rc) rc = check_img(shadow, SOC_FMT_D32F, P, "shadow");
    if (!rc) rc = check_img(clouds, SOC_FMT_RGBA8_UNORM, P, "clouds");
    if (rc) return rc;
    CompParams p;
    p.inv_proj = mat4(g->camera_inverse_projection_matrix);
    p.inv_view = mat4(g->camera_inverse_view_matrix);
    mat4_mul_host(p.sun_pv.m, g->sun_info.projection_matrix, g->sun_info.view_matrix);
    {
        float t[16];
        mat4_mul_host(t, p.sun_pv.m, g->camera_inverse_view_matrix);
        mat4_mul_host(p.sun_clip.m, t, g->camera_inverse_projection_matrix);
    }
    for (int i = 0; i < 3; ++i) {
        p.sun_dir[i] = g->sun_info.direction[i];
        p.ambient[i] = g->ambient[i];
        p.cam[i] = g->camera_position[i];
    }
    p.ef = g->sun_info.exponential_factor;
    p.df = g->sun_info.darkening_factor;
    p.emissive_strength = g->emissive_bloom_strength;
    p.ao_strength = g->ambient_occlussion_strength;
    p.npl = g->point_light_count < SOC_MAX_POINT_LIGHTS ? g->point_light_count : SOC_MAX_POINT_LIGHTS;
    p.nsl = g->spot_light_count < SOC_MAX_SPOT_LIGHTS ? g->spot_light_count : SOC_MAX_SPOT_LIGHTS;
    p.dg = d_globals;
    // non-temporal G-buffer loads and colour store (default); SOC_COMP_NT=0 selects the default cache policy for the
    // variant-identity test
    const bool nt = tuning_knob("SOC_COMP_NT", 3) == 3;
    // SOC_COMP_AOP=0: the AO taps as 4 byte loads per pixel after the depth test (round 4); 1: sample_r8_pair
    const bool aop = tuning_knob("SOC_COMP_AOP", 1) != 0;
    p.swz = 0;   // row-major (the strip order measured 66 -> 77 us)
    p.rw = recip_rn(target.width);
    p.rh = recip_rn(target.height);
    p.bins = nullptr;
    p.sky_external = 0;
    if ((p.npl || p.nsl) && !d_globals)
        return set_error(SOC_E_INVALID_ARG, "%s: frame has lights but no device globals (soc_upload_globals)", P);

    const int W = target.width, H = target.height;
    auto same = [&](const soc_img& im) { return im.width == W && im.height == H; };
    const bool fast = same(albedo) && same(emissive) && same(normal) && same(depth) && same(clouds) && (W % 2 == 0) &&
                      W <= 8192 && H <= 8192 && aligned16(target) && aligned16(albedo) && aligned16(emissive) &&
                      aligned16(normal) && (reinterpret_cast<uintptr_t>(depth.data) & 7u) == 0 && (depth.pitch_bytes & 7) == 0;
    if (bins && !(fast && W == g->resolution[0] && H == g->resolution[1])) return 1;
    if (sky_external && !bins) return set_error(SOC_E_INVALID_ARG, "%s: sky_external needs the fused histogram", P);
    if (bloom_mip1) {
        rc = check_img(*bloom_mip1, SOC_FMT_RGBA16F, P, "bloom mip1");
        if (rc) return rc;
        if (!bins || !fast || bloom_mip1->width * 2 != W || bloom_mip1->height * 2 != H)
            return set_error(SOC_E_SHAPE, "%s: the in-kernel bloom needs the fused histogram's pair path and mip1 = W/2 x H/2", P);
    }
    if (fast) {
        dim3 grd(ceil_div(W, 32), ceil_div(H, 16));
        const bool lights = (p.npl | p.nsl) != 0;
#define SOC_COMP_PAIR(HI, LI) launch("composition_pair", kWorkgroup, composition_pair<HI, LI>, grd, kWorkgroup, 0, hs(stream), dimg(target), dimg(albedo), \
            dimg(emissive), dimg(normal), dimg(depth), dimg(ssao), dimg(shadow), dimg(clouds), p, DImg{})
        if (bins) {
            p.bins = scratch;
            p.sky_external = sky_external ? 1 : 0;
            p.lmin = g->log_min_luminance;
            p.lrange = g->log_max_luminance - g->log_min_luminance;
            p.bf = bin_fast_params(p.lmin, p.lrange);
            if (bloom_mip1 && lights)
                launch("composition_pair", kWorkgroup, composition_pair<true, true, 0, true>, grd, kWorkgroup, 0, hs(stream),
                       dimg(target), dimg(albedo), dimg(emissive), dimg(normal), dimg(depth), dimg(ssao), dimg(shadow),
                       dimg(clouds), p, dimg(*bloom_mip1));
            else if (bloom_mip1)
                launch("composition_pair", kWorkgroup, composition_pair<true, false, 7, true>, grd, kWorkgroup, 0, hs(stream),
                       dimg(target), dimg(albedo), dimg(emissive), dimg(normal), dimg(depth), dimg(ssao), dimg(shadow),
                       dimg(clouds), p, dimg(*bloom_mip1));
            else if (lights) SOC_COMP_PAIR(true, true);
            else if (nt && aop)
                launch("composition_pair", kWorkgroup, composition_pair<true, false, 7>, grd, kWorkgroup, 0, hs(stream), dimg(target), dimg(albedo), dimg(emissive),
                    dimg(normal), dimg(depth), dimg(ssao), dimg(shadow), dimg(clouds), p, DImg{});
            else if (nt)
                launch("composition_pair", kWorkgroup, composition_pair<true, false, 3>, grd, kWorkgroup, 0, hs(stream), dimg(target), dimg(albedo), dimg(emissive),
                    dimg(normal), dimg(depth), dimg(ssao), dimg(shadow), dimg(clouds), p, DImg{});
            else SOC_COMP_PAIR(true, false);
            if (fold) launch("histogram_fold", kBins, histogram_fold, 1, kBins, 0, hs(stream), scratch, bins);
        } else if (nt && !lights && aop) {
            launch("composition_pair", kWorkgroup, composition_pair<false, false, 7>, grd, kWorkgroup, 0, hs(stream), dimg(target), dimg(albedo), dimg(emissive),
                dimg(normal), dimg(depth), dimg(ssao), dimg(shadow), dimg(clouds), p, DImg{});
        } else if (nt && !lights) {
            // non-temporal G-buffer loads and colour store (measured at 4K: 71.5 -> 68 us; TAA, the next
            // reader of depth, +3 us: the frame is unchanged). SOC_COMP_NT=0: default cache policy.
            launch("composition_pair", kWorkgroup, composition_pair<false, false, 3>, grd, kWorkgroup, 0, hs(stream), dimg(target), dimg(albedo), dimg(emissive),
                dimg(normal), dimg(depth), dimg(ssao), dimg(shadow), dimg(clouds), p, DImg{});
        } else {
            if (lights) SOC_COMP_PAIR(false, true);
            else SOC_COMP_PAIR(false, false);
        }
#undef SOC_COMP_PAIR
    } else {
        dim3 blk(BX, BY), grd(ceil_div(W, BX), ceil_div(H, BY));
        launch("composition_generic", kWorkgroup, composition_generic, grd, blk, 0, hs(stream), dimg(target), dimg(albedo), dimg(emissive), dimg(normal),
                                                         dimg(depth), dimg(ssao), dimg(shadow), dimg(clouds), p);
    }
    return check_launch("composition");
}
}  // namespace

bool soc::composition_pair_applicable(const soc_globals* g, const soc_img& target, const soc_img& albedo,
                                      const soc_img& emissive, const soc_img& normal, const soc_img& depth,
                                      const soc_img& clouds) {
    const int W = target.width, H = target.height;
    auto same = [&](const soc_img& im) { return im.width == W && im.height == H; };
    return g && same(albedo) && same(emissive) && same(normal) && same(depth) && same(clouds) && (W % 2 == 0) &&
           W <= 8192 && H <= 8192 && aligned16(target) && aligned16(albedo) && aligned16(emissive) &&
           aligned16(normal) && (reinterpret_cast<uintptr_t>(depth.data) & 7u) == 0 && (depth.pitch_bytes & 7) == 0 &&
           W == g->resolution[0] && H == g->resolution[1];
}

int soc::sky_compose_launch(const soc_globals* g, soc_img target, soc_img depth, soc_img clouds, uint32_t* scratch,
                            soc_stream stream) {
    if (!g || !scratch) return set_error(SOC_E_INVALID_ARG, "sky compose: null globals / scratch");
    int rc = check_img(target, SOC_FMT_RGBA16F, "sky compose", "target");
    if (!rc) rc = check_img(depth, SOC_FMT_D32F, "sky compose", "depth");
    if (!rc) rc = check_img(clouds, SOC_FMT_RGBA8_UNORM, "sky compose", "clouds");
    if (rc) return rc;
    CompParams p{};
    p.bins = scratch;
    p.lmin = g->log_min_luminance;
    p.lrange = g->log_max_luminance - g->log_min_luminance;
    p.bf = bin_fast_params(p.lmin, p.lrange);
    const dim3 grd(ceil_div(target.width, 32), ceil_div(target.height, 16));
    const bool cp = (clouds.pitch_bytes % 8) == 0 && (reinterpret_cast<uintptr_t>(clouds.data) % 8) == 0 &&
                    tuning_knob("SOC_SKY_COMPOSE_PAIR_LOAD", 1);
    if (cp)
        launch("sky_compose_pair", kWorkgroup, sky_compose_pair<true>, grd, kWorkgroup, 0, hs(stream), dimg(target), dimg(depth),
               dimg(clouds), p);
    else
        launch("sky_compose_pair", kWorkgroup, sky_compose_pair<false>, grd, kWorkgroup, 0, hs(stream), dimg(target), dimg(depth),
               dimg(clouds), p);
    return check_launch("sky_compose");
}

extern "C" int soc_composition(const soc_globals* g, const soc_globals* d_globals, soc_img target, soc_img albedo,
                               soc_img emissive, soc_img normal, soc_img depth, soc_img ssao, soc_img shadow,
                               soc_img clouds, soc_stream stream) {
    return composition_launch(g, d_globals, target, albedo, emissive, normal, depth, ssao, shadow, clouds, nullptr, nullptr,
                              stream);
}

int soc::composition_luminance_histogram(const soc_globals* g, const soc_globals* d_globals, soc_img target,
                                         soc_img albedo, soc_img emissive, soc_img normal, soc_img depth, soc_img ssao,
                                         soc_img shadow, soc_img clouds, soc_auto_exposure* ae, uint32_t* scratch,
                                         bool fold, soc_stream stream, bool sky_external, const soc_img* bloom_mip1) {
    if (!g || !ae || !scratch)
        return set_error(SOC_E_INVALID_ARG, "soc_composition_luminance_histogram: null globals / auto exposure / scratch");
    int rc = composition_launch(g, d_globals, target, albedo, emissive, normal, depth, ssao, shadow, clouds,
                                ae->histogram_buckets, scratch, stream, fold, sky_external, bloom_mip1);
    if (rc <= 0) return rc;   // launched (or failed validation)
    if (bloom_mip1) return set_error(SOC_E_SHAPE, "composition: the in-kernel bloom needs the pair path");
    if (sky_external) return set_error(SOC_E_INVALID_ARG, "composition: sky_external needs the pair path");
    // not fusable: the two passes back to back (same results)
    rc = composition_launch(g, d_globals, target, albedo, emissive, normal, depth, ssao, shadow, clouds, nullptr, nullptr,
                            stream);
    if (rc) return rc;
    return soc_generate_luminance_histogram(g, target, ae, stream);
}

int soc::histogram_fold_launch(uint32_t* scratch, soc_auto_exposure* ae, soc_stream stream) {
    if (!scratch || !ae) return set_error(SOC_E_INVALID_ARG, "histogram fold: null scratch / auto exposure");
    launch("histogram_fold", kBins, histogram_fold, 1, kBins, 0, hs(stream), scratch, ae->histogram_buckets);
    return check_launch("luminance_histogram_fold");
}

extern "C" int soc_composition_luminance_histogram(const soc_globals* g, const soc_globals* d_globals, soc_img target,
                                                   soc_img albedo, soc_img emissive, soc_img normal, soc_img depth,
                                                   soc_img ssao, soc_img shadow, soc_img clouds, soc_auto_exposure* ae,
                                                   uint32_t* scratch, soc_stream stream) {
    return composition_luminance_histogram(g, d_globals, target, albedo, emissive, normal, depth, ssao, shadow, clouds, ae,
                                           scratch, true, stream);
}
