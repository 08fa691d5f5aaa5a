// taa.hip — TemporalAntiAliasingTask (src/graphics/tasks/temporal_antialiasing.inl:54-116, shader
// :137-190) and CopyImageTask (:16-37) as gfx950 kernels.
//
// One lane per output pixel, 64x4 workgroups (a wave reads 3 consecutive 512-B row segments of the
// colour and depth images; the 3x3 neighbourhood re-reads come from L1). The history copies of the
// reference graph (renderer.cpp:1182-1198) are removed: the resolved colour ping-pongs between two
// images owned by the caller, and the current velocity is written to the next frame's velocity
// history from inside this kernel (velocity_history_out), which saves the separate 16 B/px copy.
#include "agx.hpp"
#include "soc_internal.hpp"

namespace soc {
namespace {

struct TaaParams {
    float rw, rh;       // recip_rn(target extent) for the pixel-centre uv (div_rn)
    float pox, poy;     // 1 / resolution
    float accum0;       // min(0.1, frame_counter)
    int swz;            // XCD-aware tile order (pair path)
};

constexpr int BX = 64, BY = 4;

__device__ __forceinline__ f4 min4(f4 a, f4 b) { return f4{fminf(a.x, b.x), fminf(a.y, b.y), fminf(a.z, b.z), fminf(a.w, b.w)}; }
__device__ __forceinline__ f4 max4(f4 a, f4 b) { return f4{fmaxf(a.x, b.x), fmaxf(a.y, b.y), fmaxf(a.z, b.z), fmaxf(a.w, b.w)}; }

// Tail of the shader after the neighbourhood loop (:172-189).
__device__ __forceinline__ f4 resolve(const TaaParams& p, float u, float v, f4 color, f4 mn, f4 mx, f4 blurred, float2 vel,
                                      const DImg& prev, const DImg& pvel) {
    float accum = p.accum0;
    const float vx = u - vel.x, vy = v - vel.y;
    f4 acc = sample_h4(prev, vx, vy);
    if (vx < 0.0f || vy < 0.0f || vx > 1.0f || vy > 1.0f) accum = 1.0f;
    acc = f4{clampf(acc.x, mn.x, mx.x), clampf(acc.y, mn.y, mx.y), clampf(acc.z, mn.z, mx.z), clampf(acc.w, mn.w, mx.w)};
    f4 o = f4{color.x * accum + acc.x * (1.0f - accum), color.y * accum + acc.y * (1.0f - accum),
              color.z * accum + acc.z * (1.0f - accum), color.w * accum + acc.w * (1.0f - accum)};
    const f4 pv = sample_h4(pvel, vx, vy);
    const float dvx = pv.x - vel.x, dvy = pv.y - vel.y;
    const float vlen = sqrtf(dvx * dvx + dvy * dvy);
    const float dis = clampf((vlen - 0.001f) * 10.0f, 0.0f, 1.0f);
    return f4{mixf(o.x, blurred.x, dis), mixf(o.y, blurred.y, dis), mixf(o.z, blurred.z, dis), mixf(o.w, blurred.w, dis)};
}

__device__ __forceinline__ float gauss_w(int idx) {
    // 1/16 1/8 1/16 / 1/8 1/4 1/8 / 1/16 1/8 1/16
    return (idx == 4) ? 0.25f : ((idx & 1) ? 0.125f : 0.0625f);
}

// Fast path: colour, depth and velocity have the target extent (== resolution): every neighbourhood
// tap is a texel centre (clamped at the border), so plain loads replace the bilinear samples.
__global__ __launch_bounds__(kWorkgroup) void taa_fast(DImg target, DImg cur, DImg prev, DImg vel, DImg pvel, DImg depth,
                                                DImg vel_out, TaaParams p) {
    const int x = blockIdx.x * BX + threadIdx.x, y = blockIdx.y * BY + threadIdx.y;
    if (x >= target.w || y >= target.h) return;
    const float u = centre_uv(x, target.w), v = centre_uv(y, target.h);
    f4 nb5 = f4{0, 0, 0, 0};
    f4 blurred = f4{0, 0, 0, 0};
    f4 mn = f4{10.0e5f, 10.0e5f, 10.0e5f, 10.0e5f}, mx = f4{-10.0e5f, -10.0e5f, -10.0e5f, -10.0e5f};
    float closest = 1.0f;
    int bx = x, by = y;
#pragma unroll
    for (int oy = 1; oy > -2; --oy) {
        const int sy = min(max(y + oy, 0), target.h - 1);
        const uint2* crow = row_ptr<uint2>(cur, sy);
        const float* drow = row_ptr<float>(depth, sy);
#pragma unroll
        for (int ox = 1; ox > -2; --ox) {
            const int idx = (oy + 1) * 3 + (ox + 1);
            const int sx = min(max(x + ox, 0), target.w - 1);
            const f4 c = unpack_h4(crow[sx]);
            const float d = drow[sx];
            closest = fminf(d, closest);
            if (closest == d) { bx = sx; by = sy; }
            mn = min4(c, mn);
            mx = max4(c, mx);
            const float gw = gauss_w(idx);
            blurred = f4{blurred.x + gw * c.x, blurred.y + gw * c.y, blurred.z + gw * c.z, blurred.w + gw * c.w};
            if (idx == 5) nb5 = c;   // quirk Q7: the (+1, 0) neighbour is "the" colour
        }
    }
    const f4 vv = fetch_h4(vel, bx, by);
    const f4 o = resolve(p, u, v, nb5, mn, mx, blurred, float2{vv.x, vv.y}, prev, pvel);
    row_ptr_w<uint2>(target, y)[x] = pack_h4(o);
    if (vel_out.data) row_ptr_w<uint2>(vel_out, y)[x] = row_ptr<uint2>(vel, y)[x];
}

typedef uint32_t u4a8 __attribute__((ext_vector_type(4))) __attribute__((aligned(8)));

// ---- two pixels per lane, reduced instruction count (the pass is VALU-issue bound on gfx950) ----
typedef _Float16 h2 __attribute__((ext_vector_type(2)));
typedef float v2f __attribute__((ext_vector_type(2)));

__device__ __forceinline__ h2 as_h2(uint32_t u) { return __builtin_bit_cast(h2, u); }
__device__ __forceinline__ v2f h2f2(h2 h) { return v2f{(float)h.x, (float)h.y}; }

// Bilinear samples with the contract's taps; the lerps are fma(w, b - a, a) (within the RGBA16F tolerance of the
// pass; the texel selection is exactly the contract's). 16-B row-pair loads. The axes are computed once by the
// caller for the history colour and velocity (same extent).
// The f16 half HI of a packed word, as fp32 (the conversion is exact).
template <int HI>
__device__ __forceinline__ float half_f(uint32_t u) {
    return (float)__builtin_bit_cast(_Float16, (uint16_t)(HI ? u >> 16 : u & 0xffffu));
}
// b - a of the f16 halves HI of two words as one v_fma_mix_f32 (b * 1.0 - a, rounded once: the bits of
// (float)b - (float)a; the compiler would convert both halves and subtract, three instructions)
template <int HI>
__device__ __forceinline__ float sub_h(uint32_t b, uint32_t a) {
    float r;
    if (HI) asm("v_fma_mix_f32 %0, %1, 1.0, -%2 op_sel:[1,0,1] op_sel_hi:[1,0,1]" : "=v"(r) : "v"(b), "v"(a));
    else asm("v_fma_mix_f32 %0, %1, 1.0, -%2 op_sel_hi:[1,0,1]" : "=v"(r) : "v"(b), "v"(a));
    return r;
}
// Bilinear of the f16 channel HI of the words a, b (top row) and c, d (bottom row): fma(w, b - a, a) per lerp, the
// horizontal ones straight from the halves (two v_fma_mix_f32 each), the vertical one in fp32
template <int HI>
__device__ __forceinline__ float bilerp_h(uint32_t a, uint32_t b, uint32_t c, uint32_t d, float wx, float wy) {
    const float top = __builtin_fmaf(wx, sub_h<HI>(b, a), half_f<HI>(a));
    const float bot = __builtin_fmaf(wx, sub_h<HI>(d, c), half_f<HI>(c));
    return __builtin_fmaf(wy, bot - top, top);
}
// 4 x (1/4 a + 1/2 b + 1/4 c) of two f16 channels, fp32: c + (2 b + a), two v_fma_mix_f32 straight from the packed
// halves. The bits of 4 x fma(c, 1/4, fma(b, 1/2, a / 4)) (round 5's form, one conversion and one multiply more):
// scaling by a power of two commutes with each rounding (f16 inputs: no fp32 underflow or overflow), zeros' signs too.
__device__ __forceinline__ v2f gauss_col4(h2 a, h2 b, h2 c) {
    return v2f{(float)c.x + __builtin_fmaf((float)b.x, 2.0f, (float)a.x), (float)c.y + __builtin_fmaf((float)b.y, 2.0f, (float)a.y)};
}

// Same per-pixel result as taa_fast within the RGBA16F tolerance: the neighbourhood min/max run on
// packed f16 (exact), column-wise and shared by the two pixels; the 3x3 Gaussian is evaluated as
// column sums (separable weights, different rounding order); the closest-depth texel is chosen with
// the reference's iteration order and tie rule, exactly.
// Fused ToneMappingTask (tone_mapping.inl:145-176) epilogue: the resolved RGBA16F pair, exactly as it
// is stored, goes through the same AgX device function as tonemap_pair into an RGBA8_UNORM image.
struct TmOut {
    DImg out;
    const soc_auto_exposure* ae;
    TmParams p;
    int srgb;   // RGBA8_SRGB framebuffer: sRGB-encode on store
};

// The history taps of pixel k of the pair (0: colour, 1: velocity): the texel pairs (i0, i0 + 1) of rows ay.i0 and
// ay.i1, one 16-B load per row.
// The velocity history needs only the RG words of its two texels (words 0 and 2 of the pair): a 12-byte load (the
// pair's first 12 bytes, in bounds: the texel i0 + 1 exists) instead of 16 moves a quarter fewer bytes through the
// texture data path, this kernel's bound (TD busy 0.86, profiles/r04_raster_frame_sq_counters.json).
#ifndef SOC_TAA_PVEL12
#define SOC_TAA_PVEL12 1
#endif
typedef uint32_t u3a4 __attribute__((ext_vector_type(3))) __attribute__((aligned(4)));
#ifndef SOC_TAA_HIST_PAIR
#define SOC_TAA_HIST_PAIR 1
#endif
// The history images as buffer resources with 32-bit row offsets (one v_mad_u32_u24 per row address instead of the
// 64-bit pointer arithmetic: the launch checks that every image of the pair path fits the offset range, buf_ok).
struct HistLoad {
    const DImg& prev;
    const DImg& pvel;
    __device__ __forceinline__ void operator()(int, int which, const Axis& ax, const Axis& ay, u4a8& r0, u4a8& r1) const {
        if (SOC_TAA_PVEL12 && which) {
            const u3a4 a = *reinterpret_cast<const u3a4*>(row_ptr<uint2>(pvel, ay.i0) + ax.i0);
            const u3a4 b = *reinterpret_cast<const u3a4*>(row_ptr<uint2>(pvel, ay.i1) + ax.i0);
            r0 = u4a8{a.x, a.y, a.z, 0u};
            r1 = u4a8{b.x, b.y, b.z, 0u};
            return;
        }
        const DImg& im = which ? pvel : prev;
        r0 = *reinterpret_cast<const u4a8*>(row_ptr<uint2>(im, ay.i0) + ax.i0);
        r1 = *reinterpret_cast<const u4a8*>(row_ptr<uint2>(im, ay.i1) + ax.i0);
    }
    // Both pixels of the pair on the same history rows with adjacent footprints (texels i0, i0 + 1 and i0 + 1, i0 + 2):
    // the three texels of each row in one 16-B + one 8-B load (colour) or one 16-B + one 4-B load (velocity RG words),
    // instead of two 16-B (two 12-B) loads. The same texels.
    // (Global loads: the same loads through a buffer resource with 32-bit offsets, 8 fewer VALU address operations,
    // made the kernel ~4 % slower, DESIGN.md §11 r6.14: these scattered 16-B gathers cost more in the texture-address
    // path as MUBUF loads.)
    __device__ __forceinline__ void pair(int which, const Axis& ax, const Axis& ay, u4a8 (&r0)[2], u4a8 (&r1)[2]) const {
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            const int row = r ? ay.i1 : ay.i0;
            u4a8 a, b;
            if (which) {
                const uint32_t* w = reinterpret_cast<const uint32_t*>(row_ptr<uint2>(pvel, row) + ax.i0);
                const u3a4 q = *reinterpret_cast<const u3a4*>(w);   // words 0..2 (the RG words are 0, 2, 4): 12 B, not 16
                const uint32_t w4 = w[4];
                a = u4a8{q.x, q.y, q.z, 0u};
                b = u4a8{q.z, 0u, w4, 0u};
            } else {
                const uint2* t = row_ptr<uint2>(prev, row) + ax.i0;
                const u4a8 q = *reinterpret_cast<const u4a8*>(t);
                const uint2 t2 = t[2];
                a = q;
                b = u4a8{q.z, q.w, t2.x, t2.y};
            }
            if (r) { r1[0] = a; r1[1] = b; } else { r0[0] = a; r0[1] = b; }
        }
    }
};
// The part of the pair kernels after the neighbourhood is loaded (:156-189 and the fused tone map): column min / max,
// Gaussian column sums, the closest-depth texel, the history resolve and the stores. Cxy / Czw / D: the 3 x 4
// neighbourhood (rows y+1, y, y-1; columns xl, x0, x0+1, xr); Sel::off(r, c): neighbourhood tap (r, c) as the
// compile-time constant the closest-depth selection carries, vel(sel): the RG word of that tap's current velocity texel;
// own_vel(): the lane's own velocity pair (the fused velocity-history copy); hist: the history row loads (HistLoad).
template <bool TM, class Sel, class VelAt, class OwnVel, class Hist>
__device__ __forceinline__ void taa_pair_tail(const DImg& target, const DImg& prev, const DImg& pvel, const DImg& vel_out,
                                              const TaaParams& p, const TmOut& tm, int x0, int y,
                                              const h2 (&Cxy)[3][4], const h2 (&Czw)[3][4], const float (&D)[3][4],
                                              float exposure, const VelAt& vel, const OwnVel& own_vel, const Hist& hist) {
    const int W = target.w, H = target.h;
    const float v = centre_uv_rn(y, H, p.rh);
    uint2 outp[2];
    // closest depth in the reference order (oy = +1..-1, ox = +1..-1, from 1.0), last equal wins. The running form takes
    // a tap iff it is <= every earlier tap (and 1.0); the last such tap is the last one equal to the minimum over all
    // nine and 1.0, and no tap is taken iff that minimum is the 1.0 no tap equals. So: the minimum first (min3 chains;
    // the six taps of the two shared columns once for the pair), then one compare + select per tap.
    const float dshared = fminf(fminf(fminf(D[0][1], D[0][2]), fminf(D[1][1], D[1][2])), fminf(D[2][1], D[2][2]));
    const float dmin[2] = {fminf(fminf(fminf(D[0][0], D[1][0]), fminf(D[2][0], 1.0f)), dshared),
                           fminf(fminf(fminf(D[0][3], D[1][3]), fminf(D[2][3], 1.0f)), dshared)};
    // per pixel: the closest-depth velocity and the history footprint; then the history loads of the pair (combined
    // when the footprints are adjacent on the same rows, SOC_TAA_HIST_PAIR); then the resolve
    float velx_[2], vely_[2], vx_[2], vy_[2];
    Axis hax_[2], hay_[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const int x = x0 + k;
        const float u = centre_uv_rn(x, W, p.rw);
        int sel = Sel::off(1, k + 1);   // the centre tap when no tap is taken
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int ox = 1; ox > -2; --ox) {
                const int c = k + 1 + ox;
                sel = D[r][c] == dmin[k] ? Sel::off(r, c) : sel;
            }
        const uint32_t vv = vel(sel);
        velx_[k] = half_f<0>(vv);
        vely_[k] = half_f<1>(vv);
        vx_[k] = u - velx_[k];
        vy_[k] = v - vely_[k];
        hax_[k] = axis_clamp(vx_[k], prev.w);   // prev and pvel: same extent
        hay_[k] = axis_clamp(vy_[k], prev.h);
    }
    u4a8 ch0[2], ch1[2], vh0[2], vh1[2];
    if (SOC_TAA_HIST_PAIR && hay_[0].i0 == hay_[1].i0 && hax_[1].i0 == hax_[0].i0 + 1) {
        hist.pair(0, hax_[0], hay_[0], ch0, ch1);
        hist.pair(1, hax_[0], hay_[0], vh0, vh1);
    } else {
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            hist(k, 0, hax_[k], hay_[k], ch0[k], ch1[k]);
            hist(k, 1, hax_[k], hay_[k], vh0[k], vh1[k]);
        }
    }
    // column min / max (packed f16) and Gaussian column sums (fp32), while the history loads are in flight (round 6:
    // they depend on the closest-depth velocity, so issuing them first leaves this arithmetic to cover their latency;
    // the same operations). The min / max as IEEE minimum / maximum of three: one v_pk_minimum3_f16 / v_pk_maximum3_f16
    // (gfx950) where min / max take two v_pk_min_f16 / v_pk_max_f16; the same values (the file is built without NaNs;
    // -0 orders below +0, which min may not: a zero's sign in the clamp bounds at most).
    h2 nxy[4], nzw[4], xxy[4], xzw[4];
    v2f sxy[4], szw[4];   // 4 x the Gaussian column sums
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        nxy[c] = __builtin_elementwise_minimum(__builtin_elementwise_minimum(Cxy[0][c], Cxy[1][c]), Cxy[2][c]);
        nzw[c] = __builtin_elementwise_minimum(__builtin_elementwise_minimum(Czw[0][c], Czw[1][c]), Czw[2][c]);
        xxy[c] = __builtin_elementwise_maximum(__builtin_elementwise_maximum(Cxy[0][c], Cxy[1][c]), Cxy[2][c]);
        xzw[c] = __builtin_elementwise_maximum(__builtin_elementwise_maximum(Czw[0][c], Czw[1][c]), Czw[2][c]);
        sxy[c] = gauss_col4(Cxy[0][c], Cxy[1][c], Cxy[2][c]);
        szw[c] = gauss_col4(Czw[0][c], Czw[1][c], Czw[2][c]);
    }
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const h2 mnxy = __builtin_elementwise_minimum(__builtin_elementwise_minimum(nxy[k], nxy[k + 1]), nxy[k + 2]);
        const h2 mnzw = __builtin_elementwise_minimum(__builtin_elementwise_minimum(nzw[k], nzw[k + 1]), nzw[k + 2]);
        const h2 mxxy = __builtin_elementwise_maximum(__builtin_elementwise_maximum(xxy[k], xxy[k + 1]), xxy[k + 2]);
        const h2 mxzw = __builtin_elementwise_maximum(__builtin_elementwise_maximum(xzw[k], xzw[k + 1]), xzw[k + 2]);
        // 16 x the blurred colour: (s2 + (2 s1 + s0)) of the 4x column sums, whose 1/16 is taken exactly in (b - o) below
        // (round 5: fma(s2, 1/4, fma(s1, 1/2, s0 / 4)) of the column sums; the same bits, see gauss_col4)
        const v2f two = v2f{2.0f, 2.0f};
        const v2f bxy = __builtin_elementwise_fma(sxy[k + 1], two, sxy[k]) + sxy[k + 2];
        const v2f bzw = __builtin_elementwise_fma(szw[k + 1], two, szw[k]) + szw[k + 2];
        const uint32_t cxy = __builtin_bit_cast(uint32_t, Cxy[1][k + 2]), czw = __builtin_bit_cast(uint32_t, Czw[1][k + 2]);
        // quirk Q7: the (+1, 0) neighbour is "the" colour
        const float velx = velx_[k], vely = vely_[k];
        // resolve (:172-189)
        float accum = p.accum0;
        const float vx = vx_[k], vy = vy_[k];
        const Axis hax = hax_[k], hay = hay_[k];
        float a4[4], pv[2];
        u4a8 h0 = ch0[k], h1 = ch1[k];
        a4[0] = bilerp_h<0>(h0.x, h0.z, h1.x, h1.z, hax.w, hay.w);
        a4[1] = bilerp_h<1>(h0.x, h0.z, h1.x, h1.z, hax.w, hay.w);
        a4[2] = bilerp_h<0>(h0.y, h0.w, h1.y, h1.w, hax.w, hay.w);
        a4[3] = bilerp_h<1>(h0.y, h0.w, h1.y, h1.w, hax.w, hay.w);
        if (vx < 0.0f || vy < 0.0f || vx > 1.0f || vy > 1.0f) accum = 1.0f;
        // clamp to the neighbourhood's [min, max] (min <= max: one v_med3 per channel)
        const uint32_t mn[2] = {__builtin_bit_cast(uint32_t, mnxy), __builtin_bit_cast(uint32_t, mnzw)};
        const uint32_t mx[2] = {__builtin_bit_cast(uint32_t, mxxy), __builtin_bit_cast(uint32_t, mxzw)};
        a4[0] = __builtin_amdgcn_fmed3f(a4[0], half_f<0>(mn[0]), half_f<0>(mx[0]));
        a4[1] = __builtin_amdgcn_fmed3f(a4[1], half_f<1>(mn[0]), half_f<1>(mx[0]));
        a4[2] = __builtin_amdgcn_fmed3f(a4[2], half_f<0>(mn[1]), half_f<0>(mx[1]));
        a4[3] = __builtin_amdgcn_fmed3f(a4[3], half_f<1>(mn[1]), half_f<1>(mx[1]));
        const float ic = 1.0f - accum;
        const v2f oxy = v2f{__builtin_fmaf(half_f<0>(cxy), accum, a4[0] * ic), __builtin_fmaf(half_f<1>(cxy), accum, a4[1] * ic)};
        const v2f ozw = v2f{__builtin_fmaf(half_f<0>(czw), accum, a4[2] * ic), __builtin_fmaf(half_f<1>(czw), accum, a4[3] * ic)};
        h0 = vh0[k];
        h1 = vh1[k];
        pv[0] = bilerp_h<0>(h0.x, h0.z, h1.x, h1.z, hax.w, hay.w);
        pv[1] = bilerp_h<1>(h0.x, h0.z, h1.x, h1.z, hax.w, hay.w);
        const float dvx = pv[0] - velx, dvy = pv[1] - vely;
        const float vlen = __builtin_amdgcn_sqrtf(__builtin_fmaf(dvx, dvx, dvy * dvy));
        const float dis = clampf((vlen - 0.001f) * 10.0f, 0.0f, 1.0f);
        const v2f dd = v2f{dis, dis};
        const v2f sixteenth = v2f{0.0625f, 0.0625f};
        const v2f rxy = __builtin_elementwise_fma(__builtin_elementwise_fma(bxy, sixteenth, -oxy), dd, oxy),
                  rzw = __builtin_elementwise_fma(__builtin_elementwise_fma(bzw, sixteenth, -ozw), dd, ozw);
        outp[k] = pack_h4(f4{rxy.x, rxy.y, rzw.x, rzw.y});
    }
    row_ptr_w<uint4>(target, y)[x0 >> 1] = uint4{outp[0].x, outp[0].y, outp[1].x, outp[1].y};
    if (vel_out.data) row_ptr_w<uint4>(vel_out, y)[x0 >> 1] = own_vel();
    if (TM) {
        const float expo = exp2f(exposure);   // pow(2.0, exposure)
        f3 c0 = agx(tm.p, unpack_h4(outp[0]), expo);
        f3 c1 = agx(tm.p, unpack_h4(outp[1]), expo);
        if (tm.srgb) {
            c0 = f3{srgb_encode(c0.x), srgb_encode(c0.y), srgb_encode(c0.z)};
            c1 = f3{srgb_encode(c1.x), srgb_encode(c1.y), srgb_encode(c1.z)};
        }
        row_ptr_w<uint2>(tm.out, y)[x0 >> 1] =
            uint2{pack_unorm8x4(f4{c0.x, c0.y, c0.z, 1.0f}), pack_unorm8x4(f4{c1.x, c1.y, c1.z, 1.0f})};
    }
}

// The closest-depth tap as r * 4 + c (taa_pair2: the row and column are looked up from it).
struct SelRC {
    static constexpr int off(int r, int c) { return r * 4 + c; }
};

// Lane i's left neighbour column (x0 - 1) is lane i-1's second pixel and its right one (x0 + 2) lane
// i+1's first: with NBR the neighbourhood's side columns come from the adjacent lanes through DPP wave
// shifts (VALU) instead of two more colour and two more depth loads per row, and only the lanes at a
// block-row edge (threadIdx.x == 0 / blockDim.x - 1) or at the image border load them. The texture path
// is the bound of this kernel (TA / TD ~83 % busy, profiles/r01_l1_counters.json).
__device__ __forceinline__ uint32_t from_left(uint32_t v) {   // lane i <- lane i-1 (wave_shr:1)
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t from_right(uint32_t v) {  // lane i <- lane i+1 (wave_shl:1)
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x130, 0xf, 0xf, false);
}

// NBR = 2 (default): 64-lane block rows whose first and last lanes only load the halo pairs for their
// neighbours (62 output pairs per wave), so no lane issues a side-column load at all: the kernel is bound
// by texture-path instructions, not bytes.
template <bool TM, int NBR = 2>
__global__ __launch_bounds__(kWorkgroup) void taa_pair2(DImg target, DImg cur, DImg prev, DImg vel, DImg pvel, DImg depth,
                                                 DImg vel_out, TaaParams p, TmOut tm) {
    int tbx, tby;
    xcd_order(p.swz, tbx, tby);
    const int x0 = NBR == 2 ? (tbx * 62 + (int)threadIdx.x - 1) * 2 : (tbx * (int)blockDim.x + threadIdx.x) * 2;
    const int y = tby * (int)blockDim.y + threadIdx.y;
    const bool halo = NBR == 2 && (threadIdx.x == 0 || threadIdx.x == 63);
    // NBR: every lane stays for the lane shifts (the grid covers whole rows of lanes; W is even, so a lane
    // is either wholly inside or wholly outside the image)
    if ((!NBR && x0 >= target.w) || y >= target.h) return;
    const bool inside_x = !halo && x0 < target.w;
    const float exposure = TM ? tm.ae->exposure : 0.0f;
    const int W = target.w, H = target.h;
    const int xl = max(x0 - 1, 0), xr = min(x0 + 2, W - 1);
    // slots c = 0..3: columns xl, x0, x0+1, xr; rows r = 0..2: y+1, y, y-1 (clamped)
    h2 Cxy[3][4], Czw[3][4];
    float D[3][4];
    int rows[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        const int sy = min(max(y + 1 - r, 0), H - 1);
        rows[r] = sy;
        const uint2* crow = row_ptr<uint2>(cur, sy);
        const float* drow = row_ptr<float>(depth, sy);
        const int xm = NBR ? min(max(x0, 0), W - 2) : x0;
        const uint4 mid = *reinterpret_cast<const uint4*>(crow + xm);
        const float2 dmid = *reinterpret_cast<const float2*>(drow + xm);
        uint2 L, R;
        float dl, dr;
        if (NBR) {
            L = uint2{from_left(mid.z), from_left(mid.w)};
            R = uint2{from_right(mid.x), from_right(mid.y)};
            dl = __builtin_bit_cast(float, from_left(__builtin_bit_cast(uint32_t, dmid.y)));
            dr = __builtin_bit_cast(float, from_right(__builtin_bit_cast(uint32_t, dmid.x)));
            if (NBR == 2) {   // image borders: the clamped side column is the pair's own pixel
                if (x0 == 0) { L = uint2{mid.x, mid.y}; dl = dmid.x; }
                if (x0 + 2 >= W) { R = uint2{mid.z, mid.w}; dr = dmid.y; }
            } else {
                if (threadIdx.x == 0) { L = crow[xl]; dl = drow[xl]; }
                if (threadIdx.x == blockDim.x - 1 || x0 + 2 >= W) { R = crow[xr]; dr = drow[xr]; }
            }
        } else {
            L = crow[xl];
            R = crow[xr];
            dl = drow[xl];
            dr = drow[xr];
        }
        Cxy[r][0] = as_h2(L.x);
        Czw[r][0] = as_h2(L.y);
        Cxy[r][1] = as_h2(mid.x);
        Czw[r][1] = as_h2(mid.y);
        Cxy[r][2] = as_h2(mid.z);
        Czw[r][2] = as_h2(mid.w);
        Cxy[r][3] = as_h2(R.x);
        Czw[r][3] = as_h2(R.y);
        D[r][0] = dl;
        D[r][1] = dmid.x;
        D[r][2] = dmid.y;
        D[r][3] = dr;
    }
    if (NBR && !inside_x) return;   // past the image: only fed its neighbours' shifts
    const int colx[4] = {xl, x0, x0 + 1, xr};
    taa_pair_tail<TM, SelRC>(target, prev, pvel, vel_out, p, tm, x0, y, Cxy, Czw, D, exposure,
                             [&](int s) { return row_ptr<uint32_t>(vel, rows[s >> 2])[2 * colx[s & 3]]; },
                             [&]() { return row_ptr<uint4>(vel, y)[x0 >> 1]; }, HistLoad{prev, pvel});
}

// LDS-staged neighbourhood: a workgroup of 64 x 4 lanes (128 x 4 output pixels, a pixel pair per lane) stages the
// colour and velocity pairs and the depth quads of its 6 rows (y0 - 1 .. y0 + 4, clamped) and 2 + 128 + 2 columns with
// 16-B loads, once; every lane then reads its 3 x 4 neighbourhood, its closest-depth velocity texel and its own
// velocity pair (the fused history copy) from LDS. Per lane about 4 staging loads instead of 9 neighbourhood, velocity
// and copy loads (the texture path is the kernel's bound), and the velocity gather no longer waits on a load level.
// The same values reach the same arithmetic (taa_pair_tail) as taa_pair2: the same bits.
constexpr int kTaaPairs = 64;                                     // output pairs per workgroup row
constexpr int kTaaTP = kTaaPairs + 2;                             // staged pairs (pair p0 - 1 .. p0 + 64)
constexpr int kTaaTQ = kTaaPairs / 2 + 2;                         // staged depth quads (quad q0 - 1 .. q0 + 32)

constexpr int kTaaLdsRows = 4;                                   // rows per workgroup: 4 measured against 2 and 8
constexpr int kTaaLdsLanes = 64 * kTaaLdsRows;                    // (profiles/r03_ab_taa_lds.txt); the launch bound
// Image-border copies in the tiles: the staged pair left of the image holds texel 0 twice and the one right of it texel
// W - 1 twice, the depth quads likewise (and the last quad of a row with W % 4 == 2 has texel W - 1 at column W), so the
// lanes at a border read their clamped side columns and closest-depth velocity texels from the tiles like every other
// lane: no per-lane border selects (round 5: 18 per lane). Applied in the border workgroups only (a uniform branch).
__device__ __forceinline__ uint4 border_pair(uint4 v, int p, int npairs) {
    if (p < 0) return uint4{v.x, v.y, v.x, v.y};            // v: pair 0 (the clamped staging)
    if (p >= npairs) return uint4{v.z, v.w, v.z, v.w};      // v: pair npairs - 1
    return v;
}
__device__ __forceinline__ float4 border_quad(float4 d, int q, int nquads, int W) {
    if (q < 0) return float4{d.x, d.x, d.x, d.x};
    if (q >= nquads) return float4{d.w, d.w, d.w, d.w};     // read only when W % 4 == 0: d.w is texel W - 1
    if (4 * q + 2 == W) d.z = d.y;
    return d;
}
// The closest-depth tap (r, c) as its word offset in the velocity tile from the lane's (ty, pl) base: tile row ty + 2 - r,
// column c = 0..3 at pair pl word 2, pair pl + 1 words 0 / 2, pair pl + 2 word 0 (the RG word of the texel).
struct SelTile {
    static constexpr int off(int r, int c) { return (2 - r) * kTaaTP * 4 + 2 * c; }
};

// SF (SOC_TAA_NBR=4, default): every staging load of a lane is issued before its first LDS store, so the staging costs
// one memory latency instead of one per loop round (2 colour / velocity rounds and a depth round); the same values.
#ifndef SOC_TAA_WAVES_PER_EU
#define SOC_TAA_WAVES_PER_EU 0   // A/B builds: a VGPR budget for taa_lds (0: the compiler's choice, 86 VGPRs = 5 waves)
#endif
template <bool TM, int kTaaRows = kTaaLdsRows, bool SF = false>
__global__ __launch_bounds__(64 * kTaaRows)
#if SOC_TAA_WAVES_PER_EU
__attribute__((amdgpu_waves_per_eu(SOC_TAA_WAVES_PER_EU)))
#endif
void taa_lds(DImg target, DImg cur, DImg prev, DImg vel, DImg pvel, DImg depth,
                                                         DImg vel_out, TaaParams p, TmOut tm) {
    constexpr int kTaaTR = kTaaRows + 2, NT = 64 * kTaaRows;   // staged rows y0 - 1 .. y0 + kTaaRows
    __shared__ uint4 ct[kTaaTR][kTaaTP];   // colour pairs
    __shared__ uint4 vt[kTaaTR][kTaaTP];   // velocity pairs
    __shared__ float4 dt[kTaaTR][kTaaTQ];  // depth quads
    int tbx, tby;
    xcd_order(p.swz, tbx, tby);
    const int W = target.w, H = target.h;
    const int tid = threadIdx.x + threadIdx.y * 64;
    const int p0 = tbx * kTaaPairs, y0 = tby * kTaaRows, q0 = tbx * (kTaaPairs / 2);
    const int npairs = W >> 1, nquads = (W + 3) >> 2;
    // staging: rows clamped into the image, pairs / quads clamped into the row (border_pair / border_quad)
    const bool edge = p0 == 0 || 2 * (p0 + kTaaTP) + 8 >= W;   // the tiles reach an image border
    auto depth_quad = [&](int i) {
        const int r = i / kTaaTQ, c = i - r * kTaaTQ;
        const int sy = min(max(y0 - 1 + r, 0), H - 1), sq = min(max(q0 - 1 + c, 0), nquads - 1);
        const float* drow = row_ptr<float>(depth, sy);
        if (4 * sq + 3 < W) return *reinterpret_cast<const float4*>(drow + 4 * sq);
        return float4{drow[4 * sq], drow[min(4 * sq + 1, W - 1)], drow[min(4 * sq + 2, W - 1)], drow[min(4 * sq + 3, W - 1)]};
    };
    if constexpr (SF) {
        constexpr int NP = kTaaTR * kTaaTP, ND = kTaaTR * kTaaTQ;
        static_assert(NP > NT && NP <= 2 * NT && ND <= NT, "two colour / velocity rounds and one depth round");
        // 32-bit byte offsets from the image bases (the launch checks their range: buf_ok)
        auto pair_off = [&](int i, int& r, int& c, int& oc, int& ov) {
            r = i / kTaaTP;
            c = i - r * kTaaTP;
            const int sy = min(max(y0 - 1 + r, 0), H - 1), sp = min(max(p0 - 1 + c, 0), npairs - 1);
            oc = __mul24(sy, cur.pitch) + sp * 16;
            ov = __mul24(sy, vel.pitch) + sp * 16;
        };
        auto ldc = [&](int o) { return *reinterpret_cast<const uint4*>(cur.data + o); };
        auto ldv = [&](int o) { return *reinterpret_cast<const uint4*>(vel.data + o); };
        int r0, c0, r1, c1, oc0, ov0, oc1, ov1;
        pair_off(tid, r0, c0, oc0, ov0);
        const bool second = tid + NT < NP, hasd = tid < ND;
        pair_off(second ? tid + NT : tid, r1, c1, oc1, ov1);
        uint4 ca = ldc(oc0), va = ldv(ov0);
        uint4 cb, vb;   // set and stored only when second
        if (second) { cb = ldc(oc1); vb = ldv(ov1); }
        // the depth quad as one 16-B buffer load even for the last quad of a row with W % 4 != 0: its texels past the
        // row end (the next row's, or 0 past the image) are never read (the border columns come from the pair itself)
        float4 dq;   // set and stored only when hasd
        if (hasd) {
            const int r = tid / kTaaTQ, c = tid - r * kTaaTQ;
            const int sy = min(max(y0 - 1 + r, 0), H - 1), sq = min(max(q0 - 1 + c, 0), nquads - 1);
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(depth.data, 0, depth.pitch * depth.h, 0x00020000);
            const auto w = __builtin_amdgcn_raw_buffer_load_b128(rs, __mul24(sy, depth.pitch) + 16 * sq, 0, 0);
            dq = make_float4(__uint_as_float(w[0]), __uint_as_float(w[1]), __uint_as_float(w[2]), __uint_as_float(w[3]));
        }
        if (edge) {
            ca = border_pair(ca, p0 - 1 + c0, npairs);
            va = border_pair(va, p0 - 1 + c0, npairs);
            if (second) {
                cb = border_pair(cb, p0 - 1 + c1, npairs);
                vb = border_pair(vb, p0 - 1 + c1, npairs);
            }
            if (hasd) dq = border_quad(dq, q0 - 1 + tid % kTaaTQ, nquads, W);
        }
        ct[r0][c0] = ca;
        vt[r0][c0] = va;
        if (second) { ct[r1][c1] = cb; vt[r1][c1] = vb; }
        if (hasd) dt[tid / kTaaTQ][tid % kTaaTQ] = dq;
    } else {
        for (int i = tid; i < kTaaTR * kTaaTP; i += NT) {
            const int r = i / kTaaTP, c = i - r * kTaaTP;
            const int sy = min(max(y0 - 1 + r, 0), H - 1), sp = min(max(p0 - 1 + c, 0), npairs - 1);
            uint4 cv = row_ptr<uint4>(cur, sy)[sp], vv = row_ptr<uint4>(vel, sy)[sp];
            if (edge) {
                cv = border_pair(cv, p0 - 1 + c, npairs);
                vv = border_pair(vv, p0 - 1 + c, npairs);
            }
            ct[r][c] = cv;
            vt[r][c] = vv;
        }
        for (int i = tid; i < kTaaTR * kTaaTQ; i += NT) {
            const int r = i / kTaaTQ, c = i - r * kTaaTQ;
            float4 dq = depth_quad(i);
            if (edge) dq = border_quad(dq, q0 - 1 + c, nquads, W);
            dt[r][c] = dq;
        }
    }
    __syncthreads();
    const int pl = threadIdx.x, ty = threadIdx.y;
    const int x0 = 2 * (p0 + pl), y = y0 + ty;
    if (x0 >= W || y >= H) return;
    const float* dtf = reinterpret_cast<const float*>(dt);
    const int dbase = 4 * (q0 - 1);   // image column of dtf[r * 4 * kTaaTQ + 0]
    h2 Cxy[3][4], Czw[3][4];
    float D[3][4];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        const int tr = ty + 2 - r;   // tile row of image row y + 1 - r (clamped)
        const uint4 mid = ct[tr][pl + 1];
        const uint2 L = uint2{ct[tr][pl].z, ct[tr][pl].w}, R = uint2{ct[tr][pl + 2].x, ct[tr][pl + 2].y};   // border copies
        const float* drow = dtf + tr * 4 * kTaaTQ - dbase;
        const float2 dmid = *reinterpret_cast<const float2*>(drow + x0);
        const float dl = drow[x0 - 1], dr = drow[x0 + 2];
        Cxy[r][0] = as_h2(L.x);
        Czw[r][0] = as_h2(L.y);
        Cxy[r][1] = as_h2(mid.x);
        Czw[r][1] = as_h2(mid.y);
        Cxy[r][2] = as_h2(mid.z);
        Czw[r][2] = as_h2(mid.w);
        Cxy[r][3] = as_h2(R.x);
        Czw[r][3] = as_h2(R.y);
        D[r][0] = dl;
        D[r][1] = dmid.x;
        D[r][2] = dmid.y;
        D[r][3] = dr;
    }
    const float exposure = TM ? tm.ae->exposure : 0.0f;
    const uint32_t* vtw = reinterpret_cast<const uint32_t*>(vt);
    const int vbase = (ty * kTaaTP + pl) * 4 + 2;
    taa_pair_tail<TM, SelTile>(target, prev, pvel, vel_out, p, tm, x0, y, Cxy, Czw, D, exposure,
                               [&](int s) { return vtw[vbase + s]; },
                               [&]() { return vt[ty + 1][pl + 1]; }, HistLoad{prev, pvel});
}

__global__ __launch_bounds__(kWorkgroup) void taa_generic(DImg target, DImg cur, DImg prev, DImg vel, DImg pvel, DImg depth,
                                                   DImg vel_out, TaaParams p) {
    const int x = blockIdx.x * BX + threadIdx.x, y = blockIdx.y * BY + threadIdx.y;
    if (x >= target.w || y >= target.h) return;
    const float u = centre_uv(x, target.w), v = centre_uv(y, target.h);
    f4 nb5 = f4{0, 0, 0, 0}, blurred = f4{0, 0, 0, 0};
    f4 mn = f4{10.0e5f, 10.0e5f, 10.0e5f, 10.0e5f}, mx = f4{-10.0e5f, -10.0e5f, -10.0e5f, -10.0e5f};
    float closest = 1.0f, du = u, dv = v;
    for (int oy = 1; oy > -2; --oy)
        for (int ox = 1; ox > -2; --ox) {
            const int idx = (oy + 1) * 3 + (ox + 1);
            const float su = u + p.pox * (float)ox, sv = v + p.poy * (float)oy;
            const f4 c = sample_h4(cur, su, sv);
            const float d = sample_f32(depth, su, sv);
            closest = fminf(d, closest);
            if (closest == d) { du = su; dv = sv; }
            mn = min4(c, mn);
            mx = max4(c, mx);
            const float gw = gauss_w(idx);
            blurred = f4{blurred.x + gw * c.x, blurred.y + gw * c.y, blurred.z + gw * c.z, blurred.w + gw * c.w};
            if (idx == 5) nb5 = c;
        }
    const f4 vv = sample_h4(vel, du, dv);
    const f4 o = resolve(p, u, v, nb5, mn, mx, blurred, float2{vv.x, vv.y}, prev, pvel);
    row_ptr_w<uint2>(target, y)[x] = pack_h4(o);
    if (vel_out.data && x < vel.w && y < vel.h) row_ptr_w<uint2>(vel_out, y)[x] = row_ptr<uint2>(vel, y)[x];
}

__global__ __launch_bounds__(kWorkgroup) void copy_rows(const char* __restrict__ src, int spitch, char* __restrict__ dst,
                                                 int dpitch, int row_bytes, int rows) {
    const int y = blockIdx.y;
    if (y >= rows) return;
    const char* s = src + (size_t)y * spitch;
    char* d = dst + (size_t)y * dpitch;
    for (int i = (blockIdx.x * 256 + threadIdx.x) * 16; i < row_bytes; i += gridDim.x * 256 * 16) {
        if (i + 16 <= row_bytes)
            *reinterpret_cast<uint4*>(d + i) = *reinterpret_cast<const uint4*>(s + i);
        else
            for (int k = i; k < row_bytes; ++k) d[k] = s[k];
    }
}

}  // namespace
}  // namespace soc

using namespace soc;

namespace {
// tm != nullptr: launch the fused TAA + tone-map kernel if the pair path applies (returns 1 otherwise,
// having launched nothing)
int taa_launch(const soc_globals* g, soc_img target, soc_img current_color, soc_img previous_color, soc_img current_velocity,
               soc_img previous_velocity, soc_img depth, soc_img velocity_history_out, const TmOut* tm, soc_stream stream) {
    static const char* P = "soc_temporal_antialiasing";
    if (!g) return set_error(SOC_E_INVALID_ARG, "%s: null globals", P);
    int rc = check_img(target, SOC_FMT_RGBA16F, P, "target");
    if (!rc) rc = check_img(current_color, SOC_FMT_RGBA16F, P, "current_color");
    if (!rc) rc = check_img(previous_color, SOC_FMT_RGBA16F, P, "previous_color");
    if (!rc) rc = check_img(current_velocity, SOC_FMT_RGBA16F, P, "current_velocity");
    if (!rc) rc = check_img(previous_velocity, SOC_FMT_RGBA16F, P, "previous_velocity");
    if (!rc) rc = check_img(depth, SOC_FMT_D32F, P, "depth");
    if (rc) return rc;
    if (target.data == current_color.data || target.data == previous_color.data)
        return set_error(SOC_E_INVALID_ARG, "%s: target aliases an input", P);
    if (velocity_history_out.data) {
        rc = check_img(velocity_history_out, SOC_FMT_RGBA16F, P, "velocity_history_out");
        if (rc) return rc;
        if (velocity_history_out.data == previous_velocity.data || velocity_history_out.data == current_velocity.data)
            return set_error(SOC_E_INVALID_ARG, "%s: velocity_history_out aliases a velocity input", P);
        if (velocity_history_out.width != current_velocity.width || velocity_history_out.height != current_velocity.height)
            return set_error(SOC_E_SHAPE, "%s: velocity_history_out extent != current_velocity extent", P);
    }
    TaaParams p;
    p.rw = recip_rn(target.width);
    p.rh = recip_rn(target.height);
    p.pox = 1.0f / (float)g->resolution[0];
    p.poy = 1.0f / (float)g->resolution[1];
    p.accum0 = fminf(0.1f, (float)g->frame_counter);
    p.swz = -16;   // XCD vertical bands of 16-tile strips: HBM traffic 1.39x -> 1.01x algorithmic
    const int W = target.width, H = target.height;
    auto same = [&](const soc_img& im) { return im.width == W && im.height == H; };
    const bool fast = W == g->resolution[0] && H == g->resolution[1] && same(current_color) && same(depth) &&
                      same(current_velocity) && W <= 8192 && H <= 8192;
    dim3 blk(BX, BY), grd(ceil_div(W, BX), ceil_div(H, BY));
    DImg vo = velocity_history_out.data ? dimg(velocity_history_out) : DImg{nullptr, 0, 0, 0};
    auto a16 = [](const soc_img& im) { return (reinterpret_cast<uintptr_t>(im.data) & 15u) == 0 && (im.pitch_bytes & 15) == 0; };
    // the pair kernels address the staged images (and the depth quads through a buffer resource) with 32-bit offsets
    // (a signed 24-bit row x pitch product)
    auto buf_ok = [](const soc_img& im) { return (long long)im.pitch_bytes * im.height < (1ll << 31) && im.pitch_bytes < (1 << 23); };
    const bool pair = fast && W % 2 == 0 && a16(target) && a16(current_color) && a16(current_velocity) &&
                      (reinterpret_cast<uintptr_t>(depth.data) & 7u) == 0 && (depth.pitch_bytes & 7) == 0 &&
                      (!velocity_history_out.data || a16(velocity_history_out)) && previous_color.width >= 2 &&
                      previous_velocity.width == previous_color.width && previous_velocity.height == previous_color.height &&
                      buf_ok(current_color) && buf_ok(current_velocity) && buf_ok(depth);
    if (tm && !pair) return 1;
    if (pair) {
        // 32 x 8 lanes (64 x 8 pixels): the 3-row neighbourhood reloads 10 rows per 8 instead of 6 per 4
        const int by = 8, bxl = 256 / by;
        dim3 blk(bxl, by), g2(ceil_div(W / 2, bxl), ceil_div(H, by));
        // neighbourhood source: 3 = LDS-staged tiles (default; needs a 16-B aligned depth image), 2 = halo lanes, 1 = lane
        // shifts + edge-lane loads, 0 = every lane loads its side columns (the same bits, tests/test_gpu_parity.py)
        const int nbr = tuning_knob("SOC_TAA_NBR", 4);
        const dim3 blk_h(64, 4), g2_h(ceil_div(W / 2, 62), ceil_div(H, 4));
        if (nbr == 4 && a16(depth)) {
            const dim3 gl(ceil_div(W / 2, kTaaPairs), ceil_div(H, 4));
            if (tm)
                launch("taa_lds", kTaaLdsLanes, taa_lds<true, kTaaLdsRows, true>, gl, blk_h, 0, hs(stream), dimg(target),
                       dimg(current_color), dimg(previous_color), dimg(current_velocity), dimg(previous_velocity), dimg(depth), vo,
                       p, *tm);
            else
                launch("taa_lds", kTaaLdsLanes, taa_lds<false, kTaaLdsRows, true>, gl, blk_h, 0, hs(stream), dimg(target),
                       dimg(current_color), dimg(previous_color), dimg(current_velocity), dimg(previous_velocity), dimg(depth), vo,
                       p, TmOut{});
        } else if (nbr == 3 && a16(depth)) {
            const dim3 gl(ceil_div(W / 2, kTaaPairs), ceil_div(H, 4));
            if (tm)
                launch("taa_lds", kTaaLdsLanes, taa_lds<true>, gl, blk_h, 0, hs(stream), dimg(target), dimg(current_color), dimg(previous_color),
                                                          dimg(current_velocity), dimg(previous_velocity), dimg(depth), vo, p, *tm);
            else
                launch("taa_lds", kTaaLdsLanes, taa_lds<false>, gl, blk_h, 0, hs(stream), dimg(target), dimg(current_color), dimg(previous_color),
                                                           dimg(current_velocity), dimg(previous_velocity), dimg(depth), vo, p,
                                                           TmOut{});
        } else if (tm && nbr >= 2)
            launch("taa_pair2", kWorkgroup, taa_pair2<true, 2>, g2_h, blk_h, 0, hs(stream), dimg(target), dimg(current_color), dimg(previous_color),
                                                       dimg(current_velocity), dimg(previous_velocity), dimg(depth), vo, p, *tm);
        else if (tm && nbr == 0)
            launch("taa_pair2", kWorkgroup, taa_pair2<true, 0>, g2, blk, 0, hs(stream), dimg(target), dimg(current_color), dimg(previous_color),
                                                       dimg(current_velocity), dimg(previous_velocity), dimg(depth), vo, p, *tm);
        else if (tm)
            launch("taa_pair2", kWorkgroup, taa_pair2<true, 1>, g2, blk, 0, hs(stream), dimg(target), dimg(current_color), dimg(previous_color),
                                                       dimg(current_velocity), dimg(previous_velocity), dimg(depth), vo, p, *tm);
        else
            launch("taa_pair2", kWorkgroup, taa_pair2<false, 2>, g2_h, blk_h, 0, hs(stream), dimg(target), dimg(current_color), dimg(previous_color),
                                                        dimg(current_velocity), dimg(previous_velocity), dimg(depth), vo, p,
                                                        TmOut{});
    } else if (fast)
        launch("taa_fast", kWorkgroup, taa_fast, grd, blk, 0, hs(stream), dimg(target), dimg(current_color), dimg(previous_color), dimg(current_velocity),
                                              dimg(previous_velocity), dimg(depth), vo, p);
    else
        launch("taa_generic", kWorkgroup, taa_generic, grd, blk, 0, hs(stream), dimg(target), dimg(current_color), dimg(previous_color),
                                                 dimg(current_velocity), dimg(previous_velocity), dimg(depth), vo, p);
    return check_launch("temporal_antialiasing");
}

}  // namespace

extern "C" int soc_temporal_antialiasing(const soc_globals* g, soc_img target, soc_img current_color, soc_img previous_color,
                                         soc_img current_velocity, soc_img previous_velocity, soc_img depth,
                                         soc_img velocity_history_out, soc_stream stream) {
    return taa_launch(g, target, current_color, previous_color, current_velocity, previous_velocity, depth,
                      velocity_history_out, nullptr, stream);
}

extern "C" int soc_temporal_antialiasing_tone_mapping(const soc_globals* g, soc_img target, soc_img current_color,
                                                      soc_img previous_color, soc_img current_velocity,
                                                      soc_img previous_velocity, soc_img depth, soc_img velocity_history_out,
                                                      const soc_auto_exposure* d_auto_exposure, soc_img output,
                                                      soc_stream stream) {
    static const char* P = "soc_temporal_antialiasing_tone_mapping";
    if (!g || !d_auto_exposure) return set_error(SOC_E_INVALID_ARG, "%s: null globals / auto exposure buffer", P);
    int rc = check_img(output, 0, P, "output");
    if (rc) return rc;
    const bool fusable = (output.format == SOC_FMT_RGBA8_UNORM || output.format == SOC_FMT_RGBA8_SRGB) &&
                         output.width == target.width &&
                         output.height == target.height && (reinterpret_cast<uintptr_t>(output.data) & 7u) == 0 &&
                         (output.pitch_bytes & 7) == 0 && output.data != target.data;
    if (fusable) {
        TmOut tm;
        tm.out = dimg(output);
        tm.ae = d_auto_exposure;
        tm.srgb = output.format == SOC_FMT_RGBA8_SRGB;
        agx_matrices(g->compression, tm.p.M.m, tm.p.Minv.m);
        tm.p.linear = g->agxDs_linear_section;
        tm.p.peak = g->peak;
        tm.p.saturation = g->saturation;
        tm_params_finish(tm.p);
        rc = taa_launch(g, target, current_color, previous_color, current_velocity, previous_velocity, depth,
                        velocity_history_out, &tm, stream);
        if (rc <= 0) return rc;   // launched (or failed validation)
    }
    // not fusable: the two passes back to back (same results)
    rc = taa_launch(g, target, current_color, previous_color, current_velocity, previous_velocity, depth,
                    velocity_history_out, nullptr, stream);
    if (rc) return rc;
    return soc_tone_mapping(g, target, d_auto_exposure, output, stream);
}

extern "C" int soc_copy_image(soc_img target, soc_img source, soc_stream stream) {
    int rc = check_img(target, 0, "soc_copy_image", "target");
    if (!rc) rc = check_img(source, 0, "soc_copy_image", "source");
    if (rc) return rc;
    if (target.format != source.format || target.width != source.width || target.height != source.height)
        return set_error(SOC_E_SHAPE, "soc_copy_image: format/extent mismatch");
    const int row_bytes = source.width * bytes_per_pixel(source.format);
    const bool vec = ((reinterpret_cast<uintptr_t>(source.data) | reinterpret_cast<uintptr_t>(target.data)) & 15u) == 0 &&
                     (source.pitch_bytes & 15) == 0 && (target.pitch_bytes & 15) == 0;
    if (!vec) {
        hipError_t e = hipMemcpy2DAsync(target.data, target.pitch_bytes, source.data, source.pitch_bytes, row_bytes,
                                        source.height, hipMemcpyDeviceToDevice, hs(stream));
        if (e != hipSuccess) return set_error(SOC_E_HIP, "soc_copy_image: %s", hipGetErrorString(e));
        return SOC_OK;
    }
    dim3 grd(ceil_div(ceil_div(row_bytes, 16), 256), source.height);
    launch("copy_rows", kWorkgroup, copy_rows, grd, kWorkgroup, 0, hs(stream), static_cast<const char*>(source.data), source.pitch_bytes,
                                           static_cast<char*>(target.data), target.pitch_bytes, row_bytes, source.height);
    return check_launch("copy_image");
}
