// bloom.hip — BloomDownsampleTask / BloomUpsampleTask (src/graphics/tasks/bloom_downsample.inl:107-141,
// bloom_upsample.inl:98-127) as gfx950 kernels.
//
// Every tap is a bilinear sample under the sampling contract. The 8-bit fixed-point tap coordinate
// `fx` is either derived from the float uv exactly as the oracle does (generic path) or, for the
// exact 1:1, 2:1 and 1:2 size ratios the reference's mip chain uses (renderer.cpp:492-513), written
// down analytically (fast paths); both then go through the same clamp rule and lerp arithmetic, so
// the fast paths are bit-identical to the generic one (extents <= 8192).
// All tap weights are powers of two, so the RGBA16F results are bit-identical to the oracle's.
#include <cstdlib>
#include <type_traits>

#include "bloom_common.hpp"

namespace soc {

namespace {

// ------------------------------------------------------------------------------------------------
// downsample
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kWorkgroup) void bloom_down_generic(DImg src, DImg dst, float sxt, float syt) {
    const int x = blockIdx.x * BX + threadIdx.x, y = blockIdx.y * BY + threadIdx.y;
    if (x >= dst.w || y >= dst.h) return;
    const float u = centre_uv(x, dst.w), v = centre_uv(y, dst.h);
    const float X = sxt, Y = syt;
    auto S = [&](float uu, float vv) {
        return tap(src, axis_from_fixed(fixed_from_uv(uu, src.w), src.w), axis_from_fixed(fixed_from_uv(vv, src.h), src.h));
    };
    f3 a = S(u - 2 * X, v + 2 * Y), b = S(u, v + 2 * Y), c = S(u + 2 * X, v + 2 * Y);
    f3 d = S(u - 2 * X, v), e = S(u, v), f = S(u + 2 * X, v);
    f3 g = S(u - 2 * X, v - 2 * Y), h = S(u, v - 2 * Y), i = S(u + 2 * X, v - 2 * Y);
    f3 j = S(u - X, v + Y), k = S(u + X, v + Y), l = S(u - X, v - Y), m = S(u + X, v - Y);
    store_rgb1(dst, x, y, SOC_DOWN13(a, b, c, d, e, f, g, h, i, j, k, l, m));
}

// ------------------------------------------------------------------------------------------------
// upsample (result overwrites the destination: quirk Q5)
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kWorkgroup) void bloom_up_generic(DImg src, DImg dst, float X, float Y) {
    const int x = blockIdx.x * BX + threadIdx.x, y = blockIdx.y * BY + threadIdx.y;
    if (x >= dst.w || y >= dst.h) return;
    const float u = centre_uv(x, dst.w), v = centre_uv(y, dst.h);
    auto S = [&](float uu, float vv) {
        return tap(src, axis_from_fixed(fixed_from_uv(uu, src.w), src.w), axis_from_fixed(fixed_from_uv(vv, src.h), src.h));
    };
    f3 a = S(u - X, v + Y), b = S(u, v + Y), c = S(u + X, v + Y);
    f3 d = S(u - X, v), e = S(u, v), f = S(u + X, v);
    f3 g = S(u - X, v - Y), h = S(u, v - Y), i = S(u + X, v - Y);
    store_rgb1(dst, x, y, SOC_UP9(a, b, c, d, e, f, g, h, i));
}

// dst is exactly twice src: the lower-mip coordinate of tap k is X/2 - 0.25 + k (weights 3/4, 1/4).
__global__ __launch_bounds__(kWorkgroup) void bloom_up_double(DImg src, DImg dst) {
    const int x = blockIdx.x * BX + threadIdx.x, y = blockIdx.y * BY + threadIdx.y;
    if (x >= dst.w || y >= dst.h) return;
    auto AX = [&](int k) { return axis_from_fixed(128 * x - 64 + 256 * k, src.w); };
    auto AY = [&](int k) { return axis_from_fixed(128 * y - 64 + 256 * k, src.h); };
    const Axis xm = AX(-1), x0 = AX(0), xp = AX(1), ym = AY(-1), y0 = AY(0), yp = AY(1);
    f3 a = tap(src, xm, yp), b = tap(src, x0, yp), c = tap(src, xp, yp);
    f3 d = tap(src, xm, y0), e = tap(src, x0, y0), f = tap(src, xp, y0);
    f3 g = tap(src, xm, ym), h = tap(src, x0, ym), i = tap(src, xp, ym);
    store_rgb1(dst, x, y, SOC_UP9(a, b, c, d, e, f, g, h, i));
}

// ------------------------------------------------------------------------------------------------
// register-window kernels: each lane loads the raw RGBA16F texels of its window once (8-B loads, L1
// shared with its neighbours) and evaluates the taps channel by channel; bilinear taps share their
// horizontal lerps between taps that use the same row and x-pair. Every tap is computed with exactly
// the arithmetic of tap()/point() above (same lerps, same order) as the oracle's per-tap restatement,
// so results are bit-identical.
// ------------------------------------------------------------------------------------------------
// same-size 13-tap downsample, 2x2 output pixels per lane from a 6x6 texel window
__global__ __launch_bounds__(kWorkgroup) void bloom_down_same_q(DImg src, DImg dst, bool vec) {
    const int m = blockIdx.x * BX + threadIdx.x, n = blockIdx.y * BY + threadIdx.y;
    const int X0 = 2 * m, Y0 = 2 * n;
    if (X0 >= dst.w || Y0 >= dst.h) return;
    uint2 T[6][6];
#pragma unroll
    for (int r = 0; r < 6; ++r)
#pragma unroll
        for (int c = 0; c < 6; ++c) T[r][c] = texel_clamped(src, X0 - 2 + c, Y0 - 2 + r);
    float out[2][2][3];
    auto run = [&](auto CH) {
        constexpr int C = decltype(CH)::value;
        float V[6][6];
#pragma unroll
        for (int r = 0; r < 6; ++r)
#pragma unroll
            for (int c = 0; c < 6; ++c) V[r][c] = chan<C>(T[r][c]);
#pragma unroll
        for (int py = 0; py < 2; ++py)
#pragma unroll
            for (int px = 0; px < 2; ++px) {
                // window index of offset o: o + 2 + parity; "+Y" taps are the row below
                auto P = [&](int ox, int oy) { return V[oy + 2 + py][ox + 2 + px]; };
                out[py][px][C] = down13(P(-2, 2), P(0, 2), P(2, 2), P(-2, 0), P(0, 0), P(2, 0), P(-2, -2), P(0, -2),
                                        P(2, -2), P(-1, 1), P(1, 1), P(-1, -1), P(1, -1));
            }
    };
    run(std::integral_constant<int, 0>{});
    run(std::integral_constant<int, 1>{});
    run(std::integral_constant<int, 2>{});
    store_quad_row(dst, X0, Y0, out[0], vec);
    store_quad_row(dst, X0, Y0 + 1, out[1], vec);
}

// same-size 9-tap tent upsample, 2x2 output pixels per lane from a 4x4 window
__global__ __launch_bounds__(kWorkgroup) void bloom_up_same_q(DImg src, DImg dst, bool vec) {
    const int m = blockIdx.x * BX + threadIdx.x, n = blockIdx.y * BY + threadIdx.y;
    const int X0 = 2 * m, Y0 = 2 * n;
    if (X0 >= dst.w || Y0 >= dst.h) return;
    uint2 T[4][4];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) T[r][c] = texel_clamped(src, X0 - 1 + c, Y0 - 1 + r);
    float out[2][2][3];
    auto run = [&](auto CH) {
        constexpr int C = decltype(CH)::value;
#pragma unroll
        for (int py = 0; py < 2; ++py)
#pragma unroll
            for (int px = 0; px < 2; ++px) {
                auto P = [&](int ox, int oy) { return chan<C>(T[oy + 1 + py][ox + 1 + px]); };
                out[py][px][C] = up9(P(-1, 1), P(0, 1), P(1, 1), P(-1, 0), P(0, 0), P(1, 0), P(-1, -1), P(0, -1), P(1, -1));
            }
    };
    run(std::integral_constant<int, 0>{});
    run(std::integral_constant<int, 1>{});
    run(std::integral_constant<int, 2>{});
    store_quad_row(dst, X0, Y0, out[0], vec);
    store_quad_row(dst, X0, Y0 + 1, out[1], vec);
}

// 2:1 downsample: one output per lane, 6x6 source window; the 13 taps are w = 0.5 blends of the 2x2
// blocks at source offsets 2x+k (k = -2..2), sharing the 30 horizontal lerps. Border pixels use tap().
__global__ __launch_bounds__(kWorkgroup) void bloom_down_half_w(DImg src, DImg dst) {
    const int x = blockIdx.x * BX + threadIdx.x, y = blockIdx.y * BY + threadIdx.y;
    if (x >= dst.w || y >= dst.h) return;
    const bool interior = 2 * x - 2 >= 0 && 2 * x + 3 <= src.w - 1 && 2 * y - 2 >= 0 && 2 * y + 3 <= src.h - 1;
    if (!interior) {
        auto AX = [&](int k) { return axis_from_fixed(256 * (2 * x + k) + 128, src.w); };
        auto AY = [&](int k) { return axis_from_fixed(256 * (2 * y + k) + 128, src.h); };
        const Axis xm2 = AX(-2), xm1 = AX(-1), x0 = AX(0), xp1 = AX(1), xp2 = AX(2);
        const Axis ym2 = AY(-2), ym1 = AY(-1), y0 = AY(0), yp1 = AY(1), yp2 = AY(2);
        f3 a = tap(src, xm2, yp2), b = tap(src, x0, yp2), c = tap(src, xp2, yp2);
        f3 d = tap(src, xm2, y0), e = tap(src, x0, y0), f = tap(src, xp2, y0);
        f3 g = tap(src, xm2, ym2), h = tap(src, x0, ym2), i = tap(src, xp2, ym2);
        f3 j = tap(src, xm1, yp1), k = tap(src, xp1, yp1), l = tap(src, xm1, ym1), m = tap(src, xp1, ym1);
        store_rgb1(dst, x, y, SOC_DOWN13(a, b, c, d, e, f, g, h, i, j, k, l, m));
        return;
    }
    uint2 T[6][6];
    const uint2* base = row_ptr<uint2>(src, 2 * y - 2) + (2 * x - 2);
    const int pitch8 = src.pitch / 8;
#pragma unroll
    for (int r = 0; r < 6; ++r)
#pragma unroll
        for (int c = 0; c < 6; ++c) T[r][c] = base[r * pitch8 + c];
    float out[3];
    auto run = [&](auto CH) {
        constexpr int C = decltype(CH)::value;
        float Hl[6][5];   // row r, x-pair k+2 = blend of window columns (k+2, k+3)
#pragma unroll
        for (int r = 0; r < 6; ++r)
#pragma unroll
            for (int k = 0; k < 5; ++k) Hl[r][k] = lerp_c(chan<C>(T[r][k]), chan<C>(T[r][k + 1]), 0.5f);
        auto S = [&](int kx, int ky) { return lerp_c(Hl[ky + 2][kx + 2], Hl[ky + 3][kx + 2], 0.5f); };
        out[C] = down13(S(-2, 2), S(0, 2), S(2, 2), S(-2, 0), S(0, 0), S(2, 0), S(-2, -2), S(0, -2), S(2, -2), S(-1, 1),
                        S(1, 1), S(-1, -1), S(1, -1));
    };
    run(std::integral_constant<int, 0>{});
    run(std::integral_constant<int, 1>{});
    run(std::integral_constant<int, 2>{});
    store_rgb1_c(dst, x, y, out[0], out[1], out[2]);
}

// 1:2 upsample: a 2x2 output quad per lane from the 5x5 source window around (m, n). Even outputs use
// x-pairs (m-2..m) at w = 3/4, odd ones (m-1..m+1) at w = 1/4 (and likewise in y). Border quads use tap().
__global__ __launch_bounds__(kWorkgroup) void bloom_up_double_q(DImg src, DImg dst, bool vec) {
    const int m = blockIdx.x * BX + threadIdx.x, n = blockIdx.y * BY + threadIdx.y;
    if (m >= src.w || n >= src.h) return;
    const int X0 = 2 * m, Y0 = 2 * n;
    const bool interior = m - 2 >= 0 && m + 2 <= src.w - 1 && n - 2 >= 0 && n + 2 <= src.h - 1;
    if (!interior) {
#pragma unroll 1
        for (int k = 0; k < 4; ++k) {
                const int px = k & 1, py = k >> 1;
                const int x = X0 + px, y = Y0 + py;
                auto AX = [&](int k) { return axis_from_fixed(128 * x - 64 + 256 * k, src.w); };
                auto AY = [&](int k) { return axis_from_fixed(128 * y - 64 + 256 * k, src.h); };
                const Axis xm = AX(-1), x0 = AX(0), xp = AX(1), ym = AY(-1), y0 = AY(0), yp = AY(1);
                f3 a = tap(src, xm, yp), b = tap(src, x0, yp), c = tap(src, xp, yp);
                f3 d = tap(src, xm, y0), e = tap(src, x0, y0), f = tap(src, xp, y0);
                f3 g = tap(src, xm, ym), h = tap(src, x0, ym), i = tap(src, xp, ym);
                store_rgb1(dst, x, y, SOC_UP9(a, b, c, d, e, f, g, h, i));
            }
        return;
    }
    uint2 T[5][5];
    const uint2* base = row_ptr<uint2>(src, n - 2) + (m - 2);
    const int pitch8 = src.pitch / 8;
#pragma unroll
    for (int r = 0; r < 5; ++r)
#pragma unroll
        for (int c = 0; c < 5; ++c) T[r][c] = base[r * pitch8 + c];
    float out[2][2][3];
    auto run = [&](auto CH) {
        constexpr int C = decltype(CH)::value;
        float V[5][5];
#pragma unroll
        for (int r = 0; r < 5; ++r)
#pragma unroll
            for (int c = 0; c < 5; ++c) V[r][c] = chan<C>(T[r][c]);
        // four times the horizontal lerps of both parities (exact: RGBA16F texels, bloom_common.hpp)
        float H0[5][3], H1[5][3];
#pragma unroll
        for (int r = 0; r < 5; ++r)
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                H0[r][k] = t_w34(V[r][k], V[r][k + 1]);
                H1[r][k] = t_w14(V[r][k + 1], V[r][k + 2]);
            }
#pragma unroll
        for (int px = 0; px < 2; ++px) {
            const float (&Hl)[5][3] = px ? H1 : H0;
            // vertical: py 0 = v_w34(rows ky+1, ky+2), py 1 = v_w14(rows ky+2, ky+3); both use the same
            // rounded product of row ky+2
            float S0[3][3], S1[3][3];
#pragma unroll
            for (int ky = -1; ky <= 1; ++ky)
#pragma unroll
                for (int kx = -1; kx <= 1; ++kx) {
                    const float p = v_prod(Hl[ky + 2][kx + 1]);
                    S0[ky + 1][kx + 1] = __builtin_fmaf(Hl[ky + 1][kx + 1], 0.0625f, p);
                    S1[ky + 1][kx + 1] = __builtin_fmaf(Hl[ky + 3][kx + 1], 0.0625f, p);
                }
            out[0][px][C] = up9(S0[2][0], S0[2][1], S0[2][2], S0[1][0], S0[1][1], S0[1][2], S0[0][0], S0[0][1], S0[0][2]);
            out[1][px][C] = up9(S1[2][0], S1[2][1], S1[2][2], S1[1][0], S1[1][1], S1[1][2], S1[0][0], S1[0][1], S1[0][2]);
        }
        __builtin_amdgcn_sched_barrier(0);   // one channel's window live at a time
    };
    run(std::integral_constant<int, 0>{});
    run(std::integral_constant<int, 1>{});
    run(std::integral_constant<int, 2>{});
    store_quad_row(dst, X0, Y0, out[0], vec);
    store_quad_row(dst, X0, Y0 + 1, out[1], vec);
}

constexpr int kFastMax = 8192;

// Below this many output pixels the 1:2 upsample runs one pixel per lane (4x the lanes of the quad
// kernel: small mips need the parallelism more than the shared window). Tuning knob:
// SOC_BLOOM_QUAD_MIN_PX overrides it.
long quad_min_px() {
    static const long v = [] {
        const char* e = getenv("SOC_BLOOM_QUAD_MIN_PX");
        return e ? atol(e) : 1L << 20;
    }();
    return v;
}

bool vec16(const soc_img& im) { return im.pitch_bytes % 16 == 0 && reinterpret_cast<uintptr_t>(im.data) % 16 == 0; }

}  // namespace

int launch_bloom_down(const soc_img& hi, const soc_img& lo, hipStream_t s, int force_generic) {
    dim3 blk(BX, BY), grd(ceil_div(lo.width, BX), ceil_div(lo.height, BY));
    DImg src = dimg(hi), dst = dimg(lo);
    const bool small = hi.width <= kFastMax && hi.height <= kFastMax;
    if (!force_generic && small && hi.width == lo.width && hi.height == lo.height) {
        dim3 g2(ceil_div(ceil_div(lo.width, 2), BX), ceil_div(ceil_div(lo.height, 2), BY));
        launch("bloom_down_same_q", kWorkgroup, bloom_down_same_q, g2, blk, 0, s, src, dst, vec16(lo));
    } else if (!force_generic && small && hi.width == 2 * lo.width && hi.height == 2 * lo.height) {
        launch("bloom_down_half_w", kWorkgroup, bloom_down_half_w, grd, blk, 0, s, src, dst);
    } else {
        launch("bloom_down_generic", kWorkgroup, bloom_down_generic, grd, blk, 0, s, src, dst, 1.0f / (float)hi.width, 1.0f / (float)hi.height);
    }
    return check_launch("bloom_downsample");
}

int launch_bloom_up(const soc_img& lo, const soc_img& hi, hipStream_t s, int force_generic) {
    dim3 blk(BX, BY), grd(ceil_div(hi.width, BX), ceil_div(hi.height, BY));
    DImg src = dimg(lo), dst = dimg(hi);
    const bool small = hi.width <= kFastMax && hi.height <= kFastMax;
    if (!force_generic && small && hi.width == lo.width && hi.height == lo.height) {
        dim3 g2(ceil_div(ceil_div(hi.width, 2), BX), ceil_div(ceil_div(hi.height, 2), BY));
        launch("bloom_up_same_q", kWorkgroup, bloom_up_same_q, g2, blk, 0, s, src, dst, vec16(hi));
    } else if (!force_generic && small && hi.width == 2 * lo.width && hi.height == 2 * lo.height) {
        if ((long)hi.width * hi.height < quad_min_px()) {
            launch("bloom_up_double", kWorkgroup, bloom_up_double, grd, blk, 0, s, src, dst);
        } else {
            dim3 g2(ceil_div(lo.width, BX), ceil_div(lo.height, BY));
            launch("bloom_up_double_q", kWorkgroup, bloom_up_double_q, g2, blk, 0, s, src, dst, vec16(hi));
        }
    } else {
        launch("bloom_up_generic", kWorkgroup, bloom_up_generic, grd, blk, 0, s, src, dst, 1.0f / (float)lo.width, 1.0f / (float)lo.height);
    }
    return check_launch("bloom_upsample");
}

}  // namespace soc

using namespace soc;

static int bloom_args(const soc_img& a, const soc_img& b, const char* pass) {
    int rc = check_img(a, SOC_FMT_RGBA16F, pass, "source");
    if (rc) return rc;
    rc = check_img(b, SOC_FMT_RGBA16F, pass, "target");
    if (rc) return rc;
    if (a.data == b.data) return set_error(SOC_E_INVALID_ARG, "%s: source and target alias", pass);
    return SOC_OK;
}

extern "C" int soc_bloom_downsample(const soc_globals* g, soc_img higher_mip, soc_img lower_mip, soc_stream stream) {
    (void)g;
    int rc = bloom_args(higher_mip, lower_mip, "soc_bloom_downsample");
    if (rc) return rc;
    return launch_bloom_down(higher_mip, lower_mip, hs(stream), 0);
}

extern "C" int soc_bloom_upsample(const soc_globals* g, soc_img lower_mip, soc_img higher_mip, soc_stream stream) {
    (void)g;
    int rc = bloom_args(lower_mip, higher_mip, "soc_bloom_upsample");
    if (rc) return rc;
    return launch_bloom_up(lower_mip, higher_mip, hs(stream), 0);
}

// Test hook: force the generic (float-uv) tap path to cross-check the fast paths.
extern "C" int soc_debug_bloom_generic(int32_t up, soc_img a, soc_img b, soc_stream stream) {
    int rc = bloom_args(a, b, "soc_debug_bloom_generic");
    if (rc) return rc;
    return up ? launch_bloom_up(a, b, hs(stream), 1) : launch_bloom_down(a, b, hs(stream), 1);
}

extern "C" int soc_bloom_weighted_stage(const soc_globals* g, soc_img emissive, const soc_img* mips, int32_t mip_count,
                                        soc_img output, int32_t stage, soc_stream stream) {
    (void)g;
    static const char* P = "soc_bloom_weighted_stage";
    if (!mips) return set_error(SOC_E_INVALID_ARG, "%s: null mips", P);
    if (stage < 0 || stage > 4) return set_error(SOC_E_INVALID_ARG, "%s: stage %d not in 0..4", P, stage);
    int rc = check_img(emissive, SOC_FMT_RGBA16F, P, "emissive");
    if (!rc) rc = check_img(output, SOC_FMT_RGBA16F, P, "output");
    for (int i = 0; !rc && i < mip_count; ++i) rc = check_img(mips[i], SOC_FMT_RGBA16F, P, "mip");
    if (rc) return rc;
    if (!bloom_fused_applicable(emissive, mips, mip_count, output))
        return set_error(SOC_E_UNSUPPORTED, "%s: needs 4 mips halving exactly from the emissive extent (<= 8192)", P);
    if ((stage == 0 || stage == 4) && output.data == mips[1].data)
        return set_error(SOC_E_INVALID_ARG, "%s: output aliases mip 1", P);
    return launch_bloom_weighted(emissive, mips, output, hs(stream), stage);
}

extern "C" int soc_bloom_chain(const soc_globals* g, soc_img emissive, const soc_img* mips, int32_t mip_count,
                               soc_stream stream) {
    if (!mips || mip_count < 1) return set_error(SOC_E_INVALID_ARG, "soc_bloom_chain: need >= 1 mip");
    int rc = soc_bloom_downsample(g, emissive, mips[0], stream);
    for (int i = 0; !rc && i < mip_count - 1; ++i) rc = soc_bloom_downsample(g, mips[i], mips[i + 1], stream);
    for (int i = mip_count - 1; !rc && i > 0; --i) rc = soc_bloom_upsample(g, mips[i], mips[i - 1], stream);
    if (!rc) rc = soc_bloom_upsample(g, mips[0], emissive, stream);
    return rc;
}
