// bloom_fused.hip — the whole bloom chain of renderer.cpp:1024-1062 (4 downsamples, 4 upsamples,
// bloom_downsample.inl:107-141, bloom_upsample.inl:98-127) as FOUR gfx950 kernels.
//
// In the reference chain the downsampled mip0 and mip2 are read once, by the next downsample, and
// then overwritten by the upsamples (quirk Q5). Each fused kernel therefore keeps such an
// intermediate in LDS, recomputing a halo per workgroup, and never writes it to HBM:
//   K1  emissive -> [mip0] -> mip1          (1:1 13-tap, then 2:1 13-tap)
//   K2  mip1 -> [mip2] -> mip3              (2:1, 2:1)
//   K3  mip3 -> mip2 -> mip1                (1:2 9-tap twice; both mips written: final state)
//   K4  mip1 -> mip0 -> output              (1:2, then 1:1 9-tap; mip0 written: final state)
// After the four kernels every mip and the output hold exactly the bits of the 8-pass chain: the
// intermediate is rounded to RGBA16F in LDS as the image store would round it, and every tap goes
// through the same clamp rule (axis_from_fixed / point) and lerp order as bloom.hip's kernels.
// Traffic at 3840x2160: ~315 MB instead of ~720 MB for the 8 separate passes.
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "bloom_common.hpp"

// Profiling builds only (tools/kernel_variants.py): 1 = K4 without its quad phase, 2 = K4 without its
// output phase, 3 = K4 without global stores. The library is always built with 0.
#ifndef SOC_BLOOM_PROFILE
#define SOC_BLOOM_PROFILE 0
#endif

namespace soc {
namespace {

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return min(max(v, lo), hi); }

// Bilinear tap from an LDS tile whose texel (0, 0) is image texel (ox, oy); identical to tap().
template <int TW>
__device__ __forceinline__ f3 tile_tap(const uint2 (*t)[TW], int ox, int oy, const Axis& ax, const Axis& ay) {
    const uint2* r0 = t[ay.i0 - oy];
    const uint2* r1 = t[ay.i1 - oy];
    const f4 a = unpack_h4(r0[ax.i0 - ox]), b = unpack_h4(r0[ax.i1 - ox]), c = unpack_h4(r1[ax.i0 - ox]),
             d = unpack_h4(r1[ax.i1 - ox]);
    return f3{bilerp1(a.x, b.x, c.x, d.x, ax.w, ay.w), bilerp1(a.y, b.y, c.y, d.y, ax.w, ay.w),
              bilerp1(a.z, b.z, c.z, d.z, ax.w, ay.w)};
}

template <int TW>
__device__ __forceinline__ f3 tile_point(const uint2 (*t)[TW], int ox, int oy, int x, int y) {
    const f4 v = unpack_h4(t[y - oy][x - ox]);
    return f3{v.x, v.y, v.z};
}

typedef float v2f __attribute__((ext_vector_type(2)));

__device__ __forceinline__ v2f mul2(v2f a, v2f b) {
#pragma clang fp contract(off)
    return a * b;
}

// up9 on two independent pixels (packed fp32, same roundings as up9)
__device__ __forceinline__ v2f up9_2(v2f a, v2f b, v2f c, v2f d, v2f e, v2f f, v2f g, v2f h, v2f i) {
#pragma clang fp contract(off)
    v2f r = e * 4.0f;
    r += (b + d + f + h) * 2.0f;
    r += (a + c + g + i);
    r *= 1.0f / 16.0f;
    return r;
}

__device__ __forceinline__ Axis ax_half(int x, int k, int n) { return axis_from_fixed(256 * (2 * x + k) + 128, n); }
__device__ __forceinline__ Axis ax_double(int x, int k, int n) { return axis_from_fixed(128 * x - 64 + 256 * k, n); }

// Clamp-to-edge tile load (8-B texels).
template <int TW, int TH, int NT>
__device__ __forceinline__ void load_tile(const DImg& im, int ox, int oy, uint2 (*t)[TW], int tid) {
    for (int i = tid; i < TW * TH; i += NT) {
        const int r = i / TW, c = i - r * TW;
        t[r][c] = row_ptr<uint2>(im, clampi(oy + r, 0, im.h - 1))[clampi(ox + c, 0, im.w - 1)];
    }
}

// Same, as 16-B texel pairs: ox even, image width even and rows 16-B aligned, so a pair is either
// wholly inside the image or wholly outside one edge.
template <int TW, int TH, int NT>
__device__ __forceinline__ void load_tile_pairs(const DImg& im, int ox, int oy, uint2 (*t)[TW], int tid) {
    constexpr int PW = TW / 2;
    for (int i = tid; i < PW * TH; i += NT) {
        const int r = i / PW, c = 2 * (i - r * PW);
        const uint2* row = row_ptr<uint2>(im, clampi(oy + r, 0, im.h - 1));
        const int gx = ox + c;
        uint4 q;
        if (gx >= 0 && gx + 1 < im.w) {
            q = *reinterpret_cast<const uint4*>(row + gx);
        } else {
            const uint2 a = row[clampi(gx, 0, im.w - 1)], b = row[clampi(gx + 1, 0, im.w - 1)];
            q = uint4{a.x, a.y, b.x, b.y};
        }
        *reinterpret_cast<uint4*>(&t[r][c]) = q;
    }
}

__device__ __forceinline__ void store_pair(const DImg& im, int x, int y, f3 a, f3 b, bool vec) {
    uint2* row = row_ptr_w<uint2>(im, y);
    const uint2 pa = pack_h4(f4{a.x, a.y, a.z, 1.0f}), pb = pack_h4(f4{b.x, b.y, b.z, 1.0f});
    if (vec && x + 1 < im.w) {
        *reinterpret_cast<uint4*>(row + x) = uint4{pa.x, pa.y, pb.x, pb.y};
        return;
    }
    row[x] = pa;
    if (x + 1 < im.w) row[x + 1] = pb;
}

// ================================================================================================
// K1: emissive (W x H) -> [mip0, same extent, LDS] -> mip1 (W/2 x H/2)
// ================================================================================================
constexpr int K1_OW = 32, K1_OH = 16;                          // mip1 outputs per workgroup
constexpr int K1_MW = 2 * K1_OW + 4, K1_MH = 2 * K1_OH + 4;    // mip0 tile 68 x 36
constexpr int K1_EW = K1_MW + 4, K1_EH = K1_MH + 4;            // emissive tile 72 x 40

template <bool PAIRS>
__global__ __launch_bounds__(256) void bloom_fused_down01(DImg E, DImg M1, bool vec) {
    __shared__ __attribute__((aligned(16))) uint2 Et[K1_EH][K1_EW];   // 22.5 KiB
    __shared__ __attribute__((aligned(16))) uint2 Mt[K1_MH][K1_MW];   // 19.1 KiB
    const int tid = threadIdx.x;
    const int X0 = blockIdx.x * K1_OW, Y0 = blockIdx.y * K1_OH;
    const int mx0 = 2 * X0 - 2, my0 = 2 * Y0 - 2, ex0 = mx0 - 2, ey0 = my0 - 2;
    const int W = E.w, H = E.h;
    if (PAIRS) load_tile_pairs<K1_EW, K1_EH, 256>(E, ex0, ey0, Et, tid);
    else load_tile<K1_EW, K1_EH, 256>(E, ex0, ey0, Et, tid);
    __syncthreads();
    // mip0 at every tile position, evaluated at the clamped coordinate (what a clamped tap reads)
    if (ex0 >= 0 && ey0 >= 0 && ex0 + K1_EW <= W && ey0 + K1_EH <= H) {
        // interior tile: no clamping, the 13 taps are fixed LDS offsets from the centre texel
        for (int i = tid; i < K1_MW * K1_MH; i += 256) {
            const int r = i / K1_MW, c = i - r * K1_MW;
            const uint2* ctr = &Et[r + 2][c + 2];
            auto P = [&](int dx, int dy) {
                const f4 v = unpack_h4(ctr[dy * K1_EW + dx]);
                return f3{v.x, v.y, v.z};
            };
            const f3 a = P(-2, 2), b = P(0, 2), cc = P(2, 2), d = P(-2, 0), e = P(0, 0), f = P(2, 0), g = P(-2, -2),
                     h = P(0, -2), ii = P(2, -2), j = P(-1, 1), k = P(1, 1), l = P(-1, -1), m = P(1, -1);
            const f3 o = SOC_DOWN13(a, b, cc, d, e, f, g, h, ii, j, k, l, m);
            Mt[r][c] = pack_h4(f4{o.x, o.y, o.z, 1.0f});
        }
    } else
    for (int i = tid; i < K1_MW * K1_MH; i += 256) {
        const int r = i / K1_MW, c = i - r * K1_MW;
        const int x = clampi(mx0 + c, 0, W - 1), y = clampi(my0 + r, 0, H - 1);
        auto P = [&](int dx, int dy) {
            return tile_point<K1_EW>(Et, ex0, ey0, clampi(x + dx, 0, W - 1), clampi(y + dy, 0, H - 1));
        };
        const f3 a = P(-2, 2), b = P(0, 2), cc = P(2, 2), d = P(-2, 0), e = P(0, 0), f = P(2, 0), g = P(-2, -2),
                 h = P(0, -2), ii = P(2, -2), j = P(-1, 1), k = P(1, 1), l = P(-1, -1), m = P(1, -1);
        const f3 o = SOC_DOWN13(a, b, cc, d, e, f, g, h, ii, j, k, l, m);
        Mt[r][c] = pack_h4(f4{o.x, o.y, o.z, 1.0f});
    }
    __syncthreads();
    // mip1: two horizontally adjacent outputs per lane
    const int x = X0 + 2 * (tid & 15), y = Y0 + (tid >> 4);
    if (x >= M1.w || y >= M1.h) return;
    f3 o[2];
    const bool interior = 2 * x - 2 >= 0 && 2 * x + 5 <= W - 1 && 2 * y - 2 >= 0 && 2 * y + 3 <= H - 1;
    if (interior) {
        // every tap is the w = 0.5 blend of a 2x2 block: share the horizontal lerps of the
        // 6 x 8 mip0 window (rows 2y-2.., cols 2x-2..) between the 13 taps of both outputs
        const int r0 = 2 * y - 2 - my0, c0 = 2 * x - 2 - mx0;
        uint2 T[6][8];
#pragma unroll
        for (int r = 0; r < 6; ++r)
#pragma unroll
            for (int c = 0; c < 8; ++c) T[r][c] = Mt[r0 + r][c0 + c];
        float out[2][3];
        auto run = [&](auto CH) {
            constexpr int C = decltype(CH)::value;
            float Hl[6][7];
#pragma unroll
            for (int r = 0; r < 6; ++r)
#pragma unroll
                for (int c = 0; c < 7; ++c) Hl[r][c] = mid(chan<C>(T[r][c]), chan<C>(T[r][c + 1]));
#pragma unroll
            for (int p = 0; p < 2; ++p) {
                auto S = [&](int kx, int ky) { return mid(Hl[ky + 2][kx + 2 + 2 * p], Hl[ky + 3][kx + 2 + 2 * p]); };
                out[p][C] = down13(S(-2, 2), S(0, 2), S(2, 2), S(-2, 0), S(0, 0), S(2, 0), S(-2, -2), S(0, -2), S(2, -2),
                                   S(-1, 1), S(1, 1), S(-1, -1), S(1, -1));
            }
        };
        run(std::integral_constant<int, 0>{});
        run(std::integral_constant<int, 1>{});
        run(std::integral_constant<int, 2>{});
        o[0] = f3{out[0][0], out[0][1], out[0][2]};
        o[1] = f3{out[1][0], out[1][1], out[1][2]};
    } else {
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            const int xp = min(x + p, M1.w - 1);
            const Axis xm2 = ax_half(xp, -2, W), xm1 = ax_half(xp, -1, W), x0 = ax_half(xp, 0, W), xp1 = ax_half(xp, 1, W),
                       xp2 = ax_half(xp, 2, W);
            const Axis ym2 = ax_half(y, -2, H), ym1 = ax_half(y, -1, H), y0 = ax_half(y, 0, H), yp1 = ax_half(y, 1, H),
                       yp2 = ax_half(y, 2, H);
            auto S = [&](const Axis& a, const Axis& b) { return tile_tap<K1_MW>(Mt, mx0, my0, a, b); };
            const f3 a = S(xm2, yp2), b = S(x0, yp2), c = S(xp2, yp2), d = S(xm2, y0), e = S(x0, y0), f = S(xp2, y0),
                     g = S(xm2, ym2), h = S(x0, ym2), i = S(xp2, ym2), j = S(xm1, yp1), k = S(xp1, yp1), l = S(xm1, ym1),
                     m = S(xp1, ym1);
            o[p] = SOC_DOWN13(a, b, c, d, e, f, g, h, i, j, k, l, m);
        }
    }
    store_pair(M1, x, y, o[0], o[1], vec);
}

// ================================================================================================
// K2: mip1 -> [mip2, LDS] -> mip3   (small levels: every tap through the generic clamp rule)
// ================================================================================================
constexpr int K2_OW = 16, K2_OH = 8;                           // mip3 outputs per workgroup
constexpr int K2_MW = 2 * K2_OW + 4, K2_MH = 2 * K2_OH + 4;    // mip2 tile 36 x 20
constexpr int K2_SW = 2 * K2_MW + 4, K2_SH = 2 * K2_MH + 4;    // mip1 tile 76 x 44

__global__ __launch_bounds__(256) void bloom_fused_down23(DImg S1, DImg M3, int W2, int H2) {
    __shared__ __attribute__((aligned(16))) uint2 St[K2_SH][K2_SW];   // 26.1 KiB
    __shared__ __attribute__((aligned(16))) uint2 Mt[K2_MH][K2_MW];   // 5.6 KiB
    const int tid = threadIdx.x;
    const int X0 = blockIdx.x * K2_OW, Y0 = blockIdx.y * K2_OH;
    const int mx0 = 2 * X0 - 2, my0 = 2 * Y0 - 2, sx0 = 2 * mx0 - 2, sy0 = 2 * my0 - 2;
    const int W1 = S1.w, H1 = S1.h;
    load_tile<K2_SW, K2_SH, 256>(S1, sx0, sy0, St, tid);
    __syncthreads();
    for (int i = tid; i < K2_MW * K2_MH; i += 256) {
        const int r = i / K2_MW, c = i - r * K2_MW;
        const int x = clampi(mx0 + c, 0, W2 - 1), y = clampi(my0 + r, 0, H2 - 1);
        const Axis xm2 = ax_half(x, -2, W1), xm1 = ax_half(x, -1, W1), x0 = ax_half(x, 0, W1), xp1 = ax_half(x, 1, W1),
                   xp2 = ax_half(x, 2, W1);
        const Axis ym2 = ax_half(y, -2, H1), ym1 = ax_half(y, -1, H1), y0 = ax_half(y, 0, H1), yp1 = ax_half(y, 1, H1),
                   yp2 = ax_half(y, 2, H1);
        auto S = [&](const Axis& a, const Axis& b) { return tile_tap<K2_SW>(St, sx0, sy0, a, b); };
        const f3 a = S(xm2, yp2), b = S(x0, yp2), cc = S(xp2, yp2), d = S(xm2, y0), e = S(x0, y0), f = S(xp2, y0),
                 g = S(xm2, ym2), h = S(x0, ym2), ii = S(xp2, ym2), j = S(xm1, yp1), k = S(xp1, yp1), l = S(xm1, ym1),
                 m = S(xp1, ym1);
        const f3 o = SOC_DOWN13(a, b, cc, d, e, f, g, h, ii, j, k, l, m);
        Mt[r][c] = pack_h4(f4{o.x, o.y, o.z, 1.0f});
    }
    __syncthreads();
    if (tid >= K2_OW * K2_OH) return;
    const int x = X0 + (tid % K2_OW), y = Y0 + (tid / K2_OW);
    if (x >= M3.w || y >= M3.h) return;
    const Axis xm2 = ax_half(x, -2, W2), xm1 = ax_half(x, -1, W2), x0 = ax_half(x, 0, W2), xp1 = ax_half(x, 1, W2),
               xp2 = ax_half(x, 2, W2);
    const Axis ym2 = ax_half(y, -2, H2), ym1 = ax_half(y, -1, H2), y0 = ax_half(y, 0, H2), yp1 = ax_half(y, 1, H2),
               yp2 = ax_half(y, 2, H2);
    auto S = [&](const Axis& a, const Axis& b) { return tile_tap<K2_MW>(Mt, mx0, my0, a, b); };
    const f3 a = S(xm2, yp2), b = S(x0, yp2), c = S(xp2, yp2), d = S(xm2, y0), e = S(x0, y0), f = S(xp2, y0),
             g = S(xm2, ym2), h = S(x0, ym2), i = S(xp2, ym2), j = S(xm1, yp1), k = S(xp1, yp1), l = S(xm1, ym1),
             m = S(xp1, ym1);
    store_rgb1(M3, x, y, SOC_DOWN13(a, b, c, d, e, f, g, h, i, j, k, l, m));
}

// 9-tap 1:2 tent upsample of destination pixel (x, y) from a tile of the source (extent sw x sh).
template <int TW>
__device__ __forceinline__ f3 up_double_tile(const uint2 (*t)[TW], int ox, int oy, int x, int y, int sw, int sh) {
    const Axis xm = ax_double(x, -1, sw), x0 = ax_double(x, 0, sw), xp = ax_double(x, 1, sw);
    const Axis ym = ax_double(y, -1, sh), y0 = ax_double(y, 0, sh), yp = ax_double(y, 1, sh);
    auto S = [&](const Axis& a, const Axis& b) { return tile_tap<TW>(t, ox, oy, a, b); };
    const f3 a = S(xm, yp), b = S(x0, yp), c = S(xp, yp), d = S(xm, y0), e = S(x0, y0), f = S(xp, y0), g = S(xm, ym),
             h = S(x0, ym), i = S(xp, ym);
    return SOC_UP9(a, b, c, d, e, f, g, h, i);
}

// ================================================================================================
// K3: mip3 -> mip2 (written) -> mip1 (written)
// ================================================================================================
constexpr int K3_OW = 32, K3_OH = 16;                          // mip1 outputs per workgroup
constexpr int K3_MW = K3_OW / 2 + 4, K3_MH = K3_OH / 2 + 4;    // mip2 tile 20 x 12
constexpr int K3_SW = K3_MW / 2 + 4, K3_SH = K3_MH / 2 + 4;    // mip3 tile 14 x 10

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void bloom_fused_up32(DImg S3, DImg M2, DImg M1, bool vec) {
    __shared__ __attribute__((aligned(16))) uint2 St[K3_SH][K3_SW];
    __shared__ __attribute__((aligned(16))) uint2 Mt[K3_MH][K3_MW];
    const int tid = threadIdx.x;
    const int X0 = blockIdx.x * K3_OW, Y0 = blockIdx.y * K3_OH;
    const int mx0 = X0 / 2 - 2, my0 = Y0 / 2 - 2;          // even
    const int sx0 = mx0 / 2 - 2, sy0 = my0 / 2 - 2;
    const int W2 = M2.w, H2 = M2.h;
    load_tile<K3_SW, K3_SH, 256>(S3, sx0, sy0, St, tid);
    __syncthreads();
    for (int i = tid; i < K3_MW * K3_MH; i += 256) {
        const int r = i / K3_MW, c = i - r * K3_MW;
        const int gx = mx0 + c, gy = my0 + r;
        const int x = clampi(gx, 0, W2 - 1), y = clampi(gy, 0, H2 - 1);
        const f3 o = up_double_tile<K3_SW>(St, sx0, sy0, x, y, S3.w, S3.h);
        const uint2 v = pack_h4(f4{o.x, o.y, o.z, 1.0f});
        Mt[r][c] = v;
        // the tile's core (not the halo) is this workgroup's share of mip2
        if (c >= 2 && c < 2 + K3_OW / 2 && r >= 2 && r < 2 + K3_OH / 2 && gx < W2 && gy < H2) row_ptr_w<uint2>(M2, gy)[gx] = v;
    }
    __syncthreads();
    const int x = X0 + 2 * (tid & 15), y = Y0 + (tid >> 4);
    if (x >= M1.w || y >= M1.h) return;
    const f3 a = up_double_tile<K3_MW>(Mt, mx0, my0, x, y, W2, H2);
    const f3 b = up_double_tile<K3_MW>(Mt, mx0, my0, min(x + 1, M1.w - 1), y, W2, H2);
    store_pair(M1, x, y, a, b, vec);
}

// ================================================================================================
// K4: mip1 -> mip0 (written) -> output (written): 1:2 tent, then 1:1 tent
// Both LDS tiles are planar fp32 (one plane per channel): the quad and tent loops read one float per
// texel and channel, with no conversions and ~80 VGPRs, so four workgroups fit a CU.
// ================================================================================================
constexpr int K4_OW = 60, K4_OH = 28;                          // output pixels per workgroup
constexpr int K4_MW = K4_OW + 4, K4_MH = K4_OH + 4;            // mip0 tile 64 x 32 = 32 x 16 quads
constexpr int K4_MP = K4_MW + 1;                               // padded row pitch (bank spread)
constexpr int K4_SW = K4_MW / 2 + 4, K4_SH = K4_MH / 2 + 4;    // mip1 tile 36 x 20

// Bilinear tap from a planar fp32 tile (plane stride PS floats, row pitch RP): identical to tap().
template <int RP, int PS>
__device__ __forceinline__ f3 plane_tap(const float* t, int ox, int oy, const Axis& ax, const Axis& ay) {
    const float* r0 = t + (ay.i0 - oy) * RP;
    const float* r1 = t + (ay.i1 - oy) * RP;
    const int a = ax.i0 - ox, b = ax.i1 - ox;
    f3 o;
    o.x = bilerp1(r0[a], r0[b], r1[a], r1[b], ax.w, ay.w);
    o.y = bilerp1(r0[PS + a], r0[PS + b], r1[PS + a], r1[PS + b], ax.w, ay.w);
    o.z = bilerp1(r0[2 * PS + a], r0[2 * PS + b], r1[2 * PS + a], r1[2 * PS + b], ax.w, ay.w);
    return o;
}

__global__ __launch_bounds__(256) void bloom_fused_up10(DImg S1, DImg M0, DImg O, bool vec) {
    constexpr int SPS = K4_SW * K4_SH, MPS = K4_MP * K4_MH;
    __shared__ float St[3 * SPS];   // 8.4 KiB
    __shared__ float Mt[3 * MPS];   // 24.4 KiB
    const int tid = threadIdx.x;
    const int X0 = blockIdx.x * K4_OW, Y0 = blockIdx.y * K4_OH;
    const int mx0 = X0 - 2, my0 = Y0 - 2;                  // even: quads of mip0 are (2m, 2m+1)
    const int qx0 = mx0 / 2, qy0 = my0 / 2;                // quad index of tile column 0 (may be -1)
    const int sx0 = qx0 - 2, sy0 = qy0 - 2;
    const int W1 = S1.w, H1 = S1.h, W = M0.w, H = M0.h;
    for (int i = tid; i < SPS; i += 256) {
        const int r = i / K4_SW, c = i - r * K4_SW;
        const f4 v = unpack_h4(row_ptr<uint2>(S1, clampi(sy0 + r, 0, H1 - 1))[clampi(sx0 + c, 0, W1 - 1)]);
        St[i] = v.x;
        St[SPS + i] = v.y;
        St[2 * SPS + i] = v.z;
    }
    __syncthreads();
#pragma unroll 1
    for (int qi = tid; qi < (SOC_BLOOM_PROFILE == 1 ? 0 : (K4_MW / 2) * (K4_MH / 2)); qi += 256) {
        const int qy = qi / (K4_MW / 2), qx = qi - qy * (K4_MW / 2);
        const int m = qx0 + qx, n = qy0 + qy;
        if (m < 0 || m >= W1 || n < 0 || n >= H1) continue;   // outside the image: never read
        float out[2][2][3];
        if (m - 2 >= 0 && m + 2 <= W1 - 1 && n - 2 >= 0 && n + 2 <= H1 - 1) {
            // interior quad: even outputs blend source pairs (m-2..m) at w = 3/4, odd ones
            // (m-1..m+1) at w = 1/4, the same in y; the horizontal lerps are shared
            const float* base = St + (n - 2 - sy0) * K4_SW + (m - 2 - sx0);
#pragma unroll
            for (int C = 0; C < 3; ++C) {
                float V[5][5];
#pragma unroll
                for (int r = 0; r < 5; ++r)
#pragma unroll
                    for (int c = 0; c < 5; ++c) V[r][c] = base[C * SPS + r * K4_SW + c];
                // both horizontal parities at once (packed fp32): px 0 is t_w34(V[k], V[k+1]) =
                // fma(V[k+1], 3, V[k]), px 1 is t_w14(V[k+1], V[k+2]) = fma(V[k+1], 3, V[k+2])
                v2f Hl[5][3];
#pragma unroll
                for (int r = 0; r < 5; ++r)
#pragma unroll
                    for (int k = 0; k < 3; ++k)
                        Hl[r][k] = __builtin_elementwise_fma(v2f{V[r][k + 1], V[r][k + 1]}, v2f{3.0f, 3.0f}, v2f{V[r][k], V[r][k + 2]});
                // vertical: py 0 = v_w34(Hl[ky+1], Hl[ky+2]), py 1 = v_w14(Hl[ky+2], Hl[ky+3]); both
                // add a multiple of the same rounded product Hl[ky+2] * 3/16
                v2f o[2];
                {
                    v2f S0[3][3], S1[3][3];
#pragma unroll
                    for (int ky = -1; ky <= 1; ++ky)
#pragma unroll
                        for (int kx = -1; kx <= 1; ++kx) {
                            const v2f p = mul2(Hl[ky + 2][kx + 1], v2f{0.1875f, 0.1875f});
                            S0[ky + 1][kx + 1] = __builtin_elementwise_fma(Hl[ky + 1][kx + 1], v2f{0.0625f, 0.0625f}, p);
                            S1[ky + 1][kx + 1] = __builtin_elementwise_fma(Hl[ky + 3][kx + 1], v2f{0.0625f, 0.0625f}, p);
                        }
                    // up9(a..i) with a = S(-1, 1), ... i = S(1, -1)
                    o[0] = up9_2(S0[2][0], S0[2][1], S0[2][2], S0[1][0], S0[1][1], S0[1][2], S0[0][0], S0[0][1], S0[0][2]);
                    o[1] = up9_2(S1[2][0], S1[2][1], S1[2][2], S1[1][0], S1[1][1], S1[1][2], S1[0][0], S1[0][1], S1[0][2]);
                }
#pragma unroll
                for (int py = 0; py < 2; ++py) {
                    out[py][0][C] = o[py].x;
                    out[py][1][C] = o[py].y;
                }
                __builtin_amdgcn_sched_barrier(0);   // one channel's window live at a time
            }
        } else {
            // border quad: every tap through the generic clamp rule, one pixel at a time
            const bool core = qx >= 1 && qx < 1 + K4_OW / 2 && qy >= 1 && qy < 1 + K4_OH / 2;
#pragma unroll 1
            for (int k = 0; k < 4; ++k) {
                const int px = k & 1, py = k >> 1;
                const int x = 2 * m + px, y = 2 * n + py;
                const Axis xm = ax_double(x, -1, W1), x0 = ax_double(x, 0, W1), xp = ax_double(x, 1, W1);
                const Axis ym = ax_double(y, -1, H1), y0 = ax_double(y, 0, H1), yp = ax_double(y, 1, H1);
                auto S = [&](const Axis& a, const Axis& b) { return plane_tap<K4_SW, SPS>(St, sx0, sy0, a, b); };
                const f3 a = S(xm, yp), b = S(x0, yp), c = S(xp, yp), d = S(xm, y0), e = S(x0, y0), f = S(xp, y0),
                         g = S(xm, ym), h = S(x0, ym), i = S(xp, ym);
                const f3 o = SOC_UP9(a, b, c, d, e, f, g, h, i);
                const uint2 v = pack_h4(f4{o.x, o.y, o.z, 1.0f});
                const f4 u = unpack_h4(v);
                float* mp = Mt + (2 * qy + py) * K4_MP + 2 * qx + px;
                mp[0] = u.x;
                mp[MPS] = u.y;
                mp[2 * MPS] = u.z;
                if (core && y < H) row_ptr_w<uint2>(M0, y)[x] = v;
            }
            continue;
        }
        const bool core = qx >= 1 && qx < 1 + K4_OW / 2 && qy >= 1 && qy < 1 + K4_OH / 2;
#pragma unroll
        for (int py = 0; py < 2; ++py) {
            const uint2 a = pack_h4(f4{out[py][0][0], out[py][0][1], out[py][0][2], 1.0f});
            const uint2 b = pack_h4(f4{out[py][1][0], out[py][1][1], out[py][1][2], 1.0f});
            // the tile keeps mip0 as stored: RGBA16F-rounded
            const f4 ua = unpack_h4(a), ub = unpack_h4(b);
            float* mrow = Mt + (2 * qy + py) * K4_MP + 2 * qx;
            mrow[0] = ua.x;
            mrow[1] = ub.x;
            mrow[MPS] = ua.y;
            mrow[MPS + 1] = ub.y;
            mrow[2 * MPS] = ua.z;
            mrow[2 * MPS + 1] = ub.z;
            if (SOC_BLOOM_PROFILE != 3 && core && 2 * n + py < H) {
                uint2* row = row_ptr_w<uint2>(M0, 2 * n + py) + 2 * m;
                if (vec) {
                    *reinterpret_cast<uint4*>(row) = uint4{a.x, a.y, b.x, b.y};
                } else {
                    row[0] = a;
                    row[1] = b;
                }
            }
        }
    }
    __syncthreads();
    // output: 1:1 tent of mip0 at clamped coordinates, one pixel per lane and iteration
    const bool inner = X0 >= 1 && Y0 >= 1 && X0 + K4_OW + 1 <= W && Y0 + K4_OH + 1 <= H;
#pragma unroll 1
    for (int i = tid; i < (SOC_BLOOM_PROFILE == 2 ? 0 : K4_OW * K4_OH); i += 256) {
        const int r = i / K4_OW, c = i - r * K4_OW;
        const int x = X0 + c, y = Y0 + r;
        if (x >= O.w || y >= O.h) continue;
        f3 o;
        if (inner) {
            const float* ctr = Mt + (r + 2) * K4_MP + (c + 2);
            float v[3];
#pragma unroll
            for (int C = 0; C < 3; ++C) {
                const float* p = ctr + C * MPS;
                auto P = [&](int dx, int dy) { return p[dy * K4_MP + dx]; };
                v[C] = up9(P(-1, 1), P(0, 1), P(1, 1), P(-1, 0), P(0, 0), P(1, 0), P(-1, -1), P(0, -1), P(1, -1));
            }
            o = f3{v[0], v[1], v[2]};
        } else {
            float v[3];
            const int xm = clampi(x - 1, 0, W - 1) - mx0, xc = x - mx0, xp = clampi(x + 1, 0, W - 1) - mx0;
            const int ym = clampi(y - 1, 0, H - 1) - my0, yc = y - my0, yp = clampi(y + 1, 0, H - 1) - my0;
#pragma unroll
            for (int C = 0; C < 3; ++C) {
                const float* p = Mt + C * MPS;
                auto P = [&](int cx, int cy) { return p[cy * K4_MP + cx]; };
                v[C] = up9(P(xm, yp), P(xc, yp), P(xp, yp), P(xm, yc), P(xc, yc), P(xp, yc), P(xm, ym), P(xc, ym), P(xp, ym));
            }
            o = f3{v[0], v[1], v[2]};
        }
        if (SOC_BLOOM_PROFILE != 3) row_ptr_w<uint2>(O, y)[x] = pack_h4(f4{o.x, o.y, o.z, 1.0f});
        else if (o.x == 12345.0f) row_ptr_w<uint2>(O, y)[x] = uint2{0, 0};
    }
}

bool aligned16(const soc_img& im) { return im.pitch_bytes % 16 == 0 && reinterpret_cast<uintptr_t>(im.data) % 16 == 0; }

}  // namespace

// The fused chain applies when the four mips halve exactly (the reference's mip chain at even
// extents, renderer.cpp:492-513) and the extents fit the 8-bit fixed-point tap range.
bool bloom_fused_applicable(const soc_img& emissive, const soc_img* mips, int mip_count, const soc_img& output) {
    if (mip_count != 4 || output.width != emissive.width || output.height != emissive.height) return false;
    if (emissive.width > 8192 || emissive.height > 8192) return false;
    if (mips[0].width != emissive.width || mips[0].height != emissive.height) return false;
    for (int i = 1; i < 4; ++i)
        if (mips[i - 1].width != 2 * mips[i].width || mips[i - 1].height != 2 * mips[i].height || mips[i].width < 2 ||
            mips[i].height < 2)
            return false;
    return true;
}

int launch_bloom_fused(const soc_img& emissive, const soc_img* mips, const soc_img& output, hipStream_t s, int stage) {
    const DImg E = dimg(emissive), M0 = dimg(mips[0]), M1 = dimg(mips[1]), M2 = dimg(mips[2]), M3 = dimg(mips[3]),
               O = dimg(output);
    if (stage == 0 || stage == 1) {
        dim3 g(ceil_div(mips[1].width, K1_OW), ceil_div(mips[1].height, K1_OH));
        if (aligned16(emissive)) bloom_fused_down01<true><<<g, 256, 0, s>>>(E, M1, aligned16(mips[1]));
        else bloom_fused_down01<false><<<g, 256, 0, s>>>(E, M1, aligned16(mips[1]));
    }
    if (stage == 0 || stage == 2) {
        dim3 g(ceil_div(mips[3].width, K2_OW), ceil_div(mips[3].height, K2_OH));
        bloom_fused_down23<<<g, 256, 0, s>>>(M1, M3, mips[2].width, mips[2].height);
    }
    if (stage == 0 || stage == 3) {
        dim3 g(ceil_div(mips[1].width, K3_OW), ceil_div(mips[1].height, K3_OH));
        bloom_fused_up32<<<g, 256, 0, s>>>(M3, M2, M1, aligned16(mips[1]));
    }
    if (stage == 0 || stage == 4) {
        dim3 g(ceil_div(output.width, K4_OW), ceil_div(output.height, K4_OH));
        bloom_fused_up10<<<g, 256, 0, s>>>(M1, M0, O, aligned16(mips[0]) && aligned16(output));
    }
    return check_launch("bloom_fused");
}

}  // namespace soc
