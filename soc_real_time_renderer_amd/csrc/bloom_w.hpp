// bloom_w.hpp — the weighted-form bloom arithmetic shared by bloom_w.hip (the chain's kernels) and composition.hip (the
// last upsample computed inside Composition, SOC_RENDERER_BLOOM_IN_COMPOSITION). The weights and footprints are those of
// bloom_w.hip's header comment (bloom_upsample.inl:98-127 at the chain's fixed ratios).
#pragma once

#include "soc_internal.hpp"

namespace soc {
namespace {

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return min(max(v, lo), hi); }

struct C3 {
    float r, g, b;
};
__device__ __forceinline__ float lo16(uint32_t u) { return (float)__builtin_bit_cast(_Float16, (uint16_t)(u & 0xffffu)); }
__device__ __forceinline__ float hi16(uint32_t u) { return (float)__builtin_bit_cast(_Float16, (uint16_t)(u >> 16)); }
// a += w * texel.rgb (one v_fma_mix_f32 per channel)
__device__ __forceinline__ void madd(C3& a, uint2 t, float w) {
    a.r = __builtin_fmaf(lo16(t.x), w, a.r);
    a.g = __builtin_fmaf(hi16(t.x), w, a.g);
    a.b = __builtin_fmaf(lo16(t.y), w, a.b);
}
__device__ __forceinline__ uint2 pack3(const C3& c) { return pack_h4(f4{c.r, c.g, c.b, 1.0f}); }

// Clamp-to-edge tile load: t[r][c] = im[clamp(oy + r)][clamp(ox + c)]. Each lane issues its loads four at a time
// before their LDS stores (one memory latency per four rounds of the 256-lane loop instead of one per round).
template <int TW, int TH>
__device__ __forceinline__ void load_tile(const DImg& im, int ox, int oy, uint2 (*t)[TW], int tid) {
    constexpr int N = TW * TH;
    auto at = [&](int i) {
        const int r = i / TW, c = i - r * TW;
        return row_ptr<uint2>(im, clampi(oy + r, 0, im.h - 1)) + clampi(ox + c, 0, im.w - 1);
    };
    for (int i0 = tid; i0 < N; i0 += 4 * 256) {
        const int i1 = i0 + 256, i2 = i1 + 256, i3 = i2 + 256;
        const uint2 a = *at(i0);
        uint2 b = uint2{0u, 0u}, c = b, d = b;
        if (i1 < N) b = *at(i1);
        if (i2 < N) c = *at(i2);
        if (i3 < N) d = *at(i3);
        t[i0 / TW][i0 % TW] = a;
        if (i1 < N) t[i1 / TW][i1 % TW] = b;
        if (i2 < N) t[i2 / TW][i2 % TW] = c;
        if (i3 < N) t[i3 / TW][i3 % TW] = d;
    }
}

// up 1:2 weights: k = 0..3 along the 4-texel footprint
__device__ __forceinline__ constexpr float u12_w(int parity, int k) {
    constexpr int E[4] = {1, 5, 7, 3}, O[4] = {3, 7, 5, 1};
    return (float)(parity ? O[k] : E[k]) * (1.0f / 16.0f);
}

// The chain's last upsample pair (W4: mip1 -> [mip0] -> output, bloomw_up10s) for an OW x OH tile of outputs at
// (X0, Y0), X0 even, by a 256-lane workgroup, in separable form: the 1:2 pass as a horizontal pass into an fp32 LDS
// tile and a vertical pass (the mip0 entries rounded to RGBA16F, as the chain stores mip0), then the 1:1 (1 2 1)
// horizontal sums; out() finishes an output pair with the vertical (1 2 1). Every value is a function of its clamped
// image coordinates only, so any tile size gives the same bits for the same output pixel.
template <int OW, int OH>
struct Up10Tile {
    static constexpr int MW = OW + 2, MH = OH + 2;           // mip0 tile, origin (X0 - 1, Y0 - 1)
    static constexpr int SW = OW / 2 + 6, SH = OH / 2 + 6;   // mip1 tile, origin (X0/2 - 3, Y0/2 - 3)
    static constexpr int HR = SH > MH ? SH : MH;             // rows of the fp32 sums (14 x MW, then MH x OW)
    // the mip1 tile is dead once the 1:2 horizontal sums are built (a barrier apart), so the mip0 tile overlays it
    // (bloomw_up10s 28 -> 23 KiB; the same bits, the same speed: profiles/r05_ab_up10_alias.txt)
    union {
        uint2 st[SH][SW];
        uint2 mt[MH][MW];
    };
    float hr[HR][MW], hg[HR][MW], hb[HR][MW];

    // the tile's horizontal 1:1 sums; ends with a barrier (out() may follow directly)
    __device__ __forceinline__ void build(const DImg& S1, int X0, int Y0, int W0, int H0, int tid) {
        const int mx0 = X0 - 1, my0 = Y0 - 1;
        const int sx0 = X0 / 2 - 3, sy0 = Y0 / 2 - 3;
        load_tile<SW, SH>(S1, sx0, sy0, st, tid);
        __syncthreads();
        // 1:2 horizontal: hr/hg/hb[sr][c] for mip0 column c (coordinate clamp(mx0 + c)) on mip1 tile row sr
        for (int i = tid; i < SH * MW; i += 256) {
            const int sr = i / MW, c = i - sr * MW;
            const int q = clampi(mx0 + c, 0, W0 - 1), px = q & 1, c0 = (q >> 1) - 2 + px - sx0;
            C3 a{0.0f, 0.0f, 0.0f};
#pragma unroll
            for (int k = 0; k < 4; ++k) madd(a, st[sr][c0 + k], u12_w(px, k));
            hr[sr][c] = a.r;
            hg[sr][c] = a.g;
            hb[sr][c] = a.b;
        }
        __syncthreads();
        // 1:2 vertical: the mip0 entries (RGBA16F, as stored by the chain)
        for (int i = tid; i < MH * MW; i += 256) {
            const int r = i / MW, c = i - r * MW;
            const int cy = clampi(my0 + r, 0, H0 - 1), py = cy & 1, r0 = (cy >> 1) - 2 + py - sy0;
            C3 a{0.0f, 0.0f, 0.0f};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float w = u12_w(py, k);
                a.r = __builtin_fmaf(hr[r0 + k][c], w, a.r);
                a.g = __builtin_fmaf(hg[r0 + k][c], w, a.g);
                a.b = __builtin_fmaf(hb[r0 + k][c], w, a.b);
            }
            mt[r][c] = pack3(a);
        }
        __syncthreads();
        // 1:1 horizontal: hr/hg/hb[r][x - X0] over mip0 row r for output column x (tile columns x - mx0 - 1 .. + 1)
        for (int i = tid; i < MH * OW; i += 256) {
            const int r = i / OW, c = i - r * OW;   // tile column c + 1
            C3 a{0.0f, 0.0f, 0.0f};
            madd(a, mt[r][c], 1.0f);
            madd(a, mt[r][c + 1], 2.0f);
            madd(a, mt[r][c + 2], 1.0f);
            hr[r][c] = a.r;
            hg[r][c] = a.g;
            hb[r][c] = a.b;
        }
        __syncthreads();
    }
    // the 1:1 vertical of the outputs at tile row r, tile columns c, c + 1 (the chain stores pack3 of each)
    __device__ __forceinline__ void out(int r, int c, C3 (&o)[2]) const {
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int cc = c + k;
            o[k].r = __builtin_fmaf(hr[r + 2][cc], 1.0f / 16.0f, __builtin_fmaf(hr[r + 1][cc], 2.0f / 16.0f, hr[r][cc] * (1.0f / 16.0f)));
            o[k].g = __builtin_fmaf(hg[r + 2][cc], 1.0f / 16.0f, __builtin_fmaf(hg[r + 1][cc], 2.0f / 16.0f, hg[r][cc] * (1.0f / 16.0f)));
            o[k].b = __builtin_fmaf(hb[r + 2][cc], 1.0f / 16.0f, __builtin_fmaf(hb[r + 1][cc], 2.0f / 16.0f, hb[r][cc] * (1.0f / 16.0f)));
        }
    }
};

}  // namespace
}  // namespace soc
