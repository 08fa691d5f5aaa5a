// texture.hip — the texture upload's mip chain (src/graphics/texture.cpp:108, 184-246) for gfx950.
//
// The reference builds each texture's chain at load with vkCmdBlitImage(LINEAR) from level k-1 to level k.
// Here one launch per level, one lane per destination texel (64x4 workgroups, coalesced 4-B rows): a
// destination texel reads the 2x2 source footprint of its blit sample point (L1/L2 resident: the source
// level was written by the previous launch) and writes one RGBA8 word. Levels are tiny next to a frame
// (a 2048^2 texture's chain is 5.6 MB), so the pass is launch-bound; it runs once per texture.
//
// sRGB: the blit filters in linear space. Decode and re-encode use tables the host computes in double
// precision (the oracle builds the same tables the same way), so the chain is bit-exact against it.
#include <cmath>

#include "soc_internal.hpp"

namespace soc {
namespace {

struct SrgbTables {
    float dec[256];   // srgb_decode(k / 255)
    float mid[256];   // mid[k] = srgb_decode((k - 0.5) / 255) (k >= 1): the linear value whose sRGB encoding rounds up
                      // to code k, as a LINEAR blit's encode-then-round does; mid[0] unused
};

double srgb_decode_d(double c) { return c <= 0.04045 ? c / 12.92 : std::pow((c + 0.055) / 1.055, 2.4); }

const SrgbTables& srgb_tables() {
    static SrgbTables t = [] {
        SrgbTables r{};
        for (int k = 0; k < 256; ++k) {
            r.dec[k] = (float)srgb_decode_d(k / 255.0);
            r.mid[k] = k ? (float)srgb_decode_d((k - 0.5) / 255.0) : 0.0f;
        }
        return r;
    }();
    return t;
}

// Blit sample axis: destination texel x of n_dst -> source taps of n_src, clamp to edge, 8-bit weights.
__device__ __forceinline__ Axis blit_axis(int x, int n_src, int n_dst) {
#pragma clang fp contract(off)
    const float t = ((float)(2 * x + 1) * (float)n_src) / (float)(2 * n_dst) - 0.5f;
    const int fx = (int)floorf(t * 256.0f + 0.5f);
    int i = fx >> 8;
    float w = (float)(fx & 255) * (1.0f / 256.0f);
    if (i < 0) { i = 0; w = 0.0f; }
    else if (i >= n_src - 1) { i = n_src - 2; w = 1.0f; }
    if (n_src == 1) { i = 0; w = 0.0f; }
    Axis a;
    a.i0 = i;
    a.i1 = min(i + 1, n_src - 1);
    a.w = w;
    return a;
}

// sRGB code of a linear value, round(encode(c) * 255): the number of boundaries mid[1..255] <= c (binary search).
__device__ __forceinline__ uint32_t srgb_encode_code(float c, const SrgbTables& t) {
    uint32_t k = 0;
#pragma unroll
    for (uint32_t step = 128; step; step >>= 1)
        if (k + step <= 255u && c >= t.mid[k + step]) k += step;
    return k;
}

__global__ __launch_bounds__(kWorkgroup) void mip_blit(DImg src, DImg dst, int srgb, SrgbTables tabs) {
#pragma clang fp contract(off)
    const int x = blockIdx.x * 64 + threadIdx.x, y = blockIdx.y * 4 + threadIdx.y;
    if (x >= dst.w || y >= dst.h) return;
    const Axis ax = blit_axis(x, src.w, dst.w), ay = blit_axis(y, src.h, dst.h);
    const uint32_t q[4] = {row_ptr<uint32_t>(src, ay.i0)[ax.i0], row_ptr<uint32_t>(src, ay.i0)[ax.i1],
                           row_ptr<uint32_t>(src, ay.i1)[ax.i0], row_ptr<uint32_t>(src, ay.i1)[ax.i1]};
    uint32_t out = 0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        float v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t b = (q[k] >> (8 * c)) & 255u;
            v[k] = (srgb && c < 3) ? tabs.dec[b] : unorm8(b);
        }
        const float f = bilerp1(v[0], v[1], v[2], v[3], ax.w, ay.w);
        const uint32_t code = (srgb && c < 3) ? srgb_encode_code(f, tabs) : to_unorm8(f);
        out |= code << (8 * c);
    }
    row_ptr_w<uint32_t>(dst, y)[x] = out;
}

// One level of the paired chain: texel i of the level's tight rows <- (albedo texel, normal texel).
__global__ __launch_bounds__(kWorkgroup) void pair_level(DImg a, DImg n, uint2* __restrict__ dst) {
    const int x = blockIdx.x * 64 + threadIdx.x, y = blockIdx.y * 4 + threadIdx.y;
    if (x >= a.w || y >= a.h) return;
    dst[(size_t)y * a.w + x] = uint2{row_ptr<uint32_t>(a, y)[x], row_ptr<uint32_t>(n, y)[x]};
}

}  // namespace
}  // namespace soc

using namespace soc;

extern "C" size_t soc_paired_texels_bytes(int32_t width, int32_t height) {
    if (width <= 0 || height <= 0) return 0;
    int wk, hk;
    const int L = mip_levels(width, height);
    return mip_offset(width, height, 8 * width, L - 1, wk, hk, 8) + (size_t)8 * wk * hk;
}

extern "C" int soc_pair_textures(soc_img albedo, soc_img normal_image, void* paired, soc_stream stream) {
    const auto rgba8 = [](const soc_img& t) { return t.format == SOC_FMT_RGBA8_UNORM || t.format == SOC_FMT_RGBA8_SRGB; };
    if (!rgba8(albedo) || !rgba8(normal_image) || !albedo.data || !normal_image.data || !paired)
        return set_error(SOC_E_INVALID_ARG, "soc_pair_textures: two RGBA8 textures with data and a target are required");
    if (albedo.width != normal_image.width || albedo.height != normal_image.height || albedo.width <= 0 || albedo.height <= 0 ||
        albedo.pitch_bytes < albedo.width * 4 || normal_image.pitch_bytes < normal_image.width * 4)
        return set_error(SOC_E_SHAPE, "soc_pair_textures: the textures must share one extent");
    const int W = albedo.width, H = albedo.height, L = mip_levels(W, H);
    for (int k = 0; k < L; ++k) {
        int wa, ha, wn, hn, wp, hp;
        const size_t oa = mip_offset(W, H, albedo.pitch_bytes, k, wa, ha);
        const size_t on = mip_offset(W, H, normal_image.pitch_bytes, k, wn, hn);
        const size_t op = mip_offset(W, H, 8 * W, k, wp, hp, 8);
        const DImg a{static_cast<char*>(albedo.data) + oa, wa, ha, k ? 4 * wa : albedo.pitch_bytes};
        const DImg n{static_cast<char*>(normal_image.data) + on, wn, hn, k ? 4 * wn : normal_image.pitch_bytes};
        launch("pair_level", kWorkgroup, pair_level, dim3(ceil_div(wa, 64), ceil_div(ha, 4)), dim3(64, 4), 0, hs(stream), a, n,
               reinterpret_cast<uint2*>(static_cast<char*>(paired) + op));
    }
    return check_launch("pair_textures");
}

extern "C" int32_t soc_mip_level_count(int32_t width, int32_t height) {
    return width > 0 && height > 0 ? mip_levels(width, height) : 0;
}

extern "C" size_t soc_mip_chain_bytes(int32_t width, int32_t height, int32_t pitch_bytes) {
    if (width <= 0 || height <= 0 || pitch_bytes < width * 4) return 0;
    int wk, hk;
    const int L = mip_levels(width, height);
    return mip_offset(width, height, pitch_bytes, L - 1, wk, hk) + (L > 1 ? (size_t)4 * wk * hk : (size_t)pitch_bytes * height);
}

extern "C" int soc_generate_mips(soc_img texture, soc_stream stream) {
    if (texture.format != SOC_FMT_RGBA8_UNORM && texture.format != SOC_FMT_RGBA8_SRGB)
        return set_error(SOC_E_INVALID_ARG, "soc_generate_mips: texture must be RGBA8_UNORM or RGBA8_SRGB");
    if (!texture.data || texture.width <= 0 || texture.height <= 0 || texture.pitch_bytes < texture.width * 4)
        return set_error(SOC_E_INVALID_ARG, "soc_generate_mips: null data, bad extent or pitch");
    const int W = texture.width, H = texture.height, L = mip_levels(W, H);
    char* base = static_cast<char*>(texture.data);
    const int srgb = texture.format == SOC_FMT_RGBA8_SRGB;
    for (int k = 1; k < L; ++k) {
        int ws, hs_, wd, hd;
        const size_t os = mip_offset(W, H, texture.pitch_bytes, k - 1, ws, hs_);
        const size_t od = mip_offset(W, H, texture.pitch_bytes, k, wd, hd);
        const DImg src{base + os, ws, hs_, k == 1 ? texture.pitch_bytes : 4 * ws};
        const DImg dst{base + od, wd, hd, 4 * wd};
        launch("mip_blit", kWorkgroup, mip_blit, dim3(ceil_div(wd, 64), ceil_div(hd, 4)), dim3(64, 4), 0, hs(stream), src, dst, srgb, srgb_tables());
    }
    return check_launch("generate_mips");
}
