// tonemap.hip — ToneMappingTask (src/graphics/tasks/tone_mapping.inl:20-70, AgX-DS shader :91-176) as a
// gfx950 kernel writing the headless framebuffer.
//
// The AgX matrices depend only on uniforms, so sRGB->adjusted and its inverse are built once per call
// on the host (soc::agx_matrices, the same fp32 arithmetic as the shader's PrimariesToMatrix /
// ComputeCompressionMatrix / inverse) and passed as kernel arguments; 2^exposure is read from the
// AutoExposure buffer. Two pixels per lane: one 16-B RGBA16F load, one 8-B RGBA8 store.
#include "agx.hpp"
#include "soc_internal.hpp"

namespace soc {
namespace {

template <int FMT>
__device__ __forceinline__ void store_px(const DImg& t, int x, int y, f3 c) {
    if constexpr (FMT == SOC_FMT_RGBA8_UNORM) {
        row_ptr_w<uint32_t>(t, y)[x] = pack_unorm8x4(f4{c.x, c.y, c.z, 1.0f});
    } else if constexpr (FMT == SOC_FMT_RGBA8_SRGB) {
        row_ptr_w<uint32_t>(t, y)[x] = pack_unorm8x4(f4{srgb_encode(c.x), srgb_encode(c.y), srgb_encode(c.z), 1.0f});
    } else if constexpr (FMT == SOC_FMT_RGBA16F) {
        row_ptr_w<uint2>(t, y)[x] = pack_h4(f4{c.x, c.y, c.z, 1.0f});
    } else {
        row_ptr_w<float4>(t, y)[x] = float4{c.x, c.y, c.z, 1.0f};
    }
}

constexpr int BX = 64, BY = 4;

// Fast path: same extent, even width, 16-B aligned source rows.
template <int FMT>
__global__ __launch_bounds__(kWorkgroup) void tonemap_pair(DImg src, DImg dst, const soc_auto_exposure* __restrict__ ae, TmParams p) {
    const int x = (blockIdx.x * BX + threadIdx.x) * 2, y = blockIdx.y * BY + threadIdx.y;
    if (x >= dst.w || y >= dst.h) return;
    const float expo = exp2f(ae->exposure);   // pow(2.0, exposure)
    const uint4 q = row_ptr<uint4>(src, y)[x >> 1];
    const f3 c0 = agx(p, unpack_h4(uint2{q.x, q.y}), expo);
    const f3 c1 = agx(p, unpack_h4(uint2{q.z, q.w}), expo);
    if constexpr (FMT == SOC_FMT_RGBA8_UNORM) {
        row_ptr_w<uint2>(dst, y)[x >> 1] =
            uint2{pack_unorm8x4(f4{c0.x, c0.y, c0.z, 1.0f}), pack_unorm8x4(f4{c1.x, c1.y, c1.z, 1.0f})};
    } else {
        store_px<FMT>(dst, x, y, c0);
        store_px<FMT>(dst, x + 1, y, c1);
    }
}

template <int FMT>
__global__ __launch_bounds__(kWorkgroup) void tonemap_generic(DImg src, DImg dst, const soc_auto_exposure* __restrict__ ae, TmParams p) {
    const int x = blockIdx.x * BX + threadIdx.x, y = blockIdx.y * BY + threadIdx.y;
    if (x >= dst.w || y >= dst.h) return;
    const float expo = exp2f(ae->exposure);
    const f4 c = sample_h4(src, centre_uv(x, dst.w), centre_uv(y, dst.h));
    store_px<FMT>(dst, x, y, agx(p, c, expo));
}

template <int FMT>
void launch(const soc_img& color, const soc_img& target, const soc_auto_exposure* ae, const TmParams& p, hipStream_t s) {
    const int W = target.width, H = target.height;
    const bool pair = color.width == W && color.height == H && W % 2 == 0 && W <= 8192 && H <= 8192 &&
                      (reinterpret_cast<uintptr_t>(color.data) & 15u) == 0 && (color.pitch_bytes & 15) == 0 &&
                      (reinterpret_cast<uintptr_t>(target.data) & 7u) == 0 && (target.pitch_bytes & 7) == 0;
    if (pair) {
        dim3 blk(BX, BY), grd(ceil_div(W / 2, BX), ceil_div(H, BY));
        launch("tonemap_pair", kWorkgroup, tonemap_pair<FMT>, grd, blk, 0, s, dimg(color), dimg(target), ae, p);
    } else {
        dim3 blk(BX, BY), grd(ceil_div(W, BX), ceil_div(H, BY));
        launch("tonemap_generic", kWorkgroup, tonemap_generic<FMT>, grd, blk, 0, s, dimg(color), dimg(target), ae, p);
    }
}

}  // namespace
}  // namespace soc

using namespace soc;

extern "C" int soc_tone_mapping(const soc_globals* g, soc_img color, const soc_auto_exposure* ae, soc_img target,
                                soc_stream stream) {
    static const char* P = "soc_tone_mapping";
    if (!g || !ae) return set_error(SOC_E_INVALID_ARG, "%s: null globals / auto exposure buffer", P);
    int rc = check_img(color, SOC_FMT_RGBA16F, P, "color");
    if (!rc) rc = check_img(target, 0, P, "target");
    if (rc) return rc;
    TmParams p;
    agx_matrices(g->compression, p.M.m, p.Minv.m);
    p.linear = g->agxDs_linear_section;
    p.peak = g->peak;
    p.saturation = g->saturation;
    tm_params_finish(p);
    switch (target.format) {
    case SOC_FMT_RGBA8_UNORM: launch<SOC_FMT_RGBA8_UNORM>(color, target, ae, p, hs(stream)); break;
    case SOC_FMT_RGBA8_SRGB: launch<SOC_FMT_RGBA8_SRGB>(color, target, ae, p, hs(stream)); break;
    case SOC_FMT_RGBA16F: launch<SOC_FMT_RGBA16F>(color, target, ae, p, hs(stream)); break;
    case SOC_FMT_RGBA32F: launch<SOC_FMT_RGBA32F>(color, target, ae, p, hs(stream)); break;
    default: return set_error(SOC_E_UNSUPPORTED, "%s: unsupported target format %d", P, target.format);
    }
    return check_launch("tone_mapping");
}
