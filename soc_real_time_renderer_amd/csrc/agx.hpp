// agx.hpp — the AgX-DS tone curve of ToneMappingTask (src/graphics/tasks/tone_mapping.inl:91-176) as a
// device function, shared by the tone-mapping pass (tonemap.hip) and the fused TAA + tone-map pass
// (taa.hip), so both produce the same bits from the same RGBA16F input.
#pragma once

#include "soc_device.hpp"

namespace soc {

struct TmParams {
    Mat3 M, Minv;
    float linear, peak, saturation;
    // DualSection constants (uniform, tm_params_finish): S = peak linear, kexp = -C / peak with
    // C = peak / (peak - S), folded into exp2: x >= S -> peak - (peak - S) exp2((x - S) kexp log2 e)
    float S, peak_minus_S, kexp2;
};

// DualSection, :127-137
__device__ __forceinline__ float dual_section(const TmParams& p, float x) {
    if (x < p.S) return x;
    return p.peak - p.peak_minus_S * __builtin_amdgcn_exp2f((x - p.S) * p.kexp2);
}

__device__ __forceinline__ f3 agx(const TmParams& p, f4 c, float expo) {
    f3 w = f3{fmaxf(c.x, 0.0f), fmaxf(c.y, 0.0f), fmaxf(c.z, 0.0f)} * expo;
    w = mul(p.M, w);
    w = f3{clampf(dual_section(p, w.x), 0.0f, 1.0f), clampf(dual_section(p, w.y), 0.0f, 1.0f),
           clampf(dual_section(p, w.z), 0.0f, 1.0f)};
    if (p.saturation != 1.0f) {   // mix(ds, w, 1) == w and w is already clamped: exact skip (uniform branch)
        const float ds = dot3(w, f3{0.2126729f, 0.7151522f, 0.0721750f});
        w = f3{mixf(ds, w.x, p.saturation), mixf(ds, w.y, p.saturation), mixf(ds, w.z, p.saturation)};
        w = f3{clampf(w.x, 0.0f, 1.0f), clampf(w.y, 0.0f, 1.0f), clampf(w.z, 0.0f, 1.0f)};
    }
    return mul(p.Minv, w);
}

// linear -> sRGB transfer for an RGBA8_SRGB framebuffer (the store of an *_SRGB swapchain image), shared by the
// tone-mapping pass and the fused TAA + tone map so both write the same codes.
__device__ __forceinline__ float srgb_encode(float c) {
    c = clampf(c, 0.0f, 1.0f);
    return c <= 0.0031308f ? c * 12.92f : 1.055f * powf(c, 1.0f / 2.4f) - 0.055f;
}

// Host: the uniform DualSection constants of a TmParams whose linear / peak / saturation are set.
inline void tm_params_finish(TmParams& p) {
    p.S = p.peak * p.linear;
    p.peak_minus_S = p.peak - p.S;
    const float C = p.peak / (p.peak - p.S);
    p.kexp2 = (-C / p.peak) * 1.44269504088896341f;
}

}  // namespace soc
