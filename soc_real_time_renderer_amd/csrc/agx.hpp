// agx.hpp — the AgX-DS tone curve of ToneMappingTask (src/graphics/tasks/tone_mapping.inl:91-176) as a
// device function, shared by the tone-mapping pass (tonemap.hip) and the fused TAA + tone-map pass
// (taa.hip), so both produce the same bits from the same RGBA16F input.
#pragma once

#include "soc_device.hpp"

namespace soc {

struct TmParams {
    Mat3 M, Minv;
    float linear, peak, saturation;
};

// DualSection, :127-137
__device__ __forceinline__ float dual_section(float x, float linear, float peak) {
    const float S = peak * linear;
    if (x < S) return x;
    const float C = peak / (peak - S);
    return peak - (peak - S) * __expf((-C * (x - S)) / peak);
}

__device__ __forceinline__ f3 agx(const TmParams& p, f4 c, float expo) {
    f3 w = f3{fmaxf(c.x, 0.0f), fmaxf(c.y, 0.0f), fmaxf(c.z, 0.0f)} * expo;
    w = mul(p.M, w);
    w = f3{clampf(dual_section(w.x, p.linear, p.peak), 0.0f, 1.0f), clampf(dual_section(w.y, p.linear, p.peak), 0.0f, 1.0f),
           clampf(dual_section(w.z, p.linear, p.peak), 0.0f, 1.0f)};
    const float ds = dot3(w, f3{0.2126729f, 0.7151522f, 0.0721750f});
    w = f3{mixf(ds, w.x, p.saturation), mixf(ds, w.y, p.saturation), mixf(ds, w.z, p.saturation)};
    w = f3{clampf(w.x, 0.0f, 1.0f), clampf(w.y, 0.0f, 1.0f), clampf(w.z, 0.0f, 1.0f)};
    return mul(p.Minv, w);
}

}  // namespace soc
