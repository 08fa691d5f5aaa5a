// luminance.hpp — the luminance-histogram bin of GenerateLuminanceHistogramTask
// (src/graphics/tasks/generate_luminance_histogram.inl:59-78) as a device function: the bit-exact contract
// of DESIGN.md §3.4 (explicit-FMA luminance and remap, deterministic log2), identical to the oracle's
// soc_oracle_luminance_bin. Shared by the histogram pass (exposure.hip) and the fused composition +
// histogram pass (composition.hip).
#pragma once

#include <cmath>

#include "../../include/soc_rt.h"
#include "soc_device.hpp"

namespace soc {

constexpr int kBins = SOC_AUTO_EXPOSURE_BIN_COUNT;


__device__ __forceinline__ float u2f(uint32_t u) { return __builtin_bit_cast(float, u); }
__device__ __forceinline__ uint32_t f2u(float f) { return __builtin_bit_cast(uint32_t, f); }

// Deterministic log2 (same operation sequence as soc_oracle_log2).
__device__ __forceinline__ float det_log2(float x) {
#pragma clang fp contract(off)
    if (x != x) return x;
    if (x < 0.0f) return u2f(0x7fc00000u);
    if (x == 0.0f) return -__builtin_inff();
    if (x == __builtin_inff()) return __builtin_inff();
    uint32_t u = f2u(x);
    int e = 0;
    if (u < 0x00800000u) { x = x * 8388608.0f; u = f2u(x); e = -23; }
    e += (int)(u >> 23) - 127;
    float m = u2f((u & 0x007fffffu) | 0x3f800000u);
    if (m > 1.41421356f) { m = m * 0.5f; e += 1; }
    float f = m - 1.0f;
    float s = f / (2.0f + f);
    float s2 = s * s;
    float p = __builtin_fmaf(s2, 1.0f / 11.0f, 1.0f / 9.0f);
    p = __builtin_fmaf(s2, p, 1.0f / 7.0f);
    p = __builtin_fmaf(s2, p, 1.0f / 5.0f);
    p = __builtin_fmaf(s2, p, 1.0f / 3.0f);
    p = __builtin_fmaf(s2, p, 1.0f);
    float ln = (2.0f * s) * p;
    return __builtin_fmaf(ln, 1.44269504088896341f, (float)e);
}

__device__ __forceinline__ uint32_t lum_bin(float r, float g, float b, float lmin, float lrange) {
#pragma clang fp contract(off)
    float lum = __builtin_fmaf(b, 0.0722f, __builtin_fmaf(g, 0.7152f, r * 0.2126f));
    if (lum < 1e-3f) lum = 0.0f;
    float q = (det_log2(lum) - lmin) / lrange;
    float mapped = __builtin_fmaf(q, (float)(kBins - 1) - 1.0f, 1.0f);
    if (mapped >= 255.0f) return 255u;
    if (mapped > 0.0f) return (uint32_t)(int32_t)mapped;
    return 0u;
}

// Fast bin with an exact fallback. lum_bin spends most of its ~70 VALU ops in det_log2's two IEEE
// divisions and polynomial; the bin only depends on which integer interval `mapped` falls in. The fast
// form uses the hardware log2 (v_log_f32) and a reciprocal multiply; over the luminances that reach it
// (finite, >= 1e-3, < 2^17 from RGBA16F inputs, so |log2| < 17) it differs from lum_bin's `mapped` by
// at most |dlog2| * 254/|lrange| + the rounding of the remap: |dlog2| <= a few ulp(16) ~ 5e-6 (both
// log2 forms are within 2-3 ulp of the true value). BinFast::eps is that bound with a 6x margin
// (host: bin_fast_params). A `mapped` farther than eps from every bin boundary (the integers 1..255)
// truncates to the same bin in both forms; anything closer, and any non-finite value, returns
// kBinExact and the caller recomputes that pixel with lum_bin, so the result is lum_bin's bit for bit.
// With the reference's range (|lrange| = 30) eps = 3.5e-4: ~0.07 % of pixels take the exact path.
struct BinFast {
    float lmin, rlr, eps;   // log_min, 1 / (log_max - log_min), fallback margin in `mapped` units
    uint32_t zero;          // lum_bin of a luminance < 1e-3 (log2(0) = -inf through the remap)
};
constexpr uint32_t kBinExact = 0xffffffffu;

// Host: the BinFast parameters of a frame. `zero` follows lum_bin for lum = 0 (det_log2(0) = -inf,
// then the same IEEE remap and clamp).
inline BinFast bin_fast_params(float lmin, float lrange) {
    BinFast f;
    f.lmin = lmin;
    f.rlr = 1.0f / lrange;
    f.eps = 3.0e-5f * ((float)(kBins - 1) - 1.0f) / std::fabs(lrange) + 1.0e-4f;
    if (!(f.eps < 0.25f)) f.eps = 0.25f;   // degenerate range (or NaN): the `> eps` test sends nearly all to lum_bin
    const float q = (-INFINITY - lmin) / lrange;
    const float mapped = std::fmaf(q, (float)(kBins - 1) - 1.0f, 1.0f);
    f.zero = mapped >= 255.0f ? 255u : (mapped > 0.0f ? (uint32_t)(int32_t)mapped : 0u);
    return f;
}

__device__ __forceinline__ uint32_t lum_bin_fast(float r, float g, float b, const BinFast& f) {
#pragma clang fp contract(off)
    const float lum = __builtin_fmaf(b, 0.0722f, __builtin_fmaf(g, 0.7152f, r * 0.2126f));   // as lum_bin
    if (lum < 1e-3f) return f.zero;
    const float mapped = __builtin_fmaf((__builtin_amdgcn_logf(lum) - f.lmin) * f.rlr, (float)(kBins - 1) - 1.0f, 1.0f);
    if (mapped < 1.0f - f.eps) return 0u;
    if (mapped >= 255.0f + f.eps) return 255u;
    if (!(__builtin_fabsf(mapped - __builtin_rintf(mapped)) > f.eps)) return kBinExact;   // near a boundary, or NaN
    return (uint32_t)(int32_t)mapped;
}

// Adds the bins of two pixels per lane into an LDS histogram with one LDS atomic per distinct bin of
// the wave (a ballot loop: neighbouring pixels mostly share a bin, so 2-3 rounds per 16x8 block).
// Lanes with valid == false contribute nothing; every lane of the wave must call it. (Device atomics per
// wave instead of the LDS copy measured 186 us at 4K: the hot bins serialise.)
// mask bit 0: pixel 0 is binned, bit 1: pixel 1
__device__ __forceinline__ void wave_bin_pair_mask(uint32_t* sh, uint32_t b0, uint32_t b1, uint32_t mask) {
    uint32_t pend = mask & 3u;   // bit 0: pixel 0 pending, bit 1: pixel 1
    const uint32_t lane = __lane_id();
    unsigned long long act = __ballot(pend != 0u);
    while (act) {
        const int leader = __builtin_ctzll(act);
        const uint32_t lb0 = (uint32_t)__shfl((int)b0, leader), lb1 = (uint32_t)__shfl((int)b1, leader);
        const uint32_t lpend = (uint32_t)__shfl((int)pend, leader);
        const uint32_t B = (lpend & 1u) ? lb0 : lb1;
        const uint32_t mine = (((pend & 1u) && b0 == B) ? 1u : 0u) + (((pend & 2u) && b1 == B) ? 1u : 0u);
        if ((pend & 1u) && b0 == B) pend &= ~1u;
        if ((pend & 2u) && b1 == B) pend &= ~2u;
        // wave sum of `mine` (0..2 per lane)
        const unsigned long long m1 = __ballot(mine & 1u), m2 = __ballot(mine & 2u);
        const uint32_t total = (uint32_t)__builtin_popcountll(m1) + 2u * (uint32_t)__builtin_popcountll(m2);
        if (lane == (uint32_t)leader) atomicAdd(&sh[B], total);
        act = __ballot(pend != 0u);
    }
}

// The same counts as wave_bin_pair_mask with one LDS atomic per lane (two when its pixels' bins differ) and no
// ballot loop: same-address atomics of a wave serialise in the LDS unit, off the VALU issue path.
__device__ __forceinline__ void lane_bin_pair_mask(uint32_t* sh, uint32_t b0, uint32_t b1, uint32_t mask) {
    const bool p0 = mask & 1u, p1 = (mask & 2u) != 0u;
    if (p0 && p1 && b0 == b1) {
        atomicAdd(&sh[b0], 2u);
    } else {
        if (p0) atomicAdd(&sh[b0], 1u);
        if (p1) atomicAdd(&sh[b1], 1u);
    }
}

__device__ __forceinline__ void wave_bin_pair(uint32_t* sh, uint32_t b0, uint32_t b1, bool valid) {
    wave_bin_pair_mask(sh, b0, b1, valid ? 3u : 0u);
}

}  // namespace soc
