// soc_internal.hpp — host-side helpers shared by the C-ABI entry points (not part of the ABI).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdarg>
#include <cstdio>
#include <string>

#include "../../include/soc_rt.h"
#include "soc_device.hpp"

namespace soc {

// Per-thread last error (soc_last_error_string).
int set_error(int code, const char* fmt, ...);
void clear_error();

inline int bytes_per_pixel(int fmt) {
    switch (fmt) {
    case SOC_FMT_RGBA16F: return 8;
    case SOC_FMT_D32F: return 4;
    case SOC_FMT_R8_UNORM: return 1;
    case SOC_FMT_RGBA8_UNORM:
    case SOC_FMT_RGBA8_SRGB: return 4;
    case SOC_FMT_RGBA32F: return 16;
    default: return 0;
    }
}

inline bool img_ok(const soc_img& im) {
    int b = bytes_per_pixel(im.format);
    return im.data != nullptr && im.width > 0 && im.height > 0 && b > 0 && im.pitch_bytes >= im.width * b;
}

// Validates `im` (and its format when fmt > 0); sets the error string on failure.
int check_img(const soc_img& im, int fmt, const char* pass, const char* what);

inline DImg dimg(const soc_img& im) { return DImg{static_cast<char*>(im.data), im.width, im.height, im.pitch_bytes}; }

inline Mat4 mat4(const float* m) {
    Mat4 r;
    for (int i = 0; i < 16; ++i) r.m[i] = m[i];
    return r;
}

inline hipStream_t hs(soc_stream s) { return reinterpret_cast<hipStream_t>(s); }

// Integer tuning knob from the environment (`dflt` when unset), read once and cached until soc_tuning_reload():
// only the variants the identity tests switch (SOC_SWZ_SSAO, SOC_SSAO_TILE, SOC_TAA_NBR, SOC_COMP_NT, SOC_GB_TEX_PAIRS,
// SOC_CLOUDS_ATMOS_POS, SOC_RENDERER_SSAO_FIRST, SOC_CLOUDS_OD_LUT) and the variants under measurement (SOC_GB_WAVE) are
// knobs; measured-and-rejected variants are removed.
int tuning_knob(const char* name, int dflt);
// RN(1 / n) for div_rn (soc_device.hpp), or 0 when n is outside the exhaustively checked range (1..16384).
inline float recip_rn(int n) {
    return n >= 1 && n <= 16384 ? 1.0f / (float)n : 0.0f;
}

// Checks the launch that was just issued (and a block shape launch() rejected: SOC_E_INVALID_ARG).
int check_launch(const char* pass);

// Launch geometry. Every kernel's flat work-group bound (its __launch_bounds__ / amdgpu_flat_work_group_size) is a
// named constant (kWorkgroup, kSunvisLanes, kSsaoTileLanes, kTaaLdsLanes, kThreads, kBins) that its launcher passes to
// launch() as `bound`. A block of more lanes than the bound, or of none, is not launched: the host records
// SOC_E_INVALID_ARG naming the kernel and the launcher's check_launch returns it, before any HIP call (a launch over
// the bound would otherwise fail on the device as "unspecified launch failure").
bool block_fits(const char* kernel, int bound, dim3 block);
template <typename... P, typename... A>
inline void launch(const char* kernel, int bound, void (*k)(P...), dim3 grid, dim3 block, size_t lds, hipStream_t s,
                   A&&... args) {
    if (!block_fits(kernel, bound, block)) return;
    k<<<grid, block, lds, s>>>(static_cast<P>(args)...);
}

inline unsigned ceil_div(unsigned a, unsigned b) { return (a + b - 1) / b; }

// Host fp32 restatements shared with the tone-mapping launcher (bit-identical to the oracle's
// float code: compiled without FMA contraction).
void agx_matrices(float compression, float M[9], float Minv[9]);
void mat4_mul_host(float out[16], const float a[16], const float b[16]);

// The bloom chain's exactly-halving mips (bloom_w.hip).
bool bloom_fused_applicable(const soc_img& emissive, const soc_img* mips, int mip_count, const soc_img& output);
// Weighted-form bloom chain (bloom_w.hip): same applicability as the fused chain.
int launch_bloom_weighted(const soc_img& emissive, const soc_img* mips, const soc_img& output, hipStream_t s, int stage);

// soc_composition_luminance_histogram with the fold of the 8 partial histograms optionally left to a
// separate histogram_fold_launch (the render graph times the fold as a pass of its own).
int composition_luminance_histogram(const soc_globals* g, const soc_globals* d_globals, soc_img target, soc_img albedo,
                                    soc_img emissive, soc_img normal, soc_img depth, soc_img ssao, soc_img shadow,
                                    soc_img clouds, soc_auto_exposure* ae, uint32_t* scratch, bool fold, soc_stream stream,
                                    bool sky_external = false, const soc_img* bloom_mip1 = nullptr);
// The fused pair path applies to these images at the globals' resolution (composition.hip).
bool composition_pair_applicable(const soc_globals* g, const soc_img& target, const soc_img& albedo,
                                 const soc_img& emissive, const soc_img& normal, const soc_img& depth,
                                 const soc_img& clouds);
// The sky pixels of the colour image (depth == 1 -> clouds texel) and their bins into the 8 partial histograms:
// the second-lane half of a Composition run with sky_external.
// soc_cloud_rendering; sky_bound (the render graph's sky lane runs at high priority): the variants that are faster
// only where the sky lane is the frame's critical path (the density grid at twice the resident set, the classification's
// hoisted depth samples). The same bits either way.
int cloud_rendering_launch(const soc_globals* g, soc_img depth, soc_img noise, soc_img target, void* workspace,
                           soc_stream stream, bool sky_bound);
int sky_compose_launch(const soc_globals* g, soc_img target, soc_img depth, soc_img clouds, uint32_t* scratch,
                       soc_stream stream);
int histogram_fold_launch(uint32_t* scratch, soc_auto_exposure* ae, soc_stream stream);
// soc_resolve_luminance_histogram that first folds the 8 partial histograms (null: none).
int resolve_luminance_histogram(const soc_globals* g, soc_auto_exposure* ae, uint64_t total_pixels, int32_t wide_accumulator,
                                uint32_t* scratch, soc_stream stream);

}  // namespace soc
