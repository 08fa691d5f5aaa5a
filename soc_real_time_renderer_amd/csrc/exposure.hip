// exposure.hip — GenerateLuminanceHistogramTask (src/graphics/tasks/generate_luminance_histogram.inl:23-47,
// shader :59-78) and ResolveLuminanceHistogramTask (resolve_luminance_histogram.inl:20-43, shader
// :56-80) as gfx950 kernels.
//
// Histogram: a grid of ~2 workgroups per CU streams the RGBA16F colour image with 16-B loads (8
// pixels = 64 B per lane per step). Each lane run-length merges the bins of its 8 consecutive pixels
// (neighbouring pixels usually share a bin) before one LDS atomic per run into its wave's private
// 256-bin copy; the block then folds the 4 copies and issues one device atomic per NON-ZERO bin.
// The bin function is the bit-exact contract of DESIGN.md §3.4 (explicit-FMA luminance and remap,
// deterministic log2), identical to the oracle's; the fast path evaluates it with the hardware log2 and
// falls back to the exact form for pixels near a bin boundary (lum_bin_fast, luminance.hpp).
#include <type_traits>
#include <algorithm>

#include <cstdlib>

#include "luminance.hpp"
#include "soc_internal.hpp"

namespace soc {
namespace {

constexpr int kThreads = 256, kWaves = kThreads / 64, kPix = 8;

// Fast path: W % 8 == 0, rows 16-B aligned. One "chunk" = 8 consecutive pixels of a row.
__global__ __launch_bounds__(kThreads) void histogram_chunks(DImg hdr, int W, int H, float lmin, float lrange,
                                                             BinFast bf, uint32_t* __restrict__ bins) {
    __shared__ uint32_t sh[kWaves][kBins];
    const int tid = threadIdx.x, wave = tid >> 6;
    for (int i = tid; i < kWaves * kBins; i += kThreads) (&sh[0][0])[i] = 0u;
    __syncthreads();
    const int cpr = W / kPix;                       // chunks per row
    const long long total = (long long)cpr * H;
    const long long stride = (long long)gridDim.x * kThreads;
    // software pipelined: the next chunk's 64 B are in flight while this chunk is binned
    auto fetch = [&](long long c, uint4 (&q)[kPix / 2]) {
        const int y = (int)(c / cpr), cx = (int)(c - (long long)y * cpr);
        const uint4* p = row_ptr<uint4>(hdr, y) + cx * (kPix / 2);
#pragma unroll
        for (int k = 0; k < kPix / 2; ++k) q[k] = p[k];
    };
    long long c = (long long)blockIdx.x * kThreads + tid;
    uint4 nxt[kPix / 2];
    if (c < total) fetch(c, nxt);
    for (; c < total; c += stride) {
        uint4 q[kPix / 2];
#pragma unroll
        for (int k = 0; k < kPix / 2; ++k) q[k] = nxt[k];
        if (c + stride < total) fetch(c + stride, nxt);
        // fast bins (hardware log2) for the 8 pixels, then lum_bin for the few near a bin boundary
        uint32_t bq[kPix], need = 0;
#pragma unroll
        for (int k = 0; k < kPix / 2; ++k) {
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const f4 c4 = unpack_h4(h ? uint2{q[k].z, q[k].w} : uint2{q[k].x, q[k].y});
                bq[2 * k + h] = lum_bin_fast(c4.x, c4.y, c4.z, bf);
                need |= (bq[2 * k + h] == kBinExact ? 1u : 0u) << (2 * k + h);
            }
        }
        if (need) {
#pragma unroll
            for (int k = 0; k < kPix / 2; ++k) {
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    if ((need >> (2 * k + h)) & 1u) {
                        const f4 c4 = unpack_h4(h ? uint2{q[k].z, q[k].w} : uint2{q[k].x, q[k].y});
                        bq[2 * k + h] = lum_bin(c4.x, c4.y, c4.z, lmin, lrange);
                    }
                }
            }
        }
        uint32_t cur = 0xffffffffu, run = 0;
#pragma unroll
        for (int k = 0; k < kPix / 2; ++k) {
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const uint32_t b = bq[2 * k + h];
                if (b == cur) {
                    ++run;
                } else {
                    if (run) atomicAdd(&sh[wave][cur], run);
                    cur = b;
                    run = 1;
                }
            }
        }
        if (run) atomicAdd(&sh[wave][cur], run);
    }
    __syncthreads();
    for (int i = tid; i < kBins; i += kThreads) {
        uint32_t s = 0;
#pragma unroll
        for (int w = 0; w < kWaves; ++w) s += sh[w][i];
        if (s) atomicAdd(&bins[i], s);
    }
}

// Generic path: one pixel per lane (any width / alignment).
__global__ __launch_bounds__(kThreads) void histogram_pixels(DImg hdr, int W, int H, float lmin, float lrange,
                                                             uint32_t* __restrict__ bins) {
    __shared__ uint32_t sh[kBins];
    const int tid = threadIdx.x;
    sh[tid] = 0u;
    __syncthreads();
    const long long total = (long long)W * H;
    for (long long i = (long long)blockIdx.x * kThreads + tid; i < total; i += (long long)gridDim.x * kThreads) {
        const int y = (int)(i / W), x = (int)(i - (long long)y * W);
        const f4 c = fetch_h4(hdr, x, y);
        atomicAdd(&sh[lum_bin(c.x, c.y, c.z, lmin, lrange)], 1u);
    }
    __syncthreads();
    if (sh[tid]) atomicAdd(&bins[tid], sh[tid]);
}

// resolve_luminance_histogram.inl:56-80, one workgroup of 256 lanes (quirk Q9: the reference's extra
// 255 workgroups only index out of bounds).
// scratch != null: the 8 partial histograms of the fused composition pass are folded in here (u32 adds,
// the same bins histogram_fold would leave) and re-zeroed, saving that launch in a single-GPU frame.
template <bool WIDE>
__global__ __launch_bounds__(kBins) void resolve_kernel(soc_auto_exposure* __restrict__ ae, float pixels, float lmin,
                                                        float lmax, float target_lum, float dt, float speed,
                                                        uint32_t* __restrict__ scratch) {
    typedef typename std::conditional<WIDE, unsigned long long, uint32_t>::type acc_t;
    __shared__ acc_t sh[kBins];
    const uint32_t i = threadIdx.x;
    uint32_t count = ae->histogram_buckets[i];
    if (scratch) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            count += scratch[k * kBins + i];
            scratch[k * kBins + i] = 0u;
        }
    }
    sh[i] = (acc_t)count * (acc_t)i;
    ae->histogram_buckets[i] = 0u;
    __syncthreads();
    for (uint32_t th = kBins / 2; th > 0; th /= 2) {
        if (i < th) sh[i] += sh[i + th];
        __syncthreads();
    }
    if (i == 0) {
        const float num_black = (float)count;
        const float x = (float)sh[0] / fmaxf(pixels - num_black, 1.0f);
        const float log2_mean = (x - 1.0f) / (256.0f - 1.0f) * (lmax - lmin) + lmin;
        const float tgt = log2f(target_lum / exp2f(log2_mean));
        const float alpha = clampf(1.0f - expf(-dt * speed), 0.0f, 1.0f);
        ae->exposure = mixf(ae->exposure, tgt, alpha);
    }
}

int g_hist_blocks = 0;

int hist_grid() {
    if (!g_hist_blocks) {
        int dev = 0, cus = 256;
        if (hipGetDevice(&dev) == hipSuccess) {
            hipDeviceProp_t prop;
            if (hipGetDeviceProperties(&prop, dev) == hipSuccess && prop.multiProcessorCount > 0) cus = prop.multiProcessorCount;
        }
        const char* e = getenv("SOC_HIST_BLOCKS_PER_CU");   // tuning knob
        g_hist_blocks = (e ? atoi(e) : 2) * cus;
    }
    return g_hist_blocks;
}

}  // namespace
}  // namespace soc

using namespace soc;

extern "C" int soc_generate_luminance_histogram(const soc_globals* g, soc_img hdr, soc_auto_exposure* ae, soc_stream stream) {
    static const char* P = "soc_generate_luminance_histogram";
    if (!g || !ae) return set_error(SOC_E_INVALID_ARG, "%s: null globals / auto exposure buffer", P);
    int rc = check_img(hdr, SOC_FMT_RGBA16F, P, "hdr");
    if (rc) return rc;
    const int W = g->resolution[0] < hdr.width ? g->resolution[0] : hdr.width;
    const int H = g->resolution[1] < hdr.height ? g->resolution[1] : hdr.height;
    if (W <= 0 || H <= 0) return SOC_OK;
    const float lmin = g->log_min_luminance, lrange = g->log_max_luminance - g->log_min_luminance;
    const long long px = (long long)W * H;
    const bool chunks = (W % kPix == 0) && (reinterpret_cast<uintptr_t>(hdr.data) & 15u) == 0 && (hdr.pitch_bytes & 15) == 0;
    const long long work = chunks ? px / kPix : px;
    int grid = (int)std::min<long long>(hist_grid(), (work + kThreads - 1) / kThreads);
    if (grid < 1) grid = 1;
    uint32_t* bins = ae->histogram_buckets;
    if (chunks)
        launch("histogram_chunks", kThreads, histogram_chunks, grid, kThreads, 0, hs(stream), dimg(hdr), W, H, lmin, lrange, bin_fast_params(lmin, lrange), bins);
    else
        launch("histogram_pixels", kThreads, histogram_pixels, grid, kThreads, 0, hs(stream), dimg(hdr), W, H, lmin, lrange, bins);
    return check_launch("generate_luminance_histogram");
}

int soc::resolve_luminance_histogram(const soc_globals* g, soc_auto_exposure* ae, uint64_t total_pixels,
                                     int32_t wide_accumulator, uint32_t* scratch, soc_stream stream) {
    if (!g || !ae) return set_error(SOC_E_INVALID_ARG, "soc_resolve_luminance_histogram: null argument");
    float pixels = total_pixels ? (float)total_pixels
                                : (float)(int32_t)((uint32_t)g->resolution[0] * (uint32_t)g->resolution[1]);
    if (wide_accumulator)
        launch("resolve_kernel", kBins, resolve_kernel<true>, 1, kBins, 0, hs(stream), ae, pixels, g->log_min_luminance, g->log_max_luminance,
                                                          g->target_luminance, g->delta_time, g->adjustment_speed, scratch);
    else
        launch("resolve_kernel", kBins, resolve_kernel<false>, 1, kBins, 0, hs(stream), ae, pixels, g->log_min_luminance, g->log_max_luminance,
                                                           g->target_luminance, g->delta_time, g->adjustment_speed, scratch);
    return check_launch("resolve_luminance_histogram");
}

extern "C" int soc_resolve_luminance_histogram(const soc_globals* g, soc_auto_exposure* ae, uint64_t total_pixels,
                                               int32_t wide_accumulator, soc_stream stream) {
    return resolve_luminance_histogram(g, ae, total_pixels, wide_accumulator, nullptr, stream);
}
