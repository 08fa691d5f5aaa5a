// hiz.hip — GenerateMinHIZTask / GenerateMaxHIZTask (generate_min_hiz.inl:23-95, generate_max_hiz.inl,
// shader generate_hiz.glsl:17-98) for gfx950: a single-pass min or max depth pyramid.
//
// Like the reference, one 256-lane workgroup reduces a 64x64 window of the full-resolution depth to mips
// 0..5 (mip 0 = half resolution; mips 2..5 through an LDS ping-pong) and the LAST workgroup to finish
// (a device-scope arrival counter, one atomic per workgroup) reduces mip 5 to the remaining levels.
// Quirks kept: the window reads clamp to the image (the gather's clamp-to-edge), values of texels
// beyond a mip's extent stay in the LDS reduction (only in-extent texels are stored), and the tail pass
// covers one 64x64 window of mip 5. min / max are exact, so the result does not depend on the order.
// Hi-Z is computed but not read by the reference graph (quirk Q12); it is here for the terrain row f3.
#include <algorithm>

#include "soc_internal.hpp"

namespace soc {
namespace {

constexpr int HIZ_MAX_MIPS = 12;   // GENERATE_HIZ_LEVELS_PER_DISPATCH

struct HizMips {
    DImg m[HIZ_MAX_MIPS];
    int count;
};

template <bool MAX>
__device__ __forceinline__ float op(float a, float b) { return MAX ? fmaxf(a, b) : fminf(a, b); }

__device__ __forceinline__ void store_mip(const HizMips& mips, int level, int x, int y, float v) {
    if (level >= mips.count) return;   // the reference's stores to absent levels are discarded
    const DImg& d = mips.m[level];
    if (x < d.w && y < d.h) row_ptr_w<float>(d, y)[x] = v;
}

// downsample_64x64 (generate_hiz.glsl:17-84). src_level -1 reads the full-res depth; otherwise mip
// src_level, clamped to src_w x src_h.
template <bool MAX>
__device__ void downsample_64x64(float (*sh)[16][16], int lx, int ly, int gx, int gy, const DImg& src, int src_w, int src_h,
                                 int src_level, int levels, const HizMips& mips) {
    float quad[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int sx = q >> 1, sy = q & 1;
        const int ix = ((gx * 16 + lx) * 2 + sx) * 2, iy = ((gy * 16 + ly) * 2 + sy) * 2;
        const int x0 = min(ix, src_w - 1), x1 = min(ix + 1, src_w - 1), y0 = min(iy, src_h - 1), y1 = min(iy + 1, src_h - 1);
        const float a = row_ptr<float>(src, y0)[x0], b = row_ptr<float>(src, y1)[x0];
        const float c = row_ptr<float>(src, y0)[x1], d = row_ptr<float>(src, y1)[x1];
        const float m = op<MAX>(op<MAX>(a, b), op<MAX>(c, d));
        store_mip(mips, src_level + 1, (gx * 16 + lx) * 2 + sx, (gy * 16 + ly) * 2 + sy, m);
        quad[q] = m;
    }
    const float m1 = op<MAX>(op<MAX>(quad[0], quad[1]), op<MAX>(quad[2], quad[3]));
    store_mip(mips, src_level + 2, gx * 16 + lx, gy * 16 + ly, m1);
    sh[0][ly][lx] = m1;
    const int ox = 32 * gx, oy = 32 * gy;   // (window * grid) / 2
    for (int i = 2; i < levels; ++i) {
        const int s = i & 1, t = (i + 1) & 1;
        __syncthreads();
        if (lx < (64 >> (i + 1)) && ly < (64 >> (i + 1))) {
            const float m = op<MAX>(op<MAX>(sh[s][2 * ly][2 * lx], sh[s][2 * ly][2 * lx + 1]),
                                    op<MAX>(sh[s][2 * ly + 1][2 * lx], sh[s][2 * ly + 1][2 * lx + 1]));
            store_mip(mips, src_level + i + 1, (ox >> i) + lx, (oy >> i) + ly, m);
            sh[t][ly][lx] = m;
        }
    }
}

template <bool MAX>
__global__ __launch_bounds__(kWorkgroup) void hiz_kernel(DImg depth, HizMips mips, uint32_t* __restrict__ counter,
                                                  uint32_t total, int res_w, int res_h) {
    __shared__ float sh[2][16][16];
    __shared__ bool last;
    const int lx = threadIdx.x, ly = threadIdx.y;
    downsample_64x64<MAX>(sh, lx, ly, blockIdx.x, blockIdx.y, depth, depth.w, depth.h, -1, 6, mips);
    __threadfence();   // this workgroup's mip stores before its arrival
    __syncthreads();
    if (lx == 0 && ly == 0) last = atomicAdd(counter, 1u) + 1u == total;
    __syncthreads();
    // the tail reads mip 5 at min(index, extent - 1) (generate_hiz.glsl:29-32): an extent of 0 (a frame under 64 texels
    // across) would read outside the image, which the reference leaves undefined; the tail levels are then not written
    if (last && mips.count > 5 && (res_w >> 6) > 0 && (res_h >> 6) > 0) {
        __threadfence();
        // mip 5 of the other workgroups, read back through L2 (the reference's coherent image accesses)
        downsample_64x64<MAX>(sh, lx, ly, 0, 0, mips.m[5], res_w >> 6, res_h >> 6, 5, mips.count - 6, mips);
    }
}

}  // namespace
}  // namespace soc

using namespace soc;

extern "C" int soc_generate_hiz(const soc_globals* g, soc_img depth, const soc_img* mips, int32_t mip_count,
                                int32_t op_max, uint32_t* counter, soc_stream stream) {
    if (!g || !mips || !counter || mip_count <= 0 || mip_count > HIZ_MAX_MIPS)
        return set_error(SOC_E_INVALID_ARG, "soc_generate_hiz: null argument or mip count outside 1..12");
    int rc = check_img(depth, SOC_FMT_D32F, "soc_generate_hiz", "depth");
    if (rc) return rc;
    const int W = g->resolution[0], H = g->resolution[1];
    if (depth.width != W || depth.height != H)
        return set_error(SOC_E_SHAPE, "soc_generate_hiz: depth must have the frame resolution");
    HizMips hm{};
    hm.count = mip_count;
    for (int i = 0; i < mip_count; ++i) {
        rc = check_img(mips[i], SOC_FMT_D32F, "soc_generate_hiz", "mip");
        if (rc) return rc;
        const int ew = std::max(1, (W / 2) >> i), eh = std::max(1, (H / 2) >> i);
        if (mips[i].width != ew || mips[i].height != eh)
            return set_error(SOC_E_SHAPE, "soc_generate_hiz: mip %d must be %dx%d", i, ew, eh);
        hm.m[i] = dimg(mips[i]);
    }
    hipStream_t s = hs(stream);
    if (hipMemsetAsync(counter, 0, sizeof(uint32_t), s) != hipSuccess)
        return set_error(SOC_E_HIP, "soc_generate_hiz: counter reset failed");
    const dim3 grd(ceil_div(W, 64), ceil_div(H, 64)), blk(16, 16);
    if (op_max) launch("hiz_kernel", kWorkgroup, hiz_kernel<true>, grd, blk, 0, s, dimg(depth), hm, counter, grd.x * grd.y, W, H);
    else launch("hiz_kernel", kWorkgroup, hiz_kernel<false>, grd, blk, 0, s, dimg(depth), hm, counter, grd.x * grd.y, W, H);
    return check_launch("generate_hiz");
}
