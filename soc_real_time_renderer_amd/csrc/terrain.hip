// terrain.hip — HeightToNormalTask (src/graphics/tasks/height_to_normal.inl:52-83) for gfx950.
//
// The reference converts its terrain heightmap (R8G8B8A8_UNORM, renderer.cpp:155) into an RGBA16F normal
// map once at load (renderer.cpp:158-190): per texel, the clamped up / down / right / left neighbours
// become points (x / size, height, y / size), and normal = normalize(cross(normalize(up - down),
// normalize(right - left))). One lane per texel, 64x4 workgroups: a wave reads three 256-B row segments
// of the heightmap (the vertical neighbours come from L1) and writes one 512-B row segment. The fp32
// arithmetic is written without contraction, in the oracle's order.
#include "soc_internal.hpp"

namespace soc {
namespace {

__device__ __forceinline__ f3 normalize_nc(f3 a) {
#pragma clang fp contract(off)
    const float l = sqrtf(a.x * a.x + a.y * a.y + a.z * a.z);
    return f3{a.x / l, a.y / l, a.z / l};
}

__global__ __launch_bounds__(256) void height_to_normal_kernel(DImg height, DImg target) {
#pragma clang fp contract(off)
    const int x = blockIdx.x * 64 + threadIdx.x, y = blockIdx.y * 4 + threadIdx.y;
    const int W = height.w, H = height.h;
    if (x >= W || y >= H) return;
    const int yu = min(y + 1, H - 1), yd = max(y - 1, 0), xr = min(x + 1, W - 1), xl = max(x - 1, 0);
    // imageLoad(u_heightmap, pos).r of an R8G8B8A8_UNORM image
    const float su = unorm8(row_ptr<uint32_t>(height, yu)[x] & 255u);
    const float sd = unorm8(row_ptr<uint32_t>(height, yd)[x] & 255u);
    const float sr = unorm8(row_ptr<uint32_t>(height, y)[xr] & 255u);
    const float sl = unorm8(row_ptr<uint32_t>(height, y)[xl] & 255u);
    const float fw = (float)W, fh = (float)H;
    const f3 pu{(float)x / fw, su, (float)yu / fh}, pd{(float)x / fw, sd, (float)yd / fh};
    const f3 pr{(float)xr / fw, sr, (float)y / fh}, pl{(float)xl / fw, sl, (float)y / fh};
    const f3 vd = normalize_nc(f3{pu.x - pd.x, pu.y - pd.y, pu.z - pd.z});
    const f3 hd = normalize_nc(f3{pr.x - pl.x, pr.y - pl.y, pr.z - pl.z});
    const f3 c = f3{vd.y * hd.z - vd.z * hd.y, vd.z * hd.x - vd.x * hd.z, vd.x * hd.y - vd.y * hd.x};
    const f3 n = normalize_nc(c);
    row_ptr_w<uint2>(target, y)[x] = pack_h4(f4{n.x, n.y, n.z, 1.0f});
}

}  // namespace
}  // namespace soc

using namespace soc;

extern "C" int soc_height_to_normal(soc_img heightmap, soc_img normal_target, soc_stream stream) {
    int rc = check_img(heightmap, SOC_FMT_RGBA8_UNORM, "soc_height_to_normal", "heightmap");
    if (!rc) rc = check_img(normal_target, SOC_FMT_RGBA16F, "soc_height_to_normal", "normal target");
    if (rc) return rc;
    if (heightmap.width != normal_target.width || heightmap.height != normal_target.height)
        return set_error(SOC_E_SHAPE, "soc_height_to_normal: the normal map must have the heightmap's extent");
    dim3 blk(64, 4), grd(ceil_div(heightmap.width, 64), ceil_div(heightmap.height, 4));
    height_to_normal_kernel<<<grd, blk, 0, hs(stream)>>>(dimg(heightmap), dimg(normal_target));
    return check_launch("height_to_normal");
}
