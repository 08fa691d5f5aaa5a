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

__global__ __launch_bounds__(kWorkgroup) void height_to_normal_kernel(DImg height, DImg target) {
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

// DrawTerrain's patch tessellation (draw_terrain.inl:138-191) of the grid_size^2 uv control grid
// (renderer.cpp:194-220): patch (i, j) has control points (i, j), (i, j+1), (i+1, j), (i+1, j+1) at uv
// (i, j) / (grid_size - 1); at level n (an odd integer: fractional_odd_spacing gives n equal segments)
// its tess vertex (a/n, b/n) has uv = lerp(lerp(cp0, cp1, a/n), lerp(cp2, cp3, a/n), b/n), the TES's
// operation order. Neighbouring patches meet on a shared vertex: the global vertex (gx, gz) of the
// ((grid-1) n + 1)^2 grid is evaluated by the lowest patch holding it. Height = the heightmap's .r,
// bilinear clamp-to-edge at that uv (linear_sampler), displaced by (h - midpoint) * height_scale along
// +y. The TES adds terrain_y_clip_trick (= projection_view * (0,1,0,0)) to its clip-space bilinear
// point; the world point below is that point before the (linear) clip transform.
struct TessParams {
    int grid, n, nv;   // control grid side, level, vertex grid side (grid - 1) n + 1
    float scale_x, scale_z, hscale, mid, off[3];
};

__global__ __launch_bounds__(kWorkgroup) void terrain_tess_vertices(DImg height, TessParams p, float* __restrict__ pos,
                                                             float* __restrict__ nrm, float* __restrict__ uvs) {
#pragma clang fp contract(off)
    const int k = blockIdx.x * 256 + threadIdx.x;
    if (k >= p.nv * p.nv) return;
    const int gz = k / p.nv, gx = k - gz * p.nv;   // gx along uv.x (control index i), gz along uv.y (j)
    const int pi = min(gx / p.n, p.grid - 2), pj = min(gz / p.n, p.grid - 2);
    const float fn = (float)p.n, side = (float)(p.grid - 1);
    const float tu = (float)(gz - pj * p.n) / fn;   // TES u: cp0 -> cp1 (j + 1)
    const float tv = (float)(gx - pi * p.n) / fn;   // TES v: (cp0, cp1) -> (cp2, cp3) (i + 1)
    const float i0 = (float)pi / side, i1 = (float)(pi + 1) / side, j0 = (float)pj / side, j1 = (float)(pj + 1) / side;
    // uv0 = (in_uv[1] - in_uv[0]) u + in_uv[0], uv1 = (in_uv[3] - in_uv[2]) u + in_uv[2], uv = (uv1 - uv0) v + uv0
    const float u0x = (i0 - i0) * tu + i0, u0y = (j1 - j0) * tu + j0;
    const float u1x = (i1 - i1) * tu + i1, u1y = (j1 - j0) * tu + j0;
    const float ux = (u1x - u0x) * tv + u0x, uy = (u1y - u0y) * tv + u0y;
    const float h = sample_rgba8(height, ux, uy).x;
    const float adj = (h - p.mid) * p.hscale;
    pos[3 * k] = ux * p.scale_x - p.off[0];
    pos[3 * k + 1] = p.off[1] + adj;
    pos[3 * k + 2] = uy * p.scale_z - p.off[2];
    nrm[3 * k] = 0.0f;   // the terrain's G-buffer normal comes from its normal map (draw_terrain.inl:206-219)
    nrm[3 * k + 1] = 1.0f;
    nrm[3 * k + 2] = 0.0f;
    uvs[2 * k] = ux;
    uvs[2 * k + 1] = uy;
}

// Two triangles per tessellated quad, counter-clockwise seen from above, the diagonal alternating with the
// triangle id's parity as the host terrain mesh (scene_synth.c).
__global__ __launch_bounds__(kWorkgroup) void terrain_tess_indices(int nv, uint32_t* __restrict__ idx) {
    const int id = blockIdx.x * 256 + threadIdx.x, segs = nv - 1;
    if (id >= 2 * segs * segs) return;
    const int q = id >> 1, qi = q % segs, qj = q / segs;
    const uint32_t v00 = (uint32_t)(qj * nv + qi), v10 = v00 + 1, v01 = v00 + (uint32_t)nv, v11 = v01 + 1;
    idx[3 * id] = v00;
    idx[3 * id + 1] = (id & 1) ? v01 : v11;
    idx[3 * id + 2] = (id & 1) ? v11 : v10;
}

}  // namespace
}  // namespace soc

using namespace soc;

extern "C" int soc_terrain_tess_counts(int32_t grid_size, int32_t tess_level, int32_t* vertices, int32_t* triangles) {
    if (grid_size < 2 || tess_level < 1 || !(tess_level & 1) || !vertices || !triangles)
        return set_error(SOC_E_INVALID_ARG, "soc_terrain_tess_counts: grid_size >= 2 and an odd tess_level >= 1");
    const long long nv = (long long)(grid_size - 1) * tess_level + 1;
    if (nv * nv > 0x7fffffffll / 3) return set_error(SOC_E_SHAPE, "soc_terrain_tess_counts: grid too large");
    *vertices = (int32_t)(nv * nv);
    *triangles = (int32_t)(2 * (nv - 1) * (nv - 1));
    return SOC_OK;
}

extern "C" int soc_terrain_tessellate(const soc_globals* g, soc_img heightmap, int32_t grid_size, int32_t tess_level,
                                      float* positions, float* normals, float* uvs, uint32_t* indices, soc_stream stream) {
    int32_t V = 0, T = 0;
    int rc = soc_terrain_tess_counts(grid_size, tess_level, &V, &T);
    if (!rc) rc = check_img(heightmap, SOC_FMT_RGBA8_UNORM, "soc_terrain_tessellate", "heightmap");
    if (rc) return rc;
    if (!g || !positions || !normals || !uvs || !indices)
        return set_error(SOC_E_INVALID_ARG, "soc_terrain_tessellate: null argument");
    TessParams p{};
    p.grid = grid_size;
    p.n = tess_level;
    p.nv = (grid_size - 1) * tess_level + 1;
    p.scale_x = g->terrain_scale[0];
    p.scale_z = g->terrain_scale[1];
    p.hscale = g->terrain_height_scale;
    p.mid = g->terrain_midpoint;
    for (int i = 0; i < 3; ++i) p.off[i] = g->terrain_offset[i];
    launch("terrain_tess_vertices", kWorkgroup, terrain_tess_vertices, ceil_div(V, 256), kWorkgroup, 0, hs(stream), dimg(heightmap), p, positions, normals, uvs);
    launch("terrain_tess_indices", kWorkgroup, terrain_tess_indices, ceil_div(T, 256), kWorkgroup, 0, hs(stream), p.nv, indices);
    return check_launch("terrain_tessellate");
}

extern "C" int soc_height_to_normal(soc_img heightmap, soc_img normal_target, soc_stream stream) {
    int rc = check_img(heightmap, SOC_FMT_RGBA8_UNORM, "soc_height_to_normal", "heightmap");
    if (!rc) rc = check_img(normal_target, SOC_FMT_RGBA16F, "soc_height_to_normal", "normal target");
    if (rc) return rc;
    if (heightmap.width != normal_target.width || heightmap.height != normal_target.height)
        return set_error(SOC_E_SHAPE, "soc_height_to_normal: the normal map must have the heightmap's extent");
    dim3 blk(64, 4), grd(ceil_div(heightmap.width, 64), ceil_div(heightmap.height, 4));
    launch("height_to_normal_kernel", kWorkgroup, height_to_normal_kernel, grd, blk, 0, hs(stream), dimg(heightmap), dimg(normal_target));
    return check_launch("height_to_normal");
}
