// raster.hip — depth prepass / G-buffer / sun-shadow rasterisation for gfx950.
//
// Replaces the reference's fixed-function raster producers upstream of the screen-space chain:
//   DepthPrepassTask      depth_prepass.inl:26-120      (cull FRONT, LESS_OR_EQUAL)
//   GBufferGenerationTask g_buffer_generation.inl:33-230 (cull FRONT, LESS_OR_EQUAL, depth LOAD)
//   SunShadowDrawTask     sun_shadow_draw.inl:27-91     (cull BACK, depth bias 1.25 / 1.75)
// gfx950 has no raster units reachable from HIP, so the raster is a compute visibility buffer:
//   1. raster_setup     one lane per vertex: object -> world -> clip -> screen (x, y, z_ndc, 1/w)
//   2. raster_small     one lane per triangle: cull, bounding box; a box of <= SMALL_PIXELS pixels is
//                       scanned by the lane itself, larger ones are split into 32x32-pixel tiles
//   3. raster_big       one wave per (triangle, tile) work item: tiles that an edge function excludes at
//                       all four corners (with a rounding margin) are skipped, else 64 lanes cover the
//                       tile's 1024 pixels
//   every covered pixel does ONE 64-bit atomicMin of (depth bits << 32 | 0xFFFFFFFE - triangle): with
//   z >= 0 the float bits order like the depths, and ties keep the LATER triangle, which is exactly the
//   serial LESS_OR_EQUAL result in draw order. The depth-only variant (shadow map) does a 32-bit
//   atomicMin of the biased depth bits straight into the D32 image.
//   4. gbuffer_resolve  one lane per pixel: the winning triangle's perspective-correct barycentrics,
//                       attribute interpolation and the GBufferGeneration fragment shader
//                       (g_buffer_generation.inl:189-225).
// The coverage, depth and barycentric arithmetic is written without FMA contraction and matches the
// oracle's (oracle/soc_oracle.c, soc_oracle_raster_*) operation for operation, so the visibility buffer
// and the depth images are bit-exact against it.
#include "luminance.hpp"
#include "soc_internal.hpp"

namespace soc {
namespace {

constexpr int SMALL_PIXELS = 64;    // bounding boxes up to this many pixels are scanned by one lane
#ifndef SOC_RASTER_TILE
#define SOC_RASTER_TILE 32
#endif
constexpr int TILE = SOC_RASTER_TILE;   // large-triangle work item: a TILE x TILE tile of its bounding box
#ifndef SOC_RASTER_FIXED_COLS
#define SOC_RASTER_FIXED_COLS 0   // A/B builds: raster_big's lanes as 32 x 2 pixels whatever the item's width
#endif
static_assert(TILE == 32 || SOC_RASTER_FIXED_COLS, "raster_big's lane layout covers items up to 32 pixels wide");
constexpr uint32_t KEY_EMPTY = 0xFFFFFFFFu;

struct RasterParams {
    Mat4 model, vp;
    int width, height, vertex_count, triangle_count;
    int cull;
    int depth_only;
    float bias_constant, bias_slope;
    int small_pixels;   // boxes up to this many pixels are scanned by one lane
};

// workspace: [float4 clip-space screen vertices[V]] [u64 counter, pad..] [uint2 entries[T]]
// The counter packs (large triangles << 40 | tiles so far): one 64-bit atomicAdd per large triangle
// returns its entry slot and the first index of its tile range together, so the entries are in
// increasing range order and a work index finds its triangle by binary search.
struct Workspace {
    float4* screen;
    unsigned long long* counter;
    uint2* entries;   // {triangle, first tile index (low 32 bits of the range start)}
    float4* vdata;    // G-buffer resolve: 4 float4 per vertex (gbuffer_vertex_setup)
};
constexpr int ENTRY_SHIFT = 40;

inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

inline Workspace carve(void* ws, int V, int T) {
    char* p = static_cast<char*>(ws);
    Workspace w;
    w.screen = reinterpret_cast<float4*>(p);
    size_t off = align_up((size_t)V * 16, 256);
    w.counter = reinterpret_cast<unsigned long long*>(p + off);
    off += 256;
    w.entries = reinterpret_cast<uint2*>(p + off);
    off = align_up(off + (size_t)T * 8, 256);
    w.vdata = reinterpret_cast<float4*>(p + off);
    return w;
}

// GLSL mat4 * vec4, summed left to right, no contraction (the oracle's mat_vec).
__device__ __forceinline__ f4 mat_vec_exact(const Mat4& M, float x, float y, float z, float w) {
#pragma clang fp contract(off)
    const float* m = M.m;
    return f4{m[0] * x + m[4] * y + m[8] * z + m[12] * w, m[1] * x + m[5] * y + m[9] * z + m[13] * w,
              m[2] * x + m[6] * y + m[10] * z + m[14] * w, m[3] * x + m[7] * y + m[11] * z + m[15] * w};
}

// Homogeneous screen-space vertex (2DH rasterisation, Olano & Greer): X = (x_c/2 + w_c/2) W,
// Y = (y_c/2 + w_c/2) H (y = 0 top row, uv = ndc * 0.5 + 0.5), Z = z_c, W = w_c. No division, so
// vertices behind the eye need no geometric clipping; fragments with z_ndc outside [0, 1] are clipped
// per pixel (Vulkan depth clipping; the reference's RH_NO projection puts z_c = 0 between near and far).
__device__ __forceinline__ float4 clip_vertex(const float* __restrict__ pos, int v, const Mat4& model, const Mat4& vp,
                                              int W, int H) {
#pragma clang fp contract(off)
    const float px = pos[3 * v], py = pos[3 * v + 1], pz = pos[3 * v + 2];
    const f4 wp = mat_vec_exact(model, px, py, pz, 1.0f);
    const f4 c = mat_vec_exact(vp, wp.x, wp.y, wp.z, wp.w);
    return float4{(c.x * 0.5f + c.w * 0.5f) * (float)W, (c.y * 0.5f + c.w * 0.5f) * (float)H, c.z, c.w};
}

__device__ __forceinline__ f3 cross_exact(f3 a, f3 b) {
#pragma clang fp contract(off)
    return f3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}

struct TriSetup {
    f3 r0, r1, r2;          // edge functions E_i(p) = r_i . (px, py, 1), sign-normalised: inside iff all >= 0
    float z0, z1, z2, w0, w1, w2;
    float bias;
    int px0, px1, py0, py1;
    bool live;
};

// Screen bounding box of the part of a triangle in front of the depth-clip plane z_c = 0: its vertices there and its
// edges' crossings of the plane, projected (wide: a point at w <= 1e-20, the box is the whole image). Plain values and
// flags in a struct (a capturing lambda here had its two flags spilled to scratch).
struct BBox {
    float minx = 3.0e38f, maxx = -3.0e38f, miny = 3.0e38f, maxy = -3.0e38f;
    bool any = false, wide = false;
};
__device__ __forceinline__ void bbox_add(BBox& b, float X, float Y, float Wc) {
#pragma clang fp contract(off)
    if (!(Wc > 1e-20f)) {
        b.wide = true;
        return;
    }
    const float x = X / Wc, y = Y / Wc;
    b.minx = fminf(b.minx, x); b.maxx = fmaxf(b.maxx, x);
    b.miny = fminf(b.miny, y); b.maxy = fmaxf(b.maxy, y);
    b.any = true;
}
// vertex a, and where the edge a -> b crosses z_c = 0
__device__ __forceinline__ void bbox_edge(BBox& bb, float4 a, float4 b) {
#pragma clang fp contract(off)
    if (a.z >= 0.0f) bbox_add(bb, a.x, a.y, a.w);
    if ((a.z >= 0.0f) != (b.z >= 0.0f)) {
        const float u = a.z / (a.z - b.z);
        bbox_add(bb, a.x + u * (b.x - a.x), a.y + u * (b.y - a.y), a.w + u * (b.w - a.w));
    }
}

// Triangle setup: the adjugate rows r_i of [v0 v1 v2] (v = (X, Y, W)), det = v0 . r0. Facing is the
// sign of det (= the sign of the framebuffer area when every w > 0; Vulkan a = -area/2 < 0 is
// clockwise = front, the reference pipelines' winding: see soc_rt.h). Bounding box from the projected vertices when every w > 1e-6, else the
// whole image. Depth bias: z_ndc = (sum z_i r_i) . p / |det| is affine in the pixel position.
__device__ __forceinline__ TriSetup tri_setup(float4 A, float4 B, float4 C, const RasterParams& p) {
#pragma clang fp contract(off)
    TriSetup t;
    t.live = false;
    // Wholly beyond the far plane: every vertex has w_c > 0 and z_c > w_c (1 + 2^-12). A covered pixel's E_i are >= 0, so
    // z_ndc = sum E_i z_i / sum E_i w_i sums non-negative terms, each fp32 rounding is relative (<= 7 of 2^-24 in all),
    // and the ratio is >= min z_i / w_i >= 1 + 2^-12: the computed z_ndc is > 1 and cover() clips every pixel. Skipping
    // the triangle writes the same (nothing). The sun's orthographic frustum leaves most of the mesh beyond its far plane.
    {
        constexpr float kFar = 1.0f + 1.0f / 4096.0f;
        if (A.w > 0.0f && B.w > 0.0f && C.w > 0.0f && A.z > A.w * kFar && B.z > B.w * kFar && C.z > C.w * kFar) return t;
    }
    const f3 v0{A.x, A.y, A.w}, v1{B.x, B.y, B.w}, v2{C.x, C.y, C.w};
    f3 r0 = cross_exact(v1, v2), r1 = cross_exact(v2, v0), r2 = cross_exact(v0, v1);
    const float det = v0.x * r0.x + v0.y * r0.y + v0.z * r0.z;
    if (!(det != 0.0f) || det != det) return t;
    if (p.cull == SOC_CULL_FRONT && det > 0.0f) return t;
    if (p.cull == SOC_CULL_BACK && det < 0.0f) return t;
    if (det < 0.0f) { r0 = -r0; r1 = -r1; r2 = -r2; }
    t.r0 = r0; t.r1 = r1; t.r2 = r2;
    t.z0 = A.z; t.z1 = B.z; t.z2 = C.z;
    t.w0 = A.w; t.w1 = B.w; t.w2 = C.w;
    // Bounding box of the triangle clipped to z_c >= 0 (fragments below it are depth-clipped anyway, and
    // there w > 0 for a perspective or orthographic projection), one pixel of margin: a superset of the
    // covered centres. The oracle scans the whole image for such triangles; coverage itself is decided
    // per pixel by the edge functions only, so the results are identical.
    {
        BBox bb;
        bbox_edge(bb, A, B);
        bbox_edge(bb, B, C);
        bbox_edge(bb, C, A);
        const float minx = bb.minx, maxx = bb.maxx, miny = bb.miny, maxy = bb.maxy;
        const bool any = bb.any, wide = bb.wide;
        if (!any && !wide) return t;   // wholly behind the depth-clip plane
        const float W = (float)p.width, H = (float)p.height;
        if (wide || minx != minx || miny != miny || maxx != maxx || maxy != maxy) {
            t.px0 = 0; t.px1 = p.width - 1; t.py0 = 0; t.py1 = p.height - 1;
        } else {
            t.px0 = max(0, (int)floorf(fminf(fmaxf(minx - 1.5f, -1.0f), W)));
            t.px1 = min(p.width - 1, (int)ceilf(fminf(fmaxf(maxx + 0.5f, -1.0f), W)));
            t.py0 = max(0, (int)floorf(fminf(fmaxf(miny - 1.5f, -1.0f), H)));
            t.py1 = min(p.height - 1, (int)ceilf(fminf(fmaxf(maxy + 0.5f, -1.0f), H)));
        }
    }
    if (t.px0 > t.px1 || t.py0 > t.py1) return t;
    t.bias = 0.0f;
    if (p.depth_only) {   // Vulkan depth bias: m * slope + r * constant
        const float adet = fabsf(det);
        const float nx = A.z * r0.x + B.z * r1.x + C.z * r2.x, ny = A.z * r0.y + B.z * r1.y + C.z * r2.y;
        const float m = fmaxf(fabsf(nx / adet), fabsf(ny / adet));
        // r = 2^(E - 23), E the exponent of the largest |z_ndc| at a vertex (in front of the eye)
        float zmax = 0.0f;
        if (A.w > 0.0f) zmax = fmaxf(zmax, fabsf(A.z / A.w));
        if (B.w > 0.0f) zmax = fmaxf(zmax, fabsf(B.z / B.w));
        if (C.w > 0.0f) zmax = fmaxf(zmax, fabsf(C.z / C.w));
        const uint32_t ebits = (__float_as_uint(zmax) >> 23) & 255u;
        const float r = (ebits == 0u || ebits == 255u) ? 0.0f : ldexpf(1.0f, (int)ebits - 127 - 23);
        t.bias = m * p.bias_slope + r * p.bias_constant;
    }
    t.live = true;
    return t;
}

// An edge owns the pixel centres exactly on it iff its normal (r.x, r.y) points to +x, or to +y when
// vertical: shared edges have exactly negated coefficients, so each such centre is covered once.
__device__ __forceinline__ bool owns(f3 r) { return r.x > 0.0f || (r.x == 0.0f && r.y > 0.0f); }

__device__ __forceinline__ float edge(f3 r, float px, float py) {
#pragma clang fp contract(off)
    return r.x * px + r.y * py + r.z;
}

// Coverage of pixel (x, y): the three edge functions at the pixel centre, the tie rule, then
// z_ndc = sum E_i z_i / sum E_i w_i and depth clipping. e0..e2 are returned for the barycentrics
// (perspective-correct b_i = E_i / sum E). z is +0 for a -0 result.
__device__ __forceinline__ bool cover(const TriSetup& t, int x, int y, float& e0, float& e1, float& e2, float& z) {
#pragma clang fp contract(off)
    const float fx = (float)x + 0.5f, fy = (float)y + 0.5f;
    e0 = edge(t.r0, fx, fy);
    e1 = edge(t.r1, fx, fy);
    e2 = edge(t.r2, fx, fy);
    if (e0 < 0.0f || e1 < 0.0f || e2 < 0.0f) return false;
    if (e0 == 0.0f && !owns(t.r0)) return false;
    if (e1 == 0.0f && !owns(t.r1)) return false;
    if (e2 == 0.0f && !owns(t.r2)) return false;
    const float num = e0 * t.z0 + e1 * t.z1 + e2 * t.z2, den = e0 * t.w0 + e1 * t.w1 + e2 * t.w2;
    if (!(den > 0.0f)) return false;   // the pixel sees the triangle's plane behind the eye (or all E = 0)
    z = num / den;
    if (z < 0.0f || z > 1.0f) return false;   // depth clipping (NaN passes here and never wins below)
    z = z + 0.0f;                              // -0 -> +0: the key's bit order needs z >= +0
    return true;
}

__device__ __forceinline__ void shade(const TriSetup& t, int id, int x, int y, const RasterParams& p, void* target,
                                      size_t pitch) {
    float e0, e1, e2, z;
    if (!cover(t, x, y, e0, e1, e2, z)) return;
    // a plain load first: values only decrease, so a stale (larger) value never skips a needed atomic
    if (p.depth_only) {
#pragma clang fp contract(off)
        const float zb = fminf(fmaxf(z + t.bias, 0.0f), 1.0f);
        uint32_t* d = reinterpret_cast<uint32_t*>(static_cast<char*>(target) + (size_t)y * pitch) + x;
        const uint32_t key = __float_as_uint(zb);
        atomicMin(d, key);
    } else {
        const unsigned long long key = ((unsigned long long)__float_as_uint(z) << 32) | (unsigned long long)(0xFFFFFFFEu - (uint32_t)id);
        unsigned long long* d = reinterpret_cast<unsigned long long*>(static_cast<char*>(target) + (size_t)y * pitch) + x;
        atomicMin(d, key);
    }
}

__device__ __forceinline__ TriSetup load_tri(const Workspace& ws, const uint32_t* __restrict__ idx, int id,
                                             const RasterParams& p) {
    const uint32_t a = idx[3 * id], b = idx[3 * id + 1], c = idx[3 * id + 2];
    return tri_setup(ws.screen[a], ws.screen[b], ws.screen[c], p);
}

__global__ __launch_bounds__(kWorkgroup) void raster_setup(const float* __restrict__ pos, Workspace ws, RasterParams p) {
    const int v = blockIdx.x * 256 + threadIdx.x;
    if (v == 0) *ws.counter = 0ull;
    if (v >= p.vertex_count) return;
    ws.screen[v] = clip_vertex(pos, v, p.model, p.vp, p.width, p.height);
}

__global__ __launch_bounds__(kWorkgroup) void raster_clear_vis(unsigned long long* vis, size_t n) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) vis[i] = ((unsigned long long)__float_as_uint(1.0f) << 32) | KEY_EMPTY;
}

// The large triangles' entries are reserved once per workgroup: an LDS atomic gives each its offset in the workgroup's
// share and one global atomic on the packed counter reserves the share (one returning atomic on the one counter per
// wave cost ~40 us at 4K: the counter serialises them). The packed adds keep the entry slots and their tile ranges
// increasing together, as raster_big's search needs (SOC_RASTER_WG_ENTRIES=0: one atomic per wave, as before).
#ifndef SOC_RASTER_WG_ENTRIES
#define SOC_RASTER_WG_ENTRIES 1
#endif
__global__ __launch_bounds__(kWorkgroup) void raster_small(const uint32_t* __restrict__ idx, Workspace ws, RasterParams p,
                                                    void* target, size_t pitch) {
    const int id = blockIdx.x * 256 + threadIdx.x;
    TriSetup t{};
    t.live = false;
    if (id < p.triangle_count) t = load_tri(ws, idx, id, p);
    const int bw = t.px1 - t.px0 + 1, bh = t.py1 - t.py0 + 1;
    const bool big = t.live && (long long)bw * bh > p.small_pixels;
    if (SOC_RASTER_WG_ENTRIES) {
        __shared__ unsigned long long wg_acc, wg_base;
        if (threadIdx.x == 0) wg_acc = 0ull;
        __syncthreads();
        unsigned long long local = 0ull;
        if (big) {
            const uint32_t chunks = (uint32_t)(((bw + TILE - 1) / TILE) * ((bh + TILE - 1) / TILE));
            local = atomicAdd(&wg_acc, (1ull << ENTRY_SHIFT) + chunks);
        }
        __syncthreads();
        if (threadIdx.x == 0 && wg_acc) wg_base = atomicAdd(ws.counter, wg_acc);
        __syncthreads();
        if (big) {
            const unsigned long long old = wg_base + local;
            ws.entries[old >> ENTRY_SHIFT] = uint2{(uint32_t)id, (uint32_t)old};
            return;
        }
    } else if (big) {
        const uint32_t chunks = (uint32_t)(((bw + TILE - 1) / TILE) * ((bh + TILE - 1) / TILE));
        const unsigned long long old = atomicAdd(ws.counter, (1ull << ENTRY_SHIFT) + chunks);
        ws.entries[old >> ENTRY_SHIFT] = uint2{(uint32_t)id, (uint32_t)old};
        return;
    }
    if (!t.live) return;
    for (int y = t.py0; y <= t.py1; ++y)
        for (int x = t.px0; x <= t.px1; ++x) shade(t, id, x, y, p, target, pitch);
}

// Upper bound of the edge function over the pixel centres of [x0, x1] x [y0, y1] (a corner), minus a
// rounding margin: < 0 means no centre of the tile can pass this edge.
__device__ __forceinline__ float edge_max(f3 r, float x0, float x1, float y0, float y1) {
    const float m = fmaxf(fmaxf(edge(r, x0, y0), edge(r, x1, y0)), fmaxf(edge(r, x0, y1), edge(r, x1, y1)));
    const float slack = 1e-4f * (fabsf(r.x) * fmaxf(fabsf(x0), fabsf(x1)) + fabsf(r.y) * fmaxf(fabsf(y0), fabsf(y1)) + fabsf(r.z));
    return m + slack;
}

// One wave per work item (triangle, 32x32 tile of its box): 64 lanes, 2 rows per step.
__global__ __launch_bounds__(kWorkgroup) void raster_big(const uint32_t* __restrict__ idx, Workspace ws, RasterParams p,
                                                  void* target, size_t pitch) {
    const unsigned long long c = *ws.counter;
    const uint32_t n_entries = (uint32_t)(c >> ENTRY_SHIFT), count = (uint32_t)(c & ((1ull << ENTRY_SHIFT) - 1));
    const int lane = threadIdx.x & 63;
    // each wave walks a contiguous slice of the work indices: one binary search for its first entry,
    // then the entry advances as the slice crosses tile ranges
    const uint32_t nwaves = gridDim.x * 4, wv = blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint32_t per = (count + nwaves - 1) / nwaves;
    const uint32_t begin = min(count, wv * per), end = min(count, begin + per);
    if (begin >= end) return;
    uint32_t lo = 0, hi = n_entries - 1;   // the last entry with first <= begin
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (ws.entries[mid].y <= begin) lo = mid;
        else hi = mid - 1;
    }
    uint32_t e_idx = lo;
    uint2 e = ws.entries[e_idx];
    uint32_t next_first = e_idx + 1 < n_entries ? ws.entries[e_idx + 1].y : 0xFFFFFFFFu;
    TriSetup t = load_tri(ws, idx, (int)e.x, p);
    for (uint32_t it = begin; it < end; ++it) {
        if (it >= next_first) {
            do {
                ++e_idx;
                e = ws.entries[e_idx];
                next_first = e_idx + 1 < n_entries ? ws.entries[e_idx + 1].y : 0xFFFFFFFFu;
            } while (it >= next_first);
            t = load_tri(ws, idx, (int)e.x, p);
        }
        const uint2 item = uint2{e.x, it - e.y};
        const int tiles_x = (t.px1 - t.px0 + TILE) / TILE;
        const int ty = (int)item.y / tiles_x, tx = (int)item.y - ty * tiles_x;
        const int x0 = t.px0 + tx * TILE, y0 = t.py0 + ty * TILE;
        const int x1 = min(x0 + TILE - 1, t.px1), y1 = min(y0 + TILE - 1, t.py1);
        const float fx0 = (float)x0 + 0.5f, fx1 = (float)x1 + 0.5f, fy0 = (float)y0 + 0.5f, fy1 = (float)y1 + 0.5f;
        if (edge_max(t.r0, fx0, fx1, fy0, fy1) < 0.0f || edge_max(t.r1, fx0, fx1, fy0, fy1) < 0.0f ||
            edge_max(t.r2, fx0, fx1, fy0, fy1) < 0.0f)
            continue;
#if SOC_RASTER_FIXED_COLS
        const int x = x0 + (lane % TILE);
        if (x > x1) continue;
        for (int y = y0 + lane / TILE; y <= y1; y += 64 / TILE) shade(t, (int)item.x, x, y, p, target, pitch);
#else
        // the wave's lanes as cols x (64 / cols) pixels, cols the smallest power of two >= the item's width (4..TILE):
        // a narrow box (the median large triangle's is 14 x 15 pixels at 4K) keeps most lanes on its pixels
        const int cw = x1 - x0 + 1;
        const int lc = cw <= 4 ? 2 : cw <= 8 ? 3 : cw <= 16 ? 4 : 5;   // log2 cols (TILE = 32)
        const int x = x0 + (lane & ((1 << lc) - 1));
        if (x > x1) continue;
        for (int y = y0 + (lane >> lc); y <= y1; y += 64 >> lc) shade(t, (int)item.x, x, y, p, target, pitch);
#endif
    }
}

// ------------------------------------------------------------------------------------------------
// G-buffer resolve (g_buffer_generation.inl:161-225)
// ------------------------------------------------------------------------------------------------
struct ResolveParams {
    Mat4 model, vp, prev_vp;
    Mat3 normal3;
    int width, height, triangle_count, material_count;
    int tex_pairs;   // share the footprint of same-extent normal image + albedo (tuning knob SOC_GB_TEX_PAIRS, default on)
    int paired;      // read a material's paired_texels when it has them (tuning knob SOC_GB_PAIRED, default on)
    int wave_shape;  // pixels of a wave / workgroup: 0 = 64 x 1 / 64 x 4, 1 = 16 x 4 / 64 x 4, 2 = 8 x 8 / 32 x 8 (default),
                     // 3 = 8 x 8 / 16 x 16, 4 = 8 x 8 / 8 x 32 (tuning knob SOC_GB_WAVE)
};

__device__ __forceinline__ float srgb_to_linear(float c) {
    return c <= 0.04045f ? c / 12.92f : powf((c + 0.055f) / 1.055f, 2.4f);
}

// lut: srgb_to_linear(unorm8(i)) for i in 0..255 (LDS, filled per workgroup)
__device__ __forceinline__ f4 decode_rgba8(uint32_t u, bool srgb, const float* lut) {
    const float a = unorm8(u >> 24);
    if (!srgb) return f4{unorm8(u & 255u), unorm8((u >> 8) & 255u), unorm8((u >> 16) & 255u), a};
    return f4{lut[u & 255u], lut[(u >> 8) & 255u], lut[(u >> 16) & 255u], a};
}
__device__ __forceinline__ f4 texel_rgba8(const DImg& im, int x, int y, bool srgb, const float* lut) {
    return decode_rgba8(row_ptr<uint32_t>(im, y)[x], srgb, lut);
}

typedef uint32_t u2a4 __attribute__((ext_vector_type(2))) __attribute__((aligned(4)));
// The two texels (x0, y), (x1, y) of a bilinear tap's row: one 8-byte load when x1 = x0 + 1 (every tap that does
// not wrap around the REPEAT edge), else two. The same texels either way.
__device__ __forceinline__ void texel_row_pair(const DImg& im, int x0, int x1, int y, uint32_t& a, uint32_t& b) {
    const uint32_t* row = row_ptr<uint32_t>(im, y);
    if (x1 == x0 + 1) {
        const u2a4 t = *reinterpret_cast<const u2a4*>(row + x0);
        a = t.x;
        b = t.y;
    } else {
        a = row[x0];
        b = row[x1];
    }
}

// REPEAT addressing for any extent (the sampling contract's 8-bit sub-texel weights).
__device__ __forceinline__ Axis axis_repeat_any(float u, int n) {
#pragma clang fp contract(off)
    float t = u * (float)n;
    t = t - 0.5f;
    t = fminf(fmaxf(t, -4194304.0f), 4194304.0f);
    const int fx = (int)floorf(t * 256.0f + 0.5f);
    const int i = fx >> 8;
    Axis a;
    a.w = (float)(fx & 255) * (1.0f / 256.0f);
    int r = i % n;
    if (r < 0) r += n;
    a.i0 = r;
    a.i1 = (r + 1) % n;
    return a;
}

// REPEAT axis of extent n: the power-of-two mask when n is one (every texture of the reference's assets),
// else the general modulo; same taps and weight either way.
__device__ __forceinline__ Axis axis_repeat_level(float u, int n) {
    return (n & (n - 1)) ? axis_repeat_any(u, n) : axis_repeat_pow2(u, n, n - 1);
}

// Bilinear REPEAT sample of one level (its image view already resolved) of a packed mip chain, from the
// level's two axes (computed once when two textures of the same extent share them).
#ifndef SOC_GB_FAST_FILTER
#define SOC_GB_FAST_FILTER 1
#endif
#if SOC_GB_FAST_FILTER
typedef unsigned short gb_u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t gb_udot2(uint32_t a, uint32_t b) {
    return __builtin_amdgcn_udot2(__builtin_bit_cast(gb_u16x2, a), __builtin_bit_cast(gb_u16x2, b), 0u, false);
}
// Bilinear of the RGBA8 texels a b (top row) / c d with the contract's 8-bit weights (w = k / 256, exact).
// UNORM: the exact integer bilinear per channel (v_dot2_u32_u16: a_k (256 - kx) + b_k kx per row, then across the rows;
// at most 255 * 65536 < 2^24, exact in fp32), one conversion and one scale per channel. sRGB: the LUT-decoded channels,
// each lerp fma(w, q - p, p). Against the oracle's unorm8-then-lerp chain this changes fp32 roundings only (the
// G-buffer's RGBA16F tolerance; the GPU LUT already differs from the oracle's powf by an ulp).
__device__ __forceinline__ f4 bilerp_rgba8(uint32_t ua, uint32_t ub, uint32_t uc, uint32_t ud, float wx, float wy, bool srgb,
                                           const float* lut) {
    if (!srgb) {
        const uint32_t kx = (uint32_t)(wx * 256.0f), ky = (uint32_t)(wy * 256.0f);
        const uint32_t wxp = (256u - kx) | (kx << 16), wyp = (256u - ky) | (ky << 16);
        constexpr float kScale = 1.0f / (255.0f * 65536.0f);
        auto ch = [&](uint32_t k) {   // channel k: bytes k of (a, b) and of (c, d) as 16-bit pairs
            const uint32_t sel = k | 0x0c00u | ((4u + k) << 16) | 0x0c000000u;
            const uint32_t top = gb_udot2(__builtin_amdgcn_perm(ub, ua, sel), wxp);
            const uint32_t bot = gb_udot2(__builtin_amdgcn_perm(ud, uc, sel), wxp);
            return (float)gb_udot2(top | (bot << 16), wyp) * kScale;
        };
        return f4{ch(0), ch(1), ch(2), ch(3)};
    }
    auto ch = [&](float a, float b, float c, float d) {
        const float top = __builtin_fmaf(wx, b - a, a), bot = __builtin_fmaf(wx, d - c, c);
        return __builtin_fmaf(wy, bot - top, top);
    };
    return f4{ch(lut[ua & 255u], lut[ub & 255u], lut[uc & 255u], lut[ud & 255u]),
              ch(lut[(ua >> 8) & 255u], lut[(ub >> 8) & 255u], lut[(uc >> 8) & 255u], lut[(ud >> 8) & 255u]),
              ch(lut[(ua >> 16) & 255u], lut[(ub >> 16) & 255u], lut[(uc >> 16) & 255u], lut[(ud >> 16) & 255u]),
              ch(unorm8(ua >> 24), unorm8(ub >> 24), unorm8(uc >> 24), unorm8(ud >> 24))};
}
// trilinear blend of two levels' samples: fma(f, s1 - s0, s0) per channel
__device__ __forceinline__ f4 lerp_levels(f4 s0, f4 s1, float f) {
    return f4{__builtin_fmaf(f, s1.x - s0.x, s0.x), __builtin_fmaf(f, s1.y - s0.y, s0.y), __builtin_fmaf(f, s1.z - s0.z, s0.z),
              __builtin_fmaf(f, s1.w - s0.w, s0.w)};
}
#else
__device__ __forceinline__ f4 lerp_levels(f4 s0, f4 s1, float f) {
    return f4{lerp_w(s0.x, s1.x, f), lerp_w(s0.y, s1.y, f), lerp_w(s0.z, s1.z, f), lerp_w(s0.w, s1.w, f)};
}
#endif

__device__ __forceinline__ f4 sample_level_ax(const DImg& im, const Axis& ax, const Axis& ay, bool srgb, const float* lut) {
    uint32_t ua, ub, uc, ud;
    texel_row_pair(im, ax.i0, ax.i1, ay.i0, ua, ub);
    texel_row_pair(im, ax.i0, ax.i1, ay.i1, uc, ud);
#if SOC_GB_FAST_FILTER
    return bilerp_rgba8(ua, ub, uc, ud, ax.w, ay.w, srgb, lut);
#else
    const f4 a = decode_rgba8(ua, srgb, lut), b = decode_rgba8(ub, srgb, lut);
    const f4 c = decode_rgba8(uc, srgb, lut), d = decode_rgba8(ud, srgb, lut);
    return bilerp4(a, b, c, d, ax.w, ay.w);
#endif
}
__device__ __forceinline__ f4 sample_texture(const soc_img& tex, float u, float v, const float* lut) {
    if (!tex.data) return f4{1.0f, 1.0f, 1.0f, 1.0f};
    const DImg im{static_cast<char*>(tex.data), tex.width, tex.height, tex.pitch_bytes};
    const bool srgb = tex.format == SOC_FMT_RGBA8_SRGB;
    return sample_level_ax(im, axis_repeat_level(u, tex.width), axis_repeat_level(v, tex.height), srgb, lut);
}


__device__ __forceinline__ f4 sample_level(const DImg& im, float u, float v, bool srgb, const float* lut) {
    return sample_level_ax(im, axis_repeat_level(u, im.w), axis_repeat_level(v, im.h), srgb, lut);
}
__device__ __forceinline__ DImg level_view(const soc_img& tex, int k) {
    int wk, hk;
    const size_t off = mip_offset(tex.width, tex.height, tex.pitch_bytes, k, wk, hk);
    return DImg{static_cast<char*>(tex.data) + off, wk, hk, k ? 4 * wk : tex.pitch_bytes};
}

// Fine uv derivatives of the pixel's quad.
struct UVGrad { float dudx, dvdx, dudy, dvdy; };

// Trilinear + anisotropic REPEAT sample of a mip-chained texture (soc_rt.h SOC_MATERIAL_MIPMAPPED).
__device__ __forceinline__ f4 sample_texture_mip(const soc_img& tex, float u, float v, const UVGrad& gr, float max_aniso, const float* lut) {
#pragma clang fp contract(off)
    if (!tex.data) return f4{1.0f, 1.0f, 1.0f, 1.0f};
    const bool srgb = tex.format == SOC_FMT_RGBA8_SRGB;
    const int L = mip_levels(tex.width, tex.height);
    const float W = (float)tex.width, H = (float)tex.height;
    const float ax = gr.dudx * W, ay = gr.dvdx * H, bx = gr.dudy * W, by = gr.dvdy * H;
    const float px = sqrtf(ax * ax + ay * ay), py = sqrtf(bx * bx + by * by);
    const float pmax = fmaxf(px, py), pmin = fminf(px, py);
    int n = 1;
    if (max_aniso > 1.0f && pmax > 0.0f && pmax <= 3.4e38f) {
        const float cap = floorf(max_aniso);
        n = (int)(pmin > 0.0f ? fminf(ceilf(pmax / pmin), cap) : cap);
    }
    int lq = 0;   // lod in 1/256 steps, clamped to [0, (L - 1) 256]
    const float rho = pmax / (float)n;
    if (rho > 0.0f && rho <= 3.4e38f) {
        const float lam = fminf(fmaxf(det_log2(rho), -64.0f), 64.0f);
        lq = min(max((int)floorf(lam * 256.0f + 0.5f), 0), (L - 1) * 256);
    }
    const int l0 = lq >> 8;
    const float f = (float)(lq & 255) * (1.0f / 256.0f);
    const DImg im0 = level_view(tex, l0), im1 = level_view(tex, min(l0 + 1, L - 1));
    const bool xmajor = px >= py;
    const float du = xmajor ? gr.dudx : gr.dudy, dv = xmajor ? gr.dvdx : gr.dvdy;
    f4 acc = f4{0.0f, 0.0f, 0.0f, 0.0f};
    for (int i = 1; i <= n; ++i) {
        float su = u, sv = v;
        if (n > 1) {
            const float t = (float)i / (float)(n + 1) - 0.5f;
            su = u + t * du;
            sv = v + t * dv;
        }
        f4 s0 = sample_level(im0, su, sv, srgb, lut);
        if (lq & 255) s0 = lerp_levels(s0, sample_level(im1, su, sv, srgb, lut), f);
        acc = f4{acc.x + s0.x, acc.y + s0.y, acc.z + s0.z, acc.w + s0.w};
    }
    if (n == 1) return acc;
    const float fn = (float)n;
    return f4{acc.x / fn, acc.y / fn, acc.z / fn, acc.w / fn};
}

// sample_texture_mip of two textures of the same extent at the same uv (the material's normal image and
// albedo): the footprint, tap count, lod and every tap's level axes depend only on the extent, so they are
// computed once; each texture's taps, lerps and sums are sample_texture_mip's, in its order (same bits).
// Precondition: both have data and ta.width == tb.width, ta.height == tb.height.
__device__ __forceinline__ void sample_texture_mip2(const soc_img& ta, const soc_img& tb, float u, float v, const UVGrad& gr,
                                    float max_aniso, const float* lut, f4& ra, f4& rb) {
#pragma clang fp contract(off)
    const bool sa = ta.format == SOC_FMT_RGBA8_SRGB, sb = tb.format == SOC_FMT_RGBA8_SRGB;
    const int L = mip_levels(ta.width, ta.height);
    const float W = (float)ta.width, H = (float)ta.height;
    const float ax = gr.dudx * W, ay = gr.dvdx * H, bx = gr.dudy * W, by = gr.dvdy * H;
    const float px = sqrtf(ax * ax + ay * ay), py = sqrtf(bx * bx + by * by);
    const float pmax = fmaxf(px, py), pmin = fminf(px, py);
    int n = 1;
    if (max_aniso > 1.0f && pmax > 0.0f && pmax <= 3.4e38f) {
        const float cap = floorf(max_aniso);
        n = (int)(pmin > 0.0f ? fminf(ceilf(pmax / pmin), cap) : cap);
    }
    int lq = 0;
    const float rho = pmax / (float)n;
    if (rho > 0.0f && rho <= 3.4e38f) {
        const float lam = fminf(fmaxf(det_log2(rho), -64.0f), 64.0f);
        lq = min(max((int)floorf(lam * 256.0f + 0.5f), 0), (L - 1) * 256);
    }
    const int l0 = lq >> 8, l1 = min(l0 + 1, L - 1);
    const float f = (float)(lq & 255) * (1.0f / 256.0f);
    const DImg a0 = level_view(ta, l0), a1 = level_view(ta, l1), b0 = level_view(tb, l0), b1 = level_view(tb, l1);
    const bool xmajor = px >= py;
    const float du = xmajor ? gr.dudx : gr.dudy, dv = xmajor ? gr.dvdx : gr.dvdy;
    f4 acca = f4{0.0f, 0.0f, 0.0f, 0.0f}, accb = acca;
    auto tri = [&](f4 s0, const f4& s1) { return lerp_levels(s0, s1, f); };
    for (int i = 1; i <= n; ++i) {
        float su = u, sv = v;
        if (n > 1) {
            const float t = (float)i / (float)(n + 1) - 0.5f;
            su = u + t * du;
            sv = v + t * dv;
        }
        const Axis x0 = axis_repeat_level(su, a0.w), y0 = axis_repeat_level(sv, a0.h);
        f4 pa = sample_level_ax(a0, x0, y0, sa, lut), pb = sample_level_ax(b0, x0, y0, sb, lut);
        if (lq & 255) {
            const Axis x1 = axis_repeat_level(su, a1.w), y1 = axis_repeat_level(sv, a1.h);
            pa = tri(pa, sample_level_ax(a1, x1, y1, sa, lut));
            pb = tri(pb, sample_level_ax(b1, x1, y1, sb, lut));
        }
        acca = f4{acca.x + pa.x, acca.y + pa.y, acca.z + pa.z, acca.w + pa.w};
        accb = f4{accb.x + pb.x, accb.y + pb.y, accb.z + pb.z, accb.w + pb.w};
    }
    if (n == 1) {
        ra = acca;
        rb = accb;
        return;
    }
    const float fn = (float)n;
    ra = f4{acca.x / fn, acca.y / fn, acca.z / fn, acca.w / fn};
    rb = f4{accb.x / fn, accb.y / fn, accb.z / fn, accb.w / fn};
}

// sample_texture_mip2 from the material's paired texels (soc_pair_textures: albedo and normal texel interleaved, 8 B):
// each tap row of both textures is one 16-B load (two 8-B loads at the REPEAT seam) instead of one 8-B load per
// texture. The same texels reach the same filter arithmetic: the same bits as sample_texture_mip2 (GPU test).
__device__ __forceinline__ DImg paired_level(const void* paired, int W, int H, int k) {
    int wk, hk;
    const size_t off = mip_offset(W, H, 8 * W, k, wk, hk, 8);
    return DImg{static_cast<char*>(const_cast<void*>(paired)) + off, wk, hk, 8 * wk};
}
typedef uint32_t u4a8g __attribute__((ext_vector_type(4))) __attribute__((aligned(8)));
__device__ __forceinline__ void paired_row(const DImg& im, int x0, int x1, int y, uint32_t& a0, uint32_t& n0, uint32_t& a1,
                                           uint32_t& n1) {
    const uint2* row = row_ptr<uint2>(im, y);
    if (x1 == x0 + 1) {
        const u4a8g t = *reinterpret_cast<const u4a8g*>(row + x0);
        a0 = t.x; n0 = t.y; a1 = t.z; n1 = t.w;
    } else {
        const uint2 p = row[x0], q = row[x1];
        a0 = p.x; n0 = p.y; a1 = q.x; n1 = q.y;
    }
}
__device__ __forceinline__ void sample_paired_level(const DImg& im, const Axis& ax, const Axis& ay, bool sn, bool sa,
                                                    const float* lut, f4& rn, f4& ra) {
    uint32_t a0, n0, a1, n1, a2, n2, a3, n3;
    paired_row(im, ax.i0, ax.i1, ay.i0, a0, n0, a1, n1);
    paired_row(im, ax.i0, ax.i1, ay.i1, a2, n2, a3, n3);
#if SOC_GB_FAST_FILTER
    rn = bilerp_rgba8(n0, n1, n2, n3, ax.w, ay.w, sn, lut);
    ra = bilerp_rgba8(a0, a1, a2, a3, ax.w, ay.w, sa, lut);
#else
    rn = bilerp4(decode_rgba8(n0, sn, lut), decode_rgba8(n1, sn, lut), decode_rgba8(n2, sn, lut), decode_rgba8(n3, sn, lut), ax.w, ay.w);
    ra = bilerp4(decode_rgba8(a0, sa, lut), decode_rgba8(a1, sa, lut), decode_rgba8(a2, sa, lut), decode_rgba8(a3, sa, lut), ax.w, ay.w);
#endif
}
// ta: the normal image, tb: the albedo (their extent and formats); results as sample_texture_mip2's (ra: normal, rb: albedo)
__device__ __forceinline__ void sample_texture_mip2p(const soc_img& ta, const soc_img& tb, const void* paired, float u, float v,
                                                     const UVGrad& gr, float max_aniso, const float* lut, f4& ra, f4& rb) {
#pragma clang fp contract(off)
    const bool sa = ta.format == SOC_FMT_RGBA8_SRGB, sb = tb.format == SOC_FMT_RGBA8_SRGB;
    const int L = mip_levels(ta.width, ta.height);
    const float W = (float)ta.width, H = (float)ta.height;
    const float ax = gr.dudx * W, ay = gr.dvdx * H, bx = gr.dudy * W, by = gr.dvdy * H;
    const float px = sqrtf(ax * ax + ay * ay), py = sqrtf(bx * bx + by * by);
    const float pmax = fmaxf(px, py), pmin = fminf(px, py);
    int n = 1;
    if (max_aniso > 1.0f && pmax > 0.0f && pmax <= 3.4e38f) {
        const float cap = floorf(max_aniso);
        n = (int)(pmin > 0.0f ? fminf(ceilf(pmax / pmin), cap) : cap);
    }
    int lq = 0;
    const float rho = pmax / (float)n;
    if (rho > 0.0f && rho <= 3.4e38f) {
        const float lam = fminf(fmaxf(det_log2(rho), -64.0f), 64.0f);
        lq = min(max((int)floorf(lam * 256.0f + 0.5f), 0), (L - 1) * 256);
    }
    const int l0 = lq >> 8, l1 = min(l0 + 1, L - 1);
    const float f = (float)(lq & 255) * (1.0f / 256.0f);
    const DImg p0 = paired_level(paired, ta.width, ta.height, l0), p1 = paired_level(paired, ta.width, ta.height, l1);
    const bool xmajor = px >= py;
    const float du = xmajor ? gr.dudx : gr.dudy, dv = xmajor ? gr.dvdx : gr.dvdy;
    f4 acca = f4{0.0f, 0.0f, 0.0f, 0.0f}, accb = acca;
    for (int i = 1; i <= n; ++i) {
        float su = u, sv = v;
        if (n > 1) {
            const float t = (float)i / (float)(n + 1) - 0.5f;
            su = u + t * du;
            sv = v + t * dv;
        }
        const Axis x0 = axis_repeat_level(su, p0.w), y0 = axis_repeat_level(sv, p0.h);
        f4 pa, pb;
        sample_paired_level(p0, x0, y0, sa, sb, lut, pa, pb);
        if (lq & 255) {
            const Axis x1 = axis_repeat_level(su, p1.w), y1 = axis_repeat_level(sv, p1.h);
            f4 qa, qb;
            sample_paired_level(p1, x1, y1, sa, sb, lut, qa, qb);
            pa = lerp_levels(pa, qa, f);
            pb = lerp_levels(pb, qb, f);
        }
        acca = f4{acca.x + pa.x, acca.y + pa.y, acca.z + pa.z, acca.w + pa.w};
        accb = f4{accb.x + pb.x, accb.y + pb.y, accb.z + pb.z, accb.w + pb.w};
    }
    if (n == 1) {
        ra = acca;
        rb = accb;
        return;
    }
    const float fn = (float)n;
    ra = f4{acca.x / fn, acca.y / fn, acca.z / fn, acca.w / fn};
    rb = f4{accb.x / fn, accb.y / fn, accb.z / fn, accb.w / fn};
}

__device__ __forceinline__ f3 mat3_vec_exact(const Mat3& M, f3 v) {
#pragma clang fp contract(off)
    const float* m = M.m;
    return f3{m[0] * v.x + m[3] * v.y + m[6] * v.z, m[1] * v.x + m[4] * v.y + m[7] * v.z, m[2] * v.x + m[5] * v.y + m[8] * v.z};
}

// Per-pixel normalize of the resolve (the interpolated normal and the TBN): v_rsq_f32 and three multiplies instead of the
// correctly rounded sqrt and three IEEE divisions (~40 VALU each, five per normal-mapped pixel). A few fp32 ulps against
// the oracle's normalize, stored as RGBA16F (the G-buffer tolerance); a zero vector still gives NaN. The per-vertex
// normal (gbuffer_vertex_setup) stays exact. SOC_GB_FAST_NORMALIZE=0 builds the exact form (A/B).
#ifndef SOC_GB_FAST_NORMALIZE
#define SOC_GB_FAST_NORMALIZE 1
#endif
__device__ __forceinline__ f3 normalize_exact(f3 a);
__device__ __forceinline__ f3 normalize_px(f3 a) {
#if SOC_GB_FAST_NORMALIZE
    const float k = __builtin_amdgcn_rsqf(__builtin_fmaf(a.z, a.z, __builtin_fmaf(a.y, a.y, a.x * a.x)));
    return f3{a.x * k, a.y * k, a.z * k};
#else
    return normalize_exact(a);
#endif
}
__device__ __forceinline__ f3 normalize_exact(f3 a) {
#pragma clang fp contract(off)
    const float l = sqrtf(a.x * a.x + a.y * a.y + a.z * a.z);
    return f3{a.x / l, a.y / l, a.z / l};
}

// The vertex stage of GBufferGeneration (g_buffer_generation.inl:169-178) for vertex v: the raster's
// homogeneous screen vertex, normalize(normal_matrix * normal), and the current / previous clip x, y, w.
// 4 float4 per vertex; computed once per vertex into the workspace (gbuffer_vertex_setup) or inline by
// the resolve; the same function either way, so both give the same bits.
struct VtxData { float4 s, n, cc, pc; };

__device__ __forceinline__ VtxData vertex_data(const soc_mesh& mesh, uint32_t v, const ResolveParams& p) {
#pragma clang fp contract(off)
    VtxData d;
    d.s = clip_vertex(mesh.positions, v, p.model, p.vp, p.width, p.height);
    const float* nr = mesh.normals;
    const f3 n = normalize_exact(mat3_vec_exact(p.normal3, f3{nr[3 * v], nr[3 * v + 1], nr[3 * v + 2]}));
    d.n = float4{n.x, n.y, n.z, 0.0f};   // .w of n, cc, pc: the world position (the TBN's out_position)
    const float* ps = mesh.positions;
    const f4 wp = mat_vec_exact(p.model, ps[3 * v], ps[3 * v + 1], ps[3 * v + 2], 1.0f);
    const f4 c = mat_vec_exact(p.vp, wp.x, wp.y, wp.z, wp.w);
    const f4 q = mat_vec_exact(p.prev_vp, wp.x, wp.y, wp.z, wp.w);
    d.n.w = wp.x;
    d.cc = float4{c.x, c.y, c.w, wp.y};
    d.pc = float4{q.x, q.y, q.w, wp.z};
    return d;
}

__global__ __launch_bounds__(kWorkgroup) void gbuffer_vertex_setup(soc_mesh mesh, float4* __restrict__ vd, ResolveParams p) {
    const int v = blockIdx.x * 256 + threadIdx.x;
    if (v >= mesh.vertex_count) return;
    const VtxData d = vertex_data(mesh, (uint32_t)v, p);
    vd[4 * v] = d.s;
    vd[4 * v + 1] = d.n;
    vd[4 * v + 2] = d.cc;
    vd[4 * v + 3] = d.pc;
}

template <bool PRE>
__device__ __forceinline__ VtxData fetch_vertex(const soc_mesh& mesh, const float4* __restrict__ vd, uint32_t v,
                                                const ResolveParams& p) {
    if (!PRE) return vertex_data(mesh, v, p);
    return VtxData{vd[4 * v], vd[4 * v + 1], vd[4 * v + 2], vd[4 * v + 3]};
}

#ifndef SOC_GB_WAVES
#define SOC_GB_WAVES 5   // waves per SIMD the resolve's registers allow: 96 VGPRs, no spill (A/B builds: 1 = unconstrained)
#endif
template <bool PRE>
__global__ __launch_bounds__(kWorkgroup) __attribute__((amdgpu_waves_per_eu(SOC_GB_WAVES))) void gbuffer_resolve(soc_mesh mesh, const soc_material* __restrict__ mats,
                                                       const unsigned long long* __restrict__ vis, DImg depth,
                                                       DImg albedo, DImg emissive, DImg normal, DImg velocity,
                                                       const float4* __restrict__ vd, ResolveParams p) {
#pragma clang fp contract(off)
    __shared__ float lut[256];
    lut[threadIdx.y * 64 + threadIdx.x] = srgb_to_linear(unorm8(threadIdx.y * 64 + threadIdx.x));
    __syncthreads();
    // row-major tiles: the XCD-aware orders measured 13-40 % slower here (profiles/r04_probe_gbuffer_order.txt).
    // A wave covers 64 x 1 pixels (shape 0), 16 x 4 (1, the workgroup a 64 x 4 tile) or 8 x 8 (2: a 32 x 8 tile, the
    // default; 3: 16 x 16; 4: 8 x 32): a compact wave footprint shares the texture lines of the anisotropic taps in L1.
    const int lane = threadIdx.x, wave = threadIdx.y;
    int x, y;
    if (p.wave_shape == 1) {
        x = blockIdx.x * 64 + wave * 16 + (lane & 15);
        y = blockIdx.y * 4 + (lane >> 4);
    } else if (p.wave_shape == 2) {
        x = blockIdx.x * 32 + wave * 8 + (lane & 7);
        y = blockIdx.y * 8 + (lane >> 3);
    } else if (p.wave_shape == 3) {
        x = blockIdx.x * 16 + (wave & 1) * 8 + (lane & 7);
        y = blockIdx.y * 16 + (wave >> 1) * 8 + (lane >> 3);
    } else if (p.wave_shape == 4) {
        x = blockIdx.x * 8 + (lane & 7);
        y = blockIdx.y * 32 + wave * 8 + (lane >> 3);
    } else {
        x = blockIdx.x * 64 + lane;
        y = blockIdx.y * 4 + wave;
    }
    if (x >= p.width || y >= p.height) return;
    const unsigned long long key = vis[(size_t)y * p.width + x];
    const uint32_t low = (uint32_t)key;
    if (low == KEY_EMPTY) {   // clear values (g_buffer_generation.inl:78-100, depth cleared to 1.0)
        row_ptr_w<float>(depth, y)[x] = 1.0f;
        row_ptr_w<uint2>(albedo, y)[x] = pack_h4(f4{0.2f, 0.4f, 1.0f, 1.0f});
        row_ptr_w<uint2>(emissive, y)[x] = pack_h4(f4{0.0f, 0.0f, 0.0f, 1.0f});
        row_ptr_w<uint2>(normal, y)[x] = pack_h4(f4{0.0f, 0.0f, 0.0f, 1.0f});
        row_ptr_w<uint2>(velocity, y)[x] = pack_h4(f4{0.0f, 0.0f, 0.0f, 1.0f});
        return;
    }
    const int id = (int)(0xFFFFFFFEu - low);
    const uint32_t ia = mesh.indices[3 * id], ib = mesh.indices[3 * id + 1], ic = mesh.indices[3 * id + 2];
    const VtxData VA = fetch_vertex<PRE>(mesh, vd, ia, p), VB = fetch_vertex<PRE>(mesh, vd, ib, p),
                  VC = fetch_vertex<PRE>(mesh, vd, ic, p);
    const float4 A = VA.s, B = VB.s, C = VC.s;
    // perspective-correct barycentrics b_i = E_i / sum E from the raster's edge functions
    const f3 v0{A.x, A.y, A.w}, v1{B.x, B.y, B.w}, v2{C.x, C.y, C.w};
    f3 r0 = cross_exact(v1, v2), r1 = cross_exact(v2, v0), r2 = cross_exact(v0, v1);
    const float det = v0.x * r0.x + v0.y * r0.y + v0.z * r0.z;
    if (det < 0.0f) { r0 = -r0; r1 = -r1; r2 = -r2; }
    const float fx = (float)x + 0.5f, fy = (float)y + 0.5f;
    const float e0 = edge(r0, fx, fy), e1 = edge(r1, fx, fy), e2 = edge(r2, fx, fy);
    const float es = e0 + e1 + e2;
    const float b1 = e1 / es, b2 = e2 / es, b0 = 1.0f - b1 - b2;

    // interpolated vertex outputs (g_buffer_generation.inl:169-178)
    const float* uv = mesh.uvs;
    const float u = b0 * uv[2 * ia] + b1 * uv[2 * ib] + b2 * uv[2 * ic];
    const float v = b0 * uv[2 * ia + 1] + b1 * uv[2 * ib + 1] + b2 * uv[2 * ic + 1];
    const uint32_t mi = mesh.materials ? min(mesh.materials[id], (uint32_t)(p.material_count - 1)) : 0u;
    const soc_material& m = mats[mi];
    // velocity and depth first: the clip positions are dead before the texture taps (123 -> fewer live VGPRs there)
    {
        f4 vel = f4{0.0f, 0.0f, 0.0f, 0.0f};
        if (!(m.flags & SOC_MATERIAL_ZERO_VELOCITY)) {
            const float4 ca = VA.cc, cb = VB.cc, cd = VC.cc, pa = VA.pc, pb = VB.pc, pd = VC.pc;
            const float cx = b0 * ca.x + b1 * cb.x + b2 * cd.x, cy = b0 * ca.y + b1 * cb.y + b2 * cd.y;
            const float cw = b0 * ca.z + b1 * cb.z + b2 * cd.z;
            const float px = b0 * pa.x + b1 * pb.x + b2 * pd.x, py = b0 * pa.y + b1 * pb.y + b2 * pd.y;
            const float pw = b0 * pa.z + b1 * pb.z + b2 * pd.z;
            vel = f4{((cx / cw) * 0.5f + 0.5f) - ((px / pw) * 0.5f + 0.5f), ((cy / cw) * 0.5f + 0.5f) - ((py / pw) * 0.5f + 0.5f),
                     0.0f, 1.0f};
        }
        row_ptr_w<float>(depth, y)[x] = __uint_as_float((uint32_t)(key >> 32));
        row_ptr_w<uint2>(velocity, y)[x] = pack_h4(vel);
    }
    f3 n;
    if ((m.flags & SOC_MATERIAL_NORMAL_MAP) && m.normal_map.data) {   // draw_terrain.inl:206-219
        const DImg nm{static_cast<char*>(m.normal_map.data), m.normal_map.width, m.normal_map.height, m.normal_map.pitch_bytes};
        const f4 t = sample_h4(nm, u, v);
        n = normalize_px(f3{t.x, t.y, t.z});
    } else {
        const float4 na = VA.n, nb = VB.n, nc = VC.n;
        n = normalize_px(f3{b0 * na.x + b1 * nb.x + b2 * nc.x, b0 * na.y + b1 * nb.y + b2 * nc.y,
                               b0 * na.z + b1 * nb.z + b2 * nc.z});
    }
    const bool tbn = (m.flags & SOC_MATERIAL_NORMAL_TEXTURE) && m.normal_image.data;
    const bool mipped = m.flags & SOC_MATERIAL_MIPMAPPED;
    // fine dFdx / dFdy: this triangle's attributes at the two centres of the pixel's 2x2 quad per direction
    // (what helper invocations evaluate); world positions only for the TBN
    f3 Q1{0.0f, 0.0f, 0.0f}, Q2{0.0f, 0.0f, 0.0f};
    UVGrad gr{0.0f, 0.0f, 0.0f, 0.0f};
    if (tbn || mipped) {
        f4 wa{0.0f, 0.0f, 0.0f, 0.0f}, wb = wa, wc = wa;
        if (tbn) {   // vertex stage out_position (:171-172), kept by the vertex stage in the .w components
            wa = f4{VA.n.w, VA.cc.w, VA.pc.w, 1.0f};
            wb = f4{VB.n.w, VB.cc.w, VB.pc.w, 1.0f};
            wc = f4{VC.n.w, VC.cc.w, VC.pc.w, 1.0f};
        }
        auto attr = [&](float sx, float sy, f3& P, float& su, float& sv) {
            const float a0 = edge(r0, sx, sy), a1 = edge(r1, sx, sy), a2 = edge(r2, sx, sy);
            const float as = a0 + a1 + a2;
            const float c1 = a1 / as, c2 = a2 / as, c0 = 1.0f - c1 - c2;
            P = f3{c0 * wa.x + c1 * wb.x + c2 * wc.x, c0 * wa.y + c1 * wb.y + c2 * wc.y, c0 * wa.z + c1 * wb.z + c2 * wc.z};
            su = c0 * uv[2 * ia] + c1 * uv[2 * ib] + c2 * uv[2 * ic];
            sv = c0 * uv[2 * ia + 1] + c1 * uv[2 * ib + 1] + c2 * uv[2 * ic + 1];
        };
        const float qx = (float)(x & ~1) + 0.5f, qy = (float)(y & ~1) + 0.5f;
        f3 px0, px1, py0, py1;
        float ux0, vx0, ux1, vx1, uy0, vy0, uy1, vy1;
        attr(qx, fy, px0, ux0, vx0);
        attr(qx + 1.0f, fy, px1, ux1, vx1);
        attr(fx, qy, py0, uy0, vy0);
        attr(fx, qy + 1.0f, py1, uy1, vy1);
        Q1 = f3{px1.x - px0.x, px1.y - px0.y, px1.z - px0.z};
        Q2 = f3{py1.x - py0.x, py1.y - py0.y, py1.z - py0.z};
        gr = UVGrad{ux1 - ux0, vx1 - vx0, uy1 - uy0, vy1 - vy0};
    }
    auto tex = [&](const soc_img& t) {
        return mipped ? sample_texture_mip(t, u, v, gr, m.max_anisotropy, lut) : sample_texture(t, u, v, lut);
    };
    // normal image and albedo of one extent on the reference sampler: one footprint for both (same bits)
    const bool pair = tbn && mipped && p.tex_pairs && m.albedo.data && m.albedo.width == m.normal_image.width &&
                      m.albedo.height == m.normal_image.height;
    f4 t_pair{0.0f, 0.0f, 0.0f, 0.0f}, al_pair = t_pair;
    if (pair && (m.flags & SOC_MATERIAL_PAIRED_TEXELS) && m.paired_texels && p.paired)
        sample_texture_mip2p(m.normal_image, m.albedo, m.paired_texels, u, v, gr, m.max_anisotropy, lut, t_pair, al_pair);
    else if (pair)
        sample_texture_mip2(m.normal_image, m.albedo, u, v, gr, m.max_anisotropy, lut, t_pair, al_pair);
    if (tbn) {   // g_buffer_generation.inl:197-211
        const f4 t = pair ? t_pair : tex(m.normal_image);
        const f3 tn{t.x * 2.0f - 1.0f, t.y * 2.0f - 1.0f, t.z * 2.0f - 1.0f};
        const float st1t = gr.dvdx, st2t = gr.dvdy;
        const f3 N = normalize_px(n);
        const f3 T = normalize_px(f3{Q1.x * st2t - Q2.x * st1t, Q1.y * st2t - Q2.y * st1t, Q1.z * st2t - Q2.z * st1t});
        const f3 B = normalize_px(cross_exact(N, T));
        n = normalize_px(f3{T.x * tn.x + B.x * tn.y + N.x * tn.z, T.y * tn.x + B.y * tn.y + N.y * tn.z,
                               T.z * tn.x + B.z * tn.y + N.z * tn.z});
    }
    f3 em = f3{0.0f, 0.0f, 0.0f};
    if (m.has_emissive) {
        const f4 e = tex(m.emissive);
        em = f3{e.x * m.emissive_factor[0], e.y * m.emissive_factor[1], e.z * m.emissive_factor[2]};
    }
    const f4 al = pair ? al_pair : tex(m.albedo);
    row_ptr_w<uint2>(albedo, y)[x] = pack_h4(f4{al.x * m.albedo_factor[0] + em.x, al.y * m.albedo_factor[1] + em.y,
                                                al.z * m.albedo_factor[2] + em.z, 1.0f});
    row_ptr_w<uint2>(emissive, y)[x] = pack_h4(f4{em.x, em.y, em.z, 1.0f});
    row_ptr_w<uint2>(normal, y)[x] = pack_h4(f4{n.x, n.y, n.z, 1.0f});
}

int check_mesh(const soc_mesh* mesh, const char* pass, bool attributes) {
    if (!mesh || !mesh->positions || !mesh->indices || mesh->vertex_count < 0 || mesh->triangle_count < 0)
        return set_error(SOC_E_INVALID_ARG, "%s: null mesh / positions / indices or negative counts", pass);
    if (attributes && (!mesh->normals || !mesh->uvs))
        return set_error(SOC_E_INVALID_ARG, "%s: the G-buffer resolve needs normals and uvs", pass);
    if ((uint32_t)mesh->triangle_count >= 0xFFFFFFFEu)
        return set_error(SOC_E_SHAPE, "%s: too many triangles for the visibility key", pass);
    return SOC_OK;
}

RasterParams make_raster_params(const soc_mesh* mesh, const float* vp, int W, int H, int cull) {
    RasterParams p{};
    p.model = mat4(mesh->model_matrix);
    p.vp = mat4(vp);
    p.width = W;
    p.height = H;
    p.vertex_count = mesh->vertex_count;
    p.triangle_count = mesh->triangle_count;
    p.cull = cull;
    p.small_pixels = SMALL_PIXELS;
    return p;
}

int launch_raster(const soc_mesh* mesh, const RasterParams& p, void* target, size_t pitch, void* workspace,
                  hipStream_t s, const char* pass) {
    Workspace ws = carve(workspace, mesh->vertex_count, mesh->triangle_count);
    launch("raster_setup", kWorkgroup, raster_setup, ceil_div(max(mesh->vertex_count, 1), 256), kWorkgroup, 0, s, mesh->positions, ws, p);
    if (mesh->triangle_count > 0) {
        launch("raster_small", kWorkgroup, raster_small, ceil_div(mesh->triangle_count, 256), kWorkgroup, 0, s, mesh->indices, ws, p, target, pitch);
        launch("raster_big", kWorkgroup, raster_big, 2048, kWorkgroup, 0, s, mesh->indices, ws, p, target, pitch);
    }
    return check_launch(pass);
}

}  // namespace
}  // namespace soc

using namespace soc;

extern "C" size_t soc_raster_workspace_size(int32_t vertex_count, int32_t triangle_count) {
    if (vertex_count < 0 || triangle_count < 0) return 0;
    return align_up(align_up((size_t)vertex_count * 16, 256) + 256 + (size_t)triangle_count * 8, 256) +
           (size_t)vertex_count * 64;
}

extern "C" int soc_raster_visibility(const soc_mesh* mesh, const float view_projection[16], int32_t cull,
                                     uint64_t* visibility, int32_t width, int32_t height, int32_t clear,
                                     void* workspace, soc_stream stream) {
    int rc = check_mesh(mesh, "soc_raster_visibility", false);
    if (rc) return rc;
    if (!view_projection || !visibility || !workspace || width <= 0 || height <= 0 || cull < 0 || cull > 2)
        return set_error(SOC_E_INVALID_ARG, "soc_raster_visibility: null argument, bad extent or cull mode");
    hipStream_t s = hs(stream);
    if (clear) {
        const size_t n = (size_t)width * height;
        launch("raster_clear_vis", kWorkgroup, raster_clear_vis, (unsigned)((n + 255) / 256), kWorkgroup, 0, s, reinterpret_cast<unsigned long long*>(visibility), n);
    }
    RasterParams p = make_raster_params(mesh, view_projection, width, height, cull);
    return launch_raster(mesh, p, visibility, (size_t)width * 8, workspace, s, "raster_visibility");
}

extern "C" int soc_raster_depth(const soc_mesh* mesh, const float view_projection[16], int32_t cull, float bias_constant,
                                float bias_slope, soc_img depth, void* workspace, soc_stream stream) {
    int rc = check_mesh(mesh, "soc_raster_depth", false);
    if (!rc) rc = check_img(depth, SOC_FMT_D32F, "soc_raster_depth", "depth");
    if (rc) return rc;
    if (!view_projection || !workspace || cull < 0 || cull > 2)
        return set_error(SOC_E_INVALID_ARG, "soc_raster_depth: null argument or bad cull mode");
    hipStream_t s = hs(stream);
    // depth clear 1.0 (sun_shadow_draw.inl:71-74)
    if (hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(depth.data), __builtin_bit_cast(int, 1.0f),
                          (size_t)depth.pitch_bytes / 4 * depth.height, s) != hipSuccess)
        return set_error(SOC_E_HIP, "soc_raster_depth: clear failed");
    RasterParams p = make_raster_params(mesh, view_projection, depth.width, depth.height, cull);
    p.depth_only = 1;
    p.bias_constant = bias_constant;
    p.bias_slope = bias_slope;
    return launch_raster(mesh, p, depth.data, (size_t)depth.pitch_bytes, workspace, s, "raster_depth");
}

extern "C" int soc_gbuffer_resolve(const soc_globals* g, const soc_mesh* mesh, const soc_material* d_materials,
                                   int32_t material_count, const uint64_t* visibility, soc_img depth, soc_img albedo,
                                   soc_img emissive, soc_img normal, soc_img velocity, void* workspace,
                                   soc_stream stream) {
    int rc = check_mesh(mesh, "soc_gbuffer_resolve", true);
    if (!rc) rc = check_img(depth, SOC_FMT_D32F, "soc_gbuffer_resolve", "depth");
    if (!rc) rc = check_img(albedo, SOC_FMT_RGBA16F, "soc_gbuffer_resolve", "albedo");
    if (!rc) rc = check_img(emissive, SOC_FMT_RGBA16F, "soc_gbuffer_resolve", "emissive");
    if (!rc) rc = check_img(normal, SOC_FMT_RGBA16F, "soc_gbuffer_resolve", "normal");
    if (!rc) rc = check_img(velocity, SOC_FMT_RGBA16F, "soc_gbuffer_resolve", "velocity");
    if (rc) return rc;
    if (!g || !d_materials || material_count <= 0 || !visibility)
        return set_error(SOC_E_INVALID_ARG, "soc_gbuffer_resolve: null globals / materials / visibility");
    const int W = depth.width, H = depth.height;
    for (const soc_img* im : {&albedo, &emissive, &normal, &velocity})
        if (im->width != W || im->height != H)
            return set_error(SOC_E_SHAPE, "soc_gbuffer_resolve: G-buffer images must share the depth extent");
    ResolveParams p{};
    p.model = mat4(mesh->model_matrix);
    p.vp = mat4(g->camera_projection_view_matrix);
    p.prev_vp = mat4(g->camera_previous_projection_view_matrix);
    const float* nm = mesh->normal_matrix;   // f32mat3x3(normal_matrix): upper 3x3, column-major
    const float n3[9] = {nm[0], nm[1], nm[2], nm[4], nm[5], nm[6], nm[8], nm[9], nm[10]};
    for (int i = 0; i < 9; ++i) p.normal3.m[i] = n3[i];
    p.width = W;
    p.height = H;
    p.triangle_count = mesh->triangle_count;
    p.material_count = material_count;
    p.tex_pairs = tuning_knob("SOC_GB_TEX_PAIRS", 1);
    p.paired = tuning_knob("SOC_GB_PAIRED", 1);
    p.wave_shape = tuning_knob("SOC_GB_WAVE", 2);   // 8 x 8-pixel waves: 687 -> 626 us at 4K (profiles/r04_probe_gbuffer_wave.txt)
    dim3 blk(64, 4), grd(ceil_div(W, 64), ceil_div(H, 4));
    if (p.wave_shape == 2) grd = dim3(ceil_div(W, 32), ceil_div(H, 8));
    else if (p.wave_shape == 3) grd = dim3(ceil_div(W, 16), ceil_div(H, 16));
    else if (p.wave_shape == 4) grd = dim3(ceil_div(W, 8), ceil_div(H, 32));
    else if (p.wave_shape != 0 && p.wave_shape != 1) return set_error(SOC_E_INVALID_ARG, "soc_gbuffer_resolve: SOC_GB_WAVE %d", p.wave_shape);
    const unsigned long long* vis = reinterpret_cast<const unsigned long long*>(visibility);
    if (workspace) {   // per-vertex outputs once, then the per-pixel resolve reads them
        const Workspace ws = carve(workspace, mesh->vertex_count, mesh->triangle_count);
        if (mesh->vertex_count > 0)
            launch("gbuffer_vertex_setup", kWorkgroup, gbuffer_vertex_setup, ceil_div(mesh->vertex_count, 256), kWorkgroup, 0, hs(stream), *mesh, ws.vdata, p);
        launch("gbuffer_resolve", kWorkgroup, gbuffer_resolve<true>, grd, blk, 0, hs(stream), *mesh, d_materials, vis, dimg(depth), dimg(albedo),
                                                           dimg(emissive), dimg(normal), dimg(velocity), ws.vdata, p);
    } else {
        launch("gbuffer_resolve", kWorkgroup, gbuffer_resolve<false>, grd, blk, 0, hs(stream), *mesh, d_materials, vis, dimg(depth), dimg(albedo),
                                                            dimg(emissive), dimg(normal), dimg(velocity), nullptr, p);
    }
    return check_launch("gbuffer_resolve");
}
