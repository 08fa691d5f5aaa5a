// ssao.hip — SSAOGenerationTask (src/graphics/tasks/ssao_generation.inl:20-68, shader :128-214) and
// SSAOBlurTask (ssao_blur.inl:19-70, shader :91-106) as gfx950 kernels.
//
// SSAO: one lane per half-res output pixel, 16x16 pixel workgroups (a wave covers 16x4 pixels so the
// 26 depth gathers of neighbouring lanes share L1/L2 lines). Each tap is a bilinear D32 sample under
// the sampling contract, fetched as two 8-byte row pairs. The per-pixel random vector of :184-188 is
// a pure function of (uv, normal-image width): it is either evaluated inline or read from a table
// filled once per resolution by the SAME device function (soc_ssao_prepare_noise), so both give
// identical bits.
#include "soc_internal.hpp"

namespace soc {
namespace {

// ssao_generation.inl:74-103
__constant__ float c_kernel[SOC_SSAO_MAX_KERNEL][3] = {
    {0.2196607f, 0.9032637f, 0.2254677f},   {0.05916681f, 0.2201506f, 0.1430302f},  {-0.4152246f, 0.1320857f, 0.7036734f},
    {-0.3790807f, 0.1454145f, 0.100605f},   {0.3149606f, -0.1294581f, 0.7044517f},  {-0.1108412f, 0.2162839f, 0.1336278f},
    {0.658012f, -0.4395972f, 0.2919373f},   {0.5377914f, 0.3112189f, 0.426864f},    {-0.2752537f, 0.07625949f, 0.1273409f},
    {-0.1915639f, -0.4973421f, 0.3129629f}, {-0.2634767f, 0.5277923f, 0.1107446f},  {0.8242752f, 0.02434147f, 0.06049098f},
    {0.06262707f, -0.2128643f, 0.03671562f}, {-0.1795662f, -0.3543862f, 0.07924347f}, {0.06039629f, 0.24629f, 0.4501176f},
    {-0.7786345f, -0.3814852f, 0.2391262f}, {0.2792919f, 0.2487278f, 0.05185341f},  {0.1841383f, 0.1696993f, 0.8936281f},
    {-0.3479781f, 0.4725766f, 0.719685f},   {-0.1365018f, -0.2513416f, 0.470937f},  {0.1280388f, -0.563242f, 0.3419276f},
    {-0.4800232f, -0.1899473f, 0.2398808f}, {0.6389147f, 0.1191014f, 0.5271206f},   {0.1932822f, -0.3692099f, 0.6060588f},
    {-0.3465451f, -0.1654651f, 0.6746758f}, {0.2448421f, -0.1610962f, 0.1289366f}};

struct SsaoParams {
    Mat4 inv_proj;
    Mat4 proj;
    Mat4 view;
    float radius, bias, kernel_size_f;
    int ksize;     // loop bound, min(kernel_size, 26)
    int noise_w;   // textureSize(u_normal_image).x
};

// ssao_generation.inl:139-141 (no FMA contraction: keeps the sin argument as the oracle's)
__device__ __forceinline__ float ssao_rand(float cx, float cy) {
#pragma clang fp contract(off)
    return fractf(sinf(cx * 12.9898f + cy * 78.233f) * 43758.5453f);
}

// ssao_generation.inl:143-155
__device__ float ssao_noise(float px, float py, float freq) {
#pragma clang fp contract(off)
    float unit = 2560.0f / freq;
    float ix = floorf(px / unit), iy = floorf(py / unit);
    float xx = (px - unit * floorf(px / unit)) / unit, yy = (py - unit * floorf(py / unit)) / unit;
    xx = 0.5f * (1.0f - cosf(3.14159265359f * xx));
    yy = 0.5f * (1.0f - cosf(3.14159265359f * yy));
    float a = ssao_rand(ix + 0.0f, iy + 0.0f);
    float b = ssao_rand(ix + 1.0f, iy + 0.0f);
    float c = ssao_rand(ix + 0.0f, iy + 1.0f);
    float d = ssao_rand(ix + 1.0f, iy + 1.0f);
    float x1 = a * (1.0f - xx) + b * xx;
    float x2 = c * (1.0f - xx) + d * xx;
    return x1 * (1.0f - yy) + x2 * yy;
}

// random_vec = normalize(vec3(noise(uv, W*2), noise(pow(uv,1.1), pow(W*4.2, 1.5 + uv.x/10)), 0)), :184-188
__device__ float2 ssao_random_vec(float u, float v, int noise_w) {
#pragma clang fp contract(off)
    float n1 = ssao_noise(u, v, (float)(noise_w * 2));
    float n2 = ssao_noise(powf(u, 1.1f), powf(v, 1.1f), powf((float)noise_w * 4.2f, 1.5f + u / 10.0f));
    float l = sqrtf(n1 * n1 + n2 * n2 + 0.0f * 0.0f);
    return float2{n1 / l, n2 / l};
}

__global__ __launch_bounds__(256) void ssao_noise_kernel(int tw, int th, int noise_w, float2* __restrict__ table) {
    const int x = blockIdx.x * 64 + threadIdx.x, y = blockIdx.y * 4 + threadIdx.y;
    if (x >= tw || y >= th) return;
    table[(size_t)y * tw + x] = ssao_random_vec(centre_uv(x, tw), centre_uv(y, th), noise_w);
}

typedef float f2a4 __attribute__((ext_vector_type(2))) __attribute__((aligned(4)));

// Bilinear D32 depth at (u, v): the two taps of each row are one 8-byte load (i0 <= w-2).
__device__ __forceinline__ float depth_tap(const DImg& depth, float u, float v) {
    Axis ax = axis_clamp(u, depth.w), ay = axis_clamp(v, depth.h);
    f2a4 r0 = *reinterpret_cast<const f2a4*>(row_ptr<float>(depth, ay.i0) + ax.i0);
    f2a4 r1 = *reinterpret_cast<const f2a4*>(row_ptr<float>(depth, ay.i1) + ax.i0);
    return bilerp1(r0.x, r0.y, r1.x, r1.y, ax.w, ay.w);
}

template <bool TABLE>
__global__ __launch_bounds__(256) void ssao_kernel(DImg depth, DImg normal, DImg target, const float2* __restrict__ table,
                                                   SsaoParams p) {
    const int x = blockIdx.x * 16 + threadIdx.x, y = blockIdx.y * 16 + threadIdx.y;
    if (x >= target.w || y >= target.h) return;
    const float u = centre_uv(x, target.w), v = centre_uv(y, target.h);

    // frag_position = get_view_position_from_depth(in_uv, depth), :177
    const float d = depth_tap(depth, u, v);
    f4 vp = mul(p.inv_proj, f4{u * 2.0f - 1.0f, v * 2.0f - 1.0f, d, 1.0f});
    const f3 frag = f3{vp.x / vp.w, vp.y / vp.w, vp.z / vp.w};
    // normal = mat3(view) * normalize(texture(normal, uv).rgb), :178
    f4 nn = sample_h4(normal, u, v);
    const f3 n = mul3of4(p.view, normalize3(f3{nn.x, nn.y, nn.z}));

    float2 rv2 = TABLE ? table[(size_t)y * target.w + x] : ssao_random_vec(u, v, p.noise_w);
    const f3 rv = f3{rv2.x, rv2.y, 0.0f};
    const f3 t = normalize3(rv - n * dot3(rv, n));
    const f3 b = cross3(t, n);

    const float* ip = p.inv_proj.m;
    const float* P = p.proj.m;
    float occ = 0.0f;
#pragma unroll
    for (int i = 0; i < SOC_SSAO_MAX_KERNEL; ++i) {
        if (i < p.ksize) {
        const float kx = c_kernel[i][0], ky = c_kernel[i][1], kz = c_kernel[i][2];
        f3 s = t * kx + b * ky + n * kz;          // TBN * kernelSamples[i]
        s = frag + s * p.radius;
        // offset = projection * vec4(sample, 1); xy /= w; xy = xy * 0.5 + 0.5
        const float cx = P[0] * s.x + P[4] * s.y + P[8] * s.z + P[12];
        const float cy = P[1] * s.x + P[5] * s.y + P[9] * s.z + P[13];
        const float cw = P[3] * s.x + P[7] * s.y + P[11] * s.z + P[15];
        const float ox = __fdividef(cx, cw) * 0.5f + 0.5f;
        const float oy = __fdividef(cy, cw) * 0.5f + 0.5f;
        const float dd = depth_tap(depth, ox, oy);
        // get_view_position_from_depth(offset.xy, depth).z
        const float ex = ox * 2.0f - 1.0f, ey = oy * 2.0f - 1.0f;
        const float vz = ip[2] * ex + ip[6] * ey + ip[10] * dd + ip[14];
        const float vw = ip[3] * ex + ip[7] * ey + ip[11] * dd + ip[15];
        const float sd = __fdividef(vz, vw);
        const float rc = clampf(__fdividef(p.radius, fabsf(frag.z - sd)), 0.0f, 1.0f);
        const float range = rc * rc * (3.0f - 2.0f * rc);   // smoothstep(0, 1, x)
        occ += (sd >= s.z + p.bias ? 1.0f : 0.0f) * range;
        }
    }
    occ = 1.0f - (occ / p.kernel_size_f);
    row_ptr_w<uint8_t>(target, y)[x] = (uint8_t)to_unorm8(occ);
}

// ssao_blur.inl:91-106: 4x4 box at offsets -2..+1 (x outer, y inner), all taps on texel centres.
__global__ __launch_bounds__(256) void ssao_blur_kernel(DImg src, DImg dst) {
#pragma clang fp contract(off)
    const int x = blockIdx.x * 64 + threadIdx.x, y = blockIdx.y * 4 + threadIdx.y;
    if (x >= dst.w || y >= dst.h) return;
    float result = 0.0f;
#pragma unroll
    for (int dx = -2; dx < 2; ++dx)
#pragma unroll
        for (int dy = -2; dy < 2; ++dy) {
            int sx = min(max(x + dx, 0), src.w - 1), sy = min(max(y + dy, 0), src.h - 1);
            result += fetch_r8(src, sx, sy);
        }
    row_ptr_w<uint8_t>(dst, y)[x] = (uint8_t)to_unorm8(result / 16.0f);
}

// Generic blur for a target whose extent differs from the source (taps are real bilinear samples).
__global__ __launch_bounds__(256) void ssao_blur_generic(DImg src, DImg dst, float tx, float ty) {
#pragma clang fp contract(off)
    const int x = blockIdx.x * 64 + threadIdx.x, y = blockIdx.y * 4 + threadIdx.y;
    if (x >= dst.w || y >= dst.h) return;
    const float u = centre_uv(x, dst.w), v = centre_uv(y, dst.h);
    float result = 0.0f;
    for (int dx = -2; dx < 2; ++dx)
        for (int dy = -2; dy < 2; ++dy) result += sample_r8(src, u + (float)dx * tx, v + (float)dy * ty);
    row_ptr_w<uint8_t>(dst, y)[x] = (uint8_t)to_unorm8(result / 16.0f);
}

SsaoParams make_params(const soc_globals* g, const soc_img& normal) {
    SsaoParams p;
    p.inv_proj = mat4(g->camera_inverse_projection_matrix);
    p.proj = mat4(g->camera_projection_matrix);
    p.view = mat4(g->camera_view_matrix);
    p.radius = g->ssao_radius;
    p.bias = g->ssao_bias;
    p.kernel_size_f = (float)g->ssao_kernel_size;
    p.ksize = g->ssao_kernel_size < SOC_SSAO_MAX_KERNEL ? g->ssao_kernel_size : SOC_SSAO_MAX_KERNEL;
    p.noise_w = normal.width;
    return p;
}

}  // namespace
}  // namespace soc

using namespace soc;

extern "C" int soc_ssao_prepare_noise(soc_img normal, soc_img target, float* noise_table, soc_stream stream) {
    if (!noise_table) return set_error(SOC_E_INVALID_ARG, "soc_ssao_prepare_noise: null table");
    if (normal.width <= 0 || target.width <= 0 || target.height <= 0)
        return set_error(SOC_E_INVALID_ARG, "soc_ssao_prepare_noise: bad extents");
    dim3 blk(64, 4), grd(ceil_div(target.width, 64), ceil_div(target.height, 4));
    ssao_noise_kernel<<<grd, blk, 0, hs(stream)>>>(target.width, target.height, normal.width,
                                                   reinterpret_cast<float2*>(noise_table));
    return check_launch("ssao_prepare_noise");
}

extern "C" int soc_ssao_generation(const soc_globals* g, soc_img depth, soc_img normal, soc_img target,
                                   const float* noise_table, soc_stream stream) {
    if (!g) return set_error(SOC_E_INVALID_ARG, "soc_ssao_generation: null globals");
    int rc = check_img(depth, SOC_FMT_D32F, "soc_ssao_generation", "depth");
    if (!rc) rc = check_img(normal, SOC_FMT_RGBA16F, "soc_ssao_generation", "normal");
    if (!rc) rc = check_img(target, SOC_FMT_R8_UNORM, "soc_ssao_generation", "target");
    if (rc) return rc;
    if (depth.width < 2 || depth.height < 2)
        return set_error(SOC_E_SHAPE, "soc_ssao_generation: depth must be at least 2x2");
    SsaoParams p = make_params(g, normal);
    dim3 blk(16, 16), grd(ceil_div(target.width, 16), ceil_div(target.height, 16));
    if (noise_table)
        ssao_kernel<true><<<grd, blk, 0, hs(stream)>>>(dimg(depth), dimg(normal), dimg(target),
                                                       reinterpret_cast<const float2*>(noise_table), p);
    else
        ssao_kernel<false><<<grd, blk, 0, hs(stream)>>>(dimg(depth), dimg(normal), dimg(target), nullptr, p);
    return check_launch("ssao_generation");
}

extern "C" int soc_ssao_blur(const soc_globals* g, soc_img ssao, soc_img target, soc_stream stream) {
    (void)g;
    int rc = check_img(ssao, SOC_FMT_R8_UNORM, "soc_ssao_blur", "ssao");
    if (!rc) rc = check_img(target, SOC_FMT_R8_UNORM, "soc_ssao_blur", "target");
    if (rc) return rc;
    if (ssao.data == target.data) return set_error(SOC_E_INVALID_ARG, "soc_ssao_blur: source and target alias");
    dim3 blk(64, 4), grd(ceil_div(target.width, 64), ceil_div(target.height, 4));
    if (ssao.width == target.width && ssao.height == target.height && ssao.width <= 8192 && ssao.height <= 8192)
        ssao_blur_kernel<<<grd, blk, 0, hs(stream)>>>(dimg(ssao), dimg(target));
    else
        ssao_blur_generic<<<grd, blk, 0, hs(stream)>>>(dimg(ssao), dimg(target), 1.0f / (float)ssao.width,
                                                       1.0f / (float)ssao.height);
    return check_launch("ssao_blur");
}
