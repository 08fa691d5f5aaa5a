// capi.cpp — host side of the C ABI: errors, ABI introspection, the globals feed (glm / camera / jitter
// restatements of application.cpp, camera.cpp and renderer.cpp), and the render graph that orders the
// passes as Renderer::rebuild_task_graph does (renderer.cpp:929-1235).
//
// Compiled with -ffp-contract=off: the host fp32 math (AgX matrices, sun view-projection, glm
// restatements) performs exactly the roundings the oracle's C performs.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdarg>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <functional>
#include <string>
#include <mutex>
#include <vector>

#include "soc_internal.hpp"

namespace soc {

static thread_local std::string t_error;

int set_error(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    t_error = buf;
    return code;
}

void clear_error() { t_error.clear(); }

int check_img(const soc_img& im, int fmt, const char* pass, const char* what) {
    if (!img_ok(im))
        return set_error(SOC_E_INVALID_ARG, "%s: %s image invalid (data=%p %dx%d pitch=%d fmt=%d)", pass, what, im.data,
                         im.width, im.height, im.pitch_bytes, im.format);
    if (fmt > 0 && im.format != fmt)
        return set_error(SOC_E_INVALID_ARG, "%s: %s image has format %d, expected %d", pass, what, im.format, fmt);
    return SOC_OK;
}

// Tuning knobs: the environment is read once per knob and cached (not per launch);
// soc_tuning_reload() drops the cache so a changed environment takes effect.
namespace {
std::mutex g_knob_mu;
// the environment's value of each knob read so far: (name, (set, value)); a knob that is not set returns the caller's
// default on every call (the default may differ between callers, e.g. per renderer flags)
std::vector<std::pair<std::string, std::pair<bool, int>>> g_knobs;
}  // namespace

int tuning_knob(const char* name, int dflt) {
    std::lock_guard<std::mutex> lock(g_knob_mu);
    for (const auto& k : g_knobs)
        if (k.first == name) return k.second.first ? k.second.second : dflt;
    const char* e = getenv(name);
    g_knobs.emplace_back(name, std::make_pair(e != nullptr, e ? atoi(e) : 0));
    return e ? atoi(e) : dflt;
}

namespace {
thread_local std::string t_shape_error;   // a block shape launch() rejected since the last check_launch
}  // namespace

bool block_fits(const char* kernel, int bound, dim3 block) {
    const long long lanes = (long long)block.x * block.y * block.z;
    if (lanes >= 1 && lanes <= bound) return true;
    char buf[256];
    std::snprintf(buf, sizeof buf, "%s: block %ux%ux%u (%lld lanes) outside the kernel's launch bound of %d lanes", kernel,
                  block.x, block.y, block.z, lanes, bound);
    if (t_shape_error.empty()) t_shape_error = buf;
    return false;
}

extern "C" int soc_check_block_shape(int32_t bound, int32_t bx, int32_t by, int32_t bz) {
    if (bx < 0 || by < 0 || bz < 0) return set_error(SOC_E_INVALID_ARG, "soc_check_block_shape: negative extent");
    if (!block_fits("soc_check_block_shape", bound, dim3((unsigned)bx, (unsigned)by, (unsigned)bz))) {
        std::string m;
        m.swap(t_shape_error);
        return set_error(SOC_E_INVALID_ARG, "%s", m.c_str());
    }
    return SOC_OK;
}

int check_launch(const char* pass) {
    if (!t_shape_error.empty()) {
        std::string m;
        m.swap(t_shape_error);
        return set_error(SOC_E_INVALID_ARG, "%s: kernel not launched: %s", pass, m.c_str());
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return set_error(SOC_E_HIP, "%s: kernel launch failed: %s", pass, hipGetErrorString(e));
    return SOC_OK;
}

void mat4_mul_host(float out[16], const float a[16], const float b[16]) {
    float t[16];
    for (int c = 0; c < 4; ++c)
        for (int r = 0; r < 4; ++r)
            t[c * 4 + r] = a[0 * 4 + r] * b[c * 4 + 0] + a[1 * 4 + r] * b[c * 4 + 1] + a[2 * 4 + r] * b[c * 4 + 2] +
                           a[3 * 4 + r] * b[c * 4 + 3];
    std::memcpy(out, t, sizeof t);
}

// ---- AgX matrices (tone_mapping.inl:103-163), fp32, same operation order as the shader ----------
namespace {
struct H3 { float x, y, z; };
struct H2 { float x, y; };

void mat3_mul(float* out, const float* a, const float* b) {
    float t[9];
    for (int c = 0; c < 3; ++c)
        for (int r = 0; r < 3; ++r) t[c * 3 + r] = a[0 * 3 + r] * b[c * 3 + 0] + a[1 * 3 + r] * b[c * 3 + 1] + a[2 * 3 + r] * b[c * 3 + 2];
    std::memcpy(out, t, sizeof t);
}
void mat3_inverse(float* o, const float* m) {
#define M(c, r) m[(c) * 3 + (r)]
    float det = M(0, 0) * (M(1, 1) * M(2, 2) - M(2, 1) * M(1, 2)) - M(1, 0) * (M(0, 1) * M(2, 2) - M(2, 1) * M(0, 2)) +
                M(2, 0) * (M(0, 1) * M(1, 2) - M(1, 1) * M(0, 2));
    float od = 1.0f / det;
    float t[9];
    t[0 * 3 + 0] = +(M(1, 1) * M(2, 2) - M(2, 1) * M(1, 2)) * od;
    t[1 * 3 + 0] = -(M(1, 0) * M(2, 2) - M(2, 0) * M(1, 2)) * od;
    t[2 * 3 + 0] = +(M(1, 0) * M(2, 1) - M(2, 0) * M(1, 1)) * od;
    t[0 * 3 + 1] = -(M(0, 1) * M(2, 2) - M(2, 1) * M(0, 2)) * od;
    t[1 * 3 + 1] = +(M(0, 0) * M(2, 2) - M(2, 0) * M(0, 2)) * od;
    t[2 * 3 + 1] = -(M(0, 0) * M(2, 1) - M(2, 0) * M(0, 1)) * od;
    t[0 * 3 + 2] = +(M(0, 1) * M(1, 2) - M(1, 1) * M(0, 2)) * od;
    t[1 * 3 + 2] = -(M(0, 0) * M(1, 2) - M(1, 0) * M(0, 2)) * od;
    t[2 * 3 + 2] = +(M(0, 0) * M(1, 1) - M(1, 0) * M(0, 1)) * od;
#undef M
    std::memcpy(o, t, sizeof t);
}
H3 unproject(H2 xy) {  // xyYToXYZ(vec3(xy, 1))
    float Y = 1.0f;
    float X = (xy.x * Y) / xy.y;
    float Z = ((1.0f - xy.x - xy.y) * Y) / xy.y;
    return H3{X, Y, Z};
}
void primaries_to_matrix(float* out, H2 r, H2 g, H2 b, H2 w) {
    H3 R = unproject(r), G = unproject(g), B = unproject(b), W = unproject(w);
    float temp[9] = {R.x, 1.0f, R.z, G.x, 1.0f, G.z, B.x, 1.0f, B.z};
    float it[9];
    mat3_inverse(it, temp);
    H3 s = H3{it[0] * W.x + it[3] * W.y + it[6] * W.z, it[1] * W.x + it[4] * W.y + it[7] * W.z,
              it[2] * W.x + it[5] * W.y + it[8] * W.z};
    float m[9] = {R.x * s.x, R.y * s.x, R.z * s.x, G.x * s.y, G.y * s.y, G.z * s.y, B.x * s.z, B.y * s.z, B.z * s.z};
    std::memcpy(out, m, sizeof m);
}
H2 mix2(H2 a, H2 b, float t) { return H2{a.x * (1.0f - t) + b.x * t, a.y * (1.0f - t) + b.y * t}; }
}  // namespace

void agx_matrices(float compression, float M[9], float Minv[9]) {
    const H2 xr{0.64f, 0.33f}, xg{0.3f, 0.6f}, xb{0.15f, 0.06f}, xw{0.3127f, 0.3290f};
    float srgb_to_xyz[9], adjusted_to_xyz[9], xyz_to_adjusted[9];
    primaries_to_matrix(srgb_to_xyz, xr, xg, xb, xw);
    const float sf = 1.0f / (1.0f - compression);
    primaries_to_matrix(adjusted_to_xyz, mix2(xw, xr, sf), mix2(xw, xg, sf), mix2(xw, xb, sf), xw);
    mat3_inverse(xyz_to_adjusted, adjusted_to_xyz);
    mat3_mul(M, srgb_to_xyz, xyz_to_adjusted);
    mat3_inverse(Minv, M);
}

}  // namespace soc

using namespace soc;

// =================================================================================================
// ABI introspection
// =================================================================================================
namespace {
struct FieldInfo { const char* type; const char* field; size_t offset; };
#define F(T, f) {#T, #f, offsetof(T, f)}
const FieldInfo kFields[] = {
    F(soc_img, data), F(soc_img, width), F(soc_img, height), F(soc_img, pitch_bytes), F(soc_img, format),
    F(soc_auto_exposure, exposure), F(soc_auto_exposure, histogram_buckets),
    F(soc_sun_info, projection_matrix), F(soc_sun_info, view_matrix), F(soc_sun_info, projection_view_matrix),
    F(soc_sun_info, terrain_y_clip_trick), F(soc_sun_info, position), F(soc_sun_info, direction),
    F(soc_sun_info, exponential_factor), F(soc_sun_info, darkening_factor), F(soc_sun_info, bias), F(soc_sun_info, intensity),
    F(soc_point_light, position), F(soc_point_light, color), F(soc_point_light, intensity),
    F(soc_spot_light, position), F(soc_spot_light, direction), F(soc_spot_light, color), F(soc_spot_light, intensity),
    F(soc_spot_light, cut_off), F(soc_spot_light, outer_cut_off),
    F(soc_camera, position), F(soc_camera, rotation), F(soc_camera, fov_degrees), F(soc_camera, near_clip), F(soc_camera, far_clip),
    F(soc_globals, camera_projection_matrix), F(soc_globals, camera_inverse_projection_matrix),
    F(soc_globals, camera_view_matrix), F(soc_globals, camera_inverse_view_matrix),
    F(soc_globals, camera_projection_view_matrix), F(soc_globals, camera_inverse_projection_view_matrix),
    F(soc_globals, camera_previous_projection_matrix), F(soc_globals, camera_previous_inverse_projection_matrix),
    F(soc_globals, camera_previous_view_matrix), F(soc_globals, camera_previous_inverse_view_matrix),
    F(soc_globals, camera_previous_projection_view_matrix), F(soc_globals, camera_previous_inverse_projection_view_matrix),
    F(soc_globals, jitter), F(soc_globals, previous_jitter), F(soc_globals, camera_position), F(soc_globals, camera_near_clip),
    F(soc_globals, camera_far_clip), F(soc_globals, resolution), F(soc_globals, elapsed_time), F(soc_globals, delta_time),
    F(soc_globals, frame_counter), F(soc_globals, sun_info), F(soc_globals, point_light_count), F(soc_globals, spot_light_count),
    F(soc_globals, point_lights), F(soc_globals, spot_lights), F(soc_globals, terrain_offset), F(soc_globals, terrain_scale),
    F(soc_globals, terrain_height_scale), F(soc_globals, terrain_midpoint), F(soc_globals, terrain_delta),
    F(soc_globals, terrain_min_depth), F(soc_globals, terrain_max_depth), F(soc_globals, terrain_min_tess_level),
    F(soc_globals, terrain_max_tess_level), F(soc_globals, terrain_y_clip_trick), F(soc_globals, terrain_previous_y_clip_trick),
    F(soc_globals, filter_radius), F(soc_globals, ssao_bias), F(soc_globals, ssao_radius), F(soc_globals, ssao_kernel_size),
    F(soc_globals, ambient), F(soc_globals, ambient_occlussion_strength), F(soc_globals, emissive_bloom_strength),
    F(soc_globals, focal_length), F(soc_globals, plane_in_focus), F(soc_globals, aperture), F(soc_globals, adjustment_speed),
    F(soc_globals, log_min_luminance), F(soc_globals, log_max_luminance), F(soc_globals, target_luminance),
    F(soc_globals, saturation), F(soc_globals, agxDs_linear_section), F(soc_globals, peak), F(soc_globals, compression),
    F(soc_frame_images, albedo), F(soc_frame_images, emissive), F(soc_frame_images, normal), F(soc_frame_images, depth),
    F(soc_frame_images, velocity), F(soc_frame_images, shadow), F(soc_frame_images, noise), F(soc_frame_images, bloom_mips),
    F(soc_frame_images, ssao), F(soc_frame_images, ssao_blur), F(soc_frame_images, clouds), F(soc_frame_images, color),
    F(soc_frame_images, history_color), F(soc_frame_images, history_velocity), F(soc_frame_images, output),
    F(soc_frame_images, ssao_noise_table), F(soc_frame_images, auto_exposure), F(soc_frame_images, d_globals),
    F(soc_frame_images, bloom_output), F(soc_frame_images, clouds_workspace),
    F(soc_mesh, positions), F(soc_mesh, normals), F(soc_mesh, uvs), F(soc_mesh, indices), F(soc_mesh, materials),
    F(soc_mesh, vertex_count), F(soc_mesh, triangle_count), F(soc_mesh, model_matrix), F(soc_mesh, normal_matrix),
    F(soc_material, albedo), F(soc_material, emissive), F(soc_material, albedo_factor), F(soc_material, emissive_factor),
    F(soc_material, flags), F(soc_material, has_emissive), F(soc_material, pad), F(soc_material, normal_map),
    F(soc_material, normal_image), F(soc_material, max_anisotropy), F(soc_material, pad2), F(soc_material, paired_texels),
    F(soc_raster_scene, mesh), F(soc_raster_scene, materials), F(soc_raster_scene, material_count),
    F(soc_raster_scene, shadow), F(soc_raster_scene, visibility), F(soc_raster_scene, workspace),
    F(soc_entity, position), F(soc_entity, rotation), F(soc_entity, scale), F(soc_entity, components),
    F(soc_entity, color), F(soc_entity, intensity), F(soc_entity, cut_off), F(soc_entity, outer_cut_off),
    F(soc_pass_desc, name), F(soc_pass_desc, group), F(soc_pass_desc, phase), F(soc_pass_desc, flags),
    F(soc_pass_desc, read_count), F(soc_pass_desc, write_count), F(soc_pass_desc, reads), F(soc_pass_desc, writes),
};
#undef F
}  // namespace

extern "C" int32_t soc_abi_version(void) { return SOC_RT_ABI_VERSION; }

extern "C" size_t soc_abi_sizeof(const char* t) {
    if (!t) return 0;
    std::string s(t);
    if (s == "soc_img") return sizeof(soc_img);
    if (s == "soc_globals") return sizeof(soc_globals);
    if (s == "soc_sun_info") return sizeof(soc_sun_info);
    if (s == "soc_point_light") return sizeof(soc_point_light);
    if (s == "soc_spot_light") return sizeof(soc_spot_light);
    if (s == "soc_auto_exposure") return sizeof(soc_auto_exposure);
    if (s == "soc_camera") return sizeof(soc_camera);
    if (s == "soc_frame_images") return sizeof(soc_frame_images);
    if (s == "soc_mesh") return sizeof(soc_mesh);
    if (s == "soc_material") return sizeof(soc_material);
    if (s == "soc_raster_scene") return sizeof(soc_raster_scene);
    if (s == "soc_pass_desc") return sizeof(soc_pass_desc);
    if (s == "soc_entity") return sizeof(soc_entity);
    return 0;
}

extern "C" int64_t soc_abi_offsetof(const char* t, const char* f) {
    if (!t || !f) return -1;
    for (const auto& e : kFields)
        if (!std::strcmp(e.type, t) && !std::strcmp(e.field, f)) return (int64_t)e.offset;
    return -1;
}

extern "C" const char* soc_last_error_string(void) { return t_error.c_str(); }
extern "C" const char* soc_device_arch(void) { return "gfx950"; }

// =================================================================================================
// glm restatements (glm 0.9.9 / 1.0 scalar code paths, RH_NO clip control: quirk Q1)
// =================================================================================================
extern "C" void soc_mat4_mul(float out[16], const float a[16], const float b[16]) { mat4_mul_host(out, a, b); }

static inline void ident(float* m) {
    std::memset(m, 0, 16 * sizeof(float));
    m[0] = m[5] = m[10] = m[15] = 1.0f;
}

extern "C" void soc_mat4_perspective_rh_no(float out[16], float fovy, float aspect, float zNear, float zFar) {
    const float tanHalfFovy = std::tan(fovy / 2.0f);
    std::memset(out, 0, 16 * sizeof(float));
    out[0 * 4 + 0] = 1.0f / (aspect * tanHalfFovy);
    out[1 * 4 + 1] = 1.0f / tanHalfFovy;
    out[2 * 4 + 2] = -(zFar + zNear) / (zFar - zNear);
    out[2 * 4 + 3] = -1.0f;
    out[3 * 4 + 2] = -(2.0f * zFar * zNear) / (zFar - zNear);
}

extern "C" void soc_mat4_ortho_rh_no(float out[16], float l, float r, float b, float t, float zNear, float zFar) {
    ident(out);
    out[0 * 4 + 0] = 2.0f / (r - l);
    out[1 * 4 + 1] = 2.0f / (t - b);
    out[2 * 4 + 2] = -2.0f / (zFar - zNear);
    out[3 * 4 + 0] = -(r + l) / (r - l);
    out[3 * 4 + 1] = -(t + b) / (t - b);
    out[3 * 4 + 2] = -(zFar + zNear) / (zFar - zNear);
}

namespace {
struct V3h { float x, y, z; };
inline V3h sub(V3h a, V3h b) { return V3h{a.x - b.x, a.y - b.y, a.z - b.z}; }
inline float dot(V3h a, V3h b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline V3h cross(V3h a, V3h b) { return V3h{a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y}; }
inline V3h normalize(V3h v) {  // glm: v * inversesqrt(dot(v, v)), inversesqrt = 1 / sqrt
    float s = 1.0f / std::sqrt(dot(v, v));
    return V3h{v.x * s, v.y * s, v.z * s};
}
}  // namespace

extern "C" void soc_mat4_look_at_rh(float out[16], const float eye_[3], const float center_[3], const float up_[3]) {
    const V3h eye{eye_[0], eye_[1], eye_[2]}, center{center_[0], center_[1], center_[2]}, up{up_[0], up_[1], up_[2]};
    const V3h f = normalize(sub(center, eye));
    const V3h s = normalize(cross(f, up));
    const V3h u = cross(s, f);
    ident(out);
    out[0 * 4 + 0] = s.x; out[1 * 4 + 0] = s.y; out[2 * 4 + 0] = s.z;
    out[0 * 4 + 1] = u.x; out[1 * 4 + 1] = u.y; out[2 * 4 + 1] = u.z;
    out[0 * 4 + 2] = -f.x; out[1 * 4 + 2] = -f.y; out[2 * 4 + 2] = -f.z;
    out[3 * 4 + 0] = -dot(s, eye);
    out[3 * 4 + 1] = -dot(u, eye);
    out[3 * 4 + 2] = dot(f, eye);
}

// glm compute_inverse<4,4> (func_matrix.inl), scalar path.
extern "C" void soc_mat4_inverse(float out[16], const float mm[16]) {
#define m(c, r) mm[(c) * 4 + (r)]
    const float Coef00 = m(2, 2) * m(3, 3) - m(3, 2) * m(2, 3);
    const float Coef02 = m(1, 2) * m(3, 3) - m(3, 2) * m(1, 3);
    const float Coef03 = m(1, 2) * m(2, 3) - m(2, 2) * m(1, 3);
    const float Coef04 = m(2, 1) * m(3, 3) - m(3, 1) * m(2, 3);
    const float Coef06 = m(1, 1) * m(3, 3) - m(3, 1) * m(1, 3);
    const float Coef07 = m(1, 1) * m(2, 3) - m(2, 1) * m(1, 3);
    const float Coef08 = m(2, 1) * m(3, 2) - m(3, 1) * m(2, 2);
    const float Coef10 = m(1, 1) * m(3, 2) - m(3, 1) * m(1, 2);
    const float Coef11 = m(1, 1) * m(2, 2) - m(2, 1) * m(1, 2);
    const float Coef12 = m(2, 0) * m(3, 3) - m(3, 0) * m(2, 3);
    const float Coef14 = m(1, 0) * m(3, 3) - m(3, 0) * m(1, 3);
    const float Coef15 = m(1, 0) * m(2, 3) - m(2, 0) * m(1, 3);
    const float Coef16 = m(2, 0) * m(3, 2) - m(3, 0) * m(2, 2);
    const float Coef18 = m(1, 0) * m(3, 2) - m(3, 0) * m(1, 2);
    const float Coef19 = m(1, 0) * m(2, 2) - m(2, 0) * m(1, 2);
    const float Coef20 = m(2, 0) * m(3, 1) - m(3, 0) * m(2, 1);
    const float Coef22 = m(1, 0) * m(3, 1) - m(3, 0) * m(1, 1);
    const float Coef23 = m(1, 0) * m(2, 1) - m(2, 0) * m(1, 1);
    const float Fac0[4] = {Coef00, Coef00, Coef02, Coef03};
    const float Fac1[4] = {Coef04, Coef04, Coef06, Coef07};
    const float Fac2[4] = {Coef08, Coef08, Coef10, Coef11};
    const float Fac3[4] = {Coef12, Coef12, Coef14, Coef15};
    const float Fac4[4] = {Coef16, Coef16, Coef18, Coef19};
    const float Fac5[4] = {Coef20, Coef20, Coef22, Coef23};
    const float Vec0[4] = {m(1, 0), m(0, 0), m(0, 0), m(0, 0)};
    const float Vec1[4] = {m(1, 1), m(0, 1), m(0, 1), m(0, 1)};
    const float Vec2[4] = {m(1, 2), m(0, 2), m(0, 2), m(0, 2)};
    const float Vec3[4] = {m(1, 3), m(0, 3), m(0, 3), m(0, 3)};
    float Inv[4][4];
    for (int i = 0; i < 4; ++i) {
        Inv[0][i] = Vec1[i] * Fac0[i] - Vec2[i] * Fac1[i] + Vec3[i] * Fac2[i];
        Inv[1][i] = Vec0[i] * Fac0[i] - Vec2[i] * Fac3[i] + Vec3[i] * Fac4[i];
        Inv[2][i] = Vec0[i] * Fac1[i] - Vec1[i] * Fac3[i] + Vec3[i] * Fac5[i];
        Inv[3][i] = Vec0[i] * Fac2[i] - Vec1[i] * Fac4[i] + Vec2[i] * Fac5[i];
    }
    const float SignA[4] = {+1.0f, -1.0f, +1.0f, -1.0f}, SignB[4] = {-1.0f, +1.0f, -1.0f, +1.0f};
    float Inverse[4][4];
    for (int i = 0; i < 4; ++i) {
        Inverse[0][i] = Inv[0][i] * SignA[i];
        Inverse[1][i] = Inv[1][i] * SignB[i];
        Inverse[2][i] = Inv[2][i] * SignA[i];
        Inverse[3][i] = Inv[3][i] * SignB[i];
    }
    const float Row0[4] = {Inverse[0][0], Inverse[1][0], Inverse[2][0], Inverse[3][0]};
    const float Dot0[4] = {m(0, 0) * Row0[0], m(0, 1) * Row0[1], m(0, 2) * Row0[2], m(0, 3) * Row0[3]};
    const float Dot1 = (Dot0[0] + Dot0[1]) + (Dot0[2] + Dot0[3]);
    const float OneOverDeterminant = 1.0f / Dot1;
    for (int c = 0; c < 4; ++c)
        for (int r = 0; r < 4; ++r) out[c * 4 + r] = Inverse[c][r] * OneOverDeterminant;
#undef m
}

static inline float radians(float deg) { return deg * 0.01745329251994329576923690768489f; }

// glm::rotateX/Y/Z (gtx/rotate_vector.inl)
static V3h rotate_x(V3h v, float a) { float c = std::cos(a), s = std::sin(a); return V3h{v.x, v.y * c - v.z * s, v.y * s + v.z * c}; }
static V3h rotate_y(V3h v, float a) { float c = std::cos(a), s = std::sin(a); return V3h{v.x * c + v.z * s, v.y, -v.x * s + v.z * c}; }
static V3h rotate_z(V3h v, float a) { float c = std::cos(a), s = std::sin(a); return V3h{v.x * c - v.y * s, v.x * s + v.y * c, v.z}; }

extern "C" void soc_tuning_reload(void) {
    std::lock_guard<std::mutex> lock(g_knob_mu);
    g_knobs.clear();
}

extern "C" int soc_globals_init_defaults(soc_globals* g, int32_t width, int32_t height) {
    if (!g || width <= 0 || height <= 0) return set_error(SOC_E_INVALID_ARG, "soc_globals_init_defaults: bad args");
    std::memset(g, 0, sizeof *g);
    // renderer.cpp:72-107
    g->terrain_offset[0] = g->terrain_offset[1] = g->terrain_offset[2] = 0.0f;
    g->terrain_scale[0] = g->terrain_scale[1] = 100.0f;
    g->terrain_height_scale = 70.0f;
    g->terrain_midpoint = 0.2f;
    g->terrain_delta = 8.0f;
    g->terrain_min_depth = 1.0f;
    g->terrain_max_depth = 100.0f;
    g->terrain_min_tess_level = 1;
    g->terrain_max_tess_level = 3;
    g->ssao_bias = 0.025f;
    g->ssao_radius = 0.3f;
    g->ssao_kernel_size = 26;
    g->ambient[0] = g->ambient[1] = g->ambient[2] = 0.1f;
    g->ambient_occlussion_strength = 1.2f;
    g->emissive_bloom_strength = 2.0f;
    g->focal_length = 5.0f;
    g->plane_in_focus = 1.0f;
    g->aperture = 8.0f;
    g->adjustment_speed = 1.0f;
    g->log_min_luminance = -15.0f;
    g->log_max_luminance = 15.0f;
    g->target_luminance = 0.2140f;
    g->elapsed_time = 0.0f;
    g->log_min_luminance = std::log2(g->target_luminance / std::exp2(g->log_min_luminance));
    g->log_max_luminance = std::log2(g->target_luminance / std::exp2(g->log_max_luminance));
    g->saturation = 1.0f;
    g->agxDs_linear_section = 0.18f;
    g->peak = 1.0f;
    g->compression = 0.15f;
    g->frame_counter = 0;
    // sun, renderer.cpp:109-133 (angle_direction = {4, 0, 0}, renderer.hpp:67)
    const V3h light_position{-3.2f, 40.0f, -4.0f};
    const float planes = 16.0f;
    float light_projection[16];
    soc_mat4_ortho_rh_no(light_projection, -planes, planes, -planes, planes, -planes, planes);
    V3h dir{0.0f, -1.0f, 0.0f};
    dir = rotate_x(dir, radians(4.0f));
    dir = rotate_y(dir, radians(0.0f));
    dir = rotate_z(dir, radians(0.0f));
    const float eye[3] = {light_position.x, light_position.y, light_position.z};
    const float center[3] = {light_position.x + dir.x, light_position.y + dir.y, light_position.z + dir.z};
    const float up[3] = {0.0f, -1.0f, 0.0f};
    float light_view[16], pv[16];
    soc_mat4_look_at_rh(light_view, eye, center, up);
    mat4_mul_host(pv, light_projection, light_view);
    std::memcpy(g->sun_info.projection_matrix, light_projection, sizeof light_projection);
    std::memcpy(g->sun_info.view_matrix, light_view, sizeof light_view);
    std::memcpy(g->sun_info.projection_view_matrix, pv, sizeof pv);
    for (int r = 0; r < 4; ++r) g->sun_info.terrain_y_clip_trick[r] = pv[1 * 4 + r];  // pv * (0,1,0,0)
    g->sun_info.position[0] = light_position.x; g->sun_info.position[1] = light_position.y; g->sun_info.position[2] = light_position.z;
    g->sun_info.direction[0] = dir.x; g->sun_info.direction[1] = dir.y; g->sun_info.direction[2] = dir.z;
    g->sun_info.exponential_factor = -80.0f;
    g->sun_info.darkening_factor = 1.0f;
    g->sun_info.bias = 0.0001f;
    g->sun_info.intensity = 1.0f;
    g->resolution[0] = width;
    g->resolution[1] = height;
    // Camera3D defaults (camera.hpp:74-75)
    g->camera_near_clip = 0.1f;
    g->camera_far_clip = 1000.0f;
    return SOC_OK;
}

extern "C" int soc_globals_frame_update(soc_globals* g, const soc_camera* cam, int32_t width, int32_t height, float delta_time,
                                        uint32_t* jitter_index) {
    if (!g || !cam || !jitter_index || width <= 0 || height <= 0)
        return set_error(SOC_E_INVALID_ARG, "soc_globals_frame_update: bad args");
    // Camera3D::resize (camera.cpp:6-10)
    float proj[16];
    const float aspect = (float)width / (float)height;
    soc_mat4_perspective_rh_no(proj, radians(cam->fov_degrees), aspect, cam->near_clip, cam->far_clip);
    proj[1 * 4 + 1] *= -1.0f;
    // ControlledCamera3D::update (camera.cpp:36-56), no input
    float ry = cam->rotation[1];
    const float MAX_ROT = 1.56825555556f;
    if (ry > MAX_ROT) ry = MAX_ROT;
    if (ry < -MAX_ROT) ry = -MAX_ROT;
    const float rx = cam->rotation[0];
    const V3h fwd = normalize(V3h{std::cos(rx) * std::cos(ry), -std::sin(ry), std::sin(rx) * std::cos(ry)});
    const float eye[3] = {cam->position[0], cam->position[1], cam->position[2]};
    const float center[3] = {eye[0] + fwd.x, eye[1] + fwd.y, eye[2] + fwd.z};
    const float up[3] = {0.0f, 1.0f, 0.0f};
    float view[16];
    soc_mat4_look_at_rh(view, eye, center, up);
    // Application::update jitter (application.cpp:113-131)
    const float gr = 1.32471795724474602596f, a1 = 1.0f / gr, a2 = 1.0f / (gr * gr);
    auto gmod = [](float x, float y) { return x - y * std::floor(x / y); };
    const float idx = (float)(*jitter_index);
    float jx = gmod(0.5f + a1 * (idx + 1.0f), 1.0f) - 0.5f;
    float jy = gmod(0.5f + a2 * (idx + 1.0f), 1.0f) - 0.5f;
    jx = jx * (1.0f / (float)width);
    jy = jy * (1.0f / (float)height);
    *jitter_index = (*jitter_index + 1) % 32;
    proj[3 * 4 + 0] += jx;
    proj[3 * 4 + 1] += jy;
    float inv_proj[16], inv_view[16], pv[16], inv_pv[16];
    soc_mat4_inverse(inv_proj, proj);
    soc_mat4_inverse(inv_view, view);
    mat4_mul_host(pv, proj, view);
    mat4_mul_host(inv_pv, inv_proj, inv_view);
    // shift current -> previous (application.cpp:139-146)
    std::memcpy(g->camera_previous_projection_matrix, g->camera_projection_matrix, 64);
    std::memcpy(g->camera_previous_inverse_projection_matrix, g->camera_inverse_projection_matrix, 64);
    std::memcpy(g->camera_previous_view_matrix, g->camera_view_matrix, 64);
    std::memcpy(g->camera_previous_inverse_view_matrix, g->camera_inverse_view_matrix, 64);
    std::memcpy(g->camera_previous_projection_view_matrix, g->camera_projection_view_matrix, 64);
    std::memcpy(g->camera_previous_inverse_projection_view_matrix, g->camera_inverse_projection_view_matrix, 64);
    std::memcpy(g->terrain_previous_y_clip_trick, g->terrain_y_clip_trick, 16);
    std::memcpy(g->previous_jitter, g->jitter, 8);
    std::memcpy(g->camera_projection_matrix, proj, 64);
    std::memcpy(g->camera_inverse_projection_matrix, inv_proj, 64);
    std::memcpy(g->camera_view_matrix, view, 64);
    std::memcpy(g->camera_inverse_view_matrix, inv_view, 64);
    std::memcpy(g->camera_projection_view_matrix, pv, 64);
    std::memcpy(g->camera_inverse_projection_view_matrix, inv_pv, 64);
    for (int r = 0; r < 4; ++r) g->terrain_y_clip_trick[r] = pv[1 * 4 + r];
    g->jitter[0] = jx;
    g->jitter[1] = jy;
    g->camera_near_clip = cam->near_clip;
    g->camera_far_clip = cam->far_clip;
    g->resolution[0] = width;
    g->resolution[1] = height;
    for (int i = 0; i < 3; ++i) g->camera_position[i] = cam->position[i];
    g->delta_time = delta_time;
    g->elapsed_time += delta_time;
    g->frame_counter++;
    return SOC_OK;
}

// Scene::update (src/ecs/scene.cpp:47-118): transforms (glm translate * toMat4(quat(euler)) * scale, and
// transpose(inverse(model))) and the light lists.
static void quat_euler_to_mat4(float out[16], const float euler_rad[3]) {
    // glm::qua(vec3 eulerAngle) (gtc/quaternion.inl) then mat3_cast / toMat4 (gtx/quaternion.inl)
    const float cx = std::cos(euler_rad[0] * 0.5f), cy = std::cos(euler_rad[1] * 0.5f), cz = std::cos(euler_rad[2] * 0.5f);
    const float sx = std::sin(euler_rad[0] * 0.5f), sy = std::sin(euler_rad[1] * 0.5f), sz = std::sin(euler_rad[2] * 0.5f);
    const float w = cx * cy * cz + sx * sy * sz;
    const float x = sx * cy * cz - cx * sy * sz;
    const float y = cx * sy * cz + sx * cy * sz;
    const float z = cx * cy * sz - sx * sy * cz;
    const float qxx = x * x, qyy = y * y, qzz = z * z, qxz = x * z, qxy = x * y, qyz = y * z, qwx = w * x, qwy = w * y,
                qwz = w * z;
    ident(out);
    out[0 * 4 + 0] = 1.0f - 2.0f * (qyy + qzz);
    out[0 * 4 + 1] = 2.0f * (qxy + qwz);
    out[0 * 4 + 2] = 2.0f * (qxz - qwy);
    out[1 * 4 + 0] = 2.0f * (qxy - qwz);
    out[1 * 4 + 1] = 1.0f - 2.0f * (qxx + qzz);
    out[1 * 4 + 2] = 2.0f * (qyz + qwx);
    out[2 * 4 + 0] = 2.0f * (qxz + qwy);
    out[2 * 4 + 1] = 2.0f * (qyz - qwx);
    out[2 * 4 + 2] = 1.0f - 2.0f * (qxx + qyy);
}

extern "C" int soc_scene_update(soc_globals* g, const soc_entity* e, int32_t count, float* model_matrices,
                                float* normal_matrices) {
    if (!g || count < 0 || (count > 0 && !e)) return set_error(SOC_E_INVALID_ARG, "soc_scene_update: bad arguments");
    int np = 0, ns = 0;
    for (int i = 0; i < count; ++i) {
        np += (e[i].components & SOC_ENTITY_POINT_LIGHT) ? 1 : 0;
        ns += (e[i].components & SOC_ENTITY_SPOT_LIGHT) ? 1 : 0;
    }
    if (np > SOC_MAX_POINT_LIGHTS || ns > SOC_MAX_SPOT_LIGHTS)
        return set_error(SOC_E_SHAPE, "soc_scene_update: %d point / %d spot lights exceed %d / %d", np, ns,
                         SOC_MAX_POINT_LIGHTS, SOC_MAX_SPOT_LIGHTS);
    g->point_light_count = 0;
    g->spot_light_count = 0;
    for (int i = 0; i < count; ++i) {
        const soc_entity& t = e[i];
        if (model_matrices || normal_matrices) {   // scene.cpp:64-68
            float T[16], R[16], S[16], TR[16], M[16], inv[16];
            ident(T);
            T[12] = t.position[0];
            T[13] = t.position[1];
            T[14] = t.position[2];
            const float eul[3] = {radians(t.rotation[0]), radians(t.rotation[1]), radians(t.rotation[2])};
            quat_euler_to_mat4(R, eul);
            ident(S);
            S[0] = t.scale[0];
            S[5] = t.scale[1];
            S[10] = t.scale[2];
            mat4_mul_host(TR, T, R);
            mat4_mul_host(M, TR, S);
            if (model_matrices) std::memcpy(model_matrices + 16 * i, M, sizeof M);
            if (normal_matrices) {
                soc_mat4_inverse(inv, M);
                for (int c = 0; c < 4; ++c)
                    for (int r = 0; r < 4; ++r) normal_matrices[16 * i + c * 4 + r] = inv[r * 4 + c];
            }
        }
        if (t.components & SOC_ENTITY_POINT_LIGHT) {   // scene.cpp:87-96
            soc_point_light& L = g->point_lights[g->point_light_count++];
            for (int k = 0; k < 3; ++k) {
                L.position[k] = t.position[k];
                L.color[k] = t.color[k];
            }
            L.intensity = t.intensity;
        }
        if (t.components & SOC_ENTITY_SPOT_LIGHT) {    // scene.cpp:98-116
            V3h dir{0.0f, -1.0f, 0.0f};
            dir = rotate_x(dir, radians(t.rotation[0]));
            dir = rotate_y(dir, radians(t.rotation[1]));
            dir = rotate_z(dir, radians(t.rotation[2]));
            soc_spot_light& L = g->spot_lights[g->spot_light_count++];
            for (int k = 0; k < 3; ++k) {
                L.position[k] = t.position[k];
                L.color[k] = t.color[k];
            }
            L.direction[0] = dir.x;
            L.direction[1] = dir.y;
            L.direction[2] = dir.z;
            L.intensity = t.intensity;
            L.cut_off = std::cos(radians(t.cut_off));
            L.outer_cut_off = std::cos(radians(t.outer_cut_off));
        }
    }
    return SOC_OK;
}

extern "C" int soc_upload_globals(const soc_globals* g, soc_globals* d_globals, soc_stream stream) {
    if (!g || !d_globals) return set_error(SOC_E_INVALID_ARG, "soc_upload_globals: null argument");
    hipError_t e = hipMemcpyAsync(d_globals, g, sizeof(soc_globals), hipMemcpyHostToDevice, hs(stream));
    if (e != hipSuccess) return set_error(SOC_E_HIP, "soc_upload_globals: %s", hipGetErrorString(e));
    return SOC_OK;
}

// =================================================================================================
// Render graph (renderer.cpp:929-1235, live passes only; SSR / Hi-Z / DOF are dead or disabled)
//
// Every pass declares the frame resources it reads and writes (the Daxa task-uses block,
// e.g. composition.inl:10-21). The graph keeps the registration order, which is the reference's
// add_task order, and derives from the uses what Daxa derives its barriers from: each pass's
// dependencies on earlier passes (RAW, WAR, WAW). On one HIP stream stream order already satisfies
// them; they matter for SOC_PASS_ASYNC passes, which run on a second stream of the renderer
// (the async-compute queue the reference leaves unused): such a pass waits only for the passes it
// depends on, and a pass on the caller's stream waits for it only if it depends on it.
// =================================================================================================
struct soc_renderer {
    using PassFn = std::function<int(const soc_globals*, hipStream_t)>;
    struct Pass {
        std::string name, group;
        int phase = SOC_PHASE_PRE_EXPOSURE;
        uint64_t reads = 0, writes = 0;
        uint32_t flags = 0;
        PassFn run;
        std::function<bool()> skip;   // true: the pass has no work this call (no launch, no timing)
        std::vector<int> deps;        // derived: earlier passes this one must follow
        std::vector<int> carry;       // derived: passes of the PREVIOUS frame this one must follow (ring edges)
        bool signal = false;          // derived: a pass of the other lane depends on this one (records `done`)
        bool timed = false;
        std::vector<hipEvent_t> ev0, ev1;  // timing ring of SOC_RENDERER_TIMING_RING frames
        int next = 0, count = 0, last = -1;
        hipEvent_t done = nullptr;    // cross-lane completion event (created on first use)
        bool done_recorded = false;   // `done` holds this pass's latest run
    };
    struct UserPass {
        soc_pass_desc desc;
        std::string name, group, before;
        soc_pass_callback fn;
        void* user;
    };
    soc_frame_images img{};
    soc_raster_scene scene{};
    bool has_scene = false;
    std::vector<Pass> passes;
    std::vector<UserPass> user_passes;
    uint32_t flags = 0;
    int hist = 0;               // history slot read as "previous" this frame
    uint64_t total_pixels = 0;  // 0 = this frame
    int wide = 0;
    // pinned staging ring for the device globals upload (lights)
    soc_globals* staging = nullptr;
    hipEvent_t staging_ev[4] = {nullptr, nullptr, nullptr, nullptr};
    int staging_slot = 0;
    // second lane (SOC_PASS_ASYNC passes: CloudRendering is VALU-bound and reads only depth and noise, so
    // it overlaps the memory-bound bloom / SSAO passes)
    bool async = true;
    int side_device = -1;
    hipStream_t side = nullptr;
    hipEvent_t fork_ev = nullptr, join_ev = nullptr;
    // the second lane's hardware queue (ensure_side_lane): a stream of high or low priority, so the lane never shares
    // the caller's queue. Auto mode (the default) times frames with each and keeps the faster: lane_q = {high, low},
    // side_queue = 1 (high) / 2 (low) once chosen, -1 while the probe runs; 0 = normal priority (shared pool).
    hipStream_t lane_q[2] = {nullptr, nullptr};
    int side_queue = -1;
    int probe_frames = 0;
    hipEvent_t probe_ev[16] = {};
    hipEvent_t switch_ev = nullptr;
    // 8 partial luminance histograms of the fused composition + histogram pass (renderer-owned, 8 KiB)
    uint32_t* hist_scratch = nullptr;
    // a raster workspace of the sun shadow draw's own, so it can run on the second lane beside the depth prepass and
    // the G-buffer (they share scene.workspace's screen vertices and entry lists otherwise)
    void* shadow_ws = nullptr;
    size_t shadow_ws_bytes = 0;
    // this execute call runs both phases: the resolve folds the partial histograms itself (no fold launch)
    bool fold_in_resolve = false;
    // sky split configured (graph) / active this frame (the pair path applies at the globals' resolution)
    bool sky_split = false, sky_split_active = false;
    bool bloom_in_comp = false;          // SOC_RENDERER_BLOOM_IN_COMPOSITION applies to this graph
    bool bloom_in_comp_ok = false;       // ... and the fused pair path applies at this frame's globals resolution
    // the caller's stream is ordered after all second-lane work of the previous call (its join or an equivalent wait)
    bool main_after_side = true;
    // SOC_RENDERER_STATIC_INPUTS: a call of this graph has completed, so the frame inputs the caller wrote before its
    // first call are ordered before the second lane (that call's fork). Until then every second-lane pass waits for the
    // fork, as without the flag (the first call after create or a graph rebuild may follow the caller's input writes).
    bool inputs_ordered = false;
};

namespace {
using PassFn = soc_renderer::PassFn;

uint64_t res_mask(std::initializer_list<int> ids) {
    uint64_t m = 0;
    for (int i : ids) m |= 1ull << i;
    return m;
}

// SOC_RENDERER_VELOCITY_SLOTS: the frame's velocity image is the history_velocity slot the next frame reads as its
// previous velocity, so VELOCITY and PREVIOUS_VELOCITY name the two slots of one ping-pong pair; a use of either is
// taken as a use of both, which orders a next frame's velocity write after every reader of the slot it overwrites.
uint64_t widen_velocity(const soc_renderer* r, uint64_t m) {
    const uint64_t both = (1ull << SOC_RES_VELOCITY) | (1ull << SOC_RES_PREVIOUS_VELOCITY);
    return (r->flags & SOC_RENDERER_VELOCITY_SLOTS) && (m & both) ? m | both : m;
}

// The frame's velocity image: images.velocity, or with SOC_RENDERER_VELOCITY_SLOTS the history_velocity slot this frame
// resolves into (the reference copies velocity there after TAA, renderer.cpp:1185-1189; here its producer writes it there).
soc_img frame_velocity(const soc_renderer* r) {
    return (r->flags & SOC_RENDERER_VELOCITY_SLOTS) ? r->img.history_velocity[1 - r->hist] : r->img.velocity;
}

// The sky lane runs at high priority in this frame: chosen by the lane probe (or the knob), or one of the probe's
// high-priority windows. Evaluated inside the pass callbacks, after this call's frame_lane_probe.
bool sky_lane_high(const soc_renderer* r) {
    return r->side_queue == 1 || (r->side_queue == -1 && r->lane_q[0] && r->side == r->lane_q[0]);
}
// SOC_RENDERER_BLOOM_IN_COMPOSITION in this frame: the bloom's last stage inside Composition where the sky lane is the
// critical path (high priority, as the lane probe's high windows too, so the probe times what would run), the fourth
// bloom pass then recording nothing. Both callbacks of a frame see the same lane (set before the passes are issued).
// Re-checked every frame: a frame whose globals resolution differs from the images takes Composition's generic
// path, which cannot compute the bloom, so the fourth pass must run then.
bool bloom_in_comp_active(const soc_renderer* r) {
    // SOC_RENDERER_BLOOM_IN_COMP_ANY_LANE=1: also beside the low-priority sky lane (measurement knob)
    return r->bloom_in_comp && r->bloom_in_comp_ok && (sky_lane_high(r) || tuning_knob("SOC_RENDERER_BLOOM_IN_COMP_ANY_LANE", 0));
}

soc_renderer::Pass& add_pass(soc_renderer* r, std::string name, std::string group, int phase, uint64_t reads,
                             uint64_t writes, PassFn fn, uint32_t flags = 0) {
    soc_renderer::Pass p;
    p.name = std::move(name);
    p.group = std::move(group);
    p.phase = phase;
    p.reads = widen_velocity(r, reads);
    p.writes = widen_velocity(r, writes);
    p.flags = flags;
    p.run = std::move(fn);
    r->passes.push_back(std::move(p));
    return r->passes.back();
}

// The fused histogram's 8 partial copies: allocated on the first PRE phase and cleared on the caller's stream
// BEFORE the second lane is forked, so the fork orders the clear ahead of the sky lane's sky_compose bins.
// (Round 2 cleared it with hipMemset on the null stream from inside the sky lane's pass: a non-blocking stream
// is not ordered after null-stream work, so a first frame's sky bins could land before the clear and be wiped,
// or land in stale memory: DESIGN.md §2.2.)
int ensure_hist_scratch(soc_renderer* r, hipStream_t s) {
    if (r->hist_scratch) return SOC_OK;
    if (hipMalloc((void**)&r->hist_scratch, SOC_HISTOGRAM_SCRATCH_WORDS * sizeof(uint32_t)) != hipSuccess) {
        r->hist_scratch = nullptr;
        return set_error(SOC_E_HIP, "soc_renderer_execute: histogram scratch allocation failed");
    }
    if (hipMemsetAsync(r->hist_scratch, 0, SOC_HISTOGRAM_SCRATCH_WORDS * sizeof(uint32_t), s) != hipSuccess)
        return set_error(SOC_E_HIP, "soc_renderer_execute: histogram scratch clear failed");
    return SOC_OK;
}

// Raster head of the graph (renderer.cpp:965-1021): depth prepass, sun shadow, G-buffer.
void build_raster_passes(soc_renderer* r) {
    if (!r->has_scene) return;
    const int pre = SOC_PHASE_PRE_EXPOSURE;
    // DepthPrepassTask writes depth (depth_prepass.inl); here the visibility buffer it becomes
    add_pass(r, "DepthPrepass", "Depth Prepass", pre, 0, res_mask({SOC_RES_VISIBILITY}),
             [r](const soc_globals* g, hipStream_t s) {
                 const soc_img& d = r->img.depth;
                 return soc_raster_visibility(&r->scene.mesh, g->camera_projection_view_matrix, SOC_CULL_FRONT,
                                              r->scene.visibility, d.width, d.height, 1, r->scene.workspace, (soc_stream)s);
             });
    // With its own workspace the shadow draw reads nothing the main lane writes in the frame: it runs on the second lane
    // beside the depth prepass and the G-buffer (SOC_RENDERER_SHADOW_LANE=0: on the main lane, in the shared workspace).
    const bool shadow_lane = r->shadow_ws && tuning_knob("SOC_RENDERER_SHADOW_LANE", 1);
    if (r->scene.shadow)
        add_pass(r, "SunShadowDraw", "Shadows", pre, 0, res_mask({SOC_RES_SUN_SHADOW}),
                 [r, shadow_lane](const soc_globals* g, hipStream_t s) {
                     return soc_raster_depth(&r->scene.mesh, g->sun_info.projection_view_matrix, SOC_CULL_BACK, 1.25f,
                                             1.75f, r->img.shadow, shadow_lane ? r->shadow_ws : r->scene.workspace,
                                             (soc_stream)s);
                 }, shadow_lane ? SOC_PASS_ASYNC : 0);
    // GBufferGenerationTask uses (renderer.cpp:993-1005): albedo, emissive, normal, velocity, depth
    add_pass(r, "GBufferGeneration", "Rendering G-Buffer", pre, res_mask({SOC_RES_VISIBILITY}),
             res_mask({SOC_RES_ALBEDO, SOC_RES_EMISSIVE, SOC_RES_NORMAL, SOC_RES_VELOCITY, SOC_RES_DEPTH}),
             [r](const soc_globals* g, hipStream_t s) {
                 const soc_frame_images& I = r->img;
                 return soc_gbuffer_resolve(g, &r->scene.mesh, r->scene.materials, r->scene.material_count,
                                            r->scene.visibility, I.depth, I.albedo, I.emissive, I.normal,
                                            frame_velocity(r), r->scene.workspace, (soc_stream)s);
             });
}

// Bloom passes of the graph (renderer.cpp:1024-1062); build_passes_tail adds the rest.
void build_passes(soc_renderer* r) {
    auto& I = r->img;
    const int pre = SOC_PHASE_PRE_EXPOSURE;
    const int nm = 4;
    const soc_img& bloom_dst = I.bloom_output.data ? I.bloom_output : I.emissive;
    const int dst_res = I.bloom_output.data ? SOC_RES_BLOOM_OUTPUT : SOC_RES_EMISSIVE;
    const int mip[4] = {SOC_RES_BLOOM_MIP0, SOC_RES_BLOOM_MIP1, SOC_RES_BLOOM_MIP2, SOC_RES_BLOOM_MIP3};
    const bool chain_ok = bloom_fused_applicable(I.emissive, I.bloom_mips, nm, bloom_dst);
    r->bloom_in_comp = false;
    if (chain_ok && !(r->flags & (SOC_RENDERER_EXACT_BLOOM | SOC_RENDERER_UNFUSED_BLOOM))) {
        // weighted form (bloom_w.hip): 4 launches, mip0 / mip2 only in LDS, within the RGBA16F tolerance
        static const char* names[4] = {"BloomDownsample - 0+1", "BloomDownsample - 2+3", "BloomUpsample - 3+2",
                                       "BloomUpsample - 1+0"};
        const uint64_t rd[4] = {res_mask({SOC_RES_EMISSIVE}), res_mask({mip[1]}), res_mask({mip[3]}), res_mask({mip[1]})};
        const uint64_t wr[4] = {res_mask({mip[1]}), res_mask({mip[3]}), res_mask({mip[1]}), res_mask({dst_res})};
        // SOC_RENDERER_BLOOM_IN_COMPOSITION: where the fused composition + histogram's pair path applies, the last stage
        // (mip1 -> [mip0] -> output) may run inside that launch (composition_pair<..., BL>) in a frame whose sky lane is
        // the critical path (high priority, bloom_in_comp_active): the fourth pass then records nothing and the bloom
        // output is not written. Beside a low-priority sky lane the fused kernel's 19 KiB of LDS per workgroup do not fit next to
        // the sun-visibility march's noise tables (C3: Composition 76 -> 122 us in the frame, -0.6 % fps; C4 +2.9 %,
        // profiles/r05_ab_bloom_in_composition.txt), so those frames keep the separate pass.
        soc_globals gres{};
        gres.resolution[0] = I.color.width;
        gres.resolution[1] = I.color.height;
        r->bloom_in_comp = (r->flags & SOC_RENDERER_BLOOM_IN_COMPOSITION) && !(r->flags & SOC_RENDERER_UNFUSED_HISTOGRAM) &&
                           soc::composition_pair_applicable(&gres, I.color, I.albedo, bloom_dst, I.normal, I.depth, I.clouds);
        for (int st = 1; st <= 4; ++st)
            add_pass(r, names[st - 1], "Bloom", pre, rd[st - 1], wr[st - 1], [r, st](const soc_globals* g, hipStream_t s) {
                if (st == 4 && bloom_in_comp_active(r)) return (int)SOC_OK;   // Composition computes it this frame
                const soc_img& dst = r->img.bloom_output.data ? r->img.bloom_output : r->img.emissive;
                return soc_bloom_weighted_stage(g, r->img.emissive, r->img.bloom_mips, 4, dst, st, (soc_stream)s);
            });
        return;
    }
    // renderer.cpp:1024-1042: the bit-exact per-pass chain (SOC_RENDERER_EXACT_BLOOM / _UNFUSED_BLOOM, or mips that do
    // not halve exactly)
    add_pass(r, "BloomDownsample - 0", "Bloom", pre, res_mask({SOC_RES_EMISSIVE}), res_mask({mip[0]}),
             [r](const soc_globals* g, hipStream_t s) {
                 return soc_bloom_downsample(g, r->img.emissive, r->img.bloom_mips[0], (soc_stream)s);
             });
    for (int i = 0; i < nm - 1; ++i)
        add_pass(r, "BloomDownsample - " + std::to_string(i + 1), "Bloom", pre, res_mask({mip[i]}),
                 res_mask({mip[i + 1]}), [r, i](const soc_globals* g, hipStream_t s) {
                     return soc_bloom_downsample(g, r->img.bloom_mips[i], r->img.bloom_mips[i + 1], (soc_stream)s);
                 });
    // renderer.cpp:1044-1062 (load_op CLEAR: the upsample overwrites its target, quirk Q5)
    for (int i = nm - 1; i > 0; --i)
        add_pass(r, "BloomUpsample - " + std::to_string(i), "Bloom", pre, res_mask({mip[i]}), res_mask({mip[i - 1]}),
                 [r, i](const soc_globals* g, hipStream_t s) {
                     return soc_bloom_upsample(g, r->img.bloom_mips[i], r->img.bloom_mips[i - 1], (soc_stream)s);
                 });
    add_pass(r, "BloomUpsample - 0", "Bloom", pre, res_mask({mip[0]}), res_mask({dst_res}),
             [r](const soc_globals* g, hipStream_t s) {
                 const soc_img& dst = r->img.bloom_output.data ? r->img.bloom_output : r->img.emissive;
                 return soc_bloom_upsample(g, r->img.bloom_mips[0], dst, (soc_stream)s);
             });
}

void build_passes_tail(soc_renderer* r) {
    auto& I = r->img;
    const int pre = SOC_PHASE_PRE_EXPOSURE, post = SOC_PHASE_POST_EXPOSURE;
    const int em_res = I.bloom_output.data ? SOC_RES_BLOOM_OUTPUT : SOC_RES_EMISSIVE;
    // renderer.cpp:1064-1079
    add_pass(r, "SSAOGeneration", "Ambient Occlusion", pre, res_mask({SOC_RES_DEPTH, SOC_RES_NORMAL}),
             res_mask({SOC_RES_SSAO}), [r](const soc_globals* g, hipStream_t s) {
                 return soc_ssao_generation(g, r->img.depth, r->img.normal, r->img.ssao, r->img.ssao_noise_table,
                                            (soc_stream)s);
             });
    add_pass(r, "SSAOBlur", "Ambient Occlusion", pre, res_mask({SOC_RES_SSAO}), res_mask({SOC_RES_SSAO_BLUR}),
             [r](const soc_globals* g, hipStream_t s) { return soc_ssao_blur(g, r->img.ssao, r->img.ssao_blur, (soc_stream)s); });
    // Sky split: with the fused histogram on the pair path, the clouds lane also writes and bins the colour
    // image's sky pixels (sky_compose_launch), and Composition skips them, so it does not wait for the clouds.
    const bool fused_hist = !(r->flags & SOC_RENDERER_UNFUSED_HISTOGRAM);
    const soc_img& em_img = I.bloom_output.data ? I.bloom_output : I.emissive;
    soc_globals gres{};
    gres.resolution[0] = I.color.width;
    gres.resolution[1] = I.color.height;
    r->sky_split = fused_hist && !(r->flags & SOC_RENDERER_NO_SKY_SPLIT) &&
                   soc::composition_pair_applicable(&gres, I.color, I.albedo, em_img, I.normal, I.depth, I.clouds);
    const uint64_t sky_w = r->sky_split ? res_mask({SOC_RES_SKY_COLOR, SOC_RES_SKY_HISTOGRAM_PARTIALS}) : 0;
    const uint64_t parts = res_mask({SOC_RES_HISTOGRAM_PARTIALS}) | (r->sky_split ? res_mask({SOC_RES_SKY_HISTOGRAM_PARTIALS}) : 0);
    // renderer.cpp:1094-1101. Under the sky split the second lane then writes and bins the colour's sky pixels
    // (SkyCompose, composition.inl:220-222): a pass of its own, so CloudRendering itself has no cross-lane ring edge
    // (it writes only CLOUDS) and, with SOC_RENDERER_STATIC_INPUTS, may start before the fork.
    add_pass(r, "CloudRendering", "Sky Rendering", pre, res_mask({SOC_RES_DEPTH, SOC_RES_NOISE}), res_mask({SOC_RES_CLOUDS}),
             [r](const soc_globals* g, hipStream_t s) {
                 // a sky lane at high priority (the lane probe found the frame sky-bound): the density grid at twice
                 // the resident set (C4 +2.7 %, C3 -0.8 %: profiles/r05_ab_clouds_density_mult.txt) and the hoisted
                 // classification (C4 +1.8 %, C3 -1.1 %); else the knobs
                 // (also during the lane probe's high-priority windows, so the probe compares the two alternatives
                 // as they run: high with these variants against low without)
                 const bool sky_bound = sky_lane_high(r) && tuning_knob("SOC_RENDERER_SKY_BOUND_VARIANTS", 1);
                 return soc::cloud_rendering_launch(g, r->img.depth, r->img.noise, r->img.clouds, r->img.clouds_workspace,
                                                    (soc_stream)s, sky_bound);
             }, SOC_PASS_ASYNC);
    if (r->sky_split)
        add_pass(r, "SkyCompose", "Sky Rendering", pre, res_mask({SOC_RES_CLOUDS, SOC_RES_DEPTH}), sky_w,
                 [r](const soc_globals* g, hipStream_t s) {
                     return soc::sky_compose_launch(g, r->img.color, r->img.depth, r->img.clouds, r->hist_scratch,
                                                    (soc_stream)s);
                 }, SOC_PASS_ASYNC);
    // renderer.cpp:1103-1117 (composition uses) and 1155-1162 (histogram): one launch by default (the colour
    // is binned as it is written), two with SOC_RENDERER_UNFUSED_HISTOGRAM (measured in composition.hip)
    const uint64_t comp_reads = res_mask({SOC_RES_ALBEDO, em_res, SOC_RES_NORMAL, SOC_RES_DEPTH, SOC_RES_SSAO_BLUR,
                                          SOC_RES_SUN_SHADOW}) | (r->bloom_in_comp ? res_mask({SOC_RES_BLOOM_MIP1}) : 0) |
                                (r->sky_split ? 0 : res_mask({SOC_RES_CLOUDS}));
    if (fused_hist) {
        add_pass(r, "Composition+GenerateLuminanceHistogram", "Composition", pre, comp_reads,
                 res_mask({SOC_RES_COLOR, SOC_RES_HISTOGRAM_PARTIALS}), [r](const soc_globals* g, hipStream_t s) {
                     const auto& I = r->img;
                     const soc_img& em = I.bloom_output.data ? I.bloom_output : I.emissive;
                     return soc::composition_luminance_histogram(g, I.d_globals, I.color, I.albedo, em, I.normal, I.depth,
                                                                 I.ssao_blur, I.shadow, I.clouds, I.auto_exposure,
                                                                 r->hist_scratch, false, (soc_stream)s,
                                                                 r->sky_split_active,
                                                                 bloom_in_comp_active(r) ? &I.bloom_mips[1] : nullptr);
                 });
        // the 8 partial histograms of the fused launch into the AutoExposure bins. Before a multi-GPU exchange
        // (PRE and POST in separate calls) the fold must precede it; in a one-call frame the resolve folds them
        // itself and this pass has no work (it is then neither launched nor timed).
        auto& fold = add_pass(r, "LuminanceHistogramFold", "Auto Exposure", pre, parts,
                              res_mask({SOC_RES_AUTO_EXPOSURE}) | parts,
                              [r](const soc_globals* g, hipStream_t s) {
                                  (void)g;
                                  return soc::histogram_fold_launch(r->hist_scratch, r->img.auto_exposure, (soc_stream)s);
                              });
        fold.skip = [r] { return r->fold_in_resolve; };
    } else {
        add_pass(r, "Composition", "Composition", pre, comp_reads, res_mask({SOC_RES_COLOR}),
                 [r](const soc_globals* g, hipStream_t s) {
                     const auto& I = r->img;
                     const soc_img& em = I.bloom_output.data ? I.bloom_output : I.emissive;
                     return soc_composition(g, I.d_globals, I.color, I.albedo, em, I.normal, I.depth, I.ssao_blur,
                                            I.shadow, I.clouds, (soc_stream)s);
                 });
        add_pass(r, "GenerateLuminanceHistogram", "Auto Exposure", pre, res_mask({SOC_RES_COLOR}),
                 res_mask({SOC_RES_AUTO_EXPOSURE}), [r](const soc_globals* g, hipStream_t s) {
                     return soc_generate_luminance_histogram(g, r->img.color, r->img.auto_exposure, (soc_stream)s);
                 });
    }
    // renderer.cpp:1164-1168
    add_pass(r, "ResolveLuminanceHistogram", "Auto Exposure", post, res_mask({SOC_RES_AUTO_EXPOSURE}) | parts,
             res_mask({SOC_RES_AUTO_EXPOSURE}) | parts, [r](const soc_globals* g, hipStream_t s) {
                 return soc::resolve_luminance_histogram(g, r->img.auto_exposure, r->total_pixels, r->wide,
                                                         r->fold_in_resolve ? r->hist_scratch : nullptr, (soc_stream)s);
             });
    // renderer.cpp:1170-1198: TAA + both history copies (ping-pong + fused velocity history; with
    // SOC_RENDERER_VELOCITY_SLOTS the velocity is already in its history slot: no copy), and
    // renderer.cpp:1210-1217: tone mapping, fused into the TAA launch for an RGBA8 (UNORM or SRGB) framebuffer
    const bool vslots = r->flags & SOC_RENDERER_VELOCITY_SLOTS;
    const uint64_t taa_reads = res_mask({SOC_RES_COLOR, SOC_RES_PREVIOUS_COLOR, SOC_RES_VELOCITY,
                                         SOC_RES_PREVIOUS_VELOCITY, SOC_RES_DEPTH}) |
                               (r->sky_split ? res_mask({SOC_RES_SKY_COLOR}) : 0);
    const uint64_t taa_writes = vslots ? res_mask({SOC_RES_RESOLVED}) : res_mask({SOC_RES_RESOLVED, SOC_RES_PREVIOUS_VELOCITY});
    const bool fuse_tm = !(r->flags & SOC_RENDERER_UNFUSED_TONEMAP) &&
                         (I.output.format == SOC_FMT_RGBA8_UNORM || I.output.format == SOC_FMT_RGBA8_SRGB);
    if (fuse_tm) {
        add_pass(r, "TemporalAntiAliasing+ToneMapping", "Temporal Anti-Aliasing", post,
                 taa_reads | res_mask({SOC_RES_AUTO_EXPOSURE}), taa_writes | res_mask({SOC_RES_OUTPUT}),
                 [r](const soc_globals* g, hipStream_t s) {
                     const auto& I = r->img;
                     const int p = r->hist, q = 1 - r->hist;
                     const bool slots = r->flags & SOC_RENDERER_VELOCITY_SLOTS;
                     return soc_temporal_antialiasing_tone_mapping(g, I.history_color[q], I.color, I.history_color[p],
                                                                   frame_velocity(r), I.history_velocity[p], I.depth,
                                                                   slots ? soc_img{} : I.history_velocity[q],
                                                                   I.auto_exposure, I.output, (soc_stream)s);
                 });
    } else {
        add_pass(r, "TemporalAntiAliasing", "Temporal Anti-Aliasing", post, taa_reads, taa_writes,
                 [r](const soc_globals* g, hipStream_t s) {
                     const auto& I = r->img;
                     const int p = r->hist, q = 1 - r->hist;
                     const bool slots = r->flags & SOC_RENDERER_VELOCITY_SLOTS;
                     return soc_temporal_antialiasing(g, I.history_color[q], I.color, I.history_color[p],
                                                      frame_velocity(r), I.history_velocity[p], I.depth,
                                                      slots ? soc_img{} : I.history_velocity[q], (soc_stream)s);
                 });
        add_pass(r, "ToneMapping", "Tone Mapping", post, res_mask({SOC_RES_RESOLVED, SOC_RES_AUTO_EXPOSURE}),
                 res_mask({SOC_RES_OUTPUT}), [r](const soc_globals* g, hipStream_t s) {
                     const auto& I = r->img;
                     return soc_tone_mapping(g, I.history_color[1 - r->hist], I.auto_exposure, I.output, (soc_stream)s);
                 });
    }
}

// The frame as a caller pass sees it: history slot 0 = PREVIOUS, 1 = RESOLVED of this frame.
soc_frame_images callback_view(const soc_renderer* r) {
    soc_frame_images v = r->img;
    const int p = r->hist, q = 1 - r->hist;
    v.history_color[0] = r->img.history_color[p];
    v.history_color[1] = r->img.history_color[q];
    v.history_velocity[0] = r->img.history_velocity[p];
    v.history_velocity[1] = r->img.history_velocity[q];
    v.velocity = frame_velocity(r);
    return v;
}

uint64_t desc_mask(const int32_t* ids, int32_t n) {
    uint64_t m = 0;
    for (int i = 0; i < n; ++i) m |= 1ull << ids[i];
    return m;
}

// Under the sky split COLOR is the non-sky pixels and SKY_COLOR the sky pixels of the same image (and the partial
// histograms have a sky copy): a caller pass declaring COLOR (or the partials) gets both, so it is ordered against
// the second lane's sky writes too.
uint64_t widen_sky(const soc_renderer* r, uint64_t m) {
    if (!r->sky_split) return m;
    if (m & (1ull << SOC_RES_COLOR)) m |= 1ull << SOC_RES_SKY_COLOR;
    if (m & (1ull << SOC_RES_HISTOGRAM_PARTIALS)) m |= 1ull << SOC_RES_SKY_HISTOGRAM_PARTIALS;
    return m;
}

// Insert the caller passes: before their anchor, or at the end of their phase. Returns an error for an
// unknown or cross-phase anchor.
int insert_user_passes(soc_renderer* r) {
    for (auto& up : r->user_passes) {
        soc_renderer::Pass p;
        p.name = up.name;
        p.group = up.group;
        p.phase = up.desc.phase;
        p.reads = widen_velocity(r, widen_sky(r, desc_mask(up.desc.reads, up.desc.read_count)));
        p.writes = widen_velocity(r, widen_sky(r, desc_mask(up.desc.writes, up.desc.write_count)));
        p.flags = up.desc.flags;
        const soc_pass_callback fn = up.fn;
        void* user = up.user;
        p.run = [r, fn, user](const soc_globals* g, hipStream_t s) {
            const soc_frame_images v = callback_view(r);
            const int32_t rc = fn(user, g, &v, (soc_stream)s);
            return rc ? set_error(rc, "caller pass failed with %d", (int)rc) : (int)SOC_OK;
        };
        size_t at = r->passes.size();
        if (!up.before.empty()) {
            at = r->passes.size() + 1;
            for (size_t i = 0; i < r->passes.size(); ++i)
                if (r->passes[i].name == up.before) { at = i; break; }
            if (at > r->passes.size())
                return set_error(SOC_E_INVALID_ARG, "soc_renderer_add_pass: no pass named \"%s\"", up.before.c_str());
            if (r->passes[at].phase != p.phase)
                return set_error(SOC_E_INVALID_ARG, "soc_renderer_add_pass: \"%s\" is in another phase", up.before.c_str());
        } else {
            for (size_t i = 0; i < r->passes.size(); ++i)
                if (r->passes[i].phase > p.phase) { at = i; break; }
        }
        r->passes.insert(r->passes.begin() + (long)at, std::move(p));
    }
    return SOC_OK;
}

// Dependencies from the declared uses: for every resource a pass reads, the latest earlier writer (RAW);
// for every resource it writes, the latest earlier writer (WAW) and the readers since then (WAR).
//
// Cross-frame (ring) edges: the graph runs frame after frame, so the pass list is a ring. For a resource that no
// earlier pass of its own frame writes, the walk goes on into the PREVIOUS frame, from the last pass back to the
// pass itself: the latest writer there (RAW / WAW) and, for a write, the readers since that writer (WAR). The TAA
// history pair swaps each frame (ping-pong: this frame's PREVIOUS_COLOR is the last frame's RESOLVED), so in the
// previous frame the walk looks at the swapped resource. Example: GBufferGeneration writes DEPTH, which the
// previous frame's CloudRendering (second lane) still reads: a WAR ring edge across the lanes.
int prev_frame_resource(int b) {
    if (b == SOC_RES_PREVIOUS_COLOR) return SOC_RES_RESOLVED;
    if (b == SOC_RES_RESOLVED) return SOC_RES_PREVIOUS_COLOR;
    return b;
}

void derive_dependencies(soc_renderer* r) {
    const int n = (int)r->passes.size();
    for (int i = 0; i < n; ++i) {
        auto& p = r->passes[i];
        p.deps.clear();
        p.carry.clear();
        std::vector<char> dep(n, 0), carry(n, 0);
        for (int b = 0; b < SOC_RES_COUNT; ++b) {
            const uint64_t bit = 1ull << b;
            if (!((p.reads | p.writes) & bit)) continue;
            bool writer = false;
            for (int j = i - 1; j >= 0 && !writer; --j) {
                const auto& q = r->passes[j];
                if (q.writes & bit) { dep[j] = 1; writer = true; }       // RAW / WAW: the latest writer
                else if ((p.writes & bit) && (q.reads & bit)) dep[j] = 1; // WAR: readers since that writer
            }
            if (writer) continue;
            const uint64_t pbit = 1ull << prev_frame_resource(b);
            for (int j = n - 1; j >= i; --j) {                           // the previous frame, back to pass i itself
                const auto& q = r->passes[j];
                if (q.writes & pbit) { carry[j] = 1; break; }
                if ((p.writes & bit) && (q.reads & pbit)) carry[j] = 1;
            }
        }
        for (int j = 0; j < n; ++j) {
            if (dep[j]) p.deps.push_back(j);
            if (carry[j]) p.carry.push_back(j);
        }
    }
}

void destroy_pass_events(soc_renderer* r) {
    for (auto& p : r->passes) {
        for (auto e : p.ev0) (void)hipEventDestroy(e);
        for (auto e : p.ev1) (void)hipEventDestroy(e);
        if (p.done) (void)hipEventDestroy(p.done);
    }
}

// A pass records its completion event when a pass of the other lane may wait on it: an in-frame dependency across
// the lanes, or a ring edge from a main-lane pass onto a second-lane pass (waited on only when the previous call ended
// without its join). Ring edges from second-lane passes onto main-lane passes are covered by the fork, so a main-lane
// pass whose only cross-lane dependents are such edges records nothing (an event record costs its queue a marker).
void derive_signals(soc_renderer* r) {
    const int n = (int)r->passes.size();
    for (auto& p : r->passes) p.signal = false;
    for (int i = 0; i < n; ++i) {
        const bool li = (r->passes[i].flags & SOC_PASS_ASYNC) != 0;
        for (int j : r->passes[i].deps)
            if (((r->passes[j].flags & SOC_PASS_ASYNC) != 0) != li) r->passes[j].signal = true;
        if (!li)
            for (int j : r->passes[i].carry)
                if ((r->passes[j].flags & SOC_PASS_ASYNC) != 0) r->passes[j].signal = true;
    }
}

int build_graph(soc_renderer* r) {
    r->inputs_ordered = false;
    destroy_pass_events(r);
    r->passes.clear();
    build_raster_passes(r);
    build_passes(r);
    build_passes_tail(r);
    int rc = insert_user_passes(r);
    derive_dependencies(r);
    derive_signals(r);
    return rc;
}
}  // namespace

extern "C" soc_renderer* soc_renderer_create(const soc_frame_images* images, uint32_t flags) {
    if (!images) {
        set_error(SOC_E_INVALID_ARG, "soc_renderer_create: null images");
        return nullptr;
    }
    if (!images->auto_exposure) {
        set_error(SOC_E_INVALID_ARG, "soc_renderer_create: auto_exposure buffer required");
        return nullptr;
    }
    if ((flags & SOC_RENDERER_VELOCITY_SLOTS) &&
        (!images->history_velocity[0].data || !images->history_velocity[1].data ||
         images->history_velocity[0].data == images->history_velocity[1].data)) {
        set_error(SOC_E_INVALID_ARG, "soc_renderer_create: SOC_RENDERER_VELOCITY_SLOTS needs two distinct history_velocity images");
        return nullptr;
    }
    soc_renderer* r = new soc_renderer();
    r->img = *images;
    r->flags = flags;
    r->async = !(flags & SOC_RENDERER_SERIAL);
    (void)build_graph(r);
    if ((flags & SOC_RENDERER_TIMING) && soc_renderer_set_pass_timing(r, -1, 1) != SOC_OK) {
        soc_renderer_destroy(r);
        return nullptr;
    }
    return r;
}

static void destroy_side_lane(soc_renderer* r);

extern "C" void soc_renderer_destroy(soc_renderer* r) {
    if (!r) return;
    destroy_pass_events(r);
    for (auto& e : r->staging_ev)
        if (e) (void)hipEventDestroy(e);
    if (r->staging) (void)hipHostFree(r->staging);
    destroy_side_lane(r);
    if (r->hist_scratch) (void)hipFree(r->hist_scratch);
    if (r->shadow_ws) (void)hipFree(r->shadow_ws);
    delete r;
}

static int upload_lights(soc_renderer* r, const soc_globals* g, hipStream_t s) {
    if (!r->img.d_globals) return set_error(SOC_E_INVALID_ARG, "soc_renderer_execute: lights need frame d_globals");
    if (!r->staging) {
        if (hipHostMalloc((void**)&r->staging, 4 * sizeof(soc_globals), 0) != hipSuccess)
            return set_error(SOC_E_HIP, "soc_renderer_execute: hipHostMalloc failed");
        for (auto& e : r->staging_ev)
            if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess)
                return set_error(SOC_E_HIP, "soc_renderer_execute: hipEventCreate failed");
    }
    const int slot = r->staging_slot;
    r->staging_slot = (slot + 1) & 3;
    (void)hipEventSynchronize(r->staging_ev[slot]);  // slot's previous copy has landed
    std::memcpy(&r->staging[slot], g, sizeof(soc_globals));
    hipError_t e = hipMemcpyAsync(r->img.d_globals, &r->staging[slot], sizeof(soc_globals), hipMemcpyHostToDevice, s);
    if (e != hipSuccess) return set_error(SOC_E_HIP, "soc_renderer_execute: globals upload: %s", hipGetErrorString(e));
    (void)hipEventRecord(r->staging_ev[slot], s);
    return SOC_OK;
}

// Flags of the renderer's cross-lane synchronisation events (a pass's `done`, the lane switch): they order CloudRendering /
// SkyCompose writes before the Composition / TAA reads on another hardware queue of a multi-XCD device, so they keep the
// default system-scope release (the L2 writeback an event record implies) (round 5 had made them fence-free
// for a gain within noise). SOC_RENDERER_EVENT_FENCE=1 drops the fence (hipEventDisableSystemFence), a measurement knob
// only. Timing events keep the default too: without the fence a start event's timestamp may be taken after the next kernel
// has begun (6.5 us into SSAO, tools/event_trace_check.py).
static unsigned device_event_flags() {
    return (unsigned)hipEventDisableTiming |
           (tuning_knob("SOC_RENDERER_EVENT_FENCE", 0) == 1 ? (unsigned)hipEventDisableSystemFence : 0u);
}

static int run_pass(soc_renderer::Pass& p, const soc_globals* g, hipStream_t s) {
    const int slot = p.next;
    if (p.timed) (void)hipEventRecord(p.ev0[slot], s);
    int rc = p.run(g, s);
    if (rc) return rc;
    if (p.timed) {
        (void)hipEventRecord(p.ev1[slot], s);
        p.last = slot;
        p.next = (slot + 1) % SOC_RENDERER_TIMING_RING;
        if (p.count < SOC_RENDERER_TIMING_RING) p.count++;
    }
    return SOC_OK;
}

// The second lane's stream(s) and events (all of them: a device change rebuilds the lane there).
static void destroy_side_lane(soc_renderer* r) {
    for (hipEvent_t* e : {&r->fork_ev, &r->join_ev, &r->switch_ev})
        if (*e) { (void)hipEventDestroy(*e); *e = nullptr; }
    for (auto& e : r->probe_ev)
        if (e) { (void)hipEventDestroy(e); e = nullptr; }
    if (r->lane_q[0] || r->lane_q[1]) {
        for (auto& q : r->lane_q)
            if (q) { (void)hipStreamDestroy(q); q = nullptr; }
    } else if (r->side) {
        (void)hipStreamDestroy(r->side);
    }
    r->side = nullptr;
    r->side_queue = -1;
    r->probe_frames = 0;
}

// HIP maps streams onto at most GPU_MAX_HW_QUEUES (4) hardware queues per priority, reusing the least-used queue once
// the pool is full. With RCCL's and torch's streams created first (a process group), a normal-priority second lane was
// given the caller's queue and the two lanes ran serialised (bench --exchange 0.79 vs 0.62 ms per frame, DESIGN.md §11
// r5.8). A stream of another priority comes from a pool of its own, so the lane keeps a queue of its own whatever the
// caller created. Which priority is faster depends on which lane is the frame's critical path (C3: the main lane, the
// sky lane low; C4 / C2: the sky lane, high is 3-10 % faster than low). The flags fix it (round 6: one queue per
// configuration, so a command runs the same kernels every time): low by default, SOC_RENDERER_SKY_LANE_HIGH high,
// SOC_RENDERER_SKY_LANE_PROBE the round-5 timed probe (frame_lane_probe: both timed over the first 273 frames). Tuning
// knob SOC_RENDERER_SIDE_QUEUE overrides (1 = high, 2 = low, 3 = probe, 0 = normal priority).
static int ensure_side_lane(soc_renderer* r) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return set_error(SOC_E_HIP, "soc_renderer_execute: hipGetDevice failed");
    if (r->side && r->side_device == dev) return SOC_OK;
    if (r->side) {   // the caller moved to another device: rebuild the lane (and its events) there
        destroy_side_lane(r);
        for (auto& p : r->passes)
            if (p.done) { (void)hipEventDestroy(p.done); p.done = nullptr; p.done_recorded = false; }
    }
    // the lane's queue is fixed by the flags (deterministic: the same kernels every run): low priority by
    // default, high with SOC_RENDERER_SKY_LANE_HIGH, the timed probe only with SOC_RENDERER_SKY_LANE_PROBE
    const int sq_flags = (r->flags & SOC_RENDERER_SKY_LANE_HIGH) ? 1 : (r->flags & SOC_RENDERER_SKY_LANE_PROBE) ? 3 : 2;
    int sq = tuning_knob("SOC_RENDERER_SIDE_QUEUE", sq_flags);
    int least = 0, greatest = 0;
    if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess || least == greatest) sq = 0;
    hipError_t se = hipSuccess;
    if (sq == 3) {
        se = hipStreamCreateWithPriority(&r->lane_q[0], hipStreamNonBlocking, greatest);
        if (se == hipSuccess) se = hipStreamCreateWithPriority(&r->lane_q[1], hipStreamNonBlocking, least);
        if (se == hipSuccess) se = hipEventCreateWithFlags(&r->switch_ev, device_event_flags());
        for (auto& e : r->probe_ev)
            if (se == hipSuccess) se = hipEventCreate(&e);
        r->side = r->lane_q[0];
        r->side_queue = -1;
        r->probe_frames = 0;
    } else if (const int cus = tuning_knob("SOC_RENDERER_SKY_CUS", 0); cus > 0 && cus < 32) {
        // measurement knob: the sky lane on a CU-masked queue of its own, `cus` of every 32 mask bits:
        // SOC_RENDERER_SKY_CU_LAYOUT 0 = bit i set when (i / 8) % 32 < cus (the driver hands mask bits to the XCDs
        // round-robin, so cus CUs of every XCD), 1 = when i % 32 < cus
        int dev_cus = 256;
        (void)hipDeviceGetAttribute(&dev_cus, hipDeviceAttributeMultiprocessorCount, dev);
        const int layout = tuning_knob("SOC_RENDERER_SKY_CU_LAYOUT", 0);
        std::vector<uint32_t> mask((size_t)(dev_cus + 31) / 32, 0u);
        for (int i = 0; i < dev_cus; ++i)
            if ((layout ? i % 32 : (i / 8) % 32) < cus) mask[(size_t)i / 32] |= 1u << (i % 32);
        se = hipExtStreamCreateWithCUMask(&r->side, (uint32_t)mask.size(), mask.data());
        r->side_queue = 0;
    } else if (sq == 1 || sq == 2) {
        se = hipStreamCreateWithPriority(&r->side, hipStreamNonBlocking, sq == 2 ? least : greatest);
        r->side_queue = sq;
    } else {
        se = hipStreamCreateWithFlags(&r->side, hipStreamNonBlocking);
        r->side_queue = 0;
    }
    if (se != hipSuccess ||
        hipEventCreateWithFlags(&r->fork_ev, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&r->join_ev, hipEventDisableTiming) != hipSuccess) {
        destroy_side_lane(r);
        return set_error(SOC_E_HIP, "soc_renderer_execute: second lane stream/event creation failed");
    }
    r->side_device = dev;
    return SOC_OK;
}

// Move the second lane to stream q: q waits for everything queued on the current lane stream, so the lane stays one
// in-order sequence (the passes' done events recorded on the old stream stay valid for waits).
static int switch_side_lane(soc_renderer* r, hipStream_t q) {
    if (q == r->side) return SOC_OK;
    if (hipEventRecord(r->switch_ev, r->side) != hipSuccess || hipStreamWaitEvent(q, r->switch_ev, 0) != hipSuccess)
        return set_error(SOC_E_HIP, "soc_renderer_execute: second lane switch failed");
    r->side = q;
    return SOC_OK;
}

// Auto mode's probe, at the start of each frame (a call with the PRE phase): after 16 frames left to the clocks, eight
// windows (32 frames at 4K, up to 128 for smaller frames: probe_window) run the sky lane at high, low, low, high, high,
// low, low, high priority; timing events on the caller's stream at each window's frame 8 and its end give its mean
// frame interval (the first 8 after a switch skipped). The ABBA order cancels a linear drift of the clocks over the probe (a plain high-then-low order read
// the warm-up as a slower high lane). High is kept only if its windows are faster by more than 2 % (C3 prefers low by
// ~1 %, C4 and C2 high by 3-10 % with the in-Composition bloom of high windows; at 1.5 % C3 took high in 2 of 6 runs,
// profiles/r05_ab_lane_probe.txt),
// once the last event has completed (queried, never waited on), for the renderer's life.
// Frames per probe window: 32 at 3840x2160 and above, more for smaller frames (their intervals are shorter, so a
// 32-frame window is within the timing noise), up to 128.
static int probe_window(const soc_renderer* r) {
    const long long px = (long long)r->img.color.width * r->img.color.height;
    if (px <= 0) return 32;
    return (int)std::min<long long>(128, std::max<long long>(32, 32LL * 8294400LL / px));
}
constexpr int kProbeStart = 16, kProbeWins = 8;
static int probe_end(const soc_renderer* r) { return kProbeStart + kProbeWins * probe_window(r); }

static int frame_lane_probe(soc_renderer* r, hipStream_t s) {
    if (r->side_queue != -1 || !r->lane_q[0]) return SOC_OK;
    const int kStart = kProbeStart, kWindow = probe_window(r), kSkip = 8, kEnd = probe_end(r);
    constexpr int kWins = kProbeWins;
    constexpr bool kHigh[kWins] = {true, false, false, true, true, false, false, true};
    const int f = r->probe_frames;
    if (f <= kEnd) {
        if (f >= kStart) {
            const int w = (f - kStart) / kWindow, o = (f - kStart) % kWindow;
            int slot = -1;
            if (o == kSkip && w < kWins) slot = 2 * w;
            else if (o == 0 && w > 0) slot = 2 * (w - 1) + 1;
            if (slot >= 0 && hipEventRecord(r->probe_ev[slot], s) != hipSuccess)
                return set_error(SOC_E_HIP, "soc_renderer_execute: lane probe event failed");
            if (o == 0 && w < kWins) {
                int rc = switch_side_lane(r, r->lane_q[kHigh[w] ? 0 : 1]);
                if (rc) return rc;
            }
        }
        r->probe_frames++;
        return SOC_OK;
    }
    if (hipEventQuery(r->probe_ev[2 * kWins - 1]) != hipSuccess) {   // not reached yet (or an error: the lane stays)
        (void)hipGetLastError();
        return SOC_OK;
    }
    float hi = 0.0f, lo = 0.0f;
    for (int w = 0; w < kWins; ++w) {
        float t = 0.0f;
        if (hipEventElapsedTime(&t, r->probe_ev[2 * w], r->probe_ev[2 * w + 1]) != hipSuccess) {
            (void)hipGetLastError();
            r->side_queue = 2;
            return switch_side_lane(r, r->lane_q[1]);
        }
        (kHigh[w] ? hi : lo) += t;
    }
    r->side_queue = (hi < 0.98f * lo) ? 1 : 2;
    return switch_side_lane(r, r->lane_q[r->side_queue - 1]);
}

// Lane of pass i with the second lane on or off: 0 = the caller's stream, 1 = the renderer's second lane.
static int static_lane(const soc_renderer* r, int i) {
    return (r->async && (r->passes[i].flags & SOC_PASS_ASYNC)) ? 1 : 0;
}

// An aborted frame (a pass or a caller pass returned an error after the fork): join the second lane so nothing of
// this call is left unordered against the caller's next work, and drop the frame's partial histograms (the resolve
// that would clear them did not run) so they are not counted into the next frame's exposure. The TAA history is
// not flipped: the next frame reads the last completed frame's history.
static int abort_frame(soc_renderer* r, hipStream_t s, bool forked, int rc) {
    if (forked && r->side && hipEventRecord(r->join_ev, r->side) == hipSuccess &&
        hipStreamWaitEvent(s, r->join_ev, 0) == hipSuccess)
        r->main_after_side = true;
    else if (forked)
        r->main_after_side = false;
    if (r->hist_scratch) (void)hipMemsetAsync(r->hist_scratch, 0, SOC_HISTOGRAM_SCRATCH_WORDS * sizeof(uint32_t), s);
    if (r->img.auto_exposure)
        (void)hipMemsetAsync(r->img.auto_exposure->histogram_buckets, 0, sizeof(r->img.auto_exposure->histogram_buckets), s);
    return rc;
}

extern "C" int soc_renderer_execute(soc_renderer* r, const soc_globals* g, int32_t phase, soc_stream stream) {
    if (!r || !g) return set_error(SOC_E_INVALID_ARG, "soc_renderer_execute: null argument");
    hipStream_t s = hs(stream);
    r->fold_in_resolve = (phase & SOC_PHASE_ALL) == SOC_PHASE_ALL && !(r->flags & SOC_RENDERER_UNFUSED_HISTOGRAM);
    if (phase & SOC_PHASE_PRE_EXPOSURE) {
        const soc_img& em = r->img.bloom_output.data ? r->img.bloom_output : r->img.emissive;
        const bool pair_ok = soc::composition_pair_applicable(g, r->img.color, r->img.albedo, em, r->img.normal,
                                                             r->img.depth, r->img.clouds);
        r->sky_split_active = r->sky_split && pair_ok;
        r->bloom_in_comp_ok = pair_ok;
        // the graph was derived with Composition independent of the clouds: it cannot fall back to reading them
        if (r->sky_split && !r->sky_split_active)
            return set_error(SOC_E_SHAPE, "soc_renderer_execute: globals resolution %dx%d differs from the frame images %dx%d",
                             g->resolution[0], g->resolution[1], r->img.color.width, r->img.color.height);
        if (!(r->flags & SOC_RENDERER_UNFUSED_HISTOGRAM)) {   // the fused histogram's partial copies, cleared on `s`
            int rc = ensure_hist_scratch(r, s);
            if (rc) return rc;
        }
    }
    if ((phase & SOC_PHASE_PRE_EXPOSURE) && (g->point_light_count || g->spot_light_count)) {
        int rc = upload_lights(r, g, s);
        if (rc) return rc;
    }
    const int n = (int)r->passes.size();
    // lane of every pass run by this call (-1: not run)
    std::vector<int> lane(n, -1);
    bool lanes = false;
    for (int i = 0; i < n; ++i) {
        const auto& p = r->passes[i];
        if (!(p.phase & phase) || (p.skip && p.skip())) continue;
        lane[i] = static_lane(r, i);
        lanes |= lane[i] == 1;
    }
    // dependencies among the passes run by this call; a skipped pass (no work this call) hands its own
    // dependencies on to its dependents
    std::vector<std::vector<int>> deps(n);
    for (int i = 0; i < n; ++i) {
        const auto& p = r->passes[i];
        if (lane[i] < 0 && !(p.phase & phase)) continue;
        for (int j : p.deps) {
            if (lane[j] >= 0) deps[i].push_back(j);
            else if (r->passes[j].phase & phase) deps[i].insert(deps[i].end(), deps[j].begin(), deps[j].end());
        }
    }
    // Edges whose source is not run by this call, onto the other lane: the ring edges to the previous frame
    // (pass.carry) and this frame's edges to a pass of another phase's call (PRE -> POST of a multi-GPU frame).
    // Each waits on the source's latest `done` event; on the same lane stream order covers them.
    std::vector<std::vector<int>> ext(n);
    for (int i = 0; i < n; ++i) {
        if (lane[i] < 0) continue;
        const auto& p = r->passes[i];
        for (int j : p.carry)
            if (static_lane(r, j) != lane[i]) ext[i].push_back(j);
        for (int j : p.deps)
            if (lane[j] < 0 && !(r->passes[j].phase & phase) && static_lane(r, j) != lane[i]) ext[i].push_back(j);
    }
    // The fork orders the second lane after everything the caller queued on `stream` before this call: the frame
    // inputs it wrote (e.g. the depth image), and the previous frame's main-lane passes that second-lane passes have
    // ring edges on (SkyCompose after TAA and the resolve). With SOC_RENDERER_STATIC_INPUTS the caller does not rewrite
    // the frame inputs between frames, so second-lane passes without such a ring edge (CloudRendering, which writes
    // only CLOUDS) run before the fork: the second lane starts the frame's clouds as soon as the previous frame's
    // second-lane work is done, overlapping the previous frame's composition and TAA.
    bool forked_wait = false;
    if (lanes) {
        int rc = ensure_side_lane(r);
        if (!rc && (phase & SOC_PHASE_PRE_EXPOSURE)) rc = frame_lane_probe(r, s);
        if (rc) return rc;
        if (hipEventRecord(r->fork_ev, s) != hipSuccess)
            return set_error(SOC_E_HIP, "soc_renderer_execute: second lane fork failed");
    }
    // issue order (tuning knob SOC_RENDERER_SSAO_FIRST): the AO passes move within the main lane, ahead of passes they do
    // not depend on (same passes, same per-pass results). Default (-1): just before the last bloom pass, so SSAO's
    // 1024-lane workgroups start once the small bloom mips are done and overlap the sky lane's density / sun-visibility
    // kernels with the full-resolution upsample after them (C3 1370-1380 -> 1446-1451 fps, C2 +6 %, C4 +1 % against
    // AO first). 1: AO first; 0: registration order (AO after every bloom pass); k >= 2: after
    // k - 1 other passes.
    std::vector<int> order(n);
    for (int i = 0; i < n; ++i) order[i] = i;
    const int ao_pos = tuning_knob("SOC_RENDERER_SSAO_FIRST", -1);
    if (ao_pos) {
        std::vector<int> ao, rest;
        for (int i = 0; i < n; ++i) (r->passes[i].group == "Ambient Occlusion" ? ao : rest).push_back(i);
        bool free = !ao.empty();   // the AO passes may move only if none depends on an earlier non-AO pass
        for (int a : ao)
            for (int j : deps[a])
                if (r->passes[j].group != "Ambient Occlusion") free = false;
        if (free) {
            size_t at = 0;
            if (ao_pos >= 2) at = std::min(rest.size(), (size_t)(ao_pos - 1));
            if (ao_pos < 0)
                for (size_t k = 0; k < rest.size(); ++k)
                    if (r->passes[rest[k]].group == "Bloom") at = k;   // the last bloom pass
            order.assign(rest.begin(), rest.begin() + at);
            order.insert(order.end(), ao.begin(), ao.end());
            order.insert(order.end(), rest.begin() + at, rest.end());
        }
    }
    std::vector<char> needs_fork(n, 0);
    bool pre_fork = true;
    for (int oi = 0; oi < n; ++oi) {
        const int i = order[oi];
        if (lane[i] != 1) continue;
        bool carry_main = false;
        for (int j : r->passes[i].carry) carry_main |= static_lane(r, j) == 0;
        if (!(r->flags & SOC_RENDERER_STATIC_INPUTS) || !r->inputs_ordered || carry_main) pre_fork = false;
        needs_fork[i] = !pre_fork;
    }
    // Each lane is one in-order stream, so a wait on the other lane's pass at position k (in this call's issue order on
    // that lane) also covers every earlier pass of it: waits already covered are not issued again (each costs the
    // waiting queue a barrier packet, ~10 us of idle measured between dependent kernels).
    std::vector<int> pos(n, -1);
    int next_pos[2] = {0, 0}, waited[2] = {-1, -1};
    for (int oi = 0; oi < n; ++oi) {
        const int i = order[oi];
        if (lane[i] < 0) continue;
        auto& p = r->passes[i];
        const int L = lane[i];
        hipStream_t ls = L ? r->side : s;
        if (L == 1 && needs_fork[i] && !forked_wait) {
            if (hipStreamWaitEvent(r->side, r->fork_ev, 0) != hipSuccess)
                return abort_frame(r, s, lanes, set_error(SOC_E_HIP, "soc_renderer_execute: second lane fork failed"));
            forked_wait = true;
        }
        for (int j : deps[i])
            if (lane[j] != L && pos[j] > waited[L]) {
                if (hipStreamWaitEvent(ls, r->passes[j].done, 0) != hipSuccess)
                    return abort_frame(r, s, lanes, set_error(SOC_E_HIP, "soc_renderer_execute: %s: cross-lane wait failed", p.name.c_str()));
                waited[L] = pos[j];
            }
        // ring edges and edges into another phase's call: sources of an earlier call. The second lane is ordered after
        // them by this call's fork; the caller's stream by the end of that earlier call (its join, or a main-lane wait
        // on the second lane's last pass), so a wait is issued only if that call ended without either.
        for (int j : ext[i])
            if (L == 0 && !r->main_after_side && r->passes[j].done_recorded &&
                hipStreamWaitEvent(ls, r->passes[j].done, 0) != hipSuccess)
                return abort_frame(r, s, lanes, set_error(SOC_E_HIP, "soc_renderer_execute: %s: ring-edge wait failed", p.name.c_str()));
        // SOC_RENDERER_PROBE_SKIP_PASS=<pass name>: profiling only (wrong results), that pass launches nothing; bounds
        // what removing it (e.g. by fusing it into a neighbour) could gain in the frame
        static const char* probe_skip = getenv("SOC_RENDERER_PROBE_SKIP_PASS");
        int rc = (probe_skip && p.name == probe_skip) ? (int)SOC_OK : run_pass(p, g, ls);
        if (rc) return abort_frame(r, s, lanes, rc);
        pos[i] = next_pos[L]++;
        if (p.signal) {
            if (!p.done && hipEventCreateWithFlags(&p.done, device_event_flags()) != hipSuccess)
                return abort_frame(r, s, lanes, set_error(SOC_E_HIP, "soc_renderer_execute: hipEventCreate failed"));
            if (hipEventRecord(p.done, ls) != hipSuccess)
                return abort_frame(r, s, lanes, set_error(SOC_E_HIP, "soc_renderer_execute: %s: event record failed", p.name.c_str()));
            p.done_recorded = true;
        }
    }
    // join (the caller's edge): everything of this call is ordered before whatever the caller queues next on `stream`.
    // Not issued when a main-lane pass already waited on the second lane's last pass.
    const bool side_joined = waited[0] >= next_pos[1] - 1;
    if (lanes && !side_joined &&
        (hipEventRecord(r->join_ev, r->side) != hipSuccess || hipStreamWaitEvent(s, r->join_ev, 0) != hipSuccess))
        return abort_frame(r, s, lanes, set_error(SOC_E_HIP, "soc_renderer_execute: second lane join failed"));
    r->main_after_side = true;
    r->inputs_ordered = true;
    if (phase & SOC_PHASE_POST_EXPOSURE) r->hist = 1 - r->hist;   // ping-pong the TAA history
    return SOC_OK;
}

// The sun shadow draw's own workspace (SOC_RENDERER_SHADOW_LANE). Tuning knob SOC_TEST_FAIL_SHADOW_WS=1 injects the
// allocation failure for the tests (a real hipMalloc that fails, so HIP's last error is set as by a true OOM).
static hipError_t shadow_ws_alloc(void** p, size_t n) {
    if (tuning_knob("SOC_TEST_FAIL_SHADOW_WS", 0)) return hipMalloc(p, (size_t)1 << 62);
    return hipMalloc(p, n);
}

extern "C" int soc_renderer_set_raster_scene(soc_renderer* r, const soc_raster_scene* scene) {
    if (!r) return set_error(SOC_E_INVALID_ARG, "soc_renderer_set_raster_scene: null renderer");
    if (scene) {
        if (!scene->materials || scene->material_count <= 0 || !scene->visibility || !scene->workspace ||
            !scene->mesh.positions || !scene->mesh.normals || !scene->mesh.uvs || !scene->mesh.indices)
            return set_error(SOC_E_INVALID_ARG, "soc_renderer_set_raster_scene: incomplete scene");
        if (scene->shadow && !r->img.shadow.data)
            return set_error(SOC_E_INVALID_ARG, "soc_renderer_set_raster_scene: shadow pass needs images.shadow");
    }
    if (scene && scene->shadow) {
        const size_t need = soc_raster_workspace_size(scene->mesh.vertex_count, scene->mesh.triangle_count);
        if (need > r->shadow_ws_bytes) {
            if (r->shadow_ws) (void)hipFree(r->shadow_ws);
            r->shadow_ws = nullptr;
            r->shadow_ws_bytes = 0;
            // on failure: the shared workspace; clear HIP's sticky last error so the next pass's check_launch() does
            // not report this allocation's out-of-memory as a launch failure
            if (shadow_ws_alloc(&r->shadow_ws, need) != hipSuccess) {
                r->shadow_ws = nullptr;
                (void)hipGetLastError();
            } else {
                r->shadow_ws_bytes = need;
            }
        }
    }
    r->has_scene = scene != nullptr;
    if (scene) r->scene = *scene;
    int rc = build_graph(r);
    if (rc) return rc;
    if (r->flags & SOC_RENDERER_TIMING) return soc_renderer_set_pass_timing(r, -1, 1);
    return SOC_OK;
}

extern "C" int soc_renderer_add_pass(soc_renderer* r, const soc_pass_desc* d, soc_pass_callback fn, void* user,
                                     const char* before) {
    if (!r || !d || !fn || !d->name || !d->name[0])
        return set_error(SOC_E_INVALID_ARG, "soc_renderer_add_pass: null renderer, descriptor, callback or name");
    if (d->phase != SOC_PHASE_PRE_EXPOSURE && d->phase != SOC_PHASE_POST_EXPOSURE)
        return set_error(SOC_E_INVALID_ARG, "soc_renderer_add_pass: %s: phase must be PRE or POST", d->name);
    if (d->read_count < 0 || d->read_count > SOC_PASS_MAX_USES || d->write_count < 0 || d->write_count > SOC_PASS_MAX_USES)
        return set_error(SOC_E_INVALID_ARG, "soc_renderer_add_pass: %s: at most %d reads / writes", d->name, SOC_PASS_MAX_USES);
    for (int i = 0; i < d->read_count + d->write_count; ++i) {
        const int id = i < d->read_count ? d->reads[i] : d->writes[i - d->read_count];
        if (id < 0 || id >= SOC_RES_COUNT)
            return set_error(SOC_E_INVALID_ARG, "soc_renderer_add_pass: %s: bad resource id %d", d->name, id);
    }
    for (const auto& p : r->passes)
        if (p.name == d->name) return set_error(SOC_E_INVALID_ARG, "soc_renderer_add_pass: duplicate pass name \"%s\"", d->name);
    soc_renderer::UserPass up;
    up.desc = *d;
    up.name = d->name;
    up.group = d->group ? d->group : "";
    up.before = before ? before : "";
    up.fn = fn;
    up.user = user;
    up.desc.name = nullptr;
    up.desc.group = nullptr;
    r->user_passes.push_back(up);
    int rc = build_graph(r);
    if (rc) {   // roll back
        r->user_passes.pop_back();
        (void)build_graph(r);
        return rc;
    }
    if (r->flags & SOC_RENDERER_TIMING) return soc_renderer_set_pass_timing(r, -1, 1);
    return SOC_OK;
}

extern "C" int soc_renderer_pass_uses(const soc_renderer* r, int32_t i, uint64_t* reads, uint64_t* writes) {
    if (!r || i < 0 || i >= (int32_t)r->passes.size() || !reads || !writes)
        return set_error(SOC_E_INVALID_ARG, "soc_renderer_pass_uses: bad arguments");
    *reads = r->passes[i].reads;
    *writes = r->passes[i].writes;
    return SOC_OK;
}

extern "C" int32_t soc_renderer_pass_dependencies(const soc_renderer* r, int32_t i, int32_t* out, int32_t cap) {
    if (!r || i < 0 || i >= (int32_t)r->passes.size() || cap < 0 || (cap > 0 && !out))
        return set_error(SOC_E_INVALID_ARG, "soc_renderer_pass_dependencies: bad arguments");
    const auto& d = r->passes[i].deps;
    for (int k = 0; k < (int)d.size() && k < cap; ++k) out[k] = d[k];
    return (int32_t)d.size();
}

extern "C" int32_t soc_renderer_pass_carry_dependencies(const soc_renderer* r, int32_t i, int32_t* out, int32_t cap) {
    if (!r || i < 0 || i >= (int32_t)r->passes.size() || cap < 0 || (cap > 0 && !out))
        return set_error(SOC_E_INVALID_ARG, "soc_renderer_pass_carry_dependencies: bad arguments");
    const auto& d = r->passes[i].carry;
    for (int k = 0; k < (int)d.size() && k < cap; ++k) out[k] = d[k];
    return (int32_t)d.size();
}

extern "C" int32_t soc_renderer_pass_lane(const soc_renderer* r, int32_t i) {
    if (!r || i < 0 || i >= (int32_t)r->passes.size()) return set_error(SOC_E_INVALID_ARG, "soc_renderer_pass_lane: bad index");
    return (r->passes[i].flags & SOC_PASS_ASYNC) ? 1 : 0;
}

extern "C" int soc_renderer_set_async(soc_renderer* r, int32_t enable) {
    if (!r) return set_error(SOC_E_INVALID_ARG, "soc_renderer_set_async: null renderer");
    r->async = enable != 0;
    return SOC_OK;
}

extern "C" int soc_renderer_set_exposure_pixels(soc_renderer* r, uint64_t total_pixels, int32_t wide_accumulator) {
    if (!r) return set_error(SOC_E_INVALID_ARG, "soc_renderer_set_exposure_pixels: null renderer");
    r->total_pixels = total_pixels;
    r->wide = wide_accumulator;
    return SOC_OK;
}

extern "C" int32_t soc_renderer_pass_count(const soc_renderer* r) { return r ? (int32_t)r->passes.size() : 0; }

extern "C" const char* soc_renderer_pass_name(const soc_renderer* r, int32_t i) {
    if (!r || i < 0 || i >= (int32_t)r->passes.size()) return nullptr;
    return r->passes[i].name.c_str();
}

extern "C" const char* soc_renderer_pass_group(const soc_renderer* r, int32_t i) {
    if (!r || i < 0 || i >= (int32_t)r->passes.size()) return nullptr;
    return r->passes[i].group.c_str();
}

extern "C" float soc_renderer_pass_ms(soc_renderer* r, int32_t i) {
    if (!r || i < 0 || i >= (int32_t)r->passes.size()) return -1.0f;
    auto& p = r->passes[i];
    if (!p.timed || p.last < 0) return -1.0f;
    float ms = -1.0f;
    if (hipEventElapsedTime(&ms, p.ev0[p.last], p.ev1[p.last]) != hipSuccess) return -1.0f;
    return ms;
}

// The "GPU Metric" record of the most recent frame (renderer.cpp:769-806): every timed pass's ms, summed
// into the reference's 12 groups (renderer.cpp:577-588; absent groups are 0), and their total.
extern "C" int64_t soc_renderer_metrics_json(soc_renderer* r, uint64_t frame, char* buf, size_t cap) {
    if (!r) return set_error(SOC_E_INVALID_ARG, "soc_renderer_metrics_json: null renderer");
    static const char* kGroups[12] = {"Depth Prepass", "Composition", "Tone Mapping", "Bloom", "Depth Of Field",
                                      "Shadows", "Rendering G-Buffer", "Screen Space Reflections", "Ambient Occlusion",
                                      "Auto Exposure", "Sky Rendering", "Temporal Anti-Aliasing"};
    double group_ms[12] = {0};
    double total = 0.0;
    std::string passes;
    for (int i = 0; i < (int)r->passes.size(); ++i) {
        const float ms = soc_renderer_pass_ms(r, i);
        if (ms < 0.0f) continue;
        total += ms;
        char item[160];
        std::snprintf(item, sizeof item, "%s\"%s\": %.6f", passes.empty() ? "" : ", ", r->passes[i].name.c_str(), ms);
        passes += item;
        for (int k = 0; k < 12; ++k)
            if (r->passes[i].group == kGroups[k]) group_ms[k] += ms;
    }
    std::string out = "{\"frame\": " + std::to_string(frame) + ", \"total_gpu_ms\": ";
    char num[64];
    std::snprintf(num, sizeof num, "%.6f", total);
    out += num;
    out += ", \"groups\": {";
    for (int k = 0; k < 12; ++k) {
        std::snprintf(num, sizeof num, "%s\"%s\": %.6f", k ? ", " : "", kGroups[k], group_ms[k]);
        out += num;
    }
    out += "}, \"passes\": {" + passes + "}}";
    if (buf && cap) {
        const size_t n = std::min(cap - 1, out.size());
        std::memcpy(buf, out.data(), n);
        buf[n] = 0;
    }
    return (int64_t)out.size();
}

extern "C" int soc_renderer_set_pass_timing(soc_renderer* r, int32_t index, int32_t enable) {
    if (!r) return set_error(SOC_E_INVALID_ARG, "soc_renderer_set_pass_timing: null renderer");
    const int n = (int)r->passes.size();
    if (index < -1 || index >= n) return set_error(SOC_E_INVALID_ARG, "soc_renderer_set_pass_timing: bad index %d", index);
    for (int i = (index < 0 ? 0 : index); i < (index < 0 ? n : index + 1); ++i) {
        auto& p = r->passes[i];
        if (enable && p.ev0.empty()) {
            p.ev0.assign(SOC_RENDERER_TIMING_RING, nullptr);
            p.ev1.assign(SOC_RENDERER_TIMING_RING, nullptr);
            for (int k = 0; k < SOC_RENDERER_TIMING_RING; ++k)
                if (hipEventCreate(&p.ev0[k]) != hipSuccess || hipEventCreate(&p.ev1[k]) != hipSuccess)
                    return set_error(SOC_E_HIP, "soc_renderer_set_pass_timing: hipEventCreate failed");
        }
        p.timed = enable != 0;
    }
    return SOC_OK;
}

extern "C" int soc_renderer_reset_timing(soc_renderer* r) {
    if (!r) return set_error(SOC_E_INVALID_ARG, "soc_renderer_reset_timing: null renderer");
    for (auto& p : r->passes) { p.next = 0; p.count = 0; p.last = -1; }
    return SOC_OK;
}

extern "C" int soc_renderer_pass_stats(soc_renderer* r, int32_t i, float* total_ms, int32_t* frames) {
    if (!r || i < 0 || i >= (int32_t)r->passes.size() || !total_ms || !frames)
        return set_error(SOC_E_INVALID_ARG, "soc_renderer_pass_stats: bad arguments");
    auto& p = r->passes[i];
    double sum = 0.0;
    for (int k = 0; k < p.count; ++k) {
        float ms = 0.0f;
        hipError_t e = hipEventElapsedTime(&ms, p.ev0[k], p.ev1[k]);
        if (e != hipSuccess) return set_error(SOC_E_HIP, "soc_renderer_pass_stats: %s", hipGetErrorString(e));
        sum += ms;
    }
    *total_ms = (float)sum;
    *frames = p.count;
    return SOC_OK;
}

extern "C" int32_t soc_renderer_side_queue(const soc_renderer* r) { return (r && r->side) ? r->side_queue : -1; }

extern "C" int32_t soc_renderer_side_queue_probe_frames(const soc_renderer* r) {
    if (!r || !r->async || tuning_knob("SOC_RENDERER_SIDE_QUEUE", 3) != 3) return 0;
    return probe_end(r) + 1;
}

extern "C" int32_t soc_renderer_pass_event_times(soc_renderer* r, int32_t i, void* base, float* start_ms, float* end_ms,
                                                 int32_t n) {
    if (!r || i < 0 || i >= (int32_t)r->passes.size() || !base || !start_ms || !end_ms || n < 0)
        return set_error(SOC_E_INVALID_ARG, "soc_renderer_pass_event_times: bad arguments");
    auto& p = r->passes[i];
    const int first = p.count < SOC_RENDERER_TIMING_RING ? 0 : p.next;   // the oldest recorded slot
    const int m = std::min(p.count, n);
    for (int k = 0; k < m; ++k) {
        const int slot = (first + (p.count - m) + k) % SOC_RENDERER_TIMING_RING;
        hipError_t e = hipEventElapsedTime(&start_ms[k], (hipEvent_t)base, p.ev0[slot]);
        if (e == hipSuccess) e = hipEventElapsedTime(&end_ms[k], (hipEvent_t)base, p.ev1[slot]);
        if (e != hipSuccess) return set_error(SOC_E_HIP, "soc_renderer_pass_event_times: %s", hipGetErrorString(e));
    }
    return m;
}

extern "C" int32_t soc_renderer_current_history(const soc_renderer* r) { return r ? r->hist : -1; }

// Resume from a checkpoint (SURVEY.md §5 "Checkpoint / resume"): the slot whose history_color / history_velocity hold
// the previous frame's TAA result and velocity. The images and the AutoExposure block are caller-owned and restored by
// the caller; this is the renderer's one piece of temporal state.
extern "C" int soc_renderer_set_current_history(soc_renderer* r, int32_t index) {
    if (!r) return set_error(SOC_E_INVALID_ARG, "soc_renderer_set_current_history: null renderer");
    if (index != 0 && index != 1) return set_error(SOC_E_INVALID_ARG, "soc_renderer_set_current_history: index %d", index);
    r->hist = index;
    return SOC_OK;
}
