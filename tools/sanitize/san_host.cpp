// san_host — drives the host code under AddressSanitizer + UndefinedBehaviorSanitizer (tools/sanitize/Makefile).
// No GPU call is made: the globals feed and ECS scene feed, ABI introspection, the render graph (construction,
// caller passes, derived and ring dependencies, raster head, error paths), the PNG / EXR writers, the scene
// synthesiser, and every pass of the CPU oracle on small images (odd extents included). Exit 0 when every check
// passes; a sanitizer report aborts the run (-fno-sanitize-recover).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "soc_oracle.h"
#include "soc_rt.h"

extern "C" {
int soc_scene_gbuffer(int scene_id, const soc_globals* g, int W, int H, uint16_t* albedo, uint16_t* emissive,
                      uint16_t* normal, float* depth, uint16_t* velocity);
int soc_scene_shadow(int scene_id, const soc_globals* g, int S, float* shadow);
int soc_scene_mesh_counts(int scene_id, int* vertices, int* triangles);
int soc_scene_mesh(int scene_id, const soc_globals* g, float* positions, float* normals, float* uvs, uint32_t* indices,
                   uint32_t* materials);
int soc_scene_material_count(int scene_id);
int soc_scene_material_textures(int scene_id, const soc_globals* g, int size, uint8_t* rgba, float* emissive_rgb);
int soc_scene_terrain_heightmap(int size, uint8_t* rgba);
}

namespace {
int g_fail = 0;
void expect(bool ok, const char* what) {
    if (!ok) {
        std::fprintf(stderr, "FAILED: %s (%s)\n", what, soc_last_error_string());
        ++g_fail;
    }
}

struct HostImg {
    std::vector<uint8_t> data;
    soc_img img;
    HostImg(int w, int h, int fmt, int bpp, uint8_t fill = 0) : data((size_t)w * h * bpp, fill) {
        img = soc_img{data.data(), w, h, w * bpp, fmt};
    }
};

uint32_t lcg(uint32_t& s) { return s = s * 1664525u + 1013904223u; }

void fill_rgba16f(HostImg& im, uint32_t seed, float lo, float hi) {
    uint16_t* p = reinterpret_cast<uint16_t*>(im.data.data());
    for (size_t i = 0; i < im.data.size() / 2; ++i)
        p[i] = soc_oracle_f32_to_f16(lo + (hi - lo) * (float)(lcg(seed) >> 8) / 16777216.0f);
}

int32_t count_pass(void* user, const soc_globals*, const soc_frame_images*, soc_stream) {
    ++*static_cast<int*>(user);
    return 0;
}

void globals_and_scene_feed(soc_globals& g, int W, int H) {
    expect(soc_globals_init_defaults(&g, W, H) == SOC_OK, "soc_globals_init_defaults");
    soc_camera cam{{-14.0f, 2.2f, 0.3f}, {0.0f, -0.42f, 0.0f}, 90.0f, 0.1f, 1000.0f};
    uint32_t ji = 0;
    for (int i = 0; i < 3; ++i) {
        expect(soc_globals_frame_update(&g, &cam, W, H, 0.016f, &ji) == SOC_OK, "soc_globals_frame_update");
        cam.position[0] += 0.05f;
    }
    std::vector<soc_entity> ents(SOC_MAX_POINT_LIGHTS + SOC_MAX_SPOT_LIGHTS);
    for (size_t i = 0; i < ents.size(); ++i) {
        soc_entity& e = ents[i];
        std::memset(&e, 0, sizeof e);
        e.position[0] = -10.0f + 0.1f * (float)i;
        e.position[1] = 2.0f;
        e.scale[0] = e.scale[1] = e.scale[2] = 1.0f;
        e.rotation[0] = 5.0f * (float)i;
        e.components = i < SOC_MAX_POINT_LIGHTS ? SOC_ENTITY_POINT_LIGHT : SOC_ENTITY_SPOT_LIGHT;
        e.color[0] = e.color[1] = e.color[2] = 0.8f;
        e.intensity = 2.0f;
        e.cut_off = 12.5f;
        e.outer_cut_off = 17.5f;
    }
    std::vector<float> models(ents.size() * 16), normals(ents.size() * 16);
    expect(soc_scene_update(&g, ents.data(), (int)ents.size(), models.data(), normals.data()) == SOC_OK, "soc_scene_update");
    expect(g.point_light_count == SOC_MAX_POINT_LIGHTS && g.spot_light_count == SOC_MAX_SPOT_LIGHTS, "light counts");
    ents.push_back(ents.front());   // one light too many: an error, no write past the arrays
    expect(soc_scene_update(&g, ents.data(), (int)ents.size(), nullptr, nullptr) != SOC_OK, "light overflow rejected");
    float m[16], inv[16];
    const float eye[3] = {1, 2, 3}, at[3] = {0, 0, 0}, up[3] = {0, 1, 0};
    soc_mat4_look_at_rh(m, eye, at, up);
    soc_mat4_inverse(inv, m);
    soc_mat4_perspective_rh_no(m, 1.5707964f, 16.0f / 9.0f, 0.1f, 1000.0f);
    soc_mat4_ortho_rh_no(m, -16, 16, -16, 16, -100, 100);
    soc_mat4_mul(inv, m, inv);
}

void abi_introspection() {
    static const char* types[] = {"soc_globals", "soc_img", "soc_frame_images", "soc_auto_exposure", "soc_mesh",
                                  "soc_material", "soc_pass_desc", "soc_camera", "soc_entity", "no_such_type"};
    for (const char* t : types) (void)soc_abi_sizeof(t);
    expect(soc_abi_offsetof("soc_globals", "resolution") >= 0, "offsetof");
    expect(soc_abi_offsetof("soc_globals", "no_such_field") == -1, "offsetof unknown");
    expect(soc_abi_version() == 1, "abi version");
}

void render_graph(const soc_globals& g, int W, int H) {
    // fake (never dereferenced) device pointers: graph construction makes no GPU call
    char* fake = reinterpret_cast<char*>(0x100000);
    auto im = [&](int w, int h, int fmt, int bpp) { return soc_img{fake, w, h, w * bpp, fmt}; };
    soc_frame_images fi;
    std::memset(&fi, 0, sizeof fi);
    fi.albedo = fi.emissive = fi.normal = fi.velocity = fi.color = im(W, H, SOC_FMT_RGBA16F, 8);
    fi.depth = im(W, H, SOC_FMT_D32F, 4);
    fi.shadow = im(4096, 4096, SOC_FMT_D32F, 4);
    fi.noise = im(64, 64, SOC_FMT_RGBA8_UNORM, 4);
    for (int i = 0; i < 4; ++i) fi.bloom_mips[i] = im(W >> i, H >> i, SOC_FMT_RGBA16F, 8);
    fi.ssao = fi.ssao_blur = im(W / 2, H / 2, SOC_FMT_R8_UNORM, 1);
    fi.clouds = im(W, H, SOC_FMT_RGBA8_UNORM, 4);
    for (int i = 0; i < 2; ++i) fi.history_color[i] = fi.history_velocity[i] = im(W, H, SOC_FMT_RGBA16F, 8);
    fi.output = im(W, H, SOC_FMT_RGBA8_UNORM, 4);
    fi.auto_exposure = reinterpret_cast<soc_auto_exposure*>(fake);
    fi.d_globals = reinterpret_cast<soc_globals*>(fake);
    expect(soc_renderer_create(nullptr, 0) == nullptr, "create(null) rejected");
    for (uint32_t flags : {0u, (uint32_t)SOC_RENDERER_UNFUSED_BLOOM | SOC_RENDERER_UNFUSED_TONEMAP | SOC_RENDERER_UNFUSED_HISTOGRAM,
                           (uint32_t)SOC_RENDERER_NO_SKY_SPLIT, (uint32_t)SOC_RENDERER_EXACT_BLOOM}) {
        soc_renderer* r = soc_renderer_create(&fi, flags);
        expect(r != nullptr, "soc_renderer_create");
        if (!r) continue;
        int calls = 0;
        soc_pass_desc d;
        std::memset(&d, 0, sizeof d);
        d.name = "CallerPass";
        d.group = "Ambient Occlusion";
        d.phase = SOC_PHASE_PRE_EXPOSURE;
        d.read_count = 2;
        d.reads[0] = SOC_RES_SSAO;
        d.reads[1] = SOC_RES_COLOR;
        d.write_count = 1;
        d.writes[0] = SOC_RES_USER0 + 5;
        expect(soc_renderer_add_pass(r, &d, count_pass, &calls, "SSAOBlur") == SOC_OK, "add_pass");
        expect(soc_renderer_add_pass(r, &d, count_pass, &calls, nullptr) != SOC_OK, "duplicate name rejected");
        d.name = "Other";
        expect(soc_renderer_add_pass(r, &d, count_pass, &calls, "NoSuchPass") != SOC_OK, "unknown anchor rejected");
        d.reads[0] = 64;
        expect(soc_renderer_add_pass(r, &d, count_pass, &calls, nullptr) != SOC_OK, "bad resource rejected");
        d.reads[0] = SOC_RES_SSAO;
        d.phase = SOC_PHASE_POST_EXPOSURE;
        d.flags = SOC_PASS_ASYNC;
        expect(soc_renderer_add_pass(r, &d, count_pass, &calls, nullptr) == SOC_OK, "async post pass");
        soc_raster_scene sc;
        std::memset(&sc, 0, sizeof sc);
        sc.mesh.positions = sc.mesh.normals = sc.mesh.uvs = reinterpret_cast<const float*>(fake);
        sc.mesh.indices = reinterpret_cast<const uint32_t*>(fake);
        sc.mesh.vertex_count = 3;
        sc.mesh.triangle_count = 1;
        sc.materials = reinterpret_cast<const soc_material*>(fake);
        sc.material_count = 1;
        sc.visibility = reinterpret_cast<uint64_t*>(fake);
        sc.workspace = fake;
        sc.shadow = 1;
        expect(soc_renderer_set_raster_scene(r, &sc) == SOC_OK, "set_raster_scene");
        const int n = soc_renderer_pass_count(r);
        int32_t deps[64];
        for (int i = 0; i < n; ++i) {
            uint64_t rd = 0, wr = 0;
            expect(soc_renderer_pass_name(r, i) && soc_renderer_pass_group(r, i), "name / group");
            expect(soc_renderer_pass_uses(r, i, &rd, &wr) == SOC_OK, "uses");
            expect(soc_renderer_pass_dependencies(r, i, deps, 64) >= 0, "deps");
            expect(soc_renderer_pass_carry_dependencies(r, i, deps, 64) >= 0, "carry deps");
            expect(soc_renderer_pass_dependencies(r, i, nullptr, 0) >= 0, "deps count");
            (void)soc_renderer_pass_lane(r, i);
            expect(soc_renderer_pass_ms(r, i) < 0.0f, "no timing recorded");
        }
        expect(soc_renderer_pass_dependencies(r, n, deps, 64) < 0, "out-of-range index rejected");
        char buf[4096];
        expect(soc_renderer_metrics_json(r, 0, buf, sizeof buf) > 0, "metrics json");
        expect(soc_renderer_metrics_json(r, 0, buf, 8) > 8, "metrics json truncated");
        expect(soc_renderer_set_raster_scene(r, nullptr) == SOC_OK, "clear raster scene");
        expect(soc_renderer_set_exposure_pixels(r, (uint64_t)W * H * 8, 1) == SOC_OK, "exposure pixels");
        soc_renderer_destroy(r);
    }
    (void)g;
}

void writers(int W, int H) {
    HostImg rgba(W, H, SOC_FMT_RGBA8_UNORM, 4, 200);
    HostImg half(W, H, SOC_FMT_RGBA16F, 8);
    fill_rgba16f(half, 7, -4.0f, 70000.0f);   // includes overflow to inf
    const char* dir = std::getenv("SAN_TMP") ? std::getenv("SAN_TMP") : "/tmp";
    char path[512];
    std::snprintf(path, sizeof path, "%s/san_host.png", dir);
    expect(soc_write_png(path, rgba.data.data(), W, H, W * 4) == SOC_OK, "png");
    std::snprintf(path, sizeof path, "%s/san_host.exr", dir);
    expect(soc_write_exr(path, half.data.data(), W, H, W * 8) == SOC_OK, "exr");
    expect(soc_write_png("/nonexistent-dir/x.png", rgba.data.data(), W, H, W * 4) != SOC_OK, "png bad path");
}

void oracle_frame(const soc_globals& g0, int W, int H) {
    soc_globals g = g0;
    g.resolution[0] = W;
    g.resolution[1] = H;
    HostImg albedo(W, H, SOC_FMT_RGBA16F, 8), emissive(W, H, SOC_FMT_RGBA16F, 8), normal(W, H, SOC_FMT_RGBA16F, 8),
        velocity(W, H, SOC_FMT_RGBA16F, 8), depth(W, H, SOC_FMT_D32F, 4);
    expect(soc_scene_gbuffer(0, &g, W, H, (uint16_t*)albedo.data.data(), (uint16_t*)emissive.data.data(),
                             (uint16_t*)normal.data.data(), (float*)depth.data.data(), (uint16_t*)velocity.data.data()) == 0,
           "scene gbuffer");
    const int S = 128;
    HostImg shadow(S, S, SOC_FMT_D32F, 4);
    for (size_t i = 0; i < shadow.data.size() / 4; ++i) reinterpret_cast<float*>(shadow.data.data())[i] = 1.0f;
    expect(soc_scene_shadow(0, &g, S, (float*)shadow.data.data()) == 0, "scene shadow");
    HostImg noise(64, 64, SOC_FMT_RGBA8_UNORM, 4);
    uint32_t seed = 11;
    for (auto& b : noise.data) b = (uint8_t)(lcg(seed) >> 24);
    std::vector<HostImg> mips;
    for (int i = 0; i < 4; ++i) mips.emplace_back(std::max(W >> i, 1), std::max(H >> i, 1), SOC_FMT_RGBA16F, 8);
    // bloom chain (renderer.cpp:1024-1062)
    expect(soc_oracle_bloom_downsample(&g, emissive.img, mips[0].img) == SOC_OK, "bloom down 0");
    for (int i = 0; i < 3; ++i) expect(soc_oracle_bloom_downsample(&g, mips[i].img, mips[i + 1].img) == SOC_OK, "bloom down");
    for (int i = 3; i > 0; --i) expect(soc_oracle_bloom_upsample(&g, mips[i].img, mips[i - 1].img) == SOC_OK, "bloom up");
    expect(soc_oracle_bloom_upsample(&g, mips[0].img, emissive.img) == SOC_OK, "bloom up 0");
    HostImg ssao(W / 2, H / 2, SOC_FMT_R8_UNORM, 1), blur(W / 2, H / 2, SOC_FMT_R8_UNORM, 1);
    expect(soc_oracle_ssao_generation(&g, depth.img, normal.img, ssao.img) == SOC_OK, "ssao");
    expect(soc_oracle_ssao_blur(&g, ssao.img, blur.img) == SOC_OK, "ssao blur");
    HostImg clouds(W, H, SOC_FMT_RGBA8_UNORM, 4), color(W, H, SOC_FMT_RGBA16F, 8);
    expect(soc_oracle_cloud_rendering(&g, depth.img, noise.img, clouds.img) == SOC_OK, "clouds");
    soc_globals gl = g;
    gl.point_light_count = 2;
    gl.spot_light_count = 2;
    expect(soc_oracle_composition(&gl, color.img, albedo.img, emissive.img, normal.img, depth.img, blur.img, shadow.img,
                                  clouds.img) == SOC_OK, "composition (lights)");
    expect(soc_oracle_composition(&g, color.img, albedo.img, emissive.img, normal.img, depth.img, blur.img, shadow.img,
                                  clouds.img) == SOC_OK, "composition");
    soc_auto_exposure ae;
    std::memset(&ae, 0, sizeof ae);
    expect(soc_oracle_generate_luminance_histogram(&g, color.img, &ae) == SOC_OK, "histogram");
    expect(soc_oracle_resolve_luminance_histogram(&g, &ae, 0, 0) == SOC_OK, "resolve");
    expect(soc_oracle_generate_luminance_histogram(&g, color.img, &ae) == SOC_OK, "histogram 2");
    expect(soc_oracle_resolve_luminance_histogram(&g, &ae, (uint64_t)W * H * 8, 1) == SOC_OK, "resolve wide");
    HostImg prev(W, H, SOC_FMT_RGBA16F, 8), pvel(W, H, SOC_FMT_RGBA16F, 8), resolved(W, H, SOC_FMT_RGBA16F, 8);
    fill_rgba16f(prev, 3, 0.0f, 2.0f);
    expect(soc_oracle_temporal_antialiasing(&g, resolved.img, color.img, prev.img, velocity.img, pvel.img, depth.img) == SOC_OK,
           "taa");
    for (int fmt : {SOC_FMT_RGBA8_UNORM, SOC_FMT_RGBA8_SRGB}) {
        HostImg out(W, H, fmt, 4);
        expect(soc_oracle_tone_mapping(&g, resolved.img, &ae, out.img) == SOC_OK, "tone map 8");
    }
    HostImg out16(W, H, SOC_FMT_RGBA16F, 8), out32(W, H, SOC_FMT_RGBA32F, 16);
    expect(soc_oracle_tone_mapping(&g, resolved.img, &ae, out16.img) == SOC_OK, "tone map 16f");
    expect(soc_oracle_tone_mapping(&g, resolved.img, &ae, out32.img) == SOC_OK, "tone map 32f");
    // Hi-Z (min and max pyramids) of the depth
    std::vector<HostImg> hiz;
    int hw = std::max(W / 2, 1), hh = std::max(H / 2, 1), levels = 0;
    while (levels < 6) { hiz.emplace_back(hw, hh, SOC_FMT_D32F, 4); ++levels; if (hw == 1 && hh == 1) break; hw = std::max(hw / 2, 1); hh = std::max(hh / 2, 1); }
    std::vector<soc_img> hz;
    for (auto& h : hiz) hz.push_back(h.img);
    expect(soc_oracle_generate_hiz(&g, depth.img, hz.data(), (int)hz.size(), 0) == SOC_OK, "hiz min");
    expect(soc_oracle_generate_hiz(&g, depth.img, hz.data(), (int)hz.size(), 1) == SOC_OK, "hiz max");
}

void oracle_raster(const soc_globals& g0, int W, int H) {
    soc_globals g = g0;
    int nv = 0, nt = 0;
    expect(soc_scene_mesh_counts(0, &nv, &nt) == 0, "mesh counts");
    std::vector<float> pos(3 * nv), nrm(3 * nv), uv(2 * nv);
    std::vector<uint32_t> idx(3 * nt), mat(nt);
    expect(soc_scene_mesh(0, &g, pos.data(), nrm.data(), uv.data(), idx.data(), mat.data()) == 0, "mesh");
    const int nm = soc_scene_material_count(0), T = 32;
    std::vector<uint8_t> tex((size_t)nm * T * T * 4);
    std::vector<float> em(3 * nm);
    expect(soc_scene_material_textures(0, &g, T, tex.data(), em.data()) == 0, "material textures");
    soc_mesh m;
    std::memset(&m, 0, sizeof m);
    m.positions = pos.data();
    m.normals = nrm.data();
    m.uvs = uv.data();
    m.indices = idx.data();
    m.materials = mat.data();
    m.vertex_count = nv;
    m.triangle_count = nt;
    for (int i = 0; i < 4; ++i) m.model_matrix[i * 5] = m.normal_matrix[i * 5] = 1.0f;
    std::vector<soc_material> mats(nm);
    for (int i = 0; i < nm; ++i) {
        std::memset(&mats[i], 0, sizeof mats[i]);
        mats[i].albedo = soc_img{tex.data() + (size_t)i * T * T * 4, T, T, T * 4, SOC_FMT_RGBA8_SRGB};
        for (int k = 0; k < 4; ++k) mats[i].albedo_factor[k] = 1.0f;
        for (int k = 0; k < 3; ++k) mats[i].emissive_factor[k] = em[3 * i + k];
    }
    std::vector<uint64_t> vis((size_t)W * H, ~0ull);
    expect(soc_oracle_raster_visibility(&m, g.camera_projection_view_matrix, SOC_CULL_FRONT, vis.data(), W, H) == SOC_OK,
           "raster visibility");
    HostImg sh(64, 64, SOC_FMT_D32F, 4);
    for (size_t i = 0; i < sh.data.size() / 4; ++i) reinterpret_cast<float*>(sh.data.data())[i] = 1.0f;
    expect(soc_oracle_raster_depth(&m, g.sun_info.projection_view_matrix, SOC_CULL_BACK, 1.25f, 1.75f, sh.img) == SOC_OK,
           "raster depth");
    HostImg albedo(W, H, SOC_FMT_RGBA16F, 8), emissive(W, H, SOC_FMT_RGBA16F, 8), normal(W, H, SOC_FMT_RGBA16F, 8),
        velocity(W, H, SOC_FMT_RGBA16F, 8), depth(W, H, SOC_FMT_D32F, 4);
    expect(soc_oracle_gbuffer_resolve(&g, &m, mats.data(), nm, vis.data(), depth.img, albedo.img, emissive.img, normal.img,
                                      velocity.img) == SOC_OK, "gbuffer resolve");
    // mip chain of an odd-sized sRGB texture, packed after level 0
    const int TW = 37, TH = 5;
    const size_t bytes = soc_mip_chain_bytes(TW, TH, TW * 4);
    std::vector<uint8_t> chain(bytes, 128);
    expect(soc_oracle_generate_mips(soc_img{chain.data(), TW, TH, TW * 4, SOC_FMT_RGBA8_SRGB}) == SOC_OK, "mips");
    // terrain: heightmap -> normal map, tessellation
    const int HM = 64;
    std::vector<uint8_t> hm((size_t)HM * HM * 4);
    expect(soc_scene_terrain_heightmap(HM, hm.data()) == 0, "heightmap");
    HostImg hn(HM, HM, SOC_FMT_RGBA16F, 8);
    const soc_img hmi{hm.data(), HM, HM, HM * 4, SOC_FMT_RGBA8_UNORM};
    expect(soc_oracle_height_to_normal(hmi, hn.img) == SOC_OK, "height to normal");
    const int grid = 8, level = 3, nvert = ((grid - 1) * level + 1) * ((grid - 1) * level + 1), ntri = 2 * (grid - 1) * level * (grid - 1) * level;
    std::vector<float> tp(3 * nvert), tn(3 * nvert), tu(2 * nvert);
    std::vector<uint32_t> ti(3 * ntri);
    expect(soc_oracle_terrain_tessellate(&g, hmi, grid, level, tp.data(), tn.data(), tu.data(), ti.data()) == SOC_OK,
           "terrain tessellate");
    std::vector<uint16_t> tal((size_t)W * H * 4), tem((size_t)W * H * 4), tno((size_t)W * H * 4), tve((size_t)W * H * 4);
    std::vector<float> tde((size_t)W * H);
    expect(soc_scene_gbuffer(1, &g, W, H, tal.data(), tem.data(), tno.data(), tde.data(), tve.data()) == 0, "terrain gbuffer");
}
}  // namespace

int main() {
    soc_globals g;
    for (int pass = 0; pass < 2; ++pass) {
        const int W = pass ? 97 : 128, H = pass ? 55 : 72;   // even and odd extents
        globals_and_scene_feed(g, W, H);
        abi_introspection();
        render_graph(g, W, H);
        writers(W, H);
        oracle_frame(g, W, H);
        oracle_raster(g, W, H);
    }
    for (float v : {0.0f, 1e-8f, 0.5f, 1.0f, 65504.0f, 1e9f, -3.0f, INFINITY, NAN})
        (void)soc_oracle_f16_to_f32(soc_oracle_f32_to_f16(v));
    for (float v : {0.0f, 1e-3f, 1.0f, 4096.0f, NAN, INFINITY}) (void)soc_oracle_luminance_bin(v, v, v, 12.77568f, -17.22432f);
    std::printf("san_host: %s (%d failed checks)\n", g_fail ? "FAILED" : "ok", g_fail);
    return g_fail ? 1 : 0;
}
