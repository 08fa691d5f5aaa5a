// soc_headless — a compiled C++ consumer of include/soc_rt.h (no Python, no ctypes).
//
// The caller shape SURVEY.md §8b names for the drop-in boundary: a host frame loop in the shape of
// Application::run -> Renderer::render (src/application.cpp:89-107, src/graphics/renderer.cpp:633-812) driving the
// render graph of Renderer::rebuild_task_graph (renderer.cpp:929-1235) through the C ABI, headless: the final
// framebuffer goes to a host PNG instead of a swapchain.
//
//   soc_headless W H FRAMES OUT.png [OUT.raw]
//
// 1. globals: soc_globals_init_defaults (renderer.cpp:72-133) + two soc_globals_frame_update calls (application.cpp:
//    109-165) for the Sponza-proxy camera, as tests/helpers.globals_for does;
// 2. inputs: the box atrium's G-buffer and 1024^2 sun shadow map from libsoc_scene (scene_synth.c), the clouds noise
//    fixture; every image in caller-owned device memory (hipMalloc), as the boundary requires;
// 3. soc_renderer_create + soc_renderer_add_pass: a caller pass "RawAO" between SSAOBlur and Composition that copies
//    the raw AO over the blurred one (declared reads {SSAO}, writes {SSAO_BLUR}: the Daxa uses block);
// 4. per frame: soc_renderer_execute PRE_EXPOSURE, (the multi-GPU histogram exchange would go here), POST_EXPOSURE;
// 5. soc_read_image of the framebuffer -> soc_write_png (+ the raw RGBA8 rows), the GPU-metric JSON of the last frame,
//    and one JSON summary line on stdout.
// Exit code 0 on success; any soc_* error prints soc_last_error_string() and exits 1.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "soc_rt.h"

extern "C" {   // scene_synth.c (libsoc_scene.so): the host G-buffer producer of the unit-test scene
int soc_scene_gbuffer(int scene_id, const soc_globals* g, int W, int H, uint16_t* albedo, uint16_t* emissive,
                      uint16_t* normal, float* depth, uint16_t* velocity);
int soc_scene_shadow(int scene_id, const soc_globals* g, int S, float* shadow);
}

namespace {

void die(const char* what) {
    std::fprintf(stderr, "soc_headless: %s: %s\n", what, soc_last_error_string());
    std::exit(1);
}
void check(int rc, const char* what) {
    if (rc != SOC_OK) die(what);
}
void hip_check(hipError_t e, const char* what) {
    if (e != hipSuccess) {
        std::fprintf(stderr, "soc_headless: %s: %s\n", what, hipGetErrorString(e));
        std::exit(1);
    }
}

int bpp(int fmt) {
    switch (fmt) {
    case SOC_FMT_RGBA16F: return 8;
    case SOC_FMT_D32F: return 4;
    case SOC_FMT_R8_UNORM: return 1;
    case SOC_FMT_RGBA8_UNORM: case SOC_FMT_RGBA8_SRGB: return 4;
    case SOC_FMT_RGBA32F: return 16;
    default: return 0;
    }
}

// Caller-owned device images (the boundary never allocates on the hot path).
struct DeviceImages {
    std::vector<void*> blocks;
    soc_img make(int w, int h, int fmt) {
        void* p = nullptr;
        const size_t pitch = (size_t)w * bpp(fmt);
        hip_check(hipMalloc(&p, pitch * h), "hipMalloc");
        hip_check(hipMemset(p, 0, pitch * h), "hipMemset");
        blocks.push_back(p);
        return soc_img{p, w, h, (int32_t)pitch, fmt};
    }
    void* raw(size_t n) {
        void* p = nullptr;
        hip_check(hipMalloc(&p, n), "hipMalloc");
        hip_check(hipMemset(p, 0, n), "hipMemset");
        blocks.push_back(p);
        return p;
    }
    ~DeviceImages() {
        for (void* p : blocks) (void)hipFree(p);
    }
};

void upload(const soc_img& im, const void* host) {
    hip_check(hipMemcpy2D(im.data, im.pitch_bytes, host, (size_t)im.width * bpp(im.format), (size_t)im.width * bpp(im.format),
                          im.height, hipMemcpyHostToDevice), "upload");
}

// The caller pass: the Daxa task callback (e.g. composition.inl:56-78) recording its work on the frame's stream.
struct RawAO {
    int calls = 0;
};
int32_t raw_ao(void* user, const soc_globals*, const soc_frame_images* images, soc_stream stream) {
    static_cast<RawAO*>(user)->calls++;
    return soc_copy_image(images->ssao_blur, images->ssao, stream);
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 5) {
        std::fprintf(stderr, "usage: %s W H FRAMES OUT.png [OUT.raw]\n", argv[0]);
        return 2;
    }
    const int W = std::atoi(argv[1]), H = std::atoi(argv[2]), frames = std::atoi(argv[3]);
    const char* png = argv[4];
    const char* raw_path = argc > 5 ? argv[5] : nullptr;
    if (W < 2 || H < 2 || frames < 1) {
        std::fprintf(stderr, "soc_headless: bad extent or frame count\n");
        return 2;
    }
    if (std::string(soc_device_arch()) != "gfx950") die("soc_device_arch");

    // ---- globals feed (Application::update) ----
    soc_globals g;
    check(soc_globals_init_defaults(&g, W, H), "soc_globals_init_defaults");
    soc_camera cam{{-14.0f, 2.2f, 0.3f}, {0.0f, -0.42f, 0.0f}, 90.0f, 0.1f, 1000.0f};
    uint32_t jitter = 0;
    for (int i = 0; i < 2; ++i) {
        check(soc_globals_frame_update(&g, &cam, W, H, 0.016f, &jitter), "soc_globals_frame_update");
        cam.position[0] += 0.05f;
    }

    // ---- inputs: host G-buffer + shadow map, uploaded once ----
    const size_t P = (size_t)W * H;
    std::vector<uint16_t> albedo(P * 4), emissive(P * 4), normal(P * 4), velocity(P * 4);
    std::vector<float> depth(P, 1.0f);
    if (soc_scene_gbuffer(0, &g, W, H, albedo.data(), emissive.data(), normal.data(), depth.data(), velocity.data()))
        die("soc_scene_gbuffer");
    const int S = 1024;
    std::vector<float> shadow((size_t)S * S, 1.0f);
    if (soc_scene_shadow(0, &g, S, shadow.data())) die("soc_scene_shadow");
    std::vector<uint8_t> noise(64 * 64 * 4);
    {
        const std::string exe(argv[0]);
        const std::string root = exe.substr(0, exe.rfind('/') + 1) + "../";
        FILE* f = std::fopen((root + "data/clouds_noise_64x64.u8").c_str(), "rb");
        if (!f) { std::fprintf(stderr, "soc_headless: noise fixture not found under %s\n", root.c_str()); return 1; }
        std::vector<uint8_t> grey(64 * 64);
        if (std::fread(grey.data(), 1, grey.size(), f) != grey.size()) { std::fclose(f); return 1; }
        std::fclose(f);
        for (int i = 0; i < 64 * 64; ++i) {   // assets/Clouds/noise.png loaded as R8G8B8A8_UNORM (renderer.cpp:152)
            noise[i * 4 + 0] = noise[i * 4 + 1] = noise[i * 4 + 2] = grey[i];
            noise[i * 4 + 3] = 255;
        }
    }

    DeviceImages mem;
    soc_frame_images fi;
    std::memset(&fi, 0, sizeof fi);
    fi.albedo = mem.make(W, H, SOC_FMT_RGBA16F);
    fi.emissive = mem.make(W, H, SOC_FMT_RGBA16F);
    fi.normal = mem.make(W, H, SOC_FMT_RGBA16F);
    fi.depth = mem.make(W, H, SOC_FMT_D32F);
    fi.velocity = mem.make(W, H, SOC_FMT_RGBA16F);
    fi.shadow = mem.make(S, S, SOC_FMT_D32F);
    fi.noise = mem.make(64, 64, SOC_FMT_RGBA8_UNORM);
    for (int i = 0; i < 4; ++i) fi.bloom_mips[i] = mem.make(std::max(W >> i, 1), std::max(H >> i, 1), SOC_FMT_RGBA16F);
    fi.ssao = mem.make(W / 2, H / 2, SOC_FMT_R8_UNORM);
    fi.ssao_blur = mem.make(W / 2, H / 2, SOC_FMT_R8_UNORM);
    fi.clouds = mem.make(W, H, SOC_FMT_RGBA8_UNORM);
    fi.color = mem.make(W, H, SOC_FMT_RGBA16F);
    for (int i = 0; i < 2; ++i) {
        fi.history_color[i] = mem.make(W, H, SOC_FMT_RGBA16F);
        fi.history_velocity[i] = mem.make(W, H, SOC_FMT_RGBA16F);
    }
    fi.output = mem.make(W, H, SOC_FMT_RGBA8_UNORM);
    fi.ssao_noise_table = static_cast<float*>(mem.raw((size_t)(W / 2) * (H / 2) * 2 * sizeof(float)));
    fi.auto_exposure = static_cast<soc_auto_exposure*>(mem.raw(sizeof(soc_auto_exposure)));
    fi.d_globals = static_cast<soc_globals*>(mem.raw(sizeof(soc_globals)));
    fi.clouds_workspace = mem.raw(soc_cloud_rendering_workspace_size(W, H));
    upload(fi.albedo, albedo.data());
    upload(fi.emissive, emissive.data());
    upload(fi.normal, normal.data());
    upload(fi.depth, depth.data());
    upload(fi.velocity, velocity.data());
    upload(fi.shadow, shadow.data());
    upload(fi.noise, noise.data());
    hipStream_t stream;
    hip_check(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking), "hipStreamCreate");
    check(soc_ssao_prepare_noise(fi.normal, fi.ssao, fi.ssao_noise_table, (soc_stream)stream), "soc_ssao_prepare_noise");

    // ---- the render graph + a caller pass (TaskGraph::add_task with a uses block) ----
    soc_renderer* r = soc_renderer_create(&fi, SOC_RENDERER_TIMING);
    if (!r) die("soc_renderer_create");
    RawAO state;
    soc_pass_desc d;
    std::memset(&d, 0, sizeof d);
    d.name = "RawAO";
    d.group = "Ambient Occlusion";
    d.phase = SOC_PHASE_PRE_EXPOSURE;
    d.read_count = 1;
    d.reads[0] = SOC_RES_SSAO;
    d.write_count = 1;
    d.writes[0] = SOC_RES_SSAO_BLUR;
    check(soc_renderer_add_pass(r, &d, raw_ao, &state, "Composition+GenerateLuminanceHistogram"), "soc_renderer_add_pass");

    // ---- the frame loop (Renderer::render: execute, then wait_idle) ----
    const auto t0 = std::chrono::steady_clock::now();
    for (int f = 0; f < frames; ++f) {
        check(soc_renderer_execute(r, &g, SOC_PHASE_PRE_EXPOSURE, (soc_stream)stream), "soc_renderer_execute PRE");
        // a multi-GPU caller all-reduces fi.auto_exposure->histogram_buckets here
        check(soc_renderer_execute(r, &g, SOC_PHASE_POST_EXPOSURE, (soc_stream)stream), "soc_renderer_execute POST");
        hip_check(hipStreamSynchronize(stream), "hipStreamSynchronize");
    }
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() / frames;

    // ---- headless present: the framebuffer to a host image ----
    std::vector<uint8_t> out(P * 4);
    check(soc_read_image(fi.output, out.data(), W * 4, (soc_stream)stream), "soc_read_image");
    soc_auto_exposure ae;
    hip_check(hipMemcpyAsync(&ae, fi.auto_exposure, sizeof ae, hipMemcpyDeviceToHost, stream), "exposure readback");
    hip_check(hipStreamSynchronize(stream), "hipStreamSynchronize");
    check(soc_write_png(png, out.data(), W, H, W * 4), "soc_write_png");
    if (raw_path) {
        FILE* f = std::fopen(raw_path, "wb");
        if (!f || std::fwrite(out.data(), 1, out.size(), f) != out.size()) { std::fprintf(stderr, "soc_headless: raw write failed\n"); return 1; }
        std::fclose(f);
    }
    uint64_t sum = 0;
    for (uint8_t v : out) sum = sum * 1099511628211ull + v;   // FNV-style rolling checksum of the framebuffer
    char metrics[8192];
    const int64_t mlen = soc_renderer_metrics_json(r, (uint64_t)frames - 1, metrics, sizeof metrics);
    std::printf("{\"width\": %d, \"height\": %d, \"frames\": %d, \"caller_pass_calls\": %d, \"exposure\": %.9g, "
                "\"history\": %d, \"checksum\": \"%016llx\", \"ms_per_frame_host\": %.4f, \"passes\": %d, \"metrics\": %s}\n",
                W, H, frames, state.calls, (double)ae.exposure, soc_renderer_current_history(r), (unsigned long long)sum, ms,
                soc_renderer_pass_count(r), (mlen > 0 && mlen < (int64_t)sizeof metrics) ? metrics : "null");
    soc_renderer_destroy(r);
    hip_check(hipStreamDestroy(stream), "hipStreamDestroy");
    return 0;
}
