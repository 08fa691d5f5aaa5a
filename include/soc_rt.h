/*
 * soc_rt.h — C ABI of the MI355X-native screen-space deferred-shading and post-processing
 * passes of lukasino1214/soc_real_time_renderer.
 *
 * Every entry point below replaces ONE render-graph task of the reference (a Daxa task struct whose
 * callback() records a fullscreen draw / compute dispatch). The reference file:line of the task that
 * each function replaces is cited next to it. Shader-level semantics (sampling, formats, quirks
 * Q1..Q12 of SURVEY.md §8a) are documented in DESIGN.md.
 *
 * Conventions:
 *   - The caller owns all device memory. No function allocates on the hot path, and none keeps a
 *     pointer after it returns.
 *   - Calls are stream-ordered and asynchronous on the given HIP stream; the caller synchronises.
 *   - Return value: 0 on success, < 0 on error (SOC_E_*); soc_last_error_string() gives the
 *     message of the calling thread's last error. No C++ exception crosses this ABI.
 *   - Images are pitch-linear, row-major, y = 0 is the TOP row (the reference's uv.y = 0).
 *   - `const soc_globals* g` is a HOST pointer to the per-frame globals (mirror of ShaderGlobals,
 *     src/graphics/shared.inl:47-131). Only the fields a pass reads are consumed; they are packed
 *     into the kernel arguments at call time (the reference memcpy's the whole block into a UBO
 *     ring slot, src/graphics/renderer.cpp:648-657).
 */
#ifndef SOC_RT_H
#define SOC_RT_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SOC_RT_ABI_VERSION 1

/* Error codes. */
#define SOC_OK 0
#define SOC_E_INVALID_ARG (-1)   /* null pointer, bad format, bad extent            */
#define SOC_E_SHAPE (-2)         /* image extents inconsistent with the pass        */
#define SOC_E_HIP (-3)           /* a HIP runtime call failed (launch, memcpy, ...) */
#define SOC_E_UNSUPPORTED (-4)   /* format / configuration not implemented          */

struct ihipStream_t;
typedef struct ihipStream_t* soc_stream; /* == hipStream_t; NULL = the null stream */

/* Image formats: the reference's Vulkan formats (src/graphics/renderer.cpp:348-470). */
typedef enum soc_format {
    SOC_FMT_RGBA16F = 1,     /* R16G16B16A16_SFLOAT, 8 B/px (albedo, emissive, normal, color, velocity, bloom mips) */
    SOC_FMT_D32F = 2,        /* D32_SFLOAT, 4 B/px (depth, sun shadow map)                                      */
    SOC_FMT_R8_UNORM = 3,    /* R8_UNORM, 1 B/px (ssao, ssao blur)                                              */
    SOC_FMT_RGBA8_UNORM = 4, /* R8G8B8A8_UNORM, 4 B/px (clouds, noise texture, headless swapchain)              */
    SOC_FMT_RGBA8_SRGB = 5,  /* R8G8B8A8_SRGB, 4 B/px (optional headless swapchain with sRGB encode on store)   */
    SOC_FMT_RGBA32F = 6      /* R32G32B32A32_SFLOAT, 16 B/px (debug / exact tone-map output)                     */
} soc_format;

/* A borrowed view of a 2-D image in device memory (host memory for the CPU oracle). */
typedef struct soc_img {
    void* data;
    int32_t width;
    int32_t height;
    int32_t pitch_bytes; /* bytes between rows; >= width * bytes_per_pixel(format) */
    int32_t format;      /* soc_format */
} soc_img;

/* --- Globals: POD mirror of ShaderGlobals (src/graphics/shared.inl:5-131). ----------------------
 * Matrices are glm-layout column-major float[16] (m[col*4 + row]). Daxa sampler / image ids and the
 * AutoExposure buffer pointer are not part of this struct: samplers are fixed by the pass contract
 * (DESIGN.md "Sampling contract") and images/buffers are explicit arguments. */
typedef struct soc_point_light {   /* shared.inl:5-9 */
    float position[3];
    float color[3];
    float intensity;
} soc_point_light;

typedef struct soc_spot_light {    /* shared.inl:13-20 */
    float position[3];
    float direction[3];
    float color[3];
    float intensity;
    float cut_off;
    float outer_cut_off;
} soc_spot_light;

typedef struct soc_sun_info {      /* shared.inl:24-37 */
    float projection_matrix[16];
    float view_matrix[16];
    float projection_view_matrix[16];
    float terrain_y_clip_trick[4];
    float position[3];
    float direction[3];
    float exponential_factor;
    float darkening_factor;
    float bias;
    float intensity;
} soc_sun_info;

#define SOC_MAX_POINT_LIGHTS 128
#define SOC_MAX_SPOT_LIGHTS 128
#define SOC_AUTO_EXPOSURE_BIN_COUNT 256
#define SOC_SSAO_MAX_KERNEL 26

typedef struct soc_globals {       /* shared.inl:47-131 */
    float camera_projection_matrix[16];
    float camera_inverse_projection_matrix[16];
    float camera_view_matrix[16];
    float camera_inverse_view_matrix[16];
    float camera_projection_view_matrix[16];
    float camera_inverse_projection_view_matrix[16];

    float camera_previous_projection_matrix[16];
    float camera_previous_inverse_projection_matrix[16];
    float camera_previous_view_matrix[16];
    float camera_previous_inverse_view_matrix[16];
    float camera_previous_projection_view_matrix[16];
    float camera_previous_inverse_projection_view_matrix[16];

    float jitter[2];
    float previous_jitter[2];

    float camera_position[3];
    float camera_near_clip;
    float camera_far_clip;

    int32_t resolution[2];
    float elapsed_time;
    float delta_time;
    uint32_t frame_counter;

    soc_sun_info sun_info;

    uint32_t point_light_count;
    uint32_t spot_light_count;
    soc_point_light point_lights[SOC_MAX_POINT_LIGHTS];
    soc_spot_light spot_lights[SOC_MAX_SPOT_LIGHTS];

    float terrain_offset[3];
    float terrain_scale[2];
    float terrain_height_scale;
    float terrain_midpoint;
    float terrain_delta;
    float terrain_min_depth;
    float terrain_max_depth;
    int32_t terrain_min_tess_level;
    int32_t terrain_max_tess_level;
    float terrain_y_clip_trick[4];
    float terrain_previous_y_clip_trick[4];

    float filter_radius;           /* bloom (unused by the reference shaders) */

    float ssao_bias;
    float ssao_radius;
    int32_t ssao_kernel_size;

    float ambient[3];
    float ambient_occlussion_strength;
    float emissive_bloom_strength;

    float focal_length;            /* depth of field (disabled in the reference graph) */
    float plane_in_focus;
    float aperture;

    float adjustment_speed;
    float log_min_luminance;
    float log_max_luminance;
    float target_luminance;

    float saturation;
    float agxDs_linear_section;
    float peak;
    float compression;
} soc_globals;

/* AutoExposure buffer (shared.inl:39-45), device memory, caller-owned. */
typedef struct soc_auto_exposure {
    float exposure;
    uint32_t histogram_buckets[SOC_AUTO_EXPOSURE_BIN_COUNT];
} soc_auto_exposure;

/* --- Library / ABI introspection ---------------------------------------------------------------- */
int32_t soc_abi_version(void);
size_t soc_abi_sizeof(const char* type_name);                        /* "soc_globals", "soc_img", ... */
int64_t soc_abi_offsetof(const char* type_name, const char* field);  /* -1 if unknown */
const char* soc_last_error_string(void);
/* Tuning knobs (SOC_* environment variables of the profiling variants) are read once and cached;
 * this drops the cache so the current environment applies to the next launches. */
void soc_tuning_reload(void);
const char* soc_device_arch(void);                                   /* "gfx950" the kernels were built for */
/* Launch geometry (no GPU needed): SOC_OK when a block of bx x by x bz lanes fits a kernel whose flat work-group bound
 * (__launch_bounds__) is `bound`, else SOC_E_INVALID_ARG with the reason. Every launcher in the library applies the
 * same check with its kernel's own bound before the launch, so a block over the bound is never issued (it would fail
 * on the device as an "unspecified launch failure"). */
int soc_check_block_shape(int32_t bound, int32_t bx, int32_t by, int32_t bz);

/* --- Host-side globals feed (native C++, no GPU needed) ----------------------------------------- */
/* Renderer defaults: renderer.cpp:72-133 (terrain, ssao, composition, dof, auto exposure incl. the
 * log_min/log_max re-derivation of :103-104, tone mapping, sun ortho/lookAt/dir of :109-133). */
int soc_globals_init_defaults(soc_globals* g, int32_t width, int32_t height);

/* Camera state of ControlledCamera3D (camera.hpp:105-119): position + rotation (x = yaw, y = pitch). */
typedef struct soc_camera {
    float position[3];
    float rotation[3];
    float fov_degrees;   /* Camera3D::fov  = 90  (camera.hpp:74) */
    float near_clip;     /* Camera3D::near = 0.1 */
    float far_clip;      /* Camera3D::far  = 1000 */
} soc_camera;

/* One Application::update() (application.cpp:109-165) without input: rebuilds the camera view
 * (camera.cpp:40-56) and projection (camera.cpp:6-10, Y flip), the R2 jitter (period 32, :113-127,
 * applied to proj[3][0..1], :129-131), shifts current -> previous matrices, and advances
 * delta_time / elapsed_time / frame_counter. *jitter_index is advanced like the reference's. */
int soc_globals_frame_update(soc_globals* g, const soc_camera* cam, int32_t width, int32_t height,
                             float delta_time, uint32_t* jitter_index);

/* ECS scene feed: Scene::update (src/ecs/scene.cpp:47-118). An entity carries a TransformComponent (position,
 * rotation in degrees, scale; components.hpp) and optionally a PointLightComponent or SpotLightComponent
 * (color, intensity, cut_off / outer_cut_off in degrees; defaults components.hpp:55-66). soc_scene_update
 * clears the light counts, then walks the entities in order: every transform gets model = translate(position) *
 * toMat4(quat(radians(rotation))) * scale(scale) and normal = transpose(inverse(model)) (:64-68); a point light
 * appends {position, color, intensity}; a spot light appends {position, dir = rotateZ(rotateY(rotateX((0,-1,0),
 * rx), ry), rz), color, intensity, cos(radians(cut_off)), cos(radians(outer_cut_off))} (:87-116). More than
 * SOC_MAX_POINT_LIGHTS / SOC_MAX_SPOT_LIGHTS lights (an out-of-bounds write in the reference) is an error. */
#define SOC_ENTITY_POINT_LIGHT 1
#define SOC_ENTITY_SPOT_LIGHT 2
typedef struct soc_entity {
    float position[3];
    float rotation[3];       /* degrees */
    float scale[3];
    int32_t components;      /* SOC_ENTITY_* (a transform is always present) */
    float color[3];
    float intensity;
    float cut_off, outer_cut_off;   /* degrees (spot lights) */
} soc_entity;
/* model_matrices / normal_matrices: optional outputs, count x float[16] (column-major), or NULL. */
int soc_scene_update(soc_globals* g, const soc_entity* entities, int32_t count, float* model_matrices,
                     float* normal_matrices);

/* glm restatements used by the feed (exported for tests): column-major float[16]. */
void soc_mat4_perspective_rh_no(float out[16], float fovy_radians, float aspect, float znear, float zfar);
void soc_mat4_ortho_rh_no(float out[16], float l, float r, float b, float t, float znear, float zfar);
void soc_mat4_look_at_rh(float out[16], const float eye[3], const float center[3], const float up[3]);
void soc_mat4_inverse(float out[16], const float m[16]);
void soc_mat4_mul(float out[16], const float a[16], const float b[16]);

/* --- ★ Passes (one per reference task) ---------------------------------------------------------- */

/* BloomDownsampleTask (src/graphics/tasks/bloom_downsample.inl:19-68, shader :107-141):
 * 13-tap COD:AW filter of `higher_mip` written to `lower_mip` (any size ratio; exact 1:1 and 2:1
 * fast paths). RGBA16F -> RGBA16F. */
int soc_bloom_downsample(const soc_globals* g, soc_img higher_mip, soc_img lower_mip, soc_stream stream);

/* BloomUpsampleTask (bloom_upsample.inl:19-77, shader :98-127): 9-tap tent of `lower_mip` that
 * OVERWRITES `higher_mip` (CLEAR + ONE/ONE blend == overwrite, quirk Q5). RGBA16F -> RGBA16F. */
int soc_bloom_upsample(const soc_globals* g, soc_img lower_mip, soc_img higher_mip, soc_stream stream);

/* Whole bloom chain as scheduled by renderer.cpp:1024-1062: down(emissive->mip0), down(mip i ->
 * mip i+1), up(mip i -> mip i-1), up(mip0 -> emissive). `mips` holds mip_count images (4 in the
 * reference, renderer.hpp:51). The reference's 8 passes, bit-exact. */
int soc_bloom_chain(const soc_globals* g, soc_img emissive, const soc_img* mips, int32_t mip_count,
                    soc_stream stream);

/* The bloom chain in weighted form (bloom_w.hip): at the chain's fixed ratios every tap of the sampling
 * contract has exact weights on clamp-to-edge texels, so each pass is evaluated as one fixed weighted
 * sum of RGBA16F texels with fp32 FMAs (same weights, different rounding order: within the RGBA16F
 * tolerance, not bit-exact). Stages: 1 emissive -> [mip0] -> mips[1], 2 mips[1] -> [mip2] -> mips[3],
 * 3 mips[3] -> [mip2] -> mips[1], 4 mips[1] -> [mip0] -> output; 0 = all four. mips[0] and mips[2] are
 * scratch (never written: their final contents are unobservable in the reference graph). Needs 4 mips halving
 * exactly from the emissive extent (<= 8192); output may be `emissive` (in place, as the reference) but not mips[1]. */
int soc_bloom_weighted_stage(const soc_globals* g, soc_img emissive, const soc_img* mips, int32_t mip_count, soc_img output,
                             int32_t stage, soc_stream stream);

/* SSAOGenerationTask (ssao_generation.inl:20-68, shader :176-214): half-res R8 ambient occlusion from
 * full-res depth (D32F) and normal (RGBA16F). `target` is (W/2)x(H/2) R8_UNORM. `noise_table` is an
 * optional device workspace of (target.w * target.h * 2) floats holding the per-pixel random vector
 * of :184-188 (a pure function of uv and the normal-image size, filled by
 * soc_ssao_prepare_noise); pass NULL to evaluate it inline. */
int soc_ssao_prepare_noise(soc_img normal, soc_img target, float* noise_table, soc_stream stream);
int soc_ssao_generation(const soc_globals* g, soc_img depth, soc_img normal, soc_img target,
                        const float* noise_table, soc_stream stream);

/* SSAOBlurTask (ssao_blur.inl:19-70, shader :91-106): 4x4 box, offsets -2..+1. R8 -> R8. */
int soc_ssao_blur(const soc_globals* g, soc_img ssao, soc_img target, soc_stream stream);

/* CloudRenderingTask (cloud_rendering.inl:27-54, shader :441-481): atmosphere + volumetric clouds on
 * sky pixels (depth == 1), constant (0.2,0.4,1.0) elsewhere. `noise` is the 64x64 RGBA8 or R8
 * noise texture (assets/Clouds/noise.png, REPEAT). target: RGBA8_UNORM full-res (quirk Q6).
 * `workspace` (optional, soc_cloud_rendering_workspace_size(target.width, target.height) bytes of
 * device memory) enables the compacted path: sky pixels are listed, and the cloud march is split at
 * its dense steps into (pixel, step) pairs so the sun-visibility marches are spread evenly over the
 * lanes; the result is bit-identical to the workspace-free single kernel. */
size_t soc_cloud_rendering_workspace_size(int32_t width, int32_t height);
int soc_cloud_rendering(const soc_globals* g, soc_img depth, soc_img noise, soc_img target, void* workspace,
                        soc_stream stream);

/* CompositionTask (composition.inl:29-79, shader :162-225): deferred lighting with the sun ESM
 * shadow, point/spot lights, ambient * AO^strength, emissive * strength, clouds on sky pixels.
 * `d_globals` is a DEVICE copy of *g (soc_upload_globals) and is only read when the frame has
 * point or spot lights (it may be NULL otherwise). Writes RGBA16F `target`. */
int soc_composition(const soc_globals* g, const soc_globals* d_globals, soc_img target, soc_img albedo,
                    soc_img emissive, soc_img normal, soc_img depth, soc_img ssao, soc_img shadow,
                    soc_img clouds, soc_stream stream);

/* CompositionTask followed by GenerateLuminanceHistogramTask (renderer.cpp:1103-1168) in one launch
 * when the composition pair path applies at g->resolution: the bins of the stored RGBA16F pixels are
 * accumulated while they are written (bit-identical bins, no re-read of `target`). Otherwise the two
 * passes run back to back. The bins are ADDED to ae->histogram_buckets, as the histogram pass does.
 * `scratch`: device, SOC_HISTOGRAM_SCRATCH_WORDS u32, zero-filled by the caller once; every call leaves
 * it zeroed again (8 partial histograms, folded into the bins by a second small launch). */
#define SOC_HISTOGRAM_SCRATCH_WORDS 2048
int soc_composition_luminance_histogram(const soc_globals* g, const soc_globals* d_globals, soc_img target,
                                        soc_img albedo, soc_img emissive, soc_img normal, soc_img depth,
                                        soc_img ssao, soc_img shadow, soc_img clouds, soc_auto_exposure* d_auto_exposure,
                                        uint32_t* scratch, soc_stream stream);

/* GenerateLuminanceHistogramTask (generate_luminance_histogram.inl:23-47, shader :59-78): adds the
 * frame's 256-bin log-luminance histogram into d_auto_exposure->histogram_buckets. */
int soc_generate_luminance_histogram(const soc_globals* g, soc_img hdr, soc_auto_exposure* d_auto_exposure,
                                     soc_stream stream);

/* ResolveLuminanceHistogramTask (resolve_luminance_histogram.inl:20-43, shader :56-80): weighted mean
 * of the bins -> exposure (exponential adaptation), then clears the bins.
 * total_pixels == 0 -> resolution.x*resolution.y (reference). wide_accumulator != 0 -> 64-bit
 * weighted sum (multi-GPU all-reduced bins); 0 -> reference u32 wrap semantics. */
int soc_resolve_luminance_histogram(const soc_globals* g, soc_auto_exposure* d_auto_exposure,
                                    uint64_t total_pixels, int32_t wide_accumulator, soc_stream stream);

/* TemporalAntiAliasingTask (temporal_antialiasing.inl:54-116, shader :137-190). Writes RGBA16F
 * `target`. If `velocity_history_out` has data != NULL, the kernel also writes a copy of
 * current_velocity into it (fused CopyImageTask of renderer.cpp:1191-1198); it must not alias
 * previous_velocity. */
int soc_temporal_antialiasing(const soc_globals* g, soc_img target, soc_img current_color,
                              soc_img previous_color, soc_img current_velocity, soc_img previous_velocity,
                              soc_img depth, soc_img velocity_history_out, soc_stream stream);

/* TemporalAntiAliasingTask followed by ToneMappingTask (renderer.cpp:1170-1217) in one launch when
 * `output` is RGBA8_UNORM at the target extent and the TAA pair path applies: the resolved RGBA16F
 * pixels are tone-mapped as stored (same AgX device code as soc_tone_mapping), saving the re-read of
 * `target`. Otherwise the two passes run back to back. Results equal soc_temporal_antialiasing +
 * soc_tone_mapping. */
int soc_temporal_antialiasing_tone_mapping(const soc_globals* g, soc_img target, soc_img current_color,
                                           soc_img previous_color, soc_img current_velocity,
                                           soc_img previous_velocity, soc_img depth, soc_img velocity_history_out,
                                           const soc_auto_exposure* d_auto_exposure, soc_img output,
                                           soc_stream stream);

/* CopyImageTask (temporal_antialiasing.inl:16-37): same-format, same-extent image copy. */
int soc_copy_image(soc_img target, soc_img source, soc_stream stream);

/* ToneMappingTask (tone_mapping.inl:20-70, shader :145-176): AgX-DS with exposure from
 * d_auto_exposure->exposure. target: RGBA8_UNORM / RGBA8_SRGB / RGBA16F / RGBA32F. */
int soc_tone_mapping(const soc_globals* g, soc_img color, const soc_auto_exposure* d_auto_exposure,
                     soc_img target, soc_stream stream);

/* Device copy of the globals block (the reference's per-frame UBO upload, renderer.cpp:648-657). */
int soc_upload_globals(const soc_globals* g, soc_globals* d_globals, soc_stream stream);

/* --- Render graph (host C++ mirror of Renderer::rebuild_task_graph, renderer.cpp:929-1235) ------ */

/* Frame images. The caller allocates them (device memory) and keeps them alive. */
typedef struct soc_frame_images {
    soc_img albedo, emissive, normal, depth, velocity;  /* G-buffer (produced upstream) */
    soc_img shadow;                                     /* sun shadow map, D32F 4096^2 */
    soc_img noise;                                      /* clouds noise 64^2 */
    soc_img bloom_mips[4];                              /* RGBA16F W,W/2,W/4,W/8 */
    soc_img ssao, ssao_blur;                            /* R8 (W/2)x(H/2) */
    soc_img clouds;                                     /* RGBA8 WxH */
    soc_img color;                                      /* RGBA16F composition output */
    soc_img history_color[2];                           /* RGBA16F TAA resolved / previous (ping-pong) */
    soc_img history_velocity[2];                        /* RGBA16F previous velocity (ping-pong) */
    soc_img output;                                     /* tone-mapped framebuffer (RGBA8) */
    float* ssao_noise_table;                            /* optional (ssao.w*ssao.h*2 floats) or NULL */
    soc_auto_exposure* auto_exposure;                   /* device */
    soc_globals* d_globals;                             /* device copy of the globals */
    /* Optional target of the last bloom upsample, read by composition as "emissive". data == NULL:
     * bloom overwrites `emissive` in place, as the reference graph does (renderer.cpp:1055-1062). */
    soc_img bloom_output;
    void* clouds_workspace;                             /* optional, soc_cloud_rendering_workspace_size */
} soc_frame_images;

typedef struct soc_renderer soc_renderer;

/* Phases of one frame. The luminance all-reduce of a multi-GPU run sits between PRE and POST. */
#define SOC_PHASE_PRE_EXPOSURE 1   /* bloom, ssao, blur, clouds, composition, histogram */
#define SOC_PHASE_POST_EXPOSURE 2  /* resolve, taa (+ fused velocity history), tone mapping */
#define SOC_PHASE_ALL 3

/* flags */
#define SOC_RENDERER_TIMING 1      /* record hipEvents around every pass (GPUMetric, gpu_metric.cpp:18-42) */
#define SOC_RENDERER_UNFUSED_BLOOM 2  /* bloom as the reference's 8 bit-exact passes (as EXACT_BLOOM) */
#define SOC_RENDERER_SERIAL 4      /* every pass on the caller's stream (no concurrent sky lane) */
#define SOC_RENDERER_UNFUSED_TONEMAP 8  /* TAA and tone mapping as two passes (default: one launch for RGBA8) */
#define SOC_RENDERER_FUSED_HISTOGRAM 16  /* composition + luminance histogram in one launch (the default; kept
                                            for callers that set it) */
#define SOC_RENDERER_EXACT_BLOOM 32       /* bit-exact 8-pass bloom chain instead of the weighted form (bloom_w.hip) */
#define SOC_RENDERER_UNFUSED_HISTOGRAM 64 /* composition and luminance histogram as two passes */
#define SOC_RENDERER_NO_SKY_SPLIT 128     /* Composition writes the sky pixels itself (waits for the clouds) */
/* The caller does not rewrite the frame's input images (G-buffer, shadow map, noise) between frames, e.g. a resident
 * G-buffer, or one produced in the graph by the raster head. Second-lane passes whose only cross-frame dependencies are
 * on the second lane (CloudRendering: it writes only CLOUDS) may then start before the fork, i.e. before the caller's
 * stream reaches this frame: the clouds of frame N+1 overlap the composition / TAA of frame N. Same results. The
 * second lane's intermediate CLOUDS image may then already hold the next frame's clouds when work the caller queued
 * between two calls reads it: a caller that reads CLOUDS between frames leaves the flag off. */
#define SOC_RENDERER_STATIC_INPUTS 256
/* Velocity history by slot rotation instead of a copy. The reference copies the velocity image into
 * previous_velocity after TAA every frame (CopyImageTask, renderer.cpp:1185-1189; without this flag the TAA launch
 * writes that copy into the history_velocity slot it resolves into). With the flag, the frame's velocity image IS that
 * slot: the velocity producer (GBufferGeneration of the raster head, or the caller) writes frame N's velocity into
 * history_velocity[1 - soc_renderer_current_history(r)] (read before executing frame N), TAA reads it there and frame
 * N + 1 reads it as its previous velocity, so no copy is made. images.velocity is then unused; caller passes receive the
 * slot as `images->velocity`, and VELOCITY / PREVIOUS_VELOCITY declared by a pass count as uses of both slots. Same
 * results as the copy for the same velocity fields. */
#define SOC_RENDERER_VELOCITY_SLOTS 512
/* The bloom chain's last stage (upsample 1 + 0: mip1 -> [mip0] -> bloom output, renderer.cpp:1044-1062) may be computed
 * inside the fused Composition + histogram launch, per 32 x 16 tile in LDS, from BLOOM_MIP1 (the same values per pixel,
 * rounded to RGBA16F as the chain stores them, so the same colour bits). The renderer does so in frames whose sky lane
 * is the critical path (a high-priority sky lane: soc_renderer_side_queue() == 1, and the lane probe's high-priority
 * windows); the chain's fourth pass then records nothing and the
 * full-resolution bloom output (images.bloom_output, or the emissive image in place) is NOT written. Composition
 * declares BLOOM_MIP1 besides the bloom output. Applies with the weighted chain and the fused histogram's pair path. A
 * caller that reads the bloom output leaves the flag off. */
#define SOC_RENDERER_BLOOM_IN_COMPOSITION 1024
/* The sky lane's hardware queue (soc_renderer_side_queue): a low-priority stream by default (frames whose main lane is
 * the critical path, e.g. the Sponza frames at 4K); SOC_RENDERER_SKY_LANE_HIGH a high-priority stream (sky-bound frames:
 * the terrain / 1080p frames), which also selects the sky-bound variants (BLOOM_IN_COMPOSITION, the clouds' density grid
 * at twice the resident set, hoisted classification); SOC_RENDERER_SKY_LANE_PROBE times both over the first frames and
 * keeps the faster (round 5's default; the choice can then differ between runs). Same results in every case. */
#define SOC_RENDERER_SKY_LANE_HIGH 2048
#define SOC_RENDERER_SKY_LANE_PROBE 4096

soc_renderer* soc_renderer_create(const soc_frame_images* images, uint32_t flags);
void soc_renderer_destroy(soc_renderer* r);
int soc_renderer_execute(soc_renderer* r, const soc_globals* g, int32_t phase, soc_stream stream);
/* Histogram normalisation for a multi-GPU resolve: total pixels over all ranks (0 = this frame). */
int soc_renderer_set_exposure_pixels(soc_renderer* r, uint64_t total_pixels, int32_t wide_accumulator);
int32_t soc_renderer_pass_count(const soc_renderer* r);
const char* soc_renderer_pass_name(const soc_renderer* r, int32_t index);
const char* soc_renderer_pass_group(const soc_renderer* r, int32_t index);   /* renderer.cpp:558-588 names */
/* Milliseconds of pass `index` in the most recent executed frame (needs timing enabled for the pass
 * and a completed stream); < 0 if unavailable. */
float soc_renderer_pass_ms(soc_renderer* r, int32_t index);
/* Per-pass timing control: hipEvents bracket a timed pass on the launch stream every frame, kept in
 * a ring of SOC_RENDERER_TIMING_RING frames. index -1 = every pass. Event creation happens here, not
 * in soc_renderer_execute. */
#define SOC_RENDERER_TIMING_RING 256
int soc_renderer_set_pass_timing(soc_renderer* r, int32_t index, int32_t enable);
int soc_renderer_reset_timing(soc_renderer* r);
/* Sum of the pass's durations (ms) over the frames recorded since the last reset (at most the last
 * SOC_RENDERER_TIMING_RING) and their count. Needs a completed stream. */
int soc_renderer_pass_stats(soc_renderer* r, int32_t index, float* total_ms, int32_t* frames);
/* The recorded frames' start / end event times of the pass (ms after the caller's hipEvent `base`, recorded on the same
 * device before them), oldest first; at most n entries; returns the count written or < 0. Needs a completed stream.
 * For checking the pass events against a kernel trace of the same run (tools/event_trace_check.py). */
int32_t soc_renderer_pass_event_times(soc_renderer* r, int32_t index, void* base, float* start_ms, float* end_ms,
                                      int32_t n);
/* Index (0/1) of the history_color slot holding this frame's TAA result (= tone-map input). */
int32_t soc_renderer_current_history(const soc_renderer* r);
/* Restore that index when resuming from a checkpoint of the temporal state (SURVEY.md §5 "Checkpoint / resume"; the
 * reference keeps it only in its TAA history images and AutoExposure, renderer.cpp:1170-1198): the caller writes back
 * history_color[index] / history_velocity[index] and the AutoExposure block, then sets the index. 0 or 1. */
int soc_renderer_set_current_history(soc_renderer* r, int32_t index);
/* Sky lane on/off (default on unless SOC_RENDERER_SERIAL). On: CloudRendering runs on a renderer-owned
 * stream of the current device, forked from `stream` at the start of the PRE phase and joined before
 * Composition, so it overlaps bloom and SSAO. Results are identical either way. */
int soc_renderer_set_async(soc_renderer* r, int32_t enable);
/* The sky lane's hardware queue: 1 = a high-priority stream, 2 = low priority, 0 = normal priority (a queue HIP may
 * share with the caller's stream), -1 = not chosen yet (SOC_RENDERER_SKY_LANE_PROBE: after 16 frames, eight windows of
 * 32-128 frames alternate high / low priority as ABBA pairs; high is kept if it is faster by more than 2 % once their
 * timing events have completed, else low) or no sky lane created. Same results either way. */
int32_t soc_renderer_side_queue(const soc_renderer* r);
/* Frames the auto probe spans from the renderer's first call (the choice is made at the first call after they have
 * completed on the GPU); 0 when no probe runs. A caller that times frames runs at least this many first. */
int32_t soc_renderer_side_queue_probe_frames(const soc_renderer* r);

/* --- Pass declaration (the Daxa task-uses block + TaskGraph::add_task, e.g. composition.inl:10-21 and
 * renderer.cpp:1103-1117) ------------------------------------------------------------------------
 * Every pass of the graph, built-in or added, declares the frame resources it reads and writes. The graph
 * keeps the registration order (the reference executes tasks in add_task order) and derives from the
 * declared uses what Daxa derives barriers from: each pass's dependencies (read-after-write,
 * write-after-read, write-after-write on the latest earlier user of a resource) and the placement of
 * SOC_PASS_ASYNC passes on the renderer's second lane: such a pass waits only for the passes it depends
 * on, and a later pass on the caller's stream waits for it only if it depends on it. */
enum soc_resource {
    SOC_RES_ALBEDO = 0, SOC_RES_EMISSIVE, SOC_RES_NORMAL, SOC_RES_DEPTH, SOC_RES_VELOCITY,
    SOC_RES_SUN_SHADOW, SOC_RES_NOISE,
    SOC_RES_BLOOM_MIP0, SOC_RES_BLOOM_MIP1, SOC_RES_BLOOM_MIP2, SOC_RES_BLOOM_MIP3,
    SOC_RES_BLOOM_OUTPUT,        /* images.bloom_output (aliases EMISSIVE when that image is absent) */
    SOC_RES_SSAO, SOC_RES_SSAO_BLUR, SOC_RES_CLOUDS, SOC_RES_COLOR,
    SOC_RES_PREVIOUS_COLOR, SOC_RES_RESOLVED,          /* TAA history pair, renderer.cpp:1170-1198 */
    SOC_RES_PREVIOUS_VELOCITY,
    SOC_RES_AUTO_EXPOSURE,       /* AutoExposure buffer (histogram bins + exposure) */
    SOC_RES_OUTPUT,              /* tone-mapped framebuffer (the reference's swapchain image) */
    SOC_RES_VISIBILITY,          /* raster visibility buffer (raster head) */
    SOC_RES_HISTOGRAM_PARTIALS,  /* the fused composition + histogram pass's partial bins */
    SOC_RES_SKY_COLOR,           /* the colour image's sky pixels, when the second lane writes them (see below) */
    SOC_RES_SKY_HISTOGRAM_PARTIALS,  /* their partial bins */
    SOC_RES_USER0 = 32,          /* SOC_RES_USER0 .. SOC_RES_USER0 + 31: caller-defined resources */
    SOC_RES_COUNT = 64
};
#define SOC_PASS_MAX_USES 16
#define SOC_PASS_ASYNC 1          /* may run on the second lane (the reference's unused async-compute queue) */
typedef struct soc_pass_desc {
    const char* name;             /* task name, unique in the graph */
    const char* group;            /* GPU-metric group (renderer.cpp:577-588) or any label */
    int32_t phase;                /* SOC_PHASE_PRE_EXPOSURE or SOC_PHASE_POST_EXPOSURE */
    uint32_t flags;               /* SOC_PASS_ASYNC */
    int32_t read_count, write_count;
    int32_t reads[SOC_PASS_MAX_USES];    /* enum soc_resource */
    int32_t writes[SOC_PASS_MAX_USES];
} soc_pass_desc;
/* Sky split (the default with the fused histogram and the pair path): Composition's sky pixels (depth == 1 ->
 * the clouds texel, composition.inl:220-222) are written and binned on the second lane right after
 * CloudRendering, so Composition does not wait for the clouds. COLOR is then the non-sky pixels and SKY_COLOR the
 * sky pixels of the same image: a caller pass that needs the whole colour image declares both.
 * SOC_RENDERER_NO_SKY_SPLIT turns it off (same bits either way). */
/* The callback of a caller pass: record its work on `stream`, return 0 (or a negative code, which aborts the
 * frame with that code). `images` is the renderer's frame, with history_color[0] / history_velocity[0] the
 * PREVIOUS and [1] the RESOLVED slots of this frame. */
typedef int32_t (*soc_pass_callback)(void* user, const soc_globals* g, const soc_frame_images* images, soc_stream stream);
/* Add a caller pass. before = name of the pass it precedes, or NULL to append at the end of its phase.
 * Caller passes survive soc_renderer_set_raster_scene. Errors: duplicate name, unknown `before` or a `before`
 * in another phase, bad resource id, more than SOC_PASS_MAX_USES uses. */
int soc_renderer_add_pass(soc_renderer* r, const soc_pass_desc* desc, soc_pass_callback fn, void* user,
                          const char* before);
/* Declared uses of pass `index` as resource bitmasks (bit = enum soc_resource). */
int soc_renderer_pass_uses(const soc_renderer* r, int32_t index, uint64_t* reads, uint64_t* writes);
/* Derived dependencies of pass `index`: the indices of the earlier passes it must follow (ascending).
 * Returns their count (at most cap are written) or a negative error. */
int32_t soc_renderer_pass_dependencies(const soc_renderer* r, int32_t index, int32_t* out, int32_t cap);
/* Derived cross-frame (ring) dependencies of pass `index`: the passes of the PREVIOUS frame it must follow, for the
 * resources no earlier pass of its own frame writes (e.g. GBufferGeneration's depth write after the previous
 * frame's CloudRendering read it; CloudRendering's sky-colour write after the previous frame's TAA read the colour).
 * Indices ascending; returns their count (at most cap written) or a negative error. Cross-lane ring edges are
 * enforced by waits on the source pass's completion event; the fork at the start of a call orders the second lane
 * after everything queued on `stream` before the call. */
int32_t soc_renderer_pass_carry_dependencies(const soc_renderer* r, int32_t index, int32_t* out, int32_t cap);
/* Derived lane of pass `index` with the second lane enabled: 0 = the caller's stream, 1 = the second lane. */
int32_t soc_renderer_pass_lane(const soc_renderer* r, int32_t index);

/* --- Rasterisation: depth prepass, G-buffer and sun shadow map ---------------
 * Replaces the raster producers upstream of the hot path: DepthPrepassTask (depth_prepass.inl:26-120),
 * GBufferGenerationTask (g_buffer_generation.inl:33-230) and SunShadowDrawTask (sun_shadow_draw.inl:27-91).
 * A visibility buffer (one u64 per pixel: depth bits << 32 | triangle key) is filled by 64-bit atomicMin,
 * then one per-pixel resolve writes the reference's G-buffer images. Raster rules (the Vulkan ones the
 * reference pipelines select): pixel centres, a consistent tie rule for centres on shared edges (each is
 * covered once), depth clipping to [0, 1], LESS_OR_EQUAL test in draw order
 * (equal depth: the later triangle wins), culling by facing. Front faces are CLOCKWISE in the framebuffer
 * (Vulkan area a < 0): the reference culls FRONT for its glTF meshes, whose outward faces are counter-
 * clockwise as seen, so its pipelines' (Daxa default, not in the mount) front face must be clockwise.
 * Edge functions are homogeneous (2DH), so geometry behind the eye needs no clipping. The scene is one
 * mesh (the reference's draws concatenated). */
typedef struct soc_mesh {              /* device pointers (Vertex, shared.inl:152-157) */
    const float* positions;            /* vertex_count x float3, object space */
    const float* normals;              /* vertex_count x float3, object space */
    const float* uvs;                  /* vertex_count x float2 */
    const uint32_t* indices;           /* triangle_count x 3 */
    const uint32_t* materials;         /* triangle_count material indices, or NULL (all 0) */
    int32_t vertex_count, triangle_count;
    float model_matrix[16];            /* TransformComponent.model_matrix (column-major) */
    float normal_matrix[16];           /* TransformComponent.normal_matrix; its upper 3x3 transforms normals */
} soc_mesh;

/* Material (shared.inl:159-170, as GBufferGeneration's fragment shader reads it, g_buffer_generation.inl:
 * 189-225): albedo = sample(albedo).rgb * albedo_factor + emissive; emissive = sample(emissive).rgb *
 * emissive_factor (zero without an emissive image). Textures are RGBA8 (SRGB decoded to linear per
 * texel), bilinear, REPEAT; data == NULL samples white (model.cpp:188). Without SOC_MATERIAL_MIPMAPPED only
 * level 0 is read; with it every RGBA8 texture of the material carries its packed mip chain
 * (soc_generate_mips) and is sampled trilinear + anisotropic (the reference's sampler, texture.cpp:121-136):
 * see SOC_MATERIAL_MIPMAPPED. */
typedef struct soc_material {
    soc_img albedo, emissive;
    float albedo_factor[4], emissive_factor[4];
    int32_t flags;                     /* SOC_MATERIAL_* */
    int32_t has_emissive;              /* 0: emissive = 0 (has_emissive_image) */
    int32_t pad[2];
    soc_img normal_map;                /* RGBA16F, used with SOC_MATERIAL_NORMAL_MAP */
    soc_img normal_image;              /* RGBA8_UNORM tangent-space normal texture, with SOC_MATERIAL_NORMAL_TEXTURE */
    float max_anisotropy;              /* with SOC_MATERIAL_MIPMAPPED: 16 in the reference (texture.cpp:129-130) */
    int32_t pad2;
    /* optional, read only with SOC_MATERIAL_PAIRED_TEXELS set (with SOC_MATERIAL_MIPMAPPED and a normal_image of the
     * albedo's extent): the two mip chains interleaved texel by texel (soc_pair_textures), which the G-buffer resolve
     * then reads with one load per texel row pair for both textures (the same texels and results); without the flag
     * the two images are read separately. The field took bytes that were padding before: zero-initialise the struct. */
    void* paired_texels;
} soc_material;
#define SOC_MATERIAL_ZERO_VELOCITY 1   /* write velocity 0 (the terrain draw, draw_terrain.inl:221) */
#define SOC_MATERIAL_NORMAL_MAP 2      /* normal = normalize(bilinear normal_map(uv).xyz) (draw_terrain.inl:206-219) */
/* has_normal_image (g_buffer_generation.inl:197-211): n = normalize(TBN * (sample(normal_image).xyz * 2 - 1)) with
 * T = normalize(Q1 * st2.t - Q2 * st1.t), B = normalize(cross(N, T)); Q1/Q2 and st1/st2 are dFdx/dFdy of the world
 * position and uv, taken as FINE derivatives: the same triangle's perspective-correct attributes at the two pixel
 * centres of the pixel's 2x2 quad in that direction (what helper invocations evaluate). */
#define SOC_MATERIAL_NORMAL_TEXTURE 4
/* Mip-mapped sampling (texture.cpp:108-136: LINEAR min/mag/mip, REPEAT, anisotropy max_anisotropy, lod in
 * [0, levels]). Per texture, from the FINE uv derivatives of the pixel's quad (as the TBN above), in level-0
 * texels: Px = |(du/dx W, dv/dx H)|, Py = |(du/dy W, dv/dy H)|, N = min(ceil(Pmax / Pmin), floor(max_anisotropy))
 * (1 when max_anisotropy <= 1, Pmax is 0 or not finite; floor(max_anisotropy) when Pmin is 0),
 * lod = log2(Pmax / N) (the deterministic log2 of the histogram contract) rounded to 1/256 and clamped to
 * [0, levels - 1]; result = (1/N) sum_{i=1..N} trilinear(uv + (i / (N + 1) - 1/2) d_major) with d_major the uv
 * derivative of the longer axis (EXT_texture_filter_anisotropic's reference filter; N = 1 samples uv itself);
 * trilinear = lerp of the bilinear REPEAT samples of levels floor(lod) and floor(lod) + 1. */
#define SOC_MATERIAL_MIPMAPPED 8
/* paired_texels holds the soc_pair_textures buffer of this material's albedo + normal_image (explicit opt-in: a caller
 * that fills the struct field by field without zeroing it never has stale padding read as a pointer) */
#define SOC_MATERIAL_PAIRED_TEXELS 16

#define SOC_CULL_NONE 0
#define SOC_CULL_FRONT 1               /* depth prepass / G-buffer (depth_prepass.inl:45) */
#define SOC_CULL_BACK 2                /* sun shadow (sun_shadow_draw.inl:46) */

/* Workspace of the raster passes for a mesh (screen-space vertices, large-triangle list). */
size_t soc_raster_workspace_size(int32_t vertex_count, int32_t triangle_count);
/* Visibility buffer (u64 per pixel, width*height, tight): clear = 1 resets it to "empty, depth 1.0"
 * first. `view_projection` is the camera's projection*view (camera_projection_view_matrix). */
int soc_raster_visibility(const soc_mesh* mesh, const float view_projection[16], int32_t cull,
                          uint64_t* visibility, int32_t width, int32_t height, int32_t clear,
                          void* workspace, soc_stream stream);
/* Depth-only raster into a D32 image (cleared to 1.0), with the pipeline's depth bias: z += slope *
 * max(|dz/dx|, |dz/dy|) + constant * 2^(e - 23), e = the exponent of the triangle's largest |z|
 * (sun_shadow_draw.inl:47-50: 1.25 / 1.75). */
int soc_raster_depth(const soc_mesh* mesh, const float view_projection[16], int32_t cull, float bias_constant,
                     float bias_slope, soc_img depth, void* workspace, soc_stream stream);
/* G-buffer from a visibility buffer: depth (D32), albedo / emissive / normal / velocity (RGBA16F), with the
 * clear values of GBufferGeneration for empty pixels. `d_materials` is a device array. `workspace`
 * (soc_raster_workspace_size bytes, may be the raster's) lets the vertex stage run once per vertex;
 * NULL evaluates it per pixel. Same bits either way. */
int soc_gbuffer_resolve(const soc_globals* g, const soc_mesh* mesh, const soc_material* d_materials,
                        int32_t material_count, const uint64_t* visibility, soc_img depth, soc_img albedo,
                        soc_img emissive, soc_img normal, soc_img velocity, void* workspace, soc_stream stream);

/* DrawTerrain / SunShadowDrawTerrain patch tessellation (renderer.cpp:194-220 builds a grid_size^2 uv control
 * grid, 100 in the reference, of 4-point quad patches; draw_terrain.inl:144-191 tessellates each at
 * terrain_max_tess_level (3) with fractional_odd_spacing and displaces it by (heightmap(uv).r -
 * terrain_midpoint) * terrain_height_scale). Odd integer levels only (n equal segments). Output: the
 * ((grid - 1) n + 1)^2 shared vertices in world space (x = u scale.x - offset.x, y = offset.y + height,
 * z = v scale.y - offset.z; the TES's clip-space point before the linear clip transform), up normals (the
 * G-buffer normal comes from the terrain normal map), uvs, and 2 triangles per tessellated quad,
 * counter-clockwise seen from above. Heightmap: RGBA8_UNORM, bilinear clamp-to-edge (.r). */
int soc_terrain_tess_counts(int32_t grid_size, int32_t tess_level, int32_t* vertices, int32_t* triangles);
int soc_terrain_tessellate(const soc_globals* g, soc_img heightmap, int32_t grid_size, int32_t tess_level,
                           float* positions, float* normals, float* uvs, uint32_t* indices, soc_stream stream);

/* Texture mip chains (texture.cpp:108, 184-246): floor(log2(max(W, H))) + 1 levels, level k of max(1, W >> k) x
 * max(1, H >> k) texels. Packed chain layout: level 0 is the soc_img itself (any pitch); level k >= 1 follows at
 * data + pitch_bytes * H + sum_{1 <= j < k} 4 w_j h_j with tight rows. soc_mip_chain_bytes is the size of the
 * whole allocation (level 0 included). */
int32_t soc_mip_level_count(int32_t width, int32_t height);
size_t soc_mip_chain_bytes(int32_t width, int32_t height, int32_t pitch_bytes);
/* The load-time blit chain (texture.cpp:190-246): level k from level k-1 by a LINEAR blit (vkCmdBlitImage):
 * destination texel (x, y) samples the source at ((x + 0.5) Ws / Wd, (y + 0.5) Hs / Hd) bilinearly, clamp to
 * edge, 8-bit sub-texel weights; RGBA8_SRGB filters in linear space (per-texel decode, re-encoded to the
 * nearest sRGB code: the largest k with linear >= the midpoint of codes k-1 and k), RGBA8_UNORM and alpha
 * round to nearest. Runs once per texture at load (upload), one launch per level on `stream`. */
int soc_generate_mips(soc_img texture, soc_stream stream);
/* A material's albedo and normal image mip chains (both generated, one extent) interleaved texel by texel into
 * `paired` (soc_paired_texels_bytes(width, height) bytes, device): level k holds, for texel i of its tight
 * w_k x h_k rows, the albedo texel then the normal texel (8 B), levels packed after one another from level 0.
 * Runs once per material at load, on `stream`. */
size_t soc_paired_texels_bytes(int32_t width, int32_t height);
int soc_pair_textures(soc_img albedo, soc_img normal_image, void* paired, soc_stream stream);

/* HeightToNormalTask (height_to_normal.inl:52-83): RGBA8 heightmap (.r) -> RGBA16F normal map of the same
 * extent; run once at terrain load (renderer.cpp:158-190). */
int soc_height_to_normal(soc_img heightmap, soc_img normal_target, soc_stream stream);

/* GenerateMinHIZTask / GenerateMaxHIZTask (generate_min_hiz.inl:23-95, generate_hiz.glsl:17-98): single-pass
 * min (op_max = 0) or max depth pyramid. mips[i] is D32 of (W/2 >> i) x (H/2 >> i) (at least 1), i <
 * mip_count <= 12 (the reference uses ceil(log2(max(W, H) / 2)) levels); `counter` is one device u32 of
 * scratch (reset by the call). Computed but unused by the reference graph (quirk Q12). */
int soc_generate_hiz(const soc_globals* g, soc_img depth, const soc_img* mips, int32_t mip_count, int32_t op_max,
                     uint32_t* counter, soc_stream stream);

/* Render-graph raster head (renderer.cpp:965-1021: DepthPrepass, SunShadowDraw, GBufferGeneration): with a
 * scene set, every PRE phase first rasterises the mesh into the frame's G-buffer images (depth, albedo,
 * emissive, normal, velocity) and, with `shadow`, the sun shadow map into images.shadow, on the caller's
 * stream before the sky lane forks. The renderer copies the struct (the arrays stay caller-owned). Passes
 * are rebuilt: per-pass timing set before this call is re-enabled only through SOC_RENDERER_TIMING. */
typedef struct soc_raster_scene {
    soc_mesh mesh;                     /* device arrays */
    const soc_material* materials;     /* device array */
    int32_t material_count;
    int32_t shadow;                    /* 1: SunShadowDraw into images.shadow (cull BACK, bias 1.25 / 1.75) */
    uint64_t* visibility;              /* width*height u64, device */
    void* workspace;                   /* soc_raster_workspace_size(mesh) bytes, device */
} soc_raster_scene;
/* NULL: clear. With shadow = 1 the renderer allocates a second raster workspace (soc_raster_workspace_size of the mesh)
 * for the sun shadow draw, which then runs on its second lane beside the depth prepass and the G-buffer. */
int soc_renderer_set_raster_scene(soc_renderer* r, const soc_raster_scene* scene);

/* --- Headless output and metrics (replaces the swapchain present of tone_mapping.inl:
 * 172-176 and the ImGui "GPU Metric" window of renderer.cpp:769-806) ------------------------------- */
/* The most recent frame's timed passes as one JSON object: {"frame", "total_gpu_ms", "groups" (the 12
 * group names of renderer.cpp:577-588, 0 when absent), "passes"}. Writes at most cap-1 bytes + NUL;
 * returns the full length (snprintf-style) or < 0. Needs a completed stream. */
int64_t soc_renderer_metrics_json(soc_renderer* r, uint64_t frame, char* buf, size_t cap);
/* Device image -> host rows, stream-ordered. */
int soc_read_image(soc_img image, void* host, int32_t host_pitch_bytes, soc_stream stream);
/* 8-bit RGBA host image -> PNG file (uncompressed deflate; no external library). */
int soc_write_png(const char* path, const void* rgba8, int32_t width, int32_t height, int32_t pitch_bytes);
/* RGBA16F host image (e.g. the HDR composition / TAA colour) -> OpenEXR 2 scanline file, uncompressed HALF
 * channels (the f16 framebuffer dump; the reference reads EXR through tinyexr, texture.cpp:300-412). */
int soc_write_exr(const char* path, const void* rgba16f, int32_t width, int32_t height, int32_t pitch_bytes);

#ifdef __cplusplus
}
#endif

#endif /* SOC_RT_H */
