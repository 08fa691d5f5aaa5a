/*
 * soc_oracle.h — CPU restatement ("oracle") of the reference's screen-space passes.
 *
 * TEST INFRASTRUCTURE ONLY. Nothing in the product path (soc_real_time_renderer_amd/) may link,
 * load or call this code. Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use
 * it, as the checker and as the timed CPU baseline.
 *
 * Parity status: the reference (Vulkan/GLSL via Daxa) cannot be built or run here
 * and ships no tests, golden vectors or fixtures. The restatement is therefore
 * pinned by hand-derived known-answer tests of the reference formulas (tests/test_oracle_kat.py)
 * and cross-checked against an independent numpy restatement of the GLSL (oracle/np_oracle.py,
 * tests/test_np_oracle.py) — "parity unpinned" against a run of the reference itself.
 *
 * Functions take the same arguments as the C ABI in include/soc_rt.h, with HOST pointers.
 */
#ifndef SOC_ORACLE_H
#define SOC_ORACLE_H

#include "../include/soc_rt.h"

#ifdef __cplusplus
extern "C" {
#endif

int soc_oracle_bloom_downsample(const soc_globals* g, soc_img higher_mip, soc_img lower_mip);
int soc_oracle_bloom_upsample(const soc_globals* g, soc_img lower_mip, soc_img higher_mip);
int soc_oracle_ssao_generation(const soc_globals* g, soc_img depth, soc_img normal, soc_img target);
/* The same taps with the random vectors given per target pixel (x, y pairs), e.g. the GPU's table: isolates the tap
   arithmetic from the Q8 hash's sinf precision in the parity checks. */
int soc_oracle_ssao_generation_rv(const soc_globals* g, soc_img depth, soc_img normal, const float* rv_table,
                                  soc_img target);
int soc_oracle_ssao_random_vectors(int32_t normal_width, int32_t tw, int32_t th, float* out);
int soc_oracle_ssao_blur(const soc_globals* g, soc_img ssao, soc_img target);
int soc_oracle_cloud_rendering(const soc_globals* g, soc_img depth, soc_img noise, soc_img target);
int soc_oracle_composition(const soc_globals* g, soc_img target, soc_img albedo, soc_img emissive,
                           soc_img normal, soc_img depth, soc_img ssao, soc_img shadow, soc_img clouds);
int soc_oracle_generate_luminance_histogram(const soc_globals* g, soc_img hdr, soc_auto_exposure* ae);
int soc_oracle_resolve_luminance_histogram(const soc_globals* g, soc_auto_exposure* ae,
                                           uint64_t total_pixels, int32_t wide_accumulator);
int soc_oracle_temporal_antialiasing(const soc_globals* g, soc_img target, soc_img current_color,
                                     soc_img previous_color, soc_img current_velocity,
                                     soc_img previous_velocity, soc_img depth);
int soc_oracle_tone_mapping(const soc_globals* g, soc_img color, const soc_auto_exposure* ae, soc_img target);

/* Rasterisation: host-pointer mesh / materials, same arguments as the C ABI. */
int soc_oracle_raster_visibility(const soc_mesh* mesh, const float view_projection[16], int32_t cull,
                                 uint64_t* visibility, int32_t width, int32_t height);
int soc_oracle_raster_depth(const soc_mesh* mesh, const float view_projection[16], int32_t cull, float bias_constant,
                            float bias_slope, soc_img depth);
int soc_oracle_gbuffer_resolve(const soc_globals* g, const soc_mesh* mesh, const soc_material* materials,
                               int32_t material_count, const uint64_t* visibility, soc_img depth, soc_img albedo,
                               soc_img emissive, soc_img normal, soc_img velocity);

/* soc_generate_mips (texture.cpp:184-246): levels 1.. of a packed RGBA8 chain from level 0, in place. */
int soc_oracle_generate_mips(soc_img texture);
int soc_oracle_height_to_normal(soc_img heightmap, soc_img target);
/* soc_terrain_tessellate (draw_terrain.inl:138-191): the tessellated terrain vertices / indices. */
int soc_oracle_terrain_tessellate(const soc_globals* g, soc_img heightmap, int32_t grid_size, int32_t tess_level,
                                  float* positions, float* normals, float* uvs, uint32_t* indices);
int soc_oracle_generate_hiz(const soc_globals* g, soc_img depth, const soc_img* mips, int32_t mip_count, int32_t op_max);

/* Scalar helpers exposed for known-answer tests. */
uint32_t soc_oracle_luminance_bin(float r, float g, float b, float log_min, float log_max);
float soc_oracle_log2(float x);
/* The SSAO noise hash's deterministic sin / cos / pow (quirk Q8; the same operation sequence as ssao.hip's random-vector
   table): double evaluation with IEEE operations only, one rounding to float. */
float soc_oracle_det_sin(float x);
float soc_oracle_det_cos(float x);
float soc_oracle_det_pow(float x, float y);
uint16_t soc_oracle_f32_to_f16(float x);
float soc_oracle_f16_to_f32(uint16_t h);
/* Per-sky-pixel operation tallies of the clouds pass (filled by the last soc_oracle_cloud_rendering
 * call with counting enabled): [0]=sky pixels, [1]=cloud-march steps with density, [2]=get_clouds
 * evaluations, [3]=noise taps. */
/* Tallies of the last soc_oracle_cloud_rendering call (tools/clouds_flops.py): sky pixels, dense cloud steps,
   get_clouds calls, noise taps, get_clouds calls past the altitude test, full atmosphere evaluations, cloud marches,
   pixels. */
#define SOC_ORACLE_CLOUD_COUNTERS 8
void soc_oracle_clouds_counters(uint64_t out[SOC_ORACLE_CLOUD_COUNTERS]);
int soc_oracle_num_threads(void);

#ifdef __cplusplus
}
#endif
#endif
