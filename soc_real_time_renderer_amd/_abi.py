"""ctypes mirror of include/soc_rt.h (the C ABI of the MI355X pass library).

The struct layouts here are checked against the library's own offsetof/sizeof tables by
tests/test_abi.py, so a drift between this file and the header fails loudly.
"""
from __future__ import annotations

import ctypes as C

SOC_OK = 0
SOC_E_INVALID_ARG = -1
SOC_E_SHAPE = -2
SOC_E_HIP = -3
SOC_E_UNSUPPORTED = -4

FMT_RGBA16F = 1
FMT_D32F = 2
FMT_R8_UNORM = 3
FMT_RGBA8_UNORM = 4
FMT_RGBA8_SRGB = 5
FMT_RGBA32F = 6

BYTES_PER_PIXEL = {FMT_RGBA16F: 8, FMT_D32F: 4, FMT_R8_UNORM: 1, FMT_RGBA8_UNORM: 4, FMT_RGBA8_SRGB: 4,
                   FMT_RGBA32F: 16}

MAX_POINT_LIGHTS = 128
MAX_SPOT_LIGHTS = 128
BIN_COUNT = 256
SSAO_MAX_KERNEL = 26

PHASE_PRE_EXPOSURE = 1
PHASE_POST_EXPOSURE = 2
PHASE_ALL = 3
RENDERER_TIMING = 1
RENDERER_UNFUSED_BLOOM = 2
RENDERER_SERIAL = 4
RENDERER_UNFUSED_TONEMAP = 8
RENDERER_FUSED_HISTOGRAM = 16
RENDERER_EXACT_BLOOM = 32
RENDERER_UNFUSED_HISTOGRAM = 64
RENDERER_NO_SKY_SPLIT = 128
RENDERER_STATIC_INPUTS = 256
RENDERER_VELOCITY_SLOTS = 512
RENDERER_BLOOM_IN_COMPOSITION = 1024
RENDERER_SKY_LANE_HIGH = 2048
RENDERER_SKY_LANE_PROBE = 4096
HISTOGRAM_SCRATCH_WORDS = 2048

Mat4 = C.c_float * 16
Vec2 = C.c_float * 2
Vec3 = C.c_float * 3
Vec4 = C.c_float * 4


class SocImg(C.Structure):
    _fields_ = [("data", C.c_void_p), ("width", C.c_int32), ("height", C.c_int32), ("pitch_bytes", C.c_int32),
                ("format", C.c_int32)]


class PointLight(C.Structure):
    _fields_ = [("position", Vec3), ("color", Vec3), ("intensity", C.c_float)]


class SpotLight(C.Structure):
    _fields_ = [("position", Vec3), ("direction", Vec3), ("color", Vec3), ("intensity", C.c_float),
                ("cut_off", C.c_float), ("outer_cut_off", C.c_float)]


class SunInfo(C.Structure):
    _fields_ = [("projection_matrix", Mat4), ("view_matrix", Mat4), ("projection_view_matrix", Mat4),
                ("terrain_y_clip_trick", Vec4), ("position", Vec3), ("direction", Vec3),
                ("exponential_factor", C.c_float), ("darkening_factor", C.c_float), ("bias", C.c_float),
                ("intensity", C.c_float)]


class Globals(C.Structure):
    """Mirror of ShaderGlobals (src/graphics/shared.inl:47-131)."""
    _fields_ = [
        ("camera_projection_matrix", Mat4), ("camera_inverse_projection_matrix", Mat4),
        ("camera_view_matrix", Mat4), ("camera_inverse_view_matrix", Mat4),
        ("camera_projection_view_matrix", Mat4), ("camera_inverse_projection_view_matrix", Mat4),
        ("camera_previous_projection_matrix", Mat4), ("camera_previous_inverse_projection_matrix", Mat4),
        ("camera_previous_view_matrix", Mat4), ("camera_previous_inverse_view_matrix", Mat4),
        ("camera_previous_projection_view_matrix", Mat4), ("camera_previous_inverse_projection_view_matrix", Mat4),
        ("jitter", Vec2), ("previous_jitter", Vec2),
        ("camera_position", Vec3), ("camera_near_clip", C.c_float), ("camera_far_clip", C.c_float),
        ("resolution", C.c_int32 * 2), ("elapsed_time", C.c_float), ("delta_time", C.c_float),
        ("frame_counter", C.c_uint32),
        ("sun_info", SunInfo),
        ("point_light_count", C.c_uint32), ("spot_light_count", C.c_uint32),
        ("point_lights", PointLight * MAX_POINT_LIGHTS), ("spot_lights", SpotLight * MAX_SPOT_LIGHTS),
        ("terrain_offset", Vec3), ("terrain_scale", Vec2), ("terrain_height_scale", C.c_float),
        ("terrain_midpoint", C.c_float), ("terrain_delta", C.c_float), ("terrain_min_depth", C.c_float),
        ("terrain_max_depth", C.c_float), ("terrain_min_tess_level", C.c_int32), ("terrain_max_tess_level", C.c_int32),
        ("terrain_y_clip_trick", Vec4), ("terrain_previous_y_clip_trick", Vec4),
        ("filter_radius", C.c_float),
        ("ssao_bias", C.c_float), ("ssao_radius", C.c_float), ("ssao_kernel_size", C.c_int32),
        ("ambient", Vec3), ("ambient_occlussion_strength", C.c_float), ("emissive_bloom_strength", C.c_float),
        ("focal_length", C.c_float), ("plane_in_focus", C.c_float), ("aperture", C.c_float),
        ("adjustment_speed", C.c_float), ("log_min_luminance", C.c_float), ("log_max_luminance", C.c_float),
        ("target_luminance", C.c_float),
        ("saturation", C.c_float), ("agxDs_linear_section", C.c_float), ("peak", C.c_float), ("compression", C.c_float),
    ]


class AutoExposure(C.Structure):
    _fields_ = [("exposure", C.c_float), ("histogram_buckets", C.c_uint32 * BIN_COUNT)]


class Camera(C.Structure):
    _fields_ = [("position", Vec3), ("rotation", Vec3), ("fov_degrees", C.c_float), ("near_clip", C.c_float),
                ("far_clip", C.c_float)]


class FrameImages(C.Structure):
    _fields_ = [
        ("albedo", SocImg), ("emissive", SocImg), ("normal", SocImg), ("depth", SocImg), ("velocity", SocImg),
        ("shadow", SocImg), ("noise", SocImg), ("bloom_mips", SocImg * 4), ("ssao", SocImg), ("ssao_blur", SocImg),
        ("clouds", SocImg), ("color", SocImg), ("history_color", SocImg * 2), ("history_velocity", SocImg * 2),
        ("output", SocImg), ("ssao_noise_table", C.c_void_p), ("auto_exposure", C.c_void_p), ("d_globals", C.c_void_p),
        ("bloom_output", SocImg), ("clouds_workspace", C.c_void_p),
    ]


class Mesh(C.Structure):
    _fields_ = [("positions", C.c_void_p), ("normals", C.c_void_p), ("uvs", C.c_void_p), ("indices", C.c_void_p),
                ("materials", C.c_void_p), ("vertex_count", C.c_int32), ("triangle_count", C.c_int32),
                ("model_matrix", Mat4), ("normal_matrix", Mat4)]


class Material(C.Structure):
    _fields_ = [("albedo", SocImg), ("emissive", SocImg), ("albedo_factor", C.c_float * 4),
                ("emissive_factor", C.c_float * 4), ("flags", C.c_int32), ("has_emissive", C.c_int32),
                ("pad", C.c_int32 * 2), ("normal_map", SocImg), ("normal_image", SocImg),
                ("max_anisotropy", C.c_float), ("pad2", C.c_int32), ("paired_texels", C.c_void_p)]


class RasterScene(C.Structure):
    _fields_ = [("mesh", Mesh), ("materials", C.c_void_p), ("material_count", C.c_int32), ("shadow", C.c_int32),
                ("visibility", C.c_void_p), ("workspace", C.c_void_p)]


ENTITY_POINT_LIGHT, ENTITY_SPOT_LIGHT = 1, 2


class Entity(C.Structure):
    """soc_entity: TransformComponent + optional Point/SpotLightComponent (src/ecs/components.hpp)."""
    _fields_ = [("position", Vec3), ("rotation", Vec3), ("scale", Vec3), ("components", C.c_int32), ("color", Vec3),
                ("intensity", C.c_float), ("cut_off", C.c_float), ("outer_cut_off", C.c_float)]


# enum soc_resource (include/soc_rt.h): the frame resources a pass declares it reads / writes
RESOURCES = ["ALBEDO", "EMISSIVE", "NORMAL", "DEPTH", "VELOCITY", "SUN_SHADOW", "NOISE", "BLOOM_MIP0", "BLOOM_MIP1",
             "BLOOM_MIP2", "BLOOM_MIP3", "BLOOM_OUTPUT", "SSAO", "SSAO_BLUR", "CLOUDS", "COLOR", "PREVIOUS_COLOR",
             "RESOLVED", "PREVIOUS_VELOCITY", "AUTO_EXPOSURE", "OUTPUT", "VISIBILITY", "HISTOGRAM_PARTIALS",
             "SKY_COLOR", "SKY_HISTOGRAM_PARTIALS"]
RES = {n: i for i, n in enumerate(RESOURCES)}
RES_USER0 = 32
RES_COUNT = 64
PASS_MAX_USES = 16
PASS_ASYNC = 1


class PassDesc(C.Structure):
    _fields_ = [("name", C.c_char_p), ("group", C.c_char_p), ("phase", C.c_int32), ("flags", C.c_uint32),
                ("read_count", C.c_int32), ("write_count", C.c_int32), ("reads", C.c_int32 * PASS_MAX_USES),
                ("writes", C.c_int32 * PASS_MAX_USES)]


# int32_t (*soc_pass_callback)(void* user, const soc_globals*, const soc_frame_images*, soc_stream)
PASS_CALLBACK = C.CFUNCTYPE(C.c_int32, C.c_void_p, C.POINTER(Globals), C.POINTER(FrameImages), C.c_void_p)

CULL_NONE, CULL_FRONT, CULL_BACK = 0, 1, 2
MATERIAL_ZERO_VELOCITY = 1
MATERIAL_NORMAL_MAP = 2
MATERIAL_NORMAL_TEXTURE = 4
MATERIAL_MIPMAPPED = 8
MATERIAL_PAIRED_TEXELS = 16

STRUCTS = {"soc_img": SocImg, "soc_globals": Globals, "soc_sun_info": SunInfo, "soc_point_light": PointLight,
           "soc_spot_light": SpotLight, "soc_auto_exposure": AutoExposure, "soc_camera": Camera,
           "soc_frame_images": FrameImages, "soc_mesh": Mesh, "soc_material": Material,
           "soc_raster_scene": RasterScene, "soc_pass_desc": PassDesc, "soc_entity": Entity}

_I = C.c_int
_P = C.c_void_p
_IMG = SocImg
_G = C.POINTER(Globals)

# name -> (restype, argtypes); every function declared in include/soc_rt.h
FUNCTIONS = {
    "soc_abi_version": (C.c_int32, []),
    "soc_abi_sizeof": (C.c_size_t, [C.c_char_p]),
    "soc_abi_offsetof": (C.c_int64, [C.c_char_p, C.c_char_p]),
    "soc_last_error_string": (C.c_char_p, []),
    "soc_tuning_reload": (None, []),
    "soc_check_block_shape": (C.c_int, [C.c_int32] * 4),
    "soc_device_arch": (C.c_char_p, []),
    "soc_globals_init_defaults": (_I, [_G, C.c_int32, C.c_int32]),
    "soc_globals_frame_update": (_I, [_G, C.POINTER(Camera), C.c_int32, C.c_int32, C.c_float, C.POINTER(C.c_uint32)]),
    "soc_mat4_perspective_rh_no": (None, [C.POINTER(C.c_float), C.c_float, C.c_float, C.c_float, C.c_float]),
    "soc_mat4_ortho_rh_no": (None, [C.POINTER(C.c_float)] + [C.c_float] * 6),
    "soc_mat4_look_at_rh": (None, [C.POINTER(C.c_float)] * 4),
    "soc_mat4_inverse": (None, [C.POINTER(C.c_float)] * 2),
    "soc_mat4_mul": (None, [C.POINTER(C.c_float)] * 3),
    "soc_bloom_downsample": (_I, [_G, _IMG, _IMG, _P]),
    "soc_bloom_upsample": (_I, [_G, _IMG, _IMG, _P]),
    "soc_bloom_chain": (_I, [_G, _IMG, C.POINTER(SocImg), C.c_int32, _P]),
    "soc_bloom_weighted_stage": (_I, [_G, _IMG, C.POINTER(SocImg), C.c_int32, _IMG, C.c_int32, _P]),
    "soc_ssao_prepare_noise": (_I, [_IMG, _IMG, _P, _P]),
    "soc_ssao_generation": (_I, [_G, _IMG, _IMG, _IMG, _P, _P]),
    "soc_ssao_blur": (_I, [_G, _IMG, _IMG, _P]),
    "soc_cloud_rendering_workspace_size": (C.c_size_t, [C.c_int32, C.c_int32]),
    "soc_cloud_rendering": (_I, [_G, _IMG, _IMG, _IMG, _P, _P]),
    "soc_composition_luminance_histogram": (_I, [_G, _P, _IMG, _IMG, _IMG, _IMG, _IMG, _IMG, _IMG, _IMG, _P, _P, _P]),
    "soc_composition": (_I, [_G, _P, _IMG, _IMG, _IMG, _IMG, _IMG, _IMG, _IMG, _IMG, _P]),
    "soc_generate_luminance_histogram": (_I, [_G, _IMG, _P, _P]),
    "soc_resolve_luminance_histogram": (_I, [_G, _P, C.c_uint64, C.c_int32, _P]),
    "soc_temporal_antialiasing_tone_mapping": (_I, [_G, _IMG, _IMG, _IMG, _IMG, _IMG, _IMG, _IMG, _P, _IMG, _P]),
    "soc_temporal_antialiasing": (_I, [_G, _IMG, _IMG, _IMG, _IMG, _IMG, _IMG, _IMG, _P]),
    "soc_copy_image": (_I, [_IMG, _IMG, _P]),
    "soc_tone_mapping": (_I, [_G, _IMG, _P, _IMG, _P]),
    "soc_upload_globals": (_I, [_G, _P, _P]),
    "soc_renderer_create": (_P, [C.POINTER(FrameImages), C.c_uint32]),
    "soc_renderer_destroy": (None, [_P]),
    "soc_renderer_execute": (_I, [_P, _G, C.c_int32, _P]),
    "soc_renderer_set_exposure_pixels": (_I, [_P, C.c_uint64, C.c_int32]),
    "soc_renderer_pass_count": (C.c_int32, [_P]),
    "soc_renderer_pass_name": (C.c_char_p, [_P, C.c_int32]),
    "soc_renderer_pass_group": (C.c_char_p, [_P, C.c_int32]),
    "soc_renderer_pass_ms": (C.c_float, [_P, C.c_int32]),
    "soc_renderer_current_history": (C.c_int32, [_P]),
    "soc_renderer_set_current_history": (C.c_int, [_P, C.c_int32]),
    "soc_renderer_set_async": (C.c_int, [_P, C.c_int32]),
    "soc_scene_update": (_I, [C.POINTER(Globals), C.POINTER(Entity), C.c_int32, C.POINTER(C.c_float),
                              C.POINTER(C.c_float)]),
    "soc_renderer_add_pass": (_I, [_P, C.POINTER(PassDesc), PASS_CALLBACK, _P, C.c_char_p]),
    "soc_renderer_pass_uses": (_I, [_P, C.c_int32, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    "soc_renderer_pass_dependencies": (C.c_int32, [_P, C.c_int32, C.POINTER(C.c_int32), C.c_int32]),
    "soc_renderer_pass_carry_dependencies": (C.c_int32, [_P, C.c_int32, C.POINTER(C.c_int32), C.c_int32]),
    "soc_renderer_pass_lane": (C.c_int32, [_P, C.c_int32]),
    "soc_renderer_set_pass_timing": (_I, [_P, C.c_int32, C.c_int32]),
    "soc_renderer_reset_timing": (_I, [_P]),
    "soc_renderer_pass_stats": (_I, [_P, C.c_int32, C.POINTER(C.c_float), C.POINTER(C.c_int32)]),
    "soc_renderer_pass_event_times": (C.c_int32, [_P, C.c_int32, _P, C.POINTER(C.c_float), C.POINTER(C.c_float),
                                                  C.c_int32]),
    "soc_renderer_side_queue": (C.c_int32, [_P]),
    "soc_renderer_side_queue_probe_frames": (C.c_int32, [_P]),
    "soc_raster_workspace_size": (C.c_size_t, [C.c_int32, C.c_int32]),
    "soc_paired_texels_bytes": (C.c_size_t, [C.c_int32, C.c_int32]),
    "soc_renderer_set_raster_scene": (_I, [_P, C.POINTER(RasterScene)]),
    "soc_height_to_normal": (_I, [_IMG, _IMG, _P]),
    "soc_terrain_tess_counts": (_I, [_I, _I, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    "soc_terrain_tessellate": (_I, [_G, _IMG, _I, _I, _P, _P, _P, _P, _P]),
    "soc_mip_level_count": (_I, [_I, _I]),
    "soc_mip_chain_bytes": (C.c_size_t, [_I, _I, _I]),
    "soc_generate_mips": (_I, [_IMG, _P]),
    "soc_pair_textures": (_I, [_IMG, _IMG, _P, _P]),
    "soc_generate_hiz": (_I, [_G, _IMG, C.POINTER(SocImg), C.c_int32, C.c_int32, _P, _P]),
    "soc_renderer_metrics_json": (C.c_int64, [_P, C.c_uint64, C.c_char_p, C.c_size_t]),
    "soc_read_image": (_I, [_IMG, _P, C.c_int32, _P]),
    "soc_write_png": (_I, [C.c_char_p, _P, C.c_int32, C.c_int32, C.c_int32]),
    "soc_write_exr": (_I, [C.c_char_p, _P, C.c_int32, C.c_int32, C.c_int32]),
    "soc_raster_visibility": (_I, [C.POINTER(Mesh), C.POINTER(C.c_float), C.c_int32, _P, C.c_int32, C.c_int32,
                                   C.c_int32, _P, _P]),
    "soc_raster_depth": (_I, [C.POINTER(Mesh), C.POINTER(C.c_float), C.c_int32, C.c_float, C.c_float, _IMG, _P, _P]),
    "soc_gbuffer_resolve": (_I, [_G, C.POINTER(Mesh), _P, C.c_int32, _P, _IMG, _IMG, _IMG, _IMG, _IMG, _P, _P]),
}

# not in the public header: test hooks
DEBUG_FUNCTIONS = {
    "soc_debug_bloom_generic": (_I, [C.c_int32, _IMG, _IMG, _P]),
}


def bind(lib: C.CDLL, table: dict) -> None:
    for name, (res, args) in table.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
