"""MI355X-native screen-space deferred shading + post-processing for lukasino1214/soc_real_time_renderer.

The product path is the HIP pass library ``lib/libsoc_rt.so`` (C ABI: ``include/soc_rt.h``), built for
gfx950 by ``__graft_entry__.build()``. This module is a thin host binding over that ABI: torch provides
device memory and streams; every pass runs in the library. There is no CPU fallback — if the library
is missing, importing the pass functions raises.

Pass functions mirror the reference's task structs (src/graphics/tasks/*.inl); see include/soc_rt.h
for the file:line each replaces.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional

import numpy as np
import torch  # noqa: F401  (loads the HIP runtime first: libsoc_rt.so then shares it)

from . import _abi
from ._abi import (FMT_D32F, FMT_R8_UNORM, FMT_RGBA8_SRGB, FMT_RGBA8_UNORM, FMT_RGBA16F, FMT_RGBA32F,
                   PHASE_ALL, PHASE_POST_EXPOSURE, PHASE_PRE_EXPOSURE, AutoExposure, Camera, FrameImages, Globals,
                   SocImg)

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG_DIR, "lib", os.environ.get("SOC_RT_LIB_VARIANT", "libsoc_rt.so"))   # variant: A/B builds

__all__ = ["SocError", "lib", "img", "Globals", "Camera", "AutoExposure", "globals_defaults", "frame_update",
           "bloom_downsample", "bloom_upsample", "bloom_chain", "ssao_prepare_noise", "ssao_generation",
           "ssao_blur", "cloud_rendering", "composition", "generate_luminance_histogram",
           "resolve_luminance_histogram", "temporal_antialiasing", "copy_image", "tone_mapping", "upload_globals",
           "Renderer", "read_image", "write_png", "write_exr", "FMT_RGBA16F", "FMT_D32F", "FMT_R8_UNORM", "FMT_RGBA8_UNORM", "FMT_RGBA8_SRGB",
           "FMT_RGBA32F", "PHASE_PRE_EXPOSURE", "PHASE_POST_EXPOSURE", "PHASE_ALL"]


class SocError(RuntimeError):
    def __init__(self, rc: int, msg: str):
        super().__init__(f"[soc rc={rc}] {msg}")
        self.rc = rc


_LIB: Optional[C.CDLL] = None


def lib() -> C.CDLL:
    """The HIP pass library; raises if it has not been built (no fallback path exists)."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} not built: run `python -c 'import __graft_entry__ as g; g.build()'`")
        l = C.CDLL(LIB_PATH)
        _abi.bind(l, _abi.FUNCTIONS)
        _abi.bind(l, _abi.DEBUG_FUNCTIONS)
        _LIB = l
    return _LIB


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise SocError(rc, f"{what}: {lib().soc_last_error_string().decode(errors='replace')}")


# ------------------------------------------------------------------------------------------------
# images
# ------------------------------------------------------------------------------------------------
def infer_format(shape, dtype) -> int:
    nd = len(shape)
    if dtype in (torch.float16, np.float16) and nd == 3 and shape[2] == 4:
        return FMT_RGBA16F
    if dtype in (torch.float32, np.float32) and nd == 2:
        return FMT_D32F
    if dtype in (torch.float32, np.float32) and nd == 3 and shape[2] == 4:
        return FMT_RGBA32F
    if dtype in (torch.uint8, np.uint8) and nd == 2:
        return FMT_R8_UNORM
    if dtype in (torch.uint8, np.uint8) and nd == 3 and shape[2] == 4:
        return FMT_RGBA8_UNORM
    raise ValueError(f"cannot infer image format for shape {tuple(shape)} dtype {dtype}")


def img(t, fmt: Optional[int] = None) -> SocImg:
    """soc_img view of an (H, W[, 4]) torch tensor (device or host) or numpy array; rows may be padded."""
    if t is None:
        return SocImg(None, 0, 0, 0, 0)
    if isinstance(t, torch.Tensor):
        f = fmt or infer_format(tuple(t.shape), t.dtype)
        if t.dim() == 3 and t.stride(2) != 1 or t.stride(1) != (t.shape[2] if t.dim() == 3 else 1):
            raise ValueError("image tensor must have contiguous pixels (only the row stride may be padded)")
        pitch = t.stride(0) * t.element_size()
        return SocImg(t.data_ptr(), int(t.shape[1]), int(t.shape[0]), int(pitch), f)
    a = t
    f = fmt or infer_format(a.shape, a.dtype.type)
    if not a.flags["C_CONTIGUOUS"] and a.strides[1] != a.itemsize * (a.shape[2] if a.ndim == 3 else 1):
        raise ValueError("numpy image must have contiguous pixels")
    return SocImg(a.ctypes.data, int(a.shape[1]), int(a.shape[0]), int(a.strides[0]), f)


def _stream(stream) -> Optional[int]:
    if stream is None:
        return torch.cuda.current_stream().cuda_stream
    if isinstance(stream, torch.cuda.Stream):
        return stream.cuda_stream
    return int(stream)


def _gp(g: Globals):
    return C.byref(g)


def _ptr(t) -> Optional[int]:
    if t is None:
        return None
    if isinstance(t, torch.Tensor):
        return t.data_ptr()
    return int(t)


# ------------------------------------------------------------------------------------------------
# globals feed
# ------------------------------------------------------------------------------------------------
def globals_defaults(width: int, height: int) -> Globals:
    """Renderer defaults (renderer.cpp:72-133) for a width x height frame."""
    g = Globals()
    _check(lib().soc_globals_init_defaults(C.byref(g), width, height), "soc_globals_init_defaults")
    return g


def make_camera(position, rotation=(0.0, 0.0, 0.0), fov=90.0, near=0.1, far=1000.0) -> Camera:
    c = Camera()
    c.position[:] = [float(v) for v in position]
    c.rotation[:] = [float(v) for v in rotation]
    c.fov_degrees, c.near_clip, c.far_clip = fov, near, far
    return c


def frame_update(g: Globals, camera: Camera, width: int, height: int, delta_time: float, jitter_index: C.c_uint32) -> None:
    """One Application::update() (application.cpp:109-165)."""
    _check(lib().soc_globals_frame_update(C.byref(g), C.byref(camera), width, height, delta_time, C.byref(jitter_index)),
           "soc_globals_frame_update")


def entity(position=(0.0, 0.0, 0.0), rotation=(0.0, 0.0, 0.0), scale=(1.0, 1.0, 1.0), point_light=False,
           spot_light=False, color=(1.0, 1.0, 1.0), intensity=16.0, cut_off=20.0, outer_cut_off=30.0) -> "_abi.Entity":
    """soc_entity with the reference component defaults (src/ecs/components.hpp:55-66)."""
    e = _abi.Entity()
    e.position[:] = [float(v) for v in position]
    e.rotation[:] = [float(v) for v in rotation]
    e.scale[:] = [float(v) for v in scale]
    e.components = (_abi.ENTITY_POINT_LIGHT if point_light else 0) | (_abi.ENTITY_SPOT_LIGHT if spot_light else 0)
    e.color[:] = [float(v) for v in color]
    e.intensity, e.cut_off, e.outer_cut_off = float(intensity), float(cut_off), float(outer_cut_off)
    return e


def scene_update(g: Globals, entities):
    """Scene::update (scene.cpp:47-118): fills g's light lists; returns the (N, 4, 4) model and normal matrices
    (row index = glm column, i.e. m[c][r] like glm)."""
    n = len(entities)
    arr = (_abi.Entity * max(n, 1))(*entities)
    models = np.zeros((max(n, 1), 16), np.float32)
    normals = np.zeros((max(n, 1), 16), np.float32)
    fp = C.POINTER(C.c_float)
    _check(lib().soc_scene_update(C.byref(g), arr, n, models.ctypes.data_as(fp), normals.ctypes.data_as(fp)),
           "soc_scene_update")
    return models[:n].reshape(n, 4, 4), normals[:n].reshape(n, 4, 4)


def auto_exposure_buffer(device="cuda", exposure: float = 0.0) -> torch.Tensor:
    """Device AutoExposure block (shared.inl:39-45) as 257 int32 words: [exposure f32 bits, 256 bins]."""
    t = torch.zeros(1 + _abi.BIN_COUNT, dtype=torch.int32, device=device)
    t[0] = int(np.array([exposure], dtype=np.float32).view(np.int32)[0])
    return t


def exposure_of(ae: torch.Tensor) -> float:
    return float(ae[0:1].cpu().view(torch.float32).item())


# ------------------------------------------------------------------------------------------------
# passes (one per reference task; see include/soc_rt.h)
# ------------------------------------------------------------------------------------------------
def bloom_downsample(g, higher_mip, lower_mip, stream=None):
    _check(lib().soc_bloom_downsample(_gp(g), img(higher_mip), img(lower_mip), _stream(stream)), "bloom_downsample")


def bloom_upsample(g, lower_mip, higher_mip, stream=None):
    _check(lib().soc_bloom_upsample(_gp(g), img(lower_mip), img(higher_mip), _stream(stream)), "bloom_upsample")


def bloom_chain(g, emissive, mips, stream=None):
    arr = (SocImg * len(mips))(*[img(m) for m in mips])
    _check(lib().soc_bloom_chain(_gp(g), img(emissive), arr, len(mips), _stream(stream)), "bloom_chain")


def bloom_weighted_stage(g, emissive, mips, output, stage=0, stream=None):
    """One stage (1-4, 0 = all) of the weighted-form bloom chain (soc_bloom_weighted_stage)."""
    arr = (SocImg * len(mips))(*[img(m) for m in mips])
    _check(lib().soc_bloom_weighted_stage(_gp(g), img(emissive), arr, len(mips), img(output), int(stage),
                                          _stream(stream)), "bloom_weighted_stage")


def read_image(t, stream=None) -> np.ndarray:
    """Device image (torch tensor view) -> host numpy array of the same shape (soc_read_image), synchronised."""
    host = np.empty(tuple(t.shape), dtype=t.cpu().numpy().dtype if t.numel() == 0 else
                    {torch.uint8: np.uint8, torch.float16: np.float16, torch.float32: np.float32}[t.dtype])
    _check(lib().soc_read_image(img(t), host.ctypes.data, int(host.strides[0]), _stream(stream)), "soc_read_image")
    torch.cuda.synchronize()
    return host


def write_png(path: str, rgba8: np.ndarray) -> None:
    """(H, W, 4) uint8 host image -> PNG (soc_write_png)."""
    a = np.ascontiguousarray(rgba8, np.uint8)
    _check(lib().soc_write_png(path.encode(), a.ctypes.data, int(a.shape[1]), int(a.shape[0]), int(a.strides[0])),
           "soc_write_png")


def reload_tuning() -> None:
    """Re-read the SOC_* tuning-knob environment variables on the next launches (soc_tuning_reload)."""
    lib().soc_tuning_reload()


def write_exr(path: str, rgba16f: np.ndarray) -> None:
    """(H, W, 4) float16 host image -> OpenEXR, uncompressed HALF (soc_write_exr)."""
    a = np.ascontiguousarray(rgba16f, np.float16)
    if a.ndim != 3 or a.shape[2] != 4:
        raise ValueError("write_exr needs an (H, W, 4) float16 image")
    _check(lib().soc_write_exr(path.encode(), a.ctypes.data, int(a.shape[1]), int(a.shape[0]), int(a.strides[0])),
           "soc_write_exr")


def ssao_prepare_noise(normal, target, table, stream=None):
    _check(lib().soc_ssao_prepare_noise(img(normal), img(target), _ptr(table), _stream(stream)), "ssao_prepare_noise")


def ssao_generation(g, depth, normal, target, noise_table=None, stream=None):
    _check(lib().soc_ssao_generation(_gp(g), img(depth), img(normal), img(target), _ptr(noise_table), _stream(stream)),
           "ssao_generation")


def ssao_blur(g, ssao, target, stream=None):
    _check(lib().soc_ssao_blur(_gp(g), img(ssao), img(target), _stream(stream)), "ssao_blur")


def cloud_rendering_workspace(width: int, height: int, device="cuda") -> torch.Tensor:
    return torch.zeros(int(lib().soc_cloud_rendering_workspace_size(width, height)), dtype=torch.uint8, device=device)


def cloud_rendering(g, depth, noise, target, workspace=None, stream=None):
    _check(lib().soc_cloud_rendering(_gp(g), img(depth), img(noise), img(target), _ptr(workspace), _stream(stream)),
           "cloud_rendering")


def composition(g, target, albedo, emissive, normal, depth, ssao, shadow, clouds, d_globals=None, stream=None):
    _check(lib().soc_composition(_gp(g), _ptr(d_globals), img(target), img(albedo), img(emissive), img(normal),
                                 img(depth), img(ssao), img(shadow), img(clouds), _stream(stream)), "composition")


def histogram_scratch(device="cuda") -> torch.Tensor:
    """Zeroed scratch of soc_composition_luminance_histogram (SOC_HISTOGRAM_SCRATCH_WORDS u32)."""
    return torch.zeros(_abi.HISTOGRAM_SCRATCH_WORDS, dtype=torch.int32, device=device)


def composition_luminance_histogram(g, target, albedo, emissive, normal, depth, ssao, shadow, clouds, auto_exposure,
                                    scratch, d_globals=None, stream=None):
    """Composition + luminance histogram (bins added to auto_exposure's buckets; scratch left zeroed)."""
    _check(lib().soc_composition_luminance_histogram(
        _gp(g), _ptr(d_globals), img(target), img(albedo), img(emissive), img(normal), img(depth), img(ssao), img(shadow),
        img(clouds), _ptr(auto_exposure), _ptr(scratch), _stream(stream)), "composition_luminance_histogram")


def generate_luminance_histogram(g, hdr, auto_exposure, stream=None):
    _check(lib().soc_generate_luminance_histogram(_gp(g), img(hdr), _ptr(auto_exposure), _stream(stream)),
           "generate_luminance_histogram")


def resolve_luminance_histogram(g, auto_exposure, total_pixels=0, wide=False, stream=None):
    _check(lib().soc_resolve_luminance_histogram(_gp(g), _ptr(auto_exposure), int(total_pixels), int(bool(wide)),
                                                 _stream(stream)), "resolve_luminance_histogram")


def temporal_antialiasing(g, target, current_color, previous_color, current_velocity, previous_velocity, depth,
                          velocity_history_out=None, stream=None):
    _check(lib().soc_temporal_antialiasing(_gp(g), img(target), img(current_color), img(previous_color),
                                           img(current_velocity), img(previous_velocity), img(depth),
                                           img(velocity_history_out), _stream(stream)), "temporal_antialiasing")


def temporal_antialiasing_tone_mapping(g, target, current_color, previous_color, current_velocity, previous_velocity,
                                       depth, auto_exposure, output, velocity_history_out=None, output_format=None,
                                       stream=None):
    """TAA followed by AgX tone mapping into `output` (one launch for an RGBA8_UNORM or RGBA8_SRGB output)."""
    _check(lib().soc_temporal_antialiasing_tone_mapping(
        _gp(g), img(target), img(current_color), img(previous_color), img(current_velocity), img(previous_velocity),
        img(depth), img(velocity_history_out), _ptr(auto_exposure), img(output, output_format), _stream(stream)),
        "temporal_antialiasing_tone_mapping")


def copy_image(target, source, stream=None):
    _check(lib().soc_copy_image(img(target), img(source), _stream(stream)), "copy_image")


def tone_mapping(g, color, auto_exposure, target, target_format=None, stream=None):
    _check(lib().soc_tone_mapping(_gp(g), img(color), _ptr(auto_exposure), img(target, target_format),
                                  _stream(stream)), "tone_mapping")


def upload_globals(g, d_globals, stream=None):
    _check(lib().soc_upload_globals(_gp(g), _ptr(d_globals), _stream(stream)), "upload_globals")


def globals_device_buffer(device="cuda") -> torch.Tensor:
    return torch.zeros(C.sizeof(Globals), dtype=torch.uint8, device=device)


# ------------------------------------------------------------------------------------------------
# render graph
# ------------------------------------------------------------------------------------------------
def alloc_frame(width: int, height: int, device="cuda", output_format=FMT_RGBA8_UNORM, noise_table=True,
                bloom_output=False):
    """Device images of one frame (renderer.cpp:310-513 formats/extents). G-buffer inputs included."""
    W, H = width, height
    hw, hh = W // 2, H // 2
    f16 = dict(dtype=torch.float16, device=device)
    t = {
        "albedo": torch.zeros(H, W, 4, **f16), "emissive": torch.zeros(H, W, 4, **f16),
        "normal": torch.zeros(H, W, 4, **f16), "depth": torch.ones(H, W, dtype=torch.float32, device=device),
        "velocity": torch.zeros(H, W, 4, **f16),
        "shadow": torch.ones(4096, 4096, dtype=torch.float32, device=device),
        "noise": torch.zeros(64, 64, 4, dtype=torch.uint8, device=device),
        "bloom_mips": [torch.zeros(max(H >> i, 1), max(W >> i, 1), 4, **f16) for i in range(4)],
        "ssao": torch.zeros(hh, hw, dtype=torch.uint8, device=device),
        "ssao_blur": torch.zeros(hh, hw, dtype=torch.uint8, device=device),
        "clouds": torch.zeros(H, W, 4, dtype=torch.uint8, device=device),
        "color": torch.zeros(H, W, 4, **f16),
        "history_color": [torch.zeros(H, W, 4, **f16) for _ in range(2)],
        "history_velocity": [torch.zeros(H, W, 4, **f16) for _ in range(2)],
        "auto_exposure": auto_exposure_buffer(device),
        "d_globals": globals_device_buffer(device),
    }
    if output_format in (FMT_RGBA8_UNORM, FMT_RGBA8_SRGB):
        t["output"] = torch.zeros(H, W, 4, dtype=torch.uint8, device=device)
    elif output_format == FMT_RGBA16F:
        t["output"] = torch.zeros(H, W, 4, **f16)
    else:
        t["output"] = torch.zeros(H, W, 4, dtype=torch.float32, device=device)
    t["output_format"] = output_format
    t["ssao_noise_table"] = torch.zeros(hh * hw * 2, dtype=torch.float32, device=device) if noise_table else None
    t["bloom_output"] = torch.zeros(H, W, 4, **f16) if bloom_output else None
    t["clouds_workspace"] = cloud_rendering_workspace(W, H, device)
    return t


class Renderer:
    """Host render graph (C++ soc_renderer): the live passes of Renderer::rebuild_task_graph in order."""

    def __init__(self, frame: dict, timing: bool = False, stream=None, fused_bloom: bool = True, sky_lane: bool = True,
                 fused_tonemap: bool = True, fused_histogram: bool = True,
                 exact_bloom: bool = False, sky_split: bool = True, static_inputs: bool = False,
                 velocity_slots: bool = False, bloom_in_composition: bool = False, sky_lane_queue: str = "low"):
        """sky_lane_queue: the sky lane's hardware queue, "low" (default), "high" (sky-bound frames) or "probe" (timed
        choice over the first frames; SOC_RENDERER_SKY_LANE_HIGH / _PROBE)."""
        if sky_lane_queue not in ("low", "high", "probe"):
            raise ValueError(f"sky_lane_queue must be low, high or probe, not {sky_lane_queue!r}")
        self.frame = frame
        fi = FrameImages()
        for k in ("albedo", "emissive", "normal", "depth", "velocity", "shadow", "noise", "ssao", "ssao_blur", "clouds",
                  "color"):
            setattr(fi, k, img(frame[k]))
        for i in range(4):
            fi.bloom_mips[i] = img(frame["bloom_mips"][i])
        for i in range(2):
            fi.history_color[i] = img(frame["history_color"][i])
            fi.history_velocity[i] = img(frame["history_velocity"][i])
        fi.output = img(frame["output"], frame.get("output_format"))
        fi.ssao_noise_table = _ptr(frame.get("ssao_noise_table"))
        fi.auto_exposure = _ptr(frame["auto_exposure"])
        fi.d_globals = _ptr(frame.get("d_globals"))
        fi.bloom_output = img(frame.get("bloom_output"))
        fi.clouds_workspace = _ptr(frame.get("clouds_workspace"))
        self._fi = fi
        flags = ((_abi.RENDERER_TIMING if timing else 0) | (0 if fused_bloom else _abi.RENDERER_UNFUSED_BLOOM)
                 | (0 if sky_lane else _abi.RENDERER_SERIAL) | (0 if fused_tonemap else _abi.RENDERER_UNFUSED_TONEMAP)
                 | (0 if fused_histogram else _abi.RENDERER_UNFUSED_HISTOGRAM)
                 | (_abi.RENDERER_EXACT_BLOOM if exact_bloom else 0) | (0 if sky_split else _abi.RENDERER_NO_SKY_SPLIT)
                 | (_abi.RENDERER_STATIC_INPUTS if static_inputs else 0)
                 | (_abi.RENDERER_VELOCITY_SLOTS if velocity_slots else 0)
                 | (_abi.RENDERER_BLOOM_IN_COMPOSITION if bloom_in_composition else 0)
                 | {"low": 0, "high": _abi.RENDERER_SKY_LANE_HIGH, "probe": _abi.RENDERER_SKY_LANE_PROBE}[sky_lane_queue])
        h = lib().soc_renderer_create(C.byref(fi), flags)
        if not h:
            raise SocError(-1, lib().soc_last_error_string().decode())
        self.handle = h
        if frame.get("ssao_noise_table") is not None:
            ssao_prepare_noise(frame["normal"], frame["ssao"], frame["ssao_noise_table"], stream)

    def set_raster_scene(self, mesh, d_materials, material_count: int, visibility, workspace, shadow: bool = True):
        """Raster head (DepthPrepass / SunShadowDraw / GBufferGeneration) from a raster.MeshBuffers of device
        arrays; None clears it (the G-buffer images are inputs again)."""
        if mesh is None:
            _check(lib().soc_renderer_set_raster_scene(self.handle, None), "soc_renderer_set_raster_scene")
            self._scene = None
            return
        sc = _abi.RasterScene()
        sc.mesh = mesh.struct
        sc.materials = _ptr(d_materials)
        sc.material_count = int(material_count)
        sc.shadow = int(bool(shadow))
        sc.visibility = _ptr(visibility)
        sc.workspace = _ptr(workspace)
        self._scene = (mesh, d_materials, visibility, workspace)   # keep the arrays alive
        _check(lib().soc_renderer_set_raster_scene(self.handle, C.byref(sc)), "soc_renderer_set_raster_scene")

    def metrics_json(self, frame: int = 0) -> str:
        """The last frame's GPU-metric record (renderer.cpp:769-806) as a JSON string (needs timing and a
        completed stream)."""
        n = lib().soc_renderer_metrics_json(self.handle, int(frame), None, 0)
        if n < 0:
            _check(int(n), "soc_renderer_metrics_json")
        buf = C.create_string_buffer(int(n) + 1)
        lib().soc_renderer_metrics_json(self.handle, int(frame), buf, len(buf))
        return buf.value.decode()

    def execute(self, g: Globals, phase: int = PHASE_ALL, stream=None) -> None:
        _check(lib().soc_renderer_execute(self.handle, _gp(g), phase, _stream(stream)), "soc_renderer_execute")

    def set_exposure_pixels(self, total_pixels: int, wide: bool) -> None:
        _check(lib().soc_renderer_set_exposure_pixels(self.handle, int(total_pixels), int(bool(wide))),
               "soc_renderer_set_exposure_pixels")

    def pass_names(self):
        n = lib().soc_renderer_pass_count(self.handle)
        return [lib().soc_renderer_pass_name(self.handle, i).decode() for i in range(n)]

    def pass_groups(self):
        n = lib().soc_renderer_pass_count(self.handle)
        return [lib().soc_renderer_pass_group(self.handle, i).decode() for i in range(n)]

    def pass_ms(self):
        n = lib().soc_renderer_pass_count(self.handle)
        return [float(lib().soc_renderer_pass_ms(self.handle, i)) for i in range(n)]

    def set_pass_timing(self, index: int = -1, enable: bool = True) -> None:
        _check(lib().soc_renderer_set_pass_timing(self.handle, index, int(enable)), "soc_renderer_set_pass_timing")

    def reset_timing(self) -> None:
        _check(lib().soc_renderer_reset_timing(self.handle), "soc_renderer_reset_timing")

    def pass_stats(self):
        """[(name, group, mean_ms, frames)] over the frames recorded since reset_timing (stream must be idle)."""
        out = []
        for i, (n, gname) in enumerate(zip(self.pass_names(), self.pass_groups())):
            tot, cnt = C.c_float(0), C.c_int32(0)
            _check(lib().soc_renderer_pass_stats(self.handle, i, C.byref(tot), C.byref(cnt)), "soc_renderer_pass_stats")
            out.append((n, gname, (tot.value / cnt.value) if cnt.value else float("nan"), cnt.value))
        return out

    def pass_event_times(self, index: int, base_event, n: int = 256):
        """(start_ms, end_ms) arrays of the pass's recorded frames, oldest first, in ms after `base_event` (a recorded
        torch.cuda.Event of the same device; stream must be idle)."""
        s0, s1 = (C.c_float * n)(), (C.c_float * n)()
        m = int(lib().soc_renderer_pass_event_times(self.handle, index, C.c_void_p(base_event.cuda_event), s0, s1, n))
        if m < 0:
            _check(m, "soc_renderer_pass_event_times")
        return np.array(s0[:m], np.float64), np.array(s1[:m], np.float64)

    def side_queue(self) -> int:
        """The sky lane's hardware-queue priority (soc_renderer_side_queue): 1 high, 2 low, 0 normal, -1 not chosen."""
        return int(lib().soc_renderer_side_queue(self.handle))

    def side_queue_probe_frames(self) -> int:
        """Frames the sky-lane queue probe spans from the first call (0: no probe)."""
        return int(lib().soc_renderer_side_queue_probe_frames(self.handle))

    def add_pass(self, name: str, fn, reads=(), writes=(), phase: int = PHASE_PRE_EXPOSURE, group: str = "",
                 before: Optional[str] = None, async_compute: bool = False) -> None:
        """Register a caller pass (soc_renderer_add_pass): `fn(globals_ptr, frame_images_ptr, stream_handle)` records
        its work on the stream and returns 0. reads / writes are resource names ("SSAO_BLUR", ...) or ids; the
        pass runs before `before` (a pass name) or at the end of its phase."""
        def ids(xs):
            return [(_abi.RES[x] if isinstance(x, str) else int(x)) for x in xs]
        d = _abi.PassDesc()
        d.name, d.group, d.phase = name.encode(), group.encode(), int(phase)
        d.flags = _abi.PASS_ASYNC if async_compute else 0
        r_, w_ = ids(reads), ids(writes)
        d.read_count, d.write_count = len(r_), len(w_)
        for i, x in enumerate(r_):
            d.reads[i] = x
        for i, x in enumerate(w_):
            d.writes[i] = x

        def tramp(user, g, images, stream):
            try:
                rc = fn(g, images, stream if stream is not None else 0)   # NULL = the null stream
                return int(rc or 0)
            except Exception:   # an exception must not cross the C ABI
                return -1
        cb = _abi.PASS_CALLBACK(tramp)
        _check(lib().soc_renderer_add_pass(self.handle, C.byref(d), cb, None, before.encode() if before else None),
               "soc_renderer_add_pass")
        self._callbacks = getattr(self, "_callbacks", []) + [cb]    # keep the trampolines alive

    def pass_uses(self, index: int):
        """(reads, writes) of pass `index` as sets of resource names (ids >= 32 as 'USER<k>')."""
        rd, wr = C.c_uint64(0), C.c_uint64(0)
        _check(lib().soc_renderer_pass_uses(self.handle, index, C.byref(rd), C.byref(wr)), "soc_renderer_pass_uses")

        def names(m):
            return {(_abi.RESOURCES[b] if b < len(_abi.RESOURCES) else f"USER{b - _abi.RES_USER0}")
                    for b in range(_abi.RES_COUNT) if (m >> b) & 1}
        return names(rd.value), names(wr.value)

    def pass_dependencies(self, index: int):
        """Indices of the earlier passes pass `index` depends on (derived from the declared uses)."""
        buf = (C.c_int32 * 64)()
        n = lib().soc_renderer_pass_dependencies(self.handle, index, buf, 64)
        if n < 0:
            _check(int(n), "soc_renderer_pass_dependencies")
        return [int(buf[i]) for i in range(min(n, 64))]

    def pass_carry_dependencies(self, index: int):
        """Ring edges: indices of the PREVIOUS frame's passes this pass must follow (soc_renderer_pass_carry_dependencies)."""
        buf = (C.c_int32 * 64)()
        n = lib().soc_renderer_pass_carry_dependencies(self.handle, index, buf, 64)
        if n < 0:
            _check(int(n), "soc_renderer_pass_carry_dependencies")
        return [int(buf[k]) for k in range(n)]

    def pass_lane(self, index: int) -> int:
        return int(lib().soc_renderer_pass_lane(self.handle, index))

    def set_async(self, enable: bool) -> None:
        """Second lane: SOC_PASS_ASYNC passes (CloudRendering) on a concurrent renderer-owned stream (identical
        results)."""
        _check(lib().soc_renderer_set_async(self.handle, int(bool(enable))), "soc_renderer_set_async")

    def current_history(self) -> int:
        return int(lib().soc_renderer_current_history(self.handle))

    def velocity_slot(self) -> int:
        """With velocity_slots (SOC_RENDERER_VELOCITY_SLOTS): the history_velocity slot the NEXT frame's velocity goes
        into (its producer writes it there; TAA reads it there and the frame after as its previous velocity)."""
        return 1 - self.current_history()

    def resolved(self) -> torch.Tensor:
        return self.frame["history_color"][self.current_history()]

    STATE_VERSION = 1

    def save_state(self, path: Optional[str] = None) -> dict:
        """Checkpoint of the frame's temporal state (SURVEY.md §5 "Checkpoint / resume"; the reference keeps it in its TAA
        history images and AutoExposure, renderer.cpp:1170-1198): the previous frame's resolved colour and velocity,
        the AutoExposure block (exposure + bins) and the history slot index. Synchronises the device. With `path`,
        also written with numpy.savez (plain arrays, loadable without pickle)."""
        torch.cuda.synchronize()
        h = self.current_history()
        st = {"version": np.int32(self.STATE_VERSION), "history_index": np.int32(h),
              "history_color": self.frame["history_color"][h].cpu().numpy(),
              "history_velocity": self.frame["history_velocity"][h].cpu().numpy(),
              "auto_exposure": self.frame["auto_exposure"].cpu().numpy()}
        if path:
            np.savez(path, **st)
        return st

    def load_state(self, state) -> None:
        """Resume from save_state()'s dict or file: writes the history images and the AutoExposure block back into this
        renderer's frame and restores the history slot (soc_renderer_set_current_history). The frame's extents and
        formats must match the checkpoint's; every check runs before anything is written. The checkpoint does not hold
        the globals: the caller restores its frame_counter (TAA's accumulation factor) and its jitter index (the
        projection jitter) in the globals of the resumed frames, as the application's update() state."""
        st = dict(np.load(state, allow_pickle=False)) if isinstance(state, (str, os.PathLike)) else state
        if int(st["version"]) != self.STATE_VERSION:
            raise ValueError(f"load_state: checkpoint version {int(st['version'])}, expected {self.STATE_VERSION}")
        h = int(st["history_index"])
        if h not in (0, 1):
            raise ValueError(f"load_state: history_index {h} is not 0 or 1")
        srcs = {}
        for key in ("history_color", "history_velocity"):
            dst = self.frame[key][h]
            src = np.asarray(st[key])
            if tuple(src.shape) != tuple(dst.shape) or src.dtype != np.float16:
                raise ValueError(f"load_state: {key} {src.shape} {src.dtype} does not match the frame's {tuple(dst.shape)}")
            srcs[key] = src
        ae = np.asarray(st["auto_exposure"])
        if ae.shape != tuple(self.frame["auto_exposure"].shape) or ae.dtype != np.int32:
            raise ValueError(f"load_state: AutoExposure block {ae.shape} {ae.dtype} does not match the frame's "
                             f"{tuple(self.frame['auto_exposure'].shape)} int32")
        # every check passed: nothing of the frame is written before this point
        for key, src in srcs.items():
            self.frame[key][h].copy_(torch.from_numpy(np.ascontiguousarray(src)))
        self.frame["auto_exposure"].copy_(torch.from_numpy(np.ascontiguousarray(ae)))
        _check(lib().soc_renderer_set_current_history(self.handle, h), "soc_renderer_set_current_history")
        torch.cuda.synchronize()

    def close(self):
        if getattr(self, "handle", None):
            lib().soc_renderer_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
