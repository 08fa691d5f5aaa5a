"""C-ABI checks (CPU only): the HIP library loads, exports every function include/soc_rt.h declares, and
its struct layouts match the ctypes mirror. No kernel is launched."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "soc_rt.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = re.sub(r"//[^\n]*", "", src)
    names = set(re.findall(r"\b(soc_[a-z0-9_]+)\s*\(", src))
    return sorted(names)


def test_header_declares_the_pass_api():
    names = declared_functions()
    for must in ("soc_composition", "soc_ssao_generation", "soc_ssao_blur", "soc_bloom_downsample", "soc_bloom_upsample",
                 "soc_cloud_rendering", "soc_generate_luminance_histogram", "soc_resolve_luminance_histogram",
                 "soc_temporal_antialiasing", "soc_tone_mapping", "soc_last_error_string", "soc_renderer_execute"):
        assert must in names


def test_every_declared_symbol_is_exported(soc):
    lib = soc.lib()
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing


def test_ctypes_table_covers_header():
    from soc_real_time_renderer_amd import _abi
    assert set(declared_functions()) == set(_abi.FUNCTIONS)


def test_renderer_flags_match_header():
    """Every SOC_RENDERER_* flag bit of the header has its ctypes constant with the same value (and the bits are
    distinct), so a Python caller sets the flag the C side tests."""
    from soc_real_time_renderer_amd import _abi
    src = open(HEADER).read()
    flags = {m.group(1): int(m.group(2)) for m in re.finditer(r"#define SOC_RENDERER_([A-Z_]+)\s+(\d+)", src)}
    flags.pop("TIMING_RING")   # a ring length, not a flag
    assert {"STATIC_INPUTS", "VELOCITY_SLOTS", "SERIAL"} <= set(flags)
    for name, value in flags.items():
        assert getattr(_abi, "RENDERER_" + name) == value, name
        assert value & (value - 1) == 0, name
    assert len(set(flags.values())) == len(flags)


@pytest.mark.parametrize("name", ["soc_img", "soc_globals", "soc_sun_info", "soc_point_light", "soc_spot_light",
                                  "soc_auto_exposure", "soc_camera", "soc_frame_images", "soc_mesh", "soc_material",
                                  "soc_raster_scene"])
def test_struct_sizes(soc, name):
    from soc_real_time_renderer_amd import _abi
    assert soc.lib().soc_abi_sizeof(name.encode()) == C.sizeof(_abi.STRUCTS[name])


def test_struct_offsets(soc):
    from soc_real_time_renderer_amd import _abi
    lib = soc.lib()
    checked = 0
    for tname, st in _abi.STRUCTS.items():
        for fname, _ in st._fields_:
            off = lib.soc_abi_offsetof(tname.encode(), fname.encode())
            assert off == getattr(st, fname).offset, (tname, fname)
            checked += 1
    assert checked > 100


def test_abi_version_and_arch(soc):
    lib = soc.lib()
    assert lib.soc_abi_version() == 1
    assert lib.soc_device_arch() == b"gfx950"


def test_argument_errors_without_gpu(soc):
    """Validation happens before any HIP call: bad images return SOC_E_INVALID_ARG with a message."""
    g = soc.globals_defaults(64, 36)
    bad = soc.SocImg(None, 0, 0, 0, 0)
    rc = soc.lib().soc_ssao_blur(C.byref(g), bad, bad, None)
    assert rc == soc._abi.SOC_E_INVALID_ARG
    assert b"soc_ssao_blur" in soc.lib().soc_last_error_string()
    with pytest.raises(soc.SocError):
        soc.cloud_rendering(g, None, None, None, stream=0)


def test_block_shape_over_the_launch_bound_is_rejected_without_gpu(soc):
    """The launch-geometry check (soc_check_block_shape; every launcher applies it with its kernel's bound before the
    launch): round 3's 64 x 16 SSAO-blur block against the kernel's 256-lane bound is refused on the host with
    SOC_E_INVALID_ARG, the shapes the library launches pass, an empty block is refused."""
    from soc_real_time_renderer_amd import _abi
    lib = soc.lib()
    assert lib.soc_check_block_shape(256, 64, 16, 1) == _abi.SOC_E_INVALID_ARG
    assert b"1024 lanes" in lib.soc_last_error_string() and b"256" in lib.soc_last_error_string()
    assert lib.soc_check_block_shape(256, 64, 4, 1) == 0
    assert lib.soc_check_block_shape(1024, 1024, 1, 1) == 0       # the SSAO tile kernel
    assert lib.soc_check_block_shape(512, 512, 1, 1) == 0         # clouds_sunvis
    assert lib.soc_check_block_shape(512, 1024, 1, 1) == _abi.SOC_E_INVALID_ARG
    assert lib.soc_check_block_shape(256, 0, 4, 1) == _abi.SOC_E_INVALID_ARG
    assert lib.soc_check_block_shape(256, -1, 4, 1) == _abi.SOC_E_INVALID_ARG


def test_every_launch_goes_through_the_geometry_check():
    """No kernel is launched with a bare triple-chevron outside the checked launch() helper (soc_internal.hpp), and
    every 256-lane kernel declares its bound through the shared kWorkgroup constant."""
    import glob
    import re
    csrc = os.path.join(ROOT, "soc_real_time_renderer_amd", "csrc")
    for f in glob.glob(os.path.join(csrc, "*.hip")) + glob.glob(os.path.join(csrc, "*.cpp")):
        src = open(f).read()
        assert "<<<" not in src, f
        assert not re.search(r"__launch_bounds__\(\s*\d+\s*\)", src), f
    assert "k<<<grid, block, lds, s>>>" in open(os.path.join(csrc, "soc_internal.hpp")).read()


def test_library_is_a_gfx950_code_object():
    """The in-tree .so carries a gfx950 offload bundle (built by __graft_entry__.build)."""
    so = os.path.join(ROOT, "soc_real_time_renderer_amd", "lib", "libsoc_rt.so")
    data = open(so, "rb").read()
    assert b"gfx950" in data
    assert b"__hip_fatbin" in data or b"HIP_FATBIN" in data or b".hip_fatbin" in data


def test_raster_and_output_argument_errors_without_gpu(soc):
    """The raster / Hi-Z / height-to-normal / output entry points validate before any HIP call."""
    from soc_real_time_renderer_amd import _abi
    lib = soc.lib()
    g = soc.globals_defaults(64, 36)
    vp = (C.c_float * 16)()
    bad = soc.SocImg(None, 0, 0, 0, 0)
    E_ARG, E_SHAPE = _abi.SOC_E_INVALID_ARG, _abi.SOC_E_SHAPE
    assert lib.soc_raster_visibility(None, vp, 1, None, 64, 36, 1, None, None) == E_ARG
    mesh = _abi.Mesh()
    assert lib.soc_raster_visibility(C.byref(mesh), vp, 1, None, 64, 36, 1, None, None) == E_ARG
    assert b"soc_raster_visibility" in lib.soc_last_error_string()
    assert lib.soc_raster_depth(C.byref(mesh), vp, 2, 1.25, 1.75, bad, None, None) == E_ARG
    assert lib.soc_gbuffer_resolve(C.byref(g), C.byref(mesh), None, 1, None, bad, bad, bad, bad, bad, None, None) == E_ARG
    assert lib.soc_generate_hiz(C.byref(g), bad, None, 13, 0, None, None) == E_ARG
    h = np.zeros((8, 8, 4), np.uint8)
    n = np.zeros((8, 4, 4), np.float16)
    assert lib.soc_height_to_normal(soc.img(h), soc.img(n), None) == E_SHAPE
    assert lib.soc_write_png(b"/tmp/x.png", None, 4, 4, 16) == E_ARG
    assert lib.soc_read_image(bad, None, 0, None) == E_ARG
    assert lib.soc_renderer_set_raster_scene(None, None) == E_ARG
    assert lib.soc_raster_workspace_size(-1, 0) == 0
