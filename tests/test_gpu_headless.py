"""The compiled C++ consumer of include/soc_rt.h (tools/headless/soc_headless.cpp): the caller shape of SURVEY.md
§8b (a host frame loop -> render graph -> framebuffer in a host image, renderer.cpp:929-1235 <- application.cpp:89-107)
without Python or ctypes. It creates a renderer over caller-owned device images, adds a caller pass, runs PRE / POST
per frame and writes the framebuffer; the test runs the same frames through the Python binding and requires the
same framebuffer bytes and the same exposure."""
import json
import os
import subprocess

import numpy as np
import pytest
import torch

from helpers import globals_for

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "soc_real_time_renderer_amd", "build", "soc_headless")


def test_headless_binary_is_built_and_checks_its_arguments():
    """CPU: the consumer links against libsoc_rt / libsoc_scene and rejects a bad command line (before any HIP call)."""
    assert os.path.exists(EXE), "build() makes soc_headless"
    p = subprocess.run([EXE], capture_output=True, text=True, timeout=60)
    assert p.returncode == 2 and "usage" in p.stderr


@pytest.mark.gpu
def test_headless_consumer_matches_the_python_binding(soc, tmp_path):
    from soc_real_time_renderer_amd import scene
    W, H, frames = 320, 180, 3
    png, raw = str(tmp_path / "frame.png"), str(tmp_path / "frame.raw")
    p = subprocess.run([EXE, str(W), str(H), str(frames), png, raw], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    line = json.loads(p.stdout.strip().splitlines()[-1])
    assert line["caller_pass_calls"] == frames and line["frames"] == frames
    assert len(line["metrics"]["groups"]) == 12 and "RawAO" in line["metrics"]["passes"]   # renderer.cpp:558-588 names
    out_cpp = np.fromfile(raw, np.uint8).reshape(H, W, 4)
    from PIL import Image
    assert np.array_equal(np.asarray(Image.open(png).convert("RGBA")), out_cpp)

    # the same frames through the Python binding
    g = globals_for(W, H)
    gb = scene.gbuffer(g, W, H)
    fr = soc.alloc_frame(W, H, "cuda")
    for k in ("albedo", "emissive", "normal", "velocity", "depth"):
        fr[k].copy_(torch.from_numpy(gb[k]))
    fr["shadow"] = torch.from_numpy(scene.shadow_map(g, 1024)).cuda()
    fr["noise"].copy_(torch.from_numpy(scene.noise_texture()))
    r = soc.Renderer(fr, timing=True)
    r.add_pass("RawAO", lambda gp, im, s: soc.copy_image(fr["ssao_blur"], fr["ssao"], s), reads=["SSAO"],
               writes=["SSAO_BLUR"], before="Composition+GenerateLuminanceHistogram", group="Ambient Occlusion")
    for _ in range(frames):
        r.execute(g, soc.PHASE_PRE_EXPOSURE)
        r.execute(g, soc.PHASE_POST_EXPOSURE)
    torch.cuda.synchronize()
    assert np.array_equal(fr["output"].cpu().numpy(), out_cpp)
    assert np.float32(soc.exposure_of(fr["auto_exposure"])) == np.float32(line["exposure"])
    assert r.current_history() == line["history"]
    r.close()
