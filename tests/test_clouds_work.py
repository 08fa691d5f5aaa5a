"""CloudRendering's compute roofline inputs and the atmosphere's optical-depth table, on the CPU.

* tools/clouds_flops.py: the per-function FLOP / transcendental / tap tallies of the reference GLSL
  (cloud_rendering.inl:92-481) times the instrumented oracle's entry counts; the committed profile the bench line reads
  (profiles/*clouds_flops.json) is consistent with the tally function.
* tools/od_lut_check.py: the secondary-ray optical-depth table the GPU atmosphere interpolates (clouds.hip
  clouds_od_lut) against marching the ray (cloud_rendering.inl:399-423): the attenuation differs by at most 1e-3
  anywhere the table serves and 5e-5 for the reference sun's mu > 0.9.
"""
import glob
import json
import os
import subprocess
import sys

import numpy as np

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "tools"))


def test_clouds_tally_from_oracle_counters(oracle):
    import clouds_flops
    from helpers import terrain_inputs
    W, H = 160, 90
    g, gb = terrain_inputs(W, H, elapsed=10.0)
    out = np.zeros((H, W, 4), np.uint8)
    oracle.cloud_rendering(g, gb["depth"], gb["noise"], out)
    c = oracle.clouds_counters()
    assert c["pixels"] == W * H
    # the sky test is the bilinear depth at ray_uv = pixel / (resolution - 1) (:445-460), not the texel itself
    assert c["sky_pixels"] > 0 and abs(c["sky_pixels"] - int((gb["depth"] == 1.0).sum())) <= 0.02 * W * H
    assert c["noise_taps"] == 8 * c["get_clouds_full"]           # 4 octaves x 2 taps
    assert c["get_clouds"] == 24 * c["cloud_marches"] + 10 * c["dense_steps"]
    t = clouds_flops.tally(c)
    # every sky pixel at least enters the atmosphere; a full one costs 3664 FLOP + 498 transcendentals (:360-438)
    assert t["flops"] >= c["sky_pixels"] * (58 + 3664) and t["transcendentals"] >= c["atmosphere_full"] * 498
    assert t["taps"] == c["pixels"] + c["noise_taps"]


def test_committed_clouds_profile_matches_the_tally():
    import clouds_flops
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*clouds_flops.json")))
    assert files
    d = json.load(open(files[-1]))
    for name, cfg in d["configs"].items():
        t = clouds_flops.tally(cfg["counters"])
        assert t["flops"] == cfg["flops"] and t["transcendentals"] == cfg["transcendentals"], name
        r = clouds_flops.roofline(t, cfg["gpu_standalone"]["avg_launch_us"])
        assert 0.0 < r["frac"] < 1.0 and 0.0 < r["frac_of_floor"] < 1.0


def test_od_table_accuracy():
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "od_lut_check.py"), "--samples", "60000"],
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    line = [ln for ln in p.stdout.splitlines() if "secondary attenuation error" in ln][0]
    mx = float(line.split("max")[-1])
    up = float([ln for ln in p.stdout.splitlines() if "mu > 0.9" in ln][0].split("max")[-1])
    assert mx <= 1e-3 and up <= 5e-5, p.stdout


def test_sky_table_accuracy():
    """The sky-view table's interpolation error (tools/sky_table_check.py, float64, the C3 and C4 view frusta sampled
    every 24 pixels): well under one RGBA8 level of the atmosphere colour (0.15 measured, at the grazing rows)."""
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "sky_table_check.py"), "--sub", "24"],
                       capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-2000:]
    worst = float(p.stdout.strip().splitlines()[-1].split()[2])
    assert worst < 0.5, p.stdout
