"""bench.py's readers of the committed profile tables (CPU): the HBM traffic of the headline kernels and the
SSAOGeneration texture-path ceiling come from the same workload's rocprofv3 tables under profiles/."""
import os
import sys

from conftest import ROOT

sys.path.insert(0, ROOT)


def test_pmc_traffic_of_the_headline_kernels():
    import bench
    comp, src = bench.pmc_traffic("composition_pair<true, false, 3>", 3840, 2160, "mesh")
    ssao, _ = bench.pmc_traffic(bench.SSAO_KERNEL, 3840, 2160, "mesh")
    assert src and os.path.exists(os.path.join(ROOT, src))
    algo = bench.algorithmic_bytes(3840, 2160, 0.0)
    # measured HBM bytes per launch: at least the algorithmic minimum's order, no more than a few times it
    assert 0.9 * algo["SSAOGeneration"] < ssao < 3.5 * algo["SSAOGeneration"]
    assert comp > 0.9 * 40.25 * 3840 * 2160
    # a template-signature change still finds the one instantiation of that kernel
    assert bench.pmc_traffic("ssao_kernel<true, true, true, 7>", 3840, 2160, "mesh")[0] == ssao
    # another workload's table is not used
    assert bench.pmc_traffic(bench.SSAO_KERNEL, 1920, 1080, "mesh") == (None, None)


def test_ssao_gather_bound():
    import bench
    gb = bench.ssao_gather_bound(3840, 2160, "mesh", 170.0)
    assert gb is not None
    assert gb["us_if_coalesced"] < gb["us_if_scattered"]
    # 26 taps x 2 row pairs per wave of non-sky half-res pixels (plus the centre / normal / noise loads)
    waves = 1920 * 1080 // 64
    assert 52 * 0.8 * waves < gb["wave_loads_per_launch"] < 60 * waves
    assert abs(gb["frac_of_scattered_rate"] - gb["us_if_scattered"] / 170.0) < 1e-3
    assert bench.ssao_gather_bound(1920, 1080, "mesh", 50.0) is None


def test_cpu_baseline_per_pass_medians():
    """The CPU baseline: the oracle frame timed per frame and per pass (median after a warm-up)."""
    import bench
    from helpers import sponza_inputs
    W, H = 64, 36
    g, gb = sponza_inputs(W, H, elapsed=10.0, frame_counter=2)
    host = {k: gb[k] for k in ("albedo", "emissive", "normal", "velocity", "depth", "shadow", "noise")}
    cb = bench.cpu_baseline(W, H, host, g)
    assert cb["kind"] == "port" and cb["value"] > 0 and cb["cores"] >= 1
    assert set(cb["ms_per_pass_median"]) == {"Bloom", "SSAOGeneration", "SSAOBlur", "CloudRendering", "Composition",
                                            "GenerateLuminanceHistogram", "ResolveLuminanceHistogram",
                                            "TemporalAntiAliasing", "ToneMapping"}
    assert sum(cb["ms_per_pass_median"].values()) <= 1.5 * cb["ms_per_frame_median"] + 1.0
