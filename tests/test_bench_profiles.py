"""bench.py's readers of the committed profile tables (CPU): the HBM traffic of the headline kernels and the
SSAOGeneration VALU issue time come from the same workload's rocprofv3 tables under profiles/."""
import os
import sys

from conftest import ROOT

sys.path.insert(0, ROOT)


def test_pmc_traffic_of_the_headline_kernels():
    import bench
    comp, src = bench.pmc_traffic("composition_pair<true, false, 7, false>", 3840, 2160, "mesh")
    ssao, _ = bench.pmc_traffic(bench.SSAO_KERNEL, 3840, 2160, "mesh")
    assert src and os.path.exists(os.path.join(ROOT, src))
    algo = bench.algorithmic_bytes(3840, 2160, 0.0)
    # measured HBM bytes per launch: at least the algorithmic minimum's order, no more than a few times it
    assert 0.9 * algo["SSAOGeneration"] < ssao < 3.5 * algo["SSAOGeneration"]
    assert comp > 0.9 * 40.25 * 3840 * 2160
    # a template-signature change still finds the one instantiation of that kernel, or the one whose arguments extend
    # (or are extended by) the name asked for; an ambiguous name finds none
    assert bench.pmc_traffic("ssao_pipe_kernel<64, 16, 32, true, 0>", 3840, 2160, "mesh")[0] == ssao
    assert bench.pmc_traffic("composition_pair<true, false, 7, false, 1>", 3840, 2160, "mesh")[0] == comp
    assert bench.pmc_traffic("composition_pair", 3840, 2160, "mesh")[0] is None   # two instantiations in the table
    # another workload's table is not used
    assert bench.pmc_traffic(bench.SSAO_KERNEL, 1920, 1080, "mesh") == (None, None)


def test_ssao_bounds():
    """The VALU issue model of the current kernels (profiles/*valu_model.json)."""
    import bench
    vb = bench.valu_bound(bench.SSAO_KERNEL, 110.0)
    assert vb is not None and 20.0 < vb["valu_issue_us"] < 110.0
    assert abs(vb["frac_of_launch"] - vb["valu_issue_us"] / 110.0) < 1e-3
    assert bench.valu_bound("no_such_kernel", 1.0) is None


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
