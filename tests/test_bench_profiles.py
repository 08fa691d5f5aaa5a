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
