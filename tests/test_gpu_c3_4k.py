"""The benchmarked configurations at their own size: bench.py's default command (C3) and its sky-heavy terrain line
(C4, f_sky ~0.5: CloudRendering dominates) rendered by the render graph at 3840x2160 and compared with the oracle's
frame of the same inputs.

The inputs come from bench.build_inputs, exactly as the bench builds them: the Sponza-proxy mesh rasterised once by
the HIP rasteriser (mip-mapped anisotropic textures), the 4096^2 sun shadow map, the C3 globals (elapsed 10 s,
frame counter 2). The renderer runs the bench's graph: the concurrent sky lane, the sky split, the AO-first issue
order, the fused composition + histogram and the fused TAA + tone map. Two frames (the second one resolves TAA
against the first one's history). Bounds: helpers.frame_parity: every pass within its SURVEY.md §8d
tolerance on every pixel given the GPU's own inputs to it, SSAO / clouds against the oracle's with a hard maximum, and
the end-to-end colour, framebuffer and exposure at §8d's bounds; the achieved errors are printed in the session
summary. Reference: renderer.cpp:1024-1217."""
import numpy as np
import pytest
import torch

from helpers import frame_parity, host_frame

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("config,sky_range", [("c3", (0.05, 0.2)), ("c4", (0.4, 0.65))])
def test_bench_frame_4k_vs_oracle(soc, oracle, config, sky_range):
    import bench
    W, H = 3840, 2160
    dev = torch.device("cuda", 0)
    g, gb, shadow, noise, sc, fr = bench.build_inputs(config, "mesh", W, H, 0, dev)
    r = soc.Renderer(fr, static_inputs=True)          # the bench's renderer flags
    r.set_exposure_pixels(W * H, False)
    assert r.pass_names() == ["BloomDownsample - 0+1", "BloomDownsample - 2+3", "BloomUpsample - 3+2",
                              "BloomUpsample - 1+0", "SSAOGeneration", "SSAOBlur", "CloudRendering",
                              "SkyCompose", "Composition+GenerateLuminanceHistogram", "LuminanceHistogramFold",
                              "ResolveLuminanceHistogram", "TemporalAntiAliasing+ToneMapping"]
    assert r.pass_lane(r.pass_names().index("CloudRendering")) == 1
    f_sky = float((gb["depth"] == 1.0).mean())
    assert sky_range[0] < f_sky < sky_range[1], f_sky
    hf = host_frame(W, H, {**gb, "shadow": shadow, "noise": noise})
    ae = soc.AutoExposure()
    hist = 0
    for f in range(2):
        e0 = soc.exposure_of(fr["auto_exposure"])
        r.execute(g)
        hf["emissive"][...] = gb["emissive"]          # the bench writes bloom into bloom_output (emissive kept)
        hist = oracle.frame(g, hf, ae, hist=hist)
        torch.cuda.synchronize()
        assert r.current_history() == hist
        frame_parity(soc, oracle, g, fr, hf, ae, hist, f"{config} 3840x2160 frame {f}", e0)
    r.close()
