"""The benchmarked configurations at their own size: bench.py's default command (C3), its sky-heavy terrain line
(C4, f_sky ~0.5: CloudRendering dominates) at 3840x2160 and its C2 line (the same Sponza-proxy mesh and HIP-rastered
4096^2 sun shadow map at 1920x1080: deferred lighting + the shadow map, composition.inl:164-173,
sun_shadow_draw.inl:27-91) rendered by the render graph and compared with the oracle's frame of the same inputs.
`test_c3_linear_tonemap_tolerance` checks SURVEY.md §8d's final bound on the headline frame: the tone map into an
RGBA32F target, linear RGB |d| <= 2e-3 on >= 99.9 % of the values.

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


@pytest.mark.parametrize("config,sky_range", [("c3", (0.05, 0.2)), ("c4", (0.4, 0.65)), ("c2", (0.05, 0.2))])
def test_bench_frame_4k_vs_oracle(soc, oracle, config, sky_range):
    import bench
    W, H = (1920, 1080) if config == "c2" else (3840, 2160)
    dev = torch.device("cuda", 0)
    g, gb, shadow, noise, sc, fr = bench.build_inputs(config, "mesh", W, H, 0, dev)
    # the bench's renderer flags: static inputs, the velocity history by slot rotation (the resident velocity in both
    # history slots, as bench.py sets it up; the oracle's frame is given the same history) and the bloom chain's last
    # stage inside Composition
    for hv in fr["history_velocity"]:
        hv.copy_(fr["velocity"])
    # the bench's sky-lane queue for the config (bench.py --sky-lane-queue auto): low at C3, high (with the sky-bound
    # variants: the bloom's last stage inside Composition, the clouds' doubled density grid, hoisted classification) at C2 / C4
    r = soc.Renderer(fr, static_inputs=True, velocity_slots=True, bloom_in_composition=True,
                     sky_lane_queue="low" if config == "c3" else "high")
    r.set_exposure_pixels(W * H, False)
    assert r.pass_names() == ["BloomDownsample - 0+1", "BloomDownsample - 2+3", "BloomUpsample - 3+2",
                              "BloomUpsample - 1+0", "SSAOGeneration", "SSAOBlur", "CloudRendering",
                              "SkyCompose", "Composition+GenerateLuminanceHistogram", "LuminanceHistogramFold",
                              "ResolveLuminanceHistogram", "TemporalAntiAliasing+ToneMapping"]
    assert r.pass_lane(r.pass_names().index("CloudRendering")) == 1
    f_sky = float((gb["depth"] == 1.0).mean())
    assert sky_range[0] < f_sky < sky_range[1], f_sky
    hf = host_frame(W, H, {**gb, "shadow": shadow, "noise": noise})
    for hv in hf["history_velocity"]:
        hv[...] = gb["velocity"]
    ae = soc.AutoExposure()
    hist = 0
    for f in range(2):
        e0 = soc.exposure_of(fr["auto_exposure"])
        r.execute(g)
        assert r.side_queue() == (2 if config == "c3" else 1)
        hf["emissive"][...] = gb["emissive"]          # the bench writes bloom into bloom_output (emissive kept)
        hist = oracle.frame(g, hf, ae, hist=hist)
        # where Composition computed the bloom in-kernel (a frame with a high-priority sky lane), its output
        # materialised from the GPU's mip1 by the chain's own last stage (the same bits:
        # test_bloom_in_composition_bit_identical) for frame_parity's conditional checks; else the same values again
        soc.bloom_weighted_stage(g, fr["emissive"], fr["bloom_mips"], fr["bloom_output"], stage=4)
        torch.cuda.synchronize()
        assert r.current_history() == hist
        frame_parity(soc, oracle, g, fr, hf, ae, hist, f"{config} {W}x{H} frame {f}", e0)
    if config == "c2":   # the benched C2 shadow map is the HIP-rastered 4096^2 one, and it reaches the lit pixels
        assert shadow.shape == (4096, 4096) and (shadow < 1.0).any()
    r.close()


def test_c3_linear_tonemap_tolerance(soc, oracle):
    """SURVEY.md §8d, "final tone-mapped linear RGB |d| <= 2e-3 for 99.9 %": the C3 bench frame with the tone map
    writing linear RGBA32F (tone_mapping.inl:145-176 before the swapchain's encode), two frames, against the oracle.
    Asserted: the tone map given the GPU's own resolved colour and exposure within 2e-3 on every value, the end-to-end
    output within 2e-3 on >= 99.9 % of ALL pixels (§8d as written; round 5 met it only on the pixels whose upstream inputs
    equal the oracle's: 99.47 % over all, every miss a sky pixel whose clouds texel was a level off; round 6's noise hash
    and clouds chain follow the oracle's roundings), and on >= 99.9 % of the pixels whose upstream inputs equal the
    oracle's (the AO texels and clouds texels of frame_parity, dilated by the TAA footprint, over both frames)."""
    import bench
    from helpers import PARITY_REPORTS
    W, H = 3840, 2160
    dev = torch.device("cuda", 0)
    g, gb, shadow, noise, sc, fr = bench.build_inputs("c3", "mesh", W, H, 0, dev, output_format=soc.FMT_RGBA32F)
    assert fr["output"].dtype == torch.float32
    r = soc.Renderer(fr, static_inputs=True)
    r.set_exposure_pixels(W * H, False)
    hf = host_frame(W, H, {**gb, "shadow": shadow, "noise": noise}, output_format=soc.FMT_RGBA32F)
    ae = soc.AutoExposure()
    hist = 0
    upstream_any = np.zeros((H, W), bool)
    for f in range(2):
        e0 = soc.exposure_of(fr["auto_exposure"])
        r.execute(g)
        hf["emissive"][...] = gb["emissive"]
        hist = oracle.frame(g, hf, ae, hist=hist)
        torch.cuda.synchronize()
        masks = {}
        frame_parity(soc, oracle, g, fr, hf, ae, hist, f"c3 {W}x{H} RGBA32F frame {f}", e0, check=False, masks=masks)
        PARITY_REPORTS.pop()
        up = masks["upstream"]
        # TAA reads the 3x3 colour neighbourhood and the reprojected history (velocity of a few pixels at most here)
        for dy in range(-3, 4):
            for dx in range(-3, 4):
                upstream_any |= np.roll(np.roll(up, dy, 0), dx, 1)
        out = fr["output"].cpu().numpy()[..., :3].astype(np.float64)
        ref = hf["output"][..., :3].astype(np.float64)
        # conditional: the oracle's tone map of the GPU's resolved colour with the GPU's exposure
        ae2 = soc.AutoExposure()
        ae2.exposure = soc.exposure_of(fr["auto_exposure"])
        tc = np.zeros((H, W, 4), np.float32)
        oracle.tone_mapping(g, fr["history_color"][hist].cpu().numpy(), ae2, tc, soc.FMT_RGBA32F)
        dc = np.abs(out - tc[..., :3])
        d = np.abs(out - ref).max(axis=-1)
        ok = d <= 2e-3
        rep = {"label": f"c3 3840x2160 linear tone map (RGBA32F) frame {f}",
               "cond_max": float(dc.max()),
               "e2e_within_2e-3": float(ok.mean()), "e2e_nonsky_within_2e-3": float(ok[~masks["sky"]].mean()),
               "e2e_within_2e-3_where_upstream_equal": float(ok[~upstream_any].mean()),
               "upstream_differs_dilated": float(upstream_any.mean()),
               "e2e_p99.9": float(np.percentile(d, 99.9)), "e2e_max": float(d.max()),
               "exposure_delta": abs(soc.exposure_of(fr["auto_exposure"]) - ae.exposure)}
        PARITY_REPORTS.append(rep)
        assert np.isfinite(out).all()
        assert rep["cond_max"] <= 2e-3, rep
        assert rep["e2e_within_2e-3_where_upstream_equal"] >= 0.999, rep
        assert rep["e2e_within_2e-3"] >= 0.999, rep
        assert rep["exposure_delta"] <= 1e-5, rep
    r.close()
