"""Caller passes in the render graph, on the GPU (soc_renderer_add_pass; the Daxa add_task of
renderer.cpp:1103-1117 with a uses block like composition.inl:10-21).

A pass registered between SSAOBlur and Composition that declares reads {SSAO}, writes {SSAO_BLUR} and copies
the raw AO over the blurred one must change the composition exactly as the oracle's composition with the raw
AO; a SOC_PASS_ASYNC caller pass runs on the second lane and its consumer on the caller's stream sees its
result."""
import numpy as np
import pytest
import torch

from helpers import f16_close, sponza_inputs

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _frame(soc, W, H, gb):
    fr = soc.alloc_frame(W, H, DEV)
    for k in ("albedo", "emissive", "normal", "velocity", "depth"):
        fr[k].copy_(torch.from_numpy(gb[k]))
    fr["shadow"] = torch.from_numpy(gb["shadow"]).to(DEV)
    fr["noise"].copy_(torch.from_numpy(gb["noise"]))
    return fr


def test_caller_pass_between_ssao_blur_and_composition(soc, oracle):
    W, H = 256, 128
    g, gb = sponza_inputs(W, H, elapsed=10.0)
    fr = _frame(soc, W, H, gb)
    r = soc.Renderer(fr)
    calls = []

    def raw_ao(gp, images, stream):
        calls.append(stream)
        soc.copy_image(fr["ssao_blur"], fr["ssao"], stream)
        return 0
    r.add_pass("RawAO", raw_ao, reads=["SSAO"], writes=["SSAO_BLUR"], before="Composition+GenerateLuminanceHistogram",
               group="Ambient Occlusion")
    r.execute(g)
    torch.cuda.synchronize()
    assert len(calls) == 1
    ssao = fr["ssao"].cpu().numpy()
    assert np.array_equal(fr["ssao_blur"].cpu().numpy(), ssao)
    # the oracle's composition of the GPU's own inputs with the RAW AO
    color = np.zeros((H, W, 4), np.float16)
    oracle.composition(g, color, gb["albedo"], fr["emissive"].cpu().numpy(), gb["normal"], gb["depth"], ssao,
                       gb["shadow"], fr["clouds"].cpu().numpy())
    ok = f16_close(fr["color"].cpu().numpy(), color)
    assert ok.mean() >= 0.999, ok.mean()
    r.close()


def test_async_caller_pass_and_its_consumer(soc):
    W, H = 256, 128
    g, gb = sponza_inputs(W, H, elapsed=10.0)
    fr = _frame(soc, W, H, gb)
    r = soc.Renderer(fr)
    mask = torch.zeros(H, W, dtype=torch.float32, device=DEV)
    seen = torch.zeros(H, W, dtype=torch.float32, device=DEV)
    U = soc._abi.RES_USER0
    r.add_pass("DepthCopy", lambda gp, im, s: soc.copy_image(mask, fr["depth"], s), reads=["DEPTH"], writes=[U],
               before="SSAOGeneration", async_compute=True)
    r.add_pass("UseCopy", lambda gp, im, s: soc.copy_image(seen, mask, s), reads=[U], writes=[U + 1],
               before="Composition+GenerateLuminanceHistogram")
    names = r.pass_names()
    assert r.pass_lane(names.index("DepthCopy")) == 1 and r.pass_lane(names.index("UseCopy")) == 0
    for _ in range(2):
        r.execute(g)
    torch.cuda.synchronize()
    assert torch.equal(seen, fr["depth"])
    r.close()


@pytest.mark.parametrize("where", ["post", "pre"])
def test_aborted_frame_leaves_next_frame_exact(soc, oracle, where):
    """A caller pass that returns an error aborts its frame after the second lane was forked: the call
    returns the error, joins the second lane, and drops the frame's partial histograms (the composition's and the
    sky lane's bins, which the resolve would have folded and cleared). The next frame then equals the oracle's frame
    that follows the last COMPLETED frame: same colour, framebuffer and exposure, and the TAA history of that frame.
    post: the failing pass sits before the resolve (every PRE pass ran, bins in the scratch); pre: before the
    composition (the sky lane's bins only)."""
    from helpers import host_frame, terrain_inputs
    W, H = 320, 180
    g, gb = terrain_inputs(W, H, elapsed=10.0)       # half the frame is sky: the sky lane bins many pixels
    fr = _frame(soc, W, H, gb)
    r = soc.Renderer(fr)
    calls = []

    def flaky(gp, images, stream):
        calls.append(1)
        return -7 if len(calls) == 2 else 0
    if where == "post":
        r.add_pass("Flaky", flaky, reads=["COLOR"], writes=[soc._abi.RES_USER0], phase=soc.PHASE_POST_EXPOSURE,
                   before="ResolveLuminanceHistogram")
    else:
        r.add_pass("Flaky", flaky, reads=["SSAO_BLUR"], writes=[soc._abi.RES_USER0],
                   before="Composition+GenerateLuminanceHistogram")
    hf = host_frame(W, H, gb)
    ae = soc.AutoExposure()
    hist = 0
    for f in range(3):
        fr["emissive"].copy_(torch.from_numpy(gb["emissive"]))
        if f == 1:
            with pytest.raises(soc.SocError, match="-7|caller pass"):
                r.execute(g)
            torch.cuda.synchronize()
            assert int(fr["auto_exposure"][1:].abs().sum()) == 0     # no partial bins left for the next frame
            continue
        r.execute(g)
        hf["emissive"][...] = gb["emissive"]
        hist = oracle.frame(g, hf, ae, hist=hist)
        torch.cuda.synchronize()
        assert r.current_history() == hist
        ok = f16_close(fr["color"].cpu().numpy(), hf["color"], atol=4e-3, rtol=8e-3)
        assert ok.mean() >= 0.999, (f, ok.mean())
        d = np.abs(fr["output"].cpu().numpy().astype(np.int32) - hf["output"].astype(np.int32))
        assert (d <= 2).mean() >= 0.995, (f, (d <= 2).mean())
        assert abs(soc.exposure_of(fr["auto_exposure"]) - ae.exposure) <= 1e-4, (f, soc.exposure_of(fr["auto_exposure"]),
                                                                                ae.exposure)
    assert len(calls) == 3
    r.close()


def test_checkpoint_resume_bit_identical(soc, tmp_path):
    """SURVEY.md §5 "Checkpoint / resume": the frame's temporal state is the TAA history (previous resolved colour and
    velocity), the AutoExposure block and the history slot (renderer.cpp:1170-1198). A renderer runs frames 0-4 with a
    moving, jittered camera; a checkpoint written after frame 2 (Renderer.save_state -> .npz) and loaded into a FRESH
    renderer and frame (zeroed histories, default exposure) continues with frames 3-4 bit-identically: colour,
    resolved history, framebuffer and the AutoExposure block. The fresh renderer without the checkpoint differs."""
    from helpers import globals_for
    W, H = 320, 180
    _, gb = sponza_inputs(W, H, elapsed=10.0)
    gs = [globals_for(W, H, frames=f + 1, elapsed=10.0 + 0.016 * f) for f in range(5)]

    def run(r, fr, frames):
        for f in frames:
            # the G-buffer producer rewrites emissive every frame; the graph's bloom writes its result into it
            fr["emissive"].copy_(torch.from_numpy(gb["emissive"]))
            r.execute(gs[f])
        torch.cuda.synchronize()
        return {"color": fr["color"].clone(), "resolved": r.resolved().clone(), "output": fr["output"].clone(),
                "auto_exposure": fr["auto_exposure"].clone()}

    fr_a = _frame(soc, W, H, gb)
    ra = soc.Renderer(fr_a)
    run(ra, fr_a, range(3))
    ckpt = str(tmp_path / "state.npz")
    st = ra.save_state(ckpt)
    assert int(st["history_index"]) == ra.current_history()
    want = run(ra, fr_a, range(3, 5))
    ra.close()

    fr_b = _frame(soc, W, H, gb)
    rb = soc.Renderer(fr_b)
    rb.load_state(ckpt)
    assert rb.current_history() == int(st["history_index"])
    got = run(rb, fr_b, range(3, 5))
    for k in want:
        assert torch.equal(got[k], want[k]), k
    rb.close()

    fr_c = _frame(soc, W, H, gb)
    rc = soc.Renderer(fr_c)
    cold = run(rc, fr_c, range(3, 5))
    assert not torch.equal(cold["resolved"], want["resolved"])
    rc.close()
    with pytest.raises(ValueError):
        soc.Renderer(_frame(soc, 64, 36, sponza_inputs(64, 36)[1])).load_state(ckpt)


def test_checkpoint_rejected_before_any_write(soc):
    """load_state checks the whole checkpoint before it writes anything: a history_index outside {0, 1} or an
    AutoExposure block of another dtype raises ValueError and leaves the frame's history images and AutoExposure as
    they were."""
    W, H = 64, 36
    _, gb = sponza_inputs(W, H, elapsed=10.0)
    fr = _frame(soc, W, H, gb)
    r = soc.Renderer(fr)
    r.execute(globals_for_frames(W, H))
    torch.cuda.synchronize()
    st = r.save_state()
    before = {"h0": fr["history_color"][0].clone(), "h1": fr["history_color"][1].clone(),
              "ae": fr["auto_exposure"].clone()}
    junk = dict(st)
    junk["history_color"] = np.full_like(st["history_color"], 7.0)
    for bad in ({**junk, "history_index": np.int32(-1)}, {**junk, "history_index": np.int32(2)},
                {**junk, "auto_exposure": st["auto_exposure"].astype(np.float32)}):
        with pytest.raises(ValueError):
            r.load_state(bad)
        torch.cuda.synchronize()
        assert torch.equal(fr["history_color"][0], before["h0"]) and torch.equal(fr["history_color"][1], before["h1"])
        assert torch.equal(fr["auto_exposure"], before["ae"])
    r.close()


def globals_for_frames(W, H):
    from helpers import globals_for
    return globals_for(W, H, elapsed=10.0)
