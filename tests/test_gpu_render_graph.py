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
