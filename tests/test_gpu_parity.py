"""Parity of every HIP pass against the CPU oracle, called through the C ABI (-m gpu).

Tolerances: bloom, SSAO blur and the histogram are bit-exact; RGBA16F outputs
|d| <= 1e-3 + 2e-3|ref|; SSAO R8 within 2/255 on >= 99.5 % of pixels and mean |d| <= 0.5/255;
exposure |d| <= 1e-5; tone-mapped RGBA8 within 1 level on >= 99.9 %; clouds RGBA8 within 2 levels on
>= 99.5 %.
"""
import ctypes as C

import numpy as np
import pytest
import torch

from helpers import (f16_close, frame_parity, globals_for, host_frame, mesh_inputs, random_rgba16, random_shadow, sponza_inputs,
                     terrain_inputs)

pytestmark = pytest.mark.gpu

DEV = "cuda"


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def host(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


SIZES = [(64, 36), (97, 55), (512, 512), (1920, 1080)]


# ------------------------------------------------------------------------------------------------ bloom
@pytest.mark.parametrize("W,H", SIZES)
def test_bloom_passes_bit_exact(soc, oracle, W, H):
    g = globals_for(W, H)
    src = random_rgba16(H, W, seed=W)
    dims = [(max(W >> i, 1), max(H >> i, 1)) for i in range(4)]
    # down: emissive -> mip0 (1:1), mip0 -> mip1 (2:1 when even)
    for (sw, sh), (dw, dh) in [((W, H), dims[0]), (dims[0], dims[1]), (dims[1], dims[2])]:
        s = random_rgba16(sh, sw, seed=sw * 7 + sh)
        ref = np.zeros((dh, dw, 4), np.float16)
        oracle.bloom_downsample(g, s, ref)
        out = torch.zeros(dh, dw, 4, dtype=torch.float16, device=DEV)
        soc.bloom_downsample(g, dev(s), out)
        got = host(out)
        assert np.array_equal(got[..., :3].view(np.uint16), ref[..., :3].view(np.uint16)), (sw, sh, dw, dh)
    # up: mip1 -> mip0 (1:2), mip0 -> emissive (1:1)
    for (sw, sh), (dw, dh) in [(dims[1], dims[0]), (dims[0], (W, H)), (dims[3], dims[2])]:
        s = random_rgba16(sh, sw, seed=sw * 3 + sh)
        ref = np.zeros((dh, dw, 4), np.float16)
        oracle.bloom_upsample(g, s, ref)
        out = torch.zeros(dh, dw, 4, dtype=torch.float16, device=DEV)
        soc.bloom_upsample(g, dev(s), out)
        got = host(out)
        assert np.array_equal(got[..., :3].view(np.uint16), ref[..., :3].view(np.uint16)), (sw, sh, dw, dh)
    del src


@pytest.mark.parametrize("W,H", [(64, 36), (1920, 1080)])
def test_bloom_fast_paths_equal_generic(soc, W, H):
    """The analytic 1:1 / 2:1 / 1:2 tap paths give the same bits as the float-uv generic path."""
    lib = soc.lib()
    for up, (sw, sh), (dw, dh) in [(0, (W, H), (W, H)), (0, (W, H), (W // 2, H // 2)), (1, (W // 2, H // 2), (W, H)),
                                   (1, (W, H), (W, H))]:
        s = dev(random_rgba16(sh, sw, seed=dw + 11 * up))
        a = torch.zeros(dh, dw, 4, dtype=torch.float16, device=DEV)
        b = torch.zeros_like(a)
        g = globals_for(W, H)
        (soc.bloom_upsample if up else soc.bloom_downsample)(g, s, a)
        rc = lib.soc_debug_bloom_generic(up, soc.img(s), soc.img(b), torch.cuda.current_stream().cuda_stream)
        assert rc == 0
        assert torch.equal(a[..., :3].view(torch.int16), b[..., :3].view(torch.int16))


@pytest.mark.parametrize("W,H", [(64, 36), (200, 136), (512, 512), (1920, 1080)])
def test_bloom_chain_bit_exact(soc, oracle, W, H):
    """soc_bloom_chain (fused stages where the mips halve exactly) leaves every mip and the emissive
    image with the oracle's bits."""
    g = globals_for(W, H)
    em = random_rgba16(H, W, seed=5, hi=8.0)
    mips_h = [np.zeros((max(H >> i, 1), max(W >> i, 1), 4), np.float16) for i in range(4)]
    em_h = em.copy()
    oracle.bloom_chain(g, em_h, mips_h)
    em_d = dev(em)
    mips_d = [torch.zeros(m.shape, dtype=torch.float16, device=DEV) for m in mips_h]
    soc.bloom_chain(g, em_d, mips_d)
    assert np.array_equal(host(em_d)[..., :3].view(np.uint16), em_h[..., :3].view(np.uint16))
    for i in range(4):
        assert np.array_equal(host(mips_d[i])[..., :3].view(np.uint16), mips_h[i][..., :3].view(np.uint16)), i


@pytest.mark.parametrize("sep", ["1", "0"])
@pytest.mark.parametrize("W,H", [(64, 40), (200, 136), (968, 552), (1920, 1080), (3840, 2160)])
def test_bloom_weighted_chain(soc, monkeypatch, W, H, sep):
    """The weighted-form chain (bloom_w.hip, 4 kernels) against the reference's 8 separate passes
    (bit-exact to the oracle): output and the observable mips (1 upswept, 3 downswept) within the
    RGBA16F tolerance, and almost all texels bit-identical (the weights are the taps' exact weights;
    only the fp32 rounding order differs). Stage by stage equals the whole chain; the emissive input of
    a separate output is untouched. sep: the upsample launches in separable form (default) or 2-D."""
    monkeypatch.setenv("SOC_BLOOM_UP_SEP", sep)
    soc.reload_tuning()
    g = globals_for(W, H)
    em = dev(random_rgba16(H, W, seed=23, hi=16.0))
    shapes = [(H >> i, W >> i, 4) for i in range(4)]
    ref = [torch.zeros(sh, dtype=torch.float16, device=DEV) for sh in shapes]
    ref_out = torch.zeros_like(em)
    soc.bloom_downsample(g, em, ref[0])
    for i in range(3):
        soc.bloom_downsample(g, ref[i], ref[i + 1])
    ref3 = ref[3].clone()
    for i in range(3, 0, -1):
        soc.bloom_upsample(g, ref[i], ref[i - 1])
    soc.bloom_upsample(g, ref[0], ref_out)
    em_before = em.clone()
    mips = [torch.full(sh, 7.0, dtype=torch.float16, device=DEV) for sh in shapes]
    out = torch.zeros_like(em)
    soc.bloom_weighted_stage(g, em, mips, out, 0)
    mips2 = [torch.zeros(sh, dtype=torch.float16, device=DEV) for sh in shapes]
    out2 = torch.zeros_like(em)
    for st in (1, 2, 3, 4):
        soc.bloom_weighted_stage(g, em, mips2, out2, st)
    torch.cuda.synchronize()
    assert torch.equal(em, em_before)
    assert torch.equal(out, out2) and torch.equal(mips[1], mips2[1]) and torch.equal(mips[3], mips2[3])
    for got, want in ((out, ref_out), (mips[1], ref[1]), (mips[3], ref3)):
        g_, w_ = host(got)[..., :3], host(want)[..., :3]
        assert f16_close(g_, w_).all()
        assert (g_.view(np.uint16) == w_.view(np.uint16)).mean() >= 0.99
    assert torch.all(mips[0] == 7.0) and torch.all(mips[2] == 7.0)   # scratch mips are not written


@pytest.mark.parametrize("W,H", [(64, 40), (200, 136), (968, 552), (3840, 2160)])
def test_bloom_up10_register_form_bit_identical(soc, monkeypatch, W, H):
    """The last upsample in register form (bloomw_up10r: a wave walks a 62-column strip down 16 rows, sliding sums in
    registers, neighbours by DPP) gives the tiled separable kernel's bits (bloomw_up10s: the same operations in the same
    order), borders included."""
    g = globals_for(W, H)
    em = dev(random_rgba16(H, W, seed=29, hi=16.0))
    shapes = [(H >> i, W >> i, 4) for i in range(4)]
    outs = []
    for reg in ("1", "0"):
        monkeypatch.setenv("SOC_BLOOM_UP10_REG", reg)
        soc.reload_tuning()
        mips = [torch.zeros(sh, dtype=torch.float16, device=DEV) for sh in shapes]
        out = torch.zeros_like(em)
        soc.bloom_weighted_stage(g, em, mips, out, 0)
        outs.append(out)
    torch.cuda.synchronize()
    monkeypatch.delenv("SOC_BLOOM_UP10_REG")
    soc.reload_tuning()
    assert torch.equal(outs[0], outs[1]), (outs[0] != outs[1]).float().mean().item()


@pytest.mark.parametrize("W,H", [(3840, 2160), (1920, 1080), (968, 552), (136, 40), (256, 16)])
def test_bloom_w1_register_runs_bit_identical(soc, monkeypatch, W, H):
    """The first downsample's 1:1 stage register-blocked (bloomw_down01p<1>: 30 x 8 mip1 outputs per workgroup, each
    lane a run of 5 mip0 entries at row stride 2 from a sliding window of texels; <2>: 30 x 16, runs of 9 and the 2:1
    stage in vertical output pairs) gives the 32 x 8 per-entry kernel's bits (the same fmas per entry and output in the
    same order): mip1 and the chain's output. 136 x 40 / 256 x 16: every tile
    touches the image's top or bottom (the per-entry fallback) or a right edge inside a tile."""
    g = globals_for(W, H)
    em = dev(random_rgba16(H, W, seed=31, hi=16.0))
    shapes = [(H >> i, W >> i, 4) for i in range(4)]
    res = []
    for reg in ("0", "1", "2"):
        monkeypatch.setenv("SOC_BLOOM_W1_REG", reg)
        soc.reload_tuning()
        mips = [torch.zeros(sh, dtype=torch.float16, device=DEV) for sh in shapes]
        out = torch.zeros_like(em)
        soc.bloom_weighted_stage(g, em, mips, out, 0)
        res.append((mips[1], out))
    torch.cuda.synchronize()
    monkeypatch.delenv("SOC_BLOOM_W1_REG")
    soc.reload_tuning()
    for m1, out in res[1:]:
        assert torch.equal(res[0][0], m1), (res[0][0] != m1).float().mean().item()
        assert torch.equal(res[0][1], out)


@pytest.mark.parametrize("W,H", [(3840, 2160), (1920, 1080), (968, 552), (136, 40), (512, 64)])
def test_bloom_w2_register_runs_bit_identical(soc, monkeypatch, W, H):
    """The second downsample's 2:1 mip1 -> mip2 stage in vertical runs of 3 entries per lane (bloomw_down23<true>: each
    run's mip1 rows read once) gives the per-entry kernel's bits (the same 36 fmas per entry in the same order): mip3
    and the chain's output; small extents: tiles at the image's top and bottom (the per-entry fallback)."""
    g = globals_for(W, H)
    em = dev(random_rgba16(H, W, seed=37, hi=16.0))
    shapes = [(H >> i, W >> i, 4) for i in range(4)]
    res = []
    for reg in ("0", "1"):
        monkeypatch.setenv("SOC_BLOOM_W2_REG", reg)
        soc.reload_tuning()
        mips = [torch.zeros(sh, dtype=torch.float16, device=DEV) for sh in shapes]
        out = torch.zeros_like(em)
        soc.bloom_weighted_stage(g, em, mips, out, 0)
        res.append((mips[3], out))
    torch.cuda.synchronize()
    monkeypatch.delenv("SOC_BLOOM_W2_REG")
    soc.reload_tuning()
    assert torch.equal(res[0][0], res[1][0]), (res[0][0] != res[1][0]).float().mean().item()
    assert torch.equal(res[0][1], res[1][1])


@pytest.mark.parametrize("W,H", [(3840, 2160), (1920, 1080), (968, 552), (136, 40)])
def test_bloom_w3_runs_bit_identical(soc, monkeypatch, W, H):
    """The first upsample's last vertical 1:2 phase in runs of 4 output rows per lane (bloomw_up32s<true>) gives the
    per-pair loop's bits (the same 4 fmas per output in the same order): mip1 after stage 3 and the chain's output."""
    g = globals_for(W, H)
    em = dev(random_rgba16(H, W, seed=41, hi=16.0))
    shapes = [(H >> i, W >> i, 4) for i in range(4)]
    res = []
    for runs in ("0", "1"):
        monkeypatch.setenv("SOC_BLOOM_W3_RUNS", runs)
        soc.reload_tuning()
        mips = [torch.zeros(sh, dtype=torch.float16, device=DEV) for sh in shapes]
        out = torch.zeros_like(em)
        soc.bloom_weighted_stage(g, em, mips, out, 0)
        res.append(out)
    torch.cuda.synchronize()
    monkeypatch.delenv("SOC_BLOOM_W3_RUNS")
    soc.reload_tuning()
    assert torch.equal(res[0], res[1]), (res[0] != res[1]).float().mean().item()


def test_bloom_weighted_in_place(soc):
    """output == emissive (the reference's in-place bloom) gives the separate-output result."""
    W, H = 968, 552
    g = globals_for(W, H)
    em = dev(random_rgba16(H, W, seed=29, hi=4.0))
    shapes = [(H >> i, W >> i, 4) for i in range(4)]
    out = torch.zeros_like(em)
    soc.bloom_weighted_stage(g, em, [torch.zeros(sh, dtype=torch.float16, device=DEV) for sh in shapes], out, 0)
    soc.bloom_weighted_stage(g, em, [torch.zeros(sh, dtype=torch.float16, device=DEV) for sh in shapes], em, 0)
    torch.cuda.synchronize()
    assert torch.equal(em, out)


# ------------------------------------------------------------------------------------------------ ssao
@pytest.mark.parametrize("W,H,inputs", [(128, 72, "boxes"), (97, 55, "boxes"), (1920, 1080, "boxes"),
                                         (1920, 1080, "mesh"), (961, 541, "mesh")])
def test_ssao_generation(soc, oracle, W, H, inputs):
    """boxes: the box atrium; mesh: the Sponza-proxy mesh the bench renders (curved, normal-mapped surfaces)."""
    g, gb = (sponza_inputs if inputs == "boxes" else mesh_inputs)(W, H)
    ref = np.zeros((H // 2, W // 2), np.uint8)
    oracle.ssao_generation(g, gb["depth"], gb["normal"], ref)
    out = torch.zeros(H // 2, W // 2, dtype=torch.uint8, device=DEV)
    soc.ssao_generation(g, dev(gb["depth"]), dev(gb["normal"]), out)
    d = np.abs(host(out).astype(np.int32) - ref.astype(np.int32))
    assert (d <= 2).mean() >= 0.995, (d.max(), (d <= 2).mean())
    assert d.mean() <= 0.5, d.mean()


def test_ssao_noise_table_is_bit_identical(soc):
    W, H = 256, 144
    g, gb = sponza_inputs(W, H)
    depth, normal = dev(gb["depth"]), dev(gb["normal"])
    a = torch.zeros(H // 2, W // 2, dtype=torch.uint8, device=DEV)
    b = torch.zeros_like(a)
    table = torch.zeros((H // 2) * (W // 2) * 2, dtype=torch.float32, device=DEV)
    soc.ssao_prepare_noise(normal, a, table)
    soc.ssao_generation(g, depth, normal, a, table)
    soc.ssao_generation(g, depth, normal, b, None)
    assert torch.equal(a, b)


@pytest.mark.parametrize("W,H,inputs", [(97, 55, "boxes"), (1920, 1080, "boxes"), (1920, 1080, "mesh"), (3840, 2160, "mesh"),
                                         (130, 1200, "boxes"), (2000, 34, "boxes")])
def test_ssao_tile_orders_bit_identical(soc, monkeypatch, W, H, inputs):
    """The LDS-tiled kernel (default: depth tile + 32-texel halo in LDS, the other taps gathered, the software-pipelined
    tap loop with the affine range test, SOC_SSAO_PIPE=2) and the plain gather kernel (SOC_SSAO_TILE=0) give the same
    bits (the round-5 tap loop,
    SOC_SSAO_PIPE=0, with its per-pixel fetches issued before the barrier
    and the centre depth from the tile, SOC_SSAO_EARLY=1; its staging loads all issued first, 2, the default; neither, 0), in every workgroup order of the gather kernel (row-major, XCD-aware
    eighths, horizontal and vertical XCD bands: SOC_SWZ_SSAO; the orders are bijections, also for ragged grids), on the
    box atrium and on the mesh (near geometry: many taps leave the tile), at odd, tall and wide extents (partial tiles,
    tiles hanging over every image edge)."""
    if inputs == "mesh":
        from soc_real_time_renderer_amd import raster, scene
        import bench
        g = bench.make_globals(W, H, bench.multi_gpu.camera_for_rank(0))
        sc = raster.scene_setup(g, scene.SPONZA_MESH, tex_size=64, device=DEV)
        gbd = raster.render_gbuffer(g, sc, W, H, 256, DEV)
        depth, normal = gbd["depth"], gbd["normal"]
    else:
        g, gb = sponza_inputs(W, H)
        depth, normal = dev(gb["depth"]), dev(gb["normal"])
    table = torch.zeros((H // 2) * (W // 2) * 2, dtype=torch.float32, device=DEV)
    outs = []
    for tile, swz, early, pipe in (("1", None, "2", "2"), ("1", None, "1", "0"), ("1", None, "0", "0"), ("1", None, "2", "0"),
                                   ("0", "0", "1", "0"), ("0", "1", "1", "0"), ("0", "4", "1", "0"), ("0", "16", "1", "0"),
                                   ("0", "-16", "1", "0"), ("0", "-3", "1", "0")):
        monkeypatch.setenv("SOC_SSAO_TILE", tile)
        monkeypatch.setenv("SOC_SSAO_EARLY", early)
        monkeypatch.setenv("SOC_SSAO_PIPE", pipe)
        if swz is None:
            monkeypatch.delenv("SOC_SWZ_SSAO", raising=False)
        else:
            monkeypatch.setenv("SOC_SWZ_SSAO", swz)
        soc.reload_tuning()
        out = torch.zeros(H // 2, W // 2, dtype=torch.uint8, device=DEV)
        soc.ssao_prepare_noise(normal, out, table)
        soc.ssao_generation(g, depth, normal, out, table)
        outs.append(host(out))
    monkeypatch.delenv("SOC_SSAO_TILE")
    monkeypatch.delenv("SOC_SSAO_EARLY")
    monkeypatch.delenv("SOC_SSAO_PIPE")
    monkeypatch.delenv("SOC_SWZ_SSAO", raising=False)
    soc.reload_tuning()
    for o in outs[1:]:
        assert np.array_equal(o, outs[0]), int((o != outs[0]).sum())
    # the default: the pipelined loop with the range test's sample depth from the tap's w' (the reference perspective's
    # w row, PERSP): a different rounding of (s.z - frag.z) / r, so a tap whose range test sits on its edge may flip
    out = torch.zeros(H // 2, W // 2, dtype=torch.uint8, device=DEV)
    soc.ssao_generation(g, depth, normal, out, table)
    d = np.abs(host(out).astype(np.int32) - outs[0].astype(np.int32))
    assert (d > 0).mean() <= 1e-4 and d.max() <= 10, ((d > 0).sum(), d.max())


@pytest.mark.parametrize("W,H", [(64, 36), (97, 55), (1920, 1080), (3840, 2160), (100, 40), (16, 8)])
def test_ssao_blur_bit_exact(soc, oracle, W, H):
    """Up to the 4K frame's 1920 x 1080 half-res image, and extents of 8 and 50 half-res pixels (every lane near a border)."""
    g = globals_for(W, H)
    rng = np.random.default_rng(3)
    src = rng.integers(0, 256, (H // 2, W // 2), dtype=np.uint8)
    ref = np.zeros_like(src)
    oracle.ssao_blur(g, src, ref)
    out = torch.zeros_like(dev(src))
    soc.ssao_blur(g, dev(src), out)
    assert np.array_equal(host(out), ref)


# ------------------------------------------------------------------------------------------------ composition
@pytest.mark.parametrize("W,H", [(1920, 1080), (130, 1200), (2002, 34), (66, 4)])
def test_composition_cache_policy_variants_bit_identical(soc, monkeypatch, W, H):
    """The non-temporal load/store variant of the fast path (default) gives the plain variant's bits, and so do the
    pixel pair's AO taps as one 8-B row load per row (SOC_COMP_AOP, default) against per-texel byte loads, with and
    without the fused histogram (same bins), at extents whose half-res AO rows end at every byte of a dword."""
    g, gb = sponza_inputs(W, H)
    shadow = dev(random_shadow(256, seed=3))
    rng = np.random.default_rng(5)
    ssao = dev(rng.integers(0, 256, (H // 2, W // 2), dtype=np.uint8))
    clouds = dev(rng.integers(0, 256, (H, W, 4), dtype=np.uint8))
    ins = [dev(gb[k]) for k in ("albedo", "emissive", "normal", "depth")]
    outs, bins = [], []
    for nt, aop in (("3", "1"), ("3", "0"), ("0", "1"), ("0", "0")):
        monkeypatch.setenv("SOC_COMP_NT", nt)
        monkeypatch.setenv("SOC_COMP_AOP", aop)
        soc.reload_tuning()
        out = torch.zeros(H, W, 4, dtype=torch.float16, device=DEV)
        soc.composition(g, out, *ins, ssao, shadow, clouds)
        outs.append(host(out))
        out2 = torch.zeros(H, W, 4, dtype=torch.float16, device=DEV)
        ae = soc.auto_exposure_buffer()
        soc.composition_luminance_histogram(g, out2, *ins, ssao, shadow, clouds, ae, soc.histogram_scratch())
        assert np.array_equal(host(out2).view(np.uint16), outs[-1].view(np.uint16))
        bins.append(host(ae))
    monkeypatch.delenv("SOC_COMP_NT")
    monkeypatch.delenv("SOC_COMP_AOP")
    soc.reload_tuning()
    for o, b in zip(outs[1:], bins[1:]):
        assert np.array_equal(outs[0].view(np.uint16), o.view(np.uint16))
        assert np.array_equal(bins[0], b)


@pytest.mark.parametrize("W,H,inputs", [(64, 36, "boxes"), (97, 55, "boxes"), (512, 288, "boxes"), (1920, 1080, "boxes"),
                                         (1920, 1080, "mesh")])
@pytest.mark.parametrize("lights", [0, 3])
def test_composition(soc, oracle, W, H, inputs, lights):
    g, gb = (sponza_inputs if inputs == "boxes" else mesh_inputs)(W, H)
    shadow = random_shadow(256, seed=W)
    rng = np.random.default_rng(W + lights)
    ssao = rng.integers(120, 256, (H // 2, W // 2), dtype=np.uint8)
    clouds = rng.integers(0, 256, (H, W, 4), dtype=np.uint8)
    g.point_light_count = lights
    g.spot_light_count = lights
    for i in range(lights):
        pl = g.point_lights[i]
        pl.position[:] = [-10.0 + 5 * i, 2.0, 0.5 * i]
        pl.color[:] = [1.0, 0.8, 0.6]
        pl.intensity = 3.0
        sl = g.spot_lights[i]
        sl.position[:] = [-6.0 + 4 * i, 4.0, -1.0]
        sl.direction[:] = [0.3, -1.0, 0.1]
        sl.color[:] = [0.5, 0.7, 1.0]
        sl.intensity = 5.0
        sl.cut_off, sl.outer_cut_off = 0.95, 0.85
    ref = np.zeros((H, W, 4), np.float16)
    oracle.composition(g, ref, gb["albedo"], gb["emissive"], gb["normal"], gb["depth"], ssao, shadow, clouds)
    dg = soc.globals_device_buffer()
    soc.upload_globals(g, dg)
    out = torch.zeros(H, W, 4, dtype=torch.float16, device=DEV)
    soc.composition(g, out, dev(gb["albedo"]), dev(gb["emissive"]), dev(gb["normal"]), dev(gb["depth"]), dev(ssao),
                    dev(shadow), dev(clouds), d_globals=dg)
    got = host(out)
    # the mesh's normal-mapped G-buffer normals are not unit length after RGBA16F rounding, and the reference feeds
    # them to acos(dot(halfway, normal)) unnormalised (composition.inl:133, 154): |dot| > 1 gives NaN on both sides,
    # but which pixels round across 1 depends on the dot's rounding (0.16 % of the pixels at 1080p, 3 + 3 lights)
    nan_tol = 5e-3 if (inputs == "mesh" and lights) else 0.0
    ok = f16_close(got, ref, nan_mismatch=nan_tol)
    if nan_tol:
        both = ~(np.isnan(got.astype(np.float32)) | np.isnan(ref.astype(np.float32)))
        assert abs(np.isnan(got.astype(np.float32)).mean() - np.isnan(ref.astype(np.float32)).mean()) < 1e-3
        ok = ok | ~both
    assert ok.all(), (ok.mean(), np.argwhere(~ok)[:5])
    sky = gb["depth"] == 1.0
    assert np.array_equal(got[sky].view(np.uint16), ref[sky].view(np.uint16))   # sky = clouds texel, exact


@pytest.mark.parametrize("W,H", [(64, 36), (98, 56), (97, 55), (1920, 1080), (3840, 2160)])
def test_composition_histogram_fused(soc, W, H):
    """One-launch composition + histogram: the colour equals soc_composition's bit-for-bit and the bins
    equal those the histogram pass computes from it (98x56: partial tiles; 97x55: two-pass fallback).
    Pre-existing bin counts are added to, not overwritten."""
    g, gb = sponza_inputs(W, H, elapsed=10.0)
    rng = np.random.default_rng(W)
    ssao = dev(rng.integers(120, 256, (H // 2, W // 2), dtype=np.uint8))
    clouds = dev(rng.integers(0, 256, (H, W, 4), dtype=np.uint8))
    ins = [dev(gb[k]) for k in ("albedo", "emissive", "normal", "depth")]
    shadow = dev(gb["shadow"])
    c1 = torch.zeros(H, W, 4, dtype=torch.float16, device=DEV)
    soc.composition(g, c1, *ins, ssao, shadow, clouds)
    a1 = soc.auto_exposure_buffer()
    a1[1:] = 7
    soc.generate_luminance_histogram(g, c1, a1)
    c2 = torch.zeros_like(c1)
    a2 = soc.auto_exposure_buffer()
    a2[1:] = 7
    scratch = soc.histogram_scratch()
    for _ in range(2):   # the scratch is left zeroed: a second call adds the same bins again
        soc.composition_luminance_histogram(g, c2, *ins, ssao, shadow, clouds, a2, scratch)
    torch.cuda.synchronize()
    assert int(scratch.abs().sum()) == 0
    a2[1:] = (a2[1:] - 7) // 2 + 7
    assert torch.equal(c1, c2)
    assert torch.equal(a1, a2)
    assert int(a2[1:].sum()) == W * H + 7 * 256


# ------------------------------------------------------------------------------------------------ exposure
@pytest.mark.parametrize("W,H", [(64, 36), (97, 55), (1920, 1080), (3840, 2160)])
def test_histogram_bit_exact(soc, oracle, W, H):
    g = globals_for(W, H)
    rng = np.random.default_rng(W)
    img = np.exp(rng.normal(-1.0, 3.0, (H, W, 4))).astype(np.float16)
    img[rng.uniform(size=(H, W)) < 0.05] = 0.0          # black pixels -> bin 255 (quirk Q9)
    img[0, 0] = np.float16(np.nan)
    ae = soc.AutoExposure()
    oracle.generate_luminance_histogram(g, img, ae)
    ref = np.array(ae.histogram_buckets, np.int64)
    buf = soc.auto_exposure_buffer()
    soc.generate_luminance_histogram(g, dev(img), buf)
    got = host(buf)[1:].astype(np.int64)
    assert got.sum() == W * H
    assert np.array_equal(got, ref)


def _boundary_colours(g, n, rng):
    """RGBA16F colours whose luminance maps within ~1e-3 of a bin boundary (the integers 1..255 of the
    remap of generate_luminance_histogram.inl:64-69), half of them within the fast path's fallback margin:
    the pixels where lum_bin_fast must hand over to the exact lum_bin."""
    lmin, lmax = float(g.log_min_luminance), float(g.log_max_luminance)
    out = []
    while sum(len(o) for o in out) < n:
        k = rng.integers(1, 256, 200_000)
        t = (k - 1 + rng.uniform(-2e-3, 2e-3, k.size)) / 254.0       # target mapped - 1, over 254
        lum = np.exp2(lmin + t * (lmax - lmin))
        ok = (lum > 1.5e-3) & (lum < 6.0e4)
        w = rng.dirichlet((1.0, 1.0, 1.0), k.size)[ok]               # random channel split of the luminance
        lum = lum[ok]
        rgb = w * (lum / (w @ np.array([0.2126, 0.7152, 0.0722])))[:, None]
        rgb = rgb[(rgb < 6.0e4).all(axis=1)].astype(np.float16).astype(np.float64)
        m = 1.0 + 254.0 * (np.log2(np.maximum(rgb @ np.array([0.2126, 0.7152, 0.0722]), 1e-30)) - lmin) / (lmax - lmin)
        keep = np.abs(m - np.rint(m)) < 1e-3
        out.append(rgb[keep])
    rgb = np.concatenate(out)[:n]
    return np.concatenate([rgb, np.ones((n, 1))], axis=1).astype(np.float16)


@pytest.mark.parametrize("W,H", [(512, 256), (1920, 1080)])
def test_histogram_bin_boundaries_bit_exact(soc, oracle, W, H):
    """Every pixel near a bin boundary (the fast bin's exact fallback), mixed with ordinary pixels."""
    g = globals_for(W, H)
    rng = np.random.default_rng(H)
    img = np.exp(rng.normal(-1.0, 3.0, (H, W, 4))).astype(np.float16)
    sel = rng.uniform(size=(H, W)) < 0.5
    img[sel] = _boundary_colours(g, int(sel.sum()), rng)
    ae = soc.AutoExposure()
    oracle.generate_luminance_histogram(g, img, ae)
    ref = np.array(ae.histogram_buckets, np.int64)
    buf = soc.auto_exposure_buffer()
    soc.generate_luminance_histogram(g, dev(img), buf)
    got = host(buf)[1:].astype(np.int64)
    assert got.sum() == W * H
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("wide", [False, True])
def test_resolve(soc, oracle, wide):
    g = globals_for(640, 360)
    rng = np.random.default_rng(1)
    bins = rng.integers(0, 3000, 256).astype(np.uint32)
    ae = soc.AutoExposure()
    ae.exposure = 0.37
    ae.histogram_buckets[:] = [int(b) for b in bins]
    total = 640 * 360 * (8 if wide else 1)
    oracle.resolve_luminance_histogram(g, ae, total if wide else 0, wide)
    buf = soc.auto_exposure_buffer(exposure=0.37)
    buf[1:] = torch.from_numpy(bins.astype(np.int32)).to(DEV)
    soc.resolve_luminance_histogram(g, buf, total if wide else 0, wide)
    assert abs(soc.exposure_of(buf) - ae.exposure) <= 1e-5
    assert int(host(buf)[1:].sum()) == 0


# ------------------------------------------------------------------------------------------------ TAA
@pytest.mark.parametrize("W,H,inputs", [(64, 36, "boxes"), (97, 55, "boxes"), (1920, 1080, "boxes"), (1920, 1080, "mesh")])
def test_taa(soc, oracle, W, H, inputs):
    g, gb = (sponza_inputs if inputs == "boxes" else mesh_inputs)(W, H)
    cur = random_rgba16(H, W, seed=1, hi=3.0)
    prev = random_rgba16(H, W, seed=2, hi=3.0)
    pvel = gb["velocity"].copy()
    pvel[..., :2] += np.float16(0.0015)
    ref = np.zeros((H, W, 4), np.float16)
    oracle.temporal_antialiasing(g, ref, cur, prev, gb["velocity"], pvel, gb["depth"])
    out = torch.zeros(H, W, 4, dtype=torch.float16, device=DEV)
    vout = torch.zeros(H, W, 4, dtype=torch.float16, device=DEV)
    soc.temporal_antialiasing(g, out, dev(cur), dev(prev), dev(gb["velocity"]), dev(pvel), dev(gb["depth"]), vout)
    ok = f16_close(host(out), ref)
    assert ok.all(), ok.mean()
    assert np.array_equal(host(vout).view(np.uint16), gb["velocity"].view(np.uint16))


@pytest.mark.parametrize("W,H,noisy", [(100, 40, False), (102, 42, False), (102, 45, True), (1920, 1080, False),
                                       (1920, 1080, True)])
def test_taa_lane_shift_neighbours_identical(soc, oracle, monkeypatch, W, H, noisy):
    """Every neighbourhood source gives the bits of the per-lane loads (SOC_TAA_NBR=0): the LDS-staged tiles with every
    staging load issued first (4, default) and staged round by round (3), the side columns from the adjacent lanes (DPP wave shifts) with halo-only first / last lanes (2) and with
    edge-lane loads (1). 100 px: 50
    pairs in one 64-pair LDS tile row (14 lanes past the image) / a 62-pair wave row (12 lanes past), 32-lane block rows
    of which the second has 18 lanes inside; 102 x 42: a partial last depth quad (W % 4 == 2) and a last tile row with
    2 of its 4 rows inside (H % 4 == 2); 102 x 45: an odd height (the last two-row lanes have one row inside); 1920 px:
    15 LDS tiles, 15.5 wave rows. noisy: per-pixel velocity noise of a few texels (history taps scattered, not a smooth
    field)."""
    g, gb = sponza_inputs(W, H)
    cur = dev(random_rgba16(H, W, seed=3, hi=3.0))
    prev = dev(random_rgba16(H, W, seed=4, hi=3.0))
    velocity = gb["velocity"].copy()
    if noisy:
        rng = np.random.default_rng(5)
        velocity[..., 0] += (rng.integers(-3, 4, (H, W)) / W).astype(np.float16)
        velocity[..., 1] += (rng.integers(-3, 4, (H, W)) / H).astype(np.float16)
    pvel = velocity.copy()
    pvel[..., :2] += np.float16(0.0015)
    vel, pvel, depth = dev(velocity), dev(pvel), dev(gb["depth"])
    if (W * 4) % 16:   # the LDS tiles stage 16-B depth quads: a row pitch padded to 16 B (rows may be padded)
        dp = torch.zeros(H, W + 2, dtype=torch.float32, device=DEV)
        dp[:, :W] = depth
        depth = dp[:, :W]
    ae = soc.auto_exposure_buffer(exposure=0.37)
    outs = []
    for nbr in ("4", "3", "2", "1", "0"):
        monkeypatch.setenv("SOC_TAA_NBR", nbr)
        soc.reload_tuning()
        t = torch.zeros(H, W, 4, dtype=torch.float16, device=DEV)
        o = torch.zeros(H, W, 4, dtype=torch.uint8, device=DEV)
        vo = torch.zeros(H, W, 4, dtype=torch.float16, device=DEV)
        soc.temporal_antialiasing_tone_mapping(g, t, cur, prev, vel, pvel, depth, ae, o, vo)
        t2 = torch.zeros(H, W, 4, dtype=torch.float16, device=DEV)   # the TAA pass alone
        soc.temporal_antialiasing(g, t2, cur, prev, vel, pvel, depth)
        outs.append((t, o, vo, t2))
    torch.cuda.synchronize()
    for t, o, vo, t2 in outs[1:]:
        assert torch.equal(outs[0][0], t)
        assert torch.equal(outs[0][1], o)
        assert torch.equal(outs[0][2], vo)
        assert torch.equal(outs[0][0], t2)
    assert torch.equal(outs[0][2], vel)
    ref = np.zeros((H, W, 4), np.float16)
    oracle.temporal_antialiasing(g, ref, host(cur), host(prev), velocity, host(pvel), gb["depth"])
    ok = f16_close(host(outs[0][0]), ref)
    assert ok.all(), ok.mean()


@pytest.mark.parametrize("W,H,srgb", [(64, 36, False), (97, 55, False), (1920, 1080, False), (64, 36, True),
                                      (1920, 1080, True)])
def test_taa_tone_mapping_fused_equals_two_passes(soc, W, H, srgb):
    """The fused TAA + tone-map launch gives the TAA pass's bits and the tone-map pass's bits (97x55:
    odd width, the two-pass fallback), for an RGBA8_UNORM and an RGBA8_SRGB framebuffer (sRGB-encoded store)."""
    fmt = soc.FMT_RGBA8_SRGB if srgb else None
    g, gb = sponza_inputs(W, H)
    cur = dev(random_rgba16(H, W, seed=1, hi=3.0))
    prev = dev(random_rgba16(H, W, seed=2, hi=3.0))
    pvel = gb["velocity"].copy()
    pvel[..., :2] += np.float16(0.0015)
    vel, pvel, depth = dev(gb["velocity"]), dev(pvel), dev(gb["depth"])
    ae = soc.auto_exposure_buffer(exposure=0.37)
    t1 = torch.zeros(H, W, 4, dtype=torch.float16, device=DEV)
    o1 = torch.zeros(H, W, 4, dtype=torch.uint8, device=DEV)
    soc.temporal_antialiasing(g, t1, cur, prev, vel, pvel, depth)
    soc.tone_mapping(g, t1, ae, o1, target_format=fmt)
    t2, o2, v2 = torch.zeros_like(t1), torch.zeros_like(o1), torch.zeros_like(t1)
    soc.temporal_antialiasing_tone_mapping(g, t2, cur, prev, vel, pvel, depth, ae, o2, velocity_history_out=v2,
                                           output_format=fmt)
    torch.cuda.synchronize()
    assert torch.equal(t1, t2)
    assert torch.equal(v2, vel)
    d = (o1.int() - o2.int()).abs()
    assert int(d.max()) <= 1 and float((d > 0).float().mean()) < 1e-4


# ------------------------------------------------------------------------------------------------ tone mapping
@pytest.mark.parametrize("W,H", [(64, 36), (97, 55), (1920, 1080)])
@pytest.mark.parametrize("fmt", ["RGBA8_UNORM", "RGBA32F", "RGBA8_SRGB"])
def test_tone_mapping(soc, oracle, W, H, fmt):
    g = globals_for(W, H)
    img = random_rgba16(H, W, seed=4, lo=-0.5, hi=6.0)
    ae = soc.AutoExposure()
    ae.exposure = -0.8
    F = getattr(soc, "FMT_" + fmt)
    if fmt == "RGBA32F":
        ref = np.zeros((H, W, 4), np.float32)
        out = torch.zeros(H, W, 4, dtype=torch.float32, device=DEV)
    else:
        ref = np.zeros((H, W, 4), np.uint8)
        out = torch.zeros(H, W, 4, dtype=torch.uint8, device=DEV)
    oracle.tone_mapping(g, img, ae, ref, F)
    soc.tone_mapping(g, dev(img), soc.auto_exposure_buffer(exposure=-0.8), out, F)
    got = host(out)
    if fmt == "RGBA32F":
        assert np.abs(got - ref).max() <= 2e-3
    else:
        d = np.abs(got.astype(np.int32) - ref.astype(np.int32))
        assert (d <= 1).mean() >= 0.999 and d.max() <= 2


# ------------------------------------------------------------------------------------------------ clouds
@pytest.mark.parametrize("W,H,pitch,inputs", [(96, 64, -0.42, "boxes"), (160, 90, -0.9, "boxes"), (480, 270, -0.42, "boxes"),
                                               (1920, 1080, -0.6, "boxes"), (1920, 1080, -0.42, "mesh")])
@pytest.mark.parametrize("compact", [False, True])
def test_clouds(soc, oracle, W, H, pitch, inputs, compact):
    g, gb = (sponza_inputs if inputs == "boxes" else mesh_inputs)(W, H, camera=((-14.0, 2.2, 0.3), (0.0, pitch, 0.0)),
                                                                  elapsed=10.0)
    if inputs == "mesh":
        assert (gb["depth"] == 1.0).mean() > 0.05
    ref = np.zeros((H, W, 4), np.uint8)
    oracle.cloud_rendering(g, gb["depth"], gb["noise"], ref)
    out = torch.zeros(H, W, 4, dtype=torch.uint8, device=DEV)
    ws = soc.cloud_rendering_workspace(W, H) if compact else None
    soc.cloud_rendering(g, dev(gb["depth"]), dev(gb["noise"]), out, ws)
    d = np.abs(host(out).astype(np.int32) - ref.astype(np.int32))
    assert (d <= 2).mean() >= 0.995, ((d <= 2).mean(), d.max())
    nonsky = gb["depth"] < 1.0
    assert (host(out)[nonsky][:, :3] == np.array([51, 102, 255], np.uint8)).all()


@pytest.mark.parametrize("W,H,pitch,all_sky", [(320, 180, 0.35, False), (1920, 1080, 0.35, False), (256, 144, 0.9, True)])
def test_clouds_pair_path_equals_single_lane(soc, monkeypatch, W, H, pitch, all_sky):
    """The workspace path (classify, atmosphere, density / sunvis / resolve over dense-step pairs) gives
    the single-lane kernel's bits: od and vis are evaluated at the same positions with the same
    additions and accumulated in the same order, with the atmosphere kernel in any of its positions in the lane
    (SOC_CLOUDS_ATMOS_POS 0 / 1 / 2). An all-sky frame overflows the pair lists (2 pairs per image pixel) and
    exercises the per-batch single-lane fallback. The secondary-ray table is off here (SOC_CLOUDS_OD_LUT=0); the next test
    bounds what it changes."""
    g, gb = sponza_inputs(W, H, camera=((-14.0, 2.2, 0.3), (0.0, pitch, 0.0)), elapsed=10.0)
    depth = np.ones_like(gb["depth"]) if all_sky else gb["depth"]
    a = torch.zeros(H, W, 4, dtype=torch.uint8, device=DEV)
    ws = soc.cloud_rendering_workspace(W, H)
    soc.cloud_rendering(g, dev(depth), dev(gb["noise"]), a, None)
    monkeypatch.setenv("SOC_CLOUDS_OD_LUT", "0")   # every secondary ray marched, as the single-lane kernel does
    # wide: the sun-visibility kernel over the float-form row table (2, default; f16 pairs, v_fma_mix_f32), the float-form
    # quads (1) or the byte quads' integer form (0, as the single-lane kernel); the density over the row table or the
    # byte quads (0)
    for pos, geom, ntab, wide in (("0", "1", "1", "2"), ("1", "1", "1", "2"), ("2", "1", "1", "2"), ("2", "0", "1", "2"),
                                  ("2", "1", "0", "2"), ("2", "1", "1", "1"), ("2", "1", "0", "1"), ("2", "1", "1", "0"),
                                  ("2", "1", "0", "0")):
        monkeypatch.setenv("SOC_CLOUDS_ATMOS_POS", pos)
        monkeypatch.setenv("SOC_CLOUDS_GEOM", geom)   # the march geometry stored by density, or re-derived per pair
        monkeypatch.setenv("SOC_CLOUDS_NOISE_TABLE", ntab)   # noise quads prebuilt once per frame, or staged per workgroup
        monkeypatch.setenv("SOC_CLOUDS_SUNVIS_WIDE", wide)
        monkeypatch.setenv("SOC_CLOUDS_DENSITY_ROWS", "0" if wide == "0" else "1")
        soc.reload_tuning()
        b = torch.zeros_like(a)
        soc.cloud_rendering(g, dev(depth), dev(gb["noise"]), b, ws)
        torch.cuda.synchronize()
        assert torch.equal(a, b), (pos, geom, ntab, wide, (a != b).float().mean().item())
    monkeypatch.delenv("SOC_CLOUDS_SUNVIS_WIDE")
    monkeypatch.delenv("SOC_CLOUDS_DENSITY_ROWS")
    # with the secondary-ray table (the default) the prebuilt noise quads give the per-workgroup staging's bits too, for
    # the R8 and the RGBA8 noise image
    monkeypatch.delenv("SOC_CLOUDS_OD_LUT")
    noise_rgba = dev(gb["noise"]).clone()
    noise_rgba[..., 1:] = 77
    noise_r8 = noise_rgba[..., 0].contiguous()
    # ... and the resolve's od / vis loads (batches of 4, default, or 8 steps) and the density's od scratch reads (8, default, or 4) give
    # the one-step loops' bits
    outs = []
    for nz in (noise_r8, noise_rgba):
        for ntab, rb, dbt, pf, hoist in (("1", "4", "8", "1", "0"), ("0", "4", "4", "1", "1"), ("1", "1", "1", "0", "0"),
                                         ("1", "8", "8", "1", "1"), ("1", "4", "1", "0", "0")):
            monkeypatch.setenv("SOC_CLOUDS_CLASSIFY_HOIST", hoist)   # the classification's depth samples hoisted
            monkeypatch.setenv("SOC_CLOUDS_DENSITY_MULT", "2" if hoist == "1" else "1")
            monkeypatch.setenv("SOC_CLOUDS_NOISE_TABLE", ntab)
            monkeypatch.setenv("SOC_CLOUDS_RESOLVE_BATCH", rb)
            monkeypatch.setenv("SOC_CLOUDS_DENSITY_BATCH", dbt)
            monkeypatch.setenv("SOC_CLOUDS_SUNVIS_PF", pf)   # the sun-visibility kernel's next pair word loaded ahead
            soc.reload_tuning()
            b = torch.zeros_like(a)
            soc.cloud_rendering(g, dev(depth), nz, b, ws)
            outs.append(b)
    torch.cuda.synchronize()
    monkeypatch.delenv("SOC_CLOUDS_RESOLVE_BATCH")
    monkeypatch.delenv("SOC_CLOUDS_DENSITY_BATCH")
    monkeypatch.delenv("SOC_CLOUDS_SUNVIS_PF")
    monkeypatch.delenv("SOC_CLOUDS_CLASSIFY_HOIST")
    monkeypatch.delenv("SOC_CLOUDS_DENSITY_MULT")
    for o in outs[1:]:
        assert torch.equal(outs[0], o)
    monkeypatch.delenv("SOC_CLOUDS_ATMOS_POS")
    monkeypatch.delenv("SOC_CLOUDS_GEOM")
    monkeypatch.delenv("SOC_CLOUDS_NOISE_TABLE")
    soc.reload_tuning()


@pytest.mark.parametrize("config", ["c3", "c4"])
def test_clouds_od_table_against_marched_secondary_rays(soc, monkeypatch, config):
    """The atmosphere's secondary-ray optical-depth table (clouds.hip clouds_od_lut, the default) against marching every
    secondary ray (SOC_CLOUDS_OD_LUT=0) on the bench's 4K frames: the interpolated depths change a pixel by at most one
    RGBA8 level, on at most 0.1 % of the sky pixels (the oracle comparisons of test_clouds and the 4K frame tests bound
    the result against the reference restatement)."""
    import bench
    W, H = 3840, 2160
    g, gb, _sh, _nz, _sc, fr = bench.build_inputs(config, "mesh", W, H, 0, torch.device(DEV, 0))
    outs = []
    monkeypatch.setenv("SOC_CLOUDS_SKY_TABLE", "0")   # the secondary-ray table alone (the sky-view table: the next test)
    for lut in ("1", "0"):
        monkeypatch.setenv("SOC_CLOUDS_OD_LUT", lut)
        soc.reload_tuning()
        o = torch.zeros(H, W, 4, dtype=torch.uint8, device=DEV)
        soc.cloud_rendering(g, fr["depth"], fr["noise"], o, fr["clouds_workspace"])
        outs.append(o)
    torch.cuda.synchronize()
    d = (outs[0].int() - outs[1].int()).abs().amax(dim=-1)
    sky = torch.from_numpy(gb["depth"] == 1.0).to(DEV)
    assert int(d.max()) <= 1, int(d.max())
    assert float((d[sky] > 0).float().mean()) <= 1e-3, float((d[sky] > 0).float().mean())


@pytest.mark.parametrize("config", ["c3", "c4"])
def test_clouds_sky_table_against_every_pixel(soc, monkeypatch, config):
    """The atmosphere's per-frame sky-view table (clouds.hip clouds_sky_table, the default: the in-scattering integrals
    over elevation x azimuth-from-the-sun in three branches at the grazing directions, the phase applied per pixel)
    against evaluating the atmosphere for every sky pixel (SOC_CLOUDS_SKY_TABLE=0), both with the secondary-ray table, on
    the bench's 4K frames: at most one RGBA8 level anywhere, on at most 2 % of the sky pixels (the interpolation moves a
    channel by <= 0.04 levels in the float64 study, tools/sky_table_check.py, so only values next to a rounding edge
    flip). The oracle comparisons of test_clouds and the 4K frame tests bound the result against the restatement."""
    import bench
    W, H = 3840, 2160
    g, gb, _sh, _nz, _sc, fr = bench.build_inputs(config, "mesh", W, H, 0, torch.device(DEV, 0))
    outs = []
    for tab in ("1", "0"):
        monkeypatch.setenv("SOC_CLOUDS_SKY_TABLE", tab)
        soc.reload_tuning()
        o = torch.zeros(H, W, 4, dtype=torch.uint8, device=DEV)
        soc.cloud_rendering(g, fr["depth"], fr["noise"], o, fr["clouds_workspace"])
        outs.append(o)
    torch.cuda.synchronize()
    d = (outs[0].int() - outs[1].int()).abs().amax(dim=-1)
    sky = torch.from_numpy(gb["depth"] == 1.0).to(DEV)
    frac = float((d[sky] > 0).float().mean())
    print(f"sky table {config}: max {int(d.max())} levels, {frac:.5f} of the sky pixels differ")
    assert int(d.max()) <= 1, int(d.max())
    assert frac <= 0.02, frac


@pytest.mark.parametrize("cam_y", [2.2, 900.0])
def test_clouds_tables_sun_sweep(soc, monkeypatch, cam_y):
    """the two per-frame atmosphere tables (clouds.hip clouds_od_lut, clouds_sky_table) away from the bench's
    sun and camera: sun elevations from below the horizon to the zenith (the sky table's fallback axis), two azimuths,
    camera heights 2.2 and 900, an all-sky 960x540 frame looking at the horizon and up. Sky-view table on vs every
    pixel evaluated (SOC_CLOUDS_SKY_TABLE), and the secondary-ray table vs every secondary ray marched
    (SOC_CLOUDS_OD_LUT, sky table off): at most one RGBA8 level anywhere (cloud_rendering.inl:353-439)."""
    W, H = 960, 540
    worst = {}
    for pitch in (0.0, 0.7):
        g, gb = sponza_inputs(W, H, camera=((-14.0, cam_y, 0.3), (0.0, pitch, 0.0)), elapsed=10.0)
        depth = dev(np.ones_like(gb["depth"]))
        noise = dev(gb["noise"])
        ws = soc.cloud_rendering_workspace(W, H)
        for elev in (-8.0, 3.0, 35.0, 90.0):
            for az in (0.0, 2.4):
                e, a_ = np.radians(elev), az
                d = -np.array([np.cos(e) * np.cos(a_), np.sin(e), np.cos(e) * np.sin(a_)], np.float32)
                if elev == 90.0:
                    d = np.array([0.0, -1.0, 0.0], np.float32)
                g.sun_info.direction[:] = [float(v) for v in d]
                for knob, other in (("SOC_CLOUDS_SKY_TABLE", {}), ("SOC_CLOUDS_OD_LUT", {"SOC_CLOUDS_SKY_TABLE": "0"})):
                    outs = []
                    for v in ("1", "0"):
                        for k, vv in other.items():
                            monkeypatch.setenv(k, vv)
                        monkeypatch.setenv(knob, v)
                        soc.reload_tuning()
                        o = torch.zeros(H, W, 4, dtype=torch.uint8, device=DEV)
                        soc.cloud_rendering(g, depth, noise, o, ws)
                        outs.append(o)
                    for k in list(other) + [knob]:
                        monkeypatch.delenv(k)
                    torch.cuda.synchronize()
                    diff = (outs[0].int() - outs[1].int()).abs().amax(dim=-1)
                    key = (knob, pitch, elev, az)
                    worst[key] = (int(diff.max()), float((diff > 0).float().mean()))
    soc.reload_tuning()
    print("clouds tables sun sweep (max levels, fraction differing):", worst)
    bad = {k: v for k, v in worst.items() if v[0] > 1}
    assert not bad, bad


# ------------------------------------------------------------------------------------------------ full frame
@pytest.mark.parametrize("W,H,frames,inputs", [(256, 144, 3, "sponza"), (1920, 1080, 2, "sponza"),
                                               (320, 180, 2, "terrain"), (960, 540, 2, "terrain"),
                                               (97, 55, 2, "sponza"), (8200, 18, 2, "sponza"), (18, 1200, 2, "sponza")])
def test_render_graph_frames(soc, oracle, W, H, frames, inputs):
    """Multi-frame render graph (ping-pong TAA history, fused velocity history) vs the oracle frame, on the
    Sponza-proxy (C2/C3) and on the terrain (C4: half the frame is sky, so clouds dominate). Ragged and extreme
    shapes: an odd extent (no pair paths), a frame wider than the 8192-texel fast paths (TAA falls back to the
    generic kernel and the tone map runs as its own pass) and a tall narrow one (one-tile-wide grids)."""
    g, gb = (sponza_inputs if inputs == "sponza" else terrain_inputs)(W, H, elapsed=10.0)
    fr = soc.alloc_frame(W, H, DEV)
    for k in ("albedo", "emissive", "normal", "velocity", "depth"):
        fr[k].copy_(torch.from_numpy(gb[k]))
    fr["shadow"] = dev(gb["shadow"])
    fr["noise"].copy_(torch.from_numpy(gb["noise"]))
    r = soc.Renderer(fr, timing=True)
    hf = host_frame(W, H, gb)
    ae = soc.AutoExposure()
    hist = 0
    for f in range(frames):
        emis = dev(gb["emissive"])           # bloom overwrites emissive each frame (quirk Q5)
        fr["emissive"].copy_(emis)
        hf["emissive"][...] = gb["emissive"]
        e0 = soc.exposure_of(fr["auto_exposure"])
        r.execute(g)
        hist = oracle.frame(g, hf, ae, hist=hist)
        torch.cuda.synchronize()
        assert r.current_history() == hist
        frame_parity(soc, oracle, g, fr, hf, ae, hist, f"{inputs} {W}x{H} frame {f}", e0)
    ms = dict(zip(r.pass_names(), r.pass_ms()))
    # a one-call frame folds the partial histograms in the resolve: the fold pass is neither launched nor timed
    assert ms.pop("LuminanceHistogramFold") < 0
    assert all(m >= 0 for m in ms.values())
    r.close()


def test_render_graph_ao_first_issue_order_bit_identical(soc, monkeypatch):
    """The issue order of SSAOGeneration / SSAOBlur among the bloom passes they do not depend on
    (SOC_RENDERER_SSAO_FIRST: -1 default, before the last bloom pass; 1 first; 3 after two bloom passes; 0 the
    registration order) gives the same bits over 3 frames."""
    W, H = 960, 540
    g, gb = sponza_inputs(W, H, elapsed=10.0)
    outs = []
    for first in ("-1", "1", "3", "0"):
        monkeypatch.setenv("SOC_RENDERER_SSAO_FIRST", first)
        soc.reload_tuning()
        fr = soc.alloc_frame(W, H, DEV, bloom_output=True)
        for k in ("albedo", "emissive", "normal", "velocity", "depth"):
            fr[k].copy_(torch.from_numpy(gb[k]))
        fr["shadow"] = dev(gb["shadow"])
        fr["noise"].copy_(torch.from_numpy(gb["noise"]))
        r = soc.Renderer(fr)
        for _ in range(3):
            r.execute(g)
        torch.cuda.synchronize()
        outs.append({k: fr[k].clone() for k in ("color", "output", "auto_exposure", "ssao_blur", "bloom_output")})
        r.close()
    monkeypatch.delenv("SOC_RENDERER_SSAO_FIRST")
    soc.reload_tuning()
    for o in outs[1:]:
        for k in outs[0]:
            assert torch.equal(outs[0][k], o[k]), k


@pytest.mark.parametrize("W,H", [(320, 180), (1920, 1080)])
def test_fresh_renderers_first_frame_exposure(soc, oracle, W, H):
    """A renderer's first frame on a sky-heavy (terrain) view: the histogram scratch is allocated and cleared on
    first use, while the sky lane (a non-blocking stream) bins the sky pixels into it; the clear must land first.
    Several fresh renderers in a row (their frame buffers reuse freed memory), each frame 0 against the oracle."""
    g, gb = terrain_inputs(W, H, elapsed=10.0)
    hf0 = host_frame(W, H, gb)
    ae0 = soc.AutoExposure()
    oracle.frame(g, hf0, ae0, hist=0)
    for k in range(6):
        fr = soc.alloc_frame(W, H, DEV)
        for key in ("albedo", "emissive", "normal", "velocity", "depth"):
            fr[key].copy_(torch.from_numpy(gb[key]))
        fr["shadow"] = dev(gb["shadow"])
        fr["noise"].copy_(torch.from_numpy(gb["noise"]))
        r = soc.Renderer(fr)
        r.execute(g)
        torch.cuda.synchronize()
        assert abs(soc.exposure_of(fr["auto_exposure"]) - ae0.exposure) <= 1e-4, (k, soc.exposure_of(fr["auto_exposure"]),
                                                                                ae0.exposure)
        r.close()
        del fr


# ------------------------------------------------------------------------------------------------ 4K properties
def test_4k_properties(soc):
    """Size-independent properties at the benchmark resolution (oracle would take too long)."""
    W, H = 3840, 2160
    g = globals_for(W, H)
    # bloom chain of a constant emissive image stays constant (weights sum to 1, all exact)
    em = torch.full((H, W, 4), 0.5, dtype=torch.float16, device=DEV)
    mips = [torch.zeros(H >> i, W >> i, 4, dtype=torch.float16, device=DEV) for i in range(4)]
    soc.bloom_chain(g, em, mips)
    assert torch.all(em[..., :3] == 0.5)
    # blur of a constant AO image is the constant
    ao = torch.full((H // 2, W // 2), 200, dtype=torch.uint8, device=DEV)
    out = torch.zeros_like(ao)
    soc.ssao_blur(g, ao, out)
    assert torch.all(out == 200)
    # histogram counts every pixel exactly once
    buf = soc.auto_exposure_buffer()
    img = torch.rand(H, W, 4, device=DEV).half()
    soc.generate_luminance_histogram(g, img, buf)
    assert int(buf[1:].sum()) == W * H
    # TAA with identical history, zero velocity, and constant colour returns the colour
    c = torch.full((H, W, 4), 0.25, dtype=torch.float16, device=DEV)
    z = torch.zeros(H, W, 4, dtype=torch.float16, device=DEV)
    d = torch.full((H, W), 0.9, dtype=torch.float32, device=DEV)
    t = torch.zeros_like(c)
    soc.temporal_antialiasing(g, t, c, c.clone(), z, z.clone(), d)
    assert torch.all(t == 0.25)


# ------------------------------------------------------------------------------------------------ sky lane
def test_render_graph_sky_lane_bit_identical(soc):
    """The concurrent sky lane (CloudRendering on a renderer-owned stream, joined before Composition)
    changes scheduling only: 3 frames with and without it give bit-identical images."""
    W, H = 1920, 1080
    g, gb = sponza_inputs(W, H, elapsed=10.0)
    outs = []
    for lane in (True, False):
        fr = soc.alloc_frame(W, H, DEV, bloom_output=True)
        for k in ("albedo", "emissive", "normal", "velocity", "depth"):
            fr[k].copy_(torch.from_numpy(gb[k]))
        fr["shadow"] = dev(gb["shadow"])
        fr["noise"].copy_(torch.from_numpy(gb["noise"]))
        r = soc.Renderer(fr, sky_lane=lane)
        for _ in range(3):
            r.execute(g)
        torch.cuda.synchronize()
        outs.append({k: fr[k].clone() for k in ("clouds", "color", "output", "auto_exposure")})
        outs[-1]["resolved"] = r.resolved().clone()
        r.close()
    for o in outs[1:]:
        for k in outs[0]:
            assert torch.equal(outs[0][k], o[k]), k


def test_render_graph_split_phases_bit_identical(soc):
    """A multi-GPU frame runs PRE and POST in separate calls (the fused pass's partial histograms folded by
    the LuminanceHistogramFold launch before the exchange); a one-call frame folds them in the resolve.
    Without an exchange both give the same bits, over 3 frames, and leave the scratch zeroed."""
    W, H = 1920, 1080
    g, gb = sponza_inputs(W, H, elapsed=10.0)
    outs = []
    for split in (False, True):
        fr = soc.alloc_frame(W, H, DEV, bloom_output=True)
        for k in ("albedo", "emissive", "normal", "velocity", "depth"):
            fr[k].copy_(torch.from_numpy(gb[k]))
        fr["shadow"] = dev(gb["shadow"])
        fr["noise"].copy_(torch.from_numpy(gb["noise"]))
        r = soc.Renderer(fr)
        for _ in range(3):
            if split:
                r.execute(g, soc.PHASE_PRE_EXPOSURE)
                r.execute(g, soc.PHASE_POST_EXPOSURE)
            else:
                r.execute(g)
        torch.cuda.synchronize()
        outs.append({k: fr[k].clone() for k in ("color", "output", "auto_exposure")})
        r.close()
    for o in outs[1:]:
        for k in outs[0]:
            assert torch.equal(outs[0][k], o[k]), k
    assert int(outs[0]["auto_exposure"][1:].abs().sum()) == 0   # bins consumed by the resolve


def test_render_graph_c3b_lights(soc, oracle):
    """Config C3b: 128 point lights from the ECS scene feed (soc_scene_update, scene.cpp:47-118) through the render
    graph (per-frame globals upload, composition light loops) against the oracle's composition."""
    import bench
    W, H = 320, 180
    g, gb = sponza_inputs(W, H, elapsed=10.0)
    soc.scene_update(g, bench.point_lights_c3b())
    assert g.point_light_count == 128
    fr = soc.alloc_frame(W, H, DEV, bloom_output=True)
    for k in ("albedo", "emissive", "normal", "velocity", "depth"):
        fr[k].copy_(torch.from_numpy(gb[k]))
    fr["shadow"] = dev(gb["shadow"])
    fr["noise"].copy_(torch.from_numpy(gb["noise"]))
    r = soc.Renderer(fr)
    r.execute(g)
    torch.cuda.synchronize()
    ref = np.zeros((H, W, 4), np.float16)
    oracle.composition(g, ref, gb["albedo"], host(fr["bloom_output"]), gb["normal"], gb["depth"], host(fr["ssao_blur"]),
                       gb["shadow"], host(fr["clouds"]))
    ok = f16_close(host(fr["color"]), ref)
    assert ok.mean() >= 0.9995, ok.mean()
    r.close()


@pytest.mark.parametrize("phases", ["one-call", "split"])
def test_render_graph_sky_split_bit_identical(soc, monkeypatch, phases):
    """Sky split: the second lane writes and bins the colour image's sky pixels after the clouds, Composition skips
    them and does not wait. Against Composition writing them itself: the same bits over 3 frames (colour, output,
    exposure, resolved history), for one-call frames and PRE / POST frames (the multi-GPU shape), with the sky pass
    reading a pixel pair's clouds texels in one load (default) or one by one (SOC_SKY_COMPOSE_PAIR_LOAD=0)."""
    W, H = 1920, 1080
    g, gb = sponza_inputs(W, H, elapsed=10.0, camera=((-14.0, 2.2, 0.3), (0.0, -0.9, 0.0)))   # looking up: more sky
    assert (gb["depth"] == 1.0).mean() > 0.05
    outs = []
    for split, cp in ((True, "1"), (True, "0"), (False, "1")):
        monkeypatch.setenv("SOC_SKY_COMPOSE_PAIR_LOAD", cp)
        soc.reload_tuning()
        fr = soc.alloc_frame(W, H, DEV, bloom_output=True)
        for k in ("albedo", "emissive", "normal", "velocity", "depth"):
            fr[k].copy_(torch.from_numpy(gb[k]))
        fr["shadow"] = dev(gb["shadow"])
        fr["noise"].copy_(torch.from_numpy(gb["noise"]))
        r = soc.Renderer(fr, sky_split=split)
        for _ in range(3):
            if phases == "split":
                r.execute(g, soc.PHASE_PRE_EXPOSURE)
                r.execute(g, soc.PHASE_POST_EXPOSURE)
            else:
                r.execute(g)
        torch.cuda.synchronize()
        outs.append({k: fr[k].clone() for k in ("clouds", "color", "output", "auto_exposure")})
        outs[-1]["resolved"] = r.resolved().clone()
        r.close()
    monkeypatch.delenv("SOC_SKY_COMPOSE_PAIR_LOAD")
    soc.reload_tuning()
    for o in outs[1:]:
        for k in outs[0]:
            assert torch.equal(outs[0][k], o[k]), k


@pytest.mark.parametrize("inputs", ["sponza", "terrain"])
def test_render_graph_static_inputs_bit_identical(soc, inputs):
    """SOC_RENDERER_STATIC_INPUTS lets the second lane start a frame's CloudRendering before the fork (it has no ring
    edge onto the main lane), overlapping the previous frame's composition and TAA; SkyCompose still waits for the
    previous frame's TAA and resolve. Four frames with per-frame globals (camera moving, jitter, time) on one resident
    G-buffer: the same bits as forking at every frame start, sky-heavy terrain included."""
    import ctypes as C
    W, H = 1920, 1080
    g0, gb = (sponza_inputs if inputs == "sponza" else terrain_inputs)(W, H, elapsed=10.0)
    outs = []
    for static in (True, False):
        fr = soc.alloc_frame(W, H, DEV, bloom_output=True)
        for k in ("albedo", "emissive", "normal", "velocity", "depth"):
            fr[k].copy_(torch.from_numpy(gb[k]))
        fr["shadow"] = dev(gb["shadow"])
        fr["noise"].copy_(torch.from_numpy(gb["noise"]))
        r = soc.Renderer(fr, static_inputs=static)
        cam = soc.make_camera((-14.0, 2.2, 0.3), (0.0, -0.42, 0.0))
        ji = C.c_uint32(0)
        g = soc.globals_defaults(W, H)
        seq = []
        for f in range(4):
            soc.frame_update(g, cam, W, H, 0.016, ji)
            cam.position[0] += 0.05
            r.execute(g)
            # main-lane outputs read on the caller's stream between frames (CLOUDS, the second lane's intermediate, may
            # already hold the next frame's clouds by then: not read between frames under the flag)
            seq.append({k: fr[k].clone() for k in ("color", "output")})
        torch.cuda.synchronize()
        seq.append({"auto_exposure": fr["auto_exposure"].clone(), "resolved": r.resolved().clone(),
                    "clouds": fr["clouds"].clone()})
        outs.append(seq)
        r.close()
    for a, b in zip(*outs):
        for k in a:
            assert torch.equal(a[k], b[k]), k


def test_velocity_slots_bit_identical(soc):
    """SOC_RENDERER_VELOCITY_SLOTS: the frame's velocity is written into the history_velocity slot the next frame reads as
    its previous velocity (Renderer.velocity_slot()), instead of TAA copying images.velocity there (renderer.cpp:1185-1189).
    Four frames with a different velocity field each (written by the caller before the frame) and a moving camera: every
    frame's colour, framebuffer and resolved history, and the final velocity history slot, have the same bits as the
    copy. A caller pass declaring VELOCITY receives the slot as images->velocity, and its declared uses widen to both
    slots (PREVIOUS_VELOCITY too), which orders the next frame's velocity write after it."""
    import ctypes as C
    W, H = 1920, 1080
    _g0, gb = sponza_inputs(W, H, elapsed=10.0)
    gen = torch.Generator(device=DEV).manual_seed(7)
    base = torch.from_numpy(gb["velocity"]).to(DEV)
    fields = [base + (torch.rand(base.shape, generator=gen, device=DEV).half() - 0.5) * (0.002 * f) for f in range(4)]
    outs = []
    for slots in (False, True):
        fr = soc.alloc_frame(W, H, DEV, bloom_output=True)
        for k in ("albedo", "emissive", "normal", "velocity", "depth"):
            fr[k].copy_(torch.from_numpy(gb[k]))
        fr["shadow"] = dev(gb["shadow"])
        fr["noise"].copy_(torch.from_numpy(gb["noise"]))
        r = soc.Renderer(fr, velocity_slots=slots)
        seen = []

        def probe(gp, images, s):
            seen.append(images.contents.velocity.data)
            return 0
        r.add_pass("VelocityProbe", probe, reads=["VELOCITY"], phase=soc.PHASE_POST_EXPOSURE)
        idx = r.pass_names().index("VelocityProbe")
        reads, _writes = r.pass_uses(idx)
        assert ("PREVIOUS_VELOCITY" in reads) == slots, reads
        cam = soc.make_camera((-14.0, 2.2, 0.3), (0.0, -0.42, 0.0))
        ji = C.c_uint32(0)
        g = soc.globals_defaults(W, H)
        seq, expect = [], []
        for f in range(4):
            soc.frame_update(g, cam, W, H, 0.016, ji)
            cam.position[0] += 0.05
            target = fr["history_velocity"][r.velocity_slot()] if slots else fr["velocity"]
            target.copy_(fields[f])
            expect.append(target.data_ptr())
            r.execute(g)
            seq.append({k: fr[k].clone() for k in ("color", "output")} | {"resolved": r.resolved().clone()})
        torch.cuda.synchronize()
        seq.append({"velocity_history": fr["history_velocity"][r.current_history()].clone(),
                    "auto_exposure": fr["auto_exposure"].clone()})
        assert seen == expect, (slots, seen, expect)
        outs.append(seq)
        r.close()
    for a, b in zip(*outs):
        for k in a:
            assert torch.equal(a[k], b[k]), k
    assert torch.equal(outs[1][-1]["velocity_history"], fields[-1])


@pytest.mark.parametrize("inputs,lights", [("sponza", False), ("terrain", False), ("sponza", True)])
def test_bloom_in_composition_bit_identical(soc, monkeypatch, inputs, lights):
    """SOC_RENDERER_BLOOM_IN_COMPOSITION: the bloom chain's last stage (mip1 -> [mip0] -> output) computed per 32 x 16
    tile inside the fused Composition + histogram launch instead of its own pass (bloomw_up10s, 64 x 16 tiles) writing
    the full-resolution bloom output that Composition reads back; active in frames whose sky lane is the critical path
    (here forced: a high-priority sky lane, SOC_RENDERER_SIDE_QUEUE=1). Three frames with per-frame
    globals: the colour, framebuffer, exposure and resolved history have the same bits (the bloom values are functions
    of their clamped coordinates only, rounded to RGBA16F as the chain stores them), with and without point lights (the
    lights kernel); Composition declares BLOOM_MIP1, and the fourth bloom pass is skipped: the bloom output image is not
    written."""
    import ctypes as C

    import bench
    monkeypatch.setenv("SOC_RENDERER_SIDE_QUEUE", "1")
    soc.reload_tuning()
    W, H = 1920, 1080
    g0, gb = (sponza_inputs if inputs == "sponza" else terrain_inputs)(W, H, elapsed=10.0)
    # a dense emissive field on top of the scene's (the box atrium's lamps cover 0.7 % of the pixels, the terrain none)
    gen = torch.Generator(device=DEV).manual_seed(3)
    emis = torch.from_numpy(gb["emissive"]).to(DEV) + (torch.rand((H, W, 4), generator=gen, device=DEV) ** 4 * 3).half()
    outs = []
    for fused in (False, True):
        fr = soc.alloc_frame(W, H, DEV, bloom_output=True)
        for k in ("albedo", "normal", "velocity", "depth"):
            fr[k].copy_(torch.from_numpy(gb[k]))
        fr["emissive"].copy_(emis)
        fr["shadow"] = dev(gb["shadow"])
        fr["noise"].copy_(torch.from_numpy(gb["noise"]))
        fr["bloom_output"].fill_(7.0)
        r = soc.Renderer(fr, static_inputs=True, bloom_in_composition=fused)
        names = r.pass_names()
        assert "BloomUpsample - 1+0" in names, names
        reads, _w = r.pass_uses(names.index("Composition+GenerateLuminanceHistogram"))
        assert ("BLOOM_MIP1" in reads) == fused and "BLOOM_OUTPUT" in reads, reads
        cam = soc.make_camera((-14.0, 2.2, 0.3), (0.0, -0.42, 0.0))
        ji = C.c_uint32(0)
        g = soc.globals_defaults(W, H)
        seq = []
        for f in range(3):
            soc.frame_update(g, cam, W, H, 0.016, ji)
            if lights:
                soc.scene_update(g, bench.point_lights_c3b())
            cam.position[0] += 0.05
            r.execute(g)
            seq.append({k: fr[k].clone() for k in ("color", "output")})
            if f == 0:   # the lane takes its (forced) queue in the first call: in-kernel from the second frame on
                assert r.side_queue() == 1
                fr["bloom_output"].fill_(7.0)
        torch.cuda.synchronize()
        seq.append({"auto_exposure": fr["auto_exposure"].clone(), "resolved": r.resolved().clone()})
        assert bool((fr["bloom_output"] == 7.0).all()) == fused
        outs.append(seq)
        r.close()
    monkeypatch.delenv("SOC_RENDERER_SIDE_QUEUE")
    soc.reload_tuning()
    for a, b in zip(*outs):
        for k in a:
            assert torch.equal(a[k], b[k]), k


def test_bloom_in_composition_generic_resolution_frame(soc):
    """the in-Composition bloom stage is decided per frame. A frame whose globals resolution differs from the
    image extent takes Composition's generic path, which cannot compute the bloom, so the chain's fourth pass must run:
    with the sky split off, a high-priority sky lane and bloom_in_composition, such a frame executes (round 5 skipped the
    fourth pass and Composition then returned SOC_E_SHAPE) and writes the bloom output, and a matching frame after it
    computes the bloom in Composition again (the bloom output untouched)."""
    W, H = 640, 360
    g, gb = sponza_inputs(W, H, elapsed=10.0)
    fr = soc.alloc_frame(W, H, DEV, bloom_output=True)
    for k in ("albedo", "emissive", "normal", "velocity", "depth"):
        fr[k].copy_(torch.from_numpy(gb[k]))
    fr["shadow"] = dev(gb["shadow"])
    fr["noise"].copy_(torch.from_numpy(gb["noise"]))
    r = soc.Renderer(fr, static_inputs=True, sky_split=False, bloom_in_composition=True, sky_lane_queue="high")
    r.execute(g)                                   # the lane takes its queue in the first call
    torch.cuda.synchronize()
    assert r.side_queue() == 1
    g_generic = type(g)()
    C.pointer(g_generic)[0] = g
    g_generic.resolution[0] = W - 2                # the generic composition path
    fr["bloom_output"].fill_(7.0)
    r.execute(g_generic)
    torch.cuda.synchronize()
    assert not bool((fr["bloom_output"] == 7.0).all())   # the fourth pass ran
    fr["bloom_output"].fill_(7.0)
    r.execute(g)
    torch.cuda.synchronize()
    assert bool((fr["bloom_output"] == 7.0).all())       # in Composition again
    r.close()


@pytest.mark.parametrize("inputs", ["sponza", "terrain"])
def test_sky_lane_queue_probe_bit_identical(soc, monkeypatch, inputs):
    """The sky lane's hardware queue (SOC_RENDERER_SIDE_QUEUE): auto (3, default) runs eight windows alternating between
    a high- and a low-priority stream (ABBA pairs; with the sky-bound clouds variants in the high windows) and then keeps
    one, moving the lane between streams with an event wait; 1 / 2 fix it, 0 is the normal-priority stream. Every
    frame's output (every 8th texel) and the final temporal state have the same bits in every mode (the probe's frames
    + 3, per-frame globals, static inputs: the clouds of frame N+1 start before frame N's TAA, also across the
    switches), and auto has chosen a queue by the end."""
    import ctypes as C
    W, H = 1920, 1080
    g0, gb = (sponza_inputs if inputs == "sponza" else terrain_inputs)(W, H, elapsed=10.0)
    outs, chosen = [], []
    n_frames = 0
    for mode in ("3", "0", "1", "2"):   # auto first: its probe length sets the frame count of every mode
        monkeypatch.setenv("SOC_RENDERER_SIDE_QUEUE", mode)
        soc.reload_tuning()
        fr = soc.alloc_frame(W, H, DEV, bloom_output=True)
        for k in ("albedo", "emissive", "normal", "velocity", "depth"):
            fr[k].copy_(torch.from_numpy(gb[k]))
        fr["shadow"] = dev(gb["shadow"])
        fr["noise"].copy_(torch.from_numpy(gb["noise"]))
        r = soc.Renderer(fr, static_inputs=True)
        cam = soc.make_camera((-14.0, 2.2, 0.3), (0.0, -0.42, 0.0))
        ji = C.c_uint32(0)
        g = soc.globals_defaults(W, H)
        seq = []
        if mode == "3":
            n_frames = r.side_queue_probe_frames() + 3
            assert n_frames > 16
        for f in range(n_frames):
            soc.frame_update(g, cam, W, H, 0.016, ji)
            cam.position[0] += 0.001
            r.execute(g)
            seq.append(fr["output"][::8, ::8].clone())   # every 8th texel of every frame (and the final state in full)
            if f == n_frames - 3:
                torch.cuda.synchronize()   # the probe's last event has completed: the next frames decide
        torch.cuda.synchronize()
        seq.append(fr["output"].clone())
        seq.append(fr["auto_exposure"].clone())
        seq.append(r.resolved().clone())
        outs.append(seq)
        chosen.append(r.side_queue())
        r.close()
    monkeypatch.delenv("SOC_RENDERER_SIDE_QUEUE")
    soc.reload_tuning()
    assert chosen[0] in (1, 2) and chosen[1] == 0 and chosen[2] == 1 and chosen[3] == 2, chosen
    for o in outs[1:]:
        for f, (a, b) in enumerate(zip(outs[0], o)):
            assert torch.equal(a, b), f


def test_sky_lane_queue_flags(soc):
    """The sky lane's queue is fixed by the renderer flags (round 6, VERDICT r5 #2: the same kernels every run): low
    priority by default, high with sky_lane_queue="high" (SOC_RENDERER_SKY_LANE_HIGH), the timed probe only with
    "probe" (undecided after one frame); no tuning knob set. The frames have the same bits in every mode."""
    W, H = 640, 360
    g, gb = terrain_inputs(W, H, elapsed=10.0)
    outs = []
    for q, want in (("low", 2), ("high", 1), ("probe", -1)):
        fr = soc.alloc_frame(W, H, DEV, bloom_output=True)
        for k in ("albedo", "emissive", "normal", "velocity", "depth"):
            fr[k].copy_(torch.from_numpy(gb[k]))
        fr["shadow"] = dev(gb["shadow"])
        fr["noise"].copy_(torch.from_numpy(gb["noise"]))
        r = soc.Renderer(fr, static_inputs=True, sky_lane_queue=q)
        r.execute(g)
        torch.cuda.synchronize()
        assert r.side_queue() == want, (q, r.side_queue())
        outs.append(fr["output"].clone())
        r.close()
    for o in outs[1:]:
        assert torch.equal(o, outs[0])
    with pytest.raises(ValueError):
        soc.Renderer(fr, sky_lane_queue="fast")


def test_static_inputs_first_call_after_async_input_write(soc):
    """SOC_RENDERER_STATIC_INPUTS: the first call after create (and after a graph rebuild) forks the second
    lane before CloudRendering, so inputs the caller wrote on its stream just before that call are seen. The terrain
    depth is written by a copy queued on the caller's stream behind ~tens of ms of other work (the depth image holds
    zeros, i.e. no sky, until then); the frame must equal the one rendered from synchronously written inputs."""
    W, H = 1920, 1080
    g, gb = terrain_inputs(W, H, elapsed=10.0)
    outs = []
    for delayed in (False, True):
        fr = soc.alloc_frame(W, H, DEV, bloom_output=True)
        for k in ("albedo", "emissive", "normal", "velocity"):
            fr[k].copy_(torch.from_numpy(gb[k]))
        fr["shadow"] = dev(gb["shadow"])
        fr["noise"].copy_(torch.from_numpy(gb["noise"]))
        src = dev(gb["depth"])
        s = torch.cuda.Stream()
        r = soc.Renderer(fr, static_inputs=True, stream=s)
        torch.cuda.synchronize()
        if delayed:
            fr["depth"].zero_()
            torch.cuda.synchronize()
            with torch.cuda.stream(s):
                a = torch.randn(4096, 4096, device=DEV)
                for _ in range(40):            # keep the caller's stream busy before the depth write
                    a = torch.tanh(a @ a * 1e-3)
                fr["depth"].copy_(src)
        else:
            fr["depth"].copy_(src)
            torch.cuda.synchronize()
        r.execute(g, stream=s)
        torch.cuda.synchronize()
        outs.append({k: fr[k].clone() for k in ("clouds", "color", "output")})
        r.close()
    for k in outs[0]:
        assert torch.equal(outs[0][k], outs[1][k]), k
