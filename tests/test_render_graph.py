"""The render graph's pass declarations (CPU: no GPU call is made; graph construction and introspection only).

The reference registers tasks with add_task in renderer.cpp:965-1217, each with a uses block (e.g.
composition.inl:10-21); Daxa derives the barriers from those uses. The graph here keeps the registration
order and derives the dependencies and the second-lane placement from the declared uses."""
import ctypes as C

import pytest

# the live task order of Renderer::rebuild_task_graph (renderer.cpp:1024-1217) without a raster head:
# SSR (dead, Q12) and the ImGui draw are not rebuilt; the two CopyImageTasks are the TAA ping-pong
REFERENCE_ORDER = ["BloomDownsample - 0", "BloomDownsample - 1", "BloomDownsample - 2", "BloomDownsample - 3",
                   "BloomUpsample - 3", "BloomUpsample - 2", "BloomUpsample - 1", "BloomUpsample - 0",
                   "SSAOGeneration", "SSAOBlur", "CloudRendering", "Composition", "GenerateLuminanceHistogram",
                   "ResolveLuminanceHistogram", "TemporalAntiAliasing", "ToneMapping"]


def _renderer(soc, **kw):
    fr = soc.alloc_frame(128, 64, device="cpu", noise_table=False)   # exactly halving bloom mips
    return soc.Renderer(fr, **kw)


def _deps(r):
    names = r.pass_names()
    return {names[i]: {names[j] for j in r.pass_dependencies(i)} for i in range(len(names))}


def test_unfused_graph_is_the_reference_task_list(soc):
    r = _renderer(soc, fused_bloom=False, fused_tonemap=False, fused_histogram=False)
    assert r.pass_names() == REFERENCE_ORDER


def test_default_graph_order(soc):
    r = _renderer(soc)
    assert r.pass_names() == ["BloomDownsample - 0+1", "BloomDownsample - 2+3", "BloomUpsample - 3+2",
                              "BloomUpsample - 1+0", "SSAOGeneration", "SSAOBlur", "CloudRendering", "SkyCompose",
                              "Composition+GenerateLuminanceHistogram", "LuminanceHistogramFold",
                              "ResolveLuminanceHistogram", "TemporalAntiAliasing+ToneMapping"]


def test_declared_uses_follow_the_reference_bindings(soc):
    r = _renderer(soc, fused_bloom=False, fused_tonemap=False, fused_histogram=False)
    uses = {n: r.pass_uses(i) for i, n in enumerate(r.pass_names())}
    # renderer.cpp:1064-1079, 1094-1117, 1155-1217
    assert uses["SSAOGeneration"] == ({"DEPTH", "NORMAL"}, {"SSAO"})
    assert uses["SSAOBlur"] == ({"SSAO"}, {"SSAO_BLUR"})
    assert uses["CloudRendering"] == ({"DEPTH", "NOISE"}, {"CLOUDS"})
    assert uses["Composition"] == ({"ALBEDO", "EMISSIVE", "NORMAL", "DEPTH", "SSAO_BLUR", "SUN_SHADOW", "CLOUDS"},
                                   {"COLOR"})
    assert uses["GenerateLuminanceHistogram"] == ({"COLOR"}, {"AUTO_EXPOSURE"})
    assert uses["ToneMapping"] == ({"RESOLVED", "AUTO_EXPOSURE"}, {"OUTPUT"})
    assert uses["BloomUpsample - 0"] == ({"BLOOM_MIP0"}, {"EMISSIVE"})   # quirk Q5: overwrites emissive


def test_derived_dependencies(soc):
    r = _renderer(soc, fused_bloom=False, fused_tonemap=False, fused_histogram=False)
    d = _deps(r)
    assert d["BloomDownsample - 0"] == set()
    assert d["BloomDownsample - 1"] == {"BloomDownsample - 0"}
    # reads mip3 (RAW on down 3), overwrites mip2 (WAW on down 2, WAR on down 3 which read it)
    assert d["BloomUpsample - 3"] == {"BloomDownsample - 2", "BloomDownsample - 3"}
    assert d["SSAOGeneration"] == set()
    assert d["SSAOBlur"] == {"SSAOGeneration"}
    assert d["CloudRendering"] == set()
    # composition reads the bloomed emissive, the blurred AO and the clouds; the bloom chain read the emissive
    assert d["Composition"] == {"BloomUpsample - 0", "SSAOBlur", "CloudRendering"}
    assert d["GenerateLuminanceHistogram"] == {"Composition"}
    assert d["ResolveLuminanceHistogram"] == {"GenerateLuminanceHistogram"}
    assert d["TemporalAntiAliasing"] == {"Composition"}
    assert d["ToneMapping"] == {"TemporalAntiAliasing", "ResolveLuminanceHistogram"}


def test_every_pass_reaches_the_framebuffer(soc):
    """No dead pass: every pass is an ancestor of the one that writes the framebuffer."""
    for kw in ({}, dict(fused_bloom=False, fused_tonemap=False, fused_histogram=False)):
        r = _renderer(soc, **kw)
        names = r.pass_names()
        deps = [r.pass_dependencies(i) for i in range(len(names))]
        last = max(i for i in range(len(names)) if "OUTPUT" in r.pass_uses(i)[1])
        seen, todo = {last}, [last]
        while todo:
            for j in deps[todo.pop()]:
                if j not in seen:
                    seen.add(j)
                    todo.append(j)
        assert seen == set(range(len(names))), [names[i] for i in set(range(len(names))) - seen]


def test_second_lane_is_derived(soc):
    r = _renderer(soc)
    names = r.pass_names()
    lanes = {n: r.pass_lane(i) for i, n in enumerate(names)}
    assert [n for n, l in lanes.items() if l == 1] == ["CloudRendering", "SkyCompose"]
    # sky split (default): the second lane also writes and bins the colour's sky pixels (SkyCompose), so Composition
    # does not wait for it; the histogram fold (its partial bins) and TAA (the sky pixels) do
    assert r.pass_uses(names.index("CloudRendering"))[1] == {"CLOUDS"}
    assert r.pass_uses(names.index("SkyCompose")) == ({"CLOUDS", "DEPTH"}, {"SKY_COLOR", "SKY_HISTOGRAM_PARTIALS"})
    assert "CLOUDS" not in r.pass_uses(names.index("Composition+GenerateLuminanceHistogram"))[0]
    waiters = [n for n, d in _deps(r).items() if "SkyCompose" in d]
    assert waiters == ["LuminanceHistogramFold", "TemporalAntiAliasing+ToneMapping"]
    assert [n for n, d in _deps(r).items() if "CloudRendering" in d] == ["SkyCompose"]
    # without the split only the composition waits for it
    r2 = _renderer(soc, sky_split=False)
    waiters = [n for n, d in _deps(r2).items() if "CloudRendering" in d]
    assert waiters == ["Composition+GenerateLuminanceHistogram"]


def test_raster_head_dependencies(soc):
    """With a raster head the clouds wait for the G-buffer (they read depth), not for the frame start."""
    r = _renderer(soc)
    sc = soc._abi.RasterScene()
    for f in ("positions", "normals", "uvs", "indices"):
        setattr(sc.mesh, f, 1)
    sc.mesh.vertex_count, sc.mesh.triangle_count = 3, 1
    sc.materials, sc.material_count, sc.shadow, sc.visibility, sc.workspace = 1, 1, 1, 1, 1
    assert soc.lib().soc_renderer_set_raster_scene(r.handle, C.byref(sc)) == 0
    names = r.pass_names()
    assert names[:3] == ["DepthPrepass", "SunShadowDraw", "GBufferGeneration"]
    d = _deps(r)
    assert d["GBufferGeneration"] == {"DepthPrepass"}
    assert d["CloudRendering"] == {"GBufferGeneration"}
    assert d["SSAOGeneration"] == {"GBufferGeneration"}
    assert "SunShadowDraw" in d["Composition+GenerateLuminanceHistogram"]
    # the bloom reads the emissive the G-buffer pass writes
    assert d["BloomDownsample - 0+1"] == {"GBufferGeneration"}


def test_add_pass(soc):
    r = _renderer(soc)
    calls = []
    r.add_pass("RawAO", lambda g, im, s: calls.append(s), reads=["SSAO"], writes=["SSAO_BLUR"],
               before="Composition+GenerateLuminanceHistogram", group="Ambient Occlusion")
    names = r.pass_names()
    assert names.index("RawAO") == names.index("Composition+GenerateLuminanceHistogram") - 1
    d = _deps(r)
    assert d["RawAO"] == {"SSAOGeneration", "SSAOBlur"}      # RAW on SSAO, WAW on SSAO_BLUR
    assert "RawAO" in d["Composition+GenerateLuminanceHistogram"]
    # appended at the end of its phase when no anchor is given
    r.add_pass("PostFx", lambda g, im, s: 0, reads=["OUTPUT"], writes=["OUTPUT"], phase=soc.PHASE_POST_EXPOSURE)
    assert r.pass_names()[-1] == "PostFx"
    assert _deps(r)["PostFx"] == {"TemporalAntiAliasing+ToneMapping"}
    # a caller resource
    r.add_pass("MakeMask", lambda g, im, s: 0, reads=["DEPTH"], writes=[soc._abi.RES_USER0 + 3],
               before="SSAOGeneration")
    r.add_pass("UseMask", lambda g, im, s: 0, reads=[soc._abi.RES_USER0 + 3], writes=["SSAO"], before="SSAOBlur")
    assert _deps(r)["UseMask"] == {"MakeMask", "SSAOGeneration"}
    assert r.pass_uses(r.pass_names().index("MakeMask"))[1] == {"USER3"}


def test_add_pass_errors(soc):
    r = _renderer(soc)
    n0 = r.pass_names()
    with pytest.raises(soc.SocError, match="duplicate"):
        r.add_pass("SSAOBlur", lambda *a: 0)
    with pytest.raises(soc.SocError, match="no pass named"):
        r.add_pass("X", lambda *a: 0, before="NoSuchPass")
    with pytest.raises(soc.SocError, match="another phase"):
        r.add_pass("X", lambda *a: 0, before="ResolveLuminanceHistogram")     # PRE pass before a POST one
    with pytest.raises(soc.SocError, match="bad resource"):
        r.add_pass("X", lambda *a: 0, reads=[64])
    assert r.pass_names() == n0                                               # failed adds leave the graph as it was


def test_caller_passes_survive_raster_scene_changes(soc):
    r = _renderer(soc)
    r.add_pass("RawAO", lambda *a: 0, reads=["SSAO"], writes=["SSAO_BLUR"], before="Composition+GenerateLuminanceHistogram")
    assert soc.lib().soc_renderer_set_raster_scene(r.handle, None) == 0
    assert "RawAO" in r.pass_names()


def _carry(r):
    names = r.pass_names()
    return {names[i]: {names[j] for j in r.pass_carry_dependencies(i)} for i in range(len(names))}


def _cross_lane_ring_edges(r):
    names = r.pass_names()
    return {(names[i], names[j]) for i in range(len(names)) for j in r.pass_carry_dependencies(i)
            if r.pass_lane(i) != r.pass_lane(j)}


def _raster_renderer(soc, **kw):
    r = _renderer(soc, **kw)
    sc = soc._abi.RasterScene()
    for f in ("positions", "normals", "uvs", "indices"):
        setattr(sc.mesh, f, 1)
    sc.mesh.vertex_count, sc.mesh.triangle_count = 3, 1
    sc.materials, sc.material_count, sc.shadow, sc.visibility, sc.workspace = 1, 1, 1, 1, 1
    assert soc.lib().soc_renderer_set_raster_scene(r.handle, C.byref(sc)) == 0
    return r


def test_ring_edges(soc):
    """Cross-frame dependencies: the pass list as a ring (renderer.cpp:1155-1217 run frame after frame)."""
    r = _renderer(soc)
    c = _carry(r)
    # the second lane's sky writes follow the previous frame's readers of the colour's sky pixels (TAA) and the
    # resolve that folded and cleared the partial bins; CLOUDS is rewritten after the previous frame's SkyCompose read it
    assert c["SkyCompose"] == {"SkyCompose", "ResolveLuminanceHistogram", "TemporalAntiAliasing+ToneMapping"}
    assert c["CloudRendering"] == {"CloudRendering", "SkyCompose"}      # no cross-lane ring edge
    # composition's colour write follows the previous frame's TAA read and its own write (same lane); its partials
    # follow the resolve
    assert c["Composition+GenerateLuminanceHistogram"] == {"Composition+GenerateLuminanceHistogram",
                                                           "ResolveLuminanceHistogram", "TemporalAntiAliasing+ToneMapping"}
    # the TAA history ping-pong: this frame's PREVIOUS_COLOR is the last frame's RESOLVED (and vice versa)
    assert c["TemporalAntiAliasing+ToneMapping"] == {"TemporalAntiAliasing+ToneMapping"}
    # the bloom writes follow the previous frame's readers of its mips / output (same lane)
    assert "Composition+GenerateLuminanceHistogram" in c["BloomUpsample - 1+0"]
    assert _cross_lane_ring_edges(r) == {("SkyCompose", "ResolveLuminanceHistogram"),
                                         ("SkyCompose", "TemporalAntiAliasing+ToneMapping")}


def test_ring_edges_raster_head(soc):
    """With a raster head the G-buffer pass rewrites depth every frame: it must follow the previous frame's
    CloudRendering (second lane), which reads depth: the cross-lane WAR edge the end-of-call join used to cover."""
    r = _raster_renderer(soc)
    c = _carry(r)
    assert "CloudRendering" in c["GBufferGeneration"]
    assert {"SSAOGeneration", "TemporalAntiAliasing+ToneMapping"} <= c["GBufferGeneration"]
    assert c["DepthPrepass"] == {"DepthPrepass", "GBufferGeneration"}   # WAW / WAR on the visibility buffer
    assert _cross_lane_ring_edges(r) == {("SkyCompose", "ResolveLuminanceHistogram"),
                                         ("SkyCompose", "TemporalAntiAliasing+ToneMapping"),
                                         ("GBufferGeneration", "CloudRendering"), ("GBufferGeneration", "SkyCompose")}


def test_ring_edges_without_sky_split(soc):
    r = _renderer(soc, sky_split=False)
    # CloudRendering rewrites CLOUDS, which the previous frame's composition read (across the lanes)
    assert _cross_lane_ring_edges(r) == {("CloudRendering", "Composition+GenerateLuminanceHistogram")}


def test_caller_colour_use_includes_sky_pixels(soc):
    """Under the sky split a caller pass declaring COLOR also orders against the second lane's sky writes."""
    r = _renderer(soc)
    r.add_pass("ColorProbe", lambda *a: 0, reads=["COLOR"], writes=[soc._abi.RES_USER0], phase=soc.PHASE_POST_EXPOSURE,
               before="TemporalAntiAliasing+ToneMapping")
    names = r.pass_names()
    i = names.index("ColorProbe")
    assert r.pass_uses(i)[0] == {"COLOR", "SKY_COLOR"}
    assert "SkyCompose" in _deps(r)["ColorProbe"]
    r2 = _renderer(soc, sky_split=False)
    r2.add_pass("ColorProbe", lambda *a: 0, reads=["COLOR"], phase=soc.PHASE_POST_EXPOSURE)
    assert r2.pass_uses(r2.pass_names().index("ColorProbe"))[0] == {"COLOR"}
