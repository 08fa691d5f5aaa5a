#!/usr/bin/env python
"""Benchmark: frames/sec + ms/pass of the screen-space hot path (BASELINE.json metric).

One step = one full frame of the reference's live screen-space passes (renderer.cpp:1024-1217): bloom x8,
SSAO + blur, atmosphere/clouds, composition, luminance histogram (+ RCCL all-reduce when N > 1) +
resolve, TAA (with the fused velocity history), AgX tone mapping into an RGBA8 framebuffer, at
3840x2160 on the Sponza-proxy G-buffer (synthetic; Sponza.bin is missing from the reference). Inputs
are resident in HBM before timing starts. N GPUs: one process per GPU, each renders its own camera
(frame-per-GPU sharding, SURVEY.md §8e, weak scaling); value = frames of all ranks / max rank time.

Prints ONE JSON line on rank 0. See DESIGN.md §6 for the roofline accounting.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def _launch_ranks() -> None:
    """`bench.py --gpus N` (N > 1) started without a torch.distributed.run environment: start the N ranks
    through the launcher as a CHILD process, before anything touches the GPU, and exit with its code."""
    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--gpus", type=int, default=1)
    a, _ = ap.parse_known_args()
    if a.gpus <= 1 or "WORLD_SIZE" in os.environ:
        return
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # dmabuf IPC only on this host driver (RCCL)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    sys.exit(subprocess.call(cmd, env=env))


if __name__ == "__main__":
    _launch_ranks()

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import soc_real_time_renderer_amd as soc  # noqa: E402
from soc_real_time_renderer_amd import multi_gpu, raster, scene  # noqa: E402
from soc_real_time_renderer_amd.scene import sponza_mesh  # noqa: E402

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
SSAO_KERNEL = "ssao_pipe_kernel<64, 16, 32, true>"   # the default SSAOGeneration kernel (ssao.hip)


def make_globals(W, H, camera):
    g = soc.globals_defaults(W, H)
    cam = soc.make_camera(*camera)
    ji = C.c_uint32(0)
    soc.frame_update(g, cam, W, H, 0.016, ji)
    cam.position[0] += 0.05
    soc.frame_update(g, cam, W, H, 0.016, ji)
    g.elapsed_time = 10.0      # SURVEY.md §8d pinned globals (C3)
    g.frame_counter = 2
    return g


def point_lights_c3b(n=128, seed=0x3B):
    """C3b: 128 point-light entities (PointLightComponent defaults, components.hpp:55-58) scattered
    through the Sponza-proxy atrium, seeded; fed through Scene::update (soc_scene_update)."""
    rng = np.random.default_rng(seed)
    return [soc.entity(position=(rng.uniform(-15.0, 12.0), rng.uniform(0.3, 7.0), rng.uniform(-4.5, 4.5)),
                       point_light=True, color=rng.uniform(0.3, 1.0, 3), intensity=float(rng.uniform(0.5, 4.0)))
            for _ in range(n)]


def algorithmic_bytes(W, H, f_sky, velocity_slots=False, bloom_in_composition=False):
    """Bytes each pass must move at the reference formats, per launch. velocity_slots: the velocity
    history by slot rotation (SOC_RENDERER_VELOCITY_SLOTS), so TAA writes no velocity copy. bloom_in_composition: the
    bloom chain's last stage inside Composition (SOC_RENDERER_BLOOM_IN_COMPOSITION), which reads mip1 (2 B/px) instead
    of the bloom output (8 B/px)."""
    P = W * H
    vcopy = 0.0 if velocity_slots else 8.0
    em = 2.0 if bloom_in_composition else 8.0
    b = {
        "BloomDownsample - 0": 16.0 * P, "BloomDownsample - 1": (8.0 + 2.0) * P, "BloomDownsample - 2": (2.0 + 0.5) * P,
        "BloomDownsample - 3": (0.5 + 0.125) * P, "BloomUpsample - 3": (0.125 + 0.5) * P,
        "BloomUpsample - 2": (0.5 + 2.0) * P, "BloomUpsample - 1": (2.0 + 8.0) * P, "BloomUpsample - 0": 16.0 * P,
        # weighted-form chain (bloom_w.hip): mip0 / mip2 stay in LDS (emissive -> mip1 -> mip3 -> mip1 -> output)
        "BloomDownsample - 0+1": (8.0 + 2.0) * P, "BloomDownsample - 2+3": (2.0 + 0.125) * P,
        "BloomUpsample - 3+2": (0.125 + 2.0) * P, "BloomUpsample - 1+0": (2.0 + 8.0) * P,
        "SSAOGeneration": 12.25 * P, "SSAOBlur": 0.5 * P, "CloudRendering": 8.0 * P,
        "Composition": (40.25 + 4.0 * f_sky) * P, "GenerateLuminanceHistogram": 8.0 * P,
        # fused composition + histogram: the bins come from the stored pixels in registers (+1 KiB)
        "Composition+GenerateLuminanceHistogram": (40.25 - 8.0 + em + 4.0 * f_sky) * P,
        "ResolveLuminanceHistogram": 2.0 * 1028.0,
        "TemporalAntiAliasing": (44.0 + vcopy) * P,   # 44 B/px reference TAA + 8 B/px fused velocity history write
        "ToneMapping": 12.0 * P,
        # fused TAA + tone map: the tone map reads the resolved pixels from registers (writes 4 B/px)
        "TemporalAntiAliasing+ToneMapping": (44.0 + vcopy + 4.0) * P,
    }
    return b


def pmc_traffic(kernel, W, H, scene_name="mesh"):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC table (profiles/, written by
    tools/pmc_summary.py --traffic from a run of this same workload), or None."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc_traffic.json")))
    if not files:
        return None, None
    with open(files[-1]) as fh:
        t = json.load(fh)
    ks = t.get("kernels", {})
    k = ks.get(kernel)
    if k is None:   # a table from another template signature: the one instantiation of that kernel, or the one whose
        # arguments start with the given ones (a table with fewer template arguments than the name asked for, or more)
        base = [(n, v) for n, v in ks.items() if n.split("<")[0] == kernel.split("<")[0]]
        pre = [(n, v) for n, v in base if n.rstrip(">").startswith(kernel.rstrip(">")) or kernel.rstrip(">").startswith(n.rstrip(">"))]
        k = base[0][1] if len(base) == 1 else (pre[0][1] if len(pre) == 1 else None)
    if not k or list(t.get("resolution", [])) != [W, H] or t.get("scene", "boxes") != scene_name:
        return None, None
    return k["hbm_bytes"], os.path.relpath(files[-1], ROOT)


def valu_bound(kernel, us):
    """The kernel's VALU issue time from the committed issue model (profiles/*valu_model.json, tools/valu_calibrate.py:
    SQ_INSTS_VALU per launch of the same C3 command at the measured cost of one wave64 VALU instruction over 1024 SIMDs
    at the launch's clock) against its measured time `us`, or None. A model written before a template
    signature change matches on the kernel's base name when it holds one instantiation of it."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*valu_model.json")))
    if not files:
        return None
    with open(files[-1]) as fh:
        t = json.load(fh)
    for rows in t.get("runs", {}).values():
        if kernel not in rows:
            base = [n for n in rows if n.split("<")[0] == kernel.split("<")[0]]
            if len(base) == 1:
                kernel = base[0]
        if kernel in rows:
            r = rows[kernel]
            issue = r.get("valu_issue_us", r.get("issue_bound_us"))
            return {"valu_issue_us": issue, "frac_of_launch": round(issue / us, 3),
                    "serial_us": r["us"], "source": os.path.relpath(files[-1], ROOT)}
    return None


def clouds_roofline(config, W, H, us):
    """CloudRendering against the FP32 VALU / transcendental peaks: the reference GLSL's FLOPs and
    transcendentals of this frame, tallied per function by tools/clouds_flops.py from an instrumented oracle run on the
    same inputs (committed as profiles/*clouds_flops.json), over the pass's measured time `us` (the serial per-pass
    loop: the pass alone on the GPU)."""
    import glob
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import clouds_flops
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*clouds_flops.json")))
    if not files or not us:
        return None
    with open(files[-1]) as fh:
        t = json.load(fh)
    c = t.get("configs", {}).get(config)
    if c is None or list(t.get("resolution", [])) != [W, H]:
        return None
    r = clouds_flops.roofline(c, us)
    r.update({"flops_per_frame": c["flops"], "transcendentals_per_frame": c["transcendentals"],
              "per_sky_pixel": c["per_sky_pixel"], "source": os.path.relpath(files[-1], ROOT)})
    return r


def cpu_baseline(W, H, host_inputs, g):
    """The oracle (plain-C restatement, OpenMP over rows) timed on this box's host cores."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    oracle.lib()
    fr = dict(host_inputs)
    fr["bloom_mips"] = [np.zeros((H >> i, W >> i, 4), np.float16) for i in range(4)]
    fr["ssao"] = np.zeros((H // 2, W // 2), np.uint8)
    fr["ssao_blur"] = np.zeros((H // 2, W // 2), np.uint8)
    fr["clouds"] = np.zeros((H, W, 4), np.uint8)
    fr["color"] = np.zeros((H, W, 4), np.float16)
    fr["history_color"] = [np.zeros((H, W, 4), np.float16) for _ in range(2)]
    fr["history_velocity"] = [np.zeros((H, W, 4), np.float16) for _ in range(2)]
    fr["output"] = np.zeros((H, W, 4), np.uint8)
    fr["emissive"] = host_inputs["emissive"].copy()
    ae = soc.AutoExposure()
    frames, t_total, times, frame_s = 0, 0.0, {}, []
    while frames < 2 or (t_total < 12.0 and frames < 30):
        fr["emissive"][...] = host_inputs["emissive"]
        t0 = time.perf_counter()
        oracle.frame(g, fr, ae, hist=frames % 2, times=times if frames else None)   # frame 0: warm-up for the medians
        dt = time.perf_counter() - t0
        t_total += dt
        if frames:
            frame_s.append(dt)
        frames += 1
    return {"value": round(frames / t_total, 4), "unit": "frames/sec", "cores": oracle.num_threads(),
            "kind": "port",
            "sample": f"{frames} full {W}x{H} frame(s) of all passes (bloom x8, ssao+blur, clouds, composition, "
                      f"histogram+resolve, taa, tone map) on the oracle, {t_total:.1f} s",
            "ms_per_frame_median": round(float(np.median(frame_s)) * 1e3, 1),
            "ms_per_pass_median": {k: round(float(np.median(v)) * 1e3, 2) for k, v in times.items()}}


REFERENCE_GROUPS = ("Depth Prepass", "Composition", "Tone Mapping", "Bloom", "Depth Of Field", "Shadows",
                    "Rendering G-Buffer", "Screen Space Reflections", "Ambient Occlusion", "Auto Exposure",
                    "Sky Rendering", "Temporal Anti-Aliasing")   # renderer.cpp:576-587
# fused launches -> (the unfused passes whose time ratio splits them, their groups)
FUSED_SPLIT = {"Composition+GenerateLuminanceHistogram": (("Composition", "GenerateLuminanceHistogram"),
                                                          ("Composition", "Auto Exposure")),
               "TemporalAntiAliasing+ToneMapping": (("TemporalAntiAliasing", "ToneMapping"),
                                                    ("Temporal Anti-Aliasing", "Tone Mapping"))}


def unfused_group_ms(fr, renderer_kw, g, frames):
    """The serial per-pass loop of a renderer with the reference's pass structure (composition, histogram, TAA and tone
    map as separate launches; bloom in its own passes) on the same frame images: ms per pass name and per reference
    group. After the timed region; it renders into the same images (their contents are not used afterwards)."""
    kw = dict(renderer_kw, fused_histogram=False, bloom_in_composition=False, sky_lane=False)
    ru = soc.Renderer(fr, fused_tonemap=False, **kw)
    ru.set_pass_timing(-1, True)
    for _ in range(2):
        ru.execute(g)
    torch.cuda.synchronize()
    ru.reset_timing()
    for _ in range(max(1, frames)):
        ru.execute(g)
    torch.cuda.synchronize()
    st = [x for x in ru.pass_stats() if x[3]]
    ru.close()
    groups = {k: 0.0 for k in REFERENCE_GROUPS}
    for n, gname, ms, _ in st:
        groups[gname] = groups.get(gname, 0.0) + ms
    return {"passes": {n: round(ms, 4) for n, _, ms, _ in st}, "groups": {k: round(v, 4) for k, v in groups.items()}}


def reference_groups(stats, no_launch, unfused):
    """ms per reference group from the serial loop's passes; fused launches split by the unfused passes' time ratio."""
    out = {k: 0.0 for k in REFERENCE_GROUPS}
    for n, gname, ms, _ in stats:
        if n in no_launch:
            continue
        if n in FUSED_SPLIT and unfused:
            (pa, pb), (ga, gb_) = FUSED_SPLIT[n]
            ta, tb = unfused["passes"].get(pa), unfused["passes"].get(pb)
            if ta and tb:
                out[ga] = out.get(ga, 0.0) + ms * ta / (ta + tb)
                out[gb_] = out.get(gb_, 0.0) + ms * tb / (ta + tb)
                continue
        out[gname] = out.get(gname, 0.0) + ms
    return {k: round(v, 4) for k, v in out.items()}


def build_inputs(config, scene_name, W, H, rank, device, mips=True, output_format=None):
    """The frame inputs of a bench configuration (shared with the 4K C3 parity test): globals of rank `rank`'s camera,
    the G-buffer + 4096^2 sun shadow map (the Sponza-proxy mesh rasterised once by the HIP rasteriser, or the
    host-synthesised box atrium / terrain), the noise texture, and the device frame images holding them.
    Returns (g, host G-buffer dict, host shadow, host noise, mesh scene or None, device frame)."""
    terrain = config == "c4"
    scene_id = scene.TERRAIN if terrain else (scene.SPONZA_PROXY if scene_name == "boxes" else scene.SPONZA_MESH)
    g = make_globals(W, H, (multi_gpu.terrain_camera_for_rank if terrain else multi_gpu.camera_for_rank)(rank))
    if config == "c3b":
        soc.scene_update(g, point_lights_c3b())
    sc = None
    if scene_id == scene.SPONZA_MESH:
        # rasterised once by the HIP rasteriser (DepthPrepass + GBufferGeneration + SunShadowDraw), not timed
        # the reference's Sponza images at their own resolution (1024^2) when build() copied them, else the
        # committed 256^2 fixture
        native = sponza_mesh.native_available()
        sc = raster.scene_setup(g, scene_id, tex_size=None if native else 256, device=device, mips=mips, native=native)
        sc["texture_set"] = "native 1024^2" if native else "256^2 fixture"
        gbd = raster.render_gbuffer(g, sc, W, H, 4096, device)
        torch.cuda.synchronize()
        gb = {k: gbd[k].cpu().numpy() for k in ("albedo", "emissive", "normal", "velocity", "depth")}
        shadow = gbd["shadow"].cpu().numpy()
        del gbd
    else:
        gb = scene.gbuffer(g, W, H, scene_id=scene_id)
        shadow = scene.shadow_map(g, 4096, scene_id=scene_id)
    noise = scene.noise_texture()
    fr = soc.alloc_frame(W, H, device, bloom_output=True,
                         **({} if output_format is None else {"output_format": output_format}))
    for k in ("albedo", "emissive", "normal", "velocity", "depth"):
        fr[k].copy_(torch.from_numpy(gb[k]))
    fr["shadow"].copy_(torch.from_numpy(shadow))
    fr["noise"].copy_(torch.from_numpy(noise))
    return g, gb, shadow, noise, sc, fr


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--config", choices=("c2", "c3", "c3b", "c4"), default="c3",
                    help="c3: Sponza-proxy full chain at 4K (the metric's config); c3b: C3 with 128 point lights fed "
                         "through the ECS scene feed (SURVEY.md §8d); c2: the same scene at 1920x1080 "
                         "(with --raster: deferred lighting + sun shadow map rendered per frame); c4: terrain + "
                         "atmosphere/clouds")
    ap.add_argument("--scene", choices=("mesh", "boxes"), default="mesh",
                    help="c2/c3/c3b scene: mesh = the Sponza-proxy mesh (~256k triangles, the reference's Sponza "
                         "textures; rasterised by the HIP rasteriser); boxes = the round-1 analytic box atrium")
    ap.add_argument("--width", type=int, default=None, help="default 3840 (1920 for c2)")
    ap.add_argument("--height", type=int, default=None, help="default 2160 (1080 for c2)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--profile-frames", type=int, default=20)
    ap.add_argument("--no-sky-lane", action="store_true", help="run CloudRendering on the frame stream too")
    ap.add_argument("--no-static-inputs", action="store_true",
                    help="fork the second lane at every frame start (no cross-frame overlap of the clouds)")
    ap.add_argument("--no-velocity-slots", action="store_true",
                    help="velocity history as the reference's per-frame copy (fused into TAA) instead of slot rotation "
                         "(SOC_RENDERER_VELOCITY_SLOTS: the G-buffer's velocity lives in the history slot the next frame "
                         "reads as previous)")
    ap.add_argument("--no-bloom-in-composition", action="store_true",
                    help="the bloom chain's last stage as its own pass writing the full-resolution bloom output "
                         "(default: computed inside the fused Composition launch, SOC_RENDERER_BLOOM_IN_COMPOSITION)")
    ap.add_argument("--unfused-histogram", action="store_true",
                    help="Composition and the luminance histogram as two launches (SOC_RENDERER_UNFUSED_HISTOGRAM)")
    ap.add_argument("--write-frame", default="", help="write the last frame: tone-mapped framebuffer (.png) or HDR composition colour (.exr, f16)")
    ap.add_argument("--metrics-jsonl", default="", help="one GPU-metric JSON line per profiled frame")
    ap.add_argument("--no-mips", action="store_true",
                    help="mesh scene: level-0 bilinear textures instead of the reference's mip chains + 16x anisotropic sampler")
    ap.add_argument("--exchange", action="store_true",
                    help="take the multi-GPU frame path at any N: PRE -> histogram all-reduce (RCCL, a world-size-1 "
                         "group at N = 1) -> POST, with the all-reduce timed (SURVEY.md §8e)")
    ap.add_argument("--sky-lane-queue", choices=("auto", "low", "high", "probe"), default="auto",
                    help="the sky lane's hardware queue (SOC_RENDERER_SKY_LANE_HIGH / _PROBE): auto = the configuration's "
                         "fixed choice (low for c3 / c3b, whose main lane is the critical path; high for the sky-bound "
                         "c2 / c4 frames), so a command runs the same kernels every time; probe = round 5's timed choice")
    ap.add_argument("--raster", action="store_true",
                    help="end-to-end frame: rasterise the scene mesh into the G-buffer and the 4096^2 sun shadow "
                         "map every frame (DepthPrepass / SunShadowDraw / GBufferGeneration in the graph)")
    args = ap.parse_args()

    rank, world, local_rank = multi_gpu.env()
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but the launcher started {world} rank(s) (WORLD_SIZE)")
    # rehearsal of the N-rank path on a 1-GPU box: SOC_BENCH_SHARE_DEVICE=1 puts every rank on device 0
    # and SOC_DIST_BACKEND=gloo replaces RCCL (which refuses two ranks on one device)
    dev_index = 0 if os.environ.get("SOC_BENCH_SHARE_DEVICE") == "1" else local_rank
    torch.cuda.set_device(dev_index)
    device = torch.device("cuda", dev_index)
    multi_gpu.init(device, backend=os.environ.get("SOC_DIST_BACKEND", "nccl"), force_exchange=args.exchange)
    exchange = multi_gpu.exchange_active()
    W = args.width or (1920 if args.config == "c2" else 3840)
    H = args.height or (1080 if args.config == "c2" else 2160)

    # ---- inputs (Sponza-proxy mesh or terrain G-buffer + 4096^2 sun shadow map), resident in HBM ----
    terrain = args.config == "c4"
    g, gb, shadow, noise, sc, fr = build_inputs(args.config, args.scene, W, H, rank, device, mips=not args.no_mips)
    scene_id = scene.TERRAIN if terrain else (scene.SPONZA_PROXY if args.scene == "boxes" else scene.SPONZA_MESH)
    f_sky = float((gb["depth"] == 1.0).mean())
    # the G-buffer, shadow map and noise stay resident and unchanged between frames (or come from the raster head):
    # the second lane may start a frame's clouds before the previous frame's TAA is done (SOC_RENDERER_STATIC_INPUTS)
    # velocity history by slot rotation: the G-buffer's velocity is produced into the history slot the next frame reads
    # as its previous velocity (the raster head writes it there every frame; the resident G-buffer holds it in both)
    vslots = not args.no_velocity_slots
    if vslots:
        for hv in fr["history_velocity"]:
            hv.copy_(fr["velocity"])
    lane_q = args.sky_lane_queue if args.sky_lane_queue != "auto" else ("low" if args.config in ("c3", "c3b") else "high")
    renderer_kw = dict(sky_lane=not args.no_sky_lane, fused_histogram=not args.unfused_histogram,
                       static_inputs=not args.no_static_inputs, velocity_slots=vslots,
                       bloom_in_composition=not args.no_bloom_in_composition, sky_lane_queue=lane_q)
    r = soc.Renderer(fr, **renderer_kw)
    if args.raster:
        if sc is None:
            sc = raster.scene_setup(g, scene_id, tex_size=1024, device=device)
        vis = torch.empty((H, W), dtype=torch.int64, device=device)
        r.set_raster_scene(sc["mesh"], sc["materials"], sc["material_count"], vis, sc["workspace"], shadow=True)
    r.set_exposure_pixels(*multi_gpu.exposure_pixels(world, W, H))
    bins = fr["auto_exposure"][1:]
    names = r.pass_names()
    groups = r.pass_groups()
    stream = torch.cuda.current_stream()

    xev = []   # (start, end) events around the histogram exchange of every timed frame (N > 1)

    def frame(timed=False):
        ev = None
        if timed and exchange:
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            xev.append(ev)
        # PRE, RCCL all-reduce of the 1 KiB histogram (N > 1), POST
        multi_gpu.render_frame(r, g, bins, exchange_events=ev)

    for _ in range(args.warmup):
        frame()
    # the sky-lane queue is fixed by the configuration (no timing probe): --warmup frames exactly. Only --sky-lane-queue
    # probe runs the renderer's probe, in extra untimed frames until it has chosen (the same count on every rank: each
    # frame of the exchange path is a collective)
    probe_frames = 0
    if lane_q == "probe" and not args.no_sky_lane and r.side_queue() == -1:
        probe_frames = max(0, r.side_queue_probe_frames() - args.warmup)
        for _ in range(probe_frames):
            frame()
        torch.cuda.synchronize()
        frame()
        probe_frames += 1
    torch.cuda.synchronize()

    # HIP events around the north-star kernels on the launch stream, inside the timed region
    comp = "Composition+GenerateLuminanceHistogram" if "Composition+GenerateLuminanceHistogram" in names else "Composition"
    timed = [names.index(comp), names.index("SSAOGeneration")]
    probe_no_events = os.environ.get("SOC_BENCH_NO_PASS_EVENTS") == "1"   # diagnostic: frame time without them
    for i in timed:
        r.set_pass_timing(i, not probe_no_events)
    r.reset_timing()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    base_ev = torch.cuda.Event(enable_timing=True)
    base_ev.record()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        frame(timed=True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    xchg_us = (sum(a.elapsed_time(b) for a, b in xev) / len(xev) * 1e3) if xev else 0.0
    per_rank = multi_gpu.gather_objects({"rank": rank, "fps": round(args.steps / elapsed, 3),
                                         "allreduce_us_per_frame": round(xchg_us, 2),
                                         **multi_gpu.rank_inventory(device)})
    stats_timed = {n: ms for n, _, ms, cnt in r.pass_stats() if cnt}
    events_out = os.environ.get("SOC_BENCH_EVENTS_OUT")   # every timed frame's pass events, for tools/event_trace_check.py
    if events_out and rank == 0 and not probe_no_events:
        # "warmup": the frames before the timed ones (warm-up + the lane probe's untimed frames), i.e. the launches of
        # each kernel that tools/event_trace_check.py skips in the trace
        dump = {"frames": args.steps, "warmup": args.warmup + probe_frames, "passes": {}}
        for i in timed:
            s0, s1 = r.pass_event_times(i, base_ev, args.steps)
            dump["passes"][names[i]] = {"start_ms": s0.tolist(), "end_ms": s1.tolist()}
        with open(events_out, "w") as fh:
            json.dump(dump, fh)
    max_elapsed = multi_gpu.max_over_ranks(elapsed, device)
    ms_per_step = max_elapsed / args.steps * 1e3
    value = world * args.steps / max_elapsed

    # ---- per-pass breakdown (separate, all passes evented, sky lane off so passes do not overlap) ----
    r.set_async(False)
    r.set_pass_timing(-1, True)
    r.reset_timing()
    metrics_lines = []
    for i in range(args.profile_frames):
        frame()
        if args.metrics_jsonl:   # the reference's per-frame "GPU Metric" record (renderer.cpp:769-806)
            torch.cuda.synchronize()
            metrics_lines.append(r.metrics_json(i))
    torch.cuda.synchronize()
    stats = r.pass_stats()
    if args.metrics_jsonl and rank == 0:
        with open(args.metrics_jsonl, "w") as f:
            f.write("\n".join(metrics_lines) + "\n")
    if args.write_frame and rank == 0:   # headless present: the RGBA8 framebuffer (PNG) or the HDR colour (EXR f16)
        if args.write_frame.endswith(".exr"):
            soc.write_exr(args.write_frame, soc.read_image(fr["color"]))
        else:
            soc.write_png(args.write_frame, soc.read_image(fr["output"]))
    r.set_async(not args.no_sky_lane)
    stats = [st for st in stats if st[3]]     # passes with no work this frame (the folded fold pass) have no record
    # the renderer computes the bloom's last stage inside Composition in frames whose sky lane is the critical path
    # (SOC_RENDERER_BLOOM_IN_COMPOSITION with a high-priority sky lane): the fourth bloom pass then launches nothing
    bloom_in_comp = not args.no_bloom_in_composition and "BloomUpsample - 3+2" in names and r.side_queue() == 1
    no_launch = {"BloomUpsample - 1+0"} if bloom_in_comp else set()
    ms_pass = {n: (None if n in no_launch else round(ms, 4)) for n, _, ms, _ in stats}
    ms_group_unfused = unfused_group_ms(fr, renderer_kw, g, args.profile_frames) if not args.raster else None
    ms_group = reference_groups(stats, no_launch, ms_group_unfused)
    algo = algorithmic_bytes(W, H, f_sky, velocity_slots=vslots, bloom_in_composition=bloom_in_comp)
    # Two durations per north-star kernel: alone = the serial per-pass loop above (every pass evented,
    # second lane off: nothing shares the CUs with the kernel), and in-frame = the timed frames' events (lanes
    # concurrent: the sky lane's kernels share the CUs, so the duration also carries their share). The roofline's
    # headline is the kernel alone: it is the kernel's own speed, and a profiler reproduces it (a kernel trace changes
    # how the two lanes overlap, so in-frame durations of a traced run differ from an untraced one; within one traced
    # run events and trace agree, tools/event_trace_check.py)
    comp_frame_ms = stats_timed.get(comp)
    ssao_frame_ms = stats_timed.get("SSAOGeneration")
    comp_ms = ms_pass.get(comp, comp_frame_ms)
    ssao_ms = ms_pass.get("SSAOGeneration", ssao_frame_ms)
    ns_bytes = algo[comp] + algo["SSAOGeneration"]
    ns_us = (comp_ms + ssao_ms) * 1e3
    # GB/s of every pass that launched work (a pass that launched nothing this frame reports null, not its event overhead)
    pass_gbs = {n: (None if n in no_launch else round(algo[n] / (ms * 1e-3) / 1e9, 1))
                for n, _, ms, _ in stats if ms > 0 and n in algo}
    # the committed PMC table comes from the default command (C3, G-buffer resident): other workloads get null
    pmc_ok = args.config == "c3" and not args.raster
    # the Composition kernel the timed frames ran (its fourth template argument: the in-kernel bloom of a sky-bound frame)
    comp_kernel = (f"composition_pair<true, false, 7, {'true' if bloom_in_comp else 'false'}>" if comp != "Composition"
                   else "composition_pair<false, false, 7, false>")
    traffic, traffic_src = pmc_traffic(comp_kernel, W, H, args.scene) if pmc_ok else (None, None)
    ssao_traffic, _ = pmc_traffic(SSAO_KERNEL, W, H, args.scene) if pmc_ok else (None, None)
    pair_traffic = traffic + ssao_traffic if traffic is not None and ssao_traffic is not None else None
    pair_achieved = ns_bytes / (ns_us * 1e-6) / 1e9

    def kernel_entry(n, ms, ms_frame, traffic_b, extra=None):
        e = {"achieved": round(algo[n] / (ms * 1e-3) / 1e9, 1), "frac": round(algo[n] / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
             "avg_launch_us": round(ms * 1e3, 2), "basis": "alone (serial per-pass loop, HIP events)",
             "traffic": traffic_b, "algorithmic_bytes_per_launch": int(algo[n])}
        if ms_frame:
            e["in_frame"] = {"avg_launch_us": round(ms_frame * 1e3, 2),
                             "frac": round(algo[n] / (ms_frame * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
        e.update(extra or {})
        return e

    def pair_in_frame():
        if not (comp_frame_ms and ssao_frame_ms):
            return None
        t = (comp_frame_ms + ssao_frame_ms) * 1e3
        return {"avg_launch_us": round(t, 2), "frac": round(ns_bytes / (t * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
                "basis": "timed frames, lanes concurrent (HIP events on the launch stream)"}

    def pair_valu_floor():
        # the pair's VALU issue time (the committed, calibrated issue model of the same two kernels, valu_bound): the
        # time their instructions need at the measured issue rate, beside the 0.60 target's time
        vs = [valu_bound(SSAO_KERNEL, 1.0), valu_bound(comp_kernel, 1.0)]
        if not pmc_ok or not all(vs):
            return None
        fl = sum(v["valu_issue_us"] for v in vs)
        return {"valu_issue_us": round(fl, 1), "frac_at_valu_floor": round(ns_bytes / (fl * 1e-6) / 1e9 / HBM_PEAK_GBS, 4),
                "target_us_at_60pct": round(ns_bytes / (0.6 * HBM_PEAK_GBS * 1e9) * 1e6, 2), "source": vs[0]["source"]}

    if world > 1:
        dist.barrier()
    if rank != 0:
        dist.destroy_process_group()
        return

    out = {
        "metric": "frames/sec + ms/pass, Sponza 3840x2160 deferred+SSAO+TAA",
        "value": round(value, 3),
        "unit": "frames/sec",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32 (fp16/unorm8/d32 storage)",
        "data": (f"synthetic: fBm terrain (seed 0x7E44) G-buffer + 4096^2 sun shadow map (scene_synth.c)" if terrain else
                 f"synthetic: Sponza-proxy {'box atrium (scene_synth.c)' if sc is None else 'mesh (procedural atrium, ' + str(int(sc['mesh'].struct.triangle_count)) + ' triangles, the reference Sponza baseColor/normal textures (' + sc['texture_set'] + ')' + ('' if args.no_mips else ' with mip chains + 16x anisotropic sampling') + ', seed 0x5050)'}; "
                 f"G-buffer + 4096^2 sun shadow map {'ray-cast on the host' if sc is None else 'rasterised once by the HIP rasteriser'}"),
        "config": {"workload": f"{'Terrain' if terrain else 'Sponza-proxy'} {W}x{H} full screen-space chain "
                               f"({args.config.upper()}): bloom x8, SSAO+blur, clouds, composition"
                               f"{' with 128 point lights' if args.config == 'c3b' else ''}, auto-exposure, "
                               f"TAA, AgX tone map",
                   "resolution": [W, H], "f_sky": round(f_sky, 4), "parallelism": f"frame-per-gpu x{world}",
                   "profile_frames": args.profile_frames,
                   "histogram_allreduce": exchange,
                   "collective_backend": (dist.get_backend() if exchange else None),
                   "sky_lane": ("CloudRendering + SkyCompose on a concurrent stream; " +
                                ("the clouds of frame N+1 may start before frame N's TAA (static inputs)"
                                 if not args.no_static_inputs else "forked at every frame start")),
                   "sky_lane_queue": {1: "high priority", 2: "low priority", 0: "normal priority",
                                      -1: "not chosen"}.get(r.side_queue(), "?"),
                   "sky_lane_queue_choice": ("timed probe" if lane_q == "probe" else
                                             f"fixed ({lane_q}: {'--sky-lane-queue' if args.sky_lane_queue != 'auto' else 'the configuration default'})"),
                   "untimed_lane_probe_frames": probe_frames,
                   "bloom_last_stage": ("inside Composition (mip1 -> [mip0] -> emissive term per tile in LDS; the "
                                        "full-resolution bloom output is not written)" if bloom_in_comp
                                        else "its own pass (writes the bloom output)"),
                   "velocity_history": ("slot rotation (the G-buffer's velocity in the slot the next frame reads; "
                                        "no copy)" if vslots else "copy fused into TAA"),
                   "raster": (f"in-frame: DepthPrepass + SunShadowDraw (4096^2) + GBufferGeneration of the "
                              f"{int(sc['mesh'].struct.triangle_count)}-triangle scene mesh") if args.raster
                   else "off: G-buffer and shadow map are resident inputs"},
        # headline: the north-star pair (SURVEY.md §8d target: SSAO + deferred lighting >= 0.60 of HBM peak), each
        # kernel alone; the same kernels' in-frame figures beside them
        "roofline": {"kernels": ["SSAOGeneration", comp], "bound": "hbm", "achieved": round(pair_achieved, 1),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(pair_achieved / HBM_PEAK_GBS, 4),
                     "basis": "each kernel alone (serial per-pass loop, HIP events on the launch stream)",
                     "traffic": pair_traffic, "traffic_source": traffic_src,
                     "algorithmic_bytes_per_launch": int(ns_bytes), "avg_launch_us": round(ns_us, 2),
                     "target_us_at_60pct": round(ns_bytes / (0.6 * HBM_PEAK_GBS * 1e9) * 1e6, 2),
                     "in_frame": pair_in_frame(),
                     "valu_floor": pair_valu_floor(),
                     "per_kernel": {
                         comp: kernel_entry(comp, comp_ms, comp_frame_ms, traffic),
                         "SSAOGeneration": kernel_entry(
                             "SSAOGeneration", ssao_ms, ssao_frame_ms, ssao_traffic,
                             {"valu_bound": valu_bound(SSAO_KERNEL, ssao_ms * 1e3) if pmc_ok else None}),
                         # the largest pass of the frame is VALU-bound: its compute roofline
                         "CloudRendering": (clouds_roofline({"c3b": "c3"}.get(args.config, args.config) if args.scene == "mesh" or terrain else "", W, H,
                                                            ms_pass.get("CloudRendering", 0.0) * 1e3)
                                            if not args.raster else None)}},
        "ranks": per_rank,
        "allreduce_us_per_frame": (round(sum(p["allreduce_us_per_frame"] for p in per_rank) / world, 2)
                                   if exchange else None),
        "ms_per_pass": ms_pass,
        # the reference's 12 GPU-metric groups (renderer.cpp:558-588) from the serial per-pass loop; a fused launch's time
        # is split between its groups in the ratio of the same passes unfused (ms_per_group_unfused: the reference's own
        # pass structure, one launch per task, measured in the same run)
        "ms_per_group": ms_group,
        "ms_per_group_basis": ("serial per-pass loop; Composition+GenerateLuminanceHistogram split into Composition / "
                               "Auto Exposure and TemporalAntiAliasing+ToneMapping into Temporal Anti-Aliasing / Tone "
                               "Mapping by the unfused passes' time ratio"),
        "ms_per_group_unfused": ms_group_unfused,
        "gbs_per_pass": pass_gbs,
    }
    if not args.no_cpu_baseline and world == 1:
        host_inputs = dict(gb)
        host_inputs["shadow"] = shadow
        host_inputs["noise"] = noise
        out["cpu_baseline"] = cpu_baseline(W, H, host_inputs, g)
    else:
        out["cpu_baseline"] = None
    emit(json.dumps(out))
    r.close()
    if dist.is_initialized():
        dist.destroy_process_group()


_RESULT_FD = None   # the process's original stdout when run as a script (everything else goes to stderr)


def emit(line):
    """The bench's one stdout line. Run as a script, fd 1 is pointed at stderr for the whole run (RCCL prints its
    version banner to stdout when a communicator is created, and native code may print too), and the result line
    alone is written to the saved original stdout."""
    if _RESULT_FD is None:
        print(line, flush=True)
    else:
        sys.stdout.flush()
        os.write(_RESULT_FD, (line + "\n").encode())


if __name__ == "__main__":
    sys.stdout.flush()
    _RESULT_FD = os.dup(1)
    os.dup2(2, 1)
    main()
