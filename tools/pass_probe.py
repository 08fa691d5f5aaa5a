"""Time one pass alone on the GPU for A/B library builds (soc_real_time_renderer_amd/csrc `make variant`), on the bench's
own inputs, and hash its output so exact variants can be checked for identical bits.

    python tools/pass_probe.py --pass clouds|ssao|gbuffer|taa|raster|bloom1 --configs c3,c4 --variants libsoc_rt.so,libsoc_rt_x.so [--reps 100] [--rounds 3]

A variant is a library file name (SOC_RT_LIB_VARIANT) or NAME=VALUE[+NAME=VALUE...] (tuning knobs on the default library). Each
variant runs in its own process; the rounds interleave the variants so clock drift hits
them alike. Prints one line per (round, variant, config): mean microseconds per launch and the output digest.
"""
import argparse
import hashlib
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(pass_name, configs, reps):
    sys.path.insert(0, ROOT)
    import torch

    import bench
    import soc_real_time_renderer_amd as soc
    dev = torch.device("cuda", 0)
    out = {}
    for config in configs:
        W, H = (1920, 1080) if config == "c2" else (3840, 2160)
        g, _gb, _sh, _nz, _sc, fr = bench.build_inputs(config, "mesh", W, H, 0, dev)
        if pass_name == "clouds":
            tgt = torch.zeros(H, W, 4, dtype=torch.uint8, device=dev)
            run = lambda: soc.cloud_rendering(g, fr["depth"], fr["noise"], tgt, fr["clouds_workspace"])  # noqa: E731
        elif pass_name == "ssao":
            tgt = fr["ssao"]
            soc.ssao_prepare_noise(fr["normal"], fr["ssao"], fr["ssao_noise_table"])
            run = lambda: soc.ssao_generation(g, fr["depth"], fr["normal"], tgt, fr["ssao_noise_table"])  # noqa: E731
        elif pass_name == "gbuffer":   # GBufferGeneration's resolve of the mesh scene (visibility rasterised once)
            import numpy as np
            from soc_real_time_renderer_amd import raster
            sc = _sc
            vis = torch.empty((H, W), dtype=torch.int64, device=dev)
            raster.raster_visibility(sc["mesh"], np.ctypeslib.as_array(g.camera_projection_view_matrix), raster.CULL_FRONT,
                                     vis, sc["workspace"])
            tgt = fr["albedo"]
            run = lambda: raster.gbuffer_resolve(g, sc["mesh"], sc["materials"], sc["material_count"], vis,  # noqa: E731
                                                 fr["depth"], fr["albedo"], fr["emissive"], fr["normal"], fr["velocity"],
                                                 sc["workspace"])
        elif pass_name == "raster":   # DepthPrepass (visibility) + SunShadowDraw (4096^2 depth) of the mesh
            import numpy as np
            from soc_real_time_renderer_amd import raster
            sc = _sc
            vis = torch.empty((H, W), dtype=torch.int64, device=dev)
            shadow = torch.ones((4096, 4096), dtype=torch.float32, device=dev)
            vp = np.ctypeslib.as_array(g.camera_projection_view_matrix)
            svp = np.ctypeslib.as_array(g.sun_info.projection_view_matrix)

            class Both:   # digest over both outputs
                def cpu(self):
                    return torch.cat([vis.view(torch.int32).reshape(-1), shadow.view(torch.int32).reshape(-1)]).cpu()
            tgt = Both()

            def run():
                raster.raster_visibility(sc["mesh"], vp, raster.CULL_FRONT, vis, sc["workspace"])
                shadow.fill_(1.0)
                raster.raster_depth(sc["mesh"], svp, raster.CULL_BACK, shadow, sc["workspace"], raster.SHADOW_BIAS_CONSTANT,
                                    raster.SHADOW_BIAS_SLOPE)
        elif pass_name == "taa":   # the fused TemporalAntiAliasing + ToneMapping launch (SOC_TAA_NBR picks the kernel)
            hc, hv = fr["history_color"], fr["history_velocity"]
            gen = torch.Generator(device=dev).manual_seed(1)
            for im in (fr["color"], hc[0]):
                im.copy_(torch.rand(im.shape, generator=gen, device=dev).half() * 3)
            hv[0].copy_(fr["velocity"])
            ae = fr["auto_exposure"]
            tgt = hc[1]
            # SOC_PROBE_TAA_VOUT=0: no fused velocity-history write (the renderer's velocity slots, SOC_RENDERER_VELOCITY_SLOTS)
            vout = hv[1] if os.environ.get("SOC_PROBE_TAA_VOUT", "1") != "0" else None
            run = lambda: soc.temporal_antialiasing_tone_mapping(g, hc[1], fr["color"], hc[0], fr["velocity"],  # noqa: E731
                                                                 hv[0], fr["depth"], ae, fr["output"], vout)
        elif pass_name == "bloom1":   # the weighted bloom chain's first stage (emissive -> [mip0] -> mip1, bloomw_down01p)
            tgt = fr["bloom_mips"][1]
            out_img = fr.get("bloom_output")
            if out_img is None:
                out_img = torch.zeros(H, W, 4, dtype=torch.float16, device=dev)
            run = lambda: soc.bloom_weighted_stage(g, fr["emissive"], fr["bloom_mips"], out_img, stage=1)  # noqa: E731
        else:
            raise SystemExit(f"unknown pass {pass_name}")
        for _ in range(10):
            run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            run()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / reps * 1e3
        out[config] = {"us": round(us, 2), "digest": hashlib.md5(tgt.cpu().numpy().tobytes()).hexdigest()[:12]}
        del fr
        torch.cuda.empty_cache()
    print("PROBE " + json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pass", dest="pass_name", default="clouds")
    ap.add_argument("--configs", default="c3,c4")
    ap.add_argument("--variants", default="libsoc_rt.so")
    ap.add_argument("--reps", type=int, default=100)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--child", action="store_true")
    a = ap.parse_args()
    configs = a.configs.split(",")
    if a.child:
        child(a.pass_name, configs, a.reps)
        return
    for r in range(a.rounds):
        for v in a.variants.split(","):
            # NAME=VALUE[+NAME=VALUE...]: tuning knobs on the default library; else a library file name
            env = dict(os.environ, **(dict(kv.split("=", 1) for kv in v.split("+")) if "=" in v else {"SOC_RT_LIB_VARIANT": v}))
            p = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", "--pass", a.pass_name, "--configs",
                                a.configs, "--reps", str(a.reps)], env=env, capture_output=True, text=True, timeout=600)
            line = [ln for ln in p.stdout.splitlines() if ln.startswith("PROBE ")]
            if p.returncode != 0 or not line:
                print(f"round {r} {v}: FAILED rc={p.returncode}\n{p.stderr[-2000:]}", flush=True)
                sys.exit(1)
            res = json.loads(line[0][6:])
            for c in configs:
                print(f"round {r} {v:24s} {c}: {res[c]['us']:8.2f} us  {res[c]['digest']}", flush=True)


if __name__ == "__main__":
    main()
