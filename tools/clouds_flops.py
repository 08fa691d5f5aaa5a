"""CloudRendering against its compute roofline ("Clouds FLOPs: count them with an instrumented run of
the CPU oracle ... and report the VALU fraction").

The work of the reference's cloud pass is counted per function of its GLSL, as written
(/root/reference/src/graphics/tasks/cloud_rendering.inl:92-481), and multiplied by how often the instrumented oracle
(oracle/soc_oracle.c, soc_oracle_clouds_counters) enters each function on the frame's own depth image. Conventions:
- FLOP: one fp32 add, sub, mul or div (a fused multiply-add counts 2); expressions of literals and compile-time
  constants are folded; vectors count per component; min / max / abs / floor / fract / clamp and compares count 0;
- transcendental: exp, pow, sqrt, inversesqrt (normalize), each one (the quarter-rate VALU ops on gfx950);
- texture tap: one bilinear fetch (the depth test, two per noise octave). gfx950 has no texture filter, so the
  kernels filter on the VALU; `flops_with_filter` adds 9 FLOPs per tap (three lerps of one channel).

Roofline: FP32 vector peak 157.3 TFLOP/s (MI355X_MICROARCH.md: 256 CUs x 4 SIMDs x 64 FLOP/clk x 2.4 GHz); a
transcendental issues in 8 cycles per wave64 against 2 for an FMA (the guide's issue-cost row), so 8 lanes/clk/SIMD:
19.66 T/s. `floor_us` = FLOPs / 157.3 T + transcendentals / 19.66 T is the time the counted work needs at peak issue
(FMA-fused, every lane busy), `frac_of_floor` = floor_us / measured us.

Run on the GPU box (the Sponza-proxy mesh is rasterised by the HIP rasteriser, bench.build_inputs):
    python tools/clouds_flops.py [--out gpurun_out/clouds_flops.json]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]

FP32_PEAK_TFLOPS = 157.3
TRANS_PEAK_T = 256 * 4 * 8 * 2.4e9 / 1e12      # 19.66 T transcendental lane-ops per second
FILTER_FLOPS_PER_TAP = 9

# (flops, transcendentals, taps) per entry, with the oracle counter that counts the entries and the GLSL it follows.
WORK = {
    "pixel": ((70, 1, 1), "pixels",
              "main :445-458: ray_uv (2 div), ndc (4), two mat4 x vec4 (2 x 28), normalize (8 + rsq), depth tap"),
    "sky_pixel": ((35 + 23, 2, 0), "sky_pixels",
                  "bayer16 (28), r0 (3), sun factor (4) :461-477; atmosphere entry :355-359: normalize (8 + rsq), "
                  "rsi (15 + sqrt)"),
    "atmosphere_full": ((3664, 498, 0), "atmosphere_full",
                        "atmosphere :360-438 past the early exit: rsi (15 + sqrt), step size (2), phases (15 + pow), "
                        "16 primary steps x 226 FLOPs + 31 transcendentals (position 8, height 6 + sqrt, two optical "
                        "depths 4 + 2 exp, accumulators 2, secondary step size 16 + sqrt, 8 secondary steps x (21 + "
                        "sqrt + 2 exp), attenuation 9 + 3 exp, scattering sums 12, time 1), result (16)"),
    "cloud_march": ((227, 9, 0), "cloud_marches",
                    "calculate_volumetric_clouds :314-346 for ray_direction.y >= 0: two rsi (30 + 2 sqrt), start / end "
                    "/ increment / position (21), step length (5 + sqrt), phase_two_lobes (5 + 11 + 2 pow), "
                    "calculate_atmospheric_scattering_top :195-217 (39 + 3 exp), final mix (23 + sqrt), 24 x (od "
                    "scale 1 + position 3)"),
    "get_clouds": ((11, 1, 0), "get_clouds",
                   "get_clouds :236-240 up to the altitude test: length (9 + sqrt), camera offset (2)"),
    "get_clouds_full": ((89, 2, 8), "get_clouds_full",
                        "get_clouds :242-261 past the altitude test: time (1), coordinates (6), four octaves of "
                        "get_3d_noise (:219-233, 11 FLOPs + 2 taps each) with their coordinates and weights (25), "
                        "threshold (4 + 2 exp), smoothstep (6), density (2)"),
    "dense_step": ((83, 4, 0), "dense_steps",
                   "a march step with od > 0 :342-343: scatter integral (3 + exp), powder (3 + exp), getSunVisibility "
                   ":264-278 (40 + exp, its 10 get_clouds counted above), lighting (30), accumulation (6), "
                   "transmittance (1 + exp)"),
}


def tally(counters):
    """Total FLOPs, transcendentals and taps of one CloudRendering pass from the oracle's counters."""
    f = t = x = 0
    rows = {}
    for name, ((fl, tr, tp), ctr, why) in WORK.items():
        n = counters[ctr]
        rows[name] = {"entries": n, "flops_each": fl, "transcendentals_each": tr, "taps_each": tp, "glsl": why}
        f += n * fl
        t += n * tr
        x += n * tp
    return {"flops": f, "transcendentals": t, "taps": x, "flops_with_filter": f + FILTER_FLOPS_PER_TAP * x,
            "entries": rows}


def roofline(totals, us):
    """Achieved rates of the counted work in `us` microseconds against the FP32 / transcendental peaks."""
    floor_us = totals["flops"] / (FP32_PEAK_TFLOPS * 1e12) * 1e6 + totals["transcendentals"] / (TRANS_PEAK_T * 1e12) * 1e6
    floor_f_us = (totals["flops_with_filter"] / (FP32_PEAK_TFLOPS * 1e12) * 1e6
                  + totals["transcendentals"] / (TRANS_PEAK_T * 1e12) * 1e6)
    ach = totals["flops"] / (us * 1e-6) / 1e12
    return {"bound": "valu", "unit": "TFLOP/s", "peak": FP32_PEAK_TFLOPS, "avg_launch_us": round(us, 2),
            "achieved": round(ach, 2), "frac": round(ach / FP32_PEAK_TFLOPS, 4),
            "achieved_with_filter": round(totals["flops_with_filter"] / (us * 1e-6) / 1e12, 2),
            "transcendentals_per_s_T": round(totals["transcendentals"] / (us * 1e-6) / 1e12, 2),
            "transcendental_peak_T": round(TRANS_PEAK_T, 2),
            "floor_us": round(floor_us, 2), "frac_of_floor": round(floor_us / us, 4),
            "floor_with_filter_us": round(floor_f_us, 2), "frac_of_floor_with_filter": round(floor_f_us / us, 4)}


def main():
    import numpy as np
    import torch

    import bench
    import oracle
    import soc_real_time_renderer_amd as soc
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "clouds_flops.json"))
    ap.add_argument("--configs", default="c3,c4")
    ap.add_argument("--reps", type=int, default=50)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    W, H = 3840, 2160
    res = {"resolution": [W, H], "conventions": __doc__.split("Roofline:")[0].strip(), "configs": {}}
    for config in args.configs.split(","):
        g, gb, shadow, noise, _sc, fr = bench.build_inputs(config, "mesh", W, H, 0, dev)
        clouds = np.zeros((H, W, 4), np.uint8)
        t0 = time.perf_counter()
        oracle.cloud_rendering(g, gb["depth"], noise, clouds)
        cpu_s = time.perf_counter() - t0
        ctr = oracle.clouds_counters()
        tot = tally(ctr)
        # the GPU pass alone (the renderer's CloudRendering: classify, atmosphere, density, sun visibility, resolve)
        out = torch.zeros(H, W, 4, dtype=torch.uint8, device=dev)
        for _ in range(5):
            soc.cloud_rendering(g, fr["depth"], fr["noise"], out, fr["clouds_workspace"])
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.reps):
            soc.cloud_rendering(g, fr["depth"], fr["noise"], out, fr["clouds_workspace"])
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / args.reps * 1e3
        d = np.abs(out.cpu().numpy().astype(np.int32) - clouds.astype(np.int32))
        sky = max(ctr["sky_pixels"], 1)
        res["configs"][config] = {
            "f_sky": round(ctr["sky_pixels"] / ctr["pixels"], 4), "counters": ctr,
            "per_sky_pixel": {"flops": round(tot["flops"] / sky, 1), "transcendentals": round(tot["transcendentals"] / sky, 1),
                              "taps": round(tot["taps"] / sky, 1),
                              "dense_steps": round(ctr["dense_steps"] / sky, 3)},
            **{k: tot[k] for k in ("flops", "transcendentals", "taps", "flops_with_filter")},
            "gpu_standalone": roofline(tot, us),
            "oracle_seconds": round(cpu_s, 2), "oracle_threads": oracle.num_threads(),
            "gpu_vs_oracle_within2": float((d <= 2).mean()), "entries": tot["entries"]}
        print(config, json.dumps({k: v for k, v in res["configs"][config].items() if k != "entries"}), flush=True)
        del fr
        torch.cuda.empty_cache()
    with open(args.out, "w") as fh:
        json.dump(res, fh, indent=1)
    print("wrote", args.out)


if __name__ == "__main__":
    main()
