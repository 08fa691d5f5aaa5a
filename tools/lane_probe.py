#!/usr/bin/env python
"""Probe: does a third concurrent lane pay? Times the bench's C3 bloom chain (4 weighted stages), SSAO + blur and
CloudRendering (the sky lane's work) on the bench's own 4K inputs, each alone, and together on one, two or three HIP
streams (torch streams, the C-ABI pass calls), averaged over N repetitions.

    python tools/lane_probe.py [--reps 50]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
import soc_real_time_renderer_amd as soc  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    W, H = 3840, 2160
    g, _gb, _sh, _nz, _sc, fr = bench.build_inputs("c3", "mesh", W, H, 0, dev)
    soc.ssao_prepare_noise(fr["normal"], fr["ssao"], fr["ssao_noise_table"])
    ws = fr["clouds_workspace"]
    sA, sB, sC = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()

    def bloom(s):
        for k in range(1, 5):
            soc.bloom_weighted_stage(g, fr["emissive"], fr["bloom_mips"], fr["bloom_output"], k, stream=s)

    def ao(s):
        soc.ssao_generation(g, fr["depth"], fr["normal"], fr["ssao"], fr["ssao_noise_table"], stream=s)
        soc.ssao_blur(g, fr["ssao"], fr["ssao_blur"], stream=s)

    def sky(s):
        soc.cloud_rendering(g, fr["depth"], fr["noise"], fr["clouds"], ws, stream=s)

    def timed(name, plan):
        """plan: list of (stream, [work...]) run per repetition; streams joined each repetition."""
        torch.cuda.synchronize()
        for _ in range(5):
            run(plan)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            run(plan)
        e1.record()
        torch.cuda.synchronize()
        print(f"{name:45s} {e0.elapsed_time(e1) / a.reps * 1e3:8.1f} us", flush=True)

    def run(plan):
        cur = torch.cuda.current_stream()
        fork = torch.cuda.Event()
        fork.record(cur)
        for s, works in plan:
            s.wait_event(fork)
            for w in works:
                w(s)
        for s, _ in plan:
            j = torch.cuda.Event()
            j.record(s)
            cur.wait_event(j)

    timed("bloom alone", [(sA, [bloom])])
    timed("ssao+blur alone", [(sA, [ao])])
    timed("clouds alone", [(sA, [sky])])
    timed("bloom, ssao on one lane", [(sA, [bloom, ao])])
    timed("bloom | ssao (2 lanes)", [(sA, [bloom]), (sB, [ao])])
    timed("bloom, ssao | clouds (2 lanes)", [(sA, [bloom, ao]), (sC, [sky])])
    timed("ssao, bloom | clouds (2 lanes)", [(sA, [ao, bloom]), (sC, [sky])])
    timed("bloom | ssao | clouds (3 lanes)", [(sA, [bloom]), (sB, [ao]), (sC, [sky])])


if __name__ == "__main__":
    main()
