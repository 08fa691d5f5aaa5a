"""Does the host run ahead of the GPU in the bench's frame loop? The C3 4K renderer (static inputs, second lane on)
is warmed up, then N frames are enqueued back to back without a synchronize; the host time of every execute() call
and the GPU time of the whole batch are printed. A host far ahead of the GPU lets the second lane start a frame's
clouds as soon as the previous frame's SkyCompose is done; a host that returns from execute() only at GPU pace
means something in the call blocks (the lane then starts late). usage: python tools/host_ahead_probe.py [frames]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
import soc_real_time_renderer_amd as soc  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 60
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    g, gb, shadow, noise, sc, fr = bench.build_inputs("c3", "mesh", 3840, 2160, 0, dev)
    for static in (True, False):
        r = soc.Renderer(fr, sky_lane=True, static_inputs=static)
        for _ in range(10):
            r.execute(g)
        torch.cuda.synchronize()
        host = []
        t0 = time.perf_counter()
        for _ in range(n):
            a = time.perf_counter()
            r.execute(g)
            host.append(time.perf_counter() - a)
        t_enq = time.perf_counter() - t0
        torch.cuda.synchronize()
        t_all = time.perf_counter() - t0
        host_us = sorted(h * 1e6 for h in host)
        print(f"static_inputs={static}: {n} frames enqueued in {t_enq * 1e3:.2f} ms, GPU done after {t_all * 1e3:.2f} ms "
              f"({t_all / n * 1e6:.0f} us/frame); execute() host time median {host_us[n // 2]:.0f} us, "
              f"max {host_us[-1]:.0f} us, first 5 {[round(h * 1e6) for h in host[:5]]}, last 5 "
              f"{[round(h * 1e6) for h in host[-5:]]}", flush=True)
        r.close()


if __name__ == "__main__":
    main()
