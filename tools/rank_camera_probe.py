"""Per-rank workload balance of the multi-GPU bench: every rank of `bench.py --gpus N` renders its own camera
(multi_gpu.camera_for_rank / terrain_camera_for_rank) and the histogram exchange makes the frames lockstep, so the
slowest rank's frame sets the pace. This renders each rank's C3 (or C4) frame on one GPU, one after another, and
prints its sky fraction and frames/sec (the renderer and inputs exactly as bench.py builds them for that rank).

usage: python tools/rank_camera_probe.py [c3|c4] [ranks]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
import soc_real_time_renderer_amd as soc  # noqa: E402


def main():
    config = sys.argv[1] if len(sys.argv) > 1 else "c3"
    ranks = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    for rank in range(ranks):
        g, gb, shadow, noise, sc, fr = bench.build_inputs(config, "mesh", 3840, 2160, rank, dev)
        f_sky = float((gb["depth"] == 1.0).mean())
        r = soc.Renderer(fr, static_inputs=True)
        for _ in range(10):
            r.execute(g)
        torch.cuda.synchronize()
        n = 40
        t0 = time.perf_counter()
        for _ in range(n):
            r.execute(g)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        # per pass, lanes serialised, every pass evented (as bench.py's ms_per_pass)
        r.set_async(False)
        r.set_pass_timing(-1, True)
        r.reset_timing()
        for _ in range(10):
            r.execute(g)
        torch.cuda.synchronize()
        per = {name: round(ms * 1e3, 1) for name, _, ms, cnt in r.pass_stats() if cnt}
        big = {k: v for k, v in per.items() if v >= 20.0}
        print(f"{config} rank {rank}: f_sky {f_sky:.3f}, {n / dt:.1f} frames/sec ({dt / n * 1e3:.3f} ms); passes us {big}",
              flush=True)
        r.close()
        del fr, sc
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
