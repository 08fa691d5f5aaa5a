"""One rank of the frame-per-GPU path on the GPU (started by tests/test_gpu_distributed.py through
torch.distributed.run; not collected by pytest).

Every rank renders its own camera through the HIP render graph (soc_renderer): PRE_EXPOSURE phase (which
ends with the LuminanceHistogramFold of the fused composition + histogram launch), the histogram exchange
(multi_gpu.exchange_histogram: the all-reduce slotted between the reference's histogram and resolve tasks,
renderer.cpp:1155-1168), then POST_EXPOSURE with the wide resolve over N*W*H pixels. Rank 0 writes what
every rank saw to $SOC_DIST_OUT (npz) for the test to check against the oracle.

SOC_BENCH_SHARE_DEVICE=1 puts all ranks on device 0 and the backend is gloo (RCCL refuses two ranks on
one device), so the test runs on a 1-GPU box.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import soc_real_time_renderer_amd as soc  # noqa: E402
from helpers import globals_for  # noqa: E402
from soc_real_time_renderer_amd import multi_gpu, scene  # noqa: E402

W, H, FRAMES = int(os.environ.get("SOC_DIST_W", "160")), int(os.environ.get("SOC_DIST_H", "96")), 2


def main():
    rank, world, local_rank = multi_gpu.env()
    dev_index = 0 if os.environ.get("SOC_BENCH_SHARE_DEVICE") == "1" else local_rank
    torch.cuda.set_device(dev_index)
    device = torch.device("cuda", dev_index)
    multi_gpu.init(device, backend=os.environ.get("SOC_DIST_BACKEND", "gloo"))
    g = globals_for(W, H, camera=multi_gpu.camera_for_rank(rank), elapsed=10.0, frame_counter=2)
    gb = scene.gbuffer(g, W, H)
    fr = soc.alloc_frame(W, H, device)
    for k in ("albedo", "emissive", "normal", "velocity", "depth"):
        fr[k].copy_(torch.from_numpy(gb[k]))
    fr["shadow"] = torch.from_numpy(scene.shadow_map(g, 256)).to(device)
    fr["noise"].copy_(torch.from_numpy(scene.noise_texture()))
    r = soc.Renderer(fr)
    r.set_exposure_pixels(*multi_gpu.exposure_pixels(world, W, H))
    bins = fr["auto_exposure"][1:]
    rec = {"local": [], "reduced": [], "exposure": [], "color": []}
    for _ in range(FRAMES):
        r.execute(g, soc.PHASE_PRE_EXPOSURE)
        torch.cuda.synchronize()
        rec["local"].append(bins.cpu().numpy().view(np.uint32).copy())
        rec["color"].append(fr["color"].cpu().numpy().copy())
        multi_gpu.exchange_histogram(bins)
        torch.cuda.synchronize()
        rec["reduced"].append(bins.cpu().numpy().view(np.uint32).copy())
        r.execute(g, soc.PHASE_POST_EXPOSURE)
        torch.cuda.synchronize()
        rec["exposure"].append(soc.exposure_of(fr["auto_exposure"]))
        # the resolve clears the bins for the next frame (resolve_luminance_histogram.inl:63)
        assert int(bins.abs().sum()) == 0
    r.close()
    everyone = multi_gpu.gather_objects({k: np.stack(v) if k != "exposure" else np.array(v) for k, v in rec.items()})
    if rank == 0:
        out = {}
        for k in rec:
            out[k] = np.stack([e[k] for e in everyone])
        np.savez(os.environ["SOC_DIST_OUT"], world=world, W=W, H=H, **out)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
