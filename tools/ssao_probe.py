"""SSAO variant probe at 4K on the C3 G-buffer: times SSAOGeneration under tuning knobs (environment variables,
re-read through soc_tuning_reload) and checks every variant's output against the default's bits.
PROBE_SCENE=mesh (default): the Sponza-proxy mesh rasterised by the HIP rasteriser, as bench.py renders it;
PROBE_SCENE=boxes: the round-1 box atrium.

usage: python tools/ssao_probe.py KNOB=V[,KNOB=V...] ...   (each argument is one variant; "" = default)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import soc_real_time_renderer_amd as soc  # noqa: E402
from soc_real_time_renderer_amd import multi_gpu, raster, scene  # noqa: E402
from bench import make_globals  # noqa: E402


def main():
    W, H = int(os.environ.get("PROBE_W", 3840)), int(os.environ.get("PROBE_H", 2160))
    dev = torch.device("cuda", 0)
    g = make_globals(W, H, multi_gpu.camera_for_rank(0))
    if os.environ.get("PROBE_SCENE", "mesh") == "mesh":
        sc = raster.scene_setup(g, scene.SPONZA_MESH, tex_size=256, device=dev)
        gbd = raster.render_gbuffer(g, sc, W, H, 1024, dev)
        depth, normal = gbd["depth"], gbd["normal"]
    else:
        gb = scene.gbuffer(g, W, H)
        depth = torch.from_numpy(gb["depth"]).to(dev)
        normal = torch.from_numpy(gb["normal"]).to(dev)
    table = torch.zeros((H // 2) * (W // 2) * 2, dtype=torch.float32, device=dev)
    ref = torch.zeros(H // 2, W // 2, dtype=torch.uint8, device=dev)
    soc.ssao_prepare_noise(normal, ref, table)
    variants = sys.argv[1:] or [""]
    soc.ssao_generation(g, depth, normal, ref, table)
    torch.cuda.synchronize()
    for v in variants:
        env = dict(kv.split("=") for kv in v.split(",") if kv)
        saved = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        soc.reload_tuning()
        out = torch.zeros_like(ref)
        for _ in range(5):
            soc.ssao_generation(g, depth, normal, out, table)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 50
        e0.record()
        for _ in range(n):
            soc.ssao_generation(g, depth, normal, out, table)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / n * 1e3
        same = bool(torch.equal(out, ref))
        d = (out.int() - ref.int()).abs()
        bad = torch.nonzero(d)
        where = bad[:3].tolist() if len(bad) else []
        print(f"variant {v or 'default'}: {us:.1f} us per call, bit-identical to default: {same} "
              f"(differing px {len(bad)}, max |d| {int(d.max())}, first {where})", flush=True)
        for k, old in saved.items():
            if old is None:
                os.environ.pop(k)
            else:
                os.environ[k] = old


if __name__ == "__main__":
    main()
