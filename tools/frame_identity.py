"""Frame identity probe: renders the bench's frames (bench.build_inputs, the bench's renderer flags) under tuning-knob
variants and checks that every frame output (colour, framebuffer, SSAO, clouds, exposure block) is bit-identical to
the default variant's, frame after frame. An A/B tool for variants that claim the same bits (e.g. packed-f32 forms).

usage: python tools/frame_identity.py [--config c3|c4] [--frames N] KNOB=V[,KNOB=V...] ...
       python tools/frame_identity.py --hash [--config c3|c4]      (one digest per output and frame: compare two builds,
                                                                   e.g. SOC_RT_LIB_VARIANT=libsoc_rt_base.so)
"""
import argparse
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
import soc_real_time_renderer_amd as soc  # noqa: E402

KEYS = ("color", "output", "ssao", "clouds", "auto_exposure")


def render(config, frames, env):
    saved = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    soc.reload_tuning()
    try:
        W, H = 3840, 2160
        dev = torch.device("cuda", 0)
        g, gb, shadow, noise, sc, fr = bench.build_inputs(config, "mesh", W, H, 0, dev)
        r = soc.Renderer(fr, static_inputs=True)
        r.set_exposure_pixels(W * H, False)
        out = []
        for _ in range(frames):
            r.execute(g)
            torch.cuda.synchronize()
            out.append({k: fr[k].clone() for k in KEYS if k in fr})
        r.close()
        return out
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        soc.reload_tuning()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--frames", type=int, default=3)
    ap.add_argument("--hash", action="store_true")
    ap.add_argument("variants", nargs="*")
    a = ap.parse_args()
    ref = render(a.config, a.frames, {})
    if a.hash:
        d = hashlib.sha256()
        for f in ref:
            for k in sorted(f):
                d.update(f[k].cpu().numpy().tobytes())
        print(f"{a.config} {os.environ.get('SOC_RT_LIB_VARIANT', 'libsoc_rt.so')} frames {a.frames} digest {d.hexdigest()[:16]}",
              flush=True)
    for v in a.variants:
        env = dict(kv.split("=") for kv in v.split(",") if kv)
        got = render(a.config, a.frames, env)
        same = {k: all(torch.equal(f[k], r[k]) for f, r in zip(got, ref)) for k in ref[0]}
        print(f"{a.config} variant {v}: bit-identical {all(same.values())} {same}", flush=True)


if __name__ == "__main__":
    main()
