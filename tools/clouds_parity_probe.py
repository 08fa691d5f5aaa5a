"""CloudRendering against the oracle on the bench's own 4K frames, per variant: which part of the pass's arithmetic puts
sky texels an RGBA8 level away from the oracle's.

For each config (C3: the Sponza-proxy atrium, every sky pixel looking up through the court; C4: the terrain, half the
frame sky) the oracle's clouds are computed once; then the GPU pass runs under each knob set given on the command line
(KNOB=V[,KNOB=V...]; "" = the defaults) and the sky texels are compared: the fraction differing by >= 1 level, >= 2,
the maximum, and the mean signed difference per channel (a bias shows a systematic deviation, not rounding-edge noise).
The library is the one SOC_RT_LIB_VARIANT names (e.g. libsoc_rt_precise.so: clouds.hip built with
SOC_CLOUDS_PRECISE=1, the library's accurate exp / exp2 / sqrt / log2 / division instead of the hardware forms).

usage: python tools/clouds_parity_probe.py [--configs c3,c4] [--out FILE] VARIANT...
Test infrastructure (it runs the oracle); prints one JSON line per (config, variant).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle  # noqa: E402
import soc_real_time_renderer_amd as soc  # noqa: E402
from bench import build_inputs  # noqa: E402


def compare(gpu, ref, sky):
    d = gpu[..., :3].astype(np.int32) - ref[..., :3].astype(np.int32)
    a = np.abs(d).max(axis=-1)
    s = a[sky]
    return {"sky_px": int(sky.sum()), "differ": round(float((s > 0).mean()), 6), "differ2": round(float((s > 1).mean()), 6),
            "max": int(a.max()), "mean_signed": [round(float(d[..., c][sky].mean()), 5) for c in range(3)],
            "nonsky_differ": int((a[~sky] > 0).sum()),
            "worst": [[int(y), int(x), int(a[y, x]), gpu[y, x, :3].tolist(), ref[y, x, :3].tolist()]
                      for y, x in zip(*np.unravel_index(np.argsort(a, axis=None)[::-1][:6], a.shape)) if a[y, x] > 1]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c3,c4")
    ap.add_argument("--out", default="")
    ap.add_argument("variants", nargs="*")
    a = ap.parse_args()
    variants = a.variants or [""]
    dev = torch.device("cuda", 0)
    lines = []
    for config in a.configs.split(","):
        W, H = (1920, 1080) if config == "c2" else (3840, 2160)
        g, gb, _sh, nz, _sc, fr = build_inputs(config, "mesh", W, H, 0, dev)
        sky = gb["depth"] == 1.0
        ref = np.zeros((H, W, 4), np.uint8)
        t0 = time.perf_counter()
        oracle.cloud_rendering(g, gb["depth"], nz, ref)
        print(f"{config}: oracle clouds {time.perf_counter() - t0:.1f} s", file=sys.stderr, flush=True)
        for v in variants:
            env = dict(kv.split("=") for kv in v.split(",") if kv)
            old = {k: os.environ.get(k) for k in env}
            os.environ.update(env)
            soc.reload_tuning()
            o = torch.zeros(H, W, 4, dtype=torch.uint8, device=dev)
            soc.cloud_rendering(g, fr["depth"], fr["noise"], o, fr["clouds_workspace"])
            torch.cuda.synchronize()
            rep = {"config": config, "lib": os.environ.get("SOC_RT_LIB_VARIANT", "libsoc_rt.so"), "variant": v or "default",
                   **compare(o.cpu().numpy(), ref, sky)}
            for k, val in old.items():
                if val is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = val
            soc.reload_tuning()
            line = json.dumps(rep)
            print(line, flush=True)
            lines.append(line)
    if a.out:
        with open(a.out, "a") as fh:
            fh.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
