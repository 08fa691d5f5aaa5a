#!/usr/bin/env python
"""Pass events against the kernel trace of the SAME run (the bench's hipEvent interval for
Composition was shorter than the kernel's trace duration, but the two came from different runs).

  python tools/event_trace_check.py run OUT.json [--frames N --warmup W]
      the bench's C3 frame loop (bench.build_inputs, the bench's renderer flags) with the bench's pass events on
      Composition(+histogram) and SSAOGeneration; writes every timed frame's event times (ms after a base event
      recorded before the timed frames) to OUT.json. Run it under `rocprofv3 --kernel-trace` to get the trace.
      (bench.py itself writes the same file for its timed frames with SOC_BENCH_EVENTS_OUT=OUT.json.)
  python tools/event_trace_check.py compare OUT.json KERNEL_TRACE.csv
      aligns the events with the trace's launches of the same kernels (launches warmup .. warmup + frames of each)
      and prints, per kernel, the event interval, the trace duration and where each event falls against the kernel's
      begin / end.
"""
import csv
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

KERNELS = {"SSAOGeneration": "ssao_pipe_kernel", "Composition+GenerateLuminanceHistogram": "composition_pair<true"}
# round 5's SSAO kernel (SOC_SSAO_PIPE=0): traces of that build
KERNELS_R5 = {"SSAOGeneration": "ssao_lds_kernel"}


def run(out, frames, warmup):
    import torch

    import bench
    import soc_real_time_renderer_amd as soc
    dev = torch.device("cuda", 0)
    g, gb, _sh, _nz, _sc, fr = bench.build_inputs("c3", "mesh", 3840, 2160, 0, dev)
    r = soc.Renderer(fr, static_inputs=True)
    names = r.pass_names()
    for _ in range(warmup):
        r.execute(g)
    torch.cuda.synchronize()
    idx = {n: names.index(n) for n in KERNELS}
    for i in idx.values():
        r.set_pass_timing(i, True)
    r.reset_timing()
    base = torch.cuda.Event(enable_timing=True)
    base.record()
    end = torch.cuda.Event(enable_timing=True)
    for _ in range(frames):
        r.execute(g)
    end.record()
    torch.cuda.synchronize()
    res = {"frames": frames, "warmup": warmup, "total_ms": base.elapsed_time(end), "passes": {}}
    for n, i in idx.items():
        s0, s1 = r.pass_event_times(i, base, frames)
        res["passes"][n] = {"start_ms": s0.tolist(), "end_ms": s1.tolist(), "mean_us": float((s1 - s0).mean() * 1e3)}
        print(n, "event mean us", round(res["passes"][n]["mean_us"], 2))
    r.close()
    with open(out, "w") as f:
        json.dump(res, f)


def trace_launches(path, key):
    rows = list(csv.DictReader(open(path)))
    kn = "Kernel_Name" if "Kernel_Name" in rows[0] else "Name"
    sel = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows if key in r[kn]]
    return np.array(sorted(sel), np.float64)


def compare(events_json, trace_csv):
    ev = json.load(open(events_json))
    n = ev["frames"]
    out = {"events": events_json, "trace": trace_csv, "frames": n, "kernels": {}}
    offs = {}
    for name, key in KERNELS.items():
        e = ev["passes"][name]
        e0, e1 = np.array(e["start_ms"]) * 1e6, np.array(e["end_ms"]) * 1e6   # ns after the base event
        tl = trace_launches(trace_csv, key)
        if len(tl) == 0 and name in KERNELS_R5:
            tl = trace_launches(trace_csv, KERNELS_R5[name])
        tl = tl[ev["warmup"]:ev["warmup"] + n]
        tb, te = tl[:, 0], tl[:, 1]
        offs[name] = float(np.median(te - e1))    # trace clock = event clock + offset, if end events mark kernel ends
        out["kernels"][name] = {"event_us": float((e1 - e0).mean() / 1e3), "trace_us": float((te - tb).mean() / 1e3),
                                "ratio": float((e1 - e0).mean() / (te - tb).mean()), "_e": (e0, e1, tb, te)}
    # one offset for the whole run (the event clock is shared): the SSAO ends' (SSAO events agree with the trace)
    off = offs["SSAOGeneration"]
    out["offset_from_ssao_ends_ns"] = off
    out["offset_from_composition_ends_ns"] = offs["Composition+GenerateLuminanceHistogram"]
    for name, k in out["kernels"].items():
        e0, e1, tb, te = k.pop("_e")
        k["start_event_minus_kernel_begin_us_median"] = float(np.median(e0 + off - tb) / 1e3)
        k["end_event_minus_kernel_end_us_median"] = float(np.median(e1 + off - te) / 1e3)
        k["end_event_minus_kernel_begin_us_median"] = float(np.median(e1 + off - tb) / 1e3)
    print(json.dumps(out, indent=1))
    return out


if __name__ == "__main__":
    if sys.argv[1] == "run":
        a = sys.argv[2:]
        frames = int(a[a.index("--frames") + 1]) if "--frames" in a else 200
        warmup = int(a[a.index("--warmup") + 1]) if "--warmup" in a else 100
        run(a[0], frames, warmup)
    else:
        compare(sys.argv[2], sys.argv[3])
