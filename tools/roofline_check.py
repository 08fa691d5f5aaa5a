"""Agreement of the bench line's roofline durations with rocprofv3. The bench measures the north-star kernels with HIP
events on their stream twice: alone (the serial per-pass profile frames: the roofline's headline) and in its timed
frames (lanes concurrent: `in_frame`). This takes a `tools/gpu.sh kt` kernel trace of the same command (`bench.py
--steps K --warmup W`: W warm-up frames, the untimed lane-probe frames, K timed frames, then the serial per-pass profile
frames) and averages each
kernel over the same kind of launch: the profile frames for the headline, the timed frames for in_frame. The kernel
trace's own `--stats` average mixes the three segments. A kernel trace changes how the two lanes overlap, so the
in-frame pair of an untraced bench run and a traced run need not agree; within one traced run events and trace do
(tools/event_trace_check.py, SOC_BENCH_EVENTS_OUT).

usage: python tools/roofline_check.py BENCH_JSON KT_DIR [--warmup W] [--steps K] > profiles/<tag>_roofline_check.json
(W and K default to the bench line's own, i.e. a kernel trace of the same command)
"""
import csv
import glob
import json
import os
import sys

KERNELS = {"SSAOGeneration": "ssao_pipe_kernel", "Composition+GenerateLuminanceHistogram": "composition_pair<true"}
# round 5's SSAO kernel (SOC_SSAO_PIPE=0): traces of that build
KERNELS_R5 = {"SSAOGeneration": "ssao_lds_kernel"}


def main():
    args = sys.argv[1:]
    warmup = steps = None
    if "--warmup" in args:
        i = args.index("--warmup")
        warmup = int(args[i + 1])
        del args[i:i + 2]
    if "--steps" in args:
        i = args.index("--steps")
        steps = int(args[i + 1])
        del args[i:i + 2]
    bench_json, kt_dir = args
    line = json.load(open(bench_json))
    warmup = line["warmup"] if warmup is None else warmup
    steps = line["steps"] if steps is None else steps
    # the untimed frames the bench runs after the warm-up until the renderer's lane probe has decided
    probe = int(line.get("config", {}).get("untimed_lane_probe_frames") or 0)
    warmup += probe
    trace = glob.glob(os.path.join(kt_dir, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
    out = {"bench_line": bench_json, "kernel_trace": trace, "warmup": warmup, "untimed_lane_probe_frames": probe,
           "timed": steps, "kernels": {}}
    pair_events = pair_rocprof = 0.0
    # the serial per-pass profile frames follow the timed ones; after them (round 6) the unfused renderer's frames of
    # ms_per_group_unfused, which run the same SSAO kernel: excluded
    profile = int(line.get("config", {}).get("profile_frames") or 20)
    for name, key in KERNELS.items():
        d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if key in r["Kernel_Name"]]
        if not d and name in KERNELS_R5:
            d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if KERNELS_R5[name] in r["Kernel_Name"]]
        timed = d[warmup:warmup + steps]
        prof = d[warmup + steps:warmup + steps + profile]
        pk = line["roofline"]["per_kernel"][name]
        ev = pk["avg_launch_us"]                      # alone
        ev_frame = (pk.get("in_frame") or {}).get("avg_launch_us")
        rp = sum(prof) / max(1, len(prof))
        rp_frame = sum(timed) / len(timed)
        out["kernels"][name] = {"bench_events_alone_us": ev, "rocprof_profile_frames_us": round(rp, 2),
                                "ratio": round(ev / rp, 3),
                                "bench_events_in_frame_us": ev_frame, "rocprof_timed_frames_us": round(rp_frame, 2),
                                "ratio_in_frame_cross_run": round(ev_frame / rp_frame, 3) if ev_frame else None}
        pair_events += ev
        pair_rocprof += rp
    out["pair"] = {"bench_events_alone_us": round(pair_events, 2), "rocprof_profile_frames_us": round(pair_rocprof, 2),
                   "ratio": round(pair_events / pair_rocprof, 3)}
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
