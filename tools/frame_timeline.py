#!/usr/bin/env python
"""Per-frame kernel timeline from a rocprofv3 kernel trace: for frames k .. k + n (a frame starts at each launch of
the first bloom kernel), every kernel's begin / end in microseconds after the frame's start, its stream and the idle
gaps of each stream. Compares the frame shapes of two runs (e.g. the default bench and `bench.py --exchange`).

    python tools/frame_timeline.py KERNEL_TRACE.csv [--frame K] [--frames N] [--marker bloomw_down01p]
"""
import argparse
import collections
import csv


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("void ", "").replace("soc::", "")
    return n.split("(")[0][:40]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--frame", type=int, default=150)
    ap.add_argument("--frames", type=int, default=3)
    ap.add_argument("--marker", default="bloomw_down01p")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                  (r.get("Queue_Id"), r.get("Stream_Id"))) for r in rows), key=lambda t: t[0])
    starts = [k[0] for k in ks if a.marker in k[2]]
    spans = []
    for f in range(a.frame, min(a.frame + a.frames, len(starts) - 1)):
        t0, t1 = starts[f], starts[f + 1]
        sel = [k for k in ks if t0 <= k[0] < t1]
        spans.append((t1 - t0) / 1e3)
        print(f"frame {f}: {(t1 - t0) / 1e3:.1f} us")
        last_end = collections.defaultdict(lambda: None)
        for b, e, n, q in sel:
            gap = "" if last_end[q] is None else f"gap {(b - last_end[q]) / 1e3:6.1f}"
            print(f"  {(b - t0) / 1e3:8.1f} .. {(e - t0) / 1e3:8.1f}  ({(e - b) / 1e3:6.1f})  q{q[0]}/s{q[1]}  {n:40s} {gap}")
            last_end[q] = e if last_end[q] is None else max(e, last_end[q])
    all_spans = [(starts[i + 1] - starts[i]) / 1e3 for i in range(len(starts) - 1)]
    mid = sorted(all_spans[len(all_spans) // 4:])
    print(f"frames {len(all_spans)}: median span {mid[len(mid) // 2]:.1f} us (after the first quarter)")


if __name__ == "__main__":
    main()
