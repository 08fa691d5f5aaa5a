"""Kernel timelines from a rocprofv3 kernel trace of the bench.

  python tools/timeline.py <run_kernel_trace.csv>           one frame (start/end us relative to the frame's first bloom
                                                             kernel, queue id)
  python tools/timeline.py --lanes <run_kernel_trace.csv>   the timed frames (the longest run of frame periods within 1.5x of the
                                                             lower-quartile period):
                                                             per queue, busy time, the gaps between consecutive kernels
                                                             and each kernel's time, per frame
"""
import collections
import csv
import sys


def name(r):
    return (r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
            .replace("soc::", ""))


def frame(rows):
    idx = [i for i, r in enumerate(rows) if "bloomw_down01" in r["Kernel_Name"]]
    i0, i1 = idx[len(idx) // 2], idx[len(idx) // 2 + 1]
    t0 = int(rows[i0]["Start_Timestamp"])
    for r in rows[i0:i1 + 1]:
        s = (int(r["Start_Timestamp"]) - t0) / 1e3
        e = (int(r["End_Timestamp"]) - t0) / 1e3
        print(f"{name(r)[:44]:44s} q{r.get('Queue_Id', '?'):>3s} {s:8.1f} {e:8.1f} {e - s:7.1f}")


def lanes(rows):
    idx = [i for i, r in enumerate(rows) if "bloomw_down01" in r["Kernel_Name"]]
    st = [int(rows[i]["Start_Timestamp"]) for i in idx]
    d = [(b - a) / 1e3 for a, b in zip(st, st[1:])]
    lim = 1.5 * sorted(d)[len(d) // 4]   # the timed loop's periods sit near the short end; warm-up / profile frames do not
    best, i = (0, 0), 0
    while i < len(d):
        j = i
        while j < len(d) and d[j] < lim:
            j += 1
        if j - i > best[1] - best[0]:
            best = (i, j)
        i = j + 1
    sel = idx[best[0] + 1:best[1]]   # drop the run's first and last frame
    t0, t1, nfr = int(rows[sel[0]]["Start_Timestamp"]), int(rows[sel[-1]]["Start_Timestamp"]), len(sel) - 1
    print(f"frames {nfr}, {(t1 - t0) / 1e3 / nfr:.1f} us per frame")
    byq = collections.defaultdict(list)
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if t0 <= s < t1:
            byq[r["Queue_Id"]].append((s, e, name(r).split("<")[0]))
    for q, l in sorted(byq.items()):
        gaps, kt = collections.Counter(), collections.Counter()
        for s, e, n in l:
            kt[n] += (e - s) / 1e3
        for (s, e, n), (s2, _, n2) in zip(l, l[1:]):
            gaps[(n, n2)] += (s2 - e) / 1e3
        busy = sum(e - s for s, e, _ in l) / 1e3
        print(f"queue {q}: busy {busy / nfr:.1f} us per frame, gaps {sum(gaps.values()) / nfr:.1f}")
        for k, v in kt.most_common():
            print(f"   kernel {k:28s} {v / nfr:7.1f}")
        for k, v in gaps.most_common(6):
            print(f"   gap    {k[0][:24]:24s} -> {k[1][:24]:24s} {v / nfr:6.1f}")


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if a != "--lanes"]
    rows = sorted(csv.DictReader(open(args[0])), key=lambda r: int(r["Start_Timestamp"]))
    (lanes if "--lanes" in sys.argv else frame)(rows)
