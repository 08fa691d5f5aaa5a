"""One frame's kernel timeline (start/end µs relative to the frame's first bloom kernel, queue id) from a
rocprofv3 kernel trace of the bench. usage: python tools/timeline.py <run_kernel_trace.csv>"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "bloomw_down01" in r["Kernel_Name"]]
i0, i1 = idx[len(idx) // 2], idx[len(idx) // 2 + 1]
t0 = int(rows[i0]["Start_Timestamp"])
for r in rows[i0:i1 + 1]:
    s = (int(r["Start_Timestamp"]) - t0) / 1e3
    e = (int(r["End_Timestamp"]) - t0) / 1e3
    n = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0].replace("soc::", "")
    print(f"{n[:44]:44s} q{r.get('Queue_Id', '?'):>3s} {s:8.1f} {e:8.1f} {e - s:7.1f}")
