"""Summarise `tools/gpu.sh pmc|traffic` output: per-kernel mean counter values per dispatch -> JSON.

With --traffic OUT.json also writes the per-launch HBM traffic table bench.py reads for the
roofline's `traffic` field: hbm_bytes = 2 * FETCH_SIZE + WRITE_SIZE (both reported in KiB). The factor
2 is MI355X_MICROARCH.md's gfx950 correction (FETCH_SIZE counts half the bytes of 16-B-per-lane
streaming reads); WRITE_SIZE is exact for 16-B stores.
"""
import collections
import csv
import glob
import json
import os
import sys

args = [a for a in sys.argv[1:] if not a.startswith("--")]
root = args[0] if args else "gpurun_out/pmc"
out = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(root, "*", "**", "*counter_collection.csv"), recursive=True):
    with open(f) as fh:
        for row in csv.DictReader(fh):
            name = row.get("Kernel_Name", "")
            short = name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
            out[short][row["Counter_Name"]].append(float(row["Counter_Value"]))
res = {}
for k, d in out.items():
    res[k] = {c: sum(v) / len(v) for c, v in d.items()}
    res[k]["dispatch_samples"] = max(len(v) for v in d.values())
if "--traffic" in sys.argv:
    dst = sys.argv[sys.argv.index("--traffic") + 1]
    kernels = {}
    for k, v in res.items():
        if "FETCH_SIZE" in v and "WRITE_SIZE" in v and k.startswith("soc::"):
            kernels[k[5:]] = {"fetch_kib": round(v["FETCH_SIZE"], 1), "write_kib": round(v["WRITE_SIZE"], 1),
                              "hbm_bytes": int(round((2.0 * v["FETCH_SIZE"] + v["WRITE_SIZE"]) * 1024)),
                              "dispatches": v["dispatch_samples"]}
    meta = {"source": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE (separate passes, --kernel-trace only) "
                      "over `bench.py --steps 3 --warmup 1 --profile-frames 1`; per-dispatch means",
            "formula": "hbm_bytes = 2*FETCH_SIZE + WRITE_SIZE (KiB -> bytes; gfx950 FETCH_SIZE halving correction)",
            "resolution": [3840, 2160], "kernels": kernels,
            "scene": (sys.argv[sys.argv.index("--scene") + 1] if "--scene" in sys.argv else "mesh")}
    with open(dst, "w") as fh:
        json.dump(meta, fh, indent=1, sort_keys=True)
json.dump(res, sys.stdout, indent=1, sort_keys=True)
