"""Summarise tools/pmc.sh output: per-kernel mean counter values per dispatch -> JSON."""
import collections
import csv
import glob
import json
import os
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
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
json.dump(res, sys.stdout, indent=1, sort_keys=True)
