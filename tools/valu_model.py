"""VALU issue model of the clouds kernels: per kernel, the cycles its VALU stream needs at the
measured gfx950 issue costs (tools/microbench/valu_mix.hip: 4 cycles per wave64 VALU instruction per SIMD,
~9.5 for a transcendental, i.e. +5.5 over a plain op) against its measured duration.

usage: python tools/valu_model.py gpurun_out/sqmix_c4 [more dirs] > profiles/<tag>_valu_model.json
(each dir: a `tools/gpu.sh pmc` output with SQ_INSTS_VALU and SQ_INSTS_VALU_TRANS_F32 and its kernel trace)
"""
import collections
import csv
import glob
import json
import os
import sys

SIMDS, CLOCK_GHZ, VALU_CYC, TRANS_EXTRA = 1024, 2.4, 4.0, 5.5


def load(d):
    counters = collections.defaultdict(lambda: collections.defaultdict(list))
    durs = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            counters[row["Kernel_Name"]][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            durs[row["Kernel_Name"]].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3)
    return counters, durs


def main():
    out = {"model": {"valu_cycles_per_wave_instr": VALU_CYC, "trans_extra_cycles": TRANS_EXTRA, "simds": SIMDS,
                     "clock_ghz": CLOCK_GHZ, "source": "tools/microbench/valu_mix.hip (8 waves/SIMD, full chip)"},
           "runs": {}}
    for d in sys.argv[1:]:
        counters, durs = load(d)
        rows = {}
        for k, c in counters.items():
            if "clouds" not in k and "ssao_kernel" not in k and "composition_pair" not in k and "sky_compose" not in k:
                continue
            mean = {n: sum(v) / len(v) for n, v in c.items()}
            if "SQ_INSTS_VALU" not in mean or not durs.get(k):
                continue
            us = sorted(durs[k])[len(durs[k]) // 2]
            trans = mean.get("SQ_INSTS_VALU_TRANS_F32", 0.0)
            need_us = (VALU_CYC * mean["SQ_INSTS_VALU"] + TRANS_EXTRA * trans) / SIMDS / (CLOCK_GHZ * 1e3)
            short = k.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0].replace("soc::", "")
            rows[short] = {"us": round(us, 1), "valu_wave_instr": int(mean["SQ_INSTS_VALU"]), "trans": int(trans),
                           "issue_bound_us": round(need_us, 1), "valu_issue_fraction": round(need_us / us, 3),
                           "mix": {n[14:]: int(v) for n, v in mean.items() if n.startswith("SQ_INSTS_VALU_")}}
        out["runs"][os.path.basename(d.rstrip("/"))] = rows
    json.dump(out, sys.stdout, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
