"""VALU issue model of the clouds kernels: per kernel, the cycles its VALU stream needs at the
measured gfx950 issue costs (tools/microbench/valu_mix.hip: 4 cycles per wave64 VALU instruction per SIMD,
~9.5 for a transcendental, i.e. +5.5 over a plain op) against its measured duration.

usage: python tools/valu_model.py [--durations KT_DIR] [--calibration VMIX_DIR] PMC_DIR [more dirs] > profiles/<tag>_valu_model.json
(each PMC_DIR: a `tools/gpu.sh pmc` output with SQ_INSTS_VALU and SQ_INSTS_VALU_TRANS_F32; KT_DIR: a counter-free
`tools/gpu.sh kt` trace of the same build and command, whose median durations replace the counter runs' own;
VMIX_DIR: the same counters over tools/microbench/valu_mix, whose instruction counts are known, to check the counter)
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


def opt(name):
    if name in sys.argv:
        i = sys.argv.index(name)
        v = sys.argv[i + 1]
        del sys.argv[i:i + 2]
        return v
    return None


def main():
    kt_dir, vmix_dir = opt("--durations"), opt("--calibration")
    kt_durs = load(kt_dir)[1] if kt_dir else None
    out = {"model": {"valu_cycles_per_wave_instr": VALU_CYC, "trans_extra_cycles": TRANS_EXTRA, "simds": SIMDS,
                     "clock_ghz": CLOCK_GHZ, "source": "tools/microbench/valu_mix.hip (8 waves/SIMD, full chip)",
                     "caveat": "a packed f32 op (v_pk_*_f32) counts as one instruction (~1.1x the issue time of v_fma_f32, "
                               "tools/microbench/pk_rate.hip); integer / convert ops interleaved with f32 FMAs co-issue, so "
                               "the 4-cycle cost is an average, not a hard bound (DESIGN.md 5.2)"},
           "runs": {}}
    if vmix_dir:   # valu_mix: 2048 blocks x 4 waves x 2048 iterations x 8 chains x per-iteration VALU ops per dispatch
        counters, _ = load(vmix_dir)
        per_iter = {"FMA": 1, "EXP": 1, "SQRT": 1, "RCP": 1, "CVT_I32": 1, "CVT_F32": 1, "FLOOR": 1, "DOT2": 1, "PERM": 2,
                    "MIX_EXP_2FMA": 3, "MIX_SQRT_4FMA": 5}
        cal = {}
        for k, c in counters.items():
            kind = next((n for n in sorted(per_iter, key=len, reverse=True) if f"(Kind){n}" in k or f"<{n}>" in k or f"Kind){list(per_iter).index(n)}" in k), None)
            mean = {n: sum(v) / len(v) for n, v in c.items()}
            expected = 2048 * 4 * 2048 * 8 * per_iter[kind] if kind else None
            cal[k[:80]] = {"SQ_INSTS_VALU": int(mean.get("SQ_INSTS_VALU", 0)), "expected_wave_instr": expected,
                           "ratio": round(mean.get("SQ_INSTS_VALU", 0) / expected, 4) if expected else None,
                           "SQ_INSTS_VALU_TRANS_F32": int(mean.get("SQ_INSTS_VALU_TRANS_F32", 0))}
        out["counter_calibration"] = cal
    for d in sys.argv[1:]:
        counters, durs = load(d)
        if kt_durs is not None:
            durs = kt_durs
        rows = {}
        for k, c in counters.items():
            if not any(t in k for t in ("clouds", "ssao", "composition_pair", "sky_compose", "taa_pair", "taa_lds", "bloomw", "tonemap")):
                continue
            mean = {n: sum(v) / len(v) for n, v in c.items()}
            if "SQ_INSTS_VALU" not in mean or not durs.get(k):
                continue
            extra = {n: int(v) for n, v in mean.items() if n in ("SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_WAVES",
                                                                  "SQ_INSTS_VMEM_WR", "SQ_INSTS_SMEM")}
            us = sorted(durs[k])[len(durs[k]) // 2]
            trans = mean.get("SQ_INSTS_VALU_TRANS_F32", 0.0)
            need_us = (VALU_CYC * mean["SQ_INSTS_VALU"] + TRANS_EXTRA * trans) / SIMDS / (CLOCK_GHZ * 1e3)
            short = k.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0].replace("soc::", "")
            rows[short] = {"us": round(us, 1), "valu_wave_instr": int(mean["SQ_INSTS_VALU"]), "trans": int(trans),
                           "issue_bound_us": round(need_us, 1), "valu_issue_fraction": round(need_us / us, 3),
                           "mix": {n[14:]: int(v) for n, v in mean.items() if n.startswith("SQ_INSTS_VALU_")}, **extra}
        out["runs"][os.path.basename(d.rstrip("/"))] = rows
    json.dump(out, sys.stdout, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
