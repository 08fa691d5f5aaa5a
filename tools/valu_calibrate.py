#!/usr/bin/env python
"""VALU issue calibration: what one wave64 VALU instruction costs a SIMD on gfx950, measured, and the
VALU load of the frame's kernels against it.

  python tools/valu_calibrate.py RATE_TXT RATE_PMC_DIR KERNEL_PMC_DIR > profiles/<tag>_valu_model.json

RATE_TXT: tools/microbench/valu_rate output (cycles per wave-instruction per SIMD in shader cycles, per variant and
waves per SIMD: the launch figure = event time x in-kernel clock over the instructions each SIMD issues).
RATE_PMC_DIR: rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU ... over the same microbenchmark: relates the counter
SQ_ACTIVE_INST_VALU (quad-cycles in which a wave issues VALU) to the measured issue cost.
KERNEL_PMC_DIR: a `tools/gpu.sh pmc` pass with SQ_INSTS_VALU, SQ_ACTIVE_INST_VALU, SQ_WAVE_CYCLES, SQ_BUSY_CYCLES,
SQ_WAIT_ANY, SQ_WAIT_INST_ANY, SQ_ACTIVE_INST_ANY, GRBM_GUI_ACTIVE over the bench (serial lanes).

Per kernel: valu_issue_us = SQ_INSTS_VALU x the calibrated cycles per instruction / 1024 SIMDs / the clock, beside the
launch's duration; valu_busy = SQ_ACTIVE_INST_VALU x 4 / (1024 x GRBM_GUI_ACTIVE / 8) (the fraction of SIMD cycles
with a VALU issue, if the counter's quad-cycles are SIMD-exclusive: checked on the microbenchmark, whose issue rate is
known); the stall split of the wave cycles (parked on s_waitcnt / issue-stalled / issuing).
"""
import collections
import csv
import glob
import json
import os
import re
import sys

SIMDS, XCDS = 1024, 8


def parse_rate(path):
    rows = {}
    pat = re.compile(r"^(.*?)\s+waves/SIMD=(\d)\s+cycles/wave-instr/SIMD: launch ([\d.]+), median block ([\d.]+)\s+"
                     r"\(([\d.]+) ms, clock ([\d.]+) GHz\)")
    for ln in open(path):
        m = pat.match(ln.strip())
        if m:
            rows.setdefault(m.group(1).strip(), {})[int(m.group(2))] = {
                "launch_cycles": float(m.group(3)), "median_block_cycles": float(m.group(4)),
                "ms": float(m.group(5)), "clock_ghz": float(m.group(6))}
    return rows


def load_pmc(d):
    counters = collections.defaultdict(lambda: collections.defaultdict(list))
    durs = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            counters[row["Kernel_Name"]][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            durs[row["Kernel_Name"]].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e3)
    return counters, durs


def short(k):
    return k.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0].replace("soc::", "")


def main():
    rate_txt, rate_pmc, kern_pmc = sys.argv[1:4]
    rates = parse_rate(rate_txt)
    out = {"microbenchmark": {"source": "tools/microbench/valu_rate.hip (16 independent chains per lane, VGPR operands, "
                                        "inline asm; cycles = event time x in-kernel clock)", "cycles": rates}}
    # calibration: the launch cost of the plain f32 stream at 8 waves / SIMD (the kernels' occupancy), and of the mixed ones
    fma8 = rates.get("v_fma_f32 x16", {}).get(8, {}).get("launch_cycles")
    mix8 = rates.get("8 fma + 8 add_u32", {}).get(8, {}).get("launch_cycles")
    pk8 = rates.get("v_pk_fma_f32 x8", {}).get(8, {}).get("launch_cycles")
    ex8 = rates.get("v_exp_f32 x16", {}).get(8, {}).get("launch_cycles")
    out["calibration"] = {"v_fma_f32_cycles_8w": fma8, "fma_add_mix_cycles_8w": mix8, "v_pk_fma_f32_cycles_8w": pk8,
                          "v_exp_f32_cycles_8w": ex8}
    # counter check on the microbenchmark: SQ_ACTIVE_INST_VALU quad-cycles per VALU wave-instruction
    c, _ = load_pmc(rate_pmc)
    chk = {}
    for k, v in c.items():
        m = {n: sum(x) / len(x) for n, x in v.items()}
        if m.get("SQ_INSTS_VALU"):
            chk[short(k)[:60]] = {"SQ_INSTS_VALU": int(m["SQ_INSTS_VALU"]),
                                  "active_valu_cycles_per_instr": round(4.0 * m.get("SQ_ACTIVE_INST_VALU", 0) / m["SQ_INSTS_VALU"], 3),
                                  "busy_cycles": m.get("SQ_BUSY_CYCLES"), "grbm_gui_active": m.get("GRBM_GUI_ACTIVE")}
    out["counter_check"] = chk
    cyc = fma8 or 4.0
    c, durs = load_pmc(kern_pmc)
    rows = {}
    for k, v in c.items():
        m = {n: sum(x) / len(x) for n, x in v.items()}
        if not m.get("SQ_INSTS_VALU") or not durs.get(k):
            continue
        s = short(k)
        if not any(t in s for t in ("clouds", "ssao", "composition", "sky_compose", "taa", "bloomw", "tonemap")):
            continue
        us = sorted(durs[k])[len(durs[k]) // 2]
        gui = m.get("GRBM_GUI_ACTIVE", 0.0) / XCDS          # cycles of the launch (the counter sums the 8 XCDs)
        clock = gui / (us * 1e3) if us else 0.0              # GHz, effective
        wc = m.get("SQ_WAVE_CYCLES", 0.0)
        rows[s] = {"us": round(us, 1), "valu_wave_instr": int(m["SQ_INSTS_VALU"]),
                   "effective_clock_ghz": round(clock, 3),
                   "valu_issue_us": round(m["SQ_INSTS_VALU"] * cyc / SIMDS / ((clock or 2.4) * 1e3), 1),
                   "valu_busy": round(4.0 * m.get("SQ_ACTIVE_INST_VALU", 0.0) / (SIMDS * gui), 3) if gui else None,
                   "wave_cycles_split": ({"parked_waitcnt": round(m.get("SQ_WAIT_ANY", 0) / wc, 3),
                                          "issue_stalled": round(m.get("SQ_WAIT_INST_ANY", 0) / wc, 3),
                                          "issuing": round(m.get("SQ_ACTIVE_INST_ANY", 0) / wc, 3)} if wc else None)}
        rows[s]["valu_issue_fraction"] = round(rows[s]["valu_issue_us"] / us, 3)
    out["model"] = {"valu_cycles_per_wave_instr": cyc, "simds": SIMDS,
                    "source": "the launch cost of independent v_fma_f32 at 8 waves per SIMD (microbenchmark above)",
                    "clock": "each launch's effective clock, GRBM_GUI_ACTIVE / 8 / duration"}
    out["runs"] = {"serial_lanes": rows}
    json.dump(out, sys.stdout, indent=1, sort_keys=True)
    print()


if __name__ == "__main__":
    main()
