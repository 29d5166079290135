#!/usr/bin/env python3
"""Summary of the K13 issue/wait/clock passes (tools/pmc_k13_clock.sh): per-launch means of every counter,
the effective clock (GRBM_GUI_ACTIVE / 8 XCDs / launch time, MI355X_MICROARCH.md 'DVFS give-back'), the
MFMA pipe's busy fraction (SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * SIMDs)) and the wave-cycle
split (WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY = WAVE_CYCLES, all in quad-cycles).

Usage: pmc_clock_summary.py PASS_DIR OUT_JSON [kernel-substring] [config_key]
With a config_key (bench.py's cfg_key of the profiled run) the summary also carries it and clock_mhz_held at the top
level: bench.py's roofline reads them (load_clock) for clock_mhz_held / frac_at_held_clock.
"""
import csv
import json
import os
import statistics
import sys
from collections import defaultdict

SIMDS = 1024  # 256 CUs x 4


def load(path, kernel):
    per = defaultdict(dict)  # dispatch -> counter -> value
    dur = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            if kernel not in r["Kernel_Name"]:
                continue
            d = int(r["Dispatch_Id"])
            per[d][r["Counter_Name"]] = per[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            dur[d] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    return per, dur


def main():
    d, out = sys.argv[1], sys.argv[2]
    kernel = sys.argv[3] if len(sys.argv) > 3 else "k_rs_scan"
    res = {"kernel": kernel, "passes": {}}
    if len(sys.argv) > 4:
        res["config_key"] = sys.argv[4]
    for name in sorted(os.listdir(d)):
        p = os.path.join(d, name, "pmc_counter_collection.csv")
        if not os.path.exists(p):
            continue
        per, dur = load(p, kernel)
        if not per:
            continue
        names = sorted({c for v in per.values() for c in v})
        mean = {c: statistics.mean(v[c] for v in per.values() if c in v) for c in names}
        ms = statistics.mean(dur.values()) * 1e3
        pas = {"n_dispatches": len(per), "launch_ms_under_pmc": ms, "counters": mean}
        if "GRBM_GUI_ACTIVE" in mean:
            cyc = mean["GRBM_GUI_ACTIVE"] / 8.0
            pas["effective_clock_ghz"] = cyc / (ms * 1e-3) / 1e9
            if "SQ_VALU_MFMA_BUSY_CYCLES" in mean:
                pas["mfma_pipe_busy_frac"] = mean["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc * SIMDS)
            if "SQ_INSTS_MFMA" in mean:
                # 16x16x32 f16: 16 cycles per MFMA on its SIMD
                pas["mfma_issue_frac_16cyc"] = mean["SQ_INSTS_MFMA"] * 16 / (cyc * SIMDS)
        wc = mean.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_VALU",
                      "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_SCA", "SQ_BUSY_CYCLES"):
                if c in mean:
                    pas[c + "_over_wave_cycles"] = mean[c] / wc
        if mean.get("SQ_INSTS_MFMA"):
            for c in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_SMEM"):
                if c in mean:
                    pas[c + "_per_mfma"] = mean[c] / mean["SQ_INSTS_MFMA"]
        res["passes"][name] = pas
        if "effective_clock_ghz" in pas and "clock_mhz_held" not in res:
            res["clock_mhz_held"] = pas["effective_clock_ghz"] * 1e3
            res["clock_source"] = f"pass {name}: GRBM_GUI_ACTIVE / 8 XCDs / mean launch time under PMC"
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
