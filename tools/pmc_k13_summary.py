#!/usr/bin/env python3
"""K13 PMC summary from the passes of tools/pmc_k13_passes.sh: HBM bytes per launch (FETCH_SIZE x2 +
WRITE_SIZE, as tools/pmc_summary.py), the DRAM-side read requests and the SQ counters, per launch.

Usage: pmc_k13_summary.py PASS_DIR CONFIG_KEY COMPULSORY_BYTES OUT_JSON
"""
import json
import os
import statistics
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import rows  # noqa: E402

KERNEL = "k_rs_scan"


def per_counter(path):
    acc = defaultdict(lambda: defaultdict(float))
    for disp, name, v, _ in rows(path, KERNEL):
        acc[name][disp] += v
    return {n: statistics.mean(d.values()) for n, d in acc.items()}


def main():
    d, cfg_key, compulsory, out_path = sys.argv[1], sys.argv[2], float(sys.argv[3]), sys.argv[4]
    csv = lambda p: os.path.join(d, p, "pmc_counter_collection.csv")  # noqa: E731
    fr, wr = rows(csv("fetch"), KERNEL), rows(csv("write"), KERNEL)
    fetch_kib = statistics.mean(v for _, _, v, _ in fr)
    write_kib = statistics.mean(v for _, _, v, _ in wr)
    fetch_b, write_b = fetch_kib * 1024 * 2, write_kib * 1024
    ms = statistics.mean([t for *_, t in fr] + [t for *_, t in wr])
    dram = per_counter(csv("dram"))
    sq = per_counter(csv("sq"))
    rd_dram = next((v for k, v in dram.items() if "DRAM" in k), None)
    res = {
        "config_key": cfg_key,
        "kernel": KERNEL,
        "n_dispatches": {"fetch": len(fr), "write": len(wr)},
        "fetch_size_kib_raw_mean": fetch_kib,
        "write_size_kib_mean": write_kib,
        "fetch_bytes_per_launch": fetch_b,
        "write_bytes_per_launch": write_b,
        "hbm_bytes_per_launch": fetch_b + write_b,
        "launch_ms_under_pmc": ms,
        "hbm_gbs_under_pmc": (fetch_b + write_b) / (ms * 1e-3) / 1e9,
        "correction": "FETCH_SIZE x2 (gfx950, 16 B/lane streaming reads), KiB -> bytes; WRITE_SIZE exact",
        "dram": dram,
        "dram_read_bytes_per_launch": rd_dram * 128 if rd_dram is not None else None,
        "dram_note": "TCC_EA0_RDREQ_DRAM = L2 read requests served by DRAM (not the MALL), x128 B per request "
                     "(the same x2 correction as FETCH_SIZE = RDREQ x 64 B)",
        "compulsory_bytes_per_launch": compulsory,
        "traffic_over_compulsory": (fetch_b + write_b) / compulsory,
        "sq": sq,
        "sources": [csv(p) for p in ("fetch", "write", "dram", "sq")],
    }
    with open(out_path, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: res[k] for k in ("hbm_bytes_per_launch", "traffic_over_compulsory", "launch_ms_under_pmc",
                                          "dram_read_bytes_per_launch")}))


if __name__ == "__main__":
    main()
