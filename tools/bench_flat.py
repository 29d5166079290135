#!/usr/bin/env python3
"""Exact (brute-force) k-NN benchmark on one MI355X: BASELINE configs[1] (flat L2, 1M x 768 fp32,
10,000 queries, k = 10), synthetic on-device data (the bench.py mixture).

Times brute_force.search with the fp16 pre-filter (K10 over the one list + K11 exact refine) and with
the fp32 scan (K3), checks that both return the same ids and distances, and reports the pre-filter
scan's MFMA roofline (2 d N Q flops per batch against the 2.5 PF fp16 peak). One JSON line on stdout.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuvs-rag_amd"))

import torch  # noqa: E402

from mivs import _native, ops  # noqa: E402
from mivs.neighbors import brute_force  # noqa: E402


def timed(idx, q, k, reps):
    brute_force.search(idx, q, k)
    _native.set_profiling(True)
    idx.profile_collect()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        d, i = brute_force.search(idx, q, k)
    torch.cuda.synchronize()
    ts = (time.perf_counter() - t0) / reps
    pr = idx.profile_collect()
    _native.set_profiling(False)
    return ts, pr, d, i


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--queries", type=int, default=10_000)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--centers", type=int, default=65536)
    ap.add_argument("--sigma", type=float, default=0.75)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    n, d, Q, k = a.rows, a.dim, a.queries, a.k
    x = ops.synth_mixture(n, d, 0, n_centers=a.centers, sigma=a.sigma)
    q = ops.synth_mixture(Q, d, 0, n_centers=a.centers, sigma=a.sigma, row_begin=1 << 40)
    idx = brute_force.build(x)
    flops = 2.0 * d * n * Q
    ts_pf, pr_pf, d1, i1 = timed(idx, q, k, a.reps)
    st = idx.last_search_stats()
    idx.set_prefilter(False)
    ts_32, pr_32, d0, i0 = timed(idx, q, k, a.reps)
    same = bool(torch.equal(i1, i0) and torch.equal(d1.view(torch.int32), d0.view(torch.int32)))
    scan_ms = pr_pf["scan_ms"] / max(pr_pf["n_calls"], 1)
    out = {"metric": "exact k-NN QPS (flat L2, BASELINE configs[1])", "rows": n, "dim": d, "queries": Q, "k": k,
           "qps_prefilter": Q / ts_pf, "ms_per_batch_prefilter": ts_pf * 1e3,
           "qps_fp32_scan": Q / ts_32, "ms_per_batch_fp32_scan": ts_32 * 1e3,
           "identical_results": same, "overflow_queries": st.get("overflow_queries"),
           "roofline": {"bound": "mfma", "kernel": "k_pf_scan (K10, one list)", "launch_ms": scan_ms,
                        "achieved": flops / (scan_ms * 1e-3) / 1e12 if scan_ms > 0 else None, "peak": 2500.0,
                        "unit": "TFLOP/s",
                        "frac": flops / (scan_ms * 1e-3) / 1e12 / 2500.0 if scan_ms > 0 else None},
           "data": "synthetic: on-device Gaussian mixture (bench.py), fp32"}
    print(f"[flat] pre-filter {Q / ts_pf:,.0f} QPS ({ts_pf * 1e3:.2f} ms/batch, K10 {scan_ms:.2f} ms); "
          f"fp32 scan {Q / ts_32:,.0f} QPS ({ts_32 * 1e3:.2f} ms); identical={same}", file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
