#!/usr/bin/env python3
"""Scan-kernel (K3) microbenchmark: is the fine scan bound by HBM or by the fp32 MFMA pipe?

Runs brute force (the single-list form of K3, k=10 -> KCAP 16) over corpora of different sizes
with the same total work (rows x queries): a corpus that stays in L2 / the Infinity Cache vs one
that streams from HBM. Equal TF/s in all cases => MFMA/issue-bound; higher TF/s when resident
=> memory-bound. Prints one line per case.
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuvs-rag_amd"))

import torch  # noqa: E402

from mivs import _native, ops  # noqa: E402
from mivs.neighbors import brute_force  # noqa: E402


def run(n, nq, d=768, reps=3):
    x = ops.synth_mixture(n, d, 0, n_centers=4096, sigma=0.5)
    q = ops.synth_mixture(nq, d, 0, n_centers=4096, sigma=0.5, row_begin=1 << 40)
    idx = brute_force.build(x)
    brute_force.search(idx, q, 10)
    _native.set_profiling(True)
    idx.profile_collect()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        brute_force.search(idx, q, 10)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / reps
    pr = idx.profile_collect()
    _native.set_profiling(False)
    ms = pr["scan_ms"] / max(pr["n_calls"], 1)
    flops = 2.0 * n * nq * d
    tiles = (nq + 31) // 32
    streamed = tiles * n * d * 4
    print(f"n={n:>9} nq={nq:>7} corpus={n * d * 4 / 2**20:8.1f} MiB  scan {ms:8.3f} ms (wall {wall * 1e3:8.3f})  "
          f"{flops / ms / 1e9:7.1f} TF/s  streamed {streamed / ms / 1e6:7.1f} GB/s", flush=True)
    idx.close()
    del x, q
    torch.cuda.empty_cache()


if __name__ == "__main__":
    total = 2 ** 33  # rows x queries per case
    for wide, waves in (("0", "8"), ("1", "8"), ("1", "4")):
        os.environ["MIVS_SCAN_WIDE"] = wide
        os.environ["MIVS_SCAN_WIDE_WAVES"] = waves
        kind = f"K3w 64-query tiles, {waves}-wave workgroups" if wide == "1" else "K3 32-query tiles"
        print(f"--- MIVS_SCAN_WIDE={wide} MIVS_SCAN_WIDE_WAVES={waves} ({kind})", flush=True)
        for n in [1024, 1 << 20, 4 << 20]:
            run(n, max(32, total // n))
