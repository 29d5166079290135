"""Small-batch latency at configs[2] through the pre-filter path (K13) and through the exact fp32 scan (K3w),
same index, same queries: which route a small batch should take (tools/, not the bench)."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "cuvs-rag_amd"))
from mivs import ops  # noqa: E402
from mivs.neighbors import ivf_flat  # noqa: E402


def lat(idx, q, nq, np_, calls=200):
    sp = ivf_flat.SearchParams(n_probes=np_)
    for i in range(5):
        ivf_flat.search(sp, idx, q[i * nq:(i + 1) * nq], 10)
    torch.cuda.synchronize()
    w = []
    for c in range(calls):
        o = (c * nq) % (q.shape[0] - nq)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ivf_flat.search(sp, idx, q[o:o + nq], 10)
        torch.cuda.synchronize()
        w.append(time.perf_counter() - t0)
    w = np.array(w) * 1e3
    return float(np.percentile(w, 50)), float(np.percentile(w, 99))


def main():
    x = ops.synth_mixture(10_000_000, 768, 0, n_centers=65536, sigma=0.75, row_begin=0, device=0)
    q = ops.synth_mixture(10_000, 768, 0, n_centers=65536, sigma=0.75, row_begin=1 << 40, device=0)
    idx = ivf_flat.build(ivf_flat.IndexParams(n_lists=1024, kmeans_n_iters=20, kmeans_trainset_fraction=0.5), x)
    torch.cuda.synchronize()
    for mode in ("prefilter", "exact"):
        if mode == "exact":
            idx.set_prefilter(False)
        for np_ in (32, 20):
            for nq in (1, 2, 4, 8, 16, 32, 100):
                p50, p99 = lat(idx, q, nq, np_)
                print(f"{mode:9s} n_probes={np_} Q={nq:3d}: p50 {p50:.3f} ms p99 {p99:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
