#!/usr/bin/env python3
"""Pick the synthetic corpus difficulty: recall@10 (and QPS) vs n_probes for mixture sigmas / centre counts.

The reference benchmarks only isotropic torch.randn data (improved_multi_gpu_rag.py:431-434),
on which IVF recall at n_probes=32/n_lists=1024 is far below 0.95 (SURVEY.md §7 'Hard parts');
bench.py uses a clustered mixture whose parameters are chosen here so that recall@10 at the
configured n_probes=32 sits near the 0.95 target instead of saturating at 1.0.
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "cuvs-rag_amd"))
import numpy as np
import torch

from mivs import ops
from mivs.neighbors import brute_force, ivf_flat

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=10_000_000)
ap.add_argument("--configs", default="4096:0.35,4096:1.0,4096:1.25,4096:1.5,16384:1.5")
ap.add_argument("--probes", default="8,16,32,64")
ap.add_argument("--queries", type=int, default=10_000)
a = ap.parse_args()
k, d = 10, 768
for cfg in a.configs.split(","):
    centers, sigma = int(cfg.split(":")[0]), float(cfg.split(":")[1])
    x = ops.synth_mixture(a.rows, d, 0, n_centers=centers, sigma=sigma)
    q = ops.synth_mixture(a.queries, d, 0, n_centers=centers, sigma=sigma, row_begin=1 << 40)
    t0 = time.time()
    idx = ivf_flat.build(ivf_flat.IndexParams(n_lists=1024), x)
    torch.cuda.synchronize()
    tb = time.time() - t0
    bf = brute_force.build(x)
    _, gt = brute_force.search(bf, q[:1000], k)
    bf.close()
    gt = gt.cpu().numpy()
    sizes = idx.list_sizes.numpy()
    out = []
    for p in [int(v) for v in a.probes.split(",")]:
        sp = ivf_flat.SearchParams(n_probes=p)
        ivf_flat.search(sp, idx, q, k)
        torch.cuda.synchronize()
        t0 = time.time()
        _, ii = ivf_flat.search(sp, idx, q, k)
        torch.cuda.synchronize()
        dt = time.time() - t0
        ii = ii[:1000].cpu().numpy()
        rec = np.mean([len(set(a_) & set(b_)) / k for a_, b_ in zip(ii, gt)])
        out.append(f"p{p}: r={rec:.3f} {a.queries / dt / 1e3:.0f}kQPS")
    print(f"centers={centers} sigma={sigma} build={tb:.2f}s lists min/med/max={sizes.min()}/{int(np.median(sizes))}/"
          f"{sizes.max()} | " + " | ".join(out), flush=True)
    idx.close()
    del x, q
    torch.cuda.empty_cache()
