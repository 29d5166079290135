#!/usr/bin/env python3
"""K12 vs K10 vs exact fp32 scan on small shapes: mismatch counts per shape (GPU debugging aid)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "cuvs-rag_amd"))
from mivs.neighbors import ivf_flat  # noqa: E402

for (n, d, nq, nl, npb, k) in [(8000, 64, 70, 32, 4, 10), (12000, 768, 130, 24, 6, 10), (9000, 384, 300, 20, 8, 16),
                               (20000, 128, 500, 16, 4, 10)]:
    rng = np.random.default_rng(0)
    x = torch.from_numpy(rng.standard_normal((n, d)).astype(np.float32)).cuda()
    q = torch.from_numpy(rng.standard_normal((nq, d)).astype(np.float32)).cuda()
    idx = ivf_flat.build(ivf_flat.IndexParams(n_lists=nl, kmeans_n_iters=3), x)
    res = {}
    for tag, env in (("k12", "1"), ("k10", "0")):
        os.environ["MIVS_PF_REG"] = env
        idx.set_prefilter(True)
        dd, ii = ivf_flat.search(ivf_flat.SearchParams(n_probes=npb), idx, q, k)
        res[tag] = (dd.cpu().numpy(), ii.cpu().numpy(), idx.last_search_stats())
    idx.set_prefilter(False)
    dd, ii = ivf_flat.search(ivf_flat.SearchParams(n_probes=npb), idx, q, k)
    ex = (dd.cpu().numpy(), ii.cpu().numpy())
    for tag in ("k12", "k10"):
        d_, i_, st = res[tag]
        bad = (i_ != ex[1]).any(axis=1)
        print(f"n={n} d={d} nq={nq} k={k} {tag}: rows wrong {bad.sum()}/{nq} ovf {st['overflow_queries']} "
              f"qtile {st['query_tile']} win {st['window_candidates']}", flush=True)
        if bad.any():
            r = int(np.nonzero(bad)[0][0])
            print("   first bad row", r, "got", i_[r][:6], d_[r][:4], "want", ex[1][r][:6], ex[0][r][:4], flush=True)
