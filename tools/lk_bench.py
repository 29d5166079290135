"""Large-k search at configs[2] (10M x 768, n_lists 1024, n_probes 32, 10k queries) for kernel traces: one warm
search, then --reps timed searches of k (default 2000). Usage: python tools/lk_bench.py [--k 2000] [--reps 3]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuvs-rag_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=2000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--queries", type=int, default=10_000)
    a = ap.parse_args()
    import mivs
    from mivs import ops
    from mivs.neighbors import ivf_flat

    mivs.load()
    x = ops.synth_mixture(a.rows, 768, 0, n_centers=65536, sigma=0.75, row_begin=0, device=0)
    q = ops.synth_mixture(a.queries, 768, 0, n_centers=65536, sigma=0.75, row_begin=1 << 40, device=0)
    idx = ivf_flat.build(ivf_flat.IndexParams(n_lists=1024), x)
    sp = ivf_flat.SearchParams(n_probes=32)
    ivf_flat.search(sp, idx, q, a.k)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        ivf_flat.search(sp, idx, q, a.k)
    torch.cuda.synchronize()
    t = (time.perf_counter() - t0) / a.reps
    st = idx.last_search_stats()
    print(f"k={a.k}: {t * 1e3:.2f} ms per {a.queries} queries = {a.queries / t:,.0f} QPS | {st}", flush=True)


if __name__ == "__main__":
    main()
