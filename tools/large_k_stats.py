"""Distribution of the k-th neighbour key at the benchmark shape (configs[2]) for the large-k design:
for a sample of queries, the exact L2 keys to every probed row (torch fp32 on the GPU; statistics only, not the
pinned order) and, for k in KS: the global k-th key over the probed rows, the k-th over candidate pre-pass samples
and the global rank those reach, and the rows inside the refine window above the k-th key.

Usage (GPU box): python tools/large_k_stats.py [--rows 10000000] [--queries 300]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuvs-rag_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--queries", type=int, default=300)
    ap.add_argument("--n-probes", type=int, default=32)
    ap.add_argument("--window", type=float, default=0.0025)
    a = ap.parse_args()
    import mivs
    from mivs import ops
    from mivs.neighbors import ivf_flat

    mivs.load()
    dev = 0
    x = ops.synth_mixture(a.rows, 768, 0, n_centers=65536, sigma=0.75, row_begin=0, device=dev)
    q = ops.synth_mixture(a.queries, 768, 0, n_centers=65536, sigma=0.75, row_begin=1 << 40, device=dev)
    t0 = time.time()
    idx = ivf_flat.build(ivf_flat.IndexParams(n_lists=1024), x)
    print(f"build {time.time() - t0:.2f} s", file=sys.stderr)
    del x
    torch.cuda.empty_cache()
    probes = torch.empty((a.queries, a.n_probes), dtype=torch.int32, device="cuda")
    ivf_flat.search(ivf_flat.SearchParams(n_probes=a.n_probes), idx, q, 10, probes_out=probes)
    rows = idx.list_rows()  # [n, d] in list order
    sizes = idx.list_sizes.numpy()
    off = np.concatenate([[0], np.cumsum(sizes)])
    pr = probes.cpu().numpy()
    KS = [10, 100, 1000, 2000, 4000]
    out = {k: {"kth": [], "near1": [], "near1_rank": [], "q4x4": [], "q4x4_rank": [], "half2": [], "half2_rank": [],
               "win": [], "q2x4_rank": []} for k in KS}
    qn = (q * q).sum(1)
    for i in range(a.queries):
        segs = [(off[l], off[l + 1]) for l in pr[i]]
        keys = []
        for s, e in segs:
            r = rows[s:e]
            keys.append((qn[i] + (r * r).sum(1) - 2.0 * (r @ q[i])).clamp_min(0))
        allk = torch.cat(keys).sort().values
        n1 = keys[0].sort().values
        q4 = torch.cat([kk[: (kk.shape[0] + 3) // 4] for kk in keys[:4]]).sort().values
        h2 = torch.cat([kk[: (kk.shape[0] + 1) // 2] for kk in keys[:2]]).sort().values
        q24 = torch.cat([kk[: (kk.shape[0] + 1) // 2] for kk in keys[:4]]).sort().values
        for k in KS:
            kth = allk[k - 1]
            o = out[k]
            o["kth"].append(float(kth))
            o["win"].append(int((allk <= kth + a.window).sum()))
            for name, smp in (("near1", n1), ("q4x4", q4), ("half2", h2), ("q2x4", q24)):
                if smp.shape[0] >= k:
                    v = smp[k - 1]
                    if name + "_rank" in o:
                        o[name + "_rank"].append(int((allk <= v).sum()))
                    if name in o:
                        o[name].append(float(v))
    res = {}
    for k in KS:
        o = out[k]
        r = {"kth_p50": float(np.median(o["kth"])), "window_rows_p50": float(np.median(o["win"])),
             "window_rows_p99": float(np.percentile(o["win"], 99))}
        for name in ("near1", "q4x4", "half2", "q2x4"):
            rk = o[name + "_rank"]
            if rk:
                r[name + "_rank_over_k"] = {"n": len(rk), "p50": float(np.median(rk)) / k,
                                            "p90": float(np.percentile(rk, 90)) / k, "max": float(max(rk)) / k}
        res[k] = r
        print(k, json.dumps(r), flush=True)
    print(json.dumps({"rows": a.rows, "queries": a.queries, "n_probes": a.n_probes, "stats": res}))


if __name__ == "__main__":
    main()
