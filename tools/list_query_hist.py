"""Per-list query counts m_l of the default bench search (configs[2]: 10M x 768, n_lists 1024, n_probes 32,
10k queries): what an item shape over (list rows x list queries) sees. Prints the m_l distribution and, for
query tiles of W queries, the padded fraction. Measurement scaffolding (tools/), not product code."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cuvs-rag_amd"))
sys.path.insert(0, ROOT)


def main():
    import bench
    import mivs
    from mivs import ops
    from mivs.neighbors import ivf_flat

    mivs.load()
    print("building the 10M index ...", flush=True)
    n, d, Q = 10_000_000, 768, 10_000
    x = ops.synth_mixture(n, d, bench.SEED, n_centers=65536, sigma=0.75, device=0)
    q = ops.synth_mixture(Q, d, bench.SEED, n_centers=65536, sigma=0.75, row_begin=bench.QUERY_ROW_BASE, device=0)
    idx = ivf_flat.build(ivf_flat.IndexParams(n_lists=1024, kmeans_n_iters=20, kmeans_trainset_fraction=0.5), x)
    print("built", flush=True)
    probes = torch.empty((Q, 32), dtype=torch.int32, device=0)
    ivf_flat.search(ivf_flat.SearchParams(n_probes=32), idx, q, 10, probes_out=probes)
    m = np.bincount(probes.cpu().numpy().ravel(), minlength=1024)
    sizes = idx.list_sizes.numpy()
    print("m_l: mean %.1f min %d p10 %d p50 %d p90 %d max %d" % (m.mean(), m.min(), *np.percentile(m, [10, 50, 90]).astype(int), m.max()))
    print("list rows: mean %.0f p10 %d p50 %d p90 %d max %d" % (sizes.mean(), *np.percentile(sizes, [10, 50, 90]).astype(int), sizes.max()))
    work = (sizes.astype(np.float64) * m).sum()
    print("rows x queries: %.4g; row-weighted mean m %.1f" % (work, work / sizes.sum()))
    for W in (32, 160, 256, 320):
        padded = (sizes.astype(np.float64) * (np.ceil(m / W) * W)).sum()
        print("tiles of %3d queries: padded work / work = %.4f; row passes (HBM reads of each row) %.3f"
              % (W, padded / work, (sizes * np.ceil(m / W)).sum() / sizes.sum()))
    for W in (16,):
        padded = (sizes.astype(np.float64) * (np.ceil(m / W) * W)).sum()
        print("16-query blocks: padded work / work = %.4f" % (padded / work))
    hist, edges = np.histogram(m, bins=[0, 32, 64, 128, 192, 256, 320, 384, 512, 768, 1024, 4096])
    print("m_l histogram:", dict(zip([f"{int(a)}-{int(b)}" for a, b in zip(edges[:-1], edges[1:])], hist.tolist())))
    rows_in = [int(sizes[(m >= a) & (m < b)].sum()) for a, b in zip(edges[:-1], edges[1:])]
    print("rows per bin:", rows_in)


if __name__ == "__main__":
    main()
