"""Host time around one search step (tools/, not part of the product): the Python wrapper, the C call, and the GPU
idle between steps. 1M x 768 IVF-Flat (1024 lists), 10k queries, n_probes 32, k 10."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "cuvs-rag_amd"))
from mivs import _native  # noqa: E402
from mivs.neighbors import ivf_flat  # noqa: E402


def main():
    torch.manual_seed(0)
    n, d, nq = 1_000_000, 768, 10_000
    c = torch.randn(4096, d, device="cuda")
    x = c[torch.randint(0, 4096, (n,), device="cuda")] + 0.75 * torch.randn(n, d, device="cuda")
    x = torch.nn.functional.normalize(x, dim=1)
    q = x[:nq].clone()
    idx = ivf_flat.build(ivf_flat.IndexParams(n_lists=1024, kmeans_n_iters=5), x)
    sp = ivf_flat.SearchParams(n_probes=32)
    for _ in range(3):
        ivf_flat.search(sp, idx, q, 10)
    torch.cuda.synchronize()
    K = 50
    t0 = time.perf_counter()
    for _ in range(K):
        ivf_flat.search(sp, idx, q, 10)
    torch.cuda.synchronize()
    t_api = (time.perf_counter() - t0) / K
    # the C call alone, outputs preallocated, no Python checks
    dist = torch.empty((nq, 10), dtype=torch.float32, device="cuda")
    nb = torch.empty((nq, 10), dtype=torch.int64, device="cuda")
    lib = _native.lib()
    sptr = torch.cuda.current_stream().cuda_stream
    t0 = time.perf_counter()
    tc = 0.0
    for _ in range(K):
        a = time.perf_counter()
        lib.mivs_ivf_flat_search(idx.handle, sptr, q.data_ptr(), nq, 10, 32, dist.data_ptr(), nb.data_ptr(), None)
        tc += time.perf_counter() - a
    torch.cuda.synchronize()
    t_c = (time.perf_counter() - t0) / K
    # GPU time of one step: events around a step, no host sync inside measured separately
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    lib.mivs_ivf_flat_search(idx.handle, sptr, q.data_ptr(), nq, 10, 32, dist.data_ptr(), nb.data_ptr(), None)
    ev[1].record()
    torch.cuda.synchronize()
    print(f"per step: API {t_api * 1e6:.1f} us | bare C loop {t_c * 1e6:.1f} us (inside the call {tc / K * 1e6:.1f} us) "
          f"| one step by events {ev[0].elapsed_time(ev[1]) * 1e3:.1f} us")


if __name__ == "__main__":
    main()
