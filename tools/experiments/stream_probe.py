"""Timeline probe for streaming.search_host vs the serial host loop (run under rocprofv3 --kernel-trace
--memory-copy-trace). Prints host-side wall clock per variant."""
import sys
import time

import torch

sys.path.insert(0, "cuvs-rag_amd")
import mivs  # noqa: E402
from mivs import ops  # noqa: E402
from mivs.neighbors import ivf_flat, streaming  # noqa: E402

n, d, Q, k = int(sys.argv[1]) if len(sys.argv) > 1 else 2_000_000, 768, 10000, 10
mivs.load()
x = ops.synth_mixture(n, d, 0, n_centers=65536, sigma=0.75, row_begin=0, device=0)
q = ops.synth_mixture(Q, d, 0, n_centers=65536, sigma=0.75, row_begin=1 << 40, device=0)
idx = ivf_flat.build(ivf_flat.IndexParams(n_lists=1024), x)
sp = ivf_flat.SearchParams(n_probes=32)
qh = q.cpu().pin_memory()
qm = qh.repeat(6, 1).pin_memory()
for _ in range(2):
    ivf_flat.search(sp, idx, q, k)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(6):
    ivf_flat.search(sp, idx, q, k)
torch.cuda.synchronize()
print(f"device-resident: {(time.perf_counter() - t0) / 6 * 1e3:.2f} ms/batch", flush=True)
t0 = time.perf_counter()
for _ in range(6):
    dd, ii = ivf_flat.search(sp, idx, qh.to("cuda:0", non_blocking=True), k)
    dd.cpu(), ii.cpu()
print(f"serial host: {(time.perf_counter() - t0) / 6 * 1e3:.2f} ms/batch", flush=True)
t0 = time.perf_counter()
od = torch.empty((6 * Q, k), dtype=torch.float32, pin_memory=True)
oi = torch.empty((6 * Q, k), dtype=torch.int64, pin_memory=True)
print(f"pinned output alloc: {(time.perf_counter() - t0) * 1e3:.2f} ms", flush=True)
for rep in range(4):
    t0 = time.perf_counter()
    streaming.search_host(idx, qm, k, sp, batch_size=Q, distances=od, neighbors=oi)
    print(f"streamed (outputs reused): {(time.perf_counter() - t0) / 6 * 1e3:.2f} ms/batch", flush=True)
