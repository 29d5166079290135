import os, sys, time
sys.path.insert(0, '/root/repo/cuvs-rag_amd'); sys.path.insert(0, '/root/repo/oracle')
import numpy as np, torch
from mivs import ops
from mivs.neighbors import ivf_flat
import oracle as O
n = int(sys.argv[1])
x = ops.synth_mixture(n, 768, 0, n_centers=65536, sigma=0.75)
q = ops.synth_mixture(64, 768, 0, n_centers=65536, sigma=0.75, row_begin=1 << 40)
idx = ivf_flat.build(ivf_flat.IndexParams(n_lists=1024), x)
d_g, i_g = ivf_flat.search(ivf_flat.SearchParams(n_probes=32), idx, q, 10)
rows = idx.list_rows()
ids = idx.list_ids()
sel = torch.randint(0, n, (4096,), device='cuda')
ok = torch.equal(rows[sel], x[ids[sel]])
print('list_rows == x[ids] on sample:', ok, flush=True)
rows_h = rows.cpu().numpy(); ids_h = ids.cpu().numpy()
sizes = idx.list_sizes.numpy(); off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
print('sizes sum', sizes.sum(), 'ids perm ok', np.array_equal(np.sort(ids_h[:100000]), np.sort(ids_h[:100000])), flush=True)
cents = idx.centers.cpu().numpy()
O.fast_set_threads(16)
_, i_c = O.fast_ivf_search(rows_h, ids_h, off, cents, q.cpu().numpy(), 32, 10)
i_g = i_g.cpu().numpy()
print('cpu vs gpu id agreement', (i_c == i_g).mean(), flush=True)
print(i_c[0], i_g[0])
