"""debug: K9r (MFMA LUT) vs K9s (VALU LUT) vs the oracle on one PQ parity case"""
import os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "cuvs-rag_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle as O
from mivs.neighbors import ivf_pq
from test_gpu_parity import _data

n, d, n_lists, pq_dim, iters, nq, n_probes, k = 12000, 768, 32, 96, 2, 20, 6, 10
x = _data(n, d, seed=n + pq_dim, normalize=True)
q = _data(nq, d, seed=n + pq_dim + 1, normalize=True)
idx = ivf_pq.build(ivf_pq.IndexParams(n_lists=n_lists, pq_dim=pq_dim, kmeans_n_iters=iters, max_train_points_per_pq_code=32),
                   torch.from_numpy(x).cuda(), ids_offset=3)
oc, ocb, osz, oids, ocodes = O.ivfpq_build(x, n_lists, pq_dim, iters=iters, max_per_code=32, id_offset=3)
od, oi, op = O.ivfpq_search(oc, ocb, osz, oids, ocodes, q, n_probes, k)
res = {}
for name, env in [("k9r", {}), ("k9s", {"MIVS_PQ_RT": "0"})]:
    for kk in ("MIVS_PQ_RT",):
        os.environ.pop(kk, None)
    os.environ.update(env)
    dd, ii = ivf_pq.search(ivf_pq.SearchParams(n_probes=n_probes), idx, torch.from_numpy(q).cuda(), k)
    res[name] = (dd.cpu().numpy(), ii.cpu().numpy())
for name, (dd, ii) in res.items():
    print(name, "ids equal oracle:", (ii == oi).mean(), "dist max |diff|:", np.abs(dd - od).max(),
          "bit-equal:", (dd.view(np.int32) == od.view(np.int32)).mean())
print("row 0 oracle", od[0][:8])
print("row 0 k9r   ", res["k9r"][0][0][:8])
print("row 0 k9s   ", res["k9s"][0][0][:8])
