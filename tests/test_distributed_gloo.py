"""N>1 path on CPU: one process per rank (gloo, world_size 2), corpus sharded with the reference's
'even' split, per-shard top-k with global ids, one all-gather, then the global merge.

The device merge (K7) needs a GPU, so the ranks here pass a host merge_fn; everything else — the
exchange layout, id offsets, and the result being identical on every rank — is the production
code path of mivs.distributed.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _host_merge(d, i, k, metric="sqeuclidean"):
    d, i = d.numpy(), i.numpy()
    nq = d.shape[0]
    d, i = d.reshape(nq, -1), i.reshape(nq, -1)
    od, oi = np.empty((nq, k), np.float32), np.empty((nq, k), np.int64)
    for r in range(nq):
        o = np.lexsort((i[r], d[r]))[:k]
        od[r], oi[r] = d[r, o], i[r, o]
    return torch.from_numpy(od), torch.from_numpy(oi)


def _rank(rank, world, port, out):
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "cuvs-rag_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from gpu_resource_manager import GPUResourceManager
    from mivs.distributed import all_gather_raw, allreduce_max, merge_across_ranks

    rng = np.random.default_rng(0)
    x = rng.standard_normal((1003, 16)).astype(np.float32)
    q = rng.standard_normal((7, 16)).astype(np.float32)
    m = GPUResourceManager.__new__(GPUResourceManager)
    m.available_gpus = list(range(world))
    g, start, end = m.distribute_workload(x.shape[0])[rank]
    shard = x[start:end]
    d = ((q[:, None, :] - shard[None]) ** 2).sum(-1)
    loc = np.argsort(d, axis=1, kind="stable")[:, :5]
    ld = torch.from_numpy(np.take_along_axis(d, loc, 1).astype(np.float32))
    li = torch.from_numpy((loc + start).astype(np.int64))  # global ids = start_index + local id
    gd, gi = merge_across_ranks(ld, li, 5, merge_fn=_host_merge)
    t = allreduce_max(float(rank + 1))
    # the rank-major receive buffer the device merge (mivs_merge_topk_gathered) reads in place
    rd, ri = all_gather_raw(ld, li)
    assert tuple(ri.shape) == (world, 7, 5) and torch.equal(ri[rank], li) and torch.equal(rd[rank], ld)
    out[rank] = (gi.numpy().tolist(), t, ri.numpy().tolist())
    dist.destroy_process_group()


def test_two_rank_shard_merge_equals_single_shard():
    world = 2
    port = _free_port()
    with mp.Manager() as man:
        out = man.dict()
        mp.spawn(_rank, args=(world, port, out), nprocs=world, join=True)
        res = dict(out)
    rng = np.random.default_rng(0)
    x = rng.standard_normal((1003, 16)).astype(np.float32)
    q = rng.standard_normal((7, 16)).astype(np.float32)
    d = ((q[:, None, :] - x[None]) ** 2).sum(-1)
    exact = np.argsort(d, axis=1, kind="stable")[:, :5]
    for r in range(world):
        ids, t, raw = res[r]
        np.testing.assert_array_equal(np.asarray(ids), exact)
        assert t == 2.0  # max over ranks
        assert raw == res[0][2]  # every rank holds the same gathered buffer


def test_single_process_merge_is_identity():
    from mivs.distributed import merge_across_ranks

    d = torch.rand(3, 4)
    i = torch.arange(12).reshape(3, 4)
    od, oi = merge_across_ranks(d, i, 4)
    assert od is d and oi is i
