"""Host-side logic of the drop-in layer that needs no GPU (a11 / a12 had no tests).

* ``RecallEvaluator`` (improved_multi_gpu_rag.py:310-357) against hand-computed recall;
* the output hook (``pylibraft.config.set_output_as``, improved_multi_gpu_rag.py:111-114): process-wide,
  with a thread-local override for the engine's own worker threads;
* the host merge in the metric's order (inner product descending) and the aggregator's
  ``SearchConfig.exchange`` switch;
* ``parallel_search`` output shapes (a 2-D batch of one query stays 2-D).
"""
import threading

import numpy as np
import pytest
import torch

import improved_multi_gpu_rag as imr
import search_result_aggregator as sra
from mivs import config as mcfg


def test_recall_at_k_hand_computed():
    R = imr.RecallEvaluator
    retrieved = np.array([5, 3, 9, 1, 7, 2])
    relevant = np.array([1, 2, 3, 4])
    assert R.calculate_recall_at_k(retrieved, relevant, 1) == 0.0           # {5}
    assert R.calculate_recall_at_k(retrieved, relevant, 2) == 0.25          # {5,3}: 3
    assert R.calculate_recall_at_k(retrieved, relevant, 4) == 0.5           # {5,3,9,1}: 3,1
    assert R.calculate_recall_at_k(retrieved, relevant, 6) == 0.75          # + 2
    assert R.calculate_recall_at_k(np.array([]), np.array([]), 3) == 1.0
    assert R.calculate_recall_at_k(retrieved, np.array([]), 3) == 0.0
    m = R.evaluate_recall_multiple_k(retrieved, relevant, [1, 2, 4, 10])
    assert m == {1: 0.0, 2: 0.25, 4: 0.5, 10: 0.75}  # k beyond the retrieved list clamps


def test_synthetic_ground_truth_is_seeded_like_the_reference():
    a = imr.RecallEvaluator.generate_synthetic_ground_truth(3, 1000, 10)
    b = imr.RecallEvaluator.generate_synthetic_ground_truth(3, 1000, 10)
    assert set(a) == {0, 1, 2} and all((a[i] == b[i]).all() and len(set(a[i])) == 10 for i in a)


def test_output_hook_process_wide_and_thread_local_override():
    t = torch.arange(6, dtype=torch.float32).reshape(2, 3)
    try:
        mcfg.set_output_as(lambda a: a.copy_to_host())
        assert isinstance(mcfg.convert_output(t), np.ndarray)
        seen = {}

        def worker():
            with mcfg.output_as("torch"):
                seen["in"] = mcfg.convert_output(t)
                with mcfg.output_as("raft"):
                    seen["nested"] = mcfg.convert_output(t)
                seen["back"] = mcfg.convert_output(t)
            seen["after"] = mcfg.convert_output(t)

        th = threading.Thread(target=worker)
        th.start()
        th.join()
        assert isinstance(seen["in"], torch.Tensor) and isinstance(seen["back"], torch.Tensor)
        assert isinstance(seen["nested"], mcfg.DeviceArray)
        assert isinstance(seen["after"], np.ndarray)          # the driver's hook again
        assert isinstance(mcfg.convert_output(t), np.ndarray)  # this thread never saw the override
        with pytest.raises(ValueError):
            mcfg.set_output_as("pandas")
        with pytest.raises(ValueError):
            with mcfg.output_as(3):
                pass
    finally:
        mcfg.set_output_as("torch")
    assert mcfg.get_output_as() == "torch"


def test_host_merge_orders_by_metric():
    d = np.array([[0.9, 0.5, 0.1, 0.5]], np.float32)
    i = np.array([[3, 7, 1, 2]], np.int64)
    hd, hi = sra._host_merge(d, i, 3)
    np.testing.assert_array_equal(hi, [[1, 2, 7]])
    hd, hi = sra._host_merge(d, i, 3, "inner_product")
    np.testing.assert_array_equal(hi, [[3, 2, 7]])
    np.testing.assert_array_equal(hd, np.array([[0.9, 0.5, 0.5]], np.float32))
    # missing results (id -1) sort last whatever their padding distance
    d2 = np.array([[np.inf, 1.0, -np.inf]], np.float32)
    i2 = np.array([[-1, 4, -1]], np.int64)
    _, hi = sra._host_merge(d2, i2, 3, "inner_product")
    np.testing.assert_array_equal(hi, [[4, -1, -1]])


def test_merge_search_results_inner_product_without_engine(monkeypatch):
    monkeypatch.setattr(sra, "CUVS_AVAILABLE", False)
    r0 = sra.SearchResult(np.array([[8, 4]], np.float32), np.array([[80, 40]]), 0, 0.1, 2, 2)
    r1 = sra.SearchResult(np.array([[9, 1]], np.float32), np.array([[90, 10]]), 1, 0.1, 2, 2)
    agg = sra.SearchResultAggregator(None)
    d, i = agg.merge_search_results([r0, r1], 3, metric="inner_product")
    np.testing.assert_array_equal(i, [[90, 80, 40]])
    d, i = agg.merge_search_results([r0, r1], 3)
    np.testing.assert_array_equal(i, [[10, 40, 80]])


def test_search_config_exchange_switch():
    # (peer copies + K7 by default: the RCCL exchange stays opt-in until ncclCommInitAll has run on a multi-GPU node)
    assert sra.SearchConfig(k=5).exchange == "peer"
    assert sra.SearchConfig(k=5, exchange="auto").exchange == "auto"
    assert sra.SearchConfig(k=5, exchange="rccl").exchange == "rccl"
    with pytest.raises(ValueError, match="exchange"):
        sra.SearchConfig(k=5, exchange="nccl2")


class _FakeIndex:
    metric = "sqeuclidean"

    def __len__(self):
        return 100


def test_parallel_search_keeps_2d_for_one_row_batches(monkeypatch):
    """a [1, d] batch returns [1, k]; only a 1-D query returns 1-D; batch_search returns (k,)
    pairs whatever the tail size. The device pieces are replaced by CPU stand-ins."""
    k = 4

    def fake_search_on_gpu(self, gpu_id, index, query, kk):
        q = query if query.dim() == 2 else query[None]
        d = torch.arange(kk, dtype=torch.float32).repeat(q.shape[0], 1) + q[:, :1]
        return d, torch.arange(kk).repeat(q.shape[0], 1) + 10 * gpu_id

    import mivs.ops as ops

    monkeypatch.setattr(imr.ParallelSearchEngine, "search_on_gpu", fake_search_on_gpu)
    monkeypatch.setattr(ops, "merge_topk", lambda d, i, kk, metric="sqeuclidean": (d[:, :kk], i[:, :kk]))
    monkeypatch.setattr(torch.cuda, "device", lambda *_: __import__("contextlib").nullcontext())
    eng = imr.ParallelSearchEngine({0: _FakeIndex()}, imr.IndexType.IVF_FLAT,
                                   imr.SearchConfig(top_k=k, search_batch_size=5))
    d, i = eng.parallel_search(torch.zeros(1, 8))
    assert d.shape == (1, k) and i.shape == (1, k)
    d, i = eng.parallel_search(torch.zeros(8))
    assert d.shape == (k,)
    out = eng.batch_search([torch.full((8,), float(r)) for r in range(11)])
    assert len(out) == 11 and all(dd.shape == (k,) and ii.shape == (k,) for dd, ii in out)
    assert out[10][0][0] == 10.0  # the one-query tail kept its own row
