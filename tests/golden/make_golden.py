#!/usr/bin/env python3
"""Regenerate the golden fixtures in tests/golden/ (run in the build container, NOT on the GPU box).

Every fixture is data — inputs and expected outputs — pinned by the reference itself or by the
reference's own CPU baselines:

  G1 distribute_workload.json   outputs of the reference's GPUResourceManager.distribute_workload
                                (Attempt_1/gpu_resource_manager.py:170-233), obtained by importing
                                the reference module with its GPU discovery stubbed out;
  G3 merge.json                 the two merge fixtures written in
                                Attempt_1/test_search_result_aggregator.py:308-358;
  G4 knn_*.npz                  exact kNN from sklearn NearestNeighbors(algorithm='brute') — the
                                reference's CPU baseline (VectorSearch_QuestionRetrieval.ipynb:878) —
                                on (i) the reference's own sample_embeddings.pt (10x384 MiniLM
                                embeddings, stored here as data) and (ii) a seeded 10,000x768 set;
  G5 kmeans.npz                 sklearn KMeans(init=C0, n_init=1, algorithm='lloyd') on a seeded
                                20,000x64 mixture.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"


def g1():
    sys.path.insert(0, os.path.join(REF, "Attempt_1"))
    import gpu_resource_manager as ref  # the reference module (only here, to capture golden outputs)

    out = []
    for n in [1, 7, 300, 301, 10_000, 1_000_000, 80_000_000, 100_000_000]:
        for p in [1, 2, 3, 4, 8]:
            m = ref.GPUResourceManager.__new__(ref.GPUResourceManager)
            m.available_gpus = list(range(p))
            m.gpu_memory_info = {g: {"available": 16 * 2**30} for g in range(p)}
            m.gpu_configs = []
            out.append({"n": n, "gpus": p, "strategy": "even", "ranges": [list(r) for r in m.distribute_workload(n)]})
    m = ref.GPUResourceManager.__new__(ref.GPUResourceManager)
    m.available_gpus = [0, 1]
    m.gpu_memory_info = {0: {"available": 8 * 2**30}, 1: {"available": 16 * 2**30}}
    m.gpu_configs = []
    mem = {"n": 300, "gpus": 2, "strategy": "memory_based", "available": [8 * 2**30, 16 * 2**30],
           "ranges": [list(r) for r in m.distribute_workload(300, strategy="memory_based")]}
    with open(os.path.join(HERE, "distribute_workload.json"), "w") as f:
        json.dump({"source": "Attempt_1/gpu_resource_manager.py:170-233 (imported)", "even": out,
                   "memory_based": mem}, f, indent=0)


def g3():
    fx = {
        "source": "Attempt_1/test_search_result_aggregator.py:308-358",
        "single_gpu": {"distances": [[[1.0, 2.0, 3.0], [4.0, 5.0, 6.0]]], "indices": [[[10, 20, 30], [40, 50, 60]]],
                       "k": 2, "expected_distances": [[1.0, 2.0], [4.0, 5.0]],
                       "expected_indices": [[10, 20], [40, 50]]},
        "two_gpus": {"distances": [[[2.0, 4.0], [6.0, 8.0]], [[1.0, 3.0], [5.0, 7.0]]],
                     "indices": [[[20, 40], [60, 80]], [[10, 30], [50, 70]]], "k": 3,
                     "expected_distances": [[1.0, 2.0, 3.0], [5.0, 6.0, 7.0]],
                     "expected_indices": [[10, 20, 30], [50, 60, 70]]},
    }
    with open(os.path.join(HERE, "merge.json"), "w") as f:
        json.dump(fx, f, indent=1)


def g4():
    import torch
    from sklearn.neighbors import NearestNeighbors

    emb = torch.load(os.path.join(REF, "Latest/cuVS-2-gpu/medical_qa_data/sample_embeddings.pt"),
                     weights_only=True).numpy().astype(np.float32)
    nn = NearestNeighbors(n_neighbors=5, algorithm="brute", metric="euclidean").fit(emb.astype(np.float64))
    d, i = nn.kneighbors(emb.astype(np.float64))
    np.savez_compressed(os.path.join(HERE, "knn_sample_embeddings.npz"), x=emb, k=5, ids=i.astype(np.int64),
                        sqdist=(d ** 2).astype(np.float64))
    rng = np.random.default_rng(1234)
    x = rng.standard_normal((10_000, 768)).astype(np.float32)
    q = rng.standard_normal((100, 768)).astype(np.float32)
    nn = NearestNeighbors(n_neighbors=10, algorithm="brute", metric="euclidean").fit(x.astype(np.float64))
    d, i = nn.kneighbors(q.astype(np.float64))
    np.savez_compressed(os.path.join(HERE, "knn_synthetic_10k.npz"), seed=1234, n=10_000, nq=100, d=768, k=10,
                        ids=i.astype(np.int64), sqdist=(d ** 2).astype(np.float64))


def g5():
    from sklearn.cluster import KMeans

    rng = np.random.default_rng(77)
    centers = rng.standard_normal((40, 64)).astype(np.float32) * 3
    lab = rng.integers(0, 40, 20_000)
    x = (centers[lab] + rng.standard_normal((20_000, 64)).astype(np.float32)).astype(np.float32)
    # init near the true centres: no cluster ever empties (sklearn relocates empty clusters,
    # mivs keeps their centroid; the fixture pins the common Lloyd path)
    c0 = (centers + 0.5 * rng.standard_normal((40, 64))).astype(np.float32)
    km = KMeans(n_clusters=40, init=c0, n_init=1, algorithm="lloyd", max_iter=10, tol=0.0).fit(x)
    np.savez_compressed(os.path.join(HERE, "kmeans.npz"), seed=77, iters=10, c0=c0,
                        centroids=km.cluster_centers_.astype(np.float32), labels=km.labels_.astype(np.int32),
                        n_iter=km.n_iter_)


if __name__ == "__main__":
    g1()
    g3()
    g4()
    g5()
    print("golden fixtures written to", HERE)
