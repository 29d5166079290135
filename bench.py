#!/usr/bin/env python3
"""bench.py — IVF-Flat 10M x 768 on MI355X: QPS @ recall@10 >= 0.95 + index-build vectors/s.

Workload (BASELINE.json configs[2], the metric's config): per GPU a 10,000,000 x 768
fp32 corpus shard (synthetic clustered data generated ON the device, L2-normalised),
IVF-Flat n_lists=1024 (cuVS defaults: 20 k-means iterations on a 0.5 trainset
fraction), batch of Q=10,000 held-out queries, n_probes=32, k=10.

One step = one batched ivf_flat.search of the Q queries on every rank (+ for N>1 the
RCCL all-gather of the per-shard top-k and the device merge). N GPUs = one process
per GPU (torch.distributed.run). Two corpus modes:
  * default (weak scaling, "scaling": "weak"): each rank owns a 10M-row shard of an N x 10M corpus
    (BASELINE configs[3] at N=8);
  * --rows-total R (strong scaling, "scaling": "strong"): one R-row corpus split over the N ranks with the
    reference's 'even' split (gpu_resource_manager.distribute_workload), R = 10M for configs[2] at every N.
`value` is the full-corpus QPS in both: Q queries answered over the whole corpus (every shard searched and
the per-shard top-k merged) per second = Q / step time. `shard_searches_per_s` (Q * N / step time) is reported
beside it.

Also reported: build vectors/s (wall clock, data resident in HBM), recall@10 against
exact brute-force ground truth (same engine), the fine-scan kernel's roofline
(hipEvents around the kernel over the timed steps; algorithmic flops and bytes from
the engine's per-search counts) and the FAISS-algorithm CPU baseline timed on this
host's cores on a bounded query sample (rank 0, N=1 only).
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "cuvs-rag_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "QPS @ recall@10≥0.95 + index-build vectors/sec, 10M×768 IVF-Flat"
PEAK_HBM_GBS = 8000.0       # MI355X HBM3E peak (MI355X_MICROARCH.md)
PEAK_F32_MFMA_TFS = 157.3   # dense fp32 MFMA peak (v_mfma_f32_32x32x2_f32)
PEAK_F16_MFMA_TFS = 2500.0  # dense fp16 MFMA peak (v_mfma_f32_32x32x16_f16; no sparsity)
QUERY_ROW_BASE = 1 << 40    # queries: same mixture, rows never in any corpus shard
SEED = 0


def parse():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--rows", type=int, default=10_000_000, help="corpus rows per GPU (weak scaling)")
    ap.add_argument("--rows-total", type=int, default=0,
                    help="fixed corpus of this many rows split over the ranks (strong scaling; 0: --rows per GPU)")
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--queries", type=int, default=10_000)
    ap.add_argument("--n-lists", type=int, default=1024)
    ap.add_argument("--n-probes", type=int, default=32)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--kmeans-iters", type=int, default=20)
    ap.add_argument("--trainset-fraction", type=float, default=0.5)
    # 65,536 centres, sigma 0.75 (tools/tune_dataset.py, profiles/r01_dataset_tuning.log): recall@10 0.96 at
    # n_probes=32 and 0.94 at 16, i.e. 32 is the smallest swept n_probes reaching the 0.95 target
    ap.add_argument("--centers", type=int, default=65536, help="mixture centres of the synthetic corpus")
    ap.add_argument("--sigma", type=float, default=0.75)
    ap.add_argument("--gt-queries", type=int, default=2000, help="queries with exact ground truth for recall")
    ap.add_argument("--sweep", default="8,16,20,24,32,64", help="comma list of n_probes to sweep (QPS + recall each); "
                                                                "'' to skip")
    ap.add_argument("--cpu-sweep", default="16,20,24,32",
                    help="n_probes of the CPU baseline's sweep (matched-recall point); '' to skip")
    ap.add_argument("--cpu-build-rows", type=int, default=2_000_000,
                    help="corpus rows the CPU build baseline's add is timed on (scaled to the corpus; 0: skip)")
    ap.add_argument("--block-cache-gb", type=float, default=96.0,
                    help="engine block cache (opt-in, DESIGN.md §5) enabled for the warm builds after the cold one; "
                         "0 keeps it off")
    ap.add_argument("--cpu-seconds", type=float, default=8.0,
                    help="target duration of each CPU-baseline sample (the node's cores, then the job's share)")
    ap.add_argument("--latency", default="1,10,100",
                    help="side line: per-call latency of searches of this many queries (the reference searches one "
                         "query per call); '' to skip")
    ap.add_argument("--latency-probes", default="32,20", help="n_probes of the latency side line (20: cuVS default)")
    ap.add_argument("--batch-sweep", default="1000,5000,20000,32768",
                    help="side line: QPS at these query batch sizes (the headline's batch is --queries); '' to skip")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--flat-rows", type=int, default=1_000_000,
                    help="BASELINE configs[1] side line: brute force over this many rows (0: skip)")
    ap.add_argument("--pq-rows", type=int, default=12_500_000,
                    help="BASELINE configs[4] line: IVF-PQ over this many fp16 rows PER RANK (the per-GPU share of "
                         "100M x 768 on 8 GPUs), refined top-k merged across ranks over RCCL (0: skip)")
    ap.add_argument("--pq-lut16", type=int, default=1,
                    help="add the same PQ searches with the opt-in fp16 LUT (SearchParams lut_dtype float16) to the "
                         "configs[4] line as 'lut_fp16' (0: skip)")
    ap.add_argument("--large-k", default="2000,4000",
                    help="side line (rank 0, N=1): the reference's large-k requests at configs[2] "
                         "(top_k 2000, k*2 per shard: improved_multi_gpu_rag.py:40,247); '' to skip")
    ap.add_argument("--single-process", type=int, default=1,
                    help="side line (N=1 launch): the reference's one-process shape -- every visible GPU holds a "
                         "rows-per-GPU shard, ParallelIndexBuilder threads build them, SearchResultAggregator "
                         "searches them and merges over RCCL (LocalComm); 0 to skip")
    ap.add_argument("--build-warmup", type=int, default=1,
                    help="untimed warm builds between the cold (first) build and the timed warm one")
    ap.add_argument("--single-process-timeout", type=float, default=240.0,
                    help="seconds the one-process multi-GPU side line may take before it is abandoned")
    ap.add_argument("--json-out", default="")
    ap.add_argument("--ids-out", default="", help="(set by the launcher) rank 0 saves the merged ids of the timed "
                                                  "search here (.npy)")
    ap.add_argument("--launch-timeout", type=float, default=1500.0,
                    help="seconds the self-launched ranks may take (--gpus N > 1 without WORLD_SIZE)")
    ap.add_argument("--launcher-dry-run", action="store_true",
                    help="print the command --gpus N > 1 would start its ranks with, and exit")
    return ap.parse_args()


def log(rank, *a):
    if rank == 0:
        print(*a, file=sys.stderr, flush=True)


def sync_all(world):
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()


def max_over_ranks(v, world, dev):
    if world == 1:
        return float(v)
    t = torch.tensor([float(v)], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def recall_at_k(found: np.ndarray, truth: np.ndarray) -> float:
    """RecallEvaluator.calculate_recall_at_k (improved_multi_gpu_rag.py:314-327) with relevant = exact top-k."""
    k = truth.shape[1]
    hits = sum(len(set(f[:k].tolist()) & set(t.tolist())) for f, t in zip(found, truth))
    return hits / float(truth.size)


def load_traffic(cfg_key: str):
    """HBM bytes per fine-scan launch from the committed rocprofv3 --pmc summary, if one matches."""
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json")), reverse=True):
        try:
            with open(path) as f:
                j = json.load(f)
        except (OSError, ValueError):
            continue
        if j.get("config_key") == cfg_key and j.get("hbm_bytes_per_launch"):
            return float(j["hbm_bytes_per_launch"]), os.path.relpath(path, ROOT)
    return None, None


MAX_SCLK_MHZ = 2400.0  # MI355X max engine clock (MI355X_MICROARCH.md): the dense MFMA peaks are quoted at it


def load_clock(cfg_key: str):
    """The clock the fine-scan kernel held (GRBM_GUI_ACTIVE / 8 XCDs / kernel time, MI355X_MICROARCH.md 'DVFS
    give-back') from the committed rocprofv3 --pmc pass of this configuration, if one matches."""
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*clock*.json")), reverse=True):
        try:
            with open(path) as f:
                j = json.load(f)
        except (OSError, ValueError):
            continue
        if j.get("config_key") == cfg_key and j.get("clock_mhz_held"):
            return j, os.path.relpath(path, ROOT)
    return None, None


def host_cpu_info() -> dict:
    """What the CPU baseline ran on: model, logical / physical cores and NUMA nodes of the node (lscpu),
    the cores this process may run on (sched_getaffinity) and the share the job is given (OMP_NUM_THREADS,
    set per GPU by the harness)."""
    info = {"logical_cpus": os.cpu_count()}
    try:
        aff = sorted(os.sched_getaffinity(0))
        info["affinity_cpus"] = len(aff)
    except AttributeError:
        aff = []
    try:
        import subprocess

        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        kv = {}
        for ln in out.splitlines():
            if ":" in ln:
                a_, b_ = ln.split(":", 1)
                kv[a_.strip()] = b_.strip()
        info["model"] = kv.get("Model name")
        sockets = int(kv.get("Socket(s)", "0") or 0)
        cores = int(kv.get("Core(s) per socket", "0") or 0)
        info["physical_cores"] = sockets * cores if sockets and cores else None
        info["threads_per_core"] = int(kv.get("Thread(s) per core", "0") or 0) or None
        info["numa_nodes"] = int(kv.get("NUMA node(s)", "0") or 0) or None
    except Exception as e:  # lscpu missing: the counts above still stand
        info["lscpu_error"] = repr(e)
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    info["omp_num_threads"] = omp or None
    return info


def node_threads() -> int:
    """Every hardware thread this process may run on (sched_getaffinity)."""
    try:
        return max(1, len(os.sched_getaffinity(0)))
    except AttributeError:
        return os.cpu_count() or 1


def cgroup_cpu_quota():
    """CPUs' worth of time the process's cgroup may use per period (cgroup v2 cpu.max, v1 cfs_quota_us / period), or
    None when unlimited or unreadable, and the file it came from."""
    try:
        with open("/proc/self/cgroup") as f:
            rel = [ln.strip().split(":", 2)[2] for ln in f if ln.startswith("0::")]
    except (OSError, IndexError):
        rel = []
    cands = [os.path.join("/sys/fs/cgroup", r.lstrip("/"), "cpu.max") for r in rel] + ["/sys/fs/cgroup/cpu.max"]
    for path in cands:
        try:
            with open(path) as f:
                q, per = f.read().split()[:2]
            return (None if q == "max" else float(q) / float(per)), path
        except (OSError, ValueError):
            continue
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            per = int(f.read())
        return (None if q <= 0 else q / per), "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"
    except (OSError, ValueError):
        return None, None


def effective_cpus() -> dict:
    """The host cores the CPU baseline can actually use: the affinity set capped by the cgroup's CPU quota (a
    quota of 16 CPUs on a 256-thread affinity set throttles 256 threads to 16 CPUs' worth of time, with every
    thread descheduled for most of each period -- why the round-5 line ran slower on 256 threads than on 16)."""
    import math

    aff = node_threads()
    quota, src = cgroup_cpu_quota()
    eff = aff if quota is None else max(1, min(aff, int(math.floor(quota + 1e-6))))
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return {"effective": eff, "affinity": aff, "cgroup_quota_cpus": quota, "cgroup_file": src,
            "omp_num_threads": omp or None,
            "limited_by": "cgroup cpu quota" if quota is not None and eff < aff else "affinity set"}


def cpu_threads() -> int:
    """Threads for the CPU legs: the effective cores (affinity set capped by the cgroup quota)."""
    return effective_cpus()["effective"]


def host_copy_rows(t_dev, threads, chunk_rows=1 << 20):
    """A host numpy copy of a device [n, d] fp32 tensor, first-touched by `threads` OpenMP threads (orc_parallel_copy:
    the pages spread over the NUMA nodes of the threads that will scan them), staged through ~3 GB pageable chunks."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O  # (the cpu_baseline leg: an allowed oracle user)

    O.fast_set_threads(threads)
    n = t_dev.shape[0]
    out = np.empty(tuple(t_dev.shape), dtype=np.float32)
    for a0 in range(0, n, chunk_rows):
        h = t_dev[a0:a0 + chunk_rows].cpu().numpy()
        O.parallel_copy(out[a0:a0 + h.shape[0]], np.ascontiguousarray(h))
        del h
    return out


def cpu_baseline(idx, q_host, gt, n_probes, k, target_s, rank_log, sweep=(), gpu_sweep=None):
    """FAISS-algorithm IVF-Flat search (oracle/cpu_baseline.c: IndexIVFFlat's per-query scan, OpenMP over queries,
    AVX-512 / AVX2 workers picked for this host) on the effective cores (the affinity set capped by the cgroup CPU
    quota), on the same index copied to host memory first-touched in parallel. Each point on a query sample of >= 8
    queries per thread sized for ~target_s seconds; `value` at n_probes (the headline's), `n_probes_sweep` at the
    points of `sweep`, and the matched-recall point: the smallest swept n_probes reaching recall@10 >= 0.95."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O  # bench.py's cpu_baseline leg is one of the oracle's allowed users

    cpus = effective_cpus()
    threads = cpus["effective"]
    rank_log(f"[cpu] host cores: {cpus}; copying the index to host ({idx.size} rows, parallel first touch) ...")
    t0 = time.perf_counter()
    rows_dev = idx.list_rows()
    rows = host_copy_rows(rows_dev, threads)
    del rows_dev
    torch.cuda.empty_cache()
    t_copy = time.perf_counter() - t0
    ids = idx.list_ids().cpu().numpy()
    sizes = idx.list_sizes.numpy()
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    cents = idx.centers.cpu().numpy()

    def timed(nthreads, npr, tgt, q0=0, min_per_thread=8):
        O.fast_set_threads(nthreads)
        O.fast_ivf_search(rows, ids, off, cents, q_host[q0:q0 + nthreads], npr, k)  # warm threads / pages
        n0 = nthreads
        t0 = time.perf_counter()
        O.fast_ivf_search(rows, ids, off, cents, q_host[q0:q0 + n0], npr, k)
        per_q = (time.perf_counter() - t0) / n0
        ns = int(max(min_per_thread * nthreads, min(q_host.shape[0] - q0, tgt / max(per_q, 1e-9))))
        ns = min(ns, q_host.shape[0] - q0)
        t0 = time.perf_counter()
        _, ci = O.fast_ivf_search(rows, ids, off, cents, q_host[q0:q0 + ns], npr, k)
        return ns, time.perf_counter() - t0, ci

    def rec_of(ci, ns):
        nr = min(ns, gt.shape[0])
        return recall_at_k(ci[:nr], gt[:nr]) if nr > 0 else None

    ns, dt, ci = timed(threads, n_probes, target_s)
    rec = rec_of(ci, ns)
    out = {"value": ns / dt, "unit": "QPS", "cores": threads, "kind": "port", "isa": O.fast_isa(),
           "host": host_cpu_info(), "cpus": cpus, "host_copy_s": round(t_copy, 2),
           "sample": f"{ns} of the {q_host.shape[0]} benchmark queries ({ns / threads:.0f} per thread), same index "
                     f"(copied to host, pages first-touched by the {threads} threads), n_probes={n_probes}, k={k}; "
                     f"FAISS IndexIVFFlat search algorithm restated in oracle/cpu_baseline.c (faiss not installed), "
                     f"OpenMP over queries; {dt:.1f} s",
           "recall_at_10": rec,
           "cores_note": f"cores = the {threads} CPUs this process can use: its affinity set ({cpus['affinity']} "
                         f"threads) capped by the cgroup CPU quota ({cpus['cgroup_quota_cpus']} CPUs, "
                         f"{cpus['cgroup_file']})"}
    if cpus["affinity"] > threads:
        # the diagnostic behind the cap: every affinity thread against the quota (one short sample)
        ns_a, dt_a, _ = timed(cpus["affinity"], n_probes, 0.0, min_per_thread=1)
        out["all_affinity_threads"] = {"value": ns_a / dt_a, "threads": cpus["affinity"],
                                       "sample": f"{ns_a} queries, {dt_a:.1f} s",
                                       "note": "oversubscribed: more threads than the cgroup quota's CPUs"}
    pts = []
    for npr in sweep:
        if npr == n_probes:
            pts.append({"n_probes": npr, "qps": ns / dt, "recall_at_10": rec, "queries": ns})
            continue
        ns_s, dt_s, ci_s = timed(threads, npr, target_s / 2)
        pts.append({"n_probes": npr, "qps": ns_s / dt_s, "recall_at_10": rec_of(ci_s, ns_s), "queries": ns_s})
        rank_log(f"[cpu] n_probes={npr}: {ns_s / dt_s:.1f} QPS recall {pts[-1]['recall_at_10']}")
    out["n_probes_sweep"] = pts
    if pts and gpu_sweep:
        out["matched_recall"] = matched_recall(gpu_sweep, pts)
    del rows
    return out


def matched_recall(gpu_sweep, cpu_sweep, target=0.95):
    """QPS at the smallest swept n_probes with recall@10 >= target. The operating point is chosen
    on the GPU sweep's recall (--gt-queries queries against exact ground truth); the CPU baseline runs the same IVF
    search over the same index (the same lists and probes: its results differ only by fast-math rounding), so both
    sides are reported at that n_probes, the CPU's own recall on its smaller query sample beside it."""
    ok = [p for p in gpu_sweep if p.get("recall_at_10") is not None and p["recall_at_10"] >= target]
    if not ok:
        return {"target_recall_at_10": target, "gpu": None, "cpu": None}
    g = min(ok, key=lambda p: p["n_probes"])
    out = {"target_recall_at_10": target, "n_probes": g["n_probes"],
           "gpu": {"qps": round(g["qps_full_corpus"], 2), "recall_at_10": round(g["recall_at_10"], 4)}, "cpu": None}
    c = [p for p in cpu_sweep if p["n_probes"] == g["n_probes"]]
    if c:
        out["cpu"] = {"qps": round(c[0]["qps"], 2), "recall_at_10_own_sample": round(c[0]["recall_at_10"], 4),
                      "sample_queries": c[0]["queries"]}
        out["gpu_over_cpu"] = round(g["qps_full_corpus"] / c[0]["qps"], 1)
    return out


def faiss_kmeans_train(xt, n_lists, niter=10, seed=1234):
    """FAISS Clustering::train as IndexIVFFlat.train runs it (Level1Quantizer sets cp.niter = 10;
    max_points_per_centroid 256): the training set subsampled to 256 x n_lists rows (a random permutation, FAISS's
    rand_perm), the first n_lists of the permutation as the initial centroids, then per iteration the assign through
    IndexFlatL2 (BLAS: ||c||^2 - 2 x.c, argmin, per 16k-row block), the centroid means (compute_centroids) and the
    empty-cluster split (split_clusters: an empty centroid takes a copy of a large cluster's, both nudged by
    +-1/1024). Torch-CPU (MKL) tensors on the caller's threads."""
    g = torch.Generator().manual_seed(seed)
    n = xt.shape[0]
    if n > 256 * n_lists:
        xt = xt[torch.randperm(n, generator=g)[:256 * n_lists]].contiguous()
        n = xt.shape[0]
    c = xt[torch.randperm(n, generator=g)[:n_lists]].clone()
    for _ in range(niter):
        lab = faiss_assign(xt, c)
        cnt = torch.bincount(lab, minlength=n_lists)
        s = torch.zeros_like(c).index_add_(0, lab, xt)
        nz = cnt > 0
        c[nz] = s[nz] / cnt[nz].unsqueeze(1).to(c.dtype)
        for j in torch.nonzero(~nz).flatten().tolist():  # split_clusters
            big = int(torch.multinomial(cnt.double().clamp_min(0) ** 1.0, 1, generator=g))
            c[j] = c[big] * (1 + 1 / 1024.0)
            c[big] = c[big] * (1 - 1 / 1024.0)
            cnt[j] = cnt[big] // 2
            cnt[big] -= cnt[j]
    return c, n


def faiss_assign(x, c, bs=16384):
    """IndexFlatL2 k=1 over the centroids (FAISS's BLAS form for nq >= 20): argmin of ||c||^2 - 2 x.c per block"""
    cn = (c * c).sum(1)
    out = torch.empty(x.shape[0], dtype=torch.int64)
    for b0 in range(0, x.shape[0], bs):
        xb = x[b0:b0 + bs]
        out[b0:b0 + xb.shape[0]] = torch.addmm(cn[None, :], xb, c.t(), beta=1.0, alpha=-2.0).argmin(1)
    return out


def cpu_build_baseline(x_dev, n_lists, rows_total, threads, add_rows, rank_log):
    """FAISS-algorithm IndexIVFFlat build (train + add) on this host's effective cores, torch-CPU (MKL sgemm) for the
    BLAS steps as FAISS uses BLAS: train = faiss_kmeans_train on a 256 x n_lists subsample of the corpus, add = the
    quantizer assign of every row (IndexFlatL2 BLAS form) + the list fill (rows appended to their list: a stable
    gather in list order). The add is timed on `add_rows` rows of the corpus and scaled to rows_total:
    build vec/s = rows_total / (train_s + add_s * rows_total / add_rows). Reference: Latest/faiss.ipynb:554-570,
    Latest/cuVS-2-gpu/old/colab_a100_test.ipynb:472-483 (index_ivf.train + add)."""
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        xh = torch.from_numpy(host_copy_rows(x_dev[:add_rows], threads))
        faiss_assign(xh[:20000], xh[:n_lists].clone())  # warm MKL / pages
        t0 = time.perf_counter()
        c, n_train = faiss_kmeans_train(xh, n_lists)
        t_train = time.perf_counter() - t0
        t0 = time.perf_counter()
        lab = faiss_assign(xh, c)
        order = torch.sort(lab, stable=True).indices
        lists = xh.index_select(0, order)
        sizes = torch.bincount(lab, minlength=n_lists)
        t_add = time.perf_counter() - t0
        del lists, xh
    finally:
        torch.set_num_threads(prev)
    add_vps = add_rows / t_add
    total = t_train + rows_total / add_vps
    rank_log(f"[cpu-build] train {t_train:.2f} s on {n_train} rows, add {add_vps / 1e6:.2f} M vec/s -> "
             f"{rows_total / total / 1e6:.3f} M vec/s for {rows_total} rows on {threads} threads")
    return {"build_vectors_per_s": round(rows_total / total, 1), "unit": "vectors/s", "cores": threads,
            "kind": "port", "train_s": round(t_train, 3), "train_rows": n_train, "kmeans_iters": 10,
            "add_vectors_per_s": round(add_vps, 1), "add_sample_rows": add_rows, "build_s_scaled": round(total, 2),
            "list_sizes_min_max": [int(sizes.min()), int(sizes.max())],
            "sample": f"FAISS IndexIVFFlat.train (Clustering: niter 10, 256 x {n_lists} = {n_train} training rows) "
                      f"+ add (IndexFlatL2 BLAS assign + list fill) restated on torch-CPU (MKL sgemm, faiss not "
                      f"installed); add timed on {add_rows} corpus rows and scaled to {rows_total}"}


def faiss_blas_knn(x, qb, k, bs_x=65536):
    """FAISS exhaustive_L2sqr_blas restated on torch-CPU tensors: the database's squared norms (computed inside
    every search, as FAISS does), then per database block one MKL sgemm of the query block against it,
    ||q||^2 + ||x||^2 - 2 q.x, and a running top-k per query (FAISS: a max-heap per query)."""
    xn = (x * x).sum(1)
    qn = (qb * qb).sum(1)
    best_d = torch.full((qb.shape[0], k), float("inf"))
    best_i = torch.full((qb.shape[0], k), -1, dtype=torch.int64)
    for b0 in range(0, x.shape[0], bs_x):
        xb = x[b0:b0 + bs_x]
        dd = torch.addmm(qn[:, None] + xn[None, b0:b0 + bs_x], qb, xb.t(), beta=1.0, alpha=-2.0).clamp_min_(0)
        kk = min(k, dd.shape[1])
        bd, bi = torch.topk(dd, kk, dim=1, largest=False)
        cd = torch.cat([best_d, bd], 1)
        ci = torch.cat([best_i, bi + b0], 1)
        o = torch.topk(cd, k, dim=1, largest=False).indices
        best_d, best_i = cd.gather(1, o), ci.gather(1, o)
    return best_d, best_i


def faiss_blas_knn_timed(xh, qh, k, threads, target_s=6.0):
    """The BLAS form timed on `threads` threads over a query sample sized for ~target_s seconds (queries in blocks of
    FAISS's distance_compute_blas_query_bs = 4096)."""
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        x = torch.from_numpy(xh)
        q = torch.from_numpy(qh)
        faiss_blas_knn(x[:200_000], q[:64], k)  # warm MKL / pages
        t0 = time.perf_counter()
        faiss_blas_knn(x, q[:64], k)
        per_q = (time.perf_counter() - t0) / 64
        n = int(max(64, min(q.shape[0], target_s / max(per_q, 1e-9))))
        t0 = time.perf_counter()
        ids = []
        for b0 in range(0, n, 4096):
            ids.append(faiss_blas_knn(x, q[b0:min(n, b0 + 4096)], k)[1])
        dt = time.perf_counter() - t0
    finally:
        torch.set_num_threads(prev)
    return {"qps": n / dt, "n": n, "s": dt, "ids": torch.cat(ids).numpy(), "bs_q": min(n, 4096), "bs_x": 65536}


def flat_side_line(a, q, k, rl):
    """BASELINE configs[1]: exact k-NN over a 1M x 768 fp32 corpus of the same mixture on the GPU (the
    fp16 pre-filter + exact refine path, k <= 16), next to the FAISS IndexFlatL2 algorithm on this host's
    cores (oracle/cpu_baseline.c orc_fast_knn) on a bounded query sample."""
    from mivs import ops
    from mivs.neighbors import brute_force

    n = a.flat_rows
    xf = ops.synth_mixture(n, a.dim, SEED + 7, n_centers=a.centers, sigma=a.sigma, device=torch.cuda.current_device())
    bf = brute_force.build(xf)
    brute_force.search(bf, q, k)
    torch.cuda.synchronize()
    reps = 5
    t0 = time.perf_counter()
    for _ in range(reps):
        fd, fi = brute_force.search(bf, q, k)
    torch.cuda.synchronize()
    t_gpu = (time.perf_counter() - t0) / reps
    gpu_qps = q.shape[0] / t_gpu
    rl(f"[flat] {n} x {a.dim} brute force, k={k}: {gpu_qps:,.0f} QPS on the GPU")
    line = {"rows": n, "dim": a.dim, "k": k, "queries": q.shape[0], "gpu_qps": round(gpu_qps, 1),
            "gpu_ms_per_batch": round(t_gpu * 1e3, 3), "gpu_path": "fp16 pre-filter (K10) + exact fp32 refine (K11)"}
    if not a.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O  # the cpu_baseline leg (an allowed oracle user)

        threads = cpu_threads()
        O.fast_set_threads(threads)
        xh = xf.cpu().numpy()
        qh = q[:4096].cpu().numpy()
        # 1. FAISS's own path at this batch size: IndexFlatL2.search takes the BLAS form for nq >= 20
        # (distance_compute_blas_threshold; exhaustive_L2sqr_blas: row norms, sgemm of query x database blocks,
        # ||q||^2 + ||x||^2 - 2 q.x, a per-query top-k) -- restated with torch-CPU (MKL sgemm) on the same threads
        blas = faiss_blas_knn_timed(xh, qh, k, threads, target_s=6.0)
        agree = float(np.mean(blas["ids"] == fi[:blas["n"]].cpu().numpy()))
        # 2. the per-query scalar form (FAISS's path below 20 queries; oracle/cpu_baseline.c orc_fast_knn)
        O.fast_knn(xh, qh[:4], k)
        t0 = time.perf_counter()
        O.fast_knn(xh, qh[:16], k)
        per_q = (time.perf_counter() - t0) / 16
        ns = int(max(16, min(512, 4.0 / max(per_q, 1e-9))))
        t0 = time.perf_counter()
        _, ci = O.fast_knn(xh, qh[:ns], k)
        dt = time.perf_counter() - t0
        agree_port = float(np.mean(ci == fi[:ns].cpu().numpy()))
        line["cpu_baseline"] = {
            "value": round(blas["qps"], 2), "unit": "QPS", "cores": threads, "kind": "port",
            "sample": f"{blas['n']} queries in one batch (FAISS IndexFlatL2 BLAS path for nq >= 20: sgemm of "
                      f"{blas['bs_q']}-query x {blas['bs_x']}-row blocks + ||q||^2 + ||x||^2 - 2 q.x + per-query "
                      f"top-k, torch-CPU MKL on {threads} threads; faiss not installed); {blas['s']:.1f} s",
            "ids_equal_to_gpu_frac": round(agree, 4),
            "per_query_form": {"value": round(ns / dt, 2), "unit": "QPS", "cores": threads,
                               "sample": f"{ns} queries, FAISS fvec_L2sqr per (query, row) (its path for nq < 20; "
                                         f"oracle/cpu_baseline.c); {dt:.1f} s",
                               "ids_equal_to_gpu_frac": round(agree_port, 4)}}
        line["gpu_over_cpu"] = round(gpu_qps / blas["qps"], 1)
        rl(f"[flat] CPU {blas['qps']:.1f} QPS (BLAS form), {ns / dt:.1f} QPS (per-query form) on {threads} threads")
        del xh
    bf.close()
    del xf
    torch.cuda.empty_cache()
    return line


def large_k_side_line(a, idx, q, rl, scanned_rows):
    """The reference's large-k default at configs[2]: its driver asks for top_k = 2000 and each shard for
    k * 2 (improved_multi_gpu_rag.py:40,247,416). Every k > 16 runs through the fp16 pre-filter:
    T_q from an exact scan of a 1/64 sample of the probed rows, K13 streams the rows under it, K16 proves each
    query's window and recomputes it in the pinned fp32 order (the exact fp32 scan, K3 DUMP + K8, answers the
    queries it cannot prove). QPS over the full 10k-query batch; the same search through the exact path
    (MIVS_LARGE_K_PF=0) beside it, checked equal; K13's time and K16's gather of the window rows."""
    from mivs import _native
    from mivs.neighbors import ivf_flat

    out = []
    sp = ivf_flat.SearchParams(n_probes=a.n_probes)
    for kk in [int(v) for v in a.large_k.split(",") if v.strip()]:
        ivf_flat.search(sp, idx, q, kk)
        torch.cuda.synchronize()
        _native.set_profiling(True)
        idx.profile_collect()
        reps = 3
        t0 = time.perf_counter()
        for _ in range(reps):
            d, i = ivf_flat.search(sp, idx, q, kk)
        torch.cuda.synchronize()
        t = (time.perf_counter() - t0) / reps
        pr = idx.profile_collect()
        _native.set_profiling(False)
        st = idx.last_search_stats()
        batches = max(1, pr["n_calls"] // reps)
        scan_ms = pr["scan_ms"] / reps
        # the exact fp32 path for comparison (and the check that both give the same bits)
        os.environ["MIVS_LARGE_K_PF"] = "0"
        try:
            ivf_flat.search(sp, idx, q, kk)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            ed, ei = ivf_flat.search(sp, idx, q, kk)
            torch.cuda.synchronize()
            t_ex = time.perf_counter() - t0
        finally:
            del os.environ["MIVS_LARGE_K_PF"]
        same = bool(torch.equal(ei, i)) and bool(torch.equal(ed.view(torch.int32), d.view(torch.int32)))
        # K16's floor: the window rows' fp32 values gathered once per (query, window row)
        win_bytes = float(st["window_candidates"]) * a.dim * 4
        ok = bool((i[:, 0] >= 0).all()) and bool((d[:, 1:] >= d[:, :-1]).all())
        out.append({"k": kk, "queries": q.shape[0], "qps": round(q.shape[0] / t, 1), "ms_per_batch": round(t * 1e3, 3),
                    "path": "K3 DUMP sample -> T_q, K13 fp16 row-stationary scan, K16 window + pinned fp32 keys + "
                            "(key, id) sort; unproven queries -> exact K3 DUMP + K8",
                    "query_batches": batches, "k13_ms_per_search": round(scan_ms, 4),
                    "rest_ms_per_search": round(t * 1e3 - scan_ms, 3),
                    "candidates": st["candidates"], "window_rows": st["window_candidates"],
                    "window_gather_gb": round(win_bytes / 1e9, 2), "unproven_queries": st["overflow_queries"],
                    # last_search_stats() describes the last query batch of a search (ivf_search_impl splits the
                    # batch when the K16 workspace cannot hold every query's window)
                    "stats_scope": "whole search" if batches == 1 else f"last of {batches} query batches",
                    "exact_path_qps": round(q.shape[0] / t_ex, 1), "equal_to_exact_path": same, "well_formed": ok})
        rl(f"[large-k] k={kk}: {q.shape[0] / t:,.0f} QPS ({t * 1e3:.1f} ms per {q.shape[0]} queries; K13 {scan_ms:.2f} ms, "
           f"{st['candidates']} candidates, {st['window_candidates']} window rows, {st['overflow_queries']} unproven); "
           f"exact path {q.shape[0] / t_ex:,.0f} QPS, same bits: {same}")
        del d, i, ed, ei
        torch.cuda.empty_cache()
    return out


def build_roofline(kern, t_build):
    """The build's hot kernels against their peaks (device time by hipEvents during the timed build, algorithmic work
    per launch from the engine: mivs_index_build_kernels): k_as_scan (the k-means assign, per iteration, and the final
    assign of every row) in TFLOP/s against the fp16 MFMA peak -- the assign runs through the fp16 pre-filter, the
    labels are the fp32 ones -- and the byte-moving kernels (K5's centroid update, K6's pack, the fp16
    and fp8 copies) in GB/s against HBM."""
    out = {}
    for name, v in kern.items():
        if v["calls"] == 0 or v["ms"] <= 0:
            continue
        rate = v["work"] / (v["ms"] * 1e-3)
        line = {"launches": v["calls"], "ms_total": round(v["ms"], 3), "ms_per_launch": round(v["ms"] / v["calls"], 4)}
        if v["unit"] == "flop":
            line.update({"bound": "mfma", "achieved": round(rate / 1e12, 2), "peak": PEAK_F16_MFMA_TFS,
                         "unit": "TFLOP/s", "frac": round(rate / 1e12 / PEAK_F16_MFMA_TFS, 4),
                         "flops_per_launch": v["work"] / v["calls"]})
        else:
            line.update({"bound": "hbm", "achieved": round(rate / 1e9, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                         "frac": round(rate / 1e9 / PEAK_HBM_GBS, 4), "bytes_per_launch": v["work"] / v["calls"]})
        out[name] = line
    if out:
        tot = sum(v["ms_total"] for v in out.values())
        out["kernels_ms_total"] = round(tot, 3)
        out["kernels_share_of_build"] = round(tot / (t_build * 1e3), 4)
        out["timing"] = "hipEvents around each launch on the build stream (profiling on during the timed build)"
    return out


def batch_sweep_side_line(a, idx, rl, gt, dev):
    """QPS against the query batch size at the main line's index and n_probes (the headline keeps the 10k batch of
    BASELINE.md's plan). K13 streams every probed row once per batch, so its row traffic and its item transitions
    are spread over more queries as the batch grows; batches above kRsMaxBatch (32,768) are split. Queries: the same
    mixture rows as the main batch (its first rows), recall over the main line's ground-truth queries."""
    from mivs import _native, ops
    from mivs.neighbors import ivf_flat

    sp = ivf_flat.SearchParams(n_probes=a.n_probes)
    out = []
    for nq in [int(v) for v in a.batch_sweep.split(",") if v.strip()]:
        qq = ops.synth_mixture(nq, a.dim, SEED, n_centers=a.centers, sigma=a.sigma, row_begin=QUERY_ROW_BASE,
                               device=dev)
        for _ in range(2):
            ivf_flat.search(sp, idx, qq, a.k)
        _native.set_profiling(True)
        idx.profile_collect()
        reps = max(3, a.steps // 4)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            dd, ii = ivf_flat.search(sp, idx, qq, a.k)
        torch.cuda.synchronize()
        t = (time.perf_counter() - t0) / reps
        pr = idx.profile_collect()
        _native.set_profiling(False)
        st = idx.last_search_stats()
        ng = min(nq, gt.shape[0])
        rec = recall_at_k(ii[:ng].cpu().numpy(), gt[:ng])
        out.append({"queries": nq, "qps": round(nq / t, 1), "ms_per_batch": round(t * 1e3, 3),
                    "k13_ms_per_batch": round(pr["scan_ms"] / reps, 3), "recall_at_10": round(rec, 4),
                    "recall_queries": ng, "unproven_queries_last_batch": st["overflow_queries"]})
        rl(f"[batch] Q={nq}: {nq / t:,.0f} QPS ({t * 1e3:.2f} ms per batch, K13 {pr['scan_ms'] / reps:.2f} ms), "
           f"recall {rec:.4f}")
        del qq, dd, ii
        torch.cuda.empty_cache()
    return out


def latency_side_line(a, idx, q, rl):
    """The reference's own search shape (improved_multi_gpu_rag.py:209-237 search_on_gpu, :279-303 batch_search: one
    query per call; cuvs-2gpu-main.ipynb:1789-1836): per-call wall time of ivf_flat.search at small batches, each call
    on the next queries of the benchmark batch, synchronized before and after (what a caller waits for, host
    enqueue included), and the GPU time of the same calls (hipEvents on the search stream). The pre-filter path is
    the same as the main line's; recall and bits are the main search's (tests/test_gpu_baseline_configs.py checks
    Q = 1 and Q = 7 against the oracle)."""
    from mivs.neighbors import ivf_flat

    out = []
    for np_ in [int(v) for v in a.latency_probes.split(",") if v.strip()]:
        sp = ivf_flat.SearchParams(n_probes=np_)
        for nq in [int(v) for v in a.latency.split(",") if v.strip()]:
            calls = 400 if nq <= 10 else 200
            for i in range(5):  # warm (workspace sizes for this batch shape)
                ivf_flat.search(sp, idx, q[i * nq:(i + 1) * nq], a.k)
            torch.cuda.synchronize()
            wall = []
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(calls)]
            for c in range(calls):
                o = (c * nq) % (q.shape[0] - nq)
                qq = q[o:o + nq]
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                ev[c][0].record()
                ivf_flat.search(sp, idx, qq, a.k)
                ev[c][1].record()
                torch.cuda.synchronize()
                wall.append(time.perf_counter() - t0)
            gpu = [e0.elapsed_time(e1) for e0, e1 in ev]
            w = np.array(wall) * 1e3
            st = idx.last_search_stats()
            line = {"queries_per_call": nq, "n_probes": np_, "k": a.k, "calls": calls,
                    "p50_ms": round(float(np.percentile(w, 50)), 4), "p99_ms": round(float(np.percentile(w, 99)), 4),
                    "mean_ms": round(float(w.mean()), 4), "gpu_p50_ms": round(float(np.percentile(gpu, 50)), 4),
                    "qps_at_this_batch": round(nq / (w.mean() * 1e-3), 1), "path": {13: "K13", 10: "K10", 31: "K3w",
                                                                                    3: "K3"}.get(st.get("scan_kernel"),
                                                                                                 str(st.get("scan_kernel")))}
            out.append(line)
            rl(f"[latency] Q={nq} n_probes={np_}: p50 {line['p50_ms']:.3f} ms p99 {line['p99_ms']:.3f} ms "
               f"(GPU p50 {line['gpu_p50_ms']:.3f} ms) via {line['path']}")
    return {"calls": out, "reference_published": {"search_time_ms": 2.013, "hardware": "A100 (cuVS IVF-Flat)",
                                                  "corpus": "2M rows (its scaling test)",
                                                  "source": "Attempt_1/cuvs_2gpu.ipynb:1258"},
            "note": "context only: the reference's published per-query time is from other hardware and another corpus"}


def single_process_side_line(a, q, ref_ids, rl, devices, indexes=None):
    """The reference's own multi-GPU shape (improved_multi_gpu_rag.py:105,206,239-277; merge contract
    Attempt_1/test_search_result_aggregator.py:405-457): ONE process drives `devices` -- a rows-per-GPU
    shard on each (shard g = rows [g n, (g + 1) n) of the same corpus, generated on its device and built by
    ParallelIndexBuilder threads with global ids; `indexes` may hold shards already built), and
    SearchResultAggregator searches them in parallel threads and merges over RCCL (exchange='rccl':
    mivs_comm_init_all + grouped all-gather + K7). `ref_ids` (host [Q, k]): the same search's merged ids from
    the one-process-per-GPU run (torch.distributed), which the aggregator's final ids must equal."""
    from gpu_resource_manager import GPUResourceManager
    from improved_multi_gpu_rag import GPUConfig, IndexType, ParallelIndexBuilder
    from search_result_aggregator import SearchConfig, SearchResultAggregator

    from mivs import ops

    devices = list(devices)
    G = len(devices)
    shards = corpus_shards(a, G)
    indexes = dict(indexes or {})
    extra = {}
    t_build = 0.0
    todo = [g for g in devices if g not in indexes]
    if todo:
        b = ParallelIndexBuilder(G)
        params = {"n_lists": a.n_lists, "kmeans_n_iters": a.kmeans_iters,
                  "kmeans_trainset_fraction": a.trainset_fraction}

        def one(g):
            b0, b1 = shards[devices.index(g)]
            with torch.cuda.device(g):
                xg = ops.synth_mixture(b1 - b0, a.dim, SEED, n_centers=a.centers, sigma=a.sigma, row_begin=b0, device=g)
                torch.cuda.synchronize(g)
                ix, tb = b.build_index_on_gpu(GPUConfig(g), xg, IndexType.IVF_FLAT, params, ids_offset=b0)
                del xg
                torch.cuda.empty_cache()
                return g, ix, tb

        t0 = time.perf_counter()
        futs = [b.executor.submit(one, g) for g in todo]
        for f in futs:
            g, ix, _ = f.result()
            indexes[g] = extra[g] = ix
        t_build = time.perf_counter() - t0
    agg = SearchResultAggregator(GPUResourceManager())
    cfg = SearchConfig(k=a.k, search_params={"nprobe": a.n_probes}, exchange="rccl")
    r = agg.perform_distributed_search(q, indexes, cfg)  # warm (communicators, threads)
    reps = max(3, a.steps // 4)
    t0 = time.perf_counter()
    for _ in range(reps):
        r = agg.perform_distributed_search(q, indexes, cfg)
    t = (time.perf_counter() - t0) / reps
    line = {"devices": G, "rows_per_gpu": [e - b for b, e in shards], "rows_total": shards[-1][1], "queries": q.shape[0],
            "k": a.k,
            "n_probes": a.n_probes, "qps_full_corpus": round(q.shape[0] / t, 1),
            "shard_searches_per_s": round(q.shape[0] * G / t, 1), "ms_per_batch": round(t * 1e3, 3),
            "shards_built_here": len(todo), "shards_build_s": round(t_build, 3),
            "path": "SearchResultAggregator (one thread per GPU) -> mivs.comm.LocalComm RCCL all-gather + K7; "
                    "results copied to host as the reference's contract returns them"}
    if ref_ids is not None:
        line["final_ids_equal_main_search"] = bool(np.array_equal(r.final_indices, np.asarray(ref_ids)))
    rl(f"[single-process] {G} GPU(s), {shards[-1][1]} rows: {q.shape[0] / t:,.0f} QPS through the aggregator + RCCL merge"
       + (f"; ids equal to the per-rank run: {line['final_ids_equal_main_search']}" if ref_ids is not None
          else ""))
    for ix in extra.values():
        ix.close()
    torch.cuda.empty_cache()
    return line


def corpus_shards(a, world):
    """[(start, end)] row range of each rank's shard: --rows per rank (weak scaling), or --rows-total split with the
    reference's 'even' rule (strong scaling)."""
    if a.rows_total > 0:
        from gpu_resource_manager import even_split

        return even_split(a.rows_total, world)
    return [(r * a.rows, (r + 1) * a.rows) for r in range(world)]


def run_with_watchdog(fn, timeout_s):
    """fn() on a daemon thread: (result, error, hung). A hung thread is abandoned (the caller must then leave
    with os._exit, since the interpreter's teardown would wait for a thread stuck in a collective)."""
    box = {}

    def _run():
        try:
            box["r"] = fn()
        except Exception as e:  # reported by the caller
            box["e"] = e

    th = threading.Thread(target=_run, daemon=True)
    th.start()
    th.join(timeout=timeout_s)
    if th.is_alive():
        return None, None, True
    return box.get("r"), box.get("e"), False


EXIT_HUNG = 3  # a side line hung (a stuck collective): the JSON line is printed, the exit status says so


def free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def run_child(cmd, env, timeout_s, is_result=lambda s: s.startswith("{") and '"metric"' in s):
    """Start `cmd` in its own session, forward its stdout lines to stderr except the result line, and return
    (exit status, result line or None). The deadline runs from the start: stdout is read on a helper thread, so a
    child that hangs with stdout open (a rank stuck in a collective keeps torch.distributed.run alive) is killed --
    its whole process group -- when the deadline passes, and the status is then 124."""
    import subprocess

    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, env=env, text=True, start_new_session=True)
    box = {"line": None}

    def _read():
        for ln in p.stdout:
            s = ln.strip()
            if is_result(s):
                box["line"] = s
            elif s:
                print(s, file=sys.stderr, flush=True)

    th = threading.Thread(target=_read, daemon=True)
    th.start()
    try:
        rc = p.wait(timeout=timeout_s)
    except subprocess.TimeoutExpired:
        try:
            os.killpg(p.pid, 9)
        except ProcessLookupError:
            pass
        p.wait()
        rc = 124
    th.join(timeout=10)
    return rc, box["line"]


def launcher_argv(a, argv, port, ids_out):
    """The child command for `bench.py --gpus N` (N > 1) started without WORLD_SIZE: N ranks, one per GPU,
    under torch.distributed.run on this node (the same command the driver may use itself); rank 0 writes the
    merged ids of the timed search to `ids_out` for the one-process check."""
    fwd = [v for v in argv if v != "--launcher-dry-run"]
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + fwd + \
        ["--single-process", "0", "--ids-out", ids_out]


def self_launch(a, argv):
    """`python bench.py --gpus N` with N > 1 and no torch.distributed environment: start the N rank processes
    as ONE child (torch.distributed.run) before anything in this process touches a GPU, forward their stderr,
    take rank 0's JSON line, then -- the ranks gone and their HBM free -- run the reference's one-process shape
    (single_process_aggregator: every shard on its own device in this process, aggregator threads + the RCCL
    merge of mivs.comm.LocalComm) over the same N devices and check its final ids against the ranks' merged
    ids. Prints one JSON line and exits with the ranks' status (EXIT_HUNG if the one-process line hung)."""
    import tempfile

    tmpd = tempfile.mkdtemp(prefix="mivs_bench_")
    ids_out = os.path.join(tmpd, "merged_ids.npy")
    port = free_port()
    cmd = launcher_argv(a, argv, port, ids_out)
    if a.launcher_dry_run:
        print(json.dumps({"launcher": {"argv": cmd, "gpus": a.gpus}}), flush=True)
        return 0
    print(f"[launcher] {a.gpus} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    t0 = time.perf_counter()
    rc, line = run_child(cmd, env, a.launch_timeout)
    if line is None:
        print(f"[launcher] the ranks exited with {rc} and no result line", file=sys.stderr, flush=True)
        return rc or 1
    out = json.loads(line)
    out["launcher"] = {"mode": "bench.py started its ranks (torch.distributed.run child)", "ranks_rc": rc,
                       "ranks_wall_s": round(time.perf_counter() - t0, 2)}
    hung = False
    if rc == 0 and a.single_process and os.path.exists(ids_out):
        ref = np.load(ids_out, allow_pickle=False)

        def _side():
            import mivs
            from mivs import ops

            mivs.load()
            torch.cuda.set_device(0)
            q = ops.synth_mixture(a.queries, a.dim, SEED, n_centers=a.centers, sigma=a.sigma,
                                  row_begin=QUERY_ROW_BASE, device=0)
            return single_process_side_line(a, q, ref, lambda *m: log(0, *m), range(a.gpus))

        single, err, hung = run_with_watchdog(_side, a.single_process_timeout)
        if hung:
            single = {"error": f"did not finish within {a.single_process_timeout} s (abandoned)"}
        elif err is not None:
            single = {"error": repr(err)}
        out["single_process_aggregator"] = single
    print(json.dumps(out), flush=True)
    if a.json_out:
        with open(a.json_out, "w") as f:
            f.write(json.dumps(out) + "\n")
    try:
        os.remove(ids_out)
        os.rmdir(tmpd)
    except OSError:
        pass
    if hung:
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(EXIT_HUNG)
    return rc


PEAK_LDS_B128_LOOKUPS = 256 * 2.4e9 * 64  # ds_read_b128: 256 B/clk/CU = 64 fp32 LUT entries / clk / CU


def pq_lut16_leg(idx, x, q, gt, ng, k, kc, n_probes, start, world, dev):
    """The same plain and refined PQ searches with SearchParams(lut_dtype=float16) (cuVS's half-precision LUT,
    opt-in: the headline PQ numbers above stay fp32). A ds_read_b128 carries 8 fp16 entries, so its LDS peak
    is twice the fp32 one."""
    from mivs import _native
    from mivs.distributed import merge_across_ranks
    from mivs.neighbors import ivf_pq, refine

    sp = ivf_pq.SearchParams(n_probes=n_probes, lut_dtype=np.float16)
    reps = 5

    def plain():
        dd, ii = ivf_pq.search(sp, idx, q, k)
        ii = ii + start if start else ii
        return merge_across_ranks(dd, ii, k) if world > 1 else (dd, ii)

    def refined():
        _, cand = ivf_pq.search(sp, idx, q, kc)
        dd, ii = refine(x, q, cand, k)
        ii = ii + start if start else ii
        return merge_across_ranks(dd, ii, k) if world > 1 else (dd, ii)

    Q = q.shape[0]
    plain()
    _native.set_profiling(True)
    idx.profile_collect()
    sync_all(world)
    t0 = time.perf_counter()
    for _ in range(reps):
        _, ids = plain()
    torch.cuda.synchronize()
    t_plain = max_over_ranks(time.perf_counter() - t0, world, dev) / reps
    pr = idx.profile_collect()
    _native.set_profiling(False)
    refined()
    sync_all(world)
    t0 = time.perf_counter()
    for _ in range(reps):
        _, rids = refined()
    torch.cuda.synchronize()
    t_ref = max_over_ranks(time.perf_counter() - t0, world, dev) / reps
    return {"qps_pq": round(Q / t_plain, 1), "recall_at_10_pq": round(recall_at_k(ids[:ng].cpu().numpy(), gt), 4),
            "qps_pq_refined": round(Q / t_ref, 1),
            "recall_at_10_pq_refined": round(recall_at_k(rids[:ng].cpu().numpy(), gt), 4),
            "scan_ms": pr["scan_ms"] / max(pr["n_calls"], 1)}


def pq_side_line(a, rl, rank=0, world=1, dev=None):
    """BASELINE configs[4]: IVF-PQ over 12.5M x 768 fp16 rows PER RANK (100M over 8 GPUs), n_lists 4096,
    pq_dim 96, pq_bits 8 (improved_multi_gpu_rag.py:131-137), the same query batch shape; plain PQ at
    n_probes 10 and PQ + exact re-ranking of 12 k candidates (cuvs.neighbors.refine) -- the fastest point of the
    n_probes x candidates sweep that reaches recall@10 >= 0.95 on this mixture with a margin. With N ranks every rank builds its own shard (rows
    rank*n..), and one step = each rank's search (+ refine) and the RCCL all-gather + K7 merge of the
    per-shard top-k (mivs.distributed.merge_across_ranks), timed between barriers, max over ranks. The
    scan's roofline: one fp32 LUT entry read from LDS per (probed row, subspace, query), against the
    ds_read_b128 rate."""
    from mivs import _native, ops
    from mivs.distributed import merge_across_ranks
    from mivs.neighbors import brute_force, ivf_pq, refine

    dev = torch.cuda.current_device() if dev is None else dev
    # operating point (round 4, profiles/r04_ivf_pq_sweep.log): the refined recall is set by the candidate count, not by
    # n_probes in 10..16 (the coarse recall is >= 0.99 there), so the fastest sweep point with a margin over recall 0.95:
    # n_probes 10, 12 x k = 120 candidates (recall 0.976; 100 candidates give 0.952)
    n, d, Q, k, pq_dim, n_lists, n_probes, ratio = a.pq_rows, a.dim, a.queries, a.k, 96, 4096, 10, 12
    start = rank * n
    x = ops.synth_mixture(n, d, SEED + 11, n_centers=a.centers, sigma=a.sigma, row_begin=start, device=dev).half()
    torch.cuda.empty_cache()
    q = ops.synth_mixture(Q, d, SEED + 11, n_centers=a.centers, sigma=a.sigma, row_begin=QUERY_ROW_BASE, device=dev)
    sync_all(world)
    if a.build_warmup:  # (as for the IVF-Flat build: an untimed first build warms the allocator)
        ivf_pq.build(ivf_pq.IndexParams(n_lists=n_lists, pq_dim=pq_dim, pq_bits=8), x).close()
        torch.cuda.synchronize()
        sync_all(world)
    _native.set_profiling(True)
    t0 = time.perf_counter()
    idx = ivf_pq.build(ivf_pq.IndexParams(n_lists=n_lists, pq_dim=pq_dim, pq_bits=8), x)
    torch.cuda.synchronize()
    t_build = max_over_ranks(time.perf_counter() - t0, world, dev)
    phases = idx.build_phases()
    _native.set_profiling(False)
    ng = min(1000, Q)
    xf = x.float()
    bf = brute_force.build(xf, ids_offset=start)
    gd, gi = brute_force.search(bf, q[:ng], max(17, k))
    gd, gi = gd[:, :k].contiguous(), gi[:, :k].contiguous()
    bf.close()
    del bf, xf
    torch.cuda.empty_cache()
    if world > 1:
        gd, gi = merge_across_ranks(gd, gi, k)
    gt = gi.cpu().numpy()
    sp = ivf_pq.SearchParams(n_probes=n_probes)
    reps = 5

    def plain():
        dd, ii = ivf_pq.search(sp, idx, q, k)
        ii = ii + start if start else ii  # (the shard's row numbers -> global ids)
        return merge_across_ranks(dd, ii, k) if world > 1 else (dd, ii)

    kc = ratio * k

    def refined():
        _, cand = ivf_pq.search(sp, idx, q, kc)
        dd, ii = refine(x, q, cand, k)
        ii = ii + start if start else ii
        return merge_across_ranks(dd, ii, k) if world > 1 else (dd, ii)

    plain()
    _native.set_profiling(True)
    idx.profile_collect()
    sync_all(world)
    t0 = time.perf_counter()
    for _ in range(reps):
        _, ids = plain()
    torch.cuda.synchronize()
    t_plain = max_over_ranks(time.perf_counter() - t0, world, dev) / reps
    pr = idx.profile_collect()
    _native.set_profiling(False)
    rec_plain = recall_at_k(ids[:ng].cpu().numpy(), gt)
    refined()
    sync_all(world)
    t0 = time.perf_counter()
    for _ in range(reps):
        _, rids = refined()
    torch.cuda.synchronize()
    t_ref = max_over_ranks(time.perf_counter() - t0, world, dev) / reps
    rec_ref = recall_at_k(rids[:ng].cpu().numpy(), gt)
    lut16 = pq_lut16_leg(idx, x, q, gt, ng, k, kc, n_probes, start, world, dev) if a.pq_lut16 else None
    probes = torch.empty((Q, n_probes), dtype=torch.int32, device=dev)
    ivf_pq.search(sp, idx, q, k, probes_out=probes)
    rows = int(idx.list_sizes.cpu()[probes.long().cpu()].sum())
    scan_ms = pr["scan_ms"] / max(pr["n_calls"], 1)
    lookups = float(rows) * pq_dim
    ach = lookups / (scan_ms * 1e-3)
    line = {"rows_per_gpu": n, "rows_total": n * world, "n_gpus": world, "dim": d, "dtype_in": "fp16",
            "n_lists": n_lists, "pq_dim": pq_dim, "pq_bits": 8, "queries": Q, "k": k, "n_probes": n_probes,
            "build_s": round(t_build, 3), "build_vectors_per_s": round(n * world / t_build, 1),
            "build_phases_s": phases,
            "qps_pq": round(Q / t_plain, 1), "recall_at_10_pq": round(rec_plain, 4),
            "qps_pq_refined": round(Q / t_ref, 1), "recall_at_10_pq_refined": round(rec_ref, 4),
            "shard_searches_per_s_refined": round(Q * world / t_ref, 1),
            "refine": f"{kc} PQ candidates re-ranked exactly against the fp16 rows (mivs.neighbors.refine, K14)"
                      + ("; per-shard top-k merged across ranks (RCCL all-gather + K7) inside the step"
                         if world > 1 else ""),
            "scan_kernel": "mivs::k_pq_scan_rt (K9r: 16-query tiles per list, code-major LUT rows in LDS)",
            "roofline": {"bound": "lds", "achieved": round(ach / 1e9, 1), "peak": round(PEAK_LDS_B128_LOOKUPS / 1e9, 1),
                         "unit": "G LUT entries/s", "frac": round(ach / PEAK_LDS_B128_LOOKUPS, 4),
                         "launch_ms": round(scan_ms, 4), "lut_entries_per_launch": lookups, "rows_scanned": rows}}
    if lut16 is not None:
        ms16 = lut16.pop("scan_ms")
        a16 = lookups / (ms16 * 1e-3)
        lut16["roofline"] = {"bound": "lds", "achieved": round(a16 / 1e9, 1),
                             "peak": round(2 * PEAK_LDS_B128_LOOKUPS / 1e9, 1), "unit": "G LUT entries/s",
                             "frac": round(a16 / (2 * PEAK_LDS_B128_LOOKUPS), 4), "launch_ms": round(ms16, 4)}
        line["lut_fp16"] = lut16
        rl(f"[pq] lut_dtype float16 (opt-in): {lut16['qps_pq']:,.0f} QPS recall {lut16['recall_at_10_pq']:.3f}; "
           f"refined {lut16['qps_pq_refined']:,.0f} QPS recall {lut16['recall_at_10_pq_refined']:.3f}; "
           f"K9r {ms16:.3f} ms")
    rl(f"[pq] {n * world} x {d} fp16 on {world} GPU(s), build {n * world / t_build / 1e6:.2f} M vec/s {phases}; "
       f"n_probes {n_probes}: {Q / t_plain:,.0f} QPS recall {rec_plain:.3f}; refined x{ratio}: {Q / t_ref:,.0f} QPS "
       f"recall {rec_ref:.3f}")
    idx.close()
    del x, q, idx, ids, rids
    torch.cuda.empty_cache()
    return line


def main():
    a = parse()
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        # one process per GPU is how the scan scales: start the ranks as a child (never exec: nothing here has
        # touched a GPU yet, and the child is a new process either way)
        return self_launch(a, sys.argv[1:])
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        rl0 = f"[bench] --gpus {a.gpus} but WORLD_SIZE {world}: measuring the {world} launched ranks"
        print(rl0, file=sys.stderr, flush=True) if rank == 0 else None
    torch.cuda.set_device(local)
    dev = torch.device(f"cuda:{local}")
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    dist_info = {"backend": dist.get_backend() if world > 1 else None,
                 "world_size": dist.get_world_size() if world > 1 else 1,
                 "launched_by": "torch.distributed.run" if "TORCHELASTIC_RUN_ID" in os.environ or world > 1
                 else "single process"}
    import mivs
    from mivs import _native, ops
    from mivs.distributed import merge_across_ranks
    from mivs.neighbors import brute_force, ivf_flat, streaming

    mivs.load()
    rl = lambda *m: log(rank, *m)  # noqa: E731
    shards = corpus_shards(a, world)
    start, end = shards[rank]
    n, d, Q, k = end - start, a.dim, a.queries, a.k
    rows_total = shards[-1][1]
    strong = a.rows_total > 0

    # ---- data: generated on the device (no PCIe in any timed region) ----
    x = ops.synth_mixture(n, d, SEED, n_centers=a.centers, sigma=a.sigma, row_begin=start, device=local)
    q = ops.synth_mixture(Q, d, SEED, n_centers=a.centers, sigma=a.sigma, row_begin=QUERY_ROW_BASE, device=local)
    sync_all(world)

    # ---- build (wall clock, data resident) ----
    params = ivf_flat.IndexParams(n_lists=a.n_lists, kmeans_n_iters=a.kmeans_iters,
                                  kmeans_trainset_fraction=a.trainset_fraction)
    # 1. the cold build: the first in the process, as each of the reference's builds is (one per GPU thread,
    # index_building_coordinator.py:370-420): its ~54 GB of fresh device allocations are part of its time
    _native.set_block_cache_limit(0)
    sync_all(world)
    _native.set_profiling(True)  # (the build's phase clocks: one stream sync per phase)
    t0 = time.perf_counter()
    idx_cold = ivf_flat.build(params, x, ids_offset=start)
    torch.cuda.synchronize()
    t_build_cold = max_over_ranks(time.perf_counter() - t0, world, dev)
    _native.set_profiling(False)
    build_cold_phases = idx_cold.build_phases()
    idx_cold.close()
    del idx_cold
    rl(f"[build] cold (first in the process): {rows_total} rows in {t_build_cold:.2f} s -> "
       f"{rows_total / t_build_cold / 1e6:.2f} M vec/s {build_cold_phases}")
    # 2. warm: the engine's block cache (opt-in) keeps the released blocks, so a process that rebuilds reuses them
    if a.block_cache_gb > 0:
        _native.set_block_cache_limit(int(a.block_cache_gb * (1 << 30)), local)
    sync_all(world)
    for _ in range(a.build_warmup):
        ivf_flat.build(params, x, ids_offset=start).close()
        torch.cuda.synchronize()
        sync_all(world)
    _native.set_profiling(True)
    t0 = time.perf_counter()
    idx = ivf_flat.build(params, x, ids_offset=start)
    torch.cuda.synchronize()
    t_build = max_over_ranks(time.perf_counter() - t0, world, dev)
    _native.set_profiling(False)
    build_phases = idx.build_phases()
    build_roof = build_roofline(idx.build_kernels(), t_build)
    build_vps = rows_total / t_build
    index_mem = idx.memory()  # one fp32 copy (64-B row blocks) + the fp16 and fp8 copies, all built in build()
    sizes = idx.list_sizes.numpy()
    rl(f"[build] {rows_total} rows in {t_build:.2f} s -> {build_vps / 1e6:.2f} M vec/s; lists min/med/max "
       f"{sizes.min()}/{int(np.median(sizes))}/{sizes.max()}")

    sp = ivf_flat.SearchParams(n_probes=a.n_probes)

    def step(qq, params=None):
        dd, ii = ivf_flat.search(params or sp, idx, qq, k)
        if world > 1:
            dd, ii = merge_across_ranks(dd, ii, k)
        return dd, ii

    for _ in range(a.warmup):
        step(q)
    _native.set_profiling(True)
    idx.profile_collect()  # drop warmup records
    torch.cuda.synchronize()
    sync_all(world)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        res_d, res_i = step(q)
    torch.cuda.synchronize()
    t_local = time.perf_counter() - t0
    sync_all(world)
    t_steps = max_over_ranks(t_local, world, dev)
    prof = idx.profile_collect()
    _native.set_profiling(False)
    stats = idx.last_search_stats()
    ms_per_step = t_steps / a.steps * 1e3
    qps_full = Q * a.steps / t_steps
    value = qps_full  # full-corpus QPS: Q queries answered over every shard (searched + merged) per second
    rl(f"[search] {a.steps} steps x {Q} queries: {ms_per_step:.3f} ms/step -> {qps_full:,.0f} QPS (full corpus)")
    ranks_diag = None
    if world > 1:  # what a flat 1 -> 8 curve would need to be read: every rank's own step time and the step's parts
        from mivs.distributed import per_rank_values, timed_sharded_step

        per_rank = per_rank_values(t_local / a.steps * 1e3, dev)
        parts = []
        for _ in range(max(3, a.steps // 4)):
            sync_all(world)
            _, t_parts = timed_sharded_step(lambda: ivf_flat.search(sp, idx, q, k), k)
            parts.append(t_parts)
        mean = {key: sum(p_[key] for p_ in parts) / len(parts) for key in parts[0]}
        ranks_diag = {"world_size": dist.get_world_size(), "backend": dist.get_backend(),
                      "rccl_version": ".".join(str(v) for v in torch.cuda.nccl.version()),
                      "per_rank_ms": [round(v, 4) for v in per_rank],
                      "per_rank_search_ms": [round(v, 4) for v in per_rank_values(mean["search_ms"], dev)],
                      "allgather_ms": [round(v, 4) for v in per_rank_values(mean["allgather_ms"], dev)],
                      "merge_ms": [round(v, 4) for v in per_rank_values(mean["merge_ms"], dev)],
                      "allgather_bytes_per_rank": Q * k * 12,
                      "timing": f"per_rank_ms: each rank's own clock over the {a.steps} timed steps; the parts: "
                                f"hipEvents on the search stream over {len(parts)} extra steps (search | RCCL "
                                "all-gather of the [Q, k] (distance, id) tiles | K7 merge), mean per rank"}
        rl(f"[ranks] {ranks_diag}")

    # ---- PCIe-inclusive rate (not `value`): queries start in pinned host memory, results return to host ----
    q_host = q.cpu().pin_memory()
    io_steps = max(2, a.steps // 4)
    sync_all(world)
    t0 = time.perf_counter()
    for _ in range(io_steps):
        hd, hi = step(q_host.to(dev, non_blocking=True))
        hd, hi = hd.cpu(), hi.cpu()
    t_io = max_over_ranks(time.perf_counter() - t0, world, dev) / io_steps
    qps_host_io = Q / t_io
    rl(f"[search] with host queries/results over PCIe: {qps_host_io:,.0f} QPS (full corpus)")
    # the same, pipelined (streaming.search_host: H2D of batch b+1 and D2H of batch b-1 overlap the
    # search of batch b); io_steps batches of Q host queries, per-shard results (no cross-rank merge)
    st_batches = max(4, a.steps // 2)
    q_many = q_host.repeat(st_batches, 1).pin_memory()
    # two warm calls (the first uses of the side streams and of the pinned batches cost ~10-30 ms
    # once per process); the timed call reuses the pinned outputs
    st_d, st_i = streaming.search_host(idx, q_many, k, sp, batch_size=Q)
    streaming.search_host(idx, q_many, k, sp, batch_size=Q, distances=st_d, neighbors=st_i)
    sync_all(world)
    t0 = time.perf_counter()
    streaming.search_host(idx, q_many, k, sp, batch_size=Q, distances=st_d, neighbors=st_i)
    t_st = max_over_ranks(time.perf_counter() - t0, world, dev)
    qps_host_io_streamed = Q * st_batches * world / t_st
    del q_many, st_d, st_i
    rl(f"[search] host queries, pipelined over 3 streams: {qps_host_io_streamed:,.0f} QPS (per-shard searches)")

    # ---- recall@10 vs exact ground truth (brute force on the same engine, merged over shards) ----
    ng = min(a.gt_queries, Q)
    bf = brute_force.build(x, ids_offset=start)
    # exact top-k via k_gt > 16 (a different scan instantiation than the timed fine scan, so the
    # rocprof per-kernel average of the timed kernel is not mixed with this launch); the first k
    # of the (key, id)-ordered top-k_gt are exactly the top-k
    k_gt = max(17, k)
    gd, gi = brute_force.search(bf, q[:ng], k_gt)
    gd, gi = gd[:, :k].contiguous(), gi[:, :k].contiguous()
    bf.close()
    del bf
    torch.cuda.empty_cache()
    if world > 1:
        gd, gi = merge_across_ranks(gd, gi, k)
    gt = gi.cpu().numpy()
    found = res_i[:ng].cpu().numpy()
    rec = recall_at_k(found, gt)
    rl(f"[recall] recall@{k} = {rec:.4f} over {ng} queries (n_probes={a.n_probes})")

    sweep = []
    for s in [int(v) for v in a.sweep.split(",") if v.strip()]:
        spp = ivf_flat.SearchParams(n_probes=s)
        step(q, spp)
        sync_all(world)
        t0 = time.perf_counter()
        for _ in range(max(3, a.steps // 4)):
            sd, si = step(q, spp)
        torch.cuda.synchronize()
        ts = max_over_ranks(time.perf_counter() - t0, world, dev) / max(3, a.steps // 4)
        sr = recall_at_k(si[:ng].cpu().numpy(), gt)
        sweep.append({"n_probes": s, "qps_full_corpus": Q / ts, "recall_at_10": sr})
        rl(f"[sweep] n_probes={s}: {Q / ts:,.0f} QPS recall@{k}={sr:.4f}")

    # ---- roofline of the fine-scan kernel (algorithmic work per launch / avg launch time) ----
    scan_ms = prof["scan_ms"] / max(prof["n_calls"], 1)
    pf = bool(stats.get("prefilter"))
    dp = (d + 63) // 64 * 64
    flops = 2.0 * d * stats["scanned_rows"]
    # SURVEY §8(d) de-duplicated per-tile bytes: every query tile streams the rows of its list once
    # (the pre-filter scan K10 reads the fp16 copy: 2 B per padded dim; the exact scans fp32)
    row_bytes = dp * 2 if pf else d * 4
    bytes_tile = float(stats["streamed_groups"]) * 32 * row_bytes
    # compulsory bytes: every probed list once (what a kernel that shares each row among all of its
    # queries must read from HBM); the K10 tiles of one list run together on one XCD, so the per-tile
    # re-reads are L2 hits (rocprof FETCH_SIZE, profiles/r01_pf_pmc*.json)
    bytes_alg = float(stats.get("unique_groups") or stats["streamed_groups"]) * 32 * row_bytes if pf else bytes_tile
    tflops = flops / (scan_ms * 1e-3) / 1e12
    gbs = bytes_alg / (scan_ms * 1e-3) / 1e9
    metric_tag = "L2"
    kname = {13: f"mivs::k_rs_scan<{metric_tag}> (K13 row-stationary fp16 pre-filter)",
             10: f"mivs::k_pf_scan<{metric_tag}> (K10 fp16 pre-filter)",
             12: f"mivs::k_pf_scan_r<{metric_tag}> (K12)",
             31: f"mivs::k_scan_wide<{stats['kcap']},{metric_tag}> (K3w exact fp32)",
             3: f"mivs::k_scan<{stats['kcap']},{metric_tag}> (K3 exact fp32)"}.get(stats.get("scan_kernel"), "?")
    peak_mfma = PEAK_F16_MFMA_TFS if pf else PEAK_F32_MFMA_TFS
    cfg_key = f"ivf_flat_n{n}_d{d}_q{Q}_l{a.n_lists}_p{a.n_probes}_k{k}_t{stats['query_tile']}" + ("_pf" if pf else "")
    traffic, traffic_src = load_traffic(cfg_key)
    # bound: whichever peak the launch's work needs longer for -- the MFMA pipe (fp16 for K10, fp32
    # for the exact scans) for the algorithmic flops, or HBM for the algorithmic bytes
    t_mfma = flops / (peak_mfma * 1e12)
    t_hbm = bytes_alg / (PEAK_HBM_GBS * 1e9)
    if t_mfma >= t_hbm:
        roof = {"bound": "mfma", "achieved": round(tflops, 2), "peak": peak_mfma, "unit": "TFLOP/s",
                "frac": round(tflops / peak_mfma, 4)}
    else:
        roof = {"bound": "hbm", "achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                "frac": round(gbs / PEAK_HBM_GBS, 4)}
    roof["traffic"] = traffic
    clk, clk_src = load_clock(cfg_key)
    if clk is not None and roof["bound"] == "mfma":
        held = float(clk["clock_mhz_held"])
        roof["clock_mhz_held"] = round(held, 1)
        roof["frac_at_held_clock"] = round(roof["frac"] * MAX_SCLK_MHZ / held, 4)
        roof["clock_source"] = clk_src
    roof.update({"kernel": f"{kname} (fine list scan, {stats['query_tile']}-query tiles)",
                 "launch_ms": round(scan_ms, 4),
                 "algorithmic_flops_per_launch": flops, "algorithmic_bytes_per_launch": bytes_alg,
                 "per_tile_bytes_per_launch": bytes_tile,
                 "achieved_gbs_algorithmic": round(gbs, 1), "achieved_tflops": round(tflops, 2),
                 "mfma_frac": round(tflops / peak_mfma, 4), "hbm_frac_algorithmic": round(gbs / PEAK_HBM_GBS, 4),
                 "per_tile_gbs": round(bytes_tile / (scan_ms * 1e-3) / 1e9, 1),
                 "traffic_gbs": round(traffic / (scan_ms * 1e-3) / 1e9, 1) if traffic else None,
                 "traffic_source": traffic_src, "timing": "hipEvents around each fine-scan launch on the search stream, "
                                                          f"{prof['n_calls']} timed steps"})

    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        try:
            cpu = cpu_baseline(idx, q.cpu().numpy(), gt, a.n_probes, k, a.cpu_seconds, rl,
                               sweep=[int(v) for v in a.cpu_sweep.split(",") if v.strip()], gpu_sweep=sweep)
            rl(f"[cpu] {cpu['value']:.2f} QPS on {cpu['cores']} cores (recall {cpu['recall_at_10']}); matched recall: "
               f"{cpu.get('matched_recall')}")
        except Exception as e:  # the GPU result stands without the CPU column
            rl(f"[cpu] baseline failed: {e!r}")
        if cpu is not None and a.cpu_build_rows > 0:
            try:
                cb = cpu_build_baseline(x, a.n_lists, rows_total, cpu["cores"], min(a.cpu_build_rows, n), rl)
                cpu["build_vectors_per_s"] = cb["build_vectors_per_s"]
                cpu["build"] = cb
            except Exception as e:  # the search column stands without the build column
                rl(f"[cpu-build] baseline failed: {e!r}")

    flat = None
    if rank == 0 and world == 1 and a.flat_rows > 0:
        try:
            flat = flat_side_line(a, q, k, rl)
        except Exception as e:  # the IVF line stands without it
            rl(f"[flat] side line failed: {e!r}")

    large_k = None
    if rank == 0 and world == 1 and a.large_k.strip():
        try:
            large_k = large_k_side_line(a, idx, q, rl, stats["scanned_rows"])
        except Exception as e:  # the IVF line stands without it
            rl(f"[large-k] side line failed: {e!r}")

    batch_sweep = None
    if rank == 0 and world == 1 and a.batch_sweep.strip():
        try:
            batch_sweep = batch_sweep_side_line(a, idx, rl, gt, local)
        except Exception as e:  # the IVF line stands without it
            rl(f"[batch] side line failed: {e!r}")

    latency = None
    if rank == 0 and world == 1 and a.latency.strip():
        try:
            latency = latency_side_line(a, idx, q, rl)
        except Exception as e:  # the IVF line stands without it
            rl(f"[latency] side line failed: {e!r}")

    if a.ids_out and rank == 0:  # (the launcher's one-process check compares against these)
        np.save(a.ids_out, res_i.cpu().numpy())

    single = None
    single_hung = False
    if rank == 0 and world == 1 and a.single_process:
        # on a multi-GPU node this runs the one-process RCCL path (ncclCommInitAll over every local device) at
        # P > 1: a watchdog keeps a hang there from taking the IVF-Flat line with it (and the exit status says so)
        G = torch.cuda.device_count()
        single, err, single_hung = run_with_watchdog(
            lambda: single_process_side_line(a, q, res_i.cpu().numpy() if G == 1 else None, rl, range(G), {0: idx}),
            a.single_process_timeout)
        if single_hung:
            single = {"error": f"did not finish within {a.single_process_timeout} s (abandoned)"}
            rl(f"[single-process] side line did not finish within {a.single_process_timeout} s: abandoned")
        elif err is not None:
            single = {"error": repr(err)}
            rl(f"[single-process] side line failed: {err!r}")

    pq = None
    if single_hung:
        pq = {"skipped": "not run: the one-process RCCL side line hung and holds the devices"}
    elif a.pq_rows > 0:  # every rank: configs[4] is this line at N = 8
        idx.close()
        del x
        torch.cuda.empty_cache()
        try:
            pq = pq_side_line(a, rl, rank, world, local)
        except Exception as e:  # the IVF-Flat line stands without it
            rl(f"[pq] side line failed: {e!r}")
            if world > 1:
                raise  # a rank that left the collective would hang the others

    out = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "QPS",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None,
        "dtype": "f32",  # results are the exact fp32 answer (the fp16 pre-filter only selects candidates)
        "data": f"synthetic: on-device Gaussian mixture ({a.centers} centres, sigma={a.sigma}, L2-normalised), "
                f"seed {SEED}; queries = held-out rows of the same mixture",
        "config": {"workload": (f"IVF-Flat {rows_total / 1e6:g}M x {d} fp32 split over {world} GPU(s)" if strong else
                                f"IVF-Flat {n / 1e6:g}M x {d} fp32 per GPU ({rows_total / 1e6:g}M total)")
                               + f", n_lists={a.n_lists}, "
                               f"n_probes={a.n_probes}, k={k}, batch of {Q} queries",
                   "rows_per_gpu": [e - b for b, e in shards] if strong else n, "rows_total": rows_total, "dim": d,
                   "queries": Q, "n_lists": a.n_lists,
                   "n_probes": a.n_probes, "k": k, "kmeans_n_iters": a.kmeans_iters,
                   "kmeans_trainset_fraction": a.trainset_fraction, "parallelism": f"corpus-shard{world}",
                   "value_definition": "full-corpus QPS: queries answered over the whole corpus (every shard searched "
                                       "and the per-shard top-k merged) per second = queries / step time",
                   "corpus_mode": "fixed corpus split over the ranks (strong scaling)" if strong else
                                  "one shard of --rows per rank (weak scaling)"},
        "shard_searches_per_s": round(qps_full * world, 2),
        "qps_full_corpus": round(qps_full, 2),
        "qps_host_io": round(qps_host_io, 2),
        "qps_host_io_streamed": round(qps_host_io_streamed, 2),
        "recall_at_10": round(rec, 4),
        "build_vectors_per_s": round(build_vps, 1),
        "build_s": round(t_build, 3),
        "build_phases_s": build_phases,
        "build_cold_s": round(t_build_cold, 3),
        "build_cold_vectors_per_s": round(rows_total / t_build_cold, 1),
        "build_cold_phases_s": build_cold_phases,
        "build_note": "build_s: a warm rebuild (after the cold one and --build-warmup untimed builds) with the engine's "
                      f"opt-in block cache at {a.block_cache_gb:g} GB (mivs.set_block_cache_limit; released blocks "
                      "reused instead of fresh page-cleared allocations); build_cold_s: the first build in the "
                      "process, cache off, as each of the reference's builds is",
        "matched_recall": cpu.get("matched_recall") if cpu else matched_recall(sweep, []),
        "build_roofline": build_roof,
        "index_bytes_per_row": round(index_mem["total_bytes"] / max(index_mem["n_rows"], 1), 1),
        "index_memory": index_mem,
        "roofline": roof,
        "cpu_baseline": cpu,
        "search_stats": stats,
        "n_probes_sweep": sweep,
        "flat_bruteforce_1m": flat,
        "large_k": large_k,
        "latency": latency,
        "batch_sweep": batch_sweep,
        "single_process_aggregator": single,
        "ivf_pq_12m5": pq,
        "distributed": dist_info,
        "ranks": ranks_diag,
    }
    if rank == 0:
        line = json.dumps(out)
        print(line, flush=True)
        if a.json_out:
            with open(a.json_out, "w") as f:
                f.write(line + "\n")
    if single_hung:  # a thread is stuck in a collective: leave without the teardown that would wait for it, and
        # say so in the exit status (the line above still carries every measured number)
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(EXIT_HUNG)
    if pq is None:
        idx.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main() or 0)
