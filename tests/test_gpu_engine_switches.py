"""Every engine switch that selects an alternative kernel path gives the SAME bits as
the default path (VERDICT r1 "what's weak" #9: keep an A/B knob only under a bit-exact -m gpu test).

One IVF-Flat index (L2 and IP), one IVF-PQ index and one brute-force index; for each switch the search
is repeated with the variable set and compared bitwise with the default search (which the parity
suites pin to the oracle). Diagnostic switches that only print (MIVS_RS_FLAGS=24, MIVS_PF_FLAGS=32)
must not change results either. Timing-only settings that skip work (MIVS_RS_FLAGS 1/2,
MIVS_PQ_FLAGS, MIVS_PF_FLAGS other than 32) are not result paths and are not listed.
"""
import numpy as np
import pytest
import torch

import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _fresh_settings():
    """the library caches MIVS_FALLBACK_SYNC (read once): re-read it at the start of every test, after the previous
    test's monkeypatch has restored the environment"""
    from mivs import _native

    _native.load()
    _native.reload_settings()
    yield


def _setenv(monkeypatch, k, v):
    from mivs import _native

    monkeypatch.setenv(k, v)
    _native.reload_settings()


def _bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.int32)


def _data(n, d, seed):
    rng = np.random.default_rng(seed)
    c = rng.standard_normal((40, d)).astype(np.float32)
    x = c[rng.integers(0, 40, n)] + 0.35 * rng.standard_normal((n, d)).astype(np.float32)
    x /= np.linalg.norm(x, axis=1, keepdims=True)
    return x.astype(np.float32)


@pytest.fixture(scope="module")
def flat_data():
    x = _data(60_000, 768, 1)
    q = _data(70, 768, 2)
    return x, q


@pytest.fixture(scope="module", params=["sqeuclidean", "inner_product"])
def ivf(request, flat_data, mivs_lib):
    from mivs.neighbors import ivf_flat

    x, q = flat_data
    idx = ivf_flat.build(ivf_flat.IndexParams(n_lists=48, kmeans_n_iters=4, metric=request.param),
                         torch.from_numpy(x).cuda())
    yield idx, request.param
    idx.close()


def _search(idx, q, k=10, n_probes=8):
    from mivs.neighbors import ivf_flat

    d, i = ivf_flat.search(ivf_flat.SearchParams(n_probes=n_probes), idx, torch.from_numpy(q).cuda(), k)
    return d.cpu().numpy(), i.cpu().numpy()


SEARCH_SWITCHES = [
    {"MIVS_PF_ROWSTAT": "0"},                                         # K10 instead of K13
    {"MIVS_RS_PRE_DIV": "1"},
    {"MIVS_RS_PRE_DIV": "16"},
    {"MIVS_RS_PRE_F8": "0"},                                          # pre-pass: the fp16 sample (round 2)
    {"MIVS_RS_PRE_DIV": "1"},                                         # fp8 nomination over the whole list
    {"MIVS_RS_FLAGS": "24"},                                          # K13 clocks (stderr only)
    {"MIVS_RS_WAVE_CAP": "2"},                                        # K13 streams overflow: the fallback
    {"MIVS_PF_ROWSTAT": "0", "MIVS_PF_FLAGS": "32"},                  # K10 phase clocks (stderr only)
    {"MIVS_RS_BUCKET_1P": "0"},                                       # K13 bucketing: two-pass CSR runs
    {"MIVS_RS_QCAP": "4"},                                            # one-pass runs overflow: the fallback
    {"MIVS_FALLBACK_SYNC": "1"},                                      # fallback sized on the host (round 4)
    {"MIVS_FALLBACK_SYNC": "1", "MIVS_RS_QCAP": "4"},
    {"MIVS_FALLBACK_SYNC": "1", "MIVS_RS_WAVE_CAP": "2"},
    {"MIVS_PF_RAW_LISTS": "0"},                                       # pre-pass slots merged in K10 (round 6)
]


@pytest.mark.parametrize("env", SEARCH_SWITCHES, ids=lambda e: ",".join(f"{k}={v}" for k, v in e.items()))
def test_ivf_search_switch_same_bits(ivf, flat_data, monkeypatch, env):
    idx, metric = ivf
    _, q = flat_data
    d0, i0 = _search(idx, q)
    for kk, v in env.items():
        _setenv(monkeypatch, kk, v)
    d1, i1 = _search(idx, q)
    np.testing.assert_array_equal(i1, i0)
    np.testing.assert_array_equal(_bits(d1), _bits(d0))


def test_ivf_one_pass_bucketing_same_candidates(ivf, flat_data, monkeypatch):
    """K13's one-pass bucketing (fixed-capacity runs per query) and the two-pass CSR form hold the same candidates"""
    idx, _ = ivf
    _, q = flat_data
    d0, i0 = _search(idx, q)
    st0 = idx.last_search_stats()
    monkeypatch.setenv("MIVS_RS_BUCKET_1P", "0")
    d1, i1 = _search(idx, q)
    st1 = idx.last_search_stats()
    np.testing.assert_array_equal(i1, i0)
    np.testing.assert_array_equal(_bits(d1), _bits(d0))
    assert st0["candidates"] == st1["candidates"] > 0
    assert st0["overflow_queries"] == st1["overflow_queries"]  # (this small shape has unproven windows either way)


@pytest.mark.parametrize("env", [{}, {"MIVS_RS_QCAP": "4"}, {"MIVS_RS_WAVE_CAP": "2"}],
                         ids=["default", "qcap4", "lost"])
def test_device_fallback_stats_and_bits(ivf, flat_data, monkeypatch, env):
    """the exact fallback of K13's unproven queries sized on the device (no host round trip) against the host-sized
    one: the same bits; few, most and all queries unproven. The device path's stats (read back by last_search_stats)
    count K13's unproven queries and windows; the host path sends those queries through K10 first and adds its
    unproven queries and windows, so its counts are at least as large"""
    idx, _ = ivf
    _, q = flat_data
    for kk, v in env.items():
        _setenv(monkeypatch, kk, v)
    d0, i0 = _search(idx, q)
    st0 = idx.last_search_stats()
    _setenv(monkeypatch, "MIVS_FALLBACK_SYNC", "1")
    d1, i1 = _search(idx, q)
    st1 = idx.last_search_stats()
    np.testing.assert_array_equal(i0, i1)
    np.testing.assert_array_equal(_bits(d0), _bits(d1))
    assert st0["overflow_queries"] <= st1["overflow_queries"] and st0["window_candidates"] <= st1["window_candidates"]
    if env:
        assert st0["overflow_queries"] > q.shape[0] // 2, st0


def test_ivf_default_matches_oracle(ivf, flat_data):
    idx, metric = ivf
    x, q = flat_data
    d, i = _search(idx, q)
    od, oi, _ = O.ivf_search(x, idx.centers.cpu().numpy(), idx.list_sizes.numpy(), idx.list_ids().cpu().numpy(), q,
                             8, 10, metric=metric)
    np.testing.assert_array_equal(i, oi)
    np.testing.assert_array_equal(_bits(d), _bits(od))


@pytest.mark.parametrize("k,env", [(10, {"MIVS_SCAN_WIDE": "0"}), (10, {"MIVS_SCAN_WIDE_WAVES": "8"}),
                                   (100, {"MIVS_SCAN_WAVES": "8"})])
def test_exact_scan_switch_same_bits(ivf, flat_data, monkeypatch, k, env):
    """the exact fp32 scans: K3 vs K3w, K3w with 8 waves, the DUMP scan (k > 64) with 8 waves"""
    idx, _ = ivf
    _, q = flat_data
    idx.set_prefilter(False)
    try:
        d0, i0 = _search(idx, q, k=k)
        for kk, v in env.items():
            _setenv(monkeypatch, kk, v)
        d1, i1 = _search(idx, q, k=k)
    finally:
        idx.set_prefilter(True)
    np.testing.assert_array_equal(i1, i0)
    np.testing.assert_array_equal(_bits(d1), _bits(d0))


def test_build_assign_switches_same_index(flat_data, mivs_lib, monkeypatch):
    """the build's assign through K13a (default), through K12 (MIVS_PF_ASSIGN_RS=0) and in fp32 (MIVS_PF_ASSIGN=0):
    the same centroids, list sizes and list order"""
    from mivs.neighbors import ivf_flat

    x, _ = flat_data
    xt = torch.from_numpy(x).cuda()
    p = ivf_flat.IndexParams(n_lists=48, kmeans_n_iters=4)
    ref = ivf_flat.build(p, xt)
    for env in ({"MIVS_PF_ASSIGN_RS": "0"}, {"MIVS_PF_ASSIGN": "0"}):
        for kk, v in env.items():
            _setenv(monkeypatch, kk, v)
        other = ivf_flat.build(p, xt)
        for kk in env:
            monkeypatch.delenv(kk)
        np.testing.assert_array_equal(_bits(other.centers.cpu().numpy()), _bits(ref.centers.cpu().numpy()))
        np.testing.assert_array_equal(other.list_sizes.numpy(), ref.list_sizes.numpy())
        np.testing.assert_array_equal(other.list_ids().cpu().numpy(), ref.list_ids().cpu().numpy())
        other.close()
    ref.close()


@pytest.mark.parametrize("d,dup", [(128, "exact"), (768, "exact"), (768, "near")])
def test_build_assign_k13a_near_ties(mivs_lib, d, dup):
    """K13a's rows it cannot prove (a second centroid inside the refine window) go through K12 + the window
    refine: centroids 32..63 duplicate 0..31 exactly (every row a tie, resolved to the lower id) or up to a
    1e-6 nudge (inside the window, decided by the exact fp32 keys); labels equal the oracle's assign"""
    from mivs.cluster import kmeans

    x = _data(20_000, d, 7)
    rng = np.random.default_rng(3)
    c = x[rng.choice(x.shape[0], 64, replace=False)].copy()
    c[32:] = c[:32]
    if dup == "near":
        c[32:] += (1e-6 * rng.standard_normal((32, d))).astype(np.float32)
    _, lab = kmeans.build_steps(torch.from_numpy(x).cuda(), torch.from_numpy(c).cuda(), None, 0, 1, 1,
                                balance=False, return_labels=True)
    exp = O.kmeans_assign(x, c)
    if dup == "exact":
        assert exp.max() < 32
    np.testing.assert_array_equal(lab.cpu().numpy(), exp)


def test_prefilter_default_switch(flat_data, mivs_lib, monkeypatch):
    """MIVS_PREFILTER=0: indexes start with the exact scan; the answer is the same"""
    from mivs.neighbors import ivf_flat

    x, q = flat_data
    xt = torch.from_numpy(x).cuda()
    p = ivf_flat.IndexParams(n_lists=48, kmeans_n_iters=4)
    a = ivf_flat.build(p, xt)
    monkeypatch.setenv("MIVS_PREFILTER", "0")
    b = ivf_flat.build(p, xt)
    d0, i0 = _search(a, q)
    d1, i1 = _search(b, q)
    assert b.last_search_stats()["prefilter"] == 0 and a.last_search_stats()["prefilter"] == 1
    np.testing.assert_array_equal(i1, i0)
    np.testing.assert_array_equal(_bits(d1), _bits(d0))
    a.close()
    b.close()


@pytest.mark.parametrize("k", [10, 40])
@pytest.mark.parametrize("env", [{"MIVS_PQ_RT": "0"}, {"MIVS_PQ_RT": "0", "MIVS_PQ_SPLIT": "0"},
                                 {"MIVS_PQ_RT": "0", "MIVS_PQ_TILED": "1"}])
def test_ivf_pq_switch_same_bits(mivs_lib, monkeypatch, k, env):
    """IVF-PQ: K9r (default) vs K9s, K9 vs K9s, K9b (tiled; k <= 32 there): the same bits"""
    from mivs.neighbors import ivf_pq

    if env.get("MIVS_PQ_TILED") == "1" and k > 32:
        pytest.skip("K9b keeps k <= 32")
    x = _data(20_000, 128, 3)
    q = _data(33, 128, 4)
    idx = ivf_pq.build(ivf_pq.IndexParams(n_lists=32, pq_dim=32, kmeans_n_iters=3), torch.from_numpy(x).cuda())
    sp = ivf_pq.SearchParams(n_probes=6)
    qt = torch.from_numpy(q).cuda()
    d0, i0 = ivf_pq.search(sp, idx, qt, k)
    if k > 16:
        monkeypatch.setenv("MIVS_PQ_DUMP_K", "64")  # K9s: the register lists, where the switches apply
    for kk, v in env.items():
        _setenv(monkeypatch, kk, v)
    d1, i1 = ivf_pq.search(sp, idx, qt, k)
    np.testing.assert_array_equal(i1.cpu().numpy(), i0.cpu().numpy())
    np.testing.assert_array_equal(_bits(d1.cpu().numpy()), _bits(d0.cpu().numpy()))
    idx.close()


@pytest.mark.parametrize("k,metric", [(120, "sqeuclidean"), (256, "sqeuclidean"), (100, "inner_product")])
def test_ivf_pq_candidate_slots_same_bits_as_dump(mivs_lib, monkeypatch, k, metric):
    """64 < k <= 256: K9r's per-chunk candidate supersets + K8 over a query's slots (default) give the bits of
    the DUMP path (every row's key + K8, MIVS_PQ_CANDS=0), with ragged lists and chunks past 4096 rows"""
    from mivs.neighbors import ivf_pq

    x = _data(30_000, 64, 5)
    q = _data(41, 64, 6)
    idx = ivf_pq.build(ivf_pq.IndexParams(n_lists=6, pq_dim=16, kmeans_n_iters=3, metric=metric),
                       torch.from_numpy(x).cuda())
    sp = ivf_pq.SearchParams(n_probes=3)
    qt = torch.from_numpy(q).cuda()
    d0, i0 = ivf_pq.search(sp, idx, qt, k)
    _setenv(monkeypatch, "MIVS_PQ_CANDS", "0")
    d1, i1 = ivf_pq.search(sp, idx, qt, k)
    np.testing.assert_array_equal(i1.cpu().numpy(), i0.cpu().numpy())
    np.testing.assert_array_equal(_bits(d1.cpu().numpy()), _bits(d0.cpu().numpy()))
    idx.close()


@pytest.mark.parametrize("d,half,metric", [(768, True, "sqeuclidean"), (768, False, "sqeuclidean"),
                                           (64, False, "inner_product"), (200, True, "sqeuclidean")])
def test_refine_gather_switch_same_bits(mivs_lib, monkeypatch, d, half, metric):
    """refine: K14g (eight lanes per candidate row; fp16 rows at dp <= 768 with the next pass prefetched) vs one
    lane per row (MIVS_REFINE_GATHER=0): the same bits, with missing (-1) candidates and a ragged last pass"""
    from mivs.neighbors import refine

    rng = np.random.default_rng(d)
    x = torch.from_numpy(_data(4000, d, 7)).cuda()
    x = x.half() if half else x
    q = torch.from_numpy(_data(21, d, 8)).cuda()
    cand = torch.from_numpy(np.stack([rng.choice(4000, 117, replace=False) for _ in range(21)])).cuda()
    cand[torch.from_numpy(rng.random(cand.shape) < 0.1).cuda()] = -1
    d0, i0 = refine(x, q, cand, 10, metric=metric)
    _setenv(monkeypatch, "MIVS_REFINE_GATHER", "0")
    d1, i1 = refine(x, q, cand, 10, metric=metric)
    np.testing.assert_array_equal(i1.cpu().numpy(), i0.cpu().numpy())
    np.testing.assert_array_equal(_bits(d1.cpu().numpy()), _bits(d0.cpu().numpy()))


@pytest.mark.parametrize("k", [65, 120, 256])
def test_select_slots_wave_switch_same_bits(mivs_lib, monkeypatch, k):
    """K9r's candidate slots ranked by K8c (one wave per query) vs K8's block form (MIVS_SELECT_SLOTS_WAVE=0), rows
    duplicated 40 times so the k-th key is tied: the same bits"""
    from mivs.neighbors import ivf_pq

    base = _data(500, 64, 9)
    x = np.concatenate([base] * 40)
    q = _data(37, 64, 10)
    idx = ivf_pq.build(ivf_pq.IndexParams(n_lists=8, pq_dim=16, kmeans_n_iters=3), torch.from_numpy(x).cuda())
    sp = ivf_pq.SearchParams(n_probes=4)
    qt = torch.from_numpy(q).cuda()
    d0, i0 = ivf_pq.search(sp, idx, qt, k)
    _setenv(monkeypatch, "MIVS_SELECT_SLOTS_WAVE", "0")
    d1, i1 = ivf_pq.search(sp, idx, qt, k)
    np.testing.assert_array_equal(i1.cpu().numpy(), i0.cpu().numpy())
    np.testing.assert_array_equal(_bits(d1.cpu().numpy()), _bits(d0.cpu().numpy()))
    idx.close()


@pytest.mark.parametrize("n_probes", [16, 17, 32, 48])
def test_coarse_probe_equals_oracle(ivf, flat_data, n_probes):
    """the coarse probe -- K3's register top-k up to 16 probes, K3w DUMP + K8s above (slot-uniform key loads, the
    threshold from the lanes' minima) -- gives the oracle's probes in order, and the search its answer"""
    from mivs.neighbors import ivf_flat

    idx, metric = ivf
    x, q = flat_data
    qd = torch.from_numpy(q).cuda()
    p0 = torch.empty((q.shape[0], n_probes), dtype=torch.int32, device="cuda")
    d0, i0 = ivf_flat.search(ivf_flat.SearchParams(n_probes=n_probes), idx, qd, 10, probes_out=p0)
    od, oi, op = O.ivf_search(x, idx.centers.cpu().numpy(), idx.list_sizes.numpy(), idx.list_ids().cpu().numpy(), q,
                              n_probes, 10, metric=metric)
    np.testing.assert_array_equal(p0.cpu().numpy(), op)
    np.testing.assert_array_equal(i0.cpu().numpy(), oi)
    np.testing.assert_array_equal(_bits(d0.cpu().numpy()), _bits(od))


@pytest.mark.parametrize("dup", ["exact", "near"])
def test_coarse_probe_tied_centroids(flat_data, mivs_lib, dup):
    """centroids 32..63 duplicate 0..31 exactly (every probe key tied, resolved to the lower id) or up to a 1e-6 nudge:
    the coarse probe (K3w DUMP + K8s above 16 probes) gives the oracle's probes in order, and the search its answer"""
    from mivs.neighbors import ivf_flat

    x, q = flat_data
    rng = np.random.default_rng(11)
    c = x[rng.choice(x.shape[0], 32, replace=False)].copy()
    c2 = c.copy()
    if dup == "near":
        c2 += 1e-6 * rng.standard_normal(c2.shape).astype(np.float32)
    cents = np.concatenate([c, c2]).astype(np.float32)
    idx = ivf_flat.build_from_centroids(torch.from_numpy(cents).cuda(), torch.from_numpy(x[:20_000]).cuda())
    try:
        qd = torch.from_numpy(q).cuda()
        for n_probes in (20, 32):
            p0 = torch.empty((q.shape[0], n_probes), dtype=torch.int32, device="cuda")
            d0, i0 = ivf_flat.search(ivf_flat.SearchParams(n_probes=n_probes), idx, qd, 10, probes_out=p0)
            od, oi, op = O.ivf_search(x[:20_000], cents, idx.list_sizes.numpy(), idx.list_ids().cpu().numpy(), q,
                                      n_probes, 10)
            np.testing.assert_array_equal(p0.cpu().numpy(), op)
            np.testing.assert_array_equal(i0.cpu().numpy(), oi)
            np.testing.assert_array_equal(_bits(d0.cpu().numpy()), _bits(od))
    finally:
        idx.close()


def test_prepass_raw_lists_same_candidates(ivf, flat_data, monkeypatch):
    """round 6: the pre-pass's K10 leaves each slot as its 16 lane lists (K11v ranks all of them) instead of merging
    the best verify_sel in K10: the same nominees, so the same T_q, the same K13 candidates and the same answer"""
    idx, _ = ivf
    _, q = flat_data
    d0, i0 = _search(idx, q)
    st0 = idx.last_search_stats()
    _setenv(monkeypatch, "MIVS_PF_RAW_LISTS", "0")
    d1, i1 = _search(idx, q)
    st1 = idx.last_search_stats()
    np.testing.assert_array_equal(i1, i0)
    np.testing.assert_array_equal(_bits(d1), _bits(d0))
    assert st0["candidates"] == st1["candidates"] > 0


def test_k13_lost_stream_fallback_is_exact_and_reported(ivf, flat_data, monkeypatch):
    """force K13's record streams to overflow (2 records per wave): every query of the batch takes
    the fallback search, the stats say so, and the answer is the default one bit for bit"""
    idx, _ = ivf
    _, q = flat_data
    d0, i0 = _search(idx, q)
    st0 = idx.last_search_stats()
    assert st0["scan_kernel"] == 13 and st0["cand_overflow"] == 0 and st0["spun_out_waves"] == 0
    monkeypatch.setenv("MIVS_RS_WAVE_CAP", "2")
    d1, i1 = _search(idx, q)
    st1 = idx.last_search_stats()
    assert st1["cand_overflow"] == q.shape[0] and st1["overflow_queries"] >= q.shape[0]
    assert st1["spun_out_waves"] == 0
    np.testing.assert_array_equal(i1, i0)
    np.testing.assert_array_equal(_bits(d1), _bits(d0))


def test_k13_query_batches_same_bits(ivf, flat_data):
    """more queries than one K13 batch (kRsMaxBatch = 32768): the batched search equals per-slice searches"""
    idx, _ = ivf
    x, _ = flat_data
    rng = np.random.default_rng(9)
    q = x[rng.integers(0, x.shape[0], 33_000)] + 0.01 * rng.standard_normal((33_000, x.shape[1])).astype(np.float32)
    d, i = _search(idx, q)
    st = idx.last_search_stats()
    assert st["n_queries"] == 16_500  # two equal batches; the stats describe the last
    assert st["overflow_queries"] <= st["n_queries"]
    for lo, hi in ((0, 5000), (32_000, 33_000)):
        ds, is_ = _search(idx, q[lo:hi])
        np.testing.assert_array_equal(i[lo:hi], is_)
        np.testing.assert_array_equal(_bits(d[lo:hi]), _bits(ds))


def test_index_memory_single_fp32_copy_and_fp8_budget(flat_data, mivs_lib, monkeypatch):
    """the index holds ONE fp32 copy of the rows (64-B row blocks), the fp16 copy and -- within the HBM budget -- the
    fp8 copy, all built in build(); MIVS_INDEX_HBM_FRAC=0 leaves the fp8 copy out (reported in memory() and the search
    stats) and the search gives the same bits through the fp16 pre-pass sample"""
    from mivs.neighbors import ivf_flat

    x, q = flat_data
    xt = torch.from_numpy(x).cuda()
    p = ivf_flat.IndexParams(n_lists=48, kmeans_n_iters=4)
    a = ivf_flat.build(p, xt)
    m = a.memory()
    n, d = x.shape
    dp = (d + 63) // 64 * 64
    slots = m["rows_bytes"] // (4 * dp)
    assert slots >= n and m["fp16_bytes"] >= 2 * dp * slots and m["fp8_bytes"] == dp * slots, m
    assert m["copies_skipped"] == 0
    assert m["total_bytes"] == sum(m[k] for k in ("rows_bytes", "side_bytes", "centroid_bytes", "fp16_bytes",
                                                  "fp8_bytes", "pq_bytes"))
    # fp32 + fp16 + fp8 (+ norms, ids, offsets, centroids): no second fp32 copy
    assert m["total_bytes"] < (4 + 2 + 1) * dp * slots + 12 * slots + m["centroid_bytes"] + 4 * 48 * 64 + (1 << 20), m
    d0, i0 = _search(a, q)
    monkeypatch.setenv("MIVS_INDEX_HBM_FRAC", "0")
    b = ivf_flat.build(p, xt)
    mb = b.memory()
    assert mb["copies_skipped"] == 1 and mb["fp8_bytes"] == 0, mb
    d1, i1 = _search(b, q)
    assert b.last_search_stats()["copies_skipped"] == 1
    np.testing.assert_array_equal(i1, i0)
    np.testing.assert_array_equal(_bits(d1), _bits(d0))
    a.close()
    b.close()


def test_back_to_back_searches_without_sync(ivf, flat_data):
    """the k <= 16 search is stream-ordered (no host round trip since round 5): several searches enqueued back to back
    on one stream, of different batch sizes (one grows the workspaces), each equal to the same search run alone"""
    from mivs.neighbors import ivf_flat

    idx, _ = ivf
    _, q = flat_data
    sp = ivf_flat.SearchParams(n_probes=8)
    qt = torch.from_numpy(q).cuda()
    # (batch, k): k = 40 takes the large-k path (K16, host-sized) between stream-ordered ones
    parts = [(qt[:50], 10), (qt[50:], 10), (qt[:7], 16), (qt, 40), (qt, 5), (qt[:1], 10)]
    alone = []
    for p, k in parts:
        d, i = ivf_flat.search(sp, idx, p, k)
        torch.cuda.synchronize()
        alone.append((d.cpu().numpy(), i.cpu().numpy()))
    outs = [ivf_flat.search(sp, idx, p, k) for p, k in parts]  # (no synchronisation in between)
    torch.cuda.synchronize()
    for (d, i), (d0, i0) in zip(outs, alone):
        np.testing.assert_array_equal(i.cpu().numpy(), i0)
        np.testing.assert_array_equal(_bits(d.cpu().numpy()), _bits(d0))
