/*
 * mivs CPU oracle — TEST INFRASTRUCTURE ONLY (see mivs_oracle.h header).
 *
 * Bit-exact restatement of the arithmetic the HIP path performs
 * (DESIGN.md §3). Every function cites the reference
 * call site whose behaviour it restates. Build: oracle/Makefile
 * (-O2 -mfma -ffp-contract=off: every fused multiply-add below is an explicit
 * fmaf, nothing else may be contracted or reassociated).
 */
#include "mivs_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* dims are zero-padded to a multiple of 64 (kDimAlign in mivs_common.hpp); zero dims add exact
 * fmaf(0,0,acc) == acc steps (acc is never -0), so the padding is bitwise neutral */
int orc_dim_pad(int d) { return (d + 63) & ~63; }

/* The dot product in mivs k-order. The HIP kernels compute x·q with
 * v_mfma_f32_32x32x2_f32, whose result is bit-for-bit the fmaf chain
 * fma(a[k1],b[k1], fma(a[k0],b[k0], acc)) (verified on MI355X).
 * Lane (row r, half h) feeds dims 8s+4h+j, j=0..3, so the chain visits
 * k = 8s+j then 8s+4+j for j = 0..3, s = 0..dpad/8-1. Dims >= d are zero. */
float orc_dot(const float* a, const float* b, int d) {
  const int dp = orc_dim_pad(d);
  float acc = 0.0f;
  for (int s = 0; s < dp; s += 8) {
    for (int j = 0; j < 4; ++j) {
      const int k0 = s + j, k1 = s + 4 + j;
      const float a0 = k0 < d ? a[k0] : 0.0f, b0 = k0 < d ? b[k0] : 0.0f;
      const float a1 = k1 < d ? a[k1] : 0.0f, b1 = k1 < d ? b[k1] : 0.0f;
      acc = fmaf(a0, b0, acc);
      acc = fmaf(a1, b1, acc);
    }
  }
  return acc;
}

void orc_norms(const float* x, int64_t n, int d, float* out) {
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; ++i) out[i] = orc_dot(x + i * d, x + i * d, d);
}

/* cosine: x / sqrt(||x||^2) per row with the pinned norm, zero rows stay zero (sklearn normalize,
 * as in cosine_similarity / NearestNeighbors(metric='cosine') at
 * Attempt_1/VectorSearch_QuestionRetrieval.ipynb:839,878). */
void orc_normalize_rows(const float* x, int64_t n, int d, float* out) {
  for (int64_t i = 0; i < n; ++i) {
    const float nrm = sqrtf(orc_dot(x + i * d, x + i * d, d));
    for (int j = 0; j < d; ++j) out[i * d + j] = nrm > 0.0f ? x[i * d + j] / nrm : 0.0f;
  }
}

/* L2: the expanded squared distance ‖x‖² + ‖q‖² − 2 x·q, one fused rounding
 * for the −2·dot term, clamped at 0 (FAISS/cuVS "L2Expanded" semantics,
 * reached via ivf_flat.search at improved_multi_gpu_rag.py:227).
 * IP: key = −x·q so that "smaller key is better" for both metrics. */
float orc_key(float dot, float xn, float qn, int metric) {
  if (metric == ORC_IP) return -dot;
  const float t = xn + qn;
  const float v = fmaf(-2.0f, dot, t);
  return v > 0.0f ? v : 0.0f;
}

static float key_to_dist(float key, int metric) { return metric == ORC_IP ? -key : key; }

/* ---- bounded max-heap on (key, id): keeps the k smallest pairs ---- */
typedef struct { float key; int64_t id; } kv_t;

static int kv_less(kv_t a, kv_t b) { return a.key < b.key || (a.key == b.key && a.id < b.id); }

static void heap_push(kv_t* h, int* sz, int k, kv_t v) {
  if (*sz < k) {
    int i = (*sz)++;
    h[i] = v;
    while (i > 0) {
      int p = (i - 1) / 2;
      if (kv_less(h[p], h[i])) { kv_t t = h[p]; h[p] = h[i]; h[i] = t; i = p; } else break;
    }
  } else if (k > 0 && kv_less(v, h[0])) {
    h[0] = v;
    int i = 0;
    for (;;) {
      int l = 2 * i + 1, r = l + 1, m = i;
      if (l < k && kv_less(h[m], h[l])) m = l;
      if (r < k && kv_less(h[m], h[r])) m = r;
      if (m == i) break;
      kv_t t = h[m]; h[m] = h[i]; h[i] = t; i = m;
    }
  }
}

static int kv_cmp(const void* a, const void* b) {
  kv_t x = *(const kv_t*)a, y = *(const kv_t*)b;
  return kv_less(x, y) ? -1 : (kv_less(y, x) ? 1 : 0);
}

/* sorted ascending output; missing slots -> (+inf key, id -1) (FAISS convention) */
static void heap_emit(kv_t* h, int sz, int k, int metric, float* od, int64_t* oi) {
  qsort(h, (size_t)sz, sizeof(kv_t), kv_cmp);
  for (int j = 0; j < k; ++j) {
    if (j < sz) { od[j] = key_to_dist(h[j].key, metric); oi[j] = h[j].id; }
    else { od[j] = key_to_dist(INFINITY, metric); oi[j] = -1; }
  }
}

/* Exact kNN — FAISS IndexFlatL2.search (colab_a100_test.ipynb:454) / sklearn
 * NearestNeighbors(brute) (VectorSearch_QuestionRetrieval.ipynb:878), with
 * ties broken by id. */
void orc_knn(const float* x, int64_t n, const float* q, int64_t nq, int d, int k, int metric,
             int64_t id_offset, float* out_d, int64_t* out_i) {
  float* xn = (float*)malloc(sizeof(float) * (size_t)(n > 0 ? n : 1));
  orc_norms(x, n, d, xn);
#pragma omp parallel for schedule(dynamic, 1)
  for (int64_t qi = 0; qi < nq; ++qi) {
    kv_t* h = (kv_t*)malloc(sizeof(kv_t) * (size_t)(k > 0 ? k : 1));
    int sz = 0;
    const float* qq = q + qi * d;
    const float qn = orc_dot(qq, qq, d);
    for (int64_t i = 0; i < n; ++i) {
      kv_t v = {orc_key(orc_dot(x + i * d, qq, d), xn[i], qn, metric), i + id_offset};
      heap_push(h, &sz, k, v);
    }
    heap_emit(h, sz, k, metric, out_d + qi * k, out_i + qi * k);
    free(h);
  }
  free(xn);
}

/* Exact re-ranking of candidate rows -- cuvs.neighbors.refine(dataset, queries, candidates, k)
 * (cuvs 25.06, third-party; the step after an IVF-PQ search, improved_multi_gpu_rag.py:228-230):
 * per query the pinned key of every candidate row (id -1 or out of range: skipped), top-k by
 * (key, id). */
void orc_refine(const float* x, int64_t n, int d, const float* q, int64_t nq, const int64_t* cand, int nc, int k,
                int metric, float* out_d, int64_t* out_i) {
#pragma omp parallel for schedule(dynamic, 1)
  for (int64_t qi = 0; qi < nq; ++qi) {
    kv_t* h = (kv_t*)malloc(sizeof(kv_t) * (size_t)(k > 0 ? k : 1));
    int sz = 0;
    const float* qq = q + qi * d;
    const float qn = orc_dot(qq, qq, d);
    for (int c = 0; c < nc; ++c) {
      const int64_t r = cand[qi * nc + c];
      if (r < 0 || r >= n) continue;
      const float* xr = x + r * d;
      kv_t v = {orc_key(orc_dot(xr, qq, d), orc_dot(xr, xr, d), qn, metric), r};
      heap_push(h, &sz, k, v);
    }
    heap_emit(h, sz, k, metric, out_d + qi * k, out_i + qi * k);
    free(h);
  }
}

/* Global top-k merge of per-shard / per-probe candidate lists — the contract of
 * SearchResultAggregator.merge_search_results (test_search_result_aggregator.py:308-358)
 * and the notebook merge (cuvs-2gpu-main.ipynb:1820-1834), ties by id. */
void orc_merge(const float* in_d, const int64_t* in_i, int64_t nq, int m, int kin, int k, int metric,
               float* out_d, int64_t* out_i) {
  kv_t* h = (kv_t*)malloc(sizeof(kv_t) * (size_t)(k > 0 ? k : 1));
  for (int64_t qi = 0; qi < nq; ++qi) {
    int sz = 0;
    for (int64_t c = 0; c < (int64_t)m * kin; ++c) {
      const int64_t id = in_i[qi * m * kin + c];
      if (id < 0) continue;
      const float dd = in_d[qi * m * kin + c];
      kv_t v = {metric == ORC_IP ? -dd : dd, id};
      heap_push(h, &sz, k, v);
    }
    heap_emit(h, sz, k, metric, out_d + qi * k, out_i + qi * k);
  }
  free(h);
}

/* k-means assign (cuVS kmeans predict inside ivf_flat::build, reached from
 * index_building_coordinator.py:396): argmin over centroids of the ranking key,
 * ties to the lower centroid id. */
void orc_kmeans_assign(const float* x, const int64_t* rows, int64_t nr, const float* c, int nc, int d,
                       int metric, int32_t* labels) {
  float* cn = (float*)malloc(sizeof(float) * (size_t)nc);
  orc_norms(c, nc, d, cn);
#pragma omp parallel for schedule(static)
  for (int64_t t = 0; t < nr; ++t) {
    const float* xr = x + (rows ? rows[t] : t) * (int64_t)d;
    const float xn = orc_dot(xr, xr, d);
    float best = INFINITY;
    int32_t bi = 0;
    for (int j = 0; j < nc; ++j) {
      const float kk = orc_key(orc_dot(c + (int64_t)j * d, xr, d), cn[j], xn, metric);
      if (kk < best) { best = kk; bi = j; }
    }
    labels[t] = bi;
  }
  free(cn);
}

/* number of members summed per partial in the deterministic centroid update;
 * MUST equal MIVS_KM_CHUNK in cuvs-rag_amd/csrc/mivs_common.hpp */
#define ORC_KM_CHUNK 256

/* stable counting sort of 0..nr-1 by label -> order[], offs[nc+1] */
static void stable_by_label(const int32_t* labels, int64_t nr, int nc, int64_t* order, int64_t* offs) {
  memset(offs, 0, sizeof(int64_t) * (size_t)(nc + 1));
  for (int64_t t = 0; t < nr; ++t) offs[labels[t] + 1]++;
  for (int j = 0; j < nc; ++j) offs[j + 1] += offs[j];
  int64_t* fill = (int64_t*)malloc(sizeof(int64_t) * (size_t)nc);
  memcpy(fill, offs, sizeof(int64_t) * (size_t)nc);
  for (int64_t t = 0; t < nr; ++t) order[fill[labels[t]]++] = t;
  free(fill);
}

/* Lloyd update: centroid = mean of its members, summed in fp64 over fixed
 * chunks of ORC_KM_CHUNK members (member order = ascending train position),
 * chunk partials added in chunk order; an empty cluster keeps its centroid. */
void orc_kmeans_update(const float* x, const int64_t* rows, int64_t nr, const int32_t* labels, int nc, int d,
                       float* c) {
  int64_t* order = (int64_t*)malloc(sizeof(int64_t) * (size_t)(nr > 0 ? nr : 1));
  int64_t* offs = (int64_t*)malloc(sizeof(int64_t) * (size_t)(nc + 1));
  stable_by_label(labels, nr, nc, order, offs);
#pragma omp parallel
  {
    /* per dim kk: s = sum of the chunk's members in member order, total += s in chunk order (the loops run
     * member-outer so that each row is read contiguously; every (kk) sum sees the same sequence) */
    double* total = (double*)malloc(sizeof(double) * (size_t)d);
    double* s = (double*)malloc(sizeof(double) * (size_t)d);
#pragma omp for schedule(dynamic, 1)
    for (int j = 0; j < nc; ++j) {
      const int64_t b = offs[j], e = offs[j + 1], cnt = e - b;
      if (cnt == 0) continue;
      for (int kk = 0; kk < d; ++kk) total[kk] = 0.0;
      for (int64_t cb = b; cb < e; cb += ORC_KM_CHUNK) {
        const int64_t ce = cb + ORC_KM_CHUNK < e ? cb + ORC_KM_CHUNK : e;
        for (int kk = 0; kk < d; ++kk) s[kk] = 0.0;
        for (int64_t m = cb; m < ce; ++m) {
          const int64_t t = order[m];
          const float* xr = x + (rows ? rows[t] : t) * (int64_t)d;
          for (int kk = 0; kk < d; ++kk) s[kk] += (double)xr[kk];
        }
        for (int kk = 0; kk < d; ++kk) total[kk] += s[kk];
      }
      for (int kk = 0; kk < d; ++kk) c[(int64_t)j * d + kk] = (float)(total[kk] / (double)cnt);
    }
    free(total);
    free(s);
  }
  free(order);
  free(offs);
}

static uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

/* Balancing step — restates cuVS kmeans_balanced's adjust_centers (the balanced k-means inside
 * ivf_flat::build): every centroid j whose cluster holds fewer than ORC_BAL_FRAC x the average
 * members is pulled next to the centroid of an over-average cluster L:
 *     c_j = (wc * c_L + x_t) / (wc + 1),  wc = min(size_j, ORC_BAL_WC)
 * where x_t is the first member of an over-average cluster met by probing train positions
 * (r0 + p*ORC_BAL_STEP) mod nr, p < ORC_BAL_PROBES, r0 = splitmix64(ORC_BAL_SEED ^ (it << 32) ^ j) mod nr
 * (our deterministic probe sequence; cuVS uses its own). Placed that close to c_L, c_j splits L
 * in the next assignment. MUST match k_km_rebalance in cuvs-rag_amd/csrc/lists.hip. */
#define ORC_BAL_WC 4.0f
#define ORC_BAL_FRAC 0.25
#define ORC_BAL_PROBES 64
#define ORC_BAL_STEP 2654435761ull
#define ORC_BAL_SEED 0x5851F42D4C957F2Dull
#define ORC_BAL_KEEP_LAST 2 /* the last iterations are plain Lloyd */

void orc_kmeans_rebalance(const float* x, const int64_t* rows, int64_t nr, const int32_t* labels, int nc, int d,
                          int it, float* c) {
  int64_t* sizes = (int64_t*)calloc((size_t)nc, sizeof(int64_t));
  for (int64_t t = 0; t < nr; ++t) sizes[labels[t]]++;
  const double avg = (double)nr / (double)nc;
  for (int j = 0; j < nc; ++j) {
    if (!((double)sizes[j] < ORC_BAL_FRAC * avg)) continue;
    const uint64_t r0 = splitmix64(ORC_BAL_SEED ^ ((uint64_t)it << 32) ^ (uint64_t)j) % (uint64_t)nr;
    for (int p = 0; p < ORC_BAL_PROBES; ++p) {
      const int64_t t = (int64_t)((r0 + (uint64_t)p * ORC_BAL_STEP) % (uint64_t)nr);
      const int32_t L = labels[t];
      if ((double)sizes[L] > avg) {
        const float wc = (float)sizes[j] < ORC_BAL_WC ? (float)sizes[j] : ORC_BAL_WC;
        const float* xr = x + (rows ? rows[t] : t) * (int64_t)d;
        for (int kk = 0; kk < d; ++kk) {
          float v = wc * c[(int64_t)L * d + kk];
          v = v + xr[kk];
          c[(int64_t)j * d + kk] = v / (wc + 1.0f);
        }
        break;
      }
    }
  }
  free(sizes);
}

void orc_kmeans_fit(const float* x, const int64_t* rows, int64_t nr, int nc, int d, int iters, int metric,
                    float* c) {
  orc_kmeans_fit_ex(x, rows, nr, nc, d, iters, metric, 0, c);
}

void orc_kmeans_fit_ex(const float* x, const int64_t* rows, int64_t nr, int nc, int d, int iters, int metric,
                       int balance, float* c) {
  int32_t* labels = (int32_t*)malloc(sizeof(int32_t) * (size_t)(nr > 0 ? nr : 1));
  for (int it = 0; it < iters; ++it) {
    orc_kmeans_assign(x, rows, nr, c, nc, d, metric, labels);
    orc_kmeans_update(x, rows, nr, labels, nc, d, c);
    if (balance && it < iters - ORC_BAL_KEEP_LAST) orc_kmeans_rebalance(x, rows, nr, labels, nc, d, it, c);
  }
  free(labels);
}

/* Trainset size: cuVS IndexParams.kmeans_trainset_fraction (default 0.5) with an
 * optional FAISS-style cap of max_per_list rows per list (FAISS
 * max_points_per_centroid = 256), never fewer rows than lists. */
int64_t orc_train_count(int64_t n, int n_lists, double fraction, int64_t max_per_list) {
  int64_t nt = (int64_t)((double)n * fraction);
  if (max_per_list > 0 && nt > (int64_t)n_lists * max_per_list) nt = (int64_t)n_lists * max_per_list;
  if (nt < n_lists) nt = n_lists;
  if (nt > n) nt = n;
  return nt;
}

/* strided trainset rows (cuVS subsamples the dataset with a fixed stride) */
void orc_train_rows(int64_t n, int64_t n_train, int64_t* rows) {
  for (int64_t i = 0; i < n_train; ++i) rows[i] = (i * n) / n_train;
}

/* initial centroid j = train row floor(j * n_train / n_lists) */
void orc_init_rows(int64_t n_train, int n_lists, int64_t* which) {
  for (int j = 0; j < n_lists; ++j) which[j] = ((int64_t)j * n_train) / n_lists;
}

/* cuVS ivf_flat::extend restated: label every row with the trained centroids,
 * lists hold their rows in ascending id order (stable). */
void orc_ivf_lists_from_centroids(const float* x, int64_t n, int d, const float* centroids, int n_lists,
                                  int metric, int64_t id_offset, int64_t* list_sizes, int64_t* list_ids) {
  int32_t* labels = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n > 0 ? n : 1));
  orc_kmeans_assign(x, NULL, n, centroids, n_lists, d, metric, labels);
  int64_t* order = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
  int64_t* offs = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n_lists + 1));
  stable_by_label(labels, n, n_lists, order, offs);
  for (int j = 0; j < n_lists; ++j) list_sizes[j] = offs[j + 1] - offs[j];
  for (int64_t i = 0; i < n; ++i) list_ids[i] = order[i] + id_offset;
  free(labels);
  free(order);
  free(offs);
}

/* ivf_flat.build(IndexParams(n_lists=...), dataset) — index_building_coordinator.py:392-396 */
void orc_ivf_build(const float* x, int64_t n, int d, int n_lists, int iters, double fraction,
                   int64_t max_per_list, int metric, int balance, int64_t id_offset, float* centroids,
                   int64_t* list_sizes, int64_t* list_ids) {
  const int64_t nt = orc_train_count(n, n_lists, fraction, max_per_list);
  int64_t* rows = (int64_t*)malloc(sizeof(int64_t) * (size_t)nt);
  int64_t* which = (int64_t*)malloc(sizeof(int64_t) * (size_t)n_lists);
  orc_train_rows(n, nt, rows);
  orc_init_rows(nt, n_lists, which);
  for (int j = 0; j < n_lists; ++j)
    memcpy(centroids + (int64_t)j * d, x + rows[which[j]] * (int64_t)d, sizeof(float) * (size_t)d);
  orc_kmeans_fit_ex(x, rows, nt, n_lists, d, iters, ORC_L2, balance, centroids);
  orc_ivf_lists_from_centroids(x, n, d, centroids, n_lists, metric, id_offset, list_sizes, list_ids);
  free(rows);
  free(which);
}

/* ivf_flat.search(SearchParams(n_probes), index, q, k) — improved_multi_gpu_rag.py:225-227:
 * coarse top-n_probes lists by (key, list id), exhaustive scan of those lists,
 * top-k by (key, id). */
void orc_ivf_search(const float* x, int64_t id_offset, int d, const float* centroids, int n_lists,
                    const int64_t* list_sizes, const int64_t* list_ids, const float* q, int64_t nq,
                    int n_probes, int k, int metric, float* out_d, int64_t* out_i, int32_t* out_probes) {
  if (n_probes > n_lists) n_probes = n_lists;
  int64_t* offs = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n_lists + 1));
  offs[0] = 0;
  for (int j = 0; j < n_lists; ++j) offs[j + 1] = offs[j] + list_sizes[j];
  float* cn = (float*)malloc(sizeof(float) * (size_t)n_lists);
  orc_norms(centroids, n_lists, d, cn);
#pragma omp parallel for schedule(dynamic, 1)
  for (int64_t qi = 0; qi < nq; ++qi) {
    const float* qq = q + qi * d;
    const float qn = orc_dot(qq, qq, d);
    kv_t* ph = (kv_t*)malloc(sizeof(kv_t) * (size_t)n_probes);
    int psz = 0;
    for (int j = 0; j < n_lists; ++j) {
      kv_t v = {orc_key(orc_dot(centroids + (int64_t)j * d, qq, d), cn[j], qn, metric), j};
      heap_push(ph, &psz, n_probes, v);
    }
    qsort(ph, (size_t)psz, sizeof(kv_t), kv_cmp);
    kv_t* h = (kv_t*)malloc(sizeof(kv_t) * (size_t)(k > 0 ? k : 1));
    int sz = 0;
    for (int p = 0; p < psz; ++p) {
      const int l = (int)ph[p].id;
      if (out_probes) out_probes[qi * n_probes + p] = l;
      for (int64_t m = offs[l]; m < offs[l + 1]; ++m) {
        const int64_t id = list_ids[m];
        const float* xr = x + (id - id_offset) * (int64_t)d;
        kv_t v = {orc_key(orc_dot(xr, qq, d), orc_dot(xr, xr, d), qn, metric), id};
        heap_push(h, &sz, k, v);
      }
    }
    heap_emit(h, sz, k, metric, out_d + qi * k, out_i + qi * k);
    free(h);
    free(ph);
  }
  free(offs);
  free(cn);
}

/* ======================================================================================
 * IVF-PQ — cuVS ivf_pq (cuvs 25.6.0) as the reference reaches it:
 *   index_building_coordinator.py:398-404  ivf_pq.IndexParams(n_lists, pq_bits=8,
 *                                           pq_dim=min(64, d // 4)); ivf_pq.build
 *   improved_multi_gpu_rag.py:131-137,228-230  pq_dim=96, pq_bits=8; ivf_pq.search
 * Published algorithm restated (no reference fixture pins PQ numerics: parity unpinned beyond
 * the pinned Lloyd k-means it is built from):
 *   coarse k-means on the trainset (as IVF-Flat) -> lists by L2 assignment;
 *   rot_dim = pq_dim * pq_len, pq_len = ceil(d / pq_dim); identity rotation, dims >= d read 0;
 *   per subspace j a 2^pq_bits-entry codebook = k-means on the residual sub-vectors
 *   (x - c_label)[j*pq_len, (j+1)*pq_len) of min(n, max_per_code * 2^pq_bits) strided rows;
 *   code_j(x) = argmin_c ||r_j - B_j[c]||^2 (ties: lowest c);
 *   search: per probed list l, LUT_j[c] = ||(q - c_l)_j - B_j[c]||^2 and
 *   dist(x) = sum_j LUT_j[code_j(x)] (j ascending, fp32); top-k by (dist, id) over all probes.
 * Pinned order: ||a - b||^2 over pq_len dims = acc = fmaf(a_i - b_i, a_i - b_i, acc), i ascending.
 * ====================================================================================== */
int orc_pq_len(int d, int pq_dim) { return (d + pq_dim - 1) / pq_dim; }

int64_t orc_pq_train_count(int64_t n, int pq_bits, int64_t max_per_code) {
  const int64_t cap = max_per_code << pq_bits;
  return n < cap ? n : cap;
}

float orc_pq_l2(const float* a, const float* b, int pl) {
  float acc = 0.0f;
  for (int i = 0; i < pl; ++i) {
    const float t = a[i] - b[i];
    acc = fmaf(t, t, acc);
  }
  return acc;
}

/* The search LUT's L2 entry (round 4: the expanded form, so that the GPU builds it on MFMA,
 * pq.hip k_pq_scan_rt): ||r - b||^2 = ||r||^2 + ||b||^2 - 2 r.b, as
 *   rn = fmaf chain of r_i r_i, bn = fmaf chain of b_i b_i (i ascending, from 0),
 *   acc = rn + bn, then acc = fmaf(r_i, -2 b_i, acc) for i ascending.
 * v_mfma_f32_16x16x4_f32 computes fma(a3,b3, fma(a2,b2, fma(a1,b1, fma(a0,b0, c)))) (measured:
 * tools/mfma_f32_order.hip), so MFMA s fed dims 4s..4s+3
 * with c = rn + bn is this chain; -2 b_i is exact. cuVS builds the difference form
 * (ivf_pq compute_similarity); the two agree to fp32 rounding (tests/test_oracle_pq.py checks the ranking
 * against fp64 ||q - x_hat||^2). The encoder's argmin keeps the difference form (orc_pq_l2). */
float orc_pq_l2_lut(const float* r, const float* b, int pl) {
  float rn = 0.0f, bn = 0.0f;
  for (int i = 0; i < pl; ++i) rn = fmaf(r[i], r[i], rn);
  for (int i = 0; i < pl; ++i) bn = fmaf(b[i], b[i], bn);
  float acc = rn + bn;
  for (int i = 0; i < pl; ++i) acc = fmaf(r[i], -2.0f * b[i], acc);
  return acc;
}

/* residual sub-vector j (pq_len dims) of row x w.r.t. centre c; dims >= d are 0 */
/* the IP LUT entry's dot, dims ascending (the GPU K9/K9s chain): -(sum_i q_i b_i) */
float orc_pq_ip(const float* a, const float* b, int pl) {
  float acc = 0.0f;
  for (int i = 0; i < pl; ++i) acc = fmaf(a[i], b[i], acc);
  return -acc;
}

static void pq_residual(const float* x, const float* c, int d, int j, int pl, float* out) {
  for (int i = 0; i < pl; ++i) {
    const int k = j * pl + i;
    out[i] = k < d ? x[k] - c[k] : 0.0f;
  }
}

void orc_ivfpq_train_codebooks(const float* x, int64_t n, int d, const float* centroids, const int32_t* labels,
                               int pq_dim, int pq_bits, int iters, int balance, int64_t max_per_code,
                               float* codebooks /* [pq_dim][2^pq_bits][pq_len] */) {
  const int pl = orc_pq_len(d, pq_dim);
  const int nc = 1 << pq_bits;
  const int64_t nt = orc_pq_train_count(n, pq_bits, max_per_code);
  int64_t* rows = (int64_t*)malloc(sizeof(int64_t) * (size_t)nt);
  orc_train_rows(n, nt, rows);
  int64_t* which = (int64_t*)malloc(sizeof(int64_t) * (size_t)nc);
  orc_init_rows(nt, nc, which);
  float* r = (float*)malloc(sizeof(float) * (size_t)nt * pl);
  for (int j = 0; j < pq_dim; ++j) {
    for (int64_t t = 0; t < nt; ++t)
      pq_residual(x + rows[t] * (int64_t)d, centroids + (int64_t)labels[rows[t]] * d, d, j, pl, r + t * pl);
    float* cb = codebooks + (int64_t)j * nc * pl;
    for (int c = 0; c < nc; ++c) memcpy(cb + (int64_t)c * pl, r + which[c] * pl, sizeof(float) * (size_t)pl);
    orc_kmeans_fit_ex(r, NULL, nt, nc, pl, iters, ORC_L2, balance, cb);
  }
  free(r);
  free(which);
  free(rows);
}

void orc_ivfpq_encode(const float* x, const int64_t* rows, int64_t nr, int d, const float* centroids,
                      const int32_t* labels /* per row of x */, const float* codebooks, int pq_dim, int pq_bits,
                      uint8_t* codes /* [nr][pq_dim] */) {
  const int pl = orc_pq_len(d, pq_dim);
  const int nc = 1 << pq_bits;
#pragma omp parallel
  {
    float* r = (float*)malloc(sizeof(float) * (size_t)pl);
#pragma omp for
    for (int64_t t = 0; t < nr; ++t) {
      const int64_t row = rows ? rows[t] : t;
      for (int j = 0; j < pq_dim; ++j) {
        pq_residual(x + row * (int64_t)d, centroids + (int64_t)labels[row] * d, d, j, pl, r);
        const float* cb = codebooks + (int64_t)j * nc * pl;
        int best = 0;
        float bd = orc_pq_l2(r, cb, pl);
        for (int c = 1; c < nc; ++c) {
          const float v = orc_pq_l2(r, cb + (int64_t)c * pl, pl);
          if (v < bd) { bd = v; best = c; }
        }
        codes[t * pq_dim + j] = (uint8_t)best;
      }
    }
    free(r);
  }
}

void orc_ivfpq_build(const float* x, int64_t n, int d, int n_lists, int iters, double fraction, int pq_dim,
                     int pq_bits, int64_t max_per_code, int balance, int64_t id_offset, float* centroids,
                     float* codebooks, int64_t* list_sizes, int64_t* list_ids, uint8_t* codes) {
  const int64_t nt = orc_train_count(n, n_lists, fraction, 0);
  int64_t* rows = (int64_t*)malloc(sizeof(int64_t) * (size_t)nt);
  int64_t* which = (int64_t*)malloc(sizeof(int64_t) * (size_t)n_lists);
  orc_train_rows(n, nt, rows);
  orc_init_rows(nt, n_lists, which);
  for (int j = 0; j < n_lists; ++j)
    memcpy(centroids + (int64_t)j * d, x + rows[which[j]] * (int64_t)d, sizeof(float) * (size_t)d);
  orc_kmeans_fit_ex(x, rows, nt, n_lists, d, iters, ORC_L2, balance, centroids);
  int32_t* labels = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n > 0 ? n : 1));
  orc_kmeans_assign(x, NULL, n, centroids, n_lists, d, ORC_L2, labels);
  orc_ivfpq_train_codebooks(x, n, d, centroids, labels, pq_dim, pq_bits, iters, balance, max_per_code, codebooks);
  int64_t* order = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n > 0 ? n : 1));
  int64_t* offs = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n_lists + 1));
  stable_by_label(labels, n, n_lists, order, offs);
  for (int j = 0; j < n_lists; ++j) list_sizes[j] = offs[j + 1] - offs[j];
  for (int64_t t = 0; t < n; ++t) list_ids[t] = order[t] + id_offset;
  orc_ivfpq_encode(x, order, n, d, centroids, labels, codebooks, pq_dim, pq_bits, codes);
  free(offs);
  free(order);
  free(labels);
  free(rows);
  free(which);
}

/* fp32 -> the nearest fp16 (ties to even, fp16 subnormals kept, |v| >= 65520 -> inf) -> fp32: what a LUT entry
 * stored as fp16 (v_cvt_f16_f32, round to nearest even) and read back (v_cvt_f32_f16) holds. gcc 11 has no
 * _Float16 on x86, so the rounding is done in double: spacing 2^(e - 10) at binary exponent e >= -14, 2^-24 below. */
float orc_round_f16(float v) {
  if (!(fabsf(v) < INFINITY)) return v;
  int e = 0;
  (void)frexp((double)v, &e); /* |v| in [2^(e-1), 2^e) */
  int ex = e - 1;
  if (ex < -14) ex = -14;
  const double sp = ldexp(1.0, ex - 10);
  const double r = rint((double)v / sp) * sp;
  if (fabs(r) >= 65536.0) return v < 0.0f ? -INFINITY : INFINITY;
  return (float)r;
}

/* IVF-PQ search (cuvs.neighbors.ivf_pq.search, improved_multi_gpu_rag.py:228-230). metric ORC_L2: a row's key
 * is sum_j LUT_j[code_j] (j ascending, from 0) with LUT_j[c] = ||(q - c_l)_j - B_j[c]||^2 in the expanded form
 * of orc_pq_l2_lut. ORC_IP: LUT_j[c] =
 * -(q_j . B_j[c]) and subspace 0's row also carries the probe's coarse key -(q . c_l) (orc_dot), so the key
 * estimates -(q . x_hat); distances out are the inner products (-key). Probes rank by the metric's key. */
/* lut_fp16 (cuvs SearchParams.lut_dtype = float16; ORC_L2 only): every LUT entry is rounded to fp16 (orc_round_f16)
 * when the LUT is built, the row sums stay fp32 in the same order */
void orc_ivfpq_search_ex(const float* centroids, int n_lists, int d, const float* codebooks, int pq_dim, int pq_bits,
                         const int64_t* list_sizes, const int64_t* list_ids, const uint8_t* codes, const float* q,
                         int64_t nq, int n_probes, int k, int metric, float* out_d, int64_t* out_i,
                         int32_t* out_probes, int lut_fp16) {
  if (n_probes > n_lists) n_probes = n_lists;
  const int pl = orc_pq_len(d, pq_dim);
  const int nc = 1 << pq_bits;
  int64_t* offs = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n_lists + 1));
  offs[0] = 0;
  for (int j = 0; j < n_lists; ++j) offs[j + 1] = offs[j] + list_sizes[j];
  float* cn = (float*)malloc(sizeof(float) * (size_t)n_lists);
  orc_norms(centroids, n_lists, d, cn);
#pragma omp parallel for schedule(dynamic, 1)
  for (int64_t qi = 0; qi < nq; ++qi) {
    const float* qq = q + qi * d;
    const float qn = orc_dot(qq, qq, d);
    kv_t* ph = (kv_t*)malloc(sizeof(kv_t) * (size_t)n_probes);
    int psz = 0;
    for (int j = 0; j < n_lists; ++j) {
      kv_t v = {orc_key(orc_dot(centroids + (int64_t)j * d, qq, d), cn[j], qn, metric), j};
      heap_push(ph, &psz, n_probes, v);
    }
    qsort(ph, (size_t)psz, sizeof(kv_t), kv_cmp);
    float* lut = (float*)malloc(sizeof(float) * (size_t)pq_dim * nc);
    float* r = (float*)malloc(sizeof(float) * (size_t)pl);
    kv_t* h = (kv_t*)malloc(sizeof(kv_t) * (size_t)(k > 0 ? k : 1));
    int sz = 0;
    for (int p = 0; p < psz; ++p) {
      const int l = (int)ph[p].id;
      if (out_probes) out_probes[qi * n_probes + p] = l;
      for (int j = 0; j < pq_dim; ++j) {
        if (metric == ORC_IP) {
          for (int i = 0; i < pl; ++i) r[i] = j * pl + i < d ? qq[j * pl + i] : 0.0f;
          for (int c = 0; c < nc; ++c) {
            float v = orc_pq_ip(r, codebooks + ((int64_t)j * nc + c) * pl, pl);
            if (j == 0) v = v + ph[p].key; /* the probe's coarse key -(q . c_l) */
            lut[j * nc + c] = v;
          }
        } else {
          pq_residual(qq, centroids + (int64_t)l * d, d, j, pl, r);
          for (int c = 0; c < nc; ++c) {
            const float v = orc_pq_l2_lut(r, codebooks + ((int64_t)j * nc + c) * pl, pl);
            lut[j * nc + c] = lut_fp16 ? orc_round_f16(v) : v;
          }
        }
      }
      for (int64_t m = offs[l]; m < offs[l + 1]; ++m) {
        const uint8_t* cd = codes + m * pq_dim;
        float dist = 0.0f;
        for (int j = 0; j < pq_dim; ++j) dist = dist + lut[j * nc + cd[j]];
        kv_t v = {dist, list_ids[m]};
        heap_push(h, &sz, k, v);
      }
    }
    heap_emit(h, sz, k, metric, out_d + qi * k, out_i + qi * k);
    free(h);
    free(r);
    free(lut);
    free(ph);
  }
  free(offs);
  free(cn);
}

void orc_ivfpq_search(const float* centroids, int n_lists, int d, const float* codebooks, int pq_dim, int pq_bits,
                      const int64_t* list_sizes, const int64_t* list_ids, const uint8_t* codes, const float* q,
                      int64_t nq, int n_probes, int k, int metric, float* out_d, int64_t* out_i,
                      int32_t* out_probes) {
  orc_ivfpq_search_ex(centroids, n_lists, d, codebooks, pq_dim, pq_bits, list_sizes, list_ids, codes, q, nq, n_probes,
                      k, metric, out_d, out_i, out_probes, 0);
}
