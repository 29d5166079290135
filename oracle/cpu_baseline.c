/*
 * FAISS-algorithm CPU baseline (faiss is not installed on this image or the
 * GPU box) — TEST/BENCH INFRASTRUCTURE ONLY, part of the oracle library.
 *
 * Restates FAISS 1.7.2's CPU search loops, which the reference times as its CPU
 * path (Latest/faiss.ipynb:1051 `index.search`, colab_a100_test.ipynb:433-490):
 *   IndexFlatL2     -> per query, fvec_L2sqr over every row + bounded max-heap
 *   IndexIVFFlat    -> coarse IndexFlatL2 over centroids, top-nprobe lists,
 *                      fvec_L2sqr over every row of each probed list + heap
 * parallelised over queries with OpenMP (FAISS parallel_mode 0). Direct-form
 * squared L2, vectorised (compiled -O3 -ffast-math): results are NOT bit-exact
 * with mivs_oracle.c; tests check them against it by recall.
 */
#include "mivs_oracle.h"

#include <math.h>
#include <omp.h>
#include <stdlib.h>

int orc_fast_threads(void) { return omp_get_max_threads(); }
void orc_fast_set_threads(int t) { omp_set_num_threads(t); }

static inline float l2sqr(const float* a, const float* b, int d) {
  float s = 0.0f;
#pragma omp simd reduction(+ : s)
  for (int k = 0; k < d; ++k) {
    const float t = a[k] - b[k];
    s += t * t;
  }
  return s;
}

typedef struct { float d; int64_t i; } hv_t;

static inline void hpush(hv_t* h, int* sz, int k, float d, int64_t i) {
  if (*sz < k) {
    int c = (*sz)++;
    h[c].d = d; h[c].i = i;
    while (c > 0) {
      int p = (c - 1) >> 1;
      if (h[p].d < h[c].d || (h[p].d == h[c].d && h[p].i < h[c].i)) { hv_t t = h[p]; h[p] = h[c]; h[c] = t; c = p; }
      else break;
    }
  } else if (d < h[0].d || (d == h[0].d && i < h[0].i)) {
    h[0].d = d; h[0].i = i;
    int c = 0;
    for (;;) {
      int l = 2 * c + 1, r = l + 1, m = c;
      if (l < k && (h[m].d < h[l].d || (h[m].d == h[l].d && h[m].i < h[l].i))) m = l;
      if (r < k && (h[m].d < h[r].d || (h[m].d == h[r].d && h[m].i < h[r].i))) m = r;
      if (m == c) break;
      hv_t t = h[m]; h[m] = h[c]; h[c] = t; c = m;
    }
  }
}

static void hsort_emit(hv_t* h, int sz, int k, float* od, int64_t* oi) {
  /* heap-sort in place: repeatedly move the max to the end */
  for (int end = sz - 1; end > 0; --end) {
    hv_t t = h[0]; h[0] = h[end]; h[end] = t;
    int c = 0;
    for (;;) {
      int l = 2 * c + 1, r = l + 1, m = c;
      if (l < end && (h[m].d < h[l].d || (h[m].d == h[l].d && h[m].i < h[l].i))) m = l;
      if (r < end && (h[m].d < h[r].d || (h[m].d == h[r].d && h[m].i < h[r].i))) m = r;
      if (m == c) break;
      hv_t u = h[m]; h[m] = h[c]; h[c] = u; c = m;
    }
  }
  for (int j = 0; j < k; ++j) {
    if (j < sz) { od[j] = h[j].d; oi[j] = h[j].i; } else { od[j] = INFINITY; oi[j] = -1; }
  }
}

void orc_fast_knn(const float* x, int64_t n, const float* q, int64_t nq, int d, int k,
                  float* out_d, int64_t* out_i) {
#pragma omp parallel for schedule(dynamic, 1)
  for (int64_t qi = 0; qi < nq; ++qi) {
    hv_t* h = (hv_t*)malloc(sizeof(hv_t) * (size_t)k);
    int sz = 0;
    const float* qq = q + qi * d;
    for (int64_t i = 0; i < n; ++i) hpush(h, &sz, k, l2sqr(x + i * d, qq, d), i);
    hsort_emit(h, sz, k, out_d + qi * k, out_i + qi * k);
    free(h);
  }
}

void orc_fast_ivf_search(const float* list_rows, const int64_t* list_ids, const int64_t* offsets,
                         const float* centroids, int n_lists, int d, const float* q, int64_t nq,
                         int n_probes, int k, float* out_d, int64_t* out_i) {
  if (n_probes > n_lists) n_probes = n_lists;
#pragma omp parallel for schedule(dynamic, 1)
  for (int64_t qi = 0; qi < nq; ++qi) {
    const float* qq = q + qi * d;
    hv_t* ph = (hv_t*)malloc(sizeof(hv_t) * (size_t)n_probes);
    int psz = 0;
    for (int j = 0; j < n_lists; ++j) hpush(ph, &psz, n_probes, l2sqr(centroids + (int64_t)j * d, qq, d), j);
    hv_t* h = (hv_t*)malloc(sizeof(hv_t) * (size_t)k);
    int sz = 0;
    for (int p = 0; p < psz; ++p) {
      const int64_t l = ph[p].i;
      for (int64_t m = offsets[l]; m < offsets[l + 1]; ++m)
        hpush(h, &sz, k, l2sqr(list_rows + m * (int64_t)d, qq, d), list_ids[m]);
    }
    hsort_emit(h, sz, k, out_d + qi * k, out_i + qi * k);
    free(h);
    free(ph);
  }
}
