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
 *
 * The per-query workers are built for AVX-512, AVX2+FMA and baseline x86-64 and the
 * best the host runs is picked at the call (__builtin_cpu_supports): the library is
 * built in a container whose CPU is not the GPU box's, so -march=native would be the
 * wrong host's ISA, and FAISS itself dispatches to its AVX-512 / AVX2 kernels.
 * orc_parallel_copy first-touches its destination from every thread (OpenMP static
 * chunks), so a host copy of the lists is spread over the NUMA nodes of the threads
 * that scan it instead of sitting on the node of one copying thread.
 */
#include "mivs_oracle.h"

#include <math.h>
#include <omp.h>
#include <stdlib.h>
#include <string.h>

/* the per-query workers, instantiated per ISA (gcc 11's target_clones cannot group avx2 with fma) and picked once
 * by __builtin_cpu_supports */
#define ORC_ISA_AVX512 __attribute__((target("avx512f,avx512vl,avx512dq,avx2,fma")))
#define ORC_ISA_AVX2 __attribute__((target("avx2,fma")))
#define ORC_ISA_BASE

int orc_fast_threads(void) { return omp_get_max_threads(); }
void orc_fast_set_threads(int t) { omp_set_num_threads(t); }

static inline __attribute__((always_inline)) float l2sqr(const float* a, const float* b, int d) {
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

/* one query of IndexFlatL2's per-query form: every row into a bounded max-heap */
#define KNN_ONE(NAME, ISA)                                                                                        \
  ISA static void NAME(const float* x, int64_t n, const float* qq, int d, int k, float* od, int64_t* oi, hv_t* h) { \
    int sz = 0;                                                                                                   \
    for (int64_t i = 0; i < n; ++i) hpush(h, &sz, k, l2sqr(x + i * d, qq, d), i);                                 \
    hsort_emit(h, sz, k, od, oi);                                                                                 \
  }
KNN_ONE(knn_one_avx512, ORC_ISA_AVX512)
KNN_ONE(knn_one_avx2, ORC_ISA_AVX2)
KNN_ONE(knn_one_base, ORC_ISA_BASE)

/* one query of IndexIVFFlat's search: coarse top-n_probes over the centroids, then every row of each probed list */
#define IVF_ONE(NAME, ISA)                                                                                        \
  ISA static void NAME(const float* list_rows, const int64_t* list_ids, const int64_t* offsets,                   \
                       const float* centroids, int n_lists, int d, const float* qq, int n_probes, int k, float* od, \
                       int64_t* oi, hv_t* ph, hv_t* h) {                                                          \
    int psz = 0;                                                                                                  \
    for (int j = 0; j < n_lists; ++j) hpush(ph, &psz, n_probes, l2sqr(centroids + (int64_t)j * d, qq, d), j);    \
    int sz = 0;                                                                                                   \
    for (int p = 0; p < psz; ++p) {                                                                               \
      const int64_t l = ph[p].i;                                                                                  \
      for (int64_t m = offsets[l]; m < offsets[l + 1]; ++m)                                                       \
        hpush(h, &sz, k, l2sqr(list_rows + m * (int64_t)d, qq, d), list_ids[m]);                                  \
    }                                                                                                             \
    hsort_emit(h, sz, k, od, oi);                                                                                 \
  }
IVF_ONE(ivf_one_avx512, ORC_ISA_AVX512)
IVF_ONE(ivf_one_avx2, ORC_ISA_AVX2)
IVF_ONE(ivf_one_base, ORC_ISA_BASE)

static int isa_level(void) {  /* 2: AVX-512, 1: AVX2 + FMA, 0: baseline */
  __builtin_cpu_init();
  if (__builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512vl") && __builtin_cpu_supports("avx512dq"))
    return 2;
  if (__builtin_cpu_supports("avx2") && __builtin_cpu_supports("fma")) return 1;
  return 0;
}

void orc_fast_knn(const float* x, int64_t n, const float* q, int64_t nq, int d, int k,
                  float* out_d, int64_t* out_i) {
  const int lv = isa_level();
#pragma omp parallel
  {
    hv_t* h = (hv_t*)malloc(sizeof(hv_t) * (size_t)k);
#pragma omp for schedule(dynamic, 1)
    for (int64_t qi = 0; qi < nq; ++qi) {
      const float* qq = q + qi * d;
      if (lv == 2) knn_one_avx512(x, n, qq, d, k, out_d + qi * k, out_i + qi * k, h);
      else if (lv == 1) knn_one_avx2(x, n, qq, d, k, out_d + qi * k, out_i + qi * k, h);
      else knn_one_base(x, n, qq, d, k, out_d + qi * k, out_i + qi * k, h);
    }
    free(h);
  }
}

void orc_fast_ivf_search(const float* list_rows, const int64_t* list_ids, const int64_t* offsets,
                         const float* centroids, int n_lists, int d, const float* q, int64_t nq,
                         int n_probes, int k, float* out_d, int64_t* out_i) {
  if (n_probes > n_lists) n_probes = n_lists;
  const int lv = isa_level();
#pragma omp parallel
  {
    hv_t* ph = (hv_t*)malloc(sizeof(hv_t) * (size_t)n_probes);
    hv_t* h = (hv_t*)malloc(sizeof(hv_t) * (size_t)k);
#pragma omp for schedule(dynamic, 1)
    for (int64_t qi = 0; qi < nq; ++qi) {
      const float* qq = q + qi * d;
      float* od = out_d + qi * k;
      int64_t* oi = out_i + qi * k;
      if (lv == 2) ivf_one_avx512(list_rows, list_ids, offsets, centroids, n_lists, d, qq, n_probes, k, od, oi, ph, h);
      else if (lv == 1) ivf_one_avx2(list_rows, list_ids, offsets, centroids, n_lists, d, qq, n_probes, k, od, oi, ph, h);
      else ivf_one_base(list_rows, list_ids, offsets, centroids, n_lists, d, qq, n_probes, k, od, oi, ph, h);
    }
    free(h);
    free(ph);
  }
}

/* dst <- src (nbytes), 2 MiB chunks dealt to the threads in static round-robin: each thread first-touches the pages
 * it writes, so the copy's pages spread over the NUMA nodes the threads run on */
void orc_parallel_copy(void* dst, const void* src, int64_t nbytes) {
  const int64_t chunk = (int64_t)2 << 20;
  const int64_t nc = (nbytes + chunk - 1) / chunk;
#pragma omp parallel for schedule(static, 1)
  for (int64_t c = 0; c < nc; ++c) {
    const int64_t o = c * chunk;
    const int64_t len = nbytes - o < chunk ? nbytes - o : chunk;
    memcpy((char*)dst + o, (const char*)src + o, (size_t)len);
  }
}

/* the ISA the workers run with on this host */
const char* orc_fast_isa(void) {
  static const char* names[3] = {"x86-64", "avx2+fma", "avx512"};
  return names[isa_level()];
}
