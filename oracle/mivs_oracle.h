/*
 * mivs CPU oracle — TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C restatement of the IVF-Flat / brute-force k-NN algorithm the
 * reference reaches through cuVS 25.6.0 (`cuvs.neighbors.ivf_flat`, pinned in
 * /root/reference/Attempt_1/requirements.txt:103,224) and FAISS 1.7.2
 * (`IndexFlatL2`, `IndexIVFFlat`, /root/reference/Latest/faiss.ipynb:29).
 * Neither library is vendored in the reference nor importable here, so the
 * ANN arithmetic below is a restatement of their published algorithms with
 * the arithmetic order pinned down exactly (see DESIGN.md "Arithmetic
 * contract"); parity of the shipped HIP path is then BIT-EXACT against this
 * file. The reference's own numeric pins (merge fixtures, shard splits) and
 * sklearn's brute-force / Lloyd k-means pin this oracle (tests/golden/).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library. The product path (cuvs-rag_amd/) never does.
 */
#ifndef MIVS_ORACLE_H
#define MIVS_ORACLE_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

/* metric codes match include/mivs.h */
#define ORC_L2 0
#define ORC_IP 1

int orc_dim_pad(int d);
/* dot in the mivs k-order (MFMA 32x32x2 f32 chain) */
float orc_dot(const float* a, const float* b, int d);
void orc_norms(const float* x, int64_t n, int d, float* out);
void orc_normalize_rows(const float* x, int64_t n, int d, float* out);
/* key used for ranking: L2 -> clamped expanded squared distance, IP -> -dot */
float orc_key(float dot, float xn, float qn, int metric);

/* exact brute-force kNN (rows of x carry ids = row index + id_offset) */
void orc_refine(const float* x, int64_t n, int d, const float* q, int64_t nq, const int64_t* cand, int nc, int k,
                int metric, float* out_d, int64_t* out_i);
void orc_knn(const float* x, int64_t n, const float* q, int64_t nq, int d, int k, int metric,
             int64_t id_offset, float* out_d, int64_t* out_i);

/* top-k merge of m candidate lists of length kin per query: [nq][m][kin] -> [nq][k] */
void orc_merge(const float* in_d, const int64_t* in_i, int64_t nq, int m, int kin, int k, int metric,
               float* out_d, int64_t* out_i);

/* k-means (Lloyd) on rows x[train_idx[t]] from explicit initial centroids (in/out) */
void orc_kmeans_assign(const float* x, const int64_t* rows, int64_t nr, const float* c, int nc, int d,
                       int metric, int32_t* labels);
void orc_kmeans_update(const float* x, const int64_t* rows, int64_t nr, const int32_t* labels, int nc, int d,
                       float* c /* in: previous, out: updated */);
void orc_kmeans_fit(const float* x, const int64_t* rows, int64_t nr, int nc, int d, int iters, int metric,
                    float* c /* in: init, out: final */);
/* balance != 0: re-seed under-filled clusters after each update except the last two iterations */
void orc_kmeans_fit_ex(const float* x, const int64_t* rows, int64_t nr, int nc, int d, int iters, int metric,
                       int balance, float* c);
void orc_kmeans_rebalance(const float* x, const int64_t* rows, int64_t nr, const int32_t* labels, int nc, int d,
                          int it, float* c);

/* trainset + init selection used by mivs_ivf_flat_build */
int64_t orc_train_count(int64_t n, int n_lists, double fraction, int64_t max_per_list);
void orc_train_rows(int64_t n, int64_t n_train, int64_t* rows);
void orc_init_rows(int64_t n_train, int n_lists, int64_t* which /* indices into train rows */);

/* IVF-Flat build: centroids out [n_lists][d]; list_sizes out [n_lists];
 * list_ids out [n] (lists concatenated in list order, each list by ascending id) */
void orc_ivf_build(const float* x, int64_t n, int d, int n_lists, int iters, double fraction,
                   int64_t max_per_list, int metric, int balance, int64_t id_offset, float* centroids,
                   int64_t* list_sizes, int64_t* list_ids);
void orc_ivf_lists_from_centroids(const float* x, int64_t n, int d, const float* centroids, int n_lists,
                                  int metric, int64_t id_offset, int64_t* list_sizes, int64_t* list_ids);

/* IVF-Flat search over an index given as (centroids, list sizes, list ids) + the source rows;
 * row of id j is x[j - id_offset]. */
void orc_ivf_search(const float* x, int64_t id_offset, int d, const float* centroids, int n_lists,
                    const int64_t* list_sizes, const int64_t* list_ids, const float* q, int64_t nq,
                    int n_probes, int k, int metric, float* out_d, int64_t* out_i, int32_t* out_probes);

/* ---- IVF-PQ (cuVS ivf_pq restated; see mivs_oracle.c) ----
 * codes: [n][pq_dim] uint8 in list order (row t of list storage = list_ids[t]) */
int orc_pq_len(int d, int pq_dim);
int64_t orc_pq_train_count(int64_t n, int pq_bits, int64_t max_per_code);
float orc_pq_l2(const float* a, const float* b, int pl);
float orc_pq_l2_lut(const float* r, const float* b, int pl);
float orc_pq_ip(const float* a, const float* b, int pl);
void orc_ivfpq_train_codebooks(const float* x, int64_t n, int d, const float* centroids, const int32_t* labels,
                               int pq_dim, int pq_bits, int iters, int balance, int64_t max_per_code,
                               float* codebooks);
void orc_ivfpq_encode(const float* x, const int64_t* rows, int64_t nr, int d, const float* centroids,
                      const int32_t* labels, const float* codebooks, int pq_dim, int pq_bits, uint8_t* codes);
void orc_ivfpq_build(const float* x, int64_t n, int d, int n_lists, int iters, double fraction, int pq_dim,
                     int pq_bits, int64_t max_per_code, int balance, int64_t id_offset, float* centroids,
                     float* codebooks, int64_t* list_sizes, int64_t* list_ids, uint8_t* codes);
float orc_round_f16(float v);
void orc_ivfpq_search_ex(const float* centroids, int n_lists, int d, const float* codebooks, int pq_dim, int pq_bits,
                         const int64_t* list_sizes, const int64_t* list_ids, const uint8_t* codes, const float* q,
                         int64_t nq, int n_probes, int k, int metric, float* out_d, int64_t* out_i,
                         int32_t* out_probes, int lut_fp16);
void orc_ivfpq_search(const float* centroids, int n_lists, int d, const float* codebooks, int pq_dim, int pq_bits,
                      const int64_t* list_sizes, const int64_t* list_ids, const uint8_t* codes, const float* q,
                      int64_t nq, int n_probes, int k, int metric, float* out_d, int64_t* out_i,
                      int32_t* out_probes);

/* ---- FAISS-algorithm CPU baseline (cpu_baseline.c; OpenMP, vectorised, NOT bit-exact) ---- */
int orc_fast_threads(void);
void orc_fast_set_threads(int t);
void orc_fast_knn(const float* x, int64_t n, const float* q, int64_t nq, int d, int k,
                  float* out_d, int64_t* out_i);
/* lists given as contiguous row-major list storage + ids + offsets[n_lists+1] */
void orc_fast_ivf_search(const float* list_rows, const int64_t* list_ids, const int64_t* offsets,
                         const float* centroids, int n_lists, int d, const float* q, int64_t nq,
                         int n_probes, int k, float* out_d, int64_t* out_i);
/* dst <- src, first-touched in 2 MiB chunks by every OpenMP thread (NUMA spread of a host copy) */
void orc_parallel_copy(void* dst, const void* src, int64_t nbytes);
/* the ISA the workers run with on this host: "avx512", "avx2+fma" or "x86-64" */
const char* orc_fast_isa(void);

#ifdef __cplusplus
}
#endif
#endif
