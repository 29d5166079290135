/*
 * mivs — MI355X-native IVF-Flat / brute-force k-NN engine: the C-ABI.
 *
 * This is the drop-in boundary for the reference's hot path. The reference
 * (tanujdargan/cuVS-rag) reaches its ANN arithmetic only through four Python
 * call shapes into cuVS 25.6.0; each entry point below
 * names the reference call it replaces. Host code (the Python package cuvs-rag_amd/mivs)
 * binds these with ctypes; INTEGRATION.md shows the binding.
 *
 * Conventions
 *  - every function is re-entrant across devices and returns 0 (MIVS_OK) or
 *    an MIVS_ERR_* code; mivs_last_error() returns a thread-local message;
 *  - `stream` is a hipStream_t passed as void* (NULL = default stream); all
 *    device work of a call is enqueued on it; pointers named d_* are device
 *    pointers on `device` (borrowed, contiguous, row-major), h_* are host;
 *  - results are ordered ascending by (distance, id) for L2 and descending by
 *    inner product (ties: ascending id) for IP; missing results are
 *    id = -1, distance = +inf (L2) / -inf (IP) (FAISS convention);
 *  - arithmetic: DESIGN.md §3 (bit-exact with oracle/).
 */
#ifndef MIVS_H
#define MIVS_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MIVS_OK 0
#define MIVS_ERR_INVALID 1     /* bad argument (shape, k, n_probes, metric ...) */
#define MIVS_ERR_OOM 2         /* hipErrorOutOfMemory (maps to torch.cuda.OutOfMemoryError) */
#define MIVS_ERR_HIP 3         /* any other HIP runtime error */
#define MIVS_ERR_UNSUPPORTED 4 /* valid request outside this build's limits */

#define MIVS_METRIC_L2 0 /* cuVS "sqeuclidean" / FAISS METRIC_L2 */
#define MIVS_METRIC_IP 1 /* cuVS "inner_product" / FAISS METRIC_INNER_PRODUCT */

#define MIVS_MAX_K 4096         /* largest k / n_probes (k > 64 runs the DUMP scan + K8 select path) */
#define MIVS_MAX_REGISTER_K 64 /* largest k served by the register top-k scan + K7 wave merge */

typedef struct mivs_index_s* mivs_index_t;

/* cuvs.neighbors.ivf_flat.IndexParams (index_building_coordinator.py:395 sets only n_lists) */
typedef struct {
  int32_t n_lists;                  /* default in the coordinator: max(1, min(256, N // 1000 + 1)) */
  int32_t metric;                   /* MIVS_METRIC_* */
  int32_t kmeans_n_iters;           /* cuVS default 20 */
  double kmeans_trainset_fraction;  /* cuVS default 0.5 */
  int64_t kmeans_max_train_per_list;/* 0 = no cap; FAISS-style 256 caps the trainset at 256*n_lists */
  int32_t add_data_on_build;        /* cuVS default true */
  int32_t chunk_rows;               /* rows per scan work item (0 = 1024) */
  int32_t kmeans_balance;           /* 1: re-seed under-filled clusters (balanced lists, the role of cuVS's
                                       balanced k-means); 0: plain Lloyd */
  int32_t prefilter;                /* 1: also keep an fp16 copy of the lists for the exact-result fp16
                                       pre-filter search (k <= 16); 0: fp32 scan only */
} mivs_ivf_flat_params;

/* cuvs.neighbors.ivf_pq.IndexParams (index_building_coordinator.py:398-404: n_lists, pq_bits=8,
 * pq_dim=min(64, d // 4); improved_multi_gpu_rag.py:131-137: pq_dim=96, pq_bits=8) */
typedef struct {
  int32_t n_lists;
  int32_t metric;                   /* MIVS_METRIC_L2 (this build) */
  int32_t kmeans_n_iters;           /* coarse and codebook k-means iterations (cuVS default 20) */
  double kmeans_trainset_fraction;  /* coarse trainset fraction (cuVS default 0.5) */
  int32_t pq_dim;                   /* sub-quantizers; pq_len = ceil(dim / pq_dim) dims each */
  int32_t pq_bits;                  /* 8 (256-entry codebooks) in this build */
  int64_t max_train_points_per_pq_code; /* codebook trainset = min(n, this * 2^pq_bits) rows (cuVS 256) */
  int32_t kmeans_balance;
  int32_t add_data_on_build;        /* 1: encode the dataset during build */
} mivs_ivf_pq_params;

/* what the last search on an index did (algorithmic counts for the bench roofline). Searches that run in
 * query batches (K13 above 32,768 queries, large k) report the last batch: n_queries is its size. */
typedef struct {
  int64_t n_queries;
  int32_t n_probes;
  int32_t k;
  int64_t scanned_rows;     /* sum over (query, probed list) of list size: algorithmic rows */
  int64_t streamed_groups;  /* sum over fine-scan work items of 32-row groups streamed from HBM */
  int64_t work_items;       /* fine-scan work items */
  int32_t query_tile;       /* queries per fine-scan work item: 32 (K3 k_scan) or 64 (K3w k_scan_wide) */
  int32_t kcap;             /* register top-k capacity of the fine scan (0: DUMP mode + K8 select) */
  int32_t prefilter;        /* 1: the fp16 pre-filter scan (K10) + exact refine (K11) served the search */
  int64_t overflow_queries; /* queries the refine could not prove, re-run through the exact fp32 scan */
  int64_t window_candidates;/* candidates recomputed in fp32 by the refine (sum over queries) */
  int64_t unique_groups;    /* 32-row groups of the lists probed by at least one query (compulsory bytes) */
  int32_t scan_kernel;      /* fine scan that served it: 3 K3, 31 K3w, 10 K10, 12 K12, 13 K13 */
  int64_t candidates;       /* K13: (approximate key <= T_q, row) pairs appended, all queries */
  int64_t cand_overflow;    /* K13: queries sent to the fallback because a record stream overflowed */
  int64_t spun_out_waves;   /* K13: waves that gave up waiting for a tile (~40 ms; never expected): their
                               batch took the fallback search, as for a stream overflow */
  int32_t copies_skipped;   /* MIVS_COPY_SKIPPED_F8: the index has no fp8 copy (HBM budget): K13's pre-pass ran on
                               the fp16 sample */
} mivs_search_stats;

/* what an index holds in HBM (mivs_index_memory_info). The optional copies are built at build / extend /
 * set_prefilter(1) only while the index stays within MIVS_INDEX_HBM_FRAC (default 0.6) of the device's HBM and 4 GiB
 * stay free beside it; a skipped copy is reported in copies_skipped (the search then takes the path without it). */
#define MIVS_COPY_SKIPPED_F8 1
typedef struct {
  int64_t n_rows;
  int64_t rows_bytes;      /* the fp32 rows (64-B row blocks): the only fp32 copy */
  int64_t side_bytes;      /* row norms, ids, list offsets */
  int64_t centroid_bytes;  /* the coarse centroids */
  int64_t fp16_bytes;      /* the pre-filter's fp16 copy of the rows (+ its per-group minima) */
  int64_t fp8_bytes;       /* K13's pre-pass fp8 copy */
  int64_t pq_bytes;        /* IVF-PQ codes + codebooks */
  int64_t total_bytes;
  int32_t copies_skipped;  /* MIVS_COPY_SKIPPED_* bits */
} mivs_index_memory;
int32_t mivs_index_memory_info(mivs_index_t index, mivs_index_memory* out);

/* device time of the searches issued since the last collect while profiling was on
 * (hipEvents recorded on each call's stream; no host sync inside the calls) */
typedef struct {
  int32_t n_calls;
  float coarse_ms;   /* sum: query norms + coarse probe selection */
  float scan_ms;     /* sum: fine list-scan kernel (the roofline kernel) */
  float scan_ms_min, scan_ms_max;
  float total_ms;    /* sum: whole search call */
} mivs_profile;

const char* mivs_last_error(void);
int32_t mivs_version(void);
/* enable hipEvent timing of search calls (mivs_index_profile_collect); 0 = off */
void mivs_set_profiling(int32_t on);

/* ---- IVF-Flat: replaces cuvs.neighbors.ivf_flat.build (index_building_coordinator.py:396,
 *      improved_multi_gpu_rag.py:130, cuvs-2gpu-main.ipynb:1767) ---- */
int32_t mivs_ivf_flat_build(int32_t device, void* stream, const float* d_data, int64_t n, int32_t dim,
                            const mivs_ivf_flat_params* params, int64_t id_offset, mivs_index_t* out);
/* build lists from given centroids (fixed-centroid parity; FAISS IndexIVFFlat with a trained quantizer) */
int32_t mivs_ivf_flat_build_from_centroids(int32_t device, void* stream, const float* d_data, int64_t n,
                                           int32_t dim, const float* d_centroids, int32_t n_lists,
                                           int32_t metric, int64_t id_offset, int32_t chunk_rows,
                                           mivs_index_t* out);

/* Rebuild an IVF-Flat index from its exported parts: rows [n][dim] and ids [n] in list order (device),
 * per-list sizes [n_lists] (HOST), centroids [n_lists][dim] (device). The lists keep the given order.
 * Replaces the deserialize half of cuvs.neighbors.ivf_flat.save/load (cuvs 25.06, third-party; the
 * reference's FAISS-side equivalent is faiss.read_index, Latest/faiss.ipynb:682-693). */
int32_t mivs_ivf_flat_build_from_lists(int32_t device, void* stream, const float* d_rows, const int64_t* d_ids,
                                       const int64_t* h_list_sizes, int64_t n, int32_t dim, const float* d_centroids,
                                       int32_t n_lists, int32_t metric, int32_t chunk_rows, int32_t prefilter,
                                       mivs_index_t* out);

/* Append n_new rows [n_new][dim] (device) to an IVF-Flat index: each goes to its nearest list (the
 * build's assign) after the list's current rows. d_new_ids == NULL: ids id_offset + n_old ..
 * id_offset + n_old + n_new - 1 (id_offset as given at build).
 * Replaces cuvs.neighbors.ivf_flat.extend (cuvs 25.06; FAISS IndexIVFFlat.add,
 * colab_a100_test.ipynb:479). */
int32_t mivs_ivf_flat_extend(mivs_index_t index, void* stream, const float* d_new, const int64_t* d_new_ids,
                             int64_t n_new);
/* ---- replaces cuvs.neighbors.ivf_flat.search(SearchParams(n_probes), index, q, k)
 *      (improved_multi_gpu_rag.py:225-227, cuvs-2gpu-main.ipynb:1801) ----
 *  d_probes (optional, may be NULL): [nq][n_probes] int32 probed list ids in probe order.
 *  Stream-ordered: the call enqueues on `stream` and may return before the device has finished,
 *  so synchronise `stream` before reading d_distances / d_neighbors on the host. (Some shapes still wait on the host
 *  inside the call -- k > 16, very large batches, an index without the pre-filter copies -- but callers must not
 *  rely on either behaviour.) */
int32_t mivs_ivf_flat_search(mivs_index_t index, void* stream, const float* d_queries, int64_t nq, int32_t k,
                             int32_t n_probes, float* d_distances, int64_t* d_neighbors, int32_t* d_probes);
int32_t mivs_ivf_flat_get_centroids(mivs_index_t index, void* stream, float* d_out /* [n_lists][dim] */);
int32_t mivs_ivf_flat_get_list_sizes(mivs_index_t index, int64_t* h_out /* [n_lists] */);
/* ids / rows of all lists concatenated in list order ([n_rows], [n_rows][dim]) */
int32_t mivs_ivf_flat_get_list_ids(mivs_index_t index, void* stream, int64_t* d_out);
int32_t mivs_ivf_flat_get_list_rows(mivs_index_t index, void* stream, float* d_out);

/* ---- brute force: replaces FAISS IndexFlatL2.add/search (colab_a100_test.ipynb:433-456) and
 *      cuvs.neighbors.brute_force build/search ---- */
int32_t mivs_brute_force_build(int32_t device, void* stream, const float* d_data, int64_t n, int32_t dim,
                               int32_t metric, int64_t id_offset, mivs_index_t* out);
int32_t mivs_brute_force_search(mivs_index_t index, void* stream, const float* d_queries, int64_t nq, int32_t k,
                                float* d_distances, int64_t* d_neighbors);

int32_t mivs_index_info(mivs_index_t index, int64_t* n_rows, int32_t* dim, int32_t* n_lists, int32_t* metric,
                        int32_t* device);
int32_t mivs_index_last_search_stats(mivs_index_t index, mivs_search_stats* out);
int32_t mivs_index_profile_collect(mivs_index_t index, mivs_profile* out);
/* host wall time (s) of the build's phases, recorded when profiling was on during the build (stream syncs
 * between phases): ivf_flat {prepare, coarse k-means, assign + pack, fp16 copy}; ivf_pq {prepare, coarse
 * k-means, assign + sort, codebooks, encode}. *n_out = phases recorded (0: profiling was off). */
int32_t mivs_index_build_phases(mivs_index_t index, double* out_s, int32_t n_max, int32_t* n_out);
/* device time (hipEvents) and algorithmic work of an ivf_flat build's hot kernels, recorded when profiling was on
 * during the build (the build's roofline): per kind its launches, summed ms and work -- flops for the
 * assign scans (2 x rows x centroids x dim per launch), bytes for the rest. Replaces no reference call: it reports on
 * ivf_flat.build (index_building_coordinator.py:392-396). out[k] for k < min(n_max, MIVS_BUILD_KERNEL_KINDS). */
enum {
  MIVS_BUILD_KMEANS_ASSIGN = 0, /* k_as_scan (K13a) in the k-means iterations: flops */
  MIVS_BUILD_FINAL_ASSIGN = 1,  /* k_as_scan for the final assign of every row: flops */
  MIVS_BUILD_KMEANS_UPDATE = 2, /* K5 k_km_partial + k_km_final: bytes (member rows read once) */
  MIVS_BUILD_PACK = 3,          /* K6 k_pack: bytes (rows read, written in the group layout, norms, ids) */
  MIVS_BUILD_FP16_COPY = 4,     /* k_groups_to_half: bytes */
  MIVS_BUILD_FP8_COPY = 5,      /* k_groups_to_f8: bytes */
  MIVS_BUILD_KERNEL_KINDS = 6
};
typedef struct {
  int32_t kind;
  int32_t calls;
  double ms;
  double work;
} mivs_build_kernel;
int32_t mivs_index_build_kernels(mivs_index_t index, mivs_build_kernel* out, int32_t n_max, int32_t* n_out);
/* keep (1) or drop (0) the fp16 copy of the lists that the pre-filter search uses (ivf_flat, brute force).
 * Results are identical either way (the refine recomputes every candidate that can reach the top-k in
 * the pinned fp32 order); the copy costs 2 bytes per padded dimension per row of HBM. */
int32_t mivs_index_set_prefilter(mivs_index_t index, void* stream, int32_t enable);
int32_t mivs_index_get_prefilter(mivs_index_t index, int32_t* enabled);
/* Waits for the calls enqueued on the index (an event per stream they used, not the whole device), then frees its
 * device memory: back to the driver, or into the block cache when its limit allows (mivs_set_block_cache_limit). */
void mivs_index_free(mivs_index_t index);

/* ---- device block cache ----
 * Large engine allocations (>= 64 MB) released by an index or a call may be kept for reuse by later allocations of
 * the process (a fresh hipMalloc of tens of GB can stall for seconds while the driver clears pages). OFF by default:
 * the per-device limit is 0 (MIVS_BLOCK_CACHE_MB at load sets another default). Cached blocks are invisible to
 * torch's allocator and count as used in hipMemGetInfo / torch.cuda.mem_get_info until released.
 * Replaces no reference call: the drop-ins call mivs_release_cached_memory from the reference's cleanup and OOM
 * paths -- cleanup_gpu_resources (Attempt_1/gpu_resource_manager.py:235-255), CUDAMemoryManager's OOM handler
 * (Latest/cuVS-2-gpu/improved_multi_gpu_rag.py:74-97), cleanup_failed_builds / cleanup_all_indices
 * (Attempt_1/index_building_coordinator.py:472-497,583-603) -- before torch.cuda.empty_cache(). */
/* device -1: every device. Lowering the limit frees the blocks above it. */
int32_t mivs_set_block_cache_limit(int32_t device, int64_t bytes);
/* free every cached block of `device` (-1: of every device); *freed_bytes (may be NULL) = bytes returned */
int32_t mivs_release_cached_memory(int32_t device, int64_t* freed_bytes);
/* bytes cached on `device` (-1: all devices) and its limit (-1 for device -1); either pointer may be NULL */
int32_t mivs_cached_memory(int32_t device, int64_t* bytes, int64_t* limit);
/* re-read the engine settings the library caches from the environment (MIVS_FALLBACK_SYNC) */
void mivs_reload_settings(void);

/* ---- IVF-PQ: replaces ivf_pq.build (index_building_coordinator.py:404, improved_multi_gpu_rag.py:137)
 * and ivf_pq.search (improved_multi_gpu_rag.py:228-230). L2, pq_bits 8, k <= 64. Codes live on the
 * device (pq_dim bytes per row); the dataset is only read during build. */
int32_t mivs_ivf_pq_build(int32_t device, void* stream, const float* d_data, int64_t n, int32_t dim,
                          const mivs_ivf_pq_params* params, int64_t id_offset, mivs_index_t* out);
int32_t mivs_ivf_pq_search(mivs_index_t index, void* stream, const float* d_queries, int64_t n_queries, int32_t k,
                           int32_t n_probes, float* d_distances, int64_t* d_neighbors, int32_t* d_probes);
/* pq_dim, pq_bits, pq_len of an IVF-PQ index */
/* The same with cuvs.neighbors.ivf_pq.SearchParams.lut_dtype: MIVS_LUT_FP32 (cuVS's default) or MIVS_LUT_FP16 --
 * every LUT entry rounded to fp16 when stored, row sums in fp32 (L2 metric, pq_len a multiple of 4 in 4..16; else
 * MIVS_ERR_UNSUPPORTED). */
enum { MIVS_LUT_FP32 = 0, MIVS_LUT_FP16 = 1 };
int32_t mivs_ivf_pq_search_ex(mivs_index_t index, void* stream, const float* d_queries, int64_t n_queries, int32_t k,
                              int32_t n_probes, int32_t lut_dtype, float* d_distances, int64_t* d_neighbors,
                              int32_t* d_probes);
int32_t mivs_ivf_pq_info(mivs_index_t index, int32_t* pq_dim, int32_t* pq_bits, int32_t* pq_len);
/* d_out: [pq_dim][2^pq_bits][pq_len] fp32 codebooks */
int32_t mivs_ivf_pq_get_codebooks(mivs_index_t index, void* stream, float* d_out);
/* d_out: [n_rows][pq_dim] uint8 codes in list order (row t belongs to mivs_ivf_flat_get_list_ids()[t]) */
int32_t mivs_ivf_pq_get_codes(mivs_index_t index, void* stream, uint8_t* d_out);

/* ---- k-means (the trainer inside ivf_flat::build; cuvs.cluster.kmeans) ----
 * d_rows: optional [n_train] int64 row ids of the trainset (NULL: rows 0..n_train-1).
 * d_centroids: in = initial centroids, out = centroids after n_iters Lloyd iterations. */
int32_t mivs_kmeans_fit(int32_t device, void* stream, const float* d_data, int64_t n, int32_t dim,
                        const int64_t* d_rows, int64_t n_train, int32_t n_clusters, int32_t n_iters,
                        float* d_centroids);
int32_t mivs_kmeans_predict(int32_t device, void* stream, const float* d_data, int64_t n, int32_t dim,
                            const float* d_centroids, int32_t n_clusters, int32_t metric, int64_t* d_labels);
/* iterations it_begin .. it_begin + n_steps - 1 of the IVF build's k-means (its assign through the fp16
 * pre-filter, the fp64 update and, when balance != 0, the re-seed on all but the last 2 of it_total
 * iterations): the build's trainer one step at a time, for full-size parity checks. d_centroids in/out;
 * d_labels (optional, [n_train] int64): the last step's assignment. */
int32_t mivs_kmeans_steps(int32_t device, void* stream, const float* d_data, int64_t n, int32_t dim,
                          const int64_t* d_rows, int64_t n_train, int32_t n_clusters, int32_t it_begin, int32_t n_steps,
                          int32_t it_total, int32_t balance, float* d_centroids, int64_t* d_labels);

/* ---- K7: merge m sorted candidate lists per query -> top-k (cross-shard merge after the
 *      RCCL all-gather; replaces the host numpy merge at improved_multi_gpu_rag.py:266-275) ----
 * inputs [nq][m][k_in], outputs [nq][k] */
int32_t mivs_merge_topk(int32_t device, void* stream, const float* d_in_dist, const int64_t* d_in_ids, int64_t nq,
                        int32_t m, int32_t k_in, int32_t k, int32_t metric, float* d_out_dist,
                        int64_t* d_out_ids);

/* K7 over an all-gather receive buffer: d_in_* = [parts][nq][k_in] (rank-major, what
 * ncclAllGather / torch all_gather_into_tensor leave), outputs [nq][k]. Same order and padding as
 * mivs_merge_topk. */
int32_t mivs_merge_topk_gathered(int32_t device, void* stream, const float* d_in_dist, const int64_t* d_in_ids,
                                 int32_t parts, int64_t nq, int32_t k_in, int32_t k, int32_t metric,
                                 float* d_out_dist, int64_t* d_out_ids);

/* ---- cross-shard exchange over RCCL (xGMI), single process, one communicator per local device.
 * Replaces the reference's host gather + numpy argsort of the per-GPU results
 * (Latest/cuVS-2-gpu/improved_multi_gpu_rag.py:239-277, cuvs-2gpu-main.ipynb:1820-1834), the merge
 * behind SearchResultAggregator.perform_distributed_search (Attempt_1/test_search_result_aggregator.py:
 * 405-457). RCCL is loaded at mivs_comm_init_all (the copy already in the process, e.g. PyTorch's, when
 * there is one); without it these return MIVS_ERR_UNSUPPORTED. ---- */
typedef struct mivs_comm_s* mivs_comm_t;
/* ncclCommInitAll over devs[0..ndev-1]; rank r = devs[r] */
int32_t mivs_comm_init_all(int32_t ndev, const int32_t* devs, mivs_comm_t* out);
int32_t mivs_comm_size(mivs_comm_t comm, int32_t* ndev);
/* Every rank r contributes its shard's top-k_in (d_dist[r], d_ids[r]: [nq][k_in] on devs[r], ids already
 * global); one grouped ncclAllGather per array, then the K7 merge on every rank whose d_out_dist[r] is
 * non-NULL -> [nq][k] global top-k. streams[r] (NULL = default) orders it after the producer. */
int32_t mivs_merge_topk_allgather(mivs_comm_t comm, void* const* streams, const float* const* d_dist,
                                  const int64_t* const* d_ids, int64_t nq, int32_t k_in, int32_t k,
                                  int32_t metric, float* const* d_out_dist, int64_t* const* d_out_ids);
void mivs_comm_destroy(mivs_comm_t comm);

/* ---- exact re-ranking: replaces cuvs.neighbors.refine(dataset, queries, candidates, k) (cuvs 25.06), the
 * step that makes an IVF-PQ search (improved_multi_gpu_rag.py:228-230) exact over its top-(r*k)
 * candidates. d_data [n][dim] fp32 (or fp16 when data_is_half), d_candidates [nq][n_candidates] row
 * numbers (-1: none); outputs [nq][k] by (distance, id) in the contract's pinned arithmetic. k <= 64. */
int32_t mivs_refine(int32_t device, void* stream, const void* d_data, int32_t data_is_half, int64_t n, int32_t dim,
                    const float* d_queries, int64_t nq, const int64_t* d_candidates, int32_t n_candidates, int32_t k,
                    int32_t metric, float* d_distances, int64_t* d_neighbors);

/* ---- helpers exposed for parity tests and the bench ---- */
int32_t mivs_row_norms(int32_t device, void* stream, const float* d_x, int64_t n, int32_t dim, float* d_out);
/* cosine metric support: d_out[i] = d_x[i] / sqrt(pinned ||x_i||^2), zero rows stay zero (may alias
 * d_x). Replaces the normalisation inside sklearn cosine_similarity / NearestNeighbors(metric='cosine')
 * (Attempt_1/VectorSearch_QuestionRetrieval.ipynb:839,878); ivf_flat / brute_force "cosine" build an
 * inner-product index over normalised rows and report 1 - ip. */
int32_t mivs_normalize_rows(int32_t device, void* stream, const float* d_x, int64_t n, int32_t dim, float* d_out);
int32_t mivs_synth_mixture(int32_t device, void* stream, float* d_out, int64_t row_begin, int64_t n, int32_t dim,
                           uint64_t seed, int32_t n_centers, float sigma, int32_t normalize);

#ifdef __cplusplus
}
#endif
#endif /* MIVS_H */
