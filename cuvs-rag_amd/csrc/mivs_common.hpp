// mivs — MI355X-native IVF-Flat / brute-force k-NN. Shared device/host definitions.
//
// Data layout in HBM:
//   * dims are zero-padded to dp = round_up(d, 32);
//   * rows are stored in GROUPS of 32 rows; inside a group the row-major
//     [32][dp] block is re-ordered as [dp/8][32 rows][8 floats] so that the
//     32x32x2 f32 MFMA operand of one k-step (lane (r,h) needs dims
//     8s+4h..8s+4h+3 of row r) is ONE contiguous 1 KiB wave load;
//   * every inverted list starts on a group boundary; pad rows are zero with
//     norm = +inf and id = -1, so they can never enter a top-k.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mivs {

constexpr int kGroupRows = 32;     // rows per interleaved group (= MFMA M)
constexpr int kQTile = 32;         // queries per work item (= MFMA N)
constexpr int kDimAlign = 64;      // dp = round_up(d, 64): k-steps come in blocks of 8
constexpr int kScanWaves = 8;      // waves per scan workgroup (2 per SIMD)
constexpr int kScanThreads = kScanWaves * 64;
constexpr int kKmChunk = 256;      // members per fp64 partial in the k-means update (== ORC_KM_CHUNK)
constexpr int kDefaultChunkGroups = 32;  // groups (1024 rows) per scan work item
constexpr int kMaxK = 64;          // register top-k capacity of scan + merge kernels
constexpr int kMaxSelectK = 4096;  // largest k / n_probes (K8 select path above kMaxK)

enum Metric : int { kL2 = 0, kIP = 1 };

__host__ __device__ inline int dim_pad(int d) { return (d + kDimAlign - 1) / kDimAlign * kDimAlign; }

// The fp32 rows of every list: groups of 32 rows, inside a group 256-B row blocks
// [dp/64][32 rows][64 floats]. One MFMA k-step of the scans (lane (r, h): dims 8s + 4h .. + 3 of row r) reads
// 32 B of each of the 32 rows, eight k-steps per block, 8 KiB of one group per eight k-steps; a row gather (the
// exact recompute of a candidate) reads whole 256-B blocks, nothing of the neighbour rows.
constexpr int kRowBlk = 64;                          // floats per row block (dp is a multiple of 64)
constexpr int kRowBlkStride = kGroupRows * kRowBlk;  // floats between a row's consecutive blocks
// offset of dim c of a row from its dim 0
__host__ __device__ inline int64_t row_dim(int c) { return (int64_t)(c / kRowBlk) * kRowBlkStride + c % kRowBlk; }
// element offset of dim c of row slot `slot` (g * 32 + r)
__host__ __device__ inline int64_t row_elem(int64_t slot, int c, int dp) {
  return (slot >> 5) * (int64_t)(kGroupRows * dp) + (slot & 31) * kRowBlk + row_dim(c);
}
// offset of a row's 8-dim block b (dims 8b .. 8b + 7) from its dim 0 (row_elem(slot, 0, dp))
__host__ __device__ inline int row_blk8(int b) { return (int)row_dim(8 * b); }
__host__ __device__ inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------------------
// Scan job: (lists of interleaved groups) x (buckets of queries probing them).
// Work item w -> list l (binary search over work_off), then
//   local = w - work_off[l], tiles_l = ceil(m_l / 32),
//   chunk = local / tiles_l, tile = local % tiles_l     (tiles of one chunk adjacent)
// Output slot of bucket entry e for chunk c = bucket_slot[e] + c; each slot
// holds k (dist, id) pairs sorted ascending by (key, id).
// ---------------------------------------------------------------------------
struct ScanArgs {
  const float* groups;        // interleaved rows
  const float* row_norms;     // [total_groups*32]; +inf on pad rows
  const int64_t* row_ids;     // [total_groups*32]; -1 on pad rows
  const int64_t* list_goff;   // [n_lists+1] group offsets
  int n_lists;
  int chunk_groups;           // G
  const float* queries;       // row-major [*, d]
  const float* qnorms;        // indexed by query row id
  const int64_t* bucket_q;    // query row id per bucket entry
  const int64_t* bucket_slot; // output slot base per bucket entry
  const int* bucket_off;      // [n_lists+1]
  const int* work_off;        // [n_lists+1]; total = work_off[n_lists]
  int* work_counter;          // zeroed before launch
  float* out_d;               // [slots][k]; DUMP mode (kcap 0): raw keys [slots][chunk_groups*32]
  int64_t* out_i;             // [slots][k]; DUMP mode: [slots][2] = (first row position, rows)
  int d, dp, k, metric;
  int qtile;                  // queries per work item: 32 (K3) or 64 (K3w)
};

// Large-k select job (K8): per query, the k smallest (key, id) among its candidates.
//   DUMP source (slot_info != nullptr): slots [slot_begin[q], slot_begin[q+1]) (or
//     q*slots_per_q.. when slot_begin == nullptr) of keys[slot][slot_rows], ids from row_ids;
//   EXPLICIT source (slot_info == nullptr): keys = distances [nq][n_in], ids [nq][n_in].
struct SelectArgs {
  const float* keys;
  const int64_t* ids;
  const int64_t* row_ids;
  const int64_t* slot_info;
  const int64_t* slot_begin;
  int64_t slots_per_q;
  int64_t n_in;
  int slot_rows;
  int64_t nq;
  int k, metric;
  float* out_d;
  int64_t* out_i;
};

// Merge job: per query q, candidates = slots [slot_begin[q], slot_begin[q+1])
// (or [q*slots_per_q, (q+1)*slots_per_q) when slot_begin == nullptr), each of
// k_in sorted (dist, id) pairs -> top-k.
struct MergeArgs {
  const float* in_d;
  const int64_t* in_i;
  const int64_t* slot_begin;
  int64_t slots_per_q;
  int64_t nq;
  int k_in, k, metric;
  float* out_d;
  int64_t* out_i;
  // > 0: gathered layout [slots_per_q parts][nq][k_in] with parts part_stride elements apart (the
  // all-gather receive buffer, rank-major); 0: [nq][slots][k_in] / slot_begin as above
  int64_t part_stride;
  // the device-sized exact fallback: only queries q < *nq_dev (<= nq) are merged, and query q's top-k goes to
  // output row out_rows[q] (the unproven query's row in the batch) instead of row q
  const int* nq_dev = nullptr;
  const int64_t* out_rows = nullptr;
};

// IVF-PQ scan job (K9, pq.hip): one workgroup per (query, probe) slot = q * n_probes + p.
struct PqScanArgs {
  const float* queries;        // [nq][d]
  const float* cents;          // [n_lists][d] row-major
  const float* books;          // [pq_dim][256][pq_len]
  const float* book_norms;     // [pq_dim][256] the fmaf chain of b_i b_i (L2 LUT start, oracle orc_pq_l2_lut)
  const uint8_t* codes;        // interleaved groups [g][pq_dim_pad/16][32][16]
  const int64_t* row_ids;      // [groups*32]
  const int64_t* list_off;     // [n_lists+1] rows
  const int64_t* list_goff;    // [n_lists+1] groups
  const int64_t* probes;       // [nq][n_probes] list ids
  int64_t n_slots;             // nq * n_probes
  int n_probes, d, rot_dim_pad, pq_dim, pq_dim_pad, pq_len, k;
  float* out_d;                // [n_slots][k]
  int64_t* out_i;
  int flags;                   // timing experiments only (MIVS_PQ_FLAGS): 1 skip LUT, 2 skip scan, 4 skip merge
  // optional list-sorted order (the probe map with one chunk per list): workgroup b serves entry e
  // (XCD-aware: XCD b % 8 walks its contiguous eighth of the entries), query ent_q[e], output slot
  // ent_slot[e], list = the bucket of e in ent_off. nullptr: workgroup b serves slot b = q*n_probes+p.
  const int64_t* ent_q;
  const int64_t* ent_slot;
  const int* ent_off;          // [n_lists+1]
  int n_lists;
  int pq_half;                 // K9s: subspaces per LUT half (a multiple of 16, 2 * pq_half >= pq_dim)
  int ip;                      // inner product: LUT -(q_j . B_j[c]), coarse term in subspace 0, out = -key
  const float* probes_d;       // IP: [nq][n_probes] coarse distances q . c_l (K3, the probes' order)
  int dump_rows;               // K9 DUMP (kcap 0, k > 64): out_d is [n_slots][dump_rows] keys
  int64_t* slot_info;          //   and slot_info [n_slots][2] = (first row position, rows)
};

// IVF-PQ tiled scan (K9b, pq.hip): work item = (list, <= 16 queries, 512-row chunk) from the probe map.
constexpr int kPqTileQueries = 16;
constexpr int kPqChunkGroups = 16;  // 512 rows
struct PqTileArgs {
  const float* queries;
  const float* cents;
  const float* books;
  const float* book_norms;  // [pq_dim][256] (PqScanArgs)
  // K9r's MFMA LUT operands [pq_dim][256][4][pq_len/4]: entry (j, c) dim 4s + g at g * pq_len/4 + s, scaled
  // by -2 (L2) or -1 (IP) -- exact (pq_book_prep)
  const float* books_mfma;
  const uint8_t* codes;
  const int64_t* row_ids;
  const int64_t* list_off;
  const int64_t* list_goff;
  int n_lists;
  const int64_t* bucket_q;
  const int64_t* bucket_slot;
  const int* bucket_off;
  const int* work_off;
  int* work_counter;
  int d, rot_dim_pad, pq_dim, pq_dim_pad, pq_len, k;
  float* out_d;     // [slots][k]
  int64_t* out_i;
  // K9r only (k_pq_scan_rt): inner product (the probes' coarse keys by list id), DUMP mode outputs
  int ip;
  const int64_t* probes;    // [nq][n_probes]
  const float* probes_d;    // [nq][n_probes]
  int n_probes;
  int64_t* slot_info;       // DUMP: [slots][2] = (first row position, rows); out_d is [slots][kRtRows]
  int flags;                // timing experiments only (MIVS_PQ_FLAGS): 1 skip LUT build, 2 skip row scan
  int lut16 = 0;            // K9r: LUT entries stored as fp16 (cuvs SearchParams.lut_dtype = float16; L2 only)
  // K9r, kMaxK < k <= kRtCandMax: each (query, chunk) slot receives a SUPERSET of its top-k by (key, id), unsorted,
  // slot_cap entries (id -1 past its end), which K8 ranks over the query's slots (EXPLICIT with slot_begin)
  int slot_cap = 0;
};

// K9r (k_pq_scan_rt, pq.hip): work item = (list, <= 16 queries probing it, chunk of kRtRows rows); the
// 16 queries' LUT of one subspace ([code][query], 80-B rows) in LDS, each of 512 threads holds 8 rows x
// 16 queries of sums in registers
constexpr int kRtThreads = 512;
constexpr int kRtQ = 16;
constexpr int kRtRpt = 8;
constexpr int kRtRows = kRtThreads * kRtRpt;  // 4096
constexpr int kRtGroups = kRtRows / 32;
constexpr int kRtCandMax = 256;  // K9r candidate-superset slots up to this k (the refine's 12 x k candidates); DUMP above
constexpr int kRtSlotCap = 256;  // entries per candidate-superset slot (>= kRtCandMax)
size_t pq_rt_lds_bytes(int rot_dim_pad, int pq_dim, int k, bool lut16 = false);
// book_norms and books_mfma from the codebooks (after training; pq.hip)
hipError_t launch_pq_book_prep(const float* books, int pq_dim, int pq_len, int ip, float* book_norms,
                               float* books_mfma, hipStream_t s);
bool pq_rt_supported(int rot_dim_pad, int pq_dim, int pq_len, int k);
hipError_t launch_pq_scan_rt(const PqTileArgs& a, int grid, hipStream_t s);

// ---------------------------------------------------------------------------
// fp16 pre-filter + exact refine (prefilter.hip).
//   K10 scans an fp16 copy of the lists (same group layout, scaled by 2^hx_exp)
//   against fp16 queries (per-query scale) with v_mfma_f32_32x32x16_f16 and keeps,
//   per (query, probe, chunk) slot, the slot_k smallest APPROXIMATE keys + a
//   lower bound of every key it dropped. K11 then takes, per query, every
//   candidate whose approximate key is within 2*delta of the k-th (delta = a
//   rigorous bound on |approx key - pinned fp32 key|), recomputes those in the
//   pinned fp32 order and emits the exact top-k. Queries whose dropped-key bound
//   reaches the window are listed for the exact scan (never silently wrong).
// ---------------------------------------------------------------------------
constexpr int kPfQTile = 64;     // queries per K10 work item
constexpr int kPfLaneK = 8;      // per-lane approximate list length in K10
constexpr int kPfSlotKMax = 32;  // approximate candidates kept per slot: 16 for k <= 10, else 32
constexpr int kPfMaxK = 16;      // largest k served by the pre-filter path
constexpr int kPfRefineMaxK = 32;  // largest k K11 ranks (the pre-filter search itself serves k <= kPfMaxK)
constexpr int kPfCap = 64;       // refine capacity (window candidates per query)
constexpr int kPfSelRegs = 8;    // K11 phase 1: candidates per query held in registers (x 64) for the radix select
constexpr int kPfChunkGroups = 512;  // default groups (16384 rows) per K10 work item (MIVS_PF_CHUNK_ROWS)

struct PfScanArgs {
  const uint16_t* groups_h;   // fp16 lists, group layout [g][dp/8][32][8]
  const float* row_norms;     // pinned fp32 norms (+inf on pad rows)
  const int64_t* list_goff;
  int n_lists;
  int chunk_groups;
  const uint16_t* qh;         // fp16 queries [nq][dp], query q scaled by 2^qexp[q]
  const float* qscale;        // 2^-(hx_exp + qexp[q]): fp16 dot -> approximate fp32 dot (exact scaling)
  const float* qnorms;        // pinned fp32 query norms
  const int64_t* bucket_q;
  const int64_t* bucket_slot;
  const int* bucket_off;
  const int* work_off;
  int* work_counter;          // [8 queues x 16] (one cache line each), zeroed before launch
  float* slot_key;            // [slots][slot_k] ascending approximate keys (+inf: empty)
  int* slot_pos;              // [slots][slot_k] row positions
  float* slot_bound;          // [slots] every dropped candidate's approximate key is >= this
  int slot_k;
  int slot_out;               // > 0: a slot's merge stops after this many keys (and their ties) -- the pre-pass's
                              // nomination, whose verify reads only the best verify_sel of a slot; 0: slot_k
  int dp, metric;
  const float* qres;          // [nq] ||q - q_h|| (the window bound theta of the scan)
  float x_norm_max, x_res_max;
  unsigned* qtheta;           // [nq] order-mapped window bound per query, shared by all work items
                              // (set to the mapping of +inf before the launch)
  int k;
  int flags;                  // timing experiments only (MIVS_PF_FLAGS): 1 skip epilogue, 8 skip staging,
                              // 16 skip merge, 32 phase clocks into prof
  unsigned long long* prof;   // [16] diagnostic phase clocks, or nullptr
  int no_theta;               // 1: no query has another work item (one list, one chunk): skip qtheta updates
  int* chunk_pos;             // [n_lists * chunk_stride] K10 convoy: the pair a chunk's tiles are scanning
                              // (zeroed before launch), or nullptr (every tile scans from pair 0)
  int chunk_stride;           // max chunks per list
  int rows_nt;                // 1: the rows are read once (K13's pre-pass: one tile per list sample) -- load them
                              // with the non-temporal policy (pair mode only)
  int raw_lists;              // 1: no per-slot merge -- each slot is the query's 16 lane lists as they are (slot_k =
                              // 16 x kPfLaneK, unsorted, +inf padded) and its bound; K11 / K11v rank every entry
  const uint8_t* groups_f8;   // optional (K13's pre-pass nomination, pair mode): fp8 rows (launch_groups_to_f8);
  const uint8_t* q8;          //   then the fp8 queries (launch_queries_to_f8) and their scales replace groups_h,
  const float* qscale8;       //   qh and qscale
};

// K13 row-stationary pre-filter scan (rsscan.hip): work item = (list, block of
// kRsBlockGroups groups), one group per wave held in registers, the list's queries streamed past in
// kRsQTile-query tiles; every (approximate key <= T_q, row) goes to the query's candidate buffer.
constexpr int kRsWaves = 8;
constexpr int kRsQTile = 32;
constexpr int kRsBlockGroups = kRsWaves;
// K13's pre-pass scans the first 1 / kRsPreDiv of each query's nearest list (MIVS_RS_PRE_DIV); with the fp8 copies
// (MIVS_RS_PRE_F8, default) the sample is scored on fp8 rows and queries over every dim and the kRsPreSel best rows
// of each query are verified with fp32 keys
constexpr int kRsPreDiv = 4;
constexpr int kRsPreDivF8 = 4;
constexpr int kRsPreSel = 10;
// K13 one-pass bucketing: least candidates per query run (MIVS_RS_QCAP), and the batch's runs: 256M entries (2 GiB of
// key + position). A query past its run's capacity is unproven and takes the exact fallback (~0.2 ms each at configs[2]):
// at 1 GiB / 4,096 a 32,768-query batch had 13 of them (profiles/r05_qsweep.txt)
constexpr int kRsQCap = 8192;
constexpr int64_t kRsCandBudget = int64_t(1) << 28;
constexpr int kRsWaveCapMax = 16384;  // records of a K13 wave's candidate stream (more: all queries fall back)
constexpr int kRsWaveCapMaxLk = 1 << 18;  // the same for large k (K16: thousands of candidates per query)
constexpr int kRsRecInt4 = 3;         // a record: 8 dots of one lane and query half + {first row position, query}
constexpr int kRsMaxBatch = 32768;    // queries per K13 search batch (the LDS-histogram bucketing's bins)

struct RsScanArgs {
  const uint16_t* groups_h;  // fp16 lists, group layout [g][dp/8][32][8]
  const float* row_norms;    // pinned fp32 norms (+inf on pad rows)
  const int64_t* list_goff;
  int n_lists;
  const int64_t* bucket_q;   // probe map with chunk = kRsBlockGroups groups and one query tile per list
  const int* bucket_off;
  const int* work_off;
  const int4* items;         // [items] {first group, end group, first tile slot, tiles} (k_rs_items)
  const char* tiles;         // query tile images (k_rs_tiles): per list ceil(m/32) x [dp/16 + 1] x 1 KiB
  const float* qnorms;       // [nq] pinned fp32 query norms (exact key of a candidate)
  int nq;
  int metric;
  const float* group_nmin;   // [groups] the smallest row norm of each group (L2 filter bound)
  int4* wave_buf;            // [grid * kRsWaves][wave_cap][kRsRecInt4] per-wave record streams
  int wave_cap;              // records per stream
  int* wave_cnt;             // [grid * kRsWaves] stream lengths (may exceed wave_cap: records lost)
  int* queue;                // [8] per-queue item counters, zero at launch (dynamic dealing)
  const int* bounds;         // [9] the queues' item ranges by tile work (k_rs_bounds)
  int flags;                 // timing experiments only (MIVS_RS_FLAGS): 1 skip epilogue, 2 skip staging,
                             // 4 keep the rows at item transitions, 8 per-block clocks into prof, 16 phase clocks
  unsigned long long* prof;  // flags & 8: [grid][3] {start, end, tiles}
};

// K16 large-k search through the pre-filter (largek.hip): K13's candidates -> per query the refine
// window (K16w) -> pinned fp32 keys of the window rows (K16r) -> (key, id) sort and the first k (K16s)
constexpr int kCopySkippedF8 = 1;  // == MIVS_COPY_SKIPPED_F8
constexpr int kLkMaxCap = 8192;    // window rows per query at most (more: the exact scan)
constexpr int kLkSampleDiv = 64;   // T_q's sample: the first 1 / kLkSampleDiv of every probed list (MIVS_LK_SAMPLE_DIV)
constexpr float kLkSampleZ = 4.0f; // sample rank margin in standard deviations (binomial)
struct LkArgs {
  const int64_t* cand_off;  // [nq + 1] K13's per-query candidate runs
  const float* cand_key;    // approximate keys
  const int* cand_pos;      // row positions
  const float* tq;          // [nq] T_q (+inf: every probed row is a candidate)
  const float* qnorms;      // [nq] pinned query norms
  const float* qres;        // [nq] ||q - q_h||
  float x_norm_max, x_res_max;
  int d, dp, k, cap, metric;
  int64_t nq;
  const int* force_ovf;     // optional: nonzero -> no query is provable (K13 lost records)
  int* win_pos;             // [nq][cap] window row positions
  float* win_key;           // [nq][cap] their pinned keys
  int* win_n;               // [nq] window rows (-1: the query takes the exact scan)
  int* ovf_count;
  int64_t* ovf_q;
  int64_t* n_window;        // optional: total window rows (stats)
  const int64_t* chunk_off; // [nq + 1] exclusive prefix of the windows' 64-row chunks (K16r's items)
  const float* groups;      // fp32 rows (row_elem layout)
  const float* row_norms;
  const int64_t* row_ids;
  const float* queries;     // fp32 [nq][d]
  float* out_d;
  int64_t* out_i;
};
int lk_cap(int k);
hipError_t launch_lk_sample_probes(const int64_t* probes, int64_t n, int64_t* out, hipStream_t s);
constexpr int kLkMaxSampleSlots = 1024;  // K3 DUMP slots of one query's sample (more: T_q = +inf)
// T_q's key per query: the r_q-th smallest key of the sample's DUMP slots (r_q from the binomial margin)
hipError_t launch_lk_sample_kth(const int64_t* probes, int64_t nq, int np, const int64_t* list_off, const int64_t* goff2,
                                int k, float z, const float* keys, const int64_t* slot_info, const int64_t* slot_begin,
                                int slot_rows, float* kth, hipStream_t s);
hipError_t launch_lk_window(const LkArgs& a, hipStream_t s);
hipError_t launch_lk_chunks(const int* win_n, int64_t nq, int64_t* chunks, hipStream_t s);
hipError_t launch_lk_recompute(const LkArgs& a, int cus, hipStream_t s);  // cus: the device's CUs
hipError_t launch_lk_sort(const LkArgs& a, hipStream_t s);

// K13a k-means assign on the row-stationary loop (assign.hip)
struct AsScanArgs {
  const uint16_t* qh;        // data rows fp16 [n][dp], row r scaled by its own power of two (k_queries_to_half)
  const float* qscale;       // [n] 2^-(hx + row exp): the fp16 dot -> approximate fp32 dot
  const float* qnorms;       // [n] pinned fp32 norms of the data rows
  const float* qres;         // [n] ||x - x_h|| of the data rows
  const int64_t* rows;       // optional: assign row r is data row rows[r] (the k-means trainset), else r
  int64_t nr;                // rows to assign
  const char* ctiles;        // centroid tile images (k_as_ctiles): [n_ctiles][dp/16 + 1] x 1 KiB
  int n_ctiles;              // tiles of 32 centroids (> 1)
  const unsigned* cstat;     // {max pinned centroid norm, max ||c - c_h||} as float bits (k_as_ctiles)
  int dp;
  int64_t* labels;           // [nr] the argmin of every proven row
  int* ovf_count;            // [2] rows handed to the exact scan; [1] != 0: a wait gave up (rerun every row)
  int64_t* ovf_rows;         // [nr] those rows (assign-row indices)
  int* queue;                // item counter, zero at launch
  int flags;                 // timing only: 2 skip staging
};
bool as_scan_supported(int dp, int64_t n_centroids);
size_t as_ctiles_bytes(int64_t n_groups, int dp);
hipError_t launch_as_ctiles(const float* groups, const float* norms, int64_t n_groups, int dp, int hx, char* tiles,
                            unsigned* stat, hipStream_t s);
hipError_t launch_as_scan(const AsScanArgs& a, int grid, hipStream_t s);

// K14 exact re-ranking of candidates (refine.hip): cuvs.neighbors.refine
struct RefineArgs {
  const void* data;       // [n][d] fp32, or fp16 when half
  int64_t n;
  int d, dp;              // dp = the contract's padded dim (multiple of 64, <= 1024)
  int half;
  const float* queries;   // [nq][d]
  int64_t nq;
  const int64_t* cand;    // [nq][n_cand] row numbers of data (-1: none)
  int n_cand;
  const int64_t* id_map;  // optional: reported id of row r (default r)
  int k, metric;
  float* out_d;
  int64_t* out_i;
};

struct PfRefineArgs {
  const float* slot_key;
  const int* slot_pos;
  const float* slot_bound;
  const int64_t* slot_begin;  // [nq+1]
  int slot_k;
  int64_t nq;
  int k, d, dp, metric;
  const float* groups;        // fp32 lists (row_elem layout) for the exact recompute
  const float* row_norms;
  const int64_t* row_ids;
  const float* queries;       // fp32 [nq][d]
  const float* qnorms;
  const float* qres;          // [nq] ||q - q_h|| (fp16 rounding residual, unscaled)
  float x_norm_max, x_res_max;  // max ||x||, max ||x - x_h|| over the index rows
  float* out_d;
  int64_t* out_i;
  int* ovf_count;             // queries that need the exact scan
  int64_t* ovf_q;
  int64_t* n_window;          // optional: total window candidates (stats)
  const int64_t* qrows;       // optional: query q is row qrows[q] of queries / qnorms / qres (k-means trainset)
  int labels_only;            // k = 1: a window of ONE candidate is the answer without its exact key
                              // (out_d then holds its approximate key)
  const int* force_ovf;       // optional (K13): nonzero -> no query is provable (candidates were lost)
  const float* window_cap;    // optional (K13): [nq] T_q -- a query whose window exceeds it is not proven
  float* kth_out;             // optional (K13's pre-pass): only the k-th smallest approximate key per query
                              // (+inf: fewer than k candidates), no refine
  int verify_sel;             // with kth_out: > 0 -> the candidates with the verify_sel smallest keys (nomination
                              // scores) get fp32 keys (within delta of their pinned keys), and kth_out is the k-th
                              // smallest of THOSE
  const int* slot_cnt;        // optional (K13's one-pass bucketing): query q's run is [q * slot_cap, + min(cnt, cap))
  int slot_cap;               // instead of slot_begin; cnt > cap: candidates were dropped, the query is not proven
};

hipError_t launch_pf_scan(const PfScanArgs& a, int grid, size_t lds, hipStream_t s);
size_t pf_scan_lds_bytes(int dp, int chunk_groups);
bool pf_pair_mode();  // K10 two groups per pass (default; MIVS_PF_PAIR=0: one), which also frees the chunk
                      // size from LDS (the row norms are loaded per pass)
constexpr int kPfMaxPairGroups = 1 << 15;  // K10 chunk cap in pair mode (1M rows; positions stay int)
// K12: register-resident 128-query tiles, LDS-DMA row ring (dp/16 in {4,8,12,16,24,32,48})
constexpr int kPrQTile = 128;
constexpr int kPrSlotK = 16;  // K12 slot: the query's 4 lane lists of 4 approximate candidates
constexpr int kPrChunkGroups = 256;  // default groups (8192 rows) per K12 work item (MIVS_PR_CHUNK_ROWS)
bool pr_scan_supported(int dp);
hipError_t launch_pr_scan(const PfScanArgs& a, int grid, hipStream_t s);
hipError_t launch_pf_refine(const PfRefineArgs& a, hipStream_t s);
hipError_t launch_refine(const RefineArgs& a, hipStream_t s);
// engine switches the kernel launchers read: the environment variable's integer value, read once and
// kept until mivs_reload_settings (capi.cpp) -- one getenv per process, not per call
enum EngineSetting { kSetRefineGather = 0, kSetSelectSlotsWave = 1, kSetPfRawLists = 2, kSetCount = 3 };
int engine_setting(EngineSetting id, const char* name, int dflt);
void engine_settings_reset();
size_t rs_scan_lds_bytes(int dp);
bool rs_scan_supported(int dp);
hipError_t launch_rs_scan(const RsScanArgs& a, int dp, int grid, hipStream_t s);
int64_t rs_tiles_bytes(int64_t ne, int n_lists, int dp);
// order one wave's LDS stores before its later LDS loads (and the loads before later stores) across its lanes: a
// wave-scope release/acquire pair around a wave barrier, so an LDS hand-off between lanes of one wave does not depend
// on the compiler keeping the accesses in program order
__device__ inline void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// block-wide exclusive scan of one value per thread (returns exclusive prefix, total via *tot)
__device__ inline int64_t block_excl_scan(int64_t v, int64_t* sh, int64_t* tot) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = blockDim.x >> 6;
  int64_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int64_t y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  if (lane == 63) sh[wave] = x;
  __syncthreads();
  if (wave == 0) {
    int64_t s = lane < nw ? sh[lane] : 0;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int64_t y = __shfl_up(s, o);
      if (lane >= o) s += y;
    }
    if (lane < nw) sh[lane] = s;  // inclusive wave totals
  }
  __syncthreads();
  const int64_t base = wave > 0 ? sh[wave - 1] : 0;
  if (tot) *tot = sh[nw - 1];
  __syncthreads();
  return base + x - v;
}

// K13's per-wave record streams -> per-query CSR runs (cand_off [nq + 1]) of (approximate key, row position);
// tmp >= rs_bucket_tmp_bytes; lost: set when a stream overflowed; grid: workgroups of the flat count / scatter
size_t rs_bucket_tmp_bytes(int nq, int n_waves);
hipError_t launch_rs_bucket(const int4* wave_buf, int wave_cap, const int* wave_cnt, int n_waves, int nq,
                            const float4* qhdr, const float* row_norms, int metric, int64_t* cand_off,
                            float* cand_key, int* cand_pos, void* tmp, int* lost, int grid, hipStream_t s,
                            void* zero2 = nullptr, int zero2_bytes = 0);  // (zero2: also zeroed, 16-B words)
// the same in two halves (large k sizes the candidate arrays from cand_off[nq] between them): count -> cand_off,
// then the scatter
hipError_t launch_rs_bucket_count(const int4* wave_buf, int wave_cap, const int* wave_cnt, int n_waves, int nq,
                                  const float4* qhdr, const float* row_norms, int metric, int64_t* cand_off, void* tmp,
                                  int* lost, hipStream_t s, void* zero2 = nullptr, int zero2_bytes = 0);
// one pass (the k <= 16 path): each query's candidates go to a fixed-capacity run [q * cap, q * cap + qcnt[q]) (entries
// past cap are dropped and counted: K11 then proves nothing for that query); qcnt [nq] must be zero on entry
hipError_t launch_rs_bucket_fused(const int4* wave_buf, int wave_cap, const int* wave_cnt, int n_waves, int nq,
                                  const float4* qhdr, const float* row_norms, int metric, int cap, int* qcnt,
                                  float* cand_key, int* cand_pos, hipStream_t s);
hipError_t launch_rs_bucket_scatter(const int4* wave_buf, int wave_cap, const int* wave_cnt, int n_waves, int nq,
                                    const float4* qhdr, const float* row_norms, int metric, const int64_t* cand_off,
                                    float* cand_key, int* cand_pos, void* tmp, hipStream_t s);
// fp8 (e4m3) copies for K13's pre-pass nomination: rows at scale 2^hx8 in the operand layout of
// k_pf_scan<.., F8> (dp % 32 == 0), queries at their own power of two (qscale8[q] = the fp8 dot -> fp32 dot)
hipError_t launch_groups_to_f8(const float* groups, int64_t n_groups, int dp, int hx8, uint8_t* out, hipStream_t s);
hipError_t launch_queries_to_f8(const float* q, int64_t nq, int d, int dp, int hx8, uint8_t* out, float* qscale8,
                                hipStream_t s);
// per group of 32 rows the smallest row norm (K13's filter bound)
hipError_t launch_group_nmin(const float* norms, int64_t n_groups, float* out, hipStream_t s);
hipError_t launch_rs_pre_lists(const int64_t* goff, int n_lists, int div, int min_groups, const int64_t* probes,
                               int64_t nq, int np, int64_t* goff2, int64_t* probes2, hipStream_t s);
hipError_t launch_rs_items(const int* work_off, const int* bucket_off, const int64_t* list_goff, int n_lists,
                           int max_items, int4* items, int* bounds, hipStream_t s,
                           int* zero = nullptr, int nzero = 0);
hipError_t launch_rs_tiles(const int64_t* bucket_q, const int* bucket_off, int n_lists, int64_t ne, const uint16_t* qh,
                           const float4* qhdr, int nq, int dp, char* tiles, hipStream_t s);
// tq (optional): T_q per query, the bound K11 checks its final window against
hipError_t launch_rs_headers(const float* pre_kth, int64_t nq, const float* qscale, const float* qnorms,
                             const float* qres, float x_norm_max, float x_res_max, int dp, int metric, float4* hdr,
                             float* tq, hipStream_t s, int* zero = nullptr, int64_t nzero = 0,
                             int* zero2 = nullptr, int nzero2 = 0);
hipError_t launch_gather_ids(const int64_t* src, const int64_t* idx, int64_t n, int64_t* out, hipStream_t s);
constexpr unsigned kPfOrdInf = 0xFF800000u;  // order mapping of +inf (qtheta's initial value)
// fp32 groups -> fp16 groups scaled by 2^hx_exp (FTZ below the fp16 normal range), per-index maxima of
// ||x - x_h|| and max |x| (as float bits, atomicMax) into stats[0..1] (zeroed by the caller)
hipError_t launch_groups_to_half(const float* groups, int64_t n_groups, int dp, int hx_exp, uint16_t* out,
                                 unsigned* stats, hipStream_t s);
hipError_t launch_abs_max(const float* x, int64_t n, unsigned* out, hipStream_t s);
hipError_t launch_norm_max(const float* norms, int64_t n, unsigned* out, hipStream_t s);
// queries fp32 [nq][d] -> fp16 [nq][dp] with a per-query power-of-two scale, qscale = 2^-(hx_exp+e_q),
// qres = ||q - q_h|| (unscaled)
hipError_t launch_queries_to_half(const float* q, int64_t nq, int d, int dp, int hx_exp, uint16_t* qh, float* qscale,
                                  float* qres, hipStream_t s);
int pf_hx_exp(float abs_max);  // row-side fp16 scale exponent from max |x|
hipError_t launch_scatter_results(const float* in_d, const int64_t* in_i, const int64_t* rows, int64_t n, int k,
                                  float* out_d, int64_t* out_i, hipStream_t s);

// ---- host-side launchers (implemented in the .hip files) ----
hipError_t launch_scan(const ScanArgs& a, int kcap, int grid, size_t lds_bytes, hipStream_t s);
hipError_t launch_scan_ex(const ScanArgs& a, int kcap, int grid, size_t lds_bytes, float* gmerge, hipStream_t s);
size_t scan_lds_bytes(int dp, int kcap, int chunk_groups);
bool scan_merge_in_lds(int dp, int kcap, int chunk_groups);
size_t scan_gmerge_bytes(int grid, int kcap);
// K3w: 64-query tiles with slab-staged queries (scan_wide.hip)
size_t scan_wide_lds_bytes(int kcap, int chunk_groups);
bool scan_wide_supported(int kcap, int d, int dp, int chunk_groups);
hipError_t launch_scan_wide(const ScanArgs& a, int kcap, int grid, size_t lds_bytes, hipStream_t s);
// workgroups of the scan kernel resident per CU at this LDS request (hipOccupancy: LDS + registers)
int scan_occupancy(int kcap, int metric, size_t lds_bytes);
int scan_wide_occupancy(int kcap, int metric, size_t lds_bytes);
int scan_kcap(int k);
int scan_waves(int kcap);  // waves per K3 workgroup for this register list length
hipError_t launch_train_rows(int64_t* rows, int64_t n, int64_t n_train, hipStream_t s);
hipError_t launch_i64_to_i32(const int64_t* in, int64_t n, int32_t* out, hipStream_t s);
hipError_t launch_merge(const MergeArgs& a, hipStream_t s);
hipError_t launch_select(const SelectArgs& a, hipStream_t s);

hipError_t launch_pack_groups(const float* src, int64_t src_rows_total, int d, int dp, const int64_t* src_index,
                              const int64_t* list_off, const int64_t* list_goff, const int* group_list,
                              int64_t n_groups, float* groups, float* norms, int64_t* ids_out,
                              const int64_t* id_map, int64_t id_offset, hipStream_t s);
hipError_t launch_row_norms(const float* x, int64_t n, int d, float* out, hipStream_t s);
// one pass over the query batch: norms (launch_row_norms), fp16 copy (launch_queries_to_half) and, q8 != nullptr,
// fp8 copy (launch_queries_to_f8); d % 4 == 0 and 16-B aligned rows
hipError_t launch_queries_prep(const float* q, int64_t nq, int d, int dp, int hx_exp, int hx8, float* qn, uint16_t* qh,
                               float* qscale, float* qres, uint8_t* q8, float* qscale8, hipStream_t s);
// cosine: out = x / sqrt(pinned ‖x‖²) per row (zero rows stay zero); n2: [n] scratch (the squared norms)
hipError_t launch_normalize_rows(const float* x, int64_t n, int d, float* n2, float* out, hipStream_t s);
hipError_t launch_iota_i64(int64_t* out, int64_t n, int64_t start, int64_t step, hipStream_t s);
hipError_t launch_fill_i32(int* out, int64_t n, int v, hipStream_t s);
hipError_t launch_fill2_i32(int* o1, int64_t n1, int v1, int* o2, int64_t n2, int v2, hipStream_t s);

// single-list job prep: bucket = identity over nq queries, slot base = q * chunks
hipError_t launch_single_list_job(int64_t nq, int64_t chunks, int qtile, int64_t* bucket_q, int64_t* bucket_slot,
                                  int* bucket_off, int* work_off, int64_t* slot_begin, hipStream_t s, int* zero = nullptr);
// The exact fallback's probe map sized on the device: entries (i, p) for i < min(*n_dev, cap) are probe p of query
// ovf_q[i] in probes [.][np]; bucket_q holds the query's own row, bucket_slot / slot_begin number the slots by i.
// One workgroup (n_lists <= probe_map_dev_max_lists()); zero: the scan's work counter, zeroed here.
int probe_map_dev_max_lists();
hipError_t launch_probe_map_dev(const int* n_dev, int64_t cap, const int64_t* ovf_q, const int64_t* probes, int np,
                                int n_lists, const int64_t* list_goff, int chunk_groups, int qtile, int* counts,
                                int* bucket_off, int* work_off, int64_t* bucket_q, int64_t* bucket_slot,
                                int64_t* slot_begin, int* zero, hipStream_t s);
// IVF probe map: probes [nq][np] (int64 list ids) -> buckets, work offsets, slot bases
hipError_t launch_probe_map(const int64_t* probes, int64_t nq, int np, int n_lists, const int64_t* list_goff,
                            int chunk_groups, int qtile, int* counts, int* fill, int* bucket_off, int* work_off,
                            int64_t* bucket_q, int64_t* bucket_slot, int64_t* qp_slots, int64_t* slot_begin,
                            void* scan_tmp, size_t scan_tmp_bytes, hipStream_t s);

// device-wide exclusive scan (int64) — tmp >= scan_tmp_bytes(n)
size_t scan_tmp_bytes(int64_t n);
hipError_t launch_exclusive_scan_i64(const int64_t* in, int64_t* out, int64_t n, void* tmp, hipStream_t s);

// stable counting sort of positions 0..n-1 by label (labels int64 in [0, nl))
size_t csort_tmp_bytes(int64_t n, int nl);
hipError_t launch_counting_sort(const int64_t* labels, int64_t n, int nl, int64_t* perm /*[n]*/,
                                int64_t* list_off /*[nl+1]*/, void* tmp, size_t tmp_bytes, hipStream_t s);

// k-means deterministic update
hipError_t launch_km_update(const float* x, int d, const int64_t* rows, const int64_t* perm,
                            const int64_t* list_off, int nc, int64_t n_members, double* partial,
                            int64_t* chunk_off, void* tmp, float* centroids, hipStream_t s);
size_t km_partial_rows(int64_t n_members, int nc);
constexpr int kBalanceKeepLast = 2;  // last k-means iterations without re-seeding (== ORC_BAL_KEEP_LAST)
hipError_t launch_km_rebalance(const float* x, int d, const int64_t* rows, const int64_t* labels,
                               const int64_t* list_off, int nc, int64_t n_train, int it, float* centroids,
                               hipStream_t s);

// IVF-PQ (pq.hip)
size_t pq_scan_lds_bytes(int rot_dim_pad, int pq_dim, int kcap);
hipError_t launch_pq_residuals(const float* x, int d, const int64_t* rows, int64_t nt, const int64_t* labels,
                               const float* cents, int pq_dim, int pl, float* out, hipStream_t s);
hipError_t launch_pq_encode(const float* x, int d, const int64_t* perm, int64_t n, const int64_t* list_off,
                            const int64_t* list_goff, int n_lists, const float* cents, const float* books, int pq_dim,
                            int pl, int pq_dim_pad, uint8_t* codes, hipStream_t s);
hipError_t launch_pq_ids(const int64_t* perm, int64_t n, const int64_t* list_off, const int64_t* list_goff,
                         int n_lists, int64_t id_offset, int64_t* ids, hipStream_t s);
hipError_t launch_pq_unpack(const uint8_t* codes, int64_t n, const int64_t* list_off, const int64_t* list_goff,
                            int n_lists, int pq_dim, int pq_dim_pad, uint8_t* out, hipStream_t s);
hipError_t launch_pq_scan(const PqScanArgs& a, int kcap, hipStream_t s);
// K9s (split LUT, three workgroups per CU); hipErrorNotSupported when its shape limits are not met
size_t pq_split_lds_bytes(int rot_dim_pad, int pq_half, int kcap);
hipError_t launch_pq_scan_split(const PqScanArgs& a, int kcap, hipStream_t s);
size_t pq_tile_lds_bytes(int rot_dim_pad, int pq_len);
hipError_t launch_pq_scan_tiled(const PqTileArgs& a, int kcap, int grid, hipStream_t s);

hipError_t launch_gather_rows(const float* src, int d, const int64_t* rows, int64_t n, float* dst, hipStream_t s);
hipError_t launch_unpack_rows(const float* groups, int dp, int d, const int64_t* list_off, const int64_t* list_goff,
                              int n_lists, int64_t n_rows, float* out, hipStream_t s);
hipError_t launch_compact_ids(const int64_t* row_ids, const int64_t* list_off, const int64_t* list_goff,
                              int n_lists, int64_t n_rows, int64_t* out, hipStream_t s);
hipError_t launch_synth_mixture(float* out, int64_t row_begin, int64_t n, int d, uint64_t seed, int n_centers,
                                float sigma, int normalize, hipStream_t s);
hipError_t launch_group_list(const int64_t* list_goff, int n_lists, int64_t n_groups, int* group_list,
                             hipStream_t s);
hipError_t launch_labels_from_ids(const int64_t* ids, int64_t n, int64_t* labels, hipStream_t s);

}  // namespace mivs
