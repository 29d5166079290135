// mivs C-ABI (include/mivs.h): index objects and the build / search pipelines.
//
// Build  (replaces cuvs ivf_flat::build, index_building_coordinator.py:392-396):
//   trainset rows -> strided init -> n_iters x {pack centroids, K4 assign (scan
//   k=1), stable counting sort, K5 fp64 update} -> K4 assign of every row ->
//   stable counting sort -> K6 pack of the interleaved lists.
// Search (replaces cuvs ivf_flat::search, improved_multi_gpu_rag.py:225-227):
//   query norms -> coarse scan over the centroid list (k = n_probes) -> probe
//   map (list -> query buckets, work items, output slots) -> K3 fine scan ->
//   K7 merge of the per-(probe, chunk) partials.
// Everything is enqueued on the caller's stream; the only host syncs are in
// build (list sizes) and in stats collection when profiling is on.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <atomic>
#include <memory>
#include <cstring>
#include <mutex>
#include <numeric>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/mivs.h"
#include "capi_util.hpp"
#include "mivs_common.hpp"

using namespace mivs;
using namespace mivs_capi;

namespace mivs {
namespace {
std::atomic<int> g_engine_settings[kSetCount];
}  // namespace

int engine_setting(EngineSetting id, const char* name, int dflt) {
  constexpr int kUnset = INT32_MIN;
  static std::once_flag init;
  std::call_once(init, [] {
    for (auto& v : g_engine_settings) v.store(kUnset, std::memory_order_relaxed);
  });
  int v = g_engine_settings[id].load(std::memory_order_relaxed);
  if (v == kUnset) {
    v = env_int(name, dflt);
    g_engine_settings[id].store(v, std::memory_order_relaxed);
  }
  return v;
}

void engine_settings_reset() {
  for (auto& v : g_engine_settings) v.store(INT32_MIN, std::memory_order_relaxed);
}
}  // namespace mivs

namespace {

// hipEvent pairs around the build's hot kernels while profiling is on (the build's phase clock syncs the stream
// anyway): k_as_scan per k-means iteration and for the final assign (flops), K5's update, K6's pack and the fp16 / fp8
// copies (bytes). Set per build on the building thread (ParallelIndexBuilder builds one index per thread).
struct BuildProf {
  struct Rec {
    int kind;
    double work;
    hipEvent_t e0, e1;
  };
  std::vector<Rec> recs;
  int assign_kind = MIVS_BUILD_KMEANS_ASSIGN;  // the assign the build is in: k-means iterations, then the final
  ~BuildProf() {
    for (auto& r : recs) {
      (void)hipEventDestroy(r.e0);
      (void)hipEventDestroy(r.e1);
    }
  }
  size_t begin(int kind, double work, hipStream_t s) {
    Rec r{kind, work, nullptr, nullptr};
    HIPCHK(hipEventCreate(&r.e0));
    HIPCHK(hipEventCreate(&r.e1));
    HIPCHK(hipEventRecord(r.e0, s));
    recs.push_back(r);
    return recs.size() - 1;
  }
  void end(size_t i, hipStream_t s) { HIPCHK(hipEventRecord(recs[i].e1, s)); }
  // (the stream synchronized) -> per kind {calls, ms, work}
  void collect(mivs_build_kernel* out) {
    for (int k = 0; k < MIVS_BUILD_KERNEL_KINDS; ++k) out[k] = mivs_build_kernel{k, 0, 0.0, 0.0};
    for (auto& r : recs) {
      float ms = 0.0f;
      HIPCHK(hipEventElapsedTime(&ms, r.e0, r.e1));
      out[r.kind].calls += 1;
      out[r.kind].ms += ms;
      out[r.kind].work += r.work;
    }
  }
};
thread_local BuildProf* g_bprof = nullptr;

// one timed build kernel (no-op unless a profiled build is running on this thread)
struct BuildTimer {
  size_t i = 0;
  hipStream_t s;
  BuildTimer(int kind, double work, hipStream_t s_) : s(s_) {
    if (g_bprof) i = g_bprof->begin(kind, work, s);
  }
  ~BuildTimer() {
    if (g_bprof) g_bprof->end(i, s);
  }
};

// A set of inverted lists in the interleaved group layout.
struct ListSet {
  int n_lists = 0;
  int64_t n_rows = 0, n_groups = 0;
  Buf groups, norms, ids, off, goff;
  std::vector<int64_t> h_off, h_goff;
  std::vector<int64_t> top_chunks_prefix;  // prefix sums of chunk counts sorted descending

  int64_t chunks_of(int l, int G) const { return ceil_div(h_goff[l + 1] - h_goff[l], G); }
  void finalize_host(int G) {
    std::vector<int64_t> c(n_lists);
    for (int l = 0; l < n_lists; ++l) c[l] = chunks_of(l, G);
    std::sort(c.begin(), c.end(), std::greater<int64_t>());
    top_chunks_prefix.assign(n_lists + 1, 0);
    for (int l = 0; l < n_lists; ++l) top_chunks_prefix[l + 1] = top_chunks_prefix[l] + c[l];
  }
};

// Pack rows into `ls` given list row offsets (host) and an optional permutation.
void pack_lists(ListSet& ls, const float* src, int d, int dp, const int64_t* perm_d, const std::vector<int64_t>& h_off,
                int64_t id_offset, const int64_t* id_map, int G, hipStream_t s) {
  ls.n_lists = (int)h_off.size() - 1;
  ls.n_rows = h_off.back();
  ls.h_off = h_off;
  ls.h_goff.assign(ls.n_lists + 1, 0);
  for (int l = 0; l < ls.n_lists; ++l)
    ls.h_goff[l + 1] = ls.h_goff[l] + ceil_div(h_off[l + 1] - h_off[l], kGroupRows);
  ls.n_groups = ls.h_goff.back();
  require(ls.n_groups * (int64_t)kGroupRows < (int64_t)INT32_MAX, "index too large for 32-bit row positions",
          MIVS_ERR_UNSUPPORTED);
  const int64_t nslot = std::max<int64_t>(ls.n_groups, 1) * kGroupRows;
  ls.groups.reserve(sizeof(float) * (size_t)nslot * dp);
  ls.norms.reserve(sizeof(float) * (size_t)nslot);
  ls.ids.reserve(sizeof(int64_t) * (size_t)nslot);
  ls.off.reserve(sizeof(int64_t) * (ls.n_lists + 1));
  ls.goff.reserve(sizeof(int64_t) * (ls.n_lists + 1));
  HIPCHK(hipMemcpyAsync(ls.off.p, h_off.data(), sizeof(int64_t) * (ls.n_lists + 1), hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(ls.goff.p, ls.h_goff.data(), sizeof(int64_t) * (ls.n_lists + 1), hipMemcpyHostToDevice, s));
  Buf group_list;
  if (ls.n_lists > 1) {
    group_list.reserve(sizeof(int) * (size_t)std::max<int64_t>(ls.n_groups, 1));
    HIPCHK(launch_group_list(ls.goff.as<int64_t>(), ls.n_lists, ls.n_groups, group_list.as<int>(), s));
  }
  {
    // (each row read once, written once in its list's group layout, plus its norm and id)
    BuildTimer bt(MIVS_BUILD_PACK, (double)ls.n_rows * ((double)d * 4 + (double)dp * 4 + 12), s);
    HIPCHK(launch_pack_groups(src, 0, d, dp, perm_d, ls.off.as<int64_t>(), ls.goff.as<int64_t>(),
                              ls.n_lists > 1 ? group_list.as<int>() : nullptr, ls.n_groups, ls.groups.as<float>(),
                              ls.norms.as<float>(), ls.ids.as<int64_t>(), id_map, id_offset, s));
  }
  ls.finalize_host(G);
  HIPCHK(hipStreamSynchronize(s));  // host vectors above are referenced by the async copies
}

struct Workspace {
  Buf qn, bucket_q, bucket_slot, bucket_off, work_off, counter, part_d, part_i, slot_begin, probes_d, probes_i,
      counts, fill, qp_slots, scan_tmp, gmerge;
  // fp16 pre-filter path (K10 / K11) and its exact-scan fallback
  Buf qh, qscale, qres, qtheta, pf_key, pf_pos, pf_bound, pf_stats, ovf_q, ovf_rows, ovf_d, ovf_i;
  Buf q8, qscale8;  // K13's fp8 nomination: the queries' fp8 copy and scales
  // the batch whose qn / qh / qscale / qres (and, prep_f8, q8 / qscale8) launch_queries_prep wrote at the start of the
  // search (pf_scan_refine skips its own conversions for it)
  HostBuf h_stats;  // pinned: the refine's fallback count and window size
  const float* prep_q = nullptr;
  int64_t prep_nq = 0;
  bool prep_f8 = false;
  // K13 row-stationary scan: the full probe list, the pre-pass result, per-query headers and candidates
  Buf pre_probes, pre_kth, pre_goff, qhdr, rs_tq, cand_off, cand_key, cand_pos, rs_bucket_tmp, rs_tiles, rs_wave_buf,
      rs_wave_cnt, rs_bounds;
  // per-list query counts of the last search's own probe map (an exact fallback re-maps its queries)
  Buf rs_qcnt;  // K13's one-pass bucketing: candidates per query
  Buf stat_counts, rs_ovf_q, rs_ovf_rows, rs_ovf_d, rs_ovf_i, rs_items;
  // K16 large-k: T_q's sample probes and selection, the per-query windows and K16r's work items
  Buf lk_probes, lk_win_pos, lk_win_key, lk_win_n, lk_chunks, lk_chunk_off;
};

// hipEvent pairs recorded on the caller's stream around the pipeline stages of
// every search call while profiling is on; summed by mivs_index_profile_collect
// (no host sync inside the timed calls).
struct ProfRec {
  hipEvent_t e[4] = {};  // search begin, coarse end / fine-scan begin, fine-scan end, search end
};

struct Profiler {
  std::vector<ProfRec> pending, pool;
  ProfRec* begin(hipStream_t s) {
    ProfRec r;
    if (!pool.empty()) { r = pool.back(); pool.pop_back(); }
    else for (auto& x : r.e) HIPCHK(hipEventCreate(&x));
    pending.push_back(r);
    HIPCHK(hipEventRecord(pending.back().e[0], s));
    return &pending.back();
  }
  ~Profiler() {
    for (auto* v : {&pending, &pool})
      for (auto& r : *v)
        for (auto& x : r.e) (void)hipEventDestroy(x);
  }
};

}  // namespace

struct mivs_index_s {
  int kind = 0;  // 0 = ivf_flat, 1 = brute force, 2 = ivf_pq
  int device = 0, d = 0, dp = 0, metric = 0, G = kDefaultChunkGroups;
  int64_t id_offset = 0;
  ListSet lists;  // data
  ListSet cents;  // IVF: the centroid "list"
  Buf centroids_rm;
  // IVF-PQ: codes in the interleaved group layout + codebooks (lists.off/goff/ids/h_* describe the lists)
  int pq_dim = 0, pq_bits = 0, pq_len = 0, pq_dim_pad = 0, rot_dim_pad = 0;
  Buf pq_codes, pq_books;
  Buf pq_book_norms, pq_books_mfma;  // derived from pq_books at build (launch_pq_book_prep)
  // fp16 copy of the lists for the K10 pre-filter; empty = exact scan only
  Buf groups_h;
  Buf group_nmin;  // K13: the smallest row norm of every 32-row group (built with groups_h)
  Buf groups_f8;   // K13's pre-pass: the lists' fp8 copy at 2^hx8 (built with groups_h when the HBM budget allows)
  int hx8 = 0;
  int copies_skipped = 0;  // kCopySkippedF8: the fp8 copy was not built (HBM budget), K13's pre-pass uses fp16
  int hx_exp = 0;
  float x_norm_max = 0.0f, x_res_max = 0.0f;
  int pf_G = kPfChunkGroups;                  // groups per K10 work item
  std::vector<int64_t> pf_top_chunks_prefix;  // as ListSet::top_chunks_prefix, for pf_G
  std::mutex mu;
  Workspace ws;
  Profiler prof;
  // what the last search did (for algorithmic roofline counts)
  int64_t last_nq = 0;
  int last_np = 0, last_k = 0, last_qtile = kQTile;
  int last_pf = 0;
  int last_scan = 0;  // fine-scan kernel of the last search: 3 K3, 31 K3w, 10 K10, 12 K12, 13 K13
  int last_rs_waves = 0;  // K13: candidate streams of the last search (the lost flag follows their counts)
  int64_t last_rs_nq = 0; // K13: queries of the last search batch (its cand_off holds last_rs_nq + 1 offsets)
  bool last_rs_one_pass = false;  // K13: the last batch's candidates are in fixed-capacity runs (ws.rs_qcnt)
  int64_t last_ovf = 0, last_window = 0;
  // the last batch's fallback count and window size are still on the device (ws.pf_stats): the device-sized
  // fallback did not read them; last_search_stats does
  bool last_stats_dev = false;
  // host wall time of the build's phases (mivs_index_build_phases; recorded while profiling is on)
  std::vector<double> build_phase_s;
  // device time and algorithmic work of the build's hot kernels (mivs_index_build_kernels; profiling on)
  mivs_build_kernel build_kern[MIVS_BUILD_KERNEL_KINDS] = {};
  // an event per stream the index's calls were enqueued on, recorded at the end of each call: mivs_index_free waits
  // for these (not for the whole device) before its buffers go back to the driver or the block cache
  struct StreamDone {
    hipStream_t s;
    hipEvent_t ev;
  };
  std::vector<StreamDone> stream_done;
  ~mivs_index_s() {
    for (auto& e : stream_done) (void)hipEventDestroy(e.ev);
  }
};

namespace {

// record the index's done-event for stream s (the index's device is current)
void note_stream(mivs_index_s* idx, hipStream_t s) {
  for (auto& e : idx->stream_done)
    if (e.s == s) {
      (void)hipEventRecord(e.ev, s);
      return;
    }
  if (idx->stream_done.size() >= 8) {  // (a caller cycling through many streams: retire the oldest)
    (void)hipEventSynchronize(idx->stream_done.front().ev);
    (void)hipEventDestroy(idx->stream_done.front().ev);
    idx->stream_done.erase(idx->stream_done.begin());
  }
  hipEvent_t ev = nullptr;
  if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
    (void)hipGetLastError();
    return;
  }
  (void)hipEventRecord(ev, s);
  idx->stream_done.push_back({s, ev});
}

// wait for every call enqueued on the index so far (its done-events; the index's device is current)
void wait_index(mivs_index_s* idx) {
  for (auto& e : idx->stream_done) HIPCHK(hipEventSynchronize(e.ev));
}

// one C-ABI call on an index: its stream is the thread's release stream while it runs (Buf::release orders a cached
// block's reuse after it), and the index's done-event for that stream is recorded when it ends
struct IndexCall {
  mivs_index_s* idx;
  hipStream_t s;
  StreamScope ss;
  IndexCall(mivs_index_s* i, hipStream_t s_) : idx(i), s(s_), ss(s_) {}
  ~IndexCall() { note_stream(idx, s); }
};

// ---- one scan job: lists x buckets -> partial slots ----
struct ScanJob {
  const ListSet* ls;
  int G;
  const float* queries;
  const float* qnorms;
  int d, dp, k, metric;
  const int64_t* bucket_q;
  const int64_t* bucket_slot;
  const int* bucket_off;
  const int* work_off;
  float* out_d;
  int64_t* out_i;
  int qtile;  // 32: K3, 64: K3w (must match the work decomposition of the probe map / single job)
  bool dump = false;  // DUMP mode (raw keys per slot for K8) whatever k: set by every caller that runs K8
  bool counter_zeroed = false;  // ws.counter[0] was zeroed on the stream already (k_single_job)
  const int64_t* goff = nullptr;  // another split of ls's groups into lists (K16's sample), else ls->goff
  int n_lists = 0;
};

// Query tile of the fine scan for k: K3w (64 queries, slab-staged) where it applies, else K3.
// MIVS_SCAN_WIDE=0 forces K3 (A/B measurements).
int pick_qtile(int k, int d, int G) {
  const char* e = getenv("MIVS_SCAN_WIDE");
  if (e && e[0] == '0') return kQTile;
  const int kcap = scan_kcap(k);
  return kcap > 0 && scan_wide_supported(kcap, d, dim_pad(d), G) ? 64 : kQTile;
}

void run_scan(const ScanJob& j, int device, Workspace& ws, hipStream_t s) {
  // 0 = DUMP mode (k > kMaxK, or asked for): raw keys per slot + (first row, rows) slot info for K8
  const int kcap = j.dump ? 0 : scan_kcap(j.k);
  require(!(j.dump && j.qtile == 64 && !scan_wide_supported(0, j.d, j.dp, j.G)), "internal: DUMP on K3w not applicable",
          MIVS_ERR_UNSUPPORTED);
  require(j.k >= 1 && j.k <= kMaxSelectK, "k must be in [1, " + std::to_string(kMaxSelectK) + "]",
          MIVS_ERR_UNSUPPORTED);
  require(j.dp <= 1024, "dim > 1024 is not supported by this build", MIVS_ERR_UNSUPPORTED);
  ws.counter.reserve(16);
  if (!j.counter_zeroed) HIPCHK(hipMemsetAsync(ws.counter.p, 0, sizeof(int), s));
  ScanArgs a{};
  a.groups = j.ls->groups.as<float>();
  a.row_norms = j.ls->norms.as<float>();
  a.row_ids = j.ls->ids.as<int64_t>();
  a.list_goff = j.goff ? j.goff : j.ls->goff.as<int64_t>();
  a.n_lists = j.goff ? j.n_lists : j.ls->n_lists;
  a.chunk_groups = j.G;
  a.queries = j.queries;
  a.qnorms = j.qnorms;
  a.bucket_q = j.bucket_q;
  a.bucket_slot = j.bucket_slot;
  a.bucket_off = j.bucket_off;
  a.work_off = j.work_off;
  a.work_counter = ws.counter.as<int>();
  a.out_d = j.out_d;
  a.out_i = j.out_i;
  a.d = j.d;
  a.dp = j.dp;
  a.k = j.k;
  a.metric = j.metric;
  a.qtile = j.qtile;
  if (j.qtile == 64) {
    require(kcap >= 0 && scan_wide_supported(kcap, j.d, j.dp, j.G), "internal: wide scan not applicable");
    const size_t lds = scan_wide_lds_bytes(kcap, j.G);
    const int grid = cu_count(device) * std::min(2, scan_wide_occupancy(kcap, j.metric, lds));
    HIPCHK(launch_scan_wide(a, kcap, grid, lds, s));
    return;
  }
  const size_t lds = scan_lds_bytes(j.dp, kcap, j.G);
  const int grid = cu_count(device) * std::max(1, std::min(2, scan_occupancy(kcap, j.metric, lds)));
  float* gmerge = nullptr;
  if (!scan_merge_in_lds(j.dp, kcap, j.G)) {
    ws.gmerge.reserve(scan_gmerge_bytes(grid, kcap));
    gmerge = ws.gmerge.as<float>();
  }
  HIPCHK(launch_scan_ex(a, kcap, grid, lds, gmerge, s));
}

// Bytes of K8 dump workspace one search call may hold (MIVS_SELECT_WORKSPACE_MB, default 4 GiB):
// large-k searches run in query batches sized to it.
size_t select_workspace_bytes() {
  const char* e = getenv("MIVS_SELECT_WORKSPACE_MB");
  const long long mb = e ? atoll(e) : 4096;
  return (size_t)std::max<long long>(mb, 1) << 20;
}

// queries per batch when each query may need `per_query_bytes` of dump workspace
int64_t select_batch(int64_t nq, size_t per_query_bytes) {
  const int64_t b = (int64_t)(select_workspace_bytes() / std::max<size_t>(per_query_bytes, 1));
  return std::max<int64_t>(1, std::min<int64_t>(nq, b));
}

// single-list job (brute force, coarse probe selection, k-means assign):
// every query (or every row id of `rows`) against every row of `ls`.
// Writes [nq][k] results into (out_d, out_i) (merging chunk partials if needed).
void single_list_topk(const ListSet& ls, int G, const float* queries, const float* qnorms, const int64_t* rows,
                      int64_t nq, int d, int dp, int k, int metric, float* out_d, int64_t* out_i, int device,
                      Workspace& ws, hipStream_t s, bool dump = false) {
  const int64_t chunks = std::max<int64_t>(1, ceil_div(ls.n_groups, G));
  require(ceil_div(nq, kQTile) * chunks < (int64_t)INT32_MAX, "too many work items", MIVS_ERR_UNSUPPORTED);
  if (k > kMaxK || dump) {  // DUMP scan + K8 select, in query batches
    // K3w's 64-query tiles where they apply (two accumulator chains per wave; K3's 32 otherwise)
    const int dq = scan_wide_supported(0, d, dp, G) ? 64 : kQTile;
    const int64_t slot_rows = (int64_t)G * kGroupRows;
    const int64_t qb = select_batch(nq, (size_t)(chunks * (slot_rows * 4 + 16)));
    for (int64_t b0 = 0; b0 < nq; b0 += qb) {
      const int64_t nb = std::min<int64_t>(qb, nq - b0);
      ws.bucket_q.reserve(sizeof(int64_t) * nb);
      ws.bucket_slot.reserve(sizeof(int64_t) * nb);
      ws.bucket_off.reserve(sizeof(int) * 2);
      ws.work_off.reserve(sizeof(int) * 2);
      ws.part_d.reserve(sizeof(float) * (size_t)(nb * chunks * slot_rows));
      ws.part_i.reserve(sizeof(int64_t) * (size_t)(nb * chunks * 2));
      ws.counter.reserve(16);
      HIPCHK(launch_single_list_job(nb, chunks, dq, ws.bucket_q.as<int64_t>(), ws.bucket_slot.as<int64_t>(),
                                    ws.bucket_off.as<int>(), ws.work_off.as<int>(), nullptr, s, ws.counter.as<int>()));
      const float* qb_ptr = queries;
      const float* qn_ptr = qnorms;
      if (rows) HIPCHK(hipMemcpyAsync(ws.bucket_q.p, rows + b0, sizeof(int64_t) * nb, hipMemcpyDeviceToDevice, s));
      else { qb_ptr = queries + b0 * (int64_t)d; qn_ptr = qnorms + b0; }
      ScanJob j{&ls, G, qb_ptr, qn_ptr, d, dp, k, metric, ws.bucket_q.as<int64_t>(), ws.bucket_slot.as<int64_t>(),
                ws.bucket_off.as<int>(), ws.work_off.as<int>(), ws.part_d.as<float>(), ws.part_i.as<int64_t>(), dq};
      j.dump = true;
      j.counter_zeroed = true;
      run_scan(j, device, ws, s);
      SelectArgs sa{};
      sa.keys = ws.part_d.as<float>();
      sa.row_ids = ls.ids.as<int64_t>();
      sa.slot_info = ws.part_i.as<int64_t>();
      sa.slot_begin = nullptr;
      sa.slots_per_q = chunks;
      sa.slot_rows = (int)slot_rows;
      sa.nq = nb;
      sa.k = k;
      sa.metric = metric;
      sa.out_d = out_d + b0 * k;
      sa.out_i = out_i + b0 * k;
      HIPCHK(launch_select(sa, s));
    }
    return;
  }
  const int qtile = pick_qtile(k, d, G);
  ws.bucket_q.reserve(sizeof(int64_t) * nq);
  ws.bucket_slot.reserve(sizeof(int64_t) * nq);
  ws.bucket_off.reserve(sizeof(int) * 2);
  ws.work_off.reserve(sizeof(int) * 2);
  HIPCHK(launch_single_list_job(nq, chunks, qtile, ws.bucket_q.as<int64_t>(), ws.bucket_slot.as<int64_t>(),
                                ws.bucket_off.as<int>(), ws.work_off.as<int>(), nullptr, s));
  if (rows) HIPCHK(hipMemcpyAsync(ws.bucket_q.p, rows, sizeof(int64_t) * nq, hipMemcpyDeviceToDevice, s));
  float* pd = out_d;
  int64_t* pi = out_i;
  if (chunks > 1) {
    ws.part_d.reserve(sizeof(float) * (size_t)(nq * chunks * k));
    ws.part_i.reserve(sizeof(int64_t) * (size_t)(nq * chunks * k));
    pd = ws.part_d.as<float>();
    pi = ws.part_i.as<int64_t>();
  }
  ScanJob j{&ls, G, queries, qnorms, d, dp, k, metric, ws.bucket_q.as<int64_t>(), ws.bucket_slot.as<int64_t>(),
            ws.bucket_off.as<int>(), ws.work_off.as<int>(), pd, pi, qtile};
  run_scan(j, device, ws, s);
  if (chunks > 1) {
    MergeArgs m{};
    m.in_d = pd;
    m.in_i = pi;
    m.slot_begin = nullptr;
    m.slots_per_q = chunks;
    m.nq = nq;
    m.k_in = k;
    m.k = k;
    m.metric = metric;
    m.out_d = out_d;
    m.out_i = out_i;
    HIPCHK(launch_merge(m, s));
  }
}

void make_single_list(ListSet& ls, const float* src, int64_t n, int d, int dp, int64_t id_offset, int G,
                      hipStream_t s) {
  std::vector<int64_t> off = {0, n};
  pack_lists(ls, src, d, dp, nullptr, off, id_offset, nullptr, G, s);
}

// k-means' centroid list, refreshed every iteration: after the first pack only the groups and norms are
// rewritten (same shape: no allocation, no host copy, no stream sync -- the codebook training runs ~2,000 of
// these, and their hipMalloc / hipFree / syncs were most of its time)
void repack_single_list(ListSet& ls, const float* src, int64_t n, int d, int dp, int G, hipStream_t s) {
  if (ls.n_lists != 1 || ls.n_rows != n || ls.groups.p == nullptr) {
    make_single_list(ls, src, n, d, dp, 0, G, s);
    return;
  }
  HIPCHK(launch_pack_groups(src, 0, d, dp, nullptr, ls.off.as<int64_t>(), ls.goff.as<int64_t>(), nullptr, ls.n_groups,
                            ls.groups.as<float>(), ls.norms.as<float>(), ls.ids.as<int64_t>(), nullptr, 0, s));
}

// ---- fp16 pre-filter assign: k-means assign and list fill as a one-list K10 scan
// (queries = data rows, rows = centroids, k = 1) + the K11 exact refine; labels equal the fp32 K4's ----
struct PfAssign {
  Buf qh, qscale, qres;  // fp16 copy of every data row: 2^hx x a per-row power of two (k_queries_to_half)
  int hx = 0;
  int64_t n = 0;         // data rows
  bool ok = false;
};

// the most groups a K10 work item may span: its chunk's norms sit in LDS beside the query tile
int pf_max_chunk_groups(int dp) {
  if (pf_scan_lds_bytes(dp, 1) <= 160 * 1024) return kPfMaxPairGroups;
  int g = 1;
  while (pf_scan_lds_bytes(dp, g + 1) <= 160 * 1024) ++g;
  return g;
}

bool pf_assign_on() {
  const char* e = getenv("MIVS_PF_ASSIGN");
  return !(e && e[0] == '0');
}

// once per build: the data's fp16 copy, scaled by hx from the data's |x| max (every centroid is a mean of
// data rows, so the same hx keeps the centroids' fp16 copies in range; their own residuals enter delta)
void pf_assign_prepare(PfAssign& P, const float* data, int64_t n, int d, int dp, hipStream_t s) {
  P.ok = false;
  if (n <= 0 || dp % 64 != 0 || dp > 1024 || !pf_assign_on()) return;
  Buf st;
  st.reserve(16);
  HIPCHK(hipMemsetAsync(st.p, 0, 16, s));
  HIPCHK(launch_abs_max(data, n * d, st.as<unsigned>(), s));
  unsigned h = 0;
  HIPCHK(hipMemcpyAsync(&h, st.p, 4, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  float absmax;
  std::memcpy(&absmax, &h, 4);
  P.hx = pf_hx_exp(absmax);
  P.qh.reserve(sizeof(uint16_t) * (size_t)n * dp);
  P.qscale.reserve(sizeof(float) * n);
  P.qres.reserve(sizeof(float) * n);
  HIPCHK(launch_queries_to_half(data, n, d, dp, P.hx, P.qh.as<uint16_t>(), P.qscale.as<float>(),
                                P.qres.as<float>(), s));
  P.n = n;
  P.ok = true;
}

void pf_assign_k12(const PfAssign& P, const float* data, const float* data_norms, const int64_t* rows, int64_t nr,
                   int d, int dp, const ListSet& cents, int G, int64_t* labels, int device, Workspace& ws,
                   hipStream_t s);

bool as_assign_on() {
  const char* e = getenv("MIVS_PF_ASSIGN_RS");
  return !(e && e[0] == '0');
}

// K13a (assign.hip): the centroids' tile images, the row-stationary scan, then K12 + the window refine for the
// rows it could not prove (a wait that gave up: every row through the exact scan)
void as_assign_rows(const PfAssign& P, const float* data, const float* data_norms, const int64_t* rows, int64_t nr,
                    int d, int dp, const ListSet& cents, int G, int64_t* labels, int device, Workspace& ws,
                    hipStream_t s) {
  Buf ct, st, cnt, dist;
  ct.reserve(as_ctiles_bytes(cents.n_groups, dp));
  st.reserve(16);
  cnt.reserve(16);
  HIPCHK(hipMemsetAsync(st.p, 0, 16, s));
  HIPCHK(hipMemsetAsync(cnt.p, 0, 16, s));
  HIPCHK(launch_as_ctiles(cents.groups.as<float>(), cents.norms.as<float>(), cents.n_groups, dp, P.hx, ct.as<char>(),
                          st.as<unsigned>(), s));
  ws.ovf_q.reserve(sizeof(int64_t) * std::max<int64_t>(nr, 1));
  AsScanArgs a{};
  a.qh = P.qh.as<uint16_t>();
  a.qscale = P.qscale.as<float>();
  a.qnorms = data_norms;
  a.qres = P.qres.as<float>();
  a.rows = rows;
  a.nr = nr;
  a.ctiles = ct.as<char>();
  a.n_ctiles = (int)cents.n_groups;
  a.cstat = st.as<unsigned>();
  a.dp = dp;
  a.labels = labels;
  a.ovf_count = cnt.as<int>();
  a.ovf_rows = ws.ovf_q.as<int64_t>();
  a.queue = cnt.as<int>() + 2;
  a.flags = env_int("MIVS_AS_FLAGS", 0);
  {
    BuildTimer bt(g_bprof ? g_bprof->assign_kind : 0, 2.0 * (double)nr * (double)cents.n_rows * d, s);
    HIPCHK(launch_as_scan(a, cu_count(device), s));
  }
  int h[2] = {0, 0};
  HIPCHK(hipMemcpyAsync(h, cnt.p, 8, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  dist.reserve(sizeof(float) * std::max<int64_t>(nr, 1));  // (the fallback's distances, unused)
  if (h[1] != 0) {  // never expected: every row through the exact scan
    single_list_topk(cents, G, data, data_norms, rows, nr, d, dp, 1, kL2, dist.as<float>(), labels, device, ws, s);
    HIPCHK(hipStreamSynchronize(s));
    return;
  }
  if (h[0] == 0) return;
  // the near ties (a second centroid inside the refine window): K12 + the window refine on those rows alone,
  // scattered back (its own unprovable rows take the exact scan)
  const int64_t hn = h[0];
  Buf ovf, drow, lab;
  ovf.reserve(sizeof(int64_t) * hn);
  drow.reserve(sizeof(int64_t) * hn);
  lab.reserve(sizeof(int64_t) * hn);
  HIPCHK(hipMemcpyAsync(ovf.p, ws.ovf_q.p, sizeof(int64_t) * hn, hipMemcpyDeviceToDevice, s));
  if (rows) HIPCHK(launch_gather_ids(rows, ovf.as<int64_t>(), hn, drow.as<int64_t>(), s));
  else HIPCHK(hipMemcpyAsync(drow.p, ovf.p, sizeof(int64_t) * hn, hipMemcpyDeviceToDevice, s));
  pf_assign_k12(P, data, data_norms, drow.as<int64_t>(), hn, d, dp, cents, G, lab.as<int64_t>(), device, ws, s);
  HIPCHK(launch_scatter_results(dist.as<float>(), lab.as<int64_t>(), ovf.as<int64_t>(), hn, 1, dist.as<float>(),
                                labels, s));
  HIPCHK(hipStreamSynchronize(s));
}

void pf_assign_rows(const PfAssign& P, const float* data, const float* data_norms, const int64_t* rows, int64_t nr,
                    int d, int dp, const ListSet& cents, int G, int64_t* labels, int device, Workspace& ws,
                    hipStream_t s) {
  if (as_assign_on() && as_scan_supported(dp, cents.n_rows) && cents.n_lists == 1) {
    as_assign_rows(P, data, data_norms, rows, nr, d, dp, cents, G, labels, device, ws, s);
    return;
  }
  pf_assign_k12(P, data, data_norms, rows, nr, d, dp, cents, G, labels, device, ws, s);
}

// K12 (register-resident rows, the centroids streamed) + K11's one-lane refine of each row's window candidates;
// rows the refine cannot prove: the exact K4 scan. `rows` may be in any order (qtheta spans every data row).
void pf_assign_k12(const PfAssign& P, const float* data, const float* data_norms, const int64_t* rows, int64_t nr,
                   int d, int dp, const ListSet& cents, int G, int64_t* labels, int device, Workspace& ws,
                   hipStream_t s) {
  // the centroids' fp16 copy (scale 2^hx) and the maxima the refine window needs
  const int64_t nslot = cents.n_groups * (int64_t)kGroupRows;
  Buf ch, st;
  ch.reserve(sizeof(uint16_t) * (size_t)nslot * dp);
  st.reserve(16);
  HIPCHK(hipMemsetAsync(st.p, 0, 16, s));
  HIPCHK(launch_norm_max(cents.norms.as<float>(), nslot, st.as<unsigned>(), s));
  HIPCHK(launch_groups_to_half(cents.groups.as<float>(), cents.n_groups, dp, P.hx, ch.as<uint16_t>(),
                               st.as<unsigned>() + 1, s));
  unsigned h[2] = {0, 0};
  HIPCHK(hipMemcpyAsync(h, st.p, 8, hipMemcpyDeviceToHost, s));
  // probe map: one list (the centroids), every query in its bucket. K12 (128 register-resident queries per
  // CU, the centroids streamed from L2) where dp is within its instantiations, else K10
  const bool use_r = pr_scan_supported(dp);
  const int cg = use_r ? std::max<int>(1, (int)std::min<int64_t>(cents.n_groups, 1 << 20))
                       : std::max(1, std::min<int>(std::min(kPfChunkGroups, pf_max_chunk_groups(dp)),
                                                   (int)cents.n_groups));
  const int64_t chunks = std::max<int64_t>(1, ceil_div(cents.n_groups, cg));
  const int64_t nslots = nr * chunks;
  ws.bucket_q.reserve(sizeof(int64_t) * nr);
  ws.bucket_slot.reserve(sizeof(int64_t) * nr);
  ws.bucket_off.reserve(sizeof(int) * 2);
  ws.work_off.reserve(sizeof(int) * 2);
  ws.slot_begin.reserve(sizeof(int64_t) * (nr + 1));
  HIPCHK(launch_single_list_job(nr, chunks, use_r ? kPrQTile : kPfQTile, ws.bucket_q.as<int64_t>(),
                                ws.bucket_slot.as<int64_t>(), ws.bucket_off.as<int>(), ws.work_off.as<int>(),
                                ws.slot_begin.as<int64_t>(), s));
  if (rows) HIPCHK(hipMemcpyAsync(ws.bucket_q.p, rows, sizeof(int64_t) * nr, hipMemcpyDeviceToDevice, s));
  const int slot_k = use_r ? kPrSlotK : 16;
  ws.pf_key.reserve(sizeof(float) * (size_t)nslots * slot_k);
  ws.pf_pos.reserve(sizeof(int) * (size_t)nslots * slot_k);
  ws.pf_bound.reserve(sizeof(float) * (size_t)nslots);
  ws.counter.reserve(8 * 16 * sizeof(int));
  HIPCHK(hipMemsetAsync(ws.counter.p, 0, 8 * 16 * sizeof(int), s));
  const int64_t n_ids = rows ? P.n : nr;  // qtheta is indexed by data row
  ws.qtheta.reserve(sizeof(unsigned) * n_ids);
  HIPCHK(launch_fill_i32(ws.qtheta.as<int>(), n_ids, (int)kPfOrdInf, s));
  HIPCHK(hipStreamSynchronize(s));
  float normmax, resmax;
  std::memcpy(&normmax, &h[0], 4);
  std::memcpy(&resmax, &h[1], 4);
  PfScanArgs a{};
  a.groups_h = ch.as<uint16_t>();
  a.row_norms = cents.norms.as<float>();
  a.list_goff = cents.goff.as<int64_t>();
  a.n_lists = 1;
  a.chunk_groups = cg;
  a.qh = P.qh.as<uint16_t>();
  a.qscale = P.qscale.as<float>();
  a.qnorms = data_norms;
  a.bucket_q = ws.bucket_q.as<int64_t>();
  a.bucket_slot = ws.bucket_slot.as<int64_t>();
  a.bucket_off = ws.bucket_off.as<int>();
  a.work_off = ws.work_off.as<int>();
  a.work_counter = ws.counter.as<int>();
  a.slot_key = ws.pf_key.as<float>();
  a.slot_pos = ws.pf_pos.as<int>();
  a.slot_bound = ws.pf_bound.as<float>();
  a.slot_k = slot_k;
  a.dp = dp;
  a.metric = kL2;
  a.qres = P.qres.as<float>();
  a.x_norm_max = sqrtf(normmax) * (1.0f + 0x1p-12f);
  a.x_res_max = resmax;
  a.qtheta = ws.qtheta.as<unsigned>();
  a.k = 1;
  a.no_theta = chunks == 1 ? 1 : 0;  // every row's one work item: no bound to share
  const int grid = std::max(8, cu_count(device) / 8 * 8);
  Buf pbuf;
  const bool pprof = (env_int("MIVS_PF_FLAGS", 0) & 32) && use_r;
  if (pprof) {  // diagnostic: K12 phase clocks of the assign to stderr
    pbuf.reserve(16 * sizeof(unsigned long long));
    HIPCHK(hipMemsetAsync(pbuf.p, 0, 16 * sizeof(unsigned long long), s));
    a.prof = pbuf.as<unsigned long long>();
  }
  if (use_r) HIPCHK(launch_pr_scan(a, grid, s));
  else HIPCHK(launch_pf_scan(a, grid, pf_scan_lds_bytes(dp, cg), s));
  if (pprof) {
    unsigned long long hp[16];
    HIPCHK(hipMemcpyAsync(hp, pbuf.p, sizeof(hp), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    const double w = (double)hp[7];
    fprintf(stderr, "[k12 assign phases] nr %lld clock %.3f GHz | fetch %.3f setup %.3f loop %.3f tail %.3f | "
            "cycles/group %.0f slow %.4f\n", (long long)nr, hp[8] ? (double)hp[7] / hp[8] * 0.1 : 0.0, hp[0] / w,
            hp[1] / w, hp[2] / w, hp[3] / w, hp[5] ? (double)hp[2] / hp[5] : 0.0,
            hp[5] ? (double)hp[6] / hp[5] : 0.0);
  }
  Buf tmp_d, stats;
  tmp_d.reserve(sizeof(float) * (size_t)std::max<int64_t>(nr, 1));
  stats.reserve(32);
  HIPCHK(hipMemsetAsync(stats.p, 0, 32, s));
  ws.ovf_q.reserve(sizeof(int64_t) * nr);
  PfRefineArgs r{};
  r.slot_key = ws.pf_key.as<float>();
  r.slot_pos = ws.pf_pos.as<int>();
  r.slot_bound = ws.pf_bound.as<float>();
  r.slot_begin = ws.slot_begin.as<int64_t>();
  r.slot_k = slot_k;
  r.nq = nr;
  r.k = 1;
  r.d = d;
  r.dp = dp;
  r.metric = kL2;
  r.groups = cents.groups.as<float>();
  r.row_norms = cents.norms.as<float>();
  r.row_ids = cents.ids.as<int64_t>();
  r.queries = data;
  r.qnorms = data_norms;
  r.qres = P.qres.as<float>();
  r.qrows = rows;
  r.labels_only = 1;
  r.x_norm_max = a.x_norm_max;
  r.x_res_max = a.x_res_max;
  r.out_d = tmp_d.as<float>();
  r.out_i = labels;
  r.ovf_count = stats.as<int>();
  r.ovf_q = ws.ovf_q.as<int64_t>();
  HIPCHK(launch_pf_refine(r, s));
  int hn = 0;
  HIPCHK(hipMemcpyAsync(&hn, stats.p, 4, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  if (hn > 0) {  // rows the refine could not prove: the exact K4 scan, scattered back
    const int64_t no = hn;
    Buf orow, od, oi;
    orow.reserve(sizeof(int64_t) * no);
    od.reserve(sizeof(float) * no);
    oi.reserve(sizeof(int64_t) * no);
    if (rows) HIPCHK(launch_gather_ids(rows, ws.ovf_q.as<int64_t>(), no, orow.as<int64_t>(), s));
    else HIPCHK(hipMemcpyAsync(orow.p, ws.ovf_q.p, sizeof(int64_t) * no, hipMemcpyDeviceToDevice, s));
    single_list_topk(cents, G, data, data_norms, orow.as<int64_t>(), no, d, dp, 1, kL2, od.as<float>(),
                     oi.as<int64_t>(), device, ws, s);
    HIPCHK(launch_scatter_results(od.as<float>(), oi.as<int64_t>(), ws.ovf_q.as<int64_t>(), no, 1,
                                  tmp_d.as<float>(), labels, s));
    HIPCHK(hipStreamSynchronize(s));
  }
}

// K4 assign of rows (rows == nullptr: all n rows) to centroids -> labels; through the fp16 pre-filter
// when `pfa` holds the data's fp16 copy (L2 only)
void assign_rows(const float* data, const float* data_norms, const int64_t* rows, int64_t nr, int d, int dp,
                 const ListSet& cents, int G, int metric, int64_t* labels, int device, Workspace& ws,
                 hipStream_t s, const PfAssign* pfa = nullptr, Buf* dist_buf = nullptr) {
  if (pfa && pfa->ok && metric == kL2 && nr > 0) {
    pf_assign_rows(*pfa, data, data_norms, rows, nr, d, dp, cents, G, labels, device, ws, s);
    return;
  }
  Buf local;
  Buf& dist = dist_buf ? *dist_buf : local;  // (a caller's buffer outlives the launch: no sync)
  dist.reserve(sizeof(float) * (size_t)std::max<int64_t>(nr, 1));
  single_list_topk(cents, G, data, data_norms, rows, nr, d, dp, 1, metric, dist.as<float>(), labels, device, ws, s);
  if (!dist_buf) HIPCHK(hipStreamSynchronize(s));  // `dist` is freed on return
}

// n_iters Lloyd iterations on trainset rows; centroids_rm in/out [nc][d]
// iterations it_begin .. it_begin + iters - 1 of a Lloyd run of it_total iterations (-1: iters); the balancing
// step runs on all but the run's last kBalanceKeepLast. labels_out: the last iteration's assignment.
void kmeans_fit_impl(const float* data, const float* data_norms, const int64_t* rows, int64_t n_train, int d, int dp,
                     int nc, int iters, float* centroids_rm, int G, int device, Workspace& ws, hipStream_t s,
                     bool balance = false, const PfAssign* pfa = nullptr, int it_begin = 0, int it_total = -1,
                     int64_t* labels_out = nullptr) {
  if (iters <= 0) return;
  if (it_total < 0) it_total = it_begin + iters;
  Buf labels, perm, off, partial, chunk_off, tmp, ctmp, dist;
  ListSet cents;  // (one allocation for every iteration)
  labels.reserve(sizeof(int64_t) * n_train);
  perm.reserve(sizeof(int64_t) * n_train);
  off.reserve(sizeof(int64_t) * (nc + 1));
  partial.reserve(sizeof(double) * km_partial_rows(n_train, nc) * d);
  chunk_off.reserve(sizeof(int64_t) * (nc + 1));
  tmp.reserve(sizeof(int64_t) * (nc + 1) + scan_tmp_bytes(nc + 1));
  const size_t cb = csort_tmp_bytes(n_train, nc);
  ctmp.reserve(cb);
  for (int it = it_begin; it < it_begin + iters; ++it) {
    repack_single_list(cents, centroids_rm, nc, d, dp, G, s);
    assign_rows(data, data_norms, rows, n_train, d, dp, cents, G, kL2, labels.as<int64_t>(), device, ws, s, pfa,
                &dist);
    if (labels_out && it == it_begin + iters - 1)
      HIPCHK(hipMemcpyAsync(labels_out, labels.p, sizeof(int64_t) * n_train, hipMemcpyDeviceToDevice, s));
    HIPCHK(launch_counting_sort(labels.as<int64_t>(), n_train, nc, perm.as<int64_t>(), off.as<int64_t>(), ctmp.p,
                                cb, s));
    {
      BuildTimer bt(MIVS_BUILD_KMEANS_UPDATE, (double)n_train * d * 4.0, s);  // (each member row read once)
      HIPCHK(launch_km_update(data, d, rows, perm.as<int64_t>(), off.as<int64_t>(), nc, n_train,
                              partial.as<double>(), chunk_off.as<int64_t>(), tmp.p, centroids_rm, s));
    }
    if (balance && it < it_total - kBalanceKeepLast)
      HIPCHK(launch_km_rebalance(data, d, rows, labels.as<int64_t>(), off.as<int64_t>(), nc, n_train, it,
                                 centroids_rm, s));
  }
  HIPCHK(hipStreamSynchronize(s));
}

// lists of `idx` from final centroids: assign every row, stable sort, pack
void build_lists(mivs_index_s* idx, const float* data, const float* data_norms, int64_t n, hipStream_t s,
                 const PfAssign* pfa = nullptr) {
  const int nl = idx->cents.n_lists == 1 ? (int)idx->cents.n_rows : idx->cents.n_lists;
  Buf labels, perm, off, ctmp;
  labels.reserve(sizeof(int64_t) * std::max<int64_t>(n, 1));
  perm.reserve(sizeof(int64_t) * std::max<int64_t>(n, 1));
  off.reserve(sizeof(int64_t) * (nl + 1));
  if (n > 0)
    assign_rows(data, data_norms, nullptr, n, idx->d, idx->dp, idx->cents, idx->G, idx->metric,
                labels.as<int64_t>(), idx->device, idx->ws, s, pfa);
  const size_t cb = csort_tmp_bytes(n, nl);
  ctmp.reserve(cb);
  HIPCHK(launch_counting_sort(labels.as<int64_t>(), n, nl, perm.as<int64_t>(), off.as<int64_t>(), ctmp.p, cb, s));
  std::vector<int64_t> h_off(nl + 1);
  HIPCHK(hipMemcpyAsync(h_off.data(), off.p, sizeof(int64_t) * (nl + 1), hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  pack_lists(idx->lists, data, idx->d, idx->dp, perm.as<int64_t>(), h_off, idx->id_offset, nullptr, idx->G, s);
}

int chunk_groups_from_rows(int32_t chunk_rows) {
  if (chunk_rows <= 0) return kDefaultChunkGroups;
  return (int)std::max<int64_t>(1, ceil_div(chunk_rows, kGroupRows));
}

void check_common(int device, const void* data, int64_t n, int32_t dim) {
  int ndev = 0;
  HIPCHK(hipGetDeviceCount(&ndev));
  require(device >= 0 && device < ndev, "invalid device " + std::to_string(device));
  require(dim >= 1, "dim must be >= 1");
  require(dim_pad(dim) <= 1024, "dim > 1024 is not supported by this build", MIVS_ERR_UNSUPPORTED);
  require(n >= 0, "n must be >= 0");
  require(n == 0 || data != nullptr, "data is NULL");
}


// ---- fp16 pre-filter (K10 / K11) ----
// The optional copies an index may build beside its fp32 rows must leave this much of the device's HBM to the
// rest of the process (an LLM or tensors sharing the GPU in a RAG pipeline): MIVS_INDEX_HBM_FRAC (default 0.6) is
// the largest fraction of the device's HBM the index may hold with the copy, and 4 GiB must stay free beside it.
bool copy_fits(const mivs_index_s* idx, size_t bytes);
bool pf_default_on() {
  const char* e = getenv("MIVS_PREFILTER");
  return !(e && e[0] == '0');
}

// K13's pre-pass operand: the lists' fp8 copy at 2^(hx - 7), built with the fp16 copy (in the
// build, counted in its time) for IVF indexes K13 serves, when the HBM budget allows; otherwise the pre-pass scans
// the fp16 sample and last_search_stats / mivs_index_memory report the skipped copy
void pf_build_f8(mivs_index_s* idx, hipStream_t s) {
  const int nsb = idx->dp / 32;
  if (idx->kind != 0 || idx->dp % 32 != 0 || (nsb % 6 != 0 && nsb % 4 != 0) || !pf_pair_mode() ||
      !rs_scan_supported(idx->dp))
    return;
  const ListSet& L = idx->lists;
  const size_t bytes = (size_t)L.n_groups * kGroupRows * idx->dp;
  if (bytes == 0) return;
  if (!copy_fits(idx, bytes)) {
    idx->copies_skipped |= kCopySkippedF8;
    return;
  }
  idx->hx8 = idx->hx_exp - 7;  // |x| max 2^hx_exp in [2^14, 2^15) -> [128, 256) under e4m3's 448
  idx->groups_f8.reserve(bytes);
  BuildTimer bt(MIVS_BUILD_FP8_COPY, (double)bytes * 5.0, s);  // (fp32 read, fp8 written)
  HIPCHK(launch_groups_to_f8(L.groups.as<float>(), L.n_groups, idx->dp, idx->hx8, idx->groups_f8.as<uint8_t>(), s));
}

size_t listset_bytes(const ListSet& L) { return L.groups.n + L.norms.n + L.ids.n + L.off.n + L.goff.n; }

mivs_index_memory index_memory(const mivs_index_s* idx) {
  mivs_index_memory m{};
  const ListSet& L = idx->lists;
  m.n_rows = L.n_rows;
  m.rows_bytes = (int64_t)L.groups.n;
  m.side_bytes = (int64_t)(L.norms.n + L.ids.n + L.off.n + L.goff.n);
  m.centroid_bytes = (int64_t)(listset_bytes(idx->cents) + idx->centroids_rm.n);
  m.fp16_bytes = (int64_t)(idx->groups_h.n + idx->group_nmin.n);
  m.fp8_bytes = (int64_t)idx->groups_f8.n;
  m.pq_bytes = (int64_t)(idx->pq_codes.n + idx->pq_books.n + idx->pq_book_norms.n + idx->pq_books_mfma.n);
  m.total_bytes = m.rows_bytes + m.side_bytes + m.centroid_bytes + m.fp16_bytes + m.fp8_bytes + m.pq_bytes;
  m.copies_skipped = idx->copies_skipped;
  return m;
}

bool copy_fits(const mivs_index_s* idx, size_t bytes) {
  size_t fr = 0, tot = 0;
  if (hipMemGetInfo(&fr, &tot) != hipSuccess) return false;
  int dev = 0;
  if (hipGetDevice(&dev) == hipSuccess) fr += BlockCache::get().cached(dev);  // (blocks this process holds for reuse)
  const char* e = getenv("MIVS_INDEX_HBM_FRAC");
  const double frac = e ? atof(e) : 0.6;
  return fr >= bytes + ((size_t)4 << 30) && (double)index_memory(idx).total_bytes + (double)bytes <= frac * (double)tot;
}

// build the fp16 copy of idx->lists (+ the per-index maxima the refine window needs)
void pf_enable(mivs_index_s* idx, hipStream_t s) {
  const ListSet& L = idx->lists;
  idx->groups_h.release();
  idx->groups_f8.release();
  idx->copies_skipped = 0;
  if (L.n_groups == 0 || idx->dp % 64 != 0) return;
  const int64_t nslot = L.n_groups * (int64_t)kGroupRows;
  Buf st;
  st.reserve(4 * sizeof(unsigned));
  HIPCHK(hipMemsetAsync(st.p, 0, 4 * sizeof(unsigned), s));
  HIPCHK(launch_abs_max(L.groups.as<float>(), nslot * idx->dp, st.as<unsigned>(), s));
  HIPCHK(launch_norm_max(L.norms.as<float>(), nslot, st.as<unsigned>() + 1, s));
  unsigned h[4] = {0, 0, 0, 0};
  HIPCHK(hipMemcpyAsync(h, st.p, 2 * sizeof(unsigned), hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  float absmax, normmax;
  std::memcpy(&absmax, &h[0], 4);
  std::memcpy(&normmax, &h[1], 4);
  idx->hx_exp = pf_hx_exp(absmax);
  idx->groups_h.reserve(sizeof(uint16_t) * (size_t)nslot * idx->dp);
  idx->group_nmin.reserve(sizeof(float) * (size_t)L.n_groups);
  HIPCHK(launch_group_nmin(L.norms.as<float>(), L.n_groups, idx->group_nmin.as<float>(), s));
  {
    BuildTimer bt(MIVS_BUILD_FP16_COPY, (double)nslot * idx->dp * 6.0, s);  // (fp32 read, fp16 written)
    HIPCHK(launch_groups_to_half(L.groups.as<float>(), L.n_groups, idx->dp, idx->hx_exp,
                                 idx->groups_h.as<uint16_t>(), st.as<unsigned>() + 2, s));
  }
  HIPCHK(hipMemcpyAsync(&h[2], st.as<unsigned>() + 2, sizeof(unsigned), hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  float resmax;
  std::memcpy(&resmax, &h[2], 4);
  idx->x_norm_max = sqrtf(normmax) * (1.0f + 0x1p-12f);
  idx->x_res_max = resmax;
  pf_build_f8(idx, s);
  std::vector<int64_t> c(L.n_lists);
  // rows per work item: kPfChunkGroups groups, or as many as the LDS holds the norms of beside the query tile (the
  // tile's staging is paid once per item)
  const int gmax = pf_max_chunk_groups(idx->dp);
  idx->pf_G = std::max(1, std::min(gmax, kPfChunkGroups));
  auto top_prefix = [&](int G, std::vector<int64_t>& out) {
    for (int l = 0; l < L.n_lists; ++l) c[l] = L.chunks_of(l, G);
    std::sort(c.begin(), c.end(), std::greater<int64_t>());
    out.assign(L.n_lists + 1, 0);
    for (int l = 0; l < L.n_lists; ++l) out[l + 1] = out[l] + c[l];
  };
  top_prefix(idx->pf_G, idx->pf_top_chunks_prefix);
}

void ivf_search_batch(mivs_index_s* idx, hipStream_t s, const float* q, int64_t nq, int k, int np, float* out_d,
                      int64_t* out_i, int32_t* out_probes, bool allow_pf = true, bool prof = true,
                      bool allow_rs = true);
bool lk_use(const mivs_index_s* idx, int k, int np);
bool rs_use(const mivs_index_s* idx, int np);
bool rs_pre_f8(mivs_index_s* idx, hipStream_t);
int64_t lk_batch(const mivs_index_s* idx, int64_t nq, int k, int np);
void ivf_search_probed(mivs_index_s* idx, hipStream_t s, const float* q, int64_t nq, int k, int np, float* out_d,
                       int64_t* out_i, bool pf, ProfRec* pr, bool prof, const int64_t* probes = nullptr,
                       bool allow_rs = true);

void pf_refine_fallback(mivs_index_s* idx, hipStream_t s, const float* q, int64_t nq, int k, int np, float* out_d,
                        int64_t* out_i, const float* slot_key, const int* slot_pos, const float* slot_bound,
                        const int* force_ovf, const int64_t* slot_begin, int slot_k, bool fallback_pf = false,
                        float* kth_out = nullptr, const float* window_cap = nullptr, int verify_sel = 0,
                        bool stats_zeroed = false, const int* slot_cnt = nullptr, int slot_cap = 0);

// K10 scan + K11 refine for a probe map built with (kPfChunkGroups, kPfQTile); queries the refine
// could not prove are re-run through the exact scan and scattered back.
// (goff / n_lists: another split of the same groups into lists -- K13's pre-pass samples)
// kth_out: K13's pre-pass -- only the k-th smallest approximate key per query (no refine, no fallback);
// verify_sel > 0 (with the fp8 scan, f8) makes kth_out the k-th smallest fp32 key of each query's verify_sel
// best-scored rows
// raw: K10 leaves each slot as its 16 lane lists (no per-slot merge; K11 / K11v rank every entry)
void pf_scan_refine(mivs_index_s* idx, hipStream_t s, const float* q, int64_t nq, int k, int np, float* out_d,
                    int64_t* out_i, ProfRec* pr, const int64_t* goff, int n_lists, float* kth_out = nullptr,
                    int verify_sel = 0, bool f8 = false, bool raw = false) {
  Workspace& ws = idx->ws;
  const ListSet& L = idx->lists;
  const int dp = idx->dp;
  const bool prepped = ws.prep_q == q && ws.prep_nq == nq;  // (launch_queries_prep wrote them for this batch)
  ws.qh.reserve(sizeof(uint16_t) * (size_t)nq * dp);
  ws.qscale.reserve(sizeof(float) * nq);
  ws.qres.reserve(sizeof(float) * nq);
  if (!prepped)
    HIPCHK(launch_queries_to_half(q, nq, idx->d, dp, idx->hx_exp, ws.qh.as<uint16_t>(), ws.qscale.as<float>(),
                                  ws.qres.as<float>(), s));
  const std::vector<int64_t>& tcp = idx->pf_top_chunks_prefix;
  const int64_t max_slots = std::max<int64_t>(1, nq * tcp[std::min<int64_t>(np, L.n_lists)]);
  // per-slot candidates: room above k so that a neighbourhood packed into one chunk does not overflow
  const int slot_k = raw ? 16 * kPfLaneK : kPfSlotKMax;
  ws.pf_key.reserve(sizeof(float) * (size_t)max_slots * slot_k);
  ws.pf_pos.reserve(sizeof(int) * (size_t)max_slots * slot_k);
  ws.pf_bound.reserve(sizeof(float) * (size_t)max_slots);
  // the 8 queue counters, then (K10) one convoy position per (list, chunk)
  const int64_t n_cpos = (int64_t)n_lists * tcp[1];
  ws.counter.reserve(sizeof(int) * (8 * 16 + n_cpos));  // (zeroed below, in the qtheta fill's launch)
  PfScanArgs a{};
  a.chunk_pos = ws.counter.as<int>() + 8 * 16;
  a.chunk_stride = (int)tcp[1];
  a.groups_h = idx->groups_h.as<uint16_t>();
  a.row_norms = L.norms.as<float>();
  if (f8) {  // K13's fp8 nomination: the fp8 queries beside the fp16 ones (the headers and tiles use those)
    ws.q8.reserve((size_t)nq * dp);
    ws.qscale8.reserve(sizeof(float) * nq);
    if (!(prepped && ws.prep_f8))
      HIPCHK(launch_queries_to_f8(q, nq, idx->d, dp, idx->hx8, ws.q8.as<uint8_t>(), ws.qscale8.as<float>(), s));
    a.groups_f8 = idx->groups_f8.as<uint8_t>();
    a.q8 = ws.q8.as<uint8_t>();
    a.qscale8 = ws.qscale8.as<float>();
  }
  a.list_goff = goff;
  a.n_lists = n_lists;
  a.chunk_groups = idx->pf_G;
  a.qh = ws.qh.as<uint16_t>();
  a.qscale = ws.qscale.as<float>();
  a.qnorms = ws.qn.as<float>();
  a.bucket_q = ws.bucket_q.as<int64_t>();
  a.bucket_slot = ws.bucket_slot.as<int64_t>();
  a.bucket_off = ws.bucket_off.as<int>();
  a.work_off = ws.work_off.as<int>();
  a.work_counter = ws.counter.as<int>();
  a.slot_key = ws.pf_key.as<float>();
  a.slot_pos = ws.pf_pos.as<int>();
  a.slot_bound = ws.pf_bound.as<float>();
  a.slot_k = slot_k;
  a.dp = dp;
  a.metric = idx->metric;
  a.qres = ws.qres.as<float>();
  a.x_norm_max = idx->x_norm_max;
  a.x_res_max = idx->x_res_max;
  ws.qtheta.reserve(sizeof(unsigned) * nq);
  HIPCHK(launch_fill2_i32(ws.qtheta.as<int>(), nq, (int)kPfOrdInf, ws.counter.as<int>(), 8 * 16 + n_cpos, 0, s));
  a.qtheta = ws.qtheta.as<unsigned>();
  a.k = verify_sel > 0 ? std::min(verify_sel, kPfMaxK) : k;  // (nomination: the slots keep the verify_sel best)
  // (nomination: K11v reads only each slot's verify_sel best keys and their ties, so the slot merge stops there)
  a.slot_out = verify_sel > 0 && !raw ? a.k : 0;
  a.raw_lists = raw ? 1 : 0;
  // K13's pre-pass (kth_out): each list sample is scanned by one tile -- its rows are read once (non-temporal)
  a.rows_nt = kth_out != nullptr;
  a.flags = env_int("MIVS_PF_FLAGS", 0);
  Buf pbuf;
  if (a.flags & 32) {  // diagnostic: K10 phase clocks to stderr
    pbuf.reserve(16 * sizeof(unsigned long long));
    HIPCHK(hipMemsetAsync(pbuf.p, 0, 16 * sizeof(unsigned long long), s));
    a.prof = pbuf.as<unsigned long long>();
  }
  if (pr) HIPCHK(hipEventRecord(pr->e[1], s));
  const int grid = std::max(8, cu_count(idx->device) / 8 * 8);
  HIPCHK(launch_pf_scan(a, grid, pf_scan_lds_bytes(dp, idx->pf_G), s));
  if (pr) HIPCHK(hipEventRecord(pr->e[2], s));
  if (a.flags & 32) {
    unsigned long long hp[16];
    HIPCHK(hipMemcpyAsync(hp, pbuf.p, sizeof(hp), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    const double w = (double)hp[7];
    fprintf(stderr, "[k10 phases] waves-cycles %.4g clock %.3f GHz | fetch %.3f staging %.3f loop %.3f "
              "barrier %.3f merge %.3f | epilogues %llu slow %.4f\n", w, hp[8] ? (double)hp[7] / hp[8] * 0.1 : 0.0,
              hp[0] / w, hp[1] / w, hp[2] / w, hp[3] / w, hp[4] / w, hp[5], hp[5] ? (double)hp[6] / hp[5] : 0.0);
  }
  pf_refine_fallback(idx, s, q, nq, k, np, out_d, out_i, ws.pf_key.as<float>(), ws.pf_pos.as<int>(),
                     ws.pf_bound.as<float>(), nullptr, ws.slot_begin.as<int64_t>(), slot_k, false, kth_out, nullptr,
                     verify_sel);
}

// The exact fallback of K13's unproven queries sized on the device: K11 leaves their count in
// ws.pf_stats[0] and their rows in ws.ovf_q; the probe map over their probes (ws.probes_i, from the search's coarse
// probe), K3 over those (query, list) pairs, and K7 writing each query's top-k straight into its row of out_d / out_i
// all take their size from that count on the device, so the search enqueues and returns without a host round trip.
// An empty fallback is three launches that leave at once (~10 us of GPU time, against the ~55-90 us turnaround of
// reading the count on the host). MIVS_FALLBACK_SYNC=1 keeps the host-sized path (A/B runs).
// (the device-sized probe map is one workgroup: up to 2M (query, probe) entries, ~1 ms when every query of such a batch
// falls back; beyond that the host-sized path keeps the multi-workgroup map)
// (MIVS_FALLBACK_SYNC is read once, at the first search after load or mivs_reload_settings)
std::atomic<int> g_fallback_sync{-1};

bool device_fallback_ok(const mivs_index_s* idx, int k, int64_t nq, int np) {
  int fs = g_fallback_sync.load(std::memory_order_relaxed);
  if (fs < 0) {
    fs = env_int("MIVS_FALLBACK_SYNC", 0) != 0 ? 1 : 0;
    g_fallback_sync.store(fs, std::memory_order_relaxed);
  }
  return fs == 0 && nq * (int64_t)np <= ((int64_t)1 << 21) && idx->kind == 0 && k <= kMaxK &&
         idx->lists.n_lists <= probe_map_dev_max_lists();
}

// K9r's candidate-superset slots for 64 < k <= kRtCandMax (MIVS_PQ_CANDS=0: the DUMP path, A/B runs); read once
// like MIVS_FALLBACK_SYNC
std::atomic<int> g_pq_cands{-1};

bool pq_cand_slots() {
  int v = g_pq_cands.load(std::memory_order_relaxed);
  if (v < 0) {
    v = env_int("MIVS_PQ_CANDS", 1) != 0 ? 1 : 0;
    g_pq_cands.store(v, std::memory_order_relaxed);
  }
  return v == 1;
}

void reload_settings() {
  g_fallback_sync.store(-1, std::memory_order_relaxed);
  g_pq_cands.store(-1, std::memory_order_relaxed);
  engine_settings_reset();
}

void exact_fallback_on_device(mivs_index_s* idx, hipStream_t s, const float* q, int64_t nq, int k, int np,
                              float* out_d, int64_t* out_i) {
  Workspace& ws = idx->ws;
  const ListSet& L = idx->lists;
  const int64_t ne = nq * np;
  const int qtile = pick_qtile(k, idx->d, idx->G);
  ws.counts.reserve(sizeof(int) * L.n_lists);
  ws.bucket_off.reserve(sizeof(int) * (L.n_lists + 1));
  ws.work_off.reserve(sizeof(int) * (L.n_lists + 1));
  ws.bucket_q.reserve(sizeof(int64_t) * ne);
  ws.bucket_slot.reserve(sizeof(int64_t) * ne);
  ws.slot_begin.reserve(sizeof(int64_t) * (nq + 1));
  ws.counter.reserve(16);
  const int* n_dev = ws.pf_stats.as<int>();
  HIPCHK(launch_probe_map_dev(n_dev, nq, ws.ovf_q.as<int64_t>(), ws.probes_i.as<int64_t>(), np, L.n_lists,
                              L.goff.as<int64_t>(), idx->G, qtile, ws.counts.as<int>(), ws.bucket_off.as<int>(),
                              ws.work_off.as<int>(), ws.bucket_q.as<int64_t>(), ws.bucket_slot.as<int64_t>(),
                              ws.slot_begin.as<int64_t>(), ws.counter.as<int>(), s));
  // the partials of every query the batch could send here (the count is not known on the host)
  const int64_t max_slots = nq * L.top_chunks_prefix[std::min<int64_t>(np, L.n_lists)];
  ws.part_d.reserve(sizeof(float) * (size_t)std::max<int64_t>(max_slots * k, 1));
  ws.part_i.reserve(sizeof(int64_t) * (size_t)std::max<int64_t>(max_slots * k, 1));
  ScanJob j{&L, idx->G, q, ws.qn.as<float>(), idx->d, idx->dp, k, idx->metric, ws.bucket_q.as<int64_t>(),
            ws.bucket_slot.as<int64_t>(), ws.bucket_off.as<int>(), ws.work_off.as<int>(), ws.part_d.as<float>(),
            ws.part_i.as<int64_t>(), qtile};
  j.counter_zeroed = true;
  run_scan(j, idx->device, ws, s);
  MergeArgs m{};
  m.in_d = ws.part_d.as<float>();
  m.in_i = ws.part_i.as<int64_t>();
  m.slot_begin = ws.slot_begin.as<int64_t>();
  m.nq = nq;
  m.k_in = k;
  m.k = k;
  m.metric = idx->metric;
  m.out_d = out_d;
  m.out_i = out_i;
  m.nq_dev = n_dev;
  m.out_rows = ws.ovf_q.as<int64_t>();
  HIPCHK(launch_merge(m, s));
}

// K11 over the scan's candidate slots, then the exact scan for the queries the refine could not prove
// (scattered back into out_d / out_i). force_ovf (K13): device flag, nonzero -> every query falls back.
void pf_refine_fallback(mivs_index_s* idx, hipStream_t s, const float* q, int64_t nq, int k, int np, float* out_d,
                        int64_t* out_i, const float* slot_key, const int* slot_pos, const float* slot_bound,
                        const int* force_ovf, const int64_t* slot_begin, int slot_k, bool fallback_pf,
                        float* kth_out, const float* window_cap, int verify_sel, bool stats_zeroed,
                        const int* slot_cnt, int slot_cap) {
  Workspace& ws = idx->ws;
  const ListSet& L = idx->lists;
  const int dp = idx->dp;
  ws.pf_stats.reserve(32);
  // (the k-th-only modes leave the stats alone; stats_zeroed: an earlier kernel of the search zeroed them)
  if (!kth_out && !stats_zeroed) HIPCHK(hipMemsetAsync(ws.pf_stats.p, 0, 32, s));
  ws.ovf_q.reserve(sizeof(int64_t) * nq);
  PfRefineArgs r{};
  r.slot_key = slot_key;
  r.slot_pos = slot_pos;
  r.slot_bound = slot_bound;
  r.force_ovf = force_ovf;
  r.window_cap = window_cap;
  r.kth_out = kth_out;
  r.verify_sel = verify_sel;
  r.slot_begin = slot_begin;
  r.slot_cnt = slot_cnt;
  r.slot_cap = slot_cap;
  r.slot_k = slot_k;
  r.nq = nq;
  r.k = k;
  r.d = idx->d;
  r.dp = dp;
  r.metric = idx->metric;
  r.groups = L.groups.as<float>();
  r.row_norms = L.norms.as<float>();
  r.row_ids = L.ids.as<int64_t>();
  r.queries = q;
  r.qnorms = ws.qn.as<float>();
  r.qres = ws.qres.as<float>();
  r.x_norm_max = idx->x_norm_max;
  r.x_res_max = idx->x_res_max;
  r.out_d = out_d;
  r.out_i = out_i;
  r.ovf_count = ws.pf_stats.as<int>();
  r.ovf_q = ws.ovf_q.as<int64_t>();
  r.n_window = reinterpret_cast<int64_t*>(ws.pf_stats.as<char>() + 8);
  HIPCHK(launch_pf_refine(r, s));
  if (kth_out) return;
  if (fallback_pf && device_fallback_ok(idx, k, nq, np)) {  // K13's unproven queries: no host round trip
    exact_fallback_on_device(idx, s, q, nq, k, np, out_d, out_i);
    idx->last_stats_dev = true;
    return;
  }
  ws.h_stats.reserve(16);
  int64_t* h = ws.h_stats.as<int64_t>();
  HIPCHK(hipMemcpyAsync(h, ws.pf_stats.p, 16, hipMemcpyDeviceToHost, s));
  spin_wait(s);  // the only host sync of the search: the fallback size
  const int64_t novf = (int64_t)(int32_t)(h[0] & 0xFFFFFFFF);
  idx->last_ovf += novf;
  idx->last_window += h[1];
  if (novf > 0 && fallback_pf) {
    // K13's unproven queries go through K10 (whose own unproven ones go to the exact scan): own buffers,
    // since the nested search uses the ovf_* ones
    ws.rs_ovf_q.reserve(sizeof(int64_t) * (size_t)novf);
    ws.rs_ovf_rows.reserve(sizeof(float) * (size_t)novf * idx->d);
    ws.rs_ovf_d.reserve(sizeof(float) * (size_t)novf * k);
    ws.rs_ovf_i.reserve(sizeof(int64_t) * (size_t)novf * k);
    HIPCHK(hipMemcpyAsync(ws.rs_ovf_q.p, ws.ovf_q.p, sizeof(int64_t) * novf, hipMemcpyDeviceToDevice, s));
    HIPCHK(launch_gather_rows(q, idx->d, ws.rs_ovf_q.as<int64_t>(), novf, ws.rs_ovf_rows.as<float>(), s));
    ivf_search_batch(idx, s, ws.rs_ovf_rows.as<float>(), novf, k, np, ws.rs_ovf_d.as<float>(),
                     ws.rs_ovf_i.as<int64_t>(), nullptr, true, false, false);
    HIPCHK(launch_scatter_results(ws.rs_ovf_d.as<float>(), ws.rs_ovf_i.as<int64_t>(), ws.rs_ovf_q.as<int64_t>(), novf,
                                  k, out_d, out_i, s));
    return;
  }
  if (novf > 0) {
    ws.ovf_rows.reserve(sizeof(float) * (size_t)novf * idx->d);
    ws.ovf_d.reserve(sizeof(float) * (size_t)novf * k);
    ws.ovf_i.reserve(sizeof(int64_t) * (size_t)novf * k);
    HIPCHK(launch_gather_rows(q, idx->d, ws.ovf_q.as<int64_t>(), novf, ws.ovf_rows.as<float>(), s));
    if (idx->kind == 1) {  // brute force: the exact scan of the one list
      ws.qn.reserve(sizeof(float) * novf);
      HIPCHK(launch_row_norms(ws.ovf_rows.as<float>(), novf, idx->d, ws.qn.as<float>(), s));
      single_list_topk(idx->lists, idx->G, ws.ovf_rows.as<float>(), ws.qn.as<float>(), nullptr, novf, idx->d, idx->dp,
                       k, idx->metric, ws.ovf_d.as<float>(), ws.ovf_i.as<int64_t>(), idx->device, ws, s);
    } else {
      ivf_search_batch(idx, s, ws.ovf_rows.as<float>(), novf, k, np, ws.ovf_d.as<float>(), ws.ovf_i.as<int64_t>(),
                       nullptr, false, false);
    }
    HIPCHK(launch_scatter_results(ws.ovf_d.as<float>(), ws.ovf_i.as<int64_t>(), ws.ovf_q.as<int64_t>(), novf, k,
                                  out_d, out_i, s));
  }
}

// The coarse probe for n_probes > 16 (beyond K3w's register top-k): K3 in DUMP mode (every key of the
// centroid list, written as computed) + K8 per query, instead of K3's 32- or 64-entry register top-k per
// lane + K7 over the chunks (same keys, same (key, id) order: bit-identical probes).
bool coarse_dump(int np) { return np > 16; }

// Centroid chunk of the coarse probe: enough (query tile, chunk) work items for >= 4 per CU -- a 10k-query
// batch over 1024 centroids is only 313 query tiles -- with K7 merging the chunks' top-n_probes
// K3w's DUMP (n_probes > 16, 64-query tiles, two workgroups of 4 waves per CU): >= 8 items per CU in chunks of a
// multiple of 4 groups (a pass is one group per wave): 194 us against 212 us at 8 groups (configs[2], 1024 lists)
int coarse_groups(const mivs_index_s* idx, int64_t nq, int np) {
  const int64_t ng = std::max<int64_t>(1, idx->cents.n_groups);
  if (coarse_dump(np) && scan_wide_supported(0, idx->d, idx->dp, 4)) {
    const int64_t tiles = std::max<int64_t>(1, ceil_div(nq, 64));
    const int64_t chunks = std::min<int64_t>(ng, std::max<int64_t>(1, ceil_div(8LL * cu_count(idx->device), tiles)));
    const int64_t g4 = ceil_div(ceil_div(ng, chunks), 4) * 4;
    return (int)std::max<int64_t>(1, std::min<int64_t>(idx->G, g4));
  }
  const int64_t tiles = std::max<int64_t>(1, ceil_div(nq, kQTile));
  const int64_t chunks = std::min<int64_t>(ng, std::max<int64_t>(1, ceil_div(4LL * cu_count(idx->device), tiles)));
  return (int)std::max<int64_t>(1, std::min<int64_t>(idx->G, ceil_div(ng, chunks)));
}

void ivf_search_batch(mivs_index_s* idx, hipStream_t s, const float* q, int64_t nq, int k, int np, float* out_d,
                      int64_t* out_i, int32_t* out_probes, bool allow_pf, bool prof, bool allow_rs) {
  Workspace& ws = idx->ws;
  ProfRec* pr = prof && g_profiling.load() ? idx->prof.begin(s) : nullptr;
  const bool pf = allow_pf && idx->groups_h.p != nullptr && (k <= kPfMaxK || (allow_rs && lk_use(idx, k, np)));
  ws.qn.reserve(sizeof(float) * nq);
  // the pre-filter search's query conversions in the same pass as the norms (one read of the batch)
  ws.prep_q = nullptr;
  if (pf && idx->d % 4 == 0 && (reinterpret_cast<uintptr_t>(q) & 15) == 0 && idx->dp <= 1024) {
    const bool f8 = rs_use(idx, np) && k <= kPfMaxK && rs_pre_f8(idx, s);
    ws.qh.reserve(sizeof(uint16_t) * (size_t)nq * idx->dp);
    ws.qscale.reserve(sizeof(float) * nq);
    ws.qres.reserve(sizeof(float) * nq);
    if (f8) {
      ws.q8.reserve((size_t)nq * idx->dp);
      ws.qscale8.reserve(sizeof(float) * nq);
    }
    HIPCHK(launch_queries_prep(q, nq, idx->d, idx->dp, idx->hx_exp, idx->hx8, ws.qn.as<float>(), ws.qh.as<uint16_t>(),
                               ws.qscale.as<float>(), ws.qres.as<float>(), f8 ? ws.q8.as<uint8_t>() : nullptr,
                               f8 ? ws.qscale8.as<float>() : nullptr, s));
    if (host_trace().on) host_trace().t_first = std::chrono::steady_clock::now();
    ws.prep_q = q;
    ws.prep_nq = nq;
    ws.prep_f8 = f8;
  } else {
    HIPCHK(launch_row_norms(q, nq, idx->d, ws.qn.as<float>(), s));
  }
  // coarse: top-n_probes centroids per query
  ws.probes_d.reserve(sizeof(float) * nq * np);
  ws.probes_i.reserve(sizeof(int64_t) * nq * np);
  single_list_topk(idx->cents, coarse_groups(idx, nq, np), q, ws.qn.as<float>(), nullptr, nq, idx->d, idx->dp, np,
                   idx->metric, ws.probes_d.as<float>(), ws.probes_i.as<int64_t>(), idx->device, ws, s,
                   coarse_dump(np));
  if (out_probes) HIPCHK(launch_i64_to_i32(ws.probes_i.as<int64_t>(), nq * np, out_probes, s));
  ivf_search_probed(idx, s, q, nq, k, np, out_d, out_i, pf, pr, prof, nullptr, allow_rs);
}

// the fine part of a search whose probes are in ws.probes_i ([nq][np]) and query norms in ws.qn:
// probe map, then the pre-filter scan + refine (pf) or the exact scan + merge / select
// K13 serves the fp16 pre-filter search of an IVF index probed by >= 2 lists per query (its bound T_q
// comes from a pre-pass over each query's nearest list); MIVS_PF_ROWSTAT=0 keeps K10 (A/B runs)
bool rs_use(const mivs_index_s* idx, int np) {
  const char* e = getenv("MIVS_PF_ROWSTAT");
  return idx->kind == 0 && np >= 2 && rs_scan_supported(idx->dp) && !(e && e[0] == '0');
}

// K13's fp8 pre-pass nomination (MIVS_RS_PRE_F8=0: off) where the index has the fp8 copy (pf_build_f8)
bool rs_pre_f8(mivs_index_s* idx, hipStream_t) {
  const char* e = getenv("MIVS_RS_PRE_F8");
  if (e && e[0] == '0') return false;
  return idx->groups_f8.p != nullptr;
}

// K13's bucketing in one pass into fixed-capacity per-query runs (MIVS_RS_BUCKET_1P=0: the two-pass CSR form);
// MIVS_RS_QCAP: the run capacity (a query with more candidates is not proven and takes the fallback)
bool rs_bucket_one_pass() {
  const char* e = getenv("MIVS_RS_BUCKET_1P");
  return !(e && e[0] == '0');
}
// (default: the batch's share of kRsCandBudget entries, at least kRsQCap, at most the rows a query can probe)
int rs_qcap(int64_t nq, int64_t max_probed) {
  const char* e = getenv("MIVS_RS_QCAP");
  if (e && atoi(e) > 0) return atoi(e);
  const int64_t c = std::max<int64_t>(kRsQCap, kRsCandBudget / std::max<int64_t>(nq, 1));
  return (int)std::max<int64_t>(1, std::min<int64_t>({c, max_probed, INT32_MAX / 2}));
}

// records per K13 stream: twice the batch's queries, at most kRsWaveCapMax (MIVS_RS_WAVE_CAP overrides it: the
// lost-stream path is then testable at small sizes). Batches are at most kRsMaxBatch queries (ivf_search_impl),
// so a stream's mean length (~160 records per 1,000 queries at the benchmark shape) stays far below the cap.
// Large k (K16): est_cand candidates per query, one record each at that hit density, twice the mean stream.
int rs_wave_cap(int64_t nq, int k = 1, int64_t est_cand = 0, int n_waves = 1) {
  const char* e = getenv("MIVS_RS_WAVE_CAP");
  if (e && atoi(e) > 0) return atoi(e);
  if (k > kPfMaxK)
    return (int)std::min<int64_t>(kRsWaveCapMaxLk, std::max<int64_t>(4096, 2 * nq * est_cand / std::max(1, n_waves)));
  return (int)std::min<int64_t>(kRsWaveCapMax, std::max<int64_t>(1024, 2 * nq));
}

// K16 serves k in (kPfMaxK, kMaxSelectK] through K13 when the index has the fp16 copy
// (MIVS_LARGE_K_PF=0: the exact K3 DUMP + K8 path, A/B runs)
bool lk_use(const mivs_index_s* idx, int k, int np) {
  const char* e = getenv("MIVS_LARGE_K_PF");
  return k > kPfMaxK && k <= kMaxSelectK && idx->groups_h.p != nullptr && rs_use(idx, np) && !(e && e[0] == '0');
}

// T_q's sample (K16): the first 1/div groups of every list (at least one); host-side bounds over the lists of
// the sample's rank r_max (every query's r_q is below it: r_q grows with the query's sample fraction, a weighted
// mean of its lists' fractions) and of the candidates per query it leads to
struct LkPlan {
  int div = kLkSampleDiv;
  int r_max = 1;
  int64_t slots_per_q = 1;  // K3 DUMP slots of a query over its sample lists (at most)
  int64_t est_cand = 1;     // candidates per query K13 is expected to stream (T_q's global rank, about r / f)
};
LkPlan lk_plan(const mivs_index_s* idx, int k, int np) {
  const ListSet& L = idx->lists;
  LkPlan p;
  const char* de = getenv("MIVS_LK_SAMPLE_DIV");
  p.div = std::max(1, de ? atoi(de) : kLkSampleDiv);
  double f_max = 0.0, rows = 0.0, smp = 0.0;
  std::vector<int64_t> ch(L.n_lists);
  for (int l = 0; l < L.n_lists; ++l) {
    const int64_t ng = L.h_goff[l + 1] - L.h_goff[l], nr = L.h_off[l + 1] - L.h_off[l];
    const int64_t sg = std::min<int64_t>(ng, std::max<int64_t>(1, ceil_div(ng, p.div)));
    const double sr = (double)std::min<int64_t>(nr, sg * kGroupRows);
    ch[l] = ceil_div(sg, idx->G);
    if (nr > 0) f_max = std::max(f_max, sr / (double)nr);
    rows += (double)nr;
    smp += sr;
  }
  std::sort(ch.begin(), ch.end(), std::greater<int64_t>());
  p.slots_per_q = 0;
  for (int l = 0; l < std::min(np, L.n_lists); ++l) p.slots_per_q += ch[l];
  p.slots_per_q = std::max<int64_t>(1, p.slots_per_q);
  const double mu = (double)k * f_max;
  p.r_max = (int)std::min<double>(kMaxSelectK, std::ceil(mu + kLkSampleZ * std::sqrt(mu) + 1.0));
  const double f_avg = rows > 0 ? smp / rows : 1.0;
  p.est_cand = (int64_t)std::ceil(std::max((double)k, (double)p.r_max / std::max(f_avg, 1e-9)));
  return p;
}

// queries per K16 batch: the record streams, the windows and the sample's DUMP slots within the large-k workspace
// (MIVS_LK_WORKSPACE_MB, default 12 GiB; K13 reads every probed row once per batch, so fewer batches are better)
int64_t lk_batch(const mivs_index_s* idx, int64_t nq, int k, int np) {
  const LkPlan p = lk_plan(idx, k, np);
  const char* e = getenv("MIVS_LK_WORKSPACE_MB");
  const size_t budget = (size_t)std::max<long long>(e ? atoll(e) : 12288, 1) << 20;
  const size_t per_q = (size_t)p.est_cand * (2 * kRsRecInt4 * 16 + 8) + (size_t)lk_cap(k) * 12 +
                       (size_t)p.slots_per_q * ((size_t)idx->G * kGroupRows * 4 + 16);
  return std::max<int64_t>(1, std::min<int64_t>(nq, (int64_t)(budget / std::max<size_t>(per_q, 1))));
}

// K16 step 1: T_q per query into ws.pre_kth from an exact scan of the sample (K3 DUMP over the
// split lists 2l = the sample of list l) and the sample's r_q-th key (k_lk_sample_kth)
void lk_prepass(mivs_index_s* idx, hipStream_t s, const float* q, int64_t nq, int k, int np, const LkPlan& p) {
  Workspace& ws = idx->ws;
  const ListSet& L = idx->lists;
  const int nl2 = 2 * L.n_lists;
  const int64_t ne = nq * np;
  ws.pre_goff.reserve(sizeof(int64_t) * ((size_t)nl2 + 1));
  HIPCHK(launch_rs_pre_lists(L.goff.as<int64_t>(), L.n_lists, p.div, 1, nullptr, 0, np, ws.pre_goff.as<int64_t>(),
                             nullptr, s));
  ws.lk_probes.reserve(sizeof(int64_t) * ne);
  HIPCHK(launch_lk_sample_probes(ws.probes_i.as<int64_t>(), ne, ws.lk_probes.as<int64_t>(), s));
  ws.counts.reserve(sizeof(int) * nl2);
  ws.fill.reserve(sizeof(int) * nl2);
  ws.bucket_off.reserve(sizeof(int) * (nl2 + 1));
  ws.work_off.reserve(sizeof(int) * (nl2 + 1));
  ws.bucket_q.reserve(sizeof(int64_t) * ne);
  ws.bucket_slot.reserve(sizeof(int64_t) * ne);
  ws.qp_slots.reserve(sizeof(int64_t) * ne);
  ws.slot_begin.reserve(sizeof(int64_t) * (nq + 1));
  const size_t stb = scan_tmp_bytes(ne) + sizeof(int64_t) * (size_t)ne;
  ws.scan_tmp.reserve(stb);
  HIPCHK(launch_probe_map(ws.lk_probes.as<int64_t>(), nq, np, nl2, ws.pre_goff.as<int64_t>(), idx->G, kQTile,
                          ws.counts.as<int>(), ws.fill.as<int>(), ws.bucket_off.as<int>(), ws.work_off.as<int>(),
                          ws.bucket_q.as<int64_t>(), ws.bucket_slot.as<int64_t>(), ws.qp_slots.as<int64_t>(),
                          ws.slot_begin.as<int64_t>(), ws.scan_tmp.p, stb, s));
  const int64_t slot_rows = (int64_t)idx->G * kGroupRows;
  const int64_t slots = nq * p.slots_per_q;
  ws.part_d.reserve(sizeof(float) * (size_t)(slots * slot_rows));
  ws.part_i.reserve(sizeof(int64_t) * (size_t)(slots * 2));
  ScanJob j{&L, idx->G, q, ws.qn.as<float>(), idx->d, idx->dp, p.r_max, idx->metric, ws.bucket_q.as<int64_t>(),
            ws.bucket_slot.as<int64_t>(), ws.bucket_off.as<int>(), ws.work_off.as<int>(), ws.part_d.as<float>(),
            ws.part_i.as<int64_t>(), kQTile};
  j.dump = true;
  j.goff = ws.pre_goff.as<int64_t>();
  j.n_lists = nl2;
  run_scan(j, idx->device, ws, s);
  ws.pre_kth.reserve(sizeof(float) * nq);
  HIPCHK(launch_lk_sample_kth(ws.probes_i.as<int64_t>(), nq, np, L.off.as<int64_t>(), ws.pre_goff.as<int64_t>(), k,
                              kLkSampleZ, ws.part_d.as<float>(), ws.part_i.as<int64_t>(), ws.slot_begin.as<int64_t>(),
                              (int)slot_rows, ws.pre_kth.as<float>(), s));
  // the fp16 queries, their scales and residuals for the headers and tiles
  ws.qh.reserve(sizeof(uint16_t) * (size_t)nq * idx->dp);
  ws.qscale.reserve(sizeof(float) * nq);
  ws.qres.reserve(sizeof(float) * nq);
  HIPCHK(launch_queries_to_half(q, nq, idx->d, idx->dp, idx->hx_exp, ws.qh.as<uint16_t>(), ws.qscale.as<float>(),
                                ws.qres.as<float>(), s));
}

// the exact search (K3 / K3w, or K3 DUMP + K8 for k > 64) of n query rows, in query batches bounded by the select
// workspace (the fallback of the pre-filter paths)
void exact_search_batched(mivs_index_s* idx, hipStream_t s, const float* rows, int64_t n, int k, int np, float* out_d,
                          int64_t* out_i) {
  int64_t qb = n;
  if (k > kMaxK) {
    const ListSet& L = idx->lists;
    const int64_t per_q_slots = std::max<int64_t>(1, L.top_chunks_prefix[std::min<int64_t>(np, L.n_lists)]);
    qb = select_batch(n, (size_t)per_q_slots * ((size_t)idx->G * kGroupRows * 4 + 16));
  }
  for (int64_t b0 = 0; b0 < n; b0 += qb) {
    const int64_t nb = std::min<int64_t>(qb, n - b0);
    ivf_search_batch(idx, s, rows + b0 * (int64_t)idx->d, nb, k, np, out_d + b0 * k, out_i + b0 * k, nullptr, false,
                     false);
  }
}

// K16 steps 3-5 over K13's candidate runs (ws.cand_off / cand_key / cand_pos, T_q in ws.rs_tq), then the exact scan
// for the queries it could not prove
void lk_finish(mivs_index_s* idx, hipStream_t s, const float* q, int64_t nq, int k, int np, float* out_d,
               int64_t* out_i, const int* lost) {
  Workspace& ws = idx->ws;
  const ListSet& L = idx->lists;
  const int cap = lk_cap(k);
  ws.lk_win_pos.reserve(sizeof(int) * (size_t)nq * cap);
  ws.lk_win_key.reserve(sizeof(float) * (size_t)nq * cap);
  ws.lk_win_n.reserve(sizeof(int) * (size_t)nq);
  ws.lk_chunks.reserve(sizeof(int64_t) * (size_t)(nq + 1));
  ws.lk_chunk_off.reserve(sizeof(int64_t) * (size_t)(nq + 1));
  ws.pf_stats.reserve(32);
  HIPCHK(hipMemsetAsync(ws.pf_stats.p, 0, 32, s));
  ws.ovf_q.reserve(sizeof(int64_t) * nq);
  LkArgs a{};
  a.cand_off = ws.cand_off.as<int64_t>();
  a.cand_key = ws.cand_key.as<float>();
  a.cand_pos = ws.cand_pos.as<int>();
  a.tq = ws.rs_tq.as<float>();
  a.qnorms = ws.qn.as<float>();
  a.qres = ws.qres.as<float>();
  a.x_norm_max = idx->x_norm_max;
  a.x_res_max = idx->x_res_max;
  a.d = idx->d;
  a.dp = idx->dp;
  a.k = k;
  a.cap = cap;
  a.metric = idx->metric;
  a.nq = nq;
  a.force_ovf = lost;
  a.win_pos = ws.lk_win_pos.as<int>();
  a.win_key = ws.lk_win_key.as<float>();
  a.win_n = ws.lk_win_n.as<int>();
  a.ovf_count = ws.pf_stats.as<int>();
  a.ovf_q = ws.ovf_q.as<int64_t>();
  a.n_window = reinterpret_cast<int64_t*>(ws.pf_stats.as<char>() + 8);
  a.chunk_off = ws.lk_chunk_off.as<int64_t>();
  a.groups = L.groups.as<float>();
  a.row_norms = L.norms.as<float>();
  a.row_ids = L.ids.as<int64_t>();
  a.queries = q;
  a.out_d = out_d;
  a.out_i = out_i;
  HIPCHK(launch_lk_window(a, s));
  HIPCHK(launch_lk_chunks(a.win_n, nq, ws.lk_chunks.as<int64_t>(), s));
  ws.scan_tmp.reserve(scan_tmp_bytes(nq + 1));
  HIPCHK(launch_exclusive_scan_i64(ws.lk_chunks.as<int64_t>(), ws.lk_chunk_off.as<int64_t>(), nq + 1, ws.scan_tmp.p, s));
  HIPCHK(launch_lk_recompute(a, cu_count(idx->device), s));
  HIPCHK(launch_lk_sort(a, s));
  // (the fallback size and window count through the pinned stats: a pageable destination would make the copy
  // host-synchronous and the polling pointless)
  ws.h_stats.reserve(16);
  int64_t* h = ws.h_stats.as<int64_t>();
  HIPCHK(hipMemcpyAsync(h, ws.pf_stats.p, 16, hipMemcpyDeviceToHost, s));
  spin_wait(s);  // the fallback size
  const int64_t novf = (int64_t)(int32_t)(h[0] & 0xFFFFFFFF);
  idx->last_ovf += novf;
  idx->last_window += h[1];
  if (novf > 0) {
    ws.rs_ovf_q.reserve(sizeof(int64_t) * (size_t)novf);
    ws.rs_ovf_rows.reserve(sizeof(float) * (size_t)novf * idx->d);
    ws.rs_ovf_d.reserve(sizeof(float) * (size_t)novf * k);
    ws.rs_ovf_i.reserve(sizeof(int64_t) * (size_t)novf * k);
    HIPCHK(hipMemcpyAsync(ws.rs_ovf_q.p, ws.ovf_q.p, sizeof(int64_t) * novf, hipMemcpyDeviceToDevice, s));
    HIPCHK(launch_gather_rows(q, idx->d, ws.rs_ovf_q.as<int64_t>(), novf, ws.rs_ovf_rows.as<float>(), s));
    exact_search_batched(idx, s, ws.rs_ovf_rows.as<float>(), novf, k, np, ws.rs_ovf_d.as<float>(),
                         ws.rs_ovf_i.as<int64_t>());
    HIPCHK(launch_scatter_results(ws.rs_ovf_d.as<float>(), ws.rs_ovf_i.as<int64_t>(), ws.rs_ovf_q.as<int64_t>(), novf,
                                  k, out_d, out_i, s));
  }
}

// The K13 search of queries whose probes are in ws.probes_i and norms in ws.qn:
//   1. T_q: k <= 16, a pre-pass over a sample of each query's nearest list through K10 + K11 (the k-th key there);
//      large k, an exact scan of a uniform sample of the probed rows (lk_prepass);
//   2. per-query header {qs, uf, qn, q}: uf is the filter bound for T_q;
//   3. probe map in (list, 8-group block) items, one query tile column per list;
//   4. K13 streams every one-fma filter hit (a superset of the approximate keys <= T_q) per wave;
//   5. k <= 16: K11 over the buffers; large k: K16 (window, pinned keys, sort); then the exact fallback.
void rs_search(mivs_index_s* idx, hipStream_t s, const float* q, int64_t nq, int k, int np, float* out_d,
               int64_t* out_i, ProfRec* pr) {
  Workspace& ws = idx->ws;
  const ListSet& L = idx->lists;
  const int dp = idx->dp;
  const int64_t ne = nq * np;
  const bool large = k > kPfMaxK;
  // ws.probes_i keeps every query's probes; the pre-pass's one split list per query goes to ws.pre_probes
  ws.pre_probes.reserve(sizeof(int64_t) * nq);
  LkPlan plan;
  bool pre_f8 = false;
  int pre_div = 0, pre_sel = 0;
  if (large) {
    plan = lk_plan(idx, k, np);
    lk_prepass(idx, s, q, nq, k, np, plan);
  } else {
    // 1. a sample of the nearest list of every query (probe 0): its first 1/div groups (the rows of a list
    // are in no particular order) through K10 over the split lists, and the k-th smallest approximate key
    // of each query's candidates there (K11's first phase only)
    ws.pre_goff.reserve(sizeof(int64_t) * (2 * (size_t)L.n_lists + 1));
    // fp8 nomination (MIVS_RS_PRE_F8, default on where it applies): the sample scored on fp8 copies over every
    // dim, the kRsPreSel best rows of each query verified with fp32 keys
    pre_f8 = rs_pre_f8(idx, s);
    pre_sel = pre_f8 ? std::min(kPfMaxK, std::max(k, kRsPreSel)) : 0;
    const char* pde = getenv("MIVS_RS_PRE_DIV");
    pre_div = std::max(1, pde ? atoi(pde) : (pre_f8 ? kRsPreDivF8 : kRsPreDiv));
    HIPCHK(launch_rs_pre_lists(L.goff.as<int64_t>(), L.n_lists, pre_div, ceil_div(k, kGroupRows),
                               ws.probes_i.as<int64_t>(), nq, np, ws.pre_goff.as<int64_t>(),
                               ws.pre_probes.as<int64_t>(), s));
    const int nl2 = 2 * L.n_lists;
    ws.counts.reserve(sizeof(int) * nl2);
    ws.fill.reserve(sizeof(int) * nl2);
    ws.bucket_off.reserve(sizeof(int) * (nl2 + 1));
    ws.work_off.reserve(sizeof(int) * (nl2 + 1));
    ws.bucket_q.reserve(sizeof(int64_t) * nq);
    ws.bucket_slot.reserve(sizeof(int64_t) * nq);
    ws.qp_slots.reserve(sizeof(int64_t) * nq);
    ws.slot_begin.reserve(sizeof(int64_t) * (nq + 1));
    const size_t stb = scan_tmp_bytes(nq) + sizeof(int64_t) * (size_t)nq;
    ws.scan_tmp.reserve(stb);
    HIPCHK(launch_probe_map(ws.pre_probes.as<int64_t>(), nq, 1, nl2, ws.pre_goff.as<int64_t>(), idx->pf_G, kPfQTile,
                            ws.counts.as<int>(), ws.fill.as<int>(), ws.bucket_off.as<int>(), ws.work_off.as<int>(),
                            ws.bucket_q.as<int64_t>(), ws.bucket_slot.as<int64_t>(), ws.qp_slots.as<int64_t>(),
                            ws.slot_begin.as<int64_t>(), ws.scan_tmp.p, stb, s));
    ws.pre_kth.reserve(sizeof(float) * nq);
    pf_scan_refine(idx, s, q, nq, k, 1, nullptr, nullptr, nullptr, ws.pre_goff.as<int64_t>(), nl2,
                   ws.pre_kth.as<float>(), pre_sel, pre_f8,
                   engine_setting(kSetPfRawLists, "MIVS_PF_RAW_LISTS", 1) != 0);
  }
  // 2. headers (the pre-pass left the fp16 queries, their scales and residuals in ws.qh / qscale / qres)
  ws.qhdr.reserve(sizeof(float4) * (nq + 1));
  float4* qhdr = ws.qhdr.as<float4>();
  ws.rs_tq.reserve(sizeof(float) * nq);
  const bool one_pass = !large && rs_bucket_one_pass();
  idx->last_rs_one_pass = one_pass;
  if (one_pass) {  // (the headers' launch zeroes the one-pass bucketing's counts and the final refine's stats)
    ws.rs_qcnt.reserve(sizeof(int) * (size_t)nq);
    ws.pf_stats.reserve(32);
  }
  HIPCHK(launch_rs_headers(ws.pre_kth.as<float>(), nq, ws.qscale.as<float>(), ws.qn.as<float>(), ws.qres.as<float>(),
                           idx->x_norm_max, idx->x_res_max, dp, idx->metric, qhdr, ws.rs_tq.as<float>(), s,
                           one_pass ? ws.rs_qcnt.as<int>() : nullptr, one_pass ? nq : 0,
                           one_pass ? ws.pf_stats.as<int>() : nullptr, one_pass ? 8 : 0));
  // 3. probe map: items = (list, block of kRsBlockGroups groups); every query of a list in one tile column
  ws.counts.reserve(sizeof(int) * L.n_lists);
  ws.fill.reserve(sizeof(int) * L.n_lists);
  ws.bucket_off.reserve(sizeof(int) * (L.n_lists + 1));
  ws.work_off.reserve(sizeof(int) * (L.n_lists + 1));
  ws.bucket_q.reserve(sizeof(int64_t) * ne);
  ws.bucket_slot.reserve(sizeof(int64_t) * ne);
  ws.qp_slots.reserve(sizeof(int64_t) * ne);
  ws.slot_begin.reserve(sizeof(int64_t) * (nq + 1));
  const size_t stb = scan_tmp_bytes(ne) + sizeof(int64_t) * (size_t)ne;
  ws.scan_tmp.reserve(stb);
  // (the per-list query counts go to their own buffer, which the search stats read: a nested search reuses ws.counts)
  ws.stat_counts.reserve(sizeof(int) * L.n_lists);
  HIPCHK(launch_probe_map(ws.probes_i.as<int64_t>(), nq, np, L.n_lists, L.goff.as<int64_t>(), kRsBlockGroups,
                          1 << 30, ws.stat_counts.as<int>(), ws.fill.as<int>(), ws.bucket_off.as<int>(),
                          ws.work_off.as<int>(), ws.bucket_q.as<int64_t>(), ws.bucket_slot.as<int64_t>(),
                          ws.qp_slots.as<int64_t>(), nullptr, ws.scan_tmp.p, stb, s));  // (no output slots)
  // the query tiles in the LDS image layout (one contiguous 1 KiB per DMA wave-instruction; a per-lane gather
  // straight from the fp16 query matrix was measured 0.45 ms slower per launch: 16 separate 64-B segments per
  // DMA instruction)
  ws.rs_tiles.reserve((size_t)rs_tiles_bytes(ne, L.n_lists, dp));
  HIPCHK(launch_rs_tiles(ws.bucket_q.as<int64_t>(), ws.bucket_off.as<int>(), L.n_lists, ne, ws.qh.as<uint16_t>(), qhdr,
                         (int)nq, dp, ws.rs_tiles.as<char>(), s));
  // 4. K13
  int64_t max_items = 0;  // every list probed: the item table's bound (the probe map decides the count)
  int64_t max_groups = 1;  // the largest list's groups (a query's candidates are at most np of its lists' rows)
  for (int l = 0; l < L.n_lists; ++l) {
    max_items += ceil_div(L.h_goff[l + 1] - L.h_goff[l], kRsBlockGroups);
    max_groups = std::max<int64_t>(max_groups, L.h_goff[l + 1] - L.h_goff[l]);
  }
  ws.rs_items.reserve(sizeof(int4) * (size_t)std::max<int64_t>(max_items, 1));
  // items dealt from 8 queues of equal tile work, dynamically inside a queue
  ws.rs_bounds.reserve(sizeof(int) * 9);
  const int grid = std::max(8, cu_count(idx->device) / 8 * 8);
  const int n_waves = grid * kRsWaves;
  // the wave stream counts + the lost flag, the 8 item-queue counters, the spun-out wave count (the last 10 are
  // zeroed by k_rs_items)
  ws.rs_wave_cnt.reserve(sizeof(int) * (n_waves + 1 + 8 + 1));
  HIPCHK(launch_rs_items(ws.work_off.as<int>(), ws.bucket_off.as<int>(), L.goff.as<int64_t>(), L.n_lists,
                         (int)max_items, ws.rs_items.as<int4>(), ws.rs_bounds.as<int>(), s,
                         ws.rs_wave_cnt.as<int>() + n_waves, 10));
  RsScanArgs a{};
  a.groups_h = idx->groups_h.as<uint16_t>();
  a.row_norms = L.norms.as<float>();
  a.list_goff = L.goff.as<int64_t>();
  a.n_lists = L.n_lists;
  a.bucket_q = ws.bucket_q.as<int64_t>();
  a.bucket_off = ws.bucket_off.as<int>();
  a.work_off = ws.work_off.as<int>();
  a.items = ws.rs_items.as<int4>();
  a.tiles = ws.rs_tiles.as<char>();
  a.qnorms = ws.qn.as<float>();
  a.group_nmin = idx->group_nmin.as<float>();
  a.nq = (int)nq;
  a.metric = idx->metric;
  idx->last_rs_waves = n_waves;
  idx->last_rs_nq = nq;
  a.wave_cap = rs_wave_cap(nq, k, plan.est_cand, n_waves);
  ws.rs_wave_buf.reserve(sizeof(int4) * kRsRecInt4 * (size_t)n_waves * a.wave_cap);
  a.wave_buf = ws.rs_wave_buf.as<int4>();
  a.wave_cnt = ws.rs_wave_cnt.as<int>();
  a.queue = a.wave_cnt + n_waves + 1;
  a.bounds = ws.rs_bounds.as<int>();
  a.flags = env_int("MIVS_RS_FLAGS", 0);
  if (a.flags & 2) a.flags |= 1;  // stale LDS tiles: never run an epilogue on them
  Buf pbuf;
  if (a.flags & 24) {  // diagnostic: per-block clocks (8) / per-phase wave-cycles (16) to stderr
    pbuf.reserve(sizeof(unsigned long long) * (3 * grid + 16));
    HIPCHK(hipMemsetAsync(pbuf.p, 0, sizeof(unsigned long long) * (3 * grid + 16), s));
    a.prof = pbuf.as<unsigned long long>();
  }
  if (pr) HIPCHK(hipEventRecord(pr->e[1], s));
  HIPCHK(launch_rs_scan(a, dp, grid, s));
  if (pr) HIPCHK(hipEventRecord(pr->e[2], s));
  if (a.flags & 24) {
    std::vector<unsigned long long> h(3 * (size_t)grid + 16);
    HIPCHK(hipMemcpyAsync(h.data(), pbuf.p, sizeof(unsigned long long) * h.size(), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    unsigned long long t0 = ~0ull, t1 = 0, tiles_max = 0, tiles_sum = 0;
    double busy_sum = 0, busy_max = 0;
    for (int b = 0; b < grid; ++b) {
      t0 = std::min(t0, h[3 * b]);
      t1 = std::max(t1, h[3 * b + 1]);
      const double busy = (double)(h[3 * b + 1] - h[3 * b]);
      busy_sum += busy;
      busy_max = std::max(busy_max, busy);
      tiles_sum += h[3 * b + 2];
      tiles_max = std::max(tiles_max, h[3 * b + 2]);
    }
    fprintf(stderr, "[k13 blocks] span %.1f us | busy mean %.1f max %.1f us | tiles mean %.1f max %llu\n",
            (t1 - t0) / 100.0, busy_sum / grid / 100.0, busy_max / 100.0, (double)tiles_sum / grid, tiles_max);
    const double wc = (double)(h[3 * grid] + h[3 * grid + 1] + h[3 * grid + 2] + h[3 * grid + 3] + h[3 * grid + 4]);
    if (wc > 0)
      fprintf(stderr, "[k13 phases] wave-cycles %.4g | ready-wait %.3f mfma-loop %.3f own-dma-wait %.3f epilogue %.3f | "
              "cycles/tile/wave %.0f\n", wc, h[3 * grid] / wc, h[3 * grid + 1] / wc, h[3 * grid + 3] / wc,
              h[3 * grid + 2] / wc,
              tiles_sum ? wc / ((double)tiles_sum * kRsWaves) : 0.0);
    if (wc > 0)
      fprintf(stderr, "[k13 phases] mfma-result-wait %.3f (in epilogue: hit path %.3f) | wave-tiles taking the hit path "
              "%.4f of %llu\n", h[3 * grid + 4] / wc, h[3 * grid + 5] / wc,
              h[3 * grid + 7] ? (double)h[3 * grid + 6] / (double)h[3 * grid + 7] : 0.0, h[3 * grid + 7]);
    if (wc > 0 && h[3 * grid + 9] && h[3 * grid + 7] > h[3 * grid + 9])
      fprintf(stderr, "[k13 phases] k-loop cycles: items' first tile %.0f, other tiles %.0f | wave lifetime %.4g cycles "
              "(tile phases %.3f of it)\n", (double)h[3 * grid + 8] / h[3 * grid + 9],
              (double)(h[3 * grid + 1] - h[3 * grid + 8]) / (double)(h[3 * grid + 7] - h[3 * grid + 9]),
              (double)h[3 * grid + 10], wc / (double)h[3 * grid + 10]);
  }
  // the streams into per-query CSR runs (a record expands to at most 8 candidates)
  ws.cand_off.reserve(sizeof(int64_t) * (nq + 1));
  ws.rs_bucket_tmp.reserve(rs_bucket_tmp_bytes((int)nq, n_waves));
  ws.pf_stats.reserve(32);
  if (one_pass) {
    const int cap = rs_qcap(nq, (int64_t)np * max_groups * kGroupRows);
    ws.cand_key.reserve(sizeof(float) * (size_t)nq * cap);
    ws.cand_pos.reserve(sizeof(int) * (size_t)nq * cap);
    HIPCHK(launch_rs_bucket_fused(a.wave_buf, a.wave_cap, a.wave_cnt, n_waves, (int)nq, qhdr, a.row_norms, idx->metric,
                                  cap, ws.rs_qcnt.as<int>(), ws.cand_key.as<float>(), ws.cand_pos.as<int>(), s));
    // 5. exact ranking of every query's run; a window above T_q, or a run that dropped candidates, is not proven
    pf_refine_fallback(idx, s, q, nq, k, np, out_d, out_i, ws.cand_key.as<float>(), ws.cand_pos.as<int>(), nullptr,
                       a.wave_cnt + n_waves, nullptr, 1, true, nullptr, ws.rs_tq.as<float>(), 0, true,
                       ws.rs_qcnt.as<int>(), cap);
    return;
  }
  if (!large) {
    const size_t max_cand = (size_t)n_waves * a.wave_cap * 8;
    ws.cand_key.reserve(sizeof(float) * max_cand);
    ws.cand_pos.reserve(sizeof(int) * max_cand);
    HIPCHK(launch_rs_bucket(a.wave_buf, a.wave_cap, a.wave_cnt, n_waves, (int)nq, qhdr, a.row_norms,
                            idx->metric, ws.cand_off.as<int64_t>(), ws.cand_key.as<float>(), ws.cand_pos.as<int>(),
                            ws.rs_bucket_tmp.p, a.wave_cnt + n_waves, 4 * cu_count(idx->device), s, ws.pf_stats.p,
                            32));
    // 5. exact ranking of every query's run (slot = one entry); a window above T_q is not proven (its stats were
    // zeroed by the bucketing's first kernel)
    pf_refine_fallback(idx, s, q, nq, k, np, out_d, out_i, ws.cand_key.as<float>(), ws.cand_pos.as<int>(), nullptr,
                       a.wave_cnt + n_waves, ws.cand_off.as<int64_t>(), 1, true, nullptr, ws.rs_tq.as<float>(), 0,
                       true);
    return;
  }
  // large k: the candidate arrays sized by the count (one host sync: up to 8 candidates per record would be
  // several GB at this k)
  HIPCHK(launch_rs_bucket_count(a.wave_buf, a.wave_cap, a.wave_cnt, n_waves, (int)nq, qhdr, a.row_norms, idx->metric,
                                ws.cand_off.as<int64_t>(), ws.rs_bucket_tmp.p, a.wave_cnt + n_waves, s));
  ws.h_stats.reserve(16);
  HIPCHK(hipMemcpyAsync(ws.h_stats.p, ws.cand_off.as<int64_t>() + nq, sizeof(int64_t), hipMemcpyDeviceToHost, s));
  spin_wait(s);
  const int64_t total = *ws.h_stats.as<int64_t>();
  ws.cand_key.reserve(sizeof(float) * (size_t)std::max<int64_t>(total, 1));
  ws.cand_pos.reserve(sizeof(int) * (size_t)std::max<int64_t>(total, 1));
  HIPCHK(launch_rs_bucket_scatter(a.wave_buf, a.wave_cap, a.wave_cnt, n_waves, (int)nq, qhdr, a.row_norms, idx->metric,
                                  ws.cand_off.as<int64_t>(), ws.cand_key.as<float>(), ws.cand_pos.as<int>(),
                                  ws.rs_bucket_tmp.p, s));
  lk_finish(idx, s, q, nq, k, np, out_d, out_i, a.wave_cnt + n_waves);
}

void ivf_search_probed(mivs_index_s* idx, hipStream_t s, const float* q, int64_t nq, int k, int np, float* out_d,
                       int64_t* out_i, bool pf, ProfRec* pr, bool prof, const int64_t* probes, bool allow_rs) {
  Workspace& ws = idx->ws;
  if (!probes) probes = ws.probes_i.as<int64_t>();
  // probe map
  const ListSet& L = idx->lists;
  const int64_t ne = nq * np;
  const int n_lists = L.n_lists;
  const int64_t* goff = L.goff.as<int64_t>();
  ws.counts.reserve(sizeof(int) * n_lists);
  ws.fill.reserve(sizeof(int) * n_lists);
  ws.bucket_off.reserve(sizeof(int) * (n_lists + 1));
  ws.work_off.reserve(sizeof(int) * (n_lists + 1));
  ws.bucket_q.reserve(sizeof(int64_t) * ne);
  ws.bucket_slot.reserve(sizeof(int64_t) * ne);
  ws.qp_slots.reserve(sizeof(int64_t) * ne);
  ws.slot_begin.reserve(sizeof(int64_t) * (nq + 1));
  const size_t stb = scan_tmp_bytes(ne) + sizeof(int64_t) * (size_t)ne;
  ws.scan_tmp.reserve(stb);
  if (pf && k > kPfMaxK && !(allow_rs && lk_use(idx, k, np))) pf = false;  // (large k: K13 + K16 or the exact scan)
  const bool dump = k > kMaxK;
  const int qtile = pf ? kPfQTile : (dump ? kQTile : pick_qtile(k, idx->d, idx->G));
  if (prof) {
    idx->last_qtile = qtile;
    idx->last_pf = pf ? 1 : 0;
  }
  if (pf && allow_rs && rs_use(idx, np)) {
    if (prof) {
      idx->last_qtile = kRsQTile;
      idx->last_scan = 13;
    }
    rs_search(idx, s, q, nq, k, np, out_d, out_i, pr);
    if (pr) HIPCHK(hipEventRecord(pr->e[3], s));
    return;
  }
  if (prof) idx->last_scan = pf ? 10 : (qtile == 64 ? 31 : 3);
  HIPCHK(launch_probe_map(probes, nq, np, n_lists, goff,
                          pf ? idx->pf_G : idx->G, qtile, ws.counts.as<int>(), ws.fill.as<int>(),
                          ws.bucket_off.as<int>(), ws.work_off.as<int>(), ws.bucket_q.as<int64_t>(),
                          ws.bucket_slot.as<int64_t>(), ws.qp_slots.as<int64_t>(), ws.slot_begin.as<int64_t>(),
                          ws.scan_tmp.p, stb, s));
  if (pf) {
    pf_scan_refine(idx, s, q, nq, k, np, out_d, out_i, pr, goff, n_lists);
    if (pr) HIPCHK(hipEventRecord(pr->e[3], s));
    return;
  }
  // fine scan into per-(query, probe, chunk) slots: top-k partials (k <= 64) or raw keys (DUMP)
  const int64_t slot_rows = (int64_t)idx->G * kGroupRows;
  const int64_t max_slots = nq * L.top_chunks_prefix[std::min<int64_t>(np, L.n_lists)];
  const int64_t per_slot_d = dump ? slot_rows : k, per_slot_i = dump ? 2 : k;
  require(max_slots * per_slot_d < ((int64_t)1 << 40), "search workspace too large", MIVS_ERR_UNSUPPORTED);
  ws.part_d.reserve(sizeof(float) * (size_t)std::max<int64_t>(max_slots * per_slot_d, 1));
  ws.part_i.reserve(sizeof(int64_t) * (size_t)std::max<int64_t>(max_slots * per_slot_i, 1));
  ScanJob j{&L, idx->G, q, ws.qn.as<float>(), idx->d, idx->dp, k, idx->metric, ws.bucket_q.as<int64_t>(),
            ws.bucket_slot.as<int64_t>(), ws.bucket_off.as<int>(), ws.work_off.as<int>(), ws.part_d.as<float>(),
            ws.part_i.as<int64_t>(), qtile};
  j.dump = dump;
  if (pr) HIPCHK(hipEventRecord(pr->e[1], s));
  run_scan(j, idx->device, ws, s);
  if (pr) HIPCHK(hipEventRecord(pr->e[2], s));
  if (dump) {
    SelectArgs sa{};
    sa.keys = ws.part_d.as<float>();
    sa.row_ids = L.ids.as<int64_t>();
    sa.slot_info = ws.part_i.as<int64_t>();
    sa.slot_begin = ws.slot_begin.as<int64_t>();
    sa.slot_rows = (int)slot_rows;
    sa.nq = nq;
    sa.k = k;
    sa.metric = idx->metric;
    sa.out_d = out_d;
    sa.out_i = out_i;
    HIPCHK(launch_select(sa, s));
  } else {
    MergeArgs m{};
    m.in_d = ws.part_d.as<float>();
    m.in_i = ws.part_i.as<int64_t>();
    m.slot_begin = ws.slot_begin.as<int64_t>();
    m.nq = nq;
    m.k_in = k;
    m.k = k;
    m.metric = idx->metric;
    m.out_d = out_d;
    m.out_i = out_i;
    HIPCHK(launch_merge(m, s));
  }
  if (pr) HIPCHK(hipEventRecord(pr->e[3], s));
}

// K9r IVF-PQ search of queries whose probes are in ws.probes_i / probes_d: probe map in
// (list, 16-query tile, kRtRows-row chunk) items, K9r, then K7 over the (query, probe, chunk) slots'
// top-k (k <= 64) or K8 over their dumped keys (k > 64, in query batches bounded by the dump size)
bool pq_rt_use(const mivs_index_s* idx, int k) {
  const char* e = getenv("MIVS_PQ_RT");
  return !(e && e[0] == '0') && pq_rt_supported(idx->rot_dim_pad, idx->pq_dim, idx->pq_len, k);
}

void pq_search_rt(mivs_index_s* idx, hipStream_t s, const float* d_q, int64_t nq, int k, int np, float* d_dist,
                  int64_t* d_ids, ProfRec* pr, bool lut16 = false) {
  Workspace& ws = idx->ws;
  const ListSet& L = idx->lists;
  // K8 over per-slot candidate supersets of kRtSlotCap entries (64 < k <= kRtCandMax), or over every row's key
  const bool cands = k > kMaxK && k <= kRtCandMax && pq_cand_slots();
  const bool dump = k > kMaxK && !cands;
  const int per_slot = dump ? kRtRows : (cands ? kRtSlotCap : k);
  int64_t max_chunks = 0;  // slots per query at most: the np longest lists' chunk counts
  {
    std::vector<int64_t> c(L.n_lists);
    for (int l = 0; l < L.n_lists; ++l) c[l] = ceil_div(L.h_goff[l + 1] - L.h_goff[l], kRtGroups);
    std::sort(c.begin(), c.end(), std::greater<int64_t>());
    for (int l = 0; l < std::min<int>(np, L.n_lists); ++l) max_chunks += c[l];
  }
  max_chunks = std::max<int64_t>(max_chunks, 1);
  const int64_t qb = dump    ? select_batch(nq, (size_t)max_chunks * ((size_t)kRtRows * 4 + 16))
                     : cands ? select_batch(nq, (size_t)max_chunks * kRtSlotCap * 12)
                             : nq;
  const int flags = env_int("MIVS_PQ_FLAGS", 0);
  if (pr) HIPCHK(hipEventRecord(pr->e[1], s));
  for (int64_t b0 = 0; b0 < nq; b0 += qb) {
    const int64_t nb = std::min<int64_t>(qb, nq - b0);
    const int64_t ne = nb * np;
    ws.counts.reserve(sizeof(int) * L.n_lists);
    ws.fill.reserve(sizeof(int) * L.n_lists);
    ws.bucket_off.reserve(sizeof(int) * (L.n_lists + 1));
    ws.work_off.reserve(sizeof(int) * (L.n_lists + 1));
    ws.bucket_q.reserve(sizeof(int64_t) * ne);
    ws.bucket_slot.reserve(sizeof(int64_t) * ne);
    ws.qp_slots.reserve(sizeof(int64_t) * ne);
    ws.slot_begin.reserve(sizeof(int64_t) * (nb + 1));
    const size_t stb = scan_tmp_bytes(ne) + sizeof(int64_t) * (size_t)ne;
    ws.scan_tmp.reserve(stb);
    const int64_t* probes = ws.probes_i.as<int64_t>() + b0 * np;
    HIPCHK(launch_probe_map(probes, nb, np, L.n_lists, L.goff.as<int64_t>(), kRtGroups, kRtQ, ws.counts.as<int>(),
                            ws.fill.as<int>(), ws.bucket_off.as<int>(), ws.work_off.as<int>(),
                            ws.bucket_q.as<int64_t>(), ws.bucket_slot.as<int64_t>(), ws.qp_slots.as<int64_t>(),
                            ws.slot_begin.as<int64_t>(), ws.scan_tmp.p, stb, s));
    const int64_t slots = nb * max_chunks;
    ws.part_d.reserve(sizeof(float) * (size_t)slots * per_slot);
    ws.part_i.reserve(sizeof(int64_t) * (size_t)slots * (dump ? 2 : per_slot));
    ws.counter.reserve(16);
    HIPCHK(hipMemsetAsync(ws.counter.p, 0, sizeof(int), s));
    PqTileArgs a{};
    a.lut16 = lut16 ? 1 : 0;
    a.queries = d_q + b0 * (int64_t)idx->d;
    a.cents = idx->centroids_rm.as<float>();
    a.books = idx->pq_books.as<float>();
    a.book_norms = idx->pq_book_norms.as<float>();
    a.books_mfma = idx->pq_books_mfma.as<float>();
    a.codes = static_cast<const uint8_t*>(idx->pq_codes.p);
    a.row_ids = L.ids.as<int64_t>();
    a.list_off = L.off.as<int64_t>();
    a.list_goff = L.goff.as<int64_t>();
    a.n_lists = L.n_lists;
    a.bucket_q = ws.bucket_q.as<int64_t>();
    a.bucket_slot = ws.bucket_slot.as<int64_t>();
    a.bucket_off = ws.bucket_off.as<int>();
    a.work_off = ws.work_off.as<int>();
    a.work_counter = ws.counter.as<int>();
    a.d = idx->d;
    a.rot_dim_pad = idx->rot_dim_pad;
    a.pq_dim = idx->pq_dim;
    a.pq_dim_pad = idx->pq_dim_pad;
    a.pq_len = idx->pq_len;
    a.k = k;
    a.out_d = ws.part_d.as<float>();
    a.out_i = dump ? nullptr : ws.part_i.as<int64_t>();
    a.slot_info = dump ? ws.part_i.as<int64_t>() : nullptr;
    a.ip = idx->metric == MIVS_METRIC_IP ? 1 : 0;
    a.probes = probes;
    a.probes_d = ws.probes_d.as<float>() + b0 * np;
    a.n_probes = np;
    a.flags = flags;
    a.slot_cap = cands ? kRtSlotCap : 0;
    HIPCHK(launch_pq_scan_rt(a, cu_count(idx->device), s));
    if (cands) {  // K8 over each query's slots of candidates (EXPLICIT, slot ranges)
      SelectArgs sa{};
      sa.keys = ws.part_d.as<float>();
      sa.ids = ws.part_i.as<int64_t>();
      sa.slot_begin = ws.slot_begin.as<int64_t>();
      sa.n_in = kRtSlotCap;
      sa.nq = nb;
      sa.k = k;
      sa.metric = idx->metric;
      sa.out_d = d_dist + b0 * k;
      sa.out_i = d_ids + b0 * k;
      HIPCHK(launch_select(sa, s));
    } else if (dump) {
      SelectArgs sa{};
      sa.keys = ws.part_d.as<float>();
      sa.row_ids = L.ids.as<int64_t>();
      sa.slot_info = ws.part_i.as<int64_t>();
      sa.slot_begin = ws.slot_begin.as<int64_t>();
      sa.slot_rows = kRtRows;
      sa.nq = nb;
      sa.k = k;
      sa.metric = idx->metric;
      sa.out_d = d_dist + b0 * k;
      sa.out_i = d_ids + b0 * k;
      HIPCHK(launch_select(sa, s));
    } else {
      MergeArgs m{};
      m.in_d = ws.part_d.as<float>();
      m.in_i = ws.part_i.as<int64_t>();
      m.slot_begin = ws.slot_begin.as<int64_t>();
      m.nq = nb;
      m.k_in = k;
      m.k = k;
      m.metric = idx->metric;
      m.out_d = d_dist + b0 * k;
      m.out_i = d_ids + b0 * k;
      HIPCHK(launch_merge(m, s));
    }
  }
  if (pr) HIPCHK(hipEventRecord(pr->e[2], s));
}

void ivf_search_impl(mivs_index_s* idx, hipStream_t s, const float* q, int64_t nq, int k, int np, float* out_d,
                     int64_t* out_i, int32_t* out_probes) {
  int64_t qb = nq;
  if (lk_use(idx, k, np)) {  // K16: the record streams and windows bound the batch
    qb = std::min<int64_t>(std::min<int64_t>(nq, kRsMaxBatch), lk_batch(idx, nq, k, np));
  } else if (k > kMaxK) {  // DUMP workspace: bound it by batching queries
    const ListSet& L = idx->lists;
    const int64_t per_q_slots = std::max<int64_t>(1, L.top_chunks_prefix[std::min<int64_t>(np, L.n_lists)]);
    qb = select_batch(nq, (size_t)per_q_slots * ((size_t)idx->G * kGroupRows * 4 + 16));
  } else if (idx->groups_h.p != nullptr && k <= kPfMaxK && rs_use(idx, np)) {
    qb = std::min<int64_t>(nq, kRsMaxBatch);  // K13: bounded record streams and LDS-histogram bucketing
  }
  qb = ceil_div(nq, ceil_div(nq, std::max<int64_t>(qb, 1)));  // equal batches (a small last one rescans every list)
  int64_t nb = 0;
  for (int64_t b0 = 0; b0 < nq; b0 += qb) {
    nb = std::min<int64_t>(qb, nq - b0);
    idx->last_ovf = 0;  // (every stat describes the last batch, as n_queries does)
    idx->last_window = 0;
    idx->last_stats_dev = false;
    ivf_search_batch(idx, s, q + b0 * (int64_t)idx->d, nb, k, np, out_d + b0 * k, out_i + b0 * k,
                     out_probes ? out_probes + b0 * np : nullptr);
  }
  idx->last_nq = nb;  // (the stats describe the last batch)
  idx->last_np = np;
  idx->last_k = k;
}

}  // namespace

extern "C" {

const char* mivs_last_error(void) { return g_err.c_str(); }
int32_t mivs_version(void) { return 100; }
void mivs_set_profiling(int32_t on) { g_profiling.store(on ? 1 : 0); }

int32_t mivs_ivf_flat_build(int32_t device, void* stream, const float* d_data, int64_t n, int32_t dim,
                            const mivs_ivf_flat_params* p, int64_t id_offset, mivs_index_t* out) {
  return guarded([&] {
    require(p != nullptr && out != nullptr, "params/out is NULL");
    check_common(device, d_data, n, dim);
    require(p->metric == MIVS_METRIC_L2 || p->metric == MIVS_METRIC_IP, "unknown metric");
    require(p->n_lists >= 1, "n_lists must be >= 1");
    require(n >= p->n_lists, "n_rows (" + std::to_string(n) + ") must be >= n_lists (" + std::to_string(p->n_lists) + ")");
    require(p->n_lists <= 32768, "n_lists > 32768 is not supported by this build", MIVS_ERR_UNSUPPORTED);
    require(p->kmeans_n_iters >= 0, "kmeans_n_iters must be >= 0");
    require(p->kmeans_trainset_fraction > 0.0 && p->kmeans_trainset_fraction <= 1.0,
            "kmeans_trainset_fraction must be in (0, 1]");
    DeviceGuard dg(device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    auto idx = std::make_unique<mivs_index_s>();
    IndexCall ic(idx.get(), s);
    idx->kind = 0;
    idx->device = device;
    idx->d = dim;
    idx->dp = dim_pad(dim);
    idx->metric = p->metric;
    idx->G = chunk_groups_from_rows(p->chunk_rows);
    idx->id_offset = id_offset;
    const int nl = p->n_lists;
    // trainset + strided init (oracle orc_train_count / orc_train_rows / orc_init_rows)
    int64_t nt = (int64_t)((double)n * p->kmeans_trainset_fraction);
    if (p->kmeans_max_train_per_list > 0 && nt > (int64_t)nl * p->kmeans_max_train_per_list)
      nt = (int64_t)nl * p->kmeans_max_train_per_list;
    nt = std::max<int64_t>(nt, nl);
    nt = std::min<int64_t>(nt, n);
    Buf rows, init_rows, norms;
    rows.reserve(sizeof(int64_t) * nt);
    HIPCHK(launch_train_rows(rows.as<int64_t>(), n, nt, s));
    std::vector<int64_t> h_init(nl);
    for (int j = 0; j < nl; ++j) h_init[j] = ((((int64_t)j * nt) / nl) * n) / nt;
    init_rows.reserve(sizeof(int64_t) * nl);
    HIPCHK(hipMemcpyAsync(init_rows.p, h_init.data(), sizeof(int64_t) * nl, hipMemcpyHostToDevice, s));
    idx->centroids_rm.reserve(sizeof(float) * (size_t)nl * dim);
    HIPCHK(launch_gather_rows(d_data, dim, init_rows.as<int64_t>(), nl, idx->centroids_rm.as<float>(), s));
    norms.reserve(sizeof(float) * n);
    HIPCHK(launch_row_norms(d_data, n, dim, norms.as<float>(), s));
    HIPCHK(hipStreamSynchronize(s));
    // phase clock (profiling on): prepare | coarse k-means | assign + pack | fp16 copy
    const bool clk = g_profiling.load();
    auto t_ph = std::chrono::steady_clock::now();
    auto phase = [&]() {
      if (!clk) return;
      HIPCHK(hipStreamSynchronize(s));
      const auto t1 = std::chrono::steady_clock::now();
      idx->build_phase_s.push_back(std::chrono::duration<double>(t1 - t_ph).count());
      t_ph = t1;
    };
    // (profiling: the hot kernels' hipEvents, collected after the last phase)
    std::unique_ptr<BuildProf> bprof(clk ? new BuildProf() : nullptr);
    struct ProfScope {
      ProfScope(BuildProf* p) { g_bprof = p; }
      ~ProfScope() { g_bprof = nullptr; }
    } prof_scope(bprof.get());
    PfAssign pfa;  // the data's fp16 copy: k-means assign + list fill through the pre-filter
    pf_assign_prepare(pfa, d_data, n, dim, idx->dp, s);
    phase();
    kmeans_fit_impl(d_data, norms.as<float>(), rows.as<int64_t>(), nt, dim, idx->dp, nl, p->kmeans_n_iters,
                    idx->centroids_rm.as<float>(), idx->G, device, idx->ws, s, p->kmeans_balance != 0, &pfa);
    make_single_list(idx->cents, idx->centroids_rm.as<float>(), nl, dim, idx->dp, 0, idx->G, s);
    phase();
    if (bprof) bprof->assign_kind = MIVS_BUILD_FINAL_ASSIGN;
    if (p->add_data_on_build) {
      build_lists(idx.get(), d_data, norms.as<float>(), n, s, &pfa);
    } else {
      build_lists(idx.get(), d_data, norms.as<float>(), 0, s);
    }
    phase();
    if (p->prefilter && pf_default_on()) pf_enable(idx.get(), s);
    phase();
    HIPCHK(hipStreamSynchronize(s));
    if (bprof) bprof->collect(idx->build_kern);
    *out = idx.release();
  });
}

int32_t mivs_ivf_flat_build_from_centroids(int32_t device, void* stream, const float* d_data, int64_t n,
                                           int32_t dim, const float* d_centroids, int32_t n_lists,
                                           int32_t metric, int64_t id_offset, int32_t chunk_rows,
                                           mivs_index_t* out) {
  return guarded([&] {
    require(out != nullptr && d_centroids != nullptr, "centroids/out is NULL");
    check_common(device, d_data, n, dim);
    require(metric == MIVS_METRIC_L2 || metric == MIVS_METRIC_IP, "unknown metric");
    require(n_lists >= 1 && n_lists <= 32768, "n_lists must be in [1, 32768]");
    DeviceGuard dg(device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    auto idx = std::make_unique<mivs_index_s>();
    IndexCall ic(idx.get(), s);
    idx->kind = 0;
    idx->device = device;
    idx->d = dim;
    idx->dp = dim_pad(dim);
    idx->metric = metric;
    idx->G = chunk_groups_from_rows(chunk_rows);
    idx->id_offset = id_offset;
    idx->centroids_rm.reserve(sizeof(float) * (size_t)n_lists * dim);
    HIPCHK(hipMemcpyAsync(idx->centroids_rm.p, d_centroids, sizeof(float) * (size_t)n_lists * dim,
                          hipMemcpyDeviceToDevice, s));
    make_single_list(idx->cents, idx->centroids_rm.as<float>(), n_lists, dim, idx->dp, 0, idx->G, s);
    Buf norms;
    norms.reserve(sizeof(float) * std::max<int64_t>(n, 1));
    HIPCHK(launch_row_norms(d_data, n, dim, norms.as<float>(), s));
    build_lists(idx.get(), d_data, norms.as<float>(), n, s);
    if (pf_default_on()) pf_enable(idx.get(), s);
    HIPCHK(hipStreamSynchronize(s));
    *out = idx.release();
  });
}

int32_t mivs_ivf_flat_build_from_lists(int32_t device, void* stream, const float* d_rows, const int64_t* d_ids,
                                       const int64_t* h_list_sizes, int64_t n, int32_t dim, const float* d_centroids,
                                       int32_t n_lists, int32_t metric, int32_t chunk_rows, int32_t prefilter,
                                       mivs_index_t* out) {
  return guarded([&] {
    require(out != nullptr && d_centroids != nullptr && h_list_sizes != nullptr, "centroids/sizes/out is NULL");
    check_common(device, d_rows, n, dim);
    require(n == 0 || d_ids != nullptr, "ids is NULL");
    require(metric == MIVS_METRIC_L2 || metric == MIVS_METRIC_IP, "unknown metric");
    require(n_lists >= 1 && n_lists <= 32768, "n_lists must be in [1, 32768]");
    std::vector<int64_t> h_off(n_lists + 1, 0);
    for (int l = 0; l < n_lists; ++l) {
      require(h_list_sizes[l] >= 0, "negative list size");
      h_off[l + 1] = h_off[l] + h_list_sizes[l];
    }
    require(h_off[n_lists] == n, "list sizes do not add up to n");
    DeviceGuard dg(device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    auto idx = std::make_unique<mivs_index_s>();
    IndexCall ic(idx.get(), s);
    idx->kind = 0;
    idx->device = device;
    idx->d = dim;
    idx->dp = dim_pad(dim);
    idx->metric = metric;
    idx->G = chunk_groups_from_rows(chunk_rows);
    idx->centroids_rm.reserve(sizeof(float) * (size_t)n_lists * dim);
    HIPCHK(hipMemcpyAsync(idx->centroids_rm.p, d_centroids, sizeof(float) * (size_t)n_lists * dim,
                          hipMemcpyDeviceToDevice, s));
    make_single_list(idx->cents, idx->centroids_rm.as<float>(), n_lists, dim, idx->dp, 0, idx->G, s);
    pack_lists(idx->lists, d_rows, dim, idx->dp, nullptr, h_off, 0, d_ids, idx->G, s);
    if (prefilter && pf_default_on()) pf_enable(idx.get(), s);
    HIPCHK(hipStreamSynchronize(s));
    *out = idx.release();
  });
}

int32_t mivs_ivf_flat_extend(mivs_index_t idx, void* stream, const float* d_new, const int64_t* d_new_ids,
                             int64_t n_new) {
  return guarded([&] {
    require(idx != nullptr && idx->kind == 0, "not an ivf_flat index");
    require(n_new >= 0, "n_new must be >= 0");
    require(n_new == 0 || d_new != nullptr, "new vectors are NULL");
    if (n_new == 0) return;
    std::lock_guard<std::mutex> g(idx->mu);
    DeviceGuard dg(idx->device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    IndexCall ic(idx, s);
    ListSet& L = idx->lists;
    const int d = idx->d;
    const int nl = idx->cents.n_lists == 1 ? (int)idx->cents.n_rows : idx->cents.n_lists;
    const int64_t n_old = L.n_rows, n_all = n_old + n_new;
    // every row in list order (old rows first, so each list keeps its current order), ids beside them
    Buf rows, ids, labels, norms, perm, off, ctmp;
    rows.reserve(sizeof(float) * (size_t)n_all * d);
    ids.reserve(sizeof(int64_t) * (size_t)n_all);
    labels.reserve(sizeof(int64_t) * (size_t)n_all);
    if (n_old > 0) {
      HIPCHK(launch_unpack_rows(L.groups.as<float>(), idx->dp, d, L.off.as<int64_t>(), L.goff.as<int64_t>(), L.n_lists,
                                n_old, rows.as<float>(), s));
      HIPCHK(launch_compact_ids(L.ids.as<int64_t>(), L.off.as<int64_t>(), L.goff.as<int64_t>(), L.n_lists, n_old,
                                ids.as<int64_t>(), s));
      std::vector<int64_t> h_lab(n_old);
      for (int l = 0; l < L.n_lists; ++l)
        for (int64_t r = L.h_off[l]; r < L.h_off[l + 1]; ++r) h_lab[r] = l;
      HIPCHK(hipMemcpyAsync(labels.p, h_lab.data(), sizeof(int64_t) * n_old, hipMemcpyHostToDevice, s));
      HIPCHK(hipStreamSynchronize(s));
    }
    float* new_rows = rows.as<float>() + n_old * d;
    HIPCHK(hipMemcpyAsync(new_rows, d_new, sizeof(float) * (size_t)n_new * d, hipMemcpyDeviceToDevice, s));
    if (d_new_ids) HIPCHK(hipMemcpyAsync(ids.as<int64_t>() + n_old, d_new_ids, sizeof(int64_t) * n_new,
                                         hipMemcpyDeviceToDevice, s));
    // default ids continue the index's own global range: a shard built with ids_offset = start_index
    // keeps its new rows inside that range instead of colliding with shard 0's ids
    else HIPCHK(launch_iota_i64(ids.as<int64_t>() + n_old, n_new, idx->id_offset + n_old, 1, s));
    norms.reserve(sizeof(float) * (size_t)n_new);
    HIPCHK(launch_row_norms(new_rows, n_new, d, norms.as<float>(), s));
    assign_rows(new_rows, norms.as<float>(), nullptr, n_new, d, idx->dp, idx->cents, idx->G, idx->metric,
                labels.as<int64_t>() + n_old, idx->device, idx->ws, s);
    // stable counting sort by list, then re-pack every list
    perm.reserve(sizeof(int64_t) * (size_t)n_all);
    off.reserve(sizeof(int64_t) * (nl + 1));
    const size_t cb = csort_tmp_bytes(n_all, nl);
    ctmp.reserve(cb);
    HIPCHK(launch_counting_sort(labels.as<int64_t>(), n_all, nl, perm.as<int64_t>(), off.as<int64_t>(), ctmp.p, cb, s));
    std::vector<int64_t> h_off(nl + 1);
    HIPCHK(hipMemcpyAsync(h_off.data(), off.p, sizeof(int64_t) * (nl + 1), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    const bool had_pf = idx->groups_h.p != nullptr;
    idx->groups_h.release();
    idx->groups_f8.release();  // (copies of the old lists; pf_enable would drop them too)
    pack_lists(L, rows.as<float>(), d, idx->dp, perm.as<int64_t>(), h_off, 0, ids.as<int64_t>(), idx->G, s);
    if (had_pf) pf_enable(idx, s);
    HIPCHK(hipStreamSynchronize(s));
  });
}

int32_t mivs_ivf_flat_search(mivs_index_t idx, void* stream, const float* d_q, int64_t nq, int32_t k,
                             int32_t n_probes, float* d_dist, int64_t* d_ids, int32_t* d_probes) {
  return guarded([&] {
    require(idx != nullptr && idx->kind == 0, "not an ivf_flat index");
    require(nq >= 0, "nq must be >= 0");
    require(k >= 1 && k <= kMaxSelectK, "k must be in [1, " + std::to_string(kMaxSelectK) + "]",
            MIVS_ERR_UNSUPPORTED);
    require(n_probes >= 1, "n_probes must be >= 1");
    require(nq == 0 || (d_q && d_dist && d_ids), "NULL query/output pointer");
    if (nq == 0) return;
    std::lock_guard<std::mutex> g(idx->mu);
    DeviceGuard dg(idx->device);
    const int np = std::min<int>(n_probes, idx->lists.n_lists);
    require(np <= kMaxSelectK, "n_probes must be <= " + std::to_string(kMaxSelectK), MIVS_ERR_UNSUPPORTED);
    require(np == n_probes || d_probes == nullptr, "n_probes > n_lists with a probes output");
    HostTrace& ht = host_trace();
    static const bool trace = env_int("MIVS_HOST_TRACE", 0) == 1;
    ht.on = trace;
    if (trace) {
      ht.n_wait = 0;
      ht.t0 = std::chrono::steady_clock::now();
    }
    IndexCall ic(idx, static_cast<hipStream_t>(stream));
    ivf_search_impl(idx, static_cast<hipStream_t>(stream), d_q, nq, k, np, d_dist, d_ids, d_probes);
    if (trace) {
      const auto t1 = std::chrono::steady_clock::now();
      auto us = [](auto a, auto b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
      fprintf(stderr, "[host] entry->first launch %.1f us, ->wait %.1f us, wait %.1f us (%d), wait->exit %.1f us\n",
              us(ht.t0, ht.t_first), us(ht.t_first, ht.t_wait0), us(ht.t_wait0, ht.t_wait1), ht.n_wait,
              us(ht.t_wait1, t1));
    }
  });
}

int32_t mivs_ivf_flat_get_centroids(mivs_index_t idx, void* stream, float* d_out) {
  return guarded([&] {
    require(idx != nullptr && (idx->kind == 0 || idx->kind == 2), "not an IVF index");
    DeviceGuard dg(idx->device);
    IndexCall ic(idx, static_cast<hipStream_t>(stream));
    HIPCHK(hipMemcpyAsync(d_out, idx->centroids_rm.p, sizeof(float) * (size_t)idx->lists.n_lists * idx->d,
                          hipMemcpyDeviceToDevice, static_cast<hipStream_t>(stream)));
  });
}

int32_t mivs_ivf_flat_get_list_sizes(mivs_index_t idx, int64_t* h_out) {
  return guarded([&] {
    require(idx != nullptr, "index is NULL");
    for (int l = 0; l < idx->lists.n_lists; ++l) h_out[l] = idx->lists.h_off[l + 1] - idx->lists.h_off[l];
  });
}

int32_t mivs_ivf_flat_get_list_ids(mivs_index_t idx, void* stream, int64_t* d_out) {
  return guarded([&] {
    require(idx != nullptr, "index is NULL");
    DeviceGuard dg(idx->device);
    IndexCall ic(idx, static_cast<hipStream_t>(stream));
    const ListSet& L = idx->lists;
    HIPCHK(launch_compact_ids(L.ids.as<int64_t>(), L.off.as<int64_t>(), L.goff.as<int64_t>(), L.n_lists, L.n_rows,
                              d_out, static_cast<hipStream_t>(stream)));
  });
}

int32_t mivs_ivf_flat_get_list_rows(mivs_index_t idx, void* stream, float* d_out) {
  return guarded([&] {
    require(idx != nullptr, "index is NULL");
    DeviceGuard dg(idx->device);
    IndexCall ic(idx, static_cast<hipStream_t>(stream));
    const ListSet& L = idx->lists;
    HIPCHK(launch_unpack_rows(L.groups.as<float>(), idx->dp, idx->d, L.off.as<int64_t>(), L.goff.as<int64_t>(),
                              L.n_lists, L.n_rows, d_out, static_cast<hipStream_t>(stream)));
  });
}

int32_t mivs_ivf_pq_build(int32_t device, void* stream, const float* d_data, int64_t n, int32_t dim,
                          const mivs_ivf_pq_params* p, int64_t id_offset, mivs_index_t* out) {
  return guarded([&] {
    require(p != nullptr && out != nullptr, "params/out is NULL");
    check_common(device, d_data, n, dim);
    require(p->metric == MIVS_METRIC_L2 || p->metric == MIVS_METRIC_IP, "unknown metric");
    require(p->pq_bits == 8, "ivf_pq: pq_bits must be 8 in this build", MIVS_ERR_UNSUPPORTED);
    require(p->pq_dim >= 1 && p->pq_dim <= dim, "pq_dim must be in [1, dim]");
    require(p->n_lists >= 1 && p->n_lists <= 32768, "n_lists must be in [1, 32768]");
    require(n >= p->n_lists, "n_rows must be >= n_lists");
    require(p->kmeans_n_iters >= 0, "kmeans_n_iters must be >= 0");
    require(p->kmeans_trainset_fraction > 0.0 && p->kmeans_trainset_fraction <= 1.0,
            "kmeans_trainset_fraction must be in (0, 1]");
    require(p->max_train_points_per_pq_code >= 1, "max_train_points_per_pq_code must be >= 1");
    const int pl = (dim + p->pq_dim - 1) / p->pq_dim;
    require(pl <= 64, "pq_len = ceil(dim / pq_dim) must be <= 64", MIVS_ERR_UNSUPPORTED);
    const int64_t n_pq = std::min<int64_t>(n, p->max_train_points_per_pq_code << p->pq_bits);
    require(n_pq >= (1 << p->pq_bits), "ivf_pq: need at least 2^pq_bits rows to train the codebooks");
    DeviceGuard dg(device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    auto idx = std::make_unique<mivs_index_s>();
    IndexCall ic(idx.get(), s);
    idx->kind = 2;
    idx->device = device;
    idx->d = dim;
    idx->dp = dim_pad(dim);
    // (the coarse lists and the codebooks are trained in L2 for both metrics, as for ivf_flat; the
    // metric is the search's ranking)
    idx->metric = p->metric;
    idx->id_offset = id_offset;
    idx->pq_dim = p->pq_dim;
    idx->pq_bits = p->pq_bits;
    idx->pq_len = pl;
    idx->pq_dim_pad = (p->pq_dim + 15) / 16 * 16;
    idx->rot_dim_pad = (p->pq_dim * pl + 3) / 4 * 4;
    const int nl = p->n_lists;
    const int nc = 1 << p->pq_bits;
    // phase clock (profiling on): prepare | coarse k-means | assign + sort | codebooks | encode
    const bool clk = g_profiling.load();
    auto tnow = [] { return std::chrono::steady_clock::now(); };
    auto t_ph = tnow();
    auto phase = [&]() {
      if (!clk) return;
      HIPCHK(hipStreamSynchronize(s));
      const auto t1 = tnow();
      idx->build_phase_s.push_back(std::chrono::duration<double>(t1 - t_ph).count());
      t_ph = t1;
    };
    // ---- coarse k-means (as ivf_flat: trainset, strided init) ----
    int64_t nt = (int64_t)((double)n * p->kmeans_trainset_fraction);
    nt = std::min<int64_t>(std::max<int64_t>(nt, nl), n);
    Buf rows, init_rows, norms, labels, perm, off, ctmp;
    rows.reserve(sizeof(int64_t) * nt);
    HIPCHK(launch_train_rows(rows.as<int64_t>(), n, nt, s));
    std::vector<int64_t> h_init(nl);
    for (int j = 0; j < nl; ++j) h_init[j] = ((((int64_t)j * nt) / nl) * n) / nt;
    init_rows.reserve(sizeof(int64_t) * std::max(nl, nc));
    HIPCHK(hipMemcpyAsync(init_rows.p, h_init.data(), sizeof(int64_t) * nl, hipMemcpyHostToDevice, s));
    idx->centroids_rm.reserve(sizeof(float) * (size_t)nl * dim);
    HIPCHK(launch_gather_rows(d_data, dim, init_rows.as<int64_t>(), nl, idx->centroids_rm.as<float>(), s));
    norms.reserve(sizeof(float) * n);
    HIPCHK(launch_row_norms(d_data, n, dim, norms.as<float>(), s));
    HIPCHK(hipStreamSynchronize(s));
    {
      PfAssign pfa;  // coarse k-means + list assign through the fp16 pre-filter
      pf_assign_prepare(pfa, d_data, n, dim, idx->dp, s);
      phase();
      kmeans_fit_impl(d_data, norms.as<float>(), rows.as<int64_t>(), nt, dim, idx->dp, nl, p->kmeans_n_iters,
                      idx->centroids_rm.as<float>(), idx->G, device, idx->ws, s, p->kmeans_balance != 0, &pfa);
      make_single_list(idx->cents, idx->centroids_rm.as<float>(), nl, dim, idx->dp, 0, idx->G, s);
      phase();
      // ---- lists: L2 assignment of every row, stable order by label ----
      labels.reserve(sizeof(int64_t) * n);
      perm.reserve(sizeof(int64_t) * n);
      off.reserve(sizeof(int64_t) * (nl + 1));
      assign_rows(d_data, norms.as<float>(), nullptr, n, dim, idx->dp, idx->cents, idx->G, kL2,
                  labels.as<int64_t>(), device, idx->ws, s, &pfa);
    }
    const size_t cb = csort_tmp_bytes(n, nl);
    ctmp.reserve(cb);
    HIPCHK(launch_counting_sort(labels.as<int64_t>(), n, nl, perm.as<int64_t>(), off.as<int64_t>(), ctmp.p, cb, s));
    ListSet& L = idx->lists;
    L.n_lists = nl;
    L.n_rows = n;
    L.h_off.assign(nl + 1, 0);
    HIPCHK(hipMemcpyAsync(L.h_off.data(), off.p, sizeof(int64_t) * (nl + 1), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    L.h_goff.assign(nl + 1, 0);
    for (int l = 0; l < nl; ++l) L.h_goff[l + 1] = L.h_goff[l] + ceil_div(L.h_off[l + 1] - L.h_off[l], kGroupRows);
    L.n_groups = L.h_goff.back();
    L.off.reserve(sizeof(int64_t) * (nl + 1));
    L.goff.reserve(sizeof(int64_t) * (nl + 1));
    HIPCHK(hipMemcpyAsync(L.off.p, L.h_off.data(), sizeof(int64_t) * (nl + 1), hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(L.goff.p, L.h_goff.data(), sizeof(int64_t) * (nl + 1), hipMemcpyHostToDevice, s));
    L.finalize_host(idx->G);
    phase();
    // ---- codebooks: per subspace k-means on residual sub-vectors of a strided trainset ----
    Buf prow, resid, rnorm;
    prow.reserve(sizeof(int64_t) * n_pq);
    HIPCHK(launch_train_rows(prow.as<int64_t>(), n, n_pq, s));
    resid.reserve(sizeof(float) * (size_t)p->pq_dim * n_pq * pl);
    HIPCHK(launch_pq_residuals(d_data, dim, prow.as<int64_t>(), n_pq, labels.as<int64_t>(),
                               idx->centroids_rm.as<float>(), p->pq_dim, pl, resid.as<float>(), s));
    std::vector<int64_t> h_cinit(nc);
    for (int c = 0; c < nc; ++c) h_cinit[c] = ((int64_t)c * n_pq) / nc;
    HIPCHK(hipMemcpyAsync(init_rows.p, h_cinit.data(), sizeof(int64_t) * nc, hipMemcpyHostToDevice, s));
    idx->pq_books.reserve(sizeof(float) * (size_t)p->pq_dim * nc * pl);
    rnorm.reserve(sizeof(float) * n_pq);
    for (int j = 0; j < p->pq_dim; ++j) {
      const float* rj = resid.as<float>() + (size_t)j * n_pq * pl;
      float* bj = idx->pq_books.as<float>() + (size_t)j * nc * pl;
      HIPCHK(launch_gather_rows(rj, pl, init_rows.as<int64_t>(), nc, bj, s));
      HIPCHK(launch_row_norms(rj, n_pq, pl, rnorm.as<float>(), s));
      kmeans_fit_impl(rj, rnorm.as<float>(), nullptr, n_pq, pl, dim_pad(pl), nc, p->kmeans_n_iters, bj, idx->G,
                      device, idx->ws, s, p->kmeans_balance != 0);
    }
    // the codes' norms (the L2 LUT's start) and K9r's MFMA operand copy of the codebooks
    idx->pq_book_norms.reserve(sizeof(float) * (size_t)p->pq_dim * nc);
    idx->pq_books_mfma.reserve(sizeof(float) * (size_t)p->pq_dim * nc * pl);
    HIPCHK(launch_pq_book_prep(idx->pq_books.as<float>(), p->pq_dim, pl, idx->metric == MIVS_METRIC_IP ? 1 : 0,
                               idx->pq_book_norms.as<float>(), idx->pq_books_mfma.as<float>(), s));
    phase();
    // ---- encode + ids into the interleaved layout ----
    const int64_t slots = std::max<int64_t>(L.n_groups, 1) * kGroupRows;
    idx->pq_codes.reserve((size_t)slots * idx->pq_dim_pad);
    HIPCHK(hipMemsetAsync(idx->pq_codes.p, 0, (size_t)slots * idx->pq_dim_pad, s));
    L.ids.reserve(sizeof(int64_t) * slots);
    HIPCHK(hipMemsetAsync(L.ids.p, 0xFF, sizeof(int64_t) * slots, s));
    if (p->add_data_on_build) {
      HIPCHK(launch_pq_encode(d_data, dim, perm.as<int64_t>(), n, L.off.as<int64_t>(), L.goff.as<int64_t>(), nl,
                              idx->centroids_rm.as<float>(), idx->pq_books.as<float>(), p->pq_dim, pl,
                              idx->pq_dim_pad, static_cast<uint8_t*>(idx->pq_codes.p), s));
      HIPCHK(launch_pq_ids(perm.as<int64_t>(), n, L.off.as<int64_t>(), L.goff.as<int64_t>(), nl, id_offset,
                           L.ids.as<int64_t>(), s));
      phase();
    } else {
      L.n_rows = 0;
      std::fill(L.h_off.begin(), L.h_off.end(), 0);
      std::fill(L.h_goff.begin(), L.h_goff.end(), 0);
      L.n_groups = 0;
      HIPCHK(hipMemcpyAsync(L.off.p, L.h_off.data(), sizeof(int64_t) * (nl + 1), hipMemcpyHostToDevice, s));
      HIPCHK(hipMemcpyAsync(L.goff.p, L.h_goff.data(), sizeof(int64_t) * (nl + 1), hipMemcpyHostToDevice, s));
      L.finalize_host(idx->G);
    }
    HIPCHK(hipStreamSynchronize(s));
    *out = idx.release();
  });
}

int32_t mivs_ivf_pq_search(mivs_index_t idx, void* stream, const float* d_q, int64_t nq, int32_t k,
                           int32_t n_probes, float* d_dist, int64_t* d_ids, int32_t* d_probes) {
  return mivs_ivf_pq_search_ex(idx, stream, d_q, nq, k, n_probes, MIVS_LUT_FP32, d_dist, d_ids, d_probes);
}

int32_t mivs_ivf_pq_search_ex(mivs_index_t idx, void* stream, const float* d_q, int64_t nq, int32_t k,
                              int32_t n_probes, int32_t lut_dtype, float* d_dist, int64_t* d_ids, int32_t* d_probes) {
  return guarded([&] {
    require(idx != nullptr && idx->kind == 2, "not an ivf_pq index");
    require(lut_dtype == MIVS_LUT_FP32 || lut_dtype == MIVS_LUT_FP16, "lut_dtype must be MIVS_LUT_FP32 or MIVS_LUT_FP16");
    const bool lut16 = lut_dtype == MIVS_LUT_FP16;
    require(!lut16 || (idx->metric == kL2 && pq_rt_use(idx, k)),
            "ivf_pq: the fp16 LUT is served by the K9r scan, for the L2 metric with pq_len % 4 == 0 (4..16)",
            MIVS_ERR_UNSUPPORTED);
    require(nq >= 0, "nq must be >= 0");
    require(k >= 1 && k <= kMaxSelectK, "ivf_pq: k must be in [1, " + std::to_string(kMaxSelectK) + "]",
            MIVS_ERR_UNSUPPORTED);
    require(n_probes >= 1, "n_probes must be >= 1");
    require(nq == 0 || (d_q && d_dist && d_ids), "NULL query/output pointer");
    if (nq == 0) return;
    std::lock_guard<std::mutex> g(idx->mu);
    DeviceGuard dg(idx->device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    IndexCall ic(idx, s);
    const int np = std::min<int>(n_probes, idx->lists.n_lists);
    require(np <= kMaxSelectK, "n_probes must be <= " + std::to_string(kMaxSelectK), MIVS_ERR_UNSUPPORTED);
    require(np == n_probes || d_probes == nullptr, "n_probes > n_lists with a probes output");
    const int kcap = scan_kcap(k);  // (0: k > 64, the DUMP scan + K8)
    require(k > kMaxK || pq_tile_lds_bytes(idx->rot_dim_pad, idx->pq_len) <= 160 * 1024 ||
                pq_scan_lds_bytes(idx->rot_dim_pad, idx->pq_dim, kcap) <= 160 * 1024 ||
                pq_split_lds_bytes(idx->rot_dim_pad, (int)ceil_div(ceil_div(idx->pq_dim, 2), 16) * 16, kcap) <=
                    160 * 1024,
            "ivf_pq: the LUT scan does not fit the 160 KB LDS for this pq_dim / pq_len", MIVS_ERR_UNSUPPORTED);
    Workspace& ws = idx->ws;
    ProfRec* pr = g_profiling.load() ? idx->prof.begin(s) : nullptr;
    ws.qn.reserve(sizeof(float) * nq);
    HIPCHK(launch_row_norms(d_q, nq, idx->d, ws.qn.as<float>(), s));
    ws.probes_d.reserve(sizeof(float) * nq * np);
    ws.probes_i.reserve(sizeof(int64_t) * nq * np);
    single_list_topk(idx->cents, coarse_groups(idx, nq, np), d_q, ws.qn.as<float>(), nullptr, nq, idx->d, idx->dp, np,
                     idx->metric, ws.probes_d.as<float>(), ws.probes_i.as<int64_t>(), idx->device, ws, s,
                     coarse_dump(np));
    if (d_probes) HIPCHK(launch_i64_to_i32(ws.probes_i.as<int64_t>(), nq * np, d_probes, s));
    const ListSet& L = idx->lists;
    // k > 16 (the candidate pools of IVF-PQ + refine): K9 in DUMP mode writes every probed row's key and
    // K8 selects per query, in query batches bounded by the select workspace -- measured 3x faster than
    // the 32/64-entry register lists at 40 candidates (profiles/r02_ivf_pq_refine_bench.log);
    // MIVS_PQ_DUMP_K raises the threshold (up to 64) for the register path
    if (pq_rt_use(idx, k)) {
      pq_search_rt(idx, s, d_q, nq, k, np, d_dist, d_ids, pr, lut16);
      if (pr) HIPCHK(hipEventRecord(pr->e[3], s));
      idx->last_nq = nq;
      idx->last_np = np;
      idx->last_k = k;
      return;
    }
    const char* dke = getenv("MIVS_PQ_DUMP_K");
    const int dump_k = std::min(kMaxK, std::max(16, dke ? atoi(dke) : 16));
    if (k > dump_k) {
      require(pq_scan_lds_bytes(idx->rot_dim_pad, idx->pq_dim, 0) <= 160 * 1024,
              "ivf_pq: k > 64 needs the whole LUT in LDS, which does not fit this pq_dim", MIVS_ERR_UNSUPPORTED);
      int64_t slot_rows = 1;
      for (int l = 0; l < L.n_lists; ++l) slot_rows = std::max<int64_t>(slot_rows, L.h_off[l + 1] - L.h_off[l]);
      require(slot_rows < INT32_MAX, "ivf_pq: list too long for the DUMP scan", MIVS_ERR_UNSUPPORTED);
      const int64_t qb = select_batch(nq, (size_t)np * ((size_t)slot_rows * 4 + 16));
      ws.part_d.reserve(sizeof(float) * (size_t)(qb * np * slot_rows));
      ws.part_i.reserve(sizeof(int64_t) * (size_t)(qb * np * 2));
      if (pr) HIPCHK(hipEventRecord(pr->e[1], s));
      for (int64_t b0 = 0; b0 < nq; b0 += qb) {
        const int64_t nb = std::min<int64_t>(qb, nq - b0);
        PqScanArgs a{};
        a.queries = d_q + b0 * (int64_t)idx->d;
        a.cents = idx->centroids_rm.as<float>();
        a.books = idx->pq_books.as<float>();
        a.book_norms = idx->pq_book_norms.as<float>();
        a.codes = static_cast<const uint8_t*>(idx->pq_codes.p);
        a.row_ids = L.ids.as<int64_t>();
        a.list_off = L.off.as<int64_t>();
        a.list_goff = L.goff.as<int64_t>();
        a.probes = ws.probes_i.as<int64_t>() + b0 * np;
        a.probes_d = ws.probes_d.as<float>() + b0 * np;
        a.n_slots = nb * np;
        a.n_probes = np;
        a.d = idx->d;
        a.rot_dim_pad = idx->rot_dim_pad;
        a.pq_dim = idx->pq_dim;
        a.pq_dim_pad = idx->pq_dim_pad;
        a.pq_len = idx->pq_len;
        a.k = k;
        a.ip = idx->metric == MIVS_METRIC_IP ? 1 : 0;
        a.out_d = ws.part_d.as<float>();
        a.dump_rows = (int)slot_rows;
        a.slot_info = ws.part_i.as<int64_t>();
        HIPCHK(launch_pq_scan(a, 0, s));
        SelectArgs sa{};
        sa.keys = ws.part_d.as<float>();
        sa.row_ids = L.ids.as<int64_t>();
        sa.slot_info = ws.part_i.as<int64_t>();
        sa.slot_begin = nullptr;
        sa.slots_per_q = np;
        sa.slot_rows = (int)slot_rows;
        sa.nq = nb;
        sa.k = k;
        sa.metric = idx->metric;
        sa.out_d = d_dist + b0 * k;
        sa.out_i = d_ids + b0 * k;
        HIPCHK(launch_select(sa, s));
      }
      if (pr) HIPCHK(hipEventRecord(pr->e[2], s));
      if (pr) HIPCHK(hipEventRecord(pr->e[3], s));
      idx->last_nq = nq;
      idx->last_np = np;
      idx->last_k = k;
      return;
    }
    const char* tiled_env = getenv("MIVS_PQ_TILED");
    // K9s (two LUT halves) applies when pq_len is a multiple of 4 up to 16 and each half has <= 64
    // subspaces; K9 needs the whole LUT plus its merge area in LDS; K9b otherwise
    const int pq_half = (int)ceil_div(ceil_div(idx->pq_dim, 2), 16) * 16;
    const bool split_ok = (idx->pq_len & 3) == 0 && idx->pq_len <= 16 && pq_half <= 64 &&
                          pq_split_lds_bytes(idx->rot_dim_pad, pq_half, kcap) <= 160 * 1024;
    const bool tiled = (tiled_env && tiled_env[0] == '1') ||
                       (!split_ok && pq_scan_lds_bytes(idx->rot_dim_pad, idx->pq_dim, kcap) > 160 * 1024);
    require(!tiled || kcap <= 32, "ivf_pq: k > 32 needs the whole-LUT scan (K9/K9s), which does not fit this "
            "pq_dim in LDS", MIVS_ERR_UNSUPPORTED);
    require(!tiled || idx->metric == MIVS_METRIC_L2, "ivf_pq: inner product needs the whole-LUT scan (K9/K9s), "
            "which does not fit this pq_dim in LDS", MIVS_ERR_UNSUPPORTED);
    if (tiled && pq_tile_lds_bytes(idx->rot_dim_pad, idx->pq_len) <= 160 * 1024) {
      // K9b (used when K9's whole-LUT LDS does not fit, or MIVS_PQ_TILED=1): probe map
      // (list -> 16-query tiles x 512-row chunks), tiled scan, K7 merge of the slots
      const int64_t ne = nq * np;
      ws.counts.reserve(sizeof(int) * L.n_lists);
      ws.fill.reserve(sizeof(int) * L.n_lists);
      ws.bucket_off.reserve(sizeof(int) * (L.n_lists + 1));
      ws.work_off.reserve(sizeof(int) * (L.n_lists + 1));
      ws.bucket_q.reserve(sizeof(int64_t) * ne);
      ws.bucket_slot.reserve(sizeof(int64_t) * ne);
      ws.qp_slots.reserve(sizeof(int64_t) * ne);
      ws.slot_begin.reserve(sizeof(int64_t) * (nq + 1));
      const size_t stb = scan_tmp_bytes(ne) + sizeof(int64_t) * (size_t)ne;
      ws.scan_tmp.reserve(stb);
      HIPCHK(launch_probe_map(ws.probes_i.as<int64_t>(), nq, np, L.n_lists, L.goff.as<int64_t>(), kPqChunkGroups,
                              kPqTileQueries, ws.counts.as<int>(), ws.fill.as<int>(), ws.bucket_off.as<int>(),
                              ws.work_off.as<int>(), ws.bucket_q.as<int64_t>(), ws.bucket_slot.as<int64_t>(),
                              ws.qp_slots.as<int64_t>(), ws.slot_begin.as<int64_t>(), ws.scan_tmp.p, stb, s));
      // slots: per (query, probe) one per 512-row chunk of the probed list
      int64_t max_chunks = 0;
      {
        std::vector<int64_t> c(L.n_lists);
        for (int l = 0; l < L.n_lists; ++l) c[l] = ceil_div(L.h_goff[l + 1] - L.h_goff[l], kPqChunkGroups);
        std::sort(c.begin(), c.end(), std::greater<int64_t>());
        for (int l = 0; l < std::min<int>(np, L.n_lists); ++l) max_chunks += c[l];
      }
      const int64_t max_slots = std::max<int64_t>(nq * max_chunks, 1);
      ws.part_d.reserve(sizeof(float) * (size_t)(max_slots * k));
      ws.part_i.reserve(sizeof(int64_t) * (size_t)(max_slots * k));
      ws.counter.reserve(16);
      HIPCHK(hipMemsetAsync(ws.counter.p, 0, sizeof(int), s));
      PqTileArgs a{};
      a.queries = d_q;
      a.cents = idx->centroids_rm.as<float>();
      a.books = idx->pq_books.as<float>();
      a.book_norms = idx->pq_book_norms.as<float>();
      a.codes = static_cast<const uint8_t*>(idx->pq_codes.p);
      a.row_ids = L.ids.as<int64_t>();
      a.list_off = L.off.as<int64_t>();
      a.list_goff = L.goff.as<int64_t>();
      a.n_lists = L.n_lists;
      a.bucket_q = ws.bucket_q.as<int64_t>();
      a.bucket_slot = ws.bucket_slot.as<int64_t>();
      a.bucket_off = ws.bucket_off.as<int>();
      a.work_off = ws.work_off.as<int>();
      a.work_counter = ws.counter.as<int>();
      a.d = idx->d;
      a.rot_dim_pad = idx->rot_dim_pad;
      a.pq_dim = idx->pq_dim;
      a.pq_dim_pad = idx->pq_dim_pad;
      a.pq_len = idx->pq_len;
      a.k = k;
      a.out_d = ws.part_d.as<float>();
      a.out_i = ws.part_i.as<int64_t>();
      const size_t lds = pq_tile_lds_bytes(idx->rot_dim_pad, idx->pq_len);
      const int per_cu = std::max<int>(1, std::min<int>(3, (int)((160 * 1024) / lds)));
      if (pr) HIPCHK(hipEventRecord(pr->e[1], s));
      HIPCHK(launch_pq_scan_tiled(a, kcap, cu_count(idx->device) * per_cu, s));
      if (pr) HIPCHK(hipEventRecord(pr->e[2], s));
      MergeArgs m{};
      m.in_d = ws.part_d.as<float>();
      m.in_i = ws.part_i.as<int64_t>();
      m.slot_begin = ws.slot_begin.as<int64_t>();
      m.nq = nq;
      m.k_in = k;
      m.k = k;
      m.metric = kL2;
      m.out_d = d_dist;
      m.out_i = d_ids;
      HIPCHK(launch_merge(m, s));
    } else {
      // K9: one workgroup per (query, probe) with the whole pq_dim x 256 LUT in LDS
      ws.part_d.reserve(sizeof(float) * (size_t)(nq * np * k));
      ws.part_i.reserve(sizeof(int64_t) * (size_t)(nq * np * k));
      PqScanArgs a{};
      a.queries = d_q;
      a.cents = idx->centroids_rm.as<float>();
      a.books = idx->pq_books.as<float>();
      a.book_norms = idx->pq_book_norms.as<float>();
      a.codes = static_cast<const uint8_t*>(idx->pq_codes.p);
      a.row_ids = L.ids.as<int64_t>();
      a.list_off = L.off.as<int64_t>();
      a.list_goff = L.goff.as<int64_t>();
      a.probes = ws.probes_i.as<int64_t>();
      a.n_slots = nq * np;
      a.n_probes = np;
      a.d = idx->d;
      a.rot_dim_pad = idx->rot_dim_pad;
      a.pq_dim = idx->pq_dim;
      a.pq_dim_pad = idx->pq_dim_pad;
      a.pq_len = idx->pq_len;
      a.k = k;
      a.out_d = ws.part_d.as<float>();
      a.out_i = ws.part_i.as<int64_t>();
      a.flags = env_int("MIVS_PQ_FLAGS", 0);
      // list-sorted, XCD-aware slot order: the probe map with one chunk per list gives, per list, the queries
      // probing it and their output slots
      {
        const int64_t ne = nq * np;
        ws.counts.reserve(sizeof(int) * L.n_lists);
        ws.fill.reserve(sizeof(int) * L.n_lists);
        ws.bucket_off.reserve(sizeof(int) * (L.n_lists + 1));
        ws.work_off.reserve(sizeof(int) * (L.n_lists + 1));
        ws.bucket_q.reserve(sizeof(int64_t) * ne);
        ws.bucket_slot.reserve(sizeof(int64_t) * ne);
        ws.qp_slots.reserve(sizeof(int64_t) * ne);
        ws.slot_begin.reserve(sizeof(int64_t) * (nq + 1));
        const size_t stb = scan_tmp_bytes(ne) + sizeof(int64_t) * (size_t)ne;
        ws.scan_tmp.reserve(stb);
        HIPCHK(launch_probe_map(ws.probes_i.as<int64_t>(), nq, np, L.n_lists, L.goff.as<int64_t>(), 1 << 28, 1,
                                ws.counts.as<int>(), ws.fill.as<int>(), ws.bucket_off.as<int>(), ws.work_off.as<int>(),
                                ws.bucket_q.as<int64_t>(), ws.bucket_slot.as<int64_t>(), ws.qp_slots.as<int64_t>(),
                                ws.slot_begin.as<int64_t>(), ws.scan_tmp.p, stb, s));
        a.ent_q = ws.bucket_q.as<int64_t>();
        a.ent_slot = ws.bucket_slot.as<int64_t>();
        a.ent_off = ws.bucket_off.as<int>();
        a.n_lists = L.n_lists;
      }
      a.pq_half = (int)ceil_div(ceil_div(idx->pq_dim, 2), 16) * 16;
      a.ip = idx->metric == MIVS_METRIC_IP ? 1 : 0;
      a.probes_d = ws.probes_d.as<float>();
      // (MIVS_PQ_SPLIT=0 asks for K9 where its whole LUT and merge area fit LDS)
      const char* spe = getenv("MIVS_PQ_SPLIT");
      const bool k9_fits = pq_scan_lds_bytes(idx->rot_dim_pad, idx->pq_dim, kcap) <= 160 * 1024;
      const bool split = (!(spe && spe[0] == '0') || !k9_fits) && !(a.flags & 7);
      if (pr) HIPCHK(hipEventRecord(pr->e[1], s));
      hipError_t se = split ? launch_pq_scan_split(a, kcap, s) : hipErrorNotSupported;
      if (se == hipErrorNotSupported) se = launch_pq_scan(a, kcap, s);
      HIPCHK(se);
      if (pr) HIPCHK(hipEventRecord(pr->e[2], s));
      MergeArgs m{};
      m.in_d = ws.part_d.as<float>();
      m.in_i = ws.part_i.as<int64_t>();
      m.slot_begin = ws.slot_begin.as<int64_t>();
      m.slots_per_q = np;
      m.nq = nq;
      m.k_in = k;
      m.k = k;
      m.metric = idx->metric;
      m.out_d = d_dist;
      m.out_i = d_ids;
      HIPCHK(launch_merge(m, s));
    }
    if (pr) HIPCHK(hipEventRecord(pr->e[3], s));
    idx->last_nq = nq;
    idx->last_np = np;
    idx->last_k = k;
  });
}

int32_t mivs_ivf_pq_info(mivs_index_t idx, int32_t* pq_dim, int32_t* pq_bits, int32_t* pq_len) {
  return guarded([&] {
    require(idx != nullptr && idx->kind == 2, "not an ivf_pq index");
    if (pq_dim) *pq_dim = idx->pq_dim;
    if (pq_bits) *pq_bits = idx->pq_bits;
    if (pq_len) *pq_len = idx->pq_len;
  });
}

int32_t mivs_ivf_pq_get_codebooks(mivs_index_t idx, void* stream, float* d_out) {
  return guarded([&] {
    require(idx != nullptr && idx->kind == 2, "not an ivf_pq index");
    DeviceGuard dg(idx->device);
    IndexCall ic(idx, static_cast<hipStream_t>(stream));
    HIPCHK(hipMemcpyAsync(d_out, idx->pq_books.p, sizeof(float) * (size_t)idx->pq_dim * (1 << idx->pq_bits) * idx->pq_len,
                          hipMemcpyDeviceToDevice, static_cast<hipStream_t>(stream)));
  });
}

int32_t mivs_ivf_pq_get_codes(mivs_index_t idx, void* stream, uint8_t* d_out) {
  return guarded([&] {
    require(idx != nullptr && idx->kind == 2, "not an ivf_pq index");
    DeviceGuard dg(idx->device);
    IndexCall ic(idx, static_cast<hipStream_t>(stream));
    const ListSet& L = idx->lists;
    HIPCHK(launch_pq_unpack(static_cast<const uint8_t*>(idx->pq_codes.p), L.n_rows, L.off.as<int64_t>(),
                            L.goff.as<int64_t>(), L.n_lists, idx->pq_dim, idx->pq_dim_pad, d_out,
                            static_cast<hipStream_t>(stream)));
  });
}

int32_t mivs_brute_force_build(int32_t device, void* stream, const float* d_data, int64_t n, int32_t dim,
                               int32_t metric, int64_t id_offset, mivs_index_t* out) {
  return guarded([&] {
    require(out != nullptr, "out is NULL");
    check_common(device, d_data, n, dim);
    require(metric == MIVS_METRIC_L2 || metric == MIVS_METRIC_IP, "unknown metric");
    DeviceGuard dg(device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    auto idx = std::make_unique<mivs_index_s>();
    IndexCall ic(idx.get(), s);
    idx->kind = 1;
    idx->device = device;
    idx->d = dim;
    idx->dp = dim_pad(dim);
    idx->metric = metric;
    idx->id_offset = id_offset;
    make_single_list(idx->lists, d_data, n, dim, idx->dp, id_offset, idx->G, s);
    if (pf_default_on()) pf_enable(idx.get(), s);  // k <= 16 searches go through the fp16 pre-filter
    *out = idx.release();
  });
}

int32_t mivs_brute_force_search(mivs_index_t idx, void* stream, const float* d_q, int64_t nq, int32_t k,
                                float* d_dist, int64_t* d_ids) {
  return guarded([&] {
    require(idx != nullptr && idx->kind == 1, "not a brute-force index");
    require(nq >= 0, "nq must be >= 0");
    require(k >= 1 && k <= kMaxSelectK, "k must be in [1, " + std::to_string(kMaxSelectK) + "]", MIVS_ERR_UNSUPPORTED);
    require(nq == 0 || (d_q && d_dist && d_ids), "NULL query/output pointer");
    if (nq == 0) return;
    std::lock_guard<std::mutex> g(idx->mu);
    DeviceGuard dg(idx->device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    IndexCall ic(idx, s);
    ProfRec* pr = g_profiling.load() ? idx->prof.begin(s) : nullptr;
    idx->ws.qn.reserve(sizeof(float) * nq);
    HIPCHK(launch_row_norms(d_q, nq, idx->d, idx->ws.qn.as<float>(), s));
    if (idx->groups_h.p != nullptr && k <= kPfMaxK) {
      // the fp16 pre-filter + exact refine, as an IVF search in which every query probes the one list
      idx->ws.probes_i.reserve(sizeof(int64_t) * nq);
      HIPCHK(hipMemsetAsync(idx->ws.probes_i.p, 0, sizeof(int64_t) * nq, s));
      idx->last_ovf = 0;
      idx->last_window = 0;
      idx->last_stats_dev = false;
      ivf_search_probed(idx, s, d_q, nq, k, 1, d_dist, d_ids, true, pr, true);
      idx->last_nq = nq;
      idx->last_np = 1;
      idx->last_k = k;
      return;
    }
    // the exact fp32 scan: no pre-filter ran, nothing overflowed (stats must not keep a previous search's)
    idx->last_pf = 0;
    idx->last_ovf = 0;
    idx->last_window = 0;
    idx->last_stats_dev = false;
    if (pr) HIPCHK(hipEventRecord(pr->e[1], s));
    single_list_topk(idx->lists, idx->G, d_q, idx->ws.qn.as<float>(), nullptr, nq, idx->d, idx->dp, k, idx->metric,
                     d_dist, d_ids, idx->device, idx->ws, s);
    if (pr) {
      HIPCHK(hipEventRecord(pr->e[2], s));
      HIPCHK(hipEventRecord(pr->e[3], s));
    }
    idx->last_nq = nq;
    idx->last_np = 1;
    idx->last_k = k;
    idx->last_qtile = k > kMaxK ? kQTile : pick_qtile(k, idx->d, idx->G);
  });
}

int32_t mivs_index_info(mivs_index_t idx, int64_t* n_rows, int32_t* dim, int32_t* n_lists, int32_t* metric,
                        int32_t* device) {
  return guarded([&] {
    require(idx != nullptr, "index is NULL");
    if (n_rows) *n_rows = idx->lists.n_rows;
    if (dim) *dim = idx->d;
    if (n_lists) *n_lists = idx->lists.n_lists;
    if (metric) *metric = idx->metric;
    if (device) *device = idx->device;
  });
}

int32_t mivs_index_last_search_stats(mivs_index_t idx, mivs_search_stats* out) {
  return guarded([&] {
    require(idx != nullptr && out != nullptr, "NULL argument");
    DeviceGuard dg(idx->device);
    std::lock_guard<std::mutex> g(idx->mu);
    mivs_search_stats st{};
    st.n_queries = idx->last_nq;
    st.n_probes = idx->last_np;
    st.k = idx->last_k;
    st.query_tile = idx->last_qtile;
    st.kcap = idx->last_k > 0 ? scan_kcap(idx->last_k) : 0;
    st.prefilter = idx->last_pf;
    st.scan_kernel = idx->last_scan;
    st.overflow_queries = idx->last_ovf;
    st.window_candidates = idx->last_window;
    wait_index(idx);  // (the last search may still run on its stream: its stats are written by the device)
    if (idx->last_stats_dev) {  // (the device-sized fallback left them in ws.pf_stats: {count, pad, window})
      int64_t h[2] = {0, 0};
      HIPCHK(hipMemcpy(h, idx->ws.pf_stats.p, sizeof(h), hipMemcpyDeviceToHost));
      st.overflow_queries = (int64_t)(int32_t)(h[0] & 0xFFFFFFFF);
      st.window_candidates = h[1];
    }
    st.copies_skipped = idx->copies_skipped;
    const ListSet& L = idx->lists;
    if (idx->last_nq > 0 && idx->kind == 0) {
      std::vector<int> counts(L.n_lists), woff(L.n_lists + 1);
      // K13: its own probe map's counts (the exact fallback of unproven queries maps only those)
      const Buf& cb = idx->last_scan == 13 ? idx->ws.stat_counts : idx->ws.counts;
      HIPCHK(hipMemcpy(counts.data(), cb.p, sizeof(int) * L.n_lists, hipMemcpyDeviceToHost));
      HIPCHK(hipMemcpy(woff.data(), idx->ws.work_off.p, sizeof(int) * (L.n_lists + 1), hipMemcpyDeviceToHost));
      for (int l = 0; l < L.n_lists; ++l) {
        st.scanned_rows += (int64_t)counts[l] * (L.h_off[l + 1] - L.h_off[l]);
        // K13 streams every probed row once (the query tiles move, the rows stay in registers)
        st.streamed_groups += (idx->last_scan == 13 ? (counts[l] > 0 ? 1 : 0) : ceil_div(counts[l], idx->last_qtile)) *
                              (L.h_goff[l + 1] - L.h_goff[l]);
        if (counts[l] > 0) st.unique_groups += L.h_goff[l + 1] - L.h_goff[l];
      }
      st.work_items = woff[L.n_lists];
      if (idx->last_scan == 13) {
        st.work_items = 0;
        for (int l = 0; l < L.n_lists; ++l)
          if (counts[l] > 0) st.work_items += ceil_div(L.h_goff[l + 1] - L.h_goff[l], kRsBlockGroups);
        // the candidates K13 appended; a lost stream entry sends every query to the fallback
        int64_t total = 0;
        int lost[10] = {};
        if (idx->last_rs_one_pass) {  // (per-query counts of the fixed-capacity runs, dropped entries included)
          std::vector<int> qc((size_t)idx->last_rs_nq);
          HIPCHK(hipMemcpy(qc.data(), idx->ws.rs_qcnt.p, sizeof(int) * qc.size(), hipMemcpyDeviceToHost));
          for (int c : qc) total += c;
        } else {
          HIPCHK(hipMemcpy(&total, idx->ws.cand_off.as<int64_t>() + idx->last_rs_nq, sizeof(int64_t),
                           hipMemcpyDeviceToHost));
        }
        HIPCHK(hipMemcpy(lost, idx->ws.rs_wave_cnt.as<int>() + idx->last_rs_waves, sizeof(lost), hipMemcpyDeviceToHost));
        st.candidates = total;
        st.spun_out_waves = lost[9];
        st.cand_overflow = lost[0] && !lost[9] ? idx->last_rs_nq : 0;
      }
    } else if (idx->last_nq > 0) {
      // brute force: the pre-filter scan (K10) works in pf_G-group chunks, the exact scans in G
      const int G = idx->last_pf ? idx->pf_G : idx->G;
      st.scanned_rows = idx->last_nq * L.n_rows;
      st.streamed_groups = ceil_div(idx->last_nq, idx->last_qtile) * L.n_groups;
      st.unique_groups = L.n_groups;
      st.work_items = ceil_div(idx->last_nq, idx->last_qtile) * std::max<int64_t>(1, ceil_div(L.n_groups, G));
    }
    *out = st;
  });
}

int32_t mivs_index_memory_info(mivs_index_t idx, mivs_index_memory* out) {
  return guarded([&] {
    require(idx != nullptr && out != nullptr, "NULL argument");
    std::lock_guard<std::mutex> g(idx->mu);
    *out = index_memory(idx);
  });
}

int32_t mivs_index_build_kernels(mivs_index_t idx, mivs_build_kernel* out, int32_t n_max, int32_t* n_out) {
  return guarded([&] {
    require(idx != nullptr, "index is NULL");
    int n = 0;
    for (int k = 0; k < MIVS_BUILD_KERNEL_KINDS && k < n_max; ++k) {
      if (out) out[k] = idx->build_kern[k];
      ++n;
    }
    if (n_out) *n_out = n;
  });
}

int32_t mivs_index_build_phases(mivs_index_t idx, double* out_s, int32_t n_max, int32_t* n_out) {
  return guarded([&] {
    require(idx != nullptr && n_out != nullptr, "NULL argument");
    const int n = (int)idx->build_phase_s.size();
    for (int i = 0; i < n && i < n_max && out_s; ++i) out_s[i] = idx->build_phase_s[i];
    *n_out = n;
  });
}

int32_t mivs_index_profile_collect(mivs_index_t idx, mivs_profile* out) {
  return guarded([&] {
    require(idx != nullptr && out != nullptr, "NULL argument");
    DeviceGuard dg(idx->device);
    std::lock_guard<std::mutex> g(idx->mu);
    mivs_profile p{};
    p.scan_ms_min = 0.0f;
    for (auto& r : idx->prof.pending) {
      HIPCHK(hipEventSynchronize(r.e[3]));
      float a = 0, b = 0, c = 0;
      HIPCHK(hipEventElapsedTime(&a, r.e[0], r.e[1]));
      HIPCHK(hipEventElapsedTime(&b, r.e[1], r.e[2]));
      HIPCHK(hipEventElapsedTime(&c, r.e[0], r.e[3]));
      p.coarse_ms += a;
      p.scan_ms += b;
      p.total_ms += c;
      p.scan_ms_min = p.n_calls == 0 ? b : std::min(p.scan_ms_min, b);
      p.scan_ms_max = std::max(p.scan_ms_max, b);
      p.n_calls += 1;
      idx->prof.pool.push_back(r);
    }
    idx->prof.pending.clear();
    *out = p;
  });
}

int32_t mivs_index_set_prefilter(mivs_index_t idx, void* stream, int32_t enable) {
  return guarded([&] {
    require(idx != nullptr, "index is NULL");
    require(idx->kind == 0 || idx->kind == 1, "the fp16 pre-filter applies to ivf_flat / brute_force indexes",
            MIVS_ERR_UNSUPPORTED);
    std::lock_guard<std::mutex> g(idx->mu);
    DeviceGuard dg(idx->device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    IndexCall ic(idx, s);
    HIPCHK(hipStreamSynchronize(s));
    if (enable) {
      if (!idx->groups_h.p) pf_enable(idx, s);
    } else {
      idx->groups_h.release();
      idx->groups_f8.release();
    }
  });
}

int32_t mivs_index_get_prefilter(mivs_index_t idx, int32_t* enabled) {
  return guarded([&] {
    require(idx != nullptr && enabled != nullptr, "NULL argument");
    *enabled = idx->groups_h.p != nullptr ? 1 : 0;
  });
}

void mivs_index_free(mivs_index_t idx) {
  if (!idx) return;
  int prev = -1;
  (void)hipGetDevice(&prev);
  (void)hipSetDevice(idx->device);
  // wait for the index's own calls (their done-events), not for the device: a concurrent search on another index of
  // this GPU keeps running; the buffers then go back without further waiting
  bool synced = true;
  for (auto& e : idx->stream_done) synced = hipEventSynchronize(e.ev) == hipSuccess && synced;
  (void)hipGetLastError();
  tl_release_synced = synced && !idx->stream_done.empty();
  delete idx;
  tl_release_synced = false;
  if (prev >= 0) (void)hipSetDevice(prev);
}

int32_t mivs_set_block_cache_limit(int32_t device, int64_t bytes) {
  return guarded([&] {
    require(bytes >= 0, "bytes must be >= 0");
    require(device >= -1 && device < BlockCache::kMaxDev, "device out of range");
    BlockCache::get().set_limit(device, (size_t)bytes);
  });
}

int32_t mivs_release_cached_memory(int32_t device, int64_t* freed_bytes) {
  return guarded([&] {
    require(device >= -1 && device < BlockCache::kMaxDev, "device out of range");
    const size_t f = BlockCache::get().flush(device);
    if (freed_bytes) *freed_bytes = (int64_t)f;
  });
}

int32_t mivs_cached_memory(int32_t device, int64_t* bytes, int64_t* limit) {
  return guarded([&] {
    require(device >= -1 && device < BlockCache::kMaxDev, "device out of range");
    if (bytes) *bytes = (int64_t)BlockCache::get().cached(device);
    if (limit) *limit = device >= 0 ? (int64_t)BlockCache::get().limit_of(device) : -1;
  });
}

void mivs_reload_settings(void) { reload_settings(); }

int32_t mivs_kmeans_fit(int32_t device, void* stream, const float* d_data, int64_t n, int32_t dim,
                        const int64_t* d_rows, int64_t n_train, int32_t n_clusters, int32_t n_iters,
                        float* d_centroids) {
  return guarded([&] {
    check_common(device, d_data, n, dim);
    require(n_clusters >= 1 && n_clusters <= 32768, "n_clusters must be in [1, 32768]");
    require(n_train >= 1 && (d_rows != nullptr || n_train <= n), "bad trainset");
    DeviceGuard dg(device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    StreamScope ss(s);
    Workspace ws;
    Buf norms;
    norms.reserve(sizeof(float) * std::max<int64_t>(n, 1));
    HIPCHK(launch_row_norms(d_data, n, dim, norms.as<float>(), s));
    kmeans_fit_impl(d_data, norms.as<float>(), d_rows, n_train, dim, dim_pad(dim), n_clusters, n_iters, d_centroids,
                    kDefaultChunkGroups, device, ws, s);
  });
}

int32_t mivs_kmeans_steps(int32_t device, void* stream, const float* d_data, int64_t n, int32_t dim,
                          const int64_t* d_rows, int64_t n_train, int32_t n_clusters, int32_t it_begin, int32_t n_steps,
                          int32_t it_total, int32_t balance, float* d_centroids, int64_t* d_labels) {
  return guarded([&] {
    check_common(device, d_data, n, dim);
    require(n_clusters >= 1 && n_clusters <= 32768, "n_clusters must be in [1, 32768]");
    require(n_train >= 1 && (d_rows != nullptr || n_train <= n), "bad trainset");
    require(it_begin >= 0 && n_steps >= 0 && it_total >= it_begin + n_steps, "bad iteration range");
    if (n_steps == 0) return;
    DeviceGuard dg(device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    StreamScope ss(s);
    Workspace ws;
    Buf norms;
    norms.reserve(sizeof(float) * std::max<int64_t>(n, 1));
    HIPCHK(launch_row_norms(d_data, n, dim, norms.as<float>(), s));
    PfAssign pfa;  // the assign of the IVF build, as ivf_flat_build runs it
    pf_assign_prepare(pfa, d_data, n, dim, dim_pad(dim), s);
    kmeans_fit_impl(d_data, norms.as<float>(), d_rows, n_train, dim, dim_pad(dim), n_clusters, n_steps, d_centroids,
                    kDefaultChunkGroups, device, ws, s, balance != 0, &pfa, it_begin, it_total, d_labels);
  });
}

int32_t mivs_kmeans_predict(int32_t device, void* stream, const float* d_data, int64_t n, int32_t dim,
                            const float* d_centroids, int32_t n_clusters, int32_t metric, int64_t* d_labels) {
  return guarded([&] {
    check_common(device, d_data, n, dim);
    require(n_clusters >= 1, "n_clusters must be >= 1");
    require(metric == MIVS_METRIC_L2 || metric == MIVS_METRIC_IP, "unknown metric");
    if (n == 0) return;
    DeviceGuard dg(device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    StreamScope ss(s);
    Workspace ws;
    ListSet cents;
    make_single_list(cents, d_centroids, n_clusters, dim, dim_pad(dim), 0, kDefaultChunkGroups, s);
    Buf norms;
    norms.reserve(sizeof(float) * n);
    HIPCHK(launch_row_norms(d_data, n, dim, norms.as<float>(), s));
    assign_rows(d_data, norms.as<float>(), nullptr, n, dim, dim_pad(dim), cents, kDefaultChunkGroups, metric,
                d_labels, device, ws, s);
  });
}

int32_t mivs_merge_topk(int32_t device, void* stream, const float* d_in_dist, const int64_t* d_in_ids, int64_t nq,
                        int32_t m, int32_t k_in, int32_t k, int32_t metric, float* d_out_dist,
                        int64_t* d_out_ids) {
  return guarded([&] {
    require(k >= 1 && k <= kMaxSelectK, "k must be in [1, " + std::to_string(kMaxSelectK) + "]", MIVS_ERR_UNSUPPORTED);
    require(m >= 0 && k_in >= 0 && nq >= 0, "bad shape");
    require(metric == MIVS_METRIC_L2 || metric == MIVS_METRIC_IP, "unknown metric");
    if (nq == 0) return;
    DeviceGuard dg(device);
    if (k > kMaxK) {  // K8 select over the explicit [nq][m*k_in] candidates
      SelectArgs sa{};
      sa.keys = d_in_dist;
      sa.ids = d_in_ids;
      sa.n_in = (int64_t)m * k_in;
      sa.nq = nq;
      sa.k = k;
      sa.metric = metric;
      sa.out_d = d_out_dist;
      sa.out_i = d_out_ids;
      HIPCHK(launch_select(sa, static_cast<hipStream_t>(stream)));
      return;
    }
    MergeArgs a{};
    a.in_d = d_in_dist;
    a.in_i = d_in_ids;
    a.slot_begin = nullptr;
    a.slots_per_q = m;
    a.nq = nq;
    a.k_in = k_in;
    a.k = k;
    a.metric = metric;
    a.out_d = d_out_dist;
    a.out_i = d_out_ids;
    HIPCHK(launch_merge(a, static_cast<hipStream_t>(stream)));
  });
}

int32_t mivs_refine(int32_t device, void* stream, const void* d_data, int32_t data_is_half, int64_t n, int32_t dim,
                    const float* d_queries, int64_t nq, const int64_t* d_candidates, int32_t n_candidates, int32_t k,
                    int32_t metric, float* d_distances, int64_t* d_neighbors) {
  return guarded([&] {
    require(dim >= 1 && dim_pad(dim) <= 1024, "dim must be in [1, 1024]", MIVS_ERR_UNSUPPORTED);
    require(n >= 0 && nq >= 0 && n_candidates >= 1, "bad shape");
    require(k >= 1 && k <= kMaxK && k <= n_candidates,
            "k must be in [1, min(n_candidates, " + std::to_string(kMaxK) + ")]", MIVS_ERR_UNSUPPORTED);
    require(metric == MIVS_METRIC_L2 || metric == MIVS_METRIC_IP, "unknown metric");
    if (nq == 0) return;
    require(d_data && d_queries && d_candidates && d_distances && d_neighbors, "null pointer");
    DeviceGuard dg(device);
    RefineArgs a{};
    a.data = d_data;
    a.n = n;
    a.d = dim;
    a.dp = dim_pad(dim);
    a.half = data_is_half ? 1 : 0;
    a.queries = d_queries;
    a.nq = nq;
    a.cand = d_candidates;
    a.n_cand = n_candidates;
    a.k = k;
    a.metric = metric;
    a.out_d = d_distances;
    a.out_i = d_neighbors;
    HIPCHK(launch_refine(a, static_cast<hipStream_t>(stream)));
  });
}

int32_t mivs_row_norms(int32_t device, void* stream, const float* d_x, int64_t n, int32_t dim, float* d_out) {
  return guarded([&] {
    check_common(device, d_x, n, dim);
    DeviceGuard dg(device);
    HIPCHK(launch_row_norms(d_x, n, dim, d_out, static_cast<hipStream_t>(stream)));
  });
}

int32_t mivs_normalize_rows(int32_t device, void* stream, const float* d_x, int64_t n, int32_t dim, float* d_out) {
  return guarded([&] {
    require(dim >= 1 && n >= 0, "bad shape");
    require(n == 0 || (d_x && d_out), "null pointer");
    DeviceGuard dg(device);
    hipStream_t s = static_cast<hipStream_t>(stream);
    Buf n2;
    n2.reserve(sizeof(float) * (size_t)std::max<int64_t>(n, 1));
    HIPCHK(launch_normalize_rows(d_x, n, dim, n2.as<float>(), d_out, s));
    HIPCHK(hipStreamSynchronize(s));  // n2 is freed on return
  });
}

int32_t mivs_synth_mixture(int32_t device, void* stream, float* d_out, int64_t row_begin, int64_t n, int32_t dim,
                           uint64_t seed, int32_t n_centers, float sigma, int32_t normalize) {
  return guarded([&] {
    require(n_centers >= 1, "n_centers must be >= 1");
    require(dim >= 1 && n >= 0, "bad shape");
    DeviceGuard dg(device);
    HIPCHK(launch_synth_mixture(d_out, row_begin, n, dim, seed, n_centers, sigma, normalize,
                                static_cast<hipStream_t>(stream)));
  });
}

}  // extern "C"
