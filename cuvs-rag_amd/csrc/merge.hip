// K7 — wave-level top-k merge of sorted candidate lists.
//
// One wave per query. The wave holds the running top-k distributed over its
// lanes (lane r = rank r, k <= 64). Candidates stream in 64 at a time; one
// compare against the broadcast k-th entry rejects almost all of them, the
// ballot of survivors is inserted one by one with a shfl_up shift.
// Serves (i) the nprobe x chunk partials of an IVF search, (ii) the chunk
// partials of brute force / coarse probe selection, (iii) the cross-shard merge
// after the RCCL all-gather — the merge the reference does on the host with
// numpy (improved_multi_gpu_rag.py:266-275, cuvs-2gpu-main.ipynb:1820-1834,
// contract test_search_result_aggregator.py:308-358).
#include <algorithm>
#include <climits>

#include "mivs_common.hpp"

namespace mivs {

namespace {

__device__ __forceinline__ bool kv_lt(float ak, int64_t ai, float bk, int64_t bi) {
  return ak < bk || (ak == bk && ai < bi);
}

template <int METRIC>
__device__ __forceinline__ void merge_query(const MergeArgs& a, int64_t q, int lane) {
  int64_t sb, se;
  if (a.slot_begin) { sb = a.slot_begin[q]; se = a.slot_begin[q + 1]; }
  else if (a.part_stride > 0) { sb = 0; se = a.slots_per_q; }
  else { sb = q * a.slots_per_q; se = sb + a.slots_per_q; }
  const int64_t c1 = se * a.k_in;
  const int k = a.k;
  // candidate c -> element: contiguous, or (part c / k_in, rank c % k_in) of the rank-major gather
  auto at = [&](int64_t c) {
    if (a.part_stride <= 0) return c;
    const int64_t p = c / a.k_in;
    return p * a.part_stride + q * a.k_in + (c - p * a.k_in);
  };

  float mk = INFINITY;      // rank `lane` of the running top-k
  int64_t mi = LLONG_MAX;
  float tk = INFINITY;      // rank k-1 (threshold)
  int64_t ti = LLONG_MAX;
  for (int64_t c = sb * a.k_in; c < c1; c += 64) {
    const int64_t cc = c + lane;
    float ck = INFINITY;
    int64_t ci = LLONG_MAX;
    if (cc < c1) {
      const int64_t e = at(cc);
      const int64_t id = a.in_i[e];
      if (id >= 0) {
        const float dd = a.in_d[e];
        ck = METRIC == kIP ? -dd : dd;
        ci = id;
      }
    }
    uint64_t mask = __ballot(kv_lt(ck, ci, tk, ti));
    while (mask) {
      const int b = __ffsll((unsigned long long)mask) - 1;
      const float nk = __shfl(ck, b);
      const int64_t ni = __shfl(ci, b);
      const int pos = __popcll(__ballot(lane < k && kv_lt(mk, mi, nk, ni)));
      const float pk = __shfl_up(mk, 1);
      const int64_t pi = __shfl_up(mi, 1);
      if (lane == pos) { mk = nk; mi = ni; }
      else if (lane > pos) { mk = pk; mi = pi; }
      tk = __shfl(mk, k - 1);
      ti = __shfl(mi, k - 1);
      mask &= ~(1ull << b);
      mask &= __ballot(kv_lt(ck, ci, tk, ti));
    }
  }
  if (lane < k) {
    const bool valid = mi != LLONG_MAX;
    const int64_t o = a.out_rows ? a.out_rows[q] : q;
    a.out_d[o * k + lane] = valid ? (METRIC == kIP ? -mk : mk) : (METRIC == kIP ? -INFINITY : INFINITY);
    a.out_i[o * k + lane] = valid ? mi : (int64_t)-1;
  }
}

// one wave per query; with nq_dev (the device-sized fallback) a fixed grid strides over the *nq_dev queries, so
// an empty fallback costs one launch of workgroups that leave at once
template <int METRIC>
__global__ __launch_bounds__(256) void k_merge(MergeArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t q0 = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (!a.nq_dev) {
    if (q0 < a.nq) merge_query<METRIC>(a, q0, lane);
    return;
  }
  const int64_t n = *a.nq_dev < a.nq ? (int64_t)*a.nq_dev : a.nq;
  for (int64_t q = q0; q < n; q += (int64_t)gridDim.x * 4) merge_query<METRIC>(a, q, lane);
}

}  // namespace

hipError_t launch_merge(const MergeArgs& a, hipStream_t s) {
  if (a.k < 1 || a.k > kMaxK) return hipErrorInvalidValue;
  if (a.nq <= 0) return hipSuccess;
  const dim3 grid((unsigned)(a.nq_dev ? std::min<int64_t>(ceil_div(a.nq, 4), 1024) : ceil_div(a.nq, 4)));
  if (a.metric == kIP) hipLaunchKernelGGL(k_merge<kIP>, grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL(k_merge<kL2>, grid, dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace mivs
