// K14 — exact re-ranking of candidate neighbours (cuVS cuvs.neighbors.refine, cuvs 25.06, the step
// that turns IVF-PQ's approximate top-(r*k) into an exact top-k).
//
// One wave per query: the query sits in LDS (zero-padded to dp), each lane takes one candidate row at
// a time and forms its dot and its norm in the pinned fp32 order of the arithmetic contract (k-step s:
// dims 8s+j then 8s+4+j, j = 0..3 -- oracle/mivs_oracle.c orc_dot), so keys are bit-identical to the
// exact scans; the wave keeps the running top-k by (key, id) with K7's ballot insertion. Rows are read
// straight from the caller's dataset ([n][d], fp32 or fp16 widened exactly to fp32).
#include <climits>

#include "mivs_common.hpp"

namespace mivs {

namespace {

template <typename T>
__device__ __forceinline__ float rf_ld(const T* p) { return (float)p[0]; }

template <typename T>
__device__ __forceinline__ void rf_ld8(const T* p, float (&v)[8]) {
  if constexpr (sizeof(T) == 4) {
    const float4 a = *reinterpret_cast<const float4*>(p);
    const float4 b = *reinterpret_cast<const float4*>(p + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  } else {
    typedef _Float16 h8 __attribute__((ext_vector_type(8)));
    const h8 h = *reinterpret_cast<const h8*>(p);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (float)h[i];
  }
}

__device__ __forceinline__ bool rf_lt(float ak, int64_t ai, float bk, int64_t bi) {
  return ak < bk || (ak == bk && ai < bi);
}

template <int METRIC, typename T>
__global__ __launch_bounds__(256) void k_refine(RefineArgs a) {
  __shared__ __attribute__((aligned(16))) float s_q[4][1024];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t q = (int64_t)blockIdx.x * 4 + wv;
  if (q >= a.nq) return;
  const int d = a.d, dp = a.dp;
  const T* data = static_cast<const T*>(a.data);
  float* qv = s_q[wv];
  for (int i = lane; i < dp; i += 64) qv[i] = i < d ? a.queries[q * d + i] : 0.0f;
  // (one wave per query: its own LDS slice, written and read by this wave only)
  __builtin_amdgcn_wave_barrier();
  float qn = 0.0f;
  for (int s = 0; s < dp; s += 8)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      qn = fmaf(qv[s + j], qv[s + j], qn);
      qn = fmaf(qv[s + 4 + j], qv[s + 4 + j], qn);
    }
  const bool vec = (d & 7) == 0 && (reinterpret_cast<uintptr_t>(data) & 15) == 0;
  const int k = a.k;
  float mk = INFINITY, tk = INFINITY;  // rank `lane` of the running top-k, and rank k-1
  int64_t mi = LLONG_MAX, ti = LLONG_MAX;
  for (int c0 = 0; c0 < a.n_cand; c0 += 64) {
    const int c = c0 + lane;
    float key = INFINITY;
    int64_t id = LLONG_MAX;
    const int64_t cid = c < a.n_cand ? a.cand[q * a.n_cand + c] : -1;
    if (cid >= 0 && cid < a.n) {
      const T* row = data + cid * d;
      float dot = 0.0f, xn = 0.0f;
      for (int s = 0; s < dp; s += 8) {
        float v[8];
        if (vec) {  // d % 8 == 0: a block is all in the row (s < d) or all padding
          if (s < d) {
            rf_ld8<T>(row + s, v);
          } else {
#pragma unroll
            for (int i = 0; i < 8; ++i) v[i] = 0.0f;
          }
        } else {
#pragma unroll
          for (int i = 0; i < 8; ++i) v[i] = s + i < d ? rf_ld<T>(row + s + i) : 0.0f;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          dot = fmaf(v[j], qv[s + j], dot);
          dot = fmaf(v[4 + j], qv[s + 4 + j], dot);
          xn = fmaf(v[j], v[j], xn);
          xn = fmaf(v[4 + j], v[4 + j], xn);
        }
      }
      if (METRIC == kL2) {
        const float t = fmaf(-2.0f, dot, xn + qn);
        key = t > 0.0f ? t : 0.0f;
      } else {
        key = -dot;
      }
      id = a.id_map ? a.id_map[cid] : cid;
    }
    uint64_t mask = __ballot(rf_lt(key, id, tk, ti));
    while (mask) {
      const int b = __ffsll((unsigned long long)mask) - 1;
      const float nk = __shfl(key, b);
      const int64_t ni = __shfl(id, b);
      const int pos = __popcll(__ballot(lane < k && rf_lt(mk, mi, nk, ni)));
      const float pk = __shfl_up(mk, 1);
      const int64_t pi = __shfl_up(mi, 1);
      if (lane == pos) { mk = nk; mi = ni; }
      else if (lane > pos) { mk = pk; mi = pi; }
      tk = __shfl(mk, k - 1);
      ti = __shfl(mi, k - 1);
      mask &= ~(1ull << b);
      mask &= __ballot(rf_lt(key, id, tk, ti));
    }
  }
  if (lane < k) {
    const bool valid = mi != LLONG_MAX;
    a.out_d[q * k + lane] = valid ? (METRIC == kIP ? -mk : mk) : (METRIC == kIP ? -INFINITY : INFINITY);
    a.out_i[q * k + lane] = valid ? mi : (int64_t)-1;
  }
}

// K14g: the same keys with the candidate rows gathered coalesced. One lane per row (k_refine) reads 16 B of 64
// different rows per load instruction, 96-192 dependent loads per row: the configs[4] refine (120 candidates x 10k
// queries, 1.84 GB of fp16 rows) ran at ~1.1 TB/s. Here eight lanes share a row, as in K11's exact recompute
// (prefilter.hip): lane (j, p) = (lane >> 3, lane & 7) of a pass holds the 8-dim blocks b = 8 B + p of candidate
// r0 + j, so a group of eight reads 128 B (fp16) / 256 B (fp32) contiguous per 64-dim block, every block of the row
// in flight at once. The row's two fmaf chains (dot and norm, dims in the contract's order) run over the blocks
// b = 0, 1, 2, ... by handing the accumulators to the next lane of the group with a DPP move (row_shr:1; part 7 ->
// part 0 of the next 64-dim block by row_shl:7): lane (j, h) extends them at hop h, the other lanes' values are
// discarded. Needs d % 8 == 0 (a block is all in the row or all padding) and 16-B aligned rows.
template <int METRIC, typename T>
__global__ __launch_bounds__(256) void k_refine_g(RefineArgs a) {
  constexpr int CH = 12;  // 64-dim blocks of a row in flight per pass (d = 768: the whole row)
  __shared__ __attribute__((aligned(16))) float s_q[4][1024];
  __shared__ float s_key[4][64];
  __shared__ int64_t s_id[4][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t q = (int64_t)blockIdx.x * 4 + wv;
  if (q >= a.nq) return;  // (wave-uniform; no workgroup barrier below)
  const int d = a.d, dp = a.dp;
  const T* data = static_cast<const T*>(a.data);
  float* qv = s_q[wv];
  for (int i = lane; i < dp; i += 64) qv[i] = i < d ? a.queries[q * d + i] : 0.0f;
  wave_lds_sync();
  float qn = 0.0f;
  for (int s = 0; s < dp; s += 8)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      qn = fmaf(qv[s + j], qv[s + j], qn);
      qn = fmaf(qv[s + 4 + j], qv[s + 4 + j], qn);
    }
  const int k = a.k;
  const int j8 = lane >> 3, p8 = lane & 7;
  const int nB = dp >> 6;
  float mk = INFINITY, tk = INFINITY;  // rank `lane` of the running top-k, and rank k-1
  int64_t mi = LLONG_MAX, ti = LLONG_MAX;
  for (int c0 = 0; c0 < a.n_cand; c0 += 64) {
    // 8 passes of 8 rows: each row's key lands in s_key[wv][row - c0] (lane p == 7 ends its chains)
    for (int r0 = 0; r0 < 64; r0 += 8) {
      const int c = c0 + r0 + j8;
      const int64_t cid = c < a.n_cand ? a.cand[q * a.n_cand + c] : -1;
      const bool ok = cid >= 0 && cid < a.n;
      if (__ballot(ok) == 0) {  // (a pass with no row: nothing to read)
        if (p8 == 7) { s_key[wv][r0 + j8] = INFINITY; s_id[wv][r0 + j8] = LLONG_MAX; }
        continue;
      }
      const T* rowp = data + (ok ? cid : 0) * (int64_t)d + 8 * p8;
      float dot = 0.0f, xn = 0.0f;
      for (int B0 = 0; B0 < nB; B0 += CH) {
        float v[CH][8];
#pragma unroll
        for (int u = 0; u < CH; ++u) {
          const int dim = 64 * (B0 + u) + 8 * p8;
          if (B0 + u < nB && dim < d) {
            rf_ld8<T>(rowp + 64 * (B0 + u), v[u]);
          } else {
#pragma unroll
            for (int i = 0; i < 8; ++i) v[u][i] = 0.0f;
          }
        }
#pragma unroll
        for (int u = 0; u < CH; ++u) {
          if (B0 + u >= nB) break;
          const float* y = qv + 64 * (B0 + u) + 8 * p8;
          const float4 y0 = *reinterpret_cast<const float4*>(y);
          const float4 y1 = *reinterpret_cast<const float4*>(y + 4);
          const float yy[8] = {y0.x, y0.y, y0.z, y0.w, y1.x, y1.y, y1.z, y1.w};
#pragma unroll
          for (int h = 0; h < 8; ++h) {
            if (h > 0) {
              dot = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, dot), 0x111, 0xF, 0xF, false));
              xn = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, xn), 0x111, 0xF, 0xF, false));
            } else if (B0 + u > 0) {
              dot = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, dot), 0x107, 0xF, 0xF, false));
              xn = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, xn), 0x107, 0xF, 0xF, false));
            }
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
              dot = fmaf(v[u][jj], yy[jj], dot);
              dot = fmaf(v[u][4 + jj], yy[4 + jj], dot);
              xn = fmaf(v[u][jj], v[u][jj], xn);
              xn = fmaf(v[u][4 + jj], v[u][4 + jj], xn);
            }
          }
        }
      }
      if (p8 == 7) {
        float key = INFINITY;
        int64_t id = LLONG_MAX;
        if (ok) {
          if (METRIC == kL2) {
            const float t = fmaf(-2.0f, dot, xn + qn);
            key = t > 0.0f ? t : 0.0f;
          } else {
            key = -dot;
          }
          id = a.id_map ? a.id_map[cid] : cid;
        }
        s_key[wv][r0 + j8] = key;
        s_id[wv][r0 + j8] = id;
      }
    }
    wave_lds_sync();
    const float key = s_key[wv][lane];
    const int64_t id = s_id[wv][lane];
    wave_lds_sync();  // (the next round's stores come after every lane's reads)
    // the running top-k by (key, id): K7's ballot insertion, as k_refine
    uint64_t mask = __ballot(rf_lt(key, id, tk, ti));
    while (mask) {
      const int b = __ffsll((unsigned long long)mask) - 1;
      const float nk = __shfl(key, b);
      const int64_t ni = __shfl(id, b);
      const int pos = __popcll(__ballot(lane < k && rf_lt(mk, mi, nk, ni)));
      const float pk = __shfl_up(mk, 1);
      const int64_t pi = __shfl_up(mi, 1);
      if (lane == pos) { mk = nk; mi = ni; }
      else if (lane > pos) { mk = pk; mi = pi; }
      tk = __shfl(mk, k - 1);
      ti = __shfl(mi, k - 1);
      mask &= ~(1ull << b);
      mask &= __ballot(rf_lt(key, id, tk, ti));
    }
  }
  if (lane < k) {
    const bool valid = mi != LLONG_MAX;
    a.out_d[q * k + lane] = valid ? (METRIC == kIP ? -mk : mk) : (METRIC == kIP ? -INFINITY : INFINITY);
    a.out_i[q * k + lane] = valid ? mi : (int64_t)-1;
  }
}

}  // namespace

hipError_t launch_refine(const RefineArgs& a, hipStream_t s) {
  if (a.k < 1 || a.k > kMaxK || a.dp > 1024 || a.dp < a.d) return hipErrorInvalidValue;
  if (a.nq <= 0) return hipSuccess;
  const dim3 grid((unsigned)ceil_div(a.nq, 4));
  static const bool lane_per_row = [] {  // (MIVS_REFINE_GATHER=0: the one-lane-per-row kernel, for A/B runs)
    const char* e = getenv("MIVS_REFINE_GATHER");
    return e && e[0] == '0';
  }();
  const bool gather = !lane_per_row && (a.d & 7) == 0 && (a.dp & 63) == 0 &&
                      (reinterpret_cast<uintptr_t>(a.data) & 15) == 0;
  if (gather) {
    if (a.half) {
      if (a.metric == kIP) hipLaunchKernelGGL((k_refine_g<kIP, _Float16>), grid, dim3(256), 0, s, a);
      else hipLaunchKernelGGL((k_refine_g<kL2, _Float16>), grid, dim3(256), 0, s, a);
    } else {
      if (a.metric == kIP) hipLaunchKernelGGL((k_refine_g<kIP, float>), grid, dim3(256), 0, s, a);
      else hipLaunchKernelGGL((k_refine_g<kL2, float>), grid, dim3(256), 0, s, a);
    }
    return hipGetLastError();
  }
  if (a.half) {
    if (a.metric == kIP) hipLaunchKernelGGL((k_refine<kIP, _Float16>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((k_refine<kL2, _Float16>), grid, dim3(256), 0, s, a);
  } else {
    if (a.metric == kIP) hipLaunchKernelGGL((k_refine<kIP, float>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((k_refine<kL2, float>), grid, dim3(256), 0, s, a);
  }
  return hipGetLastError();
}

}  // namespace mivs
