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

typedef float f32x2 __attribute__((ext_vector_type(2)));

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
// A pass = 8 candidates (rows c0 .. c0 + 7 of the query's list). PF (fp16 rows, dp <= 768): the next pass's loads
// are issued before this pass's chains run, two passes' raw blocks in registers (12 x 16 B each), so a wave has a row
// set in flight while it computes -- one pass at a time left every pass waiting a full HBM round trip.
template <typename T>
struct RfRaw {  // one lane's 8-dim block of a row, as loaded
  typedef uint4 type;
};
template <>
struct RfRaw<float> {
  struct type {
    float4 a, b;
  };
};

template <typename T>
__device__ __forceinline__ typename RfRaw<T>::type rf_raw_ld(const T* p) {
  typename RfRaw<T>::type r;
  if constexpr (sizeof(T) == 4) {
    r.a = *reinterpret_cast<const float4*>(p);
    r.b = *reinterpret_cast<const float4*>(p + 4);
  } else {
    r = *reinterpret_cast<const uint4*>(p);
  }
  return r;
}

template <typename T>
__device__ __forceinline__ void rf_raw_cvt(const typename RfRaw<T>::type& r, float (&v)[8]) {
  if constexpr (sizeof(T) == 4) {
    v[0] = r.a.x; v[1] = r.a.y; v[2] = r.a.z; v[3] = r.a.w; v[4] = r.b.x; v[5] = r.b.y; v[6] = r.b.z; v[7] = r.b.w;
  } else {
    typedef _Float16 h8 __attribute__((ext_vector_type(8)));
    const h8 h = __builtin_bit_cast(h8, r);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (float)h[i];
  }
}

constexpr int kRfCh = 12;  // K14g: 64-dim blocks of a row in flight per pass (d = 768: the whole row)

template <int METRIC, typename T, bool PF>
__global__ __launch_bounds__(256) void k_refine_g(RefineArgs a) {
  constexpr int CH = kRfCh;  // (PF loads the next pass's whole rows: valid only for dp <= 64 CH, checked at launch)
  typedef typename RfRaw<T>::type Raw;
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
  const int nB = dp >> 6;  // (PF: nB <= CH)
  const int npass = (a.n_cand + 7) >> 3;
  float mk = INFINITY, tk = INFINITY;  // rank `lane` of the running top-k, and rank k-1
  int64_t mi = LLONG_MAX, ti = LLONG_MAX;
  // candidate row of pass p for this lane's group (-1: none)
  auto cand_of = [&](int p) {
    const int c = 8 * p + j8;
    const int64_t cid = c < a.n_cand ? a.cand[q * a.n_cand + c] : -1;
    return cid >= 0 && cid < a.n ? cid : (int64_t)-1;
  };
  auto load_blocks = [&](int64_t cid, int B0, Raw (&r)[CH]) {
    const T* rowp = data + (cid >= 0 ? cid : 0) * (int64_t)d + 8 * p8;
#pragma unroll
    for (int u = 0; u < CH; ++u) {
      const int dim = 64 * (B0 + u) + 8 * p8;
      if (B0 + u < nB && dim < d) r[u] = rf_raw_ld<T>(rowp + 64 * (B0 + u));
      else r[u] = Raw{};
    }
  };
  // the two chains over blocks B0 .. B0 + CH - 1 (see above), from (dot, xn)
  auto chains = [&](const Raw (&r)[CH], int B0, float& dot, float& xn) {
#pragma unroll
    for (int u = 0; u < CH; ++u) {
      if (B0 + u >= nB) break;
      float v[8];
      rf_raw_cvt<T>(r[u], v);
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
        // the two chains side by side in one v_pk_fma_f32 per dim ((dot, xn) += (x, x) * (y, x): each half of the
        // pair is an fmaf, so the bits are the two separate chains')
        f32x2 acc2 = {dot, xn};
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const f32x2 x0 = {v[jj], v[jj]}, w0 = {yy[jj], v[jj]};
          acc2 = __builtin_elementwise_fma(x0, w0, acc2);
          const f32x2 x1 = {v[4 + jj], v[4 + jj]}, w1 = {yy[4 + jj], v[4 + jj]};
          acc2 = __builtin_elementwise_fma(x1, w1, acc2);
        }
        dot = acc2[0];
        xn = acc2[1];
      }
    }
  };
  // pass p's key -> s_key[(p & 7) * 8 + j8] (lane p8 == 7 ends its group's chains); every 8 passes, or at the end, the
  // 64 keys go through the running top-k by (key, id): K7's ballot insertion, as k_refine
  auto finish_pass = [&](int p, int64_t cid, float dot, float xn) {
    const int slot = (p & 7) * 8 + j8;
    if (p8 == 7) {
      float key = INFINITY;
      int64_t id = LLONG_MAX;
      if (cid >= 0) {
        if (METRIC == kL2) {
          const float t = fmaf(-2.0f, dot, xn + qn);
          key = t > 0.0f ? t : 0.0f;
        } else {
          key = -dot;
        }
        id = a.id_map ? a.id_map[cid] : cid;
      }
      s_key[wv][slot] = key;
      s_id[wv][slot] = id;
    }
    if ((p & 7) != 7 && p + 1 < npass) return;
    wave_lds_sync();
    const int nk_ = ((p & 7) + 1) * 8;  // keys written this round
    const float key = lane < nk_ ? s_key[wv][lane] : INFINITY;
    const int64_t id = lane < nk_ ? s_id[wv][lane] : LLONG_MAX;
    wave_lds_sync();  // (the next round's stores come after every lane's reads)
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
  };
  if constexpr (PF) {
    // two named buffers, passes in pairs: A holds pass p, B pass p + 1 (loaded while A's chains run)
    Raw ra[CH], rb[CH];
    int64_t ca = cand_of(0), cb = -1;
    load_blocks(ca, 0, ra);
    for (int p = 0; p < npass; p += 2) {
      if (p + 1 < npass) {
        cb = cand_of(p + 1);
        load_blocks(cb, 0, rb);
      }
      float dot = 0.0f, xn = 0.0f;
      chains(ra, 0, dot, xn);
      finish_pass(p, ca, dot, xn);
      if (p + 1 >= npass) break;
      if (p + 2 < npass) {
        ca = cand_of(p + 2);
        load_blocks(ca, 0, ra);
      }
      dot = 0.0f;
      xn = 0.0f;
      chains(rb, 0, dot, xn);
      finish_pass(p + 1, cb, dot, xn);
    }
  } else {
    for (int p = 0; p < npass; ++p) {
      const int64_t cid = cand_of(p);
      float dot = 0.0f, xn = 0.0f;
      if (__ballot(cid >= 0) != 0) {  // (a pass with no row: nothing to read)
        for (int B0 = 0; B0 < nB; B0 += CH) {
          Raw r[CH];
          load_blocks(cid, B0, r);
          chains(r, B0, dot, xn);
        }
      }
      finish_pass(p, cid, dot, xn);
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
  // (MIVS_REFINE_GATHER=0: the one-lane-per-row kernel, for A/B runs)
  const bool lane_per_row = engine_setting(kSetRefineGather, "MIVS_REFINE_GATHER", 1) == 0;
  const bool gather = !lane_per_row && (a.d & 7) == 0 && (a.dp & 63) == 0 &&
                      (reinterpret_cast<uintptr_t>(a.data) & 15) == 0;
  if (gather) {
    const bool pf = a.dp <= 64 * kRfCh;  // (fp16 rows: the next pass's CH blocks fit beside the current pass's)
    if (a.half && pf) {
      if (a.metric == kIP) hipLaunchKernelGGL((k_refine_g<kIP, _Float16, true>), grid, dim3(256), 0, s, a);
      else hipLaunchKernelGGL((k_refine_g<kL2, _Float16, true>), grid, dim3(256), 0, s, a);
    } else if (a.half) {
      if (a.metric == kIP) hipLaunchKernelGGL((k_refine_g<kIP, _Float16, false>), grid, dim3(256), 0, s, a);
      else hipLaunchKernelGGL((k_refine_g<kL2, _Float16, false>), grid, dim3(256), 0, s, a);
    } else {
      if (a.metric == kIP) hipLaunchKernelGGL((k_refine_g<kIP, float, false>), grid, dim3(256), 0, s, a);
      else hipLaunchKernelGGL((k_refine_g<kL2, float, false>), grid, dim3(256), 0, s, a);
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
