// K13a — the k-means assign (nearest centroid of every train / data row) on K13's row-stationary loop
// (DESIGN.md §7).
//
// K12 keeps the rows' fp16 vectors as MFMA B operands and streams the centroids through LDS, one ds_read_b128
// per MFMA: at 4 SIMDs x 1 KiB per 16-cycle MFMA that is the LDS's own 256 B/clk, so the assign runs at ~0.2-0.3
// of the fp16 peak. K13a turns it round as K13 does for search: wave w holds 32 rows (all dims) as A operands in
// registers, and the centroids pass in 32-centroid tiles (the 16x16x32 B image of k_rs_tiles, built per
// iteration by k_as_ctiles), one ds_read_b128 per TWO MFMAs. An item is 256 rows x EVERY centroid tile (1024
// centroids: 32 tiles), so the rows are reloaded once per 32 tiles (K13 search: once per ~10).
//
// The result is the pinned fp32 argmin: per row the lanes keep the smallest approximate key, its centroid and
// the second smallest; a row whose second smallest is above the refine window of its smallest has exactly one
// candidate (the true argmin's approximate key is inside that window), any other row (a near
// tie) goes to the exact fp32 K4 scan (the caller's fallback).
#include "mivs_common.hpp"
#include "pf_math.hpp"

namespace mivs {

namespace {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef int v4i __attribute__((ext_vector_type(4)));

constexpr int kAsWaves = 8;
constexpr int kAsThreads = kAsWaves * 64;
constexpr int kAsRows = kAsWaves * 32;  // rows per item

__device__ __forceinline__ v4i as_desc(const void* p, int bytes) {
  const uint64_t v = reinterpret_cast<uint64_t>(p);
  v4i r;
  r.x = (int)__builtin_amdgcn_readfirstlane((uint32_t)v);
  r.y = (int)(__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) & 0xFFFFu);
  r.z = __builtin_amdgcn_readfirstlane(bytes);
  r.w = 0x00020000;
  return r;
}

// LDS-DMA the compiler does not see (as K13's: ordered by the kernel's own counted waits)
__device__ __forceinline__ void as_dma(v4i desc, const void* lds, int voff, int soff) {
  const uint32_t m0 = __builtin_amdgcn_readfirstlane((uint32_t)reinterpret_cast<uintptr_t>(lds));
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
               :: "s"(m0), "v"(voff), "s"(desc), "s"(soff) : "memory");
}

__device__ __forceinline__ void as_wait_vm(int v) {
#define AS_VM(n) ((n & 15) | (0x7 << 4) | ((n >> 4) << 14))
  if (v >= 48) __builtin_amdgcn_s_waitcnt(AS_VM(48));
  else if (v >= 40) __builtin_amdgcn_s_waitcnt(AS_VM(40));
  else if (v >= 32) __builtin_amdgcn_s_waitcnt(AS_VM(32));
  else if (v >= 24) __builtin_amdgcn_s_waitcnt(AS_VM(24));
  else if (v >= 16) __builtin_amdgcn_s_waitcnt(AS_VM(16));
  else if (v >= 8) __builtin_amdgcn_s_waitcnt(AS_VM(8));
  else if (v >= 4) __builtin_amdgcn_s_waitcnt(AS_VM(4));
  else if (v >= 2) __builtin_amdgcn_s_waitcnt(AS_VM(2));
  else if (v >= 1) __builtin_amdgcn_s_waitcnt(AS_VM(1));
  else __builtin_amdgcn_s_waitcnt(AS_VM(0));
#undef AS_VM
}

__device__ __forceinline__ bool as_spin(int* ctr, int target) {
  for (int i = 0; i < (1 << 20); ++i) {
    if (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= target) {
      asm volatile("" ::: "memory");
      return true;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  return false;
}

__device__ __forceinline__ void as_signal(int* ctr) {
  asm volatile("" ::: "memory");
  if (__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)) == 0)
    __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

template <bool B>
struct AsBool {
  static constexpr bool value = B;
};

constexpr int kAsBPrefetch = 2;

// per lane: the running (smallest key, its centroid, second smallest key) of its 8 rows over the centroids it sees
struct AsRun {
  float m1[8], m2[8];
  int id1[8];
};

__device__ __forceinline__ void as_reset(AsRun& r) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    r.m1[j] = INFINITY;
    r.m2[j] = INFINITY;
    r.id1[j] = INT_MAX;
  }
}

template <int NK>
__global__ __launch_bounds__(kAsThreads, 1) void k_as_scan(AsScanArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int BUF = NK * 1024 + 1024;
  constexpr int64_t IMG = (int64_t)(NK + 1) * 1024;
  constexpr int STAGERS = kAsWaves;
  static_assert((NK + STAGERS) / STAGERS < NK, "the image's pieces are issued over k-steps 1..");
  constexpr int ROWS_AFTER = [] {
    int c = 0;
    for (int s = NK / STAGERS + 2; s < NK; ++s) c += (s & 1) ? 2 : 0;
    return c - 2 > 0 ? c - 2 : 0;
  }();
  int* s_ready = reinterpret_cast<int*>(smem + 2 * BUF);
  int* s_next = s_ready + 4;  // [2] the workgroup's next items
  // [2 item parities][waves][32 rows] {qscale, pinned norm} of the rows: 4 ds_read_b128 per tile instead of 16
  // registers per lane
  float* s_meta = reinterpret_cast<float*>(smem + 2 * BUF + 64);
  const int tid = threadIdx.x, lane = tid & 63, kq = lane >> 4, c = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ntl = a.n_ctiles;
  const int64_t n_items = (a.nr + kAsRows - 1) / kAsRows;
  int w = blockIdx.x;
  int tt = 0;  // tiles this wave has started
  if (tid == 0) {
    *s_ready = 0;
    s_next[1] = (int)gridDim.x + atomicAdd(a.queue, 1);  // item 1 of this workgroup
  }
  __syncthreads();
  if (w >= n_items) return;
  // the rows of item wi: lane (c, kq) holds rows 16 rb + c of the wave's 32 (A operand layout); returns the
  // data-row index of row r of the item (-1 past nr)
  auto data_row = [&](int64_t wi, int r) -> int64_t {
    const int64_t ar = wi * kAsRows + 32 * wave + r;
    if (ar >= a.nr) return -1;
    return a.rows ? a.rows[ar] : ar;
  };
  auto row_ptr = [&](int64_t dr) -> const uint16_t* {
    return a.qh + (dr >= 0 ? dr : 0) * (int64_t)(NK * 16) + 8 * kq;
  };
  // per-row meta of item wi into parity p (lanes < 32: row `lane` of the wave)
  auto load_meta = [&](int64_t wi, int p) {
    if (lane < 32) {
      const int64_t dr = data_row(wi, lane);
      const float qs = dr >= 0 ? a.qscale[dr] : 0.0f;
      const float qn = dr >= 0 ? a.qnorms[dr] : INFINITY;  // (an absent row: every key +inf)
      s_meta[((p * kAsWaves + wave) * 2 + 0) * 32 + lane] = qs;
      s_meta[((p * kAsWaves + wave) * 2 + 1) * 32 + lane] = qn;
    }
  };
  const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
  bool spun_out = false;
  // tile 0's pieces
  {
    const v4i d0 = as_desc(a.ctiles, (int)IMG);
#pragma unroll
    for (int p0 = 0; p0 <= NK; p0 += STAGERS)
      if (p0 + wave <= NK) as_dma(d0, smem + (p0 + wave) * 1024, lane * 16, (p0 + wave) * 1024);
  }
  h8 ra[NK];
  {
    const uint16_t* p0 = row_ptr(data_row(w, c));
    const uint16_t* p1 = row_ptr(data_row(w, 16 + c));
#pragma unroll
    for (int s = 0; s < NK; ++s) ra[s] = *reinterpret_cast<const h8*>((s & 1 ? p1 : p0) + 32 * (s >> 1));
  }
  load_meta(w, 0);
  __builtin_amdgcn_s_waitcnt(0x0070);  // vmcnt(0) lgkmcnt(0): tile 0's pieces (and the rows) have landed
  as_signal(s_ready);                  // (signal #0: tile 0 staged)
  int cur = 0, ii = 0;
  const f32x4 zero4 = {0.f, 0.f, 0.f, 0.f};
  AsRun run;
  as_reset(run);
  // the item's closing step: reduce (m1, id1, m2) over the 16 lanes of each kq, then lanes with c == 0 prove or
  // hand over their 8 rows
  auto finish = [&](int64_t wi) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) {
        const float om1 = __shfl_xor(run.m1[j], off), om2 = __shfl_xor(run.m2[j], off);
        const int oid = __shfl_xor(run.id1[j], off);
        const bool take = om1 < run.m1[j] || (om1 == run.m1[j] && oid < run.id1[j]);
        const float hi = take ? run.m1[j] : om1;  // the larger of the two smallest
        run.m2[j] = fminf(fminf(run.m2[j], om2), hi);
        if (take) {
          run.m1[j] = om1;
          run.id1[j] = oid;
        }
      }
    }
    if (c == 0) {
      const float cnm = sqrtf(__uint_as_float(a.cstat[0])) * (1.0f + 0x1p-12f);
      const float crm = __uint_as_float(a.cstat[1]);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int r = 16 * (j >> 2) + 4 * kq + (j & 3);
        const int64_t ar = wi * kAsRows + 32 * wave + r;
        if (ar >= a.nr) continue;
        const int64_t dr = a.rows ? a.rows[ar] : ar;
        const float delta = pf_delta<kL2>(a.qnorms[dr], a.qres[dr], cnm, crm, a.dp);
        const float W = pf_window(run.m1[j], delta);
        if (run.m1[j] < INFINITY && run.m2[j] > W) {
          a.labels[ar] = run.id1[j];
        } else {
          const int at = atomicAdd(a.ovf_count, 1);
          a.ovf_rows[at] = ar;
        }
      }
    }
    as_reset(run);
  };
  for (;;) {
    const int wn = s_next[(ii + 1) & 1];
    const bool has_next = wn < n_items;
    // the next item's first rows (read in the last tile: written with the grabber's signal of this item's tile 0)
    int64_t dn0 = -1, dn1 = -1;
    const float* meta = s_meta + (ii & 1) * kAsWaves * 64 + wave * 64;
    auto tile = [&](int t, auto last_c) __attribute__((always_inline)) {
      constexpr bool LAST = decltype(last_c)::value;
      if (!spun_out && !as_spin(s_ready, kAsWaves * (tt + 1))) spun_out = true;
      ++tt;
      const bool grabber = t == 0 && wave == 0 && lane == 0;
      int grabbed = 0;
      if (grabber) grabbed = (int)gridDim.x + atomicAdd(a.queue, 1);
      if (LAST && has_next) {
        dn0 = data_row(wn, c);
        dn1 = data_row(wn, 16 + c);
      }
      // the next tile: of this item, or the next item's first (every item runs the same centroid tiles)
      const int tn = LAST ? 0 : t + 1;
      const bool stage = (!LAST || has_next) && !(a.flags & 2);
      const v4i sdesc = as_desc(a.ctiles + tn * IMG, stage ? (int)IMG : 0);
      const int nxt = cur ^ 1;
      char* sbuf = smem + nxt * BUF;
      const bool reload = LAST && has_next;
      const uint16_t* np0 = row_ptr(dn0);
      const uint16_t* np1 = row_ptr(dn1);
      f32x4 acc4[4] = {zero4, zero4, zero4, zero4};
      auto kloop = [&](auto reload_c) __attribute__((always_inline)) {
        constexpr bool RL = decltype(reload_c)::value;
        const char* bb = smem + cur * BUF + lane * 16;
        constexpr int PD = kAsBPrefetch;
        h8 b[PD + 1];
#pragma unroll
        for (int u = 0; u < PD; ++u) b[u] = *reinterpret_cast<const h8*>(bb + (u < NK ? u : 0) * 1024);
#pragma unroll
        for (int s = 0; s < NK; ++s) {
          if (s + PD < NK) b[(s + PD) % (PD + 1)] = *reinterpret_cast<const h8*>(bb + (s + PD) * 1024);
          const int t2 = 2 * (s >> 1), qb = s & 1;
          acc4[2 * qb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ra[t2], b[s % (PD + 1)], acc4[2 * qb], 0, 0, 0);
          acc4[2 * qb + 1] =
              __builtin_amdgcn_mfma_f32_16x16x32_f16(ra[t2 + 1], b[s % (PD + 1)], acc4[2 * qb + 1], 0, 0, 0);
          if constexpr (RL) {
            if (s & 1) {
              ra[s - 1] = *reinterpret_cast<const h8*>(np0 + 32 * (s >> 1));
              ra[s] = *reinterpret_cast<const h8*>(np1 + 32 * (s >> 1));
            }
          }
          if (s >= 1 && (s - 1) * STAGERS <= NK) {
            const int p = min((s - 1) * STAGERS + wave, NK);
            as_dma(sdesc, sbuf + p * 1024, lane * 16, p * 1024);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      };
      if (LAST && reload) kloop(AsBool<true>{});
      else kloop(AsBool<false>{});
      // the tile's centroid headers {pinned norm, index} for centroids c and 16 + c, and the rows' meta
      const float4 hq0 = *reinterpret_cast<const float4*>(smem + cur * BUF + NK * 1024 + c * 16);
      const float4 hq1 = *reinterpret_cast<const float4*>(smem + cur * BUF + NK * 1024 + (16 + c) * 16);
      const float4 qs0 = *reinterpret_cast<const float4*>(meta + 4 * kq);
      const float4 qs1 = *reinterpret_cast<const float4*>(meta + 16 + 4 * kq);
      const float4 qn0 = *reinterpret_cast<const float4*>(meta + 32 + 4 * kq);
      const float4 qn1 = *reinterpret_cast<const float4*>(meta + 48 + 4 * kq);
      as_wait_vm(reload ? ROWS_AFTER : 0);
      if (grabber) s_next[ii & 1] = grabbed;  // (read in the next item's last tile)
      as_signal(s_ready);
      // the epilogue: 16 approximate keys (8 rows x 2 centroids) into the running minima, branch-free.
      // key = max(fl(fl(cn + qn) - 2 acc qs), 0) is pf_key's value: -2 qs is a power of two, so
      // fma(acc, -2 qs, s) rounds once as fma(-2, acc qs, s) does
      const float qsv[8] = {qs0.x, qs0.y, qs0.z, qs0.w, qs1.x, qs1.y, qs1.z, qs1.w};
      const float qnv[8] = {qn0.x, qn0.y, qn0.z, qn0.w, qn1.x, qn1.y, qn1.z, qn1.w};
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) {
        const float4 h = qb ? hq1 : hq0;
        const int cid = __float_as_int(h.y);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float t = fmaf(acc4[2 * qb + (j >> 2)][j & 3], -2.0f * qsv[j], h.x + qnv[j]);
          const float key = t > 0.0f ? t : 0.0f;
          // (m1 <= m2: the new second smallest is the median of {m1, key, m2} -- one v_med3 for the select and
          // the min of the two-way form)
          run.m2[j] = __builtin_amdgcn_fmed3f(run.m1[j], key, run.m2[j]);
          run.id1[j] = key < run.m1[j] ? cid : run.id1[j];
          run.m1[j] = fminf(run.m1[j], key);
        }
      }
      cur = nxt;
    };
    for (int t = 0; t + 1 < ntl; ++t) tile(t, AsBool<false>{});
    tile(ntl - 1, AsBool<true>{});
    finish(w);
    if (!has_next) break;
    // the next item's meta, in the other parity (its rows are in flight since the last tile)
    load_meta(wn, (ii + 1) & 1);
    ++ii;
    w = wn;
  }
  if (spun_out && lane == 0) atomicOr(a.ovf_count + 1, 1);  // (never expected: the caller then reruns exactly)
  (void)t_start;
}

// the centroid tile images: tile t = centroids 32 t .. 32 t + 31 (group t of the single-list ListSet), piece
// s = 2 u + qb: lane (c, kq) = dims 32 u + 8 kq .. + 8 of centroid 16 qb + c, fp16 at the data's scale 2^hx (the
// K12 assign's), header piece: lanes j, j + 32 = {pinned norm, index as int bits} of centroid j. stat[0] =
// max pinned norm, stat[1] = max ||c - c_h 2^-hx|| (both as ordered float bits, non-negative)
__global__ __launch_bounds__(256) void k_as_ctiles(const float* __restrict__ groups, const float* __restrict__ norms,
                                                   int64_t n_groups, int dp, int hx, char* __restrict__ tiles,
                                                   unsigned* __restrict__ stat) {
  const int nk = dp / 16;
  const int64_t img = (int64_t)(nk + 1) * 1024;
  const int64_t t = blockIdx.x;  // one block per tile (group)
  if (t >= n_groups) return;
  const float sc = ldexpf(1.0f, hx), isc = ldexpf(1.0f, -hx);
  char* base = tiles + t * img;
  __shared__ float s_res[32];
  if (threadIdx.x < 32) s_res[threadIdx.x] = 0.0f;
  __syncthreads();
  for (int i = threadIdx.x; i < nk * 64; i += blockDim.x) {
    const int s = i >> 6, L = i & 63;
    const int cj = 16 * (s & 1) + (L & 15);  // centroid within the tile
    const int b = 4 * (s >> 1) + (L >> 4);   // 8-dim block: dims 32 (s >> 1) + 8 kq
    const float* src = groups + row_elem(t * kGroupRows + cj, 0, dp) + row_blk8(b);
    const float4 v0 = *reinterpret_cast<const float4*>(src), v1 = *reinterpret_cast<const float4*>(src + 4);
    const float v[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
    _Float16 hv[8];
    float res = 0.0f;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      _Float16 h = (_Float16)(v[e] * sc);
      if (fabsf((float)h) < 0x1p-14f) h = (_Float16)0.0f;  // no fp16 subnormals reach the MFMA
      const float r = v[e] - (float)h * isc;                // exact
      res = fmaf(r, r, res);
      hv[e] = h;
    }
    *reinterpret_cast<uint4*>(base + s * 1024 + L * 16) = __builtin_bit_cast(uint4, hv);
    atomicAdd(&s_res[cj], res);  // (order irrelevant: a bound, padded below)
  }
  __syncthreads();
  if (threadIdx.x < 64) {
    const int j = threadIdx.x & 31;
    const float n = norms[t * kGroupRows + j];
    *reinterpret_cast<float4*>(base + (int64_t)nk * 1024 + threadIdx.x * 16) =
        make_float4(n, __int_as_float((int)(t * kGroupRows + j)), 0.0f, 0.0f);
    if (threadIdx.x < 32 && n < INFINITY) {
      atomicMax(stat, __float_as_uint(n));
      // every term of the residual sum is exact; the sum's roundings are covered by a relative pad
      atomicMax(stat + 1, __float_as_uint(sqrtf(s_res[j]) * (1.0f + 0x1p-10f)));
    }
  }
}

}  // namespace

bool as_scan_supported(int dp, int64_t n_centroids) {
  return dp % 64 == 0 && dp >= 128 && dp <= 768 && n_centroids > 32;
}

size_t as_ctiles_bytes(int64_t n_groups, int dp) { return (size_t)n_groups * (size_t)(dp / 16 + 1) * 1024; }

hipError_t launch_as_ctiles(const float* groups, const float* norms, int64_t n_groups, int dp, int hx, char* tiles,
                            unsigned* stat, hipStream_t s) {
  if (n_groups <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_as_ctiles, dim3((unsigned)n_groups), dim3(256), 0, s, groups, norms, n_groups, dp, hx, tiles, stat);
  return hipGetLastError();
}

template <int NK>
static hipError_t launch_as_k(const AsScanArgs& a, int grid, hipStream_t s) {
  const size_t lds = (size_t)2 * (NK * 1024 + 1024) + 64 + 2 * kAsWaves * 64 * sizeof(float);
  static const hipError_t attr =
      hipFuncSetAttribute((const void*)k_as_scan<NK>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (attr != hipSuccess) return attr;
  hipLaunchKernelGGL((k_as_scan<NK>), dim3(grid), dim3(kAsThreads), lds, s, a);
  return hipGetLastError();
}

hipError_t launch_as_scan(const AsScanArgs& a, int grid, hipStream_t s) {
  if (!as_scan_supported(a.dp, (int64_t)a.n_ctiles * 32) || grid < 1) return hipErrorInvalidValue;
  switch (a.dp / 16) {
    case 8: return launch_as_k<8>(a, grid, s);
    case 12: return launch_as_k<12>(a, grid, s);
    case 16: return launch_as_k<16>(a, grid, s);
    case 20: return launch_as_k<20>(a, grid, s);
    case 24: return launch_as_k<24>(a, grid, s);
    case 28: return launch_as_k<28>(a, grid, s);
    case 32: return launch_as_k<32>(a, grid, s);
    case 36: return launch_as_k<36>(a, grid, s);
    case 40: return launch_as_k<40>(a, grid, s);
    case 44: return launch_as_k<44>(a, grid, s);
    case 48: return launch_as_k<48>(a, grid, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace mivs
