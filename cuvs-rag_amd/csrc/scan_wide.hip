// K3w — the fine list scan with 64-query tiles (DESIGN.md §"Kernels").
//
// Same job, same arithmetic and same output as K3 (scan.hip), but every list
// row streamed from HBM feeds TWO 32x32 MFMA column tiles (64 queries), which
// halves the HBM bytes per flop: at the fp32 MFMA peak K3 would need ~9.8 TB/s,
// K3w ~4.9 TB/s, below the HBM roofline.
//
// A 64-query tile of fp32 rows does not fit LDS next to anything else at d=768
// (197 KB), so the queries are staged in 128-dim SLABS (double-buffered, 2 x 33 KB):
//   for each pass of 8 row groups (one per wave):
//     for each slab s (16 k-steps = register blocks A and B):
//       issue the global loads of the next query slab;
//       A: 8 k-steps x (2 tiles x 4 MFMA), refill A for the next step; the same for B;
//       write the next slab to LDS; barrier
//     epilogue: dot tiles -> keys -> per-lane register top-K (one list per tile)
//   merge the 16 lane lists of each query in LDS (two rounds of 32 queries).
// The k-order of every dot is the K3 order (slab-major = k-step-major), so results
// are bit-identical to K3 and to the oracle.
#include <climits>

#include "mivs_common.hpp"

namespace mivs {

namespace {

constexpr int kWQ = 64;             // queries per tile
constexpr int kSlab = 128;          // dims per staged query slab = one step (16 k-steps: blocks A and B)
constexpr int kSld = kSlab + 4;     // LDS row stride of a slab (floats); = 4 mod 64 banks
constexpr int kPassG = kScanWaves;  // 8 groups per pass (one per wave)
constexpr int kWSmall = 64 * 8 + 64 * 8 + 64 * 4 + 16;  // s_q, s_slot, s_qn, s_misc

template <int KCAP>
__device__ __forceinline__ void wlane_insert(float (&lk)[KCAP], int (&lp)[KCAP], float key, int pos) {
#pragma unroll
  for (int t = KCAP - 1; t >= 0; --t) {
    const float prev = t > 0 ? lk[t > 0 ? t - 1 : 0] : -INFINITY;
    const int prevp = t > 0 ? lp[t > 0 ? t - 1 : 0] : 0;
    const bool shift = key < prev;
    const bool place = !shift && key < lk[t];
    lk[t] = shift ? prev : (place ? key : lk[t]);
    lp[t] = shift ? prevp : (place ? pos : lp[t]);
  }
}

template <int KCAP, int METRIC>
__device__ __forceinline__ void wepilogue(const f32x16& acc, const float* __restrict__ gnorm, int64_t rbase, int h,
                                          float qn, bool qvalid, float (&lk)[KCAP], int (&lp)[KCAP]) {
  float xn[16];
#pragma unroll
  for (int q4 = 0; q4 < 4; ++q4) {
    const float4 t = *reinterpret_cast<const float4*>(gnorm + 8 * q4 + 4 * h);
    xn[4 * q4 + 0] = t.x; xn[4 * q4 + 1] = t.y; xn[4 * q4 + 2] = t.z; xn[4 * q4 + 3] = t.w;
  }
  if (!qvalid) return;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    float key;
    if (METRIC == kL2) {
      const float v = fmaf(-2.0f, acc[r], xn[r] + qn);
      key = v > 0.0f ? v : 0.0f;
    } else {
      key = xn[r] < INFINITY ? -acc[r] : INFINITY;
    }
    if (key < lk[KCAP - 1]) wlane_insert<KCAP>(lk, lp, key, (int)(rbase + (r & 3) + 8 * (r >> 2) + 4 * h));
  }
}

// 8 k-steps (half a slab) of one row group against both query tiles of the slab in LDS
__device__ __forceinline__ void mma8(f32x16& c0, f32x16& c1, const float4 (&v)[8], const float* __restrict__ q0,
                                     const float* __restrict__ q1) {
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const float4 b0 = *reinterpret_cast<const float4*>(q0 + u * 8);
    const float4 b1 = *reinterpret_cast<const float4*>(q1 + u * 8);
    c0 = __builtin_amdgcn_mfma_f32_32x32x2f32(v[u].x, b0.x, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_32x32x2f32(v[u].x, b1.x, c1, 0, 0, 0);
    c0 = __builtin_amdgcn_mfma_f32_32x32x2f32(v[u].y, b0.y, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_32x32x2f32(v[u].y, b1.y, c1, 0, 0, 0);
    c0 = __builtin_amdgcn_mfma_f32_32x32x2f32(v[u].z, b0.z, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_32x32x2f32(v[u].z, b1.z, c1, 0, 0, 0);
    c0 = __builtin_amdgcn_mfma_f32_32x32x2f32(v[u].w, b0.w, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_32x32x2f32(v[u].w, b1.w, c1, 0, 0, 0);
  }
}

__device__ __forceinline__ void load8(float4 (&v)[8], const float* __restrict__ p) {
#pragma unroll
  for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const float4*>(p + u * 256);
}

template <int KCAP, int METRIC>
__global__ __launch_bounds__(kScanThreads, 1) void k_scan_wide(ScanArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int64_t* s_q = reinterpret_cast<int64_t*>(smem);       // [64] query row ids (-1: empty)
  int64_t* s_slot = s_q + kWQ;                            // [64] output slot (already + chunk)
  float* s_qn = reinterpret_cast<float*>(s_slot + kWQ);   // [64]
  int* s_misc = reinterpret_cast<int*>(s_qn + kWQ);       // [4]
  float* s_norm = reinterpret_cast<float*>(smem + kWSmall);  // [G*32]
  float* qs = s_norm + a.chunk_groups * kGroupRows;       // [2][64][kSld]; merge area after the scan
  float* mkey = qs;
  int* mpos = reinterpret_cast<int*>(mkey + 32 * 16 * KCAP);

  const int dp = a.dp;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int j = lane & 31;
  const int h = lane >> 5;
  const int total = a.work_off[a.n_lists];
  const int64_t gstride = (int64_t)kGroupRows * dp;  // floats per group

  for (;;) {
    if (tid == 0) s_misc[0] = atomicAdd(a.work_counter, 1);
    __syncthreads();
    const int w = s_misc[0];
    if (w >= total) break;

    int lo = 0, hi = a.n_lists - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (a.work_off[mid] <= w) lo = mid; else hi = mid - 1;
    }
    const int l = lo;
    const int m = a.bucket_off[l + 1] - a.bucket_off[l];
    const int tiles = (m + kWQ - 1) / kWQ;
    const int local = w - a.work_off[l];
    const int chunk = local / tiles;
    const int tile = local - chunk * tiles;
    const int64_t g_begin = a.list_goff[l] + (int64_t)chunk * a.chunk_groups;
    const int64_t g_lim = a.list_goff[l + 1];
    const int64_t g_end = g_begin + a.chunk_groups < g_lim ? g_begin + a.chunk_groups : g_lim;
    const int e0 = a.bucket_off[l] + tile * kWQ;
    const int nqt = m - tile * kWQ < kWQ ? m - tile * kWQ : kWQ;

    if (tid < kWQ) {
      if (tid < nqt) {
        const int64_t q = a.bucket_q[e0 + tid];
        s_q[tid] = q;
        s_slot[tid] = a.bucket_slot[e0 + tid] + chunk;
        s_qn[tid] = a.qnorms[q];
      } else {
        s_q[tid] = -1;
        s_slot[tid] = -1;
        s_qn[tid] = INFINITY;
      }
    }
    {
      const int nn = (int)(g_end - g_begin) * kGroupRows;
      for (int i = tid; i < nn; i += kScanThreads) s_norm[i] = a.row_norms[g_begin * kGroupRows + i];
    }
    __syncthreads();

    float lk0[KCAP], lk1[KCAP];
    int lp0[KCAP], lp1[KCAP];
#pragma unroll
    for (int t = 0; t < KCAP; ++t) { lk0[t] = INFINITY; lp0[t] = INT_MAX; lk1[t] = INFINITY; lp1[t] = INT_MAX; }
    const float qn0 = s_qn[j], qn1 = s_qn[32 + j];
    const bool qv0 = s_q[j] >= 0, qv1 = s_q[32 + j] >= 0;

    // slab staging: the 64 x 128 slab is 2048 float4s, thread tid owns float4s tid + 512 i (i < 4):
    // query row (tid >> 5) + 16 i, dims ((tid & 31) << 2) .. + 3
    const int sr = tid >> 5;
    const int sc = (tid & 31) << 2;
    const int64_t sq0 = s_q[sr], sq1 = s_q[sr + 16], sq2 = s_q[sr + 32], sq3 = s_q[sr + 48];
    // per staged float4: source offset (floats) into a.queries and a validity mask; an invalid
    // query lane reads query row 0 (always mapped) and is zeroed by the mask: the staging loads are
    // branch- and select-free, so no VMEM wait is forced inside the step loop (d % 4 == 0 required)
    const int64_t so0 = sq0 >= 0 ? sq0 * (int64_t)a.d : 0, so1 = sq1 >= 0 ? sq1 * (int64_t)a.d : 0;
    const int64_t so2 = sq2 >= 0 ? sq2 * (int64_t)a.d : 0, so3 = sq3 >= 0 ? sq3 * (int64_t)a.d : 0;
    auto stage_one = [&](int64_t off, bool qok, int c) {
      const bool ok = qok && c < a.d;
      const uint32_t m = ok ? 0xFFFFFFFFu : 0u;
      const float4 t = *reinterpret_cast<const float4*>(a.queries + (ok ? off + c : 0));
      return make_float4(__uint_as_float(__float_as_uint(t.x) & m), __uint_as_float(__float_as_uint(t.y) & m),
                         __uint_as_float(__float_as_uint(t.z) & m), __uint_as_float(__float_as_uint(t.w) & m));
    };
#define MIVS_STAGE_LOAD(S, V0, V1, V2, V3)            \
  do {                                                \
    const int c_ = (S) * kSlab + sc;                  \
    V0 = stage_one(so0, sq0 >= 0, c_);                \
    V1 = stage_one(so1, sq1 >= 0, c_);                \
    V2 = stage_one(so2, sq2 >= 0, c_);                \
    V3 = stage_one(so3, sq3 >= 0, c_);                \
  } while (0)
#define MIVS_STAGE_STORE(BUF, V0, V1, V2, V3)                                   \
  do {                                                                        \
    float* b_ = qs + (BUF) * (kWQ * kSld) + sr * kSld + sc;                   \
    *reinterpret_cast<float4*>(b_) = V0;                                      \
    *reinterpret_cast<float4*>(b_ + 16 * kSld) = V1;                          \
    *reinterpret_cast<float4*>(b_ + 32 * kSld) = V2;                          \
    *reinterpret_cast<float4*>(b_ + 48 * kSld) = V3;                          \
  } while (0)

    // ONE stream of (pass, slab) steps: pass = one group per wave, slab = 16 k-steps = register
    // blocks A (k-steps 0-7) and B (8-15). The loads of step t+1 (both blocks + the next query slab)
    // are issued during step t, across pass boundaries too; past the end the current blocks are
    // re-read (L2 hits, never consumed).
    const int ns = dp / kSlab;
    const int npass = (int)((g_end - g_begin + kPassG - 1) / kPassG);
    const int nsteps = npass * ns;
    auto grp_ptr = [&](int pass) {
      const int64_t g = g_begin + pass * kPassG + wave;
      return a.groups + (g < g_end ? g : g_begin) * gstride + j * 8 + 4 * h;
    };
    float4 A[8], B[8];
    {
      float4 v0, v1, v2, v3;
      MIVS_STAGE_LOAD(0, v0, v1, v2, v3);
      MIVS_STAGE_STORE(0, v0, v1, v2, v3);
      // same issue order as the loop body (all of A, then all of B): the wait counts the loop head
      // inherits from this path then match the steady state
      __builtin_amdgcn_sched_barrier(0);
      load8(A, grp_ptr(0));
      __builtin_amdgcn_sched_barrier(0);
      load8(B, grp_ptr(0) + 8 * 256);
      __builtin_amdgcn_sched_barrier(0);
    }
    __syncthreads();
    f32x16 c0 = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const f32x16 zero = c0;
    f32x16 c1 = c0;
    int p = 0, s = 0;
    for (int t = 0; t < nsteps; ++t) {
      const int tn = t + 1 < nsteps ? t + 1 : t;
      const int pn = tn / ns, sn = tn - pn * ns;
      float4 n0, n1, n2, n3;
      MIVS_STAGE_LOAD(sn, n0, n1, n2, n3);
      const float* qb = qs + (t & 1) * (kWQ * kSld) + 4 * h;
      const float* q0 = qb + j * kSld;
      const float* q1 = qb + (32 + j) * kSld;
      const float* pnext = grp_ptr(pn) + sn * (16 * 256);
      // sched_barrier: keep each refill right behind the MFMAs that free its registers, so a full
      // block of MFMAs (64) covers it; left alone the scheduler sinks both refills to the step end
      mma8(c0, c1, A, q0, q1);
      __builtin_amdgcn_sched_barrier(0);
      load8(A, pnext);
      __builtin_amdgcn_sched_barrier(0);
      mma8(c0, c1, B, q0 + 64, q1 + 64);
      __builtin_amdgcn_sched_barrier(0);
      load8(B, pnext + 8 * 256);
      __builtin_amdgcn_sched_barrier(0);
      if (t + 1 < nsteps) MIVS_STAGE_STORE((t + 1) & 1, n0, n1, n2, n3);
      __syncthreads();
      if (s == ns - 1) {  // pass p complete: keys -> lane lists
        const int64_t g = g_begin + p * kPassG + wave;
        if (g < g_end) {
          const float* gn = s_norm + (g - g_begin) * kGroupRows;
          wepilogue<KCAP, METRIC>(c0, gn, g * kGroupRows, h, qn0, qv0, lk0, lp0);
          wepilogue<KCAP, METRIC>(c1, gn, g * kGroupRows, h, qn1, qv1, lk1, lp1);
        }
        c0 = zero;
        c1 = zero;
        s = 0;
        ++p;
      } else {
        ++s;
      }
    }

#undef MIVS_STAGE_LOAD
#undef MIVS_STAGE_STORE
    // ---- merge: two rounds of 32 queries, 16 lane lists (8 waves x 2 halves) per query ----
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      __syncthreads();  // slab buffers / previous round done
      {
        const int src = wave * 2 + h;
#pragma unroll
        for (int i = 0; i < KCAP; ++i) {
          mkey[(j * 16 + src) * KCAP + i] = t == 0 ? lk0[i] : lk1[i];
          mpos[(j * 16 + src) * KCAP + i] = t == 0 ? lp0[i] : lp1[i];
        }
      }
      __syncthreads();
      const int jj = tid >> 4;
      const int ss = tid & 15;
      const float* myk = mkey + (jj * 16 + ss) * KCAP;
      const int* myp = mpos + (jj * 16 + ss) * KCAP;
      const int64_t slot = s_slot[t * 32 + jj];
      int head = 0;
      float hk = myk[0];
      int hp = myp[0];
      for (int r = 0; r < a.k; ++r) {
        float bk = hk;
        int bp = hp;
#pragma unroll
        for (int off = 8; off >= 1; off >>= 1) {
          const float ok = __shfl_xor(bk, off, 16);
          const int op = __shfl_xor(bp, off, 16);
          if (ok < bk || (ok == bk && op < bp)) { bk = ok; bp = op; }
        }
        if (ss == 0 && slot >= 0) {
          const bool valid = bp != INT_MAX;
          a.out_d[slot * a.k + r] = valid ? (METRIC == kIP ? -bk : bk) : (METRIC == kIP ? -INFINITY : INFINITY);
          a.out_i[slot * a.k + r] = valid ? a.row_ids[bp] : (int64_t)-1;
        }
        if (hk == bk && hp == bp && head < KCAP) {
          ++head;
          hk = head < KCAP ? myk[head] : INFINITY;
          hp = head < KCAP ? myp[head] : INT_MAX;
        }
      }
    }
    __syncthreads();
  }
}

template <int KCAP, int METRIC>
hipError_t launch_wm(const ScanArgs& a, int grid, size_t lds, hipStream_t s) {
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_scan_wide<KCAP, METRIC>),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  if (attr != hipSuccess) return attr;
  hipLaunchKernelGGL((k_scan_wide<KCAP, METRIC>), dim3(grid), dim3(kScanThreads), lds, s, a);
  return hipGetLastError();
}

template <int KCAP>
hipError_t launch_w(const ScanArgs& a, int grid, size_t lds, hipStream_t s) {
  return a.metric == kIP ? launch_wm<KCAP, kIP>(a, grid, lds, s) : launch_wm<KCAP, kL2>(a, grid, lds, s);
}

}  // namespace

size_t scan_wide_lds_bytes(int kcap, int chunk_groups) {
  const size_t slabs = (size_t)2 * kWQ * kSld * 4;
  const size_t merge = (size_t)32 * 16 * kcap * 8;
  return kWSmall + (size_t)chunk_groups * kGroupRows * 4 + (slabs > merge ? slabs : merge);
}

bool scan_wide_supported(int kcap, int d, int dp, int chunk_groups) {
  return (kcap == 1 || kcap == 4 || kcap == 8 || kcap == 16) && d % 4 == 0 && dp % kSlab == 0 &&
         scan_wide_lds_bytes(kcap, chunk_groups) <= 160 * 1024;
}

template <int KCAP, int METRIC>
static int wocc_km(size_t lds) {
  int n = 0;
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_scan_wide<KCAP, METRIC>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, reinterpret_cast<const void*>(&k_scan_wide<KCAP, METRIC>),
                                                   kScanThreads, lds) != hipSuccess)
    return 1;
  return n > 0 ? n : 1;
}

template <int KCAP>
static int wocc_k(int metric, size_t lds) { return metric == kIP ? wocc_km<KCAP, kIP>(lds) : wocc_km<KCAP, kL2>(lds); }

int scan_wide_occupancy(int kcap, int metric, size_t lds) {
  switch (kcap) {
    case 1: return wocc_k<1>(metric, lds);
    case 4: return wocc_k<4>(metric, lds);
    case 8: return wocc_k<8>(metric, lds);
    case 16: return wocc_k<16>(metric, lds);
    default: return 1;
  }
}

hipError_t launch_scan_wide(const ScanArgs& a, int kcap, int grid, size_t lds, hipStream_t s) {
  switch (kcap) {
    case 1: return launch_w<1>(a, grid, lds, s);
    case 4: return launch_w<4>(a, grid, lds, s);
    case 8: return launch_w<8>(a, grid, lds, s);
    case 16: return launch_w<16>(a, grid, lds, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace mivs
