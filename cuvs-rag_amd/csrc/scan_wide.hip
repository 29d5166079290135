// K3w — the fine list scan with 64-query tiles.
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

// 8 k-steps of one row group against both query tiles, each k-step's A register refilled from
// `next` right after its 8 MFMAs. The sched_group_barriers pin the per-k-step issue pattern
// (8 MFMA, 1 VMEM, 2 DS): one wide load per 8 MFMAs keeps the stream in flight without ever
// stalling the two accumulator chains (tools/mfma_probe.hip P7: 96 % of the fp32 MFMA peak).
template <int U0, int U1>
__device__ __forceinline__ void mma8_refill(f32x16& c0, f32x16& c1, float4 (&v)[8], const float* __restrict__ q0,
                                            const float* __restrict__ q1, const float* __restrict__ next) {
#pragma unroll
  for (int u = U0; u < U1; ++u) {
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
    v[u] = *reinterpret_cast<const float4*>(next + row_blk8(u));
    __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);  // MFMA
    __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // VMEM read
    __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);  // DS read
  }
}

// DUMP mode (KCAP == 0): the group's keys of one query tile straight to the query's slot (K3's epilogue_dump; rows
// 8 r4 + 4 h + 0..3 of this lane are contiguous: 4 dwordx4 stores)
template <int METRIC>
__device__ __forceinline__ void wepilogue_dump(const f32x16& acc, const float* __restrict__ gnorm, int h, float qn,
                                               float* __restrict__ dst) {
  if (dst == nullptr) return;
#pragma unroll
  for (int r4 = 0; r4 < 4; ++r4) {
    const float4 xn = *reinterpret_cast<const float4*>(gnorm + 8 * r4 + 4 * h);
    const float xs[4] = {xn.x, xn.y, xn.z, xn.w};
    float kv[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (METRIC == kL2) {
        const float v = fmaf(-2.0f, acc[4 * r4 + i], xs[i] + qn);
        kv[i] = v > 0.0f ? v : 0.0f;
      } else {
        kv[i] = xs[i] < INFINITY ? -acc[4 * r4 + i] : INFINITY;
      }
    }
    *reinterpret_cast<float4*>(dst + 8 * r4 + 4 * h) = make_float4(kv[0], kv[1], kv[2], kv[3]);
  }
}

__device__ __forceinline__ void load8(float4 (&v)[8], const float* __restrict__ p) {
#pragma unroll
  for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const float4*>(p + row_blk8(u));
}

// W waves per workgroup (4: two workgroups per CU interleave their barriers / merges on every
// SIMD; 8: one workgroup per CU). A pass covers W row groups, one per wave.
template <int KCAP, int METRIC, int W>
__global__ __launch_bounds__(W * 64, 1) void k_scan_wide(ScanArgs a) {
  constexpr bool DUMP = KCAP == 0;     // every key to the query's slot (the coarse probe: K8 selects)
  constexpr int KR = DUMP ? 1 : KCAP;  // register list length
  constexpr int NT = W * 64;
  constexpr int NS = 2 * W;          // lane lists per query (W waves x 2 halves)
  constexpr int SPT = 2048 / NT;     // staged float4s per thread per slab (64 queries x 128 dims)
  constexpr int RS = NT / 32;        // query rows covered per staging sub-pass
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int64_t* s_q = reinterpret_cast<int64_t*>(smem);       // [64] query row ids (-1: empty)
  int64_t* s_slot = s_q + kWQ;                            // [64] output slot (already + chunk)
  float* s_qn = reinterpret_cast<float*>(s_slot + kWQ);   // [64]
  int* s_misc = reinterpret_cast<int*>(s_qn + kWQ);       // [4]
  float* s_norm = reinterpret_cast<float*>(smem + kWSmall);  // [G*32]
  float* qs = s_norm + a.chunk_groups * kGroupRows;       // [2][64][kSld]; merge area after the scan
  float* mkey = qs;
  int* mpos = reinterpret_cast<int*>(mkey + 32 * NS * KR);

  const int dp = a.dp;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int j = lane & 31;
  const int h = lane >> 5;
  const int total = a.work_off[a.n_lists];
  const int64_t gstride = (int64_t)kGroupRows * dp;  // floats per group
  const int ns = dp / kSlab;
  const int sr = tid >> 5;          // staging: query row (+ RS i) and dim offset within the slab
  const int sc = (tid & 31) << 2;

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
      for (int i = tid; i < nn; i += NT) s_norm[i] = a.row_norms[g_begin * kGroupRows + i];
      if (DUMP && tid < nqt) {  // slot header: first row position + rows of this chunk
        const int64_t slot = a.bucket_slot[e0 + tid] + chunk;
        a.out_i[2 * slot] = g_begin * kGroupRows;
        a.out_i[2 * slot + 1] = nn;
      }
    }
    __syncthreads();

    float lk0[KR], lk1[KR];
    int lp0[KR], lp1[KR];
#pragma unroll
    for (int t = 0; t < KR; ++t) { lk0[t] = INFINITY; lp0[t] = INT_MAX; lk1[t] = INFINITY; lp1[t] = INT_MAX; }
    const float qn0 = s_qn[j], qn1 = s_qn[32 + j];
    const bool qv0 = s_q[j] >= 0, qv1 = s_q[32 + j] >= 0;
    const int slot_rows = a.chunk_groups * kGroupRows;
    float* const dump0 = DUMP && qv0 ? a.out_d + s_slot[j] * (int64_t)slot_rows : nullptr;
    float* const dump1 = DUMP && qv1 ? a.out_d + s_slot[32 + j] * (int64_t)slot_rows : nullptr;

    // query-slab staging: staged float4 i of this thread = query row sr + RS i (int32 row id kept,
    // -1: empty lane), dims slab * 128 + sc .. + 3. An invalid float4 reads query row 0 (always
    // mapped) and is zeroed by a mask: the loads are branch- and select-free (d % 4 == 0 required).
    // Slabs are staged in two halves of SPT / 2 float4s to keep the in-flight registers low.
    int sq[SPT];
#pragma unroll
    for (int i = 0; i < SPT; ++i) sq[i] = (int)s_q[sr + RS * i];
    auto stage_load = [&](int slab, int half, float4 (&v)[SPT / 2]) {
      const int c = slab * kSlab + sc;
#pragma unroll
      for (int i = 0; i < SPT / 2; ++i) {
        const int qi = sq[half * (SPT / 2) + i];
        const uint32_t m2 = (qi >= 0 && c < a.d) ? 0xFFFFFFFFu : 0u;
        const float4 t = *reinterpret_cast<const float4*>(a.queries + (m2 ? (int64_t)qi * a.d + c : 0));
        v[i] = make_float4(__uint_as_float(__float_as_uint(t.x) & m2), __uint_as_float(__float_as_uint(t.y) & m2),
                           __uint_as_float(__float_as_uint(t.z) & m2), __uint_as_float(__float_as_uint(t.w) & m2));
      }
    };
    auto stage_store = [&](int buf, int half, const float4 (&v)[SPT / 2]) {
      float* b = qs + buf * (kWQ * kSld) + (sr + RS * half * (SPT / 2)) * kSld + sc;
#pragma unroll
      for (int i = 0; i < SPT / 2; ++i) *reinterpret_cast<float4*>(b + RS * i * kSld) = v[i];
    };

    // ONE stream of (pass, slab) steps: pass = one group per wave, slab = 16 k-steps = register
    // blocks A (k-steps 0-7) and B (8-15). The loads of step t+1 (both blocks + the next query slab)
    // are issued during step t, across pass boundaries too; past the end the current blocks are
    // re-read (L2 hits, never consumed).
    const int npass = (int)((g_end - g_begin + W - 1) / W);
    const int nsteps = npass * ns;
    auto grp_ptr = [&](int pass) {
      const int64_t g = g_begin + pass * W + wave;
      return a.groups + (g < g_end ? g : g_begin) * gstride + j * kRowBlk + 4 * h;
    };
    float4 A[8], B[8];
    {
      float4 v[SPT / 2];
      stage_load(0, 0, v);
      stage_store(0, 0, v);
      stage_load(0, 1, v);
      stage_store(0, 1, v);
      // same issue order as the loop body (all of A, then all of B)
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
      const float* qb = qs + (t & 1) * (kWQ * kSld) + 4 * h;
      const float* q0 = qb + j * kSld;
      const float* q1 = qb + (32 + j) * kSld;
      const float* pnext = grp_ptr(pn) + sn * (16 * 256);
      // issue order per step: A block (8 x [8 MFMA, 1 refill]), slab half 0 loads, B k-steps 0-3,
      // slab half 0 stores + half 1 loads, B k-steps 4-7, slab half 1 stores. sched_barriers keep
      // the slab loads out of the refill slots.
      const bool stage = t + 1 < nsteps;
      const int nb = (t + 1) & 1;
      float4 nv[SPT / 2];
      __builtin_amdgcn_sched_barrier(0);
      mma8_refill<0, 8>(c0, c1, A, q0, q1, pnext);
      __builtin_amdgcn_sched_barrier(0);
      stage_load(sn, 0, nv);
      __builtin_amdgcn_sched_barrier(0);
      mma8_refill<0, 4>(c0, c1, B, q0 + 64, q1 + 64, pnext + 8 * 256);
      __builtin_amdgcn_sched_barrier(0);
      if (stage) stage_store(nb, 0, nv);
      stage_load(sn, 1, nv);
      __builtin_amdgcn_sched_barrier(0);
      mma8_refill<4, 8>(c0, c1, B, q0 + 64, q1 + 64, pnext + 8 * 256);
      __builtin_amdgcn_sched_barrier(0);
      if (stage) stage_store(nb, 1, nv);
      __syncthreads();
      if (s == ns - 1) {  // pass p complete: keys -> lane lists
        const int64_t g = g_begin + p * W + wave;
        if (g < g_end) {
          const float* gn = s_norm + (g - g_begin) * kGroupRows;
          if constexpr (DUMP) {
            const int64_t ro = (g - g_begin) * kGroupRows;
            wepilogue_dump<METRIC>(c0, gn, h, qn0, dump0 ? dump0 + ro : nullptr);
            wepilogue_dump<METRIC>(c1, gn, h, qn1, dump1 ? dump1 + ro : nullptr);
          } else {
            wepilogue<KCAP, METRIC>(c0, gn, g * kGroupRows, h, qn0, qv0, lk0, lp0);
            wepilogue<KCAP, METRIC>(c1, gn, g * kGroupRows, h, qn1, qv1, lk1, lp1);
          }
        }
        c0 = zero;
        c1 = zero;
        s = 0;
        ++p;
      } else {
        ++s;
      }
    }

    if constexpr (DUMP) {
      __syncthreads();  // LDS (s_*, slabs) reused by the next work item
      continue;
    } else {
    // ---- merge: two rounds of 32 queries, NS lane lists (W waves x 2 halves) per query ----
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      __syncthreads();  // slab buffers / previous round done
      {
        const int src = wave * 2 + h;
#pragma unroll
        for (int i = 0; i < KCAP; ++i) {
          mkey[(j * NS + src) * KCAP + i] = t == 0 ? lk0[i] : lk1[i];
          mpos[(j * NS + src) * KCAP + i] = t == 0 ? lp0[i] : lp1[i];
        }
      }
      __syncthreads();
      const int jj = tid / NS;
      const int ss = tid % NS;
      const float* myk = mkey + (jj * NS + ss) * KCAP;
      const int* myp = mpos + (jj * NS + ss) * KCAP;
      const int64_t slot = s_slot[t * 32 + jj];
      int head = 0;
      float hk = myk[0];
      int hp = myp[0];
      for (int r = 0; r < a.k; ++r) {
        float bk = hk;
        int bp = hp;
#pragma unroll
        for (int off = NS / 2; off >= 1; off >>= 1) {
          const float ok = __shfl_xor(bk, off, NS);
          const int op = __shfl_xor(bp, off, NS);
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
}

// waves per K3w workgroup: MIVS_SCAN_WIDE_WAVES (4 or 8), default 4
int wide_waves() {
  const char* e = getenv("MIVS_SCAN_WIDE_WAVES");
  return e && atoi(e) == 8 ? 8 : 4;
}

template <int KCAP, int METRIC, int W>
hipError_t launch_wmw(const ScanArgs& a, int grid, size_t lds, hipStream_t s) {
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_scan_wide<KCAP, METRIC, W>),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  if (attr != hipSuccess) return attr;
  hipLaunchKernelGGL((k_scan_wide<KCAP, METRIC, W>), dim3(grid), dim3(W * 64), lds, s, a);
  return hipGetLastError();
}

template <int KCAP>
hipError_t launch_w(const ScanArgs& a, int grid, size_t lds, hipStream_t s) {
  if (wide_waves() == 8)
    return a.metric == kIP ? launch_wmw<KCAP, kIP, 8>(a, grid, lds, s) : launch_wmw<KCAP, kL2, 8>(a, grid, lds, s);
  return a.metric == kIP ? launch_wmw<KCAP, kIP, 4>(a, grid, lds, s) : launch_wmw<KCAP, kL2, 4>(a, grid, lds, s);
}

}  // namespace

size_t scan_wide_lds_bytes(int kcap, int chunk_groups) {
  const size_t slabs = (size_t)2 * kWQ * kSld * 4;
  const size_t merge = (size_t)32 * 2 * wide_waves() * kcap * 8;
  return kWSmall + (size_t)chunk_groups * kGroupRows * 4 + (slabs > merge ? slabs : merge);
}

bool scan_wide_supported(int kcap, int d, int dp, int chunk_groups) {
  return (kcap == 0 || kcap == 1 || kcap == 4 || kcap == 8 || kcap == 12 || kcap == 16) && d % 4 == 0 &&
         dp % kSlab == 0 &&
         scan_wide_lds_bytes(kcap, chunk_groups) <= 160 * 1024;
}

template <int KCAP, int METRIC, int W>
static int wocc_kmw(size_t lds) {
  int n = 0;
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_scan_wide<KCAP, METRIC, W>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, reinterpret_cast<const void*>(&k_scan_wide<KCAP, METRIC, W>),
                                                   W * 64, lds) != hipSuccess)
    return 1;
  return n > 0 ? n : 1;
}

template <int KCAP>
static int wocc_k(int metric, size_t lds) {
  if (wide_waves() == 8) return metric == kIP ? wocc_kmw<KCAP, kIP, 8>(lds) : wocc_kmw<KCAP, kL2, 8>(lds);
  return metric == kIP ? wocc_kmw<KCAP, kIP, 4>(lds) : wocc_kmw<KCAP, kL2, 4>(lds);
}

int scan_wide_occupancy(int kcap, int metric, size_t lds) {
  switch (kcap) {
    case 0: return wocc_k<0>(metric, lds);
    case 1: return wocc_k<1>(metric, lds);
    case 4: return wocc_k<4>(metric, lds);
    case 8: return wocc_k<8>(metric, lds);
    case 12: return wocc_k<12>(metric, lds);
    case 16: return wocc_k<16>(metric, lds);
    default: return 1;
  }
}

hipError_t launch_scan_wide(const ScanArgs& a, int kcap, int grid, size_t lds, hipStream_t s) {
  switch (kcap) {
    case 0: return launch_w<0>(a, grid, lds, s);
    case 1: return launch_w<1>(a, grid, lds, s);
    case 4: return launch_w<4>(a, grid, lds, s);
    case 8: return launch_w<8>(a, grid, lds, s);
    case 12: return launch_w<12>(a, grid, lds, s);
    case 16: return launch_w<16>(a, grid, lds, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace mivs
