// K1/K2/K3/K4 — the fused distance + top-k list-scan kernel.
//
// One workgroup (8 waves, 512 threads) takes a work item = (list l, one tile of
// up to 32 queries probing l, one chunk of <= G row groups of l). The query
// tile is staged once in LDS; each wave streams its row groups straight from
// HBM (one contiguous 1 KiB dwordx4 wave load per k-step, thanks to the
// interleaved group layout) into v_mfma_f32_32x32x2_f32 (A = 32 list rows,
// B = 32 queries). The epilogue turns the 32x32 dot tile into ranking keys and
// keeps a per-lane register top-K (lane = query, 16 rows per group per lane);
// at the end of the work item the 16 lane lists of each query are merged in
// LDS by 16-lane shuffle min-reductions and the chunk's top-k (dist, id) is
// written to the query's output slot.
//
// Replaces the list scan inside cuVS ivf_flat::search (reached from
// improved_multi_gpu_rag.py:227 / cuvs-2gpu-main.ipynb:1801), the exhaustive
// scan of FAISS IndexFlatL2.search (colab_a100_test.ipynb:454) and the k-means
// predict inside ivf_flat::build (index_building_coordinator.py:396).
#include <climits>

#include "mivs_common.hpp"

namespace mivs {

namespace {

constexpr int kSmallBytes = 32 * 8 + 32 * 8 + 32 * 4 + 16;  // s_q, s_slot, s_qn, s_misc (16-B multiple)

__device__ __forceinline__ float4 load_row4(const float* __restrict__ row, int c, int d) {
  if ((d & 3) == 0 && c + 4 <= d) return *reinterpret_cast<const float4*>(row + c);
  float4 v;
  v.x = c + 0 < d ? row[c + 0] : 0.0f;
  v.y = c + 1 < d ? row[c + 1] : 0.0f;
  v.z = c + 2 < d ? row[c + 2] : 0.0f;
  v.w = c + 3 < d ? row[c + 3] : 0.0f;
  return v;
}

// Insert (key, pos) into an ascending register list; positions reach a lane in
// increasing order, so an equal key lands after the existing ones (ties by id).
template <int KCAP>
__device__ __forceinline__ void lane_insert(float (&lk)[KCAP], int (&lp)[KCAP], float key, int pos) {
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

// Block of BLK k-steps of one row group (p at an even k-step): BLK dwordx4 loads per lane, 32 rows x 32 B each
template <int BLK>
__device__ __forceinline__ void load_block(float4 (&v)[BLK], const float* __restrict__ p) {
#pragma unroll
  for (int u = 0; u < BLK; ++u) v[u] = *reinterpret_cast<const float4*>(p + row_blk8(u));
}

template <int BLK>
__device__ __forceinline__ void mma_block(f32x16& acc, const float4 (&v)[BLK], const float* __restrict__ qrow) {
#pragma unroll
  for (int u = 0; u < BLK; ++u) {
    const float4 b = *reinterpret_cast<const float4*>(qrow + u * 8);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(v[u].x, b.x, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(v[u].y, b.y, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(v[u].z, b.z, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(v[u].w, b.w, acc, 0, 0, 0);
  }
}

// Dot tile of one finished group -> ranking keys -> this lane's register top-K.
// Row norms come from LDS (staged per work item) so no VMEM wait can drain the prefetch stream.
template <int KCAP, int METRIC>
__device__ __forceinline__ void epilogue(const f32x16& acc, const float* __restrict__ gnorm, int64_t rbase, int h,
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
    if (key < lk[KCAP - 1]) lane_insert<KCAP>(lk, lp, key, (int)(rbase + (r & 3) + 8 * (r >> 2) + 4 * h));
  }
}

// DUMP mode (KCAP == 0, k > 64): the group's keys go straight to the query's slot; rows
// 8*r4 + 4h + {0..3} of this lane are contiguous, so each lane issues 4 dwordx4 stores.
template <int METRIC>
__device__ __forceinline__ void epilogue_dump(const f32x16& acc, const float* __restrict__ gnorm, int h, float qn,
                                              float* __restrict__ dst /*slot keys + group row base*/) {
  if (dst == nullptr) return;
#pragma unroll
  for (int r4 = 0; r4 < 4; ++r4) {
    const float4 xn = *reinterpret_cast<const float4*>(gnorm + 8 * r4 + 4 * h);
    float kv[4];
    const float xs[4] = {xn.x, xn.y, xn.z, xn.w};
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

// W waves per workgroup: 16 (4 per SIMD; needs <= 128 VGPRs, KCAP <= 16) or 8
template <int KCAP, int METRIC, int W>
__global__ __launch_bounds__(W * 64, 1) void k_scan(ScanArgs a, float* __restrict__ gmerge) {
  // k-steps per register buffer: 8 (2 KiB of list rows in flight per lane-pair ring slot) unless the
  // register top-K is large
  constexpr int BLK = KCAP >= 32 ? 4 : 8;
  constexpr bool DUMP = KCAP == 0;
  constexpr int NT = W * 64;
  constexpr int NS = 2 * W;  // lane lists per query (W waves x 2 halves)
  constexpr int KR = DUMP ? 1 : KCAP;  // register list length
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int64_t* s_q = reinterpret_cast<int64_t*>(smem);          // [32] query row ids (-1: empty lane)
  int64_t* s_slot = s_q + 32;                                // [32] output slot (already + chunk)
  float* s_qn = reinterpret_cast<float*>(s_slot + 32);       // [32]
  int* s_misc = reinterpret_cast<int*>(s_qn + 32);           // [4]
  float* s_norm = reinterpret_cast<float*>(smem + kSmallBytes);  // [G*32] row norms of the chunk
  float* qtile = s_norm + a.chunk_groups * kGroupRows;
  const int dp = a.dp;
  const int qstride = dp + 4;  // +16 B per row: conflict-free ds_read_b128 of the B operand

  // merge area: LDS after the scan when it fits, else this block's global scratch
  float* mkey = gmerge ? gmerge + (size_t)blockIdx.x * (kQTile * NS * KR * 2) : qtile;
  int* mpos = reinterpret_cast<int*>(mkey + kQTile * NS * KR);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int j = lane & 31;  // query column of this lane in the MFMA tile
  const int h = lane >> 5;  // k-half / row-half of this lane
  const int total = a.work_off[a.n_lists];
  const int bpg = (dp >> 3) / BLK;  // blocks per group (dp is a multiple of 64)

  for (;;) {
    if (tid == 0) s_misc[0] = atomicAdd(a.work_counter, 1);
    __syncthreads();
    const int w = s_misc[0];
    if (w >= total) break;

    // ---- decode the work item ----
    int lo = 0, hi = a.n_lists - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (a.work_off[mid] <= w) lo = mid; else hi = mid - 1;
    }
    const int l = lo;
    const int m = a.bucket_off[l + 1] - a.bucket_off[l];
    const int tiles = (m + kQTile - 1) / kQTile;
    const int local = w - a.work_off[l];
    const int chunk = local / tiles;
    const int tile = local - chunk * tiles;
    const int64_t g_begin = a.list_goff[l] + (int64_t)chunk * a.chunk_groups;
    const int64_t g_lim = a.list_goff[l + 1];
    const int64_t g_end = g_begin + a.chunk_groups < g_lim ? g_begin + a.chunk_groups : g_lim;
    const int e0 = a.bucket_off[l] + tile * kQTile;
    const int nqt = m - tile * kQTile < kQTile ? m - tile * kQTile : kQTile;

    if (tid < kQTile) {
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
    {  // row norms of the chunk -> LDS
      const int nn = (int)(g_end - g_begin) * kGroupRows;
      for (int i = tid; i < nn; i += NT) s_norm[i] = a.row_norms[g_begin * kGroupRows + i];
      if (DUMP && tid < nqt) {  // slot header: first row position + rows of this chunk
        const int64_t slot = a.bucket_slot[e0 + tid] + chunk;
        a.out_i[2 * slot] = g_begin * kGroupRows;
        a.out_i[2 * slot + 1] = nn;
      }
    }
    __syncthreads();

    // ---- stage the query tile in LDS (zero-padded dims, zero rows for empty lanes) ----
    {
      const int c4 = dp >> 2;
      for (int i = tid; i < kQTile * c4; i += NT) {
        const int r = i / c4;
        const int c = (i - r * c4) << 2;
        const int64_t q = s_q[r];
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (q >= 0) v = load_row4(a.queries + q * (int64_t)a.d, c, a.d);
        *reinterpret_cast<float4*>(qtile + r * qstride + c) = v;
      }
    }
    __syncthreads();

    float lk[KR];
    int lp[KR];
#pragma unroll
    for (int t = 0; t < KR; ++t) { lk[t] = INFINITY; lp[t] = INT_MAX; }
    const float qn = s_qn[j];
    const bool qvalid = s_q[j] >= 0;
    const int slot_rows = a.chunk_groups * kGroupRows;
    float* const dump_base = DUMP && qvalid ? a.out_d + s_slot[j] * (int64_t)slot_rows : nullptr;
    const float* qrow = qtile + j * qstride + 4 * h;

    // ---- this wave's row groups g_begin+wave, +8, ... as ONE stream of BLK-step blocks, two
    //      register buffers (A: even blocks, B: odd blocks): the load of block b+2 is issued right
    //      after block b's MFMAs, so a full block of MFMAs covers every load, across group
    //      boundaries too ----
    const int64_t g0 = g_begin + wave;
    const int ng = g_end > g0 ? (int)((g_end - g0 + W - 1) / W) : 0;
    const int nb = ng * bpg;
    if (nb > 0) {
      const float* lane_base = a.groups + g0 * (int64_t)(kGroupRows * dp) + j * kRowBlk + 4 * h;
      const int64_t gstride = (int64_t)W * kGroupRows * dp;
      auto bptr = [&](int b) {
        const int bb = b < nb ? b : nb - 1;  // past the end: re-read the last block (never consumed)
        const int gi = bb / bpg;
        return lane_base + gi * gstride + row_blk8((bb - gi * bpg) * BLK);
      };
      float4 A[BLK], B[BLK];
      load_block<BLK>(A, bptr(0));
      load_block<BLK>(B, bptr(1));
      f32x16 acc = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      const f32x16 zero = acc;
      int gi = 0, sb = 0;  // group / block-in-group of the block being consumed
      // Both halves run unconditionally (an odd stream gets one dummy block whose result is never
      // used): every path through the body then issues the same loads in the same order, so the
      // compiler's vmcnt at the loop head can keep the other buffer's loads in flight.
      for (int b = 0; b < nb; b += 2) {
        mma_block<BLK>(acc, A, qrow + sb * (BLK * 8));
        load_block<BLK>(A, bptr(b + 2));
        if (++sb == bpg) {
          if constexpr (DUMP)
            epilogue_dump<METRIC>(acc, s_norm + (wave + gi * W) * kGroupRows, h, qn,
                                  dump_base ? dump_base + (wave + gi * W) * kGroupRows : nullptr);
          else
            epilogue<KCAP, METRIC>(acc, s_norm + (wave + gi * W) * kGroupRows,
                                   (g0 + (int64_t)gi * W) * kGroupRows, h, qn, qvalid, lk, lp);
          acc = zero;
          sb = 0;
          ++gi;
        }
        mma_block<BLK>(acc, B, qrow + sb * (BLK * 8));
        load_block<BLK>(B, bptr(b + 3));
        if (++sb == bpg && b + 1 < nb) {
          if constexpr (DUMP)
            epilogue_dump<METRIC>(acc, s_norm + (wave + gi * W) * kGroupRows, h, qn,
                                  dump_base ? dump_base + (wave + gi * W) * kGroupRows : nullptr);
          else
            epilogue<KCAP, METRIC>(acc, s_norm + (wave + gi * W) * kGroupRows,
                                   (g0 + (int64_t)gi * W) * kGroupRows, h, qn, qvalid, lk, lp);
          acc = zero;
          sb = 0;
          ++gi;
        }
      }
    }

    if constexpr (DUMP) {
      __syncthreads();  // LDS (s_*, qtile) reused by the next work item
      continue;
    }
    // ---- merge the NS lane lists (W waves x 2 halves) of every query ----
    __syncthreads();  // every wave is done with qtile (the merge area may alias it)
    {
      const int src = wave * 2 + h;
#pragma unroll
      for (int t = 0; t < KCAP; ++t) {
        mkey[(j * NS + src) * KCAP + t] = lk[t];
        mpos[(j * NS + src) * KCAP + t] = lp[t];
      }
    }
    __syncthreads();
    {
      const int jj = tid / NS;  // query of this NS-thread segment
      const int ss = tid % NS;  // source list of this thread
      const float* myk = mkey + (jj * NS + ss) * KCAP;
      const int* myp = mpos + (jj * NS + ss) * KCAP;
      const int64_t slot = s_slot[jj];
      int head = 0;
      float hk = myk[0];
      int hp = myp[0];
      for (int t = 0; t < a.k; ++t) {
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
          a.out_d[slot * a.k + t] = valid ? (METRIC == kIP ? -bk : bk) : (METRIC == kIP ? -INFINITY : INFINITY);
          a.out_i[slot * a.k + t] = valid ? a.row_ids[bp] : (int64_t)-1;
        }
        if (hk == bk && hp == bp && head < KCAP) {
          ++head;
          hk = head < KCAP ? myk[head] : INFINITY;
          hp = head < KCAP ? myp[head] : INT_MAX;
        }
      }
    }
    __syncthreads();  // LDS (s_*, merge area) reused by the next work item
  }
}

template <int KCAP, int METRIC, int W>
hipError_t launch_kmw(const ScanArgs& a, int grid, size_t lds, float* gmerge, hipStream_t s) {
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_scan<KCAP, METRIC, W>),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  if (attr != hipSuccess) return attr;
  hipLaunchKernelGGL((k_scan<KCAP, METRIC, W>), dim3(grid), dim3(W * 64), lds, s, a, gmerge);
  return hipGetLastError();
}

template <int KCAP>
hipError_t launch_k(const ScanArgs& a, int grid, size_t lds, float* gmerge, hipStream_t s) {
  if constexpr (KCAP <= 16) {
    if (scan_waves(KCAP) == 16)
      return a.metric == kIP ? launch_kmw<KCAP, kIP, 16>(a, grid, lds, gmerge, s)
                             : launch_kmw<KCAP, kL2, 16>(a, grid, lds, gmerge, s);
  }
  return a.metric == kIP ? launch_kmw<KCAP, kIP, 8>(a, grid, lds, gmerge, s)
                         : launch_kmw<KCAP, kL2, 8>(a, grid, lds, gmerge, s);
}

}  // namespace

int scan_kcap(int k) {
  if (k > kMaxK) return 0;  // DUMP mode + K8 select
  if (k <= 1) return 1;
  if (k <= 4) return 4;
  if (k <= 8) return 8;
  if (k <= 12) return 12;  // k = 10 (the benchmark's k): 8 fewer list registers than 16
  if (k <= 16) return 16;
  if (k <= 32) return 32;
  if (k <= 64) return 64;
  return -1;
}

// waves per K3 workgroup: 16 (4 waves per SIMD, register budget <= 128) for the DUMP scan, else 8.
// MIVS_SCAN_WAVES=8 forces 8 (A/B measurements).
int scan_waves(int kcap) {
  // 16 waves need <= 128 VGPRs: only the DUMP instantiation fits without spilling
  const char* e = getenv("MIVS_SCAN_WAVES");
  if (e && atoi(e) == 8) return 8;
  return kcap == 0 ? 16 : 8;
}

static size_t merge_bytes(int kcap) { return (size_t)kQTile * 2 * scan_waves(kcap) * kcap * 8; }
static size_t qtile_bytes(int dp) { return (size_t)kQTile * (dp + 4) * 4; }
static size_t norm_bytes(int chunk_groups) { return (size_t)chunk_groups * kGroupRows * 4; }
static constexpr size_t kLdsMax = 160 * 1024;

// LDS request: [small][chunk norms][query tile | merge area]; the merge area moves to global
// scratch when it does not fit beside the norms
size_t scan_lds_bytes(int dp, int kcap, int chunk_groups) {
  const size_t base = kSmallBytes + norm_bytes(chunk_groups);
  const size_t q = qtile_bytes(dp), m = merge_bytes(kcap);
  const size_t both = base + (q > m ? q : m);
  return both <= kLdsMax ? both : base + q;
}

bool scan_merge_in_lds(int dp, int kcap, int chunk_groups) {
  const size_t base = kSmallBytes + norm_bytes(chunk_groups);
  return base + merge_bytes(kcap) <= kLdsMax && base + qtile_bytes(dp) <= kLdsMax;
}

size_t scan_gmerge_bytes(int grid, int kcap) { return (size_t)grid * merge_bytes(kcap); }

hipError_t launch_scan_ex(const ScanArgs& a, int kcap, int grid, size_t lds, float* gmerge, hipStream_t s) {
  switch (kcap) {
    case 0: return launch_k<0>(a, grid, lds, gmerge, s);
    case 1: return launch_k<1>(a, grid, lds, gmerge, s);
    case 4: return launch_k<4>(a, grid, lds, gmerge, s);
    case 8: return launch_k<8>(a, grid, lds, gmerge, s);
    case 12: return launch_k<12>(a, grid, lds, gmerge, s);
    case 16: return launch_k<16>(a, grid, lds, gmerge, s);
    case 32: return launch_k<32>(a, grid, lds, gmerge, s);
    case 64: return launch_k<64>(a, grid, lds, gmerge, s);
    default: return hipErrorInvalidValue;
  }
}

template <int KCAP, int METRIC, int W>
static int occ_kmw(size_t lds) {
  int n = 0;
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_scan<KCAP, METRIC, W>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, reinterpret_cast<const void*>(&k_scan<KCAP, METRIC, W>),
                                                   W * 64, lds) != hipSuccess)
    return 1;
  return n > 0 ? n : 1;
}

template <int KCAP>
static int occ_k(int metric, size_t lds) {
  if constexpr (KCAP <= 16) {
    if (scan_waves(KCAP) == 16) return metric == kIP ? occ_kmw<KCAP, kIP, 16>(lds) : occ_kmw<KCAP, kL2, 16>(lds);
  }
  return metric == kIP ? occ_kmw<KCAP, kIP, 8>(lds) : occ_kmw<KCAP, kL2, 8>(lds);
}

int scan_occupancy(int kcap, int metric, size_t lds) {
  switch (kcap) {
    case 0: return occ_k<0>(metric, lds);
    case 1: return occ_k<1>(metric, lds);
    case 4: return occ_k<4>(metric, lds);
    case 8: return occ_k<8>(metric, lds);
    case 12: return occ_k<12>(metric, lds);
    case 16: return occ_k<16>(metric, lds);
    case 32: return occ_k<32>(metric, lds);
    case 64: return occ_k<64>(metric, lds);
    default: return 1;
  }
}

hipError_t launch_scan(const ScanArgs& a, int kcap, int grid, size_t lds_bytes, hipStream_t s) {
  return launch_scan_ex(a, kcap, grid, lds_bytes, nullptr, s);
}

}  // namespace mivs
