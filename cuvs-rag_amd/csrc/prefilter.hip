// K10 / K11 — fp16 pre-filter list scan + exact fp32 refine.
//
// Why: at the benchmark shape every list is probed by ~300 queries, so the exact
// fp32 scan (K3w) is bound by the fp32 MFMA rate (157 TF). The fp16 MFMA runs 16x
// faster per FLOP and an fp16 copy of the lists streams half the bytes. The price
// is an approximate dot; the refine step makes the RESULT exact again:
//
//   K10: per (list, 2048-row chunk, 64-query tile): approximate keys from
//        v_mfma_f32_32x32x16_f16 (fp16 rows x fp16 queries, fp32 accumulate, exact
//        power-of-two unscaling); per query the slot_k smallest approximate keys
//        of the chunk + a LOWER BOUND of every approximate key it dropped.
//   K11: per query, Ak = k-th smallest approximate key, delta = a rigorous bound of
//        |approx key - pinned fp32 key| (Cauchy-Schwarz on the fp16 rounding
//        residuals + worst-case fp32 summation error of both dot products),
//        window T = Ak + 2 delta. Every candidate with approx key <= T is recomputed
//        in the pinned fp32 order (= oracle orc_dot / the fp32 MFMA chain); the true
//        top-k is inside the window, so the output equals the exact scan bit for bit.
//        If a dropped key could be inside the window (bound <= T) or the window holds
//        more than kPfCap candidates, the query is listed for the exact scan.
#include <climits>
#include <utility>
#include <cstdlib>

#include "mivs_common.hpp"
#include "pf_math.hpp"

namespace mivs {

namespace {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));

constexpr int kPfWaves = 8;
constexpr int kPfThreads = kPfWaves * 64;
constexpr int kPfSmall = kPfQTile * 8 * 2 + kPfQTile * 4 * 2 + 16;  // s_q, s_slot, s_qn, s_qs, s_misc
constexpr int kPfMergeBytes = kPfQTile * 16 * kPfLaneK * 8;          // [64 queries][16 lane lists][KL] (key, pos)

__device__ __forceinline__ h8 ld_h8(const uint16_t* p) { return *reinterpret_cast<const h8*>(p); }
// a row operand; NT: non-temporal policy (rows read once)
template <bool NT>
__device__ __forceinline__ h8 ld_row_h8(const uint16_t* p) {
  if constexpr (NT) return __builtin_nontemporal_load(reinterpret_cast<const h8*>(p));
  else return *reinterpret_cast<const h8*>(p);
}

// ---- 16-lane (DPP row) reductions: a butterfly over quad_perm [1,0,3,2], quad_perm [2,3,0,1],
// row_half_mirror, row_mirror -- every lane of the row ends with the row's result, without the LDS
// round trips of ds_bpermute (__shfl_xor) ----
template <int CTRL>
__device__ __forceinline__ int pf_dpp(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false);
}
template <int CTRL>
__device__ __forceinline__ float pf_dpp(float v) {
  return __builtin_bit_cast(float, pf_dpp<CTRL>(__builtin_bit_cast(int, v)));
}
template <int CTRL>
__device__ __forceinline__ void pf_row_min_step(float& k, int& p) {
  const float ok = pf_dpp<CTRL>(k);
  const int op = pf_dpp<CTRL>(p);
  if (ok < k || (ok == k && op < p)) { k = ok; p = op; }
}
// lexicographic (key, pos) minimum over the 16 lanes of a DPP row
__device__ __forceinline__ void pf_row_min(float& k, int& p) {
  pf_row_min_step<0xB1>(k, p);
  pf_row_min_step<0x4E>(k, p);
  pf_row_min_step<0x141>(k, p);
  pf_row_min_step<0x140>(k, p);
}
__device__ __forceinline__ float pf_row_fmin(float v) {
  v = fminf(v, pf_dpp<0xB1>(v));
  v = fminf(v, pf_dpp<0x4E>(v));
  v = fminf(v, pf_dpp<0x141>(v));
  return fminf(v, pf_dpp<0x140>(v));
}

template <int KL>
__device__ __forceinline__ void pf_insert(float (&lk)[KL], int (&lp)[KL], float key, int pos) {
#pragma unroll
  for (int t = KL - 1; t >= 0; --t) {
    const float prev = t > 0 ? lk[t > 0 ? t - 1 : 0] : -INFINITY;
    const int prevp = t > 0 ? lp[t > 0 ? t - 1 : 0] : 0;
    const bool shift = key < prev;
    const bool place = !shift && key < lk[t];
    lk[t] = shift ? prev : (place ? key : lk[t]);
    lp[t] = shift ? prevp : (place ? pos : lp[t]);
  }
}

template <int METRIC>
__device__ __forceinline__ bool pf_epilogue(const f32x16& c0, const f32x16& c1, const float* __restrict__ s_gnorm,
                                            int64_t rb, int h, float qn0, float qs0, float th0, float uf0, float qn1,
                                            float qs1, float th1, float uf1, float (&lk0)[kPfLaneK],
                                            int (&lp0)[kPfLaneK], float (&lk1)[kPfLaneK], int (&lp1)[kPfLaneK]) {
  float xn[16];
#pragma unroll
  for (int q4 = 0; q4 < 4; ++q4) {
    const float4 t = *reinterpret_cast<const float4*>(s_gnorm + 8 * q4 + 4 * h);
    xn[4 * q4 + 0] = t.x; xn[4 * q4 + 1] = t.y; xn[4 * q4 + 2] = t.z; xn[4 * q4 + 3] = t.w;
  }
  // fast path: one fma + one compare per element; once theta is tight almost every group ends here
  const float m0 = METRIC == kL2 ? -2.0f * qs0 : -qs0;
  const float m1 = METRIC == kL2 ? -2.0f * qs1 : -qs1;
  float mn0 = INFINITY, mn1 = INFINITY;  // (no NaN reaches here: accumulators are finite, pad norms +inf)
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const float b = METRIC == kL2 ? xn[r] : 0.0f;
    mn0 = fminf(mn0, fmaf(c0[r], m0, b));
    mn1 = fminf(mn1, fmaf(c1[r], m1, b));
  }
  if (__ballot(mn0 < uf0 || mn1 < uf1) == 0) return false;
  // a key is kept if it beats the lane list AND lies within the query's window bound theta
  // (th = -inf for empty query slots: nothing is kept)
  // the exact key only where the one-fma filter passes (it never rejects a key the exact test keeps)
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int pos = (int)(rb + (r & 3) + 8 * (r >> 2) + 4 * h);
    const float b = METRIC == kL2 ? xn[r] : 0.0f;
    if (fmaf(c0[r], m0, b) < uf0) {
      const float k0 = pf_key<METRIC>(c0[r], qs0, xn[r], qn0);
      if (k0 < lk0[kPfLaneK - 1] && k0 <= th0) pf_insert<kPfLaneK>(lk0, lp0, k0, pos);
    }
    if (fmaf(c1[r], m1, b) < uf1) {
      const float k1 = pf_key<METRIC>(c1[r], qs1, xn[r], qn1);
      if (k1 < lk1[kPfLaneK - 1] && k1 <= th1) pf_insert<kPfLaneK>(lk1, lp1, k1, pos);
    }
  }
  return true;
}

// theta of a query from its 16 lane lists' last entries (s_l8[16]): with m full lists whose last entries are
// v1 <= .. <= vm, at least 8 m >= k kept keys are <= vm, so the query's k-th approximate key over the whole
// search is <= vm and the refine window is <= pf_window(vm). m = 2 for k <= 16, ceil(k / 8) <= 4 for k <= 32.
__device__ __forceinline__ float pf_theta(const float* __restrict__ l8, float delta, int m) {
  float v0 = INFINITY, v1 = INFINITY, v2 = INFINITY, v3 = INFINITY;  // the 4 smallest, ascending
#pragma unroll
  for (int i = 0; i < 16; i += 4) {
    const float4 v = *reinterpret_cast<const float4*>(l8 + i);
    const float e[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const float x = e[t];
      v3 = fminf(v3, fmaxf(v2, x));
      v2 = fminf(v2, fmaxf(v1, x));
      v1 = fminf(v1, fmaxf(v0, x));
      v0 = fminf(v0, x);
    }
  }
  const float vm = m <= 2 ? v1 : (m == 3 ? v2 : v3);
  return vm < INFINITY ? pf_window(vm, delta) : INFINITY;
}

// K10. One workgroup (8 waves) per CU, persistent over (list, chunk, 64-query tile) work items.
// The query tile stays in LDS for the whole chunk as the B operand ([2][dp/8][32] x 16 B: each
// k-step's operand is one contiguous 1 KiB wave read), next to the chunk's row norms. Each wave streams its own 32-row groups (pass p: group g_begin + 8p + wave)
// as the A operand straight from HBM: one 1 KiB contiguous wave load per k-step, D k-steps in
// flight across pass boundaries (a ring of D registers refilled right after their MFMAs); 2 MFMAs
// (the two 32-query column tiles) per load.
// Work items are dealt from 8 queues, one per XCD group (blockIdx % 8): queue g holds the g-th
// eighth of the (list, chunk, tile)-ordered items, so the query tiles of one chunk run at the same
// time on CUs sharing an L2 and all but the first read the chunk's rows as L2 hits. A workgroup
// whose queue is empty takes items from the next queues.
// F8 (K13's pre-pass nomination, pair mode only): the rows and queries are fp8 copies (groups_f8 / q8, the
// [32-dim superblock][32 rows][2 halves][16 B] operand layout of k_groups_to_f8), each 16-B load feeds two
// v_mfma_f32_32x32x16_fp8_fp8 k-steps; the keys only nominate rows whose pinned keys K11 then computes
template <int METRIC, int D, int R, bool NT = false, bool F8 = false>
__global__ __launch_bounds__(kPfThreads, 1) void k_pf_scan(PfScanArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int64_t* s_q = reinterpret_cast<int64_t*>(smem);          // [64] query ids (-1: empty)
  int64_t* s_slot = s_q + kPfQTile;                          // [64] output slot (already + chunk)
  float* s_qn = reinterpret_cast<float*>(s_slot + kPfQTile);  // [64]
  float* s_qs = s_qn + kPfQTile;                              // [64]
  int* s_misc = reinterpret_cast<int*>(s_qs + kPfQTile);
  float* s_dl = reinterpret_cast<float*>(smem + kPfSmall);    // [64] per-query window delta
  float* s_th = s_dl + kPfQTile;                                // [64] theta at item start
  float* s_l8 = s_th + kPfQTile;                                // [64][16] lane lists' last entries
  // per wave the row norms of its current pass's groups [8 waves][64] (loaded one pass ahead), so the
  // chunk size is not bound by LDS
  float* s_norm = s_l8 + kPfQTile * 16;
  char* s_b = reinterpret_cast<char*>(s_norm + kPfWaves * 64);
  float* mkey = reinterpret_cast<float*>(s_b);
  int* mpos = reinterpret_cast<int*>(mkey + kPfQTile * 16 * kPfLaneK);

  const int dp = a.dp;
  const int nb = dp >> 3;  // 8-dim blocks
  // 16-dim k-steps (a multiple of D)
  const int nk = F8 ? dp >> 5 : dp >> 4;
  static_assert(!F8 || R == 2, "fp8 rows: pair mode only");
  const int bq1off = F8 ? dp * 32 : nb * 512;  // B image: query group 1's bytes after group 0's
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: the k-loop is a scalar loop
  const int j = lane & 31;
  const int h = lane >> 5;
  const int total = a.work_off[a.n_lists];
  const int grp = blockIdx.x & 7;
  // halves between a wave's consecutive groups (F8: a group is 32 dp bytes)
  const int64_t pstride = F8 ? (int64_t)kPfWaves * 16 * dp : (int64_t)kPfWaves * nb * 256;
  const float xnmax2 = a.x_norm_max * a.x_norm_max;       // >= every row's pinned norm
  const int mth = a.k > 16 ? (a.k + kPfLaneK - 1) / kPfLaneK : 2;  // lane lists theta needs (pf_theta)
  if (tid == 0) s_misc[1] = 0;                            // queues exhausted so far
  // diagnostic phase clocks (a.prof != nullptr only under MIVS_PF_FLAGS & 32)
  unsigned long long pr_top = 0, pr_item = 0, pr_stage = 0, pr_loop = 0, pr_bar = 0, pr_slow = 0, pr_epi = 0;
  const unsigned long long pr_t0 = a.prof ? __builtin_amdgcn_s_memtime() : 0;
  const unsigned long long pr_r0 = a.prof ? __builtin_amdgcn_s_memrealtime() : 0;

  for (;;) {
    const unsigned long long pr_a = a.prof ? __builtin_amdgcn_s_memtime() : 0;
    if (tid == 0) {
      int qs = s_misc[1], w = total;
      while (qs < 8) {
        const int g = (grp + qs) & 7;
        const int lo_g = (int)((int64_t)total * g / 8), hi_g = (int)((int64_t)total * (g + 1) / 8);
        const int i = atomicAdd(a.work_counter + 16 * g, 1);
        if (lo_g + i < hi_g) { w = lo_g + i; break; }
        ++qs;
      }
      s_misc[1] = qs;
      s_misc[0] = w;
    }
    __syncthreads();
    const int w = s_misc[0];
    if (w >= total) break;
    const unsigned long long pr_b = a.prof ? __builtin_amdgcn_s_memtime() : 0;

    int lo = 0, hi = a.n_lists - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (a.work_off[mid] <= w) lo = mid; else hi = mid - 1;
    }
    const int l = lo;
    const int m = a.bucket_off[l + 1] - a.bucket_off[l];
    const int tiles = (m + kPfQTile - 1) / kPfQTile;
    const int local = w - a.work_off[l];
    const int chunk = local / tiles;
    const int tile = local - chunk * tiles;
    const int64_t g_begin = a.list_goff[l] + (int64_t)chunk * a.chunk_groups;
    const int64_t g_lim = a.list_goff[l + 1];
    const int64_t g_end = g_begin + a.chunk_groups < g_lim ? g_begin + a.chunk_groups : g_lim;
    const int e0 = a.bucket_off[l] + tile * kPfQTile;
    const int nqt = m - tile * kPfQTile < kPfQTile ? m - tile * kPfQTile : kPfQTile;
    const int ng = (int)(g_end - g_begin);

    if (tid < kPfQTile) {
      if (tid < nqt) {
        const int64_t q = a.bucket_q[e0 + tid];
        s_q[tid] = q;
        s_slot[tid] = a.bucket_slot[e0 + tid] + chunk;
        const float qn = a.qnorms[q];
        s_qn[tid] = qn;
        s_qs[tid] = F8 ? a.qscale8[q] : a.qscale[q];
        // (F8: the window only widens which nominees a slot keeps; 2^7 x the fp16 bound)
        s_dl[tid] = pf_delta<METRIC>(qn, a.qres[q], a.x_norm_max, a.x_res_max, dp) * (F8 ? 128.0f : 1.0f);
        s_th[tid] = pf_unord(__hip_atomic_load(a.qtheta + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
      } else {
        s_q[tid] = -1;
        s_slot[tid] = -1;
        s_qn[tid] = INFINITY;
        s_qs[tid] = 0.0f;
        s_dl[tid] = 0.0f;
        s_th[tid] = -INFINITY;
      }
    }
    for (int i = tid; i < kPfQTile * 16; i += kPfThreads) s_l8[i] = INFINITY;
    int* const cpos = a.chunk_pos ? a.chunk_pos + (int64_t)l * a.chunk_stride + chunk : nullptr;
    if (tid == 0) s_misc[2] = cpos ? __hip_atomic_load(cpos, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
    __syncthreads();
    // stage the fp16 query tile. B image: [2 query groups][nb blocks][32 queries] x 16 B, so that the
    // operand of (group t, k-step s) for lane (j, h) sits at t*nb*512 + s*1024 + lane*16: one contiguous
    // 1 KiB wave read (conflict-free) at an immediate offset per k-step. Piece i of the image is
    // written by thread i mod 512 (linear, conflict-free); its source is a 16-B piece of query row
    // (i/32/nb)*32 + i%32. nb/8 pieces per thread (dp % 64 == 0), loads batched by 4.
    if (F8 && !(a.flags & 8)) {
      // fp8 B image: [2 query groups][dp/32 superblocks][64 lanes (j, h)] x 16 B, piece (S, j, h) = bytes
      // 32 S + 16 h .. + 16 of query j's fp8 row (k_queries_to_f8 lays them out as the operands)
      const int nsb = dp >> 5;
      const int per = dp >> 7;  // 4 dp pieces over 512 threads
      for (int i0 = 0; i0 < per; i0 += 2) {
        uint4 v[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int i = tid + (i0 + u) * kPfThreads;
          const int qg = i / (nsb * 64), rem = i - qg * (nsb * 64);
          const int S = rem >> 6, L = rem & 63;
          const int64_t q = (i0 + u < per) ? s_q[qg * 32 + (L & 31)] : -1;
          v[u] = make_uint4(0u, 0u, 0u, 0u);
          if (q >= 0) v[u] = *reinterpret_cast<const uint4*>(a.q8 + q * dp + S * 32 + (L >> 5) * 16);
        }
#pragma unroll
        for (int u = 0; u < 2; ++u)
          if (i0 + u < per) *reinterpret_cast<uint4*>(s_b + (size_t)(tid + (i0 + u) * kPfThreads) * 16) = v[u];
      }
    }
    if (!F8 && !(a.flags & 8)) {
      const int per = nb >> 3;
      for (int i0 = 0; i0 < per; i0 += 4) {
        uint4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int i = tid + (i0 + u) * kPfThreads;
          const int gb = i >> 5;
          const int qg = gb / nb, b = gb - qg * nb;
          const int64_t q = (i0 + u < per) ? s_q[qg * 32 + (i & 31)] : -1;
          v[u] = make_uint4(0u, 0u, 0u, 0u);
          if (q >= 0 && b < 2 * nk) v[u] = *reinterpret_cast<const uint4*>(a.qh + q * dp + 8 * b);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (i0 + u < per) *reinterpret_cast<uint4*>(s_b + (size_t)(tid + (i0 + u) * kPfThreads) * 16) = v[u];
      }
    }
    __syncthreads();
    const unsigned long long pr_c = a.prof ? __builtin_amdgcn_s_memtime() : 0;

    float lk0[kPfLaneK], lk1[kPfLaneK];
    int lp0[kPfLaneK], lp1[kPfLaneK];
#pragma unroll
    for (int t = 0; t < kPfLaneK; ++t) { lk0[t] = INFINITY; lp0[t] = INT_MAX; lk1[t] = INFINITY; lp1[t] = INT_MAX; }
    const float qn0 = s_qn[j], qn1 = s_qn[32 + j], qs0 = s_qs[j], qs1 = s_qs[32 + j];
    const float dl0 = s_dl[j], dl1 = s_dl[32 + j];
    // per-query window bound theta (refreshed after every pass from all lane lists); -inf: empty slot
    // starts from the query's window bound over the items finished so far (qtheta, all workgroups)
    float th0 = s_th[j], th1 = s_th[32 + j];
    float uf0 = pf_uf<METRIC>(INFINITY, th0, qn0, xnmax2), uf1 = pf_uf<METRIC>(INFINITY, th1, qn1, xnmax2);
    const int src = wave * 2 + h;  // this lane's list index among the query's 16

    const char* s_bl = s_b + lane * 16;  // this lane's B operand at k-step s: + s * 1024 (+ nb * 512: group 1)
    const int npw = wave < ng ? (ng - wave + kPfWaves - 1) / kPfWaves : 0;  // groups (passes) of this wave
    // the epilogue of one finished group (its 32 x 64 dots) + the theta refresh
    auto epilogue = [&](const f32x16& c0, const f32x16& c1, int lg, const float* gnorm) {
      if (a.flags & 1) return;
      if (a.prof) ++pr_epi;
      const bool slow = pf_epilogue<METRIC>(c0, c1, gnorm, (g_begin + lg) * kGroupRows, h, qn0,
                                            qs0, th0, uf0, qn1, qs1, th1, uf1, lk0, lp0, lk1, lp1);
      if (a.prof && slow) ++pr_slow;
      // no insertion anywhere in this wave: its lists, and so its published ends, did not change (the
      // other waves' ends may have, but a stale theta is only looser, still valid)
      if (!slow) return;
      // publish this lane's list ends, refresh theta from all 16 (no barrier: every value ever
      // stored is the end of a real list, so a stale read only gives a looser, still valid theta)
      s_l8[j * 16 + src] = lk0[kPfLaneK - 1];
      s_l8[(32 + j) * 16 + src] = lk1[kPfLaneK - 1];
      th0 = fminf(th0, pf_theta(s_l8 + j * 16, dl0, mth));
      th1 = fminf(th1, pf_theta(s_l8 + (32 + j) * 16, dl1, mth));
      uf0 = pf_uf<METRIC>(lk0[kPfLaneK - 1], th0, qn0, xnmax2);
      uf1 = pf_uf<METRIC>(lk1[kPfLaneK - 1], th1, qn1, xnmax2);
    };
    if constexpr (R == 2) {
      // two groups per pass (g = wave + 8i, pairs i = 2p, 2p + 1): every B operand read from LDS feeds
      // 4 MFMAs instead of 2, halving the LDS traffic per flop; an odd last pair re-reads its first group
      // Convoy: the tiles of one chunk start at different times on CUs of one XCD; a late tile joins
      // the pair the earlier ones are scanning (cpos, published after every pair) and wraps round to the
      // pairs it skipped, so the tiles read the chunk together as L2 hits instead of a second time from
      // HBM once their lag exceeds the L2's reach. The visiting order changes no result.
      const int npair = (npw + 1) >> 1;
      if (npw > 0) {
        const int rot = s_misc[2] % npair;
        auto phys = [&](int pr) { return pr + rot < npair ? pr + rot : pr + rot - npair; };
        const uint16_t* abase = F8 ? reinterpret_cast<const uint16_t*>(a.groups_f8) + (g_begin + wave) * 16 * dp + j * 16 + h * 8
                                   : a.groups_h + ((g_begin + wave) * nb + h) * 256 + j * 8;
        int lp_ = 0, ls = 0;  // pair / k-step of the next load (past the end: re-read the last pair)
        auto pair_ptr = [&](int pr, int which) {
          int gi = 2 * phys(pr) + which;
          gi = gi < npw ? gi : npw - 1;
          return abase + (int64_t)gi * pstride;
        };
        const uint16_t* na = pair_ptr(0, 0);
        const uint16_t* nbp = pair_ptr(0, 1);
        // row norms of a pair: lane L holds row L & 31 of its group 2 * pair + (L >> 5) (an odd last pair
        // repeats its first group, as the rows do); written to this wave's LDS slot at the pair's end
        float* const wn = s_norm + wave * 64;
        auto pair_norm = [&](int pr) {
          int gi = 2 * phys(pr) + (lane >> 5);
          gi = gi < npw ? gi : npw - 1;
          return a.row_norms[(g_begin + wave + (int64_t)gi * kPfWaves) * kGroupRows + (lane & 31)];
        };
        float nrm = pair_norm(0);
        h8 ra[D], rb[D];
#pragma unroll
        for (int u = 0; u < D; ++u) {
          ra[u] = ld_row_h8<NT>(na + (ls + u) * 512);
          rb[u] = ld_row_h8<NT>(nbp + (ls + u) * 512);
          __builtin_amdgcn_sched_barrier(0);
        }
        ls += D;
        if (ls == nk) { ls = 0; if (++lp_ < npair) { na = pair_ptr(lp_, 0); nbp = pair_ptr(lp_, 1); } }
        const f32x16 zero = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        f32x16 a0 = zero, a1 = zero, b0 = zero, b1 = zero;
        int p = 0, s = 0;
        h8 bq0[2], bq1[2];
        bq0[0] = *reinterpret_cast<const h8*>(s_bl);
        bq1[0] = *reinterpret_cast<const h8*>(s_bl + bq1off);
        for (int t0 = 0; t0 < npair * nk; t0 += D) {
#pragma unroll
          for (int u = 0; u < D; ++u) {
            int sn = s + u + 1;
            if (sn >= nk) sn -= nk;
            bq0[(u + 1) & 1] = *reinterpret_cast<const h8*>(s_bl + sn * 1024);
            bq1[(u + 1) & 1] = *reinterpret_cast<const h8*>(s_bl + bq1off + sn * 1024);
            if constexpr (F8) {
              typedef long l2 __attribute__((ext_vector_type(2)));
              const l2 xa = __builtin_bit_cast(l2, ra[u]), xb = __builtin_bit_cast(l2, rb[u]);
              const l2 y0 = __builtin_bit_cast(l2, bq0[u & 1]), y1 = __builtin_bit_cast(l2, bq1[u & 1]);
#pragma unroll
              for (int e = 0; e < 2; ++e) {
                a0 = __builtin_amdgcn_mfma_f32_32x32x16_fp8_fp8(xa[e], y0[e], a0, 0, 0, 0);
                a1 = __builtin_amdgcn_mfma_f32_32x32x16_fp8_fp8(xa[e], y1[e], a1, 0, 0, 0);
                b0 = __builtin_amdgcn_mfma_f32_32x32x16_fp8_fp8(xb[e], y0[e], b0, 0, 0, 0);
                b1 = __builtin_amdgcn_mfma_f32_32x32x16_fp8_fp8(xb[e], y1[e], b1, 0, 0, 0);
              }
            } else {
              a0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ra[u], bq0[u & 1], a0, 0, 0, 0);
              a1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ra[u], bq1[u & 1], a1, 0, 0, 0);
              b0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(rb[u], bq0[u & 1], b0, 0, 0, 0);
              b1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(rb[u], bq1[u & 1], b1, 0, 0, 0);
            }
            ra[u] = ld_row_h8<NT>(na + (ls + u) * 512);
            rb[u] = ld_row_h8<NT>(nbp + (ls + u) * 512);
            __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);            // DS read
            __builtin_amdgcn_sched_group_barrier(0x008, F8 ? 8 : 4, 0);   // MFMA
            __builtin_amdgcn_sched_group_barrier(0x020, 2, 0);            // VMEM read
          }
          ls += D;
          if (ls == nk) { ls = 0; if (++lp_ < npair) { na = pair_ptr(lp_, 0); nbp = pair_ptr(lp_, 1); } }
          s += D;
          if (s == nk) {
            const int pp = phys(p);
            if (cpos && wave == 0 && lane == 0)
              __hip_atomic_store(cpos, pp + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            wn[lane] = nrm;  // this pair's norms (read back by this wave only: LDS keeps its order)
            if (p + 1 < npair) nrm = pair_norm(p + 1);
            epilogue(a0, a1, 2 * pp * kPfWaves + wave, wn);
            if (2 * pp + 1 < npw) epilogue(b0, b1, (2 * pp + 1) * kPfWaves + wave, wn + kGroupRows);
            a0 = zero; a1 = zero; b0 = zero; b1 = zero;
            s = 0;
            ++p;
          }
        }
      }
    } else {
    if (npw > 0) {
      // convoy start as in the pair path, in passes of one group per wave
      const int rot = s_misc[2] % npw;
      auto phys1 = [&](int pr) { return pr + rot < npw ? pr + rot : pr + rot - npw; };
      const uint16_t* abase = a.groups_h + ((g_begin + wave) * nb + h) * 256 + j * 8;
      const uint16_t* nptr = abase + (int64_t)phys1(0) * pstride;  // pass base of the next load
      int ls = 0, lpass = 0;         // k-step / pass of the next load (past the end: re-read the last pass)
      float* const wn = s_norm + wave * 64;
      auto pass_norm = [&](int pr) {
        return a.row_norms[(g_begin + wave + (int64_t)phys1(pr) * kPfWaves) * kGroupRows + (lane & 31)];
      };
      float nrm = pass_norm(0);
      h8 ring[D];
      // the ring holds one block of D k-steps; (nptr, ls) = the next block to load (nk % D == 0)
#pragma unroll
      for (int u = 0; u < D; ++u) {
        ring[u] = ld_h8(nptr + (ls + u) * 512);
        __builtin_amdgcn_sched_barrier(0);  // issue in ring order: the loop header then waits vmcnt(D-1)
      }
      ls += D;
      if (ls == nk) { ls = 0; if (++lpass < npw) nptr = abase + (int64_t)phys1(lpass) * pstride; }
      const f32x16 zero = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      f32x16 c0 = zero, c1 = zero;
      int p = 0, s = 0;
      // B operands PB k-steps ahead (slot u % (PB + 1)): the LDS latency hides behind PB k-steps of MFMAs
      constexpr int PB = D % 3 == 0 ? 2 : 1;
      h8 bq0[PB + 1], bq1[PB + 1];
#pragma unroll
      for (int t = 0; t < PB; ++t) {
        bq0[t] = *reinterpret_cast<const h8*>(s_bl + (t % nk) * 1024);
        bq1[t] = *reinterpret_cast<const h8*>(s_bl + nb * 512 + (t % nk) * 1024);
      }
      // ONE flat loop over (pass, k-step) in blocks of D (nk % D == 0, so a pass ends on a block end):
      // the compiler then keeps the ring's loads counted (vmcnt(D-1)) across pass boundaries
      for (int t0 = 0; t0 < npw * nk; t0 += D) {
#pragma unroll
        for (int u = 0; u < D; ++u) {
          int sn = s + u + PB;  // the k-step PB ahead (B is per k-step; wraps into the next pass)
          if (sn >= nk) sn -= nk;
          bq0[(u + PB) % (PB + 1)] = *reinterpret_cast<const h8*>(s_bl + sn * 1024);
          bq1[(u + PB) % (PB + 1)] = *reinterpret_cast<const h8*>(s_bl + nb * 512 + sn * 1024);
          c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ring[u], bq0[u % (PB + 1)], c0, 0, 0, 0);
          c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(ring[u], bq1[u % (PB + 1)], c1, 0, 0, 0);
          ring[u] = ld_h8(nptr + (ls + u) * 512);
          // pin the per-k-step issue order (2 DS reads, 2 MFMAs, then the refill) so the refill of
          // ring[u] is issued right after its last use and D loads stay in flight
          __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);  // DS read
          __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);  // MFMA
          __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // VMEM read
        }
        ls += D;
        if (ls == nk) { ls = 0; if (++lpass < npw) nptr = abase + (int64_t)phys1(lpass) * pstride; }
        s += D;
        if (s == nk) {
          const int pp = phys1(p);
          if (cpos && wave == 0 && lane == 0)
            __hip_atomic_store(cpos, pp + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          wn[lane] = nrm;
          if (p + 1 < npw) nrm = pass_norm(p + 1);
          epilogue(c0, c1, pp * kPfWaves + wave, wn);
        }
        if (s == nk) {
          c0 = zero;
          c1 = zero;
          s = 0;
          ++p;
        }
      }
    }

    }

    // ---- per query: 16 lane lists (8 waves x 2 halves) -> slot top-slot_k + dropped-key bound ----
    const unsigned long long pr_d = a.prof ? __builtin_amdgcn_s_memtime() : 0;
    __syncthreads();  // the B image is dead
    const unsigned long long pr_e = a.prof ? __builtin_amdgcn_s_memtime() : 0;
    if (a.raw_lists) {
      // raw slots (slot_k = 16 lists x kPfLaneK): every lane's two lists straight into its queries' slots, unsorted --
      // K11 and K11v rank all of a slot's entries -- and per query the dropped-key bound (as the merge's: the 16 lists'
      // last entries, +inf where a list is not full, and the theta term), one thread per query from the list ends the
      // epilogues published in s_l8. No per-query merge rounds (the pre-pass's took ~0.1 of its time, in the three
      // waves holding a list's ~10 queries while the other five waited).
      const int64_t sl0 = s_slot[j], sl1 = s_slot[32 + j];
      if (sl0 >= 0) {
        float* kd = a.slot_key + sl0 * a.slot_k + src * kPfLaneK;
        int* pd = a.slot_pos + sl0 * a.slot_k + src * kPfLaneK;
#pragma unroll
        for (int i = 0; i < kPfLaneK; ++i) { kd[i] = lk0[i]; pd[i] = lp0[i]; }
      }
      if (sl1 >= 0) {
        float* kd = a.slot_key + sl1 * a.slot_k + src * kPfLaneK;
        int* pd = a.slot_pos + sl1 * a.slot_k + src * kPfLaneK;
#pragma unroll
        for (int i = 0; i < kPfLaneK; ++i) { kd[i] = lk1[i]; pd[i] = lp1[i]; }
      }
      if (a.slot_bound && tid < kPfQTile) {
        const int64_t sl = s_slot[tid];
        if (sl >= 0) {
          float bnd = nextafterf(fminf(s_th[tid], pf_theta(s_l8 + tid * 16, s_dl[tid], mth)), INFINITY);
#pragma unroll
          for (int i = 0; i < 16; ++i) bnd = fminf(bnd, s_l8[tid * 16 + i]);
          a.slot_bound[sl] = bnd;
        }
      }
    } else {
    {
#pragma unroll
      for (int i = 0; i < kPfLaneK; ++i) {
        mkey[(j * 16 + src) * kPfLaneK + i] = lk0[i];
        mpos[(j * 16 + src) * kPfLaneK + i] = lp0[i];
        mkey[((32 + j) * 16 + src) * kPfLaneK + i] = lk1[i];
        mpos[((32 + j) * 16 + src) * kPfLaneK + i] = lp1[i];
      }
    }
    __syncthreads();
#pragma unroll
    for (int rnd = 0; rnd < 2; ++rnd) {
      if (a.flags & 16) break;
      const int qi = rnd * 32 + (tid >> 4);
      const int src = tid & 15;
      const float* myk = mkey + (qi * 16 + src) * kPfLaneK;
      const int* myp = mpos + (qi * 16 + src) * kPfLaneK;
      const int64_t slot = s_slot[qi];
      // a full lane list dropped keys >= its last entry; keys above theta were dropped, and every
      // lane's theta is >= the one from the final list ends
      float bnd = myk[kPfLaneK - 1];
      // (theta drops are keys > theta: the bound is the next float up, so a theta equal to the
      // refine's window -- the common case when one slot holds the whole top-k -- is no overflow)
      if (src == 0) bnd = fminf(bnd, nextafterf(fminf(s_th[qi], pf_theta(s_l8 + qi * 16, s_dl[qi], mth)), INFINITY));
      bnd = pf_row_fmin(bnd);
      // fast path (the common case once theta is tight): fewer than k kept keys in all 16 lists
      // -> compact them unsorted into the slot (the refine needs no order), pad with +inf
      int cnt = 0;
#pragma unroll
      for (int i = 0; i < kPfLaneK; ++i) cnt += myk[i] < INFINITY ? 1 : 0;
      // inclusive prefix over the query's 16 lists (DPP row_shr 1, 2, 4, 8 with zero fill) and the total
      int pre = cnt;
      pre += __builtin_amdgcn_update_dpp(0, pre, 0x111, 0xF, 0xF, true);
      pre += __builtin_amdgcn_update_dpp(0, pre, 0x112, 0xF, 0xF, true);
      pre += __builtin_amdgcn_update_dpp(0, pre, 0x114, 0xF, 0xF, true);
      pre += __builtin_amdgcn_update_dpp(0, pre, 0x118, 0xF, 0xF, true);
      int total = cnt;
      total += pf_dpp<0xB1>(total);
      total += pf_dpp<0x4E>(total);
      total += pf_dpp<0x141>(total);
      total += pf_dpp<0x140>(total);
      if (total < a.k) {  // uniform within the 16-lane group
        if (slot >= 0) {
          const int64_t sb = slot * a.slot_k;
          const int base = pre - cnt;
#pragma unroll
          for (int i = 0; i < kPfLaneK; ++i)
            if (i < cnt) { a.slot_key[sb + base + i] = myk[i]; a.slot_pos[sb + base + i] = myp[i]; }
          for (int t = total + src; t < a.slot_k; t += 16) { a.slot_key[sb + t] = INFINITY; a.slot_pos[sb + t] = INT_MAX; }
          if (src == 0) a.slot_bound[slot] = bnd;
        }
        continue;
      }
      int head = 0;
      float hk = myk[0];
      int hp = myp[0];
      float lastk = -INFINITY;
      for (int r = 0; r <= a.slot_k; ++r) {  // slot_k outputs, then the smallest key left behind
        float bk = hk;
        int bp = hp;
        pf_row_min(bk, bp);
        if (!(bk < INFINITY)) {  // every list is exhausted: the rest of the slot is empty, nothing left behind
          if (src == 0 && slot >= 0)
            for (int t = r; t < a.slot_k; ++t) { a.slot_key[slot * a.slot_k + t] = INFINITY; a.slot_pos[slot * a.slot_k + t] = INT_MAX; }
          break;
        }
        // nomination (slot_out): past slot_out keys and their ties, the slot's reader takes nothing more; the rest
        // is empty and bk is the smallest key left behind (uniform within the 16-lane group, like bk)
        if (a.slot_out > 0 && r >= a.slot_out && r < a.slot_k && bk != lastk) {
          if (slot >= 0)
            for (int t = r + src; t < a.slot_k; t += 16) { a.slot_key[slot * a.slot_k + t] = INFINITY; a.slot_pos[slot * a.slot_k + t] = INT_MAX; }
          bnd = fminf(bnd, bk);
          break;
        }
        lastk = bk;
        if (r < a.slot_k) {
          if (src == 0 && slot >= 0) {
            a.slot_key[slot * a.slot_k + r] = bk;
            a.slot_pos[slot * a.slot_k + r] = bp;
            // the query's k-th key over the whole search is <= this slot's k-th: tighten its theta
            if (r == a.k - 1 && bk < INFINITY)
              atomicMin(a.qtheta + s_q[qi], pf_ord(pf_window(bk, s_dl[qi])));
          }
        } else {
          bnd = fminf(bnd, bk);
        }
        if (hk == bk && hp == bp && head < kPfLaneK) {
          ++head;
          hk = head < kPfLaneK ? myk[head] : INFINITY;
          hp = head < kPfLaneK ? myp[head] : INT_MAX;
        }
      }
      if (src == 0 && slot >= 0) a.slot_bound[slot] = bnd;
    }
    }  // (raw_lists)
    __syncthreads();
    if (a.prof) {
      const unsigned long long pr_f = __builtin_amdgcn_s_memtime();
      pr_top += pr_b - pr_a; pr_item += pr_c - pr_b; pr_stage += pr_d - pr_c; pr_loop += pr_e - pr_d;
      pr_bar += pr_f - pr_e;
    }
  }
  if (a.prof && lane == 0) {
    // [0] fetch, [1] staging, [2] main loop, [3] post-loop barrier wait, [4] merge (cycles, summed over
    // waves), [5] epilogues, [6] slow-path epilogues, [7] wave-cycles, [8] 100 MHz ticks
    atomicAdd(a.prof + 0, pr_top); atomicAdd(a.prof + 1, pr_item); atomicAdd(a.prof + 2, pr_stage);
    atomicAdd(a.prof + 3, pr_loop); atomicAdd(a.prof + 4, pr_bar); atomicAdd(a.prof + 5, pr_epi);
    atomicAdd(a.prof + 6, pr_slow);
    atomicAdd(a.prof + 7, __builtin_amdgcn_s_memtime() - pr_t0);
    atomicAdd(a.prof + 8, __builtin_amdgcn_s_memrealtime() - pr_r0);
  }
}

// K11. One wave per query (4 per workgroup; every wave reaches every barrier).
template <int METRIC>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8))) void k_pf_refine(PfRefineArgs a) {
  __shared__ float s_ck[4][kPfCap];
  __shared__ int s_cp[4][kPfCap];
  __shared__ __attribute__((aligned(16))) float s_qv[4][1024];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int64_t q = (int64_t)blockIdx.x * 4 + wv;
  const bool live = q < a.nq;
  const int k = a.k;
  int64_t sb = 0, se = 0;
  bool cap_ovf = false;  // (slot_cnt: the query's fixed-capacity run dropped candidates)
  if (live) {
    if (a.slot_cnt) {
      const int c = a.slot_cnt[q];
      sb = q * (int64_t)a.slot_cap;
      se = sb + (c < a.slot_cap ? c : a.slot_cap);
      cap_ovf = c > a.slot_cap;
    } else {
      sb = a.slot_begin[q];
      se = a.slot_begin[q + 1];
    }
  }
  const int64_t c1 = se * a.slot_k;
  // (K13: slot_k = 1 and slot_begin the per-query CSR runs of unsorted candidates, or slot_cnt the fixed-capacity runs)
  const bool cnt_ovf = (a.force_ovf && *a.force_ovf) || cap_ovf;

  // phase 1: Ak = k-th smallest approximate key. Up to kPfSelRegs * 64 candidates (K13's runs: ~200 per query at the
  // benchmark shape): held in registers, a 32-step radix select over their orderable bits -- the largest u with
  // fewer than k keys below it is the k-th smallest (ties counted), no shuffles; more: the running top-k
  // (K7's ballot insertion). Both return the same value.
  float mk = INFINITY, tk = INFINITY;
  const int64_t n_c = c1 - sb * a.slot_k;
  if (n_c <= kPfSelRegs * 64) {
    uint32_t u[kPfSelRegs];
#pragma unroll
    for (int i = 0; i < kPfSelRegs; ++i) {
      const int64_t cc = sb * a.slot_k + i * 64 + lane;
      const float f = cc < c1 ? a.slot_key[cc] : INFINITY;
      const uint32_t b = __float_as_uint(f == 0.0f ? 0.0f : f);  // (-0 and +0: one key)
      u[i] = (b & 0x80000000u) ? ~b : (b | 0x80000000u);
    }
    uint32_t ans = 0;
    for (int bit = 31; bit >= 0; --bit) {
      const uint32_t t = ans | (1u << bit);
      int below = 0;
#pragma unroll
      for (int i = 0; i < kPfSelRegs; ++i) below += __popcll(__ballot(u[i] < t));
      if (below < k) ans = t;
    }
    const uint32_t b = (ans & 0x80000000u) ? (ans & 0x7FFFFFFFu) : ~ans;
    tk = __uint_as_float(b);
  } else
  for (int64_t c = sb * a.slot_k; c < c1; c += 64) {
    const int64_t cc = c + lane;
    const float ck = cc < c1 ? a.slot_key[cc] : INFINITY;
    uint64_t mask = __ballot(ck < tk);
    while (mask) {
      const int b = __ffsll((unsigned long long)mask) - 1;
      const float nk = __shfl(ck, b);
      const int pos = __popcll(__ballot(lane < k && mk <= nk));
      const float pk = __shfl_up(mk, 1);
      if (lane == pos) mk = nk;
      else if (lane > pos) mk = pk;
      tk = __shfl(mk, k - 1);
      mask &= ~(1ull << b);
      mask &= __ballot(ck < tk);
    }
  }
  if (a.kth_out) {  // (kernel-uniform: every wave of the block leaves here)
    if (live && lane == 0) a.kth_out[q] = tk;
    return;
  }
  float bmin = cnt_ovf ? -INFINITY : INFINITY;
  if (a.slot_bound)
    for (int64_t sl = sb + lane; sl < se; sl += 64) bmin = fminf(bmin, a.slot_bound[sl]);
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) bmin = fminf(bmin, __shfl_xor(bmin, off));

  // the window: delta >= |approx key - pinned key| for every candidate of this query
  const int64_t qrow = live && a.qrows ? a.qrows[q] : q;  // the query's row in queries / qnorms / qres
  const float qn = live ? a.qnorms[qrow] : 0.0f;
  const float delta = pf_delta<METRIC>(qn, live ? a.qres[qrow] : 0.0f, a.x_norm_max, a.x_res_max, a.dp);
  const float T = pf_window(tk, delta);  // +inf when fewer than k candidates
  bool ovf = bmin < INFINITY && (bmin <= T || bmin == -INFINITY);
  // K13: its candidates are every row whose approximate key is <= T_q (a superset); the window is complete
  // only if it lies below T_q, which the analysis of T_q guarantees -- checked here, not assumed
  if (live && a.window_cap && !(T <= a.window_cap[q])) ovf = true;

  // phase 2: collect the window (ballot prefix, no atomics)
  int cnt = 0;
  for (int64_t c = sb * a.slot_k; c < c1; c += 64) {
    const int64_t cc = c + lane;
    const float ck = cc < c1 ? a.slot_key[cc] : INFINITY;
    const bool take = ck <= T && ck < INFINITY;  // +inf: an empty slot entry (fewer than k candidates: T = +inf)
    const uint64_t msk = __ballot(take);
    if (take) {
      const int at = cnt + __popcll(msk & ((1ull << lane) - 1));
      if (at < kPfCap) { s_ck[wv][at] = ck; s_cp[wv][at] = a.slot_pos[cc]; }
    }
    cnt += __popcll(msk);
  }
  ovf = ovf || cnt > kPfCap;
  if (live && ovf && lane == 0) {
    const int at = atomicAdd(a.ovf_count, 1);
    a.ovf_q[at] = q;
  }
  // window-size stats: one atomic per workgroup (10k same-address atomics per launch were a serial tail)
  __shared__ int s_win[4];
  if (lane == 0) s_win[wv] = live && !ovf ? cnt : 0;
  // the query row in LDS (zero past d), for the exact recompute
  for (int i = lane; i < a.dp; i += 64) s_qv[wv][i] = (live && i < a.d) ? a.queries[qrow * a.d + i] : 0.0f;
  __syncthreads();
  if (threadIdx.x == 0 && a.n_window) {
    const int w = s_win[0] + s_win[1] + s_win[2] + s_win[3];
    if (w) atomicAdd(reinterpret_cast<unsigned long long*>(a.n_window), (unsigned long long)w);
  }

  // phase 3: exact keys in the pinned order (oracle orc_dot), then a bitonic sort by (key, id).
  // Eight lanes per window row, eight rows per pass: lane (j, p) = (lane >> 3, lane & 7) loads the 8-dim blocks
  // b = 8 B + p of row j (32 B each, the group of eight reading a whole 256-B row block), every block of the pass in
  // flight at once, and the row's one fmaf chain runs over the blocks in order b = 0, 1, 2, ... by handing the
  // accumulator to the next lane of the group with a DPP move (row_shr:1; part 7 -> part 0 of the next 64-dim
  // block by row_shl:7): lane (j, h) extends it at hop h, the other lanes' results are discarded. One lane per row
  // issued 192 16-B loads per row (12 lanes active), ~8 dependent memory rounds a query (profiles/DESIGN_history_r01_r05.md §6d-6).
  float P = INFINITY;
  int64_t id = LLONG_MAX;
  if (live && !ovf) {  // (wave-uniform)
    const int j8 = lane >> 3, p8 = lane & 7;
    const int nB = a.dp >> 6;
    const float* qv = s_qv[wv];
    float* s_dot = s_ck[wv];  // (the window's approximate keys are dead: their slots take the dots)
    // 64-dim blocks of a pass in flight: 4 (64 VGPRs, 8 waves / SIMD) rather than the whole row at once (CH 12: 128
    // VGPRs, 4 waves): more queries in flight hide the rows' latency better -- 153-159 vs 175-178 us per 10k-query
    // refine, CH 6 at 6 waves 158-160 us (alternating runs, profiles/r06x_k11_occupancy.txt)
    constexpr int CH = 4;
    for (int r0 = 0; r0 < cnt; r0 += 8) {
      const int rj = r0 + j8;
      const float* rowp = a.groups + row_elem(s_cp[wv][rj < cnt ? rj : r0], 0, a.dp) + 8 * p8;
      float acc = 0.0f;
      for (int B0 = 0; B0 < nB; B0 += CH) {
        float4 x[CH][2];
#pragma unroll
        for (int u = 0; u < CH; ++u)
          if (B0 + u < nB) {
            x[u][0] = *reinterpret_cast<const float4*>(rowp + (int64_t)(B0 + u) * kRowBlkStride);
            x[u][1] = *reinterpret_cast<const float4*>(rowp + (int64_t)(B0 + u) * kRowBlkStride + 4);
          }
#pragma unroll
        for (int u = 0; u < CH; ++u) {
          if (B0 + u >= nB) break;
          const int b = 8 * (B0 + u) + p8;
          const float4 y0 = *reinterpret_cast<const float4*>(qv + 8 * b);
          const float4 y1 = *reinterpret_cast<const float4*>(qv + 8 * b + 4);
          const float4 x0 = x[u][0], x1 = x[u][1];
#pragma unroll
          for (int h = 0; h < 8; ++h) {
            if (h > 0) acc = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, acc), 0x111, 0xF, 0xF, false));
            else if (B0 + u > 0) acc = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, acc), 0x107, 0xF, 0xF, false));
            acc = fmaf(x0.x, y0.x, acc); acc = fmaf(x1.x, y1.x, acc);
            acc = fmaf(x0.y, y0.y, acc); acc = fmaf(x1.y, y1.y, acc);
            acc = fmaf(x0.z, y0.z, acc); acc = fmaf(x1.z, y1.z, acc);
            acc = fmaf(x0.w, y0.w, acc); acc = fmaf(x1.w, y1.w, acc);
          }
        }
      }
      if (p8 == 7 && rj < cnt) s_dot[rj] = acc;  // (part 7 ends the row's chain)
    }
  }
  // s_dot (= s_ck[wv]) is written by lanes p8 == 7 and read below by other lanes of the same wave: order the LDS
  // stores before the loads explicitly instead of relying on in-order LDS within a wave
  wave_lds_sync();
  if (live && !ovf && lane < cnt) {
    const int pos = s_cp[wv][lane];
    const float acc = s_ck[wv][lane];
    if (METRIC == kL2) {
      const float v = fmaf(-2.0f, acc, a.row_norms[pos] + qn);
      P = v > 0.0f ? v : 0.0f;
    } else {
      P = -acc;
    }
    id = a.row_ids[pos];
  }
#pragma unroll
  for (int size = 2; size <= 64; size <<= 1) {
#pragma unroll
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      const float oP = __shfl_xor(P, stride);
      const int64_t oid = __shfl_xor(id, stride);
      const bool want_min = ((lane & stride) == 0) == ((lane & size) == 0);  // ascending blocks keep min low
      const bool o_lt = oP < P || (oP == P && oid < id);
      const bool o_gt = oP > P || (oP == P && oid > id);
      if (want_min ? o_lt : o_gt) { P = oP; id = oid; }
    }
  }
  if (live && !ovf && lane < k) {
    const bool valid = id != LLONG_MAX;
    a.out_d[q * k + lane] = valid ? (METRIC == kIP ? -P : P) : (METRIC == kIP ? -INFINITY : INFINITY);
    a.out_i[q * k + lane] = valid ? id : (int64_t)-1;
  }
}

// K11v: K13's pre-pass verification (verify_sel > 0, kth_out): phase 1 of K11 at rank verify_sel, then fp32 keys of
// the nominees and the k-th smallest of them (a kernel of its own: inside K11 its code changed how the compiler
// unrolled K11's exact recompute, 0.18 -> 0.33 ms per final refine)
template <int METRIC>
// (8 waves / SIMD, 64 VGPRs: 82 vs 85-88 us at its own 76-VGPR 6-wave default, profiles/r06x_k11_occupancy.txt)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8))) void k_pf_verify(PfRefineArgs a) {
  __shared__ int s_cp[4][kPfCap];
  __shared__ __attribute__((aligned(16))) float s_qv[4][1024];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int64_t q = (int64_t)blockIdx.x * 4 + wv;
  const bool live = q < a.nq;
  const int k = a.k;
  int64_t sb = 0, se = 0;
  if (live) { sb = a.slot_begin[q]; se = a.slot_begin[q + 1]; }
  const int64_t c1 = se * a.slot_k;

  // K11's phase 1 at rank ksel: tk = the ksel-th smallest nomination score
  float mk = INFINITY, tk = INFINITY;
  const int ksel = a.verify_sel;
  const int64_t n_c = c1 - sb * a.slot_k;
  if (n_c <= kPfSelRegs * 64) {
    uint32_t u[kPfSelRegs];
#pragma unroll
    for (int i = 0; i < kPfSelRegs; ++i) {
      const int64_t cc = sb * a.slot_k + i * 64 + lane;
      const float f = cc < c1 ? a.slot_key[cc] : INFINITY;
      const uint32_t b = __float_as_uint(f == 0.0f ? 0.0f : f);  // (-0 and +0: one key)
      u[i] = (b & 0x80000000u) ? ~b : (b | 0x80000000u);
    }
    uint32_t ans = 0;
    for (int bit = 31; bit >= 0; --bit) {
      const uint32_t t = ans | (1u << bit);
      int below = 0;
#pragma unroll
      for (int i = 0; i < kPfSelRegs; ++i) below += __popcll(__ballot(u[i] < t));
      if (below < ksel) ans = t;
    }
    const uint32_t b = (ans & 0x80000000u) ? (ans & 0x7FFFFFFFu) : ~ans;
    tk = __uint_as_float(b);
  } else
  for (int64_t c = sb * a.slot_k; c < c1; c += 64) {
    const int64_t cc = c + lane;
    const float ck = cc < c1 ? a.slot_key[cc] : INFINITY;
    uint64_t mask = __ballot(ck < tk);
    while (mask) {
      const int b = __ffsll((unsigned long long)mask) - 1;
      const float nk = __shfl(ck, b);
      const int pos = __popcll(__ballot(lane < ksel && mk <= nk));
      const float pk = __shfl_up(mk, 1);
      if (lane == pos) mk = nk;
      else if (lane > pos) mk = pk;
      tk = __shfl(mk, ksel - 1);
      mask &= ~(1ull << b);
      mask &= __ballot(ck < tk);
    }
  }
  {
    // verify: the nominees (key <= the verify_sel-th smallest; ties beyond 64 dropped: any probed rows bound the
    // final k-th key) get fp32 keys, the wave summing each row's dot in parallel (not the pinned order: the key is
    // within the pinned one's summation-error term of delta, so kth + 2 delta still bounds the final window's
    // k-th approximate key, k_rs_headers); kth_out = the k-th smallest (+inf: fewer than k)
    int cnt = 0;
    for (int64_t c = sb * a.slot_k; c < c1; c += 64) {
      const int64_t cc = c + lane;
      const float ck = cc < c1 ? a.slot_key[cc] : INFINITY;
      const bool take = ck <= tk && ck < INFINITY;
      const uint64_t msk = __ballot(take);
      if (take) {
        const int at = cnt + __popcll(msk & ((1ull << lane) - 1));
        if (at < 64) s_cp[wv][at] = a.slot_pos[cc];
      }
      cnt += __popcll(msk);
    }
    const int64_t qrow = live && a.qrows ? a.qrows[q] : q;
    const float qn = live ? a.qnorms[qrow] : 0.0f;
    for (int i = lane; i < a.dp; i += 64) s_qv[wv][i] = (live && i < a.d) ? a.queries[qrow * a.d + i] : 0.0f;
    __syncthreads();
    float P = INFINITY;
    const int nvf = live ? (cnt < 64 ? cnt : 64) : 0;
    const int nb = a.dp >> 3;
    // two nominees' rows in flight at a time (lane: 8-dim blocks lane, lane + 64; dp <= 1024), at 8 waves / SIMD:
    // one row at a time, each nominee was a dependent memory round of its own (~10 per query); four rows at a time
    // took 112 VGPRs (4 waves / SIMD) and measured 87 -> 93 us
    constexpr int RW = 2;
    for (int n0 = 0; n0 < nvf; n0 += RW) {
      float4 xs[RW][2][2];
      int pos[RW];
#pragma unroll
      for (int r = 0; r < RW; ++r) {
        pos[r] = s_cp[wv][n0 + r < nvf ? n0 + r : n0];
        const float* rowp = a.groups + row_elem(pos[r], 0, a.dp);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int b = lane + 64 * i;
          xs[r][i][0] = xs[r][i][1] = make_float4(0.f, 0.f, 0.f, 0.f);
          if (n0 + r < nvf && b < nb) {
            xs[r][i][0] = *reinterpret_cast<const float4*>(rowp + row_blk8(b));
            xs[r][i][1] = *reinterpret_cast<const float4*>(rowp + row_blk8(b) + 4);
          }
        }
      }
#pragma unroll
      for (int r = 0; r < RW; ++r) {
        if (n0 + r >= nvf) break;
        float acc = 0.0f;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int b = lane + 64 * i;
          if (b < nb) {
            const float4 x0 = xs[r][i][0], x1 = xs[r][i][1];
            const float4 y0 = *reinterpret_cast<const float4*>(s_qv[wv] + 8 * b);
            const float4 y1 = *reinterpret_cast<const float4*>(s_qv[wv] + 8 * b + 4);
            acc = fmaf(x0.x, y0.x, acc); acc = fmaf(x0.y, y0.y, acc); acc = fmaf(x0.z, y0.z, acc); acc = fmaf(x0.w, y0.w, acc);
            acc = fmaf(x1.x, y1.x, acc); acc = fmaf(x1.y, y1.y, acc); acc = fmaf(x1.z, y1.z, acc); acc = fmaf(x1.w, y1.w, acc);
          }
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) acc += __shfl_xor(acc, o);
        if (lane == n0 + r) {
          if (METRIC == kL2) {
            const float v = fmaf(-2.0f, acc, a.row_norms[pos[r]] + qn);
            P = v > 0.0f ? v : 0.0f;
          } else {
            P = -acc;
          }
        }
      }
    }
#pragma unroll
    for (int size = 2; size <= 64; size <<= 1) {
#pragma unroll
      for (int stride = size >> 1; stride > 0; stride >>= 1) {
        const float oP = __shfl_xor(P, stride);
        const bool want_min = ((lane & stride) == 0) == ((lane & size) == 0);
        if (want_min ? oP < P : oP > P) P = oP;
      }
    }
    const float kx = __shfl(P, k - 1);
    if (live && lane == 0) a.kth_out[q] = kx;
    return;
  }
}

typedef unsigned int pf_u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int pf_exp_for(float m) {
  if (!(m > 0.0f) || !(m < INFINITY)) return 0;
  int e = 14 - ilogbf(m);  // m * 2^e in [2^14, 2^15)
  return e < -60 ? -60 : (e > 60 ? 60 : e);
}

__device__ __forceinline__ uint16_t pf_to_half(float v, float sc, float isc, float& res) {
  _Float16 hv = (_Float16)(v * sc);
  if (fabsf((float)hv) < 0x1p-14f) hv = (_Float16)0.0f;  // no fp16 subnormals reach the MFMA
  const float e = v - (float)hv * isc;                      // exact (Sterbenz, or hv == 0)
  res = fmaf(e, e, res);
  return __builtin_bit_cast(uint16_t, hv);
}

__global__ void k_groups_to_half(const float* __restrict__ groups, int64_t n_groups, int dp, int hx_exp,
                                 uint16_t* __restrict__ out, unsigned* __restrict__ stats) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t g = t >> 5;
  const int r = (int)(t & 31);
  float res = 0.0f;
  if (g < n_groups) {
    const int nb = dp >> 3;
    const float sc = ldexpf(1.0f, hx_exp), isc = ldexpf(1.0f, -hx_exp);
    const float* row = groups + row_elem(g * kGroupRows + r, 0, dp);
    // a 64-dim block of the row (256 B, 16 loads) in flight at a time (dp % 64 == 0): one 32-B step at a time the
    // copy ran at 3.7 TB/s (build_roofline "fp16_copy")
    for (int b0 = 0; b0 < nb; b0 += 8) {
      float4 x[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) x[u] = *reinterpret_cast<const float4*>(row + row_blk8(b0 + (u >> 1)) + 4 * (u & 1));
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int64_t o = ((g * nb + b0 + u) * kGroupRows + r) * 8;  // (the fp16 copy: [dp/8][32][8] per group)
        const float4 x0 = x[2 * u], x1 = x[2 * u + 1];
        uint4 pk;
        pk.x = pf_to_half(x0.x, sc, isc, res) | ((unsigned)pf_to_half(x0.y, sc, isc, res) << 16);
        pk.y = pf_to_half(x0.z, sc, isc, res) | ((unsigned)pf_to_half(x0.w, sc, isc, res) << 16);
        pk.z = pf_to_half(x1.x, sc, isc, res) | ((unsigned)pf_to_half(x1.y, sc, isc, res) << 16);
        pk.w = pf_to_half(x1.z, sc, isc, res) | ((unsigned)pf_to_half(x1.w, sc, isc, res) << 16);
        __builtin_nontemporal_store(__builtin_bit_cast(pf_u32x4, pk), reinterpret_cast<pf_u32x4*>(out + o));
      }
    }
  }
  float rn = sqrtf(res) * (1.0f + 0x1p-12f);
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) rn = fmaxf(rn, __shfl_xor(rn, off));
  if ((threadIdx.x & 63) == 0) atomicMax(stats, __float_as_uint(rn));
}

__global__ void k_abs_max(const float* __restrict__ x, int64_t n, unsigned* __restrict__ out) {
  float m = 0.0f;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    m = fmaxf(m, fabsf(x[i]));
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) m = fmaxf(m, __shfl_xor(m, off));
  if ((threadIdx.x & 63) == 0) atomicMax(out, __float_as_uint(m));
}

__global__ void k_norm_max(const float* __restrict__ x, int64_t n, unsigned* __restrict__ out) {
  float m = 0.0f;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float v = x[i];
    if (v < INFINITY) m = fmaxf(m, v);
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) m = fmaxf(m, __shfl_xor(m, off));
  if ((threadIdx.x & 63) == 0) atomicMax(out, __float_as_uint(m));
}

// one wave per query
__global__ __launch_bounds__(256) void k_queries_to_half(const float* __restrict__ q, int64_t nq, int d, int dp,
                                                         int hx_exp, uint16_t* __restrict__ qh,
                                                         float* __restrict__ qscale, float* __restrict__ qres) {
  const int lane = threadIdx.x & 63;
  const int64_t qi = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (qi >= nq) return;
  const float* row = q + qi * d;
  float m = 0.0f;
  for (int i = lane; i < d; i += 64) m = fmaxf(m, fabsf(row[i]));
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) m = fmaxf(m, __shfl_xor(m, off));
  const int e = pf_exp_for(m);
  const float sc = ldexpf(1.0f, e), isc = ldexpf(1.0f, -e);
  float res = 0.0f;
  for (int i = lane; i < dp; i += 64) qh[qi * dp + i] = pf_to_half(i < d ? row[i] : 0.0f, sc, isc, res);
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) res += __shfl_xor(res, off);
  if (lane == 0) {
    qscale[qi] = ldexpf(1.0f, -(hx_exp + e));
    qres[qi] = sqrtf(res) * (1.0f + 0x1p-12f);
  }
}

// k_queries_to_half for d % 4 == 0: the wave's row loaded once as NV float4 per lane (dp <= 256 NV),
// all loads in flight together, max and conversion from registers, 8-byte stores
template <int NV>
__global__ __launch_bounds__(256) void k_queries_to_half_v(const float* __restrict__ q, int64_t nq, int d, int dp,
                                                           int hx_exp, uint16_t* __restrict__ qh,
                                                           float* __restrict__ qscale, float* __restrict__ qres) {
  const int lane = threadIdx.x & 63;
  const int64_t qi = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (qi >= nq) return;
  const float4* row = reinterpret_cast<const float4*>(q + qi * d);
  float4 v[NV];
  float m = 0.0f;
#pragma unroll
  for (int u = 0; u < NV; ++u) {
    const int c4 = lane + 64 * u;
    v[u] = 4 * c4 < d ? row[c4] : make_float4(0.f, 0.f, 0.f, 0.f);
    m = fmaxf(m, fmaxf(fmaxf(fabsf(v[u].x), fabsf(v[u].y)), fmaxf(fabsf(v[u].z), fabsf(v[u].w))));
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) m = fmaxf(m, __shfl_xor(m, off));
  const int e = pf_exp_for(m);
  const float sc = ldexpf(1.0f, e), isc = ldexpf(1.0f, -e);
  float res = 0.0f;
#pragma unroll
  for (int u = 0; u < NV; ++u) {
    const int c4 = lane + 64 * u;
    if (4 * c4 < dp) {
      uint2 pk;
      pk.x = pf_to_half(v[u].x, sc, isc, res) | ((unsigned)pf_to_half(v[u].y, sc, isc, res) << 16);
      pk.y = pf_to_half(v[u].z, sc, isc, res) | ((unsigned)pf_to_half(v[u].w, sc, isc, res) << 16);
      *reinterpret_cast<uint2*>(qh + qi * dp + 4 * c4) = pk;
    }
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) res += __shfl_xor(res, off);
  if (lane == 0) {
    qscale[qi] = ldexpf(1.0f, -(hx_exp + e));
    qres[qi] = sqrtf(res) * (1.0f + 0x1p-12f);
  }
}

__global__ void k_scatter_results(const float* __restrict__ in_d, const int64_t* __restrict__ in_i,
                                  const int64_t* __restrict__ rows, int64_t n, int k, float* __restrict__ out_d,
                                  int64_t* __restrict__ out_i) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n * k) return;
  const int64_t i = t / k, c = t - i * k;
  out_d[rows[i] * k + c] = in_d[t];
  out_i[rows[i] * k + c] = in_i[t];
}

// ---------------------------------------------------------------------------------------------
// K12 `k_pf_scan_r` — the pre-filter scan with REGISTER-resident query tiles.
//
// K10 keeps a 64-query tile in LDS and streams rows into VGPRs, so every row read from HBM/L2 feeds
// 64 queries and the scan needs 64 B/clk/CU at the MFMA rate. K12 swaps the roles: one workgroup of
// 8 waves per CU, persistent over (list, chunk, 128-query tile) items; wave w holds queries
// 32(w&3)..+31 of the tile as the MFMA B operand in registers for ONE HALF of the dims (k-steps
// [(w>>2)NK/2, ...), 96 VGPRs at d = 768), so a wave pair (w, w^4) covers 32 queries x all dims at
// two waves per SIMD. The chunk's fp16 32-row groups are staged HBM -> VGPR ring (two groups ahead)
// -> LDS double buffer; each wave reads its half of each k-step's A operand once from LDS (inline-asm
// ds_read, counted lgkmcnt). A row read from HBM/L2 thus feeds 128 queries (32 B/clk/CU at the MFMA
// rate). Per group the pair exchanges half of its 32x32 partial dots through LDS (2 KiB per wave), so
// each wave finishes 8 of the 16 keys per lane; the filter + exact insertion of group g run during
// group g+1 (two accumulators). Per query the 4 lane lists (row quarter h, dh) of kPrLaneK keys go to
// one slot of 32 candidates + a lower bound of every key dropped; K11 then refines as for K10.
// The two partial sums add in a different order than one MFMA chain: the approximate keys stay
// within pf_delta (its MFMA term bounds any summation order).
// ---------------------------------------------------------------------------------------------
constexpr int kPrWaves = 8;
constexpr int kPrThreads = kPrWaves * 64;
constexpr int kPrLaneK = 4;
constexpr int kPrLists = 4;  // lane lists per query: row half h x dim half dh
static_assert(kPrLists * kPrLaneK == kPrSlotK, "K12 slot size");

__host__ __device__ constexpr int pr_waitcnt(int vm, int lgkm) {
  return (vm & 0xF) | (((vm >> 4) & 3) << 14) | (0x7 << 4) | ((lgkm & 0xF) << 8);
}

// lk[k-1] as a select chain (the empty asm keeps hipcc from turning it into an indexed load, which
// would put the list in scratch memory)
template <int KL>
__device__ __forceinline__ float pr_kth(const float (&lk)[KL], int k) {
  float v = lk[0];
#pragma unroll
  for (int t = 1; t < KL; ++t) {
    v = (t == k - 1) ? lk[t] : v;
    asm volatile("" : "+v"(v));
  }
  return v;
}

// two 16-B LDS reads in one inline-asm statement with its own lgkmcnt(0) (a plain ds_read here makes
// hipcc wait for the counted A reads in flight; offsets in bytes)
__device__ __forceinline__ void pr_ld8(unsigned addr0, unsigned addr1, float (&v)[8]) {
  float4 t0, t1;
  asm volatile(
      "ds_read_b128 %0, %2\n\t"
      "ds_read_b128 %1, %3\n\t"
      "s_waitcnt lgkmcnt(0)"
      : "=&v"(t0), "=&v"(t1)
      : "v"(addr0), "v"(addr1)
      : "memory");
  v[0] = t0.x; v[1] = t0.y; v[2] = t0.z; v[3] = t0.w;
  v[4] = t1.x; v[5] = t1.y; v[6] = t1.z; v[7] = t1.w;
}

__device__ __forceinline__ unsigned lds_off(const void* p) { return (unsigned)(uintptr_t)p; }

// compile-time loop: f(std::integral_constant<int, I>) for I = 0..N-1 (immediate LDS offsets in asm)
template <typename F, int... I>
__device__ __forceinline__ void pr_sfor_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void pr_sfor(F&& f) {
  pr_sfor_impl(f, std::make_integer_sequence<int, N>{});
}
template <int OFF>
__device__ __forceinline__ void pr_ds_read(h8& d, unsigned addr) {
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(d) : "v"(addr), "i"(OFF));
}
template <int N>
__device__ __forceinline__ void pr_lgkm(h8& d) {
  asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(d) : "i"(N));
}

// shader-clock stamp with its own lgkmcnt(0) (s_memtime returns out of order with LDS reads)
__device__ __forceinline__ unsigned long long pr_stamp() {
  unsigned long long t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
  return t;
}

template <int METRIC, int NK>
__global__ __launch_bounds__(kPrThreads, 1) void k_pf_scan_r(PfScanArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int GB = NK * 1024;       // bytes of one fp16 group
  constexpr int NH = NK / 2;          // k-steps of one dim half
  constexpr int NPW = NK / kPrWaves;  // k-step pieces each wave stages per group
  constexpr int NLOAD = NPW + 1;      // + the group's norms
  constexpr int DP = NK * 16;
  static_assert(NK % kPrWaves == 0 && NLOAD <= NH, "piece schedule");
  char* s_grp = smem;                                           // [2][GB] group double buffer
  float* s_x = reinterpret_cast<float*>(smem + 2 * GB);         // [2][8 waves][64 lanes][8] partial dots
  float* s_nrm = s_x + 2 * kPrWaves * 64 * 8;                   // [4][64] norms ring
  int* s_misc = reinterpret_cast<int*>(s_nrm + 4 * 64);
  // item-end scratch (aliases the group buffers): keys/pos [128 q][4 lists][8], bounds [128][4]
  float* s_ok = reinterpret_cast<float*>(smem);
  int* s_op = reinterpret_cast<int*>(s_ok + kPrQTile * kPrLists * kPrLaneK);
  float* s_ob = reinterpret_cast<float*>(s_op + kPrQTile * kPrLists * kPrLaneK);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int qb = wave & 3, dh = wave >> 2;
  const int j = lane & 31;
  const int h = lane >> 5;
  const int total = a.work_off[a.n_lists];
  const int grp = blockIdx.x & 7;
  const float xnmax2 = a.x_norm_max * a.x_norm_max;
  if (tid == 0) s_misc[1] = 0;
  // diagnostic phase clocks (a.prof only under MIVS_PF_FLAGS & 32): [0] fetch, [1] setup, [2] group loop,
  // [3] tail + output, [5] groups, [6] slow passes, [7] wave-cycles, [8] 100 MHz ticks
  unsigned long long pr_acc[4] = {0, 0, 0, 0}, pr_groups = 0, pr_slow = 0;
  const unsigned long long pr_t0 = a.prof ? pr_stamp() : 0;
  const unsigned long long pr_r0 = a.prof ? __builtin_amdgcn_s_memrealtime() : 0;

  for (;;) {
    const unsigned long long pa = a.prof ? pr_stamp() : 0;
    if (tid == 0) {
      int qs = s_misc[1], w = total;
      while (qs < 8) {
        const int g = (grp + qs) & 7;
        const int lo_g = (int)((int64_t)total * g / 8), hi_g = (int)((int64_t)total * (g + 1) / 8);
        const int i = atomicAdd(a.work_counter + 16 * g, 1);
        if (lo_g + i < hi_g) { w = lo_g + i; break; }
        ++qs;
      }
      s_misc[1] = qs;
      s_misc[0] = w;
    }
    __syncthreads();
    const int w = s_misc[0];
    if (w >= total) break;
    const unsigned long long pb = a.prof ? pr_stamp() : 0;
    int lo = 0, hi = a.n_lists - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (a.work_off[mid] <= w) lo = mid; else hi = mid - 1;
    }
    const int l = lo;
    const int m = a.bucket_off[l + 1] - a.bucket_off[l];
    const int tiles = (m + kPrQTile - 1) / kPrQTile;
    const int local = w - a.work_off[l];
    const int chunk = local / tiles;
    const int tile = local - chunk * tiles;
    const int64_t g_begin = a.list_goff[l] + (int64_t)chunk * a.chunk_groups;
    const int64_t g_lim = a.list_goff[l + 1];
    const int ng = (int)((g_begin + a.chunk_groups < g_lim ? g_begin + a.chunk_groups : g_lim) - g_begin);
    const int e0 = a.bucket_off[l] + tile * kPrQTile;
    const int nqt = m - tile * kPrQTile < kPrQTile ? m - tile * kPrQTile : kPrQTile;

    // this lane's query (an empty slot computes on query row 0 with th = -inf: nothing is kept)
    const int qi = qb * 32 + j;
    int64_t q = -1;
    float qn = INFINITY, qs = 0.0f, dl = 0.0f, th = -INFINITY;
    if (qi < nqt) {
      q = a.bucket_q[e0 + qi];
      qn = a.qnorms[q];
      qs = a.qscale[q];
      dl = pf_delta<METRIC>(qn, a.qres[q], a.x_norm_max, a.x_res_max, DP);
      th = pf_unord(__hip_atomic_load(a.qtheta + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    }
    h8 qr[NH];
    {
      const uint16_t* qp = a.qh + (q >= 0 ? q : 0) * (int64_t)DP + 16 * (dh * NH) + 8 * h;
#pragma unroll
      for (int t = 0; t < NH; ++t) qr[t] = ld_h8(qp + 16 * t);
    }
    const float mq = METRIC == kL2 ? -2.0f * qs : -qs;
    float lk[kPrLaneK];
    int lp[kPrLaneK];
#pragma unroll
    for (int t = 0; t < kPrLaneK; ++t) { lk[t] = INFINITY; lp[t] = INT_MAX; }
    float uf = pf_uf<METRIC>(INFINITY, th, qn, xnmax2);

    // register-staged row ring: piece i of a group (k-step wave*NPW + i) is loaded two groups ahead and
    // written to the LDS buffer of the next group while this group's MFMAs run (loads past the chunk end
    // are clamped to its last group, so the steady-state vmcnt is one constant)
    const uint16_t* gsrc = a.groups_h + g_begin * (int64_t)(NK * 512) + (wave * NPW) * 512 + lane * 8;
    const float* nsrc = a.row_norms + g_begin * kGroupRows + j;
    h8 rs0[NPW], rs1[NPW];
    float rn0, rn1;
    auto load_piece = [&](h8 (&rs)[NPW], int gg, int i) {
      const int gc = gg < ng ? gg : ng - 1;
      rs[i] = ld_h8(gsrc + (int64_t)gc * (NK * 512) + i * 512);
    };
    auto load_norm = [&](float& rn, int gg) {
      const int gc = gg < ng ? gg : ng - 1;
      rn = nsrc[(int64_t)gc * kGroupRows];
    };
    auto write_piece = [&](const h8 (&rs)[NPW], int gg, int i) {
      *reinterpret_cast<h8*>(s_grp + (gg & 1) * GB + (wave * NPW + i) * 1024 + lane * 16) = rs[i];
    };
    auto write_norm = [&](float rn, int gg) { s_nrm[(gg & 3) * 64 + lane] = rn; };
#pragma unroll
    for (int i = 0; i < NPW; ++i) load_piece(rs0, 0, i);
    load_norm(rn0, 0);
#pragma unroll
    for (int i = 0; i < NPW; ++i) write_piece(rs0, 0, i);
    write_norm(rn0, 0);
#pragma unroll
    for (int i = 0; i < NPW; ++i) load_piece(rs1, 1, i);
    load_norm(rn1, 1);
#pragma unroll
    for (int i = 0; i < NPW; ++i) load_piece(rs0, 2, i);
    load_norm(rn0, 2);

    const f32x16 zero = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    f32x16 acc = zero;
    float keep[8];  // this wave's half of the previous group's dots (the partner's half arrives via LDS)
    // rows of dot i of this lane: r = 8 dh + i -> (r & 3) + 8 (r >> 2) + 4 h
    const unsigned nrm_off = (unsigned)(16 * dh + 4 * h) * 4;
    // group gg's 8 approximate dots of this lane: this wave's half of `prev` + the partner's exchanged half
    auto dots = [&](int gg, float (&v)[8]) {
      float px[8];
      const unsigned xo = lds_off(s_x + (((gg & 1) * kPrWaves + (wave ^ 4)) * 64 + lane) * 8);
      pr_ld8(xo, xo + 16, px);
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = keep[i] + px[i];
    };
    // the one-fma filter: may any key of this wave pass the exact test?
    auto finish = [&](int gg) -> bool {
      float v[8], xn[8];
      dots(gg, v);
      const unsigned no = lds_off(s_nrm + (gg & 3) * 64) + nrm_off;
      pr_ld8(no, no + 32, xn);
      float mn = INFINITY;
#pragma unroll
      for (int i = 0; i < 8; ++i) mn = fminf(mn, fmaf(v[i], mq, METRIC == kL2 ? xn[i] : 0.0f));
      return __ballot(mn < uf) != 0;
    };
    auto slow = [&](int gg) {
      float v[8], xn[8];
      dots(gg, v);
      const unsigned no = lds_off(s_nrm + (gg & 3) * 64) + nrm_off;
      pr_ld8(no, no + 32, xn);
      const int64_t rb = (g_begin + gg) * kGroupRows + 16 * dh + 4 * h;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float key = pf_key<METRIC>(v[i], qs, xn[i], qn);
        if (key < lk[kPrLaneK - 1] && key <= th) pf_insert<kPrLaneK>(lk, lp, key, (int)(rb + (i & 3) + 8 * (i >> 2)));
      }
      if (a.k <= kPrLaneK) {
        const float kth = pr_kth<kPrLaneK>(lk, a.k);
        if (kth < INFINITY) th = fminf(th, pf_window(kth, dl));
      }
      uf = pf_uf<METRIC>(lk[kPrLaneK - 1], th, qn, xnmax2);
    };
    // the half of `acc` the partner finishes, to LDS (group gg's exchange buffer); this wave's half to keep
    auto exchange = [&](int gg) {
      float* xp = s_x + (((gg & 1) * kPrWaves + wave) * 64 + lane) * 8;
      float e[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float lo_ = acc[i], hi_ = acc[8 + i];
        asm volatile("" : "+v"(lo_), "+v"(hi_));  // keeps hipcc from indexing the vector by dh (s_set_gpr_idx)
        e[i] = dh ? lo_ : hi_;
        keep[i] = dh ? hi_ : lo_;
      }
      *reinterpret_cast<float4*>(xp) = make_float4(e[0], e[1], e[2], e[3]);
      *reinterpret_cast<float4*>(xp + 4) = make_float4(e[4], e[5], e[6], e[7]);
    };

    // one group: barrier (its LDS rows and group g-1's exchange are in), this wave's NH MFMAs with the
    // next group's staging and group g-1's filter interleaved, group g-1's exact pass if a lane hit,
    // then this group's exchange
    auto body = [&](h8 (&rs)[NPW], float& rn, int g) {
      asm volatile("" ::: "memory");
      __builtin_amdgcn_s_waitcnt(pr_waitcnt(63, 0));
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      const unsigned abase = lds_off(s_grp + (g & 1) * GB) + (dh * NH) * 1024 + lane * 16;
      constexpr int PD = 2;  // A reads in flight ahead of the MFMA (two waves per SIMD hide the rest)
      h8 ab[PD + 1];
      pr_sfor<PD>([&](auto T) { pr_ds_read<decltype(T)::value * 1024>(ab[decltype(T)::value], abase); });
      acc = zero;
      bool hit = false;
      pr_sfor<NH>([&](auto T) {
        constexpr int t = decltype(T)::value;
        if constexpr (t + PD < NH) pr_ds_read<(t + PD) * 1024>(ab[(t + PD) % (PD + 1)], abase);
        pr_lgkm<(NH - 1 - t < PD ? NH - 1 - t : PD)>(ab[t % (PD + 1)]);  // A reads issued after this one
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ab[t % (PD + 1)], qr[t], acc, 0, 0, 0);
        // the NLOAD staging ops: group g+1 from registers to LDS, the registers reloaded with group g+3
        pr_sfor<NLOAD>([&](auto P) {
          constexpr int p = decltype(P)::value;
          if constexpr (t == 1 + p * (NH - 1) / NLOAD) {
            if constexpr (p < NPW) {
              write_piece(rs, g + 1, p);
              load_piece(rs, g + 3, p);
            } else {
              write_norm(rn, g + 1);
              load_norm(rn, g + 3);
            }
          }
        });
        if constexpr (t == (NH > 4 ? 4 : NH - 1)) {
          if (g > 0) hit = finish(g - 1);
        }
      });
      if (hit) {
        slow(g - 1);
        if (a.prof) ++pr_slow;
      }
      exchange(g);
    };

    const unsigned long long pc = a.prof ? pr_stamp() : 0;
    int g = 0;
    for (; g + 1 < ng; g += 2) {
      body(rs1, rn1, g);
      body(rs0, rn0, g + 1);
    }
    if (g < ng) body(rs1, rn1, g);
    // the last group's keys: its exchange is in after one more barrier
    __builtin_amdgcn_s_waitcnt(pr_waitcnt(0, 0));  // the tail's loads (clamped re-loads) and LDS writes
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (finish(ng - 1)) slow(ng - 1);
    const unsigned long long pd = a.prof ? pr_stamp() : 0;

    // per query: the 4 lane lists -> the slot (4 x kPrLaneK candidates, unsorted), the dropped-key bound,
    // and the window above the k-th kept key into qtheta
    __syncthreads();  // every wave is done with the group buffers (the scratch aliases them)
    {
      const int li = dh * 2 + h;
      float* ok = s_ok + (qi * kPrLists + li) * kPrLaneK;
      int* op = s_op + (qi * kPrLists + li) * kPrLaneK;
#pragma unroll
      for (int t = 0; t < kPrLaneK; ++t) { ok[t] = lk[t]; op[t] = lp[t]; }
      s_ob[qi * kPrLists + li] = fminf(lk[kPrLaneK - 1], nextafterf(th, INFINITY));
    }
    __syncthreads();
    if (tid < nqt) {
      const int64_t qq = a.bucket_q[e0 + tid];
      const int64_t slot = a.bucket_slot[e0 + tid] + chunk;
      const float* ok = s_ok + tid * kPrLists * kPrLaneK;
      const int* op = s_op + tid * kPrLists * kPrLaneK;
      float* dk = a.slot_key + slot * (kPrLists * kPrLaneK);
      int* dp_ = a.slot_pos + slot * (kPrLists * kPrLaneK);
      for (int t = 0; t < kPrLists * kPrLaneK; t += 4) {
        *reinterpret_cast<float4*>(dk + t) = *reinterpret_cast<const float4*>(ok + t);
        *reinterpret_cast<int4*>(dp_ + t) = *reinterpret_cast<const int4*>(op + t);
      }
      const float4 b4 = *reinterpret_cast<const float4*>(s_ob + tid * kPrLists);
      a.slot_bound[slot] = fminf(fminf(b4.x, b4.y), fminf(b4.z, b4.w));
      // k-th smallest kept key (rank count over the slot; ties broken by position in the scratch)
      float kth = INFINITY;
      for (int c = 0; c < kPrLists * kPrLaneK && !a.no_theta; ++c) {
        const float v = ok[c];
        if (!(v < kth)) continue;
        int rank = 0;
        for (int e = 0; e < kPrLists * kPrLaneK; ++e) rank += (ok[e] < v || (ok[e] == v && e < c)) ? 1 : 0;
        if (rank == a.k - 1) kth = v;
      }
      if (kth < INFINITY) {
        const float qn2 = a.qnorms[qq];
        atomicMin(a.qtheta + qq, pf_ord(pf_window(kth, pf_delta<METRIC>(qn2, a.qres[qq], a.x_norm_max,
                                                                        a.x_res_max, DP))));
      }
    }
    __syncthreads();
    if (a.prof) {
      const unsigned long long pe = pr_stamp();
      pr_acc[0] += pb - pa; pr_acc[1] += pc - pb; pr_acc[2] += pd - pc; pr_acc[3] += pe - pd;
      pr_groups += ng;
    }
  }
  if (a.prof && lane == 0) {
    atomicAdd(a.prof + 0, pr_acc[0]); atomicAdd(a.prof + 1, pr_acc[1]); atomicAdd(a.prof + 2, pr_acc[2]);
    atomicAdd(a.prof + 3, pr_acc[3]); atomicAdd(a.prof + 5, pr_groups); atomicAdd(a.prof + 6, pr_slow);
    atomicAdd(a.prof + 7, pr_stamp() - pr_t0);
    atomicAdd(a.prof + 8, __builtin_amdgcn_s_memrealtime() - pr_r0);
  }
}

// K11 for k = 1 (the pre-filter assign): one LANE per query. The window is
// min approx key + 2 delta; its candidates (1-3 at k-means shapes) get the pinned fp32 key (the same
// chain as K11 / orc_dot, the query read from global), the smallest (key, id) is the label.
template <int METRIC>
__global__ __launch_bounds__(256) void k_pf_refine1(PfRefineArgs a) {
  const int64_t q0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool live = q0 < a.nq;  // (every lane reaches the wave reduction below)
  const int64_t q = live ? q0 : a.nq - 1;
  const int64_t qrow = a.qrows ? a.qrows[q] : q;
  const int64_t sb = live ? a.slot_begin[q] : 0, se = live ? a.slot_begin[q + 1] : 0;
  float ak = INFINITY, bmin = INFINITY;
  for (int64_t sl = sb; sl < se; ++sl) {
    bmin = fminf(bmin, a.slot_bound[sl]);
    const float* kp = a.slot_key + sl * a.slot_k;
    for (int t = 0; t < a.slot_k; t += 4) {
      const float4 v = *reinterpret_cast<const float4*>(kp + t);
      ak = fminf(fminf(ak, v.x), fminf(fminf(v.y, v.z), v.w));
    }
  }
  const float qn = a.qnorms[qrow];
  const float T = pf_window(ak, pf_delta<METRIC>(qn, a.qres[qrow], a.x_norm_max, a.x_res_max, a.dp));
  bool ovf = live && (!(ak < INFINITY) || (bmin < INFINITY && bmin <= T));
  float bestP = INFINITY;
  int64_t bestId = LLONG_MAX;
  int cnt = 0;
  const int nb = a.dp >> 3;
  const float* qv = a.queries + qrow * a.d;
  const bool vec = (a.d & 7) == 0 && (reinterpret_cast<uintptr_t>(qv) & 15) == 0;
  bool done = false;
  if (a.labels_only && !ovf) {
    // the true top-1 is inside the window: a window of one candidate needs no exact key
    int64_t only = -1;
    float only_k = INFINITY;
    for (int64_t sl = sb; sl < se && cnt < 2; ++sl)
      for (int t = 0; t < a.slot_k; ++t) {
        const float key = a.slot_key[sl * a.slot_k + t];
        if (key <= T) {
          ++cnt;
          only = sl * a.slot_k + t;
          only_k = key;
        }
      }
    if (cnt == 1) {
      bestP = only_k;
      bestId = a.row_ids[a.slot_pos[only]];
      done = true;
    }
    if (cnt != 1) cnt = 0;  // 0 or >= 2 candidates: the exact pass below decides
  }
  for (int64_t sl = sb; sl < se && !ovf && !done; ++sl) {
    for (int t = 0; t < a.slot_k; ++t) {
      const float key = a.slot_key[sl * a.slot_k + t];
      if (!(key <= T)) continue;
      if (++cnt > kPfCap) { ovf = true; break; }
      const int pos = a.slot_pos[sl * a.slot_k + t];
      const float* rowp = a.groups + row_elem(pos, 0, a.dp);
      float acc = 0.0f;
      for (int b = 0; b < nb; ++b) {
        const float4 x0 = *reinterpret_cast<const float4*>(rowp + row_blk8(b));
        const float4 x1 = *reinterpret_cast<const float4*>(rowp + row_blk8(b) + 4);
        float y[8];
        if (vec) {
          const float4 y0 = *reinterpret_cast<const float4*>(qv + 8 * b);
          const float4 y1 = *reinterpret_cast<const float4*>(qv + 8 * b + 4);
          y[0] = y0.x; y[1] = y0.y; y[2] = y0.z; y[3] = y0.w; y[4] = y1.x; y[5] = y1.y; y[6] = y1.z; y[7] = y1.w;
        } else {
#pragma unroll
          for (int i = 0; i < 8; ++i) y[i] = 8 * b + i < a.d ? qv[8 * b + i] : 0.0f;
        }
        acc = fmaf(x0.x, y[0], acc); acc = fmaf(x1.x, y[4], acc);
        acc = fmaf(x0.y, y[1], acc); acc = fmaf(x1.y, y[5], acc);
        acc = fmaf(x0.z, y[2], acc); acc = fmaf(x1.z, y[6], acc);
        acc = fmaf(x0.w, y[3], acc); acc = fmaf(x1.w, y[7], acc);
      }
      float P;
      if (METRIC == kL2) {
        const float v = fmaf(-2.0f, acc, a.row_norms[pos] + qn);
        P = v > 0.0f ? v : 0.0f;
      } else {
        P = -acc;
      }
      const int64_t id = a.row_ids[pos];
      if (P < bestP || (P == bestP && id < bestId)) { bestP = P; bestId = id; }
    }
  }
  if (a.n_window) {  // window candidates of the proven queries (stats), one atomic per wave
    unsigned long long c = ovf ? 0ull : (unsigned long long)cnt;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) c += __shfl_xor(c, off);
    if ((threadIdx.x & 63) == 0) atomicAdd(reinterpret_cast<unsigned long long*>(a.n_window), c);
  }
  if (!live) return;
  if (ovf) {
    const int at = atomicAdd(a.ovf_count, 1);
    a.ovf_q[at] = q;
    return;
  }
  const bool valid = bestId != LLONG_MAX;
  a.out_d[q] = valid ? (METRIC == kIP ? -bestP : bestP) : (METRIC == kIP ? -INFINITY : INFINITY);
  a.out_i[q] = valid ? bestId : (int64_t)-1;
}

__global__ void k_gather_ids(const int64_t* __restrict__ src, const int64_t* __restrict__ idx, int64_t n,
                             int64_t* __restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n) out[t] = src[idx[t]];
}

inline dim3 pf_grid(int64_t n, int b) { return dim3((unsigned)ceil_div(n > 0 ? n : 1, b)); }

}  // namespace

int pf_hx_exp(float abs_max) {
  if (!(abs_max > 0.0f) || !(abs_max < INFINITY)) return 0;
  const int e = 14 - ilogbf(abs_max);
  return e < -60 ? -60 : (e > 60 ? 60 : e);
}

bool pf_pair_mode() { return true; }

size_t pf_scan_lds_bytes(int dp, int chunk_groups) {
  const size_t b = (size_t)dp * kPfQTile * 2;
  (void)chunk_groups;  // the row norms go through a per-wave slot: any chunk length fits
  const size_t norms = (size_t)kPfWaves * 64 * 4;
  return kPfSmall + (size_t)kPfQTile * 18 * 4 + norms + (b > (size_t)kPfMergeBytes ? b : (size_t)kPfMergeBytes);
}

template <int METRIC, int D, int R, bool NT = false, bool F8 = false>
static hipError_t launch_pf_scan_md(const PfScanArgs& a, int grid, size_t lds, hipStream_t s) {
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_pf_scan<METRIC, D, R, NT, F8>),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  if (attr != hipSuccess) return attr;
  hipLaunchKernelGGL((k_pf_scan<METRIC, D, R, NT, F8>), dim3(grid), dim3(kPfThreads), lds, s, a);
  return hipGetLastError();
}

template <int METRIC>
static hipError_t launch_pf_scan_m(const PfScanArgs& a, int grid, size_t lds, hipStream_t s) {
  // two groups per pass with 6-deep rings (half the LDS operand traffic per flop: the kernel is power-bound,
  // DESIGN.md §6.2; one group per pass with a 16-deep ring measured slower and was retired in round 5)
  if (a.groups_f8) {  // fp8 nomination (pair mode): superblocks of 32 dims, a ring of 6 or 4
    const int nsb = a.dp / 32;
    if (a.q8 == nullptr || a.qscale8 == nullptr) return hipErrorInvalidValue;
    if (nsb % 6 == 0) return launch_pf_scan_md<METRIC, 6, 2, true, true>(a, grid, lds, s);
    if (nsb % 4 == 0) return launch_pf_scan_md<METRIC, 4, 2, true, true>(a, grid, lds, s);
    return hipErrorInvalidValue;
  }
  const int nk = a.dp / 16;
  if (a.rows_nt && nk % 6 == 0) return launch_pf_scan_md<METRIC, 6, 2, true>(a, grid, lds, s);
  return nk % 6 == 0 ? launch_pf_scan_md<METRIC, 6, 2>(a, grid, lds, s) : launch_pf_scan_md<METRIC, 4, 2>(a, grid, lds, s);
}

// grid: a multiple of 8 (one queue per XCD group); the work counters (8 x 16 ints) are zeroed by the caller
hipError_t launch_pf_scan(const PfScanArgs& a, int grid, size_t lds, hipStream_t s) {
  if (a.dp % 64 != 0 || a.dp > 1024 || lds > 160 * 1024) return hipErrorInvalidValue;
  if (a.k < 1 || a.k > 4 * kPfLaneK || a.k > a.slot_k) return hipErrorInvalidValue;  // (pf_theta: 4 lane lists)
  if (a.raw_lists && a.slot_k != 16 * kPfLaneK) return hipErrorInvalidValue;          // (a slot = the 16 lane lists)
  return a.metric == kIP ? launch_pf_scan_m<kIP>(a, grid, lds, s) : launch_pf_scan_m<kL2>(a, grid, lds, s);
}

size_t pr_scan_lds_bytes(int dp) { return (size_t)2 * dp * 64 + 2 * kPrWaves * 64 * 8 * 4 + 4 * 64 * 4 + 16; }

bool pr_scan_supported(int dp) {
  const int nk = dp / 16;
  return dp % 64 == 0 && (nk == 8 || nk == 16 || nk == 24 || nk == 32 || nk == 40 || nk == 48) &&
         pr_scan_lds_bytes(dp) <= 160 * 1024;
}

template <int METRIC, int NK>
static hipError_t launch_pr_scan_mk(const PfScanArgs& a, int grid, hipStream_t s) {
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_pf_scan_r<METRIC, NK>),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  if (attr != hipSuccess) return attr;
  hipLaunchKernelGGL((k_pf_scan_r<METRIC, NK>), dim3(grid), dim3(kPrThreads), pr_scan_lds_bytes(NK * 16), s, a);
  return hipGetLastError();
}

template <int METRIC>
static hipError_t launch_pr_scan_m(const PfScanArgs& a, int grid, hipStream_t s) {
  switch (a.dp / 16) {
    case 8: return launch_pr_scan_mk<METRIC, 8>(a, grid, s);
    case 16: return launch_pr_scan_mk<METRIC, 16>(a, grid, s);
    case 24: return launch_pr_scan_mk<METRIC, 24>(a, grid, s);
    case 32: return launch_pr_scan_mk<METRIC, 32>(a, grid, s);
    case 40: return launch_pr_scan_mk<METRIC, 40>(a, grid, s);
    case 48: return launch_pr_scan_mk<METRIC, 48>(a, grid, s);
    default: return hipErrorInvalidValue;
  }
}

// grid: a multiple of 8 (one queue per XCD group), one workgroup per CU; work counters zeroed by the caller;
// the probe map was built with kPrQTile-query tiles, slots hold kPrSlotK candidates
hipError_t launch_pr_scan(const PfScanArgs& a, int grid, hipStream_t s) {
  if (!pr_scan_supported(a.dp) || a.slot_k != kPrSlotK || a.k < 1 || a.k > kPfMaxK)
    return hipErrorInvalidValue;
  return a.metric == kIP ? launch_pr_scan_m<kIP>(a, grid, s) : launch_pr_scan_m<kL2>(a, grid, s);
}

hipError_t launch_pf_refine(const PfRefineArgs& a, hipStream_t s) {
  if (a.k < 1 || a.k > kPfRefineMaxK || a.dp > 1024) return hipErrorInvalidValue;  // (k > 16: the coarse probe)
  if (a.nq <= 0) return hipSuccess;
  if (a.k == 1 && a.slot_k % 4 == 0 && a.force_ovf == nullptr && a.kth_out == nullptr && a.slot_bound != nullptr) {  // lane per query
    if (a.metric == kIP) hipLaunchKernelGGL(k_pf_refine1<kIP>, pf_grid(a.nq, 256), dim3(256), 0, s, a);
    else hipLaunchKernelGGL(k_pf_refine1<kL2>, pf_grid(a.nq, 256), dim3(256), 0, s, a);
    return hipGetLastError();
  }
  if (a.kth_out && a.verify_sel > 0) {
    if (a.metric == kIP) hipLaunchKernelGGL(k_pf_verify<kIP>, pf_grid(a.nq, 4), dim3(256), 0, s, a);
    else hipLaunchKernelGGL(k_pf_verify<kL2>, pf_grid(a.nq, 4), dim3(256), 0, s, a);
    return hipGetLastError();
  }
  if (a.metric == kIP) hipLaunchKernelGGL(k_pf_refine<kIP>, pf_grid(a.nq, 4), dim3(256), 0, s, a);
  else hipLaunchKernelGGL(k_pf_refine<kL2>, pf_grid(a.nq, 4), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_groups_to_half(const float* groups, int64_t n_groups, int dp, int hx_exp, uint16_t* out,
                                 unsigned* stats, hipStream_t s) {
  if (n_groups <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_groups_to_half, pf_grid(n_groups * kGroupRows, 256), dim3(256), 0, s, groups, n_groups, dp,
                     hx_exp, out, stats);
  return hipGetLastError();
}

// fp8 (e4m3) copies for K13's pre-pass nomination (k_pf_scan<.., F8>): rows at 2^hx8, a query at its own
// 2^qexp (its |q| max in [128, 256)); piece (S, j, h) of a group = dims 32 S + 8 h .. + 7 and 32 S + 16 + 8 h ..
// + 7 of row j: the A operands of k-steps 2 S and 2 S + 1 of v_mfma_f32_32x32x16_fp8_fp8 for lane (j, h)
__device__ __forceinline__ uint4 f8_pack16(const float (&v)[16], float sc) {
  int w[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int x = __builtin_amdgcn_cvt_pk_fp8_f32(v[4 * i] * sc, v[4 * i + 1] * sc, 0, false);
    w[i] = __builtin_amdgcn_cvt_pk_fp8_f32(v[4 * i + 2] * sc, v[4 * i + 3] * sc, x, true);
  }
  return make_uint4((unsigned)w[0], (unsigned)w[1], (unsigned)w[2], (unsigned)w[3]);
}

__global__ void k_groups_to_f8(const float* __restrict__ groups, int64_t n_groups, int dp, int hx8,
                               uint8_t* __restrict__ out) {
  const int nsb = dp >> 5;
  const int64_t n = n_groups * nsb * 64;
  const float sc = ldexpf(1.0f, hx8);
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t g = t / (nsb * 64);
    const int rem = (int)(t - g * (nsb * 64));
    const int S = rem >> 6, jj = (rem & 63) >> 1, hh = rem & 1;
    float v[16];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const float* src = groups + row_elem(g * kGroupRows + jj, 0, dp) + row_blk8(4 * S + 2 * e + hh);
      const float4 x0 = *reinterpret_cast<const float4*>(src), x1 = *reinterpret_cast<const float4*>(src + 4);
      v[8 * e + 0] = x0.x; v[8 * e + 1] = x0.y; v[8 * e + 2] = x0.z; v[8 * e + 3] = x0.w;
      v[8 * e + 4] = x1.x; v[8 * e + 5] = x1.y; v[8 * e + 6] = x1.z; v[8 * e + 7] = x1.w;
    }
    __builtin_nontemporal_store(__builtin_bit_cast(pf_u32x4, f8_pack16(v, sc)), reinterpret_cast<pf_u32x4*>(out + t * 16));
  }
}

// one wave per query: its |q| max, then the pieces (S, h) of its fp8 row (zero past d) and qscale8 = 2^-(hx8 + qexp)
__global__ __launch_bounds__(256) void k_queries_to_f8(const float* __restrict__ q, int64_t nq, int d, int dp, int hx8,
                                                       uint8_t* __restrict__ out, float* __restrict__ qscale8) {
  const int lane = threadIdx.x & 63;
  const int64_t qi = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (qi >= nq) return;
  const float* row = q + qi * d;
  float m = 0.0f;
  for (int i = lane; i < d; i += 64) m = fmaxf(m, fabsf(row[i]));
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  const int e = (m > 0.0f && m < INFINITY) ? 7 - ilogbf(m) : 0;  // m 2^e in [128, 256)
  const float sc = ldexpf(1.0f, e);
  for (int pc = lane; pc < (dp >> 4); pc += 64) {  // piece pc = (S, h): 16 B
    const int S = pc >> 1, hh = pc & 1;
    float v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int c = 32 * S + 16 * (i >> 3) + 8 * hh + (i & 7);
      v[i] = c < d ? row[c] : 0.0f;
    }
    *reinterpret_cast<uint4*>(out + qi * dp + pc * 16) = f8_pack16(v, sc);
  }
  if (lane == 0) qscale8[qi] = ldexpf(1.0f, -(hx8 + e));
}

// The query batch's prep in one pass, each row read once: ||q||^2 (k_row_norms_w's chain), the fp16 copy, scale and
// residual bound (k_queries_to_half_v) and, with q8, the fp8 copy and scale (k_queries_to_f8). One wave per query;
// the row is staged in LDS for the norm chain and the fp8 pieces. (Three kernels had read the batch three times:
// 30 + 10 + 24 us per 10k x 768 batch.)
template <int NV>
__global__ __launch_bounds__(256) void k_queries_prep(const float* __restrict__ q, int64_t nq, int d, int dp, int hx_exp,
                                                      int hx8, float* __restrict__ qn, uint16_t* __restrict__ qh,
                                                      float* __restrict__ qscale, float* __restrict__ qres,
                                                      uint8_t* __restrict__ q8, float* __restrict__ qscale8) {
  extern __shared__ __attribute__((aligned(16))) float qp_t[];  // [4][dp]
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t qi = (int64_t)blockIdx.x * 4 + w;
  const bool live = qi < nq;
  float* my = qp_t + w * dp;
  const float4* row = reinterpret_cast<const float4*>(q + (live ? qi : 0) * d);
  float4 v[NV];
  float m = 0.0f;
#pragma unroll
  for (int u = 0; u < NV; ++u) {
    const int c4 = lane + 64 * u;
    v[u] = live && 4 * c4 < d ? row[c4] : make_float4(0.f, 0.f, 0.f, 0.f);
    m = fmaxf(m, fmaxf(fmaxf(fabsf(v[u].x), fabsf(v[u].y)), fmaxf(fabsf(v[u].z), fabsf(v[u].w))));
    if (4 * c4 < dp) *reinterpret_cast<float4*>(my + 4 * c4) = v[u];
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) m = fmaxf(m, __shfl_xor(m, off));
  // fp16 (k_queries_to_half_v)
  const int e = pf_exp_for(m);
  const float sc = ldexpf(1.0f, e), isc = ldexpf(1.0f, -e);
  float res = 0.0f;
#pragma unroll
  for (int u = 0; u < NV; ++u) {
    const int c4 = lane + 64 * u;
    if (4 * c4 < dp) {
      uint2 pk;
      pk.x = pf_to_half(v[u].x, sc, isc, res) | ((unsigned)pf_to_half(v[u].y, sc, isc, res) << 16);
      pk.y = pf_to_half(v[u].z, sc, isc, res) | ((unsigned)pf_to_half(v[u].w, sc, isc, res) << 16);
      if (live) *reinterpret_cast<uint2*>(qh + qi * dp + 4 * c4) = pk;
    }
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) res += __shfl_xor(res, off);
  if (live && lane == 0) {
    qscale[qi] = ldexpf(1.0f, -(hx_exp + e));
    qres[qi] = sqrtf(res) * (1.0f + 0x1p-12f);
  }
  __syncthreads();  // the staged rows
  if (live && lane == 0) {  // ||q||^2: k_row_norms_w's chain
    float acc = 0.0f;
    for (int s8 = 0; s8 < dp; s8 += 8) {
      const float4 a = *reinterpret_cast<const float4*>(my + s8), b = *reinterpret_cast<const float4*>(my + s8 + 4);
      acc = fmaf(a.x, a.x, acc); acc = fmaf(b.x, b.x, acc);
      acc = fmaf(a.y, a.y, acc); acc = fmaf(b.y, b.y, acc);
      acc = fmaf(a.z, a.z, acc); acc = fmaf(b.z, b.z, acc);
      acc = fmaf(a.w, a.w, acc); acc = fmaf(b.w, b.w, acc);
    }
    qn[qi] = acc;
  }
  if (live && q8) {  // fp8 (k_queries_to_f8): piece pc = (S, h) = dims 32 S + 16 (i >> 3) + 8 h + (i & 7)
    const int e8 = (m > 0.0f && m < INFINITY) ? 7 - ilogbf(m) : 0;
    const float sc8 = ldexpf(1.0f, e8);
    for (int pc = lane; pc < (dp >> 4); pc += 64) {
      const int S = pc >> 1, hh = pc & 1;
      float f[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) f[i] = my[32 * S + 16 * (i >> 3) + 8 * hh + (i & 7)];
      *reinterpret_cast<uint4*>(q8 + qi * dp + pc * 16) = f8_pack16(f, sc8);
    }
    if (lane == 0) qscale8[qi] = ldexpf(1.0f, -(hx8 + e8));
  }
}

hipError_t launch_queries_prep(const float* q, int64_t nq, int d, int dp, int hx_exp, int hx8, float* qn, uint16_t* qh,
                               float* qscale, float* qres, uint8_t* q8, float* qscale8, hipStream_t s) {
  if (nq <= 0) return hipSuccess;
  if ((d & 3) != 0 || (reinterpret_cast<uintptr_t>(q) & 15) != 0 || dp > 1024 || dp % 32 != 0 || d > dp)
    return hipErrorInvalidValue;
  const size_t lds = (size_t)4 * dp * sizeof(float);
  switch ((dp + 255) / 256) {
    case 1: hipLaunchKernelGGL(k_queries_prep<1>, pf_grid(nq, 4), dim3(256), lds, s, q, nq, d, dp, hx_exp, hx8, qn, qh, qscale, qres, q8, qscale8); break;
    case 2: hipLaunchKernelGGL(k_queries_prep<2>, pf_grid(nq, 4), dim3(256), lds, s, q, nq, d, dp, hx_exp, hx8, qn, qh, qscale, qres, q8, qscale8); break;
    case 3: hipLaunchKernelGGL(k_queries_prep<3>, pf_grid(nq, 4), dim3(256), lds, s, q, nq, d, dp, hx_exp, hx8, qn, qh, qscale, qres, q8, qscale8); break;
    default: hipLaunchKernelGGL(k_queries_prep<4>, pf_grid(nq, 4), dim3(256), lds, s, q, nq, d, dp, hx_exp, hx8, qn, qh, qscale, qres, q8, qscale8); break;
  }
  return hipGetLastError();
}

hipError_t launch_groups_to_f8(const float* groups, int64_t n_groups, int dp, int hx8, uint8_t* out, hipStream_t s) {
  if (n_groups <= 0) return hipSuccess;
  if (dp % 32 != 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_groups_to_f8, pf_grid(n_groups * (dp / 32) * 64, 256), dim3(256), 0, s, groups, n_groups, dp,
                     hx8, out);
  return hipGetLastError();
}

hipError_t launch_queries_to_f8(const float* q, int64_t nq, int d, int dp, int hx8, uint8_t* out, float* qscale8,
                                hipStream_t s) {
  if (nq <= 0) return hipSuccess;
  if (dp % 32 != 0 || d > dp) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_queries_to_f8, dim3((unsigned)ceil_div(nq, (int64_t)4)), dim3(256), 0, s, q, nq, d, dp, hx8,
                     out, qscale8);
  return hipGetLastError();
}

hipError_t launch_abs_max(const float* x, int64_t n, unsigned* out, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const int64_t blocks = ceil_div(n, 256) < 4096 ? ceil_div(n, 256) : 4096;
  hipLaunchKernelGGL(k_abs_max, dim3((unsigned)blocks), dim3(256), 0, s, x, n, out);
  return hipGetLastError();
}

hipError_t launch_norm_max(const float* x, int64_t n, unsigned* out, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const int64_t blocks = ceil_div(n, 256) < 4096 ? ceil_div(n, 256) : 4096;
  hipLaunchKernelGGL(k_norm_max, dim3((unsigned)blocks), dim3(256), 0, s, x, n, out);
  return hipGetLastError();
}

hipError_t launch_queries_to_half(const float* q, int64_t nq, int d, int dp, int hx_exp, uint16_t* qh, float* qscale,
                                  float* qres, hipStream_t s) {
  if (nq <= 0) return hipSuccess;
  const bool vec = (d & 3) == 0 && (reinterpret_cast<uintptr_t>(q) & 15) == 0 && dp <= 1024;
  const int nv = (dp + 255) / 256;
  if (vec && nv == 1) hipLaunchKernelGGL(k_queries_to_half_v<1>, pf_grid(nq, 4), dim3(256), 0, s, q, nq, d, dp, hx_exp, qh, qscale, qres);
  else if (vec && nv == 2) hipLaunchKernelGGL(k_queries_to_half_v<2>, pf_grid(nq, 4), dim3(256), 0, s, q, nq, d, dp, hx_exp, qh, qscale, qres);
  else if (vec && nv == 3) hipLaunchKernelGGL(k_queries_to_half_v<3>, pf_grid(nq, 4), dim3(256), 0, s, q, nq, d, dp, hx_exp, qh, qscale, qres);
  else if (vec && nv == 4) hipLaunchKernelGGL(k_queries_to_half_v<4>, pf_grid(nq, 4), dim3(256), 0, s, q, nq, d, dp, hx_exp, qh, qscale, qres);
  else hipLaunchKernelGGL(k_queries_to_half, pf_grid(nq, 4), dim3(256), 0, s, q, nq, d, dp, hx_exp, qh, qscale, qres);
  return hipGetLastError();
}

hipError_t launch_gather_ids(const int64_t* src, const int64_t* idx, int64_t n, int64_t* out, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_gather_ids, pf_grid(n, 256), dim3(256), 0, s, src, idx, n, out);
  return hipGetLastError();
}

hipError_t launch_scatter_results(const float* in_d, const int64_t* in_i, const int64_t* rows, int64_t n, int k,
                                  float* out_d, int64_t* out_i, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_scatter_results, pf_grid(n * k, 256), dim3(256), 0, s, in_d, in_i, rows, n, k, out_d, out_i);
  return hipGetLastError();
}

}  // namespace mivs
