// K8 — large-k selection (k in (64, 4096]; also n_probes > 64).
//
// The register top-k of the scan (K3) and of the wave merge (K7) stops at 64.
// For larger k the scan runs in DUMP mode: every (query, chunk) slot receives
// the raw ranking keys of the chunk's rows. This kernel then selects, per query
// (one 1024-thread workgroup), the k smallest candidates under the total order
// (key, id) — exactly the order the oracle and the k <= 64 path use:
//
//   pass 0      min / max of the orderable key bits + number of valid candidates
//   pass 1..    2048-bin histogram of the current key range, LINEAR in the
//               orderable bits (not radix digits: keys of one query crowd into a
//               few exponents, linear bins spread them and keep LDS atomics
//               uncontended); pick the bin holding the k-th candidate; stop as
//               soon as everything below it plus the bin fits in CAP slots,
//               else narrow the range to that bin (<= 3 passes for 32 bits)
//   ties        a range of ONE key value that still overflows CAP (duplicate
//               rows) is refined the same way over the ids of the tied rows
//   collect     candidates <= the final bound -> LDS (<= CAP), bitonic sort by
//               (key, id), write the first k; missing ranks get (id -1, +inf)
//               (IP: -inf) like every other path.
//
// Candidate sources: DUMP slots (keys [slot][slot_rows], slot_info = (first row
// position, rows) per slot, ids = row_ids[position]) or an EXPLICIT [nq][n_in]
// (dist, id) array (cross-shard merge of large k; id < 0 = missing), or EXPLICIT
// slots of n_in entries with slot_begin (K9r's per-chunk candidate supersets).
// Replaces the large-k select_k inside cuVS ivf_flat::search / brute_force (reference
// top_k = 2000, improved_multi_gpu_rag.py:65,247; 2*k per shard cuvs-2gpu-main.ipynb:1801).
#include <climits>
#include <cstdlib>

#include "mivs_common.hpp"

namespace mivs {

namespace {

constexpr int kSelThreads = 1024;
constexpr int kBins = 2048;

__device__ __forceinline__ uint32_t ord_bits(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float from_ord(uint32_t o) {
  return __uint_as_float((o & 0x80000000u) ? (o & 0x7FFFFFFFu) : ~o);
}
constexpr uint32_t kOrdInf = 0xFF800000u;  // ord_bits(+inf); every valid key is strictly below

struct Cand {
  uint32_t u;  // orderable key bits
  bool valid;
};

// Candidate c of query q (flattened index over the query's candidate range).
template <bool EXPLICIT, int METRIC>
__device__ __forceinline__ Cand cand_key(const SelectArgs& a, int64_t base, int64_t t) {
  Cand r;
  if (EXPLICIT) {
    const int64_t c = base + t;
    const float dd = a.keys[c];
    const float key = METRIC == kIP ? -dd : dd;
    r.u = ord_bits(key);
    // (K9r's candidate slots pad with +inf keys: the key alone decides, the 8-B ids are read only when collected)
    r.valid = r.u < kOrdInf && (a.slot_begin != nullptr || a.ids[c] >= 0);
  } else {
    // (t < a query's slots x slot_rows < 2^31: a 32-bit division, not the 64-bit one)
    const uint32_t sq = (uint32_t)t / (uint32_t)a.slot_rows;
    const int64_t s = base + sq;
    const int rr = (int)((uint32_t)t - sq * (uint32_t)a.slot_rows);
    r.valid = false;
    r.u = 0xFFFFFFFFu;
    if (rr < (int)a.slot_info[2 * s + 1]) {
      r.u = ord_bits(a.keys[s * a.slot_rows + rr]);
      r.valid = r.u < kOrdInf;  // pad rows carry +inf
    }
  }
  return r;
}

template <bool EXPLICIT>
__device__ __forceinline__ int64_t cand_id(const SelectArgs& a, int64_t base, int64_t t) {
  if (EXPLICIT) return a.ids[base + t];
  const uint32_t sq = (uint32_t)t / (uint32_t)a.slot_rows;
  const int64_t s = base + sq;
  const int rr = (int)((uint32_t)t - sq * (uint32_t)a.slot_rows);
  return a.row_ids[a.slot_info[2 * s] + rr];
}

// every candidate of a query, strided over the block: f(cand, id_of) with id_of() its id. DUMP slots are walked
// slot by slot over their valid rows, so no key pays cand_key's division of its flat index by slot_rows (a 64-bit
// division per key and pass: K8 over a k = 100 IVF-PQ dump of ~75k keys per query was bound by them)
// (four keys per thread and step, loaded before any is used: one at a time a pass waited on memory latency)
template <bool EXPLICIT, int METRIC, class F>
__device__ __forceinline__ void visit_cands(const SelectArgs& a, int64_t base, int64_t ncand, int64_t nslots, F&& f) {
  constexpr int U = 4;
  if constexpr (EXPLICIT) {
    for (int64_t t0 = threadIdx.x; t0 < ncand; t0 += U * kSelThreads) {
      Cand c[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t t = t0 + (int64_t)u * kSelThreads;
        c[u].valid = false;
        c[u].u = 0xFFFFFFFFu;
        if (t < ncand) c[u] = cand_key<true, METRIC>(a, base, t);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t t = t0 + (int64_t)u * kSelThreads;
        if (t < ncand) f(c[u], [&]() { return a.ids[base + t]; });
      }
    }
  } else {
    for (int64_t sq = 0; sq < nslots; ++sq) {
      const int64_t sl = base + sq;
      const int nr = (int)a.slot_info[2 * sl + 1];
      const int64_t r0 = a.slot_info[2 * sl];
      const float* kp = a.keys + sl * a.slot_rows;
      for (int rr0 = threadIdx.x; rr0 < nr; rr0 += U * kSelThreads) {
        float v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int rr = rr0 + u * kSelThreads;
          v[u] = rr < nr ? kp[rr] : INFINITY;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int rr = rr0 + u * kSelThreads;
          if (rr < nr) {
            Cand c;
            c.u = ord_bits(v[u]);
            c.valid = c.u < kOrdInf;  // pad rows carry +inf
            f(c, [&]() { return a.row_ids[r0 + rr]; });
          }
        }
      }
    }
  }
}

// Linear bins of width bw = ceil(w / 2048) over a range [lo, lo + w): bin = (v - lo) / bw.
// Key ranges are < 2^32 wide, so the hot key passes use 32-bit division.
__device__ __forceinline__ uint64_t bin_width(uint64_t w) { return (w + kBins - 1) / kBins; }
__device__ __forceinline__ int bin_of_key(uint32_t u, uint32_t lo, uint32_t bw) { return (int)((u - lo) / bw); }
__device__ __forceinline__ int bin_of_id(uint64_t v, uint64_t lo, uint64_t bw) { return (int)((v - lo) / bw); }

template <typename T>
__device__ __forceinline__ T block_reduce(T v, T* sbuf, int op /*0 sum, 1 min, 2 max*/) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const T x = __shfl_xor(v, o);
    v = op == 0 ? v + x : (op == 1 ? (x < v ? x : v) : (x > v ? x : v));
  }
  __syncthreads();
  if (lane == 0) sbuf[wave] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    T r = sbuf[0];
    for (int i = 1; i < kSelThreads / 64; ++i) {
      const T x = sbuf[i];
      r = op == 0 ? r + x : (op == 1 ? (x < r ? x : r) : (x > r ? x : r));
    }
    sbuf[0] = r;
  }
  __syncthreads();
  const T r = sbuf[0];
  __syncthreads();
  return r;
}

// Among bins, find b with below(b) < need <= below(b) + hist[b]; thread 0 writes (b, below).
__device__ __forceinline__ void find_bin(const int* hist, int need, int* s_res) {
  // each thread owns 2 consecutive bins; block-wide exclusive scan over 1024 pair sums
  __shared__ int wsum[kSelThreads / 64];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int h0 = hist[2 * t], h1 = hist[2 * t + 1];
  int inc = h0 + h1;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int x = __shfl_up(inc, o);
    if (lane >= o) inc += x;
  }
  if (lane == 63) wsum[wave] = inc;
  __syncthreads();
  int woff = 0;
  for (int i = 0; i < wave; ++i) woff += wsum[i];
  const int excl = woff + inc - (h0 + h1);
  if (excl < need && need <= excl + h0) { s_res[0] = 2 * t; s_res[1] = excl; }
  else if (excl + h0 < need && need <= excl + h0 + h1) { s_res[0] = 2 * t + 1; s_res[1] = excl + h0; }
  __syncthreads();
}

template <int CAP, bool EXPLICIT, int METRIC>
__global__ __launch_bounds__(kSelThreads) void k_select(SelectArgs a) {
  __shared__ int hist[kBins];
  __shared__ uint32_t sk[CAP];
  __shared__ int64_t si[CAP];
  __shared__ int s_res[4];
  __shared__ uint64_t s_red[kSelThreads / 64];

  const int64_t q = blockIdx.x;
  const int tid = threadIdx.x;
  int64_t base, ncand, nslots = 0;
  if (EXPLICIT && a.slot_begin) {  // slots of n_in (dist, id) entries each, query q's in [slot_begin[q], [q + 1]) (K9r)
    base = a.slot_begin[q] * a.n_in;
    ncand = (a.slot_begin[q + 1] - a.slot_begin[q]) * a.n_in;
  } else if (EXPLICIT) {
    base = q * a.n_in;
    ncand = a.n_in;
  } else {
    const int64_t sb = a.slot_begin ? a.slot_begin[q] : q * a.slots_per_q;
    const int64_t se = a.slot_begin ? a.slot_begin[q + 1] : sb + a.slots_per_q;
    base = sb;
    nslots = se - sb;
    ncand = nslots * a.slot_rows;
  }
  const int k = a.k;

  // ---- pass 0: valid count + key range ----
  uint64_t cnt = 0, mn = 0xFFFFFFFFull, mx = 0;
  visit_cands<EXPLICIT, METRIC>(a, base, ncand, nslots, [&](const Cand& c, auto) {
    if (c.valid) {
      ++cnt;
      mn = c.u < mn ? c.u : mn;
      mx = c.u > mx ? c.u : mx;
    }
  });
  const int64_t n_valid = (int64_t)block_reduce<uint64_t>(cnt, s_red, 0);
  uint64_t klo = block_reduce<uint64_t>(mn, s_red, 1);
  uint64_t khi = block_reduce<uint64_t>(mx, s_red, 2);

  // selection bound: key u < klo always selected; u in [klo, khi] selected (key phase) or,
  // in the id phase (klo == khi), with id in [ilo, ihi]
  int64_t below = 0;  // candidates strictly below the current range
  bool id_phase = false;
  uint64_t ilo = 0, ihi = 0;
  bool select_all = n_valid <= CAP;
  const int need = (int)(n_valid < k ? n_valid : k);

  while (!select_all) {
    // range exhausted on the key: refine by id among the tied candidates
    if (!id_phase && klo == khi) {
      uint64_t imn = ~0ull, imx = 0;
      visit_cands<EXPLICIT, METRIC>(a, base, ncand, nslots, [&](const Cand& c, auto id_of) {
        if (c.valid && c.u == klo) {
          const uint64_t id = (uint64_t)id_of();
          imn = id < imn ? id : imn;
          imx = id > imx ? id : imx;
        }
      });
      ilo = block_reduce<uint64_t>(imn, s_red, 1);
      ihi = block_reduce<uint64_t>(imx, s_red, 2);
      id_phase = true;
      if (ilo == ihi) break;  // identical (key, id) duplicates: nothing left to order
    }
    const uint64_t lo = id_phase ? ilo : klo;
    const uint64_t w = (id_phase ? ihi : khi) - lo + 1;
    const uint64_t bw = bin_width(w);
    for (int i = tid; i < kBins; i += kSelThreads) hist[i] = 0;
    __syncthreads();
    visit_cands<EXPLICIT, METRIC>(a, base, ncand, nslots, [&](const Cand& c, auto id_of) {
      if (!c.valid) return;
      if (!id_phase) {
        if (c.u >= klo && c.u <= khi) atomicAdd(&hist[bin_of_key(c.u, (uint32_t)klo, (uint32_t)bw)], 1);
      } else if (c.u == klo) {
        const uint64_t id = (uint64_t)id_of();
        if (id >= ilo && id <= ihi) atomicAdd(&hist[bin_of_id(id, ilo, bw)], 1);
      }
    });
    __syncthreads();
    find_bin(hist, need - (int)below, s_res);
    const int b = s_res[0];
    below += s_res[1];
    const int hb = hist[b];
    const uint64_t nlo = lo + (uint64_t)b * bw;
    const uint64_t last = lo + w - 1;
    const uint64_t nhi = nlo + bw - 1 < last ? nlo + bw - 1 : last;
    __syncthreads();
    if (id_phase) { ilo = nlo; ihi = nhi; }
    else { klo = nlo; khi = nhi; }
    if (below + hb <= CAP) break;
    if (id_phase && ilo == ihi) break;
  }

  // ---- collect: everything at or below the bound ----
  if (tid == 0) s_res[2] = 0;
  __syncthreads();
  visit_cands<EXPLICIT, METRIC>(a, base, ncand, nslots, [&](const Cand& c, auto id_of) {
    if (!c.valid) return;
    bool take;
    if (select_all) take = true;
    else if (!id_phase) take = c.u <= khi;
    else take = c.u < klo || (c.u == klo && (uint64_t)id_of() <= ihi);
    if (take) {
      const int pos = atomicAdd(&s_res[2], 1);
      if (pos < CAP) {
        sk[pos] = c.u;
        si[pos] = id_of();
      }
    }
  });
  __syncthreads();
  const int n_sel = s_res[2] < CAP ? s_res[2] : CAP;
  int p2 = 1;
  while (p2 < n_sel) p2 <<= 1;
  for (int i = n_sel + tid; i < p2; i += kSelThreads) {
    sk[i] = 0xFFFFFFFFu;
    si[i] = LLONG_MAX;
  }
  __syncthreads();
  // ---- bitonic sort of p2 (key, id) pairs ----
  for (int size = 2; size <= p2; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = tid; i < (p2 >> 1); i += kSelThreads) {
        const int lo_i = 2 * i - (i & (stride - 1));
        const int hi_i = lo_i + stride;
        const bool up = (lo_i & size) == 0;
        const uint32_t ka = sk[lo_i], kb = sk[hi_i];
        const int64_t ia = si[lo_i], ib = si[hi_i];
        const bool gt = ka > kb || (ka == kb && ia > ib);
        if (gt == up) {
          sk[lo_i] = kb; sk[hi_i] = ka;
          si[lo_i] = ib; si[hi_i] = ia;
        }
      }
      __syncthreads();
    }
  }
  for (int t = tid; t < k; t += kSelThreads) {
    const bool valid = t < n_sel && t < need;
    const float key = valid ? from_ord(sk[t]) : INFINITY;
    a.out_d[q * k + t] = valid ? (METRIC == kIP ? -key : key) : (METRIC == kIP ? -INFINITY : INFINITY);
    a.out_i[q * k + t] = valid ? si[t] : (int64_t)-1;
  }
}

// K8s: the same selection for small k over few DUMP keys (k <= 64, slots x slot_rows <= 1024 per query: the
// coarse probe's top-n_probes of the centroid list), one WAVE per query instead of a 1024-thread block
// with 2048-bin histograms and a 1024-wide bitonic sort. Each lane holds <= 16 candidates in registers:
//   1. T = the need-th smallest orderable key: binary search over the 32 key bits, counts by wave sums;
//   2. among keys equal to T, the (need - #(key < T)) smallest ids: binary search over the id bits (only
//      when the tie is larger than what is needed);
//   3. the need chosen (key, id) pairs -> one per lane (ballot prefix into LDS) -> 64-lane bitonic sort
//      by (key, id) -> the first k, the missing ranks (id -1, +inf / IP -inf) as in K8.
constexpr int kSmallPer = 16;
constexpr int kSmallWaves = 4;

// V2 (default; MIVS_SELECT_SMALL_V2=0 keeps the bit search only): T0 = the need-th smallest of the 64 lanes' minima bounds the need-th
// smallest key from above (need <= 64 lanes, each minimum a distinct key at or below it); when at most 64 keys lie
// at or below T0 they are the candidates -- one per lane, bitonic-sorted by (key, id) -- without the bit search
template <int METRIC, bool V2, bool FAST>
__global__ __launch_bounds__(64 * kSmallWaves) void k_select_small(SelectArgs a) {
  __shared__ uint32_t s_u[kSmallWaves][64];
  __shared__ int64_t s_i[kSmallWaves][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t q = (int64_t)blockIdx.x * kSmallWaves + wv;
  if (q >= a.nq) return;
  const int k = a.k;
  const int64_t base = q * a.slots_per_q;
  const int n_total = (int)(a.slots_per_q * a.slot_rows);
  uint32_t u[kSmallPer];
  int nv = 0;
  // Slots of whole 64-row multiples (the coarse probe's DUMP: 128): key i of every lane lies in slot i / (slot_rows /
  // 64), uniform over the wave, so the slot headers are read once (lane s holds slot s's) and each key is one load at
  // a scalar base -- cand_key's per-key header load and 64-bit address kept ~118 VGPRs live (4 waves per SIMD)
  constexpr bool fast = FAST;  // (launched where slot_rows % 64 == 0 and slots_per_q <= 64)
  const int spr = a.slot_rows >> 6;  // (fast) 64-key rows per slot
  int nr_v = 0;
  int64_t f_v = 0;
  if (fast && lane < a.slots_per_q) {
    nr_v = (int)a.slot_info[2 * (base + lane) + 1];
    f_v = a.slot_info[2 * (base + lane)];
  }
  if constexpr (fast) {
    int sq = 0, ri = 0;  // (uniform) slot of key i and its 64-row block in the slot
#pragma unroll
    for (int i = 0; i < kSmallPer; ++i) {
      u[i] = 0xFFFFFFFFu;
      if (64 * i < n_total) {
        const int rr = 64 * ri + lane;
        const int nr = __builtin_amdgcn_readlane(nr_v, sq);
        if (rr < nr) {
          const uint32_t o = ord_bits(a.keys[(base + sq) * a.slot_rows + rr]);
          if (o < kOrdInf) u[i] = o;  // pad rows carry +inf
        }
      }
      nv += __popcll(__ballot(u[i] != 0xFFFFFFFFu));
      if (++ri == spr) { ri = 0; ++sq; }
    }
  } else {
#pragma unroll
  for (int i = 0; i < kSmallPer; ++i) {
    const int t = lane + 64 * i;
    u[i] = 0xFFFFFFFFu;
    bool ok = false;
    if (t < n_total) {
      const Cand c = cand_key<false, METRIC>(a, base, t);
      if (c.valid) {
        u[i] = c.u;
        ok = true;
      }
    }
    nv += __popcll(__ballot(ok));
  }
  }
  const int need = nv < k ? nv : k;
  // the valid keys' range bounds the search (a few of the 32 bits once the keys share an exponent)
  uint32_t umin = 0xFFFFFFFFu, umax = 0u;
#pragma unroll
  for (int i = 0; i < kSmallPer; ++i)
    if (u[i] != 0xFFFFFFFFu) {
      umin = u[i] < umin ? u[i] : umin;
      umax = u[i] > umax ? u[i] : umax;
    }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const uint32_t a0 = __shfl_xor(umin, o), a1 = __shfl_xor(umax, o);
    umin = a0 < umin ? a0 : umin;
    umax = a1 > umax ? a1 : umax;
  }
  // counts over the wave by ballot + popcount (scalar): a shuffle reduction per count put six LDS round trips
  // on every step of the searches below
  auto count_le = [&](uint32_t m) {
    int c = 0;
#pragma unroll
    for (int i = 0; i < kSmallPer; ++i) c += __popcll(__ballot(u[i] <= m));  // (invalid = 0xFFFFFFFF > every valid m)
    return c;
  };
  uint32_t T = 0;
  int64_t I = LLONG_MAX;  // among keys == T: ids <= I are chosen
  bool searched = false;
  if (V2 && need > 0) {
    uint32_t lm = 0xFFFFFFFFu;
#pragma unroll
    for (int i = 0; i < kSmallPer; ++i) lm = u[i] < lm ? u[i] : lm;
    // bitonic sort of the 64 lane minima, ascending
#pragma unroll
    for (int size = 2; size <= 64; size <<= 1) {
#pragma unroll
      for (int stride = size >> 1; stride > 0; stride >>= 1) {
        const uint32_t o = __shfl_xor(lm, stride);
        const bool lower = (lane & stride) == 0, up = (lane & size) == 0;
        lm = (lower == up) ? (o < lm ? o : lm) : (o > lm ? o : lm);
      }
    }
    const uint32_t T0 = __shfl(lm, need - 1);
    if (T0 != 0xFFFFFFFFu && count_le(T0) <= 64) {
      T = T0;  // every key <= T0 is taken (I = +inf): at most 64, the need smallest among them
      searched = true;
    }
  }
  if (need > 0 && !searched) {
    uint32_t lo = umin, hi = umax;  // the need-th smallest valid key lies in [lo, hi]
    while (lo < hi) {
      const uint32_t mid = lo + ((hi - lo) >> 1);
      if (count_le(mid) >= need) hi = mid; else lo = mid + 1;
    }
    T = lo;
    const int c_lt = T > 0 ? count_le(T - 1) : 0;
    const int c_eq = count_le(T) - c_lt;
    const int m = need - c_lt;
    if (c_eq > m) {  // a tie larger than needed: the m smallest ids among keys == T (ids are distinct)
      auto count_id = [&](int64_t x) {
        int c = 0;
#pragma unroll
        for (int i = 0; i < kSmallPer; ++i)
          c += __popcll(__ballot(u[i] == T && cand_id<false>(a, base, lane + 64 * i) <= x));
        return c;
      };
      int64_t ilo = 0, ihi = LLONG_MAX;  // (valid candidates have ids >= 0; count_id(LLONG_MAX) = c_eq >= m)
      while (ilo < ihi) {
        const int64_t mid = ilo + ((ihi - ilo) >> 1);
        if (count_id(mid) >= m) ihi = mid; else ilo = mid + 1;
      }
      I = ilo;
    }
  }
  // the chosen pairs, one per lane
  int nsel = 0;
  int sq = 0, ri = 0;  // (fast) as in the key loads
#pragma unroll
  for (int i = 0; i < kSmallPer; ++i) {
    const int t = lane + 64 * i;
    bool take = need > 0 && u[i] <= T && u[i] != 0xFFFFFFFFu;
    int64_t id = 0;
    if constexpr (fast) {
      const uint64_t f = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)((uint64_t)f_v >> 32), sq) << 32) |
                         (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(uint64_t)f_v, sq);
      if (take) id = a.row_ids[(int64_t)f + 64 * ri + lane];
      if (++ri == spr) { ri = 0; ++sq; }
    } else if (take) {
      id = cand_id<false>(a, base, t);
    }
    if (take && u[i] == T && id > I) take = false;
    const uint64_t bm = __ballot(take);
    if (take) {
      const int at = nsel + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bm, 0u));
      if (at < 64) {
        s_u[wv][at] = u[i];
        s_i[wv][at] = id;
      }
    }
    nsel += __popcll(bm);
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  const int ncand = searched ? (nsel < 64 ? nsel : 64) : need;
  uint32_t ku = lane < ncand ? s_u[wv][lane] : 0xFFFFFFFFu;
  int64_t ki = lane < ncand ? s_i[wv][lane] : LLONG_MAX;
  // bitonic sort of the 64 lanes by (key, id), ascending
#pragma unroll
  for (int size = 2; size <= 64; size <<= 1) {
#pragma unroll
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      const uint32_t ou = __shfl_xor(ku, stride);
      const int64_t oi = __shfl_xor(ki, stride);
      const bool lower = (lane & stride) == 0;
      const bool up = (lane & size) == 0;
      const bool o_less = ou < ku || (ou == ku && oi < ki);
      // the lower lane of a pair keeps the smaller in an ascending block, the larger in a descending one
      const bool take_o = (lower == up) ? o_less : !o_less && !(ou == ku && oi == ki);
      if (take_o) {
        ku = ou;
        ki = oi;
      }
    }
  }
  if (lane < k) {
    const bool valid = lane < need;
    const float key = valid ? from_ord(ku) : INFINITY;
    a.out_d[q * k + lane] = valid ? (METRIC == kIP ? -key : key) : (METRIC == kIP ? -INFINITY : INFINITY);
    a.out_i[q * k + lane] = valid ? ki : (int64_t)-1;
  }
}

// K8c: the k <= 256 smallest (key, id) over a query's candidate slots (EXPLICIT with slot_begin: K9r's per-chunk
// supersets for IVF-PQ + refine pools), one WAVE per query instead of K8's 1024-thread block -- a query has a few
// thousand entries (~10 slots x 256, about half of them +inf padding), where K8's block barriers (a 1024-wide bitonic
// sort among them) cost ~60 us of latency per query: 0.63 ms per 10k queries.
//   1. T = the need-th smallest orderable key (need = min(k, valid)): four 8-bit digit passes, MSB first, each a
//      256-bin LDS histogram of the keys that share the digits found so far and a wave scan to the digit holding
//      the remaining rank (the keys stream from global each pass; a query's ~10 KB stay in L2);
//   2. when more keys equal T than are needed, the same digit passes over their 64-bit ids give the largest id I
//      taken among them (ids are distinct);
//   3. the chosen (key < T, or key == T with id <= I: exactly need of them) -> LDS, bitonic sort by (key, id) in the
//      wave, the first k out; missing ranks (id -1, +inf / IP -inf) as in K8.
constexpr int kScWaves = 4;
constexpr int kScMaxK = 256;

template <int METRIC>
__global__ __launch_bounds__(64 * kScWaves) void k_select_slots(SelectArgs a) {
  __shared__ int s_hist[kScWaves][256];
  __shared__ uint32_t s_u[kScWaves][kScMaxK];
  __shared__ int64_t s_i[kScWaves][kScMaxK];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t q = (int64_t)blockIdx.x * kScWaves + wv;
  if (q >= a.nq) return;  // (wave-uniform; no workgroup barrier below)
  const int k = a.k;
  const int64_t base = a.slot_begin[q] * a.n_in;
  const int64_t n = (a.slot_begin[q + 1] - a.slot_begin[q]) * a.n_in;
  int* hist = s_hist[wv];
  auto key_at = [&](int64_t t) {  // orderable key bits; invalid (+inf padding) = 0xFFFFFFFF
    const float dd = a.keys[base + t];
    const uint32_t u = ord_bits(METRIC == kIP ? -dd : dd);
    return u < kOrdInf ? u : 0xFFFFFFFFu;
  };
  // every candidate t of this lane with its key: f(t, u), the keys read from global (L2 after the first pass) four
  // at a time, all four loads issued before any is used (held in registers for the whole selection, 64 per lane,
  // the kernel ran 2.6x slower: the unrolled passes spilled)
  auto for_each = [&](auto f) {
    for (int64_t t0 = lane; t0 < n; t0 += 256) {
      uint32_t u[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) u[j] = t0 + 64 * j < n ? key_at(t0 + 64 * j) : 0xFFFFFFFFu;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (t0 + 64 * j < n) f(t0 + 64 * j, u[j]);
    }
  };
  int nv = 0;
  uint32_t umin = 0xFFFFFFFFu, umax = 0u;
  for_each([&](int64_t, uint32_t u) {
    if (u == 0xFFFFFFFFu) return;
    ++nv;
    umin = u < umin ? u : umin;
    umax = u > umax ? u : umax;
  });
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    nv += __shfl_xor(nv, o);
    const uint32_t a0 = __shfl_xor(umin, o), a1 = __shfl_xor(umax, o);
    umin = a0 < umin ? a0 : umin;
    umax = a1 > umax ? a1 : umax;
  }
  const int need = nv < k ? nv : k;
  // digit passes (MSB first) over a 32- or 64-bit value of the members: the rank-th smallest value. The passes start
  // at the highest byte in which the members can differ (top_shift; prefix = the bytes above it, common to all)
  auto digit_select = [&](int top_shift, uint64_t prefix, auto value_of, auto member, int rank) {
    for (int shift = top_shift; shift >= 0; shift -= 8) {
      for (int b = lane; b < 256; b += 64) hist[b] = 0;
      wave_lds_sync();
      for_each([&](int64_t t, uint32_t u) {
        if (!member(t, u)) return;
        const uint64_t v = value_of(t, u);
        if (shift + 8 < 64 && (v >> (shift + 8)) != prefix) return;
        atomicAdd(&hist[(int)((v >> shift) & 255)], 1);
      });
      wave_lds_sync();
      // the bin holding the rank-th: each lane sums 4 consecutive bins, a wave-inclusive scan over the lanes
      int h[4], c = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) { h[j] = hist[4 * lane + j]; c += h[j]; }
      int inc = c;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int x = __shfl_up(inc, o);
        if (lane >= o) inc += x;
      }
      int excl = inc - c, bin = -1, below = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (bin < 0 && excl < rank && rank <= excl + h[j]) { bin = 4 * lane + j; below = excl; }
        excl += h[j];
      }
      const uint64_t found = __ballot(bin >= 0);
      const int src = found ? __builtin_ctzll(found) : 0;
      bin = __shfl(bin, src);
      below = __shfl(below, src);
      rank -= below;
      prefix = (prefix << 8) | (uint64_t)bin;
      wave_lds_sync();  // (the next pass clears the bins after every lane read them)
    }
    return prefix;
  };
  uint32_t T = 0xFFFFFFFFu;
  int64_t I = LLONG_MAX;  // among keys == T, ids <= I are chosen
  if (need > 0) {
    // (keys of one query share their high bytes: the passes start at the first byte where umin and umax differ)
    const uint32_t diff = umin ^ umax;
    const int top = diff == 0 ? 0 : ((31 - __builtin_clz(diff)) / 8) * 8;
    const uint64_t pre = top + 8 < 32 ? (uint64_t)(umin >> (top + 8)) : 0;
    T = (uint32_t)digit_select(top, pre, [&](int64_t, uint32_t u) { return (uint64_t)u; },
                               [&](int64_t, uint32_t u) { return u != 0xFFFFFFFFu; }, need);
    int lt = 0, eq = 0;
    for_each([&](int64_t, uint32_t u) {
      lt += u < T ? 1 : 0;
      eq += u == T ? 1 : 0;
    });
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      lt += __shfl_xor(lt, o);
      eq += __shfl_xor(eq, o);
    }
    if (eq > need - lt)  // a tie larger than needed: the (need - lt) smallest ids among keys == T (ids >= 0, distinct)
      I = (int64_t)digit_select(56, 0, [&](int64_t t, uint32_t) { return (uint64_t)a.ids[base + t]; },
                                [&](int64_t, uint32_t u) { return u == T; }, need - lt);
  }
  // the need chosen pairs -> LDS (ballot prefix positions; exactly need of them, <= kScMaxK)
  if (need > 0) {
    int cnt = 0;
    auto collect = [&](int64_t t, uint32_t u) {  // (every lane calls it: the ballot is wave-wide)
      bool take = false;
      int64_t id = LLONG_MAX;
      if (t < n && u <= T) {
        id = a.ids[base + t];
        take = u < T || id <= I;
      }
      const uint64_t m = __ballot(take);
      if (take) {
        const int at = cnt + __popcll(m & ((1ull << lane) - 1));
        if (at < kScMaxK) { s_u[wv][at] = u; s_i[wv][at] = id; }
      }
      cnt += __popcll(m);
    };
    for (int64_t t0 = 0; t0 < n; t0 += 64) collect(t0 + lane, t0 + lane < n ? key_at(t0 + lane) : 0xFFFFFFFFu);
  }
  int p2 = 1;
  while (p2 < need) p2 <<= 1;
  for (int i = need + lane; i < p2; i += 64) { s_u[wv][i] = 0xFFFFFFFFu; s_i[wv][i] = LLONG_MAX; }
  wave_lds_sync();
  // bitonic sort of p2 (<= 256) pairs by (key, id) in the wave's LDS slice
  for (int size = 2; size <= p2; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = lane; i < (p2 >> 1); i += 64) {
        const int lo = 2 * i - (i & (stride - 1));
        const int hi = lo + stride;
        const bool up = (lo & size) == 0;
        const uint32_t ka = s_u[wv][lo], kb = s_u[wv][hi];
        const int64_t ia = s_i[wv][lo], ib = s_i[wv][hi];
        const bool gt = ka > kb || (ka == kb && ia > ib);
        if (gt == up) {
          s_u[wv][lo] = kb; s_u[wv][hi] = ka;
          s_i[wv][lo] = ib; s_i[wv][hi] = ia;
        }
      }
      wave_lds_sync();
    }
  }
  for (int t = lane; t < k; t += 64) {
    const bool valid = t < need;
    const float key = valid ? from_ord(s_u[wv][t]) : INFINITY;
    a.out_d[q * k + t] = valid ? (METRIC == kIP ? -key : key) : (METRIC == kIP ? -INFINITY : INFINITY);
    a.out_i[q * k + t] = valid ? s_i[wv][t] : (int64_t)-1;
  }
}

template <int CAP>
hipError_t launch_cap(const SelectArgs& a, bool expl, hipStream_t s) {
  const dim3 grid((unsigned)a.nq), block(kSelThreads);
  if (expl) {
    if (a.metric == kIP) hipLaunchKernelGGL((k_select<CAP, true, kIP>), grid, block, 0, s, a);
    else hipLaunchKernelGGL((k_select<CAP, true, kL2>), grid, block, 0, s, a);
  } else {  // dump keys are already ranking keys; METRIC only sets the sign of the output distance
    if (a.metric == kIP) hipLaunchKernelGGL((k_select<CAP, false, kIP>), grid, block, 0, s, a);
    else hipLaunchKernelGGL((k_select<CAP, false, kL2>), grid, block, 0, s, a);
  }
  return hipGetLastError();
}

}  // namespace

hipError_t launch_select(const SelectArgs& a, hipStream_t s) {
  if (a.k < 1 || a.k > kMaxSelectK) return hipErrorInvalidValue;
  if (a.nq <= 0) return hipSuccess;
  if (a.nq > 0x7FFFFFFF) return hipErrorInvalidValue;
  const bool expl = a.slot_info == nullptr;
  if (!expl && a.k <= 64 && a.slots_per_q * a.slot_rows <= 64 * kSmallPer) {  // K8s
    const dim3 grid((unsigned)ceil_div(a.nq, (int64_t)kSmallWaves)), block(64 * kSmallWaves);
    // (the threshold from the 64 lanes' minima: 122 -> 72 us for the coarse probe's 10k x 1024 keys; the bit search
    // alone was retired in round 5)
    const bool fast = (a.slot_rows & 63) == 0 && a.slots_per_q <= 64;  // slot-uniform key loads
    if (fast) {
      if (a.metric == kIP) hipLaunchKernelGGL((k_select_small<kIP, true, true>), grid, block, 0, s, a);
      else hipLaunchKernelGGL((k_select_small<kL2, true, true>), grid, block, 0, s, a);
    } else {
      if (a.metric == kIP) hipLaunchKernelGGL((k_select_small<kIP, true, false>), grid, block, 0, s, a);
      else hipLaunchKernelGGL((k_select_small<kL2, true, false>), grid, block, 0, s, a);
    }
    return hipGetLastError();
  }
  // (MIVS_SELECT_SLOTS_WAVE=0: K8's block form for the slots, A/B runs)
  const bool slots_wave = engine_setting(kSetSelectSlotsWave, "MIVS_SELECT_SLOTS_WAVE", 1) != 0;
  if (expl && a.slot_begin && a.k <= kScMaxK && slots_wave) {  // K8c
    const dim3 grid((unsigned)ceil_div(a.nq, (int64_t)kScWaves)), block(64 * kScWaves);
    if (a.metric == kIP) hipLaunchKernelGGL((k_select_slots<kIP>), grid, block, 0, s, a);
    else hipLaunchKernelGGL((k_select_slots<kL2>), grid, block, 0, s, a);
    return hipGetLastError();
  }
  if (a.k <= 512) return launch_cap<1024>(a, expl, s);
  if (a.k <= 1024) return launch_cap<2048>(a, expl, s);
  if (a.k <= 2048) return launch_cap<4096>(a, expl, s);
  return launch_cap<8192>(a, expl, s);
}

}  // namespace mivs
