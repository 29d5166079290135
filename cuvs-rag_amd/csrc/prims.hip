// Integer primitives of the IVF pipeline: device-wide exclusive scan, stable
// counting sort (list fill order / k-means member order), and the per-batch
// probe map that turns coarse probes into (list -> query bucket) work items.
// All HBM-bound integer work: plain coalesced loads/stores, LDS histograms, no
// MFMA.
#include "mivs_common.hpp"

namespace mivs {

namespace {

constexpr int kScanBlock = 1024;
constexpr int kScanPerThread = 4;
constexpr int kScanTile = kScanBlock * kScanPerThread;


__global__ __launch_bounds__(kScanBlock) void k_scan_reduce(const int64_t* __restrict__ in, int64_t n,
                                                            int64_t* __restrict__ sums) {
  __shared__ int64_t sh[16];
  const int64_t base = (int64_t)blockIdx.x * kScanTile + (int64_t)threadIdx.x * kScanPerThread;
  int64_t v = 0;
#pragma unroll
  for (int i = 0; i < kScanPerThread; ++i) v += base + i < n ? in[base + i] : 0;
  int64_t tot;
  block_excl_scan(v, sh, &tot);
  if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

// single block: exclusive scan of the block sums in place (any count, carried)
__global__ __launch_bounds__(kScanBlock) void k_scan_sums(int64_t* __restrict__ sums, int64_t nb) {
  __shared__ int64_t sh[16];
  int64_t carry = 0;
  for (int64_t b0 = 0; b0 < nb; b0 += kScanBlock) {
    const int64_t i = b0 + threadIdx.x;
    const int64_t v = i < nb ? sums[i] : 0;
    int64_t tot;
    const int64_t ex = block_excl_scan(v, sh, &tot);
    if (i < nb) sums[i] = carry + ex;
    carry += tot;
  }
}

__global__ __launch_bounds__(kScanBlock) void k_scan_down(const int64_t* __restrict__ in, int64_t n,
                                                          const int64_t* __restrict__ sums,
                                                          int64_t* __restrict__ out) {
  __shared__ int64_t sh[16];
  const int64_t base = (int64_t)blockIdx.x * kScanTile + (int64_t)threadIdx.x * kScanPerThread;
  int64_t vals[kScanPerThread];
  int64_t v = 0;
#pragma unroll
  for (int i = 0; i < kScanPerThread; ++i) { vals[i] = base + i < n ? in[base + i] : 0; v += vals[i]; }
  int64_t run = sums[blockIdx.x] + block_excl_scan(v, sh, nullptr);
#pragma unroll
  for (int i = 0; i < kScanPerThread; ++i) {
    if (base + i < n) out[base + i] = run;
    run += vals[i];
  }
}

// one block for small n (the per-query offsets of a batch): the three launches above cost ~5 us each at any size
constexpr int64_t kScanSmallMax = 4 * kScanTile;
__global__ __launch_bounds__(kScanBlock) void k_scan_small(const int64_t* __restrict__ in, int64_t n,
                                                           int64_t* __restrict__ out) {
  __shared__ int64_t sh[16];
  int64_t carry = 0;
  for (int64_t b0 = 0; b0 < n; b0 += kScanTile) {
    const int64_t base = b0 + (int64_t)threadIdx.x * kScanPerThread;
    int64_t vals[kScanPerThread];
    int64_t v = 0;
#pragma unroll
    for (int i = 0; i < kScanPerThread; ++i) { vals[i] = base + i < n ? in[base + i] : 0; v += vals[i]; }
    int64_t tot;
    int64_t run = carry + block_excl_scan(v, sh, &tot);
#pragma unroll
    for (int i = 0; i < kScanPerThread; ++i) {
      if (base + i < n) out[base + i] = run;
      run += vals[i];
    }
    carry += tot;
  }
}

// ---------------- stable counting sort by label ----------------
constexpr int kSortBlock = 1024;  // rows per histogram block (16 waves)

__global__ __launch_bounds__(kSortBlock) void k_sort_hist(const int64_t* __restrict__ labels, int64_t n, int nl,
                                                          int64_t nb, int64_t* __restrict__ counts) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int* hist = reinterpret_cast<int*>(smem);
  for (int i = threadIdx.x; i < nl; i += kSortBlock) hist[i] = 0;
  __syncthreads();
  const int64_t r = (int64_t)blockIdx.x * kSortBlock + threadIdx.x;
  if (r < n) atomicAdd(&hist[(int)labels[r]], 1);
  __syncthreads();
  for (int i = threadIdx.x; i < nl; i += kSortBlock) counts[(int64_t)i * nb + blockIdx.x] = hist[i];
}

// positions: offs[l*nb + b] = first output slot of block b's rows with label l
__global__ __launch_bounds__(kSortBlock) void k_sort_scatter(const int64_t* __restrict__ labels, int64_t n, int nl,
                                                             int64_t nb, const int64_t* __restrict__ offs,
                                                             int64_t* __restrict__ perm) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int* running = reinterpret_cast<int*>(smem);
  for (int i = threadIdx.x; i < nl; i += kSortBlock) running[i] = 0;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t r = (int64_t)blockIdx.x * kSortBlock + threadIdx.x;
  const int lab = r < n ? (int)labels[r] : -1;
  // rank among earlier lanes of this wave with the same label, and the wave's count of it
  int rank = 0, cnt = 0;
  for (int t = 0; t < 64; ++t) {
    const int o = __shfl(lab, t);
    if (o == lab) { ++cnt; if (t < lane) ++rank; }
  }
  __syncthreads();
  for (int wv = 0; wv < kSortBlock / 64; ++wv) {
    if (wave == wv && lab >= 0) {
      const int64_t pos = offs[(int64_t)lab * nb + blockIdx.x] + running[lab] + rank;
      perm[pos] = r;
    }
    __syncthreads();
    if (wave == wv && lab >= 0 && rank == cnt - 1) running[lab] += cnt;
    __syncthreads();
  }
}

__global__ void k_list_off_from_offs(const int64_t* __restrict__ offs, int nl, int64_t nb, int64_t n,
                                     int64_t* __restrict__ list_off) {
  const int l = blockIdx.x * blockDim.x + threadIdx.x;
  if (l < nl) list_off[l] = offs[(int64_t)l * nb];
  if (l == 0) list_off[nl] = n;
}

// ---------------- probe map ----------------
__global__ void k_probe_count(const int64_t* __restrict__ probes, int64_t n, int* __restrict__ counts) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && probes[i] >= 0) atomicAdd(&counts[(int)probes[i]], 1);  // -1: query without probes (NaN)
}

__global__ __launch_bounds__(1024) void k_probe_prefix(const int* __restrict__ counts, int n_lists,
                                                       const int64_t* __restrict__ list_goff, int G, int qtile,
                                                       int* __restrict__ bucket_off, int* __restrict__ work_off,
                                                       int* __restrict__ fill) {
  __shared__ int64_t sh[16];
  int64_t cb = 0, cw = 0;
  for (int l0 = 0; l0 < n_lists; l0 += 1024) {
    const int l = l0 + threadIdx.x;
    int64_t c = 0, wk = 0;
    if (l < n_lists) {
      c = counts[l];
      const int64_t chunks = ceil_div(list_goff[l + 1] - list_goff[l], G);
      wk = ceil_div(c, qtile) * chunks;
      fill[l] = 0;
    }
    int64_t tb, tw;
    const int64_t eb = block_excl_scan(c, sh, &tb);
    const int64_t ew = block_excl_scan(wk, sh, &tw);
    if (l < n_lists) { bucket_off[l] = (int)(cb + eb); work_off[l] = (int)(cw + ew); }
    cb += tb;
    cw += tw;
  }
  if (threadIdx.x == 0) { bucket_off[n_lists] = (int)cb; work_off[n_lists] = (int)cw; }
}

__global__ void k_probe_fill(const int64_t* __restrict__ probes, int64_t n, int np, const int* __restrict__ bucket_off,
                             int* __restrict__ fill, int64_t* __restrict__ bucket_q, int64_t* __restrict__ bucket_qp,
                             const int64_t* __restrict__ list_goff, int G, int64_t* __restrict__ qp_slots) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int l = (int)probes[i];
  if (l < 0) { qp_slots[i] = 0; return; }
  const int e = bucket_off[l] + atomicAdd(&fill[l], 1);
  bucket_q[e] = i / np;
  bucket_qp[e] = i;
  qp_slots[i] = ceil_div(list_goff[l + 1] - list_goff[l], G);
}

// The same count and fill with an LDS histogram per chunk of kPmChunk entries: a list probed by m queries
// took m contended global atomics per pass, now one per (chunk, list). The order of the queries inside a
// bucket was the atomics' order before and still is (nothing downstream depends on it).
constexpr int kPmChunk = 2048;  // (8192: fill 23 us, 2048: 13 us, 1024: 16 us for K13's 320k-entry map)
constexpr int kPmMaxLists = 32768;  // 128 KiB of int bins

__device__ __forceinline__ void pm_chunk_hist(const int64_t* __restrict__ probes, int64_t n, int n_lists, int* bins) {
  for (int l = threadIdx.x; l < n_lists; l += blockDim.x) bins[l] = 0;
  __syncthreads();
  const int64_t i0 = (int64_t)blockIdx.x * kPmChunk;
  const int64_t i1 = i0 + kPmChunk < n ? i0 + kPmChunk : n;
  for (int64_t i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
    const int64_t l = probes[i];
    if (l >= 0) atomicAdd(bins + l, 1);
  }
  __syncthreads();
}

__global__ __launch_bounds__(1024) void k_probe_count_lds(const int64_t* __restrict__ probes, int64_t n, int n_lists,
                                                          int* __restrict__ counts) {
  extern __shared__ int bins[];
  pm_chunk_hist(probes, n, n_lists, bins);
  for (int l = threadIdx.x; l < n_lists; l += blockDim.x)
    if (bins[l]) atomicAdd(counts + l, bins[l]);
}

__global__ __launch_bounds__(1024) void k_probe_fill_lds(const int64_t* __restrict__ probes, int64_t n, int np,
                                                         int n_lists, const int* __restrict__ bucket_off,
                                                         int* __restrict__ fill, int64_t* __restrict__ bucket_q,
                                                         int64_t* __restrict__ bucket_qp,
                                                         const int64_t* __restrict__ list_goff, int G,
                                                         int64_t* __restrict__ qp_slots) {
  extern __shared__ int bins[];
  pm_chunk_hist(probes, n, n_lists, bins);
  for (int l = threadIdx.x; l < n_lists; l += blockDim.x) {
    const int c = bins[l];
    if (c) bins[l] = bucket_off[l] + atomicAdd(fill + l, c);  // this chunk's range of list l's bucket
  }
  __syncthreads();
  const int64_t i0 = (int64_t)blockIdx.x * kPmChunk;
  const int64_t i1 = i0 + kPmChunk < n ? i0 + kPmChunk : n;
  for (int64_t i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
    const int l = (int)probes[i];
    if (l < 0) { qp_slots[i] = 0; continue; }
    const int e = atomicAdd(bins + l, 1);
    bucket_q[e] = i / np;
    bucket_qp[e] = i;
    qp_slots[i] = ceil_div(list_goff[l + 1] - list_goff[l], G);
  }
}

// The whole probe map in ONE workgroup for a small batch (n entries <= kPmSmallMax, n_lists <= kPmSmallLists: K13's
// pre-pass map, one probe per query): LDS count, prefix, fill, and with slot_begin the scan of the per-(query, probe)
// slot counts, the entries' slots and the queries' first slots -- the six launches of the general path (memset,
// count, prefix, fill, scan, slots) cost ~5 us each however small the batch.
constexpr int kPmSmallPer = 32;  // entries per thread: a thread keeps its contiguous run of entries in registers
constexpr int64_t kPmSmallMax = 1024 * kPmSmallPer;
constexpr int kPmSmallLists = 8192;
__global__ __launch_bounds__(1024) void k_probe_map_small(const int64_t* __restrict__ probes, int64_t nq, int np,
                                                          int n_lists, const int64_t* __restrict__ list_goff, int G,
                                                          int qtile, int* __restrict__ counts,
                                                          int* __restrict__ bucket_off, int* __restrict__ work_off,
                                                          int64_t* __restrict__ bucket_q, int64_t* __restrict__ bucket_slot,
                                                          int64_t* __restrict__ qp_slots, int64_t* __restrict__ slot_begin) {
  __shared__ int bins[kPmSmallLists];
  __shared__ int chunks[kPmSmallLists];
  __shared__ int64_t sh[16];
  const int64_t n = nq * np;
  const int per = (int)((n + 1023) / 1024);
  const int64_t i0 = (int64_t)threadIdx.x * per;
  for (int l = threadIdx.x; l < n_lists; l += 1024) bins[l] = 0;
  int li[kPmSmallPer];
#pragma unroll
  for (int j = 0; j < kPmSmallPer; ++j) li[j] = j < per && i0 + j < n ? (int)probes[i0 + j] : -1;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kPmSmallPer; ++j)
    if (li[j] >= 0) atomicAdd(bins + li[j], 1);
  __syncthreads();
  // bucket and work offsets (k_probe_prefix); bins become each list's next free bucket entry
  int64_t cb = 0, cw = 0;
  for (int l0 = 0; l0 < n_lists; l0 += 1024) {
    const int l = l0 + threadIdx.x;
    int64_t c = 0, wk = 0;
    if (l < n_lists) {
      c = bins[l];
      const int ch = (int)ceil_div(list_goff[l + 1] - list_goff[l], G);
      chunks[l] = ch;
      wk = ceil_div(c, qtile) * ch;
      counts[l] = (int)c;
    }
    int64_t tb, tw;
    const int64_t eb = block_excl_scan(c, sh, &tb);
    const int64_t ew = block_excl_scan(wk, sh, &tw);
    if (l < n_lists) {
      bucket_off[l] = (int)(cb + eb);
      work_off[l] = (int)(cw + ew);
      bins[l] = (int)(cb + eb);
    }
    cb += tb;
    cw += tw;
  }
  if (threadIdx.x == 0) { bucket_off[n_lists] = (int)cb; work_off[n_lists] = (int)cw; }
  __syncthreads();
  // fill (k_probe_fill) from the registers: the entry's bucket position and its (query, probe)'s slot count
  int ei[kPmSmallPer];
  int64_t tsum = 0;
#pragma unroll
  for (int j = 0; j < kPmSmallPer; ++j) {
    ei[j] = -1;
    if (li[j] >= 0) {
      ei[j] = atomicAdd(bins + li[j], 1);
      bucket_q[ei[j]] = (i0 + j) / np;
      tsum += chunks[li[j]];
    }
    if (j < per && i0 + j < n) qp_slots[i0 + j] = li[j] >= 0 ? chunks[li[j]] : 0;
  }
  if (slot_begin == nullptr) {
#pragma unroll
    for (int j = 0; j < kPmSmallPer; ++j)
      if (ei[j] >= 0) bucket_slot[ei[j]] = i0 + j;
    return;
  }
  // the slots: an exclusive scan of the slot counts in entry order (a thread's entries are contiguous)
  int64_t tot;
  int64_t run = block_excl_scan(tsum, sh, &tot);
#pragma unroll
  for (int j = 0; j < kPmSmallPer; ++j) {
    const int64_t i = i0 + j;
    if (j < per && i < n) {
      if (i % np == 0) slot_begin[i / np] = run;
      if (ei[j] >= 0) {
        bucket_slot[ei[j]] = run;
        run += chunks[li[j]];
      }
    }
  }
  if (threadIdx.x == 0) slot_begin[nq] = tot;
}

// The exact fallback's probe map, sized on the device: the unproven queries of a pre-filter search
// are ovf_q[0 .. *n_dev) (K11 appends them); entry e = i * np + p is probe p of query ovf_q[i]. One workgroup, as
// k_probe_map_small, but over a count it reads on the device: LDS count, prefix, then the fill in entry order in
// rounds of 1024 entries, each round's slots numbered by a block scan. bucket_q = the query's own row (K3 reads the
// batch's rows and norms), bucket_slot / slot_begin number the slots by i (K7 merges query i into row ovf_q[i]).
// With nothing to fall back on it writes empty offsets: one launch, no host round trip.
__global__ __launch_bounds__(1024) void k_probe_map_dev(const int* __restrict__ n_dev, int64_t cap,
                                                        const int64_t* __restrict__ ovf_q,
                                                        const int64_t* __restrict__ probes, int np, int n_lists,
                                                        const int64_t* __restrict__ list_goff, int G, int qtile,
                                                        int* __restrict__ counts, int* __restrict__ bucket_off,
                                                        int* __restrict__ work_off, int64_t* __restrict__ bucket_q,
                                                        int64_t* __restrict__ bucket_slot,
                                                        int64_t* __restrict__ slot_begin, int* __restrict__ zero) {
  __shared__ int bins[kPmSmallLists];
  __shared__ int chunks[kPmSmallLists];
  __shared__ int64_t sh[16];
  const int nr = *n_dev;
  const int64_t nf = nr <= 0 ? 0 : (nr < cap ? nr : cap);
  const int64_t n = nf * np;
  if (threadIdx.x == 0 && zero) *zero = 0;
  for (int l = threadIdx.x; l < n_lists; l += 1024) bins[l] = 0;
  __syncthreads();
  auto list_of = [&](int64_t e) {
    const int64_t i = e / np;
    return (int)probes[ovf_q[i] * np + (e - i * np)];
  };
  for (int64_t e = threadIdx.x; e < n; e += 1024) {
    const int l = list_of(e);
    if (l >= 0) atomicAdd(bins + l, 1);
  }
  __syncthreads();
  int64_t cb = 0, cw = 0;
  for (int l0 = 0; l0 < n_lists; l0 += 1024) {
    const int l = l0 + threadIdx.x;
    int64_t c = 0, wk = 0;
    if (l < n_lists) {
      c = bins[l];
      const int ch = (int)ceil_div(list_goff[l + 1] - list_goff[l], G);
      chunks[l] = ch;
      wk = ceil_div(c, qtile) * ch;
      counts[l] = (int)c;
    }
    int64_t tb, tw;
    const int64_t eb = block_excl_scan(c, sh, &tb);
    const int64_t ew = block_excl_scan(wk, sh, &tw);
    if (l < n_lists) {
      bucket_off[l] = (int)(cb + eb);
      work_off[l] = (int)(cw + ew);
      bins[l] = (int)(cb + eb);
    }
    cb += tb;
    cw += tw;
  }
  if (threadIdx.x == 0) { bucket_off[n_lists] = (int)cb; work_off[n_lists] = (int)cw; }
  __syncthreads();
  int64_t carry = 0;
  for (int64_t e0 = 0; e0 < n; e0 += 1024) {  // (a uniform trip count: every thread reaches every scan)
    const int64_t e = e0 + threadIdx.x;
    const int l = e < n ? list_of(e) : -1;
    int64_t tot;
    const int64_t run = carry + block_excl_scan(l >= 0 ? (int64_t)chunks[l] : 0, sh, &tot);
    if (e < n) {
      if (e % np == 0) slot_begin[e / np] = run;
      if (l >= 0) {
        const int at = atomicAdd(bins + l, 1);
        bucket_q[at] = ovf_q[e / np];
        bucket_slot[at] = run;
      }
    }
    carry += tot;
  }
  if (threadIdx.x == 0) slot_begin[nf] = carry;
}

// the output slot of every bucket entry (its (query, probe)'s first slot) and each query's first slot, one launch
// (thread t: bucket entry t and query t)
__global__ void k_bucket_slot_begin(int64_t* __restrict__ bucket_slot, int64_t n, const int64_t* __restrict__ qp_base,
                                    const int64_t* __restrict__ qp_slots, int64_t nq, int np,
                                    int64_t* __restrict__ slot_begin) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n) bucket_slot[t] = qp_base[bucket_slot[t]];
  if (t < nq) slot_begin[t] = qp_base[t * np];
  if (t == nq) slot_begin[nq] = qp_base[nq * np - 1] + qp_slots[nq * np - 1];
}

__global__ void k_single_job(int64_t nq, int64_t chunks, int qtile, int64_t* __restrict__ bucket_q,
                             int64_t* __restrict__ bucket_slot, int* __restrict__ bucket_off,
                             int* __restrict__ work_off, int64_t* __restrict__ slot_begin, int* __restrict__ zero) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (zero && q == 0) *zero = 0;  // (the scan's work counter: no memset launch of its own)
  if (q < nq) {
    bucket_q[q] = q;
    bucket_slot[q] = q * chunks;
    if (slot_begin) slot_begin[q] = q * chunks;
  }
  if (q == 0) {
    bucket_off[0] = 0;
    bucket_off[1] = (int)nq;
    work_off[0] = 0;
    work_off[1] = (int)(ceil_div(nq, qtile) * chunks);
    if (slot_begin) slot_begin[nq] = nq * chunks;
  }
}

__global__ void k_iota(int64_t* __restrict__ out, int64_t n, int64_t start, int64_t step) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = start + i * step;
}

__global__ void k_fill_i32(int* __restrict__ out, int64_t n, int v) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = v;
}

// two fills in one launch (thread i: element i of each)
__global__ void k_fill2_i32(int* __restrict__ o1, int64_t n1, int v1, int* __restrict__ o2, int64_t n2, int v2) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n1) o1[i] = v1;
  if (i < n2) o2[i] = v2;
}

__global__ void k_group_list(const int64_t* __restrict__ list_goff, int n_lists, int64_t n_groups,
                             int* __restrict__ group_list) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n_groups) return;
  int lo = 0, hi = n_lists - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (list_goff[mid] <= g) lo = mid; else hi = mid - 1;
  }
  group_list[g] = lo;
}

// strided trainset row ids: rows[i] = floor(i * n / n_train) (oracle orc_train_rows)
__global__ void k_train_rows(int64_t* __restrict__ rows, int64_t n, int64_t n_train) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n_train) rows[i] = (i * n) / n_train;
}

__global__ void k_i64_to_i32(const int64_t* __restrict__ in, int64_t n, int32_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = (int32_t)in[i];
}

inline dim3 grid1(int64_t n, int b) { return dim3((unsigned)ceil_div(n > 0 ? n : 1, b)); }

}  // namespace

hipError_t launch_train_rows(int64_t* rows, int64_t n, int64_t n_train, hipStream_t s) {
  if (n_train <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_train_rows, grid1(n_train, 256), dim3(256), 0, s, rows, n, n_train);
  return hipGetLastError();
}

hipError_t launch_i64_to_i32(const int64_t* in, int64_t n, int32_t* out, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_i64_to_i32, grid1(n, 256), dim3(256), 0, s, in, n, out);
  return hipGetLastError();
}

size_t scan_tmp_bytes(int64_t n) { return (size_t)(ceil_div(n > 0 ? n : 1, kScanTile) + 1) * sizeof(int64_t); }

hipError_t launch_exclusive_scan_i64(const int64_t* in, int64_t* out, int64_t n, void* tmp, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  if (n <= kScanSmallMax) {
    hipLaunchKernelGGL(k_scan_small, dim3(1), dim3(kScanBlock), 0, s, in, n, out);
    return hipGetLastError();
  }
  const int64_t nb = ceil_div(n, kScanTile);
  int64_t* sums = static_cast<int64_t*>(tmp);
  hipLaunchKernelGGL(k_scan_reduce, dim3((unsigned)nb), dim3(kScanBlock), 0, s, in, n, sums);
  hipLaunchKernelGGL(k_scan_sums, dim3(1), dim3(kScanBlock), 0, s, sums, nb);
  hipLaunchKernelGGL(k_scan_down, dim3((unsigned)nb), dim3(kScanBlock), 0, s, in, n, sums, out);
  return hipGetLastError();
}

size_t csort_tmp_bytes(int64_t n, int nl) {
  const int64_t nb = ceil_div(n > 0 ? n : 1, kSortBlock);
  const int64_t m = nb * nl;
  return (size_t)m * 2 * sizeof(int64_t) + scan_tmp_bytes(m) + 256;
}

hipError_t launch_counting_sort(const int64_t* labels, int64_t n, int nl, int64_t* perm, int64_t* list_off,
                                void* tmp, size_t tmp_bytes, hipStream_t s) {
  if (tmp_bytes < csort_tmp_bytes(n, nl)) return hipErrorInvalidValue;
  if ((size_t)nl * sizeof(int) > 160 * 1024) return hipErrorInvalidValue;
  const int64_t nb = ceil_div(n > 0 ? n : 1, kSortBlock);
  const int64_t m = nb * nl;
  int64_t* counts = static_cast<int64_t*>(tmp);
  int64_t* offs = counts + m;
  void* stmp = offs + m;
  const size_t lds = (size_t)nl * sizeof(int);
  static const hipError_t a1 = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_sort_hist),
                                                   hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  static const hipError_t a2 = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_sort_scatter),
                                                   hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  if (a1 != hipSuccess) return a1;
  if (a2 != hipSuccess) return a2;
  if (n > 0) {
    hipLaunchKernelGGL(k_sort_hist, dim3((unsigned)nb), dim3(kSortBlock), lds, s, labels, n, nl, nb, counts);
    hipError_t e = launch_exclusive_scan_i64(counts, offs, m, stmp, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_sort_scatter, dim3((unsigned)nb), dim3(kSortBlock), lds, s, labels, n, nl, nb, offs, perm);
    hipLaunchKernelGGL(k_list_off_from_offs, grid1(nl + 1, 256), dim3(256), 0, s, offs, nl, nb, n, list_off);
  } else {
    hipError_t e = hipMemsetAsync(list_off, 0, sizeof(int64_t) * (nl + 1), s);
    if (e != hipSuccess) return e;
  }
  return hipGetLastError();
}

hipError_t launch_probe_map(const int64_t* probes, int64_t nq, int np, int n_lists, const int64_t* list_goff,
                            int chunk_groups, int qtile, int* counts, int* fill, int* bucket_off, int* work_off,
                            int64_t* bucket_q, int64_t* bucket_slot, int64_t* qp_slots, int64_t* slot_begin,
                            void* scan_tmp, size_t scan_tmp_bytes_, hipStream_t s) {
  const int64_t n = nq * np;
  if (scan_tmp_bytes_ < scan_tmp_bytes(n) + sizeof(int64_t) * (size_t)n) return hipErrorInvalidValue;
  int64_t* qp_base = static_cast<int64_t*>(scan_tmp);
  void* stmp = qp_base + n;
  if (n > 0 && n <= kPmSmallMax && n_lists <= kPmSmallLists) {
    hipLaunchKernelGGL(k_probe_map_small, dim3(1), dim3(1024), 0, s, probes, nq, np, n_lists, list_goff, chunk_groups,
                       qtile, counts, bucket_off, work_off, bucket_q, bucket_slot, qp_slots, slot_begin);
    (void)fill;
    return hipGetLastError();
  }
  hipError_t e = hipMemsetAsync(counts, 0, sizeof(int) * n_lists, s);
  if (e != hipSuccess) return e;
  // LDS-histogram form once the entries outnumber the lists (a chunk then repeats lists)
  const bool lds = n_lists <= kPmMaxLists && n >= 2 * (int64_t)n_lists;
  const size_t lds_bytes = sizeof(int) * (size_t)n_lists;
  if (lds) {
    static const hipError_t a1 = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_probe_count_lds),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize,
                                                     (int)(sizeof(int) * kPmMaxLists));
    static const hipError_t a2 = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_probe_fill_lds),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize,
                                                     (int)(sizeof(int) * kPmMaxLists));
    if (a1 != hipSuccess) return a1;
    if (a2 != hipSuccess) return a2;
    hipLaunchKernelGGL(k_probe_count_lds, grid1(n, kPmChunk), dim3(1024), lds_bytes, s, probes, n, n_lists, counts);
  } else {
    hipLaunchKernelGGL(k_probe_count, grid1(n, 256), dim3(256), 0, s, probes, n, counts);
  }
  hipLaunchKernelGGL(k_probe_prefix, dim3(1), dim3(1024), 0, s, counts, n_lists, list_goff, chunk_groups, qtile,
                     bucket_off, work_off, fill);
  if (lds)
    hipLaunchKernelGGL(k_probe_fill_lds, grid1(n, kPmChunk), dim3(1024), lds_bytes, s, probes, n, np, n_lists,
                       bucket_off, fill, bucket_q, bucket_slot, list_goff, chunk_groups, qp_slots);
  else
    hipLaunchKernelGGL(k_probe_fill, grid1(n, 256), dim3(256), 0, s, probes, n, np, bucket_off, fill, bucket_q,
                       bucket_slot, list_goff, chunk_groups, qp_slots);
  if (slot_begin == nullptr) return hipGetLastError();  // (K13: no per-(query, probe) output slots)
  e = launch_exclusive_scan_i64(qp_slots, qp_base, n, stmp, s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_bucket_slot_begin, grid1(n > nq ? n : nq + 1, 256), dim3(256), 0, s, bucket_slot, n, qp_base,
                     qp_slots, nq, np, slot_begin);
  return hipGetLastError();
}

int probe_map_dev_max_lists() { return kPmSmallLists; }

hipError_t launch_probe_map_dev(const int* n_dev, int64_t cap, const int64_t* ovf_q, const int64_t* probes, int np,
                                int n_lists, const int64_t* list_goff, int chunk_groups, int qtile, int* counts,
                                int* bucket_off, int* work_off, int64_t* bucket_q, int64_t* bucket_slot,
                                int64_t* slot_begin, int* zero, hipStream_t s) {
  if (n_lists <= 0 || n_lists > kPmSmallLists || np <= 0 || cap < 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_probe_map_dev, dim3(1), dim3(1024), 0, s, n_dev, cap, ovf_q, probes, np, n_lists, list_goff,
                     chunk_groups, qtile, counts, bucket_off, work_off, bucket_q, bucket_slot, slot_begin, zero);
  return hipGetLastError();
}

hipError_t launch_single_list_job(int64_t nq, int64_t chunks, int qtile, int64_t* bucket_q, int64_t* bucket_slot,
                                  int* bucket_off, int* work_off, int64_t* slot_begin, hipStream_t s, int* zero) {
  hipLaunchKernelGGL(k_single_job, grid1(nq, 256), dim3(256), 0, s, nq, chunks, qtile, bucket_q, bucket_slot,
                     bucket_off, work_off, slot_begin, zero);
  return hipGetLastError();
}

hipError_t launch_iota_i64(int64_t* out, int64_t n, int64_t start, int64_t step, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_iota, grid1(n, 256), dim3(256), 0, s, out, n, start, step);
  return hipGetLastError();
}

hipError_t launch_fill_i32(int* out, int64_t n, int v, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_fill_i32, grid1(n, 256), dim3(256), 0, s, out, n, v);
  return hipGetLastError();
}

hipError_t launch_fill2_i32(int* o1, int64_t n1, int v1, int* o2, int64_t n2, int v2, hipStream_t s) {
  const int64_t n = n1 > n2 ? n1 : n2;
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_fill2_i32, grid1(n, 256), dim3(256), 0, s, o1, n1, v1, o2, n2, v2);
  return hipGetLastError();
}

hipError_t launch_group_list(const int64_t* list_goff, int n_lists, int64_t n_groups, int* group_list,
                             hipStream_t s) {
  if (n_groups <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_group_list, grid1(n_groups, 256), dim3(256), 0, s, list_goff, n_lists, n_groups, group_list);
  return hipGetLastError();
}

}  // namespace mivs
