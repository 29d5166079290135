// K6 list fill + row norms, K5 deterministic k-means update, and the synthetic
// corpus generator. All HBM-bound streaming kernels.
#include "mivs_common.hpp"

namespace mivs {

namespace {

__device__ __forceinline__ float4 ld4(const float* __restrict__ row, int c, int d) {
  if ((d & 3) == 0 && c + 4 <= d) return *reinterpret_cast<const float4*>(row + c);
  float4 v;
  v.x = c + 0 < d ? row[c + 0] : 0.0f;
  v.y = c + 1 < d ? row[c + 1] : 0.0f;
  v.z = c + 2 < d ? row[c + 2] : 0.0f;
  v.w = c + 3 < d ? row[c + 3] : 0.0f;
  return v;
}

// One wave per destination group: gathers its 32 source rows (sorted list order) into the group image (a row's
// dims in 256-B blocks of 64, the 32 rows' blocks side by side: [dp/64][32][64]) and writes the row norms in the
// mivs k-order (k = 8s+j then 8s+4+j). Per 64-dim block the copy moves whole 256-B row pieces -- lane (i, c) =
// (lane >> 4, lane & 15) carries dims 4c .. 4c + 3 of rows 4 rb + i -- so each wave-instruction reads four 256-B
// source segments and writes 1 KiB contiguous (the round-4 kernel moved 32-B pieces both ways: 2.2 TB/s,
// build_roofline "pack"); the next block's loads are in flight while this one is stored. The norm chain runs over
// a padded LDS copy of the block (row stride 68 floats: conflict-free ds_read_b128), lane (rr, h) = (lane & 31,
// lane >> 5) holding dims 8t + 4h .. + 3 of row rr and taking its lane^32 partner's by shuffle, as before.
__global__ __launch_bounds__(256) void k_pack(const float* __restrict__ src, int d, int dp,
                                              const int64_t* __restrict__ src_index,
                                              const int64_t* __restrict__ list_off,
                                              const int64_t* __restrict__ list_goff,
                                              const int* __restrict__ group_list, int64_t n_groups,
                                              float* __restrict__ groups, float* __restrict__ norms,
                                              int64_t* __restrict__ ids_out, const int64_t* __restrict__ id_map,
                                              int64_t id_offset) {
  constexpr int LDSR = kRowBlk + 4;  // padded row stride of the staged block (floats)
  __shared__ __attribute__((aligned(16))) float s_blk[4][kGroupRows * LDSR];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t g = (int64_t)blockIdx.x * 4 + w;
  if (g >= n_groups) return;  // (no workgroup barrier below: each wave stages in its own LDS slice)
  const int l = group_list ? group_list[g] : 0;
  const int64_t r0 = (g - list_goff[l]) * kGroupRows;
  const int64_t size = list_off[l + 1] - list_off[l];
  const int i4 = lane >> 4, c = lane & 15;
  const float* rp[8];
  bool rv[8];
#pragma unroll
  for (int rb = 0; rb < 8; ++rb) {
    const int64_t r = r0 + 4 * rb + i4;
    rv[rb] = r < size;
    const int64_t sidx = list_off[l] + r;
    rp[rb] = src + (rv[rb] ? (src_index ? src_index[sidx] : sidx) : 0) * (int64_t)d;
  }
  float* gb = groups + g * (int64_t)(kGroupRows * dp) + (int64_t)i4 * kRowBlk + 4 * c;
  float* sb = s_blk[w];
  const int rr = lane & 31, h = lane >> 5;
  float acc = 0.0f;
  const int NB = dp / kRowBlk;
  float4 v[8];
  auto load = [&](int blk, float4 (&o)[8]) {
#pragma unroll
    for (int rb = 0; rb < 8; ++rb) {
      o[rb] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (rv[rb]) o[rb] = ld4(rp[rb], kRowBlk * blk + 4 * c, d);
    }
  };
  load(0, v);
  for (int blk = 0; blk < NB; ++blk) {
    float4 nv[8];
    if (blk + 1 < NB) load(blk + 1, nv);
#pragma unroll
    for (int rb = 0; rb < 8; ++rb) {
      __builtin_nontemporal_store(__builtin_bit_cast(f32x4, v[rb]), reinterpret_cast<f32x4*>(gb + (int64_t)blk * kRowBlkStride + 4 * rb * kRowBlk));
      *reinterpret_cast<float4*>(sb + (4 * rb + i4) * LDSR + 4 * c) = v[rb];
    }
    // the reads below take other lanes' stores above (and the next block's stores must not pass this block's reads):
    // order them explicitly at wave scope rather than relying on in-order LDS within a wave
    wave_lds_sync();
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const float4 u = *reinterpret_cast<const float4*>(sb + rr * LDSR + 8 * t + 4 * h);
      const float px = __shfl_xor(u.x, 32), py = __shfl_xor(u.y, 32);
      const float pz = __shfl_xor(u.z, 32), pw = __shfl_xor(u.w, 32);
      acc = fmaf(u.x, u.x, acc); acc = fmaf(px, px, acc);
      acc = fmaf(u.y, u.y, acc); acc = fmaf(py, py, acc);
      acc = fmaf(u.z, u.z, acc); acc = fmaf(pz, pz, acc);
      acc = fmaf(u.w, u.w, acc); acc = fmaf(pw, pw, acc);
    }
#pragma unroll
    for (int rb = 0; rb < 8; ++rb) v[rb] = nv[rb];
    wave_lds_sync();
  }
  if (h == 0) {
    const int64_t r = r0 + rr;
    const bool valid = r < size;
    const int64_t sidx = list_off[l] + r;
    const int64_t srow = valid ? (src_index ? src_index[sidx] : sidx) : 0;
    const int64_t pos = g * kGroupRows + rr;
    norms[pos] = valid ? acc : INFINITY;
    if (ids_out) ids_out[pos] = valid ? (id_map ? id_map[srow] : srow + id_offset) : (int64_t)-1;
  }
}

// ‖x‖² of plain row-major rows in the mivs k-order (one thread per row)
__global__ void k_row_norms(const float* __restrict__ x, int64_t n, int d, float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float* row = x + i * (int64_t)d;
  const int S = dim_pad(d) >> 3;
  float acc = 0.0f;
  for (int s = 0; s < S; ++s) {
    const float4 a = ld4(row, 8 * s, d), b = ld4(row, 8 * s + 4, d);
    acc = fmaf(a.x, a.x, acc); acc = fmaf(b.x, b.x, acc);
    acc = fmaf(a.y, a.y, acc); acc = fmaf(b.y, b.y, acc);
    acc = fmaf(a.z, a.z, acc); acc = fmaf(b.z, b.z, acc);
    acc = fmaf(a.w, a.w, acc); acc = fmaf(b.w, b.w, acc);
  }
  out[i] = acc;
}

// cosine metric: x / sqrt(‖x‖²) per row (‖x‖² from k_row_norms: the pinned order), a zero row stays
// zero (sklearn normalize / cosine_similarity; VectorSearch_QuestionRetrieval.ipynb:839,878). One
// thread per 4 consecutive floats of the row-major matrix (d % 4 == 0) or per float.
template <int V>
__global__ void k_scale_rows(const float* __restrict__ x, const float* __restrict__ n2, int64_t n, int d,
                             float* __restrict__ out) {
  const int64_t nv = n * (int64_t)d / V;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nv; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = t * V;
    const float nrm = sqrtf(n2[e / d]);
    if constexpr (V == 4) {
      float4 v = *reinterpret_cast<const float4*>(x + e);
      if (nrm > 0.0f) { v.x /= nrm; v.y /= nrm; v.z /= nrm; v.w /= nrm; }
      else v = make_float4(0.f, 0.f, 0.f, 0.f);
      *reinterpret_cast<float4*>(out + e) = v;
    } else {
      out[e] = nrm > 0.0f ? x[e] / nrm : 0.0f;
    }
  }
}

// The same ‖x‖² for few rows (the query batch): one wave per row, the row staged coalesced in LDS and
// lane 0 running the chain (every row's loads in flight at once: 16 us for 10k x 768 against 247 us
// for a thread per row, whose lanes each touch their own cache lines)
__global__ __launch_bounds__(256) void k_row_norms_w(const float* __restrict__ x, int64_t n, int d,
                                                     float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) float t[];  // [4][dpad]
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t r = (int64_t)blockIdx.x * 4 + w;
  const int dpad = dim_pad(d);
  if (r < n)
    for (int c = lane; c < dpad; c += 64) t[w * dpad + c] = c < d ? x[r * d + c] : 0.0f;
  __syncthreads();
  if (r < n && lane == 0) {
    const float* my = t + w * dpad;
    float acc = 0.0f;
    for (int s = 0; s < dpad; s += 8) {
      const float4 a = *reinterpret_cast<const float4*>(my + s), b = *reinterpret_cast<const float4*>(my + s + 4);
      acc = fmaf(a.x, a.x, acc); acc = fmaf(b.x, b.x, acc);
      acc = fmaf(a.y, a.y, acc); acc = fmaf(b.y, b.y, acc);
      acc = fmaf(a.z, a.z, acc); acc = fmaf(b.z, b.z, acc);
      acc = fmaf(a.w, a.w, acc); acc = fmaf(b.w, b.w, acc);
    }
    out[r] = acc;
  }
}

__device__ __forceinline__ int find_list(const int64_t* __restrict__ off, int n_lists, int64_t r) {
  int lo = 0, hi = n_lists - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (off[mid] <= r) lo = mid; else hi = mid - 1;
  }
  return lo;
}

// interleaved groups -> row-major rows in list order (for parity tests / export)
__global__ void k_unpack(const float* __restrict__ groups, int dp, int d, const int64_t* __restrict__ list_off,
                         const int64_t* __restrict__ list_goff, int n_lists, int64_t n_rows,
                         float* __restrict__ out) {
  // grid-stride: n_rows * d can exceed the 2^32 work-item limit of one launch
  const int64_t total = n_rows * (int64_t)d;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += stride) {
    const int64_t row = t / d;
    const int c = (int)(t - row * d);
    const int l = find_list(list_off, n_lists, row);
    const int64_t r = row - list_off[l];
    const int64_t g = list_goff[l] + r / kGroupRows;
    const int rr = (int)(r % kGroupRows);
    out[t] = groups[row_elem(g * kGroupRows + rr, c, dp)];
  }
}

__global__ void k_compact_ids(const int64_t* __restrict__ row_ids, const int64_t* __restrict__ list_off,
                              const int64_t* __restrict__ list_goff, int n_lists, int64_t n_rows,
                              int64_t* __restrict__ out) {
  const int64_t row = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= n_rows) return;
  const int l = find_list(list_off, n_lists, row);
  out[row] = row_ids[list_goff[l] * kGroupRows + (row - list_off[l])];
}

__global__ void k_gather_rows(const float* __restrict__ src, int d, const int64_t* __restrict__ rows, int64_t n,
                              float* __restrict__ dst) {
  const int64_t total = n * (int64_t)d;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += stride) {
    const int64_t i = t / d;
    const int c = (int)(t - i * d);
    dst[t] = src[rows[i] * (int64_t)d + c];
  }
}

// ---- k-means update (K5): fixed member order, fp64 partials over kKmChunk members ----
__global__ void k_km_chunks(const int64_t* __restrict__ list_off, int nc, int64_t* __restrict__ cnt) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c < nc) cnt[c] = ceil_div(list_off[c + 1] - list_off[c], kKmChunk);
  if (c == nc) cnt[nc] = 0;
}

__global__ __launch_bounds__(256) void k_km_partial(const float* __restrict__ x, int d,
                                                    const int64_t* __restrict__ rows,
                                                    const int64_t* __restrict__ perm,
                                                    const int64_t* __restrict__ list_off,
                                                    const int64_t* __restrict__ chunk_off, int nc,
                                                    double* __restrict__ partial) {
  const int64_t b = blockIdx.x;
  if (b >= chunk_off[nc]) return;
  int lo = 0, hi = nc - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (chunk_off[mid] <= b) lo = mid; else hi = mid - 1;
  }
  const int c = lo;
  const int64_t m0 = list_off[c] + (b - chunk_off[c]) * kKmChunk;
  const int64_t m1 = m0 + kKmChunk < list_off[c + 1] ? m0 + kKmChunk : list_off[c + 1];
  const int cnt = (int)(m1 - m0);
  // the chunk's member rows once into LDS (the perm -> rows -> x chain is then one load deep), then 8
  // member loads in flight per dim; the fp64 sum keeps the member order (orc_kmeans_update)
  __shared__ int64_t s_row[kKmChunk];
  for (int i = threadIdx.x; i < cnt; i += blockDim.x) {
    const int64_t t = perm[m0 + i];
    s_row[i] = rows ? rows[t] : t;
  }
  __syncthreads();
  for (int dim = threadIdx.x; dim < d; dim += blockDim.x) {
    double s = 0.0;
    int m = 0;
    for (; m + 8 <= cnt; m += 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = x[s_row[m + u] * d + dim];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += (double)v[u];
    }
    for (; m < cnt; ++m) s += (double)x[s_row[m] * d + dim];
    partial[b * d + dim] = s;
  }
}

__global__ __launch_bounds__(256) void k_km_final(const double* __restrict__ partial,
                                                  const int64_t* __restrict__ chunk_off,
                                                  const int64_t* __restrict__ list_off, int d,
                                                  float* __restrict__ cent) {
  const int c = blockIdx.x;
  const int64_t cnt = list_off[c + 1] - list_off[c];
  if (cnt == 0) return;  // empty cluster keeps its centroid
  for (int dim = threadIdx.x; dim < d; dim += blockDim.x) {
    double tot = 0.0;
    for (int64_t b = chunk_off[c]; b < chunk_off[c + 1]; ++b) tot += partial[b * d + dim];
    cent[(int64_t)c * d + dim] = (float)(tot / (double)cnt);
  }
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// Balancing step (cuVS kmeans_balanced adjust_centers, restated in oracle orc_kmeans_rebalance):
// a centroid j whose cluster holds fewer than kBalFrac x the average members is pulled next to the
// centroid of an over-average cluster L found by probing train positions (r0 + p*kBalStep) mod n:
// c_j = (wc * c_L + x_t) / (wc + 1), wc = min(size_j, 4). Big clusters are never written, so the
// blocks are independent. One block per centroid.
constexpr double kBalFrac = 0.25;
constexpr float kBalWc = 4.0f;
constexpr int kBalProbes = 64;
constexpr uint64_t kBalStep = 2654435761ull;
constexpr uint64_t kBalSeed = 0x5851F42D4C957F2Dull;

__global__ __launch_bounds__(256) void k_km_rebalance(const float* __restrict__ x, int d,
                                                      const int64_t* __restrict__ rows,
                                                      const int64_t* __restrict__ labels,
                                                      const int64_t* __restrict__ list_off, int nc,
                                                      int64_t n_train, int it, float* __restrict__ cent) {
  __shared__ int64_t donor;
  const int c = blockIdx.x;
  const double avg = (double)n_train / (double)nc;
  const int64_t size = list_off[c + 1] - list_off[c];
  if (!((double)size < kBalFrac * avg)) return;
  if (threadIdx.x == 0) {
    donor = -1;
    const uint64_t r0 = splitmix64(kBalSeed ^ ((uint64_t)it << 32) ^ (uint64_t)c) % (uint64_t)n_train;
    for (int p = 0; p < kBalProbes; ++p) {
      const int64_t t = (int64_t)((r0 + (uint64_t)p * kBalStep) % (uint64_t)n_train);
      const int64_t l = labels[t];
      if ((double)(list_off[l + 1] - list_off[l]) > avg) { donor = t; break; }
    }
  }
  __syncthreads();
  if (donor < 0) return;
  const int64_t row = rows ? rows[donor] : donor;
  const int64_t L = labels[donor];
  const float wc = (float)size < kBalWc ? (float)size : kBalWc;
  for (int dim = threadIdx.x; dim < d; dim += blockDim.x) {
    float v = wc * cent[L * d + dim];
    v = v + x[row * d + dim];
    cent[(int64_t)c * d + dim] = v / (wc + 1.0f);
  }
}

// ---- synthetic clustered corpus (bench / large-scale tests) ----

// Irwin-Hall(4) approximation of N(0,1) from one 64-bit hash (exact integer -> fp32 steps)
__device__ __forceinline__ float gauss4(uint64_t h) {
  float s = 0.0f;
#pragma unroll
  for (int i = 0; i < 4; ++i) s += ((float)((h >> (16 * i)) & 0xFFFFull) + 0.5f) * (1.0f / 65536.0f);
  return (s - 2.0f) * 1.7320508075688772f;
}

// row i: centre c = H(seed, i) mod n_centers; x = C[c] + sigma * e; optionally L2-normalised.
__global__ __launch_bounds__(256) void k_synth(float* __restrict__ out, int64_t row_begin, int64_t n, int d,
                                               uint64_t seed, int n_centers, float sigma, int normalize) {
  const int lane = threadIdx.x & 63;
  const int64_t li = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (li >= n) return;
  const uint64_t gi = (uint64_t)(row_begin + li);
  const uint64_t cs = splitmix64(seed ^ 0xC2B2AE3D27D4EB4Full);
  const uint64_t es = splitmix64(seed ^ 0x165667B19E3779F9ull);
  const uint64_t c = splitmix64(seed * 0xD1B54A32D192ED03ull + gi) % (uint64_t)n_centers;
  float ss = 0.0f;
  float* row = out + li * (int64_t)d;
  for (int k = lane; k < d; k += 64) {
    const float cv = gauss4(splitmix64(cs + c * 0x100000001B3ull * 1315423911ull + (uint64_t)k));
    const float ev = gauss4(splitmix64(es + gi * 0x9E3779B97F4A7C15ull + (uint64_t)k * 0xBF58476D1CE4E5B9ull));
    const float v = cv + sigma * ev;
    row[k] = v;
    ss = fmaf(v, v, ss);
  }
  if (normalize) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) ss += __shfl_xor(ss, o);
    const float inv = ss > 0.0f ? 1.0f / sqrtf(ss) : 0.0f;
    for (int k = lane; k < d; k += 64) row[k] *= inv;
  }
}

inline dim3 grid1(int64_t n, int b) { return dim3((unsigned)ceil_div(n > 0 ? n : 1, b)); }
// for grid-stride kernels: cap so blocks * 256 stays far below the 2^32 work-item limit
inline dim3 grid_capped(int64_t n, int b) {
  const int64_t g = ceil_div(n > 0 ? n : 1, b);
  return dim3((unsigned)(g < (1 << 20) ? g : (1 << 20)));
}

}  // namespace

hipError_t launch_pack_groups(const float* src, int64_t /*src_rows_total*/, int d, int dp, const int64_t* src_index,
                              const int64_t* list_off, const int64_t* list_goff, const int* group_list,
                              int64_t n_groups, float* groups, float* norms, int64_t* ids_out,
                              const int64_t* id_map, int64_t id_offset, hipStream_t s) {
  if (n_groups <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_pack, grid1(n_groups, 4), dim3(256), 0, s, src, d, dp, src_index, list_off, list_goff,
                     group_list, n_groups, groups, norms, ids_out, id_map, id_offset);
  return hipGetLastError();
}

hipError_t launch_normalize_rows(const float* x, int64_t n, int d, float* n2, float* out, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipError_t e = launch_row_norms(x, n, d, n2, s);
  if (e != hipSuccess) return e;
  const bool v4 = d % 4 == 0 && (reinterpret_cast<uintptr_t>(x) % 16) == 0 && (reinterpret_cast<uintptr_t>(out) % 16) == 0;
  const int64_t nv = n * (int64_t)d / (v4 ? 4 : 1);
  const int grid = (int)std::min<int64_t>((nv + 255) / 256, 65536);
  if (v4) hipLaunchKernelGGL(k_scale_rows<4>, dim3(grid), dim3(256), 0, s, x, n2, n, d, out);
  else hipLaunchKernelGGL(k_scale_rows<1>, dim3(grid), dim3(256), 0, s, x, n2, n, d, out);
  return hipGetLastError();
}

hipError_t launch_row_norms(const float* x, int64_t n, int d, float* out, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  // few rows (query batches): a wave per row; many rows: a thread per row (12 ms at 10M x 768 against
  // 14.5 ms for the wave-per-row and 21.9 ms for the 64-row LDS-tile kernels, measured)
  if (n <= (1 << 20) && dim_pad(d) <= 4096)
    hipLaunchKernelGGL(k_row_norms_w, dim3((unsigned)((n + 3) / 4)), dim3(256), (size_t)16 * dim_pad(d), s, x, n, d,
                       out);
  else hipLaunchKernelGGL(k_row_norms, grid1(n, 256), dim3(256), 0, s, x, n, d, out);
  return hipGetLastError();
}

hipError_t launch_unpack_rows(const float* groups, int dp, int d, const int64_t* list_off, const int64_t* list_goff,
                              int n_lists, int64_t n_rows, float* out, hipStream_t s) {
  if (n_rows <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_unpack, grid_capped(n_rows * d, 256), dim3(256), 0, s, groups, dp, d, list_off, list_goff, n_lists,
                     n_rows, out);
  return hipGetLastError();
}

hipError_t launch_compact_ids(const int64_t* row_ids, const int64_t* list_off, const int64_t* list_goff,
                              int n_lists, int64_t n_rows, int64_t* out, hipStream_t s) {
  if (n_rows <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_compact_ids, grid1(n_rows, 256), dim3(256), 0, s, row_ids, list_off, list_goff, n_lists,
                     n_rows, out);
  return hipGetLastError();
}

hipError_t launch_gather_rows(const float* src, int d, const int64_t* rows, int64_t n, float* dst, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_gather_rows, grid_capped(n * d, 256), dim3(256), 0, s, src, d, rows, n, dst);
  return hipGetLastError();
}

size_t km_partial_rows(int64_t n_members, int nc) { return (size_t)(ceil_div(n_members, kKmChunk) + nc); }

hipError_t launch_km_update(const float* x, int d, const int64_t* rows, const int64_t* perm,
                            const int64_t* list_off, int nc, int64_t n_members, double* partial,
                            int64_t* chunk_off, void* tmp, float* centroids, hipStream_t s) {
  hipLaunchKernelGGL(k_km_chunks, grid1(nc + 1, 256), dim3(256), 0, s, list_off, nc, chunk_off);
  // in-place exclusive scan via tmp copy: chunk_off holds counts; scan into tmp area then copy back
  int64_t* cnt_copy = static_cast<int64_t*>(tmp);
  hipError_t e = hipMemcpyAsync(cnt_copy, chunk_off, sizeof(int64_t) * (nc + 1), hipMemcpyDeviceToDevice, s);
  if (e != hipSuccess) return e;
  e = launch_exclusive_scan_i64(cnt_copy, chunk_off, nc + 1, cnt_copy + (nc + 1), s);
  if (e != hipSuccess) return e;
  const int64_t bound = (int64_t)km_partial_rows(n_members, nc);
  hipLaunchKernelGGL(k_km_partial, dim3((unsigned)bound), dim3(256), 0, s, x, d, rows, perm, list_off, chunk_off, nc,
                     partial);
  hipLaunchKernelGGL(k_km_final, dim3((unsigned)nc), dim3(256), 0, s, partial, chunk_off, list_off, d, centroids);
  return hipGetLastError();
}

hipError_t launch_km_rebalance(const float* x, int d, const int64_t* rows, const int64_t* labels,
                               const int64_t* list_off, int nc, int64_t n_train, int it, float* centroids,
                               hipStream_t s) {
  if (nc <= 0 || n_train <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_km_rebalance, dim3((unsigned)nc), dim3(256), 0, s, x, d, rows, labels, list_off, nc, n_train,
                     it, centroids);
  return hipGetLastError();
}

hipError_t launch_synth_mixture(float* out, int64_t row_begin, int64_t n, int d, uint64_t seed, int n_centers,
                                float sigma, int normalize, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  // one wave per row: launch in slices of 2^24 rows so a launch stays under 2^32 work-items
  constexpr int64_t kSlice = int64_t(1) << 24;
  for (int64_t b = 0; b < n; b += kSlice) {
    const int64_t m = n - b < kSlice ? n - b : kSlice;
    hipLaunchKernelGGL(k_synth, grid1(m, 4), dim3(256), 0, s, out + b * (int64_t)d, row_begin + b, m, d, seed,
                       n_centers, sigma, normalize);
  }
  return hipGetLastError();
}

}  // namespace mivs
