// IVF-PQ kernels (DESIGN.md §"IVF-PQ"): residual extraction for codebook training, encoding
// into the interleaved code layout, and the LUT scan with its per-(query, probe) top-k.
//
// Code layout in HBM: like the IVF-Flat rows, every list starts on a 32-row group; a group
// holds [pq_dim_pad / 16][32 rows][16 codes] bytes, so a half-wave reading one 16-code chunk of
// 32 consecutive rows loads 512 contiguous bytes. Pad rows carry code 0 and id -1 and are skipped
// by the row count of their list.
//
// Arithmetic (oracle/mivs_oracle.c orc_ivfpq_*):
//   residual r = x - c (fp32), dims >= d are 0;
//   ||a - b||^2 over pq_len dims: acc = fmaf(a_i - b_i, a_i - b_i, acc), i ascending;
//   code = argmin over the 2^pq_bits entries (ties: lowest index);
//   dist(row) = sum_j LUT[j][code_j], j ascending, fp32 adds from 0.
#include <climits>

#include "mivs_common.hpp"

namespace mivs {

namespace {

constexpr int kPqCodes = 256;  // pq_bits = 8

__device__ __forceinline__ int pq_find_list(const int64_t* __restrict__ off, int n_lists, int64_t p) {
  int lo = 0, hi = n_lists - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (off[mid] <= p) lo = mid; else hi = mid - 1;
  }
  return lo;
}

// R[j][t][i] = x[rows[t]][j*pl+i] - c[labels[rows[t]]][j*pl+i]   (0 for dims >= d)
__global__ void k_pq_residuals(const float* __restrict__ x, int d, const int64_t* __restrict__ rows, int64_t nt,
                               const int64_t* __restrict__ labels, const float* __restrict__ cents, int pq_dim,
                               int pl, float* __restrict__ out) {
  const int64_t total = nt * (int64_t)pq_dim * pl;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += stride) {
    const int i = (int)(e % pl);
    const int64_t t = (e / pl) % nt;
    const int j = (int)(e / ((int64_t)pl * nt));
    const int k = j * pl + i;
    const int64_t row = rows[t];
    out[e] = k < d ? x[row * d + k] - cents[labels[row] * d + k] : 0.0f;
  }
}

// One thread per list position p (list order), one subspace per blockIdx.y. The codebook of the
// subspace sits in LDS (256 x pl floats); the residual sub-vector in registers (PLMAX >= pl).
template <int PLMAX>
__global__ __launch_bounds__(256) void k_pq_encode(const float* __restrict__ x, int d, const int64_t* __restrict__ perm,
                                                   int64_t n, const int64_t* __restrict__ list_off,
                                                   const int64_t* __restrict__ list_goff, int n_lists,
                                                   const float* __restrict__ cents, const float* __restrict__ books,
                                                   int pl, int pq_dim_pad, uint8_t* __restrict__ codes) {
  extern __shared__ float cb[];  // [256][pl]
  const int j = blockIdx.y;
  for (int i = threadIdx.x; i < kPqCodes * pl; i += blockDim.x) cb[i] = books[(int64_t)j * kPqCodes * pl + i];
  __syncthreads();
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  const int l = pq_find_list(list_off, n_lists, p);
  const int64_t row = perm[p];
  float r[PLMAX];
#pragma unroll
  for (int i = 0; i < PLMAX; ++i) {
    const int k = j * pl + i;
    r[i] = (i < pl && k < d) ? x[row * d + k] - cents[(int64_t)l * d + k] : 0.0f;
  }
  int best = 0;
  float bd = INFINITY;
  for (int c = 0; c < kPqCodes; ++c) {
    const float* b = cb + c * pl;
    float acc = 0.0f;
#pragma unroll
    for (int i = 0; i < PLMAX; ++i) {
      if (i < pl) {
        const float t = r[i] - b[i];
        acc = fmaf(t, t, acc);
      }
    }
    if (acc < bd) { bd = acc; best = c; }
  }
  const int64_t pos = p - list_off[l];
  const int64_t g = list_goff[l] + pos / kGroupRows;
  const int rr = (int)(pos % kGroupRows);
  codes[g * (int64_t)kGroupRows * pq_dim_pad + (int64_t)(j >> 4) * (kGroupRows * 16) + rr * 16 + (j & 15)] =
      (uint8_t)best;
}

// ids of the packed lists: position p -> perm[p] + id_offset; pad rows keep -1 (memset before)
__global__ void k_pq_ids(const int64_t* __restrict__ perm, int64_t n, const int64_t* __restrict__ list_off,
                         const int64_t* __restrict__ list_goff, int n_lists, int64_t id_offset,
                         int64_t* __restrict__ ids) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  const int l = pq_find_list(list_off, n_lists, p);
  ids[list_goff[l] * kGroupRows + (p - list_off[l])] = perm[p] + id_offset;
}

// packed codes -> row-major [n][pq_dim] in list order (export / parity tests)
__global__ void k_pq_unpack(const uint8_t* __restrict__ codes, int64_t n, const int64_t* __restrict__ list_off,
                            const int64_t* __restrict__ list_goff, int n_lists, int pq_dim, int pq_dim_pad,
                            uint8_t* __restrict__ out) {
  const int64_t total = n * (int64_t)pq_dim;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += stride) {
    const int64_t p = e / pq_dim;
    const int j = (int)(e - p * pq_dim);
    const int l = pq_find_list(list_off, n_lists, p);
    const int64_t pos = p - list_off[l];
    const int64_t g = list_goff[l] + pos / kGroupRows;
    const int rr = (int)(pos % kGroupRows);
    out[e] = codes[g * (int64_t)kGroupRows * pq_dim_pad + (int64_t)(j >> 4) * (kGroupRows * 16) + rr * 16 + (j & 15)];
  }
}

template <int KCAP>
__device__ __forceinline__ void pq_insert(float (&lk)[KCAP], int (&lp)[KCAP], float key, int pos) {
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

// K9: one workgroup per (query, probe) slot. LDS: [qres d_pad][LUT pq_dim x 256 | merge area].
//   1. residual q - c_l -> LDS;  2. LUT[j][c] = ||res_j - B_j[c]||^2 -> LDS;
//   3. each thread scans rows tid, tid + NT, ... of the list: dist = sum_j LUT[j][code_j],
//      register top-KCAP by (dist, row position);
//   4. the NT lane lists -> LDS; wave w merges its 64 lists (64-lane min-reduction per rank),
//      then wave 0 merges the NT/64 wave lists; the slot's top-k (dist, id) -> out.
template <int KCAP>
__global__ __launch_bounds__(512) void k_pq_scan(PqScanArgs a) {
  constexpr int NT = 512;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* s_res = reinterpret_cast<float*>(smem);                 // [rot_dim]
  float* lut = s_res + a.rot_dim_pad;                            // [pq_dim][256]
  float* mkey = lut;                                             // merge area (after the scan)
  int* mpos = reinterpret_cast<int*>(mkey + NT * KCAP);
  float* wkey = mkey + 2 * NT * KCAP;                            // [NT/64][k] wave results
  int* wpos = reinterpret_cast<int*>(wkey + (NT / 64) * KCAP);

  const int64_t slot = blockIdx.x;  // = q * n_probes + probe
  const int64_t q = slot / a.n_probes;
  const int l = (int)a.probes[slot];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  if (l < 0) {  // no probe (degenerate query): empty slot
    for (int t = tid; t < a.k; t += NT) {
      a.out_d[slot * a.k + t] = INFINITY;
      a.out_i[slot * a.k + t] = -1;
    }
    return;
  }
  const int pl = a.pq_len;
  for (int i = tid; i < a.rot_dim_pad; i += NT)
    s_res[i] = i < a.d ? a.queries[q * a.d + i] - a.cents[(int64_t)l * a.d + i] : 0.0f;
  __syncthreads();
  const int nlut = a.pq_dim * kPqCodes;
  for (int e = tid; e < nlut; e += NT) {
    const int j = e >> 8;
    const float* b = a.books + (int64_t)e * pl;
    const float* r = s_res + j * pl;
    float acc = 0.0f;
    for (int i = 0; i < pl; ++i) {
      const float t = r[i] - b[i];
      acc = fmaf(t, t, acc);
    }
    lut[e] = acc;
  }
  __syncthreads();

  float lk[KCAP];
  int lp[KCAP];
#pragma unroll
  for (int t = 0; t < KCAP; ++t) { lk[t] = INFINITY; lp[t] = INT_MAX; }
  const int64_t r0 = a.list_off[l], nrows = a.list_off[l + 1] - r0;
  const int64_t g0 = a.list_goff[l];
  const int nchunk = a.pq_dim_pad >> 4;
  for (int64_t r = tid; r < nrows; r += NT) {
    const uint8_t* cg = a.codes + (g0 + r / kGroupRows) * (int64_t)kGroupRows * a.pq_dim_pad + (r % kGroupRows) * 16;
    float dist = 0.0f;
    int j = 0;
    for (int ch = 0; ch < nchunk; ++ch) {
      const uint4 w = *reinterpret_cast<const uint4*>(cg + (int64_t)ch * (kGroupRows * 16));
      const uint32_t wv[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
      for (int b = 0; b < 16; ++b) {
        if (j + b < a.pq_dim) dist = dist + lut[((j + b) << 8) + ((wv[b >> 2] >> (8 * (b & 3))) & 0xFF)];
      }
      j += 16;
    }
    if (dist < lk[KCAP - 1]) pq_insert<KCAP>(lk, lp, dist, (int)r);
  }
  __syncthreads();  // LUT dead: the merge area aliases it
#pragma unroll
  for (int t = 0; t < KCAP; ++t) {
    mkey[tid * KCAP + t] = lk[t];
    mpos[tid * KCAP + t] = lp[t];
  }
  __syncthreads();
  // stage 1: wave w merges lane lists w*64 .. w*64+63
  {
    const float* myk = mkey + tid * KCAP;
    const int* myp = mpos + tid * KCAP;
    int head = 0;
    float hk = myk[0];
    int hp = myp[0];
    for (int t = 0; t < a.k; ++t) {
      float bk = hk;
      int bp = hp;
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) {
        const float ok = __shfl_xor(bk, off);
        const int op = __shfl_xor(bp, off);
        if (ok < bk || (ok == bk && op < bp)) { bk = ok; bp = op; }
      }
      if (lane == 0) { wkey[wave * KCAP + t] = bk; wpos[wave * KCAP + t] = bp; }
      if (hk == bk && hp == bp && head < KCAP) {
        ++head;
        hk = head < KCAP ? myk[head] : INFINITY;
        hp = head < KCAP ? myp[head] : INT_MAX;
      }
    }
  }
  __syncthreads();
  // stage 2: wave 0, lanes 0..NT/64-1 hold the wave lists
  if (wave == 0) {
    constexpr int NW = NT / 64;
    const bool src = lane < NW;
    const float* myk = wkey + (src ? lane : 0) * KCAP;
    const int* myp = wpos + (src ? lane : 0) * KCAP;
    int head = 0;
    float hk = src ? myk[0] : INFINITY;
    int hp = src ? myp[0] : INT_MAX;
    for (int t = 0; t < a.k; ++t) {
      float bk = hk;
      int bp = hp;
#pragma unroll
      for (int off = NW / 2; off >= 1; off >>= 1) {
        const float ok = __shfl_xor(bk, off, NW);
        const int op = __shfl_xor(bp, off, NW);
        if (ok < bk || (ok == bk && op < bp)) { bk = ok; bp = op; }
      }
      if (lane == 0) {
        const bool valid = bp != INT_MAX;
        a.out_d[slot * a.k + t] = valid ? bk : INFINITY;
        a.out_i[slot * a.k + t] = valid ? a.row_ids[g0 * kGroupRows + bp] : (int64_t)-1;
      }
      if (src && hk == bk && hp == bp && head < a.k) {
        ++head;
        hk = head < a.k ? myk[head] : INFINITY;
        hp = head < a.k ? myp[head] : INT_MAX;
      }
    }
  }
}

inline dim3 gridc(int64_t n, int b) {
  const int64_t g = ceil_div(n > 0 ? n : 1, b);
  return dim3((unsigned)(g < (1 << 20) ? g : (1 << 20)));
}

}  // namespace

size_t pq_scan_lds_bytes(int rot_dim_pad, int pq_dim, int kcap) {
  const size_t lut = (size_t)pq_dim * kPqCodes * 4;
  const size_t merge = (size_t)512 * kcap * 8 + (size_t)8 * kcap * 8;
  return (size_t)rot_dim_pad * 4 + (lut > merge ? lut : merge);
}

hipError_t launch_pq_residuals(const float* x, int d, const int64_t* rows, int64_t nt, const int64_t* labels,
                               const float* cents, int pq_dim, int pl, float* out, hipStream_t s) {
  if (nt <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_pq_residuals, gridc(nt * pq_dim * pl, 256), dim3(256), 0, s, x, d, rows, nt, labels, cents,
                     pq_dim, pl, out);
  return hipGetLastError();
}

hipError_t launch_pq_encode(const float* x, int d, const int64_t* perm, int64_t n, const int64_t* list_off,
                            const int64_t* list_goff, int n_lists, const float* cents, const float* books, int pq_dim,
                            int pl, int pq_dim_pad, uint8_t* codes, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  if (pl > 64) return hipErrorInvalidValue;
  const dim3 grid((unsigned)ceil_div(n, 256), (unsigned)pq_dim);
  const size_t lds = (size_t)kPqCodes * pl * 4;
  if (pl <= 8) hipLaunchKernelGGL(k_pq_encode<8>, grid, dim3(256), lds, s, x, d, perm, n, list_off, list_goff, n_lists, cents, books, pl, pq_dim_pad, codes);
  else if (pl <= 16) hipLaunchKernelGGL(k_pq_encode<16>, grid, dim3(256), lds, s, x, d, perm, n, list_off, list_goff, n_lists, cents, books, pl, pq_dim_pad, codes);
  else if (pl <= 32) hipLaunchKernelGGL(k_pq_encode<32>, grid, dim3(256), lds, s, x, d, perm, n, list_off, list_goff, n_lists, cents, books, pl, pq_dim_pad, codes);
  else hipLaunchKernelGGL(k_pq_encode<64>, grid, dim3(256), lds, s, x, d, perm, n, list_off, list_goff, n_lists, cents, books, pl, pq_dim_pad, codes);
  return hipGetLastError();
}

hipError_t launch_pq_ids(const int64_t* perm, int64_t n, const int64_t* list_off, const int64_t* list_goff,
                         int n_lists, int64_t id_offset, int64_t* ids, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_pq_ids, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, s, perm, n, list_off, list_goff,
                     n_lists, id_offset, ids);
  return hipGetLastError();
}

hipError_t launch_pq_unpack(const uint8_t* codes, int64_t n, const int64_t* list_off, const int64_t* list_goff,
                            int n_lists, int pq_dim, int pq_dim_pad, uint8_t* out, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_pq_unpack, gridc(n * pq_dim, 256), dim3(256), 0, s, codes, n, list_off, list_goff, n_lists,
                     pq_dim, pq_dim_pad, out);
  return hipGetLastError();
}

template <int KCAP>
static hipError_t launch_pq_scan_k(const PqScanArgs& a, size_t lds, hipStream_t s) {
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_pq_scan<KCAP>),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  if (attr != hipSuccess) return attr;
  hipLaunchKernelGGL(k_pq_scan<KCAP>, dim3((unsigned)a.n_slots), dim3(512), lds, s, a);
  return hipGetLastError();
}

hipError_t launch_pq_scan(const PqScanArgs& a, int kcap, hipStream_t s) {
  if (a.n_slots <= 0) return hipSuccess;
  if (a.n_slots > 0x7FFFFFFF) return hipErrorInvalidValue;
  const size_t lds = pq_scan_lds_bytes(a.rot_dim_pad, a.pq_dim, kcap);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  switch (kcap) {
    case 1: return launch_pq_scan_k<1>(a, lds, s);
    case 4: return launch_pq_scan_k<4>(a, lds, s);
    case 8: return launch_pq_scan_k<8>(a, lds, s);
    case 12: return launch_pq_scan_k<12>(a, lds, s);
    case 16: return launch_pq_scan_k<16>(a, lds, s);
    case 32: return launch_pq_scan_k<32>(a, lds, s);
    case 64: return launch_pq_scan_k<64>(a, lds, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace mivs
