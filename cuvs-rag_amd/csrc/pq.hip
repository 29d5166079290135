// IVF-PQ kernels: residual extraction for codebook training, encoding
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
constexpr int kPqTileQ = 16;         // queries per K9b work item
constexpr int kPqChunkRows = 512;    // rows per K9b work item (one per thread)
constexpr int kPqMaxChunks = 8;      // K9 register path: pq_dim <= 128 (8 x 16 codes per row)

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

// The search LUT (oracle orc_pq_l2_lut / orc_pq_ip). L2: the expanded form ||r||^2 + ||b||^2 - 2 r.b as one
// chain -- acc = rn + bn, then fmaf(r_i, -2 b_i, acc), dims ascending (r = q - c_l; rn = the fmaf chain of
// r_i r_i, bn = the codebook entry's, precomputed in book_norms) -- which K9r runs on MFMA. IP: the chain of
// q_i b_i from 0, negated by pq_lut_entry.
__device__ __forceinline__ float pq_lut_term(bool ip, float r, float b, float acc) {
  return ip ? fmaf(r, b, acc) : fmaf(r, -2.0f * b, acc);
}

// the chain's start for the entry (j, c): L2 rn_j + bn_jc, IP 0
__device__ __forceinline__ float pq_lut_start(bool ip, const float* __restrict__ r, int pl, float bn) {
  if (ip) return 0.0f;
  float rn = 0.0f;
  for (int i = 0; i < pl; ++i) rn = fmaf(r[i], r[i], rn);
  return rn + bn;
}

// the entry: L2 acc; IP -acc, plus the probe's coarse key -(q . c_l) in subspace 0
__device__ __forceinline__ float pq_lut_entry(bool ip, float acc, bool j0, float base0) {
  if (!ip) return acc;
  const float v = -acc;
  return j0 ? v + base0 : v;
}

// Inner product (a.ip): the LUT is LUT_j[c] = -(q_j . B_j[c]) (the fmaf chain of the dims, negated) and
// the coarse term -(q . c_l) -- the probe's coarse key, bit-equal to the oracle's -orc_dot -- is added to
// subspace 0's row, so a row's key is the same j-ordered sum from 0 as for L2. This finds the probe's
// coarse distance (q . c_l, K3's output for IP) by its list id among the query's probes.
__device__ __forceinline__ float pq_ip_base(const PqScanArgs& a, int64_t q, int l) {
  const int lane = threadIdx.x & 63;
  for (int p0 = 0; p0 < a.n_probes; p0 += 64) {
    const int p = p0 + lane;
    const uint64_t m = __ballot(p < a.n_probes && a.probes[q * a.n_probes + p] == l);
    if (m) return -a.probes_d[q * a.n_probes + p0 + __builtin_ctzll(m)];
  }
  return 0.0f;  // (unreachable: l is one of the query's probes)
}

// the slot's output distance: the key (L2) or the inner product (IP, -key); missing ranks +inf / -inf
__device__ __forceinline__ float pq_out(const PqScanArgs& a, bool valid, float key) {
  return valid ? (a.ip ? -key : key) : (a.ip ? -INFINITY : INFINITY);
}

// K9: one workgroup per (query, probe) slot. LDS: [qres d_pad][LUT pq_dim x 256 | merge area].
//   1. residual q - c_l -> LDS;  2. LUT[j][c] = ||res_j - B_j[c]||^2 -> LDS;
//   3. each thread scans rows tid, tid + NT, ... of the list: dist = sum_j LUT[j][code_j],
//      register top-KCAP by (dist, row position);
//   4. the NT lane lists -> LDS; wave w merges its 64 lists (64-lane min-reduction per rank),
//      then wave 0 merges the NT/64 wave lists; the slot's top-k (dist, id) -> out.
// KCAP = 0 (DUMP, k > 64): every row's key -> out_d[slot][dump_rows], (first row position, rows) ->
// slot_info[slot]; K8 selects per query (as the IVF-Flat DUMP scan).
template <int KCAP, int NT>
__global__ __launch_bounds__(NT) void k_pq_scan(PqScanArgs a) {
  constexpr bool DUMP = KCAP == 0;
  constexpr int KR = DUMP ? 1 : KCAP;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* s_res = reinterpret_cast<float*>(smem);                 // [rot_dim]
  float* lut = s_res + a.rot_dim_pad;                            // [pq_dim][256]
  float* mkey = lut;                                             // merge area (after the scan)
  int* mpos = reinterpret_cast<int*>(mkey + NT * KR);
  float* wkey = mkey + 2 * NT * KR;                              // [NT/64][k] wave results
  int* wpos = reinterpret_cast<int*>(wkey + (NT / 64) * KR);

  int64_t slot, q;
  int l;
  if (a.ent_q) {
    // list-sorted entries, XCD-aware: the workgroups of XCD x = b % 8 take the x-th contiguous range in
    // order, so the ~m_l queries probing list l run together on one XCD and share its codes in L2
    const int64_t nb = gridDim.x, b = blockIdx.x, x = b & 7;
    int64_t e = b >> 3;
    for (int y = 0; y < x; ++y) e += (nb - y + 7) >> 3;
    if (e >= a.ent_off[a.n_lists]) return;
    int lo = 0, hi = a.n_lists - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (a.ent_off[mid] <= e) lo = mid; else hi = mid - 1;
    }
    l = lo;
    if (a.list_goff[l + 1] == a.list_goff[l]) return;  // an empty list owns no output slot
    q = a.ent_q[e];
    slot = a.ent_slot[e];
  } else {
    slot = blockIdx.x;  // = q * n_probes + probe
    q = slot / a.n_probes;
    l = (int)a.probes[slot];
  }
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  if (l < 0) {  // no probe (degenerate query): empty slot
    if constexpr (DUMP) {
      if (tid == 0) { a.slot_info[2 * slot] = 0; a.slot_info[2 * slot + 1] = 0; }
      return;
    }
    for (int t = tid; t < a.k; t += NT) {
      a.out_d[slot * a.k + t] = pq_out(a, false, 0.0f);
      a.out_i[slot * a.k + t] = -1;
    }
    return;
  }
  const int pl = a.pq_len;
  for (int i = tid; i < a.rot_dim_pad; i += NT)
    s_res[i] = i < a.d ? (a.ip ? a.queries[q * a.d + i] : a.queries[q * a.d + i] - a.cents[(int64_t)l * a.d + i]) : 0.0f;
  const float base0 = a.ip ? pq_ip_base(a, q, l) : 0.0f;
  __syncthreads();
  const int nlut = a.flags & 1 ? 0 : a.pq_dim * kPqCodes;
  if ((pl & 3) == 0 && pl <= 16) {
    // 4 entries per thread in flight: their codebook rows (pl/4 float4 each) are all requested
    // before the first FMA, so the L2 latency is paid once per 4 entries, not once per entry
    const int nv = pl >> 2;
    for (int base = tid; base < nlut; base += 4 * NT) {
      float4 bv[4][4];
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int e = base + v * NT;
#pragma unroll
        for (int c4 = 0; c4 < 4; ++c4)
          if (c4 < nv && e < nlut) bv[v][c4] = *reinterpret_cast<const float4*>(a.books + (int64_t)e * pl + 4 * c4);
      }
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int e = base + v * NT;
        if (e >= nlut) break;
        const float* r = s_res + (e >> 8) * pl;
        float acc = pq_lut_start(a.ip, r, pl, a.book_norms[e]);
#pragma unroll
        for (int c4 = 0; c4 < 4; ++c4) {
          if (c4 < nv) {
            const float b4[4] = {bv[v][c4].x, bv[v][c4].y, bv[v][c4].z, bv[v][c4].w};
#pragma unroll
            for (int u = 0; u < 4; ++u) acc = pq_lut_term(a.ip, r[4 * c4 + u], b4[u], acc);
          }
        }
        lut[e] = pq_lut_entry(a.ip, acc, e < kPqCodes, base0);
      }
    }
  } else {
    for (int e = tid; e < nlut; e += NT) {
      const int j = e >> 8;
      const float* b = a.books + (int64_t)e * pl;
      const float* r = s_res + j * pl;
      float acc = pq_lut_start(a.ip, r, pl, a.book_norms[e]);
      for (int i = 0; i < pl; ++i) acc = pq_lut_term(a.ip, r[i], b[i], acc);
      lut[e] = pq_lut_entry(a.ip, acc, e < kPqCodes, base0);
    }
  }
  __syncthreads();

  float lk[KR];
  int lp[KR];
#pragma unroll
  for (int t = 0; t < KR; ++t) { lk[t] = INFINITY; lp[t] = INT_MAX; }
  const int64_t r0 = a.list_off[l], nrows = a.flags & 2 ? 0 : a.list_off[l + 1] - r0;
  const int64_t g0 = a.list_goff[l];
  const int nchunk = a.pq_dim_pad >> 4;
  auto row_codes = [&](int64_t r) {
    return a.codes + (g0 + r / kGroupRows) * (int64_t)kGroupRows * a.pq_dim_pad + (r % kGroupRows) * 16;
  };
  if (nchunk <= kPqMaxChunks) {
    // all code chunks of the NEXT row are requested before the current row's LUT lookups
    uint4 cur[kPqMaxChunks], nxt[kPqMaxChunks];
    auto load_row = [&](int64_t r, uint4 (&w)[kPqMaxChunks]) {
      const uint8_t* cg = row_codes(r < nrows ? r : 0);
#pragma unroll
      for (int ch = 0; ch < kPqMaxChunks; ++ch)
        if (ch < nchunk) w[ch] = *reinterpret_cast<const uint4*>(cg + (int64_t)ch * (kGroupRows * 16));
    };
    if (tid < nrows) load_row(tid, cur);
    for (int64_t r = tid; r < nrows; r += NT) {
      if (r + NT < nrows) load_row(r + NT, nxt);
      float dist = 0.0f;
#pragma unroll
      for (int ch = 0; ch < kPqMaxChunks; ++ch) {
        if (ch < nchunk) {
          const uint32_t wv[4] = {cur[ch].x, cur[ch].y, cur[ch].z, cur[ch].w};
#pragma unroll
          for (int b = 0; b < 16; ++b) {
            const int j = ch * 16 + b;
            if (j < a.pq_dim) dist = dist + lut[(j << 8) + ((wv[b >> 2] >> (8 * (b & 3))) & 0xFF)];
          }
        }
      }
      if constexpr (DUMP) a.out_d[slot * a.dump_rows + r] = dist;
      else if (dist < lk[KCAP - 1]) pq_insert<KCAP>(lk, lp, dist, (int)r);
#pragma unroll
      for (int ch = 0; ch < kPqMaxChunks; ++ch) cur[ch] = nxt[ch];
    }
  } else {
    for (int64_t r = tid; r < nrows; r += NT) {
      const uint8_t* cg = row_codes(r);
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
      if constexpr (DUMP) a.out_d[slot * a.dump_rows + r] = dist;
      else if (dist < lk[KCAP - 1]) pq_insert<KCAP>(lk, lp, dist, (int)r);
    }
  }
  if constexpr (DUMP) {
    if (tid == 0) { a.slot_info[2 * slot] = g0 * kGroupRows; a.slot_info[2 * slot + 1] = nrows; }
    return;
  } else {
  if (a.flags & 4) {  // timing experiment: no merge, one store keeps the scan alive
    if (lk[0] < -1.0f) a.out_d[slot * a.k] = lk[0] + (float)lp[0];
    return;
  }
  __syncthreads();  // LUT dead: the merge area aliases it
  // lane lists transposed ([rank][thread]): the stores and every head read are conflict-free
#pragma unroll
  for (int t = 0; t < KCAP; ++t) {
    mkey[t * NT + tid] = lk[t];
    mpos[t * NT + tid] = lp[t];
  }
  __syncthreads();
  // stage 1: wave w merges lane lists w*64 .. w*64+63
  {
    const float* myk = mkey + tid;
    const int* myp = mpos + tid;
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
        hk = head < KCAP ? myk[head * NT] : INFINITY;
        hp = head < KCAP ? myp[head * NT] : INT_MAX;
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
        a.out_d[slot * a.k + t] = pq_out(a, valid, bk);
        a.out_i[slot * a.k + t] = valid ? a.row_ids[g0 * kGroupRows + bp] : (int64_t)-1;
      }
      if (src && hk == bk && hp == bp && head < a.k) {
        ++head;
        hk = head < a.k ? myk[head] : INFINITY;
        hp = head < a.k ? myp[head] : INT_MAX;
      }
    }
  }
  }  // (not DUMP)
}

// LUT entries e < nlut (subspace e >> 8, code e & 255) of a pq_len = 4 * PL4 codebook slice: each
// thread keeps V = 8 / PL4 entries' codebook rows (32 floats) in flight before the first FMA; the
// fmaf chain of K9 / the oracle
template <int PL4, int NT>
__device__ __forceinline__ void pq_lut_build(const float* __restrict__ books, const float* __restrict__ bnorms,
                                             const float* res, int nlut, int tid, float* lut, bool ip, bool with_base,
                                             float base0) {
  constexpr int pl = 4 * PL4, V = PL4 >= 4 ? 2 : 8 / PL4;
  for (int base = tid; base < nlut; base += V * NT) {
    float4 bv[V][PL4];
#pragma unroll
    for (int v = 0; v < V; ++v) {
      const int e = base + v * NT < nlut ? base + v * NT : base;
#pragma unroll
      for (int c4 = 0; c4 < PL4; ++c4) bv[v][c4] = *reinterpret_cast<const float4*>(books + (int64_t)e * pl + 4 * c4);
    }
#pragma unroll
    for (int v = 0; v < V; ++v) {
      const int e = base + v * NT;
      if (e >= nlut) break;
      const float* r = res + (e >> 8) * pl;
      float acc = pq_lut_start(ip, r, pl, bnorms[e]);
#pragma unroll
      for (int c4 = 0; c4 < PL4; ++c4) {
        const float b4[4] = {bv[v][c4].x, bv[v][c4].y, bv[v][c4].z, bv[v][c4].w};
#pragma unroll
        for (int u = 0; u < 4; ++u) acc = pq_lut_term(ip, r[4 * c4 + u], b4[u], acc);
      }
      lut[e] = pq_lut_entry(ip, acc, with_base && e < kPqCodes, base0);
    }
  }
}

// K9s: K9 with the LUT built and consumed in two halves of the subspaces (j < ph, then j >= ph), so a
// workgroup (4 waves) needs ph x 256 x 4 B of LDS (48 KiB at pq_dim 96) instead of the whole LUT and
// three workgroups share a CU: one's LUT build, barrier waits and merge overlap the others' scans. Each
// thread keeps the partial sums of its rows (<= 16 per 4096-row block) in registers across the two
// halves, so every row's sum still runs j = 0, 1, ..., pq_dim-1 from 0 (the oracle's order); a list
// longer than 4096 rows is scanned block by block (the LUT halves rebuilt per block). The lane lists
// merge in registers (per wave, k rounds of a 64-lane min), then wave 0 merges the 4 wave lists.
template <int KCAP>
__global__ __launch_bounds__(256) void k_pq_scan_split(PqScanArgs a) {
  constexpr int NT = 256, NW = NT / 64, RM = 16;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int ph = a.pq_half;
  float* s_res = reinterpret_cast<float*>(smem);  // [rot_dim_pad]
  float* lut = s_res + a.rot_dim_pad;             // [ph][256]
  float* wkey = lut + ph * kPqCodes;              // [NW][KCAP]
  int* wpos = reinterpret_cast<int*>(wkey + NW * KCAP);

  int64_t slot, q;
  int l;
  if (a.ent_q) {
    const int64_t nb = gridDim.x, b = blockIdx.x, x = b & 7;
    int64_t e = b >> 3;
    for (int y = 0; y < x; ++y) e += (nb - y + 7) >> 3;
    if (e >= a.ent_off[a.n_lists]) return;
    int lo = 0, hi = a.n_lists - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (a.ent_off[mid] <= e) lo = mid; else hi = mid - 1;
    }
    l = lo;
    if (a.list_goff[l + 1] == a.list_goff[l]) return;  // an empty list owns no output slot
    q = a.ent_q[e];
    slot = a.ent_slot[e];
  } else {
    slot = blockIdx.x;
    q = slot / a.n_probes;
    l = (int)a.probes[slot];
  }
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  if (l < 0) {
    for (int t = tid; t < a.k; t += NT) {
      a.out_d[slot * a.k + t] = pq_out(a, false, 0.0f);
      a.out_i[slot * a.k + t] = -1;
    }
    return;
  }
  const int pl = a.pq_len;
  for (int i = tid; i < a.rot_dim_pad; i += NT)
    s_res[i] = i < a.d ? (a.ip ? a.queries[q * a.d + i] : a.queries[q * a.d + i] - a.cents[(int64_t)l * a.d + i]) : 0.0f;
  const float base0 = a.ip ? pq_ip_base(a, q, l) : 0.0f;

  float lk[KCAP];
  int lp[KCAP];
#pragma unroll
  for (int t = 0; t < KCAP; ++t) { lk[t] = INFINITY; lp[t] = INT_MAX; }
  const int64_t nrows = a.list_off[l + 1] - a.list_off[l];
  const int64_t g0 = a.list_goff[l];
  auto row_codes = [&](int64_t r) {
    return a.codes + (g0 + r / kGroupRows) * (int64_t)kGroupRows * a.pq_dim_pad + (r % kGroupRows) * 16;
  };
  for (int64_t rb = 0; rb < nrows; rb += (int64_t)NT * RM) {
    float ps[RM];
#pragma unroll
    for (int i = 0; i < RM; ++i) ps[i] = 0.0f;
    for (int h = 0; h < 2; ++h) {
      const int j0 = h * ph, j1 = j0 + ph < a.pq_dim ? j0 + ph : a.pq_dim;
      if (j0 >= j1) break;
      __syncthreads();  // s_res is written / the previous half's scan is done with the LUT
      // LUT[j - j0][c] = ||res_j - B_j[c]||^2 for j in [j0, j1): the K9 fmaf chain, entries 4 at a time
      const int nlut = (j1 - j0) * kPqCodes;
      const float* books = a.books + (int64_t)j0 * kPqCodes * pl;
      const float* bnorms = a.book_norms + (int64_t)j0 * kPqCodes;
      const float* res = s_res + j0 * pl;
      switch (pl >> 2) {
        case 1: pq_lut_build<1, NT>(books, bnorms, res, nlut, tid, lut, a.ip, h == 0, base0); break;
        case 2: pq_lut_build<2, NT>(books, bnorms, res, nlut, tid, lut, a.ip, h == 0, base0); break;
        case 3: pq_lut_build<3, NT>(books, bnorms, res, nlut, tid, lut, a.ip, h == 0, base0); break;
        default: pq_lut_build<4, NT>(books, bnorms, res, nlut, tid, lut, a.ip, h == 0, base0); break;
      }
      __syncthreads();
      // this half's code chunks of each of my rows (<= 4 x 16 codes), the next row's requested first
      const int c0 = j0 >> 4, nch = ((j1 + 15) >> 4) - c0;
      uint4 cur[4], nxt[4];
      auto load_row = [&](int64_t r, uint4 (&w)[4]) {
        const uint8_t* cg = row_codes(r < nrows ? r : 0);
#pragma unroll
        for (int ch = 0; ch < 4; ++ch)
          if (ch < nch) w[ch] = *reinterpret_cast<const uint4*>(cg + (int64_t)(c0 + ch) * (kGroupRows * 16));
      };
      load_row(rb + tid, cur);
      // one row per iteration (not unrolled: the register budget is three workgroups per CU); the
      // partial sums rotate through ps so that ps[0] is always the current row's
#pragma unroll 1
      for (int i = 0; i < RM; ++i) {
        const int64_t r = rb + tid + (int64_t)i * NT;
        const bool more = i + 1 < RM && r + NT < nrows;
        if (more) load_row(r + NT, nxt);
        float dist = ps[0];
        if (r < nrows) {
#pragma unroll
          for (int ch = 0; ch < 4; ++ch) {
            if (ch < nch) {
              const uint32_t wv[4] = {cur[ch].x, cur[ch].y, cur[ch].z, cur[ch].w};
              const float* lj = lut + (ch << 12);  // subspace (c0 + ch) * 16 - j0 = ch * 16
              const int jn = j1 - j0 - ch * 16;    // valid subspaces of this chunk (16 unless the last)
#pragma unroll
              for (int b = 0; b < 16; ++b)
                if (b < jn) dist = dist + lj[(b << 8) + ((wv[b >> 2] >> (8 * (b & 3))) & 0xFF)];
              __builtin_amdgcn_sched_barrier(0);  // one chunk's 16 lookups in flight: bounds the VGPRs
            }
          }
        }
#pragma unroll
        for (int t = 0; t + 1 < RM; ++t) ps[t] = ps[t + 1];
        ps[RM - 1] = dist;
        if (more) {
#pragma unroll
          for (int ch = 0; ch < 4; ++ch) cur[ch] = nxt[ch];
        }
      }
    }
#pragma unroll
    for (int i = 0; i < RM; ++i) {
      const int64_t r = rb + tid + (int64_t)i * NT;
      if (r < nrows && ps[i] < lk[KCAP - 1]) pq_insert<KCAP>(lk, lp, ps[i], (int)r);
    }
  }
  // stage 1 (registers): per wave, k rounds of the 64-lane (dist, row) minimum; the winner lane drops
  // its head by shifting its sorted list down (rows are unique, so one lane wins; exhausted lanes
  // hold (+inf, INT_MAX) and shifting those changes nothing)
  for (int t = 0; t < a.k; ++t) {
    float bk = lk[0];
    int bp = lp[0];
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      const float ok = __shfl_xor(bk, off);
      const int op = __shfl_xor(bp, off);
      if (ok < bk || (ok == bk && op < bp)) { bk = ok; bp = op; }
    }
    if (lane == 0) { wkey[wave * KCAP + t] = bk; wpos[wave * KCAP + t] = bp; }
    if (lk[0] == bk && lp[0] == bp) {
#pragma unroll
      for (int i = 0; i + 1 < KCAP; ++i) { lk[i] = lk[i + 1]; lp[i] = lp[i + 1]; }
      lk[KCAP - 1] = INFINITY;
      lp[KCAP - 1] = INT_MAX;
    }
  }
  __syncthreads();
  // stage 2: wave 0, lanes 0..NW-1 hold the wave lists
  if (wave == 0) {
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
        a.out_d[slot * a.k + t] = pq_out(a, valid, bk);
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

// K9b: work item = (list l, tile of <= 16 queries probing l, chunk of 16 groups = 512 rows), dequeued
// like K3 from the IVF probe map. Subspace-outer loop: per subspace j the codebook B_j (256 x pl)
// and the tile's 16 LUT rows LUT_j[q][c] = ||(q - c_l)_j - B_j[c]||^2 are built in LDS once and
// every thread (one row of the chunk) adds LUT_j[q][code_j(row)] for the 16 queries: each
// codebook byte crosses L2 once per work item instead of once per (query, probe), and the sums
// run in the oracle's order (j ascending). Then per query a wave picks the chunk's top-k.
template <int KCAP>
__global__ __launch_bounds__(512) void k_pq_scan_tiled(PqTileArgs a) {
  constexpr int NT = 512, TQ = kPqTileQ, ROWS = kPqChunkRows;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int64_t* s_q = reinterpret_cast<int64_t*>(smem);          // [TQ]
  int64_t* s_slot = s_q + TQ;                               // [TQ]
  int* s_misc = reinterpret_cast<int*>(s_slot + TQ);        // [4]
  float* s_cb = reinterpret_cast<float*>(smem + 256 + 16);  // [2][256 * pl]   codebook, double-buffered
  float* s_lut = s_cb + 2 * 256 * a.pq_len;                 // [2][TQ][256]
  float* s_rj = s_lut + 2 * TQ * 256;                       // [2][TQ][pl]    query residuals of subspace j
  float* s_dist = s_cb;                                     // [TQ][ROWS], after the subspace loop
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int pl = a.pq_len;
  const int total = a.work_off[a.n_lists];
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
    const int tiles = (m + TQ - 1) / TQ;
    const int local = w - a.work_off[l];
    const int chunk = local / tiles;
    const int tile = local - chunk * tiles;
    const int e0 = a.bucket_off[l] + tile * TQ;
    const int nqt = m - tile * TQ < TQ ? m - tile * TQ : TQ;
    const int64_t nrows = a.list_off[l + 1] - a.list_off[l];
    const int64_t r0 = (int64_t)chunk * ROWS;                      // first row of the chunk in the list
    const int nr = (int)(nrows - r0 < ROWS ? nrows - r0 : ROWS);   // valid rows of the chunk
    const int64_t g0 = a.list_goff[l];
    if (tid < TQ) {
      if (tid < nqt) {
        s_q[tid] = a.bucket_q[e0 + tid];
        s_slot[tid] = a.bucket_slot[e0 + tid] + chunk;
      } else {
        s_q[tid] = -1;
        s_slot[tid] = -1;
      }
    }
    __syncthreads();
    // this thread's row and its code address
    const int row = tid;
    const bool rvalid = row < nr;
    const int64_t rpos = r0 + (rvalid ? row : 0);
    const uint8_t* cg = a.codes + (g0 + rpos / kGroupRows) * (int64_t)kGroupRows * a.pq_dim_pad +
                        (rpos % kGroupRows) * 16;
    float acc[TQ];
#pragma unroll
    for (int t = 0; t < TQ; ++t) acc[t] = 0.0f;
    // stage subspace j: codebook B_j and the tile's residual sub-vectors (q - c_l)_j (dims >= d: 0)
    auto load_stage = [&](int j, int buf) {
      const float* src = a.books + (int64_t)j * 256 * pl;
      float* dst = s_cb + buf * 256 * pl;
      for (int i = tid; i < 256 * pl; i += NT) dst[i] = src[i];
      for (int i = tid; i < TQ * pl; i += NT) {
        const int t = i / pl, k = j * pl + (i - t * pl);
        const int64_t q = s_q[t];
        s_rj[buf * TQ * pl + i] = (q >= 0 && k < a.d) ? a.queries[q * a.d + k] - a.cents[(int64_t)l * a.d + k] : 0.0f;
      }
    };
    load_stage(0, 0);
    __syncthreads();
    uint4 cw = make_uint4(0, 0, 0, 0);
    for (int j = 0; j < a.pq_dim; ++j) {
      const int buf = j & 1;
      // LUT_j for the tile: entry e = (t, c), t < TQ, c < 256 -> 4096 entries, 8 per thread
      const float* cb = s_cb + buf * 256 * pl;
      float* lut = s_lut + buf * TQ * 256;
      for (int e = tid; e < TQ * 256; e += NT) {
        const int t = e >> 8, c = e & 255;
        const float* r = s_rj + buf * TQ * pl + t * pl;
        const float* b = cb + c * pl;
        float v = pq_lut_start(false, r, pl, a.book_norms[j * 256 + c]);
        for (int i = 0; i < pl; ++i) v = pq_lut_term(false, r[i], b[i], v);
        lut[e] = v;
      }
      if (j + 1 < a.pq_dim) load_stage(j + 1, buf ^ 1);
      if ((j & 15) == 0) cw = *reinterpret_cast<const uint4*>(cg + (int64_t)(j >> 4) * (kGroupRows * 16));
      __syncthreads();
      const int jb = j & 15;
      const uint32_t word = jb < 4 ? cw.x : (jb < 8 ? cw.y : (jb < 12 ? cw.z : cw.w));
      const int code = (word >> (8 * (jb & 3))) & 0xFF;
#pragma unroll
      for (int t = 0; t < TQ; ++t) acc[t] = acc[t] + lut[t * 256 + code];
    }
    // distances of the chunk -> LDS [TQ][ROWS] (+inf on pad rows; overlays the dead codebook / LUT
    // buffers), then per query a wave's top-k
    __syncthreads();
#pragma unroll
    for (int t = 0; t < TQ; ++t) s_dist[t * ROWS + row] = rvalid ? acc[t] : INFINITY;
    __syncthreads();
    for (int t = wave; t < TQ; t += NT / 64) {
      const int64_t slot = s_slot[t];
      if (slot < 0) continue;
      float lk[KCAP];
      int lp[KCAP];
#pragma unroll
      for (int i = 0; i < KCAP; ++i) { lk[i] = INFINITY; lp[i] = INT_MAX; }
      for (int r = lane; r < ROWS; r += 64) {
        const float v = s_dist[t * ROWS + r];
        if (v < lk[KCAP - 1]) pq_insert<KCAP>(lk, lp, v, r);
      }
      // 64-lane merge: per rank the (dist, row) minimum; the winner lane advances its head
      float hk = lk[0];
      int hp = lp[0];
      for (int rk = 0; rk < a.k; ++rk) {
        float bk = hk;
        int bp = hp;
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
          const float ok = __shfl_xor(bk, off);
          const int op = __shfl_xor(bp, off);
          if (ok < bk || (ok == bk && op < bp)) { bk = ok; bp = op; }
        }
        if (lane == 0) {
          const bool valid = bp != INT_MAX;
          a.out_d[slot * a.k + rk] = valid ? bk : INFINITY;
          a.out_i[slot * a.k + rk] = valid ? a.row_ids[g0 * kGroupRows + r0 + bp] : (int64_t)-1;
        }
        if (hk == bk && hp == bp) {
          // registers cannot be indexed dynamically: shift the list down by one instead
#pragma unroll
          for (int i = 0; i + 1 < KCAP; ++i) { lk[i] = lk[i + 1]; lp[i] = lp[i + 1]; }
          lk[KCAP - 1] = INFINITY;
          lp[KCAP - 1] = INT_MAX;
          hk = lk[0];
          hp = lp[0];
        }
      }
    }
    __syncthreads();
  }
}

// K9r: the IVF-PQ scan with the QUERIES of a list tiled and the ROWS register-stationary.
//
// K9/K9s build one query's whole LUT per (query, probe) and gather LUT_j[code] with ds_read_b32: 64
// random 4-B addresses per wave-instruction, ~3.5-way bank-conflicted, one useful float per lane.
// K9r turns the gather around. A work item is (list l, tile of <= 16 queries probing l, chunk of
// kRtRows rows); per subspace j the tile's LUT_j is stored code-major -- row c holds LUT_j[c] of the 16
// queries (64 B, padded to 80 B so that the 16-lane groups of ds_read_b128 spread over the 64 banks)
// -- and each thread adds, for each of its 8 rows, the 16 queries' entries of the row's code: four
// ds_read_b128 per (row, subspace), 16 useful floats per lane per 4 reads. The sums of 8 rows x 16
// queries stay in registers across all subspaces, each row's sum running j = 0, 1, ... from 0 as in
// K9 and the oracle. LUT_{j+1} is built (the K9 fmaf chain, thread = (code, 8 queries), its codebook
// row prefetched from L2 a subspace ahead) into the other half of a double buffer while LUT_j is read.
//
// Output (CQ > 0, k <= 64): per (query, chunk) slot the exact top-k by (key, row) for K7: bound_q =
// the k-th smallest of the 512 per-thread minima (>= k distinct rows lie at or below it, so every row
// of the slot's top-k does too); rows <= bound_q -> LDS (at most 8 (k - 1) below it plus ties), and a
// wave picks k by rounds of 64-lane minima. A slot whose list overflows CQ (many tied keys) is finished
// by block-wide rounds over the registers instead. 64 < k <= kRtCandMax (slot_cap > 0): the slot takes the rows
// at or below bound_q as they are (a superset of its top-k), or
// its exact top-k when they exceed slot_cap, and K8 ranks a query's slots -- the refine's 12 x k candidates had
// taken the DUMP path, 1.9 GB of keys written and read back per 10k queries. CQ == 0 (DUMP, k > kRtCandMax):
// every row's key -> out_d[slot][kRtRows] and (first row position, rows) -> slot_info for K8.
__device__ __forceinline__ uint32_t rt_ord(float f) {  // orderable bits, -0 and +0 equal
  const uint32_t u = __float_as_uint(f == 0.0f ? 0.0f : f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__device__ __forceinline__ bool rt_less(float ka, int ra, float kb, int rb) {
  return ka < kb || (ka == kb && ra < rb);
}

typedef uint32_t pq_u32x4 __attribute__((ext_vector_type(4)));

// acc + (float)(half `hi` of w) in one VALU op: v_fma_mix_f32 with the f16 operand times 1.0 is exact, so its one
// rounding is the fp32 add's (the compiler folds fmaf(h, 1, acc) to a cvt + add, two ops per entry)
__device__ __forceinline__ float rt_add_f16(float acc, uint32_t w, int hi) {
  if (hi)
    asm("v_fma_mix_f32 %0, %1, 1.0, %0 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "+v"(acc) : "v"(w));
  else
    asm("v_fma_mix_f32 %0, %1, 1.0, %0 op_sel_hi:[1,0,0]" : "+v"(acc) : "v"(w));
  return acc;
}

// H16 (cuvs SearchParams.lut_dtype = float16, L2): each LUT entry is rounded to fp16 when it is stored (RNE, as
// oracle orc_round_f16) and a code row is 16 halves padded to 48 B (its 16-lane groups start at quad 3c mod 16: a
// permutation over c mod 16, like the 80-B fp32 rows' 5c), so a (row, subspace) takes two ds_read_b128 instead of
// four; the row sums stay fp32 in the same order.
template <int PL4, int CQ, bool H16 = false>
__global__ __launch_bounds__(kRtThreads) void k_pq_scan_rt(PqTileArgs a) {
  constexpr int NT = kRtThreads, TQ = kRtQ, RPT = kRtRpt, R = kRtRows, PL = 4 * PL4;
  constexpr int LS = H16 ? 12 : 20;  // code row stride in 4-B words (fp16: 24 halves = 48 B; fp32: 20 floats)
  constexpr bool DUMP = CQ == 0;
  const int SC = a.slot_cap;         // > 0: candidate-superset slots of SC entries (k > kMaxK)
  const int ST = SC > 0 ? SC : a.k;  // entries per output slot
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int64_t* s_q = reinterpret_cast<int64_t*>(smem);        // [TQ] query (-1: no query)
  int64_t* s_slot = s_q + TQ;                             // [TQ] output slot
  int* s_misc = reinterpret_cast<int*>(s_slot + TQ);      // [16]
  int* s_cnt = s_misc + 16;                               // [TQ] candidates <= bound
  uint32_t* s_bound = reinterpret_cast<uint32_t*>(s_cnt + TQ);  // [TQ]
  float* s_base = reinterpret_cast<float*>(s_bound + TQ);       // [TQ] IP: the probe's coarse key
  const int rdp = a.rot_dim_pad;
  float* s_res = reinterpret_cast<float*>(smem + 512);    // [TQ][rdp] residuals (IP: the queries)
  float* s_lut = s_res + TQ * rdp;                        // [4][256][LS]: two subspace pairs
  float* s_rn = s_lut + 4 * kPqCodes * LS;                // [pq_dim][TQ] L2: ||r_j||^2 of the tile's queries
  // after the subspace loop (aliasing s_res / s_lut)
  uint32_t* s_min = reinterpret_cast<uint32_t*>(smem + 512);   // [TQ][NT]
  float* s_ck = reinterpret_cast<float*>(s_min + TQ * NT);     // [TQ][CQ]
  int* s_cr = reinterpret_cast<int*>(s_ck + TQ * (CQ > 0 ? CQ : 1));
  float* s_wk = reinterpret_cast<float*>(smem + 512);          // slow path: [NT/64] wave minima
  int* s_wr = reinterpret_cast<int*>(s_wk + NT / 64);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // LUT build on v_mfma_f32_16x16x4_f32, whose result is the chain fma(a3,b3, fma(a2,b2, fma(a1,b1, fma(a0,b0,
  // c)))) (tools/mfma_f32_order.hip: every output of 1M random trials): wave w builds codes 32w..32w+31 of LUT_j
  // for the tile as two 16-code blocks. Lane (g = lane >> 4, i = lane & 15) feeds A[i][g] = dim 4s + g of
  // query i's residual and B[g][i] = dim 4s + g of code 32w + 16cb + i (books_mfma: x(-2) for L2, x(-1) for
  // IP), so the pl / 4 MFMAs of a block run the oracle's chain over the dims in ascending order from C =
  // rn_j[query] + bn_j[code] (L2) or 0 (IP). D register r = query 4g + r of code 32w + 16cb + i.
  const int bg = lane >> 4, bi = lane & 15;
  const int total = a.work_off[a.n_lists];
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
    const int tiles = (m + TQ - 1) / TQ;
    const int local = w - a.work_off[l];
    const int chunk = local / tiles;
    const int tile = local - chunk * tiles;
    const int e0 = a.bucket_off[l] + tile * TQ;
    const int nqt = m - tile * TQ < TQ ? m - tile * TQ : TQ;
    const int64_t nrows = a.list_off[l + 1] - a.list_off[l];
    const int64_t r0 = (int64_t)chunk * R;
    const int nr = (int)(nrows - r0 < R ? nrows - r0 : R);
    const int64_t g0 = a.list_goff[l];
    if (tid < TQ) {
      const bool v = tid < nqt;
      s_q[tid] = v ? a.bucket_q[e0 + tid] : -1;
      s_slot[tid] = v ? a.bucket_slot[e0 + tid] + chunk : -1;
      s_cnt[tid] = 0;
      s_base[tid] = 0.0f;
    }
    __syncthreads();
    if (a.ip) {  // the probe's coarse key -(q . c_l), found by list id among the query's probes
      for (int t = wave; t < TQ; t += NT / 64) {
        const int64_t q = s_q[t];
        if (q < 0) continue;
        for (int p0 = 0; p0 < a.n_probes; p0 += 64) {
          const int p = p0 + lane;
          const uint64_t mk = __ballot(p < a.n_probes && a.probes[q * a.n_probes + p] == l);
          if (mk) {
            if (lane == 0) s_base[t] = -a.probes_d[q * a.n_probes + p0 + __builtin_ctzll(mk)];
            break;
          }
        }
      }
    }
    // residuals (IP: the queries) with each subspace's dims in MFMA operand order: dim 4s + g of subspace j
    // at j * PL + g * PL4 + s (dims >= pq_dim * PL, if any, as they are)
    const int rd = a.pq_dim * PL;
    for (int i = tid; i < TQ * rdp; i += NT) {
      const int t = i / rdp, c = i - t * rdp;
      const int64_t q = s_q[t];
      float v = 0.0f;
      if (q >= 0 && c < a.d) v = a.ip ? a.queries[q * a.d + c] : a.queries[q * a.d + c] - a.cents[(int64_t)l * a.d + c];
      const int jj = c / PL, ii = c - jj * PL;
      s_res[t * rdp + (c < rd ? jj * PL + (ii & 3) * PL4 + (ii >> 2) : c)] = v;
    }
    // LUT_j (j < pq_dim) into buffer `buf` (see bg / bi above)
    float bk[2][2][PL4];  // MFMA B operands of the two code blocks of the two subspaces of the next pair
    float bnk[2][2];      // and the codes' norms
    auto load_book = [&](int j, float (&b)[2][PL4], float (&bn)[2]) {
#pragma unroll
      for (int cb = 0; cb < 2; ++cb) {
        const int c = wave * 32 + cb * 16 + bi;
        const float* src = a.books_mfma + ((int64_t)j * kPqCodes + c) * PL + bg * PL4;
#pragma unroll
        for (int u = 0; u < PL4; ++u) b[cb][u] = src[u];
        bn[cb] = a.book_norms[j * kPqCodes + c];
      }
    };
    // LUT_j0 and LUT_j0+1 into slots j0 & 3, (j0 + 1) & 3: the four MFMA chains, then one wait for their results
    auto build2 = [&](int j0, const float (&b)[2][2][PL4], const float (&bn)[2][2]) {
      f32x4 acc[2][2];
#pragma unroll
      for (int sb = 0; sb < 2; ++sb) {
        const int j = j0 + sb;
        float ra[PL4];
        const float* rsrc = s_res + bi * rdp + j * PL + bg * PL4;
#pragma unroll
        for (int u = 0; u < PL4; ++u) ra[u] = rsrc[u];
        float4 rn = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        if (!a.ip) rn = *reinterpret_cast<const float4*>(s_rn + j * TQ + 4 * bg);
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
          if (!a.ip) {
            acc[sb][cb][0] = rn.x + bn[sb][cb]; acc[sb][cb][1] = rn.y + bn[sb][cb];
            acc[sb][cb][2] = rn.z + bn[sb][cb]; acc[sb][cb][3] = rn.w + bn[sb][cb];
          } else {
            acc[sb][cb][0] = 0.0f; acc[sb][cb][1] = 0.0f; acc[sb][cb][2] = 0.0f; acc[sb][cb][3] = 0.0f;
          }
#pragma unroll
          for (int u = 0; u < PL4; ++u)
            acc[sb][cb] = __builtin_amdgcn_mfma_f32_16x16x4f32(ra[u], b[sb][cb][u], acc[sb][cb], 0, 0, 0);
        }
      }
      // the results are read next by LDS stores: the wait states of an XDL result read as LDS data, explicit
      // (the compiler placed a store one instruction after its MFMA: 12 % of the LUT entries were stale). gfx950,
      // v_mfma_f32_16x16x4_f32 (8 passes): 18 wait states between the last MFMA writing a register and an LDS store
      // (ds_write) reading it as data -- s_nop N idles N + 1 cycles, so 8 + 8 + 5 = 21 >= 18 with a margin. Another
      // target or MFMA shape needs its own count: the guard below stops the build, and the K9r-vs-K9s / oracle
      // parity tests (every pq_len K9r serves, tests/test_gpu_parity.py::test_ivf_pq_k9r_mfma_lut_every_pq_len) catch a schedule that moves a store closer.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "K9r's MFMA -> LDS-store wait states are counted for gfx950"
#endif
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 4" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int sb = 0; sb < 2; ++sb) {
        const int j = j0 + sb;
#pragma unroll
        for (int cb = 0; cb < 2; ++cb) {
          f32x4 v = acc[sb][cb];
          if (a.ip && j == 0) {  // the probe's coarse key in subspace 0 (pq_lut_entry)
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = v[r] + s_base[4 * bg + r];
          }
          if constexpr (H16) {
            typedef _Float16 hx4 __attribute__((ext_vector_type(4)));
            const hx4 hv = {(_Float16)v[0], (_Float16)v[1], (_Float16)v[2], (_Float16)v[3]};
            *reinterpret_cast<hx4*>(reinterpret_cast<char*>(s_lut + ((j & 3) * kPqCodes + wave * 32 + cb * 16 + bi) * LS) +
                                     8 * bg) = hv;
          } else {
            *reinterpret_cast<float4*>(s_lut + ((j & 3) * kPqCodes + wave * 32 + cb * 16 + bi) * LS + 4 * bg) =
                make_float4(v[0], v[1], v[2], v[3]);
          }
        }
      }
    };
    load_book(0, bk[0], bnk[0]);
    load_book(1, bk[1], bnk[1]);
    __syncthreads();  // s_res, s_base
    if (!a.ip) {  // rn_j of the tile's queries: the fmaf chain of r_i r_i, dims ascending (pq_lut_start)
      for (int e = tid; e < a.pq_dim * TQ; e += NT) {
        const int j = e / TQ, t = e - j * TQ;
        const float* r = s_res + t * rdp + j * PL;
        float rn = 0.0f;
#pragma unroll
        for (int i = 0; i < PL; ++i) rn = fmaf(r[(i & 3) * PL4 + (i >> 2)], r[(i & 3) * PL4 + (i >> 2)], rn);
        s_rn[e] = rn;
      }
      __syncthreads();
    }
    if (!(a.flags & 1)) build2(0, bk, bnk);

    // my rows: i * NT + tid of the chunk; their codes, 16 subspaces (one uint4) per chunk ch
    float acc[RPT][TQ];
#pragma unroll
    for (int i = 0; i < RPT; ++i)
#pragma unroll
      for (int t = 0; t < TQ; ++t) acc[i][t] = 0.0f;
    // my rows' code offsets from the list's first group (32-bit: a list's codes are < 2 GiB)
    const uint8_t* lcodes = a.codes + g0 * (int64_t)kGroupRows * a.pq_dim_pad;
    int coff[RPT];
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
      const int row = i * NT + tid;
      const int pos = (int)r0 + (row < nr ? row : 0);
      coff[i] = (pos / kGroupRows) * kGroupRows * a.pq_dim_pad + (pos % kGroupRows) * 16;
    }
    // one 4-B code word (4 subspaces) per row at a time, the next word requested a word ahead
    uint32_t cw[RPT], nw[RPT];
    const int nwd = (a.pq_dim + 3) >> 2;
    auto load_word = [&](int wq, uint32_t (&dst)[RPT]) {
      const uint8_t* base = lcodes + (wq >> 2) * (kGroupRows * 16) + (wq & 3) * 4;
#pragma unroll
      for (int i = 0; i < RPT; ++i) dst[i] = *reinterpret_cast<const uint32_t*>(base + coff[i]);
    };
    load_word(0, cw);
    const bool skip_scan = a.flags & 2;
    const int np4 = (nqt + 3) >> 2;  // fp32 LUT: 16-B pieces (4 queries each) of a code row the tile uses
    // row iterations of this wave inside the chunk (wave-uniform)
    const int nvi = nr > wave * 64 ? (nr - wave * 64 + NT - 1) / NT : 0;
    // subspaces in pairs, one barrier per pair: at pair (j, j + 1) the next pair's codebook rows are requested, the
    // pair is scanned, then the next pair's LUTs are built into the other two of four slots (the pair before
    // this one used them, and every wave has passed this pair's barrier, so is done with it)
    for (int wq = 0; wq < nwd; ++wq) {
      if (wq + 1 < nwd) load_word(wq + 1, nw);
#pragma unroll
      for (int b = 0; b < 4; ++b) {  // (pq_dim % 4 == 0: pq_rt_supported)
        const int j = wq * 4 + b;
        if ((b & 1) == 0) {
          __syncthreads();  // LUT_j, LUT_j+1 complete; the slots of LUT_j-2, LUT_j-1 free
          if (j + 2 < a.pq_dim) {
            load_book(j + 2, bk[0], bnk[0]);
            load_book(j + 3, bk[1], bnk[1]);
          }
        }
        const float* lut = s_lut + (j & 3) * (kPqCodes * LS);
        // fp32: only the 16-B pieces of a code row that hold the tile's queries are read (np4 is item-uniform: the
        // branches are scalar; a tile of 12 queries reads 3 of 4). fp16: both pieces always -- skipping the second for
        // tiles of <= 8 queries broke the grouped issue of the RH rows' reads (K9r 7.92 vs 8.14 ms, profiles/r06p_pq_lut16_ab/)
        if constexpr (H16) {  // RH rows' halves in flight (2: 7.97 ms, 4: 7.84 ms at configs[4])
          constexpr int RH = 4;
#pragma unroll
          for (int i0 = 0; i0 < RPT; i0 += RH) {
            if (i0 < nvi && !skip_scan) {
              pq_u32x4 v[RH][2];
#pragma unroll
              for (int r = 0; r < RH; ++r) {
                const pq_u32x4* p = reinterpret_cast<const pq_u32x4*>(lut + ((cw[i0 + r] >> (8 * b)) & 0xFF) * LS);
                v[r][0] = p[0];
                v[r][1] = p[1];
              }
              __builtin_amdgcn_sched_group_barrier(0x100, 2 * RH, 0);  // the LDS reads issue first
#pragma unroll
              for (int r = 0; r < RH; ++r) {
                if (r == 0 || i0 + r < nvi) {
#pragma unroll
                  for (int t = 0; t < 8; ++t) {
                    acc[i0 + r][t] = rt_add_f16(acc[i0 + r][t], v[r][0][t >> 1], t & 1);
                    acc[i0 + r][8 + t] = rt_add_f16(acc[i0 + r][8 + t], v[r][1][t >> 1], t & 1);
                  }
                }
              }
            }
            __builtin_amdgcn_sched_barrier(0);
          }
        } else {
#pragma unroll
          for (int i = 0; i < RPT; ++i) {
            if (i < nvi && !skip_scan) {
              const f32x4* p = reinterpret_cast<const f32x4*>(lut + ((cw[i] >> (8 * b)) & 0xFF) * LS);
              f32x4 v[4] = {p[0], {0.0f, 0.0f, 0.0f, 0.0f}, {0.0f, 0.0f, 0.0f, 0.0f}, {0.0f, 0.0f, 0.0f, 0.0f}};
              if (np4 > 1) v[1] = p[1];  // (one ds_read_b128 each, under a scalar branch)
              if (np4 > 2) v[2] = p[2];
              if (np4 > 3) v[3] = p[3];
#pragma unroll
              for (int u = 0; u < 4; ++u) {
                acc[i][4 * u] += v[u][0]; acc[i][4 * u + 1] += v[u][1];
                acc[i][4 * u + 2] += v[u][2]; acc[i][4 * u + 3] += v[u][3];
              }
            }
            __builtin_amdgcn_sched_barrier(0);  // one row's 16 LUT floats in flight: bounds the VGPRs
          }
        }
        if ((b & 1) == 1 && j + 1 < a.pq_dim && !(a.flags & 1)) build2(j + 1, bk, bnk);
      }
#pragma unroll
      for (int i = 0; i < RPT; ++i) cw[i] = nw[i];
    }
    __syncthreads();  // every wave done with the LUT / residuals (their LDS is reused below)

    if constexpr (DUMP) {
#pragma unroll
      for (int t = 0; t < TQ; ++t) {
        const int64_t slot = s_slot[t];
        if (slot < 0) continue;
#pragma unroll
        for (int i = 0; i < RPT; ++i) {
          const int row = i * NT + tid;
          if (row < nr) a.out_d[slot * R + row] = acc[i][t];
        }
      }
      if (tid < TQ && s_slot[tid] >= 0) {
        a.slot_info[2 * s_slot[tid]] = g0 * kGroupRows + r0;
        a.slot_info[2 * s_slot[tid] + 1] = nr;
      }
    } else {
      // 1. per query the minimum of my rows (query slots past the tile's nqt queries are skipped in 1-3: their sums
      // are not formed, see the scan's piece reads)
#pragma unroll
      for (int t = 0; t < TQ; ++t) {
        if (t < nqt) {  // (item-uniform)
          float mn = INFINITY;
          bool any = false;
#pragma unroll
          for (int i = 0; i < RPT; ++i) {
            if (i * NT + tid < nr) { mn = fminf(mn, acc[i][t]); any = true; }
          }
          s_min[t * NT + tid] = any ? rt_ord(mn) : 0xFFFFFFFFu;
        }
      }
      __syncthreads();
      // 2. bound_q = the k-th smallest of the NT minima (wave w: queries 2w, 2w + 1), bit by bit
      for (int t = wave; t < nqt; t += NT / 64) {
        uint32_t v[NT / 64];
#pragma unroll
        for (int u = 0; u < NT / 64; ++u) v[u] = s_min[t * NT + u * 64 + lane];
        int kk = a.k;
        uint32_t P = 0;
        for (int bit = 31; bit >= 0; --bit) {
          const uint32_t hi_mask = ~((2u << bit) - 1u);  // bits above `bit` (none for bit 31)
          int c0 = 0;
#pragma unroll
          for (int u = 0; u < NT / 64; ++u)
            c0 += __popcll(__ballot((v[u] & hi_mask) == (P & hi_mask) && !((v[u] >> bit) & 1u)));
          if (kk > c0) { kk -= c0; P |= 1u << bit; }
        }
        if (lane == 0) s_bound[t] = P;
      }
      __syncthreads();
      // 3. rows at or below the bound -> the query's candidate list
#pragma unroll
      for (int t = 0; t < TQ; ++t) {
        if (t >= nqt) continue;  // (item-uniform; unrolled, so a predicated body)
        // rt_ord(x) <= bound  <=>  x <= the bound's float (-0 == +0 both ways); all ones: every row
        const uint32_t bnd = s_bound[t];
        const float fb = bnd == 0xFFFFFFFFu ? INFINITY
                                           : __uint_as_float((bnd & 0x80000000u) ? (bnd & 0x7FFFFFFFu) : ~bnd);
#pragma unroll
        for (int i = 0; i < RPT; ++i) {
          const int row = i * NT + tid;
          if (row < nr && acc[i][t] <= fb) {
            const int p = atomicAdd(&s_cnt[t], 1);
            if (p < CQ) { s_ck[t * CQ + p] = acc[i][t]; s_cr[t * CQ + p] = row; }
          }
        }
      }
      __syncthreads();
      // 4. per query (wave w: 2w, 2w + 1) k rounds of the 64-lane (key, row) minimum; candidate-superset slots
      // (slot_cap > 0) take the n <= slot_cap rows at or below the bound as they are, unsorted (K8 ranks them)
      for (int t = wave; t < TQ; t += NT / 64) {
        const int64_t slot = s_slot[t];
        const int n = s_cnt[t];
        if (slot < 0 || n > CQ) continue;
        if (SC > 0 && n <= SC) {
          for (int e = lane; e < SC; e += 64) {
            float o = a.ip ? -INFINITY : INFINITY;
            int64_t id = -1;
            if (e < n) {
              const float x = s_ck[t * CQ + e];
              o = a.ip ? -x : x;
              id = a.row_ids[g0 * kGroupRows + r0 + s_cr[t * CQ + e]];
            }
            a.out_d[slot * SC + e] = o;
            a.out_i[slot * SC + e] = id;
          }
          continue;
        }
        constexpr int PER = CQ / 64;
        float ck[PER];
        int cr[PER];
#pragma unroll
        for (int u = 0; u < PER; ++u) {
          const int e = u * 64 + lane;
          ck[u] = e < n ? s_ck[t * CQ + e] : INFINITY;
          cr[u] = e < n ? s_cr[t * CQ + e] : INT_MAX;
        }
        for (int rk = 0; rk < a.k; ++rk) {
          float bk = ck[0];
          int br = cr[0];
#pragma unroll
          for (int u = 1; u < PER; ++u)
            if (rt_less(ck[u], cr[u], bk, br)) { bk = ck[u]; br = cr[u]; }
#pragma unroll
          for (int off = 32; off >= 1; off >>= 1) {
            const float ok = __shfl_xor(bk, off);
            const int orr = __shfl_xor(br, off);
            if (rt_less(ok, orr, bk, br)) { bk = ok; br = orr; }
          }
          const bool valid = br != INT_MAX;
          if (lane == 0) {
            a.out_d[slot * ST + rk] = valid ? (a.ip ? -bk : bk) : (a.ip ? -INFINITY : INFINITY);
            a.out_i[slot * ST + rk] = valid ? a.row_ids[g0 * kGroupRows + r0 + br] : (int64_t)-1;
          }
#pragma unroll
          for (int u = 0; u < PER; ++u)
            if (ck[u] == bk && cr[u] == br) { ck[u] = INFINITY; cr[u] = INT_MAX; }
        }
        for (int e = a.k + lane; e < SC; e += 64) {  // (superset slot holding its exact top-k: the rest is empty)
          a.out_d[slot * SC + e] = a.ip ? -INFINITY : INFINITY;
          a.out_i[slot * SC + e] = -1;
        }
      }
      // 5. (rare) slots whose candidate list overflowed: block-wide rounds over the registers
      for (int t = 0; t < TQ; ++t) {
        if (s_slot[t] < 0 || s_cnt[t] <= CQ) continue;  // block-uniform
        const int64_t slot = s_slot[t];
        float xs[RPT];  // query t's sums of my rows (selected statically: no dynamic register indexing)
#pragma unroll
        for (int i = 0; i < RPT; ++i) {
          xs[i] = acc[i][0];
#pragma unroll
          for (int u = 1; u < TQ; ++u)
            if (u == t) xs[i] = acc[i][u];
        }
        float lk = -INFINITY;
        int lr = -1;
        for (int rk = 0; rk < a.k; ++rk) {
          float bk = INFINITY;
          int br = INT_MAX;
#pragma unroll
          for (int i = 0; i < RPT; ++i) {
            const int row = i * NT + tid;
            const float x = xs[i];
            if (row < nr && rt_less(lk, lr, x, row) && rt_less(x, row, bk, br)) { bk = x; br = row; }
          }
#pragma unroll
          for (int off = 32; off >= 1; off >>= 1) {
            const float ok = __shfl_xor(bk, off);
            const int orr = __shfl_xor(br, off);
            if (rt_less(ok, orr, bk, br)) { bk = ok; br = orr; }
          }
          __syncthreads();
          if (lane == 0) { s_wk[wave] = bk; s_wr[wave] = br; }
          __syncthreads();
#pragma unroll
          for (int u = 0; u < NT / 64; ++u)
            if (rt_less(s_wk[u], s_wr[u], bk, br)) { bk = s_wk[u]; br = s_wr[u]; }
          const bool valid = br != INT_MAX;
          if (tid == 0) {
            a.out_d[slot * ST + rk] = valid ? (a.ip ? -bk : bk) : (a.ip ? -INFINITY : INFINITY);
            a.out_i[slot * ST + rk] = valid ? a.row_ids[g0 * kGroupRows + r0 + br] : (int64_t)-1;
          }
          lk = bk;
          lr = br;
        }
        for (int e = a.k + tid; e < SC; e += NT) {
          a.out_d[slot * SC + e] = a.ip ? -INFINITY : INFINITY;
          a.out_i[slot * SC + e] = -1;
        }
      }
    }
    __syncthreads();  // s_q / s_slot / s_cnt of the next item
  }
}

inline dim3 gridc(int64_t n, int b) {
  const int64_t g = ceil_div(n > 0 ? n : 1, b);
  return dim3((unsigned)(g < (1 << 20) ? g : (1 << 20)));
}

}  // namespace

size_t pq_tile_lds_bytes(int rot_dim_pad, int pq_len) {
  (void)rot_dim_pad;
  const size_t loop = (size_t)2 * 256 * pq_len * 4 + (size_t)2 * kPqTileQ * 256 * 4 + (size_t)2 * kPqTileQ * pq_len * 4;
  const size_t dist = (size_t)kPqTileQ * kPqChunkRows * 4;
  return 256 + 16 + (loop > dist ? loop : dist);
}

template <int KCAP>
static hipError_t launch_pq_tiled_k(const PqTileArgs& a, int grid, size_t lds, hipStream_t s) {
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_pq_scan_tiled<KCAP>),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  if (attr != hipSuccess) return attr;
  hipLaunchKernelGGL(k_pq_scan_tiled<KCAP>, dim3((unsigned)grid), dim3(512), lds, s, a);
  return hipGetLastError();
}

hipError_t launch_pq_scan_tiled(const PqTileArgs& a, int kcap, int grid, hipStream_t s) {
  const size_t lds = pq_tile_lds_bytes(a.rot_dim_pad, a.pq_len);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  switch (kcap) {
    case 1: return launch_pq_tiled_k<1>(a, grid, lds, s);
    case 4: return launch_pq_tiled_k<4>(a, grid, lds, s);
    case 8: return launch_pq_tiled_k<8>(a, grid, lds, s);
    case 12: return launch_pq_tiled_k<12>(a, grid, lds, s);
    case 16: return launch_pq_tiled_k<16>(a, grid, lds, s);
    case 32: return launch_pq_tiled_k<32>(a, grid, lds, s);
    default: return hipErrorInvalidValue;
  }
}

// LDS candidate capacity per query: 0 = DUMP (k > kMaxK without candidate-superset slots, or k > kRtCandMax)
static int pq_rt_cq(int k, bool cands) { return k > kMaxK && !(cands && k <= kRtCandMax) ? 0 : (k <= 16 ? 128 : 512); }

size_t pq_rt_lds_bytes(int rot_dim_pad, int pq_dim, int k, bool lut16) {
  const size_t loop = (size_t)kRtQ * rot_dim_pad * 4 + (size_t)4 * kPqCodes * (lut16 ? 12 : 20) * 4 +
                      (size_t)pq_dim * kRtQ * 4;
  const size_t sel = (size_t)kRtQ * kRtThreads * 4 + (size_t)kRtQ * pq_rt_cq(k, true) * 8;  // (the larger)
  return 512 + (loop > sel ? loop : sel);
}

bool pq_rt_supported(int rot_dim_pad, int pq_dim, int pq_len, int k) {
  return (pq_len & 3) == 0 && pq_len >= 4 && pq_len <= 16 && rot_dim_pad % 4 == 0 && k >= 1 &&
         (pq_dim & 3) == 0 &&
         k <= kMaxSelectK && pq_rt_lds_bytes(rot_dim_pad, pq_dim, k) <= 160 * 1024;
}

template <int PL4, int CQ, bool H16>
static hipError_t launch_pq_rt_kh(const PqTileArgs& a, int grid, size_t lds, hipStream_t s) {
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_pq_scan_rt<PL4, CQ, H16>),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  if (attr != hipSuccess) return attr;
  hipLaunchKernelGGL((k_pq_scan_rt<PL4, CQ, H16>), dim3((unsigned)grid), dim3(kRtThreads), lds, s, a);
  return hipGetLastError();
}

template <int PL4, int CQ>
static hipError_t launch_pq_rt_k(const PqTileArgs& a, int grid, size_t lds, hipStream_t s) {
  return a.lut16 ? launch_pq_rt_kh<PL4, CQ, true>(a, grid, lds, s) : launch_pq_rt_kh<PL4, CQ, false>(a, grid, lds, s);
}

template <int PL4>
static hipError_t launch_pq_rt_pl(const PqTileArgs& a, int grid, size_t lds, hipStream_t s) {
  switch (pq_rt_cq(a.k, a.slot_cap > 0)) {
    case 0: return launch_pq_rt_k<PL4, 0>(a, grid, lds, s);
    case 128: return launch_pq_rt_k<PL4, 128>(a, grid, lds, s);
    default: return launch_pq_rt_k<PL4, 512>(a, grid, lds, s);
  }
}

namespace {
// entry e = (j, c): the fmaf chain of b_i b_i (dims ascending, from 0), and K9r's MFMA operand copy of the
// row (dim 4s + g at g * pl / 4 + s, times -2 for L2 / -1 for IP: exact)
__global__ void k_pq_book_prep(const float* __restrict__ books, int n, int pl, float scale, float* __restrict__ norms,
                               float* __restrict__ mf) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  const float* b = books + (int64_t)e * pl;
  float bn = 0.0f;
  for (int i = 0; i < pl; ++i) {
    bn = fmaf(b[i], b[i], bn);
    mf[(int64_t)e * pl + ((pl & 3) ? i : (i & 3) * (pl / 4) + (i >> 2))] = scale * b[i];  // (pl % 4: no K9r)
  }
  norms[e] = bn;
}
}  // namespace

hipError_t launch_pq_book_prep(const float* books, int pq_dim, int pq_len, int ip, float* book_norms,
                               float* books_mfma, hipStream_t s) {
  const int n = pq_dim * kPqCodes;
  hipLaunchKernelGGL(k_pq_book_prep, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, s, books, n, pq_len,
                     ip ? -1.0f : -2.0f, book_norms, books_mfma);
  return hipGetLastError();
}

hipError_t launch_pq_scan_rt(const PqTileArgs& a, int grid, hipStream_t s) {
  if (!pq_rt_supported(a.rot_dim_pad, a.pq_dim, a.pq_len, a.k)) return hipErrorInvalidValue;
  if (a.books_mfma == nullptr || a.book_norms == nullptr) return hipErrorInvalidValue;
  const int cq = pq_rt_cq(a.k, a.slot_cap > 0);
  if (cq == 0 && a.slot_info == nullptr) return hipErrorInvalidValue;
  // (k > kMaxK without DUMP: candidate-superset slots of slot_cap >= k entries)
  if (cq > 0 && a.k > kMaxK && (a.slot_cap < a.k || a.slot_cap % 64 != 0)) return hipErrorInvalidValue;
  if ((a.k <= kMaxK || cq == 0) && a.slot_cap != 0) return hipErrorInvalidValue;
  if (a.ip && (a.probes == nullptr || a.probes_d == nullptr)) return hipErrorInvalidValue;
  if (a.lut16 && a.ip) return hipErrorInvalidValue;  // (fp16 LUT: L2 only)
  const size_t lds = pq_rt_lds_bytes(a.rot_dim_pad, a.pq_dim, a.k, a.lut16 != 0);
  switch (a.pq_len >> 2) {
    case 1: return launch_pq_rt_pl<1>(a, grid, lds, s);
    case 2: return launch_pq_rt_pl<2>(a, grid, lds, s);
    case 3: return launch_pq_rt_pl<3>(a, grid, lds, s);
    default: return launch_pq_rt_pl<4>(a, grid, lds, s);
  }
}

// K9 workgroup size: 1024 threads (4 waves per SIMD) when the merge area of 1024 lane lists
// still fits beside the LUT, else 512
static int pq_scan_threads(int rot_dim_pad, int pq_dim, int kcap) {
  const size_t lut = (size_t)pq_dim * kPqCodes * 4;
  const size_t merge = (size_t)1024 * kcap * 8 + (size_t)16 * kcap * 8;
  return (size_t)rot_dim_pad * 4 + (lut > merge ? lut : merge) <= 160 * 1024 ? 1024 : 512;
}

size_t pq_scan_lds_bytes(int rot_dim_pad, int pq_dim, int kcap) {
  const int nt = pq_scan_threads(rot_dim_pad, pq_dim, kcap);
  const size_t lut = (size_t)pq_dim * kPqCodes * 4;
  const size_t merge = (size_t)nt * kcap * 8 + (size_t)(nt / 64) * kcap * 8;
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

template <int KCAP, int NT>
static hipError_t launch_pq_scan_kn(const PqScanArgs& a, size_t lds, hipStream_t s) {
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_pq_scan<KCAP, NT>),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  if (attr != hipSuccess) return attr;
  hipLaunchKernelGGL((k_pq_scan<KCAP, NT>), dim3((unsigned)a.n_slots), dim3(NT), lds, s, a);
  return hipGetLastError();
}

template <int KCAP>
static hipError_t launch_pq_scan_k(const PqScanArgs& a, size_t lds, hipStream_t s) {
  if (pq_scan_threads(a.rot_dim_pad, a.pq_dim, KCAP) == 1024) return launch_pq_scan_kn<KCAP, 1024>(a, lds, s);
  return launch_pq_scan_kn<KCAP, 512>(a, lds, s);
}

size_t pq_split_lds_bytes(int rot_dim_pad, int pq_half, int kcap) {
  return (size_t)rot_dim_pad * 4 + (size_t)pq_half * kPqCodes * 4 + (size_t)4 * kcap * 8;
}

template <int KCAP>
static hipError_t launch_pq_split_k(const PqScanArgs& a, size_t lds, hipStream_t s) {
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_pq_scan_split<KCAP>),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  if (attr != hipSuccess) return attr;
  hipLaunchKernelGGL((k_pq_scan_split<KCAP>), dim3((unsigned)a.n_slots), dim3(256), lds, s, a);
  return hipGetLastError();
}

// K9s when it applies (pq_len <= 16 and a multiple of 4, each half <= 64 subspaces): returns
// hipErrorNotSupported otherwise, for the caller to use K9
hipError_t launch_pq_scan_split(const PqScanArgs& a, int kcap, hipStream_t s) {
  if (a.n_slots <= 0) return hipSuccess;
  if (a.n_slots > 0x7FFFFFFF) return hipErrorInvalidValue;
  if ((a.pq_len & 3) != 0 || a.pq_len > 16 || a.pq_half <= 0 || a.pq_half > 64 || (a.pq_half & 15) != 0 ||
      2 * a.pq_half < a.pq_dim)
    return hipErrorNotSupported;
  const size_t lds = pq_split_lds_bytes(a.rot_dim_pad, a.pq_half, kcap);
  if (lds > 160 * 1024) return hipErrorNotSupported;
  switch (kcap) {
    case 1: return launch_pq_split_k<1>(a, lds, s);
    case 4: return launch_pq_split_k<4>(a, lds, s);
    case 8: return launch_pq_split_k<8>(a, lds, s);
    case 12: return launch_pq_split_k<12>(a, lds, s);
    case 16: return launch_pq_split_k<16>(a, lds, s);
    case 32: return launch_pq_split_k<32>(a, lds, s);
    case 64: return launch_pq_split_k<64>(a, lds, s);
    default: return hipErrorNotSupported;
  }
}

hipError_t launch_pq_scan(const PqScanArgs& a, int kcap, hipStream_t s) {
  if (a.n_slots <= 0) return hipSuccess;
  if (a.n_slots > 0x7FFFFFFF) return hipErrorInvalidValue;
  const size_t lds = pq_scan_lds_bytes(a.rot_dim_pad, a.pq_dim, kcap);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  switch (kcap) {
    case 0: return launch_pq_scan_k<0>(a, lds, s);
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
