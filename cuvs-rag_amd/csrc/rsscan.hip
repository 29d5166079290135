// K13 — row-stationary fp16 pre-filter scan for IVF search.
//
// Why: K10 keeps a 64-query tile in LDS and streams every list chunk once per tile, so a row of
// a list probed by m queries crosses the L2 -> CU path ceil(m/64) times and, unless the tiles of a
// chunk happen to run in step on one XCD, comes from the fabric (MALL / HBM) that many times: at
// the benchmark shape 46 GB of fabric reads per launch against 15.4 GB of compulsory fp16 rows
// (profiles/r01e_pf_pmc_scan_t64.json). K13 turns the roles round:
//
//   * work item = (list, block of 8 row groups = 256 rows); wave w of the CU keeps group w of the
//     block as MFMA A operands IN REGISTERS for the whole item (NK k-steps x 16 B per lane:
//     192 VGPRs at d = 768), so every row is read from HBM exactly once per search;
//   * the list's queries stream past the rows in 32-query tiles: each tile's fp16 image
//     ([NK pieces][64 lanes] x 16 B, one conflict-free ds_read_b128 per two v_mfma_f32_16x16x32_f16)
//     plus a 16-B header per query is copied global -> LDS by LDS-DMA (buffer_load_dwordx4 ... lds, no
//     VGPRs), double buffered, an LDS tiles-ready counter per tile; the queries of a list (~0.5 MB) stay in the
//     XCD's 32 CUs work through the list's blocks (items are dealt from 8 per-XCD queues in list order);
//   * the next item's rows are loaded into the A registers during the item's last tile, each
//     register right after its last MFMA;
//   * no per-lane top-k: every query carries a bound T_q from a pre-pass (the exact k-th key over
//     its nearest list) with T_q >= the refine window of the final answer. The epilogue
//     tests, per lane and query half, ONE filter value bounding the lane's 8 rows from below (largest dot,
//     smallest row norm of the group); a lane that may hold a row with approximate key <= T_q writes its 8
//     dots as a 48-B record to the wave's stream (ballot positions, no atomics, no per-hit loop). The
//     bucketing kernels expand the records with the exact per-row filter into per-query candidate runs,
//     and K11 ranks them exactly. So a wave with hits costs three stores, not a per-hit loop that holds
//     every other wave at the next tile's ready counter.
//
// The result is the pinned fp32 answer (K11 recomputes every window candidate in the oracle's
// order; queries whose buffer overflows go to the exact scan).
#include <climits>

#include "mivs_common.hpp"
#include "pf_math.hpp"

namespace mivs {

namespace {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(1))) void* gbl_ptr_t;

constexpr int kRsThreads = kRsWaves * 64;


// a work item: {first group, end group, first tile slot, tiles} (k_rs_items)
struct RsItem {
  int g0, gend, slot, ntiles;
};

__device__ __forceinline__ RsItem rs_item(const RsScanArgs& a, int w) {
  const int4 v = a.items[w];
  return RsItem{__builtin_amdgcn_readfirstlane(v.x), __builtin_amdgcn_readfirstlane(v.y),
                __builtin_amdgcn_readfirstlane(v.z), __builtin_amdgcn_readfirstlane(v.w)};
}

// Stage one 32-query tile into an LDS buffer: the tile's image ([NK + 1] pieces x 1 KiB, built by
// k_rs_tiles in exactly the LDS layout) is copied piece by piece by LDS-DMA, pieces dealt round-robin
// over the 8 waves; every wave-instruction reads 1 KiB contiguous.
// a buffer descriptor over [p, p + bytes) for a wave-uniform p (loads past `bytes` return zeros)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t uniform_rsrc(const char* p, int bytes) {
  const uint64_t v = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), 0, bytes, 0x00020000);
}

// LDS-DMA the compiler does not see. Its wait-count pass puts vmcnt(0) before any LDS read that follows
// an LDS-DMA it knows of (it cannot tell the DMA's target from the buffer being read), which made every
// epilogue wait for the NEXT tile's DMA and, at an item's last tile, for the next item's rows. These
// copies are ordered by the kernel's own s_waitcnt vmcnt(0) + barrier at each tile start instead (the
// only point where their data is read). The hardware counter still counts them, so the compiler's own
// counted waits can only wait longer, never less.
typedef int v4i __attribute__((ext_vector_type(4)));

// buffer descriptor (raw, 4 SGPRs) over [p, p + bytes) for a wave-uniform p
__device__ __forceinline__ v4i uniform_desc(const void* p, int bytes) {
  const uint64_t v = reinterpret_cast<uint64_t>(p);
  v4i r;
  r.x = (int)__builtin_amdgcn_readfirstlane((uint32_t)v);
  r.y = (int)(__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) & 0xFFFFu);
  r.z = __builtin_amdgcn_readfirstlane(bytes);
  r.w = 0x00020000;
  return r;
}

// 64 lanes x 16 B from desc + voff (per lane) + soff to LDS lds + 16 lane
__device__ __forceinline__ void dma_b128(v4i desc, const void* lds, int voff, int soff) {
  const uint32_t m0 = __builtin_amdgcn_readfirstlane((uint32_t)reinterpret_cast<uintptr_t>(lds));
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
               :: "s"(m0), "v"(voff), "s"(desc), "s"(soff) : "memory");
}


// the image of tile t of list l: tiles of list l start at bucket_off[l] / 32 + l (at most
// floor(m_l / 32) + 1 >= ceil(m_l / 32) slots before list l + 1's first)
__device__ __forceinline__ int64_t rs_tile_slot(const int* bucket_off, int l, int t) {
  return (int64_t)(bucket_off[l] / kRsQTile) + l + t;
}

// s_waitcnt vmcnt(v') lgkmcnt(0) for the largest v' <= v in a short ladder (the count is an immediate)
__device__ __forceinline__ void rs_wait_vm(int v) {
#define RS_VM(n) ((n & 15) | (0x7 << 4) | ((n >> 4) << 14))
  if (v >= 48) __builtin_amdgcn_s_waitcnt(RS_VM(48));
  else if (v >= 40) __builtin_amdgcn_s_waitcnt(RS_VM(40));
  else if (v >= 32) __builtin_amdgcn_s_waitcnt(RS_VM(32));
  else if (v >= 24) __builtin_amdgcn_s_waitcnt(RS_VM(24));
  else if (v >= 16) __builtin_amdgcn_s_waitcnt(RS_VM(16));
  else if (v >= 12) __builtin_amdgcn_s_waitcnt(RS_VM(12));
  else if (v >= 8) __builtin_amdgcn_s_waitcnt(RS_VM(8));
  else if (v >= 6) __builtin_amdgcn_s_waitcnt(RS_VM(6));
  else if (v >= 4) __builtin_amdgcn_s_waitcnt(RS_VM(4));
  else if (v >= 3) __builtin_amdgcn_s_waitcnt(RS_VM(3));
  else if (v >= 2) __builtin_amdgcn_s_waitcnt(RS_VM(2));
  else if (v >= 1) __builtin_amdgcn_s_waitcnt(RS_VM(1));
  else __builtin_amdgcn_s_waitcnt(RS_VM(0));
#undef RS_VM
}

// the workgroup's tiles-ready counter (LDS): wait until it reaches target; false if it never did
// within the cap (a safety valve: every wave signals every tile, so the count always arrives)
__device__ __forceinline__ bool rs_spin(int* ctr, int target) {
  for (int i = 0; i < (1 << 20); ++i) {  // (~40 ms: a tile takes ~3 us)
    if (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= target) {
      asm volatile("" ::: "memory");  // (no LDS read of the tile moves above the wait)
      return true;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  return false;
}

__device__ __forceinline__ void rs_signal(int* ctr) {
  asm volatile("" ::: "memory");
  if (__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)) == 0)
    __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

constexpr int kRsBPrefetch = 3;  // k-steps between a B operand's LDS read and its MFMA

template <bool B>
struct BoolC {
  static constexpr bool value = B;
};


// K13 computes on v_mfma_f32_16x16x32_f16 (the chip holds a higher clock on this shape than on
// 32x32x16 at the same cycles per flop: MI355X_MICROARCH.md 'DVFS give-back' item 7; measured 5.44 ->
// 5.19 ms per launch). Tile piece s = 2 t + qb (1 KiB) holds queries 16 qb .. 16 qb + 15 x dims
// 32 t .. 32 t + 31 and feeds two MFMAs, one per 16-row block rb of the wave's group (A registers
// ra[2 t + rb]: lane (c, kq) = (lane & 15, lane >> 4) holds row 16 rb + c, dims 32 t + 8 kq .. + 7);
// the wave ends a tile with the dots of queries c and 16 + c with rows 16 rb + 4 kq + i in
// acc4[2 qb + rb][i].
//
// Tile protocol: two LDS tile buffers; every wave stages 1/8 of the next tile's pieces during its k-loop
// and signals once its reads of the tile are done and its pieces landed; a wave starts the next k-loop
// when all 8 signalled. (A decoupled variant -- three buffers, waves 0..3 staging, waves 4..7 a k-loop
// behind so that each epilogue would run under the SIMD partner's MFMAs -- was correct but slower,
// 5.41 vs 5.20 ms: the LDS-DMA issue cost, ~100+ cycles a piece, then sits on four waves.)
template <int METRIC, int NK>
__global__ __launch_bounds__(kRsThreads, 1) void k_rs_scan(RsScanArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int BUF = NK * 1024 + 1024;
  constexpr int NBUF = 2;
  constexpr int NB = 2 * NK;  // 8-dim blocks of a group row
  constexpr int64_t IMG = (int64_t)(NK + 1) * 1024;
  constexpr int STAGERS = kRsWaves;  // waves that stage tile pieces
  static_assert((NK + STAGERS) / STAGERS < NK, "the image's pieces are issued over k-steps 1..");
  // rows of the next item loaded (two per odd k-step) after this wave's last DMA piece (k-step
  // NK / STAGERS + 1), less two: the order of a k-step's row load and DMA piece is the compiler's
  constexpr int ROWS_AFTER = [] {
    int c = 0;
    for (int s = NK / STAGERS + 2; s < NK; ++s) c += (s & 1) ? 2 : 0;
    return c - 2 > 0 ? c - 2 : 0;
  }();
  // tiles-ready counter: every wave adds 1 per tile once it has finished reading the previous tile and its
  // DMA pieces of this one have landed (a sum over waves is a safe test: all of them wait on it, so none is
  // a tile ahead of another when one starts a tile); no workgroup barrier per tile
  int* s_ready = reinterpret_cast<int*>(smem + NBUF * BUF);
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int kq = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // XCD-aware schedule: queue x (= blockIdx % 8, the XCD under round-robin placement; speed only) holds
  // the x-th eighth of the list-ordered items, so the CUs of an XCD work through the blocks of the same
  // lists together (the lists' query tiles stay in that XCD's L2). Its P workgroups take the first P
  // items, then deal the rest dynamically from the queue's counter (a.queue[x]): a static deal left the
  // last workgroup 6.6 % behind the mean (phase clocks: busy mean 5.03 ms, max 5.36 ms). Lane 0 of
  // wave 0 grabs three items ahead into an LDS ring (s_next): grabbed during item j's first tile (after
  // its wait, published before its signal), an index is read at the start of item j + 2, when every
  // wave has seen that signal -- every item has at least one tile. Every item is taken exactly once
  // (indices past the queues' ends read as -1, and once -1 always -1).
  const int x = blockIdx.x & 7, P = gridDim.x >> 3;
  const int hi = __builtin_amdgcn_readfirstlane(a.bounds[x + 1]);
  const int lo_x = __builtin_amdgcn_readfirstlane(a.bounds[x]);
  int w = lo_x + (int)(blockIdx.x >> 3);
  int* const s_next = s_ready + 4;  // [4] ring of upcoming item indices
  // [4] their descriptors: the grabber loads item j + 2's during item j's first tile and publishes it with that
  // tile's signal, so no wave waits on a global load of the item table at an item boundary (it read
  // items[w] there before: one L2 / HBM round trip, ~4.7k cycles per item and wave)
  int4* const s_desc = reinterpret_cast<int4*>(s_ready + 8);
  // this workgroup's next item; once its own queue is dry it takes items from the other queues in turn (the
  // tail of a launch), so no CU idles while any item is left
  auto grab = [&](int) {
    int v = lo_x + P + atomicAdd(a.queue + x, 1);
    if (v < hi) return v;
    for (int k = 1; k < 8; ++k) {
      const int xq = (x + k) & 7;
      v = a.bounds[xq] + P + atomicAdd(a.queue + xq, 1);
      if (v < a.bounds[xq + 1]) return v;
    }
    return -1;
  };
  int ii = 0;  // this workgroup's item ordinal
  const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
  int n_tiles_done = 0;
  int tt = 0;               // tiles this wave has started
  bool spun_out = false;    // a wait gave up (never expected): the results are then not trusted
  uint64_t pw_wait = 0, pw_loop = 0, pw_epi = 0, pw_dma = 0;  // flags & 16: this wave's cycles per tile phase
  uint64_t pw_drain = 0, pw_hit = 0, n_hit_tiles = 0;  // flags & 16: MFMA-result wait, hit path, tiles taking it
  uint64_t pw_first = 0, n_items = 0;  // flags & 16: k-loop cycles of items' first tiles, items
  const uint64_t pw_t0 = __builtin_amdgcn_s_memtime();
  const int widx = blockIdx.x * kRsWaves + wave;
  int4* const wstream = a.wave_buf + (int64_t)widx * a.wave_cap * kRsRecInt4;
  int wcnt = 0;  // records of this wave's candidate stream
  auto block_prof = [&]() {
    // The stream length is the count of records actually written (at most wave_cap), so the bucketing never reads
    // a slot this search did not fill. A stream that overflowed, or a wave that gave up waiting (its records may
    // come from a stale LDS tile: it reports none), raises the lost flag wave_cnt[waves]: every query of the batch
    // then takes the fallback search. A spun-out wave also counts itself in wave_cnt[waves + 9] for the stats.
    if (lane == 0) {
      a.wave_cnt[widx] = spun_out ? 0 : min(wcnt, a.wave_cap);
      if (spun_out || wcnt > a.wave_cap) atomicOr(a.wave_cnt + gridDim.x * kRsWaves, 1);
      if (spun_out) atomicAdd(a.wave_cnt + gridDim.x * kRsWaves + 9, 1);
    }
    if ((a.flags & 8) && a.prof && tid == 0) {  // (timing only) flags & 8: per block {start, end, tiles}
      a.prof[3 * blockIdx.x] = t_start;
      a.prof[3 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
      a.prof[3 * blockIdx.x + 2] = (unsigned long long)n_tiles_done;
    }
    if ((a.flags & 16) && a.prof && lane == 0) {  // flags & 16: wave-cycles per phase summed
      unsigned long long* p = a.prof + 3 * gridDim.x;
      atomicAdd(p + 0, (unsigned long long)pw_wait);
      atomicAdd(p + 1, (unsigned long long)pw_loop);
      atomicAdd(p + 2, (unsigned long long)pw_epi);
      atomicAdd(p + 3, (unsigned long long)pw_dma);
      atomicAdd(p + 4, (unsigned long long)pw_drain);
      atomicAdd(p + 5, (unsigned long long)pw_hit);
      atomicAdd(p + 6, (unsigned long long)n_hit_tiles);
      atomicAdd(p + 7, (unsigned long long)n_tiles_done);
      atomicAdd(p + 8, (unsigned long long)pw_first);
      atomicAdd(p + 9, (unsigned long long)n_items);
      atomicAdd(p + 10, (unsigned long long)(__builtin_amdgcn_s_memtime() - pw_t0));
    }
  };
  if (w >= hi) {
    block_prof();
    return;
  }
  RsItem it = rs_item(a, w);
  int g = it.g0 + wave;
  bool gv = g < it.gend;
  // Buffer loads: a per-group descriptor in SGPRs (uniform base, NB * 512 bytes), this lane's 32-bit
  // offset in one VGPR and the register's offset in soffset -- no per-lane 64-bit address per register to
  // keep (the next item's 48 would not fit beside the resident rows)
  const int lane_off = kq * 512 + (lane & 15) * 16;
  auto group_rsrc = [&](int grp) {
    return uniform_rsrc(reinterpret_cast<const char*>(a.groups_h) + (int64_t)grp * (NB * 512), NB * 512);
  };
  // the rows are read once per search: non-temporal policy (aux = 2), 1.5-2.5 % shorter launches than the default
  // policy in alternating same-box runs (profiles/r03_k13_experiments.txt)
  auto ld_rows = [&](__amdgpu_buffer_rsrc_t r, int i) {  // register i = 2 t + rb
    return __builtin_bit_cast(h8, __builtin_amdgcn_raw_buffer_load_b128(r, lane_off, (i >> 1) * 2048 + (i & 1) * 256, 2));
  };
  if (tid == 0) {
    *s_ready = 0;
    s_next[1] = grab(1);
    s_next[2] = grab(2);
    if (s_next[1] >= 0) s_desc[1] = a.items[s_next[1]];
  }
  __syncthreads();  // (the only workgroup barrier: the counter is zero before any wave signals)
  {  // tile 0's pieces
    const v4i d0 = uniform_desc(a.tiles + it.slot * IMG, (int)IMG);
#pragma unroll
    for (int p0 = 0; p0 <= NK; p0 += STAGERS)
      if (p0 + wave <= NK) dma_b128(d0, smem + (p0 + wave) * 1024, lane * 16, (p0 + wave) * 1024);
  }
  // the smallest row norm of the wave's group (the filter's lower bound; pad rows: +inf, so a real row's)
  float xn_next = METRIC == kL2 ? a.group_nmin[gv ? g : it.g0] : 0.0f;
  h8 ra[NK];
  {
    const __amdgpu_buffer_rsrc_t r0 = group_rsrc(gv ? g : it.g0);
#pragma unroll
    for (int s = 0; s < NK; ++s) ra[s] = ld_rows(r0, s);
  }
  float xnmin = 0.0f;  // the smallest row norm of the wave's group in the current item
  int cur = 0;         // LDS buffer of the current tile (tt % NBUF)
  const f32x4 zero4 = {0.f, 0.f, 0.f, 0.f};

  for (;;) {
    const int ntiles = it.ntiles;
    const int wn = s_next[(ii + 1) & 3];
    const bool has_next = wn >= 0;
    // the next item's descriptor: read in this item's LAST tile, after its ready wait (the grabber wrote it
    // with its signal of the previous item's first tile; an item may have a single tile, so the item start
    // itself is too early)
    RsItem nx = it;
    int gnx = 0;
    bool gvn = false;
    // the filter over one tile's dots; h0 / h1 = the headers {qs, uf, qn, q} of queries c and 16 + c,
    // read before the wave signalled the tile (after that the buffer may be restaged). Lane (c, kq) holds the
    // dots of query 16 qb + c with rows 4 kq + i and 16 + 4 kq + i in acc4[2 qb] / acc4[2 qb + 1].
    auto epilogue = [&](const f32x4 (&acc4)[4], const float4& h0, const float4& h1, uint64_t& ph2d)
                        __attribute__((always_inline)) {
      const float mm0 = METRIC == kL2 ? -2.0f * h0.x : -h0.x;
      const float mm1 = METRIC == kL2 ? -2.0f * h1.x : -h1.x;
      // mm < 0, so every row's filter value fma(acc, mm, xn) is >= fma(max acc, mm, min xn) (exact ordering,
      // one monotone rounding): a lane whose bound does not reach uf holds no hit of that query
      float am0 = fmaxf(acc4[0][0], acc4[1][0]), am1 = fmaxf(acc4[2][0], acc4[3][0]);
#pragma unroll
      for (int i = 1; i < 4; ++i) {
        am0 = fmaxf(am0, fmaxf(acc4[0][i], acc4[1][i]));
        am1 = fmaxf(am1, fmaxf(acc4[2][i], acc4[3][i]));
      }
      const float xb = METRIC == kL2 ? xnmin : 0.0f;
      // (an empty slot of the tile has the null header: uf = -inf, never passes)
      const bool p0 = fmaf(am0, mm0, xb) < h0.y, p1 = fmaf(am1, mm1, xb) < h1.y;
      const uint64_t m0 = __ballot(p0), m1 = __ballot(p1);
      if ((m0 | m1) == 0) return;
      if (a.flags & 16) {
        ++n_hit_tiles;
        ph2d = __builtin_amdgcn_s_memtime();
      }
      // one 48-B record per (lane, query half) that passes: the 8 dots, then {first row position, query}
      const int pos0 = g * kGroupRows + 4 * kq;
      const int n0 = __popcll(m0);
      if (p0) {
        const int at = wcnt + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m0 >> 32),
                                                             __builtin_amdgcn_mbcnt_lo((uint32_t)m0, 0u));
        if (at < a.wave_cap) {
          int4* r = wstream + (int64_t)at * kRsRecInt4;
          r[0] = __builtin_bit_cast(int4, acc4[0]);
          r[1] = __builtin_bit_cast(int4, acc4[1]);
          r[2] = make_int4(pos0, __float_as_int(h0.w), 0, 0);
        }
      }
      if (p1) {
        const int at = wcnt + n0 + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m1 >> 32),
                                                                  __builtin_amdgcn_mbcnt_lo((uint32_t)m1, 0u));
        if (at < a.wave_cap) {
          int4* r = wstream + (int64_t)at * kRsRecInt4;
          r[0] = __builtin_bit_cast(int4, acc4[2]);
          r[1] = __builtin_bit_cast(int4, acc4[3]);
          r[2] = make_int4(pos0, __float_as_int(h1.w), 0, 0);
        }
      }
      wcnt += n0 + __popcll(m1);
    };

    // One tile. The item's rows have landed (the wait at the item start); this wave's DMA of the next tile
    // lands by the counted wait below, which leaves the candidate stores issued after it in flight. The last
    // tile (LAST) is a separate copy, the only one that loads the next item's rows: in a loop shared by
    // all tiles the compiler would wait for every vector-memory operation before the first MFMA.
    auto tile = [&](int t, auto last_c) __attribute__((always_inline)) {
      constexpr bool LAST = decltype(last_c)::value;
      const uint64_t ph0 = (a.flags & 16) ? __builtin_amdgcn_s_memtime() : 0;
      // every wave's pieces of this tile have landed and every wave is done with the previous tile
      if (!spun_out && !rs_spin(s_ready, kRsWaves * (tt + 1))) spun_out = true;
      ++tt;
      if (LAST && has_next) {
        const int4 v = s_desc[(ii + 1) & 3];
        nx = RsItem{__builtin_amdgcn_readfirstlane(v.x), __builtin_amdgcn_readfirstlane(v.y),
                    __builtin_amdgcn_readfirstlane(v.z), __builtin_amdgcn_readfirstlane(v.w)};
        gnx = nx.g0 + wave;
        gvn = gnx < nx.gend;
      }
      const bool grabber = t == 0 && wave == 0 && lane == 0;
      int grabbed = -1;
      int4 desc2 = make_int4(0, 0, 0, 0);
      if (grabber) {
        grabbed = grab(ii + 3);  // (its result is waited for at the signal below)
        const int w2 = s_next[(ii + 2) & 3];  // (grabbed during the previous item's first tile)
        if (w2 >= 0) desc2 = a.items[w2];
      }
      const uint64_t ph1 = (a.flags & 16) ? __builtin_amdgcn_s_memtime() : 0;
      const bool last = LAST;
      // the next tile (of this item, or the next item's first) goes into the next buffer. Its pieces are
      // issued one per k-step from the second on: issued before the first MFMA, the compiler's wait for the
      // rows there (vmcnt(0): it cannot order them across the loop) would wait for this DMA too
      // (a buffer descriptor over the image: no branch per piece; with nothing to stage -- the block's
      // last tile -- its size is 0 and the loads write zeros to a buffer no tile reads again)
      // (flags & 32, timing only: every tile of an item re-reads the item's first image, so the tile DMA only ever
      // reads L2-resident bytes -- separates the tiles' L2 / fabric latency from the rest of the ready wait)
      const char* simg = !last ? a.tiles + (it.slot + ((a.flags & 32) ? 0 : t + 1)) * IMG : a.tiles + nx.slot * IMG;
      const bool stage = (!last || has_next) && !(a.flags & 2);
      const v4i sdesc = uniform_desc(simg, stage ? (int)IMG : 0);
      const int nxt = cur + 1 == NBUF ? 0 : cur + 1;
      char* sbuf = smem + nxt * BUF;
      // (flags & 4, timing only: keep the rows, i.e. measure the item transitions' cost)
      const bool reload = LAST && has_next && !(a.flags & 4);
      const __amdgpu_buffer_rsrc_t nrs = group_rsrc(gvn ? gnx : nx.g0);
      f32x4 acc4[4] = {zero4, zero4, zero4, zero4};
      // (a wave without a group in this block runs the MFMAs on stale rows; its epilogue is skipped).
      // Copies of the k-loop with / without the next item's row loads and the staging, so no k-step branches.
      auto kloop = [&](auto reload_c) __attribute__((always_inline)) {
        constexpr bool RL = decltype(reload_c)::value;
        const char* bb = smem + cur * BUF + lane * 16;
        constexpr int PD = kRsBPrefetch;  // B operands PD pieces ahead (ring of PD + 1)
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
            // the next item's rows, right after the last use of the registers (registers 2 t, 2 t + 1 after
            // piece 2 t + 1), its group's smallest row norm first, with the first k-step
            if (s == 0 && METRIC == kL2) xn_next = a.group_nmin[gvn ? gnx : nx.g0];
            if (s & 1) {
              ra[s - 1] = ld_rows(nrs, s - 1);
              ra[s] = ld_rows(nrs, s);
            }
          }
          {
            if (s >= 1 && (s - 1) * STAGERS <= NK) {
              // (past the last piece a wave loads the last one again: the same bytes to the same place)
              const int p = min((s - 1) * STAGERS + wave, NK);
              dma_b128(sdesc, sbuf + p * 1024, lane * 16, p * 1024);
            }
          }
          // keep each k-step's operations in their k-step: left alone, the scheduler sinks the B reads
          // next to their MFMAs (one exposed LDS latency per k-step)
          __builtin_amdgcn_sched_barrier(0);
        }
      };
      if (LAST && reload) kloop(BoolC<LAST>{});
      else kloop(BoolC<false>{});
      const uint64_t ph2 = (a.flags & 16) ? __builtin_amdgcn_s_memtime() : 0;
      // (the header piece holds query j's header at lanes j and j + 32)
      const float4 hq0 = *reinterpret_cast<const float4*>(smem + cur * BUF + NK * 1024 + (lane & 15) * 16);
      const float4 hq1 = *reinterpret_cast<const float4*>(smem + cur * BUF + NK * 1024 + (16 + (lane & 15)) * 16);
      // (all four fields kept live, so each header is ONE conflict-free ds_read_b128: left alone the compiler reads
      // the three it uses as ds_read_b64 + ds_read_b32, and ds_read_b32 banks are dword mod 32 -- lanes j and j + 8 of
      // a group then collide, 2 extra LDS cycles per header read: r03b's 13.2M SQ_LDS_BANK_CONFLICT cycles)
      asm volatile("" ::"v"(hq0.z), "v"(hq1.z));
      // signal the next tile: this wave's reads of this one are done (lgkmcnt(0): the headers are in) and
      // its DMA pieces of the next have landed -- vmcnt counts, in issue order, only the next item's rows
      // issued after its last piece beyond them
      rs_wait_vm(reload ? ROWS_AFTER : 0);
      if (grabber) {
        s_next[(ii + 3) & 3] = grabbed;
        s_desc[(ii + 2) & 3] = desc2;
      }
      rs_signal(s_ready);
      const uint64_t ph2b = (a.flags & 16) ? __builtin_amdgcn_s_memtime() : 0;
      uint64_t ph2c = ph2b, ph2d = 0;
      if (a.flags & 16) {  // (timing only) the wait for the k-loop's last MFMA result
        float tv = acc4[3][3];
        asm volatile("v_mov_b32 %0, %0" : "+v"(tv));
        ph2c = __builtin_amdgcn_s_memtime();
      }
      if (gv && !(a.flags & 1)) epilogue(acc4, hq0, hq1, ph2d);
      if (a.flags & 16) {
        const uint64_t ph3 = __builtin_amdgcn_s_memtime();
        pw_wait += ph1 - ph0;
        pw_loop += ph2 - ph1;
        if (t == 0) {
          pw_first += ph2 - ph1;
          ++n_items;
        }
        pw_dma += ph2b - ph2;
        pw_drain += ph2c - ph2b;
        pw_epi += ph3 - ph2c;
        if (ph2d) pw_hit += ph3 - ph2d;
      }
      cur = nxt;
    };
    // the item's rows (loaded during the previous item's last tile) and everything before them; at the
    // first item, the prologue's DMA pieces too, which the wave then signals as tile 0's
    // The first item: wait for everything (the prologue's DMA pieces, which the wave then signals as tile 0's,
    // and the rows). Later items: the rows were issued during the previous item's last tile, in k-step order;
    // each is waited for where the first tile's k-loop first reads it (the compiler's counted vmcnt before
    // that MFMA: every DMA piece and record store it cannot see is YOUNGER, so its count only waits longer;
    // measured equal to one vmcnt(0) here, profiles/r03_k13_experiments.txt).
    if (tt == 0) __builtin_amdgcn_s_waitcnt(0x0070);  // vmcnt(0) lgkmcnt(0)
    else __builtin_amdgcn_s_waitcnt(0xC07F);                             // lgkmcnt(0)
    if (tt == 0) rs_signal(s_ready);
    xnmin = xn_next;
    for (int t = 0; t + 1 < ntiles; ++t) tile(t, BoolC<false>{});
    tile(ntiles - 1, BoolC<true>{});
    n_tiles_done += ntiles;
    if (!has_next) break;
    ++ii;
    w = wn;
    it = nx;
    g = gnx;
    gv = gvn;
  }
  block_prof();
}

// The 8 item queues of K13 as ranges of equal TILE work (bounds [9]): an item costs its list's tile count,
// and lists differ in queries, so equal item counts left one queue ~3 % heavier than the mean. Item
// weights are uniform inside a list: queue x starts at the first item whose work prefix reaches
// W x / 8 (W = all items' tiles).
__device__ void rs_bounds_block(const int* __restrict__ work_off, const int* __restrict__ bucket_off, int n_lists,
                                int* __restrict__ bounds) {
  __shared__ int64_t sh[16];
  __shared__ int64_t s_total;
  // pass 1: W
  int64_t tot = 0;
  for (int l0 = 0; l0 < n_lists; l0 += 1024) {
    const int l = l0 + threadIdx.x;
    int64_t wl = 0;
    if (l < n_lists)
      wl = (int64_t)(work_off[l + 1] - work_off[l]) * ((bucket_off[l + 1] - bucket_off[l] + kRsQTile - 1) / kRsQTile);
    int64_t t;
    block_excl_scan(wl, sh, &t);
    tot += t;
  }
  if (threadIdx.x == 0) s_total = tot;
  __syncthreads();
  const int64_t W = s_total;
  const int n_items = work_off[n_lists];
  if (W == 0) {  // nothing to weigh: equal item counts
    if (threadIdx.x <= 8) bounds[threadIdx.x] = (int)((int64_t)n_items * threadIdx.x / 8);
    return;
  }
  if (threadIdx.x == 0) { bounds[0] = 0; bounds[8] = n_items; }
  // pass 2: the list holding each target W x / 8 (x = 1..7) sets bounds[x]
  int64_t cum = 0;
  for (int l0 = 0; l0 < n_lists; l0 += 1024) {
    const int l = l0 + threadIdx.x;
    int64_t wl = 0, nt = 1;
    if (l < n_lists) {
      nt = (bucket_off[l + 1] - bucket_off[l] + kRsQTile - 1) / kRsQTile;
      wl = (int64_t)(work_off[l + 1] - work_off[l]) * nt;
    }
    int64_t t;
    const int64_t c = cum + block_excl_scan(wl, sh, &t);
    if (wl > 0) {
      for (int x = 1; x < 8; ++x) {
        const int64_t target = W * x / 8;
        if (target >= c && target < c + wl) {
          const int64_t b = work_off[l] + (target - c + nt - 1) / nt;
          bounds[x] = (int)(b < work_off[l + 1] ? b : work_off[l + 1]);
        }
      }
    }
    cum += t;
  }
}

// Work items of K13 from the probe map (chunk = kRsBlockGroups groups, one tile column per list):
// item w -> {first group, end group, first tile slot of its list, tiles of its list}
// (one launch: blocks of 1024 items, and with bounds the last block computes the queue bounds)
__global__ __launch_bounds__(1024) void k_rs_items(const int* __restrict__ work_off, const int* __restrict__ bucket_off,
                                                   const int64_t* __restrict__ list_goff, int n_lists, int max_items,
                                                   int4* __restrict__ items, int* __restrict__ zero, int nzero,
                                                   int* __restrict__ bounds) {
  if (bounds && blockIdx.x == gridDim.x - 1) {
    rs_bounds_block(work_off, bucket_off, n_lists, bounds);
    return;
  }
  const int w = blockIdx.x * blockDim.x + threadIdx.x;
  if (w < nzero) zero[w] = 0;  // K13's counters (a memset launch less)
  if (w >= max_items || w >= work_off[n_lists]) return;
  int lo = 0, hi = n_lists - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (work_off[mid] <= w) lo = mid; else hi = mid - 1;
  }
  const int64_t g0 = list_goff[lo] + (int64_t)(w - work_off[lo]) * kRsBlockGroups;
  const int64_t ge = list_goff[lo + 1] < g0 + kRsBlockGroups ? list_goff[lo + 1] : g0 + kRsBlockGroups;
  const int m = bucket_off[lo + 1] - bucket_off[lo];
  items[w] = make_int4((int)g0, (int)ge, (int)rs_tile_slot(bucket_off, lo, 0), (m + kRsQTile - 1) / kRsQTile);
}

// per query: {qs, uf, qn, q} for K13 (uf carries T_q: the one-fma filter bound for the exact k-th key over the
// sample of the nearest list from the pre-pass, widened by the refine window); row nq = the null header
template <int METRIC>
__global__ void k_rs_headers(const float* __restrict__ pre_kth, int64_t nq, const float* __restrict__ qscale,
                             const float* __restrict__ qnorms, const float* __restrict__ qres, float x_norm_max,
                             float x_res_max, int dp, float4* __restrict__ hdr, float* __restrict__ tq,
                             int* __restrict__ zero, int64_t nzero, int* __restrict__ zero2, int nzero2) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  // (zero[0 .. nzero): the one-pass bucketing's per-query counts (nzero <= nq + 1), zero2: the final refine's stats)
  if (q < nzero) zero[q] = 0;
  if (q < nzero2) zero2[q] = 0;
  if (q > nq) return;
  if (q == nq) {  // the null header
    hdr[q] = make_float4(0.0f, -INFINITY, -INFINITY, __int_as_float(-1));
    return;
  }
  const float qn = qnorms[q];
  const float delta = pf_delta<METRIC>(qn, qres[q], x_norm_max, x_res_max, dp);
  float T = INFINITY;
  // the k-th smallest approximate key (K10's) over the sample rows, or the k-th smallest fp32 key of the verified
  // nominees (K11's verify mode: each within delta of its pinned key, as an approximate key is)
  const float kth = pre_kth[q];
  if (kth < INFINITY) {
    // those k rows are probed rows: their pinned keys are <= kth + delta, so the final k-th approximate key
    // (K13's sums may round differently from K10's: each is within delta of the pinned key) is
    // Ak <= U = kth + 2 delta, and the final window pf_window(Ak) <= pf_window(U) (monotone); one more
    // relative step covers the roundings of U and T
    const float U = kth + 2.0f * delta;
    T = pf_window(U, delta);
    T = T + fabsf(T) * 0x1p-20f + 1e-30f;
  }
  const float uf = pf_uf<METRIC>(INFINITY, T, qn, x_norm_max * x_norm_max);
  hdr[q] = make_float4(qscale[q], uf, qn, __int_as_float((int)q));
  if (tq) tq[q] = T;
}

// Tile images for K13: per list l with m_l queries, ceil(m_l / 32) tiles of [NK + 1] x 1 KiB: piece
// s < NK is the MFMA B operand of k-step s (lane j + 32 h: dims 16 s + 8 h .. + 8 of the tile's j-th
// query), piece NK the 16-B headers (lane j: query j's; lanes 32..63 repeat them). One workgroup per
// list (1024 threads: the stores of a list's ~0.5 MB keep more requests in flight); a thread reads 16
// contiguous bytes of a query row (the row's pieces are consecutive threads).
// Piece s = 2 t + qb, lane (c, kq) = (L & 15, L >> 4): dims 32 t + 8 kq .. + 8 of query 16 qb + c (the B
// operand of v_mfma_f32_16x16x32_f16).
template <int NK>
// one workgroup per tile slot (rs_tile_slot: list l's tiles start at bucket_off[l] / 32 + l): wave 0 finds the slot's
// list (64 probes per round: two dependent rounds of loads up to 4,096 lists, where a one-thread binary search took
// log2(n_lists)), the tile's 32 query ids are staged in LDS, then its NK pieces in image order (lane L of piece s
// fastest: every wave-instruction stores 1 KiB contiguous; lanes L and L + 32 read the two adjacent 16-B halves of
// one query's 32 B of k-step s), all of a thread's loads issued before its stores, and the header piece.
// (A workgroup per list had ~10 tiles' worth of dependent id -> row loads per thread.)
__global__ __launch_bounds__(256) void k_rs_tiles(const int64_t* __restrict__ bucket_q, const int* __restrict__ bucket_off,
                                                 int n_lists, const uint16_t* __restrict__ qh,
                                                 const float4* __restrict__ qhdr, int nq, char* __restrict__ tiles) {
  constexpr int64_t IMG = (int64_t)(NK + 1) * 1024;
  static_assert(NK % 4 == 0, "NK * 64 pieces over 256 threads");
  constexpr int PER = NK / 4;
  __shared__ int s_l;
  __shared__ int s_q[kRsQTile];
  const int b = blockIdx.x;
  if (threadIdx.x < 64) {
    // the largest l with bucket_off[l] / 32 + l <= b (the slot function is increasing in l; l = 0 gives 0 <= b)
    const int lane = threadIdx.x;
    int lo = 0, n = n_lists;  // the answer lies in [lo, lo + n)
    while (n > 1) {
      const int step = (n + 63) / 64;
      const int l = lo + lane * step;
      const bool ok = lane * step < n && (bucket_off[l] / kRsQTile + l <= b);
      const int c = __popcll(__ballot(ok));  // probes 0 .. c - 1 pass (c >= 1: probe 0 is lo, which passes)
      lo += (c - 1) * step;
      n = min(step, n - (c - 1) * step);
    }
    if (lane == 0) s_l = lo;
  }
  __syncthreads();
  const int l = s_l;
  const int e0 = bucket_off[l], m = bucket_off[l + 1] - e0;
  const int t = b - (int)rs_tile_slot(bucket_off, l, 0);
  if (t < 0 || t * kRsQTile >= m) return;  // a padding slot between two lists' tiles (never read)
  if (threadIdx.x < kRsQTile) {
    const int e = t * kRsQTile + threadIdx.x;
    s_q[threadIdx.x] = e < m ? (int)bucket_q[e0 + e] : -1;
  }
  __syncthreads();
  char* img = tiles + (int64_t)b * IMG;
  uint4 v[PER];
#pragma unroll
  for (int u = 0; u < PER; ++u) {
    const int i = threadIdx.x + u * 256;
    const int s = i >> 6, L = i & 63;
    const int q = s_q[16 * (s & 1) + (L & 15)];
    const int dim0 = 32 * (s >> 1) + 8 * (L >> 4);
    v[u] = make_uint4(0u, 0u, 0u, 0u);
    if (q >= 0) v[u] = *reinterpret_cast<const uint4*>(qh + (int64_t)q * (NK * 16) + dim0);
  }
  float4 h = make_float4(0.f, 0.f, 0.f, 0.f);
  if (threadIdx.x < 64) {
    const int q = s_q[threadIdx.x & 31];
    h = qhdr[q >= 0 ? q : nq];
  }
  // non-temporal stores: 145 -> 138 us per step, K13 (which reads the images ~1 ms later) unchanged
  // (profiles/r05_variants_tiles.txt)
  typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
#pragma unroll
  for (int u = 0; u < PER; ++u)
    __builtin_nontemporal_store(__builtin_bit_cast(u32x4_t, v[u]), reinterpret_cast<u32x4_t*>(img + (int64_t)(threadIdx.x + u * 256) * 16));
  if (threadIdx.x < 64) *reinterpret_cast<float4*>(img + NK * 1024 + threadIdx.x * 16) = h;
}

}  // namespace

size_t rs_scan_lds_bytes(int dp) {
  const int nk = dp / 16;
  // two tile buffers + the tiles-ready counter, the item ring and its descriptors
  return (size_t)2 * (nk * 1024 + 1024) + 128;
}

bool rs_scan_supported(int dp) {
  return dp % 64 == 0 && dp >= 64 && dp <= 768;
}

template <int METRIC, int NK>
static hipError_t launch_rs_mk(const RsScanArgs& a, int grid, hipStream_t s) {
  const size_t lds = rs_scan_lds_bytes(NK * 16);
  hipError_t e = hipFuncSetAttribute((const void*)k_rs_scan<METRIC, NK>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((k_rs_scan<METRIC, NK>), dim3(grid), dim3(kRsThreads), lds, s, a);
  return hipGetLastError();
}

template <int METRIC>
static hipError_t launch_rs_m(const RsScanArgs& a, int dp, int grid, hipStream_t s) {
  switch (dp / 16) {
    case 4: return launch_rs_mk<METRIC, 4>(a, grid, s);
    case 8: return launch_rs_mk<METRIC, 8>(a, grid, s);
    case 12: return launch_rs_mk<METRIC, 12>(a, grid, s);
    case 16: return launch_rs_mk<METRIC, 16>(a, grid, s);
    case 20: return launch_rs_mk<METRIC, 20>(a, grid, s);
    case 24: return launch_rs_mk<METRIC, 24>(a, grid, s);
    case 28: return launch_rs_mk<METRIC, 28>(a, grid, s);
    case 32: return launch_rs_mk<METRIC, 32>(a, grid, s);
    case 36: return launch_rs_mk<METRIC, 36>(a, grid, s);
    case 40: return launch_rs_mk<METRIC, 40>(a, grid, s);
    case 44: return launch_rs_mk<METRIC, 44>(a, grid, s);
    case 48: return launch_rs_mk<METRIC, 48>(a, grid, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_rs_scan(const RsScanArgs& a, int dp, int grid, hipStream_t s) {
  if (!rs_scan_supported(dp)) return hipErrorInvalidValue;
  return a.metric == kIP ? launch_rs_m<kIP>(a, dp, grid, s) : launch_rs_m<kL2>(a, dp, grid, s);
}

int64_t rs_tiles_bytes(int64_t ne, int n_lists, int dp) {
  return (ne / kRsQTile + n_lists + 1) * (int64_t)(dp / 16 + 1) * 1024;
}

template <int NK>
static void launch_rs_tiles_k(const int64_t* bucket_q, const int* bucket_off, int n_lists, int64_t n_slots,
                              const uint16_t* qh, const float4* qhdr, int nq, char* tiles, hipStream_t s) {
  hipLaunchKernelGGL(k_rs_tiles<NK>, dim3((unsigned)n_slots), dim3(256), 0, s, bucket_q, bucket_off, n_lists, qh, qhdr,
                     nq, tiles);
}

hipError_t launch_rs_tiles(const int64_t* bucket_q, const int* bucket_off, int n_lists, int64_t ne, const uint16_t* qh,
                           const float4* qhdr, int nq, int dp, char* tiles, hipStream_t s) {
  const int64_t n_slots = ne / kRsQTile + n_lists + 1;  // (rs_tiles_bytes' slot bound)
  if (n_lists <= 0 || ne <= 0) return hipSuccess;
  switch (dp / 16) {
#define RS_T(NK) case NK: launch_rs_tiles_k<NK>(bucket_q, bucket_off, n_lists, n_slots, qh, qhdr, nq, tiles, s); break;
    RS_T(4) RS_T(8) RS_T(12) RS_T(16) RS_T(20) RS_T(24) RS_T(28) RS_T(32) RS_T(36) RS_T(40) RS_T(44) RS_T(48)
#undef RS_T
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_rs_items(const int* work_off, const int* bucket_off, const int64_t* list_goff, int n_lists,
                           int max_items, int4* items, int* bounds, hipStream_t s, int* zero, int nzero) {
  if (nzero > 256) return hipErrorInvalidValue;
  if (max_items <= 0 && nzero <= 0) return hipSuccess;
  const unsigned nb = (unsigned)ceil_div(max_items > 0 ? max_items : 1, 1024) + (bounds ? 1 : 0);
  hipLaunchKernelGGL(k_rs_items, dim3(nb), dim3(1024), 0, s, work_off, bucket_off, list_goff, n_lists, max_items, items,
                     zero, nzero, bounds);
  return hipGetLastError();
}

// K13's per-wave record streams -> per-query CSR runs for K11: stream offsets (one workgroup), then
// count and scatter. A record {8 dots of one lane, first row position, query} expands to the rows whose
// exact filter value fma(acc, mm, xn) passes uf -- the same test, on the same values, as a per-row test in
// K13's epilogue would make -- each with its approximate key. A stream longer than its capacity lost
// records of unknown queries: `lost` is then set and K11 proves no query (every query goes to the fallback).
// (it also zeroes the count kernel's per-query counters and the scatter's fills: zero[0 .. nzero) in 16-B words)
__global__ __launch_bounds__(1024) void k_rs_stream_off(const int* __restrict__ wave_cnt, int n_waves, int wave_cap,
                                                        int64_t* __restrict__ woff, int* __restrict__ lost,
                                                        int4* __restrict__ zero, int64_t nzero,
                                                        int4* __restrict__ zero2, int nzero2) {
  __shared__ int64_t sh[16];
  for (int64_t i = threadIdx.x; i < nzero; i += 1024) zero[i] = make_int4(0, 0, 0, 0);
  if (threadIdx.x < nzero2) zero2[threadIdx.x] = make_int4(0, 0, 0, 0);  // (the final refine's stats)
  int64_t base = 0;
  for (int w0 = 0; w0 < n_waves; w0 += 1024) {
    const int w = w0 + threadIdx.x;
    int64_t c = 0;
    if (w < n_waves) {  // (K13 reports at most wave_cap records per stream and raises `lost` itself)
      const int n = wave_cnt[w];
      if (n > wave_cap) atomicOr(lost, 1);
      c = n < 0 ? 0 : (n < wave_cap ? n : wave_cap);
    }
    int64_t tot;
    const int64_t ex = block_excl_scan(c, sh, &tot);
    if (w < n_waves) woff[w] = base + ex;
    base += tot;
  }
  if (threadIdx.x == 0) woff[n_waves] = base;
}

// one record: its query, and the rows among its 8 that pass the query's filter (bit i: row pos0 + i for i < 4,
// pos0 + 12 + i for i >= 4 -- rows 4 kq + i and 16 + 4 kq + i - 4 of the group)
struct RsRec {
  f32x4 c0, c1;
  int pos0, q;
};

__device__ __forceinline__ RsRec rs_rec_load(const int4* __restrict__ r) {
  RsRec v;
  v.c0 = __builtin_bit_cast(f32x4, r[0]);
  v.c1 = __builtin_bit_cast(f32x4, r[1]);
  const int4 m = r[2];
  v.pos0 = m.x;
  v.q = m.y;
  return v;
}

__device__ __forceinline__ int rs_rec_row(int pos0, int i) { return pos0 + (i < 4 ? i : 12 + i); }

template <int METRIC>
__device__ __forceinline__ unsigned rs_rec_hits(const RsRec& r, const float4& h, const float* __restrict__ row_norms,
                                                float (&xn)[8]) {
  const float mm = METRIC == kL2 ? -2.0f * h.x : -h.x;
  // the record's rows are pos0 .. pos0 + 3 and pos0 + 16 .. + 19 (pos0 = 32 g + 4 kq): two 16-B loads
  const float4 n0 = *reinterpret_cast<const float4*>(row_norms + r.pos0);
  const float4 n1 = *reinterpret_cast<const float4*>(row_norms + r.pos0 + 16);
  xn[0] = n0.x; xn[1] = n0.y; xn[2] = n0.z; xn[3] = n0.w;
  xn[4] = n1.x; xn[5] = n1.y; xn[6] = n1.z; xn[7] = n1.w;
  unsigned m = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const float c = i < 4 ? r.c0[i] : r.c1[i - 4];
    const float xv = METRIC == kL2 ? xn[i] : 0.0f;
    m |= (fmaf(c, mm, xv) < h.y ? 1u : 0u) << i;
  }
  return m;
}

template <int METRIC>
__device__ __forceinline__ void rs_rec_emit(const RsRec& r, unsigned m, const float4& h, const float (&xn)[8], int at,
                                            float* __restrict__ key, int* __restrict__ pos) {
#pragma unroll
  for (int i = 0; i < 8; ++i)
    if (m & (1u << i)) {
      const float c = i < 4 ? r.c0[i] : r.c1[i - 4];
      key[at] = pf_key<METRIC>(c, h.x, xn[i], h.z);
      pos[at] = rs_rec_row(r.pos0, i);
      ++at;
    }
}

// The bucketing with an LDS histogram per group of streams. Group b holds the streams of J K13
// workgroups of one item queue (x = b % 8, workgroups x + 8 (J (b / 8) + t), t < J). Those workgroups take
// consecutive items of the same lists, so their hits fall on the same lists' queries: one global atomic per
// (group, query) with a hit instead of one per candidate (the round-2 flat kernels: 329 -> 119 us per step).
// The group's records are one flat index space (a stream's ~100 records would leave most of a 1024-thread
// block idle if the streams were walked one after another): record e of the group is record e - pre[t] of
// its stream t, found in an LDS prefix of the kRsWaves * J stream lengths.
constexpr int kRsLdsMaxQ = 32768;  // 128 KiB of int bins
constexpr int kRsMaxGroupStreams = 64;
__device__ __forceinline__ int rs_group_stream(int b, int t, int J) {
  return ((b & 7) + 8 * (J * (b >> 3) + t / kRsWaves)) * kRsWaves + t % kRsWaves;
}

// the group's stream prefix in LDS (pre[0..S], S = kRsWaves * J); returns the group's record count
__device__ __forceinline__ int rs_group_prefix(const int* __restrict__ wave_cnt, int wave_cap, int J, int* pre) {
  const int S = kRsWaves * J;
  if (threadIdx.x < 64) {
    const int t = threadIdx.x;
    int n = t < S ? min(wave_cnt[rs_group_stream(blockIdx.x, t, J)], wave_cap) : 0;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(n, o);
      if (t >= o) n += y;
    }
    if (t < S) pre[t + 1] = n;
    if (t == 0) pre[0] = 0;
  }
  __syncthreads();
  return pre[S];
}

// record e of the group: its stream's base pointer
__device__ __forceinline__ const int4* rs_group_rec(const int4* __restrict__ wave_buf, int wave_cap, int J,
                                                    const int* pre, int e) {
  const int S = kRsWaves * J;
  int t = 0;
  while (t + 1 < S && pre[t + 1] <= e) ++t;  // (S <= 64: a short scan of LDS-resident prefixes)
  const int w = rs_group_stream(blockIdx.x, t, J);
  return wave_buf + ((int64_t)w * wave_cap + (e - pre[t])) * kRsRecInt4;
}

template <int METRIC>
__device__ __forceinline__ int rs_group_hist(const int4* __restrict__ wave_buf, int wave_cap,
                                             const int* __restrict__ wave_cnt, int J, int nq,
                                             const float4* __restrict__ qhdr, const float* __restrict__ row_norms,
                                             int* bins, int* pre) {
  for (int i = threadIdx.x; i < nq; i += blockDim.x) bins[i] = 0;
  const int n = rs_group_prefix(wave_cnt, wave_cap, J, pre);  // (its barrier also orders the zeroing)
  // two records per thread and round, their loads issued together (a record, then its header and row norms: two
  // dependent memory rounds each)
  for (int e0 = threadIdx.x; e0 < n; e0 += 2 * blockDim.x) {
    RsRec r[2];
    float4 h[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int e = e0 + u * (int)blockDim.x;
      r[u] = rs_rec_load(rs_group_rec(wave_buf, wave_cap, J, pre, e < n ? e : e0));
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) h[u] = qhdr[r[u].q];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      float xn[8];
      const unsigned m = rs_rec_hits<METRIC>(r[u], h[u], row_norms, xn);
      if (m && e0 + u * (int)blockDim.x < n) atomicAdd(bins + r[u].q, __popc(m));
    }
  }
  __syncthreads();
  return n;
}

template <int METRIC>
__global__ __launch_bounds__(1024) void k_rs_count_lds(const int4* __restrict__ wave_buf, int wave_cap,
                                                       const int* __restrict__ wave_cnt, int J, int nq,
                                                       const float4* __restrict__ qhdr, const float* __restrict__ row_norms,
                                                       unsigned long long* __restrict__ qcnt) {
  extern __shared__ int bins[];
  __shared__ int pre[kRsMaxGroupStreams + 1];
  rs_group_hist<METRIC>(wave_buf, wave_cap, wave_cnt, J, nq, qhdr, row_norms, bins, pre);
  for (int i = threadIdx.x; i < nq; i += blockDim.x) {
    const int c = bins[i];
    if (c) atomicAdd(qcnt + i, (unsigned long long)c);
  }
}

template <int METRIC>
__global__ __launch_bounds__(1024) void k_rs_scatter_lds(const int4* __restrict__ wave_buf, int wave_cap,
                                                         const int* __restrict__ wave_cnt, int J, int nq,
                                                         const float4* __restrict__ qhdr,
                                                         const float* __restrict__ row_norms,
                                                         const int64_t* __restrict__ off, int* __restrict__ fill,
                                                         float* __restrict__ key, int* __restrict__ pos) {
  extern __shared__ int bins[];
  __shared__ int pre[kRsMaxGroupStreams + 1];
  const int n = rs_group_hist<METRIC>(wave_buf, wave_cap, wave_cnt, J, nq, qhdr, row_norms, bins, pre);
  // this group's range of each query's run (< 2^31 entries in all: fits an int)
  for (int i = threadIdx.x; i < nq; i += blockDim.x) {
    const int c = bins[i];
    if (c) bins[i] = (int)(off[i] + atomicAdd(fill + i, c));
  }
  __syncthreads();
  for (int e = threadIdx.x; e < n; e += blockDim.x) {
    const RsRec r = rs_rec_load(rs_group_rec(wave_buf, wave_cap, J, pre, e));
    const float4 h = qhdr[r.q];
    float xn[8];
    const unsigned m = rs_rec_hits<METRIC>(r, h, row_norms, xn);
    if (m) rs_rec_emit<METRIC>(r, m, h, xn, atomicAdd(bins + r.q, __popc(m)), key, pos);
  }
}

// The one-pass bucketing (k <= 16): the group's LDS histogram, then ONE global atomic per (group, query) that reserves
// the group's range inside the query's fixed-capacity run, then the scatter -- the count kernel, the scan over the
// queries and the second pass over the records of the two-pass form are gone (K11 reads the runs by count).
template <int METRIC>
__global__ __launch_bounds__(1024) void k_rs_bucket_fused(const int4* __restrict__ wave_buf, int wave_cap,
                                                          const int* __restrict__ wave_cnt, int J, int nq,
                                                          const float4* __restrict__ qhdr,
                                                          const float* __restrict__ row_norms, int cap,
                                                          int* __restrict__ qcnt, float* __restrict__ key,
                                                          int* __restrict__ pos) {
  extern __shared__ int bins[];
  __shared__ int pre[kRsMaxGroupStreams + 1];
  const int n = rs_group_hist<METRIC>(wave_buf, wave_cap, wave_cnt, J, nq, qhdr, row_norms, bins, pre);
  // the group's first entry in each query's run: eight returning atomics in flight per thread (one after another,
  // each waited for its L2 round trip)
  constexpr int U = 8;
  for (int i0 = threadIdx.x; i0 < nq; i0 += U * (int)blockDim.x) {
    int c[U], at[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + u * (int)blockDim.x;
      c[u] = i < nq ? bins[i] : 0;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) at[u] = c[u] ? atomicAdd(qcnt + i0 + u * (int)blockDim.x, c[u]) : 0;
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (c[u]) bins[i0 + u * (int)blockDim.x] = at[u];
  }
  __syncthreads();
  for (int e0 = threadIdx.x; e0 < n; e0 += 2 * blockDim.x) {
    RsRec r[2];
    float4 h[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int e = e0 + u * (int)blockDim.x;
      r[u] = rs_rec_load(rs_group_rec(wave_buf, wave_cap, J, pre, e < n ? e : e0));
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) h[u] = qhdr[r[u].q];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (e0 + u * (int)blockDim.x >= n) continue;
      float xn[8];
      const unsigned m = rs_rec_hits<METRIC>(r[u], h[u], row_norms, xn);
      if (!m) continue;
      int at = atomicAdd(bins + r[u].q, __popc(m));
      const int64_t base = (int64_t)r[u].q * cap;
#pragma unroll
      for (int i = 0; i < 8; ++i)
        if (m & (1u << i)) {
          if (at < cap) {
            const float c = i < 4 ? r[u].c0[i] : r[u].c1[i - 4];
            key[base + at] = pf_key<METRIC>(c, h[u].x, xn[i], h[u].z);
            pos[base + at] = rs_rec_row(r[u].pos0, i);
          }
          ++at;
        }
    }
  }
}

size_t rs_bucket_tmp_bytes(int nq, int n_waves) {
  return sizeof(int64_t) * ((size_t)nq + 1) + sizeof(int) * (size_t)nq + sizeof(int64_t) * ((size_t)n_waves + 1) +
         scan_tmp_bytes(nq + 1) + 64;
}

// J: K13 workgroups per bucketing group (1: one K13 workgroup's 8 streams per LDS histogram; 2 and 4 measured slower
// and were retired in round 5); the streams come from K13's 8 item queues (n_waves = 8 queues x P workgroups x
// kRsWaves) and a batch's bins fit LDS (K13 batches are at most kRsMaxBatch = kRsLdsMaxQ queries)
static int rs_bucket_groups(int n_waves, int nq, int* J_out) {
  const int P = n_waves / (8 * kRsWaves);
  if (!(nq <= kRsLdsMaxQ && n_waves == 8 * kRsWaves * P && P > 0)) return 0;
  *J_out = 1;
  return 8 * P;
}

template <int METRIC>
static hipError_t rs_bucket_count_m(const int4* wave_buf, int wave_cap, const int* wave_cnt, int n_waves, int nq,
                                    const float4* qhdr, const float* row_norms, int64_t* cand_off, int64_t* qcnt,
                                    void* stmp, hipStream_t s) {
  int J = 1;
  const int nb = rs_bucket_groups(n_waves, nq, &J);
  if (nb == 0) return hipErrorInvalidValue;
  static const hipError_t a1 = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_rs_count_lds<METRIC>),
                                                   hipFuncAttributeMaxDynamicSharedMemorySize,
                                                   (int)(sizeof(int) * kRsLdsMaxQ));
  if (a1 != hipSuccess) return a1;
  hipLaunchKernelGGL(k_rs_count_lds<METRIC>, dim3((unsigned)nb), dim3(1024), sizeof(int) * (size_t)nq, s, wave_buf,
                     wave_cap, wave_cnt, J, nq, qhdr, row_norms, reinterpret_cast<unsigned long long*>(qcnt));
  return launch_exclusive_scan_i64(qcnt, cand_off, nq + 1, stmp, s);
}

template <int METRIC>
static hipError_t rs_bucket_scatter_m(const int4* wave_buf, int wave_cap, const int* wave_cnt, int n_waves, int nq,
                                      const float4* qhdr, const float* row_norms, const int64_t* cand_off,
                                      float* cand_key, int* cand_pos, int* fill, hipStream_t s) {
  int J = 1;
  const int nb = rs_bucket_groups(n_waves, nq, &J);
  if (nb == 0) return hipErrorInvalidValue;
  static const hipError_t a2 = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_rs_scatter_lds<METRIC>),
                                                   hipFuncAttributeMaxDynamicSharedMemorySize,
                                                   (int)(sizeof(int) * kRsLdsMaxQ));
  if (a2 != hipSuccess) return a2;
  hipLaunchKernelGGL(k_rs_scatter_lds<METRIC>, dim3((unsigned)nb), dim3(1024), sizeof(int) * (size_t)nq, s, wave_buf,
                     wave_cap, wave_cnt, J, nq, qhdr, row_norms, cand_off, fill, cand_key, cand_pos);
  return hipGetLastError();
}

// the temporaries of the bucketing inside tmp: qcnt [nq + 1], fill [nq], woff [n_waves + 1], the scan's
struct RsBucketTmp {
  int64_t* qcnt;
  int* fill;
  int64_t* woff;
  void* stmp;
};
static RsBucketTmp rs_bucket_tmp(void* tmp, int nq, int n_waves) {
  RsBucketTmp t;
  t.qcnt = static_cast<int64_t*>(tmp);
  t.fill = reinterpret_cast<int*>(t.qcnt + nq + 1);
  t.woff = reinterpret_cast<int64_t*>(
      reinterpret_cast<char*>(tmp) + ((sizeof(int64_t) * ((size_t)nq + 1) + sizeof(int) * (size_t)nq + 15) & ~(size_t)15));
  t.stmp = reinterpret_cast<char*>(t.woff) + ((sizeof(int64_t) * ((size_t)n_waves + 1) + 15) & ~(size_t)15);
  return t;
}

hipError_t launch_rs_bucket_fused(const int4* wave_buf, int wave_cap, const int* wave_cnt, int n_waves, int nq,
                                  const float4* qhdr, const float* row_norms, int metric, int cap, int* qcnt,
                                  float* cand_key, int* cand_pos, hipStream_t s) {
  if (n_waves <= 0 || nq <= 0) return hipSuccess;
  if (cap < 1 || (int64_t)cap * nq > INT64_C(1) << 40) return hipErrorInvalidValue;
  int J = 1;
  const int nb = rs_bucket_groups(n_waves, nq, &J);
  if (nb == 0) return hipErrorInvalidValue;
  const size_t lds = sizeof(int) * (size_t)nq;
  if (metric == kIP) {
    static const hipError_t a1 = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_rs_bucket_fused<kIP>),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize,
                                                     (int)(sizeof(int) * kRsLdsMaxQ));
    if (a1 != hipSuccess) return a1;
    hipLaunchKernelGGL(k_rs_bucket_fused<kIP>, dim3((unsigned)nb), dim3(1024), lds, s, wave_buf, wave_cap, wave_cnt, J,
                       nq, qhdr, row_norms, cap, qcnt, cand_key, cand_pos);
  } else {
    static const hipError_t a2 = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_rs_bucket_fused<kL2>),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize,
                                                     (int)(sizeof(int) * kRsLdsMaxQ));
    if (a2 != hipSuccess) return a2;
    hipLaunchKernelGGL(k_rs_bucket_fused<kL2>, dim3((unsigned)nb), dim3(1024), lds, s, wave_buf, wave_cap, wave_cnt, J,
                       nq, qhdr, row_norms, cap, qcnt, cand_key, cand_pos);
  }
  return hipGetLastError();
}

hipError_t launch_rs_bucket_count(const int4* wave_buf, int wave_cap, const int* wave_cnt, int n_waves, int nq,
                                  const float4* qhdr, const float* row_norms, int metric, int64_t* cand_off, void* tmp,
                                  int* lost, hipStream_t s, void* zero2, int zero2_bytes) {
  const RsBucketTmp t = rs_bucket_tmp(tmp, nq, n_waves);
  if (zero2_bytes % 16 != 0 || zero2_bytes > 16 * 1024 || (reinterpret_cast<uintptr_t>(zero2) & 15) != 0)
    return hipErrorInvalidValue;
  // qcnt [nq + 1] and fill [nq], rounded up to the 16-B boundary where woff starts (rs_bucket_tmp)
  const size_t zbytes = reinterpret_cast<char*>(t.woff) - reinterpret_cast<char*>(t.qcnt);
  if (n_waves <= 0) {
    hipError_t e = hipMemsetAsync(t.qcnt, 0, zbytes, s);
    if (e == hipSuccess && zero2_bytes > 0) e = hipMemsetAsync(zero2, 0, zero2_bytes, s);
    if (e != hipSuccess) return e;
    return launch_exclusive_scan_i64(t.qcnt, cand_off, nq + 1, t.stmp, s);
  }
  if ((reinterpret_cast<uintptr_t>(t.qcnt) & 15) != 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_rs_stream_off, dim3(1), dim3(1024), 0, s, wave_cnt, n_waves, wave_cap, t.woff, lost,
                     reinterpret_cast<int4*>(t.qcnt), (int64_t)(zbytes / 16), static_cast<int4*>(zero2), zero2_bytes / 16);
  return metric == kIP ? rs_bucket_count_m<kIP>(wave_buf, wave_cap, wave_cnt, n_waves, nq, qhdr, row_norms, cand_off,
                                                t.qcnt, t.stmp, s)
                       : rs_bucket_count_m<kL2>(wave_buf, wave_cap, wave_cnt, n_waves, nq, qhdr, row_norms, cand_off,
                                                t.qcnt, t.stmp, s);
}

hipError_t launch_rs_bucket_scatter(const int4* wave_buf, int wave_cap, const int* wave_cnt, int n_waves, int nq,
                                    const float4* qhdr, const float* row_norms, int metric, const int64_t* cand_off,
                                    float* cand_key, int* cand_pos, void* tmp, hipStream_t s) {
  if (n_waves <= 0) return hipSuccess;
  const RsBucketTmp t = rs_bucket_tmp(tmp, nq, n_waves);
  return metric == kIP ? rs_bucket_scatter_m<kIP>(wave_buf, wave_cap, wave_cnt, n_waves, nq, qhdr, row_norms, cand_off,
                                                  cand_key, cand_pos, t.fill, s)
                       : rs_bucket_scatter_m<kL2>(wave_buf, wave_cap, wave_cnt, n_waves, nq, qhdr, row_norms, cand_off,
                                                  cand_key, cand_pos, t.fill, s);
}

hipError_t launch_rs_bucket(const int4* wave_buf, int wave_cap, const int* wave_cnt, int n_waves, int nq,
                            const float4* qhdr, const float* row_norms, int metric, int64_t* cand_off,
                            float* cand_key, int* cand_pos, void* tmp, int* lost, int grid, hipStream_t s,
                            void* zero2, int zero2_bytes) {
  (void)grid;
  hipError_t e = launch_rs_bucket_count(wave_buf, wave_cap, wave_cnt, n_waves, nq, qhdr, row_norms, metric, cand_off,
                                        tmp, lost, s, zero2, zero2_bytes);
  if (e != hipSuccess) return e;
  return launch_rs_bucket_scatter(wave_buf, wave_cap, wave_cnt, n_waves, nq, qhdr, row_norms, metric, cand_off,
                                  cand_key, cand_pos, tmp, s);
}

// the smallest row norm of every group (K13's filter bound; pad rows are +inf, every group has a real row)
__global__ void k_group_nmin(const float* __restrict__ norms, int64_t n_groups, float* __restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t g = t >> 5;
  float m = g < n_groups ? norms[t] : INFINITY;
#pragma unroll
  for (int off = 16; off >= 1; off >>= 1) m = fminf(m, __shfl_xor(m, off));
  if (g < n_groups && (t & 31) == 0) out[g] = m;
}

hipError_t launch_group_nmin(const float* norms, int64_t n_groups, float* out, hipStream_t s) {
  if (n_groups <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_group_nmin, dim3((unsigned)ceil_div(n_groups * 32, 256)), dim3(256), 0, s, norms, n_groups, out);
  return hipGetLastError();
}

// The pre-pass's lists: list l split into 2l = its first ceil(groups / div) groups (at least min_groups,
// at most all) and 2l + 1 = the rest, so the n_probes = 1 search of probe 2 p0 scans a sample of the
// nearest list p0 with the unchanged K10 / probe map (the sample's rows are still rows of the probed
// lists, so its k-th exact key bounds the final k-th from above)
__global__ void k_rs_pre_lists(const int64_t* __restrict__ goff, int n_lists, int div, int min_groups,
                               int64_t* __restrict__ goff2, const int64_t* __restrict__ probes, int64_t nq, int np,
                               int64_t* __restrict__ probes2) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  // every probe of the batch's queries -> the sample list of its nearest probe (2 p0); -1 (no probe) stays -1
  if (t < nq) {
    const int64_t p = probes[t * np];
    probes2[t] = p < 0 ? p : 2 * p;
  }
  if (t > n_lists) return;
  const int l = (int)t;
  const int64_t b = goff[l];
  goff2[2 * l] = b;
  if (l == n_lists) return;
  const int64_t ng = goff[l + 1] - b;
  int64_t m = (ng + div - 1) / div;
  m = m < min_groups ? min_groups : m;
  goff2[2 * l + 1] = b + (m < ng ? m : ng);
}

hipError_t launch_rs_pre_lists(const int64_t* goff, int n_lists, int div, int min_groups, const int64_t* probes,
                               int64_t nq, int np, int64_t* goff2, int64_t* probes2, hipStream_t s) {
  if (div < 1 || min_groups < 1) return hipErrorInvalidValue;
  const int64_t n = nq > n_lists + 1 ? nq : n_lists + 1;  // (one launch for the split offsets and the probes)
  hipLaunchKernelGGL(k_rs_pre_lists, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, s, goff, n_lists, div, min_groups,
                     goff2, probes, nq, np, probes2);
  return hipGetLastError();
}

hipError_t launch_rs_headers(const float* pre_kth, int64_t nq, const float* qscale, const float* qnorms,
                             const float* qres, float x_norm_max, float x_res_max, int dp, int metric, float4* hdr,
                             float* tq, hipStream_t s, int* zero, int64_t nzero, int* zero2, int nzero2) {
  if (nzero > nq + 1 || nzero2 > 256) return hipErrorInvalidValue;  // (the grid has >= max(nq + 1, 256) threads)
  const dim3 grid((unsigned)ceil_div(nq + 1, 256));
  if (metric == kIP)
    hipLaunchKernelGGL(k_rs_headers<kIP>, grid, dim3(256), 0, s, pre_kth, nq, qscale, qnorms, qres, x_norm_max,
                       x_res_max, dp, hdr, tq, zero, nzero, zero2, nzero2);
  else
    hipLaunchKernelGGL(k_rs_headers<kL2>, grid, dim3(256), 0, s, pre_kth, nq, qscale, qnorms, qres, x_norm_max,
                       x_res_max, dp, hdr, tq, zero, nzero, zero2, nzero2);
  return hipGetLastError();
}

}  // namespace mivs
