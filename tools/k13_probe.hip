// K13 k-loop probe (tools/, not part of the product): what the row-stationary loop shape of k_rs_scan can
// sustain on its own, without the search around it. Each wave holds 32 fp16 rows x 768 dims in registers
// (48 x h8 = 192 VGPRs) and runs 32-query tiles from LDS through v_mfma_f32_16x16x32_f16 (one ds_read_b128
// per two MFMAs, B read PD k-steps ahead), as K13 does. Variants (VAR bits):
//   1  per-tile all-wave sync through an LDS counter (K13's rs_spin / rs_signal)
//   2  LDS-DMA staging of the next tile (6-7 pieces of 1 KiB per wave per tile, L2-resident source)
//   4  the common-case epilogue (16 fmax + 2 fma + ballot) instead of a plain fold
//   8  items of 10 tiles: the next item's rows (48 KiB per wave) loaded from a large HBM buffer during an
//      item's last tile, waited for at the next item's start (K13's item transition)
//   16 tile images from a 540 MB pool (11k tiles, HBM/MALL): the 32 blocks of one XCD walk one range of it
//      together, as the items of one list do (otherwise 64 L2-resident tiles)
//   2048 three tile buffers and two counters instead of one: a wave signals 'my pieces of tile t + 1 landed' at
//      k-step LANDED_AT of tile t (after a vmcnt wait) and 'done reading tile t' after its k-loop; it starts tile t + 1
//      once every wave's pieces landed, and issues its pieces of tile t + 2 (into the buffer of tile t - 1) once every
//      wave is done with tile t - 1 -- waves may drift up to about a tile apart instead of meeting at every tile
//   1024 the query pieces gathered straight from a [10k][768] fp16 query array (lane (c, kq) of piece 2 t + qb reads
//      16 B of query id(16 qb + c) at dims 32 t + 8 kq; ids spread pseudo-randomly over the 15 MB array) instead of
//      copied from a prebuilt tile image; the header piece still from the image
//   8192 (with 8) the first PF_P row registers of the next item (PF_P = 7, or 4 with 16384) LDS-DMA'd into a spare
//      56 KiB of LDS during the item's tiles 1..PF_P, one register per wave per tile, and read from LDS (not HBM) at
//      the item transition: the transition's HBM intake shrinks by PF_P / 48
// Reports TF/s, the in-kernel clock (s_memtime / s_memrealtime) and the MFMA pipe's busy fraction.
// Build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off tools/k13_probe.hip -o tools/k13_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int v4i __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                             \
  do {                                                                                       \
    hipError_t e_ = (x);                                                                     \
    if (e_ != hipSuccess) {                                                                  \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__);          \
      return 1;                                                                              \
    }                                                                                        \
  } while (0)

constexpr int NK = 48;
constexpr int BUF = NK * 1024 + 1024;
constexpr int kQ = 10000;  // queries in the VAR & 1024 query array

__device__ __forceinline__ v4i uniform_desc(const void* p, int bytes) {
  const uint64_t v = reinterpret_cast<uint64_t>(p);
  v4i r;
  r.x = (int)__builtin_amdgcn_readfirstlane((uint32_t)v);
  r.y = (int)(__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) & 0xFFFFu);
  r.z = __builtin_amdgcn_readfirstlane(bytes);
  r.w = 0x00020000;
  return r;
}

__device__ __forceinline__ void dma_b128(v4i desc, const void* lds, int voff, int soff) {
  const uint32_t m0 = __builtin_amdgcn_readfirstlane((uint32_t)reinterpret_cast<uintptr_t>(lds));
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
               :: "s"(m0), "v"(voff), "s"(desc), "s"(soff) : "memory");
}

template <bool B>
struct BoolC {
  static constexpr bool value = B;
};
template <int I>
struct IntC {
  static constexpr int value = I;
};

template <int VAR, int PD, int WAVES>
__global__ __launch_bounds__(WAVES * 64, 1) void probe(const h8* __restrict__ rows, const char* __restrict__ src,
                                                       int src_tiles, int ntiles, float* out,
                                                       unsigned long long* clk, const h8* __restrict__ big_rows,
                                                       long long big_items, const char* __restrict__ qarr) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NBUF = (VAR & 2048) ? 3 : 2;
  constexpr int LANDED_AT = (VAR & 4096) ? 16 : 40;  // (4096: the landed signal early, so waves may lag ~2/3 tile)
  int* s_ready = reinterpret_cast<int*>(smem + NBUF * BUF);
  int* s_done = s_ready + 1;
  constexpr int PF_P = (VAR & 16384) ? 4 : 7;
  char* s_pf = smem + NBUF * BUF + 64;  // [WAVES][PF_P] x 1 KiB (VAR & 8192)
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const v4i qdesc = uniform_desc(qarr, kQ * NK * 32);
  for (int i = tid; i < NBUF * BUF / 16; i += WAVES * 64) {
    const int v = (i * 2654435761u) >> 7;
    reinterpret_cast<uint4*>(smem)[i] = make_uint4(v & 0x3BFF3BFF, (v >> 3) & 0x3BFF3BFF, v & 0x37FF37FF, 0x3C003C00 ^ (v & 0x03FF03FF));
  }
  if (tid == 0) { *s_ready = 0; *s_done = 0; }
  __syncthreads();
  h8 ra[NK];
  const h8* rp = rows + ((size_t)(blockIdx.x * WAVES + wave) * NK) * 64 + lane;
#pragma unroll
  for (int s = 0; s < NK; ++s) ra[s] = rp[s * 64];
  const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  float sink = 0.f;
  int cur = 0;
  const f32x4 z = {0.f, 0.f, 0.f, 0.f};
  if (VAR & 1) {
    if (lane == 0) __hip_atomic_fetch_add(s_ready, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  // VAR & 4096 (with 2048): waves 4..7 start about half a k-loop late, so each SIMD's two waves run their epilogues
  // and waits under each other's MFMAs
  if ((VAR & 4096) && wave >= 4) {
    for (int i = 0; i < 24; ++i) __builtin_amdgcn_s_sleep(1);
  }
  // VAR & 32: staggered item transitions -- wave w reloads in the tiles t with (t + o_w) % 10 == 9, o_w spread over
  // the 10 tiles of an item (SIMD partners w, w + 4 five tiles apart; VAR & 64: two phases only, waves 4-7 at 5).
  // The reload tile and the tile after it are one straight-line pair, so the compiler's counted vmcnt before each
  // MFMA of the second waits only for the registers it reads.
  const int o_w = (VAR & 64) ? (wave >= 4 ? 5 : 0) : (wave < 4 ? wave : wave + 1);
  auto tile = [&](int t, auto rl_c, auto after_c) __attribute__((always_inline)) {
    constexpr bool RL = decltype(rl_c)::value;
    constexpr bool AFTER = decltype(after_c)::value;
    if (VAR & 1) {
      for (int i = 0; i < (1 << 20); ++i) {
        if (__hip_atomic_load(s_ready, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= WAVES * (t + 1)) break;
        __builtin_amdgcn_s_sleep(1);
      }
      asm volatile("" ::: "memory");
    }
    const char* bb = smem + cur * BUF + lane * 16;
    const int nxt = cur + 1 == NBUF ? 0 : cur + 1;
    char* sbuf = smem + nxt * BUF;
    const int tsrc = (VAR & 16) ? (int)(((blockIdx.x & 7) * 1375 + t + 1) % src_tiles) : (int)((blockIdx.x + t) % src_tiles);
    const v4i sdesc = uniform_desc(src + (size_t)tsrc * (NK + 1) * 1024, (NK + 1) * 1024);
    // VAR & 1024: the tile's query ids -> per-lane byte offsets into the query array (qb = 0, 1)
    const int c = lane & 15;
    const int gq0 = (int)(((long long)(tsrc * 32 + c) * 7919) % kQ), gq1 = (int)(((long long)(tsrc * 32 + 16 + c) * 7919) % kQ);
    const int qo0 = gq0 * (NK * 32) + (lane >> 4) * 16, qo1 = gq1 * (NK * 32) + (lane >> 4) * 16;
    const h8* nr = big_rows + ((size_t)(((long long)blockIdx.x * 7919 + t * 131) % big_items) * WAVES + wave) * NK * 64 + lane;
    // VAR & 8192: this item's reload tile t9 and the next item's rows of this wave (the same address as nr there)
    const int t9 = t - t % 10 + 9;
    const h8* nr9 = big_rows + ((size_t)(((long long)blockIdx.x * 7919 + t9 * 131) % big_items) * WAVES + wave) * NK * 64;
    const int pf_p = t % 10 - 1;  // the register prefetched in this tile (tiles 1 .. PF_P of an item)
    const v4i pdesc = uniform_desc(nr9, NK * 1024);
    if (!(VAR & 32) && (VAR & 8) && t % 10 == 0) __builtin_amdgcn_s_waitcnt(0x0070);
    f32x4 acc[4] = {z, z, z, z};
    h8 b[PD + 1];
#pragma unroll
    for (int u = 0; u < PD; ++u) b[u] = *reinterpret_cast<const h8*>(bb + u * 1024);
#pragma unroll
    for (int s = 0; s < NK; ++s) {
      if (s + PD < NK) b[(s + PD) % (PD + 1)] = *reinterpret_cast<const h8*>(bb + (s + PD) * 1024);
      const int t2 = 2 * (s >> 1), qb = s & 1;
      acc[2 * qb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ra[t2], b[s % (PD + 1)], acc[2 * qb], 0, 0, 0);
      acc[2 * qb + 1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ra[t2 + 1], b[s % (PD + 1)], acc[2 * qb + 1], 0, 0, 0);
      if (RL && (s & 1)) {
        if (VAR & 128) {  // (timing only) loads the compiler does not see: no waits for them anywhere
          asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(ra[s - 1]) : "v"(nr + (s - 1) * 64) : "memory");
          asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(ra[s]) : "v"(nr + s * 64) : "memory");
        } else if ((VAR & 8192) && s - 1 < PF_P) {  // prefetched registers from LDS
          ra[s - 1] = *reinterpret_cast<const h8*>(s_pf + (wave * PF_P + s - 1) * 1024 + lane * 16);
          if (s < PF_P) ra[s] = *reinterpret_cast<const h8*>(s_pf + (wave * PF_P + s) * 1024 + lane * 16);
          else ra[s] = __builtin_nontemporal_load(nr + s * 64);
        } else if (VAR & 256) {  // non-temporal policy (K13's rows: aux = 2)
          ra[s - 1] = __builtin_nontemporal_load(nr + (s - 1) * 64);
          ra[s] = __builtin_nontemporal_load(nr + s * 64);
        } else {
          ra[s - 1] = nr[(s - 1) * 64];
          ra[s] = nr[s * 64];
        }
      }
      if ((VAR & 2048) && s == 1 && t >= 2) {  // the buffer of tile t - 1 is free once every wave is done with it
        for (int i = 0; i < (1 << 20); ++i) {
          if (__hip_atomic_load(s_done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= WAVES * (t - 1)) break;
          __builtin_amdgcn_s_sleep(1);
        }
        asm volatile("" ::: "memory");
      }
      if ((VAR & 2048) && s == LANDED_AT) {  // this wave's pieces of tile t + 1 have landed
        __builtin_amdgcn_s_waitcnt(0x0070);
        asm volatile("" ::: "memory");
        if (lane == 0) __hip_atomic_fetch_add(s_ready, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      if (VAR & 2) {
        if (s >= 1 && (s - 1) * WAVES <= NK) {
          const int p = min((s - 1) * WAVES + wave, NK);
          if ((VAR & 1024) && p < NK) dma_b128(qdesc, sbuf + p * 1024, (p & 1) ? qo1 : qo0, 64 * (p >> 1));
          else dma_b128(sdesc, sbuf + p * 1024, lane * 16, p * 1024);
        }
      }
      if ((VAR & 8192) && s == 24 && pf_p >= 0 && pf_p < PF_P)
        dma_b128(pdesc, s_pf + (wave * PF_P + pf_p) * 1024, lane * 16, pf_p * 1024);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (VAR & 32) {
      // the reload tile: wait for the DMA pieces only (38 row loads issued after the last piece may stay in flight)
      if (RL) __builtin_amdgcn_s_waitcnt((38 & 15) | (0x7 << 4) | ((38 >> 4) << 14));
      else if (VAR & 2) __builtin_amdgcn_s_waitcnt(0x0070);
    } else {
      if ((VAR & 2) && !RL) __builtin_amdgcn_s_waitcnt(0x0070);
      if ((VAR & 2) && RL) __builtin_amdgcn_s_waitcnt(0x0070);  // (conservative: rows too)
    }
    (void)AFTER;
    if (VAR & 2048) {  // done reading tile t (the k-loop's B reads are in: lgkmcnt(0))
      __builtin_amdgcn_s_waitcnt(0xC07F);
      asm volatile("" ::: "memory");
      if (lane == 0) __hip_atomic_fetch_add(s_done, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    } else if (VAR & 1) {
      asm volatile("" ::: "memory");
      if (lane == 0) __hip_atomic_fetch_add(s_ready, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    if (VAR & 4) {
      float am0 = fmaxf(acc[0][0], acc[1][0]), am1 = fmaxf(acc[2][0], acc[3][0]);
#pragma unroll
      for (int i = 1; i < 4; ++i) {
        am0 = fmaxf(am0, fmaxf(acc[0][i], acc[1][i]));
        am1 = fmaxf(am1, fmaxf(acc[2][i], acc[3][i]));
      }
      if (__ballot(fmaf(am0, -2.f, 0.5f) < -1e30f || fmaf(am1, -2.f, 0.5f) < -1e30f)) sink += 1.f;
      sink += am0 * 1e-30f;
    } else {
      sink += acc[0][0] + acc[1][1] + acc[2][2] + acc[3][3];
    }
    cur = nxt;
  };
  for (int t = 0; t < ntiles;) {
    if ((VAR & 32) && (VAR & 512)) {  // stagger, one loop: the reload tile is NOT paired with the next
      if ((VAR & 8) && (t + o_w) % 10 == 9) tile(t, BoolC<true>{}, BoolC<false>{});
      else tile(t, BoolC<false>{}, BoolC<false>{});
      t += 1;
    } else if (VAR & 32) {
      if ((VAR & 8) && (t + o_w) % 10 == 9 && t + 1 < ntiles) {
        tile(t, BoolC<true>{}, BoolC<false>{});
        tile(t + 1, BoolC<false>{}, BoolC<true>{});
        t += 2;
      } else {
        tile(t, BoolC<false>{}, BoolC<false>{});
        t += 1;
      }
    } else {
      if ((VAR & 8) && t % 10 == 9) tile(t, BoolC<true>{}, BoolC<false>{});
      else tile(t, BoolC<false>{}, BoolC<false>{});
      t += 1;
    }
  }
  __builtin_amdgcn_s_waitcnt(0x0070);
  const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (lane == 0 && wave == 0) {
    clk[2 * blockIdx.x] = t1 - t0;
    clk[2 * blockIdx.x + 1] = r1 - r0;
  }
  out[(size_t)(blockIdx.x * WAVES + wave) * 64 + lane] = sink;
}

// 16-row waves with a double-buffered row set (VERDICT r04 item 1's candidate): each wave keeps 16 rows (24 A registers,
// 96 VGPRs) and loads the next item's 16 rows into another 24 registers three per tile over the item's first eight
// tiles (loads the compiler does not see, waited for once at the item boundary); a 32-query tile is then two B pieces
// per 32 dims, one MFMA each. The 8 waves of a workgroup hold 128 rows. VAR bits as probe's: 1 sync, 2 dma, 4 epi,
// 8 items of 10 tiles, 16 hbm tiles.
template <int VAR>
__global__ __launch_bounds__(512, 1) void probe16(const h8* __restrict__ rows, const char* __restrict__ src,
                                                  int src_tiles, int ntiles, float* out, unsigned long long* clk,
                                                  const h8* __restrict__ big_rows, long long big_items) {
  constexpr int WAVES = 8, PD = 2, NR = NK / 2;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int* s_ready = reinterpret_cast<int*>(smem + 2 * BUF);
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  for (int i = tid; i < 2 * BUF / 16; i += WAVES * 64) {
    const int v = (i * 2654435761u) >> 7;
    reinterpret_cast<uint4*>(smem)[i] = make_uint4(v & 0x3BFF3BFF, (v >> 3) & 0x3BFF3BFF, v & 0x37FF37FF, 0x3C003C00 ^ (v & 0x03FF03FF));
  }
  if (tid == 0) *s_ready = 0;
  __syncthreads();
  h8 ra[NR], rn[NR];
  const h8* rp = rows + ((size_t)(blockIdx.x * WAVES + wave) * NR) * 64 + lane;
#pragma unroll
  for (int r = 0; r < NR; ++r) { ra[r] = rp[r * 64]; rn[r] = rp[r * 64]; }
  const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  float sink = 0.f;
  int cur = 0;
  const f32x4 z = {0.f, 0.f, 0.f, 0.f};
  if (VAR & 1) {
    if (lane == 0) __hip_atomic_fetch_add(s_ready, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  auto tile = [&](int t, h8 (&A)[NR], h8 (&N)[NR], auto j_c) __attribute__((always_inline)) {
    constexpr int j = decltype(j_c)::value;  // tile of the item: registers 3j .. 3j + 2 of the next item at j < 8
    if (VAR & 1) {
      for (int i = 0; i < (1 << 20); ++i) {
        if (__hip_atomic_load(s_ready, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= WAVES * (t + 1)) break;
        __builtin_amdgcn_s_sleep(1);
      }
      asm volatile("" ::: "memory");
    }
    if ((VAR & 8) && t % 10 == 0) __builtin_amdgcn_s_waitcnt(0x0070);  // (the item's rows, loaded over its first 8 tiles)
    const char* bb = smem + cur * BUF + lane * 16;
    const int nxt = cur ^ 1;
    char* sbuf = smem + nxt * BUF;
    const int tsrc = (VAR & 16) ? (int)(((blockIdx.x & 7) * 1375 + t + 1) % src_tiles) : (int)((blockIdx.x + t) % src_tiles);
    const v4i sdesc = uniform_desc(src + (size_t)tsrc * (NK + 1) * 1024, (NK + 1) * 1024);
    const h8* nr = big_rows + ((size_t)(((long long)blockIdx.x * 7919 + (t / 10) * 131) % big_items) * WAVES + wave) * NR * 64 + lane;
    f32x4 acc[2] = {z, z};
    h8 b[PD + 1];
#pragma unroll
    for (int u = 0; u < PD; ++u) b[u] = *reinterpret_cast<const h8*>(bb + u * 1024);
#pragma unroll
    for (int s = 0; s < NK; ++s) {
      if (s + PD < NK) b[(s + PD) % (PD + 1)] = *reinterpret_cast<const h8*>(bb + (s + PD) * 1024);
      acc[s & 1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A[s >> 1], b[s % (PD + 1)], acc[s & 1], 0, 0, 0);
      if constexpr ((VAR & 8) && j < 8) {
        if (s == 12 || s == 24 || s == 36) {
          const int r = 3 * j + s / 12 - 1;
          asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(N[r]) : "v"(nr + r * 64) : "memory");
        }
      }
      if (VAR & 2) {
        if (s >= 1 && (s - 1) * WAVES <= NK) {
          const int p = min((s - 1) * WAVES + wave, NK);
          dma_b128(sdesc, sbuf + p * 1024, lane * 16, p * 1024);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if (VAR & 2) __builtin_amdgcn_s_waitcnt(0x0070);
    if (VAR & 1) {
      asm volatile("" ::: "memory");
      if (lane == 0) __hip_atomic_fetch_add(s_ready, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    if (VAR & 4) {
      float am = fmaxf(fmaxf(acc[0][0], acc[0][1]), fmaxf(acc[0][2], acc[0][3]));
      float am1 = fmaxf(fmaxf(acc[1][0], acc[1][1]), fmaxf(acc[1][2], acc[1][3]));
      if (__ballot(fmaf(am, -2.f, 0.5f) < -1e30f || fmaf(am1, -2.f, 0.5f) < -1e30f)) sink += 1.f;
      sink += am * 1e-30f;
    } else {
      sink += acc[0][0] + acc[1][1];
    }
    cur = nxt;
  };
  auto item = [&](int t, h8 (&A)[NR], h8 (&N)[NR]) __attribute__((always_inline)) {
    tile(t + 0, A, N, IntC<0>{}); tile(t + 1, A, N, IntC<1>{}); tile(t + 2, A, N, IntC<2>{});
    tile(t + 3, A, N, IntC<3>{}); tile(t + 4, A, N, IntC<4>{}); tile(t + 5, A, N, IntC<5>{});
    tile(t + 6, A, N, IntC<6>{}); tile(t + 7, A, N, IntC<7>{}); tile(t + 8, A, N, IntC<8>{});
    tile(t + 9, A, N, IntC<9>{});
  };
  for (int t = 0; t + 20 <= ntiles; t += 20) {
    item(t, ra, rn);
    item(t + 10, rn, ra);
  }
  __builtin_amdgcn_s_waitcnt(0x0070);
  const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (lane == 0 && wave == 0) {
    clk[2 * blockIdx.x] = t1 - t0;
    clk[2 * blockIdx.x + 1] = r1 - r0;
  }
  out[(size_t)(blockIdx.x * WAVES + wave) * 64 + lane] = sink;
}

// W4 (round 6): workgroups of 4 waves (one per SIMD) and TWO per CU, 16-query tiles ([NK/2 + 1] x 1 KiB images,
// double-buffered: 50 KiB of LDS per workgroup), items of 20 tiles (a list's ~312 queries), each workgroup's item
// transitions phase-shifted by PHASE tiles against the other's (the real kernel's items differ in length, so the two
// drift apart). The two waves on a SIMD belong to different workgroups: one's tile wait, epilogue and row reload can
// run under the other's MFMAs, which K13's per-tile meeting point of all 8 waves prevents. VAR bits as probe's.
template <int VAR, int PHASE>
__global__ __launch_bounds__(256, 2) void probe_w4(const h8* __restrict__ rows, const char* __restrict__ src,
                                                   int src_tiles, int ntiles, float* out, unsigned long long* clk,
                                                   const h8* __restrict__ big_rows, long long big_items) {
  constexpr int WAVES = 4, PD = 2, NT = NK / 2, BUF16 = NT * 1024 + 1024, ITEM = 20;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int* s_ready = reinterpret_cast<int*>(smem + 2 * BUF16);
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  for (int i = tid; i < 2 * BUF16 / 16; i += WAVES * 64) {
    const int v = (i * 2654435761u) >> 7;
    reinterpret_cast<uint4*>(smem)[i] = make_uint4(v & 0x3BFF3BFF, (v >> 3) & 0x3BFF3BFF, v & 0x37FF37FF, 0x3C003C00 ^ (v & 0x03FF03FF));
  }
  if (tid == 0) *s_ready = 0;
  __syncthreads();
  h8 ra[NK];
  const h8* rp = rows + ((size_t)(blockIdx.x * WAVES + wave) * NK) * 64 + lane;
#pragma unroll
  for (int s = 0; s < NK; ++s) ra[s] = rp[s * 64];
  const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  float sink = 0.f;
  int cur = 0;
  const f32x4 z = {0.f, 0.f, 0.f, 0.f};
  if (VAR & 1) {
    if (lane == 0) __hip_atomic_fetch_add(s_ready, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  const int phase = (blockIdx.x & 1) ? PHASE : 0;
  auto tile = [&](int t, auto rl_c) __attribute__((always_inline)) {
    constexpr bool RL = decltype(rl_c)::value;
    if (VAR & 1) {
      for (int i = 0; i < (1 << 20); ++i) {
        if (__hip_atomic_load(s_ready, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= WAVES * (t + 1)) break;
        __builtin_amdgcn_s_sleep(1);
      }
      asm volatile("" ::: "memory");
    }
    const char* bb = smem + cur * BUF16 + lane * 16;
    const int nxt = cur ^ 1;
    char* sbuf = smem + nxt * BUF16;
    const int tsrc = (VAR & 16) ? (int)(((blockIdx.x & 7) * 1375 + t + 1) % src_tiles) : (int)((blockIdx.x + t) % src_tiles);
    const v4i sdesc = uniform_desc(src + (size_t)tsrc * (NT + 1) * 1024, (NT + 1) * 1024);
    const h8* nr = big_rows + ((size_t)(((long long)blockIdx.x * 7919 + t * 131) % big_items) * WAVES + wave) * NK * 64 + lane;
    if ((VAR & 8) && (t + phase) % ITEM == 0) __builtin_amdgcn_s_waitcnt(0x0070);
    f32x4 acc[2] = {z, z};
    h8 b[PD + 1];
#pragma unroll
    for (int u = 0; u < PD; ++u) b[u] = *reinterpret_cast<const h8*>(bb + u * 1024);
#pragma unroll
    for (int s = 0; s < NT; ++s) {
      if (s + PD < NT) b[(s + PD) % (PD + 1)] = *reinterpret_cast<const h8*>(bb + (s + PD) * 1024);
      acc[0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ra[2 * s], b[s % (PD + 1)], acc[0], 0, 0, 0);
      acc[1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ra[2 * s + 1], b[s % (PD + 1)], acc[1], 0, 0, 0);
      if (RL) {
        ra[2 * s] = __builtin_nontemporal_load(nr + (2 * s) * 64);
        ra[2 * s + 1] = __builtin_nontemporal_load(nr + (2 * s + 1) * 64);
      }
      if (VAR & 2) {
        if (s >= 1 && (s - 1) * WAVES <= NT) {
          const int p = min((s - 1) * WAVES + wave, NT);
          dma_b128(sdesc, sbuf + p * 1024, lane * 16, p * 1024);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if (VAR & 2) __builtin_amdgcn_s_waitcnt(0x0070);
    if (VAR & 1) {
      asm volatile("" ::: "memory");
      if (lane == 0) __hip_atomic_fetch_add(s_ready, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    if (VAR & 4) {
      float am0 = fmaxf(acc[0][0], acc[1][0]);
#pragma unroll
      for (int i = 1; i < 4; ++i) am0 = fmaxf(am0, fmaxf(acc[0][i], acc[1][i]));
      if (__ballot(fmaf(am0, -2.f, 0.5f) < -1e30f)) sink += 1.f;
      sink += am0 * 1e-30f;
    } else {
      sink += acc[0][0] + acc[1][1];
    }
    cur = nxt;
  };
  for (int t = 0; t < ntiles; ++t) {
    if ((VAR & 8) && (t + phase) % ITEM == ITEM - 1) tile(t, BoolC<true>{});
    else tile(t, BoolC<false>{});
  }
  __builtin_amdgcn_s_waitcnt(0x0070);
  const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (lane == 0 && wave == 0) {
    clk[2 * blockIdx.x] = t1 - t0;
    clk[2 * blockIdx.x + 1] = r1 - r0;
  }
  out[(size_t)(blockIdx.x * WAVES + wave) * 64 + lane] = sink;
}

// W4H (round 6): as W4 (two 4-wave workgroups per CU, item transitions phase-shifted) but with K13's 32-query tiles:
// the LDS holds a ring of three HALF tiles per workgroup (pieces 0..23 = dims 0..383, pieces 24..47 + the header =
// dims 384..767; 3 x 25 KiB), so both workgroups fit; the wave signals after each half (its pieces of the half two
// ahead are issued during a half, into the buffer of the half before it). Per-tile work, epilogue and reloads as K13.
template <int VAR, int PHASE>
__global__ __launch_bounds__(256, 2) void probe_w4h(const h8* __restrict__ rows, const char* __restrict__ src,
                                                    int src_tiles, int ntiles, float* out, unsigned long long* clk,
                                                    const h8* __restrict__ big_rows, long long big_items) {
  constexpr int WAVES = 4, PD = 2, NH = NK / 2, HBUF = NH * 1024 + 1024, ITEM = 10;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  int* s_ready = reinterpret_cast<int*>(smem + 3 * HBUF);
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  for (int i = tid; i < 3 * HBUF / 16; i += WAVES * 64) {
    const int v = (i * 2654435761u) >> 7;
    reinterpret_cast<uint4*>(smem)[i] = make_uint4(v & 0x3BFF3BFF, (v >> 3) & 0x3BFF3BFF, v & 0x37FF37FF, 0x3C003C00 ^ (v & 0x03FF03FF));
  }
  if (tid == 0) *s_ready = 0;
  __syncthreads();
  h8 ra[NK];
  const h8* rp = rows + ((size_t)(blockIdx.x * WAVES + wave) * NK) * 64 + lane;
#pragma unroll
  for (int s = 0; s < NK; ++s) ra[s] = rp[s * 64];
  const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  float sink = 0.f;
  const f32x4 z = {0.f, 0.f, 0.f, 0.f};
  if (VAR & 1) {  // halves 0 and 1 are "landed" at the start (the prologue's)
    if (lane == 0) __hip_atomic_fetch_add(s_ready, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  const int phase = (blockIdx.x & 1) ? PHASE : 0;
  f32x4 acc[4] = {z, z, z, z};
  // half h of tile t = h >> 1; its buffer h % 3; during half h the wave issues its pieces of half h + 2
  auto half = [&](int h, auto rl_c, auto hi_c) __attribute__((always_inline)) {
    constexpr bool RL = decltype(rl_c)::value;
    constexpr int HI = decltype(hi_c)::value;  // 0: pieces 0..23, 1: pieces 24..47 (+ the header)
    const int t = h >> 1;
    if (VAR & 1) {
      for (int i = 0; i < (1 << 20); ++i) {
        if (__hip_atomic_load(s_ready, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= WAVES * (h + 2)) break;
        __builtin_amdgcn_s_sleep(1);
      }
      asm volatile("" ::: "memory");
    }
    const char* bb = smem + (h % 3) * HBUF + lane * 16;
    char* sbuf = smem + ((h + 2) % 3) * HBUF;
    const int h2 = h + 2, t2 = h2 >> 1;
    const int tsrc = (VAR & 16) ? (int)(((blockIdx.x & 7) * 1375 + t2) % src_tiles) : (int)((blockIdx.x + t2) % src_tiles);
    const v4i sdesc = uniform_desc(src + (size_t)tsrc * (NK + 1) * 1024 + (h2 & 1) * NH * 1024, HBUF);
    const h8* nr = big_rows + ((size_t)(((long long)blockIdx.x * 7919 + t * 131) % big_items) * WAVES + wave) * NK * 64 + lane;
    if (HI == 0) {
      if ((VAR & 8) && (t + phase) % ITEM == 0) __builtin_amdgcn_s_waitcnt(0x0070);
      acc[0] = z; acc[1] = z; acc[2] = z; acc[3] = z;
    }
    h8 b[PD + 1];
#pragma unroll
    for (int u = 0; u < PD; ++u) b[u] = *reinterpret_cast<const h8*>(bb + u * 1024);
#pragma unroll
    for (int u = 0; u < NH; ++u) {
      const int s = HI * NH + u;
      if (u + PD < NH) b[(u + PD) % (PD + 1)] = *reinterpret_cast<const h8*>(bb + (u + PD) * 1024);
      const int tt = 2 * (s >> 1), qb = s & 1;
      acc[2 * qb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ra[tt], b[u % (PD + 1)], acc[2 * qb], 0, 0, 0);
      acc[2 * qb + 1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ra[tt + 1], b[u % (PD + 1)], acc[2 * qb + 1], 0, 0, 0);
      if (RL && (s & 1)) {
        ra[s - 1] = __builtin_nontemporal_load(nr + (s - 1) * 64);
        ra[s] = __builtin_nontemporal_load(nr + s * 64);
      }
      if (VAR & 2) {  // this wave's pieces of half h + 2 (25 pieces over 4 waves: 7 per wave, the last repeats)
        if (u >= 1 && (u - 1) * WAVES <= NH) {
          const int p = min((u - 1) * WAVES + wave, NH);
          dma_b128(sdesc, sbuf + p * 1024, lane * 16, p * 1024);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    // signal: done reading half h, and my pieces of half h + 1 (issued during half h - 1) landed: everything but
    // this half's 7 DMA pieces (and, reloading, the row loads after them) may stay in flight
    if (VAR & 2) {
      if (RL) __builtin_amdgcn_s_waitcnt((31 & 15) | (0x7 << 4) | ((31 >> 4) << 14));  // + this half's 24 row loads
      else __builtin_amdgcn_s_waitcnt((7 & 15) | (0x7 << 4) | ((7 >> 4) << 14));
    }
    if (VAR & 1) {
      asm volatile("" ::: "memory");
      if (lane == 0) __hip_atomic_fetch_add(s_ready, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    if (HI == 1) {
      if (VAR & 4) {
        float am0 = fmaxf(acc[0][0], acc[1][0]), am1 = fmaxf(acc[2][0], acc[3][0]);
#pragma unroll
        for (int i = 1; i < 4; ++i) {
          am0 = fmaxf(am0, fmaxf(acc[0][i], acc[1][i]));
          am1 = fmaxf(am1, fmaxf(acc[2][i], acc[3][i]));
        }
        if (__ballot(fmaf(am0, -2.f, 0.5f) < -1e30f || fmaf(am1, -2.f, 0.5f) < -1e30f)) sink += 1.f;
        sink += am0 * 1e-30f;
      } else {
        sink += acc[0][0] + acc[1][1] + acc[2][2] + acc[3][3];
      }
    }
  };
  for (int t = 0; t < ntiles; ++t) {
    if ((VAR & 8) && (t + phase) % ITEM == ITEM - 1) {
      half(2 * t, BoolC<true>{}, IntC<0>{});
      half(2 * t + 1, BoolC<true>{}, IntC<1>{});
    } else {
      half(2 * t, BoolC<false>{}, IntC<0>{});
      half(2 * t + 1, BoolC<false>{}, IntC<1>{});
    }
  }
  __builtin_amdgcn_s_waitcnt(0x0070);
  const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (lane == 0 && wave == 0) {
    clk[2 * blockIdx.x] = t1 - t0;
    clk[2 * blockIdx.x + 1] = r1 - r0;
  }
  out[(size_t)(blockIdx.x * WAVES + wave) * 64 + lane] = sink;
}

const h8* g_big = nullptr;
const char* g_q = nullptr;
long long g_big_items = 1;

template <int VAR, int PD, int WAVES>
int run(const char* name, const h8* rows, const char* src, int src_tiles, float* out, unsigned long long* clk,
        int grid, int ntiles) {
  const size_t lds = ((VAR & 2048) ? 3 : 2) * BUF + 64 + ((VAR & 8192) ? (size_t)WAVES * 7 * 1024 : 0);
  CHECK(hipFuncSetAttribute((const void*)probe<VAR, PD, WAVES>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int rep = 0; rep < 3; ++rep)  // warm: >= 2 s of back-to-back launches before the timed one
    hipLaunchKernelGGL((probe<VAR, PD, WAVES>), dim3(grid), dim3(WAVES * 64), lds, 0, rows, src, src_tiles, ntiles, out, clk, g_big, g_big_items, g_q);
  CHECK(hipEventRecord(e0));
  hipLaunchKernelGGL((probe<VAR, PD, WAVES>), dim3(grid), dim3(WAVES * 64), lds, 0, rows, src, src_tiles, ntiles, out, clk, g_big, g_big_items, g_q);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  std::vector<unsigned long long> h(2 * grid);
  CHECK(hipMemcpy(h.data(), clk, sizeof(unsigned long long) * 2 * grid, hipMemcpyDeviceToHost));
  double ghz = 0;
  for (int b = 0; b < grid; ++b) ghz += (double)h[2 * b] / (double)h[2 * b + 1] * 0.1;
  ghz /= grid;
  const double n_mfma = (double)grid * WAVES * ntiles * 2 * NK;
  const double tf = n_mfma * 16 * 16 * 32 * 2 / (ms * 1e-3) / 1e12;
  const double pipe = n_mfma / (grid * 4.0) * 16 / (ms * 1e-3 * ghz * 1e9);
  printf("%-34s %8.3f ms  %7.1f TF/s  clock %.3f GHz  pipe busy %.3f  frac-of-2.5PF %.3f\n", name, ms, tf, ghz, pipe,
         tf / 2500.0);
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
  return 0;
}

template <int VAR>
int run16(const char* name, const h8* rows, const char* src, int src_tiles, float* out, unsigned long long* clk,
          int grid, int ntiles) {
  const size_t lds = 2 * BUF + 64;
  CHECK(hipFuncSetAttribute((const void*)probe16<VAR>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int rep = 0; rep < 3; ++rep)
    hipLaunchKernelGGL((probe16<VAR>), dim3(grid), dim3(512), lds, 0, rows, src, src_tiles, ntiles, out, clk, g_big, g_big_items);
  CHECK(hipEventRecord(e0));
  hipLaunchKernelGGL((probe16<VAR>), dim3(grid), dim3(512), lds, 0, rows, src, src_tiles, ntiles, out, clk, g_big, g_big_items);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  std::vector<unsigned long long> h(2 * grid);
  CHECK(hipMemcpy(h.data(), clk, sizeof(unsigned long long) * 2 * grid, hipMemcpyDeviceToHost));
  double ghz = 0;
  for (int b = 0; b < grid; ++b) ghz += (double)h[2 * b] / (double)h[2 * b + 1] * 0.1;
  ghz /= grid;
  const double n_mfma = (double)grid * 8 * ntiles * NK;  // one MFMA per piece per wave
  const double tf = n_mfma * 16 * 16 * 32 * 2 / (ms * 1e-3) / 1e12;
  const double pipe = n_mfma / (grid * 4.0) * 16 / (ms * 1e-3 * ghz * 1e9);
  printf("%-34s %8.3f ms  %7.1f TF/s  clock %.3f GHz  pipe busy %.3f  frac-of-2.5PF %.3f\n", name, ms, tf, ghz, pipe,
         tf / 2500.0);
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
  return 0;
}

template <int VAR, int PHASE>
int run_w4(const char* name, const h8* rows, const char* src, int src_tiles, float* out, unsigned long long* clk,
           int grid, int ntiles) {
  const size_t lds = 2 * (NK / 2 * 1024 + 1024) + 64;
  CHECK(hipFuncSetAttribute((const void*)probe_w4<VAR, PHASE>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int rep = 0; rep < 3; ++rep)
    hipLaunchKernelGGL((probe_w4<VAR, PHASE>), dim3(grid), dim3(256), lds, 0, rows, src, src_tiles, ntiles, out, clk, g_big, g_big_items);
  CHECK(hipEventRecord(e0));
  hipLaunchKernelGGL((probe_w4<VAR, PHASE>), dim3(grid), dim3(256), lds, 0, rows, src, src_tiles, ntiles, out, clk, g_big, g_big_items);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  std::vector<unsigned long long> h(2 * grid);
  CHECK(hipMemcpy(h.data(), clk, sizeof(unsigned long long) * 2 * grid, hipMemcpyDeviceToHost));
  double ghz = 0;
  for (int b = 0; b < grid; ++b) ghz += (double)h[2 * b] / (double)h[2 * b + 1] * 0.1;
  ghz /= grid;
  const double n_mfma = (double)grid * 4 * ntiles * NK;  // NK / 2 pieces x 2 MFMAs per wave and tile
  const double tf = n_mfma * 16 * 16 * 32 * 2 / (ms * 1e-3) / 1e12;
  const double pipe = n_mfma / (grid / 2 * 4.0) * 16 / (ms * 1e-3 * ghz * 1e9);
  printf("%-34s %8.3f ms  %7.1f TF/s  clock %.3f GHz  pipe busy %.3f  frac-of-2.5PF %.3f\n", name, ms, tf, ghz, pipe,
         tf / 2500.0);
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
  return 0;
}

template <int VAR, int PHASE>
int run_w4h(const char* name, const h8* rows, const char* src, int src_tiles, float* out, unsigned long long* clk,
            int grid, int ntiles) {
  const size_t lds = 3 * (NK / 2 * 1024 + 1024) + 64;
  CHECK(hipFuncSetAttribute((const void*)probe_w4h<VAR, PHASE>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int rep = 0; rep < 3; ++rep)
    hipLaunchKernelGGL((probe_w4h<VAR, PHASE>), dim3(grid), dim3(256), lds, 0, rows, src, src_tiles, ntiles, out, clk, g_big, g_big_items);
  CHECK(hipEventRecord(e0));
  hipLaunchKernelGGL((probe_w4h<VAR, PHASE>), dim3(grid), dim3(256), lds, 0, rows, src, src_tiles, ntiles, out, clk, g_big, g_big_items);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  std::vector<unsigned long long> h(2 * grid);
  CHECK(hipMemcpy(h.data(), clk, sizeof(unsigned long long) * 2 * grid, hipMemcpyDeviceToHost));
  double ghz = 0;
  for (int b = 0; b < grid; ++b) ghz += (double)h[2 * b] / (double)h[2 * b + 1] * 0.1;
  ghz /= grid;
  const double n_mfma = (double)grid * 4 * ntiles * 2 * NK;
  const double tf = n_mfma * 16 * 16 * 32 * 2 / (ms * 1e-3) / 1e12;
  const double pipe = n_mfma / (grid / 2 * 4.0) * 16 / (ms * 1e-3 * ghz * 1e9);
  printf("%-34s %8.3f ms  %7.1f TF/s  clock %.3f GHz  pipe busy %.3f  frac-of-2.5PF %.3f\n", name, ms, tf, ghz, pipe,
         tf / 2500.0);
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
  return 0;
}

int main(int argc, char** argv) {
  const int grid = 256;
  const int ntiles = argc > 1 ? atoi(argv[1]) : 4000;
  const int src_tiles = 64;  // 3.1 MB of tile images: L2/MALL-resident
  const int big_tiles = 11000;  // 540 MB of tile images (VAR 16)
  h8* rows;
  char* src;
  float* out;
  unsigned long long* clk;
  const size_t nrows = (size_t)grid * 8 * NK * 64;
  CHECK(hipMalloc(&rows, nrows * sizeof(h8)));
  CHECK(hipMalloc(&src, (size_t)big_tiles * (NK + 1) * 1024));
  {
    h8* big;
    const size_t big_bytes = (size_t)8 << 30;  // 8 GiB of rows: the item reloads come from HBM
    CHECK(hipMalloc(&big, big_bytes));
    CHECK(hipMemset(big, 0x35, big_bytes));
    g_big = big;
    g_big_items = (long long)(big_bytes / ((size_t)8 * NK * 1024));
  }
  {
    char* qa;
    CHECK(hipMalloc(&qa, (size_t)kQ * NK * 32));
    CHECK(hipMemset(qa, 0x31, (size_t)kQ * NK * 32));
    g_q = qa;
  }
  CHECK(hipMalloc(&out, (size_t)grid * 8 * 64 * sizeof(float)));
  CHECK(hipMalloc(&clk, sizeof(unsigned long long) * 4 * grid));  // (W4 runs 2 x grid workgroups)
  {
    std::vector<uint16_t> hr(nrows * 8);
    uint32_t x = 12345;
    for (auto& v : hr) {
      x = x * 1664525u + 1013904223u;
      v = (uint16_t)(0x3000 + ((x >> 9) & 0x0BFF)) ^ ((x >> 3) & 0x8000);
    }
    CHECK(hipMemcpy(rows, hr.data(), hr.size() * 2, hipMemcpyHostToDevice));
    std::vector<uint16_t> hs((size_t)big_tiles * (NK + 1) * 512);
    for (auto& v : hs) {
      x = x * 1664525u + 1013904223u;
      v = (uint16_t)(0x3000 + ((x >> 9) & 0x0BFF)) ^ ((x >> 3) & 0x8000);
    }
    CHECK(hipMemcpy(src, hs.data(), hs.size() * 2, hipMemcpyHostToDevice));
  }
  printf("grid %d, %d tiles per wave, 16x16x32 f16, 32 rows x 768 dims per wave in registers\n", grid, ntiles);
  const int mode = argc > 2 ? atoi(argv[2]) : 0;
  if (mode == 3) {  // round 6: K13's shape with the next item's first rows prefetched into spare LDS
    const int tiles = ntiles - ntiles % 10;
    for (int rep = 0; rep < 2; ++rep) {
      run<7 + 8 + 16 + 256, 2, 8>("K13 8w: sync dma epi items hbm", rows, src, big_tiles, out, clk, grid, tiles);
      run<7 + 8 + 16 + 256 + 8192, 2, 8>("+ 7 of 48 rows regs via LDS", rows, src, big_tiles, out, clk, grid, tiles);
      run<7 + 8 + 16 + 256 + 8192 + 16384, 2, 8>("+ 4 of 48 rows regs via LDS", rows, src, big_tiles, out, clk, grid, tiles);
      run<7 + 16 + 256, 2, 8>("K13 8w: no items (reload-free)", rows, src, big_tiles, out, clk, grid, tiles);
    }
    return 0;
  }
  if (mode == 2) {  // round 6: K13's shape vs W4H (2 x 4 waves, 32-query tiles in a ring of three half tiles)
    const int tiles = ntiles - ntiles % 10;
    for (int rep = 0; rep < 2; ++rep) {
      run<7 + 8 + 16 + 256, 2, 8>("K13 8w: sync dma epi items hbm", rows, src, big_tiles, out, clk, grid, tiles);
      run_w4h<7 + 8 + 16, 5>("W4H: sync dma epi items hbm", rows, src, big_tiles, out, clk, 2 * grid, tiles);
      run_w4h<7 + 8 + 16, 0>("W4H in phase", rows, src, big_tiles, out, clk, 2 * grid, tiles);
      run_w4h<7 + 16, 0>("W4H: no items (reload-free)", rows, src, big_tiles, out, clk, 2 * grid, tiles);
    }
    return 0;
  }
  if (mode == 1) {  // round 6: K13's shape (8 waves, 32-query tiles, items of 10) vs W4 (2 x 4 waves, 16-query tiles, items of 20)
    // (the same MFMAs: W4 runs twice the tiles of half the size on twice the workgroups)
    const int tiles = ntiles - ntiles % 20;
    for (int rep = 0; rep < 2; ++rep) {
      run<7 + 8 + 16 + 256, 2, 8>("K13 8w: sync dma epi items hbm", rows, src, big_tiles, out, clk, grid, tiles);
      run_w4<7 + 8 + 16, 10>("W4 2x4w: sync dma epi items hbm", rows, src, big_tiles, out, clk, 2 * grid, 2 * tiles);
      run_w4<7 + 8 + 16, 0>("W4 in phase", rows, src, big_tiles, out, clk, 2 * grid, 2 * tiles);
      run<7 + 16, 2, 8>("K13 8w: no items (reload-free)", rows, src, big_tiles, out, clk, grid, tiles);
      run_w4<7 + 16, 0>("W4: no items (reload-free)", rows, src, big_tiles, out, clk, 2 * grid, 2 * tiles);
    }
    return 0;
  }
  run<7, 2, 8>("+sync +dma +epi", rows, src, src_tiles, out, clk, grid, ntiles);
  run<7 + 2048, 2, 8>("+split sync (3 bufs) +dma +epi", rows, src, src_tiles, out, clk, grid, ntiles);
  run<7 + 2048 + 4096, 2, 8>("+split sync, waves 4-7 offset", rows, src, src_tiles, out, clk, grid, ntiles);
  run<23, 2, 8>("+sync +dma +epi +hbm tiles", rows, src, big_tiles, out, clk, grid, ntiles);
  run<23 + 2048 + 4096, 2, 8>("+split sync offset +hbm tiles", rows, src, big_tiles, out, clk, grid, ntiles);
  run<7, 2, 8>("+sync +dma +epi (again)", rows, src, src_tiles, out, clk, grid, ntiles);
  run<7 + 2048 + 4096, 2, 8>("+split sync offset (again)", rows, src, src_tiles, out, clk, grid, ntiles);
  return 0;
}
