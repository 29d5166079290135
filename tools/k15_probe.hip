// K15 loop probe (tools/, not part of the product): an output-stationary form of the IVF fine scan.
// Per workgroup (8 waves) an item is 256 list rows x up to 16*NQB queries of the list; the accumulators of
// the whole item stay in registers (wave w: rows 64 (w & 3) .. + 63, query blocks qb = (w >> 2) + 2 j), and
// BOTH operands stream through an R-stage LDS ring, one stage per 32 dims (k-step): 16 KiB of rows (8 groups
// x 2 KiB, the fp16 group layout's chunk t) + NQB KiB of query blocks, all by LDS-DMA (1 KiB pieces dealt
// over the waves). No per-item register reload (K13's item transition): the ring runs on across items.
// Sync: one LDS counter; each wave adds 1 per k-step after finishing its reads of stage S - DRIFT and its DMA
// pieces of stage S + 1 landing.
// Reports TF/s, the in-kernel clock and the MFMA pipe's busy fraction, as tools/k13_probe.hip.
// Build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off tools/k15_probe.hip -o tools/k15_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int v4i __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                    \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      return 1;                                                                     \
    }                                                                               \
  } while (0)

constexpr int NT = 24;                 // k-steps of 32 dims (d = 768)
constexpr int GROUP_BYTES = NT * 2048;  // one 32-row group, fp16

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

__device__ __forceinline__ void wait_vm(int v) {
#define VM(n) ((n & 15) | (0x7 << 4) | ((n >> 4) << 14))
  if (v >= 12) __builtin_amdgcn_s_waitcnt(VM(12));
  else if (v >= 10) __builtin_amdgcn_s_waitcnt(VM(10));
  else if (v >= 8) __builtin_amdgcn_s_waitcnt(VM(8));
  else if (v >= 6) __builtin_amdgcn_s_waitcnt(VM(6));
  else if (v >= 5) __builtin_amdgcn_s_waitcnt(VM(5));
  else if (v >= 4) __builtin_amdgcn_s_waitcnt(VM(4));
  else if (v >= 3) __builtin_amdgcn_s_waitcnt(VM(3));
  else if (v >= 2) __builtin_amdgcn_s_waitcnt(VM(2));
  else if (v >= 1) __builtin_amdgcn_s_waitcnt(VM(1));
  else __builtin_amdgcn_s_waitcnt(VM(0));
#undef VM
}

// VAR bits: 1 sync, 2 DMA (else the ring's contents stay), 4 epilogue filter per item, 8 rows from a large HBM
// buffer (else a small L2-resident pool), 16 query images from a large pool
template <int NQB, int R, int DRIFT, int VAR>
__global__ __launch_bounds__(512, 1) void k15(const char* __restrict__ rows_big, long long n_row_items,
                                              const char* __restrict__ q_pool, int q_items, int n_items,
                                              float* out, unsigned long long* clk) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int A_BYTES = 16 * 1024;
  constexpr int STAGE = A_BYTES + NQB * 1024;
  constexpr int NPIECE = 16 + NQB;
  constexpr int NJ = NQB / 2;
  constexpr int PPW = (NPIECE + 7) / 8;  // pieces per wave per stage (at most)
  int* cnt = reinterpret_cast<int*>(smem + R * STAGE);
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int rq = wave & 3, qc = wave >> 2;
  const int c = lane & 15, kq = lane >> 4;
  if (tid == 0) *cnt = 0;
  for (int i = tid; i < R * STAGE / 16; i += 512) {
    const int v = (i * 2654435761u) >> 7;
    reinterpret_cast<uint4*>(smem)[i] = make_uint4(v & 0x3BFF3BFF, (v >> 3) & 0x3BFF3BFF, v & 0x37FF37FF, 0x3C003C00 ^ (v & 0x03FF03FF));
  }
  __syncthreads();
  auto row_src = [&](int it) -> const char* {
    const long long ri = (VAR & 8) ? ((long long)blockIdx.x * 7919 + (long long)it * 131) % n_row_items : (blockIdx.x & 63);
    return rows_big + ri * (8LL * GROUP_BYTES);
  };
  auto q_src = [&](int it) -> const char* {
    const int qi = (VAR & 16) ? (int)(((blockIdx.x & 7) * 37 + it) % q_items) : (int)((blockIdx.x & 7) % q_items);
    return q_pool + (long long)qi * (NT * NQB * 1024);
  };
  // issue this wave's pieces of global stage S (item S / NT, k-step S % NT)
  auto issue = [&](int S) {
    if (!(VAR & 2)) return;
    const int it = S / NT, t = S - it * NT;
    char* st = smem + (S % R) * STAGE;
    const v4i da = uniform_desc(row_src(it), 8 * GROUP_BYTES);
    const v4i db = uniform_desc(q_src(it), NT * NQB * 1024);
#pragma unroll
    for (int j = 0; j < PPW; ++j) {
      const int p = wave + 8 * j;
      if (p < 16) {
        const int gi = p >> 1, h = p & 1;
        dma_b128(da, st + gi * 2048 + h * 1024, lane * 16, gi * GROUP_BYTES + t * 2048 + h * 1024);
      } else if (p < NPIECE) {
        const int qb = p - 16;
        dma_b128(db, st + A_BYTES + qb * 1024, lane * 16, (t * NQB + qb) * 1024);
      }
    }
  };
  auto my_pieces = [&]() { return (VAR & 2) ? ((wave < NPIECE % 8 || NPIECE % 8 == 0) ? PPW : PPW - 1) : 0; };
  const int total = n_items * NT;
  // prologue: stages 0 .. R - 2 - DRIFT
  for (int S = 0; S <= R - 2 - DRIFT && S < total; ++S) issue(S);
  __builtin_amdgcn_s_waitcnt(0x0070);
  if (VAR & 1) {
    if (lane == 0) __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  const f32x4 z = {0.f, 0.f, 0.f, 0.f};
  f32x4 acc[NJ][4];
  float sink = 0.f;
  int S = 0;
  for (int it = 0; it < n_items; ++it) {
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[j][r] = z;
    for (int t = 0; t < NT; ++t, ++S) {
      if (VAR & 1) {
        for (int i = 0; i < (1 << 20); ++i) {
          if (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= 8 * (S - DRIFT > 0 ? S - DRIFT + 1 : 1)) break;
          __builtin_amdgcn_s_sleep(1);
        }
        asm volatile("" ::: "memory");
      }
      const char* st = smem + (S % R) * STAGE;
      h8 a[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gi = 2 * rq + (r >> 1), rb = r & 1;
        a[r] = *reinterpret_cast<const h8*>(st + gi * 2048 + kq * 512 + rb * 256 + c * 16);
      }
      const char* bb = st + A_BYTES + qc * 1024 + lane * 16;
      h8 b[3];
      b[0] = *reinterpret_cast<const h8*>(bb);
      b[1] = *reinterpret_cast<const h8*>(bb + 2048);
      const int Sn = S + R - 1 - DRIFT;  // the stage this k-step stages (into the slot of stage S - 1 - DRIFT)
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        if (j + 2 < NJ) b[(j + 2) % 3] = *reinterpret_cast<const h8*>(bb + (j + 2) * 2048);
#pragma unroll
        for (int r = 0; r < 4; ++r)
          acc[j][r] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[r], b[j % 3], acc[j][r], 0, 0, 0);
        if (j == 1 && Sn < total) issue(Sn);
        __builtin_amdgcn_sched_barrier(0);
      }
      // signal S + 1: my reads of stage S are done and my pieces of stage S + 1 + DRIFT landed (younger: stages
      // S + 2 + DRIFT .. Sn); a wave starts k-step S once every wave gave signal S - DRIFT
      if (VAR & 1) {
        const int last = Sn < total ? Sn : total - 1;
        const int younger = (last - (S + 1 + DRIFT)) * my_pieces();
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
        wait_vm(younger < 0 ? 0 : younger);
        asm volatile("" ::: "memory");
        if (lane == 0) __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    }
    if (VAR & 4) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        float m = fmaxf(fmaxf(acc[j][0][0], acc[j][1][0]), fmaxf(acc[j][2][0], acc[j][3][0]));
#pragma unroll
        for (int i = 1; i < 4; ++i) m = fmaxf(m, fmaxf(fmaxf(acc[j][0][i], acc[j][1][i]), fmaxf(acc[j][2][i], acc[j][3][i])));
        if (__ballot(fmaf(m, -2.f, 0.5f) < -1e30f)) sink += 1.f;
        sink += m * 1e-30f;
      }
    } else {
#pragma unroll
      for (int j = 0; j < NJ; ++j) sink += acc[j][0][0] + acc[j][1][1] + acc[j][2][2] + acc[j][3][3];
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (lane == 0 && wave == 0) {
    clk[2 * blockIdx.x] = t1 - t0;
    clk[2 * blockIdx.x + 1] = r1 - r0;
  }
  out[(size_t)(blockIdx.x * 8 + wave) * 64 + lane] = sink;
}

const char* g_rows = nullptr;
long long g_row_items = 1;
const char* g_q = nullptr;
int g_q_items = 1;

template <int NQB, int R, int DRIFT, int VAR>
int run(const char* name, float* out, unsigned long long* clk, int grid, int n_items, int q_items) {
  constexpr int STAGE = 16 * 1024 + NQB * 1024;
  const size_t lds = (size_t)R * STAGE + 64;
  CHECK(hipFuncSetAttribute((const void*)k15<NQB, R, DRIFT, VAR>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int rep = 0; rep < 3; ++rep)
    hipLaunchKernelGGL((k15<NQB, R, DRIFT, VAR>), dim3(grid), dim3(512), lds, 0, g_rows, g_row_items, g_q, q_items, n_items, out, clk);
  CHECK(hipEventRecord(e0));
  hipLaunchKernelGGL((k15<NQB, R, DRIFT, VAR>), dim3(grid), dim3(512), lds, 0, g_rows, g_row_items, g_q, q_items, n_items, out, clk);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  CHECK(hipGetLastError());
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  std::vector<unsigned long long> h(2 * grid);
  CHECK(hipMemcpy(h.data(), clk, sizeof(unsigned long long) * 2 * grid, hipMemcpyDeviceToHost));
  double ghz = 0;
  for (int b = 0; b < grid; ++b) ghz += (double)h[2 * b] / (double)h[2 * b + 1] * 0.1;
  ghz /= grid;
  const double n_mfma = (double)grid * 8 * n_items * NT * (NQB / 2) * 4;
  const double tf = n_mfma * 16 * 16 * 32 * 2 / (ms * 1e-3) / 1e12;
  const double pipe = n_mfma / (grid * 4.0) * 16 / (ms * 1e-3 * ghz * 1e9);
  const double gbs = (double)grid * n_items * NT * (16 + NQB) * 1024.0 / (ms * 1e-3) / 1e9;
  printf("%-44s %8.3f ms %7.1f TF/s clock %.3f GHz pipe %.3f frac %.3f  staged %6.0f GB/s\n", name, ms, tf, ghz, pipe,
         tf / 2500.0, gbs);
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
  return 0;
}

int main(int argc, char** argv) {
  const int grid = 256;
  const int n_items = argc > 1 ? atoi(argv[1]) : 160;
  float* out;
  unsigned long long* clk;
  {
    char* big;
    const size_t big_bytes = (size_t)8 << 30;  // 8 GiB of rows: items from HBM
    CHECK(hipMalloc(&big, big_bytes));
    std::vector<uint16_t> hr((size_t)64 << 20);
    uint32_t x = 12345;
    for (auto& v : hr) {
      x = x * 1664525u + 1013904223u;
      v = (uint16_t)(0x3000 + ((x >> 9) & 0x0BFF)) ^ ((x >> 3) & 0x8000);
    }
    for (size_t off = 0; off < big_bytes; off += hr.size() * 2)
      CHECK(hipMemcpy(big + off, hr.data(), hr.size() * 2, hipMemcpyHostToDevice));
    g_rows = big;
    g_row_items = (long long)(big_bytes / (8LL * GROUP_BYTES));
    char* q;
    const int q_items = 1024;  // query images: 1024 lists x 24 x 20 KiB = 503 MB
    CHECK(hipMalloc(&q, (size_t)q_items * NT * 20 * 1024));
    for (size_t off = 0; off < (size_t)q_items * NT * 20 * 1024; off += hr.size() * 2) {
      const size_t n = std::min(hr.size() * 2, (size_t)q_items * NT * 20 * 1024 - off);
      CHECK(hipMemcpy(q + off, hr.data(), n, hipMemcpyHostToDevice));
    }
    g_q = q;
    g_q_items = q_items;
  }
  CHECK(hipMalloc(&out, (size_t)grid * 8 * 64 * sizeof(float)));
  CHECK(hipMalloc(&clk, sizeof(unsigned long long) * 2 * grid));
  printf("grid %d, %d items per workgroup (256 rows x 16*NQB queries x 768 dims), 16x16x32 f16\n", grid, n_items);
  run<20, 4, 0, 0>("NQB 20 loop only (R 4)", out, clk, grid, n_items, 8);
  run<20, 4, 0, 1>("NQB 20 +sync", out, clk, grid, n_items, 8);
  run<20, 4, 0, 3>("NQB 20 +sync +dma (L2 rows)", out, clk, grid, n_items, 8);
  run<20, 4, 0, 7>("NQB 20 +sync +dma +epi", out, clk, grid, n_items, 8);
  run<20, 4, 0, 15>("NQB 20 +sync +dma +epi +hbm rows", out, clk, grid, n_items, 8);
  run<20, 4, 0, 31>("NQB 20 +sync +dma +epi +hbm rows +q pool", out, clk, grid, n_items, g_q_items);
  run<20, 3, 0, 31>("NQB 20 all, R 3", out, clk, grid, n_items, g_q_items);
  run<16, 4, 0, 31>("NQB 16 all", out, clk, grid, n_items, g_q_items);
  run<10, 4, 0, 31>("NQB 10 all", out, clk, grid, n_items, g_q_items);
  run<10, 6, 1, 31>("NQB 10 all R 6 drift 1", out, clk, grid, n_items, g_q_items);
  run<4, 6, 1, 31>("NQB 4 all R 6 drift 1", out, clk, grid, n_items, g_q_items);
  return 0;
}
