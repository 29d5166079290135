// MFMA f32 issue-rate probe for the fine-scan inner loop (tools/, not part of the product).
//
// Each variant runs the K3 loop shape on one persistent grid and reports TF/s of
// v_mfma_f32_32x32x2_f32 work:
//   P1 one dependent accumulator chain, register operands
//   P2 two independent chains interleaved
//   P3 P1 + one ds_read_b128 per k-step (B operand from LDS)
//   P4 P3 + one global_load_dwordx4 per k-step (A operand streamed, 2 blocks of 8 in flight)
//   P5 P4 with two chains (A reused for two B tiles: the K3w shape)
// Build: hipcc -O3 --offload-arch=gfx950 tools/mfma_probe.hip -o /tmp/mfma_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef float f32x16 __attribute__((ext_vector_type(16)));

#define CHECK(x)                                                                \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

constexpr int kSteps = 4096;  // k-steps per wave

template <int VAR, int LDSF = 32 * 772 + 64>
__global__ __launch_bounds__(512, 1) void probe(const float* __restrict__ src, size_t src_floats, float* out) {
  __shared__ __attribute__((aligned(16))) float lds[LDSF];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int j = lane & 31, h = lane >> 5;
  for (int i = tid; i < LDSF; i += 512) lds[i] = (float)(i % 7) * 0.25f;
  __syncthreads();
  f32x16 c0 = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  f32x16 c1 = c0;
  float4 a = make_float4(1.f + lane, 2.f, 3.f, 4.f);
  float4 b = make_float4(0.5f, 0.25f, 0.125f, 1.f);
  const float* qrow = lds + (LDSF > 32 * 772 ? j * 772 : j * 4) + 4 * h;  // small variant: overlapping rows (timing only)
  // per-wave streaming window inside an L2/MALL-resident buffer
  const size_t span = src_floats / (gridDim.x * 8);
  const float* base = src + (size_t)(blockIdx.x * 8 + wave) * span + j * 8 + 4 * h;
  float4 A[8], B[8];
  if (VAR >= 4) {
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < 8; ++u) A[u] = *reinterpret_cast<const float4*>(base + u * 256);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < 8; ++u) B[u] = *reinterpret_cast<const float4*>(base + 2048 + u * 256);
    __builtin_amdgcn_sched_barrier(0);
  }
  size_t off = 4096;
  for (int s = 0; s < kSteps; s += 16) {
    if (VAR <= 2) {
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        c0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, b.x, c0, 0, 0, 0);
        if (VAR == 2) c1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, b.y, c1, 0, 0, 0);
        c0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, b.y, c0, 0, 0, 0);
        if (VAR == 2) c1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, b.z, c1, 0, 0, 0);
        c0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, b.z, c0, 0, 0, 0);
        if (VAR == 2) c1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, b.w, c1, 0, 0, 0);
        c0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, b.w, c0, 0, 0, 0);
        if (VAR == 2) c1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, b.x, c1, 0, 0, 0);
      }
    } else if (VAR == 3) {
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const float4 bb = *reinterpret_cast<const float4*>(qrow + ((s + u) & 63) * 8);
        c0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, bb.x, c0, 0, 0, 0);
        c0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, bb.y, c0, 0, 0, 0);
        c0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, bb.z, c0, 0, 0, 0);
        c0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, bb.w, c0, 0, 0, 0);
      }
    } else if (VAR >= 6) {
      // per k-step: 4 (or 8) MFMAs on A[u], then refill A[u] for the block two ahead; the
      // sched_group_barriers pin the order MFMA x4|8, VMEM x1, DS x1
      const size_t o1 = off % (span - 4096);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const float4 bb = *reinterpret_cast<const float4*>(qrow + ((s + u) & 63) * 8);
        c0 = __builtin_amdgcn_mfma_f32_32x32x2f32(A[u].x, bb.x, c0, 0, 0, 0);
        if (VAR == 7) c1 = __builtin_amdgcn_mfma_f32_32x32x2f32(A[u].x, bb.y, c1, 0, 0, 0);
        c0 = __builtin_amdgcn_mfma_f32_32x32x2f32(A[u].y, bb.y, c0, 0, 0, 0);
        if (VAR == 7) c1 = __builtin_amdgcn_mfma_f32_32x32x2f32(A[u].y, bb.z, c1, 0, 0, 0);
        c0 = __builtin_amdgcn_mfma_f32_32x32x2f32(A[u].z, bb.z, c0, 0, 0, 0);
        if (VAR == 7) c1 = __builtin_amdgcn_mfma_f32_32x32x2f32(A[u].z, bb.w, c1, 0, 0, 0);
        c0 = __builtin_amdgcn_mfma_f32_32x32x2f32(A[u].w, bb.w, c0, 0, 0, 0);
        if (VAR == 7) c1 = __builtin_amdgcn_mfma_f32_32x32x2f32(A[u].w, bb.x, c1, 0, 0, 0);
        A[u] = *reinterpret_cast<const float4*>(base + o1 + u * 256);
        __builtin_amdgcn_sched_group_barrier(0x008, VAR == 7 ? 8 : 4, 0);
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const float4 bb = *reinterpret_cast<const float4*>(qrow + ((s + 8 + u) & 63) * 8);
        c0 = __builtin_amdgcn_mfma_f32_32x32x2f32(B[u].x, bb.x, c0, 0, 0, 0);
        if (VAR == 7) c1 = __builtin_amdgcn_mfma_f32_32x32x2f32(B[u].x, bb.y, c1, 0, 0, 0);
        c0 = __builtin_amdgcn_mfma_f32_32x32x2f32(B[u].y, bb.y, c0, 0, 0, 0);
        if (VAR == 7) c1 = __builtin_amdgcn_mfma_f32_32x32x2f32(B[u].y, bb.z, c1, 0, 0, 0);
        c0 = __builtin_amdgcn_mfma_f32_32x32x2f32(B[u].z, bb.z, c0, 0, 0, 0);
        if (VAR == 7) c1 = __builtin_amdgcn_mfma_f32_32x32x2f32(B[u].z, bb.w, c1, 0, 0, 0);
        c0 = __builtin_amdgcn_mfma_f32_32x32x2f32(B[u].w, bb.w, c0, 0, 0, 0);
        if (VAR == 7) c1 = __builtin_amdgcn_mfma_f32_32x32x2f32(B[u].w, bb.x, c1, 0, 0, 0);
        B[u] = *reinterpret_cast<const float4*>(base + o1 + 2048 + u * 256);
        __builtin_amdgcn_sched_group_barrier(0x008, VAR == 7 ? 8 : 4, 0);
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
      off += 4096;
    } else {
      // two 8-k-step blocks: consume A, refill A two blocks ahead; same for B
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const float4 bb = *reinterpret_cast<const float4*>(qrow + ((s + u) & 63) * 8);
        c0 = __builtin_amdgcn_mfma_f32_32x32x2f32(A[u].x, bb.x, c0, 0, 0, 0);
        if (VAR == 5) c1 = __builtin_amdgcn_mfma_f32_32x32x2f32(A[u].x, bb.y, c1, 0, 0, 0);
        c0 = __builtin_amdgcn_mfma_f32_32x32x2f32(A[u].y, bb.y, c0, 0, 0, 0);
        if (VAR == 5) c1 = __builtin_amdgcn_mfma_f32_32x32x2f32(A[u].y, bb.z, c1, 0, 0, 0);
        c0 = __builtin_amdgcn_mfma_f32_32x32x2f32(A[u].z, bb.z, c0, 0, 0, 0);
        if (VAR == 5) c1 = __builtin_amdgcn_mfma_f32_32x32x2f32(A[u].z, bb.w, c1, 0, 0, 0);
        c0 = __builtin_amdgcn_mfma_f32_32x32x2f32(A[u].w, bb.w, c0, 0, 0, 0);
        if (VAR == 5) c1 = __builtin_amdgcn_mfma_f32_32x32x2f32(A[u].w, bb.x, c1, 0, 0, 0);
      }
      const size_t o1 = off % (span - 4096);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int u = 0; u < 8; ++u) A[u] = *reinterpret_cast<const float4*>(base + o1 + u * 256);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const float4 bb = *reinterpret_cast<const float4*>(qrow + ((s + 8 + u) & 63) * 8);
        c0 = __builtin_amdgcn_mfma_f32_32x32x2f32(B[u].x, bb.x, c0, 0, 0, 0);
        if (VAR == 5) c1 = __builtin_amdgcn_mfma_f32_32x32x2f32(B[u].x, bb.y, c1, 0, 0, 0);
        c0 = __builtin_amdgcn_mfma_f32_32x32x2f32(B[u].y, bb.y, c0, 0, 0, 0);
        if (VAR == 5) c1 = __builtin_amdgcn_mfma_f32_32x32x2f32(B[u].y, bb.z, c1, 0, 0, 0);
        c0 = __builtin_amdgcn_mfma_f32_32x32x2f32(B[u].z, bb.z, c0, 0, 0, 0);
        if (VAR == 5) c1 = __builtin_amdgcn_mfma_f32_32x32x2f32(B[u].z, bb.w, c1, 0, 0, 0);
        c0 = __builtin_amdgcn_mfma_f32_32x32x2f32(B[u].w, bb.w, c0, 0, 0, 0);
        if (VAR == 5) c1 = __builtin_amdgcn_mfma_f32_32x32x2f32(B[u].w, bb.x, c1, 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int u = 0; u < 8; ++u) B[u] = *reinterpret_cast<const float4*>(base + o1 + 2048 + u * 256);
      __builtin_amdgcn_sched_barrier(0);
      off += 4096;
    }
  }
  float r = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) r += c0[i] + c1[i];
  if (r == 12345.678f) out[blockIdx.x * 512 + tid] = r;
}

template <int VAR, int LDSF = 32 * 772 + 64>
int run(const char* name, const float* src, size_t n, float* out, int cus, int per_cu) {
  const int grid = cus * per_cu;
  hipLaunchKernelGGL((probe<VAR, LDSF>), dim3(grid), dim3(512), 0, 0, src, n, out);
  CHECK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  CHECK(hipEventRecord(e0));
  const int reps = 5;
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL((probe<VAR, LDSF>), dim3(grid), dim3(512), 0, 0, src, n, out);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  const double mfma_per_wave = (double)kSteps * 4 * ((VAR == 2 || VAR == 5 || VAR == 7) ? 2 : 1);
  const double flops = mfma_per_wave * 32 * 32 * 2 * 2 * grid * 8 * reps;
  printf("%-48s grid %5d  %8.3f ms  %7.1f TF/s\n", name, grid, ms / reps, flops / (ms * 1e-3) / 1e12);
  return 0;
}

int main() {
  int cus = 0;
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  cus = p.multiProcessorCount;
  size_t n = (size_t)64 << 20;  // 256 MiB source window
  float* src;
  float* out;
  CHECK(hipMalloc(&src, n * 4));
  CHECK(hipMalloc(&out, (size_t)cus * 4 * 512 * 4));
  CHECK(hipMemset(src, 0, n * 4));
  printf("CUs %d\n", cus);
  for (int per_cu = 1; per_cu <= 1; ++per_cu) {
    run<1>("P1 one chain, register operands", src, n, out, cus, per_cu);
    run<2>("P2 two chains, register operands", src, n, out, cus, per_cu);
    run<3>("P3 one chain + ds_read_b128 B", src, n, out, cus, per_cu);
    run<4>("P4 P3 + streamed A (2x8 k-steps in flight)", src, n, out, cus, per_cu);
    run<5>("P5 P4 with two chains (K3w shape)", src, n, out, cus, per_cu);
    run<6>("P6 P4, per-k-step refill pinned by sched_group", src, n, out, cus, per_cu);
    run<7>("P7 P6 with two chains", src, n, out, cus, per_cu);
  }
  // small LDS (8 KB): 2 workgroups per CU (4 waves per SIMD) where registers allow
  run<4, 2048>("P4s P4, 8 KB LDS, 2 WG/CU", src, n, out, cus, 2);
  run<5, 2048>("P5s P5, 8 KB LDS, 2 WG/CU", src, n, out, cus, 2);
  return 0;
}
