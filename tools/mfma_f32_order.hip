// Which fp32 rounding order does v_mfma_f32_16x16x4_f32 follow? (tools/, not part of the product)
//
// The PQ LUT build (pq.hip K9r) may run on this MFMA only if its result is a fixed chain of fmaf steps
// the oracle can restate. Each trial feeds random A (16x4), B (4x16), C (16x16) with spread exponents and
// compares every output against candidate orders computed on the host:
//   chain   fma(a3,b3, fma(a2,b2, fma(a1,b1, fma(a0,b0, c))))
//   rchain  the same chain k = 3..0
//   exact   c + sum_k a_k b_k in fp64, rounded once to fp32
//   pair    c + ((a0 b0 + a1 b1) + (a2 b2 + a3 b3)), products and sums rounded in fp32
// v_mfma_f32_32x32x2_f32 (the K3 chain) runs beside it as the control.
// Build: hipcc -O3 --offload-arch=gfx950 tools/mfma_f32_order.hip -o /tmp/mfma_f32_order
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define CHECK(x)                                                                     \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      return 1;                                                                      \
    }                                                                                \
  } while (0)

// trial t: A [16][4], B [4][16], C [16][16] -> D [16][16]; one wave per trial
__global__ void k16(const float* A, const float* B, const float* C, float* D) {
  const int t = blockIdx.x, l = threadIdx.x;
  const int i = l & 15, kk = l >> 4;
  const float a = A[t * 64 + i * 4 + kk];
  const float b = B[t * 64 + kk * 16 + i];
  f32x4 c;
  for (int r = 0; r < 4; ++r) c[r] = C[t * 256 + (4 * kk + r) * 16 + i];
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) D[t * 256 + (4 * kk + r) * 16 + i] = c[r];
}

// two chained MFMAs (dims 0..3, then 4..7): A [16][8], B [8][16] per trial
__global__ void k16x2(const float* A, const float* B, const float* C, float* D) {
  const int t = blockIdx.x, l = threadIdx.x;
  const int i = l & 15, kk = l >> 4;
  f32x4 c;
  for (int r = 0; r < 4; ++r) c[r] = C[t * 256 + (4 * kk + r) * 16 + i];
  for (int u = 0; u < 2; ++u) {
    const float a = A[t * 128 + i * 8 + 4 * u + kk];
    const float b = B[t * 128 + (4 * u + kk) * 16 + i];
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
  }
  for (int r = 0; r < 4; ++r) D[t * 256 + (4 * kk + r) * 16 + i] = c[r];
}

// control: A [32][2], B [2][32], C [32][32]
__global__ void k32(const float* A, const float* B, const float* C, float* D) {
  const int t = blockIdx.x, l = threadIdx.x;
  const int i = l & 31, kk = l >> 5;
  const float a = A[t * 64 + i * 2 + kk];
  const float b = B[t * 64 + kk * 32 + i];
  f32x16 c;
  for (int r = 0; r < 16; ++r) c[r] = C[t * 1024 + (8 * (r >> 2) + 4 * kk + (r & 3)) * 32 + i];
  c = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
  for (int r = 0; r < 16; ++r) D[t * 1024 + (8 * (r >> 2) + 4 * kk + (r & 3)) * 32 + i] = c[r];
}

static float rnd(std::mt19937& g) {
  std::uniform_real_distribution<float> u(-1.0f, 1.0f);
  std::uniform_int_distribution<int> e(-6, 6);
  return std::ldexp(u(g), e(g));
}

int main() {
  const int T = 4096;
  std::mt19937 g(7);
  // 16x16x4
  std::vector<float> A(T * 64), B(T * 64), C(T * 256), D(T * 256);
  for (auto& v : A) v = rnd(g);
  for (auto& v : B) v = rnd(g);
  for (auto& v : C) v = rnd(g);
  float *dA, *dB, *dC, *dD;
  CHECK(hipMalloc(&dA, A.size() * 4));
  CHECK(hipMalloc(&dB, B.size() * 4));
  CHECK(hipMalloc(&dC, 4 * T * 1024));
  CHECK(hipMalloc(&dD, 4 * T * 1024));
  CHECK(hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(dC, C.data(), C.size() * 4, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k16, dim3(T), dim3(64), 0, 0, dA, dB, dC, dD);
  CHECK(hipGetLastError());
  CHECK(hipDeviceSynchronize());
  CHECK(hipMemcpy(D.data(), dD, D.size() * 4, hipMemcpyDeviceToHost));
  long n = 0, m_chain = 0, m_rchain = 0, m_exact = 0, m_pair = 0;
  for (int t = 0; t < T; ++t)
    for (int i = 0; i < 16; ++i)
      for (int j = 0; j < 16; ++j) {
        const float* a = &A[t * 64 + i * 4];
        float b[4];
        for (int k = 0; k < 4; ++k) b[k] = B[t * 64 + k * 16 + j];
        const float c = C[t * 256 + i * 16 + j], d = D[t * 256 + i * 16 + j];
        float ch = c;
        for (int k = 0; k < 4; ++k) ch = fmaf(a[k], b[k], ch);
        float rc = c;
        for (int k = 3; k >= 0; --k) rc = fmaf(a[k], b[k], rc);
        double ex = c;
        for (int k = 0; k < 4; ++k) ex += (double)a[k] * (double)b[k];
        const float p0 = a[0] * b[0], p1 = a[1] * b[1], p2 = a[2] * b[2], p3 = a[3] * b[3];
        const float pr = c + ((p0 + p1) + (p2 + p3));
        ++n;
        m_chain += ch == d;
        m_rchain += rc == d;
        m_exact += (float)ex == d;
        m_pair += pr == d;
      }
  printf("16x16x4f32: %ld outputs | chain %ld rchain %ld exact %ld pair %ld\n", n, m_chain, m_rchain, m_exact, m_pair);
  {  // two chained MFMAs against the 8-step chain
    std::vector<float> A2(T * 128), B2(T * 128);
    for (auto& v : A2) v = rnd(g);
    for (auto& v : B2) v = rnd(g);
    float *dA2, *dB2;
    CHECK(hipMalloc(&dA2, A2.size() * 4));
    CHECK(hipMalloc(&dB2, B2.size() * 4));
    CHECK(hipMemcpy(dA2, A2.data(), A2.size() * 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(dB2, B2.data(), B2.size() * 4, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k16x2, dim3(T), dim3(64), 0, 0, dA2, dB2, dC, dD);
    CHECK(hipGetLastError());
    CHECK(hipDeviceSynchronize());
    CHECK(hipMemcpy(D.data(), dD, D.size() * 4, hipMemcpyDeviceToHost));
    long n2 = 0, m2 = 0, m2s = 0;
    for (int t = 0; t < T; ++t)
      for (int i = 0; i < 16; ++i)
        for (int j = 0; j < 16; ++j) {
          const float c = C[t * 256 + i * 16 + j], d = D[t * 256 + i * 16 + j];
          float ch = c;
          for (int k = 0; k < 8; ++k) ch = fmaf(A2[t * 128 + i * 8 + k], B2[t * 128 + k * 16 + j], ch);
          float h0 = c, h1 = 0.0f;  // each MFMA's own chain, the two rounded sums added
          for (int k = 0; k < 4; ++k) h0 = fmaf(A2[t * 128 + i * 8 + k], B2[t * 128 + k * 16 + j], h0);
          for (int k = 4; k < 8; ++k) h1 = fmaf(A2[t * 128 + i * 8 + k], B2[t * 128 + k * 16 + j], h1);
          ++n2;
          m2 += ch == d;
          m2s += (h0 + h1) == d;
        }
    printf("16x16x4f32 x2 chained: %ld outputs | 8-step chain %ld split-sum %ld\n", n2, m2, m2s);
  }
  // control 32x32x2
  std::vector<float> C2(T * 1024), D2(T * 1024);
  for (auto& v : C2) v = rnd(g);
  CHECK(hipMemcpy(dC, C2.data(), C2.size() * 4, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k32, dim3(T), dim3(64), 0, 0, dA, dB, dC, dD);
  CHECK(hipGetLastError());
  CHECK(hipDeviceSynchronize());
  CHECK(hipMemcpy(D2.data(), dD, D2.size() * 4, hipMemcpyDeviceToHost));
  n = 0;
  long c_chain = 0, c_exact = 0;
  for (int t = 0; t < T; ++t)
    for (int i = 0; i < 32; ++i)
      for (int j = 0; j < 32; ++j) {
        const float a0 = A[t * 64 + i * 2], a1 = A[t * 64 + i * 2 + 1];
        const float b0 = B[t * 64 + j], b1 = B[t * 64 + 32 + j];
        const float c = C2[t * 1024 + i * 32 + j], d = D2[t * 1024 + i * 32 + j];
        ++n;
        c_chain += fmaf(a1, b1, fmaf(a0, b0, c)) == d;
        c_exact += (float)((double)c + (double)a0 * b0 + (double)a1 * b1) == d;
      }
  printf("32x32x2f32: %ld outputs | chain %ld exact %ld\n", n, c_chain, c_exact);
  return 0;
}
