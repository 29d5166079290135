// Pre-filter arithmetic shared by K10/K11 (prefilter.hip) and K13 (rsscan.hip): the approximate key of
// an fp16 MFMA dot, the rigorous bound delta of |approximate - pinned fp32 key|, the refine window and
// the one-fma fast filter.
#pragma once
#include "mivs_common.hpp"

namespace mivs {

// approximate key of one accumulator element: the dot is acc * 2^-(row exp + query exp), exact
template <int METRIC>
__device__ __forceinline__ float pf_key(float acc, float qs, float xn, float qn) {
  const float v = acc * qs;
  if (METRIC == kL2) {
    const float t = fmaf(-2.0f, v, xn + qn);
    return t > 0.0f ? t : 0.0f;
  }
  return xn < INFINITY ? -v : INFINITY;
}

// delta >= |approximate key - pinned fp32 key| for every (row, query q) of the index:
//   |x.q - x_h.q_h| <= |x_h||q - q_h| + |x - x_h||q|   (Cauchy-Schwarz on the fp16 rounding residuals)
//   + 2 dp u |x_h||q_h|  (the fp16-product sum inside the MFMA, any order and rounding)
//   + 1.01 dp u |x||q|   (the pinned fp32 fma chain);  L2 keys: x2, plus the roundings of the key itself.
// Index-wide maxima of |x| and |x - x_h| stand in for the row's own values.
template <int METRIC>
__device__ __forceinline__ float pf_delta(float qn, float qres, float x_norm_max, float x_res_max, int dp) {
  const float nq = sqrtf(qn) * (1.0f + 0x1p-12f);
  const float nx = x_norm_max, rx = x_res_max;
  const float nxh = nx + rx, nqh = nq + qres;
  const float ga = 2.0f * (float)dp * 0x1p-24f;
  const float gp = 1.01f * (float)dp * 0x1p-24f;
  const float dd = nxh * qres + rx * nq + ga * nxh * nqh + gp * nx * nq;
  const float delta = METRIC == kL2 ? 2.0f * dd + 4.0f * 0x1p-24f * (nx * nx + qn) : dd;
  return delta * (1.0f + 0x1p-10f) + 1e-30f;
}

// order-preserving float <-> uint32 (atomicMin over signed keys)
__device__ __forceinline__ unsigned pf_ord(float x) {
  const unsigned b = __float_as_uint(x);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float pf_unord(unsigned u) {
  return __uint_as_float((u & 0x80000000u) ? (u & 0x7FFFFFFFu) : ~u);
}

// the refine window above a k-th approximate key kth: every candidate whose pinned key can reach the
// top-k has approximate key <= pf_window(Ak). Monotone in kth, so any kth' >= Ak gives a window >= it.
__device__ __forceinline__ float pf_window(float kth, float delta) {
  return kth + 2.0f * delta + fabsf(kth) * 0x1p-20f;
}

// the epilogue's fast filter. The exact test keeps key < lk_last && key <= th, i.e. key < U with
// U = min(lk_last, next float above th). The filter value of an accumulator element is ONE fma,
//   L2: f = fl(xn - 2 acc qs)  (key = max(fl(fl(xn + qn) - 2 acc qs), 0))     IP: f = acc * -qs = key,
// and f < pf_uf(U) for every key < U: for L2 the margin (xn_max^2 + qn + |U|) 2^-20 is 4x the sum of the
// roundings of f, of the key and of U - qn (|2 acc qs| <= 1.01 (xn + qn)). The filter only has false
// positives, which the exact test then rejects. -inf: the query slot is empty.
template <int METRIC>
__device__ __forceinline__ float pf_uf(float lk_last, float th, float qn, float xnmax2) {
  const float U = fminf(lk_last, nextafterf(th, INFINITY));
  if (!(U > -INFINITY) || !(qn < INFINITY)) return -INFINITY;
  if (!(U < INFINITY)) return INFINITY;
  if (METRIC == kL2) return (U - qn) + (xnmax2 + qn + fabsf(U)) * 0x1p-20f;
  return U;
}

}  // namespace mivs
