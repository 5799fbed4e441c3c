// Shared device helpers for the BlinDNO HIP kernels (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define BLINDNO_API extern "C" __attribute__((visibility("default")))

namespace blindno {

constexpr int kBlock = 256;

// Standard normal CDF Phi(x) = 0.5 erfc(-x/sqrt2), branch-free: erfc(u) for u >= 0 from
// the Chebyshev-fitted form erfc(u) = t exp(-u^2 + P(t)), t = 1/(1 + u/2), fractional
// error < 1.2e-7 for all u >= 0 (Numerical Recipes "erfcc").  Exact-erf GELU semantics
// (F.gelu default) within fp32 rounding, at ~1 rcp + 2 exp + 10 FMA.
__device__ __forceinline__ float norm_cdf(float x) {
  float u = fabsf(x) * 0.70710678118654752f;
  float t = __builtin_amdgcn_rcpf(fmaf(0.5f, u, 1.0f));
  float p = fmaf(t, 0.17087277f, -0.82215223f);
  p = fmaf(t, p, 1.48851587f);
  p = fmaf(t, p, -1.13520398f);
  p = fmaf(t, p, 0.27886807f);
  p = fmaf(t, p, -0.18628806f);
  p = fmaf(t, p, 0.09678418f);
  p = fmaf(t, p, 0.37409196f);
  p = fmaf(t, p, 1.00002368f);
  p = fmaf(t, p, -1.26551223f);
  float half_erfc = 0.5f * t * __expf(fmaf(-u, u, p));
  return x >= 0.f ? 1.0f - half_erfc : half_erfc;
}

__device__ __forceinline__ float gelu_f(float z) { return z * norm_cdf(z); }

// GELU'(z) = Phi(z) + z phi(z)
__device__ __forceinline__ float gelu_grad_f(float z) {
  float pdf = 0.39894228040143268f * __expf(-0.5f * z * z);
  return fmaf(z, pdf, norm_cdf(z));
}

__device__ __forceinline__ void gelu_both(float z, float& g, float& dg) {
  float cdf = norm_cdf(z);
  float pdf = 0.39894228040143268f * __expf(-0.5f * z * z);
  g = z * cdf;
  dg = fmaf(z, pdf, cdf);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

__device__ __forceinline__ int uniform_int(int v) { return __builtin_amdgcn_readfirstlane(v); }

// Hermitian weight of a complex-to-real inverse of length n at bin k (< n/2+1):
// bin 0 and the Nyquist bin (even n) count once, every other bin twice.
__device__ __forceinline__ float c2r_weight(int k, int n) {
  return (k == 0 || 2 * k == n) ? 1.0f : 2.0f;
}

// Frequency row of kept row j (see include/blindno.h).
__device__ __forceinline__ int kept_row(int j, int K1, int m1, int P1) {
  return (K1 == P1 || j < m1) ? j : P1 - 2 * m1 + j;
}

__host__ __device__ __forceinline__ int kept_rows_count(int m1, int P1) {
  return 2 * m1 < P1 ? 2 * m1 : P1;
}

inline int cdiv(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

inline int grid_for(int64_t n, int block = kBlock, int cap = 1 << 20) {
  int64_t g = (n + block - 1) / block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

}  // namespace blindno
