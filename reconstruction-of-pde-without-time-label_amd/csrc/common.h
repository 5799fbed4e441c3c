// Shared device helpers for the BlinDNO HIP kernels (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define BLINDNO_API extern "C" __attribute__((visibility("default")))

namespace blindno {

constexpr int kBlock = 256;

__device__ __forceinline__ float gelu_f(float z) {
  // exact-erf GELU (F.gelu default): 0.5 z (1 + erf(z / sqrt 2))
  return 0.5f * z * (1.0f + erff(z * 0.70710678118654752f));
}

// GELU'(z) = Phi(z) + z phi(z)
__device__ __forceinline__ float gelu_grad_f(float z) {
  float cdf = 0.5f * (1.0f + erff(z * 0.70710678118654752f));
  float pdf = 0.39894228040143268f * __expf(-0.5f * z * z);
  return cdf + z * pdf;
}

__device__ __forceinline__ void gelu_both(float z, float& g, float& dg) {
  float cdf = 0.5f * (1.0f + erff(z * 0.70710678118654752f));
  float pdf = 0.39894228040143268f * __expf(-0.5f * z * z);
  g = z * cdf;
  dg = cdf + z * pdf;
}

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
