// Shared device helpers for the BlinDNO HIP kernels (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define BLINDNO_API extern "C" __attribute__((visibility("default")))

namespace blindno {

constexpr int kBlock = 256;

// Exact-erf GELU (F.gelu default, 2d_FPE/FNOModules.py:232,238) through the standard normal
// CDF Phi(z) = 0.5 erfc(-z/sqrt2), branch-free.  erfc(u), u = |z|/sqrt2 >= 0, uses
// Abramowitz & Stegun 7.1.26: erfc(u) = t P(t) e^{-u^2}, t = 1/(1 + p u), |abs error| <=
// 1.5e-7.  Measured over z in [-12, 12] (fp32): max |GELU error| 4.2e-7, the same as the
// reference's own fp32 x*0.5*(1+erf(x/sqrt2)) (4.5e-7); max |GELU' error| 3.2e-7.
// e^{-u^2} = e^{-z^2/2} is shared with the density phi(z) of the derivative, so GELU and
// GELU' together cost one rcp + one exp + ~10 FMA.
__device__ __forceinline__ float norm_cdf_e(float z, float e) {
  // t = 1 / (1 + p |z| / sqrt2); the A&S coefficients a_i are pre-halved (h_i = a_i / 2)
  const float t = __builtin_amdgcn_rcpf(fmaf(fabsf(z), 0.3275911f * 0.70710678118654752f, 1.0f));
  float q = fmaf(t, 0.5307027145f, -0.7265760135f);
  q = fmaf(t, q, 0.7107068705f);
  q = fmaf(t, q, -0.142248368f);
  q = fmaf(t, q, 0.127414796f);
  const float half_erfc = q * t * e;
  return z >= 0.f ? 1.0f - half_erfc : half_erfc;
}

// e^{-z^2/2} on the transcendental unit (v_exp_f32 = 2^x); flushes to 0 below 2^-126
__device__ __forceinline__ float gauss_e(float z) {
  return __builtin_amdgcn_exp2f(z * z * -0.72134752044448170368f);
}

__device__ __forceinline__ float norm_cdf(float z) { return norm_cdf_e(z, gauss_e(z)); }

__device__ __forceinline__ float gelu_f(float z) { return z * norm_cdf(z); }

// GELU'(z) = Phi(z) + z phi(z)
__device__ __forceinline__ float gelu_grad_f(float z) {
  const float e = gauss_e(z);
  return fmaf(z, 0.39894228040143268f * e, norm_cdf_e(z, e));
}

__device__ __forceinline__ void gelu_both(float z, float& g, float& dg) {
  const float e = gauss_e(z);
  const float cdf = norm_cdf_e(z, e);
  g = z * cdf;
  dg = fmaf(z, 0.39894228040143268f * e, cdf);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

__device__ __forceinline__ int uniform_int(int v) { return __builtin_amdgcn_readfirstlane(v); }

// XCD-major workgroup order.  Workgroups are dispatched round-robin over the 8 XCDs (block b on
// XCD b % 8), each XCD with its own L2; renumbering so that consecutive virtual blocks share an
// XCD keeps the neighbouring work items that reuse one input (e.g. the column tiles of one
// spectrum row quad) on one L2.  A bijection on [0, nb): the last nb % 8 blocks keep their id.
__device__ __forceinline__ int xcd_block(int b, int nb) {
  const int per = nb >> 3;
  return b >= per * 8 ? b : (b & 7) * per + (b >> 3);
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

// Block-wide copy of n floats global -> LDS (16-B aligned src/dst): float4 loads, four in flight
// per thread, so a workgroup's table staging costs one memory latency rather than n/blockDim.
__device__ __forceinline__ void stage_to_lds(float* __restrict__ dst, const float* __restrict__ src,
                                             int n) {
  const int n4 = n >> 2, st = blockDim.x;
  const float4* s4 = reinterpret_cast<const float4*>(src);
  float4* d4 = reinterpret_cast<float4*>(dst);
  int e = threadIdx.x;
  for (; e + 3 * st < n4; e += 4 * st) {
    const float4 a = s4[e], b = s4[e + st], c = s4[e + 2 * st], d = s4[e + 3 * st];
    d4[e] = a;
    d4[e + st] = b;
    d4[e + 2 * st] = c;
    d4[e + 3 * st] = d;
  }
  for (; e < n4; e += st) d4[e] = s4[e];
  for (int t = (n4 << 2) + (int)threadIdx.x; t < n; t += st) dst[t] = src[t];
}

// Division by a launch-invariant divisor as one v_mul_hi_u32 + add + shift (Granlund-Montgomery
// round-up multiplier): exact for every n < 2^31.  Index maps (point -> sample, row, column;
// im2col k -> channel, tap) divide by launch constants; as generic 32-bit divisions those cost
// ~25 VALU each (a third of project_bwd's instruction stream before this).
struct FastDiv {
  unsigned m, s;
  static FastDiv make(unsigned d) {
    unsigned l = 0;
    while ((1ull << l) < d) ++l;
    const uint64_t m = (((uint64_t)1 << 32) * (((uint64_t)1 << l) - d)) / d + 1;
    return FastDiv{(unsigned)m, l};
  }
  __device__ __forceinline__ unsigned div(unsigned n) const {
    return (__umulhi(n, m) + n) >> s;
  }
};

inline int cdiv(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

inline int grid_for(int64_t n, int block = kBlock, int cap = 1 << 20) {
  int64_t g = (n + block - 1) / block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

}  // namespace blindno
