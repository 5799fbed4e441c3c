// Packed-fp32 exact-erf GELU / GELU' on k-scaled pre-activations, shared by the projection
// kernels (project.hip, bagproj.hip).
#pragma once
#include "common.h"

namespace blindno {
namespace gelu_pk {

// GELU on k-scaled pre-activations.  W1 and b1 are staged multiplied by k = sqrt(log2(e)/2),
// so the MFMA yields hk = k h and e^{-h^2/2} = 2^{-(hk)^2} costs one multiply and one v_exp;
// with half = erfc(|h|/sqrt2)/2 (A&S 7.1.26, common.h) GELU(h) = (max(hk, 0) - |hk| half)/k,
// and the 1/k is folded into W2 (forward) or applied once to the accumulated sums (backward).
constexpr float kK = 0.84932180028801904f;        // sqrt(log2(e) / 2)
constexpr float kInvK = 1.1774100225154747f;
constexpr float kT = 0.27273748087922245f;        // A&S p / (sqrt2 k)
// kp = 1 / (sqrt(2 pi) k) = 0.46971863934982566 (folded into norm_cdf_pair_pdf)

// Two GELUs per lane-instruction: the polynomial / product steps as packed fp32 (v_pk_fma_f32,
// v_pk_mul_f32 on <2 x float>); the transcendentals, |hk| (a free VOP3 source modifier on the
// scalar fma) and the sign transfer (v_bfi_b32) stay scalar.  With half = erfc(|h|/sqrt2)/2,
//     s = copysign(1/2 - half, h),   Phi(h) = 1/2 + s,
// so no compare/select and no max is needed: k GELU(h) = hk Phi(h), GELU'(h) = Phi + h phi(h).
typedef float f32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f32x2 pk_fma(f32x2 a, f32x2 b, f32x2 c) {
  return __builtin_elementwise_fma(a, b, c);
}

__device__ __forceinline__ f32x2 splat2(float v) { return (f32x2){v, v}; }

// Phi(h) (as cdf) and e = e^{-h^2/2} for a pair of k-scaled pre-activations
__device__ __forceinline__ f32x2 norm_cdf_pair(f32x2 hk, f32x2& e) {
  const f32x2 t = {__builtin_amdgcn_rcpf(fmaf(fabsf(hk.x), kT, 1.0f)),
                   __builtin_amdgcn_rcpf(fmaf(fabsf(hk.y), kT, 1.0f))};
  const f32x2 sq = hk * hk;
  e = (f32x2){__builtin_amdgcn_exp2f(-sq.x), __builtin_amdgcn_exp2f(-sq.y)};
  f32x2 q = pk_fma(t, splat2(0.5307027145f), splat2(-0.7265760135f));
  q = pk_fma(t, q, splat2(0.7107068705f));
  q = pk_fma(t, q, splat2(-0.142248368f));
  q = pk_fma(t, q, splat2(0.127414796f));
  const f32x2 m = pk_fma(-(q * t), e, splat2(0.5f));          // 1/2 - half
  const f32x2 sgn = {copysignf(m.x, hk.x), copysignf(m.y, hk.y)};
  return sgn + splat2(0.5f);
}

// Backward variant: Phi(h) and ep = phi_k(h) = kp e^{-h^2/2} (kp = 1/(sqrt(2 pi) k)), so that
// GELU'(h) = Phi + hk ep is one fma: the exp argument carries log2(kp) and the polynomial
// coefficients carry 1/kp (half = q' t ep).
constexpr float kLog2Kp = -1.0901312512086083f;
__device__ __forceinline__ f32x2 norm_cdf_pair_pdf(f32x2 hk, f32x2& ep) {
  const f32x2 t = {__builtin_amdgcn_rcpf(fmaf(fabsf(hk.x), kT, 1.0f)),
                   __builtin_amdgcn_rcpf(fmaf(fabsf(hk.y), kT, 1.0f))};
  const f32x2 ea = pk_fma(-hk, hk, splat2(kLog2Kp));
  ep = (f32x2){__builtin_amdgcn_exp2f(ea.x), __builtin_amdgcn_exp2f(ea.y)};
  f32x2 q = pk_fma(t, splat2(1.129831073415752f), splat2(-1.5468324069611348f));
  q = pk_fma(t, q, splat2(1.513048048260859f));
  q = pk_fma(t, q, splat2(-0.3028373926078324f));
  q = pk_fma(t, q, splat2(0.27125769625911544f));
  const f32x2 m = pk_fma(-(q * t), ep, splat2(0.5f));         // 1/2 - half
  const f32x2 sgn = {copysignf(m.x, hk.x), copysignf(m.y, hk.y)};
  return sgn + splat2(0.5f);
}


// norm_cdf_pair / norm_cdf_pair_pdf on N pairs in lockstep (every step issued for all N pairs
// before the next step): the same operations per value in the same order (bit-identical), but
// consecutive packed ops are independent.  One pair at a time, every Horner step read the
// previous packed result and hipcc put an s_nop between them: 766 of them per 16-row item of
// the encoder's forward row kernel (profiles/r06/r06_issue_budget_rowfuse_fwd_zc_item.txt).
template <int N>
__device__ __forceinline__ void norm_cdf_pairs(const f32x2 (&hk)[N], f32x2 (&cdf)[N]) {
  f32x2 t[N], e[N], q[N];
#pragma unroll
  for (int j = 0; j < N; ++j)
    t[j] = (f32x2){__builtin_amdgcn_rcpf(fmaf(fabsf(hk[j].x), kT, 1.0f)),
                   __builtin_amdgcn_rcpf(fmaf(fabsf(hk[j].y), kT, 1.0f))};
#pragma unroll
  for (int j = 0; j < N; ++j) {
    const f32x2 sq = hk[j] * hk[j];
    e[j] = (f32x2){__builtin_amdgcn_exp2f(-sq.x), __builtin_amdgcn_exp2f(-sq.y)};
  }
#pragma unroll
  for (int j = 0; j < N; ++j) q[j] = pk_fma(t[j], splat2(0.5307027145f), splat2(-0.7265760135f));
#pragma unroll
  for (int j = 0; j < N; ++j) q[j] = pk_fma(t[j], q[j], splat2(0.7107068705f));
#pragma unroll
  for (int j = 0; j < N; ++j) q[j] = pk_fma(t[j], q[j], splat2(-0.142248368f));
#pragma unroll
  for (int j = 0; j < N; ++j) q[j] = pk_fma(t[j], q[j], splat2(0.127414796f));
#pragma unroll
  for (int j = 0; j < N; ++j) q[j] = -(q[j] * t[j]);
#pragma unroll
  for (int j = 0; j < N; ++j) {
    const f32x2 m = pk_fma(q[j], e[j], splat2(0.5f));          // 1/2 - half
    cdf[j] = (f32x2){copysignf(m.x, hk[j].x), copysignf(m.y, hk[j].y)} + splat2(0.5f);
  }
}

template <int N>
__device__ __forceinline__ void norm_cdf_pdf_pairs(const f32x2 (&hk)[N], f32x2 (&cdf)[N],
                                                   f32x2 (&ep)[N]) {
  f32x2 t[N], q[N];
#pragma unroll
  for (int j = 0; j < N; ++j)
    t[j] = (f32x2){__builtin_amdgcn_rcpf(fmaf(fabsf(hk[j].x), kT, 1.0f)),
                   __builtin_amdgcn_rcpf(fmaf(fabsf(hk[j].y), kT, 1.0f))};
#pragma unroll
  for (int j = 0; j < N; ++j) {
    const f32x2 ea = pk_fma(-hk[j], hk[j], splat2(kLog2Kp));
    ep[j] = (f32x2){__builtin_amdgcn_exp2f(ea.x), __builtin_amdgcn_exp2f(ea.y)};
  }
#pragma unroll
  for (int j = 0; j < N; ++j) q[j] = pk_fma(t[j], splat2(1.129831073415752f), splat2(-1.5468324069611348f));
#pragma unroll
  for (int j = 0; j < N; ++j) q[j] = pk_fma(t[j], q[j], splat2(1.513048048260859f));
#pragma unroll
  for (int j = 0; j < N; ++j) q[j] = pk_fma(t[j], q[j], splat2(-0.3028373926078324f));
#pragma unroll
  for (int j = 0; j < N; ++j) q[j] = pk_fma(t[j], q[j], splat2(0.27125769625911544f));
#pragma unroll
  for (int j = 0; j < N; ++j) q[j] = -(q[j] * t[j]);
#pragma unroll
  for (int j = 0; j < N; ++j) {
    const f32x2 m = pk_fma(q[j], ep[j], splat2(0.5f));         // 1/2 - half
    cdf[j] = (f32x2){copysignf(m.x, hk[j].x), copysignf(m.y, hk[j].y)} + splat2(0.5f);
  }
}

// norm_cdf_pair_pdf without the final + 1/2: Phi(h) - 1/2 (the bag-level projection adds the
// halves back once per point, csrc/bagproj.hip)
__device__ __forceinline__ f32x2 norm_cdf_pair_pdf_centered(f32x2 hk, f32x2& ep) {
  const f32x2 t = {__builtin_amdgcn_rcpf(fmaf(fabsf(hk.x), kT, 1.0f)),
                   __builtin_amdgcn_rcpf(fmaf(fabsf(hk.y), kT, 1.0f))};
  const f32x2 ea = pk_fma(-hk, hk, splat2(kLog2Kp));
  ep = (f32x2){__builtin_amdgcn_exp2f(ea.x), __builtin_amdgcn_exp2f(ea.y)};
  f32x2 q = pk_fma(t, splat2(1.129831073415752f), splat2(-1.5468324069611348f));
  q = pk_fma(t, q, splat2(1.513048048260859f));
  q = pk_fma(t, q, splat2(-0.3028373926078324f));
  q = pk_fma(t, q, splat2(0.27125769625911544f));
  const f32x2 m = pk_fma(-(q * t), ep, splat2(0.5f));         // 1/2 - half
  return (f32x2){copysignf(m.x, hk.x), copysignf(m.y, hk.y)};
}

// norm_cdf_pair_pdf_centered on four pairs in lockstep: every step of the evaluation is issued
// for the four pairs before the next step, so consecutive packed ops are independent (a packed
// op reading the previous VALU result costs a wait state on gfx950: the one-pair chain carried
// an s_nop between each Horner step)
__device__ __forceinline__ void norm_cdf_quad_pdf_centered(const f32x2 (&hk)[4], f32x2 (&s)[4],
                                                           f32x2 (&ep)[4]) {
  f32x2 t[4], q[4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
    t[j] = (f32x2){__builtin_amdgcn_rcpf(fmaf(fabsf(hk[j].x), kT, 1.0f)),
                   __builtin_amdgcn_rcpf(fmaf(fabsf(hk[j].y), kT, 1.0f))};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const f32x2 ea = pk_fma(-hk[j], hk[j], splat2(kLog2Kp));
    ep[j] = (f32x2){__builtin_amdgcn_exp2f(ea.x), __builtin_amdgcn_exp2f(ea.y)};
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) q[j] = pk_fma(t[j], splat2(1.129831073415752f), splat2(-1.5468324069611348f));
#pragma unroll
  for (int j = 0; j < 4; ++j) q[j] = pk_fma(t[j], q[j], splat2(1.513048048260859f));
#pragma unroll
  for (int j = 0; j < 4; ++j) q[j] = pk_fma(t[j], q[j], splat2(-0.3028373926078324f));
#pragma unroll
  for (int j = 0; j < 4; ++j) q[j] = pk_fma(t[j], q[j], splat2(0.27125769625911544f));
#pragma unroll
  for (int j = 0; j < 4; ++j) q[j] = -(q[j] * t[j]);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const f32x2 m = pk_fma(q[j], ep[j], splat2(0.5f));         // 1/2 - half
    s[j] = (f32x2){copysignf(m.x, hk[j].x), copysignf(m.y, hk[j].y)};
  }
}

}  // namespace gelu_pk
}  // namespace blindno
