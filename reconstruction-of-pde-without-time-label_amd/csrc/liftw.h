// The heads' lift (fc0 + permute + pad, 2d_FPE/FNOModules.py:219-224): the bag-mean input form
// and the wide kernel's workgroup body (fields.hip).  Hosting it beside the heads' first row DFT,
// which then formed its operand rows on the fly, measured slower and was removed.
#pragma once
#include "common.h"

namespace blindno {

constexpr int kLiftMaxG = 4, kLiftMaxC = 16;

// The heads' input h formed on the fly from the bag mean instead of read from a materialised
// (B, N1, N2, width) field (NIOFP2D_FNO: h = fc0([grid, ubar]), 2d_FPE/NIOModules.py:569-575;
// bagmean_fwd_kernel below): the heads' lift reads ubar (1 value per point) and the grid, and
// its adjoint hands back d ubar (bagmean_bwd_kernel's reduction) -- no h written or read, two
// launches less.  Every value is formed with bagmean_fwd / _bwd's own fma order
// (bit-identical).
struct BagIn {
  const float* u;      // ubar (B, N1 N2); nullptr: the input is a materialised field
  const float* grid;   // (N1 N2, 2)
  const float* w;      // fc0 weight (width, 3): gx, gy, u
  const float* bias;   // (width)
  float invL;          // the u scale of bagmean_fwd (1 for a bag-level ubar)
  float invLb;         // the 1 / L of bagmean_bwd
};
// h[p][j], j < CIN, at point p (flattened over (B, N1 N2)) with grid point s
template <int CIN>
__device__ __forceinline__ void bag_point(const BagIn& bi, unsigned p, unsigned s, float (&v)[CIN]) {
  const float uu = bi.u[p];
  const float g0 = bi.grid[2 * s], g1 = bi.grid[2 * s + 1];
#pragma unroll
  for (int j = 0; j < CIN; ++j) {
    float a = bi.bias[j];
    a = fmaf(bi.w[j * 3], g0, a);
    a = fmaf(bi.w[j * 3 + 1], g1, a);
    v[j] = fmaf(bi.w[j * 3 + 2] * bi.invL, uu, a);
  }
}


// lift_fwd_wide_kernel's body: thread per point, all C channels of x0 (zero on the padding)
template <int CIN, int CM>
__device__ __forceinline__ void lift_fwd_wide_block(
    const float* __restrict__ in, const float* __restrict__ w0, const float* __restrict__ b0,
    float* __restrict__ x0, int Bn, int N1, int N2, int C, int P1, int P2, int Bg, int G,
    int64_t wgs, FastDiv dHW, FastDiv dP2, BagIn bi, int bx, int gx) {
  __shared__ float sw[kLiftMaxG][CM * CIN + CM];
  for (int e = threadIdx.x; e < G * (CM * CIN + CM); e += kBlock) {
    const int g = e / (CM * CIN + CM), q = e - g * (CM * CIN + CM);
    float v = 0.f;
    if (q < CM * CIN) {
      const int c = q / CIN, j = q - c * CIN;
      v = c < C ? w0[g * wgs + c * CIN + j] : 0.f;
    } else if (q - CM * CIN < C) {
      v = b0[g * wgs + q - CM * CIN];
    }
    sw[g][q] = v;
  }
  __syncthreads();
  const unsigned HW = (unsigned)(P1 * P2);
  const unsigned total = (unsigned)Bn * HW;
  for (unsigned idx = bx * kBlock + threadIdx.x; idx < total; idx += gx * kBlock) {
    const unsigned n = dHW.div(idx), s = idx - n * HW;
    const unsigned h = dP2.div(s), w = s - h * (unsigned)P2;
    float* xp = x0 + (size_t)n * C * HW + s;
    if (h >= (unsigned)N1 || w >= (unsigned)N2) {
#pragma unroll
      for (int c = 0; c < CM; ++c)
        if (c < C) xp[(size_t)c * HW] = 0.f;
      continue;
    }
    const int g = G > 1 ? (int)(n / (unsigned)Bg) : 0;
    const unsigned ni = n - (unsigned)g * (unsigned)Bg;
    float v[CIN];
    if (bi.u) {
      bag_point<CIN>(bi, (ni * N1 + h) * N2 + w, h * N2 + w, v);
    } else {
      const float4* ip = reinterpret_cast<const float4*>(in + ((size_t)(ni * N1 + h) * N2 + w) * CIN);
#pragma unroll
      for (int q = 0; q < CIN / 4; ++q) {
        const float4 t = ip[q];
        v[4 * q] = t.x; v[4 * q + 1] = t.y; v[4 * q + 2] = t.z; v[4 * q + 3] = t.w;
      }
    }
    const float* wg = sw[g];
#pragma unroll
    for (int c = 0; c < CM; ++c) {
      if (c >= C) break;
      float a = wg[CM * CIN + c];
#pragma unroll
      for (int j = 0; j < CIN; ++j) a = fmaf(wg[c * CIN + j], v[j], a);
      xp[(size_t)c * HW] = a;
    }
  }
}

// (workgroup bx of gx explicit: lift_bwd_both_kernel hosts it beside the weight gradient)

}  // namespace blindno
