// Workgroup bodies of the weight-gradient kernels that more than one launch hosts: the 1x1-conv
// weight / bias gradient of the wide fields runs as its own launch (fields.hip,
// blindno_conv_wgrad_g) and beside the heads' backward row DFT (spectral.hip,
// blindno_rowdft_wgrad_g).  Reference: the Conv2d(k=1) layers w of FNO2d
// (2d_FPE/FNOModules.py:226-232), whose weight gradient autograd forms as a GEMM over the points.
#pragma once
#include "common.h"

namespace blindno {

// 1x1-conv weight / bias gradient of the wide fields (the C = 12 heads) on the matrix cores:
// dWc[o][i] = sum_p dz[o][p] f(x)[i][p] is a C x C GEMM over the points (K), 16 points per
// four v_mfma_f32_16x16x4f32: lane (c16, g4) loads float4 dz[o = c16][p0 + 4 g4 ..] (A) and
// f(x)[i = c16][p0 + 4 g4 ..] (B), component s feeding step s (the same point order for both
// operands), and column C of B is 1.0 so D[o][C] accumulates the bias gradient.  The VALU
// kernel (fields.hip, conv_wgrad_kernel) staged both fields in LDS and spent ~2 C^2 LDS reads
// per point.  Waves add their 16 x 16 blocks in wave order.
// Workgroup bx of gx over the points, weight group grp of gy (256 threads):
// partial[bx][grp][C*C + C] as conv_wgrad_kernel.
template <int ACT>
__device__ __forceinline__ void conv_wgrad_mfma_block(const float* __restrict__ dz,
                                                      const float* __restrict__ x,
                                                      float* __restrict__ partial, int C, int HW,
                                                      int Bg, int bx, int gx, int grp, int gy) {
  typedef float f32x4 __attribute__((ext_vector_type(4)));
  __shared__ f32x4 sacc[4][64];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int c16 = lane & 15, g4 = lane >> 4;
  const int64_t gofs = (int64_t)grp * Bg * C * HW;
  dz += gofs;
  x += gofs;
  const int cpn = (HW + 15) >> 4;                  // 16-point chunks per sample
  const int64_t nch = (int64_t)Bg * cpn;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  const bool vec = (HW & 3) == 0;
  for (int64_t ch = (int64_t)bx * 4 + wave; ch < nch; ch += (int64_t)gx * 4) {
    const int n = (int)(ch / cpn);
    const int p = (int)(ch - (int64_t)n * cpn) * 16 + 4 * g4;
    float a[4] = {0.f, 0.f, 0.f, 0.f}, b[4] = {0.f, 0.f, 0.f, 0.f};
    if (c16 < C) {
      const float* dr = dz + ((int64_t)n * C + c16) * HW;
      const float* xr = x + ((int64_t)n * C + c16) * HW;
      if (vec && p + 3 < HW) {
        const float4 va = *reinterpret_cast<const float4*>(dr + p);
        const float4 vb = *reinterpret_cast<const float4*>(xr + p);
        a[0] = va.x; a[1] = va.y; a[2] = va.z; a[3] = va.w;
        b[0] = vb.x; b[1] = vb.y; b[2] = vb.z; b[3] = vb.w;
      } else {
#pragma unroll
        for (int s = 0; s < 4; ++s)
          if (p + s < HW) { a[s] = dr[p + s]; b[s] = xr[p + s]; }
      }
      if (ACT) {
#pragma unroll
        for (int s = 0; s < 4; ++s) b[s] = gelu_f(b[s]);
      }
    } else if (c16 == C) {
#pragma unroll
      for (int s = 0; s < 4; ++s) b[s] = p + s < HW ? 1.0f : 0.f;   // bias column
    }
#pragma unroll
    for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], b[s], acc, 0, 0, 0);
  }
  sacc[wave][lane] = acc;
  __syncthreads();
  // D[o = 4 g4 + r][i = c16] at lane (g4, c16), reg r
  const int np = C * C + C;
  float* pp = partial + ((int64_t)bx * gy + grp) * np;
  for (int e = threadIdx.x; e < np; e += 256) {
    const int o = e < C * C ? e / C : e - C * C;
    const int i = e < C * C ? e - (e / C) * C : C;
    const int ln = 16 * (o >> 2) + i, r = o & 3;
    pp[e] = ((sacc[0][ln][r] + sacc[1][ln][r]) + sacc[2][ln][r]) + sacc[3][ln][r];
  }
}

// the conv_wgrad_mfma_block shapes (fields.hip's launcher and the hosted form)
__host__ __forceinline__ bool conv_wgrad_mfma_ok(int C, int64_t HW) {
  return C >= 5 && C <= 15 && HW < INT32_MAX / 16;
}

}  // namespace blindno
