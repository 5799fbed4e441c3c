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

// The spectral weight gradient's packed layout dWt (m2, K1 = 2 m1, Ci, Co) complex (the mix
// GEMM's) -> the reference layout (Ci, Co, m1, m2) of weights1 (kept rows j < m1) and weights2
// (rows m1 .. 2 m1 - 1): what blindno_unpack_w2d does as its own launch, folded into the store
// of the kernel that finishes dWt (the deferred finalisation's mix or reduction).  Only for
// non-overlapping kept rows (2 m1 < P1, K1 = 2 m1).
struct W2dUnpack {
  float* d1;
  float* d2;
  int Ci, Co, m1, m2;
};
__device__ __forceinline__ float* w2d_unpacked(const W2dUnpack& u, int e) {
  const int o = e % u.Co;
  int t = e / u.Co;
  const int i = t % u.Ci;
  t /= u.Ci;
  const int j = t % (2 * u.m1), k = t / (2 * u.m1);
  const bool second = j >= u.m1;
  return (second ? u.d2 : u.d1) +
         ((((int64_t)i * u.Co + o) * u.m1 + (second ? j - u.m1 : j)) * u.m2 + k) * 2;
}

// Spectral weight gradient (the mix GEMM over the samples, spectral.hip / fields.hip hosts):
// dWt[k,j,i,o] = sum_n conj(X[n,k,i,j]) G[n,k,o,j]
// workgroup (bx, by, bz) of (gx, gy, gz), kBlock threads:
//   by = sample slice: out[y][idx] = sum over this slice's samples (partials when gy > 1,
//   reduced in fixed order afterwards)
//   bz = weight group: its Bn / gz samples only; out[(y G + g)][idx]
// upk (gy == 1 only): dWt of weight group bz stored unpacked through uw (wgrad.h)
__device__ __forceinline__ void mix_wgrad_block(const float2* __restrict__ X,
                                                const float2* __restrict__ G,
                                                float2* __restrict__ out, int Bn, int Ci, int Co,
                                                int K1, int m2, int bx, int by, int bz, int gx,
                                                int gy, int gz, bool upk = false,
                                                W2dUnpack uw = W2dUnpack{}) {
  const int total = m2 * K1 * Ci * Co;
  const int Bg = Bn / gz, grp = bz;
  const int ns = (Bg + gy - 1) / gy;
  const int n0 = grp * Bg + by * ns, n1 = min(grp * Bg + Bg, n0 + ns);
  const int sX = m2 * Ci * K1, sG = m2 * Co * K1;
  for (int idx = bx * kBlock + threadIdx.x; idx < total; idx += gx * kBlock) {
    const int o = idx % Co;
    int t = idx / Co;
    const int i = t % Ci;
    t /= Ci;
    const int j = t % K1;
    const int k = t / K1;
    const float2* xp = X + ((int64_t)n0 * m2 + k) * Ci * K1 + i * K1 + j;
    const float2* gp = G + ((int64_t)n0 * m2 + k) * Co * K1 + o * K1 + j;
    // fp64 accumulation: the sum over hundreds of snapshots cancels heavily once the weights
    // are trained (terms ~1e3 x the result for the encoder's first layer), and an fp32 running
    // sum then loses ~n eps of the terms' scale -- measured 4e-3 rel-L2 on
    // FNO_input.spectral_list.0.weights2 vs fp64 at config C, against 6e-5 for the reference's
    // blocked fp32 GEMM.  The kernel is memory-bound; the fp64 FMAs are free.
    double re = 0.0, im = 0.0;
#pragma unroll 4
    for (int n = n0; n < n1; ++n, xp += sX, gp += sG) {
      const float2 a = *xp;
      const float2 g = *gp;
      re = fma((double)a.x, (double)g.x, fma((double)a.y, (double)g.y, re));
      im = fma((double)a.x, (double)g.y, fma(-(double)a.y, (double)g.x, im));
    }
    if (upk) {
      float* d = w2d_unpacked(uw, idx);
      d[0] = (float)re;
      d[1] = (float)im;
    } else {
      out[((int64_t)by * gz + grp) * total + idx] = make_float2((float)re, (float)im);
    }
  }
}


constexpr int kMixMaxGw = 4;
struct MixWgradJob {
  const float2* X;
  const float2* Gs;
  float2* out;
  int Bn, Ci, Co, K1, m2, gx, gy, gz;
  int um1;                          // > 0: dWt stored unpacked (K1 = 2 um1, gy = 1) at
  float* u1[kMixMaxGw];             // weights1 / weights2 gradients of group g
  float* u2[kMixMaxGw];
};

// the conv_wgrad_mfma_block shapes (fields.hip's launcher and the hosted form)
__host__ __forceinline__ bool conv_wgrad_mfma_ok(int C, int64_t HW) {
  return C >= 5 && C <= 15 && HW < INT32_MAX / 16;
}

}  // namespace blindno
