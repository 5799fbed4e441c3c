// Field kernels of the FNO body: lift (fc0 + pad), 1x1-conv weight-gradient partial reductions,
// the projection MLP fallback for wide fields (fc1 -> GELU -> fc2, forward and backward; the
// narrow ones run on the matrix cores in project.hip), the snapshot-bag mean, loss, metrics and
// Adam.  The inverse row transform with its fused epilogue lives in rowinv.hip.
//
// Reference: FNO2d.forward 2d_FPE/FNOModules.py:218-240, FNO1d.forward
// 1d_FPE/FNOModules.py:99-122, NIOFP2D_FNO bag mean 2d_FPE/NIOModules.py:565-575,
// train loop 2d_FPE/train_fno.py:116-146.
//
// Mapping rules: row kernels put one wave on one grid row (lanes = w,
// NQ = ceil(P2/64) points per lane) and keep ALL channels of a point in registers, so the
// 1x1 conv and GELU happen once per point; per-row spectral coefficients are wave-uniform
// and come through scalar loads.
#include "common.h"
#include "blindno.h"
#include "kernels.h"
#include "wgrad.h"
#include "packw.h"
#include "liftw.h"

using namespace blindno;

// the heads' lift input and weight gradients in one launch (0: two launches, for A/B)
#ifndef LIFT_BWD_BOTH
#define LIFT_BWD_BOTH 1
#endif

namespace {

// ---------------------------------------------------------------- lift
// Grouped launches (G > 1): samples n = g Bg + n' of group g use that group's weights at
// w + g wgs and read the shared input sample n' (two FNO heads on one field).
// lift_fwd_pt_kernel: a lane quad per point (channels-last input, NCHW output coalesced
// across w).
template <int CM>
__global__ __launch_bounds__(kBlock) void lift_fwd_pt_kernel(const float* __restrict__ in,
                                                             const float* __restrict__ w0,
                                                             const float* __restrict__ b0,
                                                             float* __restrict__ x0, int Bn,
                                                             int N1, int N2, int Cin, int C,
                                                             int P1, int P2, int Bg,
                                                             int64_t wgs) {
  // four threads per point (a lane quad): lane q computes channels q, q + 4, ... (CM / 4 of
  // them) from the point's Cin inputs, so each lane runs a quarter of the C x Cin products
  // and four times as many waves hide the input reads' latency
  constexpr int CQ = CM / 4;
  const int q = threadIdx.x & 3;
  const int64_t HW = (int64_t)P1 * P2;
  const int64_t total = (int64_t)Bn * HW;
  for (int64_t idx = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 2; idx < total;
       idx += ((int64_t)gridDim.x * blockDim.x) >> 2) {
    const int64_t n = idx / HW;
    const int64_t s = idx - n * HW;
    const int h = (int)(s / P2), w = (int)(s - (s / P2) * P2);
    float* xp = x0 + n * C * HW + s;
    if (h >= N1 || w >= N2) {
      for (int c = q; c < C; c += 4) xp[c * HW] = 0.f;
      continue;
    }
    const int g = (int)(n / Bg);
    const int64_t ni = n - (int64_t)g * Bg;
    const float* wg = w0 + g * wgs;
    const float* bg = b0 + g * wgs;
    const float* ip = in + ((ni * N1 + h) * N2 + w) * Cin;
    float acc[CQ];
#pragma unroll
    for (int k = 0; k < CQ; ++k) acc[k] = q + 4 * k < C ? bg[q + 4 * k] : 0.f;
    for (int j = 0; j < Cin; ++j) {
      const float v = ip[j];
#pragma unroll
      for (int k = 0; k < CQ; ++k)
        if (q + 4 * k < C) acc[k] = fmaf(wg[(q + 4 * k) * Cin + j], v, acc[k]);
    }
#pragma unroll
    for (int k = 0; k < CQ; ++k)
      if (q + 4 * k < C) xp[(q + 4 * k) * HW] = acc[k];
  }
}

__global__ __launch_bounds__(kBlock) void lift_fwd_kernel(const float* __restrict__ in,
                                                          const float* __restrict__ w0,
                                                          const float* __restrict__ b0,
                                                          float* __restrict__ x0, int Bn, int N1,
                                                          int N2, int Cin, int C, int P1,
                                                          int P2, int Bg, int64_t wgs) {
  const int64_t total = (int64_t)Bn * C * P1 * P2;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int w = (int)(idx % P2);
    int64_t t = idx / P2;
    const int h = (int)(t % P1);
    t /= P1;
    const int c = (int)(t % C);
    const int n = (int)(t / C);
    float v = 0.f;
    if (h < N1 && w < N2) {
      const int g = n / Bg, ni = n - g * Bg;
      const float* wg = w0 + g * wgs;
      const float* ip = in + (((int64_t)ni * N1 + h) * N2 + w) * Cin;
      v = b0[g * wgs + c];
      for (int j = 0; j < Cin; ++j) v = fmaf(wg[c * Cin + j], ip[j], v);
    }
    x0[idx] = v;
  }
}

__global__ __launch_bounds__(kBlock) void lift_bwd_in_kernel(const float* __restrict__ dx0,
                                                             const float* __restrict__ w0,
                                                             float* __restrict__ d_in, int Bn,
                                                             int N1, int N2, int Cin, int C,
                                                             int P1, int P2, int G, int64_t wgs) {
  // d_in has Bn samples; with G groups the gradient sums over the groups' samples g Bn + n
  const int64_t total = (int64_t)Bn * N1 * N2 * Cin;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int j = (int)(idx % Cin);
    int64_t t = idx / Cin;
    const int w = (int)(t % N2);
    t /= N2;
    const int h = (int)(t % N1);
    const int n = (int)(t / N1);
    float v = 0.f;
    for (int g = 0; g < G; ++g)
      for (int c = 0; c < C; ++c)
        v = fmaf(w0[g * wgs + c * Cin + j], dx0[((((int64_t)g * Bn + n) * C + c) * P1 + h) * P2 + w], v);
    d_in[idx] = v;
  }
}

// Wide lifts of the FNO heads (Cin, C <= 16, Cin % 4 == 0; two heads grouped): one thread per
// point of the padded P1 x P2 grid, every channel in registers, the weights of all groups in LDS
// (broadcast reads), the point's Cin inputs as float4 loads, 32-bit index math with launch-
// invariant divisors.  Forward writes all C channels of x0 (zero on the padding); the input
// gradient sums the groups' fields: d_in[n'][h][w][j] = sum_g sum_c W_g[c][j] dx0[g Bg + n'][c].
template <int CIN, int CM>
__global__ __launch_bounds__(kBlock) void lift_fwd_wide_kernel(
    const float* __restrict__ in, const float* __restrict__ w0, const float* __restrict__ b0,
    float* __restrict__ x0, int Bn, int N1, int N2, int C, int P1, int P2, int Bg, int G,
    int64_t wgs, FastDiv dHW, FastDiv dP2, BagIn bi) {
  lift_fwd_wide_block<CIN, CM>(in, w0, b0, x0, Bn, N1, N2, C, P1, P2, Bg, G, wgs, dHW, dP2, bi,
                               blockIdx.x, gridDim.x);
}

template <int CIN, int CM>
__device__ __forceinline__ void lift_bwd_in_wide_block(
    const float* __restrict__ dx0, const float* __restrict__ w0, float* __restrict__ d_in, int Bn,
    int N1, int N2, int C, int P1, int P2, int G, int64_t wgs, FastDiv dS, FastDiv dN2, int bx,
    int gx, BagIn bi) {
  __shared__ float sw[kLiftMaxG][CM * CIN];
  for (int e = threadIdx.x; e < G * CM * CIN; e += blockDim.x) {
    const int g = e / (CM * CIN), q = e - g * (CM * CIN);
    const int c = q / CIN, j = q - c * CIN;
    sw[g][q] = c < C ? w0[g * wgs + c * CIN + j] : 0.f;
  }
  __syncthreads();
  const unsigned S = (unsigned)(N1 * N2), HW = (unsigned)(P1 * P2);
  const unsigned total = (unsigned)Bn * S;
  for (unsigned idx = bx * kBlock + threadIdx.x; idx < total; idx += gx * kBlock) {
    const unsigned n = dS.div(idx), s = idx - n * S;
    const unsigned h = dN2.div(s), w = s - h * (unsigned)N2;
    float acc[CIN];
#pragma unroll
    for (int j = 0; j < CIN; ++j) acc[j] = 0.f;
    for (int g = 0; g < G; ++g) {
      const float* dp = dx0 + ((size_t)(g * Bn + n) * C) * HW + h * (unsigned)P2 + w;
      const float* wg = sw[g];
#pragma unroll
      for (int c = 0; c < CM; ++c) {
        if (c >= C) break;
        const float d = dp[(size_t)c * HW];
#pragma unroll
        for (int j = 0; j < CIN; ++j) acc[j] = fmaf(wg[c * CIN + j], d, acc[j]);
      }
    }
    if (bi.u) {
      // d ubar: bagmean_bwd_kernel's reduction of d h over the channels
      float v = 0.f;
#pragma unroll
      for (int j = 0; j < CIN; ++j) v = fmaf(bi.w[j * 3 + 2] * bi.invLb, acc[j], v);
      d_in[idx] = v;
      continue;
    }
    float4* op = reinterpret_cast<float4*>(d_in + (size_t)idx * CIN);
#pragma unroll
    for (int q = 0; q < CIN / 4; ++q) op[q] = make_float4(acc[4 * q], acc[4 * q + 1], acc[4 * q + 2], acc[4 * q + 3]);
  }
}

template <int CIN, int CM>
__global__ __launch_bounds__(kBlock) void lift_bwd_in_wide_kernel(
    const float* __restrict__ dx0, const float* __restrict__ w0, float* __restrict__ d_in, int Bn,
    int N1, int N2, int C, int P1, int P2, int G, int64_t wgs, FastDiv dS, FastDiv dN2) {
  lift_bwd_in_wide_block<CIN, CM>(dx0, w0, d_in, Bn, N1, N2, C, P1, P2, G, wgs, dS, dN2, blockIdx.x,
                                  gridDim.x, BagIn{});
}

// Tiled outer-product reductions: partial[block][a*Cb + b] = sum_p A[a][p] B[b][p] and
// partial[block][Ca*Cb + a] = sum_p A[a][p] over the block's tile of TP points, staged in
// LDS with coalesced loads (rows padded by one float: conflict-free column sweeps).
constexpr int TP = 256;

// lift: A = dx0 on the N1 x N2 domain (NCHW, padded strides), B = in (channels-last).
// Workgroups sweep tiles grid-stride and keep their sums in registers (<= 4 parameters
// per thread), so the partial count is the (bounded) grid size.
constexpr int PPT = 4;

__global__ __launch_bounds__(kBlock) void lift_bwd_w_kernel(const float* __restrict__ dx0,
                                                            const float* __restrict__ in,
                                                            float* __restrict__ partial, int Bn,
                                                            int N1, int N2, int Cin, int C,
                                                            int P1, int P2) {
  // blockIdx.y = group g: dx0 samples g Bn + n against the shared input sample n;
  // partial[blockIdx.x][g][np]
  extern __shared__ float sm[];
  const int grp = blockIdx.y;
  dx0 += (int64_t)grp * Bn * C * P1 * P2;
  float* sa = sm;                       // [C][TP+1]
  float* sb = sa + C * (TP + 1);        // [Cin][TP+1]
  const int64_t npts = (int64_t)Bn * N1 * N2;
  const int64_t ntiles = (npts + TP - 1) / TP;
  const int t = threadIdx.x;
  const int np = C * Cin + C;
  float acc[PPT];
#pragma unroll
  for (int e = 0; e < PPT; ++e) acc[e] = 0.f;
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int64_t p0 = tile * TP;
    {
      const int64_t q = p0 + t;
      const bool ok = q < npts;
      int n = 0, h = 0, w = 0;
      if (ok) {
        w = (int)(q % N2);
        const int64_t r = q / N2;
        h = (int)(r % N1);
        n = (int)(r / N1);
      }
      for (int c = 0; c < C; ++c)
        sa[c * (TP + 1) + t] = ok ? dx0[(((int64_t)n * C + c) * P1 + h) * P2 + w] : 0.f;
    }
    for (int e = t; e < TP * Cin; e += blockDim.x) {
      const int p = e / Cin, j = e % Cin;
      const int64_t q = p0 + p;
      sb[j * (TP + 1) + p] = q < npts ? in[q * Cin + j] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int e = 0; e < PPT; ++e) {
      const int pr = t + e * kBlock;
      if (pr >= np) continue;
      float a2 = acc[e];
      if (pr < C * Cin) {
        const float* a = sa + (pr / Cin) * (TP + 1);
        const float* b = sb + (pr % Cin) * (TP + 1);
        for (int p = 0; p < TP; ++p) a2 = fmaf(a[p], b[p], a2);
      } else {
        const float* a = sa + (pr - C * Cin) * (TP + 1);
        for (int p = 0; p < TP; ++p) a2 += a[p];
      }
      acc[e] = a2;
    }
    __syncthreads();
  }
#pragma unroll
  for (int e = 0; e < PPT; ++e) {
    const int pr = t + e * kBlock;
    if (pr < np) partial[((int64_t)blockIdx.x * gridDim.y + grp) * np + pr] = acc[e];
  }
}

// conv: A = dz, B = f(x) (NCHW, HW points per sample); tiles never straddle samples.
// blockIdx.y = group: samples [g Bn', (g+1) Bn') with Bn' = ntiles / tiles_per_n;
// partial[blockIdx.x][g][np]
template <int ACT>
__global__ __launch_bounds__(kBlock) void conv_wgrad_kernel(const float* __restrict__ dz,
                                                            const float* __restrict__ x,
                                                            float* __restrict__ partial, int C,
                                                            int64_t HW, int tiles_per_n,
                                                            int64_t ntiles) {
  extern __shared__ float sm[];
  float* sa = sm;
  float* sb = sa + C * (TP + 1);
  const int t = threadIdx.x;
  const int np = C * C + C;
  const int grp = blockIdx.y;
  const int64_t gofs = (int64_t)grp * (ntiles / tiles_per_n) * C * HW;
  dz += gofs;
  x += gofs;
  float acc[PPT];
#pragma unroll
  for (int e = 0; e < PPT; ++e) acc[e] = 0.f;
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int64_t n = tile / tiles_per_n;
    const int64_t s0 = (tile % tiles_per_n) * TP;
    const bool ok = s0 + t < HW;
    for (int c = 0; c < C; ++c) {
      const int64_t off = (n * C + c) * HW + s0 + t;
      float a = 0.f, b = 0.f;
      if (ok) {
        a = dz[off];
        b = x[off];
        if (ACT) b = gelu_f(b);
      }
      sa[c * (TP + 1) + t] = a;
      sb[c * (TP + 1) + t] = b;
    }
    __syncthreads();
#pragma unroll
    for (int e = 0; e < PPT; ++e) {
      const int pr = t + e * kBlock;
      if (pr >= np) continue;
      float a2 = acc[e];
      if (pr < C * C) {
        const float* a = sa + (pr / C) * (TP + 1);
        const float* b = sb + (pr % C) * (TP + 1);
        for (int p = 0; p < TP; ++p) a2 = fmaf(a[p], b[p], a2);
      } else {
        const float* a = sa + (pr - C * C) * (TP + 1);
        for (int p = 0; p < TP; ++p) a2 += a[p];
      }
      acc[e] = a2;
    }
    __syncthreads();
  }
#pragma unroll
  for (int e = 0; e < PPT; ++e) {
    const int pr = t + e * kBlock;
    if (pr < np) partial[((int64_t)blockIdx.x * gridDim.y + grp) * np + pr] = acc[e];
  }
}

// Lift (fc0) weight / bias gradient of the wide heads on the matrix cores:
// dW0[c][j] = sum_p dx0[c][p] in[p][j], db0[c] = sum_p dx0[c][p] over the N1 x N2 points --
// a C x (Cin + 1) GEMM over the points.  16 points per chunk (one run along w; N2 % 16 == 0,
// checked by the launcher), four v_mfma_f32_16x16x4f32 per 16-column tile of (j, 1): lane
// (c16, g4) feeds float4 dx0[c = c16][h][w0 + 4 g4 ..] (A) and in[p][j = 16 jt + c16] at
// the same four points (B; column Cin is 1.0).  Waves add their blocks in wave order; the
// partial layout is lift_bwd_w_kernel's: partial[blockIdx.x][g][C Cin + C].
// (workgroup (bx, grp) of (gx, gy) explicit: lift_bwd_both_kernel hosts it)
template <int JT>
__device__ __forceinline__ void lift_bwd_w_mfma_block(const float* __restrict__ dx0,
                                                      const float* __restrict__ in,
                                                      float* __restrict__ partial, int Bn, int N1,
                                                      int N2, int Cin, int C, int P1, int P2,
                                                      int bx, int gx, int grp, int gy,
                                                      BagIn bi) {
  typedef float f32x4 __attribute__((ext_vector_type(4)));
  __shared__ f32x4 sacc[4][JT][64];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int c16 = lane & 15, g4 = lane >> 4;
  dx0 += (int64_t)grp * Bn * C * P1 * P2;
  const int cpr = N2 >> 4;                         // 16-point chunks per grid row
  const int64_t nch = (int64_t)Bn * N1 * cpr;
  f32x4 acc[JT];
#pragma unroll
  for (int t = 0; t < JT; ++t) acc[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
  for (int64_t ch = (int64_t)bx * 4 + wave; ch < nch; ch += (int64_t)gx * 4) {
    const int64_t r = ch / cpr;                    // grid row (n, h)
    const int w0 = (int)(ch - r * cpr) * 16 + 4 * g4;
    const int n = (int)(r / N1), h = (int)(r - (r / N1) * N1);
    float a[4] = {0.f, 0.f, 0.f, 0.f};
    if (c16 < C) {
      const float4 v = *reinterpret_cast<const float4*>(dx0 + (((int64_t)n * C + c16) * P1 + h) * P2 + w0);
      a[0] = v.x; a[1] = v.y; a[2] = v.z; a[3] = v.w;
    }
    const float* ip = in + (r * N2 + w0) * Cin;    // point (n, h, w0), channels-last
    float bu[4], bg0[4], bg1[4];                   // bag input: ubar and the grid at the 4 points
    if (bi.u) {
      const int64_t pp = r * N2 + w0;
      const int sp = h * N2 + w0;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        bu[s] = bi.u[pp + s];
        bg0[s] = bi.grid[2 * (sp + s)];
        bg1[s] = bi.grid[2 * (sp + s) + 1];
      }
    }
#pragma unroll
    for (int t = 0; t < JT; ++t) {
      const int j = 16 * t + c16;
      float b[4];
      if (bi.u) {
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          if (j < Cin) {
            float a = bi.bias[j];
            a = fmaf(bi.w[j * 3], bg0[s], a);
            a = fmaf(bi.w[j * 3 + 1], bg1[s], a);
            b[s] = fmaf(bi.w[j * 3 + 2] * bi.invL, bu[s], a);
          } else {
            b[s] = j == Cin ? 1.0f : 0.f;
          }
        }
      } else {
#pragma unroll
        for (int s = 0; s < 4; ++s) b[s] = j < Cin ? ip[s * Cin + j] : (j == Cin ? 1.0f : 0.f);
      }
#pragma unroll
      for (int s = 0; s < 4; ++s) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], b[s], acc[t], 0, 0, 0);
    }
  }
#pragma unroll
  for (int t = 0; t < JT; ++t) sacc[wave][t][lane] = acc[t];
  __syncthreads();
  // D[c = 4 g4 + r][j = 16 t + c16]
  const int np = C * Cin + C;
  float* pp = partial + ((int64_t)bx * gy + grp) * np;
  for (int e = threadIdx.x; e < np; e += 256) {
    const int c = e < C * Cin ? e / Cin : e - C * Cin;
    const int j = e < C * Cin ? e - (e / Cin) * Cin : Cin;
    const int t = j >> 4, ln = 16 * (c >> 2) + (j & 15), rr = c & 3;
    pp[e] = ((sacc[0][t][ln][rr] + sacc[1][t][ln][rr]) + sacc[2][t][ln][rr]) + sacc[3][t][ln][rr];
  }
}

template <int JT>
__global__ __launch_bounds__(256) void lift_bwd_w_mfma_kernel(const float* __restrict__ dx0,
                                                              const float* __restrict__ in,
                                                              float* __restrict__ partial, int Bn,
                                                              int N1, int N2, int Cin, int C,
                                                              int P1, int P2) {
  lift_bwd_w_mfma_block<JT>(dx0, in, partial, Bn, N1, N2, Cin, C, P1, P2, blockIdx.x, gridDim.x,
                            blockIdx.y, gridDim.y, BagIn{});
}

// The heads' lift backward in one launch: its input gradient (workgroups [0, nbi)) and its
// weight / bias gradient partials (the next nchunk x G) read the same dx0 and are independent;
// the rest (nbm) runs the spectral weight gradient of the heads' first layer, whose column pass
// has just run (wgrad.h).  Each part keeps the grid of its own launch (bit-identical results).
template <int JT>
__global__ __launch_bounds__(256) void lift_bwd_both_kernel(
    const float* __restrict__ dx0, const float* __restrict__ w0, float* __restrict__ d_in,
    const float* __restrict__ in, float* __restrict__ partial, int Bn, int N1, int N2, int Cin,
    int C, int P1, int P2, int G, int64_t wgs, FastDiv dS, FastDiv dN2, int nbi, int nchunk,
    MixWgradJob mw, BagIn bi) {
  const int b = blockIdx.x;
  if (b < nbi) {
    lift_bwd_in_wide_block<12, 16>(dx0, w0, d_in, Bn, N1, N2, C, P1, P2, G, wgs, dS, dN2, b, nbi,
                                   bi);
    return;
  }
  int r = b - nbi;
  if (r < nchunk * G) {
    lift_bwd_w_mfma_block<JT>(dx0, in, partial, Bn, N1, N2, Cin, C, P1, P2, r % nchunk, nchunk,
                              r / nchunk, G, bi);
    return;
  }
  r -= nchunk * G;
  mix_wgrad_block(mw.X, mw.Gs, mw.out, mw.Bn, mw.Ci, mw.Co, mw.K1, mw.m2, r % mw.gx,
                  (r / mw.gx) % mw.gy, r / (mw.gx * mw.gy), mw.gx, mw.gy, mw.gz);
}

template <int ACT>
__global__ __launch_bounds__(256) void conv_wgrad_mfma_kernel(const float* __restrict__ dz,
                                                              const float* __restrict__ x,
                                                              float* __restrict__ partial, int C,
                                                              int HW, int Bg) {
  conv_wgrad_mfma_block<ACT>(dz, x, partial, C, HW, Bg, blockIdx.x, gridDim.x, blockIdx.y,
                             gridDim.y);
}

// out[p] = sum_c partial[c][p], deterministic.  A workgroup owns PB <= 64 consecutive
// parameters and splits the chunks into S = 1024 / PB slices (thread t: parameter t % PB,
// slice t / PB); every slice sums its chunks with four independent accumulators in a fixed
// order, then the slices are added in slice order.  Small parameter counts (the lift's 16,
// a conv's 20) therefore still use all 1024 threads instead of 16 lanes.
// (e0, e1): only parameters p in [e0, e1) are stored, at out[p - e0] -- a piece of a reduction
// whose parameters land in different buffers (blindno_reduce_partials_pieces)
// upk: out is a packed spectral weight gradient, stored unpacked (wgrad.h, W2dUnpack)
__device__ __forceinline__ void reduce_partials_block(const float* __restrict__ partial,
                                                      float* __restrict__ out, int nchunk, int np,
                                                      int PB, int blk, float* red, int e0 = 0,
                                                      int e1 = INT32_MAX, bool upk = false,
                                                      W2dUnpack uw = W2dUnpack{}) {
  const int S = 1024 / PB;
  const int t = threadIdx.x;
  const int pl = t % PB, sl = t / PB;
  const int p = blk * PB + pl;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  if (sl < S && p < np) {
    int c = sl;
    for (; c + 3 * S < nchunk; c += 4 * S) {
      a0 += partial[(int64_t)c * np + p];
      a1 += partial[(int64_t)(c + S) * np + p];
      a2 += partial[(int64_t)(c + 2 * S) * np + p];
      a3 += partial[(int64_t)(c + 3 * S) * np + p];
    }
    for (; c < nchunk; c += S) a0 += partial[(int64_t)c * np + p];
  }
  red[t] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (sl == 0 && p < np && p >= e0 && p < e1) {
    float v = red[pl];
    for (int k = 1; k < S; ++k) v += red[k * PB + pl];
    if (upk)
      w2d_unpacked(uw, p >> 1)[p & 1] = v;
    else
      out[p - e0] = v;
  }
}

__global__ __launch_bounds__(1024) void reduce_partials_kernel(const float* __restrict__ partial,
                                                               float* __restrict__ out,
                                                               int nchunk, int np, int PB) {
  __shared__ float red[1024];
  reduce_partials_block(partial, out, nchunk, np, PB, blockIdx.x, red);
}

// Several reductions in one launch (the deferred weight-gradient reductions of one backward
// pass, blindno.ops.deferred_reductions): segment i owns workgroups [cum[i], cum[i+1]), each
// reduced exactly as by reduce_partials_kernel, so the results are bit-identical to separate
// launches.  A segment may be a piece of a reduction: its workgroups blk0[i] .. of that
// reduction's block grid (same PB, so the same summation order), storing only parameters
// [e0, e1) at out[p - e0] (the gradients written straight into an optimizer's flat buffer).
// Segments are passed by value (a graph capture bakes them in).
// A segment with upk[i] >= 0 is a packed spectral weight gradient stored unpacked through
// ut[upk[i]] (whole reductions only).
constexpr int kRedSegs = 48, kRedUnpack = 8;
struct ReduceSegs {
  const float* src[kRedSegs];
  float* out[kRedSegs];
  int nchunk[kRedSegs], np[kRedSegs], pb[kRedSegs], blk0[kRedSegs], e0[kRedSegs], e1[kRedSegs];
  int upk[kRedSegs];
  W2dUnpack ut[kRedUnpack];
  int cum[kRedSegs + 1];
  int nseg;
};

__global__ __launch_bounds__(1024) void reduce_partials_multi_kernel(ReduceSegs segs) {
  __shared__ float red[1024];
  const int b = blockIdx.x;
  int sg = 0;
  while (sg + 1 < segs.nseg && segs.cum[sg + 1] <= b) ++sg;    // uniform scan
  const int u = segs.upk[sg];
  reduce_partials_block(segs.src[sg], segs.out[sg], segs.nchunk[sg], segs.np[sg], segs.pb[sg],
                        segs.blk0[sg] + b - segs.cum[sg], red, segs.e0[sg], segs.e1[sg], u >= 0,
                        segs.ut[u >= 0 ? u : 0]);
}

// ---------------------------------------------------------------- projection MLP
// Forward: one lane per crop point, all hidden units looped; the MLP weights are staged in
// LDS once per workgroup and read as wave-wide broadcasts.
template <int CM, int COM>
__global__ __launch_bounds__(kBlock) void project_fwd_kernel(
    const float* __restrict__ z, const float* __restrict__ w1, const float* __restrict__ b1,
    const float* __restrict__ w2, const float* __restrict__ b2, float* __restrict__ out, int Bn,
    int C, int P1, int P2, int Ho, int Wo, int Hd, int Cout, int ostride, int ooff) {
  extern __shared__ float smp[];
  float* sw1 = smp;                 // [Hd][CM] (zero padded)
  float* sb1 = sw1 + Hd * CM;       // [Hd]
  float* sw2 = sb1 + Hd;            // [Hd][COM]
  for (int e = threadIdx.x; e < Hd * CM; e += blockDim.x) {
    const int j = e / CM, i = e % CM;
    sw1[e] = i < C ? w1[j * C + i] : 0.f;
  }
  for (int e = threadIdx.x; e < Hd; e += blockDim.x) sb1[e] = b1[e];
  for (int e = threadIdx.x; e < Hd * COM; e += blockDim.x) {
    const int j = e / COM, c = e % COM;
    sw2[e] = c < Cout ? w2[c * Hd + j] : 0.f;
  }
  __syncthreads();
  const int64_t HW = (int64_t)P1 * P2;
  const unsigned total = (unsigned)((int64_t)Bn * Ho * Wo);
  for (unsigned idx = blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += gridDim.x * blockDim.x) {
    const unsigned w = idx % (unsigned)Wo, t = idx / (unsigned)Wo;
    const unsigned h = t % (unsigned)Ho, n = t / (unsigned)Ho;
    float zi[CM];
    const float* zp = z + (int64_t)n * C * HW + (int64_t)h * P2 + w;
#pragma unroll
    for (int i = 0; i < CM; ++i) zi[i] = i < C ? zp[i * HW] : 0.f;
    float acc[COM];
#pragma unroll
    for (int c = 0; c < COM; ++c) acc[c] = c < Cout ? b2[c] : 0.f;
    for (int j = 0; j < Hd; ++j) {
      float hv = sb1[j];
#pragma unroll
      for (int i = 0; i < CM; ++i) hv = fmaf(sw1[j * CM + i], zi[i], hv);
      const float a = gelu_f(hv);
#pragma unroll
      for (int c = 0; c < COM; ++c) acc[c] = fmaf(sw2[j * COM + c], a, acc[c]);
    }
    float* op = out + idx * ostride + ooff;
#pragma unroll
    for (int c = 0; c < COM; ++c)
      if (c < Cout) op[c] = acc[c];
  }
}

// Backward for wide fields (C > 15, the 1D heads; narrower ones run on the matrix cores,
// project.hip): lanes = crop points (64-point tiles), the 16 waves of a
// 1024-thread workgroup split the hidden units (JW each); weight-gradient contributions of a
// tile are summed over lanes (wave reduction) and accumulated in the wave's own LDS slots;
// dz is summed over waves through LDS.  One workgroup partial per parameter at the end.
template <int CM, int JW, int COM>
__global__ __launch_bounds__(1024) void project_bwd_wsum_kernel(
    const float* __restrict__ z, const float* __restrict__ w1, const float* __restrict__ b1,
    const float* __restrict__ w2, const float* __restrict__ dout, float* __restrict__ dz,
    float* __restrict__ partial, int Bn, int C, int P1, int P2, int Ho, int Wo, int Hd,
    int Cout, int ostride, int ooff, int dout_div) {
  constexpr int NWV = 16;
  constexpr int PJ = CM + 1 + COM;
  constexpr int RC = CM < 16 ? CM : 16;
  extern __shared__ float smw[];
  float* sz = smw;                          // [CM][64]
  float* sg = sz + CM * 64;                 // [COM][64]
  float* red = sg + COM * 64;               // [NWV][RC][64]
  float* sw1 = red + NWV * RC * 64;         // [Hd][CM]
  float* sb1 = sw1 + Hd * CM;               // [Hd]
  float* sw2 = sb1 + Hd;                    // [Hd][COM]
  float* acc = sw2 + Hd * COM;              // [Hd][PJ] then [COM]
  const int lane = threadIdx.x & 63;
  const int wave = uniform_int(threadIdx.x >> 6);
  const int j0 = wave * JW;
  for (int e = threadIdx.x; e < Hd * CM; e += blockDim.x) {
    const int j = e / CM, i = e % CM;
    sw1[e] = i < C ? w1[j * C + i] : 0.f;
  }
  for (int e = threadIdx.x; e < Hd; e += blockDim.x) sb1[e] = b1[e];
  for (int e = threadIdx.x; e < Hd * COM; e += blockDim.x) {
    const int j = e / COM, c = e % COM;
    sw2[e] = c < Cout ? w2[c * Hd + j] : 0.f;
  }
  for (int e = threadIdx.x; e < Hd * PJ + COM; e += blockDim.x) acc[e] = 0.f;
  const int64_t HW = (int64_t)P1 * P2;
  const int64_t npts = (int64_t)Bn * Ho * Wo;
  const int64_t ntiles = (npts + 63) / 64;
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int64_t p = tile * 64 + lane;
    const bool ok = p < npts;
    const unsigned pu = ok ? (unsigned)p : 0u;
    const unsigned w = pu % (unsigned)Wo, r = pu / (unsigned)Wo;
    const unsigned h = r % (unsigned)Ho, n = r / (unsigned)Ho;
    const int64_t zo = (int64_t)n * C * HW + (int64_t)h * P2 + w;
    __syncthreads();
    for (int r = wave; r < CM + COM; r += NWV) {   // CM + COM rows over the 16 waves
      if (r < CM) {
        sz[r * 64 + lane] = (ok && r < C) ? z[zo + r * HW] : 0.f;
      } else {
        const int c = r - CM;
        const unsigned q = pu % (unsigned)(Ho * Wo);
        sg[c * 64 + lane] = (ok && c < Cout)
            ? dout[((int64_t)(n / (unsigned)dout_div) * (Ho * Wo) + q) * ostride + ooff + c] : 0.f;
      }
    }
    __syncthreads();
    float zi[CM], gv[COM], dzp[CM];
#pragma unroll
    for (int i = 0; i < CM; ++i) {
      zi[i] = sz[i * 64 + lane];
      dzp[i] = 0.f;
    }
#pragma unroll
    for (int c = 0; c < COM; ++c) gv[c] = sg[c * 64 + lane];
    for (int q = 0; q < JW; ++q) {
      const int j = j0 + q;
      const float* wj = sw1 + j * CM;
      float hv = sb1[j];
#pragma unroll
      for (int i = 0; i < CM; ++i) hv = fmaf(wj[i], zi[i], hv);
      float a, dg;
      gelu_both(hv, a, dg);
      float da = 0.f;
#pragma unroll
      for (int c = 0; c < COM; ++c) da = fmaf(sw2[j * COM + c], gv[c], da);
      const float dh = da * dg;
      float* aj = acc + j * PJ;
#pragma unroll
      for (int i = 0; i < CM; ++i) {
        dzp[i] = fmaf(wj[i], dh, dzp[i]);
        if (i < C) {
          const float sv = wave_sum(dh * zi[i]);
          if (lane == 0) aj[i] += sv;
        }
      }
      const float sb = wave_sum(dh);
      if (lane == 0) aj[CM] += sb;
#pragma unroll
      for (int c = 0; c < COM; ++c) {
        if (c >= Cout) continue;
        const float sv = wave_sum(gv[c] * a);
        if (lane == 0) aj[CM + 1 + c] += sv;
      }
    }
    if (wave == 0) {
#pragma unroll
      for (int c = 0; c < COM; ++c) {
        if (c >= Cout) continue;
        const float sv = wave_sum(gv[c]);
        if (lane == 0) acc[Hd * PJ + c] += sv;
      }
    }
    // dz summed over the waves through LDS, RC channels at a time (keeps red within LDS at CM 32)
#pragma unroll
    for (int i0 = 0; i0 < CM; i0 += RC) {
      if (i0 >= C) break;                     // uniform
      if (i0 > 0) __syncthreads();            // previous chunk's reads done
#pragma unroll
      for (int i = 0; i < RC; ++i) red[(wave * RC + i) * 64 + lane] = dzp[i0 + i];
      __syncthreads();
      for (int i = wave; i < RC && i0 + i < C; i += NWV) {
        if (ok) {
          float s2 = 0.f;
#pragma unroll
          for (int wv = 0; wv < NWV; ++wv) s2 += red[(wv * RC + i) * 64 + lane];
          dz[zo + (i0 + i) * HW] = s2;
        }
      }
    }
  }
  __syncthreads();
  const int np = Hd * C + Hd + Cout * Hd + Cout;
  float* pp = partial + (int64_t)blockIdx.x * np;
  for (int e = threadIdx.x; e < np; e += blockDim.x) {
    float v;
    if (e < Hd * C) {
      v = acc[(e / C) * PJ + e % C];
    } else if (e < Hd * C + Hd) {
      v = acc[(e - Hd * C) * PJ + CM];
    } else if (e < Hd * C + Hd + Cout * Hd) {
      const int q = e - Hd * C - Hd;
      v = acc[(q % Hd) * PJ + CM + 1 + q / Hd];
    } else {
      v = acc[Hd * PJ + (e - Hd * C - Hd - Cout * Hd)];
    }
    pp[e] = v;
  }
}

// ---------------------------------------------------------------- snapshot-bag mean
// Four threads per grid point (a quad of lanes): quad lane q sums snapshots l = q, q + 4, ...,
// the quad adds its partials in a fixed order ((q0 + q1) + (q2 + q3), deterministic), and the
// quad's lanes write channels c = q, q + 4, ... -- one thread per point left a 54-long
// dependent sum per lane on one wave per SIMD (config C: 4 x 128^2 points).
__global__ __launch_bounds__(kBlock) void bagmean_fwd_kernel(const float* __restrict__ u,
                                                             const float* __restrict__ grid,
                                                             const float* __restrict__ w,
                                                             const float* __restrict__ bias,
                                                             const float* __restrict__ lw,
                                                             float* __restrict__ y, int B, int L,
                                                             int S, int d, int width) {
  // lw (nullable): per-snapshot weights replacing 1/L (a bag of unique snapshots with
  // multiplicities: lw[l] = count_l / L_drawn)
  const int64_t total = (int64_t)B * S;
  const float invL = lw ? 1.0f : 1.0f / (float)L;
  const int q = threadIdx.x & 3;
  for (int64_t base = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 2; base < total;
       base += ((int64_t)gridDim.x * blockDim.x) >> 2) {
    const int64_t idx = base;
    const int s = (int)(idx % S);
    const int b = (int)(idx / S);
    const float* ub = u + (int64_t)b * L * S + s;
    float sum = 0.f;
    if (lw) {
#pragma unroll 4
      for (int l = q; l < L; l += 4) sum = fmaf(lw[l], ub[(int64_t)l * S], sum);
    } else {
#pragma unroll 4
      for (int l = q; l < L; l += 4) sum += ub[(int64_t)l * S];
    }
    const float s1 = sum + __shfl_xor(sum, 1, 64);        // (q0 + q1), (q2 + q3)
    sum = s1 + __shfl_xor(s1, 2, 64);                      // same order in every lane
    for (int c = q; c < width; c += 4) {
      float v = bias[c];
      for (int e = 0; e < d; ++e) v = fmaf(w[c * (d + 1) + e], grid[(int64_t)s * d + e], v);
      v = fmaf(w[c * (d + 1) + d] * invL, sum, v);
      y[idx * width + c] = v;
    }
  }
}

__global__ __launch_bounds__(kBlock) void bagmean_bwd_kernel(const float* __restrict__ dy,
                                                             const float* __restrict__ w,
                                                             float* __restrict__ s, int B, int S,
                                                             int d, int width, int L) {
  const int64_t total = (int64_t)B * S;
  const float invL = 1.0f / (float)L;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    float v = 0.f;
    for (int c = 0; c < width; ++c) v = fmaf(w[c * (d + 1) + d] * invL, dy[idx * width + c], v);
    s[idx] = v;
  }
}

// ---------------------------------------------------------------- loss / metrics / Adam
__global__ __launch_bounds__(kBlock) void mse_kernel(const float* __restrict__ p,
                                                     const float* __restrict__ t,
                                                     float* __restrict__ partial,
                                                     float* __restrict__ grad, int64_t n,
                                                     const float* __restrict__ gscale) {
  __shared__ float red[kBlock];
  float acc = 0.f;
  const float gs = grad ? (gscale ? gscale[0] : 1.0f) * 2.0f / (float)n : 0.f;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float d = p[i] - t[i];
    acc = fmaf(d, d, acc);
    if (grad) grad[i] = gs * d;
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int s = kBlock / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) partial[blockIdx.x] = red[0];
}

// loss = (sum of the nblk partials, fixed order) / n: the scalar of nn.MSELoss's forward in one
// single-workgroup launch (instead of a torch sum and a torch division)
__device__ __forceinline__ void mse_finish_block(const float* __restrict__ partial, int nblk,
                                                 int64_t n, float* __restrict__ loss,
                                                 float* __restrict__ lsum) {
  __shared__ float red[kBlock];
  float acc = 0.f;
  for (int i = threadIdx.x; i < nblk; i += kBlock) acc += partial[i];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int s = kBlock / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float l = red[0] / (float)n;
    loss[0] = l;
    if (lsum) lsum[0] += l;                      // running loss sum of a training loop
  }
}

__global__ __launch_bounds__(kBlock) void mse_finish_kernel(const float* __restrict__ partial,
                                                            int nblk, int64_t n,
                                                            float* __restrict__ loss,
                                                            float* __restrict__ lsum) {
  mse_finish_block(partial, nblk, n, loss, lsum);
}

// The forward's partials and the finish in ONE launch: every workgroup stores its partial as
// mse_kernel does, then counts itself done on a device counter (release fence, atomic add);
// the workgroup that counts last (acquire fence) sums the partials exactly as
// mse_finish_kernel, writes the loss and resets the counter for the next launch (graph replays
// reuse it).  Bit-identical to mse_kernel + mse_finish_kernel.
// grad != NULL: also the gradient for a unit upstream gradient, 2 (p - t) / n (as mse_kernel
// with gscale 1), for a backward seeded with exactly 1 (blindno.ops.MSEFn).
__global__ __launch_bounds__(kBlock) void mse_fwd_fused_kernel(const float* __restrict__ p,
                                                               const float* __restrict__ t,
                                                               float* __restrict__ partial,
                                                               int64_t n, float* __restrict__ loss,
                                                               float* __restrict__ lsum,
                                                               unsigned* __restrict__ counter,
                                                               float* __restrict__ grad) {
  __shared__ float red[kBlock];
  __shared__ unsigned last;
  float acc = 0.f;
  const float gs = 1.0f * 2.0f / (float)n;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float d = p[i] - t[i];
    acc = fmaf(d, d, acc);
    if (grad) grad[i] = gs * d;
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int s = kBlock / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    partial[blockIdx.x] = red[0];
    __threadfence();
    last = atomicAdd(counter, 1u) == gridDim.x - 1 ? 1u : 0u;
  }
  __syncthreads();
  if (last) {
    __threadfence();
    mse_finish_block(partial, (int)gridDim.x, n, loss, lsum);
    if (threadIdx.x == 0) counter[0] = 0u;
  }
}

// Row r holds n points of `stride` floats: out[2r] = sum (a[.+off_a] - b[.+off_b])^2,
// out[2r+1] = sum b[.+off_b]^2 or, with den_all, over all `stride` channels of b (the train
// loop's denominator quirk, 2d_FPE/train_fno.py:161,163).  fp64 accumulation.
__global__ __launch_bounds__(kBlock) void rowsq_kernel(const float* __restrict__ a,
                                                       const float* __restrict__ b,
                                                       double* __restrict__ out, int rows, int n,
                                                       int stride, int off_a, int off_b,
                                                       int den_all) {
  __shared__ double ra[kBlock], rb[kBlock];
  const int r = blockIdx.x;
  if (r >= rows) return;
  double sa = 0.0, sb = 0.0;
  const float* ap = a + (int64_t)r * n * stride;
  const float* bp = b + (int64_t)r * n * stride;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const float* bq = bp + (int64_t)i * stride;
    const double d = (double)ap[(int64_t)i * stride + off_a] - (double)bq[off_b];
    sa += d * d;
    if (den_all) {
      for (int e = 0; e < stride; ++e) sb += (double)bq[e] * (double)bq[e];
    } else {
      sb += (double)bq[off_b] * (double)bq[off_b];
    }
  }
  ra[threadIdx.x] = sa;
  rb[threadIdx.x] = sb;
  __syncthreads();
  for (int s = kBlock / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s) {
      ra[threadIdx.x] += ra[threadIdx.x + s];
      rb[threadIdx.x] += rb[threadIdx.x + s];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    out[2 * r] = ra[0];
    out[2 * r + 1] = rb[0];
  }
}

__global__ __launch_bounds__(kBlock) void adam_kernel(float* __restrict__ p,
                                                      const float* __restrict__ g,
                                                      float* __restrict__ m, float* __restrict__ v,
                                                      int64_t n, float beta1, float beta2,
                                                      float eps, float step_size, float bc2s,
                                                      float gscale) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float gi = g[i] * gscale;
    const float mi = fmaf(1.0f - beta1, gi - m[i], m[i]);   // exp_avg.lerp_(grad, 1-beta1)
    const float vi = fmaf((1.0f - beta2) * gi, gi, v[i] * beta2);
    m[i] = mi;
    v[i] = vi;
    const float denom = sqrtf(vi) / bc2s + eps;
    p[i] = p[i] - step_size * (mi / denom);
  }
}

}  // namespace

// ------------------------------------------------------------------------------ C ABI
BLINDNO_API int blindno_abi_version(void) { return 2; }

BLINDNO_API const char* blindno_error_string(int code) {
  return hipGetErrorString((hipError_t)code);
}

BLINDNO_API int blindno_lift_fwd_bag_g(const float* in, const float* w0, const float* b0,
                                       float* x0, int G, int64_t wgs, int Bn, int N1, int N2,
                                       int Cin, int C, int P1, int P2, const float* ubar,
                                       const float* grid, const float* bw, const float* bb,
                                       float invL, void* stream);

// the shapes for which lift_fwd_bag_g and lift_bwd_bag_mix_g take a bag-mean input (the wide
// 12-channel lift forms, the merged adjoint with its matrix-core weight gradient)
BLINDNO_API int blindno_lift_bag_ok(int G, int Bn, int N1, int N2, int Cin, int C, int P1,
                                    int P2) {
  if (G < 1 || Bn % G || N1 > P1 || N2 > P2) return 0;
  const int Bg = Bn / G;
  const int64_t npts = (int64_t)Bn * P1 * P2;
  const bool fwd = Cin == 12 && C > 4 && C <= kLiftMaxC && G <= kLiftMaxG &&
                   npts * (C > Cin ? C : Cin) < INT32_MAX;
  const bool bwd = Cin == 12 && C <= kLiftMaxC && G <= kLiftMaxG &&
                   (int64_t)Bn * C * P1 * P2 < INT32_MAX && (int64_t)Bg * N1 * N2 * Cin < INT32_MAX &&
                   C >= 5 && C <= 16 && N2 % 16 == 0 && P2 % 4 == 0 && LIFT_BWD_BOTH;
  return fwd && bwd ? 1 : 0;
}



BLINDNO_API int blindno_lift_fwd_g(const float* in, const float* w0, const float* b0, float* x0,
                                   int G, int64_t wgs, int Bn, int N1, int N2, int Cin, int C,
                                   int P1, int P2, void* stream) {
  return blindno_lift_fwd_bag_g(in, w0, b0, x0, G, wgs, Bn, N1, N2, Cin, C, P1, P2, nullptr,
                                nullptr, nullptr, nullptr, 1.0f, stream);
}

BLINDNO_API int blindno_lift_fwd_bag_g(const float* in, const float* w0, const float* b0,
                                       float* x0, int G, int64_t wgs, int Bn, int N1, int N2,
                                       int Cin, int C, int P1, int P2, const float* ubar,
                                       const float* grid, const float* bw, const float* bb,
                                       float invL, void* stream) {
  if (N1 > P1 || N2 > P2 || G < 1 || Bn % G) return (int)hipErrorInvalidValue;
  const BagIn bi{ubar, grid, bw, bb, invL, 1.0f};
  if (ubar && (!grid || !bw || !bb || Cin != 12 || C <= 4 || C > kLiftMaxC || G > kLiftMaxG))
    return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  const int Bg = G > 1 ? Bn / G : Bn;
  if (G == 1) wgs = 0;
  const int64_t npts = (int64_t)Bn * P1 * P2;
  if (Cin == 12 && C > 4 && C <= kLiftMaxC && G <= kLiftMaxG && npts * (C > Cin ? C : Cin) < INT32_MAX &&
      (ubar || (((uintptr_t)in) & 15) == 0)) {
    // the heads (width 12): thread per point, weights in LDS (lift_fwd_wide_kernel)
    lift_fwd_wide_kernel<12, 16><<<grid_for(npts, kBlock, 8192), kBlock, 0, st>>>(
        in, w0, b0, x0, Bn, N1, N2, C, P1, P2, Bg, G, wgs, FastDiv::make((unsigned)(P1 * P2)),
        FastDiv::make((unsigned)P2), bi);
    return (int)hipGetLastError();
  }
  if (ubar) return (int)hipErrorInvalidValue;
  if (C > 4 && C <= 16) {         // wide lifts (the heads): one thread per point, all channels
    const int64_t pts = (int64_t)Bn * P1 * P2;
    lift_fwd_pt_kernel<16><<<grid_for(4 * pts, kBlock, 65536), kBlock, 0, st>>>(
        in, w0, b0, x0, Bn, N1, N2, Cin, C, P1, P2, Bg, wgs);
    return (int)hipGetLastError();
  }
  const int64_t total = (int64_t)Bn * C * P1 * P2;
  lift_fwd_kernel<<<grid_for(total, kBlock, 65536), kBlock, 0, st>>>(
      in, w0, b0, x0, Bn, N1, N2, Cin, C, P1, P2, Bg, wgs);
  return (int)hipGetLastError();
}

BLINDNO_API int blindno_lift_fwd(const float* in, const float* w0, const float* b0, float* x0,
                                 int Bn, int N1, int N2, int Cin, int C, int P1, int P2,
                                 void* stream) {
  return blindno_lift_fwd_g(in, w0, b0, x0, 1, 0, Bn, N1, N2, Cin, C, P1, P2, stream);
}

BLINDNO_API int blindno_lift_bwd_nchunk(int Bn, int N1, int N2) {
  const int nt = cdiv((int64_t)Bn * N1 * N2, TP);
  return nt < 1024 ? nt : 1024;
}

BLINDNO_API int blindno_lift_bwd_bag_mix_g(const float* dx0, const float* in, const float* w0,
                                           float* d_in, float* partial, int nchunk, int G,
                                           int64_t wgs, int Bn, int N1, int N2, int Cin, int C,
                                           int P1, int P2, const float* Xs, const float* Gs,
                                           float* dWt, float* mpartial, int mnsplit, int K1,
                                           int m2, const float* ubar, const float* grid,
                                           const float* bw, const float* bb, float invL,
                                           float invLb, void* stream);

BLINDNO_API int blindno_lift_bwd_mix_g(const float* dx0, const float* in, const float* w0,
                                       float* d_in, float* partial, int nchunk, int G,
                                       int64_t wgs, int Bn, int N1, int N2, int Cin, int C, int P1,
                                       int P2, const float* Xs, const float* Gs, float* dWt,
                                       float* mpartial, int mnsplit, int K1, int m2,
                                       void* stream) {
  return blindno_lift_bwd_bag_mix_g(dx0, in, w0, d_in, partial, nchunk, G, wgs, Bn, N1, N2, Cin,
                                    C, P1, P2, Xs, Gs, dWt, mpartial, mnsplit, K1, m2, nullptr,
                                    nullptr, nullptr, nullptr, 1.0f, 1.0f, stream);
}

BLINDNO_API int blindno_lift_bwd_bag_mix_g(const float* dx0, const float* in, const float* w0,
                                           float* d_in, float* partial, int nchunk, int G,
                                           int64_t wgs, int Bn, int N1, int N2, int Cin, int C,
                                           int P1, int P2, const float* Xs, const float* Gs,
                                           float* dWt, float* mpartial, int mnsplit, int K1,
                                           int m2, const float* ubar, const float* grid,
                                           const float* bw, const float* bb, float invL,
                                           float invLb, void* stream) {
  if (G < 1 || Bn % G) return (int)hipErrorInvalidValue;
  const BagIn bi{ubar, grid, bw, bb, invL, invLb};
  if (ubar && (!grid || !bw || !bb)) return (int)hipErrorInvalidValue;
  const int Bg = Bn / G;
  hipStream_t st = (hipStream_t)stream;
  const bool wide_in = d_in && Cin == 12 && C <= kLiftMaxC && G <= kLiftMaxG &&
                       (int64_t)Bn * C * P1 * P2 < INT32_MAX &&
                       (int64_t)Bg * N1 * N2 * Cin < INT32_MAX &&
                       (ubar || (((uintptr_t)d_in) & 15) == 0);
  const bool mf = C >= 5 && C <= 16 && Cin + 1 <= 32 && N2 % 16 == 0 && P2 % 4 == 0 &&
                  (((uintptr_t)dx0) & 15) == 0;
  // the spectral weight gradient hosted in the same launch (Xs != NULL; Ci = Co = C)
  MixWgradJob mw{};
  int64_t nbm = 0;
  const int64_t mtotal = (int64_t)m2 * K1 * C * C;
  if (Xs) {
    if (!Gs || !dWt || K1 < 1 || m2 < 1 || mtotal >= INT32_MAX / 2 || mnsplit < 1 ||
        (mnsplit > 1 && !mpartial))
      return (int)hipErrorInvalidValue;
    mw.X = (const float2*)Xs;
    mw.Gs = (const float2*)Gs;
    mw.out = (float2*)(mnsplit > 1 ? mpartial : dWt);
    mw.Bn = Bn; mw.Ci = C; mw.Co = C; mw.K1 = K1; mw.m2 = m2;
    mw.gx = (int)cdiv(mtotal, kBlock);
    mw.gy = mnsplit;
    mw.gz = G;
    nbm = (int64_t)mw.gx * mnsplit * G;
  }
  // the bag input only on the merged wide path (the generic kernels read a materialised field)
  if (ubar && !(wide_in && partial && mf && LIFT_BWD_BOTH)) return (int)hipErrorInvalidValue;
  if (wide_in && partial && mf && LIFT_BWD_BOTH) {
    if (nchunk != blindno_lift_bwd_nchunk(Bg, N1, N2) || C * Cin + C > PPT * kBlock)
      return (int)hipErrorInvalidValue;
    const int nbi = grid_for((int64_t)Bg * N1 * N2, kBlock, 8192);
    const int64_t nb = nbi + (int64_t)nchunk * G + nbm;
    if (nb >= INT32_MAX) return (int)hipErrorInvalidValue;
    const FastDiv dS = FastDiv::make((unsigned)(N1 * N2)), dN2 = FastDiv::make((unsigned)N2);
    if (Cin + 1 <= 16)
      lift_bwd_both_kernel<1><<<(unsigned)nb, 256, 0, st>>>(dx0, w0, d_in, in, partial, Bg, N1, N2,
                                                            Cin, C, P1, P2, G, G > 1 ? wgs : 0, dS,
                                                            dN2, nbi, nchunk, mw, bi);
    else
      lift_bwd_both_kernel<2><<<(unsigned)nb, 256, 0, st>>>(dx0, w0, d_in, in, partial, Bg, N1, N2,
                                                            Cin, C, P1, P2, G, G > 1 ? wgs : 0, dS,
                                                            dN2, nbi, nchunk, mw, bi);
    const int e = (int)hipGetLastError();
    if (e || !Xs || mnsplit == 1) return e;
    return blindno_reduce_partials(mpartial, dWt, mnsplit, (int)(2 * mtotal * G), stream);
  }
  if (Xs) {
    const int e = blindno_mix_wgrad_g(Xs, Gs, dWt, mpartial, mnsplit, G, Bn, C, C, K1, m2, stream);
    if (e) return e;
  }
  if (d_in) {
    const int64_t total = (int64_t)Bg * N1 * N2 * Cin;
    if (wide_in) {
      lift_bwd_in_wide_kernel<12, 16><<<grid_for((int64_t)Bg * N1 * N2, kBlock, 8192), kBlock, 0, st>>>(
          dx0, w0, d_in, Bg, N1, N2, C, P1, P2, G, G > 1 ? wgs : 0,
          FastDiv::make((unsigned)(N1 * N2)), FastDiv::make((unsigned)N2));
    } else {
      lift_bwd_in_kernel<<<grid_for(total, kBlock, 65536), kBlock, 0, st>>>(
          dx0, w0, d_in, Bg, N1, N2, Cin, C, P1, P2, G, G > 1 ? wgs : 0);
    }
  }
  if (partial) {
    if (nchunk != blindno_lift_bwd_nchunk(Bg, N1, N2) || C * Cin + C > PPT * kBlock)
      return (int)hipErrorInvalidValue;
    if (mf) {
      if (Cin + 1 <= 16)
        lift_bwd_w_mfma_kernel<1><<<dim3(nchunk, G), 256, 0, st>>>(dx0, in, partial, Bg, N1, N2,
                                                                  Cin, C, P1, P2);
      else
        lift_bwd_w_mfma_kernel<2><<<dim3(nchunk, G), 256, 0, st>>>(dx0, in, partial, Bg, N1, N2,
                                                                  Cin, C, P1, P2);
      return (int)hipGetLastError();
    }
    const size_t sh = sizeof(float) * (size_t)(C + Cin) * (TP + 1);
    lift_bwd_w_kernel<<<dim3(nchunk, G), kBlock, sh, st>>>(dx0, in, partial, Bg, N1, N2, Cin, C,
                                                          P1, P2);
  }
  return (int)hipGetLastError();
}

BLINDNO_API int blindno_lift_bwd_g(const float* dx0, const float* in, const float* w0,
                                   float* d_in, float* partial, int nchunk, int G, int64_t wgs,
                                   int Bn, int N1, int N2, int Cin, int C, int P1, int P2,
                                   void* stream) {
  return blindno_lift_bwd_mix_g(dx0, in, w0, d_in, partial, nchunk, G, wgs, Bn, N1, N2, Cin, C,
                                P1, P2, nullptr, nullptr, nullptr, nullptr, 1, 0, 0, stream);
}

BLINDNO_API int blindno_lift_bwd(const float* dx0, const float* in, const float* w0,
                                 float* d_in, float* partial, int nchunk, int Bn, int N1,
                                 int N2, int Cin, int C, int P1, int P2, void* stream) {
  return blindno_lift_bwd_g(dx0, in, w0, d_in, partial, nchunk, 1, 0, Bn, N1, N2, Cin, C, P1, P2,
                            stream);
}

#ifndef CONV_WGRAD_MFMA
#define CONV_WGRAD_MFMA 1
#endif
BLINDNO_API int blindno_conv_wgrad_nchunk(int Bn, int P1, int P2) {
  const int64_t nt = (int64_t)Bn * cdiv((int64_t)P1 * P2, TP);
  return (int)(nt < 1024 ? nt : 1024);
}

BLINDNO_API int blindno_conv_wgrad_g(const float* dz, const float* x, float* partial, int nchunk,
                                     int G, int Bn, int C, int P1, int P2, int act, void* stream) {
  if (G < 1 || Bn % G) return (int)hipErrorInvalidValue;
  const int Bg = Bn / G;
  if (nchunk != blindno_conv_wgrad_nchunk(Bg, P1, P2) || C * C + C > PPT * kBlock)
    return (int)hipErrorInvalidValue;
  const int64_t HW = (int64_t)P1 * P2;
  const int tpn = cdiv(HW, TP);
  const int64_t ntiles = (int64_t)Bg * tpn;
  const size_t sh = sizeof(float) * 2 * (size_t)C * (TP + 1);
  const dim3 grid(nchunk, G);
  if (CONV_WGRAD_MFMA && conv_wgrad_mfma_ok(C, HW)) {
    if (act)
      conv_wgrad_mfma_kernel<1><<<grid, 256, 0, (hipStream_t)stream>>>(dz, x, partial, C, (int)HW, Bg);
    else
      conv_wgrad_mfma_kernel<0><<<grid, 256, 0, (hipStream_t)stream>>>(dz, x, partial, C, (int)HW, Bg);
    return (int)hipGetLastError();
  }
  if (act)
    conv_wgrad_kernel<1><<<grid, kBlock, sh, (hipStream_t)stream>>>(dz, x, partial, C, HW, tpn, ntiles);
  else
    conv_wgrad_kernel<0><<<grid, kBlock, sh, (hipStream_t)stream>>>(dz, x, partial, C, HW, tpn, ntiles);
  return (int)hipGetLastError();
}

BLINDNO_API int blindno_conv_wgrad(const float* dz, const float* x, float* partial, int nchunk,
                                   int Bn, int C, int P1, int P2, int act, void* stream) {
  return blindno_conv_wgrad_g(dz, x, partial, nchunk, 1, Bn, C, P1, P2, act, stream);
}

BLINDNO_API int blindno_reduce_partials(const float* partial, float* out, int nchunk, int np,
                                        void* stream) {
  if (nchunk < 1 || np < 1) return (int)hipErrorInvalidValue;
  const int PB = np < 64 ? np : 64;
  reduce_partials_kernel<<<cdiv(np, PB), 1024, 0, (hipStream_t)stream>>>(partial, out, nchunk, np,
                                                                           PB);
  return (int)hipGetLastError();
}

// the deferred finalisation's reductions and unpacks in one launch (0: two launches, for A/B)
#ifndef FINISH_ONE_LAUNCH
#define FINISH_ONE_LAUNCH 1
#endif
// segments s0 .. s0 + k - 1 of a blindno_reduce_partials_pieces_u call -> ReduceSegs
static int reduce_segs_build(const void* const* partials, void* const* outs, const int* nchunks,
                             const int* nps, const int* e0s, const int* e1s, const int* upks,
                             void* const* ud, const int* ushp, int s0, int k, ReduceSegs& segs,
                             int& blocks) {
  segs = ReduceSegs{};
  segs.nseg = k;
  blocks = 0;
  int nu = 0;
  for (int i = 0; i < k; ++i) {
    const int nc = nchunks[s0 + i], np = nps[s0 + i];
    const int e0 = e0s ? e0s[s0 + i] : 0, e1 = e1s ? e1s[s0 + i] : np;
    if (nc < 1 || np < 1 || e0 < 0 || e1 > np || e0 >= e1) return (int)hipErrorInvalidValue;
    segs.upk[i] = -1;
    const int uq = upks ? upks[s0 + i] : -1;
    if (uq >= 0) {
      const int* sh = ushp + 4 * uq;      // (Ci, Co, m1, m2) of descriptor uq
      if (nu == kRedUnpack || e0 != 0 || e1 != np || !ud[2 * uq] || !ud[2 * uq + 1] ||
          sh[0] < 1 || sh[1] < 1 || sh[2] < 1 || sh[3] < 1 ||
          (int64_t)4 * sh[0] * sh[1] * sh[2] * sh[3] != np)
        return (int)hipErrorInvalidValue;
      segs.ut[nu] = W2dUnpack{(float*)ud[2 * uq], (float*)ud[2 * uq + 1], sh[0], sh[1], sh[2], sh[3]};
      segs.upk[i] = nu++;
    }
    segs.src[i] = (const float*)partials[s0 + i];
    segs.out[i] = (float*)outs[s0 + i];
    segs.nchunk[i] = nc;
    segs.np[i] = np;
    const int pb = np < 64 ? np : 64;
    segs.pb[i] = pb;
    segs.blk0[i] = e0 / pb;
    segs.e0[i] = e0;
    segs.e1[i] = e1;
    segs.cum[i] = blocks;
    blocks += cdiv(e1, pb) - e0 / pb;
  }
  segs.cum[k] = blocks;
  return 0;
}

BLINDNO_API int blindno_reduce_partials_pieces_u(const void* const* partials, void* const* outs,
                                                 const int* nchunks, const int* nps,
                                                 const int* e0s, const int* e1s, const int* upks,
                                                 void* const* ud, const int* ushp, int nseg,
                                                 void* stream) {
  if (nseg < 0) return (int)hipErrorInvalidValue;
  for (int s0 = 0; s0 < nseg; s0 += kRedSegs) {
    ReduceSegs segs;
    int blocks;
    const int k = nseg - s0 < kRedSegs ? nseg - s0 : kRedSegs;
    const int e = reduce_segs_build(partials, outs, nchunks, nps, e0s, e1s, upks, ud, ushp, s0, k,
                                    segs, blocks);
    if (e) return e;
    if (blocks == 0) continue;
    reduce_partials_multi_kernel<<<blocks, 1024, 0, (hipStream_t)stream>>>(segs);
  }
  return (int)hipGetLastError();
}

// The deferred finalisation's reductions and its spectral-weight unpacks (independent of each
// other) in ONE launch of 1024-thread workgroups: [0, nred) reduce exactly as
// reduce_partials_multi_kernel, the rest run four 256-thread unpack tile teams each
// (w2d_transpose_tile, as w2d_transpose_kernel<1>).  Bit-identical to the two launches.
__global__ __launch_bounds__(1024) void finish_multi_kernel(ReduceSegs segs, PackSegs ps, int nred,
                                                           int ntr) {
  __shared__ float red[1024];
  __shared__ float2 tile[4][32][33];
  const int b = blockIdx.x;
  if (b < nred) {
    int sg = 0;
    while (sg + 1 < segs.nseg && segs.cum[sg + 1] <= b) ++sg;  // uniform scan
    const int u = segs.upk[sg];
    reduce_partials_block(segs.src[sg], segs.out[sg], segs.nchunk[sg], segs.np[sg], segs.pb[sg],
                          segs.blk0[sg] + b - segs.cum[sg], red, segs.e0[sg], segs.e1[sg], u >= 0,
                          segs.ut[u >= 0 ? u : 0]);
    return;
  }
  const int team = threadIdx.x >> 8;
  const int tb = 4 * (b - nred) + team;
  w2d_transpose_tile<1>(ps, tb < ntr ? tb : 0, threadIdx.x & 255, tile[team], tb < ntr);
}

BLINDNO_API int blindno_finish_multi(const void* const* partials, void* const* outs,
                                     const int* nchunks, const int* nps, const int* e0s,
                                     const int* e1s, const int* upks, void* const* ud,
                                     const int* ushp, int nseg, const void* const* dWts,
                                     void* const* dw1s, void* const* dw2s, const int* shapes,
                                     int nunp, void* stream) {
  if (nseg < 0 || nunp < 0) return (int)hipErrorInvalidValue;
  // one launch when everything fits one segment table and every unpack takes the tiled path
  bool one = nseg <= kRedSegs && nunp <= kPackSegs && nseg > 0 && nunp > 0 && FINISH_ONE_LAUNCH;
  PackSegs ps{};
  int64_t ntr = 0;
  if (one) {
    ps.nseg = nunp;
    for (int i = 0; i < nunp; ++i) {
      const int* sh = shapes + 5 * i;
      if (sh[2] > sh[4] || sh[0] < 1 || sh[1] < 1 || sh[2] < 1 || sh[3] < 1 || !dWts[i] ||
          !dw1s[i] || !dw2s[i])
        return (int)hipErrorInvalidValue;
      ps.w1[i] = (const float*)dw1s[i];
      ps.w2[i] = (const float*)dw2s[i];
      ps.Wt[i] = (float2*)const_cast<void*>(dWts[i]);
      ps.Ci[i] = sh[0]; ps.Co[i] = sh[1]; ps.m1[i] = sh[2]; ps.m2[i] = sh[3]; ps.P1[i] = sh[4];
    }
    one = w2d_tiled_segs(ps, ntr);
  }
  if (!one) {
    const int e = blindno_reduce_partials_pieces_u(partials, outs, nchunks, nps, e0s, e1s, upks, ud,
                                                   ushp, nseg, stream);
    if (e || nunp == 0) return e;
    return blindno_unpack_w2d_multi(dWts, dw1s, dw2s, shapes, nunp, stream);
  }
  ReduceSegs segs;
  int nred;
  const int e = reduce_segs_build(partials, outs, nchunks, nps, e0s, e1s, upks, ud, ushp, 0, nseg,
                                  segs, nred);
  if (e) return e;
  const int64_t nb = nred + (ntr + 3) / 4;
  if (nb >= INT32_MAX) return (int)hipErrorInvalidValue;
  finish_multi_kernel<<<(unsigned)nb, 1024, 0, (hipStream_t)stream>>>(segs, ps, nred, (int)ntr);
  return (int)hipGetLastError();
}

BLINDNO_API int blindno_reduce_partials_pieces(const void* const* partials, void* const* outs,
                                               const int* nchunks, const int* nps, const int* e0s,
                                               const int* e1s, int nseg, void* stream) {
  return blindno_reduce_partials_pieces_u(partials, outs, nchunks, nps, e0s, e1s, nullptr,
                                          nullptr, nullptr, nseg, stream);
}

BLINDNO_API int blindno_reduce_partials_multi(const void* const* partials, void* const* outs,
                                              const int* nchunks, const int* nps, int nseg,
                                              void* stream) {
  return blindno_reduce_partials_pieces(partials, outs, nchunks, nps, nullptr, nullptr, nseg,
                                        stream);
}

BLINDNO_API int blindno_project_fwd_g(const float* z, const float* w1, const float* b1,
                                      const float* w2, const float* b2, float* out, int G,
                                      int64_t wgs, int Bn, int C, int P1, int P2, int Ho, int Wo,
                                      int Hd, int Cout, int ostride, int ooff, void* stream) {
  if (Ho > P1 || Wo > P2 || C > 32 || Cout > 4 || (int64_t)Bn * Ho * Wo >= INT32_MAX ||
      !project_mfma_ok(C, Hd, Cout, (int64_t)Bn * C * P1 * P2))
    return (int)hipErrorInvalidValue;
  return project_fwd_mfma(z, w1, b1, w2, b2, out, Bn, C, P1, P2, Ho, Wo, Cout, ostride, ooff, G,
                          wgs, (hipStream_t)stream);
}

BLINDNO_API int blindno_project_fwd(const float* z, const float* w1, const float* b1,
                                    const float* w2, const float* b2, float* out, int Bn, int C,
                                    int P1, int P2, int Ho, int Wo, int Hd, int Cout,
                                    int ostride, int ooff, void* stream) {
  if (Ho > P1 || Wo > P2 || C > 32 || Cout > 4 || (int64_t)Bn * Ho * Wo >= INT32_MAX)
    return (int)hipErrorInvalidValue;
  if (project_mfma_ok(C, Hd, Cout, (int64_t)Bn * C * P1 * P2))
    return project_fwd_mfma(z, w1, b1, w2, b2, out, Bn, C, P1, P2, Ho, Wo, Cout, ostride, ooff, 1,
                            0, (hipStream_t)stream);
  const int64_t total = (int64_t)Bn * Ho * Wo;
  const dim3 g(grid_for(total, kBlock, 2048));
  hipStream_t st = (hipStream_t)stream;
#define PF(CM_, CO_)                                                                          \
  project_fwd_kernel<CM_, CO_><<<g, kBlock, sizeof(float) * (size_t)Hd * (CM_ + 1 + CO_), st>>>( \
      z, w1, b1, w2, b2, out, Bn, C, P1, P2, Ho, Wo, Hd, Cout, ostride, ooff)
  if (C <= 4) {
    if (Cout == 1) PF(4, 1); else PF(4, 4);
  } else if (C <= 8) {
    if (Cout == 1) PF(8, 1); else PF(8, 4);
  } else if (C <= 16) {
    if (Cout == 1) PF(16, 1); else PF(16, 4);
  } else {
    if (Cout == 1) PF(32, 1); else PF(32, 4);
  }
#undef PF
  return (int)hipGetLastError();
}

BLINDNO_API int blindno_project_bwd_nchunk(int Bn, int Ho, int Wo) {
  return project_bwd_mfma_nchunk((int64_t)Bn * Ho * Wo);
}

// the partial count the grouped heads' projection backward takes (a grid of 4 point tiles per
// wave there; any count >= 1 is valid for the kernel, which strides over its tiles)
BLINDNO_API int blindno_project_bwd_nchunk_heads(int Bg, int Ho, int Wo) {
  return project_bwd_mfma_nchunk_wide((int64_t)Bg * Ho * Wo);
}

BLINDNO_API int blindno_project_bwd_g(const float* z, const float* w1, const float* b1,
                                      const float* w2, const float* dout, float* dz,
                                      float* partial, int nchunk, int G, int64_t wgs, int Bn,
                                      int C, int P1, int P2, int Ho, int Wo, int Hd, int Cout,
                                      int ostride, int ooff, void* stream) {
  if (Ho > P1 || Wo > P2 || C > 32 || Cout > 4 || !dz || !partial || nchunk < 1 ||
      (int64_t)Bn * Ho * Wo >= INT32_MAX || !project_mfma_ok(C, Hd, Cout, (int64_t)Bn * C * P1 * P2))
    return (int)hipErrorInvalidValue;
  return project_bwd_mfma(z, w1, b1, w2, dout, dz, partial, nchunk, Bn, C, P1, P2, Ho, Wo, Cout,
                          ostride, ooff, 1, G, wgs, (hipStream_t)stream);
}

BLINDNO_API int blindno_project_bwd_w(const float* z, const float* w1, const float* b1,
                                      const float* w2, const float* dout, const float* lscale,
                                      float* dz, float* partial, int nchunk, int Bn, int C,
                                      int P1, int P2, int Ho, int Wo, int Hd, int Cout,
                                      int ostride, int ooff, int dout_div, void* stream) {
  if (Ho > P1 || Wo > P2 || dout_div < 1 || C > 32 || Cout > 4 || !dz || !partial ||
      nchunk < 1 || (int64_t)Bn * Ho * Wo >= INT32_MAX ||
      !project_mfma_ok(C, Hd, Cout, (int64_t)Bn * C * P1 * P2))
    return (int)hipErrorInvalidValue;
  return project_bwd_mfma(z, w1, b1, w2, dout, dz, partial, nchunk, Bn, C, P1, P2, Ho, Wo, Cout,
                          ostride, ooff, dout_div, 1, 0, (hipStream_t)stream, lscale);
}

BLINDNO_API int blindno_project_bwd(const float* z, const float* w1, const float* b1,
                                    const float* w2, const float* dout, float* dz,
                                    float* partial, int nchunk, int Bn, int C, int P1, int P2,
                                    int Ho, int Wo, int Hd, int Cout, int ostride, int ooff,
                                    int dout_div, void* stream) {
  if (Ho > P1 || Wo > P2 || dout_div < 1 || C > 32 || Cout > 4 || !dz || !partial ||
      nchunk < 1 || (int64_t)Bn * Ho * Wo >= INT32_MAX)
    return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  const dim3 g(nchunk);
  if (project_mfma_ok(C, Hd, Cout, (int64_t)Bn * C * P1 * P2))
    return project_bwd_mfma(z, w1, b1, w2, dout, dz, partial, nchunk, Bn, C, P1, P2, Ho, Wo, Cout,
                            ostride, ooff, dout_div, 1, 0, st);
  if (Hd != 128) return (int)hipErrorInvalidValue;   // fc1 = Linear(width, 128) everywhere
  const int cm = C <= 8 ? 8 : (C <= 16 ? 16 : 32);
  const int com = Cout == 1 ? 1 : 4;
  const size_t sh = sizeof(float) * ((size_t)cm * 64 + com * 64 + 16 * (size_t)(cm < 16 ? cm : 16) * 64 +
                                     (size_t)Hd * cm + Hd + (size_t)Hd * com +
                                     (size_t)Hd * (cm + 1 + com) + com);
  if (sh > 160 * 1024) return (int)hipErrorInvalidValue;
#define PW(CM_, CO_)                                                                        \
  project_bwd_wsum_kernel<CM_, 8, CO_><<<g, 1024, sh, st>>>(z, w1, b1, w2, dout, dz, partial, \
                                                           Bn, C, P1, P2, Ho, Wo, Hd, Cout,   \
                                                           ostride, ooff, dout_div)
  if (cm == 8) {
    if (com == 1) PW(8, 1); else PW(8, 4);
  } else if (cm == 16) {
    if (com == 1) PW(16, 1); else PW(16, 4);
  } else {
    if (com == 1) PW(32, 1); else PW(32, 4);
  }
#undef PW
  return (int)hipGetLastError();
}

BLINDNO_API int blindno_bagmean_fwd_w(const float* u, const float* grid, const float* w,
                                      const float* bias, const float* lw, float* y, int B, int L,
                                      int S, int d, int width, void* stream) {
  bagmean_fwd_kernel<<<grid_for(4 * (int64_t)B * S), kBlock, 0, (hipStream_t)stream>>>(
      u, grid, w, bias, lw, y, B, L, S, d, width);
  return (int)hipGetLastError();
}

BLINDNO_API int blindno_bagmean_fwd(const float* u, const float* grid, const float* w,
                                    const float* bias, float* y, int B, int L, int S, int d,
                                    int width, void* stream) {
  return blindno_bagmean_fwd_w(u, grid, w, bias, nullptr, y, B, L, S, d, width, stream);
}

BLINDNO_API int blindno_bagmean_bwd(const float* dy, const float* w, float* s, int B, int S,
                                    int d, int width, int L, void* stream) {
  bagmean_bwd_kernel<<<grid_for((int64_t)B * S), kBlock, 0, (hipStream_t)stream>>>(
      dy, w, s, B, S, d, width, L);
  return (int)hipGetLastError();
}

BLINDNO_API int blindno_mse_finish_acc(const float* partial, int nblk, int64_t n, float* loss,
                                       float* acc, void* stream) {
  if (nblk < 1 || n < 1) return (int)hipErrorInvalidValue;
  mse_finish_kernel<<<1, kBlock, 0, (hipStream_t)stream>>>(partial, nblk, n, loss, acc);
  return (int)hipGetLastError();
}

BLINDNO_API int blindno_mse_fwd(const float* p, const float* t, float* partial, int64_t n,
                                int nblk, float* loss, float* acc, unsigned* counter, float* grad,
                                void* stream) {
  if (n < 1 || nblk < 1 || !p || !t || !partial || !loss || !counter)
    return (int)hipErrorInvalidValue;
  mse_fwd_fused_kernel<<<nblk, kBlock, 0, (hipStream_t)stream>>>(p, t, partial, n, loss, acc,
                                                                 counter, grad);
  return (int)hipGetLastError();
}

BLINDNO_API int blindno_mse_finish(const float* partial, int nblk, int64_t n, float* loss,
                                   void* stream) {
  return blindno_mse_finish_acc(partial, nblk, n, loss, nullptr, stream);
}

BLINDNO_API int blindno_mse(const float* p, const float* t, float* partial, float* grad,
                            int64_t n, int nblk, const float* gscale, void* stream) {
  mse_kernel<<<nblk, kBlock, 0, (hipStream_t)stream>>>(p, t, partial, grad, n, gscale);
  return (int)hipGetLastError();
}

BLINDNO_API int blindno_rowsq(const float* a, const float* b, double* out, int rows, int n,
                              int stride, int off_a, int off_b, int den_all, void* stream) {
  rowsq_kernel<<<rows, kBlock, 0, (hipStream_t)stream>>>(a, b, out, rows, n, stride, off_a, off_b,
                                                         den_all);
  return (int)hipGetLastError();
}

// Flat gradient gather: up to kGatherSegs (src, dst offset, count) segments per launch, passed
// by value in the kernel arguments (so a HIP-graph capture bakes them in).  Segment i owns
// blocks [cum[i], cum[i+1]) of kGatherChunk elements, so the grid is proportional to the bytes
// moved; replaces a torch multi-tensor copy of ~100 blocks.
constexpr int kGatherSegs = 64;
constexpr int kGatherChunk = 8 * kBlock;
struct GatherSegs {
  const float* src[kGatherSegs];
  int64_t off[kGatherSegs];
  int n[kGatherSegs];
  int cum[kGatherSegs + 1];
  int nseg;
};

__global__ __launch_bounds__(kBlock) void gather_flat_kernel(GatherSegs segs, float* __restrict__ dst) {
  const int b = blockIdx.x;
  int sg = 0;
  while (sg + 1 < segs.nseg && segs.cum[sg + 1] <= b) ++sg;    // uniform scan
  const float* __restrict__ src = segs.src[sg];
  float* __restrict__ d = dst + segs.off[sg];
  const int n = segs.n[sg];
  const int i0 = (b - segs.cum[sg]) * kGatherChunk + threadIdx.x;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int i = i0 + k * kBlock;
    if (i < n) d[i] = src[i];
  }
}

BLINDNO_API int blindno_gather_flat(const void* const* srcs, const int64_t* offs, const int64_t* ns,
                                    int nseg, float* dst, void* stream) {
  if (nseg < 0) return (int)hipErrorInvalidValue;
  for (int s0 = 0; s0 < nseg; s0 += kGatherSegs) {
    GatherSegs segs{};
    const int k = nseg - s0 < kGatherSegs ? nseg - s0 : kGatherSegs;
    segs.nseg = k;
    int64_t blocks = 0;
    for (int i = 0; i < k; ++i) {
      if (ns[s0 + i] < 0 || ns[s0 + i] >= INT32_MAX) return (int)hipErrorInvalidValue;
      segs.src[i] = (const float*)srcs[s0 + i];
      segs.off[i] = offs[s0 + i];
      segs.n[i] = (int)ns[s0 + i];
      segs.cum[i] = (int)blocks;
      blocks += (ns[s0 + i] + kGatherChunk - 1) / kGatherChunk;
    }
    segs.cum[k] = (int)blocks;
    if (blocks == 0) continue;
    if (blocks >= INT32_MAX) return (int)hipErrorInvalidValue;
    gather_flat_kernel<<<(unsigned)blocks, kBlock, 0, (hipStream_t)stream>>>(segs, dst);
  }
  return (int)hipGetLastError();
}

// Batch select of the training loop (the DataLoader's batch, 2d_FPE/train_fno.py:113-116): rows
// ids[b] of up to kBatchSegs row-major tensors (bags X (n, T N1 N2), targets Y (n, N1 N2 C)) into
// their batch buffers, in ONE launch: blockIdx.y = (segment, batch row), 16-B copies when the
// rows are 16-B aligned.  ids are device int64 (the epoch's permutation slice); an id outside
// [0, n) of its source fills that batch row with NaN (the step's loss turns NaN) instead of
// reading past the tensor.
constexpr int kBatchSegs = 4;
struct BatchSegs {
  const float* src[kBatchSegs];
  float* dst[kBatchSegs];
  int64_t row[kBatchSegs];   // floats per row
  int64_t n[kBatchSegs];     // rows of each source
  int nseg, vec;
};

__global__ __launch_bounds__(kBlock) void gather_batch_kernel(BatchSegs sg, const int64_t* __restrict__ ids,
                                                              int B) {
  const int sb = blockIdx.y, seg = sb / B, b = sb - seg * B;
  const int64_t row = sg.row[seg], id = ids[b];
  const float* __restrict__ src = sg.src[seg] + id * row;
  float* __restrict__ dst = sg.dst[seg] + (int64_t)b * row;
  if (id < 0 || id >= sg.n[seg]) {
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < row; i += (int64_t)gridDim.x * kBlock)
      dst[i] = __builtin_nanf("");
    return;
  }
  if (sg.vec) {
    const int64_t n4 = row >> 2;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n4; i += (int64_t)gridDim.x * kBlock)
      reinterpret_cast<float4*>(dst)[i] = reinterpret_cast<const float4*>(src)[i];
  } else {
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < row; i += (int64_t)gridDim.x * kBlock)
      dst[i] = src[i];
  }
}

BLINDNO_API int blindno_gather_batch(const void* const* srcs, void* const* dsts, const int64_t* rows,
                                     const int64_t* nsrc, int nseg, const int64_t* ids, int B,
                                     void* stream) {
  if (nseg < 1 || nseg > kBatchSegs || B < 1 || !ids || !nsrc) return (int)hipErrorInvalidValue;
  BatchSegs sg{};
  sg.nseg = nseg;
  sg.vec = 1;
  int64_t maxrow = 0;
  for (int i = 0; i < nseg; ++i) {
    if (!srcs[i] || !dsts[i] || rows[i] < 1 || nsrc[i] < 1) return (int)hipErrorInvalidValue;
    sg.n[i] = nsrc[i];
    sg.src[i] = (const float*)srcs[i];
    sg.dst[i] = (float*)dsts[i];
    sg.row[i] = rows[i];
    if ((rows[i] & 3) || ((uintptr_t)srcs[i] & 15) || ((uintptr_t)dsts[i] & 15)) sg.vec = 0;
    if (rows[i] > maxrow) maxrow = rows[i];
  }
  const int64_t items = sg.vec ? maxrow / 4 : maxrow;
  int64_t gx = (items + kBlock * 4 - 1) / (kBlock * 4);        // ~4 elements per thread
  if (gx < 1) gx = 1;
  if (gx > 4096) gx = 4096;
  gather_batch_kernel<<<dim3((unsigned)gx, (unsigned)(nseg * B)), kBlock, 0, (hipStream_t)stream>>>(sg, ids, B);
  return (int)hipGetLastError();
}

BLINDNO_API int blindno_adam(float* p, const float* g, float* m, float* v, int64_t n, float beta1,
                             float beta2, float eps, float step_size, float bc2s, float gscale,
                             void* stream) {
  adam_kernel<<<grid_for(n, kBlock, 16384), kBlock, 0, (hipStream_t)stream>>>(
      p, g, m, v, n, beta1, beta2, eps, step_size, bc2s, gscale);
  return (int)hipGetLastError();
}
