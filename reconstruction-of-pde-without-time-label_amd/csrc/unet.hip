// Kernels of the permutation-invariant attention UNet, PermInvUNet_attn ("BlinDNO";
// 2d_FPE/NIOModules.py:1044-1181, 1D: 1d_FPE/NIOModules.py:165-443), that the generic
// convolution (conv.hip) and BatchNorm (batchnorm.hip) kernels do not cover:
//
//   dwconv    7x7 (1x7) depthwise convolution of ConvNeXtBlock (groups = C, padding 3)
//   cnx_pw    the rest of ConvNeXtBlock, per pixel: LayerNorm over C (eps 1e-6) ->
//             Linear(C, 4C) -> exact GELU -> Linear(4C, C) -> + shortcut
//   maxpool   MaxPool2d(2) / MaxPool1d(2) (floor; first maximum in scan order, NaN wins)
//   convt     ConvTranspose2d/1d(kernel = stride = 2, output_padding) of the up path
//   tok_*     TemporalSelfAttention + the bag mean that always follows it:
//             Ybar_b = mean_l LayerNorm_D(A X + X)_l,  A = softmax(X X^T / sqrt D)
//
// Temporal attention, collapsed.  The reference materialises A X + X (B x L x D) and its
// LayerNorm and then averages over the L tokens.  With M = A + I, x_t the token means and
// Gc the CENTRED Gram matrix (Gc_ts = (X_t - x_t).(X_s - x_s)):
//   mu_l   = sum_t M_lt x_t,       var_l = (1/D) m_l^T Gc m_l,     r_l = (var_l + eps)^-1/2
//   Ybar   = gamma sum_t c_t (X_t - x_t) + beta,   c_t = (1/L) sum_l r_l M_lt,
// (the token means cancel exactly: sum_t c_t x_t = (1/L) sum_l r_l mu_l), and the scores are
// (Gc + D x x^T) / sqrt D.  So the forward is: token means, one centred Gram matrix per bag
// (L x L, reduced over D), O(L^3) bag-local algebra, and a c-weighted sum of centred tokens --
// nothing of size L x D is written.  Everything is kept in centred quantities (tokens whose
// mean is large against their spread would otherwise cancel catastrophically).
// The backward is the exact adjoint.  With g = gamma dYbar, gb = mean(g), centred dots
// h_t = g.(X_t - x_t), a_l = r_l / L and P = M Gc (saved by the forward):
//   b_l  = a_l r_l^2 (sum_t M_lt h_t) / D
//   dA_lt = a_l h_t - b_l P_lt,   dS = A o (dA - rowsum(A o dA)),
//   Q = (dS + dS^T) / sqrt D,   N = M^T diag(b) M,   R = Q - N,
//   dX_t = (sum_l M_lt a_l) g + sum_s R_ts (X_s - x_s) + (sum_s Q_ts x_s - (sum_l M_lt a_l) gb).
// Every reduction is a fixed-order tree or a fixed-order sum of per-chunk partials
// (blindno_reduce_partials): deterministic, no float atomics.
#include "common.h"
#include "blindno.h"

using namespace blindno;

namespace {

__device__ __forceinline__ float block_sum(float v, float* red) {
  // red: >= 4 floats of LDS; returns the sum in every thread (fixed order)
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  float s = 0.f;
  for (int i = 0; i < nw; ++i) s += red[i];
  return s;
}

__device__ __forceinline__ float block_max(float v, float* red) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, 64));
  const int w = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  float m = red[0];
  for (int i = 1; i < nw; ++i) m = fmaxf(m, red[i]);
  return m;
}

__device__ __forceinline__ float gelu_exact(float z) {
  return 0.5f * z * (1.0f + erff(z * 0.70710678118654752f));
}

__device__ __forceinline__ float gelu_exact_grad(float z) {
  return 0.5f * (1.0f + erff(z * 0.70710678118654752f)) +
         z * 0.39894228040143268f * expf(-0.5f * z * z);
}

// ---------------------------------------------------------------------- depthwise conv
// y[n][c][h][w] = b[c] + sum_{i,j} W[c][i][j] x[n][c][h + i - KH/2][w + j - KW/2]
__global__ __launch_bounds__(kBlock) void dwconv_fwd_kernel(
    const float* __restrict__ x, const float* __restrict__ wt, const float* __restrict__ b,
    float* __restrict__ y, int C, int H, int W, int KH, int KW, int64_t total) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= total) return;
  const int w = (int)(e % W);
  const int h = (int)((e / W) % H);
  const int64_t nc = e / ((int64_t)H * W);
  const int c = (int)(nc % C);
  const float* xp = x + nc * H * W;
  const float* wp = wt + (int64_t)c * KH * KW;
  const int ph = KH / 2, pw = KW / 2;
  float acc = b ? b[c] : 0.f;
  for (int i = 0; i < KH; ++i) {
    const int hi = h + i - ph;
    if (hi < 0 || hi >= H) continue;
    for (int j = 0; j < KW; ++j) {
      const int wi = w + j - pw;
      if (wi < 0 || wi >= W) continue;
      acc = fmaf(wp[i * KW + j], xp[hi * W + wi], acc);
    }
  }
  y[e] = acc;
}

// dx[n][c][h][w] = sum_{i,j} W[c][i][j] dy[n][c][h - i + KH/2][w - j + KW/2]
__global__ __launch_bounds__(kBlock) void dwconv_bwd_data_kernel(
    const float* __restrict__ dy, const float* __restrict__ wt, float* __restrict__ dx, int C,
    int H, int W, int KH, int KW, int64_t total) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= total) return;
  const int w = (int)(e % W);
  const int h = (int)((e / W) % H);
  const int64_t nc = e / ((int64_t)H * W);
  const int c = (int)(nc % C);
  const float* gp = dy + nc * H * W;
  const float* wp = wt + (int64_t)c * KH * KW;
  const int ph = KH / 2, pw = KW / 2;
  float acc = 0.f;
  for (int i = 0; i < KH; ++i) {
    const int ho = h - i + ph;
    if (ho < 0 || ho >= H) continue;
    for (int j = 0; j < KW; ++j) {
      const int wo = w - j + pw;
      if (wo < 0 || wo >= W) continue;
      acc = fmaf(wp[i * KW + j], gp[ho * W + wo], acc);
    }
  }
  dx[e] = acc;
}

// partial[split][c][KH*KW + 1]: tap sums of dy * shifted x and the bias sum over the split's
// share of channel c's (n, h, w) outputs.
constexpr int kMaxTaps = 49;
__global__ __launch_bounds__(kBlock) void dwconv_wgrad_kernel(
    const float* __restrict__ dy, const float* __restrict__ x, float* __restrict__ partial, int N,
    int C, int H, int W, int KH, int KW, int nsplit) {
  __shared__ float red[8];
  const int c = blockIdx.y, split = blockIdx.x;
  const int T = KH * KW;
  const int64_t HW = (int64_t)H * W, P = (int64_t)N * HW;
  const int64_t per = (P + nsplit - 1) / nsplit;
  const int64_t p0 = split * per, p1 = p0 + per < P ? p0 + per : P;
  const int ph = KH / 2, pw = KW / 2;
  float acc[kMaxTaps + 1];
#pragma unroll
  for (int t = 0; t <= kMaxTaps; ++t) acc[t] = 0.f;
  for (int64_t p = p0 + threadIdx.x; p < p1; p += blockDim.x) {
    const int n = (int)(p / HW);
    const int q = (int)(p - n * HW);
    const int h = q / W, w = q - (q / W) * W;
    const int64_t base = ((int64_t)n * C + c) * HW;
    const float g = dy[base + q];
    acc[kMaxTaps] += g;
#pragma unroll
    for (int t = 0; t < kMaxTaps; ++t) {
      if (t >= T) continue;
      const int i = t / KW, j = t - (t / KW) * KW;
      const int hi = h + i - ph, wi = w + j - pw;
      if (hi >= 0 && hi < H && wi >= 0 && wi < W) acc[t] = fmaf(g, x[base + hi * W + wi], acc[t]);
    }
  }
  float* out = partial + ((int64_t)split * C + c) * (T + 1);
#pragma unroll
  for (int t = 0; t < kMaxTaps; ++t) {
    if (t >= T) continue;
    const float s = block_sum(acc[t], red);
    if (threadIdx.x == 0) out[t] = s;
  }
  const float s = block_sum(acc[kMaxTaps], red);
  if (threadIdx.x == 0) out[T] = s;
}

// ---------------------------------------------------------------------- ConvNeXt pointwise
// Weights: w1 (4C, C), b1 (4C), w2 (C, 4C), b2 (C), LayerNorm gamma/beta (C).  Staged in LDS
// for C <= 32 (w2 transposed, so a hidden unit's column is contiguous); read from global memory
// (same address in every lane: one broadcast transaction per wave) for C = 64.
template <int C>
struct CnxW {
  float w1[4 * C][C];
  float w2t[4 * C][C];     // w2t[k][c] = w2[c][k]
  float b1[4 * C];
  float b2[C], lw[C], lb[C];
};

template <int C>
struct CnxSrc {
  static constexpr bool kLds = C <= 32;
  const CnxW<kLds ? C : 1>* s;
  const float *w1, *b1, *w2, *b2, *lw, *lb;
  __device__ __forceinline__ float W1(int k, int c) const {
    if constexpr (kLds) return s->w1[k][c]; else return w1[k * C + c];
  }
  __device__ __forceinline__ float W2T(int k, int c) const {
    if constexpr (kLds) return s->w2t[k][c]; else return w2[c * 4 * C + k];
  }
  __device__ __forceinline__ float B1(int k) const {
    if constexpr (kLds) return s->b1[k]; else return b1[k];
  }
  __device__ __forceinline__ float B2(int c) const {
    if constexpr (kLds) return s->b2[c]; else return b2[c];
  }
  __device__ __forceinline__ float LW(int c) const {
    if constexpr (kLds) return s->lw[c]; else return lw[c];
  }
  __device__ __forceinline__ float LB(int c) const {
    if constexpr (kLds) return s->lb[c]; else return lb[c];
  }
};

template <int C>
__device__ __forceinline__ void stage_cnx(CnxW<C>& s, const float* w1, const float* b1,
                                          const float* w2, const float* b2, const float* lw,
                                          const float* lb) {
  for (int e = threadIdx.x; e < 4 * C * C; e += blockDim.x) {
    s.w1[e / C][e % C] = w1[e];
    s.w2t[e % (4 * C)][e / (4 * C)] = w2[e];
  }
  for (int e = threadIdx.x; e < 4 * C; e += blockDim.x) s.b1[e] = b1[e];
  for (int e = threadIdx.x; e < C; e += blockDim.x) {
    s.b2[e] = b2 ? b2[e] : 0.f;
    s.lw[e] = lw[e];
    s.lb[e] = lb[e];
  }
}

// LayerNorm over the C channels of one pixel (biased variance, eps 1e-6): x <- (x - mean) r.
// C = 2 is evaluated in closed form, u = (x0 - x1) / 2, x = (u r, -u r): the generic
// x - mean cancels catastrophically when x0 ~ x1 (and the UNet's base_ch = 1 models have a
// C = 2 level in both paths).
template <int C>
__device__ __forceinline__ float cnx_norm(float (&x)[C]) {
  if constexpr (C == 2) {
    const float u = 0.5f * (x[0] - x[1]);
    const float r = 1.0f / sqrtf(fmaf(u, u, 1e-6f));
    x[0] = u * r;
    x[1] = -x[0];
    return r;
  }
  float m = 0.f;
#pragma unroll
  for (int c = 0; c < C; ++c) m += x[c];
  m *= 1.0f / C;
  float v = 0.f;
#pragma unroll
  for (int c = 0; c < C; ++c) {
    x[c] -= m;
    v = fmaf(x[c], x[c], v);
  }
  const float r = 1.0f / sqrtf(v * (1.0f / C) + 1e-6f);
#pragma unroll
  for (int c = 0; c < C; ++c) x[c] *= r;
  return r;
}

template <int C>
__global__ __launch_bounds__(kBlock) void cnx_pw_fwd_kernel(
    const float* __restrict__ xd, const float* __restrict__ sc, const float* __restrict__ lw,
    const float* __restrict__ lb, const float* __restrict__ w1, const float* __restrict__ b1,
    const float* __restrict__ w2, const float* __restrict__ b2, float* __restrict__ y, int N,
    int HW) {
  constexpr bool kL = CnxSrc<C>::kLds;
  __shared__ CnxW<kL ? C : 1> s;
  if constexpr (kL) {
    stage_cnx<C>(s, w1, b1, w2, b2, lw, lb);
    __syncthreads();
  }
  const CnxSrc<C> W{&s, w1, b1, w2, b2, lw, lb};
  const int64_t pix = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (pix >= (int64_t)N * HW) return;
  const int n = (int)(pix / HW), q = (int)(pix - (int64_t)n * HW);
  const int64_t base = (int64_t)n * C * HW + q;
  float xh[C], acc[C];
#pragma unroll
  for (int c = 0; c < C; ++c) xh[c] = xd[base + (int64_t)c * HW];
  cnx_norm<C>(xh);
#pragma unroll
  for (int c = 0; c < C; ++c) {
    xh[c] = fmaf(W.LW(c), xh[c], W.LB(c));      // ln
    acc[c] = W.B2(c);
  }
  for (int k = 0; k < 4 * C; ++k) {
    float hk = W.B1(k);
#pragma unroll
    for (int c = 0; c < C; ++c) hk = fmaf(W.W1(k, c), xh[c], hk);
    const float gk = gelu_exact(hk);
#pragma unroll
    for (int c = 0; c < C; ++c) acc[c] = fmaf(W.W2T(k, c), gk, acc[c]);
  }
#pragma unroll
  for (int c = 0; c < C; ++c) y[base + (int64_t)c * HW] = acc[c] + sc[base + (int64_t)c * HW];
}

// Pixels per workgroup of the backward: per pixel 12 C floats go to LDS (dy, g, dh, ln, dln, xh),
// kept with the staged weights under 64 KiB
__host__ __device__ constexpr int cnx_pb(int C) { return C <= 4 ? 256 : (C <= 16 ? 1024 / C : 16); }

// Backward, two phases per workgroup of PB pixels.  Phase 1 (thread = pixel) recomputes the
// forward, writes dxd (the shortcut's gradient is dy itself) and stages per-pixel vectors in
// LDS; phase 2 (thread = weight-gradient entry) sums them over the PB pixels in pixel order.
// partial[blk][E]: [dW1 (4C x C) | db1 (4C) | dW2 (C x 4C) | db2 (C) | dgamma (C) | dbeta (C)]
template <int C>
__global__ __launch_bounds__(kBlock) void cnx_pw_bwd_kernel(
    const float* __restrict__ dy, const float* __restrict__ xd, const float* __restrict__ lw,
    const float* __restrict__ lb, const float* __restrict__ w1, const float* __restrict__ b1,
    const float* __restrict__ w2, float* __restrict__ dxd, float* __restrict__ partial, int N,
    int HW) {
  constexpr int PB = cnx_pb(C);
  constexpr int H4 = 4 * C;
  constexpr bool kL = CnxSrc<C>::kLds;
  __shared__ CnxW<kL ? C : 1> s;
  __shared__ float sdy[C][PB], sg[H4][PB], sdh[H4][PB], sln[C][PB], sdln[C][PB], sxh[C][PB];
  if constexpr (kL) {
    stage_cnx<C>(s, w1, b1, w2, nullptr, lw, lb);
    __syncthreads();
  }
  const CnxSrc<C> W{&s, w1, b1, w2, nullptr, lw, lb};
  const int64_t P = (int64_t)N * HW;
  const int64_t pix = (int64_t)blockIdx.x * PB + threadIdx.x;
  if (threadIdx.x < PB) {
    const int tp = threadIdx.x;
    if (pix < P) {
      const int n = (int)(pix / HW), q = (int)(pix - (int64_t)n * HW);
      const int64_t base = (int64_t)n * C * HW + q;
      float xh[C], g[C], dln[C];
#pragma unroll
      for (int c = 0; c < C; ++c) {
        xh[c] = xd[base + (int64_t)c * HW];
        g[c] = dy[base + (int64_t)c * HW];
        dln[c] = 0.f;
      }
      const float r = cnx_norm<C>(xh);
      for (int k = 0; k < H4; ++k) {
        float hk = W.B1(k), dg = 0.f;
#pragma unroll
        for (int c = 0; c < C; ++c) {
          hk = fmaf(W.W1(k, c), fmaf(W.LW(c), xh[c], W.LB(c)), hk);
          dg = fmaf(W.W2T(k, c), g[c], dg);
        }
        const float dh = dg * gelu_exact_grad(hk);
        sg[k][tp] = gelu_exact(hk);
        sdh[k][tp] = dh;
#pragma unroll
        for (int c = 0; c < C; ++c) dln[c] = fmaf(W.W1(k, c), dh, dln[c]);
      }
      // LayerNorm backward: dxh = gamma dln; dx = r (dxh - mean(dxh) - xh mean(dxh xh)).
      // C = 1: exactly 0.  C = 2 in closed form: with d = (dxh0 - dxh1) / 2 and xh0 = u r,
      // dx0 = r d (1 - xh0^2) = d eps r^3 = -dx1 (no cancellation of 1 - xh0^2)
      if constexpr (C <= 2) {
        float dx0 = 0.f;
        if constexpr (C == 2) dx0 = 0.5f * (W.LW(0) * dln[0] - W.LW(1) * dln[1]) * (1e-6f * r * r * r);
#pragma unroll
        for (int c = 0; c < C; ++c) {
          dxd[base + (int64_t)c * HW] = c == 0 ? dx0 : -dx0;
          sdy[c][tp] = g[c];
          sln[c][tp] = fmaf(W.LW(c), xh[c], W.LB(c));
          sdln[c][tp] = dln[c];
          sxh[c][tp] = xh[c];
        }
      } else {
      float m1 = 0.f, m2 = 0.f;
#pragma unroll
      for (int c = 0; c < C; ++c) {
        const float d = W.LW(c) * dln[c];
        m1 += d;
        m2 = fmaf(d, xh[c], m2);
      }
      m1 *= 1.0f / C;
      m2 *= 1.0f / C;
#pragma unroll
      for (int c = 0; c < C; ++c) {
        dxd[base + (int64_t)c * HW] = r * (W.LW(c) * dln[c] - m1 - xh[c] * m2);
        sdy[c][tp] = g[c];
        sln[c][tp] = fmaf(W.LW(c), xh[c], W.LB(c));
        sdln[c][tp] = dln[c];
        sxh[c][tp] = xh[c];
      }
      }
    } else {
      for (int k = 0; k < H4; ++k) sg[k][tp] = sdh[k][tp] = 0.f;
#pragma unroll
      for (int c = 0; c < C; ++c) sdy[c][tp] = sln[c][tp] = sdln[c][tp] = sxh[c][tp] = 0.f;
    }
  }
  __syncthreads();
  constexpr int E = 8 * C * C + 7 * C;
  float* out = partial + (int64_t)blockIdx.x * E;
  for (int e = threadIdx.x; e < E; e += blockDim.x) {
    double acc = 0.0;      // fp64: a PB-long sequential sum per entry (cancellation-prone biases)
    if (e < H4 * C) {                                   // dW1[k][c] = sum dh_k ln_c
      const int k = e / C, c = e % C;
      for (int p = 0; p < PB; ++p) acc += (double)sdh[k][p] * sln[c][p];
    } else if (e < H4 * C + H4) {                       // db1[k]
      const int k = e - H4 * C;
      for (int p = 0; p < PB; ++p) acc += sdh[k][p];
    } else if (e < 2 * H4 * C + H4) {                   // dW2[c][k] = sum dy_c g_k
      const int q = e - H4 * C - H4, c = q / H4, k = q % H4;
      for (int p = 0; p < PB; ++p) acc += (double)sdy[c][p] * sg[k][p];
    } else if (e < 2 * H4 * C + H4 + C) {               // db2[c]
      const int c = e - 2 * H4 * C - H4;
      for (int p = 0; p < PB; ++p) acc += sdy[c][p];
    } else if (e < 2 * H4 * C + H4 + 2 * C) {           // dgamma[c] = sum dln_c xh_c
      const int c = e - 2 * H4 * C - H4 - C;
      for (int p = 0; p < PB; ++p) acc += (double)sdln[c][p] * sxh[c][p];
    } else {                                            // dbeta[c]
      const int c = e - 2 * H4 * C - H4 - 2 * C;
      for (int p = 0; p < PB; ++p) acc += sdln[c][p];
    }
    out[e] = (float)acc;
  }
}

// ---------------------------------------------------------------------- max pool
// window KH x KW (KH = 1 for MaxPool1d), stride = window, floor; arg = index in the window
__global__ __launch_bounds__(kBlock) void maxpool_fwd_kernel(
    const float* __restrict__ x, float* __restrict__ y, uint8_t* __restrict__ arg, int H, int W,
    int Ho, int Wo, int KH, int KW, int64_t total) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= total) return;
  const int wo = (int)(e % Wo);
  const int ho = (int)((e / Wo) % Ho);
  const int64_t nc = e / ((int64_t)Ho * Wo);
  const float* xp = x + nc * H * W + (int64_t)(ho * KH) * W + wo * KW;
  float m = xp[0];
  int a = 0;
  for (int i = 0; i < KH; ++i)
    for (int j = 0; j < KW; ++j) {
      const float v = xp[i * W + j];
      if (v > m || isnan(v)) {       // first maximum wins; a NaN propagates (torch's rule)
        m = v;
        a = i * KW + j;
      }
    }
  y[e] = m;
  arg[e] = (uint8_t)a;
}

__global__ __launch_bounds__(kBlock) void maxpool_bwd_kernel(
    const float* __restrict__ dy, const uint8_t* __restrict__ arg, float* __restrict__ dx, int H,
    int W, int Ho, int Wo, int KH, int KW, int64_t total) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= total) return;
  const int w = (int)(e % W);
  const int h = (int)((e / W) % H);
  const int64_t nc = e / ((int64_t)H * W);
  const int ho = h / KH, wo = w / KW;
  float v = 0.f;
  if (ho < Ho && wo < Wo) {
    const int64_t o = (nc * Ho + ho) * Wo + wo;
    if ((int)arg[o] == (h - ho * KH) * KW + (w - wo * KW)) v = dy[o];
  }
  dx[e] = v;
}

// ---------------------------------------------------------------------- transposed conv
// kernel = stride = (KH, KW); weight (Ci, Co, KH, KW); output Ho >= KH Hi, Wo >= KW Wi (the
// rows / columns past that are output_padding: bias only)
__global__ __launch_bounds__(kBlock) void convt_fwd_kernel(
    const float* __restrict__ x, const float* __restrict__ wt, const float* __restrict__ b,
    float* __restrict__ y, int Ci, int Hi, int Wi, int Co, int KH, int KW, int Ho, int Wo,
    int64_t total) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= total) return;
  const int wo = (int)(e % Wo);
  const int ho = (int)((e / Wo) % Ho);
  const int64_t nco = e / ((int64_t)Ho * Wo);
  const int co = (int)(nco % Co);
  const int n = (int)(nco / Co);
  float acc = b ? b[co] : 0.f;
  const int hi = ho / KH, wi = wo / KW;
  if (hi < Hi && wi < Wi) {
    const int a = ho - hi * KH, bb = wo - wi * KW;
    const float* xp = x + (int64_t)n * Ci * Hi * Wi + (int64_t)hi * Wi + wi;
    const float* wp = wt + ((int64_t)co * KH + a) * KW + bb;
    for (int ci = 0; ci < Ci; ++ci)
      acc = fmaf(xp[(int64_t)ci * Hi * Wi], wp[(int64_t)ci * Co * KH * KW], acc);
  }
  y[e] = acc;
}

__global__ __launch_bounds__(kBlock) void convt_bwd_data_kernel(
    const float* __restrict__ dy, const float* __restrict__ wt, float* __restrict__ dx, int Ci,
    int Hi, int Wi, int Co, int KH, int KW, int Ho, int Wo, int64_t total) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= total) return;
  const int wi = (int)(e % Wi);
  const int hi = (int)((e / Wi) % Hi);
  const int64_t nci = e / ((int64_t)Hi * Wi);
  const int ci = (int)(nci % Ci);
  const int n = (int)(nci / Ci);
  float acc = 0.f;
  for (int co = 0; co < Co; ++co) {
    const float* gp = dy + (((int64_t)n * Co + co) * Ho + (int64_t)hi * KH) * Wo + (int64_t)wi * KW;
    const float* wp = wt + ((int64_t)ci * Co + co) * KH * KW;
    for (int a = 0; a < KH; ++a)
      for (int bb = 0; bb < KW; ++bb) acc = fmaf(wp[a * KW + bb], gp[(int64_t)a * Wo + bb], acc);
  }
  dx[e] = acc;
}

// partial[n S + s][Ci Co KH KW + Co]: dW over input-pixel chunk s of sample n (flattened
// input pixels [s Q, (s+1) Q), their KH x KW output taps) and db over output-pixel chunk s
// (flattened output pixels, output_padding included); S chunks per sample.
constexpr int kConvtChunk = 64;
__global__ __launch_bounds__(kBlock) void convt_wgrad_kernel(
    const float* __restrict__ dy, const float* __restrict__ x, float* __restrict__ partial,
    int Ci, int Hi, int Wi, int Co, int KH, int KW, int Ho, int Wo, int S) {
  const int s = blockIdx.x, n = blockIdx.y;
  const int T = KH * KW;
  const int EW = Ci * Co * T, E = EW + Co;
  const int HWi = Hi * Wi, HWo = Ho * Wo;
  const int q0 = s * kConvtChunk, q1 = min(HWi, q0 + kConvtChunk);
  const int o0 = (int)((int64_t)s * HWo / S), o1 = (int)((int64_t)(s + 1) * HWo / S);
  const float* xs = x + (int64_t)n * Ci * HWi;
  const float* gs = dy + (int64_t)n * Co * HWo;
  float* out = partial + ((int64_t)n * S + s) * E;
  for (int e = blockIdx.z * blockDim.x + threadIdx.x; e < E; e += gridDim.z * blockDim.x) {
    float acc = 0.f;
    if (e < EW) {
      const int t = e % T, co = (e / T) % Co, ci = e / (T * Co);
      const int a = t / KW, bb = t - (t / KW) * KW;
      const float* xp = xs + (int64_t)ci * HWi;
      const float* gp = gs + (int64_t)co * HWo + (int64_t)a * Wo + bb;
      for (int q = q0; q < q1; ++q) {
        const int hi = q / Wi, wi = q - hi * Wi;
        acc = fmaf(xp[q], gp[(int64_t)hi * KH * Wo + wi * KW], acc);
      }
    } else {
      const float* gp = gs + (int64_t)(e - EW) * HWo;
      for (int o = o0; o < o1; ++o) acc += gp[o];
    }
    out[e] = acc;
  }
}

// ---------------------------------------------------------------------- temporal attention
// token means: xbar[bt] = (1/D) sum_d X[bt][d]  (one workgroup per token)
__global__ __launch_bounds__(kBlock) void tok_mean_kernel(const float* __restrict__ X,
                                                          float* __restrict__ xbar, int64_t D) {
  __shared__ float red[8];
  const float* xp = X + (int64_t)blockIdx.x * D;
  float s = 0.f;
  for (int64_t d = threadIdx.x; d < D; d += blockDim.x) s += xp[d];
  s = block_sum(s, red);
  if (threadIdx.x == 0) xbar[blockIdx.x] = s / (float)D;
}

constexpr int kGramPts = 32;     // points per LDS sub-tile
constexpr int kMaxTok = 480;     // tokens per bag: the Gram kernel's LDS tile (L x 33 floats) <= 64 KiB
constexpr int kGramChunk = 128;  // points per workgroup (one partial): D = 3721 -> 30 chunks

// partial[chunk][b][L][L]: the chunk's share of the centred Gram matrix; each thread owns 4 x 4
// blocks of the upper block triangle (blockIdx.y = round of 256 blocks) and mirrors them.
__global__ __launch_bounds__(kBlock) void tok_gram_kernel(const float* __restrict__ X,
                                                          const float* __restrict__ xbar,
                                                          float* __restrict__ partial, int B,
                                                          int L, int64_t D) {
  extern __shared__ float xs[];          // [L][kGramPts + 1]
  const int b = blockIdx.z, ch = blockIdx.x;
  const int nb = (L + 3) / 4, nblk = nb * (nb + 1) / 2;
  const int blk = blockIdx.y * kBlock + threadIdx.x;
  int bi = 0, bj = 0;
  const bool own = blk < nblk;
  if (own) {
    int r = blk;
    while (r >= nb - bi) { r -= nb - bi; ++bi; }
    bj = bi + r;
  }
  float acc[4][4] = {};
  const int64_t p0 = (int64_t)ch * kGramChunk;
  const int64_t p1 = p0 + kGramChunk < D ? p0 + kGramChunk : D;
  constexpr int LD = kGramPts + 1;
  const float* Xb = X + (int64_t)b * L * D;
  for (int64_t q0 = p0; q0 < p1; q0 += kGramPts) {
    __syncthreads();
    for (int e = threadIdx.x; e < L * kGramPts; e += blockDim.x) {
      const int t = e / kGramPts, q = e % kGramPts;
      xs[t * LD + q] = q0 + q < p1 ? Xb[(int64_t)t * D + q0 + q] - xbar[(int64_t)b * L + t] : 0.f;
    }
    __syncthreads();
    if (own) {
#pragma unroll 4
      for (int q = 0; q < kGramPts; ++q) {
        float u[4], v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int ti = 4 * bi + i, tj = 4 * bj + i;
          u[i] = ti < L ? xs[ti * LD + q] : 0.f;
          v[i] = tj < L ? xs[tj * LD + q] : 0.f;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(u[i], v[j], acc[i][j]);
      }
    }
  }
  if (!own) return;
  float* out = partial + ((int64_t)ch * B + b) * L * L;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int ti = 4 * bi + i, tj = 4 * bj + j;
      if (ti < L && tj < L) {
        out[(int64_t)ti * L + tj] = acc[i][j];
        out[(int64_t)tj * L + ti] = acc[i][j];
      }
    }
}

// Forward bag algebra, one workgroup per (token row l, bag b) -- B L workgroups, every row's
// L^2 work spread over the workgroup's threads.  In: Gc[b] (L x L), xbar[b] (L).  Out: row l of
// A[b] = softmax((Gc + D xbar xbar^T) / sqrt D), row l of P[b] = M Gc (M = A + I), and
// st[b][l] = (mu_l, r_l, ., .) with mu_l = sum_s M_ls xbar_s, var_l = (1/D) sum_s P_ls M_ls.
constexpr int kRowThreads = 128;
__global__ __launch_bounds__(kRowThreads) void tok_rows_kernel(const float* __restrict__ Gc,
                                                               const float* __restrict__ xbar,
                                                               float* __restrict__ A,
                                                               float* __restrict__ Pm,
                                                               float4* __restrict__ st, int L,
                                                               int64_t D, float eps) {
  __shared__ float red[4];
  __shared__ float arow[kMaxTok];
  const int l = blockIdx.x, b = blockIdx.y;
  const float* G = Gc + (int64_t)b * L * L;
  const float* xb = xbar + (int64_t)b * L;
  const float Df = (float)D, isd = 1.0f / sqrtf(Df);
  const float xl = xb[l];
  float mx = -INFINITY;
  for (int t = threadIdx.x; t < L; t += blockDim.x) {
    const float sc = (G[(int64_t)l * L + t] + Df * xl * xb[t]) * isd;
    arow[t] = sc;
    mx = fmaxf(mx, sc);
  }
  const float m = block_max(mx, red);
  float sum = 0.f;
  for (int t = threadIdx.x; t < L; t += blockDim.x) {
    const float e = __expf(arow[t] - m);
    arow[t] = e;
    sum += e;
  }
  const float inv = 1.0f / block_sum(sum, red);
  for (int t = threadIdx.x; t < L; t += blockDim.x) {
    arow[t] *= inv;
    A[((int64_t)b * L + l) * L + t] = arow[t];
  }
  __syncthreads();
  // P_ls = Gc_ls + sum_t A_lt Gc_ts (Gc rows coalesced over s), q = sum_s P_ls M_ls, mu
  float q = 0.f, mu = 0.f;
  for (int s2 = threadIdx.x; s2 < L; s2 += blockDim.x) {
    float p = G[(int64_t)l * L + s2];
    for (int t = 0; t < L; ++t) p = fmaf(arow[t], G[(int64_t)t * L + s2], p);
    Pm[((int64_t)b * L + l) * L + s2] = p;
    const float mls = arow[s2] + (s2 == l ? 1.f : 0.f);
    q = fmaf(p, mls, q);
    mu = fmaf(mls, xb[s2], mu);
  }
  q = block_sum(q, red);
  mu = block_sum(mu, red);
  if (threadIdx.x == 0) {
    const float var = fmaxf(q / Df, 0.f);
    st[(int64_t)b * L + l] = make_float4(mu, 1.0f / sqrtf(var + eps), 0.f, 0.f);
  }
}

// c_t = (1/L) sum_l r_l M_lt (into st[b][t].z) and kappa_b = (1/L) sum_l r_l mu_l; one
// workgroup per bag, thread = token t (A rows coalesced over t)
__global__ __launch_bounds__(kBlock) void tok_coef_kernel(const float* __restrict__ A,
                                                          float4* __restrict__ st,
                                                          float* __restrict__ kap, int L) {
  __shared__ float red[8];
  __shared__ float sr[kMaxTok];
  const int b = blockIdx.x;
  for (int l = threadIdx.x; l < L; l += blockDim.x) sr[l] = st[(int64_t)b * L + l].y;
  __syncthreads();
  const float iL = 1.0f / (float)L;
  const float* Ab = A + (int64_t)b * L * L;
  for (int t = threadIdx.x; t < L; t += blockDim.x) {
    float c = sr[t];
    for (int l = 0; l < L; ++l) c = fmaf(sr[l], Ab[(int64_t)l * L + t], c);
    st[(int64_t)b * L + t].z = c * iL;
  }
  float k = 0.f;
  for (int l = threadIdx.x; l < L; l += blockDim.x) k = fmaf(sr[l], st[(int64_t)b * L + l].x, k);
  k = block_sum(k, red);
  if (threadIdx.x == 0) kap[b] = k * iL;
}

// Ybar[b][d] = gamma[d] U[b][d] + beta[d],  U = sum_t c_t (X_t[d] - xbar_t) (saved for dgamma)
__global__ __launch_bounds__(kBlock) void tok_out_kernel(const float* __restrict__ X,
                                                         const float4* __restrict__ st,
                                                         const float* __restrict__ xbar,
                                                         const float* __restrict__ lw,
                                                         const float* __restrict__ lb,
                                                         float* __restrict__ Y,
                                                         float* __restrict__ U, int L, int64_t D) {
  const int b = blockIdx.y;
  const int64_t d = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= D) return;
  const float* Xb = X + (int64_t)b * L * D + d;
  float acc = 0.f;
  for (int t = 0; t < L; ++t)
    acc = fmaf(st[(int64_t)b * L + t].z, Xb[(int64_t)t * D] - xbar[(int64_t)b * L + t], acc);
  const float u = acc;
  U[(int64_t)b * D + d] = u;
  Y[(int64_t)b * D + d] = fmaf(lw[d], u, lb[d]);
}

// backward prep: h[b][t] = sum_d gamma[d] dY[b][d] (X_t[d] - xbar_t) (one workgroup per token;
// token b L is also the one that forms gb[b] = mean_d gamma dY)
__global__ __launch_bounds__(kBlock) void tok_bwd_dot_kernel(const float* __restrict__ X,
                                                             const float* __restrict__ xbar,
                                                             const float* __restrict__ dY,
                                                             const float* __restrict__ lw,
                                                             float* __restrict__ h,
                                                             float* __restrict__ gb, int L,
                                                             int64_t D) {
  __shared__ float red[8];
  const int bt = blockIdx.x, b = bt / L;
  const float* xp = X + (int64_t)bt * D;
  const float* gp = dY + (int64_t)b * D;
  const float xm = xbar[bt];
  float s = 0.f, s2 = 0.f;
  const bool first = bt % L == 0;
  for (int64_t d = threadIdx.x; d < D; d += blockDim.x) {
    const float g = lw[d] * gp[d];
    s = fmaf(g, xp[d] - xm, s);
    if (first) s2 += g;
  }
  s = block_sum(s, red);
  if (threadIdx.x == 0) h[bt] = s;
  if (first) {
    s2 = block_sum(s2, red);
    if (threadIdx.x == 0) gb[b] = s2 / (float)D;
  }
}

// dgamma[d] = sum_b dY[b][d] U[b][d],  dbeta[d] = sum_b dY[b][d]
__global__ __launch_bounds__(kBlock) void tok_ln_wgrad_kernel(const float* __restrict__ dY,
                                                              const float* __restrict__ U,
                                                              float* __restrict__ dlw,
                                                              float* __restrict__ dlb, int B,
                                                              int64_t D) {
  const int64_t d = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= D) return;
  float a = 0.f, c = 0.f;
  for (int b = 0; b < B; ++b) {
    const float g = dY[(int64_t)b * D + d];
    a = fmaf(g, U[(int64_t)b * D + d], a);
    c += g;
  }
  if (dlw) dlw[d] = a;
  if (dlb) dlb[d] = c;
}

// Backward bag algebra, two row-parallel passes (B L workgroups each).
// Pass 1, workgroup (l, b): a_l = r_l / L, b_l = a_l r_l^2 (sum_t M_lt h_t) / D, the row
// dA_l. = a_l h - b_l P_l. and the softmax backward dS_l. = A_l. o (dA_l. - A_l..dA_l.), written
// to W[b]; ab[b][l] = (a_l, b_l).
__global__ __launch_bounds__(kRowThreads) void tok_bwd_rows_kernel(
    const float* __restrict__ A, const float* __restrict__ Pm, const float4* __restrict__ st,
    const float* __restrict__ h, float* __restrict__ Wk, float2* __restrict__ ab, int L,
    int64_t D) {
  __shared__ float red[4];
  const int l = blockIdx.x, b = blockIdx.y;
  const float* Arow = A + ((int64_t)b * L + l) * L;
  const float* Prow = Pm + ((int64_t)b * L + l) * L;
  const float* hb = h + (int64_t)b * L;
  const float Df = (float)D;
  const float r = st[(int64_t)b * L + l].y;
  float go = 0.f;
  for (int t = threadIdx.x; t < L; t += blockDim.x) go = fmaf(Arow[t] + (t == l ? 1.f : 0.f), hb[t], go);
  go = block_sum(go, red);
  const float al = r / (float)L;
  const float bl = al * r * r * go / Df;
  float dot = 0.f;
  for (int t = threadIdx.x; t < L; t += blockDim.x)
    dot = fmaf(Arow[t], al * hb[t] - bl * Prow[t], dot);
  dot = block_sum(dot, red);
  float* Wrow = Wk + ((int64_t)b * L + l) * L;
  for (int t = threadIdx.x; t < L; t += blockDim.x)
    Wrow[t] = Arow[t] * (al * hb[t] - bl * Prow[t] - dot);
  if (threadIdx.x == 0) ab[(int64_t)b * L + l] = make_float2(al, bl);
}

// Pass 2, workgroup (t, b): row t of R = (dS + dS^T)/sqrt D - N, N_ts = sum_l M_lt b_l M_ls, and
// coef[b][t] = (a_t, k_t): a_t = sum_l M_lt alpha_l, k_t = sum_s Q_ts xbar_s - a_t gb.
__global__ __launch_bounds__(kRowThreads) void tok_bwd_rrow_kernel(
    const float* __restrict__ A, const float* __restrict__ Wk, const float2* __restrict__ ab,
    const float* __restrict__ xbar, const float* __restrict__ gbar, float* __restrict__ R,
    float2* __restrict__ coef, int L, int64_t D) {
  __shared__ float red[4];
  __shared__ float mcol[kMaxTok];
  const int t = blockIdx.x, b = blockIdx.y;
  const float* Ab = A + (int64_t)b * L * L;
  const float* Wb = Wk + (int64_t)b * L * L;
  const float isd = 1.0f / sqrtf((float)D);
  float a = 0.f;
  for (int l = threadIdx.x; l < L; l += blockDim.x) {
    const float2 abl = ab[(int64_t)b * L + l];
    const float mlt = Ab[(int64_t)l * L + t] + (l == t ? 1.f : 0.f);
    mcol[l] = mlt * abl.y;                       // M_lt b_l
    a = fmaf(mlt, abl.x, a);
  }
  a = block_sum(a, red);                          // (the reduction's barriers publish mcol)
  float k = 0.f;
  for (int s2 = threadIdx.x; s2 < L; s2 += blockDim.x) {
    float n = 0.f;
    for (int l = 0; l < L; ++l) n = fmaf(mcol[l], Ab[(int64_t)l * L + s2] + (l == s2 ? 1.f : 0.f), n);
    const float qv = (Wb[(int64_t)t * L + s2] + Wb[(int64_t)s2 * L + t]) * isd;
    R[((int64_t)b * L + t) * L + s2] = qv - n;
    k = fmaf(qv, xbar[(int64_t)b * L + s2], k);
  }
  k = block_sum(k, red);
  if (threadIdx.x == 0) coef[(int64_t)b * L + t] = make_float2(a, k - a * gbar[b]);
}

// dX[b][t][d] = a_t gamma[d] dY[b][d] + sum_s R_ts (X_s[d] - xbar_s) + k_t; a thread owns kTT
// tokens of one point d (R loads are wave-uniform, X_s[d] coalesced over d)
constexpr int kTT = 8;
__global__ __launch_bounds__(kBlock) void tok_bwd_dx_kernel(const float* __restrict__ X,
                                                            const float* __restrict__ xbar,
                                                            const float* __restrict__ R,
                                                            const float2* __restrict__ coef,
                                                            const float* __restrict__ lw,
                                                            const float* __restrict__ dY,
                                                            float* __restrict__ dX, int L,
                                                            int64_t D) {
  const int b = blockIdx.z, t0 = blockIdx.y * kTT;
  const int64_t d = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= D) return;
  const float* Xb = X + (int64_t)b * L * D + d;
  const float* Rb = R + (int64_t)b * L * L;
  float acc[kTT] = {};
  for (int s = 0; s < L; ++s) {
    const float xs = Xb[(int64_t)s * D] - xbar[(int64_t)b * L + s];
#pragma unroll
    for (int i = 0; i < kTT; ++i)
      if (t0 + i < L) acc[i] = fmaf(Rb[(int64_t)(t0 + i) * L + s], xs, acc[i]);
  }
  const float g = lw[d] * dY[(int64_t)b * D + d];
#pragma unroll
  for (int i = 0; i < kTT; ++i) {
    const int t = t0 + i;
    if (t < L) {
      const float2 c = coef[(int64_t)b * L + t];
      dX[((int64_t)b * L + t) * D + d] = fmaf(c.x, g, acc[i] + c.y);
    }
  }
}

inline int blocks_for(int64_t n) { return (int)((n + kBlock - 1) / kBlock); }

}  // namespace

// ============================================================================== C ABI

BLINDNO_API int blindno_dwconv_fwd(const float* x, const float* w, const float* b, float* y, int N,
                                   int C, int H, int W, int KH, int KW, void* stream) {
  if (N < 1 || C < 1 || H < 1 || W < 1 || KH < 1 || KW < 1 || KH * KW > kMaxTaps)
    return (int)hipErrorInvalidValue;
  const int64_t total = (int64_t)N * C * H * W;
  dwconv_fwd_kernel<<<blocks_for(total), kBlock, 0, (hipStream_t)stream>>>(x, w, b, y, C, H, W, KH,
                                                                         KW, total);
  return (int)hipGetLastError();
}

BLINDNO_API int blindno_dwconv_bwd_data(const float* dy, const float* w, float* dx, int N, int C,
                                        int H, int W, int KH, int KW, void* stream) {
  if (N < 1 || C < 1 || H < 1 || W < 1 || KH < 1 || KW < 1 || KH * KW > kMaxTaps)
    return (int)hipErrorInvalidValue;
  const int64_t total = (int64_t)N * C * H * W;
  dwconv_bwd_data_kernel<<<blocks_for(total), kBlock, 0, (hipStream_t)stream>>>(dy, w, dx, C, H, W,
                                                                              KH, KW, total);
  return (int)hipGetLastError();
}

BLINDNO_API int blindno_dwconv_wgrad_nsplit(int N, int C, int H, int W) {
  // ~1024 output pixels per workgroup (4 per thread), so even a 1-channel level fills the chip
  const int64_t P = (int64_t)N * H * W;
  int64_t s = (P + 1023) / 1024;
  return (int)(s < 1 ? 1 : (s > 2048 ? 2048 : s));
}

BLINDNO_API int blindno_dwconv_bwd_weight(const float* dy, const float* x, float* dwb,
                                          float* partial, int nsplit, int N, int C, int H, int W,
                                          int KH, int KW, void* stream) {
  if (N < 1 || C < 1 || KH * KW > kMaxTaps || nsplit < 1 || (nsplit > 1 && !partial))
    return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  float* dst = nsplit > 1 ? partial : dwb;
  dwconv_wgrad_kernel<<<dim3(nsplit, C), kBlock, 0, st>>>(dy, x, dst, N, C, H, W, KH, KW, nsplit);
  if (nsplit > 1) return blindno_reduce_partials(partial, dwb, nsplit, C * (KH * KW + 1), stream);
  return (int)hipGetLastError();
}

#define CNX_DISPATCH(C_, ...)                                          \
  switch (C_) {                                                        \
    case 1: { constexpr int CC = 1; __VA_ARGS__; } break;             \
    case 2: { constexpr int CC = 2; __VA_ARGS__; } break;             \
    case 4: { constexpr int CC = 4; __VA_ARGS__; } break;             \
    case 8: { constexpr int CC = 8; __VA_ARGS__; } break;             \
    case 16: { constexpr int CC = 16; __VA_ARGS__; } break;           \
    case 32: { constexpr int CC = 32; __VA_ARGS__; } break;           \
    case 64: { constexpr int CC = 64; __VA_ARGS__; } break;           \
    default: return (int)hipErrorInvalidValue;                         \
  }

BLINDNO_API int blindno_cnx_pw_fwd(const float* xd, const float* sc, const float* lw,
                                   const float* lb, const float* w1, const float* b1,
                                   const float* w2, const float* b2, float* y, int N, int C,
                                   int HW, void* stream) {
  if (N < 1 || HW < 1) return (int)hipErrorInvalidValue;
  const int64_t P = (int64_t)N * HW;
  hipStream_t st = (hipStream_t)stream;
  CNX_DISPATCH(C, cnx_pw_fwd_kernel<CC><<<blocks_for(P), kBlock, 0, st>>>(xd, sc, lw, lb, w1, b1, w2,
                                                                          b2, y, N, HW));
  return (int)hipGetLastError();
}

BLINDNO_API int blindno_cnx_pw_bwd_nblk(int N, int C, int HW) {
  if (C < 1 || C > 64 || (C & (C - 1))) return -1;
  const int pb = cnx_pb(C);
  return (int)(((int64_t)N * HW + pb - 1) / pb);
}

// dparams = [dW1 (4C x C) | db1 (4C) | dW2 (C x 4C) | db2 (C) | dgamma (C) | dbeta (C)];
// partial: nblk x (8 C^2 + 7 C) floats
BLINDNO_API int blindno_cnx_pw_bwd(const float* dy, const float* xd, const float* lw,
                                   const float* lb, const float* w1, const float* b1,
                                   const float* w2, float* dxd, float* dparams, float* partial,
                                   int nblk, int N, int C, int HW, void* stream) {
  if (N < 1 || HW < 1 || nblk != blindno_cnx_pw_bwd_nblk(N, C, HW) || !partial)
    return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  CNX_DISPATCH(C, cnx_pw_bwd_kernel<CC><<<nblk, kBlock, 0, st>>>(dy, xd, lw, lb, w1, b1, w2, dxd,
                                                                 partial, N, HW));
  const int err = (int)hipGetLastError();
  if (err) return err;
  return blindno_reduce_partials(partial, dparams, nblk, 8 * C * C + 7 * C, stream);
}

BLINDNO_API int blindno_maxpool_fwd(const float* x, float* y, uint8_t* arg, int NC, int H, int W,
                                    int KH, int KW, void* stream) {
  if (NC < 1 || KH < 1 || KW < 1 || KH * KW > 255 || H < KH || W < KW) return (int)hipErrorInvalidValue;
  const int Ho = H / KH, Wo = W / KW;
  const int64_t total = (int64_t)NC * Ho * Wo;
  maxpool_fwd_kernel<<<blocks_for(total), kBlock, 0, (hipStream_t)stream>>>(x, y, arg, H, W, Ho, Wo,
                                                                          KH, KW, total);
  return (int)hipGetLastError();
}

BLINDNO_API int blindno_maxpool_bwd(const float* dy, const uint8_t* arg, float* dx, int NC, int H,
                                    int W, int KH, int KW, void* stream) {
  if (NC < 1 || KH < 1 || KW < 1 || H < KH || W < KW) return (int)hipErrorInvalidValue;
  const int Ho = H / KH, Wo = W / KW;
  const int64_t total = (int64_t)NC * H * W;
  maxpool_bwd_kernel<<<blocks_for(total), kBlock, 0, (hipStream_t)stream>>>(dy, arg, dx, H, W, Ho, Wo,
                                                                          KH, KW, total);
  return (int)hipGetLastError();
}

BLINDNO_API int blindno_convt_fwd(const float* x, const float* w, const float* b, float* y, int N,
                                  int Ci, int Hi, int Wi, int Co, int KH, int KW, int Ho, int Wo,
                                  void* stream) {
  if (N < 1 || Ci < 1 || Co < 1 || Ho < KH * Hi || Wo < KW * Wi || Ho >= KH * Hi + KH ||
      Wo >= KW * Wi + KW)
    return (int)hipErrorInvalidValue;
  const int64_t total = (int64_t)N * Co * Ho * Wo;
  convt_fwd_kernel<<<blocks_for(total), kBlock, 0, (hipStream_t)stream>>>(x, w, b, y, Ci, Hi, Wi, Co,
                                                                        KH, KW, Ho, Wo, total);
  return (int)hipGetLastError();
}

BLINDNO_API int blindno_convt_bwd_data(const float* dy, const float* w, float* dx, int N, int Ci,
                                       int Hi, int Wi, int Co, int KH, int KW, int Ho, int Wo,
                                       void* stream) {
  if (N < 1 || Ci < 1 || Co < 1 || Ho < KH * Hi || Wo < KW * Wi) return (int)hipErrorInvalidValue;
  const int64_t total = (int64_t)N * Ci * Hi * Wi;
  convt_bwd_data_kernel<<<blocks_for(total), kBlock, 0, (hipStream_t)stream>>>(dy, w, dx, Ci, Hi, Wi,
                                                                             Co, KH, KW, Ho, Wo, total);
  return (int)hipGetLastError();
}

// dwb = [dW (Ci Co KH KW) | db (Co)]; partial: blindno_convt_wgrad_nparts(N, Hi, Wi) x
// (Ci Co KH KW + Co) floats
BLINDNO_API int blindno_convt_wgrad_nparts(int N, int Hi, int Wi) {
  return N * ((Hi * Wi + kConvtChunk - 1) / kConvtChunk);
}

BLINDNO_API int blindno_convt_bwd_weight(const float* dy, const float* x, float* dwb,
                                         float* partial, int N, int Ci, int Hi, int Wi, int Co,
                                         int KH, int KW, int Ho, int Wo, void* stream) {
  if (N < 1 || Ci < 1 || Co < 1 || !partial) return (int)hipErrorInvalidValue;
  const int E = Ci * Co * KH * KW + Co;
  const int S = (Hi * Wi + kConvtChunk - 1) / kConvtChunk;
  int gz = (E + kBlock - 1) / kBlock;
  if (gz > 16) gz = 16;
  hipStream_t st = (hipStream_t)stream;
  convt_wgrad_kernel<<<dim3(S, N, gz), kBlock, 0, st>>>(dy, x, partial, Ci, Hi, Wi, Co, KH, KW, Ho, Wo, S);
  const int err = (int)hipGetLastError();
  if (err) return err;
  return blindno_reduce_partials(partial, dwb, N * S, E, stream);
}

BLINDNO_API int blindno_tok_gram_nchunk(int64_t D) {
  return (int)((D + kGramChunk - 1) / kGramChunk);
}

// Saved state of the temporal attention forward (floats; 16-B aligned base), kept until the
// backward:  save = [st (4 B L) | xbar (B L) | A (B L L) | P (B L L) | kappa (B) | U (B D)]
// gram: B L L floats; gram_partial: blindno_tok_gram_nchunk(D) x B L L floats (NULL if 1)
BLINDNO_API int64_t blindno_tok_attn_save_floats(int B, int L, int64_t D) {
  return (int64_t)B * L + 2 * (int64_t)B * L * L + 4 * (int64_t)B * L + B + (int64_t)B * D;
}

BLINDNO_API int blindno_tok_attn_fwd(const float* X, const float* lw, const float* lb, float* Y,
                                     float* save, float* gram_partial, float* gram, int B, int L,
                                     int64_t D, float eps, void* stream) {
  if (B < 1 || L < 1 || L > kMaxTok || D < 1 || !save || !gram) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  const int64_t BL = (int64_t)B * L, BLL = BL * L;
  float4* stt = reinterpret_cast<float4*>(save);
  float* xbar = save + 4 * BL;
  float* A = xbar + BL;
  float* Pm = A + BLL;
  float* kap = Pm + BLL;
  float* U = kap + B;
  if ((reinterpret_cast<uintptr_t>(save) & 15) != 0) return (int)hipErrorInvalidValue;
  tok_mean_kernel<<<(unsigned)BL, kBlock, 0, st>>>(X, xbar, D);
  const int nch = blindno_tok_gram_nchunk(D);
  const int nb = (L + 3) / 4, nblk = nb * (nb + 1) / 2;
  const size_t lds = (size_t)L * (kGramPts + 1) * sizeof(float);
  float* gdst = nch > 1 ? gram_partial : gram;
  if (nch > 1 && !gram_partial) return (int)hipErrorInvalidValue;
  tok_gram_kernel<<<dim3(nch, (nblk + kBlock - 1) / kBlock, B), kBlock, lds, st>>>(X, xbar, gdst, B, L, D);
  int err = (int)hipGetLastError();
  if (err) return err;
  if (nch > 1) {
    err = blindno_reduce_partials(gram_partial, gram, nch, (int)BLL, stream);
    if (err) return err;
  }
  tok_rows_kernel<<<dim3(L, B), kRowThreads, 0, st>>>(gram, xbar, A, Pm, stt, L, D, eps);
  tok_coef_kernel<<<B, kBlock, 0, st>>>(A, stt, kap, L);
  tok_out_kernel<<<dim3((unsigned)((D + kBlock - 1) / kBlock), B), kBlock, 0, st>>>(X, stt, xbar, lw, lb,
                                                                                   Y, U, L, D);
  return (int)hipGetLastError();
}

// Backward scratch (floats; 8-B aligned base): coef (2 B L) | h (B L) | gbar (B) | R (B L L) |
// W (B L L) | [pad to 8 B] | ab (2 B L)
BLINDNO_API int64_t blindno_tok_attn_bwd_scratch_floats(int B, int L) {
  const int64_t BL = (int64_t)B * L;
  return 2 * BL + BL + B + 2 * BL * L + 1 + 2 * BL;
}

BLINDNO_API int blindno_tok_attn_bwd(const float* dY, const float* X, const float* lw,
                                     const float* save, float* dX, float* dlw, float* dlb,
                                     float* scratch, int B, int L, int64_t D, void* stream) {
  if (B < 1 || L < 1 || L > kMaxTok || D < 1 || !scratch || !save ||
      (reinterpret_cast<uintptr_t>(save) & 15) || (reinterpret_cast<uintptr_t>(scratch) & 7))
    return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  const int64_t BL = (int64_t)B * L, BLL = BL * L;
  const float4* stt = reinterpret_cast<const float4*>(save);
  const float* xbar = save + 4 * BL;
  const float* A = xbar + BL;
  const float* Pm = A + BLL;
  const float* U = Pm + BLL + B;
  float2* coef = reinterpret_cast<float2*>(scratch);
  float* h = scratch + 2 * BL;
  float* gb = h + BL;
  float* R = gb + B;
  float* Wk = R + BLL;
  if (dlw || dlb)
    tok_ln_wgrad_kernel<<<(unsigned)((D + kBlock - 1) / kBlock), kBlock, 0, st>>>(dY, U, dlw, dlb, B, D);
  if (dX) {
    tok_bwd_dot_kernel<<<(unsigned)BL, kBlock, 0, st>>>(X, xbar, dY, lw, h, gb, L, D);
    float2* abv = reinterpret_cast<float2*>(h + BL + B + 2 * BLL + ((BL + B) & 1));
    tok_bwd_rows_kernel<<<dim3(L, B), kRowThreads, 0, st>>>(A, Pm, stt, h, Wk, abv, L, D);
    tok_bwd_rrow_kernel<<<dim3(L, B), kRowThreads, 0, st>>>(A, Wk, abv, xbar, gb, R, coef, L, D);
    tok_bwd_dx_kernel<<<dim3((unsigned)((D + kBlock - 1) / kBlock), (L + kTT - 1) / kTT, B), kBlock, 0,
                        st>>>(X, xbar, R, coef, lw, dY, dX, L, D);
  }
  return (int)hipGetLastError();
}
