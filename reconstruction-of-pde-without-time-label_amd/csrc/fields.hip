// Point-wise field kernels of the FNO body: lift (fc0 + pad), inverse row transform with
// the fused 1x1-conv/bias epilogue, its backward, weight-gradient partial reductions,
// the projection MLP (fc1 -> GELU -> fc2), the snapshot-bag mean, loss, metrics and Adam.
//
// Reference: FNO2d.forward 2d_FPE/FNOModules.py:218-240, FNO1d.forward
// 1d_FPE/FNOModules.py:99-122, NIOFP2D_FNO bag mean 2d_FPE/NIOModules.py:565-575,
// train loop 2d_FPE/train_fno.py:116-146.
#include "common.h"

using namespace blindno;

namespace {

// ---------------------------------------------------------------- lift
__global__ __launch_bounds__(kBlock) void lift_fwd_kernel(const float* __restrict__ in,
                                                          const float* __restrict__ w0,
                                                          const float* __restrict__ b0,
                                                          float* __restrict__ x0, int Bn, int N1,
                                                          int N2, int Cin, int C, int P1,
                                                          int P2) {
  const int64_t total = (int64_t)Bn * C * P1 * P2;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    int w = (int)(idx % P2);
    int64_t t = idx / P2;
    int h = (int)(t % P1);
    t /= P1;
    int c = (int)(t % C);
    int n = (int)(t / C);
    float v = 0.f;
    if (h < N1 && w < N2) {
      const float* ip = in + (((int64_t)n * N1 + h) * N2 + w) * Cin;
      v = b0[c];
      for (int j = 0; j < Cin; ++j) v = fmaf(w0[c * Cin + j], ip[j], v);
    }
    x0[idx] = v;
  }
}

__global__ __launch_bounds__(kBlock) void lift_bwd_in_kernel(const float* __restrict__ dx0,
                                                             const float* __restrict__ w0,
                                                             float* __restrict__ d_in, int Bn,
                                                             int N1, int N2, int Cin, int C,
                                                             int P1, int P2) {
  const int64_t total = (int64_t)Bn * N1 * N2 * Cin;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    int j = (int)(idx % Cin);
    int64_t t = idx / Cin;
    int w = (int)(t % N2);
    t /= N2;
    int h = (int)(t % N1);
    int n = (int)(t / N1);
    float v = 0.f;
    for (int c = 0; c < C; ++c)
      v = fmaf(w0[c * Cin + j], dx0[(((int64_t)n * C + c) * P1 + h) * P2 + w], v);
    d_in[idx] = v;
  }
}

// partial[chunk][c*Cin + j] = sum dx0[n,c,h,w] in[n,h,w,j];  partial[chunk][C*Cin + c] = sum dx0
__global__ __launch_bounds__(kBlock) void lift_bwd_w_kernel(const float* __restrict__ dx0,
                                                            const float* __restrict__ in,
                                                            float* __restrict__ partial,
                                                            int nchunk, int Bn, int N1, int N2,
                                                            int Cin, int C, int P1, int P2) {
  const int np = C * Cin + C;
  const int64_t npts = (int64_t)Bn * N1 * N2;
  const int64_t per = (npts + nchunk - 1) / nchunk;
  const int64_t total = (int64_t)nchunk * np;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    int p = (int)(idx % np);
    int chunk = (int)(idx / np);
    int c, j;
    if (p < C * Cin) {
      c = p / Cin;
      j = p % Cin;
    } else {
      c = p - C * Cin;
      j = -1;
    }
    int64_t beg = chunk * per, end = beg + per < npts ? beg + per : npts;
    float acc = 0.f;
    for (int64_t q = beg; q < end; ++q) {
      int w = (int)(q % N2);
      int64_t t = q / N2;
      int h = (int)(t % N1);
      int n = (int)(t / N1);
      float d = dx0[(((int64_t)n * C + c) * P1 + h) * P2 + w];
      acc = j >= 0 ? fmaf(d, in[q * Cin + j], acc) : acc + d;
    }
    partial[idx] = acc;
  }
}

// ---------------------------------------------------------------- inverse row transform + epilogue
template <int ACT>
__global__ __launch_bounds__(kBlock) void rowidft_epi_kernel(
    const float2* __restrict__ Z, const float* __restrict__ x, const float* __restrict__ wc,
    const float* __restrict__ bc, float* __restrict__ z, const float2* __restrict__ tw2, int Bn,
    int C, int P1, int P2, int m2) {
  extern __shared__ float2 s_tw[];
  for (int i = threadIdx.x; i < P2; i += blockDim.x) s_tw[i] = tw2[i];
  __syncthreads();
  const int64_t HW = (int64_t)P1 * P2;
  const int64_t total = (int64_t)Bn * C * HW;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    int w = (int)(idx % P2);
    int64_t t = idx / P2;
    int h = (int)(t % P1);
    t /= P1;
    int o = (int)(t % C);
    int n = (int)(t / C);
    const float2* zc = Z + (((int64_t)n * C + o) * P1 + h) * m2;
    float acc = 0.f;
    int ph = 0;
    for (int k = 0; k < m2; ++k) {
      float2 a = zc[k];
      float2 e = s_tw[ph];
      acc = fmaf(a.x, e.x, fmaf(-a.y, e.y, acc));
      ph += w;
      if (ph >= P2) ph -= P2;
    }
    float cv = 0.f;
    if (wc) {
      cv = bc[o];
      const float* xp = x + (int64_t)n * C * HW + (int64_t)h * P2 + w;
      for (int i = 0; i < C; ++i) {
        float v = xp[i * HW];
        if (ACT) v = gelu_f(v);
        cv = fmaf(wc[o * C + i], v, cv);
      }
    }
    z[idx] = acc + cv;
  }
}

template <int ACT>
__global__ __launch_bounds__(kBlock) void rowidft_bwd_kernel(
    const float2* __restrict__ G, const float* __restrict__ dz, const float* __restrict__ wc,
    const float* __restrict__ xpre, float* __restrict__ dx, const float2* __restrict__ tw2,
    int Bn, int C, int P1, int P2, int m2) {
  extern __shared__ float2 s_tw[];
  for (int i = threadIdx.x; i < P2; i += blockDim.x) s_tw[i] = tw2[i];
  __syncthreads();
  const int64_t HW = (int64_t)P1 * P2;
  const int64_t total = (int64_t)Bn * C * HW;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    int w = (int)(idx % P2);
    int64_t t = idx / P2;
    int h = (int)(t % P1);
    t /= P1;
    int i = (int)(t % C);
    int n = (int)(t / C);
    const float2* gc = G + (((int64_t)n * C + i) * P1 + h) * m2;
    float acc = 0.f;
    int ph = 0;
    for (int k = 0; k < m2; ++k) {
      float2 a = gc[k];
      float2 e = s_tw[ph];
      acc = fmaf(a.x, e.x, fmaf(-a.y, e.y, acc));
      ph += w;
      if (ph >= P2) ph -= P2;
    }
    if (wc) {
      const float* dzp = dz + (int64_t)n * C * HW + (int64_t)h * P2 + w;
      for (int o = 0; o < C; ++o) acc = fmaf(wc[o * C + i], dzp[o * HW], acc);
    }
    if (ACT) acc *= gelu_grad_f(xpre[idx]);
    dx[idx] = acc;
  }
}

// partial[chunk][o*C + i] = sum dz[n,o,p] f(x[n,i,p]);  partial[chunk][C*C + o] = sum dz[n,o,p]
template <int ACT>
__global__ __launch_bounds__(kBlock) void conv_wgrad_kernel(const float* __restrict__ dz,
                                                            const float* __restrict__ x,
                                                            float* __restrict__ partial,
                                                            int nchunk, int Bn, int C,
                                                            int64_t HW) {
  const int np = C * C + C;
  const int64_t npts = (int64_t)Bn * HW;
  const int64_t per = (npts + nchunk - 1) / nchunk;
  const int64_t total = (int64_t)nchunk * np;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    int p = (int)(idx % np);
    int chunk = (int)(idx / np);
    int o, i;
    if (p < C * C) {
      o = p / C;
      i = p % C;
    } else {
      o = p - C * C;
      i = -1;
    }
    int64_t beg = chunk * per, end = beg + per < npts ? beg + per : npts;
    float acc = 0.f;
    for (int64_t q = beg; q < end; ++q) {
      int64_t n = q / HW, s = q % HW;
      float d = dz[(n * C + o) * HW + s];
      if (i >= 0) {
        float v = x[(n * C + i) * HW + s];
        if (ACT) v = gelu_f(v);
        acc = fmaf(d, v, acc);
      } else {
        acc += d;
      }
    }
    partial[idx] = acc;
  }
}

__global__ __launch_bounds__(kBlock) void reduce_partials_kernel(const float* __restrict__ partial,
                                                                 float* __restrict__ out,
                                                                 int nchunk, int np) {
  for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < np; p += gridDim.x * blockDim.x) {
    float acc = 0.f;
    for (int c = 0; c < nchunk; ++c) acc += partial[(int64_t)c * np + p];
    out[p] = acc;
  }
}

// ---------------------------------------------------------------- projection MLP
template <int CM, int COM>
__global__ __launch_bounds__(kBlock) void project_fwd_kernel(
    const float* __restrict__ z, const float* __restrict__ w1, const float* __restrict__ b1,
    const float* __restrict__ w2, const float* __restrict__ b2, float* __restrict__ out, int Bn,
    int C, int P1, int P2, int Ho, int Wo, int Hd, int Cout, int ostride, int ooff) {
  const int64_t HW = (int64_t)P1 * P2;
  const int64_t total = (int64_t)Bn * Ho * Wo;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    int w = (int)(idx % Wo);
    int64_t t = idx / Wo;
    int h = (int)(t % Ho);
    int n = (int)(t / Ho);
    float zi[CM];
    const float* zp = z + (int64_t)n * C * HW + (int64_t)h * P2 + w;
#pragma unroll
    for (int i = 0; i < CM; ++i) zi[i] = i < C ? zp[i * HW] : 0.f;
    float acc[COM];
#pragma unroll
    for (int c = 0; c < COM; ++c) acc[c] = c < Cout ? b2[c] : 0.f;
    for (int j = 0; j < Hd; ++j) {
      float hv = b1[j];
#pragma unroll
      for (int i = 0; i < CM; ++i)
        if (i < C) hv = fmaf(w1[j * C + i], zi[i], hv);
      float a = gelu_f(hv);
#pragma unroll
      for (int c = 0; c < COM; ++c)
        if (c < Cout) acc[c] = fmaf(w2[c * Hd + j], a, acc[c]);
    }
    float* op = out + idx * ostride + ooff;
#pragma unroll
    for (int c = 0; c < COM; ++c)
      if (c < Cout) op[c] = acc[c];
  }
}

template <int CM, int COM>
__global__ __launch_bounds__(kBlock) void project_bwd_dz_kernel(
    const float* __restrict__ z, const float* __restrict__ w1, const float* __restrict__ b1,
    const float* __restrict__ w2, const float* __restrict__ dout, float* __restrict__ dz, int Bn,
    int C, int P1, int P2, int Ho, int Wo, int Hd, int Cout, int ostride, int ooff,
    int dout_div) {
  const int64_t HW = (int64_t)P1 * P2;
  const int64_t total = (int64_t)Bn * Ho * Wo;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    int w = (int)(idx % Wo);
    int64_t t = idx / Wo;
    int h = (int)(t % Ho);
    int n = (int)(t / Ho);
    float zi[CM], gz[CM], go[COM];
    const float* zp = z + (int64_t)n * C * HW + (int64_t)h * P2 + w;
#pragma unroll
    for (int i = 0; i < CM; ++i) {
      zi[i] = i < C ? zp[i * HW] : 0.f;
      gz[i] = 0.f;
    }
    const float* dp = dout + ((((int64_t)(n / dout_div)) * Ho + h) * Wo + w) * ostride + ooff;
#pragma unroll
    for (int c = 0; c < COM; ++c) go[c] = c < Cout ? dp[c] : 0.f;
    for (int j = 0; j < Hd; ++j) {
      float hv = b1[j];
#pragma unroll
      for (int i = 0; i < CM; ++i)
        if (i < C) hv = fmaf(w1[j * C + i], zi[i], hv);
      float da = 0.f;
#pragma unroll
      for (int c = 0; c < COM; ++c)
        if (c < Cout) da = fmaf(w2[c * Hd + j], go[c], da);
      float dh = da * gelu_grad_f(hv);
#pragma unroll
      for (int i = 0; i < CM; ++i)
        if (i < C) gz[i] = fmaf(w1[j * C + i], dh, gz[i]);
    }
    float* dzp = dz + (int64_t)n * C * HW + (int64_t)h * P2 + w;
#pragma unroll
    for (int i = 0; i < CM; ++i)
      if (i < C) dzp[i * HW] = gz[i];
  }
}

// partial[chunk][...] = [dW1 (Hd*C) | db1 (Hd) | dW2 (Cout*Hd) | db2 (Cout)]
// One thread per (chunk, hidden unit j); thread j == 0 also accumulates db2.
template <int CM, int COM>
__global__ __launch_bounds__(kBlock) void project_bwd_w_kernel(
    const float* __restrict__ z, const float* __restrict__ w1, const float* __restrict__ b1,
    const float* __restrict__ w2, const float* __restrict__ dout, float* __restrict__ partial,
    int nchunk, int Bn, int C, int P1, int P2, int Ho, int Wo, int Hd, int Cout, int ostride,
    int ooff, int dout_div) {
  const int np = Hd * C + Hd + Cout * Hd + Cout;
  const int64_t HW = (int64_t)P1 * P2;
  const int64_t npts = (int64_t)Bn * Ho * Wo;
  const int64_t per = (npts + nchunk - 1) / nchunk;
  const int64_t total = (int64_t)nchunk * Hd;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    int j = (int)(idx % Hd);
    int chunk = (int)(idx / Hd);
    float wj[CM], gw1[CM], gw2[COM], gb2[COM];
#pragma unroll
    for (int i = 0; i < CM; ++i) {
      wj[i] = i < C ? w1[j * C + i] : 0.f;
      gw1[i] = 0.f;
    }
    float w2j[COM];
#pragma unroll
    for (int c = 0; c < COM; ++c) {
      w2j[c] = c < Cout ? w2[c * Hd + j] : 0.f;
      gw2[c] = 0.f;
      gb2[c] = 0.f;
    }
    float gb1 = 0.f, bj = b1[j];
    int64_t beg = chunk * per, end = beg + per < npts ? beg + per : npts;
    for (int64_t q = beg; q < end; ++q) {
      int w = (int)(q % Wo);
      int64_t t = q / Wo;
      int h = (int)(t % Ho);
      int n = (int)(t / Ho);
      const float* zp = z + (int64_t)n * C * HW + (int64_t)h * P2 + w;
      float zi[CM];
      float hv = bj;
#pragma unroll
      for (int i = 0; i < CM; ++i) {
        zi[i] = i < C ? zp[i * HW] : 0.f;
        hv = fmaf(wj[i], zi[i], hv);
      }
      const float* dp = dout + ((((int64_t)(n / dout_div)) * Ho + h) * Wo + w) * ostride + ooff;
      float go[COM];
      float da = 0.f;
#pragma unroll
      for (int c = 0; c < COM; ++c) {
        go[c] = c < Cout ? dp[c] : 0.f;
        da = fmaf(w2j[c], go[c], da);
      }
      float a, g;
      gelu_both(hv, a, g);
      float dh = da * g;
#pragma unroll
      for (int i = 0; i < CM; ++i) gw1[i] = fmaf(dh, zi[i], gw1[i]);
      gb1 += dh;
#pragma unroll
      for (int c = 0; c < COM; ++c) {
        gw2[c] = fmaf(go[c], a, gw2[c]);
        gb2[c] += go[c];
      }
    }
    float* pp = partial + (int64_t)chunk * np;
#pragma unroll
    for (int i = 0; i < CM; ++i)
      if (i < C) pp[j * C + i] = gw1[i];
    pp[Hd * C + j] = gb1;
#pragma unroll
    for (int c = 0; c < COM; ++c)
      if (c < Cout) pp[Hd * C + Hd + c * Hd + j] = gw2[c];
    if (j == 0) {
#pragma unroll
      for (int c = 0; c < COM; ++c)
        if (c < Cout) pp[Hd * C + Hd + Cout * Hd + c] = gb2[c];
    }
  }
}

// ---------------------------------------------------------------- snapshot-bag mean
__global__ __launch_bounds__(kBlock) void bagmean_fwd_kernel(const float* __restrict__ u,
                                                             const float* __restrict__ grid,
                                                             const float* __restrict__ w,
                                                             const float* __restrict__ bias,
                                                             float* __restrict__ y, int B, int L,
                                                             int S, int d, int width) {
  const int64_t total = (int64_t)B * S;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    int s = (int)(idx % S);
    int b = (int)(idx / S);
    float sum = 0.f;
    for (int l = 0; l < L; ++l) sum += u[((int64_t)b * L + l) * S + s];
    for (int c = 0; c < width; ++c) {
      float v = bias[c];
      for (int e = 0; e < d; ++e) v = fmaf(w[c * (d + 1) + e], grid[(int64_t)s * d + e], v);
      float wl = w[c * (d + 1) + d] / (float)L;
      v = fmaf(wl, sum, v);
      y[idx * width + c] = v;
    }
  }
}

__global__ __launch_bounds__(kBlock) void bagmean_bwd_kernel(const float* __restrict__ dy,
                                                             const float* __restrict__ w,
                                                             float* __restrict__ s, int B, int S,
                                                             int d, int width, int L) {
  const int64_t total = (int64_t)B * S;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    float v = 0.f;
    for (int c = 0; c < width; ++c) v = fmaf(w[c * (d + 1) + d] / (float)L, dy[idx * width + c], v);
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
    float d = p[i] - t[i];
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

// Row r of a/b holds n points with `stride` floats each; a point's value is at offset
// off_a / off_b.  den_all = 1 takes the denominator over all `stride` channels of b
// (the train-loop quirk of 2d_FPE/train_fno.py:161,163).
__global__ __launch_bounds__(kBlock) void rowsq_kernel(const float* __restrict__ a,
                                                       const float* __restrict__ b,
                                                       double* __restrict__ out, int rows, int n,
                                                       int stride, int off_a, int off_b,
                                                       int den_all) {
  __shared__ double ra[kBlock], rb[kBlock];
  int r = blockIdx.x;
  if (r >= rows) return;
  double sa = 0.0, sb = 0.0;
  const float* ap = a + (int64_t)r * n * stride;
  const float* bp = b + (int64_t)r * n * stride;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const float* bq = bp + (int64_t)i * stride;
    double d = (double)ap[(int64_t)i * stride + off_a] - (double)bq[off_b];
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
    float gi = g[i] * gscale;
    float mi = fmaf(1.0f - beta1, gi - m[i], m[i]);   // exp_avg.lerp_(grad, 1-beta1)
    float vi = fmaf((1.0f - beta2) * gi, gi, v[i] * beta2);
    m[i] = mi;
    v[i] = vi;
    float denom = sqrtf(vi) / bc2s + eps;
    p[i] = p[i] - step_size * (mi / denom);
  }
}

}  // namespace

// ------------------------------------------------------------------------------ C ABI
BLINDNO_API int blindno_abi_version(void) { return 1; }

BLINDNO_API int blindno_lift_fwd(const float* in, const float* w0, const float* b0, float* x0,
                                 int Bn, int N1, int N2, int Cin, int C, int P1, int P2,
                                 void* stream) {
  if (N1 > P1 || N2 > P2) return (int)hipErrorInvalidValue;
  int64_t total = (int64_t)Bn * C * P1 * P2;
  lift_fwd_kernel<<<grid_for(total, kBlock, 65536), kBlock, 0, (hipStream_t)stream>>>(
      in, w0, b0, x0, Bn, N1, N2, Cin, C, P1, P2);
  return (int)hipGetLastError();
}

BLINDNO_API int blindno_lift_bwd(const float* dx0, const float* in, const float* w0,
                                 float* d_in, float* partial, int nchunk, int Bn, int N1,
                                 int N2, int Cin, int C, int P1, int P2, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (d_in) {
    int64_t total = (int64_t)Bn * N1 * N2 * Cin;
    lift_bwd_in_kernel<<<grid_for(total, kBlock, 65536), kBlock, 0, st>>>(dx0, w0, d_in, Bn, N1,
                                                                          N2, Cin, C, P1, P2);
  }
  if (partial) {
    int64_t total = (int64_t)nchunk * (C * Cin + C);
    lift_bwd_w_kernel<<<grid_for(total), kBlock, 0, st>>>(dx0, in, partial, nchunk, Bn, N1, N2,
                                                          Cin, C, P1, P2);
  }
  return (int)hipGetLastError();
}

BLINDNO_API int blindno_rowidft_epi(const float* Z, const float* x, const float* wc,
                                    const float* bc, float* z, const float* tw2, int Bn, int C,
                                    int P1, int P2, int m2, int act, void* stream) {
  int64_t total = (int64_t)Bn * C * P1 * P2;
  dim3 g(grid_for(total, kBlock, 65536));
  size_t sh = sizeof(float2) * P2;
  if (act)
    rowidft_epi_kernel<1><<<g, kBlock, sh, (hipStream_t)stream>>>(
        (const float2*)Z, x, wc, bc, z, (const float2*)tw2, Bn, C, P1, P2, m2);
  else
    rowidft_epi_kernel<0><<<g, kBlock, sh, (hipStream_t)stream>>>(
        (const float2*)Z, x, wc, bc, z, (const float2*)tw2, Bn, C, P1, P2, m2);
  return (int)hipGetLastError();
}

BLINDNO_API int blindno_rowidft_bwd(const float* G, const float* dz, const float* wc,
                                    const float* xpre, float* dx, const float* tw2, int Bn,
                                    int C, int P1, int P2, int m2, int act, void* stream) {
  int64_t total = (int64_t)Bn * C * P1 * P2;
  dim3 g(grid_for(total, kBlock, 65536));
  size_t sh = sizeof(float2) * P2;
  if (act)
    rowidft_bwd_kernel<1><<<g, kBlock, sh, (hipStream_t)stream>>>(
        (const float2*)G, dz, wc, xpre, dx, (const float2*)tw2, Bn, C, P1, P2, m2);
  else
    rowidft_bwd_kernel<0><<<g, kBlock, sh, (hipStream_t)stream>>>(
        (const float2*)G, dz, wc, xpre, dx, (const float2*)tw2, Bn, C, P1, P2, m2);
  return (int)hipGetLastError();
}

BLINDNO_API int blindno_conv_wgrad(const float* dz, const float* x, float* partial, int nchunk,
                                   int Bn, int C, int P1, int P2, int act, void* stream) {
  int64_t total = (int64_t)nchunk * (C * C + C);
  int64_t HW = (int64_t)P1 * P2;
  if (act)
    conv_wgrad_kernel<1><<<grid_for(total), kBlock, 0, (hipStream_t)stream>>>(dz, x, partial,
                                                                               nchunk, Bn, C, HW);
  else
    conv_wgrad_kernel<0><<<grid_for(total), kBlock, 0, (hipStream_t)stream>>>(dz, x, partial,
                                                                               nchunk, Bn, C, HW);
  return (int)hipGetLastError();
}

BLINDNO_API int blindno_reduce_partials(const float* partial, float* out, int nchunk, int np,
                                        void* stream) {
  reduce_partials_kernel<<<grid_for(np), kBlock, 0, (hipStream_t)stream>>>(partial, out, nchunk,
                                                                           np);
  return (int)hipGetLastError();
}

#define BLINDNO_PROJ_DISPATCH(KERNEL, GRID, ...)                                        \
  do {                                                                                 \
    if (Cout > 4 || C > 64) return (int)hipErrorInvalidValue;                          \
    hipStream_t st_ = (hipStream_t)stream;                                             \
    if (C <= 4) {                                                                      \
      if (Cout <= 1) KERNEL<4, 1><<<GRID, kBlock, 0, st_>>>(__VA_ARGS__);              \
      else KERNEL<4, 4><<<GRID, kBlock, 0, st_>>>(__VA_ARGS__);                        \
    } else if (C <= 8) {                                                               \
      if (Cout <= 1) KERNEL<8, 1><<<GRID, kBlock, 0, st_>>>(__VA_ARGS__);              \
      else KERNEL<8, 4><<<GRID, kBlock, 0, st_>>>(__VA_ARGS__);                        \
    } else if (C <= 16) {                                                              \
      if (Cout <= 1) KERNEL<16, 1><<<GRID, kBlock, 0, st_>>>(__VA_ARGS__);             \
      else KERNEL<16, 4><<<GRID, kBlock, 0, st_>>>(__VA_ARGS__);                       \
    } else if (C <= 32) {                                                              \
      if (Cout <= 1) KERNEL<32, 1><<<GRID, kBlock, 0, st_>>>(__VA_ARGS__);             \
      else KERNEL<32, 4><<<GRID, kBlock, 0, st_>>>(__VA_ARGS__);                       \
    } else {                                                                           \
      if (Cout <= 1) KERNEL<64, 1><<<GRID, kBlock, 0, st_>>>(__VA_ARGS__);             \
      else KERNEL<64, 4><<<GRID, kBlock, 0, st_>>>(__VA_ARGS__);                       \
    }                                                                                  \
  } while (0)

BLINDNO_API int blindno_project_fwd(const float* z, const float* w1, const float* b1,
                                    const float* w2, const float* b2, float* out, int Bn, int C,
                                    int P1, int P2, int Ho, int Wo, int Hd, int Cout,
                                    int ostride, int ooff, void* stream) {
  if (Ho > P1 || Wo > P2) return (int)hipErrorInvalidValue;
  int64_t total = (int64_t)Bn * Ho * Wo;
  dim3 g(grid_for(total, kBlock, 65536));
  BLINDNO_PROJ_DISPATCH(project_fwd_kernel, g, z, w1, b1, w2, b2, out, Bn, C, P1, P2, Ho, Wo, Hd,
                        Cout, ostride, ooff);
  return (int)hipGetLastError();
}

BLINDNO_API int blindno_project_bwd(const float* z, const float* w1, const float* b1,
                                    const float* w2, const float* dout, float* dz,
                                    float* partial, int nchunk, int Bn, int C, int P1, int P2,
                                    int Ho, int Wo, int Hd, int Cout, int ostride, int ooff,
                                    int dout_div, void* stream) {
  if (Ho > P1 || Wo > P2 || dout_div < 1) return (int)hipErrorInvalidValue;
  int64_t total = (int64_t)Bn * Ho * Wo;
  if (dz) {
    dim3 g(grid_for(total, kBlock, 65536));
    BLINDNO_PROJ_DISPATCH(project_bwd_dz_kernel, g, z, w1, b1, w2, dout, dz, Bn, C, P1, P2, Ho,
                          Wo, Hd, Cout, ostride, ooff, dout_div);
  }
  if (partial) {
    dim3 g(grid_for((int64_t)nchunk * Hd));
    BLINDNO_PROJ_DISPATCH(project_bwd_w_kernel, g, z, w1, b1, w2, dout, partial, nchunk, Bn, C,
                          P1, P2, Ho, Wo, Hd, Cout, ostride, ooff, dout_div);
  }
  return (int)hipGetLastError();
}

BLINDNO_API int blindno_bagmean_fwd(const float* u, const float* grid, const float* w,
                                    const float* bias, float* y, int B, int L, int S, int d,
                                    int width, void* stream) {
  bagmean_fwd_kernel<<<grid_for((int64_t)B * S), kBlock, 0, (hipStream_t)stream>>>(
      u, grid, w, bias, y, B, L, S, d, width);
  return (int)hipGetLastError();
}

BLINDNO_API int blindno_bagmean_bwd(const float* dy, const float* w, float* s, int B, int S,
                                    int d, int width, int L, void* stream) {
  bagmean_bwd_kernel<<<grid_for((int64_t)B * S), kBlock, 0, (hipStream_t)stream>>>(
      dy, w, s, B, S, d, width, L);
  return (int)hipGetLastError();
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

BLINDNO_API int blindno_adam(float* p, const float* g, float* m, float* v, int64_t n, float beta1,
                             float beta2, float eps, float step_size, float bc2s, float gscale,
                             void* stream) {
  adam_kernel<<<grid_for(n, kBlock, 16384), kBlock, 0, (hipStream_t)stream>>>(
      p, g, m, v, n, beta1, beta2, eps, step_size, bc2s, gscale);
  return (int)hipGetLastError();
}

BLINDNO_API const char* blindno_error_string(int code) {
  return hipGetErrorString((hipError_t)code);
}
