// Truncated spectral transforms and per-mode channel mixing for SpectralConv1d/2d.
//
// Reference operation (yl602019618/Reconstruction-of-PDE-without-Time-Label):
//   SpectralConv2d.forward  2d_FPE/FNOModules.py:156-178  (rfft2 -> compl_mul2d on the
//   two kept corner blocks -> irfft2(s=(H,W)));  SpectralConv1d.forward
//   1d_FPE/FNOModules.py:47-59 (rfft -> DC*0.5 -> einsum -> irfft).
// The FFTs are evaluated as truncated DFTs: only m2 column modes and K1 kept rows are
// ever formed, so the full spectrum is never materialised.  Twiddles come from a
// per-length table tw[j] = (cos 2pi j/P, sin 2pi j/P) built on the host in double.
#include "common.h"

using namespace blindno;

namespace {

// ---------------------------------------------------------------- row DFT
// At[n][k][c][h] = sum_w f(x[n][c][h][w]) e^{-2 pi i k w / P2}
// One thread per output coefficient; the x row is swept from L1/L2.  The twiddle
// table is staged in LDS.
template <int ACT>
__global__ __launch_bounds__(kBlock) void rowdft_kernel(const float* __restrict__ x,
                                                        float2* __restrict__ At,
                                                        const float2* __restrict__ tw2, int Bn,
                                                        int C, int P1, int P2, int m2) {
  extern __shared__ float2 s_tw[];
  for (int i = threadIdx.x; i < P2; i += blockDim.x) s_tw[i] = tw2[i];
  __syncthreads();
  const int64_t total = (int64_t)Bn * m2 * C * P1;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    int h = (int)(idx % P1);
    int64_t t = idx / P1;
    int c = (int)(t % C);
    t /= C;
    int k = (int)(t % m2);
    int n = (int)(t / m2);
    const float* row = x + (((int64_t)n * C + c) * P1 + h) * P2;
    float re = 0.f, im = 0.f;
    int ph = 0;
    for (int w = 0; w < P2; ++w) {
      float v = row[w];
      if (ACT) v = gelu_f(v);
      float2 e = s_tw[ph];
      re = fmaf(v, e.x, re);
      im = fmaf(-v, e.y, im);
      ph += k;
      if (ph >= P2) ph -= P2;
    }
    At[idx] = make_float2(re, im);
  }
}

// ---------------------------------------------------------------- column DFT at kept rows
// X[n][k][c][j] = s_k * sum_h At[n][k][c][h] e^{-2 pi i r_j h / P1}
__global__ __launch_bounds__(kBlock) void coldft_kernel(const float2* __restrict__ At,
                                                        float2* __restrict__ X,
                                                        const float2* __restrict__ tw1, int Bn,
                                                        int C, int P1, int m1, int m2, int P2,
                                                        int scale_mode) {
  extern __shared__ float2 s_tw[];
  for (int i = threadIdx.x; i < P1; i += blockDim.x) s_tw[i] = tw1[i];
  __syncthreads();
  const int K1 = kept_rows_count(m1, P1);
  const int64_t total = (int64_t)Bn * m2 * C * K1;
  const float inv = 1.0f / ((float)P1 * (float)P2);
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    int j = (int)(idx % K1);
    int64_t t = idx / K1;  // (n, k, c)
    int k = (int)((t / C) % m2);
    const float2* col = At + t * P1;
    int r = kept_row(j, K1, m1, P1);
    float re = 0.f, im = 0.f;
    int ph = 0;
    for (int h = 0; h < P1; ++h) {
      float2 a = col[h];
      float2 e = s_tw[ph];
      // (a.x + i a.y)(e.x - i e.y)
      re = fmaf(a.x, e.x, fmaf(a.y, e.y, re));
      im = fmaf(a.y, e.x, fmaf(-a.x, e.y, im));
      ph += r;
      if (ph >= P1) ph -= P1;
    }
    if (scale_mode == 1) {
      float s = c2r_weight(k, P2) * inv;
      re *= s;
      im *= s;
    }
    X[idx] = make_float2(re, im);
  }
}

// ---------------------------------------------------------------- column inverse at kept rows
// Z[n][c][h][k] = s_k * sum_j Y[n][k][c][j] e^{+2 pi i r_j h / P1}
__global__ __launch_bounds__(kBlock) void colidft_kernel(const float2* __restrict__ Y,
                                                         float2* __restrict__ Z,
                                                         const float2* __restrict__ tw1, int Bn,
                                                         int C, int P1, int m1, int m2, int P2,
                                                         int scale_mode) {
  extern __shared__ float2 s_tw[];
  for (int i = threadIdx.x; i < P1; i += blockDim.x) s_tw[i] = tw1[i];
  __syncthreads();
  const int K1 = kept_rows_count(m1, P1);
  const int64_t total = (int64_t)Bn * C * P1 * m2;
  const float inv = 1.0f / ((float)P1 * (float)P2);
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    int k = (int)(idx % m2);
    int64_t t = idx / m2;
    int h = (int)(t % P1);
    t /= P1;
    int c = (int)(t % C);
    int n = (int)(t / C);
    const float2* yv = Y + (((int64_t)n * m2 + k) * C + c) * K1;
    float re = 0.f, im = 0.f;
    for (int j = 0; j < K1; ++j) {
      int r = kept_row(j, K1, m1, P1);
      int ph = (int)(((int64_t)r * h) % P1);
      float2 e = s_tw[ph];
      float2 a = yv[j];
      // (a.x + i a.y)(e.x + i e.y)
      re = fmaf(a.x, e.x, fmaf(-a.y, e.y, re));
      im = fmaf(a.x, e.y, fmaf(a.y, e.x, im));
    }
    float s = scale_mode == 1 ? c2r_weight(k, P2) * inv : 1.0f;
    Z[idx] = make_float2(re * s, im * s);
  }
}

// ---------------------------------------------------------------- per-mode channel mix
template <int DIR>
__global__ __launch_bounds__(kBlock) void mix_kernel(const float2* __restrict__ X,
                                                     const float2* __restrict__ Wt,
                                                     float2* __restrict__ Y, int Bn, int Ci,
                                                     int Co, int K1, int m2) {
  // DIR 0: Y[n,k,o,j] = sum_i X[n,k,i,j] W[k,j,i,o]
  // DIR 1: Y[n,k,i,j] = sum_o conj(W[k,j,i,o]) X[n,k,o,j]
  const int Cout = DIR == 0 ? Co : Ci;
  const int Cin = DIR == 0 ? Ci : Co;
  const int64_t total = (int64_t)Bn * m2 * Cout * K1;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    int j = (int)(idx % K1);
    int64_t t = idx / K1;
    int oc = (int)(t % Cout);
    int64_t nk = t / Cout;  // n * m2 + k
    int k = (int)(nk % m2);
    const float2* xv = X + nk * Cin * K1 + j;
    const float2* wv = Wt + ((int64_t)k * K1 + j) * Ci * Co;
    float re = 0.f, im = 0.f;
    for (int q = 0; q < Cin; ++q) {
      float2 a = xv[(int64_t)q * K1];
      if (DIR == 0) {
        float2 w = wv[(int64_t)q * Co + oc];
        re = fmaf(a.x, w.x, fmaf(-a.y, w.y, re));
        im = fmaf(a.x, w.y, fmaf(a.y, w.x, im));
      } else {
        float2 w = wv[(int64_t)oc * Co + q];
        // conj(w) * a
        re = fmaf(w.x, a.x, fmaf(w.y, a.y, re));
        im = fmaf(w.x, a.y, fmaf(-w.y, a.x, im));
      }
    }
    Y[idx] = make_float2(re, im);
  }
}

__global__ __launch_bounds__(kBlock) void mix_wgrad_kernel(const float2* __restrict__ X,
                                                           const float2* __restrict__ G,
                                                           float2* __restrict__ dWt, int Bn,
                                                           int Ci, int Co, int K1, int m2) {
  const int64_t total = (int64_t)m2 * K1 * Ci * Co;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    int o = (int)(idx % Co);
    int64_t t = idx / Co;
    int i = (int)(t % Ci);
    t /= Ci;
    int j = (int)(t % K1);
    int k = (int)(t / K1);
    float re = 0.f, im = 0.f;
    for (int n = 0; n < Bn; ++n) {
      float2 a = X[(((int64_t)n * m2 + k) * Ci + i) * K1 + j];
      float2 g = G[(((int64_t)n * m2 + k) * Co + o) * K1 + j];
      // conj(a) * g
      re = fmaf(a.x, g.x, fmaf(a.y, g.y, re));
      im = fmaf(a.x, g.y, fmaf(-a.y, g.x, im));
    }
    dWt[idx] = make_float2(re, im);
  }
}

// ---------------------------------------------------------------- 1D mode mix
template <int DIR>
__global__ __launch_bounds__(kBlock) void mix1d_kernel(const float2* __restrict__ At,
                                                       const float2* __restrict__ Wt,
                                                       float2* __restrict__ Xs,
                                                       float2* __restrict__ Z, int Bn, int Ci,
                                                       int Co, int m, int P2) {
  // At[n][k][c] (P1 = 1).  Forward: Xs = At * h_k ; Z[n][o][k] = c_k/P2 sum_i Xs W
  // Backward: Xs = c_k/P2 At ; Z[n][i][k] = h_k sum_o conj(W) Xs
  const int Cout = DIR == 0 ? Co : Ci;
  const int Cin = DIR == 0 ? Ci : Co;
  const int64_t total = (int64_t)Bn * Cout * m;
  const float invP = 1.0f / (float)P2;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    int k = (int)(idx % m);
    int64_t t = idx / m;
    int oc = (int)(t % Cout);
    int n = (int)(t / Cout);
    const float hk = k == 0 ? 0.5f : 1.0f;
    const float ck = c2r_weight(k, P2) * invP;
    const float2* av = At + ((int64_t)n * m + k) * Cin;
    const float2* wv = Wt + (int64_t)k * Ci * Co;
    float re = 0.f, im = 0.f;
    for (int q = 0; q < Cin; ++q) {
      float2 a = av[q];
      if (DIR == 0) {
        a.x *= hk;
        a.y *= hk;
        float2 w = wv[(int64_t)q * Co + oc];
        re = fmaf(a.x, w.x, fmaf(-a.y, w.y, re));
        im = fmaf(a.x, w.y, fmaf(a.y, w.x, im));
      } else {
        a.x *= ck;
        a.y *= ck;
        float2 w = wv[(int64_t)oc * Co + q];
        re = fmaf(w.x, a.x, fmaf(w.y, a.y, re));
        im = fmaf(w.x, a.y, fmaf(-w.y, a.x, im));
      }
    }
    float s = DIR == 0 ? ck : hk;
    Z[((int64_t)n * Cout + oc) * m + k] = make_float2(re * s, im * s);
  }
  // saved spectrum, layout Xs[n][k][c] (= colspec with K1 = 1)
  const int64_t tot2 = (int64_t)Bn * m * Cin;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < tot2;
       idx += (int64_t)gridDim.x * blockDim.x) {
    int k = (int)((idx / Cin) % m);
    float2 a = At[idx];
    float s = DIR == 0 ? (k == 0 ? 0.5f : 1.0f) : c2r_weight(k, P2) * invP;
    Xs[idx] = make_float2(a.x * s, a.y * s);
  }
}

// ---------------------------------------------------------------- weight packing
__global__ void pack_w2d_kernel(const float* __restrict__ w1, const float* __restrict__ w2,
                                float2* __restrict__ Wt, int Ci, int Co, int m1, int m2,
                                int P1) {
  const int K1 = kept_rows_count(m1, P1);
  const int64_t total = (int64_t)m2 * K1 * Ci * Co;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    int o = (int)(idx % Co);
    int64_t t = idx / Co;
    int i = (int)(t % Ci);
    t /= Ci;
    int j = (int)(t % K1);
    int k = (int)(t / K1);
    int r = kept_row(j, K1, m1, P1);
    const float* src;
    int jj;
    if (r >= P1 - m1) {
      src = w2;
      jj = r - (P1 - m1);
    } else {
      src = w1;
      jj = r;
    }
    const float* p = src + ((((int64_t)i * Co + o) * m1 + jj) * m2 + k) * 2;
    Wt[idx] = make_float2(p[0], p[1]);
  }
}

__global__ void unpack_w2d_kernel(const float2* __restrict__ dWt, float* __restrict__ dw1,
                                  float* __restrict__ dw2, int Ci, int Co, int m1, int m2,
                                  int P1) {
  const int K1 = kept_rows_count(m1, P1);
  const int64_t per = (int64_t)Ci * Co * m1 * m2;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < 2 * per;
       idx += (int64_t)gridDim.x * blockDim.x) {
    int which = idx >= per;
    int64_t e = which ? idx - per : idx;
    int k = (int)(e % m2);
    int64_t t = e / m2;
    int jj = (int)(t % m1);
    t /= m1;
    int o = (int)(t % Co);
    int i = (int)(t / Co);
    float2 v = make_float2(0.f, 0.f);
    int r, j = -1;
    if (which) {
      r = P1 - m1 + jj;
      j = (K1 == P1) ? r : m1 + jj;
    } else {
      r = jj;
      if (r < P1 - m1) j = r;  // otherwise shadowed by weights2
    }
    if (j >= 0) v = dWt[(((int64_t)k * K1 + j) * Ci + i) * Co + o];
    float* dst = (which ? dw2 : dw1) + e * 2;
    dst[0] = v.x;
    dst[1] = v.y;
  }
}

__global__ void pack_w1d_kernel(const float2* __restrict__ w, float2* __restrict__ Wt, int Ci,
                                int Co, int m, int dir) {
  const int64_t total = (int64_t)Ci * Co * m;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    int k = (int)(idx % m);
    int64_t t = idx / m;
    int o = (int)(t % Co);
    int i = (int)(t / Co);
    int64_t pidx = ((int64_t)k * Ci + i) * Co + o;
    if (dir == 0)
      Wt[pidx] = w[idx];
    else
      ((float2*)Wt)[idx] = w[pidx];  // unpack: w is dWt, Wt is dW
  }
}

}  // namespace

BLINDNO_API int blindno_rowdft(const float* x, float* At, const float* tw2, int Bn, int C,
                               int P1, int P2, int m2, int act, void* stream) {
  if (Bn <= 0 || C <= 0 || P1 <= 0 || P2 <= 0 || m2 <= 0 || m2 > P2 / 2 + 1 || P2 > 8192)
    return (int)hipErrorInvalidValue;
  int64_t total = (int64_t)Bn * m2 * C * P1;
  dim3 g(grid_for(total, kBlock, 65536)), b(kBlock);
  size_t sh = sizeof(float2) * P2;
  if (act)
    rowdft_kernel<1><<<g, b, sh, (hipStream_t)stream>>>(x, (float2*)At, (const float2*)tw2,
                                                         Bn, C, P1, P2, m2);
  else
    rowdft_kernel<0><<<g, b, sh, (hipStream_t)stream>>>(x, (float2*)At, (const float2*)tw2,
                                                         Bn, C, P1, P2, m2);
  return (int)hipGetLastError();
}

BLINDNO_API int blindno_coldft(const float* At, float* X, const float* tw1, int Bn, int C,
                               int P1, int m1, int m2, int P2, int scale_mode, void* stream) {
  if (m1 <= 0 || m1 > P1 || P1 > 8192) return (int)hipErrorInvalidValue;
  int64_t total = (int64_t)Bn * m2 * C * kept_rows_count(m1, P1);
  coldft_kernel<<<grid_for(total, kBlock, 65536), kBlock, sizeof(float2) * P1,
                  (hipStream_t)stream>>>((const float2*)At, (float2*)X, (const float2*)tw1, Bn,
                                         C, P1, m1, m2, P2, scale_mode);
  return (int)hipGetLastError();
}

BLINDNO_API int blindno_colidft(const float* Y, float* Z, const float* tw1, int Bn, int C,
                                int P1, int m1, int m2, int P2, int scale_mode, void* stream) {
  if (m1 <= 0 || m1 > P1 || P1 > 8192) return (int)hipErrorInvalidValue;
  int64_t total = (int64_t)Bn * C * P1 * m2;
  colidft_kernel<<<grid_for(total, kBlock, 65536), kBlock, sizeof(float2) * P1,
                   (hipStream_t)stream>>>((const float2*)Y, (float2*)Z, (const float2*)tw1, Bn,
                                          C, P1, m1, m2, P2, scale_mode);
  return (int)hipGetLastError();
}

BLINDNO_API int blindno_mix(const float* X, const float* Wt, float* Y, int Bn, int Ci, int Co,
                            int K1, int m2, int dir, void* stream) {
  int64_t total = (int64_t)Bn * m2 * (dir == 0 ? Co : Ci) * K1;
  dim3 g(grid_for(total, kBlock, 65536));
  if (dir == 0)
    mix_kernel<0><<<g, kBlock, 0, (hipStream_t)stream>>>((const float2*)X, (const float2*)Wt,
                                                         (float2*)Y, Bn, Ci, Co, K1, m2);
  else
    mix_kernel<1><<<g, kBlock, 0, (hipStream_t)stream>>>((const float2*)X, (const float2*)Wt,
                                                         (float2*)Y, Bn, Ci, Co, K1, m2);
  return (int)hipGetLastError();
}

BLINDNO_API int blindno_mix_wgrad(const float* X, const float* G, float* dWt, int Bn, int Ci,
                                  int Co, int K1, int m2, void* stream) {
  int64_t total = (int64_t)m2 * K1 * Ci * Co;
  mix_wgrad_kernel<<<grid_for(total, kBlock, 65536), kBlock, 0, (hipStream_t)stream>>>(
      (const float2*)X, (const float2*)G, (float2*)dWt, Bn, Ci, Co, K1, m2);
  return (int)hipGetLastError();
}

BLINDNO_API int blindno_mix1d(const float* At, const float* Wt, float* Xs, float* Z, int Bn,
                              int Ci, int Co, int m, int P2, int dir, void* stream) {
  if (m > P2 / 2 + 1) return (int)hipErrorInvalidValue;
  int64_t total = (int64_t)Bn * (dir == 0 ? Co : Ci) * m;
  int64_t t2 = (int64_t)Bn * m * (dir == 0 ? Ci : Co);
  dim3 g(grid_for(total > t2 ? total : t2, kBlock, 65536));
  if (dir == 0)
    mix1d_kernel<0><<<g, kBlock, 0, (hipStream_t)stream>>>(
        (const float2*)At, (const float2*)Wt, (float2*)Xs, (float2*)Z, Bn, Ci, Co, m, P2);
  else
    mix1d_kernel<1><<<g, kBlock, 0, (hipStream_t)stream>>>(
        (const float2*)At, (const float2*)Wt, (float2*)Xs, (float2*)Z, Bn, Ci, Co, m, P2);
  return (int)hipGetLastError();
}

BLINDNO_API int blindno_pack_w2d(const float* w1, const float* w2, float* Wt, int Ci, int Co,
                                 int m1, int m2, int P1, void* stream) {
  if (m1 > P1) return (int)hipErrorInvalidValue;
  int64_t total = (int64_t)m2 * kept_rows_count(m1, P1) * Ci * Co;
  pack_w2d_kernel<<<grid_for(total), kBlock, 0, (hipStream_t)stream>>>(w1, w2, (float2*)Wt, Ci,
                                                                       Co, m1, m2, P1);
  return (int)hipGetLastError();
}

BLINDNO_API int blindno_unpack_w2d(const float* dWt, float* dw1, float* dw2, int Ci, int Co,
                                   int m1, int m2, int P1, void* stream) {
  if (m1 > P1) return (int)hipErrorInvalidValue;
  int64_t total = 2 * (int64_t)Ci * Co * m1 * m2;
  unpack_w2d_kernel<<<grid_for(total), kBlock, 0, (hipStream_t)stream>>>(
      (const float2*)dWt, dw1, dw2, Ci, Co, m1, m2, P1);
  return (int)hipGetLastError();
}

BLINDNO_API int blindno_pack_w1d(const float* w, float* Wt, int Ci, int Co, int m, int dir,
                                 void* stream) {
  int64_t total = (int64_t)Ci * Co * m;
  pack_w1d_kernel<<<grid_for(total), kBlock, 0, (hipStream_t)stream>>>(
      (const float2*)w, (float2*)Wt, Ci, Co, m, dir);
  return (int)hipGetLastError();
}
