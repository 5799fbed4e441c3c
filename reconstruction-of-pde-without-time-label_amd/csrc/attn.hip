// Snapshot-bag token self-attention of NIOFP2D_FNO_attn (2d_FPE/NIOModules.py:365-399;
// identical in 2d_Non_conservative_FPE/NIOModules.py:364-398).
//
// Tokens of sample b: X[b] = [gx, gy, u_1 .. u_L] (T = L + 2 rows of S = nx*ny points).  The
// reference forms A = softmax(X X^T / sqrt(S)), Z = A X and fuses Z with fc0's fixed weight
// column averaged over the T tokens.  Summing Z over its tokens collapses the second GEMM:
//   sum_t Z[t,p] = sum_s c_s X[s,p],   c_s = sum_t A[t,s]   (column sums of A),
// so the forward is one Gram matrix (B x T x T, reduced over S), a T x T softmax and a
// c-weighted bag mean; nothing of size T x S is ever written besides the inputs.
//
// Backward, with dm[p] = sum_ch w[ch] dy[p,ch]:
//   dc_s   = (1/T) sum_p X[s,p] dm[p]
//   dS[t,s] = A[t,s] (dc_s - sum_s' A[t,s'] dc_s')         (softmax backward, dA[t,s] = dc_s)
//   M      = (dS + dS^T) / sqrt(S)
//   dX[s,p] = (c_s / T) dm[p] + sum_t M[s,t] X[t,p]
// Every reduction is a fixed-order sum over per-chunk partials (deterministic, no atomics).
#include "common.h"

namespace {

using namespace blindno;

constexpr int kGramPts = 32;    // points per LDS sub-tile of the Gram kernel
constexpr int kGramChunk = 512; // points per workgroup (partial sum) of the Gram kernel

__device__ __forceinline__ float token(const float* __restrict__ grid, const float* __restrict__ u,
                                       int b, int t, int p, int L, int S) {
  return t < 2 ? grid[(int64_t)p * 2 + t] : u[((int64_t)b * L + (t - 2)) * S + p];
}

// partial[b][c][T][T] = sum over the chunk c of X[t,p] X[s,p]; each thread owns one 4x4 block of
// the upper block triangle (blockIdx.y picks the round of 256 blocks) and mirrors it.
__global__ __launch_bounds__(kBlock) void gram_kernel(const float* __restrict__ grid,
                                                      const float* __restrict__ u,
                                                      float* __restrict__ partial, int L, int S,
                                                      int nch) {
  extern __shared__ float xs[];          // [T][kGramPts + 1]
  const int T = L + 2, b = blockIdx.z, c = blockIdx.x;
  const int nb = (T + 3) / 4, nblk = nb * (nb + 1) / 2;
  const int blk = blockIdx.y * kBlock + threadIdx.x;
  int bi = 0, bj = 0;
  const bool own = blk < nblk;
  if (own) {                             // blk -> (bi <= bj) in row-major upper triangle
    int r = blk;
    while (r >= nb - bi) { r -= nb - bi; ++bi; }
    bj = bi + r;
  }
  float acc[4][4] = {};
  const int p0 = c * kGramChunk, p1 = min(S, p0 + kGramChunk);
  constexpr int LD = kGramPts + 1;
  for (int q0 = p0; q0 < p1; q0 += kGramPts) {
    __syncthreads();
    for (int e = threadIdx.x; e < T * kGramPts; e += blockDim.x) {
      const int t = e / kGramPts, q = e % kGramPts;
      xs[t * LD + q] = q0 + q < p1 ? token(grid, u, b, t, q0 + q, L, S) : 0.f;
    }
    __syncthreads();
    if (own) {
#pragma unroll 4
      for (int q = 0; q < kGramPts; ++q) {
        float a[4], v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int ti = min(4 * bi + i, T - 1), tj = min(4 * bj + i, T - 1);
          a[i] = xs[ti * LD + q];
          v[i] = xs[tj * LD + q];
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(a[i], v[j], acc[i][j]);
      }
    }
  }
  if (!own) return;
  float* g = partial + ((int64_t)b * nch + c) * T * T;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int t = 4 * bi + i, s = 4 * bj + j;
      if (t < T && s < T) {
        g[t * T + s] = acc[i][j];
        g[s * T + t] = acc[i][j];
      }
    }
}

// One workgroup per sample: G = sum of the chunk partials, A = row softmax(G / sqrt(S)),
// c = column sums of A.  A (B,T,T) and c (B,T) are kept for the backward.
__global__ __launch_bounds__(kBlock) void softmax_kernel(const float* __restrict__ partial,
                                                         float* __restrict__ A,
                                                         float* __restrict__ cs, int T, int S,
                                                         int nch) {
  const int b = blockIdx.x;
  const float scale = rsqrtf((float)S);
  const float* pb = partial + (int64_t)b * nch * T * T;
  float* Ab = A + (int64_t)b * T * T;
  for (int t = threadIdx.x; t < T; t += blockDim.x) {
    float mx = -INFINITY;
    for (int s = 0; s < T; ++s) {
      float g = 0.f;
      for (int c = 0; c < nch; ++c) g += pb[((int64_t)c * T + t) * T + s];
      g *= scale;
      Ab[t * T + s] = g;
      mx = fmaxf(mx, g);
    }
    float den = 0.f;
    for (int s = 0; s < T; ++s) {
      const float e = __expf(Ab[t * T + s] - mx);
      Ab[t * T + s] = e;
      den += e;
    }
    const float inv = 1.0f / den;
    for (int s = 0; s < T; ++s) Ab[t * T + s] *= inv;
  }
  __syncthreads();
  for (int s = threadIdx.x; s < T; s += blockDim.x) {
    float v = 0.f;
    for (int t = 0; t < T; ++t) v += Ab[t * T + s];
    cs[(int64_t)b * T + s] = v;
  }
}

// y[b,p,ch] = w[ch] (1/T) sum_s c_s X[s,p] + bias[ch]
__global__ __launch_bounds__(kBlock) void fuse_fwd_kernel(const float* __restrict__ grid,
                                                          const float* __restrict__ u,
                                                          const float* __restrict__ cs,
                                                          const float* __restrict__ w,
                                                          const float* __restrict__ bias,
                                                          float* __restrict__ y, int B, int L,
                                                          int S, int width) {
  const int T = L + 2;
  const float invT = 1.0f / (float)T;
  const int64_t total = (int64_t)B * S;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int p = (int)(idx % S), b = (int)(idx / S);
    const float* cb = cs + (int64_t)b * T;
    float m = cb[0] * grid[(int64_t)p * 2] + cb[1] * grid[(int64_t)p * 2 + 1];
    for (int l = 0; l < L; ++l) m = fmaf(cb[l + 2], u[((int64_t)b * L + l) * S + p], m);
    m *= invT;
    for (int ch = 0; ch < width; ++ch) y[idx * width + ch] = fmaf(w[ch], m, bias[ch]);
  }
}

// dm[b,p] = sum_ch w[ch] dy[b,p,ch]; partial[b][c][t] = sum_{p in chunk c} X[t,p] dm[p]
// (one wave per token row, lanes over the chunk's points: coalesced).
__global__ __launch_bounds__(kBlock) void dc_kernel(const float* __restrict__ grid,
                                                    const float* __restrict__ u,
                                                    const float* __restrict__ dy,
                                                    const float* __restrict__ w,
                                                    float* __restrict__ dm,
                                                    float* __restrict__ partial, int L, int S,
                                                    int width, int nch) {
  __shared__ float dml[kGramChunk];
  const int T = L + 2, b = blockIdx.y, c = blockIdx.x;
  const int p0 = c * kGramChunk, n = min(S - p0, kGramChunk);
  for (int q = threadIdx.x; q < n; q += blockDim.x) {
    const int64_t o = (int64_t)b * S + p0 + q;
    float v = 0.f;
    for (int ch = 0; ch < width; ++ch) v = fmaf(w[ch], dy[o * width + ch], v);
    dml[q] = v;
    dm[o] = v;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (int t = wave; t < T; t += nw) {
    float v = 0.f;
    for (int q = lane; q < n; q += 64) v = fmaf(token(grid, u, b, t, p0 + q, L, S), dml[q], v);
    v = wave_sum(v);
    if (lane == 0) partial[((int64_t)b * nch + c) * T + t] = v;
  }
}

// One workgroup per sample: dc = (1/T) sum of the chunk partials; M = (dS + dS^T)/sqrt(S).
__global__ __launch_bounds__(kBlock) void mix_bwd_kernel(const float* __restrict__ partial,
                                                         const float* __restrict__ A,
                                                         float* __restrict__ M, int T, int S,
                                                         int nch) {
  extern __shared__ float sm[];          // dc[T], r[T]
  float* dc = sm;
  float* r = sm + T;
  const int b = blockIdx.x;
  const float invT = 1.0f / (float)T, scale = rsqrtf((float)S);
  const float* Ab = A + (int64_t)b * T * T;
  for (int s = threadIdx.x; s < T; s += blockDim.x) {
    float v = 0.f;
    for (int c = 0; c < nch; ++c) v += partial[((int64_t)b * nch + c) * T + s];
    dc[s] = v * invT;
  }
  __syncthreads();
  for (int t = threadIdx.x; t < T; t += blockDim.x) {
    float v = 0.f;
    for (int s = 0; s < T; ++s) v = fmaf(Ab[t * T + s], dc[s], v);
    r[t] = v;
  }
  __syncthreads();
  float* Mb = M + (int64_t)b * T * T;
  for (int e = threadIdx.x; e < T * T; e += blockDim.x) {
    const int t = e / T, s = e % T;
    const float d1 = Ab[t * T + s] * (dc[s] - r[t]);
    const float d2 = Ab[s * T + t] * (dc[t] - r[s]);
    Mb[e] = (d1 + d2) * scale;
  }
}

// dX[s,p] = (c_s/T) dm[p] + sum_t M[s,t] X[t,p]: the workgroup stages X[:, 64 points] in LDS,
// lane = point, each wave produces 8 token rows per pass.  Rows 0,1 (grid tokens) go to dgt
// (B,2,S) when it is non-null, rows s >= 2 to du (B,L,S).
constexpr int kDxRows = 8;
__global__ __launch_bounds__(kBlock) void dx_kernel(const float* __restrict__ grid,
                                                    const float* __restrict__ u,
                                                    const float* __restrict__ dm,
                                                    const float* __restrict__ cs,
                                                    const float* __restrict__ M,
                                                    float* __restrict__ du,
                                                    float* __restrict__ dgt, int L, int S) {
  extern __shared__ float xs[];          // [T][64]
  const int T = L + 2, b = blockIdx.y;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int p0 = blockIdx.x * 64, p = p0 + lane;
  const bool ok = p < S;
  for (int e = threadIdx.x; e < T * 64; e += blockDim.x) {
    const int t = e >> 6, q = e & 63;
    xs[e] = p0 + q < S ? token(grid, u, b, t, p0 + q, L, S) : 0.f;
  }
  __syncthreads();
  const float invT = 1.0f / (float)T;
  const float dmp = ok ? dm[(int64_t)b * S + p] : 0.f;
  const float* Mb = M + (int64_t)b * T * T;
  const float* cb = cs + (int64_t)b * T;
  const int s_first = dgt ? 0 : 2;
  for (int s0 = s_first + wave * kDxRows; s0 < T; s0 += nw * kDxRows) {
    float acc[kDxRows];
    const float* mr[kDxRows];
#pragma unroll
    for (int i = 0; i < kDxRows; ++i) {
      const int s = min(s0 + i, T - 1);
      mr[i] = Mb + (int64_t)s * T;
      acc[i] = cb[s] * invT * dmp;
    }
    for (int t = 0; t < T; ++t) {
      const float x = xs[t * 64 + lane];
#pragma unroll
      for (int i = 0; i < kDxRows; ++i) acc[i] = fmaf(mr[i][t], x, acc[i]);
    }
    if (ok) {
#pragma unroll
      for (int i = 0; i < kDxRows; ++i) {
        const int s = s0 + i;
        if (s >= T) break;
        if (s < 2) dgt[((int64_t)b * 2 + s) * S + p] = acc[i];
        else du[((int64_t)b * L + (s - 2)) * S + p] = acc[i];
      }
    }
  }
}

}  // namespace

BLINDNO_API int blindno_bagattn_nchunk(int S) { return (S + kGramChunk - 1) / kGramChunk; }

BLINDNO_API int blindno_bagattn_fwd(const float* grid, const float* u, const float* w,
                                    const float* bias, float* partial, float* A, float* cs,
                                    float* y, int B, int L, int S, int width, void* stream) {
  const int T = L + 2;
  if (B <= 0 || L <= 0 || S <= 0 || width <= 0 || T > 256) return (int)hipErrorInvalidValue;
  const int nch = blindno_bagattn_nchunk(S);
  const int nb = (T + 3) / 4, rounds = (nb * (nb + 1) / 2 + kBlock - 1) / kBlock;
  hipStream_t st = (hipStream_t)stream;
  gram_kernel<<<dim3(nch, rounds, B), kBlock, T * (kGramPts + 1) * sizeof(float), st>>>(
      grid, u, partial, L, S, nch);
  softmax_kernel<<<B, kBlock, 0, st>>>(partial, A, cs, T, S, nch);
  fuse_fwd_kernel<<<grid_for((int64_t)B * S), kBlock, 0, st>>>(grid, u, cs, w, bias, y, B, L, S,
                                                               width);
  return (int)hipGetLastError();
}

BLINDNO_API int blindno_bagattn_bwd(const float* grid, const float* u, const float* dy,
                                    const float* w, const float* A, const float* cs,
                                    float* partial, float* dm, float* M, float* du, float* dgt,
                                    int B, int L, int S, int width, void* stream) {
  const int T = L + 2;
  if (B <= 0 || L <= 0 || S <= 0 || width <= 0 || T > 256) return (int)hipErrorInvalidValue;
  const int nch = blindno_bagattn_nchunk(S);
  hipStream_t st = (hipStream_t)stream;
  dc_kernel<<<dim3(nch, B), kBlock, 0, st>>>(grid, u, dy, w, dm, partial, L, S, width, nch);
  mix_bwd_kernel<<<B, kBlock, 2 * T * sizeof(float), st>>>(partial, A, M, T, S, nch);
  dx_kernel<<<dim3((S + 63) / 64, B), kBlock, T * 64 * sizeof(float), st>>>(grid, u, dm, cs, M,
                                                                          du, dgt, L, S);
  return (int)hipGetLastError();
}
