// BatchNorm2d (batch statistics) fused with LeakyReLU: the ConvBlock of the NIO snapshot
// encoders, Conv -> BatchNorm2d -> LeakyReLU(0.2) (2d_FPE/Baselines.py:40-52, used by Encoder2D
// :186-249 and the 1D Encoder :254-287).
//
// Layout: z is NCHW with Npad >= N rows; only rows [0, N) are the batch (the encoders pad the
// snapshot batch to a whole number of fixed-size convolution chunks so MIOpen sees one problem
// per layer).  Output rows [N, Npad) are written as 0 (so the padded rows stay finite through the
// next convolution and contribute exactly 0 to its weight gradient).
//
// Train mode follows torch.nn.BatchNorm2d: normalise with the batch mean and the biased
// variance; running_mean/var <- (1 - momentum) running + momentum (mean, unbiased var).
// Eval mode normalises with the running statistics.  Per-channel statistics are two-level
// reductions in a fixed order (deterministic): S slices per channel write partial sums,
// one finalize thread per channel combines them.  The sums are shifted by the channel's first
// element (z[0, c, 0]) so sum/sum-of-squares keep their precision when |mean| >> std, and are
// accumulated in fp64 (as torch's CPU BatchNorm does): the backward's mean of the upstream
// gradient must be exact to fp32 rounding when that gradient is nearly constant over the batch
// -- the NIO trunk's BatchNorm1d over 16384 grid points fed a rank-B gradient, where fp32 sums
// left 7e-4 of gradient error upstream of the layer (tools/diag_trunk_graph.py; torch's GPU
// BatchNorm, fp32 sums, measured the same 7e-4, its CPU one 4e-6).
//
// HBM traffic per element: forward 2 reads + 1 write (stats pass, apply pass), backward
// 4 reads + 1 write (dy and z twice; nothing but z and the per-channel coefficients is saved).
#include "common.h"
#include "blindno.h"

using namespace blindno;

namespace {

constexpr int kBnThreads = 256;

// per-channel coefficient record (save buffer, [C][kSave]):
//   0 mean, 1 invstd, 2 a = gamma invstd, 3 beta   (forward, y = act(a (z - mean) + beta))
// The affine is applied to the CENTRED value: folding it into a z + (beta - mean a) loses
// eps |mean| / std of the pre-activation to cancellation, which for the deep 1x1 / 2x1 blocks
// of the encoders (|mean| >> std over the batch) flips LeakyReLU branches and costs ~1e-3 of
// gradient accuracy (tools/diag_encoder_bwd.py).
constexpr int kSave = 4;

__device__ __forceinline__ float leaky(float v, float slope) { return v > 0.f ? v : v * slope; }

__device__ __forceinline__ double block_sum(double v, double* red) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wave] = v;
  __syncthreads();
  double s = 0.0;
#pragma unroll
  for (int w = 0; w < kBnThreads / 64; ++w) s += red[w];
  return s;
}

// partial[(c S + s) 2 + {0, 1}] = sums of (z - shift) and (z - shift)^2 over slice s of channel c
template <bool VEC>
__global__ __launch_bounds__(kBnThreads) void bn_stats_kernel(const float* __restrict__ z,
                                                              double* __restrict__ partial, int N,
                                                              int C, int HW) {
  __shared__ double red[kBnThreads / 64];
  const int c = blockIdx.y, S = gridDim.x, s = blockIdx.x;
  const float shift = z[(int64_t)c * HW];
  double s1 = 0.0, s2 = 0.0;
  if (VEC) {
    const int HW4 = HW >> 2;
    const int64_t M4 = (int64_t)N * HW4;
    for (int64_t e = (int64_t)s * kBnThreads + threadIdx.x; e < M4; e += (int64_t)S * kBnThreads) {
      const int64_t n = e / HW4;
      const int q4 = (int)(e - n * HW4);
      const float4 v = *reinterpret_cast<const float4*>(z + (n * C + c) * HW + 4 * q4);
      const double a = v.x - shift, b = v.y - shift, d = v.z - shift, f = v.w - shift;
      s1 += (a + b) + (d + f);
      s2 = fma(a, a, s2); s2 = fma(b, b, s2); s2 = fma(d, d, s2); s2 = fma(f, f, s2);
    }
  } else {
    const int64_t M = (int64_t)N * HW;
    for (int64_t e = (int64_t)s * kBnThreads + threadIdx.x; e < M; e += (int64_t)S * kBnThreads) {
      const int64_t n = e / HW;
      const int q = (int)(e - n * HW);
      const double a = z[(n * C + c) * HW + q] - shift;
      s1 += a;
      s2 = fma(a, a, s2);
    }
  }
  s1 = block_sum(s1, red);
  s2 = block_sum(s2, red);
  if (threadIdx.x == 0) {
    partial[((int64_t)c * S + s) * 2 + 0] = s1;
    partial[((int64_t)c * S + s) * 2 + 1] = s2;
  }
}

__global__ void bn_finalize_kernel(const float* __restrict__ z, const double* __restrict__ partial,
                                   const float* __restrict__ gamma, const float* __restrict__ beta,
                                   float* __restrict__ run_mean, float* __restrict__ run_var,
                                   float* __restrict__ save, int S, int N, int C, int HW, float eps,
                                   float momentum, int training) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float mean, invstd;
  if (training) {
    const double M = (double)N * HW;
    double s1 = 0.0, s2 = 0.0;
    for (int s = 0; s < S; ++s) {
      s1 += partial[((int64_t)c * S + s) * 2 + 0];
      s2 += partial[((int64_t)c * S + s) * 2 + 1];
    }
    const float shift = z[(int64_t)c * HW];
    const double m1 = s1 / M;                                    // mean of (z - shift)
    const float var = (float)fmax(s2 / M - m1 * m1, 0.0);       // biased
    mean = (float)(shift + m1);
    invstd = 1.0f / sqrtf(var + eps);
    if (run_mean) {
      const float unbiased = M > 1.0 ? (float)(var * (M / (M - 1.0))) : var;
      run_mean[c] = (1.0f - momentum) * run_mean[c] + momentum * mean;
      run_var[c] = (1.0f - momentum) * run_var[c] + momentum * unbiased;
    }
  } else {
    mean = run_mean[c];
    invstd = 1.0f / sqrtf(run_var[c] + eps);
  }
  const float g = gamma ? gamma[c] : 1.0f, b = beta ? beta[c] : 0.0f;
  const float a = g * invstd;
  save[c * kSave + 0] = mean;
  save[c * kSave + 1] = invstd;
  save[c * kSave + 2] = a;
  save[c * kSave + 3] = b;
}

template <bool VEC>
__global__ __launch_bounds__(kBnThreads) void bn_apply_kernel(const float* __restrict__ z,
                                                              const float* __restrict__ save,
                                                              float* __restrict__ y, int N,
                                                              int Npad, int C, int HW,
                                                              float slope) {
  const int64_t rowlen = (int64_t)C * HW;
  const int64_t valid = (int64_t)N * rowlen, total = (int64_t)Npad * rowlen;
  const int64_t stride = (int64_t)gridDim.x * kBnThreads;
  if (VEC) {
    for (int64_t e = ((int64_t)blockIdx.x * kBnThreads + threadIdx.x) * 4; e < total; e += stride * 4) {
      float4 o = {0.f, 0.f, 0.f, 0.f};
      if (e < valid) {
        const int c = (int)((e / HW) % C);
        const float m = save[c * kSave + 0], a = save[c * kSave + 2], b = save[c * kSave + 3];
        const float4 v = *reinterpret_cast<const float4*>(z + e);
        o.x = leaky(fmaf(a, v.x - m, b), slope);
        o.y = leaky(fmaf(a, v.y - m, b), slope);
        o.z = leaky(fmaf(a, v.z - m, b), slope);
        o.w = leaky(fmaf(a, v.w - m, b), slope);
      }
      *reinterpret_cast<float4*>(y + e) = o;
    }
  } else {
    for (int64_t e = (int64_t)blockIdx.x * kBnThreads + threadIdx.x; e < total; e += stride) {
      float o = 0.f;
      if (e < valid) {
        const int c = (int)((e / HW) % C);
        o = leaky(fmaf(save[c * kSave + 2], z[e] - save[c * kSave + 0], save[c * kSave + 3]), slope);
      }
      y[e] = o;
    }
  }
}

// backward statistics: sums of g and g xhat, g = dy act'(a z + b), xhat = (z - mean) invstd
template <bool VEC>
__global__ __launch_bounds__(kBnThreads) void bn_bwd_stats_kernel(
    const float* __restrict__ dy, const float* __restrict__ z, const float* __restrict__ save,
    double* __restrict__ partial, int N, int C, int HW, float slope) {
  __shared__ double red[kBnThreads / 64];
  const int c = blockIdx.y, S = gridDim.x, s = blockIdx.x;
  const float mean = save[c * kSave + 0], invstd = save[c * kSave + 1];
  const float a = save[c * kSave + 2], b = save[c * kSave + 3];
  double sg = 0.0, sgx = 0.0;
  auto acc = [&](float zv, float dv) {
    const float zc = zv - mean;
    const float g = fmaf(a, zc, b) > 0.f ? dv : dv * slope;
    sg += (double)g;
    sgx = fma((double)g, (double)(zc * invstd), sgx);
  };
  if (VEC) {
    const int HW4 = HW >> 2;
    const int64_t M4 = (int64_t)N * HW4;
    for (int64_t e = (int64_t)s * kBnThreads + threadIdx.x; e < M4; e += (int64_t)S * kBnThreads) {
      const int64_t n = e / HW4;
      const int64_t off = (n * C + c) * HW + 4 * (int)(e - n * HW4);
      const float4 v = *reinterpret_cast<const float4*>(z + off);
      const float4 d = *reinterpret_cast<const float4*>(dy + off);
      acc(v.x, d.x); acc(v.y, d.y); acc(v.z, d.z); acc(v.w, d.w);
    }
  } else {
    const int64_t M = (int64_t)N * HW;
    for (int64_t e = (int64_t)s * kBnThreads + threadIdx.x; e < M; e += (int64_t)S * kBnThreads) {
      const int64_t n = e / HW;
      const int64_t off = (n * C + c) * HW + (int)(e - n * HW);
      acc(z[off], dy[off]);
    }
  }
  sg = block_sum(sg, red);
  sgx = block_sum(sgx, red);
  if (threadIdx.x == 0) {
    partial[((int64_t)c * S + s) * 2 + 0] = sg;
    partial[((int64_t)c * S + s) * 2 + 1] = sgx;
  }
}

// dgamma = sum g xhat, dbeta = sum g; coef[c] = (k1 = gamma invstd, mean g, mean g xhat)
// (train mode; eval mode has no batch-statistics terms: mean terms 0)
__global__ void bn_bwd_finalize_kernel(const double* __restrict__ partial,
                                       const float* __restrict__ gamma,
                                       const float* __restrict__ save, float* __restrict__ dgamma,
                                       float* __restrict__ dbeta, float* __restrict__ coef, int S,
                                       int N, int C, int HW, int training) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double sg = 0.0, sgx = 0.0;
  for (int s = 0; s < S; ++s) {
    sg += partial[((int64_t)c * S + s) * 2 + 0];
    sgx += partial[((int64_t)c * S + s) * 2 + 1];
  }
  if (dgamma) dgamma[c] = (float)sgx;
  if (dbeta) dbeta[c] = (float)sg;
  const double M = (double)N * HW;
  coef[c * 3 + 0] = (gamma ? gamma[c] : 1.0f) * save[c * kSave + 1];
  coef[c * 3 + 1] = training ? (float)(sg / M) : 0.f;
  coef[c * 3 + 2] = training ? (float)(sgx / M) : 0.f;
}

template <bool VEC>
__global__ __launch_bounds__(kBnThreads) void bn_bwd_apply_kernel(
    const float* __restrict__ dy, const float* __restrict__ z, const float* __restrict__ save,
    const float* __restrict__ coef, float* __restrict__ dz, int N, int Npad, int C, int HW,
    float slope) {
  const int64_t rowlen = (int64_t)C * HW;
  const int64_t valid = (int64_t)N * rowlen, total = (int64_t)Npad * rowlen;
  const int64_t stride = (int64_t)gridDim.x * kBnThreads;
  if (VEC) {
    for (int64_t e = ((int64_t)blockIdx.x * kBnThreads + threadIdx.x) * 4; e < total; e += stride * 4) {
      float4 o = {0.f, 0.f, 0.f, 0.f};
      if (e < valid) {
        const int c = (int)((e / HW) % C);
        const float mean = save[c * kSave + 0], invstd = save[c * kSave + 1];
        const float a = save[c * kSave + 2], b = save[c * kSave + 3];
        const float k1 = coef[c * 3 + 0], mg = coef[c * 3 + 1], mgx = coef[c * 3 + 2];
        const float4 v = *reinterpret_cast<const float4*>(z + e);
        const float4 d = *reinterpret_cast<const float4*>(dy + e);
        auto one = [&](float zv, float dv) {
          const float zc = zv - mean;
          const float g = fmaf(a, zc, b) > 0.f ? dv : dv * slope;
          return k1 * (g - mg - zc * invstd * mgx);
        };
        o.x = one(v.x, d.x); o.y = one(v.y, d.y); o.z = one(v.z, d.z); o.w = one(v.w, d.w);
      }
      *reinterpret_cast<float4*>(dz + e) = o;
    }
  } else {
    for (int64_t e = (int64_t)blockIdx.x * kBnThreads + threadIdx.x; e < total; e += stride) {
      float o = 0.f;
      if (e < valid) {
        const int c = (int)((e / HW) % C);
        const float zc = z[e] - save[c * kSave], dv = dy[e];
        const float g = fmaf(save[c * kSave + 2], zc, save[c * kSave + 3]) > 0.f ? dv : dv * slope;
        o = coef[c * 3 + 0] * (g - coef[c * 3 + 1] - zc * save[c * kSave + 1] * coef[c * 3 + 2]);
      }
      dz[e] = o;
    }
  }
}

int bn_slices(int N, int HW) {
  const int64_t M = (int64_t)N * HW;
  int64_t s = (M + kBnThreads * 16 - 1) / (kBnThreads * 16);
  return (int)(s < 1 ? 1 : (s > 128 ? 128 : s));
}

int apply_grid(int64_t total, bool vec) {
  int64_t items = vec ? total / 4 : total;
  int64_t g = (items + kBnThreads - 1) / kBnThreads;
  return (int)(g < 1 ? 1 : (g > 8192 ? 8192 : g));
}

bool bad_shape(int N, int Npad, int C, int HW) {
  return N < 1 || Npad < N || C < 1 || C > 65535 || HW < 1;
}

}  // namespace

BLINDNO_API int blindno_bn_act_nslices(int N, int C, int HW) {
  (void)C;
  return bn_slices(N, HW);
}

BLINDNO_API int blindno_bn_act_fwd(const float* z, const float* gamma, const float* beta,
                                   float* run_mean, float* run_var, float* y, float* save,
                                   float* partial, int N, int Npad, int C, int HW, float eps,
                                   float momentum, float slope, int training, void* stream) {
  if (bad_shape(N, Npad, C, HW) || !z || !y || !save ||
      (training && !partial) || (!training && (!run_mean || !run_var)) ||
      (run_mean == nullptr) != (run_var == nullptr))
    return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  const bool vec = (HW & 3) == 0;
  const int S = bn_slices(N, HW);
  // partial holds C S 2 doubles (8-B aligned)
  double* pd = reinterpret_cast<double*>(partial);
  if (training) {
    if (((uintptr_t)partial & 7) != 0) return (int)hipErrorInvalidValue;
    if (vec) bn_stats_kernel<true><<<dim3(S, C), kBnThreads, 0, st>>>(z, pd, N, C, HW);
    else bn_stats_kernel<false><<<dim3(S, C), kBnThreads, 0, st>>>(z, pd, N, C, HW);
  }
  bn_finalize_kernel<<<cdiv(C, 64), 64, 0, st>>>(z, pd, gamma, beta, run_mean, run_var, save,
                                                S, N, C, HW, eps, momentum, training);
  const int64_t total = (int64_t)Npad * C * HW;
  if (vec) bn_apply_kernel<true><<<apply_grid(total, true), kBnThreads, 0, st>>>(z, save, y, N, Npad, C, HW, slope);
  else bn_apply_kernel<false><<<apply_grid(total, false), kBnThreads, 0, st>>>(z, save, y, N, Npad, C, HW, slope);
  return (int)hipGetLastError();
}

BLINDNO_API int blindno_bn_act_bwd(const float* dy, const float* z, const float* gamma,
                                   const float* save, float* dz, float* dgamma, float* dbeta,
                                   float* partial, float* coef, int N, int Npad, int C, int HW,
                                   float slope, int training, void* stream) {
  if (bad_shape(N, Npad, C, HW) || !dy || !z || !save || !dz || !partial || !coef)
    return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  const bool vec = (HW & 3) == 0;
  const int S = bn_slices(N, HW);
  if (((uintptr_t)partial & 7) != 0) return (int)hipErrorInvalidValue;
  double* pd = reinterpret_cast<double*>(partial);
  if (vec) bn_bwd_stats_kernel<true><<<dim3(S, C), kBnThreads, 0, st>>>(dy, z, save, pd, N, C, HW, slope);
  else bn_bwd_stats_kernel<false><<<dim3(S, C), kBnThreads, 0, st>>>(dy, z, save, pd, N, C, HW, slope);
  bn_bwd_finalize_kernel<<<cdiv(C, 64), 64, 0, st>>>(pd, gamma, save, dgamma, dbeta, coef, S, N,
                                                    C, HW, training);
  const int64_t total = (int64_t)Npad * C * HW;
  if (vec) bn_bwd_apply_kernel<true><<<apply_grid(total, true), kBnThreads, 0, st>>>(dy, z, save, coef, dz, N, Npad, C, HW, slope);
  else bn_bwd_apply_kernel<false><<<apply_grid(total, false), kBnThreads, 0, st>>>(dy, z, save, coef, dz, N, Npad, C, HW, slope);
  return (int)hipGetLastError();
}
