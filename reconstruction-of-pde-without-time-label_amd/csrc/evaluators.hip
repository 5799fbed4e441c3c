// Density evaluators: the batched 1D GPE split-step pseudo-spectral solver (one workgroup per
// trajectory, the whole time loop resident in LDS) and the trapezoid-rule density-residual
// reduction of the 1D time-averaged L2 error.
//
// Reference (yl602019618/Reconstruction-of-PDE-without-Time-Label):
//   solve_GPE_custom / step_strang / step_fourth_order / step_linear / step_nonlinear
//     1d_GPE/datagen_GPE.py:29-115 (same copy in 1d_GPE/compute_time_error_GPE.py:108-160)
//   time_averaged_L2_error  1d_FPE/compute_time_error.py:240-295,
//                           1d_GPE/compute_time_error_GPE.py:162-203
// fp64 throughout (the reference is numpy complex128).  Floating-point contraction is off so
// each complex product rounds like numpy's (a c - b d, a d + b c).
#include "common.h"
#include "blindno.h"

#pragma clang fp contract(off)

using namespace blindno;

namespace {

struct cd {
  double re, im;
};

__device__ __forceinline__ cd cmul(cd a, cd b) {
  return {a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re};
}

// One radix-2 Stockham pass over N points held in LDS (src -> dst), natural order in and out.
// Butterfly j reads src[j], src[j + N/2]; span Ns; twiddle e^{-/+ 2 pi i k / (2 Ns)} taken from
// tw[k * N/(2 Ns)] (tw[i] = e^{-2 pi i i/N}, i < N/2), conjugated for the inverse.
template <bool INV>
__device__ __forceinline__ void fft_pass(const cd* __restrict__ src, cd* __restrict__ dst,
                                         const cd* __restrict__ tw, int N, int Ns) {
  const int half = N >> 1;
  const int tstride = half / Ns;
  for (int j = threadIdx.x; j < half; j += blockDim.x) {
    const int k = j & (Ns - 1);
    cd w = tw[k * tstride];
    if (INV) w.im = -w.im;
    const cd a0 = src[j];
    const cd a1 = cmul(src[j + half], w);
    const int d = ((j - k) << 1) + k;
    dst[d] = {a0.re + a1.re, a0.im + a1.im};
    dst[d + Ns] = {a0.re - a1.re, a0.im - a1.im};
  }
}

// Full transform of buf[0] (result ends in buf[cur], returned); log2(N) passes.
template <bool INV>
__device__ int fft(cd* buf0, cd* buf1, const cd* tw, int N) {
  cd* bufs[2] = {buf0, buf1};
  int cur = 0;
  for (int Ns = 1; Ns < N; Ns <<= 1) {
    fft_pass<INV>(bufs[cur], bufs[cur ^ 1], tw, N, Ns);
    cur ^= 1;
    __syncthreads();
  }
  return cur;
}

// psi <- exp(-i h (V + g|psi|^2 + kappa|psi|^4)) psi   (step_nonlinear, datagen_GPE.py:37-42)
__device__ __forceinline__ void nonlinear(cd* psi, const double* V, double g, double kappa,
                                          double h, int N) {
  for (int i = threadIdx.x; i < N; i += blockDim.x) {
    const cd p = psi[i];
    const double a = hypot(p.re, p.im);
    const double A = V[i] + g * (a * a) + kappa * pow(a, 4.0);
    const double th = -h * A;
    double s, c;
    sincos(th, &s, &c);
    psi[i] = cmul({c, s}, p);
  }
}

// kinetic step in Fourier space: psi_hat *= lin[i]  (step_linear, datagen_GPE.py:29-35),
// inverse FFT normalised by 1/N (numpy.fft.ifft)
__device__ void linear(cd*& psi, cd*& other, const cd* lin, const cd* tw, int N) {
  int cur = fft<false>(psi, other, tw, N);
  if (cur) {
    cd* t = psi; psi = other; other = t;
  }
  for (int i = threadIdx.x; i < N; i += blockDim.x) psi[i] = cmul(psi[i], lin[i]);
  __syncthreads();
  cur = fft<true>(psi, other, tw, N);
  if (cur) {
    cd* t = psi; psi = other; other = t;
  }
  const double invN = 1.0 / (double)N;
  for (int i = threadIdx.x; i < N; i += blockDim.x) {
    psi[i].re = psi[i].re * invN;
    psi[i].im = psi[i].im * invN;
  }
  __syncthreads();
}

__global__ void gpe_solve_kernel(const double* __restrict__ psi0, const double* __restrict__ Vg,
                                 const double* __restrict__ gg, const double* __restrict__ kg,
                                 double dx, double dt, int nsteps, int order, int rec_every,
                                 double* __restrict__ rec_abs, double* __restrict__ rec_psi,
                                 double* __restrict__ psi_out, int N, int psi0_batched) {
  extern __shared__ cd smem[];
  cd* bufA = smem;
  cd* bufB = bufA + N;
  cd* tw = bufB + N;            // N/2
  cd* lin0 = tw + N / 2;        // N
  cd* lin1 = lin0 + N;          // N (order 4 only)
  double* V = reinterpret_cast<double*>(lin1 + N);   // N
  const int b = blockIdx.x;
  const double g = gg[b], kappa = kg[b];
  const double* psi_src = psi0 + (psi0_batched ? (int64_t)b * N * 2 : 0);
  for (int i = threadIdx.x; i < N; i += blockDim.x) {
    bufA[i] = {psi_src[2 * i], psi_src[2 * i + 1]};
    V[i] = Vg[(int64_t)b * N + i];
  }
  for (int i = threadIdx.x; i < N / 2; i += blockDim.x) {
    double s, c;
    sincospi(2.0 * (double)i / (double)N, &s, &c);
    tw[i] = {c, -s};
  }
  // k = 2 pi fftfreq(N, dx): j * (1/(N dx)) for j < (N+1)/2, else (j - N) * (1/(N dx))
  // Yoshida coefficients as the reference forms them (2**(1/3) = pow(2, 1/3))
  const double cr = pow(2.0, 1.0 / 3.0);
  const double c2 = 2.0 - cr;
  const double a1 = 1.0 / c2, a2 = -cr / c2;
  const double hl0 = order == 4 ? a1 * dt : dt;
  const double hl1 = a2 * dt;
  const double val = 1.0 / ((double)N * dx);
  for (int i = threadIdx.x; i < N; i += blockDim.x) {
    const int f = i < (N + 1) / 2 ? i : i - N;
    const double k = 6.283185307179586 * ((double)f * val);
    const double k2 = k * k;
    double s, c;
    sincos((-hl0 * 0.5) * k2, &s, &c);
    lin0[i] = {c, s};
    if (order == 4) {
      sincos((-hl1 * 0.5) * k2, &s, &c);
      lin1[i] = {c, s};
    }
  }
  __syncthreads();
  const int nrec = nsteps / rec_every + 1;
  auto record = [&](const cd* psi, int r) {
    for (int i = threadIdx.x; i < N; i += blockDim.x) {
      const cd p = psi[i];
      if (rec_abs) rec_abs[((int64_t)b * nrec + r) * N + i] = hypot(p.re, p.im);
      if (rec_psi) {
        double* d = rec_psi + (((int64_t)b * nrec + r) * N + i) * 2;
        d[0] = p.re;
        d[1] = p.im;
      }
    }
  };
  cd* psi = bufA;
  cd* other = bufB;
  record(psi, 0);
  for (int n = 1; n <= nsteps; ++n) {
    if (order == 2) {
      nonlinear(psi, V, g, kappa, dt / 2, N);
      __syncthreads();
      linear(psi, other, lin0, tw, N);
      nonlinear(psi, V, g, kappa, dt / 2, N);
      __syncthreads();
    } else {
      // Yoshida: N(b1) L(a1) N(b2) L(a2) N(b1) L(a2) N(b2) L(a1) N(b1), b = a
      const double hb1 = a1 * dt, hb2 = a2 * dt;
      nonlinear(psi, V, g, kappa, hb1, N); __syncthreads();
      linear(psi, other, lin0, tw, N);
      nonlinear(psi, V, g, kappa, hb2, N); __syncthreads();
      linear(psi, other, lin1, tw, N);
      nonlinear(psi, V, g, kappa, hb1, N); __syncthreads();
      linear(psi, other, lin1, tw, N);
      nonlinear(psi, V, g, kappa, hb2, N); __syncthreads();
      linear(psi, other, lin0, tw, N);
      nonlinear(psi, V, g, kappa, hb1, N); __syncthreads();
    }
    if (n % rec_every == 0) record(psi, n / rec_every);
  }
  if (psi_out)
    for (int i = threadIdx.x; i < N; i += blockDim.x) {
      psi_out[((int64_t)b * N + i) * 2] = psi[i].re;
      psi_out[((int64_t)b * N + i) * 2 + 1] = psi[i].im;
    }
}

// out[2r] = trapz((a_r - b_r)^2, x), out[2r+1] = trapz(b_r^2, x)   (numpy.trapz: d (y1 + y0)/2)
__global__ __launch_bounds__(kBlock) void trapz_rows_kernel(const double* __restrict__ a,
                                                            const double* __restrict__ b,
                                                            const double* __restrict__ x,
                                                            double* __restrict__ out, int n) {
  __shared__ double ra[kBlock], rb[kBlock];
  const int r = blockIdx.x;
  const double* ap = a + (int64_t)r * n;
  const double* bp = b + (int64_t)r * n;
  double sa = 0.0, sb = 0.0;
  for (int i = threadIdx.x; i < n - 1; i += blockDim.x) {
    const double d = x[i + 1] - x[i];
    const double e0 = ap[i] - bp[i], e1 = ap[i + 1] - bp[i + 1];
    sa += d * (e1 * e1 + e0 * e0) / 2.0;
    sb += d * (bp[i + 1] * bp[i + 1] + bp[i] * bp[i]) / 2.0;
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


// ---------------------------------------------------------------- FPE master equation
// dp/dt = M p on a 1D / 2D grid of N = nx*ny cells (x-major, cell i = ix*ny + iy), the
// finite-volume master equation fplanck builds (fokker_planck.master_matrix; used by
// 1d_FPE/compute_time_error.py:215-238, 2d_Non_conservative_FPE/compute_time_error.py:300-319):
//   (M p)_i = cxm_i p_{i-ex} + cxp_i p_{i+ex} + cym_i p_{i-ey} + cyp_i p_{i+ey} - diag_i p_i
// coef (B, 5, N) = [diag, cxm, cxp, cym, cyp] per trajectory (in-rates from the neighbours, zero
// across a reflecting wall; neighbour indices wrap, which is the periodic case).
// One workgroup per trajectory: p (CPT cells per thread) in registers, the Taylor iterate
// ping-pongs in LDS.  Each output interval is s substeps of exp(h M) ~ degree-m Taylor polynomial
// in Horner form  w <- p + (h/k) M w,  k = m..1.
template <int CPT>
__global__ __launch_bounds__(1024) void fp_propagate_kernel(const double* __restrict__ p0,
                                                            const double* __restrict__ coef,
                                                            double* __restrict__ out, int N,
                                                            int nx, int ny, int nout, int s,
                                                            int m, double h) {
  extern __shared__ double fsm[];
  double* wa = fsm;
  double* wb = fsm + N;
  const int b = blockIdx.x;
  const double* cf = coef + (int64_t)b * 5 * N;
  double p[CPT];
#pragma unroll
  for (int c = 0; c < CPT; ++c) {
    const int i = threadIdx.x + c * blockDim.x;
    p[c] = i < N ? p0[(int64_t)b * N + i] : 0.0;
    if (i < N) out[(int64_t)b * nout * N + i] = p[c];
  }
  for (int o = 1; o < nout; ++o) {
    for (int sub = 0; sub < s; ++sub) {
#pragma unroll
      for (int c = 0; c < CPT; ++c) {
        const int i = threadIdx.x + c * blockDim.x;
        if (i < N) wa[i] = p[c];
      }
      __syncthreads();
      for (int k = m; k >= 1; --k) {
        const double hk = h / (double)k;
#pragma unroll
        for (int c = 0; c < CPT; ++c) {
          const int i = threadIdx.x + c * blockDim.x;
          if (i < N) {
            const int ix = i / ny, iy = i - ix * ny;
            const int xm = (ix == 0 ? nx - 1 : ix - 1) * ny + iy;
            const int xp = (ix == nx - 1 ? 0 : ix + 1) * ny + iy;
            const int ym = ix * ny + (iy == 0 ? ny - 1 : iy - 1);
            const int yp = ix * ny + (iy == ny - 1 ? 0 : iy + 1);
            double mw = -cf[i] * wa[i];
            mw = fma(cf[N + i], wa[xm], mw);
            mw = fma(cf[2 * N + i], wa[xp], mw);
            mw = fma(cf[3 * N + i], wa[ym], mw);
            mw = fma(cf[4 * N + i], wa[yp], mw);
            wb[i] = fma(hk, mw, p[c]);
          }
        }
        __syncthreads();
        double* t = wa; wa = wb; wb = t;
      }
#pragma unroll
      for (int c = 0; c < CPT; ++c) {
        const int i = threadIdx.x + c * blockDim.x;
        if (i < N) p[c] = wa[i];
      }
      __syncthreads();
    }
#pragma unroll
    for (int c = 0; c < CPT; ++c) {
      const int i = threadIdx.x + c * blockDim.x;
      if (i < N) out[((int64_t)b * nout + o) * N + i] = p[c];
    }
  }
}

}  // namespace

BLINDNO_API int blindno_gpe_solve(const double* psi0, const double* V, const double* g,
                                  const double* kappa, double dx, double dt, int nsteps, int order,
                                  int rec_every, double* rec_abs, double* rec_psi, double* psi_out,
                                  int B, int N, int psi0_batched, void* stream) {
  if (B <= 0 || N < 4 || (N & (N - 1)) || N > 2048 || nsteps < 0 || rec_every < 1 ||
      (order != 2 && order != 4))
    return (int)hipErrorInvalidValue;
  // lin1 is always laid out (V follows it), so size for both tables
  const size_t sh = sizeof(cd) * ((size_t)N * 2 + N / 2 + 2 * (size_t)N) + sizeof(double) * N;
  if (sh > 160 * 1024) return (int)hipErrorInvalidValue;
  int threads = N / 2;
  if (threads < 64) threads = 64;
  if (threads > 256) threads = 256;
  gpe_solve_kernel<<<B, threads, sh, (hipStream_t)stream>>>(psi0, V, g, kappa, dx, dt, nsteps,
                                                            order, rec_every, rec_abs, rec_psi,
                                                            psi_out, N, psi0_batched);
  return (int)hipGetLastError();
}

BLINDNO_API int blindno_trapz_rows(const double* a, const double* b, const double* x, double* out,
                                   int rows, int n, void* stream) {
  if (rows <= 0 || n < 1) return (int)hipErrorInvalidValue;
  trapz_rows_kernel<<<rows, kBlock, 0, (hipStream_t)stream>>>(a, b, x, out, n);
  return (int)hipGetLastError();
}

BLINDNO_API int blindno_fp_propagate(const double* p0, const double* coef, double* out, int B,
                                     int nx, int ny, int nout, int substeps, int degree,
                                     double dt_out, void* stream) {
  const int64_t N = (int64_t)nx * ny;
  if (B <= 0 || nx < 1 || ny < 1 || nout < 1 || substeps < 1 || degree < 1 || N > 8192)
    return (int)hipErrorInvalidValue;
  const size_t sh = sizeof(double) * 2 * (size_t)N;
  const int threads = N <= 256 ? 256 : (N <= 1024 ? 1024 : 1024);
  const int cpt = (int)((N + threads - 1) / threads);
  const double h = dt_out / substeps;
  hipStream_t st = (hipStream_t)stream;
#define FPL(C_) fp_propagate_kernel<C_><<<B, threads, sh, st>>>(p0, coef, out, (int)N, nx, ny, nout, \
                                                               substeps, degree, h)
  if (cpt <= 1) FPL(1);
  else if (cpt <= 2) FPL(2);
  else if (cpt <= 4) FPL(4);
  else FPL(8);
#undef FPL
  return (int)hipGetLastError();
}
