// DeepONet combiner fused with the snapshot-bag mean that consumes it (NIO models).
//
// Reference: DeepOnetNoBiasOrg.forward, 2d_FPE/DeepONetModules.py:142-151,
//     u[b, l, p] = (w[b, l, :] . basis[p, :] + b0) / sqrt(P),
// followed by the fixed-weight bag mean of NIOFP2D (2d_FPE/NIOModules.py:66-77; NC copy
// 2d_Non_conservative_FPE/NIOModules.py:65-76; 1D NIOFP 1d_FPE/NIOModules.py:62-77), which reads
// u only through its mean over the bag.  The mean commutes with the combiner:
//     ubar[b, p] = sum_l lw_l u[b, l, p] = (wbar[b] . basis[p] + b0 sum_l lw_l) / sqrt(P),
//     wbar[b, k] = sum_l lw_l w[b, l, k]        (lw_l = 1 / L, or multiplicity weights),
// so the (B, L, S) field is never formed (S = grid points): the forward reads w (B L P floats)
// and basis (S P), writes ubar (B S).  Backward, with g = dL/dubar:
//     dbasis[p, k] = scale sum_b g[b, p] wbar[b, k],
//     dwbar[b, k]  = scale sum_p g[b, p] basis[p, k],   dw[b, l, k] = lw_l dwbar[b, k],
//     db0          = scale sum_{b, p} g[b, p] sum_l lw_l.
// The two reductions over p are per-workgroup partials summed in a fixed order (no atomics).
// More than kMaxB bags run as bag chunks of kMaxB in stream order: dbasis and db0 of a later
// chunk are added to the earlier chunks' (fixed chunk order, deterministic).
#include "common.h"
#include "blindno.h"

using namespace blindno;

namespace {

constexpr int kPts = 256;          // grid points per workgroup
constexpr int kMaxP = 64;          // basis functions (n_basis = 25 in every reference script)
constexpr int kMaxB = 64;          // bags per backward launch (LDS: 148.7 KB at B = P = 64)

// ubar[b, p] for the kPts points of this workgroup and bag blockIdx.y
__global__ __launch_bounds__(kPts) void deeponet_bag_fwd_kernel(
    const float* __restrict__ w, const float* __restrict__ basis, const float* __restrict__ b0,
    const float* __restrict__ lw, float* __restrict__ wbar, float* __restrict__ ubar, int L, int S,
    int P, float scale) {
  __shared__ float sw[kMaxP];
  const int b = blockIdx.y, tid = threadIdx.x;
  if (tid < P) {
    // fixed order over the bag, the same in every workgroup of this bag
    const float* wb = w + (size_t)b * L * P + tid;
    float acc = 0.f;
    if (lw) {
      for (int l = 0; l < L; ++l) acc = fmaf(lw[l], wb[(size_t)l * P], acc);
    } else {
      for (int l = 0; l < L; ++l) acc += wb[(size_t)l * P];
      acc *= 1.0f / (float)L;
    }
    sw[tid] = acc;
    if (blockIdx.x == 0) wbar[b * P + tid] = acc;
  }
  __syncthreads();
  float lsum = 1.0f;
  if (lw) {
    lsum = 0.f;
    for (int l = 0; l < L; ++l) lsum += lw[l];
  }
  const int p = blockIdx.x * kPts + tid;
  if (p >= S) return;
  const float* bp = basis + (size_t)p * P;
  float acc = 0.f;
  for (int k = 0; k < P; ++k) acc = fmaf(sw[k], bp[k], acc);
  ubar[(size_t)b * S + p] = (acc + b0[0] * lsum) * scale;
}

// dbasis for this workgroup's points, and the workgroup's partial sums
//     partial[blk][b P + k] = scale sum_{p in blk} g[b, p] basis[p, k],  partial[blk][B P] = scale sum g
__global__ __launch_bounds__(kPts) void deeponet_bag_bwd_kernel(
    const float* __restrict__ g, const float* __restrict__ basis, const float* __restrict__ wbar,
    float* __restrict__ dbasis, float* __restrict__ partial, int B, int S, int P, float scale,
    int accumulate) {
  // dynamic LDS: sg [B][kPts + 1] (g scaled), sb [kPts][P + 1] (basis rows), sw [B][P] (wbar)
  extern __shared__ float lds[];
  float* sg = lds;
  float* sb = sg + B * (kPts + 1);
  float* sw = sb + kPts * (P + 1);
  const int tid = threadIdx.x, p0 = blockIdx.x * kPts;
  const int np = S - p0 < kPts ? S - p0 : kPts;
  for (int e = tid; e < B * P; e += kPts) sw[e] = wbar[e];
  for (int b = 0; b < B; ++b)
    sg[b * (kPts + 1) + tid] = tid < np ? g[(size_t)b * S + p0 + tid] * scale : 0.f;
  for (int e = tid; e < kPts * P; e += kPts) {
    const int q = e / P, k = e - q * P;
    sb[q * (P + 1) + k] = q < np ? basis[(size_t)(p0 + q) * P + k] : 0.f;
  }
  __syncthreads();
  // dbasis[p, k] = sum_b g[b, p] wbar[b, k] (scale folded into sg)
  for (int e = tid; e < np * P; e += kPts) {
    const int q = e / P, k = e - q * P;
    float acc = 0.f;
    for (int b = 0; b < B; ++b) acc = fmaf(sg[b * (kPts + 1) + q], sw[b * P + k], acc);
    float* o = dbasis + (size_t)(p0 + q) * P + k;
    *o = accumulate ? *o + acc : acc;
  }
  // partials: one (b, k) pair (or the b0 sum) per thread, points in order
  const int npair = B * P + 1;
  float* pp = partial + (size_t)blockIdx.x * npair;
  for (int e = tid; e < npair; e += kPts) {
    float acc = 0.f;
    if (e < B * P) {
      const int b = e / P, k = e - b * P;
      for (int q = 0; q < kPts; ++q) acc = fmaf(sg[b * (kPts + 1) + q], sb[q * (P + 1) + k], acc);
    } else {
      for (int b = 0; b < B; ++b)
        for (int q = 0; q < kPts; ++q) acc += sg[b * (kPts + 1) + q];
    }
    pp[e] = acc;
  }
}

// fixed-order sum of the partials; dw[b, l, k] = lw_l dwbar[b, k], db0 = sum g * sum_l lw_l
__global__ __launch_bounds__(256) void deeponet_bag_finish_kernel(
    const float* __restrict__ partial, const float* __restrict__ lw, float* __restrict__ dw,
    float* __restrict__ db0, int nblk, int B, int L, int P, int accumulate) {
  __shared__ float sd[kMaxB * kMaxP + 1];
  const int npair = B * P + 1;
  for (int e = threadIdx.x; e < npair; e += blockDim.x) {
    float acc = 0.f;
    for (int j = 0; j < nblk; ++j) acc += partial[(size_t)j * npair + e];
    sd[e] = acc;
  }
  __syncthreads();
  if (threadIdx.x == 0 && db0) {
    float lsum = 1.0f;
    if (lw) {
      lsum = 0.f;
      for (int l = 0; l < L; ++l) lsum += lw[l];
    }
    db0[0] = accumulate ? db0[0] + sd[B * P] * lsum : sd[B * P] * lsum;
  }
  const float inv = 1.0f / (float)L;
  const int n = B * L * P;
  for (int e = threadIdx.x; e < n; e += blockDim.x) {
    const int b = e / (L * P), r = e - b * L * P, l = r / P, k = r - l * P;
    dw[e] = sd[b * P + k] * (lw ? lw[l] : inv);
  }
}

bool dims_ok(int B, int L, int S, int P) {
  return B >= 1 && L >= 1 && S >= 1 && P >= 1 && P <= kMaxP;
}

}  // namespace

BLINDNO_API int blindno_deeponet_bag_nblk(int S) { return S < 1 ? 1 : cdiv(S, kPts); }

BLINDNO_API int blindno_deeponet_bag_fwd(const float* w, const float* basis, const float* b0,
                                         const float* lw, float* wbar, float* ubar, int B, int L,
                                         int S, int P, float scale, void* stream) {
  if (!dims_ok(B, L, S, P) || !w || !basis || !b0 || !wbar || !ubar) return (int)hipErrorInvalidValue;
  dim3 grid(cdiv(S, kPts), B);
  deeponet_bag_fwd_kernel<<<grid, kPts, 0, (hipStream_t)stream>>>(w, basis, b0, lw, wbar, ubar, L,
                                                                  S, P, scale);
  return (int)hipGetLastError();
}

BLINDNO_API int blindno_deeponet_bag_bwd(const float* g, const float* basis, const float* wbar,
                                         const float* lw, float* dw, float* dbasis, float* db0,
                                         float* partial, int nblk, int B, int L, int S, int P,
                                         float scale, void* stream) {
  if (!dims_ok(B, L, S, P) || !g || !basis || !wbar || !dw || !dbasis || !partial ||
      nblk != blindno_deeponet_bag_nblk(S))
    return (int)hipErrorInvalidValue;
  // bag chunks of <= kMaxB in stream order; each reuses the partial buffer (sized for B bags)
  for (int c0 = 0; c0 < B; c0 += kMaxB) {
    const int bc = B - c0 < kMaxB ? B - c0 : kMaxB;
    const size_t lds =
        sizeof(float) * ((size_t)bc * (kPts + 1) + (size_t)kPts * (P + 1) + (size_t)bc * P);
    deeponet_bag_bwd_kernel<<<nblk, kPts, lds, (hipStream_t)stream>>>(
        g + (size_t)c0 * S, basis, wbar + (size_t)c0 * P, dbasis, partial, bc, S, P, scale, c0 > 0);
    deeponet_bag_finish_kernel<<<1, 256, 0, (hipStream_t)stream>>>(
        partial, lw, dw + (size_t)c0 * L * P, db0, nblk, bc, L, P, c0 > 0);
  }
  return (int)hipGetLastError();
}
