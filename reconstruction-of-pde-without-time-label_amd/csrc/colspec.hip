// The column pass of FNO_input's spectral layers folded into the row kernels (colspec.h):
//   rowdft_cd_kernel  -- row DFT of a field (or of the bag's snapshots, LIFT) plus its column
//                        DFT per 16-row block, written as partials (the layer's first stage
//                        when no row inverse precedes it: the first layer, the last layer's
//                        adjoint);
//   colmix_kernel     -- the block partials of a sample summed in block order, the saved
//                        spectrum Xs (the weight gradient's operand, as the column pass saved
//                        it) and the per-mode channel mix Y that the next row inverse turns
//                        into its row coefficients (ZY).
// Reference: SpectralConv2d.forward, 2d_FPE/FNOModules.py:156-178 (rfft2 -> compl_mul2d on the
// two kept corner blocks -> irfft2); the bag lift of NIOFP2D_FNO, 2d_FPE/NIOModules.py:548-563.
#include "common.h"
#include "blindno.h"
#include "colspec.h"
#include "packw.h"

using namespace blindno;

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kCdWaves = 4;
#ifndef COLSPEC_RD_BLOCKS
#define COLSPEC_RD_BLOCKS 1024
#endif

// Row DFT + column-DFT partials.  Work item = (sample n, channel c, 16-row block b < nbv): 16
// rows x all P2 columns x the NNT column tiles of the spectrum on v_mfma_f32_16x16x4f32 (A = the
// rows, streamed as float4 per lane, two K blocks ahead; B = the row-DFT image Tp in LDS), so
// the D layout is At[h0 + 4 g + r][k' = 16 nt + c16] -- what cd_store takes.
// LIFT: the rows are the bag's snapshots X[b][idx[l]] (one channel, zero past N1 x N2); otherwise
// x[n][c][h][w], read on the valid region N1v x N2v (zero elsewhere), GELU'd first when act.
// BDZ: x is the bag projection's v and the rows are dz = lw_l ghat v (the encoder's last-layer
// gradient formed on load, colspec.h BagDz): ghat (B, N1v N2v), lw (L = U snapshots per bag)
// Body of one workgroup bx of a gx-workgroup grid (rowdft_cd_kernel, rowdft_cd_pack_kernel).
template <int NNT, bool ALIGNED, bool LIFT, bool BDZ>
__device__ __forceinline__ void rowdft_cd_block(
    const float* __restrict__ x, const int* __restrict__ idx, float* __restrict__ part,
    const float* __restrict__ Tp, const float* __restrict__ tab, int Bn, int C, int P1, int P2,
    int m2, int KB, int nbv, int N1v, int N2v, int act, int T, int L,
    const float* __restrict__ ghat, const float* __restrict__ lw, float* lds, int bx, int gx) {
  constexpr int Npad = 16 * NNT;
  float* sT = lds;                                 // [KB][4][Npad][4]
  stage_to_lds(sT, Tp, KB * 16 * Npad);
  __syncthreads();
  const float* tabT = tab + P1 * 2 * kCsK1;        // TabT (colspec.h), after Tab
  const int lane = threadIdx.x & 63;
  const int wave = uniform_int(threadIdx.x >> 6);
  const int r16 = lane & 15, kq = lane >> 4;
  const int nb = P1 >> 4;
  const int nch = colspec_nchunk(C, m2);
  const int64_t nitems = (int64_t)Bn * C * nbv;
  for (int64_t it = (int64_t)bx * kCdWaves + wave; it < nitems; it += (int64_t)gx * kCdWaves) {
    const int b = (int)(it % nbv);
    const int nc = (int)(it / nbv);
    const int c = nc % C, n = nc / C;
    const int h0 = b << 4, h = h0 + r16;
    const bool rok = h < N1v;
    const float* xr;
    const float* gr = ghat;                        // BDZ: this row of ghat
    float lwl = 0.f;
    if constexpr (BDZ) {
      const int bb = n / L, l = n - bb * L;
      gr = ghat + ((int64_t)bb * N1v + (rok ? h : 0)) * N2v;
      lwl = bagdz_scale(lw, L, l);
    }
    if constexpr (LIFT) {
      const int bb = n / L, l = n - bb * L;
      xr = x + (((int64_t)bb * T + (rok ? idx[l] : 0)) * N1v + (rok ? h : 0)) * N2v;
    } else {
      xr = x + (((int64_t)n * C + c) * P1 + (rok ? h : 0)) * P2;
    }
    f32x4 acc[NNT];
#pragma unroll
    for (int t = 0; t < NNT; ++t) acc[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
    auto load_a = [&](int kb, float (&a)[4]) {
      const int w0 = kb * 16 + kq * 4;
      if (ALIGNED && w0 + 3 < N2v) {
        const float4 v = rok ? *reinterpret_cast<const float4*>(xr + w0) : make_float4(0.f, 0.f, 0.f, 0.f);
        a[0] = v.x; a[1] = v.y; a[2] = v.z; a[3] = v.w;
        if constexpr (BDZ) {
          const float4 gv = rok ? *reinterpret_cast<const float4*>(gr + w0) : make_float4(0.f, 0.f, 0.f, 0.f);
          a[0] *= gv.x * lwl; a[1] *= gv.y * lwl; a[2] *= gv.z * lwl; a[3] *= gv.w * lwl;
        }
      } else {
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const bool ok = rok && w0 + s < N2v;
          a[s] = ok ? xr[w0 + s] : 0.f;
          if constexpr (BDZ) a[s] = ok ? a[s] * (gr[w0 + s] * lwl) : 0.f;
        }
      }
    };
    const int KBv = (N2v + 15) >> 4;              // K blocks past the valid columns are zero
    float a1[4], a2[4] = {0.f, 0.f, 0.f, 0.f};
    load_a(0, a1);
    if (KBv > 1) load_a(1, a2);
    for (int kb = 0; kb < KBv; ++kb) {
      float a[4] = {a1[0], a1[1], a1[2], a1[3]};
#pragma unroll
      for (int s = 0; s < 4; ++s) a1[s] = a2[s];
      if (kb + 2 < KBv) load_a(kb + 2, a2);
      if (!LIFT && act) {
#pragma unroll
        for (int s = 0; s < 4; ++s) a[s] = gelu_f(a[s]);
      }
#pragma unroll
      for (int t = 0; t < NNT; ++t) {
        const f32x4 bt = *reinterpret_cast<const f32x4*>(sT + (((kb * 4 + kq) * Npad) + t * 16 + r16) * 4);
#pragma unroll
        for (int s = 0; s < 4; ++s) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], bt[s], acc[t], 0, 0, 0);
      }
    }
    float* blk = part + ((int64_t)n * nb + b) * nch * 128;
    cd_store<NNT>(acc, tabT, h0, lane, blk, c, C, m2);
  }
}

template <int NNT, bool ALIGNED, bool LIFT, bool BDZ = false>
__global__ __launch_bounds__(64 * kCdWaves) void rowdft_cd_kernel(
    const float* __restrict__ x, const int* __restrict__ idx, float* __restrict__ part,
    const float* __restrict__ Tp, const float* __restrict__ tab, int Bn, int C, int P1, int P2,
    int m2, int KB, int nbv, int N1v, int N2v, int act, int T, int L,
    const float* __restrict__ ghat = nullptr, const float* __restrict__ lw = nullptr) {
  extern __shared__ float lds[];
  rowdft_cd_block<NNT, ALIGNED, LIFT, BDZ>(x, idx, part, Tp, tab, Bn, C, P1, P2, m2, KB, nbv, N1v,
                                           N2v, act, T, L, ghat, lw, lds, blockIdx.x, gridDim.x);
}

// The bag lift's rowdft_cd (workgroups [0, nmain)) with the forward's spectral-weight pack
// (blindno_pack_w2d_multi's tiled transpose, one 256-thread tile team per workgroup past nmain)
// in one launch: independent work, bit-identical to the two launches.
template <int NNT, bool ALIGNED>
__global__ __launch_bounds__(64 * kCdWaves) void rowdft_cd_pack_kernel(
    const float* __restrict__ x, const int* __restrict__ idx, float* __restrict__ part,
    const float* __restrict__ Tp, const float* __restrict__ tab, int Bn, int P1, int P2, int m2,
    int KB, int nbv, int N1v, int N2v, int T, int L, int nmain, PackSegs ps) {
  extern __shared__ float lds[];
  const int bx = blockIdx.x;
  if (bx >= nmain) {
    w2d_transpose_tile<0>(ps, bx - nmain, threadIdx.x, reinterpret_cast<float2 (*)[33]>(lds), true);
    return;
  }
  rowdft_cd_block<NNT, ALIGNED, true, false>(x, idx, part, Tp, tab, Bn, 1, P1, P2, m2, KB, nbv,
                                             N1v, N2v, 0, T, L, nullptr, nullptr, lds, bx, nmain);
}

// One workgroup per (sample n, 8 kept rows j of tile mt2): Xs[k][c][j] = the sum of the nbv
// block partials in block order, then
//   DIR 0:  Xsave = Xs,                   Y[k][o][j] = c_k / (P1 P2) sum_c Xs[k][c][j] W[k][j][c][o]
//   DIR 1:  Xsave = G = c_k/(P1 P2) Xs,   Y[k][i][j] = sum_o conj(W[k][j][i][o]) G[k][o][j]
// as the column pass (spectral.hip colfuse_kernel) forms them.  A thread reads one float4 per
// block -- neighbouring lanes (Re, Im) of one mode: Xs[k][c][j0], Xs[k][c][j0 + 1] -- with every
// block's load in flight at once; the workgroup's weight slice W[.][j][.][.] is staged in LDS
// beside them.  LIFT (DIR 0): the partials are the snapshot's (one channel, U), and
// Xs[k][c] = W0[c,0] U[k] + W0[c,1] Dg2[k][0] + W0[c,2] Dg2[k][1] + b0[c] Dg2[k][2] (the lifted
// field's spectrum, by linearity; Dg2 the grid / bias planes' spectrum).  Wt == NULL: Xsave
// only (no mix; the Dg2 precompute).
constexpr int kMixThreads = 256;
constexpr int kMixJ = 8;                           // kept rows per workgroup (one M tile's j)
constexpr int kMixMaxB = 20;                       // blocks per sample (P1 <= 320)
template <int DIR, bool LIFT>
__global__ __launch_bounds__(kMixThreads) void colmix_kernel(
    const float* __restrict__ part, int nbv, const float2* __restrict__ Wt, float2* __restrict__ Xsave,
    float2* __restrict__ Y, int C, int Cp, int P1, int P2, int m2, const float* __restrict__ w0,
    const float* __restrict__ b0, const float2* __restrict__ Dg2) {
  extern __shared__ float2 smx[];
  float2* sP = smx;                                // [m2][Cp][kMixJ]: the summed partials
  float2* sX = sP + m2 * Cp * kMixJ;               // [m2][C][kMixJ]: Xs (LIFT), else sP
  float2* sW = sX + (LIFT ? m2 * C * kMixJ : 0);   // [m2][kMixJ][C][C]: the weight slice
  const int n = blockIdx.x / kCsMT2, mt = blockIdx.x - n * kCsMT2;
  const int j0 = kMixJ * mt;
  const ColspecGeom cg = colspec_geom(Cp, m2);
  const int nch = cg.nch;
  const int nb = P1 >> 4;
  // one float4 (lanes 2 lp, 2 lp + 1 of chunk (cn, mt)) per thread and block
  const int npos = (nch / kCsMT2) * 32;
  if (Wt) {
    const int nw = m2 * kMixJ * C * C;
    for (int e = threadIdx.x; e < nw; e += kMixThreads) {
      const int io = e % (C * C), t = e / (C * C);
      const int jl = t % kMixJ, k = t / kMixJ;
      sW[e] = Wt[((int64_t)k * kCsK1 + j0 + jl) * C * C + io];
    }
  }
  for (int e = threadIdx.x; e < npos; e += kMixThreads) {
    const int cn = e >> 5, lp = e & 31;
    const float* src = part + (((int64_t)n * nb * nch + cn * kCsMT2 + mt) * 64 + 2 * lp) * 2;
    f32x4 v[kMixMaxB];
#pragma unroll
    for (int b = 0; b < kMixMaxB; ++b)
      if (b < nbv) v[b] = *reinterpret_cast<const f32x4*>(src + (int64_t)b * nch * 128);
    f32x4 acc = v[0];
#pragma unroll
    for (int b = 1; b < kMixMaxB; ++b)
      if (b < nbv) acc += v[b];
    const int ln = 2 * lp, c16 = ln & 15, g = ln >> 4;
    int c, k;
    if (cn < Cp * cg.NF) {
      c = cn / cg.NF;
      k = 8 * (cn % cg.NF) + (c16 >> 1);
    } else {                                       // the half tile of channels 2p, 2p + 1
      c = 2 * (cn - Cp * cg.NF) + (c16 >> 3);
      k = 8 * cg.NF + ((c16 & 7) >> 1);
    }
    const int jl = 2 * g;
    if (k < m2 && c < Cp) {
      float2* d = sP + ((int64_t)k * Cp + c) * kMixJ + jl;
      d[0] = make_float2(acc.x, acc.z);
      d[1] = make_float2(acc.y, acc.w);
    }
  }
  __syncthreads();
  const float inv = 1.0f / ((float)P1 * (float)P2);
  float2* Xs = LIFT ? sX : sP;
  const int nx = m2 * C * kMixJ;
  for (int e = threadIdx.x; e < nx; e += kMixThreads) {
    const int jl = e % kMixJ, t = e / kMixJ;
    const int c = t % C, k = t / C;
    float2 v;
    if constexpr (LIFT) {
      const float2 u = sP[(int64_t)k * kMixJ + jl];
      const float2* dg = Dg2 + (int64_t)k * 3 * kCsK1 + j0 + jl;
      const float2 d0 = dg[0], d1 = dg[kCsK1], d2 = dg[2 * kCsK1];
      const float a = w0[c * 3], bx = w0[c * 3 + 1], by = w0[c * 3 + 2], bb = b0[c];
      v.x = fmaf(a, u.x, fmaf(bx, d0.x, fmaf(by, d1.x, bb * d2.x)));
      v.y = fmaf(a, u.y, fmaf(bx, d0.y, fmaf(by, d1.y, bb * d2.y)));
      Xs[e] = v;
    } else {
      v = Xs[e];
      if (DIR == 1) {
        const float sc = c2r_weight(k, P2) * inv;
        v.x *= sc;
        v.y *= sc;
        Xs[e] = v;
      }
    }
    if (Xsave) Xsave[(((int64_t)n * m2 + k) * C + c) * kCsK1 + j0 + jl] = v;
  }
  if (!Wt) return;
  __syncthreads();
  // the mix: output (k, o, j), j fastest (the stores of neighbouring threads are contiguous)
  for (int e = threadIdx.x; e < nx; e += kMixThreads) {
    const int jl = e % kMixJ, t = e / kMixJ;
    const int o = t % C, k = t / C;
    const float2* wj = sW + ((int64_t)k * kMixJ + jl) * C * C;
    const float2* xp = Xs + (int64_t)k * C * kMixJ + jl;
    float re = 0.f, im = 0.f;
    for (int c = 0; c < C; ++c) {
      const float2 a = xp[c * kMixJ];
      const float2 w = DIR == 0 ? wj[c * C + o] : wj[o * C + c];
      if (DIR == 0) {
        re = fmaf(a.x, w.x, fmaf(-a.y, w.y, re));
        im = fmaf(a.x, w.y, fmaf(a.y, w.x, im));
      } else {                                      // conj(w) * a
        re = fmaf(w.x, a.x, fmaf(w.y, a.y, re));
        im = fmaf(w.x, a.y, fmaf(-w.y, a.x, im));
      }
    }
    if (DIR == 0) {
      const float sc = c2r_weight(k, P2) * inv;
      re *= sc;
      im *= sc;
    }
    Y[(((int64_t)n * m2 + k) * C + o) * kCsK1 + j0 + jl] = make_float2(re, im);
  }
}

bool cd_geom_ok(int Bn, int C, int P1, int P2, int m2) {
  return Bn > 0 && C > 0 && C <= 16 && P1 % 16 == 0 && P1 <= 512 && P2 > 0 && m2 > 0 &&
         m2 <= 16 && 2 * m2 <= P2 && (int64_t)Bn * C * P1 * P2 < INT32_MAX;
}

template <bool LIFT, bool BDZ = false>
int rowdft_cd_launch(const float* x, const int* idx, float* part, const float* Tp,
                     const float* tab, int Bn, int C, int P1, int P2, int m2, int act, int N1v,
                     int N2v, int T, int L, hipStream_t st, const float* ghat = nullptr,
                     const float* lw = nullptr, const PackSegs* ps = nullptr, int ntr = 0) {
  const int KB = (P2 + 15) / 16, NNT = (2 * m2 + 15) / 16, Npad = 16 * NNT;
  const int nbv = (N1v + 15) / 16;
  size_t sh = sizeof(float) * (size_t)KB * 16 * Npad;
  if (sh > 160 * 1024 || NNT > 2) return (int)hipErrorInvalidValue;
  const int64_t items = (int64_t)Bn * C * nbv;
  const int64_t b = (items + kCdWaves - 1) / kCdWaves;
  const int blocks = (int)(b < COLSPEC_RD_BLOCKS ? b : COLSPEC_RD_BLOCKS);
  const bool aligned = N2v % 4 == 0 && (LIFT || P2 % 4 == 0) && (((uintptr_t)x) & 15) == 0 &&
                       (((uintptr_t)ghat) & 15) == 0;
  if constexpr (LIFT && !BDZ) {
    if (ps && ntr > 0) {           // hosted pack: one transpose tile per extra workgroup
      if ((int64_t)blocks + ntr >= INT32_MAX) return (int)hipErrorInvalidValue;
      const size_t tsh = sizeof(float2) * 32 * 33;
      if (sh < tsh) sh = tsh;
#define CDP(NNT_, AL_)                                                                         \
  rowdft_cd_pack_kernel<NNT_, AL_><<<blocks + ntr, 64 * kCdWaves, sh, st>>>(                   \
      x, idx, part, Tp, tab, Bn, P1, P2, m2, KB, nbv, N1v, N2v, T, L, blocks, *ps)
      if (NNT == 1) {
        if (aligned) CDP(1, true); else CDP(1, false);
      } else {
        if (aligned) CDP(2, true); else CDP(2, false);
      }
#undef CDP
      return (int)hipGetLastError();
    }
  }
#define CDK(NNT_, AL_)                                                                         \
  rowdft_cd_kernel<NNT_, AL_, LIFT, BDZ><<<blocks, 64 * kCdWaves, sh, st>>>(                   \
      x, idx, part, Tp, tab, Bn, C, P1, P2, m2, KB, nbv, N1v, N2v, act, T, L, ghat, lw)
  if (NNT == 1) {
    if (aligned) CDK(1, true); else CDK(1, false);
  } else {
    if (aligned) CDK(2, true); else CDK(2, false);
  }
#undef CDK
  return (int)hipGetLastError();
}

}  // namespace

// Row DFT of f(x) (f = GELU when act; x read on its N1v x N2v valid region) with the column DFT
// of each 16-row block written as partials (colspec.h layout, NCH = blindno_colspec_nchunk(C,
// m2) chunks per block; blocks at or past ceil(N1v / 16) are not written).  Tp: the row-DFT
// image (blindno_rowdft's), tab: Tab[P1][2 K1].  K1 = 24 (m1 = 12).
BLINDNO_API int blindno_rowdft_cd(const float* x, float* part, const float* Tp, const float* tab,
                                  int Bn, int C, int P1, int P2, int m2, int act, int N1v, int N2v,
                                  void* stream) {
  if (!x || !part || !Tp || !tab || !cd_geom_ok(Bn, C, P1, P2, m2) || N1v < 1 || N1v > P1 ||
      N2v < 1 || N2v > P2)
    return (int)hipErrorInvalidValue;
  return rowdft_cd_launch<false>(x, nullptr, part, Tp, tab, Bn, C, P1, P2, m2, act, N1v, N2v, 0, 1,
                                 (hipStream_t)stream);
}

// blindno_rowdft_cd of the encoder's last-layer gradient dz = lw_l ghat v formed on load (v from
// blindno_project_bag_fwd, ghat (B, Ho Wo), lw (U, NULL: 1 / U); Bn = B U; act 0; crop Ho x Wo)
BLINDNO_API int blindno_rowdft_cd_bag(const float* v, const float* ghat, const float* lw, int U,
                                      float* part, const float* Tp, const float* tab, int Bn, int C,
                                      int P1, int P2, int m2, int Ho, int Wo, void* stream) {
  if (!v || !ghat || !part || !Tp || !tab || U < 1 || Bn % U || !cd_geom_ok(Bn, C, P1, P2, m2) ||
      Ho < 1 || Ho > P1 || Wo < 1 || Wo > P2)
    return (int)hipErrorInvalidValue;
  return rowdft_cd_launch<false, true>(v, nullptr, part, Tp, tab, Bn, C, P1, P2, m2, 0, Ho, Wo, 0, U,
                                       (hipStream_t)stream, ghat, lw);
}

// The snapshot encoder's first stage: row DFT + column-DFT partials of the bag's snapshots
// X[b][idx[l]] (B, T, N1, N2), one channel, zero-padded to P1 x P2 (sample n = b L + l).
BLINDNO_API int blindno_rowdft_bag_lift_cd(const float* X, const int* idx, float* part,
                                           const float* Tp, const float* tab, int B, int T, int L,
                                           int N1, int N2, int P1, int P2, int m2, void* stream) {
  if (!X || !idx || !part || !Tp || !tab || B <= 0 || L <= 0 || T <= 0 || N1 < 1 || N1 > P1 ||
      N2 < 1 || N2 > P2 || !cd_geom_ok(B * L, 1, P1, P2, m2) ||
      (int64_t)B * T * N1 * N2 >= ((int64_t)1 << 40))
    return (int)hipErrorInvalidValue;
  return rowdft_cd_launch<true>(X, idx, part, Tp, tab, B * L, 1, P1, P2, m2, 0, N1, N2, T, L,
                                (hipStream_t)stream);
}

// blindno_rowdft_bag_lift_cd with blindno_pack_w2d_multi(w1s, w2s, Wts, shapes, npk) (the
// forward's spectral-weight pack; independent of it) hosted in the same launch; two launches
// when the pack does not take the tiled path or does not fit one segment table.
BLINDNO_API int blindno_rowdft_bag_lift_cd_pack(const float* X, const int* idx, float* part,
                                                const float* Tp, const float* tab, int B, int T,
                                                int L, int N1, int N2, int P1, int P2, int m2,
                                                const void* const* w1s, const void* const* w2s,
                                                void* const* Wts, const int* shapes, int npk,
                                                void* stream) {
  if (!X || !idx || !part || !Tp || !tab || B <= 0 || L <= 0 || T <= 0 || N1 < 1 || N1 > P1 ||
      N2 < 1 || N2 > P2 || !cd_geom_ok(B * L, 1, P1, P2, m2) ||
      (int64_t)B * T * N1 * N2 >= ((int64_t)1 << 40) || npk < 0)
    return (int)hipErrorInvalidValue;
  PackSegs ps{};
  int64_t ntr = 0;
  bool host = npk > 0 && npk <= kPackSegs;
  if (host) {
    ps.nseg = npk;
    for (int i = 0; i < npk; ++i) {
      const int* sh = shapes + 5 * i;
      if (sh[2] > sh[4] || sh[0] < 1 || sh[1] < 1 || sh[2] < 1 || sh[3] < 1 || !w1s[i] ||
          !w2s[i] || !Wts[i] ||
          (int64_t)sh[3] * 2 * sh[2] * sh[0] * sh[1] >= INT32_MAX)
        return (int)hipErrorInvalidValue;
      ps.w1[i] = (const float*)w1s[i];
      ps.w2[i] = (const float*)w2s[i];
      ps.Wt[i] = (float2*)Wts[i];
      ps.Ci[i] = sh[0]; ps.Co[i] = sh[1]; ps.m1[i] = sh[2]; ps.m2[i] = sh[3]; ps.P1[i] = sh[4];
    }
    host = w2d_tiled_segs(ps, ntr) && ntr > 0;
  }
  if (!host && npk > 0) {
    const int e = blindno_pack_w2d_multi(w1s, w2s, Wts, shapes, npk, stream);
    if (e) return e;
  }
  return rowdft_cd_launch<true>(X, idx, part, Tp, tab, B * L, 1, P1, P2, m2, 0, N1, N2, T, L,
                                (hipStream_t)stream, nullptr, nullptr, host ? &ps : nullptr,
                                host ? (int)ntr : 0);
}

// The column pass's mix stage on the block partials (see colmix_kernel): part holds Cp-channel
// partials of nbv blocks per sample (stride P1 / 16 blocks); Xsave (Bn, m2, C, K1) complex,
// Y (Bn, m2, C, K1) complex; Wt (m2, K1, C, C) complex (blindno_pack_w2d) or NULL (Xsave only).
// dir 0 forward, 1 adjoint.  w0 / b0 / Dg2 (LIFT, dir 0, Cp = 1): fc0's weight (C, 3), bias (C)
// and the grid planes' spectrum Dg2 (m2, 3, K1) complex.
BLINDNO_API int blindno_colmix(const float* part, int nbv, const float* Wt, float* Xsave, float* Y,
                               int Bn, int C, int Cp, int P1, int P2, int m1, int m2, int dir,
                               const float* w0, const float* b0, const float* Dg2, void* stream) {
  const bool lift = w0 != nullptr;
  if (!part || Bn <= 0 || C <= 0 || C > 16 || m2 <= 0 || m2 > 16 || m1 != 12 ||
      kept_rows_count(m1, P1) != kCsK1 || P1 % 16 || nbv < 1 || nbv > P1 / 16 ||
      (Wt && !Y) || (!Wt && !Xsave) || (lift && (Cp != 1 || !b0 || !Dg2 || dir != 0)) ||
      (!lift && Cp != C))
    return (int)hipErrorInvalidValue;
  if (P1 / 16 > kMixMaxB) return (int)hipErrorInvalidValue;
  const size_t sh = sizeof(float2) * (size_t)m2 * kMixJ * (Cp + (lift ? C : 0) + (Wt ? C * C : 0));
  hipStream_t st = (hipStream_t)stream;
  const float2* W = (const float2*)Wt;
#define CM(D_, L_)                                                                             \
  colmix_kernel<D_, L_><<<Bn * kCsMT2, kMixThreads, sh, st>>>(                                 \
      part, nbv, W, (float2*)Xsave, (float2*)Y, C, Cp, P1, P2, m2, w0, b0, (const float2*)Dg2)
  if (lift) CM(0, true);
  else if (dir == 0) CM(0, false);
  else CM(1, false);
#undef CM
  return (int)hipGetLastError();
}
