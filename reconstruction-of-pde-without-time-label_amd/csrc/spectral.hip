// Truncated spectral transforms and per-mode channel mixing for SpectralConv1d/2d.
//
// Reference operation (yl602019618/Reconstruction-of-PDE-without-Time-Label):
//   SpectralConv2d.forward  2d_FPE/FNOModules.py:156-178  (rfft2 -> compl_mul2d on the two
//   kept corner blocks -> irfft2(s=(H,W)));  SpectralConv1d.forward 1d_FPE/FNOModules.py:47-59
//   (rfft -> DC*0.5 -> einsum bix,iox->box -> irfft).
// The FFTs are evaluated as truncated DFTs: only m2 column modes and K1 kept rows are ever
// formed.  The big, HBM-streaming stages are the row transforms (this file: forward row DFT;
// fields.hip: inverse row DFT + epilogue); the column transforms and the mix work on the
// m2/P2-sized row spectra and run one workgroup per (sample, column mode).
#include "common.h"
#include "blindno.h"
#include "kernels.h"
#include "wgrad.h"
#include "packw.h"

using namespace blindno;


namespace {

// ------------------------------------------------------------------------------ row DFT
// At[n][k][c][h] = sum_w f(x[n][c][h][w]) e^{-2 pi i k w / P2} as a skinny GEMM on the f32
// matrix cores: out (rows x 2*m2, re/im interleaved) = X (rows x P2) . T (P2 x 2*m2), with
// T[w][2k] = cos(2 pi k w/P2), T[w][2k+1] = -sin(2 pi k w/P2).
// v_mfma_f32_16x16x4f32: one wave owns a 16-row tile and NT 16-column tiles.  The A operand
// streams straight from HBM: lane l loads float4 x[row l&15][16 kb + 4 (l>>4) .. +3] and uses
// component s in MFMA step s, i.e. the k-order inside each 16-block is permuted
// (k = 16 kb + 4 (l>>4) + s); the B operand follows the same permutation from an LDS image
// Tp[kb][kq][n][s] so that one ds_read_b128 returns the four steps' twiddles of one column.
// f = GELU (act) is applied once per loaded element (VALU, beside the matrix pipe).
typedef float f32x4 __attribute__((ext_vector_type(4)));

// workgroup cap of the row DFT grid (each workgroup stages the twiddle image once; beyond the
// cap waves loop over several 16-row tiles)
#ifndef ROWDFT_MAX_BLOCKS
#define ROWDFT_MAX_BLOCKS 4096
#endif
// work items the row DFT aims at when splitting a row tile's column tiles over waves
#ifndef ROWDFT_MIN_WORK
#define ROWDFT_MIN_WORK 512
#endif
#ifndef ROWDFT_STAGE_ITEMS
#define ROWDFT_STAGE_ITEMS 1
#endif
// Valid region (N1v, N2v): only rows h < N1v and columns w < N2v of each P1 x P2 plane are
// read, the rest counts as zero -- for the gradient of a cropped FNO output (2d_FPE/
// FNOModules.py:234), which is zero on the padding by construction, so the producer
// (project_bwd) need not zero-fill it; KB then covers only the ceil(N2v / 16) live K blocks.
// STAGE: the twiddle image is staged in LDS by every workgroup; otherwise the B operands are
// read from the global image (L1/L2-resident) -- when each wave runs about one work item the
// staging is as many bytes as the wave's own x rows and costs a full latency up front.
// (the body takes its workgroup index bx of gx explicitly: rowdft_wgrad_kernel below hosts it
// beside other work in one launch)
template <int NT, int ALIGNED, bool STAGE>
__device__ __forceinline__ void rowdft_mfma_block(const float* __restrict__ x,
                                                  float* __restrict__ At,
                                                  const float* __restrict__ Tp, int nrows, int C,
                                                  int P1, int P2, int m2, int KB, int Npad,
                                                  int ntile_groups, int act, int N1v, int N2v,
                                                  int bx, int gx) {
  extern __shared__ float smT[];                 // [KB][4][Npad][4]
  if constexpr (STAGE) {
    const int nT = KB * 16 * Npad;
    stage_to_lds(smT, Tp, nT);
    __syncthreads();
  }
  const float* __restrict__ tsrc = STAGE ? smT : Tp;
  const int lane = threadIdx.x & 63;
  const int wave = uniform_int(threadIdx.x >> 6);
  const int r16 = lane & 15, kq = lane >> 4;
  const int nrt = (nrows + 15) >> 4;
  const int64_t nwork = (int64_t)nrt * ntile_groups;
  for (int64_t wk = (int64_t)bx * 4 + wave; wk < nwork; wk += (int64_t)gx * 4) {
    const int rt = (int)(wk / ntile_groups);
    const int tg = (int)(wk % ntile_groups);
    const int t0 = tg * NT;                       // first 16-column tile of this wave
    const int row = rt * 16 + r16;
    const bool rok = row < nrows && (N1v >= P1 || row % P1 < N1v);
    const float* xr = x + (int64_t)(rok ? row : 0) * P2;
    f32x4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
    // x loads run two K blocks ahead of the MFMAs (small fields are latency-bound)
    auto load_a = [&](int kb, float (&a)[4]) {
      const int w0 = kb * 16 + kq * 4;
      if (ALIGNED && w0 + 3 < N2v) {
        const float4 v = rok ? *reinterpret_cast<const float4*>(xr + w0) : make_float4(0.f, 0.f, 0.f, 0.f);
        a[0] = v.x; a[1] = v.y; a[2] = v.z; a[3] = v.w;
      } else {
#pragma unroll
        for (int s = 0; s < 4; ++s) a[s] = (rok && w0 + s < N2v) ? xr[w0 + s] : 0.f;
      }
    };
    float a1[4], a2[4] = {0.f, 0.f, 0.f, 0.f};
    load_a(0, a1);
    if (KB > 1) load_a(1, a2);
    for (int kb = 0; kb < KB; ++kb) {
      float a[4] = {a1[0], a1[1], a1[2], a1[3]};
#pragma unroll
      for (int s = 0; s < 4; ++s) a1[s] = a2[s];
      if (kb + 2 < KB) load_a(kb + 2, a2);
      if (act) {
#pragma unroll
        for (int s = 0; s < 4; ++s) a[s] = gelu_f(a[s]);
      }
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const f32x4 b = *reinterpret_cast<const f32x4*>(
            tsrc + (((kb * 4 + kq) * Npad) + (t0 + t) * 16 + r16) * 4);
#pragma unroll
        for (int s = 0; s < 4; ++s)
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], b[s], acc[t], 0, 0, 0);
      }
    }
    // D layout: lane holds rows 4*(l>>4) + r (r < 4), column l & 15
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int col = (t0 + t) * 16 + r16;
      const int k = col >> 1, part = col & 1;
      if (k >= m2) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int orow = rt * 16 + kq * 4 + r;
        if (orow >= nrows) continue;
        const int h = orow % P1;
        const int nc = orow / P1;
        const int c = nc % C;
        const int n = nc / C;
        At[((((int64_t)n * m2 + k) * C + c) * P1 + h) * 2 + part] = acc[t][r];
      }
    }
  }
}

template <int NT, int ALIGNED, bool STAGE>
__global__ __launch_bounds__(256) void rowdft_mfma_kernel(const float* __restrict__ x,
                                                          float* __restrict__ At,
                                                          const float* __restrict__ Tp,
                                                          int nrows, int C, int P1, int P2,
                                                          int m2, int KB, int Npad, int ntile_groups,
                                                          int act, int N1v, int N2v) {
  rowdft_mfma_block<NT, ALIGNED, STAGE>(x, At, Tp, nrows, C, P1, P2, m2, KB, Npad, ntile_groups,
                                        act, N1v, N2v, blockIdx.x, gridDim.x);
}

// Row DFT of the first FNO layer of the snapshot encoder with the lift folded in.  The lifted
// field x0[n][c][h][w] = W0[c,0] u[n][h][w] + W0[c,1] gx[h][w] + W0[c,2] gy[h][w] + b0[c]
// (zero-padded to P1 x P2; 2d_FPE/FNOModules.py:219-224) is affine in the snapshot u, and the
// DFT is linear, so
//     At[n][k][c][h] = W0[c,0] U[n][k][h] + Gt[k][c][h],   U = rowDFT(u),
// with Gt = rowDFT of the grid/bias part (one sample, computed once per forward).  Only the
// 1-channel snapshot is transformed, and it is read straight out of the bag tensor
// X (B, T, N1, N2) through the bag's index list (snapshot n = b L + l -> X[b][idx[l]]), so
// neither the gathered bag, the concatenated input nor x0 is ever materialised.
template <int NT, int ALIGNED>
// b0 != nullptr: Gt holds the row spectra Dg[k][j][h] of the three grid/bias planes (gx, gy,
// 1 on the crop) instead, and the grid/bias part is formed here as
// W0[c,1] Dg[k][0] + W0[c,2] Dg[k][1] + b0[c] Dg[k][2] (Dg depends on the grid only, so it is
// computed once; fc0 is trained, so a precomputed Gt would not be).
__global__ __launch_bounds__(256) void rowdft_bag_lift_kernel(
    const float* __restrict__ X, const int* __restrict__ idx, const float* __restrict__ w0,
    const float* __restrict__ b0, const float* __restrict__ Gt, float* __restrict__ At,
    const float* __restrict__ Tp, int nrows, int T, int L, int N1, int N2, int C, int P1, int m2,
    int KB, int Npad, int ntile_groups) {
  extern __shared__ float smT[];                 // [KB][4][Npad][4]
  const int nT = KB * 16 * Npad;
  stage_to_lds(smT, Tp, nT);
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int wave = uniform_int(threadIdx.x >> 6);
  const int r16 = lane & 15, kq = lane >> 4;
  const int nrt = (nrows + 15) >> 4;
  const int64_t nwork = (int64_t)nrt * ntile_groups;
  for (int64_t wk = (int64_t)blockIdx.x * 4 + wave; wk < nwork; wk += (int64_t)gridDim.x * 4) {
    const int rt = (int)(wk / ntile_groups);
    const int tg = (int)(wk % ntile_groups);
    const int t0 = tg * NT;
    const int row = rt * 16 + r16;
    const int n = row / P1, h = row - (row / P1) * P1;
    const bool rok = row < nrows && h < N1;
    const float* xr = X;
    if (rok) {
      const int b = n / L, l = n - (n / L) * L;
      xr = X + (((int64_t)b * T + idx[l]) * N1 + h) * N2;
    }
    f32x4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
    auto load_a = [&](int kb, float (&a)[4]) {
      const int w0c = kb * 16 + kq * 4;
      if (ALIGNED && w0c + 3 < N2) {
        const float4 v = rok ? *reinterpret_cast<const float4*>(xr + w0c) : make_float4(0.f, 0.f, 0.f, 0.f);
        a[0] = v.x; a[1] = v.y; a[2] = v.z; a[3] = v.w;
      } else {
#pragma unroll
        for (int s = 0; s < 4; ++s) a[s] = (rok && w0c + s < N2) ? xr[w0c + s] : 0.f;
      }
    };
    auto mma = [&](int kb, const float (&a)[4]) {
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const f32x4 bt = *reinterpret_cast<const f32x4*>(smT + (((kb * 4 + kq) * Npad) + (t0 + t) * 16 + r16) * 4);
#pragma unroll
        for (int s = 0; s < 4; ++s) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], bt[s], acc[t], 0, 0, 0);
      }
    };
    for (int kb = 0; kb < KB; ++kb) {
      float a[4];
      load_a(kb, a);
      mma(kb, a);
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int col = (t0 + t) * 16 + r16;
      const int k = col >> 1, part = col & 1;
      if (k >= m2) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int orow = rt * 16 + kq * 4 + r;
        if (orow >= nrows) continue;
        const int on = orow / P1, oh = orow - (orow / P1) * P1;
        const float u = acc[t][r];
        float dg0 = 0.f, dg1 = 0.f, dg2 = 0.f;
        if (b0) {
          const int64_t di = (((int64_t)k * 3) * P1 + oh) * 2 + part;
          dg0 = Gt[di];
          dg1 = Gt[di + 2 * P1];
          dg2 = Gt[di + 4 * P1];
        }
        for (int c = 0; c < C; ++c) {
          float g;
          if (b0) {
            g = fmaf(w0[c * 3 + 1], dg0, fmaf(w0[c * 3 + 2], dg1, b0[c] * dg2));
          } else {
            g = Gt[(((int64_t)k * C + c) * P1 + oh) * 2 + part];
          }
          At[((((int64_t)on * m2 + k) * C + c) * P1 + oh) * 2 + part] = fmaf(w0[c * 3], u, g);
        }
      }
    }
  }
}

// ------------------------------------------------------------------------------ column pass
// The column transforms are two complex GEMMs against the shared twiddle matrix
// F[h][j] = e^{-2 pi i r_j h / P1} (r_j the K1 kept frequency rows), on the f32 matrix cores
// (v_mfma_f32_16x16x4f32, four real MFMAs per complex step), with the per-mode channel mix
// fused behind the first one:
//   coldft_mix:  X[q][c][j] = sum_h At[q][c][h] F[h][j]          (q = n m2 + k, the pair)
//                DIR 0: Xs = X (saved),        Y[q][o][j] = c_k/(P1 P2) sum_c X W[k][j][c][o]
//                DIR 1: Xs = c_k/(P1 P2) X = G, Y[q][i][j] = sum_o conj(W[k][j][i][o]) G
//   colidft:     Z[n][h][k][o] = sum_j Y[q][o][j] conj(F[h][j])
// Y is a K1p = 16 ceil(K1/16) padded scratch spectrum.  Both GEMMs take their B operand from
// host-built twiddle images in MFMA lane order (one 32-byte load per lane and k-block) and
// permute the k order inside each 16-block exactly like the row DFT (k = 16 kb + 4 kq + s),
// so every lane streams 4 consecutive complex A values.
typedef float f32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void cmfma4(const float (&ar)[4], const float (&ai)[4],
                                       const f32x4& b0, const f32x4& b1, f32x4& dr, f32x4& di) {
  const float br[4] = {b0.x, b0.z, b1.x, b1.z};
  const float bi[4] = {b0.y, b0.w, b1.y, b1.w};
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    dr = __builtin_amdgcn_mfma_f32_16x16x4f32(ar[s], br[s], dr, 0, 0, 0);
    dr = __builtin_amdgcn_mfma_f32_16x16x4f32(-ai[s], bi[s], dr, 0, 0, 0);
    di = __builtin_amdgcn_mfma_f32_16x16x4f32(ar[s], bi[s], di, 0, 0, 0);
    di = __builtin_amdgcn_mfma_f32_16x16x4f32(ai[s], br[s], di, 0, 0, 0);
  }
}

// 4 consecutive complex values src[0..3] (zero past len) split into re / im
__device__ __forceinline__ void load4c(const float2* src, int len, bool vec, float (&re)[4],
                                       float (&im)[4]) {
  if (vec && len >= 4) {
    const f32x4 v0 = *reinterpret_cast<const f32x4*>(src);
    const f32x4 v1 = *reinterpret_cast<const f32x4*>(src + 2);
    re[0] = v0.x; im[0] = v0.y; re[1] = v0.z; im[1] = v0.w;
    re[2] = v1.x; im[2] = v1.y; re[3] = v1.z; im[3] = v1.w;
  } else {
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const float2 v = s < len ? src[s] : make_float2(0.f, 0.f);
      re[s] = v.x;
      im[s] = v.y;
    }
  }
}

// FULL: every h block's operands are loaded before the first MFMA (HB <= kFullHB): the head
// layers launch one workgroup per (sample, mode) pair -- one wave per SIMD -- so a one-block
// lookahead leaves each step waiting a full memory latency (measured ~16 us for 10 steps)
constexpr int kFullHB = 10;
// unroll of the mix's input-channel loop (weight loads in flight per output)
#ifndef COLMIX_UNROLL
#define COLMIX_UNROLL 4
#endif
// 16-row DFT tiles a column-pass workgroup aims at (pairs per workgroup grow until reached)
#ifndef COLPASS_WAVE_TILES
#define COLPASS_WAVE_TILES 4
#endif
#ifndef COLMIX_C12
#define COLMIX_C12 1
#endif
#ifndef COLFUSE_C12
#define COLFUSE_C12 1
#endif
// H16 (config E, blindno.ops.set_mix_precision("fp16")): the channel mix takes fp16 operands
// with fp32 accumulation -- each complex multiply-add is two v_dot2c_f32_f16 (packed fp16
// pairs, exact products, fp32 sum).  The column spectra are block-scaled first: the workgroup's
// largest |Re|, |Im| is brought to [2^14, 2^15) by an exact power of two, undone after the sum,
// so neither the unnormalised forward spectra (up to P1 P2 |x|) overflow fp16 nor the small
// gradient spectra of the adjoint flush to zero.  The weights are converted unscaled (their
// magnitudes sit far inside fp16's normal range).  Not on the matrix cores: the mix is a
// batch of complex GEMVs (one Ci x Co matrix per kept mode, one row per sample), which would
// fill a quarter of an MFMA tile at best.
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
template <int DIR, bool FULL, bool H16>
__global__ __launch_bounds__(256) void coldft_mix_kernel(const float2* __restrict__ At,
                                                         const float2* __restrict__ Wt,
                                                         const f32x4* __restrict__ FB,
                                                         float2* __restrict__ Xs,
                                                         float2* __restrict__ Y, int npairs,
                                                         int Ci, int Co, int P1, int m1, int m2,
                                                         int P2, int G, int vec, int Bg,
                                                         int64_t wtgs) {
  // grouped launches: samples n of weight group n / Bg use Wt + (n / Bg) wtgs (in floats)
  extern __shared__ float2 sX[];                  // [G Cin][K1p + 1]
  const int K1 = kept_rows_count(m1, P1);
  const int Jt = (K1 + 15) >> 4, K1p = Jt * 16, LDX = K1p + 1;
  const int Cin = DIR == 0 ? Ci : Co;
  const int Cout = DIR == 0 ? Co : Ci;
  const int HB = (P1 + 15) >> 4;
  const int q0 = blockIdx.x * G;
  const int np = min(G, npairs - q0);
  const int rows = np * Cin;
  const int Mt = (rows + 15) >> 4;
  const int lane = threadIdx.x & 63;
  const int wave = uniform_int(threadIdx.x >> 6);
  const int r16 = lane & 15, kq = lane >> 4;
  const float inv = 1.0f / ((float)P1 * (float)P2);
  const int nout = np * Cout * K1p;

  // weights of output e = (p, j, o), o fastest: W[k][j][c][o] (DIR 0) / W[k][j][o][c] (DIR 1)
  auto wrow = [&](int e, int& o, int& j, int& p, int& k) -> const float2* {
    o = e % Cout;
    const int t = e / Cout;
    j = t % K1p;
    p = t / K1p;
    k = (q0 + p) % m2;
    const float2* wg = wtgs ? reinterpret_cast<const float2*>(
                                  reinterpret_cast<const float*>(Wt) + ((q0 + p) / m2 / Bg) * wtgs)
                            : Wt;
    return wg + ((int64_t)k * K1 + (j < K1 ? j : 0)) * Ci * Co;
  };
  for (int item = wave; item < Mt * Jt; item += 4) {
    const int mt = item / Jt, jt = item % Jt;
    const int row = mt * 16 + r16;
    const bool rok = row < rows;
    const float2* ar = At + ((int64_t)q0 * Cin + (rok ? row : 0)) * P1;
    const f32x4* fb = FB + ((int64_t)jt * HB * 64 + lane) * 2;
    f32x4 dr = {0.f, 0.f, 0.f, 0.f}, di = {0.f, 0.f, 0.f, 0.f};
    if constexpr (FULL) {
      float are[kFullHB][4], aim[kFullHB][4];
      f32x4 af0[kFullHB], af1[kFullHB];
#pragma unroll
      for (int hb = 0; hb < kFullHB; ++hb) {
        if (hb < HB) {
          const int h1 = hb * 16 + kq * 4;
          load4c(ar + h1, rok ? P1 - h1 : 0, vec, are[hb], aim[hb]);
          af0[hb] = fb[hb * 128];
          af1[hb] = fb[hb * 128 + 1];
        }
      }
#pragma unroll
      for (int hb = 0; hb < kFullHB; ++hb)
        if (hb < HB) cmfma4(are[hb], aim[hb], af0[hb], af1[hb], dr, di);
    } else {
      // operands of the next 16-row block are loaded before this block's MFMAs
      float nre[4], nim[4];
      load4c(ar + kq * 4, rok ? P1 - kq * 4 : 0, vec, nre, nim);
      f32x4 nf0 = fb[0], nf1 = fb[1];
      for (int hb = 0; hb < HB; ++hb) {
        float re[4], im[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) { re[s] = nre[s]; im[s] = nim[s]; }
        const f32x4 f0 = nf0, f1 = nf1;
        if (hb + 1 < HB) {
          const int h1 = (hb + 1) * 16 + kq * 4;
          load4c(ar + h1, rok ? P1 - h1 : 0, vec, nre, nim);
          nf0 = fb[(hb + 1) * 128];
          nf1 = fb[(hb + 1) * 128 + 1];
        }
        cmfma4(re, im, f0, f1, dr, di);
      }
    }
    const int j = jt * 16 + r16;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int orow = mt * 16 + kq * 4 + r;
      if (orow >= rows) continue;
      float sc = 1.0f;
      if (DIR == 1) sc = c2r_weight((q0 + orow / Cin) % m2, P2) * inv;
      const float2 v = make_float2(dr[r] * sc, di[r] * sc);
      sX[orow * LDX + j] = v;
      if (j < K1) Xs[((int64_t)q0 * Cin + orow) * K1 + j] = v;
    }
  }
  __syncthreads();

  // H16: block scale 2^e with max |component| * 2^e in [2^14, 2^15)
  float hs = 1.0f, hinv = 1.0f;
  if constexpr (H16) {
    __shared__ float smax[4];
    float mx = 0.f;
    for (int e = threadIdx.x; e < rows * K1p; e += blockDim.x) {
      const float2 v = sX[(e / K1p) * LDX + e % K1p];
      mx = fmaxf(mx, fmaxf(fabsf(v.x), fabsf(v.y)));
    }
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) mx = fmaxf(mx, __shfl_xor(mx, m, 64));
    if (lane == 0) smax[wave] = mx;
    __syncthreads();
    mx = fmaxf(fmaxf(smax[0], smax[1]), fmaxf(smax[2], smax[3]));
    if (mx > 0.f && mx < 3.0e38f) {
      int ex;
      frexpf(mx, &ex);                            // mx in [2^(ex-1), 2^ex)
      hs = ldexpf(1.0f, 15 - ex);
      hinv = ldexpf(1.0f, ex - 15);
    }
  }

  // the mix: output channel o fastest across threads, so the weight loads W[k][j][c][o] of
  // neighbouring threads are contiguous (j fastest put every lane on its own cache line)
  auto mix_one = [&](int e) {
    int o, j, p, k;
    const float2* wj = wrow(e, o, j, p, k);
    float re = 0.f, im = 0.f;
    if (j < K1) {
      const float2* xp = sX + p * Cin * LDX + j;
      auto wload = [&](int c) -> float2 { return DIR == 0 ? wj[c * Co + o] : wj[o * Co + c]; };
      if constexpr (H16) {
#pragma unroll 4
        for (int c = 0; c < Cin; ++c) {
          const float2 a = xp[c * LDX];
          const f16x2 ah = {(_Float16)(a.x * hs), (_Float16)(a.y * hs)};
          const float2 w = wload(c);
          const _Float16 wr = (_Float16)w.x, wi = (_Float16)w.y;
          if (DIR == 0) {                             // a w
            re = __builtin_amdgcn_fdot2(ah, (f16x2){wr, (_Float16)(-wi)}, re, false);
            im = __builtin_amdgcn_fdot2(ah, (f16x2){wi, wr}, im, false);
          } else {                                    // conj(w) a
            re = __builtin_amdgcn_fdot2(ah, (f16x2){wr, wi}, re, false);
            im = __builtin_amdgcn_fdot2(ah, (f16x2){(_Float16)(-wi), wr}, im, false);
          }
        }
        re *= hinv;
        im *= hinv;
      } else {
        auto mac = [&](int c) {
          const float2 a = xp[c * LDX];
          const float2 w = wload(c);
          if (DIR == 0) {
            re = fmaf(a.x, w.x, fmaf(-a.y, w.y, re));
            im = fmaf(a.x, w.y, fmaf(a.y, w.x, im));
          } else {                                    // conj(w) * a
            re = fmaf(w.x, a.x, fmaf(w.y, a.y, re));
            im = fmaf(w.x, a.y, fmaf(-w.y, a.x, im));
          }
        };
        if (COLMIX_C12 && Cin == 12) {
          // the 12-channel heads: every weight load of the output in flight at once (the
          // small head launches are bound by these L2 round trips; same summation order)
#pragma unroll
          for (int c = 0; c < 12; ++c) mac(c);
        } else {
#pragma unroll COLMIX_UNROLL
          for (int c = 0; c < Cin; ++c) mac(c);
        }
      }
      if (DIR == 0) {
        const float sc = c2r_weight(k, P2) * inv;
        re *= sc;
        im *= sc;
      }
    }
    Y[((int64_t)(q0 + p) * Cout + o) * K1p + j] = make_float2(re, im);
  };
  for (int e = threadIdx.x; e < nout; e += blockDim.x) mix_one(e);
}

// The fused column pass (default for fp32 mixes of up to 16 channels and K1 <= 64 kept rows):
// coldft_mix + colidft in ONE workgroup per 16-row M tile (G = 16 / Cin (sample, mode) pairs of
// Cin channels), so the spectrum Y never leaves LDS and each layer pays one launch:
//   1. column DFT X = At F on the matrix cores; the 4 waves split the K1p / 16 column tiles and,
//      when there are fewer than 4 tiles, the P1 rows into KS chunks (partials summed in LDS,
//      fixed order); every chunk's operands are loaded before its first MFMA;
//   2. the per-mode channel mix (as coldft_mix) from LDS into LDS;
//   3. column inverse Z = Y conj(F) on the matrix cores, the 4 waves over the P1 / 16 row tiles.
// Same twiddle images (FB, GB) and the same summation order within each K chunk as the split
// kernels; Xs (the saved spectrum) is written as before, Y is not.
// NW waves per workgroup: 8 for the small head launches (one (sample, mode) pair of 12 channels
// per workgroup and only Bn m2 of them: with 4 waves the chip runs one wave per SIMD)
// H16: the fp16-operand mix of coldft_mix (config E), block-scaled over this workgroup's rows
#ifndef COLFUSE_PROBE
#define COLFUSE_PROBE 0
#endif
#ifndef COLFUSE_PREFETCH
#define COLFUSE_PREFETCH 1
#endif
#if COLFUSE_PROBE
// diagnostic build only (tools/probe_colfuse.py): per-wave realtime stamps at the phase edges
__device__ unsigned long long g_colfuse_probe[4096 * 8];
#define CF_MARK(i)                                                                          \
  do {                                                                                      \
    __builtin_amdgcn_sched_barrier(0);                                                      \
    const unsigned long long t_ = __builtin_amdgcn_s_memrealtime();                         \
    const int slot_ = blockIdx.x * NW + (threadIdx.x >> 6);                                 \
    if ((threadIdx.x & 63) == 0 && slot_ < 4096) g_colfuse_probe[slot_ * 8 + (i)] = t_;     \
    __builtin_amdgcn_sched_barrier(0);                                                      \
  } while (0)
#else
#define CF_MARK(i) do {} while (0)
#endif
template <int DIR, int HBC, int NW = 4, bool H16 = false>
__global__ __launch_bounds__(64 * NW) void colfuse_kernel(const float2* __restrict__ At,
                                                      const float2* __restrict__ Wt,
                                                      const f32x4* __restrict__ FB,
                                                      const f32x4* __restrict__ GB,
                                                      float2* __restrict__ Xs,
                                                      float2* __restrict__ Z, int npairs, int Ci,
                                                      int Co, int P1, int m1, int m2, int P2, int G,
                                                      int KS, int vec, int Bg, int64_t wtgs,
                                                      int tiled) {
  constexpr int kLd = 65;                          // LDS row stride (float2) for K1p <= 64
  constexpr int kLdP = 16 * NW + 1;                 // DFT partials: KS K1p <= 16 NW
  constexpr int kT = 64 * NW;
  CF_MARK(7);
  // DFT partials, chunk kc in columns [kc K1p, (kc + 1) K1p), then Y
  __shared__ float2 sP[16][kLdP];
  __shared__ float2 sX[16][kLd];
  const int K1 = kept_rows_count(m1, P1);
  const int Jt = (K1 + 15) >> 4, K1p = Jt * 16;
  const int Cin = DIR == 0 ? Ci : Co;
  const int Cout = DIR == 0 ? Co : Ci;
  const int HB = (P1 + 15) >> 4;
  const int q0 = blockIdx.x * G;
  const int np = min(G, npairs - q0);
  const int rows = np * Cin, orows = np * Cout;
  const int lane = threadIdx.x & 63;
  const int wave = uniform_int(threadIdx.x >> 6);
  const int r16 = lane & 15, kq = lane >> 4;
  const float inv = 1.0f / ((float)P1 * (float)P2);
  CF_MARK(0);

  // PF (the 8-wave head launches): the mix weights and the column inverse's twiddles are
  // loaded here, in flight together with the column DFT's operands.  Each phase otherwise
  // opened with its own round trip to L2 / MALL at the start of the kernel (per-wave phase
  // stamps, tools/probe_colfuse.py: mix 1.8 us, inverse 4-5.7 us of a 13 us wave)
  constexpr bool PF = COLFUSE_PREFETCH && NW == 8 && HBC <= 5 && !H16;   // 239 VGPRs at HBC 5
  const bool c12 = COLFUSE_C12 && !H16 && Cin == 12 && Cout == 12 && 16 * K1p <= 2 * kT && np == 1;
  constexpr int kC = 12;
  float2 wv[2][kC];
  int jv[2], ov[2];
  bool live[2];
  auto load_mix_weights = [&]() {
    const int k = q0 % m2;
    const float2* wg = wtgs ? reinterpret_cast<const float2*>(
                                  reinterpret_cast<const float*>(Wt) + (q0 / m2 / Bg) * wtgs)
                            : Wt;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int e = threadIdx.x + i * kT;
      ov[i] = e % kC;
      const int t = e / kC;
      jv[i] = t % K1p;
      live[i] = e < 16 * K1p && t < K1p && jv[i] < K1;      // p == 0 (one pair)
      const float2* wj = wg + ((int64_t)k * K1 + (live[i] ? jv[i] : 0)) * kC * kC;
#pragma unroll
      for (int c = 0; c < kC; ++c) wv[i][c] = DIR == 0 ? wj[c * kC + ov[i]] : wj[ov[i] * kC + c];
    }
  };
  f32x4 pg0[2][4], pg1[2][4];
  if constexpr (PF) {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int ht = wave + t * NW;
      if (ht < HB) {
        const f32x4* gb = GB + ((int64_t)ht * Jt * 64 + lane) * 2;
#pragma unroll
        for (int jb = 0; jb < 4; ++jb)
          if (jb < Jt) {
            pg0[t][jb] = gb[jb * 128];
            pg1[t][jb] = gb[jb * 128 + 1];
          }
      }
    }
    if (c12) load_mix_weights();
  }

  // ---- 1. column DFT: unit u = (tile jt, chunk kc), u = wave, wave + 4, ...
  const int HBc = (HB + KS - 1) / KS;
  {
    const bool rok = r16 < rows;
    const float2* ar = At + ((int64_t)q0 * Cin + (rok ? r16 : 0)) * P1;
    for (int u = wave; u < Jt * KS; u += NW) {
      const int jt = u % Jt, kc = u / Jt;
      const int hb0 = kc * HBc;
      const int nhb = min(HBc, HB - hb0);
      const f32x4* fb = FB + ((int64_t)jt * HB * 64 + lane) * 2;
      float are[HBC][4], aim[HBC][4];
      f32x4 af0[HBC], af1[HBC];
#pragma unroll
      for (int i = 0; i < HBC; ++i) {
        if (i < nhb) {
          const int h1 = (hb0 + i) * 16 + kq * 4;
          load4c(ar + h1, rok ? P1 - h1 : 0, vec, are[i], aim[i]);
          af0[i] = fb[(hb0 + i) * 128];
          af1[i] = fb[(hb0 + i) * 128 + 1];
        }
      }
      f32x4 dr = {0.f, 0.f, 0.f, 0.f}, di = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < HBC; ++i)
        if (i < nhb) cmfma4(are[i], aim[i], af0[i], af1[i], dr, di);
#pragma unroll
      for (int r = 0; r < 4; ++r) sP[kq * 4 + r][kc * K1p + jt * 16 + r16] = make_float2(dr[r], di[r]);
    }
  }
  CF_MARK(1);
  __syncthreads();
  CF_MARK(2);
  // chunk sum in order, the adjoint's c_k / (P1 P2) scale, the saved spectrum
  for (int e = threadIdx.x; e < 16 * K1p; e += kT) {
    const int row = e / K1p, j = e - row * K1p;
    float2 v = sP[row][j];
    for (int kc = 1; kc < KS; ++kc) {
      const float2 w = sP[row][kc * K1p + j];
      v.x += w.x;
      v.y += w.y;
    }
    if (row < rows) {
      if (DIR == 1) {
        const float sc = c2r_weight((q0 + row / Cin) % m2, P2) * inv;
        v.x *= sc;
        v.y *= sc;
      }
      if (j < K1) Xs[((int64_t)q0 * Cin + row) * K1 + j] = v;
    }
    sX[row][j] = v;
  }
  __syncthreads();
  CF_MARK(3);

  // H16: block scale 2^e with max |component| * 2^e in [2^14, 2^15) over the spectra rows
  float hs = 1.0f, hinv = 1.0f;
  if constexpr (H16) {
    __shared__ float smax[NW];
    float mx = 0.f;
    for (int e = threadIdx.x; e < rows * K1p; e += kT) {
      const float2 v = sX[e / K1p][e % K1p];
      mx = fmaxf(mx, fmaxf(fabsf(v.x), fabsf(v.y)));
    }
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) mx = fmaxf(mx, __shfl_xor(mx, m, 64));
    if (lane == 0) smax[wave] = mx;
    __syncthreads();
    mx = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) mx = fmaxf(mx, smax[w]);
    if (mx > 0.f && mx < 3.0e38f) {
      int ex;
      frexpf(mx, &ex);
      hs = ldexpf(1.0f, 15 - ex);
      hinv = ldexpf(1.0f, ex - 15);
    }
  }

  // ---- 2. the mix: Y[p o][j] into sP (rows >= orows and columns >= K1 zero)
  // the 12-channel heads (one pair per workgroup, 16 K1p = 1024 outputs, 2 per thread at 8
  // waves): every weight load of the thread's outputs issued before the first multiply (with
  // the generic 4-unrolled loop each output waited on three L2 round trips in turn); same
  // summation order
  if (c12) {
    const int k = q0 % m2;
    if constexpr (!PF) load_mix_weights();
    const float sc = DIR == 0 ? c2r_weight(k, P2) * inv : 1.0f;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int e = threadIdx.x + i * kT;
      if (e >= 16 * K1p) continue;
      const int t = e / kC;
      if (t >= K1p) continue;                        // rows >= 12 are zeroed below
      float re = 0.f, im = 0.f;
      if (live[i]) {
        const float2* xp = &sX[0][jv[i]];
#pragma unroll
        for (int c = 0; c < kC; ++c) {
          const float2 a = xp[c * kLd];
          const float2 w = wv[i][c];
          if (DIR == 0) {
            re = fmaf(a.x, w.x, fmaf(-a.y, w.y, re));
            im = fmaf(a.x, w.y, fmaf(a.y, w.x, im));
          } else {
            re = fmaf(w.x, a.x, fmaf(w.y, a.y, re));
            im = fmaf(w.x, a.y, fmaf(-w.y, a.x, im));
          }
        }
        re *= sc;
        im *= sc;
      }
      sP[ov[i]][jv[i]] = make_float2(re, im);
    }
  } else
  for (int e = threadIdx.x; e < 16 * K1p; e += kT) {
    const int o = e % Cout;                       // output channel fastest: contiguous weights
    const int t = e / Cout;
    const int j = t % K1p, p = t / K1p;
    const int orow = p * Cout + o;
    if (orow >= 16) continue;
    float re = 0.f, im = 0.f;
    if (p < np && j < K1) {
      const int k = (q0 + p) % m2;
      const float2* wg = wtgs ? reinterpret_cast<const float2*>(
                                    reinterpret_cast<const float*>(Wt) + ((q0 + p) / m2 / Bg) * wtgs)
                              : Wt;
      const float2* wj = wg + ((int64_t)k * K1 + j) * Ci * Co;
      const float2* xp = &sX[p * Cin][j];
      if constexpr (H16) {
#pragma unroll 4
        for (int c = 0; c < Cin; ++c) {
          const float2 a = xp[c * kLd];
          const f16x2 ah = {(_Float16)(a.x * hs), (_Float16)(a.y * hs)};
          const float2 w = DIR == 0 ? wj[c * Co + o] : wj[o * Co + c];
          const _Float16 wr = (_Float16)w.x, wi = (_Float16)w.y;
          if (DIR == 0) {
            re = __builtin_amdgcn_fdot2(ah, (f16x2){wr, (_Float16)(-wi)}, re, false);
            im = __builtin_amdgcn_fdot2(ah, (f16x2){wi, wr}, im, false);
          } else {
            re = __builtin_amdgcn_fdot2(ah, (f16x2){wr, wi}, re, false);
            im = __builtin_amdgcn_fdot2(ah, (f16x2){(_Float16)(-wi), wr}, im, false);
          }
        }
        re *= hinv;
        im *= hinv;
      } else {
#pragma unroll 4
        for (int c = 0; c < Cin; ++c) {
          const float2 a = xp[c * kLd];
          const float2 w = DIR == 0 ? wj[c * Co + o] : wj[o * Co + c];
          if (DIR == 0) {
            re = fmaf(a.x, w.x, fmaf(-a.y, w.y, re));
            im = fmaf(a.x, w.y, fmaf(a.y, w.x, im));
          } else {                                    // conj(w) * a
            re = fmaf(w.x, a.x, fmaf(w.y, a.y, re));
            im = fmaf(w.x, a.y, fmaf(-w.y, a.x, im));
          }
        }
      }
      if (DIR == 0) {
        const float sc = c2r_weight(k, P2) * inv;
        re *= sc;
        im *= sc;
      }
    }
    sP[orow][j] = make_float2(re, im);
  }
  // rows past G Cout (e.g. 12-channel pairs) are zero: the inverse's A operand reads all 16
  for (int e = threadIdx.x; e < 16 * K1p; e += kT) {
    const int row = e / K1p;
    if (row >= min(16, (16 / Cout) * Cout)) sP[row][e - row * K1p] = make_float2(0.f, 0.f);
  }
  CF_MARK(4);
  __syncthreads();
  CF_MARK(5);

  // ---- 3. column inverse: D[orow][h] = sum_j Y[orow][j] conj F[h][j], h tiles over the waves
  const int Ht = HB;
  const int R = m2 * Cout;
  auto inv_tile = [&](const int ht, const f32x4 (&g0)[4], const f32x4 (&g1)[4]) {
    f32x4 dr = {0.f, 0.f, 0.f, 0.f}, di = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int jb = 0; jb < 4; ++jb) {
      if (jb >= Jt) break;
      float re[4], im[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const float2 v = sP[r16][jb * 16 + kq * 4 + s];
        re[s] = v.x;
        im[s] = v.y;
      }
      cmfma4(re, im, g0[jb], g1[jb], dr, di);
    }
    const int h = ht * 16 + r16;
    if (h >= P1) return;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int orow = kq * 4 + r;
      if (orow >= orows) continue;
      const int p = orow / Cout, o = orow - p * Cout;
      const int q = q0 + p, n = q / m2, k = q - n * m2;
      const float2 v = make_float2(dr[r], di[r]);
      if (!tiled) {
        Z[((int64_t)n * P1 + h) * R + k * Cout + o] = v;
      } else {
        const int gr = n * P1 + h;
        const int c16 = 4 * (gr & 3) + (o & 3);
        float* zt = reinterpret_cast<float*>(Z) +
                    ((int64_t)((gr >> 2) * (Cout >> 2) + (o >> 2)) * (m2 >> 1) + (k >> 1)) * 64;
        zt[32 * (k & 1) + c16] = v.x;
        zt[32 * (k & 1) + 16 + c16] = v.y;
      }
    }
  };
  // every j block's twiddles in flight before the first MFMA (Jt <= 4)
  auto load_inv_twiddles = [&](const int ht, f32x4 (&g0)[4], f32x4 (&g1)[4]) {
    const f32x4* gb = GB + ((int64_t)ht * Jt * 64 + lane) * 2;
#pragma unroll
    for (int jb = 0; jb < 4; ++jb)
      if (jb < Jt) {
        g0[jb] = gb[jb * 128];
        g1[jb] = gb[jb * 128 + 1];
      }
  };
  int ht0 = wave;
  if constexpr (PF) {
#pragma unroll
    for (int t = 0; t < 2; ++t)
      if (wave + t * NW < Ht) inv_tile(wave + t * NW, pg0[t], pg1[t]);
    ht0 = wave + 2 * NW;
  }
  for (int ht = ht0; ht < Ht; ht += NW) {
    f32x4 g0[4], g1[4];
    load_inv_twiddles(ht, g0, g1);
    inv_tile(ht, g0, g1);
  }
  CF_MARK(6);
}
#if COLFUSE_PROBE
BLINDNO_API int blindno_colfuse_probe_read(unsigned long long* dst, int n) {
  return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_colfuse_probe),
                                  sizeof(unsigned long long) * (size_t)n, 0, hipMemcpyDeviceToHost);
}
#endif

// Z[n][h][k][o] = sum_j Y[n m2 + k][o][j] conj(F[h][j]).  Workgroup = (sample, 16-row h
// tile, 64 spectrum rows (k, o)); one 16-row MFMA tile per wave; the result is transposed
// through LDS so that each h row of Z is written as one contiguous run.  tiled: Z in the
// A-tile order of the wide row inverse instead (rowinv_tile_layout, rowinv.hip).
__global__ __launch_bounds__(256) void colidft_kernel(const float2* __restrict__ Y,
                                                      const f32x4* __restrict__ GB,
                                                      float2* __restrict__ Z, int Cout, int P1,
                                                      int m1, int m2, int tiled) {
  __shared__ float2 sZ[16][65];
  const int K1 = kept_rows_count(m1, P1);
  const int Jt = (K1 + 15) >> 4, K1p = Jt * 16;
  const int Ht = (P1 + 15) >> 4;
  const int R = m2 * Cout;
  const int Mt = (R + 15) >> 4;
  const int n = blockIdx.x / Ht, ht = blockIdx.x % Ht;
  const int lane = threadIdx.x & 63;
  const int wave = uniform_int(threadIdx.x >> 6);
  const int r16 = lane & 15, kq = lane >> 4;
  const int mt = blockIdx.y * 4 + wave;
  if (mt < Mt) {
    const int row = mt * 16 + r16;
    const bool rok = row < R;
    const float2* yr = Y + ((int64_t)n * R + (rok ? row : 0)) * K1p;
    const f32x4* gb = GB + ((int64_t)ht * Jt * 64 + lane) * 2;
    f32x4 dr = {0.f, 0.f, 0.f, 0.f}, di = {0.f, 0.f, 0.f, 0.f};
    for (int jb = 0; jb < Jt; ++jb) {
      float re[4], im[4];
      load4c(yr + jb * 16 + kq * 4, rok ? 4 : 0, true, re, im);
      cmfma4(re, im, gb[jb * 128], gb[jb * 128 + 1], dr, di);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) sZ[r16][wave * 16 + kq * 4 + r] = make_float2(dr[r], di[r]);
  }
  __syncthreads();
  const int row0 = blockIdx.y * 64;
  for (int e = threadIdx.x; e < 16 * 64; e += blockDim.x) {
    const int hl = e >> 6, rl = e & 63;
    const int h = ht * 16 + hl, row = row0 + rl;
    if (h < P1 && row < R) {
      if (!tiled) {
        Z[((int64_t)n * P1 + h) * R + row] = sZ[hl][rl];
      } else {
        // grid row gr = n P1 + h -> quad gr / 4, A row (gr & 3); channel o -> group o / 4,
        // column o & 3; mode k -> K step k / 2, lanes 32 (k & 1) + (0: Re | 16: Im) + c16
        const float2 v = sZ[hl][rl];
        const int k = row / Cout, o = row - (row / Cout) * Cout;
        const int gr = n * P1 + h;
        const int c16 = 4 * (gr & 3) + (o & 3);
        float* zt = reinterpret_cast<float*>(Z) +
                    ((int64_t)((gr >> 2) * (Cout >> 2) + (o >> 2)) * (m2 >> 1) + (k >> 1)) * 64;
        zt[32 * (k & 1) + c16] = v.x;
        zt[32 * (k & 1) + 16 + c16] = v.y;
      }
    }
  }
}

__global__ __launch_bounds__(kBlock) void mix_wgrad_kernel(const float2* __restrict__ X,
                                                           const float2* __restrict__ G,
                                                           float2* __restrict__ out, int Bn,
                                                           int Ci, int Co, int K1, int m2) {
  mix_wgrad_block(X, G, out, Bn, Ci, Co, K1, m2, blockIdx.x, blockIdx.y, blockIdx.z, gridDim.x,
                  gridDim.y, gridDim.z);
}

// The heads' backward, one layer (reverse order k = n-1 .. 0): the row DFT of dz_k, the 1x1-conv
// weight gradient of (dz_k, f(x_k)) and the spectral weight gradient of layer k + 1 (whose
// column pass has just run) are independent of each other, and each is a few-microsecond,
// latency-bound launch at the heads' size (Bn = 8 at config C).  One launch hosts all three:
// workgroups [0, nbr) run the row DFT, the next nchunk G the conv gradient, the rest the mix
// gradient (nbm = 0: none), each with the grid coordinates of its own launch, so the results
// are bit-identical to the three separate launches.
struct ConvWgradJob {
  const float* dz;
  const float* x;
  float* partial;
  int C, HW, Bg, nchunk, G;
};

template <int NT, int ALIGNED, int ACT>
__global__ __launch_bounds__(256) void rowdft_wgrad_kernel(const float* __restrict__ x,
                                                           float* __restrict__ At,
                                                           const float* __restrict__ Tp,
                                                           int nrows, int C, int P1, int P2,
                                                           int m2, int KB, int Npad,
                                                           int ntile_groups, int nbr,
                                                           ConvWgradJob cw, MixWgradJob mw) {
  int b = blockIdx.x;
  if (b < nbr) {
    rowdft_mfma_block<NT, ALIGNED, false>(x, At, Tp, nrows, C, P1, P2, m2, KB, Npad, ntile_groups,
                                          0, P1, P2, b, nbr);
    return;
  }
  b -= nbr;
  const int nbc = cw.nchunk * cw.G;
  if (b < nbc) {
    conv_wgrad_mfma_block<ACT>(cw.dz, cw.x, cw.partial, cw.C, cw.HW, cw.Bg, b % cw.nchunk,
                               cw.nchunk, b / cw.nchunk, cw.G);
    return;
  }
  b -= nbc;
  mix_wgrad_block(mw.X, mw.Gs, mw.out, mw.Bn, mw.Ci, mw.Co, mw.K1, mw.m2, b % mw.gx,
                  (b / mw.gx) % mw.gy, b / (mw.gx * mw.gy), mw.gx, mw.gy, mw.gz);
}

// Several spectral weight gradients in one launch (the deferred ones of a backward pass,
// blindno.ops.deferred_reductions: the heads' layers and the encoder's): job q owns workgroups
// [cum[q], cum[q+1]) with the grid of its own blindno_mix_wgrad_g launch (bit-identical).
constexpr int kMixJobs = 8;
struct MixJobs {
  MixWgradJob j[kMixJobs];
  int cum[kMixJobs + 1];
  int n;
};

__global__ __launch_bounds__(kBlock) void mix_wgrad_multi_kernel(MixJobs jobs) {
  const int b = blockIdx.x;
  int q = 0;
  while (q + 1 < jobs.n && jobs.cum[q + 1] <= b) ++q;             // uniform scan
  const MixWgradJob& m = jobs.j[q];
  const int r = b - jobs.cum[q];
  const int grp = r / (m.gx * m.gy);
  const bool upk = m.um1 > 0;
  W2dUnpack uw{};
  if (upk) uw = W2dUnpack{m.u1[grp], m.u2[grp], m.Ci, m.Co, m.um1, m.m2};
  mix_wgrad_block(m.X, m.Gs, m.out, m.Bn, m.Ci, m.Co, m.K1, m.m2, r % m.gx, (r / m.gx) % m.gy,
                  grp, m.gx, m.gy, m.gz, upk, uw);
}

// ------------------------------------------------------------------------------ 1D mode mix
// At[n][k][c] (P1 = 1).  Forward: Xs = h_k At (DC halved) ; Z[n][k][o] = c_k/P2 sum_i Xs W.
// Backward: Xs = c_k/P2 At (= spectrum gradient) ; Z[n][k][i] = h_k sum_o conj(W) Xs.
template <int DIR>
__global__ __launch_bounds__(kBlock) void mix1d_kernel(const float2* __restrict__ At,
                                                       const float2* __restrict__ Wt,
                                                       float2* __restrict__ Xs,
                                                       float2* __restrict__ Z, int Bn, int Ci,
                                                       int Co, int m, int P2) {
  const int Cout = DIR == 0 ? Co : Ci;
  const int Cin = DIR == 0 ? Ci : Co;
  const float invP = 1.0f / (float)P2;
  const int64_t total = (int64_t)Bn * m * Cout;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int oc = (int)(idx % Cout);
    const int64_t nk = idx / Cout;
    const int k = (int)(nk % m);
    const float hk = k == 0 ? 0.5f : 1.0f;
    const float ck = c2r_weight(k, P2) * invP;
    const float2* av = At + nk * Cin;
    const float2* wv = Wt + (int64_t)k * Ci * Co;
    float re = 0.f, im = 0.f;
    for (int q = 0; q < Cin; ++q) {
      float2 a = av[q];
      if (DIR == 0) {
        const float2 w = wv[q * Co + oc];
        re = fmaf(a.x, w.x, fmaf(-a.y, w.y, re));
        im = fmaf(a.x, w.y, fmaf(a.y, w.x, im));
      } else {
        const float2 w = wv[oc * Co + q];
        re = fmaf(w.x, a.x, fmaf(w.y, a.y, re));
        im = fmaf(w.x, a.y, fmaf(-w.y, a.x, im));
      }
    }
    const float sc = DIR == 0 ? hk * ck : ck * hk;
    Z[idx] = make_float2(re * sc, im * sc);
  }
  const int64_t tot2 = (int64_t)Bn * m * Cin;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < tot2;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int k = (int)((idx / Cin) % m);
    const float2 a = At[idx];
    const float sc = DIR == 0 ? (k == 0 ? 0.5f : 1.0f) : c2r_weight(k, P2) * invP;
    Xs[idx] = make_float2(a.x * sc, a.y * sc);
  }
}

// ------------------------------------------------------------------------------ weight packing
// blockIdx.y selects one of up to two weight sets (the two heads, packed in one launch)
__global__ void pack_w2d_kernel(const float* __restrict__ w1a, const float* __restrict__ w2a,
                                const float* __restrict__ w1b, const float* __restrict__ w2b,
                                float2* __restrict__ Wt, int Ci, int Co, int m1, int m2,
                                int P1) {
  const int K1 = kept_rows_count(m1, P1);
  const int64_t total = (int64_t)m2 * K1 * Ci * Co;
  const float* w1 = blockIdx.y ? w1b : w1a;
  const float* w2 = blockIdx.y ? w2b : w2a;
  Wt += blockIdx.y * total;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int o = (int)(idx % Co);
    int64_t t = idx / Co;
    const int i = (int)(t % Ci);
    t /= Ci;
    const int j = (int)(t % K1);
    const int k = (int)(t / K1);
    const int r = kept_row(j, K1, m1, P1);
    const bool second = r >= P1 - m1;
    const float* src = second ? w2 : w1;
    const int jj = second ? r - (P1 - m1) : r;
    const float* p = src + ((((int64_t)i * Co + o) * m1 + jj) * m2 + k) * 2;
    Wt[idx] = make_float2(p[0], p[1]);
  }
}

__global__ void unpack_w2d_kernel(const float2* __restrict__ dWt, float* __restrict__ dw1a,
                                  float* __restrict__ dw2a, float* __restrict__ dw1b,
                                  float* __restrict__ dw2b, int Ci, int Co, int m1, int m2,
                                  int P1) {
  const int K1 = kept_rows_count(m1, P1);
  const int64_t per = (int64_t)Ci * Co * m1 * m2;
  float* dw1 = blockIdx.y ? dw1b : dw1a;
  float* dw2 = blockIdx.y ? dw2b : dw2a;
  dWt += blockIdx.y * (int64_t)m2 * K1 * Ci * Co;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < 2 * per;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int which = idx >= per;
    const int64_t e = which ? idx - per : idx;
    const int k = (int)(e % m2);
    int64_t t = e / m2;
    const int jj = (int)(t % m1);
    t /= m1;
    const int o = (int)(t % Co);
    const int i = (int)(t / Co);
    int j = -1;
    if (which) {
      const int r = P1 - m1 + jj;
      j = (K1 == P1) ? r : m1 + jj;
    } else if (jj < P1 - m1) {
      j = jj;                     // otherwise shadowed by weights2 (overlapping rows)
    }
    float2 v = make_float2(0.f, 0.f);
    if (j >= 0) v = dWt[(((int64_t)k * K1 + j) * Ci + i) * Co + o];
    float* dst = (which ? dw2 : dw1) + e * 2;
    dst[0] = v.x;
    dst[1] = v.y;
  }
}

__global__ void pack_w1d_kernel(const float2* __restrict__ src, float2* __restrict__ dst, int Ci,
                                int Co, int m, int dir) {
  const int64_t total = (int64_t)Ci * Co * m;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int k = (int)(idx % m);
    const int64_t t = idx / m;
    const int o = (int)(t % Co);
    const int i = (int)(t / Co);
    const int64_t pidx = ((int64_t)k * Ci + i) * Co + o;
    if (dir == 0)
      dst[pidx] = src[idx];          // (Ci,Co,m) -> (m,Ci,Co)
    else
      dst[idx] = src[pidx];          // (m,Ci,Co) -> (Ci,Co,m)
  }
}

}  // namespace

// launch shape of the row DFT over (Bn C P1) rows, columns < N2v live
struct RowdftPlan {
  int nrows, KB, Npad, nt, groups, blocks;
  int64_t nwork;
  size_t sh;
  bool aligned, stage;
};
static int rowdft_plan(const float* x, int Bn, int C, int P1, int P2, int m2, int N1v, int N2v,
                       RowdftPlan& p) {
  if (Bn <= 0 || C <= 0 || P1 <= 0 || P2 <= 0 || m2 <= 0 || m2 > P2 / 2 + 1 || N1v < 1 ||
      N1v > P1 || N2v < 1 || N2v > P2)
    return (int)hipErrorInvalidValue;
  const int64_t nrows64 = (int64_t)Bn * C * P1;
  if (nrows64 > INT32_MAX) return (int)hipErrorInvalidValue;
  p.nrows = (int)nrows64;
  p.KB = (N2v + 15) / 16;                         // K blocks past the valid columns are zero
  p.Npad = ((2 * m2 + 15) / 16) * 16;
  const int ntiles = p.Npad / 16;
  p.sh = sizeof(float) * (size_t)p.KB * 16 * p.Npad;
  if (p.sh > 160 * 1024) return (int)hipErrorInvalidValue;
  // tiles per wave: all of them when there are many row tiles, else split for parallelism
  const int nrt = (p.nrows + 15) / 16;
  int nt = ntiles;
  if (nt > 4) nt = 4;
  while (nt > 1 && (int64_t)nrt * ((ntiles + nt - 1) / nt) < ROWDFT_MIN_WORK) nt >>= 1;
  while (ntiles % nt) --nt;
  p.nt = nt;
  p.groups = ntiles / nt;
  p.nwork = (int64_t)nrt * p.groups;
  p.blocks = (int)((p.nwork + 3) / 4 < ROWDFT_MAX_BLOCKS ? (p.nwork + 3) / 4 : ROWDFT_MAX_BLOCKS);
  p.aligned = (P2 % 4) == 0 && (((uintptr_t)x) & 15) == 0;
  // stage the twiddle image only when the waves reuse it (>= ROWDFT_STAGE_ITEMS work items
  // per wave)
  p.stage = p.nwork >= (int64_t)ROWDFT_STAGE_ITEMS * 4 * p.blocks;
  return 0;
}

BLINDNO_API int blindno_rowdft_crop(const float* x, float* At, const float* Tp, int Bn, int C,
                                    int P1, int P2, int m2, int act, int N1v, int N2v,
                                    void* stream) {
  RowdftPlan p;
  const int e = rowdft_plan(x, Bn, C, P1, P2, m2, N1v, N2v, p);
  if (e) return e;
  hipStream_t st = (hipStream_t)stream;
#define RD(NT_, AL_)                                                                        \
  do {                                                                                      \
    if (p.stage)                                                                            \
      rowdft_mfma_kernel<NT_, AL_, true><<<p.blocks, 256, p.sh, st>>>(                      \
          x, At, Tp, p.nrows, C, P1, P2, m2, p.KB, p.Npad, p.groups, act, N1v, N2v);        \
    else                                                                                    \
      rowdft_mfma_kernel<NT_, AL_, false><<<p.blocks, 256, 0, st>>>(                        \
          x, At, Tp, p.nrows, C, P1, P2, m2, p.KB, p.Npad, p.groups, act, N1v, N2v);        \
  } while (0)
#define RD_AL(NT_) \
  if (p.aligned) RD(NT_, 1); else RD(NT_, 0);
  switch (p.nt) {
    case 1: RD_AL(1) break;
    case 2: RD_AL(2) break;
    case 3: RD_AL(3) break;
    default: RD_AL(4) break;
  }
#undef RD_AL
#undef RD
  return (int)hipGetLastError();
}

BLINDNO_API int blindno_rowdft(const float* x, float* At, const float* Tp, int Bn, int C,
                               int P1, int P2, int m2, int act, void* stream) {
  return blindno_rowdft_crop(x, At, Tp, Bn, C, P1, P2, m2, act, P1, P2, stream);
}

BLINDNO_API int blindno_rowdft_bag_lift_dg(const float* X, const int* idx, const float* w0,
                                           const float* b0, const float* Gt, float* At,
                                           const float* Tp, int B, int T, int L, int N1, int N2,
                                           int C, int P1, int P2, int m2, void* stream) {
  if (B <= 0 || L <= 0 || T <= 0 || C <= 0 || N1 > P1 || N2 > P2 || m2 <= 0 || m2 > P2 / 2 + 1)
    return (int)hipErrorInvalidValue;
  const int64_t nrows64 = (int64_t)B * L * P1;
  if (nrows64 > INT32_MAX || (int64_t)B * T * N1 * N2 >= ((int64_t)1 << 40))
    return (int)hipErrorInvalidValue;
  const int nrows = (int)nrows64;
  const int KB = (P2 + 15) / 16;
  const int Npad = ((2 * m2 + 15) / 16) * 16;
  const int ntiles = Npad / 16;
  const size_t sh = sizeof(float) * (size_t)KB * 16 * Npad;
  if (sh > 160 * 1024) return (int)hipErrorInvalidValue;
  const int nrt = (nrows + 15) / 16;
  int nt = ntiles;
  if (nt > 4) nt = 4;
  while (nt > 1 && (int64_t)nrt * ((ntiles + nt - 1) / nt) < ROWDFT_MIN_WORK) nt >>= 1;
  while (ntiles % nt) --nt;
  const int groups = ntiles / nt;
  const int64_t nwork = (int64_t)nrt * groups;
  const int blocks = (int)((nwork + 3) / 4 < 4096 ? (nwork + 3) / 4 : 4096);
  const bool aligned = (N2 % 4) == 0 && (((uintptr_t)X) & 15) == 0;
  hipStream_t st = (hipStream_t)stream;
#define RB(NT_, AL_)                                                                          \
  rowdft_bag_lift_kernel<NT_, AL_><<<blocks, 256, sh, st>>>(X, idx, w0, b0, Gt, At, Tp, nrows, T, \
                                                            L, N1, N2, C, P1, m2, KB, Npad, groups)
#define RB_AL(NT_) \
  if (aligned) RB(NT_, 1); else RB(NT_, 0);
  switch (nt) {
    case 1: RB_AL(1) break;
    case 2: RB_AL(2) break;
    case 3: RB_AL(3) break;
    default: RB_AL(4) break;
  }
#undef RB_AL
#undef RB
  return (int)hipGetLastError();
}

BLINDNO_API int blindno_rowdft_bag_lift(const float* X, const int* idx, const float* w0,
                                        const float* Gt, float* At, const float* Tp, int B, int T,
                                        int L, int N1, int N2, int C, int P1, int P2, int m2,
                                        void* stream) {
  return blindno_rowdft_bag_lift_dg(X, idx, w0, nullptr, Gt, At, Tp, B, T, L, N1, N2, C, P1, P2,
                                    m2, stream);
}

// BLINDNO_COLFUSE=0 (or blindno_set_colfuse(0)): the split coldft_mix + colidft kernels
int g_colfuse = -1;
bool colfuse_on() {
  if (g_colfuse < 0) {
    const char* e = getenv("BLINDNO_COLFUSE");
    g_colfuse = (e && e[0] == '0') ? 0 : 1;
  }
  return g_colfuse != 0;
}

BLINDNO_API int blindno_set_colfuse(int on) {
  const int prev = colfuse_on() ? 1 : 0;
  g_colfuse = on ? 1 : 0;
  return prev;
}

BLINDNO_API int blindno_colpass_g(const float* At, const float* Wt, float* Xs, float* Y, float* Z,
                                  const float* FB, const float* GB, int Gw, int64_t wtgs, int Bn,
                                  int Ci, int Co, int P1, int m1, int m2, int P2, int dir,
                                  void* stream) {
  // dir bit 0: 0 forward / 1 adjoint; bit 1: fp16-operand mix (H16 above)
  if (Bn <= 0 || m1 <= 0 || m1 > P1 || m2 <= 0 || m2 > P2 / 2 + 1 || (dir & ~3) || Gw < 1 ||
      Bn % Gw)
    return (int)hipErrorInvalidValue;
  const bool h16 = (dir & 2) != 0;
  dir &= 1;
  const int Bg = Bn / Gw;
  if (Gw == 1) wtgs = 0;
  const int K1 = kept_rows_count(m1, P1);
  const int Jt = (K1 + 15) / 16, K1p = Jt * 16;
  const int cin = dir == 0 ? Ci : Co, cout = dir == 0 ? Co : Ci;
  const int64_t npairs = (int64_t)Bn * m2;
  if (npairs * (cin > cout ? cin : cout) * (P1 > K1p ? P1 : K1p) >= INT32_MAX)
    return (int)hipErrorInvalidValue;
  const int HB = (P1 + 15) / 16;
  hipStream_t st = (hipStream_t)stream;
  // the fused pass: fp32 mix, Cin and Cout equal (G pairs fill the same 16 rows on both sides),
  // at most 64 kept rows, at most 10 row blocks per K chunk
  // workgroups of 8 waves when the launch has fewer than two workgroups per CU (the heads)
  const int G16 = 16 / cin;
  const int NWf = cdiv(npairs, G16 > 0 ? G16 : 1) < 512 ? 8 : 4;
  const int KSf = Jt >= NWf ? 1 : NWf / Jt;      // K chunks so that the waves have units
  if (colfuse_on() && Ci == Co && Ci <= 16 && K1p <= 64 &&
      (HB + KSf - 1) / KSf <= 10) {
    const int tiled = rowinv_tile_layout(Bn, cout, P1, P2, m2) ? 1 : 0;
    const int G = G16;
    const int KS = KSf;
    const int HBc = (HB + KS - 1) / KS;
    const int vec = (P1 % 2 == 0) && ((((uintptr_t)At) & 15) == 0);
    const dim3 g((unsigned)cdiv(npairs, G));
#define CF16_(D_, H_, W_, F_)                                                                   \
  colfuse_kernel<D_, H_, W_, F_><<<g, 64 * W_, 0, st>>>((const float2*)At, (const float2*)Wt,    \
                                                        (const f32x4*)FB, (const f32x4*)GB,      \
                                                        (float2*)Xs, (float2*)Z, (int)npairs, Ci, \
                                                        Co, P1, m1, m2, P2, G, KS, vec, Bg, wtgs, \
                                                        tiled)
#define CF_(D_, H_, W_) do { if (h16) CF16_(D_, H_, W_, true); else CF16_(D_, H_, W_, false); } while (0)
#define CFW_(H_, W_) do { if (dir == 0) CF_(0, H_, W_); else CF_(1, H_, W_); } while (0)
#define CFD_(H_) do { if (NWf == 8) CFW_(H_, 8); else CFW_(H_, 4); } while (0)
    if (HBc <= 3) CFD_(3);
    else if (HBc <= 5) CFD_(5);
    else if (HBc <= 10) CFD_(10);
    else return (int)hipErrorInvalidValue;
#undef CFD_
#undef CFW_
#undef CF_
#undef CF16_
    return (int)hipGetLastError();
  }
  // pairs per workgroup: enough 16-row tiles for the four waves, tiles filled
  int G = 1;
  while (((G * cin + 15) / 16) * Jt < COLPASS_WAVE_TILES && G * cin < 64) ++G;
  G = ((G * cin + 15) / 16) * 16 / cin;
  if (G < 1) G = 1;
  const size_t sh = sizeof(float2) * (size_t)G * cin * (K1p + 1);
  if (sh > 160 * 1024) return (int)hipErrorInvalidValue;
  const int vec = (P1 % 2 == 0) && ((((uintptr_t)At) & 15) == 0);
  const dim3 g1((unsigned)cdiv(npairs, G));
  const int tiled = rowinv_tile_layout(Bn, cout, P1, P2, m2) ? 1 : 0;
  // full operand prefetch when the launch is too small to hide latency with waves
  const bool full = (P1 + 15) / 16 <= kFullHB && (int64_t)g1.x * 4 < 4096;
#define CM3_(D_, F_, H_)                                                                    \
  coldft_mix_kernel<D_, F_, H_><<<g1, 256, sh, st>>>(                                       \
      (const float2*)At, (const float2*)Wt, (const f32x4*)FB, (float2*)Xs, (float2*)Y,     \
      (int)npairs, Ci, Co, P1, m1, m2, P2, G, vec, Bg, wtgs)
#define CM_(D_, F_) do { if (h16) CM3_(D_, F_, true); else CM3_(D_, F_, false); } while (0)
  if (dir == 0) {
    if (full) CM_(0, true); else CM_(0, false);
  } else {
    if (full) CM_(1, true); else CM_(1, false);
  }
#undef CM_
#undef CM3_
  int e = (int)hipGetLastError();
  if (e) return e;
  const int Ht = (P1 + 15) / 16;
  const int Mt = (m2 * cout + 15) / 16;
  const dim3 g2((unsigned)(Bn * Ht), (unsigned)((Mt + 3) / 4));
  colidft_kernel<<<g2, 256, 0, st>>>((const float2*)Y, (const f32x4*)GB, (float2*)Z, cout, P1, m1,
                                     m2, tiled);
  return (int)hipGetLastError();
}

BLINDNO_API int blindno_colpass(const float* At, const float* Wt, float* Xs, float* Y, float* Z,
                                const float* FB, const float* GB, int Bn, int Ci, int Co, int P1,
                                int m1, int m2, int P2, int dir, void* stream) {
  return blindno_colpass_g(At, Wt, Xs, Y, Z, FB, GB, 1, 0, Bn, Ci, Co, P1, m1, m2, P2, dir, stream);
}

BLINDNO_API int blindno_mix_wgrad_nsplit(int Bn, int Ci, int Co, int K1, int m2) {
  const int64_t total = (int64_t)m2 * K1 * Ci * Co;
  const int64_t bx = cdiv(total, kBlock);
  int64_t ns = cdiv(2048, bx);                 // aim at >= 2048 workgroups
  const int64_t per = cdiv(Bn, 8);             // but >= 8 samples per slice
  if (ns > per) ns = per;
  if (ns < 1) ns = 1;
  return (int)(ns > 1024 ? 1024 : ns);
}

// The split weight gradient's partials only (nsplit > 1): partial[y][Gw][m2 K1 Ci Co] complex,
// reduced by the caller (blindno.ops' deferred finalisation batches that reduction).
BLINDNO_API int blindno_mix_wgrad_part(const float* X, const float* G, float* partial, int nsplit,
                                       int Gw, int Bn, int Ci, int Co, int K1, int m2,
                                       void* stream) {
  const int64_t total = (int64_t)m2 * K1 * Ci * Co;
  if (total >= INT32_MAX / 2 || nsplit < 2 || !partial || Gw < 1 || Bn % Gw)
    return (int)hipErrorInvalidValue;
  const dim3 g((unsigned)cdiv(total, kBlock), nsplit, Gw);
  mix_wgrad_kernel<<<g, kBlock, 0, (hipStream_t)stream>>>((const float2*)X, (const float2*)G,
                                                          (float2*)partial, Bn, Ci, Co, K1, m2);
  return (int)hipGetLastError();
}

BLINDNO_API int blindno_rowdft_wgrad_ok(int Bn, int C, int P1, int P2, int m2) {
  RowdftPlan p;
  return conv_wgrad_mfma_ok(C, (int64_t)P1 * P2) &&
                 rowdft_plan(nullptr, Bn, C, P1, P2, m2, P1, P2, p) == 0
             ? 1
             : 0;
}

// One layer of the heads' backward in one launch (rowdft_wgrad_kernel): At = rowDFT(dz) as
// blindno_rowdft, the conv gradient partials of (dz, f(src)) as blindno_conv_wgrad_g and, when
// Xs != NULL, the previous layer's spectral weight gradient as blindno_mix_wgrad_g.
BLINDNO_API int blindno_rowdft_wgrad_g(const float* dz, const float* src, float* At,
                                       const float* Tp, float* cpartial, int cnchunk, int act,
                                       const float* Xs, const float* Gs, float* dWt,
                                       float* mpartial, int mnsplit, int K1, int G, int Bn, int C,
                                       int P1, int P2, int m2, void* stream) {
  if (G < 1 || Bn % G || !dz || !src || !At || !Tp || !cpartial) return (int)hipErrorInvalidValue;
  const int Bg = Bn / G;
  const int64_t HW = (int64_t)P1 * P2;
  if (!conv_wgrad_mfma_ok(C, HW) || cnchunk != blindno_conv_wgrad_nchunk(Bg, P1, P2))
    return (int)hipErrorInvalidValue;
  RowdftPlan p;
  int e = rowdft_plan(dz, Bn, C, P1, P2, m2, P1, P2, p);
  if (e) return e;
  MixWgradJob mw{(const float2*)Xs, (const float2*)Gs, nullptr, Bn, C, C, K1, m2, 1, 1, G};
  int64_t nbm = 0;
  const int64_t total = (int64_t)m2 * K1 * C * C;
  if (Xs) {
    if (!Gs || !dWt || K1 < 1 || total >= INT32_MAX / 2 || mnsplit < 1 ||
        (mnsplit > 1 && !mpartial))
      return (int)hipErrorInvalidValue;
    mw.out = (float2*)(mnsplit > 1 ? mpartial : dWt);
    mw.gx = (int)cdiv(total, kBlock);
    mw.gy = mnsplit;
    nbm = (int64_t)mw.gx * mw.gy * G;
  }
  const ConvWgradJob cw{dz, src, cpartial, C, (int)HW, Bg, cnchunk, G};
  const int64_t nb = p.blocks + (int64_t)cnchunk * G + nbm;
  if (nb >= INT32_MAX) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
#define RW(NT_, AL_, A_)                                                                      \
  rowdft_wgrad_kernel<NT_, AL_, A_><<<(unsigned)nb, 256, 0, st>>>(                            \
      dz, At, Tp, p.nrows, C, P1, P2, m2, p.KB, p.Npad, p.groups, p.blocks, cw, mw)
#define RW_A(NT_, AL_) do { if (act) RW(NT_, AL_, 1); else RW(NT_, AL_, 0); } while (0)
#define RW_AL(NT_) do { if (p.aligned) RW_A(NT_, 1); else RW_A(NT_, 0); } while (0)
  switch (p.nt) {
    case 1: RW_AL(1); break;
    case 2: RW_AL(2); break;
    case 3: RW_AL(3); break;
    default: RW_AL(4); break;
  }
#undef RW_AL
#undef RW_A
#undef RW
  e = (int)hipGetLastError();
  if (e || !Xs || mnsplit == 1) return e;
  return blindno_reduce_partials(mpartial, dWt, mnsplit, (int)(2 * total * G), stream);
}

// jobs q < njobs: X[q], G[q] -> out[q] (dWt when nsplit == 1, else the nsplit x Gw partials,
// reduced by the caller); shp[7 q ..] = (Bn, Ci, Co, K1, m2, nsplit, Gw)
BLINDNO_API int blindno_mix_wgrad_multi_u(const void* const* X, const void* const* G,
                                          void* const* out, const int* shp, void* const* ud,
                                          const int* um1, int njobs, void* stream) {
  if (njobs < 0) return (int)hipErrorInvalidValue;
  for (int q0 = 0; q0 < njobs; q0 += kMixJobs) {
    MixJobs jobs{};
    const int k = njobs - q0 < kMixJobs ? njobs - q0 : kMixJobs;
    jobs.n = k;
    int64_t blocks = 0;
    for (int i = 0; i < k; ++i) {
      const int* sh = shp + 7 * (q0 + i);
      const int Bn = sh[0], Ci = sh[1], Co = sh[2], K1 = sh[3], m2 = sh[4], ns = sh[5], Gw = sh[6];
      const int64_t total = (int64_t)m2 * K1 * Ci * Co;
      if (Bn < 1 || Ci < 1 || Co < 1 || K1 < 1 || m2 < 1 || ns < 1 || Gw < 1 || Bn % Gw ||
          total >= INT32_MAX / 2 || !X[q0 + i] || !G[q0 + i] || !out[q0 + i])
        return (int)hipErrorInvalidValue;
      MixWgradJob& m = jobs.j[i];
      m.X = (const float2*)X[q0 + i];
      m.Gs = (const float2*)G[q0 + i];
      m.out = (float2*)out[q0 + i];
      m.Bn = Bn; m.Ci = Ci; m.Co = Co; m.K1 = K1; m.m2 = m2;
      m.gx = (int)cdiv(total, kBlock);
      m.gy = ns;
      m.gz = Gw;
      m.um1 = um1 ? um1[q0 + i] : 0;
      if (m.um1 > 0) {
        if (ns != 1 || Gw > kMixMaxGw || K1 != 2 * m.um1) return (int)hipErrorInvalidValue;
        for (int g = 0; g < Gw; ++g) {
          m.u1[g] = (float*)ud[(q0 + i) * 2 * kMixMaxGw + 2 * g];
          m.u2[g] = (float*)ud[(q0 + i) * 2 * kMixMaxGw + 2 * g + 1];
          if (!m.u1[g] || !m.u2[g]) return (int)hipErrorInvalidValue;
        }
      }
      jobs.cum[i] = (int)blocks;
      blocks += (int64_t)m.gx * ns * Gw;
    }
    if (blocks >= INT32_MAX) return (int)hipErrorInvalidValue;
    jobs.cum[k] = (int)blocks;
    if (blocks == 0) continue;
    mix_wgrad_multi_kernel<<<(unsigned)blocks, kBlock, 0, (hipStream_t)stream>>>(jobs);
  }
  return (int)hipGetLastError();
}

BLINDNO_API int blindno_mix_wgrad_multi(const void* const* X, const void* const* G,
                                        void* const* out, const int* shp, int njobs,
                                        void* stream) {
  return blindno_mix_wgrad_multi_u(X, G, out, shp, nullptr, nullptr, njobs, stream);
}

BLINDNO_API int blindno_mix_wgrad_g(const float* X, const float* G, float* dWt, float* partial,
                                    int nsplit, int Gw, int Bn, int Ci, int Co, int K1, int m2,
                                    void* stream) {
  const int64_t total = (int64_t)m2 * K1 * Ci * Co;
  if (total >= INT32_MAX / 2 || nsplit < 1 || (nsplit > 1 && !partial) || Gw < 1 || Bn % Gw)
    return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  const dim3 g((unsigned)cdiv(total, kBlock), nsplit, Gw);
  mix_wgrad_kernel<<<g, kBlock, 0, st>>>((const float2*)X, (const float2*)G,
                                         (float2*)(nsplit > 1 ? partial : dWt), Bn, Ci, Co, K1,
                                         m2);
  if (nsplit > 1) {
    const int e = (int)hipGetLastError();
    if (e) return e;
    return blindno_reduce_partials(partial, dWt, nsplit, (int)(2 * total * Gw), stream);
  }
  return (int)hipGetLastError();
}

BLINDNO_API int blindno_mix_wgrad(const float* X, const float* G, float* dWt, float* partial,
                                  int nsplit, int Bn, int Ci, int Co, int K1, int m2,
                                  void* stream) {
  return blindno_mix_wgrad_g(X, G, dWt, partial, nsplit, 1, Bn, Ci, Co, K1, m2, stream);
}

BLINDNO_API int blindno_mix1d(const float* At, const float* Wt, float* Xs, float* Z, int Bn,
                              int Ci, int Co, int m, int P2, int dir, void* stream) {
  if (m > P2 / 2 + 1) return (int)hipErrorInvalidValue;
  const int64_t t1 = (int64_t)Bn * m * (dir == 0 ? Co : Ci);
  const int64_t t2 = (int64_t)Bn * m * (dir == 0 ? Ci : Co);
  dim3 g(grid_for(t1 > t2 ? t1 : t2, kBlock, 65536));
  hipStream_t st = (hipStream_t)stream;
  if (dir == 0)
    mix1d_kernel<0><<<g, kBlock, 0, st>>>((const float2*)At, (const float2*)Wt, (float2*)Xs,
                                          (float2*)Z, Bn, Ci, Co, m, P2);
  else
    mix1d_kernel<1><<<g, kBlock, 0, st>>>((const float2*)At, (const float2*)Wt, (float2*)Xs,
                                          (float2*)Z, Bn, Ci, Co, m, P2);
  return (int)hipGetLastError();
}

BLINDNO_API int blindno_pack_w2d(const float* w1, const float* w2, float* Wt, int Ci, int Co,
                                 int m1, int m2, int P1, void* stream) {
  if (m1 > P1) return (int)hipErrorInvalidValue;
  const int64_t total = (int64_t)m2 * kept_rows_count(m1, P1) * Ci * Co;
  pack_w2d_kernel<<<grid_for(total), kBlock, 0, (hipStream_t)stream>>>(w1, w2, w1, w2, (float2*)Wt,
                                                                       Ci, Co, m1, m2, P1);
  return (int)hipGetLastError();
}

BLINDNO_API int blindno_pack_w2d_2(const float* w1a, const float* w2a, const float* w1b,
                                   const float* w2b, float* Wt, int Ci, int Co, int m1, int m2,
                                   int P1, void* stream) {
  if (m1 > P1) return (int)hipErrorInvalidValue;
  const int64_t total = (int64_t)m2 * kept_rows_count(m1, P1) * Ci * Co;
  pack_w2d_kernel<<<dim3(grid_for(total), 2), kBlock, 0, (hipStream_t)stream>>>(
      w1a, w2a, w1b, w2b, (float2*)Wt, Ci, Co, m1, m2, P1);
  return (int)hipGetLastError();
}

BLINDNO_API int blindno_unpack_w2d(const float* dWt, float* dw1, float* dw2, int Ci, int Co,
                                   int m1, int m2, int P1, void* stream) {
  if (m1 > P1) return (int)hipErrorInvalidValue;
  const int64_t total = 2 * (int64_t)Ci * Co * m1 * m2;
  unpack_w2d_kernel<<<grid_for(total), kBlock, 0, (hipStream_t)stream>>>(
      (const float2*)dWt, dw1, dw2, dw1, dw2, Ci, Co, m1, m2, P1);
  return (int)hipGetLastError();
}

BLINDNO_API int blindno_unpack_w2d_2(const float* dWt, float* dw1a, float* dw2a, float* dw1b,
                                     float* dw2b, int Ci, int Co, int m1, int m2, int P1,
                                     void* stream) {
  if (m1 > P1) return (int)hipErrorInvalidValue;
  const int64_t total = 2 * (int64_t)Ci * Co * m1 * m2;
  unpack_w2d_kernel<<<dim3(grid_for(total), 2), kBlock, 0, (hipStream_t)stream>>>(
      (const float2*)dWt, dw1a, dw2a, dw1b, dw2b, Ci, Co, m1, m2, P1);
  return (int)hipGetLastError();
}

// Several blindno_pack_w2d in one launch: segment i packs (w1s[i], w2s[i]) of shape
// (Ci, Co, m1, m2) at row count P1 into Wts[i] (m2, K1, Ci, Co) complex -- the spectral weights
// of every layer of one FNO body (or of both grouped heads) before its forward chain.

__global__ __launch_bounds__(kBlock) void pack_w2d_multi_kernel(PackSegs segs) {
  const int b = blockIdx.x;
  int sg = 0;
  while (sg + 1 < segs.nseg && segs.cum[sg + 1] <= b) ++sg;    // uniform scan
  const int Ci = segs.Ci[sg], Co = segs.Co[sg], m1 = segs.m1[sg], m2 = segs.m2[sg];
  const int P1 = segs.P1[sg];
  const int K1 = kept_rows_count(m1, P1);
  const int idx = (b - segs.cum[sg]) * kBlock + threadIdx.x;
  if (idx >= m2 * K1 * Ci * Co) return;
  const int o = idx % Co;
  int t = idx / Co;
  const int i = t % Ci;
  t /= Ci;
  const int j = t % K1;
  const int k = t / K1;
  const int r = kept_row(j, K1, m1, P1);
  const bool second = r >= P1 - m1;
  const float* src = second ? segs.w2[sg] : segs.w1[sg];
  const int jj = second ? r - (P1 - m1) : r;
  const float* p = src + ((((int64_t)i * Co + o) * m1 + jj) * m2 + k) * 2;
  segs.Wt[sg][idx] = make_float2(p[0], p[1]);
}

template <int DIR>
__global__ __launch_bounds__(256) void w2d_transpose_kernel(PackSegs segs) {
  __shared__ float2 tile[32][33];
  w2d_transpose_tile<DIR>(segs, blockIdx.x, threadIdx.x, tile, true);
}

#ifndef W2D_TILED
#define W2D_TILED 1
#endif

BLINDNO_API int blindno_pack_w2d_multi(const void* const* w1s, const void* const* w2s,
                                       void* const* Wts, const int* shapes, int nseg,
                                       void* stream) {
  // shapes: 5 ints per segment (Ci, Co, m1, m2, P1)
  if (nseg < 0) return (int)hipErrorInvalidValue;
  for (int s0 = 0; s0 < nseg; s0 += kPackSegs) {
    PackSegs segs{};
    const int k = nseg - s0 < kPackSegs ? nseg - s0 : kPackSegs;
    segs.nseg = k;
    int64_t blocks = 0;
    for (int i = 0; i < k; ++i) {
      const int* sh = shapes + 5 * (s0 + i);
      if (sh[2] > sh[4] || sh[0] < 1 || sh[1] < 1 || sh[2] < 1 || sh[3] < 1) return (int)hipErrorInvalidValue;
      const int64_t total = (int64_t)sh[3] * kept_rows_count(sh[2], sh[4]) * sh[0] * sh[1];
      if (total >= INT32_MAX) return (int)hipErrorInvalidValue;
      segs.w1[i] = (const float*)w1s[s0 + i];
      segs.w2[i] = (const float*)w2s[s0 + i];
      segs.Wt[i] = (float2*)Wts[s0 + i];
      segs.Ci[i] = sh[0]; segs.Co[i] = sh[1]; segs.m1[i] = sh[2]; segs.m2[i] = sh[3]; segs.P1[i] = sh[4];
      segs.cum[i] = (int)blocks;
      blocks += (total + kBlock - 1) / kBlock;
    }
    segs.cum[k] = (int)blocks;
    if (blocks == 0) continue;
    if (blocks >= INT32_MAX) return (int)hipErrorInvalidValue;
    int64_t tb = 0;
    if (W2D_TILED && w2d_tiled_segs(segs, tb)) {
      w2d_transpose_kernel<0><<<(unsigned)tb, 256, 0, (hipStream_t)stream>>>(segs);
      continue;
    }
    pack_w2d_multi_kernel<<<(unsigned)blocks, kBlock, 0, (hipStream_t)stream>>>(segs);
  }
  return (int)hipGetLastError();
}

// Several unpacks in one launch (blindno.ops.deferred_reductions): segment i = one weight set
// (dWt slice -> dw1, dw2) of shape (Ci, Co, m1, m2) at row count P1; workgroups
// [cum[i], cum[i+1]) cover its 2 Ci Co m1 m2 complex entries, kBlock per workgroup.
constexpr int kUnpackSegs = 16;
struct UnpackSegs {
  const float2* dWt[kUnpackSegs];
  float* dw1[kUnpackSegs];
  float* dw2[kUnpackSegs];
  int Ci[kUnpackSegs], Co[kUnpackSegs], m1[kUnpackSegs], m2[kUnpackSegs], P1[kUnpackSegs];
  int cum[kUnpackSegs + 1];
  int nseg;
};

__global__ __launch_bounds__(kBlock) void unpack_w2d_multi_kernel(UnpackSegs segs) {
  const int b = blockIdx.x;
  int sg = 0;
  while (sg + 1 < segs.nseg && segs.cum[sg + 1] <= b) ++sg;    // uniform scan
  const int Ci = segs.Ci[sg], Co = segs.Co[sg], m1 = segs.m1[sg], m2 = segs.m2[sg];
  const int P1 = segs.P1[sg];
  const int K1 = kept_rows_count(m1, P1);
  const int per = Ci * Co * m1 * m2;
  const int idx = (b - segs.cum[sg]) * kBlock + threadIdx.x;
  if (idx >= 2 * per) return;
  const int which = idx >= per;
  const int e = which ? idx - per : idx;
  const int k = e % m2;
  int t = e / m2;
  const int jj = t % m1;
  t /= m1;
  const int o = t % Co;
  const int i = t / Co;
  int j = -1;
  if (which) {
    const int r = P1 - m1 + jj;
    j = (K1 == P1) ? r : m1 + jj;
  } else if (jj < P1 - m1) {
    j = jj;                       // otherwise shadowed by weights2 (overlapping rows)
  }
  float2 v = make_float2(0.f, 0.f);
  if (j >= 0) v = segs.dWt[sg][(((int64_t)k * K1 + j) * Ci + i) * Co + o];
  float* dst = (which ? segs.dw2[sg] : segs.dw1[sg]) + (int64_t)e * 2;
  dst[0] = v.x;
  dst[1] = v.y;
}

BLINDNO_API int blindno_unpack_w2d_multi(const void* const* dWts, void* const* dw1s,
                                         void* const* dw2s, const int* shapes, int nseg,
                                         void* stream) {
  // shapes: 5 ints per segment (Ci, Co, m1, m2, P1)
  if (nseg < 0) return (int)hipErrorInvalidValue;
  for (int s0 = 0; s0 < nseg; s0 += kUnpackSegs) {
    UnpackSegs segs{};
    const int k = nseg - s0 < kUnpackSegs ? nseg - s0 : kUnpackSegs;
    segs.nseg = k;
    int64_t blocks = 0;
    for (int i = 0; i < k; ++i) {
      const int* sh = shapes + 5 * (s0 + i);
      if (sh[2] > sh[4] || sh[0] < 1 || sh[1] < 1 || sh[2] < 1 || sh[3] < 1) return (int)hipErrorInvalidValue;
      const int64_t total = 2 * (int64_t)sh[0] * sh[1] * sh[2] * sh[3];
      if (total >= INT32_MAX) return (int)hipErrorInvalidValue;
      segs.dWt[i] = (const float2*)dWts[s0 + i];
      segs.dw1[i] = (float*)dw1s[s0 + i];
      segs.dw2[i] = (float*)dw2s[s0 + i];
      segs.Ci[i] = sh[0]; segs.Co[i] = sh[1]; segs.m1[i] = sh[2]; segs.m2[i] = sh[3]; segs.P1[i] = sh[4];
      segs.cum[i] = (int)blocks;
      blocks += (total + kBlock - 1) / kBlock;
    }
    segs.cum[k] = (int)blocks;
    if (blocks == 0) continue;
    if (blocks >= INT32_MAX) return (int)hipErrorInvalidValue;
    if (W2D_TILED) {
      PackSegs ps{};
      ps.nseg = k;
      for (int i = 0; i < k; ++i) {
        ps.w1[i] = segs.dw1[i];
        ps.w2[i] = segs.dw2[i];
        ps.Wt[i] = const_cast<float2*>(segs.dWt[i]);
        ps.Ci[i] = segs.Ci[i]; ps.Co[i] = segs.Co[i]; ps.m1[i] = segs.m1[i];
        ps.m2[i] = segs.m2[i]; ps.P1[i] = segs.P1[i];
      }
      int64_t tb = 0;
      if (w2d_tiled_segs(ps, tb)) {
        w2d_transpose_kernel<1><<<(unsigned)tb, 256, 0, (hipStream_t)stream>>>(ps);
        continue;
      }
    }
    unpack_w2d_multi_kernel<<<(unsigned)blocks, kBlock, 0, (hipStream_t)stream>>>(segs);
  }
  return (int)hipGetLastError();
}

BLINDNO_API int blindno_pack_w1d(const float* w, float* Wt, int Ci, int Co, int m, int dir,
                                 void* stream) {
  const int64_t total = (int64_t)Ci * Co * m;
  pack_w1d_kernel<<<grid_for(total), kBlock, 0, (hipStream_t)stream>>>(
      (const float2*)w, (float2*)Wt, Ci, Co, m, dir);
  return (int)hipGetLastError();
}
