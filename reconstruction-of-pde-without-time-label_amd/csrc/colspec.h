// The column pass of a 2D spectral layer folded into the row kernels that surround it
// (FNO_input of the snapshot encoder: C = 4 channels, m1 = 12 -> K1 = 24 kept frequency rows,
// m2 = 12 column modes; 2d_FPE/FNOModules.py:156-178, 226-232).
//
// The separate column pass (colfuse_kernel) read the row spectrum At and wrote the row
// coefficients Z of every layer: 2 x 18 MB round trips plus a launch per layer at config C.
// Here only the K1 x m2 column spectrum crosses kernels:
//   * CD ("column DFT"): the row kernel that produces At (the row DFT, or the row inverse that
//     takes the next layer's row DFT in its pass) also takes At's column DFT over its own
//     16-row block, Xs_blk[k][c][j] = sum_{h in blk} At[h][k][c] F[h][j] (F = e^{-2 pi i r_j h / P1}),
//     and writes it as a per-block partial (fixed layout, below);
//   * colmix (colspec.hip): sums the P1 / 16 block partials of a sample in block order (fixed
//     order, deterministic), forms the saved spectrum Xs and the mixed spectrum Y as the column
//     pass did (Y = c_k / (P1 P2) sum_c Xs W, or the adjoint's conj(W) mix);
//   * ZY ("Z from Y"): the next row inverse rebuilds the row coefficients of its 16 rows,
//     Z[h][k][c] = sum_j Y[k][c][j] conj(F[h][j]), on the matrix cores in its prologue (72
//     v_mfma_f32_16x16x4f32 per 16-row block), straight into its B-operand registers.
// Both folded GEMMs read the twiddles (cos, sin)(2 pi r_j h / P1) of their 16 rows straight from
// global memory (L2-resident, 30 KB per layout at P1 = 160), in two layouts: Tab[h][2 j + p] for
// ZY (a lane streams one row) and TabT[h / 4][2 j + p][h % 4] for CD (a lane takes four rows of
// one (j, p)).  No LDS staging: it kept two workgroups per CU at most.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "wgrad.h"

namespace blindno {

typedef float cs_f32x4 __attribute__((ext_vector_type(4)));

constexpr int kCsK1 = 24;                  // kept frequency rows (m1 = 12)
constexpr int kCsMT2 = 2 * kCsK1 / 16;     // 16-row M tiles of the column DFT (rows (j, p))
constexpr int kCsKQ = kCsK1 / 4;           // complex Y values per lane and k in the ZY GEMM

struct SpecCol {
  const float* Y;     // ZY: Y[n][k][c][j] (complex, j < K1) from colmix; nullptr: read Z
  float* part;        // CD: per-block partials (layout below); nullptr: write At instead
  const float* tab;   // Tab[h][2 K1]
  const float* tabT;  // TabT[h / 4][2 K1][4]
  int nblk;           // CD: 16-row blocks per sample in the partial buffer (P1 / 16)
  int w3;             // launch choice: the 3-wave register budget (rowinv.hip, MODE 0)
  // the bag-mean gradient of the encoder's last layer formed on load (BagDz, below): the
  // adjoint's dz argument is then the bag projection's v
  const float* dzg;   // ghat (B, S): the bag-level upstream gradient, S = Ho Wo
  const float* dzl;   // lw (U) multiplicity weights, NULL: 1 / U
  int dzU, dzWo, dzS;
  // spectral weight gradients hosted by the launch (nmixb > 0): workgroups nmain .. run the
  // nmj jobs mj (job q owns mcum[q] .. mcum[q + 1] - 1 of them), independent of the row kernel
  int nmain, nmixb, nmj;
  int mcum[3];
  MixWgradJob mj[2];
};

// dz of the encoder's last layer (csrc/bagproj.hip): dz[b U + l][c][h][w] = lw_l ghat[b][h Wo + w]
// v[b U + l][c][h][w] on the Ho x Wo crop.  Its consumers form it on load from v instead of the
// projection backward writing it (one field write and read less per step).
__device__ __forceinline__ float bagdz_scale(const float* lw, int U, int l) {
  return lw ? lw[l] : 1.0f / (float)U;
}

// Partials of one (sample n, 16-row block b): NCH chunks of 64 lanes x float2,
//   part[((n nblk + b) NCH + ch) 128 + 2 lane + e],
// lane = 16 g + c16 holding Xs_part[k][c][j] component q = c16 & 1 (0: Re, 1: Im),
// j = 8 mt2 + 2 g + e.  The row spectrum's NNT = ceil(2 m2 / 16) column tiles: NF full ones,
//   ch = (c NF + nt) MT2 + mt2,              k = 8 nt + (c16 >> 1),
// and, when 2 m2 % 16 == 8 (m2 = 12: columns 16..23 of the second tile), a half tile whose 8
// live columns of channels 2p and 2p + 1 share one chunk (a quarter less partial traffic):
//   ch = (C NF + p) MT2 + mt2,  c = 2 p + (c16 >> 3),  k = 8 (NNT - 1) + ((c16 & 7) >> 1).
struct ColspecGeom {
  int NNT, NF, half, nch;
};
__host__ __device__ __forceinline__ ColspecGeom colspec_geom(int C, int m2) {
  ColspecGeom g;
  g.NNT = (2 * m2 + 15) / 16;
  g.half = (2 * m2) % 16 == 8 ? 1 : 0;
  g.NF = g.NNT - g.half;
  g.nch = (C * g.NF + (g.half ? (C + 1) / 2 : 0)) * kCsMT2;
  return g;
}
__host__ __device__ __forceinline__ int colspec_nchunk(int C, int m2) { return colspec_geom(C, m2).nch; }

// swap with the neighbouring lane (lane ^ 1): DPP quad_perm [1, 0, 3, 2]
__device__ __forceinline__ float cs_swap1(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false));
}

// CD epilogue of channel c: acc[nt] = At[h0 + 4 g + r][k' = 16 nt + c16] (the row spectrum of
// the block in the MFMA D layout, k' = 2 k + Re/Im), tabT the twiddle table.  Writes the
// channel's chunks of the block at blk = part + (n nblk + b) NCH 128 (layout above; in the half
// tile only lanes c16 < 8 store, at lane + 8 for odd channels).
//   Out[(j, p)][k'] = sum_h F_p[j][h] At[h][k'],  F_0 = cos, F_1 = sin  (A = Tab, B = acc)
//   Xs_re = Out[(j,0)][re] + Out[(j,1)][im],  Xs_im = Out[(j,0)][im] - Out[(j,1)][re]
// rows m = 2 j + p of tile mt2 hold (j = 8 mt2 + 2 g + (r >> 1), p = r & 1) in a lane's D, and
// the Re / Im columns of one mode sit in neighbouring lanes: one DPP swap per pair.
template <int NNT>
__device__ __forceinline__ void cd_store(const cs_f32x4 (&acc)[NNT], const float* __restrict__ tabT,
                                         int h0, int lane, float* __restrict__ blk, int c, int C,
                                         int m2) {
  const int c16 = lane & 15, g = lane >> 4;
  cs_f32x4 ft[kCsMT2];
#pragma unroll
  for (int mt = 0; mt < kCsMT2; ++mt)
    ft[mt] = *reinterpret_cast<const cs_f32x4*>(tabT + (((h0 >> 2) + g) * (2 * kCsK1) + 16 * mt + c16) * 4);
  const float sg = (lane & 1) ? -1.0f : 1.0f;
#pragma unroll
  for (int nt = 0; nt < NNT; ++nt)
#pragma unroll
    for (int mt = 0; mt < kCsMT2; ++mt) {
      cs_f32x4 o = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int r = 0; r < 4; ++r) o = __builtin_amdgcn_mfma_f32_16x16x4f32(ft[mt][r], acc[nt][r], o, 0, 0, 0);
      const float p1 = cs_swap1(o[1]), p3 = cs_swap1(o[3]);
      float2 v;
      v.x = fmaf(sg, p1, o[0]);
      v.y = fmaf(sg, p3, o[2]);
      const ColspecGeom cg = colspec_geom(C, m2);
      if (nt < cg.NF) {
        *reinterpret_cast<float2*>(blk + ((c * cg.NF + nt) * kCsMT2 + mt) * 128 + 2 * lane) = v;
      } else if (c16 < 8) {
        const int ln = (c & 1) ? lane + 8 : lane;
        *reinterpret_cast<float2*>(blk + ((C * cg.NF + (c >> 1)) * kCsMT2 + mt) * 128 + 2 * ln) = v;
      }
    }
}

// ZY prologue: the row coefficients of rows h0 .. h0 + 15 of sample n, as the transposed row
// inverse's B operand zb[c][sp] = Z[h0 + c16][kk = S g + sp][c] (kk = 2 k + Re/Im).
//   D[(kk, c)][h] = sum_{(j, q)} A[(kk, c)][(j, q)] B[(j, q)][h]
//   A: Re rows (Y_re, -Y_im), Im rows (Y_im, Y_re);  B[(j, q)][h] = Tab[h][2 j + q]
// M rows m = 16 mt + 4 g' + r' <-> (kk = S g' + mt, c = r'), so a lane's D of tile mt is
// zb[r][mt]; K index (j, q) = 2 j + q = (K1 / 2) g + s over the K1 / 2 steps s (each lane group
// streams K1 / 4 consecutive complex Y values of one (k, c)).
// (split in two so that the caller can issue its own first loads between them: zy_fetch
// issues the Y loads and the twiddle reads, zy_mfma consumes them)
template <int S, int C>
struct ZyOperands {
  float bt[kCsK1 / 2];
  float yv[S / 2][2 * kCsKQ];
};

template <int S, int C>
__device__ __forceinline__ void zy_fetch(const float* __restrict__ Y, const float* __restrict__ tab,
                                         int n, int m2, int h0, int lane, ZyOperands<S, C>& op) {
  static_assert(C == 4 && S % 2 == 0, "zy_fetch: C = 4, even S");
  const int c16 = lane & 15, g = lane >> 4;
#pragma unroll
  for (int i = 0; i < S / 2; ++i) {
    const int k = (S / 2) * (c16 >> 2) + i;
    const cs_f32x4* yp = reinterpret_cast<const cs_f32x4*>(
        Y + ((((int64_t)n * m2 + k) * C + (c16 & 3)) * kCsK1 + kCsKQ * g) * 2);
#pragma unroll
    for (int q = 0; q < kCsKQ / 2; ++q) {
      const cs_f32x4 v = yp[q];
      op.yv[i][4 * q] = v.x; op.yv[i][4 * q + 1] = v.y; op.yv[i][4 * q + 2] = v.z; op.yv[i][4 * q + 3] = v.w;
    }
  }
  const cs_f32x4* tr = reinterpret_cast<const cs_f32x4*>(tab + (h0 + c16) * (2 * kCsK1) + (kCsK1 / 2) * g);
#pragma unroll
  for (int q = 0; q < kCsK1 / 8; ++q) {
    const cs_f32x4 v = tr[q];
    op.bt[4 * q] = v.x; op.bt[4 * q + 1] = v.y; op.bt[4 * q + 2] = v.z; op.bt[4 * q + 3] = v.w;
  }
}

template <int S, int C>
__device__ __forceinline__ void zy_mfma(const ZyOperands<S, C>& op, float (&zb)[C][S]) {
  cs_f32x4 za[S];
#pragma unroll
  for (int i = 0; i < S; ++i) za[i] = (cs_f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < S / 2; ++i)
#pragma unroll
    for (int s = 0; s < kCsK1 / 2; ++s) {
      const float yr = op.yv[i][2 * (s >> 1)], yi = op.yv[i][2 * (s >> 1) + 1];
      const float are = (s & 1) ? -yi : yr;
      const float aim = (s & 1) ? yr : yi;
      za[2 * i] = __builtin_amdgcn_mfma_f32_16x16x4f32(are, op.bt[s], za[2 * i], 0, 0, 0);
      za[2 * i + 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(aim, op.bt[s], za[2 * i + 1], 0, 0, 0);
    }
#pragma unroll
  for (int c = 0; c < C; ++c)
#pragma unroll
    for (int sp = 0; sp < S; ++sp) zb[c][sp] = za[sp][c];
}

}  // namespace blindno
