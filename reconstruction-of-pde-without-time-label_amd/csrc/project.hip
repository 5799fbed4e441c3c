// Projection MLP of FNO1d/FNO2d on the matrix cores: crop -> fc1 (C -> 128) -> GELU ->
// fc2 (128 -> Cout), forward and backward, with the 128-wide hidden layer never leaving
// registers (2d_FPE/FNOModules.py:234-239, 1d_FPE/FNOModules.py:116-121).
//
// Orientation "points x hidden": a wave takes 16 crop points at a time and sweeps the 8
// hidden tiles of 16 units.  For each tile one v_mfma_f32_16x16x4f32 chain forms
//     H^T (16 pts x 16 hid) = Z^T (16 pts x C) . W1^T (C x 16 hid)          (K = C)
// so lane l holds h for points 4 (l>>4) + r (r < 4) of the tile and hidden unit l & 15.
// The GELU (and in the backward its derivative) is VALU work on those 4 values.  The
// backward keeps the fc1 weight gradient on the matrix cores too, in the same layout:
//     dW1^T-tile (16 hid x 16 cols) += dH (16 hid x 4 pts) . [Z^T | 1] (4 pts x 16 cols)
// where column C of the B operand is 1.0, which accumulates db1 for free; the D-layout rows of
// the forward MFMA are exactly the K index of this one, so no transposition is needed.
// fc2, its gradients and dz = W1^T dH stay on the VALU (they would waste 15/16 or 3/4 of an
// MFMA); dz is summed over the 16 hidden lanes by a reduce-scatter of 4 shuffles.
#include "common.h"
#include "blindno.h"
#include "kernels.h"
#include "gelu_pk.h"

using namespace blindno;
using namespace blindno::gelu_pk;

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kHd = 128;          // fc1 = Linear(width, 128) in every reference FNO
constexpr int kNT = kHd / 16;     // hidden tiles
constexpr int kWaves = 4;
// point tiles per wave step for the width-4 (FNO_input) projections
#ifndef PROJ_FWD_NP4
#define PROJ_FWD_NP4 4
#endif
#ifndef PROJ_BWD_NP4
#define PROJ_BWD_NP4 2
#endif
constexpr int kFwdNP4 = PROJ_FWD_NP4;
// point tiles per wave when sizing the grids (small fields: more workgroups)
#ifndef PF_TPW
#define PF_TPW 2
#endif
// point tiles per wave of the backward (the grid size: the kernel strides over its tiles);
// the grouped 2D heads take PB_TPW_WIDE (project_bwd_mfma_nchunk_tpw): 4 halves their workgroup
// partials (config C 3417 -> 3430 bags/s; 8: 3383, 1: 3405), while the 1D configs lose
// 12-18 % with 4 (profiles/r05/r05u_ab_project_bwd_tpw.txt)
#ifndef PB_TPW
#define PB_TPW 2
#endif
#ifndef PB_TPW_WIDE
#define PB_TPW_WIDE 4
#endif
constexpr int kBwdNP4 = PROJ_BWD_NP4;
// hidden-tile loop unroll of the backward (1: rolled)
// CK >= 8 (the heads' 12 channels), T16: dz = (W1 w2)^T dH on the matrix cores -- dH staged
// through a wave-private LDS tile into the B layout (hidden x points), 4 v_mfma_f32_16x16x4f32 per
// hidden tile into one accumulator -- instead of 2 CK packed FMAs per hidden tile and a
// reduce-scatter of 4 CK values over the 16 hidden lanes per point tile
#ifndef PB_DZMFMA
#define PB_DZMFMA 1
#endif
#ifndef PB_TUNROLL
#define PB_TUNROLL 1
#endif

// Grouped launches: G weight groups (two FNO heads over one field), each owning gpts
// consecutive points (Bg samples); group g's weights sit at + g wgs and its outputs at channel
// offset ooff + g goff of the shared output sample.
constexpr int kMaxGroups = 2;

struct Groups {
  int G;
  unsigned gpts;
  int64_t wgs;
  int goff;
  const float* lscale;   // backward: dout of sample n scaled by lscale[n % dout_div] (nullable)
  FastDiv dHoWo, dWo, dDoutDiv;   // divisors Ho*Wo, Wo, dout_div (backward)
};

struct PointMap {
  unsigned HoWo, Wo;
  int64_t HW;
  int P2, C;
  FastDiv dHoWo, dWo;
  // 32-bit offsets: the launchers require the field to hold < 2^31 elements
  // (project_mfma_ok), so n C HW + h P2 + w never wraps
  __device__ __forceinline__ unsigned zoff(unsigned p, unsigned& n, unsigned& q) const {
    n = dHoWo.div(p);
    q = p - n * HoWo;
    const unsigned h = dWo.div(q), w = q - h * Wo;
    return n * (unsigned)(C * HW) + h * (unsigned)P2 + w;
  }
};

// sum v over the 16 lanes sharing (lane >> 4): butterfly, result in every lane
__device__ __forceinline__ float sum16(float v) {
#pragma unroll
  for (int m = 8; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
  return v;
}

// Weights staged once per workgroup: W1 rows zero-padded to CK, b1, W2 (COM rows).
template <int CK, int COM>
struct ProjWeights {
  float w1[kHd][CK];
  float b1[kHd];
  float w2[COM][kHd];
};

template <int CK, int COM>
__device__ __forceinline__ void stage_weights(ProjWeights<CK, COM>& sw, const float* w1,
                                              const float* b1, const float* w2, int C, int Cout,
                                              float w2scale) {
  for (int e = threadIdx.x; e < kHd * CK; e += blockDim.x) {
    const int j = e / CK, i = e % CK;
    sw.w1[j][i] = i < C ? kK * w1[j * C + i] : 0.f;
  }
  for (int e = threadIdx.x; e < kHd; e += blockDim.x) sw.b1[e] = kK * b1[e];
  for (int e = threadIdx.x; e < COM * kHd; e += blockDim.x) {
    const int c = e / kHd, j = e % kHd;
    sw.w2[c][j] = c < Cout ? w2scale * w2[c * kHd + j] : 0.f;
  }
}

// A operand of fc1 for NP point tiles: lane supplies z[ch 4 kk + g4][pt 16 tile + c16]
template <int KS>
__device__ __forceinline__ void load_az(const float* __restrict__ z, const PointMap& pm,
                                        unsigned p, unsigned npts, int g4, float (&az)[KS]) {
  unsigned n, q;
  const unsigned zo = pm.zoff(p < npts ? p : 0, n, q);
#pragma unroll
  for (int kk = 0; kk < KS; ++kk) {
    const int ch = 4 * kk + g4;
    az[kk] = (p < npts && ch < pm.C) ? z[zo + (unsigned)ch * (unsigned)pm.HW] : 0.f;
  }
}

// Forward: each wave owns NP point tiles (16 points each) per step and sweeps the 8 hidden
// tiles in a rolled loop (weights from LDS), so NP independent MFMA -> GELU chains overlap.
template <int CK, int COM, int NP, bool T16>
__global__ __launch_bounds__(256) void project_fwd_mfma_kernel(
    const float* __restrict__ z, const float* __restrict__ w1, const float* __restrict__ b1,
    const float* __restrict__ w2, const float* __restrict__ b2, float* __restrict__ out, int C,
    int P1, int P2, int Ho, int Wo, int Cout, int ostride, int ooff, unsigned npts, Groups gr) {
  constexpr int KS = CK / 4;
  __shared__ ProjWeights<CK, COM> sws[kMaxGroups];
  for (int g = 0; g < gr.G; ++g)
    stage_weights<CK, COM>(sws[g], w1 + g * gr.wgs, b1 + g * gr.wgs, w2 + g * gr.wgs, C, Cout, kInvK);
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int wave = uniform_int(threadIdx.x >> 6);
  const int c16 = lane & 15, g4 = lane >> 4;
  const PointMap pm{(unsigned)(Ho * Wo), (unsigned)Wo, (int64_t)P1 * P2, P2, C, gr.dHoWo, gr.dWo};
  const unsigned ngroups = (npts + 16 * NP - 1) / (16 * NP);
  for (unsigned grp = blockIdx.x * kWaves + wave; grp < ngroups; grp += gridDim.x * kWaves) {
    // weight group of this step's points (uniform: the launcher checks group alignment)
    const int g = gr.G > 1 ? uniform_int((int)((grp * NP * 16) / gr.gpts)) : 0;
    const ProjWeights<CK, COM>& sw = sws[g];
    float b2v[COM];
#pragma unroll
    for (int c = 0; c < COM; ++c) b2v[c] = c < Cout ? b2[g * gr.wgs + c] : 0.f;
    float az[NP][KS];
#pragma unroll
    for (int np = 0; np < NP; ++np) {
      const unsigned tile = grp * NP + np;
      if constexpr (T16) {           // tile in one grid row: map its first point once (uniform)
        const bool live = tile * 16 < npts;
        unsigned n0, q0;
        const unsigned zo0 = pm.zoff(live ? tile * 16 : 0u, n0, q0);
#pragma unroll
        for (int kk = 0; kk < KS; ++kk) {
          const int ch = 4 * kk + g4;
          az[np][kk] = (live && ch < C) ? z[zo0 + (unsigned)c16 + (unsigned)ch * (unsigned)pm.HW] : 0.f;
        }
      } else {
        load_az<KS>(z, pm, tile * 16 + c16, npts, g4, az[np]);
      }
    }
    f32x2 acc[NP][COM][2];                        // (r0, r1), (r2, r3)
#pragma unroll
    for (int np = 0; np < NP; ++np)
#pragma unroll
      for (int c = 0; c < COM; ++c) acc[np][c][0] = acc[np][c][1] = (f32x2){0.f, 0.f};
#pragma unroll 1
    for (int t = 0; t < kNT; ++t) {
      const int j = 16 * t + c16;
      float bw[KS];
#pragma unroll
      for (int kk = 0; kk < KS; ++kk) bw[kk] = sw.w1[j][4 * kk + g4];
      const float bb = sw.b1[j];
      float w2v[COM];
#pragma unroll
      for (int c = 0; c < COM; ++c) w2v[c] = sw.w2[c][j];
#pragma unroll
      for (int np = 0; np < NP; ++np) {
        f32x4 d = {bb, bb, bb, bb};
#pragma unroll
        for (int kk = 0; kk < KS; ++kk) d = __builtin_amdgcn_mfma_f32_16x16x4f32(az[np][kk], bw[kk], d, 0, 0, 0);
        const f32x2 hh[2] = {{d[0], d[1]}, {d[2], d[3]}};
        f32x2 cdf[2];
        norm_cdf_pairs<2>(hh, cdf);                                 // both pairs in lockstep
        const f32x2 g01 = hh[0] * cdf[0];                           // k GELU
        const f32x2 g23 = hh[1] * cdf[1];
#pragma unroll
        for (int c = 0; c < COM; ++c) {
          const f32x2 wv = splat2(w2v[c]);
          acc[np][c][0] = pk_fma(wv, g01, acc[np][c][0]);
          acc[np][c][1] = pk_fma(wv, g23, acc[np][c][1]);
        }
      }
    }
    // fc2: sum over the 16 hidden lanes; lane with c16 == r (< 4) writes point 4 g4 + r
#pragma unroll
    for (int np = 0; np < NP; ++np) {
      float accs[COM][4];
#pragma unroll
      for (int c = 0; c < COM; ++c) {
        accs[c][0] = sum16(acc[np][c][0].x);
        accs[c][1] = sum16(acc[np][c][0].y);
        accs[c][2] = sum16(acc[np][c][1].x);
        accs[c][3] = sum16(acc[np][c][1].y);
      }
      if (c16 < 4) {
        const unsigned p = (grp * NP + np) * 16 + 4 * g4 + c16;
        if (p < npts) {
          float* op = out + (int64_t)(p - g * gr.gpts) * ostride + ooff + g * gr.goff;
#pragma unroll
          for (int c = 0; c < COM; ++c) {
            float v = accs[c][0];
            if (c16 == 1) v = accs[c][1];
            if (c16 == 2) v = accs[c][2];
            if (c16 == 3) v = accs[c][3];
            if (c < Cout) op[c] = v + b2v[c];
          }
        }
      }
    }
  }
}

// Backward.  Per wave and NP point tiles: recompute H^T (MFMA), GELU and GELU' (VALU),
// dH = (W2^T g) * GELU', accumulate dW2 (VALU) and dW1 / db1 (MFMA) -- both kept per lane in
// LDS between steps because the hidden-tile loop is rolled -- and dz = W1^T dH (VALU,
// summed over the 16 hidden lanes by a reduce-scatter of four shuffles per value block).
// The four waves of a workgroup fold their accumulators into one partial per workgroup
// (fixed order; reduced afterwards by blindno_reduce_partials).
template <int CK, int COM, int NP, bool T16>
__global__ __launch_bounds__(256) void project_bwd_mfma_kernel(
    const float* __restrict__ z, const float* __restrict__ w1, const float* __restrict__ b1,
    const float* __restrict__ w2, const float* __restrict__ dout, float* __restrict__ dz,
    float* __restrict__ partial, int C, int P1, int P2, int Ho, int Wo, int Cout, int ostride,
    int ooff, int dout_div, unsigned gpts, Groups gr) {
  // blockIdx.y = weight group g: points [g gpts, (g+1) gpts), weights at + g wgs, dout sample
  // n - g Bg at channel offset ooff + g goff, partial[blockIdx.x][g]
  constexpr int KS = CK / 4;
  const int g = blockIdx.y;
  w1 += g * gr.wgs;
  b1 += g * gr.wgs;
  w2 += g * gr.wgs;
  const unsigned pbase = g * gpts, npts = pbase + gpts;
  const unsigned nbase = g * (gpts / (unsigned)(Ho * Wo));
  constexpr int NV = 4 * CK;                       // dz values per lane per tile: (ch, r)
  __shared__ ProjWeights<CK, COM> sw;
  // dW1 (/ db1) accumulators in MFMA D layout.  CK == 4: v_mfma_f32_4x4x1f32, 16 blocks of
  // (4 hidden x 4 channels), block b = 4 g4 + (c16 >> 2) <-> hidden 4 (c16 >> 2) + reg, channel
  // c16 & 3, K = one point of group g4 per instruction; db1 then sums on the VALU (sgb1).
  // CK > 4: v_mfma_f32_16x16x4f32 against [Z^T | 1] (column C = db1).
  constexpr bool kGW44 = CK == 4;
  constexpr bool kFoldW2 = COM == 1;
  __shared__ f32x4 sgw1[kWaves][kNT][64];
  __shared__ float sgb1[kWaves][kNT][64];
  __shared__ float sgw2[kWaves][kNT][COM][64];     // dW2 accumulators (lane = hidden c16)
  __shared__ float sdh[PB_DZMFMA && CK >= 8 ? kWaves : 1][16 * 17];   // dH transpose tiles
  stage_weights<CK, COM>(sw, w1, b1, w2, C, Cout, 1.0f);
  const int lane = threadIdx.x & 63;
  const int wave = uniform_int(threadIdx.x >> 6);
  const int c16 = lane & 15, g4 = lane >> 4;
  for (int t = 0; t < kNT; ++t) {
    sgw1[wave][t][lane] = (f32x4){0.f, 0.f, 0.f, 0.f};
    sgb1[wave][t][lane] = 0.f;
#pragma unroll
    for (int c = 0; c < COM; ++c) sgw2[wave][t][c][lane] = 0.f;
  }
  __syncthreads();
  float gb2[COM];
#pragma unroll
  for (int c = 0; c < COM; ++c) gb2[c] = 0.f;
  const PointMap pm{(unsigned)(Ho * Wo), (unsigned)Wo, (int64_t)P1 * P2, P2, C, gr.dHoWo, gr.dWo};
  const bool row4 = (Wo & 3) == 0;
  const unsigned ntiles = (gpts + 15) / 16;
  const unsigned ngroups = (gpts + 16 * NP - 1) / (16 * NP);
  for (unsigned grp = blockIdx.x * kWaves + wave; grp < ngroups; grp += gridDim.x * kWaves) {
    float az[NP][KS], zb[NP][4], gv[NP][4][COM];
    int zo4[NP][4];                                 // element offsets (< 2^31, checked)
#pragma unroll
    for (int np = 0; np < NP; ++np) {
      const unsigned tile = grp * NP + np;
      if constexpr (T16) {
        // Wo % 16 == 0: the tile's 16 points lie in one grid row of one sample, so its first
        // point is mapped once, wave-uniformly (scalar unit), and every lane point is an offset
        // (lane c16 for the A operand, 4 g4 + r for the D-layout rows).  A tile past the end
        // (last step, odd tile count) is uniformly dead.
        const bool live = tile < ntiles;
        unsigned n0, q0;
        const unsigned zo0 = pm.zoff(pbase + (live ? tile : 0u) * 16u, n0, q0);
        const unsigned nb = gr.dDoutDiv.div(n0 - nbase);
        const float ls = gr.lscale ? gr.lscale[(n0 - nbase) - nb * (unsigned)dout_div] : 1.0f;
        const float* gp0 = dout + ((nb * pm.HoWo + q0) * (unsigned)ostride + (unsigned)(ooff + g * gr.goff));
#pragma unroll
        for (int kk = 0; kk < KS; ++kk) {
          const int ch = 4 * kk + g4;
          az[np][kk] = (live && ch < C) ? z[zo0 + (unsigned)c16 + (unsigned)ch * (unsigned)pm.HW] : 0.f;
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const unsigned off = 4u * g4 + r;
          zo4[np][r] = (int)(zo0 + off);
          const int zc = kGW44 ? (c16 & 3) : c16;
          zb[np][r] = !live ? 0.f : (zc < C ? z[zo0 + off + (unsigned)zc * (unsigned)pm.HW] : (zc == C ? 1.f : 0.f));
#pragma unroll
          for (int c = 0; c < COM; ++c) gv[np][r][c] = (live && c < Cout) ? gp0[off * (unsigned)ostride + c] * ls : 0.f;
        }
        if (c16 == 0) {
#pragma unroll
          for (int c = 0; c < COM; ++c) gb2[c] += (gv[np][0][c] + gv[np][1][c]) + (gv[np][2][c] + gv[np][3][c]);
        }
        continue;
      }
      load_az<KS>(z, pm, pbase + tile * 16 + c16, npts, g4, az[np]);
      // this lane's 4 points (D layout rows): z column c16 (1.0 at c16 == C: db1), dout
      // When Wo % 4 == 0 the lane's 4 points (4-aligned) share one sample and grid row, so one
      // point -> offset mapping serves all four (row4, kernel-uniform)
      unsigned zo = 0, n = 0, q = 0;
      const float* gp = dout;
      float ls = 1.0f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const unsigned p = pbase + tile * 16 + 4 * g4 + r;
        const bool ok = p < npts;
        if (r == 0 || !row4) {
          zo = pm.zoff(ok ? p : 0, n, q);
          const unsigned nb = gr.dDoutDiv.div(n - nbase);
          gp = dout + ((nb * pm.HoWo + q) * (unsigned)ostride + (unsigned)(ooff + g * gr.goff));
          ls = gr.lscale ? gr.lscale[(n - nbase) - nb * (unsigned)dout_div] : 1.0f;
        } else {
          zo += 1;
          gp += ostride;
        }
        zo4[np][r] = (int)zo;
        const int zc = kGW44 ? (c16 & 3) : c16;
        zb[np][r] = !ok ? 0.f : (zc < C ? z[zo + (unsigned)zc * (unsigned)pm.HW] : (zc == C ? 1.f : 0.f));
#pragma unroll
        for (int c = 0; c < COM; ++c) gv[np][r][c] = (ok && c < Cout) ? gp[c] * ls : 0.f;
      }
      if (c16 == 0) {
#pragma unroll
        for (int c = 0; c < COM; ++c) gb2[c] += (gv[np][0][c] + gv[np][1][c]) + (gv[np][2][c] + gv[np][3][c]);
      }
    }
    constexpr bool kDzM = PB_DZMFMA && CK >= 8 && NP == 1 && T16;
    float dzp[kDzM ? 1 : NP][kDzM ? 1 : NV];
#pragma unroll
    for (int np = 0; np < (kDzM ? 1 : NP); ++np)
#pragma unroll
      for (int e = 0; e < (kDzM ? 1 : NV); ++e) dzp[np][e] = 0.f;
    f32x4 dzacc = {0.f, 0.f, 0.f, 0.f};            // kDzM: D[channel 4 g4 + r][point c16]
#pragma unroll PB_TUNROLL
    for (int t = 0; t < kNT; ++t) {
      const int j = 16 * t + c16;
      float bw[KS], wr[CK];
#pragma unroll
      for (int kk = 0; kk < KS; ++kk) bw[kk] = sw.w1[j][4 * kk + g4];
      // Cout == 1: W1 rows pre-multiplied by w2_j, so dz = (W1 w2)^T (gout GELU') with no
      // per-value w2 product; dW1 / db1 take the w2_j factor at the fold
      const float w2f = kFoldW2 ? sw.w2[0][j] : 1.0f;
#pragma unroll
      for (int i = 0; i < CK; i += 4) {
        const float4 v = *reinterpret_cast<const float4*>(&sw.w1[j][i]);
        wr[i] = v.x * w2f; wr[i + 1] = v.y * w2f; wr[i + 2] = v.z * w2f; wr[i + 3] = v.w * w2f;
      }
      const float bb = sw.b1[j];
      float w2v[COM];
      f32x2 gw2[COM];
#pragma unroll
      for (int c = 0; c < COM; ++c) {
        w2v[c] = sw.w2[c][j];
        gw2[c] = (f32x2){sgw2[wave][t][c][lane], 0.f};
      }
      f32x4 gw1 = sgw1[wave][t][lane];
      float gb1 = kGW44 ? sgb1[wave][t][lane] : 0.f;
#pragma unroll
      for (int np = 0; np < NP; ++np) {
        f32x4 d = {bb, bb, bb, bb};
#pragma unroll
        for (int kk = 0; kk < KS; ++kk) d = __builtin_amdgcn_mfma_f32_16x16x4f32(az[np][kk], bw[kk], d, 0, 0, 0);
        const f32x2 h01 = {d[0], d[1]}, h23 = {d[2], d[3]};
        const f32x2 hh[2] = {h01, h23};
        f32x2 cdfv[2], epv[2];
        norm_cdf_pdf_pairs<2>(hh, cdfv, epv);                       // both pairs in lockstep
        const f32x2 cdf01 = cdfv[0], cdf23 = cdfv[1], ep01 = epv[0], ep23 = epv[1];
        f32x2 da01 = {0.f, 0.f}, da23 = {0.f, 0.f};
#pragma unroll
        for (int c = 0; c < COM; ++c) {
          const f32x2 g01v = {gv[np][0][c], gv[np][1][c]}, g23v = {gv[np][2][c], gv[np][3][c]};
          if constexpr (kFoldW2) {
            da01 = g01v;
            da23 = g23v;
          } else {
            const f32x2 wv = splat2(w2v[c]);
            da01 = pk_fma(wv, g01v, da01);
            da23 = pk_fma(wv, g23v, da23);
          }
          // k dW2 (scaled at the fold), pair accumulators
          gw2[c] = pk_fma(g01v, h01 * cdf01, gw2[c]);
          gw2[c] = pk_fma(g23v, h23 * cdf23, gw2[c]);
        }
        // GELU' = Phi + h phi  (dh / w2_j when folded)
        const f32x2 dh01 = da01 * pk_fma(h01, ep01, cdf01);
        const f32x2 dh23 = da23 * pk_fma(h23, ep23, cdf23);
        const float dh[4] = {dh01.x, dh01.y, dh23.x, dh23.y};
        if constexpr (kDzM) {
          // dH (points 4 g4 + r, hidden c16) -> wave-private LDS [hidden][point] -> B operands
          // (hidden 4 g4 + r, point c16); A = row c16 (channel) of (W1 w2)^T
          float* sd = sdh[wave];
#pragma unroll
          for (int r = 0; r < 4; ++r) sd[c16 * 17 + 4 * g4 + r] = dh[r];
          // the tile is shared by the wave's lanes: order the writes before the cross-lane
          // reads, and the reads before the next point tile's writes (LDS ops of one wave
          // complete in order; the barrier keeps the compiler from moving them across)
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
          float bv[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) bv[r] = sd[(4 * g4 + r) * 17 + c16];
          __builtin_amdgcn_wave_barrier();
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int jr = 16 * t + 4 * g4 + r;
            const float a = c16 < C ? sw.w1[jr][c16] * (kFoldW2 ? sw.w2[0][jr] : 1.0f) : 0.f;
            dzacc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bv[r], dzacc, 0, 0, 0);
          }
        } else {
#pragma unroll
          for (int i = 0; i < CK; ++i) {                               // k dz (scaled at the store)
            const f32x2 wi = {wr[i], wr[i]};
            f32x2 p01 = {dzp[np][i * 4 + 0], dzp[np][i * 4 + 1]};
            f32x2 p23 = {dzp[np][i * 4 + 2], dzp[np][i * 4 + 3]};
            p01 = __builtin_elementwise_fma(dh01, wi, p01);
            p23 = __builtin_elementwise_fma(dh23, wi, p23);
            dzp[np][i * 4 + 0] = p01.x; dzp[np][i * 4 + 1] = p01.y;
            dzp[np][i * 4 + 2] = p23.x; dzp[np][i * 4 + 3] = p23.y;
          }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          if constexpr (kGW44) gw1 = __builtin_amdgcn_mfma_f32_4x4x1f32(dh[r], zb[np][r], gw1, 0, 0, 0);
          else gw1 = __builtin_amdgcn_mfma_f32_16x16x4f32(dh[r], zb[np][r], gw1, 0, 0, 0);
        }
        if constexpr (kGW44) gb1 += (dh[0] + dh[1]) + (dh[2] + dh[3]);
      }
      sgw1[wave][t][lane] = gw1;
      if constexpr (kGW44) sgb1[wave][t][lane] = gb1;
#pragma unroll
      for (int c = 0; c < COM; ++c) sgw2[wave][t][c][lane] = gw2[c].x + gw2[c].y;
    }
    if constexpr (kDzM) {
      // lane (g4, c16): channels 4 g4 + r of point c16 of the tile (one sample row: T16)
      const unsigned tile = grp;
      if (tile < ntiles) {
        unsigned n0, q0;
        const unsigned zo0 = pm.zoff(pbase + tile * 16u, n0, q0);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int ch = 4 * g4 + r;
          if (ch < C) dz[zo0 + (unsigned)c16 + (unsigned)ch * (unsigned)pm.HW] = kInvK * dzacc[r];
        }
      }
      continue;
    }
    // reduce-scatter dzp over the 16 hidden lanes: lane keeps value index e = 16 m + c16,
    // i.e. channel 4 m + (c16 >> 2), point 4 g4 + (c16 & 3)
#pragma unroll
    for (int np = 0; np < (kDzM ? 1 : NP); ++np) {
#pragma unroll
      for (int s = 8; s >= 1; s >>= 1) {
        const bool up = (c16 & s) != 0;
#pragma unroll
        for (int e = 0; e < NV; ++e) {
          if ((e & 15) >= s) continue;          // live pairs: (e, e + s) in each 16-block
          const float keep = up ? dzp[np][e + s] : dzp[np][e];
          const float send = up ? dzp[np][e] : dzp[np][e + s];
          dzp[np][e] = keep + __shfl_xor(send, s, 64);
        }
      }
      const int r = c16 & 3;
      const unsigned p = pbase + (grp * NP + np) * 16 + 4 * g4 + r;
      if (T16 ? (grp * NP + np) < ntiles : p < npts) {
#pragma unroll
        for (int m = 0; m < NV / 16; ++m) {
          const int ch = 4 * m + (c16 >> 2);
          if (ch < C) dz[(unsigned)zo4[np][r] + (unsigned)ch * (unsigned)pm.HW] = kInvK * dzp[np][16 * m];
        }
      }
    }
  }
  // ---- fold the accumulators of the four waves into this workgroup's partial
  // layout: [dW1 (Hd*C) | db1 (Hd) | dW2 (Cout*Hd) | db2 (Cout)]
  __shared__ float sgb2[kWaves][COM];
#pragma unroll
  for (int c = 0; c < COM; ++c) {
    const float v = wave_sum(gb2[c]);
    if (lane == 0) sgb2[wave][c] = v;
  }
  __syncthreads();
  const int np_ = kHd * C + kHd + Cout * kHd + Cout;
  float* pp = partial + ((int64_t)blockIdx.x * gridDim.y + g) * np_;
  for (int e = threadIdx.x; e < np_; e += blockDim.x) {
    float v = 0.f;
    if (e < kHd * C + kHd) {
      const int j = e < kHd * C ? e / C : e - kHd * C;
      const int col = e < kHd * C ? e % C : C;
      const int t = j >> 4, row = j & 15;
      if (kGW44) {
        // hidden row = 4 hg + r'; dW1: lanes 16 g4 + 4 hg + col, reg r' (all four point groups);
        // db1: lanes 16 g4 + row
        const int hg = row >> 2, rr = row & 3;
#pragma unroll
        for (int w = 0; w < kWaves; ++w)
#pragma unroll
          for (int g = 0; g < 4; ++g)
            v += col < C ? sgw1[w][t][16 * g + 4 * hg + col][rr] : sgb1[w][t][16 * g + row];
      } else {
        // 16x16 D layout: t = j/16, row = j%16 = 4 g4 + r, lane = 16 g4 + col
        const int ln = 16 * (row >> 2) + col, r = row & 3;
#pragma unroll
        for (int w = 0; w < kWaves; ++w) v += sgw1[w][t][ln][r];
      }
      if (kFoldW2) v *= sw.w2[0][j];
    } else if (e < kHd * C + kHd + Cout * kHd) {
      const int q = e - kHd * C - kHd, c = q / kHd, j = q % kHd;
      const int t = j >> 4, cl = j & 15;
#pragma unroll
      for (int w = 0; w < kWaves; ++w)
#pragma unroll
        for (int g = 0; g < 4; ++g) v += sgw2[w][t][c][16 * g + cl];
      v *= kInvK;
    } else {
      const int c = e - kHd * C - kHd - Cout * kHd;
#pragma unroll
      for (int w = 0; w < kWaves; ++w) v += sgb2[w][c];
    }
    pp[e] = v;
  }
}

}  // namespace

namespace blindno {

bool project_mfma_ok(int C, int Hd, int Cout, int64_t field_elems) {
  return Hd == kHd && C >= 1 && C <= 15 && Cout >= 1 && Cout <= 2 && field_elems < INT32_MAX;
}

int project_fwd_mfma(const float* z, const float* w1, const float* b1, const float* w2,
                     const float* b2, float* out, int Bn, int C, int P1, int P2, int Ho, int Wo,
                     int Cout, int ostride, int ooff, int G, int64_t wgs, hipStream_t st) {
  if (G < 1 || G > kMaxGroups || Bn % G) return (int)hipErrorInvalidValue;
  const unsigned npts = (unsigned)((int64_t)Bn * Ho * Wo);
  const Groups gr{G, npts / (unsigned)G, G > 1 ? wgs : 0, Cout, nullptr,
                  FastDiv::make((unsigned)(Ho * Wo)), FastDiv::make((unsigned)Wo), FastDiv::make(1)};
  const unsigned ntiles = (npts + 15) / 16;
  unsigned blocks = (ntiles + kWaves * PF_TPW - 1) / (kWaves * PF_TPW);
  if (blocks > 2048) blocks = 2048;
  if (blocks < 1) blocks = 1;
  const int ck = (C + 3) / 4 * 4;
  const int np = ck <= 4 ? kFwdNP4 : (ck <= 8 ? 4 : 2);
  if (G > 1 && gr.gpts % (16u * np)) return (int)hipErrorInvalidValue;   // steps within a group
  const bool t16 = Wo % 16 == 0;
#define PF2(CK_, CO_, T_)                                                                      \
  project_fwd_mfma_kernel<CK_, CO_, (CK_ <= 4 ? kFwdNP4 : (CK_ <= 8 ? 4 : 2)), T_><<<blocks, 256, 0, st>>>( \
      z, w1, b1, w2, b2, out, C, P1, P2, Ho, Wo, Cout, ostride, ooff, npts, gr)
#define PF(CK_, CO_) do { if (t16) PF2(CK_, CO_, true); else PF2(CK_, CO_, false); } while (0)
  if (Cout == 1) {
    if (ck == 4) PF(4, 1); else if (ck == 8) PF(8, 1); else if (ck == 12) PF(12, 1); else PF(16, 1);
  } else {
    if (ck == 4) PF(4, 2); else if (ck == 8) PF(8, 2); else if (ck == 12) PF(12, 2); else PF(16, 2);
  }
#undef PF
#undef PF2
  return (int)hipGetLastError();
}

int project_bwd_mfma_nchunk_tpw(int64_t npts, int tpw) {
  const int64_t tiles = (npts + 15) / 16;
  int64_t b = (tiles + kWaves * tpw - 1) / (kWaves * tpw);
  return (int)(b < 1 ? 1 : (b > 1024 ? 1024 : b));
}

int project_bwd_mfma_nchunk(int64_t npts) { return project_bwd_mfma_nchunk_tpw(npts, PB_TPW); }

int project_bwd_mfma_nchunk_wide(int64_t npts) {
  return project_bwd_mfma_nchunk_tpw(npts, PB_TPW_WIDE);
}

int project_bwd_mfma(const float* z, const float* w1, const float* b1, const float* w2,
                     const float* dout, float* dz, float* partial, int nchunk, int Bn, int C,
                     int P1, int P2, int Ho, int Wo, int Cout, int ostride, int ooff,
                     int dout_div, int G, int64_t wgs, hipStream_t st, const float* lscale) {
  if (G < 1 || G > kMaxGroups || Bn % G || dout_div < 1) return (int)hipErrorInvalidValue;
  // 32-bit dout offsets (see PointMap)
  if ((int64_t)(Bn / G / dout_div + 1) * Ho * Wo * ostride + ooff + Cout >= INT32_MAX)
    return (int)hipErrorInvalidValue;
  const unsigned gpts = (unsigned)((int64_t)(Bn / G) * Ho * Wo);
  const Groups gr{G, gpts, G > 1 ? wgs : 0, Cout, lscale, FastDiv::make((unsigned)(Ho * Wo)),
                  FastDiv::make((unsigned)Wo), FastDiv::make((unsigned)dout_div)};
  const dim3 grid(nchunk, G);
  const bool t16 = Wo % 16 == 0;
#define PB2(CK_, CO_, T_)                                                                     \
  project_bwd_mfma_kernel<CK_, CO_, (CK_ <= 4 ? kBwdNP4 : 1), T_><<<grid, 256, 0, st>>>(        \
      z, w1, b1, w2, dout, dz, partial, C, P1, P2, Ho, Wo, Cout, ostride, ooff, dout_div, gpts, gr)
#define PB(CK_, CO_) do { if (t16) PB2(CK_, CO_, true); else PB2(CK_, CO_, false); } while (0)
  const int ck = (C + 3) / 4 * 4;
  if (Cout == 1) {
    if (ck == 4) PB(4, 1); else if (ck == 8) PB(8, 1); else if (ck == 12) PB(12, 1); else PB(16, 1);
  } else {
    if (ck == 4) PB(4, 2); else if (ck == 8) PB(8, 2); else if (ck == 12) PB(12, 2); else PB(16, 2);
  }
#undef PB
#undef PB2
  return (int)hipGetLastError();
}

}  // namespace blindno
