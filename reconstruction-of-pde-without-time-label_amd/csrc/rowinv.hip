// Inverse row transform of the spectral layers on the matrix cores, with the FNO layer
// epilogue fused (irfft2 second stage + nn.Conv2d(k=1) + bias + residual add, and the GELU of
// the layer input; 2d_FPE/FNOModules.py:177,226-232; 1d_FPE/FNOModules.py:58,108-114) and its
// adjoint (with the GELU' of the layer input and, for narrow fields, the 1x1-conv weight
// gradient reduced in the same pass).
//
// GEMM view: for a group of 4 grid rows (n, h) and 4 channels,
//     out[(row, c)][w] = sum_k Re(Z[row][k][c] e^{+2 pi i k w / P2})
//                      = sum_kk A[(row, c)][kk] B[kk][w],   kk = 2 k + part,
//     A = (Re Z, Im Z) interleaved,  B = (cos, -sin)(2 pi k w / P2)
// one v_mfma_f32_16x16x4f32 chain of ceil(m2 / 2) steps per 16-column tile: M = 16 = (4 rows x
// 4 channels), N = 16 columns, K = 2 m2.  The D layout puts rows 4 (l>>4) + r of column l & 15 in
// lane l; with M index 4 row + channel, lane l therefore holds ALL FOUR channels of one point
// (row l>>4, column l&15), so the 1x1 conv / bias / GELU epilogue stays in registers.  Wider
// fields (the C = 12 heads) run as channel groups of 4.  The B operand comes from a host-built
// image in MFMA lane order (twiddle_rowinv, staged once per workgroup in LDS).
#include "common.h"
#include "blindno.h"
#include "gelu_pk.h"
#include "kernels.h"
#include "colspec.h"

using namespace blindno;

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kW = 4;      // waves per workgroup

// Snapshot-encoder lift source (LIFT kernels): the layer input is x0 = fc0([u, gx, gy]),
// zero outside the N1 x N2 crop, recomputed from the bag tensor instead of being stored.
struct BagLift {
  const float* X;      // bags (B, T, N1, N2); snapshot n = b L + l -> X[b][idx[l]]
  const int* idx;      // (L,) device indices of the bag draw
  const float* grid;   // (N1, N2, 2)
  const float* w0;     // fc0.weight (C, 3)
  const float* b0;     // fc0.bias (C)
  int T, L, N1, N2;
};

// The next layer's row DFT taken in the row-inverse pass (RD kernels): At (Bn, m2, C, P1, 2) as
// blindno_rowdft writes it, Tp its twiddle image (KB = ceil(P2 / 16), Npad = 16 ceil(2 m2 / 16)),
// act: GELU of the field first (the next layer's input activation).
struct RowDftNext {
  float* At;
  const float* Tp;
  int Npad, act;
};

// MODE 0 (forward epilogue): z = acc + bc + Wc f(x)                (f = GELU if ACT)
// MODE 1 (adjoint):          dx = (acc + Wc^T dz) * (ACT ? GELU'(xsrc) : 1)
//                            + with WG (C <= 4, one group): per-lane dWc / dbc sums
// CM: channel bound of the conv (C rounded up to 4, 8, 16, 32).
// LIFT: the layer input is the snapshot encoder's lifted field (BagLift); MODE 0 recomputes
// x0 for the conv term, MODE 1 (with WG, ACT 0, C <= 4) recomputes it for dWc and, instead of
// writing dx0, reduces fc0's gradient dW0[c][j] = sum dx0[c] [u, gx, gy]_j, db0[c] = sum dx0[c]
// over the crop into partial[..][C*C + C + 4 C] (after the conv terms).
// (The next layer's row DFT in the same pass is rowfuse_kernel's, below.)
template <int CM, int KSM, int MODE, int ACT, int WG, int LDSB, int LIFT>
__global__ __launch_bounds__(256) void rowinv_mfma_kernel(
    const float* __restrict__ Z, const float* __restrict__ xs, const float* __restrict__ dz,
    const float* __restrict__ wc, const float* __restrict__ bc, float* __restrict__ out,
    const float* __restrict__ TB, float* __restrict__ partial, int Bn, int C, int P1, int P2,
    int m2, int TPW, BagLift bl, int Bg, int64_t wgs, int dN1, int dN2) {
  // MODE 1: dz is read only on its valid region h < dN1, w < dN2 (zero elsewhere: the gradient
  // of a cropped FNO output; see rowdft_mfma_kernel)
  extern __shared__ float sTB[];                    // [KS][NT][64] when LDSB
  const int KS = (m2 + 1) >> 1;
  const int NT = (P2 + 15) >> 4;
  if (LDSB) {
    stage_to_lds(sTB, TB, KS * NT * 64);
    __syncthreads();
  }
  const int lane = threadIdx.x & 63;
  const int wave = uniform_int(threadIdx.x >> 6);
  const int c16 = lane & 15, g4 = lane >> 4;
  const int NG = (C + 3) >> 2;                      // channel groups of 4
  const int nrows = Bn * P1;
  const int nquads = (nrows + 3) >> 2;
  const int NC = (NT + TPW - 1) / TPW;              // column chunks per (quad, group)
  const int nitems = nquads * NG * NC;
  const int64_t HW = (int64_t)P1 * P2;
  const bool has_wc = wc != nullptr;
  constexpr int NWC = WG ? CM * CM + CM : 0;      // conv weight / bias sums
  constexpr int NWL = LIFT && MODE == 1 ? 4 * CM : 0;   // fc0 weight / bias sums
  constexpr int NW = NWC + NWL > 0 ? NWC + NWL : 1;
  float wacc[NW];
#pragma unroll
  for (int e = 0; e < NW; ++e) wacc[e] = 0.f;
  for (int item = blockIdx.x * kW + wave; item < nitems; item += gridDim.x * kW) {
    const int chunk = item % NC;
    const int qg = item / NC;
    const int g = qg % NG, quad = qg / NG;
    const int c0 = 4 * g;
    // A operand row of this lane: grid row R0 + (c16 >> 2), channel c0 + (c16 & 3)
    const int ra = 4 * quad + (c16 >> 2), ca = c0 + (c16 & 3);
    const bool aok = ra < nrows && ca < C;
    const float* zrow = Z + ((int64_t)(aok ? ra : 0) * m2) * C * 2;
    float av[KSM];                                  // A operand, reused by every column tile
#pragma unroll
    for (int s = 0; s < KSM; ++s) {
      const int kk = 4 * s + g4;                    // K index supplied by this lane
      const int k = kk >> 1;
      av[s] = (aok && s < KS && k < m2) ? zrow[(k * C + ca) * 2 + (kk & 1)] : 0.f;
    }
    // this lane's output point: row R0 + g4, column 16 tile + c16, channels c0 + r
    const int ro = 4 * quad + g4;
    const bool rok = ro < nrows;
    const int n = rok ? ro / P1 : 0, h = rok ? ro - (ro / P1) * P1 : 0;
    const int64_t rbase = (int64_t)n * C * HW + (int64_t)h * P2;
    // weight group of this quad of rows (two heads batched over one launch: wc / bc at + g wgs;
    // wave-uniform -- the launcher requires P1 % 4 == 0 when grouped -- so the weights stay
    // scalar loads)
    const int64_t goff = wgs ? (int64_t)uniform_int((4 * quad) / P1 / Bg) * wgs : 0;
    const float* wcg = wc + goff;
    const float* bcg = bc + goff;
    const float* urow = nullptr;                    // LIFT: snapshot row / grid row
    const float* grow = nullptr;
    if (LIFT && rok && h < bl.N1) {
      const int b = n / bl.L, l = n - (n / bl.L) * bl.L;
      urow = bl.X + (((int64_t)b * bl.T + bl.idx[l]) * bl.N1 + h) * bl.N2;
      grow = bl.grid + (int64_t)h * bl.N2 * 2;
    }
    const int t0 = chunk * TPW, t1 = min(NT, t0 + TPW);
    // epilogue operands of a column tile (raw loads), fetched one tile ahead so their latency
    // overlaps the previous tile's MFMA chain and epilogue
    struct Ops {
      float fv[CM];        // MODE 0: x of every input channel; MODE 1: dz of every output channel
      float sv[4];         // MODE 1: xsrc of this group's channels
      float lin[3];        // LIFT: [u, gx, gy] at this point
      bool lok;
    };
    auto load_ops = [&](int tile, Ops& o) {
      const int w = 16 * tile + c16;
      const bool pok = rok && w < P2;
      const bool dok = pok && (MODE == 0 || (h < dN1 && w < dN2));
      o.lok = false;
      o.lin[0] = o.lin[1] = o.lin[2] = 0.f;
      if (LIFT) {
        o.lok = pok && urow != nullptr && w < bl.N2;
        if (o.lok) {
          o.lin[0] = urow[w];
          o.lin[1] = grow[2 * w];
          o.lin[2] = grow[2 * w + 1];
        }
      }
#pragma unroll
      for (int i = 0; i < CM; ++i)
        o.fv[i] = (!(LIFT && MODE == 0) && dok && has_wc && i < C)
                      ? (MODE == 0 ? xs[rbase + i * HW + w] : dz[rbase + i * HW + w]) : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r)
        o.sv[r] = (!LIFT && MODE == 1 && (ACT || WG) && pok && c0 + r < C) ? xs[rbase + (c0 + r) * HW + w] : 0.f;
    };
    // (forward epilogue of narrow fields only: the adjoint's and the 12-channel heads' larger
    // operand sets cost more occupancy than the lookahead gains -- measured)
    constexpr bool kPre = MODE == 0 && CM <= 8;
    Ops nx;
    if (kPre) load_ops(t0, nx);
    for (int tile = t0; tile < t1; ++tile) {
      const int w = 16 * tile + c16;
      const bool pok = rok && w < P2;
      float fv[CM], sv[4];
      bool lok = false;
      float lin[3] = {0.f, 0.f, 0.f};
      if constexpr (kPre) {
        const Ops cur = nx;
        if (tile + 1 < t1) load_ops(tile + 1, nx);
        lok = cur.lok;
#pragma unroll
        for (int j = 0; j < 3; ++j) lin[j] = cur.lin[j];
#pragma unroll
        for (int i = 0; i < CM; ++i) fv[i] = cur.fv[i];
#pragma unroll
        for (int r = 0; r < 4; ++r) sv[r] = cur.sv[r];
      } else {
        // operands of this tile, loaded in place (as before the lookahead variant)
        if (LIFT) {
          lok = pok && urow != nullptr && w < bl.N2;
          if (lok) {
            lin[0] = urow[w];
            lin[1] = grow[2 * w];
            lin[2] = grow[2 * w + 1];
          }
        }
        const bool dok = pok && (MODE == 0 || (h < dN1 && w < dN2));
#pragma unroll
        for (int i = 0; i < CM; ++i)
          fv[i] = (!(LIFT && MODE == 0) && dok && has_wc && i < C)
                      ? (MODE == 0 ? xs[rbase + i * HW + w] : dz[rbase + i * HW + w]) : 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r)
          sv[r] = (!LIFT && MODE == 1 && (ACT || WG) && pok && c0 + r < C) ? xs[rbase + (c0 + r) * HW + w] : 0.f;
      }
      auto x0 = [&](int c) -> float {               // the lifted field (0 outside the crop)
        return lok ? fmaf(bl.w0[c * 3], lin[0], fmaf(bl.w0[c * 3 + 1], lin[1],
                                                     fmaf(bl.w0[c * 3 + 2], lin[2], bl.b0[c]))) : 0.f;
      };
      if (LIFT) {
#pragma unroll
        for (int i = 0; i < CM; ++i)
          if (MODE == 0) fv[i] = (has_wc && i < C) ? x0(i) : 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (MODE == 1) sv[r] = c0 + r < C ? x0(c0 + r) : 0.f;
      }
      f32x4 d = {0.f, 0.f, 0.f, 0.f};
      const float* tb = (LDSB ? (const float*)sTB : TB) + tile * 64 + lane;
#pragma unroll
      for (int s = 0; s < KSM; ++s)
        if (s < KS) d = __builtin_amdgcn_mfma_f32_16x16x4f32(av[s], tb[s * NT * 64], d, 0, 0, 0);
      if (pok) {
      if (MODE == 0) {
        if (has_wc) {
          float xv[CM];
#pragma unroll
          for (int i = 0; i < CM; ++i) xv[i] = ACT ? gelu_f(fv[i]) : fv[i];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int o = c0 + r;
            if (o >= C) continue;
            float v = d[r] + bcg[o];
#pragma unroll
            for (int i = 0; i < CM; ++i)
              if (i < C) v = fmaf(wcg[o * C + i], xv[i], v);
            out[rbase + o * HW + w] = v;
          }
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (c0 + r < C) {
              out[rbase + (c0 + r) * HW + w] = d[r];
            }
        }
      } else {
        if (has_wc) {
          float xa[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int i = c0 + r;
            float gi = d[r];
#pragma unroll
            for (int o = 0; o < CM; ++o) gi = fmaf((o < C && i < C) ? wcg[o * C + i] : 0.f, fv[o], gi);
            xa[r] = sv[r];
            if (ACT) {
              float a, dg;
              gelu_both(sv[r], a, dg);
              gi *= dg;
              xa[r] = a;
            }
            if (LIFT) {
              if (i < C && lok) {
#pragma unroll
                for (int j = 0; j < 3; ++j) wacc[NWC + 4 * r + j] = fmaf(gi, lin[j], wacc[NWC + 4 * r + j]);
                wacc[NWC + 4 * r + 3] += gi;
              }
            } else if (i < C) {
              out[rbase + i * HW + w] = gi;
            }
          }
          if constexpr (WG != 0) {
#pragma unroll
            for (int o = 0; o < CM; ++o) {
#pragma unroll
              for (int r = 0; r < 4; ++r)
                if (r < CM) wacc[o * CM + r] = fmaf(fv[o], xa[r], wacc[o * CM + r]);
              wacc[CM * CM + o] += fv[o];
            }
          }
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (c0 + r < C) {
              out[rbase + (c0 + r) * HW + w] = d[r];
            }
        }
      }
      }  // pok
    }
  }
  if (WG) {
    // block reduction of the per-lane partials -> partial[blockIdx.x][np],
    // np = C*C + C (+ 4 C for LIFT: dW0 (C x 3) then db0 (C))
    __syncthreads();
    float* red = sTB;                               // reuse LDS (sized by the launcher)
    const int np = C * C + C + (NWL ? 4 * C : 0);
#pragma unroll
    for (int e = 0; e < NW; ++e) {
      int pidx;
      if (e < CM * CM) {
        const int o = e / CM, i = e % CM;
        if (o >= C || i >= C) continue;
        pidx = o * C + i;
      } else if (e < NWC) {
        const int o = e - CM * CM;
        if (o >= C) continue;
        pidx = C * C + o;
      } else {
        const int c = (e - NWC) >> 2, j = (e - NWC) & 3;
        if (c >= C) continue;
        pidx = C * C + C + (j < 3 ? c * 3 + j : 3 * C + c);
      }
      const float s = wave_sum(wacc[e]);
      if (lane == 0) red[wave * np + pidx] = s;
      __builtin_amdgcn_sched_barrier(0);
    }
    __syncthreads();
    for (int p = threadIdx.x; p < np; p += blockDim.x) {
      float s = 0.f;
      for (int w = 0; w < kW; ++w) s += red[w * np + p];
      partial[(int64_t)blockIdx.x * np + p] = s;
    }
  }
}

// Wide fields (C = 8, 12, 16: the FNO heads, C = 12).  One work item = 4 grid rows x TPW
// column tiles x ALL channel groups (the kernel above takes one group per item): the layer
// input (MODE 0) or dz (MODE 1) of a point is loaded and GELU'd once instead of once per group,
// the twiddle operand is loaded once per tile for every group, and the groups' MFMA chains
// share it.  The spectrum arrives in A-tile order (rowinv_tile_layout: colidft writes it so),
// so each A operand is one coalesced 256-B load; gathered from the [row][k][c] order instead,
// those loads were half of the kernel's time (measured).  Items run XCD-major (xcd_block) so
// the column tiles of one row quad read its spectrum through one L2.  The 1x1 conv weights (C x
// C + C per weight group, transposed for MODE 1) sit in LDS: as scalar operands they would not
// fit the SGPR file.  No weight-gradient or LIFT variants (C > 4 uses conv_wgrad).
constexpr int kWideMaxG = 4;
#ifndef ROWINV_WIDE_WAVES
#define ROWINV_WIDE_WAVES 2
#endif
// EX (the heads' m2 = 32): budgeted for 4 waves per SIMD (128 VGPRs, a few spilled).  At 3
// waves (136-146 VGPRs) the grouped heads' 3200 one-tile items took 800 workgroups for 768
// resident slots, and the last 32 ran as a second round (bench +1.9 %, r06y)
#ifndef ROWINV_WIDE_WAVES_EX
#define ROWINV_WIDE_WAVES_EX 4
#endif
#ifndef ROWINV_WIDE_PROBE
#define ROWINV_WIDE_PROBE 0
#endif
#if ROWINV_WIDE_PROBE
// diagnostic build only (tools/kbench.py with KBENCH_PROBE=2): per-wave realtime stamps
__device__ unsigned long long g_rowinv_wide_probe[8192 * 8];
#define RW_MARK(i)                                                                          \
  do {                                                                                      \
    __builtin_amdgcn_sched_barrier(0);                                                      \
    const unsigned long long t_ = __builtin_amdgcn_s_memrealtime();                         \
    const int slot_ = blockIdx.x * 4 + (threadIdx.x >> 6);                                  \
    if ((threadIdx.x & 63) == 0 && slot_ < 8192) g_rowinv_wide_probe[slot_ * 8 + (i)] = t_; \
    __builtin_amdgcn_sched_barrier(0);                                                      \
  } while (0)
#else
#define RW_MARK(i) do {} while (0)
#endif
// EX: m2 == 2 KSM (the heads: m2 = 32), every mode bound a compile-time constant
template <int CM, int KSM, int MODE, int ACT, bool EX>
__global__ __launch_bounds__(256, EX ? ROWINV_WIDE_WAVES_EX : ROWINV_WIDE_WAVES) void rowinv_wide_kernel(
    const float* __restrict__ Z, const float* __restrict__ xs, const float* __restrict__ dz,
    const float* __restrict__ wc, const float* __restrict__ bc, float* __restrict__ out,
    const float* __restrict__ TB, int Bn, int P1, int P2, int m2_, int TPW, int Bg,
    int64_t wgs) {
  constexpr int NGM = CM / 4;
  constexpr int C = CM;
  const int m2 = EX ? 2 * KSM : m2_;
  const int KS = m2 >> 1;                           // m2 even (rowinv_tile_layout)
  const int NT = (P2 + 15) >> 4;
  const int lane = threadIdx.x & 63;
  const int wave = uniform_int(threadIdx.x >> 6);
  const int c16 = lane & 15, g4 = lane >> 4;
  const int nrows = Bn * P1;                        // a multiple of 4
  const int nquads = nrows >> 2;
  const int NC = (NT + TPW - 1) / TPW;
  const int nitems = nquads * NC;
  const int HW = P1 * P2;                           // field < 2^31 elements (launcher)
  const bool has_wc = wc != nullptr;
  // conv weights of every weight group: [g][c][i] = wc[c][i] (MODE 0) or wc[i][c] (MODE 1),
  // then the bias
  constexpr int per = CM * CM + CM;
  __shared__ float swc[kWideMaxG][per];
  const int ngw = wgs ? Bn / Bg : 1;
  RW_MARK(0);
  if (has_wc) {
    for (int e = threadIdx.x; e < ngw * per; e += blockDim.x) {
      const int g = e / per, q = e - g * per;
      float v = 0.f;
      if (q < CM * CM) {
        const int a = q / CM, b = q - (q / CM) * CM;
        v = MODE == 0 ? wc[g * wgs + a * C + b] : wc[g * wgs + b * C + a];
      } else if (MODE == 0) {
        v = bc[g * wgs + q - CM * CM];
      }
      swc[g][q] = v;
    }
    __syncthreads();
  }
  const int vb = xcd_block(blockIdx.x, gridDim.x);
  RW_MARK(1);
  for (int item = vb * kW + wave; item < nitems; item += gridDim.x * kW) {
    const int chunk = item % NC, quad = item / NC;
    // A operands of every group: one coalesced load per (group, K step), tile order
    float av[NGM][KSM];
#pragma unroll
    for (int g = 0; g < NGM; ++g)
#pragma unroll
      for (int s = 0; s < KSM; ++s)
        av[g][s] = s < KS ? Z[(unsigned)(((quad * NGM + g) * KS + s) * 64 + lane)] : 0.f;
    // this lane's output point: row 4 quad + g4, column 16 tile + c16, channels 4 g + r.
    // 32-bit element offsets from the uniform bases: one VGPR per address
    const int ro = 4 * quad + g4;
    const int n = ro / P1, h = ro - (ro / P1) * P1;
    const unsigned rbase = (unsigned)(n * C * HW + h * P2);
    const float* sw = swc[wgs ? uniform_int((4 * quad) / P1 / Bg) : 0];
    const int t0 = chunk * TPW, t1 = min(NT, t0 + TPW);
    for (int tile = t0; tile < t1; ++tile) {
      const int w = 16 * tile + c16;
      const bool pok = w < P2;
      float fv[CM], sv[CM], bv[KSM];
#pragma unroll
      for (int s = 0; s < KSM; ++s) bv[s] = s < KS ? TB[(unsigned)((s * NT + tile) * 64 + lane)] : 0.f;
#pragma unroll
      for (int i = 0; i < CM; ++i) {
        // unconditional loads from clamped offsets, then a select: a guarded load per value
        // would be a branch with its own saved exec mask (SGPR pressure -> spills)
        const unsigned off = pok ? rbase + (unsigned)(i * HW + w) : 0u;
        fv[i] = 0.f;
        sv[i] = 0.f;
        if (has_wc) {
          const float v = (MODE == 0 ? xs : dz)[off];
          fv[i] = pok ? v : 0.f;
          if (MODE == 1 && ACT) {
            const float u = xs[off];
            sv[i] = pok ? u : 0.f;
          }
        }
      }
      if (MODE == 0 && ACT) {
#pragma unroll
        for (int i = 0; i < CM; ++i) fv[i] = gelu_f(fv[i]);
      }
      if (MODE == 1 && ACT) {
#pragma unroll
        for (int i = 0; i < CM; ++i) sv[i] = gelu_grad_f(sv[i]);
      }
#if ROWINV_WIDE_PROBE
      if (tile == t0) {
        // the operands are in registers once every load has returned
        float s_ = fv[0] + sv[0] + bv[0] + av[0][0] + av[NGM - 1][KSM - 1];
        asm volatile("" :: "v"(s_));
        RW_MARK(2);
      }
#endif
#pragma unroll
      for (int g = 0; g < NGM; ++g) {
        f32x4 d = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < KSM; ++s)
          if (s < KS) d = __builtin_amdgcn_mfma_f32_16x16x4f32(av[g][s], bv[s], d, 0, 0, 0);
        if (!pok) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int c = 4 * g + r;
          float v = d[r];
          if (has_wc) {
            // row c of the staged (MODE 0) or transposed (MODE 1) conv weights
            if (MODE == 0) v += sw[CM * CM + c];
#pragma unroll
            for (int i = 0; i < CM; i += 4) {
              const float4 wv = *reinterpret_cast<const float4*>(sw + c * CM + i);
              v = fmaf(wv.x, fv[i], v);
              v = fmaf(wv.y, fv[i + 1], v);
              v = fmaf(wv.z, fv[i + 2], v);
              v = fmaf(wv.w, fv[i + 3], v);
            }
            if (MODE == 1 && ACT) v *= sv[c];
          }
          out[rbase + (unsigned)(c * HW + w)] = v;
        }
      }
    }
#if ROWINV_WIDE_PROBE
    if (item == vb * kW + wave) RW_MARK(3);
#endif
  }
  RW_MARK(4);
}
#if ROWINV_WIDE_PROBE
BLINDNO_API int blindno_rowinv_wide_probe_reset() {
  void* p = nullptr;
  if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_rowinv_wide_probe)) != hipSuccess) return 1;
  return (int)hipMemset(p, 0, sizeof(g_rowinv_wide_probe));
}
BLINDNO_API int blindno_rowinv_wide_probe_read(unsigned long long* dst, int n) {
  return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_rowinv_wide_probe),
                                  sizeof(unsigned long long) * (size_t)n, 0, hipMemcpyDeviceToHost);
}
#endif

// ------------------------------------------------------------ transposed row inverse (C = 4)
// The snapshot encoder's layers (FNO_input: C = 4, m2 = 12, P2 = 160 at 128^2), whole rows per
// work item.  The row inverse is taken TRANSPOSED: for a block of 16 rows (sample n, rows
// h0 .. h0 + 15) and a 16-column tile t,
//     D_c[w][h] = sum_kk T'[kk][w] Z[n][h][kk][c]        (A = twiddles, B = the spectrum)
// so the D layout puts 4 CONSECUTIVE columns w = 16 t + 4 (l>>4) + r of one row h = h0 + (l&15)
// in lane l.  Consequences:
//   * every field operand and result of the epilogue is one 16-B access per channel (a wave
//     instruction covers 16 rows x 64 contiguous bytes; the next tile's instruction the other
//     half of each 128-B line), where the untransposed kernel above issues 4-B accesses;
//   * the field values a lane produces are exactly the operand the next layer's row DFT takes
//     from that lane (rowdft_mfma_kernel's k order w = 16 kb + 4 kq + s), so the RD fusion runs
//     straight from registers, with no LDS transposition (the earlier RD variant's cost);
//   * the row DFT is taken transposed as well (D = T^T f(y)^T): lane l then holds spectrum
//     columns k' = 16 nt + 4 (l>>4) + r of row h, i.e. whole (Re, Im) pairs, stored as float2.
// K order of the row inverse: lane group g = l>>4 supplies kk = S g + s' (s' < S = m2 / 2), i.e.
// the S/2 complex modes S g / 2 .. of all 4 channels: 4 S contiguous floats of the spectrum row
// (one float4 per K step).  The twiddle image of the untransposed kernel (twiddle_rowinv, K order
// 4 s + g) is permuted into this order while it is staged.
// MODE / ACT / WG / LIFT as rowinv_mfma_kernel; RD: 0 none, 1 next row DFT of the field, 2 of
// GELU(field).  S = m2 / 2 (m2 % 4 == 0, m2 <= 16); P1 % 16 == 0, P2 % 32 == 0.
// the epilogue GELUs of the transposed kernel on packed fp32 pairs (gelu_pk.h: the same A&S
// evaluation, two values per v_pk instruction)
#ifndef ROWFUSE_PKGELU
#define ROWFUSE_PKGELU 1
#endif
__device__ __forceinline__ f32x4 gelu4(f32x4 x) {
#if ROWFUSE_PKGELU
  using namespace blindno::gelu_pk;
  // both pairs in lockstep (norm_cdf_pairs): no wait state between dependent packed steps
  const f32x2 v[2] = {{x[0], x[1]}, {x[2], x[3]}};
  const f32x2 hk[2] = {v[0] * splat2(kK), v[1] * splat2(kK)};
  f32x2 cdf[2];
  norm_cdf_pairs<2>(hk, cdf);
  const f32x2 g0 = v[0] * cdf[0], g1 = v[1] * cdf[1];
  return (f32x4){g0.x, g0.y, g1.x, g1.y};
#else
  return (f32x4){gelu_f(x[0]), gelu_f(x[1]), gelu_f(x[2]), gelu_f(x[3])};
#endif
}
// GELU and GELU' of four values (the adjoint's input activation and its derivative)
__device__ __forceinline__ void gelu_both4(f32x4 x, f32x4& a, f32x4& dg) {
#if ROWFUSE_PKGELU
  using namespace blindno::gelu_pk;
  const f32x2 v[2] = {{x[0], x[1]}, {x[2], x[3]}};
  const f32x2 hk[2] = {v[0] * splat2(kK), v[1] * splat2(kK)};
  f32x2 cdf[2], ep[2];
  norm_cdf_pdf_pairs<2>(hk, cdf, ep);
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const f32x2 gv = v[i] * cdf[i];
    const f32x2 dv = pk_fma(hk[i], ep[i], cdf[i]);    // Phi + h phi(h)
    a[2 * i] = gv.x;
    a[2 * i + 1] = gv.y;
    dg[2 * i] = dv.x;
    dg[2 * i + 1] = dv.y;
  }
#else
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float ar, dr;
    gelu_both(x[r], ar, dr);
    a[r] = ar;
    dg[r] = dr;
  }
#endif
}
// timing experiments only (wrong results): RF_GELU(x) = x drops the epilogue GELUs, RF_NORD
// the next layer's row-DFT MFMAs
#ifndef RF_GELU
#define RF_GELU(x) gelu4(x)
#endif
#ifndef RF_NORD
#define RF_NORD 0
#endif
#ifndef ROWFUSE_BLOCKS
#define ROWFUSE_BLOCKS 512
#endif
#ifndef ROWFUSE_ZPRE
#define ROWFUSE_ZPRE 0
#endif
#ifndef ROWFUSE_STAGE_N
#define ROWFUSE_STAGE_N 16
#endif
// operand prefetch (ping-pong buffers) in the adjoint
#ifndef ROWFUSE_PF1
#define ROWFUSE_PF1 1
#endif
// NH column tiles per step (1 or 2): with NH = 2 lane group g owns the 8 consecutive columns
// w = 32 st + 8 g + 4 hf + r of a 32-column step (hf: the step's two MFMA tiles), so the two
// 16-B accesses a lane issues per channel and step are adjacent and each pair of wave
// instructions covers whole 128-B lines of 16 rows (NH = 1: 64-B half lines, the other halves
// one step later).  The MFMA row i of tile (st, hf) is column w = 16 NH st + 4 NH (i>>2) + 4 hf
// + (i&3); the staged twiddle images follow that order.
// (per mode: the adjoint carries twice the operands, so NH = 2 costs it occupancy)
#ifndef ROWFUSE_NH0
#define ROWFUSE_NH0 2
#endif
#ifndef ROWFUSE_NH1
#define ROWFUSE_NH1 1
#endif
#ifndef ROWFUSE_NH0_NORD
#define ROWFUSE_NH0_NORD 2
#endif

#ifndef ROWFUSE_PROBE
#define ROWFUSE_PROBE 0
#endif
#if ROWFUSE_PROBE
// diagnostic build only (tools/kbench.py with KBENCH_PROBE=1): per-wave realtime stamps
__device__ unsigned long long g_rowfuse_probe[8192 * 8];
#define RF_MARK(i)                                                                          \
  do {                                                                                      \
    __builtin_amdgcn_sched_barrier(0);                                                      \
    const unsigned long long t_ = __builtin_amdgcn_s_memrealtime();                         \
    const int slot_ = blockIdx.x * 4 + (threadIdx.x >> 6);                                  \
    if ((threadIdx.x & 63) == 0 && slot_ < 8192) g_rowfuse_probe[slot_ * 8 + (i)] = t_;     \
    __builtin_amdgcn_sched_barrier(0);                                                      \
  } while (0)
#else
#define RF_MARK(i) do {} while (0)
#endif
// HW: the layer has its 1x1 conv (wc != NULL) -- a compile-time flag: a runtime test around each
// operand load made hipcc branch around the loads and count their waits conservatively.
// NSC: steps per row block as a compile-time constant (P2 / (16 NH)), 0 = a runtime loop.
// ZY / CD (colspec.h): the row coefficients built from the mixed column spectrum sc.Y in the
// prologue of each 16-row block instead of read as Z; the next row DFT taken in the opposite
// orientation (D = f(y) T: rows on the M side) and its column DFT over the block written as
// partials to sc.part instead of At.
// ZW: waves per SIMD the registers are budgeted for (0: unconstrained, two at most for the
// kernels with the next row DFT).  The persistent grid of 4-wave workgroups at 2 waves per SIMD
// holds 2048 16-row work items at once; beyond that the rest ran as a second round (Bn = 208
// snapshots = 2080 items: 75 us, where 2000 items took 56).  The MODE 0 ZY / CD kernels take a
// 3-wave budget (one column tile per step) when their items fit 3072 slots but not 2048
// DZB (MODE 1): dz = lw_l ghat v formed on load (SpecCol.dzg / dzl; the dz argument is v)
template <int MODE, int ACT, int WG, int LIFT, int RD, int S, int NH, bool HW_ = true, int NSC = 0,
          bool ZY = false, bool CD = false, int ZW = 0, bool DZB = false>
__global__ __launch_bounds__(256, ZW > 0 ? ZW : 1)
void rowfuse_kernel(
    const float* __restrict__ Z, const float* __restrict__ xs, const float* __restrict__ dz,
    const float* __restrict__ wc, const float* __restrict__ bc, float* __restrict__ out,
    const float* __restrict__ TB, float* __restrict__ partial, int Bn, int P1, int P2,
    BagLift bl, int dN1, int dN2, RowDftNext rd, SpecCol sc) {
  constexpr int C = 4;
  constexpr int m2 = 2 * S;
  constexpr int NNT = (4 * S + 15) / 16;          // 16-column tiles of the next row DFT
  constexpr int Npad = 16 * NNT;
  static_assert(!CD || RD, "CD takes the column DFT of the next row DFT");
  // hosted spectral weight gradients (SpecCol.mj): only the encoder's first-layer adjoint
  // (MODE 1, LIFT) takes them -- the branch costs the other forms registers
  constexpr bool kHost = MODE == 1 && LIFT;
  if constexpr (kHost) {
    if (sc.nmixb > 0 && (int)blockIdx.x >= sc.nmain) {
      int r = (int)blockIdx.x - sc.nmain;
      const int q = (sc.nmj > 1 && r >= sc.mcum[1]) ? 1 : 0;
      r -= sc.mcum[q];
      const MixWgradJob& mj = sc.mj[q];
      mix_wgrad_block(mj.X, mj.Gs, mj.out, mj.Bn, mj.Ci, mj.Co, mj.K1, mj.m2, r % mj.gx,
                      (r / mj.gx) % mj.gy, r / (mj.gx * mj.gy), mj.gx, mj.gy, mj.gz);
      return;
    }
  }
  const int gxm = (kHost && sc.nmixb > 0) ? sc.nmain : (int)gridDim.x;   // the row kernel's grid
  RF_MARK(0);
#if ROWFUSE_PROBE
  if ((threadIdx.x & 63) == 0 && blockIdx.x * 4 + (threadIdx.x >> 6) < 8192)
    for (int i = 2; i < 7; ++i) g_rowfuse_probe[(blockIdx.x * 4 + (threadIdx.x >> 6)) * 8 + i] = 0;
  int it_probe = 0;
#endif
  const int NT = P2 >> 4;                           // MFMA column tiles (NT % NH == 0)
  extern __shared__ float lds[];
  float* sA = lds;                                  // [NT][64 lanes][S]
  float* sT = lds + NT * 64 * S;                    // RD: [NT][4][Npad][4] (rowdft's image)

  auto tb_at = [&](int e) {
    const int t = e / (64 * S), rem = e - t * (64 * S);
    const int ln = rem / S, sp = rem - ln * S;
    const int kk = S * (ln >> 4) + sp;
    const int w = 16 * NH * (t / NH) + 4 * NH * ((ln & 15) >> 2) + 4 * (t % NH) + (ln & 3);
    return TB[((kk >> 2) * NT + (w >> 4)) * 64 + (kk & 3) * 16 + (w & 15)];
  };
  {
    // the twiddle image, read in TB order (coalesced) and scattered into LDS: sA[tb_slot(q)] =
    // TB[q] (the inverse of tb_at, a bijection of the NT 64 S slots).  Gathered in sA order, every
    // wave load touched up to 64 cache lines and the staging took ~4.5 us per workgroup
    // (per-wave stamps, kbench KBENCH_PROBE); the first ROWFUSE_STAGE_N values per thread are
    // loaded together, the next row DFT's image staged while they are in flight
    static_assert(NH == 1 || NH == 2, "column tiles per step");
    const int n = NT * 64 * S, st = blockDim.x;
    auto tb_slot = [&](int q) {
      const int s4 = q / (NT * 64), r = q - s4 * (NT * 64);
      const int l64 = r & 63, w = 16 * (r >> 6) + (l64 & 15);
      const int kk = 4 * s4 + (l64 >> 4), lg = kk / S, sp = kk - lg * S;
      int t, lo;
      if (NH == 1) {
        t = w >> 4;
        lo = w & 15;
      } else {
        t = 2 * (w >> 5) + ((w >> 2) & 1);
        lo = 4 * ((w & 31) >> 3) + (w & 3);
      }
      return (t * 64 + 16 * lg + lo) * S + sp;
    };
    int e = threadIdx.x;
#if ROWFUSE_STAGE_N > 0
    float v0[ROWFUSE_STAGE_N];
#pragma unroll
    for (int j = 0; j < ROWFUSE_STAGE_N; ++j) {
      const int ej = e + j * st;
      v0[j] = TB[ej < n ? ej : n - 1];
    }
    if (RD) stage_to_lds(sT, rd.Tp, NT * 16 * Npad);
#pragma unroll
    for (int j = 0; j < ROWFUSE_STAGE_N; ++j)
      if (e + j * st < n) sA[tb_slot(e + j * st)] = v0[j];
    e += ROWFUSE_STAGE_N * st;
    for (; e < n; e += st) sA[tb_slot(e)] = TB[e];
#else
    for (; e + 3 * st < n; e += 4 * st) {
      float v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = tb_at(e + j * st);
#pragma unroll
      for (int j = 0; j < 4; ++j) sA[e + j * st] = v[j];
    }
    for (; e < n; e += st) sA[e] = tb_at(e);
    if (RD) stage_to_lds(sT, rd.Tp, NT * 16 * Npad);
#endif
  }
  __syncthreads();
  RF_MARK(1);
  const int lane = threadIdx.x & 63;
  const int wave = uniform_int(threadIdx.x >> 6);
  const int c16 = lane & 15, g = lane >> 4;
  // MODE 0 without the next row DFT: the output is written on its crop h < dN1, w < dN2 only
  // (the encoder's last layer, read by the projection on the crop alone): whole 16-row blocks and
  // 16 NH-column steps past the crop are skipped
  constexpr bool OCROP = MODE == 0 && RD == 0;
  const int HB = OCROP ? (dN1 + 15) >> 4 : P1 >> 4;
  const int nitems = Bn * HB;
  const int HW = P1 * P2;                           // field < 2^31 elements (launcher)
  const int NS = OCROP ? (dN2 + 16 * NH - 1) / (16 * NH) : NT / NH;   // steps per row block
  constexpr bool has_wc = HW_;
  float W[C][C], bv[C], w0[C][3], b0[C];
#pragma unroll
  for (int o = 0; o < C; ++o) {
    bv[o] = (MODE == 0 && has_wc && bc) ? bc[o] : 0.f;
#pragma unroll
    for (int i = 0; i < C; ++i) W[o][i] = has_wc ? wc[o * C + i] : 0.f;
    b0[o] = LIFT ? bl.b0[o] : 0.f;
#pragma unroll
    for (int j = 0; j < 3; ++j) w0[o][j] = LIFT ? bl.w0[o * 3 + j] : 0.f;
  }
  constexpr int NWC = WG ? C * C + C : 0;          // [o][i] dWc, then dbc
  constexpr int NWL = (LIFT && MODE == 1) ? 4 * C : 0;   // [c][j] dW0, then db0
  constexpr int NW = NWC + NWL > 0 ? NWC + NWL : 1;
  float wacc[NW];
#pragma unroll
  for (int e = 0; e < NW; ++e) wacc[e] = 0.f;
  const f32x4 zero4 = {0.f, 0.f, 0.f, 0.f};
  // the spectrum rows (B operand) of a work item: 4 S contiguous floats per lane; the next
  // item's are loaded while this one runs (ROWFUSE_ZPRE), so only a wave's first item waits
  auto load_z = [&](int item, f32x4 (&zr)[S]) {
    const int it = item < nitems ? item : nitems - 1;
    const int n = it / HB;
    const int h = ((it - n * HB) << 4) + c16;
    const f32x4* src = reinterpret_cast<const f32x4*>(Z + (int64_t)(n * P1 + h) * (m2 * C * 2) + 4 * S * g);
#pragma unroll
    for (int q = 0; q < S; ++q) zr[q] = src[q];
  };
  f32x4 znext[S];
  const int item0 = blockIdx.x * kW + wave;
  if (ROWFUSE_ZPRE && !ZY) load_z(item0, znext);
  for (int item = item0; item < nitems; item += gxm * kW) {
    const int n = item / HB;
    const int h0 = (item - n * HB) << 4;
    const int h = h0 + c16;
    float zb[C][S];
    // ZY: the Y loads go out first; the row coefficients are formed after the first field
    // loads are issued (below), so their latencies overlap
    ZyOperands<ZY ? S : 2, C> zop;
    if constexpr (ZY) {
      zy_fetch<S, C>(sc.Y, sc.tab, n, m2, h0, lane, zop);
    } else {
      f32x4 zcur[S];
      if (ROWFUSE_ZPRE) {
#pragma unroll
        for (int q = 0; q < S; ++q) zcur[q] = znext[q];
      } else {
        load_z(item, zcur);
      }
      float zz[4 * S];
#pragma unroll
      for (int q = 0; q < S; ++q) {
        const f32x4 v = zcur[q];
        zz[4 * q] = v.x; zz[4 * q + 1] = v.y; zz[4 * q + 2] = v.z; zz[4 * q + 3] = v.w;
      }
#pragma unroll
      for (int c = 0; c < C; ++c)
#pragma unroll
        for (int sp = 0; sp < S; ++sp) zb[c][sp] = zz[((sp >> 1) * C + c) * 2 + (sp & 1)];
    }
    const int64_t fbase = (int64_t)n * C * HW + (int64_t)h * P2;
    const float* urow = bl.X;
    const float* grow = bl.grid;
    const bool lrow = LIFT && h < bl.N1;
    if (LIFT && lrow) {
      const int b = n / bl.L, l = n - (n / bl.L) * bl.L;
      urow = bl.X + (((int64_t)b * bl.T + bl.idx[l]) * bl.N1 + h) * bl.N2;
      grow = bl.grid + (int64_t)h * bl.N2 * 2;
    }
    const bool drow = MODE == 0 || h < dN1;
    // DZB: this item's ghat row and lw_l (dz = lw_l ghat v on the dN1 x dN2 crop)
    const float* dzrow = sc.dzg;
    float dzlw = 0.f;
    if constexpr (DZB) {
      const int b = n / sc.dzU, l = n - b * sc.dzU;
      dzrow = sc.dzg + (int64_t)b * sc.dzS + (int64_t)(drow ? h : 0) * sc.dzWo;
      dzlw = bagdz_scale(sc.dzl, sc.dzU, l);
    }
    // field operands of one step: 16-B loads from clamped offsets, then selects
    struct Ops {
      f32x4 a[C][NH];      // MODE 0: layer input x; MODE 1: dz of every output channel
      f32x4 s[C][NH];      // MODE 1: the layer input (GELU' / dWc)
      f32x4 u[NH], g0[NH], g1[NH];   // LIFT: snapshot and grid (gx, gy interleaved)
      bool lok[NH];
    };
    auto load = [&](int st, Ops& o) {
#pragma unroll
      for (int hf = 0; hf < NH; ++hf) {
        const int w = 16 * NH * st + 4 * NH * g + 4 * hf;
        f32x4 gsc = zero4;                           // DZB: lw_l ghat of the lane's 4 points
        if constexpr (DZB && MODE == 1) {
          const bool ok = drow && w < dN2;
          const f32x4 gv = *reinterpret_cast<const f32x4*>(dzrow + (ok ? w : 0));
          gsc = ok ? gv * dzlw : zero4;
        }
#pragma unroll
        for (int c = 0; c < C; ++c) {
          o.a[c][hf] = zero4;
          o.s[c][hf] = zero4;
          if (MODE == 0 && !LIFT && has_wc) o.a[c][hf] = *reinterpret_cast<const f32x4*>(xs + fbase + c * HW + w);
          if (MODE == 1 && has_wc) {
            const bool ok = drow && w < dN2;
            const f32x4 v = *reinterpret_cast<const f32x4*>(dz + (ok ? fbase + c * HW + w : 0));
            if constexpr (DZB) o.a[c][hf] = ok ? v * gsc : zero4;
            else o.a[c][hf] = ok ? v : zero4;
          }
          if (MODE == 1 && !LIFT && (ACT || WG))
            o.s[c][hf] = *reinterpret_cast<const f32x4*>(xs + fbase + c * HW + w);
        }
        o.lok[hf] = false;
        o.u[hf] = o.g0[hf] = o.g1[hf] = zero4;
        if (LIFT) {
          o.lok[hf] = lrow && w < bl.N2;
          const int wl = o.lok[hf] ? w : 0;
          const f32x4 u = *reinterpret_cast<const f32x4*>(urow + wl);
          const f32x4 g0 = *reinterpret_cast<const f32x4*>(grow + 2 * wl);
          const f32x4 g1 = *reinterpret_cast<const f32x4*>(grow + 2 * wl + 4);
          o.u[hf] = o.lok[hf] ? u : zero4;
          o.g0[hf] = o.lok[hf] ? g0 : zero4;
          o.g1[hf] = o.lok[hf] ? g1 : zero4;
        }
      }
    };
    f32x4 racc[C][NNT];
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int nt = 0; nt < NNT; ++nt) racc[c][nt] = zero4;
    // one step of MFMA tiles + epilogue on the operands ``cur`` (loaded one step earlier)
    auto step = [&](const int st, const Ops& cur) {
#pragma unroll
      for (int hf = 0; hf < NH; ++hf) {
        const int t = st * NH + hf;
        float av[S];
        const float2* ta = reinterpret_cast<const float2*>(sA + (t * 64 + lane) * S);
#pragma unroll
        for (int q = 0; q < S / 2; ++q) {
          const float2 v = ta[q];
          av[2 * q] = v.x;
          av[2 * q + 1] = v.y;
        }
        f32x4 d[C];
#pragma unroll
        for (int c = 0; c < C; ++c) {
          d[c] = zero4;
#pragma unroll
          for (int sp = 0; sp < S; ++sp) d[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[sp], zb[c][sp], d[c], 0, 0, 0);
        }
        const int w = 16 * NH * st + 4 * NH * g + 4 * hf;
        f32x4 ya[C];                                // RD operand (this lane's field values)
        // LIFT: the lifted field x0 = fc0([u, gx, gy]) at the lane's 4 points (0 off the crop)
        auto x0 = [&](int c, int r) -> float {
          const float gx = r < 2 ? cur.g0[hf][2 * r] : cur.g1[hf][2 * r - 4];
          const float gy = r < 2 ? cur.g0[hf][2 * r + 1] : cur.g1[hf][2 * r - 3];
          return cur.lok[hf] ? fmaf(w0[c][0], cur.u[hf][r], fmaf(w0[c][1], gx, fmaf(w0[c][2], gy, b0[c]))) : 0.f;
        };
        if (MODE == 0) {
          f32x4 xin[C];
#pragma unroll
          for (int c = 0; c < C; ++c) {
            if (LIFT) {
#pragma unroll
              for (int r = 0; r < 4; ++r) xin[c][r] = x0(c, r);
            } else {
              xin[c] = ACT ? RF_GELU(cur.a[c][hf]) : cur.a[c][hf];
            }
          }
#pragma unroll
          for (int o = 0; o < C; ++o) {
            f32x4 y = d[o];
            if (has_wc) {
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                float v = y[r] + bv[o];
#pragma unroll
                for (int i = 0; i < C; ++i) v = fmaf(W[o][i], xin[i][r], v);
                y[r] = v;
              }
            }
            *reinterpret_cast<f32x4*>(out + fbase + o * HW + w) = y;
            if (RD) ya[o] = RD == 2 ? RF_GELU(y) : y;
          }
        } else {
          if (WG) {
#pragma unroll
            for (int o = 0; o < C; ++o)
#pragma unroll
              for (int r = 0; r < 4; ++r) wacc[C * C + o] += cur.a[o][hf][r];
          }
#pragma unroll
          for (int c = 0; c < C; ++c) {
            f32x4 dg = d[c];
            f32x4 a4 = zero4, dg4 = zero4;
            if (!LIFT && ACT) gelu_both4(cur.s[c][hf], a4, dg4);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              float v = dg[r];
              if (has_wc) {
#pragma unroll
                for (int o = 0; o < C; ++o) v = fmaf(W[o][c], cur.a[o][hf][r], v);
              }
              float ain;
              if (LIFT) {
                ain = x0(c, r);
              } else if (ACT) {
                ain = a4[r];
                v *= dg4[r];
              } else {
                ain = cur.s[c][hf][r];
              }
              if (WG) {
#pragma unroll
                for (int o = 0; o < C; ++o) wacc[o * C + c] = fmaf(cur.a[o][hf][r], ain, wacc[o * C + c]);
              }
              if (LIFT) {
                if (cur.lok[hf]) {
                  const float gx = r < 2 ? cur.g0[hf][2 * r] : cur.g1[hf][2 * r - 4];
                  const float gy = r < 2 ? cur.g0[hf][2 * r + 1] : cur.g1[hf][2 * r - 3];
                  wacc[NWC + 3 * c] = fmaf(v, cur.u[hf][r], wacc[NWC + 3 * c]);
                  wacc[NWC + 3 * c + 1] = fmaf(v, gx, wacc[NWC + 3 * c + 1]);
                  wacc[NWC + 3 * c + 2] = fmaf(v, gy, wacc[NWC + 3 * c + 2]);
                  wacc[NWC + 3 * C + c] += v;
                }
              }
              dg[r] = v;
            }
            if (!LIFT) *reinterpret_cast<f32x4*>(out + fbase + c * HW + w) = dg;
            if (RD) ya[c] = dg;
          }
        }
        if (RD && !RF_NORD) {
          // next layer's row DFT, transposed: A = its twiddles (lane: column k' = 16 nt + c16;
          // K = w = 16 kb + 4 kq + s of rowdft's image), B = the field values this lane holds
          const int kb = (16 * NH * st + 4 * NH * g + 4 * hf) >> 4, kq = (NH * g + hf) & 3;
#pragma unroll
          for (int nt = 0; nt < NNT; ++nt) {
            const f32x4 tb = *reinterpret_cast<const f32x4*>(sT + ((kb * 4 + kq) * Npad + 16 * nt + c16) * 4);
#pragma unroll
            for (int c = 0; c < C; ++c)
#pragma unroll
              for (int s = 0; s < 4; ++s) {
                if constexpr (CD)       // D[h][k']: the block's rows on the M side
                  racc[c][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(ya[c][s], tb[s], racc[c][nt], 0, 0, 0);
                else                    // D[k'][h]
                  racc[c][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(tb[s], ya[c][s], racc[c][nt], 0, 0, 0);
              }
          }
        }
      }
    };
    // ping-pong operand buffers: the loads of step st + 1 are in flight while step st computes,
    // and no register copy of a pending load forces an early wait (a rotating cur = next copy
    // made hipcc wait for the prefetch inside the same step)
    // (sched_barrier: keep each prefetch issued where it is written -- the scheduler otherwise
    // sinks the loads next to their first use)
    Ops buf[2];
    load(0, buf[0]);
    if constexpr (ZY) zy_mfma<S, C>(zop, zb);
    if (ROWFUSE_ZPRE && !ZY) load_z(item + gxm * kW, znext);   // after this item's first loads
    if constexpr (NSC > 0) {
      // the step count is a compile-time constant: straight-line steps, the waits counted exactly
#pragma unroll
      for (int st = 0; st < NSC; ++st) {
        if (st + 1 < NSC) load(st + 1, buf[(st + 1) & 1]);
        __builtin_amdgcn_sched_barrier(0);
        step(st, buf[st & 1]);
      }
    } else if (MODE == 1 && !(ROWFUSE_PF1 && RD == 0)) {
      // the adjoint without operand prefetch (its operand set is twice the forward's; the
      // registers buy occupancy instead): always with the next row DFT in the pass (one wave
      // per SIMD with the prefetch buffers, two without: bwd_rd_crop 115 -> 108 us, r04g)
      for (int st = 0; st < NS; ++st) {
        if (st > 0) load(st, buf[0]);
        step(st, buf[0]);
      }
    } else {
      for (int st = 0; st < NS; st += 2) {
        load(st + 1 < NS ? st + 1 : st, buf[1]);
        __builtin_amdgcn_sched_barrier(0);
        step(st, buf[0]);
        if (st + 1 < NS) {
          load(st + 2 < NS ? st + 2 : st + 1, buf[0]);
          __builtin_amdgcn_sched_barrier(0);
          step(st + 1, buf[1]);
        }
      }
    }
    if constexpr (CD) {
      const int nch = colspec_nchunk(C, m2);
      float* blk = sc.part + ((int64_t)(n * sc.nblk + (h0 >> 4)) * nch) * 128;
#pragma unroll
      for (int c = 0; c < C; ++c) cd_store<NNT>(racc[c], sc.tabT, h0, lane, blk, c, C, m2);
    } else if (RD) {
      // lane: row h, spectrum columns k' = 16 nt + 4 g + r -> modes 8 nt + 2 g + r/2 (Re, Im)
#pragma unroll
      for (int c = 0; c < C; ++c)
#pragma unroll
        for (int nt = 0; nt < NNT; ++nt)
#pragma unroll
          for (int rp = 0; rp < 2; ++rp) {
            const int k = 8 * nt + 2 * g + rp;
            if (k < m2)
              *reinterpret_cast<float2*>(rd.At + ((((int64_t)n * m2 + k) * C + c) * P1 + h) * 2) =
                  make_float2(racc[c][nt][2 * rp], racc[c][nt][2 * rp + 1]);
          }
    }
#if ROWFUSE_PROBE
    if (it_probe < 5) RF_MARK(2 + it_probe);
    ++it_probe;
#endif
  }
  if (WG || NWL) {
    // block reduction of the per-lane partials -> partial[blockIdx.x][np] (np = C*C + C, + 4 C
    // for LIFT: dW0 (C x 3) then db0 (C)), index = wacc index
    __syncthreads();
    float* red = lds;
    constexpr int np = NWC + NWL;
#pragma unroll
    for (int e = 0; e < np; ++e) {
      const float s = wave_sum(wacc[e]);
      if (lane == 0) red[wave * np + e] = s;
      __builtin_amdgcn_sched_barrier(0);
    }
    __syncthreads();
    for (int p = threadIdx.x; p < np; p += blockDim.x) {
      float s = 0.f;
      for (int wv = 0; wv < kW; ++wv) s += red[wv * np + p];
      partial[(int64_t)blockIdx.x * np + p] = s;
    }
  }
  RF_MARK(7);
}
#if ROWFUSE_PROBE
BLINDNO_API int blindno_rowfuse_probe_reset() {
  void* p = nullptr;
  if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_rowfuse_probe)) != hipSuccess) return 1;
  return (int)hipMemset(p, 0, sizeof(g_rowfuse_probe));
}
BLINDNO_API int blindno_rowfuse_probe_read(unsigned long long* dst, int n) {
  return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_rowfuse_probe),
                                  sizeof(unsigned long long) * (size_t)n, 0, hipMemcpyDeviceToHost);
}
#endif

}  // namespace

namespace blindno {
// The spectrum of a 2D layer whose inverse runs in rowinv_wide_kernel is written by colidft in
// A-tile order: for row quad q (grid rows 4q..4q+3 of the Bn P1 rows), channel group g, K step s
// and lane l, Zt[((q NG + g) KS + s) 64 + l] = Re / Im Z[row 4q + (l&15)/4][k][4g + (l&3)] with
// kk = 4s + l/16, k = kk/2, Re for even kk.  Shapes: C in {8, 12, 16}, m2 even with m2/2 <= 16
// (<= 24 for C = 8), P1 % 4 == 0 and P1 >= 16 (2D), field < 2^31 elements.
bool rowinv_tile_layout(int Bn, int C, int P1, int P2, int m2) {
  if (!(C == 8 || C == 12 || C == 16) || m2 <= 0 || (m2 & 1) || P1 < 16 || (P1 & 3) || Bn <= 0)
    return false;
  if (m2 / 2 > (C == 8 ? 24 : 16)) return false;
  return (int64_t)Bn * C * P1 * P2 < INT32_MAX && (int64_t)Bn * P1 * m2 * C * 2 < INT32_MAX;
}
}  // namespace blindno

namespace {

struct RowinvGeom {
  int nitems, TPW, blocks;
  bool ldsb;
  size_t lds;
};

#ifndef ROWINV_MIN_ITEMS
#define ROWINV_MIN_ITEMS 4096
#endif
// fewest work items for which the twiddle image is staged in LDS (with the 1024-block cap,
// >= 4 items per workgroup); 8192 left the FNO_input layers of bags with U < 52 distinct
// snapshots (Bn < 205 at 160^2) on the L2-read path, ~20% slower per launch (r02e profile)
#ifndef ROWINV_LDSB_ITEMS
#define ROWINV_LDSB_ITEMS 4096
#endif
// work items the wide kernel aims at when splitting rows into column chunks
#ifndef ROWINV_WIDE_ITEMS
#define ROWINV_WIDE_ITEMS 2048
#endif

// shapes the transposed C = 4 kernel (rowfuse_kernel) takes; BLINDNO_ROWFUSE=0 turns it off
int g_rowfuse = -1;                                 // -1: from the environment on first use
bool rowfuse_on() {
  if (g_rowfuse < 0) {
    const char* e = getenv("BLINDNO_ROWFUSE");
    g_rowfuse = (e && e[0] == '0') ? 0 : 1;
  }
  return g_rowfuse != 0;
}
bool rowfuse_shape(int Bn, int C, int P1, int P2, int m2) {
  return rowfuse_on() && C == 4 && m2 >= 4 && m2 <= 16 && m2 % 4 == 0 && P1 % 16 == 0 &&
         P2 % 32 == 0 &&
         2 * m2 <= P2 && Bn > 0 && (int64_t)Bn * C * P1 * P2 < INT32_MAX;
}

// the general kernel's geometry (rowinv_mfma_kernel)
RowinvGeom rowinv_geom_general(int Bn, int C, int P1, int P2, int m2) {
  RowinvGeom g;
  const int KS = (m2 + 1) / 2, NT = (P2 + 15) / 16;
  const int NG = (C + 3) / 4;
  const int64_t base = (int64_t)((Bn * P1 + 3) / 4) * NG;
  // columns per work item: all of a row group when there is plenty of row parallelism,
  // split down to one tile for the small head layers
  int tpw = NT;
  while (tpw > 1 && base * ((NT + tpw - 1) / tpw) < ROWINV_MIN_ITEMS) tpw = (tpw + 1) / 2;
  g.TPW = tpw;
  g.nitems = (int)(base * ((NT + tpw - 1) / tpw));
  // persistent workgroups; the twiddle image is staged in LDS only when each workgroup
  // reuses it over several items (otherwise every MFMA step reads it from L1/L2)
  const int b = (g.nitems + kW - 1) / kW;
  const size_t tbytes = sizeof(float) * (size_t)KS * NT * 64;
  // staging pays when a workgroup's items read the table at least twice over (each item reads
  // TPW of its NT column tiles)
  const int64_t items_per_block = (g.nitems + 1023) / 1024;
  g.ldsb = tbytes <= 48 * 1024 && g.nitems >= ROWINV_LDSB_ITEMS && items_per_block * tpw >= 2 * NT;
  const int cap = g.ldsb ? 1024 : 2048;
  g.blocks = b < cap ? b : cap;
  g.lds = g.ldsb ? tbytes : 0;
  return g;
}

RowinvGeom rowinv_geom(int Bn, int C, int P1, int P2, int m2) {
  if (!rowfuse_shape(Bn, C, P1, P2, m2)) return rowinv_geom_general(Bn, C, P1, P2, m2);
  // whole 16-row blocks per work item, one per wave; partials are per workgroup
  RowinvGeom g;
  g.TPW = P2 / 16;
  g.nitems = Bn * (P1 / 16);
  const int b = (g.nitems + kW - 1) / kW;
  g.blocks = b < ROWFUSE_BLOCKS ? b : ROWFUSE_BLOCKS;
  g.ldsb = false;
  g.lds = 0;
  return g;
}

// ZC: the column pass folded in (colspec.h; sc.Y for ZY, sc.part for CD with the next row
// DFT): the transposed C = 4 kernel only, m2 = 12, with the 1x1 conv; no fallback
template <int MODE, int ACT, int WG, int LIFT = 0, bool ZC = false>
int rowinv_launch(const float* Z, const float* xs, const float* dz, const float* wc,
                  const float* bc, float* out, const float* TB, float* partial, int nblocks,
                  int Bn, int C, int P1, int P2, int m2, hipStream_t st, BagLift bl = BagLift{},
                  int G = 1, int64_t wgs = 0, int dN1 = 0, int dN2 = 0,
                  RowDftNext rd = RowDftNext{nullptr, nullptr, 0, 0},
                  SpecCol sc = SpecCol{nullptr, nullptr, nullptr, nullptr, 0, 0, nullptr, nullptr, 0, 0, 0}) {
  sc.nmain = nblocks;                              // the row kernel's grid (hosted jobs after it)
  if (dN1 <= 0) dN1 = P1;
  if (dN2 <= 0) dN2 = P2;
  if (dN1 > P1 || dN2 > P2) return (int)hipErrorInvalidValue;
  if (G < 1 || Bn % G || (G > 1 && (WG || LIFT || P1 % 4))) return (int)hipErrorInvalidValue;
  const int Bg = Bn / G;
  if (G == 1) wgs = 0;
  if (Bn <= 0 || C <= 0 || C > 32 || m2 <= 0 || P2 <= 0) return (int)hipErrorInvalidValue;
  if (WG && C > 4) return (int)hipErrorInvalidValue;
  const int64_t zel = (int64_t)Bn * P1 * m2 * C * 2, fel = (int64_t)Bn * C * P1 * P2;
  if (zel >= INT32_MAX || fel >= ((int64_t)1 << 40)) return (int)hipErrorInvalidValue;
  const int cm = C <= 4 ? 4 : (C <= 8 ? 8 : (C <= 16 ? 16 : 32));
  const int ks = (m2 + 1) / 2;
  if (ks > 24) return (int)hipErrorInvalidValue;               // m2 <= 48
  {
    // the transposed C = 4 kernel: 16-B field accesses need aligned bases and a crop width
    // (dz's valid region, the snapshot) in whole float4s
    auto al = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
    const bool rd_ok = (!rd.At && !(ZC && sc.part)) || rd.Npad == 16 * ((2 * m2 + 15) / 16);
    const bool zc_ok = !ZC || (m2 == 12 && wc && sc.tab && sc.tabT && al(sc.Y) && al(sc.tab) && al(sc.tabT) &&
                              (!sc.part || (rd.Tp && sc.nblk == P1 / 16)) && (sc.Y || sc.part));
    if (ZC && !(rowfuse_shape(Bn, C, P1, P2, m2) && zc_ok)) return (int)hipErrorInvalidValue;
    if (rowfuse_shape(Bn, C, P1, P2, m2) && G == 1 && al(Z) && al(xs) && al(dz) && al(out) &&
        dN2 % 4 == 0 && rd_ok && zc_ok && (!LIFT || (bl.N2 % 4 == 0 && al(bl.X) && al(bl.grid)))) {
      const int NT = P2 / 16, S = m2 / 2;
      const bool rdx = rd.At || (ZC && sc.part);          // the next row DFT taken in the pass
      size_t shf = sizeof(float) * ((size_t)NT * 64 * S + (rdx ? (size_t)NT * 16 * rd.Npad : 0));
      const size_t red = sizeof(float) * (size_t)kW * (C * C + C + 4 * C);
      if (shf < red) shf = red;
      if (shf > 160 * 1024) return (int)hipErrorInvalidValue;
      // column tiles per step: 2 in the forward (ROWFUSE_NH0; without the next row DFT
      // ROWFUSE_NH0_NORD: 1 tile gives 4 waves per SIMD instead of 2 -- 124 vs 176 VGPRs -- but
      // the step measured 0.5 % slower, r04h), 1 in the adjoint
#define NHX(RD_) (MODE == 0 ? ((RD_) == 0 ? ROWFUSE_NH0_NORD : ROWFUSE_NH0) : ROWFUSE_NH1)
      // P2 = 160 (the encoder at 128^2), forward: the step loop fully unrolled (the adjoint's
      // larger operand set and in-pass weight-gradient sums spill when unrolled: runtime loop)
      const bool p160 = P2 == 160 && MODE == 0;
      // the output crop (MODE 0, no next row DFT): 128 of the 160 columns, 4 steps
      const bool crop128 = MODE == 0 && !rd.At && dN2 == 128;
#define RFG(RD_, S_, ZY_, CD_, NH_, ZW_)                                                       \
  do {                                                                                         \
    if (wc && p160 && crop128 && RD_ == 0)                                                     \
      rowfuse_kernel<MODE, ACT, WG, LIFT, RD_, S_, NH_, true, MODE == 0 ? 128 / (16 * NH_) : 0, \
                     ZY_, CD_, ZW_>                                                            \
          <<<nblocks + sc.nmixb, 256, shf, st>>>(Z, xs, dz, wc, bc, out, TB, partial, Bn, P1, P2, bl, dN1, \
                                      dN2, rd, sc);                                            \
    else if (wc && p160 && (dN2 == P2 || RD_ != 0))                                            \
      rowfuse_kernel<MODE, ACT, WG, LIFT, RD_, S_, NH_, true, MODE == 0 ? 160 / (16 * NH_) : 0, \
                     ZY_, CD_, ZW_>                                                            \
          <<<nblocks + sc.nmixb, 256, shf, st>>>(Z, xs, dz, wc, bc, out, TB, partial, Bn, P1, P2, bl, dN1, \
                                      dN2, rd, sc);                                            \
    else if (wc)                                                                               \
      rowfuse_kernel<MODE, ACT, WG, LIFT, RD_, S_, NH_, true, 0, ZY_, CD_, ZW_>                \
          <<<nblocks + sc.nmixb, 256, shf, st>>>(Z, xs, dz, wc, bc, out, TB, partial, Bn, P1, P2, bl, dN1, \
                                      dN2, rd, sc);                                            \
    else if (!ZY_)                                                                             \
      rowfuse_kernel<MODE, ACT, WG, LIFT, RD_, S_, NH_, false>                                 \
          <<<nblocks + sc.nmixb, 256, shf, st>>>(Z, xs, dz, wc, bc, out, TB, partial, Bn, P1, P2, bl, dN1, \
                                      dN2, rd, sc);                                            \
  } while (0)
#define RFX(RD_, S_, ZY_, CD_) RFG(RD_, S_, ZY_, CD_, NHX(RD_), 0)
#define RF(RD_, S_) RFX(RD_, S_, false, false)
#define RF_S(RD_) \
  do { if (S == 2) RF(RD_, 2); else if (S == 4) RF(RD_, 4); else if (S == 6) RF(RD_, 6); else RF(RD_, 8); } while (0)
      if constexpr (ZC) {
        // ZY always; CD with the next row DFT (act: of GELU(field)); m2 = 12 (zc_ok); the 3-wave
        // budget (sc.w3: one column tile per step in the forward) chosen by the caller
        if (MODE == 0 && sc.w3) {
          if (!sc.part) RFG(0, 6, true, false, ROWFUSE_NH0_NORD, 3);
          else if (rd.act) RFG(2, 6, true, true, 1, 3);
          else RFG(1, 6, true, true, 1, 3);
        } else if (sc.dzg) {
          // the encoder's last-layer adjoint with dz formed on load (MODE 1 with its weight
          // gradient and the previous layer's partials; no NSC unroll in MODE 1)
          if constexpr (MODE == 1 && WG == 1 && LIFT == 0) {
            if (!sc.part || rd.act || !wc) return (int)hipErrorInvalidValue;
            rowfuse_kernel<MODE, ACT, WG, LIFT, 1, 6, ROWFUSE_NH1, true, 0, true, true, 0, true>
                <<<nblocks + sc.nmixb, 256, shf, st>>>(Z, xs, dz, wc, bc, out, TB, partial, Bn, P1, P2, bl, dN1,
                                            dN2, rd, sc);
          } else {
            return (int)hipErrorInvalidValue;
          }
        } else {
          if (!sc.part) RFX(0, 6, true, false);
          else if (rd.act) RFX(2, 6, true, true);
          else RFX(1, 6, true, true);
        }
      } else {
        if (!rd.At) RF_S(0);
        else if (rd.act) RF_S(2);
        else RF_S(1);
      }
#undef RF_S
#undef RF
#undef RFX
#undef RFG
#undef NHX
      return (int)hipGetLastError();
    }
  }
  // the general kernel's own geometry also where the shape suits rowfuse but a launch-time gate
  // (G, alignment, crop width) sent it here; nblocks stays the caller's (it sized the partials,
  // and the persistent general kernel strides its items over any grid)
  const RowinvGeom g = rowinv_geom_general(Bn, C, P1, P2, m2);
  size_t sh = g.lds;
  if (WG) {
    const size_t need = sizeof(float) * (size_t)kW * (C * C + C + (LIFT ? 4 * C : 0));
    if (need > sh) sh = need;
  }
  if (sh > 160 * 1024) return (int)hipErrorInvalidValue;
  if constexpr (!WG && !LIFT) {
    // wide fields with the spectrum in A-tile order (rowinv_tile_layout; full-field dz only)
    if (rowinv_tile_layout(Bn, C, P1, P2, m2) && dN1 == P1 && dN2 == P2) {
      if (G > kWideMaxG) return (int)hipErrorInvalidValue;
      const int NT = (P2 + 15) / 16, nquads = Bn * P1 / 4;
      int tpw = NT;
      while (tpw > 1 && (int64_t)nquads * ((NT + tpw - 1) / tpw) < ROWINV_WIDE_ITEMS) tpw = (tpw + 1) / 2;
      const int nitems = nquads * ((NT + tpw - 1) / tpw);
      int nbw = (nitems + kW - 1) / kW;
      if (nbw > 2048) nbw = 2048;
#define RW(CM_, KS_)                                                                          \
  do {                                                                                        \
    if (m2 == 2 * KS_)                                                                        \
      rowinv_wide_kernel<CM_, KS_, MODE, ACT, true><<<nbw, 256, 0, st>>>(                     \
          Z, xs, dz, wc, bc, out, TB, Bn, P1, P2, m2, tpw, Bg, wgs);                          \
    else                                                                                      \
      rowinv_wide_kernel<CM_, KS_, MODE, ACT, false><<<nbw, 256, 0, st>>>(                    \
          Z, xs, dz, wc, bc, out, TB, Bn, P1, P2, m2, tpw, Bg, wgs);                          \
  } while (0)
      if (C == 8) {
        if (ks <= 8) RW(8, 8); else if (ks <= 16) RW(8, 16); else RW(8, 24);
      } else if (C == 12) {
        if (ks <= 8) RW(12, 8); else RW(12, 16);
      } else {
        if (ks <= 8) RW(16, 8); else RW(16, 16);
      }
#undef RW
      const int e = (int)hipGetLastError();
      if (e || !rd.At) return e;
      return blindno_rowdft(out, rd.At, rd.Tp, Bn, C, P1, P2, m2, rd.act, (void*)st);
    }
  }
  // the next layer's row DFT otherwise runs as its own launch after this one
  if (rd.At && (G != 1 || (MODE == 1 && LIFT))) return (int)hipErrorInvalidValue;
#define RI(CM_, KS_)                                                                         \
  do {                                                                                       \
    if (g.ldsb)                                                                              \
      rowinv_mfma_kernel<CM_, KS_, MODE, ACT, WG, 1, LIFT><<<nblocks, 256, sh, st>>>(        \
          Z, xs, dz, wc, bc, out, TB, partial, Bn, C, P1, P2, m2, g.TPW, bl, Bg, wgs, dN1,   \
          dN2);                                                                              \
    else                                                                                     \
      rowinv_mfma_kernel<CM_, KS_, MODE, ACT, WG, 0, LIFT><<<nblocks, 256, sh, st>>>(        \
          Z, xs, dz, wc, bc, out, TB, partial, Bn, C, P1, P2, m2, g.TPW, bl, Bg, wgs, dN1,   \
          dN2);                                                                              \
  } while (0)
#define RI_K(CM_) \
  if (ks <= 8) RI(CM_, 8); else if (ks <= 16) RI(CM_, 16); else RI(CM_, 24);
  if (cm == 4) {
    RI_K(4)
  } else if constexpr (!WG && !LIFT) {
    if (cm == 8) { RI_K(8) }
    else if (cm == 16) { RI_K(16) }
    else { RI_K(32) }
  }
#undef RI_K
#undef RI
  int e = (int)hipGetLastError();
  if (e || !rd.At) return e;
  // unfused: the next layer's row DFT of the field just written
  return blindno_rowdft(out, rd.At, rd.Tp, Bn, C, P1, P2, m2, rd.act, (void*)st);
}

}  // namespace

// The encoder's last layer: the row inverse + epilogue written on the output crop h < oN1,
// w < oN2 only (its one reader, the projection, reads nothing else); the rest of z is left
// unwritten.  Other shapes take the full-field kernels.
BLINDNO_API int blindno_rowidft_epi_crop(const float* Z, const float* x, const float* wc,
                                         const float* bc, float* z, const float* tb, int Bn,
                                         int C, int P1, int P2, int m2, int act, int oN1, int oN2,
                                         void* stream) {
  if (oN1 < 1 || oN1 > P1 || oN2 < 1 || oN2 > P2) return (int)hipErrorInvalidValue;
  RowinvGeom g = rowinv_geom(Bn, C, P1, P2, m2);
  if (rowfuse_shape(Bn, C, P1, P2, m2)) {
    const int items = Bn * ((oN1 + 15) / 16);
    const int b = (items + kW - 1) / kW;
    g.blocks = b < ROWFUSE_BLOCKS ? b : ROWFUSE_BLOCKS;
  }
  hipStream_t st = (hipStream_t)stream;
  if (act)
    return rowinv_launch<0, 1, 0>(Z, x, nullptr, wc, bc, z, tb, nullptr, g.blocks, Bn, C, P1, P2,
                                  m2, st, BagLift{}, 1, 0, oN1, oN2);
  return rowinv_launch<0, 0, 0>(Z, x, nullptr, wc, bc, z, tb, nullptr, g.blocks, Bn, C, P1, P2, m2,
                                st, BagLift{}, 1, 0, oN1, oN2);
}

BLINDNO_API int blindno_rowidft_epi_g(const float* Z, const float* x, const float* wc,
                                      const float* bc, float* z, const float* tb, int G,
                                      int64_t wgs, int Bn, int C, int P1, int P2, int m2, int act,
                                      void* stream) {
  const int nb = rowinv_geom(Bn, C, P1, P2, m2).blocks;
  hipStream_t st = (hipStream_t)stream;
  if (act)
    return rowinv_launch<0, 1, 0>(Z, x, nullptr, wc, bc, z, tb, nullptr, nb, Bn, C, P1, P2, m2, st,
                                  BagLift{}, G, wgs);
  return rowinv_launch<0, 0, 0>(Z, x, nullptr, wc, bc, z, tb, nullptr, nb, Bn, C, P1, P2, m2, st,
                                BagLift{}, G, wgs);
}

BLINDNO_API int blindno_rowidft_epi(const float* Z, const float* x, const float* wc,
                                    const float* bc, float* z, const float* tb, int Bn, int C,
                                    int P1, int P2, int m2, int act, void* stream) {
  return blindno_rowidft_epi_g(Z, x, wc, bc, z, tb, 1, 0, Bn, C, P1, P2, m2, act, stream);
}

BLINDNO_API int blindno_spectrum_tile_layout(int Bn, int C, int P1, int P2, int m2) {
  return rowinv_tile_layout(Bn, C, P1, P2, m2) ? 1 : 0;
}

BLINDNO_API int blindno_set_rowfuse(int on) {
  const int prev = rowfuse_on() ? 1 : 0;
  g_rowfuse = on ? 1 : 0;
  return prev;
}

BLINDNO_API int blindno_rowidft_bwd_nchunk(int Bn, int C, int P1, int P2, int m2) {
  return C <= 4 ? rowinv_geom(Bn, C, P1, P2, m2).blocks : 0;
}

BLINDNO_API int blindno_rowidft_bwd_g(const float* Gs, const float* dz, const float* wc,
                                      const float* xsrc, float* dx, const float* tb, int G,
                                      int64_t wgs, int Bn, int C, int P1, int P2, int m2, int act,
                                      void* stream) {
  const int nb = rowinv_geom(Bn, C, P1, P2, m2).blocks;
  hipStream_t st = (hipStream_t)stream;
  if (act)
    return rowinv_launch<1, 1, 0>(Gs, xsrc, dz, wc, nullptr, dx, tb, nullptr, nb, Bn, C, P1, P2, m2,
                                  st, BagLift{}, G, wgs);
  return rowinv_launch<1, 0, 0>(Gs, xsrc, dz, wc, nullptr, dx, tb, nullptr, nb, Bn, C, P1, P2, m2,
                                st, BagLift{}, G, wgs);
}

BLINDNO_API int blindno_rowidft_bwd_crop(const float* G, const float* dz, const float* wc,
                                         const float* xsrc, float* dx, const float* tb,
                                         float* partial, int Bn, int C, int P1, int P2, int m2,
                                         int act, int dN1, int dN2, void* stream) {
  if (dN1 < 1 || dN1 > P1 || dN2 < 1 || dN2 > P2) return (int)hipErrorInvalidValue;
  const int nb = rowinv_geom(Bn, C, P1, P2, m2).blocks;
  hipStream_t st = (hipStream_t)stream;
  const BagLift nb0{};
  if (partial) {
    if (C > 4 || !wc) return (int)hipErrorInvalidValue;
    if (act)
      return rowinv_launch<1, 1, 1>(G, xsrc, dz, wc, nullptr, dx, tb, partial, nb, Bn, C, P1, P2, m2, st,
                                    nb0, 1, 0, dN1, dN2);
    return rowinv_launch<1, 0, 1>(G, xsrc, dz, wc, nullptr, dx, tb, partial, nb, Bn, C, P1, P2, m2, st,
                                  nb0, 1, 0, dN1, dN2);
  }
  if (act)
    return rowinv_launch<1, 1, 0>(G, xsrc, dz, wc, nullptr, dx, tb, nullptr, nb, Bn, C, P1, P2, m2, st,
                                  nb0, 1, 0, dN1, dN2);
  return rowinv_launch<1, 0, 0>(G, xsrc, dz, wc, nullptr, dx, tb, nullptr, nb, Bn, C, P1, P2, m2, st,
                                nb0, 1, 0, dN1, dN2);
}

// blindno_rowidft_bwd_crop plus the row DFT of dx for the previous layer's adjoint
// (blindno_rowdft(dx, At, Tp, ..., act = 0) in the same pass when the geometry allows)
BLINDNO_API int blindno_rowidft_bwd_rd(const float* G, const float* dz, const float* wc,
                                       const float* xsrc, float* dx, const float* tb,
                                       float* partial, int Bn, int C, int P1, int P2, int m2,
                                       int act, int dN1, int dN2, float* At, const float* Tp,
                                       void* stream) {
  if (dN1 < 1 || dN1 > P1 || dN2 < 1 || dN2 > P2 || !At || !Tp || m2 > P2 / 2 + 1)
    return (int)hipErrorInvalidValue;
  const int nb = rowinv_geom(Bn, C, P1, P2, m2).blocks;
  hipStream_t st = (hipStream_t)stream;
  const BagLift nb0{};
  const RowDftNext rd{At, Tp, ((2 * m2 + 15) / 16) * 16, 0};
  if (partial) {
    if (C > 4 || !wc) return (int)hipErrorInvalidValue;
    if (act)
      return rowinv_launch<1, 1, 1>(G, xsrc, dz, wc, nullptr, dx, tb, partial, nb, Bn, C, P1, P2, m2, st,
                                    nb0, 1, 0, dN1, dN2, rd);
    return rowinv_launch<1, 0, 1>(G, xsrc, dz, wc, nullptr, dx, tb, partial, nb, Bn, C, P1, P2, m2, st,
                                  nb0, 1, 0, dN1, dN2, rd);
  }
  if (act)
    return rowinv_launch<1, 1, 0>(G, xsrc, dz, wc, nullptr, dx, tb, nullptr, nb, Bn, C, P1, P2, m2, st,
                                  nb0, 1, 0, dN1, dN2, rd);
  return rowinv_launch<1, 0, 0>(G, xsrc, dz, wc, nullptr, dx, tb, nullptr, nb, Bn, C, P1, P2, m2, st,
                                nb0, 1, 0, dN1, dN2, rd);
}

BLINDNO_API int blindno_rowidft_bwd(const float* G, const float* dz, const float* wc,
                                    const float* xsrc, float* dx, const float* tb,
                                    float* partial, int Bn, int C, int P1, int P2, int m2,
                                    int act, void* stream) {
  return blindno_rowidft_bwd_crop(G, dz, wc, xsrc, dx, tb, partial, Bn, C, P1, P2, m2, act, P1, P2,
                                  stream);
}

// Snapshot-encoder first layer (LIFT): the layer input is fc0([u, gx, gy]) recomputed from
// the bag tensor (see BagLift); forward epilogue / adjoint with fc0's gradient reduced in pass.
BLINDNO_API int blindno_rowidft_epi_lift(const float* Z, const float* X, const int* idx,
                                         const float* grid, const float* w0, const float* b0,
                                         const float* wc, const float* bc, float* z,
                                         const float* tb, int B, int T, int L, int N1, int N2,
                                         int C, int P1, int P2, int m2, void* stream) {
  if (!wc || !bc || C > 4 || N1 > P1 || N2 > P2) return (int)hipErrorInvalidValue;
  const BagLift bl{X, idx, grid, w0, b0, T, L, N1, N2};
  const int Bn = B * L;
  const int nb = rowinv_geom(Bn, C, P1, P2, m2).blocks;
  return rowinv_launch<0, 0, 0, 1>(Z, nullptr, nullptr, wc, bc, z, tb, nullptr, nb, Bn, C, P1, P2,
                                   m2, (hipStream_t)stream, bl);
}

// blindno_rowidft_epi_lift plus the next layer's row DFT of its input GELU(z) (act = 1) or z
// (act = 0): At / Tp as blindno_rowdft's, in the same pass when the geometry allows
BLINDNO_API int blindno_rowidft_epi_lift_rd(const float* Z, const float* X, const int* idx,
                                            const float* grid, const float* w0, const float* b0,
                                            const float* wc, const float* bc, float* z,
                                            const float* tb, int B, int T, int L, int N1, int N2,
                                            int C, int P1, int P2, int m2, float* At,
                                            const float* Tp, int act, void* stream) {
  if (!wc || !bc || C > 4 || N1 > P1 || N2 > P2 || !At || !Tp || m2 > P2 / 2 + 1)
    return (int)hipErrorInvalidValue;
  const BagLift bl{X, idx, grid, w0, b0, T, L, N1, N2};
  const int Bn = B * L;
  const int nb = rowinv_geom(Bn, C, P1, P2, m2).blocks;
  const RowDftNext rd{At, Tp, ((2 * m2 + 15) / 16) * 16, act};
  return rowinv_launch<0, 0, 0, 1>(Z, nullptr, nullptr, wc, bc, z, tb, nullptr, nb, Bn, C, P1, P2,
                                   m2, (hipStream_t)stream, bl, 1, 0, 0, 0, rd);
}

// blindno_rowidft_epi plus the next layer's row DFT of f(z) (f = GELU when act_next)
BLINDNO_API int blindno_rowidft_epi_rd(const float* Z, const float* x, const float* wc,
                                       const float* bc, float* z, const float* tb, int Bn, int C,
                                       int P1, int P2, int m2, int act, float* At, const float* Tp,
                                       int act_next, void* stream) {
  if (!At || !Tp || m2 > P2 / 2 + 1) return (int)hipErrorInvalidValue;
  const int nb = rowinv_geom(Bn, C, P1, P2, m2).blocks;
  hipStream_t st = (hipStream_t)stream;
  const RowDftNext rd{At, Tp, ((2 * m2 + 15) / 16) * 16, act_next};
  if (act)
    return rowinv_launch<0, 1, 0>(Z, x, nullptr, wc, bc, z, tb, nullptr, nb, Bn, C, P1, P2, m2, st,
                                  BagLift{}, 1, 0, 0, 0, rd);
  return rowinv_launch<0, 0, 0>(Z, x, nullptr, wc, bc, z, tb, nullptr, nb, Bn, C, P1, P2, m2, st,
                                BagLift{}, 1, 0, 0, 0, rd);
}

BLINDNO_API int blindno_rowidft_bwd_lift(const float* G, const float* dz, const float* X,
                                         const int* idx, const float* grid, const float* w0,
                                         const float* b0, const float* wc, const float* tb,
                                         float* partial, int B, int T, int L, int N1, int N2,
                                         int C, int P1, int P2, int m2, void* stream) {
  if (!wc || !partial || C > 4 || N1 > P1 || N2 > P2) return (int)hipErrorInvalidValue;
  const BagLift bl{X, idx, grid, w0, b0, T, L, N1, N2};
  const int Bn = B * L;
  const int nb = rowinv_geom(Bn, C, P1, P2, m2).blocks;
  return rowinv_launch<1, 0, 1, 1>(G, nullptr, dz, wc, nullptr, nullptr, tb, partial,
                                   nb, Bn, C, P1, P2, m2, (hipStream_t)stream, bl);
}

// ------------------------------------------------------------ folded column pass (colspec.h)
// The row kernels of FNO_input with the column pass folded in: Y (Bn, m2, C, K1) complex from
// blindno_colmix replaces Z; part (Bn, P1 / 16, NCH, 64, 2) receives the column-DFT partials of
// the next row spectrum (blindno_colspec_nchunk) instead of At; tab = Tab[P1][2 K1]
// (blindno.ops.twiddle_colspec).  Shapes: blindno_colspec_ok.
namespace {
SpecCol spec_col(const float* Y, float* part, const float* tab, int P1, int w3 = 0) {
  // tab: Tab (P1 x 2 K1) followed by TabT (the same values, P1 / 4 x 2 K1 x 4)
  return SpecCol{Y, part, tab, tab ? tab + (size_t)P1 * 2 * kCsK1 : nullptr, P1 / 16, w3,
                 nullptr, nullptr, 0, 0, 0};
}
}  // namespace

// persistent grid of the MODE 0 ZY / CD kernels: 4-wave workgroups filling ROWFUSE_ZC_WAVES0
// waves per SIMD (256 CUs x 4 SIMDs)
int zc_blocks(int items, int waves) {
  const int cap = waves > 2 ? 256 * waves : ROWFUSE_BLOCKS;
  const int b = (items + kW - 1) / kW;
  return b < cap ? b : cap;
}
// the MODE 0 kernels: the 3-wave budget for item counts in (ROWFUSE_ZC3_MIN, ROWFUSE_ZC3_MAX]
// (measured: 2000 items 55.6 -> 51.9 us, 2080 items 74.7 -> 69.8 us, 3000 items 89.9 -> 102.8 us)
#ifndef ROWFUSE_ZC3_MIN
#define ROWFUSE_ZC3_MIN 0
#endif
#ifndef ROWFUSE_ZC3_MAX
#define ROWFUSE_ZC3_MAX 2600
#endif
bool zc_w3(int items) { return items > ROWFUSE_ZC3_MIN && items <= ROWFUSE_ZC3_MAX; }
int zc_blocks0(int items) { return zc_blocks(items, zc_w3(items) ? 3 : 2); }
int zc_blocks1(int items) { return zc_blocks(items, 2); }

BLINDNO_API int blindno_colspec_ok(int Bn, int C, int P1, int P2, int m1, int m2) {
  return (rowfuse_shape(Bn, C, P1, P2, m2) && m2 == 12 && m1 == 12 && kept_rows_count(m1, P1) == kCsK1 &&
          P1 % 16 == 0) ? 1 : 0;
}

BLINDNO_API int blindno_colspec_nchunk(int C, int m2) { return colspec_nchunk(C, m2); }

// weight-gradient partial rows of blindno_rowidft_bwd_zc / _bwd_lift_zc (one per workgroup)
BLINDNO_API int blindno_colspec_bwd_nchunk(int Bn, int P1) { return zc_blocks1(Bn * (P1 / 16)); }

// blindno_rowidft_epi (+ crop oN1 x oN2 when part is NULL) with Z built from Y; part != NULL:
// also the next layer's row DFT of f(z) (f = GELU when act_next) as column-DFT partials
BLINDNO_API int blindno_rowidft_epi_zc(const float* Y, const float* x, const float* wc,
                                       const float* bc, float* z, const float* tb,
                                       const float* tab, float* part, const float* Tp, int Bn,
                                       int C, int P1, int P2, int m1, int m2, int act, int act_next,
                                       int oN1, int oN2, void* stream) {
  if (!blindno_colspec_ok(Bn, C, P1, P2, m1, m2) || !Y || !tab || (part && !Tp) ||
      oN1 < 1 || oN1 > P1 || oN2 < 1 || oN2 > P2 || (part && (oN1 != P1 || oN2 != P2)))
    return (int)hipErrorInvalidValue;
  const int items = Bn * (((part ? P1 : oN1) + 15) / 16);
  const int nb = zc_blocks0(items);
  hipStream_t st = (hipStream_t)stream;
  const RowDftNext rd{nullptr, part ? Tp : nullptr, ((2 * m2 + 15) / 16) * 16, act_next};
  const SpecCol sc = spec_col(Y, part, tab, P1, zc_w3(items));
  if (act)
    return rowinv_launch<0, 1, 0, 0, true>(nullptr, x, nullptr, wc, bc, z, tb, nullptr, nb, Bn, C, P1,
                                           P2, m2, st, BagLift{}, 1, 0, oN1, oN2, rd, sc);
  return rowinv_launch<0, 0, 0, 0, true>(nullptr, x, nullptr, wc, bc, z, tb, nullptr, nb, Bn, C, P1,
                                         P2, m2, st, BagLift{}, 1, 0, oN1, oN2, rd, sc);
}

// blindno_rowidft_epi_lift(_rd) with Z built from Y and, with part != NULL, the next row DFT of
// GELU(z) (act_next) or z as column-DFT partials
BLINDNO_API int blindno_rowidft_epi_lift_zc(const float* Y, const float* X, const int* idx,
                                            const float* grid, const float* w0, const float* b0,
                                            const float* wc, const float* bc, float* z,
                                            const float* tb, const float* tab, float* part,
                                            const float* Tp, int B, int T, int L, int N1, int N2,
                                            int C, int P1, int P2, int m1, int m2, int act_next,
                                            void* stream) {
  const int Bn = B * L;
  if (!blindno_colspec_ok(Bn, C, P1, P2, m1, m2) || !Y || !tab || (part && !Tp) || !wc || !bc ||
      N1 > P1 || N2 > P2)
    return (int)hipErrorInvalidValue;
  const BagLift bl{X, idx, grid, w0, b0, T, L, N1, N2};
  const int items = Bn * (P1 / 16);
  const int nb = zc_blocks0(items);
  const RowDftNext rd{nullptr, part ? Tp : nullptr, ((2 * m2 + 15) / 16) * 16, act_next};
  return rowinv_launch<0, 0, 0, 1, true>(nullptr, nullptr, nullptr, wc, bc, z, tb, nullptr, nb, Bn, C,
                                         P1, P2, m2, (hipStream_t)stream, bl, 1, 0, 0, 0, rd,
                                         spec_col(Y, part, tab, P1, zc_w3(items)));
}

// blindno_rowidft_bwd_rd / _crop with Z built from Y; part != NULL: the row DFT of dx as
// column-DFT partials (the previous layer's adjoint); partial: the 1x1-conv weight-gradient
// partials (blindno_rowidft_bwd_nchunk, C <= 4) or NULL
BLINDNO_API int blindno_rowidft_bwd_zc(const float* Y, const float* dz, const float* wc,
                                       const float* xsrc, float* dx, const float* tb,
                                       const float* tab, float* part, const float* Tp,
                                       float* partial, int Bn, int C, int P1, int P2, int m1,
                                       int m2, int act, int dN1, int dN2, void* stream) {
  if (!blindno_colspec_ok(Bn, C, P1, P2, m1, m2) || !Y || !tab || (part && !Tp) || dN1 < 1 ||
      dN1 > P1 || dN2 < 1 || dN2 > P2 || !wc)
    return (int)hipErrorInvalidValue;
  const int nb = zc_blocks1(Bn * (P1 / 16));
  hipStream_t st = (hipStream_t)stream;
  const BagLift nb0{};
  const RowDftNext rd{nullptr, part ? Tp : nullptr, ((2 * m2 + 15) / 16) * 16, 0};
  const SpecCol sc = spec_col(Y, part, tab, P1);
  if (partial) {
    if (act)
      return rowinv_launch<1, 1, 1, 0, true>(nullptr, xsrc, dz, wc, nullptr, dx, tb, partial, nb, Bn, C,
                                             P1, P2, m2, st, nb0, 1, 0, dN1, dN2, rd, sc);
    return rowinv_launch<1, 0, 1, 0, true>(nullptr, xsrc, dz, wc, nullptr, dx, tb, partial, nb, Bn, C,
                                           P1, P2, m2, st, nb0, 1, 0, dN1, dN2, rd, sc);
  }
  if (act)
    return rowinv_launch<1, 1, 0, 0, true>(nullptr, xsrc, dz, wc, nullptr, dx, tb, nullptr, nb, Bn, C,
                                           P1, P2, m2, st, nb0, 1, 0, dN1, dN2, rd, sc);
  return rowinv_launch<1, 0, 0, 0, true>(nullptr, xsrc, dz, wc, nullptr, dx, tb, nullptr, nb, Bn, C, P1,
                                         P2, m2, st, nb0, 1, 0, dN1, dN2, rd, sc);
}

// blindno_rowidft_bwd_zc (with the 1x1-conv weight-gradient partials and the previous layer's
// column-DFT partials) for the encoder's last layer, whose dz = lw_l ghat v is formed on load:
// v (Bn, C, P1, P2) from blindno_project_bag_fwd, ghat (B, Ho Wo), lw (U, NULL: 1 / U), Bn = B U
BLINDNO_API int blindno_rowidft_bwd_zc_bag(const float* Y, const float* v, const float* ghat,
                                           const float* lw, int U, const float* wc,
                                           const float* xsrc, float* dx, const float* tb,
                                           const float* tab, float* part, const float* Tp,
                                           float* partial, int Bn, int C, int P1, int P2, int m1,
                                           int m2, int act, int Ho, int Wo, void* stream) {
  if (!blindno_colspec_ok(Bn, C, P1, P2, m1, m2) || !Y || !v || !ghat || U < 1 || Bn % U || !tab ||
      !part || !Tp || !partial || !wc || Ho < 1 || Ho > P1 || Wo < 1 || Wo > P2 || Wo % 4)
    return (int)hipErrorInvalidValue;
  const int nb = zc_blocks1(Bn * (P1 / 16));
  hipStream_t st = (hipStream_t)stream;
  const RowDftNext rd{nullptr, Tp, ((2 * m2 + 15) / 16) * 16, 0};
  SpecCol sc = spec_col(Y, part, tab, P1);
  sc.dzg = ghat;
  sc.dzl = lw;
  sc.dzU = U;
  sc.dzWo = Wo;
  sc.dzS = Ho * Wo;
  if (act)
    return rowinv_launch<1, 1, 1, 0, true>(nullptr, xsrc, v, wc, nullptr, dx, tb, partial, nb, Bn, C, P1,
                                           P2, m2, st, BagLift{}, 1, 0, Ho, Wo, rd, sc);
  return rowinv_launch<1, 0, 1, 0, true>(nullptr, xsrc, v, wc, nullptr, dx, tb, partial, nb, Bn, C, P1,
                                         P2, m2, st, BagLift{}, 1, 0, Ho, Wo, rd, sc);
}

// blindno_rowidft_bwd_lift with Z built from Y
BLINDNO_API int blindno_rowidft_bwd_lift_zc_mix(const float* Y, const float* dz, const float* X,
                                                const int* idx, const float* grid, const float* w0,
                                                const float* b0, const float* wc, const float* tb,
                                                const float* tab, float* partial, int B, int T,
                                                int L, int N1, int N2, int C, int P1, int P2,
                                                int m1, int m2, const void* const* mX,
                                                const void* const* mG, void* const* mOut,
                                                const int* mshp, int nmj, void* stream) {
  const int Bn = B * L;
  if (!blindno_colspec_ok(Bn, C, P1, P2, m1, m2) || !Y || !tab || !wc || !partial || N1 > P1 ||
      N2 > P2 || nmj < 0 || nmj > 2)
    return (int)hipErrorInvalidValue;
  const BagLift bl{X, idx, grid, w0, b0, T, L, N1, N2};
  const int nb = zc_blocks1(Bn * (P1 / 16));
  SpecCol sc = spec_col(Y, nullptr, tab, P1);
  int64_t blocks = 0;
  for (int q = 0; q < nmj; ++q) {
    const int* sh = mshp + 7 * q;
    const int mBn = sh[0], Ci = sh[1], Co = sh[2], K1 = sh[3], mm2 = sh[4], ns = sh[5], Gw = sh[6];
    const int64_t total = (int64_t)mm2 * K1 * Ci * Co;
    if (mBn < 1 || Ci < 1 || Co < 1 || K1 < 1 || mm2 < 1 || ns < 1 || Gw < 1 || mBn % Gw ||
        total >= INT32_MAX / 2 || !mX[q] || !mG[q] || !mOut[q])
      return (int)hipErrorInvalidValue;
    MixWgradJob& m = sc.mj[q];
    m = MixWgradJob{};
    m.X = (const float2*)mX[q];
    m.Gs = (const float2*)mG[q];
    m.out = (float2*)mOut[q];
    m.Bn = mBn; m.Ci = Ci; m.Co = Co; m.K1 = K1; m.m2 = mm2;
    m.gx = (int)cdiv(total, kBlock);
    m.gy = ns;
    m.gz = Gw;
    sc.mcum[q] = (int)blocks;
    blocks += (int64_t)m.gx * ns * Gw;
  }
  if (blocks + nb >= INT32_MAX) return (int)hipErrorInvalidValue;
  sc.mcum[nmj] = (int)blocks;
  sc.nmj = nmj;
  sc.nmixb = (int)blocks;
  return rowinv_launch<1, 0, 1, 1, true>(nullptr, nullptr, dz, wc, nullptr, nullptr, tb, partial, nb, Bn,
                                         C, P1, P2, m2, (hipStream_t)stream, bl, 1, 0, 0, 0,
                                         RowDftNext{nullptr, nullptr, 0, 0}, sc);
}

BLINDNO_API int blindno_rowidft_bwd_lift_zc(const float* Y, const float* dz, const float* X,
                                            const int* idx, const float* grid, const float* w0,
                                            const float* b0, const float* wc, const float* tb,
                                            const float* tab, float* partial, int B, int T, int L,
                                            int N1, int N2, int C, int P1, int P2, int m1, int m2,
                                            void* stream) {
  return blindno_rowidft_bwd_lift_zc_mix(Y, dz, X, idx, grid, w0, b0, wc, tb, tab, partial, B, T, L,
                                         N1, N2, C, P1, P2, m1, m2, nullptr, nullptr, nullptr,
                                         nullptr, 0, stream);
}
