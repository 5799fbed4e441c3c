// 2D convolution (nn.Conv2d with bias, any kernel / stride / padding, groups 1) of the NIO
// snapshot encoders' ConvBlocks (2d_FPE/Baselines.py:40-52, Encoder2D :186-249, 1D Encoder
// :254-287), forward and both adjoints, as implicit GEMMs on the fp32 matrix cores
// (v_mfma_f32_16x16x4f32: exact fp32 products, fixed accumulation order -- deterministic).
//
//   FWD   y[n][co][p]   = b[co] + sum_{ci,kh,kw} W[co][ci][kh][kw] x[n][ci][tap(p,kh,kw)]
//         GEMM  M = Co, N = pixels (n, ho, wo), K = Ci KH KW
//   BWD_D dx[n][ci][q]  = sum_{co,kh,kw} W[co][ci][kh][kw] dy[n][co][(q + pad - k) / stride]
//         split into stride-phase classes (sub-pixel decomposition): input pixels with
//         (hi + ph) % sh = ah, (wi + pw) % sw = aw only meet taps kh = ah + sh j, kw = aw + sw j',
//         so each class (blockIdx.z) is its own GEMM  M = Ci, N = class pixels,
//         K = Co x (its taps) -- a stride-2 3x3 layer does 9/4 taps per pixel, not 9 (the taps
//         off the stride lattice are never visited)
//   BWD_W dW[co][ci][kh][kw] = sum_{n,p} dy[n][co][p] x[n][ci][tap(p,kh,kw)],  db[co] = sum dy
//         GEMM  M = Co, N = Ci KH KW + 1 (the extra column is the bias: B = 1), K = pixels,
//         split over blockIdx.z into fixed K ranges; the partials are reduced in a fixed order
//         afterwards (blindno_reduce_partials).
//
// Tiling for CDNA4 wave64: a 256-thread workgroup computes a BM x BN tile (128 x 128 for the
// large layers, 64 x 64 otherwise) as 2 x 2 waves of (BM/2) x (BN/2) (up to 4 x 4 MFMA blocks
// per wave, 4 accumulator VGPRs each), K in steps of 16 staged through double-buffered LDS.
// Where the channel count is a multiple of 16, the forward and the input gradient can order K
// tap-major (k = tap x C + c: no index divisions in the loop; see launch_igemm for where it is
// used), and layers whose output pixels leave the chip short of workgroups split K into
// partial slabs summed in a fixed order (blindno_conv2d_{fwd,bwd_data}_split).
// The LDS tiles are k-contiguous per row (A[m][k], B[n][k], rows padded to 20 floats) and the
// MFMA K order is permuted (step s takes k = 4 (lane>>4) + s), so one ds_read_b128 brings a
// lane's operands of four MFMA steps.  The next step's global loads are issued before the
// current step's MFMAs, so their latency hides behind 16 (64 x 64) or 64 (128 x 128) MFMAs per
// wave.  im2col is never materialised: each loader lane decodes its (channel, tap) / pixel
// indices with multiply-high divisions by the launch's constants (FastDiv).
#include "common.h"
#include "blindno.h"

using namespace blindno;

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

// MFMA shape: v_mfma_f32_16x16x4f32 (4 accumulators per lane).  The 32x32x2 form with the same
// wave tile measured the same (r03r: 39.1 vs 38.8 ms over the encoder's layers).
constexpr int MF = 16;
using Acc = f32x4;
constexpr int NR = 4;                             // accumulator registers per block
constexpr int KPL = 4;                            // k per lane in a 16-k chunk
__device__ __forceinline__ Acc mfma_step(float a, float b, Acc c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
// row of accumulator register r in a block for lane group gm
__device__ __forceinline__ int acc_row(int r, int gm) { return 4 * gm + r; }

// K per step and LDS row stride (floats) of the k-contiguous tiles.  BK = 32 (one barrier per 32
// k, 2 workgroups per CU) and a conflict-free-read stride of 24 measured slower / the same
// (r03q); the row stride 20 keeps the B tile's 16-B stores conflict-free.
constexpr int BK = 16;
constexpr int SK = BK + 4;

enum { FWD = 0, BWD_D = 1, BWD_W = 2 };

// one stride-phase class of BWD_D: input pixels hi = hi0 + sh t (t < Hc), wi = wi0 + sw u (u < Wc),
// taps kh = ah + sh jh (jh < nKh), kw = aw + sw jw (jw < nKw); output pixel ho = oh0 + t - jh,
// wo = ow0 + u - jw
constexpr int kMaxPhases = 16;   // sh, sw <= 4
struct Phase {
  int hi0, wi0, Hc, Wc, ah, aw, nKh, nKw, oh0, ow0, Ncol, K;
  FastDiv dHcWc, dWc, dKhw, dKw;
};

struct ConvArgs {
  int N, Ci, Hi, Wi, Co, Ho, Wo, KH, KW, sh, sw, ph, pw;
  int M, Ncol, K;               // GEMM sizes of this mode
  int kchunk;                   // K per split (multiple of BK; FWD / BWD_D: >= K unless split)
  int nph;                      // BWD_D: stride-phase classes (blockIdx.z = class + nph split)
  int64_t slab;                 // FWD / BWD_D split: floats per partial output slab
  int wt;                       // BWD_D tap-major: the weights come as Wt[tap][ci][co]
  int bsep;                     // BWD_W: the bias column (the last of Ncol) is not a GEMM column;
                                // the first column tile's workgroups form it as row sums of dy
  FastDiv dKHW, dKW, dHoWo, dWo, dHiWi, dWi;
  Phase phase[kMaxPhases];      // BWD_D
};

// ---- A operand (BM x BK tile), element (m, k) of global (m0 + m, k0 + k)
template <int MODE>
__device__ __forceinline__ float load_a(const float* __restrict__ pa, const ConvArgs& g,
                                        const Phase& ph, int mg, int kg, int kend) {
  if (mg >= g.M || kg >= kend) return 0.f;
  const int KHW = g.KH * g.KW;
  if (MODE == FWD) return pa[(int64_t)mg * g.K + kg];                       // W[co][k]
  if (MODE == BWD_D) {                                    // W[co][ci][ah + sh jh][aw + sw jw]
    const int nkk = ph.nKh * ph.nKw;
    const int co = (int)ph.dKhw.div((unsigned)kg), j = kg - co * nkk;
    const int jh = (int)ph.dKw.div((unsigned)j), jw = j - jh * ph.nKw;
    return pa[((int64_t)co * g.Ci + mg) * KHW + (ph.ah + g.sh * jh) * g.KW + ph.aw + g.sw * jw];
  }
  // BWD_W: dy[n][co][q], k = pixel
  const int HoWo = g.Ho * g.Wo;
  const int n = (int)g.dHoWo.div((unsigned)kg), q = kg - n * HoWo;
  return pa[((int64_t)n * g.Co + mg) * HoWo + q];
}

// pixel decomposition of the B operand's N index (FWD: output pixel, BWD_D: input pixel)
struct Pix {
  int64_t base;   // FWD: x offset of (n, 0, 0, 0); BWD_D: dy offset of (n, 0, 0, 0)
  int r, c;       // FWD: ho sh - ph, wo sw - pw; BWD_D: hi + ph, wi + pw
  bool ok;
};

template <int MODE>
__device__ __forceinline__ Pix decode_pix(const ConvArgs& g, const Phase& ph, int ng) {
  Pix p;
  p.ok = ng < (MODE == BWD_D ? ph.Ncol : g.Ncol);
  const int v = p.ok ? ng : 0;
  if (MODE == FWD) {
    const int HoWo = g.Ho * g.Wo;
    const int n = (int)g.dHoWo.div((unsigned)v), q = v - n * HoWo;
    const int ho = (int)g.dWo.div((unsigned)q), wo = q - ho * g.Wo;
    p.base = (int64_t)n * g.Ci * g.Hi * g.Wi;
    p.r = ho * g.sh - g.ph;
    p.c = wo * g.sw - g.pw;
  } else {
    // class-local pixel (n, t, u): output rows of its taps ho = oh0 + t - jh, wo = ow0 + u - jw
    const int HcWc = ph.Hc * ph.Wc;
    const int n = (int)ph.dHcWc.div((unsigned)v), q = v - n * HcWc;
    const int t = (int)ph.dWc.div((unsigned)q), u = q - t * ph.Wc;
    p.base = (int64_t)n * g.Co * g.Ho * g.Wo;
    p.r = ph.oh0 + t;
    p.c = ph.ow0 + u;
  }
  return p;
}

// output offset of BWD_D's class-local pixel
__device__ __forceinline__ int64_t dx_offset(const ConvArgs& g, const Phase& ph, int ng, int ci) {
  const int HcWc = ph.Hc * ph.Wc;
  const int n = (int)ph.dHcWc.div((unsigned)ng), q = ng - n * HcWc;
  const int t = (int)ph.dWc.div((unsigned)q), u = q - t * ph.Wc;
  return (((int64_t)n * g.Ci + ci) * g.Hi + ph.hi0 + g.sh * t) * g.Wi + ph.wi0 + g.sw * u;
}

// B element (k, pixel) for FWD / BWD_D
template <int MODE>
__device__ __forceinline__ float load_b_pix(const float* __restrict__ pb, const ConvArgs& g,
                                            const Phase& ph, const Pix& p, int kg, int kend) {
  if (!p.ok || kg >= kend) return 0.f;
  if (MODE == FWD) {
    const int KHW = g.KH * g.KW;
    const int ch = (int)g.dKHW.div((unsigned)kg), khw = kg - ch * KHW;
    const int kh = (int)g.dKW.div((unsigned)khw), kw = khw - kh * g.KW;
    const int hi = p.r + kh, wi = p.c + kw;
    if ((unsigned)hi >= (unsigned)g.Hi || (unsigned)wi >= (unsigned)g.Wi) return 0.f;
    return pb[p.base + ((int64_t)ch * g.Hi + hi) * g.Wi + wi];
  }
  const int nkk = ph.nKh * ph.nKw;
  const int co = (int)ph.dKhw.div((unsigned)kg), j = kg - co * nkk;
  const int jh = (int)ph.dKw.div((unsigned)j), jw = j - jh * ph.nKw;
  const int ho = p.r - jh, wo = p.c - jw;
  if ((unsigned)ho >= (unsigned)g.Ho || (unsigned)wo >= (unsigned)g.Wo) return 0.f;
  return pb[p.base + ((int64_t)co * g.Ho + ho) * g.Wo + wo];
}

// BWD_W B operand: column n = (ci, kh, kw) (or the bias column) fixed per thread and tile
struct Tap {
  int64_t coff;   // ci Hi Wi
  int kh, kw;
  int kind;       // 0 out of range, 1 tap, 2 bias column
};

__device__ __forceinline__ Tap decode_tap(const ConvArgs& g, int ng) {
  Tap t{0, 0, 0, 0};
  const int KHW = g.KH * g.KW;
  if (ng < g.Ci * KHW) {
    const int ci = (int)g.dKHW.div((unsigned)ng), khw = ng - ci * KHW;
    t.kh = (int)g.dKW.div((unsigned)khw);
    t.kw = khw - t.kh * g.KW;
    t.coff = (int64_t)ci * g.Hi * g.Wi;
    t.kind = 1;
  } else if (ng == g.Ci * KHW && !g.bsep) {
    t.kind = 2;
  }
  return t;
}

template <int MODE, int BM, int BN, bool TM = false>
__global__ __launch_bounds__(256) void conv_igemm_kernel(const float* __restrict__ pa,
                                                         const float* __restrict__ pb,
                                                         const float* __restrict__ bias,
                                                         float* __restrict__ out, ConvArgs g) {
  constexpr int EA = BM * BK / 256, EB = BN * BK / 256;  // loads per thread per K step (A, B)
  constexpr int AR = 256 / BK;                     // A rows (BWD_W: B columns) per load round
  constexpr int MI = BM / 2 / MF, NJ = BN / 2 / MF;  // MFMA blocks per wave
  __shared__ float As[2][BM * SK];
  __shared__ float Bs[2][BN * SK];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = uniform_int(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int cm = lane % MF, gm = lane / MF;         // block row / column, k group
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  // blockIdx.z: the K split (FWD, BWD_W), or class + nph x split (BWD_D).  Split FWD / BWD_D
  // launches write partial output slabs (out + split x slab), reduced afterwards in split order;
  // a split past a class's K writes its zeros (every slab covers every pixel)
  const int split = MODE == BWD_D ? (int)blockIdx.z / g.nph : (int)blockIdx.z;
  const Phase& ph = g.phase[MODE == BWD_D ? (int)blockIdx.z - split * g.nph : 0];
  if (MODE == BWD_D && n0 >= ph.Ncol) return;        // this class has fewer pixels (whole block)
  const int kbeg = split * g.kchunk;
  const int kend = min(MODE == BWD_D ? ph.K : g.K, kbeg + g.kchunk);
  if (MODE != BWD_W) out += split * g.slab;
  const int nk = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;

  // loader roles.  A: k = tid % 16 (contiguous in memory for all modes), m = tid / 16 + 16 e.
  // B (FWD / BWD_D): pixel n = tid % BN fixed for the tile, k = tid / BN + (256 / BN) e.
  // B (BWD_W): pixel k = tid % 16, column n = tid / 16 + 16 e (fixed taps for the tile).
  const int ak = tid % BK, am = tid / BK;
  const int bn = tid % BN, bk = tid / BN;
  constexpr int KS = 256 / BN;                    // k stride of a thread's B loads
  Pix pix{};
  Tap taps[EB];
  if (MODE != BWD_W) {
    pix = decode_pix<MODE>(g, ph, n0 + bn);
  } else {
#pragma unroll
    for (int e = 0; e < EB; ++e) taps[e] = decode_tap(g, n0 + am + AR * e);
  }

  // Tap-major K order (TM; FWD with Ci % 16 == 0, BWD_D with Co % 16 == 0): k = tap x C + c, so
  // the 16 k of a K-step share one tap and the channel advances by 16 per step.  The tap and
  // channel are uniform per step, each thread's A / B offsets are fixed per tile plus a uniform
  // part, and the only per-element work left is one add (and, for B, the padding select) --
  // no index divisions in the loop.  A rows past M read a clamped row (their results are never
  // stored); B columns whose tap falls in the padding read 0.
  // Offsets are 32-bit byte offsets from the uniform base (tensors < 2^30 floats, checked on the
  // host), so the loads take the scalar-base + vector-offset form.
  unsigned aoff[EA];
  int boff = 0, bstride = 0, tc = 0, t1 = 0, t2 = 0;   // uniform: channel, tap row, tap col
  bool bok = false;                                    // this step's tap inside the image
  if constexpr (TM && MODE != BWD_W) {
    const int KHW = g.KH * g.KW;
    const int C = MODE == FWD ? g.Ci : g.Co;
#pragma unroll
    for (int e = 0; e < EA; ++e) {
      const int mg = min(m0 + am + AR * e, g.M - 1);
      // g.wt: the weights were re-laid out tap-major (FWD Wf[co][tap][ci], BWD_D
      // Wt[tap][ci][co]), so a row's 16 k of a step are 64 contiguous bytes
      aoff[e] = 4u * (unsigned)(MODE == FWD ? (g.wt ? mg * g.K + ak : mg * g.K + ak * KHW)
                                : (g.wt ? mg * g.Co + ak : (ak * g.Ci + mg) * KHW));
    }
    const int cs = MODE == FWD ? g.Hi * g.Wi : g.Ho * g.Wo;   // B's channel stride
    boff = (int)pix.base + bk * EB * cs;             // this thread's EB consecutive channels
    bstride = cs;
    const int tap = kbeg / C;
    tc = kbeg - tap * C;
    const int ntw = MODE == FWD ? g.KW : ph.nKw;
    t1 = tap / ntw;
    t2 = tap - t1 * ntw;
  }

  // register staging: loads run one K-step ahead of the MFMAs (two steps ahead, with two
  // register sets, costs the 128 x 128 kernels an occupancy step: 3-8 % slower, r03t)
  float ra[EA], rb[EB];
  // BWD_W with g.bsep: db[co] = sum dy[co] over this split's pixels, summed on the A loads by
  // the first column tile's workgroups (the GEMM then has exactly Ci KH KW columns: a tile
  // holding only the bias column cost up to 10 % of the MFMAs, e.g. 1153 = 9 x 128 + 1)
  constexpr int EA4 = (TM && MODE == BWD_W) ? EA / 4 : 1;
  float bsum[EA4];
#pragma unroll
  for (int e = 0; e < EA4; ++e) bsum[e] = 0.f;
  const bool bcol = MODE == BWD_W && TM && g.bsep && blockIdx.x == 0;
  auto gload = [&](int kt) {
    const int k0 = kbeg + kt * BK;
    if constexpr (TM && MODE != BWD_W) {
      const int KHW = g.KH * g.KW;
      int hi, wi, u, cu;
      if (MODE == FWD) {
        hi = pix.r + t1;
        wi = pix.c + t2;
        u = g.wt ? (t1 * g.KW + t2) * g.Ci + tc : tc * KHW + t1 * g.KW + t2;
        cu = tc * g.Hi * g.Wi + hi * g.Wi + wi;
      } else {
        hi = pix.r - t1;
        wi = pix.c - t2;
        const int tap = (ph.ah + g.sh * t1) * g.KW + ph.aw + g.sw * t2;
        u = g.wt ? tap * g.Ci * g.Co + tc : tc * g.Ci * KHW + tap;
        cu = tc * g.Ho * g.Wo + hi * g.Wo + wi;
      }
      const int Hb = MODE == FWD ? g.Hi : g.Ho, Wb = MODE == FWD ? g.Wi : g.Wo;
      bok = pix.ok && (unsigned)hi < (unsigned)Hb && (unsigned)wi < (unsigned)Wb;
      const unsigned bo = bok ? 4u * (unsigned)(boff + cu) : 0u;
      const char* ca = reinterpret_cast<const char*>(pa) + 4u * (unsigned)u;
      const char* cb = reinterpret_cast<const char*>(pb);
#pragma unroll
      for (int e = 0; e < EA; ++e) ra[e] = *reinterpret_cast<const float*>(ca + aoff[e]);
      // the padding select happens at the LDS store (after the MFMAs), not here, so the
      // loads stay in flight
#pragma unroll
      for (int e = 0; e < EB; ++e) rb[e] = *reinterpret_cast<const float*>(cb + (bo + 4u * (unsigned)(e * bstride)));
      // next step: channel + 16, carrying into the tap
      const int C = MODE == FWD ? g.Ci : g.Co;
      const int ntw = MODE == FWD ? g.KW : ph.nKw;
      tc += BK;
      if (tc == C) {
        tc = 0;
        if (++t2 == ntw) {
          t2 = 0;
          ++t1;
        }
      }
      return;
    }
    if constexpr (TM && MODE == BWD_W) {
      // vectorised A (dy): thread (row t / 4 + 64 e, pixels 4 (t % 4) .. + 3) -- one 16-B load
      // per 4 pixels of one plane (HoWo % 4 == 0, the host checks; kend is a multiple of 4)
      const int kg = k0 + 4 * (tid & 3);
      const bool kok = kg < kend;
      const int HoWo = g.Ho * g.Wo;
      const int v = kok ? kg : 0;
      const int n = (int)g.dHoWo.div((unsigned)v), q = v - n * HoWo;
#pragma unroll
      for (int e = 0; e < EA / 4; ++e) {
        const int mg = min(m0 + (tid >> 2) + 64 * e, g.M - 1);
        const f32x4 a4 = kok ? *reinterpret_cast<const f32x4*>(pa + ((int64_t)n * g.Co + mg) * HoWo + q)
                             : (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int r = 0; r < 4; ++r) ra[4 * e + r] = a4[r];
        if (bcol) bsum[e] += (a4[0] + a4[1]) + (a4[2] + a4[3]);
      }
    } else {
#pragma unroll
      for (int e = 0; e < EA; ++e) ra[e] = load_a<MODE>(pa, g, ph, m0 + am + AR * e, k0 + ak, kend);
    }
    if (MODE != BWD_W) {
#pragma unroll
      for (int e = 0; e < EB; ++e) rb[e] = load_b_pix<MODE>(pb, g, ph, pix, k0 + bk + KS * e, kend);
    } else {
      const int kg = k0 + ak;                          // this thread's pixel
      const bool kok = kg < kend;
      const int HoWo = g.Ho * g.Wo;
      const int v = kok ? kg : 0;
      const int n = (int)g.dHoWo.div((unsigned)v), q = v - n * HoWo;
      const int ho = (int)g.dWo.div((unsigned)q), wo = q - ho * g.Wo;
      const int64_t xb = (int64_t)n * g.Ci * g.Hi * g.Wi;
      const int r0 = ho * g.sh - g.ph, c0 = wo * g.sw - g.pw;
#pragma unroll
      for (int e = 0; e < EB; ++e) {
        float v2 = 0.f;
        if (kok && taps[e].kind == 1) {
          const int hi = r0 + taps[e].kh, wi = c0 + taps[e].kw;
          if ((unsigned)hi < (unsigned)g.Hi && (unsigned)wi < (unsigned)g.Wi)
            v2 = pb[xb + taps[e].coff + (int64_t)hi * g.Wi + wi];
        } else if (kok && taps[e].kind == 2) {
          v2 = 1.f;
        }
        rb[e] = v2;
      }
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int e = 0; e < EA; ++e)
      if constexpr (!(TM && MODE == BWD_W)) As[buf][(am + AR * e) * SK + ak] = ra[e];
    if constexpr (TM && MODE == BWD_W) {
#pragma unroll
      for (int e = 0; e < EA / 4; ++e)
        *reinterpret_cast<f32x4*>(&As[buf][((tid >> 2) + 64 * e) * SK + 4 * (tid & 3)]) =
            (f32x4){ra[4 * e], ra[4 * e + 1], ra[4 * e + 2], ra[4 * e + 3]};
    }
    if constexpr (TM && MODE != BWD_W) {
      // k = bk EB + e: 16-B stores of consecutive k; 8 lanes of consecutive rows cover all 32
      // banks (row stride SK = 20 / 36 floats), so the stores are conflict-free
#pragma unroll
      for (int q = 0; q < EB / 4; ++q) {
        f32x4 v;
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = bok ? rb[4 * q + r] : 0.f;
        *reinterpret_cast<f32x4*>(&Bs[buf][bn * SK + bk * EB + 4 * q]) = v;
      }
    } else if (MODE != BWD_W) {
#pragma unroll
      for (int e = 0; e < EB; ++e) Bs[buf][bn * SK + bk + KS * e] = rb[e];
    } else {
#pragma unroll
      for (int e = 0; e < EB; ++e) Bs[buf][(am + AR * e) * SK + ak] = rb[e];
    }
  };

  Acc acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < NR; ++r) acc[i][j][r] = 0.f;

  if (nk > 0) {
    gload(0);
    sstore(0);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1;
      if (kt + 1 < nk) gload(kt + 1);
      const float* as = As[cur];
      const float* bs = Bs[cur];
      // lane (cm, gm) supplies k = 16 kq + KPL gm + s in MFMA step s: KPL / 4 16-B reads per
      // block (the MFMA K order is permuted consistently for A and B)
#pragma unroll
      for (int kq = 0; kq < BK / 16; ++kq) {
        f32x4 av[MI][KPL / 4], bv[NJ][KPL / 4];
#pragma unroll
        for (int q = 0; q < KPL / 4; ++q) {
#pragma unroll
          for (int i = 0; i < MI; ++i)
            av[i][q] = *reinterpret_cast<const f32x4*>(as + (wm * (BM / 2) + i * MF + cm) * SK + 16 * kq + KPL * gm + 4 * q);
#pragma unroll
          for (int j = 0; j < NJ; ++j)
            bv[j][q] = *reinterpret_cast<const f32x4*>(bs + (wn * (BN / 2) + j * MF + cm) * SK + 16 * kq + KPL * gm + 4 * q);
        }
#pragma unroll
        for (int st = 0; st < KPL; ++st)
#pragma unroll
          for (int i = 0; i < MI; ++i)
#pragma unroll
            for (int j = 0; j < NJ; ++j)
              acc[i][j] = mfma_step(av[i][st >> 2][st & 3], bv[j][st >> 2][st & 3], acc[i][j]);
      }
      if (kt + 1 < nk) sstore(cur ^ 1);
      __syncthreads();
    }
  }

  if constexpr (MODE == BWD_W && TM) {
    if (bcol) {
      // the 4 threads of a row (tid & 3: adjacent lanes) in a fixed butterfly order
#pragma unroll
      for (int e = 0; e < EA4; ++e) {
        float v = bsum[e];
        v += __shfl_xor(v, 1, 64);
        v += __shfl_xor(v, 2, 64);
        const int mg = m0 + (tid >> 2) + 64 * e;
        if ((tid & 3) == 0 && mg < g.M) out[((int64_t)blockIdx.z * g.M + mg) * g.Ncol + g.Ncol - 1] = v;
      }
    }
  }

  // epilogue: lane holds rows acc_row(r, gm) of column cm of each MF x MF block
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int ng = n0 + wn * (BN / 2) + j * MF + cm;
    if (ng >= g.Ncol - (MODE == BWD_W ? g.bsep : 0)) continue;
    if (MODE == BWD_W) {
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int r = 0; r < NR; ++r) {
          const int mg = m0 + wm * (BM / 2) + i * MF + acc_row(r, gm);
          if (mg < g.M) out[((int64_t)blockIdx.z * g.M + mg) * g.Ncol + ng] = acc[i][j][r];
        }
    } else if (MODE == FWD) {
      const int HW = g.Ho * g.Wo;
      const int n = (int)g.dHoWo.div((unsigned)ng), q = ng - n * HW;
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int r = 0; r < NR; ++r) {
          const int mg = m0 + wm * (BM / 2) + i * MF + acc_row(r, gm);
          if (mg < g.M) out[((int64_t)n * g.M + mg) * HW + q] = acc[i][j][r] + (bias && split == 0 ? bias[mg] : 0.f);
        }
    } else {
      if (ng >= ph.Ncol) continue;
      const int64_t o0 = dx_offset(g, ph, ng, 0), cs = (int64_t)g.Hi * g.Wi;
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int r = 0; r < NR; ++r) {
          const int mg = m0 + wm * (BM / 2) + i * MF + acc_row(r, gm);
          if (mg < g.M) out[o0 + mg * cs] = acc[i][j][r];
        }
    }
  }
}

// Tap-major weight layouts of the A operand (one pass over the weights, <= 9.4 MB):
//   FWD   W[co][ci][tap] -> Wf[co][tap][ci]   (k = tap Ci + ci contiguous per output channel)
//   BWD_D W[co][ci][tap] -> Wt[tap][ci][co]   (k = co contiguous per (tap, input channel))
// Without them the tap-major loaders read 16 k of a step at a stride of KH KW (forward) or
// Ci KH KW (input gradient) floats, a cache line per lane: the input gradient ran 71 -> 101
// TFLOP/s with the re-layout (r03zd).
template <int MODE>
__global__ void weight_relayout_kernel(const float* __restrict__ w, float* __restrict__ wt, int Co,
                                       int Ci, int KHW) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;     // output index
  if (i >= Co * Ci * KHW) return;
  int co, ci, tap;
  if (MODE == FWD) {
    ci = i % Ci;
    const int r = i / Ci;
    tap = r % KHW;
    co = r / KHW;
  } else {
    co = i % Co;
    const int r = i / Co;
    ci = r % Ci;
    tap = r / Ci;
  }
  wt[i] = w[((int64_t)co * Ci + ci) * KHW + tap];
}

bool make_args(ConvArgs& g, int N, int Ci, int Hi, int Wi, int Co, int KH, int KW, int sh, int sw,
               int ph, int pw) {
  if (N < 1 || Ci < 1 || Hi < 1 || Wi < 1 || Co < 1 || KH < 1 || KW < 1 || sh < 1 || sw < 1 ||
      ph < 0 || pw < 0)
    return false;
  const int Ho = (Hi + 2 * ph - KH) / sh + 1, Wo = (Wi + 2 * pw - KW) / sw + 1;
  if (Ho < 1 || Wo < 1) return false;
  // every tensor index and GEMM extent below 2^31 (32-bit pixel / k indices, FastDiv range)
  const int64_t xin = (int64_t)N * Ci * Hi * Wi, yout = (int64_t)N * Co * Ho * Wo;
  if (xin >= INT32_MAX || yout >= INT32_MAX || (int64_t)Co * Ci * KH * KW >= INT32_MAX) return false;
  g.N = N; g.Ci = Ci; g.Hi = Hi; g.Wi = Wi; g.Co = Co; g.Ho = Ho; g.Wo = Wo;
  g.KH = KH; g.KW = KW; g.sh = sh; g.sw = sw; g.ph = ph; g.pw = pw;
  g.kchunk = 0;
  g.nph = 1;
  g.slab = 0;
  g.wt = 0;
  g.bsep = 0;
  g.dKHW = FastDiv::make((unsigned)(KH * KW));
  g.dKW = FastDiv::make((unsigned)KW);
  g.dHoWo = FastDiv::make((unsigned)(Ho * Wo));
  g.dWo = FastDiv::make((unsigned)Wo);
  g.dHiWi = FastDiv::make((unsigned)(Hi * Wi));
  g.dWi = FastDiv::make((unsigned)Wi);
  return true;
}

// 128 x 128 tiles where the GEMM has the rows and enough column tiles (over all stride-phase
// classes) to fill the chip -- two workgroups per CU; 64 x 64 otherwise.  BWD_W (split over K)
// only needs the extents, and so does a forward with >= 4 column tiles, whose K split then
// fills the chip (dk_splits; the 8 x 4 and 4 x 2 outputs of the last blocks, r03z: -4 / -9 %).
// The input gradient keeps 64 x 64 rather than split its classes' uneven K (r03z: 1.5x slower).
#ifndef CONV_BIG_MIN_TILES
#define CONV_BIG_MIN_TILES 512
#endif
bool big_tiles(int mode, int M, int Ncol, int classes) {
  if (M < 128 || Ncol < 128) return false;
  if (mode == BWD_W || (mode == FWD && Ncol >= 512)) return true;
  return (int64_t)cdiv(M, 128) * cdiv(Ncol, 128) * classes >= CONV_BIG_MIN_TILES;
}

// 64 x 128 tiles for the input gradients with 64 input channels and many columns (the second
// block's, r03zb: 1.85 -> 1.40 ms with the tap-major order; the first block's forward, memory-
// bound, gains nothing)
bool wide_tiles(int mode, int M, int Ncol, int classes) {
  if (mode != BWD_D || M > 64 || M < 48) return false;
  return (int64_t)cdiv(Ncol, 128) * classes >= CONV_BIG_MIN_TILES;
}

#ifndef CONV_TM
#define CONV_TM 1
#endif
template <int MODE, bool TM>
void launch_igemm_t(dim3 g3, int M, int Ncol, const float* pa, const float* pb, const float* bias,
                    float* out, const ConvArgs& g, hipStream_t st) {
  if (big_tiles(MODE, M, Ncol, MODE == BWD_D ? g.nph : 1)) {
    g3.x = cdiv(Ncol, 128);
    g3.y = cdiv(M, 128);
    conv_igemm_kernel<MODE, 128, 128, TM><<<g3, 256, 0, st>>>(pa, pb, bias, out, g);
  } else if (wide_tiles(MODE, M, Ncol, MODE == BWD_D ? g.nph : 1)) {
    g3.x = cdiv(Ncol, 128);
    g3.y = cdiv(M, 64);
    conv_igemm_kernel<MODE, 64, 128, TM><<<g3, 256, 0, st>>>(pa, pb, bias, out, g);
  } else {
    g3.x = cdiv(Ncol, 64);
    g3.y = cdiv(M, 64);
    conv_igemm_kernel<MODE, 64, 64, TM><<<g3, 256, 0, st>>>(pa, pb, bias, out, g);
  }
}

// the tap-major loaders where the K-step channel blocks are whole (C % 16 == 0) and the tensors'
// byte offsets fit 32 bits
#ifndef CONV_VA
#define CONV_VA 1
#endif
bool use_tm(int mode, const ConvArgs& g) {
  const int64_t big = (int64_t)1 << 30;
  // where it pays (measured, profiles/r03/r03ze_conv_weight_relayout_ab.txt): with the weights
  // re-laid out, every input gradient and every forward with >= 16 output pixels per image (the
  // 4 x 2 and 1 x 1 outputs of the last blocks keep the channel-major order: -8 / -16 % there)
  const bool pays = CONV_TM == 2 || mode == BWD_D || g.Ho * g.Wo >= 16;
  if (mode == BWD_W)   // vectorised dy loads (16-B aligned planes)
    return CONV_VA && (g.Ho * g.Wo) % 4 == 0 && (int64_t)g.N * g.Co * g.Ho * g.Wo < big;
  return CONV_TM && pays && (mode == FWD ? g.Ci : g.Co) % BK == 0 &&
         (int64_t)g.N * g.Ci * g.Hi * g.Wi < big && (int64_t)g.N * g.Co * g.Ho * g.Wo < big &&
         (int64_t)g.Co * g.Ci * g.KH * g.KW < big;
}

template <int MODE>
void launch_igemm(dim3 g3, int M, int Ncol, const float* pa, const float* pb, const float* bias,
                  float* out, const ConvArgs& g, hipStream_t st) {
  // BWD_W's vector loads read dy (pa) as f32x4: a C host may hand an offset pointer
  const bool aligned = MODE != BWD_W || ((uintptr_t)pa & 15) == 0;
  if (aligned && use_tm(MODE, g)) return launch_igemm_t<MODE, true>(g3, M, Ncol, pa, pb, bias, out, g, st);
  launch_igemm_t<MODE, false>(g3, M, Ncol, pa, pb, bias, out, g, st);
}

// the weights in the tap-major layout of `mode` into wscratch (when given and the launch uses
// the tap-major loaders): returns the A operand to use
template <int MODE>
const float* relayout_weights(const float* w, float* wscratch, ConvArgs& g, hipStream_t st) {
  g.wt = 0;
  if (!wscratch || !use_tm(MODE, g)) return w;
  const int KHW = g.KH * g.KW;
  const int total = g.Co * g.Ci * KHW;
  weight_relayout_kernel<MODE><<<cdiv(total, 256), 256, 0, st>>>(w, wscratch, g.Co, g.Ci, KHW);
  g.wt = 1;
  return wscratch;
}

// FWD / BWD_D: split K when the output tiles leave the chip short of workgroups (the encoder's
// last layers: a few thousand output pixels, K = 512 x 9).  Aim at >= 1024 workgroups with
// >= 16 K-steps per split.
#ifndef CONV_SPLIT
#define CONV_SPLIT 1
#endif
int dk_splits(int mode, int M, int Ncol, int K, int classes) {
  if (!CONV_SPLIT) return 1;
  const bool big = big_tiles(mode, M, Ncol, classes);
  const int TM_ = big ? 128 : 64, TN = big || wide_tiles(mode, M, Ncol, classes) ? 128 : 64;
  const int64_t tiles = (int64_t)cdiv(M, TM_) * cdiv(Ncol, TN) * classes;
  if (tiles >= 512) return 1;
  int64_t s = cdiv(1024, tiles);
  const int64_t maxs = cdiv(K, 16 * BK);
  if (s > maxs) s = maxs;
  if (s > 16) s = 16;
  return (int)(s < 1 ? 1 : s);
}

int wgrad_splits(const ConvArgs& g) {
  const int T = big_tiles(BWD_W, g.M, g.Ncol, 1) ? 128 : 64;
  const int64_t tiles = (int64_t)cdiv(g.M, T) * cdiv(g.Ncol, T);
  const int64_t ksteps = cdiv(g.K, BK);
  // aim at >= 4096 workgroups: more, shorter K ranges hide the gather latency better than
  // the partial sums cost (config D 121.6 -> 122.6 bags/s; 1024 / 512: 117.9 / 111.4, r03zi-j)
  int64_t s = cdiv(4096, tiles);
  const int64_t maxs = cdiv(ksteps, 8);          // but >= 8 K-steps per split
  if (s > maxs) s = maxs;
  if (s > 1024) s = 1024;
  return (int)(s < 1 ? 1 : s);
}

}  // namespace

namespace {

bool fwd_args(ConvArgs& g, int N, int Ci, int Hi, int Wi, int Co, int KH, int KW, int sh, int sw,
              int ph, int pw) {
  if (!make_args(g, N, Ci, Hi, Wi, Co, KH, KW, sh, sw, ph, pw)) return false;
  g.M = Co;
  g.Ncol = N * g.Ho * g.Wo;
  g.K = Ci * KH * KW;
  g.kchunk = cdiv(g.K, BK) * BK;
  g.slab = (int64_t)N * Co * g.Ho * g.Wo;
  return true;
}

// stride-phase classes of BWD_D; returns the largest class's pixel count, *uncovered when some
// pixels' classes have no taps (they receive no gradient: only when the stride exceeds the
// kernel extent)
int bwd_data_args(ConvArgs& g, int N, int Ci, int Hi, int Wi, int Co, int KH, int KW, int sh,
                  int sw, int ph, int pw, bool* uncovered) {
  if (sh * sw > kMaxPhases || !make_args(g, N, Ci, Hi, Wi, Co, KH, KW, sh, sw, ph, pw)) return -1;
  g.M = Ci;
  g.Ncol = N * Hi * Wi;
  g.K = Co * KH * KW;
  g.nph = sh * sw;
  g.slab = (int64_t)N * Ci * Hi * Wi;
  int maxcol = 1, maxk = BK;
  *uncovered = false;
  for (int ah = 0; ah < sh; ++ah)
    for (int aw = 0; aw < sw; ++aw) {
      Phase& p = g.phase[ah * sw + aw];
      p.ah = ah;
      p.aw = aw;
      p.hi0 = ((ah - ph) % sh + sh) % sh;
      p.wi0 = ((aw - pw) % sw + sw) % sw;
      p.Hc = p.hi0 < Hi ? (Hi - p.hi0 + sh - 1) / sh : 0;
      p.Wc = p.wi0 < Wi ? (Wi - p.wi0 + sw - 1) / sw : 0;
      p.nKh = ah < KH ? (KH - ah + sh - 1) / sh : 0;
      p.nKw = aw < KW ? (KW - aw + sw - 1) / sw : 0;
      p.oh0 = (p.hi0 + ph - ah) / sh;
      p.ow0 = (p.wi0 + pw - aw) / sw;
      p.Ncol = N * p.Hc * p.Wc;
      p.K = Co * p.nKh * p.nKw;
      if (p.K == 0 && p.Ncol > 0) *uncovered = true;
      if (p.K == 0) p.Ncol = 0;
      p.dHcWc = FastDiv::make((unsigned)(p.Hc * p.Wc > 0 ? p.Hc * p.Wc : 1));
      p.dWc = FastDiv::make((unsigned)(p.Wc > 0 ? p.Wc : 1));
      p.dKhw = FastDiv::make((unsigned)(p.nKh * p.nKw > 0 ? p.nKh * p.nKw : 1));
      p.dKw = FastDiv::make((unsigned)(p.nKw > 0 ? p.nKw : 1));
      if (p.Ncol > maxcol) maxcol = p.Ncol;
      if (p.K > maxk) maxk = p.K;
    }
  g.kchunk = cdiv(maxk, BK) * BK;
  return maxcol;
}

// the K range of each of nsplit splits (multiple of BK); the number of splits that remain
int set_split(ConvArgs& g, int nsplit) {
  const int kmax = g.kchunk;
  g.kchunk = cdiv(cdiv(kmax, nsplit), BK) * BK;
  return cdiv(kmax, g.kchunk);
}

}  // namespace

BLINDNO_API int blindno_conv2d_fwd_nsplit(int N, int Ci, int Hi, int Wi, int Co, int KH, int KW,
                                          int sh, int sw, int ph, int pw) {
  ConvArgs g;
  if (!fwd_args(g, N, Ci, Hi, Wi, Co, KH, KW, sh, sw, ph, pw)) return -1;
  return dk_splits(FWD, g.M, g.Ncol, g.K, 1);
}

namespace {
// A convolution whose kernel covers the whole (unpadded) input is a dense layer: its input
// gradient dX (N, Ci KH KW) = dY (N, Co) W (Co, Ci KH KW) runs as a forward 1x1 convolution of dY
// with W^T (from the weight scratch) instead of an implicit GEMM whose taps are 1 / (KH KW)
// inside the image (the 1x1-output last encoder block: 190 -> ~40 us)
bool full_kernel(int Hi, int Wi, int KH, int KW, int ph, int pw) {
  return KH == Hi && KW == Wi && ph == 0 && pw == 0 && Hi * Wi > 1;
}

}  // namespace

BLINDNO_API int blindno_conv2d_wscratch_floats(int mode, int N, int Ci, int Hi, int Wi, int Co,
                                               int KH, int KW, int sh, int sw, int ph, int pw) {
  ConvArgs g;
  bool unc;
  if (mode == FWD) {
    if (!fwd_args(g, N, Ci, Hi, Wi, Co, KH, KW, sh, sw, ph, pw)) return -1;
  } else if (mode == BWD_D) {
    if (bwd_data_args(g, N, Ci, Hi, Wi, Co, KH, KW, sh, sw, ph, pw, &unc) < 0) return -1;
    if (full_kernel(Hi, Wi, KH, KW, ph, pw)) return Co * Ci * KH * KW;   // W^T
  } else {
    return -1;
  }
  return use_tm(mode, g) ? Co * Ci * KH * KW : 0;
}

BLINDNO_API int blindno_conv2d_fwd_split(const float* x, const float* w, const float* b, float* y,
                                         float* partial, int nsplit, float* wscratch, int N, int Ci,
                                         int Hi, int Wi, int Co, int KH, int KW, int sh, int sw,
                                         int ph, int pw, void* stream) {
  ConvArgs g;
  if (!x || !w || !y || nsplit < 1 || (nsplit > 1 && !partial) ||
      !fwd_args(g, N, Ci, Hi, Wi, Co, KH, KW, sh, sw, ph, pw))
    return (int)hipErrorInvalidValue;
  const int nz = set_split(g, nsplit);
  if (nz > 1 && g.slab >= INT32_MAX / nz) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  const float* wa = relayout_weights<FWD>(w, wscratch, g, st);
  launch_igemm<FWD>(dim3(1, 1, nz), g.M, g.Ncol, wa, x, b, nz > 1 ? partial : y, g, st);
  const int e = (int)hipGetLastError();
  if (e || nz == 1) return e;
  return blindno_reduce_partials(partial, y, nz, (int)g.slab, stream);
}

BLINDNO_API int blindno_conv2d_fwd(const float* x, const float* w, const float* b, float* y, int N,
                                   int Ci, int Hi, int Wi, int Co, int KH, int KW, int sh, int sw,
                                   int ph, int pw, void* stream) {
  return blindno_conv2d_fwd_split(x, w, b, y, nullptr, 1, nullptr, N, Ci, Hi, Wi, Co, KH, KW, sh, sw,
                                  ph, pw, stream);
}

BLINDNO_API int blindno_conv2d_bwd_data_nsplit(int N, int Ci, int Hi, int Wi, int Co, int KH, int KW,
                                               int sh, int sw, int ph, int pw) {
  ConvArgs g;
  bool unc;
  const int maxcol = bwd_data_args(g, N, Ci, Hi, Wi, Co, KH, KW, sh, sw, ph, pw, &unc);
  if (maxcol < 0) return -1;
  if (full_kernel(Hi, Wi, KH, KW, ph, pw)) {
    ConvArgs f;
    if (!fwd_args(f, N, Co, 1, 1, Ci * KH * KW, 1, 1, 1, 1, 0, 0)) return -1;
    return dk_splits(FWD, f.M, f.Ncol, f.K, 1);
  }
  return dk_splits(BWD_D, g.M, maxcol, g.kchunk, g.nph);
}

BLINDNO_API int blindno_conv2d_bwd_data_split(const float* dy, const float* w, float* dx,
                                              float* partial, int nsplit, float* wscratch, int N,
                                              int Ci, int Hi, int Wi, int Co, int KH, int KW, int sh,
                                              int sw, int ph, int pw, void* stream) {
  ConvArgs g;
  bool uncovered;
  if (!dy || !w || !dx || nsplit < 1 || (nsplit > 1 && !partial)) return (int)hipErrorInvalidValue;
  const int maxcol = bwd_data_args(g, N, Ci, Hi, Wi, Co, KH, KW, sh, sw, ph, pw, &uncovered);
  if (maxcol < 0) return (int)hipErrorInvalidValue;
  if (wscratch && full_kernel(Hi, Wi, KH, KW, ph, pw)) {
    const int K = Ci * KH * KW;
    ConvArgs f;
    if (!fwd_args(f, N, Co, 1, 1, K, 1, 1, 1, 1, 0, 0)) return (int)hipErrorInvalidValue;
    const int nzf = set_split(f, nsplit);
    if (nzf > 1 && f.slab >= INT32_MAX / nzf) return (int)hipErrorInvalidValue;
    hipStream_t st = (hipStream_t)stream;
    // W (Co, K) -> W^T (K, Co): the relayout kernel with one tap and K "input channels"
    weight_relayout_kernel<BWD_D><<<cdiv(Co * K, 256), 256, 0, st>>>(w, wscratch, Co, K, 1);
    launch_igemm<FWD>(dim3(1, 1, nzf), f.M, f.Ncol, wscratch, dy, nullptr, nzf > 1 ? partial : dx, f,
                      st);
    const int e = (int)hipGetLastError();
    if (e || nzf == 1) return e;
    return blindno_reduce_partials(partial, dx, nzf, (int)f.slab, stream);
  }
  const int nz = set_split(g, nsplit);
  if (nz > 1 && g.slab >= INT32_MAX / nz) return (int)hipErrorInvalidValue;
  float* out = nz > 1 ? partial : dx;
  hipStream_t st = (hipStream_t)stream;
  if (uncovered) {
    const hipError_t e = hipMemsetAsync(out, 0, sizeof(float) * (size_t)g.slab * nz, st);
    if (e != hipSuccess) return (int)e;
  }
  const float* wa = relayout_weights<BWD_D>(w, wscratch, g, st);
  launch_igemm<BWD_D>(dim3(1, 1, g.nph * nz), g.M, maxcol, wa, dy, nullptr, out, g, st);
  const int e = (int)hipGetLastError();
  if (e || nz == 1) return e;
  return blindno_reduce_partials(partial, dx, nz, (int)g.slab, stream);
}

BLINDNO_API int blindno_conv2d_bwd_data(const float* dy, const float* w, float* dx, int N, int Ci,
                                        int Hi, int Wi, int Co, int KH, int KW, int sh, int sw,
                                        int ph, int pw, void* stream) {
  return blindno_conv2d_bwd_data_split(dy, w, dx, nullptr, 1, nullptr, N, Ci, Hi, Wi, Co, KH, KW, sh,
                                       sw, ph, pw, stream);
}

BLINDNO_API int blindno_conv2d_wgrad_nsplit(int N, int Ci, int Hi, int Wi, int Co, int KH, int KW,
                                            int sh, int sw, int ph, int pw) {
  ConvArgs g;
  if (!make_args(g, N, Ci, Hi, Wi, Co, KH, KW, sh, sw, ph, pw)) return -1;
  g.M = Co;
  g.Ncol = Ci * KH * KW + 1;
  g.K = N * g.Ho * g.Wo;
  return wgrad_splits(g);
}

#ifndef CONV_BSEP
#define CONV_BSEP 1
#endif
BLINDNO_API int blindno_conv2d_bwd_weight(const float* dy, const float* x, float* dwb,
                                          float* partial, int nsplit, int N, int Ci, int Hi, int Wi,
                                          int Co, int KH, int KW, int sh, int sw, int ph, int pw,
                                          void* stream) {
  ConvArgs g;
  if (!dy || !x || !dwb || nsplit < 1 || (nsplit > 1 && !partial) ||
      !make_args(g, N, Ci, Hi, Wi, Co, KH, KW, sh, sw, ph, pw))
    return (int)hipErrorInvalidValue;
  g.M = Co;
  g.Ncol = Ci * KH * KW + 1;
  g.K = N * g.Ho * g.Wo;
  g.kchunk = cdiv(cdiv(g.K, nsplit), BK) * BK;
  const int nz = cdiv(g.K, g.kchunk);
  if ((int64_t)g.M * g.Ncol >= INT32_MAX / (nz > 0 ? nz : 1)) return (int)hipErrorInvalidValue;
  hipStream_t st = (hipStream_t)stream;
  // the vectorised (tap-major) loaders form the bias column from dy's row sums (bsep); the
  // column grid then covers the Ci KH KW weight columns only (launch_igemm takes the TM form
  // under exactly this condition)
  g.bsep = (CONV_BSEP && ((uintptr_t)dy & 15) == 0 && use_tm(BWD_W, g)) ? 1 : 0;
  launch_igemm<BWD_W>(dim3(1, 1, nz), g.M, g.Ncol - g.bsep, dy, x, nullptr, nz > 1 ? partial : dwb, g,
                      st);
  if (nz > 1) {
    const int e = (int)hipGetLastError();
    if (e) return e;
    return blindno_reduce_partials(partial, dwb, nz, g.M * g.Ncol, stream);
  }
  return (int)hipGetLastError();
}
