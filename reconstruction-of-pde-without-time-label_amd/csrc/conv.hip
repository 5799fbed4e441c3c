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

constexpr int BK = 16;
constexpr int SK = BK + 4;                     // LDS row stride (floats) of the k-contiguous tiles

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
  int kchunk;                   // BWD_W: K per split (multiple of BK)
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
  } else if (ng == g.Ci * KHW) {
    t.kind = 2;
  }
  return t;
}

template <int MODE, int BM, int BN>
__global__ __launch_bounds__(256) void conv_igemm_kernel(const float* __restrict__ pa,
                                                         const float* __restrict__ pb,
                                                         const float* __restrict__ bias,
                                                         float* __restrict__ out, ConvArgs g) {
  constexpr int EA = BM / 16, EB = BN * BK / 256;  // loads per thread per K step (A, B)
  constexpr int MI = BM / 32, NJ = BN / 32;        // MFMA blocks per wave
  __shared__ float As[2][BM * SK];
  __shared__ float Bs[2][BN * SK];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = uniform_int(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int c16 = lane & 15, g4 = lane >> 4;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  const Phase& ph = g.phase[MODE == BWD_D ? blockIdx.z : 0];
  if (MODE == BWD_D && n0 >= ph.Ncol) return;        // this class has fewer pixels (whole block)
  int kbeg = 0, kend = MODE == BWD_D ? ph.K : g.K;
  if (MODE == BWD_W) {
    kbeg = blockIdx.z * g.kchunk;
    kend = min(g.K, kbeg + g.kchunk);
  }
  const int nk = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;

  // loader roles.  A: k = tid % 16 (contiguous in memory for all modes), m = tid / 16 + 16 e.
  // B (FWD / BWD_D): pixel n = tid % BN fixed for the tile, k = tid / BN + (256 / BN) e.
  // B (BWD_W): pixel k = tid % 16, column n = tid / 16 + 16 e (fixed taps for the tile).
  const int ak = tid & 15, am = tid >> 4;
  const int bn = tid % BN, bk = tid / BN;
  constexpr int KS = 256 / BN;                    // k stride of a thread's B loads
  Pix pix{};
  Tap taps[EB];
  if (MODE != BWD_W) {
    pix = decode_pix<MODE>(g, ph, n0 + bn);
  } else {
#pragma unroll
    for (int e = 0; e < EB; ++e) taps[e] = decode_tap(g, n0 + (tid >> 4) + 16 * e);
  }

  float ra[EA], rb[EB];
  auto gload = [&](int kt) {
    const int k0 = kbeg + kt * BK;
#pragma unroll
    for (int e = 0; e < EA; ++e) ra[e] = load_a<MODE>(pa, g, ph, m0 + am + 16 * e, k0 + ak, kend);
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
    for (int e = 0; e < EA; ++e) As[buf][(am + 16 * e) * SK + ak] = ra[e];
    if (MODE != BWD_W) {
#pragma unroll
      for (int e = 0; e < EB; ++e) Bs[buf][bn * SK + bk + KS * e] = rb[e];
    } else {
#pragma unroll
      for (int e = 0; e < EB; ++e) Bs[buf][((tid >> 4) + 16 * e) * SK + ak] = rb[e];
    }
  };

  f32x4 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  if (nk > 0) {
    gload(0);
    sstore(0);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1;
      if (kt + 1 < nk) gload(kt + 1);
      const float* as = As[cur];
      const float* bs = Bs[cur];
      // lane (c16, g4) supplies k = 4 g4 + s in MFMA step s: one 16-B read per block
      f32x4 av[MI], bv[NJ];
#pragma unroll
      for (int i = 0; i < MI; ++i)
        av[i] = *reinterpret_cast<const f32x4*>(as + (wm * (BM / 2) + i * 16 + c16) * SK + 4 * g4);
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        bv[j] = *reinterpret_cast<const f32x4*>(bs + (wn * (BN / 2) + j * 16 + c16) * SK + 4 * g4);
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i][s4], bv[j][s4], acc[i][j], 0, 0, 0);
      if (kt + 1 < nk) sstore(cur ^ 1);
      __syncthreads();
    }
  }

  // epilogue: lane holds rows 4 g4 + r of column c16 of each 16 x 16 block
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int ng = n0 + wn * (BN / 2) + j * 16 + c16;
    if (ng >= g.Ncol) continue;
    if (MODE == BWD_W) {
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int mg = m0 + wm * (BM / 2) + i * 16 + 4 * g4 + r;
          if (mg < g.M) out[((int64_t)blockIdx.z * g.M + mg) * g.Ncol + ng] = acc[i][j][r];
        }
    } else if (MODE == FWD) {
      const int HW = g.Ho * g.Wo;
      const int n = (int)g.dHoWo.div((unsigned)ng), q = ng - n * HW;
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int mg = m0 + wm * (BM / 2) + i * 16 + 4 * g4 + r;
          if (mg < g.M) out[((int64_t)n * g.M + mg) * HW + q] = acc[i][j][r] + (bias ? bias[mg] : 0.f);
        }
    } else {
      if (ng >= ph.Ncol) continue;
      const int64_t o0 = dx_offset(g, ph, ng, 0), cs = (int64_t)g.Hi * g.Wi;
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int mg = m0 + wm * (BM / 2) + i * 16 + 4 * g4 + r;
          if (mg < g.M) out[o0 + mg * cs] = acc[i][j][r];
        }
    }
  }
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
  g.dKHW = FastDiv::make((unsigned)(KH * KW));
  g.dKW = FastDiv::make((unsigned)KW);
  g.dHoWo = FastDiv::make((unsigned)(Ho * Wo));
  g.dWo = FastDiv::make((unsigned)Wo);
  g.dHiWi = FastDiv::make((unsigned)(Hi * Wi));
  g.dWi = FastDiv::make((unsigned)Wi);
  return true;
}

// 128 x 128 tiles where the GEMM has the rows and enough column tiles to fill the chip
// (two workgroups per CU); 64 x 64 otherwise.  BWD_W (split over K) only needs the extents.
#ifndef CONV_BIG_MIN_TILES
#define CONV_BIG_MIN_TILES 512
#endif
#ifndef CONV_BIG
#define CONV_BIG 1
#endif
bool big_tiles(int mode, int M, int Ncol) {
  if (!CONV_BIG || M < 128 || Ncol < 128) return false;
  return mode == BWD_W || (int64_t)cdiv(M, 128) * cdiv(Ncol, 128) >= CONV_BIG_MIN_TILES;
}

template <int MODE>
void launch_igemm(dim3 g3, int M, int Ncol, const float* pa, const float* pb, const float* bias,
                  float* out, const ConvArgs& g, hipStream_t st) {
  if (big_tiles(MODE, M, Ncol)) {
    g3.x = cdiv(Ncol, 128);
    g3.y = cdiv(M, 128);
    conv_igemm_kernel<MODE, 128, 128><<<g3, 256, 0, st>>>(pa, pb, bias, out, g);
  } else {
    g3.x = cdiv(Ncol, 64);
    g3.y = cdiv(M, 64);
    conv_igemm_kernel<MODE, 64, 64><<<g3, 256, 0, st>>>(pa, pb, bias, out, g);
  }
}

int wgrad_splits(const ConvArgs& g) {
  const int T = big_tiles(BWD_W, g.M, g.Ncol) ? 128 : 64;
  const int64_t tiles = (int64_t)cdiv(g.M, T) * cdiv(g.Ncol, T);
  const int64_t ksteps = cdiv(g.K, BK);
  int64_t s = cdiv(2048, tiles);                 // aim at >= 2048 workgroups
  const int64_t maxs = cdiv(ksteps, 8);          // but >= 8 K-steps per split
  if (s > maxs) s = maxs;
  if (s > 1024) s = 1024;
  return (int)(s < 1 ? 1 : s);
}

}  // namespace

BLINDNO_API int blindno_conv2d_fwd(const float* x, const float* w, const float* b, float* y, int N,
                                   int Ci, int Hi, int Wi, int Co, int KH, int KW, int sh, int sw,
                                   int ph, int pw, void* stream) {
  ConvArgs g;
  if (!x || !w || !y || !make_args(g, N, Ci, Hi, Wi, Co, KH, KW, sh, sw, ph, pw))
    return (int)hipErrorInvalidValue;
  g.M = Co;
  g.Ncol = N * g.Ho * g.Wo;
  g.K = Ci * KH * KW;
  launch_igemm<FWD>(dim3(1, 1, 1), g.M, g.Ncol, w, x, b, y, g, (hipStream_t)stream);
  return (int)hipGetLastError();
}

BLINDNO_API int blindno_conv2d_bwd_data(const float* dy, const float* w, float* dx, int N, int Ci,
                                        int Hi, int Wi, int Co, int KH, int KW, int sh, int sw,
                                        int ph, int pw, void* stream) {
  ConvArgs g;
  if (!dy || !w || !dx || sh * sw > kMaxPhases ||
      !make_args(g, N, Ci, Hi, Wi, Co, KH, KW, sh, sw, ph, pw))
    return (int)hipErrorInvalidValue;
  g.M = Ci;
  g.Ncol = N * Hi * Wi;
  g.K = Co * KH * KW;
  // stride-phase classes; pixels of a class whose taps are all off the kernel (nKh or nKw = 0)
  // receive no gradient, so they are zeroed first (only possible when the stride exceeds the
  // kernel extent)
  int maxcol = 1;
  bool uncovered = false;
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
      if (p.K == 0 && p.Ncol > 0) uncovered = true;
      if (p.K == 0) p.Ncol = 0;
      p.dHcWc = FastDiv::make((unsigned)(p.Hc * p.Wc > 0 ? p.Hc * p.Wc : 1));
      p.dWc = FastDiv::make((unsigned)(p.Wc > 0 ? p.Wc : 1));
      p.dKhw = FastDiv::make((unsigned)(p.nKh * p.nKw > 0 ? p.nKh * p.nKw : 1));
      p.dKw = FastDiv::make((unsigned)(p.nKw > 0 ? p.nKw : 1));
      if (p.Ncol > maxcol) maxcol = p.Ncol;
    }
  hipStream_t st = (hipStream_t)stream;
  if (uncovered) {
    const hipError_t e = hipMemsetAsync(dx, 0, sizeof(float) * (size_t)N * Ci * Hi * Wi, st);
    if (e != hipSuccess) return (int)e;
  }
  launch_igemm<BWD_D>(dim3(1, 1, sh * sw), g.M, maxcol, w, dy, nullptr, dx, g, st);
  return (int)hipGetLastError();
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
  launch_igemm<BWD_W>(dim3(1, 1, nz), g.M, g.Ncol, dy, x, nullptr, nz > 1 ? partial : dwb, g, st);
  if (nz > 1) {
    const int e = (int)hipGetLastError();
    if (e) return e;
    return blindno_reduce_partials(partial, dwb, nz, g.M * g.Ncol, stream);
  }
  return (int)hipGetLastError();
}
