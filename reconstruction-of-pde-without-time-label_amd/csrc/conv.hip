// 2D convolution (nn.Conv2d with bias, any kernel / stride / padding, groups 1) of the NIO
// snapshot encoders' ConvBlocks (2d_FPE/Baselines.py:40-52, Encoder2D :186-249, 1D Encoder
// :254-287), forward and both adjoints, as implicit GEMMs on the fp32 matrix cores
// (v_mfma_f32_16x16x4f32: exact fp32 products, fixed accumulation order -- deterministic).
//
//   FWD   y[n][co][p]   = b[co] + sum_{ci,kh,kw} W[co][ci][kh][kw] x[n][ci][tap(p,kh,kw)]
//         GEMM  M = Co, N = pixels (n, ho, wo), K = Ci KH KW
//   BWD_D dx[n][ci][q]  = sum_{co,kh,kw} W[co][ci][kh][kw] dy[n][co][(q + pad - k) / stride]
//         GEMM  M = Ci, N = input pixels (n, hi, wi), K = Co KH KW (taps that do not land on
//         an output pixel -- off the grid or off the stride lattice -- contribute 0)
//   BWD_W dW[co][ci][kh][kw] = sum_{n,p} dy[n][co][p] x[n][ci][tap(p,kh,kw)],  db[co] = sum dy
//         GEMM  M = Co, N = Ci KH KW + 1 (the extra column is the bias: B = 1), K = pixels,
//         split over blockIdx.z into fixed K ranges; the partials are reduced in a fixed order
//         afterwards (blindno_reduce_partials).
//
// Tiling for CDNA4 wave64: a 256-thread workgroup computes a 64 x 64 tile as 2 x 2 waves of
// 32 x 32 (2 x 2 MFMA blocks each, 4 accumulator VGPRs per block), K in steps of 16 staged
// through double-buffered LDS (k-major, rows padded by 16 floats: the four k-groups of a wave's
// operand read land in disjoint banks).  The next step's global loads are issued before the
// current step's MFMAs, so their latency hides behind 16 MFMAs per wave.  im2col is never
// materialised: each loader lane decodes its (channel, tap) / pixel indices with
// multiply-high divisions by the launch's constants (FastDiv).
#include "common.h"
#include "blindno.h"

using namespace blindno;

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int BM = 64, BN = 64, BK = 16;
constexpr int SA = BM + 16, SB = BN + 16;      // LDS row strides (floats)

enum { FWD = 0, BWD_D = 1, BWD_W = 2 };

struct ConvArgs {
  int N, Ci, Hi, Wi, Co, Ho, Wo, KH, KW, sh, sw, ph, pw;
  int M, Ncol, K;               // GEMM sizes of this mode
  int kchunk;                   // BWD_W: K per split (multiple of BK)
  FastDiv dKHW, dKW, dHoWo, dWo, dHiWi, dWi;
};

// ---- A operand (BM x BK tile), element (m, k) of global (m0 + m, k0 + k)
template <int MODE>
__device__ __forceinline__ float load_a(const float* __restrict__ pa, const ConvArgs& g, int mg,
                                        int kg, int kend) {
  if (mg >= g.M || kg >= kend) return 0.f;
  const int KHW = g.KH * g.KW;
  if (MODE == FWD) return pa[(int64_t)mg * g.K + kg];                       // W[co][k]
  if (MODE == BWD_D) {                                                         // W[co][ci][khw]
    const int co = (int)g.dKHW.div((unsigned)kg), khw = kg - co * KHW;
    return pa[((int64_t)co * g.Ci + mg) * KHW + khw];
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
__device__ __forceinline__ Pix decode_pix(const ConvArgs& g, int ng) {
  Pix p;
  p.ok = ng < g.Ncol;
  const int v = p.ok ? ng : 0;
  if (MODE == FWD) {
    const int HoWo = g.Ho * g.Wo;
    const int n = (int)g.dHoWo.div((unsigned)v), q = v - n * HoWo;
    const int ho = (int)g.dWo.div((unsigned)q), wo = q - ho * g.Wo;
    p.base = (int64_t)n * g.Ci * g.Hi * g.Wi;
    p.r = ho * g.sh - g.ph;
    p.c = wo * g.sw - g.pw;
  } else {
    const int HiWi = g.Hi * g.Wi;
    const int n = (int)g.dHiWi.div((unsigned)v), q = v - n * HiWi;
    const int hi = (int)g.dWi.div((unsigned)q), wi = q - hi * g.Wi;
    p.base = (int64_t)n * g.Co * g.Ho * g.Wo;
    p.r = hi + g.ph;
    p.c = wi + g.pw;
  }
  return p;
}

// B element (k, pixel) for FWD / BWD_D
template <int MODE>
__device__ __forceinline__ float load_b_pix(const float* __restrict__ pb, const ConvArgs& g,
                                            const Pix& p, int kg) {
  if (!p.ok || kg >= g.K) return 0.f;
  const int KHW = g.KH * g.KW;
  const int ch = (int)g.dKHW.div((unsigned)kg), khw = kg - ch * KHW;
  const int kh = (int)g.dKW.div((unsigned)khw), kw = khw - kh * g.KW;
  if (MODE == FWD) {
    const int hi = p.r + kh, wi = p.c + kw;
    if ((unsigned)hi >= (unsigned)g.Hi || (unsigned)wi >= (unsigned)g.Wi) return 0.f;
    return pb[p.base + ((int64_t)ch * g.Hi + hi) * g.Wi + wi];
  }
  int th = p.r - kh, tw = p.c - kw;                    // = ho sh, wo sw when on the lattice
  if (th < 0 || tw < 0) return 0.f;
  int ho = th, wo = tw;
  if (g.sh != 1) {
    ho = th / g.sh;
    if (ho * g.sh != th) return 0.f;
  }
  if (g.sw != 1) {
    wo = tw / g.sw;
    if (wo * g.sw != tw) return 0.f;
  }
  if (ho >= g.Ho || wo >= g.Wo) return 0.f;
  return pb[p.base + ((int64_t)ch * g.Ho + ho) * g.Wo + wo];
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

template <int MODE>
__global__ __launch_bounds__(256) void conv_igemm_kernel(const float* __restrict__ pa,
                                                         const float* __restrict__ pb,
                                                         const float* __restrict__ bias,
                                                         float* __restrict__ out, ConvArgs g) {
  __shared__ float As[2][BK * SA];
  __shared__ float Bs[2][BK * SB];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = uniform_int(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int c16 = lane & 15, g4 = lane >> 4;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  int kbeg = 0, kend = g.K;
  if (MODE == BWD_W) {
    kbeg = blockIdx.z * g.kchunk;
    kend = min(g.K, kbeg + g.kchunk);
  }
  const int nk = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;

  // loader roles.  A: k = tid % 16 (contiguous in memory for all modes), m = tid / 16 + 16 e.
  const int ak = tid & 15, am = tid >> 4;
  // B (FWD / BWD_D): pixel n = tid % 64 fixed for the tile, k = tid / 64 + 4 e.
  // B (BWD_W): pixel k = tid % 16, column n = tid / 16 + 16 e (fixed taps for the tile).
  const int bn = tid & 63, bk = tid >> 6;
  Pix pix{};
  Tap taps[4];
  if (MODE != BWD_W) {
    pix = decode_pix<MODE>(g, n0 + bn);
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e) taps[e] = decode_tap(g, n0 + (tid >> 4) + 16 * e);
  }

  float ra[4], rb[4];
  auto gload = [&](int kt) {
    const int k0 = kbeg + kt * BK;
#pragma unroll
    for (int e = 0; e < 4; ++e) ra[e] = load_a<MODE>(pa, g, m0 + am + 16 * e, k0 + ak, kend);
    if (MODE != BWD_W) {
#pragma unroll
      for (int e = 0; e < 4; ++e) rb[e] = load_b_pix<MODE>(pb, g, pix, k0 + bk + 4 * e);
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
      for (int e = 0; e < 4; ++e) {
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
    for (int e = 0; e < 4; ++e) As[buf][ak * SA + am + 16 * e] = ra[e];
    if (MODE != BWD_W) {
#pragma unroll
      for (int e = 0; e < 4; ++e) Bs[buf][(bk + 4 * e) * SB + bn] = rb[e];
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) Bs[buf][ak * SB + (tid >> 4) + 16 * e] = rb[e];
    }
  };

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  if (nk > 0) {
    gload(0);
    sstore(0);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1;
      if (kt + 1 < nk) gload(kt + 1);
      const float* as = As[cur];
      const float* bs = Bs[cur];
#pragma unroll
      for (int kk = 0; kk < BK / 4; ++kk) {
        const int kr = 4 * kk + g4;
        float av[2], bv[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) av[i] = as[kr * SA + wm * 32 + i * 16 + c16];
#pragma unroll
        for (int j = 0; j < 2; ++j) bv[j] = bs[kr * SB + wn * 32 + j * 16 + c16];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i], bv[j], acc[i][j], 0, 0, 0);
      }
      if (kt + 1 < nk) sstore(cur ^ 1);
      __syncthreads();
    }
  }

  // epilogue: lane holds rows 4 g4 + r of column c16 of each 16 x 16 block
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int ng = n0 + wn * 32 + j * 16 + c16;
    if (ng >= g.Ncol) continue;
    if (MODE == BWD_W) {
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int mg = m0 + wm * 32 + i * 16 + 4 * g4 + r;
          if (mg < g.M) out[((int64_t)blockIdx.z * g.M + mg) * g.Ncol + ng] = acc[i][j][r];
        }
    } else {
      const int HW = MODE == FWD ? g.Ho * g.Wo : g.Hi * g.Wi;
      const int n = (int)(MODE == FWD ? g.dHoWo : g.dHiWi).div((unsigned)ng), q = ng - n * HW;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int mg = m0 + wm * 32 + i * 16 + 4 * g4 + r;
          if (mg < g.M) {
            float v = acc[i][j][r];
            if (MODE == FWD && bias) v += bias[mg];
            out[((int64_t)n * g.M + mg) * HW + q] = v;
          }
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

int wgrad_splits(const ConvArgs& g) {
  const int64_t tiles = (int64_t)cdiv(g.M, BM) * cdiv(g.Ncol, BN);
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
  const dim3 grid(cdiv(g.Ncol, BN), cdiv(g.M, BM), 1);
  conv_igemm_kernel<FWD><<<grid, 256, 0, (hipStream_t)stream>>>(w, x, b, y, g);
  return (int)hipGetLastError();
}

BLINDNO_API int blindno_conv2d_bwd_data(const float* dy, const float* w, float* dx, int N, int Ci,
                                        int Hi, int Wi, int Co, int KH, int KW, int sh, int sw,
                                        int ph, int pw, void* stream) {
  ConvArgs g;
  if (!dy || !w || !dx || !make_args(g, N, Ci, Hi, Wi, Co, KH, KW, sh, sw, ph, pw))
    return (int)hipErrorInvalidValue;
  g.M = Ci;
  g.Ncol = N * Hi * Wi;
  g.K = Co * KH * KW;
  const dim3 grid(cdiv(g.Ncol, BN), cdiv(g.M, BM), 1);
  conv_igemm_kernel<BWD_D><<<grid, 256, 0, (hipStream_t)stream>>>(w, dy, nullptr, dx, g);
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
  const dim3 grid(cdiv(g.Ncol, BN), cdiv(g.M, BM), nz);
  hipStream_t st = (hipStream_t)stream;
  conv_igemm_kernel<BWD_W><<<grid, 256, 0, st>>>(dy, x, nullptr, nz > 1 ? partial : dwb, g);
  if (nz > 1) {
    const int e = (int)hipGetLastError();
    if (e) return e;
    return blindno_reduce_partials(partial, dwb, nz, g.M * g.Ncol, stream);
  }
  return (int)hipGetLastError();
}
