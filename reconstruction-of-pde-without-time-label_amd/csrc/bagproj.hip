// Bag-level projection of the snapshot encoder: the FNO_input projection (crop -> fc1 -> GELU
// -> fc2, 2d_FPE/FNOModules.py:234-239) of every snapshot of a bag fused with the fixed-weight
// bag mean that consumes it (2d_FPE/NIOModules.py:569-575), with the backward reduced to
// bag-level sufficient statistics.
//
// The bag mean hands every snapshot l of bag b the same upstream gradient up to its weight:
// dy[l, p] = lw_l ghat[b, p] (ghat = W'[:, 2] . dL/dh[b, p], lw_l = multiplicity / L).  With
// h = W1 z + b1 per snapshot point, a = GELU(h) and g = GELU'(h), every parameter gradient is
// therefore a ghat-weighted sum of per-(bag, point) statistics that the forward forms while h
// is in registers:
//     A[k] = sum_l lw_l a_k,   S[k] = sum_l lw_l g_k,   Q[k][c] = sum_l lw_l g_k z_c,
//     dW2 = sum_bp ghat A,  db1 = w2 * sum_bp ghat S,  dW1 = w2 * sum_bp ghat Q,
//     db2 = sum_bp ghat * sum_l lw_l,
// and the input gradient is dz[l, p, c] = lw_l ghat[b, p] v[l, p, c] with v = W1^T (w2 * g).
// The forward's output is the bag mean of the projections itself,
//     ubar[b, p] = sum_l lw_l (w2 . a_l + b2) = w2 . A + b2 sum_l lw_l,
// so no per-snapshot output is written, and the backward reads 3 KB of statistics per (bag,
// point) instead of recomputing fc1, GELU and GELU' for every snapshot point.
//
// Forward layout ("hidden x points", one v_mfma_f32_16x16x4f32 per 16 x 16 tile, K = C <= 4):
//     H (16 hid x 16 pts) = W1 (16 hid x C) . Z (C x 16 pts)
// lane l holds h for hidden units 4 (l >> 4) + r (r < 4) and point l & 15, so the lane's Q
// update needs only its own point's C channels and v reduces over the 4 lane groups (a
// reduce-scatter of 3 lane swaps) instead of over 16 lanes.  A workgroup owns a 16-point tile;
// its 4 waves split the 128 hidden units (2 tiles each, weights in registers) and walk the
// bag's snapshots in double-buffered chunks staged through LDS, where the waves' v partials are
// also summed.
#include "common.h"
#include "blindno.h"
#include "gelu_pk.h"

using namespace blindno;
using namespace blindno::gelu_pk;

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kHd = 128;            // fc1 = Linear(width, 128)
constexpr int kNStat = 6;           // A, S, Q_0..Q_3
constexpr int kTileF4 = (kHd / 16) * kNStat * 64;   // float4 slots per 16-point tile: 3072
constexpr int kMaxU = 1024;
#ifndef BAGPROJ_QUAD
#define BAGPROJ_QUAD 1
#endif
#ifndef BAGPROJ_FWD_WAVES
#define BAGPROJ_FWD_WAVES 3
#endif
// 1: the workgroup set-up off the critical path -- the first tile's first z chunk is loaded
// before the weights, and sum_l lw_l is accumulated in the snapshot loop (same order) instead
// of a U-step LDS chain of its own (per-wave phase stamps, tools/probe_bagproj.py: the set-up
// took ~13 us of a one-tile workgroup's ~70 us)
#ifndef BAGPROJ_SETUP2
#define BAGPROJ_SETUP2 1
#endif

// point f of the flattened (bag, crop point) space -> offset of (bag b, snapshot 0, channel 0,
// row h, column w) in z (B U, C, P1, P2); 32-bit (the launchers bound the field below 2^31)
struct BagGeom {
  unsigned npts, S, Wo, P2, HW, C, U;
  FastDiv dS, dWo;
  __device__ __forceinline__ unsigned base(unsigned f) const {
    const unsigned b = dS.div(f), s = f - b * S;
    const unsigned h = dWo.div(s), w = s - h * Wo;
    return b * U * C * HW + h * P2 + w;
  }
};

// The forward.  Per (snapshot, point, hidden unit) the GELU / GELU' and statistics arithmetic;
// around it (round 4; round 3's kernel: 340 -> 328 us at config C):
//   * v's reduce-scatter over the 4 lane groups with v_permlane32_swap / v_permlane16_swap (3
//     swaps + 3 adds, no LDS round trip, no lane-index arithmetic) instead of ds_bpermute;
//   * v's 1/2 sum_k (w2 W1)[k] part added once at the store (the accumulation starts with a
//     multiply), zbar summed by the staging threads, w2 re-read at the statistics write:
//     no per-snapshot register moves and 20 fewer live VGPRs;
//   * double-buffered 8-snapshot chunks: one barrier per chunk instead of three per 16.
// statistics tiles of a backward step whose loads the compiler may overlap (1: one tile's 12
// float4 at a time)
#ifndef BAGPROJ_BWD_UNROLL
#define BAGPROJ_BWD_UNROLL 1
#endif
#ifndef BAGPROJ_SC
#define BAGPROJ_SC 8
#endif
constexpr int kSC2 = BAGPROJ_SC;        // snapshots per staged chunk (a multiple of 4)

__device__ __forceinline__ float swap_sum32(float a, float b) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

__device__ __forceinline__ float swap_sum16(float a, float b) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(b), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

#ifndef BAGPROJ_PROBE
#define BAGPROJ_PROBE 0
#endif
#if BAGPROJ_PROBE
// diagnostic build only (tools/probe_bagproj.py): per-wave realtime stamps at the phase edges
__device__ unsigned long long g_bagproj_probe[32768 * 8];
#define BP_MARK(i)                                                                          \
  do {                                                                                      \
    __builtin_amdgcn_sched_barrier(0);                                                      \
    const unsigned long long t_ = __builtin_amdgcn_s_memrealtime();                         \
    const int slot_ = blockIdx.x * 4 + (threadIdx.x >> 6);                                  \
    if ((threadIdx.x & 63) == 0 && slot_ < 32768) g_bagproj_probe[slot_ * 8 + (i)] = t_;    \
    __builtin_amdgcn_sched_barrier(0);                                                      \
  } while (0)
#else
#define BP_MARK(i) do {} while (0)
#endif
__global__ __launch_bounds__(256, BAGPROJ_FWD_WAVES) void bagproj_fwd_kernel(
    const float* __restrict__ z, const float* __restrict__ w1, const float* __restrict__ b1,
    const float* __restrict__ w2, const float* __restrict__ b2, const float* __restrict__ lw,
    float* __restrict__ ubar, float* __restrict__ stats, float* __restrict__ v, BagGeom g) {
  __shared__ float slw[kMaxU];
  __shared__ float zs[2][kSC2][16][4];        // [buffer][snapshot][point][channel]
  __shared__ float zw[2][kSC2][16][4];        // the same times lw_l (Q's operand)
  __shared__ float vred[2][4][kSC2][64];      // [buffer][wave][snapshot][16 channel + point]
  __shared__ float zbr[4][64];                // zbar partials [ls][16 cs + point]
  __shared__ float vpart[16][4];              // per (wave, g4): 1/2 sum over its 8 hidden of (w2 W1)[k][c]
  __shared__ float vhalf[4];                  // 1/2 sum_k (w2 W1)[k][c]
  __shared__ float ured[4][16];
  __shared__ float2 swr[4][4][2][2][4];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = uniform_int(tid >> 6);
  const int c16 = lane & 15, g4 = lane >> 4;
  const int C = (int)g.C, U = (int)g.U;
  BP_MARK(0);
  // staging / v-output role of this thread: point tid & 15 (= the compute lane's c16),
  // channel (tid >> 4) & 3, snapshots (tid >> 6) + 4 i of each chunk
  const int cs = (tid >> 4) & 3, ls = tid >> 6;
  const unsigned ntiles = (g.npts + 15) / 16;
  auto zload = [&](unsigned bo, bool ok, int ch, float (&zr)[kSC2 / 4]) {
#pragma unroll
    for (int i = 0; i < kSC2 / 4; ++i) {
      const int lg = ch * kSC2 + ls + 4 * i;
#if BAGPROJ_SETUP2
      // unconditional loads from clamped offsets (bo is a valid point), then a select: a
      // guarded load is a branch the compiler will not hoist the load out of
      const int lc = lg < U ? lg : U - 1, cc = cs < C ? cs : C - 1;
      const float zv = z[bo + (unsigned)(lc * C + cc) * g.HW];
      zr[i] = (ok && lg < U && cs < C) ? zv : 0.f;
#else
      zr[i] = (ok && lg < U && cs < C) ? z[bo + (unsigned)(lg * C + cs) * g.HW] : 0.f;
#endif
    }
  };
  float wa[2], bb[2][4], vloc[4] = {0.f, 0.f, 0.f, 0.f};
#if BAGPROJ_SETUP2
  // the weights staged through LDS by coalesced loads (one round trip) before the per-lane
  // set-up reads them: as global loads inside per-channel branches, each (w2[k], w1[k][c])
  // pair was its own L2 round trip.  Their loads go out before the first z chunk's, so that
  // the LDS stores wait for them alone (vector-memory counts retire in order)
  __shared__ float sw1[kHd * 4], sb1[kHd], sw2[kHd];
  constexpr int kLwIt = kMaxU / 256;
  float lwv[kLwIt], w1v[2], b1v = 0.f, w2v = 0.f;
#pragma unroll
  for (int i = 0; i < kLwIt; ++i) {
    const int l = tid + 256 * i;
    lwv[i] = l < U ? (lw ? lw[l] : 1.0f / (float)U) : 0.f;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) w1v[i] = tid + 256 * i < kHd * C ? w1[tid + 256 * i] : 0.f;
  if (tid < kHd) {
    b1v = b1[tid];
    w2v = w2[tid];
  }
  float zfirst[kSC2 / 4];
  {
    const unsigned f = blockIdx.x * 16 + (unsigned)c16;
    const bool ok = f < g.npts;
    zload(g.base(ok ? f : 0u), ok, 0, zfirst);
  }
#pragma unroll
  for (int i = 0; i < kLwIt; ++i)
    if (tid + 256 * i < U) slw[tid + 256 * i] = lwv[i];
#pragma unroll
  for (int i = 0; i < 2; ++i)
    if (tid + 256 * i < kHd * C) sw1[tid + 256 * i] = w1v[i];
  if (tid < kHd) {
    sb1[tid] = b1v;
    sw2[tid] = w2v;
  }
  __syncthreads();
#pragma unroll
  for (int tt = 0; tt < 2; ++tt) {
    const int k0 = 16 * (2 * wave + tt);
    wa[tt] = g4 < C ? kK * sw1[(k0 + c16) * C + g4] : 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int k = k0 + 4 * g4 + r;
      bb[tt][r] = kK * sb1[k];
      if (c16 == 0) {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const float wrv = c < C ? sw2[k] * sw1[k * C + c] : 0.f;
          vloc[c] += wrv;
          float2& e = swr[wave][g4][tt][r >> 1][c];
          if (r & 1) e.y = wrv; else e.x = wrv;
        }
      }
    }
  }
#else
  float zfirst[kSC2 / 4];
  for (int l = tid; l < U; l += 256) slw[l] = lw ? lw[l] : 1.0f / (float)U;
#pragma unroll
  for (int tt = 0; tt < 2; ++tt) {
    const int k0 = 16 * (2 * wave + tt);
    wa[tt] = g4 < C ? kK * w1[(k0 + c16) * C + g4] : 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int k = k0 + 4 * g4 + r;
      bb[tt][r] = kK * b1[k];
      if (c16 == 0) {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const float wrv = c < C ? w2[k] * w1[k * C + c] : 0.f;
          vloc[c] += wrv;
          float2& e = swr[wave][g4][tt][r >> 1][c];
          if (r & 1) e.y = wrv; else e.x = wrv;
        }
      }
    }
  }
#endif
  if (c16 == 0) {
#pragma unroll
    for (int c = 0; c < 4; ++c) vpart[4 * wave + g4][c] = 0.5f * vloc[c];
  }
  __syncthreads();
  if (tid < 4) {
    float acc = 0.f;
    for (int j = 0; j < 16; ++j) acc += vpart[j][tid];
    vhalf[tid] = acc;                          // read after the first chunk's barrier
  }
#if !BAGPROJ_SETUP2
  float lsum = 0.f;                            // sum_l lw_l, same order in every thread
  for (int l = 0; l < U; ++l) lsum += slw[l];
  const float b2l = b2[0] * lsum;
#endif
  BP_MARK(1);

  const int nch = (U + kSC2 - 1) / kSC2;
  for (unsigned tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const unsigned f = tile * 16 + (unsigned)c16;
    const bool ok = f < g.npts;
    const unsigned bo = g.base(ok ? f : 0u);
    float zbp = 0.f;                           // sum over this thread's staged snapshots of lw z
    // staging is split so that the next chunk's global loads are in flight during this
    // chunk's compute: load() into registers, store() into the LDS buffer after the compute
    float zn[kSC2 / 4];
    auto load = [&](int ch) { zload(bo, ok, ch, zn); };
    auto store = [&](int ch, int buf) {
#pragma unroll
      for (int i = 0; i < kSC2 / 4; ++i) {
        const int l = ls + 4 * i, lg = ch * kSC2 + l;
        const float wv = zn[i] * slw[lg < U ? lg : 0];
        zs[buf][l][c16][cs] = zn[i];
        zw[buf][l][c16][cs] = wv;
        zbp += wv;
      }
    };
    auto vwrite = [&](int ch, int buf) {
#pragma unroll
      for (int i = 0; i < kSC2 / 4; ++i) {
        const int l = ls + 4 * i, lg = ch * kSC2 + l;
        if (ok && lg < U && cs < C)
          v[bo + (unsigned)(lg * C + cs) * g.HW] =
              (((vred[buf][0][l][lane] + vred[buf][1][l][lane]) + vred[buf][2][l][lane]) +
               vred[buf][3][l][lane]) + vhalf[cs];
      }
    };
    f32x2 A[2][2], S[2][2], Q[2][4][2];
#pragma unroll
    for (int tt = 0; tt < 2; ++tt)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        A[tt][i] = S[tt][i] = (f32x2){0.f, 0.f};
#pragma unroll
        for (int c = 0; c < 4; ++c) Q[tt][c][i] = (f32x2){0.f, 0.f};
      }
    if (BAGPROJ_SETUP2 && tile == blockIdx.x) {
#pragma unroll
      for (int i = 0; i < kSC2 / 4; ++i) zn[i] = zfirst[i];
    } else {
      load(0);
    }
    store(0, 0);
    if (nch > 1) load(1);
#if BAGPROJ_SETUP2
    float lsum = 0.f;                          // sum_l lw_l in l order, as the stand-alone loop
#endif
    __syncthreads();
    BP_MARK(2);
    for (int ch = 0; ch < nch; ++ch) {
      const int buf = ch & 1, l0 = ch * kSC2;
      const int nl = U - l0 < kSC2 ? U - l0 : kSC2;
      for (int l = 0; l < nl; ++l) {
        int zo;                                // opaque zero: keeps the swr reads in the loop
        asm volatile("v_mov_b32 %0, 0" : "=v"(zo));
        const float4 zc = *reinterpret_cast<const float4*>(&zw[buf][l][c16][0]);
        const float az = zs[buf][l][c16][g4];
        const float lwl = slw[l0 + l];
        const f32x2 wl = splat2(lwl);
#if BAGPROJ_SETUP2
        lsum += lwl;
#endif
        f32x2 vp[4];
#if BAGPROJ_QUAD
        // both tiles' pre-activations first, then the four pairs' GELU / GELU' in lockstep
        f32x2 hq[4], sq[4], eq[4];
#pragma unroll
        for (int tt = 0; tt < 2; ++tt) {
          f32x4 d = {bb[tt][0], bb[tt][1], bb[tt][2], bb[tt][3]};
          d = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[tt], az, d, 0, 0, 0);
          hq[2 * tt] = (f32x2){d[0], d[1]};
          hq[2 * tt + 1] = (f32x2){d[2], d[3]};
        }
        norm_cdf_quad_pdf_centered(hq, sq, eq);
#endif
#pragma unroll
        for (int tt = 0; tt < 2; ++tt) {
#if !BAGPROJ_QUAD
          f32x4 d = {bb[tt][0], bb[tt][1], bb[tt][2], bb[tt][3]};
          d = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[tt], az, d, 0, 0, 0);
          const f32x2 h[2] = {{d[0], d[1]}, {d[2], d[3]}};
#else
          const f32x2 h[2] = {hq[2 * tt], hq[2 * tt + 1]};
#endif
#pragma unroll
          for (int i = 0; i < 2; ++i) {
#if BAGPROJ_QUAD
            const f32x2 ep = eq[2 * tt + i], sg = sq[2 * tt + i];
#else
            f32x2 ep;
            const f32x2 sg = norm_cdf_pair_pdf_centered(h[i], ep);   // Phi - 1/2
#endif
            const f32x2 gd = pk_fma(h[i], ep, sg);                  // GELU' - 1/2
            A[tt][i] = pk_fma(wl, h[i] * sg, A[tt][i]);             // lw k h (Phi - 1/2)
            S[tt][i] = pk_fma(wl, gd, S[tt][i]);
            Q[tt][0][i] = pk_fma(gd, splat2(zc.x), Q[tt][0][i]);
            Q[tt][1][i] = pk_fma(gd, splat2(zc.y), Q[tt][1][i]);
            Q[tt][2][i] = pk_fma(gd, splat2(zc.z), Q[tt][2][i]);
            Q[tt][3][i] = pk_fma(gd, splat2(zc.w), Q[tt][3][i]);
            const float4* wq = reinterpret_cast<const float4*>(&swr[wave][g4][tt][i][0]) + zo;
            const float4 wq0 = wq[0], wq1 = wq[1];
            const f32x2 q0 = {wq0.x, wq0.y}, q1 = {wq0.z, wq0.w}, q2 = {wq1.x, wq1.y}, q3 = {wq1.z, wq1.w};
            if (tt == 0 && i == 0) {
              vp[0] = gd * q0; vp[1] = gd * q1; vp[2] = gd * q2; vp[3] = gd * q3;
            } else {
              vp[0] = pk_fma(gd, q0, vp[0]);
              vp[1] = pk_fma(gd, q1, vp[1]);
              vp[2] = pk_fma(gd, q2, vp[2]);
              vp[3] = pk_fma(gd, q3, vp[3]);
            }
          }
        }
        // v over this wave's 32 hidden units, reduce-scattered over the 4 lane groups: lanes
        // 0-31 / 32-63 first (channels 0, 1 / 2, 3), then the 16-lane rows, so that group g4
        // keeps channel g4 of point c16
        const float a = swap_sum32(vp[0].x + vp[0].y, vp[2].x + vp[2].y);
        const float b = swap_sum32(vp[1].x + vp[1].y, vp[3].x + vp[3].y);
        vred[buf][wave][l][lane] = swap_sum16(a, b);
      }
      if (ch + 1 < nch) {
        store(ch + 1, buf ^ 1);                // its loads were issued one chunk ago
        if (ch + 2 < nch) load(ch + 2);
      }
      if (ch >= 1) vwrite(ch - 1, buf ^ 1);
      __syncthreads();
    }
    vwrite(nch - 1, (nch - 1) & 1);
#if BAGPROJ_SETUP2
    const float b2l = b2[0] * lsum;
#endif
    zbr[ls][lane] = zbp;
    BP_MARK(3);
    __syncthreads();
    // statistics of this tile: slot ((t 6 + comp) 64 + lane) holds hidden 16 t + 4 g4 + r
    // (r = the float4 component) of point c16
    float4* st = reinterpret_cast<float4*>(stats) + (size_t)tile * kTileF4 + lane;
    float zb[4];
#pragma unroll
    for (int c = 0; c < 4; ++c)
      zb[c] = ((zbr[0][16 * c + c16] + zbr[1][16 * c + c16]) + zbr[2][16 * c + c16]) + zbr[3][16 * c + c16];
    float up = 0.f;
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
      const int t = 2 * wave + tt;
      float av[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int k = 16 * t + 4 * g4 + r;
#if BAGPROJ_SETUP2
        float hb = sb1[k] * lsum;
#pragma unroll
        for (int c = 0; c < 4; ++c) hb = c < C ? fmaf(sw1[k * C + c], zb[c], hb) : hb;
#else
        float hb = b1[k] * lsum;
#pragma unroll
        for (int c = 0; c < 4; ++c) hb = c < C ? fmaf(w1[k * C + c], zb[c], hb) : hb;
#endif
        const float acc = r == 0 ? A[tt][0].x : (r == 1 ? A[tt][0].y : (r == 2 ? A[tt][1].x : A[tt][1].y));
        av[r] = fmaf(kInvK, acc, 0.5f * hb);
      }
      const float4 a4 = {av[0], av[1], av[2], av[3]};
      const int kb = 16 * t + 4 * g4;
#if BAGPROJ_SETUP2
      up += (sw2[kb] * a4.x + sw2[kb + 1] * a4.y) + (sw2[kb + 2] * a4.z + sw2[kb + 3] * a4.w);
#else
      up += (w2[kb] * a4.x + w2[kb + 1] * a4.y) + (w2[kb + 2] * a4.z + w2[kb + 3] * a4.w);
#endif
      st[(t * kNStat + 0) * 64] = a4;
      const float hs = 0.5f * lsum;
      st[(t * kNStat + 1) * 64] = (float4){S[tt][0].x + hs, S[tt][0].y + hs, S[tt][1].x + hs, S[tt][1].y + hs};
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const float hz = 0.5f * zb[c];
        st[(t * kNStat + 2 + c) * 64] =
            (float4){Q[tt][c][0].x + hz, Q[tt][c][0].y + hz, Q[tt][c][1].x + hz, Q[tt][c][1].y + hz};
      }
    }
    up += __shfl_xor(up, 16, 64);
    up += __shfl_xor(up, 32, 64);
    if (g4 == 0) ured[wave][c16] = up;
    __syncthreads();
    if (tid < 16 && ok) ubar[f] = (((ured[0][tid] + ured[1][tid]) + ured[2][tid]) + ured[3][tid]) + b2l;
  }
  BP_MARK(4);
#if BAGPROJ_PROBE
  if ((threadIdx.x & 63) == 0) {
    const int slot_ = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (slot_ < 32768) {
      g_bagproj_probe[slot_ * 8 + 5] = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_ID
      g_bagproj_probe[slot_ * 8 + 6] = __builtin_amdgcn_s_getreg((31 << 11) | 20);   // XCC_ID
    }
  }
#endif
}
#if BAGPROJ_PROBE
BLINDNO_API int blindno_bagproj_probe_read(unsigned long long* dst, int n) {
  return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_bagproj_probe),
                                  sizeof(unsigned long long) * (size_t)n, 0, hipMemcpyDeviceToHost);
}
#endif

// Backward: ghat-weighted reduction of the statistics (thread tid owns float4 slots tid + 256 j
// of every tile, all of point tid & 15) into one partial per workgroup
//     [dW1 (Hd C) | db1 (Hd) | dW2 (Hd) | db2]
// and dz = lw_l ghat v on the crop.
__global__ __launch_bounds__(256) void bagproj_bwd_kernel(
    const float* __restrict__ stats, const float* __restrict__ gs, const float* __restrict__ w2,
    const float* __restrict__ lw, const float* __restrict__ v, float* __restrict__ dz,
    float* __restrict__ partial, BagGeom g) {
  constexpr int kJ = kTileF4 / 256;          // 12 slots per thread
  __shared__ float slw[kMaxU];
  __shared__ float4 red[kJ * 4][4];          // [t 6 + comp][g4] -> r
  __shared__ float sgs;
  const int tid = threadIdx.x, lane = tid & 63, c16 = lane & 15;
  const int C = (int)g.C, U = (int)g.U;
  for (int l = tid; l < U; l += 256) slw[l] = lw ? lw[l] : 1.0f / (float)U;
  __syncthreads();
  float4 acc[kJ];
#pragma unroll
  for (int j = 0; j < kJ; ++j) acc[j] = (float4){0.f, 0.f, 0.f, 0.f};
  float gsum = 0.f;
  // four consecutive 16-point tiles per step: the dz = lw ghat v stream then covers 64
  // consecutive points per wave instruction (256-B runs of one channel plane; a 16-point tile
  // gave 64-B runs), wave w taking channel w over every snapshot
  const int cw = tid >> 6, p64 = tid & 63;
  const unsigned ntiles = (g.npts + 15) / 16;
  const unsigned ntg = (ntiles + 3) / 4;
  for (unsigned tg = blockIdx.x; tg < ntg; tg += gridDim.x) {
    if (dz) {
      // (dz NULL: the consumers form dz = lw ghat v on load, csrc/colspec.h BagDz)
      const unsigned f = tg * 64 + (unsigned)p64;
      if (f < g.npts && cw < C) {
        const float gh = gs[f];
        const unsigned bo = g.base(f) + (unsigned)cw * g.HW;
        const unsigned ls = (unsigned)C * g.HW;
        int l = 0;
        for (; l + 3 < U; l += 4) {                 // four loads in flight per thread
          float vv[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) vv[i] = v[bo + (unsigned)(l + i) * ls];
#pragma unroll
          for (int i = 0; i < 4; ++i) dz[bo + (unsigned)(l + i) * ls] = slw[l + i] * gh * vv[i];
        }
        for (; l < U; ++l) dz[bo + (unsigned)l * ls] = slw[l] * gh * v[bo + (unsigned)l * ls];
      }
    }
#pragma unroll BAGPROJ_BWD_UNROLL
    for (int t4 = 0; t4 < 4; ++t4) {
      const unsigned tile = tg * 4 + (unsigned)t4;
      if (tile >= ntiles) break;
      const unsigned f = tile * 16 + (unsigned)c16;
      const float gh = f < g.npts ? gs[f] : 0.f;
      const float4* st = reinterpret_cast<const float4*>(stats) + (size_t)tile * kTileF4 + tid;
      float4 sv[kJ];
#pragma unroll
      for (int j = 0; j < kJ; ++j) sv[j] = st[256 * j];
      if (tid < 16) gsum += gh;
#pragma unroll
      for (int j = 0; j < kJ; ++j) {
        acc[j].x = fmaf(gh, sv[j].x, acc[j].x);
        acc[j].y = fmaf(gh, sv[j].y, acc[j].y);
        acc[j].z = fmaf(gh, sv[j].z, acc[j].z);
        acc[j].w = fmaf(gh, sv[j].w, acc[j].w);
      }
    }
  }
  // sum over the 16 points (lanes c16) in a fixed butterfly order
#pragma unroll
  for (int j = 0; j < kJ; ++j) {
#pragma unroll
    for (int m = 1; m <= 8; m <<= 1) {
      acc[j].x += __shfl_xor(acc[j].x, m, 64);
      acc[j].y += __shfl_xor(acc[j].y, m, 64);
      acc[j].z += __shfl_xor(acc[j].z, m, 64);
      acc[j].w += __shfl_xor(acc[j].w, m, 64);
    }
    if (c16 == 0) red[(tid >> 6) + 4 * j][(tid >> 4) & 3] = acc[j];
  }
  if (tid < 64) {
    float s = gsum;
#pragma unroll
    for (int m = 1; m <= 8; m <<= 1) s += __shfl_xor(s, m, 64);
    if (tid == 0) sgs = s;
  }
  __syncthreads();
  float lsum = 0.f;                          // in l order; the LDS reads eight at a time
#pragma unroll 8
  for (int l = 0; l < U; ++l) lsum += slw[l];
  const int np_ = kHd * C + 2 * kHd + 1;
  float* pp = partial + (size_t)blockIdx.x * np_;
  for (int e = tid; e < np_; e += 256) {
    float val;
    int k, comp;
    if (e < kHd * C) {
      k = e / C;
      comp = 2 + e % C;
    } else if (e < kHd * C + kHd) {
      k = e - kHd * C;
      comp = 1;
    } else if (e < kHd * C + 2 * kHd) {
      k = e - kHd * C - kHd;
      comp = 0;
    } else {
      pp[e] = sgs * lsum;
      continue;
    }
    const float4 q = red[(k >> 4) * kNStat + comp][(k >> 2) & 3];
    const int r = k & 3;
    val = r == 0 ? q.x : (r == 1 ? q.y : (r == 2 ? q.z : q.w));
    pp[e] = comp == 0 ? val : w2[k] * val;
  }
}

bool bag_geom(int B, int U, int C, int P1, int P2, int Ho, int Wo, int Hd, BagGeom& g) {
  if (B < 1 || U < 1 || U > kMaxU || C < 1 || C > 4 || Hd != kHd || Ho < 1 || Wo < 1 || Ho > P1 ||
      Wo > P2)
    return false;
  if ((int64_t)B * U * C * P1 * P2 >= INT32_MAX || (int64_t)B * Ho * Wo >= INT32_MAX) return false;
  g.npts = (unsigned)(B * Ho * Wo);
  g.S = (unsigned)(Ho * Wo);
  g.Wo = (unsigned)Wo;
  g.P2 = (unsigned)P2;
  g.HW = (unsigned)(P1 * P2);
  g.C = (unsigned)C;
  g.U = (unsigned)U;
  g.dS = FastDiv::make(g.S);
  g.dWo = FastDiv::make(g.Wo);
  return true;
}

}  // namespace

BLINDNO_API int64_t blindno_project_bag_stats_floats(int B, int Ho, int Wo) {
  return ((int64_t)B * Ho * Wo + 15) / 16 * (int64_t)kTileF4 * 4;
}

#ifndef BAGPROJ_BWD_BLOCKS
#define BAGPROJ_BWD_BLOCKS 1024
#endif
BLINDNO_API int blindno_project_bag_bwd_nchunk(int B, int Ho, int Wo) {
  const int64_t tiles = ((int64_t)B * Ho * Wo + 15) / 16;
  return (int)(tiles < 1 ? 1 : (tiles > BAGPROJ_BWD_BLOCKS ? BAGPROJ_BWD_BLOCKS : tiles));
}

BLINDNO_API int blindno_project_bag_fwd(const float* z, const float* w1, const float* b1,
                                        const float* w2, const float* b2, const float* lw,
                                        float* ubar, float* stats, float* v, int B, int U, int C,
                                        int P1, int P2, int Ho, int Wo, int Hd, void* stream) {
  BagGeom g;
  if (!bag_geom(B, U, C, P1, P2, Ho, Wo, Hd, g) || !z || !ubar || !stats || !v)
    return (int)hipErrorInvalidValue;
  const unsigned ntiles = (g.npts + 15) / 16;
  bagproj_fwd_kernel<<<ntiles, 256, 0, (hipStream_t)stream>>>(z, w1, b1, w2, b2, lw, ubar, stats,
                                                               v, g);
  return (int)hipGetLastError();
}

BLINDNO_API int blindno_project_bag_bwd(const float* stats, const float* gs, const float* w2,
                                        const float* lw, const float* v, float* dz,
                                        float* partial, int nchunk, int B, int U, int C, int P1,
                                        int P2, int Ho, int Wo, int Hd, void* stream) {
  BagGeom g;
  if (!bag_geom(B, U, C, P1, P2, Ho, Wo, Hd, g) || !stats || !gs || (dz && !v) || !partial ||
      nchunk < 1)
    return (int)hipErrorInvalidValue;
  bagproj_bwd_kernel<<<nchunk, 256, 0, (hipStream_t)stream>>>(stats, gs, w2, lw, v, dz, partial, g);
  return (int)hipGetLastError();
}
