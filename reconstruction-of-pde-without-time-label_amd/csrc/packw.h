// The spectral weights' packed layout <-> the reference layout (weights1 / weights2 of
// SpectralConv2d, 2d_FPE/FNOModules.py:141-146), shared by the pack / unpack launches
// (spectral.hip) and the deferred finalisation launch that hosts the unpack beside the gradient
// reductions (fields.hip, blindno_finish_multi).
#pragma once
#include "common.h"

namespace blindno {

// Several blindno_pack_w2d in one launch: segment i packs (w1s[i], w2s[i]) of shape
// (Ci, Co, m1, m2) at row count P1 into Wts[i] (m2, K1, Ci, Co) complex -- the spectral weights
// of every layer of one FNO body (or of both grouped heads) before its forward chain.
constexpr int kPackSegs = 16;
struct PackSegs {
  const float* w1[kPackSegs];
  const float* w2[kPackSegs];
  float2* Wt[kPackSegs];
  int Ci[kPackSegs], Co[kPackSegs], m1[kPackSegs], m2[kPackSegs], P1[kPackSegs];
  int cum[kPackSegs + 1];
  int nseg;
};

// LDS-tiled packing / unpacking when no kept row overlaps (2 m1 < P1: kept row j < m1 is
// weights1 row j, j >= m1 is weights2 row j - m1).  For each (which, jj) the move is a
// transpose of the [Ci Co] x [m2] complex block (reference layout: k fastest; packed: (i, o)
// fastest); a workgroup moves one 32 x 32 tile through LDS so that both the reads and the
// writes are 256-B runs (the element-wise kernels read or wrote with an m1 m2 or Ci Co stride).
// Block b of segment s -> (which, jj, io tile, k tile); DIR 0 packs, DIR 1 unpacks.
// One tile: block b of the tile grid, thread t < 256 of the 32 x 8 tile team, tile the team's
// 32 x 33 LDS buffer.  !active: the team only takes part in the barrier (a hosting launch whose
// workgroups run several teams).
template <int DIR>
__device__ __forceinline__ void w2d_transpose_tile(const PackSegs& segs, int b, int t,
                                                   float2 (*tile)[33], bool active) {
  int sg = 0;
  while (sg + 1 < segs.nseg && segs.cum[sg + 1] <= b) ++sg;    // uniform scan
  const int Ci = segs.Ci[sg], Co = segs.Co[sg], m1 = segs.m1[sg], m2 = segs.m2[sg];
  const int CC = Ci * Co, K1 = 2 * m1;
  const int nio = (CC + 31) >> 5, nk = (m2 + 31) >> 5;
  int q = b - segs.cum[sg];
  const int kt = q % nk; q /= nk;
  const int iot = q % nio; q /= nio;
  const int jj = q % m1;
  const int which = q / m1;
  // reference-layout block: w[io][jj][k] (complex, k fastest), io = i Co + o
  const float2* wsrc = reinterpret_cast<const float2*>(which ? segs.w2[sg] : segs.w1[sg]);
  float2* wdst = reinterpret_cast<float2*>(const_cast<float*>(which ? segs.w2[sg] : segs.w1[sg]));
  float2* W = segs.Wt[sg];                       // packed: W[k][j][io], j = which m1 + jj
  const int j = which * m1 + jj;
  const int tx = t & 31, ty = t >> 5;                          // 32 x 8 threads
  if (DIR == 0) {
#pragma unroll
    for (int r = 0; r < 32; r += 8) {
      const int io = iot * 32 + ty + r, k = kt * 32 + tx;
      if (active && io < CC && k < m2) tile[ty + r][tx] = wsrc[((int64_t)io * m1 + jj) * m2 + k];
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 32; r += 8) {
      const int k = kt * 32 + ty + r, io = iot * 32 + tx;
      if (active && io < CC && k < m2) W[((int64_t)k * K1 + j) * CC + io] = tile[tx][ty + r];
    }
  } else {
#pragma unroll
    for (int r = 0; r < 32; r += 8) {
      const int k = kt * 32 + ty + r, io = iot * 32 + tx;
      if (active && io < CC && k < m2) tile[tx][ty + r] = W[((int64_t)k * K1 + j) * CC + io];
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 32; r += 8) {
      const int io = iot * 32 + ty + r, k = kt * 32 + tx;
      if (active && io < CC && k < m2) wdst[((int64_t)io * m1 + jj) * m2 + k] = tile[ty + r][tx];
    }
  }
}


// segments -> block table for w2d_transpose_tile; false if a segment has overlapping kept rows
// (the element-wise kernels handle those)
inline bool w2d_tiled_segs(PackSegs& segs, int64_t& blocks) {
  blocks = 0;
  for (int i = 0; i < segs.nseg; ++i) {
    if (2 * segs.m1[i] >= segs.P1[i]) return false;
    segs.cum[i] = (int)blocks;
    const int64_t nio = (segs.Ci[i] * segs.Co[i] + 31) / 32, nk = (segs.m2[i] + 31) / 32;
    blocks += 2 * (int64_t)segs.m1[i] * nio * nk;
  }
  segs.cum[segs.nseg] = (int)blocks;
  return blocks < INT32_MAX;
}

}  // namespace blindno
