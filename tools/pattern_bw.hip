// Access-pattern bandwidth probe for the encoder's row kernels (standalone; not part of the
// library).  Copies a (Bn, 4, P, P) fp32 field (Bn = 300, P = 160: 123 MB each way) with:
//   copy      contiguous: every lane 16 B, a wave instruction 1 KiB
//   frag<D>   the row kernels' fragment order: a wave owns 16 rows x 160 columns of all 4
//             channels, lane (r16, g) moves float4 [row r16][16 t + 4 g ..] per channel and
//             column tile t, with D tiles of loads in flight ahead of the stores
//   frag_alu  frag<1> plus ~the epilogue's VALU work per element (GELU + 4x4 conv)
// Prints GB/s (read + write) per pattern.  Build: hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void copy_kernel(const f32x4* __restrict__ x, f32x4* __restrict__ y, long n4) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x)
    y[i] = x[i];
}

__device__ __forceinline__ float gelu_like(float z) {
  const float t = __builtin_amdgcn_rcpf(fmaf(fabsf(z), 0.23f, 1.0f));
  const float e = __builtin_amdgcn_exp2f(z * z * -0.72f);
  float q = fmaf(t, 0.53f, -0.72f);
  q = fmaf(t, q, 0.71f);
  q = fmaf(t, q, -0.14f);
  q = fmaf(t, q, 0.12f);
  const float h = q * t * e;
  return z * (z >= 0.f ? 1.f - h : h);
}

__global__ void fill_kernel(float* x, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    x[i] = __sinf((float)(i % 100003) * 0.37f);
}

// MFMA: 4 chains of 6 v_mfma_f32_16x16x4f32 per tile (the row inverse's work), the A operand
// from an LDS image like the real kernel's twiddles
template <int D, bool ALU, bool MF = false, bool RANDOP = false>
__global__ __launch_bounds__(256) void frag_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                   int Bn, int P, float w) {
  __shared__ float sA[10 * 64 * 6];
  for (int e = threadIdx.x; e < 10 * 64 * 6; e += 256) sA[e] = RANDOP ? __sinf(1.3f * e + 0.7f) : 0.001f * (e % 17);
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r16 = lane & 15, g = lane >> 4;
  const int HB = P / 16, NT = P / 16, HW = P * P;
  const int nitems = Bn * HB;
  for (int item = blockIdx.x * 4 + wave; item < nitems; item += gridDim.x * 4) {
    const int n = item / HB, h = (item - n * HB) * 16 + r16;
    const long base = (long)n * 4 * HW + (long)h * P + 4 * g;
    f32x4 buf[D][4];
#pragma unroll
    for (int d = 0; d < D; ++d)
#pragma unroll
      for (int c = 0; c < 4; ++c) buf[d][c] = *reinterpret_cast<const f32x4*>(x + base + c * HW + 16 * d);
    for (int t = 0; t < NT; ++t) {
      f32x4 cur[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) cur[c] = buf[0][c];
#pragma unroll
      for (int d = 0; d + 1 < D; ++d)
#pragma unroll
        for (int c = 0; c < 4; ++c) buf[d][c] = buf[d + 1][c];
      const int tn = t + D < NT ? t + D : NT - 1;
#pragma unroll
      for (int c = 0; c < 4; ++c) buf[D - 1][c] = *reinterpret_cast<const f32x4*>(x + base + c * HW + 16 * tn);
      if (MF) {
        float zb[4][6];
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
          for (int s = 0; s < 6; ++s) zb[c][s] = RANDOP ? cur[c][s & 3] * 0.37f + (float)s : 0.01f * (c + s + r16);
        const float2* ta = reinterpret_cast<const float2*>(sA + (t * 64 + lane) * 6);
        float av[6];
#pragma unroll
        for (int q = 0; q < 3; ++q) { const float2 v = ta[q]; av[2 * q] = v.x; av[2 * q + 1] = v.y; }
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          f32x4 d = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int s = 0; s < 6; ++s) d = __builtin_amdgcn_mfma_f32_16x16x4f32(av[s], zb[c][s], d, 0, 0, 0);
          cur[c] += d;
        }
      }
      if (ALU) {
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
          for (int r = 0; r < 4; ++r) cur[c][r] = gelu_like(cur[c][r]);
        f32x4 o[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          o[c] = cur[c];
#pragma unroll
          for (int i = 0; i < 4; ++i) o[c] += w * cur[i];
        }
#pragma unroll
        for (int c = 0; c < 4; ++c) cur[c] = o[c];
      }
#pragma unroll
      for (int c = 0; c < 4; ++c) *reinterpret_cast<f32x4*>(y + base + c * HW + 16 * t) = cur[c];
    }
  }
}

int main() {
  const int Bn = 300, P = 160;
  const long n = (long)Bn * 4 * P * P;
  float *x, *y;
  hipMalloc(&x, n * 4);
  hipMalloc(&y, n * 4);
  fill_kernel<<<4096, 256>>>(x, n);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto run = [&](const char* name, auto launch) {
    for (int i = 0; i < 3; ++i) launch();
    hipEventRecord(e0);
    const int reps = 20;
    for (int i = 0; i < reps; ++i) launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double us = ms * 1e3 / reps;
    printf("%-24s %8.1f us  %7.0f GB/s\n", name, us, 2.0 * n * 4 / (us * 1e-6) / 1e9);
  };
  const int items = Bn * P / 16;
  run("copy", [&] { copy_kernel<<<4096, 256>>>((const f32x4*)x, (f32x4*)y, n / 4); });
  for (int blocks : {256, 512, 750}) {
    char nm[64];
    const int b = blocks < (items + 3) / 4 ? blocks : (items + 3) / 4;
    snprintf(nm, sizeof nm, "frag<1> b%d", b);
    run(nm, [&] { frag_kernel<1, false><<<b, 256>>>(x, y, Bn, P, 0.1f); });
    snprintf(nm, sizeof nm, "frag<2> b%d", b);
    run(nm, [&] { frag_kernel<2, false><<<b, 256>>>(x, y, Bn, P, 0.1f); });
    snprintf(nm, sizeof nm, "frag<4> b%d", b);
    run(nm, [&] { frag_kernel<4, false><<<b, 256>>>(x, y, Bn, P, 0.1f); });
    snprintf(nm, sizeof nm, "frag_alu<1> b%d", b);
    run(nm, [&] { frag_kernel<1, true><<<b, 256>>>(x, y, Bn, P, 0.1f); });
    snprintf(nm, sizeof nm, "frag_alu<2> b%d", b);
    run(nm, [&] { frag_kernel<2, true><<<b, 256>>>(x, y, Bn, P, 0.1f); });
    snprintf(nm, sizeof nm, "frag_mfma_alu<1> b%d", b);
    run(nm, [&] { frag_kernel<1, true, true><<<b, 256>>>(x, y, Bn, P, 0.1f); });
    snprintf(nm, sizeof nm, "frag_mfma_alu<2> b%d", b);
    run(nm, [&] { frag_kernel<2, true, true><<<b, 256>>>(x, y, Bn, P, 0.1f); });
    snprintf(nm, sizeof nm, "frag_mfma_alu_rand<1> b%d", b);
    run(nm, [&] { frag_kernel<1, true, true, true><<<b, 256>>>(x, y, Bn, P, 0.1f); });
  }
  hipFree(x);
  hipFree(y);
  return 0;
}
