// Cost of executing cold straight-line code at kernel start (instruction fetch), gfx950.
//
//   hipcc -O3 --offload-arch=gfx950 tools/icache_probe.hip -o tools/icache_probe && tools/icache_probe
//
// Two kernels execute the same number of dependent v_add_f32 (4-byte encodings): "straight"
// as one unrolled block of N instructions (N x 4 bytes of code, each fetched once per CU
// pair), "loop" as a 64-instruction body run N / 64 times.  Grid: 2048 waves (2 per SIMD),
// like the small head launches.  Per launch: the HIP-event time, averaged over 200 launches.
// The difference over N says what a cold instruction line costs.
#include <hip/hip_runtime.h>
#include <cstdio>

#define A1 asm volatile("v_add_f32 %0, %0, %1" : "+v"(x) : "v"(y));
#define A4 A1 A1 A1 A1
#define A16 A4 A4 A4 A4
#define A64 A16 A16 A16 A16
#define A256 A64 A64 A64 A64
#define A1024 A256 A256 A256 A256

template <int N>
__global__ __launch_bounds__(256) void straight(float* out, float y) {
  float x = threadIdx.x;
  if constexpr (N >= 1024) { A1024 }
  if constexpr (N >= 2048) { A1024 }
  if constexpr (N >= 3072) { A1024 }
  if constexpr (N >= 4096) { A1024 }
  if constexpr (N >= 5120) { A1024 }
  if constexpr (N >= 6144) { A1024 }
  if constexpr (N >= 7168) { A1024 }
  if constexpr (N >= 8192) { A1024 }
  if (x == -1.f) out[threadIdx.x] = x;
}

__global__ __launch_bounds__(256) void loop(float* out, float y, int n64) {
  float x = threadIdx.x;
#pragma unroll 1
  for (int i = 0; i < n64; ++i) { A64 }
  if (x == -1.f) out[threadIdx.x] = x;
}

template <typename F>
static float time_it(F f) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int i = 0; i < 20; ++i) f();
  hipEventRecord(a);
  for (int i = 0; i < 200; ++i) f();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms * 1000.f / 200.f;
}

template <int N>
static void row(float* out) {
  const dim3 g(512), blk(256);
  const float ts = time_it([&] { straight<N><<<g, blk>>>(out, 1.0f); });
  const float tl = time_it([&] { loop<<<g, blk>>>(out, 1.0f, N / 64); });
  printf("N %5d  code %6d B  straight %7.2f us  loop %7.2f us  diff %6.2f us  (%.1f ns per 64-B line)\n", N,
         N * 4, ts, tl, ts - tl, (ts - tl) * 1000.f / (N * 4 / 64));
}

int main() {
  float* out;
  hipMalloc(&out, 4096);
  row<1024>(out);
  row<2048>(out);
  row<4096>(out);
  row<8192>(out);
  hipFree(out);
  return 0;
}
