// Issue-cost probe for the instruction classes of the bag-level projection's inner loop
// (csrc/bagproj.hip): VALU-pipe cycles per wave64 instruction of v_pk_fma_f32, v_fma_f32,
// v_rcp_f32, v_exp_f32, v_bfi_b32 and v_mfma_f32_4x4x1f32, with 1..4 waves per SIMD.
//
//     hipcc -O3 -fno-slp-vectorize --offload-arch=gfx950 tools/valu_probe.hip -o tools/valu_probe && tools/valu_probe
//
// Each wave runs 8 independent chains of the instruction (no dependency stalls at >= 2 waves);
// cycles per instruction = elapsed * clock * SIMDs / (waves * instructions per wave), with the
// clock read from hipDeviceAttributeClockRate (the reported peak, so the numbers are upper
// bounds on the cost at the real clock).
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s\n", hipGetErrorString(e_)); return 1; } } while (0)

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int kIter = 4096;

template <int OP>
__global__ __launch_bounds__(256) void probe(float* out, float seed) {
  float a[8];
  f32x2 p[8];
  f32x4 d[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    a[j] = seed + 0.001f * (threadIdx.x + j);
    p[j] = (f32x2){a[j], a[j] + 1.f};
  }
  for (int i = 0; i < kIter; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (OP == 0) p[j] = __builtin_elementwise_fma(p[j], (f32x2){0.999f, 0.998f}, (f32x2){1e-3f, 2e-3f});
      if (OP == 1) a[j] = fmaf(a[j], 0.999f, 1e-3f);
      if (OP == 2) a[j] = __builtin_amdgcn_rcpf(a[j]);
      if (OP == 3) a[j] = __builtin_amdgcn_exp2f(a[j]);
      if (OP == 4) asm volatile("v_bfi_b32 %0, %1, %0, %2" : "+v"(a[j]) : "v"(0x7fffffff), "v"(seed));
    }
    if (OP == 6) {     // 8 v_pk_fma_f32 beside 4 v_mfma_f32_4x4x1f32 (does the matrix pipe overlap?)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        p[j] = __builtin_elementwise_fma(p[j], (f32x2){0.999f, 0.998f}, (f32x2){1e-3f, 2e-3f});
        if (j & 1) d[(j >> 1) & 1] = __builtin_amdgcn_mfma_f32_4x4x1f32(a[j], a[7 - j], d[(j >> 1) & 1], 0, 0, 0);
      }
    }
    if (OP == 5) {
#pragma unroll
      for (int j = 0; j < 8; ++j) d[j & 1] = __builtin_amdgcn_mfma_f32_4x4x1f32(a[j], a[7 - j], d[j & 1], 0, 0, 0);
    }
  }
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) s += a[j] + p[j].x + p[j].y;
  s += d[0][0] + d[1][1];
  if (s == 1234.5f) out[threadIdx.x] = s;
}

template <int OP>
int run(const char* name, int per_inst_extra, int cus, float ghz) {
  float* out;
  CHK(hipMalloc(&out, 4096));
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  for (int waves = 1; waves <= 4; ++waves) {
    const int blocks = cus * waves;           // 256 threads = 4 waves per block, one per SIMD
    probe<OP><<<blocks, 256>>>(out, 0.5f);
    CHK(hipEventRecord(e0));
    probe<OP><<<blocks, 256>>>(out, 0.5f);
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    float ms;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    const double insts = (double)kIter * 8 * (1 + per_inst_extra);
    const double cyc = ms * 1e-3 * ghz * 1e9 / (waves * insts);
    printf("%-22s waves/SIMD %d  %.2f cycles per wave-instruction\n", name, waves, cyc);
  }
  CHK(hipFree(out));
  return 0;
}

int main() {
  int cus = 0, khz = 0;
  CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  CHK(hipDeviceGetAttribute(&khz, hipDeviceAttributeClockRate, 0));
  const float ghz = khz * 1e-6f;
  printf("CUs %d, clock %.3f GHz\n", cus, ghz);
  if (run<0>("v_pk_fma_f32", 0, cus, ghz)) return 1;
  if (run<1>("v_fma_f32", 0, cus, ghz)) return 1;
  if (run<2>("v_rcp_f32", 0, cus, ghz)) return 1;
  if (run<3>("v_exp_f32", 0, cus, ghz)) return 1;
  if (run<4>("v_bfi_b32", 0, cus, ghz)) return 1;
  if (run<5>("v_mfma_f32_4x4x1f32", 0, cus, ghz)) return 1;
  if (run<6>("8 pk_fma + 4 mfma4x4 (per pk)", 0, cus, ghz)) return 1;
  return 0;
}
