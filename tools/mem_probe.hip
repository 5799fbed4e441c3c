// Load latency seen by the waves of a small launch, gfx950 (why the head kernels' phases are
// slow): each wave stamps s_memrealtime (100 MHz) around two dependent 16-B loads.
//
//   hipcc -O3 --offload-arch=gfx950 tools/mem_probe.hip -o tools/mem_probe && tools/mem_probe
//
// Grid: 2048 waves (256 workgroups of 8 waves, like colfuse at the heads).  Wave w reads at
// offset (w * stride) mod span (+ its lane).  First load: a line no one touched in this launch
// unless span is small; second load: 64 KB further on (another line, maybe another page).
// Printed per case: median / 90th percentile of the two load latencies and of the wave's life.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(512) void probe(const f4* __restrict__ buf, long span4, long stride4,
                                             unsigned long long* stamps, float* sink) {
  const int wave = blockIdx.x * 8 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  long off = ((long)wave * stride4) % span4;
  f4 v = buf[off + lane];
  float s = v.x + v.y + v.z + v.w;
  __builtin_amdgcn_sched_barrier(0);
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime() + (s == -1.f ? 1 : 0);
  off = (off + 4096 + (s == -2.f ? 1 : 0)) % span4;
  v = buf[off + lane];
  s += v.x + v.y + v.z + v.w;
  __builtin_amdgcn_sched_barrier(0);
  const unsigned long long t2 = __builtin_amdgcn_s_memrealtime() + (s == -1.f ? 1 : 0);
  if (lane == 0) {
    stamps[wave * 4 + 0] = t0;
    stamps[wave * 4 + 1] = t1;
    stamps[wave * 4 + 2] = t2;
  }
  if (s == -3.f) sink[threadIdx.x] = s;
}

__global__ void touch(f4* buf, long n4) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x)
    buf[i] = f4{1.f, 2.f, 3.f, 4.f};
}

static double pct(std::vector<double> v, double p) {
  std::sort(v.begin(), v.end());
  return v[(size_t)(p * (v.size() - 1))];
}

int main() {
  const int nw = 2048;
  const long big = 256L << 20;                   // 256 MB buffer
  f4* buf;
  float* sink;
  unsigned long long* st;
  hipMalloc(&buf, big);
  hipMalloc(&sink, 4096);
  hipMalloc(&st, sizeof(unsigned long long) * nw * 4);
  std::vector<unsigned long long> h(nw * 4);
  struct Case { const char* name; long span; long stride; bool rewrite; };
  const Case cases[] = {
      {"span 64 KB, same lines for all waves", 64L << 10, 1024, false},
      {"span 4 MB, 2 KB per wave", 4L << 20, 2048 / 16, false},
      {"span 4 MB, 2 KB per wave, written by the previous kernel", 4L << 20, 2048 / 16, true},
      {"span 64 MB, 32 KB per wave", 64L << 20, 32768 / 16, false},
      {"span 256 MB, 128 KB per wave", 256L << 20, 131072 / 16, false},
  };
  for (const Case& c : cases) {
    for (int rep = 0; rep < 4; ++rep) {
      if (c.rewrite || rep == 0) touch<<<1024, 256>>>(buf, c.span / 16);
      probe<<<nw / 8, 512>>>(buf, c.span / 16, c.stride, st, sink);
      hipDeviceSynchronize();
    }
    hipMemcpy(h.data(), st, sizeof(unsigned long long) * nw * 4, hipMemcpyDeviceToHost);
    std::vector<double> l1, l2, start;
    unsigned long long t0 = ~0ull;
    for (int w = 0; w < nw; ++w) t0 = std::min(t0, h[w * 4]);
    for (int w = 0; w < nw; ++w) {
      l1.push_back((h[w * 4 + 1] - h[w * 4]) * 0.01);
      l2.push_back((h[w * 4 + 2] - h[w * 4 + 1]) * 0.01);
      start.push_back((h[w * 4] - t0) * 0.01);
    }
    printf("%-58s first %5.2f / %5.2f us  second %5.2f / %5.2f us  start spread %5.2f us\n", c.name,
           pct(l1, 0.5), pct(l1, 0.9), pct(l2, 0.5), pct(l2, 0.9), pct(start, 1.0));
  }
  return 0;
}
