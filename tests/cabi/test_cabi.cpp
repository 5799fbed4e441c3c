// C++ caller of libblindno's C ABI -- no Python, no torch: the whole-op spectral convolutions
// (include/blindno.h, blindno_spectral_conv{2,1}d_*) on small shapes against a double-precision
// host restatement of the reference operation (2d_FPE/FNOModules.py:156-178: truncated rfft2 ->
// corner mix, weights2 winning on overlapping rows -> irfft2; 1d_FPE/FNOModules.py:47-59 with the
// DC bin halved), and the backward through the adjoint identities of the bilinear op:
//   <dy, y(x, w)> = <dx, x> = <dw1, w1> + <dw2, w2>.
// Built by build.py (hipcc, linked against blindno/libblindno.so); run by
// tests/test_gpu_cabi.py.  Exit status 0 = every check within tolerance.
#include <hip/hip_runtime.h>

#include <cmath>
#include <complex>
#include <cstdint>
#include <cstdio>
#include <vector>

#include "blindno.h"

namespace {

typedef std::complex<double> cd;
const double kPi = 3.14159265358979323846;
int g_fail = 0;

struct Rng {
  uint64_t s;
  double next() {  // uniform in [-1, 1)
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    return ((s >> 11) * (1.0 / 9007199254740992.0)) * 2.0 - 1.0;
  }
};

std::vector<float> randv(size_t n, Rng& r, double scale = 1.0) {
  std::vector<float> v(n);
  for (auto& x : v) x = (float)(scale * r.next());
  return v;
}

#define HIPCHECK(e)                                                                     \
  do {                                                                                  \
    hipError_t err_ = (e);                                                              \
    if (err_ != hipSuccess) {                                                           \
      std::fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(err_), __FILE__, \
                   __LINE__);                                                           \
      std::exit(2);                                                                     \
    }                                                                                   \
  } while (0)

#define ABICHECK(e)                                                                      \
  do {                                                                                   \
    int rc_ = (e);                                                                       \
    if (rc_ != 0) {                                                                      \
      std::fprintf(stderr, "%s failed: %s\n", #e, blindno_error_string(rc_));            \
      std::exit(3);                                                                      \
    }                                                                                    \
  } while (0)

struct Dev {
  void* p = nullptr;
  explicit Dev(size_t bytes) { HIPCHECK(hipMalloc(&p, bytes < 4 ? 4 : bytes)); }
  ~Dev() { (void)hipFree(p); }
  float* f() const { return (float*)p; }
};

Dev upload(const std::vector<float>& v) {
  Dev d(v.size() * sizeof(float));
  HIPCHECK(hipMemcpy(d.p, v.data(), v.size() * sizeof(float), hipMemcpyHostToDevice));
  return d;
}

std::vector<float> download(const Dev& d, size_t n) {
  std::vector<float> v(n);
  HIPCHECK(hipMemcpy(v.data(), d.p, n * sizeof(float), hipMemcpyDeviceToHost));
  return v;
}

double dot(const std::vector<float>& a, const std::vector<float>& b) {
  double s = 0.0;
  for (size_t i = 0; i < a.size(); ++i) s += (double)a[i] * b[i];
  return s;
}

void check(const char* what, double err, double tol) {
  const bool ok = err <= tol;
  std::printf("%-44s %.3e (tol %.0e) %s\n", what, err, tol, ok ? "ok" : "FAIL");
  if (!ok) ++g_fail;
}

// Hermitian weight of bin k of a length-n complex-to-real inverse
double c2r(int k, int n) { return (k == 0 || 2 * k == n) ? 1.0 : 2.0; }

void test2d(int Bn, int Ci, int Co, int P1, int P2, int m1, int m2, uint64_t seed) {
  std::printf("-- spectral_conv2d Bn=%d Ci=%d Co=%d P=%dx%d m=%dx%d\n", Bn, Ci, Co, P1, P2, m1, m2);
  Rng r{seed};
  const size_t nx = (size_t)Bn * Ci * P1 * P2, ny = (size_t)Bn * Co * P1 * P2;
  const size_t nw = (size_t)Ci * Co * m1 * m2 * 2;
  auto x = randv(nx, r), w1 = randv(nw, r, 0.5), w2 = randv(nw, r, 0.5), dy = randv(ny, r);
  // host reference: kept rows [0, m1) from weights1, [P1 - m1, P1) from weights2 (second wins)
  std::vector<int> rows, owner, jrow;
  std::vector<int> own(P1, 0), jr(P1, 0);
  for (int j = 0; j < m1; ++j) { own[j] = 1; jr[j] = j; }
  for (int j = 0; j < m1; ++j) { own[P1 - m1 + j] = 2; jr[P1 - m1 + j] = j; }
  for (int rr = 0; rr < P1; ++rr)
    if (own[rr]) { rows.push_back(rr); owner.push_back(own[rr]); jrow.push_back(jr[rr]); }
  std::vector<double> yref(ny, 0.0);
  for (int b = 0; b < Bn; ++b)
    for (size_t q = 0; q < rows.size(); ++q)
      for (int k = 0; k < m2; ++k) {
        const int rr = rows[q];
        std::vector<cd> xh(Ci, 0.0);
        for (int i = 0; i < Ci; ++i)
          for (int h = 0; h < P1; ++h)
            for (int w = 0; w < P2; ++w) {
              const double ph = -2 * kPi * ((double)((int64_t)rr * h % P1) / P1 + (double)((int64_t)k * w % P2) / P2);
              xh[i] += (double)x[(((size_t)b * Ci + i) * P1 + h) * P2 + w] * cd(std::cos(ph), std::sin(ph));
            }
        const std::vector<float>& W = owner[q] == 1 ? w1 : w2;
        for (int o = 0; o < Co; ++o) {
          cd acc = 0.0;
          for (int i = 0; i < Ci; ++i) {
            const size_t wi = ((((size_t)i * Co + o) * m1 + jrow[q]) * m2 + k) * 2;
            acc += xh[i] * cd(W[wi], W[wi + 1]);
          }
          for (int h = 0; h < P1; ++h)
            for (int w = 0; w < P2; ++w) {
              const double ph = 2 * kPi * ((double)((int64_t)rr * h % P1) / P1 + (double)((int64_t)k * w % P2) / P2);
              yref[(((size_t)b * Co + o) * P1 + h) * P2 + w] +=
                  c2r(k, P2) * (acc * cd(std::cos(ph), std::sin(ph))).real() / ((double)P1 * P2);
            }
        }
      }
  const int64_t tb = blindno_spectral2d_tables_bytes(P1, P2, m1, m2);
  const int64_t wf = blindno_spectral_conv2d_workspace_bytes(Bn, Ci, Co, P1, P2, m1, m2, 0);
  const int64_t wb = blindno_spectral_conv2d_workspace_bytes(Bn, Ci, Co, P1, P2, m1, m2, 1);
  const int64_t sb = blindno_spectral_conv2d_saved_bytes(Bn, Ci, P1, m1, m2);
  if (tb <= 0 || wf <= 0 || wb <= 0 || sb <= 0) { std::printf("bad size query\n"); ++g_fail; return; }
  Dev tables(tb), work(wf > wb ? wf : wb), saved(sb);
  ABICHECK(blindno_spectral2d_tables_init(tables.p, P1, P2, m1, m2));
  Dev dx_(nx * 4), y_(ny * 4), dw1_(nw * 4), dw2_(nw * 4);
  Dev x_ = upload(x), w1_ = upload(w1), w2_ = upload(w2), dy_ = upload(dy);
  hipStream_t st;
  HIPCHECK(hipStreamCreate(&st));
  ABICHECK(blindno_spectral_conv2d_fwd(x_.f(), w1_.f(), w2_.f(), y_.f(), saved.f(), work.p, tables.p, Bn, Ci,
                                       Co, P1, P2, m1, m2, st));
  ABICHECK(blindno_spectral_conv2d_bwd(dy_.f(), saved.f(), w1_.f(), w2_.f(), dx_.f(), dw1_.f(), dw2_.f(), work.p,
                                       tables.p, Bn, Ci, Co, P1, P2, m1, m2, st));
  HIPCHECK(hipStreamSynchronize(st));
  HIPCHECK(hipStreamDestroy(st));
  auto y = download(y_, ny), dx = download(dx_, nx), dw1 = download(dw1_, nw), dw2 = download(dw2_, nw);
  double num = 0, den = 0;
  for (size_t i = 0; i < ny; ++i) { num += (y[i] - yref[i]) * (y[i] - yref[i]); den += yref[i] * yref[i]; }
  check("forward rel-L2 vs double restatement", std::sqrt(num / den), 1e-5);
  double dyy = 0;
  for (size_t i = 0; i < ny; ++i) dyy += (double)dy[i] * yref[i];
  check("<dy,y> = <dx,x>   (input adjoint)", std::fabs(dot(dx, x) - dyy) / std::fabs(dyy), 1e-5);
  check("<dy,y> = <dw,w>   (weight adjoint)", std::fabs(dot(dw1, w1) + dot(dw2, w2) - dyy) / std::fabs(dyy), 1e-5);
  // invalid shapes are rejected with an error code, not a crash
  const int rc = blindno_spectral_conv2d_fwd(x_.f(), w1_.f(), w2_.f(), y_.f(), saved.f(), work.p, tables.p, Bn,
                                             Ci, Co, P1, P2, m1, P2, nullptr);
  check("invalid m2 rejected (rc != 0)", rc != 0 ? 0.0 : 1.0, 0.5);
}

void test1d(int Bn, int Ci, int Co, int P2, int m, uint64_t seed) {
  std::printf("-- spectral_conv1d Bn=%d Ci=%d Co=%d P=%d m=%d\n", Bn, Ci, Co, P2, m);
  Rng r{seed};
  const size_t nx = (size_t)Bn * Ci * P2, ny = (size_t)Bn * Co * P2, nw = (size_t)Ci * Co * m * 2;
  auto x = randv(nx, r), w = randv(nw, r, 0.5), dy = randv(ny, r);
  std::vector<double> yref(ny, 0.0);
  for (int b = 0; b < Bn; ++b)
    for (int k = 0; k < m; ++k) {
      std::vector<cd> xh(Ci, 0.0);
      for (int i = 0; i < Ci; ++i) {
        for (int t = 0; t < P2; ++t) {
          const double ph = -2 * kPi * (double)((int64_t)k * t % P2) / P2;
          xh[i] += (double)x[((size_t)b * Ci + i) * P2 + t] * cd(std::cos(ph), std::sin(ph));
        }
        if (k == 0) xh[i] *= 0.5;                     // x_ft[:, :, 0] *= 0.5
      }
      for (int o = 0; o < Co; ++o) {
        cd acc = 0.0;
        for (int i = 0; i < Ci; ++i) {
          const size_t wi = (((size_t)i * Co + o) * m + k) * 2;
          acc += xh[i] * cd(w[wi], w[wi + 1]);
        }
        for (int t = 0; t < P2; ++t) {
          const double ph = 2 * kPi * (double)((int64_t)k * t % P2) / P2;
          yref[((size_t)b * Co + o) * P2 + t] += c2r(k, P2) * (acc * cd(std::cos(ph), std::sin(ph))).real() / P2;
        }
      }
    }
  const int64_t tb = blindno_spectral1d_tables_bytes(P2, m);
  const int64_t wf = blindno_spectral_conv1d_workspace_bytes(Bn, Ci, Co, P2, m, 0);
  const int64_t wb = blindno_spectral_conv1d_workspace_bytes(Bn, Ci, Co, P2, m, 1);
  const int64_t sb = blindno_spectral_conv1d_saved_bytes(Bn, Ci, m);
  if (tb <= 0 || wf <= 0 || wb <= 0 || sb <= 0) { std::printf("bad size query\n"); ++g_fail; return; }
  Dev tables(tb), work(wf > wb ? wf : wb), saved(sb);
  ABICHECK(blindno_spectral1d_tables_init(tables.p, P2, m));
  Dev dx_(nx * 4), y_(ny * 4), dw_(nw * 4);
  Dev x_ = upload(x), w_ = upload(w), dy_ = upload(dy);
  ABICHECK(blindno_spectral_conv1d_fwd(x_.f(), w_.f(), y_.f(), saved.f(), work.p, tables.p, Bn, Ci, Co, P2, m,
                                       nullptr));
  ABICHECK(blindno_spectral_conv1d_bwd(dy_.f(), saved.f(), w_.f(), dx_.f(), dw_.f(), work.p, tables.p, Bn, Ci,
                                       Co, P2, m, nullptr));
  HIPCHECK(hipDeviceSynchronize());
  auto y = download(y_, ny), dx = download(dx_, nx), dw = download(dw_, nw);
  double num = 0, den = 0;
  for (size_t i = 0; i < ny; ++i) { num += (y[i] - yref[i]) * (y[i] - yref[i]); den += yref[i] * yref[i]; }
  check("forward rel-L2 vs double restatement", std::sqrt(num / den), 1e-5);
  double dyy = 0;
  for (size_t i = 0; i < ny; ++i) dyy += (double)dy[i] * yref[i];
  check("<dy,y> = <dx,x>   (input adjoint)", std::fabs(dot(dx, x) - dyy) / std::fabs(dyy), 1e-5);
  check("<dy,y> = <dw,w>   (weight adjoint)", std::fabs(dot(dw, w) - dyy) / std::fabs(dyy), 1e-5);
}

}  // namespace

int main() {
  std::printf("blindno ABI version %d\n", blindno_abi_version());
  test2d(3, 3, 4, 20, 18, 4, 5, 1);      // rows [0,4) and [16,20), even P2 (Nyquist bin unused)
  test2d(2, 2, 3, 6, 10, 4, 6, 2);       // P1 < 2 m1: overlapping rows (weights2 wins); m2 = P2/2+1
  test2d(2, 5, 5, 40, 40, 12, 12, 3);    // FNO_input-like geometry
  test1d(3, 3, 2, 18, 6, 4);
  test1d(2, 4, 4, 20, 11, 5);            // m = P2/2 + 1: the Nyquist bin
  std::printf(g_fail ? "FAILED (%d)\n" : "ALL OK\n", g_fail);
  return g_fail ? 1 : 0;
}
