// Whole-op C ABI of the spectral convolutions for C / C++ hosts: SpectralConv2d
// (2d_FPE/FNOModules.py:156-178) and SpectralConv1d (1d_FPE/FNOModules.py:47-59), forward and
// backward, each ONE call.  The stage entry points (blindno_rowdft / _colpass / _mix1d /
// _rowidft_*, _mix_wgrad, _pack_*) need MFMA-lane-order twiddle images that the Python layer
// builds; here the library builds them itself (host, double precision, the same formulas as
// blindno/ops.py) into a caller-owned device buffer, and carves every intermediate out of a
// caller-owned workspace -- so the ABI's ownership rule holds (the library never allocates
// device memory) and a host needs nothing but these calls:
//
//   tables = alloc(blindno_spectral2d_tables_bytes(P1, P2, m1, m2));
//   blindno_spectral2d_tables_init(tables, P1, P2, m1, m2);            (once per shape)
//   work   = alloc(blindno_spectral_conv2d_workspace_bytes(...));
//   saved  = alloc(blindno_spectral_conv2d_saved_bytes(...));          (the spectrum, for bwd)
//   blindno_spectral_conv2d_fwd(x, w1, w2, y, saved, work, tables, ..., stream);
//   blindno_spectral_conv2d_bwd(dy, saved, w1, w2, dx, dw1, dw2, work, tables, ..., stream);
#include <cmath>
#include <vector>

#include "common.h"
#include "blindno.h"

using namespace blindno;

namespace {

constexpr double kTwoPi = 6.283185307179586476925286766559;

int kept_rows_host(int m1, int P1) { return 2 * m1 < P1 ? 2 * m1 : P1; }
int kept_row_host(int j, int K1, int m1, int P1) { return (K1 == P1 || j < m1) ? j : P1 - 2 * m1 + j; }

// twiddle_mfma (blindno/ops.py): Tp[kb][kq][n][s] = T[16 kb + 4 kq + s][n], T[w][2k] = cos,
// T[w][2k+1] = -sin of 2 pi ((w k) mod P2) / P2, zero for w >= P2 or n >= 2 m2
size_t tp_floats(int P2, int m2) {
  const int KB = (P2 + 15) / 16, Npad = ((2 * m2 + 15) / 16) * 16;
  return (size_t)KB * 16 * Npad;
}
void build_tp(float* out, int P2, int m2) {
  const int KB = (P2 + 15) / 16, Npad = ((2 * m2 + 15) / 16) * 16;
  for (int kb = 0; kb < KB; ++kb)
    for (int kq = 0; kq < 4; ++kq)
      for (int n = 0; n < Npad; ++n)
        for (int s = 0; s < 4; ++s) {
          const int w = 16 * kb + 4 * kq + s, k = n / 2;
          double v = 0.0;
          if (w < P2 && k < m2) {
            const double ph = (double)(((int64_t)w * k) % P2) * (kTwoPi / P2);
            v = (n & 1) ? -std::sin(ph) : std::cos(ph);
          }
          out[(((size_t)kb * 4 + kq) * Npad + n) * 4 + s] = (float)v;
        }
}

// twiddle_rowinv: tb[s][t][l] = cos (kk even) / -sin (kk odd) of 2 pi ((k w) mod P2) / P2,
// kk = 4 s + (l >> 4), k = kk / 2, w = 16 t + (l & 15); zero for k >= m2 or w >= P2
size_t tb_floats(int P2, int m2) { return (size_t)((m2 + 1) / 2) * ((P2 + 15) / 16) * 64; }
void build_tb(float* out, int P2, int m2) {
  const int KS = (m2 + 1) / 2, NT = (P2 + 15) / 16;
  for (int s = 0; s < KS; ++s)
    for (int t = 0; t < NT; ++t)
      for (int l = 0; l < 64; ++l) {
        const int kk = 4 * s + (l >> 4), k = kk / 2, w = 16 * t + (l & 15);
        double v = 0.0;
        if (k < m2 && w < P2) {
          const double ph = (double)(((int64_t)k * w) % P2) * (kTwoPi / P2);
          v = (kk % 2 == 0) ? std::cos(ph) : -std::sin(ph);
        }
        out[((size_t)s * NT + t) * 64 + l] = (float)v;
      }
}

// twiddle_cols: F[h][j] = e^{-2 pi i (h r_j mod P1) / P1} (h < P1, j < K1, else 0);
// FB[jt][hb][kq][c][s] = F[16 hb + 4 kq + s][16 jt + c], GB[ht][jb][kq][c][s] =
// conj F[16 ht + c][16 jb + 4 kq + s]; complex interleaved
size_t fb_floats(int P1, int m1) {
  const int K1 = kept_rows_host(m1, P1);
  return (size_t)((K1 + 15) / 16) * ((P1 + 15) / 16) * 256 * 2;
}
void build_fb_gb(float* fb, float* gb, int P1, int m1) {
  const int K1 = kept_rows_host(m1, P1);
  const int Jt = (K1 + 15) / 16, Ht = (P1 + 15) / 16;
  auto F = [&](int h, int j, double& re, double& im) {
    re = im = 0.0;
    if (h >= P1 || j >= K1) return;
    const int r = kept_row_host(j, K1, m1, P1);
    const double ph = (double)(((int64_t)h * r) % P1) * (kTwoPi / P1);
    re = std::cos(ph);
    im = -std::sin(ph);
  };
  for (int jt = 0; jt < Jt; ++jt)
    for (int hb = 0; hb < Ht; ++hb)
      for (int kq = 0; kq < 4; ++kq)
        for (int c = 0; c < 16; ++c)
          for (int s = 0; s < 4; ++s) {
            double re, im;
            F(16 * hb + 4 * kq + s, 16 * jt + c, re, im);
            const size_t o = ((((size_t)jt * Ht + hb) * 4 + kq) * 16 + c) * 4 + s;
            fb[2 * o] = (float)re;
            fb[2 * o + 1] = (float)im;
          }
  for (int ht = 0; ht < Ht; ++ht)
    for (int jb = 0; jb < Jt; ++jb)
      for (int kq = 0; kq < 4; ++kq)
        for (int c = 0; c < 16; ++c)
          for (int s = 0; s < 4; ++s) {
            double re, im;
            F(16 * ht + c, 16 * jb + 4 * kq + s, re, im);
            const size_t o = ((((size_t)ht * Jt + jb) * 4 + kq) * 16 + c) * 4 + s;
            gb[2 * o] = (float)re;
            gb[2 * o + 1] = (float)-im;
          }
}

constexpr size_t kAlign = 256;
size_t round_up(size_t b) { return (b + kAlign - 1) / kAlign * kAlign; }

struct Carve {
  char* base;
  size_t off = 0;
  float* take(size_t nfloats) {
    float* p = base ? reinterpret_cast<float*>(base + off) : nullptr;
    off += round_up(nfloats * sizeof(float));
    return p;
  }
};

// table offsets (in floats, each rounded to the alignment) inside the tables buffer
struct Tables2D {
  const float *Tp, *FB, *GB, *tb;
};
Tables2D tables2d(const void* t, int P1, int P2, int m1, int m2) {
  Carve c{(char*)t};
  Tables2D r;
  r.Tp = c.take(tp_floats(P2, m2));
  r.FB = c.take(fb_floats(P1, m1));
  r.GB = c.take(fb_floats(P1, m1));
  r.tb = c.take(tb_floats(P2, m2));
  return r;
}

bool shape2d_ok(int Bn, int Ci, int Co, int P1, int P2, int m1, int m2) {
  return Bn >= 1 && Ci >= 1 && Co >= 1 && Ci <= 32 && Co <= 32 && m1 >= 1 && m1 <= P1 && m2 >= 1 &&
         m2 <= P2 / 2 + 1 && m2 <= 48 && (int64_t)Bn * (Ci > Co ? Ci : Co) * P1 * P2 < INT32_MAX;
}

// workspace layout of the 2D ops
struct Work2D {
  float *Wt, *At, *Y, *Z, *G, *dWt, *partial;
};
Work2D carve2d(void* w, int Bn, int Ci, int Co, int P1, int m1, int m2, int bwd,
               size_t* bytes = nullptr) {
  Carve c{(char*)w};
  const int K1 = kept_rows_host(m1, P1), K1p = 16 * ((K1 + 15) / 16);
  Work2D r{};
  r.Wt = c.take((size_t)m2 * K1 * Ci * Co * 2);
  if (!bwd) {
    r.At = c.take((size_t)Bn * m2 * Ci * P1 * 2);
    r.Y = c.take((size_t)Bn * m2 * Co * K1p * 2);
    r.Z = c.take((size_t)Bn * P1 * m2 * Co * 2);
  } else {
    const int ns = blindno_mix_wgrad_nsplit(Bn, Ci, Co, K1, m2);
    r.At = c.take((size_t)Bn * m2 * Co * P1 * 2);
    r.G = c.take((size_t)Bn * m2 * Co * K1 * 2);
    r.Y = c.take((size_t)Bn * m2 * Ci * K1p * 2);
    r.Z = c.take((size_t)Bn * P1 * m2 * Ci * 2);
    r.dWt = c.take((size_t)m2 * K1 * Ci * Co * 2);
    r.partial = c.take(ns > 1 ? (size_t)ns * m2 * K1 * Ci * Co * 2 : 1);
  }
  if (bytes) *bytes = c.off;
  return r;
}

#define BLINDNO_TRY(expr)          \
  do {                             \
    const int rc_ = (expr);        \
    if (rc_ != 0) return rc_;      \
  } while (0)

}  // namespace

// ------------------------------------------------------------------------------ 2D
BLINDNO_API int64_t blindno_spectral2d_tables_bytes(int P1, int P2, int m1, int m2) {
  if (P1 < 1 || P2 < 1 || m1 < 1 || m2 < 1) return -1;
  Carve c{nullptr};
  c.take(tp_floats(P2, m2));
  c.take(fb_floats(P1, m1));
  c.take(fb_floats(P1, m1));
  c.take(tb_floats(P2, m2));
  return (int64_t)c.off;
}

BLINDNO_API int blindno_spectral2d_tables_init(void* tables, int P1, int P2, int m1, int m2) {
  const int64_t bytes = blindno_spectral2d_tables_bytes(P1, P2, m1, m2);
  if (!tables || bytes < 0) return (int)hipErrorInvalidValue;
  std::vector<float> host((size_t)bytes / sizeof(float), 0.f);
  Carve c{(char*)host.data()};
  float* tp = c.take(tp_floats(P2, m2));
  float* fb = c.take(fb_floats(P1, m1));
  float* gb = c.take(fb_floats(P1, m1));
  float* tb = c.take(tb_floats(P2, m2));
  build_tp(tp, P2, m2);
  build_fb_gb(fb, gb, P1, m1);
  build_tb(tb, P2, m2);
  return (int)hipMemcpy(tables, host.data(), (size_t)bytes, hipMemcpyHostToDevice);
}

BLINDNO_API int64_t blindno_spectral_conv2d_workspace_bytes(int Bn, int Ci, int Co, int P1, int P2,
                                                            int m1, int m2, int bwd) {
  if (!shape2d_ok(Bn, Ci, Co, P1, P2, m1, m2)) return -1;
  size_t b = 0;
  (void)carve2d(nullptr, Bn, Ci, Co, P1, m1, m2, bwd, &b);
  return (int64_t)b;
}

BLINDNO_API int64_t blindno_spectral_conv2d_saved_bytes(int Bn, int Ci, int P1, int m1, int m2) {
  if (Bn < 1 || Ci < 1 || P1 < 1 || m1 < 1 || m2 < 1) return -1;
  return (int64_t)sizeof(float) * Bn * m2 * Ci * kept_rows_host(m1, P1) * 2;
}

BLINDNO_API int blindno_spectral_conv2d_fwd(const float* x, const float* w1, const float* w2,
                                            float* y, float* saved, void* work, const void* tables,
                                            int Bn, int Ci, int Co, int P1, int P2, int m1, int m2,
                                            void* stream) {
  if (!x || !w1 || !w2 || !y || !saved || !work || !tables || !shape2d_ok(Bn, Ci, Co, P1, P2, m1, m2))
    return (int)hipErrorInvalidValue;
  const Tables2D t = tables2d(tables, P1, P2, m1, m2);
  const Work2D w = carve2d(work, Bn, Ci, Co, P1, m1, m2, 0);
  BLINDNO_TRY(blindno_pack_w2d(w1, w2, w.Wt, Ci, Co, m1, m2, P1, stream));
  BLINDNO_TRY(blindno_rowdft(x, w.At, t.Tp, Bn, Ci, P1, P2, m2, 0, stream));
  BLINDNO_TRY(blindno_colpass(w.At, w.Wt, saved, w.Y, w.Z, t.FB, t.GB, Bn, Ci, Co, P1, m1, m2, P2, 0,
                              stream));
  return blindno_rowidft_epi(w.Z, nullptr, nullptr, nullptr, y, t.tb, Bn, Co, P1, P2, m2, 0, stream);
}

BLINDNO_API int blindno_spectral_conv2d_bwd(const float* dy, const float* saved, const float* w1,
                                            const float* w2, float* dx, float* dw1, float* dw2,
                                            void* work, const void* tables, int Bn, int Ci, int Co,
                                            int P1, int P2, int m1, int m2, void* stream) {
  if (!dy || !saved || !w1 || !w2 || !dw1 || !dw2 || !work || !tables ||
      !shape2d_ok(Bn, Ci, Co, P1, P2, m1, m2))
    return (int)hipErrorInvalidValue;
  const Tables2D t = tables2d(tables, P1, P2, m1, m2);
  const Work2D w = carve2d(work, Bn, Ci, Co, P1, m1, m2, 1);
  const int K1 = kept_rows_host(m1, P1);
  const int ns = blindno_mix_wgrad_nsplit(Bn, Ci, Co, K1, m2);
  BLINDNO_TRY(blindno_pack_w2d(w1, w2, w.Wt, Ci, Co, m1, m2, P1, stream));
  BLINDNO_TRY(blindno_rowdft(dy, w.At, t.Tp, Bn, Co, P1, P2, m2, 0, stream));
  BLINDNO_TRY(blindno_colpass(w.At, w.Wt, w.G, w.Y, w.Z, t.FB, t.GB, Bn, Ci, Co, P1, m1, m2, P2, 1,
                              stream));
  BLINDNO_TRY(blindno_mix_wgrad(saved, w.G, w.dWt, ns > 1 ? w.partial : nullptr, ns, Bn, Ci, Co, K1, m2,
                                stream));
  BLINDNO_TRY(blindno_unpack_w2d(w.dWt, dw1, dw2, Ci, Co, m1, m2, P1, stream));
  if (dx)
    return blindno_rowidft_bwd(w.Z, nullptr, nullptr, nullptr, dx, t.tb, nullptr, Bn, Ci, P1, P2, m2, 0,
                               stream);
  return 0;
}

// ------------------------------------------------------------------------------ 1D
BLINDNO_API int64_t blindno_spectral1d_tables_bytes(int P2, int m) {
  if (P2 < 1 || m < 1) return -1;
  Carve c{nullptr};
  c.take(tp_floats(P2, m));
  c.take(tb_floats(P2, m));
  return (int64_t)c.off;
}

BLINDNO_API int blindno_spectral1d_tables_init(void* tables, int P2, int m) {
  const int64_t bytes = blindno_spectral1d_tables_bytes(P2, m);
  if (!tables || bytes < 0) return (int)hipErrorInvalidValue;
  std::vector<float> host((size_t)bytes / sizeof(float), 0.f);
  Carve c{(char*)host.data()};
  float* tp = c.take(tp_floats(P2, m));
  float* tb = c.take(tb_floats(P2, m));
  build_tp(tp, P2, m);
  build_tb(tb, P2, m);
  return (int)hipMemcpy(tables, host.data(), (size_t)bytes, hipMemcpyHostToDevice);
}

namespace {
bool shape1d_ok(int Bn, int Ci, int Co, int P2, int m) {
  return Bn >= 1 && Ci >= 1 && Co >= 1 && Ci <= 32 && Co <= 32 && m >= 1 && m <= P2 / 2 + 1 && m <= 48 &&
         (int64_t)Bn * (Ci > Co ? Ci : Co) * P2 < INT32_MAX;
}
struct Work1D {
  float *Wt, *At, *Z, *G, *dWt, *partial;
};
Work1D carve1d(void* p, int Bn, int Ci, int Co, int m, int bwd, size_t* bytes) {
  Carve c{(char*)p};
  Work1D r{};
  r.Wt = c.take((size_t)m * Ci * Co * 2);
  if (!bwd) {
    r.At = c.take((size_t)Bn * m * Ci * 2);
    r.Z = c.take((size_t)Bn * m * Co * 2);
  } else {
    const int ns = blindno_mix_wgrad_nsplit(Bn, Ci, Co, 1, m);
    r.At = c.take((size_t)Bn * m * Co * 2);
    r.G = c.take((size_t)Bn * m * Co * 2);
    r.Z = c.take((size_t)Bn * m * Ci * 2);
    r.dWt = c.take((size_t)m * Ci * Co * 2);
    r.partial = c.take(ns > 1 ? (size_t)ns * m * Ci * Co * 2 : 1);
  }
  if (bytes) *bytes = c.off;
  return r;
}
}  // namespace

BLINDNO_API int64_t blindno_spectral_conv1d_workspace_bytes(int Bn, int Ci, int Co, int P2, int m,
                                                            int bwd) {
  if (!shape1d_ok(Bn, Ci, Co, P2, m)) return -1;
  size_t b = 0;
  (void)carve1d(nullptr, Bn, Ci, Co, m, bwd, &b);
  return (int64_t)b;
}

BLINDNO_API int64_t blindno_spectral_conv1d_saved_bytes(int Bn, int Ci, int m) {
  if (Bn < 1 || Ci < 1 || m < 1) return -1;
  return (int64_t)sizeof(float) * Bn * m * Ci * 2;
}

BLINDNO_API int blindno_spectral_conv1d_fwd(const float* x, const float* w, float* y, float* saved,
                                            void* work, const void* tables, int Bn, int Ci, int Co,
                                            int P2, int m, void* stream) {
  if (!x || !w || !y || !saved || !work || !tables || !shape1d_ok(Bn, Ci, Co, P2, m))
    return (int)hipErrorInvalidValue;
  Carve tc{(char*)tables};
  const float* Tp = tc.take(tp_floats(P2, m));
  const float* tb = tc.take(tb_floats(P2, m));
  const Work1D k = carve1d(work, Bn, Ci, Co, m, 0, nullptr);
  BLINDNO_TRY(blindno_pack_w1d(w, k.Wt, Ci, Co, m, 0, stream));
  BLINDNO_TRY(blindno_rowdft(x, k.At, Tp, Bn, Ci, 1, P2, m, 0, stream));
  BLINDNO_TRY(blindno_mix1d(k.At, k.Wt, saved, k.Z, Bn, Ci, Co, m, P2, 0, stream));
  return blindno_rowidft_epi(k.Z, nullptr, nullptr, nullptr, y, tb, Bn, Co, 1, P2, m, 0, stream);
}

BLINDNO_API int blindno_spectral_conv1d_bwd(const float* dy, const float* saved, const float* w,
                                            float* dx, float* dw, void* work, const void* tables,
                                            int Bn, int Ci, int Co, int P2, int m, void* stream) {
  if (!dy || !saved || !w || !dw || !work || !tables || !shape1d_ok(Bn, Ci, Co, P2, m))
    return (int)hipErrorInvalidValue;
  Carve tc{(char*)tables};
  const float* Tp = tc.take(tp_floats(P2, m));
  const float* tb = tc.take(tb_floats(P2, m));
  const Work1D k = carve1d(work, Bn, Ci, Co, m, 1, nullptr);
  const int ns = blindno_mix_wgrad_nsplit(Bn, Ci, Co, 1, m);
  BLINDNO_TRY(blindno_pack_w1d(w, k.Wt, Ci, Co, m, 0, stream));
  BLINDNO_TRY(blindno_rowdft(dy, k.At, Tp, Bn, Co, 1, P2, m, 0, stream));
  BLINDNO_TRY(blindno_mix1d(k.At, k.Wt, k.G, k.Z, Bn, Ci, Co, m, P2, 1, stream));
  BLINDNO_TRY(blindno_mix_wgrad(saved, k.G, k.dWt, ns > 1 ? k.partial : nullptr, ns, Bn, Ci, Co, 1, m,
                                stream));
  BLINDNO_TRY(blindno_pack_w1d(k.dWt, dw, Ci, Co, m, 1, stream));
  if (dx)
    return blindno_rowidft_bwd(k.Z, nullptr, nullptr, nullptr, dx, tb, nullptr, Bn, Ci, 1, P2, m, 0, stream);
  return 0;
}
