// Internal launchers shared between the kernel translation units (not part of the C ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace blindno {

// project.hip: matrix-core projection MLP (Hd == 128, C <= 15, Cout <= 2, field < 2^31 elements).
// G > 1: G weight groups over consecutive Bn/G-sample blocks (weights + g wgs, output channel
// offset ooff + g Cout of sample n - g Bn/G; backward partials [nchunk][G][np]).
bool project_mfma_ok(int C, int Hd, int Cout, int64_t field_elems);
int project_fwd_mfma(const float* z, const float* w1, const float* b1, const float* w2,
                     const float* b2, float* out, int Bn, int C, int P1, int P2, int Ho, int Wo,
                     int Cout, int ostride, int ooff, int G, int64_t wgs, hipStream_t st);
int project_bwd_mfma_nchunk(int64_t npts);
int project_bwd_mfma_nchunk_wide(int64_t npts);   // the grouped 2D heads' grid
int project_bwd_mfma(const float* z, const float* w1, const float* b1, const float* w2,
                     const float* dout, float* dz, float* partial, int nchunk, int Bn, int C,
                     int P1, int P2, int Ho, int Wo, int Cout, int ostride, int ooff,
                     int dout_div, int G, int64_t wgs, hipStream_t st,
                     const float* lscale = nullptr);

// rowinv.hip: shapes whose spectrum (colidft output / rowidft input) is in A-tile order
bool rowinv_tile_layout(int Bn, int C, int P1, int P2, int m2);

}  // namespace blindno
