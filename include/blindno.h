/*
 * blindno.h -- C ABI of the MI355X-native BlinDNO FNO/NIO hot path (libblindno.so).
 *
 * Every entry point takes plain device pointers, sizes and a hipStream_t (passed as
 * void* so the header needs no HIP include), enqueues work on that stream and
 * returns a hipError_t value (0 = hipSuccess).  No entry point allocates device
 * memory, synchronises, or calls exit/abort: callers own all buffers (the Python
 * host layer uses PyTorch's caching allocator) and check the return code.
 *
 * All tensors are fp32, C-contiguous, on the current device.  Complex values are
 * interleaved (re, im) float pairs.
 *
 * Layout vocabulary (see DESIGN.md "Data layout in HBM"):
 *   field   x[n][c][h][w]    n < Bn snapshots/samples, c < C channels,
 *                            h < P1 (rows, 1 for 1D), w < P2 (padded grid)
 *   rowspec At[n][k][c][h]   row-DFT coefficients, k < m2 (column-major per mode)
 *   colspec X[n][k][c][j]    2D spectrum at the K1 kept frequency rows j
 *   rowcoef Z[n][h][k][c]    row coefficients feeding the inverse row transform
 *                            (all channels of one (row, mode) contiguous)
 *   wpack   Wt[k][j][ci][co] complex mixing weights, one block per kept mode
 * Kept rows: K1 = min(2*m1, P1); row j -> frequency r_j = j (j < m1 or K1 == P1)
 * else P1 - 2*m1 + j.  Rows r >= P1 - m1 are owned by weights2 (weights2 wins on
 * overlap, as the reference's second slice assignment does).
 *
 * Each declaration names the reference operation it replaces (file:line in
 * yl602019618/Reconstruction-of-PDE-without-Time-Label).
 */
#ifndef BLINDNO_H
#define BLINDNO_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* blindno_stream_t; /* hipStream_t */

/* ABI version: bump on any signature change. */
int blindno_abi_version(void);
/* Human-readable text of a returned error code (hipGetErrorString). */
const char* blindno_error_string(int code);

/* --- lift / projection ------------------------------------------------------------ */

/* fc0 + permute + F.pad: 2d_FPE/FNOModules.py:219-224, 1d_FPE/FNOModules.py:103-106.
 * in (Bn, N1, N2, Cin) channels-last -> x0 (Bn, C, P1, P2), zero outside h<N1, w<N2. */
int blindno_lift_fwd(const float* in, const float* w0, const float* b0, float* x0,
                     int Bn, int N1, int N2, int Cin, int C, int P1, int P2,
                     blindno_stream_t stream);

/* Backward of the lift: optional d_in (may be NULL) and per-chunk partial sums of
 * dW0 (C*Cin) then db0 (C) into partial[nchunk][C*Cin + C], nchunk =
 * blindno_lift_bwd_nchunk(Bn, N1, N2). */
int blindno_lift_bwd(const float* dx0, const float* in, const float* w0, float* d_in,
                     float* partial, int nchunk,
                     int Bn, int N1, int N2, int Cin, int C, int P1, int P2,
                     blindno_stream_t stream);
int blindno_lift_bwd_nchunk(int Bn, int N1, int N2);

/* crop + permute + fc1 + GELU + fc2: 2d_FPE/FNOModules.py:234-239, 1d_FPE/FNOModules.py:116-121.
 * z (Bn, C, P1, P2) -> out[(n*Ho + h)*Wo + w)*ostride + ooff + co] for h<Ho, w<Wo. */
int blindno_project_fwd(const float* z, const float* w1, const float* b1, const float* w2,
                        const float* b2, float* out, int Bn, int C, int P1, int P2, int Ho,
                        int Wo, int Hd, int Cout, int ostride, int ooff,
                        blindno_stream_t stream);

/* Backward of the projection: dz (Bn, C, P1, P2) (written only on the crop; caller
 * zero-fills the rest), per-workgroup partials of [dW1 (Hd*C), db1 (Hd), dW2 (Cout*Hd),
 * db2 (Cout)] into partial[nchunk][...], nchunk = blindno_project_bwd_nchunk(Bn, Ho, Wo)
 * (any value >= 1 is accepted).  dout is addressed like out in blindno_project_fwd, except
 * that the sample index n is divided by dout_div (snapshot-bag broadcast; 1 = none).
 * Hd must be a multiple of 64 (the reference's fc1 is Linear(width, 128)). */
int blindno_project_bwd(const float* z, const float* w1, const float* b1, const float* w2,
                        const float* dout, float* dz, float* partial, int nchunk,
                        int Bn, int C, int P1, int P2, int Ho, int Wo, int Hd, int Cout,
                        int ostride, int ooff, int dout_div, blindno_stream_t stream);
int blindno_project_bwd_nchunk(int Bn, int Ho, int Wo);
/* the partial count for the grouped 2D heads' blindno_project_bwd_g (a coarser grid that suits
 * them; any nchunk >= 1 is valid) */
int blindno_project_bwd_nchunk_heads(int Bg, int Ho, int Wo);
/* blindno_project_bwd (matrix-core path) with dout of sample n scaled by lscale[n % dout_div]
 * (the multiplicity weights of a deduplicated bag). */
int blindno_project_bwd_w(const float* z, const float* w1, const float* b1, const float* w2,
                          const float* dout, const float* lscale, float* dz, float* partial,
                          int nchunk, int Bn, int C, int P1, int P2, int Ho, int Wo, int Hd,
                          int Cout, int ostride, int ooff, int dout_div, blindno_stream_t stream);

/* Bag-level projection of the snapshot encoder (NIOFP2D_FNO's FNO_input projection fused with
 * the bag mean that consumes it: 2d_FPE/FNOModules.py:234-239 + 2d_FPE/NIOModules.py:569-575).
 * z (B U, C, P1, P2): the last encoder layer of the U snapshots of each of B bags (snapshot
 * n = b U + l), lw (U) the snapshot weights (multiplicity / L; NULL: 1/U).  C <= 4, Hd = 128,
 * Cout = 1, U <= 1024.  Forward writes
 *   ubar (B, Ho Wo) = sum_l lw_l (fc2(GELU(fc1(z_l))))   (the bag mean of the projections),
 *   stats (blindno_project_bag_stats_floats(B, Ho, Wo) floats): per 16-point tile the bag-level
 *         sums A = sum lw GELU(h), S = sum lw GELU'(h), Q = sum lw GELU'(h) z^T,
 *   v (B U, C, P1, P2) on the crop: W1^T (w2 * GELU'(h)) per snapshot point.
 * Backward: gs (B, Ho Wo) = the gradient of ubar; writes dz = lw_l gs v on the crop (dz NULL:
 * not written, v not read -- the consumers form it on load, blindno_rowdft_cd_bag /
 * blindno_rowidft_bwd_zc_bag) and
 * per-workgroup partials [dW1 (Hd*C) | db1 (Hd) | dW2 (Hd) | db2] into partial[nchunk][...],
 * nchunk = blindno_project_bag_bwd_nchunk(B, Ho, Wo) (any value >= 1). */
int64_t blindno_project_bag_stats_floats(int B, int Ho, int Wo);
int blindno_project_bag_bwd_nchunk(int B, int Ho, int Wo);
int blindno_project_bag_fwd(const float* z, const float* w1, const float* b1, const float* w2,
                            const float* b2, const float* lw, float* ubar, float* stats,
                            float* v, int B, int U, int C, int P1, int P2, int Ho, int Wo, int Hd,
                            blindno_stream_t stream);
int blindno_project_bag_bwd(const float* stats, const float* gs, const float* w2, const float* lw,
                            const float* v, float* dz, float* partial, int nchunk, int B, int U,
                            int C, int P1, int P2, int Ho, int Wo, int Hd,
                            blindno_stream_t stream);

/* --- truncated spectral transforms --------------------------------------------------- */

/* Row (last-axis) forward DFT of the first m2 modes: torch.fft.rfft2/rfft first stage
 * (2d_FPE/FNOModules.py:163, 1d_FPE/FNOModules.py:50).  act: 0 = identity, 1 = GELU
 * applied to x on load (x holds pre-activations).  x (Bn,C,P1,P2) -> At (rowspec).
 * Runs on the f32 matrix cores.  Tp: B-operand image of T (P2 x 2*m2, T[w][2k] = cos,
 * T[w][2k+1] = -sin of 2 pi k w/P2): Tp[kb][kq][n][s] = T[16 kb + 4 kq + s][n], KB =
 * ceil(P2/16), n < Npad = 16*ceil(2*m2/16), zero padded. */
int blindno_rowdft(const float* x, float* At, const float* Tp, int Bn, int C, int P1,
                   int P2, int m2, int act, blindno_stream_t stream);
/* blindno_rowdft reading only the valid region h < N1v, w < N2v of every P1 x P2 plane (the rest
 * counts as zero and is never read): the gradient of a cropped FNO output, left unfilled on the
 * padding by blindno_project_bwd. */
int blindno_rowdft_crop(const float* x, float* At, const float* Tp, int Bn, int C, int P1,
                        int P2, int m2, int act, int N1v, int N2v, blindno_stream_t stream);

/* Column pass of SpectralConv2d: column DFT at the K1 kept rows, per-mode complex channel
 * mix (compl_mul2d, 2d_FPE/FNOModules.py:141-154, 170-173), column inverse -- two complex
 * GEMMs against F[h][j] = e^{-2 pi i r_j h / P1} on the matrix cores.
 * FB: (ceil(K1/16), ceil(P1/16), 64, 4) complex image, FB[jt][hb][l][s] =
 *     F[16 hb + 4 (l>>4) + s][16 jt + (l&15)];  GB: (ceil(P1/16), ceil(K1/16), 64, 4) complex,
 *     GB[ht][jb][l][s] = conj F[16 ht + (l&15)][16 jb + 4 (l>>4) + s]  (zero outside).
 * Y: scratch (Bn, m2, C_out, K1p = 16 ceil(K1/16)) complex.
 * dir 0 (forward): Xs = colDFT(At) (Bn,m2,Ci,K1) saved for the weight gradient;
 *                  Z[n][h][k][o] = c_k/(P1 P2) colIDFT(sum_i Xs W)   (rowcoef, Co channels).
 * dir 1 (adjoint): At holds the row DFT of the output gradient (Co channels);
 *                  Xs = c_k/(P1 P2) colDFT(At) = spectrum gradient G (Bn,m2,Co,K1);
 *                  Z[n][h][k][i] = colIDFT(sum_o conj(W) G)             (Ci channels). */
int blindno_colpass(const float* At, const float* Wt, float* Xs, float* Y, float* Z,
                    const float* FB, const float* GB, int Bn, int Ci, int Co, int P1, int m1,
                    int m2, int P2, int dir, blindno_stream_t stream);

/* dWt[k,j,i,o] = sum_n conj(X[n,k,i,j]) G[n,k,o,j]  (weight gradient of the mix).  The
 * samples are split into nsplit slices (blindno_mix_wgrad_nsplit); with nsplit > 1 the
 * slice sums go to partial (nsplit x 2 m2 K1 Ci Co floats) and are reduced in fixed order. */
int blindno_mix_wgrad_nsplit(int Bn, int Ci, int Co, int K1, int m2);
int blindno_mix_wgrad(const float* X, const float* G, float* dWt, float* partial, int nsplit,
                      int Bn, int Ci, int Co, int K1, int m2, blindno_stream_t stream);
/* The sample-split partials of blindno_mix_wgrad only (nsplit >= 2): partial[y][Gw][...]
 * (complex); the caller reduces them (blindno_reduce_partials(_multi), 2 m2 K1 Ci Co Gw floats). */
int blindno_mix_wgrad_part(const float* X, const float* G, float* partial, int nsplit, int Gw,
                           int Bn, int Ci, int Co, int K1, int m2, blindno_stream_t stream);
/* Several blindno_mix_wgrad_g / _part launches in one (the deferred spectral weight gradients
 * of a backward pass: the heads' layers and the encoder's; bit-identical results): job q reads
 * X[q], G[q] and writes out[q] -- dWt (Gw, m2, K1, Ci, Co) when nsplit == 1, else the
 * nsplit x Gw partials for the caller to reduce; shp[7 q ..] = (Bn, Ci, Co, K1, m2, nsplit, Gw). */
int blindno_mix_wgrad_multi(const void* const* X, const void* const* G, void* const* out,
                            const int* shp, int njobs, blindno_stream_t stream);
/* ... with the unpack folded into the store: for job q with um1[q] > 0 (nsplit 1, K1 = 2 um1,
 * Gw <= 4), dWt of group g is written straight into the reference layouts (Ci, Co, um1, m2) of
 * the weights1 / weights2 gradients ud[8 q + 2 g], ud[8 q + 2 g + 1] (blindno_unpack_w2d's
 * result; out[q] is then not written).  ud / um1 NULL: blindno_mix_wgrad_multi. */
int blindno_mix_wgrad_multi_u(const void* const* X, const void* const* G, void* const* out,
                              const int* shp, void* const* ud, const int* um1, int njobs,
                              blindno_stream_t stream);

/* 1D mode mix (compl_mul1d + DC halving, 1d_FPE/FNOModules.py:43-58).  At (Bn,m,C,1).
 * dir 0 (forward):  Xs = At with X[.,0] *= 0.5 (saved); Z[n][0][k][o] = c_k/P2 sum_i Xs W.
 * dir 1 (adjoint):  Xs = c_k/P2 At (spectrum gradient); Z[n][0][k][i] = h_k sum_o conj(W) Xs
 *                   with h_0 = 0.5, h_k = 1.   W packed as Wt[k][ci][co] complex. */
int blindno_mix1d(const float* At, const float* Wt, float* Xs, float* Z, int Bn, int Ci,
                  int Co, int m, int P2, int dir, blindno_stream_t stream);

/* Inverse row transform + 1x1 conv + bias epilogue (irfft2 second stage, nn.Conv2d(k=1),
 * x1 + x2; 2d_FPE/FNOModules.py:177,226-230), on the f32 matrix cores:
 *   z[n,o,h,w] = sum_k Re(Z[n,h,k,o] e^{+2pi i k w/P2}) + sum_i Wc[o,i] f(x[n,i,h,w]) + bc[o]
 * f = identity (act 0) or GELU (act 1: x holds pre-activations).  wc == NULL drops the
 * conv/bias term (bare SpectralConv2d/1d; x, bc unused).  tb: B-operand image of the row
 * inverse, (ceil(m2/2), ceil(P2/16), 64) floats, tb[s][t][l] = cos (kk even) or -sin (kk odd)
 * of 2 pi k w / P2 with kk = 4 s + (l >> 4), k = kk / 2, w = 16 t + (l & 15), zero for k >= m2
 * or w >= P2.  C <= 32, m2 <= 48. */
int blindno_rowidft_epi(const float* Z, const float* x, const float* wc, const float* bc,
                        float* z, const float* tb, int Bn, int C, int P1, int P2, int m2,
                        int act, blindno_stream_t stream);
/* blindno_rowidft_epi writing z on the output crop h < oN1, w < oN2 only (the FNO_input body's
 * last layer, whose one reader -- the projection, FNOModules.py:234 -- reads nothing else; the
 * rest of z is left unwritten). */
int blindno_rowidft_epi_crop(const float* Z, const float* x, const float* wc, const float* bc,
                             float* z, const float* tb, int Bn, int C, int P1, int P2, int m2,
                             int act, int oN1, int oN2, blindno_stream_t stream);

/* Adjoint of rowidft_epi w.r.t. its input field:
 *   dx[n,i,h,w] = sum_k Re(G[n,h,k,i] e^{+2pi i k w/P2}) + sum_o Wc[o,i] dz[n,o,h,w]
 * then, if act == 1, dx *= GELU'(xsrc[n,i,h,w]) (xsrc = the layer input's pre-activation).
 * wc == NULL drops the conv term.  tb as in blindno_rowidft_epi.
 * If partial != NULL (requires C <= 4 and wc), the 1x1-conv gradients are reduced in the same
 * pass into partial[blindno_rowidft_bwd_nchunk(...)][C*C + C]
 * = [dWc[o][i] = sum dz_o f(xsrc_i) | dbc[o] = sum dz_o]. */
int blindno_rowidft_bwd(const float* G, const float* dz, const float* wc, const float* xsrc,
                        float* dx, const float* tb, float* partial, int Bn, int C, int P1,
                        int P2, int m2, int act, blindno_stream_t stream);
/* blindno_rowidft_bwd with dz read only on h < dN1, w < dN2 (zero elsewhere, never read). */
int blindno_rowidft_bwd_crop(const float* G, const float* dz, const float* wc, const float* xsrc,
                             float* dx, const float* tb, float* partial, int Bn, int C, int P1,
                             int P2, int m2, int act, int dN1, int dN2, blindno_stream_t stream);
int blindno_rowidft_bwd_nchunk(int Bn, int C, int P1, int P2, int m2);
/* Kernel selection of the C = 4 row inverses above (no reference counterpart; A/B measurement
 * and cross-checks): on = 1 (default, or environment BLINDNO_ROWFUSE unset / not "0") runs the
 * transposed whole-row kernel for C == 4, m2 % 4 == 0, m2 <= 16, P1 % 16 == 0, P2 % 32 == 0;
 * 0 the general kernel.  Returns the previous setting.  Not thread-safe against launches; the
 * partial count of blindno_rowidft_bwd_nchunk follows the setting. */
int blindno_set_rowfuse(int on);
/* The fused column pass (one launch per layer: column DFT, mix and column inverse with the
 * spectrum in LDS) on (1) or the split coldft_mix + colidft kernels (0); returns the previous
 * setting.  Default on; BLINDNO_COLFUSE=0 in the environment turns it off. */
int blindno_set_colfuse(int on);
/* Layer chaining (the FNO layer loop, 2d_FPE/FNOModules.py:226-232): the next spectral layer's
 * row DFT of the field a row inverse produces, taken in the same pass -- At / Tp exactly as
 * blindno_rowdft(field, At, Tp, Bn, C, P1, P2, m2, act_next) would take them (m2 of the next
 * layer equals this one's).  Fused for C <= 4, m2 <= 16 when a work item spans whole rows;
 * otherwise the entry launches blindno_rowdft itself after the row inverse.  Same results. */
/* blindno_rowidft_bwd_crop + At = rowDFT(dx) (act 0: the previous layer's adjoint input). */
int blindno_rowidft_bwd_rd(const float* G, const float* dz, const float* wc, const float* xsrc,
                           float* dx, const float* tb, float* partial, int Bn, int C, int P1,
                           int P2, int m2, int act, int dN1, int dN2, float* At, const float* Tp,
                           blindno_stream_t stream);
/* blindno_rowidft_epi + At = rowDFT(f(z)), f = GELU when act_next. */
int blindno_rowidft_epi_rd(const float* Z, const float* x, const float* wc, const float* bc,
                           float* z, const float* tb, int Bn, int C, int P1, int P2, int m2,
                           int act, float* At, const float* Tp, int act_next,
                           blindno_stream_t stream);

/* 1 when the spectrum Z that blindno_colpass(_g) writes and blindno_rowidft_epi/bwd(_g) read
 * is in A-tile order instead of Z[n][h][k][c]: C in {8, 12, 16} (the FNO heads, width 12), m2
 * even (m2/2 <= 16, <= 24 for C = 8), P1 % 4 == 0, P1 >= 16, field < 2^31 elements.  Layout:
 * Zt[((q C/4 + g) m2/2 + s) 64 + l] = Re (kk even) / Im (kk odd) of Z[row 4q + (l&15)/4][kk/2]
 * [4g + (l&3)] with kk = 4s + l/16, rows n P1 + h.  Both sides agree by construction; a caller
 * that builds Z itself for such a shape must use this order. */
int blindno_spectrum_tile_layout(int Bn, int C, int P1, int P2, int m2);

/* --- snapshot-encoder first layer with the lift folded in (NIOFP2D_FNO.FNO_input) ----------
 * The encoder input is cat(u_l, gx, gy) for snapshots u_l = X[b][idx[l]] of the bag tensor X
 * (B, T, N1, N2) (2d_FPE/NIOModules.py:548-560), lifted by fc0 (C x 3) and zero-padded to
 * P1 x P2 (2d_FPE/FNOModules.py:219-224).  These entry points read u straight from X through
 * the device index list idx (L int32) and never materialise the gathered bag, the input or x0. */

/* Row DFT of x0: At[n][k][c][h] = w0[c*3] U[n][k][h] + Gt[k][c][h] (n = b L + l), U the row
 * DFT of the zero-padded snapshot, Gt (m2, C, P1) complex the row DFT of the grid/bias part of x0
 * (x0 of an all-zero snapshot).  At as blindno_rowdft; Tp its B-operand image. */
int blindno_rowdft_bag_lift(const float* X, const int* idx, const float* w0, const float* Gt,
                            float* At, const float* Tp, int B, int T, int L, int N1, int N2,
                            int C, int P1, int P2, int m2, blindno_stream_t stream);
/* blindno_rowdft_bag_lift with the grid/bias spectrum formed in the kernel: Dg (m2, 3, P1)
 * complex holds the row spectra of the gx, gy and all-ones planes (zero past the N1 x N2 crop);
 * the grid/bias part is W0[c,1] Dg[.,0] + W0[c,2] Dg[.,1] + b0[c] Dg[.,2]. */
int blindno_rowdft_bag_lift_dg(const float* X, const int* idx, const float* w0, const float* b0,
                               const float* Dg, float* At, const float* Tp, int B, int T, int L,
                               int N1, int N2, int C, int P1, int P2, int m2,
                               blindno_stream_t stream);

/* blindno_rowidft_epi (act 0) with x = x0 recomputed from (X, idx, grid, w0, b0); C <= 4. */
int blindno_rowidft_epi_lift(const float* Z, const float* X, const int* idx, const float* grid,
                             const float* w0, const float* b0, const float* wc, const float* bc,
                             float* z, const float* tb, int B, int T, int L, int N1, int N2,
                             int C, int P1, int P2, int m2, blindno_stream_t stream);
/* blindno_rowidft_epi_lift + At = rowDFT(f(z)) for the second layer (f = GELU when act_next;
 * see blindno_rowidft_epi_rd). */
int blindno_rowidft_epi_lift_rd(const float* Z, const float* X, const int* idx, const float* grid,
                                const float* w0, const float* b0, const float* wc,
                                const float* bc, float* z, const float* tb, int B, int T, int L,
                                int N1, int N2, int C, int P1, int P2, int m2, float* At,
                                const float* Tp, int act_next, blindno_stream_t stream);

/* Adjoint of blindno_rowidft_epi_lift: dx0 = irow^H(G) + Wc^T dz is NOT written; the pass
 * reduces partial[blindno_rowidft_bwd_nchunk(B L, C, P1, P2, m2)][C*C + C + 4 C] =
 * [dWc | dbc | dW0 (C x 3) | db0 (C)] with dWc[o][i] = sum dz_o x0_i, dW0[c][j] = sum over the
 * N1 x N2 crop of dx0_c [u, gx, gy]_j, db0[c] = sum dx0_c.  C <= 4. */
int blindno_rowidft_bwd_lift(const float* G, const float* dz, const float* X, const int* idx,
                             const float* grid, const float* w0, const float* b0, const float* wc,
                             const float* tb, float* partial, int B, int T, int L, int N1, int N2,
                             int C, int P1, int P2, int m2, blindno_stream_t stream);

/* --- The column pass folded into the row kernels (FNO_input: C = 4, m1 = m2 = 12 -> K1 = 24
 *     kept rows; csrc/colspec.h).  Replaces blindno_colpass between the row kernels of
 *     SpectralConv2d.forward (2d_FPE/FNOModules.py:156-178) in the FNO_input layer chain
 *     (FNOModules.py:226-232): only the K1 x m2 column spectrum crosses kernels.
 * part: per (sample, 16-row block) column-DFT partials, blindno_colspec_nchunk(Cp, m2) chunks of
 *   64 lanes x 2 floats each (layout: colspec.h); tab: Tab[P1][2 K1] = (cos, sin)(2 pi r_j h / P1)
 *   (blindno.ops.twiddle_colspec); Y / Xsave (Bn, m2, C, K1) complex.
 * blindno_colspec_ok: 1 when a layer of this shape takes the folded path. */
int blindno_colspec_ok(int Bn, int C, int P1, int P2, int m1, int m2);
int blindno_colspec_nchunk(int C, int m2);
/* rows of the weight-gradient partials of blindno_rowidft_bwd_zc / _bwd_lift_zc */
int blindno_colspec_bwd_nchunk(int Bn, int P1);
/* row DFT of f(x) (GELU when act) on the N1v x N2v valid region + column-DFT partials */
int blindno_rowdft_cd(const float* x, float* part, const float* Tp, const float* tab, int Bn, int C,
                      int P1, int P2, int m2, int act, int N1v, int N2v, blindno_stream_t stream);
/* the same for the bag's snapshots X[b][idx[l]] (one channel; sample n = b L + l) */
int blindno_rowdft_bag_lift_cd(const float* X, const int* idx, float* part, const float* Tp,
                               const float* tab, int B, int T, int L, int N1, int N2, int P1,
                               int P2, int m2, blindno_stream_t stream);
/* blindno_rowdft_bag_lift_cd and blindno_pack_w2d_multi(w1s, w2s, Wts, shapes, npk) -- the
 * forward's spectral-weight pack, independent of it -- in one launch (bit-identical) */
int blindno_rowdft_bag_lift_cd_pack(const float* X, const int* idx, float* part, const float* Tp,
                                    const float* tab, int B, int T, int L, int N1, int N2, int P1,
                                    int P2, int m2, const void* const* w1s, const void* const* w2s,
                                    void* const* Wts, const int* shapes, int npk,
                                    blindno_stream_t stream);
/* partials of nbv blocks summed in block order -> Xsave (dir 0: X; dir 1: G = c_k/(P1 P2) X) and
 * Y (dir 0: c_k/(P1 P2) sum_c X W; dir 1: sum_o conj(W) G), as blindno_colpass forms them.
 * Lift (w0 != NULL, dir 0, Cp = 1): X[c] = w0[c,0] U + w0[c,1] Dg2[0] + w0[c,2] Dg2[1] +
 * b0[c] Dg2[2].  Wt NULL: Xsave only. */
int blindno_colmix(const float* part, int nbv, const float* Wt, float* Xsave, float* Y, int Bn, int C,
                   int Cp, int P1, int P2, int m1, int m2, int dir, const float* w0, const float* b0,
                   const float* Dg2, blindno_stream_t stream);
/* row inverses with Z built from Y (ZY) and, with part != NULL, the next row DFT as column-DFT
 * partials (CD): counterparts of blindno_rowidft_epi(_crop / _rd), _epi_lift_rd, _bwd_rd /
 * _bwd_crop and _bwd_lift.  Tp: the next row DFT's image (blindno_rowdft's). */
int blindno_rowidft_epi_zc(const float* Y, const float* x, const float* wc, const float* bc, float* z,
                           const float* tb, const float* tab, float* part, const float* Tp, int Bn,
                           int C, int P1, int P2, int m1, int m2, int act, int act_next, int oN1,
                           int oN2, blindno_stream_t stream);
int blindno_rowidft_epi_lift_zc(const float* Y, const float* X, const int* idx, const float* grid,
                                const float* w0, const float* b0, const float* wc, const float* bc,
                                float* z, const float* tb, const float* tab, float* part,
                                const float* Tp, int B, int T, int L, int N1, int N2, int C, int P1,
                                int P2, int m1, int m2, int act_next, blindno_stream_t stream);
int blindno_rowidft_bwd_zc(const float* Y, const float* dz, const float* wc, const float* xsrc,
                           float* dx, const float* tb, const float* tab, float* part,
                           const float* Tp, float* partial, int Bn, int C, int P1, int P2, int m1,
                           int m2, int act, int dN1, int dN2, blindno_stream_t stream);
/* the encoder's last layer with dz = lw_l ghat v formed on load (v from blindno_project_bag_fwd,
 * ghat (B, Ho Wo) the bag-level gradient, lw (U) or NULL for 1 / U; Bn = B U; the projection
 * backward then writes no dz): counterparts of blindno_rowdft_cd (crop Ho x Wo, act 0) and of
 * blindno_rowidft_bwd_zc with the weight-gradient and column-DFT partials */
int blindno_rowdft_cd_bag(const float* v, const float* ghat, const float* lw, int U, float* part,
                          const float* Tp, const float* tab, int Bn, int C, int P1, int P2, int m2,
                          int Ho, int Wo, blindno_stream_t stream);
int blindno_rowidft_bwd_zc_bag(const float* Y, const float* v, const float* ghat, const float* lw,
                               int U, const float* wc, const float* xsrc, float* dx, const float* tb,
                               const float* tab, float* part, const float* Tp, float* partial,
                               int Bn, int C, int P1, int P2, int m1, int m2, int act, int Ho, int Wo,
                               blindno_stream_t stream);
/* blindno_rowidft_bwd_lift_zc hosting up to two spectral weight gradients in the same launch
 * (the encoder's: both layers' Gs exist once this adjoint starts): job q as
 * blindno_mix_wgrad_multi's (mX, mG, mOut, mshp[7 q ..] = Bn, Ci, Co, K1, m2, nsplit, Gw),
 * with the grid of its own launch (bit-identical); nmj = 0: blindno_rowidft_bwd_lift_zc. */
int blindno_rowidft_bwd_lift_zc_mix(const float* Y, const float* dz, const float* X, const int* idx,
                                    const float* grid, const float* w0, const float* b0,
                                    const float* wc, const float* tb, const float* tab,
                                    float* partial, int B, int T, int L, int N1, int N2, int C,
                                    int P1, int P2, int m1, int m2, const void* const* mX,
                                    const void* const* mG, void* const* mOut, const int* mshp,
                                    int nmj, blindno_stream_t stream);
int blindno_rowidft_bwd_lift_zc(const float* Y, const float* dz, const float* X, const int* idx,
                                const float* grid, const float* w0, const float* b0,
                                const float* wc, const float* tb, const float* tab, float* partial,
                                int B, int T, int L, int N1, int N2, int C, int P1, int P2, int m1,
                                int m2, blindno_stream_t stream);

/* 1x1-conv weight/bias gradient partials (for C > 8): partial[nchunk][C*C + C] with
 * dWc[o,i] = sum dz[n,o,.] f(x[n,i,.]),  dbc[o] = sum dz[n,o,.];
 * nchunk must equal blindno_conv_wgrad_nchunk(Bn, P1, P2). */
int blindno_conv_wgrad(const float* dz, const float* x, float* partial, int nchunk, int Bn,
                       int C, int P1, int P2, int act, blindno_stream_t stream);
int blindno_conv_wgrad_nchunk(int Bn, int P1, int P2);

/* out[p] = sum_{c < nchunk} partial[c][p] (fixed order: deterministic). */
int blindno_reduce_partials(const float* partial, float* out, int nchunk, int np,
                            blindno_stream_t stream);

/* Several reductions in one launch: segment i is blindno_reduce_partials(partials[i], outs[i],
 * nchunks[i], nps[i]) (bit-identical results); the deferred weight-gradient reductions of one
 * backward pass (blindno.ops.deferred_reductions). */
int blindno_reduce_partials_multi(const void* const* partials, void* const* outs,
                                  const int* nchunks, const int* nps, int nseg,
                                  blindno_stream_t stream);
/* The same with pieces: segment i stores only parameters [e0s[i], e1s[i]) of its reduction, at
 * outs[i][p - e0s[i]] (each summed exactly as in the whole reduction), so the parameter
 * gradients of one reduction can land straight in an optimizer's flat gradient buffer
 * (blindno.ops._Deferred.redirect).  e0s / e1s NULL: whole reductions. */
int blindno_reduce_partials_pieces(const void* const* partials, void* const* outs,
                                   const int* nchunks, const int* nps, const int* e0s,
                                   const int* e1s, int nseg, blindno_stream_t stream);
/* ... where a whole segment i with upks[i] = u >= 0 is a packed spectral weight gradient
 * (m2, 2 m1, Ci, Co) complex stored unpacked into the weights1 / weights2 gradient layouts
 * ud[2 u], ud[2 u + 1] with ushp[4 u ..] = (Ci, Co, m1, m2) (the unpack folded into the
 * reduction; at most 8 per launch of 48 segments). */
int blindno_reduce_partials_pieces_u(const void* const* partials, void* const* outs,
                                     const int* nchunks, const int* nps, const int* e0s,
                                     const int* e1s, const int* upks, void* const* ud,
                                     const int* ushp, int nseg, blindno_stream_t stream);
/* The deferred finalisation in one launch: blindno_reduce_partials_pieces_u(...) and
 * blindno_unpack_w2d_multi(dWts, dw1s, dw2s, shapes, nunp) together (independent work;
 * bit-identical results); two launches when the segments do not fit one table. */
int blindno_finish_multi(const void* const* partials, void* const* outs, const int* nchunks,
                         const int* nps, const int* e0s, const int* e1s, const int* upks,
                         void* const* ud, const int* ushp, int nseg, const void* const* dWts,
                         void* const* dw1s, void* const* dw2s, const int* shapes, int nunp,
                         blindno_stream_t stream);

/* Pack reference-layout 2D weights (Ci,Co,m1,m2,2) x2 into Wt (m2,K1,Ci,Co) complex. */
int blindno_pack_w2d(const float* w1, const float* w2, float* Wt, int Ci, int Co, int m1,
                     int m2, int P1, blindno_stream_t stream);
/* Scatter dWt back to dW1/dW2 (Ci,Co,m1,m2,2); entries of weights1 shadowed by
 * weights2 (overlapping rows) receive 0. */
int blindno_unpack_w2d(const float* dWt, float* dw1, float* dw2, int Ci, int Co, int m1,
                       int m2, int P1, blindno_stream_t stream);
/* The same for two weight sets in one launch (the two heads): Wt (2, m2, K1, Ci, Co) complex. */
int blindno_pack_w2d_2(const float* w1a, const float* w2a, const float* w1b, const float* w2b,
                       float* Wt, int Ci, int Co, int m1, int m2, int P1, blindno_stream_t stream);
int blindno_unpack_w2d_2(const float* dWt, float* dw1a, float* dw2a, float* dw1b, float* dw2b,
                         int Ci, int Co, int m1, int m2, int P1, blindno_stream_t stream);
/* Several blindno_unpack_w2d in one launch: segment i unpacks dWts[i] into dw1s[i], dw2s[i]
 * with shape shapes[5 i .. 5 i + 4] = (Ci, Co, m1, m2, P1). */
int blindno_unpack_w2d_multi(const void* const* dWts, void* const* dw1s, void* const* dw2s,
                             const int* shapes, int nseg, blindno_stream_t stream);
/* Several blindno_pack_w2d in one launch: segment i packs (w1s[i], w2s[i]) into Wts[i] with
 * shape shapes[5 i .. 5 i + 4] = (Ci, Co, m1, m2, P1). */
int blindno_pack_w2d_multi(const void* const* w1s, const void* const* w2s, void* const* Wts,
                           const int* shapes, int nseg, blindno_stream_t stream);
/* 1D: (Ci,Co,m) complex <-> Wt (m,Ci,Co) complex; dir 0 pack, 1 unpack. */
int blindno_pack_w1d(const float* w, float* Wt, int Ci, int Co, int m, int dir,
                     blindno_stream_t stream);

/* --- snapshot-bag aggregation (2d_FPE/NIOModules.py:565-575; 1d_FPE/NIOModules.py:140-149) */

/* y[b,s,c] = sum_{e<d} W[c,e] grid[s,e] + (W[c,d]/L) sum_l u[b,l,s] + bias[c]
 * u (B, L, S), grid (S, d) channels-last, W (width, d+1), y (B, S, width). */
int blindno_bagmean_fwd(const float* u, const float* grid, const float* w, const float* bias,
                        float* y, int B, int L, int S, int d, int width,
                        blindno_stream_t stream);
/* As blindno_bagmean_fwd with per-snapshot weights lw (L) replacing 1/L: the bag of a step
 * given as its unique snapshots with multiplicities, lw[l] = count_l / L_drawn. */
int blindno_bagmean_fwd_w(const float* u, const float* grid, const float* w, const float* bias,
                          const float* lw, float* y, int B, int L, int S, int d, int width,
                          blindno_stream_t stream);
/* s[b,s] = sum_c (W[c,d]/L) dy[b,s,c]   (the gradient of every u[b,l,s]). */
int blindno_bagmean_bwd(const float* dy, const float* w, float* s, int B, int S, int d,
                        int width, int L, blindno_stream_t stream);

/* --- DeepONet combiner fused with the bag mean (NIO models): replaces
 *     DeepOnetNoBiasOrg.forward, 2d_FPE/DeepONetModules.py:142-151, whose (B, L, S) output the
 *     bag mean of 2d_FPE/NIOModules.py:66-77 (NC :65-76, 1d_FPE/NIOModules.py:62-77) reads only
 *     through its mean over the bag ---------------------------------------------------------
 * w (B, L, P) branch coefficients, basis (S, P) trunk output, b0 (1) device scalar, lw (L)
 * optional per-snapshot weights (NULL: 1/L).  Forward:
 *   wbar[b,k] = sum_l lw_l w[b,l,k];  ubar[b,p] = (wbar[b] . basis[p] + b0 sum_l lw_l) * scale
 * (scale = 1/sqrt(P)); wbar (B, P) is saved for the backward.  Backward from g = dL/dubar
 * (B, S): dw (B, L, P), dbasis (S, P), db0 (1, NULL: none); partial: nblk * (B P + 1) floats,
 * nblk = blindno_deeponet_bag_nblk(S).  P <= 64; any B (the backward runs bag chunks of 64
 * in stream order, dbasis / db0 summed over the chunks in that order). */
int blindno_deeponet_bag_nblk(int S);
int blindno_deeponet_bag_fwd(const float* w, const float* basis, const float* b0, const float* lw,
                             float* wbar, float* ubar, int B, int L, int S, int P, float scale,
                             blindno_stream_t stream);
int blindno_deeponet_bag_bwd(const float* g, const float* basis, const float* wbar, const float* lw,
                             float* dw, float* dbasis, float* db0, float* partial, int nblk, int B,
                             int L, int S, int P, float scale, blindno_stream_t stream);

/* --- token self-attention over the bag (NIOFP2D_FNO_attn, 2d_FPE/NIOModules.py:365-399;
 *     2d_Non_conservative_FPE/NIOModules.py:364-398) ------------------------------------
 * Tokens X[b] = [gx, gy, u_1..u_L] (T = L + 2 <= 256 rows of S points); grid (S, 2)
 * channels-last, u (B, L, S), fc0 weight w (width) and bias (width), y (B, S, width).
 * Forward: A = softmax(X X^T / sqrt(S)) (B,T,T), c = column sums of A (B,T),
 * y[b,p,:] = w (1/T) sum_s c_s X[s,p] + bias  (= the reference's (A X)^T w / T + bias).
 * partial: caller scratch of B * nchunk * T * T floats, nchunk = blindno_bagattn_nchunk(S). */
int blindno_bagattn_nchunk(int S);
int blindno_bagattn_fwd(const float* grid, const float* u, const float* w, const float* bias,
                        float* partial, float* A, float* cs, float* y, int B, int L, int S,
                        int width, blindno_stream_t stream);
/* Backward from dy (B,S,width) and the forward's A, cs: du (B,L,S) and, if dgt is non-NULL,
 * the grid tokens' gradient dgt (B,2,S).  Scratch: partial B*nchunk*T, dm B*S, M B*T*T. */
int blindno_bagattn_bwd(const float* grid, const float* u, const float* dy, const float* w,
                        const float* A, const float* cs, float* partial, float* dm, float* M,
                        float* du, float* dgt, int B, int L, int S, int width,
                        blindno_stream_t stream);

/* --- loss / metrics / optimiser -------------------------------------------------------- */

/* nn.MSELoss (2d_FPE/train_fno.py:116,142): partial sums of (p-t)^2 per block into
 * partial[nblk] and grad = gscale * 2 (p - t) / n (grad may be NULL). */
int blindno_mse(const float* p, const float* t, float* partial, float* grad, int64_t n,
                int nblk, const float* gscale, blindno_stream_t stream);
/* loss[0] = (sum_{b < nblk} partial[b]) / n, fixed order (the forward scalar of MSELoss from
 * blindno_mse's per-block partials). */
int blindno_mse_finish(const float* partial, int nblk, int64_t n, float* loss,
                       blindno_stream_t stream);
/* blindno_mse_finish that also adds the loss to *acc (a training loop's running loss sum, one
 * launch instead of a separate add); acc may be NULL. */
int blindno_mse_finish_acc(const float* partial, int nblk, int64_t n, float* loss, float* acc,
                           blindno_stream_t stream);
/* blindno_mse + blindno_mse_finish_acc in ONE launch (bit-identical): the workgroup that
 * finishes last sums the partials.  counter: one unsigned in device memory, zero before the
 * first call; every call leaves it zero again.  grad (may be NULL): blindno_mse's gradient for
 * gscale = 1 (a backward seeded with exactly 1 then needs no launch of its own). */
int blindno_mse_fwd(const float* p, const float* t, float* partial, int64_t n, int nblk,
                    float* loss, float* acc, unsigned* counter, float* grad,
                    blindno_stream_t stream);

/* Per-row sums of squares in fp64 for relative-L2 metrics (2d_FPE/train_fno.py:160-163,
 * eval_fno.py:124-128, 2d_Non_conservative_FPE/compute_time_error.py:321-333).
 * Row r holds n points of `stride` floats: out[2r] = sum (a[.+off_a] - b[.+off_b])^2,
 * out[2r+1] = sum b[.+off_b]^2, or (den_all = 1) the sum over all `stride` channels of b
 * (the train loop's denominator quirk). */
int blindno_rowsq(const float* a, const float* b, double* out, int rows, int n, int stride,
                  int off_a, int off_b, int den_all, blindno_stream_t stream);

/* Fused Adam over a flat fp32 buffer (torch.optim.Adam, no weight decay / amsgrad):
 * step_size = lr / (1 - beta1^t), bc2s = sqrt(1 - beta2^t). grad is scaled by gscale. */
/* Gather nseg gradient segments into one flat buffer: dst[offs[i] + j] = srcs[i][j], j < ns[i].
 * srcs / offs / ns are HOST arrays (device pointers inside srcs), copied into the kernel
 * arguments, so a HIP-graph capture keeps them.  Replaces FlatAdam's per-parameter gradient
 * copy (the reference's DDP bucket flatten, 2d_FPE/train_fno.py:121,143). */
int blindno_gather_flat(const void* const* srcs, const int64_t* offs, const int64_t* ns, int nseg,
                        float* dst, blindno_stream_t stream);
/* Batch select: dsts[i][b] = srcs[i][ids[b]] (rows of rows[i] floats) for nseg <= 4 tensors in
 * one launch; srcs / dsts / rows / nsrc (row count of each source) are HOST arrays, ids a DEVICE
 * int64 array of B row indices (bench.py: the bags X and targets Y of the step's batch).  An id
 * outside [0, nsrc[i]) fills its batch row of dsts[i] with NaN (no out-of-bounds read). */
int blindno_gather_batch(const void* const* srcs, void* const* dsts, const int64_t* rows,
                         const int64_t* nsrc, int nseg, const int64_t* ids, int B,
                         blindno_stream_t stream);
int blindno_adam(float* p, const float* g, float* m, float* v, int64_t n, float beta1,
                 float beta2, float eps, float step_size, float bc2s, float gscale,
                 blindno_stream_t stream);

/* --- density evaluators (fp64) ----------------------------------------------------------- */

/* Batched 1D GPE split-step pseudo-spectral solver, one workgroup per trajectory
 * (solve_GPE_custom, 1d_GPE/datagen_GPE.py:86-115; steps :29-81).  psi0 (Nx complex, or
 * B x Nx when psi0_batched), V (B, Nx), g/kappa (B); order 2 = Strang, 4 = Yoshida;
 * k = 2 pi fftfreq(Nx, dx).  Records psi at steps n = 0, rec_every, 2 rec_every, ... (n <=
 * nsteps): rec_abs (B, nrec, Nx) |psi| and/or rec_psi (B, nrec, Nx) complex, nrec =
 * nsteps/rec_every + 1 (either may be NULL); psi_out (B, Nx) complex final state (may be
 * NULL).  Nx must be a power of two <= 2048. */
int blindno_gpe_solve(const double* psi0, const double* V, const double* g, const double* kappa,
                      double dx, double dt, int nsteps, int order, int rec_every, double* rec_abs,
                      double* rec_psi, double* psi_out, int B, int Nx, int psi0_batched,
                      blindno_stream_t stream);

/* Trapezoid-rule spatial integrals of time_averaged_L2_error (1d_FPE/compute_time_error.py:
 * 268-275): out[2r] = trapz((a_r - b_r)^2, x), out[2r+1] = trapz(b_r^2, x), rows of n. */
int blindno_trapz_rows(const double* a, const double* b, const double* x, double* out, int rows,
                       int n, blindno_stream_t stream);

/* Batched FPE master-equation propagation (fplanck fokker_planck.propagate_interval, used by
 * 1d_FPE/compute_time_error.py:215-238 and 2d_Non_conservative_FPE/compute_time_error.py:
 * 300-319; fplanck is not shipped: restated, parity unpinned).  One workgroup per trajectory,
 * fp64, N = nx*ny <= 8192 cells (1D: ny = 1), cell i = ix*ny + iy.  coef (B, 5, N) =
 * [diag, cxm, cxp, cym, cyp]: (M p)_i = cxm_i p_{i-ex} + cxp_i p_{i+ex} + cym_i p_{i-ey} +
 * cyp_i p_{i+ey} - diag_i p_i (neighbour indices wrap; zero coefficients make a wall).
 * out (B, nout, N): p at t = o*dt_out, o < nout, out[:,0] = p0.  Each interval is
 * `substeps` steps of the degree-`degree` Taylor polynomial of exp(dt_out/substeps M). */
int blindno_fp_propagate(const double* p0, const double* coef, double* out, int B, int nx,
                         int ny, int nout, int substeps, int degree, double dt_out,
                         blindno_stream_t stream);

/* ---- grouped launches: two FNO heads over one field in one chain (ops.HeadPairFn) ----------
 * G weight groups over consecutive blocks of Bg = Bn/G samples.  Group g's small weights (fc0,
 * 1x1 convs, fc1/fc2 -- packed per head in one buffer) are read at + g*wgs floats from the
 * given pointers, its packed spectral weights at Wt + g*wtgs floats.  Semantics otherwise as
 * the ungrouped entry points above (which are these with G = 1), plus:
 *  lift_fwd_g:    the input holds Bg samples shared by every group (x0 sample g Bg + n reads
 *                 in[n]);
 *  lift_bwd_g:    d_in (Bg samples) sums all groups' contributions; partial[nchunk][G][np],
 *                 nchunk = blindno_lift_bwd_nchunk(Bg, N1, N2);
 *  project_fwd_g: sample g Bg + n writes output sample n at channel offset ooff + g*Cout
 *                 (matrix-core path only: Hd 128, C <= 15, Cout <= 2);
 *  project_bwd_g: dout addressed like project_fwd_g's output; partial[nchunk][G][np] with
 *                 nchunk = blindno_project_bwd_nchunk(Bg, Ho, Wo);
 *  conv_wgrad_g:  partial[nchunk][G][np], nchunk = blindno_conv_wgrad_nchunk(Bg, P1, P2);
 *  mix_wgrad_g:   dWt (G, m2, K1, Ci, Co) complex, nsplit = blindno_mix_wgrad_nsplit(Bg, ...),
 *                 partial nsplit x G x 2 m2 K1 Ci Co floats. */
int blindno_lift_fwd_g(const float* in, const float* w0, const float* b0, float* x0, int G,
                       int64_t wgs, int Bn, int N1, int N2, int Cin, int C, int P1, int P2,
                       blindno_stream_t stream);
int blindno_lift_bwd_g(const float* dx0, const float* in, const float* w0, float* d_in,
                       float* partial, int nchunk, int G, int64_t wgs, int Bn, int N1, int N2,
                       int Cin, int C, int P1, int P2, blindno_stream_t stream);
/* lift_bwd_g with, when Xs != NULL, the spectral weight gradient mix_wgrad_g(Xs, Gs) -> dWt of
 * the heads' first layer (Ci = Co = C, Bn samples) in the same launch (mnsplit =
 * blindno_mix_wgrad_nsplit(Bn / G, ...); mpartial as mix_wgrad_g's). */
/* The heads' lift on the bag mean's input formed on the fly (NIOFP2D_FNO: h = fc0([grid,
 * ubar]) with fc0 = (bw (width, 3): gx, gy, u columns; bb), 2d_FPE/NIOModules.py:569-575):
 * with ubar != NULL the lift reads ubar (B, N1 N2) and grid (N1 N2, 2) instead of in (Cin =
 * width = 12), forming h exactly as blindno_bagmean_fwd_w with L = 1 and u scale invL; the
 * adjoint writes d ubar (B, N1 N2) = blindno_bagmean_bwd's reduction (its 1 / L = invLb) into
 * d_in instead of d h, and reduces fc0-of-the-heads' gradient against the same on-the-fly h.
 * The bag-mean launches and the h field go.  ubar NULL: lift_fwd_g / lift_bwd_mix_g. */
int blindno_lift_bag_ok(int G, int Bn, int N1, int N2, int Cin, int C, int P1, int P2);
int blindno_lift_fwd_bag_g(const float* in, const float* w0, const float* b0, float* x0, int G,
                           int64_t wgs, int Bn, int N1, int N2, int Cin, int C, int P1, int P2,
                           const float* ubar, const float* grid, const float* bw, const float* bb,
                           float invL, blindno_stream_t stream);
int blindno_lift_bwd_bag_mix_g(const float* dx0, const float* in, const float* w0, float* d_in,
                               float* partial, int nchunk, int G, int64_t wgs, int Bn, int N1,
                               int N2, int Cin, int C, int P1, int P2, const float* Xs,
                               const float* Gs, float* dWt, float* mpartial, int mnsplit, int K1,
                               int m2, const float* ubar, const float* grid, const float* bw,
                               const float* bb, float invL, float invLb, blindno_stream_t stream);
int blindno_lift_bwd_mix_g(const float* dx0, const float* in, const float* w0, float* d_in,
                           float* partial, int nchunk, int G, int64_t wgs, int Bn, int N1, int N2,
                           int Cin, int C, int P1, int P2, const float* Xs, const float* Gs,
                           float* dWt, float* mpartial, int mnsplit, int K1, int m2,
                           blindno_stream_t stream);
int blindno_project_fwd_g(const float* z, const float* w1, const float* b1, const float* w2,
                          const float* b2, float* out, int G, int64_t wgs, int Bn, int C, int P1,
                          int P2, int Ho, int Wo, int Hd, int Cout, int ostride, int ooff,
                          blindno_stream_t stream);
int blindno_project_bwd_g(const float* z, const float* w1, const float* b1, const float* w2,
                          const float* dout, float* dz, float* partial, int nchunk, int G,
                          int64_t wgs, int Bn, int C, int P1, int P2, int Ho, int Wo, int Hd,
                          int Cout, int ostride, int ooff, blindno_stream_t stream);
int blindno_colpass_g(const float* At, const float* Wt, float* Xs, float* Y, float* Z,
                      const float* FB, const float* GB, int G, int64_t wtgs, int Bn, int Ci,
                      int Co, int P1, int m1, int m2, int P2, int dir, blindno_stream_t stream);
int blindno_mix_wgrad_g(const float* X, const float* Gs, float* dWt, float* partial, int nsplit,
                        int G, int Bn, int Ci, int Co, int K1, int m2, blindno_stream_t stream);
int blindno_rowidft_epi_g(const float* Z, const float* x, const float* wc, const float* bc,
                          float* z, const float* tb, int G, int64_t wgs, int Bn, int C, int P1,
                          int P2, int m2, int act, blindno_stream_t stream);
int blindno_rowidft_bwd_g(const float* Gs, const float* dz, const float* wc, const float* xsrc,
                          float* dx, const float* tb, int G, int64_t wgs, int Bn, int C, int P1,
                          int P2, int m2, int act, blindno_stream_t stream);
int blindno_conv_wgrad_g(const float* dz, const float* x, float* partial, int nchunk, int G,
                         int Bn, int C, int P1, int P2, int act, blindno_stream_t stream);
/* One layer of the grouped heads' backward in a single launch (the adjoint of FNOModules.py:
 * 226-232 per layer; three independent, latency-bound steps at the heads' size):
 *   At = blindno_rowdft(dz, act 0), the conv_wgrad_g partials of (dz, GELU^act(src)) and, when
 *   Xs != NULL, mix_wgrad_g(Xs, Gs) -> dWt (the layer processed before, Ci = Co = C), all with
 *   the grids of their own launches (bit-identical results).  cnchunk =
 *   blindno_conv_wgrad_nchunk(Bn / G, P1, P2), mnsplit = blindno_mix_wgrad_nsplit(Bn / G, ...).
 *   Shapes: blindno_rowdft_wgrad_ok (the conv gradient's matrix-core form, 5 <= C <= 15). */
int blindno_rowdft_wgrad_ok(int Bn, int C, int P1, int P2, int m2);
int blindno_rowdft_wgrad_g(const float* dz, const float* src, float* At, const float* Tp,
                           float* cpartial, int cnchunk, int act, const float* Xs,
                           const float* Gs, float* dWt, float* mpartial, int mnsplit, int K1,
                           int G, int Bn, int C, int P1, int P2, int m2, blindno_stream_t stream);

/* ---- NIO encoder ConvBlock normalisation: BatchNorm2d fused with LeakyReLU
 * (2d_FPE/Baselines.py:40-52 ConvBlock = Conv -> BatchNorm2d -> LeakyReLU(slope); replaces the
 * nn.BatchNorm2d + nn.LeakyReLU(inplace) pair of each block).  z (Npad, C, HW) NCHW, batch =
 * rows [0, N); rows [N, Npad) of y / dz are written 0.  training != 0: batch statistics
 * (biased variance), running_mean/var updated with momentum (unbiased variance) when non-NULL;
 * training == 0: running statistics.  save (C, 4) = mean, invstd, gamma invstd, beta
 * (y = act(gamma invstd (z - mean) + beta); written by the forward, read by the backward).
 * partial: 8-B aligned scratch of C * blindno_bn_act_nslices(N, C, HW) * 4 floats (2 fp64 sums
 * per slice: the statistics accumulate in fp64); coef (C, 3) scratch of the backward.
 * gamma/beta may be NULL (affine=False); dgamma/dbeta may be NULL. */
int blindno_bn_act_nslices(int N, int C, int HW);
int blindno_bn_act_fwd(const float* z, const float* gamma, const float* beta, float* run_mean,
                       float* run_var, float* y, float* save, float* partial, int N, int Npad,
                       int C, int HW, float eps, float momentum, float slope, int training,
                       blindno_stream_t stream);
int blindno_bn_act_bwd(const float* dy, const float* z, const float* gamma, const float* save,
                       float* dz, float* dgamma, float* dbeta, float* partial, float* coef, int N,
                       int Npad, int C, int HW, float slope, int training, blindno_stream_t stream);

/* ---- NIO encoder convolutions: nn.Conv2d (bias, groups 1, any kernel / stride / zero padding)
 * of the ConvBlocks (2d_FPE/Baselines.py:40-52; Encoder2D :186-249 and the 1D Encoder
 * :254-287, whose (1, k) kernels are 2D convolutions of height 1), replacing the MIOpen calls
 * of torch.nn.Conv2d.  NCHW fp32; Ho = (Hi + 2 ph - KH) / sh + 1, Wo likewise.  Implicit GEMMs
 * on the fp32 matrix cores with a fixed accumulation order (deterministic).
 *   fwd:        y (N, Co, Ho, Wo) = conv(x (N, Ci, Hi, Wi), w (Co, Ci, KH, KW)) + b (b may be NULL)
 *   bwd_data:   dx (N, Ci, Hi, Wi) = conv^T(dy, w)
 *   bwd_weight: dwb (Co, Ci KH KW + 1): columns [0, Ci KH KW) = dW, last column = db; partial:
 *               scratch of nsplit * Co * (Ci KH KW + 1) floats (nsplit from
 *               blindno_conv2d_wgrad_nsplit; NULL allowed when it is 1). */
int blindno_conv2d_fwd(const float* x, const float* w, const float* b, float* y, int N, int Ci,
                       int Hi, int Wi, int Co, int KH, int KW, int sh, int sw, int ph, int pw,
                       blindno_stream_t stream);
int blindno_conv2d_bwd_data(const float* dy, const float* w, float* dx, int N, int Ci, int Hi,
                            int Wi, int Co, int KH, int KW, int sh, int sw, int ph, int pw,
                            blindno_stream_t stream);
int blindno_conv2d_wgrad_nsplit(int N, int Ci, int Hi, int Wi, int Co, int KH, int KW, int sh,
                                int sw, int ph, int pw);
int blindno_conv2d_bwd_weight(const float* dy, const float* x, float* dwb, float* partial,
                              int nsplit, int N, int Ci, int Hi, int Wi, int Co, int KH, int KW,
                              int sh, int sw, int ph, int pw, blindno_stream_t stream);
/* Split-K / re-laid-out-weight forms of fwd / bwd_data.  K is cut into nsplit ranges whose
 * partial outputs (partial: nsplit * |y| or nsplit * |dx| floats) are summed in split order
 * (deterministic) -- for the layers whose output leaves the chip short of workgroups (the
 * encoder's last blocks); nsplit from the *_nsplit queries (1: no partial scratch, the same
 * result as the plain entries; any nsplit >= 1 is valid).  wscratch (may be NULL):
 * blindno_conv2d_wscratch_floats(mode 0 = fwd | 1 = bwd_data, ...) floats, where the weights
 * are re-laid out tap-major first so the GEMM's weight loads are contiguous (0 floats: not
 * used for this layer).  The result does not depend on wscratch. */
int blindno_conv2d_fwd_nsplit(int N, int Ci, int Hi, int Wi, int Co, int KH, int KW, int sh,
                              int sw, int ph, int pw);
int blindno_conv2d_bwd_data_nsplit(int N, int Ci, int Hi, int Wi, int Co, int KH, int KW, int sh,
                                   int sw, int ph, int pw);
int blindno_conv2d_wscratch_floats(int mode, int N, int Ci, int Hi, int Wi, int Co, int KH, int KW,
                                   int sh, int sw, int ph, int pw);
int blindno_conv2d_fwd_split(const float* x, const float* w, const float* b, float* y,
                             float* partial, int nsplit, float* wscratch, int N, int Ci, int Hi,
                             int Wi, int Co, int KH, int KW, int sh, int sw, int ph, int pw,
                             blindno_stream_t stream);
int blindno_conv2d_bwd_data_split(const float* dy, const float* w, float* dx, float* partial,
                                  int nsplit, float* wscratch, int N, int Ci, int Hi, int Wi,
                                  int Co, int KH, int KW, int sh, int sw, int ph, int pw,
                                  blindno_stream_t stream);

/* ---- whole-op spectral convolutions for C / C++ hosts (no Python needed) ---------------
 * SpectralConv2d.forward / backward (2d_FPE/FNOModules.py:156-178: rfft2 -> corner mix with
 * weights1/weights2 -> irfft2) and SpectralConv1d (1d_FPE/FNOModules.py:47-59, DC bin x0.5)
 * as ONE call each, over the stage kernels above.  The library never allocates: the caller
 * owns
 *   tables: twiddle images of one shape, blindno_spectral{2,1}d_tables_bytes bytes, filled once
 *           by blindno_spectral{2,1}d_tables_init (host-built in double, blocking copy);
 *   work:   scratch, blindno_spectral_conv{2,1}d_workspace_bytes(..., bwd) bytes;
 *   saved:  the forward's spectrum, read by the backward (..._saved_bytes).
 * Shapes: x (Bn, Ci, P1, P2) / (Bn, Ci, P2); w1, w2 (Ci, Co, m1, m2, 2) real view; 1D w
 * (Ci, Co, m) complex64 interleaved; y (Bn, Co, P1, P2) / (Bn, Co, P2).  Ci, Co <= 32,
 * m2 <= min(48, P2/2 + 1).  Backward: dx may be NULL (no input gradient).  Byte queries
 * return -1 on an invalid shape. */
int64_t blindno_spectral2d_tables_bytes(int P1, int P2, int m1, int m2);
int blindno_spectral2d_tables_init(void* tables, int P1, int P2, int m1, int m2);
int64_t blindno_spectral_conv2d_workspace_bytes(int Bn, int Ci, int Co, int P1, int P2, int m1,
                                                int m2, int bwd);
int64_t blindno_spectral_conv2d_saved_bytes(int Bn, int Ci, int P1, int m1, int m2);
int blindno_spectral_conv2d_fwd(const float* x, const float* w1, const float* w2, float* y,
                                float* saved, void* work, const void* tables, int Bn, int Ci,
                                int Co, int P1, int P2, int m1, int m2, blindno_stream_t stream);
int blindno_spectral_conv2d_bwd(const float* dy, const float* saved, const float* w1,
                                const float* w2, float* dx, float* dw1, float* dw2, void* work,
                                const void* tables, int Bn, int Ci, int Co, int P1, int P2,
                                int m1, int m2, blindno_stream_t stream);
int64_t blindno_spectral1d_tables_bytes(int P2, int m);
int blindno_spectral1d_tables_init(void* tables, int P2, int m);
int64_t blindno_spectral_conv1d_workspace_bytes(int Bn, int Ci, int Co, int P2, int m, int bwd);
int64_t blindno_spectral_conv1d_saved_bytes(int Bn, int Ci, int m);
int blindno_spectral_conv1d_fwd(const float* x, const float* w, float* y, float* saved,
                                void* work, const void* tables, int Bn, int Ci, int Co, int P2,
                                int m, blindno_stream_t stream);
int blindno_spectral_conv1d_bwd(const float* dy, const float* saved, const float* w, float* dx,
                                float* dw, void* work, const void* tables, int Bn, int Ci,
                                int Co, int P2, int m, blindno_stream_t stream);

/* ---- permutation-invariant attention UNet, PermInvUNet_attn ("BlinDNO")
 * 2d_FPE/NIOModules.py:1044-1181 (2D), 1d_FPE/NIOModules.py:165-443 (1D: height-1 fields,
 * KH = 1).  The 3x3 convolutions and the 1x1 final_conv use blindno_conv2d_*, the skip
 * BatchNorms (and the NC copy's ConvBlock BN + ReLU) blindno_bn_act_* (slope 1 / 0).
 *
 * Depthwise convolution of ConvNeXtBlock (nn.Conv2d(C, C, 7, padding=3, groups=C), :1047;
 * Conv1d(C, C, 7, padding=3, groups=C), 1d_FPE/NIOModules.py:167): x, y (N, C, H, W), w (C, KH, KW),
 * padding (KH/2, KW/2), KH KW <= 49.  bwd_weight: dwb (C, KH KW + 1), last column = db; partial:
 * nsplit x C x (KH KW + 1) floats (nsplit = blindno_dwconv_wgrad_nsplit; NULL when 1). */
int blindno_dwconv_fwd(const float* x, const float* w, const float* b, float* y, int N, int C,
                       int H, int W, int KH, int KW, blindno_stream_t stream);
int blindno_dwconv_bwd_data(const float* dy, const float* w, float* dx, int N, int C, int H,
                            int W, int KH, int KW, blindno_stream_t stream);
int blindno_dwconv_wgrad_nsplit(int N, int C, int H, int W);
int blindno_dwconv_bwd_weight(const float* dy, const float* x, float* dwb, float* partial,
                              int nsplit, int N, int C, int H, int W, int KH, int KW,
                              blindno_stream_t stream);
/* Rest of ConvNeXtBlock.forward (2d_FPE/NIOModules.py:1053-1062): per pixel of xd (the depthwise
 * output, (N, C, HW)) LayerNorm over C (eps 1e-6, gamma lw / beta lb) -> Linear(C, 4C) (w1, b1)
 * -> exact GELU -> Linear(4C, C) (w2, b2) -> + sc (the shortcut).  C in {1,2,4,...,64}.
 * bwd: dxd = gradient at xd (the shortcut's is dy itself); dparams = [dw1 (4C x C) | db1 (4C) |
 * dw2 (C x 4C) | db2 (C) | dlw (C) | dlb (C)]; partial: nblk x (8 C^2 + 7 C) floats,
 * nblk = blindno_cnx_pw_bwd_nblk(N, C, HW). */
int blindno_cnx_pw_fwd(const float* xd, const float* sc, const float* lw, const float* lb,
                       const float* w1, const float* b1, const float* w2, const float* b2, float* y,
                       int N, int C, int HW, blindno_stream_t stream);
int blindno_cnx_pw_bwd_nblk(int N, int C, int HW);
int blindno_cnx_pw_bwd(const float* dy, const float* xd, const float* lw, const float* lb,
                       const float* w1, const float* b1, const float* w2, float* dxd,
                       float* dparams, float* partial, int nblk, int N, int C, int HW,
                       blindno_stream_t stream);
/* MaxPool2d(2) / MaxPool1d(2) (:1115, 1d :239): window = stride = KH x KW, floor; arg (NC, Ho, Wo)
 * uint8 index of the window's maximum (first in scan order; a NaN wins). */
int blindno_maxpool_fwd(const float* x, float* y, uint8_t* arg, int NC, int H, int W, int KH,
                        int KW, blindno_stream_t stream);
int blindno_maxpool_bwd(const float* dy, const uint8_t* arg, float* dx, int NC, int H, int W,
                        int KH, int KW, blindno_stream_t stream);
/* ConvTranspose2d(Ci, Co, kernel = stride = 2, output_padding) of the up path (:1130-1134;
 * 1d :258-261 with KH = 1): x (N, Ci, Hi, Wi), w (Ci, Co, KH, KW), y (N, Co, Ho, Wo) with
 * KH Hi <= Ho < KH (Hi + 1) (the extra rows / columns are output_padding).  bwd_weight:
 * dwb = [dW (Ci Co KH KW) | db (Co)], partial blindno_convt_wgrad_nparts(N, Hi, Wi) x
 * (Ci Co KH KW + Co) floats. */
int blindno_convt_fwd(const float* x, const float* w, const float* b, float* y, int N, int Ci,
                      int Hi, int Wi, int Co, int KH, int KW, int Ho, int Wo,
                      blindno_stream_t stream);
int blindno_convt_bwd_data(const float* dy, const float* w, float* dx, int N, int Ci, int Hi,
                           int Wi, int Co, int KH, int KW, int Ho, int Wo, blindno_stream_t stream);
int blindno_convt_wgrad_nparts(int N, int Hi, int Wi);
int blindno_convt_bwd_weight(const float* dy, const float* x, float* dwb, float* partial, int N,
                             int Ci, int Hi, int Wi, int Co, int KH, int KW, int Ho, int Wo,
                             blindno_stream_t stream);
/* TemporalSelfAttention + the bag mean that follows it (:1065-1083 and :1163-1164 / :1171-1172):
 * Y (B, D) = mean_l LayerNorm_D(A X + X)_l, A = softmax(X X^T / sqrt D), X (B, L, D) the bag's L
 * snapshot features flattened to D = C H W, LayerNorm eps `eps` with gamma lw / beta lb (D).
 * Collapsed to a centred Gram matrix per bag (see csrc/unet.hip).  L <= 480.
 *   save: blindno_tok_attn_save_floats(B, L, D) floats (16-B aligned), written by the forward,
 *         read by the backward; gram: B L L floats; gram_partial: blindno_tok_gram_nchunk(D)
 *         x B L L floats (NULL when that is 1).
 *   bwd:  dX (B, L, D) (NULL: none), dlw / dlb (D) (NULL: none); scratch:
 *         blindno_tok_attn_bwd_scratch_floats(B, L) floats (8-B aligned). */
int blindno_tok_gram_nchunk(int64_t D);
int64_t blindno_tok_attn_save_floats(int B, int L, int64_t D);
int blindno_tok_attn_fwd(const float* X, const float* lw, const float* lb, float* Y, float* save,
                         float* gram_partial, float* gram, int B, int L, int64_t D, float eps,
                         blindno_stream_t stream);
int64_t blindno_tok_attn_bwd_scratch_floats(int B, int L);
int blindno_tok_attn_bwd(const float* dY, const float* X, const float* lw, const float* save,
                         float* dX, float* dlw, float* dlb, float* scratch, int B, int L,
                         int64_t D, blindno_stream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* BLINDNO_H */
