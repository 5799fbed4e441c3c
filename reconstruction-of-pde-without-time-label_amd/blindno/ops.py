"""Host orchestration of the HIP kernels: spectral convolutions, FNO bodies, bag mean,
loss -- each wrapped as a torch.autograd.Function whose forward and backward enqueue
only libblindno kernels on the current HIP stream.

Reference semantics followed (yl602019618/Reconstruction-of-PDE-without-Time-Label):
  SpectralConv2d  2d_FPE/FNOModules.py:124-178     SpectralConv1d 1d_FPE/FNOModules.py:27-59
  FNO2d           2d_FPE/FNOModules.py:181-240     FNO1d          1d_FPE/FNOModules.py:62-122
  bag mean        2d_FPE/NIOModules.py:565-575     1d_FPE/NIOModules.py:140-149
  MSELoss         2d_FPE/train_fno.py:116,142
There is no CPU path: CPU tensors raise.
"""
from __future__ import annotations

import contextlib
import ctypes
import math
from typing import List, Optional, Sequence, Tuple

import torch

from ._lib import BlindnoError, call, ptr, query, stream_ptr

F32 = torch.float32

# Channel-mix precision of the 2D spectral layers (BASELINE config E: "fp16 channel-mix + fp32
# spectral accumulate"): "fp32" (default, the reference's arithmetic) or "fp16" (fp16 operands,
# fp32 accumulation, block-scaled spectra; csrc/spectral.hip coldft_mix_kernel H16).  The DFT
# stages and the weight gradient stay fp32.  Read when a layer is launched (a captured graph
# keeps the mode it was captured with).
MIX_F16 = False

# The fused snapshot encoder's projection + bag mean at bag level (csrc/bagproj.hip): the
# forward leaves per-(bag, point) sufficient statistics and the backward reduces them instead
# of recomputing fc1 / GELU / GELU' per snapshot point.  False: the per-snapshot projection
# kernels (csrc/project.hip) and the bag-mean kernel, as before.
BAG_STATS = True
# the bag-statistics projection keeps 3 KB per (bag, crop point) plus v (the last layer's field
# size) from forward to backward: ~190 MB at config C, ~800 MB at config E (256^2, B = 4).
# Above this budget the per-snapshot projection runs instead (same results).
BAG_STATS_MAX_BYTES = 4 << 30

# The column pass of the snapshot encoder's spectral layers folded into the row kernels around
# it (csrc/colspec.h: column-DFT partials written by the kernel that forms the row spectrum, the
# mix on the partials, the row coefficients rebuilt from the mixed spectrum in the next row
# inverse's prologue): FNO_input at C = 4, m1 = m2 = 12 with the fp32 mix.  False: the fused
# column pass (blindno_colpass) between the row kernels, as before.
# (Kept as a module flag, not an environment switch: tests/test_gpu_colspec.py compares the two.)
# With the bag-level projection, the last layer's gradient dz = lw_l ghat v is always formed on
# load by its readers (the projection backward writes no dz field).
COLSPEC = True
# The flags below select between a fused launch and its general fallback, which other shapes
# take anyway; the tests turn them off to check both forms (tests/test_gpu_graphs.py,
# test_gpu_parity.py).  Settled defaults, no environment switches.
# the grouped heads' backward: row DFT + conv gradient + the previous layer's mix gradient in
# one launch per layer (False: three launches)
HEAD_BWD_MERGED = True
# the deferred finalisation stores the spectral weight gradients unpacked from the kernel that
# finishes them (False: a separate unpack launch)
UNPACK_FOLD = True
# the encoder's spectral weight gradients hosted by its first layer's adjoint launch
# (False: the deferred finalisation's mix launch)
HOST_ENC_MIX = True
# the bag encoder's spectral-weight pack (with the heads' pack_ahead requests) hosted by its
# first row-DFT launch (False: a pack launch of its own)
HOST_PACK = True


def set_mix_precision(name: str) -> None:
    global MIX_F16
    if name not in ("fp32", "fp16"):
        raise BlindnoError(f"mix precision must be 'fp32' or 'fp16', got {name!r}")
    MIX_F16 = name == "fp16"


def _mixdir(direction: int) -> int:
    return direction | (2 if MIX_F16 else 0)

# ---------------------------------------------------------------------------- helpers


def pad_amount(n: int) -> int:
    """int(round(n/4)) with round-half-even (2d_FPE/FNOModules.py:222-223)."""
    return int(round(n * 0.25))


def kept_rows_count(m1: int, P1: int) -> int:
    return 2 * m1 if 2 * m1 < P1 else P1


_TW = {}


def twiddle(P: int, device) -> torch.Tensor:
    """Device table tw[j] = (cos 2 pi j/P, sin 2 pi j/P), built in double."""
    dev = torch.device(device)
    key = (P, dev.index)
    t = _TW.get(key)
    if t is None:
        j = torch.arange(P, dtype=torch.float64) * (2.0 * torch.pi / P)
        t = torch.stack([torch.cos(j), torch.sin(j)], 1).to(F32).to(dev).contiguous()
        _TW[key] = t
    return t


_TWR = {}


def twiddle_rowinv(P2: int, m2: int, device) -> torch.Tensor:
    """B-operand image of the inverse row transform (include/blindno.h blindno_rowidft_epi):
    tb[s][t][l] = cos / -sin (kk = 4 s + (l >> 4) even / odd) of 2 pi k w / P2, k = kk // 2,
    w = 16 t + (l & 15); zero for k >= m2 or w >= P2.  Built in double."""
    dev = torch.device(device)
    key = (P2, m2, dev.index)
    t = _TWR.get(key)
    if t is None:
        KS, NT = (m2 + 1) // 2, (P2 + 15) // 16
        s = torch.arange(KS)[:, None, None]
        tt = torch.arange(NT)[None, :, None]
        ln = torch.arange(64)[None, None, :]
        kk = 4 * s + (ln >> 4)
        k = kk // 2
        w = 16 * tt + (ln & 15)
        ph = ((k * w) % P2).to(torch.float64) * (2.0 * torch.pi / P2)
        v = torch.where(kk % 2 == 0, torch.cos(ph), -torch.sin(ph))
        v = torch.where((k < m2) & (w < P2), v, torch.zeros_like(v))
        t = v.to(F32).to(dev).reshape(-1).contiguous()
        _TWR[key] = t
    return t


_TWM = {}


def twiddle_mfma(P2: int, m2: int, device) -> torch.Tensor:
    """B-operand image of the row-DFT matrix T (P2 x 2*m2; T[w][2k] = cos, T[w][2k+1] = -sin
    of 2 pi k w / P2) for the MFMA row DFT: Tp[kb][kq][n][s] = T[16 kb + 4 kq + s][n], zero
    padded to KB = ceil(P2/16) blocks and Npad = 16*ceil(2*m2/16) columns."""
    dev = torch.device(device)
    key = (P2, m2, dev.index)
    t = _TWM.get(key)
    if t is None:
        KB = (P2 + 15) // 16
        Npad = ((2 * m2 + 15) // 16) * 16
        w = torch.arange(KB * 16, dtype=torch.int64)[:, None]
        k = torch.arange(m2, dtype=torch.int64)[None, :]
        ph = ((w * k) % P2).to(torch.float64) * (2.0 * torch.pi / P2)
        T = torch.zeros(KB * 16, Npad, dtype=torch.float64)
        T[:, 0:2 * m2:2] = torch.cos(ph)
        T[:, 1:2 * m2:2] = -torch.sin(ph)
        T[P2:] = 0.0
        Tp = T.view(KB, 4, 4, Npad).permute(0, 1, 3, 2).contiguous()   # [kb][kq][n][s]
        t = Tp.to(F32).to(dev).reshape(-1).contiguous()
        _TWM[key] = t
    return t


_TWC = {}


def kept_rows(m1: int, P1: int):
    """Frequency rows r_j kept by SpectralConv2d: [0, m1) from weights1 and [P1-m1, P1) from
    weights2 (all rows when 2 m1 >= P1; 2d_FPE/FNOModules.py:170-173)."""
    K1 = kept_rows_count(m1, P1)
    return [j if (K1 == P1 or j < m1) else P1 - 2 * m1 + j for j in range(K1)]


def twiddle_cols(P1: int, m1: int, device):
    """MFMA B-operand images of F[h][j] = e^{-2 pi i r_j h / P1} for the column pass:
    FB[jt][hb][l][s] = F[16 hb + 4 (l>>4) + s][16 jt + (l&15)] and
    GB[ht][jb][l][s] = conj F[16 ht + (l&15)][16 jb + 4 (l>>4) + s], zero outside, complex
    interleaved (include/blindno.h blindno_colpass)."""
    dev = torch.device(device)
    key = (P1, m1, dev.index)
    t = _TWC.get(key)
    if t is None:
        K1 = kept_rows_count(m1, P1)
        Jt, Ht = (K1 + 15) // 16, (P1 + 15) // 16
        r = torch.zeros(Jt * 16, dtype=torch.int64)
        r[:K1] = torch.tensor(kept_rows(m1, P1), dtype=torch.int64)
        h = torch.arange(Ht * 16, dtype=torch.int64)
        ph = ((h[:, None] * r[None, :]) % P1).to(torch.float64) * (2.0 * torch.pi / P1)
        F = torch.complex(torch.cos(ph), -torch.sin(ph))            # (Ht*16, Jt*16)
        F[P1:, :] = 0
        F[:, K1:] = 0
        # FB: [jt][hb][kq][c][s] = F[16hb + 4kq + s][16jt + c]
        FB = F.view(Ht, 4, 4, Jt, 16).permute(3, 0, 1, 4, 2)
        # GB: [ht][jb][kq][c][s] = conj F[16ht + c][16jb + 4kq + s]
        GB = F.conj().view(Ht, 16, Jt, 4, 4).permute(0, 2, 3, 1, 4)
        cv = lambda z: torch.view_as_real(z.contiguous()).to(F32).to(dev).contiguous()
        t = (cv(FB), cv(GB))
        _TWC[key] = t
    return t


_TWS = {}


def twiddle_colspec(P1: int, m1: int, device) -> torch.Tensor:
    """Tab[h][2 j + p] = (cos, sin)(2 pi r_j h / P1) for the kept rows r_j (csrc/colspec.h):
    the column DFT's F (= cos - i sin) and the column inverse's conj(F); followed by the same
    values as TabT[h / 4][2 j + p][h % 4] (the column DFT's lane order); built in double."""
    dev = torch.device(device)
    key = (P1, m1, dev.index)
    t = _TWS.get(key)
    if t is None:
        r = torch.tensor(kept_rows(m1, P1), dtype=torch.int64)
        h = torch.arange(P1, dtype=torch.int64)
        ph = ((h[:, None] * r[None, :]) % P1).to(torch.float64) * (2.0 * torch.pi / P1)
        tab = torch.stack([torch.cos(ph), torch.sin(ph)], -1).reshape(P1, -1)
        tabT = tab.view(P1 // 4, 4, -1).permute(0, 2, 1)
        t = torch.cat([tab.reshape(-1), tabT.reshape(-1)]).to(F32).to(dev).contiguous()
        _TWS[key] = t
    return t


def colspec_ok(Bn, C, P1, P2, m1, m2) -> bool:
    """The folded column pass applies (blindno_colspec_ok; fp32 mix only)."""
    return COLSPEC and not MIX_F16 and bool(query("blindno_colspec_ok", Bn, C, P1, P2, m1, m2))


def require_device(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise BlindnoError("blindno ops need HIP device tensors; there is no CPU path "
                               "(move the model and inputs to 'cuda')")


def _c(t):
    if t is None:
        return None
    if t.dtype not in (F32, torch.complex64):
        raise BlindnoError(f"blindno ops are fp32: got {t.dtype}")
    return t if t.is_contiguous() else t.contiguous()


def _empty(*shape, like):
    return torch.empty(*shape, dtype=F32, device=like.device)


# Deferred weight-gradient finalisation.  Inside ``deferred_reductions()`` the spectral weight
# gradients (the mix GEMMs over the samples), the partial-sum reductions and the spectral-weight
# unpacks of a backward pass are only recorded; the returned gradient tensors are filled by
# three batched launches (blindno_mix_wgrad_multi, blindno_reduce_partials_pieces,
# blindno_unpack_w2d_multi) when the context exits -- 5 + 10 + 5 small latency-bound launches
# per config-C step become 3, with bit-identical results.  ``redirect`` (before the exit) makes
# those launches store parameter gradients straight into an optimizer's flat gradient buffer,
# so no gather copy follows.  The recorded sources stay referenced until the flush is enqueued,
# so the allocator cannot hand their memory to later kernels.  Only for callers that read no
# returned gradient before the exit (GraphedBagStep: the gradients are consumed by the
# optimizer after backward, and are None before it).
_DEFER = None


class _Deferred:
    def __init__(self):
        self.mix = []      # (X, G, out, (Bn, Ci, Co, K1, m2, nsplit, Gw)): spectral weight gradients
        self.red = []      # [partial, out, nchunk, np, pieces]; pieces: [(e0, e1, dst)] (redirect)
        self.unp = []      # [dWt slice, dw1, dw2, (Ci, Co, m1, m2, P1), base of dw1 / dw2]

    def redirect(self, pairs):
        """Have the flushed kernels store gradients straight into their final buffers: for
        every (param, dst) pair -- dst a float32 tensor of the parameter's real size, e.g. a
        view of an optimizer's flat gradient buffer -- whose ``.grad`` is one of the recorded
        unpack outputs or a slice of a recorded reduction's output, that gradient is written
        at dst instead (a piece of the reduction: the same summation order, bit-identical) and
        ``.grad`` is re-pointed to dst.  Called after backward, before the flush.  Returns the
        redirected parameters."""
        done = []
        for p, dst in pairs:
            g = p.grad
            if g is None:
                continue
            gr = torch.view_as_real(g) if g.is_complex() else g
            if gr.dtype != F32 or not gr.is_contiguous() or dst.numel() != gr.numel():
                continue
            gp, n = gr.data_ptr(), gr.numel()
            hit = False
            for u in self.unp:
                for k in (1, 2):
                    if u[k].data_ptr() == gp and u[k].numel() == n:
                        u[k] = dst.view(u[k].shape)
                        hit = True
                        break
                if hit:
                    break
            if not hit:
                for r in self.red:
                    op, on = r[1].data_ptr(), r[1].numel()
                    if op <= gp and gp + 4 * n <= op + 4 * on and (gp - op) % 4 == 0:
                        e0 = (gp - op) // 4
                        if all(e1 <= e0 or e0 + n <= a for a, e1, _ in r[4]):
                            r[4].append((e0, e0 + n, dst))
                            hit = True
                        break
            if hit:
                v = dst.view(gr.shape)
                p.grad = torch.view_as_complex(v) if g.is_complex() else v
                done.append(p)
        return done

    def _fold_unpacks(self):
        """Match each recorded unpack to the kernel that finishes its dWt -- a mix job with no
        sample split (all its weight groups unpacked) or a whole reduction -- so that kernel
        stores dWt unpacked (W2dUnpack, csrc/wgrad.h) and the unpack launch goes.  Returns
        ({mix job: {group: (dw1, dw2)}}, {reduction: (dw1, dw2, (Ci, Co, m1, m2))}, the
        unpacks left for blindno_unpack_w2d_multi)."""
        mixu, redu, rest = {}, {}, []
        taken = {}
        for u in self.unp:
            dW, d1, d2, (Ci, Co, m1, m2, P1), _ = u
            hit = False
            if UNPACK_FOLD and 2 * m1 < P1:
                p = dW.data_ptr()
                for qi, (_, _, out, sh) in enumerate(self.mix):
                    Bn, ci, co, K1, mm2, ns, Gw = sh
                    per = mm2 * K1 * ci * co * 2 * 4
                    off = p - out.data_ptr()
                    if (ns == 1 and Gw <= 4 and K1 == 2 * m1 and (ci, co, mm2) == (Ci, Co, m2)
                            and 4 * dW.numel() == per and 0 <= off < per * Gw and off % per == 0):
                        mixu.setdefault(qi, {})[off // per] = (d1, d2)
                        taken.setdefault(qi, []).append(u)
                        hit = True
                        break
                if not hit:
                    for ri, r in enumerate(self.red):
                        if (r[1].data_ptr() == p and r[3] == dW.numel() and not r[4] and ri not in redu
                                and r[3] == 4 * Ci * Co * m1 * m2):
                            redu[ri] = (d1, d2, (Ci, Co, m1, m2))
                            hit = True
                            break
            if not hit:
                rest.append(u)
        for qi in list(mixu):
            if len(mixu[qi]) != self.mix[qi][3][6]:      # every group of the job, or none
                rest.extend(taken[qi])
                del mixu[qi]
        return mixu, redu, rest

    def _unpacks_read_reductions(self, rest):
        """True when the dWt an unpack of ``rest`` reads overlaps memory a recorded reduction
        writes (its output buffer or a redirected piece) -- e.g. the grouped heads' (G, ...)
        reduction whose slice dWt[g] an unpack reads.  Such unpacks must run after the
        reductions, not beside them."""
        spans = []
        for _, out, _, _, pieces in self.red:
            spans.append((out.data_ptr(), out.data_ptr() + 4 * out.numel()))
            spans += [(d.data_ptr(), d.data_ptr() + 4 * d.numel()) for _, _, d in pieces]
        for u in rest:
            a = u[0].data_ptr()
            b = a + u[0].element_size() * u[0].numel()
            if any(a < e and s < b for s, e in spans):
                return True
        return False

    def flush(self):
        mixu, redu, rest = self._fold_unpacks()
        if self.mix:
            n = len(self.mix)
            xs = (ctypes.c_void_p * n)(*[m[0].data_ptr() for m in self.mix])
            gs = (ctypes.c_void_p * n)(*[m[1].data_ptr() for m in self.mix])
            os_ = (ctypes.c_void_p * n)(*[m[2].data_ptr() for m in self.mix])
            shp = (ctypes.c_int * (7 * n))(*[v for m in self.mix for v in m[3]])
            ud = [None] * (8 * n)
            um1 = [0] * n
            for qi, groups in mixu.items():
                for g, (d1, d2) in groups.items():
                    ud[8 * qi + 2 * g], ud[8 * qi + 2 * g + 1] = d1.data_ptr(), d2.data_ptr()
                um1[qi] = self.mix[qi][3][3] // 2
            call("blindno_mix_wgrad_multi_u", xs, gs, os_, shp, (ctypes.c_void_p * (8 * n))(*ud),
                 (ctypes.c_int * n)(*um1), n, stream_ptr())
        if self.red:
            segs = []          # (partial, dst address, nchunk, np, e0, e1, unpack descriptor)
            descs = []
            for ri, (partial, out, nchunk, np_, pieces) in enumerate(self.red):
                if ri in redu:
                    descs.append(redu[ri])
                    segs.append((partial, out.data_ptr(), nchunk, np_, 0, np_, len(descs) - 1))
                    continue
                pos = 0
                for e0, e1, dst in sorted(pieces, key=lambda t: t[0]):
                    if e0 > pos:
                        segs.append((partial, out.data_ptr() + 4 * pos, nchunk, np_, pos, e0, -1))
                    segs.append((partial, dst.data_ptr(), nchunk, np_, e0, e1, -1))
                    pos = e1
                if pos < np_:
                    segs.append((partial, out.data_ptr() + 4 * pos, nchunk, np_, pos, np_, -1))
            n = len(segs)
            srcs = (ctypes.c_void_p * n)(*[t[0].data_ptr() for t in segs])
            outs = (ctypes.c_void_p * n)(*[t[1] for t in segs])
            ncs = (ctypes.c_int * n)(*[t[2] for t in segs])
            nps = (ctypes.c_int * n)(*[t[3] for t in segs])
            e0s = (ctypes.c_int * n)(*[t[4] for t in segs])
            e1s = (ctypes.c_int * n)(*[t[5] for t in segs])
            upks = (ctypes.c_int * n)(*[t[6] for t in segs])
            nd = max(1, len(descs))
            ud = (ctypes.c_void_p * (2 * nd))(*[v for d in descs for v in (d[0].data_ptr(), d[1].data_ptr())])
            ushp = (ctypes.c_int * (4 * nd))(*[v for d in descs for v in d[2]])
            red_args = (srcs, outs, ncs, nps, e0s, e1s, upks, ud, ushp, n)
            if not rest:
                call("blindno_reduce_partials_pieces_u", *red_args, stream_ptr())
        if rest:
            n = len(rest)
            srcs = (ctypes.c_void_p * n)(*[u[0].data_ptr() for u in rest])
            d1 = (ctypes.c_void_p * n)(*[u[1].data_ptr() for u in rest])
            d2 = (ctypes.c_void_p * n)(*[u[2].data_ptr() for u in rest])
            shp = (ctypes.c_int * (5 * n))(*[v for u in rest for v in u[3]])
            if self.red and not self._unpacks_read_reductions(rest):
                # the reductions and the unpacks in one launch: no unpack reads what a
                # reduction of the same launch writes (blindno_finish_multi runs both
                # job lists concurrently)
                call("blindno_finish_multi", *red_args, srcs, d1, d2, shp, n, stream_ptr())
            else:
                if self.red:    # ordered: an unpack reads a reduction's output
                    call("blindno_reduce_partials_pieces_u", *red_args, stream_ptr())
                call("blindno_unpack_w2d_multi", srcs, d1, d2, shp, n, stream_ptr())
        self.mix, self.red, self.unp = [], [], []


@contextlib.contextmanager
def deferred_reductions():
    global _DEFER
    prev, _DEFER = _DEFER, _Deferred()
    try:
        yield _DEFER
        _DEFER.flush()
    finally:
        _DEFER = prev


@contextlib.contextmanager
def immediate_reductions():
    """Suspend deferred_reductions() for code that reads the reductions' results right away
    (the torch.ops.blindno backward formulas)."""
    global _DEFER
    prev, _DEFER = _DEFER, None
    try:
        yield
    finally:
        _DEFER = prev


def reduce_partials(partial: torch.Tensor, nchunk: int, np_: int) -> torch.Tensor:
    out = _empty(np_, like=partial)
    if _DEFER is not None:
        _DEFER.red.append([partial, out, int(nchunk), int(np_), []])
        return out
    call("blindno_reduce_partials", ptr(partial), ptr(out), nchunk, np_, stream_ptr())
    return out


def unpack_w2d(dWt: torch.Tensor, like: torch.Tensor, P1: int):
    """dWt (m2, K1, Ci, Co, 2) -> (dw1, dw2) in the reference layout of ``like`` (Ci, Co, m1,
    m2, 2).  Deferred, both are views of one fresh (2, ...) buffer and the list keeps the BASE
    alive, not the returned views, so autograd's AccumulateGrad still adopts the views as the
    parameters' .grad instead of cloning them (a clone before the flush would copy unwritten
    memory -- as with reduce_partials, whose returned gradients are slices of ``out``)."""
    Ci, Co, m1, m2 = like.shape[:4]
    if _DEFER is not None:
        base = torch.empty((2,) + tuple(like.shape), dtype=like.dtype, device=like.device)
        _DEFER.unp.append([dWt, base[0], base[1], (Ci, Co, m1, m2, P1), base])
        return base[0], base[1]
    # two separate tensors (torch custom ops may not return aliasing outputs)
    dw1, dw2 = torch.empty_like(like), torch.empty_like(like)
    call("blindno_unpack_w2d", ptr(dWt), ptr(dw1), ptr(dw2), Ci, Co, m1, m2, P1, stream_ptr())
    return dw1, dw2


# ---------------------------------------------------------------------------- kernel wrappers


def k_rowdft(x, Bn, C, P1, P2, m2, act, valid=None):
    """Row DFT; ``valid`` = (N1v, N2v): read only that region of each plane (zero elsewhere)."""
    At = _empty(Bn, m2, C, P1, 2, like=x)
    if valid is None:
        call("blindno_rowdft", ptr(x), ptr(At), ptr(twiddle_mfma(P2, m2, x.device)), Bn, C, P1, P2,
             m2, act, stream_ptr())
    else:
        call("blindno_rowdft_crop", ptr(x), ptr(At), ptr(twiddle_mfma(P2, m2, x.device)), Bn, C, P1,
             P2, m2, act, valid[0], valid[1], stream_ptr())
    return At


def k_colpass(At, Wt, Bn, Ci, Co, P1, m1, m2, P2, direction):
    """Column DFT at the kept rows + per-mode mix + column inverse (matrix-core GEMMs).
    Returns (saved spectrum (Bn, m2, Cin, K1), row coefficients Z (Bn, P1, m2, Cout))."""
    K1 = kept_rows_count(m1, P1)
    K1p = 16 * ((K1 + 15) // 16)
    cin, cout = (Ci, Co) if direction == 0 else (Co, Ci)
    Xs = _empty(Bn, m2, cin, K1, 2, like=At)
    Y = _empty(Bn, m2, cout, K1p, 2, like=At)
    Z = _empty(Bn, P1, m2, cout, 2, like=At)
    FB, GB = twiddle_cols(P1, m1, At.device)
    call("blindno_colpass", ptr(At), ptr(Wt), ptr(Xs), ptr(Y), ptr(Z), ptr(FB), ptr(GB), Bn,
         Ci, Co, P1, m1, m2, P2, _mixdir(direction), stream_ptr())
    return Xs, Z


def k_mix_wgrad(X, G, Bn, Ci, Co, K1, m2, deferrable=False, jobs=None):
    """Spectral weight gradient dWt (m2, K1, Ci, Co, 2).  ``deferrable``: the caller's only
    reader of dWt is itself deferred (the 2D unpack), so under deferred_reductions() the
    sample-split reduction may join the batched finalisation."""
    ns = query("blindno_mix_wgrad_nsplit", Bn, Ci, Co, K1, m2)
    if _DEFER is not None and deferrable:
        # the mix gradient itself joins the batched finalisation (one launch for every layer's,
        # before the reductions and the unpack) -- or, with ``jobs``, a later launch of the
        # caller's that hosts it (the caller launches it before the finalisation)
        q = _DEFER.mix if jobs is None else jobs
        if ns > 1:
            part = _empty(ns, m2 * K1 * Ci * Co * 2, like=X)
            q.append((X, G, part, (Bn, Ci, Co, K1, m2, ns, 1)))
            return reduce_partials(part, ns, m2 * K1 * Ci * Co * 2).view(m2, K1, Ci, Co, 2)
        dWt = _empty(m2, K1, Ci, Co, 2, like=X)
        q.append((X, G, dWt, (Bn, Ci, Co, K1, m2, 1, 1)))
        return dWt
    dWt = _empty(m2, K1, Ci, Co, 2, like=X)
    part = _empty(ns, m2 * K1 * Ci * Co * 2, like=X) if ns > 1 else None
    call("blindno_mix_wgrad", ptr(X), ptr(G), ptr(dWt), ptr(part) if part is not None else None, ns,
         Bn, Ci, Co, K1, m2, stream_ptr())
    return dWt


def k_pack_w2d(w1, w2, P1):
    Ci, Co, m1, m2 = w1.shape[:4]
    K1 = kept_rows_count(m1, P1)
    Wt = _empty(m2, K1, Ci, Co, 2, like=w1)
    call("blindno_pack_w2d", ptr(w1), ptr(w2), ptr(Wt), Ci, Co, m1, m2, P1, stream_ptr())
    return Wt


# Packs requested ahead of their consumer (pack_ahead): they ride along the next _pack_into
# launch -- the grouped heads' spectral weights are packed by the snapshot encoder's pack
# launch at the start of the forward instead of by a launch of their own between the encoder
# and the heads.  The consumer collects its buffers with take_packed.
_PACK_AHEAD = []       # [(pairs, Wts, P1, handle)] not yet launched
_PACKED = {}           # key -> (handle, request)


def _pack_key(pairs, P1):
    return tuple((w1.data_ptr(), w2.data_ptr()) for w1, w2 in pairs), int(P1)


def pack_ahead(pairs, Wts, P1, handle):
    """Register a pack of ``pairs`` into ``Wts`` (row count P1) for the next pack launch;
    ``handle`` (e.g. the tensor the Wts are views of) is what take_packed returns."""
    req = (list(pairs), list(Wts), int(P1), handle)
    _PACK_AHEAD.append(req)
    _PACKED[_pack_key(pairs, P1)] = (handle, req)


def take_packed(pairs, P1):
    """The handle of an earlier pack_ahead of exactly these pairs (launched now if no pack
    launch has taken it along yet), or None."""
    hit = _PACKED.pop(_pack_key(pairs, P1), None)
    if hit is None:
        return None
    handle, req = hit
    if any(r is req for r in _PACK_AHEAD):
        _PACK_AHEAD[:] = [r for r in _PACK_AHEAD if r is not req]
        _pack_into(req[0], req[1], req[2])
    return handle


def drop_pack_ahead():
    """Forget every request (end of a forward): nothing stale survives into the next one --
    including a held-back pack whose Wts a failed forward may already have freed."""
    _PACK_AHEAD.clear()
    _PACKED.clear()
    _PACK_DEFERRED.clear()


_PACK_DEFERRED = []     # at most one pack launch's arguments, held for take_deferred_pack


def take_deferred_pack():
    """The arguments (w1s, w2s, Wts, shapes, n) of the pack _pack_into(defer=True) held back, for
    a launch that hosts it (blindno_rowdft_bag_lift_cd_pack), or None."""
    return _PACK_DEFERRED.pop() if _PACK_DEFERRED else None


def flush_deferred_pack():
    """Launch a held-back pack now (nothing took it along)."""
    pk = take_deferred_pack()
    if pk is not None:
        call("blindno_pack_w2d_multi", *pk, stream_ptr())


def _pack_into(pairs, Wts, P1, defer=False):
    """Pack the spectral weights (w1, w2) of several 2D layers into the contiguous Wts[i]
    (m2, K1, Ci, Co, 2) with ONE launch (blindno_pack_w2d_multi), together with every pending
    pack_ahead request.  ``defer``: hold the launch's arguments for take_deferred_pack -- the
    caller's next launch hosts the pack, and nothing may read the Wts before it."""
    flush_deferred_pack()
    jobs = [(pr, W, P1) for pr, W in zip(pairs, Wts)]
    for r in _PACK_AHEAD:
        jobs += [(pr, W, r[2]) for pr, W in zip(r[0], r[1])]
    _PACK_AHEAD.clear()
    w1s, w2s, shp = [], [], []
    for (w1, w2), W, P1j in jobs:
        w1, w2 = _c(w1), _c(w2)
        Ci, Co, m1, m2 = w1.shape[:4]
        if W.shape != (m2, kept_rows_count(m1, P1j), Ci, Co, 2) or not W.is_contiguous():
            raise BlindnoError("pack: bad Wt buffer")
        w1s.append(w1.data_ptr())
        w2s.append(w2.data_ptr())
        shp += [Ci, Co, m1, m2, P1j]
    Wts = [j[1] for j in jobs]
    n = len(Wts)
    args = ((ctypes.c_void_p * n)(*w1s), (ctypes.c_void_p * n)(*w2s),
            (ctypes.c_void_p * n)(*[W.data_ptr() for W in Wts]), (ctypes.c_int * (5 * n))(*shp), n)
    if defer:
        _PACK_DEFERRED.append(args)
    else:
        call("blindno_pack_w2d_multi", *args, stream_ptr())


def pack_w2d_many(pairs, P1, defer=False):
    """One packed Wt (m2, K1, Ci, Co, 2) per (w1, w2) pair, all in one launch (``defer``: see
    _pack_into)."""
    Wts = [_empty(w1.shape[3], kept_rows_count(w1.shape[2], P1), w1.shape[0], w1.shape[1], 2, like=w1)
           for w1, _ in pairs]
    _pack_into(pairs, Wts, P1, defer=defer)
    return Wts


def k_unpack_w2d(dWt, w1, P1):
    return unpack_w2d(dWt, w1, P1)


def k_pack_w1d(w):
    Ci, Co, m = w.shape
    Wt = _empty(m, 1, Ci, Co, 2, like=torch.view_as_real(w))
    call("blindno_pack_w1d", ptr(w), ptr(Wt), Ci, Co, m, 0, stream_ptr())
    return Wt


def k_unpack_w1d(dWt, w):
    Ci, Co, m = w.shape
    dw = torch.empty_like(w)
    call("blindno_pack_w1d", ptr(dWt), ptr(dw), Ci, Co, m, 1, stream_ptr())
    return dw


def k_mix1d(At, Wt, Bn, Ci, Co, m, P2, direction):
    cin = Ci if direction == 0 else Co
    cout = Co if direction == 0 else Ci
    Xs = _empty(Bn, m, cin, 1, 2, like=At)
    Z = _empty(Bn, 1, m, cout, 2, like=At)
    call("blindno_mix1d", ptr(At), ptr(Wt), ptr(Xs), ptr(Z), Bn, Ci, Co, m, P2, direction,
         stream_ptr())
    return Xs, Z


def k_rowidft_epi(Z, x, wc, bc, Bn, C, P1, P2, m2, act):
    z = _empty(Bn, C, P1, P2, like=Z)
    call("blindno_rowidft_epi", ptr(Z), ptr(x), ptr(wc), ptr(bc), ptr(z),
         ptr(twiddle_rowinv(P2, m2, Z.device)), Bn, C, P1, P2, m2, act, stream_ptr())
    return z


def k_rowidft_epi_rd(Z, x, wc, bc, Bn, C, P1, P2, m2, act, act_next):
    """k_rowidft_epi plus the next layer's row DFT of f(z) (f = GELU if act_next) in the same
    pass: returns (z, At) with At = k_rowdft(z, ..., act_next)."""
    z = _empty(Bn, C, P1, P2, like=Z)
    At = _empty(Bn, m2, C, P1, 2, like=Z)
    call("blindno_rowidft_epi_rd", ptr(Z), ptr(x), ptr(wc), ptr(bc), ptr(z),
         ptr(twiddle_rowinv(P2, m2, Z.device)), Bn, C, P1, P2, m2, act, ptr(At),
         ptr(twiddle_mfma(P2, m2, Z.device)), act_next, stream_ptr())
    return z, At


def k_rowidft_bwd(G, dz, wc, xsrc, Bn, C, P1, P2, m2, act, want_wgrad=False, valid=None,
                  rd=False):
    """dx = irow^H(G) + Wc^T dz, times GELU'(xsrc) if act.  With want_wgrad (C <= 8) the
    1x1-conv weight/bias gradients are reduced in the same pass (C <= 4): returns (dx, gw, gb).
    ``valid`` = (N1v, N2v): dz is read only on that region (zero elsewhere).  ``rd``: also the
    row DFT of dx for the previous layer's adjoint (k_rowdft(dx, ..., 0)) in the same pass,
    appended to the result."""
    dx = _empty(Bn, C, P1, P2, like=G)
    partial, nchunk = None, 0
    if want_wgrad:
        nchunk = query("blindno_rowidft_bwd_nchunk", Bn, C, P1, P2, m2)
        partial = _empty(nchunk, C * C + C, like=G)
    dN1, dN2 = valid if valid is not None else (P1, P2)
    At = None
    if rd:
        At = _empty(Bn, m2, C, P1, 2, like=G)
        call("blindno_rowidft_bwd_rd", ptr(G), ptr(dz), ptr(wc), ptr(xsrc), ptr(dx),
             ptr(twiddle_rowinv(P2, m2, G.device)), ptr(partial), Bn, C, P1, P2, m2, act, dN1,
             dN2, ptr(At), ptr(twiddle_mfma(P2, m2, G.device)), stream_ptr())
    else:
        call("blindno_rowidft_bwd_crop", ptr(G), ptr(dz), ptr(wc), ptr(xsrc), ptr(dx),
             ptr(twiddle_rowinv(P2, m2, G.device)), ptr(partial), Bn, C, P1, P2, m2, act, dN1,
             dN2, stream_ptr())
    out = (dx, None, None)
    if want_wgrad:
        g = reduce_partials(partial, nchunk, C * C + C)
        out = (dx, g[: C * C], g[C * C:])
    return out + (At,) if rd else out


def k_conv_wgrad(dz, x, Bn, C, P1, P2, act):
    np_ = C * C + C
    nchunk = query("blindno_conv_wgrad_nchunk", Bn, P1, P2)
    partial = _empty(nchunk, np_, like=dz)
    call("blindno_conv_wgrad", ptr(dz), ptr(x), ptr(partial), nchunk, Bn, C, P1, P2, act,
         stream_ptr())
    g = reduce_partials(partial, nchunk, np_)
    return g[: C * C], g[C * C:]


# ---------------------------------------------------------------------------- spectral layer


class SpecShape:
    """Geometry of one spectral layer over a padded field (P1 = 1 for 1D)."""

    def __init__(self, Bn, Ci, Co, P1, P2, m1, m2, dim):
        self.Bn, self.Ci, self.Co, self.P1, self.P2 = Bn, Ci, Co, P1, P2
        self.m1, self.m2, self.dim = m1, m2, dim
        self.K1 = kept_rows_count(m1, P1) if dim == 2 else 1
        if m2 > P2 // 2 + 1:
            raise BlindnoError(f"modes {m2} exceed P2//2+1 = {P2 // 2 + 1}")
        if dim == 2 and m1 > P1:
            raise BlindnoError(f"modes1 {m1} exceed P1 = {P1}")


def spec_forward(x, act, Wt, sh: SpecShape, At=None):
    """Forward spectrum of layer input f(x) -> (saved spectrum X, row coefficients Z).  ``At``:
    the row DFT of f(x), when the previous layer's row inverse already took it."""
    if At is None:
        At = k_rowdft(x, sh.Bn, sh.Ci, sh.P1, sh.P2, sh.m2, act)
    if sh.dim == 2:
        return k_colpass(At, Wt, sh.Bn, sh.Ci, sh.Co, sh.P1, sh.m1, sh.m2, sh.P2, 0)
    return k_mix1d(At, Wt, sh.Bn, sh.Ci, sh.Co, sh.m2, sh.P2, 0)


def spec_backward(dz, X, Wt, sh: SpecShape, valid=None, At=None):
    """Adjoint of spec_forward: returns (dWt, GZ) for the layer's output gradient dz (read only
    on ``valid`` = (N1v, N2v) when given, 2D).  ``At``: the row DFT of dz, when the next layer's
    row-inverse adjoint already took it."""
    if At is None:
        At = k_rowdft(dz, sh.Bn, sh.Co, sh.P1, sh.P2, sh.m2, 0, valid)
    if sh.dim == 2:
        G, GZ = k_colpass(At, Wt, sh.Bn, sh.Ci, sh.Co, sh.P1, sh.m1, sh.m2, sh.P2, 1)
    else:
        G, GZ = k_mix1d(At, Wt, sh.Bn, sh.Ci, sh.Co, sh.m2, sh.P2, 1)
    # 2D: the gradient's only reader is unpack_w2d, deferred alongside (1D unpacks at once)
    dWt = k_mix_wgrad(X, G, sh.Bn, sh.Ci, sh.Co, sh.K1, sh.m2, deferrable=sh.dim == 2)
    return dWt, GZ


def pack_weights(ws, P1, dim):
    if dim == 2:
        return k_pack_w2d(_c(ws[0]), _c(ws[1]), P1)
    return k_pack_w1d(_c(ws[0]))


def unpack_weights(dWt, ws, P1, dim):
    if dim == 2:
        return k_unpack_w2d(dWt, ws[0], P1)
    return (k_unpack_w1d(dWt, ws[0]),)


class SpectralConvFn(torch.autograd.Function):
    """Bare SpectralConv1d/2d (no 1x1 conv): x (Bn, Ci, [P1,] P2) -> (Bn, Co, [P1,] P2)."""

    @staticmethod
    def forward(ctx, x, *ws):
        require_device(x, *ws)
        x = _c(x)
        dim = 2 if len(ws) == 2 else 1
        Bn, Ci = x.shape[:2]
        P1, P2 = (x.shape[2], x.shape[3]) if dim == 2 else (1, x.shape[2])
        w0 = ws[0]
        Co = w0.shape[1]
        m1 = w0.shape[2]
        m2 = w0.shape[3] if dim == 2 else w0.shape[2]
        sh = SpecShape(Bn, Ci, Co, P1, P2, m1, m2, dim)
        Wt = pack_weights(ws, P1, dim)
        X, Z = spec_forward(x, 0, Wt, sh)
        y = k_rowidft_epi(Z, None, None, None, Bn, Co, P1, P2, m2, 0)
        ctx.sh, ctx.dim, ctx.P1 = sh, dim, P1
        ctx.save_for_backward(X, Wt, *ws)
        return y.view(Bn, Co, P2) if dim == 1 else y

    @staticmethod
    def backward(ctx, gy):
        X, Wt, *ws = ctx.saved_tensors
        sh = ctx.sh
        gy = _c(gy)
        dWt, GZ = spec_backward(gy, X, Wt, sh)
        dx = None
        if ctx.needs_input_grad[0]:
            dx, _, _ = k_rowidft_bwd(GZ, None, None, None, sh.Bn, sh.Ci, sh.P1, sh.P2, sh.m2, 0)
            if ctx.dim == 1:
                dx = dx.view(sh.Bn, sh.Ci, sh.P2)
        dws = unpack_weights(dWt, ws, ctx.P1, ctx.dim)
        return (dx, *dws)


# ---------------------------------------------------------------------------- FNO body


class FNOMeta:
    def __init__(self, dim, n_layers, width, modes1, modes2, hidden, cout, cin):
        self.dim, self.n_layers, self.width = dim, n_layers, width
        self.m1, self.m2, self.hidden, self.cout, self.cin = modes1, modes2, hidden, cout, cin


def _fno_geometry(inp, meta: FNOMeta):
    """(Bn, N1, N2, Cin, P1, P2, Ho, Wo) of an FNO input (a tensor or its shape)."""
    shape = inp.shape if hasattr(inp, "shape") else tuple(inp)
    if meta.dim == 2:
        Bn, N1, N2, Cin = shape
        pH, pW = pad_amount(N1), pad_amount(N2)   # x2_padding (H), x1_padding (W)
        P1, P2 = N1 + pH, N2 + pW
        Ho, Wo = P1 - pW, P2 - pH                 # x[..., :-x1_padding, :-x2_padding]
    else:
        Bn, N2, Cin = shape
        N1 = 1
        pW = pad_amount(N2)
        P1, P2 = 1, N2 + pW
        Ho, Wo = 1, P2 - pW
        pH = 0
    if Ho <= 0 or Wo <= 0 or (meta.dim == 2 and (pH == 0 or pW == 0)) or pW == 0:
        raise BlindnoError("grid too small: the reference's crop x[..., :-pad] needs pad > 0")
    return Bn, N1, N2, Cin, P1, P2, Ho, Wo


def fno_forward(meta: FNOMeta, inp, prm, save=True):
    """prm = [fc0w, fc0b, (w1, [w2], cw, cb) * n, fc1w, fc1b, fc2w, fc2b]."""
    Bn, N1, N2, Cin, P1, P2, Ho, Wo = _fno_geometry(inp, meta)
    C, n, dim = meta.width, meta.n_layers, meta.dim
    nw = 2 if dim == 2 else 1
    fc0w, fc0b = prm[0], prm[1]
    x0 = _empty(Bn, C, P1, P2, like=inp)
    call("blindno_lift_fwd", ptr(inp), ptr(fc0w), ptr(fc0b), ptr(x0), Bn, N1, N2, Cin, C, P1, P2,
         stream_ptr())
    sh = SpecShape(Bn, C, C, P1, P2, meta.m1, meta.m2, dim)
    src, act = x0, 0
    Xs, Wts, zs = [], [], []
    off = 2
    for k in range(n):
        ws = prm[off:off + nw]
        cw, cb = prm[off + nw], prm[off + nw + 1]
        off += nw + 2
        Wt = pack_weights(ws, P1, dim)
        X, Z = spec_forward(src, act, Wt, sh)
        z = k_rowidft_epi(Z, src, cw, cb, Bn, C, P1, P2, meta.m2, act)
        Xs.append(X)
        Wts.append(Wt)
        zs.append(z)
        src, act = z, 1
    fc1w, fc1b, fc2w, fc2b = prm[off:off + 4]
    Hd, Cout = fc1w.shape[0], fc2w.shape[0]
    out = _empty(Bn, Ho, Wo, Cout, like=inp)
    call("blindno_project_fwd", ptr(zs[-1]), ptr(fc1w), ptr(fc1b), ptr(fc2w), ptr(fc2b), ptr(out),
         Bn, C, P1, P2, Ho, Wo, Hd, Cout, Cout, 0, stream_ptr())
    if dim == 1:
        out = out.view(Bn, Wo, Cout)
    saved = (x0, Xs, Wts, zs) if save else None
    return out, saved


def fno_backward(meta: FNOMeta, inp, prm, saved, gout, need_inp_grad, dout_div=1):
    Bn, N1, N2, Cin, P1, P2, Ho, Wo = _fno_geometry(inp, meta)
    C, n, dim = meta.width, meta.n_layers, meta.dim
    nw = 2 if dim == 2 else 1
    x0, Xs, Wts, zs = saved
    off_fc1 = 2 + n * (nw + 2)
    fc1w, fc1b, fc2w, fc2b = prm[off_fc1:off_fc1 + 4]
    Hd, Cout = fc1w.shape[0], fc2w.shape[0]
    gout = _c(gout)
    grads: List[Optional[torch.Tensor]] = [None] * len(prm)
    # projection
    dz = torch.zeros(Bn, C, P1, P2, dtype=F32, device=inp.device)
    np_p = Hd * C + Hd + Cout * Hd + Cout
    nchunk = query("blindno_project_bwd_nchunk", Bn, Ho, Wo)
    partial = _empty(nchunk, np_p, like=inp)
    call("blindno_project_bwd", ptr(zs[-1]), ptr(fc1w), ptr(fc1b), ptr(fc2w), ptr(gout), ptr(dz),
         ptr(partial), nchunk, Bn, C, P1, P2, Ho, Wo, Hd, Cout, Cout, 0, dout_div, stream_ptr())
    gp = reduce_partials(partial, nchunk, np_p)
    o = 0
    grads[off_fc1] = gp[o:o + Hd * C].view(Hd, C); o += Hd * C
    grads[off_fc1 + 1] = gp[o:o + Hd]; o += Hd
    grads[off_fc1 + 2] = gp[o:o + Cout * Hd].view(Cout, Hd); o += Cout * Hd
    grads[off_fc1 + 3] = gp[o:o + Cout]
    sh = SpecShape(Bn, C, C, P1, P2, meta.m1, meta.m2, dim)
    for k in reversed(range(n)):
        off = 2 + k * (nw + 2)
        ws = prm[off:off + nw]
        cw = prm[off + nw]
        src, act = (x0, 0) if k == 0 else (zs[k - 1], 1)
        dWt, GZ = spec_backward(dz, Xs[k], Wts[k], sh)
        for j, g in enumerate(unpack_weights(dWt, ws, P1, dim)):
            grads[off + j] = g
        if C <= 4:
            dz_new, gw, gb = k_rowidft_bwd(GZ, dz, cw, src, Bn, C, P1, P2, meta.m2, act, True)
        else:
            gw, gb = k_conv_wgrad(dz, src, Bn, C, P1, P2, act)
            dz_new, _, _ = k_rowidft_bwd(GZ, dz, cw, src, Bn, C, P1, P2, meta.m2, act)
        grads[off + nw] = gw.view_as(cw)
        grads[off + nw + 1] = gb
        dz = dz_new
    # lift
    fc0w = prm[0]
    np_l = C * Cin + C
    nchunk = query("blindno_lift_bwd_nchunk", Bn, N1, N2)
    partial = _empty(nchunk, np_l, like=inp)
    d_inp = torch.empty_like(inp) if need_inp_grad else None
    call("blindno_lift_bwd", ptr(dz), ptr(inp), ptr(fc0w), ptr(d_inp), ptr(partial), nchunk, Bn,
         N1, N2, Cin, C, P1, P2, stream_ptr())
    gl = reduce_partials(partial, nchunk, np_l)
    grads[0] = gl[:C * Cin].view(C, Cin)
    grads[1] = gl[C * Cin:]
    return d_inp, grads


class FNOFn(torch.autograd.Function):
    """Whole FNO1d/FNO2d forward as one autograd node (keeps the reference's parameters,
    runs only HIP kernels)."""

    @staticmethod
    def forward(ctx, meta, inp, *prm):
        require_device(inp, *prm)
        inp = _c(inp)
        prm = [_c(p) for p in prm]
        out, saved = fno_forward(meta, inp, prm, save=True)
        ctx.meta = meta
        x0, Xs, Wts, zs = saved
        ctx.n = len(Xs)
        ctx.save_for_backward(inp, x0, *Xs, *Wts, *zs, *prm)
        return out

    @staticmethod
    def backward(ctx, gout):
        meta, n = ctx.meta, ctx.n
        t = ctx.saved_tensors
        inp, x0 = t[0], t[1]
        Xs, Wts, zs = list(t[2:2 + n]), list(t[2 + n:2 + 2 * n]), list(t[2 + 2 * n:2 + 3 * n])
        prm = list(t[2 + 3 * n:])
        d_inp, grads = fno_backward(meta, inp, prm, (x0, Xs, Wts, zs), gout,
                                    ctx.needs_input_grad[1])
        grads = [g if ctx.needs_input_grad[2 + i] else None for i, g in enumerate(grads)]
        return (None, d_inp, *grads)


# ---------------------------------------------------------------------------- grouped heads
# Two FNO2d heads on the same input run as ONE chain of launches over 2 B samples: every
# kernel selects the weights of the sample's head (blindno_*_g entry points): head g's copy of a
# small weight (fc0, 1x1 convs, fc1/fc2) at base + g S.  When the heads' parameters sit at one
# fixed distance in memory (FlatAdam's flat buffer: both heads' parameter lists have the same
# layout) the kernels read them in place; otherwise they are packed into one buffer per step
# (one copy kernel).  The spectral weights go into one packed Wt per layer.


def _small_params(prm, n, nw):
    """[fc0w, fc0b, (cw, cb) * n, fc1w, fc1b, fc2w, fc2b] out of an FNO parameter list."""
    out = [prm[0], prm[1]]
    for k in range(n):
        off = 2 + k * (nw + 2)
        out += [prm[off + nw], prm[off + nw + 1]]
    off = 2 + n * (nw + 2)
    return out + list(prm[off:off + 4])


def _offsets(tensors):
    offs, o = [], 0
    for t in tensors:
        offs.append(o)
        o += t.numel()
    return offs, o


def pack_heads_ahead(meta: FNOMeta, shape, prms, device):
    """Request the grouped heads' spectral weight pack (fno_forward_grouped's) ahead of the
    forward that reaches them, for input ``shape`` (Bg, N1, N2, width)."""
    if not (GROUPED_HEADS and grouped_ok(meta, shape, prms)):
        return
    G, n = len(prms), meta.n_layers
    P1 = _fno_geometry(shape, meta)[4]
    K1 = kept_rows_count(meta.m1, P1)
    C = meta.width
    Wt_all = torch.empty(n, G, meta.m2, K1, C, C, 2, dtype=F32, device=device)
    segs = [(prms[g][2 + 4 * k], prms[g][3 + 4 * k]) for k in range(n) for g in range(G)]
    pack_ahead(segs, [Wt_all[k, g] for k in range(n) for g in range(G)], P1, Wt_all)


def grouped_ok(meta: FNOMeta, inp, prms) -> bool:
    if meta.dim != 2 or len(prms) != 2:
        return False
    n = meta.n_layers
    fc1w, fc2w = prms[0][2 + 4 * n], prms[0][4 + 4 * n]
    Hd, Cout = fc1w.shape[0], fc2w.shape[0]
    if Hd != 128 or meta.width > 15 or Cout > 2:
        return False
    if any(a.shape != b.shape for a, b in zip(prms[0], prms[1])):
        return False
    Bg, N1, N2, Cin, P1, P2, Ho, Wo = _fno_geometry(inp, meta)
    # grouped projection steps stay within one head; grouped row-inverse quads within a sample
    return (Bg * Ho * Wo) % 64 == 0 and P1 % 4 == 0


def _sub(buf, off):
    return buf[off:] if off else buf


class _GroupWeights:
    """The grouped heads' small weights: ``p(i)`` = the device pointer of head 0's tensor i,
    head g's at + g * S floats."""

    def __init__(self, smalls):
        d = None
        direct = all(t.is_contiguous() and t.dtype == F32 for sm in smalls for t in sm)
        for g in range(1, len(smalls)):
            for a, b in zip(smalls[0], smalls[g]):
                diff = b.data_ptr() - a.data_ptr()
                if diff % (4 * g) or (d is not None and diff != g * d):
                    direct = False
                    break
                d = diff // g
        if direct and d:
            self.base, self.buf, self.S = list(smalls[0]), None, d // 4
        else:
            self.offs, self.S = _offsets(smalls[0])
            self.buf = torch.cat([t.reshape(-1) for sm in smalls for t in sm])
            self.base = None

    def p(self, i):
        return ptr(self.base[i]) if self.base is not None else ptr(_sub(self.buf, self.offs[i]))


def fno_forward_grouped(meta: FNOMeta, inp, prms, bag=None):
    """Both heads' FNO2d forward in one chain; returns (out (Bg, Ho, Wo, G*Cout), saved).
    ``bag`` (BagHeadsIn): inp is the bag mean ubar, the lift forms the heads' input."""
    G = len(prms)
    Bg, N1, N2, Cin, P1, P2, Ho, Wo = _fno_geometry(inp if bag is None else bag.shape(inp), meta)
    Bn = G * Bg
    C, n = meta.width, meta.n_layers
    smalls = [_small_params(p, n, 2) for p in prms]
    small = _GroupWeights(smalls)
    S = small.S
    x0 = _empty(Bn, C, P1, P2, like=inp)
    if bag is None:
        call("blindno_lift_fwd_g", ptr(inp), small.p(0), small.p(1), ptr(x0),
             G, S, Bn, N1, N2, Cin, C, P1, P2, stream_ptr())
    else:
        call("blindno_lift_fwd_bag_g", None, small.p(0), small.p(1), ptr(x0), G, S, Bn, N1, N2, Cin, C,
             P1, P2, ptr(inp), ptr(bag.grid), ptr(bag.w), ptr(bag.b), 1.0, stream_ptr())
    K1 = kept_rows_count(meta.m1, P1)
    K1p = 16 * ((K1 + 15) // 16)
    FB, GB = twiddle_cols(P1, meta.m1, inp.device)
    src, act = x0, 0
    Xs, Wts, zs = [], [], []
    # every layer's spectral weights of both heads in one launch: Wt_all[k] = (G, m2, K1, C, C, 2)
    segs = [(prms[g][2 + 4 * k], prms[g][3 + 4 * k]) for k in range(n) for g in range(G)]
    Wt_all = take_packed(segs, P1)                 # packed ahead (pack_heads_ahead)?
    if Wt_all is None:
        Wt_all = _empty(n, G, meta.m2, K1, C, C, 2, like=inp)
        _pack_into(segs, [Wt_all[k, g] for k in range(n) for g in range(G)], P1)
    for k in range(n):
        Wt = Wt_all[k]
        At = k_rowdft(src, Bn, C, P1, P2, meta.m2, act)
        X = _empty(Bn, meta.m2, C, K1, 2, like=inp)
        Y = _empty(Bn, meta.m2, C, K1p, 2, like=inp)
        Z = _empty(Bn, P1, meta.m2, C, 2, like=inp)
        call("blindno_colpass_g", ptr(At), ptr(Wt), ptr(X), ptr(Y), ptr(Z), ptr(FB), ptr(GB), G,
             Wt[0].numel(), Bn, C, C, P1, meta.m1, meta.m2, P2, _mixdir(0), stream_ptr())
        z = _empty(Bn, C, P1, P2, like=inp)
        call("blindno_rowidft_epi_g", ptr(Z), ptr(src), small.p(2 + 2 * k),
             small.p(3 + 2 * k), ptr(z), ptr(twiddle_rowinv(P2, meta.m2, inp.device)),
             G, S, Bn, C, P1, P2, meta.m2, act, stream_ptr())
        Xs.append(X)
        Wts.append(Wt)
        zs.append(z)
        src, act = z, 1
    o1 = 2 + 2 * n
    Hd, Cout = smalls[0][o1].shape[0], smalls[0][o1 + 2].shape[0]
    out = _empty(Bg, Ho, Wo, G * Cout, like=inp)
    call("blindno_project_fwd_g", ptr(zs[-1]), small.p(o1), small.p(o1 + 1),
         small.p(o1 + 2), small.p(o1 + 3), ptr(out), G, S, Bn, C, P1, P2,
         Ho, Wo, Hd, Cout, G * Cout, 0, stream_ptr())
    return out, (small, x0, Xs, Wts, zs)


# The grouped heads' projection backward writes dz on the Ho x Wo crop only and its readers need
# zeros on the padding: one persistent buffer per shape whose padding is zeroed once (no fill
# kernel per step).  Created outside stream capture (GraphedBagStep's eager warm-up) so a graph
# references ordinary pool memory, never its own pool; a miss during capture falls back to a
# captured fill.  Only the single-chain grouped path uses it (the forked heads run two streams).
_DZ_PAD = {}


def _padded_grad_buffer(shape, device):
    key = (tuple(shape), str(device))
    t = _DZ_PAD.get(key)
    if t is None:
        t = torch.zeros(shape, dtype=F32, device=device)
        if not torch.cuda.is_current_stream_capturing():
            _DZ_PAD[key] = t
    return t


def fno_backward_grouped(meta: FNOMeta, inp, prms, saved, gout, need_inp_grad, bag=None):
    """Adjoint of fno_forward_grouped: (d_inp summed over the heads, [grads of head g]); with
    ``bag`` d_inp is d ubar."""
    G = len(prms)
    Bg, N1, N2, Cin, P1, P2, Ho, Wo = _fno_geometry(inp if bag is None else bag.shape(inp), meta)
    Bn = G * Bg
    C, n = meta.width, meta.n_layers
    small, x0, Xs, Wts, zs = saved
    smalls = [_small_params(p, n, 2) for p in prms]
    S = small.S
    o1 = 2 + 2 * n
    Hd, Cout = smalls[0][o1].shape[0], smalls[0][o1 + 2].shape[0]
    gout = _c(gout)
    grads = [[None] * len(p) for p in prms]
    off_fc1 = 2 + 4 * n
    # projection
    dz = _padded_grad_buffer((Bn, C, P1, P2), inp.device)
    np_p = Hd * C + Hd + Cout * Hd + Cout
    nchunk = query("blindno_project_bwd_nchunk_heads", Bg, Ho, Wo)
    partial = _empty(nchunk, G, np_p, like=inp)
    call("blindno_project_bwd_g", ptr(zs[-1]), small.p(o1), small.p(o1 + 1),
         small.p(o1 + 2), ptr(gout), ptr(dz), ptr(partial), nchunk, G, S, Bn, C, P1, P2,
         Ho, Wo, Hd, Cout, G * Cout, 0, stream_ptr())
    gp = reduce_partials(partial, nchunk, G * np_p).view(G, np_p)
    for g in range(G):
        o = 0
        grads[g][off_fc1] = gp[g, o:o + Hd * C].view(Hd, C); o += Hd * C
        grads[g][off_fc1 + 1] = gp[g, o:o + Hd]; o += Hd
        grads[g][off_fc1 + 2] = gp[g, o:o + Cout * Hd].view(Cout, Hd); o += Cout * Hd
        grads[g][off_fc1 + 3] = gp[g, o:o + Cout]
    K1 = kept_rows_count(meta.m1, P1)
    K1p = 16 * ((K1 + 15) // 16)
    FB, GB = twiddle_cols(P1, meta.m1, inp.device)
    tb = twiddle_rowinv(P2, meta.m2, inp.device)
    np_c = C * C + C
    ns = query("blindno_mix_wgrad_nsplit", Bg, C, C, K1, meta.m2)
    nch = query("blindno_conv_wgrad_nchunk", Bg, P1, P2)
    # one launch per layer for the row DFT of dz, the conv gradient and the previous layer's
    # spectral weight gradient (blindno_rowdft_wgrad_g); the last layer's mix gradient after
    # the loop
    merged = HEAD_BWD_MERGED and query("blindno_rowdft_wgrad_ok", Bn, C, P1, P2, meta.m2) == 1
    pending = None                  # (layer, Xs, Gs) whose mix gradient is not launched yet

    def mix_buffers():
        dWt = _empty(G, meta.m2, K1, C, C, 2, like=inp)
        part = _empty(ns, G, meta.m2 * K1 * C * C * 2, like=inp) if ns > 1 else None
        return dWt, part

    def mix_grads(kk, dWt):
        o = 2 + 4 * kk
        if _DEFER is not None:
            dws = [d for g in range(G) for d in unpack_w2d(dWt[g], prms[g][o], P1)]
        else:
            dws = [torch.empty_like(prms[g][o]) for g in range(G) for _ in range(2)]
            call("blindno_unpack_w2d_2", ptr(dWt), ptr(dws[0]), ptr(dws[1]), ptr(dws[2]), ptr(dws[3]), C,
                 C, meta.m1, meta.m2, P1, stream_ptr())
        for g in range(G):
            grads[g][o], grads[g][o + 1] = dws[2 * g], dws[2 * g + 1]

    # hosted in the merged launches (the next layer's row DFT, the lift backward for the last);
    # otherwise, under deferred_reductions(), the mix gradients join the batched finalisation
    defer_mix = _DEFER is not None and not merged

    def mix_launch(kk, Xk, Gk):
        dWt, part = mix_buffers()
        if defer_mix:
            _DEFER.mix.append((Xk, Gk, part if ns > 1 else dWt, (Bn, C, C, K1, meta.m2, ns, G)))
            if ns > 1:
                _DEFER.red.append([part, dWt, ns, dWt.numel(), []])
        else:
            call("blindno_mix_wgrad_g", ptr(Xk), ptr(Gk), ptr(dWt), ptr(part) if part is not None else None,
                 ns, G, Bn, C, C, K1, meta.m2, stream_ptr())
        mix_grads(kk, dWt)

    for k in reversed(range(n)):
        off = 2 + 4 * k
        src, act = (x0, 0) if k == 0 else (zs[k - 1], 1)
        Wt = Wts[k]
        pc = _empty(nch, G, np_c, like=inp)
        if merged:
            At = _empty(Bn, meta.m2, C, P1, 2, like=inp)
            mx = (None, None, None, None)
            if pending is not None:
                dWt, part = mix_buffers()
                mx = (pending[1], pending[2], dWt, part)
            call("blindno_rowdft_wgrad_g", ptr(dz), ptr(src), ptr(At), ptr(twiddle_mfma(P2, meta.m2, inp.device)),
                 ptr(pc), nch, act, *[ptr(t) if t is not None else None for t in mx], ns, K1, G, Bn, C,
                 P1, P2, meta.m2, stream_ptr())
            if pending is not None:
                mix_grads(pending[0], dWt)
        else:
            At = k_rowdft(dz, Bn, C, P1, P2, meta.m2, 0)
        Gs = _empty(Bn, meta.m2, C, K1, 2, like=inp)
        Y = _empty(Bn, meta.m2, C, K1p, 2, like=inp)
        GZ = _empty(Bn, P1, meta.m2, C, 2, like=inp)
        call("blindno_colpass_g", ptr(At), ptr(Wt), ptr(Gs), ptr(Y), ptr(GZ), ptr(FB), ptr(GB), G,
             Wt[0].numel(), Bn, C, C, P1, meta.m1, meta.m2, P2, _mixdir(1), stream_ptr())
        if merged and not defer_mix:
            pending = (k, Xs[k], Gs)
        else:
            mix_launch(k, Xs[k], Gs)
            if not merged:
                call("blindno_conv_wgrad_g", ptr(dz), ptr(src), ptr(pc), nch, G, Bn, C, P1, P2, act,
                     stream_ptr())
        gc = reduce_partials(pc, nch, G * np_c).view(G, np_c)
        for g in range(G):
            grads[g][off + 2] = gc[g, :C * C].view_as(prms[g][off + 2])
            grads[g][off + 3] = gc[g, C * C:]
        dz_new = _empty(Bn, C, P1, P2, like=inp)
        call("blindno_rowidft_bwd_g", ptr(GZ), ptr(dz), small.p(2 + 2 * k), ptr(src),
             ptr(dz_new), ptr(tb), G, S, Bn, C, P1, P2, meta.m2, act, stream_ptr())
        dz = dz_new
    np_l = C * Cin + C
    nchunk = query("blindno_lift_bwd_nchunk", Bg, N1, N2)
    partial = _empty(nchunk, G, np_l, like=inp)
    d_inp = torch.empty_like(inp) if need_inp_grad else None
    mx = (None, None, None, None)
    if pending is not None:            # the first layer's mix gradient in the lift's launch
        dWt, part = mix_buffers()
        mx = (pending[1], pending[2], dWt, part)
    if bag is None:
        call("blindno_lift_bwd_mix_g", ptr(dz), ptr(inp), small.p(0), ptr(d_inp), ptr(partial), nchunk, G,
             S, Bn, N1, N2, Cin, C, P1, P2, *[ptr(t) if t is not None else None for t in mx], ns, K1,
             meta.m2, stream_ptr())
    else:
        if d_inp is None:
            d_inp = torch.empty_like(inp)       # the merged kernel always forms d ubar
        call("blindno_lift_bwd_bag_mix_g", ptr(dz), None, small.p(0), ptr(d_inp), ptr(partial), nchunk,
             G, S, Bn, N1, N2, Cin, C, P1, P2, *[ptr(t) if t is not None else None for t in mx], ns,
             K1, meta.m2, ptr(inp), ptr(bag.grid), ptr(bag.w), ptr(bag.b), 1.0, 1.0, stream_ptr())
    if pending is not None:
        mix_grads(pending[0], dWt)
    gl = reduce_partials(partial, nchunk, G * np_l).view(G, np_l)
    for g in range(G):
        grads[g][0] = gl[g, :C * Cin].view(C, Cin)
        grads[g][1] = gl[g, C * Cin:]
    return d_inp, grads


GROUPED_HEADS = True    # batch the two heads into one chain of grouped launches when possible


class HeadPairFn(torch.autograd.Function):
    """Two FNO heads on the same input h (2d_FPE/NIOModules.py:577-581: cat of fno_drift and
    fno_diffusion), forward AND backward forked over two HIP streams: head 0 on the current
    stream, head 1 on ``side`` (waiting on the current stream first, joined back after).  The
    heads are small (B samples), latency-bound chains of launches, so the two chains overlap;
    doing the backward fork here rather than relying on autograd's per-node streams keeps the
    two backward chains concurrent (inside a graph capture: two parallel branches)."""

    @staticmethod
    def forward(ctx, meta0, meta1, n0, side, h, *prm):
        """``meta0`` may be (meta0, BagHeadsIn): h is then the bag mean ubar (grouped path)."""
        bag = None
        if isinstance(meta0, tuple):
            meta0, bag = meta0
        require_device(h, *prm)
        h = _c(h)
        prm = [_c(p) for p in prm]
        p0, p1 = prm[:n0], prm[n0:]
        hin = h if bag is None else bag.shape(h)
        ctx.grouped = GROUPED_HEADS and meta0.__dict__ == meta1.__dict__ and grouped_ok(meta0, hin, [p0, p1])
        ctx.bag = bag
        if bag is not None and not ctx.grouped:
            raise BlindnoError("HeadPairFn: a bag-mean input needs the grouped heads")
        if ctx.grouped:
            out, saved = fno_forward_grouped(meta0, h, [p0, p1], bag=bag)
            ctx.save_for_backward(h, *prm)
            ctx.meta = (meta0, meta1, n0, side, None)
            ctx.s0, ctx.s1 = saved, None
            return out
        main = torch.cuda.current_stream(h.device)
        side.wait_stream(main)
        o0, s0 = fno_forward(meta0, h, p0, save=True)
        with torch.cuda.stream(side):
            o1, s1 = fno_forward(meta1, h, p1, save=True)
        main.wait_stream(side)
        h.record_stream(side)
        o1.record_stream(main)
        out = torch.cat([o0, o1], dim=-1)
        ctx.save_for_backward(h, *prm)
        ctx.meta = (meta0, meta1, n0, side, o0.shape[-1])
        ctx.s0, ctx.s1 = s0, s1
        return out

    @staticmethod
    def backward(ctx, gout):
        meta0, meta1, n0, side, c0 = ctx.meta
        t = ctx.saved_tensors
        h, prm = t[0], list(t[1:])
        p0, p1 = prm[:n0], prm[n0:]
        need = ctx.needs_input_grad[4]
        gout = _c(gout)
        if ctx.grouped:
            dh, gr = fno_backward_grouped(meta0, h, [p0, p1], ctx.s0, gout, need, bag=ctx.bag)
            ctx.s0 = ctx.bag = None
            grads = [g if ctx.needs_input_grad[5 + i] else None for i, g in enumerate(gr[0] + gr[1])]
            return (None, None, None, None, dh, *grads)
        g0 = gout[..., :c0].contiguous()
        g1 = gout[..., c0:].contiguous()
        main = torch.cuda.current_stream(h.device)
        side.wait_stream(main)
        # side branch captured first: a graph replay submits nodes in capture order, and the
        # side chain must not queue behind the whole main chain
        with torch.cuda.stream(side):
            d1, gr1 = fno_backward(meta1, h, p1, ctx.s1, g1, need)
        d0, gr0 = fno_backward(meta0, h, p0, ctx.s0, g0, need)
        main.wait_stream(side)
        g1.record_stream(side)
        for g in ([d1] if d1 is not None else []) + [g for g in gr1 if g is not None]:
            g.record_stream(main)
        ctx.s0 = ctx.s1 = None
        dh = d0 + d1 if need else None
        grads = [g if ctx.needs_input_grad[5 + i] else None for i, g in enumerate(gr0 + gr1)]
        return (None, None, None, None, dh, *grads)


# ---------------------------------------------------------------------------- fused snapshot encoder


def k_rowdft_bag_lift(X, idx_t, w0, b0, Dg, B, T, L, N1, N2, C, P1, P2, m2):
    """Row DFT of the encoder's lifted first-layer input for every snapshot of the bag; the
    grid/bias part is formed in the kernel from the grid-plane spectra Dg (_grid_planes)."""
    At = _empty(B * L, m2, C, P1, 2, like=X)
    call("blindno_rowdft_bag_lift_dg", ptr(X), ptr(idx_t), ptr(w0), ptr(b0), ptr(Dg), ptr(At),
         ptr(twiddle_mfma(P2, m2, X.device)), B, T, L, N1, N2, C, P1, P2, m2, stream_ptr())
    return At


_DG_CACHE = {}


def _grid_planes(grid, N1, N2, P1, P2, m2):
    """Row spectra Dg (m2, 3, P1, 2) of the planes gx, gy and 1 on the N1 x N2 crop (zero on the
    padding): the encoder's grid/bias part W0[:,1] gx + W0[:,2] gy + b0 is linear in them, so
    its spectrum is formed per step inside the bag-lift row DFT from Dg and the CURRENT fc0
    (which is trained) -- no per-step lift / row DFT / concat.  Dg depends on the grid only and
    is cached, keyed by its storage and version; a miss during a graph capture computes it
    inside the graph without caching (the capture does not execute it)."""
    key = (grid.device, grid.data_ptr(), grid._version, N1, N2, P1, P2, m2)
    capturing = torch.cuda.is_current_stream_capturing()
    hit = _DG_CACHE.get(key)
    if hit is not None:
        return hit[-1]
    # the planes through the lift kernel: weights [[1, 0], [0, 1], [0, 0]], bias [0, 0, 1]
    w = torch.tensor([[1.0, 0.0], [0.0, 1.0], [0.0, 0.0]], dtype=F32, device=grid.device)
    b = torch.tensor([0.0, 0.0, 1.0], dtype=F32, device=grid.device)
    g0 = _empty(1, 3, P1, P2, like=grid)
    call("blindno_lift_fwd", ptr(_c(grid)), ptr(w), ptr(b), ptr(g0), 1, N1, N2, 2, 3, P1, P2,
         stream_ptr())
    Dg = k_rowdft(g0, 1, 3, P1, P2, m2, 0)
    if not capturing:
        if len(_DG_CACHE) > 16:
            _DG_CACHE.clear()
        # the entry holds the grid too, so its storage (part of the key) is never reused
        _DG_CACHE[key] = (grid, Dg)
    return Dg


_DG2_CACHE = {}


def _grid_spec2(grid, N1, N2, P1, P2, m1, m2):
    """Column spectra Dg2 (m2, 3, K1) complex of the grid / bias planes gx, gy, 1 on the crop
    (the 2D counterpart of _grid_planes, for the folded column pass: the encoder's first-layer
    spectrum is W0[:,0] U + W0[:,1] Dg2[0] + W0[:,2] Dg2[1] + b0 Dg2[2]); cached like Dg."""
    key = (grid.device, grid.data_ptr(), grid._version, N1, N2, P1, P2, m1, m2)
    hit = _DG2_CACHE.get(key)
    if hit is not None:
        return hit[-1]
    capturing = torch.cuda.is_current_stream_capturing()
    w = torch.tensor([[1.0, 0.0], [0.0, 1.0], [0.0, 0.0]], dtype=F32, device=grid.device)
    b = torch.tensor([0.0, 0.0, 1.0], dtype=F32, device=grid.device)
    g0 = _empty(1, 3, P1, P2, like=grid)
    call("blindno_lift_fwd", ptr(_c(grid)), ptr(w), ptr(b), ptr(g0), 1, N1, N2, 2, 3, P1, P2,
         stream_ptr())
    nb = P1 // 16
    part = _empty(nb * query("blindno_colspec_nchunk", 3, m2) * 128, like=grid)
    call("blindno_rowdft_cd", ptr(g0), ptr(part), ptr(twiddle_mfma(P2, m2, grid.device)),
         ptr(twiddle_colspec(P1, m1, grid.device)), 1, 3, P1, P2, m2, 0, P1, P2, stream_ptr())
    K1 = kept_rows_count(m1, P1)
    Dg2 = _empty(1, m2, 3, K1, 2, like=grid)
    call("blindno_colmix", ptr(part), nb, None, ptr(Dg2), None, 1, 3, 3, P1, P2, m1, m2, 0, None, None,
         None, stream_ptr())
    if not capturing:
        if len(_DG2_CACHE) > 16:
            _DG2_CACHE.clear()
        _DG2_CACHE[key] = (grid, Dg2)
    return Dg2


class _ColSpec:
    """Launch helpers of the folded column pass for one encoder geometry (csrc/colspec.h)."""

    def __init__(self, Bn, C, P1, P2, m1, m2, device):
        self.Bn, self.C, self.P1, self.P2, self.m1, self.m2 = Bn, C, P1, P2, m1, m2
        self.K1 = kept_rows_count(m1, P1)
        self.nb = P1 // 16
        self.tab = twiddle_colspec(P1, m1, device)
        self.Tp = twiddle_mfma(P2, m2, device)
        self.tb = twiddle_rowinv(P2, m2, device)

    def part(self, Cp, like):
        return _empty(self.Bn * self.nb * query("blindno_colspec_nchunk", Cp, self.m2) * 128, like=like)

    def mix(self, part, nbv, Wt, direction, Cp=None, lift=None):
        """(Xsave, Y) of the summed partials: direction 0 (X, Y = mix) or 1 (G, conj mix)."""
        Xs = _empty(self.Bn, self.m2, self.C, self.K1, 2, like=part)
        Y = _empty(self.Bn, self.m2, self.C, self.K1, 2, like=part)
        w0, b0, Dg2 = lift if lift is not None else (None, None, None)
        call("blindno_colmix", ptr(part), nbv, ptr(Wt), ptr(Xs), ptr(Y), self.Bn, self.C,
             Cp or self.C, self.P1, self.P2, self.m1, self.m2, direction, ptr(w0), ptr(b0), ptr(Dg2),
             stream_ptr())
        return Xs, Y


def _bag_stats_ok(B, L, C, P1, P2, Ho, Wo, Hd, Cout):
    """The bag-level projection (csrc/bagproj.hip) applies: fc1 of 128, one output channel."""
    if not (BAG_STATS and Hd == 128 and Cout == 1 and L <= 1024):
        return False
    nstats = query("blindno_project_bag_stats_floats", B, Ho, Wo)
    return 4 * (nstats + B * L * C * P1 * P2) <= BAG_STATS_MAX_BYTES


def bag_ubar_ok(meta, B, L, N1, N2, fc1w, fc2w, head_meta, G, width):
    """BagEncoderFn can hand its heads the bag mean ubar itself (emit_ubar), and the G grouped
    heads' lift kernels take it (blindno_lift_bag_ok: the 12-channel wide lift forms)."""
    fake = (B * L, N1, N2, 3)
    _, _, _, _, P1, P2, Ho, Wo = _fno_geometry(fake, meta)
    if not _bag_stats_ok(B, L, meta.width, P1, P2, Ho, Wo, fc1w.shape[0], fc2w.shape[0]):
        return False
    hP1, hP2 = _fno_geometry((B, N1, N2, width), head_meta)[4:6]
    return query("blindno_lift_bag_ok", G, G * B, N1, N2, width, head_meta.width, hP1, hP2) == 1


class BagHeadsIn:
    """The grouped heads' input given as the bag mean of the snapshot projections ubar (B, N1,
    N2) plus the fixed fc0 (bw (width, 3), bb) that maps [gx, gy, ubar] to the heads' width
    (NIOFP2D_FNO, 2d_FPE/NIOModules.py:569-575): the heads' lift forms that field on the fly
    and its adjoint returns d ubar (blindno_lift_fwd_bag_g / blindno_lift_bwd_bag_mix_g), so
    neither the (B, N1, N2, width) field nor the bag-mean launches exist.  Passed to
    HeadPairFn as (meta0, BagHeadsIn)."""

    def __init__(self, grid, bw, bb):
        self.grid, self.w, self.b = _c(grid), _c(bw.detach()), _c(bb.detach())
        self.width = bw.shape[0]

    def shape(self, ubar):
        return (ubar.shape[0], ubar.shape[1], ubar.shape[2], self.width)


class BagEncoderFn(torch.autograd.Function):
    """The snapshot-bag encoder of NIOFP2D_FNO as ONE autograd node (2d_FPE/NIOModules.py:
    548-575): FNO_input (an FNO2d of input [u, gx, gy]) on every snapshot of the bag, then the
    fixed-weight bag mean.  Snapshots are read straight from the bag tensor X (B, T, N1, N2)
    through the device index list idx_t (the bag draw); the gathered bag, the concatenated
    input and the lifted field x0 are never materialised (the lift is folded into the first
    row DFT and recomputed in the first layer's epilogue / adjoint, which also reduces fc0's
    gradient).  The bag mean's gradient reaches the projection as a per-bag field (dout_div =
    L) instead of an L-fold broadcast copy.  No gradient flows to X or grid (the caller uses
    the generic path when they require one).

    ``lw`` (optional, device float (L,)): the bag is given as its UNIQUE snapshots idx_t with
    weights lw = multiplicity / L_drawn (the draw is with replacement, so ~30% of a bag repeats
    a snapshot whose FNO_input output is identical): every encoder kernel runs on the unique
    snapshots only, the bag mean weights them by lw, and the projection backward scales the
    per-bag gradient by lw (exact up to fp32 summation order)."""

    @staticmethod
    def forward(ctx, meta, emit_ubar, X, idx_t, lw, grid, bw, bb, *prm):
        """``emit_ubar``: return the bag mean of the projections ubar (B, N1, N2) instead of the
        fc0 (bw, bb) of [grid, ubar] -- the grouped heads form that field themselves
        (BagHeadsIn); only where bag_ubar_ok holds."""
        require_device(X, grid, *prm)
        X, grid = _c(X), _c(grid)
        prm = [_c(p) for p in prm]
        bw, bb = _c(bw.detach()), _c(bb.detach())
        B, T, N1, N2 = X.shape
        L = idx_t.numel()
        Bn = B * L
        fake = torch.empty((Bn, N1, N2, 3), device="meta")
        _, _, _, _, P1, P2, Ho, Wo = _fno_geometry(fake, meta)
        C, n = meta.width, meta.n_layers
        if C > 4 or meta.dim != 2 or n < 1:
            raise BlindnoError("BagEncoderFn: needs a 2D FNO of width <= 4")
        fc0w, fc0b = prm[0], prm[1]
        sh = SpecShape(Bn, C, C, P1, P2, meta.m1, meta.m2, 2)
        Xs, Wts, zs = [], [], []
        cs = _ColSpec(Bn, C, P1, P2, meta.m1, meta.m2, X.device) \
            if colspec_ok(Bn, C, P1, P2, meta.m1, meta.m2) else None
        ctx.cs = cs
        Wts_all = pack_w2d_many([(prm[2 + 4 * k], prm[3 + 4 * k]) for k in range(n)], P1,
                                defer=HOST_PACK and cs is not None)
        if cs is not None:
            # the column pass folded into the row kernels: per layer, the kernel that forms the
            # row spectrum leaves its column-DFT partials, blindno_colmix forms Xs and the mixed Y,
            # and the row inverse rebuilds its row coefficients from Y
            try:
                Dg2 = _grid_spec2(grid, N1, N2, P1, P2, meta.m1, meta.m2)
                part = cs.part(1, X)
            finally:            # never leave the held-back pack behind (its Wts die with us)
                pk = take_deferred_pack()
            if pk is not None:      # the pack rides along the first row DFT (colmix reads it)
                call("blindno_rowdft_bag_lift_cd_pack", ptr(X), ptr(idx_t), ptr(part), ptr(cs.Tp),
                     ptr(cs.tab), B, T, L, N1, N2, P1, P2, meta.m2, *pk, stream_ptr())
            else:
                call("blindno_rowdft_bag_lift_cd", ptr(X), ptr(idx_t), ptr(part), ptr(cs.Tp), ptr(cs.tab),
                     B, T, L, N1, N2, P1, P2, meta.m2, stream_ptr())
            nbv = (N1 + 15) // 16
            for k in range(n):
                off = 2 + k * 4
                cw, cb = prm[off + 2], prm[off + 3]
                Wt = Wts_all[k]
                last = k == n - 1
                Xk, Y = cs.mix(part, nbv, Wt, 0, Cp=1 if k == 0 else C,
                               lift=(fc0w, fc0b, Dg2) if k == 0 else None)
                z = _empty(Bn, C, P1, P2, like=X)
                part = None if last else cs.part(C, X)
                if k == 0:
                    call("blindno_rowidft_epi_lift_zc", ptr(Y), ptr(X), ptr(idx_t), ptr(grid), ptr(fc0w),
                         ptr(fc0b), ptr(cw), ptr(cb), ptr(z), ptr(cs.tb), ptr(cs.tab), ptr(part), ptr(cs.Tp),
                         B, T, L, N1, N2, C, P1, P2, meta.m1, meta.m2, 1, stream_ptr())
                else:
                    # the last layer is read by the projection on its crop only
                    oN1, oN2 = (Ho, Wo) if last else (P1, P2)
                    call("blindno_rowidft_epi_zc", ptr(Y), ptr(zs[-1]), ptr(cw), ptr(cb), ptr(z), ptr(cs.tb),
                         ptr(cs.tab), ptr(part), ptr(cs.Tp), Bn, C, P1, P2, meta.m1, meta.m2, 1, 1, oN1, oN2,
                         stream_ptr())
                nbv = P1 // 16
                Xs.append(Xk)
                Wts.append(Wt)
                zs.append(z)
        Dg = _grid_planes(grid, N1, N2, P1, P2, meta.m2) if cs is None else None
        # each row inverse but the last also takes the next layer's row DFT of GELU(z) in its
        # pass (the field is not read back for it)
        At_next = None
        for k in range(n if cs is None else 0):
            off = 2 + k * 4
            w1, w2, cw, cb = prm[off:off + 4]
            Wt = Wts_all[k]
            last = k == n - 1
            if k == 0:
                At = k_rowdft_bag_lift(X, idx_t, fc0w, fc0b, Dg, B, T, L, N1, N2, C, P1, P2, meta.m2)
                Xk, Z = k_colpass(At, Wt, Bn, C, C, P1, meta.m1, meta.m2, P2, 0)
                z = _empty(Bn, C, P1, P2, like=X)
                tb = ptr(twiddle_rowinv(P2, meta.m2, X.device))
                if last:
                    call("blindno_rowidft_epi_lift", ptr(Z), ptr(X), ptr(idx_t), ptr(grid), ptr(fc0w),
                         ptr(fc0b), ptr(cw), ptr(cb), ptr(z), tb, B, T, L, N1, N2, C, P1, P2,
                         meta.m2, stream_ptr())
                else:
                    At_next = _empty(Bn, meta.m2, C, P1, 2, like=X)
                    call("blindno_rowidft_epi_lift_rd", ptr(Z), ptr(X), ptr(idx_t), ptr(grid),
                         ptr(fc0w), ptr(fc0b), ptr(cw), ptr(cb), ptr(z), tb, B, T, L, N1, N2, C, P1,
                         P2, meta.m2, ptr(At_next), ptr(twiddle_mfma(P2, meta.m2, X.device)), 1,
                         stream_ptr())
            else:
                Xk, Z = spec_forward(zs[-1], 1, Wt, sh, At=At_next)
                if last:
                    # the projection reads the output on its crop only: write nothing else
                    z = _empty(Bn, C, P1, P2, like=X)
                    call("blindno_rowidft_epi_crop", ptr(Z), ptr(zs[-1]), ptr(cw), ptr(cb), ptr(z),
                         ptr(twiddle_rowinv(P2, meta.m2, X.device)), Bn, C, P1, P2, meta.m2, 1, Ho, Wo,
                         stream_ptr())
                else:
                    z, At_next = k_rowidft_epi_rd(Z, zs[-1], cw, cb, Bn, C, P1, P2, meta.m2, 1, 1)
            Xs.append(Xk)
            Wts.append(Wt)
            zs.append(z)
        fc1w, fc1b, fc2w, fc2b = prm[2 + 4 * n:6 + 4 * n]
        Hd, Cout = fc1w.shape[0], fc2w.shape[0]
        S = Ho * Wo
        width = bw.shape[0]
        h = _empty(B, S, width, like=X)
        ctx.bag = None
        if _bag_stats_ok(B, L, C, P1, P2, Ho, Wo, Hd, Cout):
            # projection + bag mean at bag level: the backward becomes a reduction of the
            # statistics the forward leaves (csrc/bagproj.hip).  stats and v are fresh buffers
            # only this forward writes and only this backward reads (never handed to the caller),
            # so they ride on ctx without save_for_backward's version check
            ubar = _empty(B, S, like=X)
            stats = _empty(query("blindno_project_bag_stats_floats", B, Ho, Wo), like=X)
            v = _empty(Bn, C, P1, P2, like=X)
            call("blindno_project_bag_fwd", ptr(zs[-1]), ptr(fc1w), ptr(fc1b), ptr(fc2w), ptr(fc2b),
                 ptr(lw), ptr(ubar), ptr(stats), ptr(v), B, L, C, P1, P2, Ho, Wo, Hd, stream_ptr())
            if not emit_ubar:
                call("blindno_bagmean_fwd_w", ptr(ubar), ptr(grid), ptr(bw), ptr(bb), None, ptr(h), B, 1,
                     S, 2, width, stream_ptr())
            ctx.bag = (stats, v)
        elif emit_ubar:
            raise BlindnoError("BagEncoderFn: emit_ubar needs the bag-level projection (bag_ubar_ok)")
        else:
            u = _empty(Bn, Ho, Wo, Cout, like=X)
            call("blindno_project_fwd", ptr(zs[-1]), ptr(fc1w), ptr(fc1b), ptr(fc2w), ptr(fc2b), ptr(u),
                 Bn, C, P1, P2, Ho, Wo, Hd, Cout, Cout, 0, stream_ptr())
            call("blindno_bagmean_fwd_w", ptr(u), ptr(grid), ptr(bw), ptr(bb), ptr(lw), ptr(h), B, L, S,
                 2, width, stream_ptr())
        ctx.meta, ctx.n, ctx.dims = meta, n, (B, T, L, N1, N2, C, P1, P2, Ho, Wo, Hd, Cout, width)
        ctx.lw = lw
        ctx.emit_ubar = bool(emit_ubar)
        ctx.save_for_backward(X, idx_t, grid, bw, *Xs, *Wts, *zs, *prm)
        if emit_ubar:
            return ubar.view(B, N1, N2)
        return h.view(B, N1, N2, width)

    @staticmethod
    def backward(ctx, gh):
        meta, n = ctx.meta, ctx.n
        B, T, L, N1, N2, C, P1, P2, Ho, Wo, Hd, Cout, width = ctx.dims
        t = ctx.saved_tensors
        X, idx_t, grid, bw = t[:4]
        Xs, Wts, zs = list(t[4:4 + n]), list(t[4 + n:4 + 2 * n]), list(t[4 + 2 * n:4 + 3 * n])
        prm = list(t[4 + 3 * n:])
        Bn, S = B * L, Ho * Wo
        gh = _c(gh)
        grads = [None] * len(prm)
        # bag mean: every snapshot of bag b receives the same gradient s[b] (emit_ubar: the
        # heads' lift adjoint handed back d ubar = s itself)
        lw = ctx.lw
        bag = ctx.bag
        ctx.bag = None
        if ctx.emit_ubar:
            sgr = gh.view(B, S)
        else:
            sgr = _empty(B, S, like=gh)
            call("blindno_bagmean_bwd", ptr(gh), ptr(bw), ptr(sgr), B, S, 2, width,
                 1 if (lw is not None or bag is not None) else L, stream_ptr())
        # projection (dout read per bag: dout_div = L)
        off_fc1 = 2 + 4 * n
        fc1w, fc1b, fc2w = prm[off_fc1:off_fc1 + 3]
        # the projection backward writes dz on the Ho x Wo crop only; with >= 2 layers its two
        # consumers (the last layer's row DFT and row-inverse adjoint) read just that region, so
        # the padding (36% of the field at 128^2) is never zero-filled (88 MB at config C)
        crop = (Ho, Wo) if n >= 2 else None
        cs = ctx.cs
        ctx.cs = None
        # the folded column pass with the bag-level projection: dz = lw_l ghat v is formed on load
        # by its two readers (the last layer's row DFT and row-inverse adjoint), so the projection
        # backward neither writes dz nor reads v (a field write and read less per step)
        bagdz = cs is not None and bag is not None and crop is not None
        dz = None if bagdz else (_empty(Bn, C, P1, P2, like=gh) if crop else
                                 torch.zeros(Bn, C, P1, P2, dtype=F32, device=gh.device))
        np_p = Hd * C + Hd + Cout * Hd + Cout
        nchunk = query("blindno_project_bag_bwd_nchunk" if bag is not None else "blindno_project_bwd_nchunk",
                       B if bag is not None else Bn, Ho, Wo)
        partial = _empty(nchunk, np_p, like=gh)
        if bag is not None:
            call("blindno_project_bag_bwd", ptr(bag[0]), ptr(sgr), ptr(fc2w), ptr(lw), ptr(bag[1]),
                 ptr(dz), ptr(partial), nchunk, B, L, C, P1, P2, Ho, Wo, Hd, stream_ptr())
        elif lw is not None:
            call("blindno_project_bwd_w", ptr(zs[-1]), ptr(fc1w), ptr(fc1b), ptr(fc2w), ptr(sgr), ptr(lw),
                 ptr(dz), ptr(partial), nchunk, Bn, C, P1, P2, Ho, Wo, Hd, Cout, Cout, 0, L, stream_ptr())
        else:
            call("blindno_project_bwd", ptr(zs[-1]), ptr(fc1w), ptr(fc1b), ptr(fc2w), ptr(sgr), ptr(dz),
                 ptr(partial), nchunk, Bn, C, P1, P2, Ho, Wo, Hd, Cout, Cout, 0, L, stream_ptr())
        gp = reduce_partials(partial, nchunk, np_p)
        o = 0
        grads[off_fc1] = gp[o:o + Hd * C].view(Hd, C); o += Hd * C
        grads[off_fc1 + 1] = gp[o:o + Hd]; o += Hd
        grads[off_fc1 + 2] = gp[o:o + Cout * Hd].view(Cout, Hd); o += Cout * Hd
        grads[off_fc1 + 3] = gp[o:o + Cout]
        sh = SpecShape(Bn, C, C, P1, P2, meta.m1, meta.m2, 2)
        fc0w, fc0b = prm[0], prm[1]
        if cs is not None:
            # the folded column pass (forward above): the last layer's adjoint starts from the
            # row DFT + column-DFT partials of dz on its crop; each adjoint row inverse rebuilds
            # its row coefficients from the conj-mixed spectrum and leaves the previous layer's
            # partials; the weight gradient reads the saved spectra as before
            part = cs.part(C, gh)
            valid = crop or (P1, P2)
            if bagdz:
                call("blindno_rowdft_cd_bag", ptr(bag[1]), ptr(sgr), ptr(lw), L, ptr(part), ptr(cs.Tp),
                     ptr(cs.tab), Bn, C, P1, P2, meta.m2, Ho, Wo, stream_ptr())
            else:
                call("blindno_rowdft_cd", ptr(dz), ptr(part), ptr(cs.Tp), ptr(cs.tab), Bn, C, P1, P2, meta.m2,
                     0, valid[0], valid[1], stream_ptr())
            nbv = (valid[0] + 15) // 16
            # the spectral weight gradients of both layers ride along the first layer's adjoint
            # launch (blindno_rowidft_bwd_lift_zc_mix) under deferred_reductions()
            hosted = [] if (_DEFER is not None and HOST_ENC_MIX and n <= 2) else None
            for k in reversed(range(n)):
                off = 2 + 4 * k
                w1, w2, cw, cb = prm[off:off + 4]
                G, Yb = cs.mix(part, nbv, Wts[k], 1)
                dWt = k_mix_wgrad(Xs[k], G, Bn, C, C, sh.K1, meta.m2, deferrable=True, jobs=hosted)
                grads[off], grads[off + 1] = unpack_weights(dWt, (w1, w2), P1, 2)
                dv = crop if (k == n - 1 and crop) else (P1, P2)
                if k > 0:
                    nchunk = query("blindno_colspec_bwd_nchunk", Bn, P1)
                    pw = _empty(nchunk, C * C + C, like=gh)
                    dx = _empty(Bn, C, P1, P2, like=gh)
                    part = cs.part(C, gh)
                    if bagdz and k == n - 1:
                        call("blindno_rowidft_bwd_zc_bag", ptr(Yb), ptr(bag[1]), ptr(sgr), ptr(lw), L, ptr(cw),
                             ptr(zs[k - 1]), ptr(dx), ptr(cs.tb), ptr(cs.tab), ptr(part), ptr(cs.Tp), ptr(pw),
                             Bn, C, P1, P2, meta.m1, meta.m2, 1, Ho, Wo, stream_ptr())
                    else:
                        call("blindno_rowidft_bwd_zc", ptr(Yb), ptr(dz), ptr(cw), ptr(zs[k - 1]), ptr(dx),
                             ptr(cs.tb), ptr(cs.tab), ptr(part), ptr(cs.Tp), ptr(pw), Bn, C, P1, P2, meta.m1,
                             meta.m2, 1, dv[0], dv[1], stream_ptr())
                    g = reduce_partials(pw, nchunk, C * C + C)
                    grads[off + 2], grads[off + 3] = g[:C * C].view_as(cw), g[C * C:]
                    dz = dx
                    nbv = P1 // 16
                else:
                    nchunk = query("blindno_colspec_bwd_nchunk", Bn, P1)
                    npl = C * C + C + 4 * C
                    pl = _empty(nchunk, npl, like=gh)
                    jobs = hosted or []
                    nj = len(jobs)
                    call("blindno_rowidft_bwd_lift_zc_mix", ptr(Yb), ptr(dz), ptr(X), ptr(idx_t), ptr(grid),
                         ptr(fc0w), ptr(fc0b), ptr(cw), ptr(cs.tb), ptr(cs.tab), ptr(pl), B, T, L, N1, N2, C,
                         P1, P2, meta.m1, meta.m2,
                         (ctypes.c_void_p * max(1, nj))(*[j[0].data_ptr() for j in jobs]),
                         (ctypes.c_void_p * max(1, nj))(*[j[1].data_ptr() for j in jobs]),
                         (ctypes.c_void_p * max(1, nj))(*[j[2].data_ptr() for j in jobs]),
                         (ctypes.c_int * max(7, 7 * nj))(*[v for j in jobs for v in j[3]]), nj,
                         stream_ptr())
                    g = reduce_partials(pl, nchunk, npl)
                    grads[off + 2] = g[:C * C].view_as(cw)
                    grads[off + 3] = g[C * C:C * C + C]
                    grads[0] = g[C * C + C:C * C + 4 * C].view(C, 3)
                    grads[1] = g[C * C + 4 * C:]
        At_dz = None          # row DFT of dz taken by the later layer's adjoint pass
        for k in reversed(range(n if cs is None else 0)):
            off = 2 + 4 * k
            w1, w2, cw, cb = prm[off:off + 4]
            valid = crop if k == n - 1 else None
            dWt, GZ = spec_backward(dz, Xs[k], Wts[k], sh, valid, At=At_dz)
            grads[off], grads[off + 1] = unpack_weights(dWt, (w1, w2), P1, 2)
            if k > 0:
                dz, gw, gb, At_dz = k_rowidft_bwd(GZ, dz, cw, zs[k - 1], Bn, C, P1, P2, meta.m2, 1,
                                                  True, valid, rd=True)
                grads[off + 2], grads[off + 3] = gw.view_as(cw), gb
            else:
                nchunk = query("blindno_rowidft_bwd_nchunk", Bn, C, P1, P2, meta.m2)
                npl = C * C + C + 4 * C
                part = _empty(nchunk, npl, like=gh)
                call("blindno_rowidft_bwd_lift", ptr(GZ), ptr(dz), ptr(X), ptr(idx_t), ptr(grid),
                     ptr(fc0w), ptr(fc0b), ptr(cw), ptr(twiddle_rowinv(P2, meta.m2, X.device)),
                     ptr(part), B, T, L, N1, N2, C, P1, P2, meta.m2, stream_ptr())
                g = reduce_partials(part, nchunk, npl)
                grads[off + 2] = g[:C * C].view_as(cw)
                grads[off + 3] = g[C * C:C * C + C]
                grads[0] = g[C * C + C:C * C + 4 * C].view(C, 3)
                grads[1] = g[C * C + 4 * C:]
        ctx.lw = None
        grads = [gr if ctx.needs_input_grad[8 + i] else None for i, gr in enumerate(grads)]
        return (None, None, None, None, None, None, None, None, *grads)


# ---------------------------------------------------------------------------- bag mean


class BagMeanFn(torch.autograd.Function):
    """Fixed-weight snapshot-bag aggregation: u (B, L, S), grid (S, d) -> (B, S, width).
    ``w``/``bias`` are ``fc0.weight.data``/``.bias.data`` (never trained, as in the
    reference, 2d_FPE/NIOModules.py:569-570)."""

    @staticmethod
    def forward(ctx, u, grid, w, bias, lw=None):
        """lw (optional, (L,)): per-snapshot weights replacing 1/L (deduplicated bag)."""
        require_device(u, grid, w, bias)
        u, grid = _c(u), _c(grid)
        w, bias = _c(w.detach()), _c(bias.detach())
        B, L, S = u.shape
        d = grid.shape[1]
        width = w.shape[0]
        y = _empty(B, S, width, like=u)
        call("blindno_bagmean_fwd_w", ptr(u), ptr(grid), ptr(w), ptr(bias), ptr(lw), ptr(y), B, L, S, d,
             width, stream_ptr())
        ctx.save_for_backward(w)
        ctx.lw = lw
        ctx.dims = (B, L, S, d, width)
        return y

    @staticmethod
    def backward(ctx, gy):
        (w,) = ctx.saved_tensors
        B, L, S, d, width = ctx.dims
        gy = _c(gy)
        gu = ggrid = None
        if ctx.needs_input_grad[0]:
            s = _empty(B, S, like=gy)
            lw = ctx.lw
            call("blindno_bagmean_bwd", ptr(gy), ptr(w), ptr(s), B, S, d, width,
                 1 if lw is not None else L, stream_ptr())
            gu = s.unsqueeze(1).expand(B, L, S) if lw is None else s.unsqueeze(1) * lw.view(1, L, 1)
        if ctx.needs_input_grad[1]:
            ggrid = torch.einsum("bsc,ce->se", gy, w[:, :d])
        ctx.lw = None
        return gu, ggrid, None, None, None


class DeepONetBagFn(torch.autograd.Function):
    """DeepOnetNoBiasOrg (2d_FPE/DeepONetModules.py:142-151) fused with the bag mean that reads
    its output (2d_FPE/NIOModules.py:66-77): w (B, L, P) branch coefficients, basis (S, P) trunk
    output, b0 scalar -> ubar (B, S) = mean_l (w_l . basis^T + b0) / sqrt(P), without the
    (B, L, S) field (csrc/deeponet.hip).  ``lw`` (optional, (L,)): per-snapshot weights."""

    @staticmethod
    def forward(ctx, w, basis, b0, lw=None):
        require_device(w, basis, b0)
        w, basis, b0 = _c(w), _c(basis), _c(b0.reshape(1))
        B, L, P = w.shape
        S = basis.shape[0]
        if basis.shape[1] != P:
            raise BlindnoError(f"deeponet: branch {tuple(w.shape)} / trunk {tuple(basis.shape)} mismatch")
        if P > 64:
            raise BlindnoError(f"deeponet: at most 64 basis functions (n_basis = 25 in every reference "
                               f"script), got {P}")
        scale = 1.0 / math.sqrt(P)
        wbar = _empty(B, P, like=w)
        ubar = _empty(B, S, like=w)
        call("blindno_deeponet_bag_fwd", ptr(w), ptr(basis), ptr(b0), ptr(lw), ptr(wbar), ptr(ubar),
             B, L, S, P, scale, stream_ptr())
        ctx.save_for_backward(basis, wbar)
        ctx.lw = lw
        ctx.dims = (B, L, S, P, scale)
        return ubar

    @staticmethod
    def backward(ctx, g):
        basis, wbar = ctx.saved_tensors
        B, L, S, P, scale = ctx.dims
        g = _c(g)
        nblk = query("blindno_deeponet_bag_nblk", S)
        dw = _empty(B, L, P, like=g)
        dbasis = _empty(S, P, like=g)
        db0 = _empty(1, like=g)
        partial = _empty(nblk * (B * P + 1), like=g)
        call("blindno_deeponet_bag_bwd", ptr(g), ptr(basis), ptr(wbar), ptr(ctx.lw), ptr(dw), ptr(dbasis),
             ptr(db0), ptr(partial), nblk, B, L, S, P, scale, stream_ptr())
        ctx.lw = None
        return dw, dbasis, db0.reshape(()), None


class BagAttnFn(torch.autograd.Function):
    """Token self-attention + fixed-weight fusion of NIOFP2D_FNO_attn
    (2d_FPE/NIOModules.py:365-399): u (B, L, S) encoded snapshots, grid (S, 2) -> (B, S, width).
    Tokens are [gx, gy, u_1..u_L]; ``w``/``bias`` are ``fc0.weight.data``/``.bias.data``
    (fc0 = Linear(1, width), never trained).  csrc/attn.hip: Gram matrix, softmax + column
    sums, and the column-sum-weighted bag mean (the reference's Z = A X collapses to it)."""

    @staticmethod
    def forward(ctx, u, grid, w, bias):
        require_device(u, grid, w, bias)
        u, grid = _c(u), _c(grid)
        w, bias = _c(w.detach()).view(-1), _c(bias.detach())
        B, L, S = u.shape
        T = L + 2
        if T > 256:
            raise BlindnoError(f"bag attention supports at most 256 tokens (L + 2), got {T}")
        if tuple(grid.shape) != (S, 2) or w.numel() != bias.numel():
            raise BlindnoError(f"bag attention: grid {tuple(grid.shape)} / fc0 {tuple(w.shape)} "
                               f"do not match S={S}")
        width = w.numel()
        nch = query("blindno_bagattn_nchunk", S)
        partial = _empty(B, nch, T, T, like=u)
        A = _empty(B, T, T, like=u)
        cs = _empty(B, T, like=u)
        y = _empty(B, S, width, like=u)
        call("blindno_bagattn_fwd", ptr(grid), ptr(u), ptr(w), ptr(bias), ptr(partial), ptr(A),
             ptr(cs), ptr(y), B, L, S, width, stream_ptr())
        ctx.save_for_backward(u, grid, w, A, cs)
        return y

    @staticmethod
    def backward(ctx, gy):
        u, grid, w, A, cs = ctx.saved_tensors
        B, L, S = u.shape
        T = L + 2
        gy = _c(gy)
        nch = query("blindno_bagattn_nchunk", S)
        partial = _empty(B, nch, T, like=gy)
        dm = _empty(B, S, like=gy)
        M = _empty(B, T, T, like=gy)
        du = _empty(B, L, S, like=gy)
        dgt = _empty(B, 2, S, like=gy) if ctx.needs_input_grad[1] else None
        call("blindno_bagattn_bwd", ptr(grid), ptr(u), ptr(gy), ptr(w), ptr(A), ptr(cs),
             ptr(partial), ptr(dm), ptr(M), ptr(du), ptr(dgt), B, L, S, w.numel(), stream_ptr())
        ggrid = dgt.sum(0).t() if dgt is not None else None
        return (du if ctx.needs_input_grad[0] else None), ggrid, None, None


# ---------------------------------------------------------------------------- loss


def _mse_blocks(n):
    # ~1024 elements per workgroup (4 per thread): a config-C output (4 x 128^2 x 2) gets 128
    # workgroups instead of 32
    return max(1, min(1024, (n + 1023) // 1024))


_MSE_COUNTER = None     # the caller-owned completion counter (loss_counter), or None
_UNIT_SEED = None       # the constant 1.0 a caller seeds backward() with (unit_seed)


@contextlib.contextmanager
def unit_seed(one: torch.Tensor):
    """Within this context the loss functions may precompute their gradient for an upstream
    gradient of exactly 1, used when backward() is seeded with this very tensor ``one`` (a
    constant 1.0 that the caller never changes; GraphedBagStep's seed)."""
    global _UNIT_SEED
    prev, _UNIT_SEED = _UNIT_SEED, one
    try:
        yield
    finally:
        _UNIT_SEED = prev


@contextlib.contextmanager
def loss_counter(counter: torch.Tensor):
    """Within this context the fused MSE forward uses ``counter`` (one int32, zero; the
    launch's last workgroup resets it) as its completion counter instead of a fresh zeroed one.
    For a caller that owns one counter per captured graph (GraphedBagStep: the last slot of a
    key's index blob, zeroed before capture), so a replay needs no memset node.  The counter
    must not be shared by launches that may run concurrently (two streams)."""
    global _MSE_COUNTER
    if counter.dtype != torch.int32 or counter.numel() != 1 or not counter.is_cuda:
        raise BlindnoError("loss_counter: one int32 device element")
    prev, _MSE_COUNTER = _MSE_COUNTER, counter
    try:
        yield
    finally:
        _MSE_COUNTER = prev


def _mse_counter(dev):
    """The fused MSE forward's completion counter: the caller's (loss_counter), or a fresh
    zeroed one per launch -- never one shared across launches that could overlap on different
    streams (their workgroups would count into each other's finish)."""
    if _MSE_COUNTER is not None:
        return _MSE_COUNTER
    return torch.zeros(1, dtype=torch.int32, device=dev)


class MSEFn(torch.autograd.Function):
    """nn.MSELoss() (mean reduction) with a fused gradient kernel."""

    @staticmethod
    def forward(ctx, pred, target, acc=None):
        require_device(pred, target)
        pred, target = _c(pred), _c(target)
        n = pred.numel()
        nblk = _mse_blocks(n)
        partial = _empty(nblk, like=pred)
        loss = _empty((), like=pred)
        # under unit_seed(): the gradient for an upstream gradient of exactly 1 is formed in the
        # same pass, and a backward seeded with that tensor takes it without a launch
        pre = torch.empty_like(pred) if _UNIT_SEED is not None else None
        # acc (float32 scalar, optional): the loss is also added to it in the same launch; the
        # partials and their sum in one launch (the last workgroup to finish sums them)
        call("blindno_mse_fwd", ptr(pred), ptr(target), ptr(partial), n, nblk, ptr(loss), ptr(acc),
             ptr(_mse_counter(pred.device)), ptr(pre), stream_ptr())
        ctx.save_for_backward(pred, target)
        ctx.pre, ctx.seed = pre, _UNIT_SEED
        return loss

    @staticmethod
    def backward(ctx, g):
        pre, seed = ctx.pre, ctx.seed
        ctx.pre = ctx.seed = None
        if pre is not None and g.data_ptr() == seed.data_ptr():
            return pre, None, None
        pred, target = ctx.saved_tensors
        n = pred.numel()
        nblk = _mse_blocks(n)
        partial = _empty(nblk, like=pred)
        grad = torch.empty_like(pred)
        g = _c(g.reshape(1))
        call("blindno_mse", ptr(pred), ptr(target), ptr(partial), ptr(grad), n, nblk, ptr(g),
             stream_ptr())
        return grad, None, None


def mse_loss(pred, target, acc=None):
    """nn.MSELoss()(pred, target); ``acc`` (float32 scalar tensor): add the loss value to it."""
    if acc is not None and (acc.dtype != F32 or acc.numel() != 1 or acc.device != pred.device):
        raise BlindnoError("mse_loss: acc must be a float32 scalar on the prediction's device")
    return MSEFn.apply(pred, target, acc)


# ---------------------------------------------------------------------------- metrics


def rowsq(a, b, rows, n, stride, off_a, off_b, den_all):
    out = torch.empty(rows, 2, dtype=torch.float64, device=a.device)
    call("blindno_rowsq", ptr(_c(a)), ptr(_c(b)), ptr(out), rows, n, stride, off_a, off_b,
         den_all, stream_ptr())
    return out


def train_rel_l2_2ch(pred, out):
    """Per-sample train-loop metric of 2d_FPE/train_fno.py:160-163 (denominator = norm of
    BOTH output channels).  pred/out (B, ..., 2).  Returns (e_ch0, e_ch1) fp64 (B,)."""
    B = pred.shape[0]
    n = pred[0].numel() // pred.shape[-1]
    s0 = rowsq(pred, out, B, n, pred.shape[-1], 0, 0, 1)
    s1 = rowsq(pred, out, B, n, pred.shape[-1], 1, 1, 1)
    return s0[:, 0].sqrt() / s0[:, 1].sqrt(), s1[:, 0].sqrt() / s1[:, 1].sqrt()


def time_averaged_relative_l2(pt_pred, pt_ref, eps=1e-12):
    """mean_t ||P_pred[t]-P_ref[t]|| / (||P_ref[t]|| + eps)
    (2d_Non_conservative_FPE/compute_time_error.py:321-333), fp64 accumulation on device."""
    nt = pt_pred.shape[0]
    n = pt_pred[0].numel()
    s = rowsq(pt_pred.float(), pt_ref.float(), nt, n, 1, 0, 0, 0)
    return float((s[:, 0].sqrt() / (s[:, 1].sqrt() + eps)).mean())


# ---------------------------------------------------------------------------- NIO encoder blocks

def k_conv2d_bwd_data(dy, weight, g):
    """Input gradient of a conv2d with geometry g = (N, Ci, Hi, Wi, Co, KH, KW, sh, sw, ph, pw):
    K split (partial slabs reduced in order) where the input pixels are too few to fill the chip."""
    dx = torch.empty(g[0], g[1], g[2], g[3], dtype=F32, device=dy.device)
    ns = query("blindno_conv2d_bwd_data_nsplit", *g)
    part = _empty(ns, dx.numel(), like=dy) if ns > 1 else None
    call("blindno_conv2d_bwd_data_split", ptr(dy), ptr(weight), ptr(dx), ptr(part), ns,
         ptr(_wscratch(1, g, dy)), *g, stream_ptr())
    return dx


def _wscratch(mode, g, like):
    """Scratch for the tap-major weight re-layout of a conv2d launch (None where unused)."""
    n = query("blindno_conv2d_wscratch_floats", mode, *g)
    return _empty(n, like=like) if n > 0 else None


class Conv2dFn(torch.autograd.Function):
    """nn.Conv2d (bias, groups 1, zero padding) of the NIO encoders' ConvBlocks
    (2d_FPE/Baselines.py:40-52) on the HIP implicit-GEMM kernels (csrc/conv.hip): x (N, Ci, H, W),
    weight (Co, Ci, KH, KW), bias (Co) -> (N, Co, Ho, Wo).  Deterministic; any batch size N, so
    the bag needs no fixed-size chunking and the step can be captured in a HIP graph."""

    @staticmethod
    def forward(ctx, x, weight, bias, stride, padding):
        require_device(x, weight)
        x, weight = _c(x), _c(weight)
        bias = _c(bias) if bias is not None else None
        N, Ci, Hi, Wi = x.shape
        Co, _, KH, KW = weight.shape
        sh, sw = stride
        ph, pw = padding
        Ho, Wo = (Hi + 2 * ph - KH) // sh + 1, (Wi + 2 * pw - KW) // sw + 1
        y = _empty(N, Co, Ho, Wo, like=x)
        g = (N, Ci, Hi, Wi, Co, KH, KW, sh, sw, ph, pw)
        ns = query("blindno_conv2d_fwd_nsplit", *g)      # split K for the few-pixel last blocks
        part = _empty(ns, y.numel(), like=x) if ns > 1 else None
        call("blindno_conv2d_fwd_split", ptr(x), ptr(weight), ptr(bias), ptr(y), ptr(part), ns,
             ptr(_wscratch(0, g, x)), *g, stream_ptr())
        ctx.geom = g
        ctx.has_bias = bias is not None
        ctx.save_for_backward(x, weight)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        N, Ci, Hi, Wi, Co, KH, KW, sh, sw, ph, pw = ctx.geom
        g = ctx.geom
        dy = _c(dy)
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = k_conv2d_bwd_data(dy, weight, g)
        if ctx.needs_input_grad[1] or (ctx.has_bias and ctx.needs_input_grad[2]):
            ncol = Ci * KH * KW + 1
            ns = query("blindno_conv2d_wgrad_nsplit", *g)
            dwb = _empty(Co, ncol, like=dy)
            part = _empty(ns, Co * ncol, like=dy) if ns > 1 else None
            call("blindno_conv2d_bwd_weight", ptr(dy), ptr(x), ptr(dwb), ptr(part), ns, *g, stream_ptr())
            dw = dwb[:, :-1].reshape(Co, Ci, KH, KW) if ctx.needs_input_grad[1] else None
            db = dwb[:, -1].contiguous() if ctx.has_bias and ctx.needs_input_grad[2] else None
        return dx, dw, db, None, None


def conv2d(x, weight, bias, stride, padding):
    return Conv2dFn.apply(x, weight, bias, tuple(stride), tuple(padding))


def linear(x, weight, bias):
    """nn.Linear on libblindno: x (..., K) @ weight (N, K)^T + bias as a 1x1 convolution of
    (rows, K, 1, 1) images (csrc/conv.hip implicit GEMMs: fp32 matrix cores, the bias a GEMM
    column of the weight gradient, fixed-order split-K) -- no rocBLAS / hipBLASLt and no torch
    reduction in a captured step.  Used by the NIO branch's final Linear and the FFN trunk
    (2d_FPE/Baselines.py:202,249; 2d_FPE/DeepONetModules.py:155-185)."""
    shp = x.shape
    K, N = shp[-1], weight.shape[0]
    y = conv2d(x.reshape(-1, K, 1, 1), weight.view(N, K, 1, 1), bias, (1, 1), (0, 0))
    return y.view(*shp[:-1], N)


class BNActFn(torch.autograd.Function):
    """BatchNorm2d + LeakyReLU of a ConvBlock (2d_FPE/Baselines.py:40-52) on rows [0, n) of z
    (rows [n, Npad) are the convolution chunks' padding and come out 0).  Running statistics
    are updated like torch.nn.BatchNorm2d (momentum, or the cumulative average when momentum
    is None)."""

    @staticmethod
    def forward(ctx, z, gamma, beta, bn, n, slope):
        require_device(z)
        z = _c(z)
        Npad, C = z.shape[0], z.shape[1]
        HW = z[0, 0].numel()
        use_batch = bn.training or bn.running_mean is None
        track = bn.training and bn.track_running_stats and bn.running_mean is not None
        mom = 0.0
        if track:
            bn.num_batches_tracked.add_(1)
            mom = bn.momentum if bn.momentum is not None else 1.0 / float(bn.num_batches_tracked)
        S = query("blindno_bn_act_nslices", n, C, HW)
        partial = torch.empty(C * S * 4, device=z.device, dtype=F32)   # C S 2 fp64 sums
        save = torch.empty(C, 4, device=z.device, dtype=F32)
        y = torch.empty_like(z)
        rm = bn.running_mean if (track or not use_batch) else None
        rv = bn.running_var if (track or not use_batch) else None
        call("blindno_bn_act_fwd", ptr(z), ptr(gamma), ptr(beta), ptr(rm), ptr(rv), ptr(y), ptr(save),
             ptr(partial), n, Npad, C, HW, float(bn.eps), float(mom), float(slope), int(use_batch),
             stream_ptr())
        ctx.save_for_backward(z, gamma, save)
        ctx.meta = (n, Npad, C, HW, float(slope), int(use_batch), S)
        return y

    @staticmethod
    def backward(ctx, dy):
        z, gamma, save = ctx.saved_tensors
        n, Npad, C, HW, slope, use_batch, S = ctx.meta
        dy = _c(dy)
        dz = torch.empty_like(z)
        dgamma = torch.empty(C, device=z.device, dtype=F32) if gamma is not None and ctx.needs_input_grad[1] else None
        dbeta = torch.empty(C, device=z.device, dtype=F32) if ctx.needs_input_grad[2] else None
        partial = torch.empty(C * S * 4, device=z.device, dtype=F32)   # C S 2 fp64 sums
        coef = torch.empty(C, 3, device=z.device, dtype=F32)
        call("blindno_bn_act_bwd", ptr(dy), ptr(z), ptr(gamma), ptr(save), ptr(dz), ptr(dgamma), ptr(dbeta),
             ptr(partial), ptr(coef), n, Npad, C, HW, slope, use_batch, stream_ptr())
        return dz, dgamma, dbeta, None, None, None
