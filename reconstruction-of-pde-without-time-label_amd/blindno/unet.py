"""The permutation-invariant attention UNet, PermInvUNet_attn -- the model the reference's plots
call "BlinDNO"  -- on the HIP kernels.

Drop-in for (same class names, constructor signatures, attribute names, parameter shapes and
creation order, so reference checkpoints load and a seeded construction gives identical
weights):
  * ``PermInvUNet_attn``      2d_FPE/NIOModules.py:1086-1181 (ConvNeXt down/up blocks)
  * ``PermInvUNet_attn_NC``   the 2d_Non_conservative_FPE copy of PermInvUNet_attn
                              (2d_Non_conservative_FPE/NIOModules.py:932-1053: Conv2d +
                              BatchNorm2d + ReLU blocks, heads fno_Fx / fno_Fy; the dropin shim of
                              that experiment exports it under the reference's name)
  * ``PermInvUNet_attn1D``    1d_FPE/NIOModules.py:212-322 (all T snapshots)
  * ``PermInvUNet_attn1D_bag`` 1d_FPE/NIOModules.py:326-443 (train-mode bag draw); the 1d_GPE
                              copies (one head fno_V): ``PermInvUNet_attn1D_bag_V`` and
                              ``PermInvUNet_attn1D_bag_GPE`` (1d_GPE/NIOModules.py:342-560)

Per-snapshot layers (3x3 conv, 7x7 depthwise conv, the ConvNeXt pointwise MLP with its
LayerNorm, 2x2 max pool) run on the B*L snapshots of a bag; the temporal self-attention + bag
mean of every level is one collapsed HIP op (csrc/unet.hip: centred Gram matrix per bag, no
(B, L, D) intermediate); the decoder (transposed conv, skip BatchNorm, conv, ConvNeXt) runs on
B samples and the two FNO heads on the fused 12-channel field (ops.HeadPairFn, grouped).
1D models are height-1 fields through the same kernels.  There is no CPU path.
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch
import torch.nn as nn

from . import ops
from ._lib import call, ptr, query, stream_ptr
from .fno import FNO1d, FNO2d
from .nio import _run_heads, draw_bag

F32 = torch.float32


def _c(t):
    return t if t.is_contiguous() else t.contiguous()


def _e(*shape, like):
    return torch.empty(*shape, device=like.device, dtype=F32)


def _as4(x):
    """(N, C, L) 1D fields as (N, C, 1, L)."""
    return x if x.dim() == 4 else x.unsqueeze(2)


# ---------------------------------------------------------------------------- kernel launchers
# (shared by the autograd Functions below and the torch.ops.blindno.* operators of torch_ops.py)

def dwconv_fwd(x, w, b):
    """Depthwise KHxKW convolution, padding (KH/2, KW/2), with bias: ConvNeXtBlock.dwconv
    (2d_FPE/NIOModules.py:1047; 1d_FPE/NIOModules.py:169).  x (N, C, H, W); w (C, 1, KH, KW)."""
    ops.require_device(x, w)
    x, w, b = _c(x), _c(w), _c(b)
    N, C, H, W = x.shape
    y = torch.empty_like(x)
    call("blindno_dwconv_fwd", ptr(x), ptr(w), ptr(b), ptr(y), N, C, H, W, w.shape[-2], w.shape[-1], stream_ptr())
    return y


def dwconv_bwd(dy, x, w, need_dx=True, need_w=True):
    N, C, H, W = x.shape
    KH, KW = w.shape[-2], w.shape[-1]
    dy = _c(dy)
    dx = dw = db = None
    if need_dx:
        dx = torch.empty_like(x)
        call("blindno_dwconv_bwd_data", ptr(dy), ptr(w), ptr(dx), N, C, H, W, KH, KW, stream_ptr())
    if need_w:
        ns = query("blindno_dwconv_wgrad_nsplit", N, C, H, W)
        dwb = _e(C, KH * KW + 1, like=dy)
        part = _e(ns * C * (KH * KW + 1), like=dy) if ns > 1 else None
        call("blindno_dwconv_bwd_weight", ptr(dy), ptr(x), ptr(dwb), ptr(part), ns, N, C, H, W, KH, KW,
             stream_ptr())
        dw = dwb[:, :-1].reshape(w.shape)
        db = dwb[:, -1].contiguous()
    return dx, dw, db


def cnx_pw_fwd(xd, sc, lw, lb, w1, b1, w2, b2):
    """ConvNeXtBlock after the depthwise conv (2d_FPE/NIOModules.py:1053-1062): per pixel
    LayerNorm(C, eps 1e-6) -> pwconv1 -> exact GELU -> pwconv2 -> + shortcut.  xd, sc (N, C, *S)."""
    ops.require_device(xd, sc)
    xd, sc = _c(xd), _c(sc)
    lw, lb, w1, b1, w2, b2 = (_c(t) for t in (lw, lb, w1, b1, w2, b2))
    N, C = xd.shape[0], xd.shape[1]
    HW = xd[0, 0].numel()
    y = torch.empty_like(xd)
    call("blindno_cnx_pw_fwd", ptr(xd), ptr(sc), ptr(lw), ptr(lb), ptr(w1), ptr(b1), ptr(w2), ptr(b2), ptr(y),
         N, C, HW, stream_ptr())
    return y


def cnx_pw_bwd(dy, xd, lw, lb, w1, b1, w2):
    """-> (dxd, dlw, dlb, dw1, db1, dw2, db2); the shortcut's gradient is dy itself."""
    N, C = xd.shape[0], xd.shape[1]
    HW = xd[0, 0].numel()
    dy = _c(dy)
    nblk = query("blindno_cnx_pw_bwd_nblk", N, C, HW)
    E = 8 * C * C + 7 * C
    dxd = torch.empty_like(xd)
    dp = _e(E, like=dy)
    part = _e(nblk * E, like=dy)
    call("blindno_cnx_pw_bwd", ptr(dy), ptr(_c(xd)), ptr(_c(lw)), ptr(_c(lb)), ptr(_c(w1)), ptr(_c(b1)),
         ptr(_c(w2)), ptr(dxd), ptr(dp), ptr(part), nblk, N, C, HW, stream_ptr())
    H4 = 4 * C
    o = 0
    dw1 = dp[o:o + H4 * C].view(H4, C); o += H4 * C
    db1 = dp[o:o + H4]; o += H4
    dw2 = dp[o:o + C * H4].view(C, H4); o += C * H4
    db2 = dp[o:o + C]; o += C
    dlw = dp[o:o + C]; o += C
    dlb = dp[o:o + C]
    return dxd, dlw, dlb, dw1, db1, dw2, db2


def maxpool_fwd(x, KH, KW):
    """MaxPool2d(2) / MaxPool1d(2) (2d_FPE/NIOModules.py:1115; 1d_FPE/NIOModules.py:239) on
    (N, C, H, W) with window (KH, KW) -> (y, arg uint8)."""
    ops.require_device(x)
    x = _c(x)
    N, C, H, W = x.shape
    Ho, Wo = H // KH, W // KW
    y = _e(N, C, Ho, Wo, like=x)
    arg = torch.empty(N, C, Ho, Wo, device=x.device, dtype=torch.uint8)
    call("blindno_maxpool_fwd", ptr(x), ptr(y), ptr(arg), N * C, H, W, KH, KW, stream_ptr())
    return y, arg


def maxpool_bwd(dy, arg, H, W, KH, KW):
    N, C = dy.shape[0], dy.shape[1]
    dy = _c(dy)
    dx = _e(N, C, H, W, like=dy)
    call("blindno_maxpool_bwd", ptr(dy), ptr(_c(arg)), ptr(dx), N * C, H, W, KH, KW, stream_ptr())
    return dx


def convt_fwd(x, w, b, Ho, Wo):
    """ConvTranspose2d(Ci, Co, kernel = stride = 2, output_padding) (2d_FPE/NIOModules.py:
    1130-1134; 1D: kernel (1, 2)).  x (N, Ci, Hi, Wi), w (Ci, Co, KH, KW) -> (N, Co, Ho, Wo)."""
    ops.require_device(x, w)
    x, w, b = _c(x), _c(w), _c(b)
    N, Ci, Hi, Wi = x.shape
    Co, KH, KW = w.shape[1], w.shape[2], w.shape[3]
    y = _e(N, Co, Ho, Wo, like=x)
    call("blindno_convt_fwd", ptr(x), ptr(w), ptr(b), ptr(y), N, Ci, Hi, Wi, Co, KH, KW, Ho, Wo, stream_ptr())
    return y


def convt_bwd(dy, x, w, need_dx=True, need_w=True):
    N, Ci, Hi, Wi = x.shape
    Co, KH, KW = w.shape[1], w.shape[2], w.shape[3]
    Ho, Wo = dy.shape[2], dy.shape[3]
    g = (N, Ci, Hi, Wi, Co, KH, KW, Ho, Wo)
    dy = _c(dy)
    dx = dw = db = None
    if need_dx:
        dx = torch.empty_like(x)
        call("blindno_convt_bwd_data", ptr(dy), ptr(_c(w)), ptr(dx), *g, stream_ptr())
    if need_w:
        E = Ci * Co * KH * KW + Co
        dwb = _e(E, like=dy)
        part = _e(query("blindno_convt_wgrad_nparts", N, Hi, Wi) * E, like=dy)
        call("blindno_convt_bwd_weight", ptr(dy), ptr(_c(x)), ptr(dwb), ptr(part), *g, stream_ptr())
        dw = dwb[:E - Co].view(w.shape)
        db = dwb[E - Co:]
    return dx, dw, db


def tok_attn_fwd(X, lw, lb, eps):
    """TemporalSelfAttention followed by the bag mean (2d_FPE/NIOModules.py:1065-1083 with
    :1163-1164 / :1171-1172): X (B, L, D) -> (mean_l LayerNorm_D(softmax(X X^T/sqrt D) X + X)_l
    (B, D), the saved state of the backward)."""
    ops.require_device(X, lw)
    X, lw, lb = _c(X), _c(lw), _c(lb)
    B, L, D = X.shape
    save = _e(query("blindno_tok_attn_save_floats", B, L, D), like=X)
    nch = query("blindno_tok_gram_nchunk", D)
    gram = _e(B * L * L, like=X)
    gp = _e(nch * B * L * L, like=X) if nch > 1 else None
    Y = _e(B, D, like=X)
    call("blindno_tok_attn_fwd", ptr(X), ptr(lw), ptr(lb), ptr(Y), ptr(save), ptr(gp), ptr(gram), B, L, D,
         float(eps), stream_ptr())
    return Y, save


def tok_attn_bwd(dY, X, lw, save, need_dx=True, need_lw=True, need_lb=True):
    B, L, D = X.shape
    dY = _c(dY)
    dX = torch.empty_like(X) if need_dx else None
    dlw = _e(D, like=dY) if need_lw else None
    dlb = _e(D, like=dY) if need_lb else None
    scratch = _e(query("blindno_tok_attn_bwd_scratch_floats", B, L), like=dY)
    call("blindno_tok_attn_bwd", ptr(dY), ptr(_c(X)), ptr(_c(lw)), ptr(save), ptr(dX), ptr(dlw), ptr(dlb),
         ptr(scratch), B, L, D, stream_ptr())
    return dX, dlw, dlb


# ---------------------------------------------------------------------------- autograd ops

class DWConvFn(torch.autograd.Function):
    """``dwconv_fwd`` with its adjoint."""

    @staticmethod
    def forward(ctx, x, w, b):
        y = dwconv_fwd(x, w, b)
        ctx.save_for_backward(_c(x), _c(w))
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        return dwconv_bwd(dy, x, w, ctx.needs_input_grad[0],
                          ctx.needs_input_grad[1] or ctx.needs_input_grad[2])


class CnxPwFn(torch.autograd.Function):
    """``cnx_pw_fwd`` with its adjoint (one kernel each way)."""

    @staticmethod
    def forward(ctx, xd, sc, lw, lb, w1, b1, w2, b2):
        y = cnx_pw_fwd(xd, sc, lw, lb, w1, b1, w2, b2)
        ctx.save_for_backward(*(_c(t) for t in (xd, lw, lb, w1, b1, w2)))
        return y

    @staticmethod
    def backward(ctx, dy):
        xd, lw, lb, w1, b1, w2 = ctx.saved_tensors
        dxd, dlw, dlb, dw1, db1, dw2, db2 = cnx_pw_bwd(dy, xd, lw, lb, w1, b1, w2)
        return dxd, dy, dlw, dlb, dw1, db1, dw2, db2


class MaxPoolFn(torch.autograd.Function):
    """``maxpool_fwd`` with its adjoint."""

    @staticmethod
    def forward(ctx, x, KH, KW):
        y, arg = maxpool_fwd(x, KH, KW)
        ctx.save_for_backward(arg)
        ctx.geom = (x.shape[2], x.shape[3], KH, KW)
        return y

    @staticmethod
    def backward(ctx, dy):
        (arg,) = ctx.saved_tensors
        return maxpool_bwd(dy, arg, *ctx.geom), None, None


class ConvTFn(torch.autograd.Function):
    """``convt_fwd`` with its adjoint."""

    @staticmethod
    def forward(ctx, x, w, b, Ho, Wo):
        y = convt_fwd(x, w, b, Ho, Wo)
        ctx.save_for_backward(_c(x), _c(w))
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dx, dw, db = convt_bwd(dy, x, w, ctx.needs_input_grad[0],
                               ctx.needs_input_grad[1] or ctx.needs_input_grad[2])
        return dx, dw, db, None, None


class TokAttnMeanFn(torch.autograd.Function):
    """``tok_attn_fwd`` with its adjoint: one collapsed HIP op each way (csrc/unet.hip)."""

    @staticmethod
    def forward(ctx, X, lw, lb, eps):
        Y, save = tok_attn_fwd(X, lw, lb, eps)
        ctx.save_for_backward(_c(X), _c(lw), save)
        return Y

    @staticmethod
    def backward(ctx, dY):
        X, lw, save = ctx.saved_tensors
        n = ctx.needs_input_grad
        dX, dlw, dlb = tok_attn_bwd(dY, X, lw, save, n[0], n[1], n[2])
        return dX, dlw, dlb, None


# ---------------------------------------------------------------------------- building blocks

def _conv3(conv: nn.Module, x):
    """nn.Conv2d / nn.Conv1d(kernel 3, padding 1) (or final_conv's kernel 1) on the HIP
    implicit-GEMM convolution; 1D fields as height-1 2D ones."""
    w = conv.weight
    if w.dim() == 3:
        w = w.unsqueeze(2)
    k = w.shape[-1]
    ph = (w.shape[-2] - 1) // 2
    pw = (k - 1) // 2
    y = ops.conv2d(_as4(x), w, conv.bias, (1, 1), (ph, pw))
    return y if x.dim() == 4 else y.squeeze(2)


def _bn(bn: nn.Module, x, slope):
    """BatchNorm{1,2}d (+ LeakyReLU(slope): 1.0 = none, 0.0 = ReLU) on the HIP kernel; batch
    statistics in train mode, running statistics in eval mode."""
    return ops.BNActFn.apply(_c(x), bn.weight, bn.bias, bn, x.shape[0], float(slope))


class ConvNeXtBlock(nn.Module):
    """ConvNeXtBlock, 2d_FPE/NIOModules.py:1044-1062."""

    def __init__(self, dim):
        super().__init__()
        self.dwconv = nn.Conv2d(dim, dim, kernel_size=7, padding=3, groups=dim)
        self.norm = nn.LayerNorm(dim, eps=1e-6)
        self.pwconv1 = nn.Linear(dim, 4 * dim)
        self.act = nn.GELU()
        self.pwconv2 = nn.Linear(4 * dim, dim)

    def forward(self, x):
        x4 = _as4(x)
        w = self.dwconv.weight
        xd = DWConvFn.apply(x4, w if w.dim() == 4 else w.unsqueeze(2), self.dwconv.bias)
        y = CnxPwFn.apply(xd, x4, self.norm.weight, self.norm.bias, self.pwconv1.weight,
                          self.pwconv1.bias, self.pwconv2.weight, self.pwconv2.bias)
        return y if x.dim() == 4 else y.squeeze(2)


class ConvNeXtBlock1D(ConvNeXtBlock):
    """ConvNeXtBlock1D, 1d_FPE/NIOModules.py:165-184."""

    def __init__(self, dim):
        nn.Module.__init__(self)
        self.dwconv = nn.Conv1d(dim, dim, kernel_size=7, padding=3, groups=dim)
        self.norm = nn.LayerNorm(dim, eps=1e-6)
        self.pwconv1 = nn.Linear(dim, 4 * dim)
        self.act = nn.GELU()
        self.pwconv2 = nn.Linear(4 * dim, dim)


class TemporalSelfAttention(nn.Module):
    """TemporalSelfAttention, 2d_FPE/NIOModules.py:1065-1083 (D = C H W, LayerNorm(D)).
    ``forward`` is the reference's (B, L, C, H, W) -> same; the UNet itself only ever uses the
    bag mean of it, ``bag_mean`` (the collapsed HIP op)."""

    def __init__(self, C, H, W):
        super().__init__()
        self.C, self.H, self.W = C, H, W
        self.D = C * H * W
        self.norm = nn.LayerNorm(self.D)

    def bag_mean(self, x):
        """x (B, L, *feat) -> mean over the bag of forward(x): (B, *feat)."""
        B, L = x.shape[:2]
        y = TokAttnMeanFn.apply(x.reshape(B, L, -1), self.norm.weight, self.norm.bias, self.norm.eps)
        return y.view(B, *x.shape[2:])


class TemporalSelfAttention1D(TemporalSelfAttention):
    """TemporalSelfAttention1D, 1d_FPE/NIOModules.py:186-209 (D = C L)."""

    def __init__(self, C, L):
        nn.Module.__init__(self)
        self.C, self.L = C, L
        self.D = C * L
        self.norm = nn.LayerNorm(self.D)


def _sizes_and_pads(n, depth):
    """Skip sizes and ConvTranspose output_padding (2d_FPE/NIOModules.py:1094-1107)."""
    s = [n]
    for _ in range(depth):
        s.append(s[-1] // 2)
    pads, cur = [], s[-1]
    for sz in reversed(s[:-1]):
        pads.append(sz - ((cur - 1) * 2 + 2))
        cur = sz
    return s, pads


class _UNetBase(nn.Module):
    """Shared forward of the four UNet variants (construction is per class, in the reference's
    order).  Subclasses set: dim (1 or 2), _block ("convnext" or "convbn"), _heads, _bag
    (train-mode bag draw)."""

    dim = 2
    _block = "convnext"
    _heads = ("fno_drift", "fno_diffusion")
    _bag = True
    _taps = None        # diagnostics: a list collects (name, tensor) of the per-level activations

    @property
    def unused_prefixes(self):
        """Registered parameters the forward never uses (no gradient; the reference trains with
        find_unused_parameters=True): the bottom level's skip BatchNorm and, in the NC copy,
        the fno_drift / fno_diffusion heads."""
        p = [f"skip_norms.{self.depth}."]
        if tuple(self._heads) != ("fno_drift", "fno_diffusion"):
            p += ["fno_drift.", "fno_diffusion."]
        return tuple(p)

    def _tap(self, name, t):
        if self._taps is not None:
            t.retain_grad()
            self._taps.append((name, t))
        return t

    def _block_fwd(self, seq, h):
        if self._block == "convbn":
            return _bn(seq[1], _conv3(seq[0], h), 0.0)     # Conv -> BatchNorm -> ReLU
        return seq[1](_conv3(seq[0], h))                     # Conv -> ConvNeXtBlock

    def _bag_of(self, x, bag_idx):
        if torch.is_tensor(bag_idx) and bag_idx.is_cuda:
            return x.index_select(1, bag_idx)                # device-resident indices (graphs)
        if bag_idx is not None:
            idx = np.asarray(bag_idx)
        elif self.training and self._bag:
            _, idx = draw_bag(x.shape[1])
        else:
            return x
        return x.index_select(1, torch.as_tensor(idx, device=x.device))

    def forward(self, x, grid=None, bag_idx=None):
        """x (B, T, H, W) [2D] / (B, T, L) [1D] -> (B, H, W, 2) / (B, L, 2).  ``grid`` is
        accepted and ignored (the reference's UNet takes none; the training harness passes
        one); ``bag_idx`` overrides the train-mode draw (parity harness, graph replays)."""
        x = self._bag_of(x, bag_idx)
        B, L = x.shape[:2]
        spatial = x.shape[2:]
        h = x.reshape(B * L, 1, *spatial)
        feats = []
        kpool = (2, 2) if self.dim == 2 else (1, 2)
        for i in range(self.depth + 1):
            h = self._tap(f"feat{i}", self._block_fwd(self.down_convs[i], h))
            feats.append(h)
            if i < self.depth:
                h = MaxPoolFn.apply(_as4(h), *kpool)
                if self.dim == 1:
                    h = h.squeeze(2)

        def agg(level):
            f = feats[level]
            return self._tap(f"agg{level}", self.temp_atts[level].bag_mean(f.view(B, L, *f.shape[1:])))

        h = agg(self.depth)
        for i in range(self.depth):
            lv = self.depth - 1 - i
            skip_shape = feats[lv].shape[2:]
            up = self.up_transposes[i]
            w = up.weight if up.weight.dim() == 4 else up.weight.unsqueeze(2)
            Ho, Wo = (skip_shape[0], skip_shape[1]) if self.dim == 2 else (1, skip_shape[0])
            h4 = ConvTFn.apply(_as4(h), w, up.bias, Ho, Wo)
            h = h4 if self.dim == 2 else h4.squeeze(2)
            s = _bn(self.skip_norms[lv], agg(lv), 1.0)
            h = torch.cat([h, s], dim=1)
            h = self._tap(f"up{i}", self._block_fwd(self.up_convs[i], h))
        fused = self._tap("fused", _conv3(self.final_conv, h))
        fused = fused.permute(0, 2, 3, 1) if self.dim == 2 else fused.permute(0, 2, 1)
        return _run_heads(self, fused.contiguous())


class PermInvUNet_attn(_UNetBase):
    """PermInvUNet_attn, 2d_FPE/NIOModules.py:1086-1181."""

    def __init__(self, in_ch=1, out_ch=2, base_ch=1, depth=4, input_size=(61, 61)):
        super().__init__()
        self.depth = depth
        self.width = 12
        self.chs = [base_ch * (2 ** i) for i in range(depth + 1)]
        sh, pads_h = _sizes_and_pads(input_size[0], depth)
        sw, pads_w = _sizes_and_pads(input_size[1], depth)
        self.down_convs = nn.ModuleList()
        self.pools = nn.ModuleList()
        self.down_convs.append(nn.Sequential(nn.Conv2d(in_ch, self.chs[0], kernel_size=3, padding=1),
                                             self._down_block(self.chs[0])))
        for i in range(depth):
            self.pools.append(nn.MaxPool2d(2))
            self.down_convs.append(nn.Sequential(
                nn.Conv2d(self.chs[i], self.chs[i + 1], kernel_size=3, padding=1),
                self._down_block(self.chs[i + 1])))
        self.skip_norms = nn.ModuleList([nn.BatchNorm2d(ch) for ch in self.chs])
        self.temp_atts = nn.ModuleList([TemporalSelfAttention(self.chs[i], sh[i], sw[i])
                                        for i in range(depth + 1)])
        self.up_transposes = nn.ModuleList()
        self.up_convs = nn.ModuleList()
        for (ph, pw), i in zip(zip(pads_h, pads_w), reversed(range(depth))):
            self.up_transposes.append(nn.ConvTranspose2d(self.chs[i + 1], self.chs[i], kernel_size=2,
                                                         stride=2, output_padding=(ph, pw)))
            self.up_convs.append(nn.Sequential(
                nn.Conv2d(self.chs[i] * 2, self.chs[i], kernel_size=3, padding=1),
                self._down_block(self.chs[i])))
        self.final_conv = nn.Conv2d(self.chs[0], self.width, kernel_size=1)
        self._make_heads()

    def _down_block(self, ch):
        return ConvNeXtBlock(ch)

    def _make_heads(self):
        self.fno_drift = FNO2d(modes=32, width=self.width, n_layers=3, input_dim=self.width, output_dim=1)
        self.fno_diffusion = FNO2d(modes=32, width=self.width, n_layers=3, input_dim=self.width, output_dim=1)


class PermInvUNet_attn_NC(PermInvUNet_attn):
    """PermInvUNet_attn of 2d_Non_conservative_FPE (NIOModules.py:932-1053): the down/up blocks
    are Conv2d -> BatchNorm2d -> ReLU (batch statistics over the B*L snapshots in train mode),
    four heads are registered (fno_drift, fno_diffusion unused) and the output is
    cat(fno_Fx, fno_Fy)."""

    _block = "convbn"
    _heads = ("fno_Fx", "fno_Fy")

    def __init__(self, in_ch=1, out_ch=2, base_ch=1, depth=4, input_size=(61, 61)):
        super().__init__(in_ch, out_ch, base_ch, depth, input_size)

    def _down_block(self, ch):
        # nn.Sequential(Conv2d, BatchNorm2d, ReLU): the conv is created by the caller, so this
        # returns the BN; the ReLU has no parameters (indices 0 and 1 match the reference)
        return nn.BatchNorm2d(ch)

    def _make_heads(self):
        super()._make_heads()
        self.fno_Fx = FNO2d(modes=32, width=self.width, n_layers=3, input_dim=self.width, output_dim=1)
        self.fno_Fy = FNO2d(modes=32, width=self.width, n_layers=3, input_dim=self.width, output_dim=1)


class PermInvUNet_attn1D(_UNetBase):
    """PermInvUNet_attn1D, 1d_FPE/NIOModules.py:212-322: every one of the T snapshots (no bag
    draw); heads FNO1d(modes 15, width 30, 3 layers)."""

    dim = 1
    _bag = False

    _width = 30

    def __init__(self, in_ch=1, out_ch=2, base_ch=1, depth=4, input_size=61, device=None):
        super().__init__()
        self.device = device
        self.depth = depth
        self.width = self._width
        self.chs = [base_ch * (2 ** i) for i in range(depth + 1)]
        sl, pads = _sizes_and_pads(input_size, depth)
        self.down_convs = nn.ModuleList()
        self.pools = nn.ModuleList()
        self.down_convs.append(nn.Sequential(nn.Conv1d(in_ch, self.chs[0], 3, padding=1),
                                             ConvNeXtBlock1D(self.chs[0])))
        for i in range(depth):
            self.pools.append(nn.MaxPool1d(2))
            self.down_convs.append(nn.Sequential(nn.Conv1d(self.chs[i], self.chs[i + 1], 3, padding=1),
                                                 ConvNeXtBlock1D(self.chs[i + 1])))
        self.skip_norms = nn.ModuleList([nn.BatchNorm1d(ch) for ch in self.chs])
        self.temp_atts = nn.ModuleList([TemporalSelfAttention1D(self.chs[i], sl[i]) for i in range(depth + 1)])
        self.up_transposes = nn.ModuleList()
        self.up_convs = nn.ModuleList()
        for pad, i in zip(pads, reversed(range(depth))):
            self.up_transposes.append(nn.ConvTranspose1d(self.chs[i + 1], self.chs[i], 2, stride=2,
                                                         output_padding=pad))
            self.up_convs.append(nn.Sequential(nn.Conv1d(self.chs[i] * 2, self.chs[i], 3, padding=1),
                                               ConvNeXtBlock1D(self.chs[i])))
        self.final_conv = nn.Conv1d(self.chs[0], self.width, 1)
        self._make_heads()

    def _make_heads(self):
        self.fno_drift = FNO1d(modes=15, width=self.width, n_layers=3, input_dim=self.width, output_dim=1,
                               device=self.device)
        self.fno_diffusion = FNO1d(modes=15, width=self.width, n_layers=3, input_dim=self.width,
                                   output_dim=1, device=self.device)


class PermInvUNet_attn1D_bag(PermInvUNet_attn1D):
    """PermInvUNet_attn1D_bag, 1d_FPE/NIOModules.py:326-443: as PermInvUNet_attn1D with the
    train-mode bag draw L = randint(50, T), idx = choice(T, L) (with replacement)."""

    _bag = True


class PermInvUNet_attn1D_bag_V(PermInvUNet_attn1D_bag):
    """The 1d_GPE copy of PermInvUNet_attn1D_bag (1d_GPE/NIOModules.py:342-453): width 10 and one
    head fno_V = FNO1d(modes 30) (the GPE potential); the dropin shim of 1d_GPE exports it under
    the reference's name."""

    _width = 10
    _heads = ("fno_V",)

    def _make_heads(self):
        self.fno_V = FNO1d(modes=30, width=self.width, n_layers=3, input_dim=self.width, output_dim=1,
                           device=self.device)


class PermInvUNet_attn1D_bag_GPE(PermInvUNet_attn1D_bag):
    """PermInvUNet_attn1D_bag_GPE, 1d_GPE/NIOModules.py:455-560: as the 1d_GPE bag UNet with the
    head's ``width`` and ``modes`` as constructor arguments."""

    _heads = ("fno_V",)

    def __init__(self, in_ch=1, out_ch=2, base_ch=1, depth=4, input_size=61, device=None, width=None,
                 modes=None):
        self._width = width
        self.modes = modes
        super().__init__(in_ch, out_ch, base_ch, depth, input_size, device)
        self.modes = modes

    def _make_heads(self):
        self.fno_V = FNO1d(modes=self.modes, width=self.width, n_layers=3, input_dim=self.width,
                           output_dim=1, device=self.device)
