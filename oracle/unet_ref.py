"""Float64 CPU restatement of the permutation-invariant attention UNet ("BlinDNO",
PermInvUNet_attn) -- TEST INFRASTRUCTURE only (tests/, smoke(), bench.py's cpu_baseline).

Restated from the reference's behaviour:
  * 2D: ConvNeXtBlock, TemporalSelfAttention, PermInvUNet_attn (2d_FPE/NIOModules.py:1044-1181).
  * 2D NC: the 2d_Non_conservative_FPE copy of PermInvUNet_attn (2d_Non_conservative_FPE/
    NIOModules.py:897-1053) is a different network: its down/up blocks are Conv2d +
    BatchNorm2d (batch statistics over the B*L snapshots in train mode) + ReLU instead of
    ConvNeXt blocks, and its forward uses the heads fno_Fx / fno_Fy (fno_drift /
    fno_diffusion are registered but unused).
  * 1D: ConvNeXtBlock1D, TemporalSelfAttention1D, PermInvUNet_attn1D (all T snapshots) and
    PermInvUNet_attn1D_bag (train-mode bag draw) (1d_FPE/NIOModules.py:165-443; the 1d_GPE copies with one head fno_V, 1d_GPE/NIOModules.py:342-560).

The per-snapshot layers are written with torch's functional convolutions (the reference's own
building blocks, evaluated here in float64); the temporal attention is written out as the
explicit (B, L, L) score matrix, softmax, A X + X and LayerNorm over D = C*H*W, so the HIP
path's collapsed form (Gram matrix + per-token statistics, csrc/unet.hip) is checked against
the literal definition.  The FNO heads come from oracle.fno_ref (explicit truncated DFTs).

Parameters are a dict keyed exactly like the reference's state_dict.
"""
from __future__ import annotations

import math
from typing import Dict, Optional, Sequence

import torch
import torch.nn.functional as F

from . import fno_ref
from .fno_ref import sub_params


def _dt():
    return fno_ref.DT


def _gelu(x):
    return 0.5 * x * (1.0 + torch.erf(x / math.sqrt(2.0)))


def convnext(p: Dict[str, torch.Tensor], x: torch.Tensor, dim: int) -> torch.Tensor:
    """ConvNeXtBlock(1D) (2d_FPE/NIOModules.py:1044-1062, 1d_FPE/NIOModules.py:165-184):
    7(x7) depthwise conv, LayerNorm over channels (eps 1e-6), Linear(C,4C), exact GELU,
    Linear(4C,C), residual."""
    C = x.shape[1]
    conv = F.conv2d if dim == 2 else F.conv1d
    pad = (3, 3) if dim == 2 else 3
    h = conv(x, p["dwconv.weight"], p["dwconv.bias"], padding=pad, groups=C)
    perm = (0, 2, 3, 1) if dim == 2 else (0, 2, 1)
    h = h.permute(*perm)
    mu = h.mean(-1, keepdim=True)
    var = ((h - mu) ** 2).mean(-1, keepdim=True)
    h = (h - mu) / torch.sqrt(var + 1e-6) * p["norm.weight"] + p["norm.bias"]
    h = h @ p["pwconv1.weight"].T + p["pwconv1.bias"]
    h = _gelu(h)
    h = h @ p["pwconv2.weight"].T + p["pwconv2.bias"]
    inv = (0, 3, 1, 2) if dim == 2 else (0, 2, 1)
    return h.permute(*inv) + x


def temporal_attention(p: Dict[str, torch.Tensor], x: torch.Tensor) -> torch.Tensor:
    """TemporalSelfAttention(1D) (2d_FPE/NIOModules.py:1065-1083, 1d_FPE/NIOModules.py:186-209):
    tokens = the L snapshots of a bag flattened to D = C*H*W; A = softmax(X X^T / sqrt(D)),
    LayerNorm_D(A X + X) (eps 1e-5, elementwise affine of size D).  x: (B, L, C, *S)."""
    B, L = x.shape[:2]
    D = x[0, 0].numel()
    xf = x.reshape(B, L, D)
    a = torch.softmax(xf @ xf.transpose(1, 2) / math.sqrt(D), dim=-1)
    o = a @ xf + xf
    mu = o.mean(-1, keepdim=True)
    var = ((o - mu) ** 2).mean(-1, keepdim=True)
    o = (o - mu) / torch.sqrt(var + 1e-5) * p["norm.weight"] + p["norm.bias"]
    return o.reshape(x.shape)


def batch_norm_train(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, eps: float = 1e-5):
    """BatchNorm{1,2}d in train mode (batch statistics, biased variance)."""
    dims = [0] + list(range(2, x.dim()))
    mu = x.mean(dims, keepdim=True)
    var = ((x - mu) ** 2).mean(dims, keepdim=True)
    shp = [1, -1] + [1] * (x.dim() - 2)
    return (x - mu) / torch.sqrt(var + eps) * w.view(shp) + b.view(shp)


def batch_norm_eval(x, w, b, rm, rv, eps: float = 1e-5):
    shp = [1, -1] + [1] * (x.dim() - 2)
    return (x - rm.view(shp)) / torch.sqrt(rv.view(shp) + eps) * w.view(shp) + b.view(shp)


def skip_sizes(n: int, depth: int):
    s = [n]
    for _ in range(depth):
        s.append(s[-1] // 2)
    return s


def output_paddings(sizes):
    """ConvTranspose output_padding of each up step (2d_FPE/NIOModules.py:1094-1107)."""
    pads, cur = [], sizes[-1]
    for sz in reversed(sizes[:-1]):
        pads.append(sz - ((cur - 1) * 2 + 2))
        cur = sz
    return pads


def _bn(p, prefix, x, bn_train):
    w, b = p[prefix + ".weight"], p[prefix + ".bias"]
    if bn_train:
        return batch_norm_train(x, w, b)
    return batch_norm_eval(x, w, b, p[prefix + ".running_mean"].to(_dt()),
                           p[prefix + ".running_var"].to(_dt()))


def perminv_unet_attn(p: Dict[str, torch.Tensor], x: torch.Tensor, depth: int, dim: int,
                      idx: Optional[Sequence[int]] = None, bn_train: bool = True,
                      variant: str = "fpe", taps: Optional[list] = None) -> torch.Tensor:
    """PermInvUNet_attn.forward (2d_FPE/NIOModules.py:1144-1181) for dim 2, x (B, T, H, W);
    PermInvUNet_attn1D(_bag).forward (1d_FPE/NIOModules.py:283-322, 398-443) for dim 1,
    x (B, T, L); ``variant="nc"``: the 2d_Non_conservative_FPE model (ConvBlocks, heads
    fno_Fx/fno_Fy; 2d_Non_conservative_FPE/NIOModules.py:1009-1053).  ``idx`` is the
    train-mode bag (drawn with replacement by the reference); ``bn_train`` selects batch
    statistics (train mode) or running ones for every BatchNorm."""
    def tap(name, t):
        if taps is not None:
            t.retain_grad()
            taps.append((name, t))
        return t

    x = x.to(_dt())
    p = {k: (v.to(_dt()) if v.is_floating_point() else v) for k, v in p.items()}
    if idx is not None:
        x = x[:, list(idx)]
    B, L = x.shape[:2]
    spatial = x.shape[2:]
    h = x.reshape(B * L, 1, *spatial)
    conv = F.conv2d if dim == 2 else F.conv1d
    convT = F.conv_transpose2d if dim == 2 else F.conv_transpose1d
    pool = F.max_pool2d if dim == 2 else F.max_pool1d
    feats = []
    for i in range(depth + 1):
        h = conv(h, p[f"down_convs.{i}.0.weight"], p[f"down_convs.{i}.0.bias"], padding=1)
        if variant == "nc":
            h = torch.relu(_bn(p, f"down_convs.{i}.1", h, bn_train))
        else:
            h = convnext(sub_params(p, f"down_convs.{i}.1"), h, dim)
        feats.append(tap(f"feat{i}", h))
        if i < depth:
            h = pool(h, 2)

    def agg(level):
        f = feats[level]
        seq = f.reshape(B, L, *f.shape[1:])
        return tap(f"agg{level}", temporal_attention(sub_params(p, f"temp_atts.{level}"), seq).mean(1))

    h = agg(depth)
    sizes = [skip_sizes(n, depth) for n in spatial]
    pads = list(zip(*[output_paddings(s) for s in sizes]))
    for i in range(depth):
        lv = depth - 1 - i
        op = pads[i] if dim == 2 else pads[i][0]
        h = convT(h, p[f"up_transposes.{i}.weight"], p[f"up_transposes.{i}.bias"], stride=2,
                  output_padding=op)
        s = _bn(p, f"skip_norms.{lv}", agg(lv), bn_train)
        h = torch.cat([h, s], 1)
        h = conv(h, p[f"up_convs.{i}.0.weight"], p[f"up_convs.{i}.0.bias"], padding=1)
        if variant == "nc":
            h = torch.relu(_bn(p, f"up_convs.{i}.1", h, bn_train))
        else:
            h = convnext(sub_params(p, f"up_convs.{i}.1"), h, dim)
        tap(f"up{i}", h)
    fused = tap("fused", conv(h, p["final_conv.weight"], p["final_conv.bias"]))
    names = ("fno_Fx", "fno_Fy") if variant == "nc" else ("fno_drift", "fno_diffusion")
    if dim == 2:
        fused = fused.permute(0, 2, 3, 1)
        heads = [fno_ref.fno2d(sub_params(p, hd), fused) for hd in names]
    else:
        fused = fused.permute(0, 2, 1)
        names = ("fno_V",) if "fno_V.fc0.weight" in p else ("fno_drift", "fno_diffusion")
        heads = [fno_ref.fno1d(sub_params(p, hd), fused) for hd in names]
    return torch.cat(heads, dim=-1)
