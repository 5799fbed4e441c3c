"""Float64 CPU restatement of the reference's FNO/NIO hot path (TEST INFRASTRUCTURE).

Written from the reference's behaviour, not its code: spectral convolutions are
evaluated as explicit truncated DFT sums (no ``torch.fft``), so agreement with
the reference (which uses pocketfft via ``torch.fft``) is an independent check.
Gradients come from torch autograd on these float64 expressions.

Parameters are passed as ``dict[str, Tensor]`` keyed exactly like the
reference's ``state_dict`` (e.g. ``"spectral_list.0.weights1"``), so golden
fixtures captured from the reference plug straight in.
"""
from __future__ import annotations

import math
from typing import Dict, Optional, Sequence

import numpy as np
import torch
import torch.nn.functional as F

DT = torch.float64
CDT = torch.complex128

def set_precision(name: str = "fp64") -> None:
    """Switch the oracle's arithmetic type ("fp64" for parity checks, "fp32" to time it as
    the CPU baseline in the reference's own precision)."""
    global DT, CDT
    DT, CDT = (torch.float32, torch.complex64) if name == "fp32" else (torch.float64, torch.complex128)


__all__ = ["set_precision", 
    "pad_amount", "gelu", "c2r_weights", "spectral_conv2d", "spectral_conv1d",
    "fno2d", "fno1d", "bag_mean", "bag_attention", "niofp2d_fno", "niofp2d_fno_attn", "niofp_fno", "encoder2d",
    "ffn", "deeponet_nobias", "niofp2d", "encoder1d", "niofp", "mse", "train_rel_l2_2ch", "rel_l2",
    "time_averaged_relative_l2", "time_averaged_L2_error", "adam_step",
    "sub_params", "n_layers_of",
]


def pad_amount(n: int) -> int:
    """``int(round(n * 1/4))`` with Python's round-half-even.

    2d_FPE/FNOModules.py:222-223 (``x1_padding``/``x2_padding``);
    1d_FPE/FNOModules.py:105 (``x_padding``).
    """
    return int(round(n * 0.25))


def gelu(x: torch.Tensor) -> torch.Tensor:
    """Exact-erf GELU (``F.gelu`` default), 2d_FPE/FNOModules.py:232,238."""
    return 0.5 * x * (1.0 + torch.erf(x / math.sqrt(2.0)))


def c2r_weights(n: int, m: int, device=None) -> torch.Tensor:
    """Hermitian weights of a length-``n`` complex-to-real inverse over bins [0, m).

    irfft counts bin 0 (and the Nyquist bin n/2 for even n) once and every other
    bin twice; the imaginary part of the once-counted bins is ignored.
    """
    c = torch.full((m,), 2.0, dtype=DT, device=device)
    c[0] = 1.0
    if n % 2 == 0 and m > n // 2:
        c[n // 2] = 1.0
    return c


def _as_complex(w: torch.Tensor) -> torch.Tensor:
    if w.is_complex():
        return w.to(CDT)
    # real view (..., 2) -> complex; 2d_FPE/FNOModules.py:138-139,176
    w = w.to(DT)
    return torch.complex(w[..., 0], w[..., 1])


def _dft(n: int, k: int, sign: float, device=None) -> torch.Tensor:
    """(n, k) matrix exp(sign * 2*pi*i * j*kk / n) with exact integer phases."""
    j = torch.arange(n, dtype=torch.int64, device=device)[:, None]
    kk = torch.arange(k, dtype=torch.int64, device=device)[None, :]
    ph = ((j * kk) % n).to(DT) * (2.0 * math.pi / n)
    return torch.complex(torch.cos(ph), sign * torch.sin(ph))


def kept_rows(H: int, m1: int):
    """Frequency rows kept by SpectralConv2d and the weight that owns each.

    Rows [0, m1) use weights1[:, :, j]; rows [H-m1, H) use weights2[:, :, j];
    where the two ranges overlap (H < 2*m1) the second assignment wins
    (2d_FPE/FNOModules.py:170-173).  Returns a sorted list of
    ``(row, which, j)`` with ``which`` in {1, 2}.
    """
    if m1 > H:
        raise ValueError(f"modes1={m1} exceeds grid rows {H}")
    owner = {}
    for j in range(m1):
        owner[j] = (1, j)
    for j in range(m1):
        owner[H - m1 + j] = (2, j)
    return [(r, owner[r][0], owner[r][1]) for r in sorted(owner)]


def spectral_conv2d(x: torch.Tensor, w1: torch.Tensor, w2: torch.Tensor) -> torch.Tensor:
    """SpectralConv2d.forward, 2d_FPE/FNOModules.py:156-178 (and the cfloat
    variant 1d_FPE/FNOModules.py:146-161).

    x (B, Ci, H, W) real; w1/w2 (Ci, Co, m1, m2, 2) real-view or (Ci, Co, m1, m2)
    complex.  rfft2 -> per-mode complex channel mix on the kept corner blocks ->
    irfft2(s=(H, W)), evaluated as truncated DFTs.
    """
    x = x.to(DT)
    w1c, w2c = _as_complex(w1), _as_complex(w2)
    m1, m2 = w1c.shape[2], w1c.shape[3]
    H, W = x.shape[-2], x.shape[-1]
    if m2 > W // 2 + 1:
        raise ValueError(f"modes2={m2} exceeds W//2+1={W // 2 + 1}")
    dev = x.device
    rows = kept_rows(H, m1)
    r_idx = torch.tensor([r for r, _, _ in rows], dtype=torch.int64, device=dev)
    wt = torch.stack([(w1c if which == 1 else w2c)[:, :, j, :] for _, which, j in rows], 0)  # (K,Ci,Co,m2)
    fw = _dft(W, m2, -1.0, dev)                   # (W, m2)
    a = torch.einsum("bihw,wk->bihk", x.to(CDT), fw)
    fh = _dft(H, H, -1.0, dev)[:, r_idx].T        # (K, H): exp(-2 pi i r h / H)
    xh = torch.einsum("rh,bihk->birk", fh, a)
    yh = torch.einsum("birk,riok->bork", xh, wt)
    gh = _dft(H, H, +1.0, dev)[:, r_idx] / H     # (H, K)
    z = torch.einsum("hr,bork->bohk", gh, yh)
    c = c2r_weights(W, m2, dev).to(CDT) / W
    gw = _dft(W, m2, +1.0, dev).T                 # (m2, W)
    y = torch.einsum("bohk,kw->bohw", z * c, gw)
    return y.real


def spectral_conv1d(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """SpectralConv1d.forward, 1d_FPE/FNOModules.py:47-59.

    rfft -> DC bin halved (``x_ft[:, :, 0] *= 0.5``, :51) -> einsum bix,iox->box on
    the first m modes -> irfft(n=W).
    """
    x = x.to(DT)
    wc = _as_complex(w)
    m = wc.shape[2]
    W = x.shape[-1]
    if m > W // 2 + 1:
        raise ValueError(f"modes={m} exceeds W//2+1={W // 2 + 1}")
    dev = x.device
    xf = torch.einsum("biw,wk->bik", x.to(CDT), _dft(W, m, -1.0, dev))
    half = torch.ones(m, dtype=CDT, device=dev)
    half[0] = 0.5
    xf = xf * half
    yf = torch.einsum("bik,iok->bok", xf, wc)
    c = c2r_weights(W, m, dev).to(CDT) / W
    y = torch.einsum("bok,kw->bow", yf * c, _dft(W, m, +1.0, dev).T)
    return y.real


def sub_params(p: Dict[str, torch.Tensor], prefix: str) -> Dict[str, torch.Tensor]:
    n = len(prefix) + 1
    return {k[n:]: v for k, v in p.items() if k.startswith(prefix + ".")}


def n_layers_of(p: Dict[str, torch.Tensor]) -> int:
    return len({k.split(".")[1] for k in p if k.startswith("spectral_list.")})


def _linear(x, p, name):
    y = x @ p[name + ".weight"].to(DT).T
    b = p.get(name + ".bias")
    return y if b is None else y + b.to(DT)


def fno2d(p: Dict[str, torch.Tensor], x: torch.Tensor) -> torch.Tensor:
    """FNO2d.forward, 2d_FPE/FNOModules.py:218-240.

    fc0 -> NCHW -> zero-pad right/bottom by round(N/4) -> n x [spectral + 1x1 conv,
    GELU except after the last] -> crop (with the reference's swapped pad names,
    :234) -> fc1 -> GELU -> fc2 (Linear(128, 1) regardless of output_dim, :214).
    """
    n = n_layers_of(p)
    x = _linear(x.to(DT), p, "fc0").permute(0, 3, 1, 2)
    p1 = pad_amount(x.shape[-1])    # x1_padding: from W, pads W
    p2 = pad_amount(x.shape[-2])    # x2_padding: from H, pads H
    x = F.pad(x, [0, p1, 0, p2])
    for k in range(n):
        s = spectral_conv2d(x, p[f"spectral_list.{k}.weights1"], p[f"spectral_list.{k}.weights2"])
        cw = p[f"conv_list.{k}.weight"].to(DT)[:, :, 0, 0]
        c = torch.einsum("oi,bihw->bohw", cw, x) + p[f"conv_list.{k}.bias"].to(DT)[None, :, None, None]
        x = s + c
        if k != n - 1:
            x = gelu(x)
    x = x[..., : x.shape[-2] - p1, : x.shape[-1] - p2]   # x[..., :-x1_padding, :-x2_padding]
    x = x.permute(0, 2, 3, 1)
    x = gelu(_linear(x, p, "fc1"))
    return _linear(x, p, "fc2")


def fno1d(p: Dict[str, torch.Tensor], x: torch.Tensor) -> torch.Tensor:
    """FNO1d.forward, 1d_FPE/FNOModules.py:99-122 (fc2 = Linear(128, output_dim))."""
    n = n_layers_of(p)
    x = _linear(x.to(DT), p, "fc0").permute(0, 2, 1)
    pad = pad_amount(x.shape[-1])
    x = F.pad(x, [0, pad])
    for k in range(n):
        s = spectral_conv1d(x, p[f"spectral_list.{k}.weights1"])
        cw = p[f"conv_list.{k}.weight"].to(DT)[:, :, 0]
        c = torch.einsum("oi,biw->bow", cw, x) + p[f"conv_list.{k}.bias"].to(DT)[None, :, None]
        x = s + c
        if k != n - 1:
            x = gelu(x)
    x = x[..., : x.shape[-1] - pad]
    x = x.permute(0, 2, 1)
    x = gelu(_linear(x, p, "fc1"))
    return _linear(x, p, "fc2")


def bag_mean(u: torch.Tensor, grid_cf: torch.Tensor, w: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """Fixed-weight snapshot-bag aggregation (C4).

    2d_FPE/NIOModules.py:565-575 / 1d_FPE/NIOModules.py:140-149: concatenate
    [grid channels, u_1..u_L] and multiply by W' = [W[:, :d], W[:, d]/L repeated
    L times]^T plus bias, i.e. W_grid.grid + W_u.mean_l(u_l) + b.  ``w``/``b``
    are ``fc0.weight.data``/``fc0.bias.data`` (no gradient).

    u: (B, L, *S); grid_cf: (B, d, *S) channel-first grid.  Returns (B, *S, width).
    """
    L = u.shape[1]
    d = grid_cf.shape[1]
    w = w.detach().to(DT)
    wt = torch.cat([w[:, :d], w[:, d].view(-1, 1).repeat(1, L) / L], dim=1)
    xcat = torch.cat((grid_cf.to(DT), u.to(DT)), 1)
    perm = (0,) + tuple(range(2, xcat.dim())) + (1,)
    return xcat.permute(*perm) @ wt.T + b.detach().to(DT)


def niofp2d_fno(p: Dict[str, torch.Tensor], x: torch.Tensor, grid: torch.Tensor,
                idx: Optional[Sequence[int]] = None,
                heads: Sequence[str] = ("fno_drift", "fno_diffusion")) -> torch.Tensor:
    """NIOFP2D_FNO.forward, 2d_FPE/NIOModules.py:543-581 (NC copy with heads
    fno_Fx/fno_Fy: 2d_Non_conservative_FPE/NIOModules.py:539-577).

    ``idx`` replaces the numpy draw of train mode (:548-553, with replacement);
    ``None`` is eval mode (L = T).
    """
    x = x.to(DT)
    if idx is not None:
        x = x[:, list(idx)]
    B, L, nx, ny = x.shape
    g = grid.to(DT)
    x_in = x.reshape(B * L, 1, nx, ny)
    grid_r = g.permute(2, 0, 1).unsqueeze(0).repeat(B * L, 1, 1, 1)
    inp = torch.cat((x_in, grid_r), 1).permute(0, 2, 3, 1)
    u = fno2d(sub_params(p, "FNO_input"), inp).view(B, L, nx, ny)
    gcf = g.unsqueeze(0).repeat(B, 1, 1, 1).permute(0, 3, 1, 2)
    h = bag_mean(u, gcf, p["fc0.weight"], p["fc0.bias"])
    outs = [fno2d(sub_params(p, hd), h) for hd in heads]
    return torch.cat(outs, dim=-1)


def bag_attention(u: torch.Tensor, grid_cf: torch.Tensor, w: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """Token self-attention + fixed-weight fusion of NIOFP2D_FNO_attn
    (2d_FPE/NIOModules.py:365-399; NC copy 2d_Non_conservative_FPE/NIOModules.py:364-398).

    Tokens X = [gx, gy, u_1..u_L] flattened to d = nx*ny (:369-375); scores X X^T / sqrt(d)
    (:376-378), row softmax (:379), Z = A X (:381); fused = Z^T w[:, 0] / T + bias with
    T = L + 2 (:391-399; fc0 = Linear(1, width), ``.data``: no gradient).
    u: (B, L, nx, ny); grid_cf: (B, 2, nx, ny).  Returns (B, nx, ny, width)."""
    xt = torch.cat((grid_cf.to(DT), u.to(DT)), 1)
    B, T, nx, ny = xt.shape
    d = nx * ny
    xf = xt.reshape(B, T, d)
    a = torch.softmax(xf @ xf.transpose(1, 2) / math.sqrt(d), dim=-1)
    z = (a @ xf).view(B, T, nx, ny)
    wt = w.detach().to(DT)[:, 0:1].repeat(1, T) / T
    return z.permute(0, 2, 3, 1) @ wt.T + b.detach().to(DT)


def niofp2d_fno_attn(p: Dict[str, torch.Tensor], x: torch.Tensor, grid: torch.Tensor,
                     idx: Optional[Sequence[int]] = None,
                     heads: Sequence[str] = ("fno_drift", "fno_diffusion")) -> torch.Tensor:
    """NIOFP2D_FNO_attn.forward, 2d_FPE/NIOModules.py:338-408 (NC: fno_Fx/fno_Fy).
    ``idx`` replaces the train-mode draw (:343-346, WITHOUT replacement); None = eval."""
    x = x.to(DT)
    if idx is not None:
        x = x[:, list(idx)]
    B, L, nx, ny = x.shape
    g = grid.to(DT)
    x_in = x.reshape(B * L, 1, nx, ny)
    grid_r = g.permute(2, 0, 1).unsqueeze(0).repeat(B * L, 1, 1, 1)
    inp = torch.cat((x_in, grid_r), 1).permute(0, 2, 3, 1)
    u = fno2d(sub_params(p, "FNO_input"), inp).view(B, L, nx, ny)
    gcf = g.unsqueeze(0).repeat(B, 1, 1, 1).permute(0, 3, 1, 2)
    h = bag_attention(u, gcf, p["fc0.weight"], p["fc0.bias"])
    return torch.cat([fno2d(sub_params(p, hd), h) for hd in heads], dim=-1)


def niofp_fno(p: Dict[str, torch.Tensor], x: torch.Tensor, grid: torch.Tensor,
              idx: Optional[Sequence[int]] = None,
              heads: Sequence[str] = ("fno_drift", "fno_diffusion")) -> torch.Tensor:
    """NIOFP_FNO.forward, 1D FPE 1d_FPE/NIOModules.py:119-155; 1D GPE
    1d_GPE/NIOModules.py:255-289 (single head ``fno_V``)."""
    x = x.to(DT)
    if idx is not None:
        x = x[:, list(idx)]
    B, L, nx = x.shape
    g = grid.to(DT)                               # (nx, 1)
    x_in = x.reshape(B * L, nx, 1)
    grid_r = g.unsqueeze(0).repeat(B * L, 1, 1)
    inp = torch.cat((x_in, grid_r), dim=2)
    u = fno1d(sub_params(p, "FNO_input"), inp).view(B, L, nx)
    gcf = g.unsqueeze(0).repeat(B, 1, 1).permute(0, 2, 1)
    h = bag_mean(u, gcf, p["fc0.weight"], p["fc0.bias"])
    outs = [fno1d(sub_params(p, hd), h) for hd in heads]
    return torch.cat(outs, dim=-1) if len(outs) > 1 else outs[0]


# --------------------------------------------------------------------------- NIO branch/trunk
_ENC2D_BLOCKS = [
    # name, stride, padding  (2d_FPE/Baselines.py:190-200)
    ("convblock1", (1, 2), (0, 3)),
    ("convblock2_1", (2, 2), (1, 1)),
    ("convblock2_2", (1, 1), (1, 1)),
    ("convblock3_1", (2, 2), (1, 1)),
    ("convblock3_2", (1, 1), (1, 1)),
    ("convblock4_1", (2, 2), (1, 1)),
    ("convblock4_2", (1, 1), (1, 1)),
    ("convblock7_1", (2, 2), (1, 1)),
    ("convblock7_2", (2, 2), (1, 1)),
    ("convblock7_3", (1, 1), (0, 0)),
]


def encoder2d(p: Dict[str, torch.Tensor], x: torch.Tensor,
              masks: Optional[Sequence[torch.Tensor]] = None, record: Optional[list] = None) -> torch.Tensor:
    """Encoder2D.forward (train-mode BatchNorm), 2d_FPE/Baselines.py:203-249.

    ConvBlock = Conv2d -> BatchNorm2d (batch statistics) -> LeakyReLU(0.2)
    (2d_FPE/Baselines.py:40-52).  x (B, L, 1, nx, ny) -> (B, L, n_out).

    ``masks`` (optional, one bool tensor per block, True where the pre-activation is > 0): take
    each LeakyReLU's branch from the path under test instead of from this evaluation.  The model
    is piecewise linear, its gradient jumps across a branch, and a pre-activation within fp32
    rounding of 0 can land on either side in two correct evaluations; with the checked path's own
    branches the comparison is of one linear piece (tests/test_gpu_encoder.py, test_gpu_configs.py).
    ``record`` (optional list): receives this evaluation's own branch masks (pre-activation > 0).
    """
    B, L = x.shape[:2]
    h = x.reshape(B * L, *x.shape[2:]).to(DT)
    for k, (name, stride, pad) in enumerate(_ENC2D_BLOCKS):
        h = F.conv2d(h, p[f"{name}.layers.0.weight"].to(DT), p[f"{name}.layers.0.bias"].to(DT),
                     stride=stride, padding=pad)
        h = F.batch_norm(h, None, None, p[f"{name}.layers.1.weight"].to(DT),
                         p[f"{name}.layers.1.bias"].to(DT), training=True, eps=1e-5)
        if record is not None:
            record.append(h.detach() > 0)
        h = F.leaky_relu(h, 0.2) if masks is None else torch.where(masks[k], h, 0.2 * h)
    h = h.flatten(1).view(B, L, -1)
    return _linear(h, p, "linear")


def encoder1d(p: Dict[str, torch.Tensor], x: torch.Tensor, kernels=(5, 4, 15), conv4: bool = False,
              masks: Optional[Sequence[torch.Tensor]] = None) -> torch.Tensor:
    """1D snapshot Encoder.forward (train-mode BatchNorm), 1d_FPE/Baselines.py:254-287 (final
    kernels 5, 4, 15; final_conv1..3 applied) and 1d_GPE/Baselines.py:254-287 (5, 7, 4;
    final_conv1..4 applied).  Each (1, k) ConvBlock is a Conv2d over a (B L, C, 1, N) image.
    x (B, L, N) -> (B, L, n_out).  ``masks``: see encoder2d."""
    B, L, N = x.shape
    h = x.reshape(B * L, 1, 1, N).to(DT)
    blocks = [("conv1", (1, 2), (0, 1)), ("conv2", (1, 2), (0, 1)), ("conv3", (1, 2), (0, 1)),
              ("final_conv1", (1, 1), (0, 1)), ("final_conv2", (1, 1), (0, 0)),
              ("final_conv3", (1, 1), (0, 0))]
    if conv4:
        blocks.append(("final_conv4", (1, 1), (0, 0)))
    for k, (name, stride, pad) in enumerate(blocks):
        h = F.conv2d(h, p[f"{name}.layers.0.weight"].to(DT), p[f"{name}.layers.0.bias"].to(DT),
                     stride=stride, padding=pad)
        h = F.batch_norm(h, None, None, p[f"{name}.layers.1.weight"].to(DT),
                         p[f"{name}.layers.1.bias"].to(DT), training=True, eps=1e-5)
        h = F.leaky_relu(h, 0.2) if masks is None else torch.where(masks[k], h, 0.2 * h)
    return _linear(h.reshape(B, L, -1), p, "linear")


def niofp(p: Dict[str, torch.Tensor], x: torch.Tensor, grid: torch.Tensor,
          idx: Optional[Sequence[int]] = None, n_hidden_layers: int = 3,
          heads: Sequence[str] = ("fno_drift", "fno_diffusion"), kernels=(5, 4, 15),
          conv4: bool = False, branch_masks: Optional[Sequence[torch.Tensor]] = None) -> torch.Tensor:
    """1D NIO: NIOFP.forward 1d_FPE/NIOModules.py:55-84; NIOFP_schrodinger.forward
    1d_GPE/NIOModules.py:194-223 (heads ("fno_V",), kernels (5, 7, 4), conv4=True).
    x (B, T, N), grid (N, 1)."""
    x = x.to(DT)
    if idx is not None:
        x = x[:, list(idx)]
    B, L, nx = x.shape
    g = grid.to(DT)
    w = encoder1d(sub_params(p, "branch"), x, kernels, conv4, branch_masks)
    basis = ffn(sub_params(p, "trunk"), g.reshape(-1, 1), n_hidden_layers)
    u = deeponet_nobias(w, basis, p["deeponet.b0"]).view(B, L, nx)
    gcf = g.unsqueeze(0).repeat(B, 1, 1).permute(0, 2, 1)
    h = bag_mean(u, gcf, p["fc0.weight"], p["fc0.bias"])
    outs = [fno1d(sub_params(p, hd), h) for hd in heads]
    return torch.cat(outs, dim=-1) if len(outs) > 1 else outs[0]


def ffn(p: Dict[str, torch.Tensor], x: torch.Tensor, n_hidden_layers: int) -> torch.Tensor:
    """FFN.forward (leaky_relu slope 0.01, dropout 0, train-mode BatchNorm1d),
    2d_FPE/DeepONetModules.py:155-185."""
    h = F.leaky_relu(_linear(x.to(DT), p, "input_layer"), 0.01)
    for k in range(n_hidden_layers - 1):
        h = F.leaky_relu(_linear(h, p, f"hidden_layers.{k}"), 0.01)
        h = F.batch_norm(h, None, None, p[f"batch_layers.{k}.weight"].to(DT),
                         p[f"batch_layers.{k}.bias"].to(DT), training=True, eps=1e-5)
    return _linear(h, p, "output_layer")


def deeponet_nobias(weights: torch.Tensor, basis: torch.Tensor, b0: torch.Tensor) -> torch.Tensor:
    """DeepOnetNoBiasOrg.forward, 2d_FPE/DeepONetModules.py:142-151:
    (weights @ basis^T + b0) / sqrt(p)."""
    p = basis.shape[-1]
    return (weights @ basis.T + b0.to(DT)) / p ** 0.5


def niofp2d(p: Dict[str, torch.Tensor], x: torch.Tensor, grid: torch.Tensor,
            idx: Optional[Sequence[int]] = None, n_hidden_layers: int = 3,
            heads: Sequence[str] = ("fno_drift", "fno_diffusion"),
            branch_masks: Optional[Sequence[torch.Tensor]] = None) -> torch.Tensor:
    """NIOFP2D.forward, 2d_FPE/NIOModules.py:47-83 (NC: heads fno_Fx/fno_Fy,
    2d_Non_conservative_FPE/NIOModules.py:46-82).  ``branch_masks``: see encoder2d."""
    x = x.to(DT)
    if idx is not None:
        x = x[:, list(idx)]
    B, L, nx, ny = x.shape
    g = grid.to(DT)
    w = encoder2d(sub_params(p, "branch"), x.unsqueeze(2), branch_masks)
    basis = ffn(sub_params(p, "trunk"), g.reshape(-1, 2), n_hidden_layers)
    u = deeponet_nobias(w, basis, p["deeponet.b0"]).view(B, L, nx, ny)
    gcf = g.unsqueeze(0).repeat(B, 1, 1, 1).permute(0, 3, 1, 2)
    h = bag_mean(u, gcf, p["fc0.weight"], p["fc0.bias"])
    return torch.cat([fno2d(sub_params(p, hd), h) for hd in heads], dim=-1)


# --------------------------------------------------------------------------- losses / metrics
def mse(pred: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
    """nn.MSELoss() (mean), 2d_FPE/train_fno.py:116,142."""
    return ((pred.to(DT) - target.to(DT)) ** 2).mean()


def train_rel_l2_2ch(pred: torch.Tensor, out: torch.Tensor):
    """Train-loop test metric, 2d_FPE/train_fno.py:160-163.

    Per sample ||p_c - y_c||_2 / ||y||_2 where the denominator is the norm of
    BOTH output channels (the reference's quirk).  Returns (err_ch0, err_ch1),
    each of shape (B,).
    """
    pred, out = pred.to(DT), out.to(DT)
    B = pred.shape[0]
    den = torch.norm(out.reshape(B, -1), dim=1)
    e0 = torch.norm((pred[..., 0] - out[..., 0]).reshape(B, -1), dim=1) / den
    e1 = torch.norm((pred[..., 1] - out[..., 1]).reshape(B, -1), dim=1) / den
    return e0, e1


def rel_l2(a: np.ndarray, b: np.ndarray, eps: float = 1e-12) -> float:
    """||a-b||_2 / (||b||_2 + eps), 2d_FPE/eval_fno.py:124-128."""
    a = np.asarray(a, dtype=np.float64).ravel()
    b = np.asarray(b, dtype=np.float64).ravel()
    return float(np.sqrt(np.sum((a - b) ** 2)) / (np.sqrt(np.sum(b * b)) + eps))


def time_averaged_relative_l2(pt_pred: np.ndarray, pt_ref: np.ndarray, eps: float = 1e-12) -> float:
    """Mean over frames of per-frame relative L2,
    2d_Non_conservative_FPE/compute_time_error.py:321-333."""
    pt_pred = np.asarray(pt_pred, dtype=np.float64)
    pt_ref = np.asarray(pt_ref, dtype=np.float64)
    if pt_pred.shape != pt_ref.shape:
        raise ValueError("Pred/ref density shapes must match.")
    nt = pt_pred.shape[0]
    d = (pt_pred - pt_ref).reshape(nt, -1)
    r = pt_ref.reshape(nt, -1)
    num = np.sqrt(np.sum(d * d, axis=1))
    den = np.sqrt(np.sum(r * r, axis=1)) + eps
    return float(np.mean(num / den))


def _trapz_rows(f: np.ndarray, x: np.ndarray) -> np.ndarray:
    dx = np.diff(x)
    return np.sum(0.5 * (f[:, 1:] + f[:, :-1]) * dx[None, :], axis=1)


def time_averaged_L2_error(time_ref, rho_ref, time_pred, rho_pred, grid, eps: float = 1e-12) -> float:
    """1d_FPE/compute_time_error.py:240-295: per-t sqrt(trapz(diff^2, x)) /
    (sqrt(trapz(ref^2, x)) + eps), then a trapezoid time average / (t_end - t_0)."""
    rho_ref = np.asarray(rho_ref, dtype=np.float64)
    rho_pred = np.asarray(rho_pred, dtype=np.float64)
    if rho_ref.shape != rho_pred.shape:
        raise ValueError("rho_ref / rho_pred shape mismatch")
    g = np.asarray(grid[0] if isinstance(grid, (list, tuple)) else grid, dtype=np.float64)
    if g.ndim == 2 and g.shape[0] == 1:
        g = g[0]
    if g.ndim != 1:
        raise ValueError(f"unsupported grid shape {g.shape}")
    diff = _trapz_rows((rho_pred - rho_ref) ** 2, g)
    ref = _trapz_rows(rho_ref ** 2, g)
    rel = np.sqrt(np.maximum(diff, 0.0)) / (np.sqrt(np.maximum(ref, 0.0)) + eps)
    t = np.asarray(time_ref, dtype=np.float64)
    if not np.allclose(t, np.asarray(time_pred, dtype=np.float64)):
        raise ValueError("time_ref and time_pred differ")
    integral = np.sum(0.5 * (rel[:-1] + rel[1:]) * np.diff(t))
    return float(integral / (t[-1] - t[0]))


def adam_step(param: torch.Tensor, grad: torch.Tensor, exp_avg: torch.Tensor, exp_avg_sq: torch.Tensor,
              step: int, lr: float, beta1: float = 0.9, beta2: float = 0.999, eps: float = 1e-8):
    """torch.optim.Adam single-tensor update (no weight decay, no amsgrad) as used
    by every train script (2d_FPE/train_fno.py:117,144).  Complex params are
    updated through their real view.  Returns new (param, exp_avg, exp_avg_sq)."""
    def rv(t):
        return torch.view_as_real(t).to(DT) if t.is_complex() else t.to(DT)
    p, g, m, v = rv(param), rv(grad), rv(exp_avg), rv(exp_avg_sq)
    m = beta1 * m + (1 - beta1) * g
    v = beta2 * v + (1 - beta2) * g * g
    bc1 = 1 - beta1 ** step
    bc2 = 1 - beta2 ** step
    denom = v.sqrt() / math.sqrt(bc2) + eps
    p = p - (lr / bc1) * m / denom
    return p, m, v
