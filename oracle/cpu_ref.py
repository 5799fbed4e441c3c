"""Float32 CPU restatement of the FNO-NIO training step on ``torch.fft`` -- TEST / BASELINE
INFRASTRUCTURE (``bench.py``'s ``cpu_baseline`` leg and ``tests/``), never the product path.

Device- and dtype-generic (the same code runs the fp64 arbiter of ``bench.py``'s parity leg
on the GPU with plain torch ops).  ``fno_ref`` evaluates spectral layers as explicit O(N^2) DFT sums in float64: an independent
checker, but ~3.5x slower than the reference's own CPU path.  This module restates the same
algorithm the way the reference executes it on a CPU -- pocketfft ``rfft2``/``irfft2`` with an
fp32 spectrum buffer, corner-block complex channel mixes, channels-last linear layers -- so the
CPU baseline that ``bench.py`` times beside the GPU is the reference's own speed class
(1.29 bags/s at config C on 8 threads), and so the GPU output can be compared
against a reference-precision (fp32) CPU evaluation of the same step.

Written from the reference's behaviour (citations per function); parameters are the
reference's ``state_dict`` keys, as in ``fno_ref``.  Pinned to the reference's golden vectors
by ``tests/test_oracle_golden.py::test_cpu_ref_*``.
"""
from __future__ import annotations

from typing import Dict, Optional, Sequence

import torch

from .fno_ref import pad_amount, sub_params

__all__ = ["spectral_conv2d_fft", "spectral_conv1d_fft", "fno2d_fft", "fno1d_fft",
           "niofp2d_fno_fft", "niofp_fno_fft", "encoder2d_conv", "niofp2d_fft"]


def _gelu(x):
    """Exact-erf GELU, 2d_FPE/FNOModules.py:232,238 (``F.gelu`` default: one fused op, as the
    reference calls it)."""
    return torch.nn.functional.gelu(x)


def _cplx(w):
    return w if w.is_complex() else torch.complex(w[..., 0], w[..., 1])


def spectral_conv2d_fft(x, w1, w2):
    """SpectralConv2d.forward, 2d_FPE/FNOModules.py:156-178: rfft2 -> mix the kept corners
    [:m1, :m2] (weights1) and [-m1:, :m2] (weights2; written second, so it wins on overlap,
    :170-173) -> irfft2(s=(H, W)).  The spectrum buffer is complex64 (:167)."""
    B, Ci, H, W = x.shape
    w1c, w2c = _cplx(w1), _cplx(w2)
    Co, m1, m2 = w1c.shape[1], w1c.shape[2], w1c.shape[3]
    xf = torch.fft.rfft2(x)
    out = torch.zeros(B, Co, H, W // 2 + 1, dtype=xf.dtype, device=x.device)
    out[:, :, :m1, :m2] = torch.einsum("bixy,ioxy->boxy", xf[:, :, :m1, :m2], w1c.to(xf.dtype))
    out[:, :, H - m1:, :m2] = torch.einsum("bixy,ioxy->boxy", xf[:, :, H - m1:, :m2], w2c.to(xf.dtype))
    return torch.fft.irfft2(out, s=(H, W))


def spectral_conv1d_fft(x, w):
    """SpectralConv1d.forward, 1d_FPE/FNOModules.py:47-59 (rfft, DC bin x0.5, mix the first m
    modes, irfft(n=W))."""
    B, Ci, W = x.shape
    wc = _cplx(w)
    Co, m = wc.shape[1], wc.shape[2]
    xf = torch.fft.rfft(x)
    scale = torch.ones(xf.shape[-1], dtype=xf.real.dtype, device=x.device)
    scale[0] = 0.5
    xf = xf * scale
    out = torch.zeros(B, Co, W // 2 + 1, dtype=xf.dtype, device=x.device)
    out[:, :, :m] = torch.einsum("bix,iox->box", xf[:, :, :m], wc.to(xf.dtype))
    return torch.fft.irfft(out, n=W)


def _lin(x, p, name):
    """nn.Linear (F.linear: one fused addmm, as the reference's layers run)."""
    return torch.nn.functional.linear(x, p[name + ".weight"], p.get(name + ".bias"))


def fno2d_fft(p: Dict[str, torch.Tensor], x: torch.Tensor) -> torch.Tensor:
    """FNO2d.forward, 2d_FPE/FNOModules.py:218-240 (pads right/bottom by round(N/4), exact GELU
    except after the last layer, swapped-name crop, fc2 = Linear(128, 1))."""
    n = len({k.split(".")[1] for k in p if k.startswith("spectral_list.")})
    x = _lin(x, p, "fc0").permute(0, 3, 1, 2)
    p1, p2 = pad_amount(x.shape[-1]), pad_amount(x.shape[-2])
    x = torch.nn.functional.pad(x, [0, p1, 0, p2])
    for k in range(n):
        s = spectral_conv2d_fft(x, p[f"spectral_list.{k}.weights1"], p[f"spectral_list.{k}.weights2"])
        c = torch.nn.functional.conv2d(x, p[f"conv_list.{k}.weight"], p[f"conv_list.{k}.bias"])
        x = s + c
        if k != n - 1:
            x = _gelu(x)
    x = x[..., : x.shape[-2] - p1, : x.shape[-1] - p2].permute(0, 2, 3, 1)
    return _lin(_gelu(_lin(x, p, "fc1")), p, "fc2")


def fno1d_fft(p: Dict[str, torch.Tensor], x: torch.Tensor) -> torch.Tensor:
    """FNO1d.forward, 1d_FPE/FNOModules.py:99-122."""
    n = len({k.split(".")[1] for k in p if k.startswith("spectral_list.")})
    x = _lin(x, p, "fc0").permute(0, 2, 1)
    pad = pad_amount(x.shape[-1])
    x = torch.nn.functional.pad(x, [0, pad])
    for k in range(n):
        s = spectral_conv1d_fft(x, p[f"spectral_list.{k}.weights1"])
        c = torch.nn.functional.conv1d(x, p[f"conv_list.{k}.weight"], p[f"conv_list.{k}.bias"])
        x = s + c
        if k != n - 1:
            x = _gelu(x)
    x = x[..., : x.shape[-1] - pad].permute(0, 2, 1)
    return _lin(_gelu(_lin(x, p, "fc1")), p, "fc2")


def _bag_mean(u, grid_cf, w, b):
    """Fixed-weight bag aggregation, 2d_FPE/NIOModules.py:565-575 (fc0 ``.data``: no grad)."""
    L, d = u.shape[1], grid_cf.shape[1]
    w = w.detach()
    wt = torch.cat([w[:, :d], w[:, d].view(-1, 1).repeat(1, L) / L], dim=1)
    xcat = torch.cat((grid_cf, u), 1)
    perm = (0,) + tuple(range(2, xcat.dim())) + (1,)
    return xcat.permute(*perm) @ wt.T + b.detach()


def niofp2d_fno_fft(p: Dict[str, torch.Tensor], x: torch.Tensor, grid: torch.Tensor,
                    idx: Optional[Sequence[int]] = None,
                    heads: Sequence[str] = ("fno_drift", "fno_diffusion")) -> torch.Tensor:
    """NIOFP2D_FNO.forward, 2d_FPE/NIOModules.py:543-581 (``idx``: the train-mode draw of
    :548-553, with replacement; None = eval, L = T)."""
    if idx is not None:
        x = x[:, torch.as_tensor(list(idx), device=x.device)]
    B, L, nx, ny = x.shape
    x_in = x.reshape(B * L, 1, nx, ny)
    grid_r = grid.permute(2, 0, 1).unsqueeze(0).expand(B * L, 2, nx, ny)
    inp = torch.cat((x_in, grid_r), 1).permute(0, 2, 3, 1)
    u = fno2d_fft(sub_params(p, "FNO_input"), inp).view(B, L, nx, ny)
    gcf = grid.permute(2, 0, 1).unsqueeze(0).expand(B, 2, nx, ny)
    h = _bag_mean(u, gcf, p["fc0.weight"], p["fc0.bias"])
    return torch.cat([fno2d_fft(sub_params(p, hd), h) for hd in heads], dim=-1)


def niofp_fno_fft(p: Dict[str, torch.Tensor], x: torch.Tensor, grid: torch.Tensor,
                  idx: Optional[Sequence[int]] = None,
                  heads: Sequence[str] = ("fno_drift", "fno_diffusion")) -> torch.Tensor:
    """NIOFP_FNO.forward, 1d_FPE/NIOModules.py:119-155 (GPE: ``heads=("fno_V",)``,
    1d_GPE/NIOModules.py:255-289)."""
    if idx is not None:
        x = x[:, torch.as_tensor(list(idx), device=x.device)]
    B, L, nx = x.shape
    x_in = x.reshape(B * L, nx, 1)
    inp = torch.cat((x_in, grid.unsqueeze(0).expand(B * L, nx, 1)), dim=2)
    u = fno1d_fft(sub_params(p, "FNO_input"), inp).view(B, L, nx)
    gcf = grid.unsqueeze(0).expand(B, nx, 1).permute(0, 2, 1)
    h = _bag_mean(u, gcf, p["fc0.weight"], p["fc0.bias"])
    outs = [fno1d_fft(sub_params(p, hd), h) for hd in heads]
    return torch.cat(outs, dim=-1) if len(outs) > 1 else outs[0]


# Encoder2D's ConvBlocks (name, stride, padding), 2d_FPE/Baselines.py:186-249 (the last kernel
# comes with the weights: grid-adaptive)
_ENC2D = (("convblock1", (1, 2), (0, 3)), ("convblock2_1", (2, 2), (1, 1)), ("convblock2_2", (1, 1), (1, 1)),
          ("convblock3_1", (2, 2), (1, 1)), ("convblock3_2", (1, 1), (1, 1)), ("convblock4_1", (2, 2), (1, 1)),
          ("convblock4_2", (1, 1), (1, 1)), ("convblock7_1", (2, 2), (1, 1)), ("convblock7_2", (2, 2), (1, 1)),
          ("convblock7_3", (1, 1), (0, 0)))


def encoder2d_conv(p: Dict[str, torch.Tensor], x: torch.Tensor,
                   masks: Optional[Sequence[torch.Tensor]] = None) -> torch.Tensor:
    """Encoder2D.forward in train mode, 2d_FPE/Baselines.py:203-249, executed as the reference
    does: ``F.conv2d`` -> ``F.batch_norm`` (batch statistics) -> LeakyReLU(0.2) per ConvBlock
    (:40-52), then ``linear``.  x (B, L, 1, nx, ny) -> (B, L, n_out).  ``masks``: take each
    LeakyReLU's branch from the path under test (see ``fno_ref.encoder2d``)."""
    B, L = x.shape[:2]
    h = x.reshape(B * L, *x.shape[2:])
    F = torch.nn.functional
    for k, (name, stride, pad) in enumerate(_ENC2D):
        h = F.conv2d(h, p[f"{name}.layers.0.weight"], p[f"{name}.layers.0.bias"], stride=stride, padding=pad)
        h = F.batch_norm(h, None, None, p[f"{name}.layers.1.weight"], p[f"{name}.layers.1.bias"],
                         training=True, eps=1e-5)
        h = F.leaky_relu(h, 0.2) if masks is None else torch.where(masks[k], h, 0.2 * h)
    return _lin(h.flatten(1).view(B, L, -1), p, "linear")


def _ffn(p, x, n_hidden_layers, masks=None):
    """FFN.forward, 2d_FPE/DeepONetModules.py:155-185 (leaky_relu 0.01, dropout 0, train-mode
    BatchNorm1d).  ``masks``: the LeakyReLU branches (pre-activation > 0) to take, one per
    activation -- an fp64 arbiter evaluated on the branches an fp32 run took."""
    F = torch.nn.functional

    def act(z, i):
        if masks is None:
            return F.leaky_relu(z, 0.01)
        return torch.where(masks[i].to(z.device), z, 0.01 * z)
    h = act(_lin(x, p, "input_layer"), 0)
    for k in range(n_hidden_layers - 1):
        h = act(_lin(h, p, f"hidden_layers.{k}"), k + 1)
        h = F.batch_norm(h, None, None, p[f"batch_layers.{k}.weight"], p[f"batch_layers.{k}.bias"],
                         training=True, eps=1e-5)
    return _lin(h, p, "output_layer")


def niofp2d_fft(p: Dict[str, torch.Tensor], x: torch.Tensor, grid: torch.Tensor,
                idx: Optional[Sequence[int]] = None, n_hidden_layers: int = 3,
                heads: Sequence[str] = ("fno_drift", "fno_diffusion"),
                branch_masks: Optional[Sequence[torch.Tensor]] = None,
                taps: Optional[dict] = None,
                trunk_masks: Optional[Sequence[torch.Tensor]] = None) -> torch.Tensor:
    """NIOFP2D.forward, 2d_FPE/NIOModules.py:47-83 (NC heads fno_Fx/fno_Fy:
    2d_Non_conservative_FPE/NIOModules.py:46-82): the Encoder2D branch on every drawn snapshot,
    the FFN trunk on the grid points, DeepOnetNoBiasOrg ``(w @ basis^T + b0) / sqrt(p)``
    (DeepONetModules.py:142-151), the fixed-weight bag mean, the FNO2d heads."""
    if idx is not None:
        x = x[:, torch.as_tensor(list(idx), device=x.device)]
    B, L, nx, ny = x.shape
    w = encoder2d_conv(sub_params(p, "branch"), x.unsqueeze(2), branch_masks)
    basis = _ffn(sub_params(p, "trunk"), grid.reshape(-1, 2), n_hidden_layers, trunk_masks)
    if taps is not None and basis.requires_grad:
        basis.retain_grad()          # dL/dbasis: the trunk's upstream gradient (bench.py parity)
        taps["basis"] = basis
    u = ((w @ basis.T + p["deeponet.b0"]) / basis.shape[-1] ** 0.5).view(B, L, nx, ny)
    gcf = grid.permute(2, 0, 1).unsqueeze(0).expand(B, 2, nx, ny)
    h = _bag_mean(u, gcf, p["fc0.weight"], p["fc0.bias"])
    return torch.cat([fno2d_fft(sub_params(p, hd), h) for hd in heads], dim=-1)
