"""Snapshot-bag (time-label-free) models: NIOFP2D_FNO, NIOFP_FNO, NIOFP2D, NIOFP,
NIOFP_schrodinger -- drop-in for the reference's NIOModules.

Same constructor signatures, attribute names and initialisation order as
2d_FPE/NIOModules.py:14-83,508-581, 2d_Non_conservative_FPE/NIOModules.py:13-82,503-577,
1d_FPE/NIOModules.py:15-155 and 1d_GPE/NIOModules.py:160-289.

Train mode draws the bag exactly like the reference -- ``L = np.random.randint(50, T)``,
``idx = np.random.choice(T, L)`` (with replacement) from numpy's global RNG -- so a
seeded run sees the same bags.  ``bag_idx=`` overrides the draw (parity harness).
"""
from __future__ import annotations

from typing import Optional, Sequence

import numpy as np
import torch
import torch.nn as nn

from . import ops
from .deeponet import FFN, DeepOnetNoBiasOrg
from .encoders import Encoder, Encoder2D
from .fno import FNO1d, FNO2d, fno_params


def draw_bag(T: int):
    """The reference's train-mode bag draw (2d_FPE/NIOModules.py:548-553)."""
    L = np.random.randint(50, T)
    idx = np.random.choice(T, L)
    return L, idx


def _select(module, x, bag_idx, dedup=False):
    """The bag of this step: (x[:, idx], L, lw).  With ``dedup`` (models whose per-snapshot
    encoder output does not depend on the rest of the batch -- not the BatchNorm'd NIO branch)
    the bag is reduced to its distinct snapshots and lw holds multiplicity / L."""
    if isinstance(bag_idx, tuple):
        idx_t, lw = bag_idx                       # device-resident deduplicated bag
        return x.index_select(1, idx_t), idx_t.numel(), lw
    if torch.is_tensor(bag_idx) and bag_idx.is_cuda:
        # device-resident index list (graph replays): gather on the device
        return x.index_select(1, bag_idx), bag_idx.numel(), None
    if bag_idx is not None:
        idx = np.asarray(bag_idx)
    elif module.training:
        _, idx = draw_bag(x.shape[1])
    else:
        return x, x.shape[1], None
    lw = None
    if dedup:
        idx, w = dedup_bag(idx)
        if w is not None:
            lw = torch.as_tensor(w, device=x.device)
    return x[:, torch.as_tensor(idx, device=x.device)], len(idx), lw


_SIDE = {}


HEAD_STREAMS = True     # fork the two heads over two streams (ops.HeadPairFn)
# the encoder hands the grouped heads the bag mean ubar, the heads' lift forms their input
# (False, tests only: the (B, N, N, width) field between them and two bag-mean launches)
BAG_INPUT_HEADS = True
DEDUP_BAGS = True       # run the snapshot encoder once per distinct snapshot of a bag


def dedup_bag(idx):
    """(unique indices int32, multiplicity / L float32) of a with-replacement bag draw, or
    (idx, None) when every index is distinct (or DEDUP_BAGS is off).  The encoder output of a
    repeated snapshot is identical, so the bag mean sum_l u_l = sum_u count_u u_u."""
    idx = np.asarray(idx, dtype=np.int32)
    if not DEDUP_BAGS:
        return idx, None
    uniq, counts = np.unique(idx, return_counts=True)
    if len(uniq) == len(idx):
        return idx, None
    return uniq.astype(np.int32), (counts / float(len(idx))).astype(np.float32)


def _run_heads(module, h):
    """The FNO heads on h, concatenated (2d_FPE/NIOModules.py:577-581).  On the GPU two heads run
    concurrently, forward and backward (ops.HeadPairFn: the second on a side stream forked from
    and joined back into the current one; inside a graph capture, two parallel branches).  The
    heads are small (B samples), latency-bound launches, which is why overlapping them pays."""
    heads = [getattr(module, n) for n in module._heads]
    if len(heads) != 2 or not h.is_cuda or not HEAD_STREAMS:
        return torch.cat([f(h) for f in heads], dim=-1)
    side = _SIDE.get(h.device)
    if side is None:
        side = _SIDE[h.device] = torch.cuda.Stream(h.device)
    dim = 2 if isinstance(heads[0], FNO2d) else 1
    p0, p1 = fno_params(heads[0], dim), fno_params(heads[1], dim)
    return ops.HeadPairFn.apply(heads[0].meta(h.shape[-1]), heads[1].meta(h.shape[-1]), len(p0), side,
                                h, *p0, *p1)


def _bag_mean_2d(module, u, grid, B, L, nx, ny, lw=None):
    g = grid.reshape(nx * ny, 2)
    h = ops.BagMeanFn.apply(u.reshape(B, L, nx * ny), g, module.fc0.weight.data,
                            module.fc0.bias.data, lw)
    return h.view(B, nx, ny, -1)


def _bag_mean_1d(module, u, grid, B, L, nx, lw=None):
    h = ops.BagMeanFn.apply(u.reshape(B, L, nx), grid.reshape(nx, 1), module.fc0.weight.data,
                            module.fc0.bias.data, lw)
    return h


class NIOFP2D_FNO(nn.Module):
    """FNO-NIO, 2d_FPE/NIOModules.py:508-581.  ``heads`` selects the head attribute names
    (("fno_drift", "fno_diffusion") for 2d_FPE, ("fno_Fx", "fno_Fy") for the
    non-conservative copy); ``branch_last_kernel`` is the unused Encoder2D's final kernel
    (part of the checkpoint layout)."""

    def __init__(self, input_dimensions_trunk, n_hidden_layers, neurons, n_basis, fno_layers,
                 width, modes, output_dim, heads: Sequence[str] = ("fno_drift", "fno_diffusion"),
                 branch_last_kernel=(2, 1)):
        super().__init__()
        output_dimensions = n_basis
        self.fno_layers = fno_layers
        self.branch = Encoder2D(output_dimensions, last_kernel=branch_last_kernel)
        self.fc0 = nn.Linear(3, width)
        self.FNO_input = FNO2d(modes=12, width=4, n_layers=2, input_dim=3, output_dim=1)
        self._heads = tuple(heads)
        for name in self._heads:
            setattr(self, name, FNO2d(modes=modes, width=width, n_layers=self.fno_layers,
                                      input_dim=width, output_dim=1))

    accepts_dedup_bag = True    # forward(bag_idx=(unique idx, weights)) on the fused path

    def _fused_ok(self, x, grid):
        return (x.is_cuda and x.dim() == 4 and x.dtype == torch.float32 and
                grid.dtype == torch.float32 and tuple(grid.shape) == (x.shape[2], x.shape[3], 2) and
                self.FNO_input.width <= 4 and
                not (torch.is_grad_enabled() and (x.requires_grad or grid.requires_grad)))

    def forward(self, x, grid, bag_idx=None):
        """x (B, T, Nx, Ny) standardised snapshots, grid (Nx, Ny, 2) -> (B, Nx, Ny, 2).

        Without input gradients the snapshot encoder + bag mean run as the fused HIP path
        (ops.BagEncoderFn: snapshots read from x through the bag's indices); otherwise as the
        generic composition below (same numerics, gradients for x and grid)."""
        # the grouped heads' spectral weights are packed by the encoder's pack launch
        if x.is_cuda and HEAD_STREAMS and len(self._heads) == 2 and x.dim() == 4:
            hs = [getattr(self, nm) for nm in self._heads]
            w = self.fc0.out_features
            if all(isinstance(hd, FNO2d) for hd in hs) and hs[0].meta(w).__dict__ == hs[1].meta(w).__dict__:
                ops.pack_heads_ahead(hs[0].meta(w), (x.shape[0], x.shape[2], x.shape[3], w),
                                     [fno_params(hd, 2) for hd in hs], x.device)
        try:
            out = self._encoder_heads_fused(x, grid, bag_idx)
            if out is not None:
                return out
            return self.forward_heads(self.forward_encoder(x, grid, bag_idx))
        finally:
            ops.drop_pack_ahead()

    def _encoder_heads_fused(self, x, grid, bag_idx):
        """Encoder -> grouped heads with the bag mean handed over as ubar (B, Nx, Ny): the heads'
        lift forms fc0([grid, ubar]) itself and its adjoint returns d ubar (ops.BagHeadsIn), so
        the (B, Nx, Ny, width) field and the two bag-mean launches do not exist.  None where it
        does not apply (the composition forward_heads(forward_encoder(...)) then runs)."""
        if not (BAG_INPUT_HEADS and HEAD_STREAMS and len(self._heads) == 2 and self._fused_ok(x, grid)):
            return None
        hs = [getattr(self, nm) for nm in self._heads]
        if not all(isinstance(hd, FNO2d) for hd in hs):
            return None
        w = self.fc0.out_features
        m0, m1 = hs[0].meta(w), hs[1].meta(w)
        p0, p1 = fno_params(hs[0], 2), fno_params(hs[1], 2)
        if m0.__dict__ != m1.__dict__ or not ops.GROUPED_HEADS or \
                not ops.grouped_ok(m0, (x.shape[0], x.shape[2], x.shape[3], w), [p0, p1]):
            return None
        fno = self.FNO_input
        fp = fno_params(fno, 2)
        n = len(fno.spectral_list)
        idx_t, lw = self._encoder_bag(x, bag_idx)
        if not ops.bag_ubar_ok(fno.meta(3), x.shape[0], idx_t.numel(), x.shape[2], x.shape[3],
                               fp[2 + 4 * n], fp[4 + 4 * n], m0, 2, w):
            return None
        ubar = ops.BagEncoderFn.apply(fno.meta(3), True, x, idx_t, lw, grid, self.fc0.weight.data,
                                      self.fc0.bias.data, *fp)
        side = _SIDE.get(x.device)
        if side is None:
            side = _SIDE[x.device] = torch.cuda.Stream(x.device)
        bag = ops.BagHeadsIn(grid, self.fc0.weight.data, self.fc0.bias.data)
        return ops.HeadPairFn.apply((m0, bag), m1, len(p0), side, ubar, *p0, *p1)

    def _encoder_bag(self, x, bag_idx):
        """(device bag indices, multiplicity weights or None) of the fused encoder."""
        lw = None
        if isinstance(bag_idx, tuple):
            # device-resident deduplicated bag (train.GraphedBagStep): unique indices and
            # multiplicity weights
            idx_t, lw = bag_idx
        elif torch.is_tensor(bag_idx) and bag_idx.is_cuda and bag_idx.dtype == torch.int32:
            idx_t = bag_idx                  # device-resident bag indices
        else:
            if bag_idx is not None:
                idx = np.asarray(bag_idx)
            elif self.training:
                _, idx = draw_bag(x.shape[1])
            else:
                idx = np.arange(x.shape[1])
            idx, w = dedup_bag(idx)
            idx_t = torch.as_tensor(idx, device=x.device)
            if w is not None:
                lw = torch.as_tensor(w, device=x.device)
        return idx_t, lw

    def forward_heads(self, h):
        """The two FNO heads on the bag-mean field h (B, Nx, Ny, width) (:577-581)."""
        return _run_heads(self, h)

    def forward_encoder(self, x, grid, bag_idx=None):
        """FNO_input on the bag + the fixed-weight bag mean (:548-575) -> h (B, Nx, Ny, width).
        Split from the heads so a training step can be replayed as two graphs and the heads'
        gradient all-reduce overlap the encoder's backward (train.GraphedBagStep, overlap)."""
        if self._fused_ok(x, grid):
            fno = self.FNO_input
            idx_t, lw = self._encoder_bag(x, bag_idx)
            return ops.BagEncoderFn.apply(fno.meta(3), False, x, idx_t, lw, grid, self.fc0.weight.data,
                                          self.fc0.bias.data, *fno_params(fno, 2))
        x, L, lw = _select(self, x, bag_idx, dedup=True)
        B, _, nx, ny = x.shape
        x_in = x.reshape(B * L, 1, nx, ny)
        grid_r = grid.permute(2, 0, 1).unsqueeze(0).expand(B * L, 2, nx, ny)
        inp = torch.cat((x_in, grid_r), dim=1).permute(0, 2, 3, 1).contiguous()
        u = self.FNO_input(inp)                       # (B*L, nx, ny, 1)
        return _bag_mean_2d(self, u, grid, B, L, nx, ny, lw)


def draw_bag_distinct(T: int):
    """Train-mode draw of the attention variant: WITHOUT replacement
    (2d_FPE/NIOModules.py:344-345)."""
    L = np.random.randint(50, T)
    idx = np.random.choice(T, L, replace=False)
    return L, idx


class NIOFP2D_FNO_attn(nn.Module):
    """FNO-NIO with token self-attention over the bag, 2d_FPE/NIOModules.py:300-408
    (NC copy with heads fno_Fx/fno_Fy: 2d_Non_conservative_FPE/NIOModules.py:299-407).

    The snapshot encoder FNO_input runs on every snapshot of the bag (HIP FNO2d), then
    ops.BagAttnFn forms the tokens [gx, gy, u_1..u_L], their softmax(X X^T / sqrt(nx ny))
    attention and the fc0-weighted token mean (fc0 = Linear(1, width), ``.data``), and the
    two FNO heads run as in NIOFP2D_FNO.  Registration order (FNO_input, heads, fc0) follows
    the reference, so a seeded construction gives the reference's initial weights."""

    def __init__(self, input_dimensions_trunk, n_hidden_layers, neurons, n_basis, fno_layers,
                 width, modes, output_dim, nx, ny,
                 heads: Sequence[str] = ("fno_drift", "fno_diffusion")):
        super().__init__()
        self.fno_layers = fno_layers
        self.FNO_input = FNO2d(modes=12, width=4, n_layers=2, input_dim=3, output_dim=1)
        self._heads = tuple(heads)
        for name in self._heads:
            setattr(self, name, FNO2d(modes=modes, width=width, n_layers=self.fno_layers,
                                      input_dim=width, output_dim=1))
        self.fc0 = nn.Linear(1, width)
        self.nx = nx
        self.ny = ny

    def forward(self, x, grid, bag_idx=None):
        """x (B, T, nx, ny), grid (nx, ny, 2) -> (B, nx, ny, 2).  ``bag_idx`` overrides the
        train-mode draw (a host index list or a device int tensor)."""
        ops.require_device(x, grid)
        if torch.is_tensor(bag_idx) and bag_idx.is_cuda:
            x = x.index_select(1, bag_idx)
        elif bag_idx is not None:
            x = x[:, torch.as_tensor(np.asarray(bag_idx), device=x.device)]
        elif self.training:
            _, idx = draw_bag_distinct(x.shape[1])
            x = x[:, torch.as_tensor(idx, device=x.device)]
        B, L, nx, ny = x.shape
        x_in = x.reshape(B * L, 1, nx, ny)
        grid_r = grid.permute(2, 0, 1).unsqueeze(0).expand(B * L, 2, nx, ny)
        inp = torch.cat((x_in, grid_r), dim=1).permute(0, 2, 3, 1).contiguous()
        u = self.FNO_input(inp)                                      # (B*L, nx, ny, 1)
        h = ops.BagAttnFn.apply(u.reshape(B, L, nx * ny), grid.reshape(nx * ny, 2),
                                self.fc0.weight.data, self.fc0.bias.data)
        return _run_heads(self, h.view(B, nx, ny, -1))


class NIOFP_FNO(nn.Module):
    """1D FNO-NIO: 1d_FPE/NIOModules.py:87-155 (heads fno_drift/fno_diffusion) or
    1d_GPE/NIOModules.py:228-289 (single head ``fno_V``: ``heads=("fno_V",)``)."""

    accepts_dedup_bag = True    # forward(bag_idx=(unique idx, weights)): deduplicated bag

    def __init__(self, fno_layers, width, modes, output_dim, device,
                 heads: Sequence[str] = ("fno_drift", "fno_diffusion")):
        super().__init__()
        self.device = device
        self.fno_layers = fno_layers
        self.FNO_input = FNO1d(modes=12, width=4, n_layers=2, input_dim=2, output_dim=1,
                               device=self.device)
        self.fc0 = nn.Linear(2, width)
        self._heads = tuple(heads)
        for name in self._heads:
            setattr(self, name, FNO1d(modes=modes, width=width, n_layers=self.fno_layers,
                                      input_dim=width, output_dim=1, device=self.device))

    def forward(self, x, grid, bag_idx=None):
        """x (B, T, Nx), grid (Nx, 1) -> (B, Nx, n_heads)."""
        x, L, lw = _select(self, x, bag_idx, dedup=True)
        B, _, nx = x.shape
        x_in = x.reshape(B * L, nx, 1)
        grid_r = grid.unsqueeze(0).expand(B * L, nx, 1)
        inp = torch.cat((x_in, grid_r), dim=2).contiguous()
        u = self.FNO_input(inp)                       # (B*L, nx, 1)
        h = _bag_mean_1d(self, u, grid, B, L, nx, lw)
        outs = [getattr(self, n)(h) for n in self._heads]
        return torch.cat(outs, dim=-1) if len(outs) > 1 else outs[0]


class NIOFP2D(nn.Module):
    """NIO (DeepONet branch/trunk + FNO heads), 2d_FPE/NIOModules.py:14-83 and
    2d_Non_conservative_FPE/NIOModules.py:13-82 (heads fno_Fx/fno_Fy)."""

    def __init__(self, input_dimensions_trunk, n_hidden_layers, neurons, n_basis, fno_layers,
                 width, modes, output_dim, heads: Sequence[str] = ("fno_drift", "fno_diffusion"),
                 branch_last_kernel=(2, 1)):
        super().__init__()
        output_dimensions = n_basis
        self.trunk = FFN(input_dimensions_trunk, output_dimensions, n_hidden_layers, neurons,
                         "leaky_relu", 0.0)
        self.fno_layers = fno_layers
        self.branch = Encoder2D(output_dimensions, last_kernel=branch_last_kernel)
        self.deeponet = DeepOnetNoBiasOrg(self.branch, self.trunk)
        self.fc0 = nn.Linear(3, width)
        self._heads = tuple(heads)
        for name in self._heads:
            setattr(self, name, FNO2d(modes=modes, width=width, n_layers=self.fno_layers,
                                      input_dim=width, output_dim=1))

    def forward(self, x, grid, bag_idx=None):
        """x (B, T, nx, ny), grid (nx, ny, 2) -> (B, nx, ny, 2).  The DeepONet combiner and the
        bag mean run fused (ops.DeepONetBagFn: the bag mean commutes with w basis^T + b0, so
        the (B, L, nx ny) field of DeepOnetNoBiasOrg.forward is never formed)."""
        ops.require_device(x, grid)
        x, L, _ = _select(self, x, bag_idx)
        B, _, nx, ny = x.shape
        w = self.deeponet.branch(x.unsqueeze(2))                   # (B, L, n_basis)
        basis = self.deeponet.trunk(grid.reshape(-1, 2))           # (nx ny, n_basis)
        ubar = ops.DeepONetBagFn.apply(w, basis, self.deeponet.b0)
        h = _bag_mean_2d(self, ubar.view(B, 1, nx * ny), grid, B, 1, nx, ny)
        return _run_heads(self, h)          # the two FNO heads as one grouped launch chain


class NIOFP(nn.Module):
    """1D NIO, 1d_FPE/NIOModules.py:15-84 (``heads=("fno_V",)`` + GPE encoder kernels
    give NIOFP_schrodinger, 1d_GPE/NIOModules.py:160-223)."""

    def __init__(self, input_dimensions_trunk, n_hidden_layers, neurons, n_basis, fno_layers,
                 width, modes, output_dim, device,
                 heads: Sequence[str] = ("fno_drift", "fno_diffusion"),
                 encoder_kernels=(5, 4, 15), encoder_conv4=False):
        super().__init__()
        output_dimensions = n_basis
        self.trunk = FFN(input_dimensions_trunk, output_dimensions, n_hidden_layers, neurons,
                         "leaky_relu", 0.0)
        self.fno_layers = fno_layers
        self.branch = Encoder(output_dimensions, final_kernels=encoder_kernels,
                              apply_conv4=encoder_conv4)
        self.deeponet = DeepOnetNoBiasOrg(self.branch, self.trunk)
        self.fc0 = nn.Linear(2, width)
        self.device = device
        self._heads = tuple(heads)
        for name in self._heads:
            setattr(self, name, FNO1d(modes=modes, width=width, n_layers=self.fno_layers,
                                      input_dim=width, output_dim=1, device=self.device))

    @property
    def unused_prefixes(self):
        """Parameters that never receive a gradient: the 1d_FPE encoder builds final_conv4 but
        does not apply it (1d_FPE/Baselines.py:254-287); the reference's Adam skips them."""
        return () if self.branch.apply_conv4 else ("branch.final_conv4.",)

    def forward(self, x, grid, bag_idx=None):
        ops.require_device(x, grid)
        x, L, _ = _select(self, x, bag_idx)
        B, _, nx = x.shape
        w = self.deeponet.branch(x)                                  # (B, L, n_basis)
        basis = self.deeponet.trunk(grid)                            # (nx, n_basis)
        ubar = ops.DeepONetBagFn.apply(w, basis, self.deeponet.b0)  # fused combiner + bag mean
        h = _bag_mean_1d(self, ubar.view(B, 1, nx), grid, B, 1, nx)
        outs = [getattr(self, n)(h) for n in self._heads]
        return torch.cat(outs, dim=-1) if len(outs) > 1 else outs[0]


class NIOFP_schrodinger(NIOFP):
    def __init__(self, input_dimensions_trunk, n_hidden_layers, neurons, n_basis, fno_layers,
                 width, modes, output_dim, device):
        super().__init__(input_dimensions_trunk, n_hidden_layers, neurons, n_basis, fno_layers,
                         width, modes, output_dim, device, heads=("fno_V",),
                         encoder_kernels=(5, 7, 4), encoder_conv4=True)
