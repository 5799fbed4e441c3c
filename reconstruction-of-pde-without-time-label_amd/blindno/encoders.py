"""CNN snapshot encoders of the NIO branch (OpenFWI-style ConvBlocks,
2d_FPE/Baselines.py:40-52,186-249,254-287).  The layer layout and initialisation order match
the reference (drop-in checkpoints); execution is on libblindno (below).

Divergence (documented in DESIGN.md): the reference's Encoder2D hard-codes its last
kernel to the grid ((2,1) for 61^2 in 2d_FPE, (3,2) for 80^2 in the non-conservative
copy) and crashes at 128^2.  Here ``last_kernel`` is a constructor argument and
``Encoder2D.kernel_for_grid(n)`` gives the kernel that collapses an n x n input to 1x1
((4,2) at 128^2).

MI355X execution of a ConvBlock: the convolution runs on libblindno's implicit-GEMM kernels
(ops.Conv2dFn, csrc/conv.hip: fp32 matrix cores, fixed accumulation order -- deterministic,
any batch size, graph-capturable; no MIOpen find/compile per new bag size), the BatchNorm2d
(batch statistics) and the LeakyReLU run fused in ops.BNActFn (csrc/batchnorm.hip).
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import ops

NORM_LAYERS = {"bn": nn.BatchNorm2d, "in": nn.InstanceNorm2d, "ln": nn.LayerNorm}


class ConvBlock(nn.Module):
    def __init__(self, in_fea, out_fea, kernel_size=3, stride=1, padding=1, norm="bn",
                 relu_slope=0.2, dropout=None):
        super().__init__()
        layers = [nn.Conv2d(in_channels=in_fea, out_channels=out_fea, kernel_size=kernel_size,
                            stride=stride, padding=padding)]
        if norm in NORM_LAYERS:
            layers.append(NORM_LAYERS[norm](out_fea))
        layers.append(nn.LeakyReLU(relu_slope, inplace=True))
        if dropout:
            layers.append(nn.Dropout2d(dropout))
        self.layers = nn.Sequential(*layers)
        self.relu_slope = relu_slope
        self._fused = norm == "bn" and not dropout

    def forward(self, x):
        """x (rows, C, H, W) -> (rows, C', H', W')."""
        if not self._fused:
            return self.layers(x)   # norms the reference's encoders never use (in / ln / dropout)
        ops.require_device(x)
        conv, bn = self.layers[0], self.layers[1]
        z = ops.conv2d(x, conv.weight, conv.bias, conv.stride, conv.padding)
        return ops.BNActFn.apply(z, bn.weight, bn.bias, bn, z.shape[0], self.relu_slope)


def _conv_out(n, k, s, p):
    return (n + 2 * p - k) // s + 1


class Encoder2D(nn.Module):
    """2d_FPE/Baselines.py:186-249 with a grid-adaptive final kernel."""

    def __init__(self, n_out, dim1=64, dim2=128, dim3=256, dim4=512, dim5=512, sample_spatial=1.0,
                 last_kernel=(2, 1), **kwargs):
        super().__init__()
        self.convblock1 = ConvBlock(1, dim1, kernel_size=(1, 7), stride=(1, 2), padding=(0, 3))
        self.convblock2_1 = ConvBlock(dim1, dim2, kernel_size=(3, 3), stride=(2, 2), padding=(1, 1))
        self.convblock2_2 = ConvBlock(dim2, dim2, kernel_size=(3, 3), padding=(1, 1))
        self.convblock3_1 = ConvBlock(dim2, dim3, kernel_size=(3, 3), stride=(2, 2), padding=(1, 1))
        self.convblock3_2 = ConvBlock(dim3, dim3, kernel_size=(3, 3), padding=(1, 1))
        self.convblock4_1 = ConvBlock(dim3, dim4, kernel_size=(3, 3), stride=(2, 2), padding=(1, 1))
        self.convblock4_2 = ConvBlock(dim4, dim4, kernel_size=(3, 3), padding=(1, 1))
        self.convblock7_1 = ConvBlock(dim4, dim5, kernel_size=(3, 3), stride=(2, 2), padding=(1, 1))
        self.convblock7_2 = ConvBlock(dim5, dim5, kernel_size=(3, 3), stride=(2, 2), padding=(1, 1))
        self.convblock7_3 = ConvBlock(dim5, dim5, kernel_size=tuple(last_kernel), padding=0)
        self.linear = nn.Linear(512, n_out)
        self.print_bool = False

    @staticmethod
    def kernel_for_grid(nx, ny=None):
        """Final kernel that maps an nx x ny snapshot to a 1x1x512 feature."""
        ny = nx if ny is None else ny
        h, w = nx, ny
        w = _conv_out(w, 7, 2, 3)                       # convblock1 (1,7) s(1,2) p(0,3)
        for _ in range(5):                              # 2_1, 3_1, 4_1, 7_1, 7_2 (stride 2)
            h, w = _conv_out(h, 3, 2, 1), _conv_out(w, 3, 2, 1)
        return (h, w)

    def forward(self, x):
        b, L = x.shape[0], x.shape[1]
        x = x.reshape(b * L, x.shape[2], x.shape[3], x.shape[4])
        for blk in (self.convblock1, self.convblock2_1, self.convblock2_2, self.convblock3_1,
                    self.convblock3_2, self.convblock4_1, self.convblock4_2, self.convblock7_1,
                    self.convblock7_2, self.convblock7_3):
            x = blk(x)
        return ops.linear(x.flatten(1).view(b, L, -1), self.linear.weight, self.linear.bias)


class Encoder(nn.Module):
    """1D snapshot encoder (1d_FPE/Baselines.py:254-287).  The final kernels are
    grid-specific per experiment directory: 1d_FPE uses (5, 4, 15) and applies
    final_conv1..3; 1d_GPE uses (5, 7, 4) and applies final_conv1..4."""

    def __init__(self, output_dim, dim1=64, dim2=128, dim3=256, final_kernels=(5, 4, 15),
                 apply_conv4=False):
        super().__init__()
        k2, k3, k4 = final_kernels
        self.conv1 = ConvBlock(1, dim1, kernel_size=(1, 3), stride=(1, 2), padding=(0, 1))
        self.conv2 = ConvBlock(dim1, dim2, kernel_size=(1, 3), stride=(1, 2), padding=(0, 1))
        self.conv3 = ConvBlock(dim2, dim3, kernel_size=(1, 3), stride=(1, 2), padding=(0, 1))
        self.final_conv1 = ConvBlock(dim3, dim3, kernel_size=(1, 5), stride=(1, 1), padding=(0, 1))
        self.final_conv2 = ConvBlock(dim3, dim3, kernel_size=(1, k2), stride=(1, 1), padding=(0, 0))
        self.final_conv3 = ConvBlock(dim3, dim3, kernel_size=(1, k3), stride=(1, 1), padding=(0, 0))
        self.final_conv4 = ConvBlock(dim3, dim3, kernel_size=(1, k4), stride=(1, 1), padding=(0, 0))
        self.linear = nn.Linear(dim3, output_dim)
        self.apply_conv4 = apply_conv4

    def forward(self, x):
        b, L, N = x.shape
        x = x.reshape(b * L, 1, 1, N)
        blocks = [self.conv1, self.conv2, self.conv3, self.final_conv1, self.final_conv2, self.final_conv3]
        if self.apply_conv4:
            blocks.append(self.final_conv4)
        for blk in blocks:
            x = blk(x)
        return ops.linear(x.reshape(b, L, -1), self.linear.weight, self.linear.bias)
