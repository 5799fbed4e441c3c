"""Drop-in FNO modules backed by the HIP kernels.

Class names, constructor signatures, attribute names, parameter shapes/dtypes and the
ORDER in which parameters are created match the reference
(2d_FPE/FNOModules.py and 1d_FPE/FNOModules.py), so ``state_dict`` checkpoints are
interchangeable and the same ``torch.manual_seed`` gives the same initial weights.
Only ``forward`` differs: one autograd node per FNO body (``ops.FNOFn``) running
libblindno kernels.  CPU tensors raise (no CPU path).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import ops


class MLP(nn.Module):
    """Unused add-on kept for import/layout compatibility (2d_FPE/FNOModules.py:11-21)."""

    def __init__(self, in_channels, out_channels, mid_channels):
        super().__init__()
        self.mlp1 = nn.Conv2d(in_channels, mid_channels, 1)
        self.mlp2 = nn.Conv2d(mid_channels, out_channels, 1)

    def forward(self, x):
        return self.mlp2(F.gelu(self.mlp1(x)))


class SpectralConv1d(nn.Module):
    """1d_FPE/FNOModules.py:27-59: rfft -> DC*0.5 -> per-mode complex mix -> irfft."""

    def __init__(self, in_channels, out_channels, modes1):
        super().__init__()
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.modes1 = modes1
        self.scale = 1 / (in_channels * out_channels)
        self.weights1 = nn.Parameter(
            self.scale * torch.rand(in_channels, out_channels, self.modes1, dtype=torch.cfloat))

    def forward(self, x):
        return ops.SpectralConvFn.apply(x, self.weights1)


class SpectralConv2d(nn.Module):
    """2d_FPE/FNOModules.py:124-178 (real-view weights (Ci,Co,m1,m2,2)); with
    ``complex_weights=True`` the cfloat variant of 1d_FPE/FNOModules.py:124-161."""

    def __init__(self, in_channels, out_channels, modes1, modes2, complex_weights=False):
        super().__init__()
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.modes1 = modes1
        self.modes2 = modes2
        self.scale = 1 / (in_channels * out_channels)
        if complex_weights:
            shp = (in_channels, out_channels, modes1, modes2)
            self.weights1 = nn.Parameter(self.scale * torch.rand(*shp, dtype=torch.cfloat))
            self.weights2 = nn.Parameter(self.scale * torch.rand(*shp, dtype=torch.cfloat))
        else:
            shp = (in_channels, out_channels, modes1, modes2, 2)
            self.weights1 = nn.Parameter(self.scale * torch.rand(*shp, dtype=torch.float32))
            self.weights2 = nn.Parameter(self.scale * torch.rand(*shp, dtype=torch.float32))

    def _real_view(self):
        w1, w2 = self.weights1, self.weights2
        if w1.is_complex():
            w1, w2 = torch.view_as_real(w1), torch.view_as_real(w2)
        return w1, w2

    def forward(self, x):
        w1, w2 = self._real_view()
        return ops.SpectralConvFn.apply(x, w1, w2)


def fno_params(m, dim):
    ps = [m.fc0.weight, m.fc0.bias]
    for s, c in zip(m.spectral_list, m.conv_list):
        if dim == 2:
            w1, w2 = s._real_view()
            ps += [w1, w2]
        else:
            ps += [s.weights1]
        ps += [c.weight, c.bias]
    ps += [m.fc1.weight, m.fc1.bias, m.fc2.weight, m.fc2.bias]
    return ps


class FNO1d(nn.Module):
    """1d_FPE/FNOModules.py:62-122 (fc2 = Linear(128, output_dim))."""

    def __init__(self, modes, width, n_layers, input_dim, output_dim, device="cpu"):
        super().__init__()
        self.modes = modes
        self.width = width
        self.n_layers = n_layers
        self.fc0 = nn.Linear(input_dim, self.width)
        self.conv_list = nn.ModuleList([nn.Conv1d(self.width, self.width, 1) for _ in range(self.n_layers)])
        self.spectral_list = nn.ModuleList(
            [SpectralConv1d(self.width, self.width, self.modes) for _ in range(self.n_layers)])
        self.padding_frac = 1 / 4
        self.fc1 = nn.Linear(self.width, 128)
        self.fc2 = nn.Linear(128, output_dim)
        self.to(device)

    def meta(self, cin):
        return ops.FNOMeta(1, self.n_layers, self.width, 1, self.modes, self.fc1.out_features,
                           self.fc2.out_features, cin)

    def forward(self, x):
        return ops.FNOFn.apply(self.meta(x.shape[-1]), x, *fno_params(self, 1))


class FNO2d(nn.Module):
    """2d_FPE/FNOModules.py:181-240 (fc2 = Linear(128, 1) regardless of output_dim, :214).

    ``complex_weights``/``device`` reproduce the 1d_FPE/1d_GPE copy of this class
    (cfloat spectral weights, ``self.to(device)``)."""

    def __init__(self, modes, width, n_layers, input_dim, output_dim, device=None,
                 complex_weights=False):
        super().__init__()
        self.modes1 = modes
        self.modes2 = modes
        self.width = width
        self.n_layers = n_layers
        self.padding_frac = 1 / 4
        self.fc0 = nn.Linear(input_dim, self.width)
        self.conv_list = nn.ModuleList([nn.Conv2d(self.width, self.width, 1) for _ in range(self.n_layers)])
        self.spectral_list = nn.ModuleList(
            [SpectralConv2d(self.width, self.width, self.modes1, self.modes2, complex_weights)
             for _ in range(self.n_layers)])
        self.fc1 = nn.Linear(self.width, 128)
        self.fc2 = nn.Linear(128, 1)
        if device is not None:
            self.to(device)

    def meta(self, cin):
        return ops.FNOMeta(2, self.n_layers, self.width, self.modes1, self.modes2,
                           self.fc1.out_features, self.fc2.out_features, cin)

    def forward(self, x):
        return ops.FNOFn.apply(self.meta(x.shape[-1]), x, *fno_params(self, 2))


class SpectralConv3d(nn.Module):
    """Layout-compatible placeholder for the 3D layer (2d_FPE/FNOModules.py:245-288).
    3D is outside this build's scope (no reference script uses it): forward raises."""

    def __init__(self, in_channels, out_channels, modes1, modes2, modes3):
        super().__init__()
        self.in_channels, self.out_channels = in_channels, out_channels
        self.modes1, self.modes2, self.modes3 = modes1, modes2, modes3
        self.scale = 1 / (in_channels * out_channels)
        shp = (in_channels, out_channels, modes1, modes2, modes3)
        for k in range(1, 5):
            setattr(self, f"weights{k}", nn.Parameter(self.scale * torch.rand(*shp, dtype=torch.cfloat)))

    def forward(self, x):
        raise NotImplementedError("SpectralConv3d/FNO3d are outside the blindno hot-path scope")


class FNO3d(nn.Module):
    """Layout-compatible placeholder (2d_FPE/FNOModules.py:290-366); forward raises."""

    def __init__(self, modes, width, n_layers, input_dim, output_dim, device="cpu"):
        super().__init__()
        self.modes1 = self.modes2 = self.modes3 = modes
        self.width = width
        self.padding = 2
        self.fc0 = nn.Linear(input_dim, self.width)
        for k in range(4):
            setattr(self, f"conv{k}", SpectralConv3d(width, width, modes, modes, modes))
        for k in range(4):
            setattr(self, f"w{k}", nn.Conv3d(width, width, 1))
        self.fc1 = nn.Linear(self.width, 128)
        self.fc2 = nn.Linear(128, output_dim)

    def forward(self, x):
        raise NotImplementedError("SpectralConv3d/FNO3d are outside the blindno hot-path scope")
