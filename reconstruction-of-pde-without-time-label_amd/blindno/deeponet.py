"""DeepONet building blocks (2d_FPE/DeepONetModules.py; identical in every experiment
directory).  Same classes, attribute names and initialisation as the reference; the
trunk FFN is a handful of tiny GEMMs and runs as torch ops on the device.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn


def kaiming_init(m):
    """2d_FPE/DeepONetModules.py:7-10."""
    if type(m) == nn.Linear:  # noqa: E721  (exact-type test, as the reference)
        torch.nn.init.kaiming_uniform_(m.weight.data, a=0.01, nonlinearity="leaky_relu")
        torch.nn.init.zeros_(m.bias.data)


class FourierFeatures(nn.Module):
    def __init__(self, scale, mapping_size, device):
        super().__init__()
        self.mapping_size = mapping_size
        self.B = scale * torch.randn((self.mapping_size, 2)).to(device)

    def forward(self, x):
        x_proj = torch.matmul((2.0 * np.pi * x), self.B.T)
        return torch.cat([torch.sin(x_proj), torch.cos(x_proj)], axis=-1)


class Swish(nn.Module):
    def forward(self, x):
        return x * torch.sigmoid(x)


class Sin(nn.Module):
    def forward(self, x):
        return torch.sin(x)


def activation(name):
    """2d_FPE/DeepONetModules.py:42-64."""
    table = {
        "tanh": nn.Tanh, "Tanh": nn.Tanh,
        "relu": lambda: nn.ReLU(inplace=True), "ReLU": lambda: nn.ReLU(inplace=True),
        "leaky_relu": lambda: nn.LeakyReLU(inplace=True),
        "sigmoid": nn.Sigmoid, "Sigmoid": nn.Sigmoid,
        "softplus": lambda: nn.Softplus(beta=4), "Softplus": lambda: nn.Softplus(beta=4),
        "celu": nn.CELU, "CeLU": nn.CELU, "elu": nn.ELU, "swish": Swish, "mish": nn.Mish,
        "sin": Sin,
    }
    if name not in table:
        raise ValueError("Unknown activation function")
    return table[name]()


def init_xavier(model):
    torch.manual_seed(model.retrain)

    def init_weights(m):
        if type(m) == nn.Linear and m.weight.requires_grad and m.bias.requires_grad:  # noqa: E721
            if model.act_string in ("tanh", "relu", "leaky_relu"):
                gain = nn.init.calculate_gain(model.act_string)
            else:
                gain = 1
            torch.nn.init.xavier_uniform_(m.weight, gain=gain)
            m.bias.data.fill_(0)

    model.apply(init_weights)


class _FFNBase(nn.Module):
    def _build(self, input_dimension, output_dimension, n_hidden_layers, neurons, act_string,
               dropout_rate):
        self.input_dimension = input_dimension
        self.output_dimension = output_dimension
        self.n_hidden_layers = n_hidden_layers
        self.neurons = neurons
        self.act_string = act_string
        self.dropout_rate = dropout_rate
        self.input_layer = nn.Linear(self.input_dimension, self.neurons)
        self.hidden_layers = nn.ModuleList(
            [nn.Linear(self.neurons, self.neurons) for _ in range(self.n_hidden_layers - 1)])
        self.batch_layers = nn.ModuleList(
            [nn.BatchNorm1d(self.neurons) for _ in range(self.n_hidden_layers - 1)])
        self.output_layer = nn.Linear(self.neurons, self.output_dimension)
        self.activation = activation(self.act_string)
        self.dropout = nn.Dropout(self.dropout_rate)

    def forward(self, x):
        if self._native_ok(x):
            return self._forward_native(x)
        x = self.activation(self.input_layer(x))
        for l, b in zip(self.hidden_layers, self.batch_layers):
            x = b(self.activation(self.dropout(l(x))))
        return self.output_layer(x)

    def _native_ok(self, x):
        return (x.is_cuda and x.dtype == torch.float32 and isinstance(self.activation, nn.LeakyReLU)
                and (self.dropout.p == 0.0 or not self.training)
                and all(type(b) is nn.BatchNorm1d for b in self.batch_layers))

    def _forward_native(self, x):
        """The same layers on libblindno (ops.linear: 1x1-convolution GEMMs; ops.BNActFn with
        slope 1: BatchNorm1d with batch statistics and running-statistics updates like
        nn.BatchNorm1d), LeakyReLU as the torch elementwise op: no BLAS library call and no
        torch reduction, so a step that contains the trunk can be captured in a HIP graph and
        replayed in any order (tests/test_gpu_graphs.py)."""
        from . import ops
        slope = self.activation.negative_slope
        F = torch.nn.functional
        # record_branches: a list receives each LeakyReLU's branch mask (pre-activation > 0),
        # for an fp64 arbiter that takes the same branches (bench.py's config-D parity leg)
        rec = getattr(self, "record_branches", None)

        def act(z):
            if rec is not None:
                rec.append(z.detach() > 0)
            return F.leaky_relu(z, slope)
        x = act(ops.linear(x, self.input_layer.weight, self.input_layer.bias))
        for l, b in zip(self.hidden_layers, self.batch_layers):
            x = act(ops.linear(x, l.weight, l.bias))
            x = ops.BNActFn.apply(x, b.weight, b.bias, b, x.shape[0], 1.0)
        return ops.linear(x, self.output_layer.weight, self.output_layer.bias)


class FeedForwardNN(_FFNBase):
    """2d_FPE/DeepONetModules.py:88-125."""

    def __init__(self, input_dimension, output_dimension, network_architecture):
        super().__init__()
        self.retrain = network_architecture["retrain"]
        torch.manual_seed(self.retrain)
        self._build(input_dimension, output_dimension, network_architecture["n_hidden_layers"],
                    network_architecture["neurons"], network_architecture["act_string"],
                    network_architecture["dropout_rate"])
        self.apply(kaiming_init)


class FFN(_FFNBase):
    """Trunk network, 2d_FPE/DeepONetModules.py:155-185."""

    def __init__(self, input_dimension, output_dimension, n_hidden_layers, neurons, act_string,
                 dropout_rate):
        super().__init__()
        self._build(input_dimension, output_dimension, n_hidden_layers, neurons, act_string,
                    dropout_rate)
        self.apply(kaiming_init)


class DeepOnetNoBiasOrg(nn.Module):
    """2d_FPE/DeepONetModules.py:128-151: (branch(u) @ trunk(x)^T + b0) / sqrt(p)."""

    def __init__(self, branch, trunk):
        super().__init__()
        self.branch = branch
        self.trunk = trunk
        self.b0 = torch.nn.Parameter(torch.tensor(0.0), requires_grad=True)
        self.p = self.trunk.output_dimension

    def forward(self, u_, x_):
        weights = self.branch(u_)
        basis = self.trunk(x_)
        return (torch.matmul(weights, basis.T) + self.b0) / self.p ** 0.5
