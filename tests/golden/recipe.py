"""Deterministic, numpy-only parameter recipe shared by the golden generator and
the tests.

Large reference models (the NIO Encoder2D branch has ~11M parameters) cannot be
committed as fixtures, so their golden vectors are captured by loading
recipe-generated parameters INTO the reference module; the test regenerates
the very same values from (names, shapes, seed).  Data only -- no reference code.
"""
from __future__ import annotations

import numpy as np


def _seed_of(seed: int, name: str) -> int:
    h = 2166136261
    for ch in name.encode():
        h = ((h ^ ch) * 16777619) & 0xFFFFFFFF
    return (seed * 1000003 + h) & 0x7FFFFFFF


def make_param(name: str, shape, seed: int, complex_: bool = False) -> np.ndarray:
    rs = np.random.RandomState(_seed_of(seed, name))
    shape = tuple(int(s) for s in shape)
    n = int(np.prod(shape)) if shape else 1
    if "spectral_list" in name:
        ci, co = shape[0], shape[1]
        scale = 1.0 / (ci * co)
        if complex_:
            v = scale * (rs.rand(*shape) + 1j * rs.rand(*shape))
            return v.astype(np.complex64)
        return (scale * rs.rand(*shape)).astype(np.float32)
    if name.endswith("running_var"):
        return np.ones(shape, np.float32)
    if name.endswith("running_mean"):
        return np.zeros(shape, np.float32)
    if name.endswith("num_batches_tracked"):
        return np.zeros(shape, np.int64)
    if len(shape) <= 1:
        is_bn = ".layers.1." in name or "batch_layers" in name or any("norm" in c for c in name.split(".")[:-1])
        if is_bn and name.endswith("weight"):
            return (1.0 + 0.1 * rs.uniform(-1, 1, shape)).astype(np.float32)
        return (0.1 * rs.uniform(-1, 1, shape)).astype(np.float32)
    fan_in = max(1, n // shape[0])
    bound = 1.0 / np.sqrt(fan_in)
    return rs.uniform(-bound, bound, shape).astype(np.float32)


def make_state(named_shapes, seed: int, complex_names=()):
    out = {}
    for name, shape in named_shapes:
        # NIOFP2D registers branch/trunk twice (self.branch and self.deeponet.branch share one
        # module): alias the duplicated keys to one value
        key = name[len("deeponet."):] if name.startswith(("deeponet.branch.", "deeponet.trunk.")) else name
        out[name] = np.asarray(make_param(key, shape, seed, complex_=name in complex_names))
    return out


def make_array(shape, seed: int, tag: str, dist: str = "normal") -> np.ndarray:
    rs = np.random.RandomState(_seed_of(seed, tag))
    if dist == "normal":
        return rs.standard_normal(shape).astype(np.float32)
    return rs.uniform(-1, 1, shape).astype(np.float32)
