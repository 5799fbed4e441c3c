#!/usr/bin/env python3
"""Capture golden vectors of the 1D NIO models (DeepONet branch/trunk + FNO1d heads) from the
REFERENCE (build container only; the reference never travels to the GPU box).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_nio1d.py [--ref /root/reference]

  nio1d_train      1d_FPE NIOFP (1d_FPE/NIOModules.py:15-84), N = 80 (the grid its Encoder
                   collapses to one 256-feature: 1d_FPE/Baselines.py:254-287), train mode
                   (train-mode BatchNorm, recorded numpy bag draw)
  gpe_nio1d_train  1d_GPE NIOFP_schrodinger (1d_GPE/NIOModules.py:160-223), N = 128, train mode

Same conventions as make_golden.py (one subprocess per experiment directory, seeded
cotangents) and make_golden_unet.py (parameters from recipe.py loaded INTO the reference
module, so the 1.3M-parameter encoders need not be stored; the conv biases ahead of the
train-mode BatchNorms, whose gradient is exactly zero, are kept as norms; gradients of more
than 32k entries as their norm plus their leading 8192 entries).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)


def _capture(name, m, x, grid, np_seed, cot_seed, recipe_seed):
    import numpy as np
    import torch
    from make_golden import _save
    from recipe import make_array, make_state
    named = [(k, tuple(v.shape)) for k, v in m.state_dict().items()]
    cplx = [k for k, v in m.state_dict().items() if v.is_complex()]
    st = make_state(named, recipe_seed, complex_names=cplx)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in st.items()})
    m.train()
    np.random.seed(np_seed)
    L = np.random.randint(50, x.shape[1])
    idx = np.random.choice(x.shape[1], L)
    np.random.seed(np_seed)
    x.requires_grad_(True)
    out = m(x, grid)
    cot = torch.from_numpy(make_array(tuple(out.shape), cot_seed, name + ".cot"))
    (out * cot).sum().backward()
    arr = {"out": out.detach().numpy(), "cot": cot.numpy(), "in.x": x.detach().numpy(),
           "gin.x": x.grad.numpy(), "in.grid": grid.numpy(), "L": np.array(L), "idx": idx,
           "recipe_seed": np.array(recipe_seed),
           "layout_json": json.dumps([[k, list(s)] for k, s in named]),
           "complex_json": json.dumps(cplx)}
    for k, p in m.named_parameters():
        if p.grad is None:
            continue
        # branch / deeponet.branch are one module registered twice: keep the first name only
        if k.startswith("deeponet."):
            continue
        if k.startswith("branch.") and k.endswith("layers.0.bias"):
            arr["gnorm." + k] = np.array(float(p.grad.double().norm()))
        elif p.numel() > 1 << 15:
            # the large encoder convolutions: norm + the leading 8192 entries (whole output
            # channels), which keeps the fixture small
            arr["gnorm." + k] = np.array(float(p.grad.double().norm()))
            arr["gpre." + k] = p.grad.reshape(-1)[:8192].numpy()
        else:
            arr["g." + k] = p.grad.numpy()
    _save(name, arr)


def group_1d_fpe(ref):
    import torch
    import NIOModules as NM
    from recipe import make_array
    m = NM.NIOFP(1, 3, 100, 25, 2, 6, 8, 2, "cpu")
    x = torch.from_numpy(make_array((2, 60, 80), 501, "nio1d.x"))
    grid = torch.linspace(0, 1, 80).unsqueeze(-1)
    _capture("nio1d_train", m, x, grid, np_seed=19, cot_seed=51, recipe_seed=501)


def group_1d_gpe(ref):
    import torch
    import NIOModules as NM
    from recipe import make_array
    m = NM.NIOFP_schrodinger(1, 3, 100, 25, 2, 6, 8, 1, "cpu")
    x = torch.from_numpy(make_array((2, 55, 128), 601, "gpe_nio1d.x"))
    grid = torch.linspace(0, 1, 128).unsqueeze(-1)
    _capture("gpe_nio1d_train", m, x, grid, np_seed=23, cot_seed=61, recipe_seed=601)


GROUPS = {"1d_FPE": group_1d_fpe, "1d_GPE": group_1d_gpe}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--group", default=None)
    a = ap.parse_args()
    if a.group:
        sys.path.insert(0, os.path.join(a.ref, a.group))
        import torch
        torch.set_num_threads(8)
        GROUPS[a.group](a.ref)
        return
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1")
    for gname in GROUPS:
        print(f"[group {gname}]")
        subprocess.run([sys.executable, __file__, "--ref", a.ref, "--group", gname], check=True,
                       cwd="/tmp", env=env)


if __name__ == "__main__":
    main()
