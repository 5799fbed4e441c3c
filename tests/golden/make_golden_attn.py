#!/usr/bin/env python3
"""Capture the NIOFP2D_FNO_attn golden vectors from the REFERENCE (build container only;
the reference never travels to the GPU box).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_attn.py [--ref /root/reference]

Same conventions as make_golden.py (whose helpers it reuses): one subprocess per
experiment directory, the ``timm`` stub for the Transolver import, seeded cotangents.
Writes nio2d_fno_attn_train.npz, nio2d_fno_attn_eval.npz, nc_nio2d_fno_attn_train.npz and
merges the attention models' state_dict layouts into layouts.json.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)


def _grid(n):
    import numpy as np
    import torch
    gx, gy = np.meshgrid(np.linspace(-1, 1, n, dtype=np.float32),
                         np.linspace(-1, 1, n, dtype=np.float32), indexing="ij")
    return torch.tensor(np.stack([gx, gy], axis=2))


def group(exp):
    import numpy as np
    import torch
    from make_golden import _capture, _install_timm_stub, _layout
    _install_timm_stub()
    import NIOModules as NM
    tag = "nio2d" if exp == "2d_FPE" else "nc_nio2d"
    torch.manual_seed(401 if exp == "2d_FPE" else 402)
    m = NM.NIOFP2D_FNO_attn(2, 3, 100, 25, 2, 6, 5, 2, 20, 20)
    x = torch.randn(2, 60, 20, 20)
    grid = _grid(20)
    np.random.seed(19)
    L = np.random.randint(50, x.shape[1])
    idx = np.random.choice(x.shape[1], L, replace=False)   # 2d_FPE/NIOModules.py:344-345
    np.random.seed(19)
    m.train()
    _capture(f"{tag}_fno_attn_train", m, {"x": x, "grid": grid}, lambda: m(x, grid), seed=41,
             extra={"L": L, "idx": idx})
    if exp == "2d_FPE":
        m.zero_grad()
        m.eval()
        x2, g2 = x.detach().clone(), grid.detach().clone()
        _capture(f"{tag}_fno_attn_eval", m, {"x": x2, "grid": g2}, lambda: m(x2, g2), seed=42)
    key = f"{'2d' if exp == '2d_FPE' else '2d_NC'}.NIOFP2D_FNO_attn(2,3,100,25,3,12,32,2,128,128)"
    return {key: _layout(NM.NIOFP2D_FNO_attn(2, 3, 100, 25, 3, 12, 32, 2, 128, 128))}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--group", default=None)
    a = ap.parse_args()
    if a.group:
        sys.path.insert(0, os.path.join(a.ref, a.group))
        import torch
        torch.set_num_threads(8)
        with open(os.path.join(HERE, f"_layouts_attn_{a.group}.json"), "w") as f:
            json.dump(group(a.group), f)
        return
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1")
    path = os.path.join(HERE, "layouts.json")
    layouts = json.load(open(path))
    for g in ("2d_FPE", "2d_Non_conservative_FPE"):
        subprocess.run([sys.executable, __file__, "--ref", a.ref, "--group", g], check=True,
                       cwd="/tmp", env=env)
        p = os.path.join(HERE, f"_layouts_attn_{g}.json")
        layouts.update(json.load(open(p)))
        os.remove(p)
    with open(path, "w") as f:
        json.dump(layouts, f, indent=0)
    print("updated layouts.json")


if __name__ == "__main__":
    main()
