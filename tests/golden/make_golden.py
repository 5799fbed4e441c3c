#!/usr/bin/env python3
"""Capture golden vectors from the REFERENCE implementation (run in the build
container only; the reference never travels to the GPU box).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py [--ref /root/reference]

Each experiment directory of the reference is imported in its own subprocess
(the directories define same-named modules).  The 2D ``NIOModules`` imports
the vendored Transolver (``model/``), which needs ``timm``; only
``timm.models.layers.trunc_normal_`` is referenced and only by Transolver
classes that the hot path never instantiates, so a stub module providing that
one name is registered before the import.  Nothing else is stubbed.

Output: ``tests/golden/<case>.npz`` holding inputs, parameters (or a recipe
seed), outputs, the backward cotangent and gradients; ``layouts.json`` holds
state_dict layouts (names/shapes/dtypes) of the reference models at the
BASELINE configs.  See tests/test_oracle_golden.py for how they are used.
"""
from __future__ import annotations

import argparse
import ast
import json
import os
import subprocess
import sys
import textwrap
import types

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)


def _save(name, arrays):
    import numpy as np
    path = os.path.join(HERE, f"{name}.npz")
    np.savez_compressed(path, **arrays)
    sz = os.path.getsize(path)
    print(f"  wrote {name}.npz ({sz / 1024:.1f} KiB, {len(arrays)} arrays)")


def _capture(name, module, inputs, fwd, extra=None, skip_prefixes=(), seed=0, save_params=True,
             grad_norm_prefixes=()):
    """Run fwd, backprop a seeded cotangent, store everything as numpy."""
    import numpy as np
    import torch
    from recipe import make_array
    for v in inputs.values():
        if isinstance(v, torch.Tensor) and v.is_floating_point():
            v.requires_grad_(True)
    out = fwd()
    cot = torch.from_numpy(make_array(tuple(out.shape), seed, name + ".cot"))
    (out * cot).sum().backward()
    arr = {"out": out.detach().numpy(), "cot": cot.numpy()}
    for k, v in inputs.items():
        if isinstance(v, torch.Tensor):
            arr["in." + k] = v.detach().numpy()
            if v.grad is not None:
                arr["gin." + k] = v.grad.numpy()
        else:
            arr["in." + k] = np.asarray(v)
    for k, v in module.state_dict().items():
        if any(k.startswith(s) for s in skip_prefixes):
            continue
        if save_params:
            arr["p." + k] = v.detach().numpy()
    for k, p in module.named_parameters():
        if p.grad is None:
            continue
        if any(k.startswith(s) for s in grad_norm_prefixes):
            arr["gnorm." + k] = np.array(float(p.grad.double().norm()))
            continue
        if any(k.startswith(s) for s in skip_prefixes):
            continue
        arr["g." + k] = p.grad.numpy()
    for k, v in (extra or {}).items():
        arr[k] = np.asarray(v)
    _save(name, arr)


def _layout(module):
    return [[k, list(v.shape), str(v.dtype).replace("torch.", "")] for k, v in module.state_dict().items()]


def _fn_from_source(path, fname, glb):
    """Extract ONE top-level function definition from a reference file and
    define it in ``glb`` (used for numpy-only metric helpers whose modules
    import heavy/absent dependencies at top level)."""
    src = open(path).read()
    tree = ast.parse(src)
    for node in tree.body:
        if isinstance(node, ast.FunctionDef) and node.name == fname:
            seg = ast.get_source_segment(src, node)
            exec(compile(seg, path, "exec"), glb)
            return glb[fname]
    raise KeyError(fname)


def _install_timm_stub():
    import torch
    timm = types.ModuleType("timm")
    models = types.ModuleType("timm.models")
    layers = types.ModuleType("timm.models.layers")
    layers.trunc_normal_ = torch.nn.init.trunc_normal_
    timm.models = models
    models.layers = layers
    sys.modules.update({"timm": timm, "timm.models": models, "timm.models.layers": layers})


# --------------------------------------------------------------------------- groups
def group_1d_fpe(ref):
    import numpy as np
    import torch
    import FNOModules as FM
    import NIOModules as NM
    layouts = {}

    torch.manual_seed(101)
    m = FM.SpectralConv1d(3, 4, 5)
    x = torch.randn(2, 3, 16)
    _capture("sc1d", m, {"x": x}, lambda: m(x), seed=1)

    torch.manual_seed(102)
    m = FM.SpectralConv1d(2, 3, 9)           # modes = W//2+1: Nyquist bin included
    x = torch.randn(2, 2, 16)
    _capture("sc1d_nyq", m, {"x": x}, lambda: m(x), seed=2)

    torch.manual_seed(103)
    m = FM.FNO1d(5, 6, 3, 2, 2)
    x = torch.randn(3, 20, 2)
    _capture("fno1d", m, {"x": x}, lambda: m(x), seed=3)

    torch.manual_seed(104)
    m = FM.FNO1d(12, 4, 2, 2, 1)             # FNO_input shape at config A (N=64, P=80)
    x = torch.randn(4, 64, 2)
    _capture("fno1d_input64", m, {"x": x}, lambda: m(x), seed=4)

    torch.manual_seed(105)
    m = NM.NIOFP_FNO(3, 6, 5, 2, "cpu")
    x = torch.randn(2, 60, 24)
    grid = torch.linspace(0, 1, 24).unsqueeze(-1)
    np.random.seed(7)
    L = np.random.randint(50, x.shape[1])
    idx = np.random.choice(x.shape[1], L)
    np.random.seed(7)
    m.train()
    _capture("nio1d_fno_train", m, {"x": x, "grid": grid}, lambda: m(x, grid), seed=5,
             extra={"L": L, "idx": idx})
    m.zero_grad()
    m.eval()
    x2 = x.detach().clone()
    grid2 = grid.detach().clone()
    _capture("nio1d_fno_eval", m, {"x": x2, "grid": grid2}, lambda: m(x2, grid2), seed=6)

    layouts["1d_FPE.NIOFP_FNO(3,30,15,2)"] = _layout(NM.NIOFP_FNO(3, 30, 15, 2, "cpu"))

    # metric helper (numpy only; its module imports the external fplanck at top level)
    g = {"np": np}
    f = _fn_from_source(os.path.join(ref, "1d_FPE", "compute_time_error.py"), "time_averaged_L2_error", g)
    rs = np.random.RandomState(11)
    t = np.linspace(0.0, 2.0, 41)
    xg = np.linspace(-1.0, 1.0, 33)
    rho_ref = rs.rand(41, 33) + 0.1
    rho_pred = rho_ref + 0.05 * rs.standard_normal((41, 33))
    import warnings
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        val = f(t, rho_ref, t, rho_pred, xg)
    _save("metric_time_avg_L2_1d", {"t": t, "x": xg, "rho_ref": rho_ref, "rho_pred": rho_pred,
                                    "val": np.array(val)})
    return layouts


def group_1d_gpe(ref):
    import numpy as np
    import torch
    import NIOModules as NM
    layouts = {}
    torch.manual_seed(201)
    m = NM.NIOFP_FNO(3, 5, 8, 1, "cpu")
    x = torch.randn(2, 55, 32)
    grid = torch.linspace(0, 1, 32).unsqueeze(-1)
    np.random.seed(9)
    L = np.random.randint(50, x.shape[1])
    idx = np.random.choice(x.shape[1], L)
    np.random.seed(9)
    m.train()
    _capture("gpe_nio_fno_train", m, {"x": x, "grid": grid}, lambda: m(x, grid), seed=21,
             extra={"L": L, "idx": idx})
    layouts["1d_GPE.NIOFP_FNO(3,20,40,1)"] = _layout(NM.NIOFP_FNO(3, 20, 40, 1, "cpu"))
    return layouts


def group_2d_fpe(ref):
    import numpy as np
    import torch
    _install_timm_stub()
    import FNOModules as FM
    import NIOModules as NM
    layouts = {}

    torch.manual_seed(301)
    m = FM.SpectralConv2d(3, 4, 4, 3)
    x = torch.randn(2, 3, 12, 10)
    _capture("sc2d_a", m, {"x": x}, lambda: m(x), seed=31)

    torch.manual_seed(302)
    m = FM.SpectralConv2d(2, 3, 5, 4)        # H=8 < 2*m1: overlapping corner rows, weights2 wins
    x = torch.randn(2, 2, 8, 8)
    _capture("sc2d_overlap", m, {"x": x}, lambda: m(x), seed=32)

    torch.manual_seed(303)
    m = FM.SpectralConv2d(2, 2, 3, 5)        # W=8, m2=5: Nyquist column included
    x = torch.randn(2, 2, 9, 8)
    _capture("sc2d_nyq", m, {"x": x}, lambda: m(x), seed=33)

    torch.manual_seed(304)
    m = FM.FNO2d(4, 5, 3, 3, 1)              # N=12 -> P=15 (odd)
    x = torch.randn(2, 12, 12, 3)
    _capture("fno2d", m, {"x": x}, lambda: m(x), seed=34)

    torch.manual_seed(305)
    m = FM.FNO2d(12, 4, 2, 3, 1)             # FNO_input at the reference grid 61^2 (P=76)
    x = torch.randn(2, 61, 61, 3)
    _capture("fno2d_input61", m, {"x": x}, lambda: m(x), seed=35)

    torch.manual_seed(306)
    m = FM.FNO2d(32, 4, 2, 4, 1)             # head modes (32) at 61^2, reduced width
    x = torch.randn(1, 61, 61, 4)
    _capture("fno2d_head61", m, {"x": x}, lambda: m(x), seed=36)

    # NIOFP2D_FNO at N=20 (P=25), T=60: train (recorded numpy draw) and eval
    torch.manual_seed(307)
    m = NM.NIOFP2D_FNO(2, 3, 100, 25, 2, 6, 5, 2)
    x = torch.randn(2, 60, 20, 20)
    gx, gy = np.meshgrid(np.linspace(-1, 1, 20, dtype=np.float32),
                         np.linspace(-1, 1, 20, dtype=np.float32), indexing="ij")
    grid = torch.tensor(np.stack([gx, gy], axis=2))
    np.random.seed(13)
    L = np.random.randint(50, x.shape[1])
    idx = np.random.choice(x.shape[1], L)
    np.random.seed(13)
    m.train()
    _capture("nio2d_fno_train", m, {"x": x, "grid": grid}, lambda: m(x, grid), seed=37,
             extra={"L": L, "idx": idx}, skip_prefixes=("branch.",))
    m.zero_grad()
    m.eval()
    x2 = x.detach().clone()
    grid2 = grid.detach().clone()
    _capture("nio2d_fno_eval", m, {"x": x2, "grid": grid2}, lambda: m(x2, grid2), seed=38,
             skip_prefixes=("branch.",))

    # two reference Adam steps on a small FNO2d (lr of 2d_FPE/train_fno.py:117)
    torch.manual_seed(308)
    m = FM.FNO2d(4, 3, 2, 3, 1)
    opt = torch.optim.Adam(m.parameters(), lr=0.0005)
    arr = {}
    for k, v in m.state_dict().items():
        arr["p0." + k] = v.detach().clone().numpy()
    for step in (1, 2):
        xs = torch.randn(2, 10, 10, 3)
        ys = torch.randn(2, 10, 10, 1)
        opt.zero_grad()
        loss = torch.nn.MSELoss()(m(xs), ys)
        loss.backward()
        for k, p in m.named_parameters():
            arr[f"g{step}." + k] = p.grad.detach().clone().numpy()
        opt.step()
        for k, v in m.state_dict().items():
            arr[f"p{step}." + k] = v.detach().clone().numpy()
    _save("adam_fno2d", arr)

    # train-loop relative-L2 quirk (2d_FPE/train_fno.py:160-163), evaluated from its source text
    src = open(os.path.join(ref, "2d_FPE", "train_fno.py")).read().splitlines()
    start = next(i for i, s in enumerate(src) if s.strip().startswith("errors_drift ="))
    stmt = textwrap.dedent("\n".join(src[start:start + 4]))
    predictions = torch.randn(3, 9, 9, 2)
    outputs = torch.randn(3, 9, 9, 2)
    ns = {"torch": torch, "predictions": predictions, "outputs": outputs}
    exec(stmt, ns)
    _save("metric_train_rel_l2", {"pred": predictions.numpy(), "out": outputs.numpy(),
                                  "e_drift": ns["errors_drift"].numpy(),
                                  "e_diffusion": ns["errors_diffusion"].numpy()})

    g = {"np": np}
    f = _fn_from_source(os.path.join(ref, "2d_FPE", "eval_fno.py"), "rel_l2", g)
    rs = np.random.RandomState(12)
    a = rs.standard_normal((61, 61)).astype(np.float32)
    b = rs.standard_normal((61, 61)).astype(np.float32)
    _save("metric_rel_l2", {"a": a, "b": b, "val": np.array(f(a, b))})

    layouts["2d_FPE.NIOFP2D_FNO(2,3,100,25,3,12,32,2)"] = _layout(NM.NIOFP2D_FNO(2, 3, 100, 25, 3, 12, 32, 2))
    layouts["2d_FPE.NIOFP2D(2,3,100,25,3,12,32,2)"] = _layout(NM.NIOFP2D(2, 3, 100, 25, 3, 12, 32, 2))
    return layouts


def group_2d_nc(ref):
    import numpy as np
    import torch
    _install_timm_stub()
    import NIOModules as NM
    from recipe import make_array, make_state
    layouts = {}

    # NIO branch/trunk (config D's model) at the reference grid 80^2 with recipe parameters
    m = NM.NIOFP2D(2, 3, 100, 25, 2, 6, 8, 2)
    shapes = [(k, tuple(v.shape)) for k, v in m.state_dict().items()]
    st = make_state(shapes, seed=401)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in st.items()})
    x = torch.from_numpy(make_array((1, 51, 80, 80), 401, "nio2d_nc.x"))
    gx, gy = np.meshgrid(np.linspace(-1, 1, 80, dtype=np.float32),
                         np.linspace(-1, 1, 80, dtype=np.float32), indexing="ij")
    grid = torch.tensor(np.stack([gx, gy], axis=2))
    np.random.seed(17)
    L = np.random.randint(50, x.shape[1])
    idx = np.random.choice(x.shape[1], L)
    np.random.seed(17)
    m.train()
    _capture("nio2d_nc_train", m, {"x": x, "grid": grid}, lambda: m(x, grid), seed=41,
             extra={"L": L, "idx": idx, "recipe_seed": 401,
                    "layout_json": json.dumps([[k, list(s)] for k, s in shapes])}, save_params=False,
             grad_norm_prefixes=("branch.", "deeponet.branch."))

    torch.manual_seed(402)
    m = NM.NIOFP2D_FNO(2, 3, 100, 25, 2, 6, 5, 2)
    xs = torch.randn(1, 55, 20, 20)
    gx, gy = np.meshgrid(np.linspace(-1, 1, 20, dtype=np.float32),
                         np.linspace(-1, 1, 20, dtype=np.float32), indexing="ij")
    grid20 = torch.tensor(np.stack([gx, gy], axis=2))
    m.eval()
    _capture("nc_nio2d_fno_eval", m, {"x": xs, "grid": grid20}, lambda: m(xs, grid20), seed=42,
             skip_prefixes=("branch.",))

    g = {"np": np}
    f = _fn_from_source(os.path.join(ref, "2d_Non_conservative_FPE", "compute_time_error.py"),
                        "time_averaged_relative_l2", g)
    rs = np.random.RandomState(14)
    pref = rs.rand(25, 16, 16) + 0.1
    ppred = pref + 0.03 * rs.standard_normal((25, 16, 16))
    _save("metric_time_avg_rel_l2_2d", {"pt_ref": pref, "pt_pred": ppred, "val": np.array(f(ppred, pref))})

    layouts["2d_NC.NIOFP2D_FNO(2,3,100,25,3,12,32,2)"] = _layout(NM.NIOFP2D_FNO(2, 3, 100, 25, 3, 12, 32, 2))
    layouts["2d_NC.NIOFP2D(2,3,100,25,3,12,32,2)"] = _layout(NM.NIOFP2D(2, 3, 100, 25, 3, 12, 32, 2))
    return layouts


GROUPS = {"1d_FPE": group_1d_fpe, "1d_GPE": group_1d_gpe, "2d_FPE": group_2d_fpe,
          "2d_Non_conservative_FPE": group_2d_nc}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--group", default=None)
    a = ap.parse_args()
    if a.group:
        sys.path.insert(0, os.path.join(a.ref, a.group))
        import torch
        torch.set_num_threads(8)
        lay = GROUPS[a.group](a.ref)
        with open(os.path.join(HERE, f"_layouts_{a.group}.json"), "w") as f:
            json.dump(lay, f)
        return
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1")
    layouts = {}
    for gname in GROUPS:
        print(f"[group {gname}]")
        subprocess.run([sys.executable, __file__, "--ref", a.ref, "--group", gname], check=True,
                       cwd="/tmp", env=env)
        p = os.path.join(HERE, f"_layouts_{gname}.json")
        layouts.update(json.load(open(p)))
        os.remove(p)
    with open(os.path.join(HERE, "layouts.json"), "w") as f:
        json.dump(layouts, f, indent=0)
    print("wrote layouts.json")


if __name__ == "__main__":
    main()
