#!/usr/bin/env python3
"""Capture the PermInvUNet_attn ("BlinDNO") golden vectors from the REFERENCE (build container
only; the reference never travels to the GPU box).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_unet.py [--ref /root/reference]

Same conventions as make_golden.py: one subprocess per experiment directory, the ``timm``
stub for the Transolver import, seeded cotangents.  Parameters come from recipe.py (loaded
INTO the reference module) so the two 1.8M-parameter FNO heads need not be stored; the heads'
spectral-weight gradients are stored as norms (the spectral kernels have their own goldens).
Writes unet2d_train.npz, unet2d_eval.npz, nc_unet2d_train.npz, unet1d_bag_train.npz,
unet1d_all.npz and merges the models' state_dict layouts into layouts.json.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

SPEC = ("fno_drift.spectral_list", "fno_diffusion.spectral_list", "fno_Fx.spectral_list", "fno_Fy.spectral_list")


def _load_recipe(m, seed):
    """Load recipe.py parameters into the reference module; returns the fixture fields that let a
    test regenerate them (layout + seed + complex names)."""
    import numpy as np
    import torch
    from recipe import make_state
    named = [(k, tuple(v.shape)) for k, v in m.state_dict().items()]
    cplx = [k for k, v in m.state_dict().items() if v.is_complex()]
    st = make_state(named, seed, complex_names=cplx)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in st.items()})
    return {"layout_json": json.dumps([[k, list(s)] for k, s in named]), "recipe_seed": seed,
            "complex_json": json.dumps(cplx)}


def _init_fingerprint(tag, ctor, seed):
    """Seeded construction -> per-parameter (sum, sum of squares, first four values) in float64:
    pins the creation order and init of the drop-in classes without storing 3.5M weights."""
    import numpy as np
    import torch
    torch.manual_seed(seed)
    m = ctor()
    out = {}
    for k, v in m.state_dict().items():
        a = v.detach().double().reshape(-1).numpy() if not v.is_complex() else \
            torch.view_as_real(v.detach()).double().reshape(-1).numpy()
        head = np.zeros(4)
        head[:min(4, a.size)] = a[:4]
        out[f"{tag}|{k}"] = np.concatenate([[a.sum(), (a * a).sum()], head])
    return out


def group(exp):
    import numpy as np
    import torch
    from make_golden import _capture, _install_timm_stub, _layout
    from recipe import make_array
    _install_timm_stub()
    import NIOModules as NM
    out = {}
    if exp in ("2d_FPE", "2d_Non_conservative_FPE"):
        tag = "unet2d" if exp == "2d_FPE" else "nc_unet2d"
        # 2d_FPE: the reference's depth 4 at 52x52 (output_padding 0 and 1; the modes-32 heads need N >= 50);
        # NC: base_ch 2, depth 3 at 50x50
        base, depth, n, seed = (1, 4, 52, 501) if exp == "2d_FPE" else (2, 3, 50, 502)
        m = NM.PermInvUNet_attn(in_ch=1, out_ch=2, base_ch=base, depth=depth, input_size=(n, n))
        rec = _load_recipe(m, seed)
        x = torch.from_numpy(make_array((2, 60, n, n), seed, tag + ".x"))
        np.random.seed(23)
        L = np.random.randint(50, x.shape[1])
        idx = np.random.choice(x.shape[1], L)             # 2d_FPE/NIOModules.py:1145-1148
        np.random.seed(23)
        m.train()
        _capture(f"{tag}_train", m, {"x": x}, lambda: m(x), seed=seed, save_params=False,
                 grad_norm_prefixes=SPEC,
                 extra={"L": L, "idx": idx, "base_ch": base, "depth": depth, **rec})
        # skip BatchNorm running statistics after the train-mode forward (momentum 0.1)
        run = {"run_mean": np.concatenate([m.skip_norms[i].running_mean.numpy() for i in range(depth + 1)]),
               "run_var": np.concatenate([m.skip_norms[i].running_var.numpy() for i in range(depth + 1)])}
        if exp == "2d_FPE":
            m.zero_grad()
            m.eval()
            x2 = x[:, :12].detach().clone()
            _capture(f"{tag}_eval", m, {"x": x2}, lambda: m(x2), seed=seed + 10, save_params=False,
                     grad_norm_prefixes=SPEC, extra={"base_ch": base, "depth": depth, **run, **rec})
        else:
            np.savez(os.path.join(HERE, f"{tag}_train_run.npz"), **run)
        fp = _init_fingerprint(tag, lambda: NM.PermInvUNet_attn(in_ch=1, out_ch=2, base_ch=1, depth=4,
                                                                input_size=(61, 61)), 531)
        np.savez(os.path.join(HERE, f"{tag}_init.npz"), **fp)
        key = f"{'2d' if exp == '2d_FPE' else '2d_NC'}.PermInvUNet_attn(1,2,1,4,(61,61))"
        out[key] = _layout(NM.PermInvUNet_attn(in_ch=1, out_ch=2, base_ch=1, depth=4, input_size=(61, 61)))
    elif exp == "1d_GPE":
        # the one-head copies: layouts and seeded-init fingerprints
        fp = _init_fingerprint("unet1d_gpe_bag", lambda: NM.PermInvUNet_attn1D_bag(
            in_ch=1, out_ch=2, base_ch=1, depth=4, input_size=128, device="cpu"), 534)
        fp.update(_init_fingerprint("unet1d_gpe", lambda: NM.PermInvUNet_attn1D_bag_GPE(
            in_ch=1, out_ch=2, base_ch=1, depth=4, input_size=128, device="cpu", width=20, modes=40), 535))
        np.savez(os.path.join(HERE, "unet1d_gpe_init.npz"), **fp)
        out["1d_GPE.PermInvUNet_attn1D_bag(1,2,1,4,128)"] = _layout(
            NM.PermInvUNet_attn1D_bag(in_ch=1, out_ch=2, base_ch=1, depth=4, input_size=128, device="cpu"))
        out["1d_GPE.PermInvUNet_attn1D_bag_GPE(1,2,1,4,128,20,40)"] = _layout(
            NM.PermInvUNet_attn1D_bag_GPE(in_ch=1, out_ch=2, base_ch=1, depth=4, input_size=128, device="cpu",
                                          width=20, modes=40))
    else:  # 1d_FPE
        m = NM.PermInvUNet_attn1D_bag(in_ch=1, out_ch=2, base_ch=1, depth=5, input_size=40, device="cpu")
        rec = _load_recipe(m, 511)
        x = torch.from_numpy(make_array((2, 60, 40), 511, "unet1d_bag.x"))
        np.random.seed(29)
        L = np.random.randint(50, x.shape[1])
        idx = np.random.choice(x.shape[1], L)             # 1d_FPE/NIOModules.py:398-402
        np.random.seed(29)
        m.train()
        _capture("unet1d_bag_train", m, {"x": x}, lambda: m(x), seed=511, save_params=False,
                 extra={"L": L, "idx": idx, "base_ch": 1, "depth": 5, **rec})
        m = NM.PermInvUNet_attn1D(in_ch=1, out_ch=2, base_ch=2, depth=3, input_size=24, device="cpu")
        rec = _load_recipe(m, 512)
        x = torch.from_numpy(make_array((2, 12, 24), 512, "unet1d_all.x"))
        m.train()
        _capture("unet1d_all", m, {"x": x}, lambda: m(x), seed=512, save_params=False,
                 extra={"base_ch": 2, "depth": 3, **rec})
        fp = _init_fingerprint("unet1d_bag", lambda: NM.PermInvUNet_attn1D_bag(
            in_ch=1, out_ch=2, base_ch=1, depth=5, input_size=80, device="cpu"), 532)
        fp.update(_init_fingerprint("unet1d", lambda: NM.PermInvUNet_attn1D(
            in_ch=1, out_ch=2, base_ch=1, depth=6, input_size=80, device="cpu"), 533))
        np.savez(os.path.join(HERE, "unet1d_init.npz"), **fp)
        out["1d.PermInvUNet_attn1D_bag(1,2,1,5,80)"] = _layout(
            NM.PermInvUNet_attn1D_bag(in_ch=1, out_ch=2, base_ch=1, depth=5, input_size=80, device="cpu"))
        out["1d.PermInvUNet_attn1D(1,2,1,6,80)"] = _layout(
            NM.PermInvUNet_attn1D(in_ch=1, out_ch=2, base_ch=1, depth=6, input_size=80, device="cpu"))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--group", default=None)
    a = ap.parse_args()
    if a.group:
        sys.path.insert(0, os.path.join(a.ref, a.group))
        import torch
        torch.set_num_threads(8)
        with open(os.path.join(HERE, f"_layouts_unet_{a.group}.json"), "w") as f:
            json.dump(group(a.group), f)
        return
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1")
    path = os.path.join(HERE, "layouts.json")
    layouts = json.load(open(path))
    for g in ("2d_FPE", "2d_Non_conservative_FPE", "1d_FPE", "1d_GPE"):
        subprocess.run([sys.executable, __file__, "--ref", a.ref, "--group", g], check=True,
                       cwd="/tmp", env=env)
        p = os.path.join(HERE, f"_layouts_unet_{g}.json")
        layouts.update(json.load(open(p)))
        os.remove(p)
    with open(path, "w") as f:
        json.dump(layouts, f, indent=0)
    print("updated layouts.json")


if __name__ == "__main__":
    main()
