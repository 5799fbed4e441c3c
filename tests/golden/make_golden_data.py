#!/usr/bin/env python3
"""Capture golden vectors for the data-side rows of SURVEY.md section 8 from the REFERENCE
(build container only; the reference never travels to the GPU box):

  * a14  GPE split-step solver  -- 1d_GPE/datagen_GPE.py:29-115 (solve_GPE_custom, Strang
         order 2 and Yoshida order 4) and generate_and_save_training_data (:120-191)
  * a11  dataset normalisation  -- the Dataset classes defined inside the train scripts:
         2d_FPE/train_fno.py:11-60, 2d_Non_conservative_FPE/train_fno.py:13-60,
         1d_FPE/train_fno.py:8-58, 1d_GPE/train_fno_GPE.py:33-74

    PYTHONDONTWRITEBYTECODE=1 MPLBACKEND=Agg python tests/golden/make_golden_data.py

datagen_GPE.py is main-guarded and imported as a module.  The train scripts are flat
module-level scripts (they read /home/ubuntu/... data at import), so only the one Dataset
class definition is extracted from each with ``ast`` and executed against a tiny synthetic
npz/npy written here.  Output: tests/golden/gpe_*.npz, dataset_*.npz (data only).
"""
from __future__ import annotations

import argparse
import ast
import importlib.util
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def _save(name, arrays):
    path = os.path.join(HERE, f"{name}.npz")
    np.savez_compressed(path, **arrays)
    print(f"  wrote {name}.npz ({os.path.getsize(path) / 1024:.1f} KiB)")


def _class_from_source(path, cname, glb):
    src = open(path).read()
    for node in ast.parse(src).body:
        if isinstance(node, ast.ClassDef) and node.name == cname:
            exec(compile(ast.get_source_segment(src, node), path, "exec"), glb)
            return glb[cname]
    raise KeyError(cname)


def gpe(ref):
    spec = importlib.util.spec_from_file_location("datagen_GPE", os.path.join(ref, "1d_GPE", "datagen_GPE.py"))
    dg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(dg)
    # solver: Nx=64, dt=0.005, t_final=0.5 (Nt=101), both orders; one seeded potential
    rs = np.random.RandomState(7)
    for order in (2, 4):
        x = np.linspace(-10, 10, 64)
        a, b, c, x0 = rs.uniform(0.1, 0.3), rs.uniform(0.5, 2), rs.uniform(0.5, 2), rs.uniform(-3, 3)
        V = a * (x - x0) ** 2 + b * (np.cos(c * (x - x0))) ** 2
        t, rec = dg.solve_GPE_custom(lambda xx: dg.get_initial_condition(2, xx), x, 0.005, 0.5, order, 2.0, 2.0, V)
        _save(f"gpe_solve_o{order}", {"x": x, "V": V, "t": t, "psi": rec, "g": 2.0, "kappa": 2.0,
                                      "dt": 0.005, "t_final": 0.5, "ic": 2})
    # the full training-data recipe at its native length (1001 steps, y = |psi|[::10]) on 3
    # orbits of a 128-point grid; ic 1 and 3 covered by a short solve each
    np.random.seed(42)
    with tempfile.TemporaryDirectory() as td:
        d = dg.generate_and_save_training_data(num_orbits=3, Nx=128, dt=0.005, t_final=5.0, order=2,
                                               num_time_samples=100, save_path=os.path.join(td, "d.npy"))
    _save("gpe_datagen", {"y": d["y"], "g": d["g"], "kappa": d["kappa"], "V": d["V"], "seed": 42,
                          "Nx": 128, "dt": 0.005, "t_final": 5.0})
    out = {}
    for ic in (1, 3):
        x = np.linspace(-10, 10, 32)
        V = 0.2 * x ** 2
        t, rec = dg.solve_GPE_custom(lambda xx: dg.get_initial_condition(ic, xx), x, 0.01, 0.2, 2, 1.0, 0.5, V)
        out[f"psi_ic{ic}"] = rec
        out[f"V_ic{ic}"] = V
    _save("gpe_solve_ic", out)


def datasets(ref):
    import torch
    from torch.utils.data import Dataset
    glb = {"np": np, "torch": torch, "Dataset": Dataset}
    rs = np.random.RandomState(3)
    with tempfile.TemporaryDirectory() as td:
        # 2D FPE: keys trajectories / potential / drag (physical scales ~1e-10, 1e-21, 1e-6)
        p = os.path.join(td, "fpe2d.npz")
        traj = (rs.rand(5, 7, 9, 9) * 1e-10).astype(np.float64)
        pot = rs.standard_normal((5, 9, 9)) * 1e-21
        drag = rs.rand(5, 9, 9) * 1e-6
        np.savez(p, trajectories=traj, potential=pot, drag=drag)
        C = _class_from_source(os.path.join(ref, "2d_FPE", "train_fno.py"), "TrajectoryDataset2D", glb)
        ds = C(p)
        xs, ys = zip(*[ds[i] for i in range(len(ds))])
        _save("dataset_2d_fpe", {"trajectories": traj, "potential": pot, "drag": drag,
                                 "x": torch.stack(xs).numpy(), "y": torch.stack(ys).numpy(),
                                 "traj_mean": ds.trajectories_mean, "traj_std": ds.trajectories_std,
                                 "pot_mean": ds.potential_mean, "pot_std": ds.potential_std,
                                 "drag_mean": ds.drag_mean, "drag_std": ds.drag_std})
        # 2D non-conservative: keys trajectories / F (M, 2, Nx, Ny)
        p = os.path.join(td, "nc.npz")
        F = rs.standard_normal((5, 2, 9, 9)) * 1e-12
        np.savez(p, trajectories=traj, F=F)
        C = _class_from_source(os.path.join(ref, "2d_Non_conservative_FPE", "train_fno.py"),
                               "TrajectoryDataset2D", dict(glb))
        ds = C(p)
        xs, ys = zip(*[ds[i] for i in range(len(ds))])
        _save("dataset_2d_nc", {"trajectories": traj, "F": F, "x": torch.stack(xs).numpy(),
                                "y": torch.stack(ys).numpy(), "F_mean": ds.F_mean, "F_std": ds.F_std})
        # 1D FPE: trajectories (M,T,Nx) / potential (M,Nx) / drag (M,)
        p = os.path.join(td, "fpe1d.npz")
        traj1 = rs.rand(6, 7, 11) * 1e-5
        pot1 = rs.standard_normal((6, 11)) * 1e-20
        drag1 = rs.rand(6) * 1e-5
        np.savez(p, trajectories=traj1, potential=pot1, drag=drag1)
        C = _class_from_source(os.path.join(ref, "1d_FPE", "train_fno.py"), "TrajectoryDataset1D", dict(glb))
        ds = C(p)
        xs, ys = zip(*[ds[i] for i in range(len(ds))])
        _save("dataset_1d_fpe", {"trajectories": traj1, "potential": pot1, "drag": drag1,
                                 "x": torch.stack(xs).numpy(), "y": np.stack(ys)})
        # 1D GPE: pickled dict y / g / kappa / V, divided by global maxima (y, V by max/3)
        p = os.path.join(td, "gpe.npy")
        d = {"y": rs.rand(4, 6, 16), "g": rs.uniform(1, 2.5, 4), "kappa": rs.uniform(1, 2.5, 4),
             "V": rs.rand(4, 16) * 3}
        np.save(p, d, allow_pickle=True)
        C = _class_from_source(os.path.join(ref, "1d_GPE", "train_fno_GPE.py"), "ParameterDataset", dict(glb))
        import contextlib
        import io
        with contextlib.redirect_stdout(io.StringIO()):
            ds = C(p)
        xs, ys = zip(*[ds[i] for i in range(len(ds))])
        _save("dataset_1d_gpe", {"y_raw": d["y"], "g": d["g"], "kappa": d["kappa"], "V_raw": d["V"],
                                 "x": torch.stack(xs).numpy(), "t": torch.stack(ys).numpy(),
                                 "y_max": ds.y_max, "V_max": ds.V_max})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    a = ap.parse_args()
    gpe(a.ref)
    datasets(a.ref)


if __name__ == "__main__":
    main()
