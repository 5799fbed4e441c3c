"""Density-trajectory errors of predicted fields: 2d_Non_conservative_FPE/
compute_time_error.py:361-510 (``compute_time_error``, FPE forces), 1d_FPE/
compute_time_error.py:215-420 (``compute_time_error_1d``, potential + drag) and 1d_GPE/
compute_time_error_GPE.py:208-330 (``compute_time_error_gpe``, GPE potentials), each as one
batched pipeline.

Per test index the reference normalises the bag with the train statistics, predicts (Fx, Fy)
with each model, de-normalises, propagates a Gaussian density (centre (-150, -150) nm, width
30 nm) under the true and under each predicted force with fplanck (``propagate_density_with_
force``, :300-319), and writes ``[index, model, rel_l2_Fx, rel_l2_Fy, ErrL2_density]`` to
metrics_all.csv, ErrL2 being ``time_averaged_relative_l2`` (:321-333).

Here every model's forward runs batched on the HIP path (blindno.evaluate.predict) and ALL
density propagations -- the reference one and one per model, for every index -- go into ONE
``blindno_fp_propagate`` launch (one workgroup per trajectory).  The propagator restates the
absent fplanck (blindno.fpe): parity UNPINNED.  The figures are out of scope.
"""
from __future__ import annotations

import csv
import os
from typing import Dict, Iterable, List, Optional

import numpy as np
import torch

from . import evaluate, fpe

NM = 1e-9
KIND = "2d_Non_conservative_FPE"


def time_averaged_relative_l2(pt_pred: np.ndarray, pt_ref: np.ndarray, eps: float = 1e-12) -> float:
    """compute_time_error.py:321-333: mean over t of ||P_pred[t] - P_ref[t]|| / (||P_ref[t]|| + eps)."""
    a = pt_pred.reshape(pt_pred.shape[0], -1)
    b = pt_ref.reshape(pt_ref.shape[0], -1)
    return float(np.mean(np.linalg.norm(a - b, axis=1) / (np.linalg.norm(b, axis=1) + eps)))


def build_fokker_planck(force, temperature=300.0, viscosity=8e-4, radius_nm=50.0, extent_nm=800.0,
                        resolution_nm=10.0):
    """compute_time_error.py:266-286."""
    drag = 6 * np.pi * viscosity * radius_nm * NM
    return fpe.fokker_planck(temperature=temperature, drag=drag, extent=[extent_nm * NM, extent_nm * NM],
                             resolution=resolution_nm * NM, boundary=fpe.boundary.reflecting, force=force)


def force_from_array(grid, Fx, Fy):
    """compute_time_error.py:288-298."""
    fx, fy = fpe.potential_from_data(grid, Fx), fpe.potential_from_data(grid, Fy)
    return lambda x, y: np.array([fx(x, y), fy(x, y)])


def compute_time_error(models: Dict[str, torch.nn.Module], train, test, indices: Iterable[int],
                       outdir: Optional[str] = None, nsteps: int = 500, dt: float = 10e-3,
                       batch: int = 8, device="cuda", **phys) -> List[list]:
    """Rows [index, model, rel_l2_Fx, rel_l2_Fy, ErrL2_density] in the reference's order (per
    index: the models in the given order); with ``outdir`` appended to metrics_all.csv."""
    stats = evaluate.compute_train_stats(KIND, train)
    data = np.load(test) if isinstance(test, str) else test
    traj = np.asarray(data["trajectories"])
    idx = [i for i in indices if 0 <= i < traj.shape[0]]
    if not idx:
        return []
    nx, ny = traj.shape[2], traj.shape[3]
    x = torch.tensor(np.stack([evaluate.normalize_input(np.array(traj[i], dtype=np.float32), stats)
                               for i in idx]), dtype=torch.float32, device=device)
    grid_t = evaluate.grid2d(nx, ny, device)
    preds = {name: evaluate.predict(m, x, grid_t, batch).cpu().numpy() for name, m in models.items()}
    grid = build_fokker_planck(lambda xx, yy: np.array([0 * xx, 0 * yy]), **phys).grid
    pdf = fpe.gaussian_pdf(center=(-150 * NM, -150 * NM), width=30 * NM)
    sims, fields = [], []
    for k, i in enumerate(idx):
        F = np.array(data["F"][i], dtype=np.float32)
        sims.append(build_fokker_planck(force_from_array(grid, F[0], F[1]), **phys))
        for name in models:
            pa, pb = evaluate.denormalize(KIND, preds[name][k], stats)
            fields.append((i, name, evaluate.rel_l2(pa, F[0]), evaluate.rel_l2(pb, F[1])))
            sims.append(build_fokker_planck(force_from_array(grid, pa, pb), **phys))
    res = fpe.propagate_many(sims, [pdf] * len(sims), dt, Nsteps=nsteps, device=device)
    rows = []
    per = 1 + len(models)
    for k in range(len(idx)):
        ref = res[k * per][1]
        for j in range(len(models)):
            i, name, rfx, rfy = fields[k * len(models) + j]
            rows.append([i, name, rfx, rfy, time_averaged_relative_l2(res[k * per + 1 + j][1], ref)])
    if outdir is not None:
        os.makedirs(outdir, exist_ok=True)
        path = os.path.join(outdir, "metrics_all.csv")
        header = not os.path.exists(path)
        with open(path, "a", newline="") as f:
            w = csv.writer(f)
            if header:
                w.writerow(["index", "model", "rel_l2_Fx", "rel_l2_Fy", "ErrL2_density"])
            w.writerows(rows)
    return rows


# ------------------------------------------------------------------------------- 1D GPE
def compute_time_error_gpe(models: Dict[str, torch.nn.Module], train, test, indices: Iterable[int],
                           outdir: Optional[str] = None, order: int = 2, dt: float = 0.005,
                           t_final: float = 5.0, init_ic: int = 2, batch: int = 32,
                           device="cuda") -> Dict[str, np.ndarray]:
    """1d_GPE/compute_time_error_GPE.py:208-330: per test index, V predicted by each model
    (de-normalised with the train V_max), |psi| propagated from initial condition ``init_ic`` on
    x = linspace(-10, 10, Nx) under the true V and under each prediction (true g, kappa), and
    time_averaged_L2_error of the densities.  All trajectories -- reference and every model's,
    for every index -- run in ONE blindno_gpe_solve launch; the errors' spatial integrals run on
    the GPU (blindno.gpe.time_averaged_L2_error).  Returns {model: errors in index order}; with
    ``outdir`` writes the reference's per-sample dicts <outdir>/<model>/sample_<idx>_V_and_err.npy
    and ErrL2_relative_<model>_Nsamples_<n>.npy."""
    from . import gpe
    sc = evaluate.compute_train_scalers_gpe(train)
    tn = evaluate.normalize_gpe(test, sc)
    y = np.asarray(tn["y"])
    idx = [int(i) for i in indices if 0 <= int(i) < y.shape[0]]
    if not idx:
        return {name: np.zeros(0) for name in models}
    nx = y.shape[2]
    xin = torch.tensor(np.stack([y[i] for i in idx]), dtype=torch.float32, device=device)
    grid_n = torch.linspace(0.0, 1.0, nx, device=device).unsqueeze(-1)
    preds = {}
    for name, m in models.items():
        p = evaluate.predict(m, xin, grid_n, batch).cpu().numpy()
        preds[name] = (p[..., 0] if p.ndim == 3 else p) * sc["V_max"]
    x = np.linspace(-10, 10, nx)
    V, g, kappa = [], [], []
    for k, i in enumerate(idx):
        gi = float(np.atleast_1d(test["g"][i])[0])
        ki = float(np.atleast_1d(test["kappa"][i])[0])
        for Vi in [tn["V"][i] * sc["V_max"]] + [preds[name][k] for name in models]:
            V.append(Vi)
            g.append(gi)
            kappa.append(ki)
    r = gpe.solve_batch(gpe.initial_condition(init_ic, x), x, dt, t_final, order, np.array(g),
                        np.array(kappa), np.array(V), rec_every=1, device=device)
    t, rho = r["t"], r["abs"]
    per = 1 + len(models)
    errs = {name: [] for name in models}
    for k, i in enumerate(idx):
        ref = rho[k * per]
        for j, name in enumerate(models):
            e = gpe.time_averaged_L2_error(t, ref, t, rho[k * per + 1 + j], x)
            errs[name].append(e)
            if outdir is not None:
                d = os.path.join(outdir, name)
                os.makedirs(d, exist_ok=True)
                np.save(os.path.join(d, f"sample_{i}_V_and_err.npy"),
                        {"x": x, "true_V": V[k * per], "pred_V": V[k * per + 1 + j], "g": g[k * per],
                         "kappa": kappa[k * per], "Err_L2_rel": e})
    out = {name: np.array(v, dtype=float) for name, v in errs.items()}
    if outdir is not None:
        for name, arr in out.items():
            np.save(os.path.join(outdir, f"ErrL2_relative_{name}_Nsamples_{len(idx)}.npy"), arr)
    return out


# ------------------------------------------------------------------------------- 1D FPE
def compute_time_error_1d(models: Dict[str, torch.nn.Module], train, test, indices: Iterable[int],
                          outdir: Optional[str] = None, nsteps: int = 400, dt: float = 2e-3,
                          batch: int = 32, device="cuda", temperature: float = 300.0,
                          extent_nm: float = 800.0, resolution_nm: float = 10.0,
                          init_width_nm: float = 50.0) -> Dict[str, np.ndarray]:
    """1d_FPE/compute_time_error.py:215-420: per test index, (potential, drag) predicted by each
    model (de-normalised with the train statistics, drag = x-mean of the per-point drag), the
    density from a centred Gaussian (width 50 nm) propagated under the true and under each
    predicted (U, drag) (``simulate_density_trajectory``, :215-238), and
    time_averaged_L2_error (:240-295).  All trajectories go into ONE blindno_fp_propagate
    launch.  Returns {model: errors in index order}; with ``outdir`` writes
    <outdir>/<model>/pred_sample_<idx>.npy (Nx, 2) and ErrL2_<model>_Nsamples_<n>.npy."""
    from . import gpe
    stats = evaluate.compute_train_stats_1d(train)
    data = np.load(test) if isinstance(test, str) else test
    traj = np.asarray(data["trajectories"])
    idx = [int(i) for i in indices if 0 <= int(i) < traj.shape[0]]
    if not idx:
        return {name: np.zeros(0) for name in models}
    nx = traj.shape[2]
    xin = torch.tensor(np.stack([evaluate.normalize_input_1d(np.array(traj[i], dtype=np.float32), stats)
                                 for i in idx]), device=device)
    grid_n = torch.linspace(0, 1, nx, device=device).unsqueeze(-1)
    preds = {name: evaluate.predict(m, xin, grid_n, batch).cpu().numpy() for name, m in models.items()}

    def sim(U, drag):
        proto = fpe.fokker_planck(temperature=temperature, drag=drag, extent=extent_nm * NM,
                                  resolution=resolution_nm * NM, boundary=fpe.boundary.reflecting)
        return fpe.fokker_planck(temperature=temperature, drag=drag, extent=extent_nm * NM,
                                 resolution=resolution_nm * NM, boundary=fpe.boundary.reflecting,
                                 potential=fpe.potential_from_data(proto.grid[0], U))
    sims, saved = [], []
    for k, i in enumerate(idx):
        # the reference reads potential / drag as float32 (1d_FPE/compute_time_error.py:112-117)
        sims.append(sim(np.asarray(data["potential"][i], dtype=np.float32).astype(np.float64),
                        float(np.asarray(data["drag"], dtype=np.float32)[i])))
        for name in models:
            pot, drg = evaluate.denormalize_1d(preds[name][k], stats)
            saved.append((name, i, np.stack([pot, drg], axis=1)))
            sims.append(sim(pot, float(drg.mean())))
    pdf = fpe.gaussian_pdf(center=(0 * NM), width=init_width_nm * NM)
    res = fpe.propagate_many(sims, [pdf] * len(sims), dt, Nsteps=nsteps, device=device)
    grid = sims[0].grid
    per = 1 + len(models)
    errs = {name: [] for name in models}
    for k in range(len(idx)):
        t_ref, P_ref = res[k * per]
        for j, name in enumerate(models):
            t_p, P_p = res[k * per + 1 + j]
            errs[name].append(gpe.time_averaged_L2_error(t_ref, P_ref, t_p, P_p, grid))
    if outdir is not None:
        for name, i, arr in saved:
            d = os.path.join(outdir, name)
            os.makedirs(d, exist_ok=True)
            np.save(os.path.join(d, f"pred_sample_{i}.npy"), arr)
    out = {name: np.array(v, dtype=float) for name, v in errs.items()}
    if outdir is not None:
        for name, arr in out.items():
            np.save(os.path.join(outdir, f"ErrL2_{name}_Nsamples_{len(idx)}.npy"), arr)
    return out
