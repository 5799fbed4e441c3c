"""Batched evaluation / inference of the snapshot-bag models -- the eval_fno.py paths of the
2D experiments (``evaluate``), of 1d_FPE (``evaluate_1d_fpe``) and of 1d_GPE
(``evaluate_1d_gpe``).

Reference: 2d_FPE/eval_fno.py:34-281 (drift / diffusion, npz keys potential + drag) and
2d_Non_conservative_FPE/eval_fno.py:33-300 (Fx / Fy, npz key F).  The reference evaluates one
test trajectory at a time: normalise with the TRAIN statistics (:34-54, :66-70), eval-mode
forward with L = T (every snapshot), de-normalise (:72-99), relative L2 per field (:124-128),
one ``sample_XXXX_predictions.npy`` dict per index (:228-236) and a ``metrics.csv`` row
(:180-181, :275).

Here the eval-mode forward -- the only GPU work -- runs on ``batch`` test samples per launch
chain (eval mode has no batch coupling: FNO layers are per sample and the NIO branch's
BatchNorm uses running statistics), on the HIP path.  Normalisation, de-normalisation and the
metrics keep the reference's own float32 numpy sequences, so the numbers written match what
eval_fno.py writes for the same predictions.  The figures (matplotlib) are out of scope.
"""
from __future__ import annotations

import argparse
import csv
import os
from collections import OrderedDict
from typing import Dict, Iterable, List, Optional

import numpy as np
import torch

TRAJ_SCALE = 1e10
KINDS = {
    # kind: (target npz keys / scales, output names, metric header)
    "2d_FPE": dict(fields=("drift", "diffusion"), header=["index", "rel_l2_drift", "rel_l2_diffusion"]),
    "2d_Non_conservative_FPE": dict(fields=("Fx", "Fy"), header=["index", "rel_l2_Fx", "rel_l2_Fy"]),
}
DRIFT_SCALE, DIFFUSION_SCALE, F_SCALE = 1e21, 1e6, 1e12


def load_checkpoint_robust(ckpt_path: str, device="cpu") -> "OrderedDict[str, torch.Tensor]":
    """eval_fno.py:104-122: a raw state_dict or {'state_dict': ...}; leading 'module.'
    stripped.  Loaded with ``weights_only=True`` (tensors only, nothing executed)."""
    raw = torch.load(ckpt_path, map_location=device, weights_only=True)
    if isinstance(raw, dict) and isinstance(raw.get("state_dict"), dict):
        sd = raw["state_dict"]
    elif isinstance(raw, dict):
        sd = raw
    else:
        raise RuntimeError(f"Unrecognized checkpoint format at {ckpt_path}")
    return OrderedDict((k[len("module."):] if k.startswith("module.") else k, v) for k, v in sd.items())


def rel_l2(a: np.ndarray, b: np.ndarray, eps: float = 1e-12) -> float:
    """eval_fno.py:124-128."""
    return float(np.linalg.norm((a - b).ravel(), 2) / (np.linalg.norm(b.ravel(), 2) + eps))


def compute_train_stats(kind: str, train) -> Dict[str, np.ndarray]:
    """eval_fno.py:34-54 (2d_FPE) / 2d_Non_conservative_FPE/eval_fno.py:37-58.  ``train`` is an
    npz path or a dict of arrays."""
    data = np.load(train) if isinstance(train, str) else train
    traj = np.array(data["trajectories"], dtype=np.float32) * TRAJ_SCALE
    st = {"traj_mean": traj.mean(axis=(0, 1), keepdims=True),
          "traj_std": traj.std(axis=(0, 1), keepdims=True) + 1e-8}
    if kind == "2d_FPE":
        drift = np.array(data["potential"], dtype=np.float32) * DRIFT_SCALE
        diff = np.array(data["drag"], dtype=np.float32) * DIFFUSION_SCALE
        st.update(drift_mean=drift.mean(axis=0, keepdims=True), drift_std=drift.std(axis=0, keepdims=True) + 1e-8,
                  diff_mean=diff.mean(axis=0, keepdims=True), diff_std=diff.std(axis=0, keepdims=True) + 1e-8)
    else:
        F = np.array(data["F"], dtype=np.float32) * F_SCALE
        st.update(F_mean=F.mean(axis=0, keepdims=True), F_std=F.std(axis=0, keepdims=True) + 1e-8)
    return st


def normalize_input(traj_raw: np.ndarray, stats) -> np.ndarray:
    """eval_fno.py:66-70 for one (T, Nx, Ny) trajectory."""
    return (traj_raw * TRAJ_SCALE - stats["traj_mean"].squeeze(0)) / stats["traj_std"].squeeze(0)


def denormalize(kind: str, pred: np.ndarray, stats):
    """eval_fno.py:72-99 for one (Nx, Ny, 2) prediction -> two fields in original units."""
    if kind == "2d_FPE":
        a = (pred[..., 0] * stats["drift_std"].squeeze(0) + stats["drift_mean"].squeeze(0)) / DRIFT_SCALE
        b = (pred[..., 1] * stats["diff_std"].squeeze(0) + stats["diff_mean"].squeeze(0)) / DIFFUSION_SCALE
        return a, b
    mean = np.transpose(stats["F_mean"].squeeze(0), (1, 2, 0))
    std = np.transpose(stats["F_std"].squeeze(0), (1, 2, 0))
    return ((pred[..., 0] * std[..., 0] + mean[..., 0]) / F_SCALE,
            (pred[..., 1] * std[..., 1] + mean[..., 1]) / F_SCALE)


def true_fields(kind: str, data, index: int, stats):
    """The reference's normalise -> de-normalise round trip of the true fields
    (eval_fno.py:218-223; 2d_Non_conservative_FPE/eval_fno.py:261-267)."""
    if kind == "2d_FPE":
        out = []
        for key, scale, m, s in (("potential", DRIFT_SCALE, "drift_mean", "drift_std"),
                                 ("drag", DIFFUSION_SCALE, "diff_mean", "diff_std")):
            raw = np.array(data[key][index], dtype=np.float32)
            mu, sd = stats[m].squeeze(0), stats[s].squeeze(0)
            out.append(((raw * scale - mu) / sd * sd + mu) / scale)
        return tuple(out)
    F = np.array(data["F"][index], dtype=np.float32)
    mu, sd = stats["F_mean"].squeeze(0), stats["F_std"].squeeze(0)
    return tuple(((F[c] * F_SCALE - mu[c]) / sd[c] * sd[c] + mu[c]) / F_SCALE for c in (0, 1))


def grid2d(nx: int, ny: int, device) -> torch.Tensor:
    gx, gy = np.meshgrid(np.linspace(-1, 1, nx, dtype=np.float32),
                         np.linspace(-1, 1, ny, dtype=np.float32), indexing="ij")
    return torch.tensor(np.stack([gx, gy], axis=2), device=device)


@torch.no_grad()
def predict(model: torch.nn.Module, x: torch.Tensor, grid: torch.Tensor, batch: int = 8) -> torch.Tensor:
    """Eval-mode predictions (n, Nx, Ny, 2) of normalised bags x (n, T, Nx, Ny) in HBM,
    ``batch`` samples per forward."""
    was = model.training
    model.eval()
    try:
        outs = [model(x[i:i + batch], grid) for i in range(0, x.shape[0], batch)]
    finally:
        model.train(was)
    out = torch.cat(outs, 0)
    if out.dim() == 4 and out.shape[1] == 2 and out.shape[-1] != 2:
        out = out.permute(0, 2, 3, 1)
    return out.contiguous()


def evaluate(kind: str, model: torch.nn.Module, train, test, indices: Iterable[int],
             outdir: Optional[str] = None, batch: int = 8, device="cuda") -> List[list]:
    """The eval_fno.py loop over ``indices`` (out-of-range ones skipped, :196-201).  Returns the
    metrics rows [index, rel_l2_a, rel_l2_b]; with ``outdir`` also writes the per-sample .npy
    dicts and appends metrics.csv exactly as the reference does."""
    names = KINDS[kind]["fields"]
    stats = compute_train_stats(kind, train)
    data = np.load(test) if isinstance(test, str) else test
    traj = np.asarray(data["trajectories"])
    M = traj.shape[0]
    idx = [i for i in indices if 0 <= i < M]
    nx, ny = traj.shape[2], traj.shape[3]
    x = np.stack([normalize_input(np.array(traj[i], dtype=np.float32), stats) for i in idx]) if idx else \
        np.zeros((0,) + traj.shape[1:], np.float32)
    xd = torch.tensor(x, dtype=torch.float32, device=device)
    pred = predict(model, xd, grid2d(nx, ny, device), batch).cpu().numpy() if idx else None
    rows = []
    writer = f_csv = None
    if outdir is not None:
        os.makedirs(outdir, exist_ok=True)
        path = os.path.join(outdir, "metrics.csv")
        header = not os.path.exists(path)
        f_csv = open(path, "a", newline="")
        writer = csv.writer(f_csv)
        if header:
            writer.writerow(KINDS[kind]["header"])
    try:
        for k, i in enumerate(idx):
            pa, pb = denormalize(kind, pred[k], stats)
            ta, tb = true_fields(kind, data, i, stats)
            row = [i, rel_l2(pa, ta), rel_l2(pb, tb)]
            rows.append(row)
            if writer is not None:
                np.save(os.path.join(outdir, f"sample_{i:04d}_predictions.npy"), {
                    "index": i,
                    f"{names[0]}_pred": pa.astype(np.float32), f"{names[1]}_pred": pb.astype(np.float32),
                    f"{names[0]}_true": ta.astype(np.float32), f"{names[1]}_true": tb.astype(np.float32)})
                writer.writerow(row)
    finally:
        if f_csv is not None:
            f_csv.close()
    return rows


# ------------------------------------------------------------------------------- 1D FPE
# 1d_FPE/eval_fno.py:23-190: scales 1e5 / 1e20 / 1e5, drag a per-sample scalar; the script
# predicts one sample, saves pred_sample_<idx>.npy = stack(potential, drag per point) (Nx, 2) in
# physical units and prints the x-mean of the predicted drag next to the true one.
TRAJ_SCALE_1D, POTENTIAL_SCALE_1D, DRAG_SCALE_1D = 1e5, 1e20, 1e5


def compute_train_stats_1d(train) -> Dict[str, np.ndarray]:
    """1d_FPE/eval_fno.py:30-53."""
    data = np.load(train) if isinstance(train, str) else train
    traj = np.array(data["trajectories"], dtype=np.float32) * TRAJ_SCALE_1D
    pot = np.array(data["potential"], dtype=np.float32) * POTENTIAL_SCALE_1D
    drag = (np.array(data["drag"], dtype=np.float32) * DRAG_SCALE_1D)[:, np.newaxis]
    return {"traj_mean": traj.mean(axis=(0, 1), keepdims=True),
            "traj_std": traj.std(axis=(0, 1), keepdims=True) + 1e-8,
            "pot_mean": pot.mean(axis=(0), keepdims=True), "pot_std": pot.std(axis=(0), keepdims=True) + 1e-8,
            "drag_mean": drag.mean(axis=(0), keepdims=True), "drag_std": drag.std(axis=(0), keepdims=True) + 1e-8}


def normalize_input_1d(traj_raw: np.ndarray, stats) -> np.ndarray:
    """1d_FPE/eval_fno.py:74-80."""
    t = traj_raw * TRAJ_SCALE_1D
    return ((t - stats["traj_mean"].squeeze()) / stats["traj_std"].squeeze()).astype(np.float32)


def denormalize_1d(pred: np.ndarray, stats):
    """1d_FPE/eval_fno.py:86-97: (Nx, 2) -> potential (Nx,), drag per point (Nx,)."""
    pot = (pred[:, 0] * stats["pot_std"].squeeze() + stats["pot_mean"].squeeze()) / POTENTIAL_SCALE_1D
    drg = (pred[:, 1] * stats["drag_std"].squeeze() + stats["drag_mean"].squeeze()) / DRAG_SCALE_1D
    return pot, drg


def evaluate_1d_fpe(model: torch.nn.Module, train, test, indices: Iterable[int],
                    outdir: Optional[str] = None, batch: int = 32, device="cuda") -> List[list]:
    """1d_FPE/eval_fno.py:116-190 over ``indices`` with the forward batched on the HIP path.
    Rows [index, predicted drag (x-mean), true drag, rel_l2(potential)]; with ``outdir`` also
    the reference's pred_sample_<idx>.npy (Nx, 2) files."""
    stats = compute_train_stats_1d(train)
    data = np.load(test) if isinstance(test, str) else test
    traj = np.asarray(data["trajectories"])
    idx = [i for i in indices if 0 <= i < traj.shape[0]]
    if not idx:
        return []
    nx = traj.shape[2]
    x = torch.tensor(np.stack([normalize_input_1d(np.array(traj[i], dtype=np.float32), stats) for i in idx]),
                     device=device)
    grid = torch.linspace(0, 1, nx, device=device).unsqueeze(-1)     # 1d_FPE/eval_fno.py:138
    pred = predict(model, x, grid, batch).cpu().numpy()
    rows = []
    if outdir is not None:
        os.makedirs(outdir, exist_ok=True)
    for k, i in enumerate(idx):
        pot, drg = denormalize_1d(pred[k], stats)
        pot_true = np.array(data["potential"][i], dtype=np.float32)
        drag_true = float(np.array(data["drag"], dtype=np.float32)[i])
        rows.append([i, float(drg.mean()), drag_true, rel_l2(pot, pot_true)])
        if outdir is not None:
            np.save(os.path.join(outdir, f"pred_sample_{i}.npy"), np.stack([pot, drg], axis=1))
    return rows


# ------------------------------------------------------------------------------- 1D GPE
def compute_train_scalers_gpe(train) -> Dict[str, float]:
    """1d_GPE/eval_fno_GPE.py:32-57: divide-by-max scalers (no mean removal)."""
    return {"y_max": train["y"].max() / 3.0, "V_max": train["V"].max() / 3.0,
            "g_max": train["g"].max(), "kappa_max": train["kappa"].max()}


def normalize_gpe(d, sc) -> Dict[str, np.ndarray]:
    """1d_GPE/eval_fno_GPE.py:59-67."""
    return {"y": d["y"] / sc["y_max"], "V": d["V"] / sc["V_max"], "g": d["g"] / sc["g_max"],
            "kappa": d["kappa"] / sc["kappa_max"]}


def evaluate_1d_gpe(model: torch.nn.Module, train, test, indices: Iterable[int],
                    outdir: Optional[str] = None, batch: int = 32, device="cuda") -> List[list]:
    """1d_GPE/eval_fno_GPE.py:95-171 over ``indices`` (the script takes one --sample_idx), with
    the forward batched on the HIP path.  ``train`` / ``test`` are the generator's dicts
    (y, g, kappa, V; blindno.gpe).  Rows [index, rel_l2(pred_V, true_V)]; with ``outdir`` also
    the reference's save dict (x, pred_V, true_V, V_max_used, note) per index as
    sample_pred_V_<idx>.npy."""
    sc = compute_train_scalers_gpe(train)
    tn = normalize_gpe(test, sc)
    y = np.asarray(tn["y"])
    idx = [i for i in indices if 0 <= i < y.shape[0]]
    if not idx:
        return []
    nx = y.shape[2]
    x = torch.tensor(np.stack([y[i] for i in idx]), dtype=torch.float32, device=device)
    grid = torch.linspace(0, 1, nx, device=device).unsqueeze(-1)     # :126
    pred = predict(model, x, grid, batch).cpu().numpy()
    if pred.ndim == 3:
        pred = pred[..., 0]
    xs = np.linspace(0.0, 1.0, nx)
    rows = []
    if outdir is not None:
        os.makedirs(outdir, exist_ok=True)
    for k, i in enumerate(idx):
        pred_V = pred[k] * sc["V_max"]
        true_V = tn["V"][i] * sc["V_max"]
        rows.append([i, rel_l2(pred_V, true_V)])
        if outdir is not None:
            np.save(os.path.join(outdir, f"sample_pred_V_{i}.npy"), {
                "x": xs, "pred_V": pred_V, "true_V": true_V, "V_max_used": sc["V_max"],
                "note": "Values are de-normalized using training set V_max (V_max = V_train.max()/3)."})
    return rows


def main(argv=None):
    """CLI mirroring eval_fno.py's arguments (:131-150) plus --experiment, --model, --batch."""
    from . import nio
    ap = argparse.ArgumentParser(description="Batched evaluation of a trained 2D snapshot-bag model.")
    ap.add_argument("--experiment", choices=sorted(KINDS) + ["1d_FPE", "1d_GPE"], default="2d_FPE")
    ap.add_argument("--model", choices=["NIOFP2D_FNO", "NIOFP2D_FNO_attn", "NIOFP2D", "PermInvUNet_attn",
                                        "PermInvUNet_attn1D_bag", "PermInvUNet_attn1D_bag_GPE"], default=None,
                    help="PermInvUNet_attn*: the eval_unet*.py models (attention UNet)")
    ap.add_argument("--train_data", required=True)
    ap.add_argument("--test_data", required=True)
    ap.add_argument("--ckpt", required=True)
    ap.add_argument("--outdir", default="result_fig/fno")
    ap.add_argument("--start", type=int, default=33)
    ap.add_argument("--end", type=int, default=64)
    ap.add_argument("--nx", type=int, default=61)
    ap.add_argument("--ny", type=int, default=61)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--strict", action="store_true")
    a = ap.parse_args(argv)
    a.model_given = a.model is not None
    a.model = a.model or "NIOFP2D_FNO"
    heads = ("fno_drift", "fno_diffusion") if a.experiment == "2d_FPE" else ("fno_Fx", "fno_Fy")
    from . import unet
    one_d_unet = {"1d_FPE": "PermInvUNet_attn1D_bag", "1d_GPE": "PermInvUNet_attn1D_bag_GPE"}
    if a.experiment in ("1d_FPE", "1d_GPE"):
        if a.model_given and a.model != one_d_unet[a.experiment]:
            ap.error(f"--model {a.model} is not a {a.experiment} model: the evaluation builds the "
                     f"reference's NIOFP_FNO (1d_FPE/eval_fno.py:100-114, 1d_GPE/eval_fno_GPE.py:69-83) "
                     f"or, with --model {one_d_unet[a.experiment]}, its eval_unet model")
        # the reference's 1D eval models: NIOFP_FNO(3, 30, 15, 2) (1d_FPE/eval_fno.py:100-114),
        # NIOFP_FNO(3, 20, 40, 1) head fno_V (1d_GPE/eval_fno_GPE.py:69-83); the UNets of
        # 1d_FPE/eval_unet_bag.py:102 and 1d_GPE/eval_unet_GPE.py (width 20, modes 40)
        if a.model_given and a.experiment == "1d_FPE":
            model = unet.PermInvUNet_attn1D_bag(1, 2, 1, 4, 80, device=a.device)
        elif a.model_given:
            model = unet.PermInvUNet_attn1D_bag_GPE(1, 2, 1, 4, 128, device=a.device, width=20, modes=40)
        else:
            model = nio.NIOFP_FNO(3, 30, 15, 2, a.device) if a.experiment == "1d_FPE" else \
                nio.NIOFP_FNO(3, 20, 40, 1, a.device, heads=("fno_V",))
        ret = model.load_state_dict(load_checkpoint_robust(a.ckpt), strict=a.strict)
        if ret.missing_keys or ret.unexpected_keys:
            print("[Warn] Incompatible keys when loading:", ret.missing_keys, ret.unexpected_keys)
        model = model.to(a.device)
        idx = range(a.start, a.end + 1)
        if a.experiment == "1d_FPE":
            for r in evaluate_1d_fpe(model, a.train_data, a.test_data, idx, outdir=a.outdir,
                                     batch=a.batch, device=a.device):
                print(f"[Metrics] index={r[0]}  drag_pred={r[1]:.6g}  drag_true={r[2]:.6g}  "
                      f"rel_l2_potential={r[3]:.6f}")
        else:
            # the GPE generator's files are np.save'd dicts: read by a restricted unpickler
            # (numpy arrays / scalars only), never allow_pickle
            from .data import load_npy_dict
            tr = load_npy_dict(a.train_data)
            te = load_npy_dict(a.test_data)
            for r in evaluate_1d_gpe(model, tr, te, idx, outdir=a.outdir, batch=a.batch, device=a.device):
                print(f"[Metrics] index={r[0]}  rel_l2_V={r[1]:.6f}")
        return
    if a.model in one_d_unet.values():
        ap.error(f"--model {a.model} is a 1D model")
    if a.model == "PermInvUNet_attn":
        # 2d_FPE/eval_unet.py:156 (depth 4), 2d_Non_conservative_FPE/eval_unet.py:192 (depth 5)
        model = (unet.PermInvUNet_attn(1, 2, 1, 4, (a.nx, a.ny)) if a.experiment == "2d_FPE" else
                 unet.PermInvUNet_attn_NC(1, 2, 1, 5, (a.nx, a.ny)))
    elif a.model == "NIOFP2D_FNO_attn":
        model = nio.NIOFP2D_FNO_attn(2, 3, 100, 25, 3, 12, 32, 2, a.nx, a.ny, heads=heads)
    else:
        cls = getattr(nio, a.model)
        model = cls(2, 3, 100, 25, 3, 12, 32, 2, heads=heads,
                    branch_last_kernel=(2, 1) if a.experiment == "2d_FPE" else (3, 2))
    ret = model.load_state_dict(load_checkpoint_robust(a.ckpt), strict=a.strict)
    if ret.missing_keys or ret.unexpected_keys:
        print("[Warn] Incompatible keys when loading:", ret.missing_keys, ret.unexpected_keys)
    model = model.to(a.device)
    rows = evaluate(a.experiment, model, a.train_data, a.test_data, range(a.start, a.end + 1),
                    outdir=a.outdir, batch=a.batch, device=a.device)
    for r in rows:
        print(f"[Metrics] index={r[0]}  {KINDS[a.experiment]['header'][1]}={r[1]:.6f}  "
              f"{KINDS[a.experiment]['header'][2]}={r[2]:.6f}")
    print(f"[Info] Metrics saved to: {os.path.join(a.outdir, 'metrics.csv')}")


if __name__ == "__main__":
    main()
