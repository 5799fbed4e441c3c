#!/usr/bin/env python3
"""Capture golden vectors of the reference's eval_fno.py host math (build container only).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_eval.py [--ref /root/reference]

eval_fno.py imports matplotlib (absent here) at top level, so -- as make_golden.py does for
the metric helpers -- the pure-numpy functions (compute_train_stats, normalize_input,
denormalize_output, rel_l2) and the module's scale constants are taken from the reference
file's source and run on a tiny synthetic train/test npz.  The true-field round trip of the
main loop (2d_FPE/eval_fno.py:218-223; NC :261-267) is a statement sequence, not a function:
it is restated inline below.  Writes eval_2d_fpe.npz and eval_2d_nc.npz.
"""
from __future__ import annotations

import argparse
import ast
import os
import sys
import tempfile

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)


def _namespace(path, names):
    src = open(path).read()
    tree = ast.parse(src)
    glb = {"np": np, "torch": torch, "os": os}
    for node in tree.body:
        if isinstance(node, ast.Assign) and all(isinstance(t, ast.Name) and t.id.endswith("_SCALE")
                                                for t in node.targets):
            exec(compile(ast.get_source_segment(src, node), path, "exec"), glb)
        if isinstance(node, ast.FunctionDef) and node.name in names:
            exec(compile(ast.get_source_segment(src, node), path, "exec"), glb)
    return glb


def main():
    from make_golden import _save
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    a = ap.parse_args()
    rs = np.random.RandomState(7)
    M, T, N = 4, 60, 8
    names = ("compute_train_stats", "normalize_input", "denormalize_output", "rel_l2")
    for exp, tag in (("2d_FPE", "eval_2d_fpe"), ("2d_Non_conservative_FPE", "eval_2d_nc")):
        g = _namespace(os.path.join(a.ref, exp, "eval_fno.py"), names)
        traj = (rs.rand(M, T, N, N) * 1e-10).astype(np.float32)
        test_traj = (rs.rand(2, T, N, N) * 1e-10).astype(np.float32)
        if exp == "2d_FPE":
            tr = dict(trajectories=traj, potential=(rs.randn(M, N, N) * 1e-21).astype(np.float32),
                      drag=(rs.rand(M, N, N) * 1e-6).astype(np.float32))
            te = dict(trajectories=test_traj, potential=(rs.randn(2, N, N) * 1e-21).astype(np.float32),
                      drag=(rs.rand(2, N, N) * 1e-6).astype(np.float32))
        else:
            tr = dict(trajectories=traj, F=(rs.randn(M, 2, N, N) * 1e-12).astype(np.float32))
            te = dict(trajectories=test_traj, F=(rs.randn(2, 2, N, N) * 1e-12).astype(np.float32))
        with tempfile.TemporaryDirectory() as d:
            p = os.path.join(d, "train.npz")
            np.savez(p, **tr)
            stats = g["compute_train_stats"](p)
        out = {f"train.{k}": v for k, v in tr.items()}
        out.update({f"test.{k}": v for k, v in te.items()})
        out.update({f"stats.{k}": v for k, v in stats.items()})
        pred = rs.randn(2, N, N, 2).astype(np.float32)
        out["pred"] = pred
        for i in range(2):
            xn = g["normalize_input"](test_traj[i], stats).numpy()
            pa, pb = g["denormalize_output"](torch.tensor(pred[i:i + 1]), stats)
            if exp == "2d_FPE":
                ta = ((te["potential"][i] * g["DRIFT_SCALE"] - stats["drift_mean"].squeeze(0)) / stats["drift_std"].squeeze(0)
                      * stats["drift_std"].squeeze(0) + stats["drift_mean"].squeeze(0)) / g["DRIFT_SCALE"]
                tb = ((te["drag"][i] * g["DIFFUSION_SCALE"] - stats["diff_mean"].squeeze(0)) / stats["diff_std"].squeeze(0)
                      * stats["diff_std"].squeeze(0) + stats["diff_mean"].squeeze(0)) / g["DIFFUSION_SCALE"]
            else:
                Fm, Fs = stats["F_mean"].squeeze(0), stats["F_std"].squeeze(0)
                ta = ((te["F"][i, 0] * g["F_SCALE"] - Fm[0]) / Fs[0] * Fs[0] + Fm[0]) / g["F_SCALE"]
                tb = ((te["F"][i, 1] * g["F_SCALE"] - Fm[1]) / Fs[1] * Fs[1] + Fm[1]) / g["F_SCALE"]
            out[f"x_norm{i}"] = xn[0]
            out[f"pred_a{i}"], out[f"pred_b{i}"] = pa, pb
            out[f"true_a{i}"], out[f"true_b{i}"] = ta, tb
            out[f"rel_a{i}"] = np.array(g["rel_l2"](pa, ta))
            out[f"rel_b{i}"] = np.array(g["rel_l2"](pb, tb))
        _save(tag, out)
    # 1d_FPE/eval_fno.py: compute_train_stats, normalize_with_train_stats, denormalize_outputs
    g = _namespace(os.path.join(a.ref, "1d_FPE", "eval_fno.py"),
                   ("compute_train_stats", "normalize_with_train_stats", "denormalize_outputs"))
    tr = dict(trajectories=(rs.rand(M, T, 16) * 1e-5).astype(np.float32),
              potential=(rs.randn(M, 16) * 1e-20).astype(np.float32),
              drag=(rs.rand(M) * 1e-5).astype(np.float32))
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "train.npz")
        np.savez(p, **tr)
        stats = g["compute_train_stats"](p)
    out = {f"train.{k}": v for k, v in tr.items()}
    out.update({f"stats.{k}": v for k, v in stats.items()})
    test_traj = (rs.rand(T, 16) * 1e-5).astype(np.float32)
    pred = rs.randn(16, 2).astype(np.float32)
    pot, drg = g["denormalize_outputs"](pred, stats)
    out.update({"test_traj": test_traj, "x_norm": g["normalize_with_train_stats"](test_traj, stats),
                "pred": pred, "pot": pot, "drg": drg})
    _save("eval_1d_fpe", out)


if __name__ == "__main__":
    main()
