"""1D Gross-Pitaevskii data generator / density propagator and the 1D density-error metric on
the GPU (libblindno ``blindno_gpe_solve`` / ``blindno_trapz_rows``; fp64 like the reference).

Reference (yl602019618/Reconstruction-of-PDE-without-Time-Label):
  get_initial_condition, solve_GPE_custom, generate_and_save_training_data
      1d_GPE/datagen_GPE.py:7-21, 86-115, 120-191
  time_averaged_L2_error
      1d_FPE/compute_time_error.py:240-295 = 1d_GPE/compute_time_error_GPE.py:162-203

The reference integrates one trajectory at a time in numpy (0.06 s per 1001-step trajectory at
Nx = 128); here every trajectory of a batch is one workgroup that keeps its field, twiddles and
phase tables in LDS for the whole time loop.
"""
from __future__ import annotations

from typing import Optional, Sequence, Union

import numpy as np
import torch

from ._lib import BlindnoError, call, ptr, stream_ptr

F64 = torch.float64


def initial_condition(ic: int, x: np.ndarray) -> np.ndarray:
    """get_initial_condition (1d_GPE/datagen_GPE.py:7-21)."""
    if ic == 1:
        return np.exp(-x ** 2 / 10)
    if ic == 2:
        return 2 * np.sin(x) / (np.exp(x) + np.exp(-x))
    if ic == 3:
        return 2 * np.cos(x) / (np.exp(x) + np.exp(-x))
    raise ValueError("ic must be 1, 2 or 3")


def _dev(device):
    dev = torch.device(device if device is not None else "cuda")
    if dev.type != "cuda":
        raise BlindnoError("the GPE solver runs on the HIP device only (there is no CPU path)")
    return dev


def solve_batch(psi0, x, dt: float, t_final: float, order: int, g, kappa, V, rec_every: int = 1,
                want_abs: bool = True, want_psi: bool = False, device=None):
    """Integrate B trajectories at once.

    psi0: (Nx,) or (B, Nx) complex initial field; V: (Nx,) or (B, Nx); g, kappa: scalars or
    (B,).  Returns a dict with ``t`` (numpy, the recorded times), ``abs`` (B, nrec, Nx) fp64
    device tensor of |psi| (if ``want_abs``), ``psi`` (B, nrec, Nx) complex128 (if
    ``want_psi``) and ``final`` (B, Nx) complex128.  Records every ``rec_every``-th step,
    step 0 included (``psi_abs[::rec_every]`` of the reference's full record)."""
    dev = _dev(device)
    x = np.asarray(x, dtype=np.float64)
    N = len(x)
    V = np.atleast_2d(np.asarray(V, dtype=np.float64))
    B = V.shape[0]
    psi0 = np.asarray(psi0, dtype=np.complex128)
    batched = psi0.ndim == 2
    if batched and psi0.shape[0] != B:
        raise BlindnoError("psi0 and V batch sizes differ")
    g = np.broadcast_to(np.asarray(g, dtype=np.float64), (B,)).copy()
    kappa = np.broadcast_to(np.asarray(kappa, dtype=np.float64), (B,)).copy()
    if N & (N - 1) or N < 4 or N > 2048:
        raise BlindnoError(f"Nx = {N}: the solver needs a power of two in [4, 2048]")
    nt = int(t_final / dt) + 1
    nsteps = nt - 1
    nrec = nsteps // rec_every + 1
    t_full = np.linspace(0, t_final, nt)
    p0 = torch.from_numpy(np.ascontiguousarray(psi0.view(np.float64))).to(dev)
    Vd = torch.from_numpy(np.ascontiguousarray(V)).to(dev)
    gd = torch.from_numpy(g).to(dev)
    kd = torch.from_numpy(kappa).to(dev)
    rabs = torch.empty(B, nrec, N, dtype=F64, device=dev) if want_abs else None
    rpsi = torch.empty(B, nrec, N, 2, dtype=F64, device=dev) if want_psi else None
    fin = torch.empty(B, N, 2, dtype=F64, device=dev)
    dx = float(x[1] - x[0])
    call("blindno_gpe_solve", ptr(p0), ptr(Vd), ptr(gd), ptr(kd), dx, float(dt), nsteps, int(order),
         int(rec_every), ptr(rabs), ptr(rpsi), ptr(fin), B, N, int(batched), stream_ptr(dev))
    out = {"t": t_full[::rec_every][:nrec], "final": torch.view_as_complex(fin)}
    if want_abs:
        out["abs"] = rabs
    if want_psi:
        out["psi"] = torch.view_as_complex(rpsi)
    return out


def solve_GPE_custom(init_func, x, dt, t_final, order, g, kappa, V):
    """Drop-in for the reference's ``solve_GPE_custom`` (1d_GPE/datagen_GPE.py:86-115): same
    arguments, returns (t, psi_record (Nt, Nx) complex128 numpy), computed on the GPU."""
    x = np.asarray(x, dtype=np.float64)
    r = solve_batch(init_func(x), x, dt, t_final, order, g, kappa, V, rec_every=1,
                    want_abs=False, want_psi=True)
    return np.linspace(0, t_final, int(t_final / dt) + 1), r["psi"][0].cpu().numpy()


def generate_training_data(num_orbits: int = 6000, Nx: int = 128, dt: float = 0.005,
                           t_final: float = 5.0, order: int = 2, num_time_samples: int = 100,
                           rng=np.random, device=None, batch: int = 4096):
    """generate_and_save_training_data (1d_GPE/datagen_GPE.py:120-191) without the file write:
    the same parameter draws from ``rng`` in the reference's order (a, b, c, x0, then the
    unused time-sample choice), initial condition 2, g = kappa = 2, y = |psi|[::10].  All
    orbits are integrated in batched launches.  Returns the reference's dict
    {'y': (M, Nt//10 + 1, Nx), 'g', 'kappa', 'V'} as numpy arrays."""
    x = np.linspace(-10, 10, Nx)
    nt = int(t_final / dt) + 1
    Vs, gs, ks = [], [], []
    for _ in range(num_orbits):
        a = rng.uniform(0.1, 0.3)
        b = rng.uniform(0.5, 2)
        c = rng.uniform(0.5, 2)
        x0 = rng.uniform(-3, 3)
        Vs.append(a * (x - x0) ** 2 + b * (np.cos(c * (x - x0))) ** 2)
        gs.append(2)
        ks.append(2)
        np.sort(rng.choice(np.arange(nt), size=num_time_samples, replace=False))
    V = np.stack(Vs, 0)
    psi0 = initial_condition(2, x)
    ys = []
    for s in range(0, num_orbits, batch):
        r = solve_batch(psi0, x, dt, t_final, order, 2.0, 2.0, V[s:s + batch], rec_every=10,
                        device=device)
        ys.append(r["abs"].cpu().numpy())
    return {"y": np.concatenate(ys, 0), "g": np.array(gs), "kappa": np.array(ks), "V": V}


def save_training_data(data: dict, save_path: str) -> None:
    """The reference's on-disk format: ``np.save`` of the dict (datagen_GPE.py:183-189);
    train_fno_GPE.py:38 reads it back with ``np.load(..., allow_pickle=True).item()``."""
    np.save(save_path, data, allow_pickle=True)


def time_averaged_L2_error(time_ref, rho_ref, time_pred, rho_pred, grid, eps: float = 1e-12,
                           device=None) -> float:
    """1d_FPE/compute_time_error.py:240-295: per-time sqrt(trapz((rho_pred - rho_ref)^2, x)) /
    (sqrt(trapz(rho_ref^2, x)) + eps), then the trapezoid time average / (t_end - t_0).
    rho_* are (Nt, Nx) numpy arrays or device tensors; the spatial integrals run on the GPU
    in fp64."""
    dev = _dev(device if device is not None else (rho_ref.device if torch.is_tensor(rho_ref) else None))
    if tuple(rho_ref.shape) != tuple(rho_pred.shape):
        raise ValueError(f"rho_ref shape {tuple(rho_ref.shape)} != rho_pred shape {tuple(rho_pred.shape)}")
    if isinstance(grid, (list, tuple)):
        if len(grid) != 1:
            raise ValueError(f"unsupported grid: len(grid) = {len(grid)}")
        xg = np.asarray(grid[0])
    else:
        xg = np.asarray(grid)
        if xg.ndim == 2 and xg.shape[0] == 1:
            xg = xg[0]
        elif xg.ndim != 1:
            raise ValueError(f"unsupported grid shape {xg.shape}")
    if not np.allclose(np.asarray(time_ref), np.asarray(time_pred)):
        raise ValueError("time_ref and time_pred differ")

    def d64(a):
        t = a if torch.is_tensor(a) else torch.from_numpy(np.asarray(a))
        return t.to(dev, F64).contiguous()

    a, b = d64(rho_pred), d64(rho_ref)
    xd = d64(xg)
    nt, n = a.shape
    s = torch.empty(nt, 2, dtype=F64, device=dev)
    call("blindno_trapz_rows", ptr(a), ptr(b), ptr(xd), ptr(s), nt, n, stream_ptr(dev))
    rel = s[:, 0].clamp_min(0).sqrt() / (s[:, 1].clamp_min(0).sqrt() + eps)
    t = d64(time_ref)
    integral = (0.5 * (rel[:-1] + rel[1:]) * (t[1:] - t[:-1])).sum()
    return float(integral / (t[-1] - t[0]))
