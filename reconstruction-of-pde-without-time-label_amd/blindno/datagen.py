"""FPE snapshot-bag dataset generators (§8f3) -- the reference's generator scripts with every
trajectory propagated on the GPU in one batched launch (blindno.fpe.propagate_many).

  fpe_1d_dataset     1d_FPE/dataset_1d_drift_diffusion.py:6-98  (three Gaussian wells, scalar
                     drag scaled by the same random factor; npz keys time, grid, trajectories,
                     potential, drag)
  fpe_2d_dataset     2d_FPE/test_datagen.py:6-95  (three 2D Gaussian wells, drag field
                     drag (1 + f ((x-cx)^2 + (y-cy)^2) / (250 nm)^2); keys as above, drag a field)
  fpe_2d_nc_dataset  2d_Non_conservative_FPE/testdata_gen.py:6-101  (non-conservative
                     rotational/radial force field; keys time, grid, trajectories, F)

Random parameters come from numpy's global RNG in the reference's per-simulation order (the
parameter draw, then the choice of the 100 recorded time indices -- the propagation draws
nothing in between), so a seeded run reproduces the reference's parameters.  The reference's
2D scripts run simulations in a thread pool and append them in completion order; here the
order is the simulation index.  The densities depend on fplanck (absent): parity UNPINNED
(blindno.fpe).  ``save_npz`` writes the reference's file layout.
"""
from __future__ import annotations

from typing import Optional

import numpy as np

from . import fpe

NM = 1e-9
VISCOSITY = 8e-4
RADIUS = 50 * NM
DRAG = 6 * np.pi * VISCOSITY * RADIUS
TEMPERATURE = 300


def _select(n_time, k=100):
    return np.sort(np.random.choice(range(n_time), size=k, replace=False))


def fpe_1d_dataset(M: int = 100, nsteps: int = 400, tf: float = 2e-3, device="cuda"):
    """1d_FPE/dataset_1d_drift_diffusion.py:18-98."""
    sims, pdfs, sels, pots, drags = [], [], [], [], []
    for _ in range(M):
        while True:                                  # :19-24
            centers = np.random.uniform(-150 * NM, 150 * NM, size=(3))
            if all(np.abs(centers[i] - centers[j]) > 80 * NM for i in range(3) for j in range(i + 1, 3)):
                break
        widths = np.random.uniform(20 * NM, 80 * NM, size=3)
        As = np.random.uniform(1e-20, 2e-20, size=3)
        vf = np.random.uniform(1, 2, size=1)
        U = fpe.combine(*[fpe.gaussian_potential(center=centers[i], width=widths[i], amplitude=As[i] * vf[0])
                          for i in range(3)])
        drag = DRAG * vf[0]
        sim = fpe.fokker_planck(temperature=TEMPERATURE, drag=drag, extent=800 * NM, resolution=10 * NM,
                                boundary=fpe.boundary.reflecting, potential=U)
        sims.append(sim)
        pdfs.append(fpe.gaussian_pdf(center=(0 * NM), width=50 * NM))
        sels.append(_select(nsteps))
        pots.append(U(*sim.grid))
        drags.append(drag)
    res = fpe.propagate_many(sims, pdfs, tf, Nsteps=nsteps, device=device, select=sels)
    return dict(time=np.array([t for t, _ in res]), grid=np.array([s.grid for s in sims]),
                trajectories=np.array([p for _, p in res]), potential=np.array(pots),
                drag=np.array(drags))


def fpe_2d_dataset(M: int = 400, nsteps: int = 1000, tf: float = 2e-4, device="cuda"):
    """2d_FPE/test_datagen.py:20-95 (test set generator of the 2D FPE experiment)."""
    sims, pdfs, sels, pots, drags = [], [], [], [], []
    for _ in range(M):
        while True:                                  # :21-27
            centers = np.random.uniform(-100 * NM, 100 * NM, size=(3, 2))
            dist = np.sqrt(np.sum((centers[:, None] - centers[None, :]) ** 2, axis=-1))
            if np.all(dist[np.triu_indices(3, k=1)] > 90 * NM):
                break
        widths = np.random.uniform(20 * NM, 80 * NM, size=3)
        As = np.random.uniform(1e-20, 2e-20, size=3)
        vf = np.random.uniform(0, 2, size=1)
        dc = np.random.uniform(-100 * NM, 100 * NM, size=(1, 2))
        U = fpe.combine(*[fpe.gaussian_potential(center=centers[i], width=widths[i], amplitude=As[i])
                          for i in range(3)])

        def drag_fn(x, y, vf=vf, dc=dc):
            xs = (x - dc[0, 0]) / 250 / NM
            ys = (y - dc[0, 1]) / 250 / NM
            return DRAG * (1 + vf * xs ** 2 + vf * ys ** 2)
        sim = fpe.fokker_planck(temperature=TEMPERATURE, drag=drag_fn, extent=[600 * NM, 600 * NM],
                                resolution=10 * NM, boundary=fpe.boundary.reflecting, potential=U)
        sims.append(sim)
        pdfs.append(fpe.gaussian_pdf(center=(0 * NM, 0 * NM), width=50 * NM))
        sels.append(_select(nsteps))
        pots.append(U(*sim.grid))
        drags.append(drag_fn(*sim.grid))
    res = fpe.propagate_many(sims, pdfs, tf, Nsteps=nsteps, device=device, select=sels)
    return dict(time=np.array([t for t, _ in res]), grid=np.array([s.grid for s in sims]),
                trajectories=np.array([p for _, p in res]), potential=np.array(pots),
                drag=np.array(drags))


def nc_force(x, y, L=100 * NM, a=1, b=1, c=1, d=1):
    """2d_Non_conservative_FPE/testdata_gen.py:18-27."""
    rad = np.sqrt(x ** 2 + y ** 2)
    phi = np.arctan2(y, x)
    Fphi = 1e-12 * rad / L * np.exp(-rad / L * b) * a
    Frad = 1e-12 * (1 - rad / L) * np.exp(-rad / L * d) * c
    return np.array([-np.sin(phi) * Fphi + np.cos(phi) * Frad, np.cos(phi) * Fphi + np.sin(phi) * Frad])


def fpe_2d_nc_dataset(M: int = 400, nsteps: int = 500, tf: float = 10e-3, device="cuda"):
    """2d_Non_conservative_FPE/testdata_gen.py:33-101."""
    sims, pdfs, sels, Fs = [], [], [], []
    for _ in range(M):
        L_, a_, b_, c_, d_ = (np.random.uniform(50 * NM, 150 * NM), np.random.uniform(0.5, 2),
                              np.random.uniform(0.5, 2), np.random.uniform(0.5, 2), np.random.uniform(0.5, 2))

        def force(x, y, L_=L_, a_=a_, b_=b_, c_=c_, d_=d_):
            return nc_force(x, y, L=L_, a=a_, b=b_, c=c_, d=d_)
        sim = fpe.fokker_planck(temperature=TEMPERATURE, drag=DRAG, extent=[800 * NM, 800 * NM],
                                resolution=10 * NM, boundary=fpe.boundary.reflecting, force=force)
        sims.append(sim)
        pdfs.append(fpe.gaussian_pdf(center=(-150 * NM, -150 * NM), width=30 * NM))
        sels.append(_select(nsteps))
        Fs.append(force(*sim.grid))
    res = fpe.propagate_many(sims, pdfs, tf, Nsteps=nsteps, device=device, select=sels)
    return dict(time=np.array([t for t, _ in res]), grid=np.array([s.grid for s in sims]),
                trajectories=np.array([p for _, p in res]), F=np.array(Fs))


def save_npz(path: str, data: dict) -> None:
    """np.savez with the reference's keys (dataset_1d_drift_diffusion.py:91-98)."""
    np.savez(path, **data)
