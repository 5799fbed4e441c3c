"""Fokker-Planck density propagation -- the ``fplanck`` API the reference's density-error
evaluators call, with the propagation on the GPU (§8f2).

Reference call sites: ``simulate_density_trajectory`` (1d_FPE/compute_time_error.py:215-238:
``fokker_planck(temperature, drag, extent, resolution, boundary, potential)``,
``gaussian_pdf``, ``propagate_interval(pdf, tf, Nsteps)``) and ``build_fokker_planck`` /
``propagate_density_with_force`` (2d_Non_conservative_FPE/compute_time_error.py:266-319: a
``force`` field built with ``potential_from_data``).

``fplanck`` (PyPI, J. Parker) is neither installed nor vendored, so this module restates its
published method -- the finite-volume master equation of Holubec, Kroy & Steffenoni (PRE 99,
032117, 2019): cells of width h on a centred grid of ceil(extent / resolution) points, hops to
each neighbour at rate  D_mid / h^2 * exp(-beta (dU - W) / 2)  with dU the potential step,
W = h (F_i + F_j) / 2 the work of the force over the hop, D = k_B T / drag; reflecting walls
remove the hops across the boundary, periodic ones wrap; ``propagate_interval`` evaluates
exp(M t) p0 at Nsteps equally spaced times in [0, tf] (scipy's expm_multiply there).  Parity
is UNPINNED (no fplanck output exists here); tests/test_fpe.py checks mass conservation, the
Boltzmann stationary state, detailed balance and the GPU integrator against
scipy.sparse.linalg.expm_multiply on the oracle's independently assembled matrix.

The rate construction (setup, O(N)) is host numpy; the propagation -- the hot part, N cells x
Nsteps x substeps x Taylor degree stencil passes -- is ``blindno_fp_propagate``, one
LDS-resident workgroup per trajectory, many trajectories per launch (``propagate_many``).
"""
from __future__ import annotations

import enum
import math
from typing import Callable, Optional, Sequence

import numpy as np
import torch

from ._lib import BlindnoError, call, ptr, stream_ptr

K_B = 1.380649e-23          # scipy.constants.k
TAYLOR_DEGREE = 18          # truncation (1/2)^19 / 19! ~ 1e-23 per substep at theta = 1/2
THETA = 0.5                 # bound on ||h M||_1 per substep


class boundary(enum.Enum):
    reflecting = enum.auto()
    periodic = enum.auto()


def gaussian_pdf(center, width):
    """A Gaussian bump exp(-((x - c) / w)^2) per axis (normalised by propagate_interval)."""
    center = np.atleast_1d(np.asarray(center, dtype=np.float64))
    width = np.broadcast_to(np.asarray(width, dtype=np.float64), center.shape)

    def pdf(*args):
        v = np.ones_like(np.asarray(args[0], dtype=np.float64))
        for i, a in enumerate(args):
            v = v * np.exp(-np.square((np.asarray(a) - center[i]) / width[i]))
        return v
    return pdf


def gaussian_potential(center, width, amplitude):
    """A Gaussian well -amplitude * exp(-((x - c) / w)^2) per axis (fplanck's helper used by
    1d_FPE/dataset_1d_drift_diffusion.py:45-49 and 2d_FPE/test_datagen.py:38-42)."""
    center = np.atleast_1d(np.asarray(center, dtype=np.float64))
    width = np.broadcast_to(np.asarray(width, dtype=np.float64), center.shape)

    def U(*args):
        v = np.ones_like(np.asarray(args[0], dtype=np.float64))
        for i, a in enumerate(args):
            v = v * np.exp(-np.square((np.asarray(a) - center[i]) / width[i]))
        return -amplitude * v
    return U


def combine(*funcs):
    """The sum of several potential / force callables (fplanck.combine)."""
    def f(*args):
        return sum(np.asarray(fn(*args), dtype=np.float64) for fn in funcs)
    return f


def potential_from_data(grid, data):
    """A callable interpolating ``data`` sampled on ``grid`` (an axis (N,) in 1D, or the
    simulator grid (ndim, *N)); evaluated on the same grid it returns ``data``."""
    from scipy.interpolate import RegularGridInterpolator
    data = np.asarray(data, dtype=np.float64)
    g = np.asarray(grid, dtype=np.float64)
    if data.ndim == 1:
        axes = (g.reshape(-1),)
    elif g.ndim == data.ndim + 1:                  # simulator grid (ndim, Nx, Ny)
        axes = (g[0][:, 0], g[1][0, :])
    else:                                          # a sequence of axes
        axes = tuple(np.asarray(a, dtype=np.float64) for a in grid)
    f = RegularGridInterpolator(axes, data, bounds_error=False, fill_value=None)

    def fn(*args):
        pts = np.stack([np.asarray(a, dtype=np.float64).reshape(-1) for a in args], -1)
        return f(pts).reshape(np.asarray(args[0]).shape)
    return fn


def _roll(a, shift, axis):
    return np.roll(a, shift, axis=axis)


class fokker_planck:
    """fplanck.fokker_planck (subset used by the reference): scalar / callable drag,
    potential and/or force callables, reflecting or periodic walls per axis."""

    def __init__(self, *, temperature, drag, extent, resolution, potential: Optional[Callable] = None,
                 force: Optional[Callable] = None, boundary=boundary.reflecting):
        self.extent = np.atleast_1d(np.asarray(extent, dtype=np.float64))
        self.ndim = self.extent.size
        if self.ndim not in (1, 2):
            raise BlindnoError("fokker_planck: 1D or 2D grids")
        self.resolution = np.broadcast_to(np.asarray(resolution, dtype=np.float64), (self.ndim,)).copy()
        self.temperature = float(temperature)
        self.beta = 1.0 / (K_B * self.temperature)
        bnd = boundary if isinstance(boundary, (list, tuple)) else [boundary] * self.ndim
        self.boundary = list(bnd)
        self.Ngrid = np.ceil(self.extent / self.resolution).astype(int)
        self.axes = []
        for i in range(self.ndim):
            ax = np.arange(self.Ngrid[i]) * self.resolution[i]
            self.axes.append(ax - np.average(ax))
        self.grid = np.array(np.meshgrid(*self.axes, indexing="ij"))
        shape = tuple(self.Ngrid)
        drag_v = drag(*self.grid) if callable(drag) else drag
        self.drag = np.broadcast_to(np.asarray(drag_v, dtype=np.float64), shape).copy()
        self.diffusion = K_B * self.temperature / self.drag
        self.potential_values = np.zeros(shape) if potential is None else \
            np.asarray(potential(*self.grid), dtype=np.float64).reshape(shape)
        if force is None:
            self.force_values = np.zeros((self.ndim,) + shape)
        else:
            self.force_values = np.asarray(force(*self.grid), dtype=np.float64).reshape((self.ndim,) + shape)
        self._build_rates()

    def _build_rates(self):
        U, F, D = self.potential_values, self.force_values, self.diffusion
        self.R, self.L = [], []
        for i in range(self.ndim):
            h = self.resolution[i]
            dU_r = _roll(U, -1, i) - U
            dU_l = _roll(U, 1, i) - U
            W_r = h * (F[i] + _roll(F[i], -1, i)) / 2
            W_l = -h * (F[i] + _roll(F[i], 1, i)) / 2
            D_r = (D + _roll(D, -1, i)) / 2
            D_l = (D + _roll(D, 1, i)) / 2
            R = D_r / h ** 2 * np.exp(-self.beta * (dU_r - W_r) / 2)
            Lr = D_l / h ** 2 * np.exp(-self.beta * (dU_l - W_l) / 2)
            if self.boundary[i] == boundary.reflecting:
                idx = [slice(None)] * self.ndim
                idx[i] = -1
                R[tuple(idx)] = 0.0
                idx[i] = 0
                Lr[tuple(idx)] = 0.0
            self.R.append(R)
            self.L.append(Lr)

    def coefficients(self) -> np.ndarray:
        """(5, N) float64 [diag, cxm, cxp, cym, cyp] of blindno_fp_propagate (in-rates)."""
        N = int(np.prod(self.Ngrid))
        c = np.zeros((5, N))
        diag = sum(self.R[i] + self.L[i] for i in range(self.ndim))
        c[0] = diag.reshape(-1)
        for i in range(self.ndim):
            c[1 + 2 * i] = _roll(self.R[i], 1, i).reshape(-1)     # from i - e, hopping right
            c[2 + 2 * i] = _roll(self.L[i], -1, i).reshape(-1)    # from i + e, hopping left
        return c

    def grid_dims(self):
        nx = int(self.Ngrid[0])
        ny = int(self.Ngrid[1]) if self.ndim == 2 else 1
        return nx, ny

    def propagate_interval(self, initial, tf, Nsteps=None, dt=None, normalize=True, device="cuda"):
        """(time (Nsteps,), Pt (Nsteps, *Ngrid)): exp(M t) p0 at t = linspace(0, tf, Nsteps)."""
        return propagate_many([self], [initial], tf, Nsteps=Nsteps, dt=dt, normalize=normalize,
                              device=device)[0]


# Upper bound on the Taylor substeps one launch may take in total (substeps per output interval
# x output intervals).  The step count grows like exp(beta W / 2) with the rates, so one badly
# predicted force could otherwise turn a launch into an effectively hung GPU job (or overflow
# the kernel's int argument); such a request is refused before launching.
MAX_TOTAL_SUBSTEPS = 1 << 24


def substeps_for(coef: np.ndarray, dt_out: float, theta: float = THETA) -> int:
    """Substeps per output interval so that ||h M||_1 <= theta (||M||_1 = 2 max diag) for the
    rate coefficients ``coef`` (5, N) of one trajectory (or a stack: the max over it)."""
    norm = 2.0 * float(np.max(coef[..., 0, :]))
    if not math.isfinite(norm):
        raise BlindnoError("fp propagation: non-finite hop rates (overflowing exp(-beta dU/2))")
    return max(1, int(math.ceil(norm * dt_out / theta)))


def propagate_many(sims: Sequence[fokker_planck], initials, tf, Nsteps=None, dt=None,
                   normalize=True, device="cuda", select=None):
    """propagate_interval of several simulators (same grid) in ONE launch: one workgroup per
    trajectory.  Returns [(time, Pt)] in the order given; ``select`` (per trajectory, a list of
    time indices) keeps only those records (gathered on the device before the host copy)."""
    if not sims:
        return []
    if Nsteps is None:
        Nsteps = int(np.ceil(tf / dt))
    Nsteps = int(Nsteps)
    nx, ny = sims[0].grid_dims()
    N = nx * ny
    p0 = np.zeros((len(sims), N))
    coef = np.zeros((len(sims), 5, N))
    for k, (sim, ini) in enumerate(zip(sims, initials)):
        if sim.grid_dims() != (nx, ny):
            raise BlindnoError("propagate_many: every simulator needs the same grid")
        v = np.asarray(ini(*sim.grid) if callable(ini) else ini, dtype=np.float64).reshape(-1)
        if normalize:
            v = v / np.sum(v)
        p0[k] = v
        coef[k] = sim.coefficients()
    time = np.linspace(0, tf, Nsteps)
    dt_out = tf / (Nsteps - 1) if Nsteps > 1 else 0.0
    # substeps per trajectory: one stiff trajectory must not multiply every other one's work, so
    # trajectories are launched in groups of equal substep count
    steps = [substeps_for(coef[k], dt_out) if dt_out > 0 else 1 for k in range(len(sims))]
    worst = max(steps)
    if worst * max(1, Nsteps - 1) > MAX_TOTAL_SUBSTEPS:
        k = int(np.argmax(steps))
        raise BlindnoError(
            f"fp propagation: trajectory {k} needs {worst} Taylor substeps per output interval "
            f"({worst * (Nsteps - 1)} in total, limit {MAX_TOTAL_SUBSTEPS}); its hop rates reach "
            f"{float(np.max(coef[k, 0])):.3e}/s -- a force / potential far outside the physical "
            f"range (e.g. a badly predicted field); refusing to launch")
    dev = torch.device(device)
    if dev.type != "cuda":
        raise BlindnoError("fp propagation runs on a HIP device (there is no CPU path)")
    out = torch.empty(len(sims), Nsteps, N, dtype=torch.float64, device=dev)
    for s in sorted(set(steps)):
        ks = [k for k in range(len(sims)) if steps[k] == s]
        p0_d = torch.from_numpy(np.ascontiguousarray(p0[ks])).to(dev)
        coef_d = torch.from_numpy(np.ascontiguousarray(coef[ks])).to(dev)
        dst = out if len(ks) == len(sims) else torch.empty(len(ks), Nsteps, N, dtype=torch.float64, device=dev)
        call("blindno_fp_propagate", ptr(p0_d), ptr(coef_d), ptr(dst), len(ks), nx, ny, Nsteps, s,
             TAYLOR_DEGREE, float(dt_out), stream_ptr(dev))
        if dst is not out:
            out[torch.as_tensor(ks, device=dev)] = dst
    grid_shape = tuple(int(n) for n in sims[0].Ngrid)
    if select is not None:
        res = []
        for k in range(len(sims)):
            sel = np.asarray(select[k], dtype=np.int64)
            rec = out[k].index_select(0, torch.from_numpy(sel).to(dev)).cpu().numpy()
            res.append((time[sel], rec.reshape((len(sel),) + grid_shape)))
        return res
    res = out.cpu().numpy()
    return [(time, res[k].reshape((Nsteps,) + grid_shape)) for k in range(len(sims))]
