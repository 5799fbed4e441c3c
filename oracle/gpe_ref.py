"""Float64 CPU restatement of the reference's 1D GPE split-step solver (TEST INFRASTRUCTURE).

Reference: 1d_GPE/datagen_GPE.py:7-115 (identical copy in 1d_GPE/compute_time_error_GPE.py:
96-160).  Written from its behaviour with an explicit O(N^2) DFT instead of an FFT library, so
agreement with the reference's numpy.fft is an independent check.  Pinned by
tests/golden/gpe_solve_*.npz and gpe_datagen.npz (tests/test_oracle_golden.py).
"""
from __future__ import annotations

import numpy as np

YOSHIDA_C = 2.0 - 2.0 ** (1.0 / 3.0)


def initial_condition(ic: int, x: np.ndarray) -> np.ndarray:
    """get_initial_condition, datagen_GPE.py:7-21."""
    if ic == 1:
        return np.exp(-x ** 2 / 10)
    if ic == 2:
        return 2 * np.sin(x) / (np.exp(x) + np.exp(-x))
    if ic == 3:
        return 2 * np.cos(x) / (np.exp(x) + np.exp(-x))
    raise ValueError("ic must be 1, 2 or 3")


def wavenumbers(n: int, dx: float) -> np.ndarray:
    """2 pi fftfreq(n, dx) (datagen_GPE.py:99)."""
    j = np.arange(n)
    f = np.where(j < (n + 1) // 2, j, j - n)
    return 2 * np.pi * f / (n * dx)


def _dft_mats(n: int):
    j = np.arange(n)
    ph = (np.outer(j, j) % n) * (2 * np.pi / n)
    fwd = np.exp(-1j * ph)
    return fwd, np.conj(fwd) / n


def _nonlinear(psi, h, V, g, kappa):
    a = np.abs(psi)
    return np.exp(-1j * h * (V + g * a * a + kappa * a ** 4)) * psi


def _linear(psi, h, k, mats):
    fwd, inv = mats
    return inv @ (np.exp(-1j * h * 0.5 * k * k) * (fwd @ psi))


def step(psi, dt, k, V, g, kappa, order, mats):
    """step_strang (:44-51) / step_fourth_order (:53-81)."""
    if order == 2:
        psi = _nonlinear(psi, dt / 2, V, g, kappa)
        psi = _linear(psi, dt, k, mats)
        return _nonlinear(psi, dt / 2, V, g, kappa)
    if order == 4:
        a1 = 1.0 / YOSHIDA_C
        a2 = -(2 ** (1 / 3)) / YOSHIDA_C
        b1, b2 = a1, a2
        for kind, c in (("n", b1), ("l", a1), ("n", b2), ("l", a2), ("n", b1), ("l", a2),
                        ("n", b2), ("l", a1), ("n", b1)):
            psi = _nonlinear(psi, c * dt, V, g, kappa) if kind == "n" else _linear(psi, c * dt, k, mats)
        return psi
    raise ValueError("order must be 2 or 4")


def solve(psi0, x, dt, t_final, order, g, kappa, V):
    """solve_GPE_custom (:86-115): returns (t, psi_record (Nt, Nx) complex128)."""
    x = np.asarray(x, dtype=np.float64)
    n = len(x)
    k = wavenumbers(n, x[1] - x[0])
    nt = int(t_final / dt) + 1
    t = np.linspace(0, t_final, nt)
    mats = _dft_mats(n)
    psi = np.asarray(psi0, dtype=np.complex128)
    rec = np.zeros((nt, n), dtype=np.complex128)
    rec[0] = psi
    for i in range(1, nt):
        psi = step(psi, dt, k, V, g, kappa, order, mats)
        rec[i] = psi
    return t, rec


def training_potentials(num_orbits: int, x: np.ndarray, nt: int, num_time_samples: int = 100,
                        rng=np.random):
    """The random draws of generate_and_save_training_data (:120-191), consumed in the
    reference's order (a, b, c, x0, then the unused time-sample choice) -> V (M, Nx)."""
    Vs = []
    for _ in range(num_orbits):
        a = rng.uniform(0.1, 0.3)
        b = rng.uniform(0.5, 2)
        c = rng.uniform(0.5, 2)
        x0 = rng.uniform(-3, 3)
        Vs.append(a * (x - x0) ** 2 + b * (np.cos(c * (x - x0))) ** 2)
        rng.choice(np.arange(nt), size=num_time_samples, replace=False)
    return np.stack(Vs, 0)
