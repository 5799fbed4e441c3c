"""CPU restatement of fplanck's master-equation FPE propagation (TEST INFRASTRUCTURE: only
tests/ may use it; it is the checker of blindno.fpe / blindno_fp_propagate, never the product).

PARITY UNPINNED: ``fplanck`` (PyPI, J. Parker; used by 1d_FPE/compute_time_error.py:8-12,
215-238 and 2d_Non_conservative_FPE/compute_time_error.py:44,266-319) is not installed or
vendored and no output of it exists here.  This restates its published method -- the
finite-volume master equation of Holubec, Kroy & Steffenoni, PRE 99, 032117 (2019) -- as an
explicit cell-by-cell sparse assembly (deliberately not the vectorised np.roll construction of
blindno.fpe) and propagates with scipy.sparse.linalg.expm_multiply, as fplanck's
``propagate_interval`` does:

  grid: N_d = ceil(extent_d / h_d) cell centres per axis, centred on 0;
  hop i -> j = i +- e_d at rate  (D_i + D_j) / 2 / h_d^2 * exp(-beta (U_j - U_i - W_ij) / 2),
        W_ij = +-h_d (F_d,i + F_d,j) / 2 (work of the force along the hop), D = k_B T / drag;
  reflecting walls: no hop across the boundary; periodic: hops wrap;
  M[j, i] = rate(i -> j), M[i, i] = -sum_j rate(i -> j);  p(t) = exp(M t) p0.
"""
from __future__ import annotations

import numpy as np

K_B = 1.380649e-23


def master_matrix(U, F, D, h, beta, periodic):
    """Sparse (CSC) M for potential U (shape S), force F (ndim, *S), diffusion D (S), cell
    widths h (ndim,), per-axis periodic flags."""
    import scipy.sparse as sp
    S = U.shape
    nd = len(S)
    N = int(np.prod(S))
    rows, cols, vals = [], [], []
    diag = np.zeros(N)
    for flat in range(N):
        idx = np.unravel_index(flat, S)
        for d in range(nd):
            for step in (1, -1):
                j = list(idx)
                j[d] += step
                if j[d] < 0 or j[d] >= S[d]:
                    if not periodic[d]:
                        continue
                    j[d] %= S[d]
                jt = tuple(j)
                W = step * h[d] * (F[d][idx] + F[d][jt]) / 2
                rate = (D[idx] + D[jt]) / 2 / h[d] ** 2 * np.exp(-beta * (U[jt] - U[idx] - W) / 2)
                jf = int(np.ravel_multi_index(jt, S))
                rows.append(jf)
                cols.append(flat)
                vals.append(rate)
                diag[flat] += rate
    rows += list(range(N))
    cols += list(range(N))
    vals += list(-diag)
    return sp.csc_matrix((vals, (rows, cols)), shape=(N, N))


def grid_axes(extent, resolution):
    extent = np.atleast_1d(np.asarray(extent, dtype=np.float64))
    h = np.broadcast_to(np.asarray(resolution, dtype=np.float64), extent.shape)
    axes = []
    for e, r in zip(extent, h):
        ax = np.arange(int(np.ceil(e / r))) * r
        axes.append(ax - ax.mean())
    return axes, np.array(h)


def propagate(M, p0, tf, nsteps):
    """exp(M t) p0 at t = linspace(0, tf, nsteps) (rows)."""
    from scipy.sparse.linalg import expm_multiply
    return expm_multiply(M, p0, start=0, stop=tf, num=nsteps, endpoint=True)
