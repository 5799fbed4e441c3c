"""Stand-in for the absent ``fplanck`` package imported by this experiment's scripts
(compute_time_error.py, dataset generators, cal_traj*.py): every name they import --
fokker_planck, boundary, gaussian_pdf, gaussian_potential, combine, potential_from_data --
with the propagation on the MI355X (blindno.fpe; parity unpinned).
Put this directory ahead of the experiment directory on sys.path (dropin/run.py)."""
import os as _os
import sys as _sys

_PKG = _os.environ.get("BLINDNO_PKG") or _os.path.join(
    _os.path.dirname(_os.path.abspath(__file__)), "..", "..",
    "reconstruction-of-pde-without-time-label_amd")
if _PKG not in _sys.path:
    _sys.path.insert(0, _os.path.normpath(_PKG))

from blindno.fpe import (boundary, combine, fokker_planck, gaussian_pdf,  # noqa: E402,F401
                         gaussian_potential, potential_from_data)

__all__ = ["boundary", "combine", "fokker_planck", "gaussian_pdf", "gaussian_potential",
           "potential_from_data"]
