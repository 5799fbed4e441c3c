"""Stand-in for the absent ``fplanck`` package imported by this experiment's
compute_time_error.py: the same names (fokker_planck, boundary, gaussian_pdf,
potential_from_data), with the propagation on the MI355X (blindno.fpe; parity unpinned,
DESIGN.md section 4c).  Put this directory ahead of the experiment directory on sys.path
(dropin/run.py)."""
import os as _os
import sys as _sys

_PKG = _os.environ.get("BLINDNO_PKG") or _os.path.join(
    _os.path.dirname(_os.path.abspath(__file__)), "..", "..",
    "reconstruction-of-pde-without-time-label_amd")
if _PKG not in _sys.path:
    _sys.path.insert(0, _os.path.normpath(_PKG))

from blindno.fpe import boundary, fokker_planck, gaussian_pdf, potential_from_data  # noqa: E402,F401

__all__ = ["boundary", "fokker_planck", "gaussian_pdf", "potential_from_data"]
