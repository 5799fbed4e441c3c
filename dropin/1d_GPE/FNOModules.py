"""Drop-in for the reference's 1d_GPE/FNOModules.py: the same names, backed by the MI355X HIP path
(set BLINDNO_PKG when copied elsewhere).  Put this directory ahead of the experiment directory on
sys.path (dropin/run.py), or copy this file over the reference's FNOModules.py."""
import os as _os
import sys as _sys

_PKG = _os.environ.get("BLINDNO_PKG") or _os.path.join(
    _os.path.dirname(_os.path.abspath(__file__)), "..", "..",
    "reconstruction-of-pde-without-time-label_amd")
if _PKG not in _sys.path:
    _sys.path.insert(0, _os.path.normpath(_PKG))

from blindno.dropin import install as _install  # noqa: E402

_install("1d_GPE", globals(), "FNOModules")
