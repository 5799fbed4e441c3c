"""CPU oracle for the BlinDNO FNO/NIO hot path -- TEST INFRASTRUCTURE ONLY.

This package restates, from scratch and in float64 on the CPU, the numerics of
the reference's hot path (yl602019618/Reconstruction-of-PDE-without-Time-Label):
truncated spectral convolutions, the FNO bodies, the snapshot-bag models, the
losses/metrics and the density-error reductions.  Every function cites the
reference file:line it follows.

Rules ("Oracle"):
  * Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
    ``cpu_baseline`` leg may import this package -- as the CHECKER or as the
    timed CPU baseline, never as part of the product path.
  * The product path (``blindno`` package) never imports ``oracle``; it fails
    loudly when the HIP library is missing.

Parity pinning: the oracle is checked against golden vectors captured by
importing the reference itself in the build container
(``tests/golden/make_golden.py`` -> ``tests/golden/*.npz``), see
``tests/test_oracle_golden.py``.
"""
from .fno_ref import *  # noqa: F401,F403
from . import gpe_ref  # noqa: F401,E402
from . import unet_ref  # noqa: F401,E402
