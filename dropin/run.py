#!/usr/bin/env python3
"""Run an UNCHANGED reference script against the MI355X modules.

    python dropin/run.py 2d_FPE /path/to/reference/2d_FPE/train_fno.py [script args...]

The reference scripts import their models by bare module name from the script's own
directory (``from NIOModules import NIOFP2D_FNO``, 2d_FPE/train_fno.py:8), which Python puts
at sys.path[0].  This launcher runs the script as ``__main__`` from its directory (its
relative paths keep working) with ``dropin/<experiment>`` inserted AHEAD of that directory,
so ``NIOModules`` / ``FNOModules`` / ``DeepONetModules`` / ``Baselines`` resolve to the
drop-in shims.  Everything else the script imports (numpy, torch, accelerate) is untouched.
"""
from __future__ import annotations

import os
import runpy
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def main(argv):
    if len(argv) < 2:
        print(__doc__, file=sys.stderr)
        return 2
    exp, script, rest = argv[0], os.path.abspath(argv[1]), argv[2:]
    shim = os.path.join(HERE, exp)
    if not os.path.isdir(shim):
        print(f"unknown experiment {exp!r}; have {sorted(os.listdir(HERE))}", file=sys.stderr)
        return 2
    sdir = os.path.dirname(script)
    for name in ("NIOModules", "FNOModules", "DeepONetModules", "Baselines"):
        sys.modules.pop(name, None)
    sys.path[:0] = [shim, sdir]
    sys.argv = [script] + rest
    os.chdir(sdir)
    runpy.run_path(script, run_name="__main__")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
