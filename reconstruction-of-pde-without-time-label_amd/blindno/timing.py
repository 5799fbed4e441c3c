"""Live per-kernel timing with HIP events for bench.py's roofline object.

A KernelTimer hooks every launch of one C-ABI entry point, records a pair of HIP
events on the launch stream around it, and accumulates the ALGORITHMIC bytes and flops
of that launch (the minimum traffic/work the math requires, from the launch's shape
arguments -- see DESIGN.md, "Roofline accounting").
"""
from __future__ import annotations

import os

import torch

from . import _lib

GELU_FLOPS = 20          # flop-equivalents charged per exact-erf GELU evaluation
DOMINANT = os.environ.get("BLINDNO_TIMED_KERNEL", "blindno_project_bwd")


def _i(args, k):
    return int(args[k])


def _present(a):
    return a is not None and getattr(a, "value", a) is not None


def cost(name, args):
    """(bytes, flops) of one launch of ``name`` with C-ABI arguments ``args``."""
    if name == "blindno_rowdft":
        Bn, C, P1, P2, m2 = (_i(args, k) for k in range(3, 8))
        return 4 * Bn * C * P1 * P2 + 8 * Bn * m2 * C * P1, 4 * Bn * C * P1 * P2 * m2
    if name == "blindno_rowidft_epi":
        has_wc = _present(args[2])
        Bn, C, P1, P2, m2 = (_i(args, k) for k in range(6, 11))
        pts = Bn * C * P1 * P2
        return 8 * Bn * C * P1 * m2 + 4 * pts * (2 if has_wc else 1), pts * (4 * m2 + (2 * C if has_wc else 0))
    if name == "blindno_rowidft_bwd":
        has_wc, act = _present(args[2]), _i(args, 11)
        Bn, C, P1, P2, m2 = (_i(args, k) for k in range(6, 11))
        pts = Bn * C * P1 * P2
        return (8 * Bn * C * P1 * m2 + 4 * pts * (2 + int(has_wc) + int(act > 0)),
                pts * (4 * m2 + (2 * C if has_wc else 0)))
    if name == "blindno_project_fwd":
        Bn, C, P1, P2, Ho, Wo, Hd, Cout = (_i(args, k) for k in range(6, 14))
        pts = Bn * Ho * Wo
        return 4 * pts * (C + Cout), pts * Hd * (2 * C + 2 * Cout + GELU_FLOPS)
    if name == "blindno_project_bwd":
        Bn, C, P1, P2, Ho, Wo, Hd, Cout = (_i(args, k) for k in range(8, 16))
        pts = Bn * Ho * Wo
        # recompute h (2C) + GELU/GELU' + dh (2 Cout) + dz (2C) + weight grads (2C + 2 Cout + 1)
        return 4 * pts * (2 * C + Cout), pts * Hd * (6 * C + 4 * Cout + 1 + 2 * GELU_FLOPS)
    if name == "blindno_conv_wgrad":
        nchunk, Bn, C, P1, P2 = (_i(args, k) for k in range(3, 8))
        pts = Bn * P1 * P2
        return 8 * C * pts, 2 * pts * (C * C + C)
    return 0, 0


class KernelTimer:
    def __init__(self, name: str = DOMINANT):
        self.name = name
        self.events = []
        self.bytes = 0
        self.flops = 0
        self._pending = None

    def before(self, args):
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        self._pending = ev

    def after(self, args):
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        self.events.append((self._pending, ev))
        b, f = cost(self.name, args)
        self.bytes += b
        self.flops += f

    def start(self):
        _lib._HOOKS[self.name] = self

    def stop(self):
        _lib._HOOKS.pop(self.name, None)
        torch.cuda.synchronize()

    def roofline(self, hbm_peak_gbs: float, flop_peak_tflops: float, bound: str = None):
        n = len(self.events)
        if n == 0:
            return None
        ms = sum(a.elapsed_time(b) for a, b in self.events) / n
        bytes_per = self.bytes / n
        flops_per = self.flops / n
        gbs = bytes_per / (ms * 1e-3) / 1e9
        tfs = flops_per / (ms * 1e-3) / 1e12
        if bound is None:
            # the roof the kernel's arithmetic intensity puts it under
            ridge = flop_peak_tflops * 1e12 / (hbm_peak_gbs * 1e9)
            bound = "mfma" if flops_per / max(1.0, bytes_per) > ridge else "hbm"
        if bound == "hbm":
            return {"kernel": self.name, "bound": "hbm", "achieved": round(gbs, 2), "peak": hbm_peak_gbs,
                    "unit": "GB/s", "frac": round(gbs / hbm_peak_gbs, 4), "traffic": None,
                    "launches": n, "avg_ms": round(ms, 5), "algorithmic_bytes_per_launch": int(bytes_per)}
        return {"kernel": self.name, "bound": "mfma", "achieved": round(tfs, 3), "peak": flop_peak_tflops,
                "unit": "TFLOP/s", "frac": round(tfs / flop_peak_tflops, 4), "traffic": None,
                "launches": n, "avg_ms": round(ms, 5), "algorithmic_flops_per_launch": int(flops_per),
                "algorithmic_bytes_per_launch": int(bytes_per)}
