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

# Flop accounting: one FMA = 2 flops, adds/multiplies 1; the exact-erf GELU and
# its derivative (rcp + exp + polynomial, VALU-issue work) are NOT charged as flops -- the
# projection kernels are VALU-issue-bound on exactly that work, so their flop fraction is the
# fraction of the fp32 peak spent on the layer's matrix arithmetic, nothing more.
GELU_FLOPS = 0
# the snapshot encoder's bag-level projection forward (csrc/bagproj.hip): the largest kernel of a
# config-C step (the per-snapshot projection backward, blindno_project_bwd[_w], before it)
DOMINANT = os.environ.get("BLINDNO_TIMED_KERNEL", "blindno_project_bag_fwd")
_VARIANTS = {"blindno_project_bwd": ("blindno_project_bwd", "blindno_project_bwd_w"),
             # config D's snapshot CNN: every implicit-GEMM convolution of a step (forward, input
             # gradient, weight gradient; csrc/conv.hip), reported as one family
             # (the split-K forms time the partial sums' reduction with their GEMM)
             "blindno_conv2d": ("blindno_conv2d_fwd", "blindno_conv2d_bwd_data", "blindno_conv2d_bwd_weight",
                                "blindno_conv2d_fwd_split", "blindno_conv2d_bwd_data_split")}
_CONV_ARG0 = {"blindno_conv2d_fwd": 4, "blindno_conv2d_bwd_data": 3, "blindno_conv2d_bwd_weight": 5,
              "blindno_conv2d_fwd_split": 7, "blindno_conv2d_bwd_data_split": 6}
# families whose roofline aggregates every launch (sum of flops / sum of time)
_FAMILIES = ("blindno_conv2d",)


def _conv_out(n, k, s, p):
    return (n + 2 * p - k) // s + 1


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
        # fc1 (2C) + fc2 (2 Cout) per hidden unit
        return 4 * pts * (C + Cout), pts * Hd * (2 * C + 2 * Cout + GELU_FLOPS)
    if name in ("blindno_project_bwd", "blindno_project_bwd_w"):
        o = 8 if name == "blindno_project_bwd" else 9
        Bn, C, P1, P2, Ho, Wo, Hd, Cout = (_i(args, k) for k in range(o, o + 8))
        dout_div = _i(args, o + 10)
        pts = Bn * Ho * Wo
        # read z, write dz (crop), read dout (one value per bag and point when dout_div = L);
        # per hidden unit: recompute h (2C), dh = W2^T g (2 Cout), dz (2C), dW1 (2C), db1 (1),
        # dW2 (2 Cout); GELU / GELU' uncharged
        return (8 * pts * C + 4 * (pts // max(1, dout_div)) * Cout,
                pts * Hd * (6 * C + 4 * Cout + 1 + 2 * GELU_FLOPS))
    if name == "blindno_project_bag_fwd":
        B, U, C, P1, P2, Ho, Wo, Hd = (_i(args, k) for k in range(9, 17))
        pts, bpts = B * U * Ho * Wo, B * Ho * Wo
        # read z, write v (crop), write the statistics (16 floats x 768 per 16-point tile) and
        # ubar; per snapshot point and hidden unit: fc1 (2C), lw GELU into A (2), lw GELU' into
        # S (2), GELU' z into Q (2C), (w2 W1) GELU' into v (2C); GELU / GELU' uncharged
        return (8 * pts * C + 4 * ((bpts + 15) // 16) * 16 * Hd * 6 + 4 * bpts,
                pts * Hd * (6 * C + 4 + 2 * GELU_FLOPS))
    if name == "blindno_project_bag_bwd":
        B, U, C, P1, P2, Ho, Wo, Hd = (_i(args, k) for k in range(8, 16))
        pts, bpts = B * U * Ho * Wo, B * Ho * Wo
        return 8 * pts * C + 4 * ((bpts + 15) // 16) * 16 * Hd * 6 + 4 * bpts, 2 * bpts * Hd * 6
    if name in _CONV_ARG0:
        o = _CONV_ARG0[name]
        N, Ci, Hi, Wi, Co, KH, KW, sh, sw, ph, pw = (_i(args, k) for k in range(o, o + 11))
        Ho, Wo = _conv_out(Hi, KH, sh, ph), _conv_out(Wi, KW, sw, pw)
        K = Ci * KH * KW + (1 if name == "blindno_conv2d_bwd_weight" else 0)   # + the bias column
        # FMA-only flops of the GEMM (the adjoint's FMAs equal the forward's); bytes: the
        # operands and the result once each
        flops = 2 * N * Co * Ho * Wo * K
        nbytes = 4 * (N * Ci * Hi * Wi + N * Co * Ho * Wo + Co * K)
        return nbytes, flops
    if name == "blindno_conv_wgrad":
        nchunk, Bn, C, P1, P2 = (_i(args, k) for k in range(3, 8))
        pts = Bn * P1 * P2
        return 8 * C * pts, 2 * pts * (C * C + C)
    return 0, 0


def pmc_record(root: str, name: str):
    """The profiles/pmc_traffic.json record of ``name`` (tools/pmc_traffic.py), or None."""
    import json
    p = os.path.join(root, "profiles", "pmc_traffic.json")
    if not os.path.exists(p):
        return None
    return json.load(open(p)).get(name)


def pmc_traffic(root: str, name: str):
    """HBM bytes per crop point of ``name`` measured with rocprofv3 PMC counters
    (profiles/pmc_traffic.json, written by tools/pmc_traffic.py from FETCH_SIZE x 2 + WRITE_SIZE,
    the gfx950 correction of MI355X_MICROARCH.md), or None."""
    import json
    p = os.path.join(root, "profiles", "pmc_traffic.json")
    if not os.path.exists(p):
        return None
    d = json.load(open(p)).get(name)
    return None if d is None else float(d["bytes_per_point"])


def points(name, args):
    if name == "blindno_project_bag_fwd":
        return _i(args, 9) * _i(args, 10) * _i(args, 14) * _i(args, 15)
    if name in ("blindno_project_bwd", "blindno_project_bwd_w", "blindno_project_fwd"):
        o = {"blindno_project_bwd": 8, "blindno_project_bwd_w": 9, "blindno_project_fwd": 6}[name]
        Bn, Ho, Wo = _i(args, o), _i(args, o + 4), _i(args, o + 5)
        return Bn * Ho * Wo
    return 0


class KernelTimer:
    """Times every launch of one entry point; ``roofline`` reports the launches of the
    dominant shape (those within 4x of the largest algorithmic byte count: the snapshot
    encoder's launches, not the 4-sample head layers')."""

    def __init__(self, name: str = DOMINANT):
        self.name = name
        self.entries = _VARIANTS.get(name, (name,))
        self.recs = []            # (ev0, ev1, bytes, flops, points)
        self._pending = None

    class _Hook:
        def __init__(self, timer, entry):
            self.timer, self.entry = timer, entry

        def before(self, args):
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            self.timer._pending = ev

        def after(self, args):
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            b, f = cost(self.entry, args)
            self.timer.recs.append((self.timer._pending, ev, b, f, points(self.entry, args)))

    def start(self):
        for e in self.entries:
            _lib._HOOKS[e] = KernelTimer._Hook(self, e)

    def stop(self):
        for e in self.entries:
            _lib._HOOKS.pop(e, None)
        torch.cuda.synchronize()

    def roofline(self, hbm_peak_gbs: float, flop_peak_tflops: float, bound: str = None,
                 traffic_per_point=None):
        if not self.recs:
            return None
        if self.name in _FAMILIES:
            sel = self.recs                        # every launch of the family
        else:
            bmax = max(r[2] for r in self.recs)
            sel = [r for r in self.recs if 4 * r[2] >= bmax]
        n = len(sel)
        ms = sum(a.elapsed_time(b) for a, b, *_ in sel) / n
        bytes_per = sum(r[2] for r in sel) / n
        flops_per = sum(r[3] for r in sel) / n
        pts_per = sum(r[4] for r in sel) / n
        traffic = int(traffic_per_point * pts_per) if traffic_per_point and pts_per else None
        gbs = bytes_per / (ms * 1e-3) / 1e9
        tfs = flops_per / (ms * 1e-3) / 1e12
        if bound is None:
            # the roof the kernel's arithmetic intensity puts it under
            ridge = flop_peak_tflops * 1e12 / (hbm_peak_gbs * 1e9)
            bound = "mfma" if flops_per / max(1.0, bytes_per) > ridge else "hbm"
        fam = ({"family": list(self.entries), "aggregate": "sum of flops / sum of launch times"}
               if self.name in _FAMILIES else {})
        if bound == "hbm":
            return {"kernel": self.name, "bound": "hbm", "achieved": round(gbs, 2), "peak": hbm_peak_gbs,
                    "unit": "GB/s", "frac": round(gbs / hbm_peak_gbs, 4), "traffic": traffic,
                    "launches": n, "avg_ms": round(ms, 5), "algorithmic_bytes_per_launch": int(bytes_per),
                    **fam}
        note = ("FMA-only flops of the implicit GEMMs (one FMA = 2); fp32 operands on the fp32 matrix "
                "cores (the NIO path's Linear layers run as 1x1 convolutions and are in the family)"
                if self.name in _FAMILIES else
                "FMA-only flops (one FMA = 2; exact-erf GELU / GELU' evaluation not charged); the measured "
                "limiter is fp32 VALU issue on that GELU work (valu_issue_util); gfx950 fp32 vector peak = "
                "fp32 MFMA peak = 157.3 TFLOP/s")
        return {"kernel": self.name, "bound": bound, "achieved": round(tfs, 3), "peak": flop_peak_tflops,
                "unit": "TFLOP/s", "frac": round(tfs / flop_peak_tflops, 4), "traffic": traffic,
                "launches": n, "avg_ms": round(ms, 5), "algorithmic_flops_per_launch": int(flops_per),
                "algorithmic_bytes_per_launch": int(bytes_per), "note": note, **fam}
