#!/usr/bin/env python3
"""Per-layer timing of config D's snapshot CNN (Encoder2D at 128^2, Bn = 300 snapshots): each
ConvBlock's convolution forward, input gradient and weight gradient (C ABI, HIP events), with
the FMA-only TFLOP/s of each launch.  python tools/kbench_conv.py [Bn] [layer-regex] [mode-regex]"""
import re
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "reconstruction-of-pde-without-time-label_amd"))

import torch  # noqa: E402

import blindno  # noqa: E402
from blindno._lib import call, ptr, query, stream_ptr  # noqa: E402

LAYERS = [  # name, Ci, Co, (KH, KW), (sh, sw), (ph, pw)
    ("cb1", 1, 64, (1, 7), (1, 2), (0, 3)), ("cb2_1", 64, 128, (3, 3), (2, 2), (1, 1)),
    ("cb2_2", 128, 128, (3, 3), (1, 1), (1, 1)), ("cb3_1", 128, 256, (3, 3), (2, 2), (1, 1)),
    ("cb3_2", 256, 256, (3, 3), (1, 1), (1, 1)), ("cb4_1", 256, 512, (3, 3), (2, 2), (1, 1)),
    ("cb4_2", 512, 512, (3, 3), (1, 1), (1, 1)), ("cb7_1", 512, 512, (3, 3), (2, 2), (1, 1)),
    ("cb7_2", 512, 512, (3, 3), (2, 2), (1, 1)), ("cb7_3", 512, 512, (4, 2), (1, 1), (0, 0)),
]


def timeit(fn, iters=5):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


def main():
    Bn = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    lpat = sys.argv[2] if len(sys.argv) > 2 else ""
    mpat = sys.argv[3] if len(sys.argv) > 3 else ""
    lib = blindno.load_library()
    split = hasattr(lib, "blindno_conv2d_wscratch_floats")   # older libraries: the plain entries
    H, W = 128, 128
    tot_t = tot_f = 0.0
    for name, Ci, Co, (KH, KW), (sh, sw), (ph, pw) in LAYERS:
        Ho, Wo = (H + 2 * ph - KH) // sh + 1, (W + 2 * pw - KW) // sw + 1
        if lpat and not re.fullmatch(lpat, name):
            H, W = Ho, Wo
            continue
        x = torch.randn(Bn, Ci, H, W, device="cuda")
        w = torch.randn(Co, Ci, KH, KW, device="cuda") * 0.05
        b = torch.randn(Co, device="cuda")
        y = torch.empty(Bn, Co, Ho, Wo, device="cuda")
        dy = torch.randn_like(y)
        dx = torch.empty_like(x)
        g = (Bn, Ci, H, W, Co, KH, KW, sh, sw, ph, pw)
        ns = query("blindno_conv2d_wgrad_nsplit", *g)
        dwb = torch.empty(Co, Ci * KH * KW + 1, device="cuda")
        part = torch.empty(max(ns, 1), Co * (Ci * KH * KW + 1), device="cuda")
        fl = 2.0 * Bn * Co * Ho * Wo * Ci * KH * KW
        row = [name]
        if name == "cb1":
            row[0] += " (dx unused in the step)"
        if split:   # split-K forms with the library's default split counts
            nf, nd = query("blindno_conv2d_fwd_nsplit", *g), query("blindno_conv2d_bwd_data_nsplit", *g)
            pf = torch.empty(nf, y.numel(), device="cuda")
            pd = torch.empty(nd, dx.numel(), device="cuda")
            wsf = torch.empty(max(1, query("blindno_conv2d_wscratch_floats", 0, *g)), device="cuda")
            wsd = torch.empty(max(1, query("blindno_conv2d_wscratch_floats", 1, *g)), device="cuda")
            fwd = lambda: call("blindno_conv2d_fwd_split", ptr(x), ptr(w), ptr(b), ptr(y), ptr(pf), nf,  # noqa: E731
                               ptr(wsf), *g, stream_ptr())
            bwd = lambda: call("blindno_conv2d_bwd_data_split", ptr(dy), ptr(w), ptr(dx), ptr(pd), nd,  # noqa: E731
                               ptr(wsd), *g, stream_ptr())
            row[0] += f" [{nf},{nd}]"
        else:
            fwd = lambda: call("blindno_conv2d_fwd", ptr(x), ptr(w), ptr(b), ptr(y), *g, stream_ptr())  # noqa: E731
            bwd = lambda: call("blindno_conv2d_bwd_data", ptr(dy), ptr(w), ptr(dx), *g, stream_ptr())  # noqa: E731
        for kind, fn in (("fwd", fwd), ("bwd_data", bwd),
                         ("bwd_w", lambda: call("blindno_conv2d_bwd_weight", ptr(dy), ptr(x), ptr(dwb), ptr(part), ns, *g,
                                                stream_ptr()))):
            if mpat and not re.fullmatch(mpat, kind):
                continue
            us = timeit(fn)
            tot_t += us
            tot_f += fl
            row.append(f"{kind} {us:8.1f} us {fl / us / 1e6:6.1f} TF/s")
        print("  ".join(row), flush=True)
        H, W = Ho, Wo
    print(f"total {tot_t / 1e3:.2f} ms  {tot_f / tot_t / 1e6:.1f} TF/s (FMA-only, fp32 peak 157.3)")


if __name__ == "__main__":
    main()
