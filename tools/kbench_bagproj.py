#!/usr/bin/env python3
"""bagproj_fwd (blindno_project_bag_fwd) time against its tile count: B = 4 bags of U = 52
snapshots on a 128-row crop of width Wo (16-point tiles = 4 * 128 * Wo / 16; config C: Wo = 128,
4096 tiles = 5.33 rounds of the 768 resident workgroups).  Checks whether the last partial round
costs a whole round (workgroup quantization).   python tools/kbench_bagproj.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "reconstruction-of-pde-without-time-label_amd"))

import torch  # noqa: E402

import blindno  # noqa: E402
from blindno._lib import call, ptr, query, stream_ptr  # noqa: E402


def main():
    blindno.load_library()
    dev = torch.device("cuda")
    B, U, C, P, Ho = 4, 52, 4, 160, 128
    z = torch.randn(B * U, C, P, P, device=dev)
    w1 = torch.randn(128, C, device=dev) * 0.3
    b1 = torch.randn(128, device=dev) * 0.1
    w2 = torch.randn(1, 128, device=dev) * 0.1
    b2 = torch.randn(1, device=dev)
    lw = torch.full((U,), 1.0 / U, device=dev)
    v = torch.empty_like(z)
    for Wo in (96, 108, 112, 120, 124, 128, 132, 136, 144):
        ubar = torch.empty(B, Ho * Wo, device=dev)
        stats = torch.empty(query("blindno_project_bag_stats_floats", B, Ho, Wo), device=dev)
        fn = lambda: call("blindno_project_bag_fwd", ptr(z), ptr(w1), ptr(b1), ptr(w2), ptr(b2), ptr(lw),  # noqa: E731
                          ptr(ubar), ptr(stats), ptr(v), B, U, C, P, P, Ho, Wo, 128, stream_ptr())
        for _ in range(3):
            fn()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record()
        for _ in range(10):
            fn()
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) * 100
        tiles = B * Ho * Wo // 16
        print(f"Wo {Wo:4d} tiles {tiles:5d} rounds {tiles / 768:5.2f}  {us:7.1f} us  {us / tiles * 1e3:6.1f} ns/tile",
              flush=True)


if __name__ == "__main__":
    main()
