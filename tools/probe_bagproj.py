#!/usr/bin/env python3
"""Where bagproj_fwd's launch goes: per-wave realtime stamps (100 MHz) at the phase edges of the
kernel, and the hardware slot each wave ran on, from a diagnostic build:

    python tools/build_variant.py bpprobe bagproj.hip -DBAGPROJ_PROBE=1
    BLINDNO_LIB=variants/bpprobe/libblindno.so python tools/probe_bagproj.py [U ...]

Config C's shape: 4 bags x U distinct snapshots, 128^2 crop (P = 160), width 4: 4096 one-tile
workgroups.  Phases: setup (weights, lw, sum_l lw), first (the first chunk staged), loop (the
snapshot chunks), stats (statistics + ubar).  Then the launch as a whole: workgroups live over
time, the workgroups per CU, the gap a CU slot stays empty between two workgroups, and the tail.
"""
import ctypes
import os
import sys
from collections import defaultdict

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "reconstruction-of-pde-without-time-label_amd"))

import torch  # noqa: E402

import blindno  # noqa: E402
from blindno import _lib, ops  # noqa: E402
from blindno._lib import call, ptr, query, stream_ptr  # noqa: E402


def main():
    blindno.load_library()
    lib = _lib.load()
    rd = lib.blindno_bagproj_probe_read
    rd.argtypes = [ctypes.c_void_p, ctypes.c_int]
    rd.restype = ctypes.c_int
    dev = torch.device("cuda")
    torch.manual_seed(0)
    N, C, Bb = 128, 4, 4
    P = N + ops.pad_amount(N)
    for U in [int(a) for a in sys.argv[1:]] or [52]:
        z = torch.randn(Bb * U, C, P, P, device=dev)
        w1 = torch.randn(128, C, device=dev) * 0.3
        b1 = torch.randn(128, device=dev) * 0.1
        w2 = torch.randn(1, 128, device=dev) * 0.1
        b2 = torch.randn(1, device=dev)
        lw = torch.full((U,), 1.0 / U, device=dev)
        ubar = torch.empty(Bb, N * N, device=dev)
        stats = torch.empty(query("blindno_project_bag_stats_floats", Bb, N, N), device=dev)
        vv = torch.empty_like(z)

        def run():
            call("blindno_project_bag_fwd", ptr(z), ptr(w1), ptr(b1), ptr(w2), ptr(b2), ptr(lw), ptr(ubar),
                 ptr(stats), ptr(vv), Bb, U, C, P, P, N, N, 128, stream_ptr())
        for _ in range(5):
            run()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        run()
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) * 1e3
        nwg = Bb * N * N // 16
        buf = np.zeros(nwg * 4 * 8, dtype=np.uint64)
        assert rd(buf.ctypes.data, buf.size) == 0
        r = buf.reshape(nwg, 4, 8)
        t = r[:, :, :5].astype(np.int64)
        t0 = t[:, :, 0].min()
        t = (t - t0) * 0.01                       # us
        ph = np.diff(t, axis=2)
        names = ["setup", "first", "loop", "stats"]
        cells = " ".join(f"{n} {np.median(ph[:, :, i]):6.2f}/{np.percentile(ph[:, :, i], 90):6.2f}"
                         for i, n in enumerate(names))
        print(f"U={U} event {us:7.1f} us  span {t[:, :, 4].max():7.2f} us | per wave median/p90: {cells}")
        wg_start = t[:, :, 0].min(axis=1)
        wg_end = t[:, :, 4].max(axis=1)
        life = wg_end - wg_start
        print(f"  workgroup life median {np.median(life):6.2f} us p10 {np.percentile(life, 10):6.2f} "
              f"p90 {np.percentile(life, 90):6.2f}; last start {wg_start.max():7.2f} us; first end "
              f"{wg_end.min():7.2f} us")
        hw = r[:, 0, 5].astype(np.int64)
        xcc = r[:, 0, 6].astype(np.int64) & 0xF
        cu = (hw >> 8) & 0xF
        sh = (hw >> 12) & 1
        se = (hw >> 13) & 0x7
        key = xcc * 1000 + se * 100 + sh * 20 + cu
        per = defaultdict(list)
        for i in range(nwg):
            per[int(key[i])].append((wg_start[i], wg_end[i]))
        counts = np.array([len(v) for v in per.values()])
        gaps, busy_end = [], []
        for v in per.values():
            v.sort()
            ends = []
            for (a, b) in v:
                # the slot this workgroup took: the earliest end before its start
                prior = [x for x in ends if x <= a + 1e-9]
                if prior:
                    m = max(prior)
                    gaps.append(a - m)
                    ends.remove(m)
                ends.append(b)
            busy_end.append(max(b for _, b in v))
        gaps = np.array(gaps) if gaps else np.zeros(1)
        print(f"  CUs {len(per)}; workgroups per CU min {counts.min()} median {int(np.median(counts))} max "
              f"{counts.max()}; slot refill gap median {np.median(gaps):5.2f} us p90 "
              f"{np.percentile(gaps, 90):5.2f} us; CU finish spread {np.min(busy_end):7.2f}..{np.max(busy_end):7.2f} us")
        hist = np.histogram(wg_start, bins=12, range=(0, t[:, :, 4].max()))[0]
        print("  workgroup starts per 1/12 of the span:", " ".join(str(x) for x in hist))
        live = [int(((wg_start <= x) & (wg_end > x)).sum()) for x in np.linspace(0, t[:, :, 4].max(), 13)[:-1]]
        print("  workgroups live at 0, 1/12, ..:", " ".join(str(x) for x in live), flush=True)


if __name__ == "__main__":
    main()
