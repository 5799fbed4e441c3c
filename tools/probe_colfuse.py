#!/usr/bin/env python3
"""Where the heads' fused column pass spends its time: per-wave realtime stamps (100 MHz) at
the phase edges of colfuse_kernel, from a diagnostic build of the library:

    python tools/build_variant.py cfprobe spectral.hip -DCOLFUSE_PROBE=1
    BLINDNO_LIB=variants/cfprobe/libblindno.so python tools/probe_colfuse.py [Bn ...]

Prints, per head shape (C = 12, m = 32, 128^2 grid), the launch time from HIP events, the span
from the first wave's start to the last wave's end, and per phase the median / max over waves:
  entry: the index set-up (kernel arguments)
  0-1 column DFT (At + twiddle loads, MFMAs)   1-2 barrier      2-3 chunk sum, Xs, barrier
  3-4 the mix (weight loads, FMAs)             4-5 barrier      5-6 column inverse + Z stores
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "reconstruction-of-pde-without-time-label_amd"))

import torch  # noqa: E402

import blindno  # noqa: E402
from blindno import _lib, ops  # noqa: E402


def main():
    blindno.load_library()
    lib = _lib.load()
    rd = lib.blindno_colfuse_probe_read
    rd.argtypes = [ctypes.c_void_p, ctypes.c_int]
    rd.restype = ctypes.c_int
    dev = torch.device("cuda")
    torch.manual_seed(0)
    C, m, N = 12, 32, 128
    P = N + ops.pad_amount(N)
    for Bn in [int(a) for a in sys.argv[1:]] or [4, 8]:
        for direction in (0, 1):
            z = torch.randn(Bn, C, P, P, device=dev)
            w = torch.rand(C, C, m, m, 2, device=dev) / (C * C)
            Wt = ops.k_pack_w2d(w, w.clone(), P)
            At = ops.k_rowdft(z, Bn, C, P, P, m, 1)
            for _ in range(5):
                ops.k_colpass(At, Wt, Bn, C, C, P, m, m, P, direction)
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            ops.k_colpass(At, Wt, Bn, C, C, P, m, m, P, direction)
            e.record()
            torch.cuda.synchronize()
            us = s.elapsed_time(e) * 1e3
            nwg = Bn * m                      # one (sample, mode) pair per workgroup at C = 12
            nw = nwg * 8
            buf = np.zeros(nw * 8, dtype=np.uint64)
            assert rd(buf.ctypes.data, buf.size) == 0
            t = buf.reshape(nw, 8)[:, [7, 0, 1, 2, 3, 4, 5, 6]].astype(np.int64)
            t0 = t[:, 0].min()
            t = (t - t0) * 10.0 / 1000.0     # 100 MHz ticks -> us
            span = t[:, 7].max()
            ph = np.diff(t, axis=1)
            names = ["entry", "dft", "bar1", "sum+Xs", "mix", "bar2", "inv+st"]
            cells = " ".join(f"{n} {np.median(ph[:, i]):5.2f}/{ph[:, i].max():5.2f}" for i, n in enumerate(names))
            starts = t[:, 0]
            print(f"Bn={Bn:2d} dir={direction} event {us:6.1f} us  span {span:6.2f} us  start spread "
                  f"{starts.max():5.2f} us  wave life med {np.median(t[:, 7] - t[:, 0]):5.2f} us | {cells}",
                  flush=True)


if __name__ == "__main__":
    main()
