#!/usr/bin/env python3
"""Kernel micro-benchmarks at config-C shapes (HIP events on the launch stream).

    python tools/kbench.py [filter-regex]
    KBENCH_N=256 KBENCH_MIX=fp16 python tools/kbench.py [filter-regex]     (config E's shapes)
    KBENCH_PROBE=1 BLINDNO_LIB=variants/rfprobe/libblindno.so python tools/kbench.py REGEX
        (a ROWFUSE_PROBE=1 build: per-wave staging / item times of the row kernels;
         KBENCH_PROBE=2 with a ROWINV_WIDE_PROBE=1 build: the heads' wide row inverse)

Times the C-ABI entry points of the FNO_input body (Bn = 4 * 75 snapshots, width 4,
P = 160, m = 12) and of one head layer (Bn = 4, width 12, m = 32) in isolation, so kernel
variants can be compared without a full training step.  Prints one line per case:
name, us per call, algorithmic GB/s.
"""
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "reconstruction-of-pde-without-time-label_amd"))

import torch  # noqa: E402

import blindno  # noqa: E402
from blindno import ops  # noqa: E402
from blindno._lib import call, ptr, query, stream_ptr  # noqa: E402


def timeit(fn, iters=20, warm=3):
    for _ in range(warm):
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
    pat = sys.argv[1] if len(sys.argv) > 1 else ""
    blindno.load_library()
    # KBENCH_N: the encoder grid (128: config C; 256: config E), KBENCH_MIX=fp16: config E's mix
    NG = int(os.environ.get("KBENCH_N", "128"))
    if os.environ.get("KBENCH_MIX"):
        ops.set_mix_precision(os.environ["KBENCH_MIX"])
    dev = torch.device("cuda")
    torch.manual_seed(0)
    res = []

    def case(name, fn, nbytes):
        if pat and not re.search(pat, name):
            return
        us = timeit(fn)
        res.append((name, us, nbytes / (us * 1e-6) / 1e9))
        print(f"{name:40s} {us:9.1f} us  {nbytes / (us * 1e-6) / 1e9:8.0f} GB/s", flush=True)
        if probe is not None:
            probe_report(fn)

    # KBENCH_PROBE=1 with a ROWFUSE_PROBE=1 build: per-wave phase stamps of the row kernels
    probe = None
    if os.environ.get("KBENCH_PROBE"):
        import ctypes
        import numpy as np
        from blindno import _lib
        lib = _lib.load()
        if os.environ["KBENCH_PROBE"] == "2":      # the heads' wide row inverse (ROWINV_WIDE_PROBE=1)
            probe = (lib.blindno_rowinv_wide_probe_reset, lib.blindno_rowinv_wide_probe_read, 2)
        else:
            probe = (lib.blindno_rowfuse_probe_reset, lib.blindno_rowfuse_probe_read, 1)
        probe[1].argtypes = [ctypes.c_void_p, ctypes.c_int]

    def probe_report(fn):
        torch.cuda.synchronize()
        probe[0]()
        fn()
        torch.cuda.synchronize()
        buf = np.zeros(8192 * 8, dtype=np.uint64)
        probe[1](buf.ctypes.data, buf.size)
        t = buf.reshape(8192, 8).astype(np.int64)
        slot = np.nonzero(t[:, 0] > 0)[0]
        t = t[t[:, 0] > 0]
        if not len(t):
            print("    (no row-kernel stamps)")
            return
        t0 = t[:, 0].min()
        us_ = lambda a: (a - t0) * 0.01
        if probe[2] == 2:
            ready = us_(t[:, 2]) - us_(t[:, 1])
            rest = us_(t[:, 3]) - us_(t[:, 2])
            print(f"    waves {len(t)}  start spread {us_(t[:, 0]).max():5.2f}  weights {np.median(us_(t[:, 1]) - us_(t[:, 0])):5.2f}"
                  f"  operands ready {np.median(ready):5.2f}/{ready.max():5.2f}  MFMA+epilogue+stores {np.median(rest):5.2f}/{rest.max():5.2f}"
                  f"  wave end med {np.median(us_(t[:, 4])):6.2f} max {us_(t[:, 4]).max():6.2f} us", flush=True)
            return
        stage = us_(t[:, 1]) - us_(t[:, 0])
        nit = (t[:, 2:7] > 0).sum(axis=1)
        first = us_(t[:, 2]) - us_(t[:, 1])
        later = [us_(t[i, 2 + k]) - us_(t[i, 1 + k]) for i in range(len(t)) for k in range(1, 5) if t[i, 2 + k] > 0]
        end = us_(t[:, 7])
        print(f"    waves {len(t)}  items/wave {np.bincount(nit).tolist()}  start spread {us_(t[:, 0]).max():5.2f}"
              f"  staging {np.median(stage):5.2f}/{stage.max():5.2f}  first item {np.median(first):6.2f}/{first.max():6.2f}"
              f"  later items {np.median(later) if later else 0:6.2f}  wave end med {np.median(end):6.2f} max {end.max():6.2f} us",
              flush=True)
        # a wave's first item is its slot (blockIdx 4 + wave): its 16-row block is slot % 10 at P1 = 160
        blk = slot % 10
        print("    first item by 16-row block (median us):",
              " ".join(f"{b}:{np.median(first[blk == b]):5.1f}" for b in range(10) if (blk == b).any()), flush=True)

    # "u52": the encoder at the step's mean bag size (4 bags x ~52 distinct snapshots)
    # "u50": 200 snapshots, 2000 16-row items (< the 2048 resident waves of the row kernels)
    # KBENCH_BN=160,240: further encoder-shaped sizes ("bn160", ...)
    extra = [(f"bn{b}", int(b), 4, 12, 1) for b in os.environ.get("KBENCH_BN", "").split(",") if b]
    for tag, Bn, C, m, Cout in [("input", 300, 4, 12, 1), ("u52", 208, 4, 12, 1), ("u50", 200, 4, 12, 1),
                                *extra, ("head", 4, 12, 32, 1), ("head2", 8, 12, 32, 1)]:
        N = NG
        P = N + ops.pad_amount(N)
        z = torch.randn(Bn, C, P, P, device=dev)
        w1 = torch.randn(128, C, device=dev) * 0.3
        b1 = torch.randn(128, device=dev) * 0.1
        w2 = torch.randn(Cout, 128, device=dev) * 0.1
        b2 = torch.randn(Cout, device=dev)
        out = torch.empty(Bn, N, N, Cout, device=dev)
        div = {"input": 75, "u52": 52, "u50": 50}.get(tag, 1 if C > 4 else Bn // 4)  # the encoder's bag-mean gradient: one field per bag
        dout = torch.randn(Bn // div, N, N, Cout, device=dev)
        dz = torch.zeros_like(z)
        nch = query("blindno_project_bwd_nchunk", Bn, N, N)
        npar = 128 * C + 128 + Cout * 128 + Cout
        part = torch.empty(nch, npar, device=dev)
        pts = Bn * N * N
        case(f"project_fwd[{tag}]", lambda: call("blindno_project_fwd", ptr(z), ptr(w1), ptr(b1), ptr(w2), ptr(b2),
                                                  ptr(out), Bn, C, P, P, N, N, 128, Cout, Cout, 0, stream_ptr()),
             4 * pts * (C + Cout))
        case(f"project_bwd[{tag}]", lambda: call("blindno_project_bwd", ptr(z), ptr(w1), ptr(b1), ptr(w2), ptr(dout),
                                                  ptr(dz), ptr(part), nch, Bn, C, P, P, N, N, 128, Cout, Cout, 0, div,
                                                  stream_ptr()),
             8 * pts * C + 4 * (pts // div) * Cout)
        if tag == "input":
            # bag-level projection (csrc/bagproj.hip): B = 4 bags of U = 75 snapshots
            Bb, U = 4, Bn // 4
            lw = torch.full((U,), 1.0 / U, device=dev)
            ubar = torch.empty(Bb, N * N, device=dev)
            stats = torch.empty(query("blindno_project_bag_stats_floats", Bb, N, N), device=dev)
            vv = torch.empty_like(z)
            gsb = torch.randn(Bb, N * N, device=dev)
            nbc = query("blindno_project_bag_bwd_nchunk", Bb, N, N)
            pb = torch.empty(nbc, 128 * C + 2 * 128 + 1, device=dev)
            sbytes = stats.numel() * 4
            case("project_bag_fwd[input]", lambda: call("blindno_project_bag_fwd", ptr(z), ptr(w1), ptr(b1), ptr(w2),
                                                        ptr(b2), ptr(lw), ptr(ubar), ptr(stats), ptr(vv), Bb, U, C,
                                                        P, P, N, N, 128, stream_ptr()),
                 8 * pts * C + sbytes)
            # the benched step's bag: ~52 distinct snapshots of a randint(50, 100) draw
            U52 = 52
            lw52 = torch.full((U52,), 1.0 / U52, device=dev)
            case("project_bag_fwd[u52]", lambda: call("blindno_project_bag_fwd", ptr(z), ptr(w1), ptr(b1), ptr(w2),
                                                      ptr(b2), ptr(lw52), ptr(ubar), ptr(stats), ptr(vv), Bb, U52, C,
                                                      P, P, N, N, 128, stream_ptr()),
                 8 * Bb * U52 * N * N * C + sbytes)
            case("project_bag_bwd[input]", lambda: call("blindno_project_bag_bwd", ptr(stats), ptr(gsb), ptr(w2),
                                                        ptr(lw), ptr(vv), ptr(dz), ptr(pb), nbc, Bb, U, C, P, P, N,
                                                        N, 128, stream_ptr()),
                 8 * pts * C + sbytes)
        if tag == "input":
            # calibration: the device's own copy of one field (read + write, the streaming ceiling
            # of an epilogue that reads x and writes z)
            zc = torch.empty_like(z)
            case("copy_field[input]", lambda: zc.copy_(z), 2 * 4 * z.numel())
        # spectral pieces of one layer
        sh = ops.SpecShape(Bn, C, C, P, P, m, m, 2)
        w = torch.rand(C, C, m, m, 2, device=dev) / (C * C)
        Wt = ops.k_pack_w2d(w, w.clone(), P)
        fld = 4 * Bn * C * P * P
        case(f"rowdft[{tag}]", lambda: ops.k_rowdft(z, Bn, C, P, P, m, 1), fld)
        At = ops.k_rowdft(z, Bn, C, P, P, m, 1)
        case(f"colpass[{tag}]", lambda: ops.k_colpass(At, Wt, Bn, C, C, P, m, m, P, 0), 8 * Bn * m * C * P * 3)
        X, Z = ops.k_colpass(At, Wt, Bn, C, C, P, m, m, P, 0)
        cw = torch.randn(C, C, 1, 1, device=dev) * 0.3
        cb = torch.randn(C, device=dev) * 0.1
        case(f"rowidft_epi[{tag}]", lambda: ops.k_rowidft_epi(Z, z, cw, cb, Bn, C, P, P, m, 1), 2 * fld)
        case(f"rowidft_bwd[{tag}]", lambda: ops.k_rowidft_bwd(Z, z, cw, z, Bn, C, P, P, m, 1, C <= 4), 3 * fld)
        if C <= 4:
            # layer chaining: the next row DFT in the row-inverse pass (+ its spectrum bytes)
            spb = 8 * Bn * m * C * P
            case(f"rowidft_epi_rd[{tag}]", lambda: ops.k_rowidft_epi_rd(Z, z, cw, cb, Bn, C, P, P, m, 1, 1),
                 2 * fld + 2 * spb)
            case(f"rowidft_bwd_rd_crop[{tag}]",
                 lambda: ops.k_rowidft_bwd(Z, z, cw, z, Bn, C, P, P, m, 1, True, (N, N), rd=True),
                 fld * (2 + (N * N) / (P * P)) + 2 * spb)

            def layer():
                _, Zl = ops.k_colpass(At, Wt, Bn, C, C, P, m, m, P, 0)
                return ops.k_rowidft_epi_rd(Zl, z, cw, cb, Bn, C, P, P, m, 1, 1)
            # SURVEY 8d's algorithmic bytes of one layer: read x, write y, the weights
            case(f"layer_colpass+epi_rd[{tag}]", layer, 2 * fld + 16 * C * C * m * m)
            if ops.colspec_ok(Bn, C, P, P, m, m):
                # the column pass folded into the row kernels (csrc/colspec.h)
                cs = ops._ColSpec(Bn, C, P, P, m, m, dev)
                p_in, p_out = cs.part(C, z), cs.part(C, z)
                zo = torch.empty_like(z)
                cd = lambda: call("blindno_rowdft_cd", ptr(z), ptr(p_in), ptr(cs.Tp), ptr(cs.tab), Bn, C, P, P, m, 1,
                                  P, P, stream_ptr())
                cd()
                pb = 4 * p_in.numel()
                case(f"rowdft_cd[{tag}]", cd, fld + pb)
                case(f"colmix[{tag}]", lambda: cs.mix(p_in, cs.nb, Wt, 0), pb + 2 * 8 * Bn * m * C * 24)
                _, Yc = cs.mix(p_in, cs.nb, Wt, 0)
                epi_zc = lambda: call("blindno_rowidft_epi_zc", ptr(Yc), ptr(z), ptr(cw), ptr(cb), ptr(zo), ptr(cs.tb),
                                      ptr(cs.tab), ptr(p_out), ptr(cs.Tp), Bn, C, P, P, m, m, 1, 1, P, P, stream_ptr())
                case(f"rowidft_epi_zc[{tag}]", epi_zc, 2 * fld + pb)
                case(f"rowidft_epi_zy[{tag}]",
                     lambda: call("blindno_rowidft_epi_zc", ptr(Yc), ptr(z), ptr(cw), ptr(cb), ptr(zo), ptr(cs.tb),
                                  ptr(cs.tab), None, None, Bn, C, P, P, m, m, 1, 0, P, P, stream_ptr()), 2 * fld)

                def layer_f():
                    cs.mix(p_in, cs.nb, Wt, 0)
                    epi_zc()
                case(f"layer_colmix+epi_zc[{tag}]", layer_f, 2 * fld + 16 * C * C * m * m)
                nch = query("blindno_colspec_bwd_nchunk", Bn, P)
                pw = torch.empty(nch, C * C + C, device=dev)
                case(f"rowidft_bwd_zc_crop[{tag}]",
                     lambda: call("blindno_rowidft_bwd_zc", ptr(Yc), ptr(z), ptr(cw), ptr(z), ptr(zo), ptr(cs.tb),
                                  ptr(cs.tab), ptr(p_out), ptr(cs.Tp), ptr(pw), Bn, C, P, P, m, m, 1, N, N,
                                  stream_ptr()),
                     fld * (2 + (N * N) / (P * P)) + pb)
        if C > 4:
            case(f"conv_wgrad[{tag}]", lambda: ops.k_conv_wgrad(z, z, Bn, C, P, P, 1), 2 * fld)
        inp = torch.randn(Bn, N, N, 3 if C == 4 else C, device=dev)
        fc0w = torch.randn(C, inp.shape[-1], device=dev)
        fc0b = torch.randn(C, device=dev)
        x0 = torch.empty(Bn, C, P, P, device=dev)
        case(f"lift_fwd[{tag}]", lambda: call("blindno_lift_fwd", ptr(inp), ptr(fc0w), ptr(fc0b), ptr(x0), Bn, N, N,
                                               inp.shape[-1], C, P, P, stream_ptr()), fld + inp.numel() * 4)
        nl = query("blindno_lift_bwd_nchunk", Bn, N, N)
        pl = torch.empty(nl, C * inp.shape[-1] + C, device=dev)
        case(f"lift_bwd[{tag}]", lambda: call("blindno_lift_bwd", ptr(x0), ptr(inp), ptr(fc0w), None, ptr(pl), nl, Bn,
                                               N, N, inp.shape[-1], C, P, P, stream_ptr()), fld + inp.numel() * 4)
    return res


if __name__ == "__main__":
    main()
