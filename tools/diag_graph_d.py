#!/usr/bin/env python3
"""Diagnose NIOFP2D graph replays across keys: capture keys A, B, replay A after B's capture,
compare the flat gradient with an eager step at the same parameters.

    python tools/diag_graph_d.py [N] [shared|separate]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "reconstruction-of-pde-without-time-label_amd"))
sys.path.insert(0, ROOT)
import numpy as np
import torch


def main():
    import blindno
    from blindno import Encoder2D, NIOFP2D
    from blindno.train import DataParallel, FlatAdam, GraphedBagStep, grid2d, trained_parameters
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    mode = sys.argv[2] if len(sys.argv) > 2 else "shared"
    blindno.load_library()
    torch.manual_seed(6)
    m = NIOFP2D(2, 3, 100, 25, 3, 12, 32, 2, heads=("fno_Fx", "fno_Fy"),
                branch_last_kernel=Encoder2D.kernel_for_grid(N)).cuda().train()
    B, T = 2, 100
    g = torch.Generator(device="cuda").manual_seed(7)
    x = torch.randn(B, T, N, N, device="cuda", generator=g)
    y = torch.randn(B, N, N, 2, device="cuda", generator=g)
    grid = grid2d(N, N, "cuda")
    opt = FlatAdam(trained_parameters(m, exclude_prefixes=("fc0.",)), lr=5e-4)
    gs = GraphedBagStep(m, blindno.mse_loss, opt, DataParallel(opt), x, y, grid)
    if mode == "separate":
        gs.pool = None
    names = {id(p): k for k, p in m.named_parameters()}
    rs = np.random.RandomState(13)
    draws = [rs.choice(T, rs.randint(50, T)) for _ in range(2)]

    def eager_grad(idx):
        saved = [(b, b.detach().clone()) for b in m.buffers()]
        opt.zero_grad()
        out = m(x, grid, bag_idx=idx)
        blindno.mse_loss(out, y).backward()
        gg = opt.gather_grads().clone()
        opt.zero_grad()
        with torch.no_grad():
            for b, c in saved:
                b.copy_(c)
        return out.detach(), gg

    def report(tag, idx):
        key = gs.replay(idx)
        torch.cuda.synchronize()
        gout, ggrad = gs.out[key].clone(), opt.grad.clone()
        eout, egrad = eager_grad(idx)
        e = float((gout - eout).norm() / eout.norm())
        bad = []
        for prm, off, sz in zip(opt.params, opt.offsets, opt.sizes):
            a, b = ggrad[off:off + sz], egrad[off:off + sz]
            r = float((a - b).norm() / b.norm().clamp_min(1e-30))
            if r > 1e-5:
                bad.append((names[id(prm)], f"{r:.2e}"))
        print(f"{tag}: key {key} out {e:.2e}, {len(bad)} bad grads {bad[:8]}", flush=True)

    def poison():
        # overwrite every free block of the default pool: a graph that still points at one reads NaN
        torch.cuda.synchronize()
        free = torch.cuda.mem_get_info()[0]
        blobs = []
        try:
            for _ in range(64):
                blobs.append(torch.full((1 << 28,), float("nan"), device="cuda"))   # 1 GiB each
        except RuntimeError:
            pass
        torch.cuda.synchronize()
        n = len(blobs)
        del blobs
        torch.cuda.synchronize()
        print(f"  poisoned {n} GiB (free before {free / 2**30:.0f} GiB)", flush=True)

    report("capture+replay A", draws[0])
    report("capture+replay B", draws[1])
    report("replay A after B", draws[0])
    report("replay B after A", draws[1])
    if len(sys.argv) > 3:
        import oracle
        p = {k: v.detach().double().requires_grad_(True) for k, v in m.state_dict().items()
             if v.is_floating_point() and not k.endswith(("running_mean", "running_var"))}
        ref = oracle.niofp2d(p, x.double(), grid.double(), idx=draws[1].tolist(), heads=("fno_Fx", "fno_Fy"))
        ((ref - y.double()) ** 2).mean().backward()
        del ref, p
        print("  ran the fp64 oracle", flush=True)
        report("replay A after oracle", draws[0])
        poison()
        report("replay A after poison", draws[0])
        report("replay B after poison", draws[1])
    report("replay A again", draws[0])


if __name__ == "__main__":
    main()
