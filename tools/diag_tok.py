"""Diagnostic: accuracy of the collapsed temporal-attention bag mean (TokAttnMeanFn) vs the
literal fp64 form and the literal fp32 form (conditioning), per output."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "reconstruction-of-pde-without-time-label_amd"), os.path.join(ROOT, "tests")]
import torch
import oracle
from conftest import rel_l2
from blindno.unet import TokAttnMeanFn

for (B, L, D, scale, off) in [(2, 57, 3721, 1.0, 0.5), (4, 99, 144, 1.0, 0.5), (2, 55, 1352, 1.0, 3.0),
                              (2, 55, 676, 0.2, 0.0), (2, 150, 2048, 0.5, 0.5)]:
    torch.manual_seed(5)
    X = (torch.randn(B, L, D, dtype=torch.float64) + off * torch.randn(B, L, 1, dtype=torch.float64)) * scale
    lw, lb = 1 + 0.1 * torch.randn(D, dtype=torch.float64), 0.1 * torch.randn(D, dtype=torch.float64)
    g = torch.randn(B, D, dtype=torch.float64)
    res = {}
    for dt in (torch.float64, torch.float32):
        ref = [t.to(dt).clone().requires_grad_(True) for t in (X, lw, lb)]
        yr = oracle.unet_ref.temporal_attention({"norm.weight": ref[1], "norm.bias": ref[2]},
                                                ref[0].view(B, L, 1, D)).mean(1).view(B, D)
        (yr * g.to(dt)).sum().backward()
        res[dt] = [yr.detach().double()] + [r.grad.double() for r in ref]
    dev = [t.detach().clone().cuda().float().requires_grad_(True) for t in (X, lw, lb)]
    y = TokAttnMeanFn.apply(*dev, 1e-5)
    (y * g.cuda().float()).sum().backward()
    got = [y.detach().double().cpu()] + [t.grad.double().cpu() for t in dev]
    # coherent part of dX: per-token sums over the D features (what bias-type gradients see)
    got.append(got[1].sum(-1)); res[torch.float32].append(res[torch.float32][1].sum(-1))
    res[torch.float64].append(res[torch.float64][1].sum(-1))
    names = ["Y", "dX", "dlw", "dlb", "sum_d dX"]
    print(B, L, D, scale, off, " ".join(f"{n}: hip {rel_l2(a, r):.2e} fp32 {rel_l2(b, r):.2e}"
                                   for n, a, b, r in zip(names, got, res[torch.float32], res[torch.float64])))
