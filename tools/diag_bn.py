"""Isolate the BatchNorm + LeakyReLU backward of Encoder2D's last block (convblock7_3: 74 rows,
512 channels, 1x1 outputs) on the HIP path: feed it the HIP chain's own activations and compare
z (conv output), y (block output) and dz (BN input gradient) with float64 evaluations of the same
formulas on the same fp32 inputs.  Prints per-channel conditioning (|mean| / std) too.

    python tools/diag_bn.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "reconstruction-of-pde-without-time-label_amd"))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import blindno  # noqa: E402
from blindno import ops  # noqa: E402


def rel(a, b):
    a, b = a.detach().double(), b.detach().double()
    return float((a - b).norm() / b.norm().clamp_min(1e-300))


def main():
    torch.manual_seed(1)
    enc = blindno.Encoder2D(25, last_kernel=blindno.Encoder2D.kernel_for_grid(64)).cuda().train()
    x = torch.randn(2, 37, 1, 64, 64, device="cuda")
    h = x.reshape(74, 1, 64, 64)
    names = ("convblock1", "convblock2_1", "convblock2_2", "convblock3_1", "convblock3_2", "convblock4_1",
             "convblock4_2", "convblock7_1", "convblock7_2", "convblock7_3")
    with torch.no_grad():
        for n in names[:-1]:
            h = getattr(enc, n)(h)
    for name in ("convblock7_2", "convblock7_3"):
        blk = getattr(enc, name)
        if name == "convblock7_2":
            with torch.no_grad():
                h = h  # input of 7_2 is the output of 7_1, recompute below
        conv, bn = blk.layers[0], blk.layers[1]
        hin = h.detach()
        if name == "convblock7_2":
            # rebuild the input of 7_2
            hin = x.reshape(74, 1, 64, 64)
            with torch.no_grad():
                for n in names[:-2]:
                    hin = getattr(enc, n)(hin)
        z = ops.conv2d(hin, conv.weight, conv.bias, conv.stride, conv.padding).detach().requires_grad_(True)
        y = ops.BNActFn.apply(z, bn.weight, bn.bias, bn, z.shape[0], blk.relu_slope)
        z64 = F.conv2d(hin.double(), conv.weight.double(), conv.bias.double(), conv.stride, conv.padding)
        zd = z.detach().double().requires_grad_(True)
        g64, b64 = bn.weight.detach().double().requires_grad_(True), bn.bias.detach().double().requires_grad_(True)
        y64 = F.leaky_relu(F.batch_norm(zd, None, None, g64, b64, training=True, eps=bn.eps), blk.relu_slope)
        dv = torch.randn_like(y)
        gz, gg, gb = torch.autograd.grad(y, (z, bn.weight, bn.bias), dv)
        gz64, gg64, gb64 = torch.autograd.grad(y64, (zd, g64, b64), dv.double())
        mean = zd.detach().mean((0, 2, 3))
        std = zd.detach().var((0, 2, 3), unbiased=False).sqrt()
        cond = (mean.abs() / std)
        pre = (zd.detach() - mean[None, :, None, None]) / (std[None, :, None, None] ** 2 + bn.eps).sqrt()
        print(f"[{name}] z shape {tuple(z.shape)}  conv z vs fp64 conv: {rel(z, z64):.2e}")
        print(f"[{name}] |mean|/std over channels: median {cond.median():.3g}  max {cond.max():.3g}; "
              f"min |pre-activation| {pre.abs().min():.3g}")
        print(f"[{name}] y {rel(y, y64):.2e}  dz {rel(gz, gz64):.2e}  dgamma {rel(gg, gg64):.2e}  "
              f"dbeta {rel(gb, gb64):.2e}")
        e = (gb.double() - gb64).abs() / gb64.abs().clamp_min(1e-30)
        worst = torch.topk(e, 5)
        print(f"[{name}] worst dbeta channels {worst.indices.tolist()} rel {[f'{v:.2e}' for v in worst.values.tolist()]}")
        c = int(worst.indices[0])
        print(f"[{name}]   channel {c}: dbeta hip {gb[c].item():.6e} fp64 {gb64[c].item():.6e}  "
              f"sum|dv| {dv[:, c].abs().sum().item():.3e}  pre range [{pre[:, c].min():.3g}, {pre[:, c].max():.3g}]")
        # torch fp32 on the same z for comparison
        z32 = z.detach().clone().requires_grad_(True)
        g32, b32 = bn.weight.detach().clone().requires_grad_(True), bn.bias.detach().clone().requires_grad_(True)
        y32 = F.leaky_relu(F.batch_norm(z32, None, None, g32, b32, training=True, eps=bn.eps), blk.relu_slope)
        t = torch.autograd.grad(y32, (z32, g32, b32), dv)
        print(f"[{name}] torch fp32 same z: y {rel(y32, y64):.2e} dz {rel(t[0], gz64):.2e} dgamma "
              f"{rel(t[1], gg64):.2e} dbeta {rel(t[2], gb64):.2e}")


if __name__ == "__main__":
    main()
