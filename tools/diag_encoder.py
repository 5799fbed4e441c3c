"""Per-layer numerics of Encoder2D's convolutions on MIOpen: 32-row chunks vs the full batch,
each against fp64 (fwd, bwd-data, bwd-weight).  Run once per MIOpen env variant:

    python tools/diag_encoder.py [label]

Prints one line per layer: rel-L2 of y, dx, dW for chunked and full-batch fp32.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "reconstruction-of-pde-without-time-label_amd"))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import blindno  # noqa: E402


def rel(a, b):
    return float((a.double() - b).norm() / b.norm().clamp_min(1e-300))


def main():
    label = sys.argv[1] if len(sys.argv) > 1 else "default"
    det = os.environ.get("DIAG_DETERMINISTIC") == "1"
    torch.backends.cudnn.deterministic = det
    torch.manual_seed(1)
    enc = blindno.Encoder2D(25, last_kernel=blindno.Encoder2D.kernel_for_grid(64)).cuda()
    n = 74
    h64 = torch.randn(n, 1, 64, 64, device="cuda", dtype=torch.float64)
    print(f"[{label}] deterministic={det}", flush=True)
    for name in ("convblock1", "convblock2_1", "convblock2_2", "convblock3_1", "convblock3_2",
                 "convblock4_1", "convblock4_2", "convblock7_1", "convblock7_2", "convblock7_3"):
        conv = getattr(enc, name).layers[0]
        w64, b64 = conv.weight.detach().double(), conv.bias.detach().double()
        kw = dict(stride=conv.stride, padding=conv.padding)
        x64 = h64.clone().requires_grad_(True)
        W64 = w64.clone().requires_grad_(True)
        y64 = F.conv2d(x64, W64, b64, **kw)
        cot = torch.randn_like(y64)
        (y64 * cot).sum().backward()
        res = {}
        for mode in ("chunk32", "full"):
            x = h64.float().requires_grad_(True)
            W = conv.weight.detach().clone().requires_grad_(True)
            if mode == "full":
                y = F.conv2d(x, W, conv.bias.detach(), **kw)
            else:
                xp = torch.cat([x, x.new_zeros((96 - n,) + tuple(x.shape[1:]))])
                y = torch.cat([F.conv2d(xp[i:i + 32], W, conv.bias.detach(), **kw) for i in range(0, 96, 32)])[:n]
            (y * cot.float()).sum().backward()
            res[mode] = (rel(y.detach(), y64.detach()), rel(x.grad, x64.grad), rel(W.grad, W64.grad))
        c, f = res["chunk32"], res["full"]
        print(f"[{label}] {name:13s} in{tuple(h64.shape[1:])} "
              f"chunk y {c[0]:.1e} dx {c[1]:.1e} dW {c[2]:.1e} | full y {f[0]:.1e} dx {f[1]:.1e} dW {f[2]:.1e}",
              flush=True)
        # next layer's input: a BN'd, leaky-relu'd version of this output (fp64), like the encoder
        y = y64.detach()
        y = (y - y.mean((0, 2, 3), keepdim=True)) / y.std((0, 2, 3), keepdim=True)
        h64 = F.leaky_relu(y, 0.2)


if __name__ == "__main__":
    main()
