"""Where does Encoder2D's gradient error come from?  Runs the 64x64 Encoder2D of
tests/test_gpu_encoder.py block by block on (a) the HIP path, (b) plain fp32 torch, (c) fp64 torch,
all from the same weights and input, and prints per block: rel-L2 of the block output (forward)
and of the gradient w.r.t. the block output (backward), against fp64.

    python tools/diag_encoder_bwd.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "reconstruction-of-pde-without-time-label_amd"))
import torch  # noqa: E402

import blindno  # noqa: E402

BLOCKS = ("convblock1", "convblock2_1", "convblock2_2", "convblock3_1", "convblock3_2", "convblock4_1",
          "convblock4_2", "convblock7_1", "convblock7_2", "convblock7_3")


def rel(a, b):
    a, b = a.detach(), b.detach()
    return float((a.double() - b).norm() / b.norm().clamp_min(1e-300))


def run(enc, x, hip):
    b, L = x.shape[:2]
    h = x.reshape(b * L, 1, 64, 64)
    outs = []
    for name in BLOCKS:
        blk = getattr(enc, name)
        h = blk(h) if hip else blk.layers(h)
        h.retain_grad()
        outs.append(h)
    return enc.linear(h.flatten(1).view(b, L, -1)), outs


def main():
    torch.manual_seed(1)
    mk = lambda: blindno.Encoder2D(25, last_kernel=blindno.Encoder2D.kernel_for_grid(64)).cuda().train()  # noqa
    enc, r32, r64 = mk(), mk(), mk().double()
    r32.load_state_dict(enc.state_dict())
    r64.load_state_dict(enc.state_dict())
    x = torch.randn(2, 37, 1, 64, 64, device="cuda")
    o, oh = run(enc, x, True)
    o32, oh32 = run(r32, x, False)
    o64, oh64 = run(r64, x.double(), False)
    cot = torch.randn_like(o64)
    (o * cot.float()).sum().backward()
    (o32 * cot.float()).sum().backward()
    (o64 * cot).sum().backward()
    print(f"{'block':14s} {'fwd hip':>9s} {'fwd t32':>9s} {'dout hip':>9s} {'dout t32':>9s}")
    for name, a, b, c in zip(BLOCKS, oh, oh32, oh64):
        print(f"{name:14s} {rel(a, c):9.2e} {rel(b, c):9.2e} {rel(a.grad, c.grad):9.2e} {rel(b.grad, c.grad):9.2e}")
    p32, p64 = dict(r32.named_parameters()), dict(r64.named_parameters())
    print(f"{'param':34s} {'hip':>9s} {'t32':>9s}")
    for k, p in enc.named_parameters():
        print(f"{k:34s} {rel(p.grad, p64[k].grad):9.2e} {rel(p32[k].grad, p64[k].grad):9.2e}")
    # the same blocks evaluated by the HIP path but fed the fp64 path's (rounded) gradient at each
    # block output: isolates each block's own backward error from what it inherits
    print(f"{'block (isolated bwd)':22s} {'din hip':>9s} {'din t32':>9s}")
    for i, name in enumerate(BLOCKS):
        inp64 = (x.double().reshape(74, 1, 64, 64) if i == 0 else oh64[i - 1]).detach()
        g64 = oh64[i].grad
        res = []
        for mod, dt, hip in ((getattr(enc, name), torch.float32, True), (getattr(r32, name), torch.float32, False),
                             (getattr(r64, name), torch.float64, False)):
            xi = inp64.to(dt).requires_grad_(True)
            y = mod(xi) if hip else mod.layers(xi)
            y.backward(g64.to(dt))
            res.append(xi.grad)
        print(f"{name:22s} {rel(res[0], res[2]):9.2e} {rel(res[1], res[2]):9.2e}")


if __name__ == "__main__":
    main()
