"""Config D's FFN trunk in isolation on the GPU (libblindno: ops.linear + BNActFn) vs the same
trunk in fp32 on the CPU (torch, as the reference computes) and in fp64 (arbiter), fed the
upstream gradient dL/dbasis of a real config-D step (B = 4 bags: dbasis has rank 4, which is
what makes the trunk's weight-gradient sums cancel).  Per trunk parameter: gradient rel-L2 of
both fp32 paths; then the same with single ops of the trunk swapped for torch fp32 ops, to name
the op that loses the accuracy."""
import sys
import numpy as np
import torch
sys.path.insert(0, "reconstruction-of-pde-without-time-label_amd")
sys.path.insert(0, ".")
import blindno
from blindno import ops
from blindno.train import DataParallel, FlatAdam, grid2d, synthetic_bags, trained_parameters
from oracle import cpu_ref

F = torch.nn.functional


def main():
    blindno.load_library()
    torch.manual_seed(1234)
    N, B = 128, 4
    m = blindno.NIOFP2D(2, 3, 100, 25, 3, 12, 32, 2, heads=("fno_Fx", "fno_Fy"),
                        branch_last_kernel=blindno.Encoder2D.kernel_for_grid(N)).cuda().train()
    X, Y = synthetic_bags(B, 100, (N, N), 2, seed=1234, device="cuda", bag_ids=list(range(B)))
    grid = grid2d(N, N, "cuda")
    opt = FlatAdam(trained_parameters(m, exclude_prefixes=("fc0.",)), lr=5e-4)
    rs = np.random.RandomState(0)
    cap = {}
    m.trunk.register_full_backward_hook(lambda mod, gi, go: cap.__setitem__("g", go[0].detach().clone()))
    for step in range(14):
        idx = rs.choice(100, rs.randint(50, 100))
        opt.zero_grad()
        out = m(X, grid, bag_idx=idx)
        loss = blindno.mse_loss(out, Y)
        loss.backward()
        opt.gather_grads()
        if step < 13:
            opt.step()
    gup = cap["g"]
    pts = grid.reshape(-1, 2)
    trunk = m.trunk
    sd = {k: v.detach().clone() for k, v in trunk.named_parameters()}
    rel = lambda a, b: float((a.double().cpu() - b.double().cpu()).norm() / b.double().cpu().norm())
    res = {}
    for name, dev, dt in (("cpu32", "cpu", torch.float32), ("gpu64", "cuda", torch.float64),
                          ("gpu32_torch", "cuda", torch.float32)):
        p = {k: v.detach().to(dev, dt).clone().requires_grad_(True) for k, v in sd.items()}
        o = cpu_ref._ffn(p, pts.to(dev, dt), 3)
        o.backward(gup.to(dev, dt))
        res[name] = {k: v.grad for k, v in p.items()}
    g64 = res["gpu64"]

    def native(lin_native, bn_native):
        p = {k: v.detach().clone().requires_grad_(True) for k, v in sd.items()}
        slope = 0.01

        def lin(x, pre):
            if lin_native:
                return ops.linear(x, p[pre + ".weight"], p[pre + ".bias"])
            return F.linear(x, p[pre + ".weight"], p[pre + ".bias"])
        x = F.leaky_relu(lin(pts, "input_layer"), slope)
        for k in range(2):
            x = F.leaky_relu(lin(x, f"hidden_layers.{k}"), slope)
            bn = trunk.batch_layers[k]
            if bn_native:
                x = ops.BNActFn.apply(x, p[f"batch_layers.{k}.weight"], p[f"batch_layers.{k}.bias"], bn,
                                      x.shape[0], 1.0)
            else:
                x = F.batch_norm(x, None, None, p[f"batch_layers.{k}.weight"], p[f"batch_layers.{k}.bias"],
                                 training=True, eps=1e-5)
        o = lin(x, "output_layer")
        o.backward(gup)
        return {k: v.grad for k, v in p.items()}
    res["native"] = native(True, True)
    res["lin_native_bn_torch"] = native(True, False)
    res["lin_torch_bn_native"] = native(False, True)
    cols = ("native", "lin_native_bn_torch", "lin_torch_bn_native", "gpu32_torch", "cpu32")
    print("param".ljust(28) + "".join(c.rjust(22) for c in cols) + "  |g64|")
    for k in sd:
        print(k.ljust(28) + "".join(f"{rel(res[c][k], g64[k]):22.2e}" for c in cols) + f"  {float(g64[k].norm()):.2e}")


if __name__ == "__main__":
    main()
