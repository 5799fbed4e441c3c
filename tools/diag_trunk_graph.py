"""Config D: the trunk's gradients in the graphed step vs the same trunk run eagerly (libblindno
ops, fed the replay's own dL/dbasis) vs the fp64 trunk given that dL/dbasis.  Names whether
a trunk-gradient error of the graphed step comes from the trunk's kernels or the graph."""
import sys
import numpy as np
import torch
sys.path.insert(0, "reconstruction-of-pde-without-time-label_amd")
sys.path.insert(0, ".")
import blindno
from blindno.train import DataParallel, FlatAdam, GraphedBagStep, grid2d, synthetic_bags, trained_parameters
from oracle import cpu_ref


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
    rec = []
    h = m.trunk.register_full_backward_hook(lambda mod, gi, go: rec.append(go[0].detach().clone()))
    gs = GraphedBagStep(m, blindno.mse_loss, opt, DataParallel(opt), X, Y, grid)
    draws = [rs.choice(100, rs.randint(50, 100)) for _ in range(3)]
    rec_of = {}
    for it in range(int(sys.argv[1]) if len(sys.argv) > 1 else 13):
        n1 = len(rec)
        k = gs.step(draws[it % 3])
        if len(rec) > n1:
            rec_of[len(draws[it % 3])] = len(rec) - 1     # the capture's own record
    idx = draws[0]
    n0 = len(rec)
    key = gs.replay(idx)
    torch.cuda.synchronize()
    h.remove()
    db = rec[rec_of[key]].clone()
    names = {id(q): k for k, q in m.named_parameters()}
    gg = {names[id(p)]: opt.grad[o:o + s].detach().clone().view(p.shape)
          for p, o, s in zip(opt.params, opt.offsets, opt.sizes) if names[id(p)].startswith("trunk.")}
    pts = grid.reshape(-1, 2)
    sd = {k[6:]: v.detach().clone() for k, v in m.named_parameters() if k.startswith("trunk.")}
    rel = lambda a, b: float((a.double() - b.double()).norm() / b.double().norm())
    p64 = {k: v.double().requires_grad_(True) for k, v in sd.items()}
    o64 = cpu_ref._ffn(p64, pts.double(), 3)
    o64.backward(db.double())
    p32 = {k: v.cpu().clone().requires_grad_(True) for k, v in sd.items()}
    cpu_ref._ffn(p32, pts.cpu(), 3).backward(db.cpu())
    pg = {k: v.clone().requires_grad_(True) for k, v in sd.items()}
    cpu_ref._ffn(pg, pts, 3).backward(db)        # torch fp32 ops on the GPU
    eager = []
    for rep in range(2):
        for p in m.trunk.parameters():
            p.grad = None
        out = m.trunk(pts)
        out.backward(db)
        eager.append({k: p.grad.detach().clone() for k, p in m.trunk.named_parameters()})
    print(f"replay key {key}, hook records {len(rec)} ({len(rec) - n0} in the replay call)")
    print("param".ljust(26) + "graph_vs64".rjust(12) + "eager_vs64".rjust(12) + "eager_rep".rjust(12) +
          "graph_vs_eager".rjust(16) + "cpu32_vs64".rjust(12) + "torchgpu_vs64".rjust(15))
    for k in sd:
        g = gg["trunk." + k]
        print(k.ljust(26) + f"{rel(g, p64[k].grad):12.2e}{rel(eager[0][k], p64[k].grad):12.2e}"
              f"{rel(eager[1][k], eager[0][k]):12.2e}{rel(g, eager[0][k]):16.2e}"
              f"{rel(p32[k].grad, p64[k].grad.cpu()):12.2e}{rel(pg[k].grad, p64[k].grad):15.2e}")


if __name__ == "__main__":
    main()
