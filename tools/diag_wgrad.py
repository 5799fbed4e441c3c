"""Where does the FNO_input gradient lose accuracy on trained weights?  Trains config C for 30
graphed steps (as tests/test_gpu_configs.py::test_config_c_after_training_steps), then runs
FNO_input alone (ops.FNOFn, generic path) on the bag's channels-last input with (a) a random
cotangent and (b) a bag-structured cotangent (identical for all snapshots of a bag), and
compares every parameter gradient of the HIP path and of the reference's fp32 CPU evaluation
(oracle.cpu_ref) with fp64 (oracle.cpu_ref in float64 on the GPU).  Also the bare first
spectral layer (SpectralConvFn) on x0."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "reconstruction-of-pde-without-time-label_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import blindno  # noqa: E402
from blindno import Encoder2D, NIOFP2D_FNO, ops  # noqa: E402
from blindno.fno import fno_params  # noqa: E402
from blindno.train import DataParallel, FlatAdam, GraphedBagStep, grid2d, trained_parameters  # noqa: E402
from oracle import cpu_ref  # noqa: E402
from oracle.fno_ref import sub_params  # noqa: E402


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / b.norm().clamp_min(1e-300))


def main():
    blindno.load_library()
    torch.manual_seed(0)
    m = NIOFP2D_FNO(2, 3, 100, 25, 3, 12, 32, 2, branch_last_kernel=Encoder2D.kernel_for_grid(128)).cuda().train()
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.randn(2, 100, 128, 128, device="cuda", generator=g)
    y = torch.randn(2, 128, 128, 2, device="cuda", generator=g)
    grid = grid2d(128, 128, "cuda")
    steps = int(os.environ.get("DIAG_STEPS", "30"))
    if steps:
        opt = FlatAdam(trained_parameters(m), lr=5e-4)
        gs = GraphedBagStep(m, blindno.mse_loss, opt, DataParallel(opt), x, y, grid)
        rs = np.random.RandomState(11)
        for _ in range(steps):
            gs.step(rs.choice(100, rs.randint(50, 100)))
        torch.cuda.synchronize()
        gs.release()
    fno = m.FNO_input
    idx = np.random.RandomState(12).choice(100, 60)
    u = x[:, torch.as_tensor(idx, device="cuda")]
    B, L = u.shape[:2]
    inp = torch.cat((u.reshape(B * L, 1, 128, 128), grid.permute(2, 0, 1).unsqueeze(0).expand(B * L, 2, 128, 128)),
                    1).permute(0, 2, 3, 1).contiguous()
    names = [k for k, _ in fno.named_parameters()]
    p32 = {k: v.detach().cpu().clone().requires_grad_(True) for k, v in fno.state_dict().items()}
    p64 = {k: v.detach().double().requires_grad_(True) for k, v in fno.state_dict().items()}
    cots = {"random": torch.randn(B * L, 128, 128, 1, device="cuda"),
            "bag": torch.randn(B, 1, 128, 128, 1, device="cuda").expand(B, L, 128, 128, 1).reshape(B * L, 128, 128, 1)}
    for cname, cot in cots.items():
        for prm in fno.parameters():
            prm.grad = None
        for p in list(p32.values()) + list(p64.values()):
            p.grad = None
        out = ops.FNOFn.apply(fno.meta(3), inp, *fno_params(fno, 2))
        (out * cot).sum().backward()
        o64 = cpu_ref.fno2d_fft(p64, inp.double())
        (o64 * cot.double()).sum().backward()
        o32 = cpu_ref.fno2d_fft(p32, inp.cpu())
        (o32 * cot.cpu()).sum().backward()
        print(f"[{cname}] fwd gpu {rel(out.detach(), o64.detach()):.2e}  ref32 {rel(o32.detach(), o64.detach()):.2e}",
              flush=True)
        gp = dict(fno.named_parameters())
        for k in names:
            print(f"[{cname}] {k:28s} gpu {rel(gp[k].grad, p64[k].grad):.2e}  ref32 {rel(p32[k].grad, p64[k].grad):.2e}"
                  f"  |g| {float(p64[k].grad.norm()):.3e}", flush=True)
    # the bare first spectral layer on x0
    x0 = torch.nn.functional.pad((inp @ fno.fc0.weight.detach().T + fno.fc0.bias.detach()).permute(0, 3, 1, 2),
                                 [0, 32, 0, 32]).contiguous()
    s0 = fno.spectral_list[0]
    w1, w2 = s0._real_view()
    w1 = w1.detach().clone().requires_grad_(True)
    w2 = w2.detach().clone().requires_grad_(True)
    cot = torch.randn(B * L, 4, 160, 160, device="cuda")
    ys = ops.SpectralConvFn.apply(x0, w1, w2)
    (ys * cot).sum().backward()
    w1d, w2d = w1.detach().double().requires_grad_(True), w2.detach().double().requires_grad_(True)
    y64 = cpu_ref.spectral_conv2d_fft(x0.double(), w1d, w2d)
    (y64 * cot.double()).sum().backward()
    print(f"[spectral0] fwd {rel(ys.detach(), y64.detach()):.2e} dw1 {rel(w1.grad, w1d.grad):.2e} "
          f"dw2 {rel(w2.grad, w2d.grad):.2e}", flush=True)


if __name__ == "__main__":
    main()
