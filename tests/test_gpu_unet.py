"""PermInvUNet_attn ("BlinDNO") on the HIP path (needs a GPU).

Kernel tests compare each op of csrc/unet.hip with the float64 definition on the CPU (torch
functional ops in fp64 / oracle.unet_ref): one fp32 kernel, so outputs and gradients within
rel-L2 1e-5 (the temporal attention's fp32 Gram / softmax: 2e-5).  Model tests run the drop-in
classes (blindno.unet) on the reference goldens' inputs and recipe parameters and compare with
the float64 oracle (pinned to the reference by tests/test_oracle_golden.py) and the reference's
fp32 outputs: forward 1e-5, gradients max(1e-4, 3 x the fp32 envelope: the largest distance
from fp64 among fp32 evaluations of the same model -- the oracle in fp32, unperturbed and under
three fp32-rounding-sized input perturbations, and the reference's own gradients).
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

import oracle
from conftest import load_golden, rel_l2

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import blindno
    blindno.load_library()


def _leaf(t):
    return t.detach().clone().cuda().float().requires_grad_(True)


def _grads(ts):
    return [t.grad.detach().double().cpu() for t in ts]


# ---------------------------------------------------------------------------------- kernels

@pytest.mark.parametrize("N,C,H,W,k", [(6, 3, 13, 11, (7, 7)), (5, 16, 3, 3, (7, 7)), (40, 2, 1, 40, (1, 7)),
                                       (3, 1, 61, 61, (7, 7)), (2, 8, 2, 1, (7, 7))])
def test_dwconv(N, C, H, W, k):
    from blindno.unet import DWConvFn
    torch.manual_seed(1)
    x = torch.randn(N, C, H, W, dtype=torch.float64)
    w = torch.randn(C, 1, *k, dtype=torch.float64) * 0.2
    b = torch.randn(C, dtype=torch.float64)
    g = torch.randn(N, C, H, W, dtype=torch.float64)
    ref = [t.clone().requires_grad_(True) for t in (x, w, b)]
    yr = F.conv2d(ref[0], ref[1], ref[2], padding=(k[0] // 2, k[1] // 2), groups=C)
    (yr * g).sum().backward()
    dev = [_leaf(t) for t in (x, w, b)]
    y = DWConvFn.apply(*dev)
    (y * g.cuda().float()).sum().backward()
    assert rel_l2(y.detach().cpu(), yr.detach()) <= 1e-5
    for a, r in zip(_grads(dev), ref):
        assert rel_l2(a, r.grad) <= 1e-5


@pytest.mark.parametrize("C,N,HW", [(1, 5, 3721), (2, 3, 900), (4, 7, 225), (8, 9, 49), (16, 4, 9),
                                    (32, 6, 5), (64, 40, 1)])
def test_convnext_pointwise(C, N, HW):
    """LayerNorm(C, 1e-6) -> Linear(C,4C) -> GELU -> Linear(4C,C) -> + shortcut
    (2d_FPE/NIOModules.py:1053-1062) vs fp64, forward and every gradient."""
    from blindno.unet import CnxPwFn
    torch.manual_seed(2)
    d = torch.float64
    xd = torch.randn(N, C, HW, dtype=d) * 1.5 + 0.3
    sc = torch.randn(N, C, HW, dtype=d)
    lw, lb = 1 + 0.2 * torch.randn(C, dtype=d), 0.1 * torch.randn(C, dtype=d)
    w1, b1 = torch.randn(4 * C, C, dtype=d) / C ** 0.5, 0.1 * torch.randn(4 * C, dtype=d)
    w2, b2 = torch.randn(C, 4 * C, dtype=d) / (4 * C) ** 0.5, 0.1 * torch.randn(C, dtype=d)
    g = torch.randn(N, C, HW, dtype=d)
    args = (xd, sc, lw, lb, w1, b1, w2, b2)

    def torch_ref(dt):
        ref = [t.to(dt).clone().requires_grad_(True) for t in args]
        h = F.layer_norm(ref[0].permute(0, 2, 1), (C,), ref[2], ref[3], 1e-6)
        h = F.gelu(h @ ref[4].T + ref[5]) @ ref[6].T + ref[7]
        yr = h.permute(0, 2, 1) + ref[1]
        (yr * g.to(dt)).sum().backward()
        return yr.detach().double(), [r.grad.double() for r in ref]

    yr, gr = torch_ref(d)
    _, g32 = torch_ref(torch.float32)          # conditioning: fp32 torch on the same inputs
    dev = [_leaf(t) for t in args]
    y = CnxPwFn.apply(dev[0].view(N, C, 1, HW), dev[1].view(N, C, 1, HW), *dev[2:])
    (y.view(N, C, HW) * g.cuda().float()).sum().backward()
    assert rel_l2(y.detach().cpu().view(N, C, HW), yr) <= 1e-5
    for i, (a, r, r32) in enumerate(zip(_grads(dev), gr, g32)):
        # LayerNorm over 1-2 channels makes dxd / dgamma cancellation-dominated: the bar is
        # max(1e-5, 3 x fp32 torch's own distance from fp64)
        bar = max(1e-5, 3 * rel_l2(r32, r))
        assert rel_l2(a, r) <= bar, (i, rel_l2(a, r), bar)


@pytest.mark.parametrize("N,C,H,W,k", [(3, 4, 61, 61, (2, 2)), (5, 2, 7, 6, (2, 2)), (7, 3, 1, 41, (1, 2))])
def test_maxpool(N, C, H, W, k):
    from blindno.unet import MaxPoolFn
    torch.manual_seed(3)
    x = torch.randn(N, C, H, W, dtype=torch.float64)
    x[0, 0, 0, :4] = 1.0                     # ties: the first maximum in scan order wins
    x = x.float().double()
    g = torch.randn(N, C, H // k[0], W // k[1], dtype=torch.float64)
    xr = x.clone().requires_grad_(True)
    yr = F.max_pool2d(xr, k)
    (yr * g).sum().backward()
    xd = _leaf(x)
    y = MaxPoolFn.apply(xd, *k)
    (y * g.cuda().float()).sum().backward()
    assert torch.equal(y.detach().cpu().double(), yr.detach())
    assert rel_l2(xd.grad.cpu(), xr.grad) <= 1e-7


@pytest.mark.parametrize("N,Ci,Co,Hi,Wi,k,op", [(4, 16, 8, 3, 3, (2, 2), (1, 1)), (2, 4, 2, 15, 15, (2, 2), (0, 0)),
                                                (3, 2, 1, 30, 30, (2, 2), (1, 0)), (5, 8, 4, 1, 5, (1, 2), (0, 1))])
def test_conv_transpose(N, Ci, Co, Hi, Wi, k, op):
    from blindno.unet import ConvTFn
    torch.manual_seed(4)
    d = torch.float64
    x = torch.randn(N, Ci, Hi, Wi, dtype=d)
    w = torch.randn(Ci, Co, *k, dtype=d) * 0.3
    b = torch.randn(Co, dtype=d)
    ref = [t.clone().requires_grad_(True) for t in (x, w, b)]
    yr = F.conv_transpose2d(ref[0], ref[1], ref[2], stride=k, output_padding=op)
    g = torch.randn(yr.shape, dtype=d)
    (yr * g).sum().backward()
    dev = [_leaf(t) for t in (x, w, b)]
    y = ConvTFn.apply(*dev, yr.shape[2], yr.shape[3])
    (y * g.cuda().float()).sum().backward()
    assert rel_l2(y.detach().cpu(), yr.detach()) <= 1e-5
    for a, r in zip(_grads(dev), ref):
        assert rel_l2(a, r.grad) <= 1e-5


@pytest.mark.parametrize("B,L,D,scale", [(2, 57, 3721, 1.0), (4, 99, 144, 1.0), (3, 1, 900, 1.0), (1, 7, 5000, 0.3),
                                         (2, 64, 80, 3.0), (2, 150, 2048, 0.5)])
def test_temporal_attention_bag_mean(B, L, D, scale):
    """mean_l LayerNorm_D(softmax(X X^T/sqrt D) X + X)_l (2d_FPE/NIOModules.py:1065-1083,
    1163-1164) vs the oracle's literal form in fp64; X with a per-token offset (centring)."""
    from blindno.unet import TokAttnMeanFn
    torch.manual_seed(5)
    d = torch.float64
    X = (torch.randn(B, L, D, dtype=d) + 0.5 * torch.randn(B, L, 1, dtype=d)) * scale
    lw, lb = 1 + 0.1 * torch.randn(D, dtype=d), 0.1 * torch.randn(D, dtype=d)
    g = torch.randn(B, D, dtype=d)
    ref = [t.clone().requires_grad_(True) for t in (X, lw, lb)]
    yr = oracle.unet_ref.temporal_attention({"norm.weight": ref[1], "norm.bias": ref[2]},
                                            ref[0].view(B, L, 1, D)).mean(1).view(B, D)
    (yr * g).sum().backward()
    dev = [_leaf(t) for t in (X, lw, lb)]
    y = TokAttnMeanFn.apply(*dev, 1e-5)
    (y * g.cuda().float()).sum().backward()
    assert rel_l2(y.detach().cpu(), yr.detach()) <= 2e-5
    for i, (a, r) in enumerate(zip(_grads(dev), ref)):
        assert rel_l2(a, r.grad) <= 2e-5 * (10 if i == 0 else 1), (i, rel_l2(a, r.grad))


# ---------------------------------------------------------------------------------- models

def _model(case):
    from blindno import unet
    from test_oracle_golden import unet_recipe_params
    g = load_golden(case)
    base, depth = int(g["base_ch"]), int(g["depth"])
    if case.startswith("unet1d"):
        n = g["in.x"].shape[2]
        cls = unet.PermInvUNet_attn1D_bag if "bag" in case else unet.PermInvUNet_attn1D
        m = cls(1, 2, base, depth, n, device="cpu")
    else:
        n = g["in.x"].shape[2]
        cls = unet.PermInvUNet_attn_NC if case.startswith("nc_") else unet.PermInvUNet_attn
        m = cls(1, 2, base, depth, (n, n))
    st = unet_recipe_params(g)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in st.items()})
    return m.cuda(), g


@pytest.mark.parametrize("case,dim,variant,train", [
    ("unet2d_train", 2, "fpe", True), ("unet2d_eval", 2, "fpe", False),
    ("nc_unet2d_train", 2, "nc", True), ("unet1d_bag_train", 1, "fpe", True),
    ("unet1d_all", 1, "fpe", True)])
def test_perminv_unet_attn_vs_oracle(case, dim, variant, train):
    from test_oracle_golden import unet_fp32_envelope, unet_grad_bar, unet_oracle_run
    m, g = _model(case)
    if "run_mean" in g:
        depth = int(g["depth"])
        chs = [int(g["base_ch"]) * 2 ** i for i in range(depth + 1)]
        off = np.cumsum([0] + chs)
        for i in range(depth + 1):
            m.skip_norms[i].running_mean.copy_(torch.from_numpy(g["run_mean"][off[i]:off[i + 1]]))
            m.skip_norms[i].running_var.copy_(torch.from_numpy(g["run_var"][off[i]:off[i + 1]]))
    m.train(train)
    x = torch.from_numpy(g["in.x"]).cuda().requires_grad_(True)
    idx = g["idx"].tolist() if "idx" in g else None
    y = m(x, bag_idx=idx)
    (y * torch.from_numpy(g["cot"]).cuda()).sum().backward()
    torch.cuda.synchronize()
    o64, g64, x64 = unet_oracle_run(g, dim, variant, train)
    env_o, env_g, env_x = unet_fp32_envelope(g, dim, variant, train, o64, g64, x64)
    yo = y.detach().double().cpu().numpy()
    assert rel_l2(yo, o64) <= max(1e-5, 3 * env_o), rel_l2(yo, o64)
    assert rel_l2(yo, g["out"]) <= 2e-5                      # the reference itself (fp32)
    scale = max(float(np.linalg.norm(v)) for v in g64.values())
    worst = (0.0, None)
    for k, p in m.named_parameters():
        if k not in g64:
            assert p.grad is None or float(p.grad.abs().max()) == 0.0, k    # unused heads
            continue
        if p.grad.is_complex():
            a = p.grad.detach().cpu().numpy().astype(np.complex128)
        else:
            a = p.grad.detach().double().cpu().numpy()
        if np.linalg.norm(g64[k]) <= 1e-10 * scale:
            assert np.linalg.norm(a) <= 1e-5 * scale, k       # conv bias before a train-mode BN
            continue
        e, e32 = rel_l2(a, g64[k]), env_g[k]
        assert e <= unet_grad_bar(e32), (k, e, e32)
        worst = max(worst, (e / unet_grad_bar(e32), k))
    assert rel_l2(x.grad.double().cpu().numpy(), x64) <= unet_grad_bar(env_x)
    # running statistics of the skip BatchNorms after a train-mode forward (momentum 0.1)
    if train and case in ("unet2d_train",):
        ev = load_golden("unet2d_eval")
        rm = np.concatenate([b.running_mean.cpu().numpy() for b in m.skip_norms])
        assert rel_l2(rm, ev["run_mean"]) <= 1e-5
    print(f"[{case}] fwd {rel_l2(yo, o64):.2e} worst grad / bar {worst[0]:.2f} ({worst[1]})")


@pytest.mark.parametrize("kind", ["attn", "nc"])
def test_unet_graph_replay_matches_eager(kind):
    """Three graphed training steps (train.GraphedBagStep: one graph per bag size) of the 2D
    UNet against three eager ones: parameters within 1e-6, and the BatchNorm buffers
    (running statistics and num_batches_tracked) as the eager steps leave them -- the capture's
    eager warm-up must not update them."""
    import blindno
    from blindno import unet
    from blindno.train import DataParallel, FlatAdam, GraphedBagStep, trained_parameters
    torch.manual_seed(0)
    B, T, N = 2, 60, 52
    x = torch.randn(B, T, N, N, device="cuda")
    y = torch.randn(B, N, N, 2, device="cuda")
    rs = np.random.RandomState(7)
    bags = [rs.choice(T, rs.randint(50, T)) for _ in range(3)]
    finals, bufs = [], []
    for graphed in (False, True):
        torch.manual_seed(1)
        if kind == "attn":
            m = unet.PermInvUNet_attn(1, 2, 1, 4, (N, N)).cuda().train()
        else:
            m = unet.PermInvUNet_attn_NC(1, 2, 1, 4, (N, N)).cuda().train()
        opt = FlatAdam(trained_parameters(m), lr=5e-4)
        if graphed:
            dp = DataParallel(opt)
            step = GraphedBagStep(m, blindno.mse_loss, opt, dp, x, y, None)
            for idx in bags:
                step.step(idx)
        else:
            for idx in bags:
                out = m(x, bag_idx=idx)
                loss = blindno.mse_loss(out, y)
                loss.backward()
                opt.gather_grads()
                opt.step()
                opt.zero_grad()
        torch.cuda.synchronize()
        finals.append(torch.cat([p.detach().reshape(-1) for p in m.parameters()]).cpu())
        bufs.append({k: b.detach().cpu().clone() for k, b in m.named_buffers()})
    assert rel_l2(finals[1].numpy(), finals[0].numpy()) <= 1e-6
    assert bufs[0].keys() == bufs[1].keys() and len(bufs[0]) > 0
    for k in bufs[0]:
        a, b = bufs[1][k], bufs[0][k]
        if a.is_floating_point():
            assert rel_l2(a.double().numpy(), b.double().numpy()) <= 1e-6, k
        else:
            assert torch.equal(a, b), (k, a, b)


@pytest.mark.parametrize("kind", ["bag_V", "bag_GPE"])
def test_unet_1d_gpe_copies_vs_oracle(kind):
    """The one-head 1d_GPE copies (1d_GPE/NIOModules.py:342-560) on seeded weights vs the fp64
    oracle (train mode, recorded bag): forward 1e-5, every gradient 1e-4 (fp32 envelope bar)."""
    from blindno import unet
    from test_oracle_golden import unet_grad_bar
    torch.manual_seed(11)
    if kind == "bag_V":
        m = unet.PermInvUNet_attn1D_bag_V(1, 2, 1, 4, 64, device="cpu")
    else:
        m = unet.PermInvUNet_attn1D_bag_GPE(1, 2, 2, 3, 48, device="cpu", width=12, modes=16)
    m = m.cuda().train()
    n = 64 if kind == "bag_V" else 48
    x = torch.randn(3, 60, n)
    rs = np.random.RandomState(3)
    idx = rs.choice(60, rs.randint(50, 60))
    cot = torch.randn(3, n, 1)
    y = m(x.cuda(), bag_idx=idx)
    (y * cot.cuda()).sum().backward()
    res = {}
    for prec, dt in (("fp64", torch.float64), ("fp32", torch.float32)):
        oracle.set_precision(prec)
        try:
            p = {k: (v.detach().cpu().to(torch.complex128 if v.is_complex() else dt).requires_grad_(True)
                     if v.is_floating_point() or v.is_complex() else v.cpu()) for k, v in m.state_dict().items()}
            if prec == "fp32":
                p = {k: (v.detach().to(torch.complex64).requires_grad_(True) if v.is_complex() else v)
                     for k, v in p.items()}
            yo = oracle.unet_ref.perminv_unet_attn(p, x.to(dt), m.depth, 1, idx=idx.tolist())
            (yo * cot.to(dt)).sum().backward()
        finally:
            oracle.set_precision("fp64")
        res[prec] = (yo.detach().double().numpy(), {k: v.grad for k, v in p.items()
                                                    if torch.is_tensor(v) and v.grad is not None})
    o64, g64 = res["fp64"]
    assert rel_l2(y.detach().double().cpu().numpy(), o64) <= 1e-5
    for k, prm in m.named_parameters():
        if k not in g64:
            continue
        a = prm.grad.detach().cpu()
        a = a.to(torch.complex128) if a.is_complex() else a.double()
        r, r32 = g64[k], res["fp32"][1][k]
        r32 = r32.to(torch.complex128) if r32.is_complex() else r32.double()
        if float(r.norm()) == 0.0:
            continue
        assert rel_l2(a.numpy(), r.detach().numpy()) <= unet_grad_bar(rel_l2(r32.numpy(), r.detach().numpy())), k
