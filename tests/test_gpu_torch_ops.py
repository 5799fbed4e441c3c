"""torch.ops.blindno.* on the GPU (blindno.torch_ops): every registered operator against the float64
oracle (oracle.fno_ref, plain torch ops on the GPU) or a float64 torch evaluation of the same
formula, forward and autograd backward, plus torch.library.opcheck's schema / fake-tensor /
autograd-registration checks.  Tolerances as in test_gpu_parity: fp32 HIP vs fp64, forward rel-L2
<= 1e-5, gradients <= 1e-4."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import rel_l2

pytestmark = pytest.mark.gpu

FWD_TOL = 1e-5
GRAD_TOL = 1e-4


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import blindno
    blindno.load_library()


def _err(a, b):
    return rel_l2(a.detach().cpu().numpy(), b.detach().cpu().numpy())


def _grads(out, ins, cot):
    return torch.autograd.grad(out, ins, cot)


@pytest.mark.parametrize("geom", [(3, 3, 4, 20, 18, 4, 5), (2, 2, 3, 6, 10, 4, 6), (2, 8, 8, 40, 40, 12, 12)])
def test_spectral_conv2d_op(geom):
    from blindno import torch_ops  # noqa: F401
    import oracle.fno_ref as ref
    Bn, Ci, Co, P1, P2, m1, m2 = geom
    g = torch.Generator(device="cuda").manual_seed(11)
    x = torch.randn(Bn, Ci, P1, P2, device="cuda", generator=g, requires_grad=True)
    w1 = (0.3 * torch.randn(Ci, Co, m1, m2, 2, device="cuda", generator=g)).requires_grad_(True)
    w2 = (0.3 * torch.randn(Ci, Co, m1, m2, 2, device="cuda", generator=g)).requires_grad_(True)
    y, X = torch.ops.blindno.spectral_conv2d(x, w1, w2)
    assert not X.requires_grad or X.grad_fn is not None
    xd, w1d, w2d = (t.detach().double().requires_grad_(True) for t in (x, w1, w2))
    yr = ref.spectral_conv2d(xd, w1d, w2d)
    assert _err(y, yr) <= FWD_TOL
    cot = torch.randn_like(y)
    got = _grads(y, (x, w1, w2), cot)
    exp = _grads(yr, (xd, w1d, w2d), cot.double())
    for a, b in zip(got, exp):
        assert _err(a, b) <= GRAD_TOL


def test_spectral_conv1d_op():
    from blindno import torch_ops  # noqa: F401
    import oracle.fno_ref as ref
    g = torch.Generator(device="cuda").manual_seed(12)
    x = torch.randn(3, 4, 20, device="cuda", generator=g, requires_grad=True)
    w = (0.3 * torch.randn(4, 5, 11, dtype=torch.complex64, device="cuda", generator=g)).requires_grad_(True)
    y, _ = torch.ops.blindno.spectral_conv1d(x, w)
    xd, wd = x.detach().double().requires_grad_(True), w.detach().to(torch.complex128).requires_grad_(True)
    yr = ref.spectral_conv1d(xd, wd)
    assert _err(y, yr) <= FWD_TOL
    cot = torch.randn_like(y)
    for a, b in zip(_grads(y, (x, w), cot), _grads(yr, (xd, wd), cot.double())):
        assert _err(a, b) <= GRAD_TOL


@pytest.mark.parametrize("dim", [2, 1])
def test_fno_op_matches_module_and_oracle(dim):
    from blindno import torch_ops  # noqa: F401
    from blindno.fno import FNO1d, FNO2d, fno_params
    import oracle.fno_ref as ref
    torch.manual_seed(5)
    if dim == 2:
        m = FNO2d(6, 8, 3, 5, 1).cuda()
        inp = torch.randn(2, 24, 20, 5, device="cuda")
    else:
        m = FNO1d(7, 8, 2, 3, 2).cuda()
        inp = torch.randn(4, 30, 3, device="cuda")
    inp.requires_grad_(True)
    params = fno_params(m, dim)
    out_mod = m(inp)
    if dim == 2:
        out = torch.ops.blindno.fno2d(inp, params, m.n_layers, m.modes1, m.modes2)
    else:
        out = torch.ops.blindno.fno1d(inp, params, m.n_layers, m.modes)
    assert torch.equal(out, out_mod)                   # same launch sequence as FNOFn
    cot = torch.randn_like(out)
    got = _grads(out, [inp] + list(m.parameters()), cot)
    exp_mod = _grads(out_mod, [inp] + list(m.parameters()), cot)
    for a, b in zip(got, exp_mod):
        assert _err(a, b) <= 1e-6
    p = {k: v.detach().to(torch.complex128 if v.is_complex() else torch.float64).requires_grad_(True)
         for k, v in m.state_dict().items()}
    ind = inp.detach().double().requires_grad_(True)
    yr = (ref.fno2d if dim == 2 else ref.fno1d)(p, ind)
    assert _err(out, yr) <= FWD_TOL
    exp = _grads(yr, [ind] + [p[k] for k, _ in m.named_parameters()], cot.double())
    for a, b in zip(got, exp):
        assert _err(a, b) <= GRAD_TOL


def test_project_mlp_op():
    from blindno import torch_ops  # noqa: F401
    g = torch.Generator(device="cuda").manual_seed(13)
    Bn, C, P1, P2, Ho, Wo, Hd, Co = 3, 8, 30, 25, 24, 20, 128, 2
    z = torch.randn(Bn, C, P1, P2, device="cuda", generator=g, requires_grad=True)
    w1 = (0.2 * torch.randn(Hd, C, device="cuda", generator=g)).requires_grad_(True)
    b1 = (0.1 * torch.randn(Hd, device="cuda", generator=g)).requires_grad_(True)
    w2 = (0.1 * torch.randn(Co, Hd, device="cuda", generator=g)).requires_grad_(True)
    b2 = (0.1 * torch.randn(Co, device="cuda", generator=g)).requires_grad_(True)
    out = torch.ops.blindno.project_mlp(z, w1, b1, w2, b2, Ho, Wo)
    ins = (z, w1, b1, w2, b2)
    d = [t.detach().double().requires_grad_(True) for t in ins]
    h = d[0][:, :, :Ho, :Wo].permute(0, 2, 3, 1)
    yr = F.linear(F.gelu(F.linear(h, d[1], d[2])), d[3], d[4])
    assert _err(out, yr) <= FWD_TOL
    cot = torch.randn_like(out)
    for a, b in zip(_grads(out, ins, cot), _grads(yr, d, cot.double())):
        assert _err(a, b) <= GRAD_TOL


def test_bag_mean_op():
    from blindno import torch_ops  # noqa: F401
    import oracle.fno_ref as ref
    g = torch.Generator(device="cuda").manual_seed(14)
    B, L, S, width = 3, 5, 37 * 29, 16
    u = torch.randn(B, L, S, device="cuda", generator=g, requires_grad=True)
    grid = torch.rand(S, 2, device="cuda", generator=g)
    w = torch.randn(width, 3, device="cuda", generator=g)
    b = torch.randn(width, device="cuda", generator=g)
    y = torch.ops.blindno.bag_mean(u, grid, w, b)
    ud = u.detach().double().requires_grad_(True)
    yr = ref.bag_mean(ud, grid.t().unsqueeze(0).expand(B, 2, S).double(), w, b)
    assert _err(y, yr) <= FWD_TOL
    cot = torch.randn_like(y)
    assert _err(_grads(y, u, cot)[0], _grads(yr, ud, cot.double())[0]) <= GRAD_TOL


@pytest.mark.parametrize("geom", [(7, 1, 70, 70, 16, 3, 2, 1), (4, 16, 35, 35, 32, 3, 2, 1), (2, 3, 9, 11, 5, 3, 1, 1)])
def test_conv2d_op(geom):
    from blindno import torch_ops  # noqa: F401
    N, Ci, H, W, Co, K, s, p = geom
    g = torch.Generator(device="cuda").manual_seed(15)
    x = torch.randn(N, Ci, H, W, device="cuda", generator=g, requires_grad=True)
    w = (0.2 * torch.randn(Co, Ci, K, K, device="cuda", generator=g)).requires_grad_(True)
    b = (0.1 * torch.randn(Co, device="cuda", generator=g)).requires_grad_(True)
    y = torch.ops.blindno.conv2d(x, w, b, [s, s], [p, p])
    d = [t.detach().double().requires_grad_(True) for t in (x, w, b)]
    yr = F.conv2d(d[0], d[1], d[2], s, p)
    assert _err(y, yr) <= FWD_TOL
    cot = torch.randn_like(y)
    for a, bb in zip(_grads(y, (x, w, b), cot), _grads(yr, d, cot.double())):
        assert _err(a, bb) <= GRAD_TOL


def test_mse_and_metric_ops():
    from blindno import torch_ops  # noqa: F401
    import oracle.fno_ref as ref
    g = torch.Generator(device="cuda").manual_seed(16)
    pred = torch.randn(4, 33, 17, 2, device="cuda", generator=g, requires_grad=True)
    tgt = torch.randn(4, 33, 17, 2, device="cuda", generator=g)
    loss = torch.ops.blindno.mse_loss(pred, tgt)
    pd = pred.detach().double().requires_grad_(True)
    lr = ((pd - tgt.double()) ** 2).mean()
    assert abs(loss.item() - lr.item()) <= 1e-6 * lr.item()
    assert _err(_grads(loss, pred, None)[0], _grads(lr, pd, None)[0]) <= 1e-6
    pt = tgt[..., 0].reshape(4, -1)
    e = torch.ops.blindno.time_averaged_relative_l2(pred.detach()[..., 0].reshape(4, -1), pt)
    er = ref.time_averaged_relative_l2(pred.detach()[..., 0].reshape(4, -1).cpu().numpy(), pt.cpu().numpy())
    assert e.dtype == torch.float64 and abs(e.item() - er) <= 1e-6 * er


def test_opcheck():
    from blindno import torch_ops  # noqa: F401
    utils = ("test_schema", "test_autograd_registration", "test_faketensor")
    x = torch.randn(2, 3, 20, 18, device="cuda", requires_grad=True)
    w = torch.randn(3, 4, 4, 5, 2, device="cuda", requires_grad=True)
    torch.library.opcheck(torch.ops.blindno.spectral_conv2d, (x, w, w.detach().clone().requires_grad_(True)),
                          test_utils=utils)
    xc = torch.randn(2, 3, 9, 11, device="cuda", requires_grad=True)
    wc = torch.randn(5, 3, 3, 3, device="cuda", requires_grad=True)
    bc = torch.randn(5, device="cuda", requires_grad=True)
    torch.library.opcheck(torch.ops.blindno.conv2d, (xc, wc, bc, [2, 2], [1, 1]), test_utils=utils)
    pred = torch.randn(5, 7, device="cuda", requires_grad=True)
    torch.library.opcheck(torch.ops.blindno.mse_loss, (pred, torch.randn(5, 7, device="cuda")), test_utils=utils)


def test_unet_ops_match_functions_and_opcheck():
    """torch.ops.blindno.{depthwise_conv, convnext_pointwise, max_pool, conv_transpose,
    temporal_attention_mean} give the blindno.unet autograd Functions' values and gradients
    (the same kernels), and pass torch.library.opcheck (schema, autograd registration, fake)."""
    from blindno import torch_ops  # noqa: F401
    from blindno import unet
    torch.manual_seed(3)
    utils = ("test_schema", "test_autograd_registration", "test_faketensor")

    def leaf(*shape):
        return torch.randn(*shape, device="cuda", requires_grad=True)

    cases = [
        (torch.ops.blindno.depthwise_conv, unet.DWConvFn.apply, (leaf(3, 4, 9, 8), leaf(4, 1, 7, 7), leaf(4))),
        (torch.ops.blindno.convnext_pointwise, unet.CnxPwFn.apply,
         (leaf(3, 4, 5, 6), leaf(3, 4, 5, 6), leaf(4), leaf(4), leaf(16, 4), leaf(16), leaf(4, 16), leaf(4))),
        (torch.ops.blindno.conv_transpose, unet.ConvTFn.apply, (leaf(2, 4, 5, 5), leaf(4, 3, 2, 2), leaf(3), 11, 10)),
        (torch.ops.blindno.temporal_attention_mean, unet.TokAttnMeanFn.apply,
         (leaf(2, 9, 40), leaf(40), leaf(40), 1e-5)),
    ]
    for op, fn, args in cases:
        y_op = op(*args)
        y_op = y_op[0] if isinstance(y_op, tuple) else y_op
        g = torch.randn_like(y_op)
        ts = [a for a in args if torch.is_tensor(a)]
        gr_op = torch.autograd.grad(y_op, ts, g)
        y_fn = fn(*args)
        gr_fn = torch.autograd.grad(y_fn, ts, g)
        assert torch.equal(y_op, y_fn)
        for a, b in zip(gr_op, gr_fn):
            assert torch.equal(a, b)
        torch.library.opcheck(op, args, test_utils=utils)
    x = leaf(2, 3, 7, 6)
    y, arg = torch.ops.blindno.max_pool(x, 2, 2)
    assert torch.equal(y, unet.MaxPoolFn.apply(x, 2, 2))
    torch.library.opcheck(torch.ops.blindno.max_pool, (x, 2, 2), test_utils=utils)
