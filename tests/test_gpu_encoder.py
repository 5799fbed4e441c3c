"""NIO snapshot-encoder ConvBlocks on the HIP path vs plain PyTorch fp32 (needs a GPU).

ops.Conv2dFn (csrc/conv.hip, implicit GEMM on the fp32 matrix cores) replaces nn.Conv2d and
ops.BNActFn (csrc/batchnorm.hip) BatchNorm2d + LeakyReLU(0.2) of ConvBlock
(2d_FPE/Baselines.py:40-52).  References: F.conv2d / torch.nn.BatchNorm2d / F.leaky_relu in
fp64 on the same inputs.  Tolerances: one convolution or normalisation of fp32 data, rel-L2
<= 1e-5 (outputs and gradients), running statistics 1e-6; the whole ten-block encoder: see
test_encoder2d_matches_fp64.
"""
import pytest
import torch
import torch.nn.functional as F

from conftest import rel_l2

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import blindno
    blindno.load_library()


def _ref_bn_act(z, bn, slope, training):
    return F.leaky_relu(F.batch_norm(z, bn.running_mean, bn.running_var, bn.weight, bn.bias, training,
                                     bn.momentum, bn.eps), slope)


@pytest.mark.parametrize("shape,n", [((64, 5, 6, 8), 37), ((32, 7, 3, 7), 32), ((96, 3, 1, 1), 70)])
def test_bn_act_matches_torch(shape, n):
    from blindno import ops
    torch.manual_seed(0)
    Npad, C = shape[0], shape[1]
    z = (torch.randn(shape, dtype=torch.float64) * 2.0 + 3.0).cuda()   # |mean| > std
    z[n:] = float("nan")                                                 # padding rows never read
    bn = torch.nn.BatchNorm2d(C).cuda()
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
    ref = torch.nn.BatchNorm2d(C).double().cuda()
    ref.load_state_dict(bn.state_dict())
    for it in range(2):                                   # twice: running statistics compound
        zf = z.float().requires_grad_(True)
        y = ops.BNActFn.apply(zf, bn.weight, bn.bias, bn, n, 0.2)
        zr = z[:n].clone().requires_grad_(True)
        yr = _ref_bn_act(zr, ref, 0.2, True)
        assert n == Npad or float(y[n:].detach().abs().max()) == 0.0
        assert rel_l2(y[:n].detach().cpu().numpy(), yr.detach().cpu().numpy()) <= 1e-5
        cot = torch.randn_like(yr)
        bn.weight.grad = bn.bias.grad = None
        (y[:n] * cot.float()).sum().backward()
        (yr * cot).sum().backward()
        assert n == Npad or float(zf.grad[n:].abs().max()) == 0.0
        assert rel_l2(zf.grad[:n].cpu().numpy(), zr.grad.cpu().numpy()) <= 1e-5
        assert rel_l2(bn.weight.grad.cpu().numpy(), ref.weight.grad.cpu().numpy()) <= 1e-5
        assert rel_l2(bn.bias.grad.cpu().numpy(), ref.bias.grad.cpu().numpy()) <= 1e-5
        ref.weight.grad = ref.bias.grad = None
        assert rel_l2(bn.running_mean.cpu().numpy(), ref.running_mean.cpu().numpy()) <= 1e-6
        assert rel_l2(bn.running_var.cpu().numpy(), ref.running_var.cpu().numpy()) <= 1e-6
        assert int(bn.num_batches_tracked) == it + 1
    # eval mode: running statistics, no update
    bn.eval()
    ref.eval()
    rm = bn.running_mean.clone()
    zf = z.float().requires_grad_(True)
    y = ops.BNActFn.apply(zf, bn.weight, bn.bias, bn, n, 0.2)
    zr = z[:n].clone().requires_grad_(True)
    yr = _ref_bn_act(zr, ref, 0.2, False)
    assert rel_l2(y[:n].detach().cpu().numpy(), yr.detach().cpu().numpy()) <= 1e-5
    cot = torch.randn_like(yr)
    (y[:n] * cot.float()).sum().backward()
    (yr * cot).sum().backward()
    assert rel_l2(zf.grad[:n].cpu().numpy(), zr.grad.cpu().numpy()) <= 1e-5
    assert torch.equal(rm, bn.running_mean)


# every convolution shape of Encoder2D at 128^2 and 61^2 (the reference grid, odd sizes), of the
# 1D Encoder ((1, k) kernels), plus odd channel counts / strides / paddings
CONV_CASES = [
    # (N, Ci, Hi, Wi, Co, KH, KW, sh, sw, ph, pw)
    (6, 1, 128, 128, 64, 1, 7, 1, 2, 0, 3),
    (5, 64, 128, 64, 128, 3, 3, 2, 2, 1, 1),
    (5, 128, 64, 32, 128, 3, 3, 1, 1, 1, 1),
    (7, 256, 16, 8, 512, 3, 3, 2, 2, 1, 1),
    (7, 512, 8, 4, 512, 3, 3, 1, 1, 1, 1),
    (9, 512, 4, 2, 512, 3, 3, 2, 2, 1, 1),
    (9, 512, 4, 2, 512, 4, 2, 1, 1, 0, 0),
    (4, 1, 61, 61, 64, 1, 7, 1, 2, 0, 3),
    (3, 64, 61, 31, 128, 3, 3, 2, 2, 1, 1),
    (11, 256, 1, 20, 256, 1, 5, 1, 1, 0, 1),
    (3, 5, 13, 11, 7, 3, 2, 3, 2, 2, 1),
    # large enough for the 128 x 128 tiles (>= 512 tiles; csrc/conv.hip big_tiles) in the
    # forward and the input gradient, with a ragged last tile
    (66, 128, 64, 32, 128, 3, 3, 1, 1, 1, 1),
    (40, 128, 64, 32, 256, 3, 3, 2, 2, 1, 1),
    # 64 x 128 tiles (64-row GEMMs with >= 512 column tiles): the first block's forward and the
    # second block's input gradient
    (12, 1, 128, 128, 64, 1, 7, 1, 2, 0, 3),
    (9, 64, 128, 64, 128, 3, 3, 2, 2, 1, 1),
]


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv2d_matches_fp64(case):
    from blindno import ops
    N, Ci, Hi, Wi, Co, KH, KW, sh, sw, ph, pw = case
    torch.manual_seed(sum(case))
    x = torch.randn(N, Ci, Hi, Wi, device="cuda", dtype=torch.float64)
    w = torch.randn(Co, Ci, KH, KW, device="cuda", dtype=torch.float64) / (Ci * KH * KW) ** 0.5
    b = torch.randn(Co, device="cuda", dtype=torch.float64)
    xs, ws, bs = (t.float().requires_grad_(True) for t in (x, w, b))
    y = ops.conv2d(xs, ws, bs, (sh, sw), (ph, pw))
    x64, w64, b64 = (t.clone().requires_grad_(True) for t in (x, w, b))
    y64 = F.conv2d(x64, w64, b64, stride=(sh, sw), padding=(ph, pw))
    assert y.shape == y64.shape
    assert rel_l2(y.detach().cpu().numpy(), y64.detach().cpu().numpy()) <= 1e-5
    cot = torch.randn_like(y64)
    (y * cot.float()).sum().backward()
    (y64 * cot).sum().backward()
    for got, ref in ((xs.grad, x64.grad), (ws.grad, w64.grad), (bs.grad, b64.grad)):
        assert rel_l2(got.cpu().numpy(), ref.cpu().numpy()) <= 1e-5
    # deterministic: a second evaluation is bit-identical
    y2 = ops.conv2d(xs.detach(), ws.detach(), bs.detach(), (sh, sw), (ph, pw))
    assert torch.equal(y.detach(), y2)


SPLIT_CASES = [
    (9, 512, 4, 2, 512, 4, 2, 1, 1, 0, 0),    # the 1x1-output last block: split by default
    (5, 128, 64, 32, 128, 3, 3, 1, 1, 1, 1),   # tap-major with the weight re-layout (both modes)
    (9, 512, 4, 2, 512, 3, 3, 2, 2, 1, 1),
    (3, 5, 13, 11, 7, 3, 2, 3, 2, 2, 1),
    (4, 6, 9, 10, 5, 1, 1, 3, 2, 0, 0),       # stride > kernel: pixels with no taps (zero dx)
]


@pytest.mark.parametrize("case", SPLIT_CASES)
def test_conv2d_split_k(case):
    """blindno_conv2d_{fwd,bwd_data}_split at explicit split counts (1, 2, 3, the default) vs fp64;
    nsplit = 1 is bit-identical to the unsplit entries."""
    from blindno import ops
    from blindno._lib import call, ptr, query, stream_ptr
    N, Ci, Hi, Wi, Co, KH, KW, sh, sw, ph, pw = case
    torch.manual_seed(sum(case) + 1)
    x = torch.randn(N, Ci, Hi, Wi, device="cuda", dtype=torch.float64)
    w = torch.randn(Co, Ci, KH, KW, device="cuda", dtype=torch.float64) / (Ci * KH * KW) ** 0.5
    b = torch.randn(Co, device="cuda", dtype=torch.float64)
    y64 = F.conv2d(x, w, b, stride=(sh, sw), padding=(ph, pw))
    dy64 = torch.randn_like(y64)
    x64 = x.clone().requires_grad_(True)
    F.conv2d(x64, w, b, stride=(sh, sw), padding=(ph, pw)).backward(dy64)
    xs, ws, bs, dys = x.float(), w.float(), b.float(), dy64.float()
    g = case
    y1 = torch.empty_like(y64, dtype=torch.float32)
    call("blindno_conv2d_fwd", ptr(xs), ptr(ws), ptr(bs), ptr(y1), *g, stream_ptr())
    dx1 = torch.empty_like(xs)
    call("blindno_conv2d_bwd_data", ptr(dys), ptr(ws), ptr(dx1), *g, stream_ptr())
    splits = sorted({1, 2, 3, query("blindno_conv2d_fwd_nsplit", *g), query("blindno_conv2d_bwd_data_nsplit", *g)})
    nwf, nwd = (query("blindno_conv2d_wscratch_floats", m, *g) for m in (0, 1))
    wsf = torch.full((max(1, nwf),), float("nan"), device="cuda")
    wsd = torch.full((max(1, nwd),), float("nan"), device="cuda")
    for ns in splits:
        for use_ws in (False, True):   # the weight re-layout changes the loads, not the result
            y = torch.full_like(y1, float("nan"))
            part = torch.full((ns, y.numel()), float("nan"), device="cuda")
            call("blindno_conv2d_fwd_split", ptr(xs), ptr(ws), ptr(bs), ptr(y), ptr(part), ns,
                 ptr(wsf) if use_ws else None, *g, stream_ptr())
            dx = torch.full_like(xs, float("nan"))
            partd = torch.full((ns, dx.numel()), float("nan"), device="cuda")
            call("blindno_conv2d_bwd_data_split", ptr(dys), ptr(ws), ptr(dx), ptr(partd), ns,
                 ptr(wsd) if use_ws else None, *g, stream_ptr())
            torch.cuda.synchronize()
            assert rel_l2(y.cpu().numpy(), y64.cpu().numpy()) <= 1e-5, ns
            assert rel_l2(dx.cpu().numpy(), x64.grad.cpu().numpy()) <= 1e-5, ns
            if ns == 1 and not use_ws:
                assert torch.equal(y, y1) and torch.equal(dx, dx1)
            full = KH == Hi and KW == Wi and ph == 0 and pw == 0   # dense input gradient with W^T
            if use_ws:
                assert torch.equal(y, y_nows), ns
                assert full or torch.equal(dx, dx_nows), ns
            y_nows, dx_nows = y, dx
            # deterministic at every split count
            y2 = torch.empty_like(y)
            call("blindno_conv2d_fwd_split", ptr(xs), ptr(ws), ptr(bs), ptr(y2), ptr(part), ns,
                 ptr(wsf) if use_ws else None, *g, stream_ptr())
            assert torch.equal(y, y2)
    print(f"splits {splits}, weight scratch {nwf} / {nwd} floats")


WGRAD_CASES = [
    (5, 128, 64, 32, 128, 3, 3, 1, 1, 1, 1),   # N = 1152 + 1: the bias column outside the GEMM tiles
    (4, 64, 32, 16, 128, 3, 3, 2, 2, 1, 1),    # 576 + 1: a ragged last column tile
    (6, 1, 32, 32, 64, 1, 7, 1, 2, 0, 3),      # 7 + 1, 64 x 64 tiles
    (3, 5, 13, 11, 7, 3, 2, 3, 2, 2, 1),       # odd output plane: the scalar loaders, bias as a column
]


@pytest.mark.parametrize("case", WGRAD_CASES)
def test_conv2d_wgrad_bias_column_split(case):
    """blindno_conv2d_bwd_weight at split counts 1, 2, 7 and the default: the weight and bias
    gradient (Co, Ci KH KW + 1) against fp64, deterministic, and with the vectorised loaders the
    bias column formed from dy's row sums (ConvArgs::bsep) rather than a GEMM column."""
    from blindno._lib import call, ptr, query, stream_ptr
    N, Ci, Hi, Wi, Co, KH, KW, sh, sw, ph, pw = case
    torch.manual_seed(sum(case) + 7)
    x = torch.randn(N, Ci, Hi, Wi, device="cuda", dtype=torch.float64)
    w = torch.randn(Co, Ci, KH, KW, device="cuda", dtype=torch.float64, requires_grad=True)
    b = torch.randn(Co, device="cuda", dtype=torch.float64, requires_grad=True)
    y = F.conv2d(x, w, b, stride=(sh, sw), padding=(ph, pw))
    dy = torch.randn_like(y)
    y.backward(dy)
    ref = torch.cat([w.grad.reshape(Co, -1), b.grad[:, None]], 1)
    xs, dys = x.float().contiguous(), dy.float().contiguous()
    g = case
    for ns in sorted({1, 2, 7, query("blindno_conv2d_wgrad_nsplit", *g)}):
        outs = []
        for _ in range(2):
            dwb = torch.full((Co, Ci * KH * KW + 1), float("nan"), device="cuda")
            part = torch.full((ns, dwb.numel()), float("nan"), device="cuda")
            call("blindno_conv2d_bwd_weight", ptr(dys), ptr(xs), ptr(dwb), ptr(part), ns, *g, stream_ptr())
            outs.append(dwb)
        torch.cuda.synchronize()
        assert torch.isfinite(outs[0]).all(), ns
        assert rel_l2(outs[0][:, :-1].cpu().numpy(), ref[:, :-1].cpu().numpy()) <= 1e-5, ns
        assert rel_l2(outs[0][:, -1].cpu().numpy(), ref[:, -1].cpu().numpy()) <= 1e-5, ns
        assert torch.equal(outs[0], outs[1]), ns


def _branch_masks(enc):
    """Forward hooks recording each ConvBlock's LeakyReLU branch (output > 0 <=> pre-activation > 0)."""
    masks, hooks = [], []
    for name in ("convblock1", "convblock2_1", "convblock2_2", "convblock3_1", "convblock3_2", "convblock4_1",
                 "convblock4_2", "convblock7_1", "convblock7_2", "convblock7_3"):
        hooks.append(getattr(enc, name).register_forward_hook(lambda mod, i, o: masks.append(o.detach() > 0)))
    return masks, hooks


def test_encoder2d_matches_fp64():
    """Encoder2D (64x64 snapshots, 2 bags of 37, train-mode BatchNorm) on the HIP path vs the same
    modules in fp64.  The model is piecewise linear (LeakyReLU): a pre-activation within fp32
    rounding of 0 may take either branch in two correct evaluations, and one such flip moves a
    gradient by ~1e-3 rel-L2 (tools/diag_encoder_bwd.py / diag_bn.py: plain fp32 torch lands at
    1e-6 or 2e-3 on the same tensor depending on whether it flipped).  So the fp64 evaluation takes
    every LeakyReLU branch from the HIP forward (hooks on the blocks) -- the same linear piece --
    and the SURVEY 8c bars then hold as fixed numbers: output <= 1e-5, every gradient <= 1e-4."""
    import blindno
    torch.manual_seed(1)
    enc = blindno.Encoder2D(25, last_kernel=blindno.Encoder2D.kernel_for_grid(64)).cuda().train()
    ref64 = blindno.Encoder2D(25, last_kernel=blindno.Encoder2D.kernel_for_grid(64)).cuda().double().train()
    ref64.load_state_dict(enc.state_dict())
    x = torch.randn(2, 37, 1, 64, 64, device="cuda")
    masks, hooks = _branch_masks(enc)
    out = enc(x)
    for h in hooks:
        h.remove()
    assert len(masks) == 10

    def ref_fwd(m, x):
        b, L = x.shape[:2]
        h = x.reshape(b * L, 1, 64, 64)
        for blk, mask in zip((m.convblock1, m.convblock2_1, m.convblock2_2, m.convblock3_1, m.convblock3_2,
                              m.convblock4_1, m.convblock4_2, m.convblock7_1, m.convblock7_2, m.convblock7_3),
                             masks):
            z = blk.layers[1](blk.layers[0](h))
            h = torch.where(mask, z, blk.relu_slope * z)
        return m.linear(h.flatten(1).view(b, L, -1))

    out64 = ref_fwd(ref64, x.double())
    e_out = rel_l2(out.detach().cpu().numpy(), out64.detach().cpu().numpy())
    assert e_out <= 1e-5, e_out
    cot = torch.randn_like(out64)
    (out * cot.float()).sum().backward()
    (out64 * cot).sum().backward()
    p64 = dict(ref64.named_parameters())
    worst = []
    for k, p in enc.named_parameters():
        if k.endswith("layers.0.bias"):
            continue    # conv bias ahead of a batch-statistics BatchNorm: true gradient is exactly 0
        e = rel_l2(p.grad.cpu().numpy(), p64[k].grad.cpu().numpy())
        worst.append((e, k))
        assert e <= 1e-4, (k, e)
    print("encoder2d fwd", e_out, "worst grads", sorted(worst)[-3:])
    b64 = dict(ref64.named_buffers())
    for k, b in enc.named_buffers():
        if b.dtype.is_floating_point:
            assert rel_l2(b.cpu().numpy(), b64[k].cpu().numpy()) <= 1e-5, k


@pytest.mark.parametrize("M,K,N", [(300, 512, 25), (16384, 2, 100), (16384, 100, 100), (77, 100, 25)])
def test_linear_matches_fp64(M, K, N):
    """ops.linear (nn.Linear as a 1x1 convolution on csrc/conv.hip) vs F.linear in fp64: output,
    input / weight / bias gradients."""
    from blindno import ops
    torch.manual_seed(M + K + N)
    lin = torch.nn.Linear(K, N).cuda()
    x = torch.randn(M, K, device="cuda", requires_grad=True)
    y = ops.linear(x, lin.weight, lin.bias)
    cot = torch.randn_like(y)
    (y * cot).sum().backward()
    w64 = lin.weight.detach().double().requires_grad_(True)
    b64 = lin.bias.detach().double().requires_grad_(True)
    x64 = x.detach().double().requires_grad_(True)
    y64 = F.linear(x64, w64, b64)
    (y64 * cot.double()).sum().backward()
    assert rel_l2(y.detach().cpu().numpy(), y64.detach().cpu().numpy()) <= 1e-6
    for got, want in ((x.grad, x64.grad), (lin.weight.grad, w64.grad), (lin.bias.grad, b64.grad)):
        assert rel_l2(got.cpu().numpy(), want.cpu().numpy()) <= 1e-6


def test_ffn_trunk_native_matches_fp64():
    """The FFN trunk (2d_FPE/DeepONetModules.py:155-185: Linear -> LeakyReLU(0.01) -> [Linear ->
    LeakyReLU -> BatchNorm1d (batch statistics)] x 2 -> Linear) on libblindno vs the same module
    run by torch in fp64: output, every parameter gradient, the input gradient and the running
    statistics (two steps: they compound)."""
    import copy
    from blindno.deeponet import FFN
    torch.manual_seed(3)
    f = FFN(2, 25, 3, 100, "leaky_relu", 0.0).cuda().train()
    ref = copy.deepcopy(f).double()
    gx, gy = torch.meshgrid(torch.linspace(-1, 1, 128), torch.linspace(-1, 1, 128), indexing="ij")
    grid = torch.stack([gx, gy], -1).reshape(-1, 2).cuda()
    for it in range(2):
        x = grid.clone().requires_grad_(True)
        assert f._native_ok(x)
        y = f(x)
        cot = torch.randn_like(y)
        f.zero_grad()
        (y * cot).sum().backward()
        x64 = grid.double().requires_grad_(True)
        ref.zero_grad()
        y64 = ref(x64)
        (y64 * cot.double()).sum().backward()
        assert rel_l2(y.detach().cpu().numpy(), y64.detach().cpu().numpy()) <= 1e-5
        assert rel_l2(x.grad.cpu().numpy(), x64.grad.cpu().numpy()) <= 1e-4
        p64 = dict(ref.named_parameters())
        for k, p in f.named_parameters():
            assert rel_l2(p.grad.cpu().numpy(), p64[k].grad.cpu().numpy()) <= 1e-4, k
        b64 = dict(ref.named_buffers())
        for k, b in f.named_buffers():
            if b.is_floating_point():
                assert rel_l2(b.cpu().numpy(), b64[k].cpu().numpy()) <= 1e-6, k
            else:
                assert int(b) == int(b64[k]) == it + 1, k


def test_ffn_trunk_nearly_constant_upstream_gradient():
    """The trunk as config D trains it: its upstream gradient dL/dbasis is rank B = 4 over the
    16384 grid points and nearly constant, so the BatchNorm1d backward subtracts a batch mean that
    all but cancels the gradient, and every fp32 evaluation carries an error floor of eps times
    the cancellation ratio.  Bar: the reference's own fp32 execution (torch on the CPU, whose
    BatchNorm sums in fp64 like csrc/batchnorm.hip) sets the floor; the native trunk stays within
    3x of it (or 1e-4).  torch's GPU BatchNorm (fp32 sums) is printed for context: what fp32 batch
    sums cost here (config D's trunk gradients: 1.4e-3 before the fp64 sums, bench parity leg)."""
    import copy
    from blindno.deeponet import FFN
    torch.manual_seed(5)
    f = FFN(2, 25, 3, 100, "leaky_relu", 0.0).cuda().train()
    ref = copy.deepcopy(f).double()
    cpu = copy.deepcopy(f).cpu()
    gx, gy = torch.meshgrid(torch.linspace(0, 1, 128), torch.linspace(0, 1, 128), indexing="ij")
    grid = torch.stack([gx, gy], -1).reshape(-1, 2).cuda()
    g = torch.Generator(device="cuda").manual_seed(6)
    cot = (torch.randn(1, 25, device="cuda", generator=g)
           + 1e-2 * torch.randn(grid.shape[0], 25, device="cuda", generator=g))
    y = f(grid)
    f.zero_grad()
    y.backward(cot)
    ref.zero_grad()
    ref(grid.double()).backward(cot.double())
    cpu.zero_grad()
    cpu(grid.cpu()).backward(cot.cpu())
    tg = copy.deepcopy(f)
    tg.zero_grad()
    tg._native_ok = lambda x: False           # torch's fp32 GPU ops, for context
    tg(grid).backward(cot)
    p64, pc, pt = dict(ref.named_parameters()), dict(cpu.named_parameters()), dict(tg.named_parameters())
    for k, p in f.named_parameters():
        want = p64[k].grad.cpu().numpy()
        e = rel_l2(p.grad.cpu().numpy(), want)
        ec = rel_l2(pc[k].grad.numpy(), want)
        et = rel_l2(pt[k].grad.cpu().numpy(), want)
        print(f"  {k:24s} native {e:.2e}  cpu fp32 {ec:.2e}  torch-gpu fp32 {et:.2e}")
        assert e <= max(1e-4, 3.0 * ec), k


@pytest.mark.parametrize("B,L,S,weighted", [(4, 75, 16384, False), (2, 51, 80, True), (3, 1, 6400, False),
                                             (130, 7, 600, True), (2, 1500, 300, False)])
def test_deeponet_bag_matches_fp64(B, L, S, weighted):
    """ops.DeepONetBagFn (DeepOnetNoBiasOrg + the bag mean that reads it, csrc/deeponet.hip) vs
    the reference composition in fp64: mean_l ((w basis^T + b0) / sqrt(P)), with 1/L or
    multiplicity weights; ubar and the gradients of w, basis and b0.  B = 130 runs the backward
    as three bag chunks (64 + 64 + 2, dbasis / db0 summed over them); L = 1500 is past the old
    1024-snapshot bound."""
    from blindno import ops
    torch.manual_seed(B * L + S)
    P = 25
    w = torch.randn(B, L, P, device="cuda", requires_grad=True)
    basis = torch.randn(S, P, device="cuda", requires_grad=True)
    b0 = torch.tensor(0.3, device="cuda", requires_grad=True)
    lw = None
    if weighted:
        c = torch.randint(1, 4, (L,), device="cuda").float()
        lw = c / c.sum()
    ubar = ops.DeepONetBagFn.apply(w, basis, b0, lw)
    cot = torch.randn_like(ubar)
    (ubar * cot).sum().backward()
    w64, bs64, b064 = (t.detach().double().requires_grad_(True) for t in (w, basis, b0))
    u = (w64 @ bs64.T + b064) / P ** 0.5
    ref = u.mean(1) if lw is None else (u * lw.double().view(1, L, 1)).sum(1)
    (ref * cot.double()).sum().backward()
    assert rel_l2(ubar.detach().cpu().numpy(), ref.detach().cpu().numpy()) <= 1e-6
    for got, want in ((w.grad, w64.grad), (basis.grad, bs64.grad)):
        assert rel_l2(got.cpu().numpy(), want.cpu().numpy()) <= 1e-6
    # db0 = sum of B S cotangents / sqrt(P): a cancelling sum, so the bar is relative to its
    # absolute sum (fp32 accumulation over 1e4-1e5 terms)
    assert abs(float(b0.grad) - float(b064.grad)) <= 1e-6 * float(cot.double().abs().sum()) / P ** 0.5
