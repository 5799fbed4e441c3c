"""HIP path vs the reference's golden vectors and the float64 oracle (needs a GPU).

Tolerances (fp32 kernels vs fp32 reference / fp64 oracle), stated per SURVEY.md 8c:
forward rel-L2 <= 1e-5, gradients rel-L2 <= 1e-4.
"""
import numpy as np
import pytest
import torch

from conftest import load_golden, rel_l2

pytestmark = pytest.mark.gpu

FWD_TOL = 1e-5
GRAD_TOL = 1e-4


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import blindno
    blindno.load_library()


def _load(module, g, strict=True):
    sd = {k[2:]: torch.from_numpy(v) for k, v in g.items() if k.startswith("p.")}
    missing, unexpected = module.load_state_dict(sd, strict=strict)
    assert not unexpected
    return module


def _run(module, g, fwd, inputs):
    module.cuda()
    ins = {k: torch.from_numpy(g["in." + k]).cuda().requires_grad_(("gin." + k) in g) for k in inputs}
    out = fwd(module, ins)
    torch.cuda.synchronize()
    assert rel_l2(out.detach().cpu().numpy(), g["out"]) <= FWD_TOL, rel_l2(out.detach().cpu().numpy(), g["out"])
    (out * torch.from_numpy(g["cot"]).cuda()).sum().backward()
    torch.cuda.synchronize()
    named = dict(module.named_parameters())
    n = 0
    for k, v in g.items():
        if k.startswith("g."):
            p = named[k[2:]]
            assert p.grad is not None, k
            e = rel_l2(p.grad.detach().cpu().numpy(), v)
            assert e <= GRAD_TOL, (k, e)
            n += 1
        elif k.startswith("gin."):
            e = rel_l2(ins[k[4:]].grad.detach().cpu().numpy(), v)
            assert e <= GRAD_TOL, (k, e)
            n += 1
    assert n > 0
    # parameters the reference leaves without gradient stay without gradient
    for name, p in named.items():
        if ("g." + name) not in g and not name.startswith("branch.") and p.grad is not None:
            assert float(p.grad.abs().max()) == 0.0, name


@pytest.mark.parametrize("case,args", [("sc2d_a", (3, 4, 4, 3)), ("sc2d_overlap", (2, 3, 5, 4)),
                                       ("sc2d_nyq", (2, 2, 3, 5))])
def test_spectral_conv2d(case, args):
    from blindno import SpectralConv2d
    g = load_golden(case)
    m = _load(SpectralConv2d(*args), g)
    _run(m, g, lambda m, i: m(i["x"]), ["x"])


@pytest.mark.parametrize("case,args", [("sc1d", (3, 4, 5)), ("sc1d_nyq", (2, 3, 9))])
def test_spectral_conv1d(case, args):
    from blindno import SpectralConv1d
    g = load_golden(case)
    m = _load(SpectralConv1d(*args), g)
    _run(m, g, lambda m, i: m(i["x"]), ["x"])


@pytest.mark.parametrize("case,args", [("fno2d", (4, 5, 3, 3, 1)), ("fno2d_input61", (12, 4, 2, 3, 1)),
                                       ("fno2d_head61", (32, 4, 2, 4, 1))])
def test_fno2d(case, args):
    from blindno import FNO2d
    g = load_golden(case)
    m = _load(FNO2d(*args), g)
    _run(m, g, lambda m, i: m(i["x"]), ["x"])


@pytest.mark.parametrize("case,args", [("fno1d", (5, 6, 3, 2, 2)), ("fno1d_input64", (12, 4, 2, 2, 1))])
def test_fno1d(case, args):
    from blindno import FNO1d
    g = load_golden(case)
    m = _load(FNO1d(*args), g)
    _run(m, g, lambda m, i: m(i["x"]), ["x"])


@pytest.mark.parametrize("case,heads,train", [("nio2d_fno_train", ("fno_drift", "fno_diffusion"), True),
                                              ("nio2d_fno_eval", ("fno_drift", "fno_diffusion"), False),
                                              ("nc_nio2d_fno_eval", ("fno_Fx", "fno_Fy"), False)])
def test_niofp2d_fno(case, heads, train):
    from blindno import NIOFP2D_FNO
    g = load_golden(case)
    m = _load(NIOFP2D_FNO(2, 3, 100, 25, 2, 6, 5, 2, heads=heads), g, strict=False)
    m.train(train)
    idx = g["idx"] if train else None
    _run(m, g, lambda m, i: m(i["x"], i["grid"], bag_idx=idx), ["x", "grid"])


@pytest.mark.parametrize("case,heads,train,args", [
    ("nio1d_fno_train", ("fno_drift", "fno_diffusion"), True, (3, 6, 5, 2)),
    ("nio1d_fno_eval", ("fno_drift", "fno_diffusion"), False, (3, 6, 5, 2)),
    ("gpe_nio_fno_train", ("fno_V",), True, (3, 5, 8, 1))])
def test_niofp_fno_1d(case, heads, train, args):
    from blindno import NIOFP_FNO
    g = load_golden(case)
    m = _load(NIOFP_FNO(*args, "cpu", heads=heads), g)
    m.train(train)
    idx = g["idx"] if train else None
    _run(m, g, lambda m, i: m(i["x"], i["grid"], bag_idx=idx), ["x", "grid"])


def test_niofp2d_fno_numpy_draw_matches_reference():
    """With no bag_idx, train mode must consume numpy's global RNG exactly like the
    reference (same L and idx under the same seed)."""
    from blindno import NIOFP2D_FNO
    g = load_golden("nio2d_fno_train")
    m = _load(NIOFP2D_FNO(2, 3, 100, 25, 2, 6, 5, 2), g, strict=False).cuda().train()
    x = torch.from_numpy(g["in.x"]).cuda()
    grid = torch.from_numpy(g["in.grid"]).cuda()
    np.random.seed(13)   # the seed the golden generator used
    out = m(x, grid)
    assert rel_l2(out.detach().cpu().numpy(), g["out"]) <= FWD_TOL


def test_niofp2d_fno_vs_oracle_64():
    """Mid-size NIOFP2D_FNO (64^2, T=60, B=2, config-C head geometry scaled) vs the fp64
    oracle -- shapes no fixture covers (P=80, FNO_input m=12 without row overlap)."""
    import oracle
    from blindno import NIOFP2D_FNO
    torch.manual_seed(5)
    m = NIOFP2D_FNO(2, 3, 100, 25, 3, 12, 16, 2).cuda().train()
    B, T, N = 2, 60, 64
    x = torch.randn(B, T, N, N).cuda()
    gx, gy = np.meshgrid(np.linspace(-1, 1, N, dtype=np.float32), np.linspace(-1, 1, N, dtype=np.float32),
                         indexing="ij")
    grid = torch.tensor(np.stack([gx, gy], 2)).cuda()
    rs = np.random.RandomState(3)
    idx = rs.choice(T, 57)
    out = m(x, grid, bag_idx=idx)
    cot = torch.randn_like(out)
    (out * cot).sum().backward()
    p = {k: v.detach().cpu().double().requires_grad_(True) for k, v in m.state_dict().items()
         if not k.startswith("branch.")}
    ref = oracle.niofp2d_fno(p, x.cpu(), grid.cpu(), idx=idx.tolist())
    assert rel_l2(out.detach().cpu().numpy(), ref.detach().numpy()) <= FWD_TOL
    (ref * cot.cpu().double()).sum().backward()
    for k, prm in m.named_parameters():
        if k in p and p[k].grad is not None and prm.grad is not None:
            e = rel_l2(prm.grad.cpu().numpy(), p[k].grad.numpy())
            assert e <= GRAD_TOL, (k, e)


@pytest.mark.parametrize("args,heads,N", [((3, 30, 15, 2), ("fno_drift", "fno_diffusion"), 64),
                                          ((3, 20, 40, 1), ("fno_V",), 256)])
def test_niofp_fno_1d_full_width_vs_oracle(args, heads, N):
    """The 1D models at the reference's own widths (configs A: width 30, B: width 20) vs the
    fp64 oracle: the head projections take the wide (C > 15) VALU kernels, which the
    width-5/6 fixtures never reach."""
    import oracle
    from blindno import NIOFP_FNO
    torch.manual_seed(11)
    m = NIOFP_FNO(*args, "cuda", heads=heads).cuda().train()
    B, T = 3, 40
    x = torch.randn(B, T, N).cuda()
    grid = torch.linspace(0, 1, N).unsqueeze(-1).cuda()
    idx = np.random.RandomState(4).choice(T, 33)
    out = m(x, grid, bag_idx=idx)
    cot = torch.randn_like(out)
    (out * cot).sum().backward()
    p = {k: (v.detach().cpu().to(torch.complex128) if v.is_complex() else v.detach().cpu().double())
         .requires_grad_(True) for k, v in m.state_dict().items()}
    ref = oracle.niofp_fno(p, x.cpu(), grid.cpu(), idx=idx.tolist(), heads=heads)
    assert rel_l2(out.detach().cpu().numpy(), ref.detach().numpy()) <= FWD_TOL
    (ref * cot.cpu().double()).sum().backward()
    n = 0
    for k, prm in m.named_parameters():
        if k in p and p[k].grad is not None and prm.grad is not None:
            e = rel_l2(prm.grad.cpu().numpy(), p[k].grad.numpy())
            assert e <= GRAD_TOL, (k, e)
            n += 1
    assert n > 10


def test_mse_and_metrics():
    from blindno import ops
    import oracle
    torch.manual_seed(0)
    p = torch.randn(3, 17, 19, 2, device="cuda", requires_grad=True)
    t = torch.randn(3, 17, 19, 2, device="cuda")
    loss = ops.mse_loss(p, t)
    loss.backward()
    ref = torch.nn.functional.mse_loss(p.detach().double(), t.double())
    assert abs(float(loss.detach()) - float(ref)) <= 1e-6 * float(ref)
    assert rel_l2(p.grad.cpu().numpy(), (2 * (p.detach() - t) / p.numel()).cpu().numpy()) <= 1e-6
    g = load_golden("metric_train_rel_l2")
    e0, e1 = ops.train_rel_l2_2ch(torch.from_numpy(g["pred"]).cuda(), torch.from_numpy(g["out"]).cuda())
    assert rel_l2(e0.cpu().numpy(), g["e_drift"]) <= 1e-6 and rel_l2(e1.cpu().numpy(), g["e_diffusion"]) <= 1e-6
    g = load_golden("metric_time_avg_rel_l2_2d")
    v = ops.time_averaged_relative_l2(torch.from_numpy(g["pt_pred"]).cuda(), torch.from_numpy(g["pt_ref"]).cuda())
    assert abs(v - float(g["val"])) <= 1e-5 * float(g["val"])  # inputs rounded to fp32


@pytest.mark.parametrize("case,heads,train", [("nio2d_fno_train", ("fno_drift", "fno_diffusion"), True),
                                              ("nio2d_fno_eval", ("fno_drift", "fno_diffusion"), False),
                                              ("nc_nio2d_fno_eval", ("fno_Fx", "fno_Fy"), False)])
def test_niofp2d_fno_fused_encoder(case, heads, train):
    """Same goldens through the fused snapshot-encoder path (ops.BagEncoderFn: bags read through
    the index list, lift folded into the first row DFT, fc0 gradient reduced in the adjoint),
    which NIOFP2D_FNO takes whenever x and grid need no gradient."""
    from blindno import NIOFP2D_FNO, ops
    g = load_golden(case)
    m = _load(NIOFP2D_FNO(2, 3, 100, 25, 2, 6, 5, 2, heads=heads), g, strict=False).cuda()
    m.train(train)
    x = torch.from_numpy(g["in.x"]).cuda()
    grid = torch.from_numpy(g["in.grid"]).cuda()
    assert m._fused_ok(x, grid)
    calls = []
    orig = ops.BagEncoderFn.forward
    ops.BagEncoderFn.forward = staticmethod(lambda *a: calls.append(1) or orig(*a))
    try:
        out = m(x, grid, bag_idx=g["idx"] if train else None)
    finally:
        ops.BagEncoderFn.forward = staticmethod(orig)
    assert calls, "fused encoder path not taken"
    assert rel_l2(out.detach().cpu().numpy(), g["out"]) <= FWD_TOL
    (out * torch.from_numpy(g["cot"]).cuda()).sum().backward()
    named = dict(m.named_parameters())
    n = 0
    for k, v in g.items():
        if k.startswith("g."):
            e = float(rel_l2(named[k[2:]].grad.detach().cpu().numpy(), v))
            assert e <= GRAD_TOL, (k, e)
            n += 1
    assert n > 20


@pytest.mark.parametrize("width,modes,N,B", [(12, 16, 64, 3), (6, 5, 16, 2)])
def test_head_pair_grouped_matches_separate_heads(width, modes, N, B):
    """The two heads batched into one chain of grouped launches (ops.fno_forward_grouped)
    against the same heads run one after the other through ops.FNOFn (tolerance: the
    reduction order of the weight gradients differs)."""
    from blindno import FNO2d, ops
    torch.manual_seed(21)
    heads = [FNO2d(modes, width, 3, width, 1).cuda() for _ in range(2)]
    h = torch.randn(B, N, N, width, device="cuda", requires_grad=True)
    side = torch.cuda.Stream()
    from blindno.fno import fno_params
    p0, p1 = fno_params(heads[0], 2), fno_params(heads[1], 2)
    assert ops.grouped_ok(heads[0].meta(width), h, [p0, p1])
    out = ops.HeadPairFn.apply(heads[0].meta(width), heads[1].meta(width), len(p0), side, h, *p0, *p1)
    cot = torch.randn_like(out)
    (out * cot).sum().backward()
    got = [p.grad.clone() for hd in heads for p in hd.parameters()]
    gh = h.grad.clone()
    for hd in heads:
        for p in hd.parameters():
            p.grad = None
    h.grad = None
    ref = torch.cat([heads[0](h), heads[1](h)], dim=-1)
    assert rel_l2(out.detach().cpu().numpy(), ref.detach().cpu().numpy()) <= 1e-6
    (ref * cot).sum().backward()
    want = [p.grad for hd in heads for p in hd.parameters()]
    # the grouped projection backward runs a coarser partial grid than the single head's
    # (blindno_project_bwd_nchunk_heads): fp32 sums over N^2 B points in another order,
    # ~sqrt(N^2 B) eps = 1.5e-5 apart at N = 64, B = 3
    for a, b in zip(got, want):
        assert rel_l2(a.cpu().numpy(), b.cpu().numpy()) <= 5e-5
    assert rel_l2(gh.cpu().numpy(), h.grad.cpu().numpy()) <= 1e-6


@pytest.mark.parametrize("width,modes,N,B", [(12, 16, 64, 3), (12, 32, 128, 4), (6, 5, 16, 2)])
def test_head_backward_merged_launch_bit_identical(width, modes, N, B):
    """The grouped heads' backward with the row DFT, the conv gradient and the previous layer's
    mix gradient in one launch per layer (blindno_rowdft_wgrad_g) against the three separate
    launches: every gradient bit-identical (each job keeps its own grid and summation order).
    (6, 5, 16, 2): C = 6 < the 12 of the heads, still the conv gradient's matrix-core form."""
    from blindno import FNO2d, ops
    from blindno.fno import fno_params
    torch.manual_seed(22)
    heads = [FNO2d(modes, width, 3, width, 1).cuda() for _ in range(2)]
    h = torch.randn(B, N, N, width, device="cuda", requires_grad=True)
    side = torch.cuda.Stream()
    p0, p1 = fno_params(heads[0], 2), fno_params(heads[1], 2)
    meta = heads[0].meta(width)
    Pm = ops._fno_geometry(h, meta)[4:6]
    assert ops.query("blindno_rowdft_wgrad_ok", 2 * B, width, Pm[0], Pm[1], meta.m2) == 1
    res = {}
    prev = ops.HEAD_BWD_MERGED
    try:
        for merged in (False, True):
            ops.HEAD_BWD_MERGED = merged
            for p in p0 + p1:
                p.grad = None
            h.grad = None
            out = ops.HeadPairFn.apply(meta, heads[1].meta(width), len(p0), side, h, *p0, *p1)
            cot = torch.randn(out.shape, generator=torch.Generator().manual_seed(5)).cuda()
            (out * cot).sum().backward()
            torch.cuda.synchronize()
            res[merged] = [p.grad.clone() for p in p0 + p1] + [h.grad.clone()]
    finally:
        ops.HEAD_BWD_MERGED = prev
    for a, b in zip(res[False], res[True]):
        assert torch.equal(a, b)


@pytest.mark.parametrize("dim", [2, 1])
def test_dedup_bag_matches_full_bag(dim):
    """A with-replacement bag run once per distinct snapshot (multiplicity weights in the bag
    mean and its gradient, nio.dedup_bag) against the same bag run snapshot by snapshot."""
    from blindno import NIOFP2D_FNO, NIOFP_FNO, nio
    torch.manual_seed(8)
    if dim == 2:
        m = NIOFP2D_FNO(2, 3, 100, 25, 3, 6, 8, 2).cuda().train()
        x = torch.randn(3, 60, 32, 32, device="cuda")
        gx, gy = np.meshgrid(np.linspace(-1, 1, 32, dtype=np.float32),
                             np.linspace(-1, 1, 32, dtype=np.float32), indexing="ij")
        grid = torch.tensor(np.stack([gx, gy], 2)).cuda()
    else:
        m = NIOFP_FNO(3, 30, 15, 2, "cuda").cuda().train()
        x = torch.randn(3, 60, 64, device="cuda")
        grid = torch.linspace(0, 1, 64, device="cuda").unsqueeze(-1)
    idx = np.random.RandomState(2).choice(60, 55)
    assert len(np.unique(idx)) < len(idx)
    res = []
    for dedup in (True, False):
        nio.DEDUP_BAGS = dedup
        try:
            m.zero_grad()
            out = m(x, grid, bag_idx=idx)
            (out * torch.linspace(-1, 1, out.numel(), device="cuda").view_as(out)).sum().backward()
            res.append((out.detach().cpu().numpy(), [p.grad.cpu().numpy() for p in m.FNO_input.parameters()]))
        finally:
            nio.DEDUP_BAGS = True
    assert rel_l2(res[0][0], res[1][0]) <= 1e-6
    for a, b in zip(res[0][1], res[1][1]):
        assert rel_l2(a, b) <= 1e-5


@pytest.mark.parametrize("N,B,dedup", [(32, 3, True), (30, 3, False), (61, 2, True)])
def test_bag_stats_projection_matches_per_snapshot(N, B, dedup):
    """The encoder's projection + bag mean at bag level (csrc/bagproj.hip: the forward leaves
    per-(bag, point) sums of GELU, GELU' and GELU' z; the backward reduces them) against the
    per-snapshot projection kernels plus the bag-mean kernel on the same bag.  N = 30 and 61 make
    the 16-point tiles straddle bags (Ho Wo % 16 != 0)."""
    from blindno import NIOFP2D_FNO, nio, ops
    torch.manual_seed(9)
    m = NIOFP2D_FNO(2, 3, 100, 25, 3, 6, 8, 2).cuda().train()
    x = torch.randn(B, 60, N, N, device="cuda")
    gx, gy = np.meshgrid(np.linspace(-1, 1, N, dtype=np.float32),
                         np.linspace(-1, 1, N, dtype=np.float32), indexing="ij")
    grid = torch.tensor(np.stack([gx, gy], 2)).cuda()
    idx = np.random.RandomState(3).choice(60, 57)
    res = []
    budget = ops.BAG_STATS_MAX_BYTES
    # third run: bag statistics on but over the byte budget -> the per-snapshot path, identically
    for bag_stats, max_bytes in ((True, budget), (False, budget), (True, 0)):
        ops.BAG_STATS = bag_stats
        ops.BAG_STATS_MAX_BYTES = max_bytes
        nio.DEDUP_BAGS = dedup
        try:
            m.zero_grad()
            out = m(x, grid, bag_idx=idx)
            (out * torch.linspace(-1, 1, out.numel(), device="cuda").view_as(out)).sum().backward()
            res.append((out.detach().cpu().numpy(), [p.grad.cpu().numpy() for p in m.FNO_input.parameters()]))
        finally:
            ops.BAG_STATS = True
            ops.BAG_STATS_MAX_BYTES = budget
            nio.DEDUP_BAGS = True
    assert np.array_equal(res[2][0], res[1][0])
    assert all(np.array_equal(a, b) for a, b in zip(res[2][1], res[1][1]))
    e_out = rel_l2(res[0][0], res[1][0])
    e_g = [rel_l2(a, b) for a, b in zip(res[0][1], res[1][1])]
    print(f"bag-level vs per-snapshot projection: out {e_out:.2e}, FNO_input grads max {max(e_g):.2e}")
    assert e_out <= 1e-6
    assert max(e_g) <= 1e-5


@pytest.mark.parametrize("C,m,N,Bn", [(4, 12, 128, 12), (4, 12, 61, 3), (3, 5, 30, 5)])
def test_crop_valid_region_kernels(C, m, N, Bn):
    """blindno_rowdft_crop / blindno_rowidft_bwd_crop (the encoder adjoint's dz read only on the
    N x N crop of the P x P field): garbage on the padding is never read, and the results are
    BIT-identical to the full-field kernels on the same field with a zeroed padding (the skipped
    K blocks contribute exact zeros)."""
    from blindno import ops
    P = N + ops.pad_amount(N)
    g = torch.Generator(device="cuda").manual_seed(11)
    dz = torch.randn(Bn, C, P, P, device="cuda", generator=g)
    dz_zero = dz.clone()
    dz_zero[:, :, N:, :] = 0
    dz_zero[:, :, :, N:] = 0
    dz[:, :, N:, :] = float("nan")                   # never read by the crop kernels
    dz[:, :, :, N:] = float("nan")
    a_crop = ops.k_rowdft(dz, Bn, C, P, P, m, 0, valid=(N, N))
    a_full = ops.k_rowdft(dz_zero, Bn, C, P, P, m, 0)
    assert torch.equal(a_crop, a_full)
    K1 = ops.kept_rows_count(m, P)
    G = torch.randn(Bn, P, m, C, 2, device="cuda", generator=g)
    cw = torch.randn(C, C, 1, 1, device="cuda", generator=g) * 0.3
    xs = torch.randn(Bn, C, P, P, device="cuda", generator=g)
    wg = C <= 4
    r_crop = ops.k_rowidft_bwd(G, dz, cw, xs, Bn, C, P, P, m, 1, wg, valid=(N, N))
    r_full = ops.k_rowidft_bwd(G, dz_zero, cw, xs, Bn, C, P, P, m, 1, wg)
    torch.cuda.synchronize()
    for a, b in zip(r_crop, r_full):
        if a is not None:
            assert torch.equal(a, b)
    assert K1 > 0


@pytest.mark.parametrize("C,m,P,Bn", [(4, 12, 160, 104), (3, 16, 150, 112), (4, 12, 160, 8),
                                      (4, 20, 96, 180)])
def test_rowinv_fused_next_rowdft(C, m, P, Bn):
    """blindno_rowidft_epi_rd / blindno_rowidft_bwd_rd (the next layer's row DFT taken in the row
    inverse's pass) vs the same row inverse followed by blindno_rowdft on its output: the field
    agrees to the last bit or two (the fused and unfused template instances of the transposed
    C = 4 kernel are compiled separately; 1e-7 relative) and the spectra to fp32 rounding (2e-6
    relative).  Cases: the transposed whole-row kernel (C = 4, m = 12, P = 160), a ragged last
    column tile (P = 150), the small-bag case and the m2 > 16 fallback (general kernel plus a
    separate row DFT launch)."""
    from blindno import ops
    g = torch.Generator(device="cuda").manual_seed(C * 100 + m)
    Z = torch.randn(Bn, P, m, C, 2, device="cuda", generator=g) * 0.1
    x = torch.randn(Bn, C, P, P, device="cuda", generator=g)
    cw = torch.randn(C, C, 1, 1, device="cuda", generator=g) * 0.3
    cb = torch.randn(C, device="cuda", generator=g) * 0.1
    for act in (0, 1):
        for act_next in (0, 1):
            z_ref = ops.k_rowidft_epi(Z, x, cw, cb, Bn, C, P, P, m, act)
            a_ref = ops.k_rowdft(z_ref, Bn, C, P, P, m, act_next)
            z, a = ops.k_rowidft_epi_rd(Z, x, cw, cb, Bn, C, P, P, m, act, act_next)
            torch.cuda.synchronize()
            assert rel_l2(z.cpu().numpy(), z_ref.cpu().numpy()) <= 1e-7
            assert rel_l2(a.cpu().numpy(), a_ref.cpu().numpy()) <= 2e-6
    dz = torch.randn(Bn, C, P, P, device="cuda", generator=g)
    N = P - 20
    for wg in (False, True):
        r_ref = ops.k_rowidft_bwd(Z, dz, cw, x, Bn, C, P, P, m, 1, wg, valid=(N, N))
        a_ref = ops.k_rowdft(r_ref[0], Bn, C, P, P, m, 0)
        r = ops.k_rowidft_bwd(Z, dz, cw, x, Bn, C, P, P, m, 1, wg, valid=(N, N), rd=True)
        torch.cuda.synchronize()
        assert rel_l2(r[0].cpu().numpy(), r_ref[0].cpu().numpy()) <= 1e-7
        if wg:
            assert rel_l2(r[1].cpu().numpy(), r_ref[1].cpu().numpy()) <= 1e-7
            assert rel_l2(r[2].cpu().numpy(), r_ref[2].cpu().numpy()) <= 1e-7
        assert rel_l2(r[3].cpu().numpy(), a_ref.cpu().numpy()) <= 2e-6


@pytest.mark.parametrize("C,act,G", [(12, 1, 2), (12, 0, 1), (8, 1, 1), (3, 1, 1)])
def test_conv_wgrad_vs_fp64(C, act, G):
    """1x1-conv weight / bias gradient of an FNO layer (blindno_conv_wgrad_g: the heads' C = 12
    layers, grouped over two weight groups) vs the float64 sums:
    dW[o][i] = sum_p dz[o][p] f(x)[i][p], db[o] = sum_p dz[o][p], f = GELU if act."""
    import oracle
    from blindno import ops
    from blindno._lib import call, ptr, query, stream_ptr
    Bn, P = 4 * G, 160
    g = torch.Generator(device="cuda").manual_seed(C + 10 * act)
    dz = torch.randn(Bn, C, P, P, device="cuda", generator=g)
    x = torch.randn(Bn, C, P, P, device="cuda", generator=g)
    nch = query("blindno_conv_wgrad_nchunk", Bn // G, P, P)
    part = torch.empty(nch, G, C * C + C, device="cuda")
    call("blindno_conv_wgrad_g", ptr(dz), ptr(x), ptr(part), nch, G, Bn, C, P, P, act, stream_ptr())
    got = ops.reduce_partials(part, nch, G * (C * C + C)).view(G, C * C + C).double().cpu()
    d64, x64 = dz.double().cpu(), x.double().cpu()
    f = oracle.gelu(x64) if act else x64
    for gi in range(G):
        sl = slice(gi * Bn // G, (gi + 1) * Bn // G)
        w = torch.einsum("nohw,nihw->oi", d64[sl], f[sl])
        b = d64[sl].sum(dim=(0, 2, 3))
        # fp32 sums over 1e5 points of O(1) terms with O(sqrt n) results: a few 1e-6 (the
        # 8c gradient bar is 1e-4)
        assert rel_l2(got[gi, :C * C].numpy(), w.reshape(-1).numpy()) <= 5e-5
        assert rel_l2(got[gi, C * C:].numpy(), b.numpy()) <= 5e-5


@pytest.mark.parametrize("C,Cin,N,G", [(12, 25, 128, 2), (12, 12, 64, 1), (8, 30, 48, 1), (12, 25, 61, 1)])
def test_lift_wgrad_vs_fp64(C, Cin, N, G):
    """fc0 (lift) weight / bias gradient of an FNO head (blindno_lift_bwd_g: the matrix-core
    kernel when N % 16 == 0, the LDS-staged one otherwise) vs the float64 sums over the crop:
    dW0[c][j] = sum_p dx0[c][p] in[p][j], db0[c] = sum_p dx0[c][p]."""
    from blindno import ops
    from blindno._lib import call, ptr, query, stream_ptr
    Bg, P = 4, N + ops.pad_amount(N)
    g = torch.Generator(device="cuda").manual_seed(C + Cin + N)
    dx0 = torch.randn(G * Bg, C, P, P, device="cuda", generator=g)
    inp = torch.randn(Bg, N, N, Cin, device="cuda", generator=g)
    w0 = torch.randn(G, C, Cin, device="cuda", generator=g)
    nch = query("blindno_lift_bwd_nchunk", Bg, N, N)
    part = torch.empty(nch, G, C * Cin + C, device="cuda")
    call("blindno_lift_bwd_g", ptr(dx0), ptr(inp), ptr(w0), None, ptr(part), nch, G, C * Cin, G * Bg,
         N, N, Cin, C, P, P, stream_ptr())
    got = ops.reduce_partials(part, nch, G * (C * Cin + C)).view(G, C * Cin + C).double().cpu()
    d64 = dx0.double().cpu()[:, :, :N, :N]
    i64 = inp.double().cpu()
    for gi in range(G):
        d = d64[gi * Bg:(gi + 1) * Bg]
        w = torch.einsum("nchw,nhwj->cj", d, i64)
        b = d.sum(dim=(0, 2, 3))
        assert rel_l2(got[gi, :C * Cin].numpy(), w.reshape(-1).numpy()) <= 5e-5
        assert rel_l2(got[gi, C * Cin:].numpy(), b.numpy()) <= 5e-5


@pytest.mark.parametrize("N,G", [(128, 2), (61, 1), (64, 2)])
def test_head_lift_fwd_and_input_grad_vs_fp64(N, G):
    """The heads' fc0 + pad (blindno_lift_fwd_g, width 12 -> 12: the thread-per-point kernel with
    the weights in LDS) and its input gradient (blindno_lift_bwd_g, d_in summed over the grouped
    heads) vs float64 (2d_FPE/FNOModules.py:219-224): x0 = pad(W0 in + b0), zero on the padding;
    d_in[n][h][w][j] = sum_g sum_c W_g[c][j] dx0[g Bg + n][c][h][w] on the crop."""
    from blindno import ops
    from blindno._lib import call, ptr, stream_ptr
    C = Cin = 12
    Bg, P = 4, N + ops.pad_amount(N)
    g = torch.Generator(device="cuda").manual_seed(N + G)
    inp = torch.randn(Bg, N, N, Cin, device="cuda", generator=g)
    w0 = torch.randn(G, C, Cin, device="cuda", generator=g)
    b0 = torch.randn(G, C, device="cuda", generator=g)
    # grouped weights share one group stride wgs for the weights and the biases (ops packs both
    # into per-head blocks of that stride)
    bpk = torch.zeros(G, C * Cin, device="cuda")
    bpk[:, :C] = b0
    x0 = torch.full((G * Bg, C, P, P), float("nan"), device="cuda")
    call("blindno_lift_fwd_g", ptr(inp), ptr(w0), ptr(bpk), ptr(x0), G, C * Cin, G * Bg, N, N, Cin, C, P, P,
         stream_ptr())
    dx0 = torch.randn(G * Bg, C, P, P, device="cuda", generator=g)
    d_in = torch.empty(Bg, N, N, Cin, device="cuda")
    call("blindno_lift_bwd_g", ptr(dx0), ptr(inp), ptr(w0), ptr(d_in), None, 0, G, C * Cin, G * Bg, N, N, Cin,
         C, P, P, stream_ptr())
    torch.cuda.synchronize()
    i64, w64, b64 = inp.double().cpu(), w0.double().cpu(), b0.double().cpu()
    ref = torch.zeros(G * Bg, C, P, P, dtype=torch.float64)
    for gi in range(G):
        ref[gi * Bg:(gi + 1) * Bg, :, :N, :N] = (torch.einsum("nhwj,cj->nchw", i64, w64[gi])
                                                 + b64[gi][None, :, None, None])
    got = x0.double().cpu()
    assert torch.isfinite(got).all()                     # the padding is written (zeros)
    assert float(got[:, :, N:, :].abs().max()) == 0.0 and float(got[:, :, :, N:].abs().max()) == 0.0
    assert rel_l2(got.numpy(), ref.numpy()) <= 1e-6
    d64 = dx0.double().cpu()[:, :, :N, :N]
    dref = sum(torch.einsum("nchw,cj->nhwj", d64[gi * Bg:(gi + 1) * Bg], w64[gi]) for gi in range(G))
    assert rel_l2(d_in.double().cpu().numpy(), dref.numpy()) <= 1e-6


@pytest.mark.parametrize("Bn,C,m,P,Gw", [(208, 4, 12, 160, 1), (8, 12, 32, 160, 2), (4, 12, 32, 160, 1),
                                         (8, 4, 12, 320, 1), (37, 3, 16, 150, 1), (6, 8, 20, 96, 1),
                                         (5, 16, 8, 40, 1)])
def test_fused_column_pass_matches_split(Bn, C, m, P, Gw):
    """The fused column pass (blindno_set_colfuse(1): column DFT, mix and column inverse in one
    workgroup, the spectrum in LDS) vs the split coldft_mix + colidft kernels on the same inputs,
    both directions: the saved spectrum Xs and the row coefficients Z (plain or the wide row
    inverse's tiled layout) agree to fp32 rounding (the fused kernel sums the column DFT in up to
    4 row chunks).  Cases: FNO_input at config C, the grouped heads, one head, FNO_input at 320
    rows (config E), odd widths / ragged row blocks, 16 channels."""
    import ctypes
    from blindno import ops
    from blindno._lib import call, ptr, query, stream_ptr
    g = torch.Generator(device="cuda").manual_seed(Bn + C + m)
    K1 = ops.kept_rows_count(m, P)
    K1p = 16 * ((K1 + 15) // 16)
    At = torch.randn(Bn, m, C, P, 2, device="cuda", generator=g)
    Wt = torch.randn(Gw, m, K1, C, C, 2, device="cuda", generator=g) * 0.2
    FB, GB = ops.twiddle_cols(P, m, At.device)
    wtgs = m * K1 * C * C * 2 if Gw > 1 else 0
    res = {}
    for fused in (0, 1):
        prev = query("blindno_set_colfuse", fused)
        for d in (0, 1):
            Xs = torch.full((Bn, m, C, K1, 2), float("nan"), device="cuda")
            Y = torch.empty(Bn, m, C, K1p, 2, device="cuda")
            Z = torch.full((Bn, P, m, C, 2), float("nan"), device="cuda")
            call("blindno_colpass_g", ptr(At), ptr(Wt), ptr(Xs), ptr(Y), ptr(Z), ptr(FB), ptr(GB), Gw,
                 ctypes.c_int64(wtgs), Bn, C, C, P, m, m, P, d, stream_ptr())
            res[(fused, d)] = (Xs, Z)
        query("blindno_set_colfuse", prev)
    torch.cuda.synchronize()
    for d in (0, 1):
        for a, b in zip(res[(1, d)], res[(0, d)]):
            assert torch.isfinite(a).all()
            assert rel_l2(a.cpu().numpy(), b.cpu().numpy()) <= 1e-6, d


@pytest.mark.parametrize("Bn,C,m,P,Gw", [(300, 4, 12, 320, 1), (8, 12, 32, 320, 2), (40, 4, 12, 160, 1)])
def test_fused_column_pass_fp16_mix(Bn, C, m, P, Gw):
    """The fused column pass with the fp16-operand mix (config E: dir bit 1; the spectra block-
    scaled per workgroup) vs the fp32 mix on the same inputs, both directions, next to the split
    kernels' fp16 mix: the fused kernel scales over its own 16 rows (the split one over its G
    pairs), so the two fp16 results differ at fp16 rounding; each stays within 2e-3 of the fp32
    mix and the fused one no worse than 1.5x the split one (+1e-4)."""
    import ctypes
    from blindno import ops
    from blindno._lib import call, ptr, query, stream_ptr
    g = torch.Generator(device="cuda").manual_seed(Bn + C + m + 7)
    K1 = ops.kept_rows_count(m, P)
    K1p = 16 * ((K1 + 15) // 16)
    At = torch.randn(Bn, m, C, P, 2, device="cuda", generator=g)
    Wt = torch.randn(Gw, m, K1, C, C, 2, device="cuda", generator=g) * 0.2
    FB, GB = ops.twiddle_cols(P, m, At.device)
    wtgs = m * K1 * C * C * 2 if Gw > 1 else 0
    res = {}
    for fused in (0, 1):
        prev = query("blindno_set_colfuse", fused)
        for d in (0, 1):
            for h in (0, 2):
                Xs = torch.full((Bn, m, C, K1, 2), float("nan"), device="cuda")
                Y = torch.empty(Bn, m, C, K1p, 2, device="cuda")
                Z = torch.full((Bn, P, m, C, 2), float("nan"), device="cuda")
                call("blindno_colpass_g", ptr(At), ptr(Wt), ptr(Xs), ptr(Y), ptr(Z), ptr(FB), ptr(GB), Gw,
                     ctypes.c_int64(wtgs), Bn, C, C, P, m, m, P, d | h, stream_ptr())
                res[(fused, d, h)] = Z
        query("blindno_set_colfuse", prev)
    torch.cuda.synchronize()
    for d in (0, 1):
        ref = res[(1, d, 0)].cpu().numpy()
        e_f = rel_l2(res[(1, d, 2)].cpu().numpy(), ref)
        e_s = rel_l2(res[(0, d, 2)].cpu().numpy(), ref)
        print(f"  dir {d}: fp16 mix vs fp32, fused {e_f:.2e}, split {e_s:.2e}")
        assert torch.isfinite(res[(1, d, 2)]).all()
        assert e_f <= 2e-3 and e_s <= 2e-3, (d, e_f, e_s)
        assert e_f <= 1.5 * e_s + 1e-4, (d, e_f, e_s)


def test_bag_mean_handed_to_heads_bit_identical():
    """NIOFP2D_FNO with the bag mean handed to the grouped heads as ubar (the heads' lift forms
    fc0([grid, ubar]) and returns d ubar: ops.BagHeadsIn) against the materialised
    (B, N, N, width) field with the two bag-mean launches: output and every gradient
    bit-identical (the same fma order in both forms)."""
    from blindno import NIOFP2D_FNO, nio
    torch.manual_seed(31)
    m = NIOFP2D_FNO(2, 3, 100, 25, 3, 12, 16, 2).cuda().train()
    B, T, N = 2, 40, 64
    x = torch.randn(B, T, N, N, device="cuda")
    gx, gy = np.meshgrid(np.linspace(-1, 1, N, dtype=np.float32), np.linspace(-1, 1, N, dtype=np.float32),
                         indexing="ij")
    grid = torch.tensor(np.stack([gx, gy], 2)).cuda()
    idx = np.random.RandomState(6).choice(T, 33)
    cot = torch.randn(B, N, N, 2, generator=torch.Generator().manual_seed(2)).cuda()
    res = {}
    prev = nio.BAG_INPUT_HEADS
    try:
        for on in (False, True):
            nio.BAG_INPUT_HEADS = on
            m.zero_grad(set_to_none=True)
            out = m(x, grid, bag_idx=idx)
            (out * cot).sum().backward()
            torch.cuda.synchronize()
            res[on] = [out.detach().clone()] + [p.grad.clone() for _, p in m.named_parameters()
                                                if p.grad is not None]
    finally:
        nio.BAG_INPUT_HEADS = prev
    assert len(res[True]) == len(res[False]) > 20
    for a, b in zip(res[False], res[True]):
        assert torch.equal(a, b)


def test_pack_hosted_by_bag_rowdft_bit_identical():
    """The encoder's (and the heads' pack_ahead) spectral-weight pack hosted by the bag's first
    row-DFT launch (blindno_rowdft_bag_lift_cd_pack) against its own pack launch: output and
    every gradient bit-identical, and nothing left held back."""
    from blindno import NIOFP2D_FNO, ops
    torch.manual_seed(33)
    m = NIOFP2D_FNO(2, 3, 100, 25, 3, 12, 16, 2).cuda().train()
    B, T, N = 2, 40, 64
    x = torch.randn(B, T, N, N, device="cuda")
    gx, gy = np.meshgrid(np.linspace(-1, 1, N, dtype=np.float32), np.linspace(-1, 1, N, dtype=np.float32),
                         indexing="ij")
    grid = torch.tensor(np.stack([gx, gy], 2)).cuda()
    idx = np.random.RandomState(7).choice(T, 33)
    cot = torch.randn(B, N, N, 2, generator=torch.Generator().manual_seed(3)).cuda()
    res = {}
    prev = ops.HOST_PACK
    try:
        for on in (False, True):
            ops.HOST_PACK = on
            m.zero_grad(set_to_none=True)
            out = m(x, grid, bag_idx=idx)
            (out * cot).sum().backward()
            torch.cuda.synchronize()
            assert ops.take_deferred_pack() is None
            res[on] = [out.detach().clone()] + [p.grad.clone() for _, p in m.named_parameters()
                                                if p.grad is not None]
    finally:
        ops.HOST_PACK = prev
    assert len(res[True]) == len(res[False]) > 20
    for a, b in zip(res[False], res[True]):
        assert torch.equal(a, b)
