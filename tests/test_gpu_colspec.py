"""The column pass folded into the row kernels (csrc/colspec.h; ops.COLSPEC) against the fused
column pass it replaces (blindno_colpass between the row kernels) on the same inputs, and the
snapshot encoder through it against the one through the column pass.  The folded path forms the
same sums in a different order, so the bars are fp32-rounding ones: 1e-6 on spectra and fields,
1e-5 on parameter gradients (SURVEY 8c's 1e-5 / 1e-4 against fp64 are checked by the config
tests, which take this path by default)."""
import numpy as np
import pytest
import torch

from conftest import rel_l2

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import blindno
    blindno.load_library()


def _grid(N):
    gx, gy = np.meshgrid(np.linspace(-1, 1, N, dtype=np.float32), np.linspace(-1, 1, N, dtype=np.float32),
                         indexing="ij")
    return torch.tensor(np.stack([gx, gy], 2)).cuda()


def _layer(Bn, N, seed):
    from blindno import ops
    C, m = 4, 12
    P = N + ops.pad_amount(N)
    g = torch.Generator(device="cuda").manual_seed(seed)
    x = torch.randn(Bn, C, P, P, device="cuda", generator=g)
    w1 = torch.randn(C, C, m, m, 2, device="cuda", generator=g) / (C * C)
    w2 = torch.randn(C, C, m, m, 2, device="cuda", generator=g) / (C * C)
    cw = torch.randn(C, C, device="cuda", generator=g) / C
    cb = torch.randn(C, device="cuda", generator=g)
    Wt = ops.pack_weights((w1, w2), P, 2)
    return x, Wt, cw, cb, C, m, P


@pytest.mark.parametrize("Bn,N,act", [(6, 128, 1), (3, 128, 0), (2, 256, 1)])
def test_rowdft_cd_colmix_matches_colpass(Bn, N, act):
    """blindno_rowdft_cd (row DFT + per-block column-DFT partials) + blindno_colmix (block sum,
    Xs, mix) vs blindno_rowdft + blindno_colpass: the saved spectrum Xs in both directions, and
    the forward row inverse from the mixed spectrum (ZY) vs from the column pass's Z."""
    from blindno import ops
    from blindno._lib import call, ptr, stream_ptr
    x, Wt, cw, cb, C, m, P = _layer(Bn, N, 11 + N)
    assert ops.colspec_ok(Bn, C, P, P, m, m)
    cs = ops._ColSpec(Bn, C, P, P, m, m, x.device)
    part = cs.part(C, x)
    call("blindno_rowdft_cd", ptr(x), ptr(part), ptr(cs.Tp), ptr(cs.tab), Bn, C, P, P, m, act, P, P, stream_ptr())
    At = ops.k_rowdft(x, Bn, C, P, P, m, act)
    for direction in (0, 1):
        Xs_cs, Y = cs.mix(part, cs.nb, Wt, direction)
        Xs_ref, Z = ops.k_colpass(At, Wt, Bn, C, C, P, m, m, P, direction)
        torch.cuda.synchronize()
        e = rel_l2(Xs_cs.cpu().numpy(), Xs_ref.cpu().numpy())
        print(f"Bn={Bn} N={N} act={act} dir={direction}: Xs {e:.2e}")
        assert e <= 1e-6, e
        if direction == 0:
            z_cs = torch.empty_like(x)
            call("blindno_rowidft_epi_zc", ptr(Y), ptr(x), ptr(cw), ptr(cb), ptr(z_cs), ptr(cs.tb), ptr(cs.tab),
                 None, None, Bn, C, P, P, m, m, act, 0, P, P, stream_ptr())
            z_ref = ops.k_rowidft_epi(Z, x, cw, cb, Bn, C, P, P, m, act)
            torch.cuda.synchronize()
            ez = rel_l2(z_cs.cpu().numpy(), z_ref.cpu().numpy())
            print(f"   row inverse from Y vs from Z: {ez:.2e}")
            assert ez <= 1e-6, ez


@pytest.mark.parametrize("Bn,N", [(5, 128), (2, 256)])
def test_chained_layer_cd_matches_rowdft(Bn, N):
    """The chained layer as bench.py's roofline_spectral times it: row inverse from Y with the
    next row DFT's column-DFT partials in the same pass (blindno_rowidft_epi_zc with part) vs the
    separate row DFT of the field it wrote (blindno_rowdft_cd of GELU(z)); fields identical."""
    from blindno import ops
    from blindno._lib import call, ptr, stream_ptr
    x, Wt, cw, cb, C, m, P = _layer(Bn, N, 5 + N)
    cs = ops._ColSpec(Bn, C, P, P, m, m, x.device)
    p0 = cs.part(C, x)
    call("blindno_rowdft_cd", ptr(x), ptr(p0), ptr(cs.Tp), ptr(cs.tab), Bn, C, P, P, m, 1, P, P, stream_ptr())
    _, Y = cs.mix(p0, cs.nb, Wt, 0)
    z = torch.empty_like(x)
    p1 = cs.part(C, x)
    call("blindno_rowidft_epi_zc", ptr(Y), ptr(x), ptr(cw), ptr(cb), ptr(z), ptr(cs.tb), ptr(cs.tab), ptr(p1),
         ptr(cs.Tp), Bn, C, P, P, m, m, 1, 1, P, P, stream_ptr())
    z2 = torch.empty_like(x)
    call("blindno_rowidft_epi_zc", ptr(Y), ptr(x), ptr(cw), ptr(cb), ptr(z2), ptr(cs.tb), ptr(cs.tab), None,
         None, Bn, C, P, P, m, m, 1, 0, P, P, stream_ptr())
    p2 = cs.part(C, x)
    call("blindno_rowdft_cd", ptr(z), ptr(p2), ptr(cs.Tp), ptr(cs.tab), Bn, C, P, P, m, 1, P, P, stream_ptr())
    X1, _ = cs.mix(p1, cs.nb, Wt, 0)
    X2, _ = cs.mix(p2, cs.nb, Wt, 0)
    torch.cuda.synchronize()
    assert torch.equal(z, z2)
    e = rel_l2(X1.cpu().numpy(), X2.cpu().numpy())
    print(f"Bn={Bn} N={N}: next layer's spectrum in-pass vs separate {e:.2e}")
    assert e <= 1e-6, e


@pytest.mark.parametrize("N,B,dedup", [(128, 2, True), (128, 3, False), (256, 1, True)])
def test_encoder_colspec_matches_colpass(N, B, dedup):
    """NIOFP2D_FNO's snapshot encoder (ops.BagEncoderFn, 2 layers, modes 12, width 4) with the
    folded column pass vs with the column pass: output and every FNO_input gradient."""
    from blindno import NIOFP2D_FNO, nio, ops
    torch.manual_seed(21)
    m = NIOFP2D_FNO(2, 3, 100, 25, 2, 8, 6, 2).cuda().train()
    x = torch.randn(B, 80, N, N, device="cuda")
    grid = _grid(N)
    idx = np.random.RandomState(4).choice(80, 61)
    P = N + ops.pad_amount(N)
    assert ops.colspec_ok(B * 61, 4, P, P, 12, 12)
    res = []
    for on in (True, False):
        ops.COLSPEC = on
        nio.DEDUP_BAGS = dedup
        try:
            m.zero_grad()
            out = m(x, grid, bag_idx=idx)
            (out * torch.linspace(-1, 1, out.numel(), device="cuda").view_as(out)).sum().backward()
            torch.cuda.synchronize()
            res.append((out.detach().cpu().numpy(),
                        {k: p.grad.cpu().numpy() for k, p in m.FNO_input.named_parameters()}))
        finally:
            ops.COLSPEC = True
            nio.DEDUP_BAGS = True
    e_out = rel_l2(res[0][0], res[1][0])
    e_g = {k: rel_l2(res[0][1][k], res[1][1][k]) for k in res[1][1]}
    worst = max(e_g, key=e_g.get)
    print(f"N={N} B={B} dedup={dedup}: out {e_out:.2e}, worst grad {worst} {e_g[worst]:.2e}")
    assert e_out <= 1e-6, e_out
    assert e_g[worst] <= 1e-5, (worst, e_g[worst])
