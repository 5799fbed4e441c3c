"""The transposed whole-row C = 4 row inverse (csrc/rowinv.hip rowfuse_kernel) behind the
blindno_rowidft_* entries, at the snapshot encoder's shape (width 4, m = 12, P = 160):

* against a float64 numpy restatement of the entry's definition (include/blindno.h:
  irfft row stage + 1x1 conv + bias + GELU, its adjoint, and the next layer's row DFT), and
* against the general kernel (blindno_set_rowfuse(0)) on the same inputs, for the lift
  variants of the bag encoder's first layer.

Tolerances: fp32 kernels vs float64, rel-L2 <= 1e-5 (fields, spectra) and <= 1e-4 (reduced
weight gradients) -- SURVEY.md 8c; kernel vs kernel (both fp32, different summation order)
<= 2e-6.
"""
import math

import numpy as np
import pytest
import torch

from conftest import rel_l2

pytestmark = pytest.mark.gpu

Bn, C, P, m = 6, 4, 160, 12


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import blindno
    blindno.load_library()


@pytest.fixture()
def fuse():
    from blindno._lib import query         # returns the previous setting (not an error code)
    prev = query("blindno_set_rowfuse", 1)
    yield query
    query("blindno_set_rowfuse", prev)


def _gelu(x):
    from scipy.special import erf
    return 0.5 * x * (1.0 + erf(x / math.sqrt(2.0)))


def _gelu_grad(x):
    from scipy.special import erf
    return 0.5 * (1.0 + erf(x / math.sqrt(2.0))) + x * np.exp(-0.5 * x * x) / math.sqrt(2.0 * math.pi)


def _irow(Z):
    """Z (Bn, P, m, C, 2) -> sum_k Re(Z_k e^{+2 pi i k w / P}) as (Bn, C, P, P)."""
    Zc = Z[..., 0].astype(np.float64) + 1j * Z[..., 1].astype(np.float64)
    E = np.exp(2j * np.pi * np.outer(np.arange(m), np.arange(P)) / P)
    return np.real(np.einsum("nhkc,kw->nchw", Zc, E))


def _row_dft(f):
    """f (Bn, C, P, P) -> At (Bn, m, C, P, 2) = sum_w f e^{-2 pi i k w / P}."""
    E = np.exp(-2j * np.pi * np.outer(np.arange(P), np.arange(m)) / P)
    A = np.einsum("nchw,wk->nkch", f, E)
    return np.stack([A.real, A.imag], -1)


def _inputs(seed=0):
    g = torch.Generator().manual_seed(seed)
    Z = torch.randn(Bn, P, m, C, 2, generator=g) * 0.05
    x = torch.randn(Bn, C, P, P, generator=g)
    cw = torch.randn(C, C, 1, 1, generator=g) * 0.4
    cb = torch.randn(C, generator=g) * 0.1
    return Z, x, cw, cb


@pytest.mark.parametrize("act", [0, 1])
def test_rowfuse_forward_rd_vs_fp64(fuse, act):
    from blindno import ops
    Z, x, cw, cb = _inputs(1)
    z, At = ops.k_rowidft_epi_rd(Z.cuda(), x.cuda(), cw.cuda(), cb.cuda(), Bn, C, P, P, m, act, 1)
    z1 = ops.k_rowidft_epi(Z.cuda(), x.cuda(), cw.cuda(), cb.cuda(), Bn, C, P, P, m, act)
    torch.cuda.synchronize()
    xin = x.double().numpy()
    if act:
        xin = _gelu(xin)
    ref = _irow(Z.numpy()) + np.einsum("oi,nihw->nohw", cw.double().numpy()[:, :, 0, 0], xin) \
        + cb.double().numpy()[None, :, None, None]
    e = rel_l2(z.cpu().numpy(), ref)
    print(f"rowfuse fwd act={act}: z {e:.2e}")
    assert e <= 1e-5
    assert torch.equal(z, z1)            # the RD pass does not change the field
    ea = rel_l2(At.cpu().numpy(), _row_dft(_gelu(ref)))
    print(f"rowfuse fwd act={act}: At(GELU z) {ea:.2e}")
    assert ea <= 1e-5


@pytest.mark.parametrize("act", [0, 1])
@pytest.mark.parametrize("crop", [None, (128, 128)])
def test_rowfuse_adjoint_rd_vs_fp64(fuse, act, crop):
    from blindno import ops
    G, xs, cw, _ = _inputs(2)
    dz = torch.randn(Bn, C, P, P, generator=torch.Generator().manual_seed(3))
    dx, gw, gb, At = ops.k_rowidft_bwd(G.cuda(), dz.cuda(), cw.cuda(), xs.cuda(), Bn, C, P, P, m, act,
                                       True, crop, rd=True)
    torch.cuda.synchronize()
    dzv = dz.double().numpy().copy()
    if crop is not None:
        dzv[:, :, crop[0]:, :] = 0.0
        dzv[:, :, :, crop[1]:] = 0.0
    W = cw.double().numpy()[:, :, 0, 0]
    xsv = xs.double().numpy()
    dg = _irow(G.numpy()) + np.einsum("oi,nohw->nihw", W, dzv)
    a = xsv
    if act:
        dg = dg * _gelu_grad(xsv)
        a = _gelu(xsv)
    e = rel_l2(dx.cpu().numpy(), dg)
    ew = rel_l2(gw.cpu().numpy().reshape(C, C), np.einsum("nohw,nihw->oi", dzv, a))
    eb = rel_l2(gb.cpu().numpy(), dzv.sum(axis=(0, 2, 3)))
    ea = rel_l2(At.cpu().numpy(), _row_dft(dg))
    print(f"rowfuse adjoint act={act} crop={crop}: dx {e:.2e} dWc {ew:.2e} dbc {eb:.2e} At {ea:.2e}")
    assert e <= 1e-5 and ea <= 1e-5
    assert ew <= 1e-4 and eb <= 1e-4


def _lift_inputs():
    B, T, L, N = 2, 5, 3, 128
    g = torch.Generator().manual_seed(4)
    X = torch.randn(B, T, N, N, generator=g).cuda()
    idx = torch.tensor([3, 0, 3], dtype=torch.int32).cuda()
    xs = torch.linspace(0, 1, N)
    gx, gy = torch.meshgrid(xs, xs, indexing="ij")
    grid = torch.stack([gx, gy], -1).contiguous().cuda()
    w0 = (torch.randn(C, 3, generator=g) * 0.5).cuda()
    b0 = (torch.randn(C, generator=g) * 0.1).cuda()
    return B, T, L, N, X, idx, grid, w0, b0


def test_rowfuse_lift_variants_match_general_kernel(fuse):
    """The bag encoder's first layer (lift recomputed in the epilogue / adjoint, fc0's gradient
    reduced in the pass): transposed kernel vs the general kernel, forward + RD and adjoint."""
    from blindno import ops
    from blindno._lib import call, ptr, query, stream_ptr
    B, T, L, N, X, idx, grid, w0, b0 = _lift_inputs()
    Bl = B * L
    g = torch.Generator().manual_seed(5)
    Z = (torch.randn(Bl, P, m, C, 2, generator=g) * 0.05).cuda()
    dz = torch.randn(Bl, C, P, P, generator=g).cuda()
    cw = (torch.randn(C, C, 1, 1, generator=g) * 0.4).cuda()
    cb = (torch.randn(C, generator=g) * 0.1).cuda()
    tb = ops.twiddle_rowinv(P, m, X.device)
    Tp = ops.twiddle_mfma(P, m, X.device)

    def run():
        z = torch.empty(Bl, C, P, P, device=X.device)
        At = torch.empty(Bl, m, C, P, 2, device=X.device)
        call("blindno_rowidft_epi_lift_rd", ptr(Z), ptr(X), ptr(idx), ptr(grid), ptr(w0), ptr(b0), ptr(cw),
             ptr(cb), ptr(z), ptr(tb), B, T, L, N, N, C, P, P, m, ptr(At), ptr(Tp), 1, stream_ptr())
        nch = query("blindno_rowidft_bwd_nchunk", Bl, C, P, P, m)
        part = torch.empty(nch, C * C + C + 4 * C, device=X.device)
        call("blindno_rowidft_bwd_lift", ptr(Z), ptr(dz), ptr(X), ptr(idx), ptr(grid), ptr(w0), ptr(b0),
             ptr(cw), ptr(tb), ptr(part), B, T, L, N, N, C, P, P, m, stream_ptr())
        torch.cuda.synchronize()
        return z, At, part.double().sum(0)

    z1, A1, p1 = run()
    fuse("blindno_set_rowfuse", 0)
    z0, A0, p0 = run()
    e = (rel_l2(z1.cpu().numpy(), z0.cpu().numpy()), rel_l2(A1.cpu().numpy(), A0.cpu().numpy()),
         rel_l2(p1.cpu().numpy(), p0.cpu().numpy()))
    print(f"rowfuse lift vs general kernel: z {e[0]:.2e} At {e[1]:.2e} partial sums {e[2]:.2e}")
    assert e[0] <= 2e-6 and e[1] <= 2e-6 and e[2] <= 2e-6


@pytest.mark.parametrize("act,oN1,oN2,Bn_", [(1, 128, 128, 6), (0, 128, 128, 6), (1, 100, 96, 5), (1, 160, 160, 3)])
def test_output_crop_matches_full_field(fuse, act, oN1, oN2, Bn_):
    """blindno_rowidft_epi_crop (the encoder's last layer written on the projection's crop only)
    vs blindno_rowidft_epi: the crop h < oN1, w < oN2 is identical to the bit (same kernel code per
    element; only whole row blocks and column steps past the crop are skipped); 128 x 128 is the
    fully unrolled 4-step instance, 100 x 96 the runtime-step one, 160 x 160 no crop."""
    from blindno import ops
    from blindno._lib import call, ptr, stream_ptr
    g = torch.Generator(device="cuda").manual_seed(act + oN1 + oN2)
    Z = torch.randn(Bn_, P, m, C, 2, device="cuda", generator=g) * 0.1
    x = torch.randn(Bn_, C, P, P, device="cuda", generator=g)
    cw = torch.randn(C, C, 1, 1, device="cuda", generator=g) * 0.3
    cb = torch.randn(C, device="cuda", generator=g) * 0.1
    full = ops.k_rowidft_epi(Z, x, cw, cb, Bn_, C, P, P, m, act)
    crop = torch.full_like(full, float("nan"))
    call("blindno_rowidft_epi_crop", ptr(Z), ptr(x), ptr(cw), ptr(cb), ptr(crop),
         ptr(ops.twiddle_rowinv(P, m, Z.device)), Bn_, C, P, P, m, act, oN1, oN2, stream_ptr())
    torch.cuda.synchronize()
    assert torch.equal(crop[:, :, :oN1, :oN2], full[:, :, :oN1, :oN2])
