"""HIP-graph training steps (train.GraphedBagStep: one graph per bag size L, device-resident
bag indices) against the same steps run eagerly (needs a GPU).

Same initial parameters, same bags, same index draws: after three Adam steps the parameters
must agree to rel-L2 1e-6 (identical kernels; only the launch mechanism differs).
"""
import copy

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


def _models():
    import blindno
    torch.manual_seed(3)
    yield "2d", blindno.NIOFP2D_FNO(2, 3, 100, 25, 3, 6, 6, 2), (2, 60, 32, 32), 2
    torch.manual_seed(4)
    yield "1d", blindno.NIOFP_FNO(3, 30, 15, 2, "cuda"), (4, 80, 64), 2
    torch.manual_seed(5)
    yield "1d_gpe", blindno.NIOFP_FNO(3, 20, 40, 1, "cuda", heads=("fno_V",)), (4, 70, 64), 1


@pytest.mark.parametrize("case,overlap", [("2d", False), ("2d", True), ("1d", False), ("1d_gpe", False)])
def test_graphed_steps_match_eager(case, overlap):
    """overlap=True forces the two-graph step (encoder / heads split, the heads' gradient
    reduced on a side stream) at world size 1."""
    import blindno
    from blindno.train import DataParallel, FlatAdam, GraphedBagStep, grid1d, grid2d, trained_parameters
    name, model, xshape, cout = next((m for m in _models() if m[0] == case))
    model = model.cuda().train()
    ref = copy.deepcopy(model)
    B, T = xshape[0], xshape[1]
    g = torch.Generator(device="cuda").manual_seed(9)
    x = torch.randn(*xshape, device="cuda", generator=g)
    y = torch.randn(*((B,) + xshape[2:] + (cout,)), device="cuda", generator=g)
    grid = grid2d(xshape[2], xshape[3], "cuda") if len(xshape) == 4 else grid1d(xshape[2], "cuda")
    rs = np.random.RandomState(0)
    draws = [rs.choice(T, rs.randint(50, T)) for _ in range(3)]

    opt = FlatAdam(trained_parameters(model), lr=1e-3)
    gstep = GraphedBagStep(model, blindno.mse_loss, opt, DataParallel(opt), x, y, grid, overlap=overlap)
    assert gstep.overlap == overlap
    for idx in draws:
        gstep.step(idx)
    torch.cuda.synchronize()

    ropt = FlatAdam(trained_parameters(ref), lr=1e-3)
    for idx in draws:
        out = ref(x, grid, bag_idx=idx)
        blindno.mse_loss(out, y).backward()
        ropt.step()
        ropt.zero_grad()
    torch.cuda.synchronize()
    assert rel_l2(opt.flat.cpu().numpy(), ropt.flat.cpu().numpy()) <= 1e-6


def test_gather_flat_segments():
    """blindno_gather_flat (FlatAdam's gradient gather): odd offsets, empty and multi-launch
    (> 64 segments) lists, sizes straddling the 2048-element block chunk."""
    import ctypes
    from blindno._lib import call, ptr, stream_ptr
    rs = np.random.RandomState(0)
    sizes = [0, 1, 2047, 2048, 2049, 5000] + list(rs.randint(1, 3000, 70))
    srcs = [torch.randn(n, device="cuda") for n in sizes]
    offs, o = [], 3
    for n in sizes:
        offs.append(o)
        o += n + 1
    dst = torch.full((o,), -7.0, device="cuda")
    k = len(sizes)
    call("blindno_gather_flat", (ctypes.c_void_p * k)(*[t.data_ptr() for t in srcs]),
         (ctypes.c_int64 * k)(*offs), (ctypes.c_int64 * k)(*sizes), k, ptr(dst), stream_ptr())
    ref = torch.full((o,), -7.0, device="cuda")
    for t, off in zip(srcs, offs):
        ref[off:off + t.numel()] = t
    torch.cuda.synchronize()
    assert torch.equal(dst, ref)


def test_grid_spectrum_cache_follows_fc0_and_grid():
    """The encoder's grid-plane spectra are cached across steps (ops._grid_planes) and its
    grid/bias part is formed from them with the current FNO_input.fc0 in the kernel: an in-place
    change of fc0 must show at once, one of the grid must invalidate the cache."""
    import blindno
    torch.manual_seed(3)
    m = blindno.NIOFP2D_FNO(2, 3, 100, 25, 2, 6, 5, 2).cuda().eval()
    x = torch.randn(1, 60, 20, 20, device="cuda")
    gx, gy = np.meshgrid(np.linspace(-1, 1, 20, dtype=np.float32), np.linspace(-1, 1, 20, dtype=np.float32),
                         indexing="ij")
    grid = torch.tensor(np.stack([gx, gy], 2), device="cuda")
    with torch.no_grad():
        a = m(x, grid)
        m.FNO_input.fc0.weight.mul_(1.5)
        b = m(x, grid)
        grid.mul_(0.5)
        c = m(x, grid)
    m2 = blindno.NIOFP2D_FNO(2, 3, 100, 25, 2, 6, 5, 2).cuda().eval()
    m2.load_state_dict(m.state_dict())
    with torch.no_grad():
        c2 = m2(x, grid.clone())          # fresh grid storage: computed from scratch
    assert not torch.equal(a, b) and not torch.equal(b, c)
    assert rel_l2(c.cpu().numpy(), c2.cpu().numpy()) <= 1e-6
