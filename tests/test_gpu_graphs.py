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


def test_graphed_nio_step_matches_eager():
    """Config D's benched step (bench.py --config D): NIOFP2D (Encoder2D branch with train-mode
    BatchNorm and the grid-adaptive (4, 2) last kernel, FFN trunk, DeepONet combiner, heads
    fno_Fx / fno_Fy) at 128^2, B = 2, replayed from one HIP graph per drawn L (no deduplication:
    the BatchNorm statistics count the bag's repeats), three draws, against three eager steps.
    Parameters within 1e-6; BatchNorm running statistics within 1e-6 and num_batches_tracked
    exactly as the eager steps leave them -- the capture's eager warm-up must not count, and the
    graph must take each replay's batch statistics, not the captured L's."""
    import blindno
    from blindno import Encoder2D, NIOFP2D
    from blindno.train import DataParallel, FlatAdam, GraphedBagStep, grid2d, trained_parameters
    B, T, N = 2, 100, 128
    g = torch.Generator(device="cuda").manual_seed(11)
    x = torch.randn(B, T, N, N, device="cuda", generator=g)
    y = torch.randn(B, N, N, 2, device="cuda", generator=g)
    grid = grid2d(N, N, "cuda")
    rs = np.random.RandomState(5)
    draws = [rs.choice(T, rs.randint(50, T)) for _ in range(3)]
    assert len({len(d) for d in draws}) == 3          # three graph keys
    finals, bufs = [], []
    for graphed in (False, True):
        torch.manual_seed(6)
        m = NIOFP2D(2, 3, 100, 25, 3, 12, 32, 2, heads=("fno_Fx", "fno_Fy"),
                    branch_last_kernel=Encoder2D.kernel_for_grid(N)).cuda().train()
        # bench.py config D: everything but fc0 (read through .data) is trained, the branch too
        params = trained_parameters(m, exclude_prefixes=("fc0.",))
        assert any(k.startswith("branch.") for k, p in m.named_parameters() if any(p is q for q in params))
        opt = FlatAdam(params, lr=1e-3)
        if graphed:
            gs = GraphedBagStep(m, blindno.mse_loss, opt, DataParallel(opt), x, y, grid)
            assert not gs.dedup
            for idx in draws:
                gs.step(idx)
        else:
            for idx in draws:
                out = m(x, grid, bag_idx=idx)
                blindno.mse_loss(out, y).backward()
                opt.step()
                opt.zero_grad()
        torch.cuda.synchronize()
        finals.append(opt.flat.cpu().numpy().copy())
        bufs.append({k: b.detach().cpu().clone() for k, b in m.named_buffers()})
    assert rel_l2(finals[1], finals[0]) <= 1e-6
    assert bufs[0].keys() == bufs[1].keys() and len(bufs[0]) >= 36      # 10 + 2 BatchNorms x 3
    for k in bufs[0]:
        a, b = bufs[1][k], bufs[0][k]
        if a.is_floating_point():
            assert rel_l2(a.double().numpy(), b.double().numpy()) <= 1e-6, k
        else:
            assert torch.equal(a, b) and int(a) == len(draws), (k, a, b)


def _poison_default_pool():
    """Hand every free block of the caching allocator's default pool (of the sizes a step
    allocates) to tensors filled with NaN, then free them: a captured graph that still points at
    default-pool memory it does not own reads NaN afterwards."""
    torch.cuda.synchronize()
    blobs = []
    for mb in (1, 2, 4, 8, 16, 32, 64, 128, 256, 512, 1024):
        for _ in range(8):
            blobs.append(torch.full((mb << 18,), float("nan"), device="cuda"))
    for kb in (1, 4, 16, 64, 256):
        for _ in range(64):
            blobs.append(torch.full((kb << 8,), float("nan"), device="cuda"))
    torch.cuda.synchronize()
    del blobs
    torch.cuda.synchronize()


def _graph_models():
    import blindno
    from blindno import Encoder2D, unet
    torch.manual_seed(3)
    yield "fno2d", blindno.NIOFP2D_FNO(2, 3, 100, 25, 3, 6, 6, 2), (2, 60, 32, 32), 2
    torch.manual_seed(4)
    yield "fno1d", blindno.NIOFP_FNO(3, 30, 15, 2, "cuda"), (4, 80, 64), 2
    torch.manual_seed(5)
    yield "nio2d", blindno.NIOFP2D(2, 3, 100, 25, 3, 12, 8, 2, heads=("fno_Fx", "fno_Fy"),
                                   branch_last_kernel=Encoder2D.kernel_for_grid(64)), (2, 60, 64, 64), 2
    torch.manual_seed(6)
    yield "nio1d", blindno.NIOFP(1, 3, 100, 25, 3, 30, 15, 2, "cuda"), (4, 60, 80), 2
    torch.manual_seed(7)
    yield "fno2d_attn", blindno.NIOFP2D_FNO_attn(2, 3, 100, 25, 3, 6, 6, 2, 32, 32), (2, 60, 32, 32), 2
    torch.manual_seed(8)
    yield "unet2d", unet.PermInvUNet_attn(1, 2, 1, 4, (52, 52)), (2, 60, 52, 52), 2


@pytest.mark.parametrize("case", ["fno2d", "fno1d", "nio2d", "nio1d", "fno2d_attn", "unet2d"])
def test_graph_replays_survive_default_pool_reuse(case):
    """Every graphed model: two graph keys captured, then the default pool's free blocks are
    overwritten (NaN) and each key replayed again -- its output and flat gradient must equal an
    eager step at the same parameters and bag.  A captured graph that reads memory it does not own
    (a torch op whose capture referenced a default-pool block later freed) fails here; the NIO
    step did with torch's Linear / matmul reductions in it, before they moved to libblindno."""
    import blindno
    from blindno.train import DataParallel, FlatAdam, GraphedBagStep, grid1d, grid2d, trained_parameters
    name, m, xshape, cout = next(c for c in _graph_models() if c[0] == case)
    m = m.cuda().train()
    B, T = xshape[0], xshape[1]
    g = torch.Generator(device="cuda").manual_seed(9)
    x = torch.randn(*xshape, device="cuda", generator=g)
    y = torch.randn(*((B,) + xshape[2:] + (cout,)), device="cuda", generator=g)
    grid = grid2d(xshape[2], xshape[3], "cuda") if len(xshape) == 4 else grid1d(xshape[2], "cuda")
    excl = ("fc0.",) if case.startswith("nio") else ("branch.", "fc0.")
    opt = FlatAdam(trained_parameters(m, exclude_prefixes=excl), lr=1e-3)
    gs = GraphedBagStep(m, blindno.mse_loss, opt, DataParallel(opt), x, y, grid)
    rs = np.random.RandomState(1)
    draws = [rs.choice(T, rs.randint(50, T), replace=case != "fno2d_attn") for _ in range(2)]

    def eager(idx):
        saved = [(b, b.detach().clone()) for b in m.buffers()]
        opt.zero_grad()
        out = m(x, grid, bag_idx=idx)
        blindno.mse_loss(out, y).backward()
        gg = opt.gather_grads().clone()
        opt.zero_grad()
        with torch.no_grad():
            for b, c in saved:
                b.copy_(c)
        return out.detach(), gg

    for idx in draws:
        gs.replay(idx)
    _poison_default_pool()
    for idx in list(draws) + list(reversed(draws)):
        key = gs.replay(idx)
        torch.cuda.synchronize()
        out, grad = gs.out[key].clone(), opt.grad.clone()
        eo, eg = eager(idx)
        assert torch.isfinite(grad).all() and torch.isfinite(out).all()
        assert rel_l2(out.cpu().numpy(), eo.cpu().numpy()) <= 1e-6
        assert rel_l2(grad.cpu().numpy(), eg.cpu().numpy()) <= 1e-6
        _poison_default_pool()


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


@pytest.mark.parametrize("width,B", [(12, 2), (16, 10)])
@pytest.mark.parametrize("toggle", ["default", "HEAD_BWD_MERGED", "UNPACK_FOLD", "HOST_ENC_MIX",
                                    "REDIRECT_GRADS"])
def test_deferred_finalisation_toggles_match_eager(toggle, width, B, monkeypatch):
    """The batched gradient finalisation (ops.deferred_reductions, which every graphed step
    takes) with each of its A/B switches turned off, against eager backward.  Width
    16 is outside the range the heads' merged weight-gradient kernel takes (5..15) and B = 10
    splits the weight gradient over samples: the grouped heads' (G, ...) reduction is then read
    slice-wise by the unpacks, which must not share a launch with it."""
    import blindno
    from blindno import ops, train
    from blindno.train import DataParallel, FlatAdam, GraphedBagStep, grid2d, trained_parameters
    if toggle != "default":
        mod = train if toggle == "REDIRECT_GRADS" else ops
        monkeypatch.setattr(mod, toggle, False)
    T, N = 60, 32
    g = torch.Generator(device="cuda").manual_seed(21)
    x = torch.randn(B, T, N, N, device="cuda", generator=g)
    y = torch.randn(B, N, N, 2, device="cuda", generator=g)
    grid = grid2d(N, N, "cuda")
    rs = np.random.RandomState(2)
    draws = [rs.choice(T, rs.randint(50, T)) for _ in range(2)]
    finals = []
    for graphed in (False, True):
        torch.manual_seed(13)
        m = blindno.NIOFP2D_FNO(2, 3, 100, 25, 3, width, 6, 2).cuda().train()
        opt = FlatAdam(trained_parameters(m), lr=1e-3)
        if graphed:
            gs = GraphedBagStep(m, blindno.mse_loss, opt, DataParallel(opt), x, y, grid)
            for idx in draws:
                gs.step(idx)
        else:
            for idx in draws:
                blindno.mse_loss(m(x, grid, bag_idx=idx), y).backward()
                opt.step()
                opt.zero_grad()
        torch.cuda.synchronize()
        finals.append(opt.flat.cpu().numpy().copy())
    assert np.isfinite(finals[1]).all()
    assert rel_l2(finals[1], finals[0]) <= 1e-6


def test_mse_counter_per_launch_streams():
    """The fused MSE forward's completion counter is per launch (or the caller's, per graph):
    two losses enqueued on two streams at once each return their own value."""
    import blindno
    g = torch.Generator(device="cuda").manual_seed(5)
    a = [torch.randn(4, 128, 128, 2, device="cuda", generator=g) for _ in range(4)]
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    s1.wait_stream(torch.cuda.current_stream())
    s2.wait_stream(torch.cuda.current_stream())
    outs = []
    for _ in range(20):
        with torch.cuda.stream(s1):
            l1 = blindno.mse_loss(a[0], a[1])
        with torch.cuda.stream(s2):
            l2 = blindno.mse_loss(a[2], a[3])
        outs.append((l1, l2))
    torch.cuda.synchronize()
    r1 = torch.mean((a[0].double() - a[1].double()) ** 2).item()
    r2 = torch.mean((a[2].double() - a[3].double()) ** 2).item()
    for l1, l2 in outs:
        assert abs(l1.item() - r1) <= 1e-5 * r1 and abs(l2.item() - r2) <= 1e-5 * r2
