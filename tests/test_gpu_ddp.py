"""Data-parallel training on the HIP path with two ranks on one card (SURVEY §8e parity check).

Two processes share cuda:0 and a gloo process group (RCCL refuses two ranks on one device;
the data path -- FlatAdam's flat gradient, DataParallel's bucketed all-reduce, the fused Adam
kernel -- is the same code the RCCL run executes).  Each rank draws its bags from numpy
seeded 1234 + rank (the reference's seed + process_index, 2d_FPE/train_fno.py:78-81) and
trains 3 steps.  A single-process emulation then replays both ranks' draws, sums their
gradients and applies Adam with grad_scale 1/2; parameters must agree to rel-L2 <= 1e-5.
The "graphed" mode runs the ranks through train.GraphedBagStep, which at world size > 1 replays
each step as two graphs and all-reduces the heads' gradient on a side stream while the
encoder's backward replays (the overlapped path bench.py takes at N > 1).
"""
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

B, T, N, STEPS = 2, 60, 24, 3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _setup():
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "reconstruction-of-pde-without-time-label_amd"))
    import blindno
    from blindno.train import grid2d
    torch.manual_seed(0)
    m = blindno.NIOFP2D_FNO(2, 3, 100, 25, 2, 6, 5, 2).cuda().train()
    grid = grid2d(N, N, "cuda")
    return blindno, m, grid


def _data(rank):
    g = torch.Generator().manual_seed(77 + rank)
    x = torch.randn(STEPS, B, T, N, N, generator=g)
    y = torch.randn(STEPS, B, N, N, 2, generator=g)
    return x.cuda(), y.cuda()


def _worker(rank, world, port, q, mode="eager"):
    import torch.distributed as dist
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        blindno, m, grid = _setup()
        from blindno.train import DataParallel, FlatAdam, GraphedBagStep, trained_parameters
        from blindno.nio import draw_bag
        opt = FlatAdam(trained_parameters(m), lr=5e-4)
        dp = DataParallel(opt)
        dp.broadcast_parameters(0)
        x, y = _data(rank)
        np.random.seed(1234 + rank)
        if mode == "graphed":
            xs, ys = x[0].clone(), y[0].clone()
            gstep = GraphedBagStep(m, blindno.mse_loss, opt, dp, xs, ys, grid)
            assert gstep.overlap
            for s in range(STEPS):
                _, idx = draw_bag(T)
                xs.copy_(x[s])
                ys.copy_(y[s])
                gstep.step(idx)
        else:
            for s in range(STEPS):
                loss = blindno.mse_loss(m(x[s], grid), y[s])
                loss.backward()
                dp.step()
                opt.zero_grad()
        torch.cuda.synchronize()
        q.put((rank, opt.flat.cpu().numpy().copy()))
        dist.destroy_process_group()
    except Exception as e:
        q.put((rank, repr(e)))
        raise


@pytest.mark.parametrize("mode", ["eager", "graphed"])
def test_two_ranks_match_single_process_emulation(mode):
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q, mode)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(2))
    for p in ps:
        p.join(timeout=60)
    for r in (0, 1):
        assert not isinstance(res[r], str), res[r]
    assert np.array_equal(res[0], res[1])              # every rank holds the same parameters

    # emulation: both ranks' draws and gradients in one process, averaged
    blindno, m, grid = _setup()
    from blindno.train import FlatAdam, trained_parameters
    opt = FlatAdam(trained_parameters(m), lr=5e-4)
    data = [_data(r) for r in (0, 1)]
    states = []
    for r in (0, 1):
        np.random.seed(1234 + r)
        states.append(np.random.get_state())
    for s in range(STEPS):
        total = torch.zeros_like(opt.grad)
        for r in (0, 1):
            np.random.set_state(states[r])
            x, y = data[r]
            loss = blindno.mse_loss(m(x[s], grid), y[s])
            loss.backward()
            total += opt.gather_grads()
            opt.zero_grad()
            states[r] = np.random.get_state()
        opt.grad.copy_(total)
        opt.step(grad_scale=0.5, gather=False)
    ref = opt.flat.cpu().numpy()
    d = float(np.linalg.norm(res[0] - ref) / np.linalg.norm(ref))
    assert d <= 1e-5, d
