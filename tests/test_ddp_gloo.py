"""World-size-2 data-parallel runtime on CPU (gloo): flat-gradient all-reduce averaging,
parameter broadcast, and identical parameters on every rank afterwards -- the contract
the RCCL path relies on (DESIGN.md "Multi-GPU").  The Adam kernel itself is a GPU op, so
the step is replaced here by the oracle's Adam restatement."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    try:
        _run(rank, world, port, q)
    except Exception as e:  # surface worker failures instead of a queue timeout
        q.put((rank, repr(e)))
        raise


def _run(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        sys.path.insert(0, os.path.join(root, "reconstruction-of-pde-without-time-label_amd"))
        sys.path.insert(0, root)
        import oracle
        from blindno.train import DataParallel, FlatAdam

        torch.manual_seed(100 + rank)            # ranks start different (seed + rank)
        w = torch.nn.Parameter(torch.randn(5, 3))
        c = torch.nn.Parameter(torch.randn(2, 4, dtype=torch.cfloat))
        opt = FlatAdam([w, c], lr=1e-2)

        def step(self, grad_scale=1.0, gather=True):   # test stand-in for the HIP Adam kernel
            if gather:
                self.gather_grads()
            self.t += 1
            p, m, v = oracle.adam_step(self.flat, self.grad * grad_scale, self.m, self.v, self.t, self.lr)
            self.flat.copy_(p.float())
            self.m.copy_(m.float())
            self.v.copy_(v.float())

        FlatAdam.step = step
        dp = DataParallel(opt)
        dp.broadcast_parameters(0)
        w0 = w.detach().clone()
        # per-rank gradient = rank-dependent
        w.grad = torch.full_like(w, float(rank + 1))
        c.grad = torch.full_like(c, complex(rank + 1, -(rank + 1)))
        dp.step()
        q.put((rank, w0.numpy().copy(), w.detach().numpy().copy(),
               torch.view_as_real(c.detach()).numpy().copy(), opt.grad.numpy().copy()))
    finally:
        dist.destroy_process_group()


def test_dataparallel_gloo_world2():
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for r in res:
        assert len(r) == 5, r
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort(key=lambda r: r[0])
    (_, w0a, wa, ca, ga), (_, w0b, wb, cb, gb) = res
    assert (w0a == w0b).all()                 # broadcast from rank 0
    assert (wa == wb).all() and (ca == cb).all()   # identical after the step
    # the flat gradient holds the SUM (all-reduce); Adam sees it scaled by 1/world = mean 1.5
    assert abs(float(ga[0]) - 3.0) < 1e-6 and abs(float(gb[0]) - 3.0) < 1e-6
    assert not (wa == w0a).all()


def test_synthetic_bag_set_is_keyed_by_bag_id():
    """bench.py's dataset: rank r of world w materialises bags {i : i mod w = r} of ONE global
    bag-keyed set -- the same bags whatever the world size."""
    import torch
    from blindno.train import synthetic_bags
    X, Y = synthetic_bags(8, 3, (4, 5), 2, seed=1234, device="cpu")
    for world in (2, 4):
        for r in range(world):
            ids = list(range(r, 8, world))
            xr, yr = synthetic_bags(len(ids), 3, (4, 5), 2, seed=1234, device="cpu", bag_ids=ids)
            assert torch.equal(xr, X[ids]) and torch.equal(yr, Y[ids])


def _shard_worker(rank, world, port, q, n_bags=22):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        try:
            import sys
            root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
            sys.path.insert(0, os.path.join(root, "reconstruction-of-pde-without-time-label_amd"))
            from blindno.train import shard_bag_ids, synthetic_bags
            B = 4
            ids = shard_bag_ids(n_bags, B, rank, world)
            X, Y = synthetic_bags(len(ids), 3, (4, 5), 2, seed=1234, device="cpu", bag_ids=ids)
            # every rank's ids and per-bag checksums, gathered over the process group
            n = torch.tensor([len(ids)])
            ns = [torch.zeros_like(n) for _ in range(world)]
            dist.all_gather(ns, n)
            m = int(max(int(t) for t in ns))
            pad = torch.full((m,), -1, dtype=torch.int64)
            pad[:len(ids)] = torch.tensor(ids)
            cs = torch.zeros(m, dtype=torch.float64)
            cs[:len(ids)] = X.double().sum(dim=(1, 2, 3)) + Y.double().sum(dim=(1, 2, 3))
            gi = [torch.zeros_like(pad) for _ in range(world)]
            gc = [torch.zeros_like(cs) for _ in range(world)]
            dist.all_gather(gi, pad)
            dist.all_gather(gc, cs)
            q.put((rank, [t.numpy().copy() for t in gi], [t.numpy().copy() for t in gc]))
        finally:
            dist.destroy_process_group()
    except Exception as e:
        q.put((rank, repr(e), None))
        raise


@pytest.mark.parametrize("world,n_bags", [(4, 22), (8, 42)])
def test_bag_sharding_gloo(world, n_bags):
    """bench.py's bag-keyed sharding at world 4 and at the driver's world 8 (gloo, CPU): the
    ranks' shards are disjoint, their union is the N = 1 bag set, and every bag's content equals
    the N = 1 set's."""
    from blindno.train import shard_bag_ids, synthetic_bags
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_shard_worker, args=(r, world, port, q, n_bags)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort(key=lambda r: r[0])
    assert all(r[2] is not None for r in res), res
    gi, gc = res[0][1], res[0][2]
    ids = [int(i) for a in gi for i in a if i >= 0]
    sums = {int(i): float(c) for a, b in zip(gi, gc) for i, c in zip(a, b) if i >= 0}
    full = shard_bag_ids(n_bags, 4, 0, 1)
    assert sorted(ids) == full and len(ids) == len(set(ids))
    X, Y = synthetic_bags(len(full), 3, (4, 5), 2, seed=1234, device="cpu")
    ref = X.double().sum(dim=(1, 2, 3)) + Y.double().sum(dim=(1, 2, 3))
    for i in full:
        assert sums[i] == float(ref[i])
