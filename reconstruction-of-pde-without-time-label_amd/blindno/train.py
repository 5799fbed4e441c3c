"""Training-step runtime: flat-buffer Adam, data-parallel gradient all-reduce, StepLR
semantics and on-device synthetic snapshot-bag data.

Reference loop: 2d_FPE/train_fno.py:116-146 (MSE, Adam(lr), StepLR(100, 0.5), accelerate
DDP with one NCCL all-reduce of gradients per step).  Here one process drives one GPU
(torchrun), gradients of the TRAINED parameters are flattened into one fp32 buffer,
all-reduced (RCCL over xGMI, backend "nccl") and averaged, and a single fused Adam kernel
updates the flat parameter buffer that every parameter is a view of.

Parameters that the reference never trains (the unused ``branch`` encoder and the
``fc0`` of the bag mean, whose ``.data`` is read) receive no gradient and are left out
of the flat buffers -- numerically identical to the reference, where DDP's zero-filled
gradients give Adam updates of exactly zero.
"""
from __future__ import annotations

import contextlib
import ctypes
import math
import time
from typing import Iterable, List, Optional

import numpy as np
import torch
import torch.distributed as dist

from . import ops
from ._lib import call, ptr, stream_ptr


# the graphed step's deferred finalisation writes the gradients straight into the flat buffer
# (False, tests only: into their own tensors, then one gather copy)
REDIRECT_GRADS = True


def _real(t: torch.Tensor) -> torch.Tensor:
    return torch.view_as_real(t) if t.is_complex() else t


class FlatAdam:
    """torch.optim.Adam (no weight decay, no amsgrad) over one flat fp32 buffer.

    The listed parameters are re-pointed to views of ``self.flat`` (complex parameters
    through ``view_as_complex``), so one kernel updates all of them."""

    def __init__(self, params: Iterable[torch.nn.Parameter], lr: float, betas=(0.9, 0.999),
                 eps: float = 1e-8):
        self.params: List[torch.nn.Parameter] = [p for p in params]
        if not self.params:
            raise ValueError("FlatAdam: empty parameter list")
        dev = self.params[0].device
        self.sizes = [_real(p).numel() for p in self.params]
        # complex parameters need an even (8-byte aligned) offset for view_as_complex
        offs, off = [], 0
        for p, sz in zip(self.params, self.sizes):
            if p.is_complex() and off % 2:
                off += 1
            offs.append(off)
            off += sz
        n = off + (off % 2)
        self.n = n
        self.offsets = offs
        self.flat = torch.zeros(n, dtype=torch.float32, device=dev)
        self.grad = torch.zeros(n, dtype=torch.float32, device=dev)
        self.m = torch.zeros(n, dtype=torch.float32, device=dev)
        self.v = torch.zeros(n, dtype=torch.float32, device=dev)
        self._gviews = []
        for p, sz, o in zip(self.params, self.sizes, offs):
            rv = _real(p.data)
            self.flat[o:o + sz].copy_(rv.reshape(-1))
            view = self.flat[o:o + sz].view(rv.shape)
            p.data = torch.view_as_complex(view) if p.is_complex() else view
            self._gviews.append(self.grad[o:o + sz])
        self.lr = lr
        self.betas = betas
        self.eps = eps
        self.t = 0

    def zero_grad(self):
        for p in self.params:
            p.grad = None

    def gather_grads(self, subset=None):
        """Copy every parameter's .grad (or only those of ``subset``, a list of the trained
        parameters) into the flat grad buffer (one multi-tensor copy; alignment pads stay
        zero)."""
        sel = range(len(self.params)) if subset is None else \
            [i for i, p in enumerate(self.params) if any(p is q for q in subset)]
        gs, keep = [], []
        for i in sel:
            p = self.params[i]
            if p.grad is None:
                raise RuntimeError("FlatAdam: a trained parameter received no gradient")
            g = _real(p.grad).reshape(-1)
            if g.data_ptr() == self._gviews[i].data_ptr():
                continue                   # already in place (ops._Deferred.redirect)
            gs.append(g)
            keep.append(i)
        sel = keep
        if not gs:
            return self.grad
        if self.grad.is_cuda and all(g.is_contiguous() for g in gs):
            # one blindno_gather_flat launch (segments as kernel arguments; graph-capturable)
            srcs = (ctypes.c_void_p * len(gs))(*[g.data_ptr() for g in gs])
            offs = (ctypes.c_int64 * len(gs))(*[self.offsets[i] for i in sel])
            ns = (ctypes.c_int64 * len(gs))(*[g.numel() for g in gs])
            call("blindno_gather_flat", srcs, offs, ns, len(gs), ptr(self.grad), stream_ptr())
        else:
            torch._foreach_copy_([self._gviews[i] for i in sel], gs)
        return self.grad

    def grad_targets(self, subset=None):
        """(parameter, its view of the flat gradient buffer) pairs, for the deferred
        finalisation to write the gradients in place (ops._Deferred.redirect)."""
        sel = range(len(self.params)) if subset is None else \
            [i for i, p in enumerate(self.params) if any(p is q for q in subset)]
        return [(self.params[i], self._gviews[i]) for i in sel]

    def span(self, subset):
        """[lo, hi) of the flat buffer holding ``subset`` (must be contiguous in it)."""
        idx = sorted(i for i, p in enumerate(self.params) if any(p is q for q in subset))
        if not idx or idx != list(range(idx[0], idx[-1] + 1)):
            raise ValueError("FlatAdam.span: the parameters are not one contiguous run")
        lo = self.offsets[idx[0]]
        hi = self.offsets[idx[-1]] + self.sizes[idx[-1]]
        return lo, hi

    def step(self, grad_scale: float = 1.0, gather: bool = True):
        if gather:
            self.gather_grads()
        self.t += 1
        b1, b2 = self.betas
        step_size = self.lr / (1.0 - b1 ** self.t)
        bc2s = math.sqrt(1.0 - b2 ** self.t)
        call("blindno_adam", ptr(self.flat), ptr(self.grad), ptr(self.m), ptr(self.v), self.n,
             b1, b2, self.eps, step_size, bc2s, grad_scale, stream_ptr())
        # the kernel wrote the parameters behind autograd's back: bump their version counters
        # (host-side, ~10 us for 150 tensors) so anything keyed on them (caches, saved tensors)
        # sees the update
        torch.autograd.graph.increment_version(self.params)

    def state_dict(self):
        return {"t": self.t, "m": self.m.clone(), "v": self.v.clone(), "lr": self.lr}

    def load_state_dict(self, sd):
        self.t = int(sd["t"])
        self.m.copy_(sd["m"])
        self.v.copy_(sd["v"])
        self.lr = float(sd["lr"])


def trained_parameters(model: torch.nn.Module, exclude_prefixes=("branch.", "fc0.")):
    """Parameters the reference actually trains for the FNO-NIO models (no gradient ever
    reaches ``branch.*``; ``fc0`` is read through ``.data``)."""
    excl = tuple(exclude_prefixes) + tuple(getattr(model, "unused_prefixes", ()))
    return [p for n, p in model.named_parameters() if p.requires_grad and not n.startswith(excl)]


class StepLR:
    """StepLR(step_size, gamma) stepped once per epoch.  ``world_steps`` reproduces the
    accelerate quirk of stepping the scheduler once per process per call
    (accelerate/scheduler.py:69-76)."""

    def __init__(self, opt: FlatAdam, step_size=100, gamma=0.5, world_steps: int = 1):
        self.opt, self.step_size, self.gamma = opt, step_size, gamma
        self.base_lr = opt.lr
        self.world_steps = max(1, int(world_steps))
        self.count = 0

    def step(self):
        self.count += self.world_steps
        self.opt.lr = self.base_lr * self.gamma ** (self.count // self.step_size)


class DataParallel:
    """Gradient averaging across ranks for a FlatAdam (one bucketed all-reduce of the
    flat gradient; no other collective on the data path)."""

    def __init__(self, opt: FlatAdam, group=None, bucket_bytes: int = 64 << 20):
        self.opt = opt
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
        self.bucket = max(1, bucket_bytes // 4)

    def broadcast_parameters(self, src: int = 0):
        if self.world > 1:
            dist.broadcast(self.opt.flat, src, group=self.group)

    def step(self):
        self.opt.gather_grads()
        self.reduce_and_step()

    def reduce_and_step(self):
        """All-reduce the already-gathered flat gradient and apply the fused Adam update."""
        g = self.opt.grad
        if self.world > 1:
            for off in range(0, g.numel(), self.bucket):
                dist.all_reduce(g[off:off + self.bucket], group=self.group)
        self.opt.step(grad_scale=1.0 / self.world, gather=False)

    def reduce_range(self, lo: int, hi: int):
        """All-reduce the flat gradient's [lo, hi) (buckets) on the current stream."""
        if self.world > 1:
            g = self.opt.grad
            for off in range(lo, hi, self.bucket):
                dist.all_reduce(g[off:min(hi, off + self.bucket)], group=self.group)


class GraphedBagStep:
    """One training step of a snapshot-bag model (forward, loss, backward, gradient gather)
    replayed from a HIP graph.

    The bag size L = randint(50, T) changes every step (2d_FPE/NIOModules.py:548-553), so one
    graph is captured per L, all sharing one memory pool (graphs replay one at a time and keep
    nothing alive between replays).  The bag indices reach the graph through a static device
    buffer per L, filled from a small ring of pinned host buffers; the inputs x / y are static
    buffers the caller fills (e.g. index_select(..., out=)).  After the replay the gradient
    all-reduce (RCCL, N > 1) and the fused Adam update run eagerly.  With ``overlap`` the step
    is two graphs per key and the heads' all-reduce runs beside the encoder's backward (step()).  Every kernel of the step
    still runs on every replay: the graph removes the host launch overhead, not work."""

    def __init__(self, model, loss_fn, opt: "FlatAdam", dp: "DataParallel", x, y, grid,
                 loss_acc: Optional[torch.Tensor] = None, overlap: Optional[bool] = None):
        from . import nio
        self.model, self.loss_fn, self.opt, self.dp = model, loss_fn, opt, dp
        # overlap (default: with more than one rank, for models split into encoder + heads):
        # the step is replayed as two graphs -- A: forward, loss and the heads' backward; B: the
        # encoder's backward -- and the heads' gradient all-reduce (the bulk of the flat
        # gradient: 3.54 of 3.56 M parameters at config C) runs on a side stream beside B
        split_ok = hasattr(model, "forward_encoder") and hasattr(model, "forward_heads")
        self.overlap = (dp.world > 1) if overlap is None else bool(overlap)
        self.overlap = self.overlap and split_ok
        if self.overlap:
            heads = [p for n in model._heads for p in getattr(model, n).parameters()]
            enc = [p for p in opt.params if not any(p is q for q in heads)]
            self.head_params, self.enc_params = [p for p in opt.params if any(p is q for q in heads)], enc
            self.head_span = opt.span(self.head_params)
            self.enc_span = opt.span(self.enc_params)
            self.side = torch.cuda.Stream(x.device)
        self.x, self.y, self.grid = x, y, grid
        self.loss_acc = loss_acc
        # the seed gradient of loss.backward() (a static scalar: no fill kernel per replay)
        self._one = torch.ones((), dtype=torch.float32, device=x.device)
        self.pool = torch.cuda.graph_pool_handle()
        self.graphs = {}
        self.idx = {}
        self.lw = {}
        self.ctr = {}
        self.out = {}
        self.loss = {}
        self.T = x.shape[1]
        # deduplicated bags (NIOFP2D_FNO's fused encoder): graphs keyed by the number U of
        # distinct snapshots, fed the unique indices and multiplicity weights
        self.dedup = bool(getattr(model, "accepts_dedup_bag", False)) and nio.DEDUP_BAGS
        # pinned ring of [idx (int32) | weights (float32 bits)] slots: one H2D copy per step
        self._ring = [torch.empty(2 * self.T, dtype=torch.int32).pin_memory() for _ in range(4)]
        self._ev = [None] * len(self._ring)
        self._k = 0

    def _new_blob(self, L):
        """The key's static device buffer: [idx (L) | weights (L, float32 bits) | the fused
        MSE's completion counter (1, ops.loss_counter)], zeroed before the capture."""
        blob = torch.zeros(2 * L + 1, dtype=torch.int32, device=self.x.device)
        self.blob = getattr(self, "blob", {})
        self.blob[L] = blob
        self.idx[L] = blob[:L]
        self.lw[L] = blob[L:2 * L].view(torch.float32)
        self.ctr[L] = blob[2 * L:]

    def _seeded(self, L):
        """The loss's gradient for the unit seed formed in its forward pass (ops.unit_seed),
        and the key's own loss completion counter (ops.loss_counter)."""
        st = contextlib.ExitStack()
        st.enter_context(ops.loss_counter(self.ctr[L]))
        st.enter_context(ops.unit_seed(self._one))
        return st

    def _loss(self, out, accumulate):
        """The step's loss; with the fused MSE the running loss sum is accumulated by the loss
        kernel itself (no separate add launch)."""
        acc = self.loss_acc if accumulate else None
        if (acc is not None and self.loss_fn is ops.mse_loss and acc.dtype == torch.float32
                and acc.device == self.y.device and acc.dim() == 0):
            return self.loss_fn(out, self.y, acc), False
        return self.loss_fn(out, self.y), acc is not None

    def _body(self, L, accumulate=True):
        bag = (self.idx[L], self.lw[L]) if self.dedup else self.idx[L]
        out = self.model(self.x, self.grid, bag_idx=bag)
        with self._seeded(L):                         # backward is seeded with self._one
            loss, add = self._loss(out, accumulate)
        with ops.deferred_reductions() as fin:        # one batched gradient finalisation,
            loss.backward(self._one)
            if REDIRECT_GRADS:                        # storing into the flat buffer
                fin.redirect(self.opt.grad_targets())
        self.opt.gather_grads()
        if add:
            self.loss_acc.add_(loss.detach())
        return out.detach(), loss.detach()

    def _body_a(self, L, accumulate=True):
        """Graph A: forward, loss, the heads' backward (to the bag-mean field and the head
        parameters) and their gradient gather."""
        bag = (self.idx[L], self.lw[L]) if self.dedup else self.idx[L]
        h = self.model.forward_encoder(self.x, self.grid, bag_idx=bag)
        hd = h.detach().requires_grad_(True)
        out = self.model.forward_heads(hd)
        with self._seeded(L):
            loss, add = self._loss(out, accumulate)
        with ops.deferred_reductions() as fin:
            loss.backward(self._one)
            if REDIRECT_GRADS:
                fin.redirect(self.opt.grad_targets(self.head_params))
        self.opt.gather_grads(self.head_params)
        if add:
            self.loss_acc.add_(loss.detach())
        return h, hd, out.detach(), loss.detach()

    def _body_b(self, h, hd):
        """Graph B: the encoder's backward from the heads' input gradient, and its gather."""
        with ops.deferred_reductions() as fin:
            h.backward(hd.grad)
            if REDIRECT_GRADS:
                fin.redirect(self.opt.grad_targets(self.enc_params))
        self.opt.gather_grads(self.enc_params)

    def _buffers(self):
        """Copies of the model's buffers (BatchNorm running statistics and counters): the eager
        warm-up before a capture is a train-mode forward that would update them once more than
        the reference's training does; they are restored after it."""
        return [(b, b.detach().clone()) for b in self.model.buffers()]

    @staticmethod
    def _restore(saved):
        with torch.no_grad():
            for b, c in saved:
                b.copy_(c)

    def capture(self, L: int):
        if L in self.graphs:
            return
        if self.overlap:
            return self._capture_split(L)
        self._new_blob(L)
        saved = self._buffers()
        side = torch.cuda.Stream(self.x.device)
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):                 # eager warm-up: caches, lazy init
            self._body(L, accumulate=False)           # (its loss is not a training step's)
            self.opt.zero_grad()
        torch.cuda.current_stream().wait_stream(side)
        self._restore(saved)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, pool=self.pool):
            # static output / loss of the graph: valid after each replay of this key
            self.out[L], self.loss[L] = self._body(L)
        self.opt.zero_grad()
        self.graphs[L] = g

    def _capture_split(self, L: int):
        self._new_blob(L)
        saved = self._buffers()
        side = torch.cuda.Stream(self.x.device)
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):                 # eager warm-up of both halves
            h, hd, _, _ = self._body_a(L, accumulate=False)
            self._body_b(h, hd)
            self.opt.zero_grad()
        del h, hd
        torch.cuda.current_stream().wait_stream(side)
        self._restore(saved)
        ga, gb = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        with torch.cuda.graph(ga, pool=self.pool):
            h, hd, self.out[L], self.loss[L] = self._body_a(L)
        with torch.cuda.graph(gb, pool=self.pool):
            self._body_b(h, hd)
        # what A writes and B reads (h's saved activations, hd.grad) lives in the shared pool;
        # it is only live between A(L) and B(L), which always replay back to back, so later
        # captures may reuse it (keeping h would also pin the parameters' AccumulateGrad nodes
        # to this capture's stream)
        del h, hd
        self.opt.zero_grad()
        self.graphs[L] = (ga, gb)

    def release(self):
        """Drop every captured graph and its static buffers (frees the shared graph pool)."""
        self.graphs.clear()
        self.out.clear()
        self.loss.clear()
        self.idx.clear()
        self.lw.clear()
        self.ctr.clear()
        getattr(self, "blob", {}).clear()
        torch.cuda.synchronize()
        torch.cuda.empty_cache()

    def step(self, idx) -> int:
        """One training step on the drawn bag ``idx``: replay, all-reduce, Adam.  Returns the
        graph key (``self.out[key]`` / ``self.loss[key]`` hold this step's output and loss).
        With ``overlap``: replay A, the heads' all-reduce on the side stream while B (the
        encoder's backward) replays on the main stream, then the encoder's (small) all-reduce,
        the join, and Adam."""
        ht = getattr(self, "host_times", None)
        if not self.overlap:
            t0 = time.perf_counter()
            key = self.stage(idx)
            t1 = time.perf_counter()
            self.graphs[key].replay()
            t2 = time.perf_counter()
            e = self._ar_begin("all")
            self.dp.reduce_range(0, self.opt.grad.numel())
            self._ar_end(e)
            self.opt.step(grad_scale=1.0 / self.dp.world, gather=False)
            if ht is not None:     # host-side breakdown (bench.py host_us_per_step)
                t3 = time.perf_counter()
                for k, v in (("stage", t1 - t0), ("replay", t2 - t1), ("reduce_adam", t3 - t2)):
                    ht[k] = ht.get(k, 0.0) + v
            return key
        key = self.stage(idx)
        ga, gb = self.graphs[key]
        main = torch.cuda.current_stream()
        ga.replay()
        self.side.wait_stream(main)
        with torch.cuda.stream(self.side):
            e = self._ar_begin("heads (side stream, beside the encoder backward)")
            self.dp.reduce_range(*self.head_span)
            self._ar_end(e)
        gb.replay()
        e = self._ar_begin("encoder")
        self.dp.reduce_range(*self.enc_span)
        self._ar_end(e)
        main.wait_stream(self.side)
        self.opt.step(grad_scale=1.0 / self.dp.world, gather=False)
        return key

    # all-reduce timing (bench.py at N > 1): HIP events recorded on the stream that issues the
    # collective, around it; ar_events is None (off) or a list of (name, start, end)
    ar_events = None

    def _ar_begin(self, name):
        if self.ar_events is None or self.dp.world <= 1:
            return None
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record()
        return name, e0

    def _ar_end(self, e):
        if e is None:
            return
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record()
        self.ar_events.append((e[0], e[1], e1))

    def allreduce_ms(self):
        """Mean all-reduce time per step by piece (ms), from ar_events (after a synchronize)."""
        tot, cnt = {}, {}
        for name, e0, e1 in self.ar_events or []:
            tot[name] = tot.get(name, 0.0) + e0.elapsed_time(e1)
            cnt[name] = cnt.get(name, 0) + 1
        return {k: tot[k] / cnt[k] for k in tot}

    def replay(self, idx) -> int:
        """Stage the bag and replay its graph (forward, loss, backward, gradient gather into
        ``opt.grad``) without the optimizer step.  Returns the graph key."""
        L = self.stage(idx)
        g = self.graphs[L]
        if isinstance(g, tuple):
            for gg in g:
                gg.replay()
        else:
            g.replay()
        return L

    def stage(self, idx) -> int:
        """Capture the bag's graph(s) if needed and copy its indices (and multiplicity weights)
        into the graph's static buffer through the pinned ring.  Returns the graph key."""
        idx = np.asarray(idx, dtype=np.int32)
        w = None
        if self.dedup:
            from .nio import dedup_bag
            n_drawn = len(idx)
            idx, w = dedup_bag(idx)
            if w is None:
                w = np.full(len(idx), 1.0 / n_drawn, dtype=np.float32)
        L = len(idx)
        if L not in self.graphs:
            self.capture(L)
        k = self._k
        self._k = (k + 1) % len(self._ring)
        if self._ev[k] is not None:
            self._ev[k].synchronize()                 # ring slot's previous copy has landed
        buf = self._ring[k].numpy()
        buf[:L] = idx
        n = L
        if w is not None:
            buf[L:2 * L] = np.asarray(w, dtype=np.float32).view(np.int32)
            n = 2 * L
        self.blob[L][:n].copy_(self._ring[k][:n], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self._ev[k] = ev
        return L


class BatchSelect:
    """The training loop's batch select (2d_FPE/train_fno.py:113-116: the DataLoader's batch)
    from HBM-resident tensors: ``dsts[i][b] = srcs[i][ids[b]]`` for every pair in one
    blindno_gather_batch launch (ids: a device int64 slice of the epoch permutation)."""

    def __init__(self, srcs, dsts):
        if not 1 <= len(srcs) == len(dsts) <= 4:
            raise ValueError("BatchSelect: 1..4 (src, dst) pairs")
        for s_, d_ in zip(srcs, dsts):
            if not (s_.is_contiguous() and d_.is_contiguous() and s_.dtype == d_.dtype == torch.float32
                    and s_.shape[1:] == d_.shape[1:]):
                raise ValueError("BatchSelect: contiguous fp32 tensors with matching row shapes")
        self.B = dsts[0].shape[0]
        self._keep = (list(srcs), list(dsts))
        n = len(srcs)
        self._srcs = (ctypes.c_void_p * n)(*[t.data_ptr() for t in srcs])
        self._dsts = (ctypes.c_void_p * n)(*[t.data_ptr() for t in dsts])
        self._rows = (ctypes.c_int64 * n)(*[t[0].numel() for t in srcs])
        self._nsrc = (ctypes.c_int64 * n)(*[t.shape[0] for t in srcs])
        self._n = n

    def __call__(self, ids: torch.Tensor):
        if ids.dtype != torch.int64 or not ids.is_contiguous() or ids.numel() != self.B:
            raise ValueError("BatchSelect: ids must be a contiguous int64 tensor of the batch size")
        # an id outside a source's rows fills that batch row with NaN on the device (checking
        # the range here would cost a device->host sync per step)
        call("blindno_gather_batch", self._srcs, self._dsts, self._rows, self._nsrc, self._n, ptr(ids),
             self.B, stream_ptr())


def shard_bag_ids(n_bags: int, per_rank_batch: int, rank: int, world: int):
    """Bag-keyed data-parallel sharding (the reference's accelerate sampler
    splits one dataset over the processes): rank r of ``world`` owns the global bags
    {i : i mod world = r} of a set of max(n_bags, B * world) bags -- disjoint shards whose
    union is the N = 1 set, so the data does not depend on the world size."""
    return list(range(rank, max(n_bags, per_rank_batch * world), world))


def synthetic_bags(n_bags: int, T: int, grid_shape, out_ch: int, seed: int, device,
                   bag_ids=None):
    """Standardised synthetic snapshot bags x ~ N(0,1) (n, T, *grid) and targets
    (n, *grid, out_ch), generated on the device (the real datasets are not shipped with the
    reference).  Bag ``i`` of the global set is drawn from its own generator seeded by
    (seed, i), so its content does not depend on which rank holds it: ``bag_ids`` (default
    0..n_bags-1) lists the global ids this rank materialises -- rank r of world w holds
    {i : i mod w = r}, the same data at any world size."""
    ids = list(range(n_bags)) if bag_ids is None else [int(i) for i in bag_ids]
    g = torch.Generator(device=device)
    x = torch.empty(len(ids), T, *grid_shape, dtype=torch.float32, device=device)
    y = torch.empty(len(ids), *grid_shape, out_ch, dtype=torch.float32, device=device)
    for j, i in enumerate(ids):
        g.manual_seed(seed * 1_000_003 + i)
        x[j].normal_(generator=g)
        y[j].normal_(generator=g)
    return x, y


def grid2d(nx: int, ny: int, device):
    """meshgrid(linspace(-1,1,nx), linspace(-1,1,ny), 'ij') stacked (2d_FPE/train_fno.py:109-114)."""
    gx, gy = np.meshgrid(np.linspace(-1, 1, nx, dtype=np.float32),
                         np.linspace(-1, 1, ny, dtype=np.float32), indexing="ij")
    return torch.tensor(np.stack([gx, gy], axis=2), device=device)


def grid1d(nx: int, device):
    """linspace(0,1,nx)[:, None] (1d_FPE/train_fno.py:98)."""
    return torch.linspace(0, 1, nx, device=device).unsqueeze(-1)
