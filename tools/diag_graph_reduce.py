#!/usr/bin/env python3
"""Which torch op inside a captured HIP graph reads default-pool memory that is later reused?
Each case: eager warm-up on a side stream, capture, replay, poison the default pool (NaN), replay."""
import torch


def poison():
    torch.cuda.synchronize()
    blobs = []
    try:
        for _ in range(48):
            blobs.append(torch.full((1 << 28,), float("nan"), device="cuda"))
    except RuntimeError:
        pass
    torch.cuda.synchronize()
    del blobs
    torch.cuda.synchronize()


import os
SAME = os.environ.get("SAME_STREAM") == "1"


def run(name, make):
    torch.manual_seed(0)
    fn, inputs = make()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        ref = [t.clone() for t in fn(*inputs)]
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    pool = torch.cuda.graph_pool_handle()
    with torch.cuda.graph(g, pool=pool, stream=side if SAME else None):
        outs = fn(*inputs)
    g.replay()
    torch.cuda.synchronize()
    e0 = max(float((o - r).abs().max()) for o, r in zip(outs, ref))
    poison()
    g.replay()
    torch.cuda.synchronize()
    e1 = [float((o - r).abs().max()) for o, r in zip(outs, ref)]
    print(f"{name:40s} replay err {e0:.3e}   after poison " + " ".join(f"{e:.3e}" for e in e1), flush=True)


def lin_case(bias_only=False):
    lin = torch.nn.Linear(100, 100).cuda()
    x = torch.randn(16384, 100, device="cuda")

    def fn(x):
        for p in lin.parameters():
            p.grad = None
        y = lin(x)
        y.square().sum().backward()
        return [lin.bias.grad.clone(), lin.weight.grad.clone()]
    return fn, [x]


def sum_case():
    x = torch.randn(4, 75, 16384, device="cuda")

    def fn(x):
        return [x.sum().reshape(1), x.sum(0)]
    return fn, [x]


def colsum_case():
    x = torch.randn(16384, 100, device="cuda")

    def fn(x):
        return [x.sum(0)]
    return fn, [x]


def bn_case():
    bn = torch.nn.BatchNorm1d(100).cuda()
    x = torch.randn(16384, 100, device="cuda", requires_grad=True)

    def fn(x):
        for p in bn.parameters():
            p.grad = None
        x.grad = None
        y = bn(x)
        (y * y).sum().backward()
        return [bn.weight.grad.clone(), bn.bias.grad.clone(), x.grad.clone()]
    return fn, [x]


def matmul_case():
    w = torch.randn(4, 75, 25, device="cuda", requires_grad=True)
    basis = torch.randn(16384, 25, device="cuda", requires_grad=True)
    b0 = torch.zeros((), device="cuda", requires_grad=True)

    def fn(w, basis):
        w.grad = basis.grad = b0.grad = None
        u = (torch.matmul(w, basis.T) + b0) / 5
        u.square().mean().backward()
        return [w.grad.clone(), basis.grad.clone(), b0.grad.reshape(1).clone()]
    return fn, [w, basis]


def mm_only_case(K=300, batched=True):
    def mk():
        w = torch.randn(4, K // 4, 25, device="cuda") if batched else torch.randn(K, 25, device="cuda")
        du = torch.randn(*w.shape[:-1], 16384, device="cuda")

        def fn(w, du):
            # basis.grad of u = w @ basis^T: du^T @ w summed over the batch
            if batched:
                return [torch.matmul(du.transpose(-1, -2), w).sum(0)]
            return [du.t() @ w]
        return fn, [w, du]
    return mk


def mm_fwd_case():
    w = torch.randn(4, 75, 25, device="cuda")
    basis = torch.randn(16384, 25, device="cuda")

    def fn(w, basis):
        return [torch.matmul(w, basis.T)]
    return fn, [w, basis]


def bcast_case():
    b0 = torch.zeros((), device="cuda", requires_grad=True)
    v = torch.randn(4, 75, 16384, device="cuda")

    def fn(v):
        b0.grad = None
        ((v + b0) / 5).square().mean().backward()
        return [b0.grad.reshape(1).clone()]
    return fn, [v]


if __name__ == "__main__":
    print("SAME_STREAM", SAME, "TORCH_BLAS_PREFER_HIPBLASLT", os.environ.get("TORCH_BLAS_PREFER_HIPBLASLT"))
    for name, mk in (("matmul+b0 fwd+bwd", matmul_case), ("linear fwd+bwd", lin_case)):
        run(name, mk)
